"""Dataset helpers: elastic sharding adaptor, MNIST idx / CIFAR binary loaders, ImageNet shards with
GPU augmentation, synthetic data."""
from .adaptor import ElasticShardAdaptor, shard_range
from .mnist import load_mnist, synthetic_mnist
from .synthetic import SyntheticImageNet
from .cifar import Cifar10Loader, Cifar100Loader
from .imagenet import ImageNetShards, gpu_augment
