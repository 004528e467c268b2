"""Dataset helpers: elastic sharding adaptor, MNIST idx loader, synthetic data."""
from .adaptor import ElasticShardAdaptor, shard_range
from .mnist import load_mnist, synthetic_mnist
from .synthetic import SyntheticImageNet
