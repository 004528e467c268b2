"""Model zoo used by the benchmarks and tests (random init, synthetic data)."""
from .resnet import resnet18, resnet34, resnet50, resnet101, resnet152


def get_model(name: str, **kw):
    import importlib

    table = {
        "resnet18": ("resnet", "resnet18"), "resnet34": ("resnet", "resnet34"),
        "resnet50": ("resnet", "resnet50"), "resnet101": ("resnet", "resnet101"),
        "resnet152": ("resnet", "resnet152"), "vgg16": ("vgg", "vgg16"),
        "inception_v3": ("inception", "inception_v3"), "bert_base": ("bert", "bert_base"),
        "slp": ("slp", "SLP"),
    }
    mod, fn = table[name]
    return getattr(importlib.import_module("kungfu_amd.models." + mod), fn)(**kw)
