"""Gradient size tables (element counts, in backward order) of the models the
reference benchmarks with (parity: v1/benchmarks/model_sizes.py; fake trainers
in tests/cpp/integration/{resnet50_info,vgg_info,bert}.hpp).  Derived from
this package's own model definitions rather than hard-coded."""
from __future__ import annotations

from functools import lru_cache
from typing import List


@lru_cache(maxsize=None)
def grad_sizes(model: str) -> List[int]:
    from ..models import get_model

    m = get_model(model)
    return [p.numel() for p in m.parameters() if p.requires_grad][::-1]


MODELS = ["resnet50", "vgg16", "bert_base", "inception_v3", "resnet18", "slp"]
