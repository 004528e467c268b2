"""Checkpoint / resume for data-parallel training.

The reference has no checkpoint subsystem of its own: it relies on TF
Estimator ``model_dir`` / Keras, derives a per-peer directory from ``uid()``
(``tests/python/integration/test_elastic_estimator.py:58-64``), and "resume" after a resize
is a state broadcast from the surviving root plus a step sync.  Here:

* :func:`save` -- rank 0 writes ``{model, optimizer (incl. the fused flat buffers and host
  scalars), step, trained_samples, cluster size, extra}`` atomically (write to a temporary
  file in the same directory, fsync, rename), then every peer passes a barrier, so a
  checkpoint is either complete or absent;
* :func:`load` -- rank 0 reads it (``torch.load(weights_only=True)``: nothing in the file is
  executed), every peer receives the state through the same broadcasts as an elastic
  (re)join (``broadcast_model``), and the step / sample counters are agreed on with an
  all-reduce max -- so a job restarted with a DIFFERENT number of peers resumes correctly;
* :func:`latest` -- the newest ``ckpt-<step>.pt`` in a directory (``KUNGFU_INIT_CKPT``, the
  launcher's hint for re-joining workers, also works: ``ops.get_init_checkpoint``).
"""
from __future__ import annotations

import glob
import os
import re
from typing import Any, Dict, Optional

import torch

from .. import ops
from ..initializer import broadcast_model
from ..python import _ensure, current_cluster_size, current_rank, run_barrier


def _cpu(obj):
    if isinstance(obj, torch.Tensor):
        return obj.detach().to("cpu")
    if isinstance(obj, dict):
        return {k: _cpu(v) for k, v in obj.items()}
    if isinstance(obj, (list, tuple)):
        return type(obj)(_cpu(v) for v in obj)
    return obj


def _optimizer_state(optimizer) -> Dict[str, Any]:
    if optimizer is None:
        return {}
    out = {"state_dict": _cpu(optimizer.state_dict())}
    holders = []
    for o in (optimizer, getattr(optimizer, "inner", None)):
        if o is not None and hasattr(o, "_kf_scalars") and all(o is not h for h in holders):
            holders.append(o)
    out["scalars"] = [list(map(float, h._kf_scalars())) for h in holders]
    return out


def save(path: str, model: torch.nn.Module, optimizer=None, step: int = 0, trained_samples: int = 0,
         extra: Optional[Dict[str, Any]] = None) -> Optional[str]:
    """Collective: rank 0 writes the checkpoint atomically; returns the path on rank 0."""
    _ensure()
    written = None
    if current_rank() == 0:
        blob = {
            "format": "kungfu_amd/1",
            "model": _cpu(model.state_dict()),
            "optimizer": _optimizer_state(optimizer),
            "step": int(step),
            "trained_samples": int(trained_samples),
            "cluster_size": current_cluster_size(),
            "extra": extra or {},
        }
        d = os.path.dirname(os.path.abspath(path))
        os.makedirs(d, exist_ok=True)
        tmp = os.path.join(d, ".%s.tmp-%d" % (os.path.basename(path), os.getpid()))
        with open(tmp, "wb") as f:
            torch.save(blob, f)
            f.flush()
            os.fsync(f.fileno())
        os.replace(tmp, path)
        written = path
    run_barrier()
    return written


def latest(directory: str) -> Optional[str]:
    """Newest ``ckpt-<step>.pt`` in ``directory`` (by step), or None."""
    best, best_step = None, -1
    for p in glob.glob(os.path.join(directory, "ckpt-*.pt")):
        m = re.search(r"ckpt-(\d+)\.pt$", p)
        if m and int(m.group(1)) > best_step:
            best, best_step = p, int(m.group(1))
    return best


def load(path: str, model: torch.nn.Module, optimizer=None) -> Dict[str, Any]:
    """Collective: restore ``model`` (and ``optimizer``) from rank 0's checkpoint on every
    peer.  Returns ``{"step", "trained_samples", "cluster_size", "extra"}``, identical on every
    peer (``extra`` is rank 0's, broadcast)."""
    _ensure()
    meta = torch.zeros(3, dtype=torch.int64)
    extra: Dict[str, Any] = {}
    if current_rank() == 0:
        blob = torch.load(path, map_location="cpu", weights_only=True)
        model.load_state_dict(blob["model"])
        st = blob.get("optimizer") or {}
        if optimizer is not None and st.get("state_dict") is not None:
            optimizer.load_state_dict(st["state_dict"])
            holders = []
            for o in (optimizer, getattr(optimizer, "inner", None)):
                if o is not None and hasattr(o, "_kf_load_scalars") and all(o is not h for h in holders):
                    holders.append(o)
            for h, vals in zip(holders, st.get("scalars", [])):
                h._kf_load_scalars(vals)
        space = getattr(optimizer, "space", None)
        if space is not None:
            space.check_params()
        meta = torch.tensor([blob["step"], blob["trained_samples"], blob["cluster_size"]], dtype=torch.int64)
        extra = blob.get("extra", {})
    # every peer gets rank 0's model + optimizer state exactly as after an elastic (re)join
    broadcast_model(model, optimizer)
    meta = ops.all_reduce(meta, op="max")
    # ``extra`` (data-loader position, scheduler state, ...) is rank 0's on every peer
    import io

    from ..initializer import broadcast_bytes

    if current_rank() == 0:
        bio = io.BytesIO()
        torch.save(extra, bio)
        data = bio.getvalue()
    else:
        data = None
    extra = torch.load(io.BytesIO(broadcast_bytes(data)), map_location="cpu", weights_only=True)
    return {"step": int(meta[0]), "trained_samples": int(meta[1]), "cluster_size": int(meta[2]), "extra": extra}
