"""Native library loading.

``_kungfu`` is the C++ host runtime (no torch dependency).  ``_hip`` holds the
CDNA4 kernels and the RCCL controller; it links against the HIP runtime and
RCCL, so ``torch`` is imported first: torch's bundled ``libamdhip64.so.7`` /
``librccl.so.1`` are then already resident and the extension binds to the
same copies (one HIP runtime per process).

On a machine with a GPU, a missing/broken ``_hip`` is a hard error (no silent
eager fallback); on a CPU-only machine GPU features are simply unavailable.
"""
from __future__ import annotations

import importlib
import os
import subprocess
import sys

import torch  # noqa: F401  (must precede the native modules, see above)

_ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

try:
    from . import _kungfu as runtime  # type: ignore
except ImportError as e:  # pragma: no cover - only when the build was skipped
    raise ImportError(
        "kungfu_amd native runtime is not built; run `make -j8` in %s (%s)" % (_ROOT, e)
    ) from e

_hip_mod = None
_hip_err = None


def hip():
    """Return the ``_hip`` extension module (loads on first use)."""
    global _hip_mod, _hip_err
    if _hip_mod is not None:
        return _hip_mod
    try:
        _hip_mod = importlib.import_module("kungfu_amd._hip")
    except ImportError as e:
        _hip_err = e
        raise RuntimeError(
            "kungfu_amd._hip (HIP kernels) is not built or failed to load: %s; "
            "run `make hip` (hipcc --offload-arch=gfx950)" % e
        ) from e
    from . import knobs

    if knobs.get("KUNGFU_NATIVE_BACKTRACE") == "1":
        _hip_mod.install_native_backtrace()
    return _hip_mod


# The MFMA conv kernels stage operands through buffer resources with 32-bit byte offsets
# (csrc/kernels/conv.hip kBufOOB): every operand must stay below 2 GiB; larger shapes fall back
# to the library paths.
BUF_LIMIT_BYTES = 1 << 31


def buf_ok(*numels: int, esz: int = 2) -> bool:
    """True when every operand of ``numels`` elements (``esz`` bytes each) is addressable
    by the kernels' buffer-resource staging (below 2 GiB)."""
    return all(int(n) * esz < BUF_LIMIT_BYTES for n in numels)


def hip_available() -> bool:
    try:
        hip()
        return True
    except RuntimeError:
        return False


def require_hip_on_gpu():
    """Fail loudly when a GPU is present but the HIP extension cannot load."""
    if torch.cuda.is_available():
        hip()


def bin_path(name: str) -> str:
    return os.path.join(_ROOT, "bin", name)


def build(targets=("all",), jobs: int = 8):
    """Build the native components in-tree (make)."""
    cmd = ["make", "-C", _ROOT, "-j%d" % jobs] + list(targets)
    subprocess.check_call(cmd)


DTYPE_CODES = {
    torch.uint8: 0,
    torch.int8: 4,
    torch.int16: 5,
    torch.int32: 6,
    torch.int64: 7,
    torch.float16: 8,
    torch.bfloat16: 9,
    torch.float32: 10,
    torch.float64: 11,
    torch.bool: 12,
}

OP_CODES = {"sum": 0, "min": 1, "max": 2, "prod": 3, "avg": 4}


def dtype_code(t) -> int:
    dt = t.dtype if hasattr(t, "dtype") else t
    try:
        return DTYPE_CODES[dt]
    except KeyError:
        raise TypeError("kungfu_amd: unsupported dtype %s" % dt)


def op_code(op) -> int:
    if op is None:
        return 0
    try:
        return OP_CODES[op.lower()]
    except KeyError:
        raise ValueError("kungfu_amd: unsupported reduce op %r" % (op,))
