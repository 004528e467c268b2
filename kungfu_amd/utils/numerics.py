"""Float64 references for checking fused kernels at model level.

:func:`bn_param_grads_f64` recomputes a BatchNorm's (dgamma, dbeta) in float64 from the SAME bf16
tensors the fused backward consumed: the BN input x, the gradient reaching the BN(+ReLU) output, the
batch mean / invstd and the ReLU gate.  Both sides then share every rounding up to the final
reduction, so the check can be tight (relative error ~1e-5) where a comparison against an f32 model
cannot: at random init the BN gamma/beta gradients are sums with massive cancellation, and bf16 vs
f32 differ in them by a relative error of 1.1-1.5 (profiles/r5_engine_numerics.md), a bound a
sign-flipped gradient would also meet.

No reference counterpart: the reference checks accuracy at the end of training
(``tests/python/integration/test_mnist_slp.py:149-165``), a regime this replaces for the fused
kernels with a per-parameter pin.
"""
from __future__ import annotations

from typing import Optional, Tuple

import torch


def unpack_mask(mask: torch.Tensor, rows: int, channels: int) -> torch.Tensor:
    """The fused kernels' 1-bit ReLU mask (one byte per 8 channels of an NHWC row, bit k = channel
    8j + k) as a bool [rows, channels] tensor."""
    bits = (mask.view(-1, 1).to(torch.int32) >> torch.arange(8, device=mask.device, dtype=torch.int32)) & 1
    return bits.view(rows, channels).bool()


def _rows(t: torch.Tensor) -> torch.Tensor:
    """[N, C, H, W] channels_last (or [rows, C]) -> [rows, C] in NHWC element order."""
    if t.dim() == 4:
        return t.permute(0, 2, 3, 1).reshape(-1, t.shape[1])
    return t.reshape(-1, t.shape[-1])


def bn_param_grads_f64(dz: torch.Tensor, x: torch.Tensor, mean: torch.Tensor, invstd: torch.Tensor,
                       kind: str, gate: Optional[torch.Tensor] = None) -> Tuple[torch.Tensor, torch.Tensor]:
    """(dgamma, dbeta) in float64 of ``z = act(gamma * (x - mean) * invstd + beta)``.

    ``kind``: ``"relu"`` -- act = ReLU, ``gate`` = the forward coefficients [scale(C); shift(C)]
    (relu' recomputed as x * scale + shift > 0, as the kernels do with one f32 FMA: its sign is the
    sign of the exact value, computed here in f64 -- x is bf16, so x * scale is exact in f64 and the
    one rounding of the sum keeps its sign; a separately rounded f32 product flips gates of
    elements whose BN output rounds to about zero); ``"mask"`` -- the
    ReLU gate is the 1-bit mask ``gate`` (a BN + residual + ReLU tail); ``"plain"`` -- no
    activation (``dz`` already is the gradient at the BN output)."""
    xr, dr = _rows(x), _rows(dz).double()
    C = xr.shape[1]
    if kind == "relu":
        sc, sh = gate[:C].float().double(), gate[C:2 * C].float().double()
        on = xr.double() * sc + sh > 0
        dr = dr * on
    elif kind == "mask":
        dr = dr * unpack_mask(gate, xr.shape[0], C)
    elif kind != "plain":
        raise ValueError(kind)
    xhat = (xr.double() - mean.double()) * invstd.double()
    return (dr * xhat).sum(0), dr.sum(0)


def rel_err(ref: torch.Tensor, got: torch.Tensor) -> float:
    """||got - ref|| / ||ref|| in float64 (0 when both are zero)."""
    ref, got = ref.double().reshape(-1), got.double().reshape(-1)
    n = ref.norm().item()
    d = (got - ref).norm().item()
    return d / n if n > 0 else d


def check_bn_param_grads(ref: Tuple[torch.Tensor, torch.Tensor], got: Tuple[torch.Tensor, torch.Tensor],
                         tol: float = 1e-3) -> Optional[str]:
    """None if both of ``got``'s (dgamma, dbeta) are within ``tol`` relative L2 error of ``ref``;
    otherwise a message naming the worse one.  A sign-flipped, permuted or unrelated gradient of the
    same norm scores 2, ~1.4 and ~1.4."""
    for name, r, g in (("dgamma", ref[0], got[0]), ("dbeta", ref[1], got[1])):
        e = rel_err(r, g)
        if not e <= tol:
            return "%s relative error %.3g > %.3g" % (name, e, tol)
    return None
