"""BERT-base linear weight gradients at 16 K tokens: dW[out, in] = dy^T . x accumulated into an f32
slot (what the engine's direct path does, ops/linear.py) -- ours (split-K MFMA + reduce into the slot)
vs hipBLASLt (torch.mm with out_dtype=float32, or bf16 mm + f32 add)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from kungfu_amd._lib import hip  # noqa: E402

SWEEP = "--sweep" in sys.argv  # every tile variant x split count of the split-K kernel


def _as_nhwc(t2):
    T, C = t2.shape
    return t2.as_strided((1, C, 1, T), (T * C, 1, T * C, C))


def timeit(fn, n=20):
    for _ in range(3):
        fn()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(n):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) * 1e3 / n


def main():
    T = 16384
    tot = {}
    for name, fin, fout in (("qkv", 768, 2304), ("out", 768, 768), ("fc1", 768, 3072), ("fc2", 3072, 768)):
        x = torch.randn(T, fin, device="cuda").bfloat16()
        dy = torch.randn(T, fout, device="cuda").bfloat16()
        slot = torch.zeros(fout, fin, device="cuda")
        ref = dy.float().t() @ x.float()

        def ours():
            slot.zero_()
            hip().conv_wgrad(_as_nhwc(dy), _as_nhwc(x), 1, 1, out=slot.as_strided((fout, fin, 1, 1), (fin, 1, fin, fin)),
                             accumulate=True, atomics=False)

        def blas_f32():
            torch.mm(dy.t(), x, out_dtype=torch.float32, out=slot)

        def blas_bf16():
            slot.zero_()
            slot.add_(torch.mm(dy.t(), x))

        fl = 2.0 * T * fin * fout
        row = [name]
        for lab, fn in (("ours", ours), ("blas_f32out", blas_f32), ("blas_bf16+add", blas_bf16)):
            try:
                us = timeit(fn)
                fn()
                torch.cuda.synchronize()
                err = ((slot - ref).norm() / ref.norm()).item()
                row.append("%s %.1f us (%.0f TF/s, rel %.1e)" % (lab, us, fl / us / 1e6, err))
                tot[lab] = tot.get(lab, 0.0) + us * (12 if name != "out" else 12)
            except Exception as e:  # noqa: BLE001
                row.append("%s ERR %s" % (lab, str(e)[:80]))
        print("  ".join(row), flush=True)
        if SWEEP:
            res = []
            for v in range(hip().conv_wgrad_variants()):
                seen = set()
                for sp in (4, 8, 16, 32, 64, 128, 256):
                    try:
                        sp2 = hip().conv_wgrad_plan(1, 1, T, fin, fout, 1, 1, v, sp)[1]
                    except Exception:  # noqa: BLE001
                        break
                    if sp2 in seen:
                        continue
                    seen.add(sp2)

                    def f(v=v, sp2=sp2):
                        slot.zero_()
                        hip().conv_wgrad(_as_nhwc(dy), _as_nhwc(x), 1, 1,
                                         out=slot.as_strided((fout, fin, 1, 1), (fin, 1, fin, fin)),
                                         accumulate=True, atomics=False, variant=v, splits=sp2)
                    res.append((timeit(f, n=10), v, sp2))
            res.sort()
            print("   plan %s | best: %s" % (hip().conv_wgrad_plan(1, 1, T, fin, fout, 1, 1),
                                             " ".join("v%d/s%d %.1f" % (v, sp, t) for t, v, sp in res[:5])), flush=True)
    print("per step (x12 layers):", {k: round(v, 1) for k, v in tot.items()})


if __name__ == "__main__":
    main()
