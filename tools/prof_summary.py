"""Summarise a rocprofv3 ``--kernel-trace`` CSV per training step.

Usage: python tools/prof_summary.py <kernel_trace.csv> [--marker sgd] [--steps 3] [--top 30]

A "step" is the span between consecutive launches of the marker kernel (the fused optimizer
step).  Prints, for the mean of the last ``--steps`` steps: wall time, busy time (sum of kernel
durations, overlap-free union), kernel count, a per-category breakdown and the top kernels.
Output is markdown so it can be pasted into ``profiles/``.
"""
from __future__ import annotations

import argparse
import collections
import csv
import re

CATEGORIES = [
    ("conv fwd", r"conv_fwd|igemm_fwd|naive_conv.*fwd|ConvFwd"),
    ("conv bwd-data", r"conv_bwd_data|igemm_bwd_|ConvBwdData|naive_conv.*bwd"),
    ("conv bwd-weight", r"igemm_wrw|conv_bwd_weight|batched_gemm_xdl|ConvBwdWeight|wrw"),
    ("gemm (fc/linear)", r"Cijk_|gemm|hipblaslt"),
    ("BN finalize (ours)", r"kfk::.*(bn_sums_finalize|bn_bwd_finalize|bn_stats_finalize|bn_eval_coef|stem_bwd_finalize)"),
    ("fused BN (ours)", r"kfk::.*bn_"),
    ("conv MFMA 1x1 (ours)", r"kfk::.*conv_kernel<1,"),
    ("conv MFMA 3x3 (ours)", r"kfk::.*conv3x3|kfk::.*conv_kernel<3,|kfk::.*conv_rows_kernel"),
    ("conv MFMA rect KHxKW (ours)", r"kfk::.*conv_kernel<1\d\d,"),
    ("conv MFMA stride-2 dgrad phases (ours)", r"kfk::.*conv_kernel<\d\d,"),
    ("conv weight flip (ours)", r"kfk::.*conv_flip"),
    ("conv MFMA wgrad (ours)", r"kfk::.*wgrad"),
    ("conv bias+ReLU (ours)", r"kfk::.*bias_act"),
    ("max-pool 2x2 (ours)", r"kfk::.*maxpool2"),
    ("stem conv MFMA (ours)", r"kfk::.*stem"),
    ("LayerNorm (ours)", r"kfk::.*ln_(fwd|bwd|colsum)"),
    ("attention (ours)", r"kfk::.*attn_"),
    ("pool (ours)", r"kfk::.*(gap_|avgpool|maxpool3s2)"),
    ("bias-grad colsum (ours)", r"kfk::.*colsum_stage"),
    ("gradient landing (ours)", r"kfk::.*(grad_accumulate|multi_copy)"),
    ("optimizer step (ours)", r"kfk::.*(sgd_f32|adam_f32|axpby_)"),
    ("GNS / variance monitors (ours)", r"kfk::.*(sumsq2|gns_update|variance_stage|seg_variance|square_kernel|fold1|fold2)"),
    ("casts (ours)", r"kfk::.*(cast8|cast_tail)"),
    ("K1 reduce / scale (ours)", r"kfk::.*(reduce_f32|reduce_half|reduce_plain|scale_f32|scale_kernel)"),
    ("other (ours)", r"kfk::"),
    ("rccl", r"ncclDevKernel|oneRankReduce|rccl"),
    ("casts", r"bfloat16tofloat32_copy|bfloat16_copy|float_to|copy_kernel"),
    ("accumulate/add", r"CUDAFunctor_add|AddFunctor"),
    ("fill/memset/copy", r"fillBuffer|copyBuffer|FillFunctor|SubTensorOp|Op2dTensor|Op1dTensor|CatArrayBatchedCopy"),
    ("pool", r"pool"),
    ("loss/softmax", r"softmax|SoftMax|nll|cross_entropy|log_softmax"),
    ("GELU (torch)", r"Gelu"),
    ("dropout (torch)", r"dropout|masked_scale"),
    ("embedding grad (torch)", r"sum_and_scatter|compute_grad_weight|embedding|device_block_merge|radix_sort"),
    ("LayerNorm (torch)", r"layer_norm|GradGammaBeta"),
    ("batchnorm (torch/MIOpen)", r"batch_norm|BatchNorm|MIOpenBatchNorm"),
    ("other elementwise", r"elementwise|reduce_kernel"),
]


def short_name(name: str) -> str:
    """Kernel name without namespaces noise and its argument list."""
    nm = name.replace("(anonymous namespace)::", "").replace("void ", "", 1)
    nm = re.sub(r"\(.*", "", nm)
    return nm[:110]


def categorize(name: str) -> str:
    for cat, pat in CATEGORIES:
        if re.search(pat, name):
            return cat
    return "other"


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--marker", default="sgd")
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--top", type=int, default=30)
    a = ap.parse_args()
    rows = list(csv.DictReader(open(a.trace)))
    rows.sort(key=lambda x: int(x["Start_Timestamp"]))
    marks = [i for i, x in enumerate(rows) if re.search(a.marker, x["Kernel_Name"], re.I)]
    if len(marks) < 2:
        raise SystemExit("need >= 2 marker kernels, found %d" % len(marks))
    n = min(a.steps, len(marks) - 1)
    spans = [(marks[-1 - k - 1] + 1, marks[-1 - k] + 1) for k in range(n)]
    cat_t = collections.Counter()
    cat_n = collections.Counter()
    kern_t = collections.Counter()
    kern_n = collections.Counter()
    wall = busy = count = 0
    for lo, hi in spans:
        seg = rows[lo:hi]
        s0 = int(seg[0]["Start_Timestamp"])
        s1 = max(int(x["End_Timestamp"]) for x in seg)
        wall += s1 - s0
        # union of busy intervals (kernels on several streams may overlap)
        iv = sorted((int(x["Start_Timestamp"]), int(x["End_Timestamp"])) for x in seg)
        cur_s, cur_e = iv[0]
        for s, e in iv[1:]:
            if s > cur_e:
                busy += cur_e - cur_s
                cur_s, cur_e = s, e
            else:
                cur_e = max(cur_e, e)
        busy += cur_e - cur_s
        count += len(seg)
        for x in seg:
            d = int(x["End_Timestamp"]) - int(x["Start_Timestamp"])
            nm = x["Kernel_Name"]
            c = categorize(nm)
            cat_t[c] += d
            cat_n[c] += 1
            short = short_name(nm)
            kern_t[short] += d
            kern_n[short] += 1
    ms = lambda ns: ns / n / 1e6
    tot = sum(cat_t.values())
    print("steps averaged: %d  | wall %.2f ms/step | GPU busy %.2f ms/step | kernel sum %.2f ms | %d kernels/step"
          % (n, ms(wall), ms(busy), ms(tot), count // n))
    print()
    print("| category | ms/step | % of kernel time | launches/step |")
    print("|---|---:|---:|---:|")
    for c, t in cat_t.most_common():
        print("| %s | %.2f | %.1f | %d |" % (c, ms(t), 100.0 * t / tot, cat_n[c] // n))
    print()
    print("| kernel | ms/step | launches/step |")
    print("|---|---:|---:|")
    for k, t in kern_t.most_common(a.top):
        print("| `%s` | %.3f | %d |" % (k.replace("|", "/"), ms(t), kern_n[k] // n))


if __name__ == "__main__":
    main()
