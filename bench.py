#!/usr/bin/env python3
"""Headline benchmark: ResNet-50 SynchronousSGD training throughput on MI355X.

Metric (BASELINE.json): images/sec ResNet-50 SynchronousSGD at 1/2/4/8 MI355X.
The reference's comparable number is ~344 img/s/GPU (KungFu S-SGD, 256 images
per GPU, 16 x V100); ``vs_baseline`` = value / (344.2 * n_gpus).

Config: ResNet-50 (v1.5, 25.56 M params, random init), synthetic ImageNet-shaped
data (224x224x3, 1000 classes), 256 images per GPU (weak scaling), bf16 autocast
compute with f32 master weights, channels_last, SGD momentum 0.9 + wd 1e-4 via
``kungfu_amd.optimizers.SynchronousSGDOptimizer`` (bucketed RCCL all-reduce
overlapped with backward, fused HIP SGD step), one process per GPU.

BERT-base (BASELINE.json config 5): ``--model bert_base --optimizer gns`` trains the
110 M-parameter encoder on synthetic 128-token pre-training batches (MLM on 20
masked positions + NSP, AdamW) through S-SGD with the gradient-noise-scale
monitor and reports sequences/s (and tokens/s in ``config``).

Usage:
    python bench.py [--gpus 1] [--steps 20] [--warmup 5]
    python bench.py --model bert_base --optimizer gns
    python -m torch.distributed.run --nnodes=1 --nproc-per-node N \\
        --master-addr 127.0.0.1 --master-port P bench.py --gpus N --steps K --warmup W
Rank 0 prints ONE JSON line.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

BASELINE_PER_GPU = 5507.0 / 16  # KungFu S-SGD ResNet-50, global batch 4096 on 16 x V100
METRIC = "images/sec/GPU ResNet-50 SynchronousSGD at 1/2/4/8 MI355X; scaling efficiency"
# The reference's other sync-scalability panels (global batch 4096 on 16 x V100):
# (metric, per-GPU baseline img/s) for --model; the headline (default) is ResNet-50.
MODEL_BASELINES = {
    "resnet50": (METRIC, BASELINE_PER_GPU),
    "vgg16": ("images/sec/GPU VGG16 SynchronousSGD at 1/2/4/8 MI355X", 3330.0 / 16),
    "inception_v3": ("images/sec/GPU InceptionV3 SynchronousSGD at 1/2/4/8 MI355X", 7426.0 / 16),
    # BASELINE.json config 5; the reference publishes no BERT number
    "bert_base": ("sequences/sec/GPU BERT-base (seq 128) SynchronousSGD + gradient-noise-scale monitor", None),
}


def _setup_env():
    # MIOpen tuning database shipped in-tree (find results for these shapes),
    # so a fresh box skips the multi-minute exhaustive search.  With several
    # ranks on one node each gets its own copy (no lock contention on the
    # sqlite caches when they compile / look up kernels at the same time).
    tdir = os.path.join(ROOT, "kungfu_amd", "tuning", "miopen")
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if world > 1 and "MIOPEN_USER_DB_PATH" not in os.environ:
        import shutil
        import tempfile

        dst = os.path.join(tempfile.gettempdir(), "kungfu_miopen_%s_%s" % (os.getuid(), os.environ.get("LOCAL_RANK", "0")))
        if not os.path.isdir(dst):
            shutil.copytree(tdir, dst)
        tdir = dst
    os.environ.setdefault("MIOPEN_USER_DB_PATH", tdir)
    os.environ.setdefault("MIOPEN_CUSTOM_CACHE_DIR", tdir)
    os.environ.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=30)
    p.add_argument("--warmup", type=int, default=8)
    p.add_argument("--batch", type=int, default=None, help="images (sequences) per GPU: 256 (BERT: 128)")
    p.add_argument("--model", default="resnet50")
    p.add_argument("--seq-len", type=int, default=128, help="BERT sequence length")
    p.add_argument("--adam", type=int, default=-1, help="1: AdamW inner optimizer (default for BERT), 0: SGD momentum")
    p.add_argument("--optimizer", default="ssgd", choices=["ssgd", "sma", "pair", "ada", "gns", "local"])
    p.add_argument("--force-comm", type=int, default=1,
                   help="1: S-SGD buckets go through the communicator even with one GPU (RCCL 1-rank all-reduce)")
    p.add_argument("--comm-dtype", default="f32", choices=["f32", "bf16"], help="gradient dtype on the wire")
    p.add_argument("--overlap", type=int, default=1, help="S-SGD: all-reduce buckets during backward")
    p.add_argument("--fused-bn", type=int, default=-1, help="1: HIP fused BN(+add)+ReLU; -1: auto")
    p.add_argument("--bucket-mb", type=float, default=None)
    p.add_argument("--bf16-shadow", type=int, default=1,
                   help="1: bf16 compute weights from one cast of the flat f32 master + direct bucket gradients")
    p.add_argument("--lr", type=float, default=0.1)
    p.add_argument("--json-out", default=None)
    a = p.parse_args()
    bert = a.model.startswith("bert")
    if a.batch is None:
        a.batch = 128 if bert else 256
    if a.adam < 0:
        a.adam = 1 if bert else 0
    _setup_env()

    import torch
    import torch.nn.functional as F

    import kungfu_amd as kf
    from kungfu_amd.models import get_model

    kf.init()
    rank, size = kf.current_rank(), kf.current_cluster_size()
    dev_idx = kf.get_hip_index()
    torch.cuda.set_device(dev_idx)
    dev = torch.device("cuda", dev_idx)
    torch.backends.cudnn.benchmark = False  # MIOpen immediate mode + in-tree find-db
    torch.manual_seed(1234)

    fused_bn = a.fused_bn
    if fused_bn < 0:
        from kungfu_amd.ops import fused_bn as fb

        fused_bn = 1 if fb.available() else 0
    model = (get_model(a.model, fused_bn=bool(fused_bn)) if a.model.startswith("resnet") or a.model in ("inception_v3", "vgg16")
             else get_model(a.model))
    model = model.to(dev)
    if not bert:
        model = model.to(memory_format=torch.channels_last)
    if a.adam:
        base = torch.optim.AdamW(model.parameters(), lr=1e-4, weight_decay=0.01)
        opt_desc = "AdamW lr=1e-4 wd=0.01"
    else:
        base = torch.optim.SGD(model.parameters(), lr=a.lr, momentum=0.9, weight_decay=1e-4)
        opt_desc = "SGD momentum=0.9 wd=1e-4"
    comm_dtype = torch.bfloat16 if a.comm_dtype == "bf16" else None
    if a.optimizer == "ssgd":
        opt = kf.optimizers.SynchronousSGDOptimizer(base, named_parameters=model.named_parameters(),
                                                    bucket_mb=a.bucket_mb, overlap=bool(a.overlap),
                                                    force_comm=bool(a.force_comm), comm_dtype=comm_dtype)
    elif a.optimizer == "gns":  # S-SGD + gradient-noise-scale monitor (K5 every step)
        opt = kf.optimizers.MonitorGradientNoiseScaleOptimizer(base, device_batch_size=a.batch,
                                                               named_parameters=model.named_parameters(),
                                                               monitor_single=bool(a.force_comm))
    elif a.optimizer == "local":  # diagnostics only: fused flat SGD, no gradient exchange
        from kungfu_amd.optimizers.core import KungFuOptimizer

        opt = KungFuOptimizer(base, named_parameters=model.named_parameters())
    elif a.optimizer == "sma":
        opt = kf.optimizers.SynchronousAveragingOptimizer(base, named_parameters=model.named_parameters())
    elif a.optimizer == "pair":
        opt = kf.optimizers.PairAveragingOptimizer(base, named_parameters=model.named_parameters())
    else:
        opt = kf.optimizers.AdaptiveSGDOptimizer(base, named_parameters=model.named_parameters(), change_step=10)
    kf.broadcast_parameters(model.state_dict())
    if a.bf16_shadow and getattr(opt, "space", None) is not None:
        from kungfu_amd.parallel.mixed import enable_bf16_shadow

        enable_bf16_shadow(model, opt)

    if bert:
        from kungfu_amd.models.bert import pretraining_loss, synthetic_pretraining_batch

        data = synthetic_pretraining_batch(a.batch, a.seq_len, device=dev)

        def compute_loss():
            return pretraining_loss(model, data)
    else:
        x = torch.randn(a.batch, 3, 224, 224, device=dev).to(memory_format=torch.channels_last)
        y = torch.randint(0, 1000, (a.batch,), device=dev)

        def compute_loss():
            return F.cross_entropy(model(x).float(), y)

    def step():
        opt.zero_grad()
        with torch.autocast("cuda", dtype=torch.bfloat16):
            loss = compute_loss()
        loss.backward()
        opt.step()
        return loss

    t_w0 = time.time()
    first_loss = None
    for i in range(a.warmup):
        l0 = step()
        if i == 0:
            first_loss = float(l0.detach())
    torch.cuda.synchronize()
    warm_s = time.time() - t_w0

    kf.run_barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(a.steps):
        loss = step()
    torch.cuda.synchronize()
    kf.run_barrier()
    dt = time.perf_counter() - t0
    # max over ranks
    dt_t = torch.tensor([dt], dtype=torch.float64)
    dt_max = float(kf.ops.all_reduce(dt_t, op="max")[0]) if size > 1 else dt
    value = a.batch * size * a.steps / dt_max
    reducer = getattr(opt, "reducer", None)
    comm_info = reducer.describe() if reducer is not None else {"comm_ranks": size}
    metric, base_per_gpu = MODEL_BASELINES.get(a.model, (METRIC.replace("ResNet-50", a.model), None))
    unit = "sequences/sec (aggregate over n_gpus)" if bert else "images/sec (aggregate over n_gpus)"
    res = {
        "metric": metric,
        "value": round(value, 2),
        "unit": unit,
        "n_gpus": size,
        "steps": a.steps,
        "warmup": a.warmup,
        "ms_per_step": round(1000 * dt_max / a.steps, 3),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": round(value / (base_per_gpu * size), 3) if base_per_gpu else None,
        "dtype": "bf16",
        "data": ("synthetic (random token ids, 20 masked positions per sequence, random MLM/NSP labels; "
                 "random-init weights)" if bert else
                 "synthetic (random 224x224x3 images, random labels; random-init weights)"),
        "config": {
            "model": a.model,
            "global_batch": a.batch * size,
            "per_gpu_batch": a.batch,
            "seq_len": a.seq_len if bert else None,
            "image_size": None if bert else 224,
            "parallelism": "dp%d" % size,
            "optimizer": "%s(%s)" % (a.optimizer, opt_desc),
            "fused_bn_hip": bool(fused_bn),
            "bf16_shadow_weights": bool(a.bf16_shadow),
            "per_gpu_img_s": round(value / size, 2),
            "tokens_per_s": round(value * a.seq_len, 1) if bert else None,
            "gradient_noise_scale": (opt.noise_scale if a.optimizer == "gns" else None),
            "baseline_per_gpu_img_s": round(base_per_gpu, 1) if base_per_gpu else None,
            "warmup_s": round(warm_s, 1),
            "initial_loss": round(first_loss, 4) if first_loss is not None else None,
            "final_loss": round(float(loss.detach()), 4),
            "comm": comm_info,
        },
    }
    if rank == 0:
        line = json.dumps(res)
        print(line, flush=True)
        if a.json_out:
            with open(a.json_out, "w") as f:
                f.write(line + "\n")
    kf.finalize()


if __name__ == "__main__":
    main()
