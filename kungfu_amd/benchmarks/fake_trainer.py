"""Fake trainer: replays a real model's gradient size list through the distributed
gradient path with no model compute, and reports the img/s the cluster would reach at a
given per-GPU compute rate.

Parity: tests/cpp/integration/fake_trainer.hpp:16-227 (fake gradients from the
resnet50/vgg16/bert size tables, 11 x 10 steps, img/s at an assumed compute rate) and
tests/cpp/integration/fake_in_proc_trainer.cpp.

    kungfu-run -np 4 -H 127.0.0.1:4 python -m kungfu_amd.benchmarks.fake_trainer \\
        --model resnet50 --method CPU
    torchrun --nproc-per-node 8 -m kungfu_amd.benchmarks.fake_trainer --method RCCL --fuse

Methods: CPU (host graph plane, per-tensor async + wait-all), RCCL (device all-reduce of
the flat gradient buffer in buckets, as the S-SGD engine does), GRAPH (device strategy
graphs), HOST (GPU tensors staged through the host plane).
"""
from __future__ import annotations

import argparse
import json
import os
import time

import numpy as np
import torch

import kungfu_amd as kf
from kungfu_amd import ops
from kungfu_amd.benchmarks.model_sizes import grad_sizes


def main(argv=None):
    p = argparse.ArgumentParser()
    p.add_argument("--model", default="resnet50")
    p.add_argument("--method", default="CPU", choices=["CPU", "RCCL", "GRAPH", "HOST"])
    p.add_argument("--fuse", action="store_true", help="one flat buffer instead of per-tensor collectives")
    p.add_argument("--bucket-mb", type=float, default=32.0)
    p.add_argument("--batch", type=int, default=256, help="images per worker per step")
    p.add_argument("--compute-img-s", type=float, default=9800.0,
                   help="assumed per-worker compute throughput (MI355X ResNet-50 bf16 ~9.8k img/s)")
    p.add_argument("--dtype", default="float32")
    p.add_argument("--steps", type=int, default=10)
    p.add_argument("--epochs", type=int, default=3)
    p.add_argument("--warmup", type=int, default=1)
    a = p.parse_args(argv)
    if a.method == "HOST":
        os.environ["KUNGFU_GPU_DATAPLANE"] = "host"
    kf.init()
    rank, np_ = kf.current_rank(), kf.current_cluster_size()
    gpu = a.method != "CPU"
    dev = torch.device("cuda", kf.get_hip_index()) if gpu else torch.device("cpu")
    if gpu:
        torch.cuda.set_device(dev)
    dt = getattr(torch, a.dtype)
    sizes = grad_sizes(a.model)
    total = sum(sizes)
    flat = torch.ones(total, dtype=dt, device=dev)
    views, off = [], 0
    for n in sizes:
        views.append(flat[off:off + n])
        off += n
    names = ["fake:%d" % i for i in range(len(views))]
    comm = None
    if gpu and a.method in ("RCCL", "GRAPH"):
        from kungfu_amd.parallel.comm import get_device_comm

        comm = get_device_comm()
    esz = flat.element_size()
    cap = max(1, int(a.bucket_mb * (1 << 20) / esz))

    def step():
        if a.method == "CPU":
            if a.fuse:
                ops.inplace_all_reduce_op(flat, op="sum", name="fake:fused")
            else:
                ops.group_all_reduce_(views, op="sum", names=names)
        elif a.method == "HOST":
            ops.inplace_all_reduce_op(flat, op="sum", name="fake:fused") if a.fuse else \
                ops.group_all_reduce_(views, op="sum", names=names)
            torch.cuda.synchronize()
        else:
            s = torch.cuda.current_stream()
            chunks = [flat] if a.fuse else [flat[i:i + cap] for i in range(0, total, cap)]
            for c in chunks:
                if a.method == "RCCL":
                    comm.all_reduce(c, op="sum", stream=s)
                else:
                    comm.graph_all_reduce(c, op="sum", stream=s)
            torch.cuda.synchronize()

    for _ in range(a.warmup):
        step()
    rates = []
    for ep in range(a.epochs):
        t0 = time.perf_counter()
        for _ in range(a.steps):
            step()
        dt_comm = (time.perf_counter() - t0) / a.steps
        t_compute = a.batch / a.compute_img_s
        rate = np_ * a.batch / (t_compute + dt_comm)
        rates.append(rate)
        if rank == 0:
            print("epoch %d: comm %.2f ms/step (%.2f GiB/s algo), %.1f img/s at %.0f img/s/worker compute"
                  % (ep, 1e3 * dt_comm, total * esz / dt_comm / (1 << 30), rate, a.compute_img_s), flush=True)
    if rank == 0:
        v = np.array(rates)
        attrs = {"model": a.model, "method": a.method, "np": np_, "fuse": a.fuse, "tensors": len(sizes),
                 "bytes": total * esz, "batch": a.batch, "strategy": os.environ.get("KUNGFU_ALLREDUCE_STRATEGY")}
        print("RESULT: %f +-%f (img/s) %s" % (v.mean(), 1.96 * v.std(), json.dumps(attrs, separators=(",", ":"))),
              flush=True)
    kf.finalize()


if __name__ == "__main__":
    main()
