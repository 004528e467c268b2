import argparse
import json
import os
import sys
import time

import numpy as np
import torch

import kungfu_amd as kf
from kungfu_amd import ops
from kungfu_amd.benchmarks.model_sizes import grad_sizes


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--method", default="CPU", choices=["CPU", "RCCL", "RCCL+CPU", "HIER", "GRAPH"],
                   help="CPU: host TCP graph plane; RCCL: RCCL all-reduce; RCCL+CPU: host-staged GPU; "
                        "HIER: local RCCL reduce + host cross all-reduce + local bcast; GRAPH: the session's "
                        "strategy graphs as device send/recv rounds (KUNGFU_ALLREDUCE_STRATEGY)")
    p.add_argument("--model", default="resnet50")
    p.add_argument("--fuse", action="store_true")
    p.add_argument("--max-count", type=int, default=0)
    p.add_argument("--steps", type=int, default=10)
    p.add_argument("--warmup-steps", type=int, default=3)
    p.add_argument("--dtype", default="float32")
    a = p.parse_args()
    kf.init()
    rank, np_ = kf.current_rank(), kf.current_cluster_size()
    dtype = getattr(torch, a.dtype)
    sizes = grad_sizes(a.model)
    if a.fuse:
        sizes = [sum(sizes)]
    if a.max_count > 0:
        sizes = sizes[:a.max_count]
    gpu = a.method != "CPU"
    if gpu:
        torch.cuda.set_device(kf.get_hip_index())
        if a.method == "RCCL+CPU":
            os.environ["KUNGFU_GPU_DATAPLANE"] = "host"
    dev = "cuda" if gpu else "cpu"
    xs = [torch.ones(n, dtype=dtype, device=dev) for n in sizes]
    tot = sum(x.numel() * x.element_size() for x in xs)
    mult = 4 * (np_ - 1) if np_ > 1 else 4

    def run():
        if a.method == "HIER":
            for x in xs:
                ops.hierarchical_all_reduce_(x)
        elif a.method == "GRAPH":
            for x in xs:
                ops.monitored_all_reduce_(x)
        else:
            ops.group_all_reduce_(xs, names=["bench:%d" % i for i in range(len(xs))])
        if gpu:
            torch.cuda.synchronize()

    vals = []
    for step in range(a.warmup_steps + a.steps):
        t0 = time.perf_counter()
        run()
        dt = time.perf_counter() - t0
        if step >= a.warmup_steps:
            vals.append(tot * mult / (1 << 30) / dt)
        if rank == 0:
            print("step %d took %.3fs, equivalent data rate %.3f GiB/s" % (step, dt, tot * mult / (1 << 30) / dt))
    if rank == 0:
        v = np.array(vals)
        attrs = {"method": a.method, "np": np_, "model": a.model, "fuse": a.fuse, "tensors": len(xs),
                 "bytes": tot, "strategy": os.environ.get("KUNGFU_ALLREDUCE_STRATEGY")}
        print("RESULT: %f +-%f (GiB/s) %s" % (v.mean(), 1.96 * v.std(), json.dumps(attrs, separators=(",", ":"))))
    kf.finalize()


if __name__ == "__main__":
    main()
