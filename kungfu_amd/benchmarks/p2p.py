"""Peer-to-peer model-request benchmark: every peer saves a model-sized blob in its store and
repeatedly pulls a peer's copy (the pair-averaging access pattern).

Parity: tests/go/cmd/kungfu-bench-p2p/kungfu-bench-p2p.go:42-120.

    kungfu-run -np 4 -H 127.0.0.1:4 python -m kungfu_amd.benchmarks.p2p --model resnet50
    ... --device   # HIP-IPC device model store + one-sided xGMI pulls (DeviceModelStore)
"""
from __future__ import annotations

import argparse
import json
import time

import numpy as np
import torch

import kungfu_amd as kf
from kungfu_amd import ops
from kungfu_amd.benchmarks.model_sizes import grad_sizes


def main(argv=None):
    p = argparse.ArgumentParser()
    p.add_argument("--model", default="resnet50")
    p.add_argument("--steps", type=int, default=10)
    p.add_argument("--epochs", type=int, default=3)
    p.add_argument("--device", action="store_true", help="device store with HIP-IPC one-sided pulls")
    a = p.parse_args(argv)
    kf.init()
    rank, np_ = kf.current_rank(), kf.current_cluster_size()
    n = sum(grad_sizes(a.model))
    if a.device:
        from kungfu_amd.optimizers.pair_avg import DeviceModelStore

        dev = torch.device("cuda", kf.get_hip_index())
        torch.cuda.set_device(dev)
        model = torch.full((n,), float(rank), device=dev)
        store = DeviceModelStore(n, dev, "bench")
        store.publish(model)
        store.advertise()
        other = torch.empty_like(model)
    else:
        model = torch.full((n,), float(rank))
        ops.save_variable(model, name="bench:model")
    kf.run_barrier()
    rates = []
    for ep in range(a.epochs):
        t0 = time.perf_counter()
        for s in range(a.steps):
            target = (rank + 1 + s % max(np_ - 1, 1)) % np_ if np_ > 1 else 0
            if a.device:
                ok = store.pull(target, other) if target != rank else True
                torch.cuda.synchronize()
                assert ok
            else:
                got = ops.request_variable(target, "bench:model", (n,), torch.float32)
                assert got is not None and float(got[0]) == float(target)
        dt = (time.perf_counter() - t0) / a.steps
        rates.append(n * 4 / dt / (1 << 30))
        if rank == 0:
            print("epoch %d: %.2f ms/request, %.2f GiB/s" % (ep, 1e3 * dt, rates[-1]), flush=True)
    kf.run_barrier()
    if rank == 0:
        v = np.array(rates)
        print("RESULT: %f +-%f (GiB/s) %s" % (v.mean(), 1.96 * v.std(), json.dumps(
            {"model": a.model, "np": np_, "device": a.device, "bytes": n * 4}, separators=(",", ":"))), flush=True)
    kf.finalize()


if __name__ == "__main__":
    main()
