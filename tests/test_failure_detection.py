"""Failure detection and the self-launching, self-verifying bench (CPU, multi-process).

Parity: the reference checks every NCCL result and wraps every op in a stall detector
(srcs/cpp/src/nccl/gpu_collective.cpp:96-128, srcs/go/libkungfu-comm/main.go:163-179);
the device-plane watchdog itself runs in tests/test_gpu_rccl.py."""
import json
import os
import subprocess
import sys
import time

from conftest import ROOT, kungfu_run, worker


def test_host_op_watchdog_names_stalled_op():
    t0 = time.time()
    r = kungfu_run(2, [worker("stall.py")], timeout=90, env={"KUNGFU_OP_TIMEOUT_S": "3"})
    dt = time.time() - t0
    assert r.returncode != 0, r.stdout[-3000:]
    assert "STALL_NOT_DETECTED" not in r.stdout
    assert "the-stalled-allreduce" in r.stdout and "has not completed" in r.stdout, r.stdout[-3000:]
    assert dt < 45, dt


def _bench(args, env=None, timeout=300):
    e = dict(os.environ)
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT", "KUNGFU_SELF_SPEC"):
        e.pop(k, None)
    e.update(env or {})
    return subprocess.run([sys.executable, os.path.join(ROOT, "bench.py")] + args, stdout=subprocess.PIPE,
                          stderr=subprocess.PIPE, text=True, timeout=timeout, env=e, cwd="/tmp")


def test_bench_self_launches_and_verifies_replicas():
    r = _bench(["--gpus", "2", "--steps", "2", "--warmup", "1", "--device", "cpu", "--model", "resnet18",
                "--batch", "2", "--image-size", "32"])
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout  # rank 0 only
    res = json.loads(lines[0])
    assert res["n_gpus"] == 2 and res["config"]["parallelism"] == "dp2"
    v = res["verify"]
    assert v["world_size"] == 2 and v["comm_ranks"] == 2 and v["launch"] == "torchrun"
    assert v["replicas_consistent"] is True
    assert v["per_rank_img_s"]["min"] <= v["per_rank_img_s"]["max"]


def test_bench_refuses_mislabelled_world():
    # a launcher env with one rank but --gpus 2 must fail, not report a 1-rank number as 2
    r = _bench(["--gpus", "2", "--steps", "1", "--warmup", "0", "--device", "cpu", "--model", "resnet18",
                "--batch", "2", "--image-size", "32"], env={"WORLD_SIZE": "1", "RANK": "0"})
    assert r.returncode == 2, (r.returncode, r.stderr[-2000:])
    assert "refusing" in r.stderr
