"""Benchmark tools run end to end on the CPU plane (parity: scripts/tests/run-fake-trainer.sh,
run-allreduce-benchmark.sh, kungfu-bench-p2p) and tracing output."""
import os
import subprocess
import sys

import pytest

from conftest import ROOT, kungfu_run


@pytest.mark.parametrize("fuse", [False, True])
def test_fake_trainer_cpu(fuse):
    args = ["-m", "kungfu_amd.benchmarks.fake_trainer", "--model", "resnet18", "--steps", "2", "--epochs", "1"]
    r = kungfu_run(2, args + (["--fuse"] if fuse else []), timeout=240)
    assert r.returncode == 0, r.stdout[-3000:]
    assert "RESULT:" in r.stdout and '"np":2' in r.stdout, r.stdout[-2000:]


def test_allreduce_benchmark_cpu():
    r = kungfu_run(2, ["-m", "kungfu_amd.benchmarks", "--model", "resnet18", "--steps", "2", "--warmup-steps", "1"],
                   timeout=240)
    assert r.returncode == 0, r.stdout[-3000:]
    assert "RESULT:" in r.stdout and "GiB/s" in r.stdout


def test_p2p_benchmark_cpu():
    r = kungfu_run(3, ["-m", "kungfu_amd.benchmarks.p2p", "--model", "resnet18", "--steps", "2", "--epochs", "1"],
                   timeout=240)
    assert r.returncode == 0, r.stdout[-3000:]
    assert "RESULT:" in r.stdout


def test_trace_report_native_and_python():
    code = ("import torch, kungfu_amd as kf\n"
            "from kungfu_amd.utils import trace\n"
            "kf.init()\n"
            "m = torch.nn.Linear(4, 4)\n"
            "o = kf.optimizers.SynchronousSGDOptimizer(torch.optim.SGD(m.parameters(), lr=0.1))\n"
            "m(torch.randn(2, 4)).sum().backward(); o.step()\n"
            "with trace.scope('user::scope'): pass\n"
            "kf.ops.all_reduce(torch.ones(3))\n")
    env = dict(os.environ, KUNGFU_CONFIG_ENABLE_TRACE="true", PYTHONPATH=ROOT)
    r = subprocess.run([sys.executable, "-c", code], env=env, stdout=subprocess.PIPE, stderr=subprocess.STDOUT,
                       text=True, timeout=120)
    assert r.returncode == 0, r.stdout
    for name in ["optimizer::apply", "user::scope", "session::all_reduce"]:
        assert "[trace] " + name in r.stdout, r.stdout


def test_bench_model_baselines():
    """bench.py's per-model metric and per-GPU baseline (BASELINE.md sync panels at
    global batch 4096 on 16 x V100): ResNet-50 is the headline and the default."""
    import importlib.util
    import os

    spec = importlib.util.spec_from_file_location(
        "kf_bench", os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "bench.py"))
    b = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(b)
    assert b.MODEL_BASELINES["resnet50"] == (b.METRIC, 5507.0 / 16)
    assert abs(b.MODEL_BASELINES["vgg16"][1] - 208.1) < 0.1
    assert abs(b.MODEL_BASELINES["inception_v3"][1] - 464.1) < 0.1
    assert all("SynchronousSGD" in m for m, _ in b.MODEL_BASELINES.values())
