"""Elastic resize with the flat-buffer training engines.

The engines (bucketed S-SGD with its ordered scheduler, the gradient-noise-scale monitor,
SMA, AdaSGD) run here on CPU peers over the host transport (``HostComm``) -- the same
Python engine code as on GPU, minus the RCCL calls -- under ``kungfu-run -w`` with the
builtin config server, like the reference's resize test
(``tests/python/integration/test_tensorflow_resize.py``,
``srcs/python/kungfu/tensorflow/experimental/hook/elastic.py:68-84``).
"""
import os
import re
import subprocess
import sys

import pytest
import torch

from conftest import ROOT, free_port_block, kungfu_run, worker

ENV = {"OMP_NUM_THREADS": "1"}


def _elastic(args, timeout=240):
    base = free_port_block(16)
    cfg = base + 15
    return kungfu_run(1, [worker("elastic_train.py")] + args, timeout=timeout, port_base=base, env=ENV,
                      extra=["-w", "-builtin-config-port", str(cfg), "-config-server",
                             "http://127.0.0.1:%d/config" % cfg, "-H", "127.0.0.1:4"])


def _steps(out):
    """{step: {rank: hash}} and {step: np} from the worker's STEP lines."""
    hs, nps = {}, {}
    for st, np_, rk, h in re.findall(r"STEP (\d+) np=(\d+) rank=(\d+) loss=\S+ h=(\w+)", out):
        hs.setdefault(int(st), {})[int(rk)] = h
        nps[int(st)] = int(np_)
    return hs, nps


def test_ssgd_elastic_matches_single_process_simulation():
    """1 -> 2 -> 1 peers: after every resize all replicas are bit-identical to a single
    process that averages the same shards' gradients -- the joiner received the model,
    the momentum buffer AND the fused optimizer's first-step flag, and the surviving
    worker's bucket reducer re-bound its communicator, peer count and collective order."""
    sched = "1:3,2:3,1:3"
    r = _elastic(["--schedule", sched, "--max-step", "9", "--optimizer", "ssgd"])
    assert r.returncode == 0, r.stdout[-5000:]
    hs, nps = _steps(r.stdout)
    assert [nps[s] for s in range(9)] == [1, 1, 1, 2, 2, 2, 1, 1, 1], nps
    sim = subprocess.run([sys.executable, worker("elastic_train.py"), "--simulate", "--schedule", sched,
                          "--max-step", "9"], stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True,
                         timeout=120, env=dict(os.environ, PYTHONPATH=ROOT, **ENV))
    assert sim.returncode == 0, sim.stdout[-3000:]
    ref = {int(s): h for s, h in re.findall(r"SIM (\d+) np=\d+ h=(\w+)", sim.stdout)}
    for s in range(9):
        assert len(hs[s]) == nps[s], (s, hs[s])
        assert set(hs[s].values()) == {ref[s]}, (s, hs[s], ref[s])
    m = re.search(r"ELASTIC_TRAIN_DONE rank=0 np=1 step=9 v=(\d+) rebinds=(\d+)", r.stdout)
    assert m and int(m.group(1)) == 2 and int(m.group(2)) == 2, r.stdout[-2000:]
    assert r.stdout.count("ELASTIC_TRAIN_DETACHED") == 1


def test_gns_monitor_elastic():
    """The gradient-noise-scale monitor reads the peer count at every step: no estimate
    with one peer, a finite one after growing to two, replicas identical throughout."""
    r = _elastic(["--schedule", "1:2,2:4,1:2", "--max-step", "8", "--optimizer", "gns"])
    assert r.returncode == 0, r.stdout[-5000:]
    hs, nps = _steps(r.stdout)
    for s, by_rank in hs.items():
        assert len(set(by_rank.values())) == 1, (s, by_rank)
    gns = [float(v) for v in re.findall(r"np=2 rank=\d+ loss=\S+ h=\w+ gns=(\S+)", r.stdout) if v != "None"]
    assert gns and all(abs(v) < 1e9 for v in gns), r.stdout[-3000:]


@pytest.mark.parametrize("opt", ["sma", "ada"])
def test_model_averaging_elastic(opt):
    """SMA / AdaSGD through grow and shrink: the pending model average is re-issued on
    the new communicator (no deadlock, no stale average); AdaSGD's S-SGD phase keeps
    replicas identical."""
    r = _elastic(["--schedule", "1:2,2:4,1:2", "--max-step", "8", "--optimizer", opt])
    assert r.returncode == 0, r.stdout[-5000:]
    assert "ELASTIC_TRAIN_DONE rank=0 np=1 step=8" in r.stdout, r.stdout[-3000:]
    hs, nps = _steps(r.stdout)
    assert sorted(hs) == list(range(8))
    if opt == "ada":  # change_step=4: steps 4 and 5 run S-SGD with two peers
        for s in (4, 5):
            assert len(hs[s]) == 2 and len(set(hs[s].values())) == 1, (s, hs[s])


def test_shared_parameter_buckets_two_ranks():
    r = kungfu_run(2, [worker("shared_param.py")], timeout=120, env=ENV)
    assert r.returncode == 0, r.stdout[-4000:]
    assert r.stdout.count("SHARED_OK") == 2


def test_late_direct_gradient_raises():
    """A direct gradient (bf16-shadow sink) delivered after its bucket launched is an
    error while a collective is in flight, not a silent race."""
    import kungfu_amd as kf
    from kungfu_amd.parallel.ddp import GradReducer, LateGradientError
    from kungfu_amd.parallel.flat import FlatParamSpace

    kf.init()
    w = torch.nn.Parameter(torch.randn(4))
    v = torch.nn.Parameter(torch.randn(4))
    space = FlatParamSpace([w, v])
    red = GradReducer(space, skip_single=False)  # one peer, but every bucket goes through the comm

    class Use(torch.autograd.Function):
        @staticmethod
        def forward(ctx, p):
            return p.detach().clone()

        @staticmethod
        def backward(ctx, g):
            space.sink.put(space.index(w), g)
            return None

    def step(uses):
        space.zero_grad()
        x = v * 1.0
        for _ in range(uses):
            x = x + Use.apply(w)
        x.sum().backward()

    step(1)
    step(1)
    assert torch.equal(space.grad_view(space.index(w)), torch.ones(4))
    with pytest.raises(LateGradientError):
        step(2)


def test_broadcast_optimizer_state_scalars():
    """Host-side optimizer scalars travel with broadcast_optimizer_state (single mode: identity)."""
    import kungfu_amd as kf
    from kungfu_amd.initializer import broadcast_optimizer_state

    kf.init()
    m = torch.nn.Linear(3, 2)
    opt = kf.optimizers.SynchronousSGDOptimizer(torch.optim.SGD(m.parameters(), lr=0.1, momentum=0.9), flat=True)
    assert opt.inner._first is True
    m(torch.randn(2, 3)).sum().backward()
    opt.step()
    assert opt.inner._first is False
    broadcast_optimizer_state(opt)
    assert opt.inner._first is False
