"""Python API in single mode (np=1, no launcher) -- parity: tests/python/unit/test_op.py,
test_helper_apis.py, test_tensorflow_policy.py (counter, EMA, step schedule, detached,
rank/size, global variables, policy hook) plus the local tensor utilities."""
import torch

import kungfu_amd as kf
from kungfu_amd import ops
from kungfu_amd import variables as kv


def setup_module(_):
    kf.init()


def test_rank_size_detached():
    assert kf.current_rank() == 0 and kf.current_cluster_size() == 1
    assert kf.current_local_rank() == 0 and kf.current_local_size() == 1
    assert not kf.detached()
    assert ops.peer_info() == (0, 1)
    kf.run_barrier()
    assert isinstance(kf.uid(), int)


def test_counter_and_ema():
    c = ops.counter(init=3, incr=2)
    assert [c() for _ in range(3)] == [3, 5, 7]
    e = ops.exponential_moving_average(alpha=0.5)
    assert e(4.0) == 4.0 and e(0.0) == 2.0 and e(2.0) == 2.0
    from kungfu_amd.utils import EMA

    m = EMA(0.9)
    for v in [1.0, 1.0, 1.0]:
        m.update(v)
    assert abs(m.get() - 1.0) < 1e-9


def test_step_based_schedule():
    s = ops.StepBasedSchedule("1:2,2:3,4:1")
    assert [s(i) for i in range(7)] == [1, 1, 2, 2, 2, 4, 1]
    assert ops.step_based_schedule("1:2,2:3", 3) == 2
    import pytest

    with pytest.raises(ValueError):
        ops.StepBasedSchedule("1:2", strict=True)(5)
    with pytest.raises(ValueError):
        ops.StepBasedSchedule("")


def test_single_mode_collectives_are_identity():
    x = torch.arange(10, dtype=torch.float32)
    assert torch.equal(ops.all_reduce(x), x)
    assert torch.equal(ops.broadcast(x), x)
    assert ops.all_gather(x).shape == (1, 10)
    assert ops.consensus(x)
    ops.save_variable(x, name="single:x")
    assert torch.equal(ops.request_variable(0, "single:x", (10,), torch.float32), x)


def test_fuse_defuse_and_mst():
    ts = [torch.randn(3, 4), torch.randn(5), torch.randn(2, 2, 2)]
    flat = ops.fuse(ts)
    assert flat.numel() == 12 + 5 + 8
    back = ops.defuse(flat, ts)
    assert all(torch.equal(a, b) for a, b in zip(ts, back))
    w = torch.tensor([[0, 1, 9], [1, 0, 2], [9, 2, 0]], dtype=torch.float32)
    f = ops.mst_father(w, root=0)
    assert f == [0, 0, 1]
    mask = ops.get_neighbour_mask(torch.tensor([[0, 1], [1, 2]]), cluster_size=3, self_rank=1)
    assert mask.tolist() == [True, False, True]
    rr = ops.RoundRobin()
    picks = [rr(torch.tensor([True, False, True])) for _ in range(4)]
    assert picks == [0, 2, 0, 2]


def test_global_variables_and_policy_hook():
    kv.reset()
    assert kv.get_or_create_batch_size(32) == 32
    kv.set_global_variable(kv.GraphKeys.BATCH_SIZE, 64)
    assert kv.eval_batch_size() == 64

    from kungfu_amd.policy import BasePolicy, PolicyHook

    calls = []

    class P(BasePolicy):
        def before_epoch(self):
            calls.append("be")

        def after_epoch(self):
            calls.append("ae")

        def after_train(self):
            calls.append("at")

    h = PolicyHook([P()], epoch_size=128, epoch_num=2, init_batch_size=64)
    steps = 0
    while True:
        h.before_step()
        steps += 1
        if h.after_step():
            break
    h.end()
    assert steps == 4  # 2 epochs x 128 samples / 64 per step
    assert calls.count("be") == 2 and calls.count("ae") == 2 and calls[-1] == "at"
    assert kv.get_global_variable(kv.GraphKeys.TRAINED_SAMPLES) == 256
