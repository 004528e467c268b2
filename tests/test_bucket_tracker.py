"""Native per-gradient bucket accounting (csrc/runtime/scheduler.cpp BucketTracker, used by
parallel/ddp.py's GradReducer): the learning step launches everything at flush(), later steps
launch a bucket when its last expected gradient lands, in the scheduler's order, and report a
gradient of an already launched bucket as late.  Parity: the reference's NCCLScheduler order
(srcs/cpp/src/nccl/scheduler.cpp:9-131) -- collectives start in one agreed order on every rank."""
import pytest

from kungfu_amd._lib import runtime as K


def test_learning_step_launches_at_flush_in_order():
    t = K.BucketTracker(3, [0, 0, 1, 2, 2])
    t.reset()
    assert not t.learned()
    for p in (4, 3, 2, 1, 0):  # backward order
        assert t.mark(p) == []
    assert t.flush() == [0, 1, 2]
    assert t.fires() == [1, 1, 1, 1, 1]
    t.learn()
    assert t.learned() and t.expected() == [1, 1, 1, 1, 1]


def test_learned_step_launches_each_bucket_when_complete_in_order():
    t = K.BucketTracker(3, [0, 0, 1, 2, 2])
    t.reset()
    for p in range(5):
        t.mark(p)
    t.flush()
    t.learn()
    t.set_order([2, 1, 0])  # e.g. the backward arrival order agreed by auto_order
    t.reset()
    assert t.mark(4) == []     # bucket 2 still waits for parameter 3
    assert t.mark(3) == [2]    # bucket 2 complete and first in order
    assert t.mark(0) == []     # bucket 0 waits for parameter 1, and bucket 1 precedes it
    assert t.mark(2) == [1]    # bucket 1 complete, next in order
    assert t.mark(1) == [0]
    assert t.flush() == []
    assert all(t.launched(b) for b in range(3))
    assert t.arrivals() == [2, 1, 0]  # completion order, what auto_order broadcasts


def test_out_of_order_completion_waits_for_the_order():
    t = K.BucketTracker(2, [0, 1])
    t.reset()
    t.mark(0), t.mark(1), t.flush()
    t.learn()
    t.reset()
    assert t.mark(1) == []      # bucket 1 complete but bucket 0 is first in order
    assert t.mark(0) == [0, 1]  # both go, in order


def test_late_gradient_and_repeated_fires():
    t = K.BucketTracker(2, [0, 0, 1])
    t.reset()
    for p in (0, 0, 1, 2):      # parameter 0 used twice in the step: two gradient hooks
        t.mark(p)
    t.flush()
    t.learn()
    assert t.expected() == [2, 1, 1]
    t.reset()
    assert t.mark(0) == [] and t.mark(1) == []  # bucket 0 needs parameter 0's second fire
    assert t.mark(0) == [0]
    assert t.mark(0) == [K.BucketTracker.LATE]  # an unexpected extra fire after the launch
    assert t.mark(2) == [1]


def test_bad_indices_raise():
    with pytest.raises(Exception):
        K.BucketTracker(2, [0, 2])
    t = K.BucketTracker(1, [0])
    with pytest.raises(Exception):
        t.mark(5)
