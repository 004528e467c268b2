"""Worker: rank 1 never joins a host all-reduce; rank 0's op watchdog must end the job
(exit 3) naming the stalled op, well before the test's own timeout.

Parity: the reference's stall detector around every collective
(srcs/go/libkungfu-comm/main.go:163-179, srcs/go/utils/stalldetector.go:9-46)."""
import time

import torch

import kungfu_amd as kf

kf.init()
r = kf.current_rank()
kf.run_barrier()
if r == 1:
    time.sleep(60)  # "hung" peer
else:
    kf.ops.all_reduce(torch.ones(4), name="the-stalled-allreduce")
print("STALL_NOT_DETECTED rank=%d" % r, flush=True)
