"""Worker: RCCL all-reduces captured in hipGraphs (torch.cuda.graph) and replayed, values
checked after every replay.  Phases: ``one`` (one all-reduce on the capture stream), ``two``
(two all-reduces on the capture stream), ``avg`` (ncclAvg), ``ofork`` (compute on a forked stream, the all-reduces on the capture's
origin stream), ``fork`` (two all-reduces on a side comm stream forked
from and joined back into the capture, the S-SGD engine's pattern), ``hook`` (all-reduces issued
from autograd hooks during a captured backward).  Ranks colocated on one GPU
(KUNGFU_RCCL_COLOCATE).  Measured (r4t10, ROCm 7.0 runtime in torch 2.10, RCCL 2.26.6): one / two /
avg replay correctly; ``fork`` crashes hipStreamEndCapture (unbounded recursion inside
libamdhip64 over the captured graph) -- which is why GraphedStep refuses multi-rank RCCL capture."""
import sys

import torch

import kungfu_amd as kf
from kungfu_amd.parallel.comm import get_device_comm
from kungfu_amd.parallel.graphs import track

phases = (sys.argv[1] if len(sys.argv) > 1 else "one,two,avg").split(",")
kf.init()
r, n = kf.current_rank(), kf.current_cluster_size()
dev = torch.device("cuda", kf.get_hip_index())
torch.cuda.set_device(dev)
comm = get_device_comm()
tri = n * (n + 1) // 2
x = torch.zeros(1 << 16, device=dev)
y = torch.zeros(1 << 12, device=dev)
x.fill_(r + 1)
comm.all_reduce(x, op="sum", stream=torch.cuda.current_stream())
torch.cuda.synchronize()
assert torch.all(x == tri)
cap = torch.cuda.Stream()
side = torch.cuda.Stream()
w = torch.nn.Parameter(torch.zeros(256, device=dev))


def body(phase):
    s = torch.cuda.current_stream()
    if phase == "one":
        x.mul_(2)
        comm.all_reduce(x, op="sum", stream=s)
    elif phase == "two":
        x.mul_(2)
        comm.all_reduce(x, op="sum", stream=s)
        comm.all_reduce(y, op="sum", stream=s)
    elif phase == "fork":
        x.mul_(2)
        side.wait_stream(s)
        with torch.cuda.stream(side):
            comm.all_reduce(x, op="sum", stream=side)
            comm.all_reduce(y, op="sum", stream=side)
        s.wait_stream(side)
    elif phase == "ofork":
        # the collectives on the capture's ORIGIN stream, the compute on a forked stream: the
        # layout GraphedStep uses for multi-rank steps
        side.wait_stream(s)
        with torch.cuda.stream(side):
            x.mul_(2)
        s.wait_stream(side)
        comm.all_reduce(x, op="sum", stream=s)
        side.wait_stream(s)
        with torch.cuda.stream(side):
            y.mul_(1)
        comm.all_reduce(y, op="sum", stream=s)
        s.wait_stream(side)
    elif phase == "avg":
        x.mul_(2)
        comm.all_reduce(x, op="avg", stream=s)
    elif phase == "hook":
        (w * x[:256]).sum().backward()
        side.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(side):
            comm.all_reduce(w.grad, op="sum", stream=side)
        torch.cuda.current_stream().wait_stream(side)


def fill(i):
    x.fill_(r + 1 + i)
    y.fill_(2 * (r + 1))
    w.grad = None if w.grad is None else w.grad.zero_()


def check(phase, i):
    if phase == "hook":
        assert torch.all(w.grad == sum(k + 1 + i for k in range(n))), (phase, i, w.grad[:4])
        return
    want = 2 * sum(k + 1 + i for k in range(n)) / (n if phase == "avg" else 1)
    assert torch.all(x == want), (phase, i, x[:4], want)
    if phase == "two":
        assert torch.all(y == 2 * tri), (phase, y[:4])
    if phase in ("fork", "ofork"):
        assert torch.all(y == 2 * tri), (phase, y[:4])


for phase in phases:
    print("RCCL_GRAPH phase %s begin rank=%d" % (phase, r), flush=True)
    cap.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(cap):  # warm-up on the capture stream (autograd's stream for the hook phase)
        fill(0)
        body(phase)
    torch.cuda.synchronize()
    g = track(torch.cuda.CUDAGraph())
    # relaxed, as GraphedStep's segment captures: in the default "global" mode a HIP call from any
    # other thread during the capture (the native RCCL watchdog's hipEventQuery on earlier
    # collectives) invalidates it -- phase two failed that way in a suite run (r6s2c); "thread_local"
    # fails inside RCCL's own enqueue (r6t41)
    with torch.cuda.graph(g, stream=cap, capture_error_mode="relaxed"):
        body(phase)
    print("RCCL_GRAPH phase %s captured rank=%d" % (phase, r), flush=True)
    for i in range(3):
        fill(i)
        g.replay()
        torch.cuda.synchronize()
        check(phase, i)
    print("RCCL_GRAPH phase %s ok rank=%d" % (phase, r), flush=True)
print("RCCL_GRAPH_OK rank=%d np=%d" % (r, n), flush=True)
