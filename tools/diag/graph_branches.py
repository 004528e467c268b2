"""Do independent branches of a captured hipGraph run concurrently on this ROCm?

Two streams forked from the capture stream each run K single-wave sleep kernels
(torch.cuda._sleep); eagerly the two streams overlap (time ~ K sleeps), a graph whose branches run
concurrently replays in the same time, a serialising graph executor in ~2x.  Explains why the
captured step hides side-stream work (bucket all-reduces, GNS monitors) worse than eager streams
(profiles/r4_host_overhead.md)."""
import time

import torch

K, CYC = 20, 2_000_000
dev = torch.device("cuda")
a, b = torch.cuda.Stream(), torch.cuda.Stream()


def body():
    cur = torch.cuda.current_stream()
    a.wait_stream(cur)
    b.wait_stream(cur)
    with torch.cuda.stream(a):
        for _ in range(K):
            torch.cuda._sleep(CYC)
    with torch.cuda.stream(b):
        for _ in range(K):
            torch.cuda._sleep(CYC)
    cur.wait_stream(a)
    cur.wait_stream(b)


def timed(fn, n=5):
    fn()
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(n):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t) / n * 1e3


def one_stream():
    for _ in range(2 * K):
        torch.cuda._sleep(CYC)


serial = timed(one_stream)
eager = timed(body)
g = torch.cuda.CUDAGraph()
s = torch.cuda.Stream()
s.wait_stream(torch.cuda.current_stream())
with torch.cuda.stream(s):
    body()
torch.cuda.synchronize()
with torch.cuda.graph(g):
    body()
graph = timed(g.replay)
print("one stream, 2K sleeps: %.2f ms | two streams eager: %.2f ms | two branches in one graph: %.2f ms"
      % (serial, eager, graph), flush=True)
print("graph branches concurrent: %s" % (graph < 0.75 * serial), flush=True)
