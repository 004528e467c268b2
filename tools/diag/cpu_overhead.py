"""Is the training step CPU-bound?  Runs the bench's ResNet-50 S-SGD step (same setup as
bench.py) and reports, per step, the host time spent enqueueing it (no synchronisation) next
to the GPU time per step (events).  If the host time is close to the GPU time, the GPU starves
wherever the host falls behind (the fwd/bwd boundary gaps in the kernel trace).
Also times the forward / backward / optimizer phases on the host."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
os.environ.setdefault("MIOPEN_USER_DB_PATH", os.path.join(ROOT, "kungfu_amd", "tuning", "miopen"))
import torch
import torch.nn.functional as F

import kungfu_amd as kf
from kungfu_amd.models import get_model
from kungfu_amd.parallel.mixed import enable_bf16_shadow


def main():
    """argv[1]: resnet50 | inception_v3 | vgg16 | bert_base; GRAPH=1: replay a captured step."""
    model_name = sys.argv[1] if len(sys.argv) > 1 else "resnet50"
    kf.init()
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    bert = model_name.startswith("bert")
    model = get_model(model_name, fused_bn=True) if not bert else get_model(model_name)
    model = model.to(dev)
    if not bert:
        model = model.to(memory_format=torch.channels_last)
        base = torch.optim.SGD(model.parameters(), lr=0.1, momentum=0.9, weight_decay=1e-4)
    else:
        base = torch.optim.AdamW(model.parameters(), lr=1e-4, weight_decay=0.01)
    opt = kf.optimizers.SynchronousSGDOptimizer(base, named_parameters=model.named_parameters(), force_comm=True)
    enable_bf16_shadow(model, opt)
    if bert:
        from kungfu_amd.models.bert import pretraining_loss, synthetic_pretraining_batch

        data = synthetic_pretraining_batch(128, 128, device=dev)

        def compute_loss():
            return pretraining_loss(model, data)
    else:
        x = torch.randn(256, 3, 224, 224, device=dev).to(memory_format=torch.channels_last)
        y = torch.randint(0, 1000, (256,), device=dev)

        def compute_loss():
            return F.cross_entropy(model(x).float(), y)
    ph = {"zero": 0.0, "fwd": 0.0, "bwd": 0.0, "step": 0.0}

    def step():
        t0 = time.perf_counter()
        opt.zero_grad()
        t1 = time.perf_counter()
        with torch.autocast("cuda", dtype=torch.bfloat16):
            loss = compute_loss()
        t2 = time.perf_counter()
        loss.backward()
        t3 = time.perf_counter()
        opt.step()
        t4 = time.perf_counter()
        for k, a, b in (("zero", t0, t1), ("fwd", t1, t2), ("bwd", t2, t3), ("step", t3, t4)):
            ph[k] += b - a

    run = step
    if os.environ.get("GRAPH") == "1":  # whole-step hipGraph: host cost of a replay
        from kungfu_amd.parallel.graphs import GraphedStep

        run = GraphedStep(step, opt, warmup=3)
    for _ in range(5):
        run()
    torch.cuda.synchronize()
    for k in ph:
        ph[k] = 0.0
    n = 20
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    h0 = time.perf_counter()
    for _ in range(n):
        run()
    h1 = time.perf_counter()
    e1.record()
    torch.cuda.synchronize()
    h2 = time.perf_counter()
    print("host enqueue %.2f ms/step, wall %.2f ms/step, gpu %.2f ms/step" % (
        1e3 * (h1 - h0) / n, 1e3 * (h2 - h0) / n, e0.elapsed_time(e1) / n))
    print("host phases (ms/step): " + ", ".join("%s %.2f" % (k, 1e3 * v / n) for k, v in ph.items()))
    # the loop above lets the host run ahead until the launch queue pushes back, so its "enqueue" time
    # includes waiting for the GPU; here every step starts with the GPU idle: the host's own cost
    cold = []
    for _ in range(n):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        run()
        cold.append(time.perf_counter() - t0)
    torch.cuda.synchronize()
    cold.sort()
    print("host enqueue from an idle GPU (no backpressure): median %.2f ms/step, min %.2f" % (
        1e3 * cold[len(cold) // 2], 1e3 * cold[0]))
    if os.environ.get("CPROFILE"):
        import cProfile
        import pstats

        pr = cProfile.Profile()
        pr.enable()
        for _ in range(5):
            step()
        pr.disable()
        torch.cuda.synchronize()
        pstats.Stats(pr).sort_stats("tottime").print_stats(45)
        pstats.Stats(pr).sort_stats("cumulative").print_stats(45)
    kf.finalize()


if __name__ == "__main__":
    main()
