"""Where do the BERT step's small kernels come from?  Runs the bench's BERT-base step (S-SGD, bf16
shadow weights) under torch.profiler with Python stacks and prints, per aten op among fill_/zero_/
copy_/add/embedding ops, the launch count per step and the innermost kungfu_amd / bench frames.
Also times the embedding gradient (ours vs torch) at the bench's shapes."""
import collections
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, ".")


def main():
    import kungfu_amd as kf
    from kungfu_amd.models import get_model
    from kungfu_amd.models.bert import pretraining_loss, synthetic_pretraining_batch
    from kungfu_amd.parallel.mixed import enable_bf16_shadow

    kf.init()
    dev = torch.device("cuda")
    torch.manual_seed(0)
    model = get_model("bert_base").to(dev)
    base = torch.optim.AdamW(model.parameters(), lr=1e-4, weight_decay=0.01)
    opt = kf.optimizers.SynchronousSGDOptimizer(base, named_parameters=model.named_parameters())
    enable_bf16_shadow(model, opt)
    data = synthetic_pretraining_batch(128, 128, device=dev)

    def step():
        opt.zero_grad()
        with torch.autocast("cuda", dtype=torch.bfloat16):
            loss = pretraining_loss(model, data)
        loss.backward()
        opt.step()

    for _ in range(3):
        step()
    torch.cuda.synchronize()
    steps = 2
    with torch.profiler.profile(activities=[torch.profiler.ProfilerActivity.CPU], with_stack=True,
                                record_shapes=True) as prof:
        for _ in range(steps):
            step()
        torch.cuda.synchronize()
    want = ("aten::fill_", "aten::zero_", "aten::copy_", "aten::add", "aten::add_", "aten::embedding",
            "aten::embedding_backward", "aten::sum", "aten::to", "aten::zeros", "aten::zeros_like")
    rows = collections.Counter()
    for ev in prof.events():
        if ev.name not in want:
            continue
        st = [f for f in (ev.stack or []) if ("kungfu_amd" in f or "bench" in f or "torch/autograd" in f)]
        where = " <- ".join(s.split("/")[-1] for s in st[:3]) or "(autograd engine)"
        shp = str(ev.input_shapes[:2]) if ev.input_shapes else ""
        rows[(ev.name, shp[:70], where[:160])] += 1
    for (name, shp, where), n in sorted(rows.items(), key=lambda kv: -kv[1]):
        if n >= steps:
            print("%5.1f/step %-22s %-70s %s" % (n / steps, name, shp, where))

    # embedding gradient: ours vs torch at the bench's shapes
    from kungfu_amd._lib import hip

    B, S, D = 128, 128, 768
    cases = {"tok": (30522, torch.randint(0, 30522, (B, S), device=dev)),
             "typ": (2, (torch.arange(S, device=dev) >= S // 2).long().expand(B, S).contiguous()),
             "pos": (512, torch.arange(S, device=dev))}
    for name, (V, ids) in cases.items():
        dy = torch.randn(*ids.shape, D, device=dev)
        grad = torch.zeros(V, D, device=dev)
        w = torch.zeros(V, D, device=dev, requires_grad=True)

        def ours(ch):
            def f():
                grad.zero_()
                hip().embedding_backward(grad, ids.reshape(-1), dy, ch)
            return f

        def theirs():
            torch.ops.aten.embedding_dense_backward(dy, ids, V, -1, False)

        for fn, lab in [(ours(c), "ours ch=%d" % c) for c in (0, 4, 16, 64, 128)] + [(theirs, "torch")]:
            for _ in range(3):
                fn()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(20):
                fn()
            e1.record()
            torch.cuda.synchronize()
            print("embedding grad %s V=%d T=%d: %s %.1f us" % (name, V, ids.numel(), lab, e0.elapsed_time(e1) * 50))


if __name__ == "__main__":
    main()
