"""GPU tests of the S-SGD engine's data plane: the RCCL path exercised
with one rank (``force_comm``), bf16 gradients on the wire, and elastic resize of the
GPU optimizers (2 ranks sharing the GPU over the host-staged plane)."""
import re

import pytest
import torch
import torch.nn.functional as F

from conftest import free_port_block, kungfu_run, worker

pytestmark = pytest.mark.gpu
needs_gpu = pytest.mark.skipif(not torch.cuda.is_available(), reason="no GPU")


@pytest.fixture(scope="module")
def H():
    from kungfu_amd._lib import hip

    return hip()


@needs_gpu
@pytest.mark.parametrize("n", [1, 7, 4096, (1 << 20) + 5])
def test_cast_copy_kernel(H, n):
    x = torch.randn(n, device="cuda") * 3
    b = torch.empty(n, dtype=torch.bfloat16, device="cuda")
    H.cast_copy(b, x, 0.5)
    assert torch.equal(b, (x * 0.5).bfloat16())
    y = torch.empty(n, device="cuda")
    H.cast_copy(y, b, 2.0)
    assert torch.equal(y, b.float() * 2.0)


def _mlp_run(force_comm, comm_dtype=None, steps=3):
    import kungfu_amd as kf

    kf.init()
    torch.manual_seed(0)
    m = torch.nn.Sequential(torch.nn.Linear(64, 256), torch.nn.ReLU(), torch.nn.Linear(256, 10)).cuda()
    opt = kf.optimizers.SynchronousSGDOptimizer(torch.optim.SGD(m.parameters(), lr=0.1, momentum=0.9),
                                                force_comm=force_comm, comm_dtype=comm_dtype)
    g = torch.Generator(device="cuda").manual_seed(1)
    grads = []
    for _ in range(steps):
        x = torch.randn(32, 64, device="cuda", generator=g)
        y = torch.randint(0, 10, (32,), device="cuda", generator=g)
        opt.zero_grad()
        F.cross_entropy(m(x), y).backward()
        grads.append(opt.space.flat_grad.clone())
        opt.step()
    torch.cuda.synchronize()
    return opt, grads


@needs_gpu
def test_force_comm_rccl_one_rank_matches_skip():
    """Every bucket through the comm stream + events + a 1-rank RCCL all-reduce (avg):
    bit-identical to the skip path, and the reducer reports the RCCL plane."""
    o_skip, g_skip = _mlp_run(False)
    o_rccl, g_rccl = _mlp_run(True)
    d = o_rccl.reducer.describe()
    assert d["comm_plane"] == "rccl" and d["comm_ranks"] == 1 and d["comm_bytes_per_step"] > 0, d
    assert o_skip.reducer.describe()["comm_plane"] == "skip"
    for a, b in zip(g_skip, g_rccl):
        assert torch.equal(a, b)
    assert torch.equal(o_skip.space.flat_param, o_rccl.space.flat_param)


@needs_gpu
def test_bf16_gradient_comm_within_rounding():
    """bf16 on the wire: the averaged gradient equals the f32 one rounded to bf16."""
    _, g32 = _mlp_run(True, steps=1)
    o16, g16 = _mlp_run(True, comm_dtype=torch.bfloat16, steps=1)
    assert o16.reducer.describe()["comm_dtype"] == "bfloat16"
    assert torch.equal(g16[0], g32[0].bfloat16().float())


@needs_gpu
def test_gns_single_peer_keeps_state(H):
    """B == b (one peer): the device GNS update leaves its state untouched (no inf/NaN)."""
    st = torch.zeros(4, device="cuda")
    one = torch.ones(1, device="cuda")
    H.gns_update(one, one, 32.0, 32.0, 0.6, st)
    assert torch.equal(st, torch.zeros(4, device="cuda"))


@needs_gpu
def test_gns_monitor_single_gpu_runs_kernels():
    """monitor_single: the K5 reductions run every step with one GPU (forced comm path)."""
    import kungfu_amd as kf

    kf.init()
    torch.manual_seed(0)
    m = torch.nn.Linear(128, 8).cuda()
    opt = kf.optimizers.MonitorGradientNoiseScaleOptimizer(torch.optim.SGD(m.parameters(), lr=0.1),
                                                           device_batch_size=16, monitor_single=True)
    seen = []
    orig = opt.reducer.post_finish

    def capture():
        seen.append(opt._local_sq.clone())  # |g_local|^2 accumulated by the per-bucket K5 pass
        orig()

    opt.reducer.post_finish = capture
    x = torch.randn(16, 128, device="cuda")
    opt.zero_grad()
    m(x).square().mean().backward()
    local = seen[0]
    ref = opt.space.flat_grad.double().square().sum()
    assert abs(local.item() / ref.item() - 1) < 1e-5
    opt.step()
    assert opt.noise_scale is None  # undefined with one peer


@needs_gpu
def test_elastic_resnet18_gns_two_ranks_one_gpu():
    """kungfu-run -w with 2 ranks sharing the GPU (host-staged plane), ResNet-18 with the
    gradient-noise-scale monitor through 1 -> 2 -> 1 peers: after every step all replicas
    hold bit-identical flat parameters and the monitor reports a finite noise scale while
    two peers train (VERDICT r1 'Next round' #1)."""
    base = free_port_block(16)
    cfg = base + 15
    r = kungfu_run(1, [worker("elastic_train.py"), "--schedule", "1:3,2:3,1:3", "--max-step", "9",
                       "--optimizer", "gns", "--device", "cuda", "--model", "resnet18", "--global-batch", "16"],
                   timeout=400, port_base=base,
                   env={"KUNGFU_FORCE_DEVICE": "0", "KUNGFU_GPU_DATAPLANE": "host"},
                   extra=["-w", "-builtin-config-port", str(cfg), "-config-server",
                          "http://127.0.0.1:%d/config" % cfg, "-H", "127.0.0.1:4"])
    assert r.returncode == 0, r.stdout[-5000:]
    steps = re.findall(r"STEP (\d+) np=(\d+) rank=(\d+) loss=(\S+) h=(\w+)(?: gns=(\S+))?", r.stdout)
    by = {}
    for st, np_, rk, loss, h, gns in steps:
        by.setdefault(int(st), []).append((int(np_), h, gns, float(loss)))
    assert sorted(by) == list(range(9)), r.stdout[-3000:]
    for st, rows in by.items():
        assert len(rows) == rows[0][0], (st, rows)
        assert len({h for _, h, _, _ in rows}) == 1, (st, rows)
        assert all(l == l for *_, l in rows)
    gns = [float(g) for rows in by.values() for n, _, g, _ in rows if n == 2 and g not in ("", "None")]
    assert gns and all(g == g and abs(g) < 1e12 for g in gns), r.stdout[-3000:]
    assert "ELASTIC_TRAIN_DONE rank=0 np=1 step=9 v=2" in r.stdout


@needs_gpu
def test_gns_on_bert_gradients_matches_fp64(H):
    """K5 on real BERT-base gradients: |g_small|^2 (half batch) and |g_big|^2 (full batch)
    from the one-pass sumsq kernel, then the device EMA update, against float64 torch and
    the reference formulas (grad_noise_scale.py:56-88)."""
    from kungfu_amd.models.bert import bert_base, pretraining_loss, synthetic_pretraining_batch

    torch.manual_seed(0)
    m = bert_base(layers=2).cuda()
    data = synthetic_pretraining_batch(8, 128, device="cuda")

    def flat_grad(b):
        m.zero_grad()
        with torch.autocast("cuda", dtype=torch.bfloat16):
            loss = pretraining_loss(m, b)
        loss.backward()
        return torch.cat([p.grad.reshape(-1) for p in m.parameters() if p.grad is not None]).float()

    half = tuple(t[:4] for t in data)
    g_small, g_big = flat_grad(half), flat_grad(data)
    s = H.sumsq2(g_small, g_big)
    ref = [g_small.double().square().sum().item(), g_big.double().square().sum().item()]
    for got, want in zip(s.tolist(), ref):
        assert abs(got / want - 1) < 1e-5, (got, want)
    st = torch.zeros(4, device="cuda")
    H.gns_update(s[:1], s[1:2], 4.0, 8.0, 0.6, st)
    G = (8 * ref[1] - 4 * ref[0]) / (8 - 4)
    S = (ref[0] - ref[1]) / (1 / 4 - 1 / 8)
    assert abs(st[0].item() / G - 1) < 1e-4 and abs(st[1].item() / S - 1) < 1e-4
    assert abs(st[2].item() - S / G) <= 1e-4 * abs(S / G)


@needs_gpu
def test_bench_bert_gns_json():
    import json
    import subprocess
    import sys

    from conftest import ROOT

    r = subprocess.run([sys.executable, "bench.py", "--model", "bert_base", "--optimizer", "gns", "--steps", "2",
                        "--warmup", "2", "--batch", "8"], cwd=ROOT, stdout=subprocess.PIPE, stderr=subprocess.STDOUT,
                       text=True, timeout=600)
    assert r.returncode == 0, r.stdout[-3000:]
    d = json.loads([l for l in r.stdout.splitlines() if l.startswith("{")][-1])
    assert d["unit"].startswith("sequences/sec") and d["value"] > 0 and d["config"]["seq_len"] == 128
    assert d["config"]["comm"]["comm_plane"] == "rccl"


def _resnet50_trajectory(engine: bool, steps=10, batch=64, lr=0.1):
    """Loss trajectory of ResNet-50 at 224x224 (batch 64, SGD lr 0.1 momentum 0.9 wd 1e-4,
    bf16 autocast): the bench's fused engine (HIP BN / MFMA convs / bf16 shadow weights /
    bucketed S-SGD / fused SGD) or the stock modules with torch.optim.SGD."""
    import kungfu_amd as kf
    from kungfu_amd.models import resnet50

    kf.init()
    torch.manual_seed(1234)
    model = resnet50(fused_bn=engine).cuda().to(memory_format=torch.channels_last)
    base = torch.optim.SGD(model.parameters(), lr=lr, momentum=0.9, weight_decay=1e-4)
    if engine:
        from kungfu_amd.parallel.mixed import enable_bf16_shadow

        opt = kf.optimizers.SynchronousSGDOptimizer(base)
        enable_bf16_shadow(model, opt)
    else:
        opt = base
    g = torch.Generator(device="cuda").manual_seed(99)
    x = torch.randn(batch, 3, 224, 224, device="cuda", generator=g).to(memory_format=torch.channels_last)
    y = torch.randint(0, 1000, (batch,), device="cuda", generator=g)
    out = []
    for _ in range(steps):
        opt.zero_grad()
        with torch.autocast("cuda", dtype=torch.bfloat16):
            loss = F.cross_entropy(model(x).float(), y)
        loss.backward()
        opt.step()
        out.append(loss.item())
    return out


def _stock_resnet50(state):
    from kungfu_amd.models import resnet50

    m = resnet50(fused_bn=False).cuda().to(memory_format=torch.channels_last)
    m.load_state_dict(state)
    return m


def _layer_rel(ref, got):
    return {n: ((got[n].reshape(a.shape) - a).norm() / a.norm().clamp_min(1e-30)).item() for n, a in ref.items()}


@needs_gpu
def test_resnet50_engine_gradients_within_stock_bf16_envelope():
    """Full-size numerics of the bench path (VERDICT r4 next #1a; replaces the lr-0.1 trajectory-spread
    comparison, whose outcome depended on run-to-run chaos): ResNet-50 at 224x224, batch 64, from ONE
    shared state at step 0 and after 3 stock lr-0.1 steps, the engine's (fused BN, MFMA convs, bf16
    shadow weights, bucketed S-SGD) per-parameter gradient vs a stock f32 reference.  Every one of the
    161 parameters' relative L2 error must stay within 2x the stock-bf16-vs-f32 error of the same
    parameter (max over two stock bf16 runs) + 1e-3; the loss within 3x the stock-bf16 loss error.
    Measured r5 (profiles/r5_engine_numerics.md): worst layer 1.14x the envelope, over 9 component
    variants and both states; BN gamma/beta gradients at random init are rounding-dominated in bf16
    for stock and engine alike (relative error ~1.2-1.4 vs f32), conv weights agree to ~1e-2."""
    import kungfu_amd as kf
    from kungfu_amd.models import resnet50
    from kungfu_amd.parallel.mixed import enable_bf16_shadow

    kf.init()
    g = torch.Generator(device="cuda").manual_seed(99)
    x = torch.randn(64, 3, 224, 224, device="cuda", generator=g).to(memory_format=torch.channels_last)
    y = torch.randint(0, 1000, (64,), device="cuda", generator=g)
    torch.manual_seed(1234)
    m = resnet50(fused_bn=False).cuda().to(memory_format=torch.channels_last)
    s0 = {k: v.detach().clone() for k, v in m.state_dict().items()}
    sgd = torch.optim.SGD(m.parameters(), lr=0.1, momentum=0.9, weight_decay=1e-4)
    for _ in range(3):
        sgd.zero_grad()
        with torch.autocast("cuda", dtype=torch.bfloat16):
            F.cross_entropy(m(x).float(), y).backward()
        sgd.step()
    s3 = {k: v.detach().clone() for k, v in m.state_dict().items()}
    del m, sgd

    def stock(state, amp):
        mm = _stock_resnet50(state)
        with torch.autocast("cuda", dtype=torch.bfloat16, enabled=amp):
            loss = F.cross_entropy(mm(x).float(), y)
        loss.backward()
        return loss.item(), {n: p.grad.detach().float().clone() for n, p in mm.named_parameters()}

    def engine(state):
        mm = resnet50(fused_bn=True).cuda().to(memory_format=torch.channels_last)
        mm.load_state_dict(state)
        opt = kf.optimizers.SynchronousSGDOptimizer(torch.optim.SGD(mm.parameters(), lr=0.0, momentum=0.9),
                                                    named_parameters=mm.named_parameters())
        enable_bf16_shadow(mm, opt)
        opt.zero_grad()
        with torch.autocast("cuda", dtype=torch.bfloat16):
            loss = F.cross_entropy(mm(x).float(), y)
        loss.backward()
        opt.reducer.synchronize()
        return loss.item(), {n: opt.space.grad_view(i).detach().float().clone() for i, n in enumerate(opt.space.names)}

    for tag, st in (("S0", s0), ("S3", s3)):
        lf, gf = stock(st, False)
        la, ga = stock(st, True)
        lb, gb = stock(st, True)
        le, ge = engine(st)
        assert set(ge) == set(gf), set(gf) ^ set(ge)
        ea, eb, ee = _layer_rel(gf, ga), _layer_rel(gf, gb), _layer_rel(gf, ge)
        worst = max(gf, key=lambda n: ee[n] / max(ea[n], eb[n], 1e-12))
        print("%s loss f32 %.5f bf16 %.5f %.5f engine %.5f; worst %s rel %.4f env %.4f" % (
            tag, lf, la, lb, le, worst, ee[worst], max(ea[worst], eb[worst])))
        bad = [(n, ee[n], max(ea[n], eb[n])) for n in gf if ee[n] > 2 * max(ea[n], eb[n]) + 1e-3]
        assert not bad, (tag, bad[:10])
        # the loss: within 3x the stock-bf16 error or 0.25 % of the f32 loss, whichever is larger -- the
        # S3 state comes from three non-deterministic stock steps, and when both stock bf16 runs happen
        # to land within 1e-3 of f32 the 3x bound alone sat below the engine's own rounding (r6t5: engine
        # 0.16 % off at S3, stock 0.02 %; the same code passed on the next box)
        assert abs(le - lf) <= max(3 * max(abs(la - lf), abs(lb - lf)) + 5e-3, 2.5e-3 * abs(lf)), (tag, lf, la, lb, le)
        assert all(torch.isfinite(v).all() for v in ge.values())


@needs_gpu
def test_resnet50_bn_param_grads_match_f64_on_shared_inputs():
    """the model-level pin of the 104 block-BN gamma/beta gradients (the stock-bf16
    envelope above is vacuous for them -- a sign-flipped gradient scores 2.0 against a bound of 2.2-3.0).
    One engine forward/backward of ResNet-50 (224x224, batch 32, after one lr-0.1 step so the BNs are
    not at gamma=1/beta=0) records every fused block BN's backward inputs (ops/fused_block._CAPTURE:
    the gradient at the BN(+ReLU) output, the bf16 BN input, mean/invstd, the ReLU gate); an f64
    reduction of those SAME tensors (utils/numerics.bn_param_grads_f64) must match the fused
    kernels' dgamma/dbeta -- which come from the conv epilogues' BNLink sums (slotted f64 atomics),
    the cross-block tail link and the finalize -- to 1e-3 relative L2, and the flat gradient slots
    the sink landed them in must hold exactly those values."""
    import kungfu_amd as kf
    from kungfu_amd.models import resnet50
    from kungfu_amd.ops import fused_block
    from kungfu_amd.parallel.mixed import enable_bf16_shadow
    from kungfu_amd.utils.numerics import bn_param_grads_f64, check_bn_param_grads, rel_err

    kf.init()
    torch.manual_seed(4321)
    g = torch.Generator(device="cuda").manual_seed(7)
    x = torch.randn(32, 3, 224, 224, device="cuda", generator=g).to(memory_format=torch.channels_last)
    y = torch.randint(0, 1000, (32,), device="cuda", generator=g)
    m = resnet50(fused_bn=True).cuda().to(memory_format=torch.channels_last)
    opt = kf.optimizers.SynchronousSGDOptimizer(torch.optim.SGD(m.parameters(), lr=0.1, momentum=0.9),
                                                named_parameters=m.named_parameters())
    enable_bf16_shadow(m, opt)
    for cap in (False, True):
        opt.zero_grad()
        fused_block._CAPTURE = [] if cap else None
        try:
            with torch.autocast("cuda", dtype=torch.bfloat16):
                loss = F.cross_entropy(m(x).float(), y)
            loss.backward()
            opt.reducer.synchronize()
            recs = fused_block._CAPTURE
        finally:
            fused_block._CAPTURE = None
        if not cap:
            opt.step()
    assert len(recs) == 52, len(recs)  # 16 blocks x 3 BNs + 4 downsample BNs
    index = {id(p): i for i, p in enumerate(opt.space.params)}
    kinds, worst = {}, 0.0
    for r in recs:
        ref = bn_param_grads_f64(r["dz"], r["x"], r["mean"], r["invstd"], r["kind"], r["gate"])
        msg = check_bn_param_grads(ref, (r["dg"], r["db"]), tol=1e-3)
        assert msg is None, (r["kind"], tuple(r["x"].shape), msg)
        worst = max(worst, rel_err(ref[0], r["dg"]), rel_err(ref[1], r["db"]))
        kinds[r["kind"]] = kinds.get(r["kind"], 0) + 1
        # landed in the flat slots exactly (zeroed by zero_grad, one landing per parameter)
        for prm, v in ((r["bn"].weight, r["dg"]), (r["bn"].bias, r["db"])):
            assert torch.equal(opt.space.grad_view(index[id(prm)]).view(-1), v.float().view(-1)), r["kind"]
    print("BN param grads vs f64 on shared inputs: %s, worst rel %.2e" % (kinds, worst))
    assert kinds == {"mask": 16, "relu": 32, "plain": 4}, kinds


@needs_gpu
def test_resnet50_full_size_engine_memorises_batch_like_stock():
    """lr 0.01 (no chaotic phase): stock and engine both memorise one fixed 224x224 batch of 64
    (7.16 -> ~4.2 in 10 steps) and agree within 2 % at every step (measured within 0.5 %).  The
    lr-0.1 trajectory is not compared: it amplifies a single bf16 ulp of 1 % of the weights into a
    several-% loss difference by step 3 (profiles/r5_engine_numerics.md)."""
    a = _resnet50_trajectory(False, lr=0.01)
    e = _resnet50_trajectory(True, lr=0.01)
    print("lr0.01 stock", a, "\nlr0.01 engine", e)
    for t in (a, e):  # memorising the batch: a steady decrease, then a plateau near 4.19
        assert all(y < x for x, y in zip(t[:7], t[1:7])) and t[-1] < 0.65 * t[0], t
    for x0, xe in zip(a, e):
        assert abs(xe - x0) <= 0.02 * x0, (a, e)


@needs_gpu
@pytest.mark.parametrize("D,rows,res", [(768, 4096, True), (768, 333, False), (1024, 1000, True), (256, 7, True)])
def test_add_layernorm_matches_fp32(D, rows, res):
    """Fused residual-add + LayerNorm (bf16 stream) vs the float32 torch composition:
    output, both input gradients, dgamma, dbeta."""
    from kungfu_amd.ops.layernorm import add_layer_norm

    torch.manual_seed(21)
    x = (torch.randn(rows, D, device="cuda") * 2 + 0.3).bfloat16()
    r = torch.randn(rows, D, device="cuda").bfloat16() if res else None
    w = torch.rand(D, device="cuda") + 0.5
    b = torch.randn(D, device="cuda") * 0.1
    dy = torch.randn(rows, D, device="cuda").bfloat16()
    xr = x.float().requires_grad_(True)
    rr = r.float().requires_grad_(True) if res else None
    wr, br = w.clone().requires_grad_(True), b.clone().requires_grad_(True)
    yr = F.layer_norm(xr + rr if res else xr, (D,), wr, br, 1e-12)
    yr.backward(dy.float())
    xa = x.clone().requires_grad_(True)
    ra = r.clone().requires_grad_(True) if res else None
    wa, ba = w.clone().requires_grad_(True), b.clone().requires_grad_(True)
    ya = add_layer_norm(xa, ra, wa, ba, 1e-12)
    assert ya.dtype == torch.bfloat16
    ya.backward(dy)

    def rel(a, b_):
        return ((a.float() - b_.float()).norm() / b_.float().norm()).item()

    assert rel(ya, yr) < 1e-2
    assert rel(xa.grad, xr.grad) < 2e-2 and rel(wa.grad, wr.grad) < 1e-2 and rel(ba.grad, br.grad) < 1e-3
    if res:
        assert torch.equal(xa.grad, ra.grad) and rel(ra.grad, rr.grad) < 2e-2


@needs_gpu
def test_add_layernorm_fused_residual_dropout():
    """Residual dropout fused into the add + LayerNorm kernels: the hashed keep mask (recomputed
    in torch below) reproduces y = LN(x + r * keep / (1 - p)) and the gradients (dx = ds,
    dr = ds * keep / (1 - p)) of the float32 composition; keep rate ~ 1 - p."""
    import torch.nn.functional as F

    from kungfu_amd._lib import hip
    from kungfu_amd.ops.layernorm import _AddLayerNormFn

    torch.manual_seed(31)
    rows, D, p, seed = 4096, 768, 0.1, 12345
    x = torch.randn(rows, D, device="cuda").bfloat16()
    r = torch.randn(rows, D, device="cuda").bfloat16()
    g, b = torch.rand(D, device="cuda") + 0.5, torch.randn(D, device="cuda") * 0.1
    M = 0xFFFFFFFF
    e = torch.arange(rows * D, device="cuda", dtype=torch.int64)
    from kungfu_amd.ops import dropout_seed

    h = (((e & M) * 0x9E3779B1) & M) ^ ((((e >> 32) * 0x7FEB352D) & M)) ^ dropout_seed.effective(seed)
    h ^= h >> 16
    h = (h * 0x85EBCA6B) & M
    h ^= h >> 13
    h = (h * 0xC2B2AE35) & M
    h ^= h >> 16
    keep = (h >= int(p * 2**32)).view(rows, D)
    assert abs(keep.float().mean().item() - (1 - p)) < 0.01
    xa, ra = x.clone().requires_grad_(True), r.clone().requires_grad_(True)
    y = _AddLayerNormFn.apply(xa, ra, g, b, 1e-12, p, seed)
    xr, rr = x.float().requires_grad_(True), r.float().requires_grad_(True)
    yr = F.layer_norm(xr + rr * keep / (1 - p), (D,), g, b, 1e-12)
    assert ((y.float() - yr).norm() / yr.norm()).item() < 1e-2
    dy = torch.randn(rows, D, device="cuda")
    y.backward(dy.bfloat16())
    yr.backward(dy)
    for a, c in ((xa.grad, xr.grad), (ra.grad, rr.grad)):
        assert ((a.float() - c).norm() / c.norm()).item() < 2e-2
    assert torch.equal(ra.grad == 0, ~keep | (xa.grad == 0))
    del hip


@needs_gpu
def test_linear_side_stream_wgrad_joined_without_bucket_engine(monkeypatch):
    """the linear layers' direct split-K weight gradients run on the side stream
    (ops/linear.py _WGRAD_SIDE) and reach the flat slot themselves (sink.put_direct).  With the
    default BatchedSink (SMA here: no bucket engine) and no staged put at all (an MLP, nothing but
    direct producers) the end of backward must still join the side stream: the flat gradients are
    bit-identical to the single-stream run, and no side-stream event is left pending."""
    import kungfu_amd as kf
    from kungfu_amd.ops import linear as lin
    from kungfu_amd.parallel import mixed

    kf.init()

    def run(side):
        monkeypatch.setattr(lin, "_WGRAD_SIDE", side)
        torch.manual_seed(0)
        m = torch.nn.Sequential(torch.nn.Linear(512, 1024), torch.nn.ReLU(), torch.nn.Linear(1024, 1024),
                                torch.nn.ReLU(), torch.nn.Linear(1024, 256)).cuda()
        opt = kf.optimizers.SynchronousAveragingOptimizer(torch.optim.SGD(m.parameters(), lr=0.01))
        mixed.enable_bf16_shadow(m, opt)
        assert isinstance(opt.space.sink, mixed.BatchedSink)
        g = torch.Generator(device="cuda").manual_seed(1)
        grads = []
        for _ in range(3):
            x = torch.randn(8192, 512, device="cuda", generator=g)
            opt.zero_grad()
            with torch.autocast("cuda", dtype=torch.bfloat16):
                m(x).float().square().mean().backward()
            assert not mixed.SideStream._pending  # joined at the end of backward
            grads.append(opt.space.flat_grad.clone())  # read on the main stream right away
            opt.step()
        torch.cuda.synchronize()
        mixed.disable(m)
        return grads

    g0, g1 = run(False), run(True)
    for a, b in zip(g0, g1):
        assert torch.equal(a, b), (a - b).abs().max()


@needs_gpu
def test_bert_side_stream_wgrad_vs_inplace_residual_gradient(monkeypatch):
    """Round 6 race: with no dropout, an AddLayerNorm's skip gradient IS the gradient FC2's side-stream
    weight gradient reads, and FC1's backward adds its data gradient into it in place (``g.addmm_``).
    ``SideStream.before_write`` makes that write wait for the side-stream readers of the storage.
    Without it, FC2's weight gradients differed by 25-29 % from the single-stream run
    (tools/diag/linear_gemm_ab.py, r6t12; 6 % of the whole flat gradient).  Here: flat gradients over
    two AdamW steps equal with and without the side stream, up to the embedding scatter-add's f32
    atomic-order noise (1e-5 / 1e-3 relative at steps 1 / 2)."""
    import kungfu_amd as kf
    from kungfu_amd.models.bert import BertForPreTraining, pretraining_loss, synthetic_pretraining_batch
    from kungfu_amd.ops import linear as lin
    from kungfu_amd.parallel import mixed

    kf.init()

    def run(side):
        monkeypatch.setattr(lin, "_WGRAD_SIDE", side)
        torch.manual_seed(0)
        m = BertForPreTraining(layers=2).cuda()
        for l in m.layers:
            l.dropout = 0.0
        opt = kf.optimizers.SynchronousSGDOptimizer(torch.optim.AdamW(m.parameters(), lr=1e-4),
                                                    named_parameters=m.named_parameters())
        mixed.enable_bf16_shadow(m, opt)
        g = torch.Generator(device="cuda").manual_seed(1)
        batch = synthetic_pretraining_batch(16, 128, device="cuda", generator=g)
        grads = []
        for _ in range(2):
            opt.zero_grad()
            with torch.autocast("cuda", dtype=torch.bfloat16):
                loss = pretraining_loss(m, batch)
            loss.backward()
            opt.reducer.synchronize()
            grads.append(opt.space.flat_grad.clone())
            opt.step()
        torch.cuda.synchronize()
        mixed.disable(m)
        return grads

    g0, g1 = run(False), run(True)
    for a, b, tol in zip(g0, g1, (1e-5, 1e-3)):
        rel = ((a - b).norm() / a.norm()).item()
        assert rel < tol, rel


@needs_gpu
def test_linear_direct_f32_wgrad_into_flat_slot(monkeypatch):
    """bf16-shadow linear layers (S-SGD engine, bucket reducer): the split-K weight gradient
    reduced straight into the flat f32 gradient slot (ops/linear.py, sink.put_direct) equals the
    bf16-delivered path up to that path's bf16 rounding, is closer to the f32 reference, and the
    step after it matches (no gradient lost or counted twice in the bucket accounting)."""
    import kungfu_amd as kf
    from kungfu_amd.ops import linear as lin
    from kungfu_amd.parallel import mixed

    kf.init()
    res = {}
    for direct in (False, True):
        monkeypatch.setattr(lin, "_DIRECT_WGRAD", direct)
        torch.manual_seed(0)
        m = torch.nn.Sequential(torch.nn.Linear(256, 512), torch.nn.GELU(), torch.nn.Linear(512, 256)).cuda()
        ref = [p.detach().clone() for p in m.parameters()]
        opt = kf.optimizers.SynchronousSGDOptimizer(torch.optim.SGD(m.parameters(), lr=0.01, momentum=0.9),
                                                    force_comm=True)
        mixed.enable_bf16_shadow(m, opt)
        g = torch.Generator(device="cuda").manual_seed(1)
        grads = []
        for _ in range(3):
            x = torch.randn(2048, 256, device="cuda", generator=g)
            opt.zero_grad()
            with torch.autocast("cuda", dtype=torch.bfloat16):
                loss = m(x).float().pow(2).mean()
            loss.backward()
            grads.append(opt.space.flat_grad.clone())
            opt.step()
        torch.cuda.synchronize()
        res[direct] = (grads, opt.space.flat_param.clone(), ref)
    g0, p0, _ = res[False]
    g1, p1, _ = res[True]
    for a, b in zip(g0, g1):
        assert ((a - b).norm() / a.norm()).item() < 5e-3
    assert ((p0 - p1).norm() / p0.norm()).item() < 1e-3
    # every weight got its gradient through the direct path (non-zero, finite)
    assert torch.isfinite(g1[0]).all() and (g1[0] != 0).float().mean().item() > 0.5


@needs_gpu
def test_graphed_resnet50_step_bit_identical_to_eager():
    """the whole fused ResNet-50 step (zero_grad, forward, backward with the RCCL
    bucket all-reduces through the comm stream, fused SGD, shadow refresh) captured into ONE hipGraph
    and replayed must produce bit-identical weights and losses to the eager step over 8 steps
    (3 eager warm-up steps, then the capture, then replays)."""
    import kungfu_amd as kf
    from kungfu_amd.models import resnet50
    from kungfu_amd.parallel.graphs import GraphedStep
    from kungfu_amd.parallel.mixed import enable_bf16_shadow

    kf.init()

    def run(graph):
        torch.manual_seed(1234)
        m = resnet50(fused_bn=True).cuda().to(memory_format=torch.channels_last)
        opt = kf.optimizers.SynchronousSGDOptimizer(
            torch.optim.SGD(m.parameters(), lr=0.05, momentum=0.9, weight_decay=1e-4),
            named_parameters=m.named_parameters(), force_comm=True)
        enable_bf16_shadow(m, opt)
        g = torch.Generator(device="cuda").manual_seed(5)
        x = torch.randn(32, 3, 224, 224, device="cuda", generator=g).to(memory_format=torch.channels_last)
        y = torch.randint(0, 1000, (32,), device="cuda", generator=g)

        def step():
            opt.zero_grad()
            with torch.autocast("cuda", dtype=torch.bfloat16):
                loss = F.cross_entropy(m(x).float(), y)
            loss.backward()
            opt.step()
            return loss

        fn = GraphedStep(step, opt, warmup=3) if graph else step
        losses = [float(fn().detach()) for _ in range(8)]
        torch.cuda.synchronize()
        if graph:
            assert fn.graph is not None and fn.replays == 5, (fn.graph, fn.replays)
        return losses, opt.space.flat_param.clone(), [b.clone() for b in m.buffers()]

    le, pe, be = run(False)
    lg, pg, bg = run(True)
    print("eager", le, "\ngraph", lg)
    assert le == lg, (le, lg)
    assert torch.equal(pe, pg)
    assert all(torch.equal(a, b) for a, b in zip(be, bg))


@needs_gpu
def test_graphed_bert_step_matches_eager_without_dropout_and_redraws_masks():
    """BERT under whole-step capture: with dropout 0 the replays are bit-identical to eager steps;
    with dropout and lr 0 (the weights never change) the device seed word advancing before every
    replay still gives every replay a different loss -- fresh masks, never the capture-time ones."""
    import kungfu_amd as kf
    from kungfu_amd.models.bert import BertForPreTraining, pretraining_loss, synthetic_pretraining_batch
    from kungfu_amd.parallel.graphs import GraphedStep
    from kungfu_amd.parallel.mixed import enable_bf16_shadow

    kf.init()

    def run(graph, p, lr=1e-4, freeze=True):
        torch.manual_seed(3)
        m = BertForPreTraining(layers=2).cuda()
        for l in m.layers:
            l.dropout = p
        # frozen embeddings for the bit-identity check: their gradients are f32 atomics
        # (ops/embedding.py), whose summation order varies from run to run
        for e in (m.tok, m.pos, m.typ):
            e.weight.requires_grad_(not freeze)
        opt = kf.optimizers.SynchronousSGDOptimizer(torch.optim.AdamW([q for q in m.parameters() if q.requires_grad],
                                                                      lr=lr, weight_decay=0.0),
                                                    named_parameters=m.named_parameters(), force_comm=True)
        enable_bf16_shadow(m, opt)
        g = torch.Generator(device="cuda").manual_seed(2)
        batch = synthetic_pretraining_batch(16, 128, device="cuda", generator=g)

        def step():
            opt.zero_grad()
            with torch.autocast("cuda", dtype=torch.bfloat16):
                loss = pretraining_loss(m, batch)
            loss.backward()
            opt.step()
            return loss

        fn = GraphedStep(step, opt, warmup=3) if graph else step
        emb0 = m.tok.weight.detach().clone()
        losses = [float(fn().detach()) for _ in range(7)]
        torch.cuda.synchronize()
        if graph:
            assert fn.replays == 4 and not fn.disabled
        if not freeze:
            assert not torch.equal(emb0, m.tok.weight), "embeddings did not train"
        return losses, opt.space.flat_param.clone()

    le, pe = run(False, 0.0)
    lg, pg = run(True, 0.0)
    assert le == lg and torch.equal(pe, pg), (le, lg)
    ld, _ = run(True, 0.1, lr=0.0)
    assert all(v == v for v in ld) and len(set(ld[3:])) == len(ld[3:]), ld
    # trainable embeddings (scatter-add gradient kernel, fixed launch shape): the replays follow eager
    # up to the atomics' summation order
    le, pe = run(False, 0.0, freeze=False)
    lg, pg = run(True, 0.0, freeze=False)
    torch.testing.assert_close(torch.tensor(lg), torch.tensor(le), rtol=1e-3, atol=1e-3)
    torch.testing.assert_close(pg, pe, rtol=0, atol=2e-3)


def _captured_vs_eager(build, batch, size, steps=8, lr=0.01, seed=7):
    """Losses and flat parameters of ``steps`` S-SGD steps (bf16 shadow engine, RCCL 1-rank buckets),
    eager vs GraphedStep (3 eager warm-up steps, capture, replays), for the model ``build()`` returns."""
    import kungfu_amd as kf
    from kungfu_amd.parallel.graphs import GraphedStep
    from kungfu_amd.parallel.mixed import enable_bf16_shadow

    kf.init()

    def run(graph):
        torch.manual_seed(1234)
        m = build().cuda().to(memory_format=torch.channels_last)
        opt = kf.optimizers.SynchronousSGDOptimizer(
            torch.optim.SGD(m.parameters(), lr=lr, momentum=0.9, weight_decay=1e-4),
            named_parameters=m.named_parameters(), force_comm=True)
        enable_bf16_shadow(m, opt)
        g = torch.Generator(device="cuda").manual_seed(seed)
        x = torch.randn(batch, 3, size, size, device="cuda", generator=g).to(memory_format=torch.channels_last)
        y = torch.randint(0, 1000, (batch,), device="cuda", generator=g)

        def step():
            opt.zero_grad()
            with torch.autocast("cuda", dtype=torch.bfloat16):
                loss = F.cross_entropy(m(x).float(), y)
            loss.backward()
            opt.step()
            return loss

        fn = GraphedStep(step, opt, warmup=3) if graph else step
        losses = [float(fn().detach()) for _ in range(steps)]
        torch.cuda.synchronize()
        if graph:
            assert fn.graph is not None and fn.replays == steps - 3, (fn.graph, fn.replays)
        return losses, opt.space.flat_param.clone()

    return run(False), run(True), run(True)


@needs_gpu
def test_graphed_vgg16_per_layer_step_matches_eager(monkeypatch):
    """VGG-16's per-layer path (the fallback of the fused stack,
    KUNGFU_VGG_FUSED=0) under whole-step capture.  Before round 5 the captured step gave a different
    loss in every run and went NaN in ~1 of 4 runs while eager was bit-stable; the cause was the
    bias+ReLU backward (_BiasActFn), the only in-step hipMemsetAsync plus f32 atomics (now fixed-order
    partial sums, bias_act.hip).  Dropout off (a replay draws other masks than eager): two captured
    runs and the eager run must agree bitwise -- losses and weights."""
    from kungfu_amd.models.vgg import vgg16
    from kungfu_amd.ops import vgg_fused

    monkeypatch.setattr(vgg_fused, "_ENABLED", False)

    def build():
        m = vgg16(fused_bn=True)
        for mod in m.modules():
            if isinstance(mod, torch.nn.Dropout):
                mod.p = 0.0
        assert isinstance(m.features, vgg_fused.FusedVGGFeatures)
        return m

    (le, pe), (lg, pg), (lg2, pg2) = _captured_vs_eager(build, 32, 224)
    print("eager", le, "\ngraph", lg, "\ngraph", lg2)
    assert all(v == v for v in le + lg + lg2), (le, lg, lg2)
    assert lg == lg2 and torch.equal(pg, pg2), "captured VGG-16 step not reproducible run to run"
    assert le == lg and torch.equal(pe, pg), (le, lg)


@needs_gpu
def test_graphed_inception_v3_step_matches_eager():
    """every model the bench captures by default has a captured-vs-eager bitwise test.
    Inception-v3 (fused BN, sibling MFMA convs, batched BN finalizes) at 224x224 (the bench input), batch 16: two
    captured runs and the eager run agree bitwise over 8 steps.  MIOpen's deterministic solvers for the
    layers still on MIOpen: with its defaults even two EAGER runs differ from step 4 on (r5t4,
    tools/diag/capture_repro.py), and with them eager, eager and two captures are bit-identical -- the
    run-to-run variation is MIOpen's, not a capture race."""
    from kungfu_amd.models.inception import inception_v3

    old = torch.backends.cudnn.deterministic
    torch.backends.cudnn.deterministic = True
    try:
        (le, pe), (lg, pg), (lg2, pg2) = _captured_vs_eager(lambda: inception_v3(fused_bn=True), 16, 224)
    finally:
        torch.backends.cudnn.deterministic = old
    print("eager", le, "\ngraph", lg, "\ngraph", lg2)
    assert all(v == v for v in le + lg), (le, lg)
    assert lg == lg2 and torch.equal(pg, pg2), "captured Inception-v3 step not reproducible run to run"
    assert le == lg and torch.equal(pe, pg), (le, lg)


@needs_gpu
def test_segmented_capture_with_emulated_comm_matches_eager(monkeypatch):
    """the N-rank capture layout -- graph segments cut at every bucket launch, the
    bucket collectives issued eagerly on the comm stream between segment replays -- exercised on one
    GPU through the comm emulator (an 8-rank all-reduce's footprint per bucket; it leaves the gradient
    as it is).  The replay program must hold every bucket and one join, and the losses / weights must
    match the eager step bitwise (ResNet-50, batch 16)."""
    from kungfu_amd.models import resnet50

    monkeypatch.setenv("KUNGFU_COMM_EMULATE", "ranks=8,ctas=16,busbw=350,lat_us=25")
    import kungfu_amd as kf
    from kungfu_amd.parallel.graphs import GraphedStep
    from kungfu_amd.parallel.mixed import enable_bf16_shadow

    kf.init()

    def run(graph):
        torch.manual_seed(1234)
        m = resnet50(fused_bn=True).cuda().to(memory_format=torch.channels_last)
        opt = kf.optimizers.SynchronousSGDOptimizer(
            torch.optim.SGD(m.parameters(), lr=0.05, momentum=0.9, weight_decay=1e-4),
            named_parameters=m.named_parameters(), force_comm=True)
        enable_bf16_shadow(m, opt)
        g = torch.Generator(device="cuda").manual_seed(5)
        x = torch.randn(16, 3, 224, 224, device="cuda", generator=g).to(memory_format=torch.channels_last)
        y = torch.randint(0, 1000, (16,), device="cuda", generator=g)

        def step():
            opt.zero_grad()
            with torch.autocast("cuda", dtype=torch.bfloat16):
                loss = F.cross_entropy(m(x).float(), y)
            loss.backward()
            opt.step()
            return loss

        fn = GraphedStep(step, opt, warmup=3) if graph else step
        losses = [float(fn().detach()) for _ in range(8)]
        torch.cuda.synchronize()
        assert opt.reducer.describe()["comm_plane"] == "emulate"
        if graph:
            nb = len(opt.reducer.buckets)
            kinds = [op[0] for op in fn.program]
            assert fn.replays == 5 and not fn.disabled, (fn.replays, fn.disabled)
            assert kinds.count("bucket") == nb and kinds.count("join") == 1, fn.program
            assert sorted(op[1] for op in fn.program if op[0] == "bucket") == list(range(nb)), fn.program
            # one segment before each cut point and one after the join, minus those that captured nothing
            assert len(fn.segs) == kinds.count("g") and 2 <= len(fn.segs) <= nb + 2, (len(fn.segs), fn.program)
        return losses, opt.space.flat_param.clone()

    le, pe = run(False)
    lg, pg = run(True)
    print("eager", le, "\ngraph", lg)
    assert le == lg and torch.equal(pe, pg), (le, lg)


def test_fused_adam_writes_the_bf16_shadow():
    """FusedAdam's kernel writes bf16(new weights) into the space's shadow (exactly the cast
    refresh_shadow would produce) and the next refresh skips its cast; an in-place edit of a
    weight after the step makes it recast."""
    from kungfu_amd.optimizers.fused import FusedAdam
    from kungfu_amd.parallel.flat import FlatParamSpace

    torch.manual_seed(0)
    m = torch.nn.Sequential(torch.nn.Linear(64, 1000), torch.nn.Linear(1000, 3)).cuda()
    sp = FlatParamSpace(list(m.parameters()))
    sp.enable_shadow()
    opt = FusedAdam(sp, lr=1e-2, weight_decay=0.01)
    for _ in range(2):
        opt.zero_grad()
        m(torch.randn(8, 64, device="cuda")).square().sum().backward()
        opt.step()
        torch.cuda.synchronize()
        assert torch.equal(sp.flat_shadow, sp.flat_param.to(torch.bfloat16))
        gen = sp.shadow_gen
        sp.flat_shadow.zero_()
        sp.refresh_shadow()  # skipped: the step wrote it
        assert sp.shadow_gen == gen + 1 and sp.flat_shadow.abs().sum().item() == 0
        sp.refresh_shadow()
    opt.step()
    with torch.no_grad():
        m[0].weight.mul_(3.0)
    sp.refresh_shadow()
    assert torch.equal(sp.flat_shadow, sp.flat_param.to(torch.bfloat16))
