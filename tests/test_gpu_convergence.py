"""Convergence with real signal: the fused GPU engine must LEARN a task as well
as stock PyTorch does, not just match it for a few steps on one random batch.

* ResNet-50: 1,024 synthetic 96x96 images in 10 classes -- each class a fixed low-frequency
  pattern (sums of 2-D sinusoids per channel) under heavy Gaussian noise -- trained for 150
  steps (batch 64, SGD momentum 0.9, linear warm-up to lr 0.05 then cosine decay) by (a) the
  bench's fused engine (HIP BN / MFMA convs / bf16 shadow weights / bucketed S-SGD / fused SGD)
  and (b) the stock modules with torch.optim.SGD, from the same initial weights and batches, for
  two seeds each.  Every engine run must reach >= 95 % accuracy over the whole set in eval mode
  (this also checks the fused BN's running statistics), its mean accuracy must be within 2 points
  of stock's and its last-50-step loss at most 0.5 on every seed (ln 10 = 2.30).
  Why not "losses within 10 %": measured over 3 seeds (r4t6, profiles/r4_convergence.md) the
  last-50 loss of ONE configuration spans 0.0004 .. 0.91 across seeds -- at peak lr 0.2 even
  stock PyTorch diverges on some seeds -- so a per-step loss match between two implementations
  (different bf16 rounding: the gradients at initialisation already have cosine ~0.1-0.3
  between stock f32 and stock bf16, tools/diag/grad_compare.py) is not a property either has.
* BERT (4 encoder layers of BERT-base width: the same fused attention / add+LayerNorm / MFMA
  weight-gradient kernels): masked-LM on a synthetic first-order Markov corpus over 512 tokens
  (each token has 4 successors), 20 masked positions per 128-token sequence.  The fused model
  and a plain-torch reference (nn.LayerNorm, SDPA, F.gelu, nn.Linear; same state_dict) must
  both get the MLM loss below ln(512) = 6.24 -- the best any context-free (unigram) predictor
  can do -- and agree within 10 % on the mean of the last 30 steps.

Parity: the reference pins exact accuracies for its MNIST SLP (tests/python/integration/
test_mnist_slp.py:153-165) and claims ~75 % top-1 for every optimizer (README.md:190-199);
MNIST/ImageNet are not available offline, so this is the learnable-signal stand-in.
"""
import math

import pytest
import torch
import torch.nn as nn
import torch.nn.functional as F

pytestmark = pytest.mark.gpu
needs_gpu = pytest.mark.skipif(not torch.cuda.is_available(), reason="no GPU")


# ------------------------------------------------------------------ ResNet-50
def _pattern_dataset(n=1024, classes=10, size=96, noise=2.0, seed=5):
    g = torch.Generator().manual_seed(seed)
    u = torch.arange(size, dtype=torch.float32)
    yy, xx = torch.meshgrid(u, u, indexing="ij")
    pats = torch.zeros(classes, 3, size, size)
    for c in range(classes):
        for ch in range(3):
            for _ in range(2):
                fx, fy = torch.randint(1, 4, (2,), generator=g).tolist()
                ph = float(torch.rand(1, generator=g)) * 2 * math.pi
                pats[c, ch] += torch.sin(2 * math.pi * (fx * xx + fy * yy) / size + ph)
    pats /= pats.std(dim=(1, 2, 3), keepdim=True)
    y = torch.arange(n) % classes
    y = y[torch.randperm(n, generator=g)]
    x = pats[y] + noise * torch.randn(n, 3, size, size, generator=g)
    return x, y


def _lr(step, steps, peak=0.2, warm=20):
    if step < warm:
        return peak * (step + 1) / warm
    return peak * 0.5 * (1 + math.cos(math.pi * (step - warm) / (steps - warm)))


def _train_resnet(engine: bool, steps=150, batch=64, seed=1):
    import kungfu_amd as kf
    from kungfu_amd.models import resnet50

    kf.init()
    dev = torch.device("cuda")
    x_all, y_all = _pattern_dataset()
    x_all = x_all.to(dev).to(memory_format=torch.channels_last)
    y_all = y_all.to(dev)
    torch.manual_seed(seed)
    model = resnet50(fused_bn=engine).to(dev).to(memory_format=torch.channels_last)
    base = torch.optim.SGD(model.parameters(), lr=0.0, momentum=0.9, weight_decay=5e-5)
    if engine:
        from kungfu_amd.parallel.mixed import enable_bf16_shadow

        opt = kf.optimizers.SynchronousSGDOptimizer(base, named_parameters=model.named_parameters())
        enable_bf16_shadow(model, opt)
    else:
        opt = base
    order = torch.randperm(len(y_all), generator=torch.Generator().manual_seed(77 + seed)).to(dev)
    losses = []
    nb = len(y_all) // batch
    for s in range(steps):
        for gr in opt.param_groups:
            gr["lr"] = _lr(s, steps, peak=0.05)
        idx = order[(s % nb) * batch:(s % nb + 1) * batch]
        opt.zero_grad()
        with torch.autocast("cuda", dtype=torch.bfloat16):
            loss = F.cross_entropy(model(x_all[idx]).float(), y_all[idx])
        loss.backward()
        opt.step()
        losses.append(loss.item())
    model.eval()
    correct = 0
    with torch.no_grad(), torch.autocast("cuda", dtype=torch.bfloat16):
        for i in range(0, len(y_all), 256):
            correct += int((model(x_all[i:i + 256]).float().argmax(1) == y_all[i:i + 256]).sum())
    return losses, correct / len(y_all)


@needs_gpu
def test_resnet50_engine_learns_like_stock():
    st, en = [], []
    for seed in (1, 2):
        ls, acc_s = _train_resnet(False, seed=seed)
        le, acc_e = _train_resnet(True, seed=seed)
        st.append((sum(ls[-50:]) / 50, acc_s))
        en.append((sum(le[-50:]) / 50, acc_e))
        print("seed %d stock acc %.3f last-50 loss %.4f | engine acc %.3f last-50 loss %.4f" % (
            seed, acc_s, st[-1][0], acc_e, en[-1][0]))
        print("stock", [round(v, 3) for v in ls[::10]], "\nengine", [round(v, 3) for v in le[::10]])
        assert all(math.isfinite(v) for v in ls + le)
    assert all(a >= 0.95 for _, a in en), en
    mean = lambda rows, k: sum(r[k] for r in rows) / len(rows)  # noqa: E731
    assert mean(en, 1) >= mean(st, 1) - 0.02, (st, en)
    # the loss bound is absolute: stock's own last-50 loss is not reproducible run to run (MIOpen's
    # kernels are not deterministic; r6: seed 1 gave 1.62, 0.40 and 0.09 on three runs), so a bound
    # relative to it failed on a stock run that happened to converge best (engine 0.29 / 0.09,
    # deterministic).  0.5 is far below ln(10) = 2.30 and above every engine run measured.
    assert all(l <= 0.5 for l, _ in en), (st, en)


# ------------------------------------------------------------------ BERT
VOCAB_USED, SUCC = 512, 4


def _markov(n_seq, seq_len=128, seed=9, device="cuda"):
    g = torch.Generator().manual_seed(seed)
    succ = torch.randint(0, VOCAB_USED, (VOCAB_USED, SUCC), generator=g)
    probs = torch.tensor([0.55, 0.25, 0.15, 0.05])
    seqs = torch.empty(n_seq, seq_len, dtype=torch.long)
    cur = torch.randint(0, VOCAB_USED, (n_seq,), generator=g)
    for t in range(seq_len):
        seqs[:, t] = cur
        pick = torch.multinomial(probs, n_seq, replacement=True, generator=g)
        cur = succ[cur, pick]
    return (seqs + 1000).to(device)  # token ids 1000..1511 of the 30522 vocabulary


def _mlm_batch(seqs, batch, step, preds=20, mask_id=103, seed=17):
    g = torch.Generator().manual_seed(seed * 100003 + step)
    rows = torch.randint(0, seqs.shape[0], (batch,), generator=g).to(seqs.device)
    ids = seqs[rows].clone()
    B, S = ids.shape
    pos = torch.rand(B, S, generator=g).argsort(dim=1)[:, :preds].sort(dim=1).values.to(seqs.device)
    labels = torch.gather(ids, 1, pos)
    ids.scatter_(1, pos, mask_id)
    types = (torch.arange(S, device=ids.device) >= S // 2).long().expand(B, -1).contiguous()
    nsp = torch.zeros(B, dtype=torch.long, device=ids.device)
    return ids, types, pos, labels, nsp


class _StockLayer(nn.Module):
    """Plain-torch BERT layer with the fused layer's parameter names."""

    def __init__(self, d=768, heads=12, ffn=3072, dropout=0.1):
        super().__init__()
        self.heads, self.dropout = heads, dropout
        self.qkv, self.out = nn.Linear(d, 3 * d), nn.Linear(d, d)
        self.ln1 = nn.LayerNorm(d, eps=1e-12)
        self.fc1, self.fc2 = nn.Linear(d, ffn), nn.Linear(ffn, d)
        self.ln2 = nn.LayerNorm(d, eps=1e-12)

    def forward(self, x):
        B, S, D = x.shape
        p = self.dropout if self.training else 0.0
        q, k, v = self.qkv(x).view(B, S, 3, self.heads, D // self.heads).permute(2, 0, 3, 1, 4)
        a = F.scaled_dot_product_attention(q, k, v, dropout_p=p).transpose(1, 2).reshape(B, S, D)
        x = self.ln1(x + F.dropout(self.out(a), p, self.training))
        return self.ln2(x + F.dropout(self.fc2(F.gelu(self.fc1(x))), p, self.training))


def _train_bert(engine: bool, steps=160, batch=32, layers=4):
    import kungfu_amd as kf
    from kungfu_amd.models.bert import BertForPreTraining

    kf.init()
    dev = torch.device("cuda")
    torch.manual_seed(4321)
    model = BertForPreTraining(layers=layers).to(dev)
    if not engine:
        stock = nn.ModuleList([_StockLayer() for _ in range(layers)]).to(dev)
        stock.load_state_dict(model.layers.state_dict())
        model.layers = stock
    base = torch.optim.AdamW(model.parameters(), lr=0.0, weight_decay=0.01)
    if engine:
        from kungfu_amd.parallel.mixed import enable_bf16_shadow

        opt = kf.optimizers.SynchronousSGDOptimizer(base, named_parameters=model.named_parameters())
        enable_bf16_shadow(model, opt)
    else:
        opt = base
    seqs = _markov(4096)
    losses = []
    for s in range(steps):
        for gr in opt.param_groups:
            gr["lr"] = _lr(s, steps, peak=4e-4, warm=30)
        ids, types, pos, labels, _ = _mlm_batch(seqs, batch, s)
        opt.zero_grad()
        with torch.autocast("cuda", dtype=torch.bfloat16):
            mlm, _ = model(ids, types, pos)
            loss = F.cross_entropy(mlm.float().reshape(-1, mlm.shape[-1]), labels.reshape(-1))
        loss.backward()
        opt.step()
        losses.append(loss.item())
    return losses


@needs_gpu
def test_bert_engine_learns_markov_mlm_like_stock():
    ls = _train_bert(False)
    le = _train_bert(True)
    ms, me = sum(ls[-30:]) / 30, sum(le[-30:]) / 30
    print("stock", [round(v, 3) for v in ls[::10]], "\nengine", [round(v, 3) for v in le[::10]])
    print("last-30 mean: stock %.4f engine %.4f (unigram bound %.3f)" % (ms, me, math.log(VOCAB_USED)))
    assert all(math.isfinite(v) for v in ls + le)
    bound = math.log(VOCAB_USED)
    assert ms < bound and me < bound, (ms, me)
    assert abs(me - ms) <= 0.1 * max(me, ms), (ms, me)
