"""BERT-base encoder for masked-LM pre-training throughput (BASELINE.json config 5:
"BERT-base SynchronousSGD + gradient-noise-scale monitor + elastic resize").
12 layers, hidden 768, 12 heads, FFN 3072, vocab 30522, ~110 M parameters.
Attention: the fused HIP kernels of ops/attention.py (S 64/128, no mask), else torch's
scaled_dot_product_attention."""
import math

import torch
import torch.nn as nn
import torch.nn.functional as F

from ..ops.attention import self_attention
from ..ops.embedding import embedding
from ..ops.vocab import vocab_projection
from ..ops.xent import cross_entropy
from ..ops.linear import gelu, residual_link


class BertLayer(nn.Module):
    def __init__(self, d=768, heads=12, ffn=3072, dropout=0.1):
        super().__init__()
        from ..ops.layernorm import AddLayerNorm

        self.heads = heads
        self.qkv = nn.Linear(d, 3 * d)
        self.out = nn.Linear(d, d)
        # fused residual-add + LayerNorm (HIP, bf16 residual stream) -- torch.nn.LayerNorm
        # parameters and state_dict keys, torch composition off the GPU fast path
        self.ln1 = AddLayerNorm(d, eps=1e-12)
        self.fc1 = nn.Linear(d, ffn)
        self.fc2 = nn.Linear(ffn, d)
        self.ln2 = AddLayerNorm(d, eps=1e-12)
        self.dropout = dropout

    def forward(self, x, mask=None):
        B, S, D = x.shape
        p = self.dropout if self.training else 0.0
        # x feeds exactly two consumers, the QKV projection and ln1's skip input: ln1's backward hands
        # its gradient of x to the projection's data-gradient GEMM (ops.linear.ResidualLink)
        residual_link(x)
        qkv = self.qkv(x)
        if mask is None:
            # fused HIP attention straight from / into the projections' layouts (SDPA off that path)
            a = self_attention(qkv, self.heads, p)
        else:
            q, k, v = qkv.view(B, S, 3, self.heads, D // self.heads).permute(2, 0, 3, 1, 4)
            a = F.scaled_dot_product_attention(q, k, v, attn_mask=mask, dropout_p=p)
            a = a.transpose(1, 2).reshape(B, S, D)
        # residual dropout fused into the add + LayerNorm kernels (ops/layernorm.py)
        # the projections' outputs feed only their AddLayerNorm: its backward also produces their
        # bias gradients (ops.linear.BiasLink), no column-sum pass of their own
        x = self.ln1(x, self.out(a), dropout=self.dropout, bias_link=True)
        residual_link(x)  # likewise FC1 and ln2's skip input
        h = self.fc2(gelu(self.fc1(x), bias_link=True))
        return self.ln2(x, h, dropout=self.dropout, bias_link=True)


class BertForPreTraining(nn.Module):
    def __init__(self, vocab=30522, d=768, layers=12, heads=12, ffn=3072, max_pos=512, type_vocab=2):
        super().__init__()
        self.tok = nn.Embedding(vocab, d)
        self.pos = nn.Embedding(max_pos, d)
        self.typ = nn.Embedding(type_vocab, d)
        from ..ops.layernorm import AddLayerNorm

        self.ln = AddLayerNorm(d, eps=1e-12)  # embedding LayerNorm (an nn.LayerNorm: same parameters / state dict)
        self.layers = nn.ModuleList([BertLayer(d, heads, ffn) for _ in range(layers)])
        self.mlm_dense = nn.Linear(d, d)
        self.mlm_ln = AddLayerNorm(d, eps=1e-12)  # HIP LayerNorm on the bf16 head (torch's off the GPU path)
        self.mlm_bias = nn.Parameter(torch.zeros(vocab))
        self.nsp = nn.Linear(d, 2)
        self.apply(self._init)

    @staticmethod
    def _init(m):
        if isinstance(m, (nn.Linear, nn.Embedding)):
            nn.init.normal_(m.weight, std=0.02)
        if isinstance(m, nn.Linear) and m.bias is not None:
            nn.init.zeros_(m.bias)

    def forward(self, ids, types=None, mlm_positions=None):
        """Returns (MLM logits, NSP logits).  With ``mlm_positions`` ([B, P] token indices,
        the masked positions: 20 per 128-token sequence in BERT pre-training) only those
        positions go through the MLM head -- the vocabulary projection is the largest GEMM
        of the model, and pre-training never needs it for unmasked tokens."""
        B, S = ids.shape
        pos = torch.arange(S, device=ids.device)
        types = torch.zeros_like(ids) if types is None else types
        # scatter-add embedding gradients (ops/embedding.py): fixed-shape, graph-replayable
        e = embedding(ids, self.tok.weight) + embedding(pos, self.pos.weight)[None] + embedding(types, self.typ.weight)
        if torch.is_autocast_enabled(e.device.type) and e.is_cuda:
            # bf16 residual stream from here on: the f32 embedding sum is cast BEFORE its LayerNorm, which
            # then runs on the HIP kernels (layernorm.hip: one pass each way, gamma/beta straight to the flat
            # space) instead of torch's f32 LayerNorm (input-gradient + 12-block gamma/beta kernels: 88 us,
            # plus the cast of its f32 output; r5t26)
            e = e.to(torch.get_autocast_dtype(e.device.type))
        x = self.ln(e)
        for layer in self.layers:
            x = layer(x)
        hs = x
        if mlm_positions is not None:
            hs = torch.gather(x, 1, mlm_positions.unsqueeze(-1).expand(-1, -1, x.shape[-1]))
        h = self.mlm_ln(F.gelu(self.mlm_dense(hs)))
        # tied output embedding; gemm.hip's ragged-N GEMM with padded logits rows (ops/vocab.py)
        mlm = vocab_projection(h, self.tok.weight, self.mlm_bias)
        return mlm, self.nsp(x[:, 0])


def bert_base(**kw):
    kw.pop("fused_bn", None)
    return BertForPreTraining(**kw)


def synthetic_pretraining_batch(batch: int, seq_len: int = 128, vocab: int = 30522, max_predictions: int = 20,
                                device=None, generator=None):
    """Random BERT pre-training batch of the real shapes: token ids, segment ids, masked
    positions (distinct per sequence) with their labels, and next-sentence labels."""
    kw = dict(device=device, generator=generator)
    ids = torch.randint(0, vocab, (batch, seq_len), **kw)
    types = (torch.arange(seq_len, device=device) >= seq_len // 2).long().expand(batch, -1).contiguous()
    pos = torch.rand(batch, seq_len, **kw).argsort(dim=1)[:, :max_predictions].sort(dim=1).values
    mlm_labels = torch.randint(0, vocab, (batch, max_predictions), **kw)
    nsp_labels = torch.randint(0, 2, (batch,), **kw)
    return ids, types, pos, mlm_labels, nsp_labels


def pretraining_loss(model, batch):
    ids, types, pos, mlm_labels, nsp_labels = batch
    mlm, nsp = model(ids, types, pos)
    # MLM loss straight from the bf16 logits (ops/xent.py: no f32 copies of the 2560 x 30522 logits)
    return cross_entropy(mlm, mlm_labels) + F.cross_entropy(nsp.float(), nsp_labels)
