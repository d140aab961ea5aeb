"""PAVRM reward head: QueryAttention pooling + MLP (`diffusers_lite/utils/network.py:8-152`).

Same module tree and state-dict keys as the reference (an ``nn.MultiheadAttention`` is kept as the
parameter container so `multihead_attn.in_proj_weight` etc. load unchanged).  The K/V
in-projection over all L tokens (the only large product: [L,5120]x[5120,10240]) runs on the HIP
GEMM; the single learned query's 8-head softmax pooling over L is the split-L HIP kernel
`prfl::query_pool` (csrc/pool.hip).  Precision = the reference under bf16 autocast: bf16
projections, fp32 softmax with P rounded to bf16 before P.V (flash / SDPA numerics), bf16
attention output.
"""
import torch
import torch.nn as nn
import torch.nn.functional as F

from . import custom_ops
from .linear import linear_bf16

BF16 = torch.bfloat16


class QueryAttention(nn.Module):
    def __init__(self, feature_dim, num_queries=1, num_heads=8, dropout=0.1, layer_norm=False,
                 return_type=None, product_text=False, text_dim=768):
        super().__init__()
        self.feature_dim, self.num_queries, self.num_heads = feature_dim, num_queries, num_heads
        self.layer_norm, self.return_type, self.product_text = layer_norm, return_type, product_text
        self.dropout = dropout
        self.multihead_attn = nn.MultiheadAttention(embed_dim=feature_dim, num_heads=num_heads,
                                                    dropout=dropout, batch_first=True)
        self.queries = nn.Parameter(torch.randn(num_queries, feature_dim))
        nn.init.xavier_uniform_(self.queries)
        if product_text:
            self.text_proj = nn.Linear(text_dim, feature_dim)
            nn.init.xavier_uniform_(self.text_proj.weight)
            nn.init.zeros_(self.text_proj.bias)

    def _pool(self, x, queries):
        """x [N, L, E] (any float) -> attended [N, nq, E] bf16.  The in-projections run on the
        HIP GEMM (`prfl::linear_bf16`); the single-query softmax pooling over L is the
        `prfl::query_pool` kernel (split over L, HBM-bound), one launch per query."""
        mha = self.multihead_attn
        E, H = self.feature_dim, self.num_heads
        W, b = mha.in_proj_weight, mha.in_proj_bias
        N, L, _ = x.shape
        q = linear_bf16(queries, W[:E], b[:E])                       # [N, nq, E]
        kv = linear_bf16(x.reshape(N * L, E), W[E:], b[E:]).view(N, L, 2 * E)
        scale = float((E // H) ** -0.5)
        o = torch.stack([custom_ops.query_pool(q[:, i].contiguous(), kv, H, scale)[0]
                         for i in range(q.shape[1])], dim=1)         # [N, nq, E] bf16
        return linear_bf16(o, mha.out_proj.weight, mha.out_proj.bias)

    def forward(self, x, e=None, text=None):
        if self.layer_norm:
            x = F.layer_norm(x.float(), (self.feature_dim,), eps=1e-6)
        orig = x.shape
        if x.dim() == 2:
            x = x.unsqueeze(1)
        elif x.dim() == 4:                       # [sp, B, L, E] (network.py:65-69)
            sp, bs, L, E = x.shape
            x = x.reshape(sp * bs, L, E)
        elif x.dim() != 3:
            raise ValueError(f"Unsupported input shape: {tuple(x.shape)}")
        if self.training and self.dropout > 0:
            # nn.MultiheadAttention applies attention dropout in training mode; the query_pool
            # kernel has none (every shipped config sets dropout 0 or runs the head in eval)
            raise NotImplementedError("QueryAttention: attention dropout > 0 in training mode")
        n = x.shape[0]
        queries = self.queries.unsqueeze(0).expand(n, -1, -1)
        if e is not None:
            queries = queries + e.unsqueeze(0).expand(n, -1, -1)
        att = self._pool(x, queries)
        out = att.mean(dim=1) if self.num_queries > 1 else att.squeeze(1)
        if len(orig) == 4:
            out = out.view(orig[0], orig[1], -1).mean(dim=0)
        if self.layer_norm:
            out = F.layer_norm(out.float(), (self.feature_dim,), eps=1e-6)
        if self.return_type == "query":
            out = out + queries
        if self.product_text and text is not None:
            return linear_bf16(text, self.text_proj.weight, self.text_proj.bias) * out
        return out


class MLP(nn.Module):
    """network.py:112-134: 5120 -> 1024 -> 512 -> 1 with ReLU (logit out)."""

    def __init__(self, input_dim):
        super().__init__()
        self.fc1 = nn.Linear(input_dim, 1024)
        self.fc2 = nn.Linear(1024, 512)
        self.fc3 = nn.Linear(512, 1)
        for m in self.modules():
            if isinstance(m, nn.Linear):
                nn.init.xavier_uniform_(m.weight)
                nn.init.zeros_(m.bias)

    def forward(self, x):
        x = torch.relu(linear_bf16(x, self.fc1.weight, self.fc1.bias))
        x = torch.relu(linear_bf16(x, self.fc2.weight, self.fc2.bias))
        return linear_bf16(x, self.fc3.weight, self.fc3.bias)


def forward_mlp(model, input):
    return torch.sigmoid(model(input))


def forward_siamese(model, input1, input2):
    return torch.sigmoid(model(input1) - model(input2))
