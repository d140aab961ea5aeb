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


class MultiHead(nn.Module):
    """network.py:136-149: `num_heads` independent reward MLPs over one feature; forward returns
    the stacked sigmoid scores [num_heads, ..., 1]."""

    def __init__(self, input_dim, num_heads=3):
        super().__init__()
        self.num_heads = num_heads
        self.mlps = nn.ModuleList(MLP(input_dim) for _ in range(num_heads))

    def forward_mlp(self, head_idx, x):
        return torch.sigmoid(self.mlps[head_idx](x))

    def forward(self, x):
        return torch.stack([self.forward_mlp(h, x) for h in range(self.num_heads)])


def forward_mlp(model, input):
    return torch.sigmoid(model(input))


def forward_siamese(model, input1, input2):
    return torch.sigmoid(model(input1) - model(input2))


def _scores(model, model_mode, X):
    # fp32 scores for BCELoss against fp32 targets: this package's MLP returns bf16 (its Linears
    # are autocast-style bf16 GEMMs), the reference's fp32 nn.Linear MLP returns fp32
    if model_mode == "clf":
        return forward_mlp(model, X).float()
    if model_mode == "siamese":                   # X [N, 2, ...]: pair (preferred, other)
        return forward_siamese(model, X[:, 0], X[:, 1]).float()
    raise ValueError(f"model_mode must be 'clf' or 'siamese', got {model_mode!r}")


def train_model(model, device, model_mode, X_train, y_train, X_test, y_test, epochs=3, lr=0.001,
                batch_size=512, verbose=False, ealry_stopping_patience=3):
    """network.py:164-214: fit a reward MLP on cached features with Adam + BCE.

    Each epoch runs ceil(N / batch_size) steps, every step on a fresh random subset of
    `batch_size` rows (drawn with torch.randperm, so it follows the global torch seed as the
    reference does); after the epoch the validation BCE is recorded and training stops once it
    exceeds each of the previous `ealry_stopping_patience` values (the reference's spelling of
    the keyword is kept so callers passing it by name still work).  Returns the model (the
    reference returns None; callers ignore the result).

    Device: the reference trains an fp32 nn.Linear MLP and runs on the CPU too.  This package's
    MLP runs its Linears through `prfl::linear_bf16` (bf16 operands, fp32 accumulate, as under
    the drivers' autocast), a HIP op with no CPU path: `train_model(MLP(...), "cpu", ...)` raises
    NotImplementedError from the op.  A plain torch classifier trains on any device.  The scores
    are cast to fp32 before the BCE."""
    model = model.to(device)
    bce = nn.BCELoss()
    opt = torch.optim.Adam(model.parameters(), lr=lr)
    n = X_train.shape[0]
    batch_size = min(batch_size, n)
    history = []
    for epoch in range(epochs):
        model.train()
        loss = None
        for _ in range(0, n, batch_size):
            pick = torch.randperm(n)[:batch_size]
            opt.zero_grad()
            loss = bce(_scores(model, model_mode, X_train[pick]), y_train[pick])
            loss.backward()
            opt.step()
        model.eval()
        with torch.no_grad():
            val = _scores(model, model_mode, X_test)
        val_loss = float(bce(val, y_test))
        history.append(val_loss)
        p = ealry_stopping_patience
        if len(history) > p and all(history[-1] > h for h in history[-(p + 1):-1]):
            if verbose:
                print(f"Early stopping at epoch {epoch + 1}")
            break
        if verbose:
            acc = ((val > 0.5).to(y_test.dtype) == y_test).float().mean().item()
            print(f"Epoch {epoch + 1}/{epochs}, Loss: {float(loss)}, Val Loss: {val_loss}")
            print(f"Accuracy: {acc}")
    return model


def save_model(model, path):
    """network.py:216-217."""
    torch.save(model.state_dict(), path)
