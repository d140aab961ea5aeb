from prfl_amd.network import MLP, QueryAttention, forward_mlp, forward_siamese  # noqa: F401
