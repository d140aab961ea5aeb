# import path of the reference (diffusers_lite/utils/network.py); implementation: prfl_amd.network
from prfl_amd.network import (MLP, MultiHead, QueryAttention, forward_mlp,  # noqa: F401
                              forward_siamese, save_model, train_model)
