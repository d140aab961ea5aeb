from prfl_amd.model import *  # noqa: F401,F403
from prfl_amd.model import (Head, MLPProj, WanAttentionBlock, WanI2VCrossAttention,  # noqa: F401
                            WanLayerNorm, WanModel, WanRMSNorm, WanSelfAttention,
                            WanT2VCrossAttention, rope_apply, rope_params,
                            sinusoidal_embedding_1d)
from prfl_amd.attention import flash_attention  # noqa: F401
