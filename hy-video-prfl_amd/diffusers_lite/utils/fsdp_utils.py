# import path of the reference (diffusers_lite/utils/fsdp_utils.py); implementation: prfl_amd.fsdp_utils
from prfl_amd.fsdp_utils import (apply_fsdp_checkpointing, get_dit_fsdp_kwargs,  # noqa: F401
                                 get_discriminator_fsdp_kwargs, get_mixed_precision,
                                 get_vae_fsdp_kwargs, non_reentrant_wrapper)
