"""Drop-in for `diffusers_lite/utils/fsdp_utils.py` and `diffusers_lite/utils/load.py`: the FSDP
keyword set and the activation-checkpoint policy the reference drivers apply
(`train_prfl.py:346-374`, `train_pavrm.py:264-285`), usable on the MI355X blocks unchanged.

Why it composes: `WanAttentionBlock.forward` is the `prfl::wan_block` custom op, whose inputs are
the block's parameters fetched by attribute path — under FSDP (FULL_SHARD, use_orig_params False)
those are views of the all-gathered flat parameter during forward and backward, so gradients flow
to the flat parameter through an ordinary autograd node, and `transformer.clip_grad_norm_` sees
them.  A non-reentrant `checkpoint_wrapper` around the block also composes (autograd recomputes
the op), but the op already IS the reference's per-block checkpoint (its backward recomputes the
block from the block input, `fsdp_utils.py:17-50`); wrapping it again would recompute the block
forward twice.  So `apply_fsdp_checkpointing` counts fused blocks in its selective-checkpointing
schedule exactly as the reference does and leaves them unwrapped (``wrap_fused=True`` wraps them
anyway); any other module type in `no_split_modules` is wrapped as in the reference.
"""
import functools

import torch
from torch.distributed.algorithms._checkpoint.checkpoint_wrapper import (
    CheckpointImpl,
    apply_activation_checkpointing,
    checkpoint_wrapper,
)
from torch.distributed.fsdp import MixedPrecision, ShardingStrategy
from torch.distributed.fsdp.wrap import transformer_auto_wrap_policy

non_reentrant_wrapper = functools.partial(checkpoint_wrapper,
                                          checkpoint_impl=CheckpointImpl.NO_REENTRANT)


def get_no_split_modules(transformer):
    """`utils/load.py:6-12`: the FSDP / checkpoint unit of a WanModel is the WanAttentionBlock."""
    from .model import WanAttentionBlock, WanModel
    base = transformer
    while hasattr(base, "base_model") and hasattr(base.base_model, "model"):   # PeftModel
        base = base.base_model.model
    if isinstance(base, WanModel):
        return (WanAttentionBlock,)
    raise ValueError(f"Unsupported transformer type: {type(transformer)}")


def apply_fsdp_checkpointing(model, no_split_modules, p=1, wrap_fused=False):
    """`fsdp_utils.py:23-50`: checkpoint every 1/p-th module of the `no_split_modules` types
    (p may be a fraction string such as "1/3").  Fused self-checkpointing blocks are counted but
    not wrapped unless `wrap_fused` (see the module docstring)."""
    block_idx = 0
    cut_off = 1 / 2
    p = _fraction(p)

    def selective_checkpointing(submodule):
        nonlocal block_idx, cut_off
        if isinstance(submodule, no_split_modules):
            block_idx += 1
            if block_idx * p >= cut_off:
                cut_off += 1
                fused = getattr(submodule, "self_checkpointing", False)
                if fused and wrap_fused:
                    # the wrapper's recompute must see the same (empty) attention stash
                    submodule.stash_attn = False
                return wrap_fused or not fused
        return False

    apply_activation_checkpointing(model, checkpoint_wrapper_fn=non_reentrant_wrapper,
                                   check_fn=selective_checkpointing)


def _fraction(p):
    if isinstance(p, str):
        num, _, den = p.partition("/")
        return float(num) / float(den) if den else float(num)
    return p


def get_mixed_precision(master_weight_type="fp32"):
    """`fsdp_utils.py:53-63`: fp32 (or bf16) params, gradient reduction and buffers."""
    weight_type = torch.float32 if master_weight_type == "fp32" else torch.bfloat16
    return MixedPrecision(param_dtype=weight_type, reduce_dtype=weight_type,
                          buffer_dtype=weight_type, cast_forward_inputs=False)


_STRATEGIES = {"full": ShardingStrategy.FULL_SHARD, "hybrid_full": ShardingStrategy.HYBRID_SHARD,
               "none": ShardingStrategy.NO_SHARD,
               "hybrid_zero2": ShardingStrategy._HYBRID_SHARD_ZERO2,
               "shard_grad_op": ShardingStrategy.SHARD_GRAD_OP}


def get_dit_fsdp_kwargs(transformer, sharding_strategy, use_lora=False, cpu_offload=False,
                        master_weight_type="fp32"):
    """`fsdp_utils.py:66-122` for the full fine-tune (the LoRA variant needs peft, which the
    PRFL / PAVRM configs do not use: `use_lora: false`)."""
    if use_lora:
        raise NotImplementedError("LoRA fine-tuning is out of scope (configs set use_lora: false)")
    no_split_modules = get_no_split_modules(transformer)
    auto_wrap_policy = functools.partial(transformer_auto_wrap_policy,
                                         transformer_layer_cls=no_split_modules)
    strategy = _STRATEGIES[sharding_strategy]
    if sharding_strategy == "none":
        auto_wrap_policy = None
    kwargs = {
        "auto_wrap_policy": auto_wrap_policy,
        "mixed_precision": get_mixed_precision(master_weight_type),
        "sharding_strategy": strategy,
        "device_id": torch.cuda.current_device(),
        "limit_all_gathers": True,
        "cpu_offload": (torch.distributed.fsdp.CPUOffload(offload_params=True) if cpu_offload
                        else None),
    }
    return kwargs, no_split_modules


def get_discriminator_fsdp_kwargs(master_weight_type="fp32"):
    """`fsdp_utils.py:125-140`: an unwrapped, unsharded FSDP unit for small side models."""
    return {"auto_wrap_policy": None,
            "mixed_precision": get_mixed_precision(master_weight_type),
            "sharding_strategy": ShardingStrategy.NO_SHARD,
            "device_id": torch.cuda.current_device(),
            "limit_all_gathers": True}


def get_vae_fsdp_kwargs(master_weight_type="fp32", cpu_offload=False):
    """`fsdp_utils.py:141-168`: the frozen VAE as one FULL_SHARD unit with original parameters
    (the VAE itself is outside this repo's scope; the keyword set is provided so the PRFL driver's
    import line and its `FSDP(vae, **get_vae_fsdp_kwargs(...))` call stay unchanged)."""
    return {"auto_wrap_policy": None,
            "mixed_precision": get_mixed_precision(master_weight_type),
            "sharding_strategy": ShardingStrategy.FULL_SHARD,
            "device_id": torch.cuda.current_device(),
            "limit_all_gathers": True,
            "cpu_offload": (torch.distributed.fsdp.CPUOffload(offload_params=True) if cpu_offload
                            else None),
            "use_orig_params": True}
