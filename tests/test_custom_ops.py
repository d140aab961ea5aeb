"""The torch.library operator boundary on the CPU host (no GPU): every `prfl::` op is registered
with its schema, has a fake (meta) implementation that propagates shapes / dtypes, and has NO CPU
kernel (a CPU tensor fails loudly); the FSDP / checkpoint drop-ins select modules as the
reference's `apply_fsdp_checkpointing` (`fsdp_utils.py:23-50`) does."""
import pytest
import torch
from torch._subclasses.fake_tensor import FakeTensorMode

from shapes import TOY, block_shapes

OPS = ["wan_block", "wan_block_backward", "linear_bf16", "linear_bf16_backward", "flash_attention",
       "flash_attention_backward", "query_pool", "query_pool_backward", "unipc_step",
       "unipc_step_backward"]


@pytest.fixture(scope="module")
def cops():
    from prfl_amd import custom_ops
    return custom_ops


def test_ops_registered_with_schemas(cops):
    for name in OPS:
        schema = str(getattr(torch.ops.prfl, name).default._schema)
        assert schema.startswith(f"prfl::{name}("), schema
    s = str(torch.ops.prfl.wan_block.default._schema)
    assert "Tensor[] params" in s and "bool keep_attn" in s and s.endswith("-> (Tensor, Tensor, Tensor)")


def test_no_cpu_kernel(cops):
    with pytest.raises(NotImplementedError):
        torch.ops.prfl.linear_bf16(torch.zeros(3, 8), torch.zeros(8, 8), None, False)
    with pytest.raises(NotImplementedError):
        torch.ops.prfl.flash_attention(torch.zeros(1, 4, 1, 128), torch.zeros(1, 4, 1, 128),
                                       torch.zeros(1, 4, 1, 128), None, 0.1)


def test_fake_shapes(cops):
    from prfl_amd.block import param_names
    with FakeTensorMode():
        dev = "cuda"
        x = torch.empty(1, 105, 256, device=dev)
        e = torch.empty(1, 6, 256, device=dev)
        ctx = torch.empty(1, 512, 256, device=dev, dtype=torch.bfloat16)
        shapes = dict((n[len("b."):], s) for n, s in block_shapes("b.", 256, 512))
        params = [torch.empty(shapes[n], device=dev) for n in param_names(False)]
        tab = torch.empty(1024, 64, 2, device=dev)
        out, ao, lse = torch.ops.prfl.wan_block(x, e, ctx, params, 2, [3, 5, 7], [105], tab,
                                                False, 1e-6, 0, True)
        assert out.shape == (1, 105, 256) and out.dtype == torch.float32
        assert ao.shape == (1, 105, 256) and ao.dtype == torch.bfloat16 and lse.shape == (1, 2, 105)
        _, ao0, _ = torch.ops.prfl.wan_block(x, e, ctx, params, 2, [3, 5, 7], [105], tab, False,
                                             1e-6, 0, False)
        assert ao0.numel() == 0
        g = torch.ops.prfl.wan_block_backward(out, x, e, ctx, params, ao, lse, 2, [3, 5, 7], [105],
                                              tab, False, 1e-6, 0, True, True)
        assert [t.shape for t in g[3:]] == [p.shape for p in params] and g[2].shape == ctx.shape
        o, l2, o32 = torch.ops.prfl.query_pool(torch.empty(2, 5120, device=dev, dtype=torch.bfloat16),
                                          torch.empty(2, 77, 10240, device=dev, dtype=torch.bfloat16),
                                          8, 0.04)
        assert o.shape == (2, 5120) and l2.shape == (2, 8) and o32.dtype == torch.float32
        y, pre = torch.ops.prfl.linear_bf16(x, torch.empty(512, 256, device=dev), None, True)
        assert y.shape == (1, 105, 512) and pre.shape == (105, 512)


def _toy_model():
    from prfl_amd.model import WanModel
    return WanModel(model_type="t2v", in_dim=16, **TOY)


@pytest.mark.parametrize("p,wrap_fused,expect", [(1, False, 0), (1, True, 2), ("1/2", True, 1)])
def test_apply_fsdp_checkpointing_selection(p, wrap_fused, expect):
    from torch.distributed.algorithms._checkpoint.checkpoint_wrapper import CheckpointWrapper
    from prfl_amd.fsdp_utils import apply_fsdp_checkpointing, get_no_split_modules
    m = _toy_model()
    ns = get_no_split_modules(m)
    apply_fsdp_checkpointing(m, ns, p, wrap_fused=wrap_fused)
    assert sum(isinstance(mod, CheckpointWrapper) for mod in m.modules()) == expect


def test_from_pretrained_rejects_missing_keys(tmp_path):
    from prfl_amd.model import WanModel
    m = _toy_model()
    m.save_pretrained(str(tmp_path))
    WanModel.from_pretrained(str(tmp_path))                       # complete checkpoint loads
    from safetensors.torch import load_file, save_file
    f = next(p for p in tmp_path.iterdir() if p.suffix == ".safetensors")
    sd = load_file(str(f))
    del sd["blocks.1.ffn.0.weight"]
    save_file(sd, str(f))
    with pytest.raises(RuntimeError, match="missing"):
        WanModel.from_pretrained(str(tmp_path))
    WanModel.from_pretrained(str(tmp_path), allow_missing=("blocks.1.ffn.0",))
