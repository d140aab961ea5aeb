"""CPU-side checks: C-ABI library loads and exports every declared symbol, module/state-dict
parity with the reference, import-path shim, host schedulers vs the reference fixtures, and the
no-CPU-fallback guarantee."""
import os
import re

import numpy as np
import pytest
import torch

from shapes import TOY, REAL, model_shapes

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def declared_symbols():
    src = open(os.path.join(ROOT, "include", "prfl_hip.h")).read()
    return sorted(set(re.findall(r"\b(?:int|int64_t)\s+(prfl_[a-z0-9_]+)\s*\(", src)))


def test_abi_library_exports_header():
    from prfl_amd import _lib
    lib = _lib.load()                     # dlopen works without a GPU
    syms = declared_symbols()
    assert len(syms) >= 18
    for s in syms:
        assert hasattr(lib, s), s
        assert s in _lib.SIGNATURES, f"{s} has no ctypes signature"


def test_abi_stale_rms_rope_names_removed():
    """The unsuffixed prfl_rms_rope_fwd / _bwd carried two signatures (round 2 without out_scale,
    round 3 with it); a caller built against either must fail to resolve, not run with a silently
    dropped scale (ABI history)."""
    from prfl_amd import _lib
    lib = _lib.load()
    for s in ("prfl_rms_rope_fwd", "prfl_rms_rope_bwd"):
        assert not hasattr(lib, s), s
        assert s not in declared_symbols()
    assert hasattr(lib, "prfl_rms_rope_fwd_scaled") and hasattr(lib, "prfl_rms_rope_bwd_scaled")


def test_no_cpu_fallback():
    from prfl_amd import ops
    x = torch.zeros(8, 64, dtype=torch.bfloat16)
    w = torch.zeros(64, 64, dtype=torch.bfloat16)
    with pytest.raises(RuntimeError):
        ops.linear(x, w)


@pytest.mark.parametrize("model_type", ["t2v", "i2v"])
def test_state_dict_keys_match_reference(model_type):
    from prfl_amd.model import WanModel
    m = WanModel(model_type=model_type, in_dim=16 if model_type == "t2v" else 36, **TOY)
    ours = {k: tuple(v.shape) for k, v in m.state_dict().items()}
    ref = dict(model_shapes(TOY, model_type))
    assert ours == ref


def test_real_config_param_count():
    """14B T2V: 14.288 B parameters, 351.4 M per block."""
    n = sum(int(np.prod(s)) for _, s in model_shapes(REAL, "t2v"))
    assert abs(n / 1e9 - 14.288) < 0.01
    nb = sum(int(np.prod(s)) for k, s in model_shapes(REAL, "t2v") if k.startswith("blocks.0."))
    assert abs(nb / 1e6 - 351.4) < 0.5


def _driver_imports():
    import json
    return json.load(open(os.path.join(ROOT, "tests", "golden", "driver_imports.json")))


def test_dropin_resolves_every_reference_import(monkeypatch):
    """After `prfl_amd.dropin.install()` (the INTEGRATION.md preamble), every `from <replaced
    module> import <name>` anywhere in the reference — train_prfl.py:29-97, train_pavrm.py:28-74,
    inference_pavrm.py, the package's own relative imports — resolves (VERDICT r03 missing #1:
    train_model / save_model / get_vae_fsdp_kwargs were absent and the drivers died on import)."""
    import sys
    from prfl_amd import dropin
    table = _driver_imports()
    assert set(table) == set(dropin.MODULE_MAP)
    for ref_name in dropin.MODULE_MAP:
        monkeypatch.delitem(sys.modules, ref_name, raising=False)
    dropin.install()
    n = 0
    for mod, entry in table.items():
        for name, sites in entry["imported"].items():
            ns = {}
            exec(f"from {mod} import {name}", ns)        # the driver's own statement form
            assert ns[name] is not None, (mod, name, sites)
            n += 1
    assert n >= 15
    for ref_name in dropin.MODULE_MAP:
        monkeypatch.delitem(sys.modules, ref_name, raising=False)
    from diffusers_lite.wan.modules.model import WanModel
    assert WanModel._no_split_modules == ["WanAttentionBlock"]
    assert WanModel.enable_teacache is False


def test_dropin_modules_define_every_reference_name():
    """Each replacement module exports every top-level name its reference module defines."""
    import importlib
    from prfl_amd import dropin
    for ref_name, entry in _driver_imports().items():
        ours = importlib.import_module(dropin.MODULE_MAP[ref_name])
        missing = [x for x in entry["defined"] if not hasattr(ours, x)]
        assert not missing, (ref_name, missing)


def test_driver_imports_fixture_is_current():
    """The committed fixture equals a fresh parse of the reference sources (skipped where the
    reference is absent, e.g. on the GPU box)."""
    import importlib.util
    import json
    if not os.path.isdir("/root/reference/scripts"):
        pytest.skip("reference sources not present")
    spec = importlib.util.spec_from_file_location(
        "mdi", os.path.join(ROOT, "tests", "golden", "make_driver_imports.py"))
    mdi = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mdi)
    fresh = {}
    for ref_mod in mdi.MODULE_MAP:
        path = os.path.join(mdi.REF, *ref_mod.split(".")) + ".py"
        fresh[ref_mod] = mdi.defined_names(path)
    table = _driver_imports()
    assert {k: v["defined"] for k, v in table.items()} == fresh
    assert json.dumps(table["diffusers_lite.utils.network"]["imported"]).count("train_prfl.py") >= 6


def test_train_model_and_save_model(tmp_path):
    """network.train_model / save_model (network.py:164-217) on a plain torch classifier, both
    modes; the reward MLPs themselves run on the GPU GEMM."""
    from prfl_amd.network import save_model, train_model
    torch.manual_seed(0)
    X = torch.randn(256, 8)
    y = (X[:, :1] > 0).float()
    for mode, Xt in (("clf", X), ("siamese", torch.stack([X, -X], dim=1))):
        m = torch.nn.Sequential(torch.nn.Linear(8, 16), torch.nn.ReLU(), torch.nn.Linear(16, 1))
        before = torch.nn.functional.binary_cross_entropy(
            torch.sigmoid(m(X) - (m(-X) if mode == "siamese" else 0)), y).item()
        out = train_model(m, "cpu", mode, Xt, y, Xt, y, epochs=20, lr=1e-2, batch_size=64)
        after = torch.nn.functional.binary_cross_entropy(
            torch.sigmoid(m(X) - (m(-X) if mode == "siamese" else 0)), y).item()
        assert out is m and after < 0.6 * before, (mode, before, after)
        save_model(m, tmp_path / f"{mode}.ckpt")
        sd = torch.load(tmp_path / f"{mode}.ckpt", weights_only=True)
        assert all(torch.equal(sd[k], v) for k, v in m.state_dict().items())
    with pytest.raises(ValueError):
        train_model(m, "cpu", "ranking", X, y, X, y, epochs=1)
    # this package's reward MLP is a bf16 GEMM on the HIP op: no CPU path, documented
    from prfl_amd.network import MLP
    with pytest.raises(NotImplementedError):
        train_model(MLP(8), "cpu", "clf", X, y, X, y, epochs=1)


def test_adamw_host_moment_fraction_is_the_update_order_tail():
    """state_on_host = f: the moments of the shortest tail of the parameters in update order
    (attach(): embeddings, blocks 0..n-1, head) holding >= f of the elements live on the host."""
    from prfl_amd.optim import AdamW

    class Toy(torch.nn.Module):
        def __init__(self):
            super().__init__()
            self.emb = torch.nn.Linear(8, 32)
            self.blocks = torch.nn.ModuleList([torch.nn.Linear(32, 32) for _ in range(10)])
            self.head = torch.nn.Linear(32, 4)

    m = Toy()
    total = sum(p.numel() for p in m.parameters())
    for f in (0.2, 0.5, 1.0):
        opt = AdamW(list(m.parameters()), state_on_host=f)
        opt.attach(m)
        hp = opt._host_params()
        n = sum(p.numel() for p in hp)
        k = len(hp)
        assert all(p in hp for p in opt.params[-k:]) and not any(p in hp for p in opt.params[:-k])
        assert n >= f * total and n - opt.params[-k].numel() < f * total
        assert m.head.weight in hp
    assert AdamW(list(m.parameters()), state_on_host=False)._host_params() == set()
    with pytest.raises(ValueError):
        AdamW(list(m.parameters()), state_on_host=1.5)._host_params()


def test_fp8_path_keeps_fp32_masters():
    """C5 quantises its e4m3 weights from the fp32 masters every pass: a bf16-stored trunk is
    refused in either order, and the PRFL trainer keeps an fp8 trunk in fp32."""
    from prfl_amd.model import WanModel
    from prfl_amd.train import store_frozen_bf16
    kw = dict(dim=64, ffn_dim=128, num_heads=2, num_layers=1, in_dim=16)
    m = WanModel(**kw).set_fp8_gemm(True)
    m.requires_grad_(False)
    with pytest.raises(ValueError, match="fp8"):
        store_frozen_bf16(m)
    m2 = WanModel(**kw)
    m2.requires_grad_(False)
    store_frozen_bf16(m2)
    assert m2.blocks[0].ffn[0].weight.dtype == torch.bfloat16
    with pytest.raises(ValueError, match="fp32"):
        m2.set_fp8_gemm(True)


def test_unipc_product_vs_reference(golden):
    """The product scheduler's host logic (step bookkeeping + scalar coefficients) with the
    oracle's restatement of the element-wise body standing in for the fused HIP kernel (which
    tests/test_gpu_kernels.py checks bit-exact against the same golden trajectory)."""
    from oracle.wan_oracle import unipc_update
    from prfl_amd.schedulers import FlowUniPCMultistepScheduler
    g = golden("schedulers")
    sch = FlowUniPCMultistepScheduler(num_train_timesteps=1000, shift=1, use_dynamic_shifting=False)
    sch._update = unipc_update
    sch.set_timesteps(num_inference_steps=40, device="cpu", shift=5.0)
    assert np.array_equal(sch.timesteps.numpy(), g["unipc_timesteps"])
    assert np.array_equal(sch.sigmas.numpy(), g["unipc_sigmas"])
    lat = torch.from_numpy(g["unipc_lat0"]).to(torch.bfloat16).view(1, 16, 3, 10, 14)
    for i in range(6):
        lat = sch.step(torch.from_numpy(g["unipc_model_outputs"][i]), sch.timesteps[i], lat,
                       return_dict=False)[0]
        assert lat.dtype == torch.bfloat16
        assert torch.equal(lat.float(), torch.from_numpy(g["unipc_traj"][i])), i
    mo = torch.from_numpy(g["unipc_mo6"]).requires_grad_(True)
    prev = sch.step(mo, sch.timesteps[6], lat, return_dict=False)[0]
    assert torch.equal(prev.float().detach(), torch.from_numpy(g["unipc_prev6"]))
    (prev.float() * torch.from_numpy(g["unipc_w"])).sum().backward()
    assert torch.allclose(mo.grad, torch.from_numpy(g["unipc_dmo6"]), rtol=1e-5, atol=1e-6)


def test_flowmatch_product_vs_reference(golden):
    from prfl_amd.schedulers import FlowMatchDiscreteScheduler
    g = golden("schedulers")
    fm = FlowMatchDiscreteScheduler(shift=5.0)
    fm.set_timesteps(1000, dtype=torch.int64)
    assert np.array_equal(fm.timesteps.numpy(), g["fm_timesteps"])
    assert np.array_equal(fm.sigmas.numpy(), g["fm_sigmas"])
    torch.manual_seed(7)
    t, s = fm.get_train_timestep_and_sigma(weighting_scheme="uniform", batch_size=1, n_dim=5)
    assert np.array_equal(t.numpy(), g["fm_sample_t"])
    assert np.array_equal(s.numpy(), g["fm_sample_sigma"])


def test_bench_stash_only_where_moments_leave_hbm():
    """bench.py keeps attention outputs only on the 720p workloads (AdamW moments on the host);
    at 480p the moments stay in HBM and a stash beside them runs out of memory."""
    import argparse
    import importlib.util
    spec = importlib.util.spec_from_file_location("prfl_bench", os.path.join(ROOT, "bench.py"))
    bench = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(bench)
    fits = {w: bench.big_fits(argparse.Namespace(workload=w))
            for w in ("prfl_t2v_720", "prfl_i2v_720", "prfl_t2v_480", "pavrm_t2v_480")}
    assert fits == {"prfl_t2v_720": True, "prfl_i2v_720": True, "prfl_t2v_480": False,
                    "pavrm_t2v_480": False}


@pytest.mark.parametrize("model", ["t2v", "i2v"])
def test_720p_data_parallel_memory_plan_fits(model):
    """The N = 8 plan at 720p x 81f (tools/memory_plan.py; unmeasured on hardware), T2V and the
    C5 I2V model (16.4 B): the analytic per-rank budget and the latest N = 1 measurement of that
    model adjusted to the N > 1 stash plus an RCCL buffer bound leave >= 20 GB of the 288 GiB
    card."""
    import glob
    import json
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path.insert(0, os.path.join(root, "tools"))
    import memory_plan as mp
    stash = mp.default_stash(model, 8)
    rows = mp.analytic(8, stash, model)
    assert rows["RCCL buffers"] > 0 and sum(rows.values()) < mp.CARD_GB - 20
    pat = "r0*_bench_prfl720_*.json" if model == "t2v" else "r0*_bench_prfl_i2v720_*.json"
    runs = sorted(glob.glob(os.path.join(root, "profiles", pat)))
    runs = [r for r in runs if json.load(open(r)).get("n_gpus") == 1
            and json.load(open(r)).get("config", {}).get("latent") == [16, 21, 88, 160]
            and "peak_alloc_gb_rank0" in json.load(open(r))]
    assert runs
    alloc, res = mp.from_measurement(8, stash, runs[-1])
    assert res < mp.CARD_GB - 20, (runs[-1], alloc, res)


def test_external_checkpoint_turns_the_attention_stash_off():
    """apply_fsdp_checkpointing(wrap_fused=True) wraps the fused blocks in a second, external
    non-reentrant checkpoint; its recompute must see the same keep decision as the original
    forward, so those blocks never stash.  Unwrapped blocks keep it."""
    from prfl_amd.fsdp_utils import apply_fsdp_checkpointing, get_no_split_modules
    from prfl_amd.model import WanModel
    for wrap in (False, True):
        m = WanModel(model_type="t2v", in_dim=16, **TOY)
        apply_fsdp_checkpointing(m, get_no_split_modules(m), p=1, wrap_fused=wrap)
        blocks = [mod for mod in m.modules() if type(mod).__name__ == "WanAttentionBlock"]
        assert len(blocks) == TOY["num_layers"]
        assert all(b.stash_attn is (not wrap) for b in blocks)


def test_query_attention_rejects_training_dropout():
    """nn.MultiheadAttention applies attention dropout in training mode; the pooling kernel has
    none, so QueryAttention refuses instead of silently differing."""
    from prfl_amd.network import QueryAttention
    qa = QueryAttention(64, 1, 8, dropout=0.1)
    qa.train()
    with pytest.raises(NotImplementedError):
        qa(torch.zeros(1, 4, 64))


def test_loss_guard_matches_reference_semantics():
    """`train_prfl.py:800-811` (single process): NaN / Inf -> skip; |loss| > 1e6 -> clamp, whose
    gradient is zero; otherwise the loss and its gradient pass unchanged."""
    from prfl_amd.train import guard_loss
    assert guard_loss(torch.tensor(float("nan"))) is None
    assert guard_loss(torch.tensor(float("-inf"))) is None
    x = torch.tensor(2.0, requires_grad=True)
    big = guard_loss(x * 1e6)
    assert float(big) == 1e6
    big.backward()
    assert float(x.grad) == 0.0
    y = torch.tensor(0.3, requires_grad=True)
    ok = guard_loss(y * 2)
    ok.backward()
    assert float(ok) == float(torch.tensor(0.3) * 2) and float(y.grad) == 2.0


@pytest.mark.parametrize("state", [True, False])
def test_sp_state_follows_reference_parallel_states(monkeypatch, state):
    """The drop-in reads the reference's own `parallel_states` (initialised by the drivers from
    the YAML's `sp_size`, `train_prfl.py:118`): with SP on, `prfl_amd.sp.current()` reports the
    group, rank and size of `nccl_info` and WanModel.forward runs the Ulysses path (round 5
    refused it instead); an explicit `sp.set_group(False)` overrides it."""
    import sys
    import types
    from prfl_amd import sp
    ps = types.ModuleType("diffusers_lite.utils.parallel_states")
    ps.get_sequence_parallel_state = lambda: state
    grp = object()
    ps.nccl_info = types.SimpleNamespace(sp_size=4 if state else 1, group=grp,
                                         rank_within_group=2 if state else 0)
    monkeypatch.setitem(sys.modules, "diffusers_lite.utils.parallel_states", ps)
    sp.clear()
    st = sp.current()
    if state:
        assert (st.group, st.rank, st.size) == (grp, 2, 4)
        assert sp.lookup(sp.register(st)) is st
        assert sp.split_len(73920, st) == 18480
        with pytest.raises(ValueError, match="divisible"):
            sp.split_len(10, st)
    else:
        assert st is None and sp.register(st) == 0 and sp.lookup(0) is None
    try:
        sp.set_group(False)
        assert sp.current() is None
    finally:
        sp.clear()


def test_flash_attention_length_arguments():
    """`q_lens` / `k_lens` host logic of the drop-in (wan/modules/attention.py:63-80, 110): full
    q_lens are accepted, shorter ones fail as the reference's unflatten does, bad k_lens are
    refused before any device work (the checks run ahead of the custom op, so no GPU here)."""
    from prfl_amd import attention as A
    q = torch.zeros(2, 6, 1, 128)
    k = torch.zeros(2, 9, 1, 128)
    with pytest.raises(RuntimeError, match="unflattened"):
        A.flash_attention(q, k, k, q_lens=torch.tensor([6, 4]))
    with pytest.raises(ValueError, match="entries"):
        A.flash_attention(q, k, k, k_lens=[9])
    with pytest.raises(ValueError, match="outside"):
        A.flash_attention(q, k, k, k_lens=torch.tensor([9, 10]))
    with pytest.raises(ValueError, match="outside"):
        A.flash_attention(q, k, k, k_lens=[0, 9])
    assert A._lens(torch.tensor([6, 6], dtype=torch.int32), 2, 6, "q_lens") == [6, 6]
    assert A._lens((3, 9), 2, 9, "k_lens", lo=1) == [3, 9]
