"""PRFL training-step benchmark (BASELINE.json metric) on 1..8 MI355X, one process per GPU.

    python bench.py [--gpus N] [--steps K] [--warmup W]
                    [--workload prfl_t2v_720|prfl_t2v_480|prfl_i2v_720|pavrm_t2v_480]
    torchrun --nproc-per-node N --master-addr 127.0.0.1 bench.py --gpus N ...

Workload (default): `configs/train_prfl_t2v_720.yaml` — the metric's 720p x 81f configuration
(latent [16,21,88,160] -> L = 73920 tokens) — one sample per GPU: the full PRFL iteration
(flow-matching SFT step + reward step: 19-step no-grad UniPC rollout, grad-enabled generator
step, differentiable UniPC step, 8-block latent reward model + QueryAttention + MLP, backward
through all of it, clip, AdamW every 5th micro-step; the timed window ends on an optimizer step)
on the 14B Wan2.1 T2V DiT (40 blocks, C=5120), random-init weights (head perturbed so gradients
are non-zero), synthetic latents/text.  Memory plan: on one GPU the AdamW moments
live in pinned host memory and stream through HBM during the step; with N ranks they are
ZeRO-1 sharded across the GPUs.  `--workload prfl_t2v_480` runs the 480p x 81f config (L=32760);
`--workload prfl_i2v_720` the I2V model (16.4B, 36 input channels, 257 CLIP tokens of image
cross-attention, `configs/train_prfl_i2v_720.yaml`) at 720p x 81f; `--fp8` its fp8 path (C5: the
large forward projections as per-row e4m3 on the block-scaled fp8 MFMA, backward bf16).

Multi-GPU: pure data parallel (weak scaling, one sample per rank), RCCL all-reduce of the
generator gradients overlapped with the backward (prfl_amd/dist.py).  `value` = PRFL sample-
iterations completed by all ranks per second.

Wall-clock budget (`--budget-s`, default 540 s from interpreter start, inside the driver's 600 s):
a 720p iteration takes minutes, so `--warmup W` runs min(W, 1) warm-up iterations at
mid_timestep = 1 (every kernel, both optimizer updates and the memory high-water mark of the
full iteration, minus 18 no-grad rollout forwards), then up to `--steps K` full iterations are
timed — as many as the budget holds, at least one; `steps` reports how many ran.  Every timed
iteration is an optimizer-step iteration ((step + 1) % 5 == 0: SFT and reward AdamW updates
inside it, the slowest of the five), so the window always ends on an optimizer step.
"""
import time

T_START = time.time()   # the driver's clock starts with the interpreter; the budget counts from here

import argparse  # noqa: E402
import json  # noqa: E402
import math  # noqa: E402
import os  # noqa: E402
import sys  # noqa: E402

ROOT = os.path.dirname(os.path.abspath(__file__))
# (no allocator options: this PyTorch-ROCm build ignores expandable_segments - "not supported on
# this platform" - so the plain caching allocator serves the 720p step; its fragmentation is the
# gap between peak_alloc_gb_rank0 and peak_hbm_gb)
sys.path[:0] = [ROOT, os.path.join(ROOT, "hy-video-prfl_amd")]

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

C, F, NH, NL, TXT = 5120, 13824, 40, 40, 512
PEAK_BF16_TFLOPS = 2500.0      # MI355X dense bf16 MFMA (MI355X_MICROARCH.md)
PEAK_HBM_GBS = 8000.0


CLIP_TOK = 257


def block_fwd_flops(L, Lctx=TXT, i2v=False):
    """8LC^2 + 4L^2C + 4LC^2 + 4 Lctx C^2 + 4 L Lctx C + 4LCF; I2V adds the image
    cross-attention 4*257*C^2 + 4*L*257*C (k_img/v_img projections + attention)."""
    f = 8 * L * C * C + 4 * L * L * C + 4 * L * C * C + 4 * Lctx * C * C + 4 * L * Lctx * C + 4 * L * C * F
    if i2v:
        f += 4 * CLIP_TOK * C * C + 4 * L * CLIP_TOK * C
    return f


def iteration_flops(L, mid, i2v=False):
    """Algorithmic FLOPs of one PRFL iteration (no recompute): SFT 3G + reward (mid+1)G+2G+3R."""
    G = NL * block_fwd_flops(L, i2v=i2v)
    R = 8 * block_fwd_flops(L, i2v=i2v)
    return 3 * G + (mid + 1) * G + 2 * G + 3 * R


def setup():
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    torch.cuda.set_device(local)
    if world > 1:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    return world, rank, local


def build_models(dev, seed, model_type="t2v"):
    from prfl_amd.model import WanModel
    from prfl_amd.network import MLP, QueryAttention
    torch.manual_seed(seed)
    in_dim = 16 if model_type == "t2v" else 36   # I2V: 16 latent + 4 mask + 16 condition channels
    with torch.device(dev):
        gen = WanModel(model_type=model_type, dim=C, ffn_dim=F, freq_dim=256, text_dim=4096,
                       out_dim=16, num_heads=NH, num_layers=NL, in_dim=in_dim)
        torch.nn.init.normal_(gen.head.head.weight, std=0.02)   # random-init trap
        lrm = WanModel(model_type=model_type, dim=C, ffn_dim=F, freq_dim=256, text_dim=4096,
                       out_dim=16, num_heads=NH, num_layers=8, in_dim=in_dim)   # == blocks[0:8]
        del lrm.head
        lrm.head = None
        qa = QueryAttention(C, 1, 8, 0., return_type="query")
        mlp = MLP(C)
    for p in list(lrm.parameters()) + list(qa.parameters()) + list(mlp.parameters()):
        p.requires_grad_(False)
    return gen, lrm, qa, mlp


def cpu_baseline(L_sample=4096):
    """The oracle (fp32 CPU restatement) timed on this host: one real-width 14B block forward +
    backward at L_sample tokens; extrapolated by algorithmic FLOPs to one PRFL iteration."""
    sys.path.insert(0, os.path.join(ROOT, "tests", "golden"))
    from oracle import wan_oracle as O
    from shapes import block_shapes
    threads = min(16, os.cpu_count() or 1)
    torch.set_num_threads(threads)
    g = torch.Generator().manual_seed(0)
    P = {n: (torch.randn(s, generator=g) / math.sqrt(s[-1] if len(s) > 1 else 1) * (0.02 if len(s) == 1 else 1))
         .requires_grad_(True) for n, s in block_shapes("b.", C, F)}
    for n in P:
        if "norm" in n and n.endswith("weight"):
            P[n] = (1 + P[n].detach()).requires_grad_(True)
    f, h, w = 1, 64, L_sample // 64
    x = torch.randn(1, L_sample, C, generator=g).requires_grad_(True)
    e = torch.randn(1, 6, C, generator=g) * 0.1
    ctx = torch.randn(1, TXT, C, generator=g).to(torch.bfloat16).float()
    t0 = time.time()
    out = O.block_forward(P, "b.", x, e, torch.tensor([[f, h, w]]), O.rope_freqs(128), ctx, NH,
                          seq_len=L_sample)
    out.sum().backward()
    dt = time.time() - t0
    flops = 3 * block_fwd_flops(L_sample)
    return dt, flops, threads


def pmc_traffic(L):
    """HBM-side bytes per launch of the roofline kernel from the committed rocprofv3 --pmc passes
    (FETCH_SIZE x2 gfx950 correction + WRITE_SIZE; profiles/r02_pmc_attn_fwd720_split.txt, measured on
    the isolated 720p self-attention forward, the kernel the bench runs).  PMC counters cannot be
    read inside this process."""
    path = os.path.join(ROOT, "profiles", "r02_pmc_attn_fwd720_split.txt")
    if L != 73920 or not os.path.exists(path):
        return None, None
    for line in open(path):
        if line.startswith("HBM-side traffic per launch ="):
            return float(line.rsplit("=", 1)[1].split()[0]), os.path.relpath(path, ROOT)
    return None, None


def big_fits(args):
    """The attention stash is sized for the 14B generator at 720p x 81f on a 288 GB GPU, where the
    AdamW moments live on the host; at 480p they stay in HBM (peak 254.5 GB allocated) and the
    stash would not fit beside them."""
    return args.workload.startswith("prfl") and args.workload.endswith("720")


def draw_mid(rank, world, dev):
    """mid_timestep = randint(0, 38) drawn on rank 0 and broadcast (train_prfl.py:640-651)."""
    t = torch.randint(0, 39, (1,), device=dev) if rank == 0 else torch.zeros(1, dtype=torch.long, device=dev)
    if world > 1:
        dist.broadcast(t, 0)
    return int(t.item())


def heartbeat(period=60.0):
    """A progress line on stderr every `period` s (a 720p iteration runs for minutes)."""
    import threading
    t0 = time.time()

    def run():
        while True:
            time.sleep(period)
            print(f"[bench] alive {time.time() - t0:.0f} s", file=sys.stderr, flush=True)
    threading.Thread(target=run, daemon=True).start()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=1)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--workload", default="prfl_t2v_720",
                    choices=["prfl_t2v_480", "prfl_t2v_720", "prfl_i2v_720", "pavrm_t2v_480"])
    ap.add_argument("--mid", type=int, default=19, help="mid_timestep (E[randint(0,38)] = 19)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--fp8", action="store_true",
                    help="config C5's fp8 path: e4m3 forward projections on the block-scaled MFMA")
    ap.add_argument("--budget-s", type=float, default=540.0,
                    help="wall-clock budget from interpreter start (warm-up + timed + CPU baseline)")
    ap.add_argument("--warmup-mid", type=int, default=1,
                    help="mid_timestep of the warm-up iterations (full iterations: use --mid)")
    ap.add_argument("--random-mid", action="store_true",
                    help="draw mid_timestep = randint(0, 38) per iteration on rank 0 and broadcast "
                         "it, as train_prfl.py:640-651 does (default: fixed --mid)")
    args = ap.parse_args()
    world, rank, local = setup()
    dev = torch.device("cuda", local)
    if rank == 0:
        heartbeat()
    from prfl_amd import ops
    from prfl_amd.train import PAVRMTrainer, PRFLTrainer

    # latents (gen_wanx_latent.py:117-149): 480p x 81f [16,21,60,104]; 720p x 81f [16,21,88,160]
    Fl, Hl, Wl = (21, 88, 160) if args.workload.endswith("720") else (21, 60, 104)
    L = Fl * (Hl // 2) * (Wl // 2)
    i2v = "_i2v_" in args.workload
    gen, lrm, qa, mlp = build_models(dev, 110221, "i2v" if i2v else "t2v")
    if args.fp8:
        gen.set_fp8_gemm(True)
        lrm.set_fp8_gemm(True)
    # keep the self-attention outputs of the first blocks of every graph-recording model forward
    # for the backward (bit-identical to recomputing them); the budget is per training step and
    # shared by the generator's and the reward model's forwards (block.py).  T2V: 38 GB keeps
    # all 40 generator blocks + the 8 reward-model blocks at 720p (0.77 GB each), so no
    # grad-enabled L x L attention forward is recomputed (round 1: 32 GB per model forward, peak
    # 247 GB allocated / 290 GB reserved of the 309 GB card); 20 GB when RCCL's buffers sit
    # beside it (N > 1).  I2V (16.4 B parameters): 22 GB at N = 1, none at N > 1.
    from prfl_amd import block as _blk
    default_gb = "0"
    if big_fits(args):
        default_gb = ("22" if world == 1 else "0") if i2v else ("38" if world == 1 else "20")
    stash_gb = float(os.environ.get("PRFL_ATTN_STASH_GB", default_gb))
    _blk.set_attn_stash_budget(int(stash_gb * 1e9))
    g = torch.Generator(device=dev).manual_seed(110221 + rank)   # distinct data per rank
    latents = torch.randn(1, 16, Fl, Hl, Wl, generator=g, device=dev).to(torch.bfloat16)
    text = (0.08 * torch.randn(1, 126, 4096, generator=g, device=dev)).to(torch.bfloat16)
    clip, cond = None, None
    if i2v:
        # image condition as before_train_step builds it (train_prfl.py:531-549): CLIP tokens
        # [1,257,1280]; condition latent [1,16,F,H,W] behind 4 mask channels (first frame = 1)
        clip = torch.randn(1, CLIP_TOK, 1280, generator=g, device=dev).to(torch.bfloat16)
        cond = torch.randn(1, 16, Fl, Hl, Wl, generator=g, device=dev).to(torch.bfloat16)
        mask = torch.zeros(1, 4, Fl, Hl, Wl, device=dev, dtype=torch.bfloat16)
        mask[:, :, :1] = 1
        cond = torch.cat([mask, cond], dim=1)
    if args.workload.startswith("prfl"):
        # 720p memory plan: the AdamW moments live in pinned host memory and stream
        # through HBM during the step; with DP ranks they are also ZeRO-1 sharded (each rank
        # holds and streams 1/N of them, then broadcasts the tensors it updated)
        big = args.workload.endswith("720")
        tr = PRFLTrainer(gen, lrm, qa, mlp, grad_accum=5.0,
                         optimizer_state_on_host=big or os.environ.get("PRFL_OPT_HOST") == "1",
                         optimizer_shard=big and world > 1,
                         optimizer_overlap=os.environ.get("PRFL_OPT_OVERLAP", "1") == "1")

        mids = []

        def one(step, mid=None):
            if mid is None:
                mid = draw_mid(rank, world, dev) if args.random_mid else args.mid
                mids.append(mid)
            a = tr.sft_step(step, latents, text, L, image_embeds=clip, cond=cond, generator=g)
            b = tr.reward_step(step, latents, text, L, image_embeds=clip, cond=cond,
                               mid_timestep=mid, generator=g)
            return a, b

        def flops_of(mid):
            return iteration_flops(L, mid, i2v)
    else:
        del gen
        for blk in lrm.blocks:
            blk.requires_grad_(True)
        tr = PAVRMTrainer(lrm, qa, mlp)
        label = torch.ones(1, device=dev)

        mids = []

        def one(step, mid=None):
            return tr.step(latents, text, L, label, generator=g), None

        def flops_of(mid):
            return 3 * 8 * block_fwd_flops(L)

    prfl = args.workload.startswith("prfl")
    # warm-up: min(W, 1) iterations at a short rollout (see the module docstring); step index 4
    # is an optimizer-step iteration, so both AdamW updates are warmed as well
    n_warm = min(args.warmup, 1)
    t_warm = None
    for _ in range(n_warm):
        t_w = time.time()
        one(4, mid=args.warmup_mid if prfl else None)
        torch.cuda.synchronize()
        t_warm = time.time() - t_w
        if rank == 0:
            print(f"[bench] warm-up iteration (mid_timestep {args.warmup_mid}): {t_warm:.1f} s",
                  file=sys.stderr, flush=True)
    # the CPU baseline runs after the timed window: keep room for it in the budget
    cpu_reserve = 0.0 if (args.no_cpu_baseline or rank != 0 or world > 1) else 45.0
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.reset_peak_memory_stats()
    ops.prof_enable(True)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    t0 = time.time()
    steps, durs = 0, []
    for i in range(args.steps):
        last = one(9 + 5 * i)            # every timed iteration ends on an optimizer step
        torch.cuda.synchronize()
        steps += 1
        t_it = time.time() - t0 - sum(durs)
        durs.append(t_it)
        est = max(sum(durs) / steps, t_it)     # the next iteration must fit the budget
        left = args.budget_s - (time.time() - T_START) - cpu_reserve
        go = torch.tensor([1.0 if left > 1.1 * est else 0.0], device=dev)
        if world > 1:                      # every rank runs the same number of iterations
            dist.all_reduce(go, op=dist.ReduceOp.MIN)
        if go.item() == 0.0:
            break
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    dt = time.time() - t0
    flops_it = sum(flops_of(m) for m in mids) / len(mids) if mids else flops_of(args.mid)
    ops.prof_enable(False)
    prof = ops.prof_collect()
    peak_alloc = torch.cuda.max_memory_allocated() / 1e9
    peak_res = torch.cuda.max_memory_reserved() / 1e9
    tmax = torch.tensor([dt, peak_res], device=dev)
    if world > 1:
        dist.all_reduce(tmax, op=dist.ReduceOp.MAX)
    dt, peak_res = tmax.tolist()
    if rank != 0:
        dist.destroy_process_group()
        return
    # roofline kernel: the dominant single kernel (one symbol, one shape) in the timed region —
    # the L x L self-attention forward (`attn_fwd_kernel<false>`); the GEMM family is reported
    # per family in "kernels" (it spans ten template instantiations and many shapes)
    dom = "attn_fwd"
    d = prof[dom]
    achieved = d["work"] / (d["ms"] * 1e-3) / 1e12
    traffic, traffic_src = pmc_traffic(L)
    value = world * steps / dt
    res = {
        "metric": "PRFL train steps/sec (whole node) + peak HBM GB, 14B DiT",
        "value": round(value, 6), "unit": "PRFL iterations/s (all ranks)",
        "n_gpus": world, "steps": steps, "warmup": n_warm,
        "steps_requested": args.steps, "warmup_requested": args.warmup,
        "budget_s": args.budget_s, "wall_s_at_report": None,
        "ms_per_step": round(dt / steps * 1e3, 1), "higher_is_better": True, "scaling": "weak",
        "vs_baseline": None,
        "dtype": "fp8-e4m3 fwd GEMMs / bf16" if args.fp8 else "bf16", "data": "synthetic latents/text, random-init 14B weights",
        "config": {"workload": (("train_%s: SFT + reward step, mid_timestep=%s" %
                                 (args.workload, ("randint(0, 38) per iteration: %s" % mids) if args.random_mid
                                  else args.mid))
                                if prfl else "train_pavrm_t2v_480: 8-block trunk + head, BCE"),
                   "model": ("Wan2.1-I2V-14B (40 blocks, C=5120, image cross-attn)" if i2v
                             else "Wan2.1-T2V-14B (40 blocks, C=5120)"), "latent": [16, Fl, Hl, Wl],
                   "seq_len": L, "global_batch": world, "parallelism": f"dp{world}"},
        "peak_hbm_gb": round(peak_res, 1), "peak_alloc_gb_rank0": round(peak_alloc, 1),
        "stash_gb": stash_gb,
        "algorithmic_tflop_per_step": round(flops_it / 1e12, 1),
        "achieved_tflops_per_gpu": round(flops_it * steps / dt / 1e12, 1),
        "roofline": {"kernel": dom, "bound": "mfma", "achieved": round(achieved, 1),
                     "peak": PEAK_BF16_TFLOPS, "unit": "TFLOP/s",
                     "frac": round(achieved / PEAK_BF16_TFLOPS, 4),
                     "launches": d["count"], "avg_launch_ms": round(d["ms"] / d["count"], 3),
                     "work_per_launch_tflop": round(d["work"] / d["count"] / 1e12, 3),
                     "traffic": traffic, "traffic_unit": "GB HBM per launch (PMC)",
                     "traffic_source": traffic_src,
                     "algorithmic_gb_per_launch": round(4 * L * C * 2 / 1e9, 3)},
        "kernels": {k: {"count": v["count"], "ms": round(v["ms"], 1),
                        "rate": round(v["work"] / (v["ms"] * 1e-3) / (1e9 if k in ("ln", "rms", "eltwise", "adamw") else 1e12), 1)}
                    for k, v in prof.items() if v["count"]},
    }
    if not args.no_cpu_baseline and world == 1:
        cdt, cfl, thr = cpu_baseline()
        cpu_rate = cfl / cdt
        res["cpu_baseline"] = {"value": flops_it and cpu_rate / flops_it, "unit": "PRFL iterations/s",
                               "cores": thr, "kind": "port",
                               "sample": f"oracle fp32 14B block fwd+bwd at L=4096 on host: {cdt:.1f} s "
                                         f"({cpu_rate/1e12:.2f} TFLOP/s), extrapolated by FLOPs to one "
                                         f"iteration ({flops_it/1e15:.1f} PFLOP)"}
    res["wall_s_at_report"] = round(time.time() - T_START, 1)
    print(json.dumps(res), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
