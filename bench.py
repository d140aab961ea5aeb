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
PEAK_FP8_TFLOPS = 5000.0       # dense block-scaled e4m3 MFMA (2x bf16 per clock)
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


def setup(backend="nccl"):
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1 and backend == "gloo":
        local = 0                                  # CPU-collective rehearsal: ranks share GPU 0
    torch.cuda.set_device(local)
    if world > 1:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:
            dist.init_process_group(backend)
    return world, rank, local


TOY_DIMS = dict(dim=256, ffn_dim=512, num_heads=2, num_layers=2, lrm_layers=2)


def build_models(dev, seed, model_type="t2v", toy=False):
    from prfl_amd.model import WanModel
    from prfl_amd.network import MLP, QueryAttention
    torch.manual_seed(seed)
    in_dim = 16 if model_type == "t2v" else 36   # I2V: 16 latent + 4 mask + 16 condition channels
    d = TOY_DIMS if toy else dict(dim=C, ffn_dim=F, num_heads=NH, num_layers=NL, lrm_layers=8)
    with torch.device(dev):
        gen = WanModel(model_type=model_type, dim=d["dim"], ffn_dim=d["ffn_dim"], freq_dim=256,
                       text_dim=4096, out_dim=16, num_heads=d["num_heads"],
                       num_layers=d["num_layers"], in_dim=in_dim)
        torch.nn.init.normal_(gen.head.head.weight, std=0.02)   # random-init trap
        lrm = WanModel(model_type=model_type, dim=d["dim"], ffn_dim=d["ffn_dim"], freq_dim=256,
                       text_dim=4096, out_dim=16, num_heads=d["num_heads"],
                       num_layers=d["lrm_layers"], in_dim=in_dim)   # == blocks[0:8]
        del lrm.head
        lrm.head = None
        qa = QueryAttention(d["dim"], 1, 8, 0., return_type="query")
        mlp = MLP(d["dim"])
    for p in list(lrm.parameters()) + list(qa.parameters()) + list(mlp.parameters()):
        p.requires_grad_(False)
    return gen, lrm, qa, mlp


C1_GRID = (13, 30, 52)          # 480p x 49f latent [16, 13, 60, 104] (gen_wanx_latent.py:117-149)
C1_L = C1_GRID[0] * C1_GRID[1] * C1_GRID[2]     # 20 280 tokens


def cpu_model():
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    import platform
    return platform.processor() or "unknown"


def c1_inputs(dev, seed=0):
    """Config C1 (`pre_480`): one 14B block's weights (N(0, 1/fan_in) matrices, norm
    weights 1 + 0.02 N, small biases), x [1, 20 280, 5120] ~ N(0,1) fp32, e0 [1, 6, 5120] ~
    0.1 N(0,1), 512 text tokens [1, 512, 5120] ~ N(0,1) (bf16), grid 13 x 30 x 52."""
    sys.path.insert(0, os.path.join(ROOT, "tests", "golden"))
    from shapes import block_shapes
    g = torch.Generator(device=dev).manual_seed(seed)
    P = {}
    for n, s in block_shapes("b.", C, F):
        t = torch.randn(s, generator=g, device=dev)
        if len(s) > 1:
            t /= math.sqrt(s[-1])
        elif "norm" in n and n.endswith("weight"):
            t = 1 + 0.02 * t
        else:
            t *= 0.02
        P[n] = t
    x = torch.randn(1, C1_L, C, generator=g, device=dev)
    e0 = torch.randn(1, 6, C, generator=g, device=dev) * 0.1
    ctx = torch.randn(1, TXT, C, generator=g, device=dev).to(torch.bfloat16)
    return P, x, e0, ctx


def cpu_baseline():
    """The oracle (fp32 CPU restatement of the reference block with its bf16 cast points, test
    infrastructure) timed on this host on config C1 itself: ONE 14B WanAttentionBlock forward at
    480p x 49f (L = 20 280, grid 13 x 30 x 52), no grad, min(16, nproc) threads."""
    from oracle import wan_oracle as O
    threads = min(16, os.cpu_count() or 1)
    torch.set_num_threads(threads)
    P, x, e0, ctx = c1_inputs("cpu")
    t0 = time.time()
    with torch.no_grad():
        O.block_forward(P, "b.", x, e0, torch.tensor([C1_GRID]), O.rope_freqs(128), ctx.float(), NH,
                        seq_len=C1_L)
    dt = time.time() - t0
    return dict(seconds=dt, flops=block_fwd_flops(C1_L), threads=threads, model=cpu_model(),
                nproc=os.cpu_count())


CPU_SCALING_PER_DOUBLING = 1.33    # profiles/r05_cpu_thread_scaling.txt: 47.9 s -> 35.9 s


def cores_per_socket():
    """Physical cores of one socket ('cpu cores' in /proc/cpuinfo), or None."""
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("cpu cores"):
                return int(line.split(":")[1])
    except (OSError, ValueError):
        pass
    return None


PMC_TRAFFIC_FILE = os.path.join(ROOT, "profiles", "r06_pmc_attn720.txt")


def pmc_traffic(L):
    """HBM-side bytes per launch of the roofline kernel from committed rocprofv3 --pmc passes
    (FETCH_SIZE x2 gfx950 correction + WRITE_SIZE) over an ISOLATED launch of the same kernel at
    the bench's 720p shape (PMC counters cannot be read inside this process); the scope is
    stated in the bench line."""
    path = PMC_TRAFFIC_FILE
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


def host_moments(big):
    """AdamW moments on the host: all of them at 720p (the memory plan); at 480p the
    last fifth of the parameters in update order (the last 8 generator blocks: 23 GB of HBM back,
    their ~0.8 s of PCIe per update hidden under the first 32 blocks' forwards).  PRFL_OPT_HOST
    overrides: 1 = all, 0 = none, a fraction in (0, 1) = that tail."""
    env = os.environ.get("PRFL_OPT_HOST")
    if env is not None:
        f = float(env)
        return True if f >= 1.0 else (False if f <= 0.0 else f)
    return True if big else 0.2


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


def run_c1(args, dev):
    """Config C1 (`pre_480`) on the GPU: the fused 14B block forward (`prfl::wan_block`, no grad)
    over the C1 input; a step = one block forward.  Returns (steps, seconds)."""
    from prfl_amd import block as B
    from prfl_amd import ops
    from prfl_amd.model import rope_params
    P, x, e0, ctx = c1_inputs(dev)
    Pd = {n: P["b." + n] for n in B.param_names(False)}
    em = P["b.modulation"] + e0
    d = C // NH                                   # WanModel.freqs (model.py:518-526)
    freqs = torch.cat([rope_params(1024, d - 4 * (d // 6)), rope_params(1024, 2 * (d // 6)),
                       rope_params(1024, 2 * (d // 6))], dim=1)
    meta = B.Meta(NH, [C1_GRID], [C1_L], ops.rope_table(freqs, dev), False)
    with torch.no_grad():
        for _ in range(max(args.warmup, 1)):
            B.block_apply(Pd, x, em, ctx, meta)
        torch.cuda.synchronize()
        ops.prof_enable(True)
        t0 = time.time()
        for _ in range(args.steps):
            B.block_apply(Pd, x, em, ctx, meta)
        torch.cuda.synchronize()
    return args.steps, time.time() - t0


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=1)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--workload", default="prfl_t2v_720",
                    choices=["prfl_t2v_480", "prfl_t2v_720", "prfl_i2v_720", "pavrm_t2v_480",
                             "pre_480"])
    ap.add_argument("--mid", type=int, default=19, help="mid_timestep (E[randint(0,38)] = 19)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--fp8", action="store_true",
                    help="config C5's fp8 path: e4m3 forward projections and the e4m3 self-attention "
                         "forward on the block-scaled MFMA")
    ap.add_argument("--fp8-gemm-only", action="store_true",
                    help="with --fp8: keep the self-attention forward bf16 (the round-2 fp8 path)")
    ap.add_argument("--budget-s", type=float, default=540.0,
                    help="wall-clock budget from interpreter start (warm-up + timed + CPU baseline)")
    ap.add_argument("--warmup-mid", type=int, default=1,
                    help="mid_timestep of the warm-up iterations (full iterations: use --mid)")
    ap.add_argument("--random-mid", action="store_true",
                    help="draw mid_timestep = randint(0, 38) per iteration on rank 0 and broadcast "
                         "it, as train_prfl.py:640-651 does (default: fixed --mid)")
    ap.add_argument("--toy", action="store_true",
                    help="control-path rehearsal: a 2-block 256-wide model on a [16,3,10,14] latent "
                         "with the 720p memory plan's code paths (host moments, ZeRO-1 at N > 1, "
                         "attention stash); not a measurement")
    ap.add_argument("--dist-backend", default="nccl", choices=["nccl", "gloo"],
                    help="gloo: N > 1 ranks sharing GPU 0 with CPU collectives (rehearsal only)")
    args = ap.parse_args()
    world, rank, local = setup(args.dist_backend)
    dev = torch.device("cuda", local)
    if rank == 0:
        heartbeat()
    from prfl_amd import ops
    from prfl_amd.train import PAVRMTrainer, PRFLTrainer

    c1 = args.workload == "pre_480"
    tail_ms = []
    if c1:
        if world > 1:
            raise SystemExit("pre_480 (C1) is a single-block, single-GPU configuration")
        steps, dt = run_c1(args, dev)
        L, i2v, prfl, n_warm, stash_gb, mids = C1_L, False, False, max(args.warmup, 1), 0.0, []
        Fl, Hl, Wl = 13, 60, 104

        def flops_of(mid):
            return block_fwd_flops(C1_L)
    else:
        # latents (gen_wanx_latent.py:117-149): 480p x 81f [16,21,60,104]; 720p x 81f [16,21,88,160]
        Fl, Hl, Wl = (21, 88, 160) if args.workload.endswith("720") else (21, 60, 104)
        if args.toy:
            Fl, Hl, Wl = 3, 10, 14
        L = Fl * (Hl // 2) * (Wl // 2)
        i2v = "_i2v_" in args.workload
        gen, lrm, qa, mlp = build_models(dev, 110221, "i2v" if i2v else "t2v", toy=args.toy)
        if args.fp8:
            gen.set_fp8_gemm(True, attn=not args.fp8_gemm_only)
            lrm.set_fp8_gemm(True, attn=not args.fp8_gemm_only)
        # keep the self-attention outputs of graph-recording block forwards for the backward
        # (bit-identical to recomputing them; block.py): the budget bounds the bytes kept at any
        # time.  T2V: 38 GB keeps all 40 generator blocks + the 8 reward-model blocks at 720p
        # (0.77 GB each), so no grad-enabled L x L attention forward is recomputed; 20 GB when
        # RCCL's buffers sit beside it (N > 1).  I2V (16.4 B parameters, 66 GB of fp32 gradients
        # resident through the iteration): 10 GB at N = 1, none at N > 1.
        from prfl_amd import block as _blk
        default_gb = "0"
        if big_fits(args):
            default_gb = ("10" if world == 1 else "0") if i2v else ("38" if world == 1 else "20")
        if args.toy:
            default_gb = "0.001"
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
        prfl = args.workload.startswith("prfl")
        mids = []
        if prfl:
            # 720p memory plan: the AdamW moments live in pinned host memory and
            # stream through HBM during the step; with DP ranks they are also ZeRO-1 sharded
            # (each rank holds and streams 1/N of every parameter group's elements, then one
            # all-gather per group rebuilds the parameters everywhere)
            big = args.workload.endswith("720") or args.toy
            tr = PRFLTrainer(gen, lrm, qa, mlp, grad_accum=5.0,
                             feature_layer=(TOY_DIMS["lrm_layers"],) if args.toy else (8,),
                             optimizer_state_on_host=host_moments(big),
                             optimizer_shard=big and world > 1,
                             optimizer_overlap=os.environ.get("PRFL_OPT_OVERLAP", "1") == "1")
            if world > 1:
                tr.reducer.time_tail = True

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
            tr = PAVRMTrainer(lrm, qa, mlp,
                              feature_layer=(TOY_DIMS["lrm_layers"],) if args.toy else (8,))
            label = torch.ones(1, device=dev)

            def one(step, mid=None):
                return tr.step(latents, text, L, label, generator=g), None

            def flops_of(mid):
                return 3 * 8 * block_fwd_flops(L)

        # warm-up: min(W, 1) iterations at a short rollout (see the module docstring); step
        # index 4 is an optimizer-step iteration, so both AdamW updates are warmed as well
        n_warm = min(args.warmup, 1)
        for _ in range(n_warm):
            t_w = time.time()
            one(4, mid=args.warmup_mid if prfl else None)
            torch.cuda.synchronize()
            if rank == 0:
                print(f"[bench] warm-up iteration (mid_timestep {args.warmup_mid}): "
                      f"{time.time() - t_w:.1f} s", file=sys.stderr, flush=True)
        # the CPU baseline runs after the timed window: keep room for it in the budget
        cpu_reserve = 0.0 if (args.no_cpu_baseline or rank != 0 or world > 1) else 75.0
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()
        torch.cuda.reset_peak_memory_stats()
        ops.prof_enable(True)
        ops.prof_clock()                         # drop clock slots of anything before the window
        if prfl:
            tr.reducer.collect_tail_ms()     # drop the warm-up's records
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()
        t0 = time.time()
        steps, durs = 0, []
        for i in range(args.steps):
            one(9 + 5 * i)                   # every timed iteration ends on an optimizer step
            # main stream only: the reward step's optimizer update (moments streamed over PCIe
            # on the optimizer's side streams) runs on under the next iteration's first forward,
            # each block waiting for its own parameters (optim.py attach), as in a training loop;
            # the synchronize after the loop puts the last update inside the timed window
            torch.cuda.current_stream().synchronize()
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
        if prfl:
            tail_ms = tr.reducer.collect_tail_ms()
    flops_it = sum(flops_of(m) for m in mids) / len(mids) if mids else flops_of(args.mid)
    clock = ops.prof_clock()
    ops.prof_enable(False)
    prof = ops.prof_collect()
    peak_alloc = torch.cuda.max_memory_allocated() / 1e9
    peak_res = torch.cuda.max_memory_reserved() / 1e9
    tmax = torch.tensor([dt, peak_res], device=dev)
    if world > 1:
        dist.all_reduce(tmax, op=dist.ReduceOp.MAX)
        # every rank must have run the same number of timed iterations (the MIN vote above)
        st = torch.tensor([float(steps)], device=dev)
        lo, hi = st.clone(), st.clone()
        dist.all_reduce(lo, op=dist.ReduceOp.MIN)
        dist.all_reduce(hi, op=dist.ReduceOp.MAX)
        assert lo.item() == hi.item() == steps, (rank, lo.item(), hi.item(), steps)
    dt, peak_res = tmax.tolist()
    if rank != 0:
        dist.destroy_process_group()
        return
    # roofline kernel: the dominant single kernel (one symbol, one shape) in the timed region —
    # the L x L self-attention forward (`attn_fwd_kernel<false>`); the GEMM family is reported
    # per family in "kernels" (it spans ten template instantiations and many shapes)
    dom = "attn_fwd_fp8" if args.fp8 and not args.fp8_gemm_only and not c1 else "attn_fwd"
    peak = PEAK_FP8_TFLOPS if dom == "attn_fwd_fp8" else PEAK_BF16_TFLOPS
    d = prof[dom]
    achieved = d["work"] / (d["ms"] * 1e-3) / 1e12 if d["count"] else 0.0
    traffic, traffic_src = pmc_traffic(L) if dom == "attn_fwd" else (None, None)
    value = world * steps / dt
    if c1:
        metric, unit = "C1 pre_480: 14B block forwards/s, 480p x 49f", "block forwards/s"
        workload = "pre_480: one 14B WanAttentionBlock forward, 480p x 49f (L=20280), no grad"
        model = "Wan2.1-T2V-14B block (C=5120, 40 heads, F=13824)"
    else:
        metric, unit = "PRFL train steps/sec (whole node) + peak HBM GB, 14B DiT", \
            "PRFL iterations/s (all ranks)"
        workload = (("train_%s: SFT + reward step, mid_timestep=%s" %
                     (args.workload, ("randint(0, 38) per iteration: %s" % mids)
                      if args.random_mid else args.mid))
                    if prfl else "train_pavrm_t2v_480: 8-block trunk + head, BCE")
        model = ("Wan2.1-I2V-14B (40 blocks, C=5120, image cross-attn)" if i2v
                 else "Wan2.1-T2V-14B (40 blocks, C=5120)")
        if args.toy:
            workload = "TOY control-path rehearsal (not a measurement): " + workload
            model = "toy WanModel %s" % TOY_DIMS
    res = {
        "metric": metric, "value": round(value, 6), "unit": unit,
        "n_gpus": world, "steps": steps, "warmup": n_warm,
        "steps_requested": args.steps, "warmup_requested": args.warmup,
        "budget_s": args.budget_s, "wall_s_at_report": None,
        "ms_per_step": round(dt / steps * 1e3, 1), "higher_is_better": True, "scaling": "weak",
        "vs_baseline": None,
        "dtype": ("fp8-e4m3 fwd GEMMs / bf16" if args.fp8_gemm_only else
                  "fp8-e4m3 fwd GEMMs + int8 QK / e4m3 PV self-attention fwd / bf16")
        if args.fp8 else "bf16",
        "data": "synthetic latents/text, random-init 14B weights",
        "config": {"workload": workload, "model": model, "latent": [16, Fl, Hl, Wl],
                   "seq_len": L, "global_batch": world, "parallelism": f"dp{world}"},
        "peak_hbm_gb": round(peak_res, 1), "peak_alloc_gb_rank0": round(peak_alloc, 1),
        # fp32 gradients stay allocated across iterations (AdamW.step(zero_grad=True)): the peak
        # is that of every iteration, accumulating or not
        "grad_buffers": "persistent",
        "stash_gb": stash_gb,
        "algorithmic_tflop_per_step": round(flops_it / 1e12, 1),
        "achieved_tflops_per_gpu": round(flops_it * steps / dt / 1e12, 1),
        "gpu_clock_mhz": {"mean": round(clock["mean_mhz"], 1), "min": round(clock["min_mhz"], 1),
                          "max": round(clock["max_mhz"], 1), "launches": clock["launches"],
                          "source": "s_memtime / s_memrealtime (100 MHz) over the lifetime of "
                                    "workgroup 0 of every self-attention forward launch in the "
                                    "timed window; mean weighted by launch time"},
        "roofline": {"kernel": dom, "bound": "mfma", "achieved": round(achieved, 1),
                     "peak": peak, "unit": "TFLOP/s",
                     "frac": round(achieved / peak, 4),
                     "peak_at_measured_clock": round(peak * clock["mean_mhz"] / 2400.0, 1)
                     if clock["mean_mhz"] else None,
                     "launches": d["count"],
                     "avg_launch_ms": round(d["ms"] / d["count"], 3) if d["count"] else None,
                     "work_per_launch_tflop": round(d["work"] / d["count"] / 1e12, 3)
                     if d["count"] else None,
                     "traffic": traffic, "traffic_unit": "GB HBM per launch (PMC)",
                     "traffic_scope": "rocprofv3 --pmc FETCH_SIZE x2 + WRITE_SIZE of an ISOLATED "
                                      "launch of this kernel at the bench's 720p shape (counters "
                                      "cannot be read in-process)" if traffic else None,
                     "traffic_source": traffic_src,
                     "algorithmic_gb_per_launch": round(4 * L * C * 2 / 1e9, 3)},
        "kernels": {k: {"count": v["count"], "ms": round(v["ms"], 1),
                        "rate": round(v["work"] / (v["ms"] * 1e-3) /
                                      (1e9 if k in ("ln", "rms", "eltwise", "adamw") else 1e12), 1)}
                    for k, v in prof.items() if v["count"]},
    }
    bw = [prof[k] for k in ("attn_bwd_dkdv", "attn_bwd_dq") if k in prof and prof[k]["count"]]
    if len(bw) == 2:
        # the two backward kernels are credited 8 + 6 = 14 L^2 d H (each recomputes S and dP);
        # the algorithmic backward is 8 (dV, dP, dQ, dK), FA2's with one S recompute 10
        w14, t_bw = sum(v["work"] for v in bw), sum(v["ms"] for v in bw) * 1e-3
        res["attn_bwd"] = {"ms": round(t_bw * 1e3, 1),
                           "credited_tflops": round(w14 / t_bw / 1e12, 1),
                           "fa2_tflops": round(w14 * 10 / 14 / t_bw / 1e12, 1),
                           "algorithmic_tflops": round(w14 * 8 / 14 / t_bw / 1e12, 1),
                           "units": "credited 14, FA2 10, algorithmic 8 x L^2 x d x H per backward"}
    if tail_ms:
        res["grad_allreduce_exposed_tail_ms"] = {
            "per_backward": [round(t, 2) for t in tail_ms], "backend": args.dist_backend,
            "what": "HIP-event time from the end of each backward's kernels to the completion of "
                    "its last gradient all-reduce (GradReducer.end)"}
    if not args.no_cpu_baseline and world == 1 and not args.toy:
        cb = cpu_baseline()
        cpu_rate = cb["flops"] / cb["seconds"]
        res["cpu_baseline"] = {
            "value": 1.0 / cb["seconds"] if c1 else cpu_rate / flops_it,
            "unit": unit, "cores": cb["threads"], "kind": "port",
            "cpu_model": cb["model"], "nproc": cb["nproc"],
            "c1_block_fwd_s": round(cb["seconds"], 2),
            "sample": (f"config C1 measured: the oracle (fp32 CPU restatement, test infrastructure) "
                       f"runs one 14B block forward at 480p x 49f (L={C1_L}, grid 13x30x52) in "
                       f"{cb['seconds']:.1f} s on {cb['threads']} threads of '{cb['model']}' "
                       f"(nproc {cb['nproc']}): {cpu_rate / 1e12:.2f} TFLOP/s"
                       + ("" if c1 else f"; value = that rate extrapolated by algorithmic FLOPs "
                                        f"to one PRFL iteration ({flops_it / 1e15:.1f} PFLOP)"))}
        if not c1:
            res["cpu_baseline"]["derived"] = "extrapolated (no full iteration runs on the CPU)"
        cps = cores_per_socket()
        if cps and cps > cb["threads"]:
            # the GPU box grants this process a 16-CPU share of the host: the full socket is not
            # measurable here.  Upper bound = linear scaling from the measured threads to every
            # physical core of one socket (profiles/r05_cpu_thread_scaling.txt: 8 -> 16 threads)
            doublings = math.log2(cps / cb["threads"])
            res["cpu_baseline"]["full_socket_bound"] = {
                "value": res["cpu_baseline"]["value"] * cps / cb["threads"], "cores": cps,
                "kind": "bound", "what": f"linear-scaling upper bound: {cb['threads']} measured "
                                         f"threads -> {cps} physical cores of one socket",
                "estimate_at_measured_scaling": res["cpu_baseline"]["value"] * CPU_SCALING_PER_DOUBLING ** doublings,
                "scaling_source": f"{CPU_SCALING_PER_DOUBLING}x per thread doubling, 8 -> 16 threads on "
                                  f"this workload (profiles/r05_cpu_thread_scaling.txt)"}
    res["wall_s_at_report"] = round(time.time() - T_START, 1)
    print(json.dumps(res), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
