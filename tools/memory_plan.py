"""HBM budget of one rank of the 720p x 81f PRFL iteration, T2V (14.3 B) or I2V (16.4 B, config
C5), N = 1 or N > 1 data parallel.

    python tools/memory_plan.py [--model t2v|i2v] [--world N] [--stash-gb S] [--measured JSON]

Two estimates, both per GPU:
  * analytic: the resident tensors of DESIGN.md §2 plus the reward step's peak working set;
  * from measurement: an N = 1 bench's peak allocated / reserved (profiles/r0*_bench_*.json),
    minus the stash the N = 1 run kept, plus the N > 1 stash and RCCL's buffers.
What differs at N > 1 (bench.py): the attention-output stash budget (T2V 38 -> 20 GB, I2V 10 -> 0
GB per step), the RCCL communicator buffers (estimate below), and the ZeRO-1 optimizer (the AdamW
moments stay in pinned host memory; each rank streams 1/N of them through the same 3-slot HBM
ring).  Every rank otherwise holds the same replica as the single-GPU run.
"""
import argparse
import json
import os

GB = 1e9
CARD_GB = 288 * 1.073741824          # 288 GiB = 309.2 GB
C, F, NH, NL, L = 5120, 13824, 40, 40, 73920
BLOCK = {"t2v": 351.4e6,                                   # per WanAttentionBlock
         "i2v": 351.4e6 + 2 * (C * C + C) + C}              # + k_img, v_img, norm_k_img (model.py:229-271)
P_GEN = {"t2v": 14.288e9, "i2v": 16.4e9}                   # bench.py / SURVEY §8
P_HEAD = 3 * C * C + 4 * C + C * 1024 + 1024 * 512 + 512 + 1 + 1024 + 512   # QA + MLP
STASH_PER_BLOCK = (L * C * 2 + NH * L * 4) / GB      # kept self-attention output + LSE
STASH_DEFAULT = {("t2v", 1): 38.0, ("t2v", 8): 20.0, ("i2v", 1): 10.0, ("i2v", 8): 0.0}


def rccl_buffers_gb(world, channels=32, buff_bytes=4 << 20):
    """RCCL ring/tree buffers: per channel, a send and a receive buffer per peer connection of
    NCCL_BUFFSIZE (4 MiB default) for each of the 3 protocols (simple / LL / LL128 sized at most
    the simple size here): an upper bound of channels * 2 peers (ring) * 2 * 3 * 4 MiB, plus
    one proxy / fifo allowance."""
    if world <= 1:
        return 0.0
    return (channels * 2 * 2 * 3 * buff_bytes) / GB + 0.5


def default_stash(model, world):
    return STASH_DEFAULT[(model, 1 if world == 1 else 8)]


def analytic(world, stash_gb, model="t2v"):
    act = L * C * 4 / GB                                   # one fp32 residual [L, C]
    p_emb = P_GEN[model] - NL * BLOCK[model]                        # embeddings + head
    rows = {
        "fp32 generator params": P_GEN[model] * 4 / GB,
        "fp32 generator grads (persistent, accumulated in place)": P_GEN[model] * 4 / GB,
        # round 4: the frozen trunk's block Linear weights live in bf16 (train.store_frozen_bf16)
        "reward-model trunk (8 blocks, bf16 weights) + fp32 embeddings + head (frozen)":
            (8 * BLOCK[model] * 2 + (p_emb + P_HEAD) * 4) / GB,
        "40 generator + 8 LRM block-input checkpoints (fp32)": (NL + 8) * act,
        "attention-output stash (budget)": stash_gb,
        "one block's recompute + backward working set": 20.0,
        "bf16 weight copies of the block in flight": BLOCK[model] * 2 * 2 / GB,
        "AdamW moment ring (3 slots x largest tensor x m, v)": 3 * F * C * 4 * 2 / GB,
        "RCCL buffers": rccl_buffers_gb(world),
    }
    return rows


def from_measurement(world, stash_gb, path):
    """(allocated, reserved) GB per rank at N = `world` from an N = 1 bench line.  Lines from
    before round 4 (no "grad_buffers": "persistent") timed optimizer-boundary iterations whose
    gradients were freed after the SFT step's update, so their peak lacks the fp32 gradients an
    accumulating iteration (4 of every 5 at gradient_accumulation_steps 5) holds: added here."""
    d = json.load(open(path))
    alloc, res = d["peak_alloc_gb_rank0"], d["peak_hbm_gb"]
    kept = min(d.get("stash_gb", 38.0), (NL + 8) * STASH_PER_BLOCK)
    delta = min(stash_gb, (NL + 8) * STASH_PER_BLOCK) - kept + rccl_buffers_gb(world)
    if d.get("grad_buffers") != "persistent":
        model = "i2v" if "I2V" in d.get("config", {}).get("model", "") else "t2v"
        delta += P_GEN[model] * 4 / GB
    return alloc + delta, res + delta


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="t2v", choices=["t2v", "i2v"])
    ap.add_argument("--world", type=int, default=8)
    ap.add_argument("--stash-gb", type=float, default=None)
    ap.add_argument("--measured", default=None, help="an N = 1 bench JSON line")
    a = ap.parse_args()
    stash = a.stash_gb if a.stash_gb is not None else default_stash(a.model, a.world)
    rows = analytic(a.world, stash, a.model)
    for k, v in rows.items():
        print(f"{k:58s} {v:7.1f} GB")
    tot = sum(rows.values())
    print(f"{'analytic total (' + a.model + ')':58s} {tot:7.1f} GB of {CARD_GB:.1f} GB")
    if a.measured:
        al, rs = from_measurement(a.world, stash, a.measured)
        print(f"from {os.path.basename(a.measured)}: peak allocated {al:.1f} GB, reserved {rs:.1f} GB")


if __name__ == "__main__":
    main()
