"""On-disk latent loader (prfl_amd/data.py) vs the reference's own Image2VideoTrainDataset,
BlockDistributedSampler and crop_tensor (golden: tests/golden/data.json, made by
make_golden_data.py from the reference over data_fixture.py's synthetic dataset).

CPU: sampler indices, crop windows, dataset items (exact).  GPU: the HBM staging path
(LatentPrefetcher) — bit-identical to the reference's `.to(device, dtype=bf16)` + mask/crop."""
import json
import os
import random

import numpy as np
import pytest
import torch

import data_fixture as DF
from conftest import GOLDEN


@pytest.fixture(scope="module")
def gold():
    with open(os.path.join(GOLDEN, "data.json")) as f:
        return json.load(f)


def digest(x):
    if torch.is_tensor(x):
        x = x.double()
        return {"shape": list(x.shape), "sum": x.sum().item(), "abs": x.abs().sum().item(),
                "first": x.flatten()[:4].tolist()}
    return x


def test_block_sampler_matches_reference(gold):
    from prfl_amd.data import BlockDistributedSampler
    for g in gold["sampler"]:
        n, rep, rank, shuf, seed, epoch, start, bs = g["case"]
        s = BlockDistributedSampler(list(range(n)), num_replicas=rep, rank=rank, shuffle=shuf,
                                    seed=seed, drop_last=True, batch_size=bs, start_index=start)
        s.set_epoch(epoch)
        assert len(s) == g["len"] and list(iter(s)) == g["indices"], g["case"]


def test_block_sampler_partitions_ranks():
    from prfl_amd.data import BlockDistributedSampler
    seen = []
    for r in range(4):
        seen += list(BlockDistributedSampler(list(range(37)), 4, r, shuffle=True, seed=3))
    assert len(seen) == len(set(seen)) == 36


def test_crop_matches_reference(gold):
    from prfl_amd.data import crop_tensor
    for g in gold["crop"]:
        shape, wr, hr, ty, tr, seed = g["case"]
        random.seed(seed)
        x = torch.arange(int(np.prod(shape)), dtype=torch.float64).reshape(shape)
        a, b = crop_tensor(x, x + 1, wr, hr, ty, crop_time_ratio=tr)
        assert list(a.shape) == g["shape"] and a.flatten()[0].item() == g["first"], g["case"]
        assert b.flatten()[0].item() == g["cond_first"]


@pytest.mark.parametrize("kind", ["refl", "lrm_ce"])
def test_dataset_items_match_reference(gold, tmp_path, kind):
    from prfl_amd.data import Image2VideoTrainDataset
    lst, null = DF.build(str(tmp_path))
    d = Image2VideoTrainDataset(task="i2v-14b-720p", dataset_type=kind, meta_file_list=[lst],
                                uncond_prob=[0.3, 0.0], null_dir=null)
    assert len(d) == len(gold[kind])
    for idx in range(len(d)):
        random.seed(1000 + idx)
        np.random.seed(2000 + idx)
        got = [digest(v) for v in d[idx]]
        assert got == gold[kind][idx], (kind, idx)


@pytest.mark.gpu
def test_prefetcher_stages_batches_like_reference(tmp_path):
    """Device batches equal the CPU items cast by torch (`.to(bf16)`), I2V mask channels and
    image-token regrouping as train_prfl.py:527-549, and L = F*H*W/4."""
    from prfl_amd.data import BlockDistributedSampler, Image2VideoTrainDataset, LatentPrefetcher
    lst, null = DF.build(str(tmp_path))
    ds = Image2VideoTrainDataset(task="i2v-14b-720p", dataset_type="refl", meta_file_list=[lst],
                                 null_dir=null)
    # the clips the "refl" reader accepts (imgclip_path + a text pair or text_en_path)
    ds.meta_paths = [ds.meta_paths[i] for i in (0, 2, 3)]
    sampler = BlockDistributedSampler(list(range(3)), 1, 0, shuffle=True, seed=9)
    order = []
    for ep in range(3):                                    # the reader advances the epoch
        s2 = BlockDistributedSampler(list(range(3)), 1, 0, shuffle=True, seed=9)
        s2.set_epoch(ep)
        order += list(iter(s2))
    random.seed(5)
    pf = LatentPrefetcher(ds, sampler, batch_size=1, device="cuda", task="i2v-14b-720p")
    try:
        for k in range(7):                                 # crosses an epoch boundary
            b = next(pf)
            i = order[k]
            item = ds.get_batch_lrm_refl(i)
            ref_lat = item[0][None].to(torch.bfloat16)
            assert b.latents.dtype == torch.bfloat16 and b.latents.is_cuda
            assert torch.equal(b.latents.cpu(), ref_lat), k
            cond = item[4][None].to(torch.bfloat16)
            mask = torch.zeros((1, 4) + cond.shape[2:], dtype=torch.bfloat16)
            mask[:, :, :1] = 1
            assert torch.equal(b.latents_condition.cpu(), torch.cat([mask, cond], 1))
            assert tuple(b.image_embeds.shape) == (1, 257, 1280)
            assert torch.equal(b.image_embeds.cpu(), item[3][None].to(torch.bfloat16))
            assert b.max_sequence_length == 3 * 8 * 12 // 4
            assert b.uncond_text_states.shape[-1] == 4096
    finally:
        pf.close()
