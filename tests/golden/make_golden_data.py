"""Golden fixtures for the on-disk latent loader (build container only; needs /root/reference).

    python tests/golden/make_golden_data.py      # writes tests/golden/data.json

Runs the REFERENCE Image2VideoTrainDataset (image2video_dataset.py:19-262), BlockDistributedSampler
(data_utils.py:300-381) and crop_tensor (data_utils.py:49-78) over data_fixture.py's synthetic
dataset.  Stubs: decord / PIL / torchvision / imageio / easydict are imported by those modules
for video decoding and transforms the latent reader never calls."""
import importlib
import json
import os
import random
import sys
import tempfile
import types

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
import data_fixture as DF  # noqa: E402

REF = os.environ.get("PRFL_REFERENCE", "/root/reference")


def _stub(name, **attrs):
    m = types.ModuleType(name)
    m.__dict__.update(attrs)
    sys.modules[name] = m
    return m


def import_reference_data():
    sys.path.insert(0, REF)
    _stub("decord", VideoReader=object)
    _stub("PIL", Image=types.SimpleNamespace())
    _stub("PIL.Image")
    tv = _stub("torchvision", transforms=types.SimpleNamespace())
    _stub("torchvision.transforms")
    tv.io = None
    _stub("imageio")
    _stub("easydict", EasyDict=dict)
    for pkg in ("diffusers_lite", "diffusers_lite.utils", "diffusers_lite.datasets"):
        m = types.ModuleType(pkg)
        m.__path__ = [os.path.join(REF, *pkg.split("."))]
        sys.modules[pkg] = m
    du = importlib.import_module("diffusers_lite.utils.data_utils")
    ds = importlib.import_module("diffusers_lite.datasets.image2video_dataset")
    return du, ds


def digest(x):
    if torch.is_tensor(x):
        x = x.double()
        return {"shape": list(x.shape), "sum": x.sum().item(), "abs": x.abs().sum().item(),
                "first": x.flatten()[:4].tolist()}
    return x


def main():
    du, ds = import_reference_data()
    out = {"sampler": [], "crop": [], "refl": [], "lrm_ce": []}
    for (n, rep, rank, shuf, seed, epoch, start, bs) in DF.SAMPLER_CASES:
        s = du.BlockDistributedSampler(list(range(n)), num_replicas=rep, rank=rank, shuffle=shuf,
                                       seed=seed, drop_last=True, batch_size=bs,
                                       start_index=start)
        s.set_epoch(epoch)
        out["sampler"].append({"case": [n, rep, rank, shuf, seed, epoch, start, bs],
                               "len": len(s), "indices": list(iter(s))})
    for (shape, wr, hr, ty, tr, seed) in DF.CROP_CASES:
        random.seed(seed)
        x = torch.arange(int(np.prod(shape)), dtype=torch.float64).reshape(shape)
        a, b = du.crop_tensor(x, x + 1, wr, hr, ty, crop_time_ratio=tr)
        out["crop"].append({"case": [list(shape), wr, hr, ty, tr, seed], "shape": list(a.shape),
                            "first": a.flatten()[0].item(), "cond_first": b.flatten()[0].item()})
    with tempfile.TemporaryDirectory() as root:
        lst, null = DF.build(root)
        ds.NULL_DIR = null
        cwd = os.getcwd()
        for kind in ("refl", "lrm_ce"):
            d = ds.Image2VideoTrainDataset(task="i2v-14b-720p", dataset_type=kind,
                                           meta_file_list=[lst], uncond_prob=[0.3, 0.0])
            for idx in range(len(d)):
                random.seed(1000 + idx)
                np.random.seed(2000 + idx)
                item = d[idx]
                out[kind].append([digest(v) for v in item])
        os.chdir(cwd)
    path = os.path.join(HERE, "data.json")
    with open(path, "w") as f:
        json.dump(out, f, indent=0)
    print("wrote", path, os.path.getsize(path))


if __name__ == "__main__":
    main()
