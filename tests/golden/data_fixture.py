"""Deterministic on-disk latent dataset in the reference's format (gen_wanx_latent.py:288-325):
meta JSON per clip + fp32 .npy files + a meta list, and a null_dir with wanx/{uncond,null}.npy.
Written identically by make_golden_data.py (which runs the reference dataset over it) and by
tests/test_data.py (which runs ours), so the golden holds only what the reference returned."""
import json
import os

import numpy as np

SEED = 20260130
LAT = (1, 16, 3, 8, 12)          # [1, C, F, H, W]

# (key layout, text mode, label values) per clip — covers every key fallback of the reader
CLIPS = [
    dict(lat="vae_latent_path", cond="f1_black_path", text="short_long", emb="imgclip_path",
         labels=dict(text_alignment="good", blur_quality="poor", model="wan")),
    dict(lat="video_vae_latent_path", cond="latents_condition_path", text="short_long",
         emb="image_embeds", labels=dict(physics_quality=None, human_quality="good")),
    dict(lat="latents_path", cond="f1_black_path", text="en", emb="imgclip_path", labels={}),
    dict(lat="vae_latent_path", cond="f1_black_path", text="short_long", emb="imgclip_path",
         labels=dict(text_alignment=3, blur_quality="good")),
    dict(lat="vae_latent_path", cond="f1_black_path", text="save_short", emb="imgclip_path",
         labels=dict(model="x")),
    dict(lat="vae_latent_path", cond="f1_black_path", text="short_long", emb="imgclip_path",
         labels={}, broken=True),   # latent file missing -> the reader's retry path
]


def _arr(rng, shape):
    return rng.standard_normal(shape).astype(np.float32)


def build(root):
    rng = np.random.default_rng(SEED)
    os.makedirs(os.path.join(root, "null", "wanx"), exist_ok=True)
    np.save(os.path.join(root, "null", "wanx", "uncond.npy"), _arr(rng, (1, 7, 4096)))
    np.save(os.path.join(root, "null", "wanx", "uncond_flf2v.npy"), _arr(rng, (1, 9, 4096)))
    np.save(os.path.join(root, "null", "wanx", "null.npy"), _arr(rng, (1, 1, 4096)))
    metas = []
    for i, c in enumerate(CLIPS):
        base = os.path.join(root, f"clip{i}")
        d = {"source_id": f"clip{i}"}
        p = base + ".npy"
        if not c.get("broken"):
            np.save(p, _arr(rng, LAT))
        d[c["lat"]] = p
        np.save(base + "_cond.npy", _arr(rng, LAT))
        d[c["cond"]] = base + "_cond.npy"
        np.save(base + "_clip.npy", _arr(rng, (1, 257, 1280)))
        d[c["emb"]] = base + "_clip.npy"
        if c["text"] == "short_long":
            np.save(base + "_ts.npy", _arr(rng, (1, 3 + i, 4096)))
            np.save(base + "_tl.npy", _arr(rng, (1, 11 + i, 4096)))
            d.update(textshort_path=base + "_ts.npy", textlong_path=base + "_tl.npy",
                     short_caption=f"short {i}", long_caption=f"long {i}")
        elif c["text"] == "en":
            np.save(base + "_te.npy", _arr(rng, (1, 5, 4096)))
            d.update(text_en_path=base + "_te.npy", prompt=f"prompt {i}")
        else:
            np.save(base + "_ts.npy", _arr(rng, (1, 4, 4096)))
            d.update(save_textshort_path=base + "_ts.npy")
        d.update(c["labels"])
        mp = base + "_meta_v1.json"
        with open(mp, "w") as f:
            json.dump(d, f)
        metas.append(mp)
    lst = os.path.join(root, "meta.list")
    with open(lst, "w") as f:
        f.write("\n".join(metas) + "\n")
    return lst, os.path.join(root, "null")


# sampler cases: (n, replicas, rank, shuffle, seed, epoch, start_index, batch_size)
SAMPLER_CASES = [(10, 1, 0, False, 0, 0, 0, -1), (10, 2, 1, True, 42, 0, 0, -1),
                 (11, 3, 2, True, 42, 1, 0, 1), (17, 4, 0, True, 7, 3, 1, 2),
                 (17, 4, 3, True, 7, 3, 2, 2), (8, 8, 5, True, 110221, 0, 0, 1)]
# crop cases: (shape, width_ratio, height_ratio, type, time_ratio, seed)
CROP_CASES = [((1, 16, 21, 88, 160), 1, 1, "random", 1, 1), ((1, 16, 21, 88, 160), 0.5, 0.75,
              "random", 1, 2), ((1, 16, 21, 60, 104), 0.9, 0.9, "center", 0.6, 3),
              ((1, 16, 13, 61, 105), 0.33, 0.51, "random", 0.5, 4)]
