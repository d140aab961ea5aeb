"""On-disk latent dataset of the PRFL/PAVRM drivers and its device-side staging.

Reference format (written by scripts/preprocess/gen_wanx_latent.py:288-325): one meta JSON per
clip naming fp32 ``.npy`` files —

    vae_latent_path     [1, 16, F, H, W]      video VAE latent
    f1_black_path       [1, 16, F, H, W]      I2V condition latent (first frame + black)
    imgclip_path        [1, 257, 1280]        CLIP image tokens
    textshort_path      [1, Ls, 4096]         umT5 states of short_caption
    textlong_path       [1, Ll, 4096]         umT5 states of long_caption

and a meta *list* file (one JSON path per line).  Read by
``Image2VideoTrainDataset`` (diffusers_lite/datasets/image2video_dataset.py:19-130) through a
``BlockDistributedSampler`` (diffusers_lite/utils/data_utils.py:300-381) and moved to the GPU by
``before_train_step`` (scripts/prfl/train_prfl.py:508-584).

MI355X-side design:
* files are memory-mapped (``np.load(mmap_mode="r")``, never unpickled) and copied once into
  page-locked host buffers by a background thread, so the disk read of sample i+1 overlaps the
  training step of sample i (the reference uses DataLoader worker processes for this);
* the host->HBM copy runs on its own HIP stream and moves the fp32 file bytes as they are; the
  fp32->bf16 cast happens in HBM with the library's cast kernel (bit-identical to
  ``.to(bfloat16)``), stream-ordered before the compute stream's first use by an event;
* the I2V mask channels, the crop and ``max_sequence_length`` follow ``before_train_step``.
"""
import json
import math
import os
import queue
import random
import threading

import numpy as np
import torch

NULL_DIR = os.environ.get("PRFL_NULL_DIR", "temp_data/null")   # diffusers_lite/constants.py:9


def align_floor_to(value, alignment):
    """data_utils.py:41-42"""
    return int(math.floor(value / alignment) * alignment)


def _load(path):
    # memory-mapped, never unpickled (allow_pickle stays False)
    return np.load(path, mmap_mode="r", allow_pickle=False)


def _first(d, *keys):
    for k in keys:
        if k in d:
            return d[k]
    raise KeyError(keys[-1])


class Image2VideoTrainDataset(torch.utils.data.Dataset):
    """Same constructor and item tuples as image2video_dataset.py:19-53 for the dataset types the
    PRFL (``refl``) and PAVRM (``lrm_ce``) drivers use.  Items are CPU fp32 tensors (views of the
    mapped files are copied out, so an item owns its memory)."""

    def __init__(self, task="i2v-14b-480p", dataset_type="wanx", meta_file_list=(),
                 meta_file_lose_list=(), uncond_prob=(0.0, 0.0), sp_size=1, patch_size=(1, 2, 2),
                 null_dir=None):
        self.task = task
        self.dataset_type = dataset_type
        self.uncond_prompt_prob = uncond_prob[0]
        self.uncond_image_prob = uncond_prob[-1]
        self.sp_size = sp_size
        self.patch_size = patch_size
        self.null_dir = NULL_DIR if null_dir is None else null_dir
        self.meta_paths = []
        for meta_file in meta_file_list:
            with open(meta_file) as f:
                self.meta_paths.extend(line.strip() for line in f.readlines())
        self.meta_paths_lose = []
        for meta_file in meta_file_lose_list:
            with open(meta_file) as f:
                self.meta_paths_lose.extend(line.strip() for line in f.readlines())

    def __len__(self):
        return len(self.meta_paths)

    def __getitem__(self, idx):
        # image2video_dataset.py:55-70: retry a random other index on a bad sample
        err = None
        for _ in range(100):
            try:
                if self.dataset_type == "refl":
                    return self.get_batch_lrm_refl(idx)
                if self.dataset_type == "lrm_ce":
                    return self.get_batch_lrm_ce(idx)
                raise NotImplementedError(f"dataset_type {self.dataset_type!r}")
            except NotImplementedError:
                raise
            except Exception as e:   # noqa: BLE001 — the reference skips unreadable samples
                err = e
                idx = np.random.randint(len(self.meta_paths))
        raise RuntimeError("Too many bad data.") from err

    # -- pieces shared by both item types ----------------------------------------------------
    def _uncond(self):
        name = "uncond_flf2v.npy" if "flf2v" in self.task else "uncond.npy"
        return torch.from_numpy(np.array(_load(os.path.join(self.null_dir, "wanx", name))[0]))

    @staticmethod
    def _image_embeds(path):
        a = np.array(_load(path))
        return torch.from_numpy(a.reshape(-1, a.shape[-1]))          # "b s d -> (b s) d"

    @staticmethod
    def _arr0(path):
        return torch.from_numpy(np.array(_load(path)[0]))

    def get_batch_lrm_refl(self, idx):
        """image2video_dataset.py:72-130 (dataset_type "refl", train_prfl.py:444)."""
        with open(self.meta_paths[idx]) as f:
            d = json.load(f)
        latents = self._arr0(_first(d, "video_vae_latent_path", "vae_latent_path", "latents_path"))
        if "textshort_path" in d and "textlong_path" in d:
            text_path, prompt = d["textshort_path"], d["short_caption"]
            if random.random() <= 0.7:
                text_path, prompt = d["textlong_path"], d["long_caption"]
        else:
            text_path, prompt = d["text_en_path"], d["prompt"]
        text_states = self._arr0(text_path)
        image_embeds = self._image_embeds(d["imgclip_path"])
        latents_condition = self._arr0(_first(d, "f1_black_path", "latents_condition_path"))
        uncond = self._uncond()
        if random.random() < self.uncond_prompt_prob:
            text_states = torch.from_numpy(
                np.array(_load(os.path.join(self.null_dir, "wanx", "null.npy"))[0]))
        return latents, text_states, uncond, image_embeds, latents_condition, prompt

    def get_batch_lrm_ce(self, idx):
        """image2video_dataset.py:177-262 (dataset_type "lrm_ce", the PAVRM driver)."""
        with open(self.meta_paths[idx]) as f:
            d = json.load(f)
        latents = self._arr0(_first(d, "video_vae_latent_path", "vae_latent_path"))
        text_states = self._arr0(_first(d, "save_textshort_path", "textshort_path", "text_en_path"))
        image_embeds = self._image_embeds(_first(d, "image_embeds", "imgclip_path"))
        latents_condition = self._arr0(_first(d, "f1_black_path", "latents_condition_path"))
        uncond = self._uncond()
        labels = []
        for k in ("text_alignment", "blur_quality", "physics_quality", "human_quality"):
            v = d.get(k, 0)
            labels.append(0 if v in ("poor", None) else 1 if v == "good" else v)
        return (latents, text_states, uncond, image_embeds, latents_condition,
                d.get("model", ""), *labels)


class BlockDistributedSampler(torch.utils.data.Sampler):
    """data_utils.py:300-381: each data-parallel rank takes one contiguous block of a (seeded,
    per-epoch) permutation, truncated to a multiple of ``align`` and offset by ``start_index``
    (resume)."""

    def __init__(self, dataset, num_replicas=1, rank=0, shuffle=False, seed=0, drop_last=False,
                 batch_size=-1, start_index=0, align=1):
        if rank >= num_replicas or rank < 0:
            raise ValueError(f"Invalid rank {rank}, rank should be in the interval "
                             f"[0, {num_replicas - 1}]")
        if batch_size != -1:
            align = batch_size
        if align <= 0:
            raise ValueError(f"align should be a positive integer, but got {align}.")
        self.dataset, self.num_replicas, self.rank = dataset, num_replicas, rank
        self.shuffle, self.seed, self.drop_last = shuffle, seed, drop_last
        self.batch_size, self.align, self.epoch = batch_size, align, 0
        self.start_index = start_index

    @property
    def num_samples(self):
        return len(self.dataset) // self.align * self.align // self.num_replicas - self.start_index

    def set_epoch(self, epoch):
        self.epoch = epoch

    def __len__(self):
        return self.num_samples

    def __iter__(self):
        n = len(self.dataset)
        if self.shuffle:
            g = torch.Generator()
            g.manual_seed(self.seed + self.epoch)
            indices = torch.randperm(n, generator=g).tolist()
        else:
            indices = list(range(n))
        per = n // self.align * self.align // self.num_replicas
        indices = indices[:per * self.num_replicas]
        indices = indices[self.rank * per + self.start_index:(self.rank + 1) * per]
        assert len(indices) + self.start_index == per
        return iter(indices)


def crop_window(shape, crop_width_ratio=1.0, crop_height_ratio=1.0, crop_type="center",
                crop_time_ratio=1.0):
    """data_utils.py:49-78 as (t, top, height, left, width) of the crop of a [B,C,T,H,W] latent.
    ``random`` draws from Python's ``random`` in the reference's order (top, then left)."""
    _, _, t, h, w = shape
    crop_h, crop_w = int(h * crop_height_ratio), int(w * crop_width_ratio)
    crop_t = int(t * crop_time_ratio)
    if crop_type == "center":
        top, left = (h - crop_h) // 2, (w - crop_w) // 2
    elif crop_type == "random":
        top = random.randint(0, h - crop_h)
        left = random.randint(0, w - crop_w)
    else:
        raise ValueError(crop_type)
    return (align_floor_to(crop_t, 1), top, align_floor_to(crop_h, 2), left,
            align_floor_to(crop_w, 2))


def crop_tensor(latents, image_latents=None, crop_width_ratio=1.0, crop_height_ratio=1.0,
                crop_type="center", crop_time_ratio=1.0):
    t, top, ch, left, cw = crop_window(latents.shape, crop_width_ratio, crop_height_ratio,
                                       crop_type, crop_time_ratio)
    cut = lambda x: x[:, :, :t, top:top + ch, left:left + cw]   # noqa: E731
    return cut(latents), (cut(image_latents) if image_latents is not None else None)


def collate(items):
    """default_collate of the reference's DataLoader for batch_size rows of equal shape."""
    out = []
    for field in zip(*items):
        out.append(torch.stack(field) if torch.is_tensor(field[0]) else list(field))
    return out


class DeviceBatch(dict):
    __getattr__ = dict.__getitem__


class LatentPrefetcher:
    """Iterates the sampler's indices, reading ``batch_size`` items ahead on a host thread into
    page-locked buffers and copying them to HBM on a dedicated stream; ``next()`` returns the
    ``before_train_step`` dictionary (train_prfl.py:508-584) for the current batch."""

    def __init__(self, dataset, sampler, batch_size=1, device="cuda", task="t2v-14b",
                 patch_size=(1, 2, 2), crop_ratio=(1, 1, 1), crop_type="center", depth=2):
        self.dataset, self.sampler, self.batch_size = dataset, sampler, batch_size
        self.device = torch.device(device)
        self.task, self.patch_size = task, patch_size
        self.crop_ratio, self.crop_type = crop_ratio, crop_type
        self.cond = "i2v" in task or "flf2v" in task
        self._q = queue.Queue(maxsize=depth)
        self._stop = threading.Event()
        self._epoch = 0
        self._thread = threading.Thread(target=self._reader, daemon=True)
        self._thread.start()
        self._stream = torch.cuda.Stream(self.device) if self.device.type == "cuda" else None

    def _reader(self):
        try:
            while not self._stop.is_set():
                self.sampler.set_epoch(self._epoch)
                idx = list(iter(self.sampler))
                for b in range(0, len(idx) - self.batch_size + 1, self.batch_size):
                    batch = collate([self.dataset[i] for i in idx[b:b + self.batch_size]])
                    pinned = [t.pin_memory() if torch.is_tensor(t) and self._pin() else t
                              for t in batch]
                    while not self._stop.is_set():
                        try:
                            self._q.put(pinned, timeout=0.5)
                            break
                        except queue.Full:
                            continue
                    if self._stop.is_set():
                        return
                self._epoch += 1
        except Exception as e:   # noqa: BLE001 — surfaced to the consumer
            self._q.put(e)

    def _pin(self):
        return self.device.type == "cuda"

    def close(self):
        self._stop.set()
        self._thread.join(timeout=5)

    def __iter__(self):
        return self

    def _to_device(self, t):
        """fp32 host tensor -> bf16 device tensor: raw fp32 bytes over PCIe on the copy stream,
        cast in HBM by the HIP cast kernel (the reference's `.to(device, dtype=bf16)`)."""
        from . import ops
        dev32 = t.to(self.device, non_blocking=True)
        out = torch.empty(dev32.shape, dtype=torch.bfloat16, device=self.device)
        ops.cast_bf16(dev32.contiguous(), out)
        return out

    def __next__(self):
        item = self._q.get()
        if isinstance(item, Exception):
            raise item
        latents, text, uncond, image_embeds, cond, prompt = item[:6]
        if self.device.type != "cuda":
            raise RuntimeError("LatentPrefetcher stages batches into HBM; it needs the GPU")
        with torch.cuda.stream(self._stream):
            latents = self._to_device(latents)
            text = self._to_device(text)
            uncond = self._to_device(uncond)
            cond_d = self._to_device(cond) if self.cond else None
            emb_d = self._to_device(image_embeds) if self.cond else None
            ready = torch.cuda.Event()
            ready.record(self._stream)
        cur = torch.cuda.current_stream(self.device)
        cur.wait_event(ready)
        for t in (latents, text, uncond, cond_d, emb_d):
            if t is not None:
                t.record_stream(cur)
        if cond_d is not None:
            b, c, f, h, w = cond_d.shape
            if c == 16:   # train_prfl.py:535-540: 4 mask channels, first frame = 1
                mask = torch.zeros((b, 4, f, h, w), dtype=cond_d.dtype, device=cond_d.device)
                mask[:, :, :1] = 1.0
                cond_d = torch.cat([mask, cond_d], dim=1)
        if emb_d is not None:   # "b (n s) d -> (b n) s d", n = tokens // 257
            n = emb_d.shape[1] // 257
            emb_d = emb_d.reshape(emb_d.shape[0] * n, 257, emb_d.shape[-1])
        if getattr(self.dataset, "sp_size", 1) <= 1:
            latents, cond_d = crop_tensor(latents, cond_d, self.crop_ratio[0], self.crop_ratio[1],
                                          self.crop_type, crop_time_ratio=self.crop_ratio[2])
        _, _, t, h, w = latents.shape
        L = t * h * w // (self.patch_size[1] * self.patch_size[2])
        return DeviceBatch(latents=latents, text_states=text, image_embeds=emb_d,
                           latents_condition=cond_d, max_sequence_length=L,
                           uncond_text_states=uncond, text_prompt=prompt)
