"""Deterministic synthetic weights and inputs for parity fixtures (test infrastructure).

There are no Wan2.1 checkpoints on either machine, so every parity fixture is produced with
weights drawn here from numpy's PCG64, seeded per parameter by ``crc32(name)`` so that the
draw depends only on (name, shape, seed) and not on iteration order.  ``make_golden.py`` loads
these weights into the *reference* modules (this container), and the GPU tests load the same
weights into the MI355X-native modules (GPU box) without shipping any weight file.

Scales follow the reference initialisers (`wan/modules/model.py:707-729`, `utils/network.py:30-32,
122-128`) except that biases, norm weights and the zero-initialised `head.head.weight` are
perturbed, so every op and every gradient path is exercised (SURVEY.md §7.2 "random-init trap").
"""
import zlib

import numpy as np

BASE_SEED = 110221  # train_prfl_t2v_480.yaml:71


def _rng(name: str, seed: int) -> np.random.Generator:
    return np.random.Generator(np.random.PCG64([seed, zlib.crc32(name.encode())]))


def param_scale(name: str, shape) -> tuple:
    """(mean, std) for a parameter, by its reference state-dict key."""
    leaf = name.rsplit(".", 1)[-1]
    if name.endswith("modulation"):
        return 0.0, 1.0 / np.sqrt(shape[-1])              # model.py:318, :377
    if "norm" in name and leaf == "weight":
        return 1.0, 0.1                                   # RMSNorm / affine LN weights (ones) + noise
    if leaf == "bias" or leaf == "in_proj_bias":
        return 0.0, 0.02
    if leaf == "queries":
        return 0.0, 1.0 / np.sqrt(shape[-1])
    if len(shape) >= 2:
        fan_in = int(np.prod(shape[1:]))
        std = 1.0 / np.sqrt(fan_in)
        if name.startswith("head.head"):
            std = 0.02
        return 0.0, std
    return 0.0, 0.02


def make_param(name: str, shape, seed: int = BASE_SEED) -> np.ndarray:
    mean, std = param_scale(name, shape)
    a = _rng(name, seed).standard_normal(size=tuple(shape), dtype=np.float32)
    a *= np.float32(std)
    if mean:
        a += np.float32(mean)
    return a


def make_state_dict(named_shapes, seed: int = BASE_SEED) -> dict:
    return {n: make_param(n, s, seed) for n, s in named_shapes}


def randn(name: str, shape, scale: float = 1.0, seed: int = BASE_SEED) -> np.ndarray:
    a = _rng("input:" + name, seed).standard_normal(size=tuple(shape), dtype=np.float32)
    if scale != 1.0:
        a *= np.float32(scale)
    return a
