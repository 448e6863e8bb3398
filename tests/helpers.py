"""Shared fixtures: product model + seeded synthetic weights, and the oracle fed the same weights."""
from __future__ import annotations

import functools

import torch

from models.yolo import Model
from yv7.synthetic import synthetic_frames, synthetic_state_dict


@functools.lru_cache(maxsize=None)
def model_and_weights(name: str, seed: int = 0):
    """(unfused product Model with synthetic weights, state_dict) — cached per (name, seed)."""
    torch.manual_seed(seed)
    m = Model(name)
    sd = synthetic_state_dict(m, seed=seed)
    return m, sd


@functools.lru_cache(maxsize=None)
def oracle_net(name: str, seed: int = 0):
    from oracle import yolo_ref
    m, sd = model_and_weights(name, seed)
    net = yolo_ref.parse(m.yaml)
    fused = yolo_ref.fuse(net, sd)
    return net, fused


def fresh_model(name: str, seed: int = 0, fuse=True):
    """A new product Model instance loaded with the cached synthetic weights (fused like attempt_load)."""
    m0, sd = model_and_weights(name, seed)
    m = Model(name)
    m.load_state_dict(sd)
    m = m.float().eval()
    return m.fuse() if fuse else m


def frames(B, H, W, seed=1):
    return synthetic_frames(B, H, W, seed=seed)
