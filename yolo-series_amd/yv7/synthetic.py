"""Seeded synthetic weights and frames for the yolov7 family (no checkpoints exist offline).

`synthetic_state_dict(model, seed)` fills a models.yolo.Model with reproducible random weights in
the reference's state_dict layout that behave like a trained network's:
  * conv weights: nn.Conv2d's default U(-1/sqrt(fan_in), 1/sqrt(fan_in)) from a seeded generator;
  * BatchNorm running statistics estimated layer by layer on a small batch of synthetic frames
    (the statistics a training pass accumulates), jittered, so every post-BN activation is
    ~N(beta, gamma^2) instead of vanishing or exploding with depth;
  * the Detect head gets a gain and objectness / class biases so that a 640x640 frame yields on the
    order of 10^3 NMS candidates at conf 0.25 (the reference's _initialize_biases prior alone gives
    sigmoid(obj) ~ 1e-4..1e-2, i.e. no detections — SURVEY §7.2 hard part 7).
`synthetic_frames(B, H, W, seed)` gives uint8-derived [0,1] frames as the reference's pre-processing
would (detect.py:100-104).
"""
from __future__ import annotations

import math

import torch
import torch.nn as nn
import torch.nn.functional as F

from models.common import MP, SP, SPPCSPC, Concat, Conv, ReOrg, RepConv
from models.yolo import Detect, IDetect

class _Gen:
    def __init__(self, seed):
        self.g = torch.Generator().manual_seed(seed)

    def uniform(self, shape, lo, hi):
        return torch.rand(shape, generator=self.g) * (hi - lo) + lo

    def normal(self, shape, mean, std):
        return torch.randn(shape, generator=self.g) * std + mean


def _act(m, x):
    a = m.act
    if isinstance(a, nn.SiLU):
        return F.silu(x)
    if isinstance(a, nn.LeakyReLU):
        return F.leaky_relu(x, a.negative_slope)
    return x


def _calib_bn(gen, conv, bn, x):
    """Seeded conv weight; BN running stats = this batch's per-channel statistics of the conv output
    (what a training pass would have accumulated), jittered; returns the post-BN pre-activation tensor."""
    co, ci, k, _ = conv.weight.shape
    bound = 1.0 / math.sqrt(ci * k * k)
    conv.weight.data = gen.uniform(conv.weight.shape, -bound, bound)
    y = F.conv2d(x, conv.weight, None, conv.stride, conv.padding)
    mean = y.mean(dim=(0, 2, 3))
    var = y.var(dim=(0, 2, 3)) + 1e-6
    bn.running_mean.data = mean + gen.normal((co,), 0.0, 0.1) * var.sqrt()
    bn.running_var.data = var * gen.uniform((co,), 0.8, 1.25)
    bn.weight.data = gen.uniform((co,), 0.8, 1.2)
    bn.bias.data = gen.normal((co,), 0.0, 0.2)
    bn.num_batches_tracked.data = torch.tensor(1000)
    return F.batch_norm(y, bn.running_mean, bn.running_var, bn.weight, bn.bias, False, 0.0, bn.eps)


def _calib_conv(gen, m, x):
    return _act(m, _calib_bn(gen, m.conv, m.bn, x))


@torch.no_grad()
def synthetic_state_dict(model, seed=0, head_gain=3.0, obj_bias=-2.5, cls_bias=-3.5, calib_hw=None):
    """Fill `model` (unfused) in place with seeded synthetic weights and return its state_dict.

    The BatchNorm statistics are estimated layer by layer on a small batch of synthetic frames
    (1 x 3 x calib_hw x calib_hw), the way a training pass accumulates them; this is weight
    synthesis only — inference never runs here."""
    gen = _Gen(seed)
    layers = list(model.model)
    if calib_hw is None:  # the model's native resolution: 640 for P5, 1280 for P6 (max stride 64)
        calib_hw = 1280 if float(model.stride.max()) >= 64 else 640
    x0 = synthetic_frames(1, calib_hw, calib_hw, seed=seed + 12345)
    y = []
    x = x0
    for m in layers:
        i = m.i
        if m.f != -1:
            x = y[m.f] if isinstance(m.f, int) else [x if j == -1 else y[j] for j in m.f]
        if isinstance(m, Conv):
            x = _calib_conv(gen, m, x)
        elif isinstance(m, RepConv):
            a = _calib_bn(gen, m.rbr_dense[0], m.rbr_dense[1], x)
            b = _calib_bn(gen, m.rbr_1x1[0], m.rbr_1x1[1], x)
            if isinstance(m.rbr_identity, nn.BatchNorm2d):
                bn = m.rbr_identity
                bn.running_mean.data = x.mean(dim=(0, 2, 3))
                bn.running_var.data = x.var(dim=(0, 2, 3)) + 1e-6
                bn.weight.data.fill_(1.0)
                bn.bias.data.zero_()
                a = a + F.batch_norm(x, bn.running_mean, bn.running_var, bn.weight, bn.bias, False, 0.0, bn.eps)
            x = _act(m, a + b)
        elif isinstance(m, SPPCSPC):
            x1 = _calib_conv(gen, m.cv4, _calib_conv(gen, m.cv3, _calib_conv(gen, m.cv1, x)))
            cat = torch.cat([x1] + [F.max_pool2d(x1, p.kernel_size, 1, p.kernel_size // 2) for p in m.m], 1)
            y1 = _calib_conv(gen, m.cv6, _calib_conv(gen, m.cv5, cat))
            y2 = _calib_conv(gen, m.cv2, x)
            x = _calib_conv(gen, m.cv7, torch.cat((y1, y2), 1))
        elif isinstance(m, MP):
            x = F.max_pool2d(x, m.m.kernel_size, m.m.stride)
        elif isinstance(m, SP):
            x = F.max_pool2d(x, m.m.kernel_size, m.m.stride, m.m.padding)
        elif isinstance(m, Concat):
            x = torch.cat(x, 1)
        elif isinstance(m, nn.Upsample):
            x = F.interpolate(x, scale_factor=2.0, mode='nearest')
        elif isinstance(m, ReOrg):
            x = torch.cat([x[..., ::2, ::2], x[..., 1::2, ::2], x[..., ::2, 1::2], x[..., 1::2, 1::2]], 1)
        elif isinstance(m, Detect):
            feats = x if isinstance(x, list) else [x]
            for j, conv in enumerate(m.m):
                c = conv.weight.shape[1]
                bound = head_gain / math.sqrt(c)
                w = gen.uniform(conv.weight.shape, -bound, bound)
                conv.weight.data = w
                # centre every head output on its own bias: remove the mean the features induce
                mu = F.conv2d(feats[j], w).mean(dim=(0, 2, 3))
                b = (gen.normal((m.na * m.no,), 0.0, 0.3) - mu).view(m.na, m.no)
                b[:, 4] += obj_bias
                b[:, 5:] += cls_bias
                conv.bias.data = b.reshape(-1)
            for conv in getattr(m, 'm2', []):
                c = conv.weight.shape[1]
                conv.weight.data = gen.uniform(conv.weight.shape, -1 / math.sqrt(c), 1 / math.sqrt(c))
                conv.bias.data = gen.normal((conv.bias.numel(),), 0.0, 0.3)
            if isinstance(m, IDetect) and hasattr(m, 'ia'):
                for ia in m.ia:
                    ia.implicit.data = gen.normal(ia.implicit.shape, 0.0, 0.02)
                for im in m.im:
                    im.implicit.data = gen.normal(im.implicit.shape, 1.0, 0.02)
            x = None
        else:
            raise NotImplementedError(type(m).__name__)
        y.append(x if i in model.save else None)
    return {k: v.clone() for k, v in model.state_dict().items()}


def synthetic_frames(B, H, W, seed=0, device='cpu', dtype=torch.float32):
    """uint8 frames in [0,255] -> /255 float [B,3,H,W] (the reference's img/255 pre-processing)."""
    g = torch.Generator().manual_seed(seed)
    x = torch.randint(0, 256, (B, 3, H, W), generator=g, dtype=torch.uint8)
    return (x.to(device).to(dtype) / 255.0)
