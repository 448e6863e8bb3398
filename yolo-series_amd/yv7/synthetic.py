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


def _calib_bn(gen, conv, bn, x, gamma=(0.3, 0.6), beta_sd=0.7):
    """Seeded conv weight; BN running stats = this batch's per-channel statistics of the conv output
    (what a training pass would have accumulated), jittered; returns the post-BN pre-activation tensor.

    gamma / beta: BN affine parameters U(gamma) / N(0, beta_sd).  Moderate gammas with larger betas
    keep the random network well conditioned (fp32 vs fp64 box error ~1e-5 at 640, fp16-storage drift
    ~1e-2), like a trained detector; gammas near 1 with small betas make a random 100-layer network
    chaotic (fp32 vs fp64 ~1e-3, fp16 drift O(1)), which no trained YOLOv7 is."""
    co, ci, k, _ = conv.weight.shape
    bound = 1.0 / math.sqrt(ci * k * k)
    conv.weight.data = gen.uniform(conv.weight.shape, -bound, bound)
    y = F.conv2d(x, conv.weight, None, conv.stride, conv.padding)
    mean = y.mean(dim=(0, 2, 3))
    var = y.var(dim=(0, 2, 3)) + 1e-6
    bn.running_mean.data = mean + gen.normal((co,), 0.0, 0.1) * var.sqrt()
    bn.running_var.data = var * gen.uniform((co,), 0.8, 1.25)
    bn.weight.data = gen.uniform((co,), gamma[0], gamma[1])
    bn.bias.data = gen.normal((co,), 0.0, beta_sd)
    bn.num_batches_tracked.data = torch.tensor(1000)
    return F.batch_norm(y, bn.running_mean, bn.running_var, bn.weight, bn.bias, False, 0.0, bn.eps)


def _calib_conv(gen, m, x, **kw):
    return _act(m, _calib_bn(gen, m.conv, m.bn, x, **kw))


def _tune_head_biases(logits, na, no, target, conf=0.25):
    """Shift class / objectness biases so that `target` of all anchor rows pass conf (obj*cls > conf)."""
    rows = []
    for lg in logits:  # [1, na*no, ny, nx] pre-bias logits + per-channel noise already added
        v = lg.view(na, no, -1).permute(0, 2, 1).reshape(-1, no)
        rows.append(v)
    v = torch.cat(rows, 0)
    mx = v[:, 5:].max(1).values
    c_shift = -float(mx.median())            # the median row's best class logit sits at 0 (sigmoid 0.5)
    cls = torch.sigmoid(mx + c_shift)
    lo, hi = -20.0, 20.0
    for _ in range(60):                      # bisection on the objectness shift
        mid = 0.5 * (lo + hi)
        frac = float(((torch.sigmoid(v[:, 4] + mid) > conf) & (torch.sigmoid(v[:, 4] + mid) * cls > conf))
                     .float().mean())
        lo, hi = (lo, mid) if frac > target else (mid, hi)
    return 0.5 * (lo + hi), c_shift


@torch.no_grad()
def synthetic_state_dict(model, seed=0, head_gain=2.0, target_candidates=0.06, calib_hw=None,
                         gamma=(0.3, 0.6), beta_sd=0.7):
    """Fill `model` (unfused) in place with seeded synthetic weights and return its state_dict.

    The BatchNorm statistics are estimated layer by layer on one synthetic frame
    (1 x 3 x calib_hw x calib_hw), the way a training pass accumulates them, and the head biases are
    set so that `target_candidates` of the anchor rows pass conf 0.25 on that frame; this is weight
    synthesis only — inference never runs here."""
    gen = _Gen(seed)
    bnkw = dict(gamma=gamma, beta_sd=beta_sd)
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
            x = _calib_conv(gen, m, x, **bnkw)
        elif isinstance(m, RepConv):
            a = _calib_bn(gen, m.rbr_dense[0], m.rbr_dense[1], x, **bnkw)
            b = _calib_bn(gen, m.rbr_1x1[0], m.rbr_1x1[1], x, **bnkw)
            if isinstance(m.rbr_identity, nn.BatchNorm2d):
                bn = m.rbr_identity
                bn.running_mean.data = x.mean(dim=(0, 2, 3))
                bn.running_var.data = x.var(dim=(0, 2, 3)) + 1e-6
                bn.weight.data.fill_(1.0)
                bn.bias.data.zero_()
                a = a + F.batch_norm(x, bn.running_mean, bn.running_var, bn.weight, bn.bias, False, 0.0, bn.eps)
            x = _act(m, a + b)
        elif isinstance(m, SPPCSPC):
            x1 = _calib_conv(gen, m.cv4, _calib_conv(gen, m.cv3, _calib_conv(gen, m.cv1, x, **bnkw), **bnkw), **bnkw)
            cat = torch.cat([x1] + [F.max_pool2d(x1, p.kernel_size, 1, p.kernel_size // 2) for p in m.m], 1)
            y1 = _calib_conv(gen, m.cv6, _calib_conv(gen, m.cv5, cat, **bnkw), **bnkw)
            y2 = _calib_conv(gen, m.cv2, x, **bnkw)
            x = _calib_conv(gen, m.cv7, torch.cat((y1, y2), 1), **bnkw)
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
            logits, noise = [], []
            for j, conv in enumerate(m.m):
                c = conv.weight.shape[1]
                bound = head_gain / math.sqrt(c)
                w = gen.uniform(conv.weight.shape, -bound, bound)
                conv.weight.data = w
                lg = F.conv2d(feats[j], w)
                # centre every head output on its own bias: remove the mean the features induce
                b = gen.normal((m.na * m.no,), 0.0, 0.3) - lg.mean(dim=(0, 2, 3))
                noise.append(b)
                logits.append(lg + b[None, :, None, None])
            o_shift, c_shift = _tune_head_biases(logits, m.na, m.no, target_candidates)
            for j, conv in enumerate(m.m):
                b = noise[j].view(m.na, m.no).clone()
                b[:, 4] += o_shift
                b[:, 5:] += c_shift
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
