"""Device / folding / timing helpers — mirror of the reference's utils/torch_utils.py subset on the path.

  select_device       utils/torch_utils.py:63-86  (ROCm devices are torch 'cuda' devices)
  time_synchronized   utils/torch_utils.py:89-93
  initialize_weights  utils/torch_utils.py:144-153 (BatchNorm eps=1e-3, momentum=0.03)
  fuse_conv_and_bn    utils/torch_utils.py:181-201
  scale_img           utils/torch_utils.py:247-257 (TTA resize; runs as torch GPU ops on the caller's device)
"""
from __future__ import annotations

import logging
import math
import os
import time

import torch
import torch.nn as nn
import torch.nn.functional as F

logger = logging.getLogger(__name__)


def select_device(device='', batch_size=None):
    """'cpu', '' (first GPU) or '0' / '0,1,..' -> torch.device.  On ROCm the HIP devices are 'cuda'."""
    cpu = device.lower() == 'cpu'
    if cpu:
        os.environ['CUDA_VISIBLE_DEVICES'] = '-1'
    elif device:
        os.environ['CUDA_VISIBLE_DEVICES'] = device
        assert torch.cuda.is_available(), f'ROCm device unavailable, invalid device {device} requested'
    cuda = not cpu and torch.cuda.is_available()
    if cuda and batch_size:
        n = torch.cuda.device_count()
        assert n <= 1 or batch_size % n == 0, f'batch-size {batch_size} not multiple of GPU count {n}'
    return torch.device('cuda:0' if cuda else 'cpu')


def time_synchronized():
    if torch.cuda.is_available():
        torch.cuda.synchronize()
    return time.time()


def initialize_weights(model):
    for m in model.modules():
        t = type(m)
        if t is nn.BatchNorm2d:
            m.eps = 1e-3
            m.momentum = 0.03
        elif t in [nn.Hardswish, nn.LeakyReLU, nn.ReLU, nn.ReLU6]:
            m.inplace = True


@torch.no_grad()
def fuse_conv_and_bn(conv, bn):
    """Fold BatchNorm into the preceding conv: W' = diag(g/sqrt(eps+var)) @ W, b' = W_bn b + (beta - g*mu/sqrt(var+eps))."""
    fusedconv = nn.Conv2d(conv.in_channels, conv.out_channels, kernel_size=conv.kernel_size, stride=conv.stride,
                          padding=conv.padding, groups=conv.groups, bias=True).requires_grad_(False).to(
        conv.weight.device)
    w_conv = conv.weight.clone().view(conv.out_channels, -1)
    w_bn = torch.diag(bn.weight.div(torch.sqrt(bn.eps + bn.running_var)))
    fusedconv.weight.copy_(torch.mm(w_bn, w_conv).view(fusedconv.weight.shape))
    b_conv = torch.zeros(conv.weight.size(0), device=conv.weight.device) if conv.bias is None else conv.bias
    b_bn = bn.bias - bn.weight.mul(bn.running_mean).div(torch.sqrt(bn.running_var + bn.eps))
    fusedconv.bias.copy_(torch.mm(w_bn, b_conv.reshape(-1, 1)).reshape(-1) + b_bn)
    return fusedconv


def scale_img(img, ratio=1.0, same_shape=False, gs=32):
    """Resize a [B,3,H,W] batch by ratio and pad to a gs multiple with 0.447 (TTA helper)."""
    if ratio == 1.0:
        return img
    h, w = img.shape[2:]
    s = (int(h * ratio), int(w * ratio))
    img = F.interpolate(img, size=s, mode='bilinear', align_corners=False)
    if not same_shape:
        h, w = [math.ceil(x * ratio / gs) * gs for x in (h, w)]
    return F.pad(img, [0, w - s[1], 0, h - s[0]], value=0.447)


def model_info(model, verbose=False, img_size=640):
    n_p = sum(x.numel() for x in model.parameters())
    logger.info(f'Model Summary: {len(list(model.modules()))} layers, {n_p} parameters')
