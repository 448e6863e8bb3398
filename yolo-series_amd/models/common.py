"""Layer modules of the yolov7 family — the reference's layer "plugin" names and parameter trees.

Mirror of the reference interface in models/common.py: class names (Conv, RepConv, SPPCSPC, MP, SP,
ReOrg, Concat, ImplicitA, ImplicitM) and attribute names (conv, bn, act, rbr_dense, rbr_1x1,
rbr_identity, rbr_reparam, cv1..cv7, m, implicit) are identical, so reference-keyed state_dicts
 load unchanged.  The modules are parameter containers: the computation of the
whole network runs on the MI355X through the compiled plan (yv7.graph / libyv7), never layer by
layer and never on the CPU, so calling a layer directly raises.

Folding (Model.fuse in the reference) is restated here with the reference arithmetic:
  Conv:    fuse_conv_and_bn      utils/torch_utils.py:181-201
  RepConv: fuse_repvgg_block     models/common.py:584-643 (+ fuse_conv_bn 561-582)
"""
from __future__ import annotations

import torch
import torch.nn as nn

from utils.torch_utils import fuse_conv_and_bn


def autopad(k, p=None):  # models/common.py:23-27
    if p is None:
        p = k // 2 if isinstance(k, int) else [x // 2 for x in k]
    return p


class _PlanOnly(nn.Module):
    """Layers execute only inside the compiled network (Model.forward -> libyv7)."""

    def forward(self, *args, **kwargs):
        raise RuntimeError(f'{type(self).__name__} runs only as part of models.yolo.Model.forward on a ROCm '
                           f'device (compiled plan); there is no per-layer or CPU execution path')


class MP(_PlanOnly):  # common.py:30-36
    def __init__(self, k=2):
        super().__init__()
        self.m = nn.MaxPool2d(kernel_size=k, stride=k)


class SP(_PlanOnly):  # common.py:39-45
    def __init__(self, k=3, s=1):
        super().__init__()
        self.m = nn.MaxPool2d(kernel_size=k, stride=s, padding=k // 2)


class ReOrg(_PlanOnly):  # common.py:48-53 (x(b,c,w,h) -> y(b,4c,w/2,h/2))
    pass


class Concat(_PlanOnly):  # common.py:56-62
    def __init__(self, dimension=1):
        super().__init__()
        self.d = dimension


class Conv(_PlanOnly):
    """Conv2d(bias=False) + BatchNorm2d + act (common.py:99-111); after fuse(): conv has a bias, no bn."""

    def __init__(self, c1, c2, k=1, s=1, p=None, g=1, act=True):
        super().__init__()
        self.conv = nn.Conv2d(c1, c2, k, s, autopad(k, p), groups=g, bias=False)
        self.bn = nn.BatchNorm2d(c2)
        self.act = nn.SiLU() if act is True else (act if isinstance(act, nn.Module) else nn.Identity())

    def fuse(self):
        if hasattr(self, 'bn'):
            self.conv = fuse_conv_and_bn(self.conv, self.bn)
            delattr(self, 'bn')
        return self

    def fused_weight_bias(self):
        """(W [c2,c1,k,k], b [c2]) in fp32 with BN folded, whatever the module's current state."""
        if hasattr(self, 'bn'):
            f = fuse_conv_and_bn(self.conv.float(), self.bn.float())
            return f.weight.detach().float(), f.bias.detach().float()
        b = self.conv.bias if self.conv.bias is not None else torch.zeros(self.conv.out_channels)
        return self.conv.weight.detach().float(), b.detach().float()


def _fuse_conv_bn(conv, bn):
    """RepConv.fuse_conv_bn arithmetic (common.py:561-582): returns (W*t, beta - mean*gamma/std)."""
    std = (bn.running_var + bn.eps).sqrt()
    bias = bn.bias - bn.running_mean * bn.weight / std
    t = (bn.weight / std).reshape(-1, 1, 1, 1)
    return conv.weight * t, bias


class RepConv(_PlanOnly):
    """RepVGG-style block (common.py:463-643): 3x3+BN, 1x1+BN (+ identity BN) -> one 3x3 conv when deployed."""

    def __init__(self, c1, c2, k=3, s=1, p=None, g=1, act=True, deploy=False):
        super().__init__()
        self.deploy = deploy
        self.groups = g
        self.in_channels = c1
        self.out_channels = c2
        assert k == 3
        assert autopad(k, p) == 1
        padding_11 = autopad(k, p) - k // 2
        self.act = nn.SiLU() if act is True else (act if isinstance(act, nn.Module) else nn.Identity())
        if deploy:
            self.rbr_reparam = nn.Conv2d(c1, c2, k, s, autopad(k, p), groups=g, bias=True)
        else:
            self.rbr_identity = nn.BatchNorm2d(num_features=c1) if c2 == c1 and s == 1 else None
            self.rbr_dense = nn.Sequential(nn.Conv2d(c1, c2, k, s, autopad(k, p), groups=g, bias=False),
                                           nn.BatchNorm2d(num_features=c2))
            self.rbr_1x1 = nn.Sequential(nn.Conv2d(c1, c2, 1, s, padding_11, groups=g, bias=False),
                                         nn.BatchNorm2d(num_features=c2))

    @torch.no_grad()
    def _equivalent(self):
        w3, b3 = _fuse_conv_bn(self.rbr_dense[0], self.rbr_dense[1])
        w1, b1 = _fuse_conv_bn(self.rbr_1x1[0], self.rbr_1x1[1])
        w1 = torch.nn.functional.pad(w1, [1, 1, 1, 1])
        if isinstance(self.rbr_identity, nn.BatchNorm2d):
            eye = torch.zeros(self.out_channels, self.in_channels // self.groups, 1, 1, dtype=w3.dtype)
            for i in range(self.out_channels):
                eye[i, i % (self.in_channels // self.groups), 0, 0] = 1.0
            idc = nn.Conv2d(self.in_channels, self.out_channels, 1, bias=False)
            idc.weight.data = eye
            wi, bi = _fuse_conv_bn(idc, self.rbr_identity)
            wi = torch.nn.functional.pad(wi, [1, 1, 1, 1])
        else:
            wi, bi = torch.zeros_like(w1), torch.zeros_like(b1)
        return w3 + w1 + wi, b3 + b1 + bi

    def fuse_repvgg_block(self):
        if self.deploy:
            return
        w, b = self._equivalent()
        conv = self.rbr_dense[0]
        self.rbr_reparam = nn.Conv2d(conv.in_channels, conv.out_channels, conv.kernel_size, conv.stride,
                                     conv.padding, groups=conv.groups, bias=True)
        self.rbr_reparam.weight = nn.Parameter(w.detach())
        self.rbr_reparam.bias = nn.Parameter(b.detach())
        self.deploy = True
        for name in ('rbr_identity', 'rbr_1x1', 'rbr_dense'):
            if hasattr(self, name):
                delattr(self, name)

    def fused_weight_bias(self):
        if hasattr(self, 'rbr_reparam'):
            return self.rbr_reparam.weight.detach().float(), self.rbr_reparam.bias.detach().float()
        w, b = self._equivalent()
        return w.detach().float(), b.detach().float()


class SPPCSPC(_PlanOnly):
    """CSP spatial pyramid pooling (common.py:262-280)."""

    def __init__(self, c1, c2, n=1, shortcut=False, g=1, e=0.5, k=(5, 9, 13)):
        super().__init__()
        c_ = int(2 * c2 * e)
        self.cv1 = Conv(c1, c_, 1, 1)
        self.cv2 = Conv(c1, c_, 1, 1)
        self.cv3 = Conv(c_, c_, 3, 1)
        self.cv4 = Conv(c_, c_, 1, 1)
        self.m = nn.ModuleList([nn.MaxPool2d(kernel_size=x, stride=1, padding=x // 2) for x in k])
        self.cv5 = Conv(4 * c_, c_, 1, 1)
        self.cv6 = Conv(c_, c_, 3, 1)
        self.cv7 = Conv(2 * c_, c2, 1, 1)


class ImplicitA(_PlanOnly):  # common.py:433-443
    def __init__(self, channel, mean=0., std=.02):
        super().__init__()
        self.channel = channel
        self.mean = mean
        self.std = std
        self.implicit = nn.Parameter(torch.zeros(1, channel, 1, 1))
        nn.init.normal_(self.implicit, mean=self.mean, std=self.std)


class ImplicitM(_PlanOnly):  # common.py:446-456
    def __init__(self, channel, mean=1., std=.02):
        super().__init__()
        self.channel = channel
        self.mean = mean
        self.std = std
        self.implicit = nn.Parameter(torch.ones(1, channel, 1, 1))
        nn.init.normal_(self.implicit, mean=self.mean, std=self.std)
