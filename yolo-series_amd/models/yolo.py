"""YOLOv7 model API — mirror of the reference's models/yolo.py on the inference path.

Same names, constructor arguments, attributes and return values as the reference:
  Detect / IDetect / IAuxDetect   models/yolo.py:23-94, 97-207, 311-430 (anchors, anchor_grid, stride, m, ia, im, m2)
  Model(cfg, ch, nc, anchors)     models/yolo.py:508-579 (stride probe, check_anchor_order, _initialize_biases,
                                  initialize_weights)
  Model.forward(x, augment, profile) -> (z [B,N,no], xs list of [B,na,ny,nx,no])   yolo.py:581-631
  Model.fuse()                    yolo.py:693-710
  parse_model(d, ch)              yolo.py:736-813 (module names resolved through a registry, not eval)

What differs is where the work happens: `forward` compiles the (fused) network once per
(device, dtype) into a libyv7 plan — NHWC tensors, packed weights in HBM, a flat op list — and
every call is one C-ABI call that launches the HIP kernels of the whole network on the current
stream.  There is no CPU execution path: a CPU input raises (the CPU reference is oracle/, which
is test infrastructure only).
"""
from __future__ import annotations

import logging
import math
import re
from copy import deepcopy
from pathlib import Path

import torch
import torch.nn as nn

from models.common import (MP, SP, Concat, Conv, ImplicitA, ImplicitM, ReOrg, RepConv, SPPCSPC)
from utils.general import make_divisible
from utils.torch_utils import initialize_weights, model_info, scale_img

logger = logging.getLogger(__name__)


def check_anchor_order(m):  # utils/autoanchor.py:12-20
    a = m.anchor_grid.prod(-1).view(-1)
    da = a[-1] - a[0]
    ds = m.stride[-1] - m.stride[0]
    if da.sign() != ds.sign():
        print('Reversing anchor order')
        m.anchors[:] = m.anchors.flip(0)
        m.anchor_grid[:] = m.anchor_grid.flip(0)


class Detect(nn.Module):
    stride = None
    export = False
    end2end = False
    include_nms = False
    concat = False

    def __init__(self, nc=80, anchors=(), ch=()):
        super().__init__()
        self.nc = nc
        self.no = nc + 5
        self.nl = len(anchors)
        self.na = len(anchors[0]) // 2
        self.grid = [torch.zeros(1)] * self.nl
        a = torch.tensor(anchors).float().view(self.nl, -1, 2)
        self.register_buffer('anchors', a)  # (nl, na, 2), in grid units after Model.__init__
        self.register_buffer('anchor_grid', a.clone().view(self.nl, 1, -1, 1, 1, 2))  # pixels
        self.m = nn.ModuleList(nn.Conv2d(x, self.no * self.na, 1) for x in ch)

    def head_weights(self, j):
        """Fused fp32 (W [na*no, C, 1, 1], b [na*no]) of level j."""
        return self.m[j].weight.detach().float(), self.m[j].bias.detach().float()

    def forward(self, x):
        raise RuntimeError('Detect runs only inside models.yolo.Model.forward (compiled plan)')


class IDetect(Detect):
    """Detect with ImplicitA before and ImplicitM after the head conv (yolo.py:97-207)."""

    def __init__(self, nc=80, anchors=(), ch=()):
        super().__init__(nc, anchors, ch)
        self.ia = nn.ModuleList(ImplicitA(x) for x in ch)
        self.im = nn.ModuleList(ImplicitM(self.no * self.na) for _ in ch)

    def head_weights(self, j):
        w, b = super().head_weights(j)
        if hasattr(self, 'ia'):  # unfused: fold exactly as IDetect.fuse (yolo.py:178-190)
            c1, c2 = w.shape[:2]
            ia = self.ia[j].implicit.detach().float()
            im = self.im[j].implicit.detach().float()
            b = b + torch.matmul(w.reshape(c1, c2), ia.reshape(ia.shape[1], ia.shape[0])).squeeze(1)
            b = b * im.reshape(im.shape[1])
            w = w * im.transpose(0, 1)
        return w, b

    @torch.no_grad()
    def fuse(self):
        for j in range(len(self.m)):
            w, b = self.head_weights(j)
            self.m[j].weight.data = w.to(self.m[j].weight.dtype)
            self.m[j].bias.data = b.to(self.m[j].bias.dtype)
        del self.ia
        del self.im


class IAuxDetect(IDetect):
    """Training-cfg P6 head (yolo.py:311-430): main heads m + auxiliary heads m2 (unused at inference)."""

    def __init__(self, nc=80, anchors=(), ch=()):
        nn.Module.__init__(self)
        self.nc = nc
        self.no = nc + 5
        self.nl = len(anchors)
        self.na = len(anchors[0]) // 2
        self.grid = [torch.zeros(1)] * self.nl
        a = torch.tensor(anchors).float().view(self.nl, -1, 2)
        self.register_buffer('anchors', a)
        self.register_buffer('anchor_grid', a.clone().view(self.nl, 1, -1, 1, 1, 2))
        self.m = nn.ModuleList(nn.Conv2d(x, self.no * self.na, 1) for x in ch[:self.nl])
        self.m2 = nn.ModuleList(nn.Conv2d(x, self.no * self.na, 1) for x in ch[self.nl:])
        self.ia = nn.ModuleList(ImplicitA(x) for x in ch[:self.nl])
        self.im = nn.ModuleList(ImplicitM(self.no * self.na) for _ in ch[:self.nl])


# The layer "plugin registry": names the cfg may use (the reference resolves them with eval(), yolo.py:744).
MODULES = {
    'Conv': Conv, 'RepConv': RepConv, 'SPPCSPC': SPPCSPC, 'MP': MP, 'SP': SP, 'ReOrg': ReOrg, 'Concat': Concat,
    'Detect': Detect, 'IDetect': IDetect, 'IAuxDetect': IAuxDetect, 'nn.Upsample': nn.Upsample,
    'nn.Conv2d': nn.Conv2d, 'nn.BatchNorm2d': nn.BatchNorm2d,
}
_ACTS = {'nn.SiLU()': lambda: nn.SiLU(), 'nn.ReLU()': lambda: nn.ReLU(), 'nn.Identity()': lambda: nn.Identity()}
_LEAKY = re.compile(r'nn\.LeakyReLU\(\s*([-+0-9.eE]+)\s*\)')


def _resolve_arg(a, nc, anchors):
    if not isinstance(a, str):
        return a
    if a == 'None':
        return None
    if a == 'nc':
        return nc
    if a == 'anchors':
        return anchors
    if a in ('True', 'False'):
        return a == 'True'
    if a in _ACTS:
        return _ACTS[a]()
    m = _LEAKY.fullmatch(a)
    if m:
        return nn.LeakyReLU(float(m.group(1)))
    return a


def parse_model(d, ch):
    """cfg dict -> (nn.Sequential of layers with .i/.f/.type/.np, sorted save list) (yolo.py:736-813)."""
    anchors, nc, gd, gw = d['anchors'], d['nc'], d['depth_multiple'], d['width_multiple']
    na = (len(anchors[0]) // 2) if isinstance(anchors, list) else anchors
    no = na * (nc + 5)
    layers, save, c2 = [], [], ch[-1]
    for i, (f, n, m, args) in enumerate(d['backbone'] + d['head']):
        if m not in MODULES:
            raise NotImplementedError(f'module {m!r} is not part of the yolov7-family inference path')
        mod = MODULES[m]
        args = [_resolve_arg(a, nc, anchors) for a in args]
        n = max(round(n * gd), 1) if n > 1 else n
        if mod in (nn.Conv2d, Conv, RepConv, SPPCSPC):
            c1, c2 = ch[f], args[0]
            if c2 != no:
                c2 = make_divisible(c2 * gw, 8)
            args = [c1, c2, *args[1:]]
            if mod is SPPCSPC:
                args.insert(2, n)
                n = 1
        elif mod is nn.BatchNorm2d:
            args = [ch[f]]
        elif mod is Concat:
            c2 = sum(ch[x] for x in f)
        elif mod in (Detect, IDetect, IAuxDetect):
            args.append([ch[x] for x in f])
            if isinstance(args[1], int):
                args[1] = [list(range(args[1] * 2))] * len(f)
        elif mod is ReOrg:
            c2 = ch[f] * 4
        else:
            c2 = ch[f]
        m_ = nn.Sequential(*[mod(*args) for _ in range(n)]) if n > 1 else mod(*args)
        m_.i, m_.f, m_.type, m_.np = i, f, m, sum(x.numel() for x in m_.parameters())
        save.extend(x % i for x in ([f] if isinstance(f, int) else f) if x != -1)
        layers.append(m_)
        if i == 0:
            ch = []
        ch.append(c2)
    return nn.Sequential(*layers), sorted(save)


def _levels(layers):
    """log2 spatial stride of each layer's output: what the reference's 256x256 probe forward measures."""
    lv = []
    for m in layers:
        src = m.f if isinstance(m.f, int) else m.f[0]
        prev = 0 if m.i == 0 else (lv[-1] if src == -1 else lv[src])
        if isinstance(m, (Conv,)) and m.conv.stride[0] == 2:
            prev += 1
        elif isinstance(m, RepConv) and (m.rbr_reparam.stride[0] if hasattr(m, 'rbr_reparam')
                                         else m.rbr_dense[0].stride[0]) == 2:
            prev += 1
        elif isinstance(m, (MP, ReOrg)):
            prev += 1
        elif isinstance(m, nn.Upsample):
            prev -= 1
        lv.append(prev)
    return lv


class Model(nn.Module):
    def __init__(self, cfg='yolov7.yaml', ch=3, nc=None, anchors=None):
        super().__init__()
        self.traced = False
        if isinstance(cfg, dict):
            self.yaml = cfg
        elif Path(str(cfg)).exists():
            import yaml
            self.yaml_file = Path(cfg).name
            with open(cfg) as f:
                self.yaml = yaml.load(f, Loader=yaml.SafeLoader)
        else:  # registered architecture name (the reference cfg files, regenerated by yv7.arch)
            from yv7.arch import get_cfg
            self.yaml_file = str(cfg)
            self.yaml = get_cfg(str(cfg))
        ch = self.yaml['ch'] = self.yaml.get('ch', ch)
        if nc and nc != self.yaml['nc']:
            logger.info(f"Overriding model.yaml nc={self.yaml['nc']} with nc={nc}")
            self.yaml['nc'] = nc
        if anchors:
            self.yaml['anchors'] = round(anchors)
        self.model, self.save = parse_model(deepcopy(self.yaml), ch=[ch])
        self.names = [str(i) for i in range(self.yaml['nc'])]
        m = self.model[-1]
        if isinstance(m, Detect):
            lv = _levels(self.model)
            srcs = m.f[:m.nl]
            m.stride = torch.tensor([float(2 ** lv[j]) for j in srcs])  # == 256 / H_out of the probe
            check_anchor_order(m)
            m.anchors /= m.stride.view(-1, 1, 1)
            self.stride = m.stride
            self._initialize_biases()
        initialize_weights(self)
        self._plans = {}
        self.info()

    # ------------------------------------------------------------------ reference API

    def forward(self, x, augment=False, profile=False):
        if augment:  # test-time augmentation (yolo.py:582-597); each pass is a full plan forward
            img_size = x.shape[-2:]
            s = [1, 0.83, 0.67]
            f = [None, 3, None]
            y = []
            for si, fi in zip(s, f):
                xi = scale_img(x.flip(fi) if fi else x, si, gs=int(self.stride.max()))
                yi = self.forward_once(xi)[0]
                yi[..., :4] /= si
                if fi == 2:
                    yi[..., 1] = img_size[0] - yi[..., 1]
                elif fi == 3:
                    yi[..., 0] = img_size[1] - yi[..., 0]
                y.append(yi)
            return torch.cat(y, 1), None
        return self.forward_once(x, profile)

    def forward_once(self, x, profile=False):
        if not (isinstance(x, torch.Tensor) and x.is_cuda):
            raise RuntimeError('models.yolo.Model runs on a ROCm (MI355X) device via libyv7; move the model and '
                               'input to cuda (the CPU reference lives in oracle/ and is test-only)')
        plan = self._plan(x.device)
        z, xs = plan.forward(x)
        return z, xs

    def _initialize_biases(self, cf=None):  # yolo.py:633-641
        m = self.model[-1]
        for mi, s in zip(m.m, m.stride):
            b = mi.bias.view(m.na, -1)
            b.data[:, 4] += math.log(8 / (640 / s) ** 2)
            b.data[:, 5:] += math.log(0.6 / (m.nc - 0.99)) if cf is None else torch.log(cf / cf.sum())
            mi.bias = torch.nn.Parameter(b.view(-1), requires_grad=True)

    def fuse(self):  # yolo.py:693-710
        print('Fusing layers... ')
        for m in self.model.modules():
            if isinstance(m, RepConv):
                m.fuse_repvgg_block()
            elif type(m) is Conv and hasattr(m, 'bn'):
                m.fuse()
            elif isinstance(m, (IDetect, IAuxDetect)) and hasattr(m, 'ia'):
                m.fuse()
        self._plans = {}
        self.info()
        return self

    def info(self, verbose=False, img_size=640):
        model_info(self, verbose, img_size)

    # ------------------------------------------------------------------ plan management

    def _apply(self, fn, *args, **kwargs):  # .half() / .float() / .to() / .cuda() invalidate compiled plans
        self._plans = {}
        return super()._apply(fn, *args, **kwargs)

    def load_state_dict(self, *args, **kwargs):
        self._plans = {}
        return super().load_state_dict(*args, **kwargs)

    def fp8(self, calib=None):
        """BASELINE configs[4]: half() with the 1x1 convs on OCP e4m3 weights and activations (the
        block-scaled fp8 MFMA); `calib`: [B,3,H,W] frames in [0,1] that set the activation scales
        (default: seeded synthetic frames) — yv7.runtime.Plan.fp8_from_model.  .float() leaves it."""
        self.half()
        self._fp8 = (calib,)
        self._plans = {}
        return self

    def _plan(self, device):
        dtype = next(self.parameters()).dtype
        fp8 = getattr(self, '_fp8', None) if dtype == torch.float16 else None
        key = (str(device), 'fp8' if fp8 else dtype)
        p = self._plans.get(key)
        if p is None:
            from yv7.runtime import Plan
            p = Plan.from_model(self, device=device, dtype='fp8' if fp8 else dtype, calib=fp8[0] if fp8 else None)
            self._plans[key] = p
        return p

    def plan(self, device=None, dtype=None):
        """The compiled libyv7 plan for this model (compiled on first use)."""
        device = torch.device(device) if device is not None else next(self.parameters()).device
        if dtype is not None and dtype != next(self.parameters()).dtype:
            from yv7.runtime import Plan
            return Plan.from_model(self, device=device, dtype=dtype)
        return self._plan(device)
