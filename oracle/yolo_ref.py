"""TEST INFRASTRUCTURE ONLY — CPU restatement of the reference YOLOv7 inference path (fp32, NCHW).

See oracle/__init__.py for who may import this and for the parity-pinning status.

This file restates, from the reference sources read as text (never imported or executed):
  * parse_model                 models/yolo.py:736-813 (+ make_divisible utils/general.py:177-179,
                                autopad models/common.py:23-27)
  * stride / anchor setup       models/yolo.py:542-548, utils/autoanchor.py:12-20
  * BN folding                  utils/torch_utils.py:181-201 (Conv), models/common.py:561-643 (RepConv)
  * IDetect implicit folding    models/yolo.py:178-190 (also IAuxDetect 411-423)
  * forward_once                models/yolo.py:601-631
  * layer forwards              Conv.fuseforward common.py:110-111, RepConv deploy common.py:498-500,
                                SPPCSPC common.py:276-280, MP 30-36, SP 39-45, ReOrg 48-53, Concat 56-62
  * Detect decode               models/yolo.py:42-63 (== IDetect.fuseforward 140-160)
  * test-time augmentation      models/yolo.py:582-597 (+ scale_img utils/torch_utils.py:247-257)
  * Ensemble                    models/experimental.py:69-81
It is written as plain functions over a layer table and a reference-keyed state_dict, so the
same synthetic weights can be fed to the product (models.yolo.Model.load_state_dict) and here.
"""
from __future__ import annotations

import math
import re
from dataclasses import dataclass, field

import torch
import torch.nn.functional as F

BN_EPS = 1e-3  # initialize_weights sets eps=1e-3 on every BatchNorm2d (utils/torch_utils.py:144-153)


def make_divisible(x, divisor):  # utils/general.py:177-179
    return math.ceil(x / divisor) * divisor


def autopad(k, p=None):  # models/common.py:23-27
    return k // 2 if p is None else p


_LEAKY = re.compile(r'nn\.LeakyReLU\(\s*([-+0-9.eE]+)\s*\)')


def _eval_arg(a, nc, anchors):
    """Stand-in for the `eval(a)` of string args in parse_model (models/yolo.py:745-749)."""
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
    m = _LEAKY.fullmatch(a)
    if m:
        return ('leaky', float(m.group(1)))
    if a == 'nn.SiLU()':
        return ('silu',)
    if a == 'nn.Identity()':
        return ('none',)
    return a  # e.g. 'nearest' stays a string, exactly as the bare eval failure leaves it


@dataclass
class Layer:
    i: int
    f: object
    type: str
    c1: object
    c2: int
    p: dict = field(default_factory=dict)


@dataclass
class Net:
    layers: list
    save: list
    nc: int
    na: int
    no: int
    nl: int
    anchors: list
    stride: list = None
    anchor_grid: torch.Tensor = None  # [nl, na, 2] pixels


def _act_of(a):
    if a is True or a is None:
        return ('silu',)
    if a is False:
        return ('none',)
    return a


def parse(d: dict, ch_in: int = 3) -> Net:
    """Restates parse_model (models/yolo.py:736-813) for the module subset of the yolov7 family."""
    anchors, nc, gd, gw = d['anchors'], d['nc'], d['depth_multiple'], d['width_multiple']
    na = (len(anchors[0]) // 2) if isinstance(anchors, list) else anchors
    no = na * (nc + 5)
    layers, save, ch = [], [], [ch_in]
    c2 = ch_in
    for i, (f, n, m, args) in enumerate(d['backbone'] + d['head']):
        args = [_eval_arg(a, nc, anchors) for a in args]
        if n > 1:
            n = max(round(n * gd), 1)
        if n != 1:
            raise NotImplementedError('repeated modules are not used by the yolov7 family cfgs')
        p = {}
        if m in ('Conv', 'RepConv', 'SPPCSPC'):
            c1, c2 = ch[f], args[0]
            if c2 != no:
                c2 = make_divisible(c2 * gw, 8)
            if m == 'SPPCSPC':
                p['c_'] = int(2 * c2 * 0.5)  # common.py:266 (e=0.5)
                p['pools'] = (5, 9, 13)
            else:
                k = args[1] if len(args) > 1 else (3 if m == 'RepConv' else 1)
                s = args[2] if len(args) > 2 else 1
                pad = autopad(k, args[3] if len(args) > 3 else None)
                g = args[4] if len(args) > 4 else 1
                if g != 1:
                    raise NotImplementedError('grouped conv')
                act = _act_of(args[5] if len(args) > 5 else True)
                p.update(k=k, s=s, pad=pad, act=act)
        elif m == 'Concat':
            c1, c2 = [ch[x] for x in f], sum(ch[x] for x in f)
        elif m in ('Detect', 'IDetect', 'IAuxDetect'):
            c1, c2 = [ch[x] for x in f], 0
        elif m == 'ReOrg':
            c1, c2 = ch[f], ch[f] * 4
        elif m == 'MP':
            c1 = c2 = ch[f]
            p['k'] = args[0] if args else 2
        elif m == 'SP':
            c1 = c2 = ch[f]
            p['k'] = args[0] if args else 3
            p['s'] = args[1] if len(args) > 1 else 1
        elif m == 'nn.Upsample':
            c1 = c2 = ch[f]
            p['scale'] = args[1]
            p['mode'] = args[2]
        else:
            raise NotImplementedError(f'module {m} is outside the yolov7-family hot path')
        layers.append(Layer(i, f, m, c1, c2, p))
        save.extend(x % i for x in ([f] if isinstance(f, int) else f) if x != -1)
        if i == 0:
            ch = []
        ch.append(c2)
    net = Net(layers, sorted(save), nc, na, nc + 5, len(anchors), anchors)
    _setup_strides(net)
    return net


def _levels(net: Net):
    """Spatial downsampling factor (log2) of every layer output (what the 256x256 probe forward measures)."""
    lv = []
    for L in net.layers:
        src = L.f if isinstance(L.f, int) else L.f[0]
        prev = 0 if L.i == 0 else (lv[-1] if src == -1 else lv[src])
        t = L.type
        if t in ('Conv', 'RepConv'):
            v = prev + (1 if L.p['s'] == 2 else 0)
        elif t in ('MP', 'ReOrg'):
            v = prev + 1
        elif t == 'nn.Upsample':
            v = prev - 1
        else:
            v = prev
        lv.append(v)
    return lv


def _setup_strides(net: Net):
    """models/yolo.py:542-548: stride = 256 / H_out of a 256x256 probe; check_anchor_order (autoanchor.py:12-20)."""
    lv = _levels(net)
    det = net.layers[-1]
    srcs = det.f[:net.nl]
    net.stride = [float(2 ** lv[j]) for j in srcs]
    ag = torch.tensor(net.anchors, dtype=torch.float32).view(net.nl, -1, 2)
    a = ag.prod(-1).view(-1)
    da = a[-1] - a[0]
    ds = net.stride[-1] - net.stride[0]
    sign_ds = 0.0 if ds == 0 else math.copysign(1.0, ds)
    if float(da.sign()) != sign_ds:  # 'Reversing anchor order'
        ag = ag.flip(0)
    net.anchor_grid = ag.clone()


# ---------------------------------------------------------------- folding (attempt_load -> fuse)

def fuse_conv_and_bn(w, gamma, beta, mean, var, eps=BN_EPS):
    """utils/torch_utils.py:181-201 (conv without bias)."""
    co = w.shape[0]
    w_bn = torch.diag(gamma.div(torch.sqrt(eps + var)))
    wf = torch.mm(w_bn, w.clone().view(co, -1)).view(w.shape)
    b_conv = torch.zeros(co, dtype=w.dtype)
    b_bn = beta - gamma.mul(mean).div(torch.sqrt(var + eps))
    bf = torch.mm(w_bn, b_conv.reshape(-1, 1)).reshape(-1) + b_bn
    return wf, bf


def _repconv_branch(w, gamma, beta, mean, var, eps=BN_EPS):
    """RepConv.fuse_conv_bn (models/common.py:561-582)."""
    std = (var + eps).sqrt()
    b = beta - mean * gamma / std
    t = (gamma / std).reshape(-1, 1, 1, 1)
    return w * t, b


def _bn(sd, prefix):
    return (sd[prefix + '.weight'].float(), sd[prefix + '.bias'].float(),
            sd[prefix + '.running_mean'].float(), sd[prefix + '.running_var'].float())


def fuse(net: Net, sd: dict) -> dict:
    """Fold a reference-keyed state_dict into per-conv (W, b) fp32 tensors (Model.fuse, yolo.py:693-710).

    Keys follow the reference module tree: model.{i}.conv.weight + model.{i}.bn.*,
    model.{i}.rbr_dense.{0,1}.* / rbr_1x1.{0,1}.*, model.{i}.cv{1..7}.*, model.{i}.m.{j}.*, ia/im.
    """
    sd = {k: v.float() if v.is_floating_point() else v for k, v in sd.items()}
    out = {}
    for L in net.layers:
        pre = f'model.{L.i}'
        if L.type == 'Conv':
            out[L.i] = fuse_conv_and_bn(sd[pre + '.conv.weight'], *_bn(sd, pre + '.bn'))
        elif L.type == 'RepConv':
            w3, b3 = _repconv_branch(sd[pre + '.rbr_dense.0.weight'], *_bn(sd, pre + '.rbr_dense.1'))
            w1, b1 = _repconv_branch(sd[pre + '.rbr_1x1.0.weight'], *_bn(sd, pre + '.rbr_1x1.1'))
            # identity branch is None because c1 != c2 in every yolov7 RepConv (common.py:486)
            if L.c1 == L.c2 and L.p['s'] == 1:
                raise NotImplementedError('RepConv identity branch')
            w1p = F.pad(w1, [1, 1, 1, 1])
            out[L.i] = (w3 + w1p + torch.zeros_like(w1p), b3 + b1 + torch.zeros_like(b1))
        elif L.type == 'SPPCSPC':
            out[L.i] = {j: fuse_conv_and_bn(sd[f'{pre}.cv{j}.conv.weight'], *_bn(sd, f'{pre}.cv{j}.bn'))
                        for j in range(1, 8)}
        elif L.type in ('Detect', 'IDetect', 'IAuxDetect'):
            heads = []
            for j in range(net.nl):
                w = sd[f'{pre}.m.{j}.weight'].clone()
                b = sd[f'{pre}.m.{j}.bias'].clone()
                if L.type != 'Detect':  # IDetect.fuse (yolo.py:178-190)
                    c1, c2 = w.shape[:2]
                    ia = sd[f'{pre}.ia.{j}.implicit']
                    b += torch.matmul(w.reshape(c1, c2), ia.reshape(ia.shape[1], ia.shape[0])).squeeze(1)
                    im = sd[f'{pre}.im.{j}.implicit']
                    b *= im.reshape(im.shape[1])
                    w *= im.transpose(0, 1)
                heads.append((w, b))
            out[L.i] = heads
    return out


# ---------------------------------------------------------------- forward (NCHW fp32)

def _act(x, act):
    if act[0] == 'silu':
        return F.silu(x)
    if act[0] == 'leaky':
        return F.leaky_relu(x, act[1])
    return x


def fp8_e4m3(t):
    """Round to OCP e4m3 (float8_e4m3fn: round to nearest even) with saturation at +-448, back to float."""
    return t.clamp(-448.0, 448.0).to(torch.float8_e4m3fn).to(t.dtype)


def fp8_fused(fused: dict, entries) -> dict:
    """The fp8 plan's arithmetic (BASELINE configs[4]) as an emulation of the fused network: for every
    ((layer, SPPCSPC cv index or None), xscale) in `entries`, that 1x1 conv gets per-output-channel e4m3
    weights (wscale = amax / 448, W ~ e4m3(W / wscale) * wscale) and its input is rounded to e4m3 on the
    per-tensor scale xscale (x ~ e4m3(x / xscale) * xscale) — see _conv.  Test infrastructure only."""
    out = {k: (dict(v) if isinstance(v, dict) else v) for k, v in fused.items()}
    for (layer, sub), xs in entries:
        w, b = (out[layer] if sub is None else out[layer][sub])[:2]
        wk = w.reshape(w.shape[0], -1)
        amax = wk.abs().amax(1)
        ws = torch.where(amax > 0, amax / 448.0, torch.ones_like(amax))
        wq = (fp8_e4m3(wk / ws[:, None]) * ws[:, None]).reshape(w.shape)
        if sub is None:
            out[layer] = (wq, b, float(xs))
        else:
            out[layer][sub] = (wq, b, float(xs))
    return out


def half_weights(fused: dict) -> dict:
    """The libyv7 fp16 plan's parameter storage: fp16 weights, fp32 biases; fp8 entries unchanged."""
    def r(v):
        if isinstance(v, tuple):
            return v if len(v) == 3 else (v[0].half().float(), v[1])
        if isinstance(v, dict):
            return {j: r(t) for j, t in v.items()}
        return [r(t) for t in v]
    return {k: r(v) for k, v in fused.items()}


def _conv(x, wb, k, s, pad, act):
    if len(wb) == 3:   # fp8 emulation entry (fp8_fused): e4m3 input on the per-tensor scale
        x = fp8_e4m3(x / wb[2]) * wb[2]
    return _act(F.conv2d(x, wb[0], wb[1], s, pad), act)


def _make_grid(nx, ny):  # models/yolo.py:79-82
    yv, xv = torch.meshgrid([torch.arange(ny), torch.arange(nx)], indexing='ij')
    return torch.stack((xv, yv), 2).view((1, 1, ny, nx, 2)).float()


def detect_decode(net: Net, raw: list):
    """Detect.forward inference branch (models/yolo.py:46-63) given the per-level conv outputs."""
    z, xs = [], []
    for i, v in enumerate(raw):
        bs, _, ny, nx = v.shape
        v = v.view(bs, net.na, net.no, ny, nx).permute(0, 1, 3, 4, 2).contiguous()
        xs.append(v)
        grid = _make_grid(nx, ny)
        ag = net.anchor_grid[i].view(1, net.na, 1, 1, 2)
        y = v.sigmoid()
        y[..., 0:2] = (y[..., 0:2] * 2. - 0.5 + grid) * net.stride[i]
        y[..., 2:4] = (y[..., 2:4] * 2) ** 2 * ag
        z.append(y.view(bs, -1, net.no))
    return torch.cat(z, 1), xs


def _half_round(v):
    if isinstance(v, tuple) and len(v) == 3:   # fp8 entry: e4m3 weights with fp32 scales, fp32 bias
        return v
    if isinstance(v, tuple):
        return (v[0].half().float(), v[1].half().float())
    if isinstance(v, dict):
        return {j: _half_round(t) for j, t in v.items()}
    return [_half_round(t) for t in v]


def forward(net: Net, fused: dict, x: torch.Tensor, return_all=False, half_storage=False):
    """forward_once (models/yolo.py:601-631) on the fused (deploy) network; returns (z, xs).

    half_storage=True emulates the reference's GPU half() path (detect.py:48-49,101): weights, the
    input and every layer output rounded to fp16, arithmetic (conv accumulation) in fp32."""
    y = []
    outs = {}
    if half_storage:
        fused = {k: _half_round(v) for k, v in fused.items()}
        x = x.half().float()
    for L in net.layers:
        if L.f != -1:
            x = y[L.f] if isinstance(L.f, int) else [x if j == -1 else y[j] for j in L.f]
        t = L.type
        if t in ('Conv', 'RepConv'):
            x = _conv(x, fused[L.i], L.p['k'], L.p['s'], L.p['pad'], L.p['act'])
        elif t == 'SPPCSPC':
            cv = fused[L.i]
            silu = ('silu',)
            r = (lambda t: t.half().float()) if half_storage else (lambda t: t)
            x1 = r(_conv(r(_conv(r(_conv(x, cv[1], 1, 1, 0, silu)), cv[3], 3, 1, 1, silu)), cv[4], 1, 1, 0, silu))
            cat = torch.cat([x1] + [F.max_pool2d(x1, k, 1, k // 2) for k in L.p['pools']], 1)
            y1 = r(_conv(r(_conv(cat, cv[5], 1, 1, 0, silu)), cv[6], 3, 1, 1, silu))
            y2 = r(_conv(x, cv[2], 1, 1, 0, silu))
            x = _conv(torch.cat((y1, y2), dim=1), cv[7], 1, 1, 0, silu)
        elif t == 'MP':
            x = F.max_pool2d(x, L.p['k'], L.p['k'])
        elif t == 'SP':
            x = F.max_pool2d(x, L.p['k'], L.p['s'], L.p['k'] // 2)
        elif t == 'Concat':
            x = torch.cat(x, 1)
        elif t == 'nn.Upsample':
            x = F.interpolate(x, scale_factor=float(L.p['scale']), mode=L.p['mode'])
        elif t == 'ReOrg':
            x = torch.cat([x[..., ::2, ::2], x[..., 1::2, ::2], x[..., ::2, 1::2], x[..., 1::2, 1::2]], 1)
        elif t in ('Detect', 'IDetect', 'IAuxDetect'):
            raw = [F.conv2d(x[j], fused[L.i][j][0], fused[L.i][j][1]) for j in range(net.nl)]
            x = detect_decode(net, raw)
        else:
            raise NotImplementedError(t)
        if half_storage and isinstance(x, torch.Tensor):
            x = x.half().float()
        if return_all:
            outs[L.i] = x
        y.append(x if L.i in net.save else None)
    return (x, outs) if return_all else x


def forward64(net: Net, fused: dict, x: torch.Tensor):
    """The same restatement evaluated in float64 — the accuracy yardstick for fp32 parity tolerances:
    a different fp32 summation order (another BLAS, ISA or thread count) legitimately moves the
    reference's own fp32 z by about |z32 - z64|."""
    def d(v):
        if isinstance(v, tuple):
            return (v[0].double(), v[1].double()) + tuple(v[2:])
        if isinstance(v, dict):
            return {j: d(t) for j, t in v.items()}
        return [d(t) for t in v]

    f64 = {k: d(v) for k, v in fused.items()}
    ag = net.anchor_grid
    net.anchor_grid = ag.double()
    try:
        z, xs = forward(net, f64, x.double())
    finally:
        net.anchor_grid = ag
    return z, xs


def scale_img(img, ratio=1.0, same_shape=False, gs=32):  # utils/torch_utils.py:247-257
    if ratio == 1.0:
        return img
    h, w = img.shape[2:]
    s = (int(h * ratio), int(w * ratio))
    img = F.interpolate(img, size=s, mode='bilinear', align_corners=False)
    if not same_shape:
        h, w = [math.ceil(x * ratio / gs) * gs for x in (h, w)]
    return F.pad(img, [0, w - s[1], 0, h - s[0]], value=0.447)


def forward_augment(net: Net, fused: dict, x: torch.Tensor, f64=False):
    """Model.forward(augment=True) (models/yolo.py:582-597): three passes (scale 1, 0.83 with an lr
    flip, 0.67), de-scaled / de-flipped boxes, rows concatenated.  f64: the float64 yardstick (the
    input resizes in float64 too)."""
    img_size = x.shape[-2:]
    gs = int(max(net.stride))
    if f64:
        x = x.double()
    y = []
    for si, fi in zip([1, 0.83, 0.67], [None, 3, None]):
        xi = scale_img(x.flip(fi) if fi else x, si, gs=gs)
        yi = (forward64(net, fused, xi) if f64 else forward(net, fused, xi))[0]
        yi[..., :4] /= si
        if fi == 2:
            yi[..., 1] = img_size[0] - yi[..., 1]
        elif fi == 3:
            yi[..., 0] = img_size[1] - yi[..., 0]
        y.append(yi)
    return torch.cat(y, 1)


def ensemble_forward(members, x, f64=False):
    """Ensemble.forward (models/experimental.py:74-81): each member's z, concatenated on the row axis
    ("nms ensemble").  members: [(net, fused), ...]."""
    fw = forward64 if f64 else forward
    return torch.cat([fw(net, fused, x.double() if f64 else x)[0] for net, fused in members], 1)
