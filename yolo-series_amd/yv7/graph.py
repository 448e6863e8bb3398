"""Graph compiler: a models.yolo.Model -> the flat libyv7 plan (NHWC tensors, ops, packed weights).

Walks the parsed layer list the way forward_once does (models/yolo.py:601-631) and emits one op per
kernel launch:
  Conv / RepConv           -> CONV (BN / RepVGG branches folded in fp32 first, Model.fuse arithmetic)
  SPPCSPC                  -> 7 CONV + 3 MAXPOOL(5) cascaded (5, 5∘5 = 9, 5∘5∘5 = 13: max is associative and
                              the -inf padding clips identically), concats as channel slices (common.py:276-280)
  MP / SP                  -> MAXPOOL(k, k, 0) / MAXPOOL(k, s, k//2)
  nn.Upsample(x2 nearest)  -> UPSAMPLE
  Concat                   -> nothing: producers write their channel slice of the concat tensor directly;
                              an input that already lives in another concat (or is the input image) gets a COPY
  ReOrg at layer 0         -> fused into the INPUT packing op (space-to-depth while converting NCHW -> NHWC);
                              fp16 plans of the w6 front end: ReOrg + its two convs as one STEM op
  Detect / IDetect / IAuxDetect -> one DETECT op per level (1x1 conv + bias + sigmoid + decode -> z)
Layers whose outputs never reach the head (IAuxDetect's auxiliary branch) are not emitted.

Weights: each conv's fused W [cout, cin, k, k] becomes [cout_pad32][k][k][cin_pad] (K padded to 64) in the
plan dtype, bias fp32 [cout_pad32]; every blob entry 256-byte aligned.
"""
from __future__ import annotations

import os
from dataclasses import dataclass, field

import torch
import torch.nn as nn

from models.common import MP, SP, SPPCSPC, Concat, Conv, ReOrg, RepConv
from models.yolo import Detect
from yv7 import _lib as L


@dataclass
class Graph:
    dtype: int
    tensors: list = field(default_factory=list)   # [channels, shift]
    ops: list = field(default_factory=list)       # dicts of OpDesc fields
    blobs: list = field(default_factory=list)     # (offset, uint8 tensor)
    nbytes: int = 0
    nl: int = 0
    na: int = 0
    no: int = 0
    stride: list = None
    anchor_grid: list = None
    max_shift: int = 0
    layer_tensor: dict = field(default_factory=dict)   # layer i -> (tensor, coff, channels) for debugging
    flops_per_pixel: float = 0.0                       # conv MACs*2 per input pixel (for roofline accounting)

    def add_tensor(self, channels, shift):
        self.tensors.append([channels, shift])
        return len(self.tensors) - 1

    def add_blob(self, t: torch.Tensor):
        b = t.contiguous().view(torch.uint8).reshape(-1).cpu()
        off = self.nbytes
        self.blobs.append((off, b))
        self.nbytes = (off + b.numel() + 255) // 256 * 256
        return off

    def weight_blob(self):
        out = torch.zeros(max(self.nbytes, 1), dtype=torch.uint8)
        for off, b in self.blobs:
            out[off:off + b.numel()] = b
        return out


def _vec(dtype):
    return 8 if dtype == L.DT_F16 else 4


def _rup(x, m):
    return (x + m - 1) // m * m


def _act_code(act):
    if isinstance(act, nn.SiLU):
        return L.ACT_SILU
    if isinstance(act, nn.LeakyReLU):
        if abs(act.negative_slope - 0.1) > 1e-12:
            raise NotImplementedError('LeakyReLU slope other than 0.1')
        return L.ACT_LEAKY
    if isinstance(act, nn.Identity):
        return L.ACT_NONE
    raise NotImplementedError(f'activation {type(act).__name__}')


def _pack_conv(g: Graph, w: torch.Tensor, b: torch.Tensor, cin_pad: int):
    """fp32 W [cout, cin, k, k] -> [cout_pad32][k*k*cin_pad -> K padded to 64] (plan dtype); bias fp32."""
    cout, cin, k, _ = w.shape
    tdt = torch.float16 if g.dtype == L.DT_F16 else torch.float32
    wk = w.permute(0, 2, 3, 1)  # [cout, k, k, cin]
    if cin_pad != cin:
        wk = torch.nn.functional.pad(wk, [0, cin_pad - cin])
    wk = wk.reshape(cout, -1)
    kpad = _rup(k * k * cin_pad, 64)
    cpad = _rup(cout, 32)
    wp = torch.zeros(cpad, kpad, dtype=torch.float32)
    wp[:cout, :wk.shape[1]] = wk
    bp = torch.zeros(cpad, dtype=torch.float32)
    bp[:cout] = b
    w_off = g.add_blob(wp.to(tdt))
    b_off = g.add_blob(bp)
    return w_off, b_off


def _pack_conv_f8(g: Graph, w: torch.Tensor, b: torch.Tensor, cin_pad: int):
    """fp32 1x1 W [cout, cin, 1, 1] -> OCP e4m3 [cout_pad32][cin padded to 128] with per-output-channel
    scales wscale = amax / 448 (W ~ e4m3(W / wscale) * wscale, round to nearest even); bias fp32."""
    cout, cin = w.shape[:2]
    wk = w.reshape(cout, cin).float()
    ws = fp8_weight_scales(wk)
    q = (wk / ws[:, None]).clamp(-448.0, 448.0).to(torch.float8_e4m3fn).view(torch.uint8)
    kp, cpad = _rup(cin_pad, 128), _rup(cout, 32)
    wp = torch.zeros(cpad, kp, dtype=torch.uint8)
    wp[:cout, :cin] = q
    bp = torch.zeros(cpad, dtype=torch.float32)
    bp[:cout] = b
    sp = torch.zeros(cpad, dtype=torch.float32)
    sp[:cout] = ws
    return g.add_blob(wp), g.add_blob(bp), g.add_blob(sp)


def fp8_weight_scales(wk: torch.Tensor) -> torch.Tensor:
    """Per-output-channel e4m3 scales of a [cout, K] weight matrix: amax / 448 (1 for an all-zero row)."""
    amax = wk.abs().amax(1)
    return torch.where(amax > 0, amax / 448.0, torch.ones_like(amax))


def fp8_eligible(g: Graph, o: dict) -> bool:
    """CONV ops an fp8 plan runs in e4m3: 1x1 stride-1 convs of an fp16 plan (the Detect head stays fp16)."""
    return (g.dtype == L.DT_F16 and o['kind'] == L.OP_CONV and o['k'] == 1 and o['s'] == 1 and o['pad'] == 0
            and o['cout'] <= 1024)


# fp8 pays only on wide layers: measured per op on MI355X (bs32 640 yolov7, scripts/op_profile.py
# --dtype fp8 vs f16), cout >= 512 gains 1-41 us per layer (1024->1024 @40: 156 -> 114 us) while every
# cout <= 256 layer loses 3-82 us — their time is the SiLU epilogue and the extra quantize pass, not
# the MFMA, so the 2x fp8 MFMA rate cannot win it back.
FP8_MIN_COUT = 512


def fp8_candidates(g: Graph, min_cout: int = FP8_MIN_COUT):
    """Op indices of `g` that compile_model(..., fp8={index: xscale}) marks FP8 in an fp8 plan: the
    fp8-eligible ops with at least `min_cout` output channels (min_cout=0: every eligible op)."""
    return [i for i, o in enumerate(g.ops) if fp8_eligible(g, o) and o['cout'] >= min_cout]


def _live_layers(layers, nl):
    """Layers whose output reaches the Detect head (drops IAuxDetect's auxiliary branch)."""
    n = len(layers)
    need = [False] * n
    need[n - 1] = True
    for i in range(n - 1, -1, -1):
        if not need[i]:
            continue
        m = layers[i]
        srcs = [m.f] if isinstance(m.f, int) else list(m.f)
        if isinstance(m, Detect):
            srcs = srcs[:nl]
        for j in srcs:
            jj = i + j if j < 0 else j
            if jj >= 0:
                need[jj] = True
    return need


def _stem_candidate(layers, dtype):
    """Layers 0-1 = Conv(3->32, 3x3, s1|s2) -> Conv(32->64, 3x3, s2) with layer 0 read only by layer 1:
    the yolov7 / yolov7-tiny stems, fused into one fp16 op (csrc/stem.hip).  YV7_NO_STEM=1 disables."""
    if dtype != L.DT_F16 or os.environ.get('YV7_NO_STEM') == '1' or len(layers) < 3:
        return None
    l0, l1 = layers[0], layers[1]
    if not (type(l0) is Conv and type(l1) is Conv and l1.f == -1):
        return None
    c0, c1 = l0.conv, l1.conv
    if not (c0.in_channels == 3 and c0.out_channels == 32 and c0.kernel_size[0] == 3 and c0.stride[0] in (1, 2)
            and c0.padding[0] == 1 and c1.out_channels == 64 and c1.kernel_size[0] == 3 and c1.stride[0] == 2
            and c1.padding[0] == 1 and c0.groups == 1 and c1.groups == 1 and _act_code(l0.act) == _act_code(l1.act)):
        return None
    for m in layers[2:]:
        srcs = [m.f] if isinstance(m.f, int) else list(m.f)
        if any((m.i + j if j < 0 else j) == 0 for j in srcs):
            return None
    return True


def _reorg_stem_candidate(layers, dtype):
    """Layers 0-2 = ReOrg -> Conv(12->64, 3x3, s1) -> Conv(64->128, 3x3, s2), layers 0 and 1 read only by
    their successor: the yolov7-w6 front end (cfg/deploy/yolov7-w6.yaml:14-16), fused into one fp16 op
    (csrc/stem.hip, stem_reorg_kernel).  YV7_NO_STEM=1 disables."""
    if dtype != L.DT_F16 or os.environ.get('YV7_NO_STEM') == '1' or len(layers) < 4:
        return None
    l0, l1, l2 = layers[0], layers[1], layers[2]
    if not (isinstance(l0, ReOrg) and type(l1) is Conv and type(l2) is Conv and l1.f == -1 and l2.f == -1):
        return None
    c1, c2 = l1.conv, l2.conv
    if not (c1.in_channels == 12 and c1.out_channels == 64 and c1.kernel_size[0] == 3 and c1.stride[0] == 1
            and c1.padding[0] == 1 and c2.out_channels == 128 and c2.kernel_size[0] == 3 and c2.stride[0] == 2
            and c2.padding[0] == 1 and c1.groups == 1 and c2.groups == 1 and _act_code(l1.act) == _act_code(l2.act)):
        return None
    for m in layers[3:]:
        srcs = [m.f] if isinstance(m.f, int) else list(m.f)
        if any((m.i + j if j < 0 else j) in (0, 1) for j in srcs):
            return None
    return True


def compile_model(model, dtype: int, fp8=None) -> Graph:
    """fp8: {op index: activation scale} — those ops (fp8_candidates of the same model and dtype) are
    packed as YV7_WFMT_FP8 (e4m3 weights + scales); the op list is otherwise identical."""
    layers = list(model.model)
    det = layers[-1]
    if not isinstance(det, Detect):
        raise NotImplementedError('the last layer must be a Detect / IDetect / IAuxDetect head')
    V = _vec(dtype)
    g = Graph(dtype=dtype, nl=det.nl, na=det.na, no=det.no)
    g.stride = [float(s) for s in det.stride]
    g.anchor_grid = det.anchor_grid.detach().float().cpu().reshape(-1).tolist()
    live = _live_layers(layers, det.nl)

    def absf(i, f):
        return i + f if f < 0 else f

    # ---- pass 1: output channels and spatial shift of every layer
    ch, shift = {}, {}
    c_in, s_in = model.yaml.get('ch', 3), 0
    for m in layers:
        i = m.i
        srcs = [m.f] if isinstance(m.f, int) else list(m.f)
        prev = [absf(i, j) for j in srcs]
        pc = [c_in if j < 0 else ch[j] for j in prev]
        ps = [s_in if j < 0 else shift[j] for j in prev]
        if isinstance(m, Conv):
            ch[i], shift[i] = m.conv.out_channels, ps[0] + (1 if m.conv.stride[0] == 2 else 0)
        elif isinstance(m, RepConv):
            c = m.rbr_reparam if hasattr(m, 'rbr_reparam') else m.rbr_dense[0]
            ch[i], shift[i] = c.out_channels, ps[0] + (1 if c.stride[0] == 2 else 0)
        elif isinstance(m, SPPCSPC):
            ch[i], shift[i] = m.cv7.conv.out_channels, ps[0]
        elif isinstance(m, MP):
            ch[i], shift[i] = pc[0], ps[0] + 1
        elif isinstance(m, SP):
            ch[i], shift[i] = pc[0], ps[0]
        elif isinstance(m, nn.Upsample):
            if m.mode != 'nearest' or float(m.scale_factor) != 2.0:
                raise NotImplementedError('only nn.Upsample(scale_factor=2, mode="nearest")')
            ch[i], shift[i] = pc[0], ps[0] - 1
        elif isinstance(m, ReOrg):
            if i != 0:
                raise NotImplementedError('ReOrg is supported as the first layer (fused into input packing)')
            ch[i], shift[i] = pc[0] * 4, ps[0] + 1
        elif isinstance(m, Concat):
            if len(set(ps)) != 1:
                raise ValueError(f'layer {i}: concat of different resolutions')
            ch[i], shift[i] = sum(pc), ps[0]
        elif isinstance(m, Detect):
            ch[i], shift[i] = 0, 0
        else:
            raise NotImplementedError(f'layer {i}: {type(m).__name__}')
    g.max_shift = max(shift.values())

    # ---- tensor 0: the packed network input (INPUT op; ReOrg at layer 0 is fused into it)
    loc = {}        # layer -> (tensor, coff)
    reorg0 = isinstance(layers[0], ReOrg)
    if c_in != 3:
        raise NotImplementedError('the input packing op handles 3-channel images')
    in_c = 12 if reorg0 else 3
    stem = _stem_candidate(layers, dtype) if not reorg0 else _reorg_stem_candidate(layers, dtype)
    if stem is None:
        t_in = g.add_tensor(_rup(in_c, V), 1 if reorg0 else 0)
        g.ops.append(dict(kind=L.OP_INPUT, src=-1, dst=t_in, k=2 if reorg0 else 1, cout=in_c))
    else:  # layers 0-1 run as one fused op straight from the image; tensor 0 is an unused placeholder
        t_in = g.add_tensor(V, g.max_shift)
    if reorg0 and stem is None:
        loc[0] = (t_in, 0)

    # ---- pass 2: concat placement (producers write straight into the concat tensor)
    placeable = (Conv, RepConv, SPPCSPC, MP, SP, nn.Upsample)
    placed = set()
    for m in layers:
        if isinstance(m, Concat) and live[m.i]:
            t = g.add_tensor(_rup(ch[m.i], V), shift[m.i])
            loc[m.i] = (t, 0)
            off = 0
            for j in m.f:
                jj = absf(m.i, j)
                if jj >= 0 and jj not in loc and isinstance(layers[jj], placeable) and ch[jj] % V == 0 and off % V == 0:
                    loc[jj] = (t, off)
                    placed.add((jj, m.i))
                off += ch[jj] if jj >= 0 else c_in


    def src_of(i, j):
        jj = absf(i, j)
        if jj < 0:
            return t_in, 0, in_c
        t, off = loc[jj]
        return t, off, ch[jj]

    def out_of(i):
        if i not in loc:
            loc[i] = (g.add_tensor(_rup(ch[i], V), shift[i]), 0)
        return loc[i]

    def conv_op(src, dst, w, b, k, s, pad, act, tag):
        # weights are packed after the sibling-merge pass (_merge_siblings), so they ride along unpacked;
        # tag = (layer, SPPCSPC cv index or None) names the reference conv(s) an op computes
        (ts, so, cs), (td, do) = src, dst
        cin_pad = _rup(cs, V)
        if cin_pad != cs and g.tensors[ts][0] < so + cin_pad:
            raise ValueError('channel padding would read outside the source tensor')
        g.ops.append(dict(kind=L.OP_CONV, src=ts, src_coff=so, cin=cin_pad, dst=td, dst_coff=do, cout=w.shape[0],
                          k=k, s=s, pad=pad, act=act, _w=w, _b=b, layers=[tag]))

    for m in layers:
        i = m.i
        # the fused front end: layers [0, last) are folded into the stem op written at layer `last`
        last = (2 if reorg0 else 1) if stem is not None else -1
        if not live[i] or (reorg0 and i == 0) or i < last:
            continue
        if i == last:
            l0, l1 = layers[last - 1], layers[last]
            wa, ba = l0.fused_weight_bias()
            wb, bb = l1.fused_weight_bias()
            # reorg: conv A reads the 12-channel space-to-depth image, K = tap * 16 + ci
            wa_off, ba_off = _pack_conv(g, wa, ba, 16 if reorg0 else 3)
            wb_off, bb_off = _pack_conv(g, wb, bb, l1.conv.in_channels)
            td, do = out_of(last)
            g.ops.insert(0, dict(kind=L.OP_STEM, src=-1, cin=12 if reorg0 else 3, cout=l0.conv.out_channels, k=3,
                                 s=l0.conv.stride[0], pad=1, act=_act_code(l0.act), w_off=wa_off, b_off=ba_off,
                                 dst=td, dst_coff=do, cout2=l1.conv.out_channels, act2=_act_code(l1.act),
                                 w2_off=wb_off, b2_off=bb_off))
            continue
        if isinstance(m, (Conv, RepConv)):
            w, b = m.fused_weight_bias()
            c = m.conv if isinstance(m, Conv) else (m.rbr_reparam if hasattr(m, 'rbr_reparam') else m.rbr_dense[0])
            if c.groups != 1 or c.dilation[0] != 1:
                raise NotImplementedError('grouped / dilated conv')
            conv_op(src_of(i, m.f), out_of(i), w, b, c.kernel_size[0], c.stride[0], c.padding[0], _act_code(m.act),
                    (i, None))
        elif isinstance(m, SPPCSPC):
            src = src_of(i, m.f)
            c_ = m.cv1.conv.out_channels
            s = shift[i]
            t1 = g.add_tensor(_rup(c_, V), s)
            t3 = g.add_tensor(_rup(c_, V), s)
            cat1 = g.add_tensor(_rup(4 * c_, V), s)
            t5 = g.add_tensor(_rup(c_, V), s)
            cat2 = g.add_tensor(_rup(2 * c_, V), s)
            if c_ % V:
                raise NotImplementedError('SPPCSPC hidden width must be a multiple of the vector width')

            def cv(j, a, d):
                mod = getattr(m, f'cv{j}')
                w, b = mod.fused_weight_bias()
                k = mod.conv.kernel_size[0]
                conv_op(a, d, w, b, k, 1, k // 2, _act_code(mod.act), (i, j))

            cv(1, src, (t1, 0))
            cv(3, (t1, 0, c_), (t3, 0))
            cv(4, (t3, 0, c_), (cat1, 0))
            ks = [p.kernel_size for p in m.m]
            if ks == [5, 9, 13]:  # cascade: pool9 = pool5(pool5), pool13 = pool5(pool9)
                for q in range(3):
                    g.ops.append(dict(kind=L.OP_MAXPOOL, src=cat1, src_coff=q * c_, dst=cat1, dst_coff=(q + 1) * c_,
                                      cout=c_, k=5, s=1, pad=2))
            else:
                for q, k in enumerate(ks):
                    g.ops.append(dict(kind=L.OP_MAXPOOL, src=cat1, src_coff=0, dst=cat1, dst_coff=(q + 1) * c_,
                                      cout=c_, k=k, s=1, pad=k // 2))
            cv(5, (cat1, 0, 4 * c_), (t5, 0))
            cv(6, (t5, 0, c_), (cat2, 0))
            cv(2, src, (cat2, c_))
            cv(7, (cat2, 0, 2 * c_), out_of(i))
        elif isinstance(m, (MP, SP)):
            (ts, so, cs), (td, do) = src_of(i, m.f), out_of(i)
            p = m.m
            k = p.kernel_size if isinstance(p.kernel_size, int) else p.kernel_size[0]
            st = p.stride if isinstance(p.stride, int) else p.stride[0]
            pd = p.padding if isinstance(p.padding, int) else p.padding[0]
            g.ops.append(dict(kind=L.OP_MAXPOOL, src=ts, src_coff=so, dst=td, dst_coff=do, cout=cs, k=k, s=st, pad=pd,
                              layer=i))
        elif isinstance(m, nn.Upsample):
            (ts, so, cs), (td, do) = src_of(i, m.f), out_of(i)
            g.ops.append(dict(kind=L.OP_UPSAMPLE, src=ts, src_coff=so, dst=td, dst_coff=do, cout=cs))
        elif isinstance(m, Concat):
            t, _ = loc[i]
            off = 0
            for j in m.f:
                jj = absf(i, j)
                cs_ = ch[jj] if jj >= 0 else in_c
                if (jj, i) not in placed:
                    ts, so, cs = src_of(i, j)
                    if cs % V or off % V:
                        raise NotImplementedError('concat slice not a multiple of the vector width')
                    g.ops.append(dict(kind=L.OP_COPY, src=ts, src_coff=so, dst=t, dst_coff=off, cout=cs))
                off += cs_
        elif isinstance(m, Detect):
            for lvl in range(m.nl):
                ts, so, cs = src_of(i, m.f[lvl])
                w, b = m.head_weights(lvl)
                w_off, b_off = _pack_conv(g, w, b, _rup(cs, V))
                g.ops.append(dict(kind=L.OP_DETECT, src=ts, src_coff=so, cin=_rup(cs, V), dst=-1, cout=w.shape[0],
                                  k=1, s=1, pad=0, level=lvl, w_off=w_off, b_off=b_off))
    folded = _fold_pools(g) if dtype == L.DT_F16 and os.environ.get('YV7_NO_POOLFOLD') != '1' else []
    if os.environ.get('YV7_NO_MERGE') != '1':
        _merge_siblings(g)
        if os.environ.get('YV7_NO_TMERGE') != '1':
            _merge_sibling_tensors(g, loc)
    fp8 = fp8 or {}
    for idx, o in enumerate(g.ops):
        if '_w' in o:
            w, b = o.pop('_w'), o.pop('_b')
            if idx in fp8:
                if not fp8_eligible(g, o):
                    raise ValueError(f'op {idx} cannot run in fp8 (fp16 plans, 1x1 stride-1 convs only)')
                o['w_off'], o['b_off'], o['s_off'] = _pack_conv_f8(g, w, b, o['cin'])
                o['wfmt'], o['xscale'] = L.WFMT_FP8, float(fp8[idx])
            else:
                o['w_off'], o['b_off'] = _pack_conv(g, w, b, o['cin'])
    g.layer_tensor = {i: (loc[i][0], loc[i][1], ch[i]) for i in loc if i not in folded}
    return g


def _fold_pools(g: Graph):
    """MP (2x2 / stride-2 max, models/common.py:30-36) whose output only feeds one 1x1 conv of <= 512 input
    channels (yolov7: `[-1, 1, MP, []], [-1, 1, Conv, [c, 1, 1]]`) -> that conv reads the MP's input with
    pool = 2, s = 2: the max is taken in the conv's operand loads and the pooled tensor never reaches
    HBM.  Returns the folded MP layers (their outputs no longer exist as tensors)."""
    folded = []
    i = 0
    while i < len(g.ops):
        mp = g.ops[i]
        if not (mp['kind'] == L.OP_MAXPOOL and mp['k'] == 2 and mp['s'] == 2 and mp['pad'] == 0):
            i += 1
            continue
        t = mp['dst']
        readers = [j for j, o in enumerate(g.ops) if j != i and o.get('src', -1) == t]
        writers = [j for j, o in enumerate(g.ops) if j != i and _writes(o) and _writes(o)[0] == t]
        ok = len(readers) == 1 and not writers and readers[0] > i
        if ok:
            c = g.ops[readers[0]]
            ok = (c['kind'] == L.OP_CONV and '_w' in c and c['k'] == 1 and c['s'] == 1 and c['pad'] == 0 and
                  c['src_coff'] == mp['dst_coff'] and c['cin'] == mp['cout'] and c['cin'] % 64 == 0 and
                  c['cin'] <= 512)   # deep-K (1024) pairs run faster unfused (csrc/conv_f16.hip, pool dispatch)
        if not ok:
            i += 1
            continue
        c.update(src=mp['src'], src_coff=mp['src_coff'], s=2, pool=2)
        folded.append(mp.get('layer'))
        del g.ops[i]
    return folded


def _overlaps(t, lo, n, t2, lo2, n2):
    return t == t2 and lo < lo2 + n2 and lo2 < lo + n


def _merge_sibling_tensors(g: Graph, loc: dict):
    """Sibling CONVs that read the same input slice with the same geometry but write into DIFFERENT
    tensors: when one writes the last channels of its tensor and the other the first channels of its
    own, the two tensors become one ([first | second], every reference remapped) and the convs one GEMM
    with N = cout_a + cout_b, as in _merge_siblings.  yolov7 (cfg/deploy/yolov7.yaml): layers 27 + 66
    (the P3 output into the next MP block's 1x1 and into the head's P3 route `[24, 1, Conv, [128, 1,
    1]]`), 40 + 54 (the same at P4) and SPPCSPC 51's cv1 + cv2 (models/common.py:271-280) — pairs of
    launches that each re-read a 52-210 MB input at bs 32.  Only the layout changes (the
    merged tensor's channel pitch); every layer's output keeps its values and its (tensor, offset) in
    layer_tensor."""
    key = ('src', 'src_coff', 'cin', 'k', 's', 'pad', 'act', 'pool')
    i = 0
    while i < len(g.ops):
        a = g.ops[i]
        if a['kind'] != L.OP_CONV or '_w' not in a:
            i += 1
            continue
        merged = False
        for j in range(i + 1, len(g.ops)):
            b = g.ops[j]
            wb = _writes(b)
            if (b['kind'] == L.OP_CONV and '_w' in b and all(a.get(k) == b.get(k) for k in key) and
                    b['dst'] != a['dst'] and g.tensors[a['dst']][1] == g.tensors[b['dst']][1]):
                ca, cb = g.tensors[a['dst']][0], g.tensors[b['dst']][0]
                if a['dst_coff'] + a['cout'] == ca and b['dst_coff'] == 0:
                    first, second = a, b          # [a's tensor | b's tensor]
                elif b['dst_coff'] + b['cout'] == cb and a['dst_coff'] == 0:
                    first, second = b, a          # [b's tensor | a's tensor]
                else:
                    first = None
                if first is not None:
                    # b moves up to a's position: nothing in between may write b's input or read / write
                    # b's output slice
                    ok = True
                    for o in g.ops[i + 1:j]:
                        wo = _writes(o)
                        if wo and (_overlaps(*wo, b['src'], b['src_coff'], b['cin']) or
                                   _overlaps(*wo, b['dst'], b['dst_coff'], b['cout'])):
                            ok = False
                        if o.get('src', -1) >= 0 and _overlaps(o['src'], o.get('src_coff', 0),
                                                               max(o.get('cin', 0), o.get('cout', 0)),
                                                               b['dst'], b['dst_coff'], b['cout']):
                            ok = False
                    if ok:
                        _fuse_tensors(g, loc, first['dst'], second['dst'])
                        m = dict(a)
                        m['dst'] = first['dst']
                        m['dst_coff'] = first['dst_coff']
                        m['cout'] = a['cout'] + b['cout']
                        m['_w'] = torch.cat([first['_w'], second['_w']], 0)
                        m['_b'] = torch.cat([first['_b'], second['_b']], 0)
                        m['merged'] = (first['cout'], second['cout'])
                        m['layers'] = first['layers'] + second['layers']
                        g.ops[i] = m
                        del g.ops[j]
                        merged = True
                        break
            if wb and _overlaps(*wb, a['src'], a['src_coff'], a['cin']):
                break  # a's input is overwritten from here on
        if not merged:
            i += 1


def _fuse_tensors(g: Graph, loc: dict, t1: int, t2: int):
    """Tensor t2 becomes channels [C1, C1 + C2) of tensor t1; t2's id is removed (higher ids shift down)
    in every op and in the layer -> (tensor, offset) map."""
    c1 = g.tensors[t1][0]
    g.tensors[t1][0] = c1 + g.tensors[t2][0]

    def remap(t, off):
        if t == t2:
            t, off = t1, off + c1
        return (t - 1 if t > t2 else t), off

    for o in g.ops:
        if o.get('src', -1) >= 0:
            o['src'], o['src_coff'] = remap(o['src'], o.get('src_coff', 0))
        if o.get('dst', -1) >= 0:
            o['dst'], o['dst_coff'] = remap(o['dst'], o.get('dst_coff', 0))
    for k, (t, off) in list(loc.items()):
        loc[k] = remap(t, off)
    del g.tensors[t2]


def _writes(o):
    """(tensor, first channel, channels) an op writes, or None (DETECT writes z)."""
    if o['kind'] == L.OP_DETECT:
        return None
    if o['kind'] == L.OP_STEM:
        return o['dst'], o['dst_coff'], o['cout2']
    return o['dst'], o['dst_coff'], o['cout']


def _merge_siblings(g: Graph):
    """Fold pairs of CONV ops that read the same input slice with the same geometry and activation and
    write adjacent channel slices of one tensor into a single GEMM with N = cout_a + cout_b.

    In every ELAN block the two 1x1 entry convs (e.g. yolov7.yaml:20-21 `[-1, 1, Conv, [64, 1, 1]]`,
    `[-2, 1, Conv, [64, 1, 1]]`) both read the previous layer and land side by side in the block's
    concat (`[[-1, -3, -5, -6], 1, Concat, [1]]` puts -5 and -6 next to each other): one launch then
    reads the input once and runs a GEMM twice as wide.  Output bytes are unchanged."""
    key = ('src', 'src_coff', 'cin', 'k', 's', 'pad', 'act', 'dst')
    i = 0
    while i < len(g.ops):
        a = g.ops[i]
        if a['kind'] != L.OP_CONV or '_w' not in a:
            i += 1
            continue
        for j in range(i + 1, len(g.ops)):
            b = g.ops[j]
            w = _writes(b)
            if b['kind'] == L.OP_CONV and '_w' in b and all(a[k] == b[k] for k in key):
                if b['dst_coff'] == a['dst_coff'] + a['cout']:
                    lo, hi = a, b
                elif a['dst_coff'] == b['dst_coff'] + b['cout']:
                    lo, hi = b, a
                else:
                    lo = None
                if lo is not None:
                    # b moves up to a's position: nothing in between may write b's input or read/write b's output
                    between = g.ops[i + 1:j]
                    ok = True
                    for o in between:
                        wo = _writes(o)
                        if wo and wo[0] == b['src'] and wo[1] < b['src_coff'] + b['cin'] and b['src_coff'] < wo[1] + wo[2]:
                            ok = False
                        if wo and wo[0] == b['dst'] and wo[1] < b['dst_coff'] + b['cout'] and b['dst_coff'] < wo[1] + wo[2]:
                            ok = False
                        rs = o.get('src', -1)
                        if rs == b['dst'] and o.get('src_coff', 0) < b['dst_coff'] + b['cout'] and \
                                b['dst_coff'] < o.get('src_coff', 0) + max(o.get('cin', 0), o.get('cout', 0)):
                            ok = False
                    if ok:
                        m = dict(a)
                        m['dst_coff'] = lo['dst_coff']
                        m['cout'] = a['cout'] + b['cout']
                        m['_w'] = torch.cat([lo['_w'], hi['_w']], 0)
                        m['_b'] = torch.cat([lo['_b'], hi['_b']], 0)
                        m['merged'] = (lo['cout'], hi['cout'])
                        m['layers'] = lo['layers'] + hi['layers']
                        g.ops[i] = m
                        del g.ops[j]
                        break
            if w and w[0] == a['src'] and w[1] < a['src_coff'] + a['cin'] and a['src_coff'] < w[1] + w[2]:
                break  # a's input is overwritten from here on
        i += 1
