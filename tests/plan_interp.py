"""CPU interpreter of a compiled plan (test infrastructure only, never a product path).

Executes yv7.graph.compile_model()'s op list with plain torch CPU ops on NHWC fp32 tensors, reading the
packed weight blob exactly as the HIP runtime does (csrc/runtime.cpp: tensor shapes from `shift`,
channel slices by offset, weights [cout_pad32][k][k][cin_pad] with K padded to 64).  Comparing its z
with the oracle's checks the graph compiler — concat placement, SPPCSPC pool cascade, ReOrg / stem
fusion, sibling-conv merging, detect-row layout — on CPU, independent of the GPU kernels.
"""
from __future__ import annotations

import torch
import torch.nn.functional as F

from yv7 import _lib as L
from yv7.graph import _rup


def _act(x, a):
    if a == L.ACT_SILU:
        return F.silu(x)
    if a == L.ACT_LEAKY:
        return F.leaky_relu(x, 0.1)
    return x


def _weights(blob, dtype, off, cout, k, cin):
    esz = 2 if dtype == L.DT_F16 else 4
    kpad = _rup(k * k * cin, 64)
    n = _rup(cout, 32) * kpad
    raw = blob[off:off + n * esz].view(torch.float16 if esz == 2 else torch.float32).float().view(-1, kpad)
    return raw[:cout, :k * k * cin].reshape(cout, k, k, cin).permute(0, 3, 1, 2).contiguous()


def _weights_f8(blob, off, cout, cin, s_off):
    """FP8 op: e4m3 [cout_pad32][cin padded to 128] times the fp32 per-channel scales -> [cout, cin, 1, 1]."""
    kp = _rup(cin, 128)
    raw = blob[off:off + _rup(cout, 32) * kp].view(torch.float8_e4m3fn).float().view(-1, kp)
    ws = blob[s_off:s_off + 4 * cout].view(torch.float32)
    return (raw[:cout, :cin] * ws[:, None]).reshape(cout, cin, 1, 1)


def _bias(blob, off, cout):
    return blob[off:off + 4 * cout].view(torch.float32).clone()


def run(g, x: torch.Tensor, return_tensors=False):
    """x: [B, 3, H, W] float -> z [B, N, no] (fp32 math throughout); with return_tensors also the
    plan's NCHW tensors (per-op input statistics, e.g. fp8 calibration on the CPU)."""
    B, _, H, W = x.shape
    blob = g.weight_blob()
    T = [torch.zeros(B, c, H >> s if s >= 0 else H << -s, W >> s if s >= 0 else W << -s) for c, s in g.tensors]
    zs = []
    for o in g.ops:
        kind = o['kind']
        if kind == L.OP_INPUT:
            v = x.float()
            if o['k'] == 2:   # ReOrg (models/common.py ReOrg.forward)
                v = torch.cat([v[..., ::2, ::2], v[..., 1::2, ::2], v[..., ::2, 1::2], v[..., 1::2, 1::2]], 1)
            T[o['dst']][:, :v.shape[1]] = v
        elif kind == L.OP_STEM:
            v = x.float()
            if o['cin'] == 12:   # the w6 front end: ReOrg fused (conv A's K packed as tap * 16 + ci)
                v = torch.cat([v[..., ::2, ::2], v[..., 1::2, ::2], v[..., ::2, 1::2], v[..., 1::2, 1::2]], 1)
                wa = _weights(blob, g.dtype, o['w_off'], o['cout'], 3, 16)[:, :12]
            else:
                wa = _weights(blob, g.dtype, o['w_off'], o['cout'], 3, 3)
            a = _act(F.conv2d(v, wa, _bias(blob, o['b_off'], o['cout']), o['s'], 1), o['act'])
            wb = _weights(blob, g.dtype, o['w2_off'], o['cout2'], 3, o['cout'])
            y = _act(F.conv2d(a, wb, _bias(blob, o['b2_off'], o['cout2']), 2, 1), o['act2'])
            T[o['dst']][:, o['dst_coff']:o['dst_coff'] + o['cout2']] = y
        elif kind == L.OP_CONV:
            src = T[o['src']][:, o['src_coff']:o['src_coff'] + o['cin']]
            if o.get('pool', 0) == 2:   # MP folded into the conv (yv7.graph._fold_pools)
                src = F.max_pool2d(src, 2, 2)
            if o.get('wfmt', 0) == L.WFMT_FP8:   # e4m3 input on the op's scale, e4m3 weights
                xs = o['xscale']
                src = (src / xs).clamp(-448.0, 448.0).to(torch.float8_e4m3fn).float() * xs
                w = _weights_f8(blob, o['w_off'], o['cout'], o['cin'], o['s_off'])
            else:
                w = _weights(blob, g.dtype, o['w_off'], o['cout'], o['k'], o['cin'])
            y = _act(F.conv2d(src, w, _bias(blob, o['b_off'], o['cout']), 1 if o.get('pool', 0) else o['s'],
                              o['pad']), o['act'])
            T[o['dst']][:, o['dst_coff']:o['dst_coff'] + o['cout']] = y
        elif kind == L.OP_MAXPOOL:
            src = T[o['src']][:, o['src_coff']:o['src_coff'] + o['cout']]
            y = F.max_pool2d(src, o['k'], o['s'], o['pad'])
            T[o['dst']][:, o['dst_coff']:o['dst_coff'] + o['cout']] = y
        elif kind == L.OP_UPSAMPLE:
            src = T[o['src']][:, o['src_coff']:o['src_coff'] + o['cout']]
            T[o['dst']][:, o['dst_coff']:o['dst_coff'] + o['cout']] = F.interpolate(src, scale_factor=2.0, mode='nearest')
        elif kind == L.OP_COPY:
            T[o['dst']][:, o['dst_coff']:o['dst_coff'] + o['cout']] = T[o['src']][:, o['src_coff']:o['src_coff'] + o['cout']]
        elif kind == L.OP_DETECT:
            lvl = o['level']
            src = T[o['src']][:, o['src_coff']:o['src_coff'] + o['cin']]
            w = _weights(blob, g.dtype, o['w_off'], o['cout'], 1, o['cin'])
            r = F.conv2d(src, w, _bias(blob, o['b_off'], o['cout']))          # [B, na*no, ny, nx]
            ny, nx = r.shape[2:]
            r = r.view(B, g.na, g.no, ny, nx).permute(0, 1, 3, 4, 2)         # models/yolo.py:50
            yv, xv = torch.meshgrid(torch.arange(ny), torch.arange(nx), indexing='ij')
            grid = torch.stack((xv, yv), 2).view(1, 1, ny, nx, 2).float()
            anc = torch.tensor(g.anchor_grid).view(g.nl, g.na, 2)[lvl].view(1, g.na, 1, 1, 2)
            y = r.sigmoid()                                                   # models/yolo.py:52-57
            xy = (y[..., 0:2] * 2. - 0.5 + grid) * g.stride[lvl]
            wh = (y[..., 2:4] * 2) ** 2 * anc
            zs.append(torch.cat((xy, wh, y[..., 4:]), -1).view(B, -1, g.no))
        else:
            raise ValueError(f'op kind {kind}')
    z = torch.cat(zs, 1)
    return (z, T) if return_tensors else z
