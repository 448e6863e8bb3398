"""Per-op parity of a libyv7 plan: every op's output against a plain PyTorch fp32 reference of the
same op, computed from the op's own input as the plan left it in the workspace.

This isolates each kernel from the error the network accumulates upstream, so it checks exactly the
dispatch a forward took (tile-count dependent kernel choice, split-K, persistent rings, the pooled
1x1, the fused stem, the head).  The references are the reference module's arithmetic:
  CONV      act(conv2d(x, W, b, s, k//2))       models/common.py:110-111 (Conv.fuseforward), 498-500 (RepConv)
            with pool = 2: the MP in front       common.py:30-36
  STEM      the two Convs of layers 0-1          common.py:110-111, with the kernel's own fp16 steps
                                                 (conv A stored in fp16, SiLU's -log2(e) folded into it)
  MAXPOOL   F.max_pool2d(x, k, s, pad)           common.py:30-45, 271 (SPPCSPC cascade 5∘5 = 9, 5∘5∘5 = 13)
  UPSAMPLE  nearest x2                           cfg nn.Upsample(None, 2, 'nearest')
  COPY      the concat slice                     common.py:56-62
  DETECT    1x1 conv + bias (raw logits) and the decode   models/yolo.py:46-57
Convolutions run as sums of per-tap fp32 matmuls on the device (no MIOpen: nothing is compiled at
run time).  Tolerances: an fp16 output within one fp16 ulp of the fp32 reference (+1e-4 of the op's
rms for the accumulation order; two ulps for the fused stem, whose intermediate is fp16); fp32 outputs within 1e-5 |ref| + 1e-4 rms; max / upsample / copy exact.
"""
from __future__ import annotations

import torch
import torch.nn.functional as F

from yv7 import _lib as L


def _act(y, act):
    if act == L.ACT_SILU:
        return F.silu(y)
    if act == L.ACT_LEAKY:
        return F.leaky_relu(y, 0.1)
    return y


def _weights(plan, blob, o, cin=None):
    """Packed weights of a CONV / DETECT op as fp32 [cout, k, k, cin] (plan dtype values) + bias."""
    k, cout = o.get('k', 1), o['cout']
    cin = o['cin'] if cin is None else cin
    es = 2 if plan.dtype == L.DT_F16 else 4
    kpad = (k * k * cin + 63) // 64 * 64
    cpad = (cout + 31) // 32 * 32
    w = blob[o['w_off']:o['w_off'] + cpad * kpad * es].view(torch.float16 if es == 2 else torch.float32)
    w = w.view(cpad, kpad)[:cout, :k * k * cin].float().reshape(cout, k, k, cin)
    b = blob[o['b_off']:o['b_off'] + cout * 4].view(torch.float32).clone()
    return w, b


def conv_ref(x, w, b, s, act):
    """act(conv2d) of an NHWC fp32 batch x [B,H,W,cin] with w [cout,k,k,cin], pad k//2, as per-tap
    fp32 matmuls -> NHWC fp32."""
    k = w.shape[1]
    pad = k // 2
    B, H, W, C = x.shape
    Ho, Wo = (H + 2 * pad - k) // s + 1, (W + 2 * pad - k) // s + 1
    xp = F.pad(x, [0, 0, pad, pad, pad, pad]) if pad else x
    y = b.to(x.device).expand(B * Ho * Wo, -1).clone()
    for r in range(k):
        for c in range(k):
            xs = xp[:, r:r + (Ho - 1) * s + 1:s, c:c + (Wo - 1) * s + 1:s, :].reshape(-1, C)
            y += xs @ w[:, r, c, :].t().to(x.device)
    return _act(y, act).view(B, Ho, Wo, -1)


def _ulp_check(got, ref, what, fp16, ulps=1):
    got, ref = got.float(), ref.float()
    rms = ref.pow(2).mean().sqrt().item()
    if fp16:   # `ulps` fp16 ulps of the larger of the two (a value just under a power of two may round up)
        tol = torch.maximum(ref.abs(), got.abs()) * 2.0 ** -11 * (2 * ulps) + 1e-4 * rms + 1e-7
    else:
        tol = ref.abs() * 1e-5 + 1e-4 * rms + 1e-12
    d = (got - ref).abs()
    bad = d > tol
    nbad = int(bad.sum())
    worst = (d / (ref.abs() + rms + 1e-30)).max().item()
    assert nbad == 0, (f'{what}: {nbad} of {d.numel()} elements off (max |d| {d.max().item():.3g}, '
                       f'rms(ref) {rms:.3g}, worst rel {worst:.3g})')
    return worst


def check_ops(plan, x, B, H, W, raw=None, z=None, skip_fp8=True):
    """Check every op of the last forward of `plan` on input x [B,3,H,W].  Returns {op: worst rel err}."""
    g = plan.graph
    blob = g.weight_blob().to(plan.device)
    fp16 = plan.dtype == L.DT_F16
    es_dt = torch.float16 if fp16 else torch.float32
    tv = lambda t: plan.tensor_view(t, B, H, W)   # interior NHWC views  # noqa: E731
    out = {}
    det_levels = []
    for i, o in enumerate(g.ops):
        kind = o['kind']
        what = f'op {i} ({kind}: {o.get("cin", 0)}->{o["cout"]} k{o.get("k", 1)} s{o.get("s", 1)})'
        if kind == L.OP_INPUT:
            t = tv(o['dst'])
            if o.get('k', 1) == 2:   # ReOrg (common.py:52-53) fused into the packing
                xr = torch.cat([x[..., ::2, ::2], x[..., 1::2, ::2], x[..., ::2, 1::2], x[..., 1::2, 1::2]], 1)
            else:
                xr = x
            ref = xr.to(es_dt).permute(0, 2, 3, 1)
            got = t[..., :ref.shape[-1]]
            assert torch.equal(got, ref), what
            out[i] = 0.0
        elif kind == L.OP_CONV:
            if o.get('wfmt', 0) == L.WFMT_FP8:
                if skip_fp8:
                    continue
                raise NotImplementedError('fp8 ops: tests/test_fp8.py')
            xin = tv(o['src'])[..., o['src_coff']:o['src_coff'] + o['cin']].float()
            s = o['s']
            if o.get('pool', 0) == 2:
                xin = F.max_pool2d(xin.permute(0, 3, 1, 2), 2, 2).permute(0, 2, 3, 1)
                s = 1
            w, b = _weights(plan, blob, o)
            ref = conv_ref(xin, w, b, s, o['act'])
            got = tv(o['dst'])[..., o['dst_coff']:o['dst_coff'] + o['cout']]
            out[i] = _ulp_check(got, ref, what, fp16)
        elif kind == L.OP_STEM:
            # csrc/stem.hip's arithmetic: with SiLU on both convs, conv A's weights / bias are
            # pre-scaled by -log2(e) (weights rounded to fp16 again), A is stored in fp16 as
            # -log2(e) * silu(a), conv B's bias is scaled the same way and its epilogue undoes it
            reorg = o['cin'] == 12   # the w6 front end: ReOrg (common.py:52-53) + conv A on 12 channels
            xr = torch.cat([x[..., ::2, ::2], x[..., 1::2, ::2], x[..., ::2, 1::2], x[..., 1::2, 1::2]], 1) if reorg else x
            xin = xr.to(es_dt).float().permute(0, 2, 3, 1).contiguous()
            wa, ba = _weights(plan, blob, dict(o, cin=16 if reorg else 3))
            wa = wa[..., :o['cin']]
            ob = dict(o, cin=o['cout'], cout=o['cout2'], w_off=o['w2_off'], b_off=o['b2_off'])
            wb, bb = _weights(plan, blob, ob)
            if o['act'] == L.ACT_SILU and o['act2'] == L.ACT_SILU:
                nl2e = -1.4426950408889634
                za = conv_ref(xin, (wa * nl2e).half().float(), ba * nl2e, o['s'], L.ACT_NONE)
                a = (za / (1.0 + torch.exp2(za))).half().float()
                zb = conv_ref(a, wb, bb * nl2e, 2, L.ACT_NONE)
                ref = (zb * -0.6931471805599453) / (1.0 + torch.exp2(zb))
            else:
                a = conv_ref(xin, wa, ba, o['s'], o['act']).to(es_dt).float()
                ref = conv_ref(a, wb, bb, 2, o['act2'])
            got = tv(o['dst'])[..., o['dst_coff']:o['dst_coff'] + o['cout2']]
            # conv A's fp16 rounding flips by an ulp where its fp32 sum (approximate exp2 / rcp in the
            # SiLU) lands on the other side of a rounding step than the reference's; conv B carries
            # such a flip (up to ulp(|A|) x |w|, ~1e-3 for the large A values) into its output.  So:
            # two ulps everywhere but a few 1e-4 of the elements, which stay within 5e-3 of the rms
            got, ref = got.float(), ref.float()
            rms = ref.pow(2).mean().sqrt().item()
            d = (got - ref).abs()
            loose = int((d > torch.maximum(ref.abs(), got.abs()) * 2.0 ** -9 + 1e-4 * rms).sum())
            assert loose <= 1e-3 * d.numel(), f'{what}: {loose} of {d.numel()} elements beyond two ulps'
            assert d.max().item() <= 5e-3 * rms, f'{what}: max |d| {d.max().item():.3g} (rms {rms:.3g})'
            out[i] = (d / (ref.abs() + rms)).max().item()
        elif kind == L.OP_MAXPOOL:
            xin = tv(o['src'])[..., o['src_coff']:o['src_coff'] + o['cout']]
            ref = F.max_pool2d(xin.permute(0, 3, 1, 2).float(), o['k'], o['s'], o['pad']).permute(0, 2, 3, 1)
            got = tv(o['dst'])[..., o['dst_coff']:o['dst_coff'] + o['cout']]
            assert torch.equal(got.float(), ref), what
            out[i] = 0.0
        elif kind == L.OP_UPSAMPLE:
            xin = tv(o['src'])[..., o['src_coff']:o['src_coff'] + o['cout']]
            ref = xin.repeat_interleave(2, 1).repeat_interleave(2, 2)
            got = tv(o['dst'])[..., o['dst_coff']:o['dst_coff'] + o['cout']]
            assert torch.equal(got, ref), what
            out[i] = 0.0
        elif kind == L.OP_COPY:
            xin = tv(o['src'])[..., o['src_coff']:o['src_coff'] + o['cout']]
            got = tv(o['dst'])[..., o['dst_coff']:o['dst_coff'] + o['cout']]
            assert torch.equal(got, xin), what
            out[i] = 0.0
        elif kind == L.OP_DETECT:
            det_levels.append((i, o))
    if raw is not None:
        # raw logits [B, na, ny, nx, no] per level: 1x1 conv + bias in fp32 (yolo.py:46-50)
        for (i, o), xs in zip(sorted(det_levels, key=lambda t: t[1]['level']), raw):
            xin = tv(o['src'])[..., o['src_coff']:o['src_coff'] + o['cin']].float()
            w, b = _weights(plan, blob, o)
            ref = conv_ref(xin, w, b, 1, L.ACT_NONE)     # [B, ny, nx, na*no]
            Bq, ny, nx, _ = ref.shape
            ref = ref.view(Bq, ny, nx, plan.na, plan.no).permute(0, 3, 1, 2, 4)
            scale = max(1.0, ref.abs().max().item())
            d = (xs.float() - ref).abs().max().item()
            assert d <= 1e-4 * scale, f'op {i} DETECT level {o["level"]}: raw logits max |d| {d:.3g} (scale {scale:.3g})'
            out[i] = d / scale
        if z is not None:
            # decode of the GPU's own logits, the reference's op order (yolo.py:52-57)
            zs, row = [], 0
            for (i, o), xs in zip(sorted(det_levels, key=lambda t: t[1]['level']), raw):
                lvl = o['level']
                Bq, na, ny, nx, no = xs.shape
                y = xs.float().sigmoid()
                yv, xv = torch.meshgrid(torch.arange(ny, device=y.device), torch.arange(nx, device=y.device),
                                        indexing='ij')
                grid = torch.stack((xv, yv), 2).view(1, 1, ny, nx, 2).float()
                ag = torch.tensor(g.anchor_grid, device=y.device).view(g.nl, 1, g.na, 1, 1, 2)[lvl]
                y[..., 0:2] = (y[..., 0:2] * 2. - 0.5 + grid) * g.stride[lvl]
                y[..., 2:4] = (y[..., 2:4] * 2) ** 2 * ag
                zs.append(y.view(Bq, -1, no))
            zr = torch.cat(zs, 1)
            sc = zr.abs().clamp(min=1.0)
            d = ((z.float() - zr).abs() / sc).max().item()
            assert d <= 1e-5, f'Detect decode: max rel |d| {d:.3g}'
    return out


def kernel_summary(out):
    worst = max(out.items(), key=lambda kv: kv[1]) if out else (None, 0.0)
    return f'{len(out)} ops checked, worst rel err {worst[1]:.3g} at op {worst[0]}'


def rms_rel(got, ref):
    rms = ref.float().pow(2).mean().sqrt().item()
    return (got.float() - ref.float()).pow(2).mean().sqrt().item() / max(rms, 1e-3)
