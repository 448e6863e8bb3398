"""TEST INFRASTRUCTURE ONLY — CPU restatement of the reference's frame pre-processing.

Restates utils/datasets.py:1277-1307 (`letterbox`) and the conversion of detect.py:100-104
(BGR -> RGB, HWC -> CHW, uint8 -> half/float, /255).  The resize inside letterbox is
`cv2.resize(img, new_unpad, interpolation=cv2.INTER_LINEAR)` (datasets.py:1302), a third-party
dependency that is absent from /root/reference and from this image (no cv2 wheel; version
unpinned — there is no requirements.txt).  It is restated here from OpenCV's published
generic 8-bit bilinear path (imgproc/src/resize.cpp, resizeGeneric_ with fixed-point
coefficients):
  * per destination column: fx = float((dx + 0.5) * (1 / (dst_w / src_w)) - 0.5) (double arithmetic,
    then float), sx = floor(fx), fx -= sx; sx < 0 -> (sx, fx) = (0, 0); sx >= src_w - 1 ->
    (sx, fx) = (src_w - 1, 0); alpha = (cvRound((1 - fx) * 2048), cvRound(fx * 2048)) (float32
    products, round half to even); per destination row the same without the reset — the fetched
    row indices are clamped instead;
  * horizontal pass: D[x] = S[sx] * a0 + S[sx + 1] * a1 (int32, exact);
  * vertical pass as OpenCV's vectorised VResizeLinearVec_32s8u computes it:
    dst = ((((D0 >> 4) * b0) >> 16) + (((D1 >> 4) * b1) >> 16) + 2) >> 2, saturated to [0, 255];
    the last (new_w * 3) % 16 values of a row take the scalar FixedPtCast (D0*b0 + D1*b1 + 2^21) >> 22
    (none for the 640 / 480-wide frames of the bench);
  * an exact 2x downscale in both directions runs cv2's INTER_AREA fast path instead (resize.cpp
    switches INTER_LINEAR to it): the rounded mean (a + b + c + d + 2) >> 2 of each 2 x 2 block.
PARITY UNPINNED: no cv2 here and no reference fixture holds a resized frame; IPP-accelerated cv2
builds may round differently.  The letterbox geometry (ratio, new_unpad, padding split) follows
datasets.py:1279-1306 exactly and is pinned by hand-derived cases (tests/test_preprocess.py).
"""
from __future__ import annotations

import math

import numpy as np

COEF_BITS = 11
COEF_SCALE = 1 << COEF_BITS


def letterbox_geometry(shape, new_shape=(640, 640), auto=True, scaleFill=False, scaleup=True, stride=32):
    """datasets.py:1279-1305: (new_unpad (w, h), ratio (rw, rh), (dw, dh), (top, bottom, left, right))."""
    if isinstance(new_shape, int):
        new_shape = (new_shape, new_shape)
    r = min(new_shape[0] / shape[0], new_shape[1] / shape[1])
    if not scaleup:
        r = min(r, 1.0)
    ratio = r, r
    new_unpad = int(round(shape[1] * r)), int(round(shape[0] * r))
    dw, dh = new_shape[1] - new_unpad[0], new_shape[0] - new_unpad[1]
    if auto:
        dw, dh = np.mod(dw, stride), np.mod(dh, stride)
    elif scaleFill:
        dw, dh = 0.0, 0.0
        new_unpad = (new_shape[1], new_shape[0])
        ratio = new_shape[1] / shape[1], new_shape[0] / shape[0]
    dw /= 2
    dh /= 2
    top, bottom = int(round(dh - 0.1)), int(round(dh + 0.1))
    left, right = int(round(dw - 0.1)), int(round(dw + 0.1))
    return new_unpad, ratio, (dw, dh), (top, bottom, left, right)


def linear_tables(src, dst, clamp_coef):
    """Per destination index (resizeGeneric_ tables): source index sy/sx (clamped for fetching), its
    successor (clamped), and the two fixed-point coefficients round((1 - f) * 2048), round(f * 2048)
    (float32 products, round half to even as cvRound).  Columns reset (s, f) at the borders
    (clamp_coef); rows keep f and only clamp the fetched row indices."""
    inv = dst / src
    scale = 1.0 / inv
    i0 = np.empty(dst, np.int64)
    c0 = np.empty(dst, np.int64)
    c1 = np.empty(dst, np.int64)
    for d in range(dst):
        f = np.float32((d + 0.5) * scale - 0.5)
        s = math.floor(f)
        f = np.float32(f - np.float32(s))
        if clamp_coef:
            if s < 0:
                s, f = 0, np.float32(0.0)
            if s >= src - 1:
                s, f = src - 1, np.float32(0.0)
        i0[d] = s
        c0[d] = int(np.rint(np.float32(np.float32(1.0) - f) * np.float32(COEF_SCALE)))
        c1[d] = int(np.rint(f * np.float32(COEF_SCALE)))
    i1 = np.clip(i0 + 1, 0, src - 1)
    return np.clip(i0, 0, src - 1), i1, c0, c1


SIMD_LANES = 16   # u8 lanes of OpenCV's baseline-SIMD vertical pass; the row tail takes the scalar cast


def resize_linear_u8(img, new_w, new_h):
    """cv2.resize(img, (new_w, new_h), interpolation=INTER_LINEAR) for uint8 HWC images (restated)."""
    h, w, cn = img.shape
    src = img.astype(np.int64)
    if w == 2 * new_w and h == 2 * new_h:
        # resize.cpp: INTER_LINEAR with an exact 2x downscale in both directions runs INTER_AREA's
        # fast path: the rounded mean of each 2 x 2 block
        s = src[0::2, 0::2] + src[0::2, 1::2] + src[1::2, 0::2] + src[1::2, 1::2]
        return ((s + 2) >> 2).astype(np.uint8)
    xs0, xs1, a0, a1 = linear_tables(w, new_w, True)
    ys0, ys1, b0, b1 = linear_tables(h, new_h, False)
    # horizontal pass on every source row: D[y, x, c] (exact int32)
    d = src[:, xs0, :] * a0[None, :, None] + src[:, xs1, :] * a1[None, :, None]
    d0 = d[ys0].reshape(new_h, new_w * cn)
    d1 = d[ys1].reshape(new_h, new_w * cn)
    bb0, bb1 = b0[:, None], b1[:, None]
    vec = ((((d0 >> 4) * bb0) >> 16) + (((d1 >> 4) * bb1) >> 16) + 2) >> 2
    sca = (d0 * bb0 + d1 * bb1 + (1 << 21)) >> 22
    nv = (new_w * cn) // SIMD_LANES * SIMD_LANES
    out = np.concatenate([vec[:, :nv], sca[:, nv:]], axis=1)
    return np.clip(out, 0, 255).astype(np.uint8).reshape(new_h, new_w, cn)


def letterbox(img, new_shape=(640, 640), color=(114, 114, 114), auto=True, scaleFill=False, scaleup=True,
              stride=32):
    """datasets.py:1277-1307 restated: (img, ratio, (dw, dh))."""
    shape = img.shape[:2]
    new_unpad, ratio, (dw, dh), (top, bottom, left, right) = letterbox_geometry(shape, new_shape, auto, scaleFill,
                                                                               scaleup, stride)
    if shape[::-1] != new_unpad:
        img = resize_linear_u8(img, new_unpad[0], new_unpad[1])
    out = np.empty((img.shape[0] + top + bottom, img.shape[1] + left + right, 3), np.uint8)
    out[...] = np.asarray(color, np.uint8)
    out[top:top + img.shape[0], left:left + img.shape[1]] = img
    return out, ratio, (dw, dh)


def to_input(img_hwc_bgr, half=False):
    """detect.py:100-104 / datasets.py:199: BGR -> RGB, HWC -> CHW, to half/float, /255 -> [3, H, W]."""
    import torch
    x = torch.from_numpy(np.ascontiguousarray(img_hwc_bgr[:, :, ::-1].transpose(2, 0, 1)))
    x = x.half() if half else x.float()
    if half:   # torch's half division computes in float and rounds once (the GPU path the reference runs)
        return (x.float() / 255.0).half()
    return x / 255.0
