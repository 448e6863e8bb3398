"""Frame pre-processing on the GPU — the reference's letterbox() and detect.py's input conversion.

`letterbox(img, new_shape, color, auto, scaleFill, scaleup, stride)` keeps the signature and return
value of utils/datasets.py:1277-1307 ((img, ratio, (dw, dh)); img HWC BGR uint8) with the resize and
border done by libyv7 (yv7_letterbox: cv2.resize INTER_LINEAR restated bit for bit in fixed point,
see csrc/preprocess.hip).  `letterbox_batch(frames, img_size, half, ...)` fuses it with detect.py's
conversion (img[:, :, ::-1].transpose(2, 0, 1), .half()/.float(), /= 255, detect.py:100-104) and
writes the [B, 3, S, S] model input in one launch.  There is no CPU path: inputs go to the current
HIP device and the library must be built (the ctypes binding raises otherwise).
"""
from __future__ import annotations

import numpy as np
import torch

from yv7 import _lib as L

OUT_U8_HWC, OUT_F16_CHW, OUT_F32_CHW = 0, 1, 2


def letterbox_geometry(shape, new_shape=(640, 640), auto=True, scaleFill=False, scaleup=True, stride=32):
    """datasets.py:1279-1305 for a frame of `shape` (h, w): new_unpad (w, h), ratio, (dw, dh) and the
    integer border (top, bottom, left, right) cv2.copyMakeBorder receives."""
    if isinstance(new_shape, int):
        new_shape = (new_shape, new_shape)
    r = min(new_shape[0] / shape[0], new_shape[1] / shape[1])
    if not scaleup:   # only scale down (better test mAP)
        r = min(r, 1.0)
    ratio = r, r
    new_unpad = int(round(shape[1] * r)), int(round(shape[0] * r))
    dw, dh = new_shape[1] - new_unpad[0], new_shape[0] - new_unpad[1]
    if auto:   # minimum rectangle
        dw, dh = np.mod(dw, stride), np.mod(dh, stride)
    elif scaleFill:   # stretch
        dw, dh = 0.0, 0.0
        new_unpad = (new_shape[1], new_shape[0])
        ratio = new_shape[1] / shape[1], new_shape[0] / shape[0]
    dw /= 2
    dh /= 2
    top, bottom = int(round(dh - 0.1)), int(round(dh + 0.1))
    left, right = int(round(dw - 0.1)), int(round(dw + 0.1))
    return new_unpad, ratio, (dw, dh), (top, bottom, left, right)


def _run(frames: torch.Tensor, geom, color, out_kind):
    """frames: uint8 [B, H, W, 3] on a HIP device -> letterboxed output of `out_kind`."""
    if not frames.is_cuda:
        raise RuntimeError('letterbox: frames must be on a HIP device (there is no CPU path)')
    if frames.dtype != torch.uint8 or frames.dim() != 4 or frames.shape[-1] != 3:
        raise ValueError(f'letterbox: expected uint8 [B, H, W, 3] BGR frames, got {frames.dtype} {tuple(frames.shape)}')
    frames = frames.contiguous()
    B, H, W, _ = frames.shape
    (nw, nh), _, _, (top, bottom, left, right) = geom
    oh, ow = nh + top + bottom, nw + left + right
    dev = frames.device
    if out_kind == OUT_U8_HWC:
        out = torch.empty((B, oh, ow, 3), dtype=torch.uint8, device=dev)
    else:
        out = torch.empty((B, 3, oh, ow), dtype=torch.float16 if out_kind == OUT_F16_CHW else torch.float32,
                          device=dev)
    lib = L.lib()
    ws = torch.empty(int(lib.yv7_letterbox_workspace_bytes(nh, nw)), dtype=torch.uint8, device=dev)
    c = [int(v) for v in color]
    with torch.cuda.device(dev):
        stream = torch.cuda.current_stream(dev).cuda_stream
        L.check(lib.yv7_letterbox(frames.data_ptr(), B, H, W, nh, nw, top, left, oh, ow, c[0], c[1], c[2], out_kind,
                                  out.data_ptr(), ws.data_ptr(), ws.numel(), stream), 'yv7_letterbox')
    return out


def letterbox(img, new_shape=(640, 640), color=(114, 114, 114), auto=True, scaleFill=False, scaleup=True, stride=32):
    """utils/datasets.py:1277-1307: resize and pad an HWC BGR uint8 frame (numpy array or HIP tensor).
    Returns (img, ratio, (dw, dh)); img has the input's type (numpy in -> numpy out)."""
    as_numpy = isinstance(img, np.ndarray)
    t = torch.from_numpy(np.ascontiguousarray(img)).to(f'cuda:{torch.cuda.current_device()}') if as_numpy else img
    if t.dim() != 3:
        raise ValueError(f'letterbox: expected an HWC frame, got shape {tuple(t.shape)}')
    geom = letterbox_geometry(tuple(t.shape[:2]), new_shape, auto, scaleFill, scaleup, stride)
    out = _run(t[None], geom, color, OUT_U8_HWC)[0]
    return (out.cpu().numpy() if as_numpy else out), geom[1], geom[2]


def letterbox_batch(frames, img_size=640, half=True, color=(114, 114, 114), auto=False, scaleFill=False,
                    scaleup=True, stride=32):
    """LoadImages (datasets.py:196-200) + detect.py:100-104 for a batch of same-size frames:
    uint8 [B, H, W, 3] BGR (HIP tensor) -> ([B, 3, S, S] half/float RGB in [0, 1], ratio, (dw, dh)).
    detect.py's loader letterboxes with auto=False (datasets.py:196), the default here."""
    if isinstance(frames, np.ndarray):
        frames = torch.from_numpy(np.ascontiguousarray(frames)).to(f'cuda:{torch.cuda.current_device()}')
    if frames.dim() == 3:
        frames = frames[None]
    geom = letterbox_geometry(tuple(frames.shape[1:3]), img_size, auto, scaleFill, scaleup, stride)
    x = _run(frames, geom, color, OUT_F16_CHW if half else OUT_F32_CHW)
    return x, geom[1], geom[2]


# ------------------------------------------------------------------------------------------ images
IMG_FORMATS = ('bmp', 'jpg', 'jpeg', 'png', 'tif', 'tiff', 'webp', 'mpo')


def imread(path):
    """cv2.imread(path) (BGR uint8 HWC) substitute: cv2 is absent from this image, frames are decoded by
    PIL.  JPEG decoders may differ from cv2's libjpeg by +-1 per channel (decode parity unpinned);
    everything after the decode (letterbox, model, NMS) is the path under test."""
    from PIL import Image
    with Image.open(path) as im:
        rgb = np.asarray(im.convert('RGB'))
    return np.ascontiguousarray(rgb[:, :, ::-1])


class LoadImages:
    """utils/datasets.py:133-202 for image files (a file, a directory or a glob): yields
    (path, img CHW RGB uint8 letterboxed, img0 HWC BGR, None, ratio, (dw, dh)) like the reference, with
    the letterbox done on the current HIP device (auto=False, as datasets.py:196)."""

    def __init__(self, path, img_size=640, stride=32):
        import glob
        import os
        p = str(os.path.abspath(path))
        if '*' in p:
            files = sorted(glob.glob(p, recursive=True))
        elif os.path.isdir(p):
            files = sorted(glob.glob(os.path.join(p, '*.*')))
        elif os.path.isfile(p):
            files = [p]
        else:
            raise Exception(f'ERROR: {p} does not exist')
        self.files = [x for x in files if x.split('.')[-1].lower() in IMG_FORMATS]
        self.img_size, self.stride, self.mode, self.cap = img_size, stride, 'image', None
        self.nf = len(self.files)
        assert self.nf > 0, f'No images found in {p}. Supported formats are: {IMG_FORMATS}'

    def __iter__(self):
        self.count = 0
        return self

    def __next__(self):
        if self.count == self.nf:
            raise StopIteration
        path = self.files[self.count]
        self.count += 1
        img0 = imread(path)
        img, ratio, dwdh = letterbox(img0, new_shape=(self.img_size, self.img_size), auto=False)
        img = np.ascontiguousarray(img[:, :, ::-1].transpose(2, 0, 1))   # BGR to RGB, 3 x S x S
        return path, img, img0, self.cap, ratio, dwdh

    def __len__(self):
        return self.nf
