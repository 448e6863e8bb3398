"""Frame pre-processing: letterbox geometry (datasets.py:1279-1305), the cv2 INTER_LINEAR restatement
(oracle/letterbox_ref.py) on hand-derived cases, and the GPU kernel (yv7_letterbox) bit-exact against it.

cv2 is absent here (parity of the resize itself is unpinned, see the oracle's header); the geometry is
pinned by hand-derived values, the fixed-point arithmetic by the known answers below."""
import numpy as np
import pytest
import torch

from oracle import letterbox_ref as R
from utils import datasets as D

# (frame h, w) of the reference's sample images (read from their JPEG headers) and odd sizes
SHAPES = [(1080, 810), (720, 1280), (480, 640), (1280, 1280), (333, 517), (640, 640), (17, 1000), (1000, 9)]


def test_geometry_bus_jpg():
    # samples/bus.jpg is 810 x 1080 (w x h): r = 640/1080, 480 x 640 unpadded, 80 px each side
    new_unpad, ratio, (dw, dh), border = D.letterbox_geometry((1080, 810), 640, auto=False)
    assert new_unpad == (480, 640) and ratio == (640 / 1080, 640 / 1080)
    assert (dw, dh) == (80.0, 0.0) and border == (0, 0, 80, 80)
    # auto=True (minimum rectangle, stride 32): 160 % 32 = 0 -> no padding at all
    new_unpad, _, (dw, dh), border = D.letterbox_geometry((1080, 810), 640, auto=True)
    assert new_unpad == (480, 640) and border == (0, 0, 0, 0)
    # an odd padding splits with the -0.1/+0.1 rounding: 640 - 637 = 3 -> 1 top, 2 bottom
    new_unpad, _, (dw, dh), border = D.letterbox_geometry((637, 640), 640, auto=False, scaleup=False)
    assert new_unpad == (640, 637) and dh == 1.5 and border == (1, 2, 0, 0)


@pytest.mark.parametrize('shape', SHAPES)
@pytest.mark.parametrize('kw', [dict(auto=False), dict(auto=True), dict(auto=False, scaleup=False),
                                dict(auto=False, scaleFill=True)])
def test_product_geometry_matches_oracle(shape, kw):
    assert D.letterbox_geometry(shape, 640, **kw) == R.letterbox_geometry(shape, 640, **kw)


def test_resize_known_answers():
    # 1 x 2 -> 1 x 4 (rows unchanged): columns -0.25 -> (0, 0) reset, 0.25, 0.75, 1.25 -> (1, 0) reset
    # coefficients (2048, 0) (1536, 512) (512, 1536) (2048, 0); value 255 on the right:
    #   x1: ((255*512 >> 4) * 2048 >> 16) + 2 >> 2 = 64, x2: ((255*1536 >> 4) * 2048 >> 16) + 2 >> 2 = 191
    img = np.zeros((1, 2, 3), np.uint8)
    img[0, 1] = 255
    out = R.resize_linear_u8(img, 4, 1)
    assert out[0, :, 0].tolist() == [0, 64, 191, 255]
    # a constant frame stays constant under any scaling
    c = np.full((37, 53, 3), 77, np.uint8)
    assert np.unique(R.resize_linear_u8(c, 100, 60)).tolist() == [77]
    assert np.unique(R.resize_linear_u8(c, 11, 7)).tolist() == [77]
    # exact 2x downscale = rounded 2 x 2 mean (cv2's INTER_AREA fast path): (1 + 2 + 3 + 5 + 2) >> 2 = 3
    q = np.array([[1, 2], [3, 5]], np.uint8)[:, :, None].repeat(3, 2)
    assert R.resize_linear_u8(q, 1, 1)[0, 0].tolist() == [3, 3, 3]


def test_letterbox_border_and_conversion():
    img = np.random.RandomState(0).randint(0, 256, (60, 40, 3)).astype(np.uint8)
    out, ratio, (dw, dh) = R.letterbox(img, 64, auto=False)
    assert out.shape == (64, 64, 3) and ratio == (64 / 60, 64 / 60)
    left = int(round(dw - 0.1))
    assert (out[:, :left] == 114).all() and (out[:, left + 43:] == 114).all()
    x = R.to_input(out, half=False)
    assert x.shape == (3, 64, 64) and x.dtype == torch.float32
    assert torch.equal(x[0], torch.from_numpy(out[:, :, 2].astype(np.float32)) / 255.0)   # BGR -> RGB


# ------------------------------------------------------------------------------------------ GPU
def _frames(shape, b=2, seed=0):
    return np.random.RandomState(seed).randint(0, 256, (b,) + tuple(shape) + (3,)).astype(np.uint8)


@pytest.mark.gpu
@pytest.mark.parametrize('shape', SHAPES)
@pytest.mark.parametrize('kw', [dict(auto=False), dict(auto=True), dict(auto=False, scaleup=False)])
def test_gpu_letterbox_bit_exact(shape, kw):
    frames = _frames(shape)
    g = D._run(torch.from_numpy(frames).cuda(), D.letterbox_geometry(shape, 640, **kw), (114, 114, 114),
               D.OUT_U8_HWC).cpu().numpy()
    for i in range(frames.shape[0]):
        ref, _, _ = R.letterbox(frames[i], 640, **kw)
        assert g[i].shape == ref.shape
        assert np.array_equal(g[i], ref), f'{shape} {kw}: {int((g[i] != ref).sum())} bytes differ'


@pytest.mark.gpu
@pytest.mark.parametrize('half', [True, False])
def test_gpu_letterbox_batch_model_input(half):
    frames = _frames((1080, 810), b=3, seed=1)
    x, ratio, dwdh = D.letterbox_batch(torch.from_numpy(frames).cuda(), 640, half=half)
    assert x.shape == (3, 3, 640, 640) and x.dtype == (torch.float16 if half else torch.float32)
    for i in range(3):
        ref_img, r, d = R.letterbox(frames[i], 640, auto=False)
        assert (r, d) == (ratio, dwdh)
        assert torch.equal(x[i].cpu(), R.to_input(ref_img, half=half))


@pytest.mark.gpu
def test_gpu_letterbox_numpy_api_and_colour():
    frame = _frames((333, 517), b=1, seed=2)[0]
    out, ratio, dwdh = D.letterbox(frame, 416, color=(0, 50, 200), auto=False)
    ref, r2, d2 = R.letterbox(frame, 416, color=(0, 50, 200), auto=False)
    assert isinstance(out, np.ndarray) and np.array_equal(out, ref) and (ratio, dwdh) == (r2, d2)
