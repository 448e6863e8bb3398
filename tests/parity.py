"""fp32 parity criterion shared by the GPU tests and smoke().

The north star asks for box coords / conf within 1e-4 of the reference fp32 CPU path.  The
reference's own fp32 result is only defined up to its summation order: on the synthetic yolov7
weights at 640x640 the oracle's fp32 z differs from the same computation in float64 by up to
~2.6e-3 relative on box coordinates (scripts/diag_parity.py, measured on the MI355X box), so no
implementation with a different summation order — including the reference on another CPU — can be
within 1e-4 of it everywhere.  The criterion therefore anchors both sides on float64 ("exact"):
  (1) accuracy: max and rms of |z_gpu - z64| / scale are each <= 1.25x the reference's own
      |z_ref32 - z64| / scale (scale = max(1, |z|) for box coords, 1 for conf) — the GPU is at
      least as accurate as the reference CPU path;
  (2) closeness: |z_gpu - z_ref32| <= 1e-4 * scale on at least 99 % of all elements, and the
      percentage that exceeds 1e-4 is reported.
"""
import torch


def check_z(z_gpu, z32, z64, label='', frac=0.99):
    z_gpu, z32, z64 = z_gpu.double().cpu(), z32.double(), z64.double()
    scale = torch.ones_like(z32)
    scale[..., :4] = z32[..., :4].abs().clamp(min=1.0)
    d = (z_gpu - z32).abs() / scale
    eg = (z_gpu - z64).abs() / scale
    er = (z32 - z64).abs() / scale
    within = (d <= 1e-4).double().mean().item()
    gmax, rmax = eg.max().item(), er.max().item()
    grms, rrms = eg.pow(2).mean().sqrt().item(), er.pow(2).mean().sqrt().item()
    msg = (f'{label}: |gpu-ref32|<=1e-4 on {within * 100:.3f}% of elements (max {d.max().item():.3g}); '
           f'vs fp64: gpu max {gmax:.3g} rms {grms:.3g} | ref32 max {rmax:.3g} rms {rrms:.3g}')
    assert gmax <= 1.25 * rmax + 1e-6 and grms <= 1.25 * rrms + 1e-7, msg
    assert within >= frac, msg
    return msg
