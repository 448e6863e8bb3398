"""Loader — mirror of the reference's models/experimental.py entry points on the inference path.

attempt_load(weights, map_location)   models/experimental.py:247-270
Ensemble                              models/experimental.py:69-81

A checkpoint is either the reference's pickled dict ({'model' or 'ema': models.yolo.Model, ...},
train.py:465-472) — unpickled with weights_only=False, so only for trusted local files, exactly as
the reference's torch.load does — or a plain state_dict / {'model': state_dict, 'cfg': ...}
(weights_only=True) for which the architecture must be named (cfg=...).
"""
from __future__ import annotations

import torch
import torch.nn as nn

from models.common import Conv
from models.yolo import Model


class Ensemble(nn.ModuleList):
    """NMS-ensemble of several models: outputs concatenated along the row dimension (experimental.py:69-81)."""

    def forward(self, x, augment=False):
        y = [module(x, augment)[0] for module in self]
        return torch.cat(y, 1), None


def _load_one(w, map_location, cfg):
    if isinstance(w, nn.Module):
        return w
    if isinstance(w, dict):
        ckpt = w
    else:
        try:
            ckpt = torch.load(w, map_location='cpu', weights_only=True)
        except Exception:
            # pickled models.yolo.Model objects (the reference's checkpoint format): trusted files only
            ckpt = torch.load(w, map_location='cpu', weights_only=False)
    if isinstance(ckpt, nn.Module):
        return ckpt
    obj = ckpt.get('ema') or ckpt.get('model') if isinstance(ckpt, dict) and ('ema' in ckpt or 'model' in ckpt) else ckpt
    if isinstance(obj, nn.Module):
        return obj
    sd = obj
    cfg = cfg or (ckpt.get('cfg') if isinstance(ckpt, dict) else None)
    if cfg is None:
        raise ValueError('state_dict checkpoint: pass cfg= (e.g. "yolov7" or a cfg dict/YAML)')
    m = Model(cfg)
    m.load_state_dict({k: v for k, v in sd.items() if k in m.state_dict()}, strict=False)
    return m


def attempt_load(weights, map_location=None, cfg=None):
    """Load a model (or an ensemble) and return it fused, fp32, eval — then bound to `map_location`."""
    model = Ensemble()
    for w in weights if isinstance(weights, list) else [weights]:
        m = _load_one(w, map_location, cfg)
        model.append(m.float().fuse().eval())
    for m in model.modules():
        if type(m) in [nn.Hardswish, nn.LeakyReLU, nn.ReLU, nn.ReLU6, nn.SiLU]:
            m.inplace = True
        elif type(m) is nn.Upsample:
            m.recompute_scale_factor = None
        elif type(m) is Conv:
            m._non_persistent_buffers_set = set()
    if map_location is not None:
        model.to(map_location)
    if len(model) == 1:
        return model[-1]
    print('Ensemble created with %s\n' % weights)
    for k in ['names', 'stride']:
        setattr(model, k, getattr(model[-1], k))
    return model
