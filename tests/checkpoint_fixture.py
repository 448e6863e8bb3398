"""A reference-format checkpoint for tests: the dict train.py:465-472 saves, with the whole model
pickled as an fp16 models.yolo.Model carrying exactly the reference's attribute tree.

The reference's Model.__init__ (models/yolo.py:509-579) leaves these instance attributes besides
the nn.Module internals: traced, yaml, yaml_file, model, save, names, stride; its layers carry i, f,
type, np (parse_model, yolo.py:806-808).  This package's Model adds a plan cache (`_plans`), which a
reference checkpoint cannot contain, so it is removed before pickling: attempt_load must cope with
the reference's tree as it is.
"""
from __future__ import annotations

import torch

from helpers import model_and_weights

REFERENCE_MODEL_ATTRS = {'traced', 'yaml', 'yaml_file', 'save', 'names', 'stride'}


def write_reference_checkpoint(tmp_path, name='yolov7-train', seed=0):
    """-> (path, sd16): the checkpoint file and the state_dict it holds, upcast to fp32 (what the
    reference's attempt_load sees after .float())."""
    from models.yolo import Model
    _, sd = model_and_weights(name, seed)
    m = Model(name)
    m.load_state_dict(sd)
    m = m.half()
    for k in list(vars(m)):
        if not k.startswith('_') and k not in REFERENCE_MODEL_ATTRS and k != 'training':
            raise AssertionError(f'Model has a non-reference attribute {k!r}')
    del m._plans
    ckpt = {'epoch': -1, 'best_fitness': None, 'training_results': None, 'model': m, 'ema': None,
            'updates': None, 'optimizer': None, 'wandb_id': None}
    path = tmp_path / f'{name}-ref-format.pt'
    torch.save(ckpt, path)
    sd16 = {k: (v.half().float() if v.is_floating_point() else v) for k, v in sd.items()}
    return path, sd16
