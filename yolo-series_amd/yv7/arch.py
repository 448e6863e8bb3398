"""Model graph definitions for the yolov7 family, built as dicts in the reference's cfg schema.

The reference describes each network as a YAML file (`cfg/deploy/yolov7.yaml`,
`cfg/deploy/yolov7-tiny.yaml`, `cfg/deploy/yolov7-w6.yaml`, and the `cfg/training/*` twins that
differ only in the head).  The GPU box has no copy of the reference, so the graphs are generated
here from their building blocks (stem, E-ELAN, MP-downsample, SPPCSPC, route/upsample, heads).
The result is the same dict `yaml.safe_load` returns for those files (module names and string
arguments such as 'None', 'nc', 'anchors', 'nn.LeakyReLU(0.1)' included), so `parse_model`
consumes a generated dict and a user's YAML file identically.  `tests/test_arch.py` pins every
generated graph against the reference YAML when `/root/reference` is present.
"""
from __future__ import annotations

import copy

LEAKY = 'nn.LeakyReLU(0.1)'
UP = [-1, 1, 'nn.Upsample', ['None', 2, 'nearest']]


def _conv(f, c, k=1, s=1, act=None):
    args = [c, k, s] if act is None else [c, k, s, 'None', 1, act]
    return [f, 1, 'Conv', args]


def _elan_backbone(c, out):
    """E-ELAN block of the yolov7/w6 backbone: 2 x 1x1 split, 4 x 3x3 chain, 4-way concat, 1x1 (cfg/deploy/yolov7.yaml:20-27)."""
    return [_conv(-1, c), _conv(-2, c)] + [_conv(-1, c, 3) for _ in range(4)] + \
        [[[-1, -3, -5, -6], 1, 'Concat', [1]], _conv(-1, out)]


def _elan_head(c1, c2, out):
    """E-ELAN-H block of the neck: 6-way concat (cfg/deploy/yolov7.yaml:56-63)."""
    return [_conv(-1, c1), _conv(-2, c1)] + [_conv(-1, c2, 3) for _ in range(4)] + \
        [[[-1, -2, -3, -4, -5, -6], 1, 'Concat', [1]], _conv(-1, out)]


def _mp_down(c, extra=None):
    """MP + strided-conv downsample pair with concat (cfg/deploy/yolov7.yaml:29-34)."""
    cat = [-1, -3] if extra is None else [-1, -3, extra]
    return [[-1, 1, 'MP', []], _conv(-1, c), _conv(-3, c), _conv(-1, c, 3, 2), [cat, 1, 'Concat', [1]]]


def _elan_tiny(c, out, act=LEAKY):
    """yolov7-tiny ELAN: 2 x 1x1, 2 x 3x3, 4-way concat, 1x1 (cfg/deploy/yolov7-tiny.yaml:17-22)."""
    return [_conv(-1, c, act=act), _conv(-2, c, act=act), _conv(-1, c, 3, act=act), _conv(-1, c, 3, act=act),
            [[-1, -2, -3, -4], 1, 'Concat', [1]], _conv(-1, out, act=act)]


def _params(anchors):
    return {'nc': 80, 'depth_multiple': 1.0, 'width_multiple': 1.0, 'anchors': anchors}


def yolov7(head='Detect'):
    """yolov7 P5 (cfg/deploy/yolov7.yaml; head='IDetect' gives cfg/training/yolov7.yaml)."""
    bb = [_conv(-1, 32, 3), _conv(-1, 64, 3, 2), _conv(-1, 64, 3), _conv(-1, 128, 3, 2)]
    bb += _elan_backbone(64, 256)
    bb += _mp_down(128) + _elan_backbone(128, 512)
    bb += _mp_down(256) + _elan_backbone(256, 1024)
    bb += _mp_down(512) + _elan_backbone(256, 1024)
    hd = [[-1, 1, 'SPPCSPC', [512]]]
    hd += [_conv(-1, 256), UP, _conv(37, 256), [[-1, -2], 1, 'Concat', [1]]] + _elan_head(256, 128, 256)
    hd += [_conv(-1, 128), UP, _conv(24, 128), [[-1, -2], 1, 'Concat', [1]]] + _elan_head(128, 64, 128)
    hd += _mp_down(128, 63) + _elan_head(256, 128, 256)
    hd += _mp_down(256, 51) + _elan_head(512, 256, 512)
    hd += [[75, 1, 'RepConv', [256, 3, 1]], [88, 1, 'RepConv', [512, 3, 1]], [101, 1, 'RepConv', [1024, 3, 1]]]
    hd += [[[102, 103, 104], 1, head, ['nc', 'anchors']]]
    d = _params([[12, 16, 19, 36, 40, 28], [36, 75, 76, 55, 72, 146], [142, 110, 192, 243, 459, 401]])
    d['backbone'], d['head'] = bb, hd
    return d


def yolov7_tiny(head='Detect'):
    """yolov7-tiny (cfg/deploy/yolov7-tiny.yaml; head='IDetect' gives the training twin)."""
    L = LEAKY
    bb = [_conv(-1, 32, 3, 2, L), _conv(-1, 64, 3, 2, L)] + _elan_tiny(32, 64)
    bb += [[-1, 1, 'MP', []]] + _elan_tiny(64, 128)
    bb += [[-1, 1, 'MP', []]] + _elan_tiny(128, 256)
    bb += [[-1, 1, 'MP', []]] + _elan_tiny(256, 512)
    hd = [_conv(-1, 256, act=L), _conv(-2, 256, act=L), [-1, 1, 'SP', [5]], [-2, 1, 'SP', [9]],
          [-3, 1, 'SP', [13]], [[-1, -2, -3, -4], 1, 'Concat', [1]], _conv(-1, 256, act=L),
          [[-1, -7], 1, 'Concat', [1]], _conv(-1, 256, act=L)]
    hd += [_conv(-1, 128, act=L), UP, _conv(21, 128, act=L), [[-1, -2], 1, 'Concat', [1]]] + _elan_tiny(64, 128)
    hd += [_conv(-1, 64, act=L), UP, _conv(14, 64, act=L), [[-1, -2], 1, 'Concat', [1]]] + _elan_tiny(32, 64)
    hd += [_conv(-1, 128, 3, 2, L), [[-1, 47], 1, 'Concat', [1]]] + _elan_tiny(64, 128)
    hd += [_conv(-1, 256, 3, 2, L), [[-1, 37], 1, 'Concat', [1]]] + _elan_tiny(128, 256)
    hd += [_conv(57, 128, 3, 1, L), _conv(65, 256, 3, 1, L), _conv(73, 512, 3, 1, L)]
    hd += [[[74, 75, 76], 1, head, ['nc', 'anchors']]]
    d = _params([[10, 13, 16, 30, 33, 23], [30, 61, 62, 45, 59, 119], [116, 90, 156, 198, 373, 326]])
    d['backbone'], d['head'] = bb, hd
    return d


def yolov7_w6(head='Detect'):
    """yolov7-w6 P6 (cfg/deploy/yolov7-w6.yaml; head='IAuxDetect' gives cfg/training/yolov7-w6.yaml)."""
    bb = [[-1, 1, 'ReOrg', []], _conv(-1, 64, 3), _conv(-1, 128, 3, 2)] + _elan_backbone(64, 128)
    bb += [_conv(-1, 256, 3, 2)] + _elan_backbone(128, 256)
    bb += [_conv(-1, 512, 3, 2)] + _elan_backbone(256, 512)
    bb += [_conv(-1, 768, 3, 2)] + _elan_backbone(384, 768)
    bb += [_conv(-1, 1024, 3, 2)] + _elan_backbone(512, 1024)
    hd = [[-1, 1, 'SPPCSPC', [512]]]
    hd += [_conv(-1, 384), UP, _conv(37, 384), [[-1, -2], 1, 'Concat', [1]]] + _elan_head(384, 192, 384)
    hd += [_conv(-1, 256), UP, _conv(28, 256), [[-1, -2], 1, 'Concat', [1]]] + _elan_head(256, 128, 256)
    hd += [_conv(-1, 128), UP, _conv(19, 128), [[-1, -2], 1, 'Concat', [1]]] + _elan_head(128, 64, 128)
    hd += [_conv(-1, 256, 3, 2), [[-1, 71], 1, 'Concat', [1]]] + _elan_head(256, 128, 256)
    hd += [_conv(-1, 384, 3, 2), [[-1, 59], 1, 'Concat', [1]]] + _elan_head(384, 192, 384)
    hd += [_conv(-1, 512, 3, 2), [[-1, 47], 1, 'Concat', [1]]] + _elan_head(512, 256, 512)
    hd += [_conv(83, 256, 3), _conv(93, 512, 3), _conv(103, 768, 3), _conv(113, 1024, 3)]
    if head == 'IAuxDetect':
        hd += [_conv(83, 320, 3), _conv(71, 640, 3), _conv(59, 960, 3), _conv(47, 1280, 3)]
        hd += [[[114, 115, 116, 117, 118, 119, 120, 121], 1, head, ['nc', 'anchors']]]
    else:
        hd += [[[114, 115, 116, 117], 1, head, ['nc', 'anchors']]]
    d = _params([[19, 27, 44, 40, 38, 94], [96, 68, 86, 152, 180, 137], [140, 301, 303, 264, 238, 542],
                 [436, 615, 739, 380, 925, 792]])
    d['backbone'], d['head'] = bb, hd
    return d


# name -> (builder, head) ; "-train" variants mirror cfg/training/*.yaml
REGISTRY = {
    'yolov7': (yolov7, 'Detect'),
    'yolov7-tiny': (yolov7_tiny, 'Detect'),
    'yolov7-w6': (yolov7_w6, 'Detect'),
    'yolov7-train': (yolov7, 'IDetect'),
    'yolov7-tiny-train': (yolov7_tiny, 'IDetect'),
    'yolov7-w6-train': (yolov7_w6, 'IAuxDetect'),
}


def get_cfg(name: str) -> dict:
    """Return a fresh cfg dict for a registered model name (e.g. 'yolov7', 'yolov7.yaml', 'yolov7-tiny')."""
    key = name[:-5] if name.endswith('.yaml') else name
    key = key.split('/')[-1]
    if key not in REGISTRY:
        raise KeyError(f'unknown model cfg {name!r}; known: {sorted(REGISTRY)}')
    fn, head = REGISTRY[key]
    return copy.deepcopy(fn(head))
