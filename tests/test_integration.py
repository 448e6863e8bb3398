"""INTEGRATION.md's reference-side ctypes stub is real code: it parses, its yv7_nms call passes
exactly the arguments the C prototype declares, and on the GPU it returns what the product's
non_max_suppression returns (bit for bit)."""
import ast
import os
import re

import pytest
import torch

from yv7 import _lib

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _stub_source():
    md = open(os.path.join(ROOT, 'INTEGRATION.md')).read()
    sec = md[md.index('## Binding stub'):]
    return re.search(r'```python\n(.*?)```', sec, re.S).group(1)


def test_stub_parses_and_matches_the_prototype():
    src = _stub_source()
    tree = ast.parse(src)
    calls = [n for n in ast.walk(tree) if isinstance(n, ast.Call) and isinstance(n.func, ast.Attribute)
             and n.func.attr == 'yv7_nms']
    assert len(calls) == 1
    argtypes = next(n for n in ast.walk(tree) if isinstance(n, ast.Assign)
                    and getattr(n.targets[0], 'attr', None) == 'argtypes')
    n_decl = len(argtypes.value.elts)
    assert len(calls[0].args) == n_decl == len(_lib.SIGNATURES['yv7_nms'][1])


@pytest.mark.gpu
def test_stub_runs_like_the_product():
    from utils.general import non_max_suppression
    from test_gpu_nms import _clustered_z
    ns = {'LIBYV7': _lib.LIB_PATH}
    exec(compile(_stub_source(), 'INTEGRATION.md', 'exec'), ns)
    z = _clustered_z(3, 4000, 80, seed=17).to('cuda:0')
    for kw in (dict(), dict(multi_label=True, conf_thres=0.3, iou_thres=0.6), dict(classes=[0, 3, 7]),
               dict(agnostic=True)):
        a = ns['non_max_suppression'](z, **kw)
        b = non_max_suppression(z, **kw)
        assert len(a) == len(b) and all(torch.equal(x, y) for x, y in zip(a, b)), kw
