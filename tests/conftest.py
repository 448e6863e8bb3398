"""Test configuration: import paths and the `gpu` marker.

`-m "not gpu"` runs here (no GPU): oracle vs golden fixtures / known answers, host logic, C-ABI
loading.  `-m gpu` runs on an MI355X: HIP path (through the C ABI) vs the oracle.
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, 'yolo-series_amd')
for p in (PKG, ROOT):
    if p not in sys.path:
        sys.path.insert(0, p)

import pytest  # noqa: E402


def pytest_configure(config):
    config.addinivalue_line('markers', 'gpu: needs an MI355X (gfx950) GPU')


def pytest_collection_modifyitems(config, items):
    import torch
    if torch.cuda.is_available():
        return
    skip = pytest.mark.skip(reason='no GPU in this environment')
    for item in items:
        if 'gpu' in item.keywords:
            item.add_marker(skip)
