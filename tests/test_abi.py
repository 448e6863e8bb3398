"""The C-ABI library loads and exports exactly what include/yv7.h declares (CPU only, no compute)."""
import ctypes
import os
import re
import subprocess

import pytest

from yv7 import _lib

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, 'include', 'yv7.h')


def declared_functions():
    src = open(HEADER).read()
    src = re.sub(r'/\*.*?\*/', '', src, flags=re.S)
    return sorted(set(re.findall(r'\b(yv7_[a-z0-9_]+)\s*\(', src)))


def test_header_declares_the_expected_entry_points():
    names = declared_functions()
    for required in ('yv7_plan_create', 'yv7_forward', 'yv7_nms', 'yv7_workspace_bytes', 'yv7_plan_destroy',
                     'yv7_last_error', 'yv7_end2end'):
        assert required in names


def test_library_exports_every_declared_symbol():
    lib = ctypes.CDLL(_lib.LIB_PATH)
    for name in declared_functions():
        assert hasattr(lib, name), name
    # the Python binding covers every declared symbol with a signature
    assert set(declared_functions()) == set(_lib.SIGNATURES)


def test_abi_version_and_host_only_entry_points():
    L = _lib.lib()
    assert L.yv7_abi_version() == _lib.ABI_VERSION
    assert L.yv7_nms_workspace_bytes(2, 25200, 85, 0, 30000) > 0
    assert L.yv7_nms_workspace_bytes(0, 25200, 85, 0, 30000) == 0
    assert L.yv7_end2end_workspace_bytes(1, 1000, 85, 100) > 0
    # argument errors are reported, not thrown, before any device is touched
    rc = L.yv7_plan_create(None, None, 0, 0, ctypes.byref(ctypes.c_void_p()))
    assert rc == -1 and b'null' in L.yv7_last_error()
    d = _lib.NetDesc()
    d.abi_version = 999
    rc = L.yv7_plan_create(ctypes.byref(d), None, 0, 0, ctypes.byref(ctypes.c_void_p()))
    assert rc == -4 and b'abi_version' in L.yv7_last_error()
    rc = L.yv7_nms(None, None, 1, 10, 85, 0.25, 0.45, 0, 0, None, 0, 300, 30000, None, None, None, None, 0, None)
    assert rc == -1


def test_struct_layout_matches_c(tmp_path):
    """ctypes mirrors of yv7_tensor_desc / yv7_op_desc / yv7_net_desc have the C sizes and offsets."""
    prog = tmp_path / 'layout.c'
    prog.write_text('#include <stdio.h>\n#include <stddef.h>\n#include "yv7.h"\n'
                    'int main(void){printf("%zu %zu %zu %zu %zu %zu\\n", sizeof(yv7_tensor_desc), '
                    'sizeof(yv7_op_desc), offsetof(yv7_op_desc, w_off), sizeof(yv7_net_desc), '
                    'offsetof(yv7_net_desc, stride), offsetof(yv7_net_desc, max_shift));return 0;}\n')
    exe = tmp_path / 'layout'
    subprocess.check_call(['gcc', '-I', os.path.join(ROOT, 'include'), str(prog), '-o', str(exe)])
    got = [int(v) for v in subprocess.check_output([str(exe)]).split()]
    want = [ctypes.sizeof(_lib.TensorDesc), ctypes.sizeof(_lib.OpDesc), _lib.OpDesc.w_off.offset,
            ctypes.sizeof(_lib.NetDesc), _lib.NetDesc.stride.offset, _lib.NetDesc.max_shift.offset]
    assert got == want


def test_library_is_gfx950_code_object():
    out = subprocess.run(['/opt/rocm/lib/llvm/bin/llvm-objdump', '--offloading', _lib.LIB_PATH],
                         capture_output=True, text=True)
    if out.returncode != 0:
        pytest.skip('llvm-objdump --offloading unavailable')
    assert 'gfx950' in out.stdout + out.stderr
