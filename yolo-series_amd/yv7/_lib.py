"""ctypes binding of the C ABI in include/yv7.h (libyv7.so, built in-tree for gfx950).

No torch types cross the boundary: tensors go over as device pointers (`data_ptr()`) and the
current HIP stream as a raw handle.  Any non-zero return code becomes a RuntimeError carrying
yv7_last_error(), the reference's error style (assert / raise, e.g. models/common.py:475).
There is deliberately no CPU fallback: if the library is missing the product path fails loudly.
"""
from __future__ import annotations

import ctypes
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, 'libyv7.so')

ABI_VERSION = 4
BORDER = 1          # zero frame around every workspace tensor (YV7_BORDER)
DT_F32, DT_F16 = 0, 1
ACT_NONE, ACT_SILU, ACT_LEAKY = 0, 1, 2
OP_INPUT, OP_CONV, OP_MAXPOOL, OP_UPSAMPLE, OP_COPY, OP_DETECT, OP_STEM = 0, 1, 2, 3, 4, 5, 6
WFMT_PLAN, WFMT_FP8 = 0, 1


class TensorDesc(ctypes.Structure):
    _fields_ = [('channels', ctypes.c_int32), ('shift', ctypes.c_int32)]


class OpDesc(ctypes.Structure):
    _fields_ = [('kind', ctypes.c_int32),
                ('src', ctypes.c_int32), ('src_coff', ctypes.c_int32), ('cin', ctypes.c_int32),
                ('dst', ctypes.c_int32), ('dst_coff', ctypes.c_int32), ('cout', ctypes.c_int32),
                ('k', ctypes.c_int32), ('s', ctypes.c_int32), ('pad', ctypes.c_int32), ('act', ctypes.c_int32),
                ('level', ctypes.c_int32),
                ('w_off', ctypes.c_int64), ('b_off', ctypes.c_int64),
                ('cout2', ctypes.c_int32), ('act2', ctypes.c_int32),
                ('w2_off', ctypes.c_int64), ('b2_off', ctypes.c_int64),
                ('wfmt', ctypes.c_int32), ('xscale', ctypes.c_float), ('s_off', ctypes.c_int64),
                ('pool', ctypes.c_int32), ('reserved', ctypes.c_int32)]


class NetDesc(ctypes.Structure):
    _fields_ = [('abi_version', ctypes.c_int32), ('dtype', ctypes.c_int32),
                ('n_tensors', ctypes.c_int32), ('tensors', ctypes.POINTER(TensorDesc)),
                ('n_ops', ctypes.c_int32), ('ops', ctypes.POINTER(OpDesc)),
                ('nl', ctypes.c_int32), ('na', ctypes.c_int32), ('no', ctypes.c_int32),
                ('stride', ctypes.POINTER(ctypes.c_float)), ('anchor_grid', ctypes.POINTER(ctypes.c_float)),
                ('max_shift', ctypes.c_int32)]


_vp, _i, _i64, _sz, _f = ctypes.c_void_p, ctypes.c_int, ctypes.c_int64, ctypes.c_size_t, ctypes.c_float

# name -> (restype, argtypes); every symbol include/yv7.h declares
SIGNATURES = {
    'yv7_abi_version': (ctypes.c_int32, []),
    'yv7_last_error': (ctypes.c_char_p, []),
    'yv7_plan_create': (_i, [ctypes.POINTER(NetDesc), _vp, _sz, _i, ctypes.POINTER(_vp)]),
    'yv7_plan_destroy': (None, [_vp]),
    'yv7_workspace_bytes': (_sz, [_vp, _i, _i, _i]),
    'yv7_workspace_forget': (_i, [_vp, _vp, _sz]),
    'yv7_set_op_variant': (_i, [_vp, _i, _i]),
    'yv7_num_rows': (_i64, [_vp, _i, _i]),
    'yv7_forward': (_i, [_vp, _vp, _i, _i, _i, _i, _vp, _vp, _vp, _vp, _sz, _vp]),
    'yv7_op_kernels': (_i, [_vp, _i, _i, _i, _i, ctypes.c_char_p, _sz]),
    'yv7_profile_enable': (_i, [_vp, _i]),
    'yv7_profile_read': (_i, [_vp, ctypes.POINTER(_i), ctypes.POINTER(ctypes.c_float)]),
    'yv7_tensor_info': (_i, [_vp, _i, _i, _i, _i, ctypes.POINTER(_i64), ctypes.POINTER(_i64)]),
    'yv7_f8_scratch_info': (_i, [_vp, _i, _i, _i, ctypes.POINTER(_i64), ctypes.POINTER(_i64)]),
    'yv7_nms_workspace_bytes': (_sz, [_i, _i, _i, _i, _i]),
    'yv7_nms': (_i, [_vp, _vp, _i, _i, _i, _f, _f, _i, _i, _vp, _i, _i, _i, _vp, _vp, _vp, _vp, _sz, _vp]),
    'yv7_end2end_workspace_bytes': (_sz, [_i, _i, _i, _i]),
    'yv7_end2end': (_i, [_vp, _i, _i, _i, _f, _f, _i, _vp, _vp, _vp, _vp, _vp, _sz, _vp]),
    'yv7_letterbox_workspace_bytes': (_sz, [_i, _i]),
    'yv7_letterbox': (_i, [_vp, _i, _i, _i, _i, _i, _i, _i, _i, _i, _i, _i, _i, _i, _vp, _vp, _sz, _vp]),
}

_LIB = None


def lib():
    """Load libyv7.so (raises if it has not been built: there is no fallback path)."""
    global _LIB
    if _LIB is None:
        if not os.path.exists(LIB_PATH):
            raise RuntimeError(f'libyv7.so not found at {LIB_PATH}: build it with '
                               f'`make -C {os.path.dirname(_HERE)}` (or __graft_entry__.build())')
        L = ctypes.CDLL(LIB_PATH)
        for name, (res, args) in SIGNATURES.items():
            fn = getattr(L, name)
            fn.restype = res
            fn.argtypes = args
        if L.yv7_abi_version() != ABI_VERSION:
            raise RuntimeError('libyv7.so ABI version mismatch')
        _LIB = L
    return _LIB


def check(rc: int, what: str):
    if rc != 0:
        msg = lib().yv7_last_error().decode(errors='replace')
        raise RuntimeError(f'{what} failed (code {rc}): {msg}')
