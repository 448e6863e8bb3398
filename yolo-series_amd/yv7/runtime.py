"""Plan: a compiled network resident on one MI355X, driven through the C ABI (libyv7).

Plan.from_model(model, device, dtype) compiles the model (yv7.graph), packs its weights once and
creates the libyv7 plan on that device (weights copied into plan-owned HBM).  Plan.forward(x)
allocates nothing after the first call for a given (B, H, W): the workspace and outputs are cached,
and the whole network is one yv7_forward call on the current stream.
"""
from __future__ import annotations

import ctypes
import math
import weakref

import torch

from yv7 import _lib as L
from yv7.graph import compile_model


class _RowScores:
    """z tensor -> the yv7_row_best records its forward wrote (include/yv7.h), so that
    non_max_suppression(pred) can skip re-reading every row of z.  An entry is used only for the very
    tensor object the forward returned and only while its version counter is unchanged (any in-place
    edit of z bumps it), so a modified z always takes the full path."""

    def __init__(self):
        self._m = {}

    def attach(self, z, rowbest):
        for k in [k for k, (ref, _, _) in self._m.items() if ref() is None]:
            del self._m[k]
        self._m[id(z)] = (weakref.ref(z), z._version, rowbest)

    def lookup(self, z):
        e = self._m.get(id(z))
        if e is None:
            return None
        ref, ver, rowbest = e
        return rowbest if ref() is z and z._version == ver else None


row_scores = _RowScores()


def _demangle(sym: str) -> str:
    """Itanium C++ demangling through libstdc++'s __cxa_demangle (rocprofv3 reports some names mangled)."""
    try:
        cxx = ctypes.CDLL('libstdc++.so.6')
        f = cxx.__cxa_demangle
        f.restype = ctypes.c_void_p
        st = ctypes.c_int()
        p = f(sym.encode(), None, None, ctypes.byref(st))
        if st.value != 0 or not p:
            return sym
        out = ctypes.string_at(p).decode()
        ctypes.CDLL(None).free(ctypes.c_void_p(p))
        return out
    except (OSError, AttributeError):
        return sym


def kernel_key(name: str) -> str:
    """A kernel instantiation's short key, the same for the names yv7_op_kernels reports and the
    Kernel_Name column of a rocprofv3 trace: 'void yv7::(anonymous namespace)::k<1, 2>(yv7::ConvParams)'
    -> 'k<1, 2>'."""
    n = name.strip()
    if n.startswith('_Z'):
        n = _demangle(n)
    if n.startswith('void '):
        n = n[5:]
    for pre in ('yv7::(anonymous namespace)::', 'yv7::'):
        n = n.replace(pre, '')
    depth = 0
    for i, ch in enumerate(n):   # drop the parameter list: the first '(' outside template brackets
        if ch == '<':
            depth += 1
        elif ch == '>':
            depth -= 1
        elif ch == '(' and depth == 0:
            return n[:i]
    return n


class Plan:
    def __init__(self, graph, device, weights: torch.Tensor):
        self.graph = graph
        self.device = torch.device(device)
        self.dtype = graph.dtype
        self.nl, self.na, self.no = graph.nl, graph.na, graph.no
        lib = L.lib()
        self._tensors = (L.TensorDesc * len(graph.tensors))(*[L.TensorDesc(c, s) for c, s in graph.tensors])
        ops = []
        for o in graph.ops:
            d = dict(kind=0, src=0, src_coff=0, cin=0, dst=0, dst_coff=0, cout=0, k=1, s=1, pad=0, act=0, level=0,
                     w_off=0, b_off=0, cout2=0, act2=0, w2_off=0, b2_off=0, wfmt=0, xscale=0.0, s_off=0, pool=0)
            d.update({k: v for k, v in o.items() if k in d})
            ops.append(L.OpDesc(**d))
        self._ops = (L.OpDesc * len(ops))(*ops)
        self._stride = (ctypes.c_float * graph.nl)(*graph.stride)
        self._anchors = (ctypes.c_float * len(graph.anchor_grid))(*graph.anchor_grid)
        desc = L.NetDesc(L.ABI_VERSION, graph.dtype, len(graph.tensors), self._tensors, len(ops), self._ops,
                         graph.nl, graph.na, graph.no, self._stride, self._anchors, graph.max_shift)
        self._desc = desc
        h = ctypes.c_void_p()
        dev_index = self.device.index if self.device.index is not None else torch.cuda.current_device()
        with torch.cuda.device(dev_index):
            L.check(lib.yv7_plan_create(ctypes.byref(desc), weights.data_ptr(), weights.numel(), dev_index,
                                        ctypes.byref(h)), 'yv7_plan_create')
        self._h = h
        self._ws = {}
        self.variants = {}
        self.weight_bytes = weights.numel()

    @classmethod
    def from_model(cls, model, device, dtype=torch.float32, weights=None, calib=None):
        """dtype: torch.float32 / torch.float16, or 'fp8' (fp16 plan whose 1x1 convs run in e4m3, see
        fp8_from_model; `calib` then gives its calibration frames)."""
        if isinstance(dtype, str) and dtype == 'fp8':
            return cls.fp8_from_model(model, device, calib=calib)
        code = L.DT_F16 if dtype == torch.float16 else L.DT_F32
        g = compile_model(model, code)
        blob = g.weight_blob() if weights is None else weights
        blob = blob.to(device)
        return cls(g, device, blob)

    @classmethod
    def fp8_from_model(cls, model, device, calib=None, min_cout=None):
        """BASELINE configs[4]: the fp16 plan with every 1x1 stride-1 conv (the Detect head excepted) on
        OCP e4m3 weights (per-output-channel scales) and e4m3 activations (per-tensor power-of-two
        scales), through the block-scaled fp8 MFMA (csrc/conv_f8.hip); scales from fp8_scales.
        (Multi-GPU: yv7.dist.broadcast_fp8_plan calibrates on rank 0 and broadcasts.)"""
        g = compile_model(model, L.DT_F16, fp8=cls.fp8_scales(model, device, calib, min_cout))
        return cls(g, device, g.weight_blob().to(device))

    @classmethod
    def fp8_scales(cls, model, device, calib=None, min_cout=None):
        """{op index: activation scale} of the fp8 plan's e4m3 convs, from calibration: the fp16 plan runs
        `calib` ([B,3,H,W] frames in [0,1]; default: 2 seeded synthetic frames at the model's native size)
        and each fp8 op's input amax sets xscale = 2**ceil(log2(amax / 448)), so the largest calibrated
        value still fits e4m3.  min_cout: which eligible 1x1 convs go fp8 (default
        yv7.graph.FP8_MIN_COUT; 0 = all of them)."""
        from yv7.graph import FP8_MIN_COUT, fp8_candidates
        min_cout = FP8_MIN_COUT if min_cout is None else min_cout
        base = cls.from_model(model, device, torch.float16)
        if calib is None:
            from yv7.synthetic import synthetic_frames
            hw = 1280 if float(model.stride.max()) >= 64 else 640
            calib = synthetic_frames(2, hw, hw, seed=4321)
        x = calib.to(base.device).half()
        B, _, H, W = x.shape
        N = base.num_rows(H, W)
        z = torch.empty((B, N, base.no), dtype=torch.float32, device=base.device)
        base.forward_into(x, z)
        scales = {}
        for i in fp8_candidates(base.graph, min_cout):
            o = base.graph.ops[i]
            v = base.tensor_view(o['src'], B, H, W)[..., o['src_coff']:o['src_coff'] + o['cin']]
            amax = float(v.abs().max().float())
            scales[i] = 2.0 ** math.ceil(math.log2(amax / 448.0)) if amax > 0 else 1.0
        del base
        return scales

    def __del__(self):
        self._ws = {}
        h = getattr(self, '_h', None)
        if h is not None and h.value:
            try:
                L.lib().yv7_plan_destroy(h)
            except Exception:
                pass

    # ------------------------------------------------------------------
    def num_rows(self, H, W):
        return int(L.lib().yv7_num_rows(self._h, H, W))

    def workspace(self, B, H, W, slot=0):
        """The forward workspace for a [B,3,H,W] batch; `slot` > 0 gives further ones, so that
        sub-batches can run concurrently on their own streams."""
        key = (B, H, W, slot)
        ws = self._ws.get(key)
        if ws is None:
            nbytes = L.lib().yv7_workspace_bytes(self._h, B, H, W)
            if nbytes == 0:
                L.check(-2, f'yv7_workspace_bytes(B={B}, H={H}, W={W})')
            for k in [k for k in self._ws if k[:3] != (B, H, W)]:   # keep one shape resident
                self._drop_workspace(k)
            ws = torch.empty(nbytes, dtype=torch.uint8, device=self.device)
            self._ws[key] = ws
        return ws

    def _drop_workspace(self, key):
        """Give a workspace back to the allocator.  libyv7 trusts the zero frame of a workspace it has
        seen (include/yv7.h), so it is told first: the allocator may hand the same block back later,
        after other tensors have written into it, and the next forward there must clear it again."""
        ws = self._ws.pop(key)
        L.check(L.lib().yv7_workspace_forget(self._h, ws.data_ptr(), ws.numel()), 'yv7_workspace_forget')

    def set_op_variant(self, op, variant):
        """Force op `op`'s kernel configuration (yv7_set_op_variant; 0 = tuned dispatch).  The split-K
        scratch depends on it, so the cached workspaces are dropped."""
        L.check(L.lib().yv7_set_op_variant(self._h, int(op), int(variant)), f'yv7_set_op_variant(op {op}, {variant})')
        self.variants[int(op)] = int(variant)
        for k in list(self._ws):
            self._drop_workspace(k)

    def tensor_view(self, tensor_id, B, H, W):
        """NHWC view of an intermediate activation tensor of the last forward (debug / per-layer parity)."""
        off = ctypes.c_int64()
        dims = (ctypes.c_int64 * 4)()
        L.check(L.lib().yv7_tensor_info(self._h, tensor_id, B, H, W, ctypes.byref(off), dims), 'yv7_tensor_info')
        ws = self.workspace(B, H, W)
        es = 2 if self.dtype == L.DT_F16 else 4
        n = dims[0] * dims[1] * dims[2] * dims[3]
        t = ws[off.value:off.value + n * es].view(torch.float16 if es == 2 else torch.float32)
        bd = L.BORDER   # bordered layout (include/yv7.h YV7_BORDER): return the image interior
        return t.view(dims[0], dims[1], dims[2], dims[3])[:, bd:dims[1] - bd, bd:dims[2] - bd]

    def f8_scratch(self, B, H, W):
        """uint8 view of the fp8 staging buffer (the last FP8 op's e4m3 input after a forward), or None."""
        off, n = ctypes.c_int64(), ctypes.c_int64()
        L.check(L.lib().yv7_f8_scratch_info(self._h, B, H, W, ctypes.byref(off), ctypes.byref(n)),
                'yv7_f8_scratch_info')
        if n.value == 0:
            return None
        return self.workspace(B, H, W)[off.value:off.value + n.value]

    def layer_output(self, layer_i, B, H, W):
        """NCHW fp32 copy of layer `layer_i`'s output from the last forward."""
        t, coff, c = self.graph.layer_tensor[layer_i]
        return self.tensor_view(t, B, H, W)[..., coff:coff + c].permute(0, 3, 1, 2).float().contiguous()

    # ------------------------------------------------------------------ live per-op timing
    def profile_enable(self, max_forwards):
        L.check(L.lib().yv7_profile_enable(self._h, int(max_forwards)), 'yv7_profile_enable')

    def profile_read(self):
        """(number of recorded forwards, per-op milliseconds summed over them)."""
        n = ctypes.c_int()
        ms = (ctypes.c_float * len(self.graph.ops))()
        L.check(L.lib().yv7_profile_read(self._h, ctypes.byref(n), ms), 'yv7_profile_read')
        return n.value, list(ms)

    def op_kernels(self, B, H, W, x_dtype=None):
        """Per op, the kernel names (rocprofv3's demangled symbols) the dispatch launches for a
        [B,3,H,W] forward (yv7_op_kernels: a dry run, nothing executes); [] for an op without a
        kernel of its own (the later pools of the SPPCSPC cascade)."""
        buf = ctypes.create_string_buffer(1 << 20)
        with torch.cuda.device(self.device):
            xdt = L.DT_F16 if x_dtype in (None, torch.float16) else L.DT_F32
            L.check(L.lib().yv7_op_kernels(self._h, B, H, W, xdt, buf, len(buf)), 'yv7_op_kernels')
        out = [[] for _ in self.graph.ops]
        for line in buf.value.decode().splitlines():
            i, _, names = line.partition('\t')
            out[int(i)] = names.split('|') if names else []
        return out

    def op_costs(self, B, H, W, x_bytes=4, with_raw=True):
        """Per op: (kind, algorithmic FLOPs, algorithmic HBM bytes) for a [B,3,H,W] batch.

        Bytes follow the layer-boundary model: every op reads its input slice once and
        writes its output once, weights once per batch; concat costs nothing; the head writes z in
        fp32 (and the raw logits, also fp32, which the reference returns as xs)."""
        es = 2 if self.dtype == L.DT_F16 else 4
        out = []
        for o in self.graph.ops:
            kind = o['kind']
            if kind == L.OP_STEM:
                # cin 12: the w6 front end, conv A on the 2x space-to-depth image (ReOrg fused)
                sa, cin = o['s'], o['cin']
                r = 2 if cin == 12 else 1
                Ha, Wa = H // r // sa, W // r // sa
                ca, cb = o['cout'], o['cout2']
                flops = 2.0 * B * Ha * Wa * ca * 9 * cin + 2.0 * B * (Ha // 2) * (Wa // 2) * cb * 9 * ca
                # reference-boundary bytes of the two layers it replaces (input read, A write + read, B write)
                by = B * 3 * H * W * x_bytes + 2 * B * Ha * Wa * ca * es + B * (Ha // 2) * (Wa // 2) * cb * es
                out.append((kind, flops, by))
                continue
            if kind == L.OP_INPUT:
                sh = self.graph.tensors[o['dst']][1]
                npx = B * (H >> sh) * (W >> sh)
                out.append((kind, 0.0, B * 3 * H * W * x_bytes + npx * self.graph.tensors[o['dst']][0] * es))
                continue
            si = self.graph.tensors[o['src']][1]
            Hi, Wi = H >> si, W >> si
            k, s, pad = o.get('k', 1), o.get('s', 1), o.get('pad', 0)
            Ho, Wo = (Hi + 2 * pad - k) // s + 1, (Wi + 2 * pad - k) // s + 1
            if kind in (L.OP_CONV, L.OP_DETECT):
                cin, cout = o['cin'], o['cout']
                flops = 2.0 * B * Ho * Wo * cout * k * k * cin
                wbytes = cout * k * k * cin * es + cout * 4
                obytes = B * Ho * Wo * cout * (es if kind == L.OP_CONV else (8 if with_raw else 4))
                # an MP folded into the conv (pool 2): the reference-boundary bytes of both layers, i.e.
                # also the pooled tensor's write and re-read
                mp = 2 * B * Ho * Wo * cin * es if o.get('pool', 0) == 2 else 0
                out.append((kind, flops, B * Hi * Wi * cin * es + obytes + wbytes + mp))
            elif kind == L.OP_MAXPOOL:
                c = o['cout']
                out.append((kind, 0.0, B * Hi * Wi * c * es + B * Ho * Wo * c * es))
            elif kind == L.OP_UPSAMPLE:
                c = o['cout']
                out.append((kind, 0.0, B * Hi * Wi * c * es + B * 4 * Hi * Wi * c * es))
            else:
                c = o['cout']
                out.append((kind, 0.0, 2 * B * Hi * Wi * c * es))
        return out

    def forward_into(self, x, z, raw=None, stream=None, rowbest=None, ws_slot=0):
        """Forward into caller buffers; rowbest (optional): [B, N, 4] 32-bit yv7_row_best records.
        stream: a torch.cuda.Stream (default: the current stream); on a side stream every buffer the
        forward touches is recorded on it, so the allocator cannot reuse it before the forward is done."""
        B, C, H, W = x.shape
        if C != 3:
            raise ValueError(f'expected a [B,3,H,W] image batch, got {tuple(x.shape)}')
        if x.dtype not in (torch.float32, torch.float16):
            x = x.float()
        x = x.contiguous()
        ws = self.workspace(B, H, W, ws_slot)
        xdt = L.DT_F16 if x.dtype == torch.float16 else L.DT_F32
        cur = torch.cuda.current_stream(self.device)
        if stream is None:
            stream = cur
        if stream != cur:
            for t in (x, z, raw, rowbest, ws):
                if t is not None:
                    t.record_stream(stream)
        rc = L.lib().yv7_forward(self._h, x.data_ptr(), xdt, B, H, W, z.data_ptr(),
                                 raw.data_ptr() if raw is not None else None,
                                 rowbest.data_ptr() if rowbest is not None else None, ws.data_ptr(), ws.numel(),
                                 stream.cuda_stream)
        L.check(rc, 'yv7_forward')

    def forward(self, x, want_raw=True):
        """x [B,3,H,W] on the plan's device -> (z [B,N,no] fp32, xs: list of [B,na,ny,nx,no] fp32)."""
        if x.device != self.device and not (self.device.index is None and x.is_cuda):
            raise RuntimeError(f'input on {x.device}, plan on {self.device}')
        B, _, H, W = x.shape
        N = self.num_rows(H, W)
        if N <= 0:
            L.check(-2, f'yv7_num_rows(H={H}, W={W})')
        z = torch.empty((B, N, self.no), dtype=torch.float32, device=x.device)
        raw = torch.empty((B * N * self.no,), dtype=torch.float32, device=x.device) if want_raw else None
        rowbest = torch.empty((B, N, 4), dtype=torch.float32, device=x.device)
        self.forward_into(x, z, raw, rowbest=rowbest)
        row_scores.attach(z, rowbest)
        xs = None
        if want_raw:
            xs, o = [], 0
            for lvl in range(self.nl):
                s = int(self.graph.stride[lvl])
                ny, nx = H // s, W // s
                n = B * self.na * ny * nx * self.no
                xs.append(raw[o:o + n].view(B, self.na, ny, nx, self.no))
                o += n
        return z, xs


class Inflight:
    """Several batches in flight on one plan (serving schedule; detect.py:142-153 done per batch).

    Batch k runs its forward and batched NMS on HIP stream k % S with its own workspace slot and its
    own z / row-record / detection buffers, so batch k+1's kernels fill batch k's kernel tails, its
    low-resolution layers and its few-block NMS kernels (measured on MI355X, yolov7 bs32 640 fp16:
    S = 1 -> 5.6k, 2 -> 6.2k, 3 -> 6.3k img/s).  Results are bit-identical to running the batches one
    after another (tests/test_gpu_nms.py::test_gpu_inflight_matches_serial): the kernels are
    deterministic and no scratch is shared between streams (NMS scratch is per stream).

        run = Inflight(plan, B, H, W, streams=3)
        h = run.submit(x)                 # x [B,3,H,W] on the plan's device, produced on the current stream
        det, src_row, count = run.result(h)   # waits for that batch only; valid until S more submits

    post(det, src_row, count) (optional) runs on the batch's stream after its NMS, e.g.
    yv7.dist.gather_detections; whatever it returns is what result(h) hands back for that batch.
    """

    def __init__(self, plan, B, H, W, streams=3, conf_thres=0.25, iou_thres=0.45, max_det=300, post=None,
                 priorities=None, nms=None):
        """nms(z, conf, iou, max_det, out, rowbest): the batched NMS (default utils.general.nms_batched).
        A plan on a CPU device (test doubles: the multi-rank ordering tests on gloo) runs every
        submission synchronously on the host — same slots, buffers and post() order, no streams."""
        self.plan, self.S = plan, max(1, int(streams))
        self.conf, self.iou, self.max_det, self.post = conf_thres, iou_thres, max_det, post
        if nms is None:
            from utils.general import nms_batched

            def nms(z, conf, iou, max_det, out, rowbest):
                return nms_batched(z, conf, iou, max_det=max_det, out=out, rowbest=rowbest)
        self.nms = nms
        dev = plan.device
        self.host = dev.type == 'cpu'
        N = plan.num_rows(H, W)
        if N <= 0:
            L.check(-2, f'yv7_num_rows(H={H}, W={W})')
        self.shape = (B, 3, H, W)
        S = self.S
        prios = list(priorities) if priorities is not None else [0] * S   # HIP stream priorities (-1 = high)
        self.streams = [None if self.host else torch.cuda.Stream(dev, priority=prios[i % len(prios)]) for i in range(S)]
        self.z = [torch.empty((B, N, plan.no), dtype=torch.float32, device=dev) for _ in range(S)]
        self.rowbest = [torch.empty((B, N, 4), dtype=torch.float32, device=dev) for _ in range(S)]
        self.det = [torch.empty((B, max_det, 6), dtype=torch.float32, device=dev) for _ in range(S)]
        self.src = [torch.empty((B, max_det), dtype=torch.int64, device=dev) for _ in range(S)]
        self.cnt = [torch.empty((B,), dtype=torch.int32, device=dev) for _ in range(S)]
        self.done = [None if self.host else torch.cuda.Event() for _ in range(S)]
        self.out = [None] * S   # post()'s result per slot
        self.n = 0

    def submit(self, x):
        """Queue one batch; returns its handle (the submission index)."""
        import contextlib
        if tuple(x.shape) != self.shape:
            raise ValueError(f'Inflight built for {self.shape}, got {tuple(x.shape)}')
        k = self.n % self.S
        s = self.streams[k]
        if s is not None:
            s.wait_stream(torch.cuda.current_stream(self.plan.device))   # x is ready
        self.plan.forward_into(x, self.z[k], rowbest=self.rowbest[k], stream=s, ws_slot=k)
        with (torch.cuda.stream(s) if s is not None else contextlib.nullcontext()):
            self.nms(self.z[k], self.conf, self.iou, self.max_det, (self.det[k], self.src[k], self.cnt[k]),
                     self.rowbest[k])
            out = (self.det[k], self.src[k], self.cnt[k])
            if self.post is not None:
                out = self.post(*out)
        self.out[k] = out
        if self.done[k] is not None:
            self.done[k].record(s)
        self.n += 1
        return self.n - 1

    def result(self, h):
        """(det [B,max_det,6], src_row [B,max_det], count [B]) of submission h once it has finished, or
        what post() returned for it."""
        if not (self.n - self.S <= h < self.n):
            raise IndexError(f'batch {h} is no longer buffered (last {self.S} of {self.n} submissions)')
        k = h % self.S
        if self.done[k] is not None:
            self.done[k].synchronize()
        return self.out[k]

    def close(self):
        """Wait for every batch in flight (their buffers and workspaces are then free to go)."""
        for s in self.streams:
            if s is not None:
                s.synchronize()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass
