"""Batch sharding over the GPUs of one node: one process per GPU, torch.distributed over RCCL.

Images are independent, so the data path needs no collective: rank r runs its own
contiguous slice of the global batch through its own plan.  The two collectives are the ones the
north star names:
  * broadcast_weights: rank 0 packs the fused network once; the packed blob (73.9 MB fp16 for
    yolov7) goes to every rank with one RCCL broadcast over xGMI, so every rank runs bit-identical
    weights without re-folding them.
  * broadcast_fp8_plan (BASELINE configs[4]): rank 0 calibrates the fp8 activation scales, every rank
    receives them (one small broadcast) before the weight blob, so every rank quantizes identically.
  * gather_detections: the fixed-shape per-rank NMS outputs (det [b,300,6] fp32, src_row [b,300]
    int64, count [b] int32) are all-gathered once per batch (~0.3 MB per rank for b = 32) so every
    rank holds the detections of the whole global batch in global image order.

Failure behaviour: a rank that dies or stops issuing collectives must not leave the
others waiting until an outer kill.  `init` gives the process group a timeout (YV7_DIST_TIMEOUT_S,
default 120 s) and `Watchdog` ends a rank that makes no host-side progress for that long with exit code
3 and a line naming the rank, the phase and the batch index; a collective that raises (a peer's
connection closed) is re-raised with the same attribution by `guarded`.
"""
from __future__ import annotations

import os
import sys
import threading
import time
from datetime import timedelta

import torch
import torch.distributed as dist

from yv7.graph import compile_model
from yv7.runtime import Plan
from yv7 import _lib as L

WATCHDOG_EXIT = 3


def timeout_s() -> float:
    """Seconds a rank may wait on a collective / make no progress (YV7_DIST_TIMEOUT_S, default 120)."""
    return float(os.environ.get('YV7_DIST_TIMEOUT_S', '120'))


def init(backend: str, device=None):
    """init_process_group with the timeout above (the reference's only collective, train.py:611, is
    training-only; this is the inference path's)."""
    kw = {'timeout': timedelta(seconds=timeout_s())}
    if device is not None:
        kw['device_id'] = device
    dist.init_process_group(backend, **kw)


class Watchdog:
    """Host-side progress watchdog for one rank.  `beat(phase, batch)` marks progress (batch = the one
    about to be issued); if none comes for `timeout` seconds (default 1.25 x timeout_s() + 5) the rank prints `yv7.dist: rank R stalled ... in PHASE (batch K)` to stderr and
    leaves with os._exit(WATCHDOG_EXIT) — the stuck collective (RCCL all-gather issued on a batch's
    stream, or a gloo call) can never return, so an orderly exit is not possible.  The host loop blocks
    on the batches in flight (Inflight reuses a slot only after its previous batch finished), so a
    stalled all-gather stops the beats within a few batches."""

    def __init__(self, rank: int, timeout: float | None = None, poll: float = 0.5):
        self.rank = rank
        # default: past the process group's own timeout, so a collective that raises gets to report first
        self.timeout = timeout_s() * 1.25 + 5 if timeout is None else timeout
        self.poll = poll
        self.phase, self.batch = 'start', None
        self.last = time.monotonic()
        self._stop = threading.Event()
        self._t = threading.Thread(target=self._run, name=f'yv7-watchdog-{rank}', daemon=True)
        self._t.start()

    def beat(self, phase: str | None = None, batch: int | None = None):
        if phase is not None:
            self.phase = phase
        self.batch = batch
        self.last = time.monotonic()

    def stop(self):
        self._stop.set()

    def _run(self):
        while not self._stop.wait(self.poll):
            idle = time.monotonic() - self.last
            if idle > self.timeout:
                where = self.phase + (f' (batch {self.batch})' if self.batch is not None else '')
                sys.stderr.write(f'yv7.dist: rank {self.rank} stalled for {idle:.0f} s in {where}: a peer rank '
                                 f'died or a collective hung; exiting with code {WATCHDOG_EXIT}\n')
                sys.stderr.flush()
                os._exit(WATCHDOG_EXIT)


def guarded(fn, what: str, batch=None):
    """Run collective-issuing `fn()`; an exception (a peer's connection closed, the process group's
    timeout) is re-raised naming this rank, `what` and the batch index."""
    try:
        return fn()
    except Exception as e:  # noqa: BLE001 — re-raised with the rank / batch attribution
        rk = dist.get_rank() if dist.is_initialized() else -1
        at = f' of batch {batch}' if batch is not None else ''
        raise RuntimeError(f'yv7.dist: rank {rk}: {what}{at} failed: {type(e).__name__}: {e}') from e


def fault_point(rank: int, batch: int):
    """Test hook for the failure path (tests/test_dist.py): YV7_DIST_FAULT=R:K:MODE makes rank R, at
    batch K, exit at once (MODE exit) or stop issuing collectives (MODE hang).  Unset: no effect."""
    spec = os.environ.get('YV7_DIST_FAULT')
    if not spec:
        return
    r, k, mode = spec.split(':')
    if int(r) == rank and int(k) == batch:
        if mode == 'exit':
            os._exit(9)
        while True:   # hang: the peers' watchdogs / timeouts must end the job
            time.sleep(3600)


def shard(global_batch: int, rank: int, world: int):
    """Contiguous slice [lo, hi) of the global batch owned by `rank` (images r*B/W ... (r+1)*B/W)."""
    base, rem = divmod(global_batch, world)
    lo = rank * base + min(rank, rem)
    return lo, lo + base + (1 if rank < rem else 0)


def broadcast_blob(graph, device, group=None):
    """Rank 0 packs `graph`'s weight blob, every rank receives it by one broadcast (RCCL over xGMI
    on GPU ranks, gloo on CPU ranks); the other ranks never pack."""
    if dist.get_rank(group) == 0:
        blob = graph.weight_blob().to(device)
    else:
        blob = torch.empty(max(graph.nbytes, 1), dtype=torch.uint8, device=device)
    dist.broadcast(blob, src=0, group=group)
    return blob


def broadcast_weights(model, device, dtype, group=None):
    """Compile on every rank (cheap, host-only), pack on rank 0, RCCL-broadcast the packed blob and
    create this rank's plan from it."""
    code = L.DT_F16 if dtype == torch.float16 else L.DT_F32
    g = compile_model(model, code)
    return Plan(g, device, broadcast_blob(g, device, group))


def broadcast_fp8_scales(scales, ops, device, group=None):
    """Rank 0's {op: activation scale} for the fp8 ops `ops` (the same list on every rank: it comes from
    the host-side graph) -> the same dict on every rank, by one broadcast.  A scale missing on rank 0
    travels as NaN, so every rank raises together after the collective (a KeyError on rank 0
    alone left the other ranks waiting in the broadcast)."""
    if dist.get_rank(group) == 0:
        t = torch.tensor([float(scales[i]) if scales is not None and i in scales else float('nan') for i in ops],
                         dtype=torch.float64, device=device)
    else:
        t = torch.zeros(len(ops), dtype=torch.float64, device=device)
    if len(ops):
        dist.broadcast(t, src=0, group=group)
    vals = t.tolist()
    missing = [i for i, v in zip(ops, vals) if v != v]
    if missing:
        raise KeyError(f'broadcast_fp8_scales: rank 0 has no activation scale for fp8 ops {missing}')
    return {i: float(v) for i, v in zip(ops, vals)}


def broadcast_fp8_plan(model, device, min_cout=None, calib=None, group=None, scales=None):
    """BASELINE configs[4] on N ranks: rank 0 calibrates (Plan.fp8_scales) — or takes `scales` — every
    rank receives the scales, compiles the fp8 graph with them, and gets rank 0's packed blob, as
    broadcast_weights does for the fp16 plan.  Returns (plan, graph, blob): the Plan (None on a CPU
    device: the --plumbing check), the compiled fp8 graph and rank 0's packed weight blob."""
    from yv7.graph import FP8_MIN_COUT, fp8_candidates
    min_cout = FP8_MIN_COUT if min_cout is None else min_cout
    ops = fp8_candidates(compile_model(model, L.DT_F16), min_cout)
    if dist.get_rank(group) == 0 and scales is None:
        scales = Plan.fp8_scales(model, device, calib, min_cout)
    scales = broadcast_fp8_scales(scales, ops, device, group)
    g = compile_model(model, L.DT_F16, fp8=scales)
    blob = broadcast_blob(g, device, group)
    return (None if torch.device(device).type == 'cpu' else Plan(g, device, blob)), g, blob


def gather_detections(det, src_row, count, group=None, force=False, sizes=None):
    """All-gather fixed-shape per-rank NMS outputs -> global (det, src_row, count) in image order.
    One rank: the inputs themselves, unless force (the collective is then issued anyway — a one-GPU
    check of the RCCL path).  sizes: every rank's image count (shard()), when they differ: each rank's
    rows are padded to the largest and the padding is dropped after the gather."""
    world = dist.get_world_size(group)
    if world == 1 and not force:
        return det, src_row, count
    b = det.shape[0]
    mx = max(sizes) if sizes else b
    outs = []
    for t in (det, src_row, count):
        if mx != b:
            t = torch.cat([t, torch.zeros((mx - b,) + tuple(t.shape[1:]), dtype=t.dtype, device=t.device)])
        o = torch.empty((world * mx,) + tuple(t.shape[1:]), dtype=t.dtype, device=t.device)
        dist.all_gather_into_tensor(o, t.contiguous(), group=group)
        if sizes and any(n != mx for n in sizes):
            o = torch.cat([o[r * mx:r * mx + n] for r, n in enumerate(sizes)])
        outs.append(o)
    return tuple(outs)
