"""Multi-process path on CPU (gloo, world_size 2): batch sharding, weight-blob broadcast, detection
all-gather — the same yv7.dist code the 8-GPU bench runs over RCCL."""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from yv7.dist import gather_detections, shard


def _free_port():
    s = socket.socket()
    s.bind(('127.0.0.1', 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path[:0] = [os.path.join(root, 'yolo-series_amd'), root, os.path.join(root, 'tests')]
    os.environ.update(MASTER_ADDR='127.0.0.1', MASTER_PORT=str(port))
    dist.init_process_group('gloo', rank=rank, world_size=world)
    try:
        from models.yolo import Model
        from yv7 import _lib as L
        from yv7.dist import broadcast_blob, gather_detections, shard
        from yv7.graph import compile_model
        from yv7.synthetic import synthetic_state_dict
        # every rank compiles the graph; only rank 0 packs, the blob reaches the others by broadcast
        # (yv7.dist.broadcast_blob: the code broadcast_weights runs before creating each rank's plan)
        m = Model('yolov7-tiny')
        synthetic_state_dict(m, seed=rank)     # rank 1's own weights differ: only the broadcast makes them equal
        g = compile_model(m.float().fuse(), L.DT_F16)
        blob = broadcast_blob(g, torch.device('cpu'))
        m0 = Model('yolov7-tiny')
        synthetic_state_dict(m0, seed=0)
        same_blob = torch.equal(blob, compile_model(m0.float().fuse(), L.DT_F16).weight_blob())
        # per-rank fixed-shape NMS outputs for its slice of a global batch of 6 images
        lo, hi = shard(6, rank, world)
        b = hi - lo
        det = torch.arange(lo, hi, dtype=torch.float32).view(b, 1, 1).expand(b, 300, 6).contiguous()
        src = torch.arange(lo, hi, dtype=torch.int64).view(b, 1).expand(b, 300).contiguous()
        cnt = torch.arange(lo, hi, dtype=torch.int32)
        gd, gs, gc = gather_detections(det, src, cnt)
        q.put((rank, same_blob, gd[:, 0, 0].tolist(), gs[:, 0].tolist(), gc.tolist()))
    finally:
        dist.destroy_process_group()


class _HostPlan:
    """Test double of yv7.runtime.Plan on the host: z row 0 of image b carries the image's global id
    (the x value at [b, 0, 0, 0]), so the detections that come back identify the image they belong to."""
    device = torch.device('cpu')
    no = 6

    def num_rows(self, H, W):
        return 4

    def forward_into(self, x, z, rowbest=None, stream=None, ws_slot=0):
        z.zero_()
        z[:, :, 0] = x[:, 0, 0, 0].view(-1, 1)


def _host_nms(z, conf, iou, max_det, out, rowbest):
    det, src, cnt = out
    det.zero_()
    det[:, :, 0] = z[:, 0, 0].view(-1, 1)
    src.copy_(z[:, 0, 0].to(torch.int64).view(-1, 1).expand_as(src))
    cnt.copy_(z[:, 0, 0].to(torch.int32))


def _inflight_worker(rank, world, port, q):
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path[:0] = [os.path.join(root, 'yolo-series_amd'), root]
    os.environ.update(MASTER_ADDR='127.0.0.1', MASTER_PORT=str(port))
    dist.init_process_group('gloo', rank=rank, world_size=world)
    try:
        from yv7.dist import gather_detections
        from yv7.runtime import Inflight
        B, S, nb = 3, 3, 7
        run = Inflight(_HostPlan(), B, 2, 2, streams=S, max_det=5, post=gather_detections, nms=_host_nms)
        got = {}
        for h in range(nb):
            x = torch.zeros(B, 3, 2, 2)
            x[:, 0, 0, 0] = torch.arange(B) + h * B * world + rank * B     # global image ids of this rank's slice
            assert run.submit(x) == h
            if h >= S - 1:   # S batches in flight, collect the oldest
                d, s_, c = run.result(h - S + 1)
                got[h - S + 1] = c.tolist()
        for j in range(nb - S + 1, nb):
            got[j] = run.result(j)[2].tolist()
        q.put((rank, got))
    finally:
        dist.destroy_process_group()


def test_gloo_world2_inflight_gather_order():
    """yv7.runtime.Inflight (bench.py's serving schedule: S batches in flight, post= the per-batch
    detection all-gather) across two ranks: every rank's result for batch h is batch h's detections of
    the whole global batch, in global image order — submissions pair up across ranks in order, no slot
    hands back another batch's buffers."""
    ctx = mp.get_context('spawn')
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_inflight_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = [q.get(timeout=300) for _ in procs]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for rank, got in res:
        assert sorted(got) == list(range(7))
        for h, c in got.items():
            assert c == list(range(h * 6, h * 6 + 6)), (rank, h, c)


def _uneven_drain_worker(rank, world, port, q):
    """Rank 0 collects every batch right after submitting it (nothing in flight at the end); rank 1 keeps
    S batches in flight and drains the last ones newest-first.  The all-gather is issued inside
    submit(), in submission order, on both ranks, so the ranks' different collection orders cannot
    mis-pair or deadlock the collectives."""
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path[:0] = [os.path.join(root, 'yolo-series_amd'), root]
    os.environ.update(MASTER_ADDR='127.0.0.1', MASTER_PORT=str(port))
    dist.init_process_group('gloo', rank=rank, world_size=world)
    try:
        from yv7.dist import gather_detections
        from yv7.runtime import Inflight
        B, S, nb = 3, 3, 8
        run = Inflight(_HostPlan(), B, 2, 2, streams=S, max_det=5, post=gather_detections, nms=_host_nms)
        got = {}
        for h in range(nb):
            x = torch.zeros(B, 3, 2, 2)
            x[:, 0, 0, 0] = torch.arange(B) + h * B * world + rank * B
            assert run.submit(x) == h
            if rank == 0:
                got[h] = run.result(h)[2].tolist()
            elif h >= S - 1 and h % 2 == 0:
                got[h - S + 1] = run.result(h - S + 1)[2].tolist()
        for j in reversed(range(nb - S, nb)):   # rank 1: the batches still in flight, newest first
            if j not in got:
                got[j] = run.result(j)[2].tolist()
        run.close()
        q.put((rank, got))
    finally:
        dist.destroy_process_group()


def test_gloo_world2_inflight_uneven_drain():
    """two ranks with different numbers of batches in flight when they stop
    submitting (0 on rank 0, S on rank 1) and different collection orders: every batch either rank
    collected is that batch's detections of the whole global batch, in global image order."""
    ctx = mp.get_context('spawn')
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_uneven_drain_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = [q.get(timeout=300) for _ in procs]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for rank, got in res:
        assert got, rank
        for h, c in got.items():
            assert c == list(range(h * 6, h * 6 + 6)), (rank, h, c)
    assert sorted(dict(res)[0]) == list(range(8))


def _uneven_shard_worker(rank, world, port, q):
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path[:0] = [os.path.join(root, 'yolo-series_amd'), root]
    os.environ.update(MASTER_ADDR='127.0.0.1', MASTER_PORT=str(port))
    dist.init_process_group('gloo', rank=rank, world_size=world)
    try:
        sizes = [hi - lo for lo, hi in (shard(7, r, world) for r in range(world))]
        lo, hi = shard(7, rank, world)
        b = hi - lo
        det = torch.arange(lo, hi, dtype=torch.float32).view(b, 1, 1).expand(b, 300, 6).contiguous()
        src = torch.arange(lo, hi, dtype=torch.int64).view(b, 1).expand(b, 300).contiguous()
        cnt = torch.arange(lo, hi, dtype=torch.int32)
        gd, gs, gc = gather_detections(det, src, cnt, sizes=sizes)
        q.put((rank, gd[:, 0, 0].tolist(), gs[:, 0].tolist(), gc.tolist()))
    finally:
        dist.destroy_process_group()


def test_gloo_world2_uneven_shard_gather():
    """A global batch that the ranks cannot split evenly (7 over 2: 4 + 3): the gather pads to the
    largest shard and returns exactly the 7 images in order."""
    ctx = mp.get_context('spawn')
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_uneven_shard_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = [q.get(timeout=300) for _ in procs]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for rank, d, s_, c in res:
        assert d == list(range(7)) and s_ == list(range(7)) and c == list(range(7)), rank


def test_bench_plumbing_fp8():
    """`bench.py --gpus 2 --plumbing --dtype fp8`: rank 0's fp8 activation scales and packed blob reach
    rank 1 (yv7.dist.broadcast_fp8_plan), one JSON line."""
    import json
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = {k: v for k, v in os.environ.items() if k not in ('WORLD_SIZE', 'RANK', 'LOCAL_RANK', 'MASTER_PORT')}
    out = subprocess.run([sys.executable, os.path.join(root, 'bench.py'), '--gpus', '2', '--plumbing', '--dtype', 'fp8',
                          '--model', 'yolov7-tiny', '--batch', '2'], capture_output=True, text=True, env=env,
                         timeout=600)
    assert out.returncode == 0, out.stderr[-3000:]
    lines = [json.loads(l) for l in out.stdout.splitlines() if l.startswith('{')]
    assert len(lines) == 1, out.stdout
    assert lines[0]['dtype'] == 'fp8' and lines[0]['all_ranks_ok'] and lines[0]['per_rank_world_size_seen'] == [2, 2]


def test_shard_partition():
    for B, W in [(256, 8), (32, 1), (10, 4), (3, 4)]:
        parts = [shard(B, r, W) for r in range(W)]
        assert parts[0][0] == 0 and parts[-1][1] == B
        assert all(parts[i][1] == parts[i + 1][0] for i in range(W - 1))
        assert max(h - l for l, h in parts) - min(h - l for l, h in parts) <= 1


def test_gloo_world2_broadcast_and_gather():
    ctx = mp.get_context('spawn')
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = [q.get(timeout=300) for _ in procs]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for rank, same_blob, d, s, c in res:
        assert same_blob
        assert d == [0, 1, 2, 3, 4, 5] and s == [0, 1, 2, 3, 4, 5] and c == [0, 1, 2, 3, 4, 5]


def test_bench_launcher_starts_ranks():
    """`bench.py --gpus 2` with no outer launcher starts two ranks itself (torch.distributed.run as a
    child process) and the process group they form has world size 2 (--plumbing: the CPU/gloo form of
    the multi-rank path: weight-blob broadcast + detection all-gather, no GPU, no timing)."""
    import json
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = {k: v for k, v in os.environ.items() if k not in ('WORLD_SIZE', 'RANK', 'LOCAL_RANK', 'MASTER_PORT')}
    out = subprocess.run([sys.executable, os.path.join(root, 'bench.py'), '--gpus', '2', '--plumbing',
                          '--model', 'yolov7-tiny', '--batch', '3'], capture_output=True, text=True, env=env,
                         timeout=600)
    assert out.returncode == 0, out.stderr[-3000:]
    # stdout is exactly the one JSON line (the backend's own chatter goes to stderr: bench.py dup2)
    assert len(out.stdout.strip().splitlines()) == 1, out.stdout
    lines = [json.loads(l) for l in out.stdout.splitlines() if l.startswith('{')]
    assert len(lines) == 1, out.stdout
    r = lines[0]
    assert r['n_gpus'] == 2 and r['world_size_seen'] == 2 and r['all_ranks_ok'] and r['global_batch'] == 6
    assert r['per_rank_world_size_seen'] == [2, 2] and len(r['allgather_us_per_batch']) == 2


def _start_ranks(world, extra_env, args):
    """`world` bench.py ranks started directly (no torch.distributed.run, whose agent would tear the
    survivors down itself): each rank's own failure handling is what the test sees."""
    import subprocess
    import sys
    from bench import _free_port
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    port = str(_free_port())
    procs = []
    for r in range(world):
        env = {k: v for k, v in os.environ.items() if k not in ('YV7_DIST_FAULT',)}
        env.update(extra_env, WORLD_SIZE=str(world), RANK=str(r), LOCAL_RANK=str(r), MASTER_ADDR='127.0.0.1',
                   MASTER_PORT=port, OMP_NUM_THREADS='1')
        procs.append(subprocess.Popen([sys.executable, os.path.join(root, 'bench.py')] + args, env=env,
                                      stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True))
    return procs


@pytest.mark.parametrize('mode', ['exit', 'hang'])
def test_dead_peer_fails_loudly(mode):
    """rank 1 dies (exit) or stops issuing collectives (hang) at batch 3 of the
    detection all-gathers; rank 0 must exit non-zero within the process-group timeout, naming its rank
    and the batch, instead of waiting for an outer kill.  A hung rank is ended by its own watchdog."""
    import time
    timeout = 8
    procs = _start_ranks(2, {'YV7_DIST_FAULT': f'1:3:{mode}', 'YV7_DIST_TIMEOUT_S': str(timeout)},
                         ['--gpus', '2', '--plumbing', '--model', 'yolov7-tiny', '--batch', '2'])
    t0 = time.monotonic()
    outs = []
    try:
        for p in procs:
            outs.append(p.communicate(timeout=240))
    finally:
        for p in procs:
            if p.poll() is None:
                p.kill()
    took = time.monotonic() - t0
    rc0, rc1 = procs[0].returncode, procs[1].returncode
    err0 = outs[0][1]
    assert rc0 != 0 and rc1 != 0, (rc0, rc1, err0[-2000:])
    assert 'rank 0' in err0 and 'batch 3' in err0, err0[-2000:]
    if mode == 'exit':
        assert rc1 == 9
    else:
        assert 'rank 1 stalled' in outs[1][1], outs[1][1][-2000:]
    assert took < 200, took


def test_watchdog_fires_on_stall():
    """yv7.dist.Watchdog in a child process: beats keep it quiet, a stall ends the process with exit code
    3 and the phase / batch in its message."""
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    code = ('import sys, time; sys.path[:0] = [%r, %r]\n'
            'from yv7.dist import Watchdog\n'
            'w = Watchdog(5, timeout=1.0, poll=0.1)\n'
            'for i in range(10):\n    w.beat("loop", i); time.sleep(0.3)\n'
            'w.beat("stuck phase", 42); time.sleep(30)\n') % (os.path.join(root, 'yolo-series_amd'), root)
    out = subprocess.run([sys.executable, '-c', code], capture_output=True, text=True, timeout=120)
    assert out.returncode == 3, out.stderr[-2000:]
    assert 'rank 5 stalled' in out.stderr and 'stuck phase (batch 42)' in out.stderr


def test_bench_plumbing_8rank_global_batch_256():
    """BASELINE configs[2] on CPU: `bench.py --gpus 8 --plumbing` — 8 gloo ranks of
    yolov7, 32 images each (global batch 256): every rank receives rank 0's weight blob, the shards are the
    contiguous eighths of the global batch, and the all-gathered detections hold all 256 images in global
    order on every rank."""
    import json
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = {k: v for k, v in os.environ.items() if k not in ('WORLD_SIZE', 'RANK', 'LOCAL_RANK', 'MASTER_PORT')}
    env['OMP_NUM_THREADS'] = '1'
    out = subprocess.run([sys.executable, os.path.join(root, 'bench.py'), '--gpus', '8', '--plumbing',
                          '--model', 'yolov7', '--batch', '32'], capture_output=True, text=True, env=env,
                         timeout=900)
    assert out.returncode == 0, out.stderr[-3000:]
    lines = [json.loads(l) for l in out.stdout.splitlines() if l.startswith('{')]
    assert len(lines) == 1, out.stdout
    r = lines[0]
    assert r['n_gpus'] == 8 and r['rccl_world_size'] == 8 and r['world_size_seen'] == 8
    assert r['global_batch'] == 256 and r['model'] == 'yolov7'
    assert r['shards'] == [[32 * k, 32 * k + 32] for k in range(8)]
    assert r['gathered_in_global_order'] == [True] * 8 and r['all_ranks_ok']
    assert r['per_rank_world_size_seen'] == [8] * 8 and len(r['allgather_us_per_batch']) == 8


def test_gloo_world2_fp8_scales_missing_on_rank0():
    """A scale missing from rank 0's dict fails on EVERY rank after the broadcast (rank 0 used
    to raise alone and leave the others waiting in the collective)."""
    ctx = mp.get_context('spawn')
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_fp8_missing_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=300) for _ in procs)
    for p in procs:
        p.join(timeout=60)
    assert res == [(0, 'KeyError'), (1, 'KeyError')]


def _fp8_missing_worker(rank, world, port, q):
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path[:0] = [os.path.join(root, 'yolo-series_amd'), root]
    os.environ.update(MASTER_ADDR='127.0.0.1', MASTER_PORT=str(port))
    dist.init_process_group('gloo', rank=rank, world_size=world)
    try:
        from yv7.dist import broadcast_fp8_scales
        scales = {3: 0.5, 7: 0.25} if rank == 0 else None   # op 9 has no scale on rank 0
        try:
            broadcast_fp8_scales(scales, [3, 7, 9], torch.device('cpu'))
            q.put((rank, 'ok'))
        except KeyError:
            q.put((rank, 'KeyError'))
    finally:
        dist.destroy_process_group()


@pytest.mark.gpu
def test_rccl_world1_broadcast_gather_inflight():
    """The RCCL data path on one MI355X (world size 1, the collectives issued anyway): the weight blob
    broadcast, then three batches in flight on three streams each all-gathering its detections from
    its own stream (yv7.runtime.Inflight post=) — the results equal a serial run's (the per-batch
    all-gather the 8-GPU bench issues, on the real backend)."""
    from functools import partial

    from helpers import fresh_model, frames
    from utils.general import nms_batched
    from yv7.dist import broadcast_weights
    from yv7.runtime import Inflight
    os.environ.update(MASTER_ADDR='127.0.0.1', MASTER_PORT=str(_free_port()))
    dev = torch.device('cuda:0')
    torch.cuda.set_device(dev)
    dist.init_process_group('nccl', rank=0, world_size=1, device_id=dev)
    try:
        plan = broadcast_weights(fresh_model('yolov7-tiny'), dev, torch.float16)
        B, H, W = 4, 256, 320
        xs = [frames(B, H, W, seed=70 + i).to(dev).half() for i in range(4)]
        ref = []
        for x in xs:
            z = torch.empty((B, plan.num_rows(H, W), plan.no), dtype=torch.float32, device=dev)
            plan.forward_into(x, z)
            ref.append(nms_batched(z, 0.25, 0.45))
        run = Inflight(plan, B, H, W, streams=3, post=partial(gather_detections, force=True))
        hs = [run.submit(x) for x in xs]
        for h, (det, src, cnt) in zip(hs[1:], ref[1:]):
            gd, gs, gc = run.result(h)
            assert gd.shape == det.shape and torch.equal(gc, cnt)
            for b in range(B):
                n = int(cnt[b])
                assert torch.equal(gd[b, :n], det[b, :n]) and torch.equal(gs[b, :n], src[b, :n])
        run.close()
    finally:
        dist.destroy_process_group()


@pytest.mark.gpu
def test_rccl_world1_fp8_broadcast():
    """The fp8 plan's multi-GPU creation on the real backend (world size 1): rank 0 calibrates, the scales
    and the packed blob are RCCL-broadcast (yv7.dist.broadcast_fp8_plan) — the blob and the forward equal
    Plan.fp8_from_model's (what every rank computed for itself before round 4)."""
    from helpers import fresh_model, frames
    from yv7.dist import broadcast_fp8_plan
    from yv7.runtime import Plan
    os.environ.update(MASTER_ADDR='127.0.0.1', MASTER_PORT=str(_free_port()))
    dev = torch.device('cuda:0')
    torch.cuda.set_device(dev)
    dist.init_process_group('nccl', rank=0, world_size=1, device_id=dev)
    try:
        m = fresh_model('yolov7-tiny')
        plan, g, blob = broadcast_fp8_plan(m, dev)
        ref = Plan.fp8_from_model(m, dev)
        assert torch.equal(blob.cpu(), ref.graph.weight_blob())
        x = frames(2, 256, 256, seed=5).to(dev).half()
        za, _ = plan.forward(x, want_raw=False)
        zb, _ = ref.forward(x, want_raw=False)
        assert torch.equal(za, zb)
    finally:
        dist.destroy_process_group()

