"""Throughput bench of the MI355X YOLOv7 inference path (BASELINE.json configs[1] per GPU).

One step = one batch of 32 synthetic 640x640 frames per GPU, already resident in HBM:
  libyv7 forward (fp16 plan: NHWC implicit-GEMM MFMA convs, pools, fused Detect decode -> z fp32)
  + batched NMS on the GPU (conf 0.25, iou 0.45, max_det 300: detect.py's defaults)
  + (N > 1) RCCL all-gather of the fixed-shape detections.
Weights: seeded synthetic yolov7 weights (no checkpoints offline), packed once on rank 0 and
RCCL-broadcast.  N > 1 is launched by torch.distributed.run, one process per GPU; per-GPU work is
fixed (weak scaling); value = all images processed / max-over-ranks wall time of the K timed steps.

roofline: per kernel instantiation (the kernels the dispatch picks, yv7_op_kernels): launches, mean
serial launch time (HIP event pairs on each op's own dispatches, two forwards after the timed region,
every kernel alone on the chip — the durations a rocprofv3 kernel trace of a serial forward reports),
algorithmic bytes and FLOPs per launch (layer-boundary model) and roof = max(bytes / 8 TB/s,
FLOPs / 2.5 PF); `frac` is the dominant kernel's (most time per forward) achieved / peak on its
binding roof.  The whole job against the layer-boundary HBM ceiling is `job_frac`; the conv family's
bytes over the timed region as a whole `family_stream_frac`.
cpu_baseline: the oracle (CPU restatement of the reference detect.py path: torch CPU fp32 NCHW +
restated NMS), rank 0 only, on a bounded sample of the same workload.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path[:0] = [os.path.join(ROOT, 'yolo-series_amd'), ROOT]

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

HBM_PEAK_GBS = 8000.0          # MI355X HBM3E spec (MI355X_MICROARCH.md)
# HBM bytes per conv launch from PMC counters of this same workload (scripts/pmc_traffic.sh: separate
# FETCH_SIZE / WRITE_SIZE rocprofv3 passes; scripts/pmc_traffic.py: x2 FETCH correction for gfx950)
PMC_TRAFFIC = os.path.join(ROOT, 'profiles', 'r6_pmc_traffic.json')   # per kernel (scripts/pmc_traffic_kernels.py)
MFMA_F16_PEAK_TFLOPS = 2500.0  # dense fp16 MFMA


def parse(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument('--gpus', type=int, default=1, help='ranks (one process per GPU); without an outer '
                    'torch.distributed.run, bench.py starts one itself')
    ap.add_argument('--plumbing', action='store_true', help='CPU check of the multi-rank path only (gloo, no '
                    'GPU, no timing): launcher, weight-blob broadcast, detection all-gather, world size')
    ap.add_argument('--steps', type=int, default=60)
    ap.add_argument('--warmup', type=int, default=5)
    ap.add_argument('--batch', type=int, default=32, help='images per GPU')
    ap.add_argument('--img', type=int, default=640)
    ap.add_argument('--model', default='yolov7')
    ap.add_argument('--dtype', default='f16', choices=['f16', 'f32', 'fp8'],
                    help='fp8: BASELINE configs[4] (1x1 convs on e4m3 weights/activations, fp16 elsewhere)')
    ap.add_argument('--fp8-min-cout', type=int, default=None, help='fp8: narrowest 1x1 conv run in e4m3 '
                    '(default yv7.graph.FP8_MIN_COUT; 0 = every eligible 1x1)')
    ap.add_argument('--cpu-seconds', type=float, default=12.0, help='bounded CPU-baseline sample')
    ap.add_argument('--no-cpu-baseline', action='store_true')
    ap.add_argument('--no-live-events', action='store_true', help='diagnostic: time the steps without per-op HIP events')
    ap.add_argument('--live-forwards', type=int, default=3, help='timed forwards that record per-op HIP events '
                    '(the roofline\'s per-launch durations)')
    ap.add_argument('--split', type=int, default=1, help='run the batch as this many concurrent sub-batches, '
                    'each on its own HIP stream and workspace (fills the low-resolution layers\' tails and the '
                    'kernel-boundary gaps of one stream with the other\'s work)')
    ap.add_argument('--no-pipeline', action='store_true', help='run each batch\'s NMS (+ detection all-gather) '
                    'on the forward\'s stream instead of overlapping it with the next batch\'s forward')
    ap.add_argument('--streams', type=int, default=3, help='batches in flight (MI355X, bs32 yolov7, round-6 kernels, profiles/r6_streams/: 2 -> 7.93k, 3 -> 7.93k, 4 -> 7.70k img/s): batch k runs its forward + NMS on '
                    'HIP stream k %% S with its own workspace and buffers, so consecutive batches overlap')
    ap.add_argument('--prio', default='', help='comma-separated HIP stream priorities of the --streams streams '
                    '(measured: default 6.38k, -1,0,0 6.34k, -1,-1,0 6.23k img/s — equal priorities pack best)')
    ap.add_argument('--h2d', action='store_true', help='diagnostic, never `value` of the headline: upload each '
                    'batch as uint8 frames from pinned host memory (PCIe-inclusive rate)')
    ap.add_argument('--graph', action='store_true', help='replay the step as a HIP graph (measured: same speed '
                    'as eager launches on MI355X, the inter-kernel gaps are dependency drains, not launch cost)')
    ap.add_argument('--inputs', type=int, default=4, help='distinct resident input batches the steps rotate '
                    'through (4 x 78.6 MB fp16 at bs32 640: more than the 256 MiB Infinity Cache holds)')
    ap.add_argument('--map-frames', type=int, default=16, help='frames of the mAP@0.5 parity sample')
    return ap.parse_args(argv)


def _free_port():
    import socket
    s = socket.socket()
    s.bind(('127.0.0.1', 0))
    port = s.getsockname()[1]
    s.close()
    return port


def launch_ranks(a, argv):
    """--gpus N > 1 without an outer launcher: start N ranks with torch.distributed.run as a CHILD
    process (this process has not touched the GPU; it never execs) and return its exit code."""
    import subprocess
    cmd = [sys.executable, '-m', 'torch.distributed.run', '--nnodes=1', f'--nproc-per-node={a.gpus}',
           '--master-addr=127.0.0.1', f'--master-port={_free_port()}', os.path.abspath(__file__)] + list(argv)
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY=os.environ.get('HSA_ENABLE_IPC_MODE_LEGACY', '0'))
    return subprocess.call(cmd, env=env)


def plumbing(a):
    """The N > 1 data path on CPU ranks (gloo): the same yv7.dist calls the GPU ranks make, minus the
    kernels.  Prints one JSON line with the world size the process group saw."""
    from yv7 import dist as ydist
    sys.stdout.flush()
    json_fd = os.dup(1)   # stdout: the JSON line only (gloo announces its connections on fd 1)
    os.dup2(2, 1)
    ydist.init('gloo')
    world, rank = dist.get_world_size(), dist.get_rank()
    if world != a.gpus:
        raise SystemExit(f'--gpus {a.gpus} but the process group has {world} ranks')
    wd = ydist.Watchdog(rank)
    from models.yolo import Model
    from yv7 import _lib as L
    from yv7.graph import compile_model
    from yv7.synthetic import synthetic_state_dict
    import contextlib
    with contextlib.redirect_stdout(sys.stderr):
        model = Model(a.model)
        synthetic_state_dict(model, seed=0)
        model = model.float().fuse().eval()
    if a.dtype == 'fp8':
        # the fp8 plan's path: rank 0's activation scales, then its packed blob.  Calibration needs the GPU,
        # so rank 0 stands in seeded power-of-two scales here; the other ranks must end with its scales
        # and a blob identical to the one rank 0 packed from them.
        from yv7.graph import FP8_MIN_COUT, fp8_candidates
        mc = FP8_MIN_COUT if a.fp8_min_cout is None else a.fp8_min_cout
        ops = fp8_candidates(compile_model(model, L.DT_F16), mc)
        stand_in = {i: 2.0 ** -((i * 7) % 5) for i in ops} if rank == 0 else None
        _, g, blob = ydist.broadcast_fp8_plan(model, torch.device('cpu'), min_cout=mc, scales=stand_in)
        ref = compile_model(model, L.DT_F16, fp8={i: 2.0 ** -((i * 7) % 5) for i in ops})
        same = len(ops) > 0 and torch.equal(blob, ref.weight_blob())
    else:
        g = compile_model(model, L.DT_F16)
        blob = ydist.broadcast_blob(g, torch.device('cpu'))
        same = torch.equal(blob, g.weight_blob())
    gbatch = a.batch * world
    lo, hi = ydist.shard(gbatch, rank, world)
    b = hi - lo
    # every detection row carries its image's GLOBAL index (det column 0, src_row, count), so the gathered
    # tensors show whether each rank's shard landed at its place in the global batch
    gid = torch.arange(lo, hi)
    det = gid.float().view(b, 1, 1).expand(b, 300, 6).contiguous()
    src = gid.view(b, 1).expand(b, 300).contiguous()
    cnt = gid.to(torch.int32)
    gd, gs, gc = ydist.gather_detections(det, src, cnt)
    order = list(range(gbatch))
    in_order = (gc.tolist() == order and gd[:, :, 0].amin(1).tolist() == order and gd[:, :, 0].amax(1).tolist() == order
                and gs.amin(1).tolist() == order and gs.amax(1).tolist() == order)
    ok = same and in_order and gd.shape[0] == gbatch
    flags = torch.tensor([int(ok)])
    dist.all_reduce(flags, op=dist.ReduceOp.MIN)
    # the fields the GPU run reports per rank (here on gloo): the all-gather's time per batch and the
    # world size each rank's process group saw; plus each rank's shard of the global batch
    wd.beat('plumbing all-gathers')
    t0 = time.perf_counter()
    for i in range(10):
        wd.beat(batch=i)
        ydist.fault_point(rank, i)
        ydist.guarded(lambda: ydist.gather_detections(det, src, cnt), 'detection all-gather', i)
    us = (time.perf_counter() - t0) / 10 * 1e6
    per = torch.tensor([us, float(dist.get_world_size()), float(lo), float(hi), float(in_order)], dtype=torch.float64)
    pl = [torch.zeros_like(per) for _ in range(world)]
    dist.all_gather(pl, per)
    if rank == 0:
        os.write(json_fd, (json.dumps({'plumbing': True, 'dtype': a.dtype, 'n_gpus': world, 'world_size_seen': world, 'backend': 'gloo',
                          'rccl_world_size': world, 'model': a.model,
                          'weights_broadcast_bytes': int(blob.numel()), 'global_batch': gbatch,
                          'all_ranks_ok': bool(flags.item()),
                          'shards': [[int(v[2]), int(v[3])] for v in pl],
                          'gathered_in_global_order': [bool(v[4]) for v in pl],
                          'allgather_us_per_batch': [round(float(v[0]), 1) for v in pl],
                          'per_rank_world_size_seen': [int(v[1]) for v in pl]}) + '\n').encode())
    dist.barrier()
    wd.stop()
    dist.destroy_process_group()


def _cpu_model():
    try:
        for line in open('/proc/cpuinfo'):
            if line.startswith('model name'):
                return line.split(':', 1)[1].strip()
    except OSError:
        pass
    return 'unknown'


def _cpu_quota():
    """CPUs the job's cgroup allows (cpu.max), or None."""
    try:
        q, per = open('/sys/fs/cgroup/cpu.max').read().split()[:2]
        return None if q == 'max' else round(int(q) / int(per), 2)
    except (OSError, ValueError):
        return None


def map_parity(net, fused, img, plan, dev, frames=16, batch=32):
    """mAP@0.5 (and @.5:.95) of the GPU plan's detections on `frames` synthetic frames (seed 7) against
    the oracle's fp32 detections as ground truth (detect.py settings, conf 0.25 / iou 0.45), scored with
    the product's test.py-style mAP (utils/metrics.py).  The frames run in one batch of `batch` (repeated
    to fill it), so the plan takes the bench's own dispatch (bs 32) and the first `frames` are scored."""
    from oracle import nms_ref, yolo_ref
    from utils.general import nms_batched
    from utils.metrics import dets_as_labels, map_from_lists
    from yv7.synthetic import synthetic_frames
    xs = synthetic_frames(frames, img, img, seed=7)
    with torch.no_grad():
        zr = torch.cat([yolo_ref.forward(net, fused, xs[i:i + 1])[0] for i in range(frames)])
    labels = [dets_as_labels(d) for d in nms_ref.non_max_suppression(zr, 0.25, 0.45)]
    xb = xs.repeat((batch + frames - 1) // frames, 1, 1, 1)[:max(batch, frames)]
    N = plan.num_rows(img, img)
    zg = torch.empty((xb.shape[0], N, plan.no), dtype=torch.float32, device=dev)
    plan.forward_into(xb.to(dev).to(torch.float16 if plan.dtype == 1 else torch.float32), zg)
    det, _, cnt = nms_batched(zg[:frames].contiguous(), 0.25, 0.45)
    preds = [det[i, :int(cnt[i])].cpu() for i in range(frames)]
    m50, m5095 = map_from_lists(preds, labels)
    return {'map50': round(m50, 4), 'map50_95': round(m5095, 4), 'frames': frames, 'batch': int(xb.shape[0]),
            'truth': 'oracle fp32 CPU detections (conf 0.25, iou 0.45)',
            'pred': 'libyv7 plan (in a batch of %d: the bench dispatch) + GPU NMS, same frames and weights' % xb.shape[0]}


def cpu_baseline(model_name, img, seconds, plan=None, dev=None, parity_frames=16, big_batch=32):
    """The oracle (reference CPU path restated) on the host cores this job may use: forward + NMS,
    timed separately like detect.py:142-153 (t2 - t1 forward, t3 - t2 NMS), at batch 1 (detect.py's
    loop; `value`) for about `seconds`, and one batch of `big_batch` frames (test.py's batch size).

    Also the metric's parity half (map_parity): on `parity_frames` synthetic frames the oracle's fp32
    detections are the ground truth for the GPU plan's."""
    from oracle import nms_ref, yolo_ref
    from models.yolo import Model
    from yv7.synthetic import synthetic_frames, synthetic_state_dict
    threads = torch.get_num_threads()   # OMP_NUM_THREADS / the job's CPU share: every core it may use
    m = Model(model_name)
    sd = synthetic_state_dict(m, seed=0)
    net = yolo_ref.parse(m.yaml)
    fused = yolo_ref.fuse(net, sd)

    def run(x, min_s, min_n):
        t_fwd = t_nms = 0.0
        n = 0
        while True:
            t1 = time.perf_counter()
            z, _ = yolo_ref.forward(net, fused, x)
            t2 = time.perf_counter()
            nms_ref.non_max_suppression(z, 0.25, 0.45)
            t3 = time.perf_counter()
            t_fwd += t2 - t1
            t_nms += t3 - t2
            n += 1
            if t_fwd + t_nms >= min_s and n >= min_n:
                return n, t_fwd, t_nms

    with torch.no_grad():
        x1 = synthetic_frames(1, img, img, seed=1)
        yolo_ref.forward(net, fused, x1)  # warm-up
        n1, f1, s1 = run(x1, seconds, 2)
        xb = synthetic_frames(big_batch, img, img, seed=2)
        nb, fb, sb = run(xb, 0.0, 1)
    out = {'value': round(n1 / (f1 + s1), 3), 'unit': 'images/sec', 'cores': threads, 'kind': 'port',
           'sample': f'{n1} frames of {model_name} {img}x{img}, batch 1, fp32 NCHW, forward + NMS '
                     f'(conf 0.25, iou 0.45), {f1 + s1:.1f} s; then {nb} batch(es) of {big_batch}; '
                     f'torch {torch.__version__} CPU, {threads} threads',
           'cpu': _cpu_model(), 'machine_cpus': os.cpu_count(), 'cgroup_cpus': _cpu_quota(),
           'batch1': {'images_per_s': round(n1 / (f1 + s1), 3), 'forward_ms': round(f1 / n1 * 1e3, 1),
                      'nms_ms': round(s1 / n1 * 1e3, 2)},
           f'batch{big_batch}': {'images_per_s': round(nb * big_batch / (fb + sb), 3),
                                 'forward_ms': round(fb / nb * 1e3, 1), 'nms_ms': round(sb / nb * 1e3, 2)}}
    if plan is not None and parity_frames > 0:
        out['map_parity'] = map_parity(net, fused, img, plan, dev, parity_frames)
    return out


def main(argv=None):
    argv = sys.argv[1:] if argv is None else argv
    a = parse(argv)
    if 'WORLD_SIZE' not in os.environ and a.gpus > 1:
        sys.exit(launch_ranks(a, argv))
    if a.plumbing:
        return plumbing(a)
    world = int(os.environ.get('WORLD_SIZE', '1'))
    rank = int(os.environ.get('RANK', '0'))
    local = int(os.environ.get('LOCAL_RANK', '0'))
    if world != a.gpus:
        raise SystemExit(f'--gpus {a.gpus} but WORLD_SIZE={world}')
    # YV7_BENCH_DIST=1 takes the multi-rank path (RCCL broadcast + per-batch all-gather) even with one
    # rank, so the RCCL data path can be exercised on a one-GPU box
    force_dist = os.environ.get('YV7_BENCH_DIST') == '1'
    distributed = world > 1 or force_dist
    torch.cuda.set_device(local)
    from yv7 import dist as ydist
    wd = None
    json_fd = None
    if distributed:
        # stdout carries exactly ONE line, the JSON result: RCCL prints its version banner to fd 1 when its
        # first communicator comes up, so every other write to fd 1 goes to stderr from here on
        sys.stdout.flush()
        json_fd = os.dup(1)
        os.dup2(2, 1)
        # process-group timeout + a host-side progress watchdog: a dead or hung peer ends this rank with a
        # non-zero exit naming the rank, phase and batch, not a wait for the outer kill
        ydist.init('nccl', torch.device(f'cuda:{local}'))
        if dist.get_world_size() != a.gpus:
            raise SystemExit(f'--gpus {a.gpus} but RCCL sees {dist.get_world_size()} ranks')
        wd = ydist.Watchdog(rank)
    dev = torch.device(f'cuda:{local}')

    def beat(phase=None, batch=None):
        if wd is not None:
            wd.beat(phase, batch)

    from models.yolo import Model
    from utils.general import nms_batched
    from yv7.runtime import Plan
    from yv7.synthetic import synthetic_state_dict

    torch.manual_seed(0)
    dt = torch.float32 if a.dtype == 'f32' else torch.float16
    import contextlib
    with contextlib.redirect_stdout(sys.stderr):   # Model.fuse() prints like the reference; stdout is the JSON line
        model = Model(a.model)
        synthetic_state_dict(model, seed=0)
        model = model.float().fuse().eval()
    if a.dtype == 'fp8' and distributed:   # rank 0 calibrates, every rank gets its scales and packed blob
        plan = ydist.broadcast_fp8_plan(model, dev, min_cout=a.fp8_min_cout)[0]
    elif a.dtype == 'fp8':
        plan = Plan.fp8_from_model(model, dev, min_cout=a.fp8_min_cout)
    elif distributed:
        plan = ydist.broadcast_weights(model, dev, dt)
    else:
        plan = Plan.from_model(model, dev, dt)

    B, H, W = a.batch, a.img, a.img
    g = torch.Generator(device=dev).manual_seed(1000 + rank)
    # a.inputs distinct resident batches, step k reads batch k % a.inputs (together larger than the
    # Infinity Cache: the input read is a real HBM read, as for a stream of new frames)
    xin = [(torch.randint(0, 256, (B, 3, H, W), generator=g, device=dev, dtype=torch.uint8).to(dt) / 255.0)
           for _ in range(max(1, a.inputs))]
    x = xin[0]
    N = plan.num_rows(H, W)
    # Serving pipeline: batch k's NMS (and on multi-GPU its detection all-gather) runs on a second HIP
    # stream while batch k+1's forward runs on the first, so z / row records / detections are double
    # buffered and HIP events order each buffer's reuse.  --no-pipeline (and --graph) run the whole
    # step on one stream.
    nstreams = 1 if (a.split > 1 or a.graph) else max(1, a.streams)   # --split / --graph: one batch in flight
    pipeline = not (a.no_pipeline or a.graph) and nstreams == 1
    nbuf = 2 if pipeline else 1
    h2d = None
    if a.h2d:   # PCIe-inclusive rate: pinned uint8 host frames uploaded every step
        if nstreams < 2:
            raise SystemExit('--h2d runs on the batches-in-flight schedule (--streams >= 2)')
        host = torch.randint(0, 256, (B, 3, H, W), generator=torch.Generator().manual_seed(1000 + rank),
                             dtype=torch.uint8).pin_memory()
        h2d = {'host': host, 'u8': [torch.empty((B, 3, H, W), dtype=torch.uint8, device=dev) for _ in range(nstreams)],
               'x': [torch.empty((B, 3, H, W), dtype=dt, device=dev) for _ in range(nstreams)]}
    runner = None
    if nstreams > 1:   # yv7.runtime.Inflight: the library's serving schedule, S batches in flight
        from yv7.runtime import Inflight
        prios = [int(v) for v in a.prio.split(',')] if a.prio else None
        gather = (lambda d, s_, c: ydist.guarded(lambda: ydist.gather_detections(d, s_, c, force=force_dist),
                                                 'detection all-gather', nstep[0] - 1)) if distributed else None
        runner = Inflight(plan, B, H, W, streams=nstreams, post=gather,
                          priorities=prios)
    zs = [torch.empty((B, N, plan.no), dtype=torch.float32, device=dev) for _ in range(nbuf)]
    dets = [torch.empty((B, 300, 6), dtype=torch.float32, device=dev) for _ in range(nbuf)]
    srcs = [torch.empty((B, 300), dtype=torch.int64, device=dev) for _ in range(nbuf)]
    cnts = [torch.empty((B,), dtype=torch.int32, device=dev) for _ in range(nbuf)]
    rowbests = [torch.empty((B, N, 4), dtype=torch.float32, device=dev) for _ in range(nbuf)]  # yv7_row_best
    z, det, src, cnt, rowbest = zs[0], dets[0], srcs[0], cnts[0], rowbests[0]
    nms_stream = torch.cuda.Stream(dev) if pipeline else None
    fwd_done = [torch.cuda.Event() for _ in range(nbuf)]
    nms_done = [torch.cuda.Event() for _ in range(nbuf)]
    nstep = [0]

    nsplit = max(1, a.split)
    if B % nsplit:
        raise SystemExit(f'--split {nsplit} must divide the batch {B}')
    sub = B // nsplit
    streams = [torch.cuda.current_stream(dev)] + [torch.cuda.Stream(dev) for _ in range(nsplit - 1)]

    def forward(z, rowbest, x):
        if nsplit == 1:
            plan.forward_into(x, z, rowbest=rowbest)
            return
        main = streams[0]
        for s_ in streams[1:]:
            s_.wait_stream(main)
        for i, s_ in enumerate(streams):
            sl = slice(i * sub, (i + 1) * sub)
            plan.forward_into(x[sl], z[sl], rowbest=rowbest[sl], stream=s_, ws_slot=i)
        for s_ in streams[1:]:
            main.wait_stream(s_)

    def post(k):
        nms_batched(zs[k], 0.25, 0.45, out=(dets[k], srcs[k], cnts[k]), rowbest=rowbests[k])
        if distributed:
            ydist.guarded(lambda: ydist.gather_detections(dets[k], srcs[k], cnts[k], force=force_dist),
                          'detection all-gather', nstep[0] - 1)

    def step():
        k = nstep[0] % nbuf
        xk = xin[nstep[0] % len(xin)]
        if distributed:
            ydist.fault_point(rank, nstep[0])
            beat('batches', nstep[0])
        nstep[0] += 1
        if runner is not None:
            if h2d is None:
                runner.submit(xk)
                return
            # --h2d: this batch's uint8 frames come from pinned host memory (detect.py:100-104 hands the
            # model host frames): upload + /255 on the default stream, ordered after the forward that
            # last read this slot's device frames
            j = runner.n % nstreams          # the slot this submission will use
            cur = torch.cuda.current_stream(dev)
            if runner.n >= nstreams:
                cur.wait_event(runner.done[j])
            h2d['u8'][j].copy_(h2d['host'], non_blocking=True)
            torch.div(h2d['u8'][j], 255.0, out=h2d['x'][j])
            runner.submit(h2d['x'][j])
            return
        if not pipeline:
            forward(zs[k], rowbests[k], xk)
            post(k)
            return
        main = torch.cuda.current_stream(dev)
        if nstep[0] > nbuf:
            main.wait_event(nms_done[k])      # the NMS that read buffer k two batches ago has finished
        forward(zs[k], rowbests[k], xk)
        fwd_done[k].record(main)
        nms_stream.wait_event(fwd_done[k])
        with torch.cuda.stream(nms_stream):
            post(k)
        nms_done[k].record(nms_stream)

    beat('warmup')
    for _ in range(a.warmup):
        step()
    torch.cuda.synchronize()
    # --graph: the step (~100 kernels: forward, NMS, all-gather) replayed as one captured HIP graph.
    # The first n_live timed steps run eagerly with per-op HIP events (libyv7 profile mode, on the
    # forward's own stream): they give the per-launch averages for the roofline without event packets
    # between the kernels of every step.
    graph = None
    if a.graph:
        graph = torch.cuda.CUDAGraph()
        side = torch.cuda.Stream(dev)
        side.wait_stream(torch.cuda.current_stream(dev))
        with torch.cuda.stream(side):
            step()
        torch.cuda.current_stream(dev).wait_stream(side)
        with torch.cuda.graph(graph):
            step()
        graph.replay()
        torch.cuda.synchronize()
    # Live per-op HIP events inside the timed region: libyv7's profile mode launches every op of the
    # first n_live timed forwards with a (start, stop) event pair on the op's own kernel dispatches
    # (hipExtLaunchKernel), so a duration is the kernel's begin .. end as rocprofv3 reports it — with
    # batches in flight the three streams' kernels share the chip, so these are the durations of the
    # timed regime, contention included, but not the time a kernel waits in its queue for CUs the
    # other streams hold.  Not under --graph / --split.
    n_live = 0 if (a.no_live_events or nsplit > 1 or graph is not None) else min(a.steps, a.live_forwards)
    plan.profile_enable(n_live)
    if distributed:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(a.steps):
        if graph is None:
            step()
        else:
            graph.replay()
    torch.cuda.synchronize()
    if distributed:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    beat('after the timed region')
    rank_elapsed = [elapsed]
    if distributed:   # every rank's own time (per-rank img/s), then the job's: the slowest rank
        t = torch.tensor([elapsed], device=dev, dtype=torch.float64)
        tl = [torch.zeros_like(t) for _ in range(dist.get_world_size())]
        dist.all_gather(tl, t)
        rank_elapsed = [float(v.item()) for v in tl]
        elapsed = max(rank_elapsed)

    from yv7 import _lib as L
    from yv7.runtime import kernel_key
    costs = plan.op_costs(B, H, W, x_bytes=x.element_size(), with_raw=False)
    kernels = plan.op_kernels(B, H, W, x.dtype)

    def conv_family(nf, op_ms):
        """(mean conv/DETECT launch s, bytes per launch, flops per launch, launches, forward ms, conv ms)."""
        conv_ms = conv_bytes = conv_flops = 0.0
        nconv = 0
        for (kind, fl, by), ms in zip(costs, op_ms):
            if kind in (L.OP_CONV, L.OP_DETECT):
                conv_ms += ms / max(nf, 1)
                conv_bytes += by
                conv_flops += fl
                nconv += 1
        return (max(conv_ms / 1e3 / nconv, 1e-12), conv_bytes / nconv, conv_flops / nconv, nconv,
                sum(op_ms) / max(nf, 1), conv_ms)

    def kernel_table(nf, op_ms):
        """Per kernel instantiation (the op's main kernel: its last launch): launches per forward,
        mean launch us, algorithmic bytes / FLOPs per launch, roof us = max(bytes / 8 TB/s, FLOPs / 2.5
        PF), frac = roof / time, the binding roof."""
        fam = {}
        f = None
        for i, ((kind, fl, by), ms) in enumerate(zip(costs, op_ms)):
            if not kernels[i]:
                # an op without a kernel of its own (the second op of the dual 1x1 launch, the later pools
                # of the SPPCSPC cascade) ran inside the launch before it: its bytes and FLOPs (and its
                # zero-length event interval) belong to that kernel
                if f is not None:
                    f['ms'] += ms / max(nf, 1)
                    f['bytes'] += by
                    f['flops'] += fl
                    f['ops'].append(i)
                continue
            k = kernel_key(kernels[i][-1])
            f = fam.setdefault(k, {'kernel': k, 'launches': 0, 'ms': 0.0, 'bytes': 0.0, 'flops': 0.0, 'ops': []})
            f['launches'] += 1
            f['ms'] += ms / max(nf, 1)
            f['bytes'] += by
            f['flops'] += fl
            f['ops'].append(i)
        out = []
        for f in sorted(fam.values(), key=lambda f: -f['ms']):
            n = f['launches']
            us = f['ms'] * 1e3 / n
            hb, mf = f['bytes'] / n / (HBM_PEAK_GBS * 1e9) * 1e6, f['flops'] / n / (MFMA_F16_PEAK_TFLOPS * 1e12) * 1e6
            out.append({'kernel': f['kernel'], 'launches_per_forward': n, 'us_per_launch': round(us, 2),
                        'bytes_per_launch': round(f['bytes'] / n), 'flops_per_launch': round(f['flops'] / n),
                        'roof_us': round(max(hb, mf), 2), 'bound': 'hbm' if hb >= mf else 'mfma',
                        'frac': round(max(hb, mf) / us, 4) if us > 0 else None,
                        'share_of_forward': round(f['ms'] / max(sum(op_ms) / max(nf, 1), 1e-12), 4), 'ops': f['ops']})
        return out

    nf, op_ms = plan.profile_read()
    timed = conv_family(nf, op_ms)
    live_table = kernel_table(nf, op_ms) if nf else []
    # Diagnostics after the timed region (never `value`): two serial forwards with per-op events (each
    # kernel alone on the chip) — the roofline's per-kernel launch times — then detect.py's split
    # (detect.py:142-153): forward and NMS timed apart with HIP events on one stream, one batch at a time.
    plan.profile_enable(2)
    for _ in range(2):
        plan.forward_into(x, z, rowbest=rowbest)
    torch.cuda.synchronize()
    nf_s, op_ms_s = plan.profile_read()
    plan.profile_enable(0)
    serial = conv_family(nf_s, op_ms_s)
    table = kernel_table(nf_s, op_ms_s)
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(3)]
    f_ms = n_ms = 0.0
    for _ in range(3):
        ev[0].record()
        plan.forward_into(x, z, rowbest=rowbest)
        ev[1].record()
        nms_batched(z, 0.25, 0.45, out=(det, src, cnt), rowbest=rowbest)
        ev[2].record()
        ev[2].synchronize()
        f_ms += ev[0].elapsed_time(ev[1]) / 3
        n_ms += ev[1].elapsed_time(ev[2]) / 3
    # NMS workload: candidates per image (rows passing obj > conf and best obj*cls > conf, general.py:653,
    # 684), and the NMS at a lighter threshold, where nms_fast runs to the end of its candidate list
    # instead of stopping at max_det (general.py:705-706)
    nms_load = {}
    for conf in (0.25, 0.5):
        cand = ((rowbest[..., 0] > conf) & (rowbest[..., 1] > conf)).sum(1).float()
        nms_batched(z, conf, 0.45, out=(det, src, cnt), rowbest=rowbest)
        torch.cuda.synchronize()
        ms = 0.0
        for _ in range(5):
            ev[0].record()
            nms_batched(z, conf, 0.45, out=(det, src, cnt), rowbest=rowbest)
            ev[1].record()
            ev[1].synchronize()
            ms += ev[0].elapsed_time(ev[1]) / 5
        nms_load[f'conf_{conf}'] = {'candidates_per_image': round(float(cand.mean()), 1),
                                    'candidates_min_max': [int(cand.min()), int(cand.max())],
                                    'dets_per_image': round(float(cnt.float().mean()), 1),
                                    'nms_ms_per_batch': round(ms, 4)}
    # multi-GPU: the per-batch detection all-gather alone (the collective the bench issues every step)
    gather_us = None
    if distributed:
        dist.barrier()
        for _ in range(3):
            ydist.gather_detections(det, src, cnt, force=force_dist)
        torch.cuda.synchronize()
        ev[0].record()
        for _ in range(20):
            ydist.gather_detections(det, src, cnt, force=force_dist)
        ev[1].record()
        ev[1].synchronize()
        gather_us = round(ev[0].elapsed_time(ev[1]) / 20 * 1e3, 1)
        gt = torch.tensor([gather_us], device=dev, dtype=torch.float64)
        gl = [torch.zeros_like(gt) for _ in range(dist.get_world_size())]
        dist.all_gather(gl, gt)
        gather_us = [float(v.item()) for v in gl]
    mean_launch_s, bytes_per_launch, flops_per_launch, nconv, fwd_ms, conv_ms = timed if nf else serial
    # whole-job ceiling: SURVEY §8d's canonical layer-boundary bytes per image (reference module boundaries,
    # weights once per batch) at 8 TB/s; other configs: the plan's own op costs (which already credit the
    # sibling-GEMM merges, so they slightly overstate that ceiling)
    canon = {('yolov7', 640, 'f16'): 453.9e6, ('yolov7', 640, 'fp8'): 452.8e6, ('yolov7-w6', 1280, 'f16'): 1161.9e6}
    img_bytes = canon.get((a.model, H, a.dtype), sum(by for _, _, by in costs) / B)
    job_ceiling = HBM_PEAK_GBS * 1e9 / img_bytes   # images/s per GPU
    count_mean = float((runner.cnt[0] if runner is not None else cnt).float().mean().item())
    # the dominant kernel (most serial time per forward): achieved / peak on its binding roof
    dom = table[0]
    if dom['bound'] == 'hbm':
        ach, peak, unit = dom['bytes_per_launch'] / dom['us_per_launch'] / 1e3, HBM_PEAK_GBS, 'GB/s'
    else:
        ach, peak, unit = dom['flops_per_launch'] / dom['us_per_launch'] / 1e6, MFMA_F16_PEAK_TFLOPS, 'TFLOP/s'
    traffic = None
    traffic_src = None
    if os.path.exists(PMC_TRAFFIC):
        with open(PMC_TRAFFIC) as f:
            tj = json.load(f)
        cfg = tj.get('workload', {})
        if cfg.get('model', 'yolov7') == a.model and cfg.get('batch', 32) == B and cfg.get('img', 640) == H \
                and cfg.get('dtype', 'f16') == a.dtype and dom['kernel'] in tj.get('kernels', {}):
            traffic = round(tj['kernels'][dom['kernel']]['hbm_bytes_per_launch'])
            traffic_src = f'profiles/{os.path.basename(PMC_TRAFFIC)} ({tj.get("tree", "")})'
    dispatch_env = {k: v for k, v in sorted(os.environ.items()) if k.startswith('YV7_')}

    if rank == 0:
        value = world * B * a.steps / elapsed
        res = {
            'metric': 'images/sec (640×640) + mAP@0.5 parity vs ref; 1/2/4/8 MI355X',
            'value': round(value, 2),
            'unit': 'images/sec',
            'n_gpus': world,
            'steps': a.steps,
            'warmup': a.warmup,
            'ms_per_step': round(elapsed / a.steps * 1e3, 3),
            'higher_is_better': True,
            'scaling': 'weak',
            'vs_baseline': None,
            'dtype': a.dtype,
            'data': 'synthetic',
            'config': {'workload': f'{a.model} {"P6" if plan.nl == 4 else "P5"} {H}x{W} bs={B}/GPU {a.dtype}: libyv7 forward + GPU NMS '
                                   f'(conf 0.25, iou 0.45, max_det 300)'
                                   + (' + RCCL all-gather of detections' if distributed else ''),
                       'global_batch': world * B, 'img': H, 'parallelism': f'dp{world}',
                       'rccl_world_size': dist.get_world_size() if distributed else 1,
                       'weights': 'seeded synthetic, RCCL-broadcast' if distributed else 'seeded synthetic',
                       'resident_input_batches': len(xin), 'dispatch_env': dispatch_env},
            'roofline': {'bound': dom['bound'], 'achieved': round(ach, 1), 'peak': peak, 'unit': unit,
                         'frac': round(ach / peak, 4), 'traffic': traffic,
                         'traffic_unit': 'HBM bytes per launch of this kernel (PMC: 2 x FETCH_SIZE + WRITE_SIZE, '
                                         'separate passes of a serial forward)', 'traffic_source': traffic_src,
                         'kernel': dom['kernel'], 'launches_per_forward': dom['launches_per_forward'],
                         'mean_launch_us': dom['us_per_launch'],
                         'algorithmic_bytes_per_launch': dom['bytes_per_launch'],
                         'algorithmic_flops_per_launch': dom['flops_per_launch'],
                         'timing': 'HIP event pair on each op\'s own kernel dispatches (hipExtLaunchKernel: '
                                   'dispatch begin .. end, as a rocprofv3 kernel trace reports), 2 serial '
                                   'forwards after the timed region, kernels grouped by the instantiation the '
                                   'dispatch picks (yv7_op_kernels)',
                         'kernels_top5': [{k: v for k, v in r.items() if k != 'ops'} for r in table[:5]],
                         # the whole job against the layer-boundary HBM ceiling of the forward (SURVEY §8d:
                         # 17 625 img/s for yolov7 640 bs32 fp16)
                         'job_ceiling_images_per_s': round(job_ceiling, 1),
                         'job_frac': round(value / world / job_ceiling, 4),
                         # all CONV / DETECT launches over the timed region as a whole: their
                         # algorithmic bytes per step / ms_per_step
                         'family_stream_gbs': round(nconv * bytes_per_launch / (elapsed / a.steps) / 1e9, 1),
                         'family_stream_frac': round(nconv * bytes_per_launch / (elapsed / a.steps) / 1e9
                                                     / HBM_PEAK_GBS, 4)},
            'detail': {'serial_forward_ms': round(serial[4], 3),
                       'serial_conv_launch_us': round(serial[0] * 1e6, 2),
                       'serial_conv_tflops': round(serial[2] / serial[0] / 1e12, 1),
                       'serial_sum_of_roofs_ms': round(sum(r['roof_us'] * r['launches_per_forward'] for r in table) / 1e3, 3),
                       'live_contended': {'forwards': nf, 'forward_ms_events': round(fwd_ms, 3) if nf else None,
                                          'conv_launch_us': round(timed[0] * 1e6, 2) if nf else None,
                                          'overlap': round(conv_ms / 1e3 / (elapsed / a.steps), 2) if nf else None,
                                          'note': f'event pairs on every op of {nf} forwards inside the timed region '
                                                  f'({nstreams} stream(s) in flight: launches share the chip)'},
                       'detect_py_split_ms': {'forward': round(f_ms, 3), 'nms': round(n_ms, 3),
                                              'note': 'one batch at a time on one stream, HIP events '
                                                      '(detect.py:142-153 t2-t1 / t3-t2)'},
                       'mean_dets_per_image': round(count_mean, 1), 'rows_per_image': N, 'nms_load': nms_load,
                       'nms_overlapped_with_next_forward': pipeline or nstreams > 1, 'hip_graph': graph is not None,
                       'sub_batches': nsplit, 'streams': nstreams, 'h2d_uint8_frames': bool(a.h2d)},
        }
        # the parity bars behind `map50_parity` (tests/), stated with the line
        res['parity'] = {
            'fp32_plan_vs_oracle': 'every z element within 1e-4 * scale + |ref32 - ref64| (DEVIATION from '
                                   "north_star's literal 1e-4: the second term is the oracle's own fp32 summation-order "
                                   'error against its float64 forward; yolov7 640 bs32 max |gpu - ref32| 1.15e-4 '
                                   'where the GPU is 4.5e-5 and the oracle 1.07e-4 from float64; smaller cases within '
                                   '1e-4 outright)',
            'nms': 'kept rows, classes, boxes, scores bit-exact vs the oracle NMS on identical z; end to end kept '
                   'rows / classes equal after the float-noise margin filter',
            'fp16_plan': 'every op within 1 fp16 ulp of fp32 torch on its own input; bench-dispatch mAP@0.5 vs the '
                         'fp32 oracle >= 0.984 - 0.005 (tests/test_bench_config.py)',
            'pinning': 'parity unpinned by reference-produced vectors: the reference holds none and cannot be '
                       'imported here (SURVEY §8c); the oracle is a line-cited CPU restatement'}
        if distributed:
            res['detail']['per_rank_images_per_s'] = [round(B * a.steps / t_, 1) for t_ in rank_elapsed]
            res['detail']['allgather_us_per_batch'] = gather_us
        if not a.no_cpu_baseline and world == 1:
            res['cpu_baseline'] = cpu_baseline(a.model, a.img, a.cpu_seconds, plan=plan, dev=dev,
                                               parity_frames=a.map_frames)
            if 'map_parity' in res['cpu_baseline']:
                res['map50_parity'] = res['cpu_baseline']['map_parity']['map50']
        if json_fd is None:
            print(json.dumps(res), flush=True)
        else:
            os.write(json_fd, (json.dumps(res) + '\n').encode())
    if distributed:
        beat('final barrier')
        dist.barrier()
        wd.stop()
        dist.destroy_process_group()


def run_rank(argv=None):
    """main() for one rank.  In a multi-rank job an exception (e.g. a failed collective, re-raised by
    yv7.dist.guarded with rank and batch) ends the process at once with exit code 1 after its traceback:
    the interpreter's normal shutdown would tear down a process group whose peers may be gone."""
    try:
        main(argv)
    except SystemExit:
        raise
    except BaseException:
        if dist.is_initialized() and dist.get_world_size() > 1:
            import traceback
            traceback.print_exc()
            sys.stderr.flush()
            os._exit(1)
        raise


if __name__ == '__main__':
    run_rank()
