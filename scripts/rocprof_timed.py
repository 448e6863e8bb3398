"""Cross-check of bench.py's roofline against a rocprofv3 --kernel-trace of the same bench command.

The trace is split into forwards (each yolov7 fp16 forward starts with the fused stem kernel, in
submission order); the bench's timed forwards are forwards warmup .. warmup + steps - 1.  Reports the
mean conv-family launch duration (all CONV + DETECT launches: implicit-GEMM rings, persistent rings,
weight-stationary 3x3, halo, tile kernels) over the timed forwards and over the first `live_forwards`
of them (the ones bench.py's live HIP events covered), and the NMS kernels' durations per batch.
usage: python scripts/rocprof_timed.py <kernel_trace.csv> <bench.json> [out.json]"""
import csv
import re
import json
import statistics
import sys

CONV = ('conv_f16_pring_kernel', 'conv_f16_ring_kernel', 'conv3x3_ws64_kernel', 'conv3x3_halo_kernel',
        'conv_f16_kernel', 'conv_f16_pp_kernel', 'conv_f16_p8_kernel', 'conv_f16_p8n_kernel', 'conv_f8_kernel')
NMS = ('nms_compact', 'nms_fast', 'nms_rows', 'nms_scan', 'nms_write', 'nms_sort', 'nms_greedy')

rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r['Dispatch_Id']))
bench = json.load(open(sys.argv[2]))
warm, steps = bench['warmup'], bench['steps']
nlive = int(bench.get('detail', {}).get('profiled_forwards') or 0)
fwd = -1
per = {}
for r in rows:
    n = r['Kernel_Name']
    if 'stem_kernel' in n or 'stem2_kernel' in n:
        fwd += 1
    dur = (int(r['End_Timestamp']) - int(r['Start_Timestamp'])) / 1e3
    fam = 'conv' if any(c in n for c in CONV) else ('nms' if any(c in n for c in NMS) else None)
    if fam and fwd >= 0:
        per.setdefault(fwd, {}).setdefault(fam, []).append(dur)
timed = [f for f in range(warm, warm + steps) if f in per]
conv = [d for f in timed for d in per[f].get('conv', [])]
conv_live = [d for f in timed[:nlive] for d in per[f].get('conv', [])]
nms = [sum(per[f].get('nms', [])) for f in timed]
res = {'forwards_in_trace': fwd + 1, 'timed_forwards': len(timed),
       'conv_launches_per_forward': len(per[timed[0]]['conv']) if timed else 0,
       'conv_mean_us_timed': round(statistics.mean(conv), 2) if conv else None,
       'conv_mean_us_live_forwards': round(statistics.mean(conv_live), 2) if conv_live else None,
       'bench_events_mean_launch_us': bench['roofline']['mean_launch_us'],
       'nms_kernels_us_per_batch_timed': round(statistics.median(nms), 1) if nms else None,
       'nms_kernels': sorted({re.search(r'(nms_\w+|row_best\w*)', r['Kernel_Name']).group(1) for r in rows
                              if any(c in r['Kernel_Name'] for c in NMS)})}
print(json.dumps(res, indent=1))
if len(sys.argv) > 3:
    json.dump(res, open(sys.argv[3], 'w'), indent=1)
