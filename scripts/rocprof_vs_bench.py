"""Cross-check: mean duration of the conv-family launches in a rocprofv3 --kernel-trace --stats summary
vs bench.py's roofline.mean_launch_us (live HIP events on the forward's stream).
usage: python scripts/rocprof_vs_bench.py profiles/r1_kernel_stats.csv profiles/r1_bench_v10.json"""
import csv
import json
import sys

FAMILY = ('conv_f16_pring_kernel', 'conv_f16_ring_kernel', 'conv3x3_ws64_kernel', 'conv3x3_halo_kernel',
          'conv_f16_kernel')
rows = list(csv.DictReader(open(sys.argv[1])))
sel = [r for r in rows if any(f in r['Name'] for f in FAMILY)]
tot = sum(float(r['TotalDurationNs']) for r in sel)
calls = sum(int(r['Calls']) for r in sel)
b = json.load(open(sys.argv[2]))['roofline']
print(f'rocprof conv family: {calls} launches, mean {tot / calls / 1e3:.2f} us; '
      f'bench events: mean {b["mean_launch_us"]:.2f} us over {b["launches_per_forward"]} launches per forward')
