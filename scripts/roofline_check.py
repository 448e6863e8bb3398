"""Recompute the bench line's per-kernel roofline from a rocprofv3 kernel trace of serial forwards.

usage: python scripts/roofline_check.py TRACE_DIR BENCH.json
TRACE_DIR holds rocprofv3 --kernel-trace --stats output of scripts/op_profile.py (serial forwards of
the bench plan); BENCH.json is bench.py's line.  For each of roofline.kernels_top5: the bench's serial
per-launch time (HIP event pairs) vs rocprof's mean duration of the same kernel, and the fraction
recomputed as roof_us / rocprof mean (roof_us = max(algorithmic bytes / 8 TB/s, FLOPs / 2.5 PF), the
bench's own per-launch algorithmic figures)."""
import csv
import glob
import json
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), 'yolo-series_amd'))
from yv7.runtime import kernel_key  # noqa: E402


def main(tdir, bench):
    line = json.loads([l for l in open(bench) if l.startswith('{')][-1])
    durs = {}
    for f in glob.glob(f'{tdir}/**/*kernel_trace.csv', recursive=True):
        for r in csv.DictReader(open(f)):
            k = kernel_key(r['Kernel_Name'])
            durs.setdefault(k, []).append((int(r['End_Timestamp']) - int(r['Start_Timestamp'])) / 1e3)
    rf = line['roofline']
    print(f'bench line: kernel {rf["kernel"]} frac {rf["frac"]} ({rf["achieved"]} {rf["unit"]} of {rf["peak"]})')
    for r in rf['kernels_top5']:
        d = durs.get(r['kernel'])
        if not d:
            print(f'{r["kernel"][:70]:70s} not in the trace')
            continue
        mean = sum(d) / len(d)
        print(f'{r["kernel"][:70]:70s} bench {r["us_per_launch"]:8.2f} us  rocprof {mean:8.2f} us (n={len(d)})  '
              f'frac bench {r["frac"]:.4f} rocprof {r["roof_us"] / mean:.4f}  ({r["bound"]})')


if __name__ == '__main__':
    main(sys.argv[1], sys.argv[2])
