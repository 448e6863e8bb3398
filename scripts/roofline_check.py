"""Recompute the bench line's per-kernel roofline from a rocprofv3 kernel trace of serial forwards.

usage: python scripts/roofline_check.py TRACE_DIR BENCH.json [OPS.json]
TRACE_DIR holds rocprofv3 --kernel-trace --stats output of scripts/op_profile.py (serial forwards of
the bench plan); BENCH.json is bench.py's line.  For each of roofline.kernels_top5: the bench's serial
per-launch time (HIP event pairs) vs rocprof's mean duration of the same kernel, and the fraction
recomputed as roof_us / rocprof mean (roof_us = max(algorithmic bytes / 8 TB/s, FLOPs / 2.5 PF), the
bench's own per-launch algorithmic figures).
With OPS.json (`op_profile.py --dump` of the same run: every op's kernels) the check also follows the
bench's own filing: an op that launches more than one kernel (the 8-phase ring's split-off tail, the
fp8 quantize pass) counts under its LAST kernel with its whole span, first dispatch start to last
dispatch end; the trace's forwards are found as complete runs of the dispatch sequence the ops give."""
import csv
import glob
import json
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), 'yolo-series_amd'))
from yv7.runtime import kernel_key  # noqa: E402


def op_spans(rows, ops):
    """Per family (an op's last kernel): the spans of its ops over every complete forward in rows."""
    seq = [(o['op'], kernel_key(k)) for o in ops for k in o['kernels']]
    keys = [k for _, k in seq]
    names = set(keys)
    mine = [r for r in rows if r[2] in names]
    fam = {}
    i = 0
    while i + len(seq) <= len(mine):
        if [r[2] for r in mine[i:i + len(seq)]] != keys:
            i += 1
            continue
        span = {}
        for (op, _), (t0, t1, _) in zip(seq, mine[i:i + len(seq)]):
            a, b = span.get(op, (t0, t1))
            span[op] = (min(a, t0), max(b, t1))
        for o in ops:
            if o['kernels'] and o['op'] in span:
                a, b = span[o['op']]
                fam.setdefault(kernel_key(o['kernels'][-1]), []).append((b - a) / 1e3)
        i += len(seq)
    return fam


def main(tdir, bench, ops_json=None):
    line = json.loads([l for l in open(bench) if l.startswith('{')][-1])
    durs = {}
    rows = []
    for f in glob.glob(f'{tdir}/**/*kernel_trace.csv', recursive=True):
        for r in csv.DictReader(open(f)):
            k = kernel_key(r['Kernel_Name'])
            t0, t1 = int(r['Start_Timestamp']), int(r['End_Timestamp'])
            durs.setdefault(k, []).append((t1 - t0) / 1e3)
            rows.append((t0, t1, k))
    rows.sort()
    spans = op_spans(rows, json.load(open(ops_json))) if ops_json else {}
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
        sp = spans.get(r['kernel'])
        if sp:
            m = sum(sp) / len(sp)
            print(f'{"   per op (bench filing: whole op span under its last kernel)":70s} '
                  f'rocprof {m:8.2f} us (n={len(sp)})  frac rocprof {r["roof_us"] / m:.4f}')


if __name__ == '__main__':
    main(*sys.argv[1:4])
