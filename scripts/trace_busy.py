"""Dev tool: how busy the GPU was under the bench's batches in flight — from a rocprofv3 kernel trace
(`--kernel-trace --output-format csv`): over the window from the first to the last dispatch of the
last `--frac` of the trace's kernels, the union of kernel intervals (time at least one kernel ran),
the average number of kernels running at once, and the idle gaps.
With --split-gap G (us): the trace is cut at idle gaps longer than G and the longest busy stretch is
reported (the bench's timed region: its batches in flight leave no long gap).
usage: python scripts/trace_busy.py TRACE_DIR [--frac 0.5] [--split-gap 500]"""
import argparse
import csv
import glob

ap = argparse.ArgumentParser()
ap.add_argument('trace')
ap.add_argument('--frac', type=float, default=0.5)
ap.add_argument('--split-gap', type=float, default=0.0)
a = ap.parse_args()
rows = []
for f in glob.glob(f'{a.trace}/**/*kernel_trace.csv', recursive=True):
    for r in csv.DictReader(open(f)):
        rows.append((int(r['Start_Timestamp']), int(r['End_Timestamp']), r['Kernel_Name']))
rows.sort()
rows = rows[int(len(rows) * (1 - a.frac)):]
if a.split_gap > 0:   # the longest stretch without an idle gap longer than split_gap
    segs, cur, end = [], [rows[0]], rows[0][1]
    for r in rows[1:]:
        if r[0] - end > a.split_gap * 1e3:
            segs.append(cur)
            cur = []
        cur.append(r)
        end = max(end, r[1])
    segs.append(cur)
    rows = max(segs, key=lambda sg: max(e for _, e, _ in sg) - sg[0][0])
t0, t1 = rows[0][0], max(e for _, e, _ in rows)
busy, cur_s, cur_e, gaps = 0, rows[0][0], rows[0][1], []
for s, e, _ in rows[1:]:
    if s > cur_e:
        busy += cur_e - cur_s
        gaps.append(s - cur_e)
        cur_s, cur_e = s, e
    else:
        cur_e = max(cur_e, e)
busy += cur_e - cur_s
span = t1 - t0
overlap = sum(e - s for s, e, _ in rows) / span
gaps.sort(reverse=True)
print(f'{len(rows)} kernels over {span / 1e6:.2f} ms: busy {busy / span:.3f} of the window, {overlap:.2f} kernels '
      f'running on average; {len(gaps)} idle gaps, {sum(gaps) / 1e3:.1f} us total, largest '
      + ', '.join(f'{g / 1e3:.1f}' for g in gaps[:5]) + ' us')
