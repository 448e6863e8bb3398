"""Dev tool: how busy the GPU was under the bench's batches in flight — from a rocprofv3 kernel trace
(`--kernel-trace --output-format csv`): over the window from the first to the last dispatch of the
last `--frac` of the trace's kernels, the union of kernel intervals (time at least one kernel ran),
the average number of kernels running at once, and the idle gaps.
usage: python scripts/trace_busy.py TRACE_DIR [--frac 0.5]"""
import argparse
import csv
import glob

ap = argparse.ArgumentParser()
ap.add_argument('trace')
ap.add_argument('--frac', type=float, default=0.5)
a = ap.parse_args()
rows = []
for f in glob.glob(f'{a.trace}/**/*kernel_trace.csv', recursive=True):
    for r in csv.DictReader(open(f)):
        rows.append((int(r['Start_Timestamp']), int(r['End_Timestamp']), r['Kernel_Name']))
rows.sort()
rows = rows[int(len(rows) * (1 - a.frac)):]
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
