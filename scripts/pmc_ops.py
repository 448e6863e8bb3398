"""Per-op HBM traffic from rocprofv3 PMC passes of scripts/op_profile.py (FETCH_SIZE / WRITE_SIZE in
separate runs): the last forward's dispatches are matched, in order, to the ops' kernels that
`op_profile.py --dump` recorded (yv7_op_kernels), so every layer gets its own read / write bytes next
to its algorithmic bytes (layer-boundary model).  gfx950 corrections as scripts/pmc_traffic_kernels.py:
read = 2 x FETCH_SIZE, write = WRITE_SIZE (KiB in the CSV).
usage: python scripts/pmc_ops.py OPS.json FETCH_DIR WRITE_DIR [OUT.txt]
"""
import csv
import glob
import json
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), 'yolo-series_amd'))
from yv7.runtime import kernel_key  # noqa: E402


def dispatches(d, counter):
    rows = []
    for f in glob.glob(f'{d}/**/*counter_collection.csv', recursive=True):
        for r in csv.DictReader(open(f)):
            if r['Counter_Name'] == counter:
                rows.append((int(r['Dispatch_Id']), kernel_key(r['Kernel_Name']), float(r['Counter_Value']) * 1024.0))
    rows.sort()
    return rows


def per_op(ops, rows):
    seq = [(o['op'], kernel_key(k)) for o in ops for k in o['kernels']]
    names = {k for _, k in seq}
    mine = [r for r in rows if r[1] in names]
    last = mine[-len(seq):]
    if [k for _, k in seq] != [r[1] for r in last]:
        raise SystemExit('dispatch sequence does not match the op kernels')
    out = {}
    for (op, _), (_, _, v) in zip(seq, last):
        out[op] = out.get(op, 0.0) + v
    return out


def main(ops_json, fdir, wdir, dst=None):
    ops = json.load(open(ops_json))
    rd = per_op(ops, dispatches(fdir, 'FETCH_SIZE'))
    wr = per_op(ops, dispatches(wdir, 'WRITE_SIZE'))
    lines = [f'{"op":>3} {"layer":32s} {"kernel":44s} {"us":>7} {"alg MB":>8} {"read MB":>8} {"write MB":>8} {"ratio":>6}']
    tot_a = tot_h = 0.0
    for o in ops:
        if o['op'] not in rd:
            continue
        r, w = 2.0 * rd[o['op']], wr.get(o['op'], 0.0)
        a = o['bytes']
        tot_a += a
        tot_h += r + w
        k = kernel_key(o['kernels'][0])[:44] if o['kernels'] else '-'
        lines.append(f'{o["op"]:3d} {o["desc"]:32s} {k:44s} {o["us"]:7.1f} {a / 1e6:8.1f} {r / 1e6:8.1f} {w / 1e6:8.1f} {(r + w) / max(a, 1):6.2f}')
    lines.append(f'total: algorithmic {tot_a / 1e6:.1f} MB, PMC {tot_h / 1e6:.1f} MB ({tot_h / tot_a:.2f}x)')
    txt = '\n'.join(lines)
    print(txt)
    if dst:
        open(dst, 'w').write(txt + '\n')


if __name__ == '__main__':
    main(*sys.argv[1:5])
