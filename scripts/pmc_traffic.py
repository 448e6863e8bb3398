"""Summarise scripts/pmc_traffic.sh's rocprofv3 PMC passes into per-kernel HBM bytes per launch.

gfx950 corrections (MI355X_MICROARCH.md, HBM section): FETCH_SIZE counts 64 B per 128-B request of a
wide streaming read, so read bytes = 2 x FETCH_SIZE; WRITE_SIZE is exact for 16-B-per-lane stores.
rocprofv3 reports both in KiB.  Output: profiles/<name>.json with, per kernel family, the launches
and the corrected mean bytes per launch, plus the conv family (CONV / DETECT launches) that bench.py
reports as roofline.traffic.
usage: python scripts/pmc_traffic.py gpurun_out profiles/r2_pmc_traffic.json
"""
import collections
import csv
import glob
import json
import re
import sys


def load(d, counter):
    out = collections.defaultdict(list)
    for f in glob.glob(f'{d}/pmc_{counter}/**/*counter_collection.csv', recursive=True):
        for r in csv.DictReader(open(f)):
            if r['Counter_Name'] == counter:
                out[r['Kernel_Name']].append(float(r['Counter_Value']) * 1024.0)
    return out


def family(name):
    for k in ('conv3x3_halo_kernel', 'conv3x3_ws64_kernel', 'conv_f16_pring_kernel', 'conv_f16_ring_kernel',
              'conv_f16_p8n_kernel', 'conv_f16_p8_kernel', 'conv_f16_pp_kernel', 'conv_f8_kernel',
              'conv_f16_kernel', 'conv_kernel', 'stem_kernel', 'spp_cascade_kernel', 'maxpool_kernel',
              'upsample_kernel', 'copy_kernel', 'input_reorg16_kernel', 'input_kernel', 'letterbox_kernel', 'nms_'):
        if k in name:
            return k.rstrip('_')
    return re.sub(r'\(.*', '', name)[:40]


def main(src, dst):
    fetch, write = load(src, 'FETCH_SIZE'), load(src, 'WRITE_SIZE')
    fam = collections.defaultdict(lambda: [0, 0.0, 0.0])
    for k, v in fetch.items():
        f = family(k)
        fam[f][0] += len(v)
        fam[f][1] += 2.0 * sum(v)
        fam[f][2] += sum(write.get(k, []))
    res = {'units': 'bytes per launch (read = 2 x FETCH_SIZE, write = WRITE_SIZE)', 'families': {}}
    conv_n = conv_b = 0
    for f, (n, rb, wb) in sorted(fam.items(), key=lambda kv: -kv[1][1]):
        res['families'][f] = {'launches': n, 'read_bytes_per_launch': rb / n, 'write_bytes_per_launch': wb / n,
                              'hbm_bytes_per_launch': (rb + wb) / n}
        if f in ('conv3x3_halo_kernel', 'conv3x3_ws64_kernel', 'conv_f16_pring_kernel', 'conv_f16_ring_kernel',
                 'conv_f16_p8n_kernel', 'conv_f16_p8_kernel', 'conv_f16_pp_kernel', 'conv_f8_kernel',
                 'conv_f16_kernel', 'conv_kernel'):
            conv_n += n
            conv_b += rb + wb
    res['conv_family'] = {'launches': conv_n, 'hbm_bytes_per_launch': conv_b / max(conv_n, 1)}
    json.dump(res, open(dst, 'w'), indent=1)
    print(json.dumps(res['conv_family']))


if __name__ == '__main__':
    main(sys.argv[1], sys.argv[2])
