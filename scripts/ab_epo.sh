#!/bin/bash
# A/B of the epilogue-overlap persistent ring (YV7_EPO): bit-identical z, GPU tests, per-op times, bench.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 120 python scripts/dump_z.py gpurun_out/z0.pt > gpurun_out/epo.log 2>&1 &&
YV7_EPO=1 timeout -k 10 120 python scripts/dump_z.py gpurun_out/z1.pt >> gpurun_out/epo.log 2>&1 &&
python -c "import torch; a=torch.load('gpurun_out/z0.pt'); b=torch.load('gpurun_out/z1.pt'); print('bit-identical', torch.equal(a,b), float((a-b).abs().max()))" >> gpurun_out/epo.log 2>&1 && rm -f gpurun_out/z0.pt gpurun_out/z1.pt &&
YV7_EPO=1 timeout -k 10 300 python -u -m pytest tests/test_gpu_forward.py -x -q -m gpu -p no:cacheprovider --timeout 120 --timeout-method thread >> gpurun_out/epo.log 2>&1 &&
timeout -k 10 200 python scripts/op_profile.py --iters 10 --top 0 --csv gpurun_out/ops_epo0.csv > gpurun_out/op_epo0.txt 2>&1 &&
YV7_EPO=1 timeout -k 10 200 python scripts/op_profile.py --iters 10 --top 0 --csv gpurun_out/ops_epo1.csv > gpurun_out/op_epo1.txt 2>&1 &&
timeout -k 10 200 python bench.py --no-cpu-baseline > gpurun_out/b_epo0.json 2>/dev/null &&
YV7_EPO=1 timeout -k 10 200 python bench.py --no-cpu-baseline > gpurun_out/b_epo1.json 2>/dev/null &&
for f in b_epo0 b_epo1; do python -c "import json;d=json.load(open('gpurun_out/$f.json'));print('$f',d['value'],d['ms_per_step'])"; done
