#!/bin/bash
# MP twin (conv_f16_twin_kernel): parity tests that reach it (bench config bs 32 op by op, fp16
# layerwise / model paths / variants), per-op profile, then bench A/B YV7_TWIN 0 / 1 / 2.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
export PYTHONPATH=$R/yolo-series_amd:$R
timeout -k 10 600 python -u -m pytest tests/test_bench_config.py tests/test_gpu_forward.py tests/test_gpu_model_paths.py tests/test_variants.py -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/twin_tests.log 2>&1 || { tail -40 gpurun_out/twin_tests.log; exit 1; }
tail -2 gpurun_out/twin_tests.log
for f in 0 1 2; do
  YV7_TWIN=$f timeout -k 10 200 python -u scripts/op_profile.py > gpurun_out/twin_ops_$f.txt 2>&1 || { tail gpurun_out/twin_ops_$f.txt; exit 1; }
  grep -E "^ +(9|10|18|19|73|74|88|89) " gpurun_out/twin_ops_$f.txt | head -12; grep "^forward" gpurun_out/twin_ops_$f.txt
done
for i in 1 2; do for f in 0 1 2; do
  YV7_TWIN=$f timeout -k 10 200 python -u bench.py --no-cpu-baseline > gpurun_out/twin_b${f}_$i.json 2> gpurun_out/twin_b${f}_$i.err || { tail gpurun_out/twin_b${f}_$i.err; exit 1; }
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[1], d['value'], d['detail']['serial_forward_ms'])" gpurun_out/twin_b${f}_$i.json
done; done
