set -o pipefail
mkdir -p gpurun_out
timeout -k 10 200 python scripts/op_profile.py --iters 10 --top 0 --csv gpurun_out/ops.csv > gpurun_out/op_profile.txt 2>&1 &&
timeout -k 10 300 python bench.py --dtype fp8 --no-cpu-baseline > gpurun_out/bench_fp8.json 2> gpurun_out/bench_fp8.err &&
timeout -k 10 300 python bench.py --model yolov7-w6 --img 1280 --batch 8 --no-cpu-baseline > gpurun_out/bench_w6.json 2> gpurun_out/bench_w6.err &&
cat gpurun_out/bench_fp8.json gpurun_out/bench_w6.json
