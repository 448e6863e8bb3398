set -o pipefail
O=gpurun_out/r6a; mkdir -p $O
export PYTHONPATH=$PWD/yolo-series_amd:$PWD
timeout -k 10 300 python -u scripts/op_profile.py --top 100 --b 32 > $O/ops_b32.txt 2>&1 && grep -E "^forward" $O/ops_b32.txt &&
timeout -k 10 300 python -u scripts/op_profile.py --top 100 --b 64 > $O/ops_b64.txt 2>&1 && grep -E "^forward" $O/ops_b64.txt &&
timeout -k 10 300 python -u scripts/op_profile.py --top 100 --b 128 > $O/ops_b128.txt 2>&1 && grep -E "^forward" $O/ops_b128.txt &&
timeout -k 10 300 python -u bench.py --steps 40 --warmup 5 --no-cpu-baseline > $O/bench.json 2> $O/bench.err && python -c "import json;d=json.load(open('$O/bench.json'));print(d['value'], d['detail']['serial_forward_ms'])"
