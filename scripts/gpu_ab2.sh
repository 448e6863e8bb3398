#!/bin/bash
mkdir -p gpurun_out
timeout -k 10 400 python -u scripts/ab_ops.py --ops 28,31,32,33,34,35,36,37,38,39,43,44,45,46,47,76,77,78,79,80,81,82 --variants 0,122,124,132,134,142,144,112,114,213,217,104,114 --out gpurun_out/ab_low.json > gpurun_out/ab_low.txt 2>&1
rc=$?; echo "ab rc=$rc"; tail -30 gpurun_out/ab_low.txt
