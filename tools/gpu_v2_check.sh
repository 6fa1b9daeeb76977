#!/usr/bin/env bash
# GPU tests + v1/v2 verify throughput (files in page cache) on one MI355X box.
set -o pipefail
out=${1:-gpurun_out/v2}
mkdir -p "$out"
timeout -k 10 600 python -m pytest tests -m gpu -x -q > "$out/pytest_gpu.log" 2>&1 &&
timeout -k 10 600 python tools/bench_hash.py --total-mb 4096 --piece-kb 16 1024 --reps 2 --kinds sha256 > "$out/bench_hash_v2.log" 2>&1
echo "rc=$?"
