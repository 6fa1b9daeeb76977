#!/usr/bin/env bash
# Same-box A/B of the pool's placement: load-aware plan (l3) against fixed strides (l3-fixed),
# alternated.  Usage (repo root, GPU box): bash tools/pool_place_ab.sh OUTDIR [N]
set -o pipefail
out=${1:-gpurun_out/r06_pool_place_ab}
n=${2:-4}
mkdir -p "$out"
export TMPDIR=/tmp
for i in $(seq 1 "$n"); do
  for p in l3 l3-fixed; do
    echo "[$(date +%T)] ${p}_$i"
    timeout -k 10 240 python tools/bench_pool.py --workers 8 --jobs-per-worker 400 --file-kb 1024 --placement $p \
        > "$out/${p}_$i.log" 2>&1 || { echo "${p}_$i failed"; exit 1; }
    tail -n 1 "$out/${p}_$i.log" | cut -c1-200
  done
done
