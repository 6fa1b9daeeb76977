#!/usr/bin/env bash
# A/B of the adaptive default's prefetch at 2 and 20 ms RTT, alternated: this tree
# (2 * limit + 1 deliveries over the shards: 5 per shard at limit 4) against OLD_TREE, a
# checkout of the previous formula (limit + 1: 3 per shard), with the same built .so files.
# Usage (repo root, GPU box): bash tools/prefetch_ab.sh OUTDIR OLD_TREE
set -o pipefail
out=$(realpath -m "${1:-gpurun_out/r06_prefetch_ab}")
old=${2:-.ab/old}
mkdir -p "$out"
export TMPDIR=/tmp
run() {
  local name=$1 dir=$2; shift 2
  echo "[$(date +%T)] $name"
  (cd "$dir" && timeout -k 10 300 python bench.py --no-gpu-probe --no-reference-mode "$@" > "$out/$name.log" 2>&1)
  local rc=$?; echo "[$(date +%T)] $name rc=$rc"; return $rc
}
for i in 1 2 3; do
  run rtt20_old_$i "$old" --steps 200 --warmup 30 --rtt-ms 20 || exit 1
  run rtt20_new_$i . --steps 200 --warmup 30 --rtt-ms 20 || exit 1
  run rtt2_old_$i "$old" --steps 400 --warmup 40 --rtt-ms 2 || exit 1
  run rtt2_new_$i . --steps 400 --warmup 40 --rtt-ms 2 || exit 1
done
python tools/bench_summary.py "$out"/*.log > "$out/SUMMARY.txt" 2>&1 || true
cat "$out/SUMMARY.txt"
