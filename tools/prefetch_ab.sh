#!/usr/bin/env bash
# A/B: the adaptive default's prefetch (ceil((limit + 1) / shards) per shard: 3 at limit 4)
# against floors of 4 and 5 per shard (--prefetch 4/5) at 2 and 20 ms RTT, alternated.
# Usage (repo root, GPU box): bash tools/prefetch_ab.sh OUTDIR
set -o pipefail
out=${1:-gpurun_out/r06_prefetch_ab}
mkdir -p "$out"
export TMPDIR=/tmp
step() { local name=$1 lim=$2; shift 2; echo "[$(date +%T)] $name"; timeout -k 10 "$lim" "$@" > "$out/$name.log" 2>&1; local rc=$?; echo "[$(date +%T)] $name rc=$rc"; return $rc; }
b() { step "$1" 300 python bench.py --no-gpu-probe --no-reference-mode "${@:2}"; }
for i in 1 2; do
  for p in 0 4 5; do
    b rtt20_p${p}_$i --steps 150 --warmup 20 --rtt-ms 20 --prefetch $p || exit 1
    b rtt2_p${p}_$i --steps 300 --warmup 30 --rtt-ms 2 --prefetch $p || exit 1
  done
done
python tools/bench_summary.py "$out"/*.log > "$out/SUMMARY.txt" 2>&1 || true
cat "$out/SUMMARY.txt"
