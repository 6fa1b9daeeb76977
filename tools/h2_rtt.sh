#!/usr/bin/env bash
# https jobs at 2 and 20 ms RTT against the HTTP/2 fake origin and the HTTP/1.1 one, alternated
# (default worker config: HTTP/2 offered, adaptive concurrency).  Usage: bash tools/h2_rtt.sh OUTDIR
set -o pipefail
out=${1:-gpurun_out/r06_h2_rtt}
mkdir -p "$out"
export TMPDIR=/tmp
step() { local name=$1 lim=$2; shift 2; echo "[$(date +%T)] $name"; timeout -k 10 "$lim" "$@" > "$out/$name.log" 2>&1; local rc=$?; echo "[$(date +%T)] $name rc=$rc"; return $rc; }
b() { step "$1" 300 python bench.py --no-gpu-probe --no-reference-mode --tls "${@:2}"; }
for i in 1 2; do
  b rtt20_h2_$i --h2-origin --rtt-ms 20 --steps 150 --warmup 20 || exit 1
  b rtt20_h1_$i --rtt-ms 20 --steps 150 --warmup 20 || exit 1
  b rtt2_h2_$i --h2-origin --rtt-ms 2 --steps 300 --warmup 30 || exit 1
  b rtt2_h1_$i --rtt-ms 2 --steps 300 --warmup 30 || exit 1
done
python tools/bench_summary.py "$out"/*.log > "$out/SUMMARY.txt" 2>&1 || true
cat "$out/SUMMARY.txt"
