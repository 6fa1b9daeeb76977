#!/usr/bin/env bash
# Adaptive concurrency with job intensity (v3) on an MI355X box: loopback (driver form), 2 / 20 ms
# RTT, a bandwidth-limited origin (100 MB/s per stream), and https against the HTTP/2 fake at 2 ms,
# each with the default against a fixed concurrency of 1.  Usage: bash tools/adaptive_v3.sh OUTDIR
set -o pipefail
out=${1:-gpurun_out/r06_adaptive_v3}
mkdir -p "$out"
export TMPDIR=/tmp
step() { local name=$1 lim=$2; shift 2; echo "[$(date +%T)] $name"; timeout -k 10 "$lim" "$@" > "$out/$name.log" 2>&1; local rc=$?; echo "[$(date +%T)] $name rc=$rc"; return $rc; }
b() { step "$1" 300 python bench.py --no-gpu-probe --no-reference-mode "${@:2}"; }
for i in 1 2 3; do
  step driver_$i 300 python bench.py --gpus 1 --steps 20 --warmup 5 || exit 1
done
b loop300_default --steps 300 --warmup 30 || exit 1
b rtt2_default --steps 300 --warmup 30 --rtt-ms 2 || exit 1
b rtt20_default --steps 150 --warmup 20 --rtt-ms 20 || exit 1
b slow_default --steps 100 --warmup 20 --stream-mbps 800 || exit 1
b slow_c1 --steps 40 --warmup 5 --stream-mbps 800 --concurrency 1 || exit 1
b h2rtt2_default --tls --h2-origin --rtt-ms 2 --steps 300 --warmup 30 || exit 1
b h2rtt2_c1 --tls --h2-origin --rtt-ms 2 --steps 150 --warmup 20 --concurrency 1 || exit 1
b tls_default --tls --steps 200 --warmup 20 || exit 1
python tools/bench_summary.py "$out"/*.log > "$out/SUMMARY.txt" 2>&1 || true
for f in "$out"/*.log; do
  tail -n 1 "$f" | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$f'.split('/')[-1], d['value'], d['config'].get('concurrency_limit_end'), d['diag']['concurrency']['last_decision'])"
done
