#!/usr/bin/env bash
# Round-6 box matrix: GPU tests + smoke, then the headline in the driver's form and the
# 0 / 2 / 20 ms RTT table with the worker default (adaptive concurrency) against the
# reference's fixed concurrency 1.  Usage (repo root, GPU box): bash tools/box_check.sh OUTDIR [quick]
set -o pipefail
out=${1:-gpurun_out/r06_matrix}
mkdir -p "$out"
step() { local name=$1 lim=$2; shift 2; echo "[$(date +%T)] $name"; timeout -k 10 "$lim" "$@" > "$out/$name.log" 2>&1; local rc=$?; echo "[$(date +%T)] $name rc=$rc"; return $rc; }
b() { step "$1" 300 python bench.py --no-gpu-probe --no-reference-mode "${@:2}"; }
if [ "$2" != "quick" ]; then
  step pytest_gpu 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread || exit 1
  step smoke 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" || exit 1
fi
for i in 1 2 3; do
  b drv_default_$i --steps 20 --warmup 5 || exit 1
  b drv_c1_$i --steps 20 --warmup 5 --concurrency 1 || exit 1
done
for i in 1 2; do
  b rtt0_default_$i --steps 200 --warmup 20 || exit 1
  b rtt0_c1_$i --steps 200 --warmup 20 --concurrency 1 || exit 1
  b rtt2_default_$i --steps 200 --warmup 20 --rtt-ms 2 || exit 1
  b rtt2_c1_$i --steps 100 --warmup 10 --rtt-ms 2 --concurrency 1 || exit 1
  b rtt20_default_$i --steps 100 --warmup 10 --rtt-ms 20 || exit 1
  b rtt20_c1_$i --steps 40 --warmup 5 --rtt-ms 20 --concurrency 1 || exit 1
done
# price of a lease per job: every job leased at once (--lease-after ~0), default concurrency
b lease_rtt0 --steps 200 --warmup 20 --lease-after 0.0001 || exit 1
b lease_rtt2 --steps 200 --warmup 20 --rtt-ms 2 --lease-after 0.0001 || exit 1
b lease_rtt20 --steps 100 --warmup 10 --rtt-ms 20 --lease-after 0.0001 || exit 1
python tools/bench_summary.py "$out"/*.log > "$out/SUMMARY.txt" 2>&1 || true
for f in "$out"/drv*.log "$out"/rtt*.log "$out"/lease*.log; do
  tail -n 1 "$f" | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$f', d['value'], d['config']['concurrency_limit_end'], d['cpu_ms_per_job']['worker'], d['diag']['concurrency']['last_decision'])"
done
