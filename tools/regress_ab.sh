#!/usr/bin/env bash
# Same-box A/B of the driver's bench command: this tree against OLD_TREE (a checkout with its own
# built .so files), alternated.  Usage (repo root, GPU box): bash tools/regress_ab.sh OUTDIR OLD_TREE [N]
set -o pipefail
out=$(realpath -m "${1:-gpurun_out/r06_regress_ab}")
old=${2:-.ab/base}
n=${3:-4}
mkdir -p "$out"
export TMPDIR=/tmp
run() {
  local name=$1 dir=$2; shift 2
  echo "[$(date +%T)] $name"
  (cd "$dir" && timeout -k 10 300 python bench.py "$@" > "$out/$name.log" 2>&1)
  local rc=$?; echo "[$(date +%T)] $name rc=$rc"; return $rc
}
for i in $(seq 1 "$n"); do
  run new_$i . --gpus 1 --steps 20 --warmup 5 || exit 1
  run old_$i "$old" --gpus 1 --steps 20 --warmup 5 || exit 1
done
for i in 1 2; do
  run new300_$i . --steps 300 --warmup 30 --no-reference-mode || exit 1
  run old300_$i "$old" --steps 300 --warmup 30 --no-reference-mode || exit 1
done
python tools/bench_summary.py "$out"/*.log > "$out/SUMMARY.txt" 2>&1 || true
cat "$out/SUMMARY.txt"
