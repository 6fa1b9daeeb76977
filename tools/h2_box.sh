#!/usr/bin/env bash
# The native HTTP/2 pump on an MI355X box: GPU tests + smoke on this tree, the HTTP/2 tests,
# the HTTP/2 vs HTTP/1.1 A/B, and the driver's bench command twice.
# Usage (repo root, GPU box): bash tools/h2_box.sh OUTDIR
set -o pipefail
out=${1:-gpurun_out/r06_h2_box}
mkdir -p "$out"
export TMPDIR=/tmp
step() { local name=$1 lim=$2; shift 2; echo "[$(date +%T)] $name"; timeout -k 10 "$lim" "$@" > "$out/$name.log" 2>&1; local rc=$?; echo "[$(date +%T)] $name rc=$rc"; return $rc; }
step pytest_gpu 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread || exit 1
step smoke 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" || exit 1
step test_h2 300 python -u -m pytest tests/test_h2.py -x -q --timeout 120 --timeout-method thread || exit 1
step h2_ab 600 python tools/h2_ab.py --runs 3 --out "$out/h2_ab" || exit 1
step driver_1 300 python bench.py --gpus 1 --steps 20 --warmup 5 || exit 1
step driver_2 300 python bench.py --gpus 1 --steps 20 --warmup 5 || exit 1
tail -n 5 "$out/h2_ab.log"
