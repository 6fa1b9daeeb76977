#!/usr/bin/env bash
# One-box MI355X check: GPU tests, smoke, job bench (c=1, c=4), BT swarm bench.
# Usage (from the repo root, on a GPU box): bash tools/gpu_check.sh OUTDIR
set -o pipefail
out=${1:-gpurun_out/check}
mkdir -p "$out"
step() { local name=$1 lim=$2; shift 2; echo "[$(date +%T)] $name"; timeout -k 10 "$lim" "$@" > "$out/$name.log" 2>&1; local rc=$?; echo "[$(date +%T)] $name rc=$rc"; return $rc; }
step pytest_gpu 600 python -m pytest tests -m gpu -x -q &&
step smoke 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" &&
step bench_c1 300 python bench.py --steps 100 --warmup 10 &&
step bench_c4 300 python bench.py --steps 200 --warmup 20 --concurrency 4 &&
step bench_bt_tcp 300 python tools/bench_bt.py --mb 1024 --seeds 4 &&
step bench_bt_utp 300 python tools/bench_bt.py --mb 1024 --seeds 4 --utp &&
step bench_1g 300 python bench.py --file-mb 1024 --steps 3 --warmup 1 &&
step bench_pool8 300 python tools/bench_pool.py --workers 8 --jobs-per-worker 100 --file-kb 1024
