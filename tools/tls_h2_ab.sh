#!/usr/bin/env bash
# The https headline (TLS 1.3 origin and S3, the fake origin speaks HTTP/1.1 only) with the
# worker offering HTTP/2 (ALPN h2, then the remembered HTTP/1.1 fallback) against not offering it,
# alternated, plus GPU tests and smoke on this tree.  Usage (repo root, GPU box): bash tools/tls_h2_ab.sh OUTDIR
set -o pipefail
out=${1:-gpurun_out/r06_tls_h2_ab}
mkdir -p "$out"
export TMPDIR=/tmp
step() { local name=$1 lim=$2; shift 2; echo "[$(date +%T)] $name"; timeout -k 10 "$lim" "$@" > "$out/$name.log" 2>&1; local rc=$?; echo "[$(date +%T)] $name rc=$rc"; return $rc; }
step pytest_gpu 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread || exit 1
step smoke 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" || exit 1
for i in 1 2 3; do
  step tls_h2on_$i 300 python bench.py --no-gpu-probe --no-reference-mode --tls --steps 200 --warmup 20 --http2 on || exit 1
  step tls_h2off_$i 300 python bench.py --no-gpu-probe --no-reference-mode --tls --steps 200 --warmup 20 --http2 off || exit 1
done
step driver 300 python bench.py --gpus 1 --steps 20 --warmup 5 || exit 1
python tools/bench_summary.py "$out"/*.log > "$out/SUMMARY.txt" 2>&1 || true
cat "$out/SUMMARY.txt"
