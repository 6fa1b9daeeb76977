#!/usr/bin/env bash
# Whole jobs over HTTP/2 on an MI355X box: the https headline against the HTTP/2 fake origin vs
# the HTTP/1.1 one (alternated, every job content-checked), then an 8-minute soak over HTTP/2 with
# leases, adaptive concurrency, 2 ms RTT, retries and heartbeats.  Usage: bash tools/h2_soak.sh OUTDIR
set -o pipefail
out=${1:-gpurun_out/r06_h2_soak}
mkdir -p "$out"
export TMPDIR=/tmp
step() { local name=$1 lim=$2; shift 2; echo "[$(date +%T)] $name"; timeout -k 10 "$lim" "$@" > "$out/$name.log" 2>&1; local rc=$?; echo "[$(date +%T)] $name rc=$rc"; return $rc; }
for i in 1 2 3; do
  step tls_h2origin_$i 300 python bench.py --no-gpu-probe --no-reference-mode --tls --h2-origin --steps 200 --warmup 20 || exit 1
  step tls_h1origin_$i 300 python bench.py --no-gpu-probe --no-reference-mode --tls --steps 200 --warmup 20 || exit 1
done
python tools/bench_summary.py "$out"/tls_*.log > "$out/SUMMARY.txt" 2>&1 || true
step soak 620 python -m tritondl_testkit.soak --minutes 8 --rate 50 --file-kb 1024 --torrent-jobs 0 \
    --fail-every 100 --retry-delay 2 --heartbeat 10 --tls --h2-origin --rtt-ms 2 --concurrency 0 \
    --lease-after 0.0001 --sample-seconds 60 --warmup-minutes 2 --out "$out/soak.jsonl" || exit 1
cat "$out/SUMMARY.txt"
tail -n 1 "$out/soak.jsonl" | cut -c1-2500
