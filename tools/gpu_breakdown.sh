#!/usr/bin/env bash
# Stage breakdown of the flagship job on a GPU box (tools/bench_breakdown.py).
set -o pipefail
out=${1:-gpurun_out/breakdown}
mkdir -p "$out"
TRITONDL_TRACE=1 timeout -k 10 240 python tools/bench_breakdown.py --file-mb 10 --reps 30 > "$out/bd_10m.json" 2> "$out/bd_10m.err" &&
timeout -k 10 240 python tools/bench_breakdown.py --file-mb 10 --reps 30 --payload unsigned > "$out/bd_10m_unsigned.json" 2> "$out/bd_10m_unsigned.err" &&
TRITONDL_TRACE=1 timeout -k 10 300 python tools/bench_breakdown.py --file-mb 1024 --reps 3 > "$out/bd_1g.json" 2> "$out/bd_1g.err" &&
timeout -k 10 240 python bench.py --steps 100 --warmup 10 > "$out/bench_c1.json" 2> "$out/bench_c1.err"
echo "rc=$?"
