#!/usr/bin/env bash
# rocprofv3 on the final round-6 tree's GPU path: kernel trace + stats of the v1 resume (GPU-only and
# hybrid, direct DMA from the page cache), then one counter pass over a GPU-only run (VALU issue vs
# busy cycles).  No sys/runtime trace with --pmc.  Usage (repo root, GPU box): bash tools/rocprof_r06.sh OUTDIR
set -o pipefail
OUT=${1:-gpurun_out/r06_rocprof}
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
export TRITONDL_GPU_HELPER=0          # hash in this process: nothing spawned under the profiler
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/kt" -o resume -- \
    python3 tools/bench_resume.py --gb 4 --version 1 --device gpu hybrid --reps 2 > "$OUT/resume_kt.log" 2>&1 &&
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_BUSY_CYCLES SQ_WAVE_CYCLES GRBM_GUI_ACTIVE \
    --output-format csv -d "$OUT/pmc" -o resume -- \
    python3 tools/bench_resume.py --gb 2 --version 1 --device gpu --reps 1 > "$OUT/resume_pmc.log" 2>&1
rc=$?
find "$OUT" -name "*.csv" | head -20
for f in $(find "$OUT/kt" -name "*kernel_stats.csv"); do head -12 "$f"; done
grep warm "$OUT/resume_kt.log" | cut -c1-220
exit $rc
