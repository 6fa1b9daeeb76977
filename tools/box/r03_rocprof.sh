#!/bin/bash
# rocprofv3 evidence for this round's GPU path: kernel trace + stats of the
# v1 resume (GPU-only and hybrid, direct DMA from the page cache), then one
# counter pass over the GPU-only run (VALU issue vs busy cycles).
set -o pipefail
OUT=${OUT:-gpurun_out/r03_rocprof}
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/kt -o resume -- python3 tools/bench_resume.py --gb 4 --version 1 --device gpu hybrid --reps 2 > $OUT/resume_kt.log 2>&1 &&
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_BUSY_CYCLES SQ_WAVE_CYCLES GRBM_GUI_ACTIVE --output-format csv -d $OUT/pmc -o resume -- python3 tools/bench_resume.py --gb 2 --version 1 --device gpu --reps 1 > $OUT/resume_pmc.log 2>&1
rc=$?
find $OUT -name "*.csv" | head -20
for f in $(find $OUT/kt -name "*kernel_stats.csv"); do head -12 $f; done
grep warm $OUT/resume_kt.log | cut -c1-220
exit $rc
