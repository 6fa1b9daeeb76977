#!/bin/bash
# rocprofv3 kernel trace + stats of the v1 resume at the round-5 tree
# (GPU-only and hybrid).  TRITONDL_GPU_HELPER=0 keeps the hasher in the
# profiled process: nothing is spawned under the profiler.
set -o pipefail
OUT=${OUT:-gpurun_out/r05_rocprof}
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
export TRITONDL_GPU_HELPER=0
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/kt -o resume -- python3 tools/bench_resume.py --gb 4 --version 1 --device gpu hybrid --reps 2 > $OUT/resume_kt.log 2>&1
rc=$?
for f in $(find $OUT/kt -name "*kernel_stats.csv"); do head -12 $f; done
grep warm $OUT/resume_kt.log | cut -c1-220
exit $rc
