#!/bin/bash
# Does socket placement matter for the GPU resume path?  8 GiB v1 hybrid and
# GPU-only, run pinned to two CCDs of socket 0 vs two CCDs of socket 1
# (files written there, so the page cache lands on that node), alternated.
set -o pipefail
OUT=${OUT:-gpurun_out/r03_numa_ab}
mkdir -p $OUT
export TMPDIR=/tmp
rc=0
for rep in 1 2; do
  for v in s0 s1; do
    case $v in s0) c="0-15,128-143";; s1) c="64-79,192-207";; esac
    timeout -k 10 300 python -u tools/bench_resume.py --gb 8 --version 1 --device hybrid gpu --reps 2 --cpus $c > $OUT/resume_${v}_$rep.log 2>&1 || { rc=$?; break 2; }
  done
done
for f in $OUT/resume_*.log; do echo "$(basename $f)"; grep -E 'warm|gpu_numa' $f | cut -c1-200; done
exit $rc
