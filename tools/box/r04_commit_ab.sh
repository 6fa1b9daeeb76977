#!/bin/bash
# Pipelined commit (a job's publish confirm + ack overlap the next job) vs
# serial commit, headline x4 alternated, 300 timed jobs each.
set -o pipefail
OUT=${OUT:-gpurun_out/r04_commit_ab}
mkdir -p $OUT
export TMPDIR=/tmp
for rep in 1 2 3 4; do
  for arm in on off; do
    timeout -k 10 200 python bench.py --steps 300 --warmup 10 --no-gpu-probe --pipeline-commit $arm \
        >> $OUT/ab_$arm.log 2>&1 || exit $?
  done
done
python tools/bench_summary.py $OUT/ab_on.log $OUT/ab_off.log
