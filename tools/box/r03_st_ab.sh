#!/bin/bash
# Chunk hashers per PUT with the 16-lane kernel: default (half the CPUs,
# 8 on the box) vs 4 vs 2, headline x4 alternated with --cpuprofile.
set -o pipefail
OUT=${OUT:-gpurun_out/r03_st_ab}
mkdir -p $OUT
export TMPDIR=/tmp
hd() {  # name args...
  local name=$1; shift
  timeout -k 10 200 python bench.py --steps 300 --warmup 10 --no-gpu-probe --cpuprofile $OUT/$name.prof "$@" \
    > $OUT/head_$name.log 2>&1 || return $?
}
for rep in 1 2 3 4; do
  hd st8_$rep && hd st4_$rep --sign-threads 4 && hd st2_$rep --sign-threads 2 || exit $?
done
for f in $OUT/head_*.log; do
  n=$(basename $f .log)
  echo "$n $(grep -o '"value": [0-9.]*' $f) $(grep -o '"cpu_ms_per_job[^}]*' $f) $(grep -o '"job_latency_ms_p50": [0-9.]*' $f)"
done
exit 0
