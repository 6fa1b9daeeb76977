#!/bin/bash
# With recycled files (no page allocation in the receive pumps), do parallel
# Range streams pay on the 10 MiB headline now?  default (one stream) vs a
# 5 MiB GET probe + 1 range (2 streams) vs 2.5 MiB probe + 3 ranges (4),
# alternated x3.
set -o pipefail
OUT=${OUT:-gpurun_out/r03_seg_ab}
mkdir -p $OUT
export TMPDIR=/tmp
hd() {
  local name=$1; shift
  timeout -k 10 200 python bench.py --steps 300 --warmup 10 --no-gpu-probe "$@" > $OUT/head_$name.log 2>&1 || return $?
}
for rep in ${REPS:-1 2 3}; do
  hd one_$rep && hd two_$rep --probe-kb 5120 || exit $?
  [ -n "$NO_FOUR" ] || hd four_$rep --probe-kb 2560 || exit $?
done
for f in $OUT/head_*.log; do
  n=$(basename $f .log)
  echo "$n $(grep -o '"value": [0-9.]*' $f) $(grep -o '"cpu_ms_per_job[^}]*' $f) $(grep -o '"job_latency_ms_p50": [0-9.]*' $f)"
done
exit 0
