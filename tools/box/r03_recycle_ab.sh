#!/bin/bash
# Spare-file recycling (default) vs delete every job file
# (TRITONDL_RECYCLE_BYTES=0): headline x4 alternated, with --cpuprofile, then
# the cost probe's pwrite_new / unlink / pwrite_reuse floors.
set -o pipefail
OUT=${OUT:-gpurun_out/r03_recycle_ab}
mkdir -p $OUT
export TMPDIR=/tmp
hd() {  # name args...
  local name=$1; shift
  timeout -k 10 200 python bench.py --steps 300 --warmup 10 --no-gpu-probe --cpuprofile $OUT/$name.prof "$@" \
    > $OUT/head_$name.log 2>&1 || return $?
}
for rep in ${REPS:-1 2 3 4}; do
  hd recycle_$rep && TRITONDL_RECYCLE_BYTES=0 hd delete_$rep || exit $?
done
timeout -k 10 300 python tools/cost_probe.py --dir /tmp --reps 30 > $OUT/probe.jsonl 2>&1 || exit $?
for f in $OUT/head_*.log; do
  n=$(basename $f .log)
  echo "$n $(grep -o '"value": [0-9.]*' $f) $(grep -o '"cpu_ms_per_job[^}]*' $f) $(grep -o '"job_latency_ms_p50": [0-9.]*' $f)"
done
grep -E 'pwrite|unlink' $OUT/probe.jsonl
exit 0
