#!/bin/bash
# Job-dir cleanup: reaper thread (tree) vs one executor hop per job
# (tools/box/alt/service_exec_cleanup.py, the previous service.py).
# Headline x4 alternated in one session.
set -o pipefail
OUT=${OUT:-gpurun_out/r03_reaper_ab}
mkdir -p $OUT
export TMPDIR=/tmp
cp tritondl/service.py $OUT/.service_reaper.py
hd() {  # name args...
  local name=$1; shift
  timeout -k 10 200 python bench.py --steps 300 --warmup 10 --no-gpu-probe --cpuprofile $OUT/$name.prof "$@" \
    > $OUT/head_$name.log 2>&1 || return $?
}
for rep in 1 2 3 4; do
  cp $OUT/.service_reaper.py tritondl/service.py && hd reaper_$rep || exit $?
  cp tools/box/alt/service_exec_cleanup.py tritondl/service.py && hd exec_$rep || exit $?
done
cp $OUT/.service_reaper.py tritondl/service.py
rm -f $OUT/.service_reaper.py
for f in $OUT/head_*.log; do
  n=$(basename $f .log)
  echo "$n $(grep -o '"value": [0-9.]*' $f) $(grep -o '"cpu_ms_per_job[^}]*' $f) $(grep -o '"job_latency_ms_p50": [0-9.]*' $f)"
done
exit 0
