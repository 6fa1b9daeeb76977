#!/bin/bash
# Job-dir cleanup: reaper thread (this tree) vs one executor hop per job
# (commit b531f9d, the service before the reaper), headline x4 alternated in
# one session.  Prepare the old arm locally first:
#   tools/ab_tree.sh b531f9d r03_exec
# It runs from its own tree (.ab/r03_exec); no tracked file is overwritten.
set -o pipefail
OUT=${OUT:-gpurun_out/r03_reaper_ab}
mkdir -p $OUT
export TMPDIR=/tmp
ROOT=$PWD
[ -d .ab/r03_exec ] || { echo "missing .ab/r03_exec (tools/ab_tree.sh b531f9d r03_exec)"; exit 2; }
hd() {  # name dir args...
  local name=$1 dir=$2; shift 2
  (cd $dir && timeout -k 10 200 python bench.py --steps 300 --warmup 10 --no-gpu-probe \
     --cpuprofile $ROOT/$OUT/$name.prof "$@") > $OUT/head_$name.log 2>&1 || return $?
}
for rep in 1 2 3 4; do
  hd reaper_$rep . || exit $?
  hd exec_$rep .ab/r03_exec || exit $?
done
for f in $OUT/head_*.log; do
  n=$(basename $f .log)
  echo "$n $(grep -o '"value": [0-9.]*' $f) $(grep -o '"cpu_ms_per_job[^}]*' $f) $(grep -o '"job_latency_ms_p50": [0-9.]*' $f)"
done
exit 0
