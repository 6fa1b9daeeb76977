#!/bin/bash
# Pump placement, isolated: stage breakdown (fetch-only / upload-only / job)
# with pumps on executor threads (TRITONDL_RELAY_PORT=0) vs the native pool
# + completion port, then the headline with 2 follow hashers in both modes.
# Alternated, one session.
set -o pipefail
OUT=${OUT:-gpurun_out/r03_port_ab2}
mkdir -p $OUT
export TMPDIR=/tmp
bd() {  # name env...
  local name=$1; shift
  env "$@" timeout -k 10 200 python tools/bench_breakdown.py --reps 60 > $OUT/bd_$name.log 2>&1 || return $?
}
hd() {  # name env...
  local name=$1; shift
  env "$@" timeout -k 10 200 python bench.py --steps 300 --warmup 10 --no-gpu-probe --cpuprofile $OUT/$name.prof \
    > $OUT/head_$name.log 2>&1 || return $?
}
for rep in 1 2; do
  bd exec$rep TRITONDL_RELAY_PORT=0 && bd port$rep TRITONDL_RELAY_PORT=1 || exit $?
done
for rep in 1 2 3; do
  hd exec$rep TRITONDL_RELAY_PORT=0 && hd port$rep TRITONDL_RELAY_PORT=1 || exit $?
done
for f in $OUT/bd_*.log; do echo "== $f"; grep '^{' $f | cut -c1-300; done
for f in $OUT/head_*.log; do
  n=$(basename $f .log)
  echo "$n $(grep -o '"value": [0-9.]*' $f) $(grep -o '"cpu_ms_per_job[^}]*' $f) $(grep -o '"job_spans_ms_p50": {[^}]*}' $f)"
done
exit 0
