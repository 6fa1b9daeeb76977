#!/bin/bash
# Headline, 5 alternations: old relay build vs the new build with pumps on
# executor threads and 8 vs 2 follow hashers.
set -o pipefail
OUT=${OUT:-gpurun_out/r03_cap_ab}
mkdir -p $OUT
export TMPDIR=/tmp TRITONDL_RELAY_PORT=0
SO=tritondl/_relay.cpython-310-x86_64-linux-gnu.so
use() { cp ab/_relay_$1.so $SO || exit 1; }
hd() {  # name env...
  local name=$1; shift
  env "$@" timeout -k 10 200 python bench.py --steps 300 --warmup 10 --no-gpu-probe > $OUT/head_$name.log 2>&1 || return $?
}
for rep in 1 2 3 4 5; do
  use a && hd old$rep && use b && hd h8_$rep TRITONDL_RELAY_FOLLOW_HASHERS=0 && hd cap$rep || exit $?
done
for f in $OUT/head_*.log; do
  n=$(basename $f .log)
  echo "$n $(grep -o '"value": [0-9.]*' $f) $(grep -o '"cpu_ms_per_job[^}]*' $f) $(grep -o '"job_latency_ms_p50": [0-9.]*' $f)"
done
