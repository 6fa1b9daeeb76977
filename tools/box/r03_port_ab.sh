#!/bin/bash
# Relay A/B in one session, alternated:
#   old    ab/_relay_a.so: pumps on executor threads, every hasher woken per flow advance
#   flow   new build, TRITONDL_RELAY_PORT=0, no hasher cap: targeted wake-ups only
#   port   new build, no hasher cap: + pumps on the native pool, reaped via an eventfd
#   cap    new build defaults: + 2 hashers while the PUT follows a download
set -o pipefail
OUT=${OUT:-gpurun_out/r03_port_ab}
mkdir -p $OUT
export TMPDIR=/tmp
SO=tritondl/_relay.cpython-310-x86_64-linux-gnu.so
use() { cp ab/_relay_$1.so $SO || exit 1; }
hd() {  # name env...
  local name=$1; shift
  env "$@" timeout -k 10 200 python bench.py --steps 300 --warmup 10 --no-gpu-probe --cpuprofile $OUT/$name.prof \
    > $OUT/head_$name.log 2>&1 || return $?
}
pool() {
  local name=$1; shift
  env "$@" timeout -k 10 300 python tools/bench_pool.py --workers 8 --jobs-per-worker 100 --file-kb 10240 --nodes 4 \
    > $OUT/pool_$name.log 2>&1 || return $?
}
for rep in 1 2 3; do
  use a && hd old$rep && use b && hd flow$rep TRITONDL_RELAY_PORT=0 TRITONDL_RELAY_FOLLOW_HASHERS=0 &&
    hd port$rep TRITONDL_RELAY_FOLLOW_HASHERS=0 && hd cap$rep || exit $?
done
for rep in 1 2; do
  use a && pool old$rep && use b && pool port$rep TRITONDL_RELAY_FOLLOW_HASHERS=0 && pool cap$rep || exit $?
done
for f in $OUT/head_*.log $OUT/pool_*.log; do
  n=$(basename $f .log)
  echo "$n $(grep -o '"value": [0-9.]*' $f | head -1) $(grep -o '"cpu_ms_per_job[^}]*' $f) $(grep -o '"job_latency_ms_p50": [0-9.]*' $f)"
  [ -f $OUT/${n#head_}.prof.txt ] && grep -A6 'cpu by thread class' $OUT/${n#head_}.prof.txt | tail -6
done
exit 0
