#!/bin/bash
# A/B of two builds of the relay module, alternated in one session:
# ab/_relay_a.so (before) vs ab/_relay_b.so (after).  Headline 3x each,
# 8-worker pool 2x each, then one 1 kHz profile of b over 1000 jobs.
set -o pipefail
OUT=${OUT:-gpurun_out/r03_ab_so}
mkdir -p $OUT
export TMPDIR=/tmp
SO=tritondl/_relay.cpython-310-x86_64-linux-gnu.so
use() { cp ab/_relay_$1.so $SO || exit 1; }
run() {  # name
  timeout -k 10 200 python bench.py --steps 300 --warmup 10 --no-gpu-probe --cpuprofile $OUT/$1.prof \
    > $OUT/head_$1.log 2>&1 || return $?
}
pool() {
  timeout -k 10 300 python tools/bench_pool.py --workers 8 --jobs-per-worker 100 --file-kb 10240 --nodes 4 \
    > $OUT/pool_$1.log 2>&1 || return $?
}
for rep in 1 2 3; do
  use a && run a$rep && use b && run b$rep || exit $?
done
use a && pool a1 && use b && pool b1 && use a && pool a2 && use b && pool b2 || exit $?
use b && TRITONDL_PROFILE_HZ=1000 timeout -k 10 300 python bench.py --steps 1000 --warmup 10 --no-gpu-probe \
  --cpuprofile $OUT/b_hires.prof > $OUT/head_b_hires.log 2>&1
rc=$?
for f in $OUT/head_*.log $OUT/pool_*.log; do
  n=$(basename $f .log)
  echo "$n $(grep -o '"value": [0-9.]*' $f | head -1) $(grep -o '"cpu_ms_per_job[^}]*' $f) $(grep -o '"job_latency_ms_p50": [0-9.]*' $f)"
  [ -f $OUT/${n#head_}.prof.txt ] && grep -A4 'cpu by thread class' $OUT/${n#head_}.prof.txt | tail -3
done
exit $rc
