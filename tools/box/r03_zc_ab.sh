#!/bin/bash
# Round-3 A/B, alternated in one session: zero-copy chunked PUT (sendfile +
# hashing from a mapping) vs the ring path, and splice receive on/off.
# Headline (1 worker) and the 8-worker pool, each config twice.
set -o pipefail
OUT=${OUT:-gpurun_out/r03_zc_ab}
mkdir -p $OUT
export TMPDIR=/tmp
run() {  # name env...
  local name=$1; shift
  env "$@" timeout -k 10 200 python bench.py --steps 300 --warmup 10 --no-gpu-probe > $OUT/head_$name.log 2>&1 || return $?
}
pool() {
  local name=$1; shift
  env "$@" timeout -k 10 300 python tools/bench_pool.py --workers 8 --jobs-per-worker 100 --file-kb 10240 --nodes 4 > $OUT/pool_$name.log 2>&1 || return $?
}
for rep in 1 2; do
  run ring$rep TRITONDL_RELAY_ZC=0 && run zc$rep TRITONDL_RELAY_ZC=1 && run zcsplice$rep TRITONDL_RELAY_ZC=1 TRITONDL_RELAY_SPLICE=1 || exit $?
done &&
pool ring TRITONDL_RELAY_ZC=0 && pool zc TRITONDL_RELAY_ZC=1 && pool ring2 TRITONDL_RELAY_ZC=0 && pool zc2 TRITONDL_RELAY_ZC=1 &&
timeout -k 10 200 python bench.py --steps 300 --warmup 10 --no-gpu-probe --cpuprofile $OUT/zc.prof > $OUT/head_zc_prof.log 2>&1
rc=$?
for f in $OUT/head_*.log $OUT/pool_*.log; do echo "$(basename $f) $(grep -o '"value": [0-9.]*' $f | head -1) $(grep -o '"cpu_ms_per_job[^}]*' $f) $(grep -o '"job_latency_ms_p50": [0-9.]*' $f)"; done
head -8 $OUT/zc.prof.txt
exit $rc
