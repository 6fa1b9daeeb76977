#!/bin/bash
# Splice receive (socket -> pipe -> file) vs recv + pwrite, with the 16-lane
# SHA-256 default; headline x5 alternated with --cpuprofile, pool x2.
set -o pipefail
OUT=${OUT:-gpurun_out/r03_splice_ab}
mkdir -p $OUT
export TMPDIR=/tmp
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
for rep in 1 2 3 4 5; do
  hd rp$rep TRITONDL_RELAY_SPLICE=0 && hd sp$rep TRITONDL_RELAY_SPLICE=1 || exit $?
done
for rep in 1 2; do
  env TRITONDL_RELAY_SPLICE=0 timeout -k 10 200 python bench.py --steps 12 --warmup 2 --file-mb 1024 --no-gpu-probe > $OUT/big_rp$rep.log 2>&1 &&
  env TRITONDL_RELAY_SPLICE=1 timeout -k 10 200 python bench.py --steps 12 --warmup 2 --file-mb 1024 --no-gpu-probe > $OUT/big_sp$rep.log 2>&1 || exit $?
done
for rep in 1 2; do
  pool rp$rep TRITONDL_RELAY_SPLICE=0 && pool sp$rep TRITONDL_RELAY_SPLICE=1 || exit $?
done
for f in $OUT/head_*.log $OUT/big_*.log $OUT/pool_*.log; do
  n=$(basename $f .log)
  echo "$n $(grep -o '"value": [0-9.]*' $f) $(grep -o '"cpu_ms_per_job[^}]*' $f) $(grep -o '"job_spans_ms_p50": {[^}]*}' $f)"
done
exit 0
