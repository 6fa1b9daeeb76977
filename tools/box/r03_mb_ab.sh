#!/bin/bash
# 16-lane AVX-512 SHA-256 on (default) vs off (TRITONDL_SHA_MB=0: SHA-NI
# pairs), alternated: headline x5 with --cpuprofile, 8-worker pool x2.
set -o pipefail
OUT=${OUT:-gpurun_out/r03_mb_ab}
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
  hd ni$rep TRITONDL_SHA_MB=0 && hd mb$rep TRITONDL_SHA_MB=1 || exit $?
done
for rep in 1 2; do
  pool ni$rep TRITONDL_SHA_MB=0 && pool mb$rep TRITONDL_SHA_MB=1 || exit $?
done
for f in $OUT/head_*.log $OUT/pool_*.log; do
  n=$(basename $f .log)
  echo "$n $(grep -o '"value": [0-9.]*' $f) $(grep -o '"cpu_ms_per_job[^}]*' $f) $(grep -o '"job_latency_ms_p50": [0-9.]*' $f)"
  [ -f $OUT/${n#head_}.prof.txt ] && grep -A4 'cpu by thread class' $OUT/${n#head_}.prof.txt | tail -3
done
exit 0
