#!/bin/bash
# 16-lane SHA-256 claim policy, alternated x5 (headline, --cpuprofile):
#   ni    TRITONDL_SHA_MB=0        SHA-NI pairs everywhere
#   mb0   TRITONDL_SHA_MB_TAIL=32   16-chunk claims except the last 32 chunks
#   t64   default                  16-chunk claims except the last 64 chunks
set -o pipefail
OUT=${OUT:-gpurun_out/r03_mb_ab2}
mkdir -p $OUT
export TMPDIR=/tmp
hd() {  # name env...
  local name=$1; shift
  env "$@" timeout -k 10 200 python bench.py --steps 300 --warmup 10 --no-gpu-probe --cpuprofile $OUT/$name.prof \
    > $OUT/head_$name.log 2>&1 || return $?
}
for rep in 1 2 3 4 5; do
  hd ni$rep TRITONDL_SHA_MB=0 && hd mb0_$rep TRITONDL_SHA_MB_TAIL=32 && hd t64_$rep || exit $?
done
for f in $OUT/head_*.log; do
  n=$(basename $f .log)
  echo "$n $(grep -o '"value": [0-9.]*' $f) $(grep -o '"cpu_ms_per_job[^}]*' $f) $(grep -o '"job_spans_ms_p50": {[^}]*}' $f)"
done
exit 0
