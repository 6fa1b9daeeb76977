#!/bin/bash
# 1 GiB HTTP job: S3 part size (8/16/32/64 MiB) and parallel parts (4/8).
set -o pipefail
OUT=gpurun_out/r02_big_ab2
mkdir -p $OUT
export TMPDIR=/tmp
rc=0
run() { timeout -k 10 200 python bench.py --steps 12 --warmup 2 --file-mb 1024 --no-gpu-probe "$@"; }
for rep in 1 2; do
  for part in 64 32 16 8; do
    run --s3-part-mb $part > $OUT/part${part}_$rep.log 2>&1 || { rc=$?; break 2; }
  done
  [ $rc -eq 0 ] && { TRITONDL_S3_PARALLEL_PARTS=8 run --s3-part-mb 16 > $OUT/part16_par8_$rep.log 2>&1 || { rc=$?; break; }; }
done
for f in $OUT/*.log; do echo "$(basename $f) $(grep -o '"value": [0-9.]*' $f | head -1) $(grep -o '"fetched": [0-9.]*, "download": [0-9.]*' $f) $(grep -o '"cpu_ms_per_job[^}]*' $f)"; done
exit $rc
