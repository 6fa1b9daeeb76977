#!/bin/bash
# 1 GiB HTTP job: Range streams (2/4/8) and S3 part size (64/128 MiB).
set -o pipefail
OUT=gpurun_out/r02_big_ab
mkdir -p $OUT
export TMPDIR=/tmp
rc=0
run() { timeout -k 10 200 python bench.py --steps 12 --warmup 2 --file-mb 1024 --no-gpu-probe "$@"; }
for rep in 1 2; do
  for seg in 4 8 2; do
    run --http-segments $seg > $OUT/seg${seg}_$rep.log 2>&1 || { rc=$?; break 2; }
  done
  [ $rc -eq 0 ] && { run --s3-part-mb 128 > $OUT/part128_$rep.log 2>&1 || { rc=$?; break; }; }
  [ $rc -eq 0 ] && { run --s3-part-mb 32 > $OUT/part32_$rep.log 2>&1 || { rc=$?; break; }; }
done
for f in $OUT/*.log; do echo "$(basename $f) $(grep -o '"value": [0-9.]*' $f | head -1) $(grep -o '"ingest_MB_per_sec": [0-9.]*' $f) $(grep -o '"fetched": [0-9.]*, "download": [0-9.]*' $f)"; done
exit $rc
