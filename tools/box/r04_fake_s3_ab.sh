#!/bin/bash
# Does the fake S3's verification capacity (native verifier threads per PUT,
# standing in for a remote S3 cluster) set the upload tail after the last
# fetched byte?  4 (default) vs 8 threads, alternated, 300 timed jobs each.
set -o pipefail
OUT=${OUT:-gpurun_out/r04_fake_s3}
mkdir -p $OUT
export TMPDIR=/tmp
for rep in 1 2 3; do
  for t in 4 8; do
    TRITONDL_FAKE_S3_VERIFY_THREADS=$t timeout -k 10 200 python bench.py --steps 300 --warmup 10 --no-gpu-probe >> $OUT/ab_$t.log 2>&1 || exit $?
  done
done
for f in $OUT/ab_*.log; do echo "$(basename $f) $(grep -o '"value": [0-9.]*' $f | tr '\n' ' ')"; done
