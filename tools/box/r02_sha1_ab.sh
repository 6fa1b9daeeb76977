#!/bin/bash
# SHA-1 pairs on the host (TRITONDL_SHA_NI=1, default) vs OpenSSL (=0):
# v1 resume verification of 8 GiB on cpu and hybrid, alternated.
set -o pipefail
OUT=gpurun_out/r02_sha1_ab
mkdir -p $OUT
export TMPDIR=/tmp
rc=0
for rep in 1 2; do
  for v in 0 1; do
    TRITONDL_SHA_NI=$v timeout -k 10 400 python -u tools/bench_resume.py --gb 8 --version 1 --device cpu hybrid --reps 2 > $OUT/resume_sha${v}_${rep}.log 2>&1 || { rc=$?; break 2; }
  done
done
for f in $OUT/*.log; do echo "== $f"; grep -E '^\{' $f | cut -c1-300; done
exit $rc
