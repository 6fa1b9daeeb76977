#!/bin/bash
# Round 5: chunk-signing threads per PUT.  r05_bound showed 2 threads ahead of
# the default 4 on the 10 MiB job (370 vs 352 jobs/s, two runs each).  More
# alternated repeats on 10 MiB, and the 1 GiB job (where 4 streams outrun 2
# hashers?) with 2 vs 4.
set -o pipefail
OUT=${OUT:-gpurun_out/r05_sign_ab}
mkdir -p $OUT
export TMPDIR=/tmp
b() { local name=$1; shift; timeout -k 10 240 python bench.py --no-gpu-probe --no-reference-mode "$@" > $OUT/$name.log 2>&1; }
for i in 1 2 3; do
  b s4_$i --steps 300 --warmup 10 --sign-threads 4 &&
  b s2_$i --steps 300 --warmup 10 --sign-threads 2 &&
  b s3_$i --steps 300 --warmup 10 --sign-threads 3 &&
  b s1_$i --steps 300 --warmup 10 --sign-threads 1 || break
done
rc=$?
if [ $rc = 0 ]; then
  for i in 1 2; do
    b gib_s4_$i --file-mb 1024 --steps 6 --warmup 1 --sign-threads 4 &&
    b gib_s2_$i --file-mb 1024 --steps 6 --warmup 1 --sign-threads 2 || break
  done
  rc=$?
fi
for f in $OUT/*.log; do
  echo "$(basename $f) $(grep -o '"value": [0-9.]*' $f | head -1) $(grep -o '"job_spans_ms_p50": {[^}]*}' $f | head -1) $(grep -o '"cpu_ms_per_job": {[^}]*}' $f | head -1)"
done
exit $rc
