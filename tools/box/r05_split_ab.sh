#!/bin/bash
# Round 5: split the 10 MiB headline job into two halves on both sides?  The
# upload's single PUT stream trails the single GET stream (r05_bound).  Two
# Range streams (a 5 MiB bounded probe + the rest) and a 2 x 5 MiB multipart
# upload move both halves in parallel, at the cost of four more requests
# (second GET, initiate, second part, complete).  Alternated 300-job runs.
set -o pipefail
OUT=${OUT:-gpurun_out/r05_split_ab}
mkdir -p $OUT
export TMPDIR=/tmp
b() { local name=$1; shift; timeout -k 10 200 python bench.py --steps 300 --warmup 10 --no-gpu-probe \
      --no-reference-mode "$@" > $OUT/$name.log 2>&1; }
for i in 1 2 3; do
  b default_$i &&
  b split_$i --probe-kb 5120 --http-segments 2 --s3-multipart-mb 8 --s3-part-mb 5 &&
  b get2_$i --probe-kb 5120 --http-segments 2 &&
  b put2_$i --s3-multipart-mb 8 --s3-part-mb 5 || break
done
rc=$?
for f in $OUT/*.log; do
  echo "$(basename $f) $(grep -o '"value": [0-9.]*' $f | head -1) $(grep -o '"job_spans_ms_p50": {[^}]*}' $f | head -1) $(grep -o '"cpu_ms_per_job": {[^}]*}' $f | head -1)"
done
exit $rc
