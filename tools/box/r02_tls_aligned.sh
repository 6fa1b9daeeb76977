#!/bin/bash
# https headline: Range segments aligned with multipart parts (each 5 MiB part
# streams behind its own GET segment) vs the single-stream default, alternated.
set -o pipefail
OUT=gpurun_out/r02_tls_aligned
mkdir -p $OUT
export TMPDIR=/tmp
rc=0
for rep in 1 2; do
  timeout -k 10 200 python bench.py --steps 200 --warmup 10 --tls --no-gpu-probe > $OUT/base_$rep.log 2>&1 || { rc=$?; break; }
  timeout -k 10 200 python bench.py --steps 200 --warmup 10 --tls --no-gpu-probe --probe-kb 5120 --http-segments 2 --s3-part-mb 5 --s3-multipart-mb 8 > $OUT/aligned2_$rep.log 2>&1 || { rc=$?; break; }
  timeout -k 10 200 python bench.py --steps 200 --warmup 10 --tls --no-gpu-probe --probe-kb 5120 --http-segments 2 > $OUT/seg2_$rep.log 2>&1 || { rc=$?; break; }
done
for f in $OUT/*.log; do echo "$(basename $f) $(grep -o '"value": [0-9.]*' $f | head -1) $(grep -o '"job_spans_ms_p50[^}]*' $f) $(grep -o '"cpu_ms_per_job[^}]*' $f)"; done
exit $rc
