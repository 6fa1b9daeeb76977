#!/bin/bash
# Two-stream SHA-NI (default) vs OpenSSL (TRITONDL_SHA_NI=0) for every
# SHA-256: headline bench alternated, the 8-worker pool, raw hash rates.
set -o pipefail
OUT=gpurun_out/r02_sha_ab
mkdir -p $OUT
export TMPDIR=/tmp
rc=0
timeout -k 10 120 python tools/bench_sha.py --mb 128 --threads 1,4,8 > $OUT/bench_sha.jsonl 2>&1 || rc=$?
for rep in 1 2 3; do
  for v in 0 1; do
    [ $rc -eq 0 ] || break 2
    TRITONDL_SHA_NI=$v timeout -k 10 200 python bench.py --steps 300 --warmup 10 --no-gpu-probe > $OUT/sha${v}_$rep.log 2>&1 || { rc=$?; break 2; }
  done
done
for v in 0 1; do
  [ $rc -eq 0 ] || break
  TRITONDL_SHA_NI=$v timeout -k 10 300 python tools/bench_pool.py --workers 8 --jobs-per-worker 100 --file-kb 10240 --nodes 4 > $OUT/pool_sha$v.log 2>&1 || rc=$?
done
cat $OUT/bench_sha.jsonl
for f in $OUT/*.log; do echo "$(basename $f) $(grep -o '"value": [0-9.]*' $f | head -1) $(grep -o '"cpu_ms_per_job[^}]*' $f) $(grep -o '"job_spans_ms_p50[^}]*' $f)"; done
exit $rc
