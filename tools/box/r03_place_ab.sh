#!/bin/bash
# Placement A/Bs: 8-worker pool with one L3 domain per worker vs consecutive
# CPU-id slices; headline with the fakes on the next CCD vs on the rank's;
# 1 GiB job and https pinned vs unpinned.  Alternated in one session.
set -o pipefail
OUT=${OUT:-gpurun_out/r03_place_ab}
mkdir -p $OUT
export TMPDIR=/tmp
rc=0
for rep in 1 2; do
  for v in l3 slice; do
    timeout -k 10 300 python tools/bench_pool.py --workers 8 --jobs-per-worker 100 --file-kb 10240 --nodes 4 --placement $v > $OUT/pool_${v}_$rep.log 2>&1 || { rc=$?; break 2; }
  done
  [ $rc = 0 ] || break
  for v in same apart; do
    if [ $v = apart ]; then args="--fake-cpus auto"; else args=""; fi
    timeout -k 10 200 python bench.py --steps 300 --warmup 10 --no-gpu-probe $args > $OUT/bench_fakes_${v}_$rep.log 2>&1 || { rc=$?; break 2; }
  done
  [ $rc = 0 ] || break
  for v in auto none; do
    timeout -k 10 200 python bench.py --steps 12 --warmup 2 --file-mb 1024 --no-gpu-probe --cpus $v > $OUT/bench_1g_${v}_$rep.log 2>&1 || { rc=$?; break 2; }
    timeout -k 10 200 python bench.py --steps 300 --warmup 10 --tls --no-gpu-probe --cpus $v > $OUT/bench_https_${v}_$rep.log 2>&1 || { rc=$?; break 2; }
  done
done
for f in $OUT/pool_*.log $OUT/bench_*.log; do
  echo "$(basename $f) $(grep -o '"value": [0-9.]*' $f | tr '\n' ' ') $(grep -o '"ingest_MB_per_sec": [0-9.]*' $f) $(grep -o '"fake_cpus": "[^"]*"' $f | cut -c1-40) $(grep -o '"cpu_ms_per_job[^}]*' $f) $(grep -o '"job_latency_ms_p50": [0-9.]*' $f)"
done
exit $rc
