#!/bin/bash
# bench default (rank on CCD 0, fakes on CCD 1) vs fakes on the rank's CCD vs
# unpinned, and the 1 GiB job: unpinned vs one CCD vs two CCDs (fakes apart).
set -o pipefail
OUT=${OUT:-gpurun_out/r03_place_ab2}
mkdir -p $OUT
export TMPDIR=/tmp
rc=0
for rep in 1 2; do
  for v in default same none; do
    case $v in default) args="";; same) args="--fake-cpus same";; none) args="--cpus none";; esac
    timeout -k 10 200 python bench.py --steps 300 --warmup 10 --no-gpu-probe $args > $OUT/bench_${v}_$rep.log 2>&1 || { rc=$?; break 2; }
  done
  for v in none ccd1 ccd2; do
    case $v in none) args="--cpus none";; ccd1) args="";; ccd2) args="--cpus 0-15,128-143 --fake-cpus 16-23,144-151";; esac
    timeout -k 10 200 python bench.py --steps 12 --warmup 2 --file-mb 1024 --no-gpu-probe $args > $OUT/bench_1g_${v}_$rep.log 2>&1 || { rc=$?; break 2; }
  done
done
[ $rc = 0 ] && timeout -k 10 200 python bench.py --steps 20 --warmup 5 > $OUT/bench_driver20.log 2>&1 || rc=$?
for f in $OUT/bench_*.log; do
  echo "$(basename $f) $(grep -o '"value": [0-9.]*' $f | tr '\n' ' ') $(grep -o '"ingest_MB_per_sec": [0-9.]*' $f) $(grep -o '"cpus": "[^"]*"' $f) $(grep -o '"fake_cpus": "[^"]*"' $f | cut -c1-30) $(grep -o '"cpu_ms_per_job[^}]*' $f) $(grep -o '"job_latency_ms_p50": [0-9.]*' $f)"
done
exit $rc
