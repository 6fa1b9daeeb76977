#!/bin/bash
# Round 5: adaptive pipelined commit.  Loopback headline alternated with the r04 tree and with
# pipelining off; then 2 / 20 ms RTT: adaptive (default) vs off.
set -o pipefail
OUT=${OUT:-gpurun_out/r05_adaptive}
mkdir -p $OUT
export TMPDIR=/tmp
R=$PWD
b() { local name=$1 dir=$2; shift 2; (cd $dir && timeout -k 10 200 python bench.py --no-gpu-probe --no-reference-mode "$@") > $OUT/$name.log 2>&1; }
for i in 1 2 3; do
  b r04_$i $R/.ab/r04 --steps 300 --warmup 10 &&
  b r05_$i $R --steps 300 --warmup 10 &&
  b r05_off_$i $R --steps 300 --warmup 10 --pipeline-commit off || break
done &&
b driver_form $R --steps 20 --warmup 5 &&
b rtt2_adaptive $R --steps 200 --warmup 5 --rtt-ms 2 &&
b rtt2_off $R --steps 200 --warmup 5 --rtt-ms 2 --pipeline-commit off &&
b rtt20_adaptive $R --steps 60 --warmup 5 --rtt-ms 20 &&
b rtt20_off $R --steps 60 --warmup 5 --rtt-ms 20 --pipeline-commit off
rc=$?
for f in $OUT/*.log; do echo "$(basename $f) $(grep -o '"value": [0-9.]*' $f | head -1) $(grep -o '"job_latency_ms_p50": [0-9.]*' $f | head -1)"; done
exit $rc
