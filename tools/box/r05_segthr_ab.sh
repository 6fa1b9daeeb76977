#!/bin/bash
# Round 5: should mid-size files (16-64 MiB) be fetched as parallel Range
# streams?  32 MiB jobs with the default threshold (64 MiB: one stream) vs
# 16 MiB (4 streams; the open-ended first GET is cut at its segment end),
# uncapped (loopback) and with each stream capped at 800 Mbit/s (a WAN
# origin's window / RTT).  Alternated runs.
set -o pipefail
OUT=${OUT:-gpurun_out/r05_segthr_ab}
mkdir -p $OUT
export TMPDIR=/tmp
b() { local name=$1; shift; timeout -k 10 240 python bench.py --file-mb 32 --warmup 2 --no-gpu-probe \
      --no-reference-mode "$@" > $OUT/$name.log 2>&1; }
for i in 1 2 3; do
  b open_thr64_$i --steps 60 &&
  b open_thr16_$i --steps 60 --segment-threshold-mb 16 &&
  b cap_thr64_$i --steps 12 --stream-mbps 800 &&
  b cap_thr16_$i --steps 12 --stream-mbps 800 --segment-threshold-mb 16 || break
done
rc=$?
for f in $OUT/*.log; do
  echo "$(basename $f) $(grep -o '"value": [0-9.]*' $f | head -1) $(grep -o '"ingest_MB_per_sec": [0-9.]*' $f | head -1)"
done
exit $rc
