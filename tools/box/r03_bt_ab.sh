#!/bin/bash
# BitTorrent ingest with 16-piece live verification (default) vs SHA-NI pairs
# (TRITONDL_SHA_MB=0), alternated x3; then the pack job and a profiled run.
set -o pipefail
OUT=${OUT:-gpurun_out/r03_bt_ab}
mkdir -p $OUT
export TMPDIR=/tmp
for rep in 1 2 3; do
  TRITONDL_SHA_MB=0 timeout -k 10 120 python -u tools/bench_bt.py --mb 2048 --seeds 4 > $OUT/ni$rep.jsonl 2>> $OUT/err.log &&
  TRITONDL_SHA_MB=1 timeout -k 10 120 python -u tools/bench_bt.py --mb 2048 --seeds 4 > $OUT/mb$rep.jsonl 2>> $OUT/err.log || exit $?
done
timeout -k 10 200 python -u tools/bench_bt.py --job --mb 1024 --files 8 --seeds 4 --repeat 2 --stream on > $OUT/job.jsonl 2>> $OUT/err.log &&
timeout -k 10 120 python -u tools/bench_bt.py --mb 2048 --seeds 4 --cpuprofile $OUT/bt.prof > $OUT/prof.jsonl 2>> $OUT/err.log
rc=$?
for f in $OUT/*.jsonl; do echo "$(basename $f) $(cut -c1-110 $f | tr '\n' ' ')"; done
head -12 $OUT/bt.prof.txt
exit $rc
