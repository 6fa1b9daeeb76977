#!/bin/bash
# Native serving A/B: native leecher against native vs Python seeders, plus the pack job.
set -o pipefail
OUT=gpurun_out/r02_btserve
mkdir -p $OUT
export TMPDIR=/tmp
rc=0
for rep in 1 2; do
  for v in "" "--python-seeders" "--python-wire --python-seeders"; do
    for s in 4 8; do
      timeout -k 10 120 python -u tools/bench_bt.py --mb 2048 --seeds $s $v >> $OUT/ingest.jsonl 2>> $OUT/err.log || { rc=$?; break 3; }
    done
  done
done
[ $rc -eq 0 ] && timeout -k 10 200 python -u tools/bench_bt.py --job --mb 1024 --files 8 --seeds 4 --repeat 3 --stream on >> $OUT/job.jsonl 2>> $OUT/err.log || rc=$?
[ $rc -eq 0 ] && timeout -k 10 120 python -u tools/bench_bt.py --mb 2048 --seeds 4 --profile $OUT/leecher.prof >> $OUT/profiled.jsonl 2>> $OUT/err.log && python -c "
import pstats; pstats.Stats('$OUT/leecher.prof').sort_stats('tottime').print_stats(20)" > $OUT/leecher_top.txt || rc=$?
grep -h '^{' $OUT/*.jsonl | cut -c1-250
tail -3 $OUT/err.log
exit $rc
