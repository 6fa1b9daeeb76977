#!/bin/bash
# Native peer-wire data plane (csrc/btwire) vs the pure-Python wire: raw
# swarm ingest and the full torrent pack job, alternating A/B on one box.
set -o pipefail
OUT=gpurun_out/r02_btwire
mkdir -p $OUT
export TMPDIR=/tmp
rc=0
for rep in 1 2; do
  for w in "" "--python-wire"; do
    for s in 4 8; do
      timeout -k 10 120 python -u tools/bench_bt.py --mb 2048 --seeds $s $w >> $OUT/ingest.jsonl 2>> $OUT/err.log || { rc=$?; break 3; }
    done
  done
done
[ $rc -eq 0 ] && for w in "" "--python-wire"; do
  timeout -k 10 200 python -u tools/bench_bt.py --job --mb 1024 --files 8 --seeds 4 --repeat 2 --stream on $w >> $OUT/job.jsonl 2>> $OUT/err.log || { rc=$?; break; }
done
[ $rc -eq 0 ] && timeout -k 10 120 python -u tools/bench_bt.py --mb 2048 --seeds 4 --profile $OUT/leecher.prof >> $OUT/profiled.jsonl 2>> $OUT/err.log && python -c "
import pstats; pstats.Stats('$OUT/leecher.prof').sort_stats('tottime').print_stats(20)" > $OUT/leecher_top.txt || rc=$?
grep -h '^{' $OUT/*.jsonl | cut -c1-160
tail -5 $OUT/err.log
exit $rc
