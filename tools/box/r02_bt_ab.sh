#!/bin/bash
# A/B of the BitTorrent leecher: previous commit (ab_old/) vs working tree, alternated.
set -o pipefail
OUT=gpurun_out/r02_bt_ab
mkdir -p $OUT
export TMPDIR=/tmp
rc=0
for rep in 1 2 3; do
  for v in old new; do
    if [ $v = old ]; then B=ab_old/tools/bench_bt.py; else B=tools/bench_bt.py; fi
    timeout -k 10 120 python -u $B --mb 2048 --seeds 4 | sed "s/^{/{\"variant\": \"$v\", /" >> $OUT/ingest.jsonl 2>> $OUT/err.log || { rc=$?; break 2; }
  done
done
cut -c1-140 $OUT/ingest.jsonl
exit $rc
