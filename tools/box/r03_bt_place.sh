#!/bin/bash
# BitTorrent ingest (2 GiB, 4 seeders) and the 1 GiB 8-file pack job:
# unpinned vs leecher on two CCDs with the seeders on two others, alternated.
set -o pipefail
OUT=${OUT:-gpurun_out/r03_bt_place}
mkdir -p $OUT
export TMPDIR=/tmp
rc=0
for rep in 1 2; do
  for v in none pinned; do
    case $v in none) args="";; pinned) args="--cpus 0-15,128-143 --fake-cpus 16-31,144-159";; esac
    timeout -k 10 120 python -u tools/bench_bt.py --mb 2048 --seeds 4 $args > $OUT/ingest_${v}_$rep.jsonl 2>> $OUT/err.log || { rc=$?; break 2; }
    timeout -k 10 200 python -u tools/bench_bt.py --job --mb 1024 --files 8 --seeds 4 --repeat 2 --stream on $args > $OUT/job_${v}_$rep.jsonl 2>> $OUT/err.log || { rc=$?; break 2; }
  done
done
for f in $OUT/*.jsonl; do echo "$(basename $f) $(grep -o '"value": [0-9.]*' $f | tr '\n' ' ')"; done
exit $rc
