#!/bin/bash
# Spare-file recycling for torrent jobs: 1 GiB 8-file pack job x4 per process
# (the first job of a recycling process has no spares yet) and 2 GiB ingest,
# recycle vs TRITONDL_RECYCLE_BYTES=0, alternated x2.
set -o pipefail
OUT=${OUT:-gpurun_out/r03_recycle_bt}
mkdir -p $OUT
export TMPDIR=/tmp
for rep in 1 2; do
  timeout -k 10 200 python -u tools/bench_bt.py --job --mb 1024 --files 8 --seeds 4 --repeat 4 --stream on > $OUT/job_recycle_$rep.jsonl 2>> $OUT/err.log &&
  TRITONDL_RECYCLE_BYTES=0 timeout -k 10 200 python -u tools/bench_bt.py --job --mb 1024 --files 8 --seeds 4 --repeat 4 --stream on > $OUT/job_delete_$rep.jsonl 2>> $OUT/err.log || exit $?
done
for f in $OUT/job_*.jsonl; do
  echo "$(basename $f .jsonl) $(grep -o '"value": [0-9.]*' $f | tr '\n' ' ')"
done
exit 0
