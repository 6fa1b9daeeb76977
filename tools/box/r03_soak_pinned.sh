#!/bin/bash
# Resource-leak soak at the final tree with the worker pinned to one CCD and
# the fakes on the next: 3,000 headline jobs + 60 magnet jobs + failing jobs
# (dead-lettered), sampled every 500.
set -o pipefail
OUT=${OUT:-gpurun_out/r03_soak_pinned}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -m tritondl.soak --jobs 3000 --torrent-jobs 60 --fail-every 50 --sample-every 500 \
    --warmup 500 --cpus auto --out $OUT/soak.jsonl > $OUT/soak.log 2>&1
rc=$?
tail -2 $OUT/soak.jsonl | cut -c1-900
exit $rc
