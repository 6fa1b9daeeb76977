#!/bin/bash
# Round 5: BASELINE.md's other configs on the round-5 tree (the headline has its own runs):
# a 1 GiB http job, 8 workers x 100 x 1 MiB jobs, a 2 GiB magnet job from 4 seeders,
# the same over uTP only, and an 8 GiB redelivered torrent re-verified host / hybrid.
set -o pipefail
OUT=${OUT:-gpurun_out/r05_configs}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 240 python bench.py --file-mb 1024 --steps 6 --warmup 1 --no-gpu-probe --no-reference-mode \
    > $OUT/gib.log 2>&1 &&
timeout -k 10 240 python tools/bench_pool.py --workers 8 --jobs-per-worker 100 --file-kb 1024 > $OUT/pool.log 2>&1 &&
timeout -k 10 240 python tools/bench_bt.py --mb 2048 > $OUT/bt.log 2>&1 &&
timeout -k 10 240 python tools/bench_bt.py --mb 1024 --utp > $OUT/bt_utp.log 2>&1 &&
timeout -k 10 300 python tools/bench_resume.py --gb 8 --version 1 --device cpu hybrid > $OUT/resume.log 2>&1
rc=$?
for f in $OUT/*.log; do echo "== $(basename $f)"; tail -4 $f | cut -c1-400; done
exit $rc
