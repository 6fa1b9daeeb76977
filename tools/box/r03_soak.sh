#!/bin/bash
# Round-3 resource-leak soak: one worker, 5,000 headline jobs (10 MiB) + 100
# magnet jobs (8 MiB, out-of-process seeder) + 100 failing jobs (404 ->
# 2 retries through the delay queues -> dead letter), sampled every 500 jobs.
# Then the headline twice and the 8-worker pool once on the same tree.
set -o pipefail
OUT=${OUT:-gpurun_out/r03_soak}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -m tritondl.soak --jobs 5000 --torrent-jobs 100 --fail-every 50 --sample-every 500 \
    --warmup 500 --out $OUT/soak.jsonl > $OUT/soak.log 2>&1 &&
timeout -k 10 200 python bench.py --steps 300 --warmup 10 --no-gpu-probe > $OUT/head_a.log 2>&1 &&
timeout -k 10 300 python tools/bench_pool.py --workers 8 --jobs-per-worker 100 --file-kb 10240 --nodes 4 > $OUT/pool.log 2>&1 &&
timeout -k 10 200 python bench.py --steps 300 --warmup 10 > $OUT/head_b.log 2>&1
rc=$?
tail -3 $OUT/soak.jsonl
for f in $OUT/head_*.log $OUT/pool.log; do echo "$(basename $f) $(grep -o '"value": [0-9.]*' $f | head -1) $(grep -o '"cpu_ms_per_job[^}]*' $f)"; done
exit $rc
