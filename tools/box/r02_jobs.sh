#!/bin/bash
# Round-2 box run #3: torrent pack jobs with S3 as the slower link (per-file
# streamed uploads off/on), resume bench with verify_s, headline bench http +
# https, 8-worker pool.
set -o pipefail
OUT=gpurun_out/r02_jobs
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python -u tools/bench_bt.py --job --mb 1024 --files 8 --seeds 4 --repeat 2 --s3-gbps 8 > $OUT/bt_job_s3_8gbps.log 2>&1 &&
timeout -k 10 300 python -u tools/bench_bt.py --job --mb 1024 --files 8 --seeds 4 --repeat 2 --s3-gbps 4 > $OUT/bt_job_s3_4gbps.log 2>&1 &&
TRITONDL_GPU_TRACE=1 timeout -k 10 400 python -u tools/bench_resume.py --gb 8 --version 1 --device gpu hybrid auto --reps 4 > $OUT/resume_v1.log 2>&1 &&
timeout -k 10 300 python -u bench.py --steps 200 --warmup 10 > $OUT/bench_http.log 2>&1 &&
timeout -k 10 300 python -u bench.py --steps 200 --warmup 10 --tls --no-gpu-probe > $OUT/bench_https.log 2>&1 &&
timeout -k 10 300 python tools/bench_pool.py --workers 8 --jobs-per-worker 100 --file-kb 10240 --nodes 4 > $OUT/pool8_10m_nodes4.log 2>&1
rc=$?
for f in $OUT/*.log; do echo "== $f"; grep -E '^\{|passed|failed|Error|error' $f | tail -10 | cut -c1-700; done
exit $rc
