#!/bin/bash
# Round-3 GPU experiment: aws-chunked chunk SHA-256s on the HIP kernel
# (TRITONDL_S3_HASH_DEVICE=gpu) vs SHA-NI, alternated in one session:
# headline (1 worker) and the 8-worker pool; then a rocprofv3 kernel trace
# of the GPU-hashing headline.
set -o pipefail
OUT=${OUT:-gpurun_out/r03_gpu_sha_ab}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || exit $?
for rep in 1 2; do
  timeout -k 10 200 python bench.py --steps 300 --warmup 10 --no-gpu-probe --s3-hash-device cpu > $OUT/head_cpu$rep.log 2>&1 &&
  timeout -k 10 200 python bench.py --steps 300 --warmup 10 --no-gpu-probe --s3-hash-device gpu > $OUT/head_gpu$rep.log 2>&1 &&
  timeout -k 10 300 python tools/bench_pool.py --workers 8 --jobs-per-worker 100 --file-kb 10240 --nodes 4 --s3-hash-device cpu > $OUT/pool_cpu$rep.log 2>&1 &&
  timeout -k 10 300 python tools/bench_pool.py --workers 8 --jobs-per-worker 100 --file-kb 10240 --nodes 4 --s3-hash-device gpu > $OUT/pool_gpu$rep.log 2>&1 || exit $?
done
timeout -k 10 200 python bench.py --steps 200 --warmup 10 --no-gpu-probe --s3-hash-device gpu --cpuprofile $OUT/gpu.prof > $OUT/head_gpu_prof.log 2>&1 &&
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$OUT/rocprof -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 100 --warmup 5 --no-gpu-probe --s3-hash-device gpu > $GRAFT_REPO_ROOT/$OUT/rocprof.log 2>&1
rc=$?
cd $GRAFT_REPO_ROOT
tail -2 $OUT/pytest_gpu.log
for f in $OUT/head_*.log $OUT/pool_*.log; do echo "$(basename $f) $(grep -o '"value": [0-9.]*' $f | head -1) $(grep -o '"cpu_ms_per_job[^}]*' $f) $(grep -o '"job_latency_ms_p50": [0-9.]*' $f)"; done
head -8 $OUT/gpu.prof.txt
find $OUT/rocprof -name "*stats*" | head
exit $rc
