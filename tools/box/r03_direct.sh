#!/bin/bash
# GPU resume with page-cache -> HBM direct DMA (registered file mappings) vs
# the pinned staging ring (TRITONDL_GPU_DIRECT=0): GPU tests first, then the
# 8 GiB v1 resume job, host / gpu / hybrid, alternated.
set -o pipefail
OUT=${OUT:-gpurun_out/r03_direct}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_hashing.py tests/test_bt.py -m gpu -x -v --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { tail -30 $OUT/pytest_gpu.log; exit 1; }
tail -2 $OUT/pytest_gpu.log
timeout -k 10 400 python -u tools/bench_resume.py --gb 8 --version 1 --device cpu gpu hybrid --reps 3 > $OUT/resume_direct.log 2>&1 &&
TRITONDL_GPU_DIRECT=0 timeout -k 10 400 python -u tools/bench_resume.py --gb 8 --version 1 --device gpu hybrid --reps 3 > $OUT/resume_staged.log 2>&1 &&
timeout -k 10 400 python -u tools/bench_resume.py --gb 8 --version 2 --device cpu gpu hybrid --reps 2 > $OUT/resume_v2_direct.log 2>&1
rc=$?
for f in $OUT/resume_*.log; do echo "== $(basename $f)"; grep warm $f | cut -c1-260; done
exit $rc
