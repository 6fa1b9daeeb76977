#!/bin/bash
# Round-2 box run #2: reader-pool staging ring.  GPU tests, staging probe,
# traced resume bench (GPU event timeline: H2D vs kernel overlap), rocprofv3
# kernel stats, torrent pack job bench; rocprofv3 copy trace last.
set -o pipefail
OUT=gpurun_out/r02_staging
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 &&
timeout -k 10 400 python -u tools/staging_probe.py --gb 8 > $OUT/staging_probe.log 2>&1 &&
TRITONDL_GPU_TRACE=1 timeout -k 10 400 python -u tools/bench_resume.py --gb 8 --version 1 --device cpu gpu hybrid auto --reps 3 > $OUT/resume_v1.log 2>&1 &&
TRITONDL_GPU_TRACE=1 timeout -k 10 400 python -u tools/bench_resume.py --gb 8 --version 2 --device cpu gpu hybrid auto --reps 3 > $OUT/resume_v2.log 2>&1 &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/kstats -o run -- \
    python3 tools/bench_resume.py --gb 8 --version 1 --device gpu hybrid --reps 2 > $OUT/resume_kstats.log 2>&1 &&
timeout -k 10 300 python -u tools/bench_bt.py --job --mb 1024 --files 8 --seeds 4 --repeat 2 > $OUT/bt_job.log 2>&1
rc=$?
for f in $OUT/*.log; do echo "== $f"; grep -E '^\{|passed|failed|Error|error' $f | tail -14 | cut -c1-600; done
exit $rc
