#!/bin/bash
# Round-2 box run: GPU tests (incl. production-path resume), staging probe,
# resume-job bench (cpu / gpu / hybrid / auto), rocprofv3 copy+kernel trace of
# the GPU resume path, torrent pack job bench (streamed uploads off/on).
set -o pipefail
OUT=gpurun_out/r02_resume
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 &&
timeout -k 10 400 python -u tools/staging_probe.py --gb 8 > $OUT/staging_probe.log 2>&1 &&
timeout -k 10 400 python -u tools/bench_resume.py --gb 8 --version 1 --device cpu gpu hybrid auto --reps 3 > $OUT/resume_v1.log 2>&1 &&
timeout -k 10 400 python -u tools/bench_resume.py --gb 8 --version 2 --device cpu gpu hybrid auto --reps 3 > $OUT/resume_v2.log 2>&1 &&
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --stats --output-format csv -d $OUT/trace_gpu -o run -- \
    python3 tools/bench_resume.py --gb 8 --version 1 --device gpu --reps 2 > $OUT/resume_trace_gpu.log 2>&1 &&
python tools/trace_overlap.py $OUT/trace_gpu > $OUT/overlap_gpu.json 2>&1 &&
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --stats --output-format csv -d $OUT/trace_hybrid -o run -- \
    python3 tools/bench_resume.py --gb 8 --version 1 --device hybrid --reps 2 > $OUT/resume_trace_hybrid.log 2>&1 &&
python tools/trace_overlap.py $OUT/trace_hybrid > $OUT/overlap_hybrid.json 2>&1 &&
timeout -k 10 300 python -u tools/bench_bt.py --job --mb 1024 --files 8 --seeds 4 --repeat 2 > $OUT/bt_job.log 2>&1
rc=$?
for f in $OUT/*.log $OUT/*.json; do echo "== $f"; grep -E '^\{|passed|failed|Error|error' $f | tail -12 | cut -c1-400; done
exit $rc
