#!/bin/bash
# 16-lane SHA-1 on the box: probe, GPU tests (hybrid verifier changed), 8 GiB
# v1 resume (cpu/gpu/hybrid) and BT ingest with the kernel on vs off.
set -o pipefail
OUT=${OUT:-gpurun_out/r03_sha1_mb}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 120 python tools/cost_probe.py --reps 20 > $OUT/probe.jsonl 2>&1 &&
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 &&
TRITONDL_SHA_MB=1 timeout -k 10 400 python -u tools/bench_resume.py --gb 8 --version 1 --device cpu gpu hybrid --reps 2 > $OUT/resume_mb.log 2>&1 &&
TRITONDL_SHA_MB=0 timeout -k 10 400 python -u tools/bench_resume.py --gb 8 --version 1 --device cpu hybrid --reps 2 > $OUT/resume_ni.log 2>&1 &&
TRITONDL_SHA_MB=1 timeout -k 10 120 python -u tools/bench_bt.py --mb 2048 --seeds 4 > $OUT/bt_mb.jsonl 2>> $OUT/bt_err.log &&
TRITONDL_SHA_MB=0 timeout -k 10 120 python -u tools/bench_bt.py --mb 2048 --seeds 4 > $OUT/bt_ni.jsonl 2>> $OUT/bt_err.log &&
TRITONDL_SHA_MB=1 timeout -k 10 120 python -u tools/bench_bt.py --mb 2048 --seeds 4 > $OUT/bt_mb2.jsonl 2>> $OUT/bt_err.log &&
TRITONDL_SHA_MB=0 timeout -k 10 120 python -u tools/bench_bt.py --mb 2048 --seeds 4 > $OUT/bt_ni2.jsonl 2>> $OUT/bt_err.log
rc=$?
grep sha $OUT/probe.jsonl; tail -1 $OUT/pytest_gpu.log
for f in $OUT/resume_*.log; do echo "== $f"; grep warm $f | cut -c1-150; done
for f in $OUT/bt_*.jsonl; do echo "$(basename $f) $(cut -c1-120 $f)"; done
exit $rc
