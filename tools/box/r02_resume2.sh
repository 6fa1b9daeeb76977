#!/bin/bash
# Resume verification after the SHA-NI pair paths: v1 and v2, host / GPU / hybrid.
set -o pipefail
OUT=gpurun_out/r02_resume2
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 400 python -u tools/bench_resume.py --gb 8 --version 1 --device cpu gpu hybrid auto --reps 2 > $OUT/resume_v1.log 2>&1 &&
timeout -k 10 400 python -u tools/bench_resume.py --gb 8 --version 2 --device cpu gpu hybrid auto --reps 2 > $OUT/resume_v2.log 2>&1
rc=$?
for f in $OUT/*.log; do echo "== $f"; grep -E '^\{' $f | grep warm | cut -c1-260; done
exit $rc
