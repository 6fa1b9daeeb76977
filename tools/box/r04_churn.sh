#!/bin/bash
# GPU helper churn: 120 start -> verify 256 MiB -> idle-exit cycles (tools/gpu_churn.py).
set -o pipefail
OUT=${OUT:-gpurun_out/r04_churn}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 900 python3 -u tools/gpu_churn.py --cycles ${CYCLES:-120} --mb 256 --out $OUT/churn.jsonl \
    > $OUT/churn.log 2>&1
rc=$?
tail -1 $OUT/churn.log
exit $rc
