#!/bin/bash
# Round 5, second pass: repeats of the knobs that moved (pipeline_commit), the multipart
# threshold on a 32 MiB job, and 8x8 streams without a per-stream cap (1 GiB).
set -o pipefail
OUT=${OUT:-gpurun_out/r05_rtt_ab2}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 500 python -u tools/rtt_ab.py --out $OUT/rep --rtts 0,2,20 --sets small \
    --only default,pipeline_commit,segments_1 --repeat 3 > $OUT/rep.txt 2>&1 &&
timeout -k 10 400 python -u tools/rtt_ab.py --out $OUT/mid --rtts 0,20 --sets mid,uncapped > $OUT/mid.txt 2>&1
rc=$?
tail -40 $OUT/rep/TABLE.md $OUT/mid/TABLE.md
exit $rc
