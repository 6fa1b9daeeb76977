#!/bin/bash
# Round 5: worker defaults under emulated RTT (0 / 2 / 20 ms) on one MI355X box's CPUs.
set -o pipefail
OUT=${OUT:-gpurun_out/r05_rtt_ab}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 1100 python -u tools/rtt_ab.py --out $OUT --rtts ${RTTS:-0,2,20} > $OUT/log.txt 2>&1
rc=$?
tail -50 $OUT/log.txt
exit $rc
