#!/bin/bash
# Round 5: pre-map the signed PUT's file mapping (MADV_POPULATE_READ) vs a
# minor fault per page in the hashers and the sender.  Alternated 300-job runs.
set -o pipefail
OUT=${OUT:-gpurun_out/r05_populate_ab}
mkdir -p $OUT
export TMPDIR=/tmp
uname -r > $OUT/kernel.txt
b() { local name=$1; shift; TRITONDL_TRACE=1 timeout -k 10 200 python bench.py --steps 300 --warmup 10 --no-gpu-probe \
      --no-reference-mode "$@" > $OUT/$name.log 2>&1; }
for i in 1 2 3 4; do
  b fault_$i && TRITONDL_ZC_POPULATE=1 b populate_$i || break
done
rc=$?
cat $OUT/kernel.txt
for f in $OUT/*.log; do
  echo "$(basename $f) $(grep -o '"value": [0-9.]*' $f | head -1) $(grep -o '"pgfault_per_job": [0-9.]*' $f | head -1) $(grep -o '"trace_p50_ms": {[^}]*}' $f | head -1 | grep -o '"get_pump_end": [0-9.]*, "put_sent": [0-9.]*')"
done
exit $rc
