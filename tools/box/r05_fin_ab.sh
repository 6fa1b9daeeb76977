#!/bin/bash
# Round 5: the signed PUT's final frame before joining the hashers and
# unmapping the file (this tree) vs after (.ab/prefin, its own native build).
# Alternated 300-job runs with the data-plane trace.
set -o pipefail
OUT=${OUT:-gpurun_out/r05_fin_ab}
mkdir -p $OUT
export TMPDIR=/tmp
R=$PWD
b() { local name=$1 dir=$2; shift 2; (cd $dir && TRITONDL_TRACE=1 timeout -k 10 200 python bench.py --steps 300 --warmup 10 \
      --no-gpu-probe --no-reference-mode "$@") > $OUT/$name.log 2>&1; }
for i in 1 2 3 4; do
  b fin_first_$i $R && b fin_after_$i $R/.ab/prefin || break
done
rc=$?
for f in $OUT/*.log; do
  echo "$(basename $f) $(grep -o '"value": [0-9.]*' $f | head -1) $(grep -o '"trace_p50_ms": {[^}]*}' $f | head -1 | grep -o '"get_pump_end": [0-9.]*, "put_sent": [0-9.]*, "put_pump_end": [0-9.]*')"
done
exit $rc
