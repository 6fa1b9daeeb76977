#!/bin/bash
# Round 5, end of session: the driver's exact N=1 command, six times in a row on one box.
set -o pipefail
OUT=${OUT:-gpurun_out/r05_driver_series}
mkdir -p $OUT
export TMPDIR=/tmp
for i in 1 2 3 4 5 6; do
  timeout -k 10 200 python bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/run_$i.log 2>&1 || break
done
rc=$?
for f in $OUT/*.log; do
  echo "$(basename $f) $(grep -o '"value": [0-9.]*' $f | head -1) $(grep -o '"cpus": "[^"]*"' $f | head -1)"
done
exit $rc
