#!/bin/bash
# Round 5: info-level logging with lines coalesced per loop iteration (this
# tree) vs one write + flush per line (the previous commit, ./.ab), and this
# tree at the bench's warning level.  Alternated 300-job runs, stderr to a file.
set -o pipefail
OUT=${OUT:-gpurun_out/r05_logbatch_ab}
mkdir -p $OUT
export TMPDIR=/tmp
ROOT=$PWD
b() { local name=$1 dir=$2; shift 2; (cd $dir && timeout -k 10 200 python bench.py --steps 300 --warmup 10 \
      --no-gpu-probe --no-reference-mode "$@" > $ROOT/$OUT/$name.log 2> $ROOT/$OUT/$name.err); }
for i in 1 2 3 4; do
  b info_new_$i . --log-level info &&
  b info_old_$i .ab --log-level info &&
  b warning_new_$i . || break
done
rc=$?
for f in $OUT/*.log; do
  echo "$(basename $f) $(grep -o '"value": [0-9.]*' $f | head -1) stderr_lines=$(wc -l < ${f%.log}.err)"
done
gzip -f $OUT/*.err
exit $rc
