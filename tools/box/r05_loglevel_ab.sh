#!/bin/bash
# Round 5: the bench's worker logs at warning; the reference (logrus) logs six
# info lines per job.  What does info-level logging cost the headline?
# Alternated 300-job runs; stderr (the log) to a file as a deployment would.
set -o pipefail
OUT=${OUT:-gpurun_out/r05_loglevel_ab}
mkdir -p $OUT
export TMPDIR=/tmp
b() { local name=$1; shift; timeout -k 10 200 python bench.py --steps 300 --warmup 10 --no-gpu-probe \
      --no-reference-mode "$@" > $OUT/$name.log 2> $OUT/$name.err; }
for i in ${RUNS:-1 2 3}; do
  b info_$i --log-level info &&
  b warning_$i || break
done
rc=$?
for f in $OUT/*.log; do
  echo "$(basename $f) $(grep -o '"value": [0-9.]*' $f | head -1) stderr_lines=$(wc -l < ${f%.log}.err)"
done
gzip -f $OUT/*.err
exit $rc
