#!/bin/bash
# Round 5: on loopback, with the faster round-5 data path, does pipelining the
# commit always (min 0 ms) beat the adaptive default (pipelines only while the
# confirm round trip is >= 0.3 ms, i.e. not on loopback)?  Alternated 300-job runs.
set -o pipefail
OUT=${OUT:-gpurun_out/r05_pipe_ab}
mkdir -p $OUT
export TMPDIR=/tmp
b() { local name=$1; shift; timeout -k 10 200 python bench.py --steps 300 --warmup 10 --no-gpu-probe \
      --no-reference-mode "$@" > $OUT/$name.log 2>&1; }
for i in 1 2 3 4; do
  b adaptive_$i && b always_$i --pipeline-min-ms 0 || break
done
rc=$?
for f in $OUT/*.log; do
  echo "$(basename $f) $(grep -o '"value": [0-9.]*' $f | head -1) $(grep -o '"job_spans_ms_p50": {[^}]*}' $f | head -1)"
done
exit $rc
