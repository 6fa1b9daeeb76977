#!/bin/bash
# Round 5: the reaper removes a streamed job's dir by its one known file
# (offer + rmdir) instead of os.walk + rmtree, which ran Python on the reaper
# thread, contending for the GIL while the loop starts the next job.  This tree
# vs the previous commit (./.ab), alternated 300-job traced runs.
set -o pipefail
OUT=${OUT:-gpurun_out/r05_reap_ab}
mkdir -p $OUT
export TMPDIR=/tmp
ROOT=$PWD
b() { local name=$1 dir=$2; (cd $dir && TRITONDL_TRACE=1 timeout -k 10 200 python bench.py --steps 300 --warmup 10 \
      --no-gpu-probe --no-reference-mode > $ROOT/$OUT/$name.log 2>&1); }
for i in 1 2 3 4; do
  b new_$i . &&
  b old_$i .ab || break
done
rc=$?
for f in $OUT/*.log; do
  echo "$(basename $f) $(grep -o '"value": [0-9.]*' $f | head -1) $(grep -o '"trace_p50_ms": {[^}]*}' $f | head -1)"
done
exit $rc
