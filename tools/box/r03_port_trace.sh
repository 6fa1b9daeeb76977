#!/bin/bash
# Job timeline (TRITONDL_TRACE=1 data-plane events) with pumps on executor
# threads vs the native pool + completion port; alternated.
set -o pipefail
OUT=${OUT:-gpurun_out/r03_port_trace}
mkdir -p $OUT
export TMPDIR=/tmp TRITONDL_TRACE=1
bd() {  # name env...
  local name=$1; shift
  env "$@" timeout -k 10 200 python tools/bench_breakdown.py --reps 80 > $OUT/bd_$name.log 2>&1 || return $?
}
for rep in 1 2; do
  bd exec$rep TRITONDL_RELAY_PORT=0 && bd port$rep TRITONDL_RELAY_PORT=1 || exit $?
done
for f in $OUT/bd_*.log; do
  echo "== $f"
  python3 -c "
import json,sys
for l in open('$f'):
    if l.startswith('{'):
        d=json.loads(l)
        print({k:v['ms_p50'] for k,v in d.items() if isinstance(v,dict) and 'ms_p50' in v})
        print('job', d['job'])
"
done
