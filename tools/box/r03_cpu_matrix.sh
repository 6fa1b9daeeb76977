#!/bin/bash
# Worker CPU per job by thread class across send-side hasher counts and
# download segment counts (headline, --cpuprofile), twice each, alternated;
# plus the cost probe (floors of each data-path primitive on this CPU).
set -o pipefail
OUT=${OUT:-gpurun_out/r03_cpu_matrix}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 120 python tools/cost_probe.py --dir /tmp --reps 30 > $OUT/probe.jsonl 2>&1 || exit $?
run() {  # name args...
  local name=$1; shift
  timeout -k 10 200 python bench.py --steps 300 --warmup 10 --no-gpu-probe --cpuprofile $OUT/$name.prof "$@" \
    > $OUT/head_$name.log 2>&1 || return $?
}
for rep in 1 2; do
  run st4_$rep && run st2_$rep --sign-threads 2 && run st1_$rep --sign-threads 1 && run seg1_$rep --http-segments 1 || exit $?
done
for f in $OUT/head_*.log; do
  n=$(basename $f .log); n=${n#head_}
  echo "$n $(grep -o '"value": [0-9.]*' $f | head -1) $(grep -o '"cpu_ms_per_job[^}]*' $f) $(grep -o '"job_latency_ms_p50": [0-9.]*' $f)"
  grep -A4 'cpu by thread class' $OUT/$n.prof.txt | tail -4
done
