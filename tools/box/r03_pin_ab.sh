#!/bin/bash
# Headline with the bench pinned to compact L3-domain CPU sets vs unpinned,
# alternated in one session; records the box's cache topology and quota.
set -o pipefail
OUT=${OUT:-gpurun_out/r03_pin_ab}
mkdir -p $OUT
export TMPDIR=/tmp
{ nproc; cat /sys/fs/cgroup/cpu.max; lscpu | grep -E "Model name|Socket|Core|Thread|NUMA|L3"; 
  for c in 0 1 8 16; do echo "cpu$c L3: $(cat /sys/devices/system/cpu/cpu$c/cache/index3/shared_cpu_list)"; done
  python -c "from tritondl.parallel import topology as t; d=t.l3_domains(); print(len(d), [d[i] for i in range(min(3,len(d)))])"; } > $OUT/topo.txt 2>&1
rc=0
for rep in 1 2; do
  for v in none auto auto:8 auto:32; do
    if [ $v = none ]; then args=""; else args="--cpus $v"; fi
    timeout -k 10 200 python bench.py --steps 300 --warmup 10 --no-gpu-probe $args > $OUT/bench_${v/:/_}_$rep.log 2>&1 || { rc=$?; break 2; }
  done
done
cat $OUT/topo.txt
for f in $OUT/bench_*.log; do
  echo "$(basename $f) $(grep -o '"value": [0-9.]*' $f | tr '\n' ' ') $(grep -o '"cpus": "[^"]*"' $f) $(grep -o '"cpu_ms_per_job[^}]*' $f) $(grep -o '"job_latency_ms_p50": [0-9.]*' $f)"
done
exit $rc
