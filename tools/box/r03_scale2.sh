#!/bin/bash
# Shared-broker rehearsal with ranks and their fakes paired on adjacent L3
# domains (gloo, on the box's 16-CPU quota), the driver's 1-GPU form twice,
# and where the GPU sits (NUMA node / local CPUs).
set -o pipefail
OUT=${OUT:-gpurun_out/r03_scale2}
mkdir -p $OUT
export TMPDIR=/tmp
for d in /sys/class/drm/card*/device; do echo "$d numa=$(cat $d/numa_node 2>/dev/null) cpus=$(cat $d/local_cpulist 2>/dev/null)"; done > $OUT/gpu_numa.txt 2>&1
rc=0
timeout -k 10 200 python bench.py --steps 20 --warmup 5 > $OUT/bench_driver20_a.log 2>&1 || rc=$?
[ $rc = 0 ] && { timeout -k 10 200 python bench.py --steps 20 --warmup 5 > $OUT/bench_driver20_b.log 2>&1 || rc=$?; }
p=29800
for n in 2 4 8; do
  [ $rc = 0 ] || break
  p=$((p+1))
  timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node $n --master-addr 127.0.0.1 --master-port $p bench.py --gpus $n --steps 200 --warmup 5 --dist-backend gloo --no-gpu-probe > $OUT/shared_gloo$n.log 2>&1 || rc=$?
done
cat $OUT/gpu_numa.txt
for f in $OUT/bench_*.log $OUT/shared_gloo*.log; do
  echo "$(basename $f) $(grep -o '"value": [0-9.]*' $f | tr '\n' ' ') $(grep -o '"cpus": "[^"]*"' $f) $(grep -o '"fake_cpus": "[^"]*"' $f | cut -c1-40) $(grep -o '"cpu_ms_per_job[^}]*' $f) $(grep -o '"jobs_per_rank": [^]]*' $f)"
done
exit $rc
