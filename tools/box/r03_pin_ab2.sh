#!/bin/bash
# Pinning confirmation: bench default (--cpus auto: one CCD per rank) vs
# --cpus none vs fakes on their own CCD (--fake-cpus auto) alternated x3, the driver's 20-step form, and 2/4/8-rank
# shared-broker runs pinned (gloo).
set -o pipefail
OUT=${OUT:-gpurun_out/r03_pin_ab2}
mkdir -p $OUT
export TMPDIR=/tmp
rc=0
for rep in 1 2 3; do
  for v in auto none fakeapart; do
    if [ $v = fakeapart ]; then args="--cpus auto --fake-cpus auto"; else args="--cpus $v"; fi
    timeout -k 10 200 python bench.py --steps 300 --warmup 10 --no-gpu-probe $args > $OUT/bench_${v}_$rep.log 2>&1 || { rc=$?; break 2; }
  done
done
[ $rc = 0 ] && timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-gpu-probe > $OUT/bench_driver20.log 2>&1 || rc=$?
p=29700
for n in 2 4 8; do
  [ $rc = 0 ] || break
  p=$((p+1))
  timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node $n --master-addr 127.0.0.1 --master-port $p bench.py --gpus $n --steps 200 --warmup 5 --dist-backend gloo --no-gpu-probe > $OUT/shared_gloo$n.log 2>&1 || rc=$?
done
for f in $OUT/bench_*.log $OUT/shared_gloo*.log; do
  echo "$(basename $f) $(grep -o '"value": [0-9.]*' $f | tr '\n' ' ') $(grep -o '"cpus": "[^"]*"' $f) $(grep -o "\"fake_cpus\": \"[^\"]*\"" $f) $(grep -o '"cpu_ms_per_job[^}]*' $f) $(grep -o '"job_latency_ms_p50": [0-9.]*' $f) $(grep -o '"jobs_per_rank": [^]]*' $f)"
done
exit $rc
