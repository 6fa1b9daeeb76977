#!/bin/bash
# Idle-first placement: host load per CCD at the start, the driver's 1-GPU
# form twice, 300-step headline twice, 2/4/8 ranks on one shared broker.
set -o pipefail
OUT=${OUT:-gpurun_out/r03_scale3}
mkdir -p $OUT
export TMPDIR=/tmp
python -c "
from tritondl.parallel import topology as t
d = t.l3_domains(); b = t.domain_busy(d, 1.0)
print('busy per L3 domain (1 s):', [round(x, 2) for x in b])" > $OUT/host_load.txt 2>&1
rc=0
for f in driver20_a driver20_b; do
  timeout -k 10 200 python bench.py --steps 20 --warmup 5 > $OUT/bench_$f.log 2>&1 || { rc=$?; break; }
done
for f in s300_a s300_b; do
  [ $rc = 0 ] || break
  timeout -k 10 200 python bench.py --steps 300 --warmup 10 --no-gpu-probe > $OUT/bench_$f.log 2>&1 || rc=$?
done
p=29900
for n in 2 4 8; do
  [ $rc = 0 ] || break
  p=$((p+1))
  timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node $n --master-addr 127.0.0.1 --master-port $p bench.py --gpus $n --steps 200 --warmup 5 --dist-backend gloo --no-gpu-probe > $OUT/shared_gloo$n.log 2>&1 || rc=$?
done
python -c "
from tritondl.parallel import topology as t
d = t.l3_domains(); b = t.domain_busy(d, 1.0)
print('busy per L3 domain at the end (1 s):', [round(x, 2) for x in b])" >> $OUT/host_load.txt 2>&1
cat $OUT/host_load.txt
for f in $OUT/bench_*.log $OUT/shared_gloo*.log; do
  echo "$(basename $f) $(grep -o '"value": [0-9.]*' $f | tr '\n' ' ') $(grep -o '"cpus": "[^"]*"' $f) $(grep -o '"cpus_busy_before": "[^"]*"' $f) $(grep -o '"cpu_ms_per_job[^}]*' $f) $(grep -o '"jobs_per_rank": [^]]*' $f)"
done
exit $rc
