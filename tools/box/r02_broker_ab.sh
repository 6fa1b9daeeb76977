#!/bin/bash
# Broker/producer changes A/B (ab_old = before): 1 rank and 2/4 gloo ranks sharing one broker.
set -o pipefail
OUT=gpurun_out/r02_broker_ab
mkdir -p $OUT
export TMPDIR=/tmp
rc=0
port=29600
for rep in 1 2; do
  for v in old new; do
    if [ $v = old ]; then B=ab_old/bench.py; else B=bench.py; fi
    timeout -k 10 200 python $B --steps 300 --warmup 10 --no-gpu-probe > $OUT/${v}_n1_$rep.log 2>&1 || { rc=$?; break 2; }
    for n in 2 4; do
      port=$((port+1))
      timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node $n --master-addr 127.0.0.1 --master-port $port $B --gpus $n --steps 200 --warmup 5 --dist-backend gloo --no-gpu-probe > $OUT/${v}_n${n}_$rep.log 2>&1 || { rc=$?; break 3; }
    done
  done
done
for f in $OUT/*.log; do echo "$(basename $f) $(grep -o '"value": [0-9.]*' $f | head -1) $(grep -o '"cpu_ms_per_job[^}]*' $f) $(grep -o '"ack": [0-9.]*' $f)"; done
exit $rc
