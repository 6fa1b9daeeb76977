#!/bin/bash
# Round-3 harness check: 1/2/4/8 ranks on one shared broker (gloo, CPU
# workers on this box's 16-CPU share) with the producer off rank 0's loop,
# plus two single-rank headlines.
set -o pipefail
OUT=${OUT:-gpurun_out/r03_scale}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 200 python bench.py --steps 300 --warmup 10 > $OUT/bench_1.log 2>&1 &&
for n in 2 4 8; do
  timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node $n --master-addr 127.0.0.1 --master-port $((29660+n)) bench.py --gpus $n --steps 150 --warmup 5 --dist-backend gloo --no-gpu-probe > $OUT/shared_gloo$n.log 2>&1 || exit $?
done &&
timeout -k 10 200 python bench.py --steps 300 --warmup 10 --no-gpu-probe > $OUT/bench_1b.log 2>&1
rc=$?
for f in $OUT/bench_1.log $OUT/shared_gloo*.log $OUT/bench_1b.log; do echo "$(basename $f) $(grep -o '"value": [0-9.]*' $f | head -1) $(grep -o '"jobs_per_rank": [^]]*]' $f) $(grep -o '"cpu_ms_per_job[^}]*' $f) $(grep -o '"broker_core_share": [0-9.a-z]*' $f) $(grep -o '"gpu_sha1[^,]*' $f | tr '\n' ' ')"; done
exit $rc
