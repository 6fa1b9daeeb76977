#!/bin/bash
# Round 5: is the r05 tree slower than r04's on the headline?  The same box, 300-job runs,
# alternated: r04 tree (.ab/r04, its own native build) vs this tree (defaults, i.e. pipeline on)
# vs this tree with pipeline_commit off.  Then the RCCL 1-rank path through torchrun.
set -o pipefail
OUT=${OUT:-gpurun_out/r05_regress}
mkdir -p $OUT
export TMPDIR=/tmp
R=$PWD
b() { local name=$1 dir=$2; shift 2; (cd $dir && timeout -k 10 200 python bench.py --steps 300 --warmup 10 --no-gpu-probe "$@") > $OUT/$name.log 2>&1; }
for i in 1 2 3; do
  b r04_$i $R/.ab/r04 --no-reference-mode &&
  b r05_$i $R --no-reference-mode &&
  b r05_nopipe_$i $R --no-reference-mode --pipeline-commit off || break
done
rc=$?
[ $rc = 0 ] && timeout -k 10 200 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 \
    --master-port 29541 bench.py --gpus 1 --steps 100 --warmup 5 --dist-always --no-gpu-probe > $OUT/rccl_1rank.log 2>&1
rc=$?
for f in $OUT/*.log; do echo "$(basename $f) $(grep -o '"value": [0-9.]*' $f | head -1) $(grep -o '"job_latency_ms_p50": [0-9.]*' $f | head -1) $(grep -o '"collectives": "[^"]*"' $f | head -1)"; done
exit $rc
