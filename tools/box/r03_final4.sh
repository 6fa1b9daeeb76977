#!/bin/bash
# Round-3 closing measurements at the current tree (bench pinned per rank by default): GPU tests, smoke, the
# driver's default bench, headline x3, https, 1 GiB job, 8-worker pool,
# 2/4/8-rank shared broker (gloo), BT ingest + pack job, 8 GiB resume.
set -o pipefail
OUT=${OUT:-gpurun_out/r03_final4}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 &&
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.build(); g.smoke()" > $OUT/smoke.log 2>&1 &&
timeout -k 10 200 python bench.py > $OUT/bench_default.log 2>&1 &&
timeout -k 10 200 python bench.py --steps 300 --warmup 10 > $OUT/bench_a.log 2>&1 &&
timeout -k 10 200 python bench.py --steps 300 --warmup 10 --no-gpu-probe > $OUT/bench_b.log 2>&1 &&
timeout -k 10 200 python bench.py --steps 300 --warmup 10 --no-gpu-probe > $OUT/bench_c.log 2>&1 &&
timeout -k 10 200 python bench.py --steps 300 --warmup 10 --tls --no-gpu-probe > $OUT/bench_https.log 2>&1 &&
timeout -k 10 200 python bench.py --steps 12 --warmup 2 --file-mb 1024 --no-gpu-probe > $OUT/bench_1g.log 2>&1 &&
timeout -k 10 300 python tools/bench_pool.py --workers 8 --jobs-per-worker 100 --file-kb 10240 --nodes 4 > $OUT/pool8_10m.log 2>&1 &&
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29761 bench.py --gpus 2 --steps 200 --warmup 5 --dist-backend gloo --no-gpu-probe > $OUT/shared_gloo2.log 2>&1 &&
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 4 --master-addr 127.0.0.1 --master-port 29762 bench.py --gpus 4 --steps 200 --warmup 5 --dist-backend gloo --no-gpu-probe > $OUT/shared_gloo4.log 2>&1 &&
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 8 --master-addr 127.0.0.1 --master-port 29763 bench.py --gpus 8 --steps 200 --warmup 5 --dist-backend gloo --no-gpu-probe > $OUT/shared_gloo8.log 2>&1 &&
timeout -k 10 120 python -u tools/bench_bt.py --mb 2048 --seeds 4 > $OUT/bt_ingest.jsonl 2>> $OUT/bt_err.log &&
timeout -k 10 200 python -u tools/bench_bt.py --job --mb 1024 --files 8 --seeds 4 --repeat 2 --stream on > $OUT/bt_job.jsonl 2>> $OUT/bt_err.log &&
timeout -k 10 400 python -u tools/bench_resume.py --gb 8 --version 1 --device cpu gpu hybrid --reps 2 > $OUT/resume_v1.log 2>&1
rc=$?
tail -2 $OUT/pytest_gpu.log; tail -1 $OUT/smoke.log
for f in $OUT/bench_*.log $OUT/pool8_10m.log $OUT/shared_gloo*.log; do
  echo "$(basename $f) $(grep -o '"value": [0-9.]*' $f | tr '\n' ' ') $(grep -o '"cpu_ms_per_job[^}]*' $f) $(grep -o '"ingest_MB_per_sec": [0-9.]*' $f)"
done
cut -c1-160 $OUT/bt_ingest.jsonl $OUT/bt_job.jsonl; grep warm $OUT/resume_v1.log | cut -c1-200
exit $rc
