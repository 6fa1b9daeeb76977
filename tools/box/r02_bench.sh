#!/bin/bash
# Round-2 box run: GPU tests, headline bench (http / https), node-scale pool bench.
set -o pipefail
OUT=gpurun_out/r02_bench
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 &&
timeout -k 10 200 python bench.py --steps 200 --warmup 10 > $OUT/bench_http.log 2>&1 &&
timeout -k 10 200 python bench.py --steps 200 --warmup 10 --tls --no-gpu-probe > $OUT/bench_https.log 2>&1 &&
timeout -k 10 200 python bench.py --steps 200 --warmup 10 --tls --payload streaming --no-gpu-probe > $OUT/bench_https_chunked.log 2>&1 &&
timeout -k 10 300 python tools/bench_pool.py --workers 8 --jobs-per-worker 100 --file-kb 10240 --nodes 1 > $OUT/pool8_10m_nodes1.log 2>&1 &&
timeout -k 10 300 python tools/bench_pool.py --workers 8 --jobs-per-worker 100 --file-kb 10240 --nodes 4 > $OUT/pool8_10m_nodes4.log 2>&1 &&
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 4 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 4 --steps 100 --warmup 5 --dist-backend gloo --no-gpu-probe > $OUT/bench_shared_gloo4.log 2>&1
rc=$?
for f in $OUT/*.log; do echo "== $f"; grep -E '^\{|passed|failed|Error' $f | tail -3 | cut -c1-700; done
exit $rc
