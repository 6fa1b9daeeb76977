#!/usr/bin/env bash
# Round-6 closing check on an MI355X box, in three parts (each fits one gpurun call).
#   bash tools/final_check.sh OUTDIR core     GPU tests + smoke, the driver's bench command x3,
#                                             2 / 20 ms RTT with the default, every job leased at 0 / 20 ms
#   bash tools/final_check.sh OUTDIR configs  BASELINE's other configs (1 GiB job, 8-worker pool,
#                                             2 GiB magnet, uTP, 8 GiB hybrid resume) + the RCCL one-rank path
#   bash tools/final_check.sh OUTDIR scale    1 / 2 / 4 ranks on one shared broker (gloo; the box's CPU
#                                             share is shared by every rank; the 8-rank run is the driver's)
set -o pipefail
out=${1:-gpurun_out/r06_final}
part=${2:-core}
mkdir -p "$out"
export TMPDIR=/tmp
step() { local name=$1 lim=$2; shift 2; echo "[$(date +%T)] $name"; timeout -k 10 "$lim" "$@" > "$out/$name.log" 2>&1; local rc=$?; echo "[$(date +%T)] $name rc=$rc"; return $rc; }
b() { step "$1" 300 python bench.py --no-gpu-probe --no-reference-mode "${@:2}"; }
if [ "$part" = core ]; then
  step pytest_gpu 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread || exit 1
  step smoke 300 python -c "import __graft_entry__ as g; g.build(); g.smoke(); print('smoke ok')" || exit 1
  for i in 1 2 3; do
    step driver_$i 300 python bench.py --gpus 1 --steps 20 --warmup 5 || exit 1
  done
  b rtt2_default --steps 200 --warmup 20 --rtt-ms 2 || exit 1
  b rtt20_default --steps 100 --warmup 10 --rtt-ms 20 || exit 1
  b lease_rtt0 --steps 200 --warmup 20 --lease-after 0.0001 || exit 1
  b lease_rtt20 --steps 100 --warmup 10 --rtt-ms 20 --lease-after 0.0001 || exit 1
elif [ "$part" = scale ]; then
  step n1 300 python bench.py --gpus 1 --steps 100 --warmup 10 --no-gpu-probe || exit 1
  for n in 2 4; do
    step n$n 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node $n --master-addr 127.0.0.1 \
        --master-port $((29540 + n)) bench.py --gpus $n --steps 100 --warmup 10 --no-gpu-probe --dist-backend gloo || exit 1
  done
else
  b gib --file-mb 1024 --steps 6 --warmup 1 || exit 1
  step pool 240 python tools/bench_pool.py --workers 8 --jobs-per-worker 100 --file-kb 1024 || exit 1
  step bt 240 python tools/bench_bt.py --mb 2048 || exit 1
  step bt_utp 240 python tools/bench_bt.py --mb 1024 --utp || exit 1
  step resume 300 python tools/bench_resume.py --gb 8 --version 1 --device cpu hybrid || exit 1
  step rccl 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 \
      --master-port 29533 bench.py --gpus 1 --steps 20 --warmup 5 --dist-always || exit 1
fi
for f in "$out"/*.log; do echo "== $(basename "$f")"; tail -n 2 "$f" | cut -c1-600; done
