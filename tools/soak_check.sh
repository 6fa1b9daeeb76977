#!/usr/bin/env bash
# Round-6 soak on an MI355X box: the RCCL one-rank bench path on a quiet page cache, then
# a 10-minute soak of one worker with the round-6 defaults under stress: adaptive
# concurrency, every job leased, TLS, 2 ms RTT, heartbeats, retries through delay queues,
# magnet jobs and a local DHT.  Usage (repo root, GPU box): bash tools/soak_check.sh OUTDIR
set -o pipefail
out=${1:-gpurun_out/r06_soak}
mkdir -p "$out"
export TMPDIR=/tmp
step() { local name=$1 lim=$2; shift 2; echo "[$(date +%T)] $name"; timeout -k 10 "$lim" "$@" > "$out/$name.log" 2>&1; local rc=$?; echo "[$(date +%T)] $name rc=$rc"; return $rc; }
step rccl 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 \
    --master-port 29533 bench.py --gpus 1 --steps 20 --warmup 5 --dist-always || exit 1
step driver 300 python bench.py --gpus 1 --steps 20 --warmup 5 || exit 1
step soak 780 python -m tritondl_testkit.soak --minutes 10 --rate 50 --file-kb 1024 --torrent-every 200 \
    --fail-every 100 --retry-delay 2 --heartbeat 10 --tls --rtt-ms 2 --dht-nodes 8 --concurrency 0 \
    --lease-after 0.0001 --sample-seconds 60 --warmup-minutes 2 --out "$out/soak.jsonl" || exit 1
tail -n 1 "$out/soak.jsonl" | cut -c1-3000
