#!/usr/bin/env bash
# 16-minute soak of one worker with every round-6 default and a production-like mix: https jobs
# over HTTP/2, magnet jobs from a seeder with a local DHT, failing jobs through delay-queue retries,
# AMQP heartbeats, 2 ms RTT on broker and S3, adaptive concurrency, leases for jobs past 1 s.
# Usage (repo root, GPU box): bash tools/soak_mix.sh OUTDIR
set -o pipefail
out=${1:-gpurun_out/r06_soak_mix}
mkdir -p "$out"
export TMPDIR=/tmp
timeout -k 10 1100 python -m tritondl_testkit.soak --minutes 16 --rate 50 --file-kb 1024 --torrent-every 200 \
    --fail-every 100 --retry-delay 2 --heartbeat 10 --tls --h2-origin --rtt-ms 2 --dht-nodes 8 \
    --concurrency 0 --lease-after 1 --sample-seconds 60 --warmup-minutes 3 --out "$out/soak.jsonl" \
    > "$out/soak.log" 2>&1
rc=$?
tail -n 1 "$out/soak.jsonl" | cut -c1-3000
exit $rc
