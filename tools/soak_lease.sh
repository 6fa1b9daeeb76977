#!/usr/bin/env bash
# 12-minute lease-renewal soak: every job runs several seconds (origin and S3 streams capped at
# 40 Mbit/s), is leased after 0.5 s and renewed every second (2 s TTL), beside magnets with a DHT,
# failing jobs through delay-queue retries, heartbeats, TLS, 2 ms RTT and adaptive concurrency.
# Usage (repo root, GPU box): bash tools/soak_lease.sh OUTDIR
set -o pipefail
out=${1:-gpurun_out/r06_soak_lease}
mkdir -p "$out"
export TMPDIR=/tmp
timeout -k 10 900 python -m tritondl_testkit.soak --minutes 12 --rate 2 --file-kb 8192 --torrent-every 100 \
    --fail-every 50 --retry-delay 2 --heartbeat 10 --tls --rtt-ms 2 --dht-nodes 8 --concurrency 0 \
    --lease-after 0.5 --lease-ttl 2 --stream-mbps 40 --sample-seconds 60 --warmup-minutes 2 \
    --out "$out/soak.jsonl" > "$out/soak.log" 2>&1
rc=$?
tail -n 1 "$out/soak.jsonl" | cut -c1-3000
exit $rc
