#!/bin/bash
# Round 5 (end of session tree): an 18-minute time-based soak of the r05 worker under a 2 ms emulated RTT (adaptive
# pipelined commit on), TLS, heartbeats, delay-queue retries and a local DHT; /healthz sampled.
set -o pipefail
OUT=${OUT:-gpurun_out/r05_soak2}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 1140 python -u -m tritondl_testkit.soak --minutes 18 --rate 50 --file-kb 1024 --torrent-every 200 \
    --fail-every 100 --retry-delay 2 --heartbeat 10 --tls --dht-nodes 8 --rtt-ms 2 --cpus auto \
    --sample-seconds 60 --warmup-minutes 4 --out $OUT/soak.jsonl > $OUT/soak.log 2>&1
rc=$?
tail -c 3000 $OUT/soak.jsonl
exit $rc
