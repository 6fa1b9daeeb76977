#!/bin/bash
# Round 5 pass 2: kernel TLS availability, mapped TLS send A/B (https, alternated),
# then the RTT repeats / multipart threshold / uncapped 8x8 runs.
set -o pipefail
OUT=${OUT:-gpurun_out/r05_pass2}
mkdir -p $OUT
export TMPDIR=/tmp
{ echo "tcp_available_ulp: $(cat /proc/sys/net/ipv4/tcp_available_ulp 2>&1)"; uname -r;
  openssl speed -evp aes-128-gcm -seconds 1 -bytes 16384 2>/dev/null | tail -1; } > $OUT/env.txt 2>&1
b() { local name=$1; shift; timeout -k 10 240 python bench.py --no-gpu-probe --no-reference-mode "$@" > $OUT/$name.log 2>&1; }
TRITONDL_TLS_SEND_MAP=0 b https_map0_a --steps 300 --warmup 10 --tls &&
TRITONDL_TLS_SEND_MAP=1 b https_map1_a --steps 300 --warmup 10 --tls &&
TRITONDL_TLS_SEND_MAP=0 b https_map0_b --steps 300 --warmup 10 --tls &&
TRITONDL_TLS_SEND_MAP=1 b https_map1_b --steps 300 --warmup 10 --tls &&
TRITONDL_TLS_SEND_MAP=1 b https_map1_probe2560 --steps 300 --warmup 10 --tls --probe-kb 2560 &&
OUT=$OUT bash tools/box/r05_rtt_ab2.sh > $OUT/rtt2.txt 2>&1
rc=$?
cat $OUT/env.txt
for f in $OUT/https*.log; do
  python - "$f" <<'PY'
import json, sys
f = sys.argv[1]
try:
    d = json.loads([l for l in open(f) if l.startswith("{")][-1])
except Exception:
    print(f, "no result"); sys.exit(0)
c = d.get("cpu_ms_per_job") or {}
print(f.split("/")[-1][:-4], d["value"], "fetched", d["job_spans_ms_p50"].get("fetched"), "upload",
      d["job_spans_ms_p50"].get("upload"), "send", c.get("worker_send"), "recv", c.get("worker_recv"),
      "origin", c.get("origin"), "s3", c.get("s3"), "share", d.get("fake_core_share"))
PY
done
tail -30 $OUT/rtt2.txt
exit $rc
