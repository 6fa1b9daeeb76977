#!/bin/bash
# Round 5: native timing of the signed PUT (TRITONDL_ZC_TRACE=1): when each
# chunk's bytes were on disk for its hasher, hashed, and written by the sender.
set -o pipefail
OUT=${OUT:-gpurun_out/r05_zc_trace}
mkdir -p $OUT
export TMPDIR=/tmp
TRITONDL_ZC_TRACE=1 TRITONDL_TRACE=1 timeout -k 10 200 python bench.py --steps 300 --warmup 10 --no-gpu-probe \
    --no-reference-mode > $OUT/bench.log 2>&1
rc=$?
grep -o '"value": [0-9.]*\|"trace_p50_ms": {[^}]*}' $OUT/bench.log
python3 - "$OUT/bench.log" <<'PY'
import re, sys, statistics as st
rows = [dict((k, float(v)) for k, v in re.findall(r"(\w+)=([0-9.]+)", l)) for l in open(sys.argv[1]) if l.startswith("zc-trace")]
rows = rows[-300:]
for k in ("wide", "pair", "cov_last_us", "hash_last_us", "sent_last_us", "fin_us", "max_cov_to_sent_us"):
    v = sorted(r[k] for r in rows)
    print(f"{k}: p50 {v[len(v)//2]:.1f} p10 {v[len(v)//10]:.1f} p90 {v[9*len(v)//10]:.1f}")
d = sorted(r["sent_last_us"] - r["hash_last_us"] for r in rows)
print(f"sent_last - hash_last: p50 {d[len(d)//2]:.1f} p90 {d[9*len(d)//10]:.1f}")
d = sorted(r["hash_last_us"] - r["cov_last_us"] for r in rows)
print(f"hash_last - cov_last: p50 {d[len(d)//2]:.1f} p90 {d[9*len(d)//10]:.1f}")
PY
exit $rc
