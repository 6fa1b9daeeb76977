#!/bin/bash
# Where a pinned headline job's time goes now: stage breakdown with the data
# plane trace (pinned and unpinned), and a whole-process CPU profile of 300
# pinned jobs.
set -o pipefail
OUT=${OUT:-gpurun_out/r03_breakdown}
mkdir -p $OUT
export TMPDIR=/tmp
TRITONDL_TRACE=1 timeout -k 10 300 python tools/bench_breakdown.py --reps 100 > $OUT/breakdown_pinned.jsonl 2>$OUT/err.log &&
TRITONDL_TRACE=1 timeout -k 10 300 python tools/bench_breakdown.py --reps 100 --cpus none > $OUT/breakdown_unpinned.jsonl 2>>$OUT/err.log &&
timeout -k 10 200 python bench.py --steps 300 --warmup 10 --no-gpu-probe --cpuprofile $OUT/cpu.prof > $OUT/bench_prof.log 2>&1
rc=$?
python - <<'PY'
import json
for n in ("pinned", "unpinned"):
    try:
        d = json.loads(open(f"gpurun_out/r03_breakdown/breakdown_{n}.jsonl").read().strip().splitlines()[-1])
    except Exception as e:
        print(n, "missing", e); continue
    print(n, "fetch", d["fetch"], "\n  upload", {k: v for k, v in d.items() if k.startswith("upload")}, "\n  job", d["job"])
PY
head -30 $OUT/cpu.prof.txt
exit $rc
