#!/bin/bash
# Direct DMA knobs on the 8 GiB v1 resume job, gpu-only and hybrid, with the
# event timeline: registration block size and unregistering per window vs at
# the end of the call.
set -o pipefail
OUT=${OUT:-gpurun_out/r03_direct_knobs}
mkdir -p $OUT
export TMPDIR=/tmp
run() {  # name env...
  local name=$1; shift
  env "$@" timeout -k 10 300 python -u tools/bench_resume.py --gb 8 --version 1 --device gpu hybrid --reps 2 --trace > $OUT/$name.log 2>&1
}
run b64 TRITONDL_GPU_DIRECT_BLOCK_MB=64 &&
run b64keep TRITONDL_GPU_DIRECT_BLOCK_MB=64 TRITONDL_GPU_DIRECT_KEEP=1 &&
run b256keep TRITONDL_GPU_DIRECT_BLOCK_MB=256 TRITONDL_GPU_DIRECT_KEEP=1 &&
run b1024keep TRITONDL_GPU_DIRECT_BLOCK_MB=1024 TRITONDL_GPU_DIRECT_KEEP=1 &&
run b256 TRITONDL_GPU_DIRECT_BLOCK_MB=256 &&
run staged TRITONDL_GPU_DIRECT=0
rc=$?
for f in $OUT/*.log; do echo "== $(basename $f)"; grep warm $f | python3 -c '
import json,sys
for l in sys.stdin:
    d=json.loads(l); t=d.get("gpu_timeline",{})
    print(d["device"], d["value"], d.get("gpu_share"), d.get("direct_share"), {k:t.get(k) for k in ("h2d_ms","h2d_count","kernel_ms","kernels","kernel_under_h2d_ms","span_ms","h2d_GBps_busy")})'; done
exit $rc
