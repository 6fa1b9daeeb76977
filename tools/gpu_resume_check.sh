#!/usr/bin/env bash
# Resume-verify job benchmark (v1 and v2 torrents, host vs HIP) on one MI355X box.
set -o pipefail
out=${1:-gpurun_out/resume}
mkdir -p "$out"
timeout -k 10 600 python tools/bench_resume.py --gb 8 --version 2 --device cpu gpu auto --reps 3 > "$out/resume_v2.log" 2>&1 &&
timeout -k 10 600 python tools/bench_resume.py --gb 8 --version 1 --device cpu gpu auto --reps 3 > "$out/resume_v1.log" 2>&1
echo "rc=$?"
