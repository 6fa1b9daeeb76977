#!/usr/bin/env bash
# rocprofv3 evidence for the HIP piece-hash kernels (run on a GPU box):
#  1) kernel trace + stats over the kernel micro-bench
#  2) SQ/GRBM counters (own run, --kernel-trace only, as the pool requires)
set -o pipefail
out=${1:-gpurun_out/prof}
mkdir -p "$out"
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$out/trace" -o run -- \
    python3 tools/bench_hash.py --total-mb 1024 --piece-kb 16 256 1024 --reps 3 --no-files > "$out/bench_hash_trace.log" 2>&1 &&
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d "$out/pmc" -o run \
    --pmc SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_BUSY_CYCLES -- \
    python3 tools/bench_hash.py --total-mb 1024 --piece-kb 16 1024 --reps 1 --no-files --kinds sha1 > "$out/bench_hash_pmc.log" 2>&1
echo "rc=$?"
