set -o pipefail
mkdir -p gpurun_out/lanes
timeout -k 10 300 python tools/bench_hash.py --total-mb 1024 --piece-kb 16 64 256 --reps 5 --no-files --kernel-only --lanes 64 32 16 --kinds sha1 sha256 > gpurun_out/lanes/lanes_1g.log 2>&1 &&
timeout -k 10 300 python tools/bench_hash.py --total-mb 4096 --piece-kb 16 --reps 5 --no-files --kernel-only --lanes 64 32 --kinds sha1 > gpurun_out/lanes/lanes_4g.log 2>&1
