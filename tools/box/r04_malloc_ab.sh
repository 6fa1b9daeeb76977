#!/bin/bash
# Heap policy A/B on the headline: glibc's dynamic mmap threshold (0) vs a
# fixed 256 KiB threshold (the new default) vs 256 KiB + 2 arenas, alternated,
# 300 timed jobs each; minflt/job and worker CPU come with every run.
set -o pipefail
OUT=${OUT:-gpurun_out/r04_malloc}
mkdir -p $OUT
export TMPDIR=/tmp
for rep in 1 2 3; do
  for arm in dyn fixed fixed2; do
    case $arm in
      dyn) E="TRITONDL_MALLOC_MMAP_THRESHOLD=0";;
      fixed) E="TRITONDL_MALLOC_MMAP_THRESHOLD=262144";;
      fixed2) E="TRITONDL_MALLOC_MMAP_THRESHOLD=262144 TRITONDL_MALLOC_ARENA_MAX=2";;
    esac
    env $E timeout -k 10 200 python bench.py --steps 300 --warmup 10 --no-gpu-probe >> $OUT/ab_$arm.log 2>&1 || exit $?
  done
done
python3 tools/bench_summary.py $OUT/ab_*.log 2>/dev/null || true
for f in $OUT/ab_*.log; do echo "$(basename $f) $(grep -o '"value": [0-9.]*' $f | tr '\n' ' ')"; done
