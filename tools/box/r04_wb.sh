#!/bin/bash
# Cleanup-on slower than cleanup-off on one lease (r04_final): host page-cache
# state (dirty/writeback settings and totals, stable-writes devices, the work
# dir's filesystem), the driver's command first, then 300-job runs alternating
# spare recycling on / cleanup without spares / cleanup off, each with the
# vmstat deltas of its timed region (diag.vm) and spare use (diag.work_fs).
set -o pipefail
OUT=${OUT:-gpurun_out/r04_wb}
mkdir -p $OUT
export TMPDIR=/tmp
{
  for f in /proc/sys/vm/dirty_*; do echo "$f $(cat $f)"; done
  grep -E '^(MemTotal|MemFree|Cached|Dirty|Writeback):' /proc/meminfo
  for f in /sys/block/*/queue/stable_writes; do echo "$f $(cat $f)"; done
  grep -E ' / | /tmp ' /proc/mounts
  python3 -c "from tritondl.check import mount_of; print(mount_of('/tmp'))"
} > $OUT/host.txt 2>&1
timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/bench_driver.log 2>&1 &&
for i in $(seq ${REPS:-3}); do
  for arm in spares nospares off; do
    case $arm in
      spares) args="--cleanup on";;
      nospares) args="--cleanup on --recycle-mb 0";;
      off) args="--cleanup off";;
    esac
    timeout -k 10 200 python3 bench.py --steps 300 --warmup 10 --no-gpu-probe --no-reference-mode $args \
        >> $OUT/ab_$arm.log 2>&1 || exit $?
  done
done
rc=$?
cat $OUT/host.txt
python3 - "$OUT" <<'PY'
import glob, json, sys
for f in sorted(glob.glob(sys.argv[1] + "/*.log")):
    for line in open(f):
        if line.startswith('{"metric"'):
            d = json.loads(line)
            vm = d["diag"].get("vm", {})
            print(f.rsplit("/", 1)[1], d["value"], d["job_latency_ms_p50"], d["job_spans_ms_p50"].get("fetched"),
                  vm.get("nr_dirtied_per_job"), vm.get("nr_written_per_job"), vm.get("Writeback_kB"),
                  vm.get("allocstall_normal_per_job"), (d.get("reference_mode") or {}).get("jobs_per_sec"))
PY
exit $rc
