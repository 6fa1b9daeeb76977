#!/usr/bin/env python3
"""Summarise bench JSON lines from logs: value, step, latency spread and the diag."""
import json
import sys

for path in sys.argv[1:]:
    for line in open(path):
        if not line.startswith("{"):
            continue
        d = json.loads(line)
        g = d.get("diag", {})
        lat = g.get("job_latency_ms") or {}
        mhz = (g.get("cpu_mhz_pinned") or {}).get("start") or {}
        print(f"{path.split('/')[-1]:18s} {d['value']:8.1f} jobs/s  step {d['ms_per_step']:.3f}  "
              f"p50 {d['job_latency_ms_p50']}  p90 {d['job_latency_ms_p90']}  min/max {lat.get('min')}/{lat.get('max')}  "
              f"slow {len(g.get('slow_jobs', []))} ({g.get('slow_jobs_total_ms')} ms)  "
              f"cpu {d['config'].get('cpus')} mhz {mhz.get('mean')}  fresh {g.get('lease_fresh')}  "
              f"cleanup {d['config'].get('cleanup')}  worker_ms {(d.get('cpu_ms_per_job') or {}).get('worker')}")
        for s in g.get("slow_jobs", [])[:3]:
            print("     slow:", s)
