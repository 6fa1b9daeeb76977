"""RSS of the worker's GPU path, step by step (box diagnostic)."""
import json
import os
import sys

sys.path.insert(0, os.getcwd())


def rss():
    return int(open("/proc/self/statm").read().split()[1]) * 4096 >> 20


def smaps_top(n=12):
    """Largest RSS mappings by file (anonymous grouped)."""
    out = {}
    cur = None
    for line in open("/proc/self/smaps"):
        parts = line.split()
        if not parts:
            continue
        if not parts[0].endswith(":") and "-" in parts[0]:
            cur = parts[5] if len(parts) > 5 else "[anon]"
        elif parts[0] == "Rss:":
            out[cur] = out.get(cur, 0) + int(parts[1])
    return sorted(((v >> 10, k) for k, v in out.items()), reverse=True)[:n]


mode = sys.argv[1] if len(sys.argv) > 1 else "torchlib"
steps = {"start": rss()}
from tritondl.ops import hashing  # noqa: E402
if mode == "system":
    hashing._torch_hip_runtime = lambda: None
steps["import_hashing"] = rss()
assert hashing.gpu_available()
steps["device_count"] = rss()
h = hashing.gpu_hasher()
steps["hasher"] = rss()
h.hash_buffer("sha1", b"x" * 65536, 16384)
steps["first_hash"] = rss()
h.release()
steps["released"] = rss()
print(json.dumps({"mode": mode, "rss_mb": steps, "held": h.held_bytes, "top": smaps_top()}))
