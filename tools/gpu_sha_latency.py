#!/usr/bin/env python3
"""Latency of the HIP SHA-256 piece kernel for small batches of aws-chunked
sized chunks (device-resident data) and the host round trip (pinned host
buffer -> H2D -> kernel -> D2H) through GpuHasher.hash_buffer.  Decides
whether per-job GPU chunk hashing can hide under a download (round 3)."""
import json
import sys
import time

import torch

sys.path.insert(0, ".")
from tritondl.ops import hashing  # noqa: E402

mod = hashing.gpu_module()
s = torch.cuda.current_stream().cuda_stream
out = {}
for chunk in (8 << 10, 16 << 10, 64 << 10):
    for n in (1, 16, 64, 160, 1280):
        total = n * chunk
        d = torch.randint(0, 256, (total,), dtype=torch.uint8, device="cuda")
        o = torch.empty(n * 32, dtype=torch.uint8, device="cuda")
        for _ in range(3):
            mod.hash_device("sha256", d.data_ptr(), total, chunk, o.data_ptr(), s)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        best = 1e9
        for _ in range(10):
            e0.record()
            mod.hash_device("sha256", d.data_ptr(), total, chunk, o.data_ptr(), s)
            e1.record()
            torch.cuda.synchronize()
            best = min(best, e0.elapsed_time(e1))
        out[f"kernel_ms_chunk{chunk >> 10}k_n{n}"] = round(best, 4)
h = hashing.gpu_hasher()
for chunk in (16 << 10, 64 << 10):
    for n in (16, 160):
        buf = bytearray(torch.randint(0, 256, (n * chunk,), dtype=torch.uint8).numpy().tobytes())
        h.hash_buffer("sha256", buf, chunk)
        t = []
        for _ in range(10):
            t0 = time.perf_counter()
            h.hash_buffer("sha256", buf, chunk)
            t.append(time.perf_counter() - t0)
        out[f"roundtrip_ms_chunk{chunk >> 10}k_n{n}"] = round(min(t) * 1e3, 3)
print(json.dumps(out, indent=1))
