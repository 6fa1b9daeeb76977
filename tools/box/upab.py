"""Micro A/B on the box: one aws-chunked send_body of a 10 MiB file on disk
to a native sink, run from an executor thread vs started on the native pool
through the completion port.  Prints p50/min per mode and the cgroup's CPU
throttling counters around the run."""
import asyncio
import os
import socket
import statistics
import sys
import tempfile
import threading
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from tritondl.utils import rawhttp  # noqa: E402

relay = rawhttp.relay_module()
N = 10 << 20
HASHERS = int(os.environ.get("UPAB_HASHERS", "8"))


def cpu_stat():
    try:
        with open("/sys/fs/cgroup/cpu.stat") as f:
            return dict(line.split() for line in f)
    except OSError:
        return {}


async def one(mode, fd, raw):
    a, b = socket.socketpair()
    a.setblocking(False)
    b.setblocking(False)
    out = {}
    th = threading.Thread(target=lambda: out.setdefault("r", relay.recv_body(b.fileno(), -1, 0, raw, b"", None)))
    th.start()
    loop = asyncio.get_running_loop()
    args = (b"", fd, 0, N, None, 1, b"k" * 32, "20260101T000000Z", "20260101/us-east-1/s3/aws4_request", "0" * 64,
            65536, HASHERS, 30.0, None)
    t = time.perf_counter()
    if mode == "exec":
        r = await loop.run_in_executor(None, relay.send_body, relay.Sock(a.fileno()), *args)
    else:
        r = await rawhttp._port(loop).submit(loop, relay.send_body, relay.Sock(a.fileno()), args)
    dt = time.perf_counter() - t
    th.join()
    a.close()
    b.close()
    assert r[2] == "" and out["r"][2] == "", (r, out)
    return dt


async def main():
    d = tempfile.mkdtemp()
    p = os.path.join(d, "f")
    with open(p, "wb") as f:
        f.write(os.urandom(N))
    fd = os.open(p, os.O_RDONLY)
    raw = relay.chunked_length(N)
    res = {"exec": [], "port": []}
    s0 = cpu_stat()
    for _ in range(100):
        for m in ("exec", "port"):
            res[m].append(await one(m, fd, raw))
    s1 = cpu_stat()
    for m, v in res.items():
        print(f"{m} hashers={HASHERS} p50 ms {statistics.median(v) * 1e3:.3f} min {min(v) * 1e3:.3f}")
    print("throttled periods", int(s1.get("nr_throttled", 0)) - int(s0.get("nr_throttled", 0)),
          "of", int(s1.get("nr_periods", 0)) - int(s0.get("nr_periods", 0)),
          "throttled ms", (int(s1.get("throttled_usec", 0)) - int(s0.get("throttled_usec", 0))) / 1e3)


asyncio.run(main())
