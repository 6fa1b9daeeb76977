"""``-cpuprofile``: a whole-process sampling CPU profile (reference C11,
``cmd/downloader/downloader.go:26,32-43``: Go's pprof samples every
goroutine).  Python threads are charged by their thread CPU clocks, native
pools by ``/proc`` schedstat; the output is a gzipped pprof profile.proto
plus a text summary."""

import gzip
import threading
import time

from tritondl.utils.profiler import CPUProfiler, thread_class


def _fields(buf: bytes):
    """Top-level (field number, wire type, value) of a protobuf message."""
    i = 0
    out = []

    def varint():
        nonlocal i
        v = s = 0
        while True:
            b = buf[i]
            i += 1
            v |= (b & 0x7F) << s
            s += 7
            if b < 0x80:
                return v
    while i < len(buf):
        key = varint()
        num, wt = key >> 3, key & 7
        if wt == 0:
            out.append((num, wt, varint()))
        elif wt == 2:
            n = varint()
            out.append((num, wt, buf[i:i + n]))
            i += n
        else:
            raise AssertionError(f"unexpected wire type {wt}")
    return out


def burn_python(stop):
    x = 0
    while not stop.is_set():
        for k in range(20000):
            x += k * k


def test_thread_class_names():
    assert thread_class("ThreadPoolExecutor-0_3") == "ThreadPoolExecutor"
    assert thread_class("asyncio_12") == "asyncio"
    assert thread_class("tdl-sha256") == "tdl-sha256"
    assert thread_class("MainThread") == "MainThread"


def test_profile_attributes_python_and_native_threads(tmp_path):
    from tritondl.ops import hashing
    path = tmp_path / "cpu.prof"
    p = CPUProfiler(str(path), hz=200)
    assert p.start()
    stop = threading.Event()
    t = threading.Thread(target=burn_python, args=(stop,), name="burner-7")
    t.start()
    data = bytes(64 << 20)
    t0 = time.monotonic()
    while time.monotonic() - t0 < 0.8:               # native SHA-1 pool threads (tdl-hash)
        hashing.piece_hashes(data, 1 << 20, "sha1", "cpu", threads=4)
    # stop while the burner still runs: a thread that ends between ticks takes its CPU
    # since the last tick with it, and on a loaded CI host the profiler thread may get
    # only a few ticks in (it needs the GIL the burner holds)
    p.stop()
    stop.set()
    t.join()
    raw = gzip.decompress(path.read_bytes())
    fields = _fields(raw)
    strings = [v.decode() for num, wt, v in fields if num == 6]
    assert strings[0] == "" and {"samples", "count", "cpu", "nanoseconds", "thread"} <= set(strings)
    assert "burn_python" in strings and "burner" in strings
    samples = [v for num, wt, v in fields if num == 2]
    assert samples and any(num == 10 and v > 0 for num, wt, v in fields)      # duration_nanos
    summary = (tmp_path / "cpu.prof.txt").read_text()
    assert "burn_python" in summary and "tdl-hash" in summary
    classes = summary.split("cpu by thread class:")[1].split("top functions")[0]
    assert "burner" in classes and "tdl-hash" in classes and "tdl-profiler" not in classes
    # per-thread CPU vs getrusage over the same window: the sampler saw (about)
    # all of the process's CPU, Python and native threads alike
    coverage = float(summary.split("attributed to threads")[1].split("(")[1].split("%")[0])
    assert 80.0 <= coverage <= 105.0, summary[:400]      # (a loaded CI host delays the last ticks)


def test_profiler_start_fails_softly(tmp_path):
    p = CPUProfiler(str(tmp_path / "missing-dir" / "x.prof"))
    assert not p.start()
    assert not CPUProfiler("").start()
