"""``-cpuprofile FILE``: reference C11 (``cmd/downloader/downloader.go:26,32-43``
starts ``runtime/pprof`` CPU profiling for the whole process lifetime).

Go's profiler samples every goroutine at 100 Hz with little overhead.  This
module does the same for the worker, every thread included.  At ``hz``
(default 100) a sampler thread reads, for every thread of the process, the
CPU time it used since the previous tick (``/proc/self/task/*/schedstat``,
ns) and whether it is on a CPU at that instant (state ``R``):

* **Python threads** that are running are charged at their Python stack
  (``sys._current_frames``).  A thread inside a native pump
  (``_relay.recv_body`` etc., GIL released) shows the pump as its leaf frame
  (``[native] …``).
* **Native threads** are charged to a ``[thread <name>]`` frame.  These are
  the C++ task pool (hashers, verifiers) and the HIP reader threads.  Pool
  threads carry the name of their task, set with ``pthread_setname_np``
  (``tdl-sha256``, ``tdl-hash``, …).
* CPU used by a thread that is no longer running at the tick goes to a
  ``[between samples]`` frame of its class.  It is not put on the stack the
  thread now waits in.

So the per-thread-class totals are exact (the sum is checked against
``getrusage``), and the stacks show what the running threads were doing.
Short-lived threads that start and end between two ticks are missed.  The
worker starts none: its native pools are parked threads.

Output, written at normal exit and on SIGTERM/SIGINT shutdown (the Go
``defer`` was skipped on ``log.Fatal`` paths):

* ``FILE``: a gzipped pprof ``profile.proto`` with sample types
  ``samples/count`` and ``cpu/nanoseconds``, as Go writes it.  It reads with
  ``go tool pprof FILE``, speedscope or pprof's web UI.  Every sample carries
  a ``thread`` label: the thread class, i.e. the name with its trailing
  counter stripped.
* ``FILE.txt``: a plain summary.  It gives CPU by thread class, the top
  functions (self and cumulative), the process CPU from ``getrusage`` over the
  same window, and the share of that CPU the samples attribute.

Failures to create or start the profile are warnings only, as in the
reference.  ``TRITONDL_PROFILE_HZ`` overrides the rate.
"""

from __future__ import annotations

import atexit
import collections
import gzip
import os
import re
import resource
import sys
import threading
import time

from .log import log

_TRAIL = re.compile(r"[-_ ]\d+(_\d+)?$")


def thread_class(name: str) -> str:
    """``ThreadPoolExecutor-0_3`` → ``ThreadPoolExecutor``, ``asyncio_2`` → ``asyncio``."""
    return _TRAIL.sub("", name) or name


class CPUProfiler:
    def __init__(self, path: str, hz: float | None = None) -> None:
        self.path = path
        self.hz = float(os.environ.get("TRITONDL_PROFILE_HZ", "") or hz or 100.0)
        # (thread class, stack tuple leaf-first of (name, file, line)) -> [samples, cpu ns]
        self.samples: dict[tuple, list[int]] = collections.defaultdict(lambda: [0, 0])
        self.by_class: dict[str, int] = collections.defaultdict(int)     # cpu ns per thread class
        self._last: dict[str, int] = {}          # tid -> cpu ns at the previous tick
        self._stop = threading.Event()
        self._thread: threading.Thread | None = None
        self._stopped = False
        self._tid = 0
        self._t0 = 0.0
        self._ru0 = 0.0
        self._self_ns = 0
        self.ticks = 0

    # ------------------------------------------------------------------ lifecycle
    def start(self) -> bool:
        if not self.path:
            return False
        try:
            open(self.path, "ab").close()
        except OSError as e:
            log.warn("failed to create cpu profile file: %s", e)
            return False
        if not os.path.isdir("/proc/self/task"):        # pragma: no cover - Linux has it
            log.warn("failed to start cpu profiling: no /proc/self/task")
            return False
        for tid in os.listdir("/proc/self/task"):       # CPU before the window is not ours
            v = _schedstat_ns(tid)
            if v is not None:
                self._last[tid] = v
        self._t0 = time.monotonic()
        ru = resource.getrusage(resource.RUSAGE_SELF)
        self._ru0 = ru.ru_utime + ru.ru_stime
        self._thread = threading.Thread(target=self._run, name="tdl-profiler", daemon=True)
        self._thread.start()
        log.with_fields(hz=self.hz).info("started cpu profiler")
        atexit.register(self.stop)
        return True

    def stop(self) -> None:
        if self._thread is None or self._stopped:
            return
        self._stopped = True
        self._stop.set()
        self._thread.join(timeout=5)
        self._tick()                             # the tail since the last tick
        try:
            self.write()
        except OSError as e:
            log.warn("failed to write cpu profile: %s", e)

    # ------------------------------------------------------------------ sampling
    def _run(self) -> None:
        self._tid = threading.get_native_id()
        period = 1.0 / self.hz
        nxt = time.monotonic()
        cpu_clock = time.pthread_getcpuclockid(threading.get_ident())
        while not self._stop.is_set():
            nxt += period
            delay = nxt - time.monotonic()
            if delay > 0:
                if self._stop.wait(delay):
                    break
            else:
                nxt = time.monotonic()           # fell behind: do not burst
            c0 = time.clock_gettime_ns(cpu_clock)
            self._tick()
            self.ticks += 1
            self._self_ns += time.clock_gettime_ns(cpu_clock) - c0

    def _tick(self) -> None:
        """Charge every thread's CPU since the previous tick (``schedstat``,
        ns): to its current stack if it is on a CPU now (state R), else to a
        ``[between samples]`` frame of its thread class.  Class totals are
        therefore exact; stacks are what the running threads were doing."""
        try:
            tids = os.listdir("/proc/self/task")
        except OSError:
            return
        frames = None
        by_tid = None
        for tid in tids:
            if tid == str(self._tid):
                continue
            cpu = _schedstat_ns(tid)
            if cpu is None:
                continue                          # the thread just ended
            d = cpu - self._last.get(tid, 0)      # born in the window: all of its CPU
            self._last[tid] = cpu
            if d <= 0:
                continue
            try:
                with open(f"/proc/self/task/{tid}/stat", "rb") as f:
                    st = f.read()
            except OSError:
                continue
            rp = st.rfind(b")")
            running = st[rp + 2:rp + 3] == b"R"
            if by_tid is None:
                frames = sys._current_frames()
                by_tid = {t.native_id: (ident, t) for ident, t in threading._active.items()}
            hit = by_tid.get(int(tid))
            if hit is not None:
                cls = thread_class(hit[1].name)
                frame = frames.get(hit[0]) if running else None   # type: ignore[union-attr]
            else:
                cls = thread_class(st[st.find(b"(") + 1:rp].decode(errors="replace"))
                frame = None
            if frame is not None:
                stack = []
                nat = _native_leaf(frame)
                if nat:
                    stack.append((f"[native] {nat}", "<native>", 0))
                f = frame
                while f is not None:
                    stack.append((f.f_code.co_name, f.f_code.co_filename, f.f_lineno))
                    f = f.f_back
                key = (cls, tuple(stack))
            elif hit is None and running:
                key = (cls, ((f"[thread {cls}]", "<native>", 0),))
            else:
                key = (cls, (("[between samples]", "<native>", 0), (f"[thread {cls}]", "<native>", 0)))
            s = self.samples[key]
            s[0] += 1
            s[1] += d
            self.by_class[cls] += d

    # ------------------------------------------------------------------ output
    def write(self) -> None:
        dur = time.monotonic() - self._t0
        ru = resource.getrusage(resource.RUSAGE_SELF)
        proc_ns = int((ru.ru_utime + ru.ru_stime - self._ru0) * 1e9)
        with open(self.path, "wb") as f:
            f.write(gzip.compress(encode_pprof(self.samples, dur, 1e9 / self.hz)))
        with open(self.path + ".txt", "w") as f:
            f.write(self.summary(proc_ns, dur))

    def summary(self, proc_ns: int, dur: float, top: int = 40) -> str:
        total = sum(self.by_class.values())
        lines = [f"duration {dur:.2f}s  process cpu (getrusage) {proc_ns / 1e6:.1f} ms  "
                 f"attributed to threads {total / 1e6:.1f} ms ({100 * total / max(proc_ns, 1):.1f}%)  "
                 f"profiler self {self._self_ns / 1e6:.1f} ms  ticks {self.ticks} @ {self.hz:g} Hz",
                 "", "cpu by thread class:"]
        for cls, ns in sorted(self.by_class.items(), key=lambda kv: -kv[1]):
            lines.append(f"  {ns / 1e6:10.1f} ms  {100 * ns / max(total, 1):5.1f}%  {cls}")
        selfc: dict[str, int] = collections.defaultdict(int)
        cum: dict[str, int] = collections.defaultdict(int)
        for (cls, stack), (_n, ns) in self.samples.items():
            if stack:
                selfc[_fname(stack[0])] += ns
            for fr in {_fname(x) for x in stack}:
                cum[fr] += ns
        for title, d in (("self", selfc), ("cumulative", cum)):
            lines += ["", f"top functions ({title}):"]
            for name, ns in sorted(d.items(), key=lambda kv: -kv[1])[:top]:
                lines.append(f"  {ns / 1e6:10.1f} ms  {100 * ns / max(total, 1):5.1f}%  {name}")
        return "\n".join(lines) + "\n"


def _schedstat_ns(tid: str) -> int | None:
    try:
        with open(f"/proc/self/task/{tid}/schedstat", "rb") as f:
            return int(f.read().split()[0])
    except (OSError, ValueError, IndexError):
        return None


def _native_leaf(f) -> str:
    """Name of the native pump a thread is inside, when its Python leaf frame
    is the call site (``rawhttp._counted(fn, ...)``)."""
    if f.f_code.co_name == "_counted":
        fn = f.f_locals.get("fn")
        return getattr(fn, "__name__", "") or ""
    return ""


def _fname(fr: tuple) -> str:
    name, path, _line = fr
    if path.startswith("<"):
        return name
    return f"{name} ({os.path.basename(path)})"


# ---------------------------------------------------------------------- pprof
def _varint(v: int) -> bytes:
    out = bytearray()
    v &= (1 << 64) - 1
    while True:
        b = v & 0x7F
        v >>= 7
        if v:
            out.append(b | 0x80)
        else:
            out.append(b)
            return bytes(out)


def _field(num: int, wire: int) -> bytes:
    return _varint((num << 3) | wire)


def _int(num: int, v: int) -> bytes:
    return _field(num, 0) + _varint(v)


def _bytes(num: int, b: bytes) -> bytes:
    return _field(num, 2) + _varint(len(b)) + b


def _packed(num: int, vals) -> bytes:
    return _bytes(num, b"".join(_varint(v) for v in vals))


def encode_pprof(samples: dict, duration_s: float, period_ns: float) -> bytes:
    """``perftools.profiles.Profile`` (profile.proto) for CPU samples keyed by
    (thread class, leaf-first stack); values [samples, cpu ns]."""
    strings: dict[str, int] = {"": 0}

    def s(x: str) -> int:
        i = strings.get(x)
        if i is None:
            i = strings[x] = len(strings)
        return i

    funcs: dict[tuple, int] = {}
    locs: dict[tuple, int] = {}
    out = bytearray()
    for typ, unit in (("samples", "count"), ("cpu", "nanoseconds")):
        out += _bytes(1, _int(1, s(typ)) + _int(2, s(unit)))
    for (cls, stack), (n, ns) in samples.items():
        ids = []
        for name, path, line in stack:
            fk = (name, path)
            fid = funcs.get(fk)
            if fid is None:
                fid = funcs[fk] = len(funcs) + 1
            lk = (fid, line)
            lid = locs.get(lk)
            if lid is None:
                lid = locs[lk] = len(locs) + 1
            ids.append(lid)
        label = _bytes(3, _int(1, s("thread")) + _int(2, s(cls)))
        out += _bytes(2, _packed(1, ids) + _packed(2, [n, ns]) + label)
    for (fid, line), lid in locs.items():
        out += _bytes(4, _int(1, lid) + _bytes(4, _int(1, fid) + _int(2, max(0, line))))
    for (name, path), fid in funcs.items():
        out += _bytes(5, _int(1, fid) + _int(2, s(name)) + _int(3, s(name)) + _int(4, s(path)))
    strtab = list(strings)
    for x in strtab:
        out += _bytes(6, x.encode())
    out += _int(9, time.time_ns() - int(duration_s * 1e9))
    out += _int(10, int(duration_s * 1e9))
    out += _bytes(11, _int(1, s("cpu")) + _int(2, s("nanoseconds")))
    # strings added by the period type must be in the table: re-emit new ones
    for x in list(strings)[len(strtab):]:
        out += _bytes(6, x.encode())
    out += _int(12, int(period_ns))
    return bytes(out)
