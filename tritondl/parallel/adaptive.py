"""Adaptive job concurrency: how many jobs one worker runs at a time.

The reference ran one job at a time (a single job goroutine,
``cmd/downloader/downloader.go:103-155``, with ``SetPrefetch(1)``).  That is
the right choice when a job keeps the worker's CPUs busy (a loopback or LAN
origin and S3: the worker hashes and moves ~3-4 GB/s, and a second job only
contends).  It is the wrong one when a job mostly waits on the network: at a
20 ms round trip one 10 MiB job spends most of its ~40 ms in the origin's
first byte, the S3 reply and the broker confirm, and four jobs in flight ran
2.6x as many jobs per second (``profiles/r05_rtt_ab/``).

:class:`Controller` decides from what the jobs themselves measure:

* **wait share** — for HTTP jobs, the part of the slot time (taken -> upload
  done) spent waiting on the network: the origin's connect and response head
  (``probe - dispatch``) plus the S3 reply after the last byte landed
  (``upload - fetched``);
* **CPU use** — the process's CPU seconds per second over the window, as a
  share of the CPUs it may use (affinity and cgroup quota);
* **job intensity** — the CPU its threads asked for (ran on a CPU, or waited
  on a run queue: ``/proc/self/task/*/schedstat``) over at least half a
  second, divided by the slot time of the jobs that finished in it: how
  many cores one job in flight keeps busy.  Counting run-queue waits keeps
  a starved worker on a busy host from looking idle.  A loopback job keeps ~2.8 busy (its pumps and hashers
  run in parallel).  A job fed by a bandwidth-limited origin (a CDN at
  100 MB/s per connection: 100 ms per 10 MiB) keeps ~0.07 busy.  Its wait
  share is low, because its time goes to the transfer, not to first bytes
  and replies, yet a second job would run beside it at no cost.

After every ``max(4, limit)`` finished jobs (or 2 s; the first decision
waits for ``warmup_jobs``, whose connection set-up would read as waiting),
while the median wait share is at least ``raise_at`` (0.5), or a job in
flight keeps less than ``idle_job`` (1.0) core busy, and CPU use is below
``cpu_high``, the limit doubles (up to ``cap``).  When the wait share falls
below ``lower_at`` (0.4) with jobs keeping at least ``busy_job`` (1.5) cores
busy each, or CPU use passes ``cpu_high``, it drops by one.  On the MI355X box's loopback fakes one job's wait share is ~0.2, a
job keeps ~2.9 cores busy, and the limit stays at 1 (the reference's pace,
and round 5's headline); at a 2 ms round trip the wait share is ~0.7 and at
20 ms ~0.94, and an origin capped at 100 MB/s per connection leaves ~0.07
cores busy per job: the limit goes to 4 in all three
(``profiles/r06_adaptive_v3/SUMMARY.md``).  More jobs in flight on loopback run
more jobs per second too, but only because the fake S3 verifies each PUT on
one stream: the wait there is the harness, not the network, so the
thresholds keep it out.  Jobs without HTTP marks (torrents)
count as waiting when CPU use is below ``cpu_low``.  A disk reserve below
two of the largest recent jobs pins the limit to 1 (``utils/disk.py``).
"""

from __future__ import annotations

import os
import resource
import time


def usable_cpus() -> int:
    """CPUs this process may run on: affinity, capped by a cgroup v2 quota."""
    try:
        n = len(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        n = os.cpu_count() or 1
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            quota, period = f.read().split()[:2]
        if quota != "max":
            n = min(n, max(1, int(int(quota) / int(period))))
    except (OSError, ValueError):
        pass
    return max(1, n)


def _cpu_now() -> float:
    ru = resource.getrusage(resource.RUSAGE_SELF)
    return ru.ru_utime + ru.ru_stime


def _task_demand() -> dict[str, int] | None:
    """Per thread: nanoseconds on a CPU plus nanoseconds waiting on a run
    queue (``/proc/self/task/*/schedstat``); None where that is unreadable."""
    out: dict[str, int] = {}
    try:
        tids = os.listdir("/proc/self/task")
    except OSError:
        return None
    for tid in tids:
        try:
            with open(f"/proc/self/task/{tid}/schedstat") as f:
                run, wait = f.read().split()[:2]
            out[tid] = int(run) + int(wait)
        except (OSError, ValueError):
            continue
    return out or None


class DemandClock:
    """Seconds this process's threads ran on a CPU plus the seconds they
    waited on a run queue: what the jobs asked of the CPUs, even where a busy
    or oversubscribed host did not give it.

    A thread that exits takes its counters with it, so a plain sum over the
    live threads can drop between two samples (a pump thread reaped, an
    executor shrinking) and read as an idle worker.  This accumulates each
    thread's growth since the last sample instead: monotonic, and a thread
    that exits loses only what it did after the last sample.  Falls back to
    CPU time alone."""

    def __init__(self, read=_task_demand, fallback=None) -> None:
        self._read = read
        self._fallback = fallback or _cpu_now
        self._last: dict[str, int] = {}
        self._total = 0

    def __call__(self) -> float:
        cur = self._read()
        if cur is None:
            return self._fallback()
        last = self._last
        self._total += sum(max(0, v - last.get(t, 0)) for t, v in cur.items())
        self._last = cur
        return self._total / 1e9


class Controller:
    def __init__(self, cap: int, *, start: int = 1, raise_at: float = 0.5, lower_at: float = 0.4,
                 cpu_high: float = 0.6, cpu_low: float = 0.25, idle_job: float = 1.0, busy_job: float = 1.5,
                 period_s: float = 2.0, warmup_jobs: int = 8, free_bytes=None, reserve: int = 0,
                 cpus: int | None = None, clock=time.monotonic, cpu_clock=None, demand_clock=None,
                 intensity_s: float = 0.5) -> None:
        """``clock`` / ``cpu_clock`` / ``demand_clock``: wall, process-CPU and
        CPU-demand seconds (tests pass their own); ``intensity_s``: the
        shortest span job intensity is measured over."""
        self.cap = max(1, cap)
        self.limit = min(self.cap, max(1, start))
        self.raise_at, self.lower_at = raise_at, lower_at
        self.cpu_high, self.cpu_low = cpu_high, cpu_low
        self.idle_job, self.busy_job = idle_job, busy_job
        self._clock = clock
        self._cpu_now = cpu_clock or _cpu_now
        self._demand_now = demand_clock or (cpu_clock if cpu_clock is not None else DemandClock())
        self.intensity_s = intensity_s
        self.job_cores: float | None = None   # latest job intensity (cores per job in flight)
        self.period_s = period_s
        self.free_bytes = free_bytes          # callable -> bytes free on the download fs (None: no guard)
        self.reserve = reserve
        self.cpus = cpus or usable_cpus()
        self.changes = 0
        self.last = {"wait_share": None, "cpu_share": None, "job_cores": None, "why": "start"}
        self._shares: list[float] = []
        self._slot_s = 0.0                    # slot time of the jobs finished since the last intensity sample
        self._other = 0                       # finished jobs without HTTP marks
        self._max_job_bytes = 0
        self._t0 = self._clock()
        self._cpu0 = self._cpu_now()
        self._d_t0, self._d0 = self._t0, self._demand_now()
        self._n = 0
        self._warm = warmup_jobs              # finished jobs still to see before the first decision

    def observe(self, marks: dict, nbytes: int = 0) -> bool:
        """Record one finished job; True when the limit changed."""
        if self._warm > 0:
            self._warm -= 1
            if self._warm == 0:
                self._t0, self._cpu0 = self._clock(), self._cpu_now()
                self._d_t0, self._d0, self._slot_s = self._t0, self._demand_now(), 0.0
            return False
        self._n += 1
        if nbytes > self._max_job_bytes:
            self._max_job_bytes = nbytes
        up, fet, probe = marks.get("upload"), marks.get("fetched"), marks.get("probe")
        if up and up > 0:
            self._slot_s += up
        if up and fet is not None and probe is not None and up > 0:
            head = max(0.0, probe - marks.get("dispatch", 0.0))
            self._shares.append(min(1.0, max(0.0, (head + max(0.0, up - fet)) / up)))
        else:
            self._other += 1
        now = self._clock()
        if now - self._d_t0 >= self.intensity_s and self._slot_s > 0:
            d = self._demand_now()
            self.job_cores = max(0.0, d - self._d0) / self._slot_s
            self._d_t0, self._d0, self._slot_s = now, d, 0.0
        if self._n < max(4, self.limit) and now - self._t0 < self.period_s:
            return False
        return self._decide(now)

    def tick(self, all_busy: bool) -> bool:
        """Periodic check while no job finishes (long torrents): every slot
        busy for a whole period with the CPUs mostly idle raises the limit."""
        now = self._clock()
        if self._n or now - self._t0 < self.period_s:
            return False
        cpu = self._cpu_now()
        cpu_share = (cpu - self._cpu0) / max(1e-6, now - self._t0) / self.cpus
        self._t0, self._cpu0 = now, cpu
        old = self.limit
        if all_busy and cpu_share < self.cpu_low and not self._disk_tight():
            self.limit = min(self.cap, self.limit * 2)
            self.last = {"wait_share": None, "cpu_share": round(cpu_share, 3), "job_cores": None,
                         "why": "long jobs wait (cpu idle)"}
        if self.limit != old:
            self.changes += 1
            return True
        return False

    def _decide(self, now: float) -> bool:
        dt = max(1e-6, now - self._t0)
        cpu = self._cpu_now()
        cpu_share = (cpu - self._cpu0) / dt / self.cpus
        job_cores = self.job_cores            # cores one job in flight keeps busy (sampled above)
        shares = sorted(self._shares)
        wait = shares[len(shares) // 2] if shares else None
        old = self.limit
        why = "hold"
        if self._disk_tight():
            self.limit, why = 1, "disk reserve"
        elif cpu_share > self.cpu_high:
            self.limit, why = max(1, self.limit - 1), "cpu busy"
        elif wait is not None and wait >= self.raise_at:
            self.limit, why = min(self.cap, self.limit * 2), "network waits dominate"
        elif job_cores is not None and job_cores < self.idle_job:
            self.limit, why = min(self.cap, self.limit * 2), "jobs leave the cpus idle"
        elif wait is None and self._other and cpu_share < self.cpu_low:
            self.limit, why = min(self.cap, self.limit * 2), "jobs wait (cpu idle)"
        elif wait is not None and wait < self.lower_at and (job_cores is None or job_cores >= self.busy_job):
            self.limit, why = max(1, self.limit - 1), "jobs are cpu-bound"
        self.last = {"wait_share": None if wait is None else round(wait, 3), "cpu_share": round(cpu_share, 3),
                     "job_cores": None if job_cores is None else round(job_cores, 3), "why": why}
        self._shares.clear()
        self._other = self._n = 0
        self._t0, self._cpu0 = now, cpu
        if self.limit != old:
            self.changes += 1
            return True
        return False

    def _disk_tight(self) -> bool:
        if self.free_bytes is None or self.reserve <= 0:
            return False
        try:
            free = self.free_bytes()
        except OSError:
            return False
        return free < self.reserve + 2 * self._max_job_bytes
