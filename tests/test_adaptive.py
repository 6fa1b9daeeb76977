"""Adaptive job concurrency (``tritondl/parallel/adaptive.py``): one job at a
time while jobs keep the CPUs busy (the reference's serial loop,
``cmd/downloader/downloader.go:103-155``), more while they mostly wait on
the network, up to the cap; pinned to one by a tight disk reserve."""

import asyncio
import os
import time

from tritondl.models import Media
from tritondl.parallel.adaptive import Controller, DemandClock

from .test_permissions import Env, run

WAITING = {"probe": 0.040, "fetched": 0.045, "upload": 0.070}     # 20 ms RTT: mostly waits
BUSY = {"probe": 0.0002, "fetched": 0.0021, "upload": 0.0022}      # loopback: the CPU moves bytes
SLOW = {"probe": 0.001, "fetched": 0.100, "upload": 0.101}         # a 100 MB/s origin: the transfer is the job
CPU_PER_JOB = 0.0065                                              # worker CPU seconds per 10 MiB job (box)


class Sim:
    """Wall and CPU clocks for a worker running ``limit`` jobs at a time: each
    finished job advances wall time by its slot time / limit and CPU time by
    the CPU one job costs."""

    def __init__(self) -> None:
        self.wall = 1000.0
        self.cpu = 0.0

    def clock(self) -> float:
        return self.wall

    def cpu_clock(self) -> float:
        return self.cpu


def _ctl(cap: int, **kw) -> tuple[Controller, Sim]:
    sim = Sim()
    return Controller(cap, warmup_jobs=kw.pop("warmup_jobs", 0), clock=sim.clock, cpu_clock=sim.cpu_clock,
                      intensity_s=0.0, **kw), sim


def _feed(c: Controller, sim: Sim, marks: dict, n: int, cpu_per_job: float = CPU_PER_JOB) -> list[int]:
    seen = []
    for _ in range(n):
        sim.wall += marks["upload"] / c.limit
        sim.cpu += cpu_per_job
        if c.observe(marks, 10 << 20):
            seen.append(c.limit)
    return seen


def test_waiting_jobs_double_the_limit_up_to_the_cap():
    c, sim = _ctl(4, cpus=64)
    assert c.limit == 1
    assert _feed(c, sim, WAITING, 20) == [2, 4]
    assert c.limit == 4 and c.last["why"] == "network waits dominate"
    assert _feed(c, sim, WAITING, 20) == []          # the cap holds
    c8, sim8 = _ctl(8, cpus=64)
    _feed(c8, sim8, WAITING, 40)
    assert c8.limit == 8


def test_cpu_bound_jobs_stay_at_one_and_bring_the_limit_back_down():
    c, sim = _ctl(4, cpus=64)
    assert _feed(c, sim, BUSY, 50) == [] and c.limit == 1
    assert c.last["job_cores"] > 2                     # a loopback job keeps ~3 cores busy
    _feed(c, sim, WAITING, 12)
    assert c.limit == 4
    assert _feed(c, sim, BUSY, 40) == [3, 2, 1]
    assert c.last["why"] == "jobs are cpu-bound"


def test_jobs_fed_by_a_slow_origin_raise_the_limit_though_they_barely_wait():
    """A bandwidth-limited origin: the job's time is the transfer (wait
    share ~0.02) but one job keeps ~0.06 cores busy, so more run at once."""
    c, sim = _ctl(4, cpus=16)
    assert _feed(c, sim, SLOW, 20) == [2, 4]
    assert c.last["wait_share"] < 0.1 and c.last["why"] == "jobs leave the cpus idle"
    assert _feed(c, sim, SLOW, 20) == []             # and it stays raised: no lowering on low wait alone


def test_the_first_decision_waits_for_the_warm_up_jobs():
    c, sim = _ctl(4, cpus=64, warmup_jobs=8)     # connection set-up looks like waiting
    assert _feed(c, sim, WAITING, 8) == [] and c.limit == 1
    assert _feed(c, sim, WAITING, 4) == [2]


def test_loopback_shaped_jobs_keep_one_job_at_a_time():
    """The box's loopback job: response head 0.15 ms after dispatch, S3 reply
    0.27 ms after the last byte, 2.15 ms in all: wait share ~0.2, and ~3
    cores busy per job."""
    c, sim = _ctl(4, cpus=16)
    loop = {"dispatch": 0.0001, "probe": 0.00025, "fetched": 0.00188, "upload": 0.00215}
    assert _feed(c, sim, loop, 60) == [] and c.limit == 1
    c.limit = 2                                  # a transient raise drops back while jobs look like that
    hot = {"dispatch": 0.00013, "probe": 0.0008, "fetched": 0.0030, "upload": 0.0034}   # ~0.32 at 2 in flight
    assert _feed(c, sim, hot, 8) == [1]


def test_a_busy_cpu_lowers_the_limit_whatever_the_waits():
    c = Controller(4, warmup_jobs=0, cpus=1, cpu_high=0.6)
    c.limit = 4
    t_end = time.process_time() + 0.3
    while time.process_time() < t_end:            # burn this process's CPU: share ~1.0 of one CPU
        pass
    c._t0 = time.monotonic() - 0.3
    assert c._decide(time.monotonic()) and c.limit == 3 and c.last["why"] == "cpu busy"


def test_a_tight_disk_reserve_pins_the_limit_to_one():
    free = [100 << 30]
    c, sim = _ctl(4, cpus=64, free_bytes=lambda: free[0], reserve=10 << 30)
    _feed(c, sim, WAITING, 12)
    assert c.limit == 4
    free[0] = (10 << 30) + (15 << 20)             # less than reserve + 2 jobs of 10 MiB
    _feed(c, sim, WAITING, 8)
    assert c.limit == 1 and c.last["why"] == "disk reserve"


def test_cpu_demand_survives_threads_that_exit_between_samples():
    """A thread that exits takes its schedstat counters with it; the demand
    clock keeps what every thread did up to the last sample, so it never
    goes backwards (which would read as jobs that leave the CPUs idle)."""
    samples = iter([{"1": 10**9, "2": 2 * 10**9},      # 3.0 s so far
                    {"1": 15 * 10**8},                  # thread 2 exited; thread 1 +0.5 s
                    {"1": 2 * 10**9, "3": 5 * 10**8},   # thread 3 started: all of it is new
                    None])                              # unreadable: CPU time instead
    clk = DemandClock(read=lambda: next(samples), fallback=lambda: 42.0)
    assert [clk(), clk(), clk()] == [3.0, 3.5, 4.5]
    assert clk() == 42.0
    live = DemandClock()
    a = live()
    sum(i * i for i in range(200_000))
    assert live() > a


def test_long_jobs_with_idle_cpus_raise_the_limit_on_ticks():
    c = Controller(4, warmup_jobs=0, cpus=64, period_s=0.05)
    time.sleep(0.06)
    assert c.tick(all_busy=True) and c.limit == 2
    time.sleep(0.06)
    assert not c.tick(all_busy=False) and c.limit == 2   # a free slot: nothing to gain


def test_worker_raises_concurrency_when_jobs_wait_and_keeps_one_on_loopback(tmp_path):
    """End to end: an origin that answers each request 30 ms late makes the
    jobs wait, the limit climbs to the cap and the shard consumers' prefetch
    follows; the same jobs without the latency keep one job at a time."""
    async def main():
        e = await Env().up(tmp_path, concurrency=0, concurrency_max=4)
        assert e.svc._limit == 1 and e.amqp.prefetch == 1
        data = os.urandom(200_000)
        e.origin.latency = 0.03
        for i in range(24):
            e.submit(Media(id=f"w{i}", source_uri=e.origin.add(f"/w{i}.mkv", data)), i)
        res = await e.wait_results(24, timeout=60)
        assert all(r.ok for r in res), [r for r in res if not r.ok]
        assert e.svc._limit == 4, e.svc._adapt.last
        await asyncio.sleep(0.2)
        assert e.amqp.prefetch == 5                 # (4 running + 4 committing + 1 buffered) over 2 shards
        assert e.svc.metrics.get("concurrency_limit") == 4
        assert len(e.converts()) == 24
        await e.down()
    run(main())


def test_fixed_concurrency_is_not_adapted(tmp_path):
    async def main():
        e = await Env().up(tmp_path, concurrency=1)
        assert e.svc._adapt is None and e.svc._limit == 1 and len(e.svc._workers) == 1
        e.origin.latency = 0.03
        data = os.urandom(100_000)
        for i in range(6):
            e.submit(Media(id=f"f{i}", source_uri=e.origin.add(f"/f{i}.mkv", data)), i)
        await e.wait_results(6)
        assert e.svc._limit == 1
        await e.down()
    run(main())
