"""Job orchestrator — reference component C1 (``cmd/downloader/downloader.go``).

Per job (``downloader.go:103-155``): decode ``api.Download`` → download via
the dispatcher → select media files → upload to S3 → publish
``api.Convert{CreatedAt: time.Now().String(), Media: job.Media}`` on
``v1.convert`` → ack.  Undecodable bodies are not retried (the reference
nacked them, ``:106-111``); they go to the dead-letter topic like any job
that exhausted its retries.  Startup wiring (``:28-98``): logging from env, broker
endpoint default ``127.0.0.1:5672`` (warned), prefetch 1, consume
``v1.download``, impls ``[torrent, http]``, bucket ``triton-staging``,
download dir ``$CWD/downloading``; SIGINT/SIGTERM/SIGHUP → graceful
shutdown (``:158-173``).

Differences, all documented fixes:

* B4 — a failed job is not left unacked (which stalled the channel at
  prefetch 1): it is re-published with ``X-Retries+1`` (the reference's
  unused ``Delivery.Error``) through a broker-side delay queue (the job slot
  is freed at once; the delay grows per retry) and, after ``max_retries``,
  published to the durable dead-letter topic ``<consume_topic>.dead`` with
  ``X-Failed-Stage`` / ``X-Error`` and acked.  A job is never dropped unless
  ``drop_failed`` is set.  Where the broker refuses this worker the delay
  queue (no *configure* permission, or a queue of that name with other
  arguments) the retry waits in-process instead and is re-published to the
  job's own queue — the reference's ``Error()`` exactly, needing only the
  *write* permission the reference needed; an unreachable dead-letter topic
  parks the job the same way at the longest delay.  Never a nack-requeue
  loop;
* an unusable ``S3_ENDPOINT`` is fatal at start-up, before the broker is
  dialled (the reference ``log.Fatal``-ed in ``NewUploader``,
  ``downloader.go:95-98``);
* B12 — broker connect errors are checked before use;
* jobs in flight per process: adaptive by default (1 while jobs keep the
  CPUs busy, up to ``concurrency_max`` while they wait on the network,
  :mod:`tritondl.parallel.adaptive`), or a fixed ``concurrency`` (1 = the
  reference), each job fully async so downloads / uploads of different
  jobs overlap.  A job
  frees its loop once its upload is done: the ``v1.convert`` publish, its
  broker confirm and the ack finish in the job's own task while the next
  job starts (``pipeline_commit``, on by default).  The reference published
  without confirms and acked at once (``downloader.go:147-153``), so its
  commit cost no time; this keeps the confirm-before-ack guarantee without
  a broker round trip per job on the critical path.  The ack still follows
  the confirm, and the job's dir stays locked until it is settled.  The next
  job comes from the *other* shard's consumer (prefetch 1 per shard
  consumer: the committing delivery still holds its own shard's slot until
  its ack).  With a 2 / 20 ms broker round trip it took the job rate from
  120 to 164 and from 15.8 to 23.2 jobs/s; prefetch 2 added nothing.  On
  loopback, where a confirm costs ~0.05 ms, the overlap itself cost ~4 %, so
  the worker times each publish -> confirm round trip and pipelines only
  while its EWMA is at least ``pipeline_commit_min_ms``
  (``profiles/r05_rtt_ab/``, ``profiles/r05_adaptive/``);
* a delivery whose ``X-Retries`` is past ``max_retries`` has already run
  ``max_retries + 1`` times: it goes straight to the dead-letter topic and is
  never run again (re-parked, without a download, while the dead-letter
  topic stays unreachable; ``jobs_poison_parked``).  The reference left a
  failed job unacked (a stall), never re-ran it in a loop
  (``downloader.go:117-150``);
* ``/healthz`` reflects consumption, not just the TCP connection: 503 once
  the broker connection or any shard's consumer has been down for
  ``health_down_s``, or once the worker has sat with a free job slot while
  its shard queues held ready messages for ``health_stall_s``
  (:meth:`Service.health`) — the reference's 1 s scheduler re-created dead
  processors (``client.go:139-166``), and no probe could see one that stayed
  dead;
* a job that outlives ``lease_after_s`` is leased (its delivery acked, a
  renewed copy held by the broker; :meth:`Delivery.hold`), so RabbitMQ's
  ``consumer_timeout`` never sends a running job to a second worker; a copy
  of a running job is handed back within ``job_lock_wait_s`` and a copy of a
  finished one acked through the node's done-ledger;
* in-flight jobs are drained on shutdown (the Go job goroutine was never
  joined); the work dir can optionally be cleaned after success (B15).
"""

from __future__ import annotations

import asyncio
import contextlib
import contextvars
import fcntl
import os
import queue
import shutil
import signal
import sys
import threading
import time
from concurrent.futures import ThreadPoolExecutor
from dataclasses import dataclass, field

from .amqp.client import Client, Delivery
from .fetch.http import HTTPDownloader
from .fetch.registry import ClientImpl, Dispatcher
from .models import Convert, DecodeError, Download
from .parallel.adaptive import Controller
from .s3.uploader import RESUME_SUFFIX, UploadError, Uploader
from .select import MEDIA_EXTS, dir_media, predict_media
from .utils import ledger as jobdir, rawhttp, spares
from .utils.config import Config
from .utils.gocompat import go_ext, go_join, go_time_string
from .utils.log import log
from .utils.metrics import Metrics, serve_metrics
from .utils.profiler import CPUProfiler


def default_impls(cfg: Config) -> list[ClientImpl]:
    """``[torrent.NewClient(), http.NewClient()]`` (``downloader.go:87-90``)."""
    http = HTTPDownloader(progress_interval=cfg.progress_interval_s, segments=cfg.http_segments,
                          segment_threshold=cfg.http_segment_threshold, probe_bytes=cfg.http_probe_bytes,
                          ca_file=cfg.ca_file, stripe_bytes=cfg.http_stripe_bytes,
                          disk_reserve=cfg.disk_reserve_bytes, http2=cfg.http2, h2_native=cfg.h2_native,
                          h2_conns=cfg.http2_conns)
    impls: list[ClientImpl] = []
    try:
        from .fetch.bt.client import TorrentDownloader
        impls.append(TorrentDownloader.from_config(cfg, http=http))
    except ImportError as e:  # pragma: no cover - BT stack always ships
        log.warn("bittorrent downloader unavailable: %s", e)
    impls.append(http)
    return impls


# the job slot of the delivery this task handles (pipelined commit, see Service._worker)
_SLOT: contextvars.ContextVar[asyncio.Event | None] = contextvars.ContextVar("tritondl_job_slot", default=None)


class JobBusy(Exception):
    """Another worker has held this job's dir for longer than ``job_lock_wait_s``."""


@dataclass
class JobResult:
    ok: bool
    stage: str = ""
    error: str = ""
    files: int = 0
    bytes: int = 0
    seconds: float = 0.0
    # per-job span log: stage -> seconds since the job was taken
    marks: dict = field(default_factory=dict)
    finished_at: float = 0.0           # time.monotonic() when the result was recorded


def _warm_gpu_quietly() -> bool:
    try:
        from .ops import hashing
        return hashing.warm_gpu()
    except Exception as e:  # noqa: BLE001 - optional acceleration; verification falls back to the host
        log.with_field("error", str(e)).debug("GPU hasher warm-up skipped")
        return False


class _Reaper:
    """Deletes finished job dirs on one daemon thread.  A queue put per job
    replaces an executor submit + future + loop callback per job; the
    deletion itself (mostly the kernel freeing the file's page cache) stays
    off the event loop.  ``drain`` returns once everything queued before it
    is gone (shutdown).  With a spare pool, each dir's largest file is offered
    to it first (utils/spares.py)."""

    def __init__(self) -> None:
        self._q: queue.SimpleQueue = queue.SimpleQueue()
        self._thread: threading.Thread | None = None
        self._lock = threading.Lock()
        self.pool: spares.SparePool | None = None

    def submit(self, path: str, names: list[str] | None = None) -> None:
        """Delete ``path``.  ``names``: the files the job is known to have left
        there (a streamed HTTP job's one file); they are offered to the pool
        and the dir removed with one ``rmdir`` when nothing else is in it,
        instead of walking the tree twice.  That walk runs Python on this
        thread, contending for the GIL with the event loop while it starts
        the next job."""
        if self._thread is None:
            with self._lock:
                if self._thread is None:
                    self._thread = threading.Thread(target=self._run, name="tdl-reaper", daemon=True)
                    self._thread.start()
        self._q.put((path, names))

    def _run(self) -> None:
        while True:
            item = self._q.get()
            if isinstance(item, threading.Event):
                item.set()
                continue
            path, names = item
            pool = self.pool
            if names:
                for n in names:
                    p = os.path.join(path, n)
                    if pool is None or not pool.offer(p):
                        with contextlib.suppress(OSError):
                            os.unlink(p)
                try:
                    os.rmdir(path)
                    continue
                except OSError:
                    pass                     # something else is in it: the full walk below
            if pool is not None:
                try:
                    pool.offer_dir(path)
                except OSError:
                    pass
            shutil.rmtree(path, ignore_errors=True)

    def drain(self, timeout: float = 60.0) -> bool:
        if self._thread is None:
            return True
        done = threading.Event()
        self._q.put(done)
        return done.wait(timeout)


def _touched_since(d: str, cutoff: float, limit: int = 10000) -> bool:
    """Whether ``d`` or anything under it was modified at or after ``cutoff``.
    Stops at the first such entry; a tree of more than ``limit`` entries
    counts as touched (a huge job is not worth walking to delete)."""
    if os.lstat(d).st_mtime >= cutoff:
        return True
    n = 0
    for root, dirs, files in os.walk(d):
        for name in dirs + files:
            n += 1
            if n > limit:
                return True
            try:
                if os.lstat(os.path.join(root, name)).st_mtime >= cutoff:
                    return True
            except OSError:
                pass
    return False


def _pid_alive(pid: int) -> bool:
    try:
        os.kill(pid, 0)
    except ProcessLookupError:
        return False
    except PermissionError:
        return True
    return True


TRASH_GRACE_S = 3600.0


def sweep_stale_job_dirs(base: str, max_age_s: float, skip: set[str] | frozenset = frozenset(),
                         now: float | None = None) -> list[str]:
    """Job dirs under ``base`` that nothing has touched for ``max_age_s``, and
    half-deleted ``*.deleting-<pid>-*`` dirs whose worker is gone, renamed
    aside for deletion; returns the new paths.  A job dir some worker holds
    (``flock``, :meth:`Service._job_lock`) is never taken.  These are the
    partial downloads of jobs that will not come back: their message was
    purged, or another node finished them.  The reference's work dir only
    ever grew.

    Only dirs a worker made are swept: they carry a run marker
    (:mod:`tritondl.utils.ledger`).  Anything else in ``DOWNLOAD_DIR`` (an
    operator's data, finished downloads a reference deployment kept) is left
    alone.  A trash dir whose pid is alive is skipped only while it was
    touched within ``TRASH_GRACE_S``: workers in other containers sharing
    the dir have other pid namespaces."""
    now = time.time() if now is None else now
    out: list[str] = []
    try:
        names = os.listdir(base)
    except OSError:
        return out
    for name in names:
        path = os.path.join(base, name)
        if path in skip or name.startswith("."):
            continue                                  # spare pools (.tritondl-spare-*)
        trash_pid = None
        if ".deleting-" in name:
            try:
                trash_pid = int(name.rsplit(".deleting-", 1)[1].split("-", 1)[0])
            except ValueError:
                continue
            try:
                fresh = now - os.lstat(path).st_mtime < TRASH_GRACE_S
            except OSError:
                continue
            if _pid_alive(trash_pid) and fresh:
                continue                              # its worker's reaper is on it
        elif not jobdir.is_ours(path):
            continue                                  # not made by a worker
        try:
            fd = os.open(path, os.O_RDONLY | os.O_DIRECTORY)
        except OSError:
            continue
        try:
            try:
                fcntl.flock(fd, fcntl.LOCK_EX | fcntl.LOCK_NB)
            except BlockingIOError:
                continue                              # a job is running in it (whatever its name)
            if trash_pid is not None:
                out.append(path)                      # half-deleted; its reaper died with its worker
                continue
            if _touched_since(path, now - max_age_s):
                continue
            trash = f"{path}.deleting-{os.getpid()}-stale"
            try:
                os.rename(path, trash)
            except OSError:
                continue
            out.append(trash)
        except OSError:
            continue
        finally:
            os.close(fd)
    return out


class Service:
    def __init__(self, cfg: Config, *, amqp: Client | None = None, dispatcher: Dispatcher | None = None,
                 uploader: Uploader | None = None, metrics: Metrics | None = None) -> None:
        self.cfg = cfg
        self.amqp = amqp
        self.dispatcher = dispatcher
        self.uploader = uploader
        self.metrics = metrics or Metrics()
        self._workers: list[asyncio.Task] = []
        self._tails: set[asyncio.Task] = set()     # jobs past their upload: publish confirm, ack, cleanup
        self._stop = asyncio.Event()
        self._inflight = 0
        self._limit = 1                            # jobs that may run now (see _set_limit)
        self._limit_ev = asyncio.Event()           # set (and replaced) whenever _limit changes
        self._adapt: Controller | None = None      # adaptive concurrency (cfg.concurrency == 0)
        self._adapt_task: asyncio.Task | None = None
        self._prefetch_task: asyncio.Task | None = None
        self._metrics_runner = None
        self._trimmer: asyncio.Task | None = None
        self._janitor: asyncio.Task | None = None
        self._handback: asyncio.Task | None = None
        self._busy_since = 0.0
        self.malloc_policy: dict = {}              # what tune_malloc applied at start
        self._reaper = _Reaper()                    # deletes finished job dirs off the loop
        self.results: list[JobResult] = []        # recent results (trimmed past 10,000)
        self.jobs_finished = 0                     # monotonic count of results recorded
        self._finish_waiters: list[tuple[int, asyncio.Future]] = []
        self._id_locks: dict[str, list] = {}       # media id -> [asyncio.Lock, users]
        self._locked_dirs: set[str] = set()        # job dirs _job_lock created for running jobs
        now = time.monotonic()
        self._last_finished = now                  # last job result recorded (or start)
        self._last_taken = now                     # last delivery a job loop took
        self._poison_parked = 0                    # poison jobs waiting in-process (DLQ unreachable)
        self._stall_since: float | None = None     # free slot + ready backlog, continuously since
        self._backlog = (0.0, 0)                   # (monotonic time polled, ready messages on the shards)
        self._backlog_task: asyncio.Task | None = None
        # jobs this node finished (shared by the workers on one DOWNLOAD_DIR): a copy of one
        # that comes back (a lost ack, a lease that ran out, a busy hand-back) is acked without
        # running the job again (it was uploaded and its v1.convert published)
        self.ledger: jobdir.DoneLedger | None = None
        self._housekeeper: asyncio.Task | None = None
        self.metrics.collectors.append(self._collect_gauges)

    @contextlib.asynccontextmanager
    async def _job_lock(self, media_id: str):
        """One job per media id at a time, in this process (an asyncio lock)
        and across the workers sharing ``downloading/`` (``flock`` on the job
        dir).  A job redelivered while its first delivery still runs —
        another worker whose channel died mid-job, or concurrency > 1 — would
        otherwise truncate and rewrite the very file the first delivery is
        uploading from (and the send pump maps that file).  The second
        delivery waits at most ``job_lock_wait_s`` (the first one's commit may
        be ending), then raises :class:`JobBusy` and goes back to the broker:
        an idle slot is never pinned for the length of someone else's run."""
        ent = self._id_locks.setdefault(media_id, [asyncio.Lock(), 0])
        ent[1] += 1
        fd = -1
        d = ""
        lock: asyncio.Lock = ent[0]
        try:
            if lock.locked():
                try:
                    await asyncio.wait_for(lock.acquire(), max(0.0, self.cfg.job_lock_wait_s))
                except asyncio.TimeoutError:
                    raise JobBusy(f"job {media_id} is running in another slot of this worker") from None
            else:
                await lock.acquire()
            try:
                try:
                    d = self.dispatcher.job_dir(media_id) if self.dispatcher is not None else ""
                except ValueError:
                    d = ""                          # invalid id: the job fails in its download stage
                if d:
                    try:
                        fd = await self._lock_dir(d, media_id)
                        self._locked_dirs.add(d)
                    except OSError as e:
                        log.with_fields(media_id=media_id, error=str(e)).warn("job lock unavailable")
                yield
            finally:
                lock.release()
        finally:
            self._locked_dirs.discard(d)
            if fd >= 0:
                os.close(fd)                        # releases the flock
            ent[1] -= 1
            if ent[1] == 0:
                self._id_locks.pop(media_id, None)

    async def _lock_dir(self, d: str, media_id: str) -> int:
        """Create ``d`` and ``flock`` it; returns the locked fd.

        The wait for another process's lock is a poll (``LOCK_NB`` + an
        asyncio backoff up to 0.5 s), never a blocking ``flock`` in an
        executor thread: cancellation (SIGTERM) ends it at once, and no
        thread is left blocked past shutdown.  After ``job_lock_wait_s``, or
        once shutdown has begun, it raises :class:`JobBusy` and the delivery
        goes back to the broker.
        The lock must be on the dir that is still at ``d``: with cleanup the
        holder renames its dir away when it finishes, so a lock won on an fd
        opened before that rename is on the old inode — checked by comparing
        ``fstat(fd)`` with ``stat(d)``, and retried on a fresh dir."""
        deadline = time.monotonic() + max(0.0, self.cfg.job_lock_wait_s)
        pause = 0.005
        warned = False

        async def again(why: str) -> None:
            # every retry yields to the loop and honours the deadline and shutdown, whatever
            # sent it round (a held lock, or a dir renamed away again and again)
            nonlocal pause
            if time.monotonic() >= deadline:
                raise JobBusy(f"job dir {d} {why} for {self.cfg.job_lock_wait_s:.0f}s")
            if self._stop.is_set():
                raise JobBusy(f"job dir {d} {why} at shutdown")
            await asyncio.sleep(pause)
            pause = min(pause * 2, 0.5)

        while True:
            os.makedirs(d, mode=0o755, exist_ok=True)
            try:
                fd = os.open(d, os.O_RDONLY | os.O_DIRECTORY)
            except FileNotFoundError:
                await again("kept being renamed away")  # between makedirs and open
                continue
            try:
                fcntl.flock(fd, fcntl.LOCK_EX | fcntl.LOCK_NB)
            except BlockingIOError:
                os.close(fd)
                if not warned:
                    warned = True
                    log.with_field("media_id", media_id).warn("job already running in another worker; waiting for it")
                await again("held by another worker")
                continue
            except BaseException:
                os.close(fd)
                raise
            try:
                same = os.path.samestat(os.fstat(fd), os.stat(d))
            except FileNotFoundError:
                same = False
            if same:
                return fd
            os.close(fd)                            # locked a dir that was renamed away: go again
            await again("kept being renamed away")

    async def wait_finished(self, total: int, timeout: float | None = None) -> None:
        """Wait until ``jobs_finished >= total`` (woken by the result itself,
        no polling of the event loop the jobs run on)."""
        if self.jobs_finished >= total:
            return
        fut = asyncio.get_running_loop().create_future()
        self._finish_waiters.append((total, fut))
        try:
            await asyncio.wait_for(fut, timeout)
        except asyncio.TimeoutError:
            raise TimeoutError(f"only {self.jobs_finished}/{total} jobs finished") from None
        finally:
            self._finish_waiters = [w for w in self._finish_waiters if w[1] is not fut]

    # ------------------------------------------------------------ lifecycle
    async def start(self) -> None:
        cfg = self.cfg
        self.malloc_policy = tune_malloc(cfg.malloc_mmap_threshold, cfg.malloc_arena_max,
                                         cfg.malloc_trim_threshold)
        self._size_executor()
        if self.uploader is None:
            # NewUploader (downloader.go:95-98) was fatal on a bad S3_ENDPOINT: validate
            # before dialling the broker so a misconfigured worker never takes a job
            self.uploader = Uploader.from_env(cfg.bucket, cfg.s3_endpoint, region=cfg.s3_region,
                                              part_size=cfg.s3_part_size,
                                              multipart_threshold=cfg.s3_multipart_threshold,
                                              parallel_parts=cfg.s3_parallel_parts,
                                              sign_threads=cfg.s3_sign_threads, ca_file=cfg.ca_file,
                                              hash_device=cfg.s3_hash_device, max_retries=cfg.s3_max_retries,
                                              retry_unit=cfg.s3_retry_unit_s, retry_cap=cfg.s3_retry_cap_s)
        if self.amqp is None:
            if cfg.rabbitmq_endpoint_defaulted:
                log.warn("RABBITMQ_ENDPOINT not defined, defaulting to local config: %s", cfg.rabbitmq_endpoint)
            log.info("connecting to rabbitmq ...")
            self.amqp = Client(cfg.rabbitmq_url(), prefetch=cfg.prefetch, num_shard_queues=cfg.num_shard_queues,
                               heartbeat=cfg.heartbeat_s, retry_delay=cfg.retry_delay_s,
                               declare_publish=cfg.declare_publish,
                               declare_publish_queues=cfg.declare_publish_queues)
            await self.amqp.connect()
            log.info("connected")
        else:
            self.amqp.set_prefetch(cfg.prefetch)
            if not self.amqp.connected:
                await self.amqp.connect()
        self.amqp.lease_after = cfg.lease_after_s
        self.amqp.lease_ttl = cfg.lease_s
        self._limit = self._cap if cfg.concurrency > 0 else 1
        self.amqp.set_prefetch(self._prefetch_for(self._limit))
        if self.dispatcher is None:
            self.dispatcher = Dispatcher(cfg.download_dir, default_impls(cfg), cfg.progress_log_interval_s)
        self.dispatcher.start()
        self.ledger = jobdir.DoneLedger(self.dispatcher.base_dir)
        if cfg.concurrency <= 0 and self._cap > 1:
            from .utils.disk import free_bytes
            base = self.dispatcher.base_dir
            self._adapt = Controller(self._cap, free_bytes=lambda: free_bytes(base), reserve=cfg.disk_reserve_bytes)
        if cfg.cleanup and cfg.recycle_bytes > 0:
            base = self.dispatcher.base_dir
            for stale in spares.stale_pools(base):
                self._reaper.submit(stale)
            self._reaper.pool = spares.register(spares.SparePool(
                base, max_bytes=cfg.recycle_bytes, max_files=64))
        if cfg.gpu_verify != "off":
            # HIP context + hasher set-up off the job path (first torrent resume would pay it).
            # Finished before consuming: importing torch holds the GIL for ~1-2 s, which would
            # otherwise stall the event loop under the first jobs.
            warm = asyncio.get_running_loop().run_in_executor(None, _warm_gpu_quietly)
            try:
                await asyncio.wait_for(asyncio.shield(warm), cfg.gpu_warmup_timeout_s)
            except asyncio.TimeoutError:
                log.warn("GPU hasher warm-up still running after %.0fs; consuming anyway",
                         cfg.gpu_warmup_timeout_s)
        if cfg.metrics_addr:
            self._metrics_runner = await serve_metrics(self.metrics, cfg.metrics_addr, health=self.health)
        if cfg.gc_freeze:
            freeze_startup_heap()
        await self.amqp.consume(cfg.consume_topic)
        if cfg.malloc_trim_s > 0:
            self._trimmer = asyncio.ensure_future(self._trim_heap(cfg.malloc_trim_s))
        if cfg.cleanup and cfg.stale_job_days > 0:
            self._janitor = asyncio.ensure_future(self._sweep_stale(cfg.stale_job_days * 86400.0))
        if cfg.handback_s > 0:
            self._handback = asyncio.ensure_future(self._handback_loop(cfg.handback_s))
        self._housekeeper = asyncio.ensure_future(self._housekeeping())
        self.metrics.set("concurrency_limit", self._limit)
        if self._adapt is not None:
            self._adapt_task = asyncio.ensure_future(self._adapt_ticks())
        for i in range(self._cap):
            self._workers.append(asyncio.ensure_future(self._worker(i)))

    async def _handback_loop(self, after_s: float) -> None:
        """Give buffered deliveries back to the broker while every job slot
        has been busy for ``after_s`` (:meth:`Client.pause`), so a long job
        does not hold other jobs that idle workers could run; the worker loop
        resumes consuming as soon as a slot frees."""
        assert self.amqp is not None
        while not self._stop.is_set():
            await asyncio.sleep(max(0.05, after_s / 4))
            busy = self._inflight >= self._limit
            if busy and not self.amqp.paused and time.monotonic() - self._busy_since >= after_s:
                try:
                    n = await self.amqp.pause()
                except Exception as e:  # noqa: BLE001 - an optimisation: the job carries on regardless
                    log.with_field("error", str(e)).warn("hand-back failed")
                    continue
                if n:
                    self.metrics.inc("jobs_handed_back", n)

    async def _housekeeping(self, period: float = 3600.0) -> None:
        """Hourly: drop done-ledger entries past their TTL."""
        loop = asyncio.get_running_loop()
        try:
            while True:
                await asyncio.sleep(period)
                if self.ledger is not None:
                    try:
                        n = await loop.run_in_executor(None, self.ledger.sweep)
                    except Exception as e:  # noqa: BLE001 - housekeeping must not end the worker
                        log.with_field("error", str(e)).warn("done-ledger sweep failed")
                        continue
                    if n:
                        self.metrics.inc("done_ledger_swept", n)
        except asyncio.CancelledError:
            pass

    async def _sweep_stale(self, max_age_s: float, period: float = 3600.0) -> None:
        """At start and every ``period`` s: delete job dirs untouched for
        ``max_age_s`` that no worker holds (:func:`sweep_stale_job_dirs`)."""
        loop = asyncio.get_running_loop()
        assert self.dispatcher is not None
        base = self.dispatcher.base_dir
        # its own thread: a walk over a large work dir must not hold a thread of the
        # default executor that jobs use (dir_media, warm-ups)
        pool = ThreadPoolExecutor(max_workers=1, thread_name_prefix="tdl-janitor")
        try:
            while True:
                await self._sweep_once(loop, pool, base, max_age_s)
                await asyncio.sleep(period)
        finally:
            pool.shutdown(wait=False)

    async def _sweep_once(self, loop, pool, base: str, max_age_s: float) -> None:
        try:
            gone = await loop.run_in_executor(pool, sweep_stale_job_dirs, base, max_age_s,
                                              frozenset(self._locked_dirs))
        except Exception as e:  # noqa: BLE001 - housekeeping must not end the worker
            log.with_field("error", str(e)).warn("stale job dir sweep failed")
            return
        for p in gone:
            self._reaper.submit(p)
        if gone:
            log.with_fields(dirs=len(gone)).info("removed stale job dirs")
            self.metrics.inc("stale_job_dirs_removed", len(gone))

    async def _trim_heap(self, period: float) -> None:
        """Give glibc's free arena memory back to the OS every ``period`` s.
        The native pumps, hashers and TLS streams allocate on many threads, so
        glibc keeps per-thread arenas whose freed chunks it never returns on
        its own: a 60-minute soak's RSS grew 53 -> 65 MB of arenas while the
        heap in use stayed at 14-15 MB (``profiles/r04_soak60/``).
        ``malloc_trim`` runs on an executor thread (it walks every arena)."""
        trim = _malloc_trim()
        if trim is None:
            return
        loop = asyncio.get_running_loop()
        try:
            while True:
                await asyncio.sleep(period)
                if await loop.run_in_executor(None, trim, 0):
                    self.metrics.inc("malloc_trims")
        except asyncio.CancelledError:
            pass

    def _size_executor(self) -> None:
        """Native pumps block executor threads, and an S3 send pump waits on its
        download's Flow while that download's receive pumps still need threads:
        size the loop's default pool (stdlib: min(32, cpus + 4)) so
        ``concurrency`` jobs' streams can never starve it."""
        cfg = self.cfg
        per_job = max(1, cfg.http_segments) + 2 + max(1, cfg.s3_parallel_parts)
        need = self._cap * per_job + 8
        asyncio.get_running_loop().set_default_executor(
            ThreadPoolExecutor(max_workers=max(32, need), thread_name_prefix="tritondl-io"))

    @property
    def _cap(self) -> int:
        """Most jobs this worker ever runs at once (job loops started)."""
        c = self.cfg
        return c.concurrency if c.concurrency > 0 else max(1, c.concurrency_max)

    def _prefetch_for(self, limit: int) -> int:
        """Per-shard-consumer prefetch that keeps ``limit`` jobs fed: the
        configured value (1: the reference) or, above one job, enough for
        ``limit`` running jobs, as many committing (a pipelined commit holds
        a finished job's delivery until its ``v1.convert`` is confirmed, one
        broker round trip) and one buffered, spread over the shards.  With
        only ``limit + 1`` a freed slot waited a round trip for its next
        delivery: 67 against 84 jobs/s at 20 ms RTT, 404 against 430 at 2 ms
        (``profiles/r06_prefetch_ab/``).  Buffered deliveries go back to the
        broker while every slot is held by long jobs (``handback_s``)."""
        shards = max(1, self.cfg.num_shard_queues)
        return max(self.cfg.prefetch, -(-(2 * limit + 1) // shards) if limit > 1 else 1)

    def _set_limit(self, n: int) -> None:
        """Let ``n`` jobs run at once; job loops beyond it finish their job and
        wait.  The shard consumers' prefetch follows (re-subscribed)."""
        n = max(1, min(self._cap, n))
        if n == self._limit:
            return
        log.with_fields(limit=n, was=self._limit, **(self._adapt.last if self._adapt else {})).info(
            "job concurrency changed")
        self._limit = n
        ev, self._limit_ev = self._limit_ev, asyncio.Event()
        ev.set()
        self.metrics.set("concurrency_limit", n)
        self.metrics.inc("concurrency_changes")
        want = self._prefetch_for(n)
        if self.amqp is not None and want != self.amqp.prefetch and \
                (self._prefetch_task is None or self._prefetch_task.done()):
            self._prefetch_task = asyncio.ensure_future(self._apply_prefetch())

    async def _apply_prefetch(self) -> None:
        assert self.amqp is not None
        while not self._stop.is_set():
            want = self._prefetch_for(self._limit)
            if want == self.amqp.prefetch:
                return
            try:
                await self.amqp.set_live_prefetch(want)
            except Exception as e:  # noqa: BLE001 - the next reconnect applies self.amqp.prefetch anyway
                log.with_field("error", str(e)).warn("changing the consumers' prefetch failed")
                return

    async def _adapt_ticks(self) -> None:
        assert self._adapt is not None
        try:
            while not self._stop.is_set():
                await asyncio.sleep(self._adapt.period_s)
                if self._adapt.tick(self._inflight >= self._limit):
                    self._set_limit(self._adapt.limit)
        except asyncio.CancelledError:
            pass

    async def _await_slot(self, idx: int) -> bool:
        """Wait until job loop ``idx`` may take a job (False: shutting down)."""
        while idx >= self._limit:
            if self._stop.is_set():
                return False
            waiter = asyncio.ensure_future(self._limit_ev.wait())
            stopper = asyncio.ensure_future(self._stop.wait())
            await asyncio.wait({waiter, stopper}, return_when=asyncio.FIRST_COMPLETED)
            waiter.cancel()
            stopper.cancel()
        return not self._stop.is_set()

    async def _worker(self, idx: int) -> None:
        assert self.amqp is not None
        while not self._stop.is_set():
            if idx >= self._limit and not await self._await_slot(idx):
                return
            if self.amqp.paused:
                await self.amqp.resume()    # a slot is free again: take deliveries
            try:
                # a delivery already waiting (prefetch) starts at once: no getter and
                # stopper tasks to create, race and cancel
                d = self.amqp.get_nowait()
            except asyncio.QueueEmpty:
                getter = asyncio.ensure_future(self.amqp.get())
                stopper = asyncio.ensure_future(self._stop.wait())
                done, _ = await asyncio.wait({getter, stopper}, return_when=asyncio.FIRST_COMPLETED)
                if getter not in done:
                    getter.cancel()
                    with contextlib.suppress(asyncio.CancelledError):
                        await getter
                    return
                stopper.cancel()
                d = getter.result()
            if d is None:
                return
            self._last_taken = time.monotonic()
            self._inflight += 1
            if self._inflight >= self._limit:
                self._busy_since = time.monotonic()
            self.metrics.set("jobs_inflight", self._inflight)
            if not self._pipeline_now():
                try:
                    await self.handle(d)
                finally:
                    self._inflight -= 1
                    self.metrics.set("jobs_inflight", self._inflight)
                continue
            # pipelined commit: the slot is free once the job's upload is done; its
            # publish confirm, ack and cleanup finish in the job's task meanwhile
            slot = asyncio.Event()
            t = asyncio.ensure_future(self._handle_with_slot(d, slot))
            self._tails.add(t)
            t.add_done_callback(self._tails.discard)
            freed = asyncio.ensure_future(slot.wait())
            try:
                await asyncio.wait({t, freed}, return_when=asyncio.FIRST_COMPLETED)
            finally:
                freed.cancel()
                self._inflight -= 1
                self.metrics.set("jobs_inflight", self._inflight)

    def _pipeline_now(self) -> bool:
        """Pipeline this job's commit?  Only when it is on and the broker's
        publish -> confirm round trip (EWMA over recent jobs) is long enough
        to be worth overlapping; until a confirm has been timed, not."""
        if not self.cfg.pipeline_commit:
            return False
        floor = self.cfg.pipeline_commit_min_ms / 1000.0
        if floor <= 0:
            return True
        e = self.amqp.confirm_ewma if self.amqp is not None else None
        on = e is not None and e >= floor
        self.metrics.set("pipeline_commit_active", 1.0 if on else 0.0)
        return on

    async def _handle_with_slot(self, d: Delivery, slot: asyncio.Event) -> None:
        token = _SLOT.set(slot)
        try:
            await self.handle(d)
        except Exception as e:  # noqa: BLE001 - handle() settles the delivery itself; never lose the loop
            log.with_field("error", str(e)).error("job task failed")
        finally:
            slot.set()
            _SLOT.reset(token)

    async def handle(self, msg: Delivery) -> JobResult:
        """Process one delivery end-to-end; always settles it."""
        t0 = time.monotonic()
        rawhttp.trace("job_start")
        msg.hold()                  # leased if the job outlives lease_after_s (Client.lease_after)
        if msg.metadata.retries > self.cfg.max_retries:
            # it has run max_retries + 1 times and the dead-letter publish failed after the last
            # one (it was parked with X-Retries past the budget): never download it again
            log.with_fields(retries=msg.metadata.retries, max_retries=self.cfg.max_retries).error(
                "job is past its retry budget; dead-lettering it without running it")
            self.metrics.inc("jobs", status="poison")
            await self._dead_letter(msg, "retries-exhausted",
                                    RuntimeError(f"X-Retries {msg.metadata.retries} > max_retries "
                                                 f"{self.cfg.max_retries}"))
            return self._record(JobResult(False, "poison", "retries exhausted", seconds=time.monotonic() - t0))
        try:
            job = Download.decode(msg.body)
            if job.media is None:
                raise DecodeError("missing media")
        except DecodeError as e:
            log.with_field("event", "decode-message").error(
                "failed to unmarshal rabbitmq message into protobuf format: %s", e)
            self.metrics.inc("jobs", status="undecodable")
            await self._dead_letter(msg, "decode", e)
            return self._record(JobResult(False, "decode", str(e)))

        if log.enabled("info"):
            log.with_field("job", job.to_dict()).info("got message")
        try:
            async with self._job_lock(job.media.id):
                if msg.maybe_duplicate and self.ledger is not None and self.ledger.has(msg.body):
                    # a worker on this node finished this job, and this copy came back anyway: its
                    # ack went nowhere (consumer_timeout, a channel error), its lease ran out, or
                    # it was handed back while the job ran
                    log.with_fields(media_id=job.media.id, redelivered=msg.redelivered,
                                    lease_return=msg.lease_return, busy=msg.busy).warn(
                        "job was already completed on this node; acking the copy without running it")
                    await msg.ack()
                    self._reap_job_dir(job.media.id, msg)    # the empty dir the job lock made
                    self.metrics.inc("jobs", status="duplicate")
                    return self._record(JobResult(True, "duplicate", seconds=time.monotonic() - t0))
                if msg.lease_return:
                    self.metrics.inc("lease_returns")
                if (msg.redelivered or msg.handed_back_redelivered or msg.lease_returns) and \
                        self.cfg.redelivery_limit > 0:
                    n = self._count_redelivery(job.media.id, msg)
                    if n > self.cfg.redelivery_limit:
                        log.with_fields(media_id=job.media.id, redeliveries=n).error(
                            "job keeps coming back unacknowledged (its workers die or lose their channel "
                            "mid-job); dead-lettering it without running it")
                        self.metrics.inc("jobs", status="redelivery-limit")
                        if await self._dead_letter(msg, "redelivery-limit",
                                                   RuntimeError(f"redelivered {n} times without an ack")):
                            self._reap_job_dir(job.media.id, msg)
                        self._clear_redeliveries(job.media.id)
                        with contextlib.suppress(ValueError, OSError):
                            jobdir.mark_ended(self.dispatcher.job_dir(job.media.id))
                        return self._record(JobResult(False, "redelivery-limit", f"redelivered {n} times",
                                                      seconds=time.monotonic() - t0))
                if self.ledger is not None and not msg.maybe_duplicate:
                    # a new submission of a body this node finished before (within the ledger's
                    # TTL): from here on an entry stands for THIS run, so a copy of it that comes
                    # back after a crash mid-run is run again, not acked as done
                    self.ledger.forget(msg.body)
                rawhttp.trace("job_locked")
                return await self._run_job(msg, job, t0)
        except JobBusy as e:
            # not the job's failure: hand it back without spending a retry, after a delay that
            # doubles per hand-back (X-Busy), so a copy of a long job costs a broker round trip
            # now and then, not an idle slot for the whole run
            delay = self.busy_delay(msg.busy)
            log.with_fields(media_id=job.media.id, delay_s=delay, busy=msg.busy + 1).warn(
                "%s; handing the delivery back", e)
            self.metrics.inc("jobs", status="busy")
            try:
                await msg.retry(delay, increment=0, busy=True)
            except Exception as e2:  # noqa: BLE001
                log.with_field("error", str(e2)).error("failed to hand a busy job back; parking it")
                if not (msg.settled or msg.stale):
                    self.amqp.park(msg, msg.retry_props(0, busy=True), max(delay, self.cfg.retry_delay_max_s))
            return self._record(JobResult(False, "lock", str(e), seconds=time.monotonic() - t0))

    def busy_delay(self, busy: int) -> float:
        """Delay before hand-back number ``busy + 1`` of a job another worker
        runs: max(1 s, ``retry_delay_s``) doubling, capped at ``retry_delay_max_s``."""
        base = max(1.0, self.cfg.retry_delay_s)
        return min(max(base, self.cfg.retry_delay_max_s), base * 2.0 ** min(max(0, busy), 30))

    async def _run_job(self, msg: Delivery, job: Download, t0: float) -> JobResult:
        stage = "download"
        nbytes = 0
        marks: dict[str, float] = {}

        def mark(name: str) -> None:
            marks[name] = time.monotonic() - t0

        # a run is in progress in the job dir until it settles: a dir still marked after its
        # lock is free was left by a worker that died mid-job (see _count_redelivery)
        jd = ""
        returned = msg.redelivered or msg.handed_back_redelivered or msg.lease_returns > 0
        try:
            jd = self.dispatcher.job_dir(job.media.id) if self.dispatcher is not None else ""
        except ValueError:
            pass
        if jd and jd in self._locked_dirs:
            try:
                jobdir.mark_running(jd)
            except OSError:
                jd = ""
        else:
            jd = ""
        try:
            assert self.dispatcher is not None and self.uploader is not None and self.amqp is not None
            t = time.monotonic()
            dl_dir, streamed = await self._download(job.media.id, job.media.source_uri, marks, t0)
            self.metrics.observe("stage_seconds", time.monotonic() - t, stage="download")
            mark("download")
            stage = "select"
            if streamed and len(streamed) == 1:
                files = dir_media(dl_dir)      # single-file HTTP job dir: a few entries, no executor hop
            else:
                files = await asyncio.get_running_loop().run_in_executor(None, dir_media, dl_dir)
            log.info("found %d files", len(files))
            mark("select")
            stage = "upload"
            t = time.monotonic()
            rest = [f for f in files if f not in streamed]
            res = list(streamed.values()) + (await self.uploader.upload_files(job.media.id, dl_dir, rest)
                                             if rest else [])
            nbytes = sum(r.size for r in res)
            self.metrics.observe("stage_seconds", time.monotonic() - t, stage="upload")
            mark("upload")
            stage = "publish"
            free = _SLOT.get()
            if free is not None:
                free.set()                 # the next job may start: this one only commits from here on
            log.info("creating v1.convert message")
            conv = Convert.from_download(job, go_time_string())
            await self.amqp.publish(self.cfg.publish_topic, conv.encode())
            mark("publish")
            stage = "ack"
            if log.enabled("info"):
                log.with_field("job", job.to_dict()).info("finished processing")
            if self.ledger is not None:
                # before the ack: a copy that comes back (the ack lost with its channel, a busy
                # hand-back by another worker on this node) is acked instead of run again
                try:
                    self.ledger.add(msg.body)
                except OSError as e:
                    log.with_field("error", str(e)).warn("could not record the finished job")
            await msg.ack()
            mark("ack")
            if returned:
                self._clear_redeliveries(job.media.id)
        except asyncio.CancelledError:
            if jd:
                jobdir.mark_ended(jd)         # shutdown interrupted the run: not a crash
            raise
        except Exception as e:  # noqa: BLE001 - any stage failure must settle the message
            if isinstance(e, UploadError):
                stage = "upload"             # a streamed upload fails inside the download stage
            log.with_fields(stage=stage, error=str(e)).error("job failed")
            self.metrics.inc("jobs", status="failed", stage=stage)
            if returned:
                self._clear_redeliveries(job.media.id)   # a failure handled here is X-Retries' business
            if jd:
                jobdir.mark_ended(jd)
            if await self._dispose_failed(msg, stage, e):
                self._reap_job_dir(job.media.id, msg)     # dead-lettered: no retry will resume it
            return self._record(JobResult(False, stage, str(e), seconds=time.monotonic() - t0))
        if self.cfg.cleanup:
            # a streamed single-file job left exactly its file (the .part.meta is gone) and
            # the run marker
            names = [os.path.basename(p) for p in streamed] if len(streamed) == 1 and len(files) == 1 else None
            if names is not None and jd:
                names.append(jobdir.RUNNING)
            self._reap_job_dir(dl_dir, msg, is_path=True, names=names)
        elif jd:
            jobdir.mark_ended(jd)
        dt = time.monotonic() - t0
        self.metrics.inc("jobs", status="ok")
        self.metrics.inc("bytes_uploaded", nbytes)
        self.metrics.observe("job_seconds", dt)
        if log.enabled("debug"):
            log.with_fields(media_id=job.media.id, bytes=nbytes,
                            **{k: round(v * 1000, 3) for k, v in marks.items()}).debug("job spans (ms)")
        return self._record(JobResult(True, "done", files=len(files), bytes=nbytes, seconds=dt, marks=marks))

    async def _download(self, media_id: str, url: str, marks: dict | None = None,
                        t0: float = 0.0) -> tuple[str, dict]:
        """Download the job's source.  For single-file HTTP sources whose file
        the selector will pick (a top-level media file — the root is always
        walked), the S3 upload is started right away and follows the download's
        contiguous-bytes watermark, so fetch and upload overlap instead of
        running back to back.  Returns (job dir, {path: UploadResult})."""
        assert self.dispatcher is not None and self.uploader is not None
        impl = self.dispatcher.select(url)
        if self.cfg.stream_upload and getattr(impl, "streams_files", False):
            return await self._download_torrent(impl, media_id, url, marks, t0)
        if not (self.cfg.stream_upload and isinstance(impl, HTTPDownloader)):
            return await self.dispatcher.download(media_id, url), {}
        d = self.dispatcher.job_dir(media_id)
        if d not in self._locked_dirs:          # _job_lock made, locked and checked it already
            os.makedirs(d, mode=0o755, exist_ok=True)
        if marks is not None:
            marks["dispatch"] = time.monotonic() - t0
        h = await impl.start(d, self.dispatcher.sink, url)
        if marks is not None:
            marks["probe"] = time.monotonic() - t0
        up: asyncio.Task | None = None
        fd = None
        if h.size and go_ext(h.filename) in MEDIA_EXTS:
            # the download's task (made in impl.start) runs its first step before this
            # upload's: a single stream's receive pump starts ahead of the SigV4 setup
            fd = h.open_reader()
            if h.flow is not None:
                # a PUT that follows a stalled download would idle into the store's request timeout
                h.flow.stall = self.cfg.s3_stream_stall_s
            up = asyncio.ensure_future(self.uploader.upload_stream(media_id, h.filename, fd, h.size, h.wait_bytes,
                                                                   flow=h.flow,
                                                                   resume_path=h.dst + RESUME_SUFFIX))
        try:
            await h.wait()
            if marks is not None:
                marks["fetched"] = time.monotonic() - t0
            if up is None:
                return d, {}
            return d, {h.dst: await up}
        except BaseException:
            h.cancel()
            if up is not None:
                up.cancel()
                with contextlib.suppress(BaseException):
                    await up
            raise
        finally:
            if fd is not None:
                os.close(fd)

    async def _download_torrent(self, impl, media_id: str, url: str, marks: dict | None,
                                t0: float) -> tuple[str, dict]:
        """Torrent job with per-file streamed uploads: every file the selector
        will pick starts its S3 upload the moment its last piece is verified
        (the torrent fetches those files first, in order), so upload time
        overlaps the rest of the swarm download instead of following it.  An
        upload failure cancels the download.  Returns (job dir, {path:
        UploadResult}) for the files already uploaded; anything the final
        selector walk finds beyond them is uploaded afterwards as before."""
        assert self.dispatcher is not None and self.uploader is not None
        d = self.dispatcher.job_dir(media_id)
        os.makedirs(d, mode=0o755, exist_ok=True)
        uploads: dict[str, asyncio.Task] = {}
        sem = asyncio.Semaphore(self.uploader.file_concurrency)
        dl: asyncio.Task | None = None

        def pick(paths: list[str]) -> set[str]:
            got = predict_media(d, paths)
            if got is None:
                log.with_field("dir", d).debug("job dir has foreign directories; uploads wait for the download")
                return set()
            return got

        async def upload_one(path: str):
            async with sem:
                res = await self.uploader.upload_files(media_id, d, [path])
            if marks is not None and "first_upload" not in marks:
                marks["first_upload"] = time.monotonic() - t0
            return res[0]

        def upload_failed(t: asyncio.Task) -> None:
            if not t.cancelled() and t.exception() is not None and dl is not None and not dl.done():
                dl.cancel()

        def on_file(path: str) -> None:
            path = go_join(path)
            if path in uploads:
                return
            if marks is not None and not uploads:
                marks["first_file"] = time.monotonic() - t0
            t = asyncio.ensure_future(upload_one(path))
            t.add_done_callback(upload_failed)
            uploads[path] = t

        dl = asyncio.ensure_future(impl.download(d, self.dispatcher.sink, url, pick_files=pick, on_file=on_file))
        try:
            try:
                await dl
            except asyncio.CancelledError:
                failed = [t for t in uploads.values() if t.done() and not t.cancelled() and t.exception()]
                if failed:
                    raise failed[0].exception() from None
                raise
            if marks is not None:
                marks["fetched"] = time.monotonic() - t0
            done = await asyncio.gather(*uploads.values())
            return d, dict(zip(uploads, done))
        except BaseException:
            dl.cancel()
            for t in uploads.values():
                t.cancel()
            await asyncio.gather(dl, *uploads.values(), return_exceptions=True)
            raise

    def _record(self, r: JobResult) -> JobResult:
        self._last_finished = r.finished_at = time.monotonic()
        if self._adapt is not None and r.ok and r.stage == "done" and self._adapt.observe(r.marks, r.bytes):
            self._set_limit(self._adapt.limit)
        self.results.append(r)
        if len(self.results) > 10000:
            del self.results[:5000]
        self.jobs_finished += 1
        for total, fut in self._finish_waiters:
            if total <= self.jobs_finished and not fut.done():
                fut.set_result(None)
        return r

    async def _dispose_failed(self, msg: Delivery, stage: str, err: Exception) -> bool:
        """B4 fix: retry with X-Retries+1 through a broker delay queue (the slot
        is free at once; parked in-process if the broker refuses the delay
        queue), dead-letter after ``max_retries``.  True once the job has
        left for good (dead-lettered or dropped): nothing will resume it."""
        assert self.amqp is not None
        try:
            if msg.metadata.retries < self.cfg.max_retries:
                d = self.cfg.retry_delay_for(msg.metadata.retries)
                log.with_fields(retries=msg.metadata.retries + 1, delay_s=d).warn("scheduling job retry")
                how = await msg.retry(d)
                self.metrics.inc("jobs_retried")
                if how == "parked":
                    self.metrics.inc("jobs_parked")
                return False
        except Exception as e:  # noqa: BLE001
            # the retry publish itself failed: the delivery must still be settled, or a
            # prefetch-1 consumer stalls (B4)
            log.with_field("error", str(e)).error("failed to schedule retry; dead-lettering the job")
        return await self._dead_letter(msg, stage, err)

    async def _dead_letter(self, msg: Delivery, stage: str, err: Exception) -> bool:
        """Publish the job (confirmed) to the durable dead-letter topic, then ack.
        If the dead-letter topic cannot be reached (a user that may neither
        declare nor write it), the job is parked: re-published to its own
        queue with ``X-Retries+1`` after ``retry_delay_max_s`` — the
        reference's ``Error()`` at the longest delay, never a nack-requeue
        loop, and never dropped.  True when the job was dead-lettered (or
        dropped), False when it was parked or its channel was lost."""
        assert self.amqp is not None
        try:
            if self.cfg.drop_failed:
                await msg.nack(requeue=False)
                self.metrics.inc("jobs_dropped")
                return True
            hdrs = dict(msg.msg.properties.headers or {})
            hdrs.update({"X-Retries": msg.metadata.retries, "X-Failed-Stage": stage, "X-Error": str(err)[:512],
                         "X-Original-Routing-Key": msg.routing_key})
            await self.amqp.publish(self.cfg.dlq_topic, msg.body, headers=hdrs, max_attempts=3)
            await msg.ack()
            log.with_fields(topic=self.cfg.dlq_topic, stage=stage).warn("job dead-lettered")
            self.metrics.inc("jobs_dead_lettered")
            return True
        except Exception as e:  # noqa: BLE001
            if msg.settled or msg.stale:
                return False                # its channel is gone: the broker redelivers it anyway
            log.with_fields(error=str(e), delay_s=self.cfg.retry_delay_max_s).error(
                "failed to dead-letter job; parking it")
            # X-Retries ends one past the budget, where handle() stops running the job
            poison = msg.metadata.retries > self.cfg.max_retries
            self._poison_parked += 1
            self.amqp.park(msg, msg.retry_props(0 if poison else 1), self.cfg.retry_delay_max_s,
                           on_done=self._poison_unparked)
            self.metrics.inc("jobs_parked")
            return False

    def _reap_job_dir(self, media_id: str, msg: Delivery, is_path: bool = False,
                      names: list[str] | None = None) -> None:
        """With cleanup on, a settled job's dir is moved aside (one rename, so a
        redelivered job with the same id starts clean) and deleted off the
        critical path (drained on shutdown).  After a success, and after a
        dead-letter: a poison job's partial download (GBs of torrent) would
        otherwise stay on disk forever.  Called with the job lock held."""
        if not self.cfg.cleanup:
            return
        try:
            d = media_id if is_path else self.dispatcher.job_dir(media_id)  # type: ignore[union-attr]
        except (ValueError, AttributeError):
            return
        if not os.path.isdir(d):
            return
        trash = f"{d}.deleting-{os.getpid()}-{id(msg):x}"
        try:
            os.rename(d, trash)
        except OSError:
            trash = d
        self._reaper.submit(trash, names)

    _REDELIVERIES = ".tritondl-redeliveries"

    def _count_redelivery(self, media_id: str, msg: Delivery) -> int:
        """How many times this job came back from a run that died: the larger
        of a count kept in its job dir (it survives a crashed worker, and every
        worker sharing ``downloading/`` sees it) and the lease returns carried
        in ``X-Lease-Returns`` (a lease runs out only when its holder stopped
        renewing it, on any node).

        The dir count goes up only when the previous run left its
        ``.tritondl-running`` marker (:mod:`tritondl.utils.ledger`): the run
        started and never settled.  A delivery that comes back because of a
        graceful shutdown, a broker or connection restart, or a prefetched
        delivery that never started, is not counted.  RabbitMQ's
        ``x-delivery-count`` (quorum queues) counts all of those too, so it
        is used only next to a crash marker.  Called only for returned
        deliveries, so a job's first delivery costs nothing."""
        try:
            d = self.dispatcher.job_dir(media_id)
        except (ValueError, AttributeError):
            return msg.lease_returns
        path = os.path.join(d, self._REDELIVERIES)
        try:
            with open(path) as f:
                n = int(f.read().strip() or 0)
        except (OSError, ValueError):
            n = 0
        if jobdir.was_running(d):
            n += 1
            try:
                with open(path, "w") as f:
                    f.write(str(n))
            except OSError:
                pass
            hdr = (msg.msg.properties.headers or {}).get("x-delivery-count")
            if isinstance(hdr, int) and not isinstance(hdr, bool):
                n = max(n, hdr)
        return max(n, msg.lease_returns)

    def _clear_redeliveries(self, media_id: str) -> None:
        try:
            os.unlink(os.path.join(self.dispatcher.job_dir(media_id), self._REDELIVERIES))
        except (OSError, ValueError, AttributeError):
            pass

    def _poison_unparked(self) -> None:
        self._poison_parked -= 1

    # ------------------------------------------------------------ health
    def _collect_gauges(self) -> None:
        """Gauges computed when ``/metrics`` is scraped."""
        m = self.metrics
        now = time.monotonic()
        m.set("last_job_finished_age_seconds", round(now - self._last_finished, 3))
        m.set("jobs_poison_parked", self._poison_parked)
        if self.amqp is not None:
            m.set("jobs_parked_waiting", self.amqp.parked)
            lost = self.amqp.lost_since
            m.set("broker_down_seconds", 0.0 if lost is None else round(now - lost, 3))
            m.set("consumers_paused", 1.0 if self.amqp.paused else 0.0)
            m.set("leases_held", len(self.amqp._leased))
            for kind, v in self.amqp.lease_stats.items():
                m.set("lease_events", v, kind=kind)
            for q, sh in self.amqp.shards.items():
                m.set("consumer_active", 1.0 if sh.active else 0.0, queue=q)

    async def health(self) -> tuple[bool, list[str]]:
        """(healthy, reasons) for ``/healthz``: the broker client's view (connection
        and per-shard consumers down longer than ``health_down_s``) plus a stall
        check — a free job slot while the shard queues hold ready messages, with
        no delivery taken, for ``health_stall_s``."""
        if self.amqp is None:
            return False, ["not started"]
        ok, why = self.amqp.health(self.cfg.health_down_s)
        stall = await self._stall_reason()
        if stall:
            why.append(stall)
        return not why, why

    async def _poll_backlog(self, now: float) -> None:
        """Ready messages this worker could be given now: only shards whose
        consumer has prefetch to spare count.  A shard whose consumer is full
        (a long job holds its delivery) cannot hand its backlog to a free slot
        here, and that is not a stall of this worker."""
        try:
            counts = await asyncio.wait_for(self.amqp.ready_counts(self.cfg.consume_topic), 5.0)
            sh = self.amqp.shards
            n = sum(c for q, c in counts.items() if q in sh and sh[q].has_room(self.amqp.prefetch))
            self._backlog = (now, n)
        except Exception:  # noqa: BLE001 - a missing queue is the shard check's business
            self._backlog = (now, 0)

    async def _stall_reason(self) -> str:
        limit = self.cfg.health_stall_s
        now = time.monotonic()
        if limit <= 0 or self._stop.is_set() or self.amqp is None or not self.amqp.connected or \
                self._inflight >= self._limit:
            self._stall_since = None
            return ""
        if now - self._backlog[0] >= 5.0 and (self._backlog_task is None or self._backlog_task.done()):
            # one passive declare per shard, at most every 5 s, in the background: /healthz
            # answers from the last count at once (a probe's own timeout is often 1 s)
            self._backlog_task = asyncio.ensure_future(self._poll_backlog(now))
        if self._backlog[1] <= 0:
            self._stall_since = None
            return ""
        if self._stall_since is None:
            self._stall_since = now
        idle = now - max(self._stall_since, self._last_taken)
        if idle > limit:
            return f"{self._backlog[1]} ready messages and a free job slot, no delivery taken for {idle:.0f}s"
        return ""

    async def shutdown(self, grace: float = 30.0) -> None:
        log.info("shutting down")
        self._stop.set()
        for t in (self._trimmer, self._janitor, self._handback, self._housekeeper, self._adapt_task,
                  self._prefetch_task):
            if t is not None:
                t.cancel()
        t_end = time.monotonic() + grace
        if self._workers:
            done, pending = await asyncio.wait(self._workers, timeout=grace)
            for t in pending:
                t.cancel()
            for t in pending:
                with contextlib.suppress(BaseException):
                    await t
        if self._tails:                      # jobs still committing (publish confirm, ack)
            done, pending = await asyncio.wait(set(self._tails), timeout=max(1.0, t_end - time.monotonic()))
            for t in pending:
                t.cancel()
            for t in pending:
                with contextlib.suppress(BaseException):
                    await t
        pool, self._reaper.pool = self._reaper.pool, None
        if pool is not None:
            spares.unregister(pool)
            self._reaper.submit(pool.root)
        await asyncio.get_running_loop().run_in_executor(None, self._reaper.drain)
        if pool is not None:
            pool.clear()                    # whatever was offered while the rmtree was queued
        if self.dispatcher is not None:
            await self.dispatcher.stop()
        if self.uploader is not None:
            await self.uploader.close()
        if self.amqp is not None:
            await self.amqp.close()
        if self._metrics_runner is not None:
            await self._metrics_runner.cleanup()
        log.info("finished shutdown")

    async def run_forever(self) -> None:
        loop = asyncio.get_running_loop()
        stop = asyncio.Event()
        for s in (signal.SIGINT, signal.SIGTERM, signal.SIGHUP):
            with contextlib.suppress(NotImplementedError, RuntimeError):
                loop.add_signal_handler(s, stop.set)
        await self.start()
        await stop.wait()
        await self.shutdown()


def freeze_startup_heap() -> int:
    """Collect once, then move every surviving object to CPython's permanent
    generation (``gc.freeze``), so later full collections skip them.  With
    torch imported a process holds ~180k tracked objects.  A full collection
    walks all of them on the event loop, which takes 40-100 ms: longer than
    thirty 10 MiB jobs.  Returns the number of objects frozen."""
    import gc
    gc.collect()
    gc.freeze()
    return gc.get_freeze_count()


def tune_malloc(mmap_threshold: int, arena_max: int = 0, trim_threshold: int = 0) -> dict:
    """Fix glibc's heap policy for a long-running process with many native
    threads (``mallopt``; a no-op elsewhere).  ``mmap_threshold > 0`` pins
    M_MMAP_THRESHOLD, which also turns off glibc's dynamic adjustment: left
    dynamic it rises to the largest block ever freed, so MiB-sized buffers
    are then carved from per-thread arenas that keep up to twice the
    threshold free at their top.  A 6-minute soak (TLS, DHT, heartbeats):
    arenas 102.6 MB and RSS 160 MB dynamic, 25 MB and 82 MB with 256 KiB,
    heap in use 14.7 MB in both (``profiles/r04_malloc/``).  Returns what
    was applied."""
    import ctypes
    out: dict = {}
    try:
        mallopt = ctypes.CDLL("libc.so.6").mallopt
    except (OSError, AttributeError):
        return out
    mallopt.argtypes = [ctypes.c_int, ctypes.c_int]
    mallopt.restype = ctypes.c_int
    M_TRIM_THRESHOLD, M_MMAP_THRESHOLD, M_ARENA_MAX = -1, -3, -8
    if mmap_threshold > 0 and mallopt(M_MMAP_THRESHOLD, int(mmap_threshold)):
        out["mmap_threshold"] = int(mmap_threshold)
    # pinning the mmap threshold also pins the trim threshold (128 KiB unless set):
    # free space above it at an arena's top goes back to the OS on every free().
    # Only alongside a pinned mmap threshold: setting it alone would also end
    # glibc's dynamic policy, which mmap_threshold=0 asks to keep
    if mmap_threshold > 0 and trim_threshold > 0 and mallopt(M_TRIM_THRESHOLD, int(trim_threshold)):
        out["trim_threshold"] = int(trim_threshold)
    if arena_max > 0 and mallopt(M_ARENA_MAX, int(arena_max)):
        out["arena_max"] = int(arena_max)
    return out


def _malloc_trim():
    """glibc's ``malloc_trim`` (None elsewhere, e.g. musl)."""
    import ctypes
    try:
        f = ctypes.CDLL("libc.so.6").malloc_trim
    except (OSError, AttributeError):
        return None
    f.argtypes = [ctypes.c_size_t]
    f.restype = ctypes.c_int
    return f


def raise_nofile_limit() -> int:
    """Lift the soft open-files limit to the hard one (as the Go runtime does
    at start-up since 1.19): a multi-file torrent holds one descriptor per
    file for storage and one for the native serving source, next to the
    job's sockets.  Returns the soft limit now in force."""
    try:
        import resource
        soft, hard = resource.getrlimit(resource.RLIMIT_NOFILE)
        want = hard if hard != resource.RLIM_INFINITY else max(soft, 1 << 20)
        if soft < want:
            resource.setrlimit(resource.RLIMIT_NOFILE, (want, hard))
        return resource.getrlimit(resource.RLIMIT_NOFILE)[0]
    except (ImportError, ValueError, OSError):
        return -1


def main(argv: list[str] | None = None) -> int:
    cfg = Config.from_env(argv=list(sys.argv[1:] if argv is None else argv))
    log.configure(cfg.log_level, cfg.log_format)
    raise_nofile_limit()
    if cfg.cpus:
        from .parallel.topology import pin
        try:
            cpus = pin(cfg.cpus, int(os.environ.get("LOCAL_RANK", "0") or 0),
                       int(os.environ.get("LOCAL_WORLD_SIZE", "1") or 1))
        except (ValueError, OSError) as e:      # a bad cpulist is fatal configuration
            log.error("fatal: TRITONDL_CPUS=%r: %s", cfg.cpus, e)
            return 1
        if cpus:
            log.with_field("cpus", len(cpus)).info("pinned to %d..%d", cpus[0], cpus[-1])
    prof = CPUProfiler(cfg.cpuprofile)
    prof.start()
    try:
        asyncio.run(Service(cfg).run_forever())
    except Exception as e:  # log.Fatal equivalent
        log.error("fatal: %s", e)
        prof.stop()
        return 1
    prof.stop()
    return 0


if __name__ == "__main__":  # pragma: no cover
    sys.exit(main())
