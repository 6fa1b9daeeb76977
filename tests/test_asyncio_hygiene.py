"""Control-plane race/leak detection (the Python side of what
TSan covers for the C++ cores): jobs run with the event loop in asyncio
debug mode and every warning turned into a record.  Debug mode reports
coroutines never awaited, tasks destroyed while pending, non-thread-safe
loop calls from other threads, and unclosed transports / sockets /
files (ResourceWarning).  None may appear over successful jobs, a failed
job that is retried and dead-lettered, and a worker shutdown."""

import asyncio
import gc
import logging
import warnings

from tritondl_testkit.bench_job import JobStack


class _Catch(logging.Handler):
    def __init__(self):
        super().__init__(logging.WARNING)
        self.records = []

    def emit(self, record):
        self.records.append(self.format(record))


def test_jobs_clean_under_asyncio_debug(tmp_path):
    handler = _Catch()
    alog = logging.getLogger("asyncio")
    alog.addHandler(handler)
    alog.setLevel(logging.WARNING)

    async def main():
        loop = asyncio.get_running_loop()
        loop.slow_callback_duration = 10.0      # timing is not what this test is about
        st = JobStack(file_size=512 << 10, inproc=True, tag="dbg", workdir=str(tmp_path / "w"))
        await st.setup()
        try:
            await st.run_jobs(6)
            # a job whose upload is refused (403, not retried) fails and is dead-lettered
            s3 = st.backends[-1]
            s3.fail_next(100, status=403, code="AccessDenied")
            start = st.svc.jobs_finished
            await st.submit(1)
            await st.wait_done(start + 1)
            assert not st.svc.results[-1].ok and st.svc.results[-1].stage == "upload"
            s3.fail_next(0)
            await st.run_jobs(2)                  # and the worker carries on
        finally:
            await st.teardown()

    with warnings.catch_warnings():
        warnings.simplefilter("ignore")
        gc.collect()                              # earlier tests' garbage (same xdist worker) is not ours
    with warnings.catch_warnings(record=True) as caught:
        warnings.simplefilter("always")
        asyncio.run(asyncio.wait_for(main(), 120), debug=True)
        gc.collect()
    alog.removeHandler(handler)
    bad = [f"{w.category.__name__}: {w.message} ({w.filename}:{w.lineno})" for w in caught
           if issubclass(w.category, ResourceWarning)]
    never_awaited = [str(w.message) for w in caught if "was never awaited" in str(w.message)]
    pending = [r for r in handler.records if "destroyed but it is pending" in r or "Non-thread-safe" in r
               or "exception was never retrieved" in r]
    assert not never_awaited, never_awaited
    assert not pending, pending
    assert not bad, bad
