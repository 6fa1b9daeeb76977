"""``-cpuprofile FILE`` — reference C11 (``cmd/downloader/downloader.go:26,32-43``
starts ``runtime/pprof`` for the process lifetime).

Here: ``cProfile`` for the whole run, written (pstats format, readable with
``python -m pstats FILE`` or snakeviz) at normal exit AND on SIGTERM/SIGINT
shutdown — the Go ``defer`` was skipped on ``log.Fatal`` paths.  Failures to
create or start the profile are warnings only, as in the reference.
"""

from __future__ import annotations

import atexit
import cProfile

from .log import log


class CPUProfiler:
    def __init__(self, path: str) -> None:
        self.path = path
        self.prof: cProfile.Profile | None = None
        self._stopped = False

    def start(self) -> bool:
        if not self.path:
            return False
        try:
            open(self.path, "ab").close()
        except OSError as e:
            log.warn("failed to create cpu profile file: %s", e)
            return False
        try:
            self.prof = cProfile.Profile()
            self.prof.enable()
        except Exception as e:  # pragma: no cover - another profiler active
            log.warn("failed to start cpu profiling: %s", e)
            self.prof = None
            return False
        log.info("started cpu profiler")
        atexit.register(self.stop)
        return True

    def stop(self) -> None:
        if self.prof is None or self._stopped:
            return
        self._stopped = True
        self.prof.disable()
        try:
            self.prof.dump_stats(self.path)
        except OSError as e:
            log.warn("failed to write cpu profile: %s", e)
