"""Exponential backoff with jitter — same policy as cenkalti/backoff/v4
``NewExponentialBackOff`` used by the reference's reconnect loop
(``internal/rabbitmq/client.go:305-316``): 500 ms initial, x1.5, ±50 %
randomisation, 60 s max interval, 15 min max elapsed time.

Also replaces the reference's broken publish backoff (``Backoff ^ 2`` XOR,
``client.go:226``; defect B5) with a real capped exponential.
"""

from __future__ import annotations

import random
import time
from dataclasses import dataclass


class BackoffExhausted(Exception):
    pass


@dataclass
class ExponentialBackoff:
    initial: float = 0.5
    multiplier: float = 1.5
    randomization: float = 0.5
    max_interval: float = 60.0
    max_elapsed: float | None = 15 * 60.0

    def __post_init__(self) -> None:
        self.reset()

    def reset(self) -> None:
        self._current = self.initial
        self._start = time.monotonic()

    def next_delay(self) -> float | None:
        """Return the next sleep, or None once ``max_elapsed`` is exceeded."""
        if self.max_elapsed is not None and time.monotonic() - self._start > self.max_elapsed:
            return None
        cur = self._current
        delta = self.randomization * cur
        d = random.uniform(cur - delta, cur + delta)
        self._current = min(cur * self.multiplier, self.max_interval)
        return d
