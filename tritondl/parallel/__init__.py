"""Job-level parallelism on a node: worker topology (one worker per GPU /
CPU group, torchrun-compatible ranks) and a supervised multi-process pool of
competing-consumer workers with crash detection and restart."""

from .pool import WorkerPool
from .topology import WorkerSpec, detect_gpus, plan

__all__ = ["WorkerPool", "WorkerSpec", "plan", "detect_gpus"]
