"""Logging + counters. Logger name is kept as "tensorframes" like the reference
(reference: src/main/python/tensorframes/core.py:15, src/main/scala/org/tensorframes/Logging.scala:4-9)."""
from __future__ import annotations

import logging
import os
import threading
import time
from collections import defaultdict
from contextlib import contextmanager

logger = logging.getLogger("tensorframes")


def initialize_logging(level: str = None):
    """Counterpart of the reference's `initialize_logging` (PythonInterface.scala:29-44)."""
    lvl = (level or os.environ.get("TFA_LOG_LEVEL", "WARNING")).upper()
    logging.basicConfig(format="%(asctime)s %(name)s %(levelname)s %(message)s")
    logger.setLevel(getattr(logging, lvl, logging.WARNING))


class Metrics:
    """Per-operator counters: rows processed, bytes H2D/D2H, kernel and wall ms,
    collective microseconds."""

    def __init__(self):
        self._lock = threading.Lock()
        self.counters = defaultdict(float)

    def add(self, key: str, v: float = 1.0):
        with self._lock:
            self.counters[key] += v

    def set(self, key: str, v: float):
        """a gauge (e.g. a library version), not a counter"""
        with self._lock:
            self.counters[key] = v

    @contextmanager
    def timer(self, key: str):
        t0 = time.perf_counter()
        try:
            yield
        finally:
            self.add(key + "_ms", (time.perf_counter() - t0) * 1e3)

    def snapshot(self) -> dict:
        with self._lock:
            return dict(self.counters)

    def reset(self):
        with self._lock:
            self.counters.clear()


metrics = Metrics()
