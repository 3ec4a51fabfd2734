"""Process logger: the native logrus-compatible ``Logger`` (csrc/core/log.h) configured from flags.

The reference logs through logrus' package-level logger with defaults (text formatter, stderr,
Info level; /root/reference/main.go:13, /root/reference/scale/scale.go:9), e.g.::

    time="2024-01-01T00:00:00Z" level=info msg="Found 3 messages in the queue"

The same logger object is handed to every native component, so bootstrap lines written from
Python and poll lines written from the C++ workers share one formatter and one sink.
"""
from __future__ import annotations

import os
import sys
from typing import Optional

from ..ops import native

LEVELS = ("panic", "fatal", "error", "warning", "warn", "info", "debug", "trace")


def make_logger(level: str = "info", fmt: str = "text", fd: Optional[int] = None, clock=None):
    nat = native()
    log = nat.Logger()
    log.set_level(level)
    log.set_format(fmt)
    if fd is None:
        try:
            fd = sys.stderr.fileno()
        except (AttributeError, ValueError, OSError):  # stderr replaced (pytest capture)
            log.set_sink(lambda line: sys.stderr.write(line + "\n"))
    if fd is not None:
        log.set_sink_fd(fd)
        if fmt == "text" and os.isatty(fd):
            log.set_format("text-color")  # logrus TextFormatter on a terminal
    if clock is not None:
        log.set_time_source(clock)
    return log


def capture_logger(lines: list, level: str = "info", clock=None):
    """Logger whose lines are appended to ``lines`` (tests, parity log diffs)."""
    nat = native()
    log = nat.Logger()
    log.set_level(level)
    log.set_sink(lines.append)
    if clock is not None:
        log.set_time_source(clock)
    return log
