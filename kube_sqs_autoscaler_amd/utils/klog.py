"""klog v2 text lines (k8s.io/klog/v2 v2.2.0, /root/reference/go.sum:496).

The reference's own messages go through logrus (utils/log.py), but client-go logs through klog:
``clientcmd.BuildConfigFromFlags("", "")`` (/root/reference/scale/scale.go:33) warns that
neither --kubeconfig nor --master was given, and again when the in-cluster config fails and it
falls back to the (empty) default loading rules. klog writes to stderr, one line per message:

    Lmmdd hh:mm:ss.uuuuuu <pid, 7 wide> file:line] message

with L the severity letter (I, W, E, F) and the local time. Log-based diffs against the
reference then match on these lines too.
"""
from __future__ import annotations

import os
import sys
from datetime import datetime
from typing import Optional, TextIO

# client-go v0.19.4 tools/clientcmd/client_config.go: the two klog.Warning calls of
# BuildConfigFromFlags [upstream: line numbers of that tag]
CLIENT_CONFIG_GO = "client_config.go"
NEITHER_LINE = 608
FALLBACK_LINE = 613


def format_line(severity: str, file: str, line: int, msg: str, now: Optional[datetime] = None, pid: Optional[int] = None) -> str:
    t = now or datetime.now()
    p = os.getpid() if pid is None else pid
    text = msg if msg.endswith("\n") else msg + "\n"  # klog adds the newline when missing
    return (f"{severity[0].upper()}{t.month:02d}{t.day:02d} {t.hour:02d}:{t.minute:02d}:{t.second:02d}."
            f"{t.microsecond:06d} {p:>7d} {file}:{line}] {text}")


class Klog:
    """A minimal klog sink: ``warning(msg, file, line)`` writes one formatted line."""

    def __init__(self, out: Optional[TextIO] = None) -> None:
        self.out = out

    def warning(self, msg: str, file: str = CLIENT_CONFIG_GO, line: int = 0) -> None:
        out = self.out or sys.stderr
        out.write(format_line("W", file, line, msg))
        out.flush()
