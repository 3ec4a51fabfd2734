"""The shared AWS files (``~/.aws/credentials``, ``~/.aws/config``): one INI reader for every
caller -- the start-up session check (session.py, ``session.Must(session.NewSession())`` at
/root/reference/sqs/sqs.go:36) and the credential chain (credentials.py).

aws-sdk-go v1.35.35 (/root/reference/go.mod:6) reads these files with its own INI lexer and
parser, and ``session.Must`` panics on a file it cannot parse. Which malformed inputs that parser
rejects is *parity unpinned* here (no Go toolchain or SDK to compare against), and the costs are
not symmetric: failing on a file the reference loads crash-loops the pod, while loading a file
the reference would reject only changes which error a later poll logs. So this reader fails
only on what the SDK's lexer cannot get past either -- a section header without its closing
``]`` -- and skips, with a warning, the lines it cannot use:

* key = value lines before the first section header (no profile can hold them);
* lines that are neither a comment, a section header nor a ``key = value`` / ``key: value``
  assignment.

Accepted, as before: ``#`` / ``;`` comment lines, blank lines, continuation lines -- indented
deeper than their key's line, as configparser reads them -- (appended to the previous value with
a newline, as in the SDK's nested ``s3 =`` blocks; keys and headers indented alike are read as
keys and headers), repeated
sections (merged) and keys (the last wins). Keys are lower-cased; inline ``;``/``#`` text after a
value is part of the value (neither parser strips it). Fixtures: tests/test_session.py.
"""
from __future__ import annotations

from typing import Dict, Iterator, List, Optional, Tuple


class IniError(ValueError):
    """A file this reader (and, as far as is known, the SDK) cannot parse."""


class IniFile:
    """Sections of one shared file, with the RawConfigParser calls its users make."""

    def __init__(self, path: str = ""):
        self.path = path
        self._sections: Dict[str, Dict[str, str]] = {}
        self.warnings: List[str] = []

    def has_section(self, name: str) -> bool:
        return name in self._sections

    def sections(self) -> List[str]:
        return list(self._sections)

    def items(self, section: str) -> List[Tuple[str, str]]:
        return list(self._sections[section].items())

    def __iter__(self) -> Iterator[str]:
        return iter(self._sections)


def parse(text: str, path: str = "") -> IniFile:
    out = IniFile(path)
    where = path or "<string>"
    section: Optional[Dict[str, str]] = None
    last_key: Optional[str] = None
    key_indent = 0  # leading whitespace of last_key's line
    for n, raw in enumerate(text.splitlines(), 1):
        line = raw.strip()
        if not line or line[0] in "#;":
            continue
        indent = len(raw) - len(raw.lstrip())
        if indent > key_indent and section is not None and last_key is not None:
            # a continuation of the previous value: indented deeper than its key line (as
            # configparser reads it), so a file whose keys are all indented alike is still read
            # key by key
            section[last_key] += "\n" + line
            continue
        if line.startswith("["):
            end = line.find("]")
            if end < 0:
                raise IniError(f"{where}, line {n}: section header without a closing ']': {line!r}")
            name = line[1:end].strip()
            section = out._sections.setdefault(name, {})
            last_key = None
            continue
        eq, colon = line.find("="), line.find(":")
        seps = [i for i in (eq, colon) if i > 0]
        if not seps:
            out.warnings.append(f"{where}, line {n}: not a key = value line, skipped: {line!r}")
            last_key = None
            continue
        if section is None:
            out.warnings.append(f"{where}, line {n}: key outside any [section], skipped: {line!r}")
            continue
        i = min(seps)
        key = line[:i].strip().lower()
        section[key] = line[i + 1:].strip()
        last_key, key_indent = key, indent
    return out


def read(path: str) -> Optional[IniFile]:
    """The parsed file, or None when it cannot be read (the SDK skips such files)."""
    try:
        with open(path, "r", encoding="utf-8", errors="replace") as f:
            text = f.read()
    except OSError:
        return None
    return parse(text, path)
