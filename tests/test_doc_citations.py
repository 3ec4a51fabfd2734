"""Every ``file:line`` a document cites must exist (a stale ``kube.cc:467``), and
every file of evidence under ``profiles/`` must be cited (248 files, most cited by
nothing but an index).

The reference is read-only (/root/reference), so citations of it keep their line numbers: each
cited line (or range end) must exist in the cited reference file. This repository's own files
move, so ``docs/*.md`` cite them by symbol (`` `path` `Symbol` ``) instead of by line: no repo
source may be cited by line there, and every cited symbol must still be in its file. Files of
upstream libraries that are in neither tree (client-go's ``client_config.go``) are named as such
and skipped.
"""
import os
import re

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
REF = "/root/reference"
DOCS = [os.path.join(ROOT, "docs", f) for f in sorted(os.listdir(os.path.join(ROOT, "docs"))) if f.endswith(".md")]
DOCS += [os.path.join(ROOT, "README.md")]
# the documents whose citations keep a profile (docs/HISTORY.md narrates past rounds and may name
# files pruned since: they are in the git history)
CURRENT = [os.path.join(ROOT, "README.md")] + [os.path.join(ROOT, "docs", f) for f in
                                               ("DESIGN.md", "OPERATIONS.md", "PARITY_MATRIX.md")]
UPSTREAM = {"client_config.go"}  # client-go v0.19: not vendored by the reference
CITE = re.compile(r"((?:/root/reference/)?[A-Za-z0-9_./-]+\.(?:py|cc|h|hip|go|mod|sh|toml|ya?ml)):"
                  r"(\d+(?:-\d+)?(?:,\d+(?:-\d+)?)*)")
SYMBOL = re.compile(r"`((?:csrc|kube_sqs_autoscaler_amd|scripts|tests)/[A-Za-z0-9_./-]+\.(?:py|cc|h|hip))`\s+`([A-Za-z_][\w:~]*)`")


def _files(base):
    out = {}
    for d, _, fs in os.walk(base):
        if "/.git" in d or "__pycache__" in d or "/build" in d:
            continue
        for f in fs:
            out.setdefault(f, []).append(os.path.join(d, f))
    return out


def _lines(path):
    with open(path, errors="replace") as f:
        return sum(1 for _ in f)


def _resolve(cited):
    """(where, [candidate paths]): the reference for /root/reference paths and for names found
    only there; this repo for its own paths."""
    if cited.startswith(REF + "/"):
        return "reference", [cited]
    repo = os.path.join(ROOT, cited)
    if os.path.exists(repo):
        return "repo", [repo]
    ref = os.path.join(REF, cited)
    if os.path.exists(ref):
        return "reference", [ref]
    base = os.path.basename(cited)
    refs = [p for p in _files(REF).get(base, []) if p.endswith(cited)] if os.path.isdir(REF) else []
    if refs:
        return "reference", refs
    repos = [p for p in _files(ROOT).get(base, []) if p.endswith(cited)]
    return ("repo", repos) if repos else ("missing", [])


def _citations():
    for doc in DOCS:
        with open(doc) as f:
            text = f.read()
        for m in CITE.finditer(text):
            yield doc, m.group(1), m.group(2)


def test_docs_cite_at_least_the_reference():
    assert sum(1 for _ in _citations()) >= 20


@pytest.mark.skipif(not os.path.isdir(REF), reason="the reference tree is not on this machine")
def test_every_cited_line_exists():
    bad = []
    for doc, cited, spec in _citations():
        if os.path.basename(cited) in UPSTREAM:
            continue
        where, paths = _resolve(cited)
        if where == "missing":
            bad.append(f"{os.path.relpath(doc, ROOT)}: {cited}:{spec}: no such file")
            continue
        last = max(int(part.split("-")[-1]) for part in spec.split(","))
        if not any(_lines(p) >= last for p in paths):
            bad.append(f"{os.path.relpath(doc, ROOT)}: {cited}:{spec}: past the end ({paths[0]})")
    assert not bad, "\n".join(bad)


def test_docs_cite_this_repo_by_symbol_not_line():
    bad = []
    for doc, cited, spec in _citations():
        if not doc.startswith(os.path.join(ROOT, "docs")) or os.path.basename(cited) in UPSTREAM:
            continue
        if cited.startswith(REF) or _resolve(cited)[0] != "repo":
            continue
        bad.append(f"{os.path.relpath(doc, ROOT)}: {cited}:{spec} (cite `{cited}` `Symbol` instead)")
    assert not bad, "\n".join(bad)


def test_cited_symbols_exist():
    seen, bad = 0, []
    for doc in DOCS:
        with open(doc) as f:
            text = f.read()
        for m in SYMBOL.finditer(text):
            path, sym = os.path.join(ROOT, m.group(1)), m.group(2)
            seen += 1
            if not os.path.exists(path):
                bad.append(f"{m.group(1)}: no such file")
                continue
            with open(path) as f:
                src = f.read()
            name = sym.split("::")[-1]
            if sym not in src and not re.search(r"\b" + re.escape(name) + r"\b", src):
                bad.append(f"{os.path.relpath(doc, ROOT)}: `{m.group(1)}` `{sym}` not found")
    assert seen >= 8 and not bad, "\n".join(bad)


def _tracked_profiles():
    import subprocess

    try:
        out = subprocess.run(["git", "ls-files", "profiles"], cwd=ROOT, capture_output=True, text=True, check=True)
    except (OSError, subprocess.CalledProcessError):
        pytest.skip("not a git checkout")
    return [p for p in out.stdout.splitlines() if p]


def _current_text():
    text = ""
    for doc in CURRENT:
        with open(doc) as f:
            text += f.read() + "\n"
    return text


def _cites(text, entry):
    """``entry``: a profile's path under profiles/ -- ``file``, ``dir/file``, or ``dir/`` on its own
    (citing a directory cites every file in it; a file of it cites only itself)."""
    return re.search(r"(?<![\w-])" + re.escape(entry) + r"(?![\w.-])", text)


def test_every_profile_is_cited():
    """A file under profiles/ that README.md, DESIGN, OPERATIONS or PARITY_MATRIX does not cite
    (by its path, or its directory's) is not evidence of anything: prune it."""
    text = _current_text()
    bad = []
    for path in _tracked_profiles():
        rel = path[len("profiles/"):]
        top = rel.split("/", 1)[0]
        entries = [rel] + ([top + "/"] if "/" in rel else [])
        if not any(_cites(text, e) for e in entries):
            bad.append(path)
    assert not bad, "uncited profiles (cite them or delete them):\n" + "\n".join(bad)


def test_cited_profiles_exist():
    """Every ``profiles/<entry>`` the current documents cite is in the tree (``<rev>:profiles/...``
    names a file in the git history instead)."""
    text = _current_text()
    bad = sorted({m.group(1) for m in re.finditer(r"(?<![:\w])profiles/([A-Za-z0-9_.-]+/?(?:[A-Za-z0-9_.-]+)?)", text)
                  if not os.path.exists(os.path.join(ROOT, "profiles", m.group(1).rstrip("/")))})
    assert not bad, bad


def test_readme_is_the_operators_view():
    """README.md stays what an operator switching from the reference needs (65 KB of
    round diaries); the narration lives in docs/HISTORY.md."""
    with open(os.path.join(ROOT, "README.md"), "rb") as f:
        body = f.read()
    assert len(body) < 20 * 1024, len(body)
    text = body.decode()
    for section in ("## Switching from the reference", "### Flags", "### Deliberate deviations", "## Performance",
                    "## Known limits"):
        assert section in text, section
    assert "in brief" not in text
