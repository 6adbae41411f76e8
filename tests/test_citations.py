"""The audit trail: every `File.java:N[-M]` citation in the product, oracle and test sources must
point at this reference snapshot (Weak #3: citations copied from upstream-microRTS line
numbers pointed past the end of files or at the wrong method).

Two checks, CPU-only, skipped where /root/reference is absent (the GPU box):
1. every cited file exists in the reference and every cited line range lies inside it;
2. where a citation directly follows a Java method name — `name (File.java:N-M)` — the range overlaps
   that method's body in the cited file.
"""
import collections
import glob
import os
import re
import subprocess

import pytest

REF = "/root/reference"
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CANONICAL = ("/src/tests/", "/src/rts/", "/src/ai/jni/", "/src/ai/reward/", "/src/util/", "/test/")
CITE = re.compile(r"((?:[\w.]+/)*)(\w+\.java):(\d+(?:-\d+)?(?:,\s?\d+(?:-\d+)?)*)")
# `Class.method (File.java:N-M)`: a method named with its class (or in backticks) right before it
CALLED = re.compile(r"(?:\.|`)([a-z]\w{3,})`?\s*\(\s*(?:[\w.]+/)*(\w+\.java):(\d+(?:-\d+)?(?:,\s?\d+(?:-\d+)?)*)")
DEF = re.compile(r"^\s*(?:public|private|protected|static|final|synchronized|abstract|\s)*[\w<>\[\],\s]+?\s(\w+)\s*\([^;]*$")

pytestmark = pytest.mark.skipif(not os.path.isdir(os.path.join(REF, "src")), reason="reference tree not present")


def _sources():
    out = subprocess.check_output(["git", "ls-files", "oracle", "microrts_amd", "include", "tests", "tools", "bench.py",
                                   "__graft_entry__.py", "DESIGN.md", "INTEGRATION.md", "README.md"], cwd=ROOT).decode()
    return [f for f in out.split() if f.endswith((".cpp", ".hpp", ".hip", ".h", ".py", ".md", ".sh"))]


def _index():
    idx = collections.defaultdict(list)
    for p in glob.glob(os.path.join(REF, "**", "*.java"), recursive=True):
        idx[os.path.basename(p)].append(p)
    return idx


def _resolve(idx, prefix, name):
    c = idx.get(name, [])
    if prefix:
        c = [p for p in c if p.endswith("/" + prefix + name)] or c
    if len(c) > 1:  # the three JNIGridnet* copies: the canonical src/tests one
        c = [p for p in c if any(k in p for k in CANONICAL)][:1] or c
    return c[0] if c else None


def _spans(text):
    for sp in text.split(","):
        a, _, b = sp.strip().partition("-")
        yield int(a), int(b) if b else int(a)


def _methods(path, cache={}):
    if path not in cache:
        lines = open(path, errors="replace").read().split("\n")
        out = collections.defaultdict(list)
        for i, line in enumerate(lines):
            m = DEF.match(line)
            if not m or m.group(1) in ("if", "for", "while", "switch", "catch", "return", "new"):
                continue
            depth, started, j = 0, False, i
            while j < len(lines):
                for ch in lines[j]:
                    depth += (ch == "{") - (ch == "}")
                    started = started or ch == "{"
                if (started and depth <= 0) or (not started and lines[j].rstrip().endswith(";")):
                    break
                j += 1
            out[m.group(1)].append((i + 1, j + 1))
        cache[path] = (out, len(lines) - (lines[-1] == ""))
    return cache[path]


def test_citations_point_into_the_reference():
    idx = _index()
    bad = []
    for f in _sources():
        for ln, line in enumerate(open(os.path.join(ROOT, f), errors="replace"), 1):
            for m in CITE.finditer(line):
                path = _resolve(idx, m.group(1), m.group(2))
                if path is None:
                    bad.append(f"{f}:{ln}: {m.group(0)}: no such reference file")
                    continue
                n = _methods(path)[1]
                for a, b in _spans(m.group(3)):
                    if a < 1 or b < a or b > n:
                        bad.append(f"{f}:{ln}: {m.group(0)}: {os.path.relpath(path, REF)} has {n} lines")
    assert not bad, "\n".join(bad)


def test_method_citations_cover_the_method():
    idx = _index()
    bad = []
    for f in _sources():
        for ln, line in enumerate(open(os.path.join(ROOT, f), errors="replace"), 1):
            for m in CALLED.finditer(line):
                path = _resolve(idx, "", m.group(2))
                if path is None:
                    continue
                defs = _methods(path)[0].get(m.group(1))
                if not defs:
                    continue  # not a method of that file (a word of prose)
                if not any(a <= e and b >= s for a, b in _spans(m.group(3)) for s, e in defs):
                    bad.append(f"{f}:{ln}: {m.group(1)} cited at {m.group(2)}:{m.group(3)}, defined at {defs}")
    assert not bad, "\n".join(bad)
