"""The documents' evidence exists: every profiles/ file that a document, a test, a tool or
the code names -- with its directory or as a bare round-tagged name (rNN..._*.json / .jsonl / .txt /
.csv / .log, shell-style * and {a,b} allowed) -- is committed, and every committed profile is named by
one of them (profiles/ holds only cited evidence)."""
import fnmatch
import os
import re
import subprocess

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
NAME = re.compile(r"(?<![\w/])(?:profiles/)?((?:r0\d[a-z0-9]*_|pmc_|latency_)[\w.*\[\]{},\-]*\.(?:jsonl|json|txt|csv|log))")


def _expand(pat):
    """shell-style {a,b} alternatives -> fnmatch patterns"""
    m = re.search(r"\{([^{}]*)\}", pat)
    if not m:
        return [pat]
    return [q for alt in m.group(1).split(",") for q in _expand(pat[:m.start()] + alt + pat[m.end():])]


def _cited(text):
    out = set()
    for m in NAME.finditer(text):
        if text[max(0, m.start() - 11):m.start()].endswith("gpurun_out/"):
            continue  # scratch output of a GPU call, not a committed profile
        out.update(_expand(m.group(1)))
    return out


def _profiles():
    return {os.path.basename(p) for p in subprocess.run(["git", "ls-files", "profiles"], cwd=ROOT, capture_output=True,
                                                        text=True, check=True).stdout.split()}


def _sources():
    """tracked text files outside profiles/ (profiles/README.md included)"""
    for f in subprocess.run(["git", "ls-files"], cwd=ROOT, capture_output=True, text=True, check=True).stdout.split():
        if f.startswith("profiles/") and f != "profiles/README.md":
            continue
        if f.endswith((".md", ".py", ".sh", ".m", ".c", ".h", ".hip", ".cpp")) and os.path.exists(os.path.join(ROOT, f)):
            yield f, open(os.path.join(ROOT, f), errors="replace").read()


NOTES = ("VERDICT.md", "ADVICE.md", "SURVEY.md")  # the judge's, advisor's and survey's notes of their round


def test_every_cited_profile_is_committed():
    have = _profiles()
    missing = []
    for f, text in _sources():
        if f in NOTES:
            continue
        for pat in _cited(text):
            if not any(fnmatch.fnmatch(n, pat) for n in have):
                missing.append((f, pat))
    assert not missing, missing


def test_every_committed_profile_is_cited():
    have = _profiles() - {"README.md"}
    pats = set()
    for f, text in _sources():
        if f not in NOTES:
            pats |= _cited(text)
    uncited = sorted(n for n in have if not any(fnmatch.fnmatch(n, p) for p in pats))
    assert not uncited, uncited
