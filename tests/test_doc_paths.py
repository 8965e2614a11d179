"""Every profiles/ path DESIGN.md and README.md cite exists in the tree (evidence hygiene).

A cited directory must exist and hold something; a cited file must exist; a glob (`*`) must match at least one
file.  Template paths (`<name>`) are skipped.
"""
import glob
import os
import re

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
DOCS = ["DESIGN.md", "README.md", "INTEGRATION.md"]
PAT = re.compile(r"profiles/[A-Za-z0-9_.*/+-]+")


def cited():
    out = set()
    for d in DOCS:
        p = os.path.join(ROOT, d)
        if not os.path.exists(p):
            continue
        with open(p) as f:
            text = f.read()
        for m in PAT.finditer(text):
            path = m.group(0).rstrip(".,;:)")
            if "<" in text[m.end():m.end() + 1]:  # profiles/r02/prof/<name>/...: a template
                continue
            out.add((d, path))
    return sorted(out)


@pytest.mark.parametrize("doc,path", cited(), ids=[p for _, p in cited()])
def test_cited_profile_path_exists(doc, path):
    full = os.path.join(ROOT, path)
    if "*" in path:
        assert glob.glob(full), "%s cites %s: no file matches" % (doc, path)
    elif path.endswith("/"):
        assert os.path.isdir(full) and os.listdir(full), "%s cites %s: no such directory" % (doc, path)
    else:
        assert os.path.exists(full), "%s cites %s: missing" % (doc, path)


def test_some_paths_are_cited():
    assert len(cited()) > 20
