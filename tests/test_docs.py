"""Every profiles/... path DESIGN.md, README.md, INTEGRATION.md and
profiles/README.md cite exists in the tree (a file, a directory, or -- for a
glob or a {a,b} list -- at least one match of each), so the evidence the
documents point at is the evidence committed."""
import glob
import os
import re

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
DOCS = ["DESIGN.md", "README.md", "INTEGRATION.md", os.path.join("profiles", "README.md")]
PAT = re.compile(r"profiles/[A-Za-z0-9_.*/{},-]+")


def expand(p):
    m = re.search(r"\{([^{}]*)\}", p)
    if not m:
        return [p]
    out = []
    for alt in m.group(1).split(","):
        out += expand(p[:m.start()] + alt + p[m.end():])
    return out


def cited(doc):
    with open(os.path.join(ROOT, doc)) as f:
        text = f.read()
    for m in PAT.finditer(text):
        p = m.group(0).rstrip(".,;:)`'/")
        if p.count("{") != p.count("}"):
            p = p[:p.index("{")] if "{" in p else p
        yield p


@pytest.mark.parametrize("doc", DOCS)
def test_cited_profiles_exist(doc):
    if not os.path.exists(os.path.join(ROOT, doc)):
        pytest.skip(f"{doc} absent")
    missing = []
    for p in set(cited(doc)):
        for q in expand(p):
            if not glob.glob(os.path.join(ROOT, q)):
                missing.append(q)
    assert not missing, f"{doc} cites paths that do not exist: {sorted(missing)}"
