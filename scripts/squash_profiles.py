"""Squash superseded profile sessions into one text file each.

    python scripts/squash_profiles.py DIR...   (directories under profiles/)

profiles/archive/<name>.txt keeps, per file of the session: text summaries
(*.txt, *.md) whole, logs reduced to their JSON lines (a bench line, a
host-rate line) plus their last 3 lines, small JSON files whole, and
rocprofv3 *_stats.csv summaries whole; raw traces and counter dumps are
dropped. The directory is then removed (git rm) by the caller.
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PROF = os.path.join(ROOT, "profiles")


def squash(name):
    src = os.path.join(PROF, name)
    out = [f"# profiles/{name} (squashed: summaries and result lines of the session's files)\n"]
    for dp, _, fs in sorted(os.walk(src)):
        for f in sorted(fs):
            p = os.path.join(dp, f)
            rel = os.path.relpath(p, src)
            try:
                text = open(p, errors="replace").read()
            except Exception:
                continue
            keep = None
            if f.endswith((".txt", ".md")):
                keep = text
            elif f.endswith(".json") and len(text) < 20000:
                keep = text
            elif f.endswith("_stats.csv"):
                keep = text
            elif f.endswith((".log", ".jsonl", ".out")):
                lines = text.splitlines()
                js = [ln for ln in lines if ln.lstrip().startswith("{")]
                keep = "\n".join(js + ["..."] + lines[-3:]) if js else "\n".join(lines[-3:])
            if keep is not None:
                out.append(f"\n=== {rel} ===\n{keep.rstrip()}\n")
    os.makedirs(os.path.join(PROF, "archive"), exist_ok=True)
    with open(os.path.join(PROF, "archive", name + ".txt"), "w") as fh:
        fh.write("".join(out))


if __name__ == "__main__":
    for n in sys.argv[1:]:
        squash(n.rstrip("/").split("/")[-1])
