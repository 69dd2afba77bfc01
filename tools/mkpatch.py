#!/usr/bin/env python3
"""Write an A/B patch against the working tree without touching it (tools only).

  python tools/mkpatch.py NAME FILE PYTHON_EXPR [FILE PYTHON_EXPR ...]

Each PYTHON_EXPR edits the string `s` (the file's current text); the unified
diff of the edited copies goes to tools/patches/NAME.patch, for
tools/build_variant.sh.  The working tree is never modified.
"""
import os
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
name, rest = sys.argv[1], sys.argv[2:]
out = []
for f, expr in zip(rest[0::2], rest[1::2]):
    s = open(os.path.join(ROOT, f)).read()
    orig = s
    exec(expr)
    if s == orig:
        sys.exit(f"{f}: the edit changed nothing")
    with tempfile.NamedTemporaryFile("w", suffix=os.path.basename(f), delete=False) as t:
        t.write(s)
    d = subprocess.run(["git", "diff", "--no-index", "--", os.path.join(ROOT, f), t.name], capture_output=True,
                       text=True).stdout
    os.unlink(t.name)
    lines = d.splitlines(keepends=True)
    hdr = [f"diff --git a/{f} b/{f}\n", f"--- a/{f}\n", f"+++ b/{f}\n"]
    body = [ln for ln in lines if not ln.startswith(("diff --git", "index ", "--- ", "+++ "))]
    out += hdr + body
open(os.path.join(ROOT, "tools/patches", name + ".patch"), "w").write("".join(out))
print("tools/patches/" + name + ".patch")
