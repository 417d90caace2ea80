"""Which sources the in-tree librtamd.so was built from (verdict r3: the tested binary provably HEAD's).

`make` writes lib/librtamd.build.json after every link: the SHA-256 of the library, a SHA-256 over the
sources it is compiled from (csrc/*, include/rt.h), and the git HEAD of the checkout that built it.  The
GPU box receives the tree without .git, so what a test run can prove there is: the library it loads is
the one the stamp describes, and the stamp's sources are the sources in the tree it runs from
(tests/conftest.py checks both and prints them).

    python rtamd/provenance.py stamp     # after linking (csrc/Makefile)
    python rtamd/provenance.py check     # exit 1 when the library or the sources differ from the stamp
"""
from __future__ import annotations

import hashlib
import json
import os
import subprocess
import sys

PKG = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
REPO = os.path.dirname(PKG)
CSRC = os.path.join(PKG, "csrc")
LIB = os.path.join(PKG, "lib", "librtamd.so")
STAMP = os.path.join(PKG, "lib", "librtamd.build.json")
SOURCE_EXT = (".hip", ".cpp", ".hpp", ".h")


def source_files():
    files = [os.path.join(CSRC, f) for f in sorted(os.listdir(CSRC))
             if f.endswith(SOURCE_EXT) or f == "Makefile"]
    return files + [os.path.join(REPO, "include", "rt.h")]


def sources_sha256() -> str:
    h = hashlib.sha256()
    for p in source_files():
        h.update(os.path.relpath(p, REPO).encode() + b"\0")
        with open(p, "rb") as f:
            h.update(f.read())
        h.update(b"\0")
    return h.hexdigest()


def file_sha256(path: str) -> str:
    with open(path, "rb") as f:
        return hashlib.sha256(f.read()).hexdigest()


def git_head():
    try:
        head = subprocess.run(["git", "-C", REPO, "rev-parse", "HEAD"], capture_output=True, text=True,
                              timeout=10).stdout.strip() or None
        dirty = subprocess.run(["git", "-C", REPO, "status", "--porcelain", "--", "real-time-gpu-ray-tracer_amd/csrc",
                                "include"], capture_output=True, text=True, timeout=10).stdout.strip() != ""
        return head, dirty
    except (OSError, subprocess.SubprocessError):
        return None, None


def stamp() -> dict:
    head, dirty = git_head()
    d = {"lib_sha256": file_sha256(LIB), "sources_sha256": sources_sha256(),
         "git_head": head, "sources_dirty_at_build": dirty,
         "sources": [os.path.relpath(p, REPO) for p in source_files()]}
    with open(STAMP, "w") as f:
        json.dump(d, f, indent=1)
    return d


def check():
    """(ok, message): the loaded library is the stamped one, and the stamp's sources are the tree's."""
    if not os.path.exists(STAMP):
        return False, f"no build stamp {os.path.relpath(STAMP, REPO)} (run make in csrc)"
    with open(STAMP) as f:
        d = json.load(f)
    lib = file_sha256(LIB)
    src = sources_sha256()
    msg = (f"librtamd.so sha16 {lib[:16]}, sources sha16 {src[:16]}, built at git HEAD {d.get('git_head')}"
           f"{' (+uncommitted source changes)' if d.get('sources_dirty_at_build') else ''}")
    if lib != d.get("lib_sha256"):
        return False, f"library {lib[:16]} is not the stamped build {d.get('lib_sha256', '')[:16]}; {msg}"
    if src != d.get("sources_sha256"):
        return False, f"sources {src[:16]} differ from the ones the library was built from {d.get('sources_sha256', '')[:16]}"
    return True, msg


if __name__ == "__main__":
    cmd = sys.argv[1] if len(sys.argv) > 1 else "check"
    if cmd == "stamp":
        d = stamp()
        print(f"stamped {os.path.relpath(STAMP, REPO)}: lib {d['lib_sha256'][:16]} sources {d['sources_sha256'][:16]} "
              f"HEAD {d['git_head']}")
    else:
        ok, m = check()
        print(m)
        sys.exit(0 if ok else 1)
