"""Provenance stamps for measured profiles.

A profile under ``profiles/`` (HBM traffic per cell, counter passes) is only
valid for the engine sources it was measured on.  ``source_hash()`` hashes
the files the measured kernels' behaviour depends on (kernels, packing and
dispatch, example builder); measurement tools write it into the profile, and
``bench.py`` marks a profile ``stale`` when it differs from the tree it runs
on.  The GPU box receives no ``.git``, so the hash (not the git head) is the
check; the git head is recorded beside it when known (``SK_GIT_HEAD``)."""
from __future__ import annotations

import hashlib
import os

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
# what the measured kernels' traffic depends on: the kernels, the packing and
# dispatch (sk_api.cpp), the example builder and synthetic inputs
_SRC_DIRS = ("stem_kernel_amd/csrc/kernels",)
_SRC_FILES = ("stem_kernel_amd/csrc/sk_api.cpp", "stem_kernel_amd/csrc/host/example_build.cpp",
              "stem_kernel_amd/csrc/host/synth.cpp", "stem_kernel_amd/csrc/host/sk_internal.h",
              "stem_kernel_amd/csrc/ribosum85_60.inc")
_EXT = (".hip", ".cpp", ".h", ".inc")


def source_files(root: str = ROOT) -> list:
    out = []
    for d in _SRC_DIRS:
        for base, _, files in os.walk(os.path.join(root, d)):
            for f in files:
                if f.endswith(_EXT):
                    out.append(os.path.relpath(os.path.join(base, f), root))
    out.extend(f for f in _SRC_FILES if os.path.exists(os.path.join(root, f)))
    return sorted(out)


def source_hash(root: str = ROOT) -> str:
    h = hashlib.sha256()
    for rel in source_files(root):
        h.update(rel.encode() + b"\0")
        with open(os.path.join(root, rel), "rb") as f:
            h.update(f.read())
        h.update(b"\0")
    return h.hexdigest()[:16]


def git_head(root: str = ROOT):
    env = os.environ.get("SK_GIT_HEAD")
    if env:
        return env
    try:
        import subprocess
        return subprocess.run(["git", "-C", root, "rev-parse", "--short", "HEAD"], capture_output=True,
                              text=True, timeout=10).stdout.strip() or None
    except Exception:
        return None


def stamp() -> dict:
    return {"source_hash": source_hash(), "git_head": git_head()}
