"""What libsacenv.so is built from: sources, flags and their content digest.

``__graft_entry__.build()`` compiles the library and writes the digest next to
it (``libsacenv.so.sha256``); ``_lib.load()`` recomputes it from the sources in
the tree and refuses a library whose stamp does not match, so a loaded library
is always the one these sources compile to (no stale prebuilt binary).
"""
from __future__ import annotations

import hashlib
import os

PKG_ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))   # .../sac-agent_amd
REPO_ROOT = os.path.dirname(PKG_ROOT)
CSRC = os.path.join(PKG_ROOT, "csrc")
INCLUDE = os.path.join(REPO_ROOT, "include")
BUILD = os.path.join(PKG_ROOT, "build")
LIB = os.path.join(BUILD, "libsacenv.so")
SOURCES = ("sacenv_boat.hip", "sacenv_replay.hip", "sacenv_sac.hip")
HEADERS = ("mt19937.h",)
HIPCC_FLAGS = ("--offload-arch=gfx950", "-O3", "-std=c++17", "-ffp-contract=off",
               "-fPIC", "-shared", "-Wall")


def deps() -> list[tuple[str, str]]:
    """(path relative to the repo root, absolute path) of every input file."""
    rel = [os.path.join("sac-agent_amd", "csrc", f) for f in SOURCES + HEADERS]
    rel.append(os.path.join("include", "sacenv.h"))
    return [(r, os.path.join(REPO_ROOT, r)) for r in rel]


def source_digest(extra_flags=()) -> str:
    """sha256 over the flags and every input's relative path and bytes (independent
    of where the tree lives: the GPU box runs it from another directory)."""
    h = hashlib.sha256(" ".join((*HIPCC_FLAGS, *extra_flags)).encode())
    for rel, path in deps():
        with open(path, "rb") as f:
            h.update(rel.encode() + b"\0" + f.read())
    return h.hexdigest()
