"""The GPU box compiles the library from the HEAD sources, and that build behaves
as the shipped one.

The pool's rules keep built libraries in the pushed tree (they may not be listed in
.gpurunignore), so the round-end tests load the library built in the container --
whose digest `_lib.load()` checks against the sources in the tree. This test closes
the rest: it runs hipcc on THIS box over the tree's sources with the library's own
flags (`sacenv._build`), then drives the same short workload -- init, two 64-step
persistent segments with auto-reset and a refill, a pooled step -- through the
shipped and the freshly built library in separate processes, and asserts identical
arenas (sha256 of every byte). Device code objects are not compared byte for byte:
the two builds differ in embedded paths and symbol order, not in behaviour.
"""
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "sac-agent_amd")

WORKLOAD = r"""
import hashlib, sys
import torch
sys.path.insert(0, sys.argv[1])
from sacenv import VecBoatEnv, _lib
N = 4096
env = VecBoatEnv({"base_settings": {"experiment": 6, "test_mode": 0}}, N, seed=11, device="cuda",
                 max_episode_steps=40, n_helpers=512, auto_refill=False)
env.reset()
g = torch.Generator(device="cuda"); g.manual_seed(3)
acts = torch.rand((129, N), device="cuda", generator=g) * 2 - 1
env.segment_async(acts, 64)
env.segment_async(acts[64:], 64)
env.refill()
row = torch.zeros(_lib.trans_bytes(6) * env.n_pad, dtype=torch.uint8, device="cuda")
env.step_pooled_async(acts[128].contiguous(), row)
torch.cuda.synchronize()
env.check_status()
h = hashlib.sha256(env.arena.cpu().numpy().tobytes())
h.update(row.cpu().numpy().tobytes())
print(h.hexdigest())
"""


def _run(lib_path):
    env = dict(os.environ)
    if lib_path is not None:
        env["SACENV_LIB"] = lib_path
    else:
        env.pop("SACENV_LIB", None)
    r = subprocess.run([sys.executable, "-c", WORKLOAD, PKG], env=env, capture_output=True, text=True,
                       timeout=240)
    assert r.returncode == 0, r.stderr[-2000:]
    return r.stdout.strip().splitlines()[-1]


def test_library_builds_on_this_box_and_matches_the_shipped_one(tmp_path, gpu, built_lib):
    sys.path.insert(0, PKG)
    from sacenv import _build
    import __graft_entry__ as g
    out = str(tmp_path / "libsacenv_box.so")
    cmd = [g._hipcc(), *_build.HIPCC_FLAGS, "-I", _build.INCLUDE,
           *[os.path.join(_build.CSRC, s) for s in _build.SOURCES], "-o", out]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=900)
    assert r.returncode == 0, r.stderr[-2000:]
    print(f"built {out} on this box from sources {_build.source_digest()[:16]}")
    shipped, fresh = _run(None), _run(out)
    print(f"arena digest: shipped {shipped[:16]}, box build {fresh[:16]}")
    assert shipped == fresh
