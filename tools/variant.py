"""Build diagnostic variants of libsacenv.so from text substitutions (A/B timing only).

    python tools/variant.py name 'old text' 'new text' ['old2' 'new2' ...]
    python tools/variant.py name --src FILE     (a whole sacenv_boat.hip)
    python tools/variant.py name --file sacenv_sac.hip 'old' 'new' ...   (another source)

Copies the sources to a temp dir, applies the substitutions to sacenv_boat.hip
(each must match exactly once), and builds sac-agent_amd/build/libsacenv_<name>.so.
The product sources carry no switches; variants exist only as these builds, loaded
through SACENV_LIB (never by the product path, whose library is digest-checked).
"""
import os
import shutil
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import __graft_entry__ as g  # noqa: E402


def main(argv):
    name, subs = argv[0], argv[1:]
    src, target = None, "sacenv_boat.hip"
    if subs[:1] == ["--file"]:   # the source the substitutions apply to (default sacenv_boat.hip)
        target, subs = subs[1], subs[2:]
    if subs[:1] == ["--src"]:
        src, subs = subs[1], subs[2:]
    if len(subs) % 2:
        raise SystemExit("substitutions come in pairs")
    with tempfile.TemporaryDirectory() as d:
        for f in g.SOURCES + ["mt19937.h"]:
            shutil.copy(os.path.join(g.CSRC, f), d)
        p = os.path.join(d, target)
        s = open(src or p).read()
        for a, b in zip(subs[::2], subs[1::2]):
            if s.count(a) != 1:
                raise SystemExit(f"substitution matches {s.count(a)} times: {a!r}")
            s = s.replace(a, b)
        open(p, "w").write(s)
        out = os.path.join(g.BUILD, f"libsacenv_{name}.so")
        extra = os.environ.get("EXTRA_FLAGS", "").split()
        subprocess.run([g._hipcc(), *g.HIPCC_FLAGS, *extra, "-I", os.path.join(ROOT, "include"),
                        *[os.path.join(d, f) for f in g.SOURCES], "-o", out], check=True)
    print("built", out)


if __name__ == "__main__":
    main(sys.argv[1:])
