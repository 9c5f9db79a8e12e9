"""Build diagnostic variants of libsacenv.so for A/B timing (tools/ab.sh).

    python tools/build_variants.py name:-DFLAG[,-DFLAG2] ...

Writes sac-agent_amd/build/libsacenv_<name>.so. Variants are never loaded by
the product path (only via SACENV_LIB in tools/ab.sh).
"""
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import __graft_entry__ as g  # noqa: E402

PKG = os.path.join(ROOT, "sac-agent_amd")


def main(specs):
    srcs = [os.path.join(PKG, "csrc", f) for f in g.SOURCES]
    for spec in specs:
        name, _, flags = spec.partition(":")
        defs = [f for f in flags.split(",") if f]
        out = os.path.join(PKG, "build", f"libsacenv_{name}.so")
        subprocess.run([g._hipcc(), *g.HIPCC_FLAGS, *defs, "-I", os.path.join(ROOT, "include"),
                        *srcs, "-o", out], check=True)
        print("built", out, defs)


if __name__ == "__main__":
    main(sys.argv[1:])
