"""Instruction mix of the bench's segment-kernel loop (k_rollout<2, true, false>).

Compiles sacenv_boat.hip to gfx950 assembly (or reads --asm FILE), takes the
kernel's open-loop body (the back-edge span that contains no flag spin) and
prints the opcode histogram by class: the single owner wave per SIMD is
issue-bound (~4-5 cycles per instruction of any class, f64 FMA dependent
latency ~5.7 cycles: tools/ubench/f64_latency.hip), so instruction count is
the lever.
"""
import collections
import os
import re
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def asm_text(src=None):
    import __graft_entry__ as g
    src = src or os.path.join(g.CSRC, "sacenv_boat.hip")
    out = os.path.join(tempfile.gettempdir(), "sacenv_boat_isa.s")
    flags = [f for f in g.HIPCC_FLAGS if f not in ("-shared", "-fPIC")]
    subprocess.run([g._hipcc(), *flags, "--cuda-device-only", "-S", "-I", os.path.join(ROOT, "include"),
                    "-I", g.CSRC, src, "-o", out], check=True, stderr=subprocess.DEVNULL)
    return open(out).read()


def kernel(text, name="k_rolloutILi2ELb1ELi0E"):
    lines = text.split("\n")
    start = next(i for i, l in enumerate(lines) if re.match(r"^_Z\w*%s\w*:" % name, l))
    end = next(i for i in range(start, len(lines)) if lines[i].startswith(".Lfunc_end"))
    return lines[start:end]


def loops(lines):
    labels = {m.group(1): i for i, l in enumerate(lines) if (m := re.match(r"^(\.LBB\d+_\d+):", l))}
    out = []
    for i, l in enumerate(lines):
        m = re.search(r"(s_cbranch_\w+|s_branch)\s+(\.LBB\d+_\d+)", l)
        if m and labels.get(m.group(2), 1 << 30) < i:
            out.append((labels[m.group(2)], i))
    return out


def hist(body):
    c = collections.Counter()
    for l in body:
        l = l.strip()
        if not l or l[0] in ";." or l.endswith(":"):
            continue
        c[l.split()[0]] += 1
    return c


def main():
    text = open(sys.argv[sys.argv.index("--asm") + 1]).read() if "--asm" in sys.argv else asm_text()
    k = kernel(text)
    meta = [l.strip() for l in text.split("\n") if re.search(r"\.(vgpr|sgpr|agpr)_count|vgpr_spill|sgpr_spill", l)]
    # outermost loops without a flag spin (s_sleep) = the open loop
    cands = [(a, b) for a, b in loops(k) if b - a > 500 and not any("s_sleep" in x for x in k[a:b])]
    a, b = max(cands, key=lambda ab: ab[1] - ab[0])
    h = hist(k[a:b + 1])
    cls = collections.Counter()
    for op, n in h.items():
        key = ("valu_f64" if re.search(r"_f64|_b64|_i64|_u64", op) and op.startswith("v_") else
               "valu" if op.startswith("v_") else "salu_mov" if op.startswith("s_mov") else
               "branch" if "branch" in op else "wait" if op.startswith("s_waitcnt") or op.startswith("s_nop") else
               "smem" if op.startswith("s_load") or op.startswith("s_buffer") else
               "salu" if op.startswith("s_") else "mem")
        cls[key] += n
    print(f"open loop: lines {a}..{b} ({b - a} lines)")
    print("classes:", dict(cls), "total", sum(cls.values()))
    for op, n in h.most_common(40):
        print(f"  {op:28s} {n}")


if __name__ == "__main__":
    main()


def blocks(lines, a, b):
    """Per basic block of lines[a..b]: label, counts by class, exit branch."""
    out, cur = [], None
    for i in range(a, b + 1):
        l = lines[i].strip()
        m = re.match(r"^(\.LBB\d+_\d+):", l)
        if m or cur is None:
            cur = {"label": m.group(1) if m else "(entry)", "line": i, "ops": collections.Counter(), "exit": ""}
            out.append(cur)
            if m:
                continue
        if not l or l[0] in ";." or l.endswith(":"):
            continue
        op = l.split()[0]
        cur["ops"][op] += 1
        if "branch" in op:
            cur["exit"] = l
            cur = {"label": "(fall)", "line": i + 1, "ops": collections.Counter(), "exit": ""}
            out.append(cur)
    return [x for x in out if x["ops"]]


def show_blocks(lines, a, b):
    for x in blocks(lines, a, b):
        o = x["ops"]
        v = sum(n for k, n in o.items() if k.startswith("v_"))
        s = sum(n for k, n in o.items() if k.startswith("s_") and "branch" not in k and "waitcnt" not in k)
        m = sum(n for k, n in o.items() if not k.startswith("v_") and not k.startswith("s_"))
        slow = " SLOW" if any(k in o for k in ("v_trig_preop_f64", "v_ldexp_f64", "v_frexp_mant_f64")) else ""
        print(f"{x['line']:5d} {x['label']:12s} v{v:4d} s{s:4d} m{m:3d}{slow}  {x['exit'][:60]}")
