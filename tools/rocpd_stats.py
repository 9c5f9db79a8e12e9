"""Per-kernel duration summary of a rocprofv3 rocpd database (the default output
format of rocprofv3 --kernel-trace on this image): name, calls, total/avg/median us."""
import sqlite3
import statistics
import sys


def main(path, out=None):
    c = sqlite3.connect(path)
    cols = [r[1] for r in c.execute("pragma table_info(kernels)")]
    name = "name" if "name" in cols else "kernel_name"
    rows = c.execute(f"select {name}, start, end from kernels").fetchall()
    by = {}
    for n, s, e in rows:
        by.setdefault(n, []).append((e - s) / 1e3)
    lines = ["kernel,calls,total_us,avg_us,median_us,min_us,max_us"]
    for n, d in sorted(by.items(), key=lambda kv: -sum(kv[1])):
        short = n.replace("(anonymous namespace)::", "").split("(")[0][:90].replace(",", ";")
        lines.append(f"{short},{len(d)},{sum(d):.1f},{sum(d)/len(d):.3f},{statistics.median(d):.3f},"
                     f"{min(d):.3f},{max(d):.3f}")
    txt = "\n".join(lines)
    if out:
        open(out, "w").write(txt + "\n")
    print(txt)


if __name__ == "__main__":
    main(*sys.argv[1:])
