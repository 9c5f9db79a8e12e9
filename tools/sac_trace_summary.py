"""Per-launch durations of the SAC kernels from a rocprofv3 kernel-trace CSV (grid size tells the phase)."""
import csv
import statistics
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
by = {}
for r in rows:
    name = r["Kernel_Name"]
    if "k_sac" not in name:
        continue
    key = (name.split("(")[0].split("::")[-1], int(r["Grid_Size_X"] if "Grid_Size_X" in r else r["Grid_Size"]))
    by.setdefault(key, []).append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
for k, v in sorted(by.items()):
    print(f"{k[0]:18s} grid {k[1]:8d} calls {len(v):4d} median {statistics.median(v):8.2f} us min {min(v):8.2f}")
