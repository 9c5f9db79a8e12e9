"""Reduce tools/pmc.sh's rocprofv3 output to per-launch figures for k_step.

Writes gpurun_out/pmc_k_step.json: mean duration from the kernel trace, and
per-launch FETCH_SIZE / WRITE_SIZE / TCC hit rate from the PMC passes. HBM
bytes follow MI355X_MICROARCH.md's HBM section: FETCH_SIZE (reported in KB)
is doubled on gfx950 (128-B requests tallied at 64 B), WRITE_SIZE taken as is.
"""
import csv
import glob
import json
import os
import sys

KERNEL = "k_step"


def rows(pattern):
    out = []
    for f in glob.glob(pattern, recursive=True):
        with open(f) as fh:
            out += list(csv.DictReader(fh))
    return out


def main(out_dir):
    res = {"kernel": KERNEL}
    st = [r for r in rows(os.path.join(out_dir, "prof_trace", "**", "*kernel_stats.csv"))
          if KERNEL in r.get("Name", "")]
    if st:
        r = st[0]
        res["trace_calls"] = int(r["Calls"])
        res["trace_avg_ns"] = float(r["AverageNs"])
        res["trace_min_ns"] = float(r.get("MinNs", "nan"))
        res["trace_max_ns"] = float(r.get("MaxNs", "nan"))
    for i in (1, 2, 3):
        rr = [r for r in rows(os.path.join(out_dir, f"prof_pmc{i}", "**", "*counter_collection.csv"))
              if KERNEL in r.get("Kernel_Name", "")]
        by = {}
        for r in rr:
            by.setdefault(r["Counter_Name"], []).append(float(r["Counter_Value"]))
        for name, v in by.items():
            res[name + "_mean"] = sum(v) / len(v)
            res[name + "_n"] = len(v)
    bench = os.path.join(out_dir, "prof_trace_bench.json")
    if os.path.exists(bench):
        d = json.loads(open(bench).read().strip().splitlines()[-1])
        res["envs"] = d["config"]["envs_per_gpu"]
        res["experiment"] = d["config"]["experiment"]
        res["bench_kernel_avg_us"] = d["roofline"]["kernel_avg_us"]
        res["algorithmic_bytes_per_launch"] = d["roofline"]["bytes_per_launch"]
    if "FETCH_SIZE_mean" in res and "WRITE_SIZE_mean" in res:
        fetch = 2.0 * res["FETCH_SIZE_mean"] * 1024.0
        write = res["WRITE_SIZE_mean"] * 1024.0
        res["hbm_fetch_bytes_per_launch"] = fetch
        res["hbm_write_bytes_per_launch"] = write
        res["hbm_bytes_per_launch"] = fetch + write
    if "TCC_HIT_sum_mean" in res:
        h, m = res["TCC_HIT_sum_mean"], res.get("TCC_MISS_sum_mean", 0.0)
        res["l2_hit_rate"] = h / (h + m) if h + m else None
    json.dump(res, open(os.path.join(out_dir, "pmc_k_step.json"), "w"), indent=1)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else "gpurun_out")
