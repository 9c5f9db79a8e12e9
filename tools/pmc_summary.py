"""Reduce tools/pmc.sh's rocprofv3 output to per-launch figures for the bench kernel.

Mode "step": k_step, gpurun_out/pmc_k_step.json. Mode "segment": the persistent
k_rollout of sacenv_boat_segment (bench.SEG = 256 steps per launch), gpurun_out/pmc_segment.json,
with the per-launch figures also divided into per-step ones. Mode "rollout": the same
kernel under bench --rollout 256 (every step's record to its own rows), gpurun_out/pmc_rollout.json.
Each holds:
* the kernel trace's mean duration;
* per-launch counter means for the kernel and for the calibration kernels of
  tools/probes/fetch_calib (k_calib8: k_step's 8-B/lane access pattern with
  known bytes: 10 485 760 read, 7 864 320 written per launch);
* HBM-side bytes per launch from the read requests split by size
  (32 x RDREQ_32B + 64 x RDREQ_64B + 128 x RDREQ_128B) and from WRITE_SIZE,
  each scaled by the calibration kernel's known/measured ratio, next to the
  guide's FETCH_SIZE x 2 convention (MI355X_MICROARCH.md, HBM section).
"""
import csv
import glob
import json
import os
import sys

KERNEL = "k_step"
STEPS_PER_LAUNCH = 1
MODE = "k_step"
CALIB = {"k_calib8": (10485760.0, 7864320.0), "k_calib16": (10485760.0, 7864320.0)}


def rows(pattern):
    out = []
    for f in glob.glob(pattern, recursive=True):
        with open(f) as fh:
            out += list(csv.DictReader(fh))
    return out


def means(prefix, out_dir, name):
    by = {}
    for d in sorted(glob.glob(os.path.join(out_dir, prefix + "*"))):
        for r in rows(os.path.join(d, "**", "*counter_collection.csv")):
            kn = r.get("Kernel_Name", "")
            if name in kn and (name != "k_step" or "k_step<false" in kn or "k_stepILb0E" in kn):
                by.setdefault(r["Counter_Name"], []).append(float(r["Counter_Value"]))
    if STEPS_PER_LAUNCH > 1 and name == KERNEL:
        # full-length launches only: the bench's first launch runs a few steps, and
        # averaging it in understated every per-step figure by ~8 % (rounds 3-4)
        by = {k: [x for x in v if x >= 0.25 * max(v)] for k, v in by.items()}
    return {k: sum(v) / len(v) for k, v in by.items()}


def read_bytes(m):
    if "TCC_EA0_RDREQ_128B_sum" not in m:
        return None
    return (128 * m["TCC_EA0_RDREQ_128B_sum"] + 64 * m.get("TCC_EA0_RDREQ_64B_sum", 0.0)
            + 32 * m.get("TCC_EA0_RDREQ_32B_sum", 0.0))


def main(out_dir):
    res = {"kernel": KERNEL}
    st = [r for r in rows(os.path.join(out_dir, "prof_trace", "**", "*kernel_stats.csv"))
          if KERNEL in r.get("Name", "") and "k_step<true" not in r.get("Name", "")
          and "k_stepILb1E" not in r.get("Name", "")]
    if st:
        r = max(st, key=lambda x: int(x["Calls"]))
        res.update(trace_kernel=r["Name"], trace_calls=int(r["Calls"]), trace_avg_ns=float(r["AverageNs"]),
                   trace_min_ns=float(r.get("MinNs", "nan")), trace_max_ns=float(r.get("MaxNs", "nan")))
    k = means("prof_pmc", out_dir, KERNEL)
    res["counters_per_launch"] = k
    cal = {n: means("calib_pmc", out_dir, n) for n in CALIB}
    res["calibration"] = {}
    for n, (rb, wb) in CALIB.items():
        m = cal[n]
        rd = read_bytes(m)
        wr = m.get("WRITE_SIZE", 0.0) * 1024.0
        res["calibration"][n] = {
            "known_read_bytes": rb, "known_write_bytes": wb,
            "sized_read_bytes": rd, "fetch_size_bytes": m.get("FETCH_SIZE", 0.0) * 1024.0,
            "write_size_bytes": wr,
            "read_scale": rb / rd if rd else None, "write_scale": wb / wr if wr else None}
    c8 = res["calibration"]["k_calib8"]
    rd = read_bytes(k)
    wr = k.get("WRITE_SIZE", 0.0) * 1024.0
    if rd is not None and wr:
        rs = c8["read_scale"] or 1.0
        ws = c8["write_scale"] or 1.0
        res["hbm_read_bytes_per_launch"] = rd * rs
        res["hbm_write_bytes_per_launch"] = wr * ws
        res["hbm_bytes_per_launch"] = rd * rs + wr * ws
        res["hbm_bytes_method"] = ("read: 32/64/128-B request counts x size; write: WRITE_SIZE; each x the "
                                   "k_calib8 known/measured ratio (same 8-B/lane pattern)")
        res["guide_fetch_x2_bytes"] = 2.0 * k.get("FETCH_SIZE", 0.0) * 1024.0
    if "TCC_HIT_sum" in k:
        h, mi = k["TCC_HIT_sum"], k.get("TCC_MISS_sum", 0.0)
        res["l2_hit_rate"] = h / (h + mi) if h + mi else None
    if "SQ_WAVES" in k and k["SQ_WAVES"]:
        w = k["SQ_WAVES"]
        res["per_wave"] = {n[3:]: v / w for n, v in k.items() if n.startswith("SQ_") and n != "SQ_WAVES"}
    bench = os.path.join(out_dir, "prof_trace_bench.json")
    if os.path.exists(bench):
        d = json.loads(open(bench).read().strip().splitlines()[-1])
        res["envs"] = d["config"]["envs_per_gpu"]
        res["experiment"] = d["config"].get("experiment")
        res["bench_kernel_avg_us"] = d["roofline"].get("kernel_avg_us", d["roofline"].get("kernel_avg_us_per_step"))
        res["algorithmic_bytes_per_step"] = d["roofline"].get(
            "bytes_per_step", d["roofline"].get("bytes_per_launch", d["roofline"].get("bytes_per_env_step", 0) * res["envs"]))
    if STEPS_PER_LAUNCH > 1 and "hbm_bytes_per_launch" in res:
        res["steps_per_launch"] = STEPS_PER_LAUNCH
        res["hbm_bytes_per_step"] = res["hbm_bytes_per_launch"] / STEPS_PER_LAUNCH
        # the per-step time from the full-length launches of the trace (the bench's
        # warm-up launch runs 3 steps)
        tr = [r for r in rows(os.path.join(out_dir, "prof_trace", "**", "*kernel_trace.csv"))
              if KERNEL in r.get("Kernel_Name", "")]
        d = sorted(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in tr)
        if d:
            full = [x for x in d if x >= 0.5 * d[len(d) // 2]]
            res["trace_full_launches"] = len(full)
            res["trace_avg_ns_per_step"] = sum(full) / len(full) / STEPS_PER_LAUNCH
    name = "pmc_k_step.json" if KERNEL == "k_step" else f"pmc_{MODE}.json"
    json.dump(res, open(os.path.join(out_dir, name), "w"), indent=1)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    if len(sys.argv) > 2 and sys.argv[2] in ("segment", "rollout"):
        KERNEL, STEPS_PER_LAUNCH, MODE = "k_rollout", 256, sys.argv[2]   # bench.SEG
    main(sys.argv[1] if len(sys.argv) > 1 else "gpurun_out")
