#!/bin/bash
# Effective clock of the segment kernel (MI355X_MICROARCH.md "DVFS give-back":
# GRBM_GUI_ACTIVE / 8 XCDs / dispatch duration) at one and two owner waves per SIMD.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
for n in 65536 131072; do
  timeout -s KILL 120 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_WAVE_CYCLES SQ_BUSY_CYCLES -d gpurun_out/clk_$n -o run \
    --output-format csv -- python3 bench.py --envs $n --steps 256 --warmup 128 --no-cpu-baseline \
    > gpurun_out/clk_$n.json 2> gpurun_out/clk_$n.log || { tail -5 gpurun_out/clk_$n.log; exit 1; }
done
python3 - <<'PY'
import csv, glob, collections
for n in (65536, 131072):
    f = glob.glob(f"gpurun_out/clk_{n}/**/run_counter_collection.csv", recursive=True)[0]
    rows = [r for r in csv.DictReader(open(f)) if "k_rollout" in r["Kernel_Name"]]
    by = collections.defaultdict(dict)
    for r in rows:
        by[r["Dispatch_Id"]][r["Counter_Name"]] = float(r["Counter_Value"])
        by[r["Dispatch_Id"]]["dur"] = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
    clk = [d["GRBM_GUI_ACTIVE"] / 8 / d["dur"] for d in by.values() if d["dur"] > 100000]
    clk.sort()
    print(n, "envs: k_rollout dispatches", len(clk), "effective clock GHz median", round(clk[len(clk) // 2], 3),
          "min", round(clk[0], 3), "max", round(clk[-1], 3))
PY
