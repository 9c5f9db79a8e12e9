#!/bin/bash
# The segment kernel's effective clock per dispatch over a default bench run (GRBM_GUI_ACTIVE / 8 XCDs /
# duration): profiles/r05_clock_boost.txt
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -s KILL 200 rocprofv3 --pmc GRBM_GUI_ACTIVE -d gpurun_out/clk20 -o run --output-format csv -- python3 bench.py --no-cpu-baseline --no-every-output > gpurun_out/clk20.json 2> gpurun_out/clk20.log || { tail -5 gpurun_out/clk20.log; exit 1; }
python3 - <<'PY'
import csv, glob, statistics
f = glob.glob("gpurun_out/clk20/**/run_counter_collection.csv", recursive=True)[0]
rows = [r for r in csv.DictReader(open(f)) if "k_rollout" in r["Kernel_Name"]]
d = sorted(((int(r["Dispatch_Id"]), float(r["Counter_Value"]), int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
            for r in rows), key=lambda x: x[0])
full = [(i, c / 8 / t, t) for i, c, t in d if t > 100000]
print("dispatches", len(full))
for lo, hi in ((0, 5), (5, 20), (20, 100), (100, 500), (500, len(full))):
    seg = full[lo:hi]
    if seg:
        print(f"dispatch {lo}-{hi}: clock GHz median {statistics.median(x[1] for x in seg):.3f}, "
              f"duration us median {statistics.median(x[2] for x in seg) / 1e3:.1f}")
PY
python3 -c "import json;d=json.load(open('gpurun_out/clk20.json'));print(round(d['value']/1e9,3), d['roofline']['kernel_avg_us'])"
