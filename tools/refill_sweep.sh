#!/bin/bash
# Refill kernels' durations (rocprofv3 kernel trace) and the bench line per helper count.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
for h in ${HELPERS:-8192 4096 2048}; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "gpurun_out/rs_$h" -o run --output-format csv \
    -- python3 bench.py --no-cpu-baseline --helpers $h --steps 1024 > "gpurun_out/rs_$h.json" 2> "gpurun_out/rs_$h.log" || exit 1
  python3 - "$h" <<'PY'
import csv, glob, json, sys
h = sys.argv[1]
d = json.load(open(f"gpurun_out/rs_{h}.json"))
st = {}
for f in glob.glob(f"gpurun_out/rs_{h}/**/*kernel_stats.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        n = r["Name"]
        for k in ("k_need_masks", "k_refill_fit", "k_refill(", "k_rollout"):
            if k in n:
                st[k.strip("(")] = round(float(r["AverageNs"]) / 1000, 2)
print("helpers", h, round(d["value"] / 1e9, 3), "G/s", round(d["ms_per_step"] * 1e3, 3), "us/step", st)
PY
done
