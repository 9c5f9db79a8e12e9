#!/bin/bash
# Refill kernels' steady-state durations (rocprofv3 kernel trace, median per call
# after the first three) and the untraced bench line, per helper count.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
for h in ${HELPERS:-8192 4096}; do
  timeout -k 10 200 python3 bench.py --no-cpu-baseline --helpers $h > "gpurun_out/rsb_$h.json" 2> "gpurun_out/rsb_$h.log" || exit 1
  timeout -k 10 300 rocprofv3 --kernel-trace -d "gpurun_out/rs_$h" -o run --output-format csv \
    -- python3 bench.py --no-cpu-baseline --helpers $h --steps 1024 > "gpurun_out/rs_$h.json" 2> "gpurun_out/rs_$h.log" || exit 1
  python3 - "$h" <<'PY'
import csv, glob, json, sys
import numpy as np
h = sys.argv[1]
d = json.load(open(f"gpurun_out/rsb_{h}.json"))
rows = []
for f in glob.glob(f"gpurun_out/rs_{h}/**/*kernel_trace.csv", recursive=True):
    rows += list(csv.DictReader(open(f)))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
out, prev_end, gaps = {}, None, []
for k in ("k_need_masks", "k_refill(", "k_refill_fit", "k_rollout"):
    t = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1000 for r in rows if k in r["Kernel_Name"]]
    out[k.strip("(")] = round(float(np.median(t[3:])), 2) if len(t) > 3 else None
print("helpers", h, "bench", round(d["value"] / 1e9, 3), "G/s", round(d["ms_per_step"] * 1e3, 3),
      "us/step (untraced); traced medians us:", out)
PY
done
