#!/bin/bash
# rocprofv3 kernel trace of the default bench line; per-kernel medians and the gaps
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/kt -o run --output-format csv \
  -- python3 bench.py --no-cpu-baseline ${BENCH_ARGS} > gpurun_out/kt_bench.json 2> gpurun_out/kt.log || { tail -5 gpurun_out/kt.log; exit 1; }
python3 - <<'PY'
import csv, glob, re, statistics as st
from collections import defaultdict
f = glob.glob("gpurun_out/kt/**/run_kernel_trace.csv", recursive=True)[0]
rows = list(csv.DictReader(open(f)))
name = lambda r: (re.search(r"(k_\w+)", r["Kernel_Name"]) or [None, r["Kernel_Name"][:20]])[1]
d = defaultdict(list)
for r in rows:
    d[name(r)].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
for k, v in d.items():
    print(f"{k:28s} n={len(v):5d} median={st.median(v):8.2f} us")
seq = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), name(r)) for r in rows)
g = defaultdict(list)
for a, b in zip(seq, seq[1:]):
    g[(a[2], b[2])].append((b[0] - a[1]) / 1e3)
for k, v in g.items():
    if len(v) > 10:
        print("gap", k, round(st.median(v), 2))
PY
