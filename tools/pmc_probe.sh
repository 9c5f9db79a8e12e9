#!/bin/bash
# Diagnostic PMC passes on k_step for two workloads (default / no episode ends).
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=$GRAFT_REPO_ROOT/gpurun_out/probe
mkdir -p "$OUT"
i=0
for w in "" "--test-mode 1 --episode-steps 0"; do
  i=$((i+1))
  j=0
  for c in "SQC_ICACHE_MISSES SQC_ICACHE_HITS SQC_TC_INST_REQ" \
           "SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_VMEM SQ_IFETCH" \
           "SQ_INST_CYCLES_VMEM_RD SQ_INST_CYCLES_VMEM_WR SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VMEM SQ_INSTS_SALU SQ_INSTS_LDS SQ_ACTIVE_INST_LDS SQ_INSTS_SMEM"; do
    j=$((j+1))
    timeout -k 10 300 rocprofv3 --pmc $c -d "$OUT/w${i}_p$j" -o run --output-format csv \
      -- python3 bench.py --steps 200 --warmup 100 --no-cpu-baseline --no-graph $w > /dev/null 2> "$OUT/w${i}_p$j.log" || exit 1
  done
done
python3 - <<'PY'
import csv, glob, os, statistics as S
out = os.path.join(os.environ["GRAFT_REPO_ROOT"], "gpurun_out", "probe")
for w in (1, 2):
    vals = {}
    for f in glob.glob(f"{out}/w{w}_p*/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            if "k_step" in r["Kernel_Name"]:
                vals.setdefault(r["Counter_Name"], []).append(float(r["Counter_Value"]))
    print("workload", w)
    for k in sorted(vals):
        print(f"  {k:28s} median {S.median(vals[k]):14.1f}")
PY
