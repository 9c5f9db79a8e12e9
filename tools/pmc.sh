#!/bin/bash
# rocprofv3 evidence for the bench kernel (run on the GPU box from the repo root):
#   PMC_KERNEL=segment (default: the persistent k_rollout of --launch segment),
#   rollout (the same kernel as --rollout 256 runs it: every step's record and
#   terminal obs to rows of their own, the headline's every_output) or step
#   (k_step of --launch step);
#   1. kernel trace + stats of the bench command;
#   2. PMC passes, one per run, --pmc never combined with a trace domain (pool
#      rule), each within the per-block limits (<= 4 TCC, <= 8 SQ counters):
#      memory-side read requests split by size, WRITE_SIZE + L2 hit/miss,
#      FETCH_SIZE (the guide's convention), and two SQ instruction passes;
#   3. the same memory passes over tools/probes/fetch_calib (known bytes, the
#      8-B/lane access pattern of k_step) to calibrate them.
# tools/pmc_summary.py reduces everything to gpurun_out/pmc_<kernel>.json.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=$GRAFT_REPO_ROOT/gpurun_out
mkdir -p "$OUT"
# the calibration probe is a gitignored build product: build it if this tree lacks it
[ -x tools/probes/fetch_calib ] || /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 \
  -o tools/probes/fetch_calib tools/probes/fetch_calib.hip || exit 1
MODE=${PMC_KERNEL:-segment}
if [ "$MODE" = step ]; then LAUNCH="--launch step"; PMCL="--launch step --no-graph"
elif [ "$MODE" = rollout ]; then LAUNCH="--rollout 256"; PMCL="--rollout 256"
else LAUNCH=""; PMCL=""; fi
BENCH="python3 bench.py --steps ${PMC_STEPS:-256} --warmup 128 --no-cpu-baseline --no-every-output $PMCL"
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$OUT/prof_trace" -o run --output-format csv \
  -- python3 bench.py --no-cpu-baseline --no-every-output $LAUNCH > "$OUT/prof_trace_bench.json" 2> "$OUT/prof_trace.log" || exit 1
i=0
while read -r c; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $c -d "$OUT/prof_pmc$i" -o run --output-format csv \
    -- $BENCH > "$OUT/prof_pmc${i}_bench.json" 2> "$OUT/prof_pmc$i.log" || exit 1
  timeout -s KILL 60 rocprofv3 --pmc $c -d "$OUT/calib_pmc$i" -o run --output-format csv \
    -- ./tools/probes/fetch_calib > "$OUT/calib_pmc$i.log" 2>&1 || exit 1
done <<'LIST'
TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_128B_sum
WRITE_SIZE TCC_HIT_sum TCC_MISS_sum
FETCH_SIZE
SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64
SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VMEM SQ_INSTS_VALU_TRANS_F64 SQ_INSTS_VALU_CVT SQ_INSTS_VALU_INT32
SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_MISC SQ_INST_CYCLES_SALU SQ_INSTS_BRANCH SQ_INSTS_SMEM SQ_INSTS_VALU_INT64
LIST
python3 tools/pmc_summary.py "$OUT" "$MODE" || exit 1
