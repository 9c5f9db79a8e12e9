#!/bin/bash
# HBM traffic of the staged exchange's side launch (k_rb_side) in bench's replay path
# (tools/prof_staged4.py, kind ag): the memory PMC passes of tools/pmc.sh, one per run,
# each also over tools/probes/fetch_calib for the calibration; then
# tools/pmc_side_summary.py -> gpurun_out/pmc_side.json.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=$GRAFT_REPO_ROOT/gpurun_out
mkdir -p "$OUT"
[ -x tools/probes/fetch_calib ] || /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 \
  -o tools/probes/fetch_calib tools/probes/fetch_calib.hip || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/side_trace" -o run --output-format csv \
  -- python3 tools/prof_staged4.py 8 ag > "$OUT/side_trace.log" 2>&1 || exit 1
i=0
while read -r c; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $c -d "$OUT/side_pmc$i" -o run --output-format csv \
    -- python3 tools/prof_staged4.py 8 ag > "$OUT/side_pmc$i.log" 2>&1 || exit 1
  timeout -s KILL 60 rocprofv3 --pmc $c -d "$OUT/side_calib_pmc$i" -o run --output-format csv \
    -- ./tools/probes/fetch_calib > "$OUT/side_calib_pmc$i.log" 2>&1 || exit 1
done <<'LIST'
TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_128B_sum
WRITE_SIZE TCC_HIT_sum TCC_MISS_sum
LIST
python3 tools/pmc_side_summary.py "$OUT" || exit 1
