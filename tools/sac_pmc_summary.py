"""MFMA utilisation of the SAC kernels from a rocprofv3 --pmc CSV (tools/prof_sac.py run).

Counters: SQ_INSTS_VALU_MFMA_F32, SQ_VALU_MFMA_BUSY_CYCLES (summed over SIMDs),
GRBM_GUI_ACTIVE (summed over the 8 XCDs, MI355X_MICROARCH.md). Utilisation =
MFMA-busy cycles per SIMD / active cycles per XCD, 1024 SIMDs.
"""
import collections
import csv
import json
import sys

PHASE = {65536: "rows phase 0 (256 wg)", 98304: "rows phase 1 (384 wg)", 32768: "rows phase 2 (128 wg)",
         82176: "update (321 wg)", 262144: "act, 65 536 rows (1 024 wg)"}
agg = collections.defaultdict(lambda: collections.defaultdict(list))
for r in csv.DictReader(open(sys.argv[1])):
    if "k_sac" not in r["Kernel_Name"]:
        continue
    agg[int(r["Grid_Size"])][r["Counter_Name"]].append(float(r["Counter_Value"]))
out = {}
for g, c in sorted(agg.items()):
    m = {k: sum(v) / len(v) for k, v in c.items()}
    busy = m.get("SQ_VALU_MFMA_BUSY_CYCLES", 0.0) / 1024
    act = m.get("GRBM_GUI_ACTIVE", 0.0) / 8
    out[PHASE.get(g, f"grid {g}")] = {
        "mfma_f32_insts": m.get("SQ_INSTS_VALU_MFMA_F32"), "mfma_busy_cycles_per_simd": busy,
        "active_cycles_per_xcd": act, "mfma_utilisation": busy / act if act else None}
print(json.dumps(out, indent=1))
