"""Reduce tools/pmc_side.sh's output: HBM bytes per k_rb_side launch (calibrated as
tools/pmc_summary.py does) against the launch's algorithmic bytes at bench's shape
(65 536 envs, B 1 024, 256 learns, world 1): the draws' idx (2.1 MB) and tile counts,
the pack's two 64-B rows per record read (33.6 MB) and 100-B records written (26.2 MB),
the unpack's records read (26.2 MB) and 26-word batch rows written (27.3 MB).
-> gpurun_out/pmc_side.json"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import pmc_summary as ps  # noqa: E402

SLOTS = 256 * 1024
ALGO = {"draw_idx": 8 * SLOTS, "pack_rows_read": 2 * 64 * SLOTS, "pack_records_written": 100 * SLOTS,
        "unpack_records_read": 100 * SLOTS, "unpack_words_written": 26 * 4 * SLOTS}


def main(out):
    res = {"kernel": "k_rb_side"}
    st = [r for r in ps.rows(os.path.join(out, "side_trace", "**", "*kernel_stats.csv")) if "k_rb_side" in r["Name"]]
    if st:
        res["trace_avg_ns"] = float(st[0]["AverageNs"])
        res["trace_calls"] = int(st[0]["Calls"])
    k = ps.means("side_pmc", out, "k_rb_side")
    res["counters_per_launch"] = k
    cal = ps.means("side_calib_pmc", out, "k_calib8")
    rb, wb = ps.CALIB["k_calib8"]
    rd, wr = ps.read_bytes(cal), cal.get("WRITE_SIZE", 0.0) * 1024.0
    rs = rb / rd if rd else 1.0
    wsc = wb / wr if wr else 1.0
    hr = (ps.read_bytes(k) or 0.0) * rs
    hw = k.get("WRITE_SIZE", 0.0) * 1024.0 * wsc
    algo = sum(ALGO.values())
    res.update(hbm_read_bytes=hr, hbm_write_bytes=hw, hbm_bytes=hr + hw, algorithmic_bytes=algo,
               algorithmic=ALGO, traffic_over_algorithmic=(hr + hw) / algo, read_scale=rs, write_scale=wsc)
    if "trace_avg_ns" in res:
        t = res["trace_avg_ns"] * 1e-9
        res["achieved_GBps_algorithmic"] = algo / t / 1e9
        res["achieved_GBps_hbm"] = (hr + hw) / t / 1e9
    json.dump(res, open(os.path.join(out, "pmc_side.json"), "w"), indent=1)
    print(json.dumps({k2: v for k2, v in res.items() if k2 != "counters_per_launch"}, indent=1))


if __name__ == "__main__":
    main(sys.argv[1])
