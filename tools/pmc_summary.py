#!/usr/bin/env python3
"""Summarise a tools/profile_round.sh collection into profiles/<tag>_pmc.json.

Per kernel: launches, mean duration (kernel trace), FETCH_SIZE / WRITE_SIZE
(kB per launch, as rocprofv3 reports them), HBM bytes per launch with the
gfx950 correction of MI355X_MICROARCH.md §HBM (FETCH_SIZE counts half of the
bytes of a wide coalesced streaming read: x2; WRITE_SIZE exact), VALU
instructions per wave, and the effective clock GRBM_GUI_ACTIVE / 8 / time.
bench.py reads `hbm_bytes_per_launch` of the dominant stage as `traffic`.

Usage: python tools/pmc_summary.py gpurun_out/prof_<tag> profiles/<tag>_pmc.json
"""
import collections
import csv
import json
import sys

STAGE = {"rfc_leaf_kernel": "data_root_leaves", "data_root_digest_kernel": "data_root_digest",
         "leaf_kernel": "nmt_leaves", "level_kernel": "nmt_levels", "data_root_kernel": "data_root",
         "rs8_bs_half_kernel": "rs_gf8_bs", "rs8_bs_kernel": "rs_gf8_bs", "rs8_job_kernel": "rs_gf8", "rs8_flat_kernel": "rs_gf8_flat", "rs16_cw_kernel": "rs_gf16", "rs16_lds_kernel": "rs_gf16_lds",
         "order_kernel": "order_check"}


def short(name: str) -> str:
    for k in STAGE:
        if k in name:
            return STAGE[k]
    return name.split("(")[0][-40:]


def main(src: str, dst: str):
    out = collections.defaultdict(dict)
    for row in csv.DictReader(open(f"{src}/trace/run_kernel_stats.csv")):
        s = short(row["Name"])
        out[s]["launches"] = int(row["Calls"])
        out[s]["avg_us"] = float(row["AverageNs"]) / 1e3
    import os
    for sub in ("fetch", "write", "sq", "wait"):
        if not os.path.exists(f"{src}/{sub}/run_counter_collection.csv"):
            continue
        acc = collections.defaultdict(lambda: collections.defaultdict(list))
        for row in csv.DictReader(open(f"{src}/{sub}/run_counter_collection.csv")):
            acc[short(row["Kernel_Name"])][row["Counter_Name"]].append(float(row["Counter_Value"]))
            acc[short(row["Kernel_Name"])]["_dur"].append(
                (int(row["End_Timestamp"]) - int(row["Start_Timestamp"])) * 1e-9)
        for s, counters in acc.items():
            for c, vals in counters.items():
                if c != "_dur":
                    out[s][c] = sum(vals) / len(vals)
            if sub == "sq" and "GRBM_GUI_ACTIVE" in counters:
                g = sum(counters["GRBM_GUI_ACTIVE"]) / len(counters["GRBM_GUI_ACTIVE"])
                d = sum(counters["_dur"]) / len(counters["_dur"])
                out[s]["effective_clock_ghz"] = g / 8 / d / 1e9 if d > 0 else None
    for s, d in out.items():
        if "FETCH_SIZE" in d and "WRITE_SIZE" in d:
            d["hbm_bytes_per_launch"] = (2 * d["FETCH_SIZE"] + d["WRITE_SIZE"]) * 1024
        if d.get("SQ_WAVE_CYCLES"):   # share of wave cycles waiting on anything / on instruction issue
            d["wait_any_frac"] = d.get("SQ_WAIT_ANY", 0) / d["SQ_WAVE_CYCLES"]
            d["wait_inst_any_frac"] = d.get("SQ_WAIT_INST_ANY", 0) / d["SQ_WAVE_CYCLES"]
        if "SQ_INSTS_VALU" in d and d.get("SQ_WAVES"):
            d["valu_insts_per_wave"] = d["SQ_INSTS_VALU"] / d["SQ_WAVES"]
    json.dump(out, open(dst, "w"), indent=1, sort_keys=True)
    print(json.dumps({k: {kk: v for kk, v in d.items() if kk in ("avg_us", "hbm_bytes_per_launch",
                                                                  "valu_insts_per_wave", "effective_clock_ghz", "wait_any_frac")}
                      for k, d in out.items() if k in STAGE.values()}, indent=1))


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
