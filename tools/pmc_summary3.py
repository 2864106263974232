#!/usr/bin/env python3
"""Summarise one fixed-shape rocprofv3 collection (tools/profile_round3.sh)
into a PMC summary bench.py reads (profiles/<tag>_pmc.json).

Per kernel (short name, see STAGE): launches, mean duration (kernel trace),
the per-dispatch means of every counter of the separate --pmc passes, HBM
bytes per launch with MI355X_MICROARCH.md's gfx950 correction (FETCH_SIZE
counts half the bytes of a wide coalesced streaming read: x2; WRITE_SIZE
exact; both reported in KiB), and -- because the run has a fixed shape
(one batch size, one hash stream) -- the per-step and per-square figures:

  launches_per_step_k<K>    = launches / steps_total
  hbm_bytes_per_square_k<K> = hbm_bytes_per_launch x launches_per_step / squares_per_step

so every traffic number bench.py prints is reproducible from this file.
Merges into an existing summary (one file for k = 128 and k = 512).

Usage: pmc_summary3.py <collection dir> <summary.json> <k> <steps_total> <squares_per_step> <command>
"""
import collections
import csv
import json
import os
import sys

STAGE = {"rfc_leaf_kernel": "data_root_leaves", "data_root_digest_kernel": "data_root_digest",
         "leaf_kernel": "nmt_leaves", "level_kernel": "nmt_levels", "tree_top_kernel": "nmt_tree_top",
         "data_root_kernel": "data_root", "rs8_bs_half_kernel": "rs_gf8_bs", "rs8_bs_kernel": "rs_gf8_bs",
         "rs8_job_kernel": "rs_gf8", "rs16_cw_kernel": "rs_gf16", "rs16_lds_kernel": "rs_gf16_lds",
         "rs16_half_kernel": "rs_gf16", "rs16_bs_kernel": "rs_gf16", "subtree_kernel": "nmt_levels"}   # (fused levels of k = 256 / 512 squares)


def short(name: str) -> str:
    for k in STAGE:
        if k in name:
            return STAGE[k]
    return name.split("(")[0][-40:]


def main(src, dst, k, steps_total, squares, command):
    k, steps_total, squares = int(k), int(steps_total), int(squares)
    out = json.load(open(dst)) if os.path.exists(dst) else {}
    cfg = out.setdefault("_config", {})
    cfg[f"k{k}"] = {"k": k, "steps_total": steps_total, "squares_per_step": squares, "command": command,
                    "note": "fixed launch shape: one batch size, one hash stream; counters are per-dispatch "
                            "means of separate --pmc passes"}
    cur = collections.defaultdict(dict)
    for row in csv.DictReader(open(f"{src}/trace/run_kernel_stats.csv")):
        s = short(row["Name"])
        cur[s]["launches"] = cur[s].get("launches", 0) + int(row["Calls"])
        cur[s]["total_ns"] = cur[s].get("total_ns", 0.0) + float(row["TotalDurationNs"])
    for s, d in cur.items():
        d["avg_us"] = d["total_ns"] / d["launches"] / 1e3
    for sub in sorted(os.listdir(src)):
        f = f"{src}/{sub}/run_counter_collection.csv"
        if sub == "trace" or not os.path.exists(f):
            continue
        acc = collections.defaultdict(lambda: collections.defaultdict(list))
        for row in csv.DictReader(open(f)):
            acc[short(row["Kernel_Name"])][row["Counter_Name"]].append(float(row["Counter_Value"]))
            acc[short(row["Kernel_Name"])]["_dur"].append(
                (int(row["End_Timestamp"]) - int(row["Start_Timestamp"])) * 1e-9)
        for s, counters in acc.items():
            for c, vals in counters.items():
                if c != "_dur":
                    cur[s][c] = sum(vals) / len(vals)
            if "GRBM_GUI_ACTIVE" in counters:
                g = sum(counters["GRBM_GUI_ACTIVE"]) / len(counters["GRBM_GUI_ACTIVE"])
                dd = sum(counters["_dur"]) / len(counters["_dur"])
                cur[s]["effective_clock_ghz"] = g / 8 / dd / 1e9 if dd > 0 else None
    for s, d in cur.items():
        if "launches" in d:
            d[f"launches_per_step_k{k}"] = d["launches"] / steps_total
        if "FETCH_SIZE" in d and "WRITE_SIZE" in d:
            d["hbm_bytes_per_launch"] = (2 * d["FETCH_SIZE"] + d["WRITE_SIZE"]) * 1024
            if "launches" in d:
                d[f"hbm_bytes_per_square_k{k}"] = d["hbm_bytes_per_launch"] * d["launches"] / steps_total / squares
        if d.get("SQ_WAVE_CYCLES"):
            d["wait_any_frac"] = d.get("SQ_WAIT_ANY", 0) / d["SQ_WAVE_CYCLES"]
            d["wait_inst_any_frac"] = d.get("SQ_WAIT_INST_ANY", 0) / d["SQ_WAVE_CYCLES"]
        if "SQ_INSTS_VALU" in d and d.get("SQ_WAVES"):
            d["valu_insts_per_wave"] = d["SQ_INSTS_VALU"] / d["SQ_WAVES"]
        key = s if s in STAGE.values() else s
        if key in out and isinstance(out[key], dict) and k != 128:
            # keep the k = 128 record of a kernel both runs launch; add the k-tagged keys
            for kk, v in d.items():
                if kk.endswith(f"_k{k}"):
                    out[key][kk] = v
            out[key][f"k{k}"] = d
        else:
            out[key] = {**out.get(key, {}), **d} if isinstance(out.get(key), dict) else d
    json.dump(out, open(dst, "w"), indent=1, sort_keys=True)
    show = ("avg_us", "launches", "hbm_bytes_per_launch", f"hbm_bytes_per_square_k{k}", "valu_insts_per_wave",
            "effective_clock_ghz", "wait_any_frac")
    print(json.dumps({s: {kk: v for kk, v in d.items() if kk in show} for s, d in cur.items()
                      if s in STAGE.values()}, indent=1))


if __name__ == "__main__":
    main(*sys.argv[1:7])
