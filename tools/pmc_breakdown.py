"""Per-kernel PMC breakdown from rocprofv3 --pmc passes (one directory per counter group, same workload).

Averages every counter over the matching dispatches of each pass and derives where the waves' cycles go:
SQ_WAIT_ANY (parked on s_waitcnt / barrier) + SQ_WAIT_INST_ANY (issue stall) + SQ_ACTIVE_INST_ANY (issuing)
~= SQ_WAVE_CYCLES (MI355X_MICROARCH.md, PMC table); MFMA busy as tools/summarize_profile.py; HBM read bytes =
FETCH_SIZE (KiB) x 1024 x 2 (the gfx950 correction, same source).
Usage: python tools/pmc_breakdown.py <kernel-regex> <pass-dir> [<pass-dir> ...] > summary.json
"""
from __future__ import annotations

import csv
import glob
import json
import os
import re
import statistics
import sys
from collections import defaultdict


def load(dirs: list[str], pat: str) -> tuple[dict, dict]:
    rx = re.compile(pat)
    vals: dict[str, list[float]] = defaultdict(list)
    durs: list[float] = []
    for d in dirs:
        for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
            per: dict[tuple, dict] = defaultdict(dict)
            for row in csv.DictReader(open(f)):
                if not rx.search(row["Kernel_Name"]):
                    continue
                key = (row["Dispatch_Id"],)
                per[key][row["Counter_Name"]] = per[key].get(row["Counter_Name"], 0.0) + float(row["Counter_Value"])
                per[key]["_dur"] = (int(row["End_Timestamp"]) - int(row["Start_Timestamp"])) * 1e-6
            for d_ in per.values():
                for k, v in d_.items():
                    if k == "_dur":
                        durs.append(v)
                    else:
                        vals[k].append(v)
    return {k: statistics.mean(v) for k, v in vals.items()}, {"dispatches": len(durs), "ms_mean": statistics.mean(durs) if durs else None}


def breakdown(c: dict) -> dict:
    out = {}
    wc = c.get("SQ_WAVE_CYCLES")
    if wc:
        for k, name in (("SQ_WAIT_ANY", "parked_waitcnt_or_barrier"), ("SQ_WAIT_INST_ANY", "issue_stall"),
                        ("SQ_ACTIVE_INST_ANY", "issuing"), ("SQ_WAIT_INST_LDS", "lds_issue_stall"),
                        ("SQ_ACTIVE_INST_VMEM", "vmem_issue"), ("SQ_ACTIVE_INST_LDS", "lds_issue"),
                        ("SQ_ACTIVE_INST_VALU", "valu_issue")):
            if k in c:
                out[f"{name}_frac_of_wave_cycles"] = round(c[k] / wc, 4)
    if "SQ_VALU_MFMA_BUSY_CYCLES" in c and c.get("GRBM_GUI_ACTIVE"):
        out["mfma_busy_frac"] = round(c["SQ_VALU_MFMA_BUSY_CYCLES"] / (c["GRBM_GUI_ACTIVE"] / 8 * 1024), 4)
    if c.get("SQ_LDS_IDX_ACTIVE"):
        out["lds_bank_conflict_frac_of_lds_cycles"] = round(c.get("SQ_LDS_BANK_CONFLICT", 0.0) / c["SQ_LDS_IDX_ACTIVE"], 4)
    if "FETCH_SIZE" in c:
        out["hbm_read_gb_per_dispatch"] = round(c["FETCH_SIZE"] * 1024 * 2 / 1e9, 4)
    return out


if __name__ == "__main__":
    pat, dirs = sys.argv[1], sys.argv[2:]
    counters, meta = load(dirs, pat)
    json.dump({"kernel_regex": pat, "passes": dirs, **meta, "derived": breakdown(counters),
               "counters_mean_per_dispatch": {k: round(v, 1) for k, v in sorted(counters.items())}}, sys.stdout, indent=1)
    print()
