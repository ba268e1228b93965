"""Summarise rocprofv3 CSVs of tools/profile.sh into profiles/<tag>_*.

Kernel-trace stats -> per-kernel averages.  The FILTER pass is told from the SAMPLE pass BY NAME:
since round 4 they are distinct kernel symbols (k_scan_filter / k_scan_sample / k_scan_collect, and
the 128-query FILTER k_filter_wide8).  Traces of older builds name every pass "k_scan"; for those the
FILTER set is the largest grid AND a duration above a quarter of the longest such launch (a
synchronous batch runs its SAMPLE on the full grid too -- round 3's summaries counted such a 49 us
SAMPLE as a FILTER launch).
PMC FETCH_SIZE / WRITE_SIZE are KB per dispatch; on gfx950 FETCH_SIZE reports half of a wide
coalesced stream (MI355X_MICROARCH.md §HBM), so HBM read bytes = 2 * FETCH_SIZE * 1024.
"""
import csv
import json
import os
import shutil
import statistics
import sys

FILTER_NAMES = ("k_scan_filter", "k_filter_wide8", "k_filter_q256", "k_scan_persist")
SAMPLE_NAMES = ("k_scan_sample",)
# the measured practical read ceiling (tools/stream_ceiling.hip, profiles/r02_stream_ceiling.jsonl): a summary
# whose FILTER rate exceeds it has mis-classified launches
READ_CEILING_GBS = 7076.6


def rows(path):
    with open(path) as f:
        return list(csv.DictReader(f))


def _base(name: str) -> str:
    """Kernel symbol without template arguments / parameter list (rocprofv3 may print either form)."""
    n = name.strip()
    if n.startswith("void "):
        n = n[5:]
    for c in "<(":
        n = n.split(c)[0]
    return n.strip()


def _ms(r) -> float:
    return (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6


def classify(kt):
    """(filter rows, sample rows) of a kernel trace."""
    names = {_base(r["Kernel_Name"]) for r in kt}
    if names & set(FILTER_NAMES):
        return ([r for r in kt if _base(r["Kernel_Name"]) in FILTER_NAMES],
                [r for r in kt if _base(r["Kernel_Name"]) in SAMPLE_NAMES])
    scan = [r for r in kt if _base(r["Kernel_Name"]) == "k_scan"]  # legacy single-symbol builds
    if not scan:
        return [], []
    gmax = max(int(r.get("Grid_Size_X") or r.get("Grid_Size") or 0) for r in scan)
    big = [r for r in scan if int(r.get("Grid_Size_X") or r.get("Grid_Size") or 0) == gmax]
    dmax = max(_ms(r) for r in big)
    filt = [r for r in big if _ms(r) > dmax / 4]
    fids = {id(r) for r in filt}
    return filt, [r for r in scan if id(r) not in fids]


def _pmc_filter_ids(recs, kt_filter_count):
    """Dispatch ids of the FILTER launches in a PMC pass (by name; legacy: the largest values)."""
    by = {}
    for r in recs:
        by.setdefault(r.get("Dispatch_Id") or r.get("Correlation_Id"), []).append(r)
    named = {d for d, rs in by.items() if _base(rs[0]["Kernel_Name"]) in FILTER_NAMES}
    if named:
        return named, {d for d, rs in by.items() if _base(rs[0]["Kernel_Name"]) in SAMPLE_NAMES}
    return None, None


def main(src, tag, alg_bytes=None):
    os.makedirs("profiles", exist_ok=True)
    kt = rows(os.path.join(src, "kt", "run_kernel_trace.csv"))
    shutil.copy(os.path.join(src, "kt", "run_kernel_stats.csv"), f"profiles/{tag}_kernel_stats.csv")
    dur = {}
    for r in kt:
        dur.setdefault(_base(r["Kernel_Name"]), []).append(_ms(r))
    filt_rows, samp_rows = classify(kt)
    filt, samp = [_ms(r) for r in filt_rows], [_ms(r) for r in samp_rows]
    # time during which at least one FILTER launch runs, per launch: with the dual FILTER streams
    # consecutive launches overlap, so this (not the per-launch duration) is the HBM time per launch
    busy, end = 0, None
    for s, e in sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"])) for r in filt_rows):
        if end is None or s > end:
            busy += e - s
            end = e
        elif e > end:
            busy += e - end
            end = e
    import datetime

    out = {"tag": tag, "created_utc": datetime.datetime.now(datetime.timezone.utc).strftime("%Y-%m-%dT%H:%M:%SZ"),
           "classification": "by kernel name" if {_base(r["Kernel_Name"]) for r in filt_rows} -
           {"k_scan"} else "legacy k_scan: largest grid and > 1/4 of the longest launch",
           "kernels_ms_avg": {k: statistics.mean(v) for k, v in dur.items()},
           "filter_kernels": sorted({_base(r["Kernel_Name"]) for r in filt_rows}),
           "k_scan_filter_ms_avg": statistics.mean(filt) if filt else None,
           "k_scan_filter_ms_median": statistics.median(filt) if filt else None,
           "k_scan_filter_launches": len(filt),
           "k_scan_filter_busy_ms_per_launch": busy / 1e6 / len(filt) if filt else None,
           "k_scan_sample_ms_avg": statistics.mean(samp) if samp else None, "k_scan_sample_launches": len(samp)}
    # launch PERIOD (start to start of consecutive FILTER launches): what one step costs the scan stream;
    # with overlapping launches (dual FILTER streams) it is shorter than a launch's duration
    starts = sorted(int(r["Start_Timestamp"]) for r in filt_rows)
    if len(starts) > 2:
        per = [(b - a) / 1e6 for a, b in zip(starts, starts[1:])]
        out["k_scan_filter_period_ms_median"] = statistics.median(per)
    # the bench's own JSON line from the profiled run (tools/profile.sh keeps its stdout): its ms_per_step
    # is the step the profiled kernels belong to, so the two are compared within one run
    log = os.path.join(src, "bench_kt.log")
    if os.path.exists(log):
        lines = [ln for ln in open(log, errors="replace") if ln.startswith("{")]
        if lines:
            b = json.loads(lines[-1])
            out["profiled_run"] = {"ms_per_step": b.get("ms_per_step"), "value": b.get("value"),
                                   "steps": b.get("steps"), "warmup": b.get("warmup"),
                                   "event_avg_launch_ms": (b.get("roofline") or {}).get("avg_launch_ms")}
            if b.get("ms_per_step") and filt:
                out["profiled_run"]["filter_avg_over_ms_per_step"] = statistics.mean(filt) / b["ms_per_step"]
    kt_fids = {r.get("Dispatch_Id") for r in filt_rows}
    p = os.path.join(src, "pmc_mfma", "run_counter_collection.csv")
    if os.path.exists(p):  # MFMA pipe busy fraction of the FILTER launches
        shutil.copy(p, f"profiles/{tag}_pmc_mfma.csv")
        recs = rows(p)
        fids, _ = _pmc_filter_ids(recs, len(filt))
        per = {}
        for r in recs:
            if fids is None and _base(r["Kernel_Name"]) != "k_scan":
                continue
            d = r.get("Dispatch_Id") or r.get("Correlation_Id")
            if fids is not None and d not in fids:
                continue
            per.setdefault(d, {})[r["Counter_Name"]] = float(r["Counter_Value"])
        busy = [d for d in per.values() if "SQ_VALU_MFMA_BUSY_CYCLES" in d and "GRBM_GUI_ACTIVE" in d]
        if fids is None and busy:  # legacy: the long launches
            busy = [d for d in busy if d["GRBM_GUI_ACTIVE"] > max(x["GRBM_GUI_ACTIVE"] for x in busy) / 4]
        if busy:
            # busy cycles summed over the 1024 SIMDs vs (GUI_ACTIVE / 8 XCDs) cycles x 1024 SIMDs
            frac = statistics.mean(d["SQ_VALU_MFMA_BUSY_CYCLES"] / (d["GRBM_GUI_ACTIVE"] / 8 * 1024) for d in busy)
            out["k_scan_filter_mfma_busy_frac"] = frac
    for name, key in (("pmc_fetch", "FETCH_SIZE"), ("pmc_write", "WRITE_SIZE")):
        p = os.path.join(src, name, "run_counter_collection.csv")
        if not os.path.exists(p):
            continue
        shutil.copy(p, f"profiles/{tag}_{name}.csv")
        recs = [r for r in rows(p) if r["Counter_Name"] == key]
        fids, sids = _pmc_filter_ids(recs, len(filt))
        if fids is not None:
            fv = [float(r["Counter_Value"]) for r in recs if (r.get("Dispatch_Id") or r.get("Correlation_Id")) in fids]
            sv = [float(r["Counter_Value"]) for r in recs if (r.get("Dispatch_Id") or r.get("Correlation_Id")) in sids]
        else:  # legacy single-symbol traces: the FILTER launches are the large values
            vals = [float(r["Counter_Value"]) for r in recs if _base(r["Kernel_Name"]) == "k_scan"]
            fv = [v for v in vals if v > (max(vals) / 4 if vals else 0)]
            sv = [v for v in vals if v <= (max(vals) / 4 if vals else 0)]
        if key == "FETCH_SIZE" and sv:
            # FETCH_SIZE counts Infinity-Cache hits too (MI355X_MICROARCH.md), so after the first batch this is
            # the SAMPLE's fabric traffic, most of it served on-die (its tiles are the same every batch)
            out["k_scan_sample_fetch_bytes"] = 2 * statistics.mean(sv) * 1024
        if fv:
            kb = statistics.mean(fv)
            out[f"k_scan_filter_{key}_KB_avg"] = kb
            out[f"k_scan_filter_{key}_launches"] = len(fv)
            if key == "FETCH_SIZE":
                out["k_scan_filter_hbm_read_bytes"] = 2 * kb * 1024  # gfx950 x2 correction
            else:
                out["k_scan_filter_hbm_write_bytes"] = kb * 1024
    if alg_bytes:
        out["algorithmic_bytes_per_launch"] = alg_bytes
        if "k_scan_filter_hbm_read_bytes" in out:
            out["traffic_over_algorithmic"] = out["k_scan_filter_hbm_read_bytes"] / alg_bytes
        if out["k_scan_filter_ms_avg"]:
            out["achieved_GBps_profiled"] = alg_bytes / (out["k_scan_filter_ms_avg"] * 1e-3) / 1e9
            if out["achieved_GBps_profiled"] > READ_CEILING_GBS:
                print(f"WARNING: FILTER rate {out['achieved_GBps_profiled']:.0f} GB/s exceeds the measured read ceiling "
                      f"{READ_CEILING_GBS} GB/s -- check the classification", file=sys.stderr)
        if out["k_scan_filter_busy_ms_per_launch"]:
            out["achieved_GBps_profiled_busy"] = alg_bytes / (out["k_scan_filter_busy_ms_per_launch"] * 1e-3) / 1e9
    with open(f"profiles/{tag}_summary.json", "w") as f:
        json.dump(out, f, indent=1)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2], int(sys.argv[3]) if len(sys.argv) > 3 else None)
