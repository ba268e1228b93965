"""Per-step GPU timeline from a rocprofv3 kernel trace (tools/profile.sh layout or any
run_kernel_trace.csv): for the last N FILTER scans, every kernel's start/end relative to that
scan's start, plus the gap between consecutive FILTER launches.
Usage: python tools/timeline.py <run_kernel_trace.csv> [n_steps]"""
import csv
import statistics
import sys


def main(path, n=4):
    with open(path) as f:
        rs = list(csv.DictReader(f))
    ks = sorted(((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"].replace("void ", "").replace("hr::", "")[:50],
                  r.get("Queue_Id", r.get("Stream_Id", "?"))) for r in rs))
    scans = [k for k in ks if "k_scan" in k[2]]
    if not scans:
        print("no k_scan")
        return
    durs = sorted(e - s for s, e, _, _ in scans)
    cut = (durs[0] + durs[-1]) / 2
    filt = [k for k in scans if k[1] - k[0] > cut]
    period = [b[0] - a[0] for a, b in zip(filt, filt[1:])]
    print(f"FILTER launches {len(filt)}; period median {statistics.median(period) / 1e3:.1f} us, "
          f"duration median {statistics.median([e - s for s, e, _, _ in filt]) / 1e3:.1f} us")
    # median gap per (previous kernel -> next kernel) transition on the FILTER's queue
    mq = filt[0][3]
    main = [k for k in ks if k[3] == mq and k[0] >= filt[len(filt) // 4][0]]
    gaps = {}
    for x, y in zip(main, main[1:]):
        gaps.setdefault((x[2][:24], y[2][:24]), []).append((y[0] - x[1]) / 1e3)
    for (x, y), v in sorted(gaps.items(), key=lambda kv: -len(kv[1])):
        print(f"  gap {x:24s} -> {y:24s} median {statistics.median(v):6.1f} us  (n={len(v)})")
    durs_by = {}
    for x in main:
        durs_by.setdefault(x[2][:24], []).append((x[1] - x[0]) / 1e3)
    for nm, v in durs_by.items():
        print(f"  dur {nm:24s} median {statistics.median(v):7.1f} us  (n={len(v)})")
    for a, b in (list(zip(filt, filt[1:]))[-n:] if n > 0 else []):
        t0 = a[0]
        print(f"--- step (period {(b[0] - a[0]) / 1e3:.1f} us)")
        for s, e, name, q in ks:
            if a[0] - 200_000 <= s < b[0]:
                print(f"  {(s - t0) / 1e3:9.1f} .. {(e - t0) / 1e3:9.1f} us  ({(e - s) / 1e3:7.1f})  q{q}  {name}")


if __name__ == "__main__":
    main(sys.argv[1], int(sys.argv[2]) if len(sys.argv) > 2 else 4)
