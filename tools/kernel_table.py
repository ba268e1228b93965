"""Per-kernel totals from a rocprofv3 rocpd database (the default output format): python tools/kernel_table.py
<results.db> [fraction of the run to keep, from the end (default 0.5: the steady state)] [top N]."""
import collections
import sqlite3
import sys


def main(path: str, keep: float = 0.5, top: int = 40) -> None:
    db = sqlite3.connect(path)
    rows = list(db.execute("select name, start, end from kernels order by start"))
    tail = rows[int(len(rows) * (1 - keep)):]
    agg = collections.defaultdict(lambda: [0, 0.0])
    for name, s, e in tail:
        k = name[:100] if name.startswith("void (anon") else name.split("(")[0][:100]
        agg[k][0] += 1
        agg[k][1] += (e - s) / 1e3
    busy = sum(v[1] for v in agg.values())
    span = (tail[-1][2] - tail[0][1]) / 1e3 if tail else 0.0
    print(f"kernels {len(tail)}  busy {busy:.0f} us  span {span:.0f} us")
    for k, v in sorted(agg.items(), key=lambda x: -x[1][1])[:top]:
        print(f"{v[1]:10.0f} us {v[0]:7d} x {v[1] / v[0]:8.2f} us  {k}")


if __name__ == "__main__":
    main(sys.argv[1], float(sys.argv[2]) if len(sys.argv) > 2 else 0.5, int(sys.argv[3]) if len(sys.argv) > 3 else 40)
