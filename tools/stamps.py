"""Summarise per-wave FILTER stamps written with HIPRAG_STAMPS=<file> (wall clock, 100 MHz):
{entry, staged, end, tiles} per wave.  Usage: python tools/stamps.py <file>"""
import sys

import numpy as np

a = np.fromfile(sys.argv[1], dtype=np.uint64).reshape(-1, 4).astype(np.int64)
a = a[a[:, 0] > 0]
t0 = a[:, 0].min()
us = lambda x: (x - t0) / 100.0  # 100 MHz -> us
ent, stg, end, tiles = us(a[:, 0]), us(a[:, 1]), us(a[:, 2]), a[:, 3]
q = lambda v: " ".join(f"{np.percentile(v, p):7.1f}" for p in (0, 10, 50, 90, 100))
print(f"waves {len(a)}  (percentiles 0/10/50/90/100, us from first wave entry)")
print(f"entry          {q(ent)}")
print(f"staged         {q(stg)}")
print(f"staging dur    {q(stg - ent)}")
print(f"end            {q(end)}")
print(f"tiles/wave     {q(tiles)}")
rate = tiles / np.maximum(end - stg, 1e-3)
print(f"tiles/us/wave  {q(rate)}")
print(f"kernel span {end.max():.1f} us; mean wave busy {np.mean(end - ent):.1f} us; "
      f"idle at tail (mean end gap to last) {np.mean(end.max() - end):.1f} us")
