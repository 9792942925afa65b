#!/usr/bin/env python3
"""Analyse per-wave stamps (GOL_STAMP_FILE) of one stencil launch: span, busy fraction, tail."""
import sys
import numpy as np

d = np.fromfile(sys.argv[1], dtype=np.uint64).reshape(-1, 2).astype(np.int64)
d = d[(d[:, 0] > 0) & (d[:, 1] > 0)]
t0 = d[:, 0].min()
s, e = (d[:, 0] - t0) / 100.0, (d[:, 1] - t0) / 100.0   # µs (100 MHz)
dur = e - s
span = e.max()
slots = int(sys.argv[2]) if len(sys.argv) > 2 else 2048
print(f"waves {len(d)}  span {span:.1f} us  wave dur mean {dur.mean():.1f} p5 {np.percentile(dur,5):.1f} "
      f"p95 {np.percentile(dur,95):.1f} max {dur.max():.1f}")
print(f"busy fraction (sum dur / (slots*span)) = {dur.sum() / (slots * span):.3f} with {slots} slots")
for q in (0.5, 0.9, 0.99, 1.0):
    print(f"  {int(q*100)}% of waves done by {np.quantile(e, q):.1f} us")
hist, edges = np.histogram(s, bins=12)
print("start histogram:", list(hist))
# concurrency over time
ts = np.linspace(0, span, 25)
conc = [int(((s <= t) & (e > t)).sum()) for t in ts]
print("resident waves over time:", conc)
