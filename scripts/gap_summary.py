#!/usr/bin/env python3
"""Launch-gap share of a rocprofv3 --kernel-trace CSV: busy time (union of kernel intervals) vs the wall span
of the dispatches between the first and the last of the `unet` step loop, and the idle gaps between
consecutive kernels.  Usage: python scripts/gap_summary.py kernel_trace.csv [min_gap_us]"""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
thr = float(sys.argv[2]) if len(sys.argv) > 2 else 0.0
iv = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"])) for r in rows)
busy, gaps, n_gap, big = 0, 0, 0, []
cur_s, cur_e = iv[0]
for s, e in iv[1:]:
    if s > cur_e:
        busy += cur_e - cur_s
        g = s - cur_e
        gaps += g
        n_gap += 1
        if g > thr * 1e3:
            big.append(g)
        cur_s, cur_e = s, e
    else:
        cur_e = max(cur_e, e)
busy += cur_e - cur_s
span = iv[-1][1] - iv[0][0]
print(f"dispatches {len(iv)}  span {span / 1e6:.2f} ms  busy {busy / 1e6:.2f} ms  idle {gaps / 1e6:.2f} ms "
      f"({100 * gaps / span:.2f} %)  gaps {n_gap}  mean gap {gaps / max(n_gap, 1) / 1e3:.2f} us")
big.sort(reverse=True)
print("largest gaps (us):", [round(g / 1e3, 1) for g in big[:15]])
