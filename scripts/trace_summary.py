#!/usr/bin/env python3
"""Aggregate a rocprofv3 --kernel-trace CSV by (kernel, grid, block): total / count / average µs.
Usage: python scripts/trace_summary.py kernel_trace.csv [top_n] [steps]"""
import collections
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
top = int(sys.argv[2]) if len(sys.argv) > 2 else 50
steps = float(sys.argv[3]) if len(sys.argv) > 3 else 1.0
agg = collections.defaultdict(lambda: [0, 0.0])
byk = collections.defaultdict(float)
for r in rows:
    n = r["Kernel_Name"].replace("void irx::(anonymous namespace)::", "").replace("irx::(anonymous namespace)::", "")
    n = n.split("(")[0][:58]
    wg = int(r["Workgroup_Size_X"])
    key = (n, int(r["Grid_Size_X"]) // wg, int(r["Grid_Size_Y"]), wg)
    d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
    agg[key][0] += 1
    agg[key][1] += d
    byk[n] += d
tot = sum(v[1] for v in agg.values())
print(f"total {tot / steps / 1e3:.1f} ms per step over {len(rows)} dispatches")
for k, v in sorted(byk.items(), key=lambda kv: -kv[1])[:20]:
    print(f"{v / steps / 1e3:9.2f} ms/step {100 * v / tot:5.1f}%  {k}")
print()
for k, v in sorted(agg.items(), key=lambda kv: -kv[1][1])[:top]:
    print(f"{v[1] / steps / 1e3:8.2f} ms/step {v[0] / steps:6.0f}x {v[1] / v[0]:8.1f}us  {k[0]:58s} grid {k[1]}x{k[2]} wg {k[3]}")
