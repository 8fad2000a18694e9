#!/usr/bin/env python3
"""Mean per-dispatch value of every counter in rocprofv3 counter_collection.csv files under the given
directories, for kernels whose name matches a regex (kernel-level PMC passes of scripts/kprof.py).
Usage: python scripts/pmc_dump.py <regex> <dir> [<dir> ...]"""
import csv
import re
import sys
from collections import defaultdict
from pathlib import Path

rx = re.compile(sys.argv[1])
vals = defaultdict(list)
names = set()
for d in sys.argv[2:]:
    for f in Path(d).rglob("*counter_collection.csv"):
        per = defaultdict(float)
        for r in csv.DictReader(open(f)):
            if not rx.search(r["Kernel_Name"]):
                continue
            names.add(r["Kernel_Name"][:120])
            per[(r["Dispatch_Id"], r["Counter_Name"])] += float(r["Counter_Value"])
            per[(r["Dispatch_Id"], "duration_ns")] = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
        for (disp, c), v in per.items():
            vals[c].append(v)
for n in sorted(names):
    print("kernel:", n)
for c in sorted(vals):
    v = vals[c]
    print(f"  {c:40s} {sum(v) / len(v):16.1f}   (n={len(v)})")
