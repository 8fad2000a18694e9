#!/usr/bin/env python3
"""Per-launch HBM traffic of one kernel from two rocprofv3 PMC passes (FETCH_SIZE, WRITE_SIZE), with the
gfx950 correction from /opt/skills/guides/MI355X_MICROARCH.md §HBM: FETCH_SIZE reports half the bytes of
16-B-per-lane streaming reads (global_load / buffer_load ... lds alike), so it is doubled; WRITE_SIZE is
exact for 16-B streaming stores.  Both counters are in KiB.

Usage: python scripts/pmc_traffic.py --fetch <dir of FETCH_SIZE pass> --write <dir of WRITE_SIZE pass>
           --kernel 'gemm2_kernel<128, 320, 2, 4, true, false>' --out profiles/r01_pmc_traffic.json
"""
from __future__ import annotations

import argparse
import csv
import json
import sqlite3
from pathlib import Path


def per_launch(d: Path, counter: str, kernel: str):
    vals = {}
    for f in Path(d).rglob("*results.db"):            # rocprofv3's default rocpd (sqlite) output
        con = sqlite3.connect(str(f))
        for disp, name, v in con.execute("select dispatch_id, kernel_name, value from counters_collection "
                                         "where counter_name = ?", (counter,)):
            if kernel in name:
                vals[(f, disp)] = vals.get((f, disp), 0.0) + float(v)
    for f in Path(d).rglob("*counter_collection.csv"):
        with open(f) as fh:
            for row in csv.DictReader(fh):
                if row.get("Counter_Name") != counter or kernel not in row.get("Kernel_Name", ""):
                    continue
                key = (f, row.get("Dispatch_Id") or row.get("Correlation_Id"))
                vals[key] = vals.get(key, 0.0) + float(row["Counter_Value"])
    if not vals:
        raise SystemExit(f"no {counter} rows for {kernel!r} under {d}")
    v = list(vals.values())
    return sum(v) / len(v), len(v)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--fetch", required=True)
    ap.add_argument("--write", required=True)
    ap.add_argument("--kernel", required=True)
    ap.add_argument("--out", required=True)
    a = ap.parse_args()
    fkb, nf = per_launch(Path(a.fetch), "FETCH_SIZE", a.kernel)
    wkb, nw = per_launch(Path(a.write), "WRITE_SIZE", a.kernel)
    res = {"kernel": a.kernel, "fetch_bytes_per_launch": 2 * fkb * 1024, "write_bytes_per_launch": wkb * 1024,
           "bytes_per_launch": 2 * fkb * 1024 + wkb * 1024, "launches": [nf, nw],
           "correction": "FETCH_SIZE x2 (gfx950 16-B streaming reads), WRITE_SIZE x1; KiB -> bytes"}
    Path(a.out).write_text(json.dumps(res, indent=1))
    print(json.dumps(res))


if __name__ == "__main__":
    main()
