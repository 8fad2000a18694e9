#!/usr/bin/env python3
"""MFMA utilisation and HBM traffic of the top kernels of the default bench, from
rocprofv3 PMC passes, each pass its own run (/opt/skills/guides/MI355X_MICROARCH.md, rocprofv3 PMC slots):

  pass "sq":    SQ_VALU_MFMA_BUSY_CYCLES, SQ_BUSY_CYCLES, GRBM_GUI_ACTIVE   (SQ + GRBM blocks)
  pass "fetch": FETCH_SIZE                                                   (TCC: 3 slots)
  pass "write": WRITE_SIZE                                                   (TCC: 2 slots)

Per kernel (aggregated over its launches in one bench step):
  mfma_busy   = SQ_VALU_MFMA_BUSY_CYCLES / (GRBM_GUI_ACTIVE / 8 x 1024 SIMDs)
                (GRBM_GUI_ACTIVE is reported summed over the 8 XCDs; 256 CUs x 4 SIMDs)
  hbm_bytes   = 2 x FETCH_SIZE + WRITE_SIZE  (KiB -> bytes; FETCH_SIZE x2: gfx950 reports half the bytes
                of 16-B-per-lane streaming reads, incl. LDS-DMA; WRITE_SIZE exact for 16-B stores).  These
                count L2 <-> fabric traffic: Infinity-Cache hits are included, so this is an upper bound on
                HBM bytes.
  hbm_gbps    = hbm_bytes / the kernel's duration in the same pass (profiled runs clock lower: the ratios,
                not the absolute durations, are the point).

Usage (on the GPU box; each pass is a child process, nothing is exec'd):
  python scripts/pmc_top.py run --dir gpurun_out/r3pmc [--bench-args "--steps 1 --warmup 1 ..."]
  python scripts/pmc_top.py summarize --dir gpurun_out/r3pmc --out profiles/r03_pmc_top.json [--top 8]
"""
from __future__ import annotations

import argparse
import csv
import json
import os
import re
import subprocess
import sys
from collections import defaultdict
from pathlib import Path

PASSES = {
    "sq": "SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE",
    "fetch": "FETCH_SIZE",
    "write": "WRITE_SIZE",
}
KERNELS = "gemm2_kernel|gemm_sk_kernel|attn3_kernel|attn3q_kernel|attnw_kernel|gemm_kernel|attn_kernel"   # (adding gn_apply / ln_kernel made the FETCH pass crash inside the profiler, round 3)
SIMDS = 1024
XCDS = 8


def short(name: str) -> str:
    name = re.sub(r"\(anonymous namespace\)::", "", name)
    name = re.sub(r"^void ", "", name)
    return name.split("(")[0][:160]          # drop the argument list: the bench profiler's spelling


def run(d: Path, bench_args: str, timeout: int) -> None:
    d.mkdir(parents=True, exist_ok=True)
    # eager launches: counter collection over replayed HIP graphs segfaulted the profiled process (r3d)
    env = dict(os.environ, TMPDIR="/tmp", IRX_GRAPHS="0")
    for tag, counters in PASSES.items():
        # MFMA kernels only: collecting over every kernel of the bench segfaulted the profiled process inside
        # a GroupNorm launch (r3e), whatever the graph setting
        cmd = (["timeout", "-s", "KILL", str(timeout), "rocprofv3", "--pmc", *counters.split(),
                "--kernel-include-regex", KERNELS,
                "--output-format", "csv", "-d", str(d / tag), "-o", tag, "--", sys.executable, "bench.py"]
               + bench_args.split())
        print("+", " ".join(cmd), flush=True)
        with open(d / f"{tag}.log", "w") as log:
            r = subprocess.run(cmd, stdout=log, stderr=subprocess.STDOUT, env=env)
        if r.returncode != 0:
            raise SystemExit(f"pass {tag} failed ({r.returncode}); see {d / (tag + '.log')}")


def read_pass(d: Path):
    """{(dispatch key) : {counter: value, 'name':..., 'ns': duration}}"""
    rows = {}
    for f in d.rglob("*counter_collection.csv"):
        with open(f) as fh:
            for r in csv.DictReader(fh):
                key = (str(f), r.get("Dispatch_Id") or r.get("Correlation_Id"))
                e = rows.setdefault(key, {"name": r["Kernel_Name"],
                                          "ns": int(r["End_Timestamp"]) - int(r["Start_Timestamp"])})
                e[r["Counter_Name"]] = e.get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
    return rows


def summarize(d: Path, out: Path, top: int) -> dict:
    per = defaultdict(lambda: defaultdict(float))
    for tag in PASSES:
        for e in read_pass(d / tag).values():
            k = per[e["name"]]
            k[f"ns_{tag}"] += e["ns"]
            k[f"n_{tag}"] += 1
            for c, v in e.items():
                if c not in ("name", "ns"):
                    k[c] += v
    kernels = sorted(per.items(), key=lambda kv: -kv[1].get("ns_sq", 0.0))[:top]
    res = []
    for name, k in kernels:
        n = max(k.get("n_sq", 0), 1)
        busy = k.get("SQ_VALU_MFMA_BUSY_CYCLES", 0.0)
        active = k.get("GRBM_GUI_ACTIVE", 0.0) / XCDS
        fetch = 2.0 * k.get("FETCH_SIZE", 0.0) * 1024 / max(k.get("n_fetch", 0), 1)
        write = k.get("WRITE_SIZE", 0.0) * 1024 / max(k.get("n_write", 0), 1)
        t_fetch = k.get("ns_fetch", 0.0) / max(k.get("n_fetch", 0), 1)
        t_write = k.get("ns_write", 0.0) / max(k.get("n_write", 0), 1)
        res.append({
            "kernel": short(name), "launches": int(n),
            "avg_us_sq_pass": round(k.get("ns_sq", 0.0) / n / 1e3, 2),
            "mfma_busy": round(busy / (active * SIMDS), 4) if active else None,
            "clock_ghz": round(active / (k.get("ns_sq", 0.0) / n * n) , 3) if k.get("ns_sq") else None,
            "hbm_read_bytes_per_launch": round(fetch), "hbm_write_bytes_per_launch": round(write),
            "hbm_bytes_per_launch": round(fetch + write),
            "hbm_gbps": round((fetch / t_fetch + write / t_write) if t_fetch and t_write else 0.0, 1),
        })
    doc = {"source": str(d), "note": __doc__.split("\n\n")[1].strip(), "kernels": res}
    out.parent.mkdir(parents=True, exist_ok=True)
    out.write_text(json.dumps(doc, indent=1))
    return doc


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("mode", choices=["run", "summarize"])
    ap.add_argument("--dir", required=True)
    ap.add_argument("--out", default=None)
    ap.add_argument("--top", type=int, default=8)
    ap.add_argument("--timeout", type=int, default=240)
    ap.add_argument("--bench-args", default="--steps 1 --warmup 1 --no-cpu-baseline --no-roofline")
    a = ap.parse_args()
    d = Path(a.dir)
    if a.mode == "run":
        run(d, a.bench_args, a.timeout)
    else:
        doc = summarize(d, Path(a.out or d / "pmc_top.json"), a.top)
        for k in doc["kernels"]:
            print(f"{k['avg_us_sq_pass']:9.1f} us x{k['launches']:4d}  mfma {k['mfma_busy']}  "
                  f"HBM {k['hbm_bytes_per_launch'] / 1e6:8.1f} MB {k['hbm_gbps']:7.1f} GB/s  {k['kernel'][:90]}")


if __name__ == "__main__":
    main()
