#!/usr/bin/env python3
"""Idle time of the GPU inside the bench's steady-state steps, from a rocprofv3 --kernel-trace CSV of
`bench.py --no-roofline`: a step starts at the step's `img2t_kernel` (the uint8 batch -> VAE input conversion,
once per step), so the intervals between consecutive img2t launches are whole steps.  For the last `--steps` of
them: wall span, busy time (union of kernel intervals), idle time, and the largest gaps with the kernels on
either side (where the host, not the GPU, set the pace).

  python scripts/step_gaps.py kernel_trace.csv [--steps 2] [--top 12]
"""
import argparse
import csv


def short(name: str) -> str:
    n = name.split("(")[0]
    n = n.replace("void ", "").replace("irx::(anonymous namespace)::", "")
    return n[:70]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--steps", type=int, default=2)
    ap.add_argument("--top", type=int, default=12)
    a = ap.parse_args()
    rows = list(csv.DictReader(open(a.trace)))
    ks = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]) for r in rows)
    starts = [s for s, _, n in ks if "img2t_kernel" in n]
    if len(starts) < a.steps + 1:
        # the last step has no successor: end it at the last kernel
        starts = starts + [ks[-1][1] + 1]
    bounds = list(zip(starts[-a.steps - 1:-1], starts[-a.steps:]))
    for i, (t0, t1) in enumerate(bounds):
        sel = [k for k in ks if t0 <= k[0] < t1]
        busy, idle, gaps = 0, 0, []
        cs, ce, cn = sel[0][0], sel[0][1], sel[0][2]
        for s, e, n in sel[1:]:
            if s > ce:
                busy += ce - cs
                idle += s - ce
                gaps.append((s - ce, cn, n))
                cs, ce, cn = s, e, n
            elif e > ce:
                ce, cn = e, n
        busy += ce - cs
        span = t1 - t0
        print(f"step {i}: span {span / 1e6:.2f} ms  busy {busy / 1e6:.2f} ms  idle {idle / 1e6:.2f} ms "
              f"({100 * idle / span:.1f} %)  kernels {len(sel)}  gaps {len(gaps)}")
        gaps.sort(reverse=True)
        for g, before, after in gaps[:a.top]:
            print(f"   {g / 1e3:9.1f} us  after {short(before)}  ->  {short(after)}")
        small = sum(g for g, _, _ in gaps if g < 20e3)
        print(f"   gaps < 20 us: {small / 1e6:.2f} ms over {sum(1 for g, _, _ in gaps if g < 20e3)} gaps")


if __name__ == "__main__":
    main()
