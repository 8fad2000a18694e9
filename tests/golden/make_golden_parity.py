#!/usr/bin/env python3
"""Generate tests/golden/parity_cfg0_metrics.json: the CPU reference path's per-image PSNR / SSIM on bench.py's
configs[0] parity images (run once in the build container; the oracle never travels to the GPU box).

The images are bench.synthetic_pairs(4, 512, seed=1000) (clean + noisy 512x512), the weights the seeded random
SD-1.5 state dicts (weights.random_state_dict, seed 0), the path the fp32 CPU restatement of the diffusers img2img
pipeline the reference calls (oracle/pipeline_ref.img2img_ref = src/inference.py:486-495; 20 PNDM steps x strength
0.5, CFG 5.0, seed 42).  Stored per image: PSNR and SSIM of the reference output against the clean image
(metrics.py = scikit-image 0.18.3 restatement, src/metrics.py:82-95 semantics) and a checksum of the output.

Usage:  python tests/golden/make_golden_parity.py [--ref scratch/parity_ref4.npz]
        (--ref: reuse the outputs scripts/parity_stages.py --make-ref saved; else the oracle runs, ~2 min/image)
"""
from __future__ import annotations

import argparse
import hashlib
import json
import sys
from pathlib import Path

import numpy as np

HERE = Path(__file__).resolve().parent
ROOT = HERE.parents[1]
sys.path.insert(0, str(ROOT))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--ref", default=None)
    ap.add_argument("--n", type=int, default=4)
    a = ap.parse_args()
    import bench as B
    from image_restoration_and_enhancement_amd import metrics as M
    if a.ref:
        d = np.load(a.ref)
        clean, ref = d["clean"], d["ref"]
        assert np.array_equal(clean, B.synthetic_pairs(len(ref), 512, seed=1000)[0])
    else:
        from scripts.parity_stages import make_ref
        tmp = HERE / "_parity_tmp.npz"
        make_ref(str(tmp), a.n)
        d = np.load(tmp)
        clean, ref = d["clean"], d["ref"]
        tmp.unlink()
    out = {"workload": "bench.py configs[0] parity images: synthetic_pairs(4, 512, seed=1000), weights seed 0, "
                       "20 PNDM steps x 0.5, CFG 5.0, seed 42, fp32 CPU restatement (oracle/pipeline_ref.py)",
           "psnr_gt": [float(M.psnr(clean[i], ref[i])) for i in range(len(ref))],
           "ssim_gt": [float(M.ssim(clean[i], ref[i])) for i in range(len(ref))],
           "ref_sha256": [hashlib.sha256(ref[i].tobytes()).hexdigest() for i in range(len(ref))]}
    (HERE / "parity_cfg0_metrics.json").write_text(json.dumps(out, indent=1) + "\n")
    print(json.dumps({k: out[k] for k in ("psnr_gt", "ssim_gt")}))


if __name__ == "__main__":
    main()
