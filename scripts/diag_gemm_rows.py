#!/usr/bin/env python3
"""Row-wise batch invariance of the GEMM ops at the UNet's 256x256-image shapes (fp16 / bf16): 16 images of rows as one
call vs 6 + 10 images, for plain GEMMs (+ residual) and the fused GEGLU projection; prints the max |difference|."""
import math
import sys
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
from image_restoration_and_enhancement_amd import _lib as L  # noqa: E402
from image_restoration_and_enhancement_amd.engine import geglu64_order  # noqa: E402
from tests import opref as O  # noqa: E402


def main():
    L.load()
    for o in sys.argv[1:]:
        k, v = o.split("=")
        L.call("irx_set_option", k.encode(), int(v))
    dev = torch.device("cuda")
    g = torch.Generator().manual_seed(0)
    for dt in (torch.float16, torch.bfloat16):
        for (hw, K, N, kind) in [(1024, 320, 2560, "geglu"), (256, 640, 5120, "geglu"), (64, 1280, 10240, "geglu"),
                                 (1024, 1280, 320, "res"), (256, 2560, 640, "res"), (64, 5120, 1280, "res"),
                                 (256, 640, 1920, "plain"), (64, 1280, 3840, "plain"), (64, 1280, 1280, "plain"),
                                 (256, 640, 640, "res"), (1024, 320, 960, "plain")]:
            M = 16 * hw
            A = (torch.randn(M, K, generator=g)).to(dt).to(dev)
            W = (torch.randn(N, K, generator=g) / math.sqrt(K)).to(dt).to(dev)
            R = (torch.randn(M, N, generator=g)).to(dt).to(dev) if kind == "res" else None
            bias = torch.randn(N, generator=g).to(dev)

            def run(a, r):
                if kind == "geglu":
                    Wp, bp = W[geglu64_order(N).to(dev)].contiguous(), bias[geglu64_order(N).to(dev)].contiguous()
                    out = torch.empty(a.shape[0], N // 2, dtype=dt, device=dev)
                    L.call("irx_op_gemm_geglu", O.S(), O.DT[dt], a.shape[0], N, K, O.P(a), O.P(Wp), O.P(bp), O.P(out))
                    return out
                return O.gemm(a, W, bias=bias, residual=r)
            L.call("irx_set_option", b"op_imgs", 16)
            whole = run(A, R)
            c = 6 * hw
            L.call("irx_set_option", b"op_imgs", 6)
            p1 = run(A[:c].contiguous(), R[:c].contiguous() if R is not None else None)
            L.call("irx_set_option", b"op_imgs", 10)
            p2 = run(A[c:].contiguous(), R[c:].contiguous() if R is not None else None)
            L.call("irx_set_option", b"op_imgs", 0)
            parts = torch.cat([p1, p2])
            d = (whole.float() - parts.float()).abs().view(16, hw, -1).amax(dim=(1, 2))
            print(f"{dt} {kind} hw {hw} K {K} N {N}: rows differing {int((d > 0).sum())}/16, max {float(d.max()):.3g}",
                  flush=True)


if __name__ == "__main__":
    main()
