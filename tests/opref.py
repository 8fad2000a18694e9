"""Thin torch wrappers over the single-op C ABI (irx_op_*) used by the GPU parity tests,
plus the fp32 PyTorch-CPU reference of each op."""
from __future__ import annotations

import ctypes as C
import math

import torch
import torch.nn.functional as F

from image_restoration_and_enhancement_amd import _lib as L

DT = {torch.float32: L.IRX_F32, torch.bfloat16: L.IRX_BF16, torch.float16: L.IRX_F16}


def S():
    return C.c_void_p(torch.cuda.current_stream().cuda_stream)


def P(t):
    return None if t is None else C.c_void_p(t.data_ptr())


# ------------------------------------------------------------------ convolution (NHWC)
def conv2d(x0, w_oihw, bias, stride=1, pad=(1, 1), out_hw=None, x1=None, up_hw=None, rowadd=None, residual=None,
           out_f32=False, act=0):
    """x0/x1: NHWC device tensors; w: OIHW (fp32 CPU or device); returns NHWC device tensor."""
    dt = x0.dtype
    N, H, W, C0 = x0.shape
    C1 = x1.shape[3] if x1 is not None else 0
    Co, Ci, KH, KW = w_oihw.shape
    assert Ci == C0 + C1
    wk = w_oihw.permute(0, 2, 3, 1).contiguous().to(device=x0.device, dtype=dt)
    hv, wv = up_hw if up_hw is not None else (H, W)
    if out_hw is None:
        Ho = (hv + 2 * pad[0] - KH) // stride + 1
        Wo = (wv + 2 * pad[1] - KW) // stride + 1
    else:
        Ho, Wo = out_hw
    out = torch.empty((N, Ho, Wo, Co), dtype=torch.float32 if out_f32 else dt, device=x0.device)
    b = bias.float().to(x0.device).contiguous() if bias is not None else None
    L.call("irx_op_conv2d", S(), DT[dt], P(x0), P(x1), C0, C1, N, H, W, hv, wv, P(wk), P(b), Co, KH, KW, stride,
           pad[0], pad[1], Ho, Wo, P(rowadd), rowadd.shape[1] if rowadd is not None else 0, P(residual), P(out),
           int(out_f32), act)
    return out


def gemm(A, Bw, bias=None, alpha=1.0, act=0, residual=None, out_f32=False, batch=1, guard_rows=0):
    """A [M,K] (or [b,M,K]), Bw [N,K] (or [b,N,K]) device tensors -> [M,N].  guard_rows > 0: the output is the head
    of a larger buffer whose trailing rows hold a sentinel, asserted untouched after the call (no write past M)."""
    dt = A.dtype
    if batch > 1:
        _, M, K = A.shape
        N = Bw.shape[1]
        out = torch.empty((batch, M, N), dtype=torch.float32 if out_f32 else dt, device=A.device)
        sA, sB, sC = M * K, N * K, M * N
    else:
        M, K = A.shape
        N = Bw.shape[0]
        if guard_rows:
            buf = torch.full((M + guard_rows, N), 1234.0, dtype=torch.float32 if out_f32 else dt, device=A.device)
            L.call("irx_op_gemm", S(), DT[dt], M, N, K, P(A), K, P(Bw), K, P(buf), N, P(bias), float(alpha), act,
                   P(residual), N, int(out_f32), 1, 0, 0, 0, 0)
            assert bool((buf[M:] == 1234.0).all()), "GEMM wrote past its last output row"
            return buf[:M]
        out = torch.empty((M, N), dtype=torch.float32 if out_f32 else dt, device=A.device)
        sA = sB = sC = 0
    L.call("irx_op_gemm", S(), DT[dt], M, N, K, P(A), K, P(Bw), K, P(out), N, P(bias), float(alpha), act,
           P(residual), N, int(out_f32), batch, sA, sB, sC, sC)
    return out


def group_norm(x0, gamma, beta, eps, groups=32, silu=False, x1=None):
    N, H, W, C0 = x0.shape
    C1 = x1.shape[3] if x1 is not None else 0
    ws = torch.empty(L.load().irx_op_group_norm_ws_bytes(N, H * W, groups), dtype=torch.uint8, device=x0.device)
    out = torch.empty((N, H, W, C0 + C1), dtype=x0.dtype, device=x0.device)
    L.call("irx_op_group_norm", S(), DT[x0.dtype], P(x0), P(x1), C0, C1, N, H * W, groups, float(eps),
           P(gamma), P(beta), int(silu), P(out), P(ws))
    return out


def gn_conv3(x0, gamma, beta, eps, w_oihw, bias, groups=32, silu=True, x1=None, rowadd=None, residual=None,
             query=False):
    """GroupNorm(+SiLU) folded into the halo 3x3 conv (irx_op_gn_conv3); query=True only reports whether the
    shape takes the fused path."""
    import ctypes
    N, H, W, C0 = x0.shape
    C1 = x1.shape[3] if x1 is not None else 0
    Co = w_oihw.shape[0]
    fused = ctypes.c_int(0)
    if query:
        L.call("irx_op_gn_conv3", S(), DT[x0.dtype], None, None, C0, C1, N, H, W, groups, float(eps), None, None,
               int(silu), None, None, Co, None, 0, None, None, None, ctypes.byref(fused))
        return bool(fused.value)
    wk = w_oihw.permute(0, 2, 3, 1).contiguous().to(device=x0.device, dtype=x0.dtype)
    b = bias.float().to(x0.device).contiguous() if bias is not None else None
    nb = L.load().irx_op_gn_conv3_ws_bytes(N, H * W, groups, C0 + C1)
    ws = torch.empty(nb, dtype=torch.uint8, device=x0.device)
    out = torch.empty((N, H, W, Co), dtype=x0.dtype, device=x0.device)
    L.call("irx_op_gn_conv3", S(), DT[x0.dtype], P(x0), P(x1), C0, C1, N, H, W, groups, float(eps), P(gamma),
           P(beta), int(silu), P(wk), P(b), Co, P(rowadd), rowadd.shape[1] if rowadd is not None else 0,
           P(residual), P(out), P(ws), ctypes.byref(fused))
    assert fused.value == 1
    return out


def layer_norm(x, gamma, beta, eps):
    rows, Cc = x.shape
    out = torch.empty_like(x)
    L.call("irx_op_layer_norm", S(), DT[x.dtype], P(x), rows, Cc, float(eps), P(gamma), P(beta), P(out))
    return out


def attention(q, k, v, heads, causal=False):
    """q [B,Lq,C], k/v [B,Lk,C] device tensors (possibly strided views with unit last stride)."""
    B, Lq, Cq = q.shape
    Lk = k.shape[1]
    d = Cq // heads
    o = torch.empty((B, Lq, Cq), dtype=q.dtype, device=q.device)
    L.call("irx_op_attention", S(), DT[q.dtype], B, heads, Lq, Lk, d, P(q), q.stride(1), q.stride(0), P(k),
           k.stride(1), k.stride(0), P(v), v.stride(1), v.stride(0), P(o), Cq, Lq * Cq, 1.0 / math.sqrt(d),
           int(causal))
    return o


def geglu(proj):
    M, F2 = proj.shape
    out = torch.empty((M, F2 // 2), dtype=proj.dtype, device=proj.device)
    L.call("irx_op_geglu", S(), DT[proj.dtype], P(proj), M, F2 // 2, P(out))
    return out


# ------------------------------------------------------------------ references (fp32 CPU)
def ref_attention(q, k, v, heads, causal=False):
    B, Lq, Cq = q.shape
    Lk = k.shape[1]
    d = Cq // heads
    qh = q.float().view(B, Lq, heads, d).transpose(1, 2)
    kh = k.float().reshape(B, Lk, heads, d).transpose(1, 2)
    vh = v.float().reshape(B, Lk, heads, d).transpose(1, 2)
    s = qh @ kh.transpose(-1, -2) / math.sqrt(d)
    if causal:
        s = s + torch.full((Lq, Lk), float("-inf")).triu(1)
    return (s.softmax(-1) @ vh).transpose(1, 2).reshape(B, Lq, Cq)


def rel_err(got, ref):
    got = got.detach().float().cpu()
    ref = ref.detach().float().cpu()
    return float((got - ref).abs().max() / ref.abs().max().clamp_min(1e-12))
