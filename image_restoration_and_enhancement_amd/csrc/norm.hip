// irx — GroupNorm(+SiLU) and LayerNorm for NHWC activations on gfx950.
//
// GroupNorm (ResnetBlock2D norm1/norm2, Transformer2D norm, conv_norm_out, VAE attention norm):
// two HBM-bound passes.  Pass 1 streams pixel chunks with 16-byte vector loads and accumulates
// shifted per-channel sums in fp32, merged as sum / sum of squares in fp64 (no E[x^2]-E[x]^2
// cancellation at 40k-element groups) into per-(image, chunk, group) partials; a small finalize
// kernel folds them into mean/rstd.  Pass 2 folds gamma/beta into one per-channel scale/shift, and writes
// y = x*a + b (optionally SiLU) with 16-byte vector stores.  Up-block inputs are a channel
// concat of two tensors; groups may straddle the seam, so both passes read the two sources.
#include <type_traits>

#include "ops.h"
#include "profile.h"

namespace irx {
namespace {

constexpr int kMaxChunks = 256;   // stats blocks per image (pixels per chunk grows with the image)

int n_chunks(int HW) { return std::min((HW + 63) / 64, kMaxChunks); }
int chunk_pix(int HW) { const int n = n_chunks(HW); return (HW + n - 1) / n; }

// v3 stats: channel slabs (a power of two dividing G, <= 256 16-byte vectors each, >= 2 pixel rows per
// block when C allows); 0 if G is not a power of two <= 64 (the v1 path runs)
int gn_slabs(int C, int vec, int G) {
  if (G <= 0 || G > 64 || (G & (G - 1))) return 0;
  const int nv = C / vec;
  for (int s = 1; s <= G; s *= 2)
    if (nv % s == 0 && (C / s) % (C / G) == 0 && nv / s <= 128) return s;
  for (int s = 1; s <= G; s *= 2)
    if (nv % s == 0 && (C / s) % (C / G) == 0 && nv / s <= 256) return s;
  return 0;
}
// pixel chunks per (image, slab): ~2048 blocks at kCanonImages images, >= 4 pixels per thread, <= kMaxChunks.
// A function of the per-image shape only, so an image's statistics (and bits) do not depend on the batch.
int gn_chunks3(int HW, int slabs, int rows) {
  const int N = kCanonImages;
  const int want = (2048 + N * slabs - 1) / (N * slabs);
  const int most = std::max(1, HW / (4 * rows));
  return std::max(1, std::min(std::min(want, most), kMaxChunks));
}

template <typename T>
__global__ __launch_bounds__(256) void gn_stats_kernel(const T* __restrict__ x0, const T* __restrict__ x1,
                                                       int C0, int C1, int HW, int G, int cpix, double* part) {
  constexpr int VEC = 16 / (int)sizeof(T);
  __shared__ double gs[64], gq[64];
  const int C = C0 + C1;
  const int nv = C / VEC;                      // vectors per pixel
  const int cg = C / G;
  const int n = blockIdx.y, chunk = blockIdx.x;
  const int p0 = chunk * cpix, p1 = min(HW, p0 + cpix);
  if (threadIdx.x < 64) { gs[threadIdx.x] = 0.0; gq[threadIdx.x] = 0.0; }
  __syncthreads();
  // thread -> (vector v, pixel lane r); each thread owns up to 2 vectors (C <= 4096)
  const int rows = nv >= 256 ? 1 : 256 / nv;
  const int r = threadIdx.x / (nv >= 256 ? 256 : nv);
  for (int vb = 0; vb < nv; vb += 256) {
    const int v = vb + (nv >= 256 ? threadIdx.x : threadIdx.x % nv);
    if (v >= nv || r >= rows) continue;
    // fp32 sums of (x - x0), x0 = this thread's first sample per channel (keeps the fp32 partials free of
    // mean^2 cancellation); re-expanded to raw sum / sum of squares in fp64 for the cross-thread merge
    float s[VEC], q[VEC], x0v[VEC];
    const int c = v * VEC;
    const T* src = c < C0 ? x0 + c : x1 + (c - C0);
    const int ld = c < C0 ? C0 : C1;
    int cnt = 0;
    if (p0 + r < p1) {
      Vec16<T>::unpack(*(const uint4*)(src + ((long)n * HW + p0 + r) * ld), x0v);
    } else {
#pragma unroll
      for (int e = 0; e < VEC; ++e) x0v[e] = 0.f;
    }
#pragma unroll
    for (int e = 0; e < VEC; ++e) { s[e] = 0.f; q[e] = 0.f; }
    for (int p = p0 + r; p < p1; p += rows) {
      const uint4 u = *(const uint4*)(src + ((long)n * HW + p) * ld);
      float f[VEC];
      Vec16<T>::unpack(u, f);
#pragma unroll
      for (int e = 0; e < VEC; ++e) {
        const float dv = f[e] - x0v[e];
        s[e] += dv;
        q[e] = fmaf(dv, dv, q[e]);
      }
      ++cnt;
    }
#pragma unroll
    for (int e = 0; e < VEC; ++e) {
      const int grp = (c + e) / cg;
      const double xs = x0v[e], ds = s[e];
      atomicAdd(&gs[grp], cnt * xs + ds);
      atomicAdd(&gq[grp], cnt * xs * xs + 2.0 * xs * ds + (double)q[e]);
    }
  }
  __syncthreads();
  if (threadIdx.x < G) {
    double* o = part + (((long)n * gridDim.x + chunk) * G + threadIdx.x) * 2;
    o[0] = gs[threadIdx.x];
    o[1] = gq[threadIdx.x];
  }
}

// GroupNorm statistics, v3: grid (pixel chunk, image, channel slab) sized to >= ~2048 blocks whatever the
// resolution (the 8x8 / 16x16 UNet levels have too few pixels to fill the chip with pixel chunks alone).
// Thread = one 16-byte channel vector x a pixel stride; 4 pixel loads in flight per thread; shifted fp32
// sums per channel, expanded to raw fp64 (sum, sum of squares) in LDS; 8 threads per group fold the
// block's channels/rows into one (sum, sum of squares) partial per (image, chunk, group);
// gn_finalize3_kernel folds the partials into (mean, rstd).
template <typename T>
__global__ __launch_bounds__(256) void gn_stats3_kernel(const T* __restrict__ x0, const T* __restrict__ x1, int C0,
                                                        int C1, int HW, int G, int ppc, double* part) {
  constexpr int VEC = 16 / (int)sizeof(T);
  __shared__ double Sl[256 * VEC], Ql[256 * VEC];
  const int C = C0 + C1, slabs = gridDim.z, Cs = C / slabs, nvs = Cs / VEC;
  const int rows = 256 / nvs;
  const int n = blockIdx.y, chunk = blockIdx.x, slab = blockIdx.z, nch = gridDim.x;
  const int t = threadIdx.x, v = t % nvs, r = t / nvs;
  const int p0 = chunk * ppc, p1 = min(HW, p0 + ppc);
  if (r < rows) {
    const int c = slab * Cs + v * VEC;
    const T* src = c < C0 ? x0 + (long)n * HW * C0 + c : x1 + (long)n * HW * C1 + (c - C0);
    const long ld = c < C0 ? C0 : C1;
    float s[VEC], q[VEC], xs[VEC];
#pragma unroll
    for (int e = 0; e < VEC; ++e) { s[e] = 0.f; q[e] = 0.f; xs[e] = 0.f; }
    int p = p0 + r, cnt = 0;
    if (p < p1) Vec16<T>::unpack(*(const uint4*)(src + p * ld), xs);
    auto acc = [&](const uint4& u) {
      float f[VEC];
      Vec16<T>::unpack(u, f);
#pragma unroll
      for (int e = 0; e < VEC; ++e) {
        const float dv = f[e] - xs[e];
        s[e] += dv;
        q[e] = fmaf(dv, dv, q[e]);
      }
    };
    for (; p + 3 * rows < p1; p += 4 * rows) {
      const uint4 u0 = *(const uint4*)(src + p * ld);
      const uint4 u1 = *(const uint4*)(src + (p + rows) * ld);
      const uint4 u2 = *(const uint4*)(src + (p + 2 * rows) * ld);
      const uint4 u3 = *(const uint4*)(src + (p + 3 * rows) * ld);
      acc(u0); acc(u1); acc(u2); acc(u3);
      cnt += 4;
    }
    for (; p < p1; p += rows, ++cnt) acc(*(const uint4*)(src + p * ld));
#pragma unroll
    for (int e = 0; e < VEC; ++e) {
      const double x = xs[e], sd = s[e];
      Sl[t * VEC + e] = cnt * x + sd;
      Ql[t * VEC + e] = cnt * x * x + 2.0 * x * sd + (double)q[e];
    }
  }
  __syncthreads();
  // fold rows x channels of each group (8 threads per group; G / slabs <= 32 groups in this slab)
  const int Gs = G / slabs, cg = C / G;
  {
    const int gl = t >> 3, sub = t & 7;
    double a = 0.0, b = 0.0;
    if (gl < Gs)
      for (int i = sub; i < rows * cg; i += 8) {
        const int rr = i / cg, ch = gl * cg + (i - rr * cg);
        a += Sl[rr * Cs + ch];
        b += Ql[rr * Cs + ch];
      }
#pragma unroll
    for (int o = 4; o > 0; o >>= 1) { a += __shfl_xor(a, o); b += __shfl_xor(b, o); }
    if (gl < Gs && sub == 0)
      *(double2*)(part + (((long)n * nch + chunk) * G + slab * Gs + gl) * 2) = make_double2(a, b);
  }
}

// per (image, group): fold the (chunk, slab) partials of gn_stats3 into (mean, rstd); 256 threads per
// image, 256/G threads per group with 8 loads in flight each, shuffle-combined.  (A separate launch: an
// in-kernel last-arriver finalize serialises ~2048 same-address arrival atomics, ~20 us at batch 16.)
// Then every channel's scale / shift (gn_ab_store) for gn_apply_kernel or a GroupNorm-fused conv.
__global__ __launch_bounds__(256) void gn_finalize3_kernel(const double* __restrict__ part, int nch, int G,
                                                           double cnt, float eps, float2* __restrict__ mr, int C,
                                                           const float* __restrict__ gamma,
                                                           const float* __restrict__ beta, float2* __restrict__ ab) {
  __shared__ float2 gmr[64];
  const int n = blockIdx.x, t = threadIdx.x;
  const int per = 256 / G;                 // power of two (host check)
  const int g = t / per, sub = t % per;
  double a = 0.0, b = 0.0;
  for (int base = sub; base < nch; base += 8 * per) {
    double2 v[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const int ch = min(base + u * per, nch - 1);
      v[u] = *(const double2*)(part + (((long)n * nch + ch) * G + g) * 2);
    }
#pragma unroll
    for (int u = 0; u < 8; ++u)
      if (base + u * per < nch) { a += v[u].x; b += v[u].y; }
  }
  for (int o = per / 2; o > 0; o >>= 1) { a += __shfl_xor(a, o); b += __shfl_xor(b, o); }
  if (sub == 0) {
    const double mean = a / cnt;
    double var = b / cnt - mean * mean;
    if (var < 0.0) var = 0.0;
    const float2 r = make_float2((float)mean, (float)(1.0 / sqrt(var + (double)eps)));
    mr[n * G + g] = r;
    gmr[g] = r;
  }
  __syncthreads();
  const int cg = C / G;
  for (int c = t; c < C; c += 256) {
    const float2 r = gmr[c / cg];
    const float sc = r.y * gamma[c];
    ab[(long)n * C + c] = make_float2(sc, fmaf(-r.x, sc, beta[c]));
  }
}

// One (image n, group g)'s statistics from producer partials (GemmArgs::gn_part): 32 lanes (sub = lane in the group)
// fold the image's row-block partials of the group's channels (x0 then x1, fixed order) in fp64, an xor-shuffle
// sums the lanes, and every lane returns (mean, rstd).  The one definition gn_finalize_parts_kernel and gn_fa_kernel
// share (bit-identical statistics on either path).  Called by every lane of the wave (the shuffles).
__device__ __forceinline__ float2 gn_parts_fold(const double2* __restrict__ p0, int C0, int rpi0,
                                                const double2* __restrict__ p1, int C1, int rpi1, int n, int g,
                                                bool valid, int cg, int sub, double cnt, float eps) {
  double a = 0.0, b = 0.0;
  if (valid) {
    // the group's channels [g*cg, g*cg + cg) split at the concat seam: c0s channels from x0, the rest from x1
    const int cb = g * cg, c0s = max(0, min(cg, C0 - cb));
    const int tot0 = rpi0 * c0s, tot1 = rpi1 * (cg - c0s);
    // item i = (row block i / cs, channel i % cs) walked with an incremental (row, channel) pair: no divide per item
    auto fold = [&](const double2* __restrict__ p, int rpi, int Cs, int cbase, int cs, int tot) {
      if (tot <= 0) return;
      int r = sub / cs, ch = sub - r * cs;
      const int dr = 32 / cs, dch = 32 - dr * cs;
      const double2* base = p + (long)n * rpi * Cs + cbase;
#pragma unroll 4
      for (int i = sub; i < tot; i += 32) {
        const double2 v = base[(long)r * Cs + ch];
        a += v.x;
        b += v.y;
        r += dr;
        ch += dch;
        if (ch >= cs) { ch -= cs; ++r; }
      }
    };
    fold(p0, rpi0, C0, cb, c0s, tot0);
    const int c1b = cb + c0s - C0, c1s = cg - c0s;
    fold(p1, rpi1, C1, c1b, c1s, tot1);
  }
#pragma unroll
  for (int o = 16; o > 0; o >>= 1) { a += __shfl_xor(a, o); b += __shfl_xor(b, o); }
  const double mean = a / cnt;
  double var = b / cnt - mean * mean;
  if (var < 0.0) var = 0.0;
  return make_float2((float)mean, (float)(1.0 / sqrt(var + (double)eps)));
}

// GroupNorm from producer partials: per (image, group of 8 GroupNorm groups) block, 32 threads per group
// (gn_parts_fold) -> (mean, rstd) -> the channels' scale / shift.  Replaces the statistics pass over the tensor.
__global__ __launch_bounds__(256) void gn_finalize_parts_kernel(const double2* __restrict__ p0, int C0, int rpi0,
                                                                const double2* __restrict__ p1, int C1, int rpi1,
                                                                int G, double cnt, float eps,
                                                                const float* __restrict__ gamma,
                                                                const float* __restrict__ beta,
                                                                float2* __restrict__ ab, float2* __restrict__ mr) {
  __shared__ float2 gmr[8];
  const int n = blockIdx.x, t = threadIdx.x;
  const int C = C0 + C1, cg = C / G;
  const int gl = t >> 5, sub = t & 31, g = blockIdx.y * 8 + gl;
  // this thread's output channel's gamma / beta, loaded up front (their latency hides under the fold)
  const int c0 = blockIdx.y * 8 * cg, c1 = min(C, c0 + 8 * cg);
  const bool own = c0 + t < c1 && 8 * cg <= 256;
  const float gam = own ? gamma[c0 + t] : 0.f, bet = own ? beta[c0 + t] : 0.f;
  const float2 r = gn_parts_fold(p0, C0, rpi0, p1, C1, rpi1, n, g, g < G, cg, sub, cnt, eps);
  if (sub == 0 && g < G) {
    gmr[gl] = r;
    if (mr) mr[(long)n * G + g] = r;
  }
  __syncthreads();
  if (8 * cg <= 256) {
    if (own) {
      const float2 q = gmr[t / cg];
      const float sc = q.y * gam;
      ab[(long)n * C + c0 + t] = make_float2(sc, fmaf(-q.x, sc, bet));
    }
  } else {
    for (int c = c0 + t; c < c1; c += 256) {
      const float2 q = gmr[(c - c0) / cg];
      const float sc = q.y * gamma[c];
      ab[(long)n * C + c] = make_float2(sc, fmaf(-q.x, sc, beta[c]));
    }
  }
}

// GroupNorm from producer partials, statistics and application in ONE launch (option gn_fa): block = (image n,
// GPB consecutive groups, pixel slice); its lanes fold the groups' partials exactly as gn_finalize_parts_kernel does
// (gn_parts_fold), the channels' scale / shift go to LDS, then the block applies them (gn_act, as gn_apply_kernel) to
// its channels of the slice's pixels, 16-byte chunks, four loads in flight per thread.  Bit-identical to
// gn_finalize_parts_kernel + gn_apply_kernel; one launch and one tiny kernel's ramp / drain fewer per GroupNorm.  The
// S slices of an image re-fold the same partials (a few KiB from L2 per block).  1-D grid of G / GPB x N x S blocks;
// xmap (host: N * S % 8 == 0): the G / GPB blocks of one (image, slice) are consecutive blocks of ONE XCD (blocks
// are dealt to the 8 XCDs round-robin), so the 16-byte pieces of a pixel's channels meet in one L2.
template <typename T>
__global__ __launch_bounds__(256) void gn_fa_kernel(const double2* __restrict__ p0, int C0, int rpi0,
                                                    const double2* __restrict__ p1, int C1, int rpi1, int G, int gpb,
                                                    double cnt, float eps, const float* __restrict__ gamma,
                                                    const float* __restrict__ beta, const T* __restrict__ x0,
                                                    const T* __restrict__ x1, int HW, int S, int xmap, int silu,
                                                    T* __restrict__ out) {
  constexpr int VEC = 16 / (int)sizeof(T);
  __shared__ float2 gmr[8];
  __shared__ float2 sab[256];
  const int ngb = G / gpb, L = blockIdx.x;
  int gb, u;
  if (xmap) {
    const int j = L >> 3;
    gb = j % ngb;
    u = (j / ngb) * 8 + (L & 7);
  } else {
    gb = L % ngb;
    u = L / ngb;
  }
  const int n = u / S, sl = u - n * S;
  const int hws = (HW + S - 1) / S, plo = sl * hws, np = max(0, min(HW, plo + hws) - plo);
  const int t = threadIdx.x;
  const int C = C0 + C1, cg = C / G;
  const int gl = t >> 5, sub = t & 31, g = gb * gpb + gl;
  const int c0 = gb * gpb * cg, nc = gpb * cg;
  const float gam = t < nc ? gamma[c0 + t] : 0.f, bet = t < nc ? beta[c0 + t] : 0.f;
  const float2 r = gn_parts_fold(p0, C0, rpi0, p1, C1, rpi1, n, g, gl < gpb, cg, sub, cnt, eps);
  if (sub == 0 && gl < gpb) gmr[gl] = r;
  __syncthreads();
  if (t < nc) {
    const float2 q = gmr[t / cg];
    const float sc = q.y * gam;
    sab[t] = make_float2(sc, fmaf(-q.x, sc, bet));
  }
  __syncthreads();
  const int nch = nc / VEC, tot = np * nch;
  // chunk idx = pp * nch + k (pixel pp of the slice, 16-byte channel chunk k): each thread steps idx by 256, i.e.
  // (pp, k) by (256 / nch, 256 % nch) with one carry — no integer division per chunk (nch <= 32: nc <= 256)
  const int dp = 256 / nch, dk = 256 - dp * nch;
  auto adv = [&](int& pp, int& k) {
    pp += dp;
    k += dk;
    if (k >= nch) { k -= nch; ++pp; }
  };
  auto src_at = [&](int pp, int k) -> const T* {
    const int p = plo + pp, c = c0 + k * VEC;
    return c < C0 ? x0 + ((long)n * HW + p) * C0 + c : x1 + ((long)n * HW + p) * C1 + (c - C0);
  };
  auto one = [&](const uint4& u, int pp, int k) {
    float f[VEC];
    Vec16<T>::unpack(u, f);
#pragma unroll
    for (int e = 0; e < VEC; ++e) {
      const float2 q = sab[k * VEC + e];
      f[e] = gn_act(f[e], q.x, q.y, silu);
    }
    *(uint4*)(out + ((long)n * HW + plo + pp) * C + c0 + k * VEC) = Vec16<T>::pack(f);
  };
  int idx = t, pp = t / nch, k = t - (t / nch) * nch;
  for (; idx + 3 * 256 < tot; idx += 4 * 256) {   // four 16-byte loads in flight per thread
    int p1 = pp, k1 = k;
    adv(p1, k1);
    int p2 = p1, k2 = k1;
    adv(p2, k2);
    int p3 = p2, k3 = k2;
    adv(p3, k3);
    const uint4 u0 = *(const uint4*)src_at(pp, k);
    const uint4 u1 = *(const uint4*)src_at(p1, k1);
    const uint4 u2 = *(const uint4*)src_at(p2, k2);
    const uint4 u3 = *(const uint4*)src_at(p3, k3);
    one(u0, pp, k); one(u1, p1, k1); one(u2, p2, k2); one(u3, p3, k3);
    pp = p3;
    k = k3;
    adv(pp, k);
  }
  for (; idx < tot; idx += 256) {
    const uint4 u = *(const uint4*)src_at(pp, k);
    one(u, pp, k);
    adv(pp, k);
  }
}

// per-channel scale / shift from (mean, rstd) (after the v1 finalize)
__global__ __launch_bounds__(256) void gn_ab_kernel(const float2* __restrict__ mr, int G, int C,
                                                    const float* __restrict__ gamma, const float* __restrict__ beta,
                                                    float2* __restrict__ ab) {
  const int n = blockIdx.x, cg = C / G;
  for (int c = threadIdx.x; c < C; c += 256) {
    const float2 r = mr[n * G + c / cg];
    const float sc = r.y * gamma[c];
    ab[(long)n * C + c] = make_float2(sc, fmaf(-r.x, sc, beta[c]));
  }
}

// per (image, group): fold the chunk partials into (mean, rstd) once
__global__ __launch_bounds__(64) void gn_finalize_kernel(const double* __restrict__ part, int nchunk, int G,
                                                         double cnt, float eps, float2* __restrict__ mr) {
  const int n = blockIdx.x, g = threadIdx.x;
  if (g >= G) return;
  double s = 0.0, q = 0.0;
  const double* p = part + ((long)n * nchunk) * G * 2 + g * 2;
  for (int c = 0; c < nchunk; ++c) { s += p[(long)c * G * 2]; q += p[(long)c * G * 2 + 1]; }
  const double mean = s / cnt;
  double var = q / cnt - mean * mean;
  if (var < 0.0) var = 0.0;
  mr[n * G + g] = make_float2((float)mean, (float)(1.0 / sqrt(var + (double)eps)));
}

template <typename T>
__global__ __launch_bounds__(256) void gn_apply_kernel(const T* __restrict__ x0, const T* __restrict__ x1, int C0,
                                                       int C1, int HW, const float2* __restrict__ abg, int silu,
                                                       T* __restrict__ out, int pix_per_block) {
  constexpr int VEC = 16 / (int)sizeof(T);
  const int C = C0 + C1;
  const int n = blockIdx.y;
  const float2* ab = abg + (long)n * C;
  // thread -> fixed 16-byte channel chunk (its scale/shift held in registers) x a pixel stride
  const int nv = C / VEC;
  const int rows = nv >= (int)blockDim.x ? 1 : blockDim.x / nv;
  const int r = threadIdx.x / (nv >= (int)blockDim.x ? blockDim.x : nv);
  const int p0 = blockIdx.x * pix_per_block;
  const int p1 = min(HW, p0 + pix_per_block);
  for (int vb = 0; vb < nv; vb += blockDim.x) {
    const int v = vb + (nv >= (int)blockDim.x ? threadIdx.x : threadIdx.x % nv);
    if (v >= nv || r >= rows) continue;
    const int c = v * VEC;
    float sc[VEC], sh[VEC];
#pragma unroll
    for (int e = 0; e < VEC; ++e) { const float2 v = ab[c + e]; sc[e] = v.x; sh[e] = v.y; }
    const T* src = c < C0 ? x0 + (long)n * HW * C0 + c : x1 + (long)n * HW * C1 + (c - C0);
    const int ld = c < C0 ? C0 : C1;
    T* dst = out + (long)n * HW * C + c;
    auto one = [&](const uint4& u, int p) {
      float f[VEC];
      Vec16<T>::unpack(u, f);
#pragma unroll
      for (int e = 0; e < VEC; ++e) f[e] = gn_act(f[e], sc[e], sh[e], silu);
      *(uint4*)(dst + (long)p * C) = Vec16<T>::pack(f);
    };
    int p = p0 + r;
    for (; p + 3 * rows < p1; p += 4 * rows) {   // four 16-byte loads in flight per thread
      const uint4 u0 = *(const uint4*)(src + (long)p * ld);
      const uint4 u1 = *(const uint4*)(src + (long)(p + rows) * ld);
      const uint4 u2 = *(const uint4*)(src + (long)(p + 2 * rows) * ld);
      const uint4 u3 = *(const uint4*)(src + (long)(p + 3 * rows) * ld);
      one(u0, p); one(u1, p + rows); one(u2, p + 2 * rows); one(u3, p + 3 * rows);
    }
    for (; p < p1; p += rows) one(*(const uint4*)(src + (long)p * ld), p);
  }
}

// LayerNorm: one wave per row, row held in registers, two-pass mean/var in fp32.  RPW rows per wave with all
// of their 16-byte loads issued before the first row's reductions (more bytes in flight per wave).
// MODE 0: y = ((x - mean) * rstd) * gamma + beta; 1: no affine; 2: statistics only (rstd, rstd * mean) per row
template <typename T, int MAXV, int RPW, int MODE>
__global__ __launch_bounds__(256) void ln_kernel(const T* __restrict__ x, long ldx, int rows, int C, float eps,
                                                 const float* __restrict__ gamma, const float* __restrict__ beta,
                                                 T* __restrict__ out, long ldo, float2* __restrict__ stats) {
  constexpr int VEC = 16 / (int)sizeof(T);
  const int lane = threadIdx.x & 63;
  const int row0 = (blockIdx.x * 4 + (threadIdx.x >> 6)) * RPW;
  if (row0 >= rows) return;
  const int nv = C / VEC;
  uint4 raw[RPW][MAXV];
#pragma unroll
  for (int k = 0; k < RPW; ++k)
#pragma unroll
    for (int i = 0; i < MAXV; ++i) {
      const int v = lane + 64 * i;
      if (v < nv && row0 + k < rows) raw[k][i] = *(const uint4*)(x + (long)(row0 + k) * ldx + v * VEC);
    }
#pragma unroll
  for (int k = 0; k < RPW; ++k) {
    const int row = row0 + k;
    if (row >= rows) break;
    float f[MAXV][VEC];
    float s = 0.f;
#pragma unroll
    for (int i = 0; i < MAXV; ++i) {
      const int v = lane + 64 * i;
      if (v < nv) {
        Vec16<T>::unpack(raw[k][i], f[i]);
#pragma unroll
        for (int e = 0; e < VEC; ++e) s += f[i][e];
      }
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) s += __shfl_xor(s, o);
    const float mean = s / C;
    float q = 0.f;
#pragma unroll
    for (int i = 0; i < MAXV; ++i) {
      const int v = lane + 64 * i;
      if (v < nv) {
#pragma unroll
        for (int e = 0; e < VEC; ++e) { const float dd = f[i][e] - mean; q = fmaf(dd, dd, q); }
      }
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) q += __shfl_xor(q, o);
    const float rstd = rsqrtf(q / C + eps);
    if constexpr (MODE == 2) {   // statistics only (the folded projections' epilogue applies them)
      if (lane == 0) stats[row] = make_float2(rstd, rstd * mean);
      continue;
    }
#pragma unroll
    for (int i = 0; i < MAXV; ++i) {
      const int v = lane + 64 * i;
      if (v < nv) {
        float y[VEC];
#pragma unroll
        for (int e = 0; e < VEC; ++e) {
          const int c = v * VEC + e;
          if constexpr (MODE == 0) y[e] = fmaf((f[i][e] - mean) * rstd, gamma[c], beta[c]);
          else y[e] = (f[i][e] - mean) * rstd;
        }
        *(uint4*)(out + (long)row * ldo + v * VEC) = Vec16<T>::pack(y);
      }
    }
  }
}

constexpr int kMaxC = 8192;

// statistics of the (two-source) tensor -> per-channel scale / shift `ab` [N][C]
template <typename T>
void gn_stats_t(const void* x0, const void* x1, int C0, int C1, int N, int HW, int G, float eps, const float* gamma,
                const float* beta, float2* ab, void* ws, hipStream_t s) {
  const int nch = n_chunks(HW);
  double* part = (double*)ws;
  float2* mr = (float2*)(part + (size_t)N * kMaxChunks * G * 2);
  const int C = C0 + C1;
  const int VEC = 16 / (int)sizeof(T);
  const int slabs = gn_slabs(C, VEC, G);
  ProfScope ps(prof_on() ? std::string("irx::(anonymous namespace)::gn_stats3_kernel") : std::string(), 0.0, s);
  if (g_gn_v2 && N <= 4096 && slabs > 0) {
    const int rows3 = 256 / (C / slabs / VEC);
    const int nch3 = gn_chunks3(HW, slabs, rows3);
    gn_stats3_kernel<T><<<dim3(nch3, N, slabs), 256, 0, s>>>(
        (const T*)x0, (const T*)x1, C0, C1, HW, G, (HW + nch3 - 1) / nch3, part);
    IRX_LAUNCH_CHECK();
    gn_finalize3_kernel<<<N, 256, 0, s>>>(part, nch3, G, (double)HW * (C / G), eps, mr, C, gamma, beta, ab);
    IRX_LAUNCH_CHECK();
  } else {
    gn_stats_kernel<T><<<dim3(nch, N), 256, 0, s>>>((const T*)x0, (const T*)x1, C0, C1, HW, G, chunk_pix(HW),
                                                    part);
    IRX_LAUNCH_CHECK();
    gn_finalize_kernel<<<N, 64, 0, s>>>(part, nch, G, (double)HW * (C / G), eps, mr);
    IRX_LAUNCH_CHECK();
    gn_ab_kernel<<<N, 256, 0, s>>>(mr, G, C, gamma, beta, ab);
    IRX_LAUNCH_CHECK();
  }
}

float2* gn_ab_ws(void* ws, int N, int G) {
  return (float2*)((char*)ws + (size_t)N * kMaxChunks * G * 2 * sizeof(double) + (size_t)N * G * sizeof(float2));
}

template <typename T>
void gn_t(const void* x0, const void* x1, int C0, int C1, int N, int HW, int G, float eps, const float* gamma,
          const float* beta, int silu, void* out, void* ws, hipStream_t s, const double* p0 = nullptr, int r0 = 0,
          const double* p1 = nullptr, int r1 = 0) {
  float2* ab = gn_ab_ws(ws, N, G);
  if (p0 && g_gn_fa && HW <= (g_gn_fa == 1 ? 256 : g_gn_fa)) {
    // statistics + application in one launch (gn_fa_kernel); GPB groups per block so that a block's channels are
    // whole 16-byte chunks.  Small levels (HW <= 256): one block per (image, GPB groups); larger ones (gn_fa = an
    // HW bound > 256) split each image's pixels into S slices, S so that the grid has ~2048 blocks
    const int C = C0 + C1, cg = C / G, VEC = 16 / (int)sizeof(T);
    int gpb = 1;
    while (gpb <= 8 && ((gpb * cg) % VEC != 0 || G % gpb != 0)) gpb *= 2;
    if (gpb <= 8 && gpb * cg <= 256) {
      if (HW > 256 && g_gn_fa_wide) {   // sliced levels: the widest valid channel span (longer 16-byte runs per pixel)
        for (int q = gpb * 2; q <= 8 && G % q == 0 && q * cg <= 256; q *= 2) gpb = q;
      }
      const long base = (long)(G / gpb) * N;
      int S = 1;
      if (HW > 256) {
        const long want = g_gn_fa_blocks;
        while ((long)S * 2 * base <= want && HW / (S * 2) >= 64) S *= 2;
      }
      const int xmap = ((long)N * S) % 8 == 0;
      ProfScope ps(prof_on() ? std::string("irx::(anonymous namespace)::gn_fa_kernel") : std::string(), 0.0, s);
      gn_fa_kernel<T><<<dim3((unsigned)(base * S)), 256, 0, s>>>((const double2*)p0, C0, HW / r0, (const double2*)p1,
                                                                 C1, r1 ? HW / r1 : 0, G, gpb, (double)HW * cg, eps,
                                                                 gamma, beta, (const T*)x0, (const T*)x1, HW, S, xmap,
                                                                 silu, (T*)out);
      IRX_LAUNCH_CHECK();
      return;
    }
  }
  if (p0) {
    ProfScope ps(prof_on() ? std::string("irx::(anonymous namespace)::gn_finalize_parts_kernel") : std::string(),
                 0.0, s);
    gn_finalize_parts_kernel<<<dim3(N, (G + 7) / 8), 256, 0, s>>>((const double2*)p0, C0, HW / r0,
                                                                  (const double2*)p1, C1, r1 ? HW / r1 : 0, G,
                                                                  (double)HW * ((C0 + C1) / G), eps, gamma, beta,
                                                                  ab, nullptr);
    IRX_LAUNCH_CHECK();
  } else {
    gn_stats_t<T>(x0, x1, C0, C1, N, HW, G, eps, gamma, beta, ab, ws, s);
  }
  const int C = C0 + C1;
  const int VEC = 16 / (int)sizeof(T);
  // ~16 pixels per thread per block, one fixed channel chunk per thread
  const int nv = C / VEC;
  const int rows = nv >= 256 ? 1 : 256 / nv;
  // pixels per thread: up to 16, fewer when the tensor is small, so the grid still has ~2048 blocks
  int ppt = std::max(1, std::min(16, (int)((long)N * HW / ((long)rows * 2048))));
  if (ppt >= 4) ppt &= ~3;   // whole groups of four loads in flight
  const int ppb = rows * ppt;
  ProfScope ps(prof_on() ? std::string("irx::(anonymous namespace)::gn_apply_kernel") : std::string(), 0.0, s);
  gn_apply_kernel<T><<<dim3((HW + ppb - 1) / ppb, N), 256, 0, s>>>((const T*)x0, (const T*)x1, C0, C1, HW, ab, silu,
                                                                  (T*)out, ppb);
  IRX_LAUNCH_CHECK();
}

template <typename T>
void ln_t(const void* x, long ldx, int rows, int C, float eps, const float* gamma, const float* beta, void* out,
          long ldo, hipStream_t s, float2* stats = nullptr) {
  const int VEC = 16 / (int)sizeof(T);
  const int nv = C / VEC;
  dim3 block(256);
  ProfScope ps(prof_on() ? std::string(stats ? "irx::(anonymous namespace)::ln_kernel(stats)"
                                              : "irx::(anonymous namespace)::ln_kernel") : std::string(), 0.0, s);
  // rows per wave: 4 while the row is <= 2 vectors per lane (fill the chip first: >= ~2048 blocks), else 2 / 1
  auto grid = [&](int rpw) { return dim3((rows + 4 * rpw - 1) / (4 * rpw)); };
  auto launch = [&](auto mode) {
    constexpr int MO = decltype(mode)::value;
    if (nv <= 64) {
      if (rows >= 4 * 4 * 2048) ln_kernel<T, 1, 4, MO><<<grid(4), block, 0, s>>>((const T*)x, ldx, rows, C, eps, gamma, beta, (T*)out, ldo, stats);
      else ln_kernel<T, 1, 1, MO><<<grid(1), block, 0, s>>>((const T*)x, ldx, rows, C, eps, gamma, beta, (T*)out, ldo, stats);
    } else if (nv <= 128) {
      if (rows >= 4 * 2 * 2048) ln_kernel<T, 2, 2, MO><<<grid(2), block, 0, s>>>((const T*)x, ldx, rows, C, eps, gamma, beta, (T*)out, ldo, stats);
      else ln_kernel<T, 2, 1, MO><<<grid(1), block, 0, s>>>((const T*)x, ldx, rows, C, eps, gamma, beta, (T*)out, ldo, stats);
    } else if (nv <= 256) {
      ln_kernel<T, 4, 1, MO><<<grid(1), block, 0, s>>>((const T*)x, ldx, rows, C, eps, gamma, beta, (T*)out, ldo, stats);
    } else if (nv <= 512) {
      ln_kernel<T, 8, 1, MO><<<grid(1), block, 0, s>>>((const T*)x, ldx, rows, C, eps, gamma, beta, (T*)out, ldo, stats);
    } else {
      throw Error("layer_norm: C too large");
    }
  };
  if (stats) launch(std::integral_constant<int, 2>{});
  else if (gamma) launch(std::integral_constant<int, 0>{});
  else launch(std::integral_constant<int, 1>{});
  IRX_LAUNCH_CHECK();
}

// GroupNorm folded into per-image projection weights (gn_fold_weights): one wave per (output row n, image).
// GN(x)_k = a_k x_k + b_k with b_k = beta_k - mean_g(k) a_k; the GEMM multiplies x by the STORED o_k = round(W_k a_k),
// so the bias is formed with those same rounded weights: bias + sum_k (W_k beta_k - o_k mean_g(k)).  The group mean
// then cancels exactly against the GEMM's sum_k o_k x_k and only the normalised part (x_k - mean) meets the weight
// rounding — the error of the unfused path, independent of |mean| / std.
template <typename T>
__global__ __launch_bounds__(64) void gn_fold_weights_kernel(const T* __restrict__ W, const float* __restrict__ bias,
                                                             const float2* __restrict__ ab,
                                                             const float* __restrict__ beta,
                                                             const float2* __restrict__ mr, int G, int N, int K,
                                                             T* __restrict__ Wo, float* __restrict__ bo) {
  const int n = blockIdx.x, img = blockIdx.y, lane = threadIdx.x;
  const int cg = K / G;
  const T* w = W + (long)n * K;
  const float2* a = ab + (long)img * K;
  const float2* m = mr + (long)img * G;
  T* wo = Wo + ((long)img * N + n) * K;
  float acc = 0.f;
  for (int k0 = lane * 8; k0 < K; k0 += 512) {
    float f[8], o[8];
    Vec16<T>::unpack(*(const uint4*)(w + k0), f);
#pragma unroll
    for (int e = 0; e < 8; ++e) o[e] = f[e] * a[k0 + e].x;
    const uint4 packed = Vec16<T>::pack(o);
    *(uint4*)(wo + k0) = packed;
    Vec16<T>::unpack(packed, o);   // the weights as stored
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const int k = k0 + e;
      acc = fmaf(f[e], beta[k], acc);
      acc = fmaf(-o[e], m[k / cg].x, acc);
    }
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) acc += __shfl_xor(acc, o);
  if (lane == 0) bo[(long)img * N + n] = (bias ? bias[n] : 0.f) + acc;
}

}  // namespace

const float2* gn_mr_ws(const void* ws, int N, int G) {   // (mean, rstd) per (image, group) of the last stats pass
  return (const float2*)((const char*)ws + (size_t)N * kMaxChunks * G * 2 * sizeof(double));
}

void group_norm_parts_ab(int C0, int N, int HW, int G, float eps, const float* gamma, const float* beta,
                         const double* p0, int r0, float2* ab, float2* mr, hipStream_t s) {
  IRX_CHECK(G > 0 && G <= 64 && C0 % G == 0 && C0 <= kMaxC, "GroupNorm: channel counts");
  IRX_CHECK(p0 && r0 > 0 && HW % r0 == 0 && ab, "GroupNorm partials missing");
  ProfScope ps(prof_on() ? std::string("irx::(anonymous namespace)::gn_finalize_parts_kernel") : std::string(), 0.0, s);
  gn_finalize_parts_kernel<<<dim3(N, (G + 7) / 8), 256, 0, s>>>((const double2*)p0, C0, HW / r0, nullptr, 0, 0, G,
                                                                (double)HW * (C0 / G), eps, gamma, beta, ab, mr);
  IRX_LAUNCH_CHECK();
}

void gn_fold_weights(int dtype, const void* W, const float* bias, const float2* ab, const float* beta,
                     const float2* mr, int G, int N, int K, int imgs, void* Wo, float* bo, hipStream_t s) {
  IRX_CHECK(dtype != F32 && K % 8 == 0 && K <= 4096 && N > 0 && imgs > 0, "gn_fold_weights: 16-bit, K % 8 == 0");
  IRX_CHECK(beta && mr && G > 0 && K % G == 0, "gn_fold_weights: beta and the group means");
  IRX_CHECK(((uintptr_t)W % 16) == 0 && ((uintptr_t)Wo % 16) == 0, "gn_fold_weights: 16-byte aligned rows");
  ProfScope ps(prof_on() ? std::string("irx::(anonymous namespace)::gn_fold_weights_kernel") : std::string(), 0.0, s);
  if (dtype == F16)
    gn_fold_weights_kernel<f16_t><<<dim3(N, imgs), 64, 0, s>>>((const f16_t*)W, bias, ab, beta, mr, G, N, K, (f16_t*)Wo, bo);
  else
    gn_fold_weights_kernel<bf16_t><<<dim3(N, imgs), 64, 0, s>>>((const bf16_t*)W, bias, ab, beta, mr, G, N, K, (bf16_t*)Wo, bo);
  IRX_LAUNCH_CHECK();
}

bool g_gn_v2 = true;   // irx_set_option("gn_v2", 0): v1 LDS-atomic stats + separate finalize (A/B)
int g_gn_fa_blocks = 2048;   // irx_set_option("gn_fa_blocks", n): grid size the sliced gn_fa aims at (sweeps)
int g_gn_fa_wide = 1;  // irx_set_option("gn_fa_wide", 0): sliced gn_fa blocks over the fewest groups (A/B)
int g_gn_fa = 4096;    // irx_set_option("gn_fa", 0): GroupNorm from partials as finalize + apply launches (A/B);
                       // 1: one fused launch at HW <= 256; > 1: at HW <= that value (pixel slices above 256).
                       // 4096 (the UNet's 64^2 level and below): -1.5 ms/step of norm kernels vs 1
                       // (profiles/r05_bench_gn_fa_slices.txt); the 512^2 VAE's wider levels keep two launches

size_t gn_ws_bytes(int N, int HW, int G) {
  (void)HW;   // partials for up to kMaxChunks chunks per image (v1 and v3 layouts), (mean, rstd), scale / shift
  return (size_t)N * kMaxChunks * G * 2 * sizeof(double) + (size_t)N * G * sizeof(float2) +
         (size_t)N * kMaxC * sizeof(float2);
}

void group_norm(int dtype, const void* x0, const void* x1, int C0, int C1, int N, int HW, int G, float eps,
                const float* gamma, const float* beta, int silu, void* out, void* ws, hipStream_t s) {
  const int vec = dtype == F32 ? 4 : 8;
  const int C = C0 + C1;
  IRX_CHECK(G > 0 && G <= 64 && C % G == 0, "GroupNorm: C must divide into <= 64 groups");
  IRX_CHECK(C0 % vec == 0 && C1 % vec == 0, "GroupNorm: channels must be 16-byte multiples");
  IRX_CHECK(C <= 8192, "GroupNorm: too many channels");
  IRX_CHECK(C1 == 0 || x1, "GroupNorm: concat source missing");
  if (dtype == F32) gn_t<float>(x0, x1, C0, C1, N, HW, G, eps, gamma, beta, silu, out, ws, s);
  else if (dtype == F16) gn_t<f16_t>(x0, x1, C0, C1, N, HW, G, eps, gamma, beta, silu, out, ws, s);
  else gn_t<bf16_t>(x0, x1, C0, C1, N, HW, G, eps, gamma, beta, silu, out, ws, s);
}

void group_norm_parts(int dtype, const void* x0, const void* x1, int C0, int C1, int N, int HW, int G, float eps,
                      const float* gamma, const float* beta, int silu, void* out, const double* p0, int r0,
                      const double* p1, int r1, void* ws, hipStream_t s) {
  const int vec = dtype == F32 ? 4 : 8;
  IRX_CHECK(G > 0 && G <= 64 && (C0 + C1) % G == 0, "GroupNorm: C must divide into <= 64 groups");
  IRX_CHECK(C0 % vec == 0 && C1 % vec == 0 && C0 + C1 <= kMaxC, "GroupNorm: channel counts");
  IRX_CHECK(p0 && r0 > 0 && HW % r0 == 0 && (C1 == 0 || (x1 && p1 && r1 > 0 && HW % r1 == 0)),
            "GroupNorm partials missing");
  if (dtype == F32) gn_t<float>(x0, x1, C0, C1, N, HW, G, eps, gamma, beta, silu, out, ws, s, p0, r0, p1, r1);
  else if (dtype == F16) gn_t<f16_t>(x0, x1, C0, C1, N, HW, G, eps, gamma, beta, silu, out, ws, s, p0, r0, p1, r1);
  else gn_t<bf16_t>(x0, x1, C0, C1, N, HW, G, eps, gamma, beta, silu, out, ws, s, p0, r0, p1, r1);
}

void group_norm_stats(int dtype, const void* x0, const void* x1, int C0, int C1, int N, int HW, int G, float eps,
                      const float* gamma, const float* beta, float2* ab, void* ws, hipStream_t s) {
  const int vec = dtype == F32 ? 4 : 8;
  IRX_CHECK(G > 0 && G <= 64 && (C0 + C1) % G == 0, "GroupNorm: C must divide into <= 64 groups");
  IRX_CHECK(C0 % vec == 0 && C1 % vec == 0 && C0 + C1 <= kMaxC, "GroupNorm: channel counts");
  IRX_CHECK(C1 == 0 || x1, "GroupNorm: concat source missing");
  if (dtype == F32) gn_stats_t<float>(x0, x1, C0, C1, N, HW, G, eps, gamma, beta, ab, ws, s);
  else if (dtype == F16) gn_stats_t<f16_t>(x0, x1, C0, C1, N, HW, G, eps, gamma, beta, ab, ws, s);
  else gn_stats_t<bf16_t>(x0, x1, C0, C1, N, HW, G, eps, gamma, beta, ab, ws, s);
}

void layer_norm(int dtype, const void* x, long ldx, int rows, int C, float eps, const float* gamma,
                const float* beta, void* out, long ldo, hipStream_t s) {
  const int vec = dtype == F32 ? 4 : 8;
  IRX_CHECK(C % vec == 0 && ldx % vec == 0 && ldo % vec == 0, "LayerNorm: rows must be 16-byte multiples");
  IRX_CHECK((gamma == nullptr) == (beta == nullptr), "LayerNorm: gamma and beta both or neither");
  if (dtype == F32) ln_t<float>(x, ldx, rows, C, eps, gamma, beta, out, ldo, s);
  else if (dtype == F16) ln_t<f16_t>(x, ldx, rows, C, eps, gamma, beta, out, ldo, s);
  else ln_t<bf16_t>(x, ldx, rows, C, eps, gamma, beta, out, ldo, s);
}

void layer_norm_stats(int dtype, const void* x, long ldx, int rows, int C, float eps, float2* stats, hipStream_t s) {
  const int vec = dtype == F32 ? 4 : 8;
  IRX_CHECK(C % vec == 0 && ldx % vec == 0, "LayerNorm: rows must be 16-byte multiples");
  IRX_CHECK(stats, "LayerNorm statistics: null output");
  if (dtype == F32) ln_t<float>(x, ldx, rows, C, eps, nullptr, nullptr, nullptr, 0, s, stats);
  else if (dtype == F16) ln_t<f16_t>(x, ldx, rows, C, eps, nullptr, nullptr, nullptr, 0, s, stats);
  else ln_t<bf16_t>(x, ldx, rows, C, eps, nullptr, nullptr, nullptr, 0, s, stats);
}

}  // namespace irx
