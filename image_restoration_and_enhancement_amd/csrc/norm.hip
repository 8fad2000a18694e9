// irx — GroupNorm(+SiLU) and LayerNorm for NHWC activations on gfx950.
//
// GroupNorm (ResnetBlock2D norm1/norm2, Transformer2D norm, conv_norm_out, VAE attention norm):
// two HBM-bound passes.  Pass 1 streams pixel chunks with 16-byte vector loads and accumulates
// per-channel sum / sum of squares in fp64 (no E[x^2]-E[x]^2 cancellation at 40k-element groups),
// folds them into per-group partials via LDS atomics.  Pass 2 finalises mean/rstd per (image,
// group) from the partials, folds gamma/beta into one per-channel scale/shift, and writes
// y = x*a + b (optionally SiLU) with 16-byte vector stores.  Up-block inputs are a channel
// concat of two tensors; groups may straddle the seam, so both passes read the two sources.
#include "ops.h"

namespace irx {
namespace {

constexpr int kPix = 64;   // pixels per stats chunk

size_t n_chunks(int HW) { return (HW + kPix - 1) / kPix; }

template <typename T>
__global__ __launch_bounds__(256) void gn_stats_kernel(const T* __restrict__ x0, const T* __restrict__ x1,
                                                       int C0, int C1, int HW, int G, double* part) {
  constexpr int VEC = 16 / (int)sizeof(T);
  __shared__ double gs[64], gq[64];
  const int C = C0 + C1;
  const int nv = C / VEC;                      // vectors per pixel
  const int cg = C / G;
  const int n = blockIdx.y, chunk = blockIdx.x;
  const int p0 = chunk * kPix, p1 = min(HW, p0 + kPix);
  if (threadIdx.x < 64) { gs[threadIdx.x] = 0.0; gq[threadIdx.x] = 0.0; }
  __syncthreads();
  // thread -> (vector v, pixel lane r); each thread owns up to 2 vectors (C <= 4096)
  const int rows = nv >= 256 ? 1 : 256 / nv;
  const int r = threadIdx.x / (nv >= 256 ? 256 : nv);
  for (int vb = 0; vb < nv; vb += 256) {
    const int v = vb + (nv >= 256 ? threadIdx.x : threadIdx.x % nv);
    if (v >= nv || r >= rows) continue;
    double s[VEC], q[VEC];
#pragma unroll
    for (int e = 0; e < VEC; ++e) { s[e] = 0.0; q[e] = 0.0; }
    const int c = v * VEC;
    const T* src = c < C0 ? x0 + c : x1 + (c - C0);
    const int ld = c < C0 ? C0 : C1;
    for (int p = p0 + r; p < p1; p += rows) {
      const uint4 u = *(const uint4*)(src + ((long)n * HW + p) * ld);
      float f[VEC];
      Vec16<T>::unpack(u, f);
#pragma unroll
      for (int e = 0; e < VEC; ++e) { s[e] += f[e]; q[e] += (double)f[e] * f[e]; }
    }
#pragma unroll
    for (int e = 0; e < VEC; ++e) {
      const int grp = (c + e) / cg;
      atomicAdd(&gs[grp], s[e]);
      atomicAdd(&gq[grp], q[e]);
    }
  }
  __syncthreads();
  if (threadIdx.x < G) {
    double* o = part + (((long)n * gridDim.x + chunk) * G + threadIdx.x) * 2;
    o[0] = gs[threadIdx.x];
    o[1] = gq[threadIdx.x];
  }
}

template <typename T>
__global__ __launch_bounds__(256) void gn_apply_kernel(const T* __restrict__ x0, const T* __restrict__ x1, int C0,
                                                       int C1, int HW, int G, int nchunk, const double* part,
                                                       float eps, const float* __restrict__ gamma,
                                                       const float* __restrict__ beta, int silu, T* __restrict__ out,
                                                       int pix_per_block) {
  constexpr int VEC = 16 / (int)sizeof(T);
  __shared__ float mean_s[64], rstd_s[64];
  extern __shared__ float ab[];   // [2][C]
  const int C = C0 + C1;
  const int n = blockIdx.y;
  if (threadIdx.x < G) {
    double s = 0.0, q = 0.0;
    const double* p = part + ((long)n * nchunk) * G * 2 + threadIdx.x * 2;
    for (int c = 0; c < nchunk; ++c) { s += p[(long)c * G * 2]; q += p[(long)c * G * 2 + 1]; }
    const double cnt = (double)HW * (C / G);
    const double mean = s / cnt;
    double var = q / cnt - mean * mean;
    if (var < 0.0) var = 0.0;
    mean_s[threadIdx.x] = (float)mean;
    rstd_s[threadIdx.x] = (float)(1.0 / sqrt(var + (double)eps));
  }
  __syncthreads();
  const int cg = C / G;
  for (int c = threadIdx.x; c < C; c += blockDim.x) {
    const int grp = c / cg;
    const float sc = rstd_s[grp] * gamma[c];
    ab[c] = sc;
    ab[C + c] = beta[c] - mean_s[grp] * sc;
  }
  __syncthreads();
  const int nv = C / VEC;
  const int p0 = blockIdx.x * pix_per_block;
  const int total = min(pix_per_block, HW - p0) * nv;
  for (int i = threadIdx.x; i < total; i += blockDim.x) {
    const long p = p0 + i / nv;
    const int c = (i % nv) * VEC;
    const T* src = c < C0 ? x0 + ((long)n * HW + p) * C0 + c : x1 + ((long)n * HW + p) * C1 + (c - C0);
    float f[VEC];
    Vec16<T>::unpack(*(const uint4*)src, f);
#pragma unroll
    for (int e = 0; e < VEC; ++e) {
      float y = f[e] * ab[c + e] + ab[C + c + e];
      f[e] = silu ? silu_f(y) : y;
    }
    *(uint4*)(out + ((long)n * HW + p) * C + c) = Vec16<T>::pack(f);
  }
}

// LayerNorm: one wave per row, row held in registers, two-pass mean/var in fp32.
template <typename T, int MAXV>
__global__ __launch_bounds__(256) void ln_kernel(const T* __restrict__ x, long ldx, int rows, int C, float eps,
                                                 const float* __restrict__ gamma, const float* __restrict__ beta,
                                                 T* __restrict__ out, long ldo) {
  constexpr int VEC = 16 / (int)sizeof(T);
  const int lane = threadIdx.x & 63;
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= rows) return;
  const int nv = C / VEC;
  float f[MAXV][VEC];
  float s = 0.f;
#pragma unroll
  for (int i = 0; i < MAXV; ++i) {
    const int v = lane + 64 * i;
    if (v < nv) {
      Vec16<T>::unpack(*(const uint4*)(x + (long)row * ldx + v * VEC), f[i]);
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
      for (int e = 0; e < VEC; ++e) { const float dd = f[i][e] - mean; q += dd * dd; }
    }
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) q += __shfl_xor(q, o);
  const float rstd = rsqrtf(q / C + eps);
#pragma unroll
  for (int i = 0; i < MAXV; ++i) {
    const int v = lane + 64 * i;
    if (v < nv) {
      float y[VEC];
#pragma unroll
      for (int e = 0; e < VEC; ++e) {
        const int c = v * VEC + e;
        y[e] = (f[i][e] - mean) * rstd * gamma[c] + beta[c];
      }
      *(uint4*)(out + (long)row * ldo + v * VEC) = Vec16<T>::pack(y);
    }
  }
}

template <typename T>
void gn_t(const void* x0, const void* x1, int C0, int C1, int N, int HW, int G, float eps, const float* gamma,
          const float* beta, int silu, void* out, void* ws, hipStream_t s) {
  const int nch = (int)n_chunks(HW);
  gn_stats_kernel<T><<<dim3(nch, N), 256, 0, s>>>((const T*)x0, (const T*)x1, C0, C1, HW, G, (double*)ws);
  IRX_LAUNCH_CHECK();
  const int C = C0 + C1;
  const int VEC = 16 / (int)sizeof(T);
  // ~16 vectors per thread per block
  int ppb = max(1, (256 * 16) / (C / VEC));
  gn_apply_kernel<T><<<dim3((HW + ppb - 1) / ppb, N), 256, 2 * C * sizeof(float), s>>>(
      (const T*)x0, (const T*)x1, C0, C1, HW, G, nch, (const double*)ws, eps, gamma, beta, silu, (T*)out, ppb);
  IRX_LAUNCH_CHECK();
}

template <typename T>
void ln_t(const void* x, long ldx, int rows, int C, float eps, const float* gamma, const float* beta, void* out,
          long ldo, hipStream_t s) {
  const int VEC = 16 / (int)sizeof(T);
  const int nv = C / VEC;
  dim3 grid((rows + 3) / 4), block(256);
  if (nv <= 64) ln_kernel<T, 1><<<grid, block, 0, s>>>((const T*)x, ldx, rows, C, eps, gamma, beta, (T*)out, ldo);
  else if (nv <= 128) ln_kernel<T, 2><<<grid, block, 0, s>>>((const T*)x, ldx, rows, C, eps, gamma, beta, (T*)out, ldo);
  else if (nv <= 256) ln_kernel<T, 4><<<grid, block, 0, s>>>((const T*)x, ldx, rows, C, eps, gamma, beta, (T*)out, ldo);
  else if (nv <= 512) ln_kernel<T, 8><<<grid, block, 0, s>>>((const T*)x, ldx, rows, C, eps, gamma, beta, (T*)out, ldo);
  else throw Error("layer_norm: C too large");
  IRX_LAUNCH_CHECK();
}

}  // namespace

size_t gn_ws_bytes(int N, int HW, int G) { return (size_t)N * n_chunks(HW) * G * 2 * sizeof(double); }

void group_norm(int dtype, const void* x0, const void* x1, int C0, int C1, int N, int HW, int G, float eps,
                const float* gamma, const float* beta, int silu, void* out, void* ws, hipStream_t s) {
  const int vec = dtype == F32 ? 4 : 8;
  const int C = C0 + C1;
  IRX_CHECK(G > 0 && G <= 64 && C % G == 0, "GroupNorm: C must divide into <= 64 groups");
  IRX_CHECK(C0 % vec == 0 && C1 % vec == 0, "GroupNorm: channels must be 16-byte multiples");
  IRX_CHECK(C <= 8192, "GroupNorm: too many channels");
  IRX_CHECK(C1 == 0 || x1, "GroupNorm: concat source missing");
  if (dtype == F32) gn_t<float>(x0, x1, C0, C1, N, HW, G, eps, gamma, beta, silu, out, ws, s);
  else gn_t<bf16_t>(x0, x1, C0, C1, N, HW, G, eps, gamma, beta, silu, out, ws, s);
}

void layer_norm(int dtype, const void* x, long ldx, int rows, int C, float eps, const float* gamma,
                const float* beta, void* out, long ldo, hipStream_t s) {
  const int vec = dtype == F32 ? 4 : 8;
  IRX_CHECK(C % vec == 0 && ldx % vec == 0 && ldo % vec == 0, "LayerNorm: rows must be 16-byte multiples");
  if (dtype == F32) ln_t<float>(x, ldx, rows, C, eps, gamma, beta, out, ldo, s);
  else ln_t<bf16_t>(x, ldx, rows, C, eps, gamma, beta, out, ldo, s);
}

}  // namespace irx
