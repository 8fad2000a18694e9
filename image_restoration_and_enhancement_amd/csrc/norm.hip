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

constexpr int kMaxChunks = 256;   // stats blocks per image (pixels per chunk grows with the image)

int n_chunks(int HW) { return std::min((HW + 63) / 64, kMaxChunks); }
int chunk_pix(int HW) { const int n = n_chunks(HW); return (HW + n - 1) / n; }

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

__device__ unsigned g_gn_arrivals[4096];   // per-image arrival counters of gn_stats2 (self-resetting)

// GroupNorm statistics without LDS atomics, finalised in-kernel.  Pass 1: thread (16-byte channel vector,
// pixel row r) accumulates shifted fp32 sums over its pixels and parks (shift, sum, sum of squares) per
// channel in LDS.  Pass 2: one thread per group expands and merges them in fp64 and writes the chunk
// partial.  The last chunk block of each image to arrive (agent-scope release/acquire around an arrival
// counter) folds the image's partials into (mean, rstd) — no separate finalize launch.
template <typename T>
__global__ __launch_bounds__(256) void gn_stats2_kernel(const T* __restrict__ x0, const T* __restrict__ x1, int C0,
                                                        int C1, int HW, int G, int cpix, double* part, float cnt_all,
                                                        float eps, float2* __restrict__ mr) {
  constexpr int VEC = 16 / (int)sizeof(T);
  extern __shared__ float tri[];               // [3][rows][C]: shift, sum, sum of squares
  __shared__ double red[2][256];
  __shared__ int last;
  const int C = C0 + C1;
  const int nv = C / VEC;
  const int cg = C / G;
  const int n = blockIdx.y, chunk = blockIdx.x, nch = gridDim.x;
  const int p0 = chunk * cpix, p1 = min(HW, p0 + cpix);
  const int rows = nv >= 256 ? 1 : 256 / nv;
  const int r = threadIdx.x / (nv >= 256 ? 256 : nv);
  float* X0 = tri;
  float* S = tri + rows * C;
  float* Q = tri + 2 * rows * C;
  for (int vb = 0; vb < nv; vb += 256) {
    const int v = vb + (nv >= 256 ? threadIdx.x : threadIdx.x % nv);
    if (v >= nv || r >= rows) continue;
    const int c = v * VEC;
    const T* src = c < C0 ? x0 + c : x1 + (c - C0);
    const int ld = c < C0 ? C0 : C1;
    float s[VEC], q[VEC], xs[VEC];
#pragma unroll
    for (int e = 0; e < VEC; ++e) { s[e] = 0.f; q[e] = 0.f; xs[e] = 0.f; }
    if (p0 + r < p1) Vec16<T>::unpack(*(const uint4*)(src + ((long)n * HW + p0 + r) * ld), xs);
    for (int p = p0 + r; p < p1; p += rows) {
      float f[VEC];
      Vec16<T>::unpack(*(const uint4*)(src + ((long)n * HW + p) * ld), f);
#pragma unroll
      for (int e = 0; e < VEC; ++e) {
        const float dv = f[e] - xs[e];
        s[e] += dv;
        q[e] = fmaf(dv, dv, q[e]);
      }
    }
#pragma unroll
    for (int e = 0; e < VEC; ++e) {
      X0[r * C + c + e] = xs[e];
      S[r * C + c + e] = s[e];
      Q[r * C + c + e] = q[e];
    }
  }
  __syncthreads();
  if (threadIdx.x < G) {
    const int g = threadIdx.x;
    double sd = 0.0, qd = 0.0;
    for (int rr = 0; rr < rows; ++rr) {
      const int first = p0 + rr;
      const double cnt = first < p1 ? (double)((p1 - first + rows - 1) / rows) : 0.0;
      for (int c = g * cg; c < (g + 1) * cg; ++c) {
        const double xv = X0[rr * C + c], sv = S[rr * C + c];
        sd += cnt * xv + sv;
        qd += cnt * xv * xv + 2.0 * xv * sv + (double)Q[rr * C + c];
      }
    }
    double* o = part + (((long)n * nch + chunk) * G + g) * 2;
    o[0] = sd;
    o[1] = qd;
  }
  // ---- publish this chunk; the image's last arriving block finalises
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0) {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    const unsigned prev = __hip_atomic_fetch_add(&g_gn_arrivals[n], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    last = prev == (unsigned)(nch - 1);
    if (last) {
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
  }
  __syncthreads();
  if (!last) return;
  // threads t = g + G*j sum chunks j, j + 256/G, ...
  const int per = 256 / G;
  const int g = threadIdx.x % G, j = threadIdx.x / G;
  double sd = 0.0, qd = 0.0;
  if (j < per)
    for (int ch = j; ch < nch; ch += per) {
      const double* o = part + (((long)n * nch + ch) * G + g) * 2;
      sd += o[0];
      qd += o[1];
    }
  red[0][threadIdx.x] = sd;
  red[1][threadIdx.x] = qd;
  __syncthreads();
  if (threadIdx.x < G) {
    double a = 0.0, b = 0.0;
    for (int jj = 0; jj < per; ++jj) { a += red[0][threadIdx.x + G * jj]; b += red[1][threadIdx.x + G * jj]; }
    const double cnt = (double)cnt_all;
    const double mean = a / cnt;
    double var = b / cnt - mean * mean;
    if (var < 0.0) var = 0.0;
    mr[n * G + threadIdx.x] = make_float2((float)mean, (float)(1.0 / sqrt(var + (double)eps)));
  }
  if (threadIdx.x == 0) g_gn_arrivals[n] = 0u;   // ready for the next call on this stream
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
                                                       int C1, int HW, int G, const float2* __restrict__ mr,
                                                       const float* __restrict__ gamma,
                                                       const float* __restrict__ beta, int silu, T* __restrict__ out,
                                                       int pix_per_block) {
  constexpr int VEC = 16 / (int)sizeof(T);
  __shared__ float mean_s[64], rstd_s[64];
  extern __shared__ float ab[];   // [2][C]
  const int C = C0 + C1;
  const int n = blockIdx.y;
  if (threadIdx.x < G) {
    const float2 v = mr[n * G + threadIdx.x];
    mean_s[threadIdx.x] = v.x;
    rstd_s[threadIdx.x] = v.y;
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
    for (int e = 0; e < VEC; ++e) { sc[e] = ab[c + e]; sh[e] = ab[C + c + e]; }
    const T* src = c < C0 ? x0 + (long)n * HW * C0 + c : x1 + (long)n * HW * C1 + (c - C0);
    const int ld = c < C0 ? C0 : C1;
    T* dst = out + (long)n * HW * C + c;
    for (int p = p0 + r; p < p1; p += rows) {
      float f[VEC];
      Vec16<T>::unpack(*(const uint4*)(src + (long)p * ld), f);
#pragma unroll
      for (int e = 0; e < VEC; ++e) {
        const float y = fmaf(f[e], sc[e], sh[e]);
        f[e] = silu ? y * __builtin_amdgcn_rcpf(1.0f + __expf(-y)) : y;
      }
      *(uint4*)(dst + (long)p * C) = Vec16<T>::pack(f);
    }
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
  const int nch = n_chunks(HW);
  double* part = (double*)ws;
  float2* mr = (float2*)(part + (size_t)N * nch * G * 2);
  const int C = C0 + C1;
  const int VEC = 16 / (int)sizeof(T);
  const int nvv = C / VEC;
  const int rws = nvv >= 256 ? 1 : 256 / nvv;
  if (g_gn_v2 && N <= 4096 && 3 * rws * C * sizeof(float) <= 60 * 1024) {   // default dynamic-LDS limit
    gn_stats2_kernel<T><<<dim3(nch, N), 256, 3 * rws * C * sizeof(float), s>>>(
        (const T*)x0, (const T*)x1, C0, C1, HW, G, chunk_pix(HW), part, (float)HW * (C / G), eps, mr);
    IRX_LAUNCH_CHECK();
  } else {
    gn_stats_kernel<T><<<dim3(nch, N), 256, 0, s>>>((const T*)x0, (const T*)x1, C0, C1, HW, G, chunk_pix(HW),
                                                    part);
    IRX_LAUNCH_CHECK();
    gn_finalize_kernel<<<N, 64, 0, s>>>(part, nch, G, (double)HW * (C / G), eps, mr);
    IRX_LAUNCH_CHECK();
  }
  // ~16 pixels per thread per block, one fixed channel chunk per thread
  const int nv = C / VEC;
  const int rows = nv >= 256 ? 1 : 256 / nv;
  const int ppb = rows * 16;
  gn_apply_kernel<T><<<dim3((HW + ppb - 1) / ppb, N), 256, 2 * C * sizeof(float), s>>>(
      (const T*)x0, (const T*)x1, C0, C1, HW, G, mr, gamma, beta, silu, (T*)out, ppb);
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

bool g_gn_v2 = true;   // irx_set_option("gn_v2", 0): LDS-atomic stats + separate finalize (A/B)

size_t gn_ws_bytes(int N, int HW, int G) {
  return (size_t)N * n_chunks(HW) * G * 2 * sizeof(double) + (size_t)N * G * sizeof(float2);
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
