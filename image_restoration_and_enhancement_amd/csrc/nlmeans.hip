// irx — OpenCV's fast non-local-means denoiser (the invoker behind cv2.fastNlMeansDenoisingColored, which the
// reference's classical denoise fallback calls: src/inference.py:509-515) on uint8 batches
// resident in HBM.  Integer-exact restatement of FastNlMeansDenoisingInvoker (oracle/nlm_ref.py):
//   dist(p, q) = sum_{template} sum_c (I_c(p+t) - I_c(q+t))^2,  w = lut[min(dist >> shift, lut_len)],
//   out_c = (sum_q w I_c(q) + W/2) / W over the search window, BORDER_REFLECT_101 everywhere.
// The weight table is built on the host (irx_nlm_weights) and staged once per block in LDS.
//
// Work decomposition: one block per 32x32 output tile and image; its (32+2B)^2 reflect-padded region
// (B = search/2 + template/2) of the channel group sits in LDS (bytes; a 2-channel group as 16-bit pairs so
// one v_pk_sub_i16 + v_dot2_i32_i16 forms a tap's two-channel squared distance).  Each thread owns a column strip of
// 4 pixels and keeps the strip's own template rows in registers.  For each search row offset it slides a
// (4+2r) x (2r+1) register window of the neighbour rows across the 2s+1 column offsets, loading one new LDS
// column per offset.  Row SSDs are formed once per strip row and summed into the 4 pixel distances, which is
// 4x fewer squared differences than per-pixel templates.  Compute (VALU) bound: HBM traffic is one read and
// one write of the image.
#include "ops.h"
#include "profile.h"

#include <type_traits>

namespace irx {
int g_nlm_strip = 4;                               // irx_set_option("nlm_strip", 4 | 8)
int g_nlm2_strip = 4;                              // irx_set_option("nlm2_strip", 2 | 4 | 8 | 16)
int g_nlm_v2 = 1;   // irx_set_option("nlm_v2", v): 1 = v2 centre value from LDS, 2 = v2 centre by DPP, 0 = v1
namespace {

constexpr int NLM_TW = 32, NLM_G = 8;          // 32 columns x 8 strip groups = 256 threads; strips of S rows

__device__ __forceinline__ int refl101(int p, int n) {
  if (n == 1) return 0;
  while ((unsigned)p >= (unsigned)n) p = p < 0 ? -p : 2 * (n - 1) - p;
  return p;
}

typedef short nlm_s2 __attribute__((ext_vector_type(2)));

// squared distance of one tap: CN 1 = one byte; CN 2 = both channels packed as 16-bit halves (lo = c0,
// hi = c1), one v_pk_sub_i16 + one v_dot2 per tap
template <int CN>
__device__ __forceinline__ int tap(int s, int o, int n) {
  if constexpr (CN == 1) {
    const int d = o - n;
    return s + d * d;
  } else {
    const nlm_s2 d = __builtin_bit_cast(nlm_s2, o) - __builtin_bit_cast(nlm_s2, n);
    return __builtin_amdgcn_sdot2(d, d, s, false);
  }
}

template <int CN, int TR, int SR, int NLM_S>
__global__ __launch_bounds__(256) void nlm_kernel(const uint8_t* __restrict__ src, uint8_t* __restrict__ dst,
                                                  int H, int W, int ps, int coff, const int* __restrict__ lut,
                                                  int lut_len, int shift) {
  static_assert(CN == 1 || CN == 2, "channel groups of 1 or 2");
  constexpr int NLM_TH = NLM_S * NLM_G;
  using PV = typename std::conditional<CN == 1, uint8_t, uint32_t>::type;
  constexpr int B = TR + SR, T = 2 * TR + 1, RH = NLM_TH + 2 * B, RW = NLM_TW + 2 * B, NR = NLM_S + 2 * TR;
  constexpr int PLANE = RH * RW;
  extern __shared__ int smem[];
  PV* reg = reinterpret_cast<PV*>(smem);                      // [RH][RW] pixels of the group
  int* wl = smem + (PLANE * (int)sizeof(PV) + 3) / 4;         // [lut_len + 1], last entry 0
  const int tid = threadIdx.x, x0 = blockIdx.x * NLM_TW, y0 = blockIdx.y * NLM_TH;
  const uint8_t* img = src + (size_t)blockIdx.z * H * W * ps + coff;
  for (int i = tid; i < PLANE; i += 256) {
    const int ry = i / RW, rx = i - ry * RW;
    const uint8_t* p = img + ((size_t)refl101(y0 + ry - B, H) * W + refl101(x0 + rx - B, W)) * ps;
    if constexpr (CN == 1) reg[i] = p[0];
    else reg[i] = (uint32_t)p[0] | ((uint32_t)p[1] << 16);
  }
  for (int i = tid; i <= lut_len; i += 256) wl[i] = i < lut_len ? lut[i] : 0;
  __syncthreads();

  const int col = tid & (NLM_TW - 1), grp = tid / NLM_TW;
  int own[NR][T];                                             // template rows of the strip (registers)
#pragma unroll
  for (int j = 0; j < NR; ++j)
#pragma unroll
    for (int k = 0; k < T; ++k) own[j][k] = (int)reg[(grp * NLM_S + SR + j) * RW + col + SR + k];

  int wsum[NLM_S], est[NLM_S][CN];
#pragma unroll
  for (int i = 0; i < NLM_S; ++i) {
    wsum[i] = 0;
#pragma unroll
    for (int c = 0; c < CN; ++c) est[i][c] = 0;
  }

  for (int a = 0; a <= 2 * SR; ++a) {                         // search row offset dy = a - SR
    const PV* rb = reg + (grp * NLM_S + a) * RW + col;
    int nb[NR][T];
#pragma unroll
    for (int j = 0; j < NR; ++j)
#pragma unroll
      for (int k = 0; k < T - 1; ++k) nb[j][k] = (int)rb[j * RW + k];
#pragma unroll
    for (int b = 0; b <= 2 * SR; ++b) {                       // search column offset dx = b - SR
#pragma unroll
      for (int j = 0; j < NR; ++j) nb[j][T - 1] = (int)rb[j * RW + b + T - 1];
      int R[NR];
#pragma unroll
      for (int j = 0; j < NR; ++j) {
        int s = 0;
#pragma unroll
        for (int k = 0; k < T; ++k) s = tap<CN>(s, own[j][k], nb[j][k]);
        R[j] = s;
      }
#pragma unroll
      for (int i = 0; i < NLM_S; ++i) {
        int dist = 0;
#pragma unroll
        for (int t = 0; t < T; ++t) dist += R[i + t];
        const int w = wl[min(dist >> shift, lut_len)];
        wsum[i] += w;
        const int q = nb[i + TR][TR];
        if constexpr (CN == 1) {
          est[i][0] += w * q;
        } else {
          est[i][0] += w * (q & 0xffff);
          est[i][1] += w * (q >> 16);
        }
      }
#pragma unroll
      for (int j = 0; j < NR; ++j)
#pragma unroll
        for (int k = 0; k < T - 1; ++k) nb[j][k] = nb[j][k + 1];
    }
  }

  const int x = x0 + col;
#pragma unroll
  for (int i = 0; i < NLM_S; ++i) {
    const int y = y0 + grp * NLM_S + i;
    if (y < H && x < W) {
      uint8_t* o = dst + (((size_t)blockIdx.z * H + y) * W + x) * ps + coff;
      const unsigned ws = (unsigned)wsum[i];                  // > 0: the centre offset weighs fpm
#pragma unroll
      for (int c = 0; c < CN; ++c) o[c] = (uint8_t)min(255u, ((unsigned)est[i][c] + ws / 2) / ws);
    }
  }
}

// v2: per search offset each lane squares only its own column, (S + 2r) taps for an S-row strip; the template
// sums are a running vertical sum per lane and a 2r-step horizontal sum across lanes, each step one
// v_add_u32_dpp wave_shr:1.  A wave spans 64 consecutive columns and yields 64 - 2r outputs (lane l holds
// the window ending at column l, centred on column l - r).  Search offsets run dx-major so the neighbour
// column slides down one row per dy (one LDS read per offset).
constexpr int NLM2_WAVES = 4;

template <int CN, int TR, int SR, int S, bool g_centre_lds>
__global__ __launch_bounds__(256) void nlm2_kernel(const uint8_t* __restrict__ src, uint8_t* __restrict__ dst,
                                                   int H, int W, int ps, int coff, const int* __restrict__ lut,
                                                   int lut_len, int shift) {
  static_assert(CN == 1 || CN == 2, "channel groups of 1 or 2");
  using PV = typename std::conditional<CN == 1, uint8_t, uint32_t>::type;
  constexpr int TWO = 64 - 2 * TR, TH = NLM2_WAVES * S, B = TR + SR, NR = S + 2 * TR;
  constexpr int RH = TH + 2 * B, RW = 64 + 2 * SR, PLANE = RH * RW;
  extern __shared__ int smem[];
  PV* reg = reinterpret_cast<PV*>(smem);                      // [RH][RW], origin (y0 - B, x0 - B)
  int* wl = smem + (PLANE * (int)sizeof(PV) + 3) / 4;
  const int tid = threadIdx.x, x0 = blockIdx.x * TWO, y0 = blockIdx.y * TH;
  const uint8_t* img = src + (size_t)blockIdx.z * H * W * ps + coff;
  for (int i = tid; i < PLANE; i += 256) {
    const int ry = i / RW, rx = i - ry * RW;
    const uint8_t* p = img + ((size_t)refl101(y0 + ry - B, H) * W + refl101(x0 + rx - B, W)) * ps;
    if constexpr (CN == 1) reg[i] = p[0];
    else reg[i] = (uint32_t)p[0] | ((uint32_t)p[1] << 16);
  }
  for (int i = tid; i <= lut_len; i += 256) wl[i] = i < lut_len ? lut[i] : 0;
  __syncthreads();

  const int l = tid & 63, w = tid >> 6;
  // own column (image column x0 - TR + l), rows y0 + w*S - TR + j
  int own[NR];
#pragma unroll
  for (int j = 0; j < NR; ++j) own[j] = (int)reg[(w * S + SR + j) * RW + l + SR];
  // centre pixel of the output this lane holds: column x0 - 2TR + l (window [l - 2TR, l])
  int wsum[S], est[S][CN];
#pragma unroll
  for (int i = 0; i < S; ++i) {
    wsum[i] = 0;
#pragma unroll
    for (int c = 0; c < CN; ++c) est[i][c] = 0;
  }
  for (int b = 0; b <= 2 * SR; ++b) {                         // dx = b - SR
    const PV* cb = reg + w * S * RW + l + b;                  // neighbour column, row offset a + j
    int nb[NR];
#pragma unroll
    for (int j = 0; j < NR - 1; ++j) nb[j] = (int)cb[j * RW];
    for (int a = 0; a <= 2 * SR; ++a) {                       // dy = a - SR
      nb[NR - 1] = (int)cb[(a + NR - 1) * RW];
      int D[NR];
#pragma unroll
      for (int j = 0; j < NR; ++j) D[j] = tap<CN>(0, own[j], nb[j]);
      int V[S];
      {
        int v = 0;
#pragma unroll
        for (int t = 0; t < 2 * TR + 1; ++t) v += D[t];
        V[0] = v;
#pragma unroll
        for (int i = 1; i < S; ++i) {
          v += D[i + 2 * TR] - D[i - 1];
          V[i] = v;
        }
      }
      // the centre value q of each output: neighbour at the centre column (lane l - TR), row i + TR
#pragma unroll
      for (int i = 0; i < S; ++i) {
        int hs = V[i];
#pragma unroll
        for (int u = 0; u < 2 * TR; ++u) hs = V[i] + __builtin_amdgcn_update_dpp(0, hs, 0x138, 0xf, 0xf, false);
        int qc;
        if (g_centre_lds) {
          // the centre neighbour sits TR columns left of this lane's own column (lanes < 2TR: discarded;
          // the index stays inside the region since row a + i + TR >= TR)
          qc = (int)cb[(a + i + TR) * RW - TR];
        } else {
          qc = __builtin_amdgcn_update_dpp(0, nb[i + TR], 0x138, 0xf, 0xf, false);
#pragma unroll
          for (int u = 1; u < TR; ++u) qc = __builtin_amdgcn_update_dpp(0, qc, 0x138, 0xf, 0xf, false);
        }
        const int wt = wl[min(hs >> shift, lut_len)];
        wsum[i] += wt;
        if constexpr (CN == 1) {
          est[i][0] += wt * qc;
        } else {
          est[i][0] += wt * (qc & 0xffff);
          est[i][1] += wt * (qc >> 16);
        }
      }
#pragma unroll
      for (int j = 0; j < NR - 1; ++j) nb[j] = nb[j + 1];
    }
  }
  const int x = x0 - TR + l - TR;                             // centre column of this lane's window
  if (l >= 2 * TR && x < W) {
#pragma unroll
    for (int i = 0; i < S; ++i) {
      const int y = y0 + w * S + i;
      if (y < H) {
        uint8_t* o = dst + (((size_t)blockIdx.z * H + y) * W + x) * ps + coff;
        const unsigned ws = (unsigned)wsum[i];
#pragma unroll
        for (int c = 0; c < CN; ++c) o[c] = (uint8_t)min(255u, ((unsigned)est[i][c] + ws / 2) / ws);
      }
    }
  }
}

template <int CN, int TR, int SR, int S>
void launch2s(const uint8_t* src, uint8_t* dst, int N, int H, int W, int ps, int coff, const int* lut, int lut_len,
              int shift, hipStream_t s) {
  constexpr int TWO = 64 - 2 * TR, TH = NLM2_WAVES * S, B = TR + SR;
  constexpr int PLANE = (TH + 2 * B) * (64 + 2 * SR), PB = CN == 1 ? 1 : 4;
  const size_t lds = ((PLANE * PB + 3) / 4 + lut_len + 1) * sizeof(int);
  IRX_CHECK(lds <= 160 * 1024, "nlmeans: weight table too long for LDS (h too large)");
  auto k = g_nlm_v2 == 2 ? nlm2_kernel<CN, TR, SR, S, false> : nlm2_kernel<CN, TR, SR, S, true>;
  static_assert(S >= 1, "strip rows");
  if (lds > 64 * 1024) IRX_HIP(hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize,
                                                   (int)lds));
  const dim3 grid((W + TWO - 1) / TWO, (H + TH - 1) / TH, N);
  const double ops = 3.0 * N * H * W * (2 * SR + 1) * (2 * SR + 1) * (2 * TR + 1) * (2 * TR + 1) * CN;
  ProfScope pr(prof_on() ? std::string("irx::(anonymous namespace)::nlm2_kernel") : std::string(), ops, s);
  hipLaunchKernelGGL(k, grid, dim3(256), lds, s, src, dst, H, W, ps, coff, lut, lut_len, shift);
  IRX_HIP(hipGetLastError());
}

template <int CN, int TR, int SR>
void launch2(const uint8_t* src, uint8_t* dst, int N, int H, int W, int ps, int coff, const int* lut, int lut_len,
             int shift, hipStream_t s) {
  // strip rows per wave: 4 (default; measured 1.29 vs 1.40 / 1.67 ms per 8x512^2 batch for 8 / 16) or 2 / 8 / 16
  // (irx_set_option("nlm2_strip", ...))
  if (g_nlm2_strip == 2) return launch2s<CN, TR, SR, 2>(src, dst, N, H, W, ps, coff, lut, lut_len, shift, s);
  if (g_nlm2_strip == 8) return launch2s<CN, TR, SR, 8>(src, dst, N, H, W, ps, coff, lut, lut_len, shift, s);
  if (g_nlm2_strip == 16) return launch2s<CN, TR, SR, 16>(src, dst, N, H, W, ps, coff, lut, lut_len, shift, s);
  return launch2s<CN, TR, SR, 4>(src, dst, N, H, W, ps, coff, lut, lut_len, shift, s);
}

template <int CN, int TR, int SR, int NLM_S>
void launch(const uint8_t* src, uint8_t* dst, int N, int H, int W, int ps, int coff, const int* lut, int lut_len,
            int shift, hipStream_t s) {
  constexpr int NLM_TH = NLM_S * NLM_G, B = TR + SR, PLANE = (NLM_TH + 2 * B) * (NLM_TW + 2 * B);
  constexpr int PB = CN == 1 ? 1 : 4;
  const size_t lds = ((PLANE * PB + 3) / 4 + lut_len + 1) * sizeof(int);
  IRX_CHECK(lds <= 160 * 1024, "nlmeans: weight table too long for LDS (h too large)");
  auto k = nlm_kernel<CN, TR, SR, NLM_S>;
  if (lds > 64 * 1024) IRX_HIP(hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize,
                                                   (int)lds));
  const dim3 grid((W + NLM_TW - 1) / NLM_TW, (H + NLM_TH - 1) / NLM_TH, N);
  // algorithmic integer ops of the direct form: (sub, mul, add) per template tap, channel and search offset
  const double ops = 3.0 * N * H * W * (2 * SR + 1) * (2 * SR + 1) * (2 * TR + 1) * (2 * TR + 1) * CN;
  ProfScope pr(prof_on() ? std::string("irx::(anonymous namespace)::nlm_kernel") : std::string(), ops, s);
  hipLaunchKernelGGL(k, grid, dim3(256), lds, s, src, dst, H, W, ps, coff, lut, lut_len, shift);
  IRX_HIP(hipGetLastError());
}

}  // namespace

void nlmeans_u8(const uint8_t* src, uint8_t* dst, int N, int H, int W, int ps, int coff, int cn, int tmpl,
                int search, const int* lut, int lut_len, int shift, hipStream_t s) {
  const int strip = g_nlm_strip;                   // strip rows per thread for the 1-channel group (4 or 8)
  if (g_nlm_v2) {
    if (tmpl == 7 && search == 21) {
      if (cn == 1) return launch2<1, 3, 10>(src, dst, N, H, W, ps, coff, lut, lut_len, shift, s);
      if (cn == 2) return launch2<2, 3, 10>(src, dst, N, H, W, ps, coff, lut, lut_len, shift, s);
    } else if (tmpl == 3 && search == 5) {
      if (cn == 1) return launch2<1, 1, 2>(src, dst, N, H, W, ps, coff, lut, lut_len, shift, s);
      if (cn == 2) return launch2<2, 1, 2>(src, dst, N, H, W, ps, coff, lut, lut_len, shift, s);
    }
  }
  if (tmpl == 7 && search == 21) {
    if (cn == 1 && strip == 8) return launch<1, 3, 10, 8>(src, dst, N, H, W, ps, coff, lut, lut_len, shift, s);
    if (cn == 1) return launch<1, 3, 10, 4>(src, dst, N, H, W, ps, coff, lut, lut_len, shift, s);
    if (cn == 2) return launch<2, 3, 10, 4>(src, dst, N, H, W, ps, coff, lut, lut_len, shift, s);
  } else if (tmpl == 3 && search == 5) {
    if (cn == 1 && strip == 8) return launch<1, 1, 2, 8>(src, dst, N, H, W, ps, coff, lut, lut_len, shift, s);
    if (cn == 1) return launch<1, 1, 2, 4>(src, dst, N, H, W, ps, coff, lut, lut_len, shift, s);
    if (cn == 2) return launch<2, 1, 2, 4>(src, dst, N, H, W, ps, coff, lut, lut_len, shift, s);
  }
  IRX_CHECK(false, "nlmeans: supported (template, search, cn): (7, 21) and (3, 5) with cn 1 or 2");
}

}  // namespace irx
