// irx — flash-style multi-head attention for gfx950 (wave64, MFMA 16x16).
//
// Serves the UNet's self-attention (attn1: Lq = Lk = h*w up to 9216, d = 40/80/160),
// cross-attention (attn2: Lk = 77 text tokens) and CLIP's causal self-attention (d = 64).
// "Swapped" formulation: each wave computes S^T = K Q^T so a lane owns one query COLUMN;
// its softmax statistics are lane-local (plus a 4-way shuffle for the max), the
// exponentiated tile is already the B operand of O^T = V^T P^T (no LDS round trip for P),
// and V^T fragments come straight out of the row-major V tile through the gfx950
// transposing LDS read ds_read_b64_tr_b16.  Online softmax in fp32; scores never touch HBM.
// bf16: v_mfma_f32_16x16x16_bf16 (K = 16 keeps d = 40 / 80 padding at 48 / 80);
// fp32 (parity mode): exact-f32 v_mfma_f32_16x16x4_f32.
#include "ops.h"
#include "profile.h"

namespace irx {
namespace {

constexpr int kWaves = 4;
constexpr int kQT = 2;               // 16-query column tiles per wave
constexpr int kQB = kWaves * kQT * 16;  // queries per block (128)
constexpr int kKT = 64;              // keys per LDS tile

template <typename T, int DP>
struct AttnLds {
  // K tile rows: stride chosen so 16 rows x 2 half-chunks of ds_read_b64 are bank-disjoint;
  // V tile rows: stride chosen so the transposed reads (8 rows x 4 chunks per half wave) are.
  static constexpr int SK = sizeof(T) == 2 ? DP + 8 : DP + 4;
  static constexpr int SV = sizeof(T) == 2 ? (((DP / 2) % 16 == 8) ? DP : DP + 16) : DP + 1;
};

typedef __attribute__((address_space(3))) s16x4 lds_s16x4;

template <typename T, int DP>
__global__ __launch_bounds__(256, 1) void attn_kernel(AttnArgs a) {
  using L = AttnLds<T, DP>;
  constexpr int ND = DP / 16;
  constexpr int SK = L::SK, SV = L::SV;
  __shared__ __attribute__((aligned(16))) T Ks[kKT * SK];
  __shared__ __attribute__((aligned(16))) T Vs[kKT * SV];

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int li = lane & 15, g = lane >> 4;
  const int b = blockIdx.z, h = blockIdx.y;
  const int qb0 = blockIdx.x * kQB;
  const int q0 = qb0 + wave * (kQT * 16);
  const int d = a.d;

  const T* __restrict__ Q = (const T*)a.q + (long)b * a.sq + (long)h * d;
  const T* __restrict__ K = (const T*)a.k + (long)b * a.sk + (long)h * d;
  const T* __restrict__ V = (const T*)a.v + (long)b * a.sv + (long)h * d;

  // zero the padded LDS columns once (loads only ever write columns < d)
  for (int i = tid; i < kKT * SK; i += 256) Ks[i] = T(0);
  for (int i = tid; i < kKT * SV; i += 256) Vs[i] = T(0);

  // ---- Q^T fragments in registers (B operand: k = d, col = query)
  constexpr int QV = sizeof(T) == 2 ? 1 : 4;       // f32: float4 per lane per 16-deep chunk
  typedef typename std::conditional<sizeof(T) == 2, s16x4, f32x4>::type qfrag_t;
  qfrag_t qf[kQT][ND];
#pragma unroll
  for (int qt = 0; qt < kQT; ++qt) {
    const int q = q0 + qt * 16 + li;
#pragma unroll
    for (int dc = 0; dc < ND; ++dc) {
      const int e = dc * 16 + 4 * g;
      if constexpr (sizeof(T) == 2) {
        s16x4 v = {0, 0, 0, 0};
        if (q < a.Lq && e < d) v = *(const s16x4*)(Q + (long)q * a.ldq + e);
        qf[qt][dc] = v;
      } else {
        f32x4 v = {0.f, 0.f, 0.f, 0.f};
        if (q < a.Lq && e < d) v = *(const f32x4*)(Q + (long)q * a.ldq + e);
        qf[qt][dc] = v;
      }
    }
  }
  (void)QV;

  f32x4 o[ND][kQT];
#pragma unroll
  for (int i = 0; i < ND; ++i)
#pragma unroll
    for (int j = 0; j < kQT; ++j) o[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  float mrow[kQT], lrow[kQT];
#pragma unroll
  for (int j = 0; j < kQT; ++j) { mrow[j] = -INFINITY; lrow[j] = 0.f; }

  const float sl2 = a.scale * 1.4426950408889634f;   // softmax in base 2: exp(x*scale) = exp2(x*sl2)
  int kend = a.Lk;
  if (a.causal) kend = min(kend, qb0 + kQB);
  const int cpr = d * (int)sizeof(T) / 16;           // 16-byte chunks per K/V row
  constexpr int E = 16 / (int)sizeof(T);
  // bf16: the next K/V tile is fetched into registers under the current tile's MFMAs (async-STAGE split);
  // fp32 (parity mode, register-bound at d = 160): synchronous staging.
  constexpr bool PREFETCH = sizeof(T) == 2;
  constexpr int NCH = PREFETCH ? (kKT * (DP * (int)sizeof(T) / 16) + 255) / 256 : 1;
  uint4 kreg[NCH], vreg[NCH];
  auto load_regs = [&](int j0) {
#pragma unroll
    for (int u = 0; u < NCH; ++u) {
      const int idx = tid + 256 * u;
      kreg[u] = make_uint4(0, 0, 0, 0);
      vreg[u] = make_uint4(0, 0, 0, 0);
      if (idx < kKT * cpr) {
        const int r = idx / cpr, c = idx - r * cpr;
        const int key = j0 + r;
        if (key < a.Lk) {
          kreg[u] = *(const uint4*)(K + (long)key * a.ldk + c * E);
          vreg[u] = *(const uint4*)(V + (long)key * a.ldv + c * E);
        }
      }
    }
  };
  auto store_regs = [&]() {
#pragma unroll
    for (int u = 0; u < NCH; ++u) {
      const int idx = tid + 256 * u;
      if (idx < kKT * cpr) {
        const int r = idx / cpr, c = idx - r * cpr;
        *(uint4*)(Ks + r * SK + c * E) = kreg[u];
        *(uint4*)(Vs + r * SV + c * E) = vreg[u];
      }
    }
  };
  if constexpr (PREFETCH) load_regs(0);

  for (int j0 = 0; j0 < kend; j0 += kKT) {
    __syncthreads();   // previous tile fully consumed
    if constexpr (PREFETCH) {
      store_regs();
      __syncthreads();
      if (j0 + kKT < kend) load_regs(j0 + kKT);
    } else {
      for (int idx = tid; idx < kKT * cpr; idx += 256) {
        const int r = idx / cpr, c = idx - r * cpr;
        const int key = j0 + r;
        uint4 kv = make_uint4(0, 0, 0, 0), vv = make_uint4(0, 0, 0, 0);
        if (key < a.Lk) {
          kv = *(const uint4*)(K + (long)key * a.ldk + c * E);
          vv = *(const uint4*)(V + (long)key * a.ldv + c * E);
        }
        *(uint4*)(Ks + r * SK + c * E) = kv;
        float* pv = (float*)(Vs + r * SV + c * E);
        pv[0] = __uint_as_float(vv.x); pv[1] = __uint_as_float(vv.y);
        pv[2] = __uint_as_float(vv.z); pv[3] = __uint_as_float(vv.w);
      }
      __syncthreads();
    }

    // ---- S^T = K Q^T  (rows = keys of this tile, cols = this wave's queries)
    f32x4 s[4][kQT];
#pragma unroll
    for (int kt = 0; kt < 4; ++kt)
#pragma unroll
      for (int qt = 0; qt < kQT; ++qt) s[kt][qt] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int kt = 0; kt < 4; ++kt) {
#pragma unroll
      for (int dc = 0; dc < ND; ++dc) {
        const T* kp = Ks + (kt * 16 + li) * SK + dc * 16 + 4 * g;
        if constexpr (sizeof(T) == 2) {
          const s16x4 kf = *(const s16x4*)kp;
#pragma unroll
          for (int qt = 0; qt < kQT; ++qt)
            s[kt][qt] = __builtin_amdgcn_mfma_f32_16x16x16bf16_1k(kf, qf[qt][dc], s[kt][qt], 0, 0, 0);
        } else {
          const f32x4 kf = *(const f32x4*)kp;
#pragma unroll
          for (int qt = 0; qt < kQT; ++qt) {
#pragma unroll
            for (int e = 0; e < 4; ++e)
              s[kt][qt] = __builtin_amdgcn_mfma_f32_16x16x4f32(kf[e], qf[qt][dc][e], s[kt][qt], 0, 0, 0);
          }
        }
      }
    }

    // ---- online softmax per query column
    typedef typename std::conditional<sizeof(T) == 2, s16x4, f32x4>::type pfrag_t;
    pfrag_t pf[4][kQT];
    // masking only on tiles that reach past Lk or (causal) past the wave's first query
    const bool need_mask = (j0 + kKT > a.Lk) || (a.causal && j0 + kKT - 1 > q0);
#pragma unroll
    for (int qt = 0; qt < kQT; ++qt) {
      const int q = q0 + qt * 16 + li;
      if (need_mask) {
#pragma unroll
        for (int kt = 0; kt < 4; ++kt)
#pragma unroll
          for (int i = 0; i < 4; ++i) {
            const int key = j0 + kt * 16 + 4 * g + i;
            if (key >= a.Lk || (a.causal && key > q)) s[kt][qt][i] = -INFINITY;
          }
      }
      float tmax = -INFINITY;     // max of the raw scores (scale > 0 commutes with max)
#pragma unroll
      for (int kt = 0; kt < 4; ++kt)
#pragma unroll
        for (int i = 0; i < 4; ++i) tmax = fmaxf(tmax, s[kt][qt][i]);
      tmax = fmaxf(tmax, __shfl_xor(tmax, 16));
      tmax = fmaxf(tmax, __shfl_xor(tmax, 32));
      const float mnew = fmaxf(mrow[qt], tmax);
      const bool none = mnew == -INFINITY;           // every key so far masked
      const float alpha = none ? 1.f : __builtin_amdgcn_exp2f((mrow[qt] - mnew) * sl2);
      const float nb = none ? 0.f : -mnew * sl2;
      mrow[qt] = mnew;
      float lsum = 0.f;
#pragma unroll
      for (int kt = 0; kt < 4; ++kt) {
        float p[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          p[i] = __builtin_amdgcn_exp2f(fmaf(s[kt][qt][i], sl2, nb));
          lsum += p[i];
        }
        if constexpr (sizeof(T) == 2) {
          s16x4 v;
#pragma unroll
          for (int i = 0; i < 4; ++i) v[i] = (short)f2bf(p[i]);
          pf[kt][qt] = v;
        } else {
          pf[kt][qt] = f32x4{p[0], p[1], p[2], p[3]};
        }
      }
      lrow[qt] = lrow[qt] * alpha + lsum;
#pragma unroll
      for (int dt = 0; dt < ND; ++dt) o[dt][qt] *= alpha;
    }

    // ---- O^T += V^T P^T
#pragma unroll
    for (int kt = 0; kt < 4; ++kt) {
#pragma unroll
      for (int dt = 0; dt < ND; ++dt) {
        if constexpr (sizeof(T) == 2) {
          // 16-lane group g reads V rows 16kt+4g .. +3, cols 16dt .. +15, transposed:
          // lane li gets column 16dt+li of those 4 rows = A[row d][k = 4g + j]
          const T* vp = Vs + (kt * 16 + 4 * g + (li >> 2)) * SV + dt * 16 + 4 * (li & 3);
          const s16x4 vf = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)vp);
#pragma unroll
          for (int qt = 0; qt < kQT; ++qt)
            o[dt][qt] = __builtin_amdgcn_mfma_f32_16x16x16bf16_1k(vf, pf[kt][qt], o[dt][qt], 0, 0, 0);
        } else {
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            const float vf = Vs[(kt * 16 + 4 * g + e) * SV + dt * 16 + li];
#pragma unroll
            for (int qt = 0; qt < kQT; ++qt)
              o[dt][qt] = __builtin_amdgcn_mfma_f32_16x16x4f32(vf, pf[kt][qt][e], o[dt][qt], 0, 0, 0);
          }
        }
      }
    }
  }

  // ---- normalise and store O[q][h*d + e]
  T* __restrict__ O = (T*)a.o + (long)b * a.so + (long)h * d;
#pragma unroll
  for (int qt = 0; qt < kQT; ++qt) {
    float l = lrow[qt];
    l += __shfl_xor(l, 16);
    l += __shfl_xor(l, 32);
    const float inv = l > 0.f ? 1.f / l : 0.f;
    const int q = q0 + qt * 16 + li;
    if (q >= a.Lq) continue;
#pragma unroll
    for (int dt = 0; dt < ND; ++dt) {
      const int e = dt * 16 + 4 * g;
      if (e >= d) continue;
      T* op = O + (long)q * a.ldo + e;
      if constexpr (sizeof(T) == 2) {
        s16x4 v;
#pragma unroll
        for (int i = 0; i < 4; ++i) v[i] = (short)f2bf(o[dt][qt][i] * inv);
        *(s16x4*)op = v;
      } else {
        *(f32x4*)op = o[dt][qt] * inv;
      }
    }
  }
}

// max over lanes {i, i^16, i^32, i^48} with gfx950's v_permlane16/32_swap (VALU, no LDS round trip as
// ds_bpermute would take): swapping a value with itself leaves each lane holding its partner's copy
__device__ __forceinline__ float quad_max(float x) {
  const auto a = __builtin_amdgcn_permlane16_swap(__float_as_uint(x), __float_as_uint(x), false, false);
  x = fmaxf(__uint_as_float(a[0]), __uint_as_float(a[1]));
  const auto b = __builtin_amdgcn_permlane32_swap(__float_as_uint(x), __float_as_uint(x), false, false);
  return fmaxf(__uint_as_float(b[0]), __uint_as_float(b[1]));
}

// ------------------------------------------------------------------------------------------------
// bf16 throughput kernel: v_mfma_f32_16x16x32_bf16 for both products.
//   S^T = K Q^T : K fragments by ds_read_b128 (d padded to DQ, a multiple of 32), Q^T in registers.
//   O^T += V^T P^T over 32-key chunks: P^T is the exponentiated S^T accumulator of two 16-key tiles
//   (lane group g holds keys 4g..4g+3 of each), V^T comes from two ds_read_b64_tr_b16 of the same
//   key sets, so the permuted k order matches on both operands.
// KT keys per LDS tile (128 at d <= 80, 64 at d = 160 to bound registers); 4 waves x 32 queries.
// ONES: the head dim leaves a zero pad column in V (d < DV); it is set to 1 so the PV MFMAs also produce
// the softmax row sums (O^T row d = sum_k P[q][k]) and the per-score VALU add disappears.
template <int DQ, int DV, int KT, bool ONES, int OCC = 2>
__global__ __launch_bounds__(256, OCC) void attn2_kernel(AttnArgs a) {
  constexpr int SK = DQ + 8;                                     // 16 rows x b128 reads conflict-free
  constexpr int SV = ((DV * 2 / 32) % 2 == 1) ? DV : DV + 16;    // 8 rows x 32 B tr reads conflict-free
  // QK^T contracts over DQ = 32 * NDC (head dim zero-padded).  (A 16x16x16 MFMA for a d % 32 == 8..16 tail was
  // tried: hipcc (ROCm 7.2) issues it right behind the 16x16x32 producing its accumulator with no wait states,
  // and the result is wrong — mixed-shape MFMA accumulation chains are avoided here.)
  // DQ % 32 == 16 (d = 40 -> 48): the last 16 dims go through one 16x16x16 MFMA into a SEPARATE
  // accumulator that the VALU adds to S (no mixed-shape MFMA chain), instead of padding d to 64.
  constexpr int NDC = DQ / 32, NDT = DV / 16, NKT = KT / 16, NKC = KT / 32;
  constexpr bool TAIL = DQ % 32 == 16;
  static_assert(DQ % 32 == 0 || TAIL, "head dim padding");
  typedef __attribute__((ext_vector_type(8))) short s16x8;
  __shared__ __attribute__((aligned(16))) bf16_t Ks[KT * SK];
  __shared__ __attribute__((aligned(16))) bf16_t Vs[KT * SV];

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int li = lane & 15, g = lane >> 4;
  const int b = blockIdx.z, h = blockIdx.y;
  const int qb0 = blockIdx.x * kQB;
  const int q0 = qb0 + wave * (kQT * 16);
  const int d = a.d;
  const bf16_t* __restrict__ Q = (const bf16_t*)a.q + (long)b * a.sq + (long)h * d;
  const bf16_t* __restrict__ K = (const bf16_t*)a.k + (long)b * a.sk + (long)h * d;
  const bf16_t* __restrict__ V = (const bf16_t*)a.v + (long)b * a.sv + (long)h * d;

  for (int i = tid; i < KT * SK; i += 256) Ks[i] = 0;
  for (int i = tid; i < KT * SV; i += 256) Vs[i] = (ONES && i % SV == a.d) ? (bf16_t)0x3F80 : (bf16_t)0;

  s16x8 qf[kQT][NDC];
  s16x4 qtl[kQT];
#pragma unroll
  for (int qt = 0; qt < kQT; ++qt) {
    const int q = q0 + qt * 16 + li;
#pragma unroll
    for (int dc = 0; dc < NDC; ++dc) {
      const int e = dc * 32 + 8 * g;
      s16x8 v = {0, 0, 0, 0, 0, 0, 0, 0};
      if (q < a.Lq && e < d) v = *(const s16x8*)(Q + (long)q * a.ldq + e);
      qf[qt][dc] = v;
    }
    qtl[qt] = s16x4{0, 0, 0, 0};
    if constexpr (TAIL) {
      const int e = NDC * 32 + 4 * g;
      if (q < a.Lq && e < d) qtl[qt] = *(const s16x4*)(Q + (long)q * a.ldq + e);
    }
  }
  f32x4 o[NDT][kQT];
#pragma unroll
  for (int i = 0; i < NDT; ++i)
#pragma unroll
    for (int j = 0; j < kQT; ++j) o[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  float mrow[kQT], lrow[kQT];
#pragma unroll
  for (int j = 0; j < kQT; ++j) { mrow[j] = -INFINITY; lrow[j] = 0.f; }

  const float sl2 = a.scale * 1.4426950408889634f;
  int kend = a.Lk;
  if (a.causal) kend = min(kend, qb0 + kQB);
  const int cpr = d / 8;                                   // 16-byte chunks per K/V row
  constexpr int NCH = (KT * (DV / 8) + 255) / 256;       // d <= DV
  uint4 kreg[NCH], vreg[NCH];
  auto load_regs = [&](int j0) {
#pragma unroll
    for (int u = 0; u < NCH; ++u) {
      const int idx = tid + 256 * u;
      kreg[u] = make_uint4(0, 0, 0, 0);
      vreg[u] = make_uint4(0, 0, 0, 0);
      if (idx < KT * cpr) {
        const int r = idx / cpr, c = idx - r * cpr;
        if (j0 + r < a.Lk) {
          kreg[u] = *(const uint4*)(K + (long)(j0 + r) * a.ldk + c * 8);
          vreg[u] = *(const uint4*)(V + (long)(j0 + r) * a.ldv + c * 8);
        }
      }
    }
  };
  load_regs(0);

  for (int j0 = 0; j0 < kend; j0 += KT) {
    __syncthreads();
#pragma unroll
    for (int u = 0; u < NCH; ++u) {
      const int idx = tid + 256 * u;
      if (idx < KT * cpr) {
        const int r = idx / cpr, c = idx - r * cpr;
        *(uint4*)(Ks + r * SK + c * 8) = kreg[u];
        uint2* pv = (uint2*)(Vs + r * SV + c * 8);
        pv[0] = make_uint2(vreg[u].x, vreg[u].y);
        pv[1] = make_uint2(vreg[u].z, vreg[u].w);
      }
    }
    __syncthreads();
    if (j0 + KT < kend) load_regs(j0 + KT);

    f32x4 s[NKT][kQT];
#pragma unroll
    for (int kt = 0; kt < NKT; ++kt) {
#pragma unroll
      for (int qt = 0; qt < kQT; ++qt) s[kt][qt] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int dc = 0; dc < NDC; ++dc) {
        const s16x8 kf = *(const s16x8*)(Ks + (kt * 16 + li) * SK + dc * 32 + 8 * g);
#pragma unroll
        for (int qt = 0; qt < kQT; ++qt)
          s[kt][qt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, kf),
                                                              __builtin_bit_cast(bf16x8, qf[qt][dc]), s[kt][qt], 0, 0, 0);
      }
      if constexpr (TAIL) {
        const s16x4 kt4 = *(const s16x4*)(Ks + (kt * 16 + li) * SK + NDC * 32 + 4 * g);
#pragma unroll
        for (int qt = 0; qt < kQT; ++qt) {
          const f32x4 t = __builtin_amdgcn_mfma_f32_16x16x16bf16_1k(kt4, qtl[qt], f32x4{0.f, 0.f, 0.f, 0.f}, 0, 0, 0);
          s[kt][qt] += t;
        }
      }
    }

    const bool need_mask = (j0 + KT > a.Lk) || (a.causal && j0 + KT - 1 > q0);
    float nbq[kQT];
#pragma unroll
    for (int qt = 0; qt < kQT; ++qt) {
      const int q = q0 + qt * 16 + li;
      if (need_mask) {
#pragma unroll
        for (int kt = 0; kt < NKT; ++kt)
#pragma unroll
          for (int i = 0; i < 4; ++i) {
            const int key = j0 + kt * 16 + 4 * g + i;
            if (key >= a.Lk || (a.causal && key > q)) s[kt][qt][i] = -INFINITY;
          }
      }
      float tmax = -INFINITY;
#pragma unroll
      for (int kt = 0; kt < NKT; ++kt)
        tmax = fmaxf(tmax, fmaxf(fmaxf(s[kt][qt][0], s[kt][qt][1]), fmaxf(s[kt][qt][2], s[kt][qt][3])));
      tmax = quad_max(tmax);
      const float mnew = fmaxf(mrow[qt], tmax);
      const bool none = mnew == -INFINITY;
      const float alpha = none ? 1.f : __builtin_amdgcn_exp2f((mrow[qt] - mnew) * sl2);
      nbq[qt] = none ? 0.f : -mnew * sl2;
      mrow[qt] = mnew;
      if constexpr (!ONES) lrow[qt] *= alpha;
#pragma unroll
      for (int dt = 0; dt < NDT; ++dt) o[dt][qt] *= alpha;
    }

    // per 32-key chunk: exponentiate into the B operand, then its PV MFMAs (keeps 1 chunk of P live)
#pragma unroll
    for (int c = 0; c < NKC; ++c) {
      s16x8 pf[kQT];
#pragma unroll
      for (int qt = 0; qt < kQT; ++qt) {
        float lsum = 0.f;
#pragma unroll
        for (int half = 0; half < 2; ++half)
#pragma unroll
          for (int i = 0; i < 4; ++i) {
            const float p = __builtin_amdgcn_exp2f(fmaf(s[2 * c + half][qt][i], sl2, nbq[qt]));
            if constexpr (!ONES) lsum += p;
            pf[qt][half * 4 + i] = (short)f2bf(p);
          }
        if constexpr (!ONES) lrow[qt] += lsum;
      }
#pragma unroll
      for (int dt = 0; dt < NDT; ++dt) {
        const bf16_t* v1 = Vs + (c * 32 + 4 * g + (li >> 2)) * SV + dt * 16 + 4 * (li & 3);
        const s16x4 t1 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)v1);
        const s16x4 t2 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(v1 + 16 * SV));
        const s16x8 vf = {t1[0], t1[1], t1[2], t1[3], t2[0], t2[1], t2[2], t2[3]};
#pragma unroll
        for (int qt = 0; qt < kQT; ++qt)
          o[dt][qt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, vf),
                                                              __builtin_bit_cast(bf16x8, pf[qt]), o[dt][qt], 0, 0, 0);
      }
    }
  }

  bf16_t* __restrict__ O = (bf16_t*)a.o + (long)b * a.so + (long)h * d;
#pragma unroll
  for (int qt = 0; qt < kQT; ++qt) {
    float l;
    if constexpr (ONES) {
      // row d of O^T: tile dt1 = d/16, lane group (d%16)/4, element d%4 (d % 4 == 0: element 0)
      float v = 0.f;
#pragma unroll
      for (int dt = 0; dt < NDT; ++dt)
        if (dt == d / 16) v = o[dt][qt][0];
      l = __shfl(v, li + 16 * ((d % 16) / 4));
    } else {
      l = lrow[qt];
      l += __shfl_xor(l, 16);
      l += __shfl_xor(l, 32);
    }
    const float inv = l > 0.f ? 1.f / l : 0.f;
    const int q = q0 + qt * 16 + li;
    if (q >= a.Lq) continue;
#pragma unroll
    for (int dt = 0; dt < NDT; ++dt) {
      const int e = dt * 16 + 4 * g;
      if (e >= d) continue;
      s16x4 v;
#pragma unroll
      for (int i = 0; i < 4; ++i) v[i] = (short)f2bf(o[dt][qt][i] * inv);
      *(s16x4*)(O + (long)q * a.ldo + e) = v;
    }
  }
}

void launch_bf16(const AttnArgs& a, hipStream_t s) {
  dim3 grid((a.Lq + kQB - 1) / kQB, a.H, a.B), block(256);
  const char* inst = a.d == 40 ? (g_attn_d40 == 1   ? "64, 48, 128, false"
                                  : g_attn_d40 == 2 ? "64, 48, 64, true, 3"
                                  : g_attn_d40 == 3 ? "64, 48, 64, true, 4"
                                  : g_attn_d40 == 4 ? "48, 48, 64, true, 3"
                                                    : "64, 48, 128, true, 2")
                     : a.d == 64 ? "64, 64, 128, false"
                     : a.d == 80 ? "96, 80, 64, false" : "160, 160, 32, false";
  ProfScope ps(prof_on() ? std::string("irx::(anonymous namespace)::attn2_kernel<") + inst + ">" : std::string(),
               4.0 * a.B * a.H * (double)a.Lq * a.Lk * a.d, s);
  switch (a.d) {
    case 40:
      if (g_attn_d40 == 1) attn2_kernel<64, 48, 128, false><<<grid, block, 0, s>>>(a);
      else if (g_attn_d40 == 2) attn2_kernel<64, 48, 64, true, 3><<<grid, block, 0, s>>>(a);
      else if (g_attn_d40 == 3) attn2_kernel<64, 48, 64, true, 4><<<grid, block, 0, s>>>(a);
      else if (g_attn_d40 == 4) attn2_kernel<48, 48, 64, true, 3><<<grid, block, 0, s>>>(a);
      else attn2_kernel<64, 48, 128, true><<<grid, block, 0, s>>>(a);
      break;
    case 64: attn2_kernel<64, 64, 128, false><<<grid, block, 0, s>>>(a); break;
    case 80: attn2_kernel<96, 80, 64, false><<<grid, block, 0, s>>>(a); break;
    case 160: attn2_kernel<160, 160, 32, false><<<grid, block, 0, s>>>(a); break;
    default: throw Error("attention: unsupported head dim " + std::to_string(a.d));
  }
  IRX_LAUNCH_CHECK();
}

template <typename T>
void launch_t(const AttnArgs& a, hipStream_t s) {
  dim3 grid((a.Lq + kQB - 1) / kQB, a.H, a.B), block(256);
  const int dp = (a.d + 15) / 16 * 16;
  ProfScope ps(prof_on() ? std::string("irx::(anonymous namespace)::attn_kernel<") +
                               (sizeof(T) == 2 ? "unsigned short" : "float") + ", " + std::to_string(dp) + ">"
                         : std::string(),
               4.0 * a.B * a.H * (double)a.Lq * a.Lk * a.d, s);
  switch (dp) {
    case 48: attn_kernel<T, 48><<<grid, block, 0, s>>>(a); break;
    case 64: attn_kernel<T, 64><<<grid, block, 0, s>>>(a); break;
    case 80: attn_kernel<T, 80><<<grid, block, 0, s>>>(a); break;
    case 160: attn_kernel<T, 160><<<grid, block, 0, s>>>(a); break;
    default: throw Error("attention: unsupported head dim " + std::to_string(a.d));
  }
  IRX_LAUNCH_CHECK();
}

}  // namespace

void attention(const AttnArgs& a, hipStream_t s) {
  const int es = a.dtype == F32 ? 4 : 2;
  IRX_CHECK(a.B > 0 && a.H > 0 && a.Lq > 0 && a.Lk > 0 && a.d > 0, "empty attention");
  IRX_CHECK(a.d % 4 == 0 && (a.d * es) % 16 == 0, "head dim must be a multiple of 16 bytes");
  IRX_CHECK((a.ldk * es) % 16 == 0 && (a.ldv * es) % 16 == 0, "K/V rows must be 16-byte aligned");
  IRX_CHECK((a.ldq * es) % 8 == 0 && (a.ldo * es) % 8 == 0, "Q/O rows must be 8-byte aligned");
  IRX_CHECK(((uintptr_t)a.k % 16) == 0 && ((uintptr_t)a.v % 16) == 0, "K/V base alignment");
  if (a.dtype == F32) launch_t<float>(a, s);
  else if (g_attn_v2 && a.d % 8 == 0 && (a.ldq % 8) == 0 && ((uintptr_t)a.q % 16) == 0) launch_bf16(a, s);
  else launch_t<bf16_t>(a, s);
}

bool g_attn_v2 = true;
int g_attn_d40 = 2;   // d = 40 variant (A/B): 0 128-key tiles (ones-column row sums), 1 VALU row sums,
                      // 2/3 64-key tiles at 3/4 blocks per CU (2, default: +8% self, +40% cross-attention; 3 spills)

}  // namespace irx
