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
extern int g_attn_pf80;
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

  const T* __restrict__ Q = (const T*)a.q + (long)b * a.sq + (long)h * (a.hsq ? a.hsq : d);
  const T* __restrict__ K = (const T*)a.k + (long)b * a.sk + (long)h * (a.hsk ? a.hsk : d);
  const T* __restrict__ V = (const T*)a.v + (long)b * a.sv + (long)h * (a.hsv ? a.hsv : d);

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

  const float sl2 = a.q_scaled ? 1.f : a.scale * 1.4426950408889634f;   // softmax in base 2: exp(x*scale) = exp2(x*sl2)
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
  T* __restrict__ O = (T*)a.o + (long)b * a.so + (long)h * (a.hso ? a.hso : d);
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

// ------------------------------------------------------------------------------------------------
// attn3: bf16 / fp16 flash attention on v_mfma_f32_32x32x16 (the shape that holds the SIMD's VALU issue
// for 8 of its 32 cycles instead of 8 of 16 — this kernel is bounded by the softmax VALU work at d = 40).
//   S^T = K Q^T per 32-key sub-tile: A = K rows (ds_read_b128), B = Q^T in registers (d padded to 16);
//     lane = query column (lane & 31), its 16 accumulator registers = 16 of the 32 keys, the other 16 in
//     lane ^ 32 (one v_permlane32_swap finishes a row max).
//   P^T is that accumulator converted in place: registers 8s .. 8s+7 are the B operand of k-step s of
//     O^T += V^T P^T (guide §3, "an accumulator tile as the next MFMA's operand"); the V^T A operand comes
//     out of the row-major V tile with two ds_read_b64_tr_b16 per k-step, in the matching key order.
//   Softmax in base 2 with scale*log2(e) folded into q (in the to_q weights, or here at the Q load) and
//     the running max folded into the accumulator initialisation: S' = Q K^T - m comes out of the MFMA
//     chain and p = exp2(S') needs no subtraction.  The max is deferred (guide T13): m moves only when a
//     tile's max exceeds it by more than THR = 8, so p <= 2^8 (exact in bf16/fp16 storage; row sums and
//     O in fp32).  At a move, the pending tile's S' and everything accumulated (O, row sum) are rescaled
//     once, before any of this tile's p is formed.
//   Row sums: a ones column at V column d (d % 32 != 0 leaves a zero pad column) makes the PV MFMAs
//     produce sum_k p (the same rounded p as the numerator); d % 32 == 0: fp32 VALU sums.
// Block = 4 waves x 32 queries; KT = 64 keys per tile, register-staged K/V prefetch.  Grid: (batch, head) groups of query blocks on one XCD.
template <typename T> constexpr uint16_t one_bits();
template <> constexpr uint16_t one_bits<bf16_t>() { return 0x3F80; }
template <> constexpr uint16_t one_bits<f16_t>() { return 0x3C00; }
// a large negative score offset of the storage type (-65536 in bf16, -65504 in fp16): exp2 of it is exactly 0 in fp32
template <typename T> constexpr uint16_t neg_big_bits();
template <> constexpr uint16_t neg_big_bits<bf16_t>() { return 0xC780; }
template <> constexpr uint16_t neg_big_bits<f16_t>() { return 0xFBFF; }

__device__ __forceinline__ float xlane32(float x) {   // value of lane l ^ 32
  const auto b = __builtin_amdgcn_permlane32_swap(__float_as_uint(x), __float_as_uint(x), false, false);
  return __uint_as_float((threadIdx.x & 32) ? b[0] : b[1]);
}

// waves per SIMD the register file allows without spills (d = 40 / 64-key tiles is the hot instantiation)
template <int D, int KT> constexpr int attn3_occ() {
  return D <= 40 ? (KT <= 64 ? 4 : 3) : D <= 64 ? (KT <= 64 ? 3 : 2) : D <= 80 ? 2 : 1;
}

// PF (option attn_pf, non-causal streamed tiles): every K fragment of a tile is read before its first QK^T MFMA and
// every V^T fragment right after the QK^T MFMAs are issued (under the row max / exp), instead of one LDS read in front
// of each MFMA — 14 serial LDS round trips per tile and wave become 2; the extra live fragments need 3 waves per SIMD
// (PF = the waves per SIMD the launch bounds ask for).
template <typename T, int D, int KT, bool CAUSAL, bool RES, int PF = 0>
__global__ __launch_bounds__(256, (PF ? PF : attn3_occ<D, KT>())) void attn3_kernel(AttnArgs a) {
  constexpr int QB = 128;                                  // queries per block (4 waves x 32)
  constexpr int DQ = (D + 15) / 16 * 16, NS = DQ / 16;     // QK^T contraction, 16-deep k-steps
  constexpr int NDT = (D + 31) / 32;                       // 32-row tiles of O^T
  constexpr bool ONES = D % 32 != 0;
  constexpr int DVP = NDT * 32;
  constexpr int SK = ((DQ / 8) % 2 == 0) ? DQ + 8 : DQ;   // odd 16-B slots per row: b128 reads conflict-free
  constexpr int SV = (DVP % 128 == 32 || DVP % 128 == 96) ? DVP : DVP + 32;   // tr reads conflict-free
  constexpr int NSUB = KT / 32;
  constexpr int CPR = D / 8;                               // 16-byte chunks per K/V row
  constexpr int NCH = (KT * CPR + 255) / 256;
  constexpr float THR = 8.f;
  static_assert(D % 8 == 0 && KT % 32 == 0, "attn3 shape");
  // two LDS stages: tile j+1 is written under tile j's compute, one barrier per tile
  __shared__ __attribute__((aligned(16))) uint16_t Ks2[2 * KT * SK];
  __shared__ __attribute__((aligned(16))) uint16_t Vs2[2 * KT * SV];

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int r = lane & 31, hh = lane >> 5, g = lane >> 4;
  // RES (host: non-causal, Lk <= 2 KT — the cross-attention's 77 text tokens): the whole K/V sits in the two LDS
  // stages, staged once; the block then runs qrep groups of QB queries against it with no barrier in the loop
  static_assert(!(RES && CAUSAL), "resident K/V is non-causal only");
  const int qrep = RES && a.qrep > 1 ? a.qrep : 1;
  const int nq = (a.Lq + QB * qrep - 1) / (QB * qrep);
  const int nblk = nq * a.H * a.B;
  const int lid = a.xcd ? xcd_remap(blockIdx.x, nblk) : (int)blockIdx.x;
  const int qb = lid % nq, bh = lid / nq;
  const int b = bh / a.H, h = bh - b * a.H;
  const T* __restrict__ Q = (const T*)a.q + (long)b * a.sq + (long)h * (a.hsq ? a.hsq : D);
  const T* __restrict__ K = (const T*)a.k + (long)b * a.sk + (long)h * (a.hsk ? a.hsk : D);
  const T* __restrict__ V = (const T*)a.v + (long)b * a.sv + (long)h * (a.hsv ? a.hsv : D);

  // pad columns: K[.][d] = 1 when -m rides in the padding (PADM below), V[.][d] = 1 for the row sums
  // (16-byte chunks: SK, SV and D are multiples of 8, so column d is element 0 of its chunk)
  static_assert(SK % 8 == 0 && SV % 8 == 0, "pad-column chunks");
  // (the pad element selected as a scalar: a select between two uint4 constants becomes a scratch-memory table).
  // d = 160: 164 two-byte stores per thread became 21 (self-attention L = 256 21.6 -> 17.5 us); the streamed d = 80
  // kernel without the prefetch keeps the element loop (its main loop scheduled 4 % slower with the chunked one), its
  // default PF = 2 form takes the chunks (62 -> 58.5 us, profiles/r06_kbench_attn_init.txt)
  constexpr bool VINIT = RES || D != 80 || PF != 0;
  if constexpr (VINIT) {
    for (int i = tid; i < 2 * KT * SK / 8; i += 256)
      ((uint4*)Ks2)[i] = make_uint4((DQ > D && (8 * i) % SK == D) ? (unsigned)one_bits<T>() : 0u, 0u, 0u, 0u);
    for (int i = tid; i < 2 * KT * SV / 8; i += 256)
      ((uint4*)Vs2)[i] = make_uint4((ONES && (8 * i) % SV == D) ? (unsigned)one_bits<T>() : 0u, 0u, 0u, 0u);
  } else {
    for (int i = tid; i < 2 * KT * SK; i += 256) Ks2[i] = (DQ > D && i % SK == D) ? one_bits<T>() : (uint16_t)0;
    for (int i = tid; i < 2 * KT * SV; i += 256) Vs2[i] = (ONES && i % SV == D) ? one_bits<T>() : (uint16_t)0;
  }

  // per-thread staging slots (row, 16-byte chunk) of a K/V tile, fixed for the kernel: pointers and LDS offsets
  // computed once; a full tile (every row < Lk) loads with no per-row checks
  uint4 kreg[NCH], vreg[NCH];
  const T* kp[NCH];
  const T* vp[NCH];
  int krow[NCH], ksoff[NCH], vsoff[NCH];
#pragma unroll
  for (int u = 0; u < NCH; ++u) {
    const int idx = min(tid + 256 * u, KT * CPR - 1);
    const int row = idx / CPR, c = idx - row * CPR;
    krow[u] = row;
    kp[u] = K + (long)row * a.ldk + c * 8;
    vp[u] = V + (long)row * a.ldv + c * 8;
    ksoff[u] = row * SK + c * 8;
    vsoff[u] = row * SV + c * 8;
  }
  auto slot_ok = [&](int u) { return u < NCH - 1 || tid + 256 * u < KT * CPR; };
  auto load_to = [&](int j0, uint4 (&kr)[NCH], uint4 (&vr)[NCH]) {
    const long ko = (long)j0 * a.ldk, vo = (long)j0 * a.ldv;
    if (j0 + KT <= a.Lk) {
#pragma unroll
      for (int u = 0; u < NCH; ++u)
        if (slot_ok(u)) {
          kr[u] = *(const uint4*)(kp[u] + ko);
          vr[u] = *(const uint4*)(vp[u] + vo);
        }
    } else {
#pragma unroll
      for (int u = 0; u < NCH; ++u) {
        const bool in = j0 + krow[u] < a.Lk;
        kr[u] = in ? *(const uint4*)(kp[u] + ko) : make_uint4(0, 0, 0, 0);
        vr[u] = in ? *(const uint4*)(vp[u] + vo) : make_uint4(0, 0, 0, 0);
      }
    }
  };
  auto stage_from = [&](int buf, const uint4 (&kr)[NCH], const uint4 (&vr)[NCH]) {
#pragma unroll
    for (int u = 0; u < NCH; ++u)
      if (slot_ok(u)) {
        *(uint4*)(Ks2 + buf * KT * SK + ksoff[u]) = kr[u];
        *(uint4*)(Vs2 + buf * KT * SV + vsoff[u]) = vr[u];
      }
  };
  // (the streamed loop's own copies: routed through load_to / stage_from, the d = 80 kernel's loop scheduled worse)
  auto load = [&](int j0) {
    const long ko = (long)j0 * a.ldk, vo = (long)j0 * a.ldv;
    if (j0 + KT <= a.Lk) {
#pragma unroll
      for (int u = 0; u < NCH; ++u)
        if (slot_ok(u)) {
          kreg[u] = *(const uint4*)(kp[u] + ko);
          vreg[u] = *(const uint4*)(vp[u] + vo);
        }
    } else {
#pragma unroll
      for (int u = 0; u < NCH; ++u) {
        const bool in = j0 + krow[u] < a.Lk;
        kreg[u] = in ? *(const uint4*)(kp[u] + ko) : make_uint4(0, 0, 0, 0);
        vreg[u] = in ? *(const uint4*)(vp[u] + vo) : make_uint4(0, 0, 0, 0);
      }
    }
  };
  auto stage = [&](int buf) {
#pragma unroll
    for (int u = 0; u < NCH; ++u)
      if (slot_ok(u)) {
        *(uint4*)(Ks2 + buf * KT * SK + ksoff[u]) = kreg[u];
        *(uint4*)(Vs2 + buf * KT * SV + vsoff[u]) = vreg[u];
      }
  };
  // raw Q^T fragments of query group rep (B operand): lane (r, hh) holds q[qrow][16s + 8hh .. +7].  RES: the next
  // group's are requested before the current group's MFMAs (their latency hides under them; QPF, where the register
  // budget allows), and group 0's together with both K/V tiles — one global round trip before the first MFMA
  // instead of three (K/V tile 0 -> stage -> tile 1 -> stage -> Q).  Only the order of the loads changes.
  constexpr bool QPF = RES && D <= 80;
  uint4 qn[NS];
  auto loadq = [&](int rep) {
    const int qr = (qb * qrep + rep) * QB + wave * 32 + r;
#pragma unroll
    for (int s = 0; s < NS; ++s) {
      const int e = 16 * s + 8 * hh;
      qn[s] = (qr < a.Lq && e < D) ? *(const uint4*)(Q + (long)qr * a.ldq + e) : make_uint4(0, 0, 0, 0);
    }
  };
  if constexpr (RES) {
    uint4 k1[NCH], v1[NCH];
    const bool two = KT < a.Lk;
    loadq(0);
    load(0);
    if (two) load_to(KT, k1, v1);
    __syncthreads();          // pad-column initialisation complete
    stage(0);
    if (two) stage_from(1, k1, v1);
    __syncthreads();
  }

  for (int rep = 0; rep < qrep; ++rep) {
  const int q0 = (qb * qrep + rep) * QB + wave * 32;
  const int qrow = q0 + r;
  // Q^T fragments (B operand), pre-scaled by scale*log2(e)
  uint4 qf[NS];
  const float sl2 = a.scale * 1.4426950408889634f;
  if constexpr (RES) {
    if (rep > 0 && !QPF) loadq(rep);
#pragma unroll
    for (int s = 0; s < NS; ++s) qf[s] = qn[s];
    if constexpr (QPF) {
      if (rep + 1 < qrep) loadq(rep + 1);
    }
  }
#pragma unroll
  for (int s = 0; s < NS; ++s) {
    uint4 v = RES ? qf[s] : make_uint4(0, 0, 0, 0);
    if constexpr (!RES) {   // (streamed K/V: the Q loads in front of the first K/V tile's, as before)
      const int e = 16 * s + 8 * hh;
      if (qrow < a.Lq && e < D) v = *(const uint4*)(Q + (long)qrow * a.ldq + e);
    }
    if (!a.q_scaled) {
      float f[8];
      Vec16<T>::unpack(v, f);
#pragma unroll
      for (int j = 0; j < 8; ++j) f[j] *= sl2;
      v = Vec16<T>::pack(f);
    }
    qf[s] = v;
  }

  f32x16 oacc[NDT];
#pragma unroll
  for (int i = 0; i < NDT; ++i)
#pragma unroll
    for (int k = 0; k < 16; ++k) oacc[i][k] = 0.f;
  // m: the running max, always a value of the storage type (so -m is exact in a 16-bit operand).
  // PADM (d < the 16-padded contraction): -m rides in the zero padding as one more k: K[.][d] = 1 (in LDS),
  // Q[q][d] = -m (lane half 1, k-step NS-1, element 0), so the MFMA chain itself yields S - m.  Otherwise
  // the accumulators start at -m.
  constexpr bool PADM = DQ > D;
  constexpr int PADS = D / 16, PADE = (D % 16) - 8;   // k-step and element of column d in lane half 1
  static_assert(!PADM || (D % 16 == 8 && PADE == 0), "pad column at element 0 of lane half 1");
  float m = 0.f, lsum = 0.f;
  bool first = true;
  auto set_qpad = [&]() {   // Q^T fragment element holding -m (lane half 1 only; lane half 0 holds d-8 .. d-1)
    if constexpr (PADM) {
      if (hh) qf[PADS].x = (qf[PADS].x & 0xFFFF0000u) | (Mfma<T>::pack2(-m, 0.f) & 0xFFFFu);
    }
  };

  const int kend = CAUSAL ? min(a.Lk, qb * QB + QB) : a.Lk;
  if constexpr (!RES) {
    load(0);
    __syncthreads();          // pad-column initialisation complete
    stage(0);
    __syncthreads();
    if (KT < kend) load(KT);
  }

  for (int j0 = 0, it = 0; j0 < kend; j0 += KT, ++it) {
    const uint16_t* Ks = Ks2 + (it & 1) * KT * SK;
    const uint16_t* Vs = Vs2 + (it & 1) * KT * SV;

    // ---- S'^T = K Q^T - m
    f32x16 sacc[NSUB];
    const float init = (PADM || first) ? 0.f : -m;
#pragma unroll
    for (int c = 0; c < NSUB; ++c)
#pragma unroll
      for (int k = 0; k < 16; ++k) sacc[c][k] = init;
    if constexpr (PF) {
      uint4 kf[NS][NSUB];
#pragma unroll
      for (int s = 0; s < NS; ++s)
#pragma unroll
        for (int c = 0; c < NSUB; ++c) kf[s][c] = *(const uint4*)(Ks + (c * 32 + r) * SK + 16 * s + 8 * hh);
#pragma unroll
      for (int s = 0; s < NS; ++s)
#pragma unroll
        for (int c = 0; c < NSUB; ++c) sacc[c] = Mfma<T>::m32x32x16(kf[s][c], qf[s], sacc[c]);
    } else {
      if (a.prio) __builtin_amdgcn_s_setprio(1);
#pragma unroll
      for (int s = 0; s < NS; ++s)
#pragma unroll
        for (int c = 0; c < NSUB; ++c) {
          const uint4 kf = *(const uint4*)(Ks + (c * 32 + r) * SK + 16 * s + 8 * hh);
          sacc[c] = Mfma<T>::m32x32x16(kf, qf[s], sacc[c]);
        }
      if (a.prio) __builtin_amdgcn_s_setprio(0);
    }
    // V^T fragments of the tile (PF: read now, under the softmax; otherwise in front of each PV MFMA)
    auto vfrag = [&](int c, int dt, int s2) {
      const int krow = 32 * c + 16 * s2 + 4 * (g >> 1) + ((lane & 15) >> 2);
      const int col = 32 * dt + 16 * (g & 1) + 4 * (lane & 3);
      const s16x4 t1 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(Vs + krow * SV + col));
      const s16x4 t2 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(Vs + (krow + 8) * SV + col));
      return make_uint4(__builtin_bit_cast(uint2, t1).x, __builtin_bit_cast(uint2, t1).y,
                        __builtin_bit_cast(uint2, t2).x, __builtin_bit_cast(uint2, t2).y);
    };
    uint4 vpf[PF ? NSUB : 1][PF ? NDT : 1][2];
    if constexpr (PF) {
#pragma unroll
      for (int c = 0; c < NSUB; ++c)
#pragma unroll
        for (int dt = 0; dt < NDT; ++dt)
#pragma unroll
          for (int s2 = 0; s2 < 2; ++s2) vpf[c][dt][s2] = vfrag(c, dt, s2);
    }
    if (j0 + KT > a.Lk || (CAUSAL && j0 + KT - 1 > q0)) {
#pragma unroll
      for (int c = 0; c < NSUB; ++c)
#pragma unroll
        for (int k = 0; k < 16; ++k) {
          const int key = j0 + 32 * c + (k & 3) + 8 * (k >> 2) + 4 * hh;
          if (key >= a.Lk || (CAUSAL && key > qrow)) sacc[c][k] = -INFINITY;
        }
    }
    // row max: four independent v_max3_f32 chains (short dependency chains), then the other lane half
    float mx[4];
#pragma unroll
    for (int t = 0; t < 4; ++t) mx[t] = fmaxf(sacc[0][4 * t], sacc[0][4 * t + 1]);
#pragma unroll
    for (int c = 0; c < NSUB; ++c)
#pragma unroll
      for (int t = 0; t < 4; ++t)
#pragma unroll
        for (int k = (c == 0 ? 2 : 0); k < 4; k += 2)
          mx[t] = fmaxf(fmaxf(mx[t], sacc[c][4 * t + k]), sacc[c][4 * t + k + 1]);
    float tmax = fmaxf(fmaxf(mx[0], mx[1]), fmaxf(mx[2], mx[3]));
    tmax = fmaxf(tmax, xlane32(tmax));
    if (first || __any(tmax > THR)) {
      // move m (first tile: to the tile max; later: up by the excess, deferred until it passes THR)
      const float tgt = first ? (tmax == -INFINITY ? 0.f : m + tmax) : m + fmaxf(tmax, 0.f);
      const float mn = Mfma<T>::round(tgt);
      const float delta = mn - m;
      const float alpha = __builtin_amdgcn_exp2f(-delta);
#pragma unroll
      for (int c = 0; c < NSUB; ++c)
#pragma unroll
        for (int k = 0; k < 16; ++k) sacc[c][k] -= delta;
      if (!first) {
#pragma unroll
        for (int i = 0; i < NDT; ++i)
#pragma unroll
          for (int k = 0; k < 16; ++k) oacc[i][k] *= alpha;
        if constexpr (!ONES) lsum *= alpha;
      }
      m = mn;
      first = false;
      set_qpad();
    }

    // ---- O^T += V^T P^T, one 32-key sub-tile at a time
#pragma unroll
    for (int c = 0; c < NSUB; ++c) {
      uint4 pb[2];
#pragma unroll
      for (int s2 = 0; s2 < 2; ++s2) {
        float p[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          p[j] = __builtin_amdgcn_exp2f(sacc[c][8 * s2 + j]);
          if constexpr (!ONES) lsum += p[j];
        }
        pb[s2] = make_uint4(Mfma<T>::pack2(p[0], p[1]), Mfma<T>::pack2(p[2], p[3]), Mfma<T>::pack2(p[4], p[5]),
                            Mfma<T>::pack2(p[6], p[7]));
      }
#pragma unroll
      for (int dt = 0; dt < NDT; ++dt)
#pragma unroll
        for (int s2 = 0; s2 < 2; ++s2) {
          if constexpr (PF) {
            oacc[dt] = Mfma<T>::m32x32x16(vpf[c][dt][s2], pb[s2], oacc[dt]);
          } else {
            const uint4 vf = vfrag(c, dt, s2);
            if (a.prio) __builtin_amdgcn_s_setprio(1);
            oacc[dt] = Mfma<T>::m32x32x16(vf, pb[s2], oacc[dt]);
            if (a.prio) __builtin_amdgcn_s_setprio(0);
          }
        }
    }
    // tile j+1 (registers since last iteration) into the other stage, last read in iteration it-1: every wave
    // has passed the barrier that ended it-1
    if constexpr (!RES) {
      if (j0 + KT < kend) stage((it + 1) & 1);
      __syncthreads();
      if (j0 + 2 * KT < kend) load(j0 + 2 * KT);
    }
  }

  // ---- normalise, store O[q][h*d + e] (runs of 4 consecutive e per lane)
  float l;
  if constexpr (ONES) {
    constexpr int dts = D / 32, rho = D % 32, hs = (rho >> 2) & 1, reg = (rho & 3) + 4 * (rho >> 3);
    const float v = oacc[dts][reg];
    const float o = xlane32(v);
    l = hh == hs ? v : o;
  } else {
    l = lsum + xlane32(lsum);
  }
  const float inv = l > 0.f ? 1.f / l : 0.f;
  if (qrow < a.Lq) {
    T* __restrict__ O = (T*)a.o + (long)b * a.so + (long)h * (a.hso ? a.hso : D) + (long)qrow * a.ldo;
#pragma unroll
    for (int dt = 0; dt < NDT; ++dt)
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const int e = 32 * dt + 8 * k + 4 * hh;
        if (e >= D) continue;
        *(uint2*)(O + e) = make_uint2(Mfma<T>::pack2(oacc[dt][4 * k] * inv, oacc[dt][4 * k + 1] * inv),
                                      Mfma<T>::pack2(oacc[dt][4 * k + 2] * inv, oacc[dt][4 * k + 3] * inv));
      }
  }
  }   // rep
}

// ------------------------------------------------------------------------------------------------
// attn3q: attn3 (non-causal, K/V streamed, whole-tile fragment prefetch) with TWO independent 32-query groups per
// wave (block = 4 waves x 64 queries).  Every K fragment and V^T fragment read from LDS feeds both groups' MFMAs (half
// the LDS reads per MFMA of attn3), and the two groups' softmax chains are independent, so one group's exp / convert
// work can issue beside the other group's MFMAs inside one wave instead of relying on other waves for the overlap.
// Per group the arithmetic is attn3's operation for operation (same MFMA order per accumulator, the deferred-max
// decision taken over the group's own 32 queries), so the output is bit-identical.  2 waves / SIMD.
template <typename T, int D, int KT>
__global__ __launch_bounds__(256, 2) void attn3q_kernel(AttnArgs a) {
  constexpr int G = 2;                                     // query groups per wave
  constexpr int QB = 4 * 32 * G;                           // queries per block
  constexpr int DQ = (D + 15) / 16 * 16, NS = DQ / 16;
  constexpr int NDT = (D + 31) / 32;
  constexpr bool ONES = D % 32 != 0;
  constexpr int DVP = NDT * 32;
  constexpr int SK = ((DQ / 8) % 2 == 0) ? DQ + 8 : DQ;
  constexpr int SV = (DVP % 128 == 32 || DVP % 128 == 96) ? DVP : DVP + 32;
  constexpr int NSUB = KT / 32;
  constexpr int CPR = D / 8;
  constexpr int NCH = (KT * CPR + 255) / 256;
  constexpr float THR = 8.f;
  constexpr bool PADM = DQ > D;
  static_assert(D % 8 == 0 && KT % 32 == 0 && PADM && ONES, "attn3q: the d = 40 shape");
  __shared__ __attribute__((aligned(16))) uint16_t Ks2[2 * KT * SK];
  __shared__ __attribute__((aligned(16))) uint16_t Vs2[2 * KT * SV];

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int r = lane & 31, hh = lane >> 5, g = lane >> 4;
  const int nq = (a.Lq + QB - 1) / QB;
  const int nblk = nq * a.H * a.B;
  const int lid = a.xcd ? xcd_remap(blockIdx.x, nblk) : (int)blockIdx.x;
  const int qb = lid % nq, bh = lid / nq;
  const int b = bh / a.H, h = bh - b * a.H;
  const T* __restrict__ Q = (const T*)a.q + (long)b * a.sq + (long)h * (a.hsq ? a.hsq : D);
  const T* __restrict__ K = (const T*)a.k + (long)b * a.sk + (long)h * (a.hsk ? a.hsk : D);
  const T* __restrict__ V = (const T*)a.v + (long)b * a.sv + (long)h * (a.hsv ? a.hsv : D);

  // K pad columns: d = 1 (carries -m from Q), d + 1 = the key mask (0; neg_big for keys past Lk, Q[d + 1] = 1), so
  // a ragged last key tile needs no compare / select pass over the scores
  // (16-byte chunks, the pad element selected as a scalar; SK, SV, D multiples of 8)
  for (int i = tid; i < 2 * KT * SK / 8; i += 256)
    ((uint4*)Ks2)[i] = make_uint4((8 * i) % SK == D ? (unsigned)one_bits<T>() : 0u, 0u, 0u, 0u);
  for (int i = tid; i < 2 * KT * SV / 8; i += 256)
    ((uint4*)Vs2)[i] = make_uint4((8 * i) % SV == D ? (unsigned)one_bits<T>() : 0u, 0u, 0u, 0u);

  uint4 kreg[NCH], vreg[NCH];
  const T* kp[NCH];
  const T* vp[NCH];
  int krow[NCH], ksoff[NCH], vsoff[NCH];
#pragma unroll
  for (int u = 0; u < NCH; ++u) {
    const int idx = min(tid + 256 * u, KT * CPR - 1);
    const int row = idx / CPR, c = idx - row * CPR;
    krow[u] = row;
    kp[u] = K + (long)row * a.ldk + c * 8;
    vp[u] = V + (long)row * a.ldv + c * 8;
    ksoff[u] = row * SK + c * 8;
    vsoff[u] = row * SV + c * 8;
  }
  auto slot_ok = [&](int u) { return u < NCH - 1 || tid + 256 * u < KT * CPR; };
  auto load = [&](int j0) {
    const long ko = (long)j0 * a.ldk, vo = (long)j0 * a.ldv;
    if (j0 + KT <= a.Lk) {
#pragma unroll
      for (int u = 0; u < NCH; ++u)
        if (slot_ok(u)) {
          kreg[u] = *(const uint4*)(kp[u] + ko);
          vreg[u] = *(const uint4*)(vp[u] + vo);
        }
    } else {
#pragma unroll
      for (int u = 0; u < NCH; ++u) {
        const bool in = j0 + krow[u] < a.Lk;
        kreg[u] = in ? *(const uint4*)(kp[u] + ko) : make_uint4(0, 0, 0, 0);
        vreg[u] = in ? *(const uint4*)(vp[u] + vo) : make_uint4(0, 0, 0, 0);
      }
    }
  };
  auto stage = [&](int buf, int j0) {
#pragma unroll
    for (int u = 0; u < NCH; ++u)
      if (slot_ok(u)) {
        *(uint4*)(Ks2 + buf * KT * SK + ksoff[u]) = kreg[u];
        *(uint4*)(Vs2 + buf * KT * SV + vsoff[u]) = vreg[u];
      }
    if (j0 + KT > a.Lk && tid < KT && j0 + tid >= a.Lk)   // (the last tile is the only partial one)
      Ks2[buf * KT * SK + tid * SK + D + 1] = neg_big_bits<T>();
  };

  const int q0 = qb * QB + wave * 32 * G;
  uint4 qf[G][NS];
  const float sl2 = a.scale * 1.4426950408889634f;
#pragma unroll
  for (int gq = 0; gq < G; ++gq)
#pragma unroll
    for (int s = 0; s < NS; ++s) {
      const int e = 16 * s + 8 * hh, qrow = q0 + 32 * gq + r;
      uint4 v = make_uint4(0, 0, 0, 0);
      if (qrow < a.Lq && e < D) v = *(const uint4*)(Q + (long)qrow * a.ldq + e);
      if (!a.q_scaled) {
        float f[8];
        Vec16<T>::unpack(v, f);
#pragma unroll
        for (int j = 0; j < 8; ++j) f[j] *= sl2;
        v = Vec16<T>::pack(f);
      }
      if (e == D) v.x = (uint32_t)one_bits<T>() << 16;   // Q[d + 1] = 1: the key-mask column
      qf[gq][s] = v;
    }
  f32x16 oacc[G][NDT];
#pragma unroll
  for (int gq = 0; gq < G; ++gq)
#pragma unroll
    for (int i = 0; i < NDT; ++i)
#pragma unroll
      for (int k = 0; k < 16; ++k) oacc[gq][i][k] = 0.f;
  constexpr int PADS = D / 16;
  float m[G] = {0.f, 0.f};
  bool first = true;

  const int kend = a.Lk;
  load(0);
  __syncthreads();
  stage(0, 0);
  __syncthreads();
  if (KT < kend) load(KT);

  for (int j0 = 0, it = 0; j0 < kend; j0 += KT, ++it) {
    const uint16_t* Ks = Ks2 + (it & 1) * KT * SK;
    const uint16_t* Vs = Vs2 + (it & 1) * KT * SV;
    f32x16 sacc[G][NSUB];
#pragma unroll
    for (int gq = 0; gq < G; ++gq)
#pragma unroll
      for (int c = 0; c < NSUB; ++c)
#pragma unroll
        for (int k = 0; k < 16; ++k) sacc[gq][c][k] = 0.f;
    {
      uint4 kf[NS][NSUB];
#pragma unroll
      for (int s = 0; s < NS; ++s)
#pragma unroll
        for (int c = 0; c < NSUB; ++c) kf[s][c] = *(const uint4*)(Ks + (c * 32 + r) * SK + 16 * s + 8 * hh);
      // (group-major: group 0's scores complete while group 1's MFMAs still run, so its row max can start)
#pragma unroll
      for (int gq = 0; gq < G; ++gq)
#pragma unroll
        for (int s = 0; s < NS; ++s)
#pragma unroll
          for (int c = 0; c < NSUB; ++c) sacc[gq][c] = Mfma<T>::m32x32x16(kf[s][c], qf[gq][s], sacc[gq][c]);
    }
    uint4 vpf[NSUB][NDT][2];
#pragma unroll
    for (int c = 0; c < NSUB; ++c)
#pragma unroll
      for (int dt = 0; dt < NDT; ++dt)
#pragma unroll
        for (int s2 = 0; s2 < 2; ++s2) {
          const int krow = 32 * c + 16 * s2 + 4 * (g >> 1) + ((lane & 15) >> 2);
          const int col = 32 * dt + 16 * (g & 1) + 4 * (lane & 3);
          const s16x4 t1 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(Vs + krow * SV + col));
          const s16x4 t2 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(Vs + (krow + 8) * SV + col));
          vpf[c][dt][s2] = make_uint4(__builtin_bit_cast(uint2, t1).x, __builtin_bit_cast(uint2, t1).y,
                                      __builtin_bit_cast(uint2, t2).x, __builtin_bit_cast(uint2, t2).y);
        }
    float tmax[G];
#pragma unroll
    for (int gq = 0; gq < G; ++gq) {
      float mx[4];
#pragma unroll
      for (int t = 0; t < 4; ++t) mx[t] = fmaxf(sacc[gq][0][4 * t], sacc[gq][0][4 * t + 1]);
#pragma unroll
      for (int c = 0; c < NSUB; ++c)
#pragma unroll
        for (int t = 0; t < 4; ++t)
#pragma unroll
          for (int k = (c == 0 ? 2 : 0); k < 4; k += 2)
            mx[t] = fmaxf(fmaxf(mx[t], sacc[gq][c][4 * t + k]), sacc[gq][c][4 * t + k + 1]);
      const float tm = fmaxf(fmaxf(mx[0], mx[1]), fmaxf(mx[2], mx[3]));
      tmax[gq] = fmaxf(tm, xlane32(tm));
    }
#pragma unroll
    for (int gq = 0; gq < G; ++gq) {
      if (first || __any(tmax[gq] > THR)) {
        const float tgt = first ? (tmax[gq] == -INFINITY ? 0.f : m[gq] + tmax[gq]) : m[gq] + fmaxf(tmax[gq], 0.f);
        const float mn = Mfma<T>::round(tgt);
        const float delta = mn - m[gq];
        const float alpha = __builtin_amdgcn_exp2f(-delta);
#pragma unroll
        for (int c = 0; c < NSUB; ++c)
#pragma unroll
          for (int k = 0; k < 16; ++k) sacc[gq][c][k] -= delta;
        if (!first) {
#pragma unroll
          for (int i = 0; i < NDT; ++i)
#pragma unroll
            for (int k = 0; k < 16; ++k) oacc[gq][i][k] *= alpha;
        }
        m[gq] = mn;
        if (hh) qf[gq][PADS].x = (qf[gq][PADS].x & 0xFFFF0000u) | (Mfma<T>::pack2(-m[gq], 0.f) & 0xFFFFu);
      }
    }
    first = false;
#pragma unroll
    for (int c = 0; c < NSUB; ++c) {
      uint4 pb[G][2];
#pragma unroll
      for (int gq = 0; gq < G; ++gq)
#pragma unroll
        for (int s2 = 0; s2 < 2; ++s2) {
          float p[8];
#pragma unroll
          for (int j = 0; j < 8; ++j) p[j] = __builtin_amdgcn_exp2f(sacc[gq][c][8 * s2 + j]);
          pb[gq][s2] = make_uint4(Mfma<T>::pack2(p[0], p[1]), Mfma<T>::pack2(p[2], p[3]), Mfma<T>::pack2(p[4], p[5]),
                                  Mfma<T>::pack2(p[6], p[7]));
        }
#pragma unroll
      for (int dt = 0; dt < NDT; ++dt)
#pragma unroll
        for (int s2 = 0; s2 < 2; ++s2)
#pragma unroll
          for (int gq = 0; gq < G; ++gq) oacc[gq][dt] = Mfma<T>::m32x32x16(vpf[c][dt][s2], pb[gq][s2], oacc[gq][dt]);
    }
    if (j0 + KT < kend) stage((it + 1) & 1, j0 + KT);
    __syncthreads();
    if (j0 + 2 * KT < kend) load(j0 + 2 * KT);
  }

#pragma unroll
  for (int gq = 0; gq < G; ++gq) {
    constexpr int dts = D / 32, rho = D % 32, hs = (rho >> 2) & 1, reg = (rho & 3) + 4 * (rho >> 3);
    const float v = oacc[gq][dts][reg];
    const float o = xlane32(v);
    const float l = hh == hs ? v : o;
    const float inv = l > 0.f ? 1.f / l : 0.f;
    const int qrow = q0 + 32 * gq + r;
    if (qrow < a.Lq) {
      T* __restrict__ O = (T*)a.o + (long)b * a.so + (long)h * (a.hso ? a.hso : D) + (long)qrow * a.ldo;
#pragma unroll
      for (int dt = 0; dt < NDT; ++dt)
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          const int e = 32 * dt + 8 * k + 4 * hh;
          if (e >= D) continue;
          *(uint2*)(O + e) = make_uint2(Mfma<T>::pack2(oacc[gq][dt][4 * k] * inv, oacc[gq][dt][4 * k + 1] * inv),
                                        Mfma<T>::pack2(oacc[gq][dt][4 * k + 2] * inv, oacc[gq][dt][4 * k + 3] * inv));
        }
    }
  }
}

// ------------------------------------------------------------------------------------------------
// attnw: flash attention for wide heads (the VAE mid-block's single d = 512 head), bf16 / fp16, non-causal.
// Block = 4 waves x the same 32 queries; wave w owns d-quarter w.  Per 32-key tile:
//   partial S^T_w = K[:, d_w] Q[:, d_w]^T (D/64 k-steps of v_mfma_f32_32x32x16, K fragments straight from
//   global: every K element is read by exactly one wave of the block) -> LDS -> every wave sums the four
//   partials in the same order (identical S^T in all waves) -> online softmax in base 2 (scale * log2 e at the
//   Q load; fp32 running max / row sum) -> P^T as the B operand of O^T_w += V^T P^T over the wave's D/4
//   rows (V tile staged once per block in LDS, V^T fragments by ds_read_tr16_b64).  Scores never leave LDS.
template <typename T, int D, int QG>
__global__ __launch_bounds__(256, QG == 1 ? 2 : 1) void attnw_kernel(AttnArgs a) {
  // QG query groups of 32 per block; the 4 / QG waves of a group split d (DW each)
  constexpr int KT = 32, WPG = 4 / QG, DW = D / WPG, NSW = DW / 16, NDTW = DW / 32;
  constexpr int SV = (D % 128 == 32 || D % 128 == 96) ? D : D + 32;   // ds_read_tr rows conflict-free
  constexpr int VCH = D / 8;                                           // 16-byte chunks per V row
  static_assert(D % 128 == 0 && (KT * VCH) % 256 == 0, "attnw shape");
  __shared__ float Sx[4][64 * 16];
  __shared__ __attribute__((aligned(16))) uint16_t Vs[KT * SV];

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int r = lane & 31, hh = lane >> 5, g = lane >> 4;
  const int nq = (a.Lq + 32 * QG - 1) / (32 * QG);
  const int qb = blockIdx.x % nq, bh = blockIdx.x / nq;
  const int b = bh / a.H, h = bh - b * a.H;
  const int qg = wave / WPG, dw = wave - qg * WPG;
  const int qrow = (qb * QG + qg) * 32 + r;
  const T* __restrict__ Q = (const T*)a.q + (long)b * a.sq + (long)h * (a.hsq ? a.hsq : D);
  const T* __restrict__ K = (const T*)a.k + (long)b * a.sk + (long)h * (a.hsk ? a.hsk : D);
  const T* __restrict__ V = (const T*)a.v + (long)b * a.sv + (long)h * (a.hsv ? a.hsv : D);
  const int d0 = dw * DW;

  uint4 qf[NSW];
  const float sl2 = a.scale * 1.4426950408889634f;
#pragma unroll
  for (int s = 0; s < NSW; ++s) {
    uint4 v = make_uint4(0, 0, 0, 0);
    if (qrow < a.Lq) v = *(const uint4*)(Q + (long)qrow * a.ldq + d0 + 16 * s + 8 * hh);
    if (!a.q_scaled) {
      float f[8];
      Vec16<T>::unpack(v, f);
#pragma unroll
      for (int j = 0; j < 8; ++j) f[j] *= sl2;
      v = Vec16<T>::pack(f);
    }
    qf[s] = v;
  }
  f32x16 oacc[NDTW];
#pragma unroll
  for (int i = 0; i < NDTW; ++i)
#pragma unroll
    for (int k = 0; k < 16; ++k) oacc[i][k] = 0.f;
  float m = -INFINITY, lsum = 0.f;

  // K fragments (lane (r, hh) = key j0 + r, d0 + 16 s + 8 hh .. +7) and this thread's V-tile chunks are
  // register-prefetched one tile ahead, so their latency hides under the previous tile's softmax and PV MFMAs
  constexpr int NVU = KT * VCH / 256;
  uint4 kn[NSW], vn[NVU];
  auto fetch = [&](int j) {
    const int key = j + r;
#pragma unroll
    for (int s = 0; s < NSW; ++s)
      kn[s] = key < a.Lk ? *(const uint4*)(K + (long)key * a.ldk + d0 + 16 * s + 8 * hh) : make_uint4(0, 0, 0, 0);
#pragma unroll
    for (int u = 0; u < NVU; ++u) {
      const int idx = tid + 256 * u, row = idx / VCH, c = idx - row * VCH;
      const int kk = j + row;
      vn[u] = kk < a.Lk ? *(const uint4*)(V + (long)kk * a.ldv + c * 8) : make_uint4(0, 0, 0, 0);
    }
  };
  fetch(0);
  for (int j0 = 0; j0 < a.Lk; j0 += KT) {
    f32x16 sp;
#pragma unroll
    for (int k = 0; k < 16; ++k) sp[k] = 0.f;
#pragma unroll
    for (int s = 0; s < NSW; ++s) sp = Mfma<T>::m32x32x16(kn[s], qf[s], sp);
    __syncthreads();   // the previous tile's Sx / Vs reads are done
#pragma unroll
    for (int k = 0; k < 16; ++k) Sx[wave][k * 64 + lane] = sp[k];
#pragma unroll
    for (int u = 0; u < NVU; ++u) {
      const int idx = tid + 256 * u, row = idx / VCH, c = idx - row * VCH;
      *(uint4*)(Vs + row * SV + c * 8) = vn[u];
    }
    if (j0 + KT < a.Lk) fetch(j0 + KT);   // registers free again: the next tile's loads fly under this softmax / PV
    __syncthreads();
    f32x16 sacc;
#pragma unroll
    for (int k = 0; k < 16; ++k) {
      float v = Sx[qg * WPG][k * 64 + lane];
#pragma unroll
      for (int w = 1; w < WPG; ++w) v += Sx[qg * WPG + w][k * 64 + lane];
      const int kk = j0 + (k & 3) + 8 * (k >> 2) + 4 * hh;
      sacc[k] = kk < a.Lk ? v : -INFINITY;
    }
    float tmax = sacc[0];
#pragma unroll
    for (int k = 1; k < 16; ++k) tmax = fmaxf(tmax, sacc[k]);
    tmax = fmaxf(tmax, xlane32(tmax));
    const float mn = fmaxf(m, tmax);
    const float alpha = m == -INFINITY ? 0.f : __builtin_amdgcn_exp2f(m - mn);
    m = mn;
    lsum *= alpha;
#pragma unroll
    for (int i = 0; i < NDTW; ++i)
#pragma unroll
      for (int k = 0; k < 16; ++k) oacc[i][k] *= alpha;
    uint4 pb[2];
#pragma unroll
    for (int s2 = 0; s2 < 2; ++s2) {
      float p[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        p[j] = __builtin_amdgcn_exp2f(sacc[8 * s2 + j] - mn);
        lsum += p[j];
      }
      pb[s2] = make_uint4(Mfma<T>::pack2(p[0], p[1]), Mfma<T>::pack2(p[2], p[3]), Mfma<T>::pack2(p[4], p[5]),
                          Mfma<T>::pack2(p[6], p[7]));
    }
#pragma unroll
    for (int dt = 0; dt < NDTW; ++dt)
#pragma unroll
      for (int s2 = 0; s2 < 2; ++s2) {
        const int krow = 16 * s2 + 4 * (g >> 1) + ((lane & 15) >> 2);
        const int col = d0 + 32 * dt + 16 * (g & 1) + 4 * (lane & 3);
        const s16x4 t1 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(Vs + krow * SV + col));
        const s16x4 t2 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(Vs + (krow + 8) * SV + col));
        const uint4 vf = make_uint4(__builtin_bit_cast(uint2, t1).x, __builtin_bit_cast(uint2, t1).y,
                                    __builtin_bit_cast(uint2, t2).x, __builtin_bit_cast(uint2, t2).y);
        oacc[dt] = Mfma<T>::m32x32x16(vf, pb[s2], oacc[dt]);
      }
  }
  const float l = lsum + xlane32(lsum);
  const float inv = l > 0.f ? 1.f / l : 0.f;
  if (qrow >= a.Lq) return;
  T* __restrict__ O = (T*)a.o + (long)b * a.so + (long)h * (a.hso ? a.hso : D) + (long)qrow * a.ldo;
#pragma unroll
  for (int dt = 0; dt < NDTW; ++dt)
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const int e = d0 + 32 * dt + 8 * k + 4 * hh;
      *(uint2*)(O + e) = make_uint2(Mfma<T>::pack2(oacc[dt][4 * k] * inv, oacc[dt][4 * k + 1] * inv),
                                    Mfma<T>::pack2(oacc[dt][4 * k + 2] * inv, oacc[dt][4 * k + 3] * inv));
    }
}

// (QG = 2 query groups per block was measured slower — one wave per SIMD — and spills with the prefetch: only
//  QG = 1 is instantiated)
template <typename T>
void launchw(const AttnArgs& a, hipStream_t s) {
  dim3 grid(((a.Lq + 31) / 32) * a.H * a.B), block(256);
  ProfScope ps(prof_on() ? std::string("irx::(anonymous namespace)::attnw_kernel<") +
                               (std::is_same<T, f16_t>::value ? "_Float16" : "unsigned short") + ", 512, 1>"
                         : std::string(),
               4.0 * a.B * a.H * (double)a.Lq * a.Lk * a.d, s);
  attnw_kernel<T, 512, 1><<<grid, block, 0, s>>>(a);
  IRX_LAUNCH_CHECK();
}

template <typename T, int D, int KT, bool CAUSAL>
void launch3_cfg(const AttnArgs& a, hipStream_t s) {
  // query groups per block against resident K/V (cross-attention, Lk <= 2 KT): as many as keep >= 1024 blocks at
  // d = 40 (4 blocks / CU resident), >= 512 at the wider heads (kbench sweep with the one-round-trip prologue,
  // profiles/r06_kbench_attn_qrep.txt: d = 80 19.8 -> 17.0 us at 2 groups; d = 40 best at 4, d = 160 at 1)
  const bool res = !CAUSAL && a.Lk <= 2 * KT && g_attn_qrep;
  const long min_blocks = D <= 40 ? 1024 : 512;
  int qrep = 1;
  if (res && g_attn_qrep >= 2) qrep = std::min(g_attn_qrep, 32);   // (sweeps: a forced count)
  else if (res)
    while (qrep < 8 && ((a.Lq + 128 * 2 * qrep - 1) / (128 * 2 * qrep)) * a.H * a.B >= min_blocks) qrep *= 2;
  const int nq = (a.Lq + 128 * qrep - 1) / (128 * qrep);
  dim3 grid(nq * a.H * a.B), block(256);
  // which kernel runs: resident K/V (cross-attention), two query groups per wave (d = 40 self), the prefetching
  // attn3 (PF 3), or plain attn3; the profiler names the launch as rocprofv3 demangles it
  enum { kRes, kQ2, kPf, kPlain };
  int kind = kPlain;
  if (!CAUSAL && res) kind = kRes;
  else if (!CAUSAL && D == 40 && g_attn_q2) kind = kQ2;
  else if (!CAUSAL && D == 40 && g_attn_pf) kind = kPf;
  std::string nm;
  if (prof_on()) {
    const std::string tn = std::is_same<T, f16_t>::value ? "_Float16" : "unsigned short";
    nm = kind == kQ2 ? "irx::(anonymous namespace)::attn3q_kernel<" + tn + ", " + std::to_string(D) + ", " +
                           std::to_string(KT) + ">"
                     : "irx::(anonymous namespace)::attn3_kernel<" + tn + ", " + std::to_string(D) + ", " +
                           std::to_string(KT) + ", " + (CAUSAL ? "true" : "false") + ", " +
                           (kind == kRes ? "true" : "false") + ", " +
                           (kind == kPf ? "3"
                            : (D == 160 && g_attn_pf160 && kind != kQ2) ? "1"
                            : (D == 80 && kind == kPlain && g_attn_pf80 == 2) ? "2"
                                                                                                    : "0") + ">";
    if (g_prof_shapes)
      nm += " [B " + std::to_string(a.B) + " Lq " + std::to_string(a.Lq) + " Lk " + std::to_string(a.Lk) + "]";
  }
  ProfScope ps(nm, 4.0 * a.B * a.H * (double)a.Lq * a.Lk * a.d, s);
  AttnArgs b = a;
  b.xcd = g_attn_xcd;
  b.prio = g_attn_prio;
  b.qrep = qrep;
  if constexpr (!CAUSAL) {
    if constexpr (D == 160) {   // one wave per SIMD: the whole-tile fragment prefetch in the register file's other half
      if (g_attn_pf160 && kind != kQ2) {
        if (kind == kRes) attn3_kernel<T, D, KT, false, true, 1><<<grid, block, 0, s>>>(b);
        else attn3_kernel<T, D, KT, false, false, 1><<<grid, block, 0, s>>>(b);
        IRX_LAUNCH_CHECK();
        return;
      }
    }
    if constexpr (D == 80) {   // (option attn_pf80 = 2: the whole-tile fragment prefetch at 2 waves per SIMD)
      if (kind == kPlain && g_attn_pf80 == 2) {
        attn3_kernel<T, D, KT, false, false, 2><<<grid, block, 0, s>>>(b);   // (PF 3 spills)
        IRX_LAUNCH_CHECK();
        return;
      }
    }
    if (kind == kRes) {
      attn3_kernel<T, D, KT, false, true><<<grid, block, 0, s>>>(b);
      IRX_LAUNCH_CHECK();
      return;
    }
    if constexpr (D == 40) {
      if (kind == kQ2) {
        attn3q_kernel<T, D, KT><<<dim3(((a.Lq + 255) / 256) * a.H * a.B), block, 0, s>>>(b);
        IRX_LAUNCH_CHECK();
        return;
      }
      if (kind == kPf) {
        attn3_kernel<T, D, KT, false, false, 3><<<grid, block, 0, s>>>(b);
        IRX_LAUNCH_CHECK();
        return;
      }
    }
  }
  attn3_kernel<T, D, KT, CAUSAL, false><<<grid, block, 0, s>>>(b);
  IRX_LAUNCH_CHECK();
}

template <typename T, int D>
void launch3_d(const AttnArgs& a, hipStream_t s) {
  // (96-key single-pass tiles for Lk <= 96 spill at every d: 64-key tiles everywhere, Lk = 77 in two)
  if (a.causal) launch3_cfg<T, D, 64, true>(a, s);
  else launch3_cfg<T, D, 64, false>(a, s);
}

template <typename T>
bool launch3(const AttnArgs& a, hipStream_t s) {
  switch (a.d) {
    case 40: launch3_d<T, 40>(a, s); return true;
    case 64: launch3_d<T, 64>(a, s); return true;
    case 80: launch3_d<T, 80>(a, s); return true;
    case 160: launch3_d<T, 160>(a, s); return true;
    default: return false;
  }
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
  const bool v16 = a.d % 8 == 0 && (a.ldq % 8) == 0 && ((uintptr_t)a.q % 16) == 0 && ((uintptr_t)a.o % 8) == 0 &&
                   (a.ldo % 4) == 0;
  if (a.d == 512 && a.dtype != F32) {
    IRX_CHECK(!a.causal && v16 && (a.ldk % 8) == 0 && (a.ldv % 8) == 0, "d = 512 attention: 16-byte rows, non-causal");
    if (a.dtype == F16) launchw<f16_t>(a, s);
    else launchw<bf16_t>(a, s);
    return;
  }
  if (a.dtype == F32) launch_t<float>(a, s);
  else if (a.dtype == F16) {
    IRX_CHECK(v16 && launch3<f16_t>(a, s), "fp16 attention: head dim must be 40 / 64 / 80 / 160 with 16-byte rows");
  } else if (!(v16 && launch3<bf16_t>(a, s))) {
    launch_t<bf16_t>(a, s);
  }
}
int g_attn_q2 = 1;      // irx_set_option("attn_q2", 0): d = 40 self-attention with one query group per wave (attn3, A/B)
int g_attn_pf = 1;      // irx_set_option("attn_pf", 0): d = 40 self-attention without the whole-tile fragment prefetch (A/B)
int g_attn_pf160 = 1;   // irx_set_option("attn_pf160", 0): d = 160 without the fragment prefetch (A/B)
int g_attn_pf80 = 2;    // irx_set_option("attn_pf80", 0): d = 80 self-attention without the whole-tile fragment prefetch
                        // (A/B; 2 = at 2 waves / SIMD: L = 1024 67.2 -> 61.1 us, profiles/r06_kbench_attn_init.txt)
int g_attn_xcd = 1;
int g_attn_prio = 0;    // irx_set_option("attn_prio", 1): MFMA chains of attn3 at raised wave priority (A/B)
int g_attn_qrep = 1;    // irx_set_option("attn_qrep", 0): one query group per block in cross-attention (A/B); >= 2: that many (sweeps)
int g_attn_hm = 1;

}  // namespace irx
