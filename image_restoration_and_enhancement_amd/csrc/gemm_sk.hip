// irx — streaming GEMM for the K = 320 projections of the UNet's 64x64-latent transformers, gfx950.
//
// Shapes (batch 16 at 512x512: M = 65536 pixels, K = 320 channels): proj_in, to_q, the fused q|k|v (N = 960,
// head-split stores), both to_out (+ residual) and the GEGLU feed-forward projection (N = 2560 -> 1280).  At
// K = 320 a tile's whole K fits one LDS stage and the weights are tiny, so these calls are HBM streams (A in,
// C out): 84-126 MB for 13 GFLOP at N = 320.  The large-tile kernel (gemm2.hip) re-stages its B panel with
// every 64-deep K step, keeps one K step in flight and pays a pipeline fill per 128-256-row tile, and reaches
// 2-3 TB/s on them.  This kernel instead:
//   * keeps the block's whole B slice (320 weight rows x K = 320: 80 columns x 10 K steps per wave) in VGPRs
//     for the life of the block — B is read once per block, never staged;
//   * streams A through a 3-stage LDS ring of whole 64-row x 320 tiles by LDS-DMA (40 KiB per stage, two tiles
//     in flight behind the one being multiplied), persistent over the block's tiles;
//   * multiplies with swapped operands, D^T = B_slice A^T (v_mfma_f32_16x16x32, B fragment as the first
//     operand), so each lane ends up owning 4 consecutive output channels of one pixel: the epilogue (bias /
//     folded LayerNorm, residual prefetched one tile ahead, output scale, GEGLU, head-split q|k|v layout) is
//     lane-local and stores 8-byte row pieces straight from registers — no LDS staging, no barrier;
//   * places blocks so that the slices of one N (q|k|v: 3, GEGLU: 10) walk the same row tiles on one XCD at
//     the same time: A is fetched from HBM once and served to the other slices from that XCD's L2.
// Arithmetic per output: one fp32 MFMA accumulation chain over k = 0..319 in 32-deep steps, the epilogue of
// the large-tile kernel (alpha / bias or the LayerNorm fold, rounding to the storage type, then residual and
// out_scale, rounding again; GEGLU h * gelu(g) on the rounded halves) — independent of M, the batch and the
// tile placement, so the engines stay batch invariant.
#include <algorithm>

#include "ops.h"
#include "profile.h"

// timing diagnostics only (a separately built library, scripts/build_skdbg.sh): 1 no epilogue / stores, 2 no MFMAs,
// 4 no A DMA — results are wrong when set
#ifndef IRX_SK_DBG
#define IRX_SK_DBG 0
#endif

namespace irx {

// irx_set_option("gemm_sk", m): 1 (default) the GEGLU projection only, 3 every K = 320 shape, 2 GEGLU on the one-wave-
// per-SIMD form, 0 none.  Measured (profiles/r03_kprof_sk_n.txt, M = 65536): GEGLU 179 vs 214 us on the large-tile
// kernel; the N = 320 / 960 projections 32 / 37 / 74 vs 27 / 34 / 66 us — one wave per SIMD with the B slice in
// registers leaves the MFMA pipe 14 % busy behind AGPR -> VGPR operand copies and the epilogue's VALU work
// (profiles/r03_pmc_sk_*.txt), so those stay on the large-tile kernel
int g_gemm_sk = 1;
int g_gemm_sk_blocks = 0;   // irx_set_option("gemm_sk_blocks", n): persistent blocks per XCD (0: 32 x blocks per CU)

namespace {

typedef __attribute__((address_space(3))) void lds_void;

__device__ __forceinline__ void glds16(const void* g, uint32_t lds_addr) {
  asm volatile("s_mov_b32 m0, %1\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %0, off" ::"v"(g), "s"(lds_addr)
               : "memory", "m0");
}

// wait until at most n of this wave's vector-memory operations are outstanding (n: block-uniform, from the set
// the schedule below produces)
__device__ __forceinline__ void vm_wait(int n) {
  switch (n) {
#define IRX_VM(k) case k: asm volatile("s_waitcnt vmcnt(" #k ")" ::: "memory"); break;
    IRX_VM(1) IRX_VM(2) IRX_VM(3) IRX_VM(4) IRX_VM(5) IRX_VM(6) IRX_VM(7) IRX_VM(8) IRX_VM(9) IRX_VM(10) IRX_VM(11)
    IRX_VM(12) IRX_VM(13) IRX_VM(14) IRX_VM(15) IRX_VM(16) IRX_VM(17) IRX_VM(18) IRX_VM(19) IRX_VM(20) IRX_VM(21)
    IRX_VM(22) IRX_VM(23) IRX_VM(24) IRX_VM(25) IRX_VM(26) IRX_VM(27) IRX_VM(28) IRX_VM(29) IRX_VM(30) IRX_VM(31)
    IRX_VM(32) IRX_VM(33) IRX_VM(34) IRX_VM(35) IRX_VM(36) IRX_VM(37) IRX_VM(38) IRX_VM(39) IRX_VM(40) IRX_VM(41)
    IRX_VM(42) IRX_VM(43) IRX_VM(44) IRX_VM(45) IRX_VM(46) IRX_VM(47) IRX_VM(48) IRX_VM(49) IRX_VM(50) IRX_VM(51)
    IRX_VM(52) IRX_VM(53) IRX_VM(54) IRX_VM(55) IRX_VM(56) IRX_VM(57) IRX_VM(58) IRX_VM(59) IRX_VM(60) IRX_VM(61)
    IRX_VM(62) IRX_VM(63)
#undef IRX_VM
    default: asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); break;
  }
}

template <typename T> struct Pk;
template <> struct Pk<bf16_t> {
  __device__ static void unpack4(const uint2& u, float* f) {
    f[0] = __uint_as_float(u.x << 16); f[1] = __uint_as_float(u.x & 0xffff0000u);
    f[2] = __uint_as_float(u.y << 16); f[3] = __uint_as_float(u.y & 0xffff0000u);
  }
};
template <> struct Pk<f16_t> {
  __device__ static void unpack4(const uint2& u, float* f) {
    const f16x4 h = __builtin_bit_cast(f16x4, u);
    f[0] = (float)h[0]; f[1] = (float)h[1]; f[2] = (float)h[2]; f[3] = (float)h[3];
  }
};

constexpr int kSkK = 320;          // the one K this kernel takes
constexpr int kSkKS = kSkK / 32;   // 32-deep MFMA K steps
constexpr int kSkRC = kSkK / 8;    // 16-byte chunks per A row

// NB: 16-row B blocks per wave (4 waves): 5 -> 320-column slices; GEGLU: 4 (2 value + 2 gate blocks) -> 256 weight
// rows = 128 output channels per slice.  MB: 16-row blocks per tile (BM = 16 MB rows); BPC: resident blocks per CU
// (2: two waves per SIMD, the registers of one wave <= 256); RES: residual add (a double-buffered LDS copy of the
// tile's residual rows, DMA'd one tile ahead); S: A ring stages; AF2: A fragments of the next K step requested before
// the current step's MFMAs.  groups: row groups per XCD (blocks of one group share row tiles).
//
// Every global -> LDS transfer is LDS-DMA issued from inline asm and every wait on it an explicit, exactly counted
// vmcnt (the loop issues no compiler-visible load, so the compiler adds no wait of its own that would also drain the
// DMA in flight).  Rows past M in the last tile are bound to a valid tile row (`spare`: r & 1, or row 0 when the tile
// has a single valid row): they re-read that row's A, residual and LayerNorm statistics, and their store rewrites that
// row with identical bytes — every DMA and store is issued by every wave, so the counts hold for ragged M too (M even
// when the statistics are read: they travel as row pairs; the host checks it).
template <typename T, int NB, bool GEGLU, int MB, int BPC, bool RES, int S, bool AF2>
__global__ __launch_bounds__(256, BPC) void gemm_sk_kernel(GemmArgs a, int n_slices, int groups) {
  constexpr int BM = 16 * MB, KS = kSkKS, RC = kSkRC;
  constexpr int STAGE = BM * RC;           // uint4 per ring stage (40 KiB at 64 rows)
  constexpr int PPW = STAGE / 64 / 4;      // LDS-DMA pieces (1 KiB wave-instructions) per wave per stage
  static_assert(PPW * 256 == STAGE, "whole pieces per wave");
  constexpr int NS = 4 * NB * 16;          // weight rows per block
  static_assert(!GEGLU || NB == 4, "GEGLU: 2 value + 2 gate blocks per wave");
  static_assert(!(RES && GEGLU), "no residual on the GEGLU projection");
  constexpr int OC = GEGLU ? 32 : NB * 16; // output columns per wave
  constexpr int CH = OC / 8;               // 16-byte chunks per output row piece
  constexpr int SRU = CH + 1;              // staging row stride (uint4): 44 / 20 dwords, conflict-free 8-byte writes
  constexpr int NR = MB / 2;               // 32-row epilogue rounds per tile
  constexpr int NCK = 32 * CH / 64;        // 16-byte chunks per lane per round
  static_assert(MB % 2 == 0 && (32 * CH) % 64 == 0, "32-row rounds, whole chunks per lane");
  constexpr int RESN = RES ? NR * NCK : 0; // residual DMA pieces per wave per tile
  constexpr int LNL = BM / 8;              // lanes per wave carrying the tile's LayerNorm statistics (16 B = 2 rows)
  constexpr int SN = NR * NCK;             // epilogue stores per wave per tile
  __shared__ __attribute__((aligned(16))) uint4 ring[S * STAGE];
  __shared__ __attribute__((aligned(16))) float2 lnring[S * BM];
  __shared__ __attribute__((aligned(16))) uint4 resbuf[RES ? 2 * 4 * BM * CH : 1];
  __shared__ __attribute__((aligned(16))) float sbias[NS];
  __shared__ __attribute__((aligned(16))) float su[NS];
  __shared__ __attribute__((aligned(16))) uint4 stage_buf[4 * 32 * SRU];
  __shared__ long noff_tab[4 * CH];

  const int tid = threadIdx.x, lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  // tile row r, or the valid row that stands in for it when r is past M (rem >= 1 valid rows in the tile)
  auto spare = [](int r, int rem) { return r < rem ? r : (rem > 1 ? (r & 1) : 0); };
  const int x = blockIdx.x & 7, loc = blockIdx.x >> 3;
  const int sl = loc % n_slices, grp = loc / n_slices;
  if (grp >= groups) return;
  const int tiles = (a.M + BM - 1) / BM;
  const int lo = (int)((long)x * tiles / 8), hi = (int)((long)(x + 1) * tiles / 8);
  const int t0 = lo + grp;
  if (t0 >= hi) return;
  const int nt = (hi - t0 + groups - 1) / groups;   // tiles of this block: t0, t0 + groups, ...
  const bool has_ln = !RES && (a.ln_rs != nullptr || a.ln_part != nullptr);
  const float2* const lnsrc = a.ln_part ? a.ln_part : a.ln_rs;   // (ln_T == 1: one float2 per row either way)
  const int PA = PPW + (has_ln ? 1 : 0);            // A-tile DMA pieces per wave (+ the statistics piece)

  // weight row (index into B / bias / ln_u) of slice-local row idx
  auto wrow = [&](int idx) -> int {
    if constexpr (!GEGLU) {
      return sl * NS + idx;
    } else {
      const int wv = idx / (NB * 16), j = (idx / 16) % NB, q = idx & 15;
      const int o = sl * 128 + wv * 32 + (j & 1) * 16 + q;    // output channel
      return (o >> 6) * 128 + (j >= 2 ? 64 : 0) + (o & 63);   // GEGLU64 interleave: (64 value, 64 gate) pairs
    }
  };
  for (int i = tid; i < NS; i += 256) {
    const int n = wrow(i);
    sbias[i] = a.bias ? a.bias[n] : 0.f;
    su[i] = a.ln_u ? a.ln_u[n] : 0.f;
  }
  const int n0w = GEGLU ? sl * 128 + w * 32 : sl * NS + w * OC;   // first output column of this wave
  long* const ncol = noff_tab + w * CH;   // output-column part of a chunk's address (head-split q|k|v: part/head/e)
  if (lane < CH) {
    const int n = n0w + lane * 8;
    long o = n;
    if (a.hs_L) {
      const int part = n / a.hs_C, rm = n - part * a.hs_C, hd = rm / a.hs_d, e = rm - hd * a.hs_d;
      o = (long)part * a.M * a.hs_C + (long)hd * a.hs_L * a.hs_d + e;
    }
    ncol[lane] = o;
  }

  // ---- B slice in registers: bfr[j][kk] = rows (w*NB + j)*16 + (lane & 15), k chunk kk*4 + (lane >> 4)
  uint4 bfr[NB][KS];
#pragma unroll
  for (int j = 0; j < NB; ++j) {
    const int n = wrow((w * NB + j) * 16 + (lane & 15));
    const uint16_t* p = (const uint16_t*)a.B + (long)n * a.ldb + (lane >> 4) * 8;
#pragma unroll
    for (int kk = 0; kk < KS; ++kk) bfr[j][kk] = *(const uint4*)(p + kk * 32);
  }
  // a wait the compiler sees (it then knows bfr has landed and puts no wait for it inside the loop)
  __builtin_amdgcn_s_waitcnt(0x0F70);   // vmcnt(0)

  auto tile_of = [&](int it) { return t0 + min(it, nt - 1) * groups; };   // (clamped: surplus issues re-read)
  auto lds32 = [](const void* p) { return __builtin_amdgcn_readfirstlane((uint32_t)(uintptr_t)(lds_void*)p); };
  // ---- A tile #it -> ring stage it % S: piece j of wave w covers ring chunks p = (w*PPW + j)*64 + lane (tile row
  //      p / RC, physical chunk p % RC holding logical chunk (p % RC) ^ (row & 7): conflict-free b128 fragment reads);
  //      with the LayerNorm fold, one more piece: LNL lanes x 16 B of the row statistics
  const uint16_t* Ag = (const uint16_t*)a.A;
  auto issueA = [&](int it) {
    const long m0 = (long)tile_of(it) * BM;
    const int rem = a.M - (int)m0;
    const uint16_t* base = Ag + m0 * a.lda;
    uint4* st = ring + (it % S) * STAGE + w * PPW * 64;
#pragma unroll
    for (int j = 0; j < PPW; ++j) {
      const int p = (w * PPW + j) * 64 + lane;
      const int r = p / RC, c = (p % RC) ^ (r & 7);
      glds16(base + spare(r, rem) * a.lda + c * 8, lds32(st + j * 64));
    }
    if (has_ln) {
      if (lane < LNL) {
        const int r = 2 * (w * LNL + lane);   // rows r, r + 1 (M even: both valid or both past M)
        glds16(lnsrc + m0 + (r < rem ? r : 0), lds32(lnring + (it % S) * BM + 2 * w * LNL));
      }
    }
  };
  // ---- residual rows of tile #it -> resbuf[it & 1] (the wave's OC columns; linear chunk p = lane + 64k <-> row p / CH,
  //      chunk p % CH, the order phase 2 reads them in)
  auto issueR = [&](int it) {
    if constexpr (RES) {
      const long m0 = (long)tile_of(it) * BM;
      const int rem = a.M - (int)m0;
      const uint16_t* R = (const uint16_t*)a.residual + m0 * a.ldr + n0w;
      uint4* dst = resbuf + ((it & 1) * 4 + w) * BM * CH;
#pragma unroll
      for (int k = 0; k < RESN; ++k) {
        const int p = lane + 64 * k, r = p / CH, c = p % CH;
        glds16(R + spare(r, rem) * a.ldr + c * 8, lds32(dst + 64 * k));
      }
    }
  };

  // ---- epilogue.  Phase 1 (per 32-row round): each lane turns its accumulators (4 consecutive channels of one pixel
  //      per 16x16 block) into storage-type values — alpha / bias or the LayerNorm fold, rounded; GEGLU h * gelu(g) —
  //      and writes them as 8-byte pieces into the wave's private staging rows.  Phase 2: the wave reads the rows back
  //      as 16-byte chunks (lane -> consecutive chunks of consecutive rows), adds the residual chunk, applies
  //      out_scale and stores whole 16-byte row pieces (the large-tile kernel's two-pass arithmetic).  A wave's staging
  //      rows are its own: no barrier.
  uint4* const stg = stage_buf + w * 32 * SRU;
  const int q4 = (lane >> 4) * 4;
  auto crow = [&](int k) { return (lane + 64 * k) / CH; };
  auto cch = [&](int k) { return (lane + 64 * k) % CH; };
  const long rstride = a.hs_L ? a.hs_d : a.ldc;

  // fragment read addressing: row (lane & 15) of each 16-row block, logical chunk kk*4 + (lane >> 4), stored at
  // chunk ^ (row & 7) = 8 * (kk >> 1) + 4 * ((kk & 1) ^ hb) + lo
  const int sw = lane & 7, hb = sw >> 2, lo4 = (lane >> 4) ^ (sw & 3);
  const int fb0 = (lane & 15) * RC + 4 * hb + lo4, fb1 = (lane & 15) * RC + 4 * (hb ^ 1) + lo4;

  // issue order: A(0 .. S-2), R(0); per iteration j: R(j + 1), A(j + S - 1), stores(j) — all unconditional
#pragma unroll
  for (int p = 0; p < S - 1; ++p)
    if constexpr (!(IRX_SK_DBG & 4)) issueA(p);
  issueR(0);
  for (int it = 0; it < nt; ++it) {
    // A(it) landed: younger are, it <= S-2: (S-2-it) A + R(0) + it (R + A + stores); else stores(it-S+1) + (S-2)
    // (R + A + stores) (capped at the counter's 63: waiting for a little more is safe)
    if constexpr (!(IRX_SK_DBG & 4))
      vm_wait(min(63, it <= S - 2 ? (S - 2 - it) * PA + RESN + it * (RESN + PA + SN)
                                  : SN + (S - 2) * (RESN + PA + SN)));
    // every wave's pieces of tile it landed; stage (it + S - 1) % S and resbuf[(it + 1) & 1] free (lgkmcnt: the
    // bias / column tables before the first use)
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
    issueR(it + 1);
    if constexpr (!(IRX_SK_DBG & 4)) issueA(it + S - 1);
    const uint4* As = ring + (it % S) * STAGE;
    f32x4 acc[NB][MB];
#pragma unroll
    for (int j = 0; j < NB; ++j)
#pragma unroll
      for (int i = 0; i < MB; ++i) acc[j][i] = f32x4{0.f, 0.f, 0.f, 0.f};
    if constexpr (!(IRX_SK_DBG & 2)) {
      constexpr int NAF = AF2 ? 2 : 1;
      uint4 af[NAF][MB];
      auto rdA = [&](int kk, uint4* f) {
        const int fb = (kk & 1) ? fb1 : fb0;
#pragma unroll
        for (int i = 0; i < MB; ++i) f[i] = As[fb + 8 * (kk >> 1) + i * 16 * RC];
      };
      if constexpr (AF2) rdA(0, af[0]);
#pragma unroll
      for (int kk = 0; kk < KS; ++kk) {
        if constexpr (AF2) {
          if (kk + 1 < KS) rdA(kk + 1, af[(kk + 1) & 1]);
        } else {
          rdA(kk, af[0]);
        }
        __builtin_amdgcn_s_setprio(1);
#pragma unroll
        for (int j = 0; j < NB; ++j)
#pragma unroll
          for (int i = 0; i < MB; ++i) acc[j][i] = Mfma<T>::m16x16x32(bfr[j][kk], af[AF2 ? (kk & 1) : 0][i], acc[j][i]);
        __builtin_amdgcn_s_setprio(0);
      }
    }
    if constexpr ((IRX_SK_DBG & 1) != 0) {   // diagnostics: keep the accumulators live, skip the epilogue
      float t = 0.f;
#pragma unroll
      for (int j = 0; j < NB; ++j)
#pragma unroll
        for (int i = 0; i < MB; ++i) t += acc[j][i][0] + acc[j][i][3];
      if (t == 12345.678f) ((float*)a.C)[lane] = t;
      continue;
    }

    // ---- epilogue
    // R(it) landed (the statistics came with A(it)): younger are R(it + 1) + A(it + S - 1), and for it >= 1 also
    // A(it + S - 2) + stores(it - 1)
    if constexpr (RES) vm_wait(min(63, it == 0 ? RESN + PA : 2 * PA + SN + RESN));
    const long tm0 = (long)tile_of(it) * BM;
    const int rem = a.M - (int)tm0;
    long mbase = tm0 * a.ldc;                  // element offset of the tile's first output row
    if (a.hs_L) {                              // (hs_L % BM == 0: a tile lies in one image)
      const long img = tm0 / a.hs_L;
      mbase = img * a.hs_C * a.hs_L + (tm0 - img * a.hs_L) * a.hs_d;
    }
    const float2* lst = lnring + (it % S) * BM;
    const uint4* rsb = resbuf + ((it & 1) * 4 + w) * BM * CH;
    T* Cp = (T*)a.C;
#pragma unroll
    for (int rr = 0; rr < NR; ++rr) {
      // phase 1
#pragma unroll
      for (int ih = 0; ih < 2; ++ih) {
        const int i = 2 * rr + ih;
        float2 rs = has_ln ? lst[i * 16 + (lane & 15)] : make_float2(1.f, 0.f);
        if (a.ln_part) rs = ln_fin(rs.x, rs.y, 1, a.ln_eps);   // producer partial (mean, M2): ln_rs_at's arithmetic
        float v[NB][4];
#pragma unroll
        for (int j = 0; j < NB; ++j) {
          const float4 bb = *(const float4*)(sbias + (w * NB + j) * 16 + q4);
          const float bj[4] = {bb.x, bb.y, bb.z, bb.w};
          if (has_ln) {
            const float4 uu = *(const float4*)(su + (w * NB + j) * 16 + q4);
            const float uj[4] = {uu.x, uu.y, uu.z, uu.w};
#pragma unroll
            for (int r = 0; r < 4; ++r) v[j][r] = Mfma<T>::round(fmaf(acc[j][i][r], rs.x, fmaf(-rs.y, uj[r], bj[r])));
          } else {
#pragma unroll
            for (int r = 0; r < 4; ++r) v[j][r] = Mfma<T>::round(acc[j][i][r] * a.alpha + bj[r]);
          }
        }
        uint2* srow = (uint2*)(stg + (ih * 16 + (lane & 15)) * SRU) + (lane >> 4);
        if constexpr (GEGLU) {
#pragma unroll
          for (int jj = 0; jj < 2; ++jj) {
            float o[4];
#pragma unroll
            for (int r = 0; r < 4; ++r) o[r] = v[jj][r] * gelu_erf16(v[jj + 2][r]);
            srow[jj * 4] = make_uint2(Mfma<T>::pack2(o[0], o[1]), Mfma<T>::pack2(o[2], o[3]));
          }
        } else {
#pragma unroll
          for (int j = 0; j < NB; ++j)
            srow[j * 4] = make_uint2(Mfma<T>::pack2(v[j][0], v[j][1]), Mfma<T>::pack2(v[j][2], v[j][3]));
        }
      }
      // phase 2
#pragma unroll
      for (int k = 0; k < NCK; ++k) {
        uint4 u = stg[crow(k) * SRU + cch(k)];
        if constexpr (!GEGLU) {
          if (RES || a.out_scale != 1.f) {
            float f[8];
            Vec16<T>::unpack(u, f);
            if constexpr (RES) {
              float rv[8];
              Vec16<T>::unpack(rsb[rr * 32 * CH + lane + 64 * k], rv);
#pragma unroll
              for (int e = 0; e < 8; ++e) f[e] += rv[e];
            }
#pragma unroll
            for (int e = 0; e < 8; ++e) f[e] *= a.out_scale;
            u = Vec16<T>::pack(f);
          }
        }
        const int row = rr * 32 + crow(k);
        const int srow2 = spare(row, rem);               // rows past M rewrite their stand-in row with its own bytes
        *(uint4*)(Cp + mbase + srow2 * rstride + ncol[cch(k)]) = u;
      }
    }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // surplus DMA pieces land before the block's LDS is released
}

template <typename T, int NB, bool GEGLU, int MB, int BPC, bool RES, int S, bool AF2>
void launch_sk(const GemmArgs& a, hipStream_t s) {
  constexpr int NS = 4 * NB * 16;
  const int n_slices = GEGLU ? (a.N / 2) / 128 : a.N / NS;
  const int per_xcd = std::max(n_slices, g_gemm_sk_blocks > 0 ? g_gemm_sk_blocks : 32 * BPC);
  const int groups = per_xcd / n_slices;
  const char* tn = std::is_same<T, f16_t>::value ? "_Float16" : "unsigned short";
  std::string nm;
  if (prof_on())
    nm = std::string("irx::(anonymous namespace)::gemm_sk_kernel<") + tn + ", " + std::to_string(NB) + ", " +
         (GEGLU ? "true" : "false") + ", " + std::to_string(MB) + ", " + std::to_string(BPC) + ", " +
         (RES ? "true" : "false") + ", " + std::to_string(S) + ", " + (AF2 ? "true" : "false") + ">";
  if (prof_on() && g_prof_shapes)
    nm += " [M " + std::to_string(a.M) + " N " + std::to_string(a.N) + " K " + std::to_string(a.K) + "]";
  ProfScope ps(nm, 2.0 * a.M * a.N * (double)a.K, s);
  gemm_sk_kernel<T, NB, GEGLU, MB, BPC, RES, S, AF2><<<8 * per_xcd, 256, 0, s>>>(a, n_slices, groups);
  IRX_LAUNCH_CHECK();
}

}  // namespace

// The K = 320 streaming path: dense, 16-bit, one batch, no conv / split / activation / row add / GroupNorm
// partials; N a multiple of the 320-column slice (GEGLU: of 256 interleaved weight rows); 16-byte aligned rows.
// The decision depends only on the per-call shape (not on M), so it is the same for every batch size.
bool gemm_sk_eligible(const GemmArgs& a) {
  if (!g_gemm_sk || (!a.geglu && g_gemm_sk != 3) || !is16(a.dtype) || a.conv || a.out_f32 || a.batch != 1 || a.K != kSkK) return false;
  if (a.act != ACT_NONE || a.rowadd || a.gn_part || a.gn_ab || a.b_rows || a.ln_out) return false;
  if (a.A1 || a.up2_w) return false;   // (one A source of K columns; plain row-major output)
  if (a.geglu ? (a.N % 256 != 0 || a.N / 2 / 128 > 32 || a.residual || a.hs_L || a.ldc % 4) : (a.N % 320 || a.N / 320 > 32))
    return false;
  if (a.lda % 8 || a.ldb % 8 || ((uintptr_t)a.A % 16) || ((uintptr_t)a.B % 16)) return false;
  if (((uintptr_t)a.C % 8) || (a.hs_L ? (a.hs_d % 4 || a.hs_C % 4) : a.ldc % 4)) return false;
  if (a.residual && (a.ldr % 4 || ((uintptr_t)a.residual % 8))) return false;
  if (a.hs_L && (a.residual || a.hs_L % 64)) return false;   // (a 64-row tile lies in one image)
  if ((a.ln_rs || a.ln_part) && (a.alpha != 1.f || a.M % 2)) return false;   // (statistics DMA'd as row pairs)
  if (a.ln_part && a.ln_T != 1) return false;   // (one producer partial per row: the K = 320 row)
  return a.M > 0;
}

bool gemm_sk(const GemmArgs& a0, hipStream_t s) {
  if (!gemm_sk_eligible(a0)) return false;
  const GemmArgs& a = a0;
  const bool f16 = a.dtype == F16;
  if (a.geglu) {
    if (g_gemm_sk == 2) {   // one wave per SIMD, 64-row tiles
      if (f16) launch_sk<f16_t, 4, true, 4, 1, false, 3, true>(a, s);
      else launch_sk<bf16_t, 4, true, 4, 1, false, 3, true>(a, s);
    } else {                // two waves per SIMD (the GELU epilogue's VALU work beside the other wave's MFMAs)
      if (f16) launch_sk<f16_t, 4, true, 2, 2, false, 3, false>(a, s);
      else launch_sk<bf16_t, 4, true, 2, 2, false, 3, false>(a, s);
    }
  } else if (a.residual) {  // 32-row tiles, a 4-deep A ring beside the double-buffered residual rows
    if (f16) launch_sk<f16_t, 5, false, 2, 1, true, 4, true>(a, s);
    else launch_sk<bf16_t, 5, false, 2, 1, true, 4, true>(a, s);
  } else {
    if (f16) launch_sk<f16_t, 5, false, 4, 1, false, 3, true>(a, s);
    else launch_sk<bf16_t, 5, false, 4, 1, false, 3, true>(a, s);
  }
  return true;
}

}  // namespace irx
