// irx — MFMA GEMM / implicit-GEMM convolution for gfx950.
//
// One kernel template serves every contraction of the SD-1.5 hot path:
//   * 3x3 convs (ResnetBlock2D conv1/conv2, conv_in/out, Down/Upsample2D) as implicit GEMM
//     (M = N*Ho*Wo pixels, N = Cout, K = KH*KW*Cin) with the im2col gather done while staging
//     A tiles, including zero padding, stride 2, asymmetric VAE padding, fused nearest upsample
//     (Upsample2D) and the up-block skip concat (two NHWC sources);
//   * 1x1 convs / Linear layers (proj_in/out, q/k/v/out, GEGLU proj, FF out, shortcuts, time MLP);
//   * batched GEMMs (VAE mid-block attention scores / PV).
// bf16 path: v_mfma_f32_16x16x32_bf16, fp32 accumulate.  fp32 path (parity mode): exact-f32
// v_mfma_f32_16x16x4_f32.  Tiles are staged global -> VGPR -> LDS (double buffered, one barrier
// per K step, next tile's loads in flight under the current tile's MFMAs) with a bank-spreading
// XOR swizzle; block -> tile mapping is XCD-aware.
#include "ops.h"
#include "profile.h"

namespace irx {

namespace {

constexpr int kThreads = 256;

struct RowInfo {   // per staged A row (conv mode)
  int n;           // image index, -1 if the row is past M
  int iy0, ix0;    // top-left input coordinate of the receptive field
};

template <typename T, int WM, int WN, int TM, int TN, bool CONV, bool OUTF32, bool HS = false>
__global__ __launch_bounds__(kThreads, 2) void gemm_kernel(GemmArgs a) {
  constexpr int VEC = 16 / (int)sizeof(T);      // elements per 16-byte chunk
  constexpr int BK = 8 * VEC;                   // 128-byte K step per row
  constexpr int BM = WM * TM * 16;
  constexpr int BN = WN * TN * 16;
  constexpr int AR = (BM * 8 + kThreads - 1) / kThreads;   // A chunks per thread
  constexpr int BR = (BN * 8 + kThreads - 1) / kThreads;
  static_assert(WM * WN == 4, "4 waves");
  __shared__ uint4 smem[2][(BM + BN) * 8];

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = tid >> 6;
  const int wm = wave / WN, wn = wave % WN;

  const int tiles_n = (a.N + BN - 1) / BN;
  const int tiles_m = (a.M + BM - 1) / BM;
  const int nwg = tiles_m * tiles_n;
  const int bid = xcd_remap(blockIdx.x, nwg);
  const int tile_n = bid % tiles_n, tile_m = bid / tiles_n;
  const int m0 = tile_m * BM, n0 = tile_n * BN;
  const int z = blockIdx.y;

  const T* __restrict__ Bp = (const T*)a.B + (long)z * a.sB;
  const T* __restrict__ Ap = CONV ? nullptr : (const T*)a.A + (long)z * a.sA;

  const int cc = tid & 7;             // this thread's chunk column within the 128-byte K step
  const int rbase = tid >> 3;         // first row this thread stages (then +32 per step)

  // ---- conv bookkeeping
  RowInfo ri[AR];
  int kc = 0, ky = 0, kx = 0;   // (channel, tap) of this thread's chunk in the current K tile
  const int Cin = a.g.C0 + a.g.C1;
  const bool resized = CONV && (a.g.Hv != a.g.Hin || a.g.Wv != a.g.Win);
  const float sy = resized ? (float)a.g.Hin / (float)a.g.Hv : 1.f;
  const float sx = resized ? (float)a.g.Win / (float)a.g.Wv : 1.f;
  if constexpr (CONV) {
    const int HWo = a.g.Ho * a.g.Wo;
#pragma unroll
    for (int i = 0; i < AR; ++i) {
      const int r = rbase + 32 * i;
      const int m = m0 + r;
      if (r < BM && m < a.M) {
        const int n = m / HWo;
        const int rem = m - n * HWo;
        const int oy = rem / a.g.Wo;
        const int ox = rem - oy * a.g.Wo;
        ri[i].n = n;
        ri[i].iy0 = oy * a.g.stride - a.g.pad_t;
        ri[i].ix0 = ox * a.g.stride - a.g.pad_l;
      } else {
        ri[i].n = -1; ri[i].iy0 = 0; ri[i].ix0 = 0;
      }
    }
    // position of chunk cc of K tile 0
    int k = cc * VEC;
    int tap = k / Cin;
    kc = k - tap * Cin;
    ky = tap / a.g.KW;
    kx = tap - ky * a.g.KW;
  }

  uint4 ra[AR], rb[BR];

  auto load_tiles = [&](int kt) {
    const int k = kt * BK + cc * VEC;
    const bool kvalid = k < a.K;
    // A
#pragma unroll
    for (int i = 0; i < AR; ++i) {
      const int r = rbase + 32 * i;
      uint4 v = make_uint4(0, 0, 0, 0);
      if constexpr (CONV) {
        if (r < BM && ri[i].n >= 0 && kvalid) {
          int iy = ri[i].iy0 + ky, ix = ri[i].ix0 + kx;
          if (iy >= 0 && iy < a.g.Hv && ix >= 0 && ix < a.g.Wv) {
            if (resized) {
              if (a.g.Hv == 2 * a.g.Hin) iy >>= 1; else if (a.g.Hv != a.g.Hin) iy = min((int)((float)iy * sy), a.g.Hin - 1);
              if (a.g.Wv == 2 * a.g.Win) ix >>= 1; else if (a.g.Wv != a.g.Win) ix = min((int)((float)ix * sx), a.g.Win - 1);
            }
            const long pix = ((long)ri[i].n * a.g.Hin + iy) * a.g.Win + ix;
            const T* src = kc < a.g.C0 ? (const T*)a.g.src0 + pix * a.g.C0 + kc
                                       : (const T*)a.g.src1 + pix * a.g.C1 + (kc - a.g.C0);
            v = *(const uint4*)src;
          }
        }
      } else {
        const int m = m0 + r;
        if (r < BM && m < a.M && kvalid) v = *(const uint4*)(Ap + (long)m * a.lda + k);
      }
      ra[i] = v;
    }
    // B
#pragma unroll
    for (int i = 0; i < BR; ++i) {
      const int r = rbase + 32 * i;
      const int n = n0 + r;
      uint4 v = make_uint4(0, 0, 0, 0);
      if (r < BN && n < a.N && kvalid) v = *(const uint4*)(Bp + (long)n * a.ldb + k);
      rb[i] = v;
    }
    if constexpr (CONV) {   // advance this thread's (tap, channel) to the next K tile
      kc += BK;
      while (kc >= Cin) {
        kc -= Cin;
        if (++kx == a.g.KW) { kx = 0; ++ky; }
      }
    }
  };

  // swizzled 16-byte slot of (row, chunk): rows r and r+1 share a 256-byte bank row
  auto slot = [](int row, int chunk) { return row * 8 + (chunk ^ ((row >> 1) & 7)); };

  auto store_tiles = [&](int buf) {
#pragma unroll
    for (int i = 0; i < AR; ++i) {
      const int r = rbase + 32 * i;
      if (r < BM) smem[buf][slot(r, cc)] = ra[i];
    }
#pragma unroll
    for (int i = 0; i < BR; ++i) {
      const int r = rbase + 32 * i;
      if (r < BN) smem[buf][BM * 8 + slot(r, cc)] = rb[i];
    }
  };

  f32x4 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int nk = (a.K + BK - 1) / BK;
  load_tiles(0);
  store_tiles(0);
  __syncthreads();

  const int frow = lane & 15, fgrp = lane >> 4;
  for (int kt = 0; kt < nk; ++kt) {
    const int buf = kt & 1;
    if (kt + 1 < nk) load_tiles(kt + 1);
    const uint4* As = smem[buf];
    const uint4* Bs = smem[buf] + BM * 8;
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      uint4 af[TM], bfr[TN];
#pragma unroll
      for (int i = 0; i < TM; ++i) af[i] = As[slot(wm * TM * 16 + i * 16 + frow, s * 4 + fgrp)];
#pragma unroll
      for (int j = 0; j < TN; ++j) bfr[j] = Bs[slot(wn * TN * 16 + j * 16 + frow, s * 4 + fgrp)];
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j) {
          if constexpr (sizeof(T) == 2) {
            acc[i][j] = Mfma<T>::m16x16x32(af[i], bfr[j], acc[i][j]);
          } else {
            // lane group g holds k = 16s + 4g + e in component e: four K=4 MFMAs cover the 16-deep slice
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(__uint_as_float(af[i].x), __uint_as_float(bfr[j].x), acc[i][j], 0, 0, 0);
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(__uint_as_float(af[i].y), __uint_as_float(bfr[j].y), acc[i][j], 0, 0, 0);
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(__uint_as_float(af[i].z), __uint_as_float(bfr[j].z), acc[i][j], 0, 0, 0);
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(__uint_as_float(af[i].w), __uint_as_float(bfr[j].w), acc[i][j], 0, 0, 0);
          }
        }
    }
    if (kt + 1 < nk) store_tiles(buf ^ 1);
    __syncthreads();
  }

  // ---- epilogue: D[row = 4g + r][col = lane & 15] per 16x16 tile
  const T* __restrict__ Rp = a.residual ? (const T*)a.residual + (long)z * a.sR : nullptr;
#pragma unroll
  for (int i = 0; i < TM; ++i) {
#pragma unroll
    for (int j = 0; j < TN; ++j) {
      const int n = n0 + wn * TN * 16 + j * 16 + frow;
      if (n >= a.N) continue;
      const float bias = a.bias ? a.bias[n] : 0.f;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int m = m0 + wm * TM * 16 + i * 16 + fgrp * 4 + r;
        if (m >= a.M) continue;
        float v = acc[i][j][r] * a.alpha + bias;
        if (a.rowadd) v += a.rowadd[(long)(m / a.rows_per_group) * a.rowadd_ld + n];
        v = apply_act(v, a.act);
        if (Rp) v += ld_f<T>(Rp + (long)m * a.ldr + n);
        v *= a.out_scale;
        const long off = HS ? c_off(a, m, n) : (long)m * a.ldc + n;   // HS: head-split layout (small M only)
        if constexpr (OUTF32) ((float*)a.C)[(long)z * a.sC + off] = v;
        else ((T*)a.C)[(long)z * a.sC + off] = from_f<T>(v);
      }
    }
  }
}

// kernel instantiation name as rocprofv3 prints it (demangled), used by the in-process profiler
template <typename T, int WM, int WN, int TM, int TN>
std::string kname(bool conv, bool f32out) {
  return std::string("irx::(anonymous namespace)::gemm_kernel<") + (sizeof(T) == 4 ? "float" : std::is_same<T, f16_t>::value ? "_Float16" : "unsigned short") +
         ", " + std::to_string(WM) + ", " + std::to_string(WN) + ", " + std::to_string(TM) + ", " +
         std::to_string(TN) + ", " + (conv ? "true" : "false") + ", " + (f32out ? "true" : "false") + ">";
}

template <typename T, int WM, int WN, int TM, int TN>
void launch_cfg(const GemmArgs& a, hipStream_t s) {
  constexpr int BM = WM * TM * 16, BN = WN * TN * 16;
  const int tiles = ((a.M + BM - 1) / BM) * ((a.N + BN - 1) / BN);
  dim3 grid(tiles, a.batch), block(kThreads);
  std::string nm;
  if (prof_on()) {
    nm = kname<T, WM, WN, TM, TN>(a.conv, a.out_f32);
    if (g_prof_shapes)
      nm += " [M " + std::to_string(a.M) + " N " + std::to_string(a.N) + " K " + std::to_string(a.K) + " batch " +
            std::to_string(a.batch) + (a.hs_L ? " hs" : "") + (a.residual ? " res" : "") + "]";
  }
  ProfScope ps(nm, 2.0 * a.M * a.N * (double)a.K * a.batch, s);
  if (a.hs_L) {
    IRX_CHECK(!a.conv && !a.out_f32, "head-split output: plain 16-bit GEMMs only");
    gemm_kernel<T, WM, WN, TM, TN, false, false, true><<<grid, block, 0, s>>>(a);
  } else if (a.conv) {
    if (a.out_f32) gemm_kernel<T, WM, WN, TM, TN, true, true><<<grid, block, 0, s>>>(a);
    else gemm_kernel<T, WM, WN, TM, TN, true, false><<<grid, block, 0, s>>>(a);
  } else {
    if (a.out_f32) gemm_kernel<T, WM, WN, TM, TN, false, true><<<grid, block, 0, s>>>(a);
    else gemm_kernel<T, WM, WN, TM, TN, false, false><<<grid, block, 0, s>>>(a);
  }
  IRX_LAUNCH_CHECK();
}

template <typename T>
void launch_t(const GemmArgs& a, hipStream_t s) {
  if (a.N <= 16) launch_cfg<T, 4, 1, 4, 1>(a, s);                          // 256 x 16
  else if (a.M <= 1024) launch_cfg<T, 2, 2, 2, 2>(a, s);                   // 64 x 64
  else if (a.N <= 64 || (a.N % 128) != 0) launch_cfg<T, 4, 1, 4, 4>(a, s); // 256 x 64
  else launch_cfg<T, 2, 2, 4, 4>(a, s);                                    // 128 x 128
}

}  // namespace

bool g_large_tiles = true;   // irx_set_option("large_tiles", 0) forces the 4-wave kernel (A/B tests)
int g_small_splitk = 1;

// K splits for a small-M GEMM on the 4-wave kernel (the CLIP text model's 154 rows, the time embedding's 2B rows): a
// few 64-column tiles over a long K leave most CUs idle (the CLIP fc2 [154 x 768 x 3072]: 36 blocks, 50 us).  The
// splits depend on N and K only (every M <= 256 takes the same ones: batch-invariant), whole 64-deep K steps each,
// and not on the output layout (a head-split q|k|v projection takes the same splits as its row-major twin).
static int small_splits(const GemmArgs& a) {
  if (!g_small_splitk || !is16(a.dtype) || a.conv || a.batch != 1 || a.geglu || a.A1 || a.up2_w) return 0;
  if (a.M > 256 || a.N % 8 || a.K < 1024 || a.N <= 16) return 0;
  if (a.out_f32 ? a.ldc % 4 != 0 : (a.ldc % 8 != 0 || ((uintptr_t)a.C % 16) != 0)) return 0;
  if (a.residual && (a.ldr % 8 != 0 || ((uintptr_t)a.residual % 16) != 0)) return 0;
  const long ctiles = (a.N + 63) / 64;
  if (ctiles >= 128) return 0;
  int sp = 1;
  while (sp < 8 && ctiles * sp * 2 <= 256 && a.K % (sp * 2 * 64) == 0 && a.K / (sp * 2) >= 256) sp *= 2;
  return sp > 1 ? sp : 0;
}

void gemm(const GemmArgs& a, hipStream_t s) {
  const int vec = a.dtype == F32 ? 4 : 8;
  IRX_CHECK(a.M > 0 && a.N > 0 && a.K > 0, "empty GEMM");
  IRX_CHECK(a.K % vec == 0, "K must be a multiple of 16 bytes of elements");
  IRX_CHECK(a.B && a.C, "null operand");
  IRX_CHECK(a.hs_L == 0 || (a.batch == 1 && !a.geglu && a.hs_d % 8 == 0 && a.hs_C % a.hs_d == 0 &&
                            a.N % a.hs_C == 0 && a.M % a.hs_L == 0), "head-split output layout");
  IRX_CHECK(a.ldb % vec == 0 && ((uintptr_t)a.B % 16) == 0, "B rows must be 16-byte aligned");
  if (a.conv) {
    const ConvGeom& g = a.g;
    IRX_CHECK(g.src0 && g.C0 % vec == 0 && g.C1 % vec == 0, "conv channels must be 16-byte multiples");
    IRX_CHECK(((uintptr_t)g.src0 % 16) == 0 && (!g.src1 || ((uintptr_t)g.src1 % 16) == 0), "conv source alignment");
    IRX_CHECK(g.C1 == 0 || g.src1, "concat source missing");
    IRX_CHECK(a.K == g.KH * g.KW * (g.C0 + g.C1), "conv K mismatch");
    IRX_CHECK(a.M == g.N * g.Ho * g.Wo, "conv M mismatch");
    IRX_CHECK(g.Hv >= g.Hin && g.Wv >= g.Win, "virtual (upsampled) size must not shrink");
  } else {
    IRX_CHECK(a.A && a.lda % vec == 0 && ((uintptr_t)a.A % 16) == 0, "A rows must be 16-byte aligned");
    IRX_CHECK(!a.A1 || (a.batch == 1 && a.kA1 > 0 && a.kA1 < a.K && a.lda1 % vec == 0 && ((uintptr_t)a.A1 % 16) == 0),
              "second A source: batch 1, 0 < kA1 < K, 16-byte rows");
  }
  IRX_CHECK(!(a.ln_rs || a.ln_part) || (a.ln_u && gemm_ln_foldable(a)), "folded LayerNorm needs the large-tile path");
  IRX_CHECK(!a.ln_part || (a.ln_T >= 1 && a.K == a.ln_T * kLnGroup), "LayerNorm partials must cover the K row");
  if (a.geglu) {
    IRX_CHECK(gemm_geglu_fusable(a) && gemm_large_tile(a, s), "GEGLU epilogue needs the large-tile path");
    return;
  }
  if (a.ln_rs || a.ln_part) {
    IRX_CHECK(gemm_large_tile(a, s), "folded LayerNorm needs the large-tile path");
    return;
  }
  if (a.ln_out || a.b_rows) {
    IRX_CHECK((!a.ln_out || gemm_emits_ln_parts(a)) && (!a.b_rows || gemm_bimg_ok(a)) && gemm_large_tile(a, s),
              "LayerNorm partials / per-image weights need the large-tile epilogue");
    return;
  }
  if (a.gn_part) {
    IRX_CHECK(gemm_emits_gn_parts(a) > 0 && gemm_large_tile(a, s), "GroupNorm partials need the large-tile epilogue");
    return;
  }
  if (a.gn_ab) {
    IRX_CHECK(gemm_gn_fusable(a) && gemm_large_tile(a, s), "GroupNorm-fused operand needs the halo conv path");
    return;
  }
  if (a.dtype != F32 && g_large_tiles && gemm_large_tile(a, s)) return;
  IRX_CHECK(!a.A1, "a two-source A (conv1x1_as_dense) needs the large-tile path");
  // the 4-wave kernel maps rows through c_off for head-split outputs only: a sub-pixel (up2) output would land at
  // low-resolution offsets (gemm_up2_ok does not mirror every early exit of gemm_large_tile)
  IRX_CHECK(!a.up2_w, "a per-parity upsampler conv (up2) needs the large-tile path");
  if (const int sp = small_splits(a)) {   // raw fp32 partials per K split (the batch index), then the reduce kernel
    GemmArgs p = a;
    p.K = a.K / sp;
    p.batch = sp;
    p.sA = p.K;
    p.sB = p.K;
    p.C = splitk_scratch((size_t)sp * a.M * a.N * sizeof(float));
    p.hs_L = 0;           // partials row-major; the reduce kernel maps head-split rows (c_off)
    p.ldc = a.N;
    p.sC = (long)a.M * a.N;
    p.out_f32 = 1;
    p.bias = nullptr;
    p.rowadd = nullptr;
    p.residual = nullptr;
    p.act = ACT_NONE;
    p.alpha = 1.f;
    p.out_scale = 1.f;
    if (a.dtype == F16) launch_t<f16_t>(p, s);
    else launch_t<bf16_t>(p, s);
    splitk_reduce(a, (const float*)p.C, sp, a.M, a.N, s);
    return;
  }
  if (a.dtype == F32) launch_t<float>(a, s);
  else if (a.dtype == F16) launch_t<f16_t>(a, s);
  else launch_t<bf16_t>(a, s);
}

}  // namespace irx
