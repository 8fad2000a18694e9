// irx — large-tile bf16 MFMA GEMM / implicit-GEMM convolution (8 waves, LDS-DMA staging), gfx950.
//
// The throughput path for the big contractions of the UNet and VAE (M = pixels in the thousands to
// hundreds of thousands, N = Cout in {128 .. 10240}, K = 9*Cin or Cin):
//   * 512-thread workgroups (8 waves, 2 per SIMD), block tiles 256x256 / 128x320 / 256x128 / 128x256 /
//     128x128 chosen per call so N = 320/640/960/1280/2560 and 128/256/512 tile exactly and the grid
//     fills the 256 CUs (split-K with an fp32 partial-sum pass when the output has too few tiles);
//   * A and B staged global -> LDS with 16-byte global_load_lds (LDS-DMA, no VGPR round trip):
//     the im2col gather of a 3x3 / strided / upsampled / concatenated convolution is just a per-lane
//     source address (out-of-image taps and rows past M/N point at a zero page);
//   * LDS image written lane-linearly, bank-spread by an XOR swizzle applied on the SOURCE address
//     and undone on the ds_read_b128 fragment reads; two LDS stages: the DMA of K step k+1 is in
//     flight under the 2 x (TM x TN) v_mfma_f32_16x16x32_bf16 of step k, one barrier per step;
//   * epilogue staged through LDS one slab at a time and written as whole 16-byte row chunks
//     (bias / time-embedding row add / activation / residual fused);
//   * XCD-aware block -> tile mapping (tiles sharing an A panel on one XCD's L2).
// Requirements (else the 4-wave kernel in gemm.hip runs): bf16, K % 64 == 0, conv channel
// counts % 64 == 0 (a 64-deep K step never straddles a tap or the concat seam).
#include <cmath>
#include <map>
#include <mutex>
#include <type_traits>
#include <utility>

#include "ops.h"
#include "profile.h"

namespace irx {

__device__ uint4 g_zero_page[4];   // 64 zero bytes: the source of every padded / out-of-range lane
// Timing-diagnostic knock-outs (option gemm_dbg) exist only in the diagnostic build (scripts/build_stamps.sh:
// -DIRX_DIAG / -DIRX_HALO_STAMPS, scripts/_skdbg/libirx_stamps.so); the product library compiles them out.
#if defined(IRX_DIAG) || defined(IRX_HALO_STAMPS)
constexpr int kDbgMask = ~0;
#define IRX_HALO_DIAG 1
#else
constexpr int kDbgMask = 0;
#endif
#ifdef IRX_HALO_STAMPS
constexpr int kHaloStampBlocks = 2048;
__device__ unsigned long long g_halo_stamps[kHaloStampBlocks * 8 * 8];
// (timing-diagnostic build) per (block, wave): 5 segment sums of the halo loop's taps + the tap count
extern "C" int irx_debug_halo_stamps(void* out, int n) {
  if (n > kHaloStampBlocks * 64) n = kHaloStampBlocks * 64;
  return hipMemcpyFromSymbol(out, HIP_SYMBOL(g_halo_stamps), (size_t)n * 8, 0, hipMemcpyDeviceToHost) == hipSuccess ? n : -1;
}
#endif

namespace {

typedef __attribute__((address_space(3))) void lds_void;

typedef __attribute__((address_space(1))) unsigned gu32;
constexpr int kSplitCounters = 1 << 16;
// Split arrival tickets live in one zero-initialised array PER STREAM (self-resetting: the last arriver
// stores 0 back).  Launches on one stream are ordered, so a stream's tickets are never shared by two
// GEMMs in flight; two handles on two streams get disjoint arrays (no cross-stream ticket mixing).

struct Split {
  bool inkernel = false;   // last arriving split reduces (else splitk_reduce_kernel)
  int splits = 1;      // K splits (gridDim.y = batch * splits)
  int per = 0;         // K steps per split
  float* ws = nullptr; // fp32 partials [batch*splits][Mp][Np] (M, N rounded up to the tile: unchecked stores)
  int Mp = 0, Np = 0;
  unsigned* cnt = nullptr;   // this stream's arrival tickets (in-kernel mode)
};

template <typename F, int... I>
__device__ __forceinline__ void static_for(std::integer_sequence<int, I...>, F&& f) {
  (f(std::integral_constant<int, I>{}), ...);
}

// Wait until at most n of this wave's vector-memory operations (here: LDS-DMA pieces) are outstanding.
__device__ __forceinline__ void wait_vm(int n) {
  switch (n) {
#define IRX_VM(k) case k: asm volatile("s_waitcnt vmcnt(" #k ")" ::: "memory"); break;
    IRX_VM(0) IRX_VM(1) IRX_VM(2) IRX_VM(3) IRX_VM(4) IRX_VM(5) IRX_VM(6) IRX_VM(7) IRX_VM(8) IRX_VM(9)
    IRX_VM(10) IRX_VM(11) IRX_VM(12) IRX_VM(13) IRX_VM(14) IRX_VM(15) IRX_VM(16) IRX_VM(18) IRX_VM(20)
    IRX_VM(21) IRX_VM(24) IRX_VM(28) IRX_VM(30) IRX_VM(32) IRX_VM(35) IRX_VM(36) IRX_VM(40) IRX_VM(42)
    IRX_VM(45) IRX_VM(48) IRX_VM(49) IRX_VM(54) IRX_VM(56) IRX_VM(60)
#undef IRX_VM
    default: asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); break;
  }
}

// 16-byte LDS-DMA piece issued from inline asm: the compiler does not see the LDS write, so it cannot
// insert its own conservative vmcnt(0) in front of every ds_read (it cannot prove the ring stages
// disjoint); the ring's counted waits + s_barrier below provide the ordering instead.
__device__ __forceinline__ void glds16_asm(const void* g, uint32_t lds_addr) {
  asm volatile("s_mov_b32 m0, %1\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %0, off" ::"v"(g), "s"(lds_addr)
               : "memory", "m0");
}

// The same piece in the SADDR form: a wave-uniform 64-bit base (SGPRs) + a 32-bit per-lane byte offset.
__device__ __forceinline__ void glds16_s(uint32_t voff, const void* base, uint32_t lds_addr) {
  asm volatile("s_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %0, %1" ::"v"(voff), "s"(base), "s"(lds_addr)
               : "memory", "m0");
}

// BK: K depth of one LDS stage (64: 8 chunks of 16 B per row, 32: 4); S: stages in the ring.
// S == 2 is the classic double buffer (drain + barrier per step); S > 2 keeps S-2 stages of LDS-DMA in
// flight across each (raw) barrier, waiting with a counted vmcnt for exactly the stage about to be read.
// HALO (3x3 / stride 1 / pad 1 convs whose block tile is BM/W whole image rows): the A operand is not an
// im2col gather per K step but the tile's (rows + 2) x W pixel halo of one BK-channel slab, DMA'd into
// LDS once per slab and read by all 9 taps through shifted fragment addresses.  Per slab a block moves
// one halo + 9 B panels instead of 9 A panels + 9 B panels (1.5x fewer L2 -> LDS bytes per MFMA at
// 256x160 than the 256x320 im2col tile), with whole 128-B lines per request (BK 64).
constexpr int kHaloWMax = 64;    // widest image row a halo tile takes (LDS: 2 x (BM + 2W) x 2BK B)
// strip halo tiles (HALO == 5): 8 rows x 32 columns; halo 10 x 32 pixels + the neighbouring columns at halo pixels
// kStripEdgeL + h / kStripEdgeR + h (h = halo row 0..9), inside the (BM + 2 kHaloWMax)-pixel halo buffer
constexpr int kStripW = 32, kStripEdgeL = 320, kStripEdgeR = 336;
static_assert(kStripEdgeR + 16 <= 256 + 2 * kHaloWMax, "strip halo edge columns");

template <typename T, int BM, int BN, int WM, int WN, int BK, int S, bool CONV, bool OUTF32, bool RESIZE,
          int HALO = 0, bool PP = false>
__global__ __launch_bounds__(WM * WN * 64, WM * WN == 4 ? 2 : 1) void gemm2_kernel(GemmArgs a, Split sp) {
  constexpr int NW = WM * WN, NT = NW * 64;   // 8 waves (1 block/CU) or 4 waves (2 blocks/CU)
  constexpr int TM = BM / WM / 16, TN = BN / WN / 16;
  constexpr int ROWS = BM + BN;
  constexpr int CPR = BK / 8;                // 16-byte chunks per row per stage
  constexpr int RPI = 64 / CPR;              // rows per 1 KiB LDS-DMA wave instruction
  constexpr int NINST = ROWS / RPI;          // wave instructions per stage
  constexpr int IPW = (NINST + NW - 1) / NW;  // per wave (the surplus ones are dummies into a scratch KiB)
  constexpr int STAGE = ROWS * CPR;          // uint4 per stage
  constexpr int KSUB = BK / 32;              // 32-deep MFMA sub-steps per stage
  static_assert((NW == 8 || NW == 4) && ROWS % RPI == 0 && BM % 16 == 0 && (BK == 32 || BK == 64), "tile shape");
  static_assert(!HALO || (CONV && !RESIZE && S >= 2 && S <= 8 && NW == 8), "halo tiles: 3x3 conv");
  // HALO == 5: the ping-pong halo loop over 8-row x 32-column strip tiles (images wider than kHaloWMax, or rows
  // that are no power of two): the tile's GEMM rows are the strip's pixels in (row, column) order (host: the
  // tiles of an image are its strips, row block major), the halo is 10 rows x 32 columns plus the two
  // neighbouring columns (kept in the halo buffer's spare pixel rows), and the epilogue maps rows to NHWC pixels
  // HALO == 6 / 7: the per-parity 2x2 convs of a nearest-2x upsampler (GemmArgs::up2_*) on row / strip halo tiles:
  // 4 taps per slab, (ky, kx) = (1 - pad_t + i, 1 - pad_l + j) of the 3x3 halo neighbourhood
  constexpr bool STRIP = HALO == 5 || HALO == 7;
  constexpr int NTAP = (HALO == 6 || HALO == 7 || HALO == 9) ? 4 : 9;
  // HALO == 8: 8 x 8 images (the UNet's 8x8 level), four whole images per 256-row tile: image j's halo is its own
  // 10 x 8 block at halo pixel 80 j (zero rows above / below, never DMA'd), so a tap of tile row r reads halo pixel
  // r + 16 j + 8 ky + kx - 1; K splits finish in the separate reduce kernels (host)
  constexpr bool MI = HALO == 8 || HALO == 9;   // (9: the upsampler parity convs of 8x8 images, 4 taps)
  constexpr int HB_U4 = (BM + 2 * kHaloWMax) * CPR;   // one halo slab buffer (uint4)
  constexpr int RING = HALO ? 2 * HB_U4 + S * BN * CPR + CPR + 64 : S * STAGE;
  // (+ a scratch KiB for the surplus DMA pieces, inside the epilogue's staging area when the ring is smaller)
  constexpr int RINGX = RING + (!HALO && NINST % NW ? 64 : 0);
  constexpr int SMEM = RINGX > BM * BN / 8 ? RINGX : BM * BN / 8;
  static_assert(SMEM * 16 <= 160 * 1024, "LDS budget");
  __shared__ __attribute__((aligned(16))) uint4 smem[SMEM];

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave / WN, wn = wave % WN;
  const int tiles_n = a.N / BN + (a.N % BN != 0);
  const int tiles_m = (a.M + BM - 1) / BM;
  const int bid = xcd_remap(blockIdx.x, tiles_m * tiles_n);
  int tile_m, tile_n;
  if (a.group_m > 0) {   // (GemmArgs::group_m) groups of group_m M tiles, N-major inside a group
    const int gsz = a.group_m * tiles_n, grp = bid / gsz, r = bid - grp * gsz;
    const int gm = min(a.group_m, tiles_m - grp * a.group_m);
    tile_m = grp * a.group_m + r % gm;
    tile_n = r / gm;
  } else {
    tile_n = a.nmajor ? bid / tiles_m : bid % tiles_n;
    tile_m = a.nmajor ? bid % tiles_m : bid / tiles_n;
  }
  const int m0 = tile_m * BM, n0 = tile_n * BN;
  const int z = blockIdx.y / sp.splits, ks = blockIdx.y % sp.splits;
  const int nk_all = a.K / BK;
  const int kt0 = ks * sp.per;
  const int kt1 = min(nk_all, kt0 + sp.per);
  // (per-image weights, GemmArgs::b_rows: the tile's rows lie in one image)
  const long bimg = a.b_rows ? (long)(m0 / a.b_rows) : 0;
  const uint16_t* __restrict__ Bp = (const uint16_t*)a.B + (long)z * a.sB + bimg * a.b_img_stride;
  const float* __restrict__ biasp = a.bias ? a.bias + bimg * a.bias_img_stride : nullptr;
  const uint16_t* __restrict__ Ap = CONV ? nullptr : (const uint16_t*)a.A + (long)z * a.sA;
  const uint16_t* const A1p = CONV ? nullptr : (const uint16_t*)a.A1;   // second A source from K = kA1 (batch 1)
  const uint16_t* zp = (const uint16_t*)g_zero_page;

  // ---- per-lane DMA assignment: instruction q = wave*IPW + j covers rows RPI*q .. +RPI-1;
  //      lane -> row + 16-byte slot; it fetches the logical chunk slot ^ swz(row)
  // Each lane keeps a row base pointer (nullptr = zero page) and adds a block-uniform K offset per step;
  // conv rows re-derive their base only when the K walk enters a new tap or the concat's second source.
  auto swz = [](int r) { return CPR == 8 ? ((r >> 1) & 7) : ((r >> 2) & 3); };
  const int lrow = lane / CPR, lslot = lane % CPR;
  bool isA[IPW], live[IPW];
  int lk[IPW];                       // this lane's element offset in the K step (logical chunk * 8)
  int rn[IPW], riy[IPW], rix[IPW];   // conv A rows: image index (-1 invalid), receptive-field origin
  const uint16_t* rb[IPW];           // current row base (nullptr if out of range / padded tap)
  int arow[IPW];                     // dense A rows: the row index m (-1 invalid), for the switch to A1
#pragma unroll
  for (int j = 0; j < IPW; ++j) {
    const int q = wave * IPW + j;
    const int r = RPI * q + lrow;
    live[j] = q < NINST;
    isA[j] = live[j] && r < BM;
    lk[j] = (lslot ^ swz(r)) * 8;
    rn[j] = -1; riy[j] = 0; rix[j] = 0; rb[j] = nullptr; arow[j] = -1;
    if (!live[j]) continue;
    if (r < BM) {
      const int m = m0 + r;
      if (m < a.M) {
        if constexpr (CONV) {
          const int HWo = a.g.Ho * a.g.Wo;
          const int n = m / HWo, rem = m - n * HWo;
          const int oy = rem / a.g.Wo, ox = rem - oy * a.g.Wo;
          rn[j] = n;
          riy[j] = oy * a.g.stride - a.g.pad_t;
          rix[j] = ox * a.g.stride - a.g.pad_l;
        } else {
          arow[j] = m;
          rb[j] = (A1p && kt0 * BK >= a.kA1) ? A1p + (long)m * a.lda1 : Ap + (long)m * a.lda;
        }
      }
    } else {
      const int n = n0 + (r - BM);
      if (n < a.N) rb[j] = Bp + (long)n * a.ldb;
    }
  }
  const float sy = RESIZE ? (float)a.g.Hin / (float)a.g.Hv : 1.f;
  const float sx = RESIZE ? (float)a.g.Win / (float)a.g.Wv : 1.f;
  const int Cin = a.g.C0 + a.g.C1;
  // conv: channel / tap of the K step being issued (block-uniform)
  int kc = 0, ky = 0, kx = 0;
  auto retarget = [&]() {   // A-row bases for tap (ky, kx) and the source holding channel kc
    const bool second = kc >= a.g.C0;
    const uint16_t* sb = second ? (const uint16_t*)a.g.src1 : (const uint16_t*)a.g.src0;
    const int cs = second ? a.g.C1 : a.g.C0;
#pragma unroll
    for (int j = 0; j < IPW; ++j) {
      if (!isA[j]) continue;
      int iy = riy[j] + ky, ix = rix[j] + kx;
      const bool ok = rn[j] >= 0 && iy >= 0 && iy < a.g.Hv && ix >= 0 && ix < a.g.Wv;
      if constexpr (RESIZE) {
        iy = (a.g.Hv == 2 * a.g.Hin) ? (iy >> 1) : min((int)((float)iy * sy), a.g.Hin - 1);
        ix = (a.g.Wv == 2 * a.g.Win) ? (ix >> 1) : min((int)((float)ix * sx), a.g.Win - 1);
      }
      const long pix = ((long)rn[j] * a.g.Hin + iy) * a.g.Win + ix;
      rb[j] = ok ? sb + pix * cs : nullptr;
    }
  };
  if constexpr (CONV && !HALO) {
    const int k = kt0 * BK;
    const int tap = k / Cin;
    kc = k - tap * Cin;
    ky = tap / a.g.KW;
    kx = tap - ky * a.g.KW;
    retarget();
  }

  // (LDS byte addresses from one cast of the array base: a per-piece generic -> LDS pointer cast can leave a null
  //  test on the shared aperture that the diagnostic builds' early exits fail to fold)
  const uint32_t lds_base = __builtin_amdgcn_readfirstlane((uint32_t)(uintptr_t)(lds_void*)smem);
  auto issue = [&](int kt, int stage) {
    int koffA = CONV ? (kc >= a.g.C0 ? kc - a.g.C0 : kc) : kt * BK;
    if constexpr (!CONV) {
      if (A1p && koffA >= a.kA1) {      // the concat's second source (steps are issued in order: one switch)
        if (koffA == a.kA1 && kt != kt0) {
#pragma unroll
          for (int j = 0; j < IPW; ++j)
            if (isA[j] && arow[j] >= 0) rb[j] = A1p + (long)arow[j] * a.lda1;
        }
        koffA -= a.kA1;
      }
    }
    const int koffB = kt * BK;
#pragma unroll
    for (int j = 0; j < IPW; ++j) {
      const uint16_t* src = rb[j] ? rb[j] + ((isA[j] ? koffA : koffB) + lk[j]) : zp;
      const uint32_t dst = live[j] ? lds_base + (uint32_t)(stage * STAGE + (wave * IPW + j) * 64) * 16u
                                   : lds_base + (uint32_t)(SMEM - 64) * 16u;
      glds16_asm(src, __builtin_amdgcn_readfirstlane(dst));
    }
    if constexpr (CONV) {
      kc += BK;
      if (kc == Cin) {
        kc = 0;
        if (++kx == a.g.KW) { kx = 0; ++ky; }
        retarget();
      } else if (kc == a.g.C0) {
        retarget();
      }
    }
  };

  f32x4 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int frow = lane & 15, fgrp = lane >> 4;
  auto compute = [&](int st) {
    const uint4* As = smem + st * STAGE;
    const uint4* Bs = As + BM * CPR;
#pragma unroll
    for (int s = 0; s < KSUB; ++s) {
      uint4 af[TM], bfr[TN];
#pragma unroll
      for (int i = 0; i < TM; ++i) {
        const int r = wm * TM * 16 + i * 16 + frow;
        af[i] = As[r * CPR + ((s * 4 + fgrp) ^ swz(r))];
      }
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        const int r = wn * TN * 16 + j * 16 + frow;
        bfr[j] = Bs[r * CPR + ((s * 4 + fgrp) ^ swz(r + BM))];
      }
      if constexpr (S > 2) __builtin_amdgcn_s_setprio(1);
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j)
          acc[i][j] = Mfma<T>::m16x16x32(af[i], bfr[j], acc[i][j]);
      if constexpr (S > 2) __builtin_amdgcn_s_setprio(0);
    }
  };

  if constexpr (HALO == 2 || HALO == 4 || HALO >= 5) {
    // ---- ping-pong halo main loop (the default halo path; no GroupNorm-fused operand).  The two waves that
    //      share a SIMD (w and w + 4) take opposite roles in each half of a K step (slab c = kt / 9, tap
    //      t = kt % 9), so one of them always has MFMAs to issue while the other moves data:
    //        phase 1 of step kt: group 0 (waves 0-3) runs the 40 MFMAs of step kt on fragments it read in the
    //                            previous phase; group 1 (waves 4-7) issues the LDS-DMA of B(kt + 2) and reads
    //                            its own fragments of step kt;
    //        phase 2 of step kt: group 1 runs its MFMAs of step kt; group 0 reads its fragments of step kt + 1
    //                            and, at taps 0..5 of every slab c but the last, issues one sixth of slab c + 1's
    //                            halo (into the buffer of slab c - 1, which every wave finished reading before the
    //                            barrier that ended phase 1 of step 9c - 1... group 1's last load phase of c - 1).
    //      (the lock-step form, HALO == 1, issues DMA and fragment reads in both waves of a SIMD at once, and
    //      the matrix pipe idles meanwhile.)  B ring of S = 3 stages: B(kt + 2) goes into the stage of
    //      step kt - 1; group 1 waits for B(kt + 1) at the end of its load phase of kt, where group 0 needs it;
    //      group 0 waits for slab c + 1's halo at the end of its compute phase of tap 8.
    //      Each group runs its own straight-line program (9 taps unrolled, no role or diagnostic branches):
    //      every DMA piece is one SADDR-form `global_load_lds_dwordx4` — a wave-uniform 64-bit source base in
    //      SGPRs plus ONE per-lane byte offset (the XOR swizzle of a piece's 8 rows is the same for every piece,
    //      RPI == 8), its LDS target a scalar add; the two B steps past the split's end are issued anyway, as
    //      dummies into the free stage (in-range weight rows, never read), so every wait is a constant count.
    //      HALO == 4: the same loop with the timing-diagnostic knock-outs of option gemm_dbg (bits 2 no MFMAs,
    //      4 no B DMA, 8 no halo DMA, 16 no fragment reads, 32 no barriers; results are wrong when set).
    static_assert(S == 3 && KSUB == 2 && NW == 8 && CPR == 8 && RPI == 8, "ping-pong halo: 3-stage B ring, BK 64");
    constexpr bool DG = HALO == 4;
    const int dbg = DG ? a.dbg : 0;
    const int W = a.g.Win, H = a.g.Hin;
    const int Wl = STRIP ? kStripW : W, lw = __builtin_ctz(Wl);   // pixels per halo row in LDS
    const int HW = H * W;
    const int img = m0 / HW;
    int y0 = 0, x0 = 0;   // the tile's first output row / column
    const int img0 = MI ? m0 >> 6 : 0, nimg = MI ? min(4, (a.M - m0) >> 6) : 0;   // (MI: images of the tile)
    if constexpr (MI) {
    } else if constexpr (STRIP) {
      const int t = (m0 - img * HW) / BM, ns = W / kStripW, rb = t / ns;
      y0 = rb * (BM / kStripW);
      x0 = (t - rb * ns) * kStripW;
    } else {
      y0 = (m0 - img * HW) >> lw;
    }
    // halo wave-instructions (RPI pixel rows each; MI: the 4 images' 8 rows, the pad rows are zeroed instead)
    const int nhi = MI ? 32 : (((BM >> lw) + 2) << lw) / RPI;
    constexpr int NG = NW / 2;                        // waves per group
    constexpr int HPG = (BM + 2 * kHaloWMax) / RPI / NG;   // halo pieces per group-0 wave per slab
    // ... issued in 6 parts at taps 0-5 (4 taps per slab: 2 parts at taps 0-1), waited for at the slab's last tap
    constexpr int HPARTS = NTAP == 9 ? 6 : 2, HPP = HPG / HPARTS;
    static_assert(HPG * RPI * NG == BM + 2 * kHaloWMax && HPP * HPARTS == HPG, "halo pieces");
    constexpr int NBI = BN / RPI, BPG = NBI / NG;          // B wave-instructions per step, per group-1 wave
    static_assert(BPG * NG == NBI, "B pieces");
    const int wv = __builtin_amdgcn_readfirstlane(wave);   // (scalar: the role branch stays uniform)
    const bool g1 = wv >= NG;
    const int gw = wv - (g1 ? NG : 0);
    uint4* const Hb = smem;                           // [2][HB_U4]
    uint4* const Bsm = smem + 2 * HB_U4;              // [S][BN * CPR]
    uint4* const zrow = Bsm + S * BN * CPR;           // one zero pixel row: taps left / right of the image
    uint4* const scratch = zrow + CPR;                // 1 KiB target of the surplus / out-of-image pieces
    if (tid < CPR) zrow[tid] = uint4{0u, 0u, 0u, 0u};
    const uint32_t lds0 = __builtin_amdgcn_readfirstlane((uint32_t)(uintptr_t)(lds_void*)smem);
    const uint32_t ldsX = lds0 + (uint32_t)(scratch - smem) * 16u;
    // lane -> (row lr of the piece's 8, 16-byte chunk slot); the slot holds logical chunk slot ^ lr (= row & 7)
    const int lr = lane >> 3, lch = (lane & 7) ^ lr;
    // ---- halo rows outside the image (top / bottom tiles): zero in both buffers once, never DMA'd
    if constexpr (MI) {   // every image's pad rows 0 and 9 (8 pixels each), both buffers
      for (int i = tid; i < 2 * 4 * 2 * 8 * CPR; i += NT) {
        const int buf = i / (4 * 2 * 8 * CPR), rem = i - buf * (4 * 2 * 8 * CPR);
        const int j = rem / (2 * 8 * CPR), side = (rem / (8 * CPR)) & 1, k = rem % (8 * CPR);
        Hb[buf * HB_U4 + (j * 80 + side * 72) * CPR + k] = uint4{0u, 0u, 0u, 0u};
      }
    } else {
      const int ylo = y0 - 1, yhi = y0 + (BM >> lw);   // the halo's first / last image row
      for (int i = tid; i < 2 * (Wl * CPR); i += NT) {
        const int side = i / (Wl * CPR), k = i - side * (Wl * CPR);
        const bool out = side == 0 ? ylo < 0 : yhi >= H;
        const int hrow = side == 0 ? 0 : (BM >> lw) + 1;
        if (out) {
          Hb[hrow * Wl * CPR + k] = uint4{0u, 0u, 0u, 0u};
          Hb[HB_U4 + hrow * Wl * CPR + k] = uint4{0u, 0u, 0u, 0u};
        }
      }
    }
    // group 1: B(kt) pieces j = 0 .. BPG-1 of this wave: weight rows n0 + RPI * (gw * BPG + j) + lr
    const uint32_t voffB = (uint32_t)(lr * a.ldb + lch * 8) * 2u;
    const char* const bB = (const char*)(Bp + (long)(n0 + RPI * gw * BPG) * a.ldb);
    const long pstrB = (long)RPI * a.ldb * 2;
    const uint32_t ldsB = lds0 + (uint32_t)(2 * HB_U4 + gw * BPG * 64) * 16u;
    auto issueB = [&](int c, auto tc, int st) {   // B of (slab c, tap t) into stage st
      constexpr int t = decltype(tc)::value;
      if (DG && (dbg & 4)) return;
      const char* b = bB + (long)(t * Cin + c * BK) * 2;
      const uint32_t m = ldsB + (uint32_t)st * (BN * CPR * 16);
#pragma unroll
      for (int j = 0; j < BPG; ++j) glds16_s(voffB, b + j * pstrB, m + j * 1024u);
    };
    // group 0: halo piece q = gw * HPG + j of slab c = pixels RPI * q .. + 7 of the (rows + 2) x Wl halo, which
    // starts at image pixel P0 = (img * H + y0 - 1) * W + x0; a piece is wholly inside or outside the image.
    // STRIP: a halo row is 32 pixels (4 pieces); pieces nhi .. nhi + 3 are the neighbouring columns x0 - 1 (halo
    // rows 0-7, 8-9) and x0 + 32 (same), at halo pixels 320 + h / 336 + h, their lanes each on their own pixel
    // (zeros for pixels outside the image)
    const long P0 = (long)(img * H + y0 - 1) * W + x0;
    const long Plo = (long)img * HW, Phi = Plo + HW;
    const uint32_t voffH0 = (uint32_t)(lr * a.g.C0 + lch * 8) * 2u;
    const uint32_t voffH1 = (uint32_t)(lr * a.g.C1 + lch * 8) * 2u;
    auto issueH = [&](int c, int j0, int j1) {    // pieces [j0, j1) of slab c's halo
      if (DG && (dbg & 8)) return;
      const bool second = c * BK >= a.g.C0;
      const char* sb = (const char*)(second ? a.g.src1 : a.g.src0);
      const int cs = second ? a.g.C1 : a.g.C0;
      const int ch = second ? c * BK - a.g.C0 : c * BK;
      const uint32_t vo = second ? voffH1 : voffH0;
      const uint32_t mb = lds0 + (uint32_t)((c & 1) * HB_U4) * 16u;
#pragma unroll
      for (int j = j0; j < j1; ++j) {
        const int q = gw * HPG + j;
        if constexpr (MI) {   // piece q: image j = q / 8, its row q % 8 -> halo pixel 80 j + 8 + 8 (q % 8)
          const int j = q >> 3;
          const long P = (long)(img0 + j) * 64 + (q & 7) * RPI;
          const bool ok = q < nhi && j < nimg;
          glds16_s(vo, ok ? sb + (P * cs + ch) * 2 : sb, ok ? mb + (uint32_t)(j * 10 + 1 + (q & 7)) * 1024u : ldsX);
          continue;
        }
        if constexpr (STRIP) {
          if (q >= nhi && q < nhi + 4) {   // a neighbouring column: per-lane addresses (one pixel per lane row)
            const int e = q - nhi, hr = (e & 1) * RPI + lr, yy = y0 - 1 + hr;
            const int col = (e >> 1) ? x0 + kStripW : x0 - 1;
            const bool v = hr < (BM >> lw) + 2 && (unsigned)yy < (unsigned)H && (unsigned)col < (unsigned)W;
            const uint16_t* src =
                v ? (const uint16_t*)sb + ((long)(img * H + yy) * W + col) * cs + ch + lch * 8 : zp;
            glds16_asm(src, mb + (uint32_t)q * 1024u);
            continue;
          }
          const int hr = q >> 2;   // (kStripW / RPI = 4 pieces per halo row)
          const long P = P0 + (long)hr * W + (q & 3) * RPI;
          const bool ok = q < nhi && (unsigned)(y0 - 1 + hr) < (unsigned)H;
          glds16_s(vo, ok ? sb + (P * cs + ch) * 2 : sb, ok ? mb + (uint32_t)q * 1024u : ldsX);
        } else {
          const long P = P0 + RPI * q;
          const bool ok = q < nhi && P >= Plo && P < Phi;
          glds16_s(vo, ok ? sb + (P * cs + ch) * 2 : sb, ok ? mb + (uint32_t)q * 1024u : ldsX);
        }
      }
    };
    // ---- fragment addressing, hoisted out of the K loop.  With the 9 taps of a slab unrolled, the tap (ky, kx)
    //      and the B stage (kt % 3 == t % 3: splits start at whole slabs) are compile-time, so every fragment
    //      address is a per-lane offset (6 A variants: kx x sub-step; 2 B variants) + a wave-uniform base + an
    //      immediate.  The A swizzle of halo row hp is hp & 7 = (frow + kx - 1) & 7 (W and i * 16 are
    //      multiples of 8).
    int aoff[3][KSUB], boff[KSUB];
    // NTAP == 4: the parity's tap offsets (block-uniform); aoff[0 / 1] = columns kx0 / kx0 + 1
    const int ky0 = 1 - a.g.pad_t, kx0 = 1 - a.g.pad_l;
#pragma unroll
    for (int ss = 0; ss < KSUB; ++ss) {
      const int ck = ss * 4 + fgrp;
#pragma unroll
      for (int kx = 0; kx < 3; ++kx)
        aoff[kx][ss] = frow * CPR + (ck ^ ((frow + (NTAP == 9 ? kx : kx0 + kx) - 1) & 7));
      boff[ss] = frow * CPR + (ck ^ (frow & 7));
    }
    const int awave = wm * TM * 16 * CPR, bwave = wn * TN * 16 * CPR, rowW = Wl * CPR;
    bool zl[TM], zr[TM];   // fragment rows at the image's left / right edge: taps kx = 0 / 2 read the zero row
#pragma unroll
    for (int i = 0; i < TM; ++i) {
      const int rx = (wm * TM * 16 + i * 16 + frow) & (Wl - 1);
      zl[i] = rx == 0 && (NTAP == 9 || kx0 == 0);        // (NTAP 4: only a parity whose taps reach kx = 0 / 2)
      zr[i] = rx == Wl - 1 && (NTAP == 9 || kx0 == 1);
    }
    // STRIP: the strip row of fragment i (its 16 rows lie in one 32-pixel strip row: wave-uniform); its edge lanes
    // read the neighbouring column's pixel of halo row eh + ky, logical chunk ck at slot ck ^ ((eh + ky) & 7)
    int eh[TM];
#pragma unroll
    for (int i = 0; i < TM; ++i) eh[i] = __builtin_amdgcn_readfirstlane((wm * TM * 16 + i * 16) >> lw);
    // MI: fragment i's image j (its 16 rows lie in one 64-row image) shifts its halo reads by 16 j pixels
    int mio[TM];
#pragma unroll
    for (int i = 0; i < TM; ++i) mio[i] = MI ? __builtin_amdgcn_readfirstlane(((wm * TM * 16 + i * 16) >> 6) * 16 * CPR) : 0;
    uint4 fa[KSUB][TM], fb[KSUB][TN];
    // fragments of tap t (both 32-deep sub-steps), B from stage st.  NTAP 9: (ky, kx) = (t / 3, t % 3), st = t % 3,
    // all compile-time; NTAP 4: ky = ky0 + t / 2 and column kx0 + t % 2 (block-uniform), the stage counted at run time
    auto readF = [&](auto tc, const uint4* Hs, int st) {
      constexpr int t = decltype(tc)::value;
      constexpr int kxi = NTAP == 9 ? t % 3 : t % 2;            // aoff column
      constexpr int kxe = NTAP == 9 ? t % 3 : 2 * (t % 2);      // edge side: 0 left, 2 right, 1 none
      const int ky = NTAP == 9 ? t / 3 : ky0 + t / 2;
      const int kx = NTAP == 9 ? t % 3 : kx0 + t % 2;
      if (DG && (dbg & 16)) return;
      const uint4* Bs = Bsm + st * BN * CPR + bwave;
      const uint4* Hrow = Hs + awave + ky * rowW + (kx - 1) * CPR;
#pragma unroll
      for (int ss = 0; ss < KSUB; ++ss) {
#pragma unroll
        for (int i = 0; i < TM; ++i) {
          const uint4* src = Hrow + aoff[kxi][ss] + i * 16 * CPR + mio[i];
          if constexpr (STRIP) {
            if constexpr (kxe != 1) {
              const int h = eh[i] + ky;
              const uint4* e = Hs + ((kxe == 0 ? kStripEdgeL : kStripEdgeR) + h) * CPR + ((ss * 4 + fgrp) ^ (h & 7));
              src = (kxe == 0 ? zl[i] : zr[i]) ? e : src;
            }
          } else {
            if constexpr (kxe == 0) src = zl[i] ? zrow + ss * 4 + fgrp : src;
            if constexpr (kxe == 2) src = zr[i] ? zrow + ss * 4 + fgrp : src;
          }
          fa[ss][i] = *src;
        }
#pragma unroll
        for (int j = 0; j < TN; ++j) fb[ss][j] = Bs[boff[ss] + j * 16 * CPR];
      }
    };
    auto prio = [&](bool load) {   // (diagnostics only: bit 128 load phases at priority 1, bit 256 compute phases)
      if constexpr (DG) {
        if (dbg & (load ? 128 : 256)) __builtin_amdgcn_s_setprio(1);
        else if (dbg & 384) __builtin_amdgcn_s_setprio(0);
      }
    };
    auto mma = [&]() {
      if (DG && (dbg & 2)) return;
#pragma unroll
      for (int ss = 0; ss < KSUB; ++ss)
#pragma unroll
        for (int i = 0; i < TM; ++i)
#pragma unroll
          for (int j = 0; j < TN; ++j) acc[i][j] = Mfma<T>::m16x16x32(fa[ss][i], fb[ss][j], acc[i][j]);
    };
    // (sched_barrier: the MFMAs touch no memory, so without it the scheduler hoists them across the barrier asm
    // into the load phase, right behind the fragment reads they use — one wave then runs loads and MFMAs in
    // series and the two groups no longer alternate)
    // drain = false (the barrier that ends a load phase, where no later DMA of another wave can overwrite what this
    // wave's fragment reads are still fetching): the reads stay in flight across the barrier and each MFMA waits for
    // its own operands; group 1's tap-8 reads must land first (group 0's next halo goes into the buffer they read)
    auto barrier = [&](bool drain = true) {
      __builtin_amdgcn_sched_barrier(0);
      if (DG && (dbg & 32)) asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      else if (drain) asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
      else asm volatile("s_barrier" ::: "memory");
      __builtin_amdgcn_sched_barrier(0);
    };
    // timing-diagnostic build only (-DIRX_HALO_STAMPS, HALO == 4): per wave, scalar sums of the cycles between
    // the stamps of every tap (0 -> 1 DMA issue + fragment reads landed, 1 -> 2 B wait, 2 -> 3 barrier after the load
    // phase, 3 -> 4 MFMA issue, 4 -> 5 barrier after the compute phase), stored once by lane 0 into g_halo_stamps
#ifdef IRX_HALO_STAMPS
    unsigned long long stv[6] = {0, 0, 0, 0, 0, 0}, sts[5] = {0, 0, 0, 0, 0};
#define IRX_STAMP(i)                                                                                  \
  if constexpr (DG) {                                                                                 \
    __builtin_amdgcn_sched_barrier(0);                                                                \
    asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(stv[i])::"memory");                   \
    __builtin_amdgcn_sched_barrier(0);                                                                \
    if constexpr (i > 0) sts[i - 1] += stv[i] - stv[i - 1];                                          \
  }
#else
#define IRX_STAMP(i)
#endif
    // this split's K steps [kt0, kt1): whole slabs (host: sp.per is a multiple of NTAP); >= NTAP steps per split.
    // B stage of step kt: (kt - kt0) % 3 (= t % 3 at 9 taps per slab)
    const int c0 = kt0 / NTAP, cend = (kt1 + NTAP - 1) / NTAP;
    auto st_next = [](int st) { return st == S - 1 ? 0 : st + 1; };
    using I0 = std::integral_constant<int, 0>;
    using I1 = std::integral_constant<int, 1>;
    if (g1) {
      issueB(c0, I0{}, 0);
      issueB(c0, I1{}, 1);
      wait_vm(BPG);                                      // B(kt0) landed
      barrier();                                         // (+ the zero row, the zeroed out-of-image halo rows)
      barrier();                                         // group 1 runs one phase behind group 0
      int sti = 0;                                       // (NTAP 4: the run-time stage of step kt)
      for (int c = c0; c < cend; ++c) {
        const uint4* Hs = Hb + (c & 1) * HB_U4;
        static_for(std::make_integer_sequence<int, NTAP>{}, [&](auto tc) {
          constexpr int t = decltype(tc)::value;
          const int st = NTAP == 9 ? t % S : sti, st2 = NTAP == 9 ? (t + 2) % S : st_next(st_next(sti));
          // load phase: B(kt + 2) (past the split's end: a dummy), fragments of kt, B(kt + 1) landed
          // (fragment reads first: they are what this phase waits for; the DMA issue overlaps their latency)
          IRX_STAMP(0);
          prio(true);
          readF(tc, Hs, st);
          if constexpr (t < NTAP - 2) issueB(c, std::integral_constant<int, t + 2>{}, st2);
          else issueB(c + 1, std::integral_constant<int, t + 2 - NTAP>{}, st2);
          IRX_STAMP(1);
          wait_vm(BPG);
          IRX_STAMP(2);
          barrier(t == NTAP - 1);
          IRX_STAMP(3);
          prio(false);
          mma();                                         // compute phase
          IRX_STAMP(4);
          barrier();
          IRX_STAMP(5);
          if constexpr (NTAP != 9) sti = st_next(sti);
        });
      }
    } else {
      issueH(c0, 0, HPG);
      wait_vm(0);                                        // H(c0) landed
      barrier();
      int sti = 0;
      for (int c = c0; c < cend; ++c) {
        const uint4* Hs = Hb + (c & 1) * HB_U4;
        const bool more = c + 1 < cend;
        static_for(std::make_integer_sequence<int, NTAP>{}, [&](auto tc) {
          constexpr int t = decltype(tc)::value;
          const int st = NTAP == 9 ? t % S : sti;
          // load phase: a part of slab c + 1's halo, fragments of kt (B(kt) landed: group 1 waited for it)
          IRX_STAMP(0);
          prio(true);
          readF(tc, Hs, st);
          if constexpr (t < HPARTS) {
            if (more) issueH(c + 1, t * HPP, (t + 1) * HPP);
          }
          IRX_STAMP(1);
          IRX_STAMP(2);
          barrier(false);
          IRX_STAMP(3);
          prio(false);
          mma();                                         // compute phase
          if constexpr (t == NTAP - 1) wait_vm(0);       // slab c + 1's halo landed
          IRX_STAMP(4);
          barrier();
          IRX_STAMP(5);
          if constexpr (NTAP != 9) sti = st_next(sti);
        });
      }
      barrier();
    }
#ifdef IRX_HALO_STAMPS
    if constexpr (DG) {
      if (lane == 0 && blockIdx.x < kHaloStampBlocks) {
        unsigned long long* o = g_halo_stamps + ((long)blockIdx.x * NW + wave) * 8;
#pragma unroll
        for (int i = 0; i < 5; ++i) o[i] = sts[i];
        o[5] = (unsigned long long)(cend - c0) * 9;
      }
    }
#endif
#undef IRX_STAMP
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
  } else if constexpr (HALO == 1) {
    // ---- halo main loop: K step kt = (slab c = kt / 9, tap t = kt % 9), a slab = BK channels; host
    //      guarantees W = 2^lw in [16, kHaloWMax], BM % W == 0, H % (BM / W) == 0, C0 % BK == C1 % BK == 0,
    //      one split (kt0 = 0).
    //      B panels run through an S-stage ring (S-2 steps of DMA in flight across each barrier); slab
    //      c+1's halo is issued at tap 0 of slab c into the other halo buffer.  Every wave issues the same
    //      number of DMA pieces per step (surplus pieces land in a scratch KiB), so one counted vmcnt per
    //      step covers both streams.
    const int W = a.g.Win, H = a.g.Hin, lw = __builtin_ctz(W);
    const int HW = H * W;
    const int img = m0 / HW, y0 = (m0 - img * HW) >> lw;
    const int nhi = (((BM >> lw) + 2) << lw) / RPI;   // halo wave-instructions (RPI pixel rows each)
    const int hpw = (nhi + NW - 1) / NW;              // ... per wave
    uint4* const Hb = smem;                           // [2][HB_U4]
    uint4* const Bsm = smem + 2 * HB_U4;              // [S][BN * CPR]
    uint4* const zrow = Bsm + S * BN * CPR;           // one zero pixel row: taps left / right of the image
    uint4* const scratch = zrow + CPR;                // 1 KiB target of the surplus pieces
    if (tid < CPR) zrow[tid] = uint4{0u, 0u, 0u, 0u};
    // chunk slot XOR swz(row), conflict-free ds_read_b128 fragments for any row shift in {-1, 0, +1} (the
    // kx taps), checked against the gfx950 lane groups: 128-B rows r & 7, 64-B rows 2 * bit2(r)
    auto swz = [](int r) { return CPR == 8 ? (r & 7) : (((r >> 2) & 1) << 1); };
    constexpr int NBI = BN / RPI, IPB = (NBI + NW - 1) / NW;
    const uint16_t* bro[IPB];
#pragma unroll
    for (int j = 0; j < IPB; ++j) {
      const int q = wave * IPB + j, r = RPI * q + lane / CPR;
      bro[j] = (q < NBI && n0 + r < a.N) ? Bp + (long)(n0 + r) * a.ldb + (((lane % CPR) ^ swz(r)) * 8) : nullptr;
    }
    auto issueB = [&](int kt, int st) {
      const int c = kt / 9, t = kt - 9 * c;
      const int off = t * Cin + c * BK;
#pragma unroll
      for (int j = 0; j < IPB; ++j) {
        const int q = wave * IPB + j;
        uint4* dst = q < NBI ? Bsm + st * BN * CPR + q * 64 : scratch;
        glds16_asm(bro[j] ? bro[j] + off : zp, __builtin_amdgcn_readfirstlane((uint32_t)(uintptr_t)(lds_void*)dst));
      }
    };
    auto issueH = [&](int c) {
      const bool second = c * BK >= a.g.C0;
      const uint16_t* sb = second ? (const uint16_t*)a.g.src1 : (const uint16_t*)a.g.src0;
      const int cs = second ? a.g.C1 : a.g.C0;
      const int ch = second ? c * BK - a.g.C0 : c * BK;
#pragma unroll 1
      for (int j = 0; j < hpw; ++j) {
        const int q = wave * hpw + j;
        const int p = RPI * q + lane / CPR;
        const int y = y0 - 1 + (p >> lw), x = p & (W - 1);
        const bool ok = q < nhi && y >= 0 && y < H;
        const uint16_t* src = ok ? sb + ((long)(img * H + y) * W + x) * cs + ch + (((lane % CPR) ^ swz(p)) * 8) : zp;
        uint4* dst = q < nhi ? Hb + (c & 1) * HB_U4 + q * 64 : scratch;
        glds16_asm(src, __builtin_amdgcn_readfirstlane((uint32_t)(uintptr_t)(lds_void*)dst));
      }
    };
    // GroupNorm(+SiLU) of the conv input applied in LDS, once per landed halo slab (GemmArgs::gn_ab): the same
    // gn_act + rounding as gn_apply_kernel, so the fused conv sees bit-identical operands.  Halo rows outside
    // the image (zero-page fills) stay zero: the conv pads the normalised tensor.
    const float2* gab = a.gn_ab ? a.gn_ab + (long)img * Cin : nullptr;
    // chunk j of slab c: elements tid + NT * j; chunks [j0, j1) per call
    auto transformH = [&](int c, int j0, int j1) {
      uint4* hb = Hb + (c & 1) * HB_U4;
      const int nel = min(nhi * 64, j1 * NT);
#pragma unroll 1
      for (int i = tid + j0 * NT; i < nel; i += NT) {
        const int p = i / CPR;
        const int y = y0 - 1 + (p >> lw);
        if (y < 0 || y >= H) continue;
        const float4* abp = (const float4*)(gab + c * BK + (((i % CPR) ^ swz(p)) * 8));
        float f[8];
        Vec16<T>::unpack(hb[i], f);
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const float4 v = abp[e];
          f[2 * e] = gn_act(f[2 * e], v.x, v.y, a.gn_silu);
          f[2 * e + 1] = gn_act(f[2 * e + 1], v.z, v.w, a.gn_silu);
        }
        hb[i] = Vec16<T>::pack(f);
      }
    };
    // this split's K steps [kt0, nk): whole slabs (host: sp.per is a multiple of 9)
    const int nk = kt1, c0 = kt0 / 9;
    issueH(c0);
#pragma unroll
    for (int p = 0; p < S - 1; ++p)
      if (kt0 + p < nk) issueB(kt0 + p, p);
    __syncthreads();      // zero row visible
    if (gab) {
      wait_vm(IPB * min(S - 1, nk - kt0));               // this wave's first-halo pieces landed (B pieces may fly)
      __syncthreads();
      transformH(c0, 0, 9 - S);                          // visible after the first main-loop barrier
    }
    int st = 0;
    for (int kt = kt0; kt < nk; ++kt) {
      const int c = kt / 9, t = kt - 9 * c;
      // younger than B(kt): B(kt+1 .. kt+S-2), and slab c+1's halo while it was issued after B(kt)
      int allow = IPB * min(S - 2, nk - 1 - kt);
      if (t >= 1 && t <= S - 1 && 9 * (c + 1) < nk) allow += hpw;
      wait_vm(__builtin_amdgcn_readfirstlane(allow));
      if (gab) asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");   // this wave's normalised-halo stores done
      asm volatile("s_barrier" ::: "memory");   // everyone's pieces landed; everyone finished reading kt-1
      if (kt + S - 1 < nk) issueB(kt + S - 1, st == 0 ? S - 1 : st - 1);
      if (t == 0 && 9 * (c + 1) < nk) issueH(c + 1);
      if (!(a.dbg & kDbgMask & 2)) {
        const int ky = t / 3, kx = t - 3 * ky;
        const int shift = ky * W + kx - 1;
        const uint4* Hs = Hb + (c & 1) * HB_U4;
        const uint4* Bs = Bsm + st * BN * CPR;
        // every sub-step's fragments are requested before the first MFMA: the LDS latency of sub-step
        // s+1 hides under the MFMAs of sub-step s (one register set per sub-step)
        uint4 af[KSUB][TM], bfr[KSUB][TN];
#pragma unroll
        for (int ss = 0; ss < KSUB; ++ss) {
          const int ck = ss * 4 + fgrp;
#pragma unroll
          for (int i = 0; i < TM; ++i) {
            const int r = wm * TM * 16 + i * 16 + frow;
            const int rx = r & (W - 1);
            const int hp = r + shift;
            const bool zero = (kx == 0 && rx == 0) || (kx == 2 && rx == W - 1);
            af[ss][i] = zero ? zrow[ck] : Hs[hp * CPR + (ck ^ swz(hp))];
          }
#pragma unroll
          for (int j = 0; j < TN; ++j) {
            const int r = wn * TN * 16 + j * 16 + frow;
            bfr[ss][j] = Bs[r * CPR + (ck ^ swz(r))];
          }
        }
        __builtin_amdgcn_s_setprio(1);
#pragma unroll
        for (int ss = 0; ss < KSUB; ++ss)
#pragma unroll
          for (int i = 0; i < TM; ++i)
#pragma unroll
            for (int j = 0; j < TN; ++j)
              acc[i][j] = Mfma<T>::m16x16x32(af[ss][i], bfr[ss][j], acc[i][j]);
        __builtin_amdgcn_s_setprio(0);
      }
      // taps S..8 of slab c: slab c+1's halo has landed (waited for since tap S) -> normalise it in place, one
      // NT-element chunk per tap behind this tap's MFMAs (the other resident wave's MFMAs hide its VALU work)
      if (gab && t >= S && 9 * (c + 1) < nk) transformH(c + 1, t - S, t - S + 1);
      st = st + 1 == S ? 0 : st + 1;
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
  } else if constexpr (PP && !CONV) {
    // ---- lean ping-pong for dense GEMMs (host: whole tiles, M % BM == N % BN == 0): the halo loop's form.  The
    //      waves w and w + 4 sharing a SIMD alternate a load phase (this wave's fragment reads of step kt, then its
    //      LDS-DMA pieces of step kt + 2) and a compute phase (step kt's MFMAs), group 1 one phase behind group 0.
    //      Every piece is one SADDR-form DMA: a wave-uniform row base in SGPRs + a per-lane byte offset fixed for
    //      the kernel; the step's K offset is a scalar add; the two steps past the split's end re-issue its last
    //      step into the free stage, so every wait count is a constant.  The stage index is compile-time (the K loop
    //      unrolled by 3) and the phases are pinned by sched_barrier (else the MFMAs, which touch no memory, move
    //      into the load phase).  Group 1's load barrier drains its reads: group 0's next DMA targets the stage they
    //      read; group 0's does not (each MFMA waits for its own operands).
    static_assert(S == 3 && NW == 8, "ping-pong: 3 stages, 8 waves");
    const int wv = __builtin_amdgcn_readfirstlane(wave);
    const bool g1 = wv >= NW / 2;
    const uint32_t lds0 = __builtin_amdgcn_readfirstlane((uint32_t)(uintptr_t)(lds_void*)smem);
    // two-source A (GemmArgs::A1, the 1x1 convs over a channel concat: proj_out o ff.net.2): A pieces switch to
    // the second source's row base / lane offset (pb1 / pv1) from K = kA1 on (a block-uniform choice per step)
    const char* pb[IPW];
    const char* pb1[IPW];
    uint32_t pv[IPW], pv1[IPW], pd[IPW];
    bool apc[IPW];
#pragma unroll
    for (int j = 0; j < IPW; ++j) {
      const int q = wv * IPW + j, r0 = RPI * q, r = r0 + lrow;
      const int ch = (lslot ^ swz(r)) * 8;
      apc[j] = q < NINST && r0 < BM;
      if (q < NINST && r0 < BM) {
        pb[j] = (const char*)(Ap + (long)(m0 + r0) * a.lda);
        pv[j] = (uint32_t)(lrow * a.lda + ch) * 2u;
      } else if (q < NINST) {
        pb[j] = (const char*)(Bp + (long)(n0 + r0 - BM) * a.ldb);
        pv[j] = (uint32_t)(lrow * a.ldb + ch) * 2u;
      } else {   // surplus piece: any in-range source, into the scratch KiB
        pb[j] = (const char*)(Ap + (long)m0 * a.lda);
        pv[j] = (uint32_t)lane * 16u;
      }
      pd[j] = q < NINST ? lds0 + (uint32_t)(q * 64) * 16u : lds0 + (uint32_t)(SMEM - 64) * 16u;
      pb1[j] = pb[j];
      pv1[j] = pv[j];
      if (A1p && apc[j]) {
        pb1[j] = (const char*)(A1p + (long)(m0 + r0) * a.lda1);
        pv1[j] = (uint32_t)(lrow * a.lda1 + ch) * 2u;
      }
    }
    auto issueP = [&](int kt, int st) {
      const long ko = (long)kt * BK * 2;
      const bool second = A1p && kt * BK >= a.kA1;
      const long ko1 = second ? ko - (long)a.kA1 * 2 : ko;   // (A pieces' K offset in their source)
      const uint32_t so = (uint32_t)(st * STAGE) * 16u;
#pragma unroll
      for (int j = 0; j < IPW; ++j) {
        const uint32_t dst = wv * IPW + j < NINST ? pd[j] + so : pd[j];
        if (apc[j] && second) glds16_s(pv1[j], pb1[j] + ko1, dst);
        else glds16_s(pv[j], pb[j] + ko, dst);
      }
    };
    uint4 fa[KSUB][TM], fb[KSUB][TN];
    auto readF = [&](auto stc) {
      constexpr int st = decltype(stc)::value;
      const uint4* As = smem + st * STAGE;
      const uint4* Bs = As + BM * CPR;
#pragma unroll
      for (int s = 0; s < KSUB; ++s) {
#pragma unroll
        for (int i = 0; i < TM; ++i) {
          const int r = wm * TM * 16 + i * 16 + frow;
          fa[s][i] = As[r * CPR + ((s * 4 + fgrp) ^ swz(r))];
        }
#pragma unroll
        for (int j = 0; j < TN; ++j) {
          const int r = wn * TN * 16 + j * 16 + frow;
          fb[s][j] = Bs[r * CPR + ((s * 4 + fgrp) ^ swz(r + BM))];
        }
      }
    };
    auto mma = [&]() {
#pragma unroll
      for (int s = 0; s < KSUB; ++s)
#pragma unroll
        for (int i = 0; i < TM; ++i)
#pragma unroll
          for (int j = 0; j < TN; ++j) acc[i][j] = Mfma<T>::m16x16x32(fa[s][i], fb[s][j], acc[i][j]);
    };
    auto barrier = [&](bool drain) {
      __builtin_amdgcn_sched_barrier(0);
      if (drain) asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
      else asm volatile("s_barrier" ::: "memory");
      __builtin_amdgcn_sched_barrier(0);
    };
    issueP(kt0, 0);
    issueP(min(kt0 + 1, kt1 - 1), 1);
    wait_vm(IPW);                                        // step kt0 landed
    barrier(true);
    if (g1) barrier(true);
    for (int kb = kt0; kb < kt1; kb += 3) {
      static_for(std::make_integer_sequence<int, 3>{}, [&](auto uc) {
        constexpr int u = decltype(uc)::value;
        const int kt = kb + u;
        if (kt < kt1) {
          readF(uc);                                     // load phase
          issueP(min(kt + 2, kt1 - 1), (u + 2) % 3);
          if (g1) wait_vm(IPW);                          // step kt + 1 landed (group 0 reads it next)
          barrier(g1);
          mma();                                         // compute phase
          if (!g1) wait_vm(IPW);
          barrier(true);
        }
      });
    }
    if (!g1) barrier(true);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
  } else if constexpr (PP) {
    // ---- ping-pong main loop (the dense GEMM / im2col conv counterpart of the HALO == 2 schedule): the waves
    //      w and w + 4 sharing a SIMD alternate between a load phase (LDS-DMA of step kt + 2, this wave's
    //      fragment reads of step kt) and a compute phase (step kt's MFMAs), group 1 one phase behind group 0,
    //      so every interval between barriers pairs one wave's MFMAs with its partner's loads.  S = 3 stages:
    //      step kt + 2 goes into the stage of step kt - 1, whose fragments every wave read before the barrier
    //      that ended its own load phase of kt - 1 (lgkmcnt(0) in `barrier`).  Each wave issues its IPW pieces
    //      of every step; group 1 waits for its pieces of step kt + 1 at the end of its load phase of kt,
    //      group 0 at the end of its compute phase of kt — both right before the barrier after which group 0
    //      reads step kt + 1.
    static_assert(S == 3 && NW == 8, "ping-pong: 3 stages, 8 waves");
    const int wv = __builtin_amdgcn_readfirstlane(wave);
    const bool g1 = wv >= NW / 2;
    uint4 fa[KSUB][TM], fb[KSUB][TN];
    auto readF = [&](int st) {
      const uint4* As = smem + st * STAGE;
      const uint4* Bs = As + BM * CPR;
#pragma unroll
      for (int s = 0; s < KSUB; ++s) {
#pragma unroll
        for (int i = 0; i < TM; ++i) {
          const int r = wm * TM * 16 + i * 16 + frow;
          fa[s][i] = As[r * CPR + ((s * 4 + fgrp) ^ swz(r))];
        }
#pragma unroll
        for (int j = 0; j < TN; ++j) {
          const int r = wn * TN * 16 + j * 16 + frow;
          fb[s][j] = Bs[r * CPR + ((s * 4 + fgrp) ^ swz(r + BM))];
        }
      }
    };
    auto mma = [&]() {
      if (a.dbg & kDbgMask & 2) return;
#pragma unroll
      for (int s = 0; s < KSUB; ++s)
#pragma unroll
        for (int i = 0; i < TM; ++i)
#pragma unroll
          for (int j = 0; j < TN; ++j) acc[i][j] = Mfma<T>::m16x16x32(fa[s][i], fb[s][j], acc[i][j]);
    };
    auto barrier = [] { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); };
    if (kt0 < kt1) issue(kt0, 0);
    if (kt0 + 1 < kt1) issue(kt0 + 1, 1);
    wait_vm(kt0 + 1 < kt1 ? IPW : 0);
    barrier();
    if (g1) barrier();
    int st = 0;
    for (int kt = kt0; kt < kt1; ++kt) {
      const int st2 = st == 0 ? 2 : st - 1;              // the stage of step kt - 1 == that of kt + 2
      // ---- load phase
      if (kt + 2 < kt1) issue(kt + 2, st2);
      readF(st);
      if (g1 && kt + 1 < kt1) {
        if (kt + 2 < kt1) wait_vm(IPW);
        else wait_vm(0);
      }
      barrier();
      // ---- compute phase
      mma();
      if (!g1 && kt + 1 < kt1) {
        if (kt + 2 < kt1) wait_vm(IPW);
        else wait_vm(0);
      }
      barrier();
      st = st == 2 ? 0 : st + 1;
    }
    if (!g1) barrier();
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
  } else if constexpr (S == 2) {
    if (kt0 < kt1) issue(kt0, 0);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    for (int kt = kt0; kt < kt1; ++kt) {
      const int st = (kt - kt0) & 1;
      if (kt + 1 < kt1) issue(kt + 1, st ^ 1);
      if (!(a.dbg & kDbgMask & 2)) compute(st);
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
    }
  } else {
    // prologue: stages 0 .. S-2 in flight
#pragma unroll
    for (int p = 0; p < S - 1; ++p)
      if (kt0 + p < kt1) issue(kt0 + p, p);
    int st = 0;
    for (int kt = kt0; kt < kt1; ++kt) {
      // this wave's pieces of step kt have landed once at most min(S-2, kt1-1-kt) younger stages remain
      wait_vm(IPW * min(S - 2, kt1 - 1 - kt));
      asm volatile("s_barrier" ::: "memory");   // everyone's pieces landed; everyone finished reading kt-1
      if (kt + S - 1 < kt1) issue(kt + S - 1, st == 0 ? S - 1 : st - 1);
      if (!(a.dbg & kDbgMask & 2)) compute(st);
      st = st + 1 == S ? 0 : st + 1;
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
  }

  if (a.dbg & kDbgMask & 1) {   // diagnostics: keep the accumulators live, skip the output
    float t = 0.f;
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int j = 0; j < TN; ++j) t += acc[i][j][0] + acc[i][j][1] + acc[i][j][2] + acc[i][j][3];
    if (t == 12345.678f) ((float*)a.C)[0] = t;
    return;
  }
  // ---- split-K: raw fp32 partial tile.  In-kernel mode: partials stored write-through (sc1), one relaxed
  //      agent-scope ticket per block; the tile's last arriving split adds the others' partials (sc1
  //      loads) into its accumulators and runs the normal epilogue (no release / acquire fences: they
  //      would write back / invalidate whole caches).  Otherwise splitk_reduce_kernel finishes.
  if (sp.splits > 1) {
    const long poff = (long)(m0 + wm * TM * 16 + fgrp * 4) * sp.Np + n0 + wn * TN * 16 + frow;
    float* P = sp.ws + (long)blockIdx.y * sp.Mp * sp.Np + poff;
    if (!sp.inkernel) {
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j)
#pragma unroll
          for (int r = 0; r < 4; ++r) P[(long)(i * 16 + r) * sp.Np + j * 16] = acc[i][j][r];
      return;
    }
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int j = 0; j < TN; ++j)
#pragma unroll
        for (int r = 0; r < 4; ++r)
          __hip_atomic_store((gu32*)(P + (long)(i * 16 + r) * sp.Np + j * 16), __float_as_uint(acc[i][j][r]),
                             __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // every storing wave drains its sc1 stores
    __syncthreads();
    int* flag = (int*)smem;                             // (one LDS array: no second __shared__ object)
    const int cidx = z * tiles_m * tiles_n + bid;
    if (tid == 0) {
      const unsigned prev = __hip_atomic_fetch_add((gu32*)&sp.cnt[cidx], 1u, __ATOMIC_RELAXED,
                                                   __HIP_MEMORY_SCOPE_AGENT);
      *flag = prev == (unsigned)(sp.splits - 1);
    }
    __syncthreads();
    const bool is_last = *flag != 0;
    __syncthreads();                                    // flag read by every wave before smem is reused
    if (!is_last) return;
    for (int s2 = 0; s2 < sp.splits; ++s2) {
      if (s2 == ks) continue;
      const float* Q = sp.ws + (long)(z * sp.splits + s2) * sp.Mp * sp.Np + poff;
#pragma unroll
      for (int i = 0; i < TM; ++i) {
        uint32_t v[TN][4];
#pragma unroll
        for (int j = 0; j < TN; ++j)
#pragma unroll
          for (int r = 0; r < 4; ++r)
            v[j][r] = __hip_atomic_load((gu32*)(Q + (long)(i * 16 + r) * sp.Np + j * 16), __ATOMIC_RELAXED,
                                        __HIP_MEMORY_SCOPE_AGENT);
#pragma unroll
        for (int j = 0; j < TN; ++j)
#pragma unroll
          for (int r = 0; r < 4; ++r) acc[i][j][r] += __uint_as_float(v[j][r]);
      }
    }
    if (tid == 0)   // ready for the next launch (the kernel boundary orders it)
      __hip_atomic_store((gu32*)&sp.cnt[cidx], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }

  // ---- epilogue (D[row = 4g + r][col = lane & 15] per 16x16 tile)
  const uint16_t* __restrict__ Rp = a.residual ? (const uint16_t*)a.residual + (long)z * a.sR : nullptr;
  // NHWC pixel row of GEMM row m (STRIP: the tiles of an image are its 8 x 32 strips, row block major, and a tile's
  // rows its pixels in (row, column) order; the row add and GroupNorm partials index images / tiles, unchanged)
  auto prow = [&](long m) -> long {
    if constexpr (STRIP) {
      const int HW = a.g.Hin * a.g.Win, W = a.g.Win;
      const long im = m / HW;
      const int t = (int)(m - im * HW), blk = t / BM, r = t - blk * BM, ns = W / kStripW, rb = blk / ns;
      return im * HW + (long)(rb * (BM / kStripW) + r / kStripW) * W + (blk - rb * ns) * kStripW + r % kStripW;
    } else {
      return m;
    }
  };
  if constexpr (!OUTF32) {
    if (a.vec_epilogue) {
      // Staged through LDS: pass 1 (every wave) applies alpha/bias/row-add/act and writes the bf16 tile
      // (16-byte chunks XOR-swizzled by row to spread banks); pass 2 streams whole 16-byte row chunks out,
      // adding the residual and applying out_scale, or (GEGLU) combining each 64-wide value block with its
      // gate block h * gelu(g) and writing half-width rows.
      static_assert(BM * BN * 2 <= SMEM * 16, "epilogue tile must fit the staging LDS");
      // (kept small on purpose: this straight-line part is unrolled over every accumulator; anything
      //  per-element beyond an FMA and an optional row add goes to the looped pass 2)
      uint16_t* tileS = (uint16_t*)smem;
      uint16_t* Cp = (uint16_t*)a.C + (long)z * a.sC;
      constexpr int CPR = BN / 8;               // 16-byte chunks per row
      // residual / row-add operands of the store passes requested before the first store (not for the 128x128 tiles:
      // two of them stay resident per CU only within 128 VGPRs)
      // (halo conv tiles only: the GroupNorm-partial loop of the 256x320 tiles spilled with it; on the 128x320
      //  tiles of proj_out ∘ ff.net.2 at 32^2 / 16^2 it measured no faster, profiles/r05_bench_shapes_chain.txt)
      constexpr bool kEpiPrefetch = HALO != 0;
      constexpr int kEpiPF = BN <= 128 ? 8 : 6;   // rows per residual batch (256x128: a thread's 8 rows, 256x160: 11 in 2)
      // chunk swizzle inside whole groups of 8 chunks only (BN = 160 leaves a 4-chunk tail unswizzled)
      auto csw = [](int c, int row) { return c < (CPR & ~7) ? c ^ (row & 7) : c; };
      if (a.ln_rs || a.ln_part) {
        // folded LayerNorm (GemmArgs::ln_rs / ln_part): y = rstd * acc - rstd * mean * u[n] + bias[n]  (alpha == 1)
        float uu[TN], bb[TN];
#pragma unroll
        for (int j = 0; j < TN; ++j) {
          const int n = n0 + wn * TN * 16 + j * 16 + frow;
          uu[j] = n < a.N ? a.ln_u[n] : 0.f;
          bb[j] = (biasp && n < a.N) ? biasp[n] : 0.f;
        }
#pragma unroll
        for (int i = 0; i < TM; ++i)
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const int row = wm * TM * 16 + i * 16 + fgrp * 4 + r;
            const float2 rs = m0 + row < a.M ? ln_rs_at(a.ln_rs, a.ln_part, a.ln_T, a.ln_eps, m0 + row)
                                             : make_float2(0.f, 0.f);
#pragma unroll
            for (int j = 0; j < TN; ++j) {
              const int col = wn * TN * 16 + j * 16 + frow;
              tileS[row * BN + (csw(col >> 3, row) << 3) + (col & 7)] =
                  __builtin_bit_cast(uint16_t, from_f<T>(fmaf(acc[i][j][r], rs.x, fmaf(-rs.y, uu[j], bb[j]))));
            }
          }
      } else {
#pragma unroll
        for (int j = 0; j < TN; ++j) {
          const int col = wn * TN * 16 + j * 16 + frow;
          const float bias = (biasp && n0 + col < a.N) ? biasp[n0 + col] : 0.f;
#pragma unroll
          for (int i = 0; i < TM; ++i)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
              const int row = wm * TM * 16 + i * 16 + fgrp * 4 + r;
              tileS[row * BN + (csw(col >> 3, row) << 3) + (col & 7)] =
                  __builtin_bit_cast(uint16_t, from_f<T>(acc[i][j][r] * a.alpha + bias));
            }
        }
      }
      __syncthreads();
      if (a.geglu) {
        // tile columns come in (64 value, 64 gate) pairs; output feature block = n0/2 + 64*pair
        constexpr int OCPR = CPR / 2;
#pragma unroll 1
        for (int idx = tid; idx < BM * OCPR; idx += NT) {
          const int row = idx / OCPR, oc = idx - row * OCPR;
          const int m = m0 + row;
          const int hc = (oc >> 3) * 16 + (oc & 7);       // value chunk; gate chunk is hc + 8
          if (m >= a.M || n0 + hc * 8 >= a.N) continue;
          float h[8], gt[8];
          Vec16<T>::unpack(*(const uint4*)(tileS + row * BN + ((hc ^ (row & 7)) << 3)), h);
          Vec16<T>::unpack(*(const uint4*)(tileS + row * BN + (((hc + 8) ^ (row & 7)) << 3)), gt);
#pragma unroll
          for (int e = 0; e < 8; ++e) h[e] = h[e] * gelu_erf16(gt[e]);
          *(uint4*)(Cp + (long)m * a.ldc + n0 / 2 + oc * 8) = Vec16<T>::pack(h);
        }
        return;
      }
      // one 16-byte output chunk: its operands (staged tile, residual, row add), then the final value (row add,
      // residual, output scale) formed and stored
      struct Src { uint4 u, r; float4 x, y; };
      auto fetch = [&](int row, int c, Src& q) {
        const int m = m0 + row, n = n0 + c * 8;
        q.u = *(const uint4*)(tileS + row * BN + (csw(c, row) << 3));
        if (Rp) q.r = *(const uint4*)(Rp + prow(m) * a.ldr + n);
        if (a.rowadd) {
          const float4* ra = (const float4*)(a.rowadd + (long)(m / a.rows_per_group) * a.rowadd_ld + n);
          q.x = ra[0];
          q.y = ra[1];
        }
      };
      auto combine = [&](int row, int c, const Src& q) -> uint4 {
        const int m = m0 + row, n = n0 + c * 8;
        uint4 u = q.u;
        if (Rp || a.rowadd || a.out_scale != 1.f) {
          float f[8];
          Vec16<T>::unpack(u, f);
          if (a.rowadd) {
            f[0] += q.x.x; f[1] += q.x.y; f[2] += q.x.z; f[3] += q.x.w;
            f[4] += q.y.x; f[5] += q.y.y; f[6] += q.y.z; f[7] += q.y.w;
          }
          if (Rp) {
            float rv[8];
            Vec16<T>::unpack(q.r, rv);
#pragma unroll
            for (int e = 0; e < 8; ++e) f[e] += rv[e];
          }
#pragma unroll
          for (int e = 0; e < 8; ++e) f[e] *= a.out_scale;
          u = Vec16<T>::pack(f);
        }
        *(uint4*)(Cp + c_off(a, prow(m), n)) = u;
        return u;
      };
      if (a.gn_part && NT >= BN) {
        // GroupNorm partials of the stored output, one per tile row block of BM rows (host: gemm_emits_gn_parts):
        // thread = fixed 8-channel chunk column x a row stride, shifted fp32 sums of the rounded values -> raw
        // fp64 (sum, sum of squares), folded over the row groups through LDS in a fixed order.
        constexpr int RS = NT / CPR;                 // row groups
        constexpr int TPC = NT >= BN ? NT / BN : 1;  // fold threads per column (first round)
        static_assert(NT < BN || (TPC >= 1 && RS * BN * 16 <= SMEM * 16), "GroupNorm partial staging");
        const int cc = tid % CPR, rg = tid / CPR;
        const bool colok = rg < RS && n0 + cc * 8 < a.N;
        double2* red = (double2*)smem;
        float x0[8], sm[8], sq[8];
        int cnt = 0;
#pragma unroll
        for (int e = 0; e < 8; ++e) { x0[e] = 0.f; sm[e] = 0.f; sq[e] = 0.f; }
        auto acc = [&](const uint4& u) {
          float f[8];
          Vec16<T>::unpack(u, f);
          if (cnt == 0) {
#pragma unroll
            for (int e = 0; e < 8; ++e) x0[e] = f[e];
          }
#pragma unroll
          for (int e = 0; e < 8; ++e) {
            const float dv = f[e] - x0[e];
            sm[e] += dv;
            sq[e] = fmaf(dv, dv, sq[e]);
          }
          ++cnt;
        };
        if (colok) {
          const int rend = min(BM, a.M - m0);
          if constexpr (kEpiPrefetch) {
            // every residual chunk of this thread's rows is requested before the first store (one memory latency
            // per tile instead of one per row: the stores may alias the residual, so the compiler cannot hoist the
            // loads itself); the row add is one vector per image, loaded once when the tile lies in one image
            constexpr int KMAX = (BM + RS - 1) / RS;
            const bool ra1 = a.rowadd && (m0 / a.rows_per_group) == ((m0 + rend - 1) / a.rows_per_group);
            float4 rx = make_float4(0.f, 0.f, 0.f, 0.f), ry = rx;
            if (ra1) {
              const float4* ra = (const float4*)(a.rowadd + (long)(m0 / a.rows_per_group) * a.rowadd_ld + n0 + cc * 8);
              rx = ra[0];
              ry = ra[1];
            }
            // batches of kEpiPF rows: their residual loads issued together (clamped rows, no branches: one vmcnt)
            uint4 rres[kEpiPF];
#pragma unroll 1
            for (int k0 = 0; k0 < KMAX; k0 += kEpiPF) {
              if (Rp) {
#pragma unroll
                for (int u = 0; u < kEpiPF; ++u) {
                  const int row = min(rg + (k0 + u) * RS, rend - 1);
                  rres[u] = *(const uint4*)(Rp + prow(m0 + row) * a.ldr + n0 + cc * 8);
                }
              }
#pragma unroll
            for (int u = 0; u < kEpiPF; ++u) {
              const int row = rg + (k0 + u) * RS;
              if (row >= rend) break;
              Src q;
              q.u = *(const uint4*)(tileS + row * BN + (csw(cc, row) << 3));
              q.r = rres[u];
              if (a.rowadd) {
                if (ra1) {
                  q.x = rx;
                  q.y = ry;
                } else {
                  const float4* ra = (const float4*)(a.rowadd + (long)((m0 + row) / a.rows_per_group) * a.rowadd_ld +
                                                     n0 + cc * 8);
                  q.x = ra[0];
                  q.y = ra[1];
                }
              }
              acc(combine(row, cc, q));
            }
            }
          } else {
            // (one row per step: a two-row software pipeline here pushed the 128x128 tiles past 128 VGPRs,
            //  i.e. from two resident blocks per CU to one)
#pragma unroll 1
            for (int row = rg; row < rend; row += RS) {
              Src q0;
              fetch(row, cc, q0);
              acc(combine(row, cc, q0));
            }
          }
        }
        __syncthreads();        // every read of the staged tile is done before `red` overlays it
        if (rg < RS) {
#pragma unroll
          for (int e = 0; e < 8; ++e) {
            const double x = x0[e], sd = sm[e];
            red[rg * BN + cc * 8 + e] = make_double2(cnt * x + sd, cnt * x * x + 2.0 * x * sd + (double)sq[e]);
          }
        }
        __syncthreads();
        // round 1: TPC threads per column over row groups j, j + TPC, ...; round 2: the TPC sums in order
        double2 v1 = make_double2(0.0, 0.0);
        const int col1 = tid / TPC, j1 = tid % TPC;
        if (col1 < BN)
          for (int g = j1; g < RS; g += TPC) {
            const double2 v = red[g * BN + col1];
            v1.x += v.x;
            v1.y += v.y;
          }
        __syncthreads();
        if (col1 < BN) red[tid] = v1;
        __syncthreads();
        for (int col = tid; col < BN; col += NT) {
          if (n0 + col >= a.N) continue;
          double A = 0.0, B = 0.0;
#pragma unroll
          for (int j = 0; j < TPC; ++j) {
            const double2 v = red[col * TPC + j];
            A += v.x;
            B += v.y;
          }
          long rb = m0 / BM;
          if (a.up2_w) {   // sub-pixel output: this parity's blocks of an image sit among the image's 4 x rpl
            const long rpl = (long)a.up2_h * a.up2_w / BM;
            rb = (rb / rpl * 4 + a.up2_p) * rpl + rb % rpl;
          }
          *(double2*)(a.gn_part + (rb * a.N + n0 + col) * 2) = make_double2(A, B);
        }
        return;
      }
      // LayerNorm partials of the output (GemmArgs::ln_out; host: gemm_emits_ln_parts, BN == kLnGroup): the final
      // values are written back over the staged tile, then G threads per row reduce it in two passes
      float2* const lno = BN == kLnGroup ? a.ln_out : nullptr;
      // head-split output (attention operands, GemmArgs::hs_L) with nothing to add: the tile's columns are whole
      // heads of one q / k / v part and its rows one image's tokens, so each head segment of the tile is one
      // contiguous [BM][hs_d] block of C.  Chunks are walked segment-major (consecutive lanes write consecutive
      // 16-byte chunks of a segment: whole lines per wave store) with the segment base computed once, instead of
      // c_off's three divides per chunk and stores scattered over every head of a row.
      if (a.hs_L && !Rp && !a.rowadd && !lno && a.out_scale == 1.f && (a.hs_d & 7) == 0 && a.hs_L % BM == 0 &&
          BN % a.hs_d == 0 && n0 % a.hs_d == 0 && a.hs_C % BN == 0 && m0 + BM <= a.M && n0 + BN <= a.N) {
        const int dch = a.hs_d >> 3, segc = BM * dch;
        const int part = n0 / a.hs_C, hd0 = (n0 - part * a.hs_C) / a.hs_d, heads = a.hs_C / a.hs_d;
        const long img = m0 / a.hs_L, tok0 = m0 - img * a.hs_L;
        uint16_t* const hb = Cp + (long)part * a.M * a.hs_C + ((img * heads + hd0) * a.hs_L + tok0) * a.hs_d;
        const long sstride = (long)a.hs_L * a.hs_d;
        const float inv_segc = 1.f / (float)segc, inv_dch = 1.f / (float)dch;
#pragma unroll 2
        for (int idx = tid; idx < BM * CPR; idx += NT) {
          // idx = (seg, row, cc): float-reciprocal quotients corrected by one step (exact for idx < 2^24)
          int seg = (int)((float)idx * inv_segc);
          seg += (seg + 1) * segc <= idx;
          seg -= seg * segc > idx;
          const int rem = idx - seg * segc;
          int row = (int)((float)rem * inv_dch);
          row += (row + 1) * dch <= rem;
          row -= row * dch > rem;
          const int cc = rem - row * dch, c = seg * dch + cc;
          *(uint4*)(hb + seg * sstride + (long)row * a.hs_d + cc * 8) =
              *(const uint4*)(tileS + row * BN + (csw(c, row) << 3));
        }
        return;
      }
      // one 16-byte chunk of the plain store pass: row add, residual, output scale; written back over the staged
      // tile when the LayerNorm partials below read it
      auto store_chunk = [&](int row, int c) {
        const int m = m0 + row, n = n0 + c * 8;
        uint4* const ts = (uint4*)(tileS + row * BN + (csw(c, row) << 3));
        uint4 u = *ts;
        if (Rp || a.rowadd || a.out_scale != 1.f) {
          float f[8];
          Vec16<T>::unpack(u, f);
          if (a.rowadd) {   // per-image time-embedding projection (added after the bf16 rounding of pass 1)
            const float4* ra = (const float4*)(a.rowadd + (long)(m / a.rows_per_group) * a.rowadd_ld + n);
            const float4 x = ra[0], y = ra[1];
            f[0] += x.x; f[1] += x.y; f[2] += x.z; f[3] += x.w; f[4] += y.x; f[5] += y.y; f[6] += y.z; f[7] += y.w;
          }
          if (Rp) {
            float rv[8];
            Vec16<T>::unpack(*(const uint4*)(Rp + prow(m) * a.ldr + n), rv);
#pragma unroll
            for (int e = 0; e < 8; ++e) f[e] += rv[e];
          }
#pragma unroll
          for (int e = 0; e < 8; ++e) f[e] *= a.out_scale;
          u = Vec16<T>::pack(f);
          if (lno) *ts = u;
        }
        *(uint4*)(Cp + c_off(a, prow(m), n)) = u;
      };
      // (one chunk per step: batching the residual loads of 8 steps measured no faster, 31.9 vs 31.9 us at the
      //  64^2-level to_out shape, profiles/r05_kbench_gemm_res.txt)
#pragma unroll 1
      for (int idx = tid; idx < BM * CPR; idx += NT) {
        const int row = idx / CPR, c = idx - row * CPR;
        if (m0 + row >= a.M || n0 + c * 8 >= a.N) continue;
        store_chunk(row, c);
      }
      if constexpr (BN == kLnGroup && NT % BM == 0) {
        if (lno) {
          // G adjacent lanes per row, each over CPR / G chunks: mean, then the sum of squared deviations from it
          constexpr int G = NT / BM, CPG = CPR / G;
          static_assert(CPR % G == 0 && (G == 1 || G == 2 || G == 4 || G == 8), "LayerNorm partial lanes");
          __syncthreads();
          // one pass of sums shifted by the row's first stored value x0: d = x - x0, mean = x0 + sum d / n,
          // M2 = sum d^2 - (sum d)^2 / n (x0 is a sample of the row, so the subtraction loses little)
          const int row = tid / G, g = tid % G;
          const uint16_t* trow = tileS + row * BN;
          float x0;
          {
            float f0[8];
            Vec16<T>::unpack(*(const uint4*)(trow + (csw(0, row) << 3)), f0);
            x0 = f0[0];
          }
          float s1 = 0.f, s2 = 0.f;
#pragma unroll 4
          for (int c = g * CPG; c < (g + 1) * CPG; ++c) {
            float f[8];
            Vec16<T>::unpack(*(const uint4*)(trow + (csw(c, row) << 3)), f);
#pragma unroll
            for (int e = 0; e < 8; ++e) {
              const float d = f[e] - x0;
              s1 += d;
              s2 = fmaf(d, d, s2);
            }
          }
#pragma unroll
          for (int o = 1; o < G; o <<= 1) {
            s1 += __shfl_xor(s1, o);
            s2 += __shfl_xor(s2, o);
          }
          const float ds = s1 * (1.f / (float)kLnGroup);
          if (g == 0 && m0 + row < a.M) {
            const float mean = x0 + ds, m2 = fmaxf(fmaf(-s1, ds, s2), 0.f);
            lno[(long)(m0 + row) * (a.N / kLnGroup) + n0 / kLnGroup] =
                a.ln_out_rs ? ln_fin(mean, m2, 1, a.ln_eps) : make_float2(mean, m2);
          }
        }
      }
      return;
    }
  }
#pragma unroll
  for (int i = 0; i < TM; ++i) {
#pragma unroll
    for (int j = 0; j < TN; ++j) {
      const int n = n0 + wn * TN * 16 + j * 16 + frow;
      if (n >= a.N) continue;
      const float bias = biasp ? biasp[n] : 0.f;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int m = m0 + wm * TM * 16 + i * 16 + fgrp * 4 + r;
        if (m >= a.M) continue;
        const float v = (acc[i][j][r] * a.alpha + bias) * a.out_scale;   // (no row add / residual here: eligible())
        if constexpr (OUTF32) ((float*)a.C)[(long)z * a.sC + (long)m * a.ldc + n] = v;
        else ((uint16_t*)a.C)[(long)z * a.sC + (long)m * a.ldc + n] = __builtin_bit_cast(uint16_t, from_f<T>(v));
      }
    }
  }
}

// sum of split-K partials + the full epilogue, 8 outputs (one 16-byte bf16 chunk) per thread
template <typename T, bool OUTF32>
__global__ __launch_bounds__(256) void splitk_reduce_kernel(GemmArgs a, const float* __restrict__ ws, int splits,
                                                            int Mp, int Np) {
  const int nv = a.N / 8;
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= (long)a.M * nv) return;
  const int z = blockIdx.y;
  const int m = (int)(i / nv), n = (int)(i % nv) * 8;
  float f[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) f[e] = 0.f;
  for (int s = 0; s < splits; ++s) {
    const float4* p = (const float4*)(ws + ((long)(z * splits + s) * Mp + m) * Np + n);
    const float4 x = p[0], y = p[1];
    f[0] += x.x; f[1] += x.y; f[2] += x.z; f[3] += x.w; f[4] += y.x; f[5] += y.y; f[6] += y.z; f[7] += y.w;
  }
  float rv[8];
  if (a.residual) {
    const uint16_t* R = (const uint16_t*)a.residual + (long)z * a.sR + (long)m * a.ldr + n;
    Vec16<T>::unpack(*(const uint4*)R, rv);
  }
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    const float* bp = a.bias ? a.bias + (a.b_rows ? (long)(m / a.b_rows) * a.bias_img_stride : 0) : nullptr;
    float v = f[e] * a.alpha + (bp ? bp[n + e] : 0.f);
    if (a.rowadd) v += a.rowadd[(long)(m / a.rows_per_group) * a.rowadd_ld + n + e];
    v = apply_act(v, a.act);
    if (a.residual) v += rv[e];
    f[e] = v * a.out_scale;
  }
  if constexpr (OUTF32) {
    float* C = (float*)a.C + (long)z * a.sC + c_off(a, m, n);
#pragma unroll
    for (int e = 0; e < 8; ++e) C[e] = f[e];
  } else {
    *(uint4*)((uint16_t*)a.C + (long)z * a.sC + c_off(a, m, n)) = Vec16<T>::pack(f);
  }
}

// The same reduce + epilogue for a 16-bit output that feeds a GroupNorm (GemmArgs::gn_part), also emitting the
// GroupNorm partials of the stored values per block of kRedGnRows rows (the 8x8-level convs: 64 rows = one image),
// so no statistics pass over the tensor follows.  Block = kRedGnRows rows x 64 channels: thread = one 16-byte
// channel chunk (8 of them) x a row stride of 32; shifted fp32 sums of the rounded outputs -> raw fp64, folded over
// the 32 row lanes through LDS in a fixed order (the large-tile epilogue's arithmetic; batch invariant: a row block
// never straddles two images).
constexpr int kRedGnRows = 64;
template <typename T>
__global__ __launch_bounds__(256) void splitk_reduce_gn_kernel(GemmArgs a, const float* __restrict__ ws, int splits,
                                                               int Mp, int Np) {
  __shared__ double2 red[32][64];
  const int cc = threadIdx.x & 7, rl = threadIdx.x >> 3;
  const int m0 = blockIdx.x * kRedGnRows, n = blockIdx.y * 64 + cc * 8;
  float x0[8], sm[8], sq[8];
  int cnt = 0;
#pragma unroll
  for (int e = 0; e < 8; ++e) { x0[e] = 0.f; sm[e] = 0.f; sq[e] = 0.f; }
  for (int r = rl; r < kRedGnRows; r += 32) {
    const int m = m0 + r;
    float f[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) f[e] = 0.f;
    for (int s2 = 0; s2 < splits; ++s2) {
      const float4* p = (const float4*)(ws + ((long)s2 * Mp + m) * Np + n);
      const float4 x = p[0], y = p[1];
      f[0] += x.x; f[1] += x.y; f[2] += x.z; f[3] += x.w; f[4] += y.x; f[5] += y.y; f[6] += y.z; f[7] += y.w;
    }
    float rv[8];
    if (a.residual) Vec16<T>::unpack(*(const uint4*)((const uint16_t*)a.residual + (long)m * a.ldr + n), rv);
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      float v = f[e] * a.alpha + (a.bias ? a.bias[n + e] : 0.f);
      if (a.rowadd) v += a.rowadd[(long)(m / a.rows_per_group) * a.rowadd_ld + n + e];
      v = apply_act(v, a.act);
      if (a.residual) v += rv[e];
      f[e] = v * a.out_scale;
    }
    const uint4 u = Vec16<T>::pack(f);
    *(uint4*)((uint16_t*)a.C + (long)m * a.ldc + n) = u;
    Vec16<T>::unpack(u, f);                           // the stored (rounded) values
    if (cnt == 0) {
#pragma unroll
      for (int e = 0; e < 8; ++e) x0[e] = f[e];
    }
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const float dv = f[e] - x0[e];
      sm[e] += dv;
      sq[e] = fmaf(dv, dv, sq[e]);
    }
    ++cnt;
  }
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    const double x = x0[e], sd = sm[e];
    red[rl][cc * 8 + e] = make_double2(cnt * x + sd, cnt * x * x + 2.0 * x * sd + (double)sq[e]);
  }
  __syncthreads();
  if (threadIdx.x < 64) {
    double A = 0.0, B = 0.0;
    for (int g = 0; g < 32; ++g) {
      A += red[g][threadIdx.x].x;
      B += red[g][threadIdx.x].y;
    }
    *(double2*)(a.gn_part + ((long)blockIdx.x * a.N + blockIdx.y * 64 + threadIdx.x) * 2) = make_double2(A, B);
  }
}

template <typename T, int BM, int BN, int WM, int WN, int BK, int S, int HALO, bool PP>
void launch2_t(const GemmArgs& a, const Split& sp, hipStream_t s) {
  const int tiles = ((a.M + BM - 1) / BM) * ((a.N + BN - 1) / BN);
  dim3 grid(tiles, a.batch * sp.splits), block(WM * WN * 64);
  const bool rs = a.conv && (a.g.Hv != a.g.Hin || a.g.Wv != a.g.Win);
  const char* tn = std::is_same<T, f16_t>::value ? "_Float16" : "unsigned short";
  std::string nm;
  if (prof_on())   // same spelling as the demangled name rocprofv3 reports
    nm = std::string("irx::(anonymous namespace)::gemm2_kernel<") + tn + ", " + std::to_string(BM) + ", " +
         std::to_string(BN) + ", " + std::to_string(WM) + ", " + std::to_string(WN) + ", " + std::to_string(BK) + ", " +
         std::to_string(S) + ", " + (a.conv ? "true" : "false") + ", " + (a.out_f32 ? "true" : "false") + ", " +
         (rs ? "true" : "false") + ", " + std::to_string(HALO) + ", " + (PP ? "true" : "false") + ">";
  if (prof_on() && g_prof_shapes)
    nm += " [M " + std::to_string(a.M) + " N " + std::to_string(a.N) + " K " + std::to_string(a.K) +
          (a.conv ? " conv " + std::to_string(a.g.Hin) + "x" + std::to_string(a.g.Win) : std::string()) +
          " split " + std::to_string(sp.splits) + (a.geglu ? " geglu" : "") + (a.residual ? " res" : "") +
          (a.ln_rs || a.ln_part ? " lnfold" : "") + (a.ln_out ? " lnout" : "") + (a.b_rows ? " bimg" : "") +
          (a.gn_part ? " gnpart" : "") + (a.up2_w ? " up2" : "") + "]";
  const GemmArgs& ea = a;
  {
    ProfScope ps(nm, 2.0 * a.M * a.N * (double)a.K * a.batch, s);
    if constexpr (HALO != 0) {
      gemm2_kernel<T, BM, BN, WM, WN, BK, S, true, false, false, HALO><<<grid, block, 0, s>>>(ea, sp);
    } else if (a.conv) {   // (fp32-output convs never take this path: see eligible())
      if (rs) gemm2_kernel<T, BM, BN, WM, WN, BK, S, true, false, true, 0, PP><<<grid, block, 0, s>>>(ea, sp);
      else gemm2_kernel<T, BM, BN, WM, WN, BK, S, true, false, false, 0, PP><<<grid, block, 0, s>>>(ea, sp);
    } else {
      if (a.out_f32) gemm2_kernel<T, BM, BN, WM, WN, BK, S, false, true, false, 0, PP><<<grid, block, 0, s>>>(ea, sp);
      else gemm2_kernel<T, BM, BN, WM, WN, BK, S, false, false, false, 0, PP><<<grid, block, 0, s>>>(ea, sp);
    }
    IRX_LAUNCH_CHECK();
  }
  if (sp.splits > 1 && !sp.inkernel && a.gn_part) {   // (host: gemm_emits_gn_parts checked the shape)
    ProfScope ps(prof_on() ? std::string("irx::(anonymous namespace)::splitk_reduce_gn_kernel<") + tn + ">"
                           : std::string(),
                 0.0, s);
    splitk_reduce_gn_kernel<T><<<dim3(a.M / kRedGnRows, a.N / 64), 256, 0, s>>>(a, sp.ws, sp.splits, sp.Mp, sp.Np);
    IRX_LAUNCH_CHECK();
  } else if (sp.splits > 1 && !sp.inkernel) {
    ProfScope ps(prof_on() ? std::string("irx::(anonymous namespace)::splitk_reduce_kernel<") + tn + ", " +
                                 (a.out_f32 ? "true" : "false") + ">"
                           : std::string(),
                 0.0, s);
    const long n = (long)a.M * (a.N / 8);
    dim3 g2((unsigned)((n + 255) / 256), a.batch);
    if (a.out_f32) splitk_reduce_kernel<T, true><<<g2, 256, 0, s>>>(a, sp.ws, sp.splits, sp.Mp, sp.Np);
    else splitk_reduce_kernel<T, false><<<g2, 256, 0, s>>>(a, sp.ws, sp.splits, sp.Mp, sp.Np);
    IRX_LAUNCH_CHECK();
  }
}

template <int BM, int BN, int WM, int WN, int BK, int S, int HALO = 0, bool PP = false>
void launch2(const GemmArgs& a, const Split& sp, hipStream_t s) {
  if constexpr (HALO == 4) launch2_t<bf16_t, BM, BN, WM, WN, BK, S, HALO, PP>(a, sp, s);   // (bf16 diagnostic build)
  else if (a.dtype == F16) launch2_t<f16_t, BM, BN, WM, WN, BK, S, HALO, PP>(a, sp, s);
  else launch2_t<bf16_t, BM, BN, WM, WN, BK, S, HALO, PP>(a, sp, s);
}

// ------------------------------------------------------------------ tile / split policy
constexpr int kCUs = 256;

struct Choice {
  int BM = 0, BN = 0, splits = 1, per = 0;
  bool small = false;   // 4-wave block, two resident per CU (short-K GEMMs: one block's prologue/epilogue
                        // overlaps the other's MFMA loop)
};

int step_k() { return g_gemm_deep == 1 ? 32 : 64; }   // K depth of one pipeline stage (eligibility granule)

// rows (M x batch) the policy plans for: image-indexed GEMMs at kCanonImages images (batch invariance)
long canon_rows(const GemmArgs& a) {
  const long rows = (long)a.M * a.batch;
  return a.imgs > 0 ? rows / a.imgs * kCanonImages : rows;
}
int canon_batch(const GemmArgs& a) { return (a.imgs > 0 && a.batch > 1) ? kCanonImages : a.batch; }

Choice choose(const GemmArgs& a) {
  Choice best;
  const int nk = a.K / step_k();
  if (g_gemm_small && g_gemm_deep == 0 && a.K <= g_gemm_small_kmax) {
    const int bn = (!a.geglu && a.N % 160 == 0) ? 160 : (a.N % 128 == 0 ? 128 : 0);
    if (bn) {
      best.BM = 128; best.BN = bn; best.small = true; best.splits = 1; best.per = nk;
      return best;
    }
  }
  if (g_gemm_force > 0 && g_gemm_deep == 0) {   // tuning sweeps: BM*100000 + BN*100 + splits
    const int BM = g_gemm_force / 100000, BN = (g_gemm_force / 100) % 1000, sp = g_gemm_force % 100;
    const bool ok = (BM == 256 || BM == 128 || (BM == 64 && BN == 320 && sp == 1 && !a.gn_part)) &&
                    (BN == 320 || BN == 256 || BN == 128) && a.N % BN == 0 &&
                    sp >= 1 && (sp == 1 || !((a.out_f32 && canon_batch(a) > 1) || a.geglu)) && (!a.geglu || BN % 128 == 0);
    if (ok) {
      best.BM = BM; best.BN = BN; best.splits = sp; best.per = (nk + sp - 1) / sp;
      if ((long)(sp - 1) * best.per < nk) return best;
    }
    best = Choice();
  }
  double best_score = -1.0;
  const int cands[7][2] = {{256, 320}, {256, 256}, {128, 320}, {256, 128}, {128, 256}, {128, 128}, {256, 160}};
  for (auto& c : cands) {
    const int BM = c[0], BN = c[1];
    if (BN == 160 && g_gemm_deep != 2) continue;
    if (BN == 320 && BM == 256 && (g_gemm_deep != 0 || !g_tile_256x320)) continue;
    if (a.N % BN != 0) continue;
    if (a.geglu && BN % 128 != 0) continue;      // tiles must hold whole (value, gate) block pairs
    const long tiles = (canon_rows(a) + BM - 1) / BM * (a.N / BN);
    // per-tile efficiency at full occupancy, calibrated on the batch-16 UNet / batch-8 VAE shapes
    // (scripts/gemm_sweep.py): the load path (L2 -> LDS-DMA) bounds the small tiles, 128x128 keeps two
    // blocks per CU resident (its prologue / epilogue overlap the other block's loop), 256x128 (4x2 waves)
    // loses to it everywhere measured
    const double eff = BM == 256 ? (BN >= 256 ? 1.0 : BN == 160 ? 0.9 : 0.65)
                                 : (BN == 320 ? 0.97 : BN == 256 ? 0.75 : 0.78);
    const int resident = (BM == 128 && BN == 128 && g_gemm_deep == 0) ? 2 : 1;
    const long cap = (long)kCUs * resident;
    for (int splits = 1; splits <= 8; splits *= 2) {
      if (splits > 1 && ((a.out_f32 && canon_batch(a) > 1) || a.geglu)) break;
      const int per = (nk + splits - 1) / splits;
      if (per * step_k() < 512 && splits > 1) break;    // keep >= 512 of K per split
      if ((long)(splits - 1) * per >= nk) break;        // no empty split
      const long blocks = tiles * splits;
      const double util = (double)blocks / ((double)((blocks + cap - 1) / cap) * cap);
      // split-K pays an fp32 partial write + read per split and a reduction tail, relatively more when
      // each split is short
      const double cost_split = splits > 1 ? (1.0 + 0.35 * std::log2((double)splits)) * (per < 16 ? 1.6 : 1.0) : 1.0;
      const double score = util * eff / cost_split;
      if (score > best_score + 1e-9) {
        best_score = score;
        best.BM = BM; best.BN = BN; best.splits = splits; best.per = per;
      }
    }
  }
  return best;
}

std::mutex g_ws_mu;
std::map<hipStream_t, unsigned*> g_cnt;   // per-stream split-K tickets (never freed: 256 KiB per stream)

unsigned* stream_counters(hipStream_t s) {
  std::lock_guard<std::mutex> lk(g_ws_mu);
  auto it = g_cnt.find(s);
  if (it != g_cnt.end()) return it->second;
  unsigned* p = nullptr;
  IRX_HIP(hipMalloc(&p, kSplitCounters * sizeof(unsigned)));
  IRX_HIP(hipMemset(p, 0, kSplitCounters * sizeof(unsigned)));   // synchronous: zero before any launch uses it
  g_cnt[s] = p;
  return p;
}
float* g_ws = nullptr;
size_t g_ws_bytes = 0;

float* internal_ws(size_t bytes) {
  std::lock_guard<std::mutex> lk(g_ws_mu);
  if (bytes > g_ws_bytes) {
    if (g_ws) IRX_HIP(hipFree(g_ws));
    g_ws = nullptr;
    IRX_HIP(hipMalloc(&g_ws, bytes));
    g_ws_bytes = bytes;
  }
  return g_ws;
}

bool vec_ok(const GemmArgs& a) {
  return !a.out_f32 && a.N % 8 == 0 && a.ldc % 8 == 0 && ((uintptr_t)a.C % 16) == 0 &&
         (!a.residual || (a.ldr % 8 == 0 && ((uintptr_t)a.residual % 16) == 0)) &&
         (a.batch == 1 || (a.sC % 8 == 0 && (!a.residual || a.sR % 8 == 0)));
}

bool eligible(const GemmArgs& a) {
  const int bk = step_k();
  if (!(g_large_mask & (a.conv ? 2 : 1))) return false;   // (A/B: large tiles for dense GEMMs / convs only)
  if (!a.conv && g_large_dense != 63) {   // (diagnostics: dense classes on large tiles)
    const int cls = a.geglu ? (a.K <= 320 ? 4 : a.K <= 640 ? 16 : 32) : a.hs_L ? 2 : a.N <= 1280 ? 1 : 8;
    if (!(g_large_dense & cls)) return false;
  }
  if (a.hs_L && !vec_ok(a)) return false;  // head-split stores: the 16-byte LDS-staged epilogue only
  if (a.act != ACT_NONE) return false;   // activations are fused by the 4-wave kernel only (tiny GEMMs)
  // the unrolled scalar (non-16-byte) epilogue only scales and adds bias: row add / residual need vec rows
  if (!vec_ok(a) && (a.rowadd || a.residual)) return false;
  if (a.rowadd && (a.rowadd_ld % 4 != 0 || ((uintptr_t)a.rowadd % 16) != 0)) return false;
  if (!is16(a.dtype) || a.K % bk != 0 || a.ldb % 8 != 0) return false;
  if (canon_rows(a) < 512) return false;           // tiny outputs: the 64x64 4-wave tiles waste less
  if (a.geglu && (a.out_f32 || a.residual || a.batch != 1 || a.N % 128 != 0)) return false;
  if (a.conv) return !a.out_f32 && a.g.C0 % bk == 0 && a.g.C1 % bk == 0;
  if (a.A1 && (a.batch != 1 || a.kA1 % 64 != 0 || a.lda1 % 8 != 0 || ((uintptr_t)a.A1 % 16) != 0)) return false;
  return a.lda % 8 == 0 && (a.batch == 1 || a.sA % 8 == 0);
}


}  // namespace

int g_large_dense = 63;  // irx_set_option("large_dense", m): dense classes on large tiles: 1 N <= 1280, 2 head-split,
                         // GEGLU at K 4: 320, 16: 640, 32: >= 1280, 8 other
int g_gemm_nmajor = 1;
int g_large_mask = 3;  // irx_set_option("large_mask", m): bit 0 dense GEMMs, bit 1 convs take the large tiles
int g_gemm_deep = 0;   // irx_set_option("gemm_deep", m): 0 two-stage BK 64, 1 BK-32 ring, 2 BK-64 3/4-stage ring
int g_gemm_dbg = 0;
bool g_gemm_small = false;   // irx_set_option("gemm_small", 1): 4-wave 128x160 / 128x128 tiles for K <= kmax
int g_gemm_small_kmax = 1280;
bool g_splitk_inkernel = true;   // irx_set_option("splitk_inkernel", 0): separate split-K reduce kernel (A/B)
bool g_tile_256x320 = true;      // irx_set_option("tile_256x320", 0): no 256x320 tiles (A/B)
int g_conv_halo = 1;             // irx_set_option("conv_halo", m): 0 im2col walk for every conv (A/B),
                                 // 1 halo tiles where the grid fills the chip, 2 wherever they fit (tests)
int g_gemm_force = 0;            // irx_set_option("gemm_force", BM*100000 + BN*100 + splits): tuning sweeps

int g_gn_fuse = 0;   // measured slower: the halo normalisation's VALU work does not hide under the MFMAs
int halo_bn(const GemmArgs& a);

int halo_mode(const GemmArgs& a);
int halo_split_count(const GemmArgs& a, int hbn);

bool gemm_gn_fusable(const GemmArgs& a) {   // (the lock-step halo loop, HALO == 1: 160-wide row tiles only)
  return g_gn_fuse && g_large_tiles && is16(a.dtype) && eligible(a) && halo_bn(a) == 160 && halo_mode(a) == 1;
}

int g_conv1x1_dense = 1;   // irx_set_option("conv1x1_dense", 0): 1x1 convs on the im2col conv path (A/B)

bool conv1x1_as_dense(GemmArgs& a) {
  const ConvGeom& g = a.g;
  if (!g_conv1x1_dense || !a.conv || !is16(a.dtype) || a.batch != 1 || a.gn_ab || a.up2_w || a.act != ACT_NONE) return false;
  if (g.KH != 1 || g.KW != 1 || g.stride != 1 || g.pad_t != 0 || g.pad_l != 0) return false;
  if (g.Hv != g.Hin || g.Wv != g.Win || g.Ho != g.Hin || g.Wo != g.Win) return false;
  GemmArgs d = a;
  d.conv = 0;
  d.g = ConvGeom();
  d.A = g.src0; d.lda = g.C0;
  d.A1 = g.C1 ? g.src1 : nullptr; d.lda1 = g.C1; d.kA1 = g.C1 ? g.C0 : 0;
  if (!g_large_tiles || !eligible(d) || choose(d).BM == 0) return false;
  a = d;
  return true;
}

int g_gn_parts = 1;
int g_gn_red_parts = 1;   // irx_set_option("gn_red_parts", 0): split-K reduce kernels do not emit GroupNorm partials (A/B)

int gemm_emits_gn_parts(const GemmArgs& a) {
  if (!g_gn_parts || !g_large_tiles || !is16(a.dtype) || !eligible(a) || !vec_ok(a)) return 0;
  if (a.geglu || a.hs_L || a.batch != 1 || a.out_f32) return 0;
  if (halo_bn(a)) {
    if (halo_mode(a) == 3)   // (8x8 images, K splits reduced by splitk_reduce_gn_kernel: one partial per image)
      return (g_gn_red_parts && !a.up2_w && halo_split_count(a, 160) > 1 && a.M % kRedGnRows == 0 && a.N % 64 == 0 && a.act == ACT_NONE && !a.b_rows) ? kRedGnRows
                                                                                                            : 0;
    return a.M % 256 == 0 ? 256 : 0;
  }
  const Choice c = choose(a);
  if (c.BM == 0) return 0;
  if (c.splits > 1) {   // the in-kernel split-K reduction runs the epilogue; the separate reduce kernel emits them too
    const long tiles = (long)((a.M + c.BM - 1) / c.BM) * ((a.N + c.BN - 1) / c.BN);
    if (!(g_splitk_inkernel && c.splits == 2 && tiles <= kSplitCounters))   // splitk_reduce_gn_kernel
      // (splitk_reduce_gn_kernel applies one bias vector and assumes the plain m * ldc layout: no per-image
      // weights / bias)
      return (g_gn_red_parts && !a.up2_w && !a.b_rows && !c.small && c.BM != 64 && a.M % kRedGnRows == 0 && a.N % 64 == 0 && a.act == ACT_NONE)
                 ? kRedGnRows : 0;
  }
  if (a.up2_w && ((long)a.up2_h * a.up2_w) % c.BM) return 0;   // (a sub-pixel tile's rows in one image)
  return a.M % c.BM ? 0 : c.BM;
}

bool gemm_up2_ok(const GemmArgs& a) {
  // every store of the large-tile path goes through c_off (the 16-byte epilogue, the split-K reduce kernel); the
  // scalar epilogue and the 4-wave kernel do not map rows
  // (the halo parity convs, HALO == 6 / 7, store through c_off too)
  return g_large_tiles && eligible(a) && vec_ok(a) && a.batch == 1 && !a.hs_L &&
         (halo_bn(a) || (!gemm_sk_eligible(a) && choose(a).BM != 0));
}

// Split-K partials of the 4-wave kernel (gemm.hip, small-M GEMMs) reduced with the large-tile path's kernel: the
// same fp32 sums over the splits in order, then alpha / bias / row add / activation / residual / output scale
float* splitk_scratch(size_t bytes) { return internal_ws(bytes); }

void splitk_reduce(const GemmArgs& a, const float* ws, int splits, int Mp, int Np, hipStream_t s) {
  IRX_CHECK(a.N % 8 == 0 && a.batch == 1 && is16(a.dtype), "splitk_reduce: 16-bit, N % 8 == 0, batch 1");
  const char* tn = a.dtype == F16 ? "_Float16" : "unsigned short";
  ProfScope ps(prof_on() ? std::string("irx::(anonymous namespace)::splitk_reduce_kernel<") + tn + ", " +
                               (a.out_f32 ? "true" : "false") + ">"
                         : std::string(),
               0.0, s);
  const long n = (long)a.M * (a.N / 8);
  const dim3 g2((unsigned)((n + 255) / 256), 1);
  if (a.dtype == F16) {
    if (a.out_f32) splitk_reduce_kernel<f16_t, true><<<g2, 256, 0, s>>>(a, ws, splits, Mp, Np);
    else splitk_reduce_kernel<f16_t, false><<<g2, 256, 0, s>>>(a, ws, splits, Mp, Np);
  } else {
    if (a.out_f32) splitk_reduce_kernel<bf16_t, true><<<g2, 256, 0, s>>>(a, ws, splits, Mp, Np);
    else splitk_reduce_kernel<bf16_t, false><<<g2, 256, 0, s>>>(a, ws, splits, Mp, Np);
  }
  IRX_LAUNCH_CHECK();
}

int g_gemm_pp_chain = 1;   // irx_set_option("gemm_pp_chain", 0): the two-source 1x1 chains on the two-stage loop (A/B)

int g_ln_fold = 1;

bool gemm_ln_foldable(const GemmArgs& a) {
  if (!g_large_tiles || !is16(a.dtype) || a.conv || a.alpha != 1.f || a.out_f32 || a.batch != 1) return false;
  if (!eligible(a) || !vec_ok(a)) return false;
  const Choice c = choose(a);
  if (c.BM == 0) return false;
  if (c.splits > 1) {   // only the in-kernel reduction runs the full epilogue
    const long tiles = (long)((a.M + c.BM - 1) / c.BM) * ((a.N + c.BN - 1) / c.BN);
    if (!(g_splitk_inkernel && c.splits == 2 && tiles <= kSplitCounters)) return false;
  }
  return true;
}

int g_ln_parts = 1;

// The epilogue can emit LayerNorm partials (GemmArgs::ln_out): dense 16-bit large-tile GEMMs whose tiles are 320
// columns wide (the 64x64 / 32x32-level transformer projections), run by the large-tile kernel's staged epilogue
bool gemm_emits_ln_parts(const GemmArgs& a) {
  if (!g_ln_parts || !g_large_tiles || !is16(a.dtype) || a.conv || a.geglu || a.hs_L || a.batch != 1 || a.out_f32) return false;
  if (a.gn_part || a.N % kLnGroup != 0 || !eligible(a) || !vec_ok(a) || gemm_sk_eligible(a)) return false;
  if (a.ln_out_rs && a.N != kLnGroup) return false;
  const Choice c = choose(a);
  if (c.BN != kLnGroup || c.small || (c.BM != 256 && c.BM != 128)) return false;
  if (c.splits > 1) {   // only the in-kernel reduction runs the full epilogue
    const long tiles = (long)((a.M + c.BM - 1) / c.BM) * ((a.N + c.BN - 1) / c.BN);
    if (!(g_splitk_inkernel && c.splits == 2 && tiles <= kSplitCounters)) return false;
  }
  return g_gemm_pp != 1 && g_gemm_deep == 0;
}

int g_gn_fold = 1;

// Per-image B / bias (GemmArgs::b_rows): dense 16-bit large tiles whose row tiles never straddle two images
bool gemm_bimg_ok(const GemmArgs& a) {
  if (!g_large_tiles || !is16(a.dtype) || a.conv || a.geglu || a.batch != 1 || a.out_f32 || a.b_rows <= 0) return false;
  if (a.M % a.b_rows || !eligible(a) || !vec_ok(a) || gemm_sk_eligible(a)) return false;
  const Choice c = choose(a);
  if (c.BM == 0 || c.small || a.b_rows % c.BM) return false;
  if (c.splits > 1) {   // partial sums of one tile share one image's weights; the reduce kernel indexes the bias by row
    const long tiles = (long)((a.M + c.BM - 1) / c.BM) * ((a.N + c.BN - 1) / c.BN);
    if (!(g_splitk_inkernel && c.splits == 2 && tiles <= kSplitCounters)) return false;
  }
  return g_gemm_pp != 1 && g_gemm_deep == 0;
}

int halo_splits(const GemmArgs& a, long tiles);

// K splits the large-tile path would run `a` with (1: none; 0: not a large-tile shape) — for tests / diagnostics
int gemm_large_splits(const GemmArgs& a) {
  if (!g_large_tiles || !eligible(a) || gemm_sk_eligible(a)) return 0;
  if (const int hbn = halo_bn(a)) return halo_split_count(a, hbn);
  const Choice c = choose(a);
  return c.BM ? c.splits : 0;
}

bool gemm_geglu_fusable(const GemmArgs& a) {
  if (!g_large_tiles || !a.geglu || !eligible(a) || !vec_ok(a)) return false;
  if (gemm_sk_eligible(a)) return true;
  // (round 3 kept partial per-image row tiles unfused after an fp16 batch dependence; its cause was hipcc fusing the
  // folded-LayerNorm FMA with the fp16 conversion into v_fma_mixlo_f16 at some unrolled sites only — fixed in
  // irx_common.h f16_src, tests/test_ln_parts_gpu.py::test_ln_fold_geglu_fp16_batch_invariant)
  return choose(a).BM != 0;
}

int halo_bn(const GemmArgs& a);

int halo_splits(const GemmArgs& a, long tiles);

// Tile order of a halo conv (GemmArgs::group_m; scheduling only, no numeric effect).  One XCD runs q = tiles / 8
// consecutive logical tiles at once; in the M-major order they are q / tiles_n M tiles x all tiles_n N tiles, so at
// the 16x16 level (16 M tiles x 8 N tiles of a 1280-channel conv, 29.5 MB of weights) every XCD streams all of B.
// Grouped by g M tiles the range is g x q / g: per XCD ~ g halo slabs of A + q / g B panels (bytes (BM + 2W) Cin 2
// and BN K 2).  g minimises that sum; 0 keeps the M-major order when it is within 10 % of the best.
int g_halo_group = 1;   // irx_set_option("halo_group", 0): M-major halo tile order (A/B)
int halo_group_m(const GemmArgs& a, int bn) {
  if (!g_halo_group) return 0;
  const long tiles_m = (a.M + 255) / 256, tiles_n = a.N / bn;
  if (tiles_n < 2) return 0;
  // logical tiles per XCD (xcd_remap ranges), of which one block per CU = 32 run at a time
  const long q = (tiles_m * tiles_n + 7) / 8, w = std::min(q, 32L);
  const double hpix = halo_mode(a) == 2 ? 10.0 * (kStripW + 2) : 256.0 + 2.0 * a.g.Wo;   // halo pixels per tile
  const double a_m = hpix * (a.g.C0 + a.g.C1) * 2.0, b_n = (double)bn * a.K * 2.0;
  auto cost = [&](long g) {   // A + B bytes of one XCD's w co-resident tiles in groups of g M tiles
    const bool whole = w >= g * tiles_n;   // (the window spans whole groups: w / tiles_n M tiles x every N tile)
    const long gm = whole ? (w + tiles_n - 1) / tiles_n : std::min(g, w);
    const long gn = whole ? tiles_n : (w + g - 1) / g;
    return gm * a_m + gn * b_n;
  };
  const double legacy = cost(std::max(1L, (w + tiles_n - 1) / tiles_n));   // M-major: w / tiles_n whole M rows
  long best_g = 0;
  double best = legacy;
  for (long g = 1; g <= tiles_m; g *= 2)
    if (cost(g) < best) { best = cost(g); best_g = g; }
  return best < 0.9 * legacy ? (int)best_g : 0;
}

// Tile order of a dense large-tile GEMM (scheduling only): the cost model of halo_group_m with A panel BM x K and B
// panel BN x K, over the 32 x `resident` tiles one XCD runs at once; 0 keeps the M-major / N-major order when the
// grouped one is not > 10 % better.  (The GEGLU projections at 32^2 / 16^2: every XCD streamed the whole 6.5 / 26 MB
// weight in the M-major / N-major orders.)
int g_gemm_group = 1;   // irx_set_option("gemm_group", 0): the M-major / N-major dense tile orders only (A/B)
int dense_group_m(const GemmArgs& a, int bm, int bn, int resident, bool nmajor) {
  if (!g_gemm_group) return 0;
  const long tiles_m = (a.M + bm - 1) / bm, tiles_n = (a.N + bn - 1) / bn;
  if (tiles_n < 2 || tiles_m < 2) return 0;
  const long q = (tiles_m * tiles_n + 7) / 8, w = std::min(q, 32L * resident);
  const double a_m = (double)bm * a.K * 2.0, b_n = (double)bn * a.K * 2.0;
  auto cost = [&](long g) {
    const bool whole = w >= g * tiles_n;
    const long gm = whole ? (w + tiles_n - 1) / tiles_n : std::min(g, w);
    const long gn = whole ? tiles_n : (w + g - 1) / g;
    return gm * a_m + gn * b_n;
  };
  // the current order: M-major = groups of one whole M row block; N-major = a window of w M tiles x w / tiles_m N tiles
  const double legacy = nmajor ? std::min(w, tiles_m) * a_m + (double)((w + tiles_m - 1) / tiles_m) * b_n
                               : cost(std::max(1L, (w + tiles_n - 1) / tiles_n));
  long best_g = 0;
  double best = legacy;
  for (long g = 1; g <= tiles_m; g *= 2)
    if (cost(g) < best) { best = cost(g); best_g = g; }
  return best < 0.9 * legacy ? (int)best_g : 0;
}

size_t gemm_workspace_bytes(const GemmArgs& a) {
  if (!g_large_tiles || !eligible(a)) return 0;
  if (const int hbn = halo_bn(a)) {
    const int sp = halo_split_count(a, hbn);
    return sp > 1 ? (size_t)sp * ((a.M + 255) / 256 * 256) * a.N * sizeof(float) : 0;
  }
  const Choice c = choose(a);
  if (c.BM == 0 || c.splits <= 1) return 0;
  return (size_t)c.splits * a.batch * ((a.M + c.BM - 1) / c.BM * c.BM) * ((a.N + c.BN - 1) / c.BN * c.BN) *
         sizeof(float);
}

// K splits of a halo conv (whole 64-channel slabs per split): 1 when the tiles fill the chip, 2 (in-kernel
// reduction) when two splits do, 0 = the halo path does not take the shape.
int g_halo_split = 1;   // irx_set_option("halo_split", 0): no K-split halo tiles (A/B)
int g_halo_pipe = 1;    // irx_set_option("halo_pipe", 0): the round-2 halo main loop (A/B)
// irx_set_option("gemm_pp", m): ping-pong main loops.  2 (default): the lean dense form on 256x256 tiles only (the
// 32x32 / 16x16-level GEGLU projections: ff1 -12 / -14 % at the kbench shapes, 49.9 -> 46.5 ms/step in the bench;
// profiles/r04_kbench_gemm_pp_lean.txt); 1: every dense / im2col tile (the im2col convs keep the round-3 branchy form,
// which is slower there, and the lean form loses at 128x128 / 1280-wide 16x16 shapes); 3: 256x256 + 256x320 (measured
// 513.7 vs 508.2 ms/step: off); 0: none
int g_gemm_pp = 2;

int halo_splits(const GemmArgs& a, long tiles) {
  if (tiles >= kCUs || g_conv_halo >= 2) return 1;
  if (!g_halo_split) return 0;
  const int slabs = (a.g.C0 + a.g.C1) / 64;
  if (g_splitk_inkernel && 2 * tiles >= kCUs && slabs >= 8 && tiles <= kSplitCounters) return 2;
  return 0;
}

// irx_set_option("halo_strip", m): 0 no strip tiles (VAE / 768^2 convs on the im2col walk, A/B), 1 (default) strip
// tiles where whole-row tiles do not fit (W > 64 or no power of two), 2 strip tiles wherever the shape allows (tests:
// strips == rows bit for bit at W <= 64)
int g_halo_strip = 1;
int g_halo_up2 = 1;   // irx_set_option("halo_up2", 0): upsampler parity convs on the im2col walk (A/B)
int g_halo_mi = 1;    // irx_set_option("halo_mi", 0): the 8x8-level convs on the im2col walk (A/B)

// Halo tile mode of a 3x3 / stride-1 / pad-1 conv, or of one parity's 2x2 conv of a nearest-2x upsampler
// (GemmArgs::up2_*, pad (1 - a, 1 - b)): 1 = 256-pixel tiles of whole image rows (W in {16, 32, 64}), 2 = 8 x 32
// strip tiles (W % 32 == 0, H % 8 == 0; HALO == 5 / 7), 0 = neither.  The decision does not depend on the parity.
int halo_mode(const GemmArgs& a) {
  const ConvGeom& g = a.g;
  if (!g_conv_halo || !a.conv || a.batch != 1 || a.geglu || a.out_f32 || !vec_ok(a)) return 0;
  if (g.stride != 1) return 0;
  if (a.up2_w) {   // (ping-pong loop only)
    if (!g_halo_up2 || !g_halo_pipe || a.gn_ab || g.KH != 2 || g.KW != 2 || (g.pad_t & ~1) || (g.pad_l & ~1)) return 0;
  } else if (g.KH != 3 || g.KW != 3 || g.pad_t != 1 || g.pad_l != 1) {
    return 0;
  }
  if (g.Hv != g.Hin || g.Wv != g.Win || g.Ho != g.Hin || g.Wo != g.Win) return 0;
  if (g.C0 % 64 || g.C1 % 64 || g.C0 <= 0) return 0;
  const int W = g.Win;
  if ((long)g.N * g.Hin * W != a.M) return 0;
  // 3 = four whole 8x8 images per tile (HALO == 8): any image count (a partial last tile), so the choice is
  // batch-invariant like the others
  if (W == 8 && g.Hin == 8 && g_halo_mi && g_halo_pipe && !a.gn_ab && a.M % 64 == 0) return 3;
  // (parity convs on row / strip tiles: whole 256-row tiles of one image, the sub-pixel GroupNorm partial blocks)
  if (a.up2_w && ((long)a.up2_h * a.up2_w) % 256) return 0;
  if (a.M % 256) return 0;
  const bool rows = W >= 16 && W <= kHaloWMax && !(W & (W - 1)) && 256 % W == 0 && g.Hin % (256 / W) == 0;
  // (strips: the ping-pong loop only, no GroupNorm-fused operand)
  const bool strips = g_halo_strip && g_halo_pipe && !a.gn_ab && W % kStripW == 0 && g.Hin % (256 / kStripW) == 0;
  if (strips && (g_halo_strip == 2 || !rows)) return 2;
  return rows ? 1 : 0;
}

// Halo tile (BN) for a 3x3 / stride-1 / pad-1 conv on halo tiles (halo_mode) whose grid fills the chip (alone or with
// two K splits); 0 = not applicable.  BN 160 (UNet widths), else 128 (VAE widths 128 / 256 / 512; ping-pong loop only)
int halo_bn(const GemmArgs& a) {
  const int mode = halo_mode(a);
  if (!mode) return 0;
  const int bn = a.N % 160 == 0 ? 160 : (a.N % 128 == 0 && g_halo_pipe && !a.gn_ab) ? 128 : 0;
  if (mode == 3) return bn == 160 ? 160 : 0;   // (HALO == 8 instantiated at BN 160: the UNet's 1280 channels)
  if (!bn || !halo_splits(a, canon_rows(a) / 256 * (a.N / bn))) return 0;
  if (a.up2_w && mode == 2 && bn != 128) return 0;   // (strip parity convs: the VAE widths only, HALO == 7 at BN 128)
  // (GroupNorm-fused operand: one 512-element chunk of the (256 + 2W) x 8 halo per tap, taps 3..8)
  static_assert((256 + 2 * kHaloWMax) * 8 <= 512 * 6, "halo normalisation chunks");
  return bn;
}

// K splits of a halo conv: halo_splits (1 or 2, in-kernel reduction), or for the 8x8 images (mode 3) whole slabs per
// split for about one block per CU (the canonical 16 images: 4 row tiles x N / 160), reduced by the separate kernel
int halo_split_count(const GemmArgs& a, int hbn) {
  if (halo_mode(a) != 3) return halo_splits(a, canon_rows(a) / 256 * (a.N / hbn));
  const long tiles = (canon_rows(a) + 255) / 256 * (a.N / hbn);
  const int slabs = (a.g.C0 + a.g.C1) / 64;
  const int want = (int)std::max(1L, std::min(8L, (long)kCUs / std::max(1L, tiles)));
  const int per = (slabs + want - 1) / want;
  return (slabs + per - 1) / per;
}

// Returns false (caller uses the 4-wave kernel) when the shape does not fit the large-tile path.
bool gemm_large_tile(const GemmArgs& a, hipStream_t s) {
  if (!eligible(a)) return false;
  IRX_CHECK(!a.gn_ab || halo_bn(a), "GroupNorm-fused operand needs the halo conv path");
  IRX_CHECK(!a.gn_part || gemm_emits_gn_parts(a), "GroupNorm partials need the large-tile epilogue");
  IRX_CHECK(!(a.ln_rs || a.ln_part) || gemm_ln_foldable(a), "folded LayerNorm needs the large-tile epilogue");
  IRX_CHECK(!a.ln_out || gemm_emits_ln_parts(a), "LayerNorm partials need the large-tile epilogue");
  IRX_CHECK(!a.b_rows || gemm_bimg_ok(a), "per-image weights need the large-tile path");
  if (gemm_sk(a, s)) return true;   // K = 320 streaming path (gemm_sk.hip)
  if (const int hbn = halo_bn(a)) {
    GemmArgs b = a;
    b.vec_epilogue = 1;
    b.dbg = g_gemm_dbg;
    b.group_m = halo_group_m(a, hbn);
    Split sp;
    sp.per = a.K / 64;
    const int splits = halo_split_count(a, hbn);
    const int ntap = a.up2_w ? 4 : 9;
    const bool mi = halo_mode(a) == 3;
    if (splits > 1) {   // whole slabs per split, in-kernel last-arriver reduction (fp32 partials; 8x8: reduce kernel)
      const int slabs = (a.g.C0 + a.g.C1) / 64;
      sp.splits = splits;
      sp.per = ntap * ((slabs + splits - 1) / splits);
      sp.Mp = (a.M + 255) / 256 * 256;   // (whole row tiles of partials: a partial last tile stores all its rows)
      sp.Np = a.N;
      const size_t need = (size_t)splits * sp.Mp * a.N * sizeof(float);
      sp.ws = (a.splitk_ws && a.splitk_ws_bytes >= need) ? (float*)a.splitk_ws : internal_ws(need);
      sp.inkernel = !mi;
      if (sp.inkernel) sp.cnt = stream_counters(s);
    }
#ifdef IRX_HALO_DIAG
    if (g_halo_pipe && !a.gn_ab && b.dbg && a.dtype == BF16) launch2<256, 160, 4, 2, 64, 3, 4>(b, sp, s);   // (diagnostics)
    else
#endif
    if (mi) {                           // four 8x8 images per tile (parity convs: 4 taps)
      if (a.up2_w) launch2<256, 160, 4, 2, 64, 3, 9>(b, sp, s);
      else launch2<256, 160, 4, 2, 64, 3, 8>(b, sp, s);
    } else if (a.up2_w) {               // upsampler parity convs: 4 taps per slab
      if (halo_mode(a) == 2) launch2<256, 128, 4, 2, 64, 3, 7>(b, sp, s);
      else if (hbn == 160) launch2<256, 160, 4, 2, 64, 3, 6>(b, sp, s);
      else launch2<256, 128, 4, 2, 64, 3, 6>(b, sp, s);
    } else if (halo_mode(a) == 2) {     // strip tiles (ping-pong main loop)
      if (hbn == 160) launch2<256, 160, 4, 2, 64, 3, 5>(b, sp, s);
      else launch2<256, 128, 4, 2, 64, 3, 5>(b, sp, s);
    } else if (g_halo_pipe && !a.gn_ab) {   // ping-pong main loop
      if (hbn == 160) launch2<256, 160, 4, 2, 64, 3, 2>(b, sp, s);
      else launch2<256, 128, 4, 2, 64, 3, 2>(b, sp, s);
    } else {
      launch2<256, 160, 4, 2, 64, 3, 1>(b, sp, s);
    }
    return true;
  }
  const Choice c = choose(a);
  if (c.BM == 0) return false;
  GemmArgs b = a;
  b.vec_epilogue = vec_ok(a);
  b.dbg = g_gemm_dbg;
  // tile order (scheduling only, no numeric effect): N-major when the weights outweigh the activation rows, so that an
  // XCD's consecutive tiles re-use one B panel from its L2 instead of every XCD streaming all of B
  b.nmajor = g_gemm_nmajor == 2 || (g_gemm_nmajor == 1 && (long)a.N * a.batch > (long)a.M * a.batch);
  if (a.batch == 1 && !a.hs_L) {   // grouped order where it cuts an XCD's co-resident A + B bytes (GemmArgs::group_m)
    b.group_m = dense_group_m(a, c.BM, c.BN, (c.BM == 128 && c.BN == 128) || c.small ? 2 : 1, b.nmajor);
    if (b.group_m) b.nmajor = 0;
  }
  if (a.geglu && !b.vec_epilogue) return false;
  Split sp;
  sp.splits = c.splits;
  sp.per = c.per;
  if (c.splits > 1) {
    if (!b.vec_epilogue && !a.out_f32) return false;     // reduce kernel needs 16-byte output rows
    if (a.out_f32 && (a.ldc % 8 != 0 || a.N % 8 != 0)) return false;
    sp.Mp = (a.M + c.BM - 1) / c.BM * c.BM;
    sp.Np = (a.N + c.BN - 1) / c.BN * c.BN;
    const size_t need = (size_t)c.splits * a.batch * sp.Mp * sp.Np * sizeof(float);
    sp.ws = (a.splitk_ws && a.splitk_ws_bytes >= need) ? (float*)a.splitk_ws : internal_ws(need);
    const long tiles = (long)((a.M + c.BM - 1) / c.BM) * ((a.N + c.BN - 1) / c.BN) * a.batch;
    // in-kernel reduction wins at 2 splits; with more, the serial last-arriver tail loses to the reduce kernel
    sp.inkernel = g_splitk_inkernel && c.splits == 2 && tiles <= kSplitCounters;
    if (sp.inkernel) sp.cnt = stream_counters(s);
  } else {
    sp.per = a.K / step_k();
  }
  if (c.BM == 64) {   // 64x320, 4 waves, BK 32, two stages (48 KiB of LDS: three blocks per CU)
    sp.per = a.K / 32;
    launch2<64, 320, 1, 4, 32, 2>(b, sp, s);
    return true;
  }
  if (c.small) {
    if (c.BN == 160) launch2<128, 160, 2, 2, 64, 2>(b, sp, s);
    else launch2<128, 128, 2, 2, 64, 2>(b, sp, s);
  } else if (g_gemm_deep == 0 &&
             (!a.A1 || g_gemm_pp_chain) &&   // (two-source A: the lean dense form only, a.conv == 0)
             (g_gemm_pp == 1 ||
              (g_gemm_pp >= 2 && !a.conv && !a.ln_out && !a.b_rows &&
               ((c.BM == 256 && (c.BN == 256 || (g_gemm_pp == 3 && c.BN == 320))) ||
                // the long-K two-source 1x1 convs (proj_out o ff.net.2 over (h | g), K = 5C): the ping-pong loop pays
                // where the K loop is long (unlike the K = 320 / 640 projections, which stay on the two-stage loop)
                (a.A1 && g_gemm_pp_chain && c.BN == 320 && (c.BM == 256 || c.BM == 128) && a.K >= 1024)))) &&
             (a.conv || (a.M % c.BM == 0 && a.N % c.BN == 0))) {
    // ping-pong schedule: 3 stages (BK 32 where BK 64 would not fit); dense GEMMs on whole tiles only (the lean form)
    const int key = c.BM * 1000 + c.BN;
    if (key == 256320 || key == 256256 || key == 128320) sp.per *= 2;   // K steps of 32
    switch (key) {
      case 256320: launch2<256, 320, 2, 4, 32, 3, 0, true>(b, sp, s); break;
      case 256256: launch2<256, 256, 2, 4, 32, 3, 0, true>(b, sp, s); break;
      case 128320: launch2<128, 320, 2, 4, 32, 3, 0, true>(b, sp, s); break;
      case 256128: launch2<256, 128, 4, 2, 64, 3, 0, true>(b, sp, s); break;
      case 128256: launch2<128, 256, 2, 4, 64, 3, 0, true>(b, sp, s); break;
      case 128128: launch2<128, 128, 2, 4, 64, 3, 0, true>(b, sp, s); break;
      default: return false;
    }
  } else if (g_gemm_deep == 2) {   // BK 64; a third (fourth) stage wherever it fits in 160 KiB
    switch (c.BM * 1000 + c.BN) {
      case 256256: launch2<256, 256, 2, 4, 64, 2>(b, sp, s); break;
      case 128320: launch2<128, 320, 2, 4, 64, 2>(b, sp, s); break;
      case 256128: launch2<256, 128, 4, 2, 64, 3>(b, sp, s); break;
      case 128256: launch2<128, 256, 2, 4, 64, 3>(b, sp, s); break;
      case 128128: launch2<128, 128, 2, 4, 64, 4>(b, sp, s); break;
      case 256160: launch2<256, 160, 4, 2, 64, 3>(b, sp, s); break;
      default: return false;
    }
  } else if (g_gemm_deep == 1) {
    switch (c.BM * 1000 + c.BN) {
      case 256256: launch2<256, 256, 2, 4, 32, 4>(b, sp, s); break;
      case 128320: launch2<128, 320, 2, 4, 32, 5>(b, sp, s); break;
      case 256128: launch2<256, 128, 4, 2, 32, 5>(b, sp, s); break;
      case 128256: launch2<128, 256, 2, 4, 32, 5>(b, sp, s); break;
      case 128128: launch2<128, 128, 2, 4, 32, 6>(b, sp, s); break;
      default: return false;
    }
  } else {
    switch (c.BM * 1000 + c.BN) {
      case 256320: launch2<256, 320, 2, 4, 64, 2>(b, sp, s); break;
      case 256256: launch2<256, 256, 2, 4, 64, 2>(b, sp, s); break;
      case 128320: launch2<128, 320, 2, 4, 64, 2>(b, sp, s); break;
      case 256128: launch2<256, 128, 4, 2, 64, 2>(b, sp, s); break;
      case 128256: launch2<128, 256, 2, 4, 64, 2>(b, sp, s); break;
      case 128128: launch2<128, 128, 2, 4, 64, 2>(b, sp, s); break;
      default: return false;
    }
  }
  return true;
}

}  // namespace irx
