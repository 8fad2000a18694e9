// irx — host-side launchers for the hand-written gfx950 kernels.
// Every activation is NHWC ([N][H][W][C], C fastest); weights are [Cout][KH][KW][Cin] (K-contiguous).
#pragma once
#include "irx_common.h"

namespace irx {

// ------------------------------------------------------------ implicit-GEMM convolution / GEMM
// A operand either a dense row-major matrix or an NHWC image gathered on the fly (3x3 / 1x1 convs,
// stride 1/2, asymmetric zero padding, fused nearest-neighbour upsample, fused channel concat of two
// sources).  B = weights [N][K] with K contiguous.  C[m][n] = epilogue(sum_k A[m][k] B[n][k]).
struct ConvGeom {
  const void* src0 = nullptr;   // NHWC, C0 channels
  const void* src1 = nullptr;   // optional second NHWC source (channel concat), C1 channels
  int C0 = 0, C1 = 0;
  int N = 0, Hin = 0, Win = 0;  // stored input size
  int Hv = 0, Wv = 0;           // virtual input size after nearest resize (== Hin/Win if none)
  int KH = 1, KW = 1, stride = 1, pad_t = 0, pad_l = 0;
  int Ho = 0, Wo = 0;
};

struct GemmArgs {
  int dtype = BF16;       // storage type of A, B, residual and (unless out_f32) C
  int M = 0, N = 0, K = 0;
  int conv = 0;           // 1: A is an implicit im2col of `g`
  ConvGeom g;
  const void* A = nullptr; long lda = 0; long sA = 0;    // dense A (+ batch stride)
  // dense A's second source (a 1x1 conv over a channel concat, conv1x1_as_dense): A[m][k] = A1[m][k - kA1] for
  // k >= kA1 (kA1 a multiple of the K step; batch 1; the generic large-tile loops only)
  const void* A1 = nullptr; long lda1 = 0; int kA1 = 0;
  const void* B = nullptr; long ldb = 0; long sB = 0;
  void* C = nullptr; long ldc = 0; long sC = 0;
  int out_f32 = 0;        // C stored as fp32 regardless of dtype
  float alpha = 1.f;
  const float* bias = nullptr;                  // [N]
  const float* rowadd = nullptr; long rowadd_ld = 0; int rows_per_group = 1;  // += rowadd[(m/rpg)*ld + n]
  const void* residual = nullptr; long ldr = 0; long sR = 0;                  // += residual[m][n] (dtype)
  float out_scale = 1.f;
  int act = ACT_NONE;     // applied after bias/rowadd, before residual
  int batch = 1;
  // images spanned by the M x batch rows (0: not image-indexed).  Tile / split-K / kernel choices are made for
  // the canonical kCanonImages images, so an image's bits never depend on how many images share its batch.
  int imgs = 0;
  int vec_epilogue = 0;   // set by the launcher: 16-byte LDS-staged output path is legal for this call
  // GEGLU epilogue: B rows interleaved in (64 value, 64 gate) blocks (IRX_LAYOUT_*_GEGLU64); C gets N/2
  // columns h * gelu(g).  Only the large-tile path fuses it (gemm_geglu_fusable); else see geglu().
  int geglu = 0;
  // head-split output (attention operands): columns are `parts` blocks of hs_C = heads x hs_d, rows are images of
  // hs_L tokens; element (m, n) is stored at part * (M * hs_C) + ((image * heads + head) * hs_L + token) * hs_d + e,
  // i.e. [part][image][head][token][e] (0: plain row-major with ldc)
  int hs_L = 0, hs_C = 0, hs_d = 0;
  // GroupNorm(+SiLU) applied to the conv's A operand on the fly (halo path only, gemm_gn_fusable): source
  // channel c of image n becomes gn_act(x, gn_ab[n][c].x, gn_ab[n][c].y, gn_silu); c indexes the C0 + C1
  // concat.  Zero padding stays zero (it pads the normalised tensor, as in the unfused form).
  const float2* gn_ab = nullptr; int gn_silu = 0;
  // GroupNorm statistics of the OUTPUT emitted by the epilogue: per block of R output rows (R = the tile's BM,
  // gemm_emits_gn_parts) and per output channel, the (sum, sum of squares) of the stored values as double2 at
  // gn_part[(m / R) * N + n] (shifted fp32 sums per thread, fp64 merge: gn_stats3's arithmetic)
  double* gn_part = nullptr;
  // LayerNorm of the A rows folded into the product (16-bit transformer projections, gemm_ln_foldable): B holds
  // W * gamma (columns scaled), `bias` holds bias + W beta, and the epilogue forms
  //   y[m][n] = ln_rs[m].x * acc[m][n] - ln_rs[m].y * ln_u[n] + bias[n]
  // with ln_rs[m] = (rstd, rstd * mean) of row m of A (layer_norm_stats) and ln_u[n] = sum_k B[n][k]:
  // exactly LN(x) W^T + bias, with no normalised copy of A written or read.
  const float2* ln_rs = nullptr; const float* ln_u = nullptr;
  // ... or the row statistics as producer partials (ln_out of the GEMM that wrote A): ln_part[m * ln_T + t] = (mean,
  // M2) of row m over 320-column group t of a ln_T * 320-wide row, merged in the epilogue into
  // (rstd, rstd * mean) with rstd = rsqrt(M2 / (ln_T * 320) + ln_eps) (ln_rs_at) — no statistics pass over A
  const float2* ln_part = nullptr; int ln_T = 0; float ln_eps = 1e-5f;
  // LayerNorm partials of the OUTPUT emitted by the epilogue (gemm_emits_ln_parts: the transformer's residual stream,
  // whose next consumer folds its LayerNorm): per output row m and 320-column group t, (mean, M2 = sum of squared
  // deviations from that mean) of the stored values, two-pass over the staged tile, at ln_out[m * (N / 320) + t]
  float2* ln_out = nullptr;
  // ... and with ln_out_rs (N == 320: the whole row in one group) the final (rstd, rstd * mean) of each row with
  // ln_eps instead — what a folded consumer takes as ln_rs, no merge left
  int ln_out_rs = 0;
  // per-image operands (GroupNorm folded into the weights, gn_fold_weights): rows [i * b_rows, (i + 1) * b_rows) are
  // multiplied by B + i * b_img_stride and get bias + i * bias_img_stride (0: one B / bias for every row; a tile never
  // straddles two images: gemm_bimg_ok)
  int b_rows = 0; long b_img_stride = 0; long bias_img_stride = 0;
  // sub-pixel output (a nearest-2x upsampler's conv as 4 per-parity 2x2 convs, IRX_LAYOUT_CONV_UP2): the GEMM's row m
  // is low-resolution pixel (image, y, x) of an up2_h x up2_w image and is stored at high-resolution pixel
  // (image, 2y + a, 2x + b), parity up2_p = 2a + b (0: off).  GroupNorm partials go to row block
  // (image * 4 + up2_p) * (up2_h * up2_w / BM) + the block within the image (per image contiguous).
  int up2_h = 0, up2_w = 0, up2_p = 0;
  void* splitk_ws = nullptr; size_t splitk_ws_bytes = 0;   // caller workspace for split-K partials
  // (set by the launcher) N-major tile order: consecutive tiles (one XCD's range) share a B panel instead of an A
  // panel — for the weight-heavy small-M shapes (8x8-level convs: 29.5 MB of weights for 1024 rows)
  int nmajor = 0;
  // (set by the launcher, halo convs) grouped tile order: logical tiles run in groups of group_m consecutive M tiles,
  // N-major inside a group, so one XCD's consecutive range covers a group_m x (range / group_m) rectangle of tiles —
  // its A slabs and B panels each fetched once into that XCD's L2 (0: the M-major / N-major order above)
  int group_m = 0;
  int dbg = 0;            // large-tile diagnostics (irx_set_option("gemm_dbg")): 1 skip epilogue, 2 skip MFMAs
};
constexpr int kCanonImages = 16;
constexpr int kLnGroup = 320;   // columns per LayerNorm partial (GemmArgs::ln_out / ln_part)
// LayerNorm row statistics from producer partials (mean_t, M2_t) over T equal 320-column groups: the merged (mean, M2)
// (two groups: M2 = M2_a + M2_b + 160 (mean_a - mean_b)^2; mean = (mean_a + mean_b) / 2, both exact reassociations of
// the pooled sums) and the (rstd, rstd * mean) the folded epilogue applies.  Multiplies by exact reciprocals only
// (no division): the same arithmetic wherever it runs (gemm2 / gemm_sk epilogues).
__device__ __forceinline__ float2 ln_fin(float mean, float m2, int T, float eps) {
  const float inv_n = T == 1 ? 1.f / 320.f : T == 2 ? 1.f / 640.f : 1.f / (float)(T * kLnGroup);
  const float rstd = rsqrtf(fmaf(m2, inv_n, eps));
  return make_float2(rstd, rstd * mean);
}
__device__ __forceinline__ float2 ln_merge(const float2* __restrict__ p, int T) {   // -> (mean, M2)
  if (T == 1) return p[0];
  if (T == 2) {
    const float2 x = p[0], y = p[1];
    const float d = x.x - y.x;
    return make_float2((x.x + y.x) * 0.5f, fmaf(0.5f * (float)kLnGroup * d, d, x.y + y.y));
  }
  float sm = 0.f;
  for (int t = 0; t < T; ++t) sm += p[t].x;
  const float mean = sm * (1.f / (float)T);
  float m2 = 0.f;
  for (int t = 0; t < T; ++t) {
    const float2 v = p[t];
    const float d = v.x - mean;
    m2 += fmaf((float)kLnGroup * d, d, v.y);
  }
  return make_float2(mean, m2);
}
// (rstd, rstd * mean) of row m: ln_rs[m], or merged from the row's ln_T producer partials
__device__ __forceinline__ float2 ln_rs_at(const float2* __restrict__ rs, const float2* __restrict__ part, int T,
                                           float eps, long m) {
  if (!part) return rs[m];
  const float2 v = ln_merge(part + m * T, T);
  return ln_fin(v.x, v.y, T, eps);
}
// element offset of output (m, n) in C (see GemmArgs::hs_L).  Fields passed by value: a reference to the
// kernel-argument struct would make the compiler copy all of it to scratch.
__host__ __device__ __forceinline__ long c_off_f(long m, int n, long ldc, int M, int hs_L, int hs_C, int hs_d, int up2_w,
                                                 int up2_p) {
  // (sub-pixel: (image * 2H + 2y + a) * 2W + 2x + b = 2 (m + W floor(m / W)) + 2 W a + b)
  if (up2_w) return (2 * (m + (long)up2_w * (m / up2_w)) + 2L * up2_w * (up2_p >> 1) + (up2_p & 1)) * ldc + n;
  if (hs_L == 0) return m * ldc + n;
  const int part = n / hs_C, rem = n - part * hs_C, hd = rem / hs_d, e = rem - hd * hs_d;
  const long img = m / hs_L, tok = m - img * hs_L;
  return (long)part * M * hs_C + ((img * (hs_C / hs_d) + hd) * hs_L + tok) * hs_d + e;
}
#define c_off(a, m, n) c_off_f((m), (n), (a).ldc, (a).M, (a).hs_L, (a).hs_C, (a).hs_d, (a).up2_w, (a).up2_p)
bool gemm_up2_ok(const GemmArgs& a);   // the large-tile path can store a sub-pixel (GemmArgs::up2_*) output
void gemm(const GemmArgs& a, hipStream_t s);
bool gemm_large_tile(const GemmArgs& a, hipStream_t s);   // 8-wave LDS-DMA path; false if not eligible
float* splitk_scratch(size_t bytes);                     // the library's split-K partial scratch (grown on demand)
void splitk_reduce(const GemmArgs& a, const float* ws, int splits, int Mp, int Np, hipStream_t s);
extern int g_small_splitk;   // 1 (default): small-M, long-K 4-wave GEMMs in K splits + the reduce kernel
// A 1x1 / stride-1 / unpadded conv (optionally over a channel concat) rewritten as a dense GEMM over the NHWC
// rows (A = src0, A1 = src1 from K = C0) when the large-tile path takes it (option conv1x1_dense): the
// im2col walk's per-tap machinery buys nothing at one tap.  Returns whether `a` was rewritten.
bool conv1x1_as_dense(GemmArgs& a);
extern int g_conv1x1_dense;
bool gemm_sk(const GemmArgs& a, hipStream_t s);           // K = 320 streaming path (gemm_sk.hip); false if not eligible
bool gemm_sk_eligible(const GemmArgs& a);
extern int g_gemm_sk;      // 1: the K = 320 projections take gemm_sk (0: the large-tile kernel, A/B)
extern int g_gemm_sk_blocks;
size_t gemm_workspace_bytes(const GemmArgs& a);           // split-K partial buffer the call will use
bool gemm_geglu_fusable(const GemmArgs& a);               // large-tile path can apply the GEGLU epilogue
bool gemm_gn_fusable(const GemmArgs& a);                  // conv can apply GemmArgs::gn_ab to its operand
bool gemm_ln_foldable(const GemmArgs& a);                 // large-tile epilogue can apply GemmArgs::ln_rs / ln_u
bool gemm_emits_ln_parts(const GemmArgs& a);              // large-tile epilogue can emit GemmArgs::ln_out
extern int g_up2;            // 1: nearest-2x upsampler convs as 4 per-parity 2x2 convs (IRX_LAYOUT_CONV_UP2; 0: A/B)
extern int g_ff_chain;       // 1: 16-bit UNets run ff.net.2 -> proj_out as one GEMM (IRX_LAYOUT_MAT_CHAIN; 0: two, A/B)
extern int g_gn_red_parts;   // 1: split-K reduce kernels emit GroupNorm partials (per 64-row block)
int gemm_large_splits(const GemmArgs& a);                 // K splits of the large-tile path (0: not on it)
bool gemm_bimg_ok(const GemmArgs& a);                     // large-tile path can take per-image B / bias (b_rows)
extern int g_gn_fold;      // 1: the transformer GroupNorm folded into per-image proj_in weights (0: gn_apply, A/B)
extern int g_ln_parts;     // 1: transformer producers emit LayerNorm partials, the statistics pass is skipped (0: A/B)
extern int g_ln_fold;      // 1: 16-bit UNets fold LayerNorm into the following projections (read at model creation)
int gemm_emits_gn_parts(const GemmArgs& a);   // rows per GroupNorm partial this call's epilogue emits (0: none)
extern int g_gn_parts;     // 1: producers emit GroupNorm partial sums, the stats pass is skipped (0: A/B)
extern int g_gn_fuse;      // 1: GroupNorm(+SiLU) folded into the following halo conv where it fits (0: A/B)
extern bool g_large_tiles;
extern int g_large_mask;
extern int g_large_dense;
extern int g_gemm_pp_chain;   // 1 (default): the long-K two-source 1x1 chains on the lean dense ping-pong loop
extern int g_gemm_group;   // 1 (default): grouped dense tile order where it cuts per-XCD A + B bytes by > 10 %
extern int g_halo_mi;      // 1 (default): the 8x8-level 3x3 convs on 4-image halo tiles (K splits, reduce kernel)
extern int g_halo_up2;     // 1 (default): upsampler parity convs (2x2, GemmArgs::up2_*) on 4-tap halo tiles
extern int g_halo_strip;   // 1 (default): 8 x 32 strip halo tiles where whole-row tiles do not fit; 2 wherever allowed
extern int g_halo_group;   // 1 (default): grouped halo conv tile order where it cuts per-XCD A + B bytes by > 10 %
extern int g_gemm_nmajor;   // 0 M-major tile order, 1 N-major where B outweighs A (default), 2 always N-major
extern int g_gemm_deep;    // large-tile pipeline: 0 two-stage BK 64, 1 BK-32 S-stage ring, 2 BK-64 deeper ring
extern int g_gemm_dbg;     // timing diagnostics only: results are wrong when set
extern bool g_gemm_small;  // short-K GEMMs on 4-wave 128x160 / 128x128 tiles, 2 blocks per CU
extern int g_gemm_small_kmax;

// ------------------------------------------------------------ normalisation
// GroupNorm over NHWC (optionally a channel concat of two sources). Writes the normalised (and
// optionally SiLU'd) result as one contiguous C0+C1 channel tensor.  `ws` needs gn_ws_bytes().
size_t gn_ws_bytes(int N, int HW, int G);
extern bool g_splitk_inkernel;
extern bool g_tile_256x320;
extern int g_gemm_force;
extern int g_conv_halo;      // 3x3 convs on whole-row tiles: one LDS halo per 32-channel slab for all 9 taps
extern int g_gemm_pp;        // 1: ping-pong main loop for dense GEMMs (off: measured slower, see gemm2.hip)
extern int g_halo_pipe;      // 1: software-pipelined halo main loop (fragments read one sub-step ahead)
extern int g_halo_split;     // halo convs whose tiles alone do not fill the chip take two K splits
extern int g_gn_fa;        // GroupNorm from partials as one fused finalize + apply launch (gn_fa_kernel) at HW <= g_gn_fa
extern int g_gn_fa_wide;
extern int g_gn_fa_blocks;
extern bool g_gn_v2;       // GroupNorm stats v3 (slabbed grid + finalize kernel); 0 = v1 (A/B)
void group_norm(int dtype, const void* x0, const void* x1, int C0, int C1, int N, int HW, int G, float eps,
                const float* gamma, const float* beta, int silu, void* out, void* ws, hipStream_t s);
// GroupNorm from producer partials (GemmArgs::gn_part of x0 / x1, r0 / r1 rows each, dividing HW): finalize +
// apply, no statistics pass over the tensor
void group_norm_parts(int dtype, const void* x0, const void* x1, int C0, int C1, int N, int HW, int G, float eps,
                      const float* gamma, const float* beta, int silu, void* out, const double* p0, int r0,
                      const double* p1, int r1, void* ws, hipStream_t s);
// statistics only: per (image, channel) scale / shift (gamma * rstd, beta - mean * gamma * rstd) into
// `ab` [N][C0 + C1] (float2), for a consumer that applies them itself (GemmArgs::gn_ab)
void group_norm_stats(int dtype, const void* x0, const void* x1, int C0, int C1, int N, int HW, int G, float eps,
                      const float* gamma, const float* beta, float2* ab, void* ws, hipStream_t s);
// ... the same scale / shift from producer partials (group_norm_parts' finalize alone; x1 absent)
// (mr, nullable: (mean, rstd) per (image, group) [N][G])
void group_norm_parts_ab(int C0, int N, int HW, int G, float eps, const float* gamma, const float* beta,
                         const double* p0, int r0, float2* ab, float2* mr, hipStream_t s);
// GroupNorm(+SiLU) fused into a 3x3 / stride-1 / pad-1 conv to cout <= 16 channels (the models' output heads):
// out[n][y][x][o] (ldo per pixel, fp32 or the storage type) = bias[o] + conv(act(x * ab.x + ab.y)); x [N][H][W][C]
bool gn_conv_narrow_ok(int dtype, int C, int cout);
void gn_conv_narrow(int dtype, const void* x, int N, int H, int W, int C, const float2* ab, int silu, const void* w,
                    const float* bias, int cout, void* out, int ldo, int out_f32, hipStream_t s);
extern int g_gn_narrow;   // 1: the output heads take gn_conv_narrow (0: GroupNorm pass + conv, A/B)
// (mean, rstd) per (image, group) [N][G] left in `ws` by group_norm_stats
const float2* gn_mr_ws(const void* ws, int N, int G);
// GroupNorm folded into the projection that consumes it (y = x * a + b per image and channel, then y W^T + bias):
// Wo[i][n][k] = o = round(W[n][k] * ab[i][k].x) (the storage type), bo[i][n] = bias[n] + sum_k (W[n][k] * beta[k] -
// o * mean[i][k / (K / G)]) with mr = (mean, rstd) per (image, group): the group mean cancels exactly in the GEMM
void gn_fold_weights(int dtype, const void* W, const float* bias, const float2* ab, const float* beta,
                     const float2* mr, int G, int N, int K, int imgs, void* Wo, float* bo, hipStream_t s);
// gamma / beta may be null: no affine (y = (x - mean) * rstd), the form the folded projections' fallback uses
void layer_norm(int dtype, const void* x, long ldx, int rows, int C, float eps, const float* gamma,
                const float* beta, void* out, long ldo, hipStream_t s);
// per-row (rstd, rstd * mean) only (GemmArgs::ln_rs): one read of x, the statistics of layer_norm exactly
void layer_norm_stats(int dtype, const void* x, long ldx, int rows, int C, float eps, float2* stats, hipStream_t s);

// ------------------------------------------------------------ attention
// Multi-head attention, flash-style (online softmax, never materialises scores).
// q[b][i][h*d + e] with row stride ldq (elements), batch stride sq; likewise k, v, o.
struct AttnArgs {
  int dtype = BF16;
  int B = 1, H = 1, Lq = 0, Lk = 0, d = 0;
  const void* q = nullptr; long ldq = 0, sq = 0;
  const void* k = nullptr; long ldk = 0, sk = 0;
  const void* v = nullptr; long ldv = 0, sv = 0;
  void* o = nullptr; long ldo = 0, so = 0;
  float scale = 1.f;
  int causal = 0;
  // head strides in elements (0: heads interleaved in a row, stride d) — a head-major [b][h][L][d] tensor
  // passes hs* = L * d and ld* = d
  long hsq = 0, hsk = 0, hsv = 0, hso = 0;
  int q_scaled = 0;       // q already multiplied by scale * log2(e) (folded into the to_q weights)
  int xcd = 0;            // (set by the launcher) XCD-grouped block order
  int prio = 0;           // (set by the launcher) s_setprio around the MFMA chains
  int qrep = 1;           // (set by the launcher) query groups per block over resident K/V
};
void attention(const AttnArgs& a, hipStream_t s);
extern int g_attn_q2;    // 1: non-causal streamed d = 40 attention with two 32-query groups per wave (attn3q)
extern int g_attn_pf;    // 1: non-causal streamed d = 40 attention with whole-tile K / V fragment prefetch (attn3 PF)
extern int g_attn_pf160;   // 1: d = 160 attention (streamed and resident K/V) with the whole-tile fragment prefetch
extern int g_attn_prio;
extern int g_attn_qrep;
extern int g_attn_xcd;   // 1: (batch, head) groups of q-blocks kept on one XCD (K/V shared in its L2)
extern int g_attn_hm;    // 1: the UNet's q|k|v projections write head-major attention operands

// ------------------------------------------------------------ elementwise / data movement
// out[m][f] = h * gelu_erf(g): h = proj[m][f], g = proj[m][F + f]; with interleave64 the proj columns are
// (64 value, 64 gate) block pairs (the GEGLU64 weight layout the fused epilogue uses)
void geglu(int dtype, const void* proj, long ldp, int M, int F, void* out, long ldo, int interleave64, hipStream_t s);
void timestep_embed(int dtype, const float* t, int B, int dim, int flip_sin_to_cos, float shift, void* out,
                    hipStream_t s);
void embed_tokens(int dtype, const int* ids, int B, int L, const void* tok, const void* pos, int D, void* out,
                  hipStream_t s);
void transpose2d(int dtype, const void* in, long ldi, int rows, int cols, void* out, long ldo, int batch,
                 long s_in, long s_out, hipStream_t s);
void softmax_rows(int dtype, const float* in, long ldi, int rows, int cols, void* out, long ldo, hipStream_t s);

// image uint8 NHWC (3 ch) -> [-1,1] dtype NHWC with `cpad` channels (zero padded); optional mask [N][H][W]
// (1 = inpaint) zeroes masked pixels: init_image * (mask < 0.5)
void image_to_tensor(int dtype, const uint8_t* img, const float* mask, int N, int H, int W, int cpad, void* out,
                     hipStream_t s);
// decoded dtype NHWC (ldc channels, first 3 used) -> uint8 (+ optional fp32 [0,1] copy)
void tensor_to_image(int dtype, const void* x, int N, int H, int W, int ldc, uint8_t* img, float* f01,
                     hipStream_t s);
// moments [N][h][w][mcs] (mean = ch 0..3, logvar = ch 4..7) -> z = (mean + exp(.5*clamp(logvar))*eps)*sf,
// then optionally x = a*z + b*noise.  eps/noise fp32 [N][h][w][4] (or broadcast over N if bcast).
void latent_sample(int dtype, const void* moments, int mcs, int N, int h, int w, const float* eps,
                   const float* noise, int bcast, float sf, float a, float b, float* out, hipStream_t s);

// Fused classifier-free-guidance + scheduler update + next-step UNet input packing.
struct StepArgs {
  int dtype = BF16;
  int B = 1, h = 0, w = 0;               // latent batch (images), spatial size
  const float* eps = nullptr;            // UNet output fp32 [(cfg?2B:B)][h][w][4]
  int cfg = 0; float guidance = 1.f;
  // history ring (PNDM): store the CFG-combined eps into hist_store (may be null)
  float* hist_store = nullptr;
  const float* hist[4] = {nullptr, nullptr, nullptr, nullptr};   // previous eps entries
  float hw[5] = {1.f, 0.f, 0.f, 0.f, 0.f};  // e = (hw0*eps + hw1*h0 + hw2*h1 + hw3*h2 + hw4*h3)*e_scale
  float e_div = 1.f;                        // e /= e_div  (applied after the weighted sum)
  float e_mul = 1.f;                        // e *= e_mul  (PNDM 4th-order form multiplies by 1/24)
  int mode = 0;                             // 0 = PNDM _get_prev_sample, 1 = DDIM
  float c0 = 0.f, c1 = 0.f, c2 = 0.f, c3 = 0.f;   // scalar coefficients (see kernel)
  const float* x_src = nullptr;             // sample the update applies to
  float* cur_store = nullptr;               // PNDM: keep a copy of x_src (cur_sample)
  float* x_out = nullptr;                   // new latents fp32 [B][h][w][4]
  // next UNet input (dtype) [(cfg?2B:B)][h][w][cin_pad]: latents, then (inpaint) mask + masked latents
  void* unet_in = nullptr; int cin_pad = 8; int inpaint = 0;
  const float* mask = nullptr;              // [B][h][w] (inpaint)
  const float* masked = nullptr;            // [B][h][w][4] (inpaint)
};
void sched_step(const StepArgs& a, hipStream_t s);
// pack fp32 latents into the UNet input layout (same packing as sched_step's tail)
void pack_unet_input(int dtype, const float* lat, int B, int h, int w, int cfg, int cin_pad, int inpaint,
                     const float* mask, const float* masked, void* out, hipStream_t s);
void scale_copy(int dtype_out, const float* in, long n, float scale, void* out, int in_ch, int out_ch,
                hipStream_t s);


// ------------------------------------------------------------ synthetic degradations (degrade.hip)
void degrade_noise(const uint8_t* img, uint8_t* out, long n, float sigma, const float* z, unsigned long long seed,
                   hipStream_t s);
void degrade_blur_down(const uint8_t* img, int B, int H, int W, int C, const int* ksize_dev, int scale,
                       uint8_t* blur, uint8_t* lr, hipStream_t s);
void degrade_gray(const uint8_t* img, long npix, int mode, int rgb, uint8_t* out, hipStream_t s);
void degrade_strokes(int B, int H, int W, const int* segs, const int* thick, const int* seg_off, uint8_t* mask,
                     const uint8_t* img, uint8_t* masked, hipStream_t s);


// ------------------------------------------------------------ fast non-local means (nlmeans.hip)
extern int g_nlm_strip, g_nlm_v2, g_nlm2_strip;
void nlmeans_u8(const uint8_t* src, uint8_t* dst, int N, int H, int W, int ps, int coff, int cn, int tmpl,
                int search, const int* lut, int lut_len, int shift, hipStream_t s);
// ------------------------------------------------------------ bilateral / median (filters.hip)
void bilateral_u8(const uint8_t* src, uint8_t* dst, int N, int H, int W, int radius, const float* space_w,
                  const int* space_dydx, int maxk, const float* color_w, hipStream_t s);
void lab_convert_u8(const uint8_t* src, uint8_t* dst, long npix, int dir, hipStream_t s);
void auto_mask_u8(const uint8_t* img, int B, int H, int W, uint8_t* mask, uint8_t* tmp, int* counts, hipStream_t s);
void colorize_lab_u8(const uint8_t* img, long npix, const double* lin, const uint8_t* cmap, uint8_t* out,
                     hipStream_t s);
void median5_u8(const uint8_t* src, uint8_t* dst, int N, int H, int W, int C, hipStream_t s);

}  // namespace irx
