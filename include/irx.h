/* irx — MI355X-native Stable Diffusion restoration engine: public C ABI.
 *
 * The reference has no native interface: `src/inference.py` (RestorationPipeline,
 * src/inference.py:48-890) calls diffusers pipelines whose components are the boundary this
 * library replaces.  Each entry point below names the reference-side call it stands in for.
 * Conventions:
 *   - every function returns 0 on success, non-zero on failure; irx_last_error() gives a
 *     thread-local message (reference error behaviour: the Python layer logs it and falls back,
 *     src/inference.py:496-498, :575-577, :679-681, :774-776);
 *   - tensors are raw DEVICE pointers owned by the caller (PyTorch-ROCm tensors used as
 *     containers); the library never allocates or frees caller memory;
 *   - activations are NHWC; `dtype` is IRX_F32 (parity mode), IRX_BF16 or IRX_F16 (throughput modes);
 *   - `stream` is a hipStream_t passed as void*; work is enqueued, nothing synchronises;
 *   - a model handle is not thread-safe; use one handle per stream.
 */
#ifndef IRX_H_
#define IRX_H_
#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define IRX_F32 0
#define IRX_BF16 1
#define IRX_F16 2   /* IEEE half: the reference's own GPU dtype (src/inference.py:57), BASELINE configs[4] */

#define IRX_MODEL_UNET 0
#define IRX_MODEL_VAE 1
#define IRX_MODEL_CLIP 2

/* weight layouts of manifest entries (how the host packs diffusers tensors into the blob) */
#define IRX_LAYOUT_VEC 0   /* [n] fp32, zero padded                                  */
#define IRX_LAYOUT_MAT 1   /* [N][K] from [N][K] or [N][K][1][1], zero padded         */
#define IRX_LAYOUT_CONV 2  /* [Cout][KH][KW][Cin] from OIHW, zero padded on Cout/Cin   */
#define IRX_LAYOUT_EMB 3   /* [rows][D] embedding table                                */
/* GEGLU projection (diffusers ff.net.0.proj, rows [values; gates]) re-ordered into (64 value rows,
 * 64 gate rows) block pairs: packed row r <- source row (r/128)*64 + r%64 (+ N/2 if r%128 >= 64) */
#define IRX_LAYOUT_MAT_GEGLU64 4
#define IRX_LAYOUT_VEC_GEGLU64 5
/* LayerNorm folded into the projection it feeds (16-bit UNets; diffusers BasicTransformerBlock norm1/2/3 ->
 * attn1.to_q|k|v, attn2.to_q, ff.net.0.proj).  The matrix entry names its LN weight in `aux`: the packer scales
 * its columns by gamma (after any re-ordering / row scaling, before the cast).  Two fp32 vectors follow it,
 * named after the same matrix spec:
 *   VEC_LN_U  u[n] = sum_k of the packed (cast) matrix row n
 *   VEC_LN_V  v[n] = bias[n] + sum_k W[n][k] * beta[k]  (W re-ordered / row-scaled as packed, before gamma);
 *             aux = "<beta name>;<bias spec or empty>" */
#define IRX_LAYOUT_VEC_LN_U 6
#define IRX_LAYOUT_VEC_LN_V 7
/* Two linear layers with nothing between them folded into one (16-bit UNets: a Transformer2DModel's ff.net.2 ->
 * proj_out, the residual add between them distributing over proj_out): name "<A>|<B>" with A [N][C] the second
 * layer (proj_out.weight) and B [C][K] the first (ff.net.2.weight):
 *   MAT_CHAIN  [N][C + K] = [A | A B]   (product in fp64, then the cast): proj_out(h + ff2(g)) = [A | AB] [h; g] + ...
 *   VEC_CHAIN  [N] = a + A b, aux = "<a name>;<b name>" (the biases: proj_out.bias; ff.net.2.bias) */
#define IRX_LAYOUT_MAT_CHAIN 8
#define IRX_LAYOUT_VEC_CHAIN 9
/* A nearest-2x upsampler's 3x3 conv (diffusers Upsample2D: interpolate(scale 2, nearest) -> conv 3x3 pad 1) folded per
 * output parity (16-bit engines): output pixel (2y + a, 2x + b) only sees low-resolution rows y - 1 + a .. y + a and
 * columns x - 1 + b .. x + b, so each parity p = 2a + b is a 2x2 conv of the low-resolution input.  [4][Cout][2][2][Cin]
 * (as [4 Cout][2][2][Cin]) from OIHW: tap (i, j) of parity (a, b) = sum of the original taps ky in R(a, i), kx in
 * R(b, j), R(0, 0) = {0}, R(0, 1) = {1, 2}, R(1, 0) = {0, 1}, R(1, 1) = {2} (sums in fp64, then the cast).  4 / 9 of
 * the upsampled conv's MACs. */
#define IRX_LAYOUT_CONV_UP2 10

typedef struct irx_model irx_model;

typedef struct {
  /* UNet2DConditionModel (unet/config.json) / AutoencoderKL (vae/config.json) */
  int in_channels, out_channels, latent_channels;
  int n_blocks;
  int block_out_channels[8];
  int layers_per_block;
  int heads;                /* UNet: "attention_head_dim" (= head count in SD-1.5) */
  int cross_attention_dim;
  int norm_groups;
  float norm_eps;
  int flip_sin_to_cos;
  float freq_shift;
  int down_attn[8], up_attn[8];
  /* CLIPTextModel (text_encoder/config.json) */
  int vocab_size, hidden_size, intermediate_size, num_layers, max_positions;
  float layer_norm_eps;
  int quick_gelu;
} irx_model_config;

typedef struct {
  const char* name;   /* diffusers/transformers parameter name(s); '|' joins tensors concatenated on dim 0 */
  int layout;         /* IRX_LAYOUT_* */
  int dtype;          /* IRX_F32 or IRX_BF16 storage in the blob */
  int ndim;
  int64_t shape[4];   /* engine shape (padded) */
  size_t offset;      /* byte offset in the weight blob */
  size_t bytes;
  /* the packer multiplies rows [0, scale_rows) by row_scale (in fp32, before the cast): the attention
   * softmax scale * log2(e) folded into to_q in the 16-bit engines (the kernels then take q pre-scaled) */
  float row_scale;
  int64_t scale_rows;
  const char* aux;    /* IRX_LAYOUT_MAT*: column-scale vector name ("" = none); VEC_LN_V: "<beta>;<bias>" */
} irx_param_info;

const char* irx_last_error(void);
int irx_version(void);

/* engine options: "large_tiles" (1 = 8-wave LDS-DMA GEMM/conv path where eligible, 0 = 4-wave kernel) */
int irx_set_option(const char* name, int value);
int irx_get_option(const char* name, int* value);   /* current value of a runtime option (tests save / restore) */
const char* irx_option_name(int i);                 /* i-th option name, NULL past the last */

/* ---- optional per-launch HIP-event timing of the MFMA kernels (bench.py roofline) ---- */
int irx_profile_begin(void);
int irx_profile_end(int* n_kernels);   /* synchronises, aggregates per kernel instantiation */
int irx_profile_get(int i, const char** name, long* launches, double* total_ms, double* total_flops);

/* ---- HIP-graph capture of a launch sequence (the denoising loop: every UNet eval + fused step kernel).
   begin/end bracket ordinary irx calls on `stream` (a non-default stream; the calls are recorded, not run);
   end instantiates an executable graph, launch replays it on a stream, destroy frees it.  Buffers, shapes
   and scalar arguments are baked in at capture: replay re-runs exactly the recorded launches. ---- */
typedef struct irx_graph irx_graph;
int irx_graph_begin(void* stream);
int irx_graph_end(void* stream, irx_graph** out);
int irx_graph_launch(irx_graph* g, void* stream);
int irx_graph_destroy(irx_graph* g);

/* ---- model lifetime: replaces diffusers/transformers from_pretrained (src/inference.py:162-172) ---- */
int irx_model_create(int kind, const irx_model_config* cfg, int dtype, irx_model** out);
int irx_model_destroy(irx_model* m);
int irx_model_num_params(const irx_model* m, int* n);
int irx_model_param_info(const irx_model* m, int i, irx_param_info* info);
int irx_model_blob_bytes(const irx_model* m, size_t* bytes);
/* bind a device blob packed per the manifest (after upload or RCCL broadcast) */
int irx_model_bind(irx_model* m, void* device_blob, size_t bytes);

/* ---- UNet2DConditionModel.forward (diffusers; called per step at src/inference.py:486/:566/:664/:758) ---- */
int irx_unet_workspace_bytes(const irx_model* m, int batch, int h, int w, size_t* bytes);
int irx_unet_context_bytes(const irx_model* m, int batch, int ctx_len, size_t* bytes);
/* cross-attention K/V of all transformer blocks for a fixed text context (computed once per call) */
int irx_unet_prepare_context(irx_model* m, void* stream, const void* ctx, int batch, int ctx_len, void* ctx_kv,
                             void* ws, size_t ws_bytes);
/* x: [batch][h][w][cin_pad] dtype; t: device fp32 [batch]; eps_out: fp32 [batch][h][w][out_channels] */
int irx_unet_forward(irx_model* m, void* stream, const void* x, int batch, int h, int w, const float* t,
                     const void* ctx_kv, int ctx_len, float* eps_out, void* ws, size_t ws_bytes);
int irx_unet_input_channels(const irx_model* m, int* cin_pad);

/* ---- AutoencoderKL.encode / .decode (diffusers; img2img prepare_latents / final decode) ---- */
int irx_vae_encode_workspace_bytes(const irx_model* m, int batch, int H, int W, size_t* bytes);
/* img: [batch][H][W][8] dtype in [-1,1]; moments: [batch][H/8][W/8][8] dtype (mean 0..3, logvar 4..7) */
int irx_vae_encode(irx_model* m, void* stream, const void* img, int batch, int H, int W, void* moments, void* ws,
                   size_t ws_bytes);
int irx_vae_decode_workspace_bytes(const irx_model* m, int batch, int h, int w, size_t* bytes);
/* z: [batch][h][w][8] dtype (latents / scaling_factor, channels 4..7 zero); out: [batch][8h][8w][4] dtype */
int irx_vae_decode(irx_model* m, void* stream, const void* z, int batch, int h, int w, void* out, void* ws,
                   size_t ws_bytes);

/* ---- CLIPTextModel.last_hidden_state (transformers; encode_prompt) ---- */
int irx_clip_workspace_bytes(const irx_model* m, int batch, int len, size_t* bytes);
/* ids: device int32 [batch][len]; out: [batch][len][hidden] dtype */
int irx_clip_encode(irx_model* m, void* stream, const int* ids, int batch, int len, void* out, void* ws,
                    size_t ws_bytes);

/* ---- scheduler / pipeline glue (PNDMScheduler.step_plms, DDIMScheduler.step, CFG combine, add_noise,
 *      DiagonalGaussianDistribution.sample, VaeImageProcessor pre/post) ---- */
typedef struct {
  int dtype;
  int batch, h, w;
  const float* eps; int cfg; float guidance;
  float* hist_store; const float* hist[4]; float hw[5]; float e_div; float e_mul;
  int mode; float c0, c1, c2, c3;
  const float* x_src; float* cur_store; float* x_out;
  void* unet_in; int cin_pad; int inpaint; const float* mask; const float* masked;
} irx_step_params;
int irx_sched_step(void* stream, const irx_step_params* p);
int irx_pack_unet_input(void* stream, int dtype, const float* lat, int batch, int h, int w, int cfg, int cin_pad,
                        int inpaint, const float* mask, const float* masked, void* out);
int irx_latent_sample(void* stream, int dtype, const void* moments, int batch, int h, int w, const float* eps,
                      const float* noise, int bcast, float scaling_factor, float a, float b, float* out);
int irx_latents_to_vae(void* stream, int dtype, const float* lat, int batch, int h, int w, float scaling_factor,
                       void* z);
/* mask (nullable): fp32 [batch][H][W], 1 = region to inpaint; masked pixels become 0 (init_image * (mask < 0.5)) */
int irx_image_to_tensor(void* stream, int dtype, const uint8_t* img, const float* mask, int batch, int H, int W,
                        int cpad, void* out);
int irx_tensor_to_image(void* stream, int dtype, const void* x, int batch, int H, int W, int ldc, uint8_t* img,
                        float* f01);

/* ---- synthetic degradations (scripts/make_synthetic_pairs.py) ----
 * uint8 HWC batches in device memory, one pass each, no allocation. */
/* add_gaussian_noise (make_synthetic_pairs.py:29-35): out = uint8(clip(f32(img) + f32(z) * sigma, 0, 255));
 * z = `noise` (n floats, e.g. numpy's randn draws) or, if null, Philox4x32-10 normals keyed by `seed` */
int irx_degrade_noise(void* stream, const uint8_t* img, long n, float sigma, const float* noise,
                      unsigned long long seed, uint8_t* out);
/* degrade_sr (:67-81): cv2.GaussianBlur(k, sigma 0) with k = ksize[b] in {3,5,7} (device int[batch]) into
 * `blur` [batch][H][W][C]; if `lr`, cv2.resize(INTER_CUBIC) to [batch][H/scale][W/scale][C] */
int irx_degrade_blur_down(void* stream, const uint8_t* img, int batch, int H, int W, int C, const int* ksize,
                          int scale, uint8_t* blur, uint8_t* lr);
/* to_grayscale (:84-90): mode 0 = cv2 BGR2GRAY, 1 = L of cv2 BGR2Lab; rgb != 0: input channel order R,G,B */
int irx_degrade_gray(void* stream, const uint8_t* img, long npix, int mode, int rgb, uint8_t* out);
/* random_free_form_mask (:104-114) + masked input (:196-198): segs int[nseg][4] (x0,y0,x1,y1), thick int[nseg],
 * seg_off int[batch+1]; mask [batch][H][W] = 255 inside any stroke; img/masked (nullable) [batch][H][W][3] */
int irx_degrade_strokes(void* stream, int batch, int H, int W, const int* segs, const int* thick, const int* seg_off,
                        uint8_t* mask, const uint8_t* img, uint8_t* masked);

/* ---- fast non-local means (cv2.fastNlMeansDenoising / ...Colored as src/inference.py:509-515 calls them in the
 * classical denoise fallback _denoise_opencv :500-522).  OpenCV's integer invoker, exact. ---- */
/* Host only: the invoker's weight table (almost_dist2weight) for filter strength h over `cn`-channel groups,
 * truncated at its first zero; writes *lut_len and, if `lut`, the entries (cap = capacity of lut). */
int irx_nlm_weights(float h, int cn, int template_size, int search_size, int* lut, int cap, int* lut_len);
/* Denoise one channel group (cn = 1 or 2 channels starting at ch_off) of uint8 [batch][H][W][pix_stride] images
 * from src into the same channels of dst (src != dst); lut = device copy of irx_nlm_weights' table.
 * (template, search) in {(7, 21), (3, 5)}. */
int irx_nlmeans_u8(void* stream, const uint8_t* src, uint8_t* dst, int batch, int H, int W, int pix_stride,
                   int ch_off, int cn, int template_size, int search_size, const int* lut, int lut_len);

/* ---- the filters after the NLM pass in _denoise_opencv (src/inference.py:517-520) ---- */
/* Host only: cv2.bilateralFilter's tables (BilateralFilter_8u): color_w[256*cn] = f32(exp(-i^2 / 2sc^2)), and for
 * the circular window (row-major, sqrt(i^2+j^2) <= radius) space_w[k] = f32(exp(-r^2 / 2ss^2)), space_dydx[2k] =
 * (i, j).  Null table pointers: sizes only.  Writes *maxk and *radius. */
int irx_bilateral_tables(int d, double sigma_color, double sigma_space, int cn, float* color_w, float* space_w,
                         int* space_dydx, int cap, int* maxk, int* radius);
/* cv2.bilateralFilter(img, d = 9, ...) on uint8 [batch][H][W][3] (src != dst), tables in device memory. */
int irx_bilateral_u8(void* stream, const uint8_t* src, uint8_t* dst, int batch, int H, int W, int radius,
                     const float* space_w, const int* space_dydx, int maxk, const float* color_w);
/* The colour conversions of cv2.fastNlMeansDenoisingColored (denoising.cpp): direction 0 = COLOR_LBGR2Lab,
 * 1 = COLOR_Lab2LBGR, 8-bit, `npix` packed 3-byte pixels (in place allowed); fp64, see classical.rgb_to_lab_u8. */
int irx_lab_convert_u8(void* stream, const uint8_t* src, uint8_t* dst, long npix, int direction);
/* _auto_mask_from_image (src/inference.py:805-840) for uint8 RGB [batch][H][W][3]: mask [batch][H][W] (255 = damaged)
 * after MORPH_CLOSE + MORPH_OPEN (5x5), counts[batch] = its non-zero pixels (device int); tmp = [batch][H][W]
 * scratch.  The caller applies the reference's 1 % rule. */
int irx_auto_mask_u8(void* stream, const uint8_t* img, int batch, int H, int W, uint8_t* mask, uint8_t* tmp,
                     int* counts);
/* _colorize_lab (src/inference.py:683-703) for `npix` RGB pixels: L of RGB2LAB (sRGB) via lin_lut[256] (device
 * doubles, the sRGB linearisation of each byte value), then out = color_map[L] (device uint8 [256][3]). */
int irx_colorize_lab_u8(void* stream, const uint8_t* img, long npix, const double* lin_lut, const uint8_t* color_map,
                        uint8_t* out);
/* cv2.medianBlur(img, 5) on uint8 [batch][H][W][C], C <= 4 (src != dst). */
int irx_median_blur_u8(void* stream, const uint8_t* src, uint8_t* dst, int batch, int H, int W, int C, int ksize);

/* ---- multi-GPU: RCCL over xGMI (SURVEY.md §8b `irx_weights_bcast(handle, rcclComm)`, §8e) ----
   The reference has no multi-device path (src/inference.py:52-57 picks one device; it stands in for
   `pipe.to("cuda")` at src/inference.py:175-176 on every rank but the first).  One process per GPU: rank 0
   creates the id, the caller ships its 128 bytes to the other ranks over any host channel (the torchrun
   store), each rank creates its communicator on its current HIP device, and the packed weight blob bound to
   a model is broadcast in place from `root`, enqueued on `stream`.  No per-step collectives exist. */
#define IRX_RCCL_ID_BYTES 128
int irx_rccl_available(void);                        /* 1 when librccl can be loaded, else 0 */
int irx_rccl_unique_id(unsigned char* id);           /* id: IRX_RCCL_ID_BYTES bytes (ncclGetUniqueId) */
int irx_rccl_comm_init(const unsigned char* id, int nranks, int rank, void** comm);   /* ncclCommInitRank */
/* the same with a deadline: ncclCommInitRankConfig(blocking = 0) polled with ncclCommGetAsyncError; on an error or
   after timeout_ms the half-made communicator is released with ncclCommAbort, *comm stays NULL and the call fails
   (irx_last_error says which), so a rank whose peers fail or never arrive leaves the init.  timeout_ms <= 0: the
   blocking form.  Communicators made this way are non-blocking: irx_rccl_broadcast / irx_weights_bcast wait for
   each enqueue themselves. */
int irx_rccl_comm_init_timeout(const unsigned char* id, int nranks, int rank, int timeout_ms, void** comm);
int irx_rccl_comm_destroy(void* comm);
int irx_rccl_broadcast(void* comm, void* buf, size_t bytes, int root, void* stream);  /* in place, uint8 */
/* broadcast the model's bound weight blob (irx_model_bind) from `root`; every rank must have bound a blob of
   irx_model_blob_bytes first (non-root ranks: uninitialised memory that this call fills) */
int irx_weights_bcast(irx_model* m, void* comm, int root, void* stream);

/* ---- single-op entry points (parity tests, composition) ---- */
int irx_op_conv2d(void* stream, int dtype, const void* x0, const void* x1, int c0, int c1, int n, int hin, int win,
                  int hv, int wv, const void* weight, const float* bias, int cout, int kh, int kw, int stride,
                  int pad_t, int pad_l, int ho, int wo, const float* rowadd, long rowadd_ld, const void* residual,
                  void* out, int out_f32, int act);
int irx_op_gemm(void* stream, int dtype, int M, int N, int K, const void* A, long lda, const void* B, long ldb,
                void* C, long ldc, const float* bias, float alpha, int act, const void* residual, long ldr,
                int out_f32, int batch, long sA, long sB, long sC, long sR);
int irx_op_group_norm(void* stream, int dtype, const void* x0, const void* x1, int c0, int c1, int n, int hw,
                      int groups, float eps, const float* gamma, const float* beta, int silu, void* out, void* ws);
size_t irx_op_group_norm_ws_bytes(int n, int hw, int groups);
/* GroupNorm(+SiLU) of (x0 | x1) folded into a 3x3 / stride-1 / pad-1 conv's halo operand path (the form the
   UNet / VAE resnets run); bias / rowadd / residual as irx_op_conv2d.  Fails (IRX error) when the shape does
   not take the fused path: *fused reports whether it would (query with out == NULL, nothing launched).
   ws: irx_op_gn_conv3_ws_bytes(n, h * w, groups, c0 + c1) bytes
   (= round_up(n * (c0 + c1) * 8, 256) + irx_op_group_norm_ws_bytes). */
size_t irx_op_gn_conv3_ws_bytes(int n, int hw, int groups, int channels);
int irx_op_gn_conv3(void* stream, int dtype, const void* x0, const void* x1, int c0, int c1, int n, int h, int w,
                    int groups, float eps, const float* gamma, const float* beta, int silu, const void* weight,
                    const float* bias, int cout, const float* rowadd, long rowadd_ld, const void* residual,
                    void* out, void* ws, int* fused);
/* GroupNorm(+SiLU) -> 3x3 / stride-1 / pad-1 conv to cout <= 16 channels in one kernel: the output heads of the UNet
   and VAE that src/inference.py:486 runs (conv_norm_out -> conv_out).  x [n][h][w][c] (16-bit, c % 64 == 0),
   weight [cout][3][3][c], out [n][h][w][ldo] (fp32 when out_f32, else the dtype).  Statistics by a pass over x.
   ws: irx_op_gn_conv3_ws_bytes(n, h * w, groups, c) bytes. */
int irx_op_gn_conv_narrow(void* stream, int dtype, const void* x, int n, int h, int w, int c, int groups, float eps,
                          const float* gamma, const float* beta, int silu, const void* weight, const float* bias,
                          int cout, void* out, int ldo, int out_f32, void* ws);
/* GroupNorm (no SiLU) -> projection: the diffusers Transformer2DModel norm -> proj_in of the UNet that
   src/inference.py:486 runs.  out[i][p][:] = GN(x)[i][p][:] W^T + bias for x [n][hw][k], W [nout][k], out [n][hw][nout].
   With option gn_fold (default) and a shape whose large-tile row tiles never straddle two images, GroupNorm is folded
   into per-image weights o = round(W diag(a_i)) and biases bias + W beta - o mean_i (the engine's form; the normalised
   tensor is never written); otherwise GroupNorm then GEMM.  *folded = 1 when the fold runs, *splits = the large-tile
   K splits (0: not on the large tiles); query both with out == NULL (nothing launched).
   ws: irx_op_gn_proj_ws_bytes(n, hw, groups, k, nout) bytes. */
size_t irx_op_gn_proj_ws_bytes(int n, int hw, int groups, int k, int nout);
int irx_op_gn_proj(void* stream, int dtype, const void* x, int n, int hw, int k, int groups, float eps,
                   const float* gamma, const float* beta, const void* w, const float* bias, int nout, void* out,
                   void* ws, int* folded, int* splits);
int irx_op_layer_norm(void* stream, int dtype, const void* x, int rows, int c, float eps, const float* gamma,
                      const float* beta, void* out);
int irx_op_attention(void* stream, int dtype, int batch, int heads, int lq, int lk, int d, const void* q, long ldq,
                     long sq, const void* k, long ldk, long sk, const void* v, long ldv, long sv, void* o, long ldo,
                     long so, float scale, int causal);
/* heads laid out [batch][heads][len][d] (q, k, v and o), contiguous */
int irx_op_attention_hm(void* stream, int dtype, int batch, int heads, int lq, int lk, int d, const void* q,
                        const void* k, const void* v, void* o, float scale);
int irx_op_geglu(void* stream, int dtype, const void* proj, int M, int F, void* out);
/* C[M][N/2] = GEGLU(A B^T + bias) with B/bias in the GEGLU64 row order (fused epilogue, bf16 large tiles) */
int irx_op_gemm_geglu(void* stream, int dtype, int M, int N, int K, const void* A, const void* B, const float* bias,
                      void* C);
/* Transformer residual-stream producer (the diffusers Transformer2D proj_in / attn.to_out at src/inference.py:486's
   UNet): C = A B^T + bias (+ residual, may alias C), also writing the LayerNorm statistics of C's rows:
   final_rs == 0: parts[m][N / 320] = (mean, sum of squared deviations) per 320-column group;
   final_rs != 0 (N == 320): parts[m] = (rstd, rstd * mean) with rstd = rsqrt(var + eps), the folded consumer's rs.
   Error if the shape cannot emit them. */
int irx_op_gemm_ln_out(void* stream, int dtype, int M, int N, int K, const void* A, const void* B, const float* bias,
                       const void* residual, void* C, void* parts, int final_rs, float eps);
/* LayerNorm folded into the following projection (norm1/2/3 -> to_q|k|v / attn2.to_q / ff.net.0.proj):
   C = rs.x * (A B^T) - rs.y * u + v with B = W diag(gamma), u = row sums of B, v = bias + W beta, and per row
   rs = (rstd, rstd * mean) of A given directly (rs, from a statistics pass) or merged from T producer partials
   (parts, irx_op_gemm_ln_out; K = 320 T).  geglu != 0: B / u / v in the GEGLU64 row order, C gets N / 2 columns. */
int irx_op_gemm_ln_fold(void* stream, int dtype, int M, int N, int K, const void* A, const void* B, const float* u,
                        const float* v, const void* rs, const void* parts, int T, int geglu, void* C);

#ifdef __cplusplus
}
#endif
#endif /* IRX_H_ */
