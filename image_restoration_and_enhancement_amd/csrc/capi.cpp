// irx — extern "C" boundary (include/irx.h).  Every entry point catches C++ exceptions and turns
// them into a non-zero status plus a thread-local message, so the Python layer can log and fall
// back the way src/inference.py does around its diffusers calls.
#include <algorithm>
#include <cmath>
#include <cstring>
#include <string>

#include "../../include/irx.h"
#include "models.h"
#include "profile.h"

namespace irx {
static thread_local std::string g_err;
void set_error(const std::string& m) { g_err = m; }
const char* last_error() { return g_err.c_str(); }
extern int g_attn_pf80;   // (attention.hip)
}  // namespace irx

using namespace irx;

struct irx_model {
  std::unique_ptr<Model> m;
};

#define IRX_API_BEGIN try {
#define IRX_API_END                                       \
  return 0;                                               \
  }                                                       \
  catch (const std::exception& e) {                       \
    set_error(e.what());                                  \
    return -1;                                            \
  }                                                       \
  catch (...) {                                           \
    set_error("unknown error");                           \
    return -1;                                            \
  }

static hipStream_t S(void* s) { return (hipStream_t)s; }

template <typename X>
static X* as(irx_model* h, int kind) {
  IRX_CHECK(h && h->m, "null model");
  IRX_CHECK(h->m->kind() == kind, "wrong model kind");
  return static_cast<X*>(h->m.get());
}
template <typename X>
static const X* as(const irx_model* h, int kind) {
  IRX_CHECK(h && h->m, "null model");
  IRX_CHECK(h->m->kind() == kind, "wrong model kind");
  return static_cast<const X*>(h->m.get());
}

// images spanned by the rows of irx_op_gemm / irx_op_gemm_geglu (0: not image-indexed; tests of the canonical-batch
// tile policy set it through irx_set_option("op_imgs", n))
static int g_op_imgs = 0;

extern "C" {

const char* irx_last_error(void) { return last_error(); }
int irx_version(void) { return 1; }

// every runtime option by name: an int or a bool global (irx_set_option / irx_get_option)
struct OptRef {
  int* i = nullptr;
  bool* b = nullptr;
};
static const struct { const char* name; int* i; bool* b; } kOpts[] = {
    {"large_tiles", nullptr, &g_large_tiles},
    {"gemm_deep", &g_gemm_deep, nullptr},
    {"gemm_dbg", &g_gemm_dbg, nullptr},
    {"gn_v2", nullptr, &g_gn_v2},
    {"gn_fuse", &g_gn_fuse, nullptr},
    {"gn_parts", &g_gn_parts, nullptr},
    {"gn_red_parts", &g_gn_red_parts, nullptr},
    {"ff_chain", &g_ff_chain, nullptr},
    {"up2", &g_up2, nullptr},
    {"ln_parts", &g_ln_parts, nullptr},
    {"gn_fold", &g_gn_fold, nullptr},
    {"gn_narrow", &g_gn_narrow, nullptr},
    {"attn_pf", &g_attn_pf, nullptr},
    {"attn_pf160", &g_attn_pf160, nullptr},
    {"attn_pf80", &g_attn_pf80, nullptr},
    {"attn_q2", &g_attn_q2, nullptr},
    {"conv1x1_dense", &g_conv1x1_dense, nullptr},
    {"gn_fa", &g_gn_fa, nullptr},
    {"gn_fa_wide", &g_gn_fa_wide, nullptr},
    {"gn_fa_blocks", &g_gn_fa_blocks, nullptr},
    {"halo_split", &g_halo_split, nullptr},
    {"halo_pipe", &g_halo_pipe, nullptr},
    {"gemm_pp", &g_gemm_pp, nullptr},
    {"ln_fold", &g_ln_fold, nullptr},
    {"gemm_sk", &g_gemm_sk, nullptr},
    {"large_mask", &g_large_mask, nullptr},
    {"large_dense", &g_large_dense, nullptr},
    {"arena_guard", &g_arena_guard, nullptr},
    {"gemm_nmajor", &g_gemm_nmajor, nullptr},
    {"halo_group", &g_halo_group, nullptr},
    {"halo_strip", &g_halo_strip, nullptr},
    {"halo_up2", &g_halo_up2, nullptr},
    {"halo_mi", &g_halo_mi, nullptr},
    {"gemm_group", &g_gemm_group, nullptr},
    {"small_splitk", &g_small_splitk, nullptr},
    {"gemm_pp_chain", &g_gemm_pp_chain, nullptr},
    {"prof_shapes", &g_prof_shapes, nullptr},
    {"attn_prio", &g_attn_prio, nullptr},
    {"attn_qrep", &g_attn_qrep, nullptr},
    {"op_imgs", &g_op_imgs, nullptr},
    {"gemm_sk_blocks", &g_gemm_sk_blocks, nullptr},
    {"vae_attn_rows", &g_vae_attn_rows, nullptr},
    {"vae_flash", &g_vae_flash, nullptr},
    {"splitk_inkernel", nullptr, &g_splitk_inkernel},
    {"tile_256x320", nullptr, &g_tile_256x320},
    {"gemm_force", &g_gemm_force, nullptr},
    {"conv_halo", &g_conv_halo, nullptr},
    {"gemm_small", nullptr, &g_gemm_small},
    {"attn_xcd", &g_attn_xcd, nullptr},
    {"attn_hm", &g_attn_hm, nullptr},
    {"gemm_small_kmax", &g_gemm_small_kmax, nullptr},
    {"nlm_strip", &g_nlm_strip, nullptr},
    {"nlm_v2", &g_nlm_v2, nullptr},
    {"nlm2_strip", &g_nlm2_strip, nullptr},
};
static OptRef opt_ref(const std::string& n) {
  for (const auto& o : kOpts)
    if (n == o.name) return {o.i, o.b};
  throw Error("unknown option " + n);
}

int irx_set_option(const char* name, int value) {
  IRX_API_BEGIN
  IRX_CHECK(name, "null option name");
  const OptRef r = opt_ref(name);
  if (r.i) *r.i = value;
  else *r.b = value != 0;
  IRX_API_END
}

const char* irx_option_name(int i) {
  return i >= 0 && i < (int)(sizeof(kOpts) / sizeof(kOpts[0])) ? kOpts[i].name : nullptr;
}

int irx_get_option(const char* name, int* value) {
  IRX_API_BEGIN
  IRX_CHECK(name && value, "null argument");
  const OptRef r = opt_ref(name);
  *value = r.i ? *r.i : (*r.b ? 1 : 0);
  IRX_API_END
}

struct irx_graph {
  hipGraphExec_t exec = nullptr;
};

int irx_graph_begin(void* s) {
  IRX_API_BEGIN
  IRX_CHECK(s, "graph capture needs a non-default stream");
  IRX_CHECK(!prof_on(), "graph capture with the launch profiler on");
  // relaxed: the host may allocate (torch's caching allocator) while the stream records
  IRX_HIP(hipStreamBeginCapture(S(s), hipStreamCaptureModeRelaxed));
  IRX_API_END
}

int irx_graph_end(void* s, irx_graph** out) {
  IRX_API_BEGIN
  IRX_CHECK(s && out, "null argument");
  *out = nullptr;
  hipGraph_t g = nullptr;
  IRX_HIP(hipStreamEndCapture(S(s), &g));
  IRX_CHECK(g, "empty graph capture");
  hipGraphExec_t ex = nullptr;
  const hipError_t e = hipGraphInstantiate(&ex, g, nullptr, nullptr, 0);
  (void)hipGraphDestroy(g);
  IRX_HIP(e);
  auto* r = new irx_graph;
  r->exec = ex;
  *out = r;
  IRX_API_END
}

int irx_graph_launch(irx_graph* g, void* s) {
  IRX_API_BEGIN
  IRX_CHECK(g && g->exec, "null graph");
  IRX_HIP(hipGraphLaunch(g->exec, S(s)));
  IRX_API_END
}

int irx_graph_destroy(irx_graph* g) {
  IRX_API_BEGIN
  if (g) {
    if (g->exec) IRX_HIP(hipGraphExecDestroy(g->exec));
    delete g;
  }
  IRX_API_END
}

int irx_profile_begin(void) {
  IRX_API_BEGIN
  prof_begin();
  IRX_API_END
}
int irx_profile_end(int* n) {
  IRX_API_BEGIN
  IRX_CHECK(n, "null argument");
  *n = prof_end();
  IRX_API_END
}
int irx_profile_get(int i, const char** name, long* launches, double* ms, double* flops) {
  IRX_API_BEGIN
  IRX_CHECK(name && launches && ms && flops, "null argument");
  IRX_CHECK(prof_get(i, name, launches, ms, flops), "profile index out of range");
  IRX_API_END
}

int irx_model_create(int kind, const irx_model_config* cfg, int dtype, irx_model** out) {
  IRX_API_BEGIN
  IRX_CHECK(cfg && out, "null argument");
  IRX_CHECK(dtype == IRX_F32 || dtype == IRX_BF16 || dtype == IRX_F16, "dtype must be IRX_F32, IRX_BF16 or IRX_F16");
  auto* h = new irx_model;
  try {
    if (kind == IRX_MODEL_UNET) h->m.reset(new Unet(*cfg, dtype));
    else if (kind == IRX_MODEL_VAE) h->m.reset(new Vae(*cfg, dtype));
    else if (kind == IRX_MODEL_CLIP) h->m.reset(new Clip(*cfg, dtype));
    else throw Error("unknown model kind");
  } catch (...) {
    delete h;
    throw;
  }
  *out = h;
  IRX_API_END
}

int irx_model_destroy(irx_model* m) {
  IRX_API_BEGIN
  delete m;
  IRX_API_END
}

int irx_model_num_params(const irx_model* m, int* n) {
  IRX_API_BEGIN
  IRX_CHECK(m && n, "null argument");
  *n = (int)m->m->manifest().size();
  IRX_API_END
}

int irx_model_param_info(const irx_model* m, int i, irx_param_info* info) {
  IRX_API_BEGIN
  IRX_CHECK(m && info, "null argument");
  const auto& man = m->m->manifest();
  IRX_CHECK(i >= 0 && i < (int)man.size(), "param index out of range");
  const ParamEntry& e = man[i];
  info->name = e.name.c_str();
  info->layout = e.layout;
  info->dtype = e.dtype;
  info->ndim = (int)e.shape.size();
  for (int k = 0; k < 4; ++k) info->shape[k] = k < info->ndim ? e.shape[k] : 1;
  info->offset = e.off;
  info->bytes = e.bytes;
  info->row_scale = e.row_scale;
  info->scale_rows = e.scale_rows;
  info->aux = e.aux.c_str();
  IRX_API_END
}

int irx_model_blob_bytes(const irx_model* m, size_t* bytes) {
  IRX_API_BEGIN
  IRX_CHECK(m && bytes, "null argument");
  *bytes = m->m->blob_bytes();
  IRX_API_END
}

int irx_model_bind(irx_model* m, void* blob, size_t bytes) {
  IRX_API_BEGIN
  IRX_CHECK(m, "null model");
  m->m->bind(blob, bytes);
  IRX_API_END
}

int irx_weights_bcast(irx_model* m, void* comm, int root, void* s) {
  IRX_API_BEGIN
  IRX_CHECK(m && m->m, "null model");
  IRX_CHECK(m->m->blob(), "no weight blob bound (irx_model_bind first)");
  rccl_broadcast(comm, m->m->blob(), m->m->blob_bytes(), root, S(s));
  IRX_API_END
}

// ------------------------------------------------------------------ UNet
int irx_unet_workspace_bytes(const irx_model* m, int B, int h, int w, size_t* bytes) {
  IRX_API_BEGIN
  IRX_CHECK(bytes && B > 0 && h > 0 && w > 0, "bad arguments");
  *bytes = const_cast<Unet*>(as<Unet>(m, IRX_MODEL_UNET))->workspace_bytes(B, h, w);
  IRX_API_END
}
int irx_unet_context_bytes(const irx_model* m, int B, int L, size_t* bytes) {
  IRX_API_BEGIN
  IRX_CHECK(bytes && B > 0 && L > 0, "bad arguments");
  *bytes = as<Unet>(m, IRX_MODEL_UNET)->context_bytes(B, L);
  IRX_API_END
}
int irx_unet_prepare_context(irx_model* m, void* s, const void* ctx, int B, int L, void* kv, void* ws, size_t cap) {
  IRX_API_BEGIN
  IRX_CHECK(ctx && kv, "null buffer");
  as<Unet>(m, IRX_MODEL_UNET)->prepare_context(S(s), ctx, B, L, kv, (char*)ws, cap);
  IRX_API_END
}
int irx_unet_forward(irx_model* m, void* s, const void* x, int B, int h, int w, const float* t, const void* kv, int L,
                     float* eps, void* ws, size_t cap) {
  IRX_API_BEGIN
  IRX_CHECK(x && t && kv && eps && ws, "null buffer");
  as<Unet>(m, IRX_MODEL_UNET)->forward(S(s), x, B, h, w, t, kv, L, eps, (char*)ws, cap);
  IRX_API_END
}
int irx_unet_input_channels(const irx_model* m, int* c) {
  IRX_API_BEGIN
  IRX_CHECK(c, "null argument");
  *c = as<Unet>(m, IRX_MODEL_UNET)->cin_pad();
  IRX_API_END
}

// ------------------------------------------------------------------ VAE
int irx_vae_encode_workspace_bytes(const irx_model* m, int B, int H, int W, size_t* bytes) {
  IRX_API_BEGIN
  IRX_CHECK(bytes && B > 0 && H > 0 && W > 0, "bad arguments");
  *bytes = const_cast<Vae*>(as<Vae>(m, IRX_MODEL_VAE))->encode_ws(B, H, W);
  IRX_API_END
}
int irx_vae_encode(irx_model* m, void* s, const void* img, int B, int H, int W, void* mom, void* ws, size_t cap) {
  IRX_API_BEGIN
  IRX_CHECK(img && mom && ws, "null buffer");
  as<Vae>(m, IRX_MODEL_VAE)->encode(S(s), img, B, H, W, mom, (char*)ws, cap);
  IRX_API_END
}
int irx_vae_decode_workspace_bytes(const irx_model* m, int B, int h, int w, size_t* bytes) {
  IRX_API_BEGIN
  IRX_CHECK(bytes && B > 0 && h > 0 && w > 0, "bad arguments");
  *bytes = const_cast<Vae*>(as<Vae>(m, IRX_MODEL_VAE))->decode_ws(B, h, w);
  IRX_API_END
}
int irx_vae_decode(irx_model* m, void* s, const void* z, int B, int h, int w, void* out, void* ws, size_t cap) {
  IRX_API_BEGIN
  IRX_CHECK(z && out && ws, "null buffer");
  as<Vae>(m, IRX_MODEL_VAE)->decode(S(s), z, B, h, w, out, (char*)ws, cap);
  IRX_API_END
}

// ------------------------------------------------------------------ CLIP
int irx_clip_workspace_bytes(const irx_model* m, int B, int L, size_t* bytes) {
  IRX_API_BEGIN
  IRX_CHECK(bytes && B > 0 && L > 0, "bad arguments");
  *bytes = const_cast<Clip*>(as<Clip>(m, IRX_MODEL_CLIP))->workspace_bytes(B, L);
  IRX_API_END
}
int irx_clip_encode(irx_model* m, void* s, const int* ids, int B, int L, void* out, void* ws, size_t cap) {
  IRX_API_BEGIN
  IRX_CHECK(ids && out && ws, "null buffer");
  as<Clip>(m, IRX_MODEL_CLIP)->encode(S(s), ids, B, L, out, (char*)ws, cap);
  IRX_API_END
}

// ------------------------------------------------------------------ scheduler / glue
int irx_sched_step(void* s, const irx_step_params* p) {
  IRX_API_BEGIN
  IRX_CHECK(p, "null params");
  StepArgs a;
  a.dtype = p->dtype; a.B = p->batch; a.h = p->h; a.w = p->w;
  a.eps = p->eps; a.cfg = p->cfg; a.guidance = p->guidance;
  a.hist_store = p->hist_store;
  for (int i = 0; i < 4; ++i) a.hist[i] = p->hist[i];
  for (int i = 0; i < 5; ++i) a.hw[i] = p->hw[i];
  a.e_div = p->e_div; a.e_mul = p->e_mul;
  a.mode = p->mode; a.c0 = p->c0; a.c1 = p->c1; a.c2 = p->c2; a.c3 = p->c3;
  a.x_src = p->x_src; a.cur_store = p->cur_store; a.x_out = p->x_out;
  a.unet_in = p->unet_in; a.cin_pad = p->cin_pad; a.inpaint = p->inpaint; a.mask = p->mask; a.masked = p->masked;
  sched_step(a, S(s));
  IRX_API_END
}
int irx_pack_unet_input(void* s, int dtype, const float* lat, int B, int h, int w, int cfg, int cin_pad, int inpaint,
                        const float* mask, const float* masked, void* out) {
  IRX_API_BEGIN
  IRX_CHECK(lat && out, "null buffer");
  IRX_CHECK(!inpaint || (mask && masked && cin_pad >= 9), "inpaint inputs");
  pack_unet_input(dtype, lat, B, h, w, cfg, cin_pad, inpaint, mask, masked, out, S(s));
  IRX_API_END
}
int irx_latent_sample(void* s, int dtype, const void* mom, int B, int h, int w, const float* eps, const float* noise,
                      int bcast, float sf, float a, float b, float* out) {
  IRX_API_BEGIN
  IRX_CHECK(mom && eps && out, "null buffer");
  latent_sample(dtype, mom, 8, B, h, w, eps, noise, bcast, sf, a, b, out, S(s));
  IRX_API_END
}
int irx_latents_to_vae(void* s, int dtype, const float* lat, int B, int h, int w, float sf, void* z) {
  IRX_API_BEGIN
  IRX_CHECK(lat && z, "null buffer");
  scale_copy(dtype, lat, (long)B * h * w, sf, z, 4, 8, S(s));
  IRX_API_END
}
int irx_image_to_tensor(void* s, int dtype, const uint8_t* img, const float* mask, int B, int H, int W, int cpad,
                        void* out) {
  IRX_API_BEGIN
  IRX_CHECK(img && out && cpad >= 3, "bad arguments");
  image_to_tensor(dtype, img, mask, B, H, W, cpad, out, S(s));
  IRX_API_END
}
int irx_tensor_to_image(void* s, int dtype, const void* x, int B, int H, int W, int ldc, uint8_t* img, float* f01) {
  IRX_API_BEGIN
  IRX_CHECK(x && img && ldc >= 3, "bad arguments");
  tensor_to_image(dtype, x, B, H, W, ldc, img, f01, S(s));
  IRX_API_END
}

// ------------------------------------------------------------------ synthetic degradations
int irx_degrade_noise(void* s, const uint8_t* img, long n, float sigma, const float* noise, unsigned long long seed,
                      uint8_t* out) {
  IRX_API_BEGIN
  IRX_CHECK(img && out && n >= 0, "bad arguments");
  if (n) degrade_noise(img, out, n, sigma, noise, seed, S(s));
  IRX_API_END
}
int irx_degrade_blur_down(void* s, const uint8_t* img, int batch, int H, int W, int C, const int* ksize, int scale,
                          uint8_t* blur, uint8_t* lr) {
  IRX_API_BEGIN
  IRX_CHECK(img && ksize && blur && batch >= 0 && H > 0 && W > 0 && C > 0, "bad arguments");
  IRX_CHECK(!lr || (scale >= 1 && H / scale > 0 && W / scale > 0), "bad scale");
  if (batch) degrade_blur_down(img, batch, H, W, C, ksize, scale, blur, lr, S(s));
  IRX_API_END
}
int irx_degrade_gray(void* s, const uint8_t* img, long npix, int mode, int rgb, uint8_t* out) {
  IRX_API_BEGIN
  IRX_CHECK(img && out && npix >= 0 && (mode == 0 || mode == 1), "bad arguments");
  if (npix) degrade_gray(img, npix, mode, rgb, out, S(s));
  IRX_API_END
}
int irx_degrade_strokes(void* s, int batch, int H, int W, const int* segs, const int* thick, const int* seg_off,
                        uint8_t* mask, const uint8_t* img, uint8_t* masked) {
  IRX_API_BEGIN
  IRX_CHECK(seg_off && mask && batch >= 0 && H > 0 && W > 0, "bad arguments");
  IRX_CHECK(H <= (1 << 14) && W <= (1 << 14), "stroke masks: H, W <= 16384 (exact int64 capsule test)");
  if (batch) degrade_strokes(batch, H, W, segs, thick, seg_off, mask, img, masked, S(s));
  IRX_API_END
}

// ------------------------------------------------------------------ fast non-local means
static int nlm_shift(int tmpl) {
  int s = 0;
  while ((1 << s) < tmpl * tmpl) ++s;
  return s;
}
int irx_nlm_weights(float h, int cn, int tmpl, int search, int* lut, int cap, int* lut_len) {
  IRX_API_BEGIN
  IRX_CHECK(lut_len && cn >= 1 && cn <= 4 && tmpl >= 1 && (tmpl & 1) && search >= 1 && (search & 1), "bad arguments");
  // FastNlMeansDenoisingInvoker's constructor + DistSquared::calcWeight (OpenCV 4.x, uint8 / int)
  const int tws2 = tmpl * tmpl, shift = nlm_shift(tmpl);
  const double mult = (double)(1 << shift) / tws2;
  const int fpm = (int)std::min<long>(2147483647L / ((long)search * search * 255), 2147483647L);
  const int almost_max = (int)(255.0 * 255.0 * cn / mult + 1);
  const float den = h * h * (float)cn;
  int n = 0;
  for (; n < almost_max; ++n) {
    double w = std::exp(-(n * mult) / den);
    if (std::isnan(w)) w = 1.0;
    int wt = (int)std::nearbyint(fpm * w);
    if (wt < 0.001 * fpm) wt = 0;
    if (wt == 0) break;                     // non-increasing in n: the rest of the table is zero
    if (lut) {
      IRX_CHECK(n < cap, "weight table capacity too small");
      lut[n] = wt;
    }
  }
  *lut_len = n;
  IRX_API_END
}
int irx_nlmeans_u8(void* s, const uint8_t* src, uint8_t* dst, int batch, int H, int W, int pix_stride, int ch_off,
                   int cn, int tmpl, int search, const int* lut, int lut_len) {
  IRX_API_BEGIN
  IRX_CHECK(src && dst && src != dst && lut && lut_len >= 1 && batch >= 0 && H > 0 && W > 0, "bad arguments");
  IRX_CHECK(ch_off >= 0 && ch_off + cn <= pix_stride, "channel group outside the pixel");
  if (batch) nlmeans_u8(src, dst, batch, H, W, pix_stride, ch_off, cn, tmpl, search, lut, lut_len, nlm_shift(tmpl), S(s));
  IRX_API_END
}

// ------------------------------------------------------------------ bilateral / median filters
int irx_bilateral_tables(int d, double sigma_color, double sigma_space, int cn, float* color_w, float* space_w,
                         int* space_dydx, int cap, int* maxk, int* radius) {
  IRX_API_BEGIN
  IRX_CHECK(maxk && radius && cn >= 1 && cn <= 4, "bad arguments");
  // bilateralFilter_8u (OpenCV 4.x): sigma <= 0 -> 1; radius d/2 (or cvRound(1.5 sigma_space) if d <= 0), >= 1
  if (sigma_color <= 0) sigma_color = 1;
  if (sigma_space <= 0) sigma_space = 1;
  const double gc = -0.5 / (sigma_color * sigma_color), gs = -0.5 / (sigma_space * sigma_space);
  int r = d <= 0 ? (int)std::nearbyint(sigma_space * 1.5) : d / 2;
  r = std::max(r, 1);
  if (color_w)
    for (int i = 0; i < 256 * cn; ++i) color_w[i] = (float)std::exp(i * i * gc);
  int k = 0;
  for (int i = -r; i <= r; ++i)
    for (int j = -r; j <= r; ++j) {
      const double rr = std::sqrt((double)i * i + (double)j * j);
      if (rr > r) continue;
      if (space_w) {
        IRX_CHECK(k < cap, "space table capacity too small");
        space_w[k] = (float)std::exp(rr * rr * gs);
        space_dydx[2 * k] = i;
        space_dydx[2 * k + 1] = j;
      }
      ++k;
    }
  *maxk = k;
  *radius = r;
  IRX_API_END
}
int irx_bilateral_u8(void* s, const uint8_t* src, uint8_t* dst, int batch, int H, int W, int radius,
                     const float* space_w, const int* space_dydx, int maxk, const float* color_w) {
  IRX_API_BEGIN
  IRX_CHECK(src && dst && src != dst && space_w && space_dydx && color_w && batch >= 0 && H > 0 && W > 0,
            "bad arguments");
  if (batch) bilateral_u8(src, dst, batch, H, W, radius, space_w, space_dydx, maxk, color_w, S(s));
  IRX_API_END
}
int irx_lab_convert_u8(void* s, const uint8_t* src, uint8_t* dst, long npix, int direction) {
  IRX_API_BEGIN
  IRX_CHECK(src && dst && npix >= 0 && (direction == 0 || direction == 1), "bad arguments");
  if (npix) lab_convert_u8(src, dst, npix, direction, S(s));
  IRX_API_END
}
int irx_auto_mask_u8(void* s, const uint8_t* img, int batch, int H, int W, uint8_t* mask, uint8_t* tmp,
                     int* counts) {
  IRX_API_BEGIN
  IRX_CHECK(img && mask && tmp && counts && mask != tmp && batch >= 0 && H > 0 && W > 0, "bad arguments");
  if (batch) auto_mask_u8(img, batch, H, W, mask, tmp, counts, S(s));
  IRX_API_END
}
int irx_colorize_lab_u8(void* s, const uint8_t* img, long npix, const double* lin_lut, const uint8_t* color_map,
                        uint8_t* out) {
  IRX_API_BEGIN
  IRX_CHECK(img && lin_lut && color_map && out && npix >= 0, "bad arguments");
  if (npix) colorize_lab_u8(img, npix, lin_lut, color_map, out, S(s));
  IRX_API_END
}
int irx_median_blur_u8(void* s, const uint8_t* src, uint8_t* dst, int batch, int H, int W, int C, int ksize) {
  IRX_API_BEGIN
  IRX_CHECK(src && dst && src != dst && batch >= 0 && H > 0 && W > 0, "bad arguments");
  IRX_CHECK(ksize == 5, "medianBlur: compiled for ksize 5");
  if (batch) median5_u8(src, dst, batch, H, W, C, S(s));
  IRX_API_END
}

// ------------------------------------------------------------------ single ops
int irx_op_conv2d(void* s, int dtype, const void* x0, const void* x1, int c0, int c1, int n, int hin, int win, int hv,
                  int wv, const void* weight, const float* bias, int cout, int kh, int kw, int stride, int pad_t,
                  int pad_l, int ho, int wo, const float* rowadd, long rowadd_ld, const void* residual, void* out,
                  int out_f32, int act) {
  IRX_API_BEGIN
  GemmArgs a;
  a.dtype = dtype;
  a.conv = 1;
  a.g.src0 = x0; a.g.src1 = x1; a.g.C0 = c0; a.g.C1 = c1;
  a.g.N = n; a.g.Hin = hin; a.g.Win = win; a.g.Hv = hv; a.g.Wv = wv;
  a.g.KH = kh; a.g.KW = kw; a.g.stride = stride; a.g.pad_t = pad_t; a.g.pad_l = pad_l; a.g.Ho = ho; a.g.Wo = wo;
  a.M = n * ho * wo; a.N = cout; a.K = kh * kw * (c0 + c1);
  a.B = weight; a.ldb = a.K;
  a.C = out; a.ldc = cout; a.out_f32 = out_f32;
  a.bias = bias;
  a.rowadd = rowadd; a.rowadd_ld = rowadd_ld; a.rows_per_group = ho * wo;
  a.residual = residual; a.ldr = cout;
  a.act = act;
  a.imgs = n;   // image-indexed: the same tile / split choice as the models make for this per-image shape
  conv1x1_as_dense(a);   // as the models do
  gemm(a, S(s));
  IRX_API_END
}

int irx_op_gemm(void* s, int dtype, int M, int N, int K, const void* A, long lda, const void* B, long ldb, void* C,
                long ldc, const float* bias, float alpha, int act, const void* residual, long ldr, int out_f32,
                int batch, long sA, long sB, long sC, long sR) {
  IRX_API_BEGIN
  GemmArgs a;
  a.dtype = dtype; a.M = M; a.N = N; a.K = K;
  a.A = A; a.lda = lda; a.sA = sA;
  a.B = B; a.ldb = ldb; a.sB = sB;
  a.C = C; a.ldc = ldc; a.sC = sC;
  a.bias = bias; a.alpha = alpha; a.act = act;
  a.residual = residual; a.ldr = ldr; a.sR = sR;
  a.out_f32 = out_f32;
  a.batch = batch > 0 ? batch : 1;
  a.imgs = g_op_imgs;
  gemm(a, S(s));
  IRX_API_END
}

int irx_op_group_norm(void* s, int dtype, const void* x0, const void* x1, int c0, int c1, int n, int hw, int groups,
                      float eps, const float* gamma, const float* beta, int silu, void* out, void* ws) {
  IRX_API_BEGIN
  IRX_CHECK(x0 && gamma && beta && out && ws, "null buffer");
  group_norm(dtype, x0, x1, c0, c1, n, hw, groups, eps, gamma, beta, silu, out, ws, S(s));
  IRX_API_END
}
size_t irx_op_group_norm_ws_bytes(int n, int hw, int groups) { return gn_ws_bytes(n, hw, groups); }
static size_t gn_conv3_ab_bytes(int n, int channels) {
  return ((size_t)n * channels * sizeof(float2) + 255) / 256 * 256;
}
size_t irx_op_gn_conv3_ws_bytes(int n, int hw, int groups, int channels) {
  return gn_conv3_ab_bytes(n, channels) + gn_ws_bytes(n, hw, groups);
}

int irx_op_gn_conv3(void* s, int dtype, const void* x0, const void* x1, int c0, int c1, int n, int h, int w,
                    int groups, float eps, const float* gamma, const float* beta, int silu, const void* weight,
                    const float* bias, int cout, const float* rowadd, long rowadd_ld, const void* residual,
                    void* out, void* ws, int* fused) {
  IRX_API_BEGIN
  IRX_CHECK(fused, "null argument");
  GemmArgs a;
  a.dtype = dtype;
  a.conv = 1;
  a.g.src0 = x0; a.g.src1 = x1; a.g.C0 = c0; a.g.C1 = c1;
  a.g.N = n; a.g.Hin = h; a.g.Win = w; a.g.Hv = h; a.g.Wv = w;
  a.g.KH = 3; a.g.KW = 3; a.g.stride = 1; a.g.pad_t = 1; a.g.pad_l = 1; a.g.Ho = h; a.g.Wo = w;
  a.M = n * h * w; a.N = cout; a.K = 9 * (c0 + c1);
  a.B = weight; a.ldb = a.K;
  a.C = out ? out : (void*)(uintptr_t)4096; a.ldc = cout;   // (query: an aligned stand-in, never written)
  a.bias = bias;
  a.rowadd = rowadd; a.rowadd_ld = rowadd_ld; a.rows_per_group = h * w;
  a.residual = residual; a.ldr = cout;
  a.imgs = n;
  *fused = gemm_gn_fusable(a) ? 1 : 0;
  if (!out) return 0;
  IRX_CHECK(*fused, "shape does not take the GroupNorm-fused conv path");
  IRX_CHECK(x0 && gamma && beta && weight && ws, "null buffer");
  float2* ab = (float2*)ws;
  void* gws = (char*)ws + gn_conv3_ab_bytes(n, c0 + c1);
  group_norm_stats(dtype, x0, x1, c0, c1, n, h * w, groups, eps, gamma, beta, ab, gws, S(s));
  a.gn_ab = ab;
  a.gn_silu = silu;
  gemm(a, S(s));
  IRX_API_END
}

// workspace of irx_op_gn_proj: statistics + (ab) + the normalised copy or the per-image folded weights / biases
static size_t al256(size_t b) { return (b + 255) / 256 * 256; }
size_t irx_op_gn_proj_ws_bytes(int n, int hw, int groups, int k, int nout) {
  const size_t big = std::max((size_t)n * hw * k, (size_t)n * nout * k) * 2;
  return al256(gn_ws_bytes(n, hw, groups)) + al256((size_t)n * k * sizeof(float2)) + al256(big) +
         al256((size_t)n * nout * sizeof(float));
}

int irx_op_gn_proj(void* s, int dtype, const void* x, int n, int hw, int k, int groups, float eps, const float* gamma,
                   const float* beta, const void* w, const float* bias, int nout, void* out, void* ws, int* folded,
                   int* splits) {
  IRX_API_BEGIN
  IRX_CHECK(folded && splits, "null argument");
  IRX_CHECK(dtype != F32, "irx_op_gn_proj: 16-bit engines only");
  GemmArgs a;
  a.dtype = dtype; a.M = n * hw; a.N = nout; a.K = k;
  a.A = x; a.lda = k;
  a.B = w; a.ldb = k;
  a.C = out ? out : (void*)(uintptr_t)4096; a.ldc = nout;   // (query: an aligned stand-in, never written)
  a.imgs = n;
  a.b_rows = hw; a.b_img_stride = (long)nout * k; a.bias_img_stride = nout;
  *folded = (g_gn_fold && gemm_bimg_ok(a)) ? 1 : 0;
  if (!*folded) { a.b_rows = 0; a.b_img_stride = 0; a.bias_img_stride = 0; }
  *splits = gemm_large_splits(a);
  if (!out) return 0;
  IRX_CHECK(x && gamma && beta && w && ws, "null buffer");
  char* p = (char*)ws;
  void* gws = p;
  p += al256(gn_ws_bytes(n, hw, groups));
  float2* ab = (float2*)p;
  p += al256((size_t)n * k * sizeof(float2));
  void* big = p;
  p += al256(std::max((size_t)n * hw * k, (size_t)n * nout * k) * 2);
  float* bo = (float*)p;
  if (*folded) {   // the engine's form (models.cpp Unet::transformer), statistics from a pass instead of producer partials
    group_norm_stats(dtype, x, nullptr, k, 0, n, hw, groups, eps, gamma, beta, ab, gws, S(s));
    gn_fold_weights(dtype, w, bias, ab, beta, gn_mr_ws(gws, n, groups), groups, nout, k, n, big, bo, S(s));
    a.B = big;
    a.bias = bo;
  } else {
    group_norm(dtype, x, nullptr, k, 0, n, hw, groups, eps, gamma, beta, 0, big, gws, S(s));
    a.A = big;
    a.bias = bias;
  }
  gemm(a, S(s));
  IRX_API_END
}

int irx_op_gn_conv_narrow(void* s, int dtype, const void* x, int n, int h, int w, int c, int groups, float eps,
                          const float* gamma, const float* beta, int silu, const void* weight, const float* bias,
                          int cout, void* out, int ldo, int out_f32, void* ws) {
  IRX_API_BEGIN
  IRX_CHECK(x && gamma && beta && weight && out && ws, "null buffer");
  IRX_CHECK(gn_conv_narrow_ok(dtype, c, cout), "shape/dtype does not take the fused narrow conv (16-bit, C % 64 == 0)");
  float2* ab = (float2*)ws;
  void* gws = (char*)ws + gn_conv3_ab_bytes(n, c);
  group_norm_stats(dtype, x, nullptr, c, 0, n, h * w, groups, eps, gamma, beta, ab, gws, S(s));
  gn_conv_narrow(dtype, x, n, h, w, c, ab, silu, weight, bias, cout, out, ldo, out_f32, S(s));
  IRX_API_END
}

int irx_op_layer_norm(void* s, int dtype, const void* x, int rows, int c, float eps, const float* gamma,
                      const float* beta, void* out) {
  IRX_API_BEGIN
  IRX_CHECK(x && gamma && beta && out, "null buffer");
  layer_norm(dtype, x, c, rows, c, eps, gamma, beta, out, c, S(s));
  IRX_API_END
}

int irx_op_attention(void* s, int dtype, int B, int H, int lq, int lk, int d, const void* q, long ldq, long sq,
                     const void* k, long ldk, long sk, const void* v, long ldv, long sv, void* o, long ldo, long so,
                     float scale, int causal) {
  IRX_API_BEGIN
  AttnArgs a;
  a.dtype = dtype; a.B = B; a.H = H; a.Lq = lq; a.Lk = lk; a.d = d;
  a.q = q; a.ldq = ldq; a.sq = sq;
  a.k = k; a.ldk = ldk; a.sk = sk;
  a.v = v; a.ldv = ldv; a.sv = sv;
  a.o = o; a.ldo = ldo; a.so = so;
  a.scale = scale; a.causal = causal;
  attention(a, S(s));
  IRX_API_END
}

int irx_op_attention_hm(void* s, int dtype, int B, int H, int lq, int lk, int d, const void* q, const void* k,
                        const void* v, void* o, float scale) {
  IRX_API_BEGIN
  AttnArgs a;
  a.dtype = dtype; a.B = B; a.H = H; a.Lq = lq; a.Lk = lk; a.d = d;
  a.q = q; a.ldq = d; a.sq = (long)H * lq * d; a.hsq = (long)lq * d;
  a.k = k; a.ldk = d; a.sk = (long)H * lk * d; a.hsk = (long)lk * d;
  a.v = v; a.ldv = d; a.sv = (long)H * lk * d; a.hsv = (long)lk * d;
  a.o = o; a.ldo = d; a.so = (long)H * lq * d; a.hso = (long)lq * d;
  a.scale = scale;
  attention(a, S(s));
  IRX_API_END
}

int irx_op_gemm_ln_out(void* s, int dtype, int M, int N, int K, const void* A, const void* B, const float* bias,
                       const void* residual, void* C, void* parts, int final_rs, float eps) {
  IRX_API_BEGIN
  GemmArgs a;
  a.dtype = dtype; a.M = M; a.N = N; a.K = K;
  a.A = A; a.lda = K; a.B = B; a.ldb = K;
  a.C = C; a.ldc = N; a.bias = bias;
  a.residual = residual; a.ldr = N;
  a.imgs = g_op_imgs;
  a.ln_out_rs = final_rs;
  a.ln_eps = eps;
  IRX_CHECK(parts && gemm_emits_ln_parts(a), "shape/dtype cannot emit LayerNorm partials");
  a.ln_out = (float2*)parts;
  gemm(a, S(s));
  IRX_API_END
}

int irx_op_gemm_ln_fold(void* s, int dtype, int M, int N, int K, const void* A, const void* B, const float* u,
                        const float* v, const void* rs, const void* parts, int T, int geglu, void* C) {
  IRX_API_BEGIN
  IRX_CHECK((rs != nullptr) != (parts != nullptr), "give the row statistics or the partials, not both");
  GemmArgs a;
  a.dtype = dtype; a.M = M; a.N = N; a.K = K;
  a.A = A; a.lda = K; a.B = B; a.ldb = K;
  a.C = C; a.ldc = geglu ? N / 2 : N; a.bias = v; a.geglu = geglu ? 1 : 0;
  a.ln_u = u;
  a.ln_rs = (const float2*)rs;
  a.ln_part = (const float2*)parts;
  a.ln_T = parts ? T : 0;
  a.imgs = g_op_imgs;
  IRX_CHECK(!geglu || gemm_geglu_fusable(a), "shape/dtype not eligible for the fused GEGLU epilogue");
  IRX_CHECK(gemm_ln_foldable(a), "shape/dtype not eligible for the folded LayerNorm epilogue");
  gemm(a, S(s));
  IRX_API_END
}

int irx_op_gemm_geglu(void* s, int dtype, int M, int N, int K, const void* A, const void* B, const float* bias,
                      void* C) {
  IRX_API_BEGIN
  GemmArgs a;
  a.dtype = dtype; a.M = M; a.N = N; a.K = K;
  a.A = A; a.lda = K; a.B = B; a.ldb = K;
  a.C = C; a.ldc = N / 2; a.bias = bias; a.geglu = 1;
  a.imgs = g_op_imgs;
  IRX_CHECK(gemm_geglu_fusable(a), "shape/dtype not eligible for the fused GEGLU epilogue");
  gemm(a, S(s));
  IRX_API_END
}

int irx_op_geglu(void* s, int dtype, const void* proj, int M, int F, void* out) {
  IRX_API_BEGIN
  IRX_CHECK(proj && out, "null buffer");
  geglu(dtype, proj, 2L * F, M, F, out, F, 0, S(s));
  IRX_API_END
}

}  // extern "C"
