// irx — native model graphs for the SD-1.5 restoration hot path.
//
// Each class registers its parameters under the diffusers / transformers names (the manifest the
// host packs weights by) and runs its forward pass as a sequence of irx kernel launches on one
// stream, with every temporary carved from a caller-provided workspace by a deterministic
// allocator (a dry run with no launches sizes the workspace).
//   Unet  — diffusers UNet2DConditionModel (SD-1.5 config, outputs/models/*/best/unet/config.json)
//   Vae   — diffusers AutoencoderKL encoder (+quant_conv) / decoder (+post_quant_conv)
//   Clip  — transformers CLIPTextModel (last_hidden_state)
// Fusions relative to the module-by-module reference: GroupNorm+SiLU in one pass; conv bias,
// time-embedding add and residual add in the conv/GEMM epilogues; q|k|v as one GEMM; every
// resnet's time_emb_proj as one GEMM per step; every cross-attention K|V projection as one GEMM
// per prompt (constant over the denoising loop); Upsample2D's nearest resize and the up-block
// skip concat folded into the following convolution's operand gather.
#include "models.h"

#include <cmath>
#include <cstdio>
#include <vector>

namespace irx {

static size_t align_up(size_t x, size_t a) { return (x + a - 1) / a * a; }

// ---------------------------------------------------------------------------------------------- Arena
int g_arena_guard = 0;
int g_ff_chain = 1;
int g_up2 = 1;
constexpr size_t kGuard = 64 * 1024;

void* Arena::alloc(size_t bytes) {
  bytes = align_up(bytes ? bytes : 1, 256) + (g_arena_guard ? kGuard : 0);
  size_t off = (size_t)-1;
  for (auto it = free_.begin(); it != free_.end(); ++it) {
    if (it->second >= bytes) {
      off = it->first;
      const size_t rest = it->second - bytes;
      free_.erase(it);
      if (rest) free_[off + bytes] = rest;
      break;
    }
  }
  if (off == (size_t)-1) {
    off = end_;
    end_ += bytes;
    if (end_ > peak_) peak_ = end_;
  }
  if (base_ && end_ > cap_) throw Error("workspace too small: need > " + std::to_string(end_) + " bytes");
  live_[off] = bytes;
  ids_[off] = next_id_++;
  if (g_arena_guard && base_) {
    IRX_HIP(hipDeviceSynchronize());
    IRX_HIP(hipMemset(base_ + off + bytes - kGuard, 0xA5, kGuard));
    IRX_HIP(hipDeviceSynchronize());
  }
  return base_ ? (void*)(base_ + off) : (void*)(uintptr_t)(off + 4096);
}

void Arena::free(void* p) {
  if (!p) return;
  const size_t off = base_ ? (size_t)((char*)p - base_) : (size_t)((uintptr_t)p - 4096);
  auto it = live_.find(off);
  if (it == live_.end()) throw Error("workspace: double free");
  size_t o = off, sz = it->second;
  if (g_arena_guard && base_) {
    std::vector<unsigned char> h(kGuard);
    IRX_HIP(hipDeviceSynchronize());
    IRX_HIP(hipMemcpy(h.data(), base_ + off + sz - kGuard, kGuard, hipMemcpyDeviceToHost));
    size_t bad = 0, first = kGuard;
    for (size_t i = 0; i < kGuard; ++i)
      if (h[i] != 0xA5) { ++bad; if (first == kGuard) first = i; }
    if (bad) fprintf(stderr, "arena guard: allocation #%d (%zu bytes) overrun: %zu guard bytes changed, first at +%zu\n",
                     ids_[off], sz - kGuard, bad, first);
  }
  live_.erase(it);
  auto nx = free_.lower_bound(o);
  if (nx != free_.end() && nx->first == o + sz) { sz += nx->second; free_.erase(nx); }
  auto pv = free_.lower_bound(o);
  if (pv != free_.begin()) {
    --pv;
    if (pv->first + pv->second == o) { o = pv->first; sz += pv->second; free_.erase(pv); }
  }
  if (o + sz == end_) end_ = o;
  else free_[o] = sz;
}

// ---------------------------------------------------------------------------------------------- Model
P Model::reg(const std::string& name, int layout, int dtype, std::vector<int64_t> shape, float row_scale,
            int64_t scale_rows, const std::string& aux) {
  int64_t n = 1;
  for (auto d : shape) n *= d;
  ParamEntry e{name, layout, dtype, shape, blob_bytes_, (size_t)n * dsize(dtype), row_scale, scale_rows, aux};
  params_.push_back(e);
  P p;
  p.off = blob_bytes_;
  p.set = true;
  blob_bytes_ = align_up(blob_bytes_ + e.bytes, 256);
  return p;
}

void Model::bind(void* blob, size_t bytes) {
  IRX_CHECK(blob != nullptr, "null weight blob");
  IRX_CHECK(bytes >= blob_bytes_, "weight blob too small: " + std::to_string(bytes) + " < " + std::to_string(blob_bytes_));
  IRX_CHECK(((uintptr_t)blob % 256) == 0, "weight blob must be 256-byte aligned");
  blob_ = (char*)blob;
}

Act Model::new_act(Ctx& c, int n, int h, int w, int ch) {
  Act a;
  a.n = n; a.h = h; a.w = w; a.c = ch;
  a.p = c.ws->alloc((size_t)n * h * w * ch * dsize(dt_));
  return a;
}

static GemmArgs conv_args(int dt, const Act& x0, const Act* x1, const void* w, const float* b, int cout, int k,
                          int stride, int pad_t, int pad_l, int hv, int wv, const Act& out, const float* rowadd,
                          long rowadd_ld, const void* residual, int out_f32, int ldc) {
  GemmArgs a;
  a.dtype = dt;
  a.conv = 1;
  a.g.src0 = x0.p; a.g.C0 = x0.c;
  a.g.src1 = x1 ? x1->p : nullptr; a.g.C1 = x1 ? x1->c : 0;
  a.g.N = x0.n; a.g.Hin = x0.h; a.g.Win = x0.w; a.g.Hv = hv; a.g.Wv = wv;
  a.g.KH = k; a.g.KW = k; a.g.stride = stride; a.g.pad_t = pad_t; a.g.pad_l = pad_l;
  a.g.Ho = out.h; a.g.Wo = out.w;
  a.M = out.n * out.h * out.w;
  a.N = cout;
  a.K = k * k * (a.g.C0 + a.g.C1);
  a.B = w; a.ldb = a.K;
  a.C = out.p; a.ldc = ldc < 0 ? cout : ldc;
  a.out_f32 = out_f32;
  a.bias = b;
  a.rowadd = rowadd; a.rowadd_ld = rowadd_ld; a.rows_per_group = out.h * out.w;
  a.residual = residual; a.ldr = a.ldc;
  a.imgs = out.n;
  conv1x1_as_dense(a);   // 1x1 convs (ff chains, resnet shortcuts) on the dense GEMM path
  return a;
}

void Model::gn_conv3(Ctx& c, const Act& x0, const Act* x1, P g, P gb, float eps, int silu, P w, P b, int cout,
                     Act& out, const float* rowadd, long rowadd_ld, const void* residual, bool stats) {
  const int C = x0.c + (x1 ? x1->c : 0);
  GemmArgs a = conv_args(dt_, x0, x1, ptr(w), b.set ? fptr(b) : nullptr, cout, 3, 1, 1, 1, x0.h, x0.w, out, rowadd,
                         rowadd_ld, residual, 0, -1);
  if (gemm_gn_fusable(a)) {
    float2* ab = (float2*)c.ws->alloc((size_t)x0.n * C * sizeof(float2));
    void* ws = c.ws->alloc(gn_ws_bytes(x0.n, x0.h * x0.w, cfg_.norm_groups));
    if (!c.ws->dry())
      group_norm_stats(dt_, x0.p, x1 ? x1->p : nullptr, x0.c, x1 ? x1->c : 0, x0.n, x0.h * x0.w, cfg_.norm_groups,
                       eps, fptr(g), fptr(gb), ab, ws, c.s);
    c.ws->free(ws);
    a.gn_ab = ab;
    a.gn_silu = silu;
    run_gemm(c, a, stats ? &out : nullptr);
    c.ws->free(ab);
    return;
  }
  Act n = new_act(c, x0.n, x0.h, x0.w, C);
  gnorm(c, x0, x1, g, gb, eps, silu, n);
  conv2d(c, n, nullptr, w, b, cout, 3, 1, 1, 1, x0.h, x0.w, out, rowadd, rowadd_ld, residual, 0, -1, stats);
  drop(c, n);
}

void Model::conv2d(Ctx& c, const Act& x0, const Act* x1, P w, P b, int cout, int k, int stride, int pad_t,
                   int pad_l, int hv, int wv, Act& out, const float* rowadd, long rowadd_ld,
                   const void* residual, int out_f32, int ldc, bool stats) {
  GemmArgs a = conv_args(dt_, x0, x1, ptr(w), b.set ? fptr(b) : nullptr, cout, k, stride, pad_t, pad_l, hv, wv, out,
                         rowadd, rowadd_ld, residual, out_f32, ldc);
  run_gemm(c, a, stats && ldc < 0 ? &out : nullptr);
}

void Model::run_gemm(Ctx& c, GemmArgs& a, Act* stats) {
  // GroupNorm partials of the output, kept with the activation until it is dropped (shape-only decision)
  if (stats && !stats->gnp) {
    const int r = gemm_emits_gn_parts(a);
    if (r > 0 && (long)stats->h * stats->w % r == 0) {
      stats->gnp = (double*)c.ws->alloc((size_t)(a.M / r) * a.N * 2 * sizeof(double));
      stats->gnr = r;
      a.gn_part = stats->gnp;
    }
  }
  const size_t ws = gemm_workspace_bytes(a);     // split-K partials (shape-only decision)
  void* p = ws ? c.ws->alloc(ws) : nullptr;
  if (!c.ws->dry()) {
    a.splitk_ws = p;
    a.splitk_ws_bytes = ws;
    gemm(a, c.s);
  }
  if (p) c.ws->free(p);
}

void Model::linear(Ctx& c, const void* A, long lda, int M, int K, P w, int N, const float* bias, void* C, long ldc,
                   int act, const void* residual, long ldr, int out_f32, int imgs, Act* stats) {
  GemmArgs a;
  a.dtype = dt_;
  a.M = M; a.N = N; a.K = K;
  a.A = A; a.lda = lda;
  a.B = ptr(w); a.ldb = K;
  a.C = C; a.ldc = ldc;
  a.bias = bias;
  a.act = act;
  a.residual = residual; a.ldr = ldr;
  a.out_f32 = out_f32;
  a.imgs = imgs;
  run_gemm(c, a, stats && ldc == N ? stats : nullptr);
}

void Model::gnorm(Ctx& c, const Act& x0, const Act* x1, P g, P b, float eps, int silu, const Act& out) {
  void* ws = c.ws->alloc(gn_ws_bytes(x0.n, x0.h * x0.w, cfg_.norm_groups));
  const bool parts = x0.gnp && (!x1 || x1->gnp);   // every source's producer emitted its partial sums
  if (!c.ws->dry()) {
    if (parts)
      group_norm_parts(dt_, x0.p, x1 ? x1->p : nullptr, x0.c, x1 ? x1->c : 0, x0.n, x0.h * x0.w, cfg_.norm_groups,
                       eps, fptr(g), fptr(b), silu, out.p, x0.gnp, x0.gnr, x1 ? x1->gnp : nullptr,
                       x1 ? x1->gnr : 0, ws, c.s);
    else
      group_norm(dt_, x0.p, x1 ? x1->p : nullptr, x0.c, x1 ? x1->c : 0, x0.n, x0.h * x0.w, cfg_.norm_groups, eps,
                 fptr(g), fptr(b), silu, out.p, ws, c.s);
  }
  c.ws->free(ws);
}

bool Model::gn_conv_out(Ctx& c, const Act& x, P g, P gb, float eps, P w, P b, int cout, void* out, int ldo,
                        int out_f32) {
  if (!g_gn_narrow || !gn_conv_narrow_ok(dt_, x.c, cout)) return false;
  const int HW = x.h * x.w;
  float2* ab = (float2*)c.ws->alloc((size_t)x.n * x.c * sizeof(float2));
  const bool parts = x.gnp && HW % x.gnr == 0;
  void* ws = parts ? nullptr : c.ws->alloc(gn_ws_bytes(x.n, HW, cfg_.norm_groups));
  if (!c.ws->dry()) {
    if (parts)
      group_norm_parts_ab(x.c, x.n, HW, cfg_.norm_groups, eps, fptr(g), fptr(gb), x.gnp, x.gnr, ab, nullptr, c.s);
    else
      group_norm_stats(dt_, x.p, nullptr, x.c, 0, x.n, HW, cfg_.norm_groups, eps, fptr(g), fptr(gb), ab, ws, c.s);
    gn_conv_narrow(dt_, x.p, x.n, x.h, x.w, x.c, ab, 1, ptr(w), b.set ? fptr(b) : nullptr, cout, out, ldo, out_f32,
                   c.s);
  }
  if (ws) c.ws->free(ws);
  c.ws->free(ab);
  return true;
}

P Model::up2_weights(const std::string& name, int ch) {
  if (dt_ == F32) return P();   // (the fp32 parity engine keeps the resize conv: operation for operation the oracle)
  return reg(name, IRX_LAYOUT_CONV_UP2, dt_, {4 * ch, 2, 2, ch});
}

void Model::upsample_conv(Ctx& c, const Act& x, P w, P w2, P b, int cout, Act& out, bool stats) {
  // output pixel (2y + a, 2x + b) of nearest-2x + conv3x3 only sees low-resolution rows y - 1 + a .. y + a and columns
  // x - 1 + b .. x + b: parity p = 2a + b is a 2x2 conv of x with pad (1 - a, 1 - b) (include/irx.h
  // IRX_LAYOUT_CONV_UP2), stored at the strided high-resolution pixels (GemmArgs::up2_*): 4 / 9 of the MACs
  Act lo = out;
  lo.h = x.h; lo.w = x.w;
  GemmArgs a = conv_args(dt_, x, nullptr, w2.set ? ptr(w2) : nullptr, b.set ? fptr(b) : nullptr, cout, 2, 1, 1, 1, x.h,
                         x.w, lo, nullptr, 0, nullptr, 0, -1);
  a.up2_h = x.h; a.up2_w = x.w;
  if (!(w2.set && g_up2 && out.h == 2 * x.h && out.w == 2 * x.w && x.c == cout && gemm_up2_ok(a))) {
    conv2d(c, x, nullptr, w, b, cout, 3, 1, 1, 1, out.h, out.w, out, nullptr, 0, nullptr, 0, -1, stats);
    return;
  }
  if (stats && !out.gnp) {
    const int r = gemm_emits_gn_parts(a);
    if (r > 0 && ((long)x.h * x.w) % r == 0) {
      out.gnp = (double*)c.ws->alloc((size_t)(4L * a.M / r) * cout * 2 * sizeof(double));
      out.gnr = r;
    }
  }
  const size_t wsb = gemm_workspace_bytes(a);
  void* p = wsb ? c.ws->alloc(wsb) : nullptr;
  if (!c.ws->dry()) {
    const size_t per = (size_t)cout * 4 * x.c * dsize(dt_);   // one parity's [Cout][2][2][Cin]
    for (int par = 0; par < 4; ++par) {
      GemmArgs q = a;
      q.g.pad_t = 1 - (par >> 1);
      q.g.pad_l = 1 - (par & 1);
      q.B = (const char*)ptr(w2) + par * per;
      q.up2_p = par;
      q.gn_part = out.gnp;
      q.splitk_ws = p;
      q.splitk_ws_bytes = wsb;
      gemm(q, c.s);
    }
  }
  if (p) c.ws->free(p);
}

void Model::lnorm(Ctx& c, const void* x, int rows, int C, P g, P b, float eps, void* out) {
  if (c.ws->dry()) return;
  layer_norm(dt_, x, C, rows, C, eps, fptr(g), fptr(b), out, C, c.s);
}

static std::string join(const std::vector<std::string>& v) {
  std::string s;
  for (size_t i = 0; i < v.size(); ++i) s += (i ? "|" : "") + v[i];
  return s;
}

// ---------------------------------------------------------------------------------------------- UNet
ResW Unet::make_res(const std::string& p, int cin, int cout) {
  ResW r;
  r.cin = cin; r.cout = cout;
  r.n1w = vec(p + "norm1.weight", cin); r.n1b = vec(p + "norm1.bias", cin);
  r.c1w = conv(p + "conv1.weight", cout, 3, 3, cin); r.c1b = vec(p + "conv1.bias", cout);
  r.temb_off = temb_cols_;
  temb_cols_ += cout;
  temb_names_w_.push_back(p + "time_emb_proj.weight");
  temb_names_b_.push_back(p + "time_emb_proj.bias");
  r.n2w = vec(p + "norm2.weight", cout); r.n2b = vec(p + "norm2.bias", cout);
  r.c2w = conv(p + "conv2.weight", cout, 3, 3, cout); r.c2b = vec(p + "conv2.bias", cout);
  r.shortcut = cin != cout;
  if (r.shortcut) { r.scw = mat(p + "conv_shortcut.weight", cout, cin); r.scb = vec(p + "conv_shortcut.bias", cout); }
  return r;
}

Unet::XfW Unet::make_xf(const std::string& p, int c) {
  XfW a;
  a.c = c;
  const std::string b = p + "transformer_blocks.0.";
  a.nw = vec(p + "norm.weight", c); a.nb = vec(p + "norm.bias", c);
  a.piw = mat(p + "proj_in.weight", c, c); a.pib = vec(p + "proj_in.bias", c);
  a.ln1w = vec(b + "norm1.weight", c); a.ln1b = vec(b + "norm1.bias", c);
  // 16-bit engines: softmax scale * log2(e) folded into to_q (one rounding of q instead of two; the attention
  // kernel's exp2 then needs no multiply per score)
  const bool fold = dt_ != F32;
  const float qs = fold ? 1.4426950408889634f / std::sqrt((float)(c / cfg_.heads)) : 1.f;
  // LayerNorm fold (ln_fold_): each LN's gamma scales the columns of the projection it feeds, and the packer adds
  // u = row sums of the packed matrix and v = bias + W beta (layouts IRX_LAYOUT_VEC_LN_U / _LN_V)
  const bool lnf = ln_fold_;
  const std::string qkv = b + "attn1.to_q.weight|" + b + "attn1.to_k.weight|" + b + "attn1.to_v.weight";
  a.qkvw = reg(qkv, IRX_LAYOUT_MAT, dt_, {3 * c, c}, qs, fold ? c : 0, lnf ? b + "norm1.weight" : "");
  if (lnf) {
    a.qkvu = reg(qkv, IRX_LAYOUT_VEC_LN_U, F32, {3 * c});
    a.qkvv = reg(qkv, IRX_LAYOUT_VEC_LN_V, F32, {3 * c}, 1.f, 0, b + "norm1.bias;");
  }
  a.o1w = mat(b + "attn1.to_out.0.weight", c, c); a.o1b = vec(b + "attn1.to_out.0.bias", c);
  a.ln2w = vec(b + "norm2.weight", c); a.ln2b = vec(b + "norm2.bias", c);
  a.q2w = reg(b + "attn2.to_q.weight", IRX_LAYOUT_MAT, dt_, {c, c}, qs, fold ? c : 0, lnf ? b + "norm2.weight" : "");
  if (lnf) {
    a.q2u = reg(b + "attn2.to_q.weight", IRX_LAYOUT_VEC_LN_U, F32, {c});
    a.q2v = reg(b + "attn2.to_q.weight", IRX_LAYOUT_VEC_LN_V, F32, {c}, 1.f, 0, b + "norm2.bias;");
  }
  a.kv_off = kv_cols_;
  kv_cols_ += 2 * c;
  kv_names_.push_back(b + "attn2.to_k.weight");
  kv_names_.push_back(b + "attn2.to_v.weight");
  a.o2w = mat(b + "attn2.to_out.0.weight", c, c); a.o2b = vec(b + "attn2.to_out.0.bias", c);
  a.ln3w = vec(b + "norm3.weight", c); a.ln3b = vec(b + "norm3.bias", c);
  // GEGLU projection rows interleaved in (64 value, 64 gate) blocks so one output tile holds both halves
  const std::string ff = b + "ff.net.0.proj.weight";
  a.ffw = reg(ff, IRX_LAYOUT_MAT_GEGLU64, dt_, {8 * c, c}, 1.f, 0, lnf ? b + "norm3.weight" : "");
  a.ffb = reg(b + "ff.net.0.proj.bias", IRX_LAYOUT_VEC_GEGLU64, F32, {8 * c});
  if (lnf) {
    a.ffu = reg(ff, IRX_LAYOUT_VEC_LN_U, F32, {8 * c});
    a.ffv = reg(ff, IRX_LAYOUT_VEC_LN_V, F32, {8 * c}, 1.f, 0, b + "norm3.bias;" + b + "ff.net.0.proj.bias");
  }
  a.ff2w = mat(b + "ff.net.2.weight", c, 4 * c); a.ff2b = vec(b + "ff.net.2.bias", c);
  a.pow = mat(p + "proj_out.weight", c, c); a.pob = vec(p + "proj_out.bias", c);
  if (dt_ != F32) {   // (the fp32 parity engine keeps the two layers: operation for operation the oracle)
    const std::string ch = p + "proj_out.weight|" + b + "ff.net.2.weight";
    a.pofw = reg(ch, IRX_LAYOUT_MAT_CHAIN, dt_, {c, 5 * c});
    a.pofb = reg(ch, IRX_LAYOUT_VEC_CHAIN, F32, {c}, 1.f, 0, p + "proj_out.bias;" + b + "ff.net.2.bias");
  }
  return a;
}

Unet::Unet(const irx_model_config& cfg, int dtype) : Model(IRX_MODEL_UNET, cfg, dtype) {
  IRX_CHECK(cfg.n_blocks >= 2 && cfg.n_blocks <= 8, "bad UNet block count");
  IRX_CHECK(cfg.heads > 0 && cfg.norm_groups > 0, "bad UNet config");
  const int* bo = cfg.block_out_channels;
  const int nb = cfg.n_blocks;
  // 16-bit engines: the input is padded to one 64-channel slab, so conv_in runs on the large-tile conv paths (the halo
  // tiles at 64x64 latents) instead of the 4-wave kernel (zero channels cost MFMAs, not bandwidth: 75 -> ~20 us)
  cin_pad_ = dtype != F32 ? (cfg.in_channels + 63) / 64 * 64 : (cfg.in_channels + 7) / 8 * 8;
  ln_fold_ = dtype != F32 && g_ln_fold;
  temb_dim_ = bo[0] * 4;
  conv_in_w = conv("conv_in.weight", bo[0], 3, 3, cin_pad_);
  conv_in_b = vec("conv_in.bias", bo[0]);
  t1w = mat("time_embedding.linear_1.weight", temb_dim_, bo[0]); t1b = vec("time_embedding.linear_1.bias", temb_dim_);
  t2w = mat("time_embedding.linear_2.weight", temb_dim_, temb_dim_); t2b = vec("time_embedding.linear_2.bias", temb_dim_);
  int cout = bo[0];
  for (int i = 0; i < nb; ++i) {
    Block blk;
    const int cin = cout;
    cout = bo[i];
    blk.ch = cout;
    blk.has_attn = cfg.down_attn[i] != 0;
    for (int j = 0; j < cfg.layers_per_block; ++j) {
      const std::string p = "down_blocks." + std::to_string(i) + ".";
      blk.res.push_back(make_res(p + "resnets." + std::to_string(j) + ".", j == 0 ? cin : cout, cout));
      if (blk.has_attn) blk.attn.push_back(make_xf(p + "attentions." + std::to_string(j) + ".", cout));
    }
    blk.resample = i < nb - 1;
    if (blk.resample) {
      const std::string p = "down_blocks." + std::to_string(i) + ".downsamplers.0.conv.";
      blk.rsw = conv(p + "weight", cout, 3, 3, cout); blk.rsb = vec(p + "bias", cout);
    }
    down_.push_back(blk);
  }
  const int c = bo[nb - 1];
  mid_res0_ = make_res("mid_block.resnets.0.", c, c);
  mid_attn_ = make_xf("mid_block.attentions.0.", c);
  mid_res1_ = make_res("mid_block.resnets.1.", c, c);
  // up path: diffusers channel bookkeeping (prev_output_channel / res_skip_channels)
  int out_ch = bo[nb - 1];
  for (int i = 0; i < nb; ++i) {
    Block blk;
    const int prev = out_ch;
    out_ch = bo[nb - 1 - i];
    const int in_ch = bo[std::max(nb - 2 - i, 0)];
    blk.ch = out_ch;
    blk.has_attn = cfg.up_attn[i] != 0;
    for (int j = 0; j <= cfg.layers_per_block; ++j) {
      const int skip = j == cfg.layers_per_block ? in_ch : out_ch;
      const int rin = j == 0 ? prev : out_ch;
      const std::string p = "up_blocks." + std::to_string(i) + ".";
      blk.res.push_back(make_res(p + "resnets." + std::to_string(j) + ".", rin + skip, out_ch));
      if (blk.has_attn) blk.attn.push_back(make_xf(p + "attentions." + std::to_string(j) + ".", out_ch));
    }
    blk.resample = i < nb - 1;
    if (blk.resample) {
      const std::string p = "up_blocks." + std::to_string(i) + ".upsamplers.0.conv.";
      blk.rsw = conv(p + "weight", out_ch, 3, 3, out_ch); blk.rsb = vec(p + "bias", out_ch);
      blk.rsw2 = up2_weights(p + "weight", out_ch);
    }
    up_.push_back(blk);
  }
  nout_w = vec("conv_norm_out.weight", bo[0]); nout_b = vec("conv_norm_out.bias", bo[0]);
  conv_out_w = conv("conv_out.weight", cfg.out_channels, 3, 3, bo[0]);
  conv_out_b = vec("conv_out.bias", cfg.out_channels);
  // fused projections
  tpw = mat(join(temb_names_w_), temb_cols_, temb_dim_);
  tpb = vec(join(temb_names_b_), temb_cols_);
  kvw = mat(join(kv_names_), kv_cols_, cfg.cross_attention_dim);
}

Act Unet::resnet(Ctx& c, const ResW& r, Act& x0, Act* x1, const float* tproj, float eps) {
  const int B = x0.n, H = x0.h, W = x0.w;
  const int cin = x0.c + (x1 ? x1->c : 0);
  IRX_CHECK(cin == r.cin, "resnet channel mismatch");
  Act h1 = new_act(c, B, H, W, r.cout);
  gn_conv3(c, x0, x1, r.n1w, r.n1b, eps, 1, r.c1w, r.c1b, r.cout, h1, tproj ? tproj + r.temb_off : nullptr,
           temb_cols_, nullptr, true);
  Act sc;
  const void* res = x0.p;
  if (r.shortcut) {
    sc = new_act(c, B, H, W, r.cout);
    conv2d(c, x0, x1, r.scw, r.scb, r.cout, 1, 1, 0, 0, H, W, sc);
    res = sc.p;
  }
  Act out = new_act(c, B, H, W, r.cout);
  gn_conv3(c, h1, nullptr, r.n2w, r.n2b, eps, 1, r.c2w, r.c2b, r.cout, out, nullptr, 0, res, true);
  drop(c, h1);
  if (r.shortcut) drop(c, sc);
  return out;
}

void Unet::ln_gemm(Ctx& c, GemmArgs& g, const void* x, int rows, int C, P lnw, P lnb, P u, P v, const float* bias,
                   void* nbuf, float2* st, const float2* parts) {
  g.lda = C;
  if (!ln_fold_) {
    lnorm(c, x, rows, C, lnw, lnb, 1e-5f, nbuf);
    g.A = nbuf;
    g.bias = bias;
  } else {
    g.bias = fptr(v);                 // bias + W beta
    g.A = x;
    g.ln_u = fptr(u);
    g.ln_rs = parts ? parts : st;     // (the producer of x wrote its rows' statistics: no pass over x)
    if (gemm_ln_foldable(g)) {
      if (!parts && !c.ws->dry()) layer_norm_stats(dt_, x, C, rows, C, 1e-5f, st, c.s);
    } else {                          // (W * gamma, bias + W beta) after an affine-free LayerNorm
      g.ln_rs = nullptr;
      g.ln_part = nullptr;
      g.ln_u = nullptr;
      if (!c.ws->dry()) layer_norm(dt_, x, C, rows, C, 1e-5f, nullptr, nullptr, nbuf, C, c.s);
      g.A = nbuf;
    }
  }
  run_gemm(c, g);
}

const float2* Unet::xf_proj(Ctx& c, const void* A, int M, int C, P w, const float* bias, void* out,
                            const void* residual, int imgs, float2* lnp) {
  GemmArgs a;
  a.dtype = dt_;
  a.M = M; a.N = C; a.K = C;
  a.A = A; a.lda = C;
  a.B = ptr(w); a.ldb = C;
  a.C = out; a.ldc = C;
  a.bias = bias;
  a.residual = residual; a.ldr = C;
  a.imgs = imgs;
  a.ln_out_rs = 1;
  a.ln_eps = 1e-5f;
  const bool emit = lnp && gemm_emits_ln_parts(a);   // (shape-only decision: the dry run decides the same)
  if (emit) a.ln_out = lnp;
  run_gemm(c, a);
  return emit ? lnp : nullptr;
}

Act Unet::transformer(Ctx& c, const XfW& a, Act& x, const void* kv, int L) {
  const int B = x.n, HW = x.h * x.w, C = a.c;
  const long M = (long)B * HW;
  const size_t es = dsize(dt_);
  const int heads = cfg_.heads, d = C / heads;
  const float scale = 1.0f / std::sqrt((float)d);
  Act h = new_act(c, B, x.h, x.w, C);
  // LayerNorm row statistics of the residual stream h, written by the projections that write it (GemmArgs::ln_out,
  // final (rstd, rstd * mean) rows: C == 320, the 64x64 level, where a 320-column tile holds the whole row; the
  // wider levels keep the statistics pass — their two-partial merge in the consumers' epilogues measured slower)
  float2* lnp = (ln_fold_ && C == kLnGroup) ? (float2*)c.ws->alloc(M * sizeof(float2)) : nullptr;
  const float2* parts = nullptr;
  // GroupNorm (no SiLU) -> proj_in: folded into per-image weights where they stay small next to the activation
  // (C == 320, the 64x64 level: 16 x 200 KB against 2 x 42 MB of gn_apply traffic; at 32x32 the 13 MB of per-image
  // weights cost what they save): proj_in(GN(x)) = x (W diag(a_i))^T + (bias + W b_i) for image i with
  // GN(x) = x * a_i + b_i per channel — the normalised tensor is neither written nor read
  GemmArgs pg;
  pg.dtype = dt_; pg.M = M; pg.N = C; pg.K = C;
  pg.A = x.p; pg.lda = C; pg.ldb = C;
  pg.C = h.p; pg.ldc = C;
  pg.imgs = B;
  pg.b_rows = HW; pg.b_img_stride = (long)C * C; pg.bias_img_stride = C;
  pg.B = ptr(a.piw);   // (placeholder for the shape checks: the folded copies replace it below)
  if (dt_ != F32 && g_gn_fold && C <= 320 && x.gnp && HW % x.gnr == 0 && gemm_bimg_ok(pg)) {
    float2* ab = (float2*)c.ws->alloc((size_t)B * C * sizeof(float2));
    void* wf = c.ws->alloc((size_t)B * C * C * es);
    float* bf = (float*)c.ws->alloc((size_t)B * C * sizeof(float));
    float2* mr = (float2*)c.ws->alloc((size_t)B * cfg_.norm_groups * sizeof(float2));
    if (!c.ws->dry()) {
      group_norm_parts_ab(C, B, HW, cfg_.norm_groups, 1e-6f, fptr(a.nw), fptr(a.nb), x.gnp, x.gnr, ab, mr, c.s);
      gn_fold_weights(dt_, ptr(a.piw), fptr(a.pib), ab, fptr(a.nb), mr, cfg_.norm_groups, C, C, B, wf, bf, c.s);
    }
    pg.B = wf;
    pg.bias = bf;
    pg.ln_out_rs = 1;
    pg.ln_eps = 1e-5f;
    if (lnp && gemm_emits_ln_parts(pg)) {
      pg.ln_out = lnp;
      parts = lnp;
    }
    run_gemm(c, pg);
    c.ws->free(mr);
    c.ws->free(bf);
    c.ws->free(wf);
    c.ws->free(ab);
  } else {
    Act gn = new_act(c, B, x.h, x.w, C);
    gnorm(c, x, nullptr, a.nw, a.nb, 1e-6f, 0, gn);
    parts = xf_proj(c, gn.p, M, C, a.piw, fptr(a.pib), h.p, nullptr, B, lnp);
    drop(c, gn);
  }
  void* n = c.ws->alloc(M * C * es);
  void* att = c.ws->alloc(M * C * es);
  float2* st = ln_fold_ ? (float2*)c.ws->alloc(M * sizeof(float2)) : nullptr;   // LayerNorm row statistics
  // self-attention
  void* qkv = c.ws->alloc(M * 3 * C * es);
  // 16-bit engines: q|k|v written head-major ([q|k|v][image][head][token][d], GemmArgs::hs_*) so each attention
  // block streams its head's K / V rows contiguously
  const bool hm = dt_ != F32 && g_attn_hm;
  {
    GemmArgs g;
    g.dtype = dt_; g.M = M; g.N = 3 * C; g.K = C;
    g.B = ptr(a.qkvw); g.ldb = C;
    g.C = qkv; g.ldc = 3 * C; g.imgs = B;
    if (hm) { g.hs_L = HW; g.hs_C = C; g.hs_d = d; }
    ln_gemm(c, g, h.p, M, C, a.ln1w, a.ln1b, a.qkvu, a.qkvv, nullptr, n, st, parts);
  }
  if (!c.ws->dry()) {
    AttnArgs aa;
    aa.dtype = dt_; aa.B = B; aa.H = heads; aa.Lq = HW; aa.Lk = HW; aa.d = d; aa.scale = scale;
    aa.q_scaled = dt_ != F32;
    if (hm) {
      const long hs = (long)HW * d, bs = (long)heads * hs;
      aa.q = qkv; aa.ldq = d; aa.sq = bs; aa.hsq = hs;
      aa.k = (char*)qkv + M * C * es; aa.ldk = d; aa.sk = bs; aa.hsk = hs;
      aa.v = (char*)qkv + 2 * M * C * es; aa.ldv = d; aa.sv = bs; aa.hsv = hs;
    } else {
      aa.q = qkv; aa.ldq = 3 * C; aa.sq = (long)HW * 3 * C;
      aa.k = (char*)qkv + C * es; aa.ldk = 3 * C; aa.sk = aa.sq;
      aa.v = (char*)qkv + 2 * C * es; aa.ldv = 3 * C; aa.sv = aa.sq;
    }
    aa.o = att; aa.ldo = C; aa.so = (long)HW * C;
    attention(aa, c.s);
  }
  c.ws->free(qkv);
  parts = xf_proj(c, att, M, C, a.o1w, fptr(a.o1b), h.p, h.p, B, lnp);
  // cross-attention (K|V precomputed per prompt)
  {
    GemmArgs g;
    g.dtype = dt_; g.M = M; g.N = C; g.K = C;
    g.B = ptr(a.q2w); g.ldb = C;
    g.C = att; g.ldc = C; g.imgs = B;
    if (hm) { g.hs_L = HW; g.hs_C = C; g.hs_d = d; }
    ln_gemm(c, g, h.p, M, C, a.ln2w, a.ln2b, a.q2u, a.q2v, nullptr, n, st, parts);
  }
  if (!c.ws->dry()) {
    AttnArgs aa;
    aa.dtype = dt_; aa.B = B; aa.H = heads; aa.Lq = HW; aa.Lk = L; aa.d = d; aa.scale = scale;
    aa.q_scaled = dt_ != F32;
    if (hm) { aa.q = att; aa.ldq = d; aa.sq = (long)heads * HW * d; aa.hsq = (long)HW * d; }
    else { aa.q = att; aa.ldq = C; aa.sq = (long)HW * C; }
    aa.k = (const char*)kv + a.kv_off * es; aa.ldk = kv_cols_; aa.sk = (long)L * kv_cols_;
    aa.v = (const char*)kv + (a.kv_off + C) * es; aa.ldv = kv_cols_; aa.sv = aa.sk;
    aa.o = n; aa.ldo = C; aa.so = (long)HW * C;
    attention(aa, c.s);
  }
  parts = xf_proj(c, n, M, C, a.o2w, fptr(a.o2b), h.p, h.p, B, lnp);
  // GEGLU feed-forward: fused into the projection's epilogue when the large-tile path takes the shape
  void* g = c.ws->alloc(M * 4 * C * es);
  {
    GemmArgs ga;
    ga.dtype = dt_; ga.M = M; ga.N = 8 * C; ga.K = C;
    ga.B = ptr(a.ffw); ga.ldb = C;
    ga.C = g; ga.ldc = 4 * C; ga.geglu = 1;
    ga.imgs = B;
    ga.A = h.p; ga.lda = C;
    if (gemm_geglu_fusable(ga)) {
      ln_gemm(c, ga, h.p, M, C, a.ln3w, a.ln3b, a.ffu, a.ffv, fptr(a.ffb), n, st, parts);
    } else {
      void* ff = c.ws->alloc(M * 8 * C * es);
      ga.geglu = 0; ga.C = ff; ga.ldc = 8 * C;
      ln_gemm(c, ga, h.p, M, C, a.ln3w, a.ln3b, a.ffu, a.ffv, fptr(a.ffb), n, st, parts);
      if (!c.ws->dry()) geglu(dt_, ff, 8 * C, M, 4 * C, g, 4 * C, 1, c.s);
      c.ws->free(ff);
    }
  }
  if (a.pofw.set && g_ff_chain) {
    // ff.net.2 -> (+ h) -> proj_out (+ x) as ONE GEMM: nothing non-linear sits between the two layers, so
    //   proj_out(h + ff2(g)) + x = [W_po | W_po W_ff2] [h; g] + (b_po + W_po b_ff2) + x
    // a 1x1 conv over the channel concat (h | g) (K = 5C): the ff2 output is neither written nor re-read and one
    // launch goes (include/irx.h IRX_LAYOUT_MAT_CHAIN)
    if (st) c.ws->free(st);
    c.ws->free(att);
    c.ws->free(n);
    if (lnp) c.ws->free(lnp);
    Act ga;
    ga.p = g; ga.n = B; ga.h = x.h; ga.w = x.w; ga.c = 4 * C;
    Act out = new_act(c, B, x.h, x.w, C);
    conv2d(c, h, &ga, a.pofw, a.pofb, C, 1, 1, 0, 0, x.h, x.w, out, nullptr, 0, x.p, 0, -1, true);
    c.ws->free(g);
    drop(c, h);
    return out;
  }
  linear(c, g, 4 * C, M, 4 * C, a.ff2w, C, fptr(a.ff2b), h.p, C, ACT_NONE, h.p, C, 0, B);
  c.ws->free(g);
  if (st) c.ws->free(st);
  c.ws->free(att);
  c.ws->free(n);
  if (lnp) c.ws->free(lnp);
  Act out = new_act(c, B, x.h, x.w, C);
  linear(c, h.p, C, M, C, a.pow, C, fptr(a.pob), out.p, C, ACT_NONE, x.p, C, 0, B, &out);
  drop(c, h);
  return out;
}

void Unet::run(Ctx& c, const void* x, int B, int h, int w, const float* t, const void* kv, int L, float* eps_out) {
  const int* bo = cfg_.block_out_channels;
  const float eps = cfg_.norm_eps;
  const size_t es = dsize(dt_);
  // time embedding: sinusoid -> linear_1 -> SiLU -> linear_2, then SiLU(emb) (every resnet's input) and all
  // resnets' time_emb_proj in one GEMM
  void* te0 = c.ws->alloc((size_t)B * bo[0] * es);
  void* te1 = c.ws->alloc((size_t)B * temb_dim_ * es);
  void* te2 = c.ws->alloc((size_t)B * temb_dim_ * es);
  float* tproj = (float*)c.ws->alloc((size_t)B * temb_cols_ * sizeof(float));
  if (!c.ws->dry()) timestep_embed(dt_, t, B, bo[0], cfg_.flip_sin_to_cos, cfg_.freq_shift, te0, c.s);
  linear(c, te0, bo[0], B, bo[0], t1w, temb_dim_, fptr(t1b), te1, temb_dim_, ACT_SILU, nullptr, 0, 0, B);
  linear(c, te1, temb_dim_, B, temb_dim_, t2w, temb_dim_, fptr(t2b), te2, temb_dim_, ACT_SILU, nullptr, 0, 0, B);
  linear(c, te2, temb_dim_, B, temb_dim_, tpw, temb_cols_, fptr(tpb), tproj, temb_cols_, ACT_NONE, nullptr, 0, 1, B);
  c.ws->free(te0);
  c.ws->free(te1);
  c.ws->free(te2);

  Act xin;
  xin.p = const_cast<void*>(x); xin.n = B; xin.h = h; xin.w = w; xin.c = cin_pad_;
  Act cur = new_act(c, B, h, w, bo[0]);
  conv2d(c, xin, nullptr, conv_in_w, conv_in_b, bo[0], 3, 1, 1, 1, h, w, cur, nullptr, 0, nullptr, 0, -1, true);
  std::vector<Act> skips{cur};
  bool cur_is_skip = true;
  for (auto& blk : down_) {
    for (size_t j = 0; j < blk.res.size(); ++j) {
      Act nx = resnet(c, blk.res[j], cur, nullptr, tproj, eps);
      if (!cur_is_skip) drop(c, cur);
      if (blk.has_attn) {
        Act t2 = transformer(c, blk.attn[j], nx, kv, L);
        drop(c, nx);
        nx = t2;
      }
      skips.push_back(nx);
      cur = nx;
      cur_is_skip = true;
    }
    if (blk.resample) {
      const int Ho = (cur.h - 1) / 2 + 1, Wo = (cur.w - 1) / 2 + 1;
      Act d = new_act(c, B, Ho, Wo, blk.ch);
      conv2d(c, cur, nullptr, blk.rsw, blk.rsb, blk.ch, 3, 2, 1, 1, cur.h, cur.w, d, nullptr, 0, nullptr, 0, -1, true);
      skips.push_back(d);
      cur = d;
    }
  }
  {
    Act r = resnet(c, mid_res0_, cur, nullptr, tproj, eps);
    Act a = transformer(c, mid_attn_, r, kv, L);
    drop(c, r);
    cur = resnet(c, mid_res1_, a, nullptr, tproj, eps);
    drop(c, a);
  }
  for (auto& blk : up_) {
    for (size_t j = 0; j < blk.res.size(); ++j) {
      Act skip = skips.back();
      skips.pop_back();
      Act nx = resnet(c, blk.res[j], cur, &skip, tproj, eps);
      drop(c, cur);
      drop(c, skip);
      if (blk.has_attn) {
        Act t2 = transformer(c, blk.attn[j], nx, kv, L);
        drop(c, nx);
        nx = t2;
      }
      cur = nx;
    }
    if (blk.resample) {
      // Upsample2D: nearest resize to the next skip's size (== 2x unless a latent side is not /8)
      const int th = skips.back().h, tw = skips.back().w;
      Act u = new_act(c, B, th, tw, blk.ch);
      upsample_conv(c, cur, blk.rsw, blk.rsw2, blk.rsb, blk.ch, u, true);
      drop(c, cur);
      cur = u;
    }
  }
  if (gn_conv_out(c, cur, nout_w, nout_b, eps, conv_out_w, conv_out_b, cfg_.out_channels, eps_out, cfg_.out_channels,
                  1)) {
    drop(c, cur);
  } else {
    Act gn = new_act(c, B, h, w, bo[0]);
    gnorm(c, cur, nullptr, nout_w, nout_b, eps, 1, gn);
    drop(c, cur);
    Act o;
    o.p = eps_out; o.n = B; o.h = h; o.w = w; o.c = cfg_.out_channels;
    conv2d(c, gn, nullptr, conv_out_w, conv_out_b, cfg_.out_channels, 3, 1, 1, 1, h, w, o, nullptr, 0, nullptr, 1);
    drop(c, gn);
  }
  c.ws->free(tproj);
}

size_t Unet::workspace_bytes(int B, int h, int w) {
  Arena ar;
  ar.reset(nullptr, 0);
  Ctx c{nullptr, &ar};
  run(c, nullptr, B, h, w, nullptr, nullptr, 77, nullptr);
  return ar.peak();
}

void Unet::forward(hipStream_t s, const void* x, int B, int h, int w, const float* t, const void* kv, int L,
                   float* eps, char* ws, size_t cap) {
  IRX_CHECK(blob_, "weights not bound");
  Arena ar;
  ar.reset(ws, cap);
  Ctx c{s, &ar};
  run(c, x, B, h, w, t, kv, L, eps);
}

void Unet::prepare_context(hipStream_t s, const void* ctx, int B, int L, void* kv, char* ws, size_t cap) {
  IRX_CHECK(blob_, "weights not bound");
  (void)ws; (void)cap;
  Arena ar;
  ar.reset(ws ? ws : (char*)16, cap);   // no temporaries needed
  Ctx c{s, &ar};
  linear(c, ctx, cfg_.cross_attention_dim, B * L, cfg_.cross_attention_dim, kvw, kv_cols_, nullptr, kv, kv_cols_,
         ACT_NONE, nullptr, 0, 0, B);
}

// ---------------------------------------------------------------------------------------------- VAE
ResW Vae::make_res(const std::string& p, int cin, int cout) {
  ResW r;
  r.cin = cin; r.cout = cout;
  r.n1w = vec(p + "norm1.weight", cin); r.n1b = vec(p + "norm1.bias", cin);
  r.c1w = conv(p + "conv1.weight", cout, 3, 3, cin); r.c1b = vec(p + "conv1.bias", cout);
  r.n2w = vec(p + "norm2.weight", cout); r.n2b = vec(p + "norm2.bias", cout);
  r.c2w = conv(p + "conv2.weight", cout, 3, 3, cout); r.c2b = vec(p + "conv2.bias", cout);
  r.shortcut = cin != cout;
  if (r.shortcut) { r.scw = mat(p + "conv_shortcut.weight", cout, cin); r.scb = vec(p + "conv_shortcut.bias", cout); }
  return r;
}

Vae::AttW Vae::make_attn(const std::string& p, int c) {
  AttW a;
  a.c = c;
  a.gw = vec(p + "group_norm.weight", c); a.gb = vec(p + "group_norm.bias", c);
  a.qkvw = mat(p + "to_q.weight|" + p + "to_k.weight|" + p + "to_v.weight", 3 * c, c);
  a.qkvb = vec(p + "to_q.bias|" + p + "to_k.bias|" + p + "to_v.bias", 3 * c);
  a.ow = mat(p + "to_out.0.weight", c, c); a.ob = vec(p + "to_out.0.bias", c);
  return a;
}

Vae::Vae(const irx_model_config& cfg, int dtype) : Model(IRX_MODEL_VAE, cfg, dtype) {
  const int* bo = cfg.block_out_channels;
  const int nb = cfg.n_blocks;
  const int L = cfg.latent_channels;
  IRX_CHECK(L <= 4 && cfg.in_channels <= 8 && cfg.out_channels <= 4, "VAE channel counts out of range");
  e_cin_w = conv("encoder.conv_in.weight", bo[0], 3, 3, 8); e_cin_b = vec("encoder.conv_in.bias", bo[0]);
  int cout = bo[0];
  for (int i = 0; i < nb; ++i) {
    const int cin = cout;
    cout = bo[i];
    std::vector<ResW> rs;
    for (int j = 0; j < cfg.layers_per_block; ++j)
      rs.push_back(make_res("encoder.down_blocks." + std::to_string(i) + ".resnets." + std::to_string(j) + ".",
                            j == 0 ? cin : cout, cout));
    e_res_.push_back(rs);
    if (i < nb - 1) {
      const std::string p = "encoder.down_blocks." + std::to_string(i) + ".downsamplers.0.conv.";
      e_down_w_.push_back(conv(p + "weight", cout, 3, 3, cout));
      e_down_b_.push_back(vec(p + "bias", cout));
    }
  }
  const int c = bo[nb - 1];
  e_mid0_ = make_res("encoder.mid_block.resnets.0.", c, c);
  e_att_ = make_attn("encoder.mid_block.attentions.0.", c);
  e_mid1_ = make_res("encoder.mid_block.resnets.1.", c, c);
  e_nout_w = vec("encoder.conv_norm_out.weight", c); e_nout_b = vec("encoder.conv_norm_out.bias", c);
  e_cout_w = conv("encoder.conv_out.weight", 8, 3, 3, c); e_cout_b = vec("encoder.conv_out.bias", 8);
  qw = mat("quant_conv.weight", 8, 8); qb = vec("quant_conv.bias", 8);
  pqw = mat("post_quant_conv.weight", 8, 8); pqb = vec("post_quant_conv.bias", 8);
  d_cin_w = conv("decoder.conv_in.weight", c, 3, 3, 8); d_cin_b = vec("decoder.conv_in.bias", c);
  d_mid0_ = make_res("decoder.mid_block.resnets.0.", c, c);
  d_att_ = make_attn("decoder.mid_block.attentions.0.", c);
  d_mid1_ = make_res("decoder.mid_block.resnets.1.", c, c);
  int out_ch = bo[nb - 1];
  for (int i = 0; i < nb; ++i) {
    const int prev = out_ch;
    out_ch = bo[nb - 1 - i];
    std::vector<ResW> rs;
    for (int j = 0; j <= cfg.layers_per_block; ++j)
      rs.push_back(make_res("decoder.up_blocks." + std::to_string(i) + ".resnets." + std::to_string(j) + ".",
                            j == 0 ? prev : out_ch, out_ch));
    d_res_.push_back(rs);
    if (i < nb - 1) {
      const std::string p = "decoder.up_blocks." + std::to_string(i) + ".upsamplers.0.conv.";
      d_up_w_.push_back(conv(p + "weight", out_ch, 3, 3, out_ch));
      d_up_b_.push_back(vec(p + "bias", out_ch));
      d_up2_w_.push_back(up2_weights(p + "weight", out_ch));
    }
  }
  d_nout_w = vec("decoder.conv_norm_out.weight", bo[0]); d_nout_b = vec("decoder.conv_norm_out.bias", bo[0]);
  d_cout_w = conv("decoder.conv_out.weight", 4, 3, 3, bo[0]); d_cout_b = vec("decoder.conv_out.bias", 4);
}

Act Vae::resnet(Ctx& c, const ResW& r, Act& x) {
  const float eps = cfg_.norm_eps;
  const int B = x.n, H = x.h, W = x.w;
  Act h1 = new_act(c, B, H, W, r.cout);
  gn_conv3(c, x, nullptr, r.n1w, r.n1b, eps, 1, r.c1w, r.c1b, r.cout, h1, nullptr, 0, nullptr, true);
  Act sc;
  const void* res = x.p;
  if (r.shortcut) {
    sc = new_act(c, B, H, W, r.cout);
    conv2d(c, x, nullptr, r.scw, r.scb, r.cout, 1, 1, 0, 0, H, W, sc);
    res = sc.p;
  }
  Act out = new_act(c, B, H, W, r.cout);
  gn_conv3(c, h1, nullptr, r.n2w, r.n2b, eps, 1, r.c2w, r.c2b, r.cout, out, nullptr, 0, res, true);
  drop(c, h1);
  if (r.shortcut) drop(c, sc);
  return out;
}

// Mid-block single-head attention (d = 512).  16-bit engines: one flash launch (attnw_kernel).  fp32 (the
// parity engine) and option vae_flash = 0: row-blocked, V transposed once, then per block of query rows
// (all images batched) fp32 scores S = Q K^T * C^-1/2 -> row softmax -> P V, with the score block capped
// at kVaeScoreBytes whatever the resolution (8 x 9216^2 fp32 scores at 768^2 would be 2.7 GB).  Every row
// is computed exactly as in one block (K-ordered MFMA sums, no split-K at K = 512 / HWp), so the result does
// not depend on the blocking.  The key axis is padded to a multiple of 8 (zero probabilities / zero V^T
// columns) so the PV contraction stays 16-byte aligned.
constexpr size_t kVaeScoreBytes = 128u << 20;
int g_vae_attn_rows = 0;
int g_vae_flash = 1;       // irx_set_option("vae_flash", 0): the row-blocked GEMM form in the 16-bit engines too   // irx_set_option("vae_attn_rows", R): force R query rows per block (tests); 0 = auto

Act Vae::attn(Ctx& c, const AttW& a, Act& x) {
  const int B = x.n, HW = x.h * x.w, C = a.c;
  const int HWp = (HW + 7) / 8 * 8;
  const long M = (long)B * HW;
  const size_t es = dsize(dt_);
  Act gn = new_act(c, B, x.h, x.w, C);
  gnorm(c, x, nullptr, a.gw, a.gb, cfg_.norm_eps, 0, gn);
  void* qkv = c.ws->alloc(M * 3 * C * es);
  linear(c, gn.p, C, M, C, a.qkvw, 3 * C, fptr(a.qkvb), qkv, 3 * C, ACT_NONE, nullptr, 0, 0, B);
  drop(c, gn);
  if (dt_ != F32 && C == 512 && g_vae_flash) {
    // 16-bit engines: one flash-attention launch (attnw_kernel), no score memory at all
    void* O = c.ws->alloc(M * C * es);
    if (!c.ws->dry()) {
      AttnArgs aa;
      aa.dtype = dt_; aa.B = B; aa.H = 1; aa.Lq = HW; aa.Lk = HW; aa.d = C;
      aa.scale = 1.0f / std::sqrt((float)C);
      aa.q = qkv; aa.ldq = 3 * C; aa.sq = (long)HW * 3 * C;
      aa.k = (char*)qkv + C * es; aa.ldk = 3 * C; aa.sk = aa.sq;
      aa.v = (char*)qkv + 2 * C * es; aa.ldv = 3 * C; aa.sv = aa.sq;
      aa.o = O; aa.ldo = C; aa.so = (long)HW * C;
      attention(aa, c.s);
    }
    c.ws->free(qkv);
    Act out = new_act(c, B, x.h, x.w, C);
    linear(c, O, C, M, C, a.ow, C, fptr(a.ob), out.p, C, ACT_NONE, x.p, C, 0, B, &out);
    c.ws->free(O);
    return out;
  }
  void* VT = c.ws->alloc((size_t)B * C * HWp * es);
  if (!c.ws->dry()) {
    if (HWp != HW) IRX_HIP(hipMemsetAsync(VT, 0, (size_t)B * C * HWp * es, c.s));
    transpose2d(dt_, (char*)qkv + 2 * C * es, 3 * C, HW, C, VT, HWp, B, (long)HW * 3 * C, (long)C * HWp, c.s);
  }
  // query rows per block: a multiple of 256 (whole tiles) within the score cap, or all rows
  long rb = (long)(kVaeScoreBytes / ((size_t)B * HWp * sizeof(float))) / 256 * 256;
  const int R = g_vae_attn_rows > 0 ? std::min(HW, g_vae_attn_rows) : (int)std::min<long>(HW, std::max<long>(256, rb));
  float* S = (float*)c.ws->alloc((size_t)B * R * HWp * sizeof(float));
  void* P = c.ws->alloc((size_t)B * R * HWp * es);
  void* O = c.ws->alloc(M * C * es);
  for (int r0 = 0; r0 < HW && !c.ws->dry(); r0 += R) {
    const int rows = std::min(R, HW - r0);
    GemmArgs g;
    g.dtype = dt_; g.M = rows; g.N = HW; g.K = C;
    g.A = (char*)qkv + (size_t)r0 * 3 * C * es; g.lda = 3 * C; g.sA = (long)HW * 3 * C;
    g.B = (char*)qkv + C * es; g.ldb = 3 * C; g.sB = g.sA;
    g.C = S; g.ldc = HWp; g.sC = (long)R * HWp; g.out_f32 = 1;
    g.alpha = 1.0f / std::sqrt((float)C);
    g.batch = B;
    g.imgs = B;
    gemm(g, c.s);
    softmax_rows(dt_, S, HWp, B * R, HW, P, HWp, c.s);   // writes zeros in cols [HW, HWp); rows past `rows`
                                                          // of each image hold stale scores and are never read
    GemmArgs h;
    h.dtype = dt_; h.M = rows; h.N = C; h.K = HWp;
    h.A = P; h.lda = HWp; h.sA = (long)R * HWp;
    h.B = VT; h.ldb = HWp; h.sB = (long)C * HWp;
    h.C = (char*)O + (size_t)r0 * C * es; h.ldc = C; h.sC = (long)HW * C;
    h.batch = B;
    h.imgs = B;
    gemm(h, c.s);
  }
  c.ws->free(S);
  c.ws->free(P);
  c.ws->free(qkv);
  c.ws->free(VT);
  Act out = new_act(c, B, x.h, x.w, C);
  linear(c, O, C, M, C, a.ow, C, fptr(a.ob), out.p, C, ACT_NONE, x.p, C, 0, B, &out);
  c.ws->free(O);
  return out;
}

void Vae::run_encode(Ctx& c, const void* img, int B, int H, int W, void* moments) {
  const int* bo = cfg_.block_out_channels;
  const int nb = cfg_.n_blocks;
  Act x;
  x.p = const_cast<void*>(img); x.n = B; x.h = H; x.w = W; x.c = 8;
  Act cur = new_act(c, B, H, W, bo[0]);
  conv2d(c, x, nullptr, e_cin_w, e_cin_b, bo[0], 3, 1, 1, 1, H, W, cur, nullptr, 0, nullptr, 0, -1, true);
  for (int i = 0; i < nb; ++i) {
    for (auto& r : e_res_[i]) {
      Act nx = resnet(c, r, cur);
      drop(c, cur);
      cur = nx;
    }
    if (i < nb - 1) {
      // Downsample2D(padding=0): F.pad(x, (0,1,0,1)) then 3x3 stride-2 conv
      const int Ho = (cur.h + 1 - 3) / 2 + 1, Wo = (cur.w + 1 - 3) / 2 + 1;
      Act d = new_act(c, B, Ho, Wo, cur.c);
      conv2d(c, cur, nullptr, e_down_w_[i], e_down_b_[i], cur.c, 3, 2, 0, 0, cur.h, cur.w, d, nullptr, 0, nullptr, 0, -1,
             true);
      drop(c, cur);
      cur = d;
    }
  }
  Act r = resnet(c, e_mid0_, cur);
  drop(c, cur);
  Act a = attn(c, e_att_, r);
  drop(c, r);
  cur = resnet(c, e_mid1_, a);
  drop(c, a);
  Act co = new_act(c, B, cur.h, cur.w, 8);
  if (gn_conv_out(c, cur, e_nout_w, e_nout_b, cfg_.norm_eps, e_cout_w, e_cout_b, 8, co.p, 8, 0)) {
    drop(c, cur);
  } else {
    Act gn = new_act(c, B, cur.h, cur.w, cur.c);
    gnorm(c, cur, nullptr, e_nout_w, e_nout_b, cfg_.norm_eps, 1, gn);
    drop(c, cur);
    conv2d(c, gn, nullptr, e_cout_w, e_cout_b, 8, 3, 1, 1, 1, gn.h, gn.w, co);
    drop(c, gn);
  }
  linear(c, co.p, 8, co.pix(), 8, qw, 8, fptr(qb), moments, 8, ACT_NONE, nullptr, 0, 0, B);
  drop(c, co);
}

void Vae::run_decode(Ctx& c, const void* z, int B, int h, int w, void* out) {
  const int* bo = cfg_.block_out_channels;
  const int nb = cfg_.n_blocks;
  const int cm = bo[nb - 1];
  Act zq = new_act(c, B, h, w, 8);
  linear(c, z, 8, (long)B * h * w, 8, pqw, 8, fptr(pqb), zq.p, 8, ACT_NONE, nullptr, 0, 0, B);
  Act cur = new_act(c, B, h, w, cm);
  conv2d(c, zq, nullptr, d_cin_w, d_cin_b, cm, 3, 1, 1, 1, h, w, cur, nullptr, 0, nullptr, 0, -1, true);
  drop(c, zq);
  Act r = resnet(c, d_mid0_, cur);
  drop(c, cur);
  Act a = attn(c, d_att_, r);
  drop(c, r);
  cur = resnet(c, d_mid1_, a);
  drop(c, a);
  for (int i = 0; i < nb; ++i) {
    for (auto& rr : d_res_[i]) {
      Act nx = resnet(c, rr, cur);
      drop(c, cur);
      cur = nx;
    }
    if (i < nb - 1) {
      Act u = new_act(c, B, cur.h * 2, cur.w * 2, cur.c);
      upsample_conv(c, cur, d_up_w_[i], d_up2_w_[i], d_up_b_[i], cur.c, u, true);
      drop(c, cur);
      cur = u;
    }
  }
  if (gn_conv_out(c, cur, d_nout_w, d_nout_b, cfg_.norm_eps, d_cout_w, d_cout_b, 4, out, 4, 0)) {
    drop(c, cur);
  } else {
    Act gn = new_act(c, B, cur.h, cur.w, cur.c);
    gnorm(c, cur, nullptr, d_nout_w, d_nout_b, cfg_.norm_eps, 1, gn);
    drop(c, cur);
    Act o;
    o.p = out; o.n = B; o.h = gn.h; o.w = gn.w; o.c = 4;
    conv2d(c, gn, nullptr, d_cout_w, d_cout_b, 4, 3, 1, 1, 1, gn.h, gn.w, o);
    drop(c, gn);
  }
}

size_t Vae::encode_ws(int B, int H, int W) {
  Arena ar;
  ar.reset(nullptr, 0);
  Ctx c{nullptr, &ar};
  run_encode(c, nullptr, B, H, W, nullptr);
  return ar.peak();
}
size_t Vae::decode_ws(int B, int h, int w) {
  Arena ar;
  ar.reset(nullptr, 0);
  Ctx c{nullptr, &ar};
  run_decode(c, nullptr, B, h, w, nullptr);
  return ar.peak();
}
void Vae::encode(hipStream_t s, const void* img, int B, int H, int W, void* moments, char* ws, size_t cap) {
  IRX_CHECK(blob_, "weights not bound");
  IRX_CHECK(H % 8 == 0 && W % 8 == 0, "VAE encode needs H, W multiples of 8");
  Arena ar;
  ar.reset(ws, cap);
  Ctx c{s, &ar};
  run_encode(c, img, B, H, W, moments);
}
void Vae::decode(hipStream_t s, const void* z, int B, int h, int w, void* out, char* ws, size_t cap) {
  IRX_CHECK(blob_, "weights not bound");
  Arena ar;
  ar.reset(ws, cap);
  Ctx c{s, &ar};
  run_decode(c, z, B, h, w, out);
}

// ---------------------------------------------------------------------------------------------- CLIP
Clip::Clip(const irx_model_config& cfg, int dtype) : Model(IRX_MODEL_CLIP, cfg, dtype) {
  const int D = cfg.hidden_size, F = cfg.intermediate_size;
  IRX_CHECK(D > 0 && F > 0 && cfg.num_layers > 0 && D % cfg.heads == 0, "bad CLIP config");
  const std::string p = "text_model.";
  tok = reg(p + "embeddings.token_embedding.weight", IRX_LAYOUT_EMB, dt_, {cfg.vocab_size, D});
  pos = reg(p + "embeddings.position_embedding.weight", IRX_LAYOUT_EMB, dt_, {cfg.max_positions, D});
  for (int i = 0; i < cfg.num_layers; ++i) {
    const std::string b = p + "encoder.layers." + std::to_string(i) + ".";
    const std::string s = b + "self_attn.";
    Layer l;
    l.ln1w = vec(b + "layer_norm1.weight", D); l.ln1b = vec(b + "layer_norm1.bias", D);
    l.qkvw = mat(s + "q_proj.weight|" + s + "k_proj.weight|" + s + "v_proj.weight", 3 * D, D);
    l.qkvb = vec(s + "q_proj.bias|" + s + "k_proj.bias|" + s + "v_proj.bias", 3 * D);
    l.ow = mat(s + "out_proj.weight", D, D); l.ob = vec(s + "out_proj.bias", D);
    l.ln2w = vec(b + "layer_norm2.weight", D); l.ln2b = vec(b + "layer_norm2.bias", D);
    l.f1w = mat(b + "mlp.fc1.weight", F, D); l.f1b = vec(b + "mlp.fc1.bias", F);
    l.f2w = mat(b + "mlp.fc2.weight", D, F); l.f2b = vec(b + "mlp.fc2.bias", D);
    layers_.push_back(l);
  }
  fw = vec(p + "final_layer_norm.weight", D); fb = vec(p + "final_layer_norm.bias", D);
}

void Clip::run(Ctx& c, const int* ids, int B, int L, void* out) {
  const int D = cfg_.hidden_size, F = cfg_.intermediate_size, H = cfg_.heads;
  const long M = (long)B * L;
  const size_t es = dsize(dt_);
  const float eps = cfg_.layer_norm_eps;
  void* h = c.ws->alloc(M * D * es);
  void* n = c.ws->alloc(M * D * es);
  void* qkv = c.ws->alloc(M * 3 * D * es);
  void* att = c.ws->alloc(M * D * es);
  void* f = c.ws->alloc(M * F * es);
  if (!c.ws->dry()) embed_tokens(dt_, ids, B, L, ptr(tok), ptr(pos), D, h, c.s);
  for (auto& l : layers_) {
    lnorm(c, h, M, D, l.ln1w, l.ln1b, eps, n);
    linear(c, n, D, M, D, l.qkvw, 3 * D, fptr(l.qkvb), qkv, 3 * D);
    if (!c.ws->dry()) {
      AttnArgs aa;
      aa.dtype = dt_; aa.B = B; aa.H = H; aa.Lq = L; aa.Lk = L; aa.d = D / H;
      aa.scale = 1.0f / std::sqrt((float)(D / H));
      aa.causal = 1;
      aa.q = qkv; aa.ldq = 3 * D; aa.sq = (long)L * 3 * D;
      aa.k = (char*)qkv + D * es; aa.ldk = 3 * D; aa.sk = aa.sq;
      aa.v = (char*)qkv + 2 * D * es; aa.ldv = 3 * D; aa.sv = aa.sq;
      aa.o = att; aa.ldo = D; aa.so = (long)L * D;
      attention(aa, c.s);
    }
    linear(c, att, D, M, D, l.ow, D, fptr(l.ob), h, D, ACT_NONE, h, D);
    lnorm(c, h, M, D, l.ln2w, l.ln2b, eps, n);
    linear(c, n, D, M, D, l.f1w, F, fptr(l.f1b), f, F, cfg_.quick_gelu ? ACT_QUICK_GELU : ACT_GELU);
    linear(c, f, F, M, F, l.f2w, D, fptr(l.f2b), h, D, ACT_NONE, h, D);
  }
  lnorm(c, h, M, D, fw, fb, eps, out);
  c.ws->free(f);
  c.ws->free(att);
  c.ws->free(qkv);
  c.ws->free(n);
  c.ws->free(h);
}

size_t Clip::workspace_bytes(int B, int L) {
  Arena ar;
  ar.reset(nullptr, 0);
  Ctx c{nullptr, &ar};
  run(c, nullptr, B, L, nullptr);
  return ar.peak();
}

void Clip::encode(hipStream_t s, const int* ids, int B, int L, void* out, char* ws, size_t cap) {
  IRX_CHECK(blob_, "weights not bound");
  IRX_CHECK(L <= cfg_.max_positions, "prompt longer than max_position_embeddings");
  Arena ar;
  ar.reset(ws, cap);
  Ctx c{s, &ar};
  run(c, ids, B, L, out);
}

}  // namespace irx
