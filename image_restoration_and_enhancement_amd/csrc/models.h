// irx — native model graphs (UNet2DConditionModel, AutoencoderKL, CLIPTextModel) over the irx kernels.
#pragma once
#include <map>
#include <memory>
#include <vector>

#include "../../include/irx.h"
#include "ops.h"

namespace irx {

extern int g_vae_attn_rows;   // VAE mid-block attention: query rows per score block (0 = auto, capped bytes)
extern int g_vae_flash;       // VAE mid-block attention in the 16-bit engines: flash kernel (1) / row-blocked (0)

// Deterministic first-fit allocator over a caller-owned workspace.  Run once with base == nullptr
// ("dry run": no kernels launched) to size the workspace, then for real with identical calls.
class Arena {
 public:
  void reset(char* base, size_t cap) {
    base_ = base; cap_ = cap; end_ = 0; peak_ = 0; free_.clear(); live_.clear(); ids_.clear(); next_id_ = 0;
  }
  void* alloc(size_t bytes);
  void free(void* p);
  size_t peak() const { return peak_; }
  bool dry() const { return base_ == nullptr; }

 private:
  char* base_ = nullptr;
  size_t cap_ = 0, end_ = 0, peak_ = 0;
  std::map<size_t, size_t> free_;    // offset -> size of free holes below end_
  std::map<size_t, size_t> live_;    // offset -> size
  std::map<size_t, int> ids_;        // offset -> allocation index (guard diagnostics)
  int next_id_ = 0;
};
// diagnostics (irx_set_option("arena_guard", 1)): every workspace allocation is followed by a 64 KiB guard filled with
// 0xA5, checked when the allocation is freed (device-synchronous; reports overruns on stderr)
extern int g_arena_guard;

struct P { size_t off = 0; bool set = false; };   // parameter reference into the weight blob

struct ParamEntry {
  std::string name;
  int layout, dtype;
  std::vector<int64_t> shape;
  size_t off, bytes;
  float row_scale = 1.f;     // packer scales rows [0, scale_rows) (folded attention scale)
  int64_t scale_rows = 0;
  std::string aux;           // irx_param_info::aux (LayerNorm fold sources)
};

struct Act {   // NHWC activation view
  void* p = nullptr;
  int n = 0, h = 0, w = 0, c = 0;
  double* gnp = nullptr;   // GroupNorm partials emitted by its producer (GemmArgs::gn_part), else null
  int gnr = 0;             // ... rows per partial (divides h * w)
  long pix() const { return (long)n * h * w; }
};

class Model {
 public:
  Model(int kind, const irx_model_config& cfg, int dtype) : kind_(kind), cfg_(cfg), dt_(dtype) {}
  virtual ~Model() = default;
  int kind() const { return kind_; }
  int dtype() const { return dt_; }
  const std::vector<ParamEntry>& manifest() const { return params_; }
  size_t blob_bytes() const { return blob_bytes_; }
  void bind(void* blob, size_t bytes);
  char* blob() const { return blob_; }   // the bound device blob (nullptr before bind)

 protected:
  P reg(const std::string& name, int layout, int dtype, std::vector<int64_t> shape, float row_scale = 1.f,
        int64_t scale_rows = 0, const std::string& aux = std::string());
  P vec(const std::string& name, int64_t n) { return reg(name, IRX_LAYOUT_VEC, F32, {n}); }
  P mat(const std::string& name, int64_t n, int64_t k) { return reg(name, IRX_LAYOUT_MAT, dt_, {n, k}); }
  P conv(const std::string& name, int64_t co, int64_t kh, int64_t kw, int64_t ci) {
    return reg(name, IRX_LAYOUT_CONV, dt_, {co, kh, kw, ci});
  }
  template <typename X = void> const X* ptr(P p) const { return (const X*)(blob_ + p.off); }
  const float* fptr(P p) const { return (const float*)(blob_ + p.off); }

  // ---- op helpers (skip launches in dry-run mode)
  struct Ctx { hipStream_t s; Arena* ws; };
  Act new_act(Ctx& c, int n, int h, int w, int ch);
  void drop(Ctx& c, Act& a) {
    c.ws->free(a.p);
    a.p = nullptr;
    if (a.gnp) c.ws->free(a.gnp);
    a.gnp = nullptr;
    a.gnr = 0;
  }
  // `stats`: the output feeds a GroupNorm -> the epilogue also emits its partial sums when it can (Act::gnp)
  void conv2d(Ctx& c, const Act& x0, const Act* x1, P w, P b, int cout, int k, int stride, int pad_t, int pad_l,
              int hv, int wv, Act& out, const float* rowadd = nullptr, long rowadd_ld = 0,
              const void* residual = nullptr, int out_f32 = 0, int ldc = -1, bool stats = false);
  void linear(Ctx& c, const void* A, long lda, int M, int K, P w, int N, const float* bias, void* C, long ldc,
              int act = ACT_NONE, const void* residual = nullptr, long ldr = 0, int out_f32 = 0, int imgs = 0,
              Act* stats = nullptr);
  void run_gemm(Ctx& c, GemmArgs& a, Act* stats = nullptr);   // split-K partials / GroupNorm partials
  void gnorm(Ctx& c, const Act& x0, const Act* x1, P g, P b, float eps, int silu, const Act& out);
  // GroupNorm(+SiLU) of (x0 | x1) followed by a 3x3 / stride-1 / pad-1 conv into `out`: folded into the
  // conv's halo operand path where it fits (gemm_gn_fusable), else a normalised copy and the plain conv
  void gn_conv3(Ctx& c, const Act& x0, const Act* x1, P g, P gb, float eps, int silu, P w, P b, int cout,
                Act& out, const float* rowadd = nullptr, long rowadd_ld = 0, const void* residual = nullptr,
                bool stats = false);
  void lnorm(Ctx& c, const void* x, int rows, int C, P g, P b, float eps, void* out);
  // diffusers Upsample2D (nearest resize to out's size, conv 3x3 pad 1): as 4 per-parity 2x2 convs of x (w2:
  // IRX_LAYOUT_CONV_UP2) when out is exactly 2x and the large-tile path takes the shape, else the resize conv (w)
  void upsample_conv(Ctx& c, const Act& x, P w, P w2, P b, int cout, Act& out, bool stats);
  P up2_weights(const std::string& name, int ch);   // IRX_LAYOUT_CONV_UP2 entry (16-bit engines; unset for fp32)
  // GroupNorm + SiLU + 3x3 conv to a narrow output head in one kernel (gn_conv_narrow); false: not taken
  bool gn_conv_out(Ctx& c, const Act& x, P g, P gb, float eps, P w, P b, int cout, void* out, int ldo, int out_f32);

  int kind_;
  irx_model_config cfg_;
  int dt_;
  std::vector<ParamEntry> params_;
  size_t blob_bytes_ = 0;
  char* blob_ = nullptr;
};

// ------------------------------------------------------------------ shared blocks
struct ResW {
  P n1w, n1b, c1w, c1b, n2w, n2b, c2w, c2b, scw, scb;
  int cin = 0, cout = 0;
  bool shortcut = false;
  long temb_off = -1;     // column offset into the fused time_emb_proj output (UNet only)
};

class Unet : public Model {
 public:
  Unet(const irx_model_config& cfg, int dtype);
  int cin_pad() const { return cin_pad_; }
  size_t workspace_bytes(int B, int h, int w);
  size_t context_bytes(int B, int L) const { return (size_t)B * L * kv_cols_ * dsize(dt_); }
  void prepare_context(hipStream_t s, const void* ctx, int B, int L, void* kv, char* ws, size_t cap);
  void forward(hipStream_t s, const void* x, int B, int h, int w, const float* t, const void* kv, int L, float* eps,
               char* ws, size_t cap);

 private:
  struct XfW {
    P nw, nb, piw, pib, ln1w, ln1b, qkvw, o1w, o1b, ln2w, ln2b, q2w, o2w, o2b, ln3w, ln3b, ffw, ffb, ff2w, ff2b, pow,
        pob;
    // LayerNorm fold (16-bit engines, ln_fold_): qkvw / q2w / ffw hold W * gamma; u = row sums of those, v = bias +
    // W beta (GemmArgs::ln_rs / ln_u)
    P qkvu, qkvv, q2u, q2v, ffu, ffv;
    // ff.net.2 folded through proj_out (16-bit engines): [W_po | W_po W_ff2] and b_po + W_po b_ff2 (IRX_LAYOUT_*_CHAIN)
    P pofw, pofb;
    int c = 0;
    long kv_off = 0;      // column offset into the fused cross-attention K|V cache
  };
  struct Block {
    std::vector<ResW> res;
    std::vector<XfW> attn;
    bool has_attn = false, resample = false;
    P rsw, rsb;           // down/upsampler conv
    P rsw2;               // upsampler: per-parity 2x2 weights (IRX_LAYOUT_CONV_UP2; 16-bit engines)
    int ch = 0;
  };
  ResW make_res(const std::string& p, int cin, int cout);
  XfW make_xf(const std::string& p, int c);
  void run(Ctx& c, const void* x, int B, int h, int w, const float* t, const void* kv, int L, float* eps);
  Act resnet(Ctx& c, const ResW& r, Act& x0, Act* x1, const float* tproj, float eps);
  Act transformer(Ctx& c, const XfW& a, Act& x, const void* kv, int L);
  // LayerNorm(x) -> projection g (g.A / lda / bias set here): folded into g's epilogue when ln_fold_ and the shape
  // takes it — with the statistics from `parts` (the producer of x emitted them, GemmArgs::ln_out) or from a
  // statistics pass written to `st` — else through the normalised copy `nbuf`
  void ln_gemm(Ctx& c, GemmArgs& g, const void* x, int rows, int C, P lnw, P lnb, P u, P v, const float* bias,
               void* nbuf, float2* st, const float2* parts = nullptr);
  // a transformer projection that writes the residual stream (proj_in, to_out, to_out2): out = A W^T + bias
  // (+ residual), emitting the output's LayerNorm partials into `lnp` where the epilogue can; returns lnp or null
  const float2* xf_proj(Ctx& c, const void* A, int M, int C, P w, const float* bias, void* out, const void* residual,
                        int imgs, float2* lnp);

  int cin_pad_ = 8;
  bool ln_fold_ = false;   // LayerNorm folded into the transformer projections (fixed at creation: the blob layout)
  int temb_dim_ = 1280;
  long temb_cols_ = 0, kv_cols_ = 0;
  std::vector<std::string> temb_names_w_, temb_names_b_, kv_names_;
  P conv_in_w, conv_in_b, t1w, t1b, t2w, t2b, tpw, tpb, kvw, nout_w, nout_b, conv_out_w, conv_out_b;
  std::vector<Block> down_, up_;
  ResW mid_res0_, mid_res1_;
  XfW mid_attn_;
};

class Vae : public Model {
 public:
  Vae(const irx_model_config& cfg, int dtype);
  size_t encode_ws(int B, int H, int W);
  size_t decode_ws(int B, int h, int w);
  void encode(hipStream_t s, const void* img, int B, int H, int W, void* moments, char* ws, size_t cap);
  void decode(hipStream_t s, const void* z, int B, int h, int w, void* out, char* ws, size_t cap);

 private:
  struct AttW { P gw, gb, qkvw, qkvb, ow, ob; int c = 0; };
  ResW make_res(const std::string& p, int cin, int cout);
  AttW make_attn(const std::string& p, int c);
  Act resnet(Ctx& c, const ResW& r, Act& x);
  Act attn(Ctx& c, const AttW& a, Act& x);
  void run_encode(Ctx& c, const void* img, int B, int H, int W, void* moments);
  void run_decode(Ctx& c, const void* z, int B, int h, int w, void* out);

  P e_cin_w, e_cin_b, e_nout_w, e_nout_b, e_cout_w, e_cout_b, qw, qb, pqw, pqb, d_cin_w, d_cin_b, d_nout_w,
      d_nout_b, d_cout_w, d_cout_b;
  std::vector<std::vector<ResW>> e_res_, d_res_;
  std::vector<P> e_down_w_, e_down_b_, d_up_w_, d_up_b_, d_up2_w_;
  ResW e_mid0_, e_mid1_, d_mid0_, d_mid1_;
  AttW e_att_, d_att_;
};

class Clip : public Model {
 public:
  Clip(const irx_model_config& cfg, int dtype);
  size_t workspace_bytes(int B, int L);
  void encode(hipStream_t s, const int* ids, int B, int L, void* out, char* ws, size_t cap);

 private:
  struct Layer { P ln1w, ln1b, qkvw, qkvb, ow, ob, ln2w, ln2b, f1w, f1b, f2w, f2b; };
  void run(Ctx& c, const int* ids, int B, int L, void* out);
  P tok, pos, fw, fb;
  std::vector<Layer> layers_;
};

}  // namespace irx
