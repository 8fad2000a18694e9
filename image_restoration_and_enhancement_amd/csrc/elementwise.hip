// irx — HBM-bound elementwise / data-movement kernels of the restoration hot path (gfx950).
// Compiled with -ffp-contract=off: the scheduler / add_noise / CFG arithmetic reproduces the
// reference's fp32 operation order (diffusers 0.35.2) rounding by
// rounding, which an fma contraction would change.
#include "ops.h"

namespace irx {
namespace {

constexpr int kB = 256;
inline int nblk(long n, int per = kB) { return (int)((n + per - 1) / per); }

// ------------------------------------------------------------------ GEGLU: h * gelu_erf(gate)
template <typename T>
__global__ void geglu_kernel(const T* __restrict__ p, long ldp, int M, int F, T* __restrict__ o, long ldo,
                             int il) {
  constexpr int VEC = 16 / (int)sizeof(T);
  const int nv = F / VEC;
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= (long)M * nv) return;
  const int m = (int)(i / nv), v = (int)(i % nv);
  const int f = v * VEC;
  const int hc = il ? (f / 64) * 128 + (f % 64) : f;
  const int gc = il ? hc + 64 : F + f;
  float h[VEC], g[VEC];
  Vec16<T>::unpack(*(const uint4*)(p + (long)m * ldp + hc), h);
  Vec16<T>::unpack(*(const uint4*)(p + (long)m * ldp + gc), g);
#pragma unroll
  for (int e = 0; e < VEC; ++e) h[e] = h[e] * (sizeof(T) == 4 ? gelu_erf(g[e]) : gelu_erf16(g[e]));
  *(uint4*)(o + (long)m * ldo + v * VEC) = Vec16<T>::pack(h);
}

// ------------------------------------------------------------------ sinusoidal timestep embedding
template <typename T>
__global__ void temb_kernel(const float* __restrict__ t, int B, int dim, int flip, float shift, T* __restrict__ out) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= B * dim) return;
  const int b = i / dim, j = i % dim;
  const int half = dim / 2;
  const int k = j % half;
  float e = (-9.210340371976184f * (float)k) / ((float)half - shift);
  e = expf(e);
  const float arg = t[b] * e;
  const bool first = j < half;
  float v;
  if (flip) v = first ? cosf(arg) : sinf(arg);
  else v = first ? sinf(arg) : cosf(arg);
  out[i] = from_f<T>(v);
}

// ------------------------------------------------------------------ CLIP token + position embedding
template <typename T>
__global__ void embed_kernel(const int* __restrict__ ids, int B, int L, const T* __restrict__ tok,
                             const T* __restrict__ pos, int D, T* __restrict__ out) {
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= (long)B * L * D) return;
  const int d = (int)(i % D);
  const long bl = i / D;
  const int l = (int)(bl % L);
  const int id = ids[bl];
  out[i] = from_f<T>(ld_f<T>(tok + (long)id * D + d) + ld_f<T>(pos + (long)l * D + d));
}

// ------------------------------------------------------------------ tiled transpose
template <typename T>
__global__ void transpose_kernel(const T* __restrict__ in, long ldi, int rows, int cols, T* __restrict__ out,
                                 long ldo, long s_in, long s_out) {
  __shared__ T tile[32][33];
  const int z = blockIdx.z;
  in += (long)z * s_in;
  out += (long)z * s_out;
  const int c0 = blockIdx.x * 32, r0 = blockIdx.y * 32;
  const int tx = threadIdx.x & 31, ty = threadIdx.x >> 5;   // 256 threads: 32 x 8
  for (int r = ty; r < 32; r += 8) {
    const int rr = r0 + r, cc = c0 + tx;
    if (rr < rows && cc < cols) tile[r][tx] = in[(long)rr * ldi + cc];
  }
  __syncthreads();
  for (int c = ty; c < 32; c += 8) {
    const int cc = c0 + c, rr = r0 + tx;
    if (rr < rows && cc < cols) out[(long)cc * ldo + rr] = tile[tx][c];
  }
}

// ------------------------------------------------------------------ row softmax (fp32 in)
template <typename T>
__global__ __launch_bounds__(256) void softmax_kernel(const float* __restrict__ in, long ldi, int cols,
                                                      T* __restrict__ out, long ldo) {
  __shared__ float red[4];
  const long row = blockIdx.x;
  const float* x = in + row * ldi;
  float m = -INFINITY;
  for (int c = threadIdx.x; c < cols; c += 256) m = fmaxf(m, x[c]);
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) m = fmaxf(m, __shfl_xor(m, o));
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = m;
  __syncthreads();
  m = fmaxf(fmaxf(red[0], red[1]), fmaxf(red[2], red[3]));
  __syncthreads();
  float s = 0.f;
  for (int c = threadIdx.x; c < cols; c += 256) s += expf(x[c] - m);
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) s += __shfl_xor(s, o);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = s;
  __syncthreads();
  s = red[0] + red[1] + red[2] + red[3];
  const float inv = 1.f / s;
  for (int c = threadIdx.x; c < cols; c += 256) out[row * ldo + c] = from_f<T>(expf(x[c] - m) * inv);
  for (int c = cols + threadIdx.x; c < ldo; c += 256) out[row * ldo + c] = T(0);   // zero the padded key columns
}

// ------------------------------------------------------------------ image <-> tensor
template <typename T>
__global__ void img2t_kernel(const uint8_t* __restrict__ img, const float* __restrict__ mask, long npix, int cpad,
                             T* __restrict__ out) {
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= npix * cpad) return;
  const long p = i / cpad;
  const int c = (int)(i % cpad);
  float v = 0.f;
  if (c < 3) {
    v = (float)img[p * 3 + c] / 255.0f;    // VaeImageProcessor: np.float32 / 255, then 2x - 1
    v = 2.0f * v - 1.0f;
    if (mask) v = v * (mask[p] < 0.5f ? 1.0f : 0.0f);   // inpaint: init_image * (mask < 0.5)
  }
  out[i] = from_f<T>(v);
}

template <typename T>
__global__ void t2img_kernel(const T* __restrict__ x, long npix, int ldc, uint8_t* __restrict__ img, float* f01) {
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= npix * 3) return;
  const long p = i / 3;
  const int c = (int)(i % 3);
  float v = ld_f<T>(x + p * ldc + c) * 0.5f + 0.5f;   // denormalize, clamp(0, 1)
  v = fminf(fmaxf(v, 0.f), 1.f);
  if (f01) f01[i] = v;
  img[i] = (uint8_t)rintf(v * 255.0f);                // numpy round (half to even)
}

// ------------------------------------------------------------------ posterior sample (+ add_noise)
template <typename T>
__global__ void latent_kernel(const T* __restrict__ mom, int mcs, long npix, long pix_per_img,
                              const float* __restrict__ eps, const float* __restrict__ noise, int bcast, float sf,
                              float a, float b, float* __restrict__ out) {
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= npix * 4) return;
  const long p = i >> 2;
  const int c = (int)(i & 3);
  const long ni = bcast ? (p % pix_per_img) * 4 + c : i;
  const float mean = ld_f<T>(mom + p * mcs + c);
  float logvar = ld_f<T>(mom + p * mcs + 4 + c);
  logvar = fminf(fmaxf(logvar, -30.0f), 20.0f);
  const float stdv = expf(0.5f * logvar);
  float z = mean + stdv * eps[ni];
  z = sf * z;
  if (noise) {
    const float t1 = a * z;
    const float t2 = b * noise[ni];
    z = t1 + t2;
  }
  out[i] = z;
}

// ------------------------------------------------------------------ fused CFG + scheduler step + pack
template <typename T>
__device__ __forceinline__ void pack_pixel(T* __restrict__ dst, const float* lat4, int cin_pad, int inpaint,
                                           const float* mask, const float* masked, long pix) {
  if constexpr (sizeof(T) == 2) {
    // 16-bit engines: whole 16-byte chunks (cin_pad is 64 there: conv_in runs on the 64-channel-slab conv tiles)
    alignas(16) T v[16];
#pragma unroll
    for (int e = 0; e < 16; ++e) v[e] = T(0);
#pragma unroll
    for (int e = 0; e < 4; ++e) v[e] = from_f<T>(lat4[e]);
    if (inpaint) {
      v[4] = from_f<T>(mask[pix]);
#pragma unroll
      for (int e = 0; e < 4; ++e) v[5 + e] = from_f<T>(masked[pix * 4 + e]);
    }
    uint4* d = (uint4*)dst;
    d[0] = *(const uint4*)&v[0];
    if (cin_pad >= 16) d[1] = *(const uint4*)&v[8];
    for (int k = 2; k < cin_pad / 8; ++k) d[k] = uint4{0u, 0u, 0u, 0u};
  } else {
    int c = 0;
    for (; c < 4; ++c) dst[c] = from_f<T>(lat4[c]);
    if (inpaint) {
      dst[4] = from_f<T>(mask[pix]);
      for (int e = 0; e < 4; ++e) dst[5 + e] = from_f<T>(masked[pix * 4 + e]);
      c = 9;
    }
    for (; c < cin_pad; ++c) dst[c] = T(0);
  }
}

template <typename T>
__global__ void step_kernel(StepArgs a) {
  const long npix = (long)a.B * a.h * a.w;
  const long p = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (p >= npix) return;
  float out4[4];
#pragma unroll
  for (int c = 0; c < 4; ++c) {
    const long i = p * 4 + c;
    float e0;
    if (a.cfg) {
      const float u = a.eps[i];
      const float t = a.eps[npix * 4 + i];
      const float d = t - u;
      e0 = u + a.guidance * d;
    } else {
      e0 = a.eps[i];
    }
    if (a.hist_store) a.hist_store[i] = e0;
    float e = a.hw[0] * e0;
#pragma unroll
    for (int k = 0; k < 4; ++k)
      if (a.hist[k]) { const float t = a.hw[k + 1] * a.hist[k][i]; e = e + t; }
    e = e / a.e_div;
    e = a.e_mul * e;
    const float x = a.x_src[i];
    if (a.cur_store) a.cur_store[i] = x;
    float r;
    if (a.mode == 0) {          // PNDM _get_prev_sample
      const float t1 = a.c0 * x;
      const float t2 = a.c1 * e;
      const float t3 = t2 / a.c2;
      r = t1 - t3;
    } else {                    // DDIM, eta = 0
      const float t1 = a.c0 * e;
      const float x0 = (x - t1) / a.c1;
      const float t2 = a.c2 * x0;
      const float t3 = a.c3 * e;
      r = t2 + t3;
    }
    out4[c] = r;
    a.x_out[i] = r;
  }
  if (a.unet_in) {
    const long pix_img = (long)a.h * a.w;
    const long pi = p % pix_img;
    const long b = p / pix_img;
    (void)pi;
    T* dst = (T*)a.unet_in + p * a.cin_pad;
    pack_pixel<T>(dst, out4, a.cin_pad, a.inpaint, a.mask, a.masked, p);
    if (a.cfg) pack_pixel<T>(dst + npix * a.cin_pad, out4, a.cin_pad, a.inpaint, a.mask, a.masked, p);
    (void)b;
  }
}

template <typename T>
__global__ void pack_kernel(const float* __restrict__ lat, long npix, int cfg, int cin_pad, int inpaint,
                            const float* mask, const float* masked, T* __restrict__ out) {
  const long p = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (p >= npix) return;
  float l4[4] = {lat[p * 4], lat[p * 4 + 1], lat[p * 4 + 2], lat[p * 4 + 3]};
  pack_pixel<T>(out + p * cin_pad, l4, cin_pad, inpaint, mask, masked, p);
  if (cfg) pack_pixel<T>(out + (npix + p) * cin_pad, l4, cin_pad, inpaint, mask, masked, p);
}

template <typename T>
__global__ void scale_copy_kernel(const float* __restrict__ in, long npix, float div, T* __restrict__ out, int ic,
                                  int oc) {
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= npix * oc) return;
  const long p = i / oc;
  const int c = (int)(i % oc);
  out[i] = c < ic ? from_f<T>(in[p * ic + c] / div) : T(0);
}

#define IRX_DISPATCH(dtype, KERNEL_CALL)       \
  do {                                         \
    if ((dtype) == F32) {                      \
      using T = float;                         \
      KERNEL_CALL;                             \
    } else if ((dtype) == F16) {               \
      using T = f16_t;                         \
      KERNEL_CALL;                             \
    } else {                                   \
      using T = bf16_t;                        \
      KERNEL_CALL;                             \
    }                                          \
    IRX_LAUNCH_CHECK();                        \
  } while (0)

}  // namespace

void geglu(int dtype, const void* proj, long ldp, int M, int F, void* out, long ldo, int il, hipStream_t s) {
  const int vec = dtype == F32 ? 4 : 8;
  IRX_CHECK(F % vec == 0 && ldp % vec == 0 && ldo % vec == 0, "geglu alignment");
  IRX_CHECK(!il || F % 64 == 0, "interleaved geglu needs F % 64 == 0");
  const long n = (long)M * (F / vec);
  IRX_DISPATCH(dtype, (geglu_kernel<T><<<nblk(n), kB, 0, s>>>((const T*)proj, ldp, M, F, (T*)out, ldo, il)));
}

void timestep_embed(int dtype, const float* t, int B, int dim, int flip, float shift, void* out, hipStream_t s) {
  IRX_DISPATCH(dtype, (temb_kernel<T><<<nblk((long)B * dim), kB, 0, s>>>(t, B, dim, flip, shift, (T*)out)));
}

void embed_tokens(int dtype, const int* ids, int B, int L, const void* tok, const void* pos, int D, void* out,
                  hipStream_t s) {
  IRX_DISPATCH(dtype, (embed_kernel<T><<<nblk((long)B * L * D), kB, 0, s>>>(ids, B, L, (const T*)tok,
                                                                            (const T*)pos, D, (T*)out)));
}

void transpose2d(int dtype, const void* in, long ldi, int rows, int cols, void* out, long ldo, int batch, long s_in,
                 long s_out, hipStream_t s) {
  dim3 grid((cols + 31) / 32, (rows + 31) / 32, batch);
  IRX_DISPATCH(dtype, (transpose_kernel<T><<<grid, 256, 0, s>>>((const T*)in, ldi, rows, cols, (T*)out, ldo, s_in,
                                                                s_out)));
}

void softmax_rows(int dtype, const float* in, long ldi, int rows, int cols, void* out, long ldo, hipStream_t s) {
  IRX_DISPATCH(dtype, (softmax_kernel<T><<<rows, 256, 0, s>>>(in, ldi, cols, (T*)out, ldo)));
}

void image_to_tensor(int dtype, const uint8_t* img, const float* mask, int N, int H, int W, int cpad, void* out,
                     hipStream_t s) {
  const long np = (long)N * H * W;
  IRX_DISPATCH(dtype, (img2t_kernel<T><<<nblk(np * cpad), kB, 0, s>>>(img, mask, np, cpad, (T*)out)));
}

void tensor_to_image(int dtype, const void* x, int N, int H, int W, int ldc, uint8_t* img, float* f01,
                     hipStream_t s) {
  const long np = (long)N * H * W;
  IRX_DISPATCH(dtype, (t2img_kernel<T><<<nblk(np * 3), kB, 0, s>>>((const T*)x, np, ldc, img, f01)));
}

void latent_sample(int dtype, const void* mom, int mcs, int N, int h, int w, const float* eps, const float* noise,
                   int bcast, float sf, float a, float b, float* out, hipStream_t s) {
  const long np = (long)N * h * w;
  IRX_DISPATCH(dtype, (latent_kernel<T><<<nblk(np * 4), kB, 0, s>>>((const T*)mom, mcs, np, (long)h * w, eps,
                                                                    noise, bcast, sf, a, b, out)));
}

// The 16-bit pack_pixel stores whole 16-byte chunks: the padded width must be a multiple of 8 channels
// holding the 4 (or 9) live ones, and the destination 16-byte aligned.
static void check_pack_layout(int dtype, int cin_pad, int inpaint, const void* dst) {
  if (dtype == F32 || !dst) return;
  IRX_CHECK(cin_pad % 8 == 0 && cin_pad >= (inpaint ? 16 : 8) && ((uintptr_t)dst % 16) == 0,
            "16-bit UNet input: cin_pad must be a multiple of 8 (>= 16 for inpaint) and the buffer 16-byte aligned");
}

void sched_step(const StepArgs& a, hipStream_t s) {
  IRX_CHECK(a.eps && a.x_src && a.x_out, "sched_step: missing buffers");
  IRX_CHECK(!a.inpaint || (a.mask && a.masked && a.cin_pad >= 9), "sched_step: inpaint inputs");
  check_pack_layout(a.dtype, a.cin_pad, a.inpaint, a.unet_in);
  const long np = (long)a.B * a.h * a.w;
  IRX_DISPATCH(a.dtype, (step_kernel<T><<<nblk(np), kB, 0, s>>>(a)));
}

void pack_unet_input(int dtype, const float* lat, int B, int h, int w, int cfg, int cin_pad, int inpaint,
                     const float* mask, const float* masked, void* out, hipStream_t s) {
  check_pack_layout(dtype, cin_pad, inpaint, out);
  const long np = (long)B * h * w;
  IRX_DISPATCH(dtype, (pack_kernel<T><<<nblk(np), kB, 0, s>>>(lat, np, cfg, cin_pad, inpaint, mask, masked,
                                                              (T*)out)));
}

void scale_copy(int dtype_out, const float* in, long npix, float div, void* out, int in_ch, int out_ch,
                hipStream_t s) {
  IRX_DISPATCH(dtype_out, (scale_copy_kernel<T><<<nblk(npix * out_ch), kB, 0, s>>>(in, npix, div, (T*)out, in_ch,
                                                                                   out_ch)));
}

}  // namespace irx
