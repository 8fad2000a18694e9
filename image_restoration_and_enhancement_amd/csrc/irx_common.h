// irx — MI355X-native SD-1.5 restoration engine: shared device/host helpers.
// gfx950 (CDNA4) only: wave64, MFMA 16x16 tiles, NHWC activations.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stddef.h>
#include <string>

namespace irx {

enum DType : int { F32 = 0, BF16 = 1, F16 = 2 };

typedef uint16_t bf16_t;   // storage type for bfloat16
typedef _Float16 f16_t;    // IEEE binary16 (the reference's own GPU dtype, src/inference.py:57)
typedef __attribute__((ext_vector_type(4))) float f32x4;
typedef __attribute__((ext_vector_type(4))) short s16x4;
typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8;
typedef __attribute__((ext_vector_type(4))) __bf16 bf16x4;
typedef __attribute__((ext_vector_type(8))) _Float16 f16x8;
typedef __attribute__((ext_vector_type(4))) _Float16 f16x4;
typedef __attribute__((ext_vector_type(16))) float f32x16;
typedef __attribute__((ext_vector_type(2))) float f32x2;
typedef __attribute__((ext_vector_type(2))) __bf16 bf16x2;
typedef __attribute__((ext_vector_type(2))) _Float16 f16x2;

// ---------------------------------------------------------------- conversions
__device__ __forceinline__ float bf2f(bf16_t v) { return __uint_as_float(((uint32_t)v) << 16); }
__device__ __forceinline__ bf16_t f2bf(float f) {
  __bf16 b = (__bf16)f;                       // v_cvt_pk_bf16_f32 (RNE, NaN-preserving)
  return __builtin_bit_cast(bf16_t, b);
}
template <typename T> __device__ __forceinline__ float ld_f(const T* p);
template <> __device__ __forceinline__ float ld_f<float>(const float* p) { return *p; }
template <> __device__ __forceinline__ float ld_f<bf16_t>(const bf16_t* p) { return bf2f(*p); }
template <> __device__ __forceinline__ float ld_f<f16_t>(const f16_t* p) { return (float)*p; }
// fp32 -> fp16 always as two steps, the fp32 value first: hipcc otherwise fuses an FMA feeding the conversion into
// v_fma_mixlo_f16 (one rounding, straight to fp16) at some call sites and not others — the same value then rounds
// differently with its position in an unrolled epilogue (the round-3 fp16 batch dependence: the folded-LayerNorm
// GEGLU epilogue, 17330 mixlo instructions in gemm2; scripts/diag_geglu_pos.py).  The empty asm pins the fp32 value.
__device__ __forceinline__ float f16_src(float f) {
  asm("" : "+v"(f));
  return f;
}
template <typename T> __device__ __forceinline__ T from_f(float f);
template <> __device__ __forceinline__ float from_f<float>(float f) { return f; }
template <> __device__ __forceinline__ bf16_t from_f<bf16_t>(float f) { return f2bf(f); }
template <> __device__ __forceinline__ f16_t from_f<f16_t>(float f) { return (f16_t)f16_src(f); }   // RNE

// 16-byte vector <-> floats
template <typename T> struct Vec16;
template <> struct Vec16<float> {
  static constexpr int N = 4;
  __device__ static void unpack(const uint4& u, float* f) {
    f[0] = __uint_as_float(u.x); f[1] = __uint_as_float(u.y);
    f[2] = __uint_as_float(u.z); f[3] = __uint_as_float(u.w);
  }
  __device__ static uint4 pack(const float* f) {
    return make_uint4(__float_as_uint(f[0]), __float_as_uint(f[1]), __float_as_uint(f[2]), __float_as_uint(f[3]));
  }
};
template <> struct Vec16<bf16_t> {
  static constexpr int N = 8;
  __device__ static void unpack(const uint4& u, float* f) {
    const uint32_t w[4] = {u.x, u.y, u.z, u.w};
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      f[2 * i] = __uint_as_float(w[i] << 16);
      f[2 * i + 1] = __uint_as_float(w[i] & 0xffff0000u);
    }
  }
  __device__ static uint4 pack(const float* f) {   // v_cvt_pk_bf16_f32 per pair (RNE)
    uint32_t w[4];
#pragma unroll
    for (int i = 0; i < 4; ++i)
      w[i] = __builtin_bit_cast(uint32_t, __builtin_convertvector((f32x2){f[2 * i], f[2 * i + 1]}, bf16x2));
    return make_uint4(w[0], w[1], w[2], w[3]);
  }
};

template <> struct Vec16<f16_t> {
  static constexpr int N = 8;
  __device__ static void unpack(const uint4& u, float* f) {
    const f16x8 h = __builtin_bit_cast(f16x8, u);
#pragma unroll
    for (int i = 0; i < 8; ++i) f[i] = (float)h[i];
  }
  __device__ static uint4 pack(const float* f) {   // v_cvt_pk_f16_f32 per pair (RNE)
    uint32_t w[4];
#pragma unroll
    for (int i = 0; i < 4; ++i)
      w[i] = __builtin_bit_cast(uint32_t,
                                __builtin_convertvector((f32x2){f16_src(f[2 * i]), f16_src(f[2 * i + 1])}, f16x2));
    return make_uint4(w[0], w[1], w[2], w[3]);
  }
};

// ---------------------------------------------------------------- 16-bit MFMA by storage type
// A/B fragments are raw 16-byte (8-element) or 8-byte (4-element) register images of the storage type.
template <typename T> struct Mfma;
template <> struct Mfma<bf16_t> {
  __device__ static f32x4 m16x16x32(const uint4& a, const uint4& b, f32x4 c) {
    return __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, a), __builtin_bit_cast(bf16x8, b), c,
                                                   0, 0, 0);
  }
  __device__ static f32x16 m32x32x16(const uint4& a, const uint4& b, f32x16 c) {
    return __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(bf16x8, a), __builtin_bit_cast(bf16x8, b), c,
                                                   0, 0, 0);
  }
  __device__ static f32x4 m16x16x16(const s16x4& a, const s16x4& b, f32x4 c) {
    return __builtin_amdgcn_mfma_f32_16x16x16bf16_1k(a, b, c, 0, 0, 0);
  }
  // two fp32 -> packed pair (RNE, one v_cvt_pk_bf16_f32)
  __device__ static uint32_t pack2(float lo, float hi) {
    return __builtin_bit_cast(uint32_t, __builtin_convertvector((f32x2){lo, hi}, bf16x2));
  }
  __device__ static float round(float x) { return bf2f(f2bf(x)); }   // nearest representable value
};
template <> struct Mfma<f16_t> {
  __device__ static f32x4 m16x16x32(const uint4& a, const uint4& b, f32x4 c) {
    return __builtin_amdgcn_mfma_f32_16x16x32_f16(__builtin_bit_cast(f16x8, a), __builtin_bit_cast(f16x8, b), c, 0,
                                                  0, 0);
  }
  __device__ static f32x16 m32x32x16(const uint4& a, const uint4& b, f32x16 c) {
    return __builtin_amdgcn_mfma_f32_32x32x16_f16(__builtin_bit_cast(f16x8, a), __builtin_bit_cast(f16x8, b), c, 0,
                                                  0, 0);
  }
  __device__ static f32x4 m16x16x16(const s16x4& a, const s16x4& b, f32x4 c) {
    return __builtin_amdgcn_mfma_f32_16x16x16f16(__builtin_bit_cast(f16x4, a), __builtin_bit_cast(f16x4, b), c, 0,
                                                 0, 0);
  }
  __device__ static uint32_t pack2(float lo, float hi) {   // one v_cvt_pk_f16_f32 (RNE)
    return __builtin_bit_cast(uint32_t, __builtin_convertvector((f32x2){f16_src(lo), f16_src(hi)}, f16x2));
  }
  __device__ static float round(float x) { return (float)(f16_t)f16_src(x); }
};

// ---------------------------------------------------------------- activations (epilogues)
enum ActKind : int { ACT_NONE = 0, ACT_SILU = 1, ACT_GELU = 2, ACT_QUICK_GELU = 3 };
__device__ __forceinline__ float silu_f(float x) { return x / (1.0f + __expf(-x)); }
__device__ __forceinline__ float gelu_erf(float x) { return 0.5f * x * (1.0f + erff(x * 0.70710678118654752f)); }
// erf by Abramowitz & Stegun 7.1.26 (|error| <= 1.5e-7, one rcp + one exp, no branches): 13 VALU instead of the
// range-split library erff.  The 16-bit engines' GELU (GEGLU epilogue, geglu kernel) uses it — its error is three
// orders of magnitude under a bf16 / fp16 rounding of the result; the fp32 parity engine keeps erff.
__device__ __forceinline__ float erf_as(float x) {
  const float ax = fabsf(x);
  const float t = __builtin_amdgcn_rcpf(fmaf(0.3275911f, ax, 1.0f));
  float p = fmaf(1.061405429f, t, -1.453152027f);
  p = fmaf(p, t, 1.421413741f);
  p = fmaf(p, t, -0.284496736f);
  p = fmaf(p, t, 0.254829592f);
  p *= t;
  const float r = fmaf(-p, __expf(-ax * ax), 1.0f);
  return __builtin_copysignf(r, x);
}
__device__ __forceinline__ float gelu_erf16(float x) {
  const float h = 0.5f * x;
  return fmaf(h, erf_as(x * 0.70710678118654752f), h);
}
// GroupNorm application y = x * scale + shift (+ SiLU), the one definition gn_apply_kernel and the
// GroupNorm-fused halo convolution share (bit-identical results on either path)
__device__ __forceinline__ float gn_act(float x, float sc, float sh, int silu) {
  const float y = fmaf(x, sc, sh);
  return silu ? y * __builtin_amdgcn_rcpf(1.0f + __expf(-y)) : y;
}
__device__ __forceinline__ float apply_act(float x, int act) {
  switch (act) {
    case ACT_SILU: return silu_f(x);
    case ACT_GELU: return gelu_erf(x);
    case ACT_QUICK_GELU: return x / (1.0f + __expf(-1.702f * x));
    default: return x;
  }
}

// ---------------------------------------------------------------- XCD-aware block remap (bijective)
// Consecutive logical tiles land on the same XCD (blocks b, b+8, ... share one), so tiles that
// share an operand panel hit the same 4 MiB L2.
__device__ __forceinline__ int xcd_remap(int bid, int nwg) {
  const int q = nwg >> 3, r = nwg & 7, x = bid & 7;
  return (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + (bid >> 3);
}

// ---------------------------------------------------------------- host-side errors
void set_error(const std::string& msg);
// rccl.cpp: in-place uint8 ncclBroadcast (librccl resolved at first use)
void rccl_broadcast(void* comm, void* buf, size_t bytes, int root, hipStream_t s);
const char* last_error();

struct Error : public std::exception {
  std::string msg;
  explicit Error(std::string m) : msg(std::move(m)) {}
  const char* what() const noexcept override { return msg.c_str(); }
};
#define IRX_CHECK(cond, msg)                                                          \
  do {                                                                                 \
    if (!(cond)) throw ::irx::Error(std::string(__func__) + ": " + (msg));           \
  } while (0)
#define IRX_HIP(call)                                                                 \
  do {                                                                                 \
    hipError_t e_ = (call);                                                            \
    if (e_ != hipSuccess)                                                              \
      throw ::irx::Error(std::string(#call) + " failed: " + hipGetErrorString(e_));   \
  } while (0)
#define IRX_LAUNCH_CHECK() IRX_HIP(hipGetLastError())

inline size_t dsize(int dt) { return dt == F32 ? 4 : 2; }
inline bool is16(int dt) { return dt == BF16 || dt == F16; }

}  // namespace irx
