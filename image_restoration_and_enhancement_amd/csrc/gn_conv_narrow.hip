// irx — GroupNorm(+SiLU) fused into a narrow 3x3 / stride-1 / pad-1 output convolution (16-bit engines), gfx950.
//
// The three output heads of the reference's models end in GroupNorm -> SiLU -> conv3x3 to a handful of channels:
// the UNet's conv_norm_out -> conv_out (320 -> 4, the eps prediction, fp32), the VAE encoder's (512 -> 8 moments) and
// the VAE decoder's (128 -> 3 RGB, padded to 4) — diffusers UNet2DConditionModel / AutoencoderKL as
// src/inference.py:486 runs them.  As a GEMM these have N <= 8: the large-tile kernels cannot take them and the
// 4-wave kernel ran the UNet's at 17 TF/s (88 us per batch-16 call) behind a separate GroupNorm pass that writes and
// re-reads the normalised 320-channel tensor.  Here one kernel reads the raw activation once:
//   * block = a 4-row x 64-column output tile of one image (4 waves, one output row each); per 64-channel chunk the
//     (4 + 2) x (64 + 2) input halo is loaded, normalised (y = silu(x * a_c + b_c), the gn_apply_kernel arithmetic and
//     16-bit rounding: gn_act) into LDS, out-of-image halo pixels as zeros (the conv pads the normalised tensor);
//   * 16x16x32 MFMAs with the output channels as N (padded to 16 with zero B lanes), the 9 taps as shifted A
//     fragment reads of the halo (chunk XOR-swizzled by pixel: conflict-free for 16 consecutive pixels);
//   * the next chunk's halo is loaded into registers before this chunk's MFMAs (its latency hides under them).
// Bound: the VALU of the normalisation (exp + rcp per element, 1.5 x halo overlap) and the HBM read of the input.
#include "ops.h"
#include "profile.h"

namespace irx {
namespace {

constexpr int kTR = 4, kTW = 64;                     // output tile rows x columns
constexpr int kHR = kTR + 2, kHW = kTW + 2;          // halo rows x columns
constexpr int kHPix = kHR * kHW;                     // 396 halo pixels
constexpr int kSlots = kHPix * 8;                    // 16-byte slots per 64-channel chunk (3168)
constexpr int kPer = (kSlots + 255) / 256;           // slots per thread (13)
constexpr int kMaxC = 2048;

template <typename T, bool OUTF32>
__global__ __launch_bounds__(256) void gn_conv_narrow_kernel(const T* __restrict__ x, int H, int W, int C,
                                                             const float2* __restrict__ ab, int silu,
                                                             const T* __restrict__ w, const float* __restrict__ bias,
                                                             int cout, int ldo, void* __restrict__ out, int tiles_x,
                                                             int tiles_y) {
  __shared__ __attribute__((aligned(16))) uint4 hal[kSlots];
  __shared__ float2 sab[kMaxC];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int bid = blockIdx.x;
  const int tx = bid % tiles_x, ty = (bid / tiles_x) % tiles_y, n = bid / (tiles_x * tiles_y);
  const int x0 = tx * kTW, y0 = ty * kTR;
  for (int c = tid; c < C; c += 256) sab[c] = ab[(long)n * C + c];
  const T* xn = x + (long)n * H * W * C;

  // halo slot i = pixel p (row p / kHW, column p % kHW of the halo) x logical 16-byte chunk k (channels 8k .. 8k + 7)
  uint4 v[kPer];
  auto load = [&](int ck) {
#pragma unroll
    for (int j = 0; j < kPer; ++j) {
      const int i = tid + j * 256;
      const int p = i >> 3, k = i & 7;
      const int yy = y0 - 1 + p / kHW, xx = x0 - 1 + p % kHW;
      const bool ok = i < kSlots && yy >= 0 && yy < H && xx >= 0 && xx < W;
      v[j] = ok ? *(const uint4*)(xn + ((long)yy * W + xx) * C + ck * 64 + k * 8) : uint4{0u, 0u, 0u, 0u};
    }
  };
  auto store = [&](int ck) {
#pragma unroll
    for (int j = 0; j < kPer; ++j) {
      const int i = tid + j * 256;
      if (i >= kSlots) break;
      const int p = i >> 3, k = i & 7;
      const int yy = y0 - 1 + p / kHW, xx = x0 - 1 + p % kHW;
      uint4 u = uint4{0u, 0u, 0u, 0u};
      if (yy >= 0 && yy < H && xx >= 0 && xx < W) {   // (padding stays zero: it pads the normalised tensor)
        float f[8];
        Vec16<T>::unpack(v[j], f);
        const int c0 = ck * 64 + k * 8;
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          const float2 s = sab[c0 + e];
          f[e] = gn_act(f[e], s.x, s.y, silu);
        }
        u = Vec16<T>::pack(f);
      }
      hal[p * 8 + (k ^ (p & 7))] = u;
    }
  };

  const int frow = lane & 15, kg = lane >> 4;
  const bool bcol = frow < cout;
  f32x4 acc[4];
#pragma unroll
  for (int m = 0; m < 4; ++m) acc[m] = f32x4{0.f, 0.f, 0.f, 0.f};
  const int nck = C / 64;
  load(0);
  __syncthreads();   // sab visible
  for (int ck = 0; ck < nck; ++ck) {
    store(ck);
    __syncthreads();
    if (ck + 1 < nck) load(ck + 1);   // lands under this chunk's MFMAs
#pragma unroll
    for (int t = 0; t < 9; ++t) {
      const int ky = t / 3, kx = t % 3;
#pragma unroll
      for (int s = 0; s < 2; ++s) {
        const int koff = ck * 64 + s * 32 + kg * 8;
        const uint4 b = bcol ? *(const uint4*)(w + ((long)frow * 9 + t) * C + koff) : uint4{0u, 0u, 0u, 0u};
#pragma unroll
        for (int m = 0; m < 4; ++m) {
          const int p = (wave + ky) * kHW + m * 16 + frow + kx;
          const uint4 a = hal[p * 8 + ((s * 4 + kg) ^ (p & 7))];
          acc[m] = Mfma<T>::m16x16x32(a, b, acc[m]);
        }
      }
    }
    __syncthreads();   // every wave done reading this chunk before the next store overwrites it
  }
  // D[row = 4 kg + r][col = frow] of m-tile m: output pixel (y0 + wave, x0 + 16 m + 4 kg + r), channel frow
  if (!bcol) return;
  const int y = y0 + wave;
  if (y >= H) return;
  const float bv = bias ? bias[frow] : 0.f;
#pragma unroll
  for (int m = 0; m < 4; ++m)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int xo = x0 + m * 16 + kg * 4 + r;
      if (xo >= W) continue;
      const long o = (((long)n * H + y) * W + xo) * ldo + frow;
      const float val = acc[m][r] + bv;
      if constexpr (OUTF32) ((float*)out)[o] = val;
      else ((T*)out)[o] = from_f<T>(val);
    }
}

}  // namespace

int g_gn_narrow = 1;

bool gn_conv_narrow_ok(int dtype, int C, int cout) {
  return is16(dtype) && C % 64 == 0 && C <= kMaxC && cout >= 1 && cout <= 16;
}

void gn_conv_narrow(int dtype, const void* x, int N, int H, int W, int C, const float2* ab, int silu, const void* w,
                    const float* bias, int cout, void* out, int ldo, int out_f32, hipStream_t s) {
  IRX_CHECK(gn_conv_narrow_ok(dtype, C, cout), "gn_conv_narrow: 16-bit, C % 64 == 0, C <= 2048, cout <= 16");
  IRX_CHECK(ldo >= cout && N > 0 && H > 0 && W > 0, "gn_conv_narrow: shape");
  IRX_CHECK(((uintptr_t)x % 16) == 0 && ((uintptr_t)w % 16) == 0, "gn_conv_narrow: 16-byte aligned operands");
  const int tiles_x = (W + kTW - 1) / kTW, tiles_y = (H + kTR - 1) / kTR;
  const dim3 grid((unsigned)((long)N * tiles_x * tiles_y)), block(256);
  ProfScope ps(prof_on() ? std::string("irx::(anonymous namespace)::gn_conv_narrow_kernel<") +
                               (dtype == F16 ? "_Float16" : "unsigned short") + (out_f32 ? ", true>" : ", false>")
                         : std::string(),
               2.0 * N * H * W * (double)cout * 9 * C, s);
  if (dtype == F16) {
    if (out_f32)
      gn_conv_narrow_kernel<f16_t, true><<<grid, block, 0, s>>>((const f16_t*)x, H, W, C, ab, silu, (const f16_t*)w,
                                                                bias, cout, ldo, out, tiles_x, tiles_y);
    else
      gn_conv_narrow_kernel<f16_t, false><<<grid, block, 0, s>>>((const f16_t*)x, H, W, C, ab, silu, (const f16_t*)w,
                                                                 bias, cout, ldo, out, tiles_x, tiles_y);
  } else {
    if (out_f32)
      gn_conv_narrow_kernel<bf16_t, true><<<grid, block, 0, s>>>((const bf16_t*)x, H, W, C, ab, silu,
                                                                 (const bf16_t*)w, bias, cout, ldo, out, tiles_x,
                                                                 tiles_y);
    else
      gn_conv_narrow_kernel<bf16_t, false><<<grid, block, 0, s>>>((const bf16_t*)x, H, W, C, ab, silu,
                                                                  (const bf16_t*)w, bias, cout, ldo, out, tiles_x,
                                                                  tiles_y);
  }
  IRX_LAUNCH_CHECK();
}

}  // namespace irx
