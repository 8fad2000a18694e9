// irx — synthetic degradation generator on the GPU: the pixel work of the reference's
// scripts/make_synthetic_pairs.py for whole uint8 batches resident in HBM.
//   * add_gaussian_noise  (make_synthetic_pairs.py:29-35):  clip(img + f32(z) * f32(sigma), 0, 255) -> uint8
//     truncation; z is either a caller-supplied field (numpy's draws: bit-exact) or Philox4x32-10 +
//     Box-Muller in-kernel (seeded, reproducible, not numpy's stream);
//   * degrade_sr          (:67-81, Gaussian branch):         cv2.GaussianBlur(k in {3,5,7}, sigma 0) then
//     cv2.resize(INTER_CUBIC) down by an integer scale.  For 8-bit images OpenCV takes its fixed-point
//     paths with the binomial small-kernel table (weights * 256 exact) and 11-bit cubic coefficients, so
//     both stages are restated as exact integer arithmetic (round-half-up >> 16, and >> 22);
//   * to_grayscale        (:84-90):  "simple" = BGR2GRAY fixed point (4899 R + 9617 G + 1868 B + 2^13) >> 14;
//     "lab" = L of BGR2Lab (sRGB linearisation, CIE L*, * 255 / 100), restated in fp32;
//   * random_free_form_mask (:104-114): thick cv2.line strokes rasterised as capsules (distance to the
//     segment <= thickness / 2, exact int64 test), and the masked input img * (mask == 0) (:196-198).
// All kernels are HBM-bound byte work: one pass, 16-byte-coalesced where the layout allows, no LDS.
#include "ops.h"
#include "profile.h"

namespace irx {
namespace {

// ---------------------------------------------------------------- Philox4x32-10 (Salmon et al. 2011)
__device__ __forceinline__ uint4 philox(uint4 c, uint2 k) {
#pragma unroll
  for (int r = 0; r < 10; ++r) {
    const uint32_t hi0 = __umulhi(0xD2511F53u, c.x), lo0 = 0xD2511F53u * c.x;
    const uint32_t hi1 = __umulhi(0xCD9E8D57u, c.z), lo1 = 0xCD9E8D57u * c.z;
    c = uint4{hi1 ^ c.y ^ k.x, lo1, hi0 ^ c.w ^ k.y, lo0};
    k.x += 0x9E3779B9u;
    k.y += 0xBB67AE85u;
  }
  return c;
}

__global__ __launch_bounds__(256) void noise_kernel(const uint8_t* __restrict__ img, uint8_t* __restrict__ out,
                                                    long n, float sigma, const float* __restrict__ z,
                                                    unsigned long long seed) {
  const long i0 = ((long)blockIdx.x * blockDim.x + threadIdx.x) * 4;   // 4 pixels-channels per thread
  if (i0 >= n) return;
  float zz[4];
  if (z) {
#pragma unroll
    for (int e = 0; e < 4; ++e) zz[e] = i0 + e < n ? z[i0 + e] : 0.f;
  } else {
    const uint4 r = philox(uint4{(uint32_t)(i0 >> 2), (uint32_t)(i0 >> 34), 0x1234567u, 0u},
                           uint2{(uint32_t)seed, (uint32_t)(seed >> 32)});
    const float u0 = ((float)r.x + 0.5f) * 2.3283064e-10f, u1 = ((float)r.y + 0.5f) * 2.3283064e-10f;
    const float u2 = ((float)r.z + 0.5f) * 2.3283064e-10f, u3 = ((float)r.w + 0.5f) * 2.3283064e-10f;
    const float m0 = sqrtf(-2.f * logf(u0)), m1 = sqrtf(-2.f * logf(u2));
    zz[0] = m0 * cosf(6.2831855f * u1); zz[1] = m0 * sinf(6.2831855f * u1);
    zz[2] = m1 * cosf(6.2831855f * u3); zz[3] = m1 * sinf(6.2831855f * u3);
  }
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    if (i0 + e >= n) break;
    // numpy: (randn.astype(f32) * sigma) in f32, img.astype(f32) + noise in f32, clip, astype(uint8)
    const float v = __fadd_rn((float)img[i0 + e], __fmul_rn(zz[e], sigma));
    out[i0 + e] = (uint8_t)(int)fminf(fmaxf(v, 0.f), 255.f);
  }
}

// OpenCV's small Gaussian kernels (sigma <= 0, k <= 7), times 256
__constant__ int c_gauss[4][7] = {{256, 0, 0, 0, 0, 0, 0},
                                  {64, 128, 64, 0, 0, 0, 0},
                                  {16, 64, 96, 64, 16, 0, 0},
                                  {8, 28, 56, 72, 56, 28, 8}};

__device__ __forceinline__ int reflect101(int i, int n) {
  if (n == 1) return 0;
  while (i < 0 || i >= n) i = i < 0 ? -i : 2 * n - 2 - i;
  return i;
}

// one output pixel-channel: sum_y w_y * (sum_x w_x * p) with integer weights (exact), round half up >> 16
__global__ __launch_bounds__(256) void gauss_kernel(const uint8_t* __restrict__ img, uint8_t* __restrict__ out,
                                                    int B, int H, int W, int C, const int* __restrict__ ksize) {
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  const long n = (long)B * H * W * C;
  if (i >= n) return;
  const int c = (int)(i % C);
  const long p = i / C;
  const int x = (int)(p % W), y = (int)((p / W) % H), b = (int)(p / ((long)W * H));
  const int row = min(max(ksize[b] / 2, 0), 3), r = row;   // k in {1, 3, 5, 7} (others: clamped)
  const uint8_t* base = img + (long)b * H * W * C;
  long acc = 0;
  for (int dy = -r; dy <= r; ++dy) {
    const int yy = reflect101(y + dy, H);
    int h = 0;
    for (int dx = -r; dx <= r; ++dx) h += c_gauss[row][dx + r] * base[((long)yy * W + reflect101(x + dx, W)) * C + c];
    acc += (long)c_gauss[row][dy + r] * h;
  }
  out[i] = (uint8_t)min(255L, (acc + 32768) >> 16);
}

// OpenCV INTER_CUBIC (A = -0.75), coefficients * 2048 rounded to short, horizontal int sums, vertical
// (sum + 2^21) >> 22 saturated; source taps clamped to the image
__device__ __forceinline__ void cubic_coeffs(float t, int w[4]) {
  const float A = -0.75f;
  float c[4];
  c[0] = ((A * (t + 1.f) - 5.f * A) * (t + 1.f) + 8.f * A) * (t + 1.f) - 4.f * A;
  c[1] = ((A + 2.f) * t - (A + 3.f)) * t * t + 1.f;
  c[2] = ((A + 2.f) * (1.f - t) - (A + 3.f)) * (1.f - t) * (1.f - t) + 1.f;
  c[3] = 1.f - c[0] - c[1] - c[2];
#pragma unroll
  for (int e = 0; e < 4; ++e) w[e] = (int)rintf(c[e] * 2048.f);
}

__global__ __launch_bounds__(256) void cubic_down_kernel(const uint8_t* __restrict__ src, uint8_t* __restrict__ out,
                                                         int B, int H, int W, int C, int Ho, int Wo) {
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  const long n = (long)B * Ho * Wo * C;
  if (i >= n) return;
  const int c = (int)(i % C);
  const long p = i / C;
  const int x = (int)(p % Wo), y = (int)((p / Wo) % Ho), b = (int)(p / ((long)Wo * Ho));
  const float fx = (x + 0.5f) * ((float)W / Wo) - 0.5f, fy = (y + 0.5f) * ((float)H / Ho) - 0.5f;
  const int sx = (int)floorf(fx), sy = (int)floorf(fy);
  int wx[4], wy[4];
  cubic_coeffs(fx - sx, wx);
  cubic_coeffs(fy - sy, wy);
  const uint8_t* base = src + (long)b * H * W * C;
  long acc = 0;
#pragma unroll
  for (int ky = 0; ky < 4; ++ky) {
    const int yy = min(max(sy - 1 + ky, 0), H - 1);
    int h = 0;
#pragma unroll
    for (int kx = 0; kx < 4; ++kx) h += wx[kx] * base[((long)yy * W + min(max(sx - 1 + kx, 0), W - 1)) * C + c];
    acc += (long)wy[ky] * h;
  }
  out[i] = (uint8_t)min(255L, max(0L, (acc + (1L << 21)) >> 22));
}

__device__ __forceinline__ float srgb_lin(float v) {
  return v <= 0.04045f ? v * (1.f / 12.92f) : powf((v + 0.055f) * (1.f / 1.055f), 2.4f);
}

// mode 0: BGR2GRAY fixed point; mode 1: L of BGR2Lab.  rgb != 0: channel order R, G, B in memory.
__global__ __launch_bounds__(256) void gray_kernel(const uint8_t* __restrict__ img, uint8_t* __restrict__ out,
                                                   long npix, int mode, int rgb) {
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= npix) return;
  const uint8_t c0 = img[i * 3], c1 = img[i * 3 + 1], c2 = img[i * 3 + 2];
  const int R = rgb ? c0 : c2, G = c1, Bc = rgb ? c2 : c0;
  if (mode == 0) {
    out[i] = (uint8_t)((R * 4899 + G * 9617 + Bc * 1868 + (1 << 13)) >> 14);
    return;
  }
  const float Y = 0.212671f * srgb_lin(R * (1.f / 255.f)) + 0.715160f * srgb_lin(G * (1.f / 255.f)) +
                  0.072169f * srgb_lin(Bc * (1.f / 255.f));
  const float L = Y > 0.008856f ? 116.f * cbrtf(Y) - 16.f : 903.3f * Y;
  out[i] = (uint8_t)fminf(fmaxf(rintf(L * 2.55f), 0.f), 255.f);
}

// segs: [nseg][4] (x0, y0, x1, y1), thick: [nseg], seg_off: [B+1] (image b owns segs seg_off[b] .. seg_off[b+1])
__global__ __launch_bounds__(256) void stroke_kernel(int B, int H, int W, const int* __restrict__ segs,
                                                     const int* __restrict__ thick, const int* __restrict__ seg_off,
                                                     uint8_t* __restrict__ mask, const uint8_t* __restrict__ img,
                                                     uint8_t* __restrict__ masked) {
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= (long)B * H * W) return;
  const int x = (int)(i % W), y = (int)((i / W) % H), b = (int)(i / ((long)W * H));
  bool on = false;
  for (int s = seg_off[b]; s < seg_off[b + 1] && !on; ++s) {
    const long x0 = segs[4 * s], y0 = segs[4 * s + 1], x1 = segs[4 * s + 2], y1 = segs[4 * s + 3];
    const long t = thick[s];
    const long dx = x1 - x0, dy = y1 - y0, vx = x - x0, vy = y - y0;
    const long L2 = dx * dx + dy * dy, dot = vx * dx + vy * dy;
    if (L2 == 0 || dot <= 0) {
      on = 4 * (vx * vx + vy * vy) <= t * t;
    } else if (dot >= L2) {
      const long ux = x - x1, uy = y - y1;
      on = 4 * (ux * ux + uy * uy) <= t * t;
    } else {   // perpendicular distance^2 = (|v|^2 L2 - dot^2) / L2
      on = 4 * ((vx * vx + vy * vy) * L2 - dot * dot) <= t * t * L2;
    }
  }
  mask[i] = on ? 255 : 0;
  if (img && masked) {
#pragma unroll
    for (int e = 0; e < 3; ++e) masked[i * 3 + e] = on ? 0 : img[i * 3 + e];
  }
}

unsigned blocks(long n, int per_thread = 1) { return (unsigned)((n / per_thread + 255) / 256 + 1); }

}  // namespace

void degrade_noise(const uint8_t* img, uint8_t* out, long n, float sigma, const float* z, unsigned long long seed,
                   hipStream_t s) {
  ProfScope ps(prof_on() ? std::string("irx::(anonymous namespace)::noise_kernel") : std::string(), 0.0, s);
  noise_kernel<<<blocks(n, 4), 256, 0, s>>>(img, out, n, sigma, z, seed);
  IRX_LAUNCH_CHECK();
}

void degrade_blur_down(const uint8_t* img, int B, int H, int W, int C, const int* ksize_dev, int scale,
                       uint8_t* blur, uint8_t* lr, hipStream_t s) {
  const long n = (long)B * H * W * C;
  gauss_kernel<<<blocks(n), 256, 0, s>>>(img, blur, B, H, W, C, ksize_dev);
  IRX_LAUNCH_CHECK();
  if (lr && scale >= 1) {
    const int Ho = H / scale, Wo = W / scale;
    cubic_down_kernel<<<blocks((long)B * Ho * Wo * C), 256, 0, s>>>(blur, lr, B, H, W, C, Ho, Wo);
    IRX_LAUNCH_CHECK();
  }
}

void degrade_gray(const uint8_t* img, long npix, int mode, int rgb, uint8_t* out, hipStream_t s) {
  gray_kernel<<<blocks(npix), 256, 0, s>>>(img, out, npix, mode, rgb);
  IRX_LAUNCH_CHECK();
}

void degrade_strokes(int B, int H, int W, const int* segs, const int* thick, const int* seg_off, uint8_t* mask,
                     const uint8_t* img, uint8_t* masked, hipStream_t s) {
  stroke_kernel<<<blocks((long)B * H * W), 256, 0, s>>>(B, H, W, segs, thick, seg_off, mask, img, masked);
  IRX_LAUNCH_CHECK();
}

}  // namespace irx
