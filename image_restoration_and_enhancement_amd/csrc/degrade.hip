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

// Separable binomial blur through LDS: a block owns TW x TH output pixels of one image (all channels);
// the (TH + 2r) x (TW + 2r) input tile is staged once, the exact integer row sums go to LDS, columns finish
// in registers: sum_y w_y * (sum_x w_x * p), round half up >> 16 (integer weights: exact).
constexpr int kBlurTW = 64, kBlurTH = 16, kBlurR = 3, kBlurCmax = 4;
__global__ __launch_bounds__(256) void gauss_kernel(const uint8_t* __restrict__ img, uint8_t* __restrict__ out,
                                                    int B, int H, int W, int C, const int* __restrict__ ksize) {
  __shared__ uint8_t tin[(kBlurTH + 2 * kBlurR) * (kBlurTW + 2 * kBlurR) * kBlurCmax];
  __shared__ int th[(kBlurTH + 2 * kBlurR) * kBlurTW * kBlurCmax];
  const int b = blockIdx.z, x0 = blockIdx.x * kBlurTW, y0 = blockIdx.y * kBlurTH;
  const int row = min(max(ksize[b] / 2, 0), 3), r = row;   // k in {1, 3, 5, 7} (others: clamped)
  const uint8_t* base = img + (long)b * H * W * C;
  const int IW = kBlurTW + 2 * r, IH = kBlurTH + 2 * r;
  for (int e = threadIdx.x; e < IH * IW * C; e += blockDim.x) {
    const int c = e % C, q = e / C, ix = q % IW, iy = q / IW;
    tin[e] = base[((long)reflect101(y0 - r + iy, H) * W + reflect101(x0 - r + ix, W)) * C + c];
  }
  __syncthreads();
  for (int e = threadIdx.x; e < IH * kBlurTW * C; e += blockDim.x) {
    const int c = e % C, q = e / C, ox = q % kBlurTW, iy = q / kBlurTW;
    int h = 0;
    for (int j = 0; j <= 2 * r; ++j) h += c_gauss[row][j] * tin[(iy * IW + ox + j) * C + c];
    th[e] = h;
  }
  __syncthreads();
  for (int e = threadIdx.x; e < kBlurTH * kBlurTW * C; e += blockDim.x) {
    const int c = e % C, q = e / C, ox = q % kBlurTW, oy = q / kBlurTW;
    if (x0 + ox >= W || y0 + oy >= H) continue;
    long acc = 0;
    for (int j = 0; j <= 2 * r; ++j) acc += (long)c_gauss[row][j] * th[((oy + j) * kBlurTW + ox) * C + c];
    out[(((long)b * H + y0 + oy) * W + x0 + ox) * C + c] = (uint8_t)min(255L, (acc + 32768) >> 16);
  }
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

// mode 0: BGR2GRAY fixed point; mode 1: L of BGR2Lab (the sRGB linearisation of the 256 levels is
// computed once per block into LDS).  rgb != 0: channel order R, G, B in memory.
__global__ __launch_bounds__(256) void gray_kernel(const uint8_t* __restrict__ img, uint8_t* __restrict__ out,
                                                   long npix, int mode, int rgb) {
  __shared__ float lin[256];
  if (mode == 1) {
    lin[threadIdx.x] = srgb_lin(threadIdx.x * (1.f / 255.f));
    __syncthreads();
  }
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= npix) return;
  const uint8_t c0 = img[i * 3], c1 = img[i * 3 + 1], c2 = img[i * 3 + 2];
  const int R = rgb ? c0 : c2, G = c1, Bc = rgb ? c2 : c0;
  if (mode == 0) {
    out[i] = (uint8_t)((R * 4899 + G * 9617 + Bc * 1868 + (1 << 13)) >> 14);
    return;
  }
  const float Y = 0.212671f * lin[R] + 0.715160f * lin[G] + 0.072169f * lin[Bc];
  const float L = Y > 0.008856f ? 116.f * cbrtf(Y) - 16.f : 903.3f * Y;
  out[i] = (uint8_t)fminf(fmaxf(rintf(L * 2.55f), 0.f), 255.f);
}

// segs: [nseg][4] (x0, y0, x1, y1), thick: [nseg], seg_off: [B+1] (image b owns segs seg_off[b] .. seg_off[b+1]).
// A block owns a 16 x 16 pixel tile: it first culls the image's segments to those whose bounding box,
// grown by half the thickness, touches the tile (LDS list), then every pixel runs the exact capsule
// test against that short list only.
constexpr int kStrokeT = 16, kStrokeMaxList = 1024;
__device__ __forceinline__ bool in_capsule(int x, int y, const int* sg, int t) {
  // int64 throughout, as the numpy oracle (oracle/degrade_ref.py stroke_mask): exact while every coordinate
  // lies in [-2^15, 2^15) — then (vx^2 + vy^2) * L2 < 2^62 (irx_degrade_strokes checks H, W <= 2^14; the
  // stroke generator clips its points to the image)
  const long x0 = sg[0], y0 = sg[1], x1 = sg[2], y1 = sg[3], tt = (long)t * t;
  const long dx = x1 - x0, dy = y1 - y0, vx = x - x0, vy = y - y0;
  const long L2 = dx * dx + dy * dy, dot = vx * dx + vy * dy;
  if (L2 == 0 || dot <= 0) return 4 * (vx * vx + vy * vy) <= tt;
  if (dot >= L2) {
    const long ux = x - x1, uy = y - y1;
    return 4 * (ux * ux + uy * uy) <= tt;
  }
  return 4 * ((vx * vx + vy * vy) * L2 - dot * dot) <= tt * L2;   // perpendicular distance^2 * L2
}

__global__ __launch_bounds__(256) void stroke_kernel(int B, int H, int W, const int* __restrict__ segs,
                                                     const int* __restrict__ thick, const int* __restrict__ seg_off,
                                                     uint8_t* __restrict__ mask, const uint8_t* __restrict__ img,
                                                     uint8_t* __restrict__ masked) {
  __shared__ int list[kStrokeMaxList];
  __shared__ int cnt;
  const int b = blockIdx.z, tx0 = blockIdx.x * kStrokeT, ty0 = blockIdx.y * kStrokeT;
  const int s0 = seg_off[b], s1 = seg_off[b + 1];
  if (threadIdx.x == 0) cnt = 0;
  __syncthreads();
  for (int sg = s0 + threadIdx.x; sg < s1; sg += blockDim.x) {
    const int* p = segs + 4 * sg;
    const int h = (thick[sg] + 1) / 2 + 1;
    const int xl = min(p[0], p[2]) - h, xh = max(p[0], p[2]) + h, yl = min(p[1], p[3]) - h, yh = max(p[1], p[3]) + h;
    if (xh >= tx0 && xl < tx0 + kStrokeT && yh >= ty0 && yl < ty0 + kStrokeT) {
      const int k = atomicAdd(&cnt, 1);
      if (k < kStrokeMaxList) list[k] = sg;
    }
  }
  __syncthreads();
  const int x = tx0 + (threadIdx.x & (kStrokeT - 1)), y = ty0 + threadIdx.x / kStrokeT;
  if (x >= W || y >= H) return;
  const int n = cnt;
  bool on = false;
  if (n <= kStrokeMaxList) {
    for (int k = 0; k < n && !on; ++k) on = in_capsule(x, y, segs + 4 * list[k], thick[list[k]]);
  } else {
    for (int sg = s0; sg < s1 && !on; ++sg) on = in_capsule(x, y, segs + 4 * sg, thick[sg]);
  }
  const long i = ((long)b * H + y) * W + x;
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
  IRX_CHECK(C <= kBlurCmax, "at most 4 channels");
  gauss_kernel<<<dim3((W + kBlurTW - 1) / kBlurTW, (H + kBlurTH - 1) / kBlurTH, B), 256, 0, s>>>(img, blur, B, H, W,
                                                                                                  C, ksize_dev);
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
  stroke_kernel<<<dim3((W + kStrokeT - 1) / kStrokeT, (H + kStrokeT - 1) / kStrokeT, B), 256, 0, s>>>(
      B, H, W, segs, thick, seg_off, mask, img, masked);
  IRX_LAUNCH_CHECK();
}

}  // namespace irx
