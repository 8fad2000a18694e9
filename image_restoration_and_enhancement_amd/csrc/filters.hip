// irx — the two edge-preserving filters that follow the NLM pass in the reference's classical denoise fallback
// (src/inference.py:517-520), on uint8 [B][H][W][3] batches resident in HBM:
//   * bilateral_kernel  cv2.bilateralFilter(img, 9, 75, 75) for 8-bit 3-channel images (BilateralFilter_8u):
//     circular window (offsets with sqrt(i^2 + j^2) <= r, row-major), w = space_w[k] * color_w[|db|+|dg|+|dr|]
//     in fp32 from host-built tables, per-pixel sums accumulated in window order without contraction, result
//     cvRound(sum * (1 / wsum)); BORDER_REFLECT_101.  Checked bit-exact against oracle/filters_ref.py.
//   * median_kernel     cv2.medianBlur(img, 5): per-channel 5x5 median, BORDER_REPLICATE (exact).
// Both stage a reflect/replicate-padded tile in LDS and are VALU-bound: HBM traffic is one read and one write.
#include "ops.h"
#include "profile.h"

namespace irx {
namespace {

constexpr int FT_W = 32, FT_H = 8;                            // 32x8 pixel tile, one pixel per thread

__device__ __forceinline__ int refl101f(int p, int n) {
  if (n == 1) return 0;
  while ((unsigned)p >= (unsigned)n) p = p < 0 ? -p : 2 * (n - 1) - p;
  return p;
}

template <int R>
__global__ __launch_bounds__(256) void bilateral_kernel(const uint8_t* __restrict__ src, uint8_t* __restrict__ dst,
                                                        int H, int W, const float* __restrict__ space_w,
                                                        const int* __restrict__ space_dydx, int maxk,
                                                        const float* __restrict__ color_w) {
  constexpr int RH = FT_H + 2 * R, RW = FT_W + 2 * R;
  __shared__ uint32_t tile[RH * RW];                          // packed b | g << 8 | r << 16
  __shared__ float cw[256 * 3];
  __shared__ float sw[(2 * R + 1) * (2 * R + 1)];
  __shared__ int so[(2 * R + 1) * (2 * R + 1)];
  const int tid = threadIdx.x, x0 = blockIdx.x * FT_W, y0 = blockIdx.y * FT_H;
  const uint8_t* img = src + (size_t)blockIdx.z * H * W * 3;
  for (int i = tid; i < RH * RW; i += 256) {
    const int ry = i / RW, rx = i - ry * RW;
    const uint8_t* p = img + ((size_t)refl101f(y0 + ry - R, H) * W + refl101f(x0 + rx - R, W)) * 3;
    tile[i] = (uint32_t)p[0] | ((uint32_t)p[1] << 8) | ((uint32_t)p[2] << 16);
  }
  for (int i = tid; i < 256 * 3; i += 256) cw[i] = color_w[i];
  for (int i = tid; i < maxk; i += 256) {
    sw[i] = space_w[i];
    so[i] = (space_dydx[2 * i] + R) * RW + space_dydx[2 * i + 1] + R;   // tile offset of (dy, dx)
  }
  __syncthreads();
  const int tx = tid % FT_W, ty = tid / FT_W, x = x0 + tx, y = y0 + ty;
  const uint32_t* base = tile + ty * RW + tx;
  const uint32_t c0 = base[R * RW + R];
  const int b0 = c0 & 255, g0 = (c0 >> 8) & 255, r0 = c0 >> 16;
  float wsum = 0.f, sb = 0.f, sg = 0.f, sr = 0.f;
  for (int k = 0; k < maxk; ++k) {
    const uint32_t c = base[so[k]];
    const int b = c & 255, g = (c >> 8) & 255, r = c >> 16;
    const float w = __fmul_rn(sw[k], cw[abs(b - b0) + abs(g - g0) + abs(r - r0)]);
    wsum = __fadd_rn(wsum, w);
    sb = __fadd_rn(sb, __fmul_rn((float)b, w));
    sg = __fadd_rn(sg, __fmul_rn((float)g, w));
    sr = __fadd_rn(sr, __fmul_rn((float)r, w));
  }
  if (y < H && x < W) {
    const float inv = __fdiv_rn(1.f, wsum);
    uint8_t* o = dst + (((size_t)blockIdx.z * H + y) * W + x) * 3;
    o[0] = (uint8_t)min(255, max(0, (int)rintf(__fmul_rn(sb, inv))));
    o[1] = (uint8_t)min(255, max(0, (int)rintf(__fmul_rn(sg, inv))));
    o[2] = (uint8_t)min(255, max(0, (int)rintf(__fmul_rn(sr, inv))));
  }
}

__global__ __launch_bounds__(256) void median_kernel(const uint8_t* __restrict__ src, uint8_t* __restrict__ dst,
                                                     int H, int W, int C) {
  constexpr int R = 2, RH = FT_H + 2 * R, RW = FT_W + 2 * R;
  __shared__ uint8_t tile[4][RH * RW];
  const int tid = threadIdx.x, x0 = blockIdx.x * FT_W, y0 = blockIdx.y * FT_H;
  const uint8_t* img = src + (size_t)blockIdx.z * H * W * C;
  for (int i = tid; i < RH * RW; i += 256) {
    const int ry = i / RW, rx = i - ry * RW;
    const int gy = min(max(y0 + ry - R, 0), H - 1), gx = min(max(x0 + rx - R, 0), W - 1);
    for (int c = 0; c < C; ++c) tile[c][i] = img[((size_t)gy * W + gx) * C + c];
  }
  __syncthreads();
  const int tx = tid % FT_W, ty = tid / FT_W, x = x0 + tx, y = y0 + ty;
  if (y >= H || x >= W) return;
  for (int c = 0; c < C; ++c) {
    int v[25];
#pragma unroll
    for (int i = 0; i < 5; ++i)
#pragma unroll
      for (int j = 0; j < 5; ++j) v[i * 5 + j] = tile[c][(ty + i) * RW + tx + j];
    // forgetful selection (buffer of 14 = 25/2 + 2): move the buffer's min to its front and max to its back,
    // drop both, take the next element; after the last element the one survivor is the 13th smallest
    int lo = 0, hi = 13;
#pragma unroll
    for (int nx = 14; nx <= 25; ++nx) {
#pragma unroll
      for (int i = lo + 1; i <= hi; ++i) {
        const int m = min(v[lo], v[i]);
        v[i] = max(v[lo], v[i]);
        v[lo] = m;
      }
#pragma unroll
      for (int i = lo + 1; i < hi; ++i) {
        const int M = max(v[i], v[hi]);
        v[i] = min(v[i], v[hi]);
        v[hi] = M;
      }
      ++lo;
      --hi;
      if (nx < 25) v[++hi] = v[nx];
    }
    const int med = v[lo];
    dst[(((size_t)blockIdx.z * H + y) * W + x) * C + c] = (uint8_t)med;
  }
}

// 8-bit Lab <-> linear BGR (cv2.COLOR_LBGR2Lab / COLOR_Lab2LBGR as fastNlMeansDenoisingColored applies them),
// the fp64 restatement of classical.rgb_to_lab_u8(srgb=False) / lab_u8_to_rgb(srgb=False) operation for
// operation (this file is built without contraction), one thread per pixel.
__device__ __forceinline__ double lab_f(double t) { return t > 0.008856 ? cbrt(t) : 7.787 * t + 0.13793103448275862; }
__device__ __forceinline__ double lab_finv(double t) {
  return t > 0.20689655172413793 ? t * t * t : (t - 0.13793103448275862) / 7.787;
}
__device__ __forceinline__ uint8_t sat_rint(double v) { return (uint8_t)fmin(fmax(rint(v), 0.0), 255.0); }

__global__ __launch_bounds__(256) void lab_kernel(const uint8_t* __restrict__ src, uint8_t* __restrict__ dst,
                                                  long npix, int dir) {
  const long p = (long)blockIdx.x * 256 + threadIdx.x;
  if (p >= npix) return;
  const uint8_t* s = src + p * 3;
  uint8_t* o = dst + p * 3;
  if (dir == 0) {                                             // LBGR -> Lab
    const double r = s[2] / 255.0, g = s[1] / 255.0, b = s[0] / 255.0;
    const double X = (0.412453 * r + 0.357580 * g + 0.180423 * b) / 0.950456;
    const double Y = (0.212671 * r + 0.715160 * g + 0.072169 * b) / 1.0;
    const double Z = (0.019334 * r + 0.119193 * g + 0.950227 * b) / 1.088754;
    const double fx = lab_f(X), fy = lab_f(Y), fz = lab_f(Z);
    const double L = Y > 0.008856 ? 116.0 * fy - 16.0 : 903.3 * Y;
    o[0] = sat_rint(L * 255.0 / 100.0);
    o[1] = sat_rint(500.0 * (fx - fy) + 128.0);
    o[2] = sat_rint(200.0 * (fy - fz) + 128.0);
  } else {                                                    // Lab -> LBGR
    const double L = s[0] * 100.0 / 255.0, a = s[1] - 128.0, b = s[2] - 128.0;
    const double fy = (L + 16.0) / 116.0, fx = fy + a / 500.0, fz = fy - b / 200.0;
    const double y = L > 7.9996247999999985 ? fy * fy * fy : L / 903.3;
    const double X = lab_finv(fx) * 0.950456, Y = y * 1.0, Z = lab_finv(fz) * 1.088754;
    const double R = 3.240481343200526 * X + -1.5371515162713185 * Y + -0.4985363261688878 * Z;
    const double G = -0.9692549499965682 * X + 1.8759900014898907 * Y + 0.04155592655829284 * Z;
    const double B = 0.05564663913517716 * X + -0.20404133836651123 * Y + 1.0573110696453443 * Z;
    o[0] = sat_rint(fmin(fmax(B, 0.0), 1.0) * 255.0);
    o[1] = sat_rint(fmin(fmax(G, 0.0), 1.0) * 255.0);
    o[2] = sat_rint(fmin(fmax(R, 0.0), 1.0) * 255.0);
  }
}

}  // namespace

void bilateral_u8(const uint8_t* src, uint8_t* dst, int N, int H, int W, int radius, const float* space_w,
                  const int* space_dydx, int maxk, const float* color_w, hipStream_t s) {
  IRX_CHECK(radius == 4 && maxk >= 1 && maxk <= 81, "bilateral: compiled for d = 9 (radius 4)");
  const dim3 grid((W + FT_W - 1) / FT_W, (H + FT_H - 1) / FT_H, N);
  ProfScope pr(prof_on() ? std::string("irx::(anonymous namespace)::bilateral_kernel") : std::string(), 0.0, s);
  hipLaunchKernelGGL(bilateral_kernel<4>, grid, dim3(256), 0, s, src, dst, H, W, space_w, space_dydx, maxk, color_w);
  IRX_HIP(hipGetLastError());
}

void median5_u8(const uint8_t* src, uint8_t* dst, int N, int H, int W, int C, hipStream_t s) {
  IRX_CHECK(C >= 1 && C <= 4, "median: 1 to 4 channels");
  const dim3 grid((W + FT_W - 1) / FT_W, (H + FT_H - 1) / FT_H, N);
  ProfScope pr(prof_on() ? std::string("irx::(anonymous namespace)::median_kernel") : std::string(), 0.0, s);
  hipLaunchKernelGGL(median_kernel, grid, dim3(256), 0, s, src, dst, H, W, C);
  IRX_HIP(hipGetLastError());
}

}  // namespace irx

namespace irx {
void lab_convert_u8(const uint8_t* src, uint8_t* dst, long npix, int dir, hipStream_t s) {
  ProfScope pr(prof_on() ? std::string("irx::(anonymous namespace)::lab_kernel") : std::string(), 0.0, s);
  hipLaunchKernelGGL(lab_kernel, dim3((unsigned)((npix + 255) / 256)), dim3(256), 0, s, src, dst, npix, dir);
  IRX_HIP(hipGetLastError());
}
}  // namespace irx

// ------------------------------------------------------------------------------------------------------
// _auto_mask_from_image (src/inference.py:805-840): RGB2GRAY (fixed point), dark (<= 30) | bright (> 225)
// -> 255, MORPH_CLOSE then MORPH_OPEN with a 5x5 square, border = the operation's neutral value (OpenCV's
// morphologyDefaultBorderValue), then the count of non-zero pixels (the 1 % rule is the caller's).
// One launch per stage over [B][H][W] bytes; the masks are L2-resident, HBM traffic 4 B per pixel at most.
namespace irx {
namespace {
__global__ __launch_bounds__(256) void mask_threshold_kernel(const uint8_t* __restrict__ img,
                                                             uint8_t* __restrict__ m, long npix) {
  const long p = (long)blockIdx.x * 256 + threadIdx.x;
  if (p >= npix) return;
  const uint8_t* q = img + p * 3;                              // R, G, B
  const int g = (q[0] * 4899 + q[1] * 9617 + q[2] * 1868 + (1 << 13)) >> 14;
  m[p] = (g <= 30 || g > 225) ? 255 : 0;
}

// op 0 = dilate (max, border 0), 1 = erode (min, border 255); counts != null: add this stage's non-zeros
__global__ __launch_bounds__(256) void morph5_kernel(const uint8_t* __restrict__ src, uint8_t* __restrict__ dst,
                                                     int H, int W, int op, int* __restrict__ counts) {
  const int x = blockIdx.x * 32 + (threadIdx.x & 31), y = blockIdx.y * 8 + (threadIdx.x >> 5), b = blockIdx.z;
  int v = 0;
  const bool in = x < W && y < H;
  if (in) {
    const uint8_t* s = src + (size_t)b * H * W;
    v = op == 0 ? 0 : 255;
    for (int dy = -2; dy <= 2; ++dy) {
      const int yy = y + dy;
      if (yy < 0 || yy >= H) continue;
      for (int dx = -2; dx <= 2; ++dx) {
        const int xx = x + dx;
        if (xx < 0 || xx >= W) continue;
        const int t = s[(size_t)yy * W + xx];
        v = op == 0 ? max(v, t) : min(v, t);
      }
    }
    dst[((size_t)b * H + y) * W + x] = (uint8_t)v;
  }
  if (counts) {
    __shared__ int part[4];
    unsigned long long bal = __ballot(in && v > 0);
    if ((threadIdx.x & 63) == 0) part[threadIdx.x >> 6] = __popcll(bal);
    __syncthreads();
    if (threadIdx.x == 0) atomicAdd(counts + b, part[0] + part[1] + part[2] + part[3]);
  }
}
}  // namespace

void auto_mask_u8(const uint8_t* img, int B, int H, int W, uint8_t* mask, uint8_t* tmp, int* counts, hipStream_t s) {
  const long npix = (long)B * H * W;
  ProfScope pr(prof_on() ? std::string("irx::(anonymous namespace)::auto_mask") : std::string(), 0.0, s);
  hipLaunchKernelGGL(mask_threshold_kernel, dim3((unsigned)((npix + 255) / 256)), dim3(256), 0, s, img, mask, npix);
  IRX_HIP(hipGetLastError());
  IRX_HIP(hipMemsetAsync(counts, 0, sizeof(int) * B, s));
  const dim3 grid((W + 31) / 32, (H + 7) / 8, B);
  const int ops[4] = {0, 1, 1, 0};                            // close = dilate, erode; open = erode, dilate
  for (int i = 0; i < 4; ++i) {
    const uint8_t* in = i % 2 == 0 ? mask : tmp;
    uint8_t* out = i % 2 == 0 ? tmp : mask;
    hipLaunchKernelGGL(morph5_kernel, grid, dim3(256), 0, s, in, out, H, W, ops[i], i == 3 ? counts : nullptr);
    IRX_HIP(hipGetLastError());
  }
}
}  // namespace irx

// ------------------------------------------------------------------------------------------------------
// _colorize_lab (src/inference.py:683-703): L of RGB2LAB (sRGB), then a fixed L -> RGB colour map.  The
// colour map has only 256 entries and the sRGB linearisation only 256 inputs, so both come from the host's
// fp64 restatement (classical.colorize_from_L / srgb_linear_lut) as tables; the kernel computes L in fp64
// operation for operation (Y row of the RGB->XYZ matrix, cube root, CIE L*, * 255 / 100, rint).
namespace irx {
namespace {
__global__ __launch_bounds__(256) void colorize_kernel(const uint8_t* __restrict__ img, long npix,
                                                       const double* __restrict__ lin, const uint8_t* __restrict__ cmap,
                                                       uint8_t* __restrict__ out) {
  const long p = (long)blockIdx.x * 256 + threadIdx.x;
  if (p >= npix) return;
  const uint8_t* q = img + p * 3;
  const double r = lin[q[0]], g = lin[q[1]], b = lin[q[2]];
  const double Y = (0.212671 * r + 0.715160 * g + 0.072169 * b) / 1.0;
  const double L = Y > 0.008856 ? 116.0 * lab_f(Y) - 16.0 : 903.3 * Y;
  const int l = sat_rint(L * 255.0 / 100.0);
  out[p * 3 + 0] = cmap[l * 3 + 0];
  out[p * 3 + 1] = cmap[l * 3 + 1];
  out[p * 3 + 2] = cmap[l * 3 + 2];
}
}  // namespace

void colorize_lab_u8(const uint8_t* img, long npix, const double* lin, const uint8_t* cmap, uint8_t* out,
                     hipStream_t s) {
  ProfScope pr(prof_on() ? std::string("irx::(anonymous namespace)::colorize_kernel") : std::string(), 0.0, s);
  hipLaunchKernelGGL(colorize_kernel, dim3((unsigned)((npix + 255) / 256)), dim3(256), 0, s, img, npix, lin, cmap, out);
  IRX_HIP(hipGetLastError());
}
}  // namespace irx
