// Is v_mfma_f32_16x16x32_{f16,bf16} symmetric in its operands?  gemm_sk computes D^T = B A^T (the weight fragment as
// the first operand) where the large-tile kernel computes D = A B^T with the same fragments; if the two products
// differ in the last fp32 bits, fp16 outputs of the two kernels can differ by an ulp (test_gemm_sk, VERDICT r3 #2b).
// For random fragments and accumulators this counts the elements where mfma(a, b, c)[i][j] != mfma(b, a, c^T)[j][i].
//   hipcc --offload-arch=gfx950 -O3 -o mfma_swap_check scripts/mfma_swap_check.hip && ./mfma_swap_check
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <cmath>
#include <vector>

typedef __attribute__((ext_vector_type(4))) float f32x4;
typedef __attribute__((ext_vector_type(8))) _Float16 f16x8;
typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8;

// a[t][lane] / b[t][lane]: 8 16-bit elements per lane (row lane & 15, k (lane >> 4) * 8 ..); c[t][16][16]
template <bool F16>
__global__ void swap_kernel(const uint4* a, const uint4* b, const float* c, float* d_ab, float* d_ba, int trials) {
  const int t = blockIdx.x, lane = threadIdx.x;
  if (t >= trials) return;
  const uint4 fa = a[t * 64 + lane], fb = b[t * 64 + lane];
  const int col = lane & 15, r0 = (lane >> 4) * 4;
  f32x4 c1, c2;
  for (int r = 0; r < 4; ++r) {
    c1[r] = c[t * 256 + (r0 + r) * 16 + col];   // D[row][col] layout: row = 4 * (lane >> 4) + r, col = lane & 15
    c2[r] = c[t * 256 + col * 16 + (r0 + r)];   // the transposed accumulator for the swapped product
  }
  f32x4 x, y;
  if constexpr (F16) {
    x = __builtin_amdgcn_mfma_f32_16x16x32_f16(__builtin_bit_cast(f16x8, fa), __builtin_bit_cast(f16x8, fb), c1, 0, 0, 0);
    y = __builtin_amdgcn_mfma_f32_16x16x32_f16(__builtin_bit_cast(f16x8, fb), __builtin_bit_cast(f16x8, fa), c2, 0, 0, 0);
  } else {
    x = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, fa), __builtin_bit_cast(bf16x8, fb), c1, 0, 0, 0);
    y = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, fb), __builtin_bit_cast(bf16x8, fa), c2, 0, 0, 0);
  }
  for (int r = 0; r < 4; ++r) {
    d_ab[t * 256 + (r0 + r) * 16 + col] = x[r];
    d_ba[t * 256 + col * 16 + (r0 + r)] = y[r];   // y holds (B A^T)[col'][row'] at row' = r0 + r, col' = col
  }
}

static uint16_t rnd16(bool f16, unsigned& s) {
  s = s * 1664525u + 1013904223u;
  const float v = ((s >> 8) & 0xffff) / 32768.0f - 1.0f;   // [-1, 1)
  if (f16) {
    const _Float16 h = (_Float16)v;
    return *(const uint16_t*)&h;
  }
  uint32_t u;
  std::memcpy(&u, &v, 4);
  return (uint16_t)(u >> 16);
}

int main() {
  const int trials = 4096;
  for (int f = 0; f < 2; ++f) {
    const bool f16 = f == 0;
    std::vector<uint16_t> ha(trials * 64 * 8), hb(trials * 64 * 8);
    std::vector<float> hc(trials * 256);
    unsigned s = 12345u + f;
    for (auto& x : ha) x = rnd16(f16, s);
    for (auto& x : hb) x = rnd16(f16, s);
    for (auto& x : hc) { s = s * 1664525u + 1013904223u; x = ((s >> 8) & 0xffff) / 8192.0f - 4.0f; }
    uint4 *da, *db;
    float *dc, *dab, *dba;
    hipMalloc(&da, ha.size() * 2); hipMalloc(&db, hb.size() * 2); hipMalloc(&dc, hc.size() * 4);
    hipMalloc(&dab, hc.size() * 4); hipMalloc(&dba, hc.size() * 4);
    hipMemcpy(da, ha.data(), ha.size() * 2, hipMemcpyHostToDevice);
    hipMemcpy(db, hb.data(), hb.size() * 2, hipMemcpyHostToDevice);
    for (int withc = 0; withc < 2; ++withc) {
      std::vector<float> c0(hc.size(), 0.f);
      hipMemcpy(dc, withc ? hc.data() : c0.data(), hc.size() * 4, hipMemcpyHostToDevice);
      if (f16) swap_kernel<true><<<trials, 64>>>(da, db, dc, dab, dba, trials);
      else swap_kernel<false><<<trials, 64>>>(da, db, dc, dab, dba, trials);
      if (hipDeviceSynchronize() != hipSuccess) { printf("kernel failed\n"); return 1; }
      std::vector<float> ab(hc.size()), ba(hc.size());
      hipMemcpy(ab.data(), dab, ab.size() * 4, hipMemcpyDeviceToHost);
      hipMemcpy(ba.data(), dba, ba.size() * 4, hipMemcpyDeviceToHost);
      long diff = 0;
      double maxrel = 0;
      for (size_t i = 0; i < ab.size(); ++i) {
        if (ab[i] != ba[i]) {
          ++diff;
          const double r = fabs((double)ab[i] - ba[i]) / (fabs((double)ab[i]) + 1e-30);
          if (r > maxrel) maxrel = r;
        }
      }
      printf("%s %s accumulator: %ld of %zu elements differ between mfma(a,b) and mfma(b,a)^T (max rel %.3g)\n",
             f16 ? "f16 " : "bf16", withc ? "random" : "zero  ", diff, ab.size(), maxrel);
    }
    hipFree(da); hipFree(db); hipFree(dc); hipFree(dab); hipFree(dba);
  }
  return 0;
}
