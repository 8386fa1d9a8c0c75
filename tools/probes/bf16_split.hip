// Micro-probe: can the bf16 matrix path carry f32 convolutions at f32 accuracy?
// (1) accuracy: a 16x16 GEMM with K = 64 f32 operands, every operand split exactly into three
//     bf16 parts (x = x0 + x1 + x2, truncation: each part holds the next 8 significand bits),
//     computed (a) by the f32 MFMA chain (v_mfma_f32_16x16x4_f32, the shipped form), (b) by
//     v_mfma_f32_16x16x32_bf16 over all 9 part products (exact products), (c) over the 6 leading
//     ones (x0w0, x0w1, x1w0, x0w2, x1w1, x2w0); max |err| against the f64 sum, in units of the
//     f64 sum of |x||w| (the f32 rounding scale of a dot product).
// (2) issue: ns per iteration of 8 independent bf16 MFMAs with NV VALU instructions of the split
//     (and / sub / perm) interleaved, one and two waves per SIMD.
//   hipcc --offload-arch=gfx950 -O3 tools/probes/bf16_split.hip -o /tmp/bf16_split && /tmp/bf16_split
#include <hip/hip_runtime.h>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef short s16x8 __attribute__((ext_vector_type(8)));

__device__ __forceinline__ void split3(float x, unsigned short& p0, unsigned short& p1, unsigned short& p2) {
  const unsigned u = __float_as_uint(x);
  const float h = __uint_as_float(u & 0xffff0000u);
  const float r = x - h;
  const unsigned ur = __float_as_uint(r);
  const float m = __uint_as_float(ur & 0xffff0000u);
  const float l = r - m;
  p0 = (unsigned short)(u >> 16);
  p1 = (unsigned short)(ur >> 16);
  p2 = (unsigned short)(__float_as_uint(l) >> 16);
}

__device__ __forceinline__ bf16x8 pack8(const unsigned short* v) {
  s16x8 s;
  for (int i = 0; i < 8; ++i) s[i] = (short)v[i];
  return __builtin_bit_cast(bf16x8, s);
}

// A [16][64] row-major, B [64][16] row-major, out [3][16][16]
__global__ void gemm3(const float* A, const float* B, float* out) {
  const int l = threadIdx.x, li = l & 15, lg = l >> 4;
  // (a) f32 chain: MFMA k-step s covers k = 4 s + lg
  f32x4 acc = {0.f, 0.f, 0.f, 0.f};
  for (int s = 0; s < 16; ++s)
    acc = __builtin_amdgcn_mfma_f32_16x16x4f32(A[li * 64 + 4 * s + lg], B[(4 * s + lg) * 16 + li], acc, 0, 0, 0);
  for (int i = 0; i < 4; ++i) out[0 * 256 + (4 * lg + i) * 16 + li] = acc[i];
  // (b)/(c): per 32-wide K block, lane supplies k = 8 lg .. 8 lg + 7
  f32x4 a9 = {0.f, 0.f, 0.f, 0.f}, a6 = {0.f, 0.f, 0.f, 0.f};
  for (int kb = 0; kb < 2; ++kb) {
    unsigned short ap[3][8], bp[3][8];
    for (int j = 0; j < 8; ++j) {
      const int k = kb * 32 + 8 * lg + j;
      split3(A[li * 64 + k], ap[0][j], ap[1][j], ap[2][j]);
      split3(B[k * 16 + li], bp[0][j], bp[1][j], bp[2][j]);
    }
    bf16x8 av[3], bv[3];
    for (int p = 0; p < 3; ++p) av[p] = pack8(ap[p]), bv[p] = pack8(bp[p]);
    // smallest terms first
    const int order9[9][2] = {{2, 2}, {1, 2}, {2, 1}, {0, 2}, {1, 1}, {2, 0}, {0, 1}, {1, 0}, {0, 0}};
    for (int t = 0; t < 9; ++t) a9 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(av[order9[t][0]], bv[order9[t][1]], a9, 0, 0, 0);
    const int order6[6][2] = {{0, 2}, {1, 1}, {2, 0}, {0, 1}, {1, 0}, {0, 0}};
    for (int t = 0; t < 6; ++t) a6 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(av[order6[t][0]], bv[order6[t][1]], a6, 0, 0, 0);
  }
  for (int i = 0; i < 4; ++i) {
    out[1 * 256 + (4 * lg + i) * 16 + li] = a9[i];
    out[2 * 256 + (4 * lg + i) * 16 + li] = a6[i];
  }
}

template <int NV, int MODE>
__global__ void __launch_bounds__(512) issue(float* out, int iters, float s) {
  f32x4 acc[8];
  for (int i = 0; i < 8; ++i) acc[i] = f32x4{0.f, 0.f, 0.f, 0.f};
  s16x8 sa, sb;
  for (int i = 0; i < 8; ++i) sa[i] = (short)(threadIdx.x + i), sb[i] = (short)(threadIdx.x * 3 + i);
  const bf16x8 a = __builtin_bit_cast(bf16x8, sa), b = __builtin_bit_cast(bf16x8, sb);
  float v[16];
  for (int i = 0; i < 16; ++i) v[i] = i * 0.5f + threadIdx.x;
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int m = 0; m < 8; ++m) {
      if (MODE != 2) acc[m] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, acc[m], 0, 0, 0);
#pragma unroll
      for (int k = 0; k < NV / 8; ++k) {
        const int j = (m * (NV / 8) + k) & 15;
        // the split's instruction mix: and, sub, perm
        if (k % 3 == 0) v[j] = __uint_as_float(__float_as_uint(v[j]) & 0xffff0000u) + 0.f;
        else if (k % 3 == 1) v[j] = v[j] - s;
        else v[j] = __uint_as_float(__builtin_amdgcn_perm(__float_as_uint(v[j]), __float_as_uint(v[(j + 1) & 15]), 0x07060302u));
      }
    }
    asm volatile("" ::: "memory");
  }
  float t = 0.f;
  for (int i = 0; i < 8; ++i) t += acc[i].x + acc[i].y;
  for (int i = 0; i < 16; ++i) t += v[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = t;
}

template <int NV, int MODE>
void run_issue(float* d, int threads, const char* name) {
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  const int iters = 20000;
  hipLaunchKernelGGL((issue<NV, MODE>), dim3(256), dim3(threads), 0, 0, d, 100, 0.999f);
  hipEventRecord(e0);
  hipLaunchKernelGGL((issue<NV, MODE>), dim3(256), dim3(threads), 0, 0, d, iters, 0.999f);
  hipEventRecord(e1);
  hipEventSynchronize(e1);
  float ms;
  hipEventElapsedTime(&ms, e0, e1);
  printf("%-26s waves/SIMD %d NV %3d: %8.2f ns per iteration (8 bf16 MFMA slots)\n", name, threads / 256, NV,
         ms * 1e6 / iters);
}

static float frand(unsigned& s) {
  s = s * 1664525u + 1013904223u;
  return ((s >> 8) * (1.0f / 16777216.0f)) * 2.f - 1.f;
}

int main() {
  // accuracy
  float *dA, *dB, *dO;
  hipMalloc(&dA, 16 * 64 * 4);
  hipMalloc(&dB, 64 * 16 * 4);
  hipMalloc(&dO, 3 * 256 * 4);
  std::vector<float> A(16 * 64), B(64 * 16), O(3 * 256);
  double worst[3] = {0, 0, 0}, sum_err[3] = {0, 0, 0};
  unsigned seed = 12345;
  const int trials = 200;
  for (int tr = 0; tr < trials; ++tr) {
    const float sa = std::ldexp(1.f, (tr % 7) - 3), sb = std::ldexp(1.f, (tr % 5) - 6);
    for (auto& x : A) x = frand(seed) * sa * (tr % 3 == 0 ? std::fabs(frand(seed)) * 8.f : 1.f);
    for (auto& x : B) x = frand(seed) * sb;
    hipMemcpy(dA, A.data(), A.size() * 4, hipMemcpyHostToDevice);
    hipMemcpy(dB, B.data(), B.size() * 4, hipMemcpyHostToDevice);
    hipLaunchKernelGGL(gemm3, dim3(1), dim3(64), 0, 0, dA, dB, dO);
    hipMemcpy(O.data(), dO, O.size() * 4, hipMemcpyDeviceToHost);
    for (int i = 0; i < 16; ++i)
      for (int j = 0; j < 16; ++j) {
        double ex = 0, mag = 0;
        for (int k = 0; k < 64; ++k) {
          ex += (double)A[i * 64 + k] * B[k * 16 + j];
          mag += std::fabs((double)A[i * 64 + k] * B[k * 16 + j]);
        }
        for (int f = 0; f < 3; ++f) {
          const double e = std::fabs(O[f * 256 + i * 16 + j] - ex) / mag;
          if (e > worst[f]) worst[f] = e;
          sum_err[f] += e;
        }
      }
  }
  const char* fn[3] = {"f32 mfma 16x16x4", "bf16x9 split", "bf16x6 split"};
  for (int f = 0; f < 3; ++f)
    printf("%-18s max err %.3e  mean err %.3e  (x sum|a||b|; f32 eps 5.96e-08)\n", fn[f], worst[f],
           sum_err[f] / (trials * 256.0));
  // issue
  float* d;
  hipMalloc(&d, 256 * 512 * 4);
  run_issue<0, 0>(d, 256, "bf16 mfma only");
  run_issue<8, 0>(d, 256, "bf16 mfma + split valu");
  run_issue<16, 0>(d, 256, "bf16 mfma + split valu");
  run_issue<32, 0>(d, 256, "bf16 mfma + split valu");
  run_issue<64, 0>(d, 256, "bf16 mfma + split valu");
  run_issue<32, 2>(d, 256, "split valu only");
  run_issue<64, 2>(d, 256, "split valu only");
  run_issue<0, 0>(d, 512, "bf16 mfma only");
  run_issue<32, 0>(d, 512, "bf16 mfma + split valu");
  run_issue<64, 0>(d, 512, "bf16 mfma + split valu");
  hipFree(d);
  return 0;
}
