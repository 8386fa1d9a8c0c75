// Micro-probe: do f32 MFMA (v_mfma_f32_16x16x4_f32) and f32 VALU (v_fma_f32 / v_pk_fma_f32)
// overlap on one SIMD, or add up?  One wave per SIMD (256-thread workgroups, one per CU);
// per loop iteration 8 independent MFMAs and NV independent VALU fmas (scalar or packed),
// interleaved in program order.  Prints ns per iteration for each NV.
//   hipcc --offload-arch=gfx950 -O3 tools/probes/mfma_valu.hip -o /tmp/mfma_valu && /tmp/mfma_valu
#include <hip/hip_runtime.h>
#include <cstdio>

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x2 __attribute__((ext_vector_type(2)));

template <int NV, bool PK, bool WITH_MFMA>
__global__ void __launch_bounds__(256) probe(float* out, int iters, float s) {
  f32x4 acc[8];
  for (int i = 0; i < 8; ++i) acc[i] = f32x4{0.f, 0.f, 0.f, 0.f};
  float a = threadIdx.x * 1e-3f, b = s;
  float v[16];
  f32x2 vp[16];
  for (int i = 0; i < 16; ++i) {
    v[i] = i * 0.5f + threadIdx.x;
    vp[i] = f32x2{v[i], v[i] + 1.f};
  }
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int m = 0; m < 8; ++m) {
      if (WITH_MFMA) acc[m] = __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, acc[m], 0, 0, 0);
#pragma unroll
      for (int k = 0; k < NV / 8; ++k) {
        const int j = (m * (NV / 8) + k) & 15;
        if (PK) vp[j] = __builtin_elementwise_fma(vp[j], f32x2{s, s}, f32x2{1e-7f, 1e-7f});
        else v[j] = __builtin_fmaf(v[j], s, 1e-7f);
      }
    }
    asm volatile("" ::: "memory");
  }
  float t = 0.f;
  for (int i = 0; i < 8; ++i) t += acc[i].x + acc[i].y;
  for (int i = 0; i < 16; ++i) t += v[i] + vp[i].x + vp[i].y;
  out[blockIdx.x * 256 + threadIdx.x] = t;
}

template <int NV, bool PK, bool M>
void run(float* d, const char* name) {
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  const int iters = 20000;
  hipLaunchKernelGGL((probe<NV, PK, M>), dim3(256), dim3(256), 0, 0, d, 100, 0.999f);
  hipEventRecord(e0);
  hipLaunchKernelGGL((probe<NV, PK, M>), dim3(256), dim3(256), 0, 0, d, iters, 0.999f);
  hipEventRecord(e1);
  hipEventSynchronize(e1);
  float ms;
  hipEventElapsedTime(&ms, e0, e1);
  printf("%-28s NV %3d: %8.2f ns per iteration (8 MFMA slots)\n", name, NV, ms * 1e6 / iters);
}

int main() {
  float* d;
  hipMalloc(&d, 256 * 256 * 4);
  run<0, false, true>(d, "mfma only");
  run<8, false, true>(d, "mfma + scalar fma");
  run<16, false, true>(d, "mfma + scalar fma");
  run<32, false, true>(d, "mfma + scalar fma");
  run<64, false, true>(d, "mfma + scalar fma");
  run<8, true, true>(d, "mfma + pk fma");
  run<16, true, true>(d, "mfma + pk fma");
  run<32, true, true>(d, "mfma + pk fma");
  run<32, false, false>(d, "scalar fma only");
  run<64, false, false>(d, "scalar fma only");
  run<32, true, false>(d, "pk fma only");
  hipFree(d);
  return 0;
}
