// Diagnostic build (not part of libtic): cycle breakdown of conv3x3_persist_kernel per
// workgroup — K loop vs next-tile staging + epilogue vs barrier — on a synthetic
// encode_1-shaped layer (stride 2, 32 -> 32, 128x128 -> 64x64, batch 32).
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -I tf_image_compression_amd/csrc \
//         tools/persist_probe.hip -o gpurun_out/persist_probe && gpurun_out/persist_probe
#define TIC_PERSIST_PROBE 1
#include <cstdio>
#include <vector>
#include <algorithm>
#include "conv_launch.h"

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP %s @%d\n", hipGetErrorString(e_), __LINE__); return 1; } } while (0)

int main(int argc, char** argv) {
  using namespace tic;
  const int n = argc > 1 ? atoi(argv[1]) : 32;
  const int H = 128, W = 128, CIN = 32, COUT = 32, Ho = 64, Wo = 64;
  const size_t nin = (size_t)n * H * W * CIN, nout = (size_t)n * Ho * Wo * COUT;
  std::vector<float> hin(nin), hw(9 * CIN * COUT), hb(COUT);
  for (size_t i = 0; i < nin; ++i) hin[i] = (float)((i * 2654435761u) % 1000) / 1000.f;
  for (size_t i = 0; i < hw.size(); ++i) hw[i] = (float)((i * 40503u) % 997) / 9970.f - 0.05f;
  for (int i = 0; i < COUT; ++i) hb[i] = 0.01f * i;
  float *din, *dw, *db, *dout;
  CK(hipMalloc(&din, nin * 4));
  CK(hipMalloc(&dw, hw.size() * 4));
  CK(hipMalloc(&db, COUT * 4));
  CK(hipMalloc(&dout, nout * 4));
  CK(hipMemcpy(din, hin.data(), nin * 4, hipMemcpyHostToDevice));
  CK(hipMemcpy(dw, hw.data(), hw.size() * 4, hipMemcpyHostToDevice));
  CK(hipMemcpy(db, hb.data(), COUT * 4, hipMemcpyHostToDevice));
  hipDeviceProp_t prop;
  CK(hipGetDeviceProperties(&prop, 0));
  const int ncu = prop.multiProcessorCount;
  unsigned long long* dprobe;
  CK(hipMalloc(&dprobe, (size_t)ncu * 4 * 12 * 8));
  CK(hipMemcpyToSymbol(HIP_SYMBOL(g_persist_probe), &dprobe, sizeof(dprobe)));
  ConvArgs a{};
  a.in = din; a.wp = dw; a.bias = db; a.out = dout;
  a.H = H; a.W = W; a.Ho = Ho; a.Wo = Wo; a.pad_y = a.pad_x = 0; a.num_cus = ncu;
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
  for (int i = 0; i < 5; ++i) launch_conv_persist<MODE_S2, 32, 32, 4, 4, ACT_RELU>(a, n, 0);
  CK(hipEventRecord(e0, 0));
  const int reps = 20;
  for (int i = 0; i < reps; ++i) launch_conv_persist<MODE_S2, 32, 32, 4, 4, ACT_RELU>(a, n, 0);
  CK(hipEventRecord(e1, 0));
  CK(hipEventSynchronize(e1));
  float ms; CK(hipEventElapsedTime(&ms, e0, e1));
  // one more launch alone for the stamps
  long long r0 = 0;
  launch_conv_persist<MODE_S2, 32, 32, 4, 4, ACT_RELU>(a, n, 0);
  CK(hipDeviceSynchronize());
  std::vector<unsigned long long> hp((size_t)ncu * 4 * 12);
  CK(hipMemcpy(hp.data(), dprobe, hp.size() * 8, hipMemcpyDeviceToHost));
  const int ntiles = 4 * 16 * n;
  double tot = 0, kl = 0, ep = 0, ba = 0, rt = 0, cm = 0, is = 0, pro = 0; int cnt = 0;
  unsigned long long smin = ~0ull, smax = 0, emax = 0;
  for (int b = 0; b < std::min(ncu, ntiles); ++b) for (int w = 0; w < 4; ++w) {
    const unsigned long long* q = &hp[(b * 4 + w) * 12];
    tot += q[0]; kl += q[1]; ep += q[2]; ba += q[3]; rt += q[4]; cm += q[5]; is += q[6]; pro += q[7]; ++cnt;
    smin = std::min(smin, q[8]); smax = std::max(smax, q[8]); emax = std::max(emax, q[9]);
  }
  const double tiles_per_wg = (double)ntiles / std::min(ncu, ntiles);
  printf("n=%d tiles=%d grid=%d  kernel %.2f us (events, back-to-back)\n", n, ntiles, std::min(ncu, ntiles), 1e3 * ms / reps);
  const double tw = cnt * tiles_per_wg;
  printf("per wave, cycles: prologue %.0f, loop total %.0f | per tile: K loop incl. staging %.0f (MFMA ideal %d) "
         "epilogue %.0f barrier %.0f\n", pro / cnt, tot / cnt, kl / tw, 18 * 8 * 32, ep / tw, ba / tw);
  printf("dispatch skew %.2f us, first start -> last end %.2f us\n", (smax - smin) / 100.0, (emax - smin) / 100.0);
  printf("clock %.2f GHz (memtime / memrealtime x 100 MHz); loop %.2f us per workgroup\n", tot / rt * 0.1,
         rt / cnt / 100.0);
  (void)r0;
  return 0;
}
