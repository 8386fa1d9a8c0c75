// conv_launch.h — grid computation + registry helpers for conv3x3_kernel instantiations.
#pragma once
#include "conv3x3.h"

namespace tic {

template <int MODE, int CIN, int COUT, int TH, int WR, int NSPLIT, bool WLDS, int ACT, bool RES, int IN, int OUT>
static void launch_conv(const ConvArgs& a, int n, hipStream_t s) {
  const int hg = MODE == MODE_T2 ? a.H : a.Ho;
  const int wg = MODE == MODE_T2 ? a.W : a.Wo;
  dim3 grid(((wg + 15) / 16) * NSPLIT, (hg + TH - 1) / TH, n);
  hipLaunchKernelGGL((conv3x3_kernel<MODE, CIN, COUT, TH, WR, NSPLIT, WLDS, ACT, RES, IN, OUT>), grid, dim3(256), 0, s, a);
}

template <int MODE, int CIN, int COUT, int TH, int WR, int NSPLIT, int ACT, bool RES, int IN, int OUT>
static void launch_conv_pipe(const ConvArgs& a, int n, hipStream_t s) {
  const int hg = MODE == MODE_T2 ? a.H : a.Ho;
  const int wg = MODE == MODE_T2 ? a.W : a.Wo;
  const int ntx = (wg + 15) / 16, nty = (hg + TH - 1) / TH;
  const int ntiles = ntx * nty * n * NSPLIT;
  constexpr int PS = CIN + 8;
  constexpr int lds_bytes = 2 * TileGeom<MODE, TH>::LR * TileGeom<MODE, TH>::LC * PS * 4;
  int per_cu = (160 * 1024) / lds_bytes;
  per_cu = per_cu < 1 ? 1 : (per_cu > 4 ? 4 : per_cu);
  int grid = (a.num_cus > 0 ? a.num_cus : 256) * per_cu;
  if (grid > ntiles) grid = ntiles;
  hipLaunchKernelGGL((conv3x3_pipe_kernel<MODE, CIN, COUT, TH, WR, NSPLIT, ACT, RES, IN, OUT>), dim3(grid), dim3(320),
                     0, s, a, ntx, nty, ntiles);
}

}  // namespace tic

#define TIC_PIPE(MODE, CIN, COUT, TH, WR, NSPLIT, ACT, RES, IN, OUT) \
  { MODE, CIN, COUT, ACT, RES, IN, OUT, TH, NSPLIT, 2,               \
    &tic::launch_conv_pipe<MODE, CIN, COUT, TH, WR, NSPLIT, ACT, RES, IN, OUT> }

#define TIC_CONVW(MODE, CIN, COUT, TH, WR, NSPLIT, WLDS, ACT, RES, IN, OUT)               \
  { MODE, CIN, COUT, ACT, RES, IN, OUT, TH, NSPLIT, WLDS,                                 \
    &tic::launch_conv<MODE, CIN, COUT, TH, WR, NSPLIT, WLDS, ACT, RES, IN, OUT> }
// both weight sources for one tiling
#define TIC_CONV(MODE, CIN, COUT, TH, WR, NSPLIT, ACT, RES, IN, OUT)            \
  TIC_CONVW(MODE, CIN, COUT, TH, WR, NSPLIT, false, ACT, RES, IN, OUT),          \
      TIC_CONVW(MODE, CIN, COUT, TH, WR, NSPLIT, true, ACT, RES, IN, OUT)
