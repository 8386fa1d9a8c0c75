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

}  // namespace tic

#define TIC_CONVW(MODE, CIN, COUT, TH, WR, NSPLIT, WLDS, ACT, RES, IN, OUT)               \
  { MODE, CIN, COUT, ACT, RES, IN, OUT, TH, WR, NSPLIT, WLDS,                                 \
    &tic::launch_conv<MODE, CIN, COUT, TH, WR, NSPLIT, WLDS, ACT, RES, IN, OUT> }
// both weight sources for one tiling
#define TIC_CONV(MODE, CIN, COUT, TH, WR, NSPLIT, ACT, RES, IN, OUT)            \
  TIC_CONVW(MODE, CIN, COUT, TH, WR, NSPLIT, false, ACT, RES, IN, OUT),          \
      TIC_CONVW(MODE, CIN, COUT, TH, WR, NSPLIT, true, ACT, RES, IN, OUT)
