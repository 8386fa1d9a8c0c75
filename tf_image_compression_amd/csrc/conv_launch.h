// conv_launch.h — grid computation + registry helpers for conv3x3_kernel instantiations.
#pragma once
#include "conv3x3.h"

namespace tic {

template <int MODE, int CIN, int COUT, int TH, int WR, int NSPLIT, int WSRC, int ACT, bool RES, int IN, int OUT>
static void launch_conv(const ConvArgs& a, int n, hipStream_t s) {
  const int hg = MODE == MODE_T2 ? a.H : a.Ho;
  const int wg = MODE == MODE_T2 ? a.W : a.Wo;
  dim3 grid(((wg + 15) / 16) * NSPLIT, (hg + TH - 1) / TH, n);
  hipLaunchKernelGGL((conv3x3_kernel<MODE, CIN, COUT, TH, WR, NSPLIT, WSRC, ACT, RES, IN, OUT>), grid, dim3(256), 0, s, a);
}

}  // namespace tic

#define TIC_CONVW(MODE, CIN, COUT, TH, WR, NSPLIT, WSRC, ACT, RES, IN, OUT)               \
  { MODE, CIN, COUT, ACT, RES, IN, OUT, TH, WR, NSPLIT, WSRC,                                 \
    &tic::launch_conv<MODE, CIN, COUT, TH, WR, NSPLIT, WSRC, ACT, RES, IN, OUT> }
// L2 (PF 2) and LDS-ring weight sources for one tiling
#define TIC_CONV(MODE, CIN, COUT, TH, WR, NSPLIT, ACT, RES, IN, OUT)            \
  TIC_CONVW(MODE, CIN, COUT, TH, WR, NSPLIT, 0, ACT, RES, IN, OUT),              \
      TIC_CONVW(MODE, CIN, COUT, TH, WR, NSPLIT, 1, ACT, RES, IN, OUT)
// the two L2 weight sources (PF 2 / deep prefetch) — 128-wide layers, whose per-tap slab
// (64 KB at 128 x 128) does not fit a 2-slot LDS ring beside the input tile
#define TIC_CONVL2(MODE, CIN, COUT, TH, WR, NSPLIT, ACT, RES, IN, OUT)          \
  TIC_CONVW(MODE, CIN, COUT, TH, WR, NSPLIT, 0, ACT, RES, IN, OUT),              \
      TIC_CONVW(MODE, CIN, COUT, TH, WR, NSPLIT, 2, ACT, RES, IN, OUT)
// all three weight sources (small grids: + L2 with deep prefetch)
#define TIC_CONV3(MODE, CIN, COUT, TH, WR, NSPLIT, ACT, RES, IN, OUT)           \
  TIC_CONV(MODE, CIN, COUT, TH, WR, NSPLIT, ACT, RES, IN, OUT),                  \
      TIC_CONVW(MODE, CIN, COUT, TH, WR, NSPLIT, 2, ACT, RES, IN, OUT)
