// conv_launch.h — grid computation + registry helpers for conv3x3_kernel instantiations.
#pragma once
#include "conv3x3.h"
#include "conv3x3_persist.h"

namespace tic {

template <int MODE, int CIN, int COUT, int TH, int WR, int NSPLIT, int WSRC, int ACT, bool RES, int IN, int OUT>
static void launch_conv(const ConvArgs& a, int n, hipStream_t s) {
  const int hg = MODE == MODE_T2 ? a.H : a.Ho;
  const int wg = MODE == MODE_T2 ? a.W : a.Wo;
  dim3 grid(((wg + 15) / 16) * NSPLIT, (hg + TH - 1) / TH, n);
  hipLaunchKernelGGL((conv3x3_kernel<MODE, CIN, COUT, TH, WR, NSPLIT, WSRC, ACT, RES, IN, OUT>), grid, dim3(256), 0, s, a);
}

template <int MODE, int CIN, int COUT, int TH, int WR, int ACT>
static void launch_conv_persist(const ConvArgs& a, int n, hipStream_t s) {
  const int hg = MODE == MODE_T2 ? a.H : a.Ho;
  const int wg = MODE == MODE_T2 ? a.W : a.Wo;
  const int ntx = (wg + 15) / 16, nty = (hg + TH - 1) / TH;
  const int ntiles = ntx * nty * n;
  constexpr int lds = PersistGeom<MODE, CIN, COUT, TH, WR, ACT>::LDS_BYTES;
  int per_cu = (160 * 1024) / lds;
  per_cu = per_cu < 1 ? 1 : (per_cu > 4 ? 4 : per_cu);
  int grid = (a.num_cus > 0 ? a.num_cus : 256) * per_cu;
  if (a.grid_cap > 0 && grid > a.grid_cap) grid = a.grid_cap;
  if (grid > ntiles) grid = ntiles;
  hipLaunchKernelGGL((conv3x3_persist_kernel<MODE, CIN, COUT, TH, WR, ACT>), dim3(grid), dim3(256), 0, s, a, ntx,
                     nty, ntiles);
}

}  // namespace tic

#define TIC_CONVW(MODE, CIN, COUT, TH, WR, NSPLIT, WSRC, ACT, RES, IN, OUT)               \
  { MODE, CIN, COUT, ACT, RES, IN, OUT, TH, WR, NSPLIT, WSRC,                                 \
    &tic::launch_conv<MODE, CIN, COUT, TH, WR, NSPLIT, WSRC, ACT, RES, IN, OUT> }
// persistent, weights resident in LDS (f32 in/out, no residual)
#define TIC_PERSIST(MODE, CIN, COUT, TH, WR, ACT)                                       \
  { MODE, CIN, COUT, ACT, false, IN_F32, OUT_F32, TH, WR, 1, 3,                        \
    &tic::launch_conv_persist<MODE, CIN, COUT, TH, WR, ACT> }
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
