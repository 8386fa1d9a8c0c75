// First layer (u8/f32 RGB -> normalise -> stride-2 conv) and last layer
// (transpose conv -> denormalise -> clip -> round -> u8) of every codec, with their
// tiling variants (selected per layer by tic_autotune).
#include <algorithm>

#include "conv3x3.h"
#include "convT_rgb_valu.h"
#include "dec10.h"

namespace tic {

int rgb_in_variants() { return 3; }  // TH = 4, 8, 16 output rows per workgroup

template <int COUT, int TH>
static bool rgb_in_th(bool u8_input, const RgbInArgs& a, int n, hipStream_t s) {
  dim3 grid((a.Wo + 15) / 16, (a.Ho + TH - 1) / TH, n);
  if (u8_input)
    hipLaunchKernelGGL((conv_rgb_s2_kernel<COUT, TH, true>), grid, dim3(256), 0, s, a);
  else
    hipLaunchKernelGGL((conv_rgb_s2_kernel<COUT, TH, false>), grid, dim3(256), 0, s, a);
  return true;
}

template <int COUT>
static bool rgb_in_c(bool u8_input, const RgbInArgs& a, int n, hipStream_t s, int variant) {
  switch (variant) {
    case 0: return rgb_in_th<COUT, 4>(u8_input, a, n, s);
    case 1: return rgb_in_th<COUT, 8>(u8_input, a, n, s);
    case 2: return rgb_in_th<COUT, 16>(u8_input, a, n, s);
  }
  return false;
}

bool launch_rgb_in(int cout, bool u8_input, const RgbInArgs& a, int n, hipStream_t s, int variant) {
  if (cout == 64) return rgb_in_c<64>(u8_input, a, n, s, variant);  // base_model/ch_128 encode_1
  if (cout == 32) return rgb_in_c<32>(u8_input, a, n, s, variant);
  if (cout == 16) return rgb_in_c<16>(u8_input, a, n, s, variant);
  return false;
}

// Last layer: variants 0-2 dense sub-pixel MFMA form (TH 4/8/16), 3-5 scatter MFMA form
// (TH 4/8/16), 6-11 VALU form (TW 64/32/16; 9-11 persistent, software-pipelined).  The form is a fixed policy (default VALU;
// TIC_RGB_OUT_FORM=dense|scatter for experiments); tuning picks a tiling within the form,
// so it never changes results.
// TH1 = 2, 4 (padded LDS form), 2, 4, 8 (compact form) — all bit-identical.  (Round 3 measured
// a persistent software-pipelined form and a producer / consumer form and did not keep them:
// 59 and 75 against 50 us per 32 patches)
int enc01_variants() { return 5; }

template <int C0, int C1, int TH1, bool CMP>
static bool enc01_th(bool u8_input, const Enc01Args& a, int n, hipStream_t s) {
  dim3 grid((a.W2 + 15) / 16, (a.H2 + TH1 - 1) / TH1, n);
  if (u8_input)
    hipLaunchKernelGGL((enc01_kernel<C0, C1, TH1, true, CMP>), grid, dim3(256), 0, s, a);
  else
    hipLaunchKernelGGL((enc01_kernel<C0, C1, TH1, false, CMP>), grid, dim3(256), 0, s, a);
  return true;
}

template <int C0, int C1>
static bool enc01_c(bool u8_input, const Enc01Args& a, int n, hipStream_t s, int variant) {
  switch (variant) {
    case 0: return enc01_th<C0, C1, 2, false>(u8_input, a, n, s);
    case 1: return enc01_th<C0, C1, 4, false>(u8_input, a, n, s);
    case 2: return enc01_th<C0, C1, 2, true>(u8_input, a, n, s);
    case 3: return enc01_th<C0, C1, 4, true>(u8_input, a, n, s);
    case 4: return enc01_th<C0, C1, 8, true>(u8_input, a, n, s);
  }
  return false;
}

bool launch_enc01(int c0, int c1, bool u8_input, const Enc01Args& a, int n, hipStream_t s, int variant) {
  if (c0 == 32 && c1 == 32) return enc01_c<32, 32>(u8_input, a, n, s, variant);
  if (c0 == 16 && c1 == 32) return enc01_c<16, 32>(u8_input, a, n, s, variant);
  if (c0 == 32 && c1 == 64) return enc01_c<32, 64>(u8_input, a, n, s, variant);
  return false;
}

int rgb_out_variants() { return 12; }

template <int CIN, int TH, bool SCATTER>
static bool rgb_out_th(const RgbOutArgs& a, int n, hipStream_t s) {
  dim3 grid((a.W + 15) / 16, (a.H + TH - 1) / TH, n);
  if (SCATTER)
    hipLaunchKernelGGL((convT_rgb_scatter_kernel<CIN, TH>), grid, dim3(256), 0, s, a);
  else
    hipLaunchKernelGGL((convT_rgb_kernel<CIN, TH>), grid, dim3(256), 0, s, a);
  return true;
}

template <int CIN, int TW>
static bool rgb_out_valu(const RgbOutArgs& a, int n, hipStream_t s) {
  dim3 grid((a.W + TW - 1) / TW, (a.H + 256 / TW - 1) / (256 / TW), n);
  hipLaunchKernelGGL((convT_rgb_valu_kernel<CIN, TW>), grid, dim3(256), 0, s, a);
  return true;
}

template <int CIN, int TW>
static bool rgb_out_valu_persist(const RgbOutArgs& a, int n, hipStream_t s) {
  const int ntx = (a.W + TW - 1) / TW, nty = (a.H + 256 / TW - 1) / (256 / TW);
  const int ntiles = ntx * nty * n;
  int grid = std::min(ntiles, 2 * std::max(1, a.num_cus));
  if (a.grid_cap > 0) grid = std::min(grid, a.grid_cap);
  hipLaunchKernelGGL((convT_rgb_valu_persist_kernel<CIN, TW>), dim3(grid), dim3(256), 0, s, a, ntx, nty, ntiles);
  return true;
}

template <int CIN>
static bool rgb_out_c(const RgbOutArgs& a, int n, hipStream_t s, int variant) {
  switch (variant) {
    case 0: return rgb_out_th<CIN, 4, false>(a, n, s);
    case 1: return rgb_out_th<CIN, 8, false>(a, n, s);
    case 2: return rgb_out_th<CIN, 16, false>(a, n, s);
    case 3: return rgb_out_th<CIN, 4, true>(a, n, s);
    case 4: return rgb_out_th<CIN, 8, true>(a, n, s);
    case 5: return rgb_out_th<CIN, 16, true>(a, n, s);
    case 6: return rgb_out_valu<CIN, 64>(a, n, s);
    case 7: return rgb_out_valu<CIN, 32>(a, n, s);
    case 8: return rgb_out_valu<CIN, 16>(a, n, s);
    case 9: return rgb_out_valu_persist<CIN, 64>(a, n, s);
    case 10: return rgb_out_valu_persist<CIN, 32>(a, n, s);
    case 11: return rgb_out_valu_persist<CIN, 16>(a, n, s);
  }
  return false;
}

bool launch_rgb_out(int cin, const RgbOutArgs& a, int n, hipStream_t s, int variant) {
  if (cin == 64) return rgb_out_c<64>(a, n, s, variant);  // base_model/ch_128 decode_1
  if (cin == 32) return rgb_out_c<32>(a, n, s, variant);
  if (cin == 16) return rgb_out_c<16>(a, n, s, variant);
  return false;
}

// decode_0's weights always by scalar loads here: staging them in LDS (WSH) measured 25-35 %
// slower in every form (profiles/dec10_probe_r02*.log)
template <int C1, int C0, int TA, bool CMP>
static void dec10_t(const Dec10Args& a, int n, hipStream_t s, int v) {
  const dim3 grid((a.W + 15) / 16, (a.H + TA - 1) / TA, n), block(64 * TA);
  switch (v & 3) {
    case 0: hipLaunchKernelGGL((dec10_kernel<C1, C0, false, 2, 0, TA, CMP, true>), grid, block, 0, s, a); break;
    case 1: hipLaunchKernelGGL((dec10_kernel<C1, C0, false, 2, 0, TA, CMP, false>), grid, block, 0, s, a); break;
    case 2: hipLaunchKernelGGL((dec10_kernel<C1, C0, false, 5, 0, TA, CMP, true>), grid, block, 0, s, a); break;
    default: hipLaunchKernelGGL((dec10_kernel<C1, C0, false, 5, 0, TA, CMP, false>), grid, block, 0, s, a); break;
  }
}

template <int C1, int C0>
static bool dec10_c(const Dec10Args& a, int n, hipStream_t s, int variant) {
  const dim3 grid((a.W + 15) / 16, (a.H + 3) / 4, n);
  if (variant < 16) {
    switch (variant >> 2) {
      case 0: dec10_t<C1, C0, 4, false>(a, n, s, variant); break;
      case 1: dec10_t<C1, C0, 8, false>(a, n, s, variant); break;
      case 2: dec10_t<C1, C0, 4, true>(a, n, s, variant); break;
      default: dec10_t<C1, C0, 8, true>(a, n, s, variant); break;
    }
    return true;
  }
  // timing probes of variant 8 (TIC_DEC10_VARIANT only; results invalid): without decode_1's
  // MFMAs / decode_0 / the input loads / decode_1's weight loads (dec10.h PROBE)
  switch (variant) {
    case 100: hipLaunchKernelGGL((dec10_kernel<C1, C0, false, 2, 1, 4, true>), grid, dim3(256), 0, s, a); break;
    case 101: hipLaunchKernelGGL((dec10_kernel<C1, C0, false, 2, 2, 4, true>), grid, dim3(256), 0, s, a); break;
    case 102: hipLaunchKernelGGL((dec10_kernel<C1, C0, false, 2, 4, 4, true>), grid, dim3(256), 0, s, a); break;
    case 103: hipLaunchKernelGGL((dec10_kernel<C1, C0, false, 2, 8, 4, true>), grid, dim3(256), 0, s, a); break;
    case 104: hipLaunchKernelGGL((dec10_kernel<C1, C0, false, 2, 3, 4, true>), grid, dim3(256), 0, s, a); break;
    case 105: hipLaunchKernelGGL((dec10_kernel<C1, C0, false, 2, 3 | 32, 4, true>), grid, dim3(256), 0, s, a); break;
    case 106: hipLaunchKernelGGL((dec10_kernel<C1, C0, false, 2, 3 | 32 | 16, 4, true>), grid, dim3(256), 0, s, a); break;
    case 107: hipLaunchKernelGGL((dec10_kernel<C1, C0, false, 2, 3 | 32 | 16 | 4, 4, true>), grid, dim3(256), 0, s, a); break;
    default: return false;
  }
  return true;
}

// variants 0-15, bits: 0 decode_0 by packed / plain fmas; 1 decode_1 weight prefetch 2 / 5
// steps ahead; 2 tiles of 4 / 8 decode_1 input rows; 3 the padded / compact LDS form.  All
// bit-identical.
int dec10_variants() { return 16; }

bool launch_dec10(int c1, int c0, const Dec10Args& a, int n, hipStream_t s, int variant) {
  if (variant < 0 || (variant >= dec10_variants() && (variant < 100 || variant > 107))) return false;
  if (c1 == 32 && c0 == 32) return dec10_c<32, 32>(a, n, s, variant);
  if (c1 == 32 && c0 == 16) return dec10_c<32, 16>(a, n, s, variant);
  if (c1 == 64 && c0 == 32) return dec10_c<64, 32>(a, n, s, variant);
  return false;
}

}  // namespace tic
