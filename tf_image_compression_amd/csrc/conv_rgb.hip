// First layer (u8/f32 RGB -> normalise -> stride-2 conv) and last layer
// (transpose conv -> denormalise -> clip -> round -> u8) of every codec.
#include "conv3x3.h"

namespace tic {

bool launch_rgb_in(int cout, bool u8_input, const RgbInArgs& a, int n, hipStream_t s) {
  constexpr int TH = 4;
  dim3 grid((a.Wo + 15) / 16, (a.Ho + TH - 1) / TH, n);
  if (cout == 32 && u8_input)
    hipLaunchKernelGGL((conv_rgb_s2_kernel<32, TH, true>), grid, dim3(256), 0, s, a);
  else if (cout == 16 && u8_input)
    hipLaunchKernelGGL((conv_rgb_s2_kernel<16, TH, true>), grid, dim3(256), 0, s, a);
  else if (cout == 32 && !u8_input)
    hipLaunchKernelGGL((conv_rgb_s2_kernel<32, TH, false>), grid, dim3(256), 0, s, a);
  else
    return false;
  return true;
}

bool launch_rgb_out(int cin, const RgbOutArgs& a, int n, hipStream_t s) {
  constexpr int TH = 4;
  dim3 grid((a.W + 15) / 16, (a.H + TH - 1) / TH, n);
  if (cin == 32)
    hipLaunchKernelGGL((convT_rgb_kernel<32, TH>), grid, dim3(256), 0, s, a);
  else if (cin == 16)
    hipLaunchKernelGGL((convT_rgb_kernel<16, TH>), grid, dim3(256), 0, s, a);
  else
    return false;
  return true;
}

}  // namespace tic
