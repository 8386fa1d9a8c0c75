// Chains of stride-1 64->64 layers in one launch (wino_chain.h): the codecs' residual
// stages with their neighbouring stride-1 layers (model_0/model.py:98-144,148-196).
#include "wino_chain.h"

namespace tic {

template <int WH>
static bool launch_wh(int in_mode, int out_mode, const ChainArgs& a, hipStream_t s) {
  const dim3 grid(a.n * a.rh * a.rw), block(256 * WH);
  if (in_mode == IN_F32 && out_mode == OUT_F32)
    hipLaunchKernelGGL((wino_chain_kernel<IN_F32, OUT_F32, WH>), grid, block, 0, s, a);
  else if (in_mode == IN_F32 && out_mode == OUT_QUANT)
    hipLaunchKernelGGL((wino_chain_kernel<IN_F32, OUT_QUANT, WH>), grid, block, 0, s, a);
  else if (in_mode == IN_IDX && out_mode == OUT_F32)
    hipLaunchKernelGGL((wino_chain_kernel<IN_IDX, OUT_F32, WH>), grid, block, 0, s, a);
  else
    return false;
  return true;
}

bool launch_wino_chain(int in_mode, int out_mode, const ChainArgs& a, hipStream_t s, int wh) {
  if (a.nl < 2 || a.nl > CH_MAX_LAYERS) return false;
  if (wh == 2) return launch_wh<2>(in_mode, out_mode, a, s);
  if (wh == 1) return launch_wh<1>(in_mode, out_mode, a, s);
  return false;
}

}  // namespace tic
