// Chains of stride-1 64->64 layers in one launch (wino_chain.h): the codecs' residual
// stages with their neighbouring stride-1 layers (model_0/model.py:98-144,148-196).
#include "wino_chain.h"

namespace tic {

bool launch_wino_chain(int in_mode, int out_mode, const ChainArgs& a, hipStream_t s) {
  if (a.nl < 2 || a.nl > CH_MAX_LAYERS) return false;
  const dim3 grid(a.n * a.rh * a.rw);
  if (in_mode == IN_F32 && out_mode == OUT_F32)
    hipLaunchKernelGGL((wino_chain_kernel<IN_F32, OUT_F32>), grid, dim3(256), 0, s, a);
  else if (in_mode == IN_F32 && out_mode == OUT_QUANT)
    hipLaunchKernelGGL((wino_chain_kernel<IN_F32, OUT_QUANT>), grid, dim3(256), 0, s, a);
  else if (in_mode == IN_IDX && out_mode == OUT_F32)
    hipLaunchKernelGGL((wino_chain_kernel<IN_IDX, OUT_F32>), grid, dim3(256), 0, s, a);
  else
    return false;
  return true;
}

}  // namespace tic
