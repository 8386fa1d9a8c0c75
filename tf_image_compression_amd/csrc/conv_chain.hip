// Chains of stride-1 64->64 layers in one launch (wino_chain.h): the codecs' residual
// stages with their neighbouring stride-1 layers (model_0/model.py:98-144,148-196).
#include "wino4_pchain.h"
#include "wino_chain_cs.h"

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

// channel-split shapes (wino_chain_cs.h): two workgroups per region, 256 or 512 threads
template <int WH>
static bool launch_cs(int in_mode, int out_mode, const ChainArgs& a, hipStream_t s) {
  const dim3 grid(a.n * a.rh * a.rw * 2), block(256 * WH);
  if (in_mode == IN_F32 && out_mode == OUT_F32)
    hipLaunchKernelGGL((wino_chain_cs_kernel<IN_F32, OUT_F32, WH>), grid, block, 0, s, a);
  else if (in_mode == IN_F32 && out_mode == OUT_QUANT)
    hipLaunchKernelGGL((wino_chain_cs_kernel<IN_F32, OUT_QUANT, WH>), grid, block, 0, s, a);
  else if (in_mode == IN_IDX && out_mode == OUT_F32)
    hipLaunchKernelGGL((wino_chain_cs_kernel<IN_IDX, OUT_F32, WH>), grid, block, 0, s, a);
  else
    return false;
  return true;
}

bool launch_wino_chain(int in_mode, int out_mode, const ChainArgs& a, hipStream_t s, int wh) {
  if (a.nl < 2 || a.nl > CH_MAX_LAYERS) return false;
  if (wh == 3) return launch_cs<1>(in_mode, out_mode, a, s);
  if (wh == 4) return launch_cs<2>(in_mode, out_mode, a, s);
  if (wh == 2) return launch_wh<2>(in_mode, out_mode, a, s);
  if (wh == 1) return launch_wh<1>(in_mode, out_mode, a, s);
  return false;
}

// whole-patch F(4x4,3x3) chain of a 16x16 map (wino4_pchain.h): four workgroups per patch
bool launch_wino4_pchain(int in_mode, int out_mode, const ChainArgs& a, hipStream_t s) {
  if (a.nl < 2 || a.nl > CH_MAX_LAYERS || a.H > 16 || a.W > 16 || a.H < 1 || a.W < 1 || a.layer[0].res) return false;
  const dim3 grid(a.n * 4), block(pchain::NTH);
  if (in_mode == IN_F32 && out_mode == OUT_F32)
    hipLaunchKernelGGL((wino4_pchain_kernel<IN_F32, OUT_F32>), grid, block, 0, s, a);
  else if (in_mode == IN_F32 && out_mode == OUT_QUANT)
    hipLaunchKernelGGL((wino4_pchain_kernel<IN_F32, OUT_QUANT>), grid, block, 0, s, a);
  else if (in_mode == IN_IDX && out_mode == OUT_F32)
    hipLaunchKernelGGL((wino4_pchain_kernel<IN_IDX, OUT_F32>), grid, block, 0, s, a);
  else
    return false;
  return true;
}

}  // namespace tic
