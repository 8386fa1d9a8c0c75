// Chains of stride-1 64->64 layers in one launch (wino_chain.h): the codecs' residual
// stages with their neighbouring stride-1 layers (model_0/model.py:98-144,148-196), and
// optionally the stride-2 layer in front (encode_3) / the transposed layer behind (decode_3).
#include "wino_chain.h"

namespace tic {

template <int WH, int HT>
static bool launch_wh(int in_mode, int out_mode, const ChainArgs& a, hipStream_t s) {
  const dim3 grid(a.n * a.rh * a.rw), block(256 * WH);
  if (in_mode == IN_F32 && out_mode == OUT_F32)
    hipLaunchKernelGGL((wino_chain_kernel<IN_F32, OUT_F32, WH, HT>), grid, block, 0, s, a);
  else if (in_mode == IN_F32 && out_mode == OUT_QUANT && !(HT & (CH_TAIL | CH_TAIL2 | CH_TAIL2_PW)))
    hipLaunchKernelGGL((wino_chain_kernel<IN_F32, OUT_QUANT, WH, HT & CH_HEAD>), grid, block, 0, s, a);
  else if (in_mode == IN_IDX && out_mode == OUT_F32 && !(HT & CH_HEAD))
    hipLaunchKernelGGL((wino_chain_kernel<IN_IDX, OUT_F32, WH, HT & (CH_TAIL | CH_TAIL2 | CH_TAIL2_PW)>), grid, block, 0, s, a);
  else
    return false;
  return true;
}

// ht: CH_HEAD (the stride-2 layer in front, encoder side) and / or CH_TAIL (the transposed
// layer behind, decoder side; with CH_TAIL2 the next transposed layer as well); all need the
// 512-thread workgroup
bool launch_wino_chain(int in_mode, int out_mode, const ChainArgs& a, hipStream_t s, int wh, int ht) {
  if (a.nl < 2 || a.nl > CH_MAX_LAYERS) return false;
  if (ht != 0 && wh != 2) return false;
  if (wh == 2) {
    if (ht == 0) return launch_wh<2, 0>(in_mode, out_mode, a, s);
    if (ht == CH_HEAD) return launch_wh<2, CH_HEAD>(in_mode, out_mode, a, s);
    if (ht == CH_TAIL) return launch_wh<2, CH_TAIL>(in_mode, out_mode, a, s);
    if (ht == (CH_TAIL | CH_TAIL2)) return launch_wh<2, CH_TAIL | CH_TAIL2>(in_mode, out_mode, a, s);
    if (ht == (CH_TAIL | CH_TAIL2 | CH_TAIL2_PW))
      return launch_wh<2, CH_TAIL | CH_TAIL2 | CH_TAIL2_PW>(in_mode, out_mode, a, s);
    return false;
  }
  if (wh == 1) return launch_wh<1, 0>(in_mode, out_mode, a, s);
  return false;
}

}  // namespace tic
