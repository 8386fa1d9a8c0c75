// Stride-1 'SAME' 3x3 convolutions: res_block convs (basic_block/basic_block.py:74-93),
// encode_4 / decode_4 of model_0/1 (model_0/model.py:124-134,159-169), rmbe conv_3/4.
#include "conv_launch.h"

namespace tic {
using namespace tic;
static const ConvEntry kS1[] = {
    TIC_CONV(MODE_S1, 64, 64, 4, 4, ACT_RELU, false, IN_F32, OUT_F32),
    TIC_CONV(MODE_S1, 64, 64, 4, 4, ACT_RELU, true, IN_F32, OUT_F32),
    TIC_CONV(MODE_S1, 64, 64, 4, 4, ACT_ID, false, IN_F32, OUT_QUANT),
    TIC_CONV(MODE_S1, 64, 64, 4, 4, ACT_ID, false, IN_IDX, OUT_F32),
    TIC_CONV(MODE_S1, 64, 64, 4, 4, ACT_ID, false, IN_F32, OUT_F32),
};
const ConvEntry* conv_registry_s1(int* count) {
  *count = sizeof(kS1) / sizeof(kS1[0]);
  return kS1;
}
}  // namespace tic
