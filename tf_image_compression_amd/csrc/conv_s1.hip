// Stride-1 'SAME' 3x3 convolutions: res_block convs (basic_block/basic_block.py:74-93),
// encode_4 / decode_4 of model_0/1 (model_0/model.py:124-134,159-169), rmbe conv_3/4.
// Several tilings per layer type; the runtime picks by grid size (tic_runtime.cpp).
#include "conv_launch.h"

#define S1_VARIANTS(ACT, RES, IN, OUT)                                 \
  TIC_CONV(MODE_S1, 64, 64, 4, 4, 1, ACT, RES, IN, OUT),               \
      TIC_CONV3(MODE_S1, 64, 64, 4, 4, 2, ACT, RES, IN, OUT),          \
      TIC_CONV(MODE_S1, 64, 64, 8, 4, 1, ACT, RES, IN, OUT),           \
      TIC_CONV3(MODE_S1, 64, 64, 2, 2, 1, ACT, RES, IN, OUT),          \
      TIC_CONV3(MODE_S1, 64, 64, 2, 2, 2, ACT, RES, IN, OUT),          \
      TIC_CONV3(MODE_S1, 64, 64, 4, 4, 4, ACT, RES, IN, OUT),          \
      TIC_CONV3(MODE_S1, 64, 64, 1, 1, 1, ACT, RES, IN, OUT)

namespace tic {
static const ConvEntry kS1[] = {
    S1_VARIANTS(ACT_RELU, false, IN_F32, OUT_F32),
    S1_VARIANTS(ACT_RELU, true, IN_F32, OUT_F32),
    S1_VARIANTS(ACT_ID, false, IN_F32, OUT_QUANT),
    S1_VARIANTS(ACT_ID, false, IN_IDX, OUT_F32),
    S1_VARIANTS(ACT_ID, false, IN_F32, OUT_F32),
};
const ConvEntry* conv_registry_s1(int* count) {
  *count = sizeof(kS1) / sizeof(kS1[0]);
  return kS1;
}
}  // namespace tic
