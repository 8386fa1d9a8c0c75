// Stride-2 'SAME' 3x3 convolutions of the analysis stacks (model_0/model.py:62-96,
// model_2/model.py:62-122, model_3/model.py:62-161, rmbe conv_2).
#include "conv3x3_pwino.h"
#include "conv_launch.h"

namespace tic {
static const ConvEntry kS2[] = {
    TIC_CONV(MODE_S2, 16, 32, 4, 4, 1, ACT_RELU, false, IN_F32, OUT_F32),
    TIC_CONV(MODE_S2, 16, 32, 8, 4, 1, ACT_RELU, false, IN_F32, OUT_F32),
    TIC_CONV(MODE_S2, 32, 32, 4, 4, 1, ACT_RELU, false, IN_F32, OUT_F32),
    TIC_CONV(MODE_S2, 32, 32, 8, 4, 1, ACT_RELU, false, IN_F32, OUT_F32),
    TIC_CONV(MODE_S2, 32, 64, 4, 4, 1, ACT_RELU, false, IN_F32, OUT_F32),
    TIC_CONV(MODE_S2, 32, 64, 8, 4, 1, ACT_RELU, false, IN_F32, OUT_F32),
    TIC_CONV(MODE_S2, 32, 64, 4, 4, 2, ACT_RELU, false, IN_F32, OUT_F32),
    TIC_CONV(MODE_S2, 64, 64, 4, 4, 1, ACT_RELU, false, IN_F32, OUT_F32),
    TIC_CONV(MODE_S2, 64, 64, 4, 4, 2, ACT_RELU, false, IN_F32, OUT_F32),
    TIC_CONV3(MODE_S2, 64, 64, 2, 2, 1, ACT_RELU, false, IN_F32, OUT_F32),
    TIC_CONV3(MODE_S2, 64, 64, 2, 2, 2, ACT_RELU, false, IN_F32, OUT_F32),
    TIC_CONV3(MODE_S2, 64, 64, 4, 4, 4, ACT_RELU, false, IN_F32, OUT_F32),
    TIC_CONV(MODE_S2, 64, 64, 4, 4, 1, ACT_ID, false, IN_F32, OUT_QUANT),
    TIC_CONV3(MODE_S2, 64, 64, 4, 4, 2, ACT_ID, false, IN_F32, OUT_QUANT),
    TIC_CONV3(MODE_S2, 64, 64, 2, 2, 1, ACT_ID, false, IN_F32, OUT_QUANT),
    TIC_CONV3(MODE_S2, 64, 64, 2, 2, 2, ACT_ID, false, IN_F32, OUT_QUANT),
    TIC_CONV(MODE_S2, 64, 80, 4, 4, 1, ACT_ID, false, IN_F32, OUT_QUANT),
    // base_model/ch_128 encode_2 (64 -> 128)
    TIC_CONVL2(MODE_S2, 64, 128, 4, 4, 1, ACT_RELU, false, IN_F32, OUT_F32),
    TIC_CONVL2(MODE_S2, 64, 128, 4, 4, 2, ACT_RELU, false, IN_F32, OUT_F32),
    // polyphase Winograd form (s2_form 1, conv3x3_pwino.h); new entries go at the end: tuning
    // files name entries by their index in this table
    TIC_PWINO(MODE_S2, 32, 64, 1, ACT_RELU, false, IN_F32, OUT_F32),
    TIC_PWINO(MODE_S2, 64, 64, 1, ACT_RELU, false, IN_F32, OUT_F32),
    TIC_PWINO(MODE_S2, 64, 64, 1, ACT_ID, false, IN_F32, OUT_QUANT),
    TIC_PWINO(MODE_S2, 64, 80, 1, ACT_ID, false, IN_F32, OUT_QUANT),
    TIC_PWINO(MODE_S2, 64, 128, 1, ACT_RELU, false, IN_F32, OUT_F32),
};
const ConvEntry* conv_registry_s2(int* count) {
  *count = sizeof(kS2) / sizeof(kS2[0]);
  return kS2;
}
}  // namespace tic
