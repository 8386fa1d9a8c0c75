// Stride-2 'SAME' transposed 3x3 convolutions of the synthesis stacks
// (model_0/model.py:198-234, model_2/model.py:118-180, model_3/model.py:157-286, rmbe conv_5).
#include "conv3x3_pwino.h"
#include "conv_launch.h"

namespace tic {
static const ConvEntry kT2[] = {
    TIC_CONV(MODE_T2, 64, 64, 4, 4, 1, ACT_RELU, false, IN_F32, OUT_F32),
    TIC_CONV(MODE_T2, 64, 64, 4, 4, 2, ACT_RELU, false, IN_F32, OUT_F32),
    TIC_CONV3(MODE_T2, 64, 64, 2, 2, 1, ACT_RELU, false, IN_F32, OUT_F32),
    TIC_CONV3(MODE_T2, 64, 64, 2, 2, 2, ACT_RELU, false, IN_F32, OUT_F32),
    TIC_CONV3(MODE_T2, 64, 64, 4, 4, 4, ACT_RELU, false, IN_F32, OUT_F32),
    TIC_CONV(MODE_T2, 64, 32, 4, 4, 1, ACT_RELU, false, IN_F32, OUT_F32),
    TIC_CONV(MODE_T2, 64, 32, 8, 4, 1, ACT_RELU, false, IN_F32, OUT_F32),
    TIC_CONV(MODE_T2, 32, 32, 4, 4, 1, ACT_RELU, false, IN_F32, OUT_F32),
    TIC_CONV(MODE_T2, 32, 32, 8, 4, 1, ACT_RELU, false, IN_F32, OUT_F32),
    TIC_CONV(MODE_T2, 32, 16, 4, 4, 1, ACT_RELU, false, IN_F32, OUT_F32),
    TIC_CONV(MODE_T2, 32, 16, 8, 4, 1, ACT_RELU, false, IN_F32, OUT_F32),
    TIC_CONV(MODE_T2, 64, 64, 4, 4, 1, ACT_ID, false, IN_IDX, OUT_F32),
    TIC_CONV3(MODE_T2, 64, 64, 4, 4, 2, ACT_ID, false, IN_IDX, OUT_F32),
    TIC_CONV3(MODE_T2, 64, 64, 2, 2, 1, ACT_ID, false, IN_IDX, OUT_F32),
    TIC_CONV3(MODE_T2, 64, 64, 2, 2, 2, ACT_ID, false, IN_IDX, OUT_F32),
    TIC_CONV(MODE_T2, 80, 64, 4, 4, 1, ACT_ID, false, IN_IDX, OUT_F32),
    TIC_CONV(MODE_T2, 80, 64, 4, 4, 2, ACT_ID, false, IN_IDX, OUT_F32),
    TIC_CONV(MODE_T2, 64, 64, 4, 4, 1, ACT_ID, false, IN_F32, OUT_F32),
    // base_model/ch_128 decode_2 (128 -> 64)
    TIC_CONVL2(MODE_T2, 128, 64, 4, 4, 1, ACT_RELU, false, IN_F32, OUT_F32),
    TIC_CONVL2(MODE_T2, 128, 64, 4, 4, 2, ACT_RELU, false, IN_F32, OUT_F32),
    TIC_CONVL2(MODE_T2, 128, 64, 2, 2, 1, ACT_RELU, false, IN_F32, OUT_F32),
    // polyphase Winograd form (s2_form 1, conv3x3_pwino.h); new entries go at the end
    TIC_PWINO(MODE_T2, 64, 64, 1, ACT_RELU, false, IN_F32, OUT_F32),
    TIC_PWINO(MODE_T2, 64, 32, 2, ACT_RELU, false, IN_F32, OUT_F32),
    TIC_PWINO(MODE_T2, 64, 64, 1, ACT_ID, false, IN_IDX, OUT_F32),
    TIC_PWINO(MODE_T2, 80, 64, 1, ACT_ID, false, IN_IDX, OUT_F32),
    TIC_PWINO(MODE_T2, 64, 64, 1, ACT_ID, false, IN_F32, OUT_F32),
    TIC_PWINO(MODE_T2, 128, 64, 1, ACT_RELU, false, IN_F32, OUT_F32),
};
const ConvEntry* conv_registry_t2(int* count) {
  *count = sizeof(kT2) / sizeof(kT2[0]);
  return kT2;
}
}  // namespace tic
