// Stride-1 'SAME' 3x3 convolutions: res_block convs (basic_block/basic_block.py:74-93),
// encode_4 / decode_4 of model_0/1 (model_0/model.py:124-134,159-169), rmbe conv_3/4.
// Three forms: the direct implicit GEMM (conv3x3_kernel, several tilings), Winograd
// F(2x2,3x3) (conv3x3_wino.h, weight source 4) and Winograd F(4x4,3x3) (conv3x3_wino4.h,
// weight source 5, 64 -> 64 res-block convs); the runtime picks the form by policy
// (option "s1_form") and a tiling within it by grid size or measurement (tic_runtime.cpp).
#include "conv3x3_wino.h"
#include "conv3x3_wino4.h"
#include "conv_launch.h"

#define S1_VARIANTS(ACT, RES, IN, OUT)                                 \
  TIC_CONV(MODE_S1, 64, 64, 4, 4, 1, ACT, RES, IN, OUT),               \
      TIC_CONV3(MODE_S1, 64, 64, 4, 4, 2, ACT, RES, IN, OUT),          \
      TIC_CONV(MODE_S1, 64, 64, 8, 4, 1, ACT, RES, IN, OUT),           \
      TIC_CONV3(MODE_S1, 64, 64, 2, 2, 1, ACT, RES, IN, OUT),          \
      TIC_CONV3(MODE_S1, 64, 64, 2, 2, 2, ACT, RES, IN, OUT),          \
      TIC_CONV3(MODE_S1, 64, 64, 4, 4, 4, ACT, RES, IN, OUT),          \
      TIC_CONV3(MODE_S1, 64, 64, 1, 1, 1, ACT, RES, IN, OUT)

// Winograd tilings (TTY, NN, NSPLIT): 2x32, 4x16 output pixels per 16-tile block; the
// channel splits give the 16x16 bottleneck layers of model_0/1 enough workgroups.
#define S1_WINO(ACT, RES, IN, OUT)                          \
  TIC_WINO(64, 64, 1, 1, 1, ACT, RES, IN, OUT),             \
      TIC_WINO(64, 64, 2, 1, 1, ACT, RES, IN, OUT),         \
      TIC_WINO(64, 64, 2, 1, 2, ACT, RES, IN, OUT),         \
      TIC_WINO(64, 64, 2, 1, 4, ACT, RES, IN, OUT),         \
      TIC_WINO(64, 64, 1, 1, 4, ACT, RES, IN, OUT),         \
      TIC_WINO(64, 64, 2, 2, 1, ACT, RES, IN, OUT),         \
      TIC_WINO(64, 64, 4, 2, 1, ACT, RES, IN, OUT)

// base_model/ch_128: the 128-wide res-block convs, encode_3 (128 -> 64, quantiser) and
// decode_3 (64 -> 128, dequantiser), direct and Winograd
#define S1_128(CIN, COUT, ACT, RES, IN, OUT)                           \
  TIC_CONVL2(MODE_S1, CIN, COUT, 4, 4, 2, ACT, RES, IN, OUT),          \
      TIC_CONVL2(MODE_S1, CIN, COUT, 2, 2, 2, ACT, RES, IN, OUT),      \
      TIC_CONVL2(MODE_S1, CIN, COUT, 4, 4, 4, ACT, RES, IN, OUT),      \
      TIC_WINO(CIN, COUT, 2, 1, 2, ACT, RES, IN, OUT),                 \
      TIC_WINO(CIN, COUT, 2, 1, 4, ACT, RES, IN, OUT),                 \
      TIC_WINO(CIN, COUT, 1, 1, 4, ACT, RES, IN, OUT)

// Winograd F(4x4,3x3) tilings (TTY = 1, 2, 4 tile rows: 4x64, 8x32, 16x16 output pixels per
// workgroup) for the 64 -> 64 res-block convs of model_3 and the rmbe net (form 2)
#define S1_WINO4(ACT, RES, IN, OUT)                 \
  TIC_WINO4(64, 64, 1, ACT, RES, IN, OUT),          \
      TIC_WINO4(64, 64, 2, ACT, RES, IN, OUT),      \
      TIC_WINO4(64, 64, 4, ACT, RES, IN, OUT)

namespace tic {
// new entries go at the end: tuning files name entries by their index in this table
static const ConvEntry kS1[] = {
    S1_VARIANTS(ACT_RELU, false, IN_F32, OUT_F32),
    S1_VARIANTS(ACT_RELU, true, IN_F32, OUT_F32),
    S1_VARIANTS(ACT_ID, false, IN_F32, OUT_QUANT),
    S1_VARIANTS(ACT_ID, false, IN_IDX, OUT_F32),
    S1_VARIANTS(ACT_ID, false, IN_F32, OUT_F32),
    S1_WINO(ACT_RELU, false, IN_F32, OUT_F32),
    S1_WINO(ACT_RELU, true, IN_F32, OUT_F32),
    S1_WINO(ACT_ID, false, IN_F32, OUT_QUANT),
    S1_WINO(ACT_ID, false, IN_IDX, OUT_F32),
    S1_WINO(ACT_ID, false, IN_F32, OUT_F32),
    S1_128(128, 128, ACT_RELU, false, IN_F32, OUT_F32),
    S1_128(128, 128, ACT_RELU, true, IN_F32, OUT_F32),
    S1_128(128, 64, ACT_ID, false, IN_F32, OUT_QUANT),
    S1_128(64, 128, ACT_ID, false, IN_IDX, OUT_F32),
    S1_WINO4(ACT_RELU, false, IN_F32, OUT_F32),
    S1_WINO4(ACT_RELU, true, IN_F32, OUT_F32),
    // model_0/1 encode_4 (quantiser) and decode_4 (dequantiser) in F(4x4,3x3) (s1_form 2)
    S1_WINO4(ACT_ID, false, IN_F32, OUT_QUANT),
    S1_WINO4(ACT_ID, false, IN_IDX, OUT_F32),
};
const ConvEntry* conv_registry_s1(int* count) {
  *count = sizeof(kS1) / sizeof(kS1[0]);
  return kS1;
}
}  // namespace tic
