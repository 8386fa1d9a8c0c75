// tic_kernels.h — argument blocks and the launch registry shared by the kernels
// (conv_*.hip) and the host runtime (tic_runtime.cpp).  Internal; not part of the C-ABI.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace tic {

typedef float f32x4 __attribute__((ext_vector_type(4)));

enum { MODE_S1 = 0, MODE_S2 = 1, MODE_T2 = 2 };
enum { ACT_ID = 0, ACT_RELU = 1 };
enum { IN_F32 = 0, IN_IDX = 1 };
enum { OUT_F32 = 0, OUT_QUANT = 1 };

struct ConvArgs {
  const void* in;      // f32 NHWC [N,H,W,Cin]  or u8 symbols (IN_IDX)
  const float* wp;     // packed weights [tap][Cin/16][Cout][4][4]
  const float* bias;   // [Cout]
  const float* res;    // residual [N,Ho,Wo,Cout] or nullptr
  float* out;          // f32 [N,Ho,Wo,Cout]; with OUT_QUANT: optional pre-activation
  uint8_t* qout;       // OUT_QUANT: u8 symbols [N,Ho,Wo,Cout]
  const float* lut;    // IN_IDX: dequantiser table (Q entries)
  int H, W;            // input spatial
  int Ho, Wo;          // output spatial
  int pad_y, pad_x;    // SAME pad_before (S1: 1; S2: 0 for even input, 1 for odd; T2: unused)
  float qscale;        // Q - 1
  int num_cus;         // compute units (persistent variants size their grid from it)
  int grid_cap;        // > 0: cap on the persistent grid (tests force several tiles per workgroup)
  int max_n;           // > 0: F(4x4,3x3) launches at most this many patches at a time (tests of
                       // the launch-split path; 0: split only where 32-bit offsets require it)
  unsigned long long* tstamp;  // timing probe (TIC_WINO4_TIMING, per-layer entry only): [workgroup]
                               // [TIC_W4_TS] s_memrealtime stamps + hardware ids; null: off
  int probe;                   // timing probe bits (TIC_WINO4_PROBE, per-layer entry only; results
                               // invalid): 1 weights from one step, 2 no staging loads, 4 no stores
};
#define TIC_W4_TS 24

struct RgbInArgs {
  const void* in;      // [N,H,W,3] u8 or f32
  const float* wp;     // [Cout][4][8]
  const float* bias;   // [Cout]
  float* out;          // [N,Ho,Wo,Cout]
  int H, W, Ho, Wo;
  int pad_y, pad_x;    // SAME pad_before of the stride-2 conv
  float mean[3], std[3];
};

// First two analysis layers fused through LDS (RGB -> C0 stride 2 -> C1 stride 2).
struct Enc01Args {
  const void* in;      // [N,H,W,3] u8 or f32 RGB
  const float* wp0;    // layer 0, RGB packing [C0][4][8]
  const float* b0;     // [C0]
  const float* wp1;    // layer 1, generic packing [tap][C0/16][4][C1][4]
  const float* b1;     // [C1]
  float* out;          // [N,H2,W2,C1]
  int H, W;            // RGB size
  int H1, W1;          // layer-0 output size
  int H2, W2;          // layer-1 output size
  int pad0y, pad0x, pad1y, pad1x;  // SAME pad_before of both convs
  float mean[3], std[3];
  const float* nlut;   // u8 input: [3][256] (v - mean[c]) / std[c] in f32, computed on the host
  unsigned long long* tstamp;  // phase timestamps (TIC_ENC01_TIMING) or null: [workgroup][8]
};

struct RgbOutArgs {
  const float* in;     // [N,H,W,Cin]
  const float* wp;     // dense sub-pixel form: [4 off][Cin/16][16 rows][4][4]
  const float* wp2;    // scatter form: [2 rb][Cin/16][4 g][16 rows][4 t]
  const float* wraw;   // VALU form: the TF kernel as-is, [3][3][3][Cin]
  const float* bias;   // [3]
  uint8_t* out_u8;     // [N,2H,2W,3] or nullptr
  float* out_f32;      // [N,2H,2W,3] or nullptr
  int H, W;
  float mean[3], std[3];
  int num_cus;         // persistent variants size their grid from it
  int grid_cap;        // > 0: cap on the persistent grid (tests force several tiles per workgroup)
};

// decode_1 -> decode_0 fused through LDS (dec10.h).
struct Dec10Args {
  const float* in;     // decode_1 input [N,H,W,C1]
  const float* wp1;    // decode_1 generic packing [tap][C1/16][4 g][C0][4 t]
  const float* w1raw;  // decode_1 TF kernel as-is, [3][3][C0][C1]
  const float* b1;     // [C0]
  int H, W;            // decode_1 input size (decode_0's input is 2H x 2W)
  RgbOutArgs rgb;      // decode_0: wraw, bias, normalisation, outputs; rgb.H/W = 2H/2W
};

typedef void (*ConvLaunch)(const ConvArgs&, int n, hipStream_t);

struct ConvEntry {
  int mode, cin, cout, act, res, in, out;
  int th;             // output rows per block (input rows for T2)
  int wr;             // wave row-groups
  int nsplit;         // workgroups splitting the output channels of one pixel tile
  int wlds;           // weight source: 0 L2 (prefetch 2), 1 LDS-DMA ring, 2 L2 (prefetch 6),
  ConvLaunch fn;
};

// All compiled conv3x3 variants (conv_s1.hip, conv_s2.hip, conv_t2.hip).
const ConvEntry* conv_registry_s1(int* count);
const ConvEntry* conv_registry_s2(int* count);
const ConvEntry* conv_registry_t2(int* count);

// First / last layer launchers (conv_rgb.hip); `variant` < rgb_*_variants() selects the
// tiling / formulation; return false if the width is not compiled.  Last layer: variants
// 0-2 dense sub-pixel MFMA form (TH 4/8/16), 3-5 col2im MFMA form (TH 4/8/16), 6-11 VALU
// form (TW 64/32/16, then the same persistent + software-pipelined); each form has its own summation order, the tilings of one form are
// bit-identical.
int rgb_in_variants();
int enc01_variants();
constexpr int kEnc01Default = 3;  // compact LDS form, 4 layer-1 rows
bool launch_enc01(int c0, int c1, bool u8_input, const Enc01Args& a, int n, hipStream_t s, int variant);
int rgb_out_variants();
bool launch_rgb_in(int cout, bool u8_input, const RgbInArgs& a, int n, hipStream_t s, int variant);
bool launch_rgb_out(int cin, const RgbOutArgs& a, int n, hipStream_t s, int variant);
// decode_1 (C1 -> C0) + decode_0 fused; false if (C1, C0) is not compiled.  Variants are
// bit-identical (decode_0's weights via scalar loads or LDS).
int dec10_variants();
constexpr int kDec10Default = 8;  // compact LDS form, 4 rows, decode_0 weights by scalar loads
bool launch_dec10(int c1, int c0, const Dec10Args& a, int n, hipStream_t s, int variant);

// A chain of stride-1 64->64 layers in one launch (wino_chain.h, conv_chain.hip): args in
// wino_chain.h; false if the mode combination is not compiled.
struct ChainArgs;
// wh: 1 = 256-thread workgroups, 2 = 512-thread workgroups (output channels split in halves
// over the waves)
bool launch_wino_chain(int in_mode, int out_mode, const ChainArgs& a, hipStream_t s, int wh, int ht = 0);

// Whole-image glue and the symbol histogram (image_ops.hip).
void launch_tile_reflect(const uint8_t* img, int H, int W, int P, int hn, int wn, uint8_t* out, int num_cus,
                         hipStream_t s);
void launch_stitch(const float* patches, int H, int W, int P, int wn, float* img, int num_cus, hipStream_t s);
void launch_window_copy(float* img, int W, int r0, int c0, int S, int hn, int wn, float* win, bool to_windows,
                        int num_cus, hipStream_t s);
void launch_round_u8(const float* in, size_t n, uint8_t* out, int num_cus, hipStream_t s);
void launch_sse_u8(const uint8_t* a, const uint8_t* b, size_t n, unsigned long long* acc, int num_cus,
                   hipStream_t s);
void launch_histogram(const uint8_t* sym, size_t n, int Q, unsigned long long* counts, int num_cus, hipStream_t s);

}  // namespace tic
