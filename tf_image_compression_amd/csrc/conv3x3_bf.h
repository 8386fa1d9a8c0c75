// conv3x3_bf.h — the implicit-GEMM 3x3 convolution of conv3x3.h (same modes, same tilings,
// same fused epilogue: my_conv2d / my_conv2d_transpose / res_block, basic_block/
// basic_block.py:27-93) with its f32 products carried by the bf16 matrix path.
//
// Why: on gfx950 the f32 MFMA (v_mfma_f32_16x16x4_f32) runs at the f32 VECTOR rate, 1/16 of
// the bf16 MFMA (MI355X_MICROARCH.md "Peak FP32 (matrix)"), and the vector instructions beside
// it add to its cycles.  An f32 operand splits EXACTLY into three bf16 parts,
// x = x0 + x1 + x2 (x0 = bf16_rne(x), x1 = bf16_rne(x - x0), x2 = bf16_rne(x - x0 - x1):
// 8 + 8 + 8 significand bits), and every product of two parts is exact in f32.  The six
// leading part products
//     x0w0 + (x0w1 + x1w0) + (x0w2 + x1w1 + x2w0)
// carry the f32 product to within 2^-23 |xw| (the three dropped ones are below 2^-24 |xw|
// together: |x1| <= 2^-8 |x|, |x2| <= 2^-16 |x|), i.e. the rounding of one f32 multiply; they
// are summed in f32 by v_mfma_f32_16x16x32_bf16 at 16x the f32 matrix rate — three MFMAs of
// 16 cycles per 16-channel step instead of four of 32 (2.67x less matrix time).  Accuracy
// against the f64 oracle is that of an f32 convolution with another summation order
// (tests/test_gpu_bf16.py: every layer within the f32 form's bar, error beside the f32
// form's); this is a stride / transposed-conv "form" like the Winograd forms of the
// stride-1 layers — a fixed policy, not a tuning result (tic_runtime.cpp, option "mma").
//
// MFMA v_mfma_f32_16x16x32_bf16: A = weights 16 (out ch) x 32 (k), B = activations 32 (k) x
// 16 (pixels); lane (li, lg) supplies k = 8 lg .. 8 lg + 7 of row / column li; D as in the
// f32 form (lane holds out channels 4 lg .. 4 lg + 3 of pixel li), so the epilogue is
// conv3x3_kernel's.  One MFMA covers a 16-channel chunk in two parts: lane group lg holds
// channels 4 lg .. 4 lg + 3 of the chunk in both halves of its 8 k values:
//     M1: A = [w0 | w0], B = T1 = [x1 | x0]  -> w0 x1 + w0 x0
//     M2: A = [w1 | w1], B = T1              -> w1 x1 + w1 x0
//     M3: A = [w2 | w0], B = T2 = [x0 | x2]  -> w2 x0 + w0 x2
// issued M3, M2, M1 (small terms first).
//
// LDS activation tile: per (pixel, channel quad) a 24-byte record [x1 | x0 | x2] (4 bf16
// each; 1.5x the f32 tile), split once at staging; a step reads it with three ds_read_b64
// and forms T1 / T2 in registers.  Pixel stride 6 Cin/4 + 4 dwords: the ds_read_b64 of 16
// pixels x 4 lane groups is conflict-free in both 32-lane halves.
// Weights: packed on the host as [tap][Cin/16][4 lg][Cout][w0 | w1 | w2] (4 bf16 each, 24
// bytes per lane and step: three 8-byte buffer loads), from L2 into registers two steps
// ahead; the tuples A1..A3 are register copies.
#pragma once
#include "conv3x3.h"

namespace tic {

typedef __bf16 bf16x2_t __attribute__((ext_vector_type(2)));
typedef __bf16 bf16x8_t __attribute__((ext_vector_type(8)));
typedef unsigned int u32x2_t __attribute__((ext_vector_type(2)));
typedef float f32x2_t __attribute__((ext_vector_type(2)));

__device__ __forceinline__ f32x4 mfma_bf(wu32x4 a, wu32x4 b, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8_t, a), __builtin_bit_cast(bf16x8_t, b), c,
                                                0, 0, 0);
}

// two f32 -> packed bf16 (round to nearest even: v_cvt_pk_bf16_f32) and the parts back in f32
__device__ __forceinline__ unsigned bf_pack(float a, float b) {
  return __builtin_bit_cast(unsigned, __builtin_convertvector(f32x2_t{a, b}, bf16x2_t));
}
__device__ __forceinline__ float bf_lo(unsigned p) { return __uint_as_float(p << 16); }
__device__ __forceinline__ float bf_hi(unsigned p) { return __uint_as_float(p & 0xffff0000u); }

// exact three-way split of 4 channels: x0 = rne(v), x1 = rne(v - x0), x2 = rne(v - x0 - x1)
__device__ __forceinline__ void bf_split4(f32x4 v, u32x2_t& x0, u32x2_t& x1, u32x2_t& x2) {
  const unsigned h01 = bf_pack(v.x, v.y), h23 = bf_pack(v.z, v.w);
  const float r0 = v.x - bf_lo(h01), r1 = v.y - bf_hi(h01), r2 = v.z - bf_lo(h23), r3 = v.w - bf_hi(h23);
  const unsigned m01 = bf_pack(r0, r1), m23 = bf_pack(r2, r3);
  const unsigned l01 = bf_pack(r0 - bf_lo(m01), r1 - bf_hi(m01)), l23 = bf_pack(r2 - bf_lo(m23), r3 - bf_hi(m23));
  x0 = u32x2_t{h01, h23};
  x1 = u32x2_t{m01, m23};
  x2 = u32x2_t{l01, l23};
}

template <int CIN>
struct BfTile {
  static constexpr int REC = 6;                  // dwords per (pixel, quad) record
  static constexpr int PS = REC * CIN / 4 + 4;   // dwords per pixel (conflict-free b64 reads)
};

template <int MODE, int CIN, int COUT, int TH, int WR, int NSPLIT, int ACT, bool RES, int IN, int OUT>
__global__ void __launch_bounds__(256) conv3x3_bf_kernel(const ConvArgs a) {
  static_assert(CIN % 16 == 0 && COUT % 16 == 0, "channels must be multiples of 16");
  constexpr int PS = BfTile<CIN>::PS;
  constexpr int KC = CIN / 16;
  constexpr int COUT_WG = COUT / NSPLIT;
  static_assert(COUT_WG % 16 == 0, "bad channel split");
  constexpr int NBT = COUT_WG / 16;
  constexpr int WC = 4 / WR;
  static_assert(WR * WC == 4 && TH % WR == 0 && NBT % WC == 0, "bad wave split");
  constexpr int NB = NBT / WC;
  constexpr int MB = TH / WR;
  constexpr int NPH = MODE == MODE_T2 ? 4 : 1;
  constexpr int LR = TileGeom<MODE, TH>::LR;
  constexpr int LC = TileGeom<MODE, TH>::LC;
  constexpr int C4 = CIN / 4;
  constexpr int NSTEP = 9 * KC;
  constexpr int TILE = LR * LC * PS;  // dwords of the input tile

  __shared__ __attribute__((aligned(16))) unsigned smem[TILE];

  const int tid = threadIdx.x;
  const int split = NSPLIT > 1 ? (int)(blockIdx.x % NSPLIT) : 0;
  const int gx0 = (NSPLIT > 1 ? (int)(blockIdx.x / NSPLIT) : (int)blockIdx.x) * 16;
  const int gy0 = blockIdx.y * TH;
  const int nimg = blockIdx.z;
  const int H = a.H, W = a.W;

  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int lane = tid & 63;
  const int wr = wave / WC;
  const int wc = wave % WC;
  const int li = lane & 15;
  const int lg = lane >> 4;
  const int co_wg = split * COUT_WG;
  const int co_wave = wc * NB * 16;

  // ---- weights: [tap][kc][lg][COUT][6 dwords] -> w0, w1, w2 of this lane's channels ----
  const __amdgpu_buffer_rsrc_t wrs = weight_rsrc(a.wp, 9 * KC * 4 * COUT * 24);
  const int wlb = (lg * COUT + co_wg + co_wave + li) * 24;  // lane byte offset
  struct W3 {
    u32x2_t p[3];
  };
  auto wglob = [&](int s, int nb) -> W3 {
    const int so = (s * 4 * COUT + nb * 16) * 24;
    W3 w;
#pragma unroll
    for (int q = 0; q < 3; ++q) w.p[q] = __builtin_amdgcn_raw_buffer_load_b64(wrs, wlb, so + 8 * q, 0);
    return w;
  };
  constexpr int PF = 2;
  W3 av[PF + 1][NB];
#pragma unroll
  for (int p = 0; p < PF; ++p)
#pragma unroll
    for (int nb = 0; nb < NB; ++nb)
      if (p < NSTEP) av[p][nb] = wglob(p, nb);

  // ---- stage the input tile: f32 (or dequantised symbols) -> three bf16 parts ----
  constexpr int NSTAGE = LR * LC * C4;
  constexpr int NIT = (NSTAGE + 255) / 256;
  constexpr int SB = NIT < 8 ? NIT : 8;
#pragma unroll
  for (int i0 = 0; i0 < NIT; i0 += SB) {
    f32x4 tmp[SB];
#pragma unroll
    for (int i = 0; i < SB; ++i) {
      const int e = (i0 + i) * 256 + tid;
      tmp[i] = f32x4{0.f, 0.f, 0.f, 0.f};
      if (i0 + i < NIT && e < NSTAGE) {
        const int c4 = e % C4;
        const int pe = e / C4;
        const int col = pe % LC;
        const int row = pe / LC;
        int iy, ix;
        if constexpr (MODE == MODE_S2) {
          const int plane = col >= 17 ? 1 : 0;
          iy = 2 * gy0 + row - a.pad_y;
          ix = 2 * gx0 + 2 * (col - plane * 17) + plane - a.pad_x;
        } else if constexpr (MODE == MODE_S1) {
          iy = gy0 - a.pad_y + row;
          ix = gx0 - a.pad_x + col;
        } else {
          iy = gy0 - 1 + row;
          ix = gx0 - 1 + col;
        }
        if (iy >= 0 && iy < H && ix >= 0 && ix < W) {
          const size_t off = ((size_t)(nimg * H + iy) * W + ix) * CIN + c4 * 4;
          if constexpr (IN == IN_F32) {
            tmp[i] = *reinterpret_cast<const f32x4*>(reinterpret_cast<const float*>(a.in) + off);
          } else {
            const uint32_t q = *reinterpret_cast<const uint32_t*>(reinterpret_cast<const uint8_t*>(a.in) + off);
            tmp[i].x = a.lut[q & 0xff];
            tmp[i].y = a.lut[(q >> 8) & 0xff];
            tmp[i].z = a.lut[(q >> 16) & 0xff];
            tmp[i].w = a.lut[q >> 24];
          }
        }
      }
    }
#pragma unroll
    for (int i = 0; i < SB; ++i) {
      const int e = (i0 + i) * 256 + tid;
      if (i0 + i < NIT && e < NSTAGE) {
        const int c4 = e % C4, pe = e / C4;
        u32x2_t x0, x1, x2;
        bf_split4(tmp[i], x0, x1, x2);
        unsigned* r = &smem[pe * PS + c4 * 6];
        *reinterpret_cast<u32x2_t*>(r) = x1;
        *reinterpret_cast<u32x2_t*>(r + 2) = x0;
        *reinterpret_cast<u32x2_t*>(r + 4) = x2;
      }
    }
  }
  __syncthreads();

  f32x4 acc[NPH][MB][NB];
#pragma unroll
  for (int p = 0; p < NPH; ++p)
#pragma unroll
    for (int mb = 0; mb < MB; ++mb)
#pragma unroll
      for (int nb = 0; nb < NB; ++nb) acc[p][mb][nb] = f32x4{0.f, 0.f, 0.f, 0.f};

  // this lane's parts of step s (pixel row mb): x1, x0, x2 of its channel quad
  struct X3 {
    u32x2_t p1, p0, p2;
  };
  auto load_b = [&](int s, X3* dst) {
    const int tap = s / KC, kc = s % KC;
    const int ky = tap / 3, kx = tap % 3;
#pragma unroll
    for (int mb = 0; mb < MB; ++mb) {
      const int r = wr * MB + mb;
      int lp;
      if constexpr (MODE == MODE_S1) lp = (r + ky) * LC + li + kx;
      else if constexpr (MODE == MODE_S2) lp = (2 * r + ky) * LC + (kx & 1) * 17 + li + (kx >> 1);
      else lp = (r + 1 - (ky == 2)) * LC + li + 1 - (kx == 2);
      const unsigned* rec = &smem[lp * PS + (kc * 4 + lg) * 6];
      dst[mb].p1 = *reinterpret_cast<const u32x2_t*>(rec);
      dst[mb].p0 = *reinterpret_cast<const u32x2_t*>(rec + 2);
      dst[mb].p2 = *reinterpret_cast<const u32x2_t*>(rec + 4);
    }
  };

  X3 bx[2][MB];
  load_b(0, bx[0]);
#pragma unroll
  for (int s = 0; s < NSTEP; ++s) {
    const int tap = s / KC;
    const int ky = tap / 3, kx = tap % 3;
    const int c = s & 1;
    if (s + PF < NSTEP) {
#pragma unroll
      for (int nb = 0; nb < NB; ++nb) av[(s + PF) % (PF + 1)][nb] = wglob(s + PF, nb);
    }
    if (s + 1 < NSTEP) load_b(s + 1, bx[c ^ 1]);
    __builtin_amdgcn_sched_barrier(0);
    const int ph = MODE == MODE_T2 ? (ky == 1 ? 2 : 0) + (kx == 1 ? 1 : 0) : 0;
    const int wi = s % (PF + 1);
#pragma unroll
    for (int nb = 0; nb < NB; ++nb) {
      const W3& w = av[wi][nb];
      const wu32x4 a1 = {w.p[0].x, w.p[0].y, w.p[0].x, w.p[0].y};
      const wu32x4 a2 = {w.p[1].x, w.p[1].y, w.p[1].x, w.p[1].y};
      const wu32x4 a3 = {w.p[2].x, w.p[2].y, w.p[0].x, w.p[0].y};
#pragma unroll
      for (int mb = 0; mb < MB; ++mb) {
        const X3& x = bx[c][mb];
        const wu32x4 t1 = {x.p1.x, x.p1.y, x.p0.x, x.p0.y};
        const wu32x4 t2 = {x.p0.x, x.p0.y, x.p2.x, x.p2.y};
        f32x4 v = acc[ph][mb][nb];
        v = mfma_bf(a3, t2, v);
        v = mfma_bf(a2, t1, v);
        v = mfma_bf(a1, t1, v);
        acc[ph][mb][nb] = v;
      }
    }
    __builtin_amdgcn_sched_barrier(0);
  }

  // ---- fused epilogue (conv3x3_kernel's): + bias, act, + residual, f32 store or quantiser ----
  const int Ho = a.Ho, Wo = a.Wo;
#pragma unroll
  for (int p = 0; p < NPH; ++p) {
#pragma unroll
    for (int mb = 0; mb < MB; ++mb) {
      const int r = wr * MB + mb;
      int oy, ox;
      if constexpr (MODE == MODE_T2) {
        if (gy0 + r >= H || gx0 + li >= W) continue;
        oy = 2 * (gy0 + r) + (p >> 1);
        ox = 2 * (gx0 + li) + (p & 1);
      } else {
        oy = gy0 + r;
        ox = gx0 + li;
        if (oy >= Ho || ox >= Wo) continue;
      }
#pragma unroll
      for (int nb = 0; nb < NB; ++nb) {
        const int co = co_wg + co_wave + nb * 16 + lg * 4;
        const f32x4 bb = *reinterpret_cast<const f32x4*>(a.bias + co);
        f32x4 v = acc[p][mb][nb];
        v.x = __fadd_rn(v.x, bb.x);
        v.y = __fadd_rn(v.y, bb.y);
        v.z = __fadd_rn(v.z, bb.z);
        v.w = __fadd_rn(v.w, bb.w);
        if constexpr (ACT == ACT_RELU) {
          v.x = fmaxf(v.x, 0.f);
          v.y = fmaxf(v.y, 0.f);
          v.z = fmaxf(v.z, 0.f);
          v.w = fmaxf(v.w, 0.f);
        }
        const size_t o = ((size_t)(nimg * Ho + oy) * Wo + ox) * COUT + co;
        if constexpr (RES) {
          const f32x4 rr = *reinterpret_cast<const f32x4*>(a.res + o);
          v.x = __fadd_rn(v.x, rr.x);
          v.y = __fadd_rn(v.y, rr.y);
          v.z = __fadd_rn(v.z, rr.z);
          v.w = __fadd_rn(v.w, rr.w);
        }
        if constexpr (OUT == OUT_F32) {
          *reinterpret_cast<f32x4*>(a.out + o) = v;
        } else {
          if (a.out) *reinterpret_cast<f32x4*>(a.out + o) = v;
          const uint32_t q = quant1(v.x, a.qscale) | (quant1(v.y, a.qscale) << 8) |
                             (quant1(v.z, a.qscale) << 16) | (quant1(v.w, a.qscale) << 24);
          *reinterpret_cast<uint32_t*>(a.qout + o) = q;
        }
      }
    }
  }
}

}  // namespace tic
