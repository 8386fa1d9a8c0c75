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
// LDS activation tile: per (pixel, channel quad) the two B tuples T1 = [x1 | x0] and
// T2 = [x0 | x2] (4 bf16 each half), split once at staging — per 16-channel chunk the 32
// dwords [T1 of lane groups 0..3 | T2 of lane groups 0..3]; a step reads them with two
// ds_read_b128 that land in the MFMA operand registers as they are (an operand tuple built
// by register copies cost the first build four v_mov per MFMA).  Pixel stride 2 Cin + 8
// dwords (= 8 mod 16): conflict-free in every 16-lane group of ds_read_b128.
// Weights: per (tap, output-channel split) a slab [Cin/16][4 lg][Cout/NSPLIT] of the three A
// tuples [w0 | w0], [w1 | w1], [w2 | w0] (12 dwords; row pitch 12 Cout/NSPLIT = 0 mod 64:
// conflict-free), fetched once per workgroup by LDS-DMA one tap ahead into a 2-slot ring
// (WSRC 1), or per wave from L2 PF = 4 steps ahead (WSRC 0, small grids / large slabs).
// Why the ring: with the matrix time cut 2.67x, four waves each fetching the same weight
// fragments through the CU's 64 B/clk load path became the bound.
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
  static constexpr int PS = 2 * CIN + 8;  // dwords per pixel: 8 per channel quad + 8
};

template <int MODE, int CIN, int COUT, int TH, int WR, int NSPLIT, int WSRC, int ACT, bool RES, int IN, int OUT>
__global__ void __launch_bounds__(256) conv3x3_bf_kernel(const ConvArgs a) {
  static_assert(CIN % 16 == 0 && COUT % 16 == 0, "channels must be multiples of 16");
  constexpr bool WLDS = WSRC == 1;
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
  constexpr int TILE = LR * LC * PS;       // dwords of the input tile
  constexpr int RP = bf_wpitch(COUT_WG);   // weight row pitch (dwords), 12 COUT_WG
  constexpr int SLAB = KC * 4 * RP;        // dwords of one tap's weights for this split
  static_assert(SLAB % 4 == 0, "slab of 16-byte chunks");
  constexpr int SCH = SLAB / 4;            // 16-byte chunks per slab

  __shared__ __attribute__((aligned(16))) unsigned smem[TILE + (WLDS ? 2 * SLAB : 0)];

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

  // ---- weights: slab of (tap, split) at dword ((tap * NSPLIT + split) * SLAB); inside it the
  //      A tuples of (kc, lg, co_local) at (kc * 4 + lg) * RP + co_local * 12 ----
  const unsigned* const wsrc = reinterpret_cast<const unsigned*>(a.wp) + (size_t)split * SLAB;
  struct W3 {
    wu32x4 t[3];
  };
  const int wlane = lg * RP + (co_wave + li) * 12;  // this lane's record offset in a (kc) row block
  auto wdma = [&](int tap, int slot) {  // LDS-DMA one tap slab
#pragma unroll
    for (int j = 0; j < (SCH + 255) / 256; ++j) {
      const int cbase = (j * 4 + wave) * 64;
      if (SCH % 256 == 0 || cbase < SCH) {
        const unsigned* src = wsrc + (size_t)tap * NSPLIT * SLAB + (cbase + lane) * 4;
        if (SCH % 64 == 0 || cbase + lane < SCH)
          __builtin_amdgcn_global_load_lds(src, (lds_ptr_t)(smem + TILE + slot * SLAB + cbase * 4), 16, 0, 0);
      }
    }
  };
  const __amdgpu_buffer_rsrc_t wrs = weight_rsrc(a.wp, 9 * NSPLIT * SLAB * 4);
  auto wglob = [&](int s, int nb) -> W3 {
    const int tap = s / KC, kc = s % KC;
    const int so = ((tap * NSPLIT) * SLAB + kc * 4 * RP + nb * 16 * 12) * 4;
    W3 w;
#pragma unroll
    for (int q = 0; q < 3; ++q) w.t[q] = __builtin_amdgcn_raw_buffer_load_b128(wrs, (split * SLAB + wlane) * 4, so + 16 * q, 0);
    return w;
  };
  auto wlds = [&](int s, int nb) -> W3 {
    const int tap = s / KC, kc = s % KC;
    const unsigned* r = &smem[TILE + (tap & 1) * SLAB + kc * 4 * RP + wlane + nb * 16 * 12];
    W3 w;
#pragma unroll
    for (int q = 0; q < 3; ++q) w.t[q] = *reinterpret_cast<const wu32x4*>(r + 4 * q);
    return w;
  };
  constexpr int PF = WLDS ? 1 : 4;
  W3 av[PF + 1][NB];
  if constexpr (WLDS) {
    wdma(0, 0);
  } else {
#pragma unroll
    for (int p = 0; p < PF; ++p)
#pragma unroll
      for (int nb = 0; nb < NB; ++nb)
        if (p < NSTEP) av[p][nb] = wglob(p, nb);
  }

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
        // chunk c4 / 4, lane group c4 % 4: T1 at slot (c4 % 4), T2 at slot 4 + (c4 % 4)
        unsigned* r = &smem[pe * PS + (c4 >> 2) * 32 + (c4 & 3) * 4];
        *reinterpret_cast<wu32x4*>(r) = wu32x4{x1.x, x1.y, x0.x, x0.y};
        *reinterpret_cast<wu32x4*>(r + 16) = wu32x4{x0.x, x0.y, x2.x, x2.y};
      }
    }
  }
  if constexpr (WLDS) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();

  f32x4 acc[NPH][MB][NB];
#pragma unroll
  for (int p = 0; p < NPH; ++p)
#pragma unroll
    for (int mb = 0; mb < MB; ++mb)
#pragma unroll
      for (int nb = 0; nb < NB; ++nb) acc[p][mb][nb] = f32x4{0.f, 0.f, 0.f, 0.f};

  // this lane's B tuples of step s (pixel row mb): T1 = [x1 | x0], T2 = [x0 | x2]
  struct X3 {
    wu32x4 t1, t2;
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
      const unsigned* rec = &smem[lp * PS + kc * 32 + lg * 4];
      dst[mb].t1 = *reinterpret_cast<const wu32x4*>(rec);
      dst[mb].t2 = *reinterpret_cast<const wu32x4*>(rec + 16);
    }
  };

  X3 bx[2][MB];
  load_b(0, bx[0]);
  if constexpr (WLDS) {
#pragma unroll
    for (int nb = 0; nb < NB; ++nb) av[0][nb] = wlds(0, nb);
  }
#pragma unroll
  for (int s = 0; s < NSTEP; ++s) {
    const int tap = s / KC, kc = s % KC;
    const int ky = tap / 3, kx = tap % 3;
    const int c = s & 1;
    if constexpr (WLDS) {
      if (kc == 0 && tap + 1 < 9) wdma(tap + 1, (tap + 1) & 1);
    } else if (s + PF < NSTEP) {
#pragma unroll
      for (int nb = 0; nb < NB; ++nb) av[(s + PF) % (PF + 1)][nb] = wglob(s + PF, nb);
    }
    // the next step's LDS fragments (within a tap: the slot is already resident)
    const bool pre = s + 1 < NSTEP && !(WLDS && kc == KC - 1);
    if (pre) {
      load_b(s + 1, bx[c ^ 1]);
      if constexpr (WLDS) {
#pragma unroll
        for (int nb = 0; nb < NB; ++nb) av[c ^ 1][nb] = wlds(s + 1, nb);
      }
    }
    __builtin_amdgcn_sched_barrier(0);
    const int ph = MODE == MODE_T2 ? (ky == 1 ? 2 : 0) + (kx == 1 ? 1 : 0) : 0;
    const int wi = WLDS ? c : s % (PF + 1);
#pragma unroll
    for (int nb = 0; nb < NB; ++nb) {
      const W3& w = av[wi][nb];
#pragma unroll
      for (int mb = 0; mb < MB; ++mb) {
        const X3& x = bx[c][mb];
        f32x4 v = acc[ph][mb][nb];
        v = mfma_bf(w.t[2], x.t2, v);
        v = mfma_bf(w.t[1], x.t1, v);
        v = mfma_bf(w.t[0], x.t1, v);
        acc[ph][mb][nb] = v;
      }
    }
    __builtin_amdgcn_sched_barrier(0);
    if constexpr (WLDS) {
      if (kc == KC - 1 && tap + 1 < 9) {  // the next tap's slab has landed (one barrier per tap)
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        load_b(s + 1, bx[c ^ 1]);
#pragma unroll
        for (int nb = 0; nb < NB; ++nb) av[c ^ 1][nb] = wlds(s + 1, nb);
      }
    }
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
