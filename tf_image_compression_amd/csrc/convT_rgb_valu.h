// convT_rgb_valu.h — last layer of every decoder (and of the rmbe net) on the vector ALUs:
// stride-2 transposed 3x3 conv Cin -> 3 (basic_block.py:50-71, identity) with the
// denormalise + clip (model_0/model.py:250-259) and np.around -> uint8 (decode.py:249) fused.
//
// Why VALU, not MFMA: per input position the layer computes 4 sub-pixel phases x 3
// channels = 12 outputs from 9 (phase, input offset) pairs x Cin products = 864 MACs at
// Cin = 32.  Every MFMA formulation pads that badly — the dense sub-pixel GEMM
// (convT_rgb_kernel) spends 2048 MAC slots per position (42 % useful: 3 of 4 rows, 9 of
// 16 (phase, offset) blocks), the col2im form needs an LDS reduction pass — while a wave64
// v_fma_f32 with a wave-uniform weight retires 64 useful MACs per 2 cycles per SIMD, the
// f32 MFMA rate.  At 100 % useful work the layer's arithmetic (9 x Cin x 3 x 2 FLOP per
// input position) is of the order of its HBM time (Cin x 4 bytes in, 12 bytes out per
// position), so the kernel is built to stream: one input position per thread, its 2x2
// output pixels staged in LDS and written back as 16-byte row chunks.
//
// Workgroup: TH x TW input positions (TH * TW = 256, one per thread) + one halo row / column
// above / left (input offsets d in {0,-1}: T(0) = {(k=0,d=0), (k=2,d=-1)}, T(1) = {(k=1,d=0)}),
// staged in LDS with pixel stride Cin + 4 floats (== 4 mod 8: the ds_read_b128 of 16
// consecutive positions hits 16 distinct bank slots).  Weights: the TF kernel as-is,
// [3 ky][3 kx][3 co][Cin] float32; the one-shot kernel reads them with wave-uniform
// addresses (scalar loads; many workgroups per CU hide their latency), the persistent one
// stages them once per workgroup in LDS and reads them as broadcast ds_read_b128 (scalar
// loads there share lgkmcnt with the tile's LDS reads and serialise the loop).
// Summation order per output: input offsets (0,0), (0,-1), (-1,0), (-1,-1), Cin ascending
// within each — the same for every TW and both kernels, so every tiling is bit-identical.
// The helpers below are shared with the fused decoder tail.
#pragma once
#include <type_traits>
#include "conv3x3.h"

namespace tic {

// acc[phase][co] += the 9 (phase, offset) products of one input position.  `self` points at
// the position in an LDS tile of pitch PS floats per position and LC positions per row, so
// that offset (-1, 0) is self - LC*PS and (0, -1) is self - PS.  `w` is [3][3][3][CIN].
// rgb_out_fma_g: the same with chunk c4 of offset (dy, dx) loaded by ld(dy, dx, c4); PK
// selects packed fmas (v_pk_fma_f32, whose two weights must sit in an aligned SGPR pair —
// s_mov repacking per instruction) or two interleaved plain v_fma_f32 chains (one SGPR
// operand each).  Weights in global memory (WG) are read through the constant address
// space: wave-uniform scalar loads even where the kernel also stores to global memory
// earlier on the path (the persistent forms), which would otherwise make them vector
// loads; weights staged in LDS (!WG) are read as they are.  Offsets and phases are
// template constants so every acc index is one before any optimisation runs (computed
// indices left acc in scratch in some instantiations).
namespace rgbout {
typedef const __attribute__((address_space(4))) float* cfp;
template <bool WG> using wptr = typename std::conditional<WG, cfp, const float*>::type;
typedef float f32x2 __attribute__((ext_vector_type(2)));

// kernel tap (ky or kx) of phase bit p at input offset d (0 or -1): T(0) = {(0,0), (2,-1)}, T(1) = {(1,0)}
constexpr int tap(int p, int d) { return p ? 1 : (d == 0 ? 0 : 2); }
// phases using offset OFF (py = 0 when dy = -1, px = 0 when dx = -1): 0 -> 0,1,2,3; 1 -> 0,2;
// 2 -> 0,1; 3 -> 0
constexpr int nphase(int off) { return off == 0 ? 4 : off == 3 ? 1 : 2; }
constexpr int phase(int off, int k) { return off == 1 ? 2 * k : k; }

template <int CIN, int OFF, int PA, class W>
__device__ __forceinline__ W wrow(W w, int co) {
  return w + ((tap(PA >> 1, -(OFF >> 1)) * 3 + tap(PA & 1, -(OFF & 1))) * 3 + co) * CIN;
}

// phases PA and PB (PB < 0: PA alone) of one offset, each output's chain ci ascending
template <int CIN, bool PK, int OFF, int PA, int PB, class W>
__device__ __forceinline__ void chains(const float (&x)[CIN], W w, f32x4 (&acc)[4]) {
#pragma unroll
  for (int co = 0; co < 3; ++co) {
    const W wa = wrow<CIN, OFF, PA>(w, co);
    if constexpr (PB < 0) {
#pragma unroll
      for (int ci = 0; ci < CIN; ++ci) acc[PA][co] = fmaf(x[ci], wa[ci], acc[PA][co]);
    } else {
      const W wb = wrow<CIN, OFF, PB>(w, co);
      if constexpr (PK) {
        f32x2 s2 = {acc[PA][co], acc[PB][co]};
#pragma unroll
        for (int ci = 0; ci < CIN; ++ci) {
          const f32x2 xx = {x[ci], x[ci]};
          const f32x2 ww = {wa[ci], wb[ci]};
          s2 = __builtin_elementwise_fma(xx, ww, s2);
        }
        acc[PA][co] = s2.x;
        acc[PB][co] = s2.y;
      } else {
        float sa = acc[PA][co], sb = acc[PB][co];
#pragma unroll
        for (int ci = 0; ci < CIN; ++ci) {
          sa = fmaf(x[ci], wa[ci], sa);
          sb = fmaf(x[ci], wb[ci], sb);
        }
        acc[PA][co] = sa;
        acc[PB][co] = sb;
      }
    }
  }
}

template <int CIN, bool PK, int OFF, class Ld, class W>
__device__ __forceinline__ void offset(Ld& ld, W w, f32x4 (&acc)[4]) {
  float x[CIN];
#pragma unroll
  for (int c4 = 0; c4 < CIN / 4; ++c4) {
    const f32x4 v = ld(-(OFF >> 1), -(OFF & 1), c4);
    x[4 * c4] = v.x;
    x[4 * c4 + 1] = v.y;
    x[4 * c4 + 2] = v.z;
    x[4 * c4 + 3] = v.w;
  }
  // phases paired so one packed fma advances two outputs' chains by one step each — every
  // output's own fma order is unchanged
  if constexpr (nphase(OFF) >= 2) chains<CIN, PK, OFF, phase(OFF, 0), phase(OFF, 1)>(x, w, acc);
  if constexpr (nphase(OFF) == 4) chains<CIN, PK, OFF, phase(OFF, 2), phase(OFF, 3)>(x, w, acc);
  if constexpr (nphase(OFF) == 1) chains<CIN, PK, OFF, 0, -1>(x, w, acc);
}
}  // namespace rgbout

template <int CIN, bool PK = true, bool WG = true, class Ld>
__device__ __forceinline__ void rgb_out_fma_g(Ld ld, const float* __restrict__ wg, f32x4 (&acc)[4]) {
  const rgbout::wptr<WG> w = (rgbout::wptr<WG>)wg;
  rgbout::offset<CIN, PK, 0>(ld, w, acc);
  rgbout::offset<CIN, PK, 1>(ld, w, acc);
  rgbout::offset<CIN, PK, 2>(ld, w, acc);
  rgbout::offset<CIN, PK, 3>(ld, w, acc);
}

template <int CIN, int PS, int LC, bool WG = true>
__device__ __forceinline__ void rgb_out_fma(const float* self, const float* __restrict__ w, f32x4 (&acc)[4]) {
  rgb_out_fma_g<CIN, true, WG>(
      [&](int dy, int dx, int c4) { return *reinterpret_cast<const f32x4*>(self + (dy * LC + dx) * PS + 4 * c4); }, w,
      acc);
}

// + bias, * std + mean, clip -> LDS output tile row-major [.][OW] f32 at output pixel
// (2r + py, 2c + px).
__device__ __forceinline__ void rgb_out_epilogue(const RgbOutArgs& a, const f32x4 (&acc)[4], float* lout,
                                                 int OW, int r, int c) {
#pragma unroll
  for (int ph = 0; ph < 4; ++ph) {
    const int py = ph >> 1, px = ph & 1;
#pragma unroll
    for (int co = 0; co < 3; ++co) {
      const float v = __fadd_rn(acc[ph][co], a.bias[co]);
      float d = __fadd_rn(__fmul_rn(v, a.std[co]), a.mean[co]);
      d = fminf(fmaxf(d, 0.f), 255.f);
      lout[(2 * r + py) * OW + (2 * c + px) * 3 + co] = d;
    }
  }
}

// Write the staged output tile (2TH x 2TW pixels at input origin (gy0, gx0) of image nimg):
// whole 16-byte row chunks when the tile is interior and aligned, else element-wise.
template <int TH, int TW, int NT>
__device__ __forceinline__ void rgb_out_store(const RgbOutArgs& a, const float* lout, int tid, int gy0, int gx0,
                                              int nimg) {
  constexpr int OW = 2 * TW * 3;  // floats per output tile row
  const int Ho = 2 * a.H, Wo = 2 * a.W;
  const int oy0 = 2 * gy0, ox0 = 2 * gx0;
  const int rows = min(2 * TH, Ho - oy0), cols = min(2 * TW, Wo - ox0);
  const size_t row_base = ((size_t)nimg * Ho + oy0) * Wo + ox0;  // pixel index of the tile origin
  const bool full = cols == 2 * TW;
  if (a.out_u8) {
    const bool vec = full && ((Wo * 3) % 16 == 0) && ((ox0 * 3) % 16 == 0) && ((uintptr_t)a.out_u8 % 16 == 0);
    if (vec) {
      constexpr int CH = OW / 16;  // 16-byte chunks per tile row (OW u8 bytes)
      for (int e = tid; e < rows * CH; e += NT) {
        const int rr = e / CH, ch = e % CH;
        const float* s = &lout[rr * OW + ch * 16];
        uint32_t wv[4];
#pragma unroll
        for (int k = 0; k < 4; ++k)
          wv[k] = (uint32_t)rintf(s[4 * k]) | ((uint32_t)rintf(s[4 * k + 1]) << 8) |
                  ((uint32_t)rintf(s[4 * k + 2]) << 16) | ((uint32_t)rintf(s[4 * k + 3]) << 24);
        *reinterpret_cast<uint4*>(a.out_u8 + (row_base + (size_t)rr * Wo) * 3 + ch * 16) =
            make_uint4(wv[0], wv[1], wv[2], wv[3]);
      }
    } else {
      for (int e = tid; e < rows * cols * 3; e += NT) {
        const int rr = e / (cols * 3), k = e % (cols * 3);
        a.out_u8[(row_base + (size_t)rr * Wo) * 3 + k] = (uint8_t)rintf(lout[rr * OW + k]);
      }
    }
  }
  if (a.out_f32) {
    const bool vec = full && ((Wo * 3) % 4 == 0) && ((ox0 * 3) % 4 == 0) && ((uintptr_t)a.out_f32 % 16 == 0);
    if (vec) {
      constexpr int CH = OW / 4;  // 16-byte chunks per tile row (OW floats)
      for (int e = tid; e < rows * CH; e += NT) {
        const int rr = e / CH, ch = e % CH;
        *reinterpret_cast<f32x4*>(a.out_f32 + (row_base + (size_t)rr * Wo) * 3 + ch * 4) =
            *reinterpret_cast<const f32x4*>(&lout[rr * OW + ch * 4]);
      }
    } else {
      for (int e = tid; e < rows * cols * 3; e += NT) {
        const int rr = e / (cols * 3), k = e % (cols * 3);
        a.out_f32[(row_base + (size_t)rr * Wo) * 3 + k] = lout[rr * OW + k];
      }
    }
  }
}

// The raw [3][3][3][CIN] kernel into LDS (16-byte aligned source: a device allocation).
template <int CIN, int NT>
__device__ __forceinline__ void rgb_out_load_weights(const float* __restrict__ wraw, float* wsh, int tid) {
  for (int e = tid; e < 27 * CIN / 4; e += NT)
    reinterpret_cast<f32x4*>(wsh)[e] = reinterpret_cast<const f32x4*>(wraw)[e];
}

template <int CIN, int TW>
__global__ void __launch_bounds__(256) convT_rgb_valu_kernel(const RgbOutArgs a) {
  static_assert(CIN % 4 == 0 && 256 % TW == 0, "tile");
  constexpr int TH = 256 / TW;
  constexpr int PS = CIN + 4;
  constexpr int LR = TH + 1, LC = TW + 1, C4 = CIN / 4;
  constexpr int IN_FLOATS = LR * LC * PS;
  constexpr int OUT_FLOATS = 2 * TH * 2 * TW * 3;  // f32 staging of the output tile
  __shared__ __attribute__((aligned(16))) float lds[IN_FLOATS > OUT_FLOATS ? IN_FLOATS : OUT_FLOATS];

  const int tid = threadIdx.x;
  const int gx0 = blockIdx.x * TW, gy0 = blockIdx.y * TH, nimg = blockIdx.z;
  const int H = a.H, W = a.W;
  const float* __restrict__ in = a.in;

  // ---- stage input positions (gy0-1 .. gy0+TH-1) x (gx0-1 .. gx0+TW-1), zero outside ----
  constexpr int NSTAGE = LR * LC * C4;
  constexpr int NIT = (NSTAGE + 255) / 256;
  constexpr int SB = NIT < 16 ? NIT : 16;
#pragma unroll
  for (int i0 = 0; i0 < NIT; i0 += SB) {
    f32x4 tmp[SB];
#pragma unroll
    for (int i = 0; i < SB; ++i) {
      const int e = (i0 + i) * 256 + tid;
      tmp[i] = f32x4{0.f, 0.f, 0.f, 0.f};
      if (i0 + i < NIT && e < NSTAGE) {
        const int c4 = e % C4, pe = e / C4, col = pe % LC, row = pe / LC;
        const int iy = gy0 - 1 + row, ix = gx0 - 1 + col;
        if (iy >= 0 && iy < H && ix >= 0 && ix < W)
          tmp[i] = *reinterpret_cast<const f32x4*>(in + ((size_t)(nimg * H + iy) * W + ix) * CIN + c4 * 4);
      }
    }
#pragma unroll
    for (int i = 0; i < SB; ++i) {
      const int e = (i0 + i) * 256 + tid;
      if (i0 + i < NIT && e < NSTAGE)
        *reinterpret_cast<f32x4*>(&lds[(e / C4) * PS + (e % C4) * 4]) = tmp[i];
    }
  }
  __syncthreads();

  const int r = tid / TW, c = tid % TW;
  f32x4 acc[4] = {};  // [phase][co], lane 3 unused
  rgb_out_fma<CIN, PS, LC>(&lds[((r + 1) * LC + (c + 1)) * PS], a.wraw, acc);
  __syncthreads();  // input tile no longer needed: reuse LDS for the output tile
  rgb_out_epilogue(a, acc, lds, 2 * TW * 3, r, c);
  __syncthreads();
  rgb_out_store<TH, TW, 256>(a, lds, tid, gy0, gx0, nimg);
}

// ---------------------------------------------------------------------------------------
// Persistent, software-pipelined variant: grid = min(tiles, 2 x CUs); each workgroup walks
// tiles t, t + grid, ...  The global loads of the NEXT tile are issued into registers
// right after this tile's inputs land in LDS, so they fly while this tile computes and
// writes back (the one-shot kernel's workgroups all load, then all compute, then all
// store in lock-step, which leaves HBM idle half the time).  Weights sit in LDS for the
// workgroup's lifetime.  Same arithmetic, same order: bit-identical to
// convT_rgb_valu_kernel.
// ---------------------------------------------------------------------------------------
template <int CIN, int TW>
__global__ void __launch_bounds__(256) convT_rgb_valu_persist_kernel(const RgbOutArgs a, int ntx, int nty,
                                                                     int ntiles) {
  constexpr int TH = 256 / TW;
  constexpr int PS = CIN + 4;
  constexpr int LR = TH + 1, LC = TW + 1, C4 = CIN / 4;
  constexpr int IN_FLOATS = LR * LC * PS;
  constexpr int OW = 2 * TW * 3;
  constexpr int OUT_FLOATS = 2 * TH * OW;
  constexpr int NSTAGE = LR * LC * C4;
  constexpr int NIT = (NSTAGE + 255) / 256;
  __shared__ __attribute__((aligned(16))) float smem[IN_FLOATS + OUT_FLOATS + 27 * CIN];
  float* const lin = smem;
  float* const lout = smem + IN_FLOATS;
  float* const wsh = smem + IN_FLOATS + OUT_FLOATS;

  const int tid = threadIdx.x;
  const int H = a.H, W = a.W;
  const float* __restrict__ in = a.in;
  const int r = tid / TW, c = tid % TW;

  f32x4 pre[NIT];
  auto issue = [&](int t) {
    const int gx0 = (t % ntx) * TW, gy0 = ((t / ntx) % nty) * TH, nimg = t / (ntx * nty);
#pragma unroll
    for (int i = 0; i < NIT; ++i) {
      const int e = i * 256 + tid;
      pre[i] = f32x4{0.f, 0.f, 0.f, 0.f};
      if (NSTAGE % 256 == 0 || e < NSTAGE) {
        const int c4 = e % C4, pe = e / C4, col = pe % LC, row = pe / LC;
        const int iy = gy0 - 1 + row, ix = gx0 - 1 + col;
        if (iy >= 0 && iy < H && ix >= 0 && ix < W)
          pre[i] = *reinterpret_cast<const f32x4*>(in + ((size_t)(nimg * H + iy) * W + ix) * CIN + c4 * 4);
      }
    }
  };

  int t = blockIdx.x;
  if (t >= ntiles) return;
  issue(t);
  rgb_out_load_weights<CIN, 256>(a.wraw, wsh, tid);
  for (; t < ntiles; t += gridDim.x) {
#pragma unroll
    for (int i = 0; i < NIT; ++i) {
      const int e = i * 256 + tid;
      if (NSTAGE % 256 == 0 || e < NSTAGE) *reinterpret_cast<f32x4*>(&lin[(e / C4) * PS + (e % C4) * 4]) = pre[i];
    }
    __syncthreads();
    if (t + (int)gridDim.x < ntiles) issue(t + gridDim.x);

    f32x4 acc[4] = {};  // [phase][co], lane 3 unused
    rgb_out_fma<CIN, PS, LC, false>(&lin[((r + 1) * LC + (c + 1)) * PS], wsh, acc);
    rgb_out_epilogue(a, acc, lout, OW, r, c);
    __syncthreads();

    const int gx0 = (t % ntx) * TW, gy0 = ((t / ntx) % nty) * TH, nimg = t / (ntx * nty);
    rgb_out_store<TH, TW, 256>(a, lout, tid, gy0, gx0, nimg);
  }
}

}  // namespace tic
