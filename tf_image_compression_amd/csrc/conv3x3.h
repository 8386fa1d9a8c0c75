// conv3x3.h — gfx950 (CDNA4) kernels for the 3x3 convolution stacks of the codec.
//
// One implicit-GEMM template covers every layer with Cin, Cout multiples of 16:
//   MODE_S1  tf.nn.conv2d stride 1 'SAME'       (basic_block/basic_block.py:33)
//   MODE_S2  tf.nn.conv2d stride 2 'SAME'       (pad_before = 0, pad_after = 1 on even input)
//   MODE_T2  tf.nn.conv2d_transpose stride 2 'SAME', output 2Hx2W (basic_block.py:54-57),
//            computed as its four sub-pixel phases: y[2m+p] = sum_{(k,d) in T(p)} x[m+d] W[k],
//            T(0) = {(0,0),(2,-1)}, T(1) = {(1,0)} — no zero-insertion, no wasted MACs.
// with the epilogue of my_conv2d fused: + bias, ReLU/identity, + residual (res_block,
// basic_block.py:91), and optionally the quantiser (model_0/model.py:136-138) writing u8
// symbols; the dequantiser LUT (model_0/model.py:153) is fused into the input staging.
//
// Matrix core: v_mfma_f32_16x16x4_f32 (exact fp32 fma chain, 64 FLOP/clk/SIMD — the fp32
// peak of the chip).  GEMM orientation: M = 16 output channels (A = weights),
// N = 16 output pixels along x (B = activations), K = input channels.  Each lane keeps
// 4 consecutive output channels of one pixel -> 16-byte NHWC stores.
//
// K ordering: a 16-channel chunk is consumed by 4 MFMAs; lane group g = lane>>4 supplies
// channel 4g+t to MFMA t, so ONE ds_read_b128 (activations) and ONE global_load_dwordx4
// (weights) per lane feed four MFMAs.  Weights are repacked at load time to
// [tap][Cin/16][Cout][4 (g)][4 (t)] so a wave's A fragment is one contiguous 1 KiB read.
//
// LDS: the block's input tile (with halo) is staged once, pixel stride PS = Cin + 8
// floats (== 8 mod 16): the ds_read_b128 of 16 consecutive pixels x 4 channel groups hits
// 16 distinct 16-byte bank slots in every lane group -> conflict-free.  Stride-2 tiles are
// stored column-deinterleaved (even / odd planes) so a block of 16 consecutive output
// pixels again reads 16 consecutive LDS pixels.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "tic_kernels.h"

namespace tic {

__device__ __forceinline__ f32x4 mfma4(float a, float b, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
}

// Packed-weight fragment loads through a raw buffer resource: the descriptor lives in SGPRs,
// the lane's byte offset in one VGPR and the K step's byte offset in the instruction's
// soffset / immediate — no 64-bit address add per load. At f32 MFMA every VALU instruction
// adds to the matrix time of the SIMD (probe_mfma_valu_r04.txt), so the
// address math the pointer form needs per load is paid in MFMA throughput.
typedef unsigned int wu32x4 __attribute__((ext_vector_type(4)));
__device__ __forceinline__ __amdgpu_buffer_rsrc_t weight_rsrc(const float* base, int bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(base), (short)0, bytes, 0x00020000);
}
__device__ __forceinline__ f32x4 weight_frag(__amdgpu_buffer_rsrc_t r, int lane_byte, int step_byte) {
  const wu32x4 u = __builtin_amdgcn_raw_buffer_load_b128(r, lane_byte, step_byte, 0);
  return f32x4{__uint_as_float(u.x), __uint_as_float(u.y), __uint_as_float(u.z), __uint_as_float(u.w)};
}

// XCD-aware block order (MI355X_MICROARCH.md: blocks b and b + 8 are dealt to one XCD):
// logical tile b' = (b % 8) * (N / 8) + b / 8, so each XCD walks a contiguous run of tiles —
// x fastest, then the next tile row — and a tile's halo rows, which the tile above read a
// moment earlier on the same XCD, come from that XCD's L2 instead of HBM.  Placement only:
// every tile computes exactly what it did.  (N not a multiple of 8: identity.)
__device__ __forceinline__ void xcd_tile(int& bx, int& by, int& bz) {
  const unsigned gx = gridDim.x, gy = gridDim.y, n = gx * gy * gridDim.z;
  unsigned b = blockIdx.x + gx * (blockIdx.y + gy * blockIdx.z);
  if ((n & 7u) == 0) b = (b & 7u) * (n >> 3) + (b >> 3);
  bx = (int)(b % gx);
  by = (int)((b / gx) % gy);
  bz = (int)(b / (gx * gy));
}

// Quantiser: round_half_even(sigmoid(v) * (Q-1)), clamped to [0, Q-1].
__device__ __forceinline__ uint32_t quant1(float v, float qscale) {
  float s = 1.0f / (1.0f + expf(-v));
  float q = rintf(__fmul_rn(s, qscale));
  q = fminf(fmaxf(q, 0.0f), qscale);
  return (uint32_t)q;
}

template <int MODE, int TH>
struct TileGeom {
  // LDS rows / entries per row of the staged input tile (TW = 16 output pixels wide)
  static constexpr int LR = MODE == MODE_S1 ? TH + 2 : (MODE == MODE_S2 ? 2 * TH + 1 : TH + 1);
  static constexpr int LC = MODE == MODE_S1 ? 18 : (MODE == MODE_S2 ? 34 : 17);
};

typedef __attribute__((address_space(3))) void* lds_ptr_t;

// Grid: x = ceil(Wg/16) * NSPLIT, y = ceil(Hg/TH), z = batch, where (Hg,Wg) is the
// output grid (S1/S2) or the input grid (T2).  NSPLIT workgroups share a pixel tile and
// split the output channels.  256 threads = 4 waves = WR row-groups x (4/WR) channel
// groups; each wave owns MB = TH/WR rows of 16 pixels x NB channel blocks of 16
// (x 4 phases for T2).
//
// The K loop is a flat, fully unrolled list of steps, tap-major for every mode (step =
// one 16-channel chunk of one 3x3 tap), so every tiling accumulates each output in the
// same fma order (results are bit-identical across tilings).  Weights are packed
// [tap][Cin/16][4 g][Cout][4 t]; their A fragments come either
//   WSRC=0: straight from L2 into registers, prefetched PF = 2 steps ahead,
//   WSRC=2: the same with PF = 6 (small grids run ~1 wave per SIMD, so the prefetch
//           alone has to cover the L2 latency), or
//   WSRC=1: from a 2-slot LDS ring holding one tap's slab for this workgroup's
//           channels, filled by LDS-DMA (global_load_lds_dwordx4) one tap ahead and
//           shared by the 4 waves (one barrier per tap).
template <int MODE, int CIN, int COUT, int TH, int WR, int NSPLIT, int WSRC, int ACT, bool RES, int IN, int OUT>
__global__ void __launch_bounds__(256) conv3x3_kernel(const ConvArgs a) {
  constexpr bool WLDS = WSRC == 1;
  static_assert(CIN % 16 == 0 && COUT % 16 == 0, "channels must be multiples of 16");
  constexpr int PS = CIN + 8;
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
  constexpr int TILE = LR * LC * PS;            // floats of the input tile
  constexpr int WSLAB = CIN * COUT_WG;          // floats of one tap's weights for this WG
  constexpr int WCHUNK = WSLAB / 4;             // 16-byte chunks per slab (multiple of 64)

  // ONE __shared__ array (a second object can make hipcc drain the LDS-DMA early)
  __shared__ __attribute__((aligned(16))) float smem[TILE + (WLDS ? 2 * WSLAB : 0)];
  float* const lds = smem;

  const int tid = threadIdx.x;
  const int split = NSPLIT > 1 ? (int)(blockIdx.x % NSPLIT) : 0;
  const int gx0 = (NSPLIT > 1 ? (int)(blockIdx.x / NSPLIT) : (int)blockIdx.x) * 16;
  const int gy0 = blockIdx.y * TH;
  const int nimg = blockIdx.z;
  const int H = a.H, W = a.W;

  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);  // wave-uniform (SGPR)
  const int lane = tid & 63;
  const int wr = wave / WC;
  const int wc = wave % WC;
  const int li = lane & 15;  // pixel within the 16-pixel block (B col / D col)
  const int lg = lane >> 4;  // k group (A/B) / output channel quad (D)
  const int co_wg = split * COUT_WG;      // first output channel of this workgroup
  const int co_wave = wc * NB * 16;       // first channel of this wave inside the WG

  // ---- weight source ----
#ifndef CONV_RSRC_STAGE
#define CONV_RSRC_STAGE 1
#endif
  const __amdgpu_buffer_rsrc_t wrs_dma = weight_rsrc(a.wp, 9 * CIN * COUT * 4);
  auto wdma = [&](int tap, int slot) {  // LDS-DMA one tap slab: [kc][g][co_local][4]
#pragma unroll
    for (int j = 0; j < (WCHUNK + 255) / 256; ++j) {
      const int cbase = (j * 4 + wave) * 64;  // wave-uniform first chunk
      if (WCHUNK % 256 == 0 || cbase < WCHUNK) {
        const int c = cbase + lane;
        const int col = c % COUT_WG, kg = c / COUT_WG;  // kg = kc*4 + g
#if CONV_RSRC_STAGE
        // through the weights' buffer resource: 32-bit lane offset, the tap's offset in an SGPR
        __builtin_amdgcn_raw_ptr_buffer_load_lds(wrs_dma, (lds_ptr_t)(smem + TILE + slot * WSLAB + cbase * 4), 16,
                                                 ((kg * COUT + co_wg + col) * 4) * 4, tap * KC * 4 * COUT * 16, 0, 0);
#else
        const float* src = a.wp + ((size_t)(tap * KC * 4 + kg) * COUT + co_wg + col) * 4;
        __builtin_amdgcn_global_load_lds(src, (lds_ptr_t)(smem + TILE + slot * WSLAB + cbase * 4), 16, 0, 0);
#endif
      }
    }
  };
  const __amdgpu_buffer_rsrc_t wrs = weight_rsrc(a.wp, 9 * CIN * COUT * 4);
  const int wlb = (lg * COUT + co_wg + co_wave + li) * 16;  // lane byte offset
  auto wglob = [&](int s, int nb) -> f32x4 {
    const int tap = s / KC, kc = s % KC;
    return weight_frag(wrs, wlb, ((tap * KC + kc) * 4 * COUT * 4 + nb * 64) * 4);
  };

  constexpr int PF = WSRC == 2 ? 6 : 2;  // register prefetch distance (L2 sources)
  f32x4 av[WLDS ? 1 : PF + 1][NB];
  if constexpr (WLDS) {
    wdma(0, 0);
  } else {
#pragma unroll
    for (int p = 0; p < PF; ++p)
#pragma unroll
      for (int nb = 0; nb < NB; ++nb)
        if (p < NSTEP) av[p][nb] = wglob(p, nb);
  }

  // ---- stage the input tile (with halo) into LDS; zero outside the image (SAME pad) ----
  // A thread's global loads are all issued before its first LDS write (batches of <= SB).
  // f32 inputs go through a buffer resource over this patch (32-bit byte offsets; a position
  // outside the image gets an offset past the resource's end, which the hardware reads as
  // zero): no 64-bit address, zero-initialisation or branch per chunk — the staging VALU was
  // ~60 % of encode_2's non-MFMA VALU (tools/isa_mix.py), and at f32 that VALU adds to the
  // matrix time of the workgroups sharing the SIMD.  Patches of 4 GB or more
  // (never at the shipped sizes) keep the pointer form.
  constexpr int NSTAGE = LR * LC * C4;
  constexpr int NIT = (NSTAGE + 255) / 256;
  constexpr int SB = NIT < 12 ? NIT : 12;
  const size_t img_bytes = (size_t)H * W * CIN * 4;
  const bool rsrc_in = CONV_RSRC_STAGE && IN == IN_F32 && img_bytes < 0xFFFFFF00ull;
  const __amdgpu_buffer_rsrc_t irs =
      weight_rsrc(reinterpret_cast<const float*>(a.in) + (rsrc_in ? (size_t)nimg * H * W * CIN : 0),
                  (int)(unsigned)(rsrc_in ? img_bytes : 16));
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
        const bool inside = iy >= 0 && iy < H && ix >= 0 && ix < W;
        if (IN == IN_F32 && rsrc_in) {
          const unsigned off = inside ? ((unsigned)(iy * W + ix) * CIN + c4 * 4) * 4u : 0xFFFFFFF0u;
          tmp[i] = weight_frag(irs, (int)off, 0);
        } else if (inside) {
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
        *reinterpret_cast<f32x4*>(&lds[pe * PS + c4 * 4]) = tmp[i];
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

  // fragment loaders for step s (tap-major: tap = s / KC, kc = s % KC)
  auto load_b = [&](int s, f32x4* dst) {
    const int tap = s / KC, kc = s % KC;
    const int ky = tap / 3, kx = tap % 3;
#pragma unroll
    for (int mb = 0; mb < MB; ++mb) {
      const int r = wr * MB + mb;
      int lp;
      if constexpr (MODE == MODE_S1) lp = (r + ky) * LC + li + kx;
      else if constexpr (MODE == MODE_S2) lp = (2 * r + ky) * LC + (kx & 1) * 17 + li + (kx >> 1);
      else lp = (r + 1 - (ky == 2)) * LC + li + 1 - (kx == 2);  // T2: input offset (-(ky==2), -(kx==2))
      dst[mb] = *reinterpret_cast<const f32x4*>(&lds[lp * PS + kc * 16 + lg * 4]);
    }
  };
  auto load_a_lds = [&](int s, f32x4* dst) {
    const int tap = s / KC, kc = s % KC;
#pragma unroll
    for (int nb = 0; nb < NB; ++nb)
      dst[nb] = *reinterpret_cast<const f32x4*>(
          &smem[TILE + (tap & 1) * WSLAB + ((kc * 4 + lg) * COUT_WG + co_wave + nb * 16 + li) * 4]);
  };

  // register double buffer of the LDS fragments: step s+1's ds_reads are in flight while
  // step s's MFMAs issue (except across a WLDS tap boundary, which needs the barrier).
  f32x4 bq[2][MB];
  f32x4 aq[2][WLDS ? NB : 1];
  load_b(0, bq[0]);
  if constexpr (WLDS) load_a_lds(0, aq[0]);
#pragma unroll
  for (int s = 0; s < NSTEP; ++s) {
    const int tap = s / KC, kc = s % KC;
    const int ky = tap / 3, kx = tap % 3;
    const int c = s & 1;
    if constexpr (WLDS) {
      if (kc == 0 && tap + 1 < 9) wdma(tap + 1, (tap + 1) & 1);
    } else {
      if (s + PF < NSTEP) {
#pragma unroll
        for (int nb = 0; nb < NB; ++nb) av[(s + PF) % (PF + 1)][nb] = wglob(s + PF, nb);
      }
    }
    const bool pre = s + 1 < NSTEP && !(WLDS && kc == KC - 1);
    if (pre) {
      load_b(s + 1, bq[c ^ 1]);
      if constexpr (WLDS) load_a_lds(s + 1, aq[c ^ 1]);
    }
    // keep the next step's ds_reads above this step's MFMAs (hipcc otherwise sinks them
    // below to reuse registers and then waits lgkmcnt(0) right before the next MFMAs)
    __builtin_amdgcn_sched_barrier(0);
    // T2: tap (ky,kx) feeds output phase 2*(ky==1) + (kx==1)
    const int ph = MODE == MODE_T2 ? (ky == 1 ? 2 : 0) + (kx == 1 ? 1 : 0) : 0;
#pragma unroll
    for (int t = 0; t < 4; ++t)
#pragma unroll
      for (int mb = 0; mb < MB; ++mb)
#pragma unroll
        for (int nb = 0; nb < NB; ++nb) {
          const float aval = WLDS ? aq[c][WLDS ? nb : 0][t] : av[s % (PF + 1)][nb][t];
          acc[ph][mb][nb] = mfma4(aval, bq[c][mb][t], acc[ph][mb][nb]);
        }
    __builtin_amdgcn_sched_barrier(0);
    if constexpr (WLDS) {
      if (kc == KC - 1 && tap + 1 < 9) {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        load_b(s + 1, bq[c ^ 1]);
        load_a_lds(s + 1, aq[c ^ 1]);
      }
    }
  }

  // ---- fused epilogue: + bias, act, + residual, store f32 or quantise to u8 ----
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

// ---------------------------------------------------------------------------------------
// First layer: stride-2 3x3 conv from 3-channel RGB (u8 or f32) with the normalisation
// (x - mean) / std (model_0/model.py:44) fused into the LDS staging.  K = 27 (+1 zero)
// = 7 MFMA k-steps; lane group g supplies k = 4t + g -> (tap, channel) = divmod(k, 3).
// Weights packed [Cout][4 (g)][8 (t, t=7 zero)].
// ---------------------------------------------------------------------------------------

template <int COUT, int TH, bool U8>
__global__ void __launch_bounds__(256) conv_rgb_s2_kernel(const RgbInArgs a) {
  constexpr int NBT = COUT / 16;
  constexpr int MB = TH / 4;  // 4 waves split rows
  constexpr int LR = 2 * TH + 1, LC = 34;
  constexpr int PLANE = LR * LC;
  __shared__ float lds[3 * PLANE];

  const int tid = threadIdx.x;
  const int gx0 = blockIdx.x * 16, gy0 = blockIdx.y * TH, nimg = blockIdx.z;
  const int H = a.H, W = a.W;
  for (int e = tid; e < PLANE; e += 256) {
    const int col = e % LC, row = e / LC;
    const int plane = col >= 17 ? 1 : 0;
    const int iy = 2 * gy0 + row - a.pad_y, ix = 2 * gx0 + 2 * (col - plane * 17) + plane - a.pad_x;
    float v0 = 0.f, v1 = 0.f, v2 = 0.f;
    if (iy >= 0 && iy < H && ix >= 0 && ix < W) {
      const size_t off = ((size_t)(nimg * H + iy) * W + ix) * 3;
      float x0, x1, x2;
      if constexpr (U8) {
        const uint8_t* p = reinterpret_cast<const uint8_t*>(a.in) + off;
        x0 = p[0];
        x1 = p[1];
        x2 = p[2];
      } else {
        const float* p = reinterpret_cast<const float*>(a.in) + off;
        x0 = p[0];
        x1 = p[1];
        x2 = p[2];
      }
      v0 = __fdiv_rn(__fsub_rn(x0, a.mean[0]), a.std[0]);
      v1 = __fdiv_rn(__fsub_rn(x1, a.mean[1]), a.std[1]);
      v2 = __fdiv_rn(__fsub_rn(x2, a.mean[2]), a.std[2]);
    }
    lds[e] = v0;
    lds[PLANE + e] = v1;
    lds[2 * PLANE + e] = v2;
  }
  __syncthreads();

  const int wave = tid >> 6, lane = tid & 63;
  const int li = lane & 15, lg = lane >> 4;
  f32x4 acc[MB][NBT];
#pragma unroll
  for (int mb = 0; mb < MB; ++mb)
#pragma unroll
    for (int nb = 0; nb < NBT; ++nb) acc[mb][nb] = f32x4{0.f, 0.f, 0.f, 0.f};

  f32x4 w0[NBT], w1[NBT];
#pragma unroll
  for (int nb = 0; nb < NBT; ++nb) {
    const float* wq = a.wp + ((nb * 16 + li) * 4 + lg) * 8;
    w0[nb] = *reinterpret_cast<const f32x4*>(wq);
    w1[nb] = *reinterpret_cast<const f32x4*>(wq + 4);
  }
#pragma unroll
  for (int t = 0; t < 7; ++t) {
    const int k = 4 * t + lg;  // lane-dependent (tap, channel)
    const int tap = k / 3, c = k - 3 * (k / 3);
    const int ky = tap / 3, kx = tap - 3 * (tap / 3);
#pragma unroll
    for (int mb = 0; mb < MB; ++mb) {
      const int r = wave * MB + mb;
      float b = 0.f;
      if (k < 27) b = lds[c * PLANE + (2 * r + ky) * LC + (kx & 1) * 17 + li + (kx >> 1)];
#pragma unroll
      for (int nb = 0; nb < NBT; ++nb) {
        const float av = t < 4 ? w0[nb][t & 3] : w1[nb][t & 3];
        acc[mb][nb] = mfma4(av, b, acc[mb][nb]);
      }
    }
  }
#pragma unroll
  for (int mb = 0; mb < MB; ++mb) {
    const int oy = gy0 + wave * MB + mb, ox = gx0 + li;
    if (oy >= a.Ho || ox >= a.Wo) continue;
#pragma unroll
    for (int nb = 0; nb < NBT; ++nb) {
      const int co = nb * 16 + lg * 4;
      const f32x4 bb = *reinterpret_cast<const f32x4*>(a.bias + co);
      f32x4 v = acc[mb][nb];
      v.x = fmaxf(__fadd_rn(v.x, bb.x), 0.f);
      v.y = fmaxf(__fadd_rn(v.y, bb.y), 0.f);
      v.z = fmaxf(__fadd_rn(v.z, bb.z), 0.f);
      v.w = fmaxf(__fadd_rn(v.w, bb.w), 0.f);
      *reinterpret_cast<f32x4*>(a.out + ((size_t)(nimg * a.Ho + oy) * a.Wo + ox) * COUT + co) = v;
    }
  }
}

// ---------------------------------------------------------------------------------------
// Last layer: stride-2 transpose conv Cin -> 3 (identity) with denormalise + clip
// (model_0/model.py:250-259) and the host's np.around -> uint8 (decode.py:249) fused.
// Dense sub-pixel GEMM: M = 16 rows = 4 phases x (3 channels + 1 pad), K = 4 input offsets
// x Cin, N = 16 input positions; weights [off][Cin/16][16 rows][4][4] with zeros where a
// phase does not use an offset.  Lane (li, g) ends with phase g, channels 0..2 of pixel li.
// ---------------------------------------------------------------------------------------

template <int CIN, int TH>
__global__ void __launch_bounds__(256) convT_rgb_kernel(const RgbOutArgs a) {
  constexpr int PS = CIN + 8, KC = CIN / 16, C4 = CIN / 4;
  constexpr int LR = TH + 1, LC = 17;
  constexpr int MB = TH / 4;
  __shared__ __attribute__((aligned(16))) float lds[LR * LC * PS];

  const int tid = threadIdx.x;
  const int gx0 = blockIdx.x * 16, gy0 = blockIdx.y * TH, nimg = blockIdx.z;
  const int H = a.H, W = a.W;
  for (int e = tid; e < LR * LC * C4; e += 256) {
    const int c4 = e % C4, pe = e / C4, col = pe % LC, row = pe / LC;
    const int iy = gy0 - 1 + row, ix = gx0 - 1 + col;
    f32x4 v = {0.f, 0.f, 0.f, 0.f};
    if (iy >= 0 && iy < H && ix >= 0 && ix < W)
      v = *reinterpret_cast<const f32x4*>(a.in + ((size_t)(nimg * H + iy) * W + ix) * CIN + c4 * 4);
    *reinterpret_cast<f32x4*>(&lds[(row * LC + col) * PS + c4 * 4]) = v;
  }
  __syncthreads();

  const int wave = tid >> 6, lane = tid & 63;
  const int li = lane & 15, lg = lane >> 4;
  f32x4 acc[MB];
#pragma unroll
  for (int mb = 0; mb < MB; ++mb) acc[mb] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int off = 0; off < 4; ++off) {
    const int dy = -(off >> 1), dx = -(off & 1);
#pragma unroll
    for (int kc = 0; kc < KC; ++kc) {
      const f32x4 av = *reinterpret_cast<const f32x4*>(a.wp + ((off * KC + kc) * 16 + li) * 16 + lg * 4);
#pragma unroll
      for (int mb = 0; mb < MB; ++mb) {
        const int r = wave * MB + mb;
        const f32x4 bv = *reinterpret_cast<const f32x4*>(&lds[((r + 1 + dy) * LC + li + 1 + dx) * PS + kc * 16 + lg * 4]);
#pragma unroll
        for (int t = 0; t < 4; ++t) acc[mb] = mfma4(av[t], bv[t], acc[mb]);
      }
    }
  }
  const int Ho = 2 * H, Wo = 2 * W;
#pragma unroll
  for (int mb = 0; mb < MB; ++mb) {
    const int m = gy0 + wave * MB + mb, q = gx0 + li;
    if (m >= H || q >= W) continue;
    const int oy = 2 * m + (lg >> 1), ox = 2 * q + (lg & 1);
    const size_t o = ((size_t)(nimg * Ho + oy) * Wo + ox) * 3;
    float y[3];
#pragma unroll
    for (int c = 0; c < 3; ++c) {
      const float v = __fadd_rn(acc[mb][c], a.bias[c]);
      float d = __fadd_rn(__fmul_rn(v, a.std[c]), a.mean[c]);
      d = fminf(fmaxf(d, 0.f), 255.f);
      y[c] = d;
    }
    if (a.out_f32) {
      a.out_f32[o] = y[0];
      a.out_f32[o + 1] = y[1];
      a.out_f32[o + 2] = y[2];
    }
    if (a.out_u8) {
      a.out_u8[o] = (uint8_t)rintf(y[0]);
      a.out_u8[o + 1] = (uint8_t)rintf(y[1]);
      a.out_u8[o + 2] = (uint8_t)rintf(y[2]);
    }
  }
}

// ---------------------------------------------------------------------------------------
// Last layer, scatter (col2im) form: per input position (m,q) the 27 partial products
// P[(ky,kx,co)] = sum_ci x[m,q,ci] W[ky,kx,co,ci] come from MFMA (M = 32 rows = 27 used,
// K = Cin, N = 16 positions), land in LDS, and each output pixel (2m+py, 2q+px) sums the
// 1, 2 or 4 partials of its phase: py=0 <- (ky=0 @ m, ky=2 @ m-1), py=1 <- (ky=1 @ m),
// likewise in x.  The tile carries one halo row/column of positions at the top/left.
// Then + bias, denormalise, clip, round -> u8 (and/or f32), 4 output pixels per thread.
// Weights packed [rb 2][Cin/16][4 g][16 rows][4 t], row = 16 rb + rr = 3*tap + co.
// ---------------------------------------------------------------------------------------
template <int CIN, int TH>
__global__ void __launch_bounds__(256) convT_rgb_scatter_kernel(const RgbOutArgs a) {
  constexpr int PS = CIN + 8, KC = CIN / 16, C4 = CIN / 4;
  constexpr int LR = TH + 1, LC = 17;
  constexpr int NPOS = LR * LC;
  constexpr int NPB = (NPOS + 15) / 16;
  constexpr int PP = 36;  // partial-row stride (floats): 27 used, 16-byte aligned
  constexpr int XT = LR * LC * PS;
  __shared__ __attribute__((aligned(16))) float smem[XT + NPB * 16 * PP];
  float* const part = smem + XT;

  const int tid = threadIdx.x;
  const int gx0 = blockIdx.x * 16, gy0 = blockIdx.y * TH, nimg = blockIdx.z;
  const int H = a.H, W = a.W;
  const int lane = tid & 63, wave = tid >> 6;
  const int li = lane & 15, lg = lane >> 4;

  f32x4 wa[2][KC];
#pragma unroll
  for (int rb = 0; rb < 2; ++rb)
#pragma unroll
    for (int kc = 0; kc < KC; ++kc)
      wa[rb][kc] = *reinterpret_cast<const f32x4*>(a.wp2 + (((rb * KC + kc) * 4 + lg) * 16 + li) * 4);

  constexpr int NSTAGE = LR * LC * C4;
  constexpr int NIT = (NSTAGE + 255) / 256;
  f32x4 tmp[NIT];
#pragma unroll
  for (int i = 0; i < NIT; ++i) {
    const int e = i * 256 + tid;
    tmp[i] = f32x4{0.f, 0.f, 0.f, 0.f};
    if (e < NSTAGE) {
      const int c4 = e % C4, pe = e / C4, col = pe % LC, row = pe / LC;
      const int iy = gy0 - 1 + row, ix = gx0 - 1 + col;
      if (iy >= 0 && iy < H && ix >= 0 && ix < W)
        tmp[i] = *reinterpret_cast<const f32x4*>(a.in + ((size_t)(nimg * H + iy) * W + ix) * CIN + c4 * 4);
    }
  }
#pragma unroll
  for (int i = 0; i < NIT; ++i) {
    const int e = i * 256 + tid;
    if (e < NSTAGE) *reinterpret_cast<f32x4*>(&smem[(e / C4) * PS + (e % C4) * 4]) = tmp[i];
  }
  __syncthreads();

  for (int pb = wave; pb < NPB; pb += 4) {
    const int pos = pb * 16 + li;
    f32x4 bq[KC];
#pragma unroll
    for (int kc = 0; kc < KC; ++kc)
      bq[kc] = pos < NPOS ? *reinterpret_cast<const f32x4*>(&smem[pos * PS + kc * 16 + lg * 4])
                          : f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int rb = 0; rb < 2; ++rb) {
      f32x4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int kc = 0; kc < KC; ++kc)
#pragma unroll
        for (int t = 0; t < 4; ++t) acc = mfma4(wa[rb][kc][t], bq[kc][t], acc);
      // lane holds rows 16 rb + 4 lg .. +3 of position pb*16 + li
      *reinterpret_cast<f32x4*>(&part[pos * PP + rb * 16 + lg * 4]) = acc;
    }
  }
  __syncthreads();

  const int Ho = 2 * H, Wo = 2 * W;
  constexpr int NQ = 2 * TH * 8;  // (output rows) x (quads of 4 output pixels across 32)
  for (int it = tid; it < NQ; it += 256) {
    const int oyl = it >> 3, quad = it & 7;
    const int oy = 2 * gy0 + oyl;
    const int py = oyl & 1, ml = oyl >> 1;
    if (gy0 + ml >= H) continue;
    float y[12];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const int oxl = quad * 4 + k;
      const int px = oxl & 1, ql = oxl >> 1;
#pragma unroll
      for (int co = 0; co < 3; ++co) {
        float v;
        if (py == 0) {
          if (px == 0) {
            v = part[((ml + 1) * LC + ql + 1) * PP + (0 * 3 + 0) * 3 + co];
            v = __fadd_rn(v, part[((ml + 1) * LC + ql) * PP + (0 * 3 + 2) * 3 + co]);
            v = __fadd_rn(v, part[(ml * LC + ql + 1) * PP + (2 * 3 + 0) * 3 + co]);
            v = __fadd_rn(v, part[(ml * LC + ql) * PP + (2 * 3 + 2) * 3 + co]);
          } else {
            v = part[((ml + 1) * LC + ql + 1) * PP + (0 * 3 + 1) * 3 + co];
            v = __fadd_rn(v, part[(ml * LC + ql + 1) * PP + (2 * 3 + 1) * 3 + co]);
          }
        } else {
          if (px == 0) {
            v = part[((ml + 1) * LC + ql + 1) * PP + (1 * 3 + 0) * 3 + co];
            v = __fadd_rn(v, part[((ml + 1) * LC + ql) * PP + (1 * 3 + 2) * 3 + co]);
          } else {
            v = part[((ml + 1) * LC + ql + 1) * PP + (1 * 3 + 1) * 3 + co];
          }
        }
        v = __fadd_rn(v, a.bias[co]);
        float d = __fadd_rn(__fmul_rn(v, a.std[co]), a.mean[co]);
        y[k * 3 + co] = fminf(fmaxf(d, 0.f), 255.f);
      }
    }
    const int ox0 = 2 * gx0 + quad * 4;
    if (ox0 >= Wo) continue;
    const size_t o = ((size_t)(nimg * Ho + oy) * Wo + ox0) * 3;
    const bool full = ox0 + 4 <= Wo;
    if (a.out_f32) {
#pragma unroll
      for (int k = 0; k < 12; ++k)
        if (full || ox0 + k / 3 < Wo) a.out_f32[o + k] = y[k];
    }
    if (a.out_u8) {
      uint32_t w[3] = {0, 0, 0};
#pragma unroll
      for (int k = 0; k < 12; ++k) w[k >> 2] |= (uint32_t)rintf(y[k]) << (8 * (k & 3));
      if (full && (o & 3) == 0) {
        uint32_t* d = reinterpret_cast<uint32_t*>(a.out_u8 + o);
        d[0] = w[0];
        d[1] = w[1];
        d[2] = w[2];
      } else {
#pragma unroll
        for (int k = 0; k < 12; ++k)
          if (ox0 + k / 3 < Wo) a.out_u8[o + k] = (uint8_t)(w[k >> 2] >> (8 * (k & 3)));
      }
    }
  }
}

// ---------------------------------------------------------------------------------------
// encode_0 -> encode_1 fused through LDS.  A workgroup owns TH1 rows x 16 columns of the
// layer-1 output; it stages the (4 TH1 + 3) x 67 RGB pixels that feed them (normalised,
// planar, columns split by col % 4), computes layer 0 (K = 27 -> 7 MFMA k-steps) on the
// (2 TH1 + 1) x 33 layer-0 pixels layer 1 reads — written straight into layer 1's
// column-deinterleaved LDS tile, zero outside the layer-0 image (layer 1's SAME pad) —
// then runs layer 1 (stride-2 implicit GEMM, weights from L2 with register prefetch).
// The full-resolution C0-channel layer-0 activation never reaches HBM.
// CMP: the compact LDS form — layer 0's results are held in registers until every wave has
// finished reading the RGB planes, then written into the layer-1 tile that aliases them;
// that tile is unpadded (C0 floats per slot) with its 16-byte chunks XOR-swizzled per slot
// (16 consecutive slots -> 16 distinct bank slots for ds_read_b128, 8 -> 8 for the stores):
// 39 KB instead of 64 KB
// at TH1 = 4, four workgroups per CU instead of two.  Bit-identical to the padded form.
// ---------------------------------------------------------------------------------------
template <int C0, int C1, int TH1, bool U8, bool CMP = false>
__global__ void __launch_bounds__(256, CMP ? (TH1 >= 8 ? 2 : 4) : 1) enc01_kernel(const Enc01Args a) {
  static_assert(C0 % 16 == 0 && C1 % 16 == 0 && (TH1 % 4 == 0 || TH1 == 2), "tile");
  constexpr int R0 = 4 * TH1 + 3;        // RGB rows
  constexpr int QJ = 17;                 // entries per col%4 plane (67 cols -> 17)
  // RGB row pitch (4 column planes of QJ, padded: 81 ≡ 17 mod 32, so the staging stores of two
  // consecutive rows by one 32-lane half — 17 pixel groups a row — fill the 32 banks once) and
  // channel-plane pitch (≡ 16 mod 32: the layer-0 gathers of lanes lg = 0 / 1 at one tap read two
  // channels 16 banks apart): per instruction 2.0 -> 0.71 extra LDS cycles for the gathers,
  // 2.25 -> 0 for the stores (tools/lds/enc01_banks.py)
  constexpr int RP4 = 81;
  static_assert(RP4 >= 4 * QJ, "row pitch");
  constexpr int RGBP = R0 * RP4 + ((48 - (R0 * RP4) % 32) % 32);
  constexpr int LR1 = 2 * TH1 + 1, LC1 = 34, PS1 = CMP ? C0 : C0 + 8;
  // CMP swizzle: NCH chunks per slot; the key changes every GRP slots (GRP slots = 128 bytes):
  // then the layer-1 operand reads (ds_read_b128, 16 consecutive slots at even AND odd slot
  // offsets) and layer 0's result stores (ds_write_b128, 8 consecutive slots) are conflict-free —
  // the key per 256 bytes (GRP = 16 / NCH) left the odd offsets' reads 3.1 and the stores 8
  // extra cycles per instruction (tools/lds/enc01_banks.py)
  constexpr int NCH = C0 / 4, GRP = 8 / NCH;
  constexpr int T1 = LR1 * LC1 * PS1;    // layer-1 input tile (floats)
  constexpr int NB0 = C0 / 16;
  constexpr int KC1 = C0 / 16;
  constexpr int WR = TH1 >= 4 ? 4 : 2;   // waves split rows x channel blocks for layer 1
  constexpr int WC = 4 / WR;
  constexpr int MB = TH1 / WR;
  constexpr int NB1 = C1 / 16 / WC;
  static_assert((C1 / 16) % WC == 0, "layer-1 channel split");
  // u8 input: the 3 x 256 normalised values (x - mean) / std as a table, dead once staged
  // (CMP: after the RGB planes, inside the region the layer-1 tile later takes over)
  constexpr int LUT_OFF = CMP ? 3 * RGBP : T1 + 3 * RGBP;
  constexpr int SMEM0 = CMP ? (T1 > 3 * RGBP ? T1 : 3 * RGBP) : T1 + 3 * RGBP;
  constexpr int SMEM = U8 && LUT_OFF + 768 > SMEM0 ? LUT_OFF + 768 : SMEM0;
  __shared__ __attribute__((aligned(16))) float smem[SMEM];
  float* const t1 = smem;
  float* const rgb = CMP ? smem : smem + T1;
  float* const lut = smem + LUT_OFF;
  // float offset of channel chunk c4 of layer-1 tile slot `slot`
  auto t1c = [](int slot, int c4) {
    if constexpr (CMP) return slot * PS1 + 4 * (c4 ^ ((slot / GRP) % NCH));
    else return slot * PS1 + 4 * c4;
  };

  const int tid = threadIdx.x;
  const int gx0 = blockIdx.x * 16, gy0 = blockIdx.y * TH1, nimg = blockIdx.z;
  // timing probe: s_memrealtime (100 MHz) by thread 0 at the phase boundaries
  auto stamp = [&](int k) {
    if (a.tstamp && tid == 0)
      a.tstamp[((size_t)(blockIdx.z * gridDim.y + blockIdx.y) * gridDim.x + blockIdx.x) * 8 + k] =
          __builtin_amdgcn_s_memrealtime();
  };
  stamp(0);
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int lane = tid & 63, li = lane & 15, lg = lane >> 4;

  // layer-1 weight prefetch starts before anything else
  constexpr int PF = 2, NSTEP = 9 * KC1;
  const int wr = wave / WC, wc = wave % WC;
  const int co_wave = wc * NB1 * 16;
  const __amdgpu_buffer_rsrc_t wrs = weight_rsrc(a.wp1, 9 * 16 * KC1 * C1 * 4);
  const int wlb = (lg * C1 + co_wave + li) * 16;  // lane byte offset
  auto wglob = [&](int s, int nb) -> f32x4 {
    const int tap = s / KC1, kc = s % KC1;
    return weight_frag(wrs, wlb, ((tap * KC1 + kc) * 4 * C1 * 4 + nb * 64) * 4);
  };
  f32x4 av[PF + 1][NB1];
#pragma unroll
  for (int p = 0; p < PF; ++p)
#pragma unroll
    for (int nb = 0; nb < NB1; ++nb) av[p][nb] = wglob(p, nb);

  // ---- stage normalised RGB: rows 2*(2 gy0 - pad1y) - pad0y + rr, cols likewise ----
  const int ey0 = 2 * gy0 - a.pad1y, ex0 = 2 * gx0 - a.pad1x;   // first layer-0 pixel
  const int iy0 = 2 * ey0 - a.pad0y, ix0 = 2 * ex0 - a.pad0x;   // first RGB pixel
  auto put_rgb = [&](int rr, int col, int c, float x) {
    rgb[c * RGBP + rr * RP4 + (col & 3) * QJ + (col >> 2)] = __fdiv_rn(__fsub_rn(x, a.mean[c]), a.std[c]);
  };
  // zero the planes first where the tile leaves the image (SAME padding)
  const bool edge = iy0 < 0 || ix0 < 0 || iy0 + R0 > a.H || ix0 + 68 > a.W || !U8 || (ix0 * 3) % 4 != 0;
  // interior u8 tiles: each thread unpacks 4-pixel groups (12 bytes) of the 68-pixel row
  // segments; their loads are issued first so they fly together with the table's
  constexpr int GPR = 17, NG = R0 * GPR, NGI = (NG + 255) / 256;
  // the table's loads go out first (L2-resident): with in-order load returns, its LDS copy
  // then waits only for them, not for the u8 rows behind them
  float lutv[3];
  if constexpr (U8) {
#pragma unroll
    for (int i = 0; i < 3; ++i) lutv[i] = a.nlut[i * 256 + tid];
  }
  uint32_t wpre[NGI][3];
  if constexpr (U8) {
    if (!edge) {
#pragma unroll
      for (int i = 0; i < NGI; ++i) {
        const int e = i * 256 + tid;
        if (e < NG) {
          const int rr = e / GPR, g = e % GPR;
          const uint32_t* src = reinterpret_cast<const uint32_t*>(
              reinterpret_cast<const uint8_t*>(a.in) + ((size_t)(nimg * a.H + iy0 + rr) * a.W + ix0) * 3 + 12 * g);
          wpre[i][0] = src[0];
          wpre[i][1] = src[1];
          wpre[i][2] = src[2];
        }
      }
    }
  }
  if (edge)
    for (int e = tid; e < 3 * RGBP; e += 256) rgb[e] = 0.f;
  if constexpr (U8) {  // the host's f32 table (tic_finalize), same values as (v - mean) / std here
#pragma unroll
    for (int i = 0; i < 3; ++i) lut[i * 256 + tid] = lutv[i];
  }
  if (edge || U8) __syncthreads();
  stamp(1);
  if constexpr (U8) {
    if (!edge) {
      // pixel k of group g is column 4g + k: plane k, entry g
#pragma unroll
      for (int i = 0; i < NGI; ++i) {
        const int e = i * 256 + tid;
        if (e >= NG) break;
        const int rr = e / GPR, g = e % GPR;
        float* const dst = rgb + rr * RP4 + g;
#pragma unroll
        for (int k = 0; k < 4; ++k)
#pragma unroll
          for (int c = 0; c < 3; ++c) {
            const int b = 3 * k + c;
            dst[c * RGBP + k * QJ] = lut[c * 256 + ((wpre[i][b >> 2] >> (8 * (b & 3))) & 0xff)];
          }
      }
    }
  }
  if (edge) {
    for (int e = tid; e < R0 * 67; e += 256) {
      const int rr = e / 67, col = e % 67;
      const int iy = iy0 + rr, ix = ix0 + col;
      if (iy >= 0 && iy < a.H && ix >= 0 && ix < a.W) {
        const size_t off = ((size_t)(nimg * a.H + iy) * a.W + ix) * 3;
#pragma unroll
        for (int c = 0; c < 3; ++c) {
          if constexpr (U8)
            rgb[c * RGBP + rr * RP4 + (col & 3) * QJ + (col >> 2)] =
                lut[c * 256 + reinterpret_cast<const uint8_t*>(a.in)[off + c]];
          else
            put_rgb(rr, col, c, reinterpret_cast<const float*>(a.in)[off + c]);
        }
      }
    }
  }
  __syncthreads();
  stamp(2);

  // ---- layer 0 on every slot of the layer-1 input tile ----
  {
    f32x4 w0[NB0], w1[NB0], bb[NB0];
#pragma unroll
    for (int nb = 0; nb < NB0; ++nb) {
      const float* wq = a.wp0 + ((nb * 16 + li) * 4 + lg) * 8;
      w0[nb] = *reinterpret_cast<const f32x4*>(wq);
      w1[nb] = *reinterpret_cast<const f32x4*>(wq + 4);
      bb[nb] = *reinterpret_cast<const f32x4*>(a.b0 + nb * 16 + lg * 4);
    }
    // per-lane LDS offsets of the 7 k-steps (k = 4t + lg -> channel, ky, kx), per column
    // plane of the slot: offset = c*RGBP + ky*RP4 + ((2 plane + kx) & 3)*QJ + ((2 plane + kx) >> 2)
    int dl[2][7];
#pragma unroll
    for (int t = 0; t < 7; ++t) {
      const int k = 4 * t + lg;
      const int tap = k / 3, c = k - 3 * (k / 3);
      const int ky = tap / 3, kx = tap - 3 * (tap / 3);
#pragma unroll
      for (int pl = 0; pl < 2; ++pl) {
        const int q = 2 * pl + kx;
        dl[pl][t] = k < 27 ? c * RGBP + ky * RP4 + (q & 3) * QJ + (q >> 2) : -1;
      }
    }
    // Blocks of 16 slots: block 2r + p = tile row r, column plane p, j = 0..15 — a wave's
    // blocks (wave + 4 jb) all have the plane of its own parity; blocks 2 LR1 + q = plane 0's
    // j = 16 of rows 16 q + li.  Plane 1's j = 16 (layer-0 column 33) is never read by
    // layer 1 and is not computed.
    constexpr int NBL = 2 * LR1 + (LR1 + 15) / 16;
    constexpr int NPW = (NBL + 3) / 4;  // blocks per wave
    f32x4 res[CMP ? NPW : 1][NB0];       // CMP: layer-0 results held until the RGB planes are dead
    // + bias (two packed adds), ReLU, zero outside layer 0's image, into the layer-1 tile at
    // float offset off(nb) — the same operations as conv3x3_kernel's epilogue
    auto put0v = [&](bool valid, const f32x4 (&acc)[NB0], auto&& off) {
#pragma unroll
      for (int nb = 0; nb < NB0; ++nb) {
        f32x4 v = acc[nb] + bb[nb];
        v.x = fmaxf(v.x, 0.f);
        v.y = fmaxf(v.y, 0.f);
        v.z = fmaxf(v.z, 0.f);
        v.w = fmaxf(v.w, 0.f);
        if (!valid) v = f32x4{0.f, 0.f, 0.f, 0.f};
        *reinterpret_cast<f32x4*>(&t1[off(nb)]) = v;
      }
    };
    auto put0 = [&](int slot, bool valid, const f32x4 (&acc)[NB0]) {
      put0v(valid, acc, [&](int nb) { return t1c(slot, nb * 4 + lg); });
    };
    // a main block jb of this wave (blk = wave + 4 jb < 2 LR1): slot s0 + 2 LC1 jb, its swizzle
    // key (k0 + 2 LC1 jb / GRP) mod NCH — the per-lane parts computed once
    const int s0 = (wave >> 1) * LC1 + (wave & 1) * 17 + li;
    const int k0 = (s0 / GRP) % NCH;
    static_assert((2 * LC1) % GRP == 0 && (NCH & (NCH - 1)) == 0, "main-block slot stride");
    auto put0_main = [&](int jb, bool valid, const f32x4 (&acc)[NB0]) {
      const int slot = s0 + 2 * LC1 * jb;
      if constexpr (CMP) {
        const int key = (k0 + (2 * LC1 / GRP) * jb) & (NCH - 1);
        put0v(valid, acc, [&](int nb) { return slot * PS1 + 4 * ((nb * 4 + lg) ^ key); });
      } else {
        put0v(valid, acc, [&](int nb) { return slot * PS1 + 4 * (nb * 4 + lg); });
      }
    };
    // lane li's slot in block blk, whether the block holds it, and whether it lies inside
    // layer 0's image (else it is layer 1's zero padding)
    auto lo_row = [&](int blk) { return (blk - 2 * LR1) * 16 + li; };  // leftover blocks' row
    auto blk_slot = [&](int blk) {
      return blk < 2 * LR1 ? (blk >> 1) * LC1 + (blk & 1) * 17 + li : lo_row(blk) * LC1 + 16;
    };
    auto blk_has = [&](int blk) { return blk < 2 * LR1 || (blk < NBL && lo_row(blk) < LR1); };
    const bool inner0 = ey0 >= 0 && ey0 + LR1 <= a.H1 && ex0 >= 0 && ex0 + 33 <= a.W1;  // tile inside layer 0
    auto blk_valid = [&](int blk) {
      if (inner0) return true;
      const int r = blk < 2 * LR1 ? blk >> 1 : lo_row(blk);
      const int exl = blk < 2 * LR1 ? 2 * li + (blk & 1) : 32;
      const int ey = ey0 + r, ex = ex0 + exl;
      return exl < 33 && ey >= 0 && ey < a.H1 && ex >= 0 && ex < a.W1;
    };
    // the 7 k-step offsets of this wave's plane and of plane 0 (k = 27, the zero weight row,
    // reads offset 0 and is zeroed below)
    int dw[7], dz[7];
#pragma unroll
    for (int t = 0; t < 7; ++t) {
      const int d = (wave & 1) ? dl[1][t] : dl[0][t];
      dw[t] = d < 0 ? 0 : d;
      dz[t] = dl[0][t] < 0 ? 0 : dl[0][t];
    }
    // main blocks: row (blk >> 1) = (wave >> 1) + 2 jb, so the per-lane part of the 7 offsets is
    // fixed and block jb adds a constant (the read's immediate offset)
    const float* gw[7];
#pragma unroll
    for (int t = 0; t < 7; ++t) gw[t] = rgb + (wave >> 1) * 2 * RP4 + li + dw[t];
    auto gather = [&](int jb, float (&b)[7]) {
      const int blk = wave + 4 * jb;
      if (blk < 2 * LR1) {  // wave-uniform
#pragma unroll
        for (int t = 0; t < 7; ++t) b[t] = gw[t][jb * 4 * RP4];
      } else {
        const int base = (lo_row(blk) < LR1 ? lo_row(blk) : 0) * 2 * RP4 + 16;
#pragma unroll
        for (int t = 0; t < 7; ++t) b[t] = rgb[base + dz[t]];
      }
      if (lg == 3) b[6] = 0.f;  // k = 27
    };
    float bq0[2][7];
    gather(0, bq0[0]);
#pragma unroll
    for (int jb = 0; jb < NPW; ++jb) {
      const int blk = wave + 4 * jb;
      if (blk >= NBL) break;
      // the next block's operands load under this block's MFMAs
      if (jb + 1 < NPW) gather(jb + 1, bq0[(jb + 1) & 1]);
      __builtin_amdgcn_sched_barrier(0);
      const float(&b)[7] = bq0[jb & 1];
      f32x4 acc[NB0];
#pragma unroll
      for (int nb = 0; nb < NB0; ++nb) acc[nb] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int t = 0; t < 7; ++t)
#pragma unroll
        for (int nb = 0; nb < NB0; ++nb) acc[nb] = mfma4(t < 4 ? w0[nb][t & 3] : w1[nb][t & 3], b[t], acc[nb]);
      __builtin_amdgcn_sched_barrier(0);
      // lane holds channels nb*16 + 4 lg .. +3 of its slot; relu; zero outside layer 0's image
      if constexpr (CMP) {
#pragma unroll
        for (int nb = 0; nb < NB0; ++nb) res[jb][nb] = acc[nb];
      } else if (blk < 2 * LR1) {
        put0_main(jb, inner0 || blk_valid(blk), acc);
      } else if (blk_has(blk)) {
        put0(blk_slot(blk), blk_valid(blk), acc);
      }
    }
    if constexpr (CMP) {
      __syncthreads();  // every wave is done with the RGB planes the tile overwrites
      if (inner0) {  // workgroup-uniform: no slot of the tile lies in layer 1's zero padding
#pragma unroll
        for (int jb = 0; jb < NPW; ++jb) {
          const int blk = wave + 4 * jb;
          if (blk < 2 * LR1) put0_main(jb, true, res[jb]);
          else if (blk < NBL && blk_has(blk)) put0(blk_slot(blk), true, res[jb]);
        }
      } else {
#pragma unroll
        for (int jb = 0; jb < NPW; ++jb) {
          const int blk = wave + 4 * jb;
          if (blk < 2 * LR1) put0_main(jb, blk_valid(blk), res[jb]);
          else if (blk < NBL && blk_has(blk)) put0(blk_slot(blk), blk_valid(blk), res[jb]);
        }
      }
    }
  }
  __syncthreads();
  stamp(3);

  // ---- layer 1: stride-2 implicit GEMM from the LDS tile ----
  f32x4 acc[MB][NB1];
#pragma unroll
  for (int mb = 0; mb < MB; ++mb)
#pragma unroll
    for (int nb = 0; nb < NB1; ++nb) acc[mb][nb] = f32x4{0.f, 0.f, 0.f, 0.f};
  auto load_b = [&](int s, f32x4* dst) {
    const int tap = s / KC1, kc = s % KC1, ky = tap / 3, kx = tap % 3;
#pragma unroll
    for (int mb = 0; mb < MB; ++mb) {
      const int r = wr * MB + mb;
      const int lp = (2 * r + ky) * LC1 + (kx & 1) * 17 + li + (kx >> 1);
      dst[mb] = *reinterpret_cast<const f32x4*>(&t1[t1c(lp, kc * 4 + lg)]);
    }
  };
  f32x4 bq[2][MB];
  load_b(0, bq[0]);
#pragma unroll
  for (int s = 0; s < NSTEP; ++s) {
    const int c = s & 1;
    if (s + PF < NSTEP) {
#pragma unroll
      for (int nb = 0; nb < NB1; ++nb) av[(s + PF) % (PF + 1)][nb] = wglob(s + PF, nb);
    }
    if (s + 1 < NSTEP) load_b(s + 1, bq[c ^ 1]);
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int t = 0; t < 4; ++t)
#pragma unroll
      for (int mb = 0; mb < MB; ++mb)
#pragma unroll
        for (int nb = 0; nb < NB1; ++nb) acc[mb][nb] = mfma4(av[s % (PF + 1)][nb][t], bq[c][mb][t], acc[mb][nb]);
    __builtin_amdgcn_sched_barrier(0);
  }
  stamp(4);
#pragma unroll
  for (int mb = 0; mb < MB; ++mb) {
    const int oy = gy0 + wr * MB + mb, ox = gx0 + li;
    if (oy >= a.H2 || ox >= a.W2) continue;
#pragma unroll
    for (int nb = 0; nb < NB1; ++nb) {
      const int co = co_wave + nb * 16 + lg * 4;
      const f32x4 bb = *reinterpret_cast<const f32x4*>(a.b1 + co);
      f32x4 v = acc[mb][nb];
      v.x = fmaxf(__fadd_rn(v.x, bb.x), 0.f);
      v.y = fmaxf(__fadd_rn(v.y, bb.y), 0.f);
      v.z = fmaxf(__fadd_rn(v.z, bb.z), 0.f);
      v.w = fmaxf(__fadd_rn(v.w, bb.w), 0.f);
      *reinterpret_cast<f32x4*>(a.out + ((size_t)(nimg * a.H2 + oy) * a.W2 + ox) * C1 + co) = v;
    }
  }
  stamp(5);
}

}  // namespace tic
