// enc01p.h — encode_0 -> encode_1 fused (enc01_kernel's arithmetic, operation for operation)
// as a PERSISTENT, software-pipelined kernel: two 256-thread workgroups per CU walk the
// TH1 x 16 layer-1 output tiles of the whole batch.
//
// Why: the one-shot enc01 launches 2048 short workgroups
// per 32 patches, four per CU, that start together and go through the same phases together —
// the normalisation table and the u8 RGB loads (latency-bound) at the same time, then layer 0
// (VALU / LDS-bound), then layer 1 (MFMA-bound) — so the matrix cores idle through every
// workgroup's first phases.  Here each workgroup:
//   * stages the 3 x 256-entry normalisation table and its layer-0 weights once;
//   * issues the next tile's u8 RGB loads (registers) before the current tile's layer-1 MFMAs,
//     so they land under the matrix-core phase;
//   * stages the next tile's RGB planes right after its own layer-1 (the planes are a buffer of
//     their own, not aliased with the layer-1 tile), while the other waves may still run
//     layer 1 — two barriers per tile.
// Every output is bit-identical to enc01_kernel / conv_rgb_s2_kernel + conv3x3_kernel
// (tests/test_gpu_parity.py::test_fused_first_layers_bit_identical covers it as variant 5).
#pragma once
#include "conv3x3.h"

namespace tic {

template <int C0, int C1, int TH1, bool U8>
__global__ void __launch_bounds__(256, 2) enc01p_kernel(const Enc01Args a, int ntx, int nty, int ntiles) {
  static_assert(C0 % 16 == 0 && C1 % 16 == 0 && TH1 % 4 == 0, "tile");
  constexpr int R0 = 4 * TH1 + 3;         // RGB rows
  constexpr int QJ = 17;                  // entries per col%4 plane (67 cols -> 17)
  constexpr int RGBP = R0 * 4 * QJ;       // floats per channel plane
  constexpr int LR1 = 2 * TH1 + 1, LC1 = 34, PS1 = C0;
  constexpr int NCH = C0 / 4, GRP = 16 / NCH;  // swizzle: chunks per slot, slots per 256 B
  constexpr int T1 = LR1 * LC1 * PS1;     // layer-1 input tile (floats), compact swizzled form
  constexpr int NB0 = C0 / 16, KC1 = C0 / 16;
  constexpr int WR = 4, MB = TH1 / WR, NB1 = C1 / 16;  // one layer-1 row group per wave
  __shared__ __attribute__((aligned(16))) float smem[T1 + 3 * RGBP + (U8 ? 768 : 4)];
  float* const t1 = smem;
  float* const rgb = smem + T1;
  float* const lut = rgb + 3 * RGBP;
  auto t1c = [](int slot, int c4) { return slot * PS1 + 4 * (c4 ^ ((slot / GRP) % NCH)); };

  const int tid = threadIdx.x;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int lane = tid & 63, li = lane & 15, lg = lane >> 4;
  const int wr = wave;  // WC = 1: wave = layer-1 row group

  // ---- once per workgroup: the normalisation table, layer 0's weights and bias ----
  if constexpr (U8)
    for (int e = tid; e < 768; e += 256) lut[e] = a.nlut[e];
  f32x4 w0[NB0], w1[NB0], bb0[NB0];
#pragma unroll
  for (int nb = 0; nb < NB0; ++nb) {
    const float* wq = a.wp0 + ((nb * 16 + li) * 4 + lg) * 8;
    w0[nb] = *reinterpret_cast<const f32x4*>(wq);
    w1[nb] = *reinterpret_cast<const f32x4*>(wq + 4);
    bb0[nb] = *reinterpret_cast<const f32x4*>(a.b0 + nb * 16 + lg * 4);
  }
  // layer 0's 7 k-step gather offsets (k = 4t + lg -> channel, ky, kx), per column plane
  int dw[7], dz[7];
#pragma unroll
  for (int t = 0; t < 7; ++t) {
    const int k = 4 * t + lg;
    const int tap = k / 3, c = k - 3 * (k / 3);
    const int ky = tap / 3, kx = tap - 3 * (tap / 3);
    const int q1 = 2 + kx, q0 = kx;
    const int d1 = k < 27 ? c * RGBP + ky * 4 * QJ + (q1 & 3) * QJ + (q1 >> 2) : 0;
    const int d0 = k < 27 ? c * RGBP + ky * 4 * QJ + (q0 & 3) * QJ + (q0 >> 2) : 0;
    dw[t] = (wave & 1) ? d1 : d0;
    dz[t] = d0;
  }

  // ---- the u8 RGB rows of a tile into registers (interior tiles; edge tiles load later) ----
  constexpr int GPR = 17, NG = R0 * GPR, NGI = (NG + 255) / 256;
  auto geom = [&](int t, int& gx0, int& gy0, int& nimg) {
    gx0 = (t % ntx) * 16;
    gy0 = ((t / ntx) % nty) * TH1;
    nimg = t / (ntx * nty);
  };
  auto is_edge = [&](int iy0, int ix0) {
    return iy0 < 0 || ix0 < 0 || iy0 + R0 > a.H || ix0 + 68 > a.W || !U8 || (ix0 * 3) % 4 != 0;
  };
  uint32_t wpre[NGI][3];
  auto issue = [&](int t) {
    int gx0, gy0, nimg;
    geom(t, gx0, gy0, nimg);
    const int iy0 = 2 * (2 * gy0 - a.pad1y) - a.pad0y, ix0 = 2 * (2 * gx0 - a.pad1x) - a.pad0x;
    if (!U8 || is_edge(iy0, ix0)) return;
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
  };

  // layer-1 weights: per-lane offset, re-derived opaquely every tile so the loop-invariant
  // loads are not hoisted out of the tile loop (they would need 36 x 4 VGPRs and spill)
  constexpr int PF = 2, NSTEP = 9 * KC1;
  const int woff0 = (lg * C1 + li) * 4;

  int t = blockIdx.x;
  if (t < ntiles) issue(t);
  if constexpr (U8) __syncthreads();  // the table

  for (; t < ntiles; t += gridDim.x) {
    int gx0, gy0, nimg;
    geom(t, gx0, gy0, nimg);
    const int ey0 = 2 * gy0 - a.pad1y, ex0 = 2 * gx0 - a.pad1x;  // first layer-0 pixel
    const int iy0 = 2 * ey0 - a.pad0y, ix0 = 2 * ex0 - a.pad0x;  // first RGB pixel
    const bool edge = is_edge(iy0, ix0);

    // ---- stage the normalised RGB planes (the previous tile's layer 0 is done with them) ----
    if (edge) {
      for (int e = tid; e < 3 * RGBP; e += 256) rgb[e] = 0.f;
      __syncthreads();
      for (int e = tid; e < R0 * 67; e += 256) {
        const int rr = e / 67, col = e % 67;
        const int iy = iy0 + rr, ix = ix0 + col;
        if (iy >= 0 && iy < a.H && ix >= 0 && ix < a.W) {
          const size_t off = ((size_t)(nimg * a.H + iy) * a.W + ix) * 3;
#pragma unroll
          for (int c = 0; c < 3; ++c) {
            float v;
            if constexpr (U8) v = lut[c * 256 + reinterpret_cast<const uint8_t*>(a.in)[off + c]];
            else v = __fdiv_rn(__fsub_rn(reinterpret_cast<const float*>(a.in)[off + c], a.mean[c]), a.std[c]);
            rgb[c * RGBP + (rr * 4 + (col & 3)) * QJ + (col >> 2)] = v;
          }
        }
      }
    } else if constexpr (U8) {
#pragma unroll
      for (int i = 0; i < NGI; ++i) {
        const int e = i * 256 + tid;
        if (e >= NG) break;
        const int rr = e / GPR, g = e % GPR;
        float* const dst = rgb + rr * 4 * QJ + g;
#pragma unroll
        for (int k = 0; k < 4; ++k)
#pragma unroll
          for (int c = 0; c < 3; ++c) {
            const int b = 3 * k + c;
            dst[c * RGBP + k * QJ] = lut[c * 256 + ((wpre[i][b >> 2] >> (8 * (b & 3))) & 0xff)];
          }
      }
    }
    __syncthreads();  // planes staged; every wave is done reading the previous tile's t1

    // ---- layer 0 on every slot of the layer-1 input tile (enc01_kernel's order) ----
    {
      constexpr int NBL = 2 * LR1 + (LR1 + 15) / 16;
      constexpr int NPW = (NBL + 3) / 4;
      auto lo_row = [&](int blk) { return (blk - 2 * LR1) * 16 + li; };
      auto blk_slot = [&](int blk) {
        return blk < 2 * LR1 ? (blk >> 1) * LC1 + (blk & 1) * 17 + li : lo_row(blk) * LC1 + 16;
      };
      auto blk_has = [&](int blk) { return blk < 2 * LR1 || (blk < NBL && lo_row(blk) < LR1); };
      const bool inner0 = ey0 >= 0 && ey0 + LR1 <= a.H1 && ex0 >= 0 && ex0 + 33 <= a.W1;
      auto blk_valid = [&](int blk) {
        if (inner0) return true;
        const int r = blk < 2 * LR1 ? blk >> 1 : lo_row(blk);
        const int exl = blk < 2 * LR1 ? 2 * li + (blk & 1) : 32;
        const int ey = ey0 + r, ex = ex0 + exl;
        return exl < 33 && ey >= 0 && ey < a.H1 && ex >= 0 && ex < a.W1;
      };
      auto gather = [&](int jb, float (&b)[7]) {
        const int blk = wave + 4 * jb;
        if (blk < 2 * LR1) {
          const int base = (blk >> 1) * 8 * QJ + li;
#pragma unroll
          for (int tt = 0; tt < 7; ++tt) b[tt] = rgb[base + dw[tt]];
        } else {
          const int base = (lo_row(blk) < LR1 ? lo_row(blk) : 0) * 8 * QJ + 16;
#pragma unroll
          for (int tt = 0; tt < 7; ++tt) b[tt] = rgb[base + dz[tt]];
        }
        if (lg == 3) b[6] = 0.f;  // k = 27
      };
      float bq0[2][7];
      gather(0, bq0[0]);
#pragma unroll
      for (int jb = 0; jb < NPW; ++jb) {
        const int blk = wave + 4 * jb;
        if (blk >= NBL) break;
        if (jb + 1 < NPW) gather(jb + 1, bq0[(jb + 1) & 1]);
        __builtin_amdgcn_sched_barrier(0);
        const float(&b)[7] = bq0[jb & 1];
        f32x4 acc[NB0];
#pragma unroll
        for (int nb = 0; nb < NB0; ++nb) acc[nb] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int tt = 0; tt < 7; ++tt)
#pragma unroll
          for (int nb = 0; nb < NB0; ++nb) acc[nb] = mfma4(tt < 4 ? w0[nb][tt & 3] : w1[nb][tt & 3], b[tt], acc[nb]);
        __builtin_amdgcn_sched_barrier(0);
        if (blk_has(blk)) {
          const bool valid = blk_valid(blk);
          const int slot = blk_slot(blk);
#pragma unroll
          for (int nb = 0; nb < NB0; ++nb) {
            f32x4 v = acc[nb];
            v.x = valid ? fmaxf(__fadd_rn(v.x, bb0[nb].x), 0.f) : 0.f;
            v.y = valid ? fmaxf(__fadd_rn(v.y, bb0[nb].y), 0.f) : 0.f;
            v.z = valid ? fmaxf(__fadd_rn(v.z, bb0[nb].z), 0.f) : 0.f;
            v.w = valid ? fmaxf(__fadd_rn(v.w, bb0[nb].w), 0.f) : 0.f;
            *reinterpret_cast<f32x4*>(&t1[t1c(slot, nb * 4 + lg)]) = v;
          }
        }
      }
    }
    __syncthreads();  // t1 complete

    // the next tile's u8 RGB rows fly under this tile's layer-1 MFMAs
    if (t + (int)gridDim.x < ntiles) issue(t + gridDim.x);

    // ---- layer 1: stride-2 implicit GEMM from t1 (enc01_kernel's order) ----
    int woff = woff0;
    asm volatile("" : "+v"(woff));
    const float* __restrict__ wl = a.wp1 + woff;
    auto wglob = [&](int s, int nb) -> f32x4 {
      const int tap = s / KC1, kc = s % KC1;
      return *reinterpret_cast<const f32x4*>(wl + (size_t)(tap * KC1 + kc) * 4 * C1 * 4 + nb * 64);
    };
    f32x4 av[PF + 1][NB1];
#pragma unroll
    for (int p = 0; p < PF; ++p)
#pragma unroll
      for (int nb = 0; nb < NB1; ++nb) av[p][nb] = wglob(p, nb);
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
      for (int tt = 0; tt < 4; ++tt)
#pragma unroll
        for (int mb = 0; mb < MB; ++mb)
#pragma unroll
          for (int nb = 0; nb < NB1; ++nb) acc[mb][nb] = mfma4(av[s % (PF + 1)][nb][tt], bq[c][mb][tt], acc[mb][nb]);
      __builtin_amdgcn_sched_barrier(0);
    }
#pragma unroll
    for (int mb = 0; mb < MB; ++mb) {
      const int oy = gy0 + wr * MB + mb, ox = gx0 + li;
      if (oy >= a.H2 || ox >= a.W2) continue;
#pragma unroll
      for (int nb = 0; nb < NB1; ++nb) {
        const int co = nb * 16 + lg * 4;
        const f32x4 bb = *reinterpret_cast<const f32x4*>(a.b1 + co);
        f32x4 v = acc[mb][nb];
        v.x = fmaxf(__fadd_rn(v.x, bb.x), 0.f);
        v.y = fmaxf(__fadd_rn(v.y, bb.y), 0.f);
        v.z = fmaxf(__fadd_rn(v.z, bb.z), 0.f);
        v.w = fmaxf(__fadd_rn(v.w, bb.w), 0.f);
        *reinterpret_cast<f32x4*>(a.out + ((size_t)(nimg * a.H2 + oy) * a.W2 + ox) * C1 + co) = v;
      }
    }
  }
}

}  // namespace tic
