// enc01pc.h — encode_0 -> encode_1 fused (enc01_kernel's arithmetic, operation for operation)
// as a persistent PRODUCER / CONSUMER pipeline: one 512-thread workgroup per CU walks the
// TH1 x 16 layer-1 output tiles; waves 4-7 (producers) stage tile i+1's normalised RGB and run
// its layer 0, while waves 0-3 (consumers) run tile i's layer 1 (the MFMA-heavy part) — on
// every SIMD one producer wave beside one consumer wave, so the matrix pipe has layer-1 work
// while the producer waits on memory, the table and the LDS (the one-shot enc01's
// four co-resident workgroups go through those phases together, the pipe idling meanwhile).
//
// Buffers: the layer-1 input tile (compact, swizzled) and the RGB planes are both double
// buffered, so one barrier per phase orders everything: in phase p the producers write
// t1[p % 2] (layer 0 of tile p) and rgb[(p + 1) % 2] (tile p + 1), the consumers read
// t1[(p - 1) % 2] (layer 1 of tile p - 1).  Staging writes every plane entry exactly once (zero
// outside the image), so it needs no barrier of its own.  The u8 rows of tile p + 2 are loaded
// into producer registers in phase p.
// Bit-identical to enc01_kernel (tests/test_gpu_parity.py::test_fused_first_layers_bit_identical,
// variant 6).
#pragma once
#include "conv3x3.h"

namespace tic {

template <int C0, int C1, bool U8>
__global__ void __launch_bounds__(512, 1) enc01pc_kernel(const Enc01Args a, int ntx, int nty, int ntiles) {
  constexpr int TH1 = 4;
  static_assert(C0 % 16 == 0 && C1 % 16 == 0, "tile");
  constexpr int R0 = 4 * TH1 + 3;         // RGB rows
  constexpr int QJ = 17;                  // entries per col%4 plane (68 cols)
  constexpr int RGBP = R0 * 4 * QJ;       // floats per channel plane
  constexpr int RGBB = 3 * RGBP;          // one RGB buffer
  constexpr int LR1 = 2 * TH1 + 1, LC1 = 34, PS1 = C0;
  constexpr int NCH = C0 / 4, GRP = 16 / NCH;
  constexpr int T1 = LR1 * LC1 * PS1;
  constexpr int NB0 = C0 / 16, KC1 = C0 / 16;
  constexpr int MB = TH1 / 4, NB1 = C1 / 16;  // consumer wave = one layer-1 row group
  __shared__ __attribute__((aligned(16))) float smem[2 * T1 + 2 * RGBB + (U8 ? 768 : 4)];
  float* const lut = smem + 2 * T1 + 2 * RGBB;
  auto t1c = [](int slot, int c4) { return slot * PS1 + 4 * (c4 ^ ((slot / GRP) % NCH)); };

  const int tid = threadIdx.x;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const bool producer = wave >= 4;
  const int pw = wave & 3;  // wave index within the role
  const int ptid = tid & 255;
  const int lane = tid & 63, li = lane & 15, lg = lane >> 4;
  const int G = gridDim.x;
  const int T = blockIdx.x < ntiles ? (ntiles - 1 - (int)blockIdx.x) / G + 1 : 0;  // this workgroup's tiles
  auto tile_of = [&](int i) { return (int)blockIdx.x + i * G; };
  auto geom = [&](int t, int& gx0, int& gy0, int& nimg) {
    gx0 = (t % ntx) * 16;
    gy0 = ((t / ntx) % nty) * TH1;
    nimg = t / (ntx * nty);
  };

  if (producer) {
    // ================================ producers ================================
    if constexpr (U8)
      for (int e = ptid; e < 768; e += 256) lut[e] = a.nlut[e];
    f32x4 w0[NB0], w1[NB0], bb0[NB0];
#pragma unroll
    for (int nb = 0; nb < NB0; ++nb) {
      const float* wq = a.wp0 + ((nb * 16 + li) * 4 + lg) * 8;
      w0[nb] = *reinterpret_cast<const f32x4*>(wq);
      w1[nb] = *reinterpret_cast<const f32x4*>(wq + 4);
      bb0[nb] = *reinterpret_cast<const f32x4*>(a.b0 + nb * 16 + lg * 4);
    }
    int dw[7], dz[7];
#pragma unroll
    for (int t = 0; t < 7; ++t) {
      const int k = 4 * t + lg;
      const int tap = k / 3, c = k - 3 * (k / 3);
      const int ky = tap / 3, kx = tap - 3 * (tap / 3);
      const int q1 = 2 + kx, q0 = kx;
      const int d1 = k < 27 ? c * RGBP + ky * 4 * QJ + (q1 & 3) * QJ + (q1 >> 2) : 0;
      const int d0 = k < 27 ? c * RGBP + ky * 4 * QJ + (q0 & 3) * QJ + (q0 >> 2) : 0;
      dw[t] = (pw & 1) ? d1 : d0;
      dz[t] = d0;
    }
    constexpr int GPR = 17, NG = R0 * GPR, NGI = (NG + 255) / 256;
    uint32_t wpre[NGI][3];
    auto corner = [&](int t, int& iy0, int& ix0, int& nimg) {
      int gx0, gy0;
      geom(t, gx0, gy0, nimg);
      iy0 = 2 * (2 * gy0 - a.pad1y) - a.pad0y;
      ix0 = 2 * (2 * gx0 - a.pad1x) - a.pad0x;
    };
    auto is_edge = [&](int iy0, int ix0) {
      return iy0 < 0 || ix0 < 0 || iy0 + R0 > a.H || ix0 + 68 > a.W || !U8 || (ix0 * 3) % 4 != 0;
    };
    auto issue = [&](int i) {  // u8 rows of this workgroup's i-th tile (interior tiles)
      if (i >= T) return;
      int iy0, ix0, nimg;
      corner(tile_of(i), iy0, ix0, nimg);
      if (!U8 || is_edge(iy0, ix0)) return;
#pragma unroll
      for (int k = 0; k < NGI; ++k) {
        const int e = k * 256 + ptid;
        if (e < NG) {
          const int rr = e / GPR, g = e % GPR;
          const uint32_t* src = reinterpret_cast<const uint32_t*>(
              reinterpret_cast<const uint8_t*>(a.in) + ((size_t)(nimg * a.H + iy0 + rr) * a.W + ix0) * 3 + 12 * g);
          wpre[k][0] = src[0];
          wpre[k][1] = src[1];
          wpre[k][2] = src[2];
        }
      }
    };
    // every plane entry written exactly once (zero outside the image)
    auto stage = [&](int i, float* rgb) {
      if (i >= T) return;
      int iy0, ix0, nimg;
      corner(tile_of(i), iy0, ix0, nimg);
      if (is_edge(iy0, ix0)) {
        for (int e = ptid; e < R0 * 68; e += 256) {
          const int rr = e / 68, col = e % 68;
          const int iy = iy0 + rr, ix = ix0 + col;
          const bool in = iy >= 0 && iy < a.H && ix >= 0 && ix < a.W;
          const size_t off = in ? ((size_t)(nimg * a.H + iy) * a.W + ix) * 3 : 0;
#pragma unroll
          for (int c = 0; c < 3; ++c) {
            float v = 0.f;
            if (in) {
              if constexpr (U8) v = lut[c * 256 + reinterpret_cast<const uint8_t*>(a.in)[off + c]];
              else v = __fdiv_rn(__fsub_rn(reinterpret_cast<const float*>(a.in)[off + c], a.mean[c]), a.std[c]);
            }
            rgb[c * RGBP + (rr * 4 + (col & 3)) * QJ + (col >> 2)] = v;
          }
        }
      } else if constexpr (U8) {
#pragma unroll
        for (int k = 0; k < NGI; ++k) {
          const int e = k * 256 + ptid;
          if (e >= NG) break;
          const int rr = e / GPR, g = e % GPR;
          float* const dst = rgb + rr * 4 * QJ + g;
#pragma unroll
          for (int q = 0; q < 4; ++q)
#pragma unroll
            for (int c = 0; c < 3; ++c) {
              const int b = 3 * q + c;
              dst[c * RGBP + q * QJ] = lut[c * 256 + ((wpre[k][b >> 2] >> (8 * (b & 3))) & 0xff)];
            }
        }
      }
    };
    // layer 0 of tile i from rgb into t1 (enc01_kernel's order)
    auto layer0 = [&](int i, const float* rgb, float* t1) {
      int gx0, gy0, nimg;
      geom(tile_of(i), gx0, gy0, nimg);
      const int ey0 = 2 * gy0 - a.pad1y, ex0 = 2 * gx0 - a.pad1x;
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
        const int blk = pw + 4 * jb;
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
        const int blk = pw + 4 * jb;
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
    };
    // prologue: the table, tile 0's planes, tile 1's u8 rows
    issue(0);
    __syncthreads();  // (1) the table (a whole-workgroup barrier: the consumers wait with it)
    stage(0, smem + 2 * T1);
    issue(1);
    __syncthreads();  // (2) tile 0's planes
    for (int p = 0; p <= T; ++p) {  // phase p: layer 0 of tile p, planes of tile p + 1
      if (p < T) {
        layer0(p, smem + 2 * T1 + (p & 1) * RGBB, smem + (p & 1) * T1);
        stage(p + 1, smem + 2 * T1 + ((p + 1) & 1) * RGBB);
        issue(p + 2);
      }
      __syncthreads();
    }
  } else {
    // ================================ consumers ================================
    __syncthreads();  // (1)
    __syncthreads();  // (2)
    constexpr int PF = 2, NSTEP = 9 * KC1;
    const int wr = pw;
    const int woff0 = (lg * C1 + li) * 4;
    for (int p = 0; p <= T; ++p) {  // phase p: layer 1 of tile p - 1
      if (p >= 1) {
        const int i = p - 1;
        const float* t1 = smem + (i & 1) * T1;
        int gx0, gy0, nimg;
        geom(tile_of(i), gx0, gy0, nimg);
        int woff = woff0;
        asm volatile("" : "+v"(woff));  // keep the weight loads inside the tile loop
        const float* __restrict__ wl = a.wp1 + woff;
        auto wglob = [&](int s, int nb) -> f32x4 {
          const int tap = s / KC1, kc = s % KC1;
          return *reinterpret_cast<const f32x4*>(wl + (size_t)(tap * KC1 + kc) * 4 * C1 * 4 + nb * 64);
        };
        f32x4 av[PF + 1][NB1];
#pragma unroll
        for (int q = 0; q < PF; ++q)
#pragma unroll
          for (int nb = 0; nb < NB1; ++nb) av[q][nb] = wglob(q, nb);
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
      __syncthreads();
    }
  }
}

}  // namespace tic
