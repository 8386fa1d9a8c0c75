// conv3x3_wino4.h — stride-1 'SAME' 3x3 convolutions as Winograd F(4x4, 3x3) on the matrix
// cores: the res_block convs of model_3 (basic_block/basic_block.py:74-93, model_3/model.py:
// 66-150,191-281) and the rmbe net's conv_3/4 (submit/2/rmbe/model.py).  Stride-1 form 2
// (handle option "s1_form" = 2; conv3x3_wino.h is form 1).
//
// Per 4x4 output tile with 6x6 input patch d:  Y = A^T [ U (.) V ] A,  U = G g G^T,
// V = B^T d B, on the interpolation points (0, 1, -1, 2, -1/2, inf).  A tile costs 36
// transform points x Cin x Cout MACs instead of the direct form's 16 pixels x 9 taps:
// 4x fewer matrix-core cycles (F(2x2,3x3): 2.25x).  Every entry of A^T and B^T is a dyadic
// rational (exact in f32); G has thirds and fifteenths, so U is transformed on the host in
// double and rounded once.  Of the point sets with dyadic transforms this one keeps the f32
// error lowest (tools/wino_numerics.py: 2e-6 of the layer's range per layer against
// 6e-6 for the usual (0, +-1, +-2); model_3 end to end: pre-activations 9e-7 relative, no
// symbol changes, decoder 6e-3 on the [0,255] scale against the 1e-2 bar).
//
// Workgroup: 16 4x4 tiles (TTY rows x 16/TTY columns of tiles; TTY = 1, 2, 4 for 64-, 32-,
// 16-wide layers) x one or both output-channel halves (NSPLIT, below).  The wave owning
// B^T row xi and an output-channel half forms row xi of B^T d from the staged input rows (rows 1..4
// always, row 0 / 5 for xi = 0 / 5 — the non-zeros of B^T), then the six column
// combinations V_(xi,nu) in registers, and runs the six point GEMMs (M = Cout / 2, N = 16
// tiles, K = Cin) on v_mfma_f32_16x16x4_f32 with conv3x3_kernel's fragment layout.  The
// transformed inputs never touch LDS or HBM.  The whole Cin of the input tile
// ((4 TTY + 2) x (64 / TTY + 2) pixels, zero outside the image = SAME pad) is staged once,
// columns split by (column mod 4) so the 16 tiles of a read hit 16 consecutive pixels of a
// plane (pixel stride Cin + 8 floats: conflict-free ds_read_b128; TTY = 4 pads each row by 8
// floats for the same reason).  After the K loop each wave applies A on the nu side
// (T = M A), the waves swap T through LDS (aliasing the dead input tile) and each thread
// finishes Y = A^T T for one (tile, output column, 4-channel quad), then my_conv2d's epilogue.
//
// Summation order per output is fixed by the code — M over K in MFMA order, the transforms
// in the orders written below — and does not depend on TTY: the tilings of this form are
// bit-identical to each other.  Different from forms 0 and 1 by rounding only.
#pragma once
#include "conv3x3_wino.h"

namespace tic {

// B^T (rows xi, columns i) and A^T (rows a, columns nu) of F(4x4, 3x3) on (0, 1, -1, 2, -1/2)
__device__ constexpr float kW4BT[6][6] = {{1.f, 1.5f, -2.f, -1.5f, 1.f, 0.f},  {0.f, -1.f, -2.5f, -0.5f, 1.f, 0.f},
                                          {0.f, 1.f, 0.5f, -2.5f, 1.f, 0.f},   {0.f, -0.5f, -1.f, 0.5f, 1.f, 0.f},
                                          {0.f, 2.f, -1.f, -2.f, 1.f, 0.f},    {0.f, 1.f, 1.5f, -2.f, -1.5f, 1.f}};
__device__ constexpr float kW4AT[4][6] = {{1.f, 1.f, 1.f, 1.f, 1.f, 0.f},
                                          {0.f, 1.f, -1.f, 2.f, -0.5f, 0.f},
                                          {0.f, 1.f, 1.f, 4.f, 0.25f, 0.f},
                                          {0.f, 1.f, -1.f, 8.f, -0.125f, 1.f}};

__device__ __forceinline__ f32x4 fma4s(float c, f32x4 x, f32x4 y) {
  return f32x4{__builtin_fmaf(c, x.x, y.x), __builtin_fmaf(c, x.y, y.y), __builtin_fmaf(c, x.z, y.z),
               __builtin_fmaf(c, x.w, y.w)};
}

// sum_j k[j] v[j] over the non-zero k[j] in index order: the first term k * v, then fmas
// (k a compile-time row after unrolling: the zero terms vanish, the +-1 products are exact)
template <int N>
__device__ __forceinline__ f32x4 wcomb(const float (&k)[N], const f32x4 (&v)[N]) {
  f32x4 s = f32x4{0.f, 0.f, 0.f, 0.f};
  bool first = true;
#pragma unroll
  for (int j = 0; j < N; ++j) {
    if (k[j] == 0.f) continue;
    if (first) {
      s = k[j] * v[j];
      first = false;
    } else {
      s = fma4s(k[j], v[j], s);
    }
  }
  return s;
}

template <int TTY>
struct Wino4Geom {
  static constexpr int NT = 16;              // 4x4 output tiles per workgroup
  static constexpr int TTX = NT / TTY;       // tiles per tile row
  static constexpr int LR = 4 * TTY + 2;     // staged input rows
  static constexpr int LCOL = 4 * TTX + 2;   // staged input columns
  static constexpr int HPP = TTX + 1;        // pixels per (column mod 4) plane
  static constexpr int RPAD = TTY == 4 ? 8 : 0;
};

// Weights (ConvArgs::wp): U packed [36 p][Cin/16][4 g][Cout][4 t], p = 6 xi + nu.
// NSPLIT 1: 768 threads, wave w = (xi = w / 2, output-channel half w % 2), the whole Cin of
// the input tile staged at once (117 KB: one workgroup per CU).  NSPLIT 2: two 384-thread
// workgroups per tile, one per output-channel half (wave = xi), each staging the input tile
// in two channel halves (65 KB: two workgroups per CU, so one's staging and stores overlap
// the other's matrix work).  Same per-output operation order: bit-identical.
template <int CIN, int COUT, int TTY, int NSPLIT, int ACT, bool RES, int IN, int OUT>
__global__ void __launch_bounds__(NSPLIT == 1 ? 768 : 384, 3) conv3x3_wino4_kernel(const ConvArgs a) {
  using G = Wino4Geom<TTY>;
  constexpr int NT = G::NT, TTX = G::TTX, LR = G::LR, LCOL = G::LCOL, HPP = G::HPP;
  static_assert(CIN % 32 == 0 && COUT % 32 == 0 && (NSPLIT == 1 || NSPLIT == 2), "channels");
  constexpr int NTHR = NSPLIT == 1 ? 768 : 384;
  constexpr int KST = CIN / NSPLIT;            // input channels staged at once
  constexpr int NHALF = CIN / KST;             // staging rounds
  constexpr int PS = KST + 8, KC = CIN / 16, KCH = KST / 16, C4 = KST / 4;
  constexpr int RS = 4 * HPP * PS + G::RPAD;  // floats per staged row
  constexpr int TILE = LR * RS;
  constexpr int CW = COUT / 2;                // output channels per wave
  constexpr int NBW = CW / 16;
  constexpr int CWG = COUT / NSPLIT;          // output channels per workgroup
  constexpr int XS = CWG + 4;                 // exchange pitch per (xi, b, tile)
  constexpr int XCH = 24 * NT * XS;           // [6 xi][4 b][NT][XS]
  __shared__ __attribute__((aligned(16))) float smem[TILE > XCH ? TILE : XCH];

  const int tid = threadIdx.x;
  int bx, by, bz;
  xcd_tile(bx, by, bz);
  const int split = NSPLIT > 1 ? bx % NSPLIT : 0;
  if (NSPLIT > 1) bx /= NSPLIT;
  const int oy0 = by * 4 * TTY, ox0 = bx * 4 * TTX, nimg = bz;
  const int H = a.H, W = a.W;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int xi = NSPLIT == 1 ? wave >> 1 : wave;
  const int co_w = (NSPLIT == 1 ? (wave & 1) : split) * CW;  // first output channel of this wave
  const int co_x = NSPLIT == 1 ? co_w : 0;                    // ... within the exchange
  const int lane = tid & 63, li = lane & 15, lg = lane >> 4;

  // ---- A fragments (U) from L2, prefetched PF steps ahead; step s = 6 kc + nu ----
  constexpr int NSTEP = 6 * KC, PF = NSPLIT == 1 ? 2 : 1;
  const float* __restrict__ wl = a.wp + (size_t)6 * xi * KC * 16 * COUT + (size_t)(lg * COUT + co_w + li) * 4;
  auto wglob = [&](int s, int nb) -> f32x4 {
    const int kc = s / 6, nu = s % 6;
    return *reinterpret_cast<const f32x4*>(wl + (size_t)(nu * KC + kc) * 16 * COUT + nb * 64);
  };
  f32x4 av[PF + 1][NBW];
#pragma unroll
  for (int p = 0; p < PF; ++p)
#pragma unroll
    for (int nb = 0; nb < NBW; ++nb) av[p][nb] = wglob(p, nb);

  // ---- stage channels [KST h, KST (h+1)) of the input tile, columns split by (column mod 4);
  // zero outside the image ----
  constexpr int NSTAGE = LR * LCOL * C4;
  constexpr int NIT = (NSTAGE + NTHR - 1) / NTHR;
  constexpr int SBM = NSPLIT == 1 ? 10 : 5;  // loads in flight per thread (the second half's
                                            // staging runs beside live accumulators)
  constexpr int SB = NIT < SBM ? NIT : SBM;
  auto stage = [&](int h) {
#pragma unroll
    for (int i0 = 0; i0 < NIT; i0 += SB) {
      f32x4 tmp[SB];
#pragma unroll
      for (int i = 0; i < SB; ++i) {
        const int e = (i0 + i) * NTHR + tid;
        tmp[i] = f32x4{0.f, 0.f, 0.f, 0.f};
        if (i0 + i < NIT && e < NSTAGE) {
          const int c4 = e % C4, pe = e / C4, col = pe % LCOL, row = pe / LCOL;
          const int iy = oy0 - 1 + row, ix = ox0 - 1 + col;
          if (iy >= 0 && iy < H && ix >= 0 && ix < W) {
            const size_t off = ((size_t)(nimg * H + iy) * W + ix) * CIN + h * KST + c4 * 4;
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
        const int e = (i0 + i) * NTHR + tid;
        if (i0 + i < NIT && e < NSTAGE) {
          const int c4 = e % C4, pe = e / C4, col = pe % LCOL, row = pe / LCOL;
          *reinterpret_cast<f32x4*>(&smem[row * RS + ((col & 3) * HPP + (col >> 2)) * PS + c4 * 4]) = tmp[i];
        }
      }
    }
  };

  // ---- row xi of B^T d for tile li: r_j = sum_i BT[xi][i] d[i][j] over the non-zero i ----
  const int ty = li / TTX, tx = li % TTX;
  const int tbase = (4 * ty) * RS + tx * PS + lg * 4;
  // the fifth non-zero of row xi: BT[0][0] = BT[5][5] = 1; rows 1-4 add 0 x row 0 (branch-free)
  const int re = xi == 5 ? 5 : 0;
  const float c1 = kW4BT[xi][1], c2 = kW4BT[xi][2], c3 = kW4BT[xi][3], c4 = kW4BT[xi][4];
  const float ce = (xi == 0 || xi == 5) ? 1.f : 0.f;
  auto ld = [&](int i, int j, int kcl) -> f32x4 {
    return *reinterpret_cast<const f32x4*>(&smem[tbase + i * RS + ((j & 3) * HPP + (j >> 2)) * PS + kcl * 16]);
  };
  f32x4 V[6];
  // column j of that row for chunk kc, in the operation order c1 d1 + c2 d2 + c3 d3 + c4 d4 + ce de
  auto ldcol = [&](int j, int kcl, f32x4 (&d)[5]) {
    d[0] = ld(1, j, kcl);
    d[1] = ld(2, j, kcl);
    d[2] = ld(3, j, kcl);
    d[3] = ld(4, j, kcl);
    d[4] = ld(re, j, kcl);
  };
  auto rcol = [&](const f32x4 (&d)[5]) {
    f32x4 s = c1 * d[0];
    s = fma4s(c2, d[1], s);
    s = fma4s(c3, d[2], s);
    s = fma4s(c4, d[3], s);
    return fma4s(ce, d[4], s);
  };

  f32x4 acc[6][NBW];
#pragma unroll
  for (int nu = 0; nu < 6; ++nu)
#pragma unroll
    for (int nb = 0; nb < NBW; ++nb) acc[nu][nb] = f32x4{0.f, 0.f, 0.f, 0.f};

  // Software pipeline: while the MFMAs of point nu of chunk kc issue, column nu of chunk
  // kc + 1 is read (before them) and combined (after them); the six V of chunk kc + 1 follow
  // the chunk.  The transform's VALU work thus runs in the matrix pipe's shadow of the same
  // wave instead of between its MFMA phases.
#pragma unroll
  for (int h = 0; h < NHALF; ++h) {
    if (h > 0) __syncthreads();  // every wave is done with the previous channel half
    stage(h);
    __syncthreads();
    {
      f32x4 r[6], d[5];
#pragma unroll
      for (int j = 0; j < 6; ++j) {
        ldcol(j, 0, d);
        r[j] = rcol(d);
      }
#pragma unroll
      for (int nu = 0; nu < 6; ++nu) V[nu] = wcomb(kW4BT[nu], r);
    }
#pragma unroll
    for (int kcl = 0; kcl < KCH; ++kcl) {
      const int kc = h * KCH + kcl;
      const bool next = kcl + 1 < KCH;
      f32x4 rn[6], dn[5];
#pragma unroll
      for (int nu = 0; nu < 6; ++nu) {
        const int s = kc * 6 + nu;
        if (s + PF < NSTEP) {
#pragma unroll
          for (int nb = 0; nb < NBW; ++nb) av[(s + PF) % (PF + 1)][nb] = wglob(s + PF, nb);
        }
        if (next) ldcol(nu, kcl + 1, dn);
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int t = 0; t < 4; ++t)
#pragma unroll
          for (int nb = 0; nb < NBW; ++nb) acc[nu][nb] = mfma4(av[s % (PF + 1)][nb][t], V[nu][t], acc[nu][nb]);
        __builtin_amdgcn_sched_barrier(0);
        if (next) rn[nu] = rcol(dn);
      }
      if (next) {
#pragma unroll
        for (int nu = 0; nu < 6; ++nu) V[nu] = wcomb(kW4BT[nu], rn);
      }
    }
  }

  // ---- T = M A over nu (per wave), exchanged through LDS (the input tile is dead) ----
  __syncthreads();
#pragma unroll
  for (int nb = 0; nb < NBW; ++nb) {
    const f32x4 m[6] = {acc[0][nb], acc[1][nb], acc[2][nb], acc[3][nb], acc[4][nb], acc[5][nb]};
#pragma unroll
    for (int b = 0; b < 4; ++b)
      *reinterpret_cast<f32x4*>(&smem[((xi * 4 + b) * NT + li) * XS + co_x + nb * 16 + lg * 4]) = wcomb(kW4AT[b], m);
  }
  __syncthreads();

  // ---- Y = A^T T: one (output column b, tile, 4-channel quad) per thread and pass ----
  constexpr int Q4 = CWG / 4, NTASK = 4 * NT * Q4;
  const int Ho = a.Ho, Wo = a.Wo;
#pragma unroll
  for (int it0 = 0; it0 < NTASK; it0 += NTHR) {
    const int it = it0 + tid;
    if (NTASK % NTHR != 0 && it >= NTASK) break;
    const int q = it % Q4, tile = (it / Q4) % NT, b = it / (Q4 * NT);
    const int tty = tile / TTX, ttx = tile % TTX;
    const int ox = ox0 + 4 * ttx + b;
    f32x4 T[6];
#pragma unroll
    for (int x2 = 0; x2 < 6; ++x2) T[x2] = *reinterpret_cast<const f32x4*>(&smem[((x2 * 4 + b) * NT + tile) * XS + 4 * q]);
    if (ox >= Wo) continue;
    const int co = split * CWG + 4 * q;
    const f32x4 bb = *reinterpret_cast<const f32x4*>(a.bias + co);
#pragma unroll
    for (int ay = 0; ay < 4; ++ay) {
      const int oy = oy0 + 4 * tty + ay;
      if (oy >= Ho) break;
      conv_out4<ACT, RES, OUT>(a, wcomb(kW4AT[ay], T), bb, ((size_t)(nimg * Ho + oy) * Wo + ox) * COUT + co);
    }
  }
}

template <int CIN, int COUT, int TTY, int NSPLIT, int ACT, bool RES, int IN, int OUT>
static void launch_wino4(const ConvArgs& a, int n, hipStream_t s) {
  constexpr int OW = 4 * Wino4Geom<TTY>::TTX, OH = 4 * TTY;
  dim3 grid(((a.Wo + OW - 1) / OW) * NSPLIT, (a.Ho + OH - 1) / OH, n);
  hipLaunchKernelGGL((conv3x3_wino4_kernel<CIN, COUT, TTY, NSPLIT, ACT, RES, IN, OUT>), grid,
                     dim3(NSPLIT == 1 ? 768 : 384), 0, s, a);
}

}  // namespace tic

// Winograd F(4x4,3x3) entry: th = output rows per workgroup (4 TTY), 256 / th columns,
// weight source 5 = the F(4x4,3x3) packing of U (passed as ConvArgs::wp).
#define TIC_WINO4(CIN, COUT, TTY, NSPLIT, ACT, RES, IN, OUT)                          \
  { MODE_S1, CIN, COUT, ACT, RES, IN, OUT, 4 * TTY, 1, NSPLIT, 5,                      \
    &tic::launch_wino4<CIN, COUT, TTY, NSPLIT, ACT, RES, IN, OUT> }
