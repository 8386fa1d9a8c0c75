// conv3x3_wino.h — stride-1 'SAME' 3x3 convolutions as Winograd F(2x2, 3x3) on the matrix
// cores: the res_block convs (basic_block/basic_block.py:74-93), encode_4 / decode_4 of
// model_0/1 (model_0/model.py:124-134,159-169) and the rmbe net's conv_3/4.
//
// Per 2x2 output tile with 4x4 input patch d:  Y = A^T [ U (.) V ] A,  U = G g G^T,
// V = B^T d B.  A tile costs 16 transform points x Cin x Cout MACs instead of the direct
// form's 4 pixels x 9 taps x Cin x Cout: 2.25x fewer matrix-core cycles.  For each point
// p = (xi, nu) the products are one GEMM, M = Cout (A = U_p, transformed on the host in
// double and rounded once), N = tiles (B = V_p), K = Cin, on v_mfma_f32_16x16x4_f32 with
// conv3x3_kernel's fragment layout (lane group g supplies channel 16 kc + 4 g + t to MFMA t).
//
// Workgroup: NT = 16 NN tiles (TTY rows x TTX columns of 2x2 tiles) x Cout / NSPLIT output
// channels.  Wave xi owns the points (xi, 0..3): B^T has two non-zeros per row, so a lane
// forms row xi of B^T d from two staged input rows and its tile's 4 columns, then the four
// column combinations V_(xi,nu) in registers — transformed inputs never touch LDS or HBM.
// The input tile (2 TTY + 2 rows x 2 TTX + 2 columns, zero outside the image = SAME pad) is
// staged with its columns split by parity, so the lanes reading column 2 tx + j of 16
// consecutive tiles read consecutive LDS pixels (pixel stride Cin + 8 floats, row pitch a
// multiple of 4 pixels: conflict-free ds_read_b128 as in conv3x3_kernel).  After the K loop
// each wave applies A on the nu side (T = M A), the waves swap T through LDS (aliasing the
// dead input tile) and every thread finishes Y = A^T T for one tile x 4 channels, then the
// epilogue of my_conv2d: + bias, ReLU / identity, + residual, quantiser.
//
// Summation order per output is fixed by the transforms — M over K in MFMA order (16-channel
// chunk, t, lane group), then T and Y in the orders written below — and does not depend on
// TTY, NN or NSPLIT: all Winograd tilings are bit-identical to each other.  They differ from
// the direct form by rounding only, so the form is a policy (handle option "s1_form"), never
// a tuning outcome — as for the last layer's forms.
#pragma once
#include "conv3x3.h"

namespace tic {

template <int TTY, int NN>
struct WinoGeom {
  static constexpr int NT = 16 * NN;        // 2x2 output tiles per workgroup
  static constexpr int TTX = NT / TTY;      // tiles per tile row
  static constexpr int LR = 2 * TTY + 2;    // staged input rows
  static constexpr int LCOL = 2 * TTX + 2;  // staged input columns
  static constexpr int HP = TTX + 2;        // pixels per column-parity plane (TTX + 1 used)
  static constexpr int RP = 2 * HP;         // pixels per staged row (a multiple of 4)
};

// + bias, activation, + residual, then a 16-byte f32 store or the quantiser
// (conv3x3_kernel's epilogue, same operations in the same order).
template <int ACT, bool RES, int OUT>
__device__ __forceinline__ void conv_out4(const ConvArgs& a, f32x4 v, const f32x4 bb, size_t o) {
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
    const uint32_t q = quant1(v.x, a.qscale) | (quant1(v.y, a.qscale) << 8) | (quant1(v.z, a.qscale) << 16) |
                       (quant1(v.w, a.qscale) << 24);
    *reinterpret_cast<uint32_t*>(a.qout + o) = q;
  }
}

// Weights (ConvArgs::wp): U packed [16 p][Cin/16][4 g][Cout][4 t], p = 4 xi + nu.
template <int CIN, int COUT, int TTY, int NN, int NSPLIT, int ACT, bool RES, int IN, int OUT>
__global__ void __launch_bounds__(256) conv3x3_wino_kernel(const ConvArgs a) {
  using G = WinoGeom<TTY, NN>;
  constexpr int NT = G::NT, TTX = G::TTX, LR = G::LR, LCOL = G::LCOL, HP = G::HP, RP = G::RP;
  static_assert(CIN % 16 == 0 && COUT % 16 == 0 && TTX * TTY == NT && TTX % 8 == 0, "tile");
  constexpr int PS = CIN + 8, KC = CIN / 16, C4 = CIN / 4;
  constexpr int CWG = COUT / NSPLIT;
  static_assert(CWG % 16 == 0, "channel split");
  constexpr int NBW = CWG / 16;       // 16-channel output blocks per wave
  constexpr int TILE = LR * RP * PS;  // floats of the staged input tile
  constexpr int XS = CWG + 8;         // exchange pitch per (point row, column, tile), == 8 mod 16
  constexpr int XCH = 8 * NT * XS;    // floats of the T exchange [4 xi][2 b][NT][XS]
  __shared__ __attribute__((aligned(16))) float smem[TILE > XCH ? TILE : XCH];

  const int tid = threadIdx.x;
  int lbx, lby, lbz;
  xcd_tile(lbx, lby, lbz);
  const int split = NSPLIT > 1 ? lbx % NSPLIT : 0;
  const int bx = NSPLIT > 1 ? lbx / NSPLIT : lbx;
  const int oy0 = lby * (2 * TTY), ox0 = bx * (2 * TTX), nimg = lbz;
  const int H = a.H, W = a.W;
  const int xi = __builtin_amdgcn_readfirstlane(tid >> 6);  // B^T row of this wave
  const int lane = tid & 63, li = lane & 15, lg = lane >> 4;
  const int co_wg = split * CWG;

  // ---- A fragments (U) straight from L2, prefetched PF steps ahead; step s = 4 kc + nu ----
  constexpr int NSTEP = 4 * KC, PF = 3;
  const float* __restrict__ wl = a.wp + (size_t)xi * 64 * KC * COUT + (size_t)(lg * COUT + co_wg + li) * 4;
  auto wglob = [&](int s, int nb) -> f32x4 {
    const int kc = s >> 2, nu = s & 3;
    return *reinterpret_cast<const f32x4*>(wl + (size_t)(nu * KC + kc) * 16 * COUT + nb * 64);
  };
  f32x4 av[PF + 1][NBW];
#pragma unroll
  for (int p = 0; p < PF; ++p)
#pragma unroll
    for (int nb = 0; nb < NBW; ++nb) av[p][nb] = wglob(p, nb);

  // ---- stage the input tile, columns split by parity; zero outside the image ----
  constexpr int NSTAGE = LR * LCOL * C4;
  constexpr int NIT = (NSTAGE + 255) / 256;
  constexpr int SB = NIT < 12 ? NIT : 12;
#pragma unroll
  for (int i0 = 0; i0 < NIT; i0 += SB) {
    f32x4 tmp[SB];
#pragma unroll
    for (int i = 0; i < SB; ++i) {
      const int e = (i0 + i) * 256 + tid;
      tmp[i] = f32x4{0.f, 0.f, 0.f, 0.f};
      if (i0 + i < NIT && e < NSTAGE) {
        const int c4 = e % C4, pe = e / C4, col = pe % LCOL, row = pe / LCOL;
        const int iy = oy0 - a.pad_y + row, ix = ox0 - a.pad_x + col;
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
        const int c4 = e % C4, pe = e / C4, col = pe % LCOL, row = pe / LCOL;
        *reinterpret_cast<f32x4*>(&smem[(row * RP + (col & 1) * HP + (col >> 1)) * PS + c4 * 4]) = tmp[i];
      }
    }
  }
  __syncthreads();

  // ---- row xi of B^T d from input rows iA, iB: r = sA d[iA] + sB d[iB] (exact signs) ----
  const int iA = xi == 0 ? 0 : 1, iB = xi == 3 ? 3 : 2;
  const float sA = xi == 2 ? -1.f : 1.f, sB = (xi == 0 || xi == 3) ? -1.f : 1.f;
  int offA[NN], offB[NN];
#pragma unroll
  for (int nn = 0; nn < NN; ++nn) {
    const int tile = nn * 16 + li, ty = tile / TTX, tx = tile % TTX;
    offA[nn] = ((2 * ty + iA) * RP + tx) * PS + lg * 4;
    offB[nn] = ((2 * ty + iB) * RP + tx) * PS + lg * 4;
  }
  f32x4 d[NN][2][4];
  auto load_d = [&](int kc) {
#pragma unroll
    for (int nn = 0; nn < NN; ++nn)
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int cj = ((j & 1) * HP + (j >> 1)) * PS + kc * 16;  // column 2 tx + j
        d[nn][0][j] = *reinterpret_cast<const f32x4*>(&smem[offA[nn] + cj]);
        d[nn][1][j] = *reinterpret_cast<const f32x4*>(&smem[offB[nn] + cj]);
      }
  };
  f32x4 V[NN][4];
  auto transform = [&]() {
#pragma unroll
    for (int nn = 0; nn < NN; ++nn) {
      f32x4 r[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) r[j] = sA * d[nn][0][j] + sB * d[nn][1][j];
      V[nn][0] = r[0] - r[2];
      V[nn][1] = r[1] + r[2];
      V[nn][2] = r[2] - r[1];
      V[nn][3] = r[1] - r[3];
    }
  };

  f32x4 acc[4][NN][NBW];
#pragma unroll
  for (int nu = 0; nu < 4; ++nu)
#pragma unroll
    for (int nn = 0; nn < NN; ++nn)
#pragma unroll
      for (int nb = 0; nb < NBW; ++nb) acc[nu][nn][nb] = f32x4{0.f, 0.f, 0.f, 0.f};

  load_d(0);
  transform();
#pragma unroll
  for (int kc = 0; kc < KC; ++kc) {
    if (kc + 1 < KC) load_d(kc + 1);  // next chunk's ds_reads fly under this chunk's MFMAs
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int nu = 0; nu < 4; ++nu) {
      const int s = kc * 4 + nu;
      if (s + PF < NSTEP) {
#pragma unroll
        for (int nb = 0; nb < NBW; ++nb) av[(s + PF) % (PF + 1)][nb] = wglob(s + PF, nb);
      }
      // keep each weight load PF steps ahead of its use (the scheduler otherwise sinks the
      // loads next to their consumers inside the chunk and the prefetch collapses)
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int t = 0; t < 4; ++t)
#pragma unroll
        for (int nn = 0; nn < NN; ++nn)
#pragma unroll
          for (int nb = 0; nb < NBW; ++nb)
            acc[nu][nn][nb] = mfma4(av[s % (PF + 1)][nb][t], V[nn][nu][t], acc[nu][nn][nb]);
      __builtin_amdgcn_sched_barrier(0);
    }
    __builtin_amdgcn_sched_barrier(0);
    if (kc + 1 < KC) transform();
  }

  // ---- T = M A over nu (per wave), exchanged through LDS (the input tile is dead) ----
  __syncthreads();
#pragma unroll
  for (int nn = 0; nn < NN; ++nn)
#pragma unroll
    for (int nb = 0; nb < NBW; ++nb) {
      const f32x4 m0 = acc[0][nn][nb], m1 = acc[1][nn][nb], m2 = acc[2][nn][nb], m3 = acc[3][nn][nb];
      float* x = &smem[(xi * 2 * NT + nn * 16 + li) * XS + nb * 16 + lg * 4];
      *reinterpret_cast<f32x4*>(x) = (m0 + m1) + m2;
      *reinterpret_cast<f32x4*>(x + NT * XS) = (m1 - m2) - m3;
    }
  __syncthreads();

  // ---- Y = A^T T: one (tile, 4-channel quad) per thread and pass, then the epilogue ----
  constexpr int Q4 = CWG / 4;
  const int Ho = a.Ho, Wo = a.Wo;
#pragma unroll
  for (int it0 = 0; it0 < NT * Q4; it0 += 256) {
    const int it = it0 + tid;
    if ((NT * Q4) % 256 != 0 && it >= NT * Q4) break;
    const int tile = it / Q4, q = it % Q4;
    const int ty = tile / TTX, tx = tile % TTX;
    f32x4 T[4][2];
#pragma unroll
    for (int x2 = 0; x2 < 4; ++x2)
#pragma unroll
      for (int b = 0; b < 2; ++b)
        T[x2][b] = *reinterpret_cast<const f32x4*>(&smem[((x2 * 2 + b) * NT + tile) * XS + 4 * q]);
    const int co = co_wg + 4 * q;
    const f32x4 bb = *reinterpret_cast<const f32x4*>(a.bias + co);
#pragma unroll
    for (int ay = 0; ay < 2; ++ay)
#pragma unroll
      for (int b = 0; b < 2; ++b) {
        const int oy = oy0 + 2 * ty + ay, ox = ox0 + 2 * tx + b;
        if (oy >= Ho || ox >= Wo) continue;
        const f32x4 y = ay == 0 ? (T[0][b] + T[1][b]) + T[2][b] : (T[1][b] - T[2][b]) - T[3][b];
        conv_out4<ACT, RES, OUT>(a, y, bb, ((size_t)(nimg * Ho + oy) * Wo + ox) * COUT + co);
      }
  }
}

template <int CIN, int COUT, int TTY, int NN, int NSPLIT, int ACT, bool RES, int IN, int OUT>
static void launch_wino(const ConvArgs& a, int n, hipStream_t s) {
  constexpr int OW = 2 * WinoGeom<TTY, NN>::TTX, OH = 2 * TTY;
  dim3 grid(((a.Wo + OW - 1) / OW) * NSPLIT, (a.Ho + OH - 1) / OH, n);
  hipLaunchKernelGGL((conv3x3_wino_kernel<CIN, COUT, TTY, NN, NSPLIT, ACT, RES, IN, OUT>), grid, dim3(256), 0, s, a);
}

}  // namespace tic

// Winograd stride-1 entry: th = output rows per workgroup (2 TTY), wr = NN (16-tile blocks
// per workgroup), weight source 4 = the Winograd packing of U (passed as ConvArgs::wp).
#define TIC_WINO(CIN, COUT, TTY, NN, NSPLIT, ACT, RES, IN, OUT) \
  { MODE_S1, CIN, COUT, ACT, RES, IN, OUT, 2 * TTY, NN, NSPLIT, 4, \
    &tic::launch_wino<CIN, COUT, TTY, NN, NSPLIT, ACT, RES, IN, OUT> }
