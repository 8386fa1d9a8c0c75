// conv3x3_pwino.h — stride-2 'SAME' 3x3 convolutions and their transposes as polyphase
// Winograd products on the matrix cores (stride-2 / transposed form 1, handle option
// "s2_form"): the standalone analysis / synthesis layers of models 0-3, the rmbe net's
// conv_2 / conv_5 (model_0/model.py:62-96,198-222, model_3/model.py:62-161,157-286,
// basic_block/basic_block.py:27-57).
//
// A stride-2 3-tap correlation splits into its phases: y[i] = w0 x[2i] + w2 x[2i+2] (the
// even samples, a 2-tap correlation) + w1 x[2i+1] (the odd samples, one tap).  Two outputs
// (y0, y1) read five samples s0..s4; the even part is Winograd F(2,2) — (s0 - s2) w0,
// s2 (w0 + w2), (s4 - s2) w2 — and the odd part two plain products s1 w1, s3 w1: five
// transform points for two outputs instead of six products,
//   B^T s = (s0 - s2, s2, s4 - s2, s1, s3),  U = (w0, w0 + w2, w2, w1, w1),
//   y0 = (M0 + M1) + M3,  y1 = (M1 + M2) + M4.
// The transposed conv (stride 2, 'SAME', output 2H: y[2m] = W0 x[m] + W2 x[m-1],
// y[2m+1] = W1 x[m]) is the same split read the other way: an input pair (m, m+1) with
// d = (x[m-1], x[m], x[m+1]) gives the four outputs 2m..2m+3 from
//   B^T d = (d0 - d1, d1, d2 - d1, d1, d2),  U = (W2, W2 + W0, W0, W1, W1),
//   y[2m] = M0 + M1,  y[2m+1] = M3,  y[2m+2] = M1 + M2,  y[2m+3] = M4.
// In 2-D a tile is 5 x 5 = 25 transform points (2x2 outputs of the stride-2 conv, 4x4 of the
// transpose) against the direct form's 36 products: 0.69x the matrix-core cycles.  The
// transforms have coefficients 0 / +-1 (exact); U = G g G^T is formed on the host in double
// and rounded once (tic_runtime.cpp pack_pwino).
//
// Workgroup: NT = 16 NNB tiles in one tile row; wave w owns output-channel block w % NBT and
// tile block w / NBT (16 tiles), i.e. ALL 25 points of its 16 tiles x 16 channels — so the
// output transform Y = A^T M A runs in registers, with no exchange.  For each 16-channel
// chunk and point row xi a lane forms row xi of B^T d from one or two staged input rows (its
// tile's five / three columns), then the five column combinations V_(xi,nu), and issues the
// five point GEMMs (M = 16 output channels, A = U_p from L2 through a buffer resource,
// prefetched PF steps ahead; N = 16 tiles, B = V_p; K = Cin on v_mfma_f32_16x16x4_f32 in
// conv3x3_kernel's fragment layout).  The input tile (5 x (4 NT + 1) pixels for stride 2,
// 3 x (2 NT + 1) for the transpose, zero outside the image) is staged once with its columns
// split by (column mod 4) / parity, so the 16 tiles of a read hit 16 consecutive pixels of a
// plane (pixel stride Cin + 8 floats: conflict-free ds_read_b128, as in conv3x3_kernel).
//
// Summation order per output: M over K in MFMA order (16-channel chunk, t, lane group), then
// the output transform in the order written below, then my_conv2d's epilogue (conv_out4).
// It does not depend on the launch geometry; it differs from the direct form (0) by rounding
// only, so the form is a policy, never a tuning outcome (tic_runtime.cpp layer_form).
#pragma once
#include "conv3x3_wino.h"

namespace tic {

template <int MODE, int NNB>
struct PwinoGeom {
  static constexpr int NT = 16 * NNB;                            // tiles per workgroup (one tile row)
  static constexpr int LR = MODE == MODE_S2 ? 5 : 3;             // staged input rows
  static constexpr int LCOL = MODE == MODE_S2 ? 4 * NT + 1 : 2 * NT + 1;  // staged input columns
  static constexpr int NPL = MODE == MODE_S2 ? 4 : 2;            // column planes
  static constexpr int HP = NT + 1;                              // pixels per plane
  static constexpr int RP = NPL * HP;                            // pixels per staged row
  static constexpr int NCOL = MODE == MODE_S2 ? 5 : 3;           // input columns per tile
  static constexpr int OPT = MODE == MODE_S2 ? 2 : 4;            // outputs per tile and axis
};

// The transforms, shared with the chain's decode_2 behind its tail (wino_chain.h), which must
// reproduce this kernel bit for bit.  B^T over the NCOL values of one row / column:
template <int MODE>
__device__ __forceinline__ void pw_bt(const f32x4 (&r)[MODE == MODE_S2 ? 5 : 3], f32x4 (&v)[5]) {
  if constexpr (MODE == MODE_S2) {
    v[0] = r[0] - r[2];
    v[1] = r[2];
    v[2] = r[4] - r[2];
    v[3] = r[1];
    v[4] = r[3];
  } else {
    v[0] = r[0] - r[1];
    v[1] = r[1];
    v[2] = r[2] - r[1];
    v[3] = r[1];
    v[4] = r[2];
  }
}
// transpose: row xi of B^T d from the tile's three input rows d0..d2 at column j
__device__ __forceinline__ f32x4 pw_row_t2(int xi, const f32x4& d0, const f32x4& d1, const f32x4& d2) {
  return xi == 0 ? d0 - d1 : (xi == 2 ? d2 - d1 : (xi == 4 ? d2 : d1));
}
// A^T over the five points of one row / column
template <int MODE>
__device__ __forceinline__ void pw_at(const f32x4 (&m)[5], f32x4 (&o)[MODE == MODE_S2 ? 2 : 4]) {
  if constexpr (MODE == MODE_S2) {
    o[0] = (m[0] + m[1]) + m[3];
    o[1] = (m[1] + m[2]) + m[4];
  } else {
    o[0] = m[0] + m[1];
    o[1] = m[3];
    o[2] = m[1] + m[2];
    o[3] = m[4];
  }
}

// Weights (ConvArgs::wp): U packed [25 p = 5 xi + nu][Cin/16][4 g][Cout][4 t].
// KS: the input channels are staged in KS slices (KS = 2 where the whole Cin would not leave
// room for two workgroups per CU: the 64-channel stride-2 tiles), the K loop running over one
// slice while it is resident.
template <int MODE, int CIN, int COUT, int NNB>
struct PwinoCfg {
  using G = PwinoGeom<MODE, NNB>;
  static constexpr int KS = G::LR * G::RP * (CIN + 8) * 4 > 80 * 1024 ? 2 : 1;
  static constexpr int CS = CIN / KS;  // channels per staged slice
  static constexpr int PS = CS + 8;    // pixel stride (== 8 mod 16: conflict-free ds_read_b128)
};

template <int MODE, int CIN, int COUT, int NNB, int ACT, bool RES, int IN, int OUT>
__global__ void __launch_bounds__(64 * (COUT / 16) * NNB) conv3x3_pwino_kernel(const ConvArgs a) {
  using G = PwinoGeom<MODE, NNB>;
  using CF = PwinoCfg<MODE, CIN, COUT, NNB>;
  constexpr int NT = G::NT, LR = G::LR, LCOL = G::LCOL, HP = G::HP, RP = G::RP, NCOL = G::NCOL, NPL = G::NPL;
  static_assert(CIN % 16 == 0 && COUT % 16 == 0, "channels");
  constexpr int NBT = COUT / 16, NTH = 64 * NBT * NNB;
  constexpr int KS = CF::KS, CS = CF::CS, PS = CF::PS, KC = CIN / 16, KCS = CS / 16, C4 = CS / 4;
  static_assert(CS % 16 == 0, "slice");
  __shared__ __attribute__((aligned(16))) float smem[LR * RP * PS];

  const int tid = threadIdx.x;
  int lbx, lby, lbz;
  xcd_tile(lbx, lby, lbz);
  const int nimg = lbz;
  const int H = a.H, W = a.W;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int cb = wave % NBT, nb = wave / NBT;
  const int lane = tid & 63, li = lane & 15, lg = lane >> 4;
  // first staged input row / column (stride 2: of the tile row's 2 output rows; transpose:
  // the row above its 2 input rows)
  const int ry = MODE == MODE_S2 ? 2 * (2 * lby) - a.pad_y : 2 * lby - 1;
  const int rx = MODE == MODE_S2 ? 2 * (2 * NT * lbx) - a.pad_x : 2 * NT * lbx - 1;

  // ---- U fragments straight from L2 through a buffer resource, PF steps (of 4 MFMAs) ahead.
  //      Step order: chunk kc, then the point rows in the order XO, then nu ----
  // stride 2: the staged rows stream in the order 2, 0, 4, 1, 3, one per point row (xi = 1,
  // 0, 2, 3, 4; row 2 kept for xi 0 and 2); transpose: xi in order
  constexpr int XO[5] = {MODE == MODE_S2 ? 1 : 0, MODE == MODE_S2 ? 0 : 1, 2, 3, 4};
  // a point row's five U fragments arrive one row (5 steps) ahead, in a ring of two rows
  constexpr int NSTEP = 25 * KC, PF = 5, RING = PF + 5;
  const __amdgpu_buffer_rsrc_t wrs = weight_rsrc(a.wp, 25 * CIN * COUT * 4);
  const int wlb = (lg * COUT + cb * 16 + li) * 16;
  auto wglob = [&](int s) -> f32x4 {
    const int kc = s / 25, q = (s % 25) / 5, nu = s % 5;
    const int p = 5 * XO[q] + nu;
    return weight_frag(wrs, wlb, ((p * KC + kc) * 4 * COUT * 4) * 4);
  };
  f32x4 av[RING];
#pragma unroll
  for (int p = 0; p < PF; ++p) av[p] = wglob(p);

  // ---- stage channel slice h of the input tile, columns split into NPL planes; zero
  //      outside the image ----
  constexpr int NSTAGE = LR * LCOL * C4;
  constexpr int NIT = (NSTAGE + NTH - 1) / NTH;
  constexpr int SB = NIT < 12 ? NIT : 12;
  const size_t img_bytes = (size_t)H * W * CIN * 4;
  const bool rsrc_in = IN == IN_F32 && img_bytes < 0xFFFFFF00ull;
  const __amdgpu_buffer_rsrc_t irs =
      weight_rsrc(reinterpret_cast<const float*>(a.in) + (rsrc_in ? (size_t)nimg * H * W * CIN : 0),
                  (int)(unsigned)(rsrc_in ? img_bytes : 16));
  auto stage = [&](int h) {
#pragma unroll
    for (int i0 = 0; i0 < NIT; i0 += SB) {
      f32x4 tmp[SB];
#pragma unroll
      for (int i = 0; i < SB; ++i) {
        const int e = (i0 + i) * NTH + tid;
        tmp[i] = f32x4{0.f, 0.f, 0.f, 0.f};
        if (i0 + i < NIT && (NSTAGE % NTH == 0 || e < NSTAGE)) {
          const int c4 = e % C4 + h * C4, pe = e / C4, col = pe % LCOL, row = pe / LCOL;
          const int iy = ry + row, ix = rx + col;
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
        const int e = (i0 + i) * NTH + tid;
        if (i0 + i < NIT && (NSTAGE % NTH == 0 || e < NSTAGE)) {
          const int c4 = e % C4, pe = e / C4, col = pe % LCOL, row = pe / LCOL;
          *reinterpret_cast<f32x4*>(&smem[(row * RP + (col % NPL) * HP + col / NPL) * PS + c4 * 4]) = tmp[i];
        }
      }
    }
  };

  // staged pixel of (row, column j of this lane's tile): tile t = 16 nb + li starts at
  // column NPL t, i.e. plane j % NPL, index t + j / NPL; kl = chunk within the slice
  const int t = nb * 16 + li;
  auto ld = [&](int row, int j, int kl) -> f32x4 {
    return *reinterpret_cast<const f32x4*>(&smem[(row * RP + (j % NPL) * HP + t + j / NPL) * PS + kl * 16 + lg * 4]);
  };
  // B^T applied to the NCOL values of one row / column (exact: coefficients 0, +-1)
  auto bt = [&](const f32x4 (&r)[NCOL], f32x4 (&v)[5]) { pw_bt<MODE>(r, v); };

  f32x4 acc[25];
#pragma unroll
  for (int p = 0; p < 25; ++p) acc[p] = f32x4{0.f, 0.f, 0.f, 0.f};
  // the five point GEMMs of point row xi at chunk kc and row step q (weights step 5 q + nu)
  // (t outer, nu inner: consecutive MFMAs feed five different accumulators, so no MFMA waits
  // for the one before it; each point still sums over t in order — the same bits)
  auto row_mfma = [&](int q, int xi, const f32x4 (&V)[5]) {
    f32x4 u[5];
#pragma unroll
    for (int nu = 0; nu < 5; ++nu) u[nu] = av[(5 * q + nu) % RING];
#pragma unroll
    for (int nu = 0; nu < 5; ++nu) {
      const int s = 5 * q + nu + PF;
      if (s < NSTEP) av[s % RING] = wglob(s);
    }
#pragma unroll
    for (int tt = 0; tt < 4; ++tt)
#pragma unroll
      for (int nu = 0; nu < 5; ++nu) acc[5 * xi + nu] = mfma4(u[nu][tt], V[nu][tt], acc[5 * xi + nu]);
  };

#pragma unroll
  for (int h = 0; h < KS; ++h) {
    if (h > 0) __syncthreads();  // every wave is done with slice h - 1
    stage(h);
    __syncthreads();
    if constexpr (MODE == MODE_S2) {
      // row steps q: staged row RO[q % 5] of chunk q / 5, feeding point row XO[q % 5]
      constexpr int RO[5] = {2, 0, 4, 1, 3};
      constexpr int NQ = 5 * KCS;
      f32x4 rb[2][5], r2[5];
      auto ldrow = [&](int q, f32x4 (&dst)[5]) {
#pragma unroll
        for (int j = 0; j < 5; ++j) dst[j] = ld(RO[q % 5], j, q / 5);
      };
      ldrow(0, rb[0]);
#pragma unroll
      for (int q = 0; q < NQ; ++q) {
        if (q + 1 < NQ) ldrow(q + 1, rb[(q + 1) & 1]);  // in flight under this step's MFMAs
        __builtin_amdgcn_sched_barrier(0);
        const int qq = q % 5;
        f32x4 r[5], V[5];
#pragma unroll
        for (int j = 0; j < 5; ++j) {
          if (qq == 0) r2[j] = rb[q & 1][j];
          r[j] = qq == 0 ? r2[j] : (qq <= 2 ? rb[q & 1][j] - r2[j] : rb[q & 1][j]);
        }
        bt(r, V);
        row_mfma(h * NQ + q, XO[qq], V);
        __builtin_amdgcn_sched_barrier(0);
      }
    } else {
      f32x4 db[2][3][3];
      auto ldchunk = [&](int kl, f32x4 (&dst)[3][3]) {
#pragma unroll
        for (int r = 0; r < 3; ++r)
#pragma unroll
          for (int j = 0; j < 3; ++j) dst[r][j] = ld(r, j, kl);
      };
      ldchunk(0, db[0]);
#pragma unroll
      for (int kl = 0; kl < KCS; ++kl) {
        if (kl + 1 < KCS) ldchunk(kl + 1, db[(kl + 1) & 1]);
        __builtin_amdgcn_sched_barrier(0);
        const f32x4(&d)[3][3] = db[kl & 1];
#pragma unroll
        for (int xi = 0; xi < 5; ++xi) {
          f32x4 r[3], V[5];
#pragma unroll
          for (int j = 0; j < 3; ++j)
            r[j] = pw_row_t2(xi, d[0][j], d[1][j], d[2][j]);
          bt(r, V);
          row_mfma((h * KCS + kl) * 5 + xi, xi, V);
        }
        __builtin_amdgcn_sched_barrier(0);
      }
    }
  }

  // ---- Y = A^T M A in registers (lane: tile t, output channels 16 cb + 4 lg .. + 3) ----
  // T[xi][b] = A over nu, then Y[a][b] = A over xi, in the orders written
  constexpr int O = G::OPT;
  auto at = [&](const f32x4 (&m)[5], f32x4 (&o)[O]) { pw_at<MODE>(m, o); };
  f32x4 T[5][O];
#pragma unroll
  for (int xi = 0; xi < 5; ++xi) {
    f32x4 m[5];
#pragma unroll
    for (int nu = 0; nu < 5; ++nu) m[nu] = acc[5 * xi + nu];
    at(m, T[xi]);
  }
  const int co = cb * 16 + lg * 4;
  const f32x4 bb = *reinterpret_cast<const f32x4*>(a.bias + co);
  const int Ho = a.Ho, Wo = a.Wo;
  const int oy0 = MODE == MODE_S2 ? 2 * lby : 4 * lby;
  const int ox0 = (MODE == MODE_S2 ? 2 : 4) * (NT * lbx + t);
#pragma unroll
  for (int b = 0; b < O; ++b) {
    f32x4 m[5], y[O];
#pragma unroll
    for (int xi = 0; xi < 5; ++xi) m[xi] = T[xi][b];
    at(m, y);
#pragma unroll
    for (int ay = 0; ay < O; ++ay) {
      const int oy = oy0 + ay, ox = ox0 + b;
      if (oy >= Ho || ox >= Wo) continue;
      conv_out4<ACT, RES, OUT>(a, y[ay], bb, ((size_t)(nimg * Ho + oy) * Wo + ox) * COUT + co);
    }
  }
}

template <int MODE, int CIN, int COUT, int NNB, int ACT, bool RES, int IN, int OUT>
static void launch_pwino(const ConvArgs& a, int n, hipStream_t s) {
  constexpr int NT = 16 * NNB;
  // tile rows / columns: stride 2 over the output grid (2 x 2 outputs per tile), the
  // transpose over its input grid (2 x 2 input positions per tile)
  const int gy = MODE == MODE_S2 ? a.Ho : a.H, gx = MODE == MODE_S2 ? a.Wo : a.W;
  dim3 grid((((gx + 1) / 2) + NT - 1) / NT, (gy + 1) / 2, n);
  hipLaunchKernelGGL((conv3x3_pwino_kernel<MODE, CIN, COUT, NNB, ACT, RES, IN, OUT>), grid,
                     dim3(64 * (COUT / 16) * NNB), 0, s, a);
}

}  // namespace tic

// polyphase Winograd entry: th = 2 rows of the layer's grid per workgroup, wr = NNB (16-tile
// blocks), weight source 6 = the polyphase packing of U (ConvArgs::wp)
#define TIC_PWINO(MODE, CIN, COUT, NNB, ACT, RES, IN, OUT) \
  { MODE, CIN, COUT, ACT, RES, IN, OUT, 2, NNB, 1, 6,      \
    &tic::launch_pwino<MODE, CIN, COUT, NNB, ACT, RES, IN, OUT> }
