// conv3x3_wino4.h — stride-1 'SAME' 3x3 convolutions as Winograd F(4x4, 3x3) on the matrix
// cores: the res_block convs of model_3 (basic_block/basic_block.py:74-93, model_3/model.py:
// 66-150,191-281), the rmbe net's conv_3/4 (submit/2/rmbe/model.py) and model_0/1's 16x16
// stage (model_0/model.py:98-194: the res-block convs, encode_4 with the quantiser epilogue,
// decode_4 with the dequantiser table on its input).  Stride-1 form 2 (handle option
// "s1_form" = 2; conv3x3_wino.h is form 1).
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
// Workgroup: 768 threads = 12 waves (3 per SIMD), 16 4x4 tiles (TTY rows x 16/TTY columns of
// tiles; TTY = 1, 2, 4 for 64-, 32-, 16-wide layers).  Wave w owns B^T row xi = w / 2 and
// output-channel half w % 2: it forms row xi of B^T d from the staged input rows (rows 1..4
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
// One workgroup per CU (104-117 KB of LDS, 168 VGPRs at 3 waves per SIMD).  Measured and not
// kept: two 384-thread workgroups per tile splitting the output channels, each staging the
// input in two channel halves (65 KB, two per CU): 1.4x slower; a persistent tiling walking
// tiles with the next tile's input in registers (loaded while the output transform and the
// stores of the current one run): 5-15 % slower (it spills, and the staging wait it hides is
// a small part — rocprofv3 SQ counters).
//
// Summation order per output is fixed by the code — M over K in MFMA order, the transforms
// in the orders written below — and does not depend on TTY: the tilings of this form are
// bit-identical to each other.  Different from forms 0 and 1 by rounding only.
#pragma once
#include <algorithm>

#include "conv3x3_wino.h"

namespace tic {

// B^T (rows xi, columns i) and A^T (rows a, columns nu) of F(4x4, 3x3) on (0, 1, -1, 2, -1/2);
// w4_bt / w4_at below apply them factored, the row coefficients of B^T are read from the table
__device__ constexpr float kW4BT[6][6] = {{1.f, 1.5f, -2.f, -1.5f, 1.f, 0.f},  {0.f, -1.f, -2.5f, -0.5f, 1.f, 0.f},
                                          {0.f, 1.f, 0.5f, -2.5f, 1.f, 0.f},   {0.f, -0.5f, -1.f, 0.5f, 1.f, 0.f},
                                          {0.f, 2.f, -1.f, -2.f, 1.f, 0.f},    {0.f, 1.f, 1.5f, -2.f, -1.5f, 1.f}};
__device__ constexpr float kW4AT[4][6] = {{1.f, 1.f, 1.f, 1.f, 1.f, 0.f},
                                          {0.f, 1.f, -1.f, 2.f, -0.5f, 0.f},
                                          {0.f, 1.f, 1.f, 4.f, 0.25f, 0.f},
                                          {0.f, 1.f, -1.f, 8.f, -0.125f, 1.f}};

typedef unsigned int w4u32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ f32x4 fma4s(float c, f32x4 x, f32x4 y) {
  return f32x4{__builtin_fmaf(c, x.x, y.x), __builtin_fmaf(c, x.y, y.y), __builtin_fmaf(c, x.z, y.z),
               __builtin_fmaf(c, x.w, y.w)};
}

// V_nu = sum_j BT[nu][j] r_j for all six nu, factored (16 operations instead of 26):
// a = r1 - r3, b = r4 - r2, u = r1 + r2 / 2, w = u + r2.
__device__ __forceinline__ void w4_bt(const f32x4 (&r)[6], f32x4 (&V)[6]) {
  const f32x4 a = r[1] - r[3], b = r[4] - r[2];
  V[3] = fma4s(-0.5f, a, b);
  V[4] = fma4s(2.f, a, b);
  V[0] = (fma4s(1.5f, a, r[0]) + b) - r[2];
  const f32x4 u = fma4s(0.5f, r[2], r[1]);
  V[2] = fma4s(-2.5f, r[3], r[4] + u);
  V[1] = b - fma4s(0.5f, r[3], u + r[2]);
  V[5] = (fma4s(-1.5f, b, a) - r[3]) + r[5];
}

// T_b = sum_nu AT[b][nu] M_nu for the four b, factored (12 operations instead of 18):
// s = M1 + M2, d = M1 - M2.
__device__ __forceinline__ void w4_at(const f32x4 (&M)[6], f32x4 (&T)[4]) {
  const f32x4 s = M[1] + M[2], d = M[1] - M[2];
  T[0] = ((M[0] + s) + M[3]) + M[4];
  T[1] = fma4s(-0.5f, M[4], fma4s(2.f, M[3], d));
  T[2] = fma4s(0.25f, M[4], fma4s(4.f, M[3], s));
  T[3] = fma4s(-0.125f, M[4], fma4s(8.f, M[3], d)) + M[5];
}

template <int TTY>
struct Wino4Geom {
  static constexpr int NT = 16;              // 4x4 output tiles per workgroup
  static constexpr int TTX = NT / TTY;       // tiles per tile row
  static constexpr int LR = 6 * TTY;         // staged rows: the six rows of B^T d per tile row
  static constexpr int LCOL = 4 * TTX + 2;   // staged input columns
  static constexpr int HPP = TTX + 1;        // pixels per (column mod 4) plane
  static constexpr int RPAD = TTY == 4 ? 16 : 0;  // conflict-free ds_read_b128 (lane groups)
};

// Weights (ConvArgs::wp): U packed [36 p][Cin/16][4 g][Cout][4 t], p = 6 xi + nu.
template <int CIN, int COUT, int TTY, int ACT, bool RES, int IN, int OUT>
__global__ void __launch_bounds__(768) conv3x3_wino4_kernel(const ConvArgs a) {
  using G = Wino4Geom<TTY>;
  constexpr int NT = G::NT, TTX = G::TTX, LR = G::LR, LCOL = G::LCOL, HPP = G::HPP;
  static_assert(CIN % 16 == 0 && COUT % 32 == 0, "channels");
  static_assert(!(IN == IN_IDX && RES), "the dequantiser layer has no residual");
  constexpr int NTHR = 768;
  constexpr int PS = CIN + 8, KC = CIN / 16, C4 = CIN / 4;
  constexpr int RS = 4 * HPP * PS + G::RPAD;  // floats per staged row
  constexpr int TILE = LR * RS;
  constexpr int CW = COUT / 2;                // output channels per wave
  constexpr int NBW = CW / 16;
  constexpr int XS = COUT + 4;                // exchange pitch per (xi, b, tile)
  constexpr int XCH = 24 * NT * XS;           // [6 xi][4 b][NT][XS]
  __shared__ __attribute__((aligned(16))) float smem[TILE > XCH ? TILE : XCH];

  const int tid = threadIdx.x;
  const int H = a.H, W = a.W, Ho = a.Ho, Wo = a.Wo;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int xi = wave >> 1, co_w = (wave & 1) * CW;
  const int lane = tid & 63, li = lane & 15, lg = lane >> 4;

  int bx, by, bz;
  xcd_tile(bx, by, bz);
  const int oy0 = by * 4 * TTY, ox0 = bx * 4 * TTX, nimg = bz;
  // timing probe (tools/wino4_timing.py; null in production): s_memrealtime stamps (100 MHz) —
  // [0] start, [1] loads issued, [2] staged, [3 + w] wave w's K loop done, [15] exchange done,
  // [16] end; [17] / [18] s_memtime around wave 0's K loop (the shader clock); [22] / [23] the
  // CU / XCC the workgroup ran on
  unsigned long long* const tsp =
      a.tstamp ? a.tstamp + TIC_W4_TS * (blockIdx.x + gridDim.x * (blockIdx.y + (size_t)gridDim.y * blockIdx.z))
               : nullptr;
  auto stamp = [&](int k) {
    if (tsp && tid == 0) tsp[k] = __builtin_amdgcn_s_memrealtime();
  };
  if (tsp && tid == 0) {
    tsp[22] = __builtin_amdgcn_s_getreg((31 << 11) | 4);   // HW_REG_HW_ID (CU, SE)
    tsp[23] = __builtin_amdgcn_s_getreg((31 << 11) | 20);  // HW_REG_XCC_ID
  }
  stamp(0);

  // ---- stage the row half of the input transform, B^T d, for every tile row (all Cin,
  // columns split by (column mod 4), zero outside the image = SAME pad).  Task = (tile row
  // ty, staged column col, channel quad c4): the column's six input rows 4 ty .. 4 ty + 5
  // into registers, then its six rows of B^T d (w4_bt, the factored form the column half
  // uses too) into LDS rows 6 ty .. 6 ty + 5.  Every wave then reads the one row xi it
  // needs per column — the row combination is done once per (column, channel), not once
  // per wave and tile (the two channel-half waves of a row and the two tiles sharing a
  // column each repeated it: 5.5x the VALU, which at f32 adds to the MFMA time) ----
  constexpr int NSTAGE = TTY * LCOL * C4;
  constexpr int NIT = (NSTAGE + NTHR - 1) / NTHR;
  f32x4 pre[NIT][6];
  // task i of this thread: channel quad c4 = tid % C4 (C4 divides NTHR), column
  // tid / C4 + i NTHR / C4 of the tile rows, walked incrementally (ty, col) — no divisions
  static_assert(NTHR % C4 == 0, "channel quad per thread");
  constexpr int DP = NTHR / C4, DR = DP / LCOL, DC = DP % LCOL;
  auto walk = [&](auto&& fn) {
    int t = tid;  // opaque copy: the index math is re-derived at each use instead of held live
    asm volatile("" : "+v"(t));
    const int c4 = t % C4, p0 = t / C4;
    int row = p0 / LCOL, col = p0 - (p0 / LCOL) * LCOL;
#pragma unroll
    for (int i = 0; i < NIT; ++i) {
      fn(i, row, col, c4);
      col += DC;
      row += DR;
      if (col >= LCOL) {
        col -= LCOL;
        ++row;
      }
    }
  };
  // branch-free: a raw buffer load past num_records returns zeros (the SAME padding and the
  // elements past the tile), so the loads need no control flow around them
  auto issue = [&]() {
    if (a.probe & 2) return;  // timing probe: no staging loads (results invalid)
    const __amdgpu_buffer_rsrc_t rs =
        __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(a.in), (short)0, 0x7fffffff, 0x00020000);
    const int base = nimg * H * W * CIN;  // element offset of the patch (< 2^31: the workspace chunk)
    walk([&](int i, int ty, int col, int c4) {
      // the last pass's tasks past the tile rows issue nothing (their waves skip the loads)
      if (!(NSTAGE % NTHR == 0 || i + 1 < NIT || ty < TTY)) return;
      const int ix = ox0 - 1 + col;
#pragma unroll
      for (int r = 0; r < 6; ++r) {
        const int iy = oy0 - 1 + 4 * ty + r;
        const bool in = (unsigned)iy < (unsigned)H && (unsigned)ix < (unsigned)W;
        if constexpr (IN == IN_F32) {
          const int off = in ? (base + (iy * W + ix) * CIN + c4 * 4) * 4 : 0x7fffffff;
          const w4u32x4 u = __builtin_amdgcn_raw_buffer_load_b128(rs, off, 0, 0);
          pre[i][r] = f32x4{__uint_as_float(u.x), __uint_as_float(u.y), __uint_as_float(u.z), __uint_as_float(u.w)};
        } else {  // u8 symbols through the dequantiser table (decode_4); SAME padding is 0, not lut[0]
          const int off = in ? base + (iy * W + ix) * CIN + c4 * 4 : 0x7fffffff;
          const unsigned q = __builtin_amdgcn_raw_buffer_load_b32(rs, off, 0, 0);
          pre[i][r] = in ? f32x4{a.lut[q & 0xff], a.lut[(q >> 8) & 0xff], a.lut[(q >> 16) & 0xff], a.lut[q >> 24]}
                         : f32x4{0.f, 0.f, 0.f, 0.f};
        }
      }
    });
  };
  auto commit = [&]() {
    walk([&](int i, int ty, int col, int c4) {
      if ((NSTAGE % NTHR == 0 || i + 1 < NIT) || ty < TTY) {
        f32x4 bt[6];
        w4_bt(pre[i], bt);
        float* const dst = &smem[6 * ty * RS + ((col & 3) * HPP + (col >> 2)) * PS + c4 * 4];
#pragma unroll
        for (int r = 0; r < 6; ++r) *reinterpret_cast<f32x4*>(dst + r * RS) = bt[r];
      }
    });
  };

  // ---- row xi of B^T d for tile li, column j, chunk kc: one staged value ----
  const int ty = li / TTX, tx = li % TTX;
  const int tbase = (6 * ty + xi) * RS + tx * PS + lg * 4;
  auto ld = [&](int j, int kc) -> f32x4 {
    return *reinterpret_cast<const f32x4*>(&smem[tbase + ((j & 3) * HPP + (j >> 2)) * PS + kc * 16]);
  };

  // ---- A fragments (U) from L2, prefetched PF steps ahead; step s = 6 kc + nu.  Raw buffer
  // loads: the descriptor in SGPRs, the lane's byte offset in one VGPR (made opaque after the
  // staging below, so hipcc does not precompute every step's address), the step as an
  // immediate offset.  They count on vmcnt only, so the compiler waits for them by count
  // behind the prefetch — the flat loads of a plain pointer also count on lgkmcnt, and every
  // wait for the column reads from LDS then drained the weight prefetch too (wave 0's K loop
  // 8.8 -> 5.9 us, the 64x64 launch 189 -> 172 us: tools/wino4_timing.py) ----
  constexpr int NSTEP = 6 * KC, PF = 2;
  const __amdgpu_buffer_rsrc_t wrs =
      __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(a.wp), (short)0, 36 * KC * 16 * COUT * 4, 0x00020000);
  int wl = ((6 * xi * KC * 16 * COUT) + (lg * COUT + co_w + li) * 4) * 4;  // bytes
  auto wglob = [&](int s, int nb) -> f32x4 {
    const int kc = s / 6, nu = s % 6;
    // timing probe bit 0: every step reads step 0's fragment (L1-resident; results invalid)
    const int soff = (a.probe & 1) ? 0 : ((nu * KC + kc) * 16 * COUT + nb * 64) * 4;
    const w4u32x4 u = __builtin_amdgcn_raw_buffer_load_b128(wrs, wl, soff, 0);
    return f32x4{__uint_as_float(u.x), __uint_as_float(u.y), __uint_as_float(u.z), __uint_as_float(u.w)};
  };
  // the output quad of this thread is the same in every pass of the Y phase (768 % Q4 == 0)
  constexpr int Q4 = COUT / 4, NTASK = 4 * NT * Q4;
  static_assert(NTHR % Q4 == 0, "quad per thread");
  const int q = tid % Q4;
  const f32x4 bb = *reinterpret_cast<const f32x4*>(a.bias + 4 * q);

  issue();
  stamp(1);
  {
    commit();
    __syncthreads();
    stamp(2);
    if (tsp && tid == 0) tsp[17] = __builtin_amdgcn_s_memtime();
    asm volatile("" : "+v"(wl));

    f32x4 av[PF + 1][NBW];
#pragma unroll
    for (int p = 0; p < PF; ++p)
#pragma unroll
      for (int nb = 0; nb < NBW; ++nb) av[p][nb] = wglob(p, nb);
    f32x4 V[6];
    {
      f32x4 r[6];
#pragma unroll
      for (int j = 0; j < 6; ++j) r[j] = ld(j, 0);
      w4_bt(r, V);
    }
    f32x4 acc[6][NBW];
#pragma unroll
    for (int nu = 0; nu < 6; ++nu)
#pragma unroll
      for (int nb = 0; nb < NBW; ++nb) acc[nu][nb] = f32x4{0.f, 0.f, 0.f, 0.f};

      // Software pipeline: while the MFMAs of point nu of chunk kc issue, column nu of chunk
    // kc + 1 is read (before them); the six V of chunk kc + 1 follow the chunk.
#pragma unroll
    for (int kc = 0; kc < KC; ++kc) {
      const bool next = kc + 1 < KC;
      f32x4 rn[6];
#pragma unroll
      for (int nu = 0; nu < 6; ++nu) {
        const int s = kc * 6 + nu;
        if (s + PF < NSTEP) {
#pragma unroll
          for (int nb = 0; nb < NBW; ++nb) av[(s + PF) % (PF + 1)][nb] = wglob(s + PF, nb);
        }
        if (next) rn[nu] = ld(nu, kc + 1);
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int tt = 0; tt < 4; ++tt)
#pragma unroll
          for (int nb = 0; nb < NBW; ++nb) acc[nu][nb] = mfma4(av[s % (PF + 1)][nb][tt], V[nu][tt], acc[nu][nb]);
        __builtin_amdgcn_sched_barrier(0);
      }
      if (next) w4_bt(rn, V);
    }

    // ---- T = M A over nu (per wave), exchanged through LDS (the input tile is dead) ----
    if (tsp && lane == 0) tsp[3 + wave] = __builtin_amdgcn_s_memrealtime();
    if (tsp && tid == 0) tsp[18] = __builtin_amdgcn_s_memtime();
    __syncthreads();
#pragma unroll
    for (int nb = 0; nb < NBW; ++nb) {
      const f32x4 m[6] = {acc[0][nb], acc[1][nb], acc[2][nb], acc[3][nb], acc[4][nb], acc[5][nb]};
      f32x4 tb[4];
      w4_at(m, tb);
#pragma unroll
      for (int b = 0; b < 4; ++b)
        *reinterpret_cast<f32x4*>(&smem[((xi * 4 + b) * NT + li) * XS + co_w + nb * 16 + lg * 4]) = tb[b];
    }

    // ---- Y = A^T T: one (output column b, tile, 4-channel quad) per thread and pass; the
    // residuals are read before the exchange barrier so their latency overlaps it ----
    constexpr int NPASS = (NTASK + NTHR - 1) / NTHR;
    // per pass: element offset of the task's top output pixel (32-bit: a launch's activation
    // chunk is < 2^31 floats) and how many of its 4 rows lie inside the image
    int o0[NPASS], nrow[NPASS];
    f32x4 rr[NPASS][4];
#pragma unroll
    for (int ps = 0; ps < NPASS; ++ps) {
      const int it = ps * NTHR + tid;
      const int tile = (it / Q4) % NT, b = it / (Q4 * NT);
      const int ox = ox0 + 4 * (tile % TTX) + b, oy = oy0 + 4 * (tile / TTX);
      nrow[ps] = (it < NTASK && ox < Wo) ? min(4, Ho - oy) : 0;
      o0[ps] = ((nimg * Ho + oy) * Wo + ox) * COUT + 4 * q;
      if (a.probe & 4) nrow[ps] = 0;  // timing probe: no residual loads, no stores (results invalid)
      if constexpr (RES) {
#pragma unroll
        for (int ay = 0; ay < 4; ++ay)
          rr[ps][ay] = ay < nrow[ps] ? *reinterpret_cast<const f32x4*>(a.res + o0[ps] + ay * Wo * COUT) : f32x4{};
      }
    }
    __syncthreads();
    stamp(15);
#pragma unroll
    for (int ps = 0; ps < NPASS; ++ps) {
      const int it = ps * NTHR + tid;
      if (NTASK % NTHR != 0 && it >= NTASK) break;
      const int tile = (it / Q4) % NT, b = it / (Q4 * NT);
      f32x4 T[6];
#pragma unroll
      for (int x2 = 0; x2 < 6; ++x2)
        T[x2] = *reinterpret_cast<const f32x4*>(&smem[((x2 * 4 + b) * NT + tile) * XS + 4 * q]);
      f32x4 Y[4];
      w4_at(T, Y);
#pragma unroll
      for (int ay = 0; ay < 4; ++ay) {
        if (ay >= nrow[ps]) continue;
        // my_conv2d's epilogue (conv_out4's operations and order): + bias, ReLU, + residual
        f32x4 v = Y[ay];
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
          v.x = __fadd_rn(v.x, rr[ps][ay].x);
          v.y = __fadd_rn(v.y, rr[ps][ay].y);
          v.z = __fadd_rn(v.z, rr[ps][ay].z);
          v.w = __fadd_rn(v.w, rr[ps][ay].w);
        }
        const int o = o0[ps] + ay * Wo * COUT;
        if constexpr (OUT == OUT_F32) {
          *reinterpret_cast<f32x4*>(a.out + o) = v;
        } else {  // encode_4: the optional pre-activation, then the quantiser (conv_out4's)
          if (a.out) *reinterpret_cast<f32x4*>(a.out + o) = v;
          const uint32_t qv = quant1(v.x, a.qscale) | (quant1(v.y, a.qscale) << 8) |
                              (quant1(v.z, a.qscale) << 16) | (quant1(v.w, a.qscale) << 24);
          *reinterpret_cast<uint32_t*>(a.qout + o) = qv;
        }
      }
    }
  }
  stamp(16);
}

template <int CIN, int COUT, int TTY, int ACT, bool RES, int IN, int OUT>
static void launch_wino4(const ConvArgs& a, int n, hipStream_t s) {
  constexpr int OW = 4 * Wino4Geom<TTY>::TTX, OH = 4 * TTY;
  // the kernel's offsets are 32-bit (input: buffer byte offsets below 2^31, so < 2^29 floats;
  // output: element offsets): launch at most 2^29 floats of either at a time (the codec's
  // chunks are far below that; the per-layer entry takes any batch).  A single patch of
  // 2^29 floats or more cannot run in this form: the runtime never selects it for one
  // (wino4_fits, tic_runtime.cpp).
  const size_t per = (size_t)a.H * a.W * CIN > (size_t)a.Ho * a.Wo * COUT ? (size_t)a.H * a.W * CIN
                                                                           : (size_t)a.Ho * a.Wo * COUT;
  int step = (int)std::max<size_t>(1, std::min<size_t>((size_t)n, (((size_t)1 << 29) - 1) / per));
  if (a.max_n > 0) step = std::min(step, a.max_n);
  for (int n0 = 0; n0 < n; n0 += step) {
    ConvArgs b = a;
    // (the u8 symbols of decode_4 step by bytes, the f32 activations by floats; encode_4's
    // pre-activation output is optional)
    if (IN == IN_IDX) b.in = reinterpret_cast<const uint8_t*>(a.in) + (size_t)n0 * a.H * a.W * CIN;
    else b.in = reinterpret_cast<const float*>(a.in) + (size_t)n0 * a.H * a.W * CIN;
    b.out = a.out ? a.out + (size_t)n0 * a.Ho * a.Wo * COUT : nullptr;
    if (a.qout) b.qout = a.qout + (size_t)n0 * a.Ho * a.Wo * COUT;
    if (a.res) b.res = a.res + (size_t)n0 * a.Ho * a.Wo * COUT;
    dim3 grid((a.Wo + OW - 1) / OW, (a.Ho + OH - 1) / OH, std::min(step, n - n0));
    // timing probe: every split launch restarts blockIdx.z at 0, so its stamps go after the
    // workgroups of the launches before it
    if (a.tstamp) b.tstamp = a.tstamp + (size_t)TIC_W4_TS * grid.x * grid.y * n0;
    hipLaunchKernelGGL((conv3x3_wino4_kernel<CIN, COUT, TTY, ACT, RES, IN, OUT>), grid, dim3(768), 0, s, b);
  }
}

}  // namespace tic

// Winograd F(4x4,3x3) entry: th = output rows per workgroup (4 TTY), 256 / th columns,
// weight source 5 = the F(4x4,3x3) packing of U (passed as ConvArgs::wp).
#define TIC_WINO4(CIN, COUT, TTY, ACT, RES, IN, OUT) \
  { MODE_S1, CIN, COUT, ACT, RES, IN, OUT, 4 * TTY, 1, 1, 5, &tic::launch_wino4<CIN, COUT, TTY, ACT, RES, IN, OUT> }
