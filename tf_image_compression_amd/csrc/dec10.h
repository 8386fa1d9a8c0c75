// dec10.h — the decoder's last two layers fused through LDS: decode_1 (stride-2 transposed
// conv C1 -> C0, ReLU; basic_block.py:50-71) and decode_0 (transposed conv C0 -> 3 with the
// denormalise + clip + round of model_0/model.py:250-259 and decode.py:249).  The C0-channel
// intermediate at half the output resolution (128² x 32 f32 = 2 MB per 256² patch) never
// reaches HBM: per patch the pair reads 0.5 MB and writes 0.2 MB instead of 4.9 MB.
//
// Workgroup: TA = 4 rows x 16 columns of decode_1's input.  Their decode_1 outputs are an
// 8 x 32 tile of decode_0's input; decode_0 also needs one halo row above and one halo
// column left of it (input offsets {0,-1}), which are decode_1 outputs of phase 1 of the
// input row / column before the tile.
//   1. stage decode_1's input rows m0-1 .. m0+3, columns q0-1 .. q0+15 (zero outside);
//   2. the 8 x 32 interior by MFMA exactly as conv3x3_kernel<MODE_T2> computes it (same
//      packing, same tap-major step order, same fragment layout), + bias, ReLU, into the
//      LDS tile of decode_0's input;
//   3. the 41 halo positions by two short MFMA passes (the row above: phases 2/3 of input row
//      m0-1; the column left: phases 1/3 of input column q0-1), in conv3x3_kernel's order,
//      zero where the position lies above / left of the image (decode_0's zero padding);
//   4. decode_0 per position as convT_rgb_valu_kernel (rgb_out_fma), its
//      output tile staged in the dead input tile and written back as 16-byte chunks.
// Every output is bit-identical to decode_1 by conv3x3_kernel followed by the VALU form of
// decode_0 (tests/test_gpu_parity.py::test_fused_tail_bit_identical).
#pragma once
#include "convT_rgb_valu.h"

namespace tic {

// WSH: decode_0's weights staged in LDS (broadcast ds_read_b128) or read with wave-uniform
// addresses from memory (scalar loads), as the two convT_rgb_valu kernels do.  PF: how many
// K steps ahead decode_1's weights are loaded (one step = 8 MFMAs = 256 cycles).  PROBE:
// timing experiments only, a mask of work left out (results invalid): 1 decode_1's MFMAs,
// 2 decode_0, 4 the input tile's loads, 8 decode_1's weight loads, 16 the output store,
// 32 the halo.
// CMP: the compact LDS form — decode_0's input tile unpadded (C0 floats per position, its
// 16-byte chunks XOR-swizzled per position so the ds_read_b128 of 16 consecutive positions
// still hits 16 distinct bank slots) with decode_1's input tile aliased into it (a barrier
// between decode_1's last read of it and the first write of its outputs): 38 KB instead of
// 56 KB at TA = 4, four workgroups per CU instead of two.
// PK: decode_0 by packed or plain fmas (rgb_out_fma_g).
// None of WSH / PF / TA / CMP / PK changes results.
template <int C1, int C0, bool WSH, int PF, int PROBE, int TA_ = 4, bool CMP = false, bool PK = true>
struct Dec10 {
  static constexpr int TA = TA_;                    // decode_1 input rows (x 16 columns), one per wave
  static constexpr int NT = 64 * TA;                // threads: one decode_0 input position each
  static constexpr int PSX = C1 + 8, KC = C1 / 16, C4 = C1 / 4;
  static constexpr int LRX = TA + 1, LCX = 17;
  static constexpr int XT = LRX * LCX * PSX;        // decode_1 input tile (floats)
  static constexpr int TH = 2 * TA, TW = 32;        // decode_0 input positions
  static constexpr int PSY = CMP ? C0 : C0 + 4, LRY = TH + 1, LCY = TW + 1;
  static constexpr int NCH = C0 / 4, GRP = 16 / NCH;  // CMP: chunks per position, positions per 256 B
  static constexpr int YT = LRY * LCY * PSY;        // decode_0 input tile incl. halo (floats)
  static constexpr int OT = 2 * TH * 2 * TW * 3;    // decode_0 output staging (floats)
  static constexpr int NB = C0 / 16;
  // the halo's MFMA passes: row / column x output-channel halves over 4 waves when there are
  // two channel blocks (each wave 1/4 of the halo), else row / column on waves 0 / 1
  static constexpr int HS = (NB % 2 == 0 && TA >= 4) ? 2 : 1, HNB = NB / HS, HW = 2 * HS;
  static constexpr int NSTEP = 9 * KC;
  static constexpr int NSTAGE = LRX * LCX * C4;
  static constexpr int NIT = (NSTAGE + NT - 1) / NT;
  static constexpr int XYT = CMP ? (XT > YT ? XT : YT) : XT + YT;  // xt (+) yt
  static constexpr int SMEM = XYT + (WSH ? 27 * C0 : 4);
  static constexpr bool OUT_IN_XT = !CMP && OT <= XT;  // output staging: the dead input tile, else yt
  static_assert(OT <= YT && C1 % 16 == 0 && C0 % 16 == 0 && NCH <= 16, "tile");

  // float offset of channel chunk c4 of decode_0 input position pos in yt
  __device__ __forceinline__ static int ychunk(int pos, int c4) {
    if constexpr (CMP) return pos * PSY + 4 * (c4 ^ ((pos / GRP) % NCH));
    else return pos * PSY + 4 * c4;
  }

  __device__ __forceinline__ static f32x4 wglob(const Dec10Args& a, int s, int nb, int li, int lg) {
    // raw buffer load (conv3x3.h weight_frag): descriptor and lane offset are loop-invariant
    // and CSE'd across the unrolled steps; the step offset is a constant
    const int tap = s / KC, kc = s % KC;
    return weight_frag(weight_rsrc(a.wp1, 9 * C1 * C0 * 4), (lg * C0 + li) * 16,
                       ((tap * KC + kc) * 4 * C0 * 4 + nb * 64) * 4);
  }

  // decode_1's input rows m0-1 .. m0+3, columns q0-1 .. q0+15 (zero outside) into registers
  __device__ __forceinline__ static void issue(const Dec10Args& a, f32x4 (&pre)[NIT], int q0, int m0, int nimg, int tid) {
#pragma unroll
    for (int i = 0; i < NIT; ++i) {
      const int e = i * NT + tid;
      pre[i] = f32x4{0.f, 0.f, 0.f, 0.f};
      if (e < NSTAGE) {
        const int c4 = e % C4, pe = e / C4, col = pe % LCX, row = pe / LCX;
        const int iy = m0 - 1 + row, ix = q0 - 1 + col;
        if (!(PROBE & 4) && iy >= 0 && iy < a.H && ix >= 0 && ix < a.W)
          pre[i] = *reinterpret_cast<const f32x4*>(a.in + ((size_t)(nimg * a.H + iy) * a.W + ix) * C1 + c4 * 4);
      }
    }
  }
  __device__ __forceinline__ static void land(float* xt, const f32x4 (&pre)[NIT], int tid) {
#pragma unroll
    for (int i = 0; i < NIT; ++i) {
      const int e = i * NT + tid;
      if (e < NSTAGE) *reinterpret_cast<f32x4*>(&xt[(e / C4) * PSX + (e % C4) * 4]) = pre[i];
    }
  }

  // ---- 2. decode_1's interior by MFMA: conv3x3_kernel<MODE_T2>'s step order, one input row
  //         per wave (wave < TA); av holds the first PF weight steps on entry and, with
  //         `again`, again on exit (the next tile uses the same weights) ----
  __device__ __forceinline__ static void interior(const Dec10Args& a, const float* xt, f32x4 (&av)[PF + 1][NB], f32x4 (&acc)[4][NB],
                                  int wave, int li, int lg, bool again) {
#pragma unroll
    for (int p = 0; p < 4; ++p)
#pragma unroll
      for (int nb = 0; nb < NB; ++nb) acc[p][nb] = f32x4{0.f, 0.f, 0.f, 0.f};
    auto load_b = [&](int s) -> f32x4 {
      const int tap = s / KC, kc = s % KC, ky = tap / 3, kx = tap % 3;
      const int lp = (wave + 1 - (ky == 2)) * LCX + li + 1 - (kx == 2);
      return *reinterpret_cast<const f32x4*>(&xt[lp * PSX + kc * 16 + lg * 4]);
    };
    f32x4 bq[2];
    bq[0] = load_b(0);
#pragma unroll
    for (int s = 0; s < NSTEP; ++s) {
      const int tap = s / KC, ky = tap / 3, kx = tap % 3;
      const int c = s & 1;
      if (s + PF < NSTEP) {
#pragma unroll
        for (int nb = 0; nb < NB; ++nb)
          av[(s + PF) % (PF + 1)][nb] = (PROBE & 8) ? av[s % (PF + 1)][nb] : wglob(a, s + PF, nb, li, lg);
      }
      if (s + 1 < NSTEP) bq[c ^ 1] = load_b(s + 1);
      __builtin_amdgcn_sched_barrier(0);
      const int ph = (ky == 1 ? 2 : 0) + (kx == 1 ? 1 : 0);
#pragma unroll
      for (int t = 0; t < 4; ++t)
#pragma unroll
        for (int nb = 0; nb < NB; ++nb) {
          if constexpr (PROBE & 1) acc[ph][nb][t] = fmaxf(acc[ph][nb][t], bq[c][t]);  // keep the reads live
          else acc[ph][nb] = mfma4(av[s % (PF + 1)][nb][t], bq[c][t], acc[ph][nb]);
        }
      __builtin_amdgcn_sched_barrier(0);
    }
    if (again) {
#pragma unroll
      for (int p = 0; p < PF; ++p)
#pragma unroll
        for (int nb = 0; nb < NB; ++nb) av[p][nb] = wglob(a, p, nb, li, lg);
    }
  }
  // + bias, ReLU -> yt
  __device__ __forceinline__ static void put_interior(const Dec10Args& a, float* yt, const f32x4 (&acc)[4][NB], int wave, int li,
                                      int lg) {
#pragma unroll
    for (int p = 0; p < 4; ++p) {
      const int py = p >> 1, px = p & 1;
#pragma unroll
      for (int nb = 0; nb < NB; ++nb) {
        const int co = nb * 16 + lg * 4;
        const f32x4 bb = *reinterpret_cast<const f32x4*>(a.b1 + co);
        f32x4 v = acc[p][nb];
        v.x = fmaxf(__fadd_rn(v.x, bb.x), 0.f);
        v.y = fmaxf(__fadd_rn(v.y, bb.y), 0.f);
        v.z = fmaxf(__fadd_rn(v.z, bb.z), 0.f);
        v.w = fmaxf(__fadd_rn(v.w, bb.w), 0.f);
        *reinterpret_cast<f32x4*>(&yt[ychunk((1 + 2 * wave + py) * LCY + 1 + 2 * li + px, co / 4)]) = v;
      }
    }
  }

  // ---- 3. the halo by MFMA, in conv3x3_kernel's order for those outputs (taps ascending,
  //         then chunk, then t): wave 0 the row above the tile (phases 2 and 3 of input row
  //         m0-1: taps 3, 4, 5), wave 1 the column left of it (phases 1 and 3 of input column
  //         q0-1, rows m0-1 .. m0+TA-1: taps 1, 4, 7; lane j = input row m0-1+j, j <= TA),
  //         channel blocks nb0 .. nb0+HNB-1; hacc[0]: phase 2 (row) / phase 1 (column),
  //         hacc[1]: phase 3 ----
  __device__ __forceinline__ static void halo(const Dec10Args& a, const float* xt, f32x4 (&hacc)[2][HNB], bool row,
                                              int nb0, int li, int lg) {
    f32x4 ha[3 * KC][HNB];
#pragma unroll
    for (int ti = 0; ti < 3; ++ti)
#pragma unroll
      for (int kc = 0; kc < KC; ++kc)
#pragma unroll
        for (int nb = 0; nb < HNB; ++nb)
          ha[ti * KC + kc][nb] = wglob(a, ((row ? 3 : 1) + ti * (row ? 1 : 3)) * KC + kc, nb0 + nb, li, lg);
#pragma unroll
    for (int q = 0; q < 2; ++q)
#pragma unroll
      for (int nb = 0; nb < HNB; ++nb) hacc[q][nb] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int ti = 0; ti < 3; ++ti) {
      const int tap = (row ? 3 : 1) + ti * (row ? 1 : 3);
      const int q = tap == 4 ? 1 : 0;
      int lp;
      if (row) lp = li + 1 - (tap == 5);  // input row m0-1 (LDS row 0), column q0+li (-1 for tap 5)
      else lp = min(max(li - (tap == 7), 0), LRX - 1) * LCX;  // input column q0-1 (LDS column 0)
#pragma unroll
      for (int kc = 0; kc < KC; ++kc) {
        const f32x4 b = *reinterpret_cast<const f32x4*>(&xt[lp * PSX + kc * 16 + lg * 4]);
#pragma unroll
        for (int t = 0; t < 4; ++t)
#pragma unroll
          for (int nb = 0; nb < HNB; ++nb) hacc[q][nb] = mfma4(ha[ti * KC + kc][nb][t], b[t], hacc[q][nb]);
      }
    }
  }
  // + bias, ReLU (zero where the position lies above / left of the image: decode_0's zero
  // padding) -> yt
  __device__ __forceinline__ static void put_halo(const Dec10Args& a, float* yt, const f32x4 (&hacc)[2][HNB], bool row,
                                                  int nb0, int li, int lg, int q0, int m0) {
#pragma unroll
    for (int q = 0; q < 2; ++q)
#pragma unroll
      for (int nb = 0; nb < HNB; ++nb) {
        const int co = (nb0 + nb) * 16 + lg * 4;
        int ry, cy;
        bool use;
        if (row) {
          ry = 0, cy = 1 + 2 * li + q, use = true;
        } else {
          ry = q ? 2 * li : 2 * li - 1, cy = 0, use = q ? li <= TA : (li >= 1 && li <= TA);
        }
        if (!use) continue;
        const bool inside = 2 * m0 - 1 + ry >= 0 && 2 * q0 - 1 + cy >= 0;
        const f32x4 bb = *reinterpret_cast<const f32x4*>(a.b1 + co);
        f32x4 v = hacc[q][nb];
        v.x = inside ? fmaxf(__fadd_rn(v.x, bb.x), 0.f) : 0.f;
        v.y = inside ? fmaxf(__fadd_rn(v.y, bb.y), 0.f) : 0.f;
        v.z = inside ? fmaxf(__fadd_rn(v.z, bb.z), 0.f) : 0.f;
        v.w = inside ? fmaxf(__fadd_rn(v.w, bb.w), 0.f) : 0.f;
        *reinterpret_cast<f32x4*>(&yt[ychunk(ry * LCY + cy, co / 4)]) = v;
      }
  }

  // ---- 4. decode_0 of input position (r, c) of the tile on the VALU (acc3 zeroed) ----
  __device__ __forceinline__ static void decode0(const Dec10Args& a, const float* yt, const float* wsh, f32x4 (&acc3)[4], int r,
                                 int c) {
    if constexpr ((PROBE & 2) != 0) acc3[0][0] = yt[((r + 1) * LCY + (c + 1)) * PSY];
    else
      rgb_out_fma_g<C0, PK, !WSH>(
          [&](int dy, int dx, int c4) {
            return *reinterpret_cast<const f32x4*>(&yt[ychunk((r + 1 + dy) * LCY + c + 1 + dx, c4)]);
          },
          WSH ? wsh : a.rgb.wraw, acc3);
  }

  // One tile, its input already in xt (and a barrier behind it): decode_1 by MFMA into yt,
  // the halo, decode_0 on the VALU, the output.
  __device__ __forceinline__ static void tile(const Dec10Args& a, float* xt, float* yt, const float* wsh, f32x4 (&av)[PF + 1][NB],
                              int q0, int m0, int nimg) {
    const int tid = threadIdx.x;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);  // decode_1 input row of this wave
    const int lane = tid & 63, li = lane & 15, lg = lane >> 4;
    f32x4 acc[4][NB];
    interior(a, xt, av, acc, wave, li, lg, false);
    if constexpr (!CMP) put_interior(a, yt, acc, wave, li, lg);
    const bool row = (wave & 1) == 0;
    const int nb0 = (wave >> 1) * HNB;
    f32x4 hacc[2][HNB];
    if (!(PROBE & 32) && wave < HW) halo(a, xt, hacc, row, nb0, li, lg);
    if constexpr (CMP) {  // xt lives inside yt: every read of it precedes the first write
      __syncthreads();
      put_interior(a, yt, acc, wave, li, lg);
    }
    if (!(PROBE & 32) && wave < HW) put_halo(a, yt, hacc, row, nb0, li, lg, q0, m0);
    __syncthreads();

    // decode_0; output tile staged in the dead decode_1 input tile (or, when it is too small,
    // in yt once every thread has read its inputs)
    const int r = tid / TW, c = tid % TW;
    f32x4 acc3[4] = {};
    decode0(a, yt, wsh, acc3, r, c);
    float* const ot = OUT_IN_XT ? xt : yt;
    if constexpr (!OUT_IN_XT) __syncthreads();
    rgb_out_epilogue(a.rgb, acc3, ot, 2 * TW * 3, r, c);
    __syncthreads();
    if constexpr (!(PROBE & 16)) rgb_out_store<TH, TW, NT>(a.rgb, ot, tid, 2 * m0, 2 * q0, nimg);
  }
};

// One workgroup per tile of TA x 16 decode_1 input positions (TA waves): TA = 4 runs two
// workgroups per CU, TA = 8 one of twice the size (half the halo re-read and per-tile
// overhead per position).
template <int C1, int C0, bool WSH, int PF = 2, int PROBE = 0, int TA = 4, bool CMP = false, bool PK = true>
__global__ void __launch_bounds__(64 * TA, CMP ? (TA == 4 ? (WSH ? 3 : 4) : 2) : 8 / TA)
    dec10_kernel(const Dec10Args a) {
  using D = Dec10<C1, C0, WSH, PF, PROBE, TA, CMP, PK>;
  __shared__ __attribute__((aligned(16))) float smem[D::SMEM];
  float* const xt = smem;
  float* const yt = CMP ? smem : smem + D::XT;
  float* const wsh = smem + D::XYT;
  const int tid = threadIdx.x;
  const int q0 = blockIdx.x * 16, m0 = blockIdx.y * D::TA, nimg = blockIdx.z;
  const int lane = tid & 63, li = lane & 15, lg = lane >> 4;
  f32x4 av[PF + 1][D::NB];
#pragma unroll
  for (int p = 0; p < PF; ++p)
#pragma unroll
    for (int nb = 0; nb < D::NB; ++nb) av[p][nb] = D::wglob(a, p, nb, li, lg);
  if (WSH) rgb_out_load_weights<C0, D::NT>(a.rgb.wraw, wsh, tid);
  {  // ---- 1. stage decode_1's input tile ----
    f32x4 pre[D::NIT];
    D::issue(a, pre, q0, m0, nimg, tid);
    D::land(xt, pre, tid);
  }
  __syncthreads();
  D::tile(a, xt, yt, wsh, av, q0, m0, nimg);
}

}  // namespace tic
