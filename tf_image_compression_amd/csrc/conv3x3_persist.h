// conv3x3_persist.h — persistent variant of conv3x3_kernel for the full-resolution
// layers whose whole weight tensor fits in LDS (Cin x Cout <= 32 x 64, 64 x 32: encode_1/2,
// decode_1/2 of model_0/1/2, and their 16-channel relatives).
//
// Why: conv3x3_kernel stages a workgroup's input tile and then computes on it; the
// workgroups that share a CU fall into lock-step, so the tile traffic (~40-50 KB per
// workgroup for a stride-2 32-channel tile) is never covered by MFMA work.  Here ONE
// workgroup per CU (grid = CUs x resident workgroups) walks a contiguous run of tiles:
//   * all 9 taps of the weights stay resident in LDS (one LDS-DMA copy per workgroup);
//   * the input tile is double-buffered in LDS and the staging is software-pipelined
//     INTO the K loop: K step i of tile t writes element i of tile t+1 (loaded one tile
//     earlier, register set A) to the other LDS buffer and issues the global load of
//     element i of tile t+2 (register set B).
// Measured (tools/persist_probe.hip, encode_1 shape, batch 32): the K loop alone runs at
// 95 % of the MFMA rate (4865 cycles/tile vs 4608), but every 1 KiB wave-load issued
// among the MFMAs costs its wave ~190 cycles of issue (MI355X_MICROARCH.md: 60-185 per
// piece), +~1950 cycles/tile, and with one wave per SIMD nothing covers it: the variant
// ties conv3x3_kernel (34 us) rather than beating it.  Interleaving vs a separate staging
// phase, L2-resident vs HBM input, and LDS-DMA instead of register loads all measured
// within 10 %.  It stays registered for the autotuner (it wins on decode_1/2 solo).
//   * the tile loop is unrolled by two so the register sets swap statically;
//   * the same tap-major, t-inner fma order as conv3x3_kernel -> bit-identical results.
// Registry: weight source (ConvEntry::wlds) 3.  TIC_PERSIST_PROBE builds (tools/
// persist_probe.hip) record per-wave cycle stamps.
#pragma once
#include <type_traits>

#include "conv3x3.h"

#ifdef TIC_PERSIST_PROBE
__device__ unsigned long long* g_persist_probe;
#define TIC_STAMP(v) v = __builtin_amdgcn_s_memtime()
#else
#define TIC_STAMP(v)
#endif

namespace tic {

// 16-byte-per-lane LDS-DMA: lane L's 16 bytes land at lds + 16 L (wave-uniform lds).
__device__ __forceinline__ void dma16(const float* src, float* lds) {
  __builtin_amdgcn_global_load_lds(src, (lds_ptr_t)lds, 16, 0, 0);
}

template <int MODE, int CIN, int COUT, int TH, int WR, int ACT>
struct PersistGeom {
  static constexpr int PS = CIN + 8;
  static constexpr int LR = TileGeom<MODE, TH>::LR;
  static constexpr int LC = TileGeom<MODE, TH>::LC;
  static constexpr int TILE = LR * LC * PS;   // floats of one input tile buffer
  static constexpr int WALL = 9 * CIN * COUT;  // floats of the packed weights
  static constexpr int LDS_BYTES = (WALL + 2 * TILE) * 4;
  static constexpr int NSTAGE = LR * LC * (CIN / 4);  // 16-byte elements per tile
  static constexpr int NIT = (NSTAGE + 255) / 256;    // per thread
};

template <int MODE, int CIN, int COUT, int TH, int WR, int ACT>
__global__ void __launch_bounds__(256) conv3x3_persist_kernel(const ConvArgs a, int ntx, int nty, int ntiles) {
  using G = PersistGeom<MODE, CIN, COUT, TH, WR, ACT>;
  static_assert(CIN % 16 == 0 && COUT % 16 == 0, "channels must be multiples of 16");
  static_assert(G::LDS_BYTES <= 160 * 1024, "weights + two tiles exceed LDS");
  constexpr int PS = G::PS, LC = G::LC, TILE = G::TILE, WALL = G::WALL;
  constexpr int KC = CIN / 16, C4 = CIN / 4, NSTEP = 9 * KC;
  constexpr int NBT = COUT / 16;
  constexpr int WC = 4 / WR;
  static_assert(WR * WC == 4 && TH % WR == 0 && NBT % WC == 0, "bad wave split");
  constexpr int NB = NBT / WC, MB = TH / WR;
  constexpr int NPH = MODE == MODE_T2 ? 4 : 1;
  constexpr int NSTAGE = G::NSTAGE, NIT = G::NIT;
  static_assert(NIT <= NSTEP, "staging is spread one element per K step");
  static_assert(NIT <= 32, "validity bits");
  static_assert(WALL % 256 == 0, "weights are moved in 1 KiB wave chunks");

#ifdef TIC_PERSIST_PROBE
  const unsigned long long p_start = __builtin_amdgcn_s_memtime();
  const unsigned long long p_rstart = __builtin_amdgcn_s_memrealtime();
  unsigned long long p_t0 = 0, p_k0 = 0, p_k1 = 0, p_e = 0, p_b = 0, p_kl = 0, p_ep = 0, p_ba = 0;
#endif
  __shared__ __attribute__((aligned(16))) float smem[WALL + 2 * TILE];
  float* const wsh = smem;
  float* const tiles = smem + WALL;

  const int tid = threadIdx.x;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int lane = tid & 63;
  const int wr = wave / WC, wc = wave % WC;
  const int li = lane & 15, lg = lane >> 4;
  const int co_wave = wc * NB * 16;
  const int H = a.H, W = a.W;

  // contiguous run of tiles for this workgroup (x fastest, then rows, then images)
  const int t_begin = (int)((long long)blockIdx.x * ntiles / gridDim.x);
  const int t_end = (int)((long long)(blockIdx.x + 1) * ntiles / gridDim.x);
  if (t_begin >= t_end) return;

  // ---- weights -> LDS (whole packed tensor, [tap][kc][g][Cout][4]) ----
  for (int c = wave; c < WALL / 256; c += 4)
    __builtin_amdgcn_global_load_lds(a.wp + c * 256 + lane * 4, (lds_ptr_t)(wsh + c * 256), 16, 0, 0);

  // Per-element staging geometry is the same for every tile: element i of this thread
  // sits at (dy, dx) from the tile's first input pixel, channel quad c4 — packed once.
  uint32_t geo[NIT];
#pragma unroll
  for (int i = 0; i < NIT; ++i) {
    const int e = i * 256 + tid;
    const int c4 = e % C4, pe = e / C4, col = pe % LC, row = pe / LC;
    int dx = col;
    if constexpr (MODE == MODE_S2) dx = col >= 17 ? 2 * (col - 17) + 1 : 2 * col;
    geo[i] = (NSTAGE % 256 == 0 || e < NSTAGE) ? (uint32_t)row | ((uint32_t)dx << 8) | ((uint32_t)c4 << 16)
                                                : 0xffffffffu;  // never valid
  }
  struct Origin {
    const float* img;
    int y0, x0;
  };
  auto origin = [&](int t) {
    const int tx = t % ntx, r = t / ntx;
    const int gx0 = tx * 16, gy0 = (r % nty) * TH, nimg = r / nty;
    Origin o;
    o.img = reinterpret_cast<const float*>(a.in) + (size_t)nimg * H * W * CIN;
    if constexpr (MODE == MODE_S2) {
      o.y0 = 2 * gy0 - a.pad_y;
      o.x0 = 2 * gx0 - a.pad_x;
    } else if constexpr (MODE == MODE_S1) {
      o.y0 = gy0 - a.pad_y;
      o.x0 = gx0 - a.pad_x;
    } else {
      o.y0 = gy0 - 1;
      o.x0 = gx0 - 1;
    }
    return o;
  };
  // one element: global load into a register (out-of-image elements load the image's
  // first element and are zeroed at commit via the validity bit); one LDS write
  auto issue1 = [&](const Origin& o, int i, f32x4& r, uint32_t& valid) {
    const uint32_t g = geo[i];
    const int iy = o.y0 + (int)(g & 0xff), ix = o.x0 + (int)((g >> 8) & 0xff);
    const bool ok = g != 0xffffffffu && (unsigned)iy < (unsigned)H && (unsigned)ix < (unsigned)W;
    const uint32_t off = ok ? ((uint32_t)(iy * W + ix) * CIN + ((g >> 16) & 0xff) * 4) : 0u;
    r = *reinterpret_cast<const f32x4*>(o.img + off);
    valid = (valid & ~(1u << i)) | ((uint32_t)ok << i);
  };
  auto commit1 = [&](float* buf, int i, const f32x4& r, uint32_t valid) {
    const int e = i * 256 + tid;
    const f32x4 v = ((valid >> i) & 1) ? r : f32x4{0.f, 0.f, 0.f, 0.f};
    if (NSTAGE % 256 == 0 || e < NSTAGE) *reinterpret_cast<f32x4*>(&buf[(e / C4) * PS + (e % C4) * 4]) = v;
  };

  f32x4 bias[NB];
#pragma unroll
  for (int nb = 0; nb < NB; ++nb) bias[nb] = *reinterpret_cast<const f32x4*>(a.bias + co_wave + nb * 16 + lg * 4);

  // prologue: tile t_begin staged into buffer 0 (the wait also covers the weight DMA,
  // issued earlier); tile t_begin+1 in flight in register set 1
  f32x4 rs[2][NIT];
  uint32_t vs[2] = {0u, 0u};
  {
    const Origin o0 = origin(t_begin);
#pragma unroll
    for (int i = 0; i < NIT; ++i) issue1(o0, i, rs[0][i], vs[0]);
#pragma unroll
    for (int i = 0; i < NIT; ++i) commit1(tiles, i, rs[0][i], vs[0]);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    const Origin o1 = origin(min(t_begin + 1, t_end - 1));
#pragma unroll
    for (int i = 0; i < NIT; ++i) issue1(o1, i, rs[1][i], vs[1]);
  }
  __syncthreads();
#ifdef TIC_PERSIST_PROBE
  TIC_STAMP(p_t0);
  const unsigned long long p_r0 = __builtin_amdgcn_s_memrealtime();
#endif

  // one tile: K loop over buffer P with the staging of tile t+1 (register set P^1 ->
  // buffer P^1) and tile t+2 (-> register set P) interleaved, then the epilogue and the
  // per-tile barrier.  Past the end of the run the staged tile index is clamped:
  // harmless redundant work instead of a branch inside the K loop.
  auto tile = [&](int t, auto parity) {
    constexpr int P = decltype(parity)::value;
    TIC_STAMP(p_k0);
    const float* lds = tiles + P * TILE;
    float* nbuf = tiles + (P ^ 1) * TILE;
    const Origin on = origin(min(t + 2, t_end - 1));

    f32x4 acc[NPH][MB][NB];
#pragma unroll
    for (int p = 0; p < NPH; ++p)
#pragma unroll
      for (int mb = 0; mb < MB; ++mb)
#pragma unroll
        for (int nb = 0; nb < NB; ++nb) acc[p][mb][nb] = f32x4{0.f, 0.f, 0.f, 0.f};

    auto load_b = [&](int s, f32x4* dst) {
      const int tap = s / KC, kc = s % KC;
      const int ky = tap / 3, kx = tap % 3;
#pragma unroll
      for (int mb = 0; mb < MB; ++mb) {
        const int r = wr * MB + mb;
        int lp;
        if constexpr (MODE == MODE_S1) lp = (r + ky) * LC + li + kx;
        else if constexpr (MODE == MODE_S2) lp = (2 * r + ky) * LC + (kx & 1) * 17 + li + (kx >> 1);
        else lp = (r + 1 - (ky == 2)) * LC + li + 1 - (kx == 2);
        dst[mb] = *reinterpret_cast<const f32x4*>(&lds[lp * PS + kc * 16 + lg * 4]);
      }
    };
    auto load_a = [&](int s, f32x4* dst) {
#pragma unroll
      for (int nb = 0; nb < NB; ++nb)
        dst[nb] = *reinterpret_cast<const f32x4*>(&wsh[((s * 4 + lg) * COUT + co_wave + nb * 16 + li) * 4]);
    };
    f32x4 bq[2][MB], aq[2][NB];
    load_b(0, bq[0]);
    load_a(0, aq[0]);
#pragma unroll
    for (int s = 0; s < NSTEP; ++s) {
      const int c = s & 1;
      if (s + 1 < NSTEP) {
        load_b(s + 1, bq[c ^ 1]);
        load_a(s + 1, aq[c ^ 1]);
      }
      if (s < NIT) {
        commit1(nbuf, s, rs[P ^ 1][s], vs[P ^ 1]);  // tile t+1, loaded one tile ago
        issue1(on, s, rs[P][s], vs[P]);             // tile t+2
      }
      __builtin_amdgcn_sched_barrier(0);
      const int tap = s / KC, ky = tap / 3, kx = tap % 3;
      const int ph = MODE == MODE_T2 ? (ky == 1 ? 2 : 0) + (kx == 1 ? 1 : 0) : 0;
#pragma unroll
      for (int tt = 0; tt < 4; ++tt)
#pragma unroll
        for (int mb = 0; mb < MB; ++mb)
#pragma unroll
          for (int nb = 0; nb < NB; ++nb) acc[ph][mb][nb] = mfma4(aq[c][nb][tt], bq[c][mb][tt], acc[ph][mb][nb]);
      __builtin_amdgcn_sched_barrier(0);
    }
    TIC_STAMP(p_k1);

    // ---- epilogue: + bias, act, 16-byte f32 NHWC stores ----
    const int tx = t % ntx, rr = t / ntx;
    const int gx0 = tx * 16, gy0 = (rr % nty) * TH, nimg = rr / nty;
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
          const int co = co_wave + nb * 16 + lg * 4;
          f32x4 v = acc[p][mb][nb];
          v.x = __fadd_rn(v.x, bias[nb].x);
          v.y = __fadd_rn(v.y, bias[nb].y);
          v.z = __fadd_rn(v.z, bias[nb].z);
          v.w = __fadd_rn(v.w, bias[nb].w);
          if constexpr (ACT == ACT_RELU) {
            v.x = fmaxf(v.x, 0.f);
            v.y = fmaxf(v.y, 0.f);
            v.z = fmaxf(v.z, 0.f);
            v.w = fmaxf(v.w, 0.f);
          }
          *reinterpret_cast<f32x4*>(a.out + ((size_t)(nimg * Ho + oy) * Wo + ox) * COUT + co) = v;
        }
      }
    }
    TIC_STAMP(p_e);
    __syncthreads();  // buffer P^1 complete; buffer P free for tile t+2
    TIC_STAMP(p_b);
#ifdef TIC_PERSIST_PROBE
    p_kl += p_k1 - p_k0;
    p_ep += p_e - p_k1;
    p_ba += p_b - p_e;
#endif
  };

  for (int t = t_begin; t < t_end; t += 2) {
    tile(t, std::integral_constant<int, 0>());
    if (t + 1 < t_end) tile(t + 1, std::integral_constant<int, 1>());
  }

#ifdef TIC_PERSIST_PROBE
  if (lane == 0) {
    unsigned long long* q = g_persist_probe + (blockIdx.x * 4 + wave) * 12;
    q[0] = p_b - p_t0;
    q[1] = p_kl;
    q[2] = p_ep;
    q[3] = p_ba;
    q[4] = __builtin_amdgcn_s_memrealtime() - p_r0;
    q[5] = 0;
    q[6] = 0;
    q[7] = p_t0 - p_start;
    q[8] = p_rstart;
    q[9] = __builtin_amdgcn_s_memrealtime();
  }
#endif
}

}  // namespace tic
