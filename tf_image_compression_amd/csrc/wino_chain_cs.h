// wino_chain_cs.h — the stride-1 64->64 chain (wino_chain.h) with every 8x8 region split over
// TWO workgroups by output channels ("channel-split" shape, handle option chain_wh = 3).
//
// Why: a chain launch over n patches of R regions has only n*R 16-tile Winograd blocks —
// model_0's 16x16 stages at the two-lane batch of 32 patches give 128, half the chip's 256
// CUs (0.14 of peak).  Splitting the 64 output channels in halves doubles the
// workgroups (256 for 32 patches) without shrinking the MFMA N = 16-tile block.
//
// Same arithmetic as wino_chain_kernel / conv3x3_wino_kernel, operation for operation: wave
// xi computes points (xi, 0..3) for the 32 output channels of its half (two 16-row MFMA
// blocks), K order (16-channel chunk, t, lane group) unchanged, T = M A and Y = A^T T in the
// same order, the same epilogue — so every output is bit-identical to the unfused launch.
//
// Hand-off per layer: each workgroup publishes its half of the region's new 8x8 interior
// straight from the epilogue's registers (8 KB, 16-byte write-through sc1 stores, drained,
// then a per-(layer, region, half) flag);
// it then needs its partner's half of the interior (8 KB) and the 1-pixel halo ring in all
// 64 channels from the neighbouring regions' halves (9 KB), read with 16-byte sc1 buffer
// loads after polling those flags (MI355X_MICROARCH.md hand-off table, row 1).  Progress:
// tickets are handed out in order, a patch's 2R workgroups take consecutive tickets, every
// poll is bounded (error word, never a hang) — as in wino_chain.h.
#pragma once
#include "wino_chain.h"

namespace tic {

namespace chcs {
using chain::C;
using chain::HP;
using chain::KC;
using chain::LR;
using chain::NT;
using chain::PS;
using chain::RP;
using chain::TILE;
using chain::TTX;
constexpr int CH = 32;              // output channels per workgroup
constexpr int XS = CH + 8;          // T-exchange pitch (== 8 mod 16)
constexpr int XCH = 8 * NT * XS;    // [4 xi][2 b][16 tiles][XS] floats
constexpr int HALF_FLOATS = 64 * CH;  // one region half's published interior: 8x8 px x 32 ch
}  // namespace chcs

// WH: waves per transform-point row — 1: 256 threads, wave xi computes both 16-channel
// blocks of the half; 2: 512 threads, waves xi and xi + 4 take one block each (two waves per
// SIMD hide each other's LDS / L2 latency; per-output order unchanged, bit-identical).
template <int IN, int OUT, int WH = 1>
__global__ void __launch_bounds__(256 * WH, WH == 1 ? 2 : 1) wino_chain_cs_kernel(const ChainArgs a) {
  using namespace chcs;
  using chain::tpix;
  constexpr int NTH = 256 * WH;
  __shared__ __attribute__((aligned(16))) float smem[2 * TILE + XCH];
  __shared__ __attribute__((aligned(16))) float sbias[CH_MAX_LAYERS * C];
  __shared__ unsigned sh[2];
  const int tid = threadIdx.x;
  const int wv = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int xi = wv & 3, wh = wv >> 2;  // point row, 16-channel block part (WH = 2)
  const int lane = tid & 63, li = lane & 15, lg = lane >> 4;
  const int H = a.H, W = a.W, R = a.rh * a.rw, nR = a.n * R;
  auto stamp = [&](int k) {
    if (a.tstamp && tid == 0) a.tstamp[(size_t)blockIdx.x * CH_TS + k] = __builtin_amdgcn_s_memrealtime();
  };
  stamp(0);
  if (tid == 0) {
    sh[0] = a.dispatch_order ? blockIdx.x : __hip_atomic_fetch_add(&a.ctl[0], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    sh[1] = __hip_atomic_load(&a.ctl[2], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  for (int e = tid; e < a.nl * C; e += NTH) sbias[e] = a.layer[e / C].bias[e % C];
  __syncthreads();
  const int ticket = (int)sh[0];
  const unsigned epoch = sh[1] + 1u;
  const int half = ticket & 1, g = ticket >> 1;  // region g (of all patches), channel half
  const int nimg = g / R, reg = g % R;
  const int ry = reg / a.rw, rx = reg % a.rw;
  const int oy0 = ry * 8, ox0 = rx * 8;
  const int cbase = half * CH;  // first output channel of this workgroup

  // ---- this half's weights of layer l, step s = 4 kc + nu, from L2, PF steps ahead ----
  constexpr int NSTEP = 4 * KC, PF = 3, NBW = 2 / WH;
  f32x4 av[PF + 1][NBW];
  auto wglob = [&](int l, int s, int nb) -> f32x4 {
    const int kc = s >> 2, nu = s & 3;
    const float* wl = a.layer[l].wu + (size_t)xi * 64 * KC * C + (size_t)(lg * C + li) * 4;
    return *reinterpret_cast<const f32x4*>(wl + (size_t)(nu * KC + kc) * 16 * C + (2 * half + wh * NBW + nb) * 64);
  };
#pragma unroll
  for (int p = 0; p < PF; ++p)
#pragma unroll
    for (int nb = 0; nb < NBW; ++nb) av[p][nb] = wglob(0, p, nb);

  // ---- the first layer's input tile, all 64 channels (zero outside the image) ----
  const bool first_block = a.nl > 1 && a.layer[1].res;
  float* src = first_block ? smem : smem + TILE;
  {
    constexpr int NSTAGE = LR * 10 * (C / 4);
    constexpr int NIT = (NSTAGE + NTH - 1) / NTH;
    f32x4 tmp[NIT];
#pragma unroll
    for (int i = 0; i < NIT; ++i) {
      const int e = i * NTH + tid;
      tmp[i] = f32x4{0.f, 0.f, 0.f, 0.f};
      if (e < NSTAGE) {
        const int c4 = e % 16, pe = e / 16, col = pe % 10, row = pe / 10;
        const int iy = oy0 - 1 + row, ix = ox0 - 1 + col;
        if (iy >= 0 && iy < H && ix >= 0 && ix < W) {
          const size_t off = ((size_t)(nimg * H + iy) * W + ix) * C + c4 * 4;
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
    for (int i = 0; i < NIT; ++i) {
      const int e = i * NTH + tid;
      if (e < NSTAGE) {
        const int c4 = e % 16, pe = e / 16, col = pe % 10, row = pe / 10;
        *reinterpret_cast<f32x4*>(&src[tpix(row, col) + c4 * 4]) = tmp[i];
      }
    }
  }
  __syncthreads();
  stamp(1);

  const int iA = xi == 0 ? 0 : 1, iB = xi == 3 ? 3 : 2;
  const float sA = xi == 2 ? -1.f : 1.f, sB = (xi == 0 || xi == 3) ? -1.f : 1.f;
  const int ty_l = li / TTX, tx_l = li % TTX;
  const int offA = ((2 * ty_l + iA) * RP + tx_l) * PS + lg * 4;
  const int offB = ((2 * ty_l + iB) * RP + tx_l) * PS + lg * 4;
  // epilogue ownership: tile et, channel quad eq of this half, output row ay, and (WH = 2)
  // output column b0 (WH = 1: both columns)
  const int et = (tid & 127) >> 3, eq = tid & 7, ay = (tid >> 7) & 1, b0 = WH == 1 ? 0 : tid >> 8;
  constexpr int NBC = 2 / WH;  // output columns per thread
  const int ety = et / TTX, etx = et % TTX;
  const int co = cbase + 4 * eq;
  float* const xch = smem + 2 * TILE;
  bool failed = false;

  // read descriptors of this thread, the same for every layer: the partner's half of the
  // interior (512 chunks), then the halo ring in all 64 channels (576); LDS offset in the tile
  // and byte offset inside a layer's hand-off buffer (-1: outside the image, zero)
  constexpr int NPART = 64 * (CH / 4), NHALO = 36 * 16;
  constexpr int NLD = (NPART + NHALO + NTH - 1) / NTH;
  int rlds[NLD], rsrc[NLD];
#pragma unroll
  for (int k = 0; k < NLD; ++k) {
    const int e = k * NTH + tid;
    rlds[k] = rsrc[k] = -1;
    if (e < NPART) {
      const int px = e >> 3, q = e & 7;
      const int oh = 1 - half;
      rsrc[k] = (((g * 2 + oh) * 64 + px) * CH + 4 * q) * 4;
      rlds[k] = tpix((px >> 3) + 1, (px & 7) + 1) + oh * CH + 4 * q;
    } else if (e < NPART + NHALO) {
      const int hpq = e - NPART, hp = hpq >> 4, q = hpq & 15;
      int hy, hx;
      if (hp < 10) hy = -1, hx = hp - 1;
      else if (hp < 20) hy = 8, hx = hp - 11;
      else if (hp < 28) hy = hp - 20, hx = -1;
      else hy = hp - 28, hx = 8;
      rlds[k] = tpix(hy + 1, hx + 1) + 4 * q;
      const int gy = oy0 + hy, gx = ox0 + hx;
      if (gy >= 0 && gy < H && gx >= 0 && gx < W) {
        const int nry = ry + (hy < 0 ? -1 : (hy > 7 ? 1 : 0)), nrx = rx + (hx < 0 ? -1 : (hx > 7 ? 1 : 0));
        const int npx = (hy & 7) * 8 + (hx & 7);  // pixel inside the neighbour region
        const int gn = nimg * R + nry * a.rw + nrx;
        rsrc[k] = (((gn * 2 + (q >> 3)) * 64 + npx) * CH + 4 * (q & 7)) * 4;
      }
    }
  }

  for (int l = 0; l < a.nl; ++l) {
    const bool last = l == a.nl - 1;
    const bool res = a.layer[l].res != 0;
    float* const dst = src == smem ? smem + TILE : smem;
    float* const rsd = dst;  // res layers: the block input tile
    const int ts = 2 + 6 * l;
    stamp(ts);

    // ---- K loop (conv3x3_wino_kernel's order) ----
    f32x4 d[2][4];
    auto load_d = [&](int kc) {
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int cj = ((j & 1) * HP + (j >> 1)) * PS + kc * 16;
        d[0][j] = *reinterpret_cast<const f32x4*>(&src[offA + cj]);
        d[1][j] = *reinterpret_cast<const f32x4*>(&src[offB + cj]);
      }
    };
    f32x4 V[4];
    auto transform = [&]() {
      f32x4 r[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) r[j] = sA * d[0][j] + sB * d[1][j];
      V[0] = r[0] - r[2];
      V[1] = r[1] + r[2];
      V[2] = r[2] - r[1];
      V[3] = r[1] - r[3];
    };
    f32x4 acc[4][NBW];
#pragma unroll
    for (int nu = 0; nu < 4; ++nu)
#pragma unroll
      for (int nb = 0; nb < NBW; ++nb) acc[nu][nb] = f32x4{0.f, 0.f, 0.f, 0.f};
    load_d(0);
    transform();
#pragma unroll
    for (int kc = 0; kc < KC; ++kc) {
      if (kc + 1 < KC) load_d(kc + 1);
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int nu = 0; nu < 4; ++nu) {
        const int s = kc * 4 + nu;
        if (s + PF < NSTEP) {
#pragma unroll
          for (int nb = 0; nb < NBW; ++nb) av[(s + PF) % (PF + 1)][nb] = wglob(l, s + PF, nb);
        }
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int t = 0; t < 4; ++t)
#pragma unroll
          for (int nb = 0; nb < NBW; ++nb) acc[nu][nb] = mfma4(av[s % (PF + 1)][nb][t], V[nu][t], acc[nu][nb]);
        __builtin_amdgcn_sched_barrier(0);
      }
      __builtin_amdgcn_sched_barrier(0);
      if (kc + 1 < KC) transform();
    }
    if (!last) {
#pragma unroll
      for (int p = 0; p < PF; ++p)
#pragma unroll
        for (int nb = 0; nb < NBW; ++nb) av[p][nb] = wglob(l + 1, p, nb);
    }
    stamp(ts + 1);

    // ---- T = M A over nu through the exchange buffer (its own LDS space) ----
#pragma unroll
    for (int nb = 0; nb < NBW; ++nb) {
      const f32x4 m0 = acc[0][nb], m1 = acc[1][nb], m2 = acc[2][nb], m3 = acc[3][nb];
      float* x = &xch[(xi * 2 * NT + li) * XS + (wh * NBW + nb) * 16 + lg * 4];
      *reinterpret_cast<f32x4*>(x) = (m0 + m1) + m2;
      *reinterpret_cast<f32x4*>(x + NT * XS) = (m1 - m2) - m3;
    }
    __syncthreads();

    // ---- Y = A^T T for (tile et, quad eq, row ay), + bias, act, + residual ----
    const f32x4 bb = *reinterpret_cast<const f32x4*>(&sbias[l * C + co]);
    const bool relu = a.layer[l].act == ACT_RELU;
    f32x4 y[NBC];
#pragma unroll
    for (int bi = 0; bi < NBC; ++bi) {
      const int b = b0 + bi;
      f32x4 t[3];
#pragma unroll
      for (int j = 0; j < 3; ++j)
        t[j] = *reinterpret_cast<const f32x4*>(&xch[(((ay + j) * 2 + b) * NT + et) * XS + 4 * eq]);
      f32x4 v = ay == 0 ? (t[0] + t[1]) + t[2] : (t[0] - t[1]) - t[2];
      v.x = __fadd_rn(v.x, bb.x);
      v.y = __fadd_rn(v.y, bb.y);
      v.z = __fadd_rn(v.z, bb.z);
      v.w = __fadd_rn(v.w, bb.w);
      if (relu) {
        v.x = fmaxf(v.x, 0.f);
        v.y = fmaxf(v.y, 0.f);
        v.z = fmaxf(v.z, 0.f);
        v.w = fmaxf(v.w, 0.f);
      }
      if (res) {
        const f32x4 rr = *reinterpret_cast<const f32x4*>(&rsd[tpix(2 * ety + ay + 1, 2 * etx + b + 1) + co]);
        v.x = __fadd_rn(v.x, rr.x);
        v.y = __fadd_rn(v.y, rr.y);
        v.z = __fadd_rn(v.z, rr.z);
        v.w = __fadd_rn(v.w, rr.w);
      }
      y[bi] = v;
    }

    if (last) {  // ---- the chain's output: global f32 or the quantiser, this half's channels ----
#pragma unroll
      for (int bi = 0; bi < NBC; ++bi) {
        const int oy = oy0 + 2 * ety + ay, ox = ox0 + 2 * etx + b0 + bi;
        if (oy >= H || ox >= W) continue;
        const size_t o = ((size_t)(nimg * H + oy) * W + ox) * C + co;
        const f32x4 v = y[bi];
        if constexpr (OUT == OUT_F32) {
          *reinterpret_cast<f32x4*>(a.out + o) = v;
        } else {
          if (a.out) *reinterpret_cast<f32x4*>(a.out + o) = v;
          const uint32_t q = quant1(v.x, a.qscale) | (quant1(v.y, a.qscale) << 8) |
                             (quant1(v.z, a.qscale) << 16) | (quant1(v.w, a.qscale) << 24);
          *reinterpret_cast<uint32_t*>(a.qout + o) = q;
        }
      }
      stamp(ts + 2);
      break;
    }

    // ---- this half of the next layer's tile interior (zero outside the image), written to
    // LDS and published from the same registers: 16-byte write-through stores of the region
    // half's 8x8 x 32 channels, drained, then (after the barrier) the flag ----
    // (dst's interior is read by no one in this layer: res layers read it only at their own
    // output pixel, which this thread alone reads and then overwrites)
    const int gh = g * 2 + half;
    float* const xl = a.xbuf + (size_t)l * nR * 2 * HALF_FLOATS;  // this layer's slots
    {
      const __amdgpu_buffer_rsrc_t rpub = chain::xrsrc(xl + (size_t)gh * HALF_FLOATS, HALF_FLOATS * 4);
#pragma unroll
      for (int bi = 0; bi < NBC; ++bi) {
        const int ly = 2 * ety + ay, lx = 2 * etx + b0 + bi;
        const bool in_img = oy0 + ly < H && ox0 + lx < W;
        const f32x4 v = in_img ? y[bi] : f32x4{0.f, 0.f, 0.f, 0.f};
        *reinterpret_cast<f32x4*>(&dst[tpix(ly + 1, lx + 1) + co]) = v;
        chain::st_sc1_16(rpub, ((ly * 8 + lx) * CH + 4 * eq) * 4, v);
      }
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
      if (tid == 0)
        __hip_atomic_store(&a.flags[(size_t)l * nR * 2 + gh], epoch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    stamp(ts + 2);
    stamp(ts + 3);
    // ---- wait for the partner half and both halves of the (up to 8) neighbours ----
    if (tid < 18) {
      const int nbi = tid >> 1, hh = tid & 1;
      const int nry = ry + nbi / 3 - 1, nrx = rx + nbi % 3 - 1;
      if (!(nbi == 4 && hh == half) && nry >= 0 && nry < a.rh && nrx >= 0 && nrx < a.rw) {
        const unsigned* f = &a.flags[(size_t)l * nR * 2 + (size_t)(nimg * R + nry * a.rw + nrx) * 2 + hh];
        unsigned it = 0;
        while (__hip_atomic_load(f, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != epoch) {
          if (++it > chain::kSpinLimit) {
            failed = true;
            break;
          }
          __builtin_amdgcn_s_sleep(2);
        }
      }
    }
    __syncthreads();
    stamp(ts + 4);
    // ---- read the partner's half of the interior and the halo ring (all 64 channels), from
    // the descriptors computed once before the layer loop (all loads first) ----
    {
      const __amdgpu_buffer_rsrc_t rlay = chain::xrsrc(xl, (unsigned)nR * 2 * HALF_FLOATS * 4);
      f32x4 v[NLD];
#pragma unroll
      for (int k = 0; k < NLD; ++k) v[k] = rsrc[k] >= 0 ? chain::ld_sc1_16(rlay, rsrc[k]) : f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int k = 0; k < NLD; ++k)
        if (rlds[k] >= 0) *reinterpret_cast<f32x4*>(&dst[rlds[k]]) = v[k];
    }
    __syncthreads();
    stamp(ts + 5);
    src = dst;
  }

  if (failed) __hip_atomic_store(&a.ctl[3], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  __syncthreads();
  if (tid == 0) {
    const unsigned done = __hip_atomic_fetch_add(&a.ctl[1], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (done == gridDim.x - 1) {
      __hip_atomic_store(&a.ctl[1], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store(&a.ctl[0], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store(&a.ctl[2], epoch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
}

}  // namespace tic
