// wino4_pchain.h — a run of stride-1 3x3 64->64 convolutions on a 16x16 map in ONE launch,
// every layer in Winograd F(4x4,3x3) exactly as conv3x3_wino4_kernel computes it: model_0/1's
// 16x16 stage at 256x256 patches and model_2's at 128x128 — encode_res_1..encode_4 with the
// quantiser (model_0/model.py:98-144) and decode_4 (dequantiser) .. decode_res_2 (:148-196),
// the res_block convs of basic_block/basic_block.py:74-93.
//
// A 16x16 map is exactly sixteen 4x4 output tiles = one MFMA block (N = 16 tiles), so a
// patch needs no spatial hand-off at all.  Four workgroups per patch, one per quarter q of the
// output channels (M = 16): each keeps the patch's whole 18x18x64 input tile in LDS (the
// standalone kernel's TTY = 4 layout: columns split by column mod 4, pixel stride 72 floats,
// conflict-free ds_read_b128), computes its 16 output channels for all 16 tiles and every
// transform point, and between layers publishes its slice (256 px x 16 ch = 16 KB) with
// write-through (sc1) 16-byte stores and a per-(layer, patch, quarter) flag; after the three
// partners' flags it reads their slices (48 KB, sc1 loads) into the tile (MI355X_MICROARCH.md
// hand-off table, row 1).  The res_block input a conv_1 adds is held in registers by the
// thread that computed it (the epilogue mapping is the same in every layer).
//
// Waves: 6 (384 threads), wave xi = row xi of B^T: it reads row xi of B^T d for its lane's
// tile and channel quad (staged once per layer, as conv3x3_wino4_kernel stages it: a pass over
// (tile row, column, channel quad) turns the layer's 18x18 input into the 24 rows of B^T d),
// forms the six column combinations V_(xi, nu) in registers, and runs the six point GEMMs
// (M = 16 output channels, N = 16 tiles, K = 64) as 6 x 16 v_mfma_f32_16x16x4_f32 per layer,
// issued (tt, nu)-major so consecutive MFMAs use different accumulators.  Every accumulator
// still sums in the standalone kernel's order (16-channel chunk kc, then t), the transforms
// are the same functions (w4_bt / w4_at, conv3x3_wino4.h) and the epilogue the same
// operations, so every layer is bit-identical to its conv3x3_wino4_kernel launch
// (tests/test_gpu_pchain.py).
//
// Progress: the four quarters of a patch wait for each other, so they must be co-resident;
// work is handed out by an atomic ticket (wino_chain.h: at most the last patch is incomplete
// and the ones ahead of it never wait on it), every poll is bounded (error word, never a hang),
// and the last workgroup to finish resets the ticket and advances the launch epoch the flags
// are compared against.
#pragma once
#include "conv3x3_wino4.h"
#include "wino_chain.h"

namespace tic {

namespace pchain {
constexpr int C = 64, KC = 4;
constexpr int NT = 16, TTX = 4, LR = 18, LCOL = 18, HPP = 5, PS = 72;
constexpr int RS = 4 * HPP * PS + 16;  // floats per staged row (conv3x3_wino4_kernel, TTY = 4)
constexpr int LT = 24;                 // rows of B^T d: six per tile row
constexpr int TILE = LT * RS;          // 34944 floats = 137 KB; the raw 18x18 input (rows
                                       // 0..17, same pitch) and the T exchange alias it
constexpr int CQ = 16;                // output channels per workgroup
constexpr int XS = CQ + 4;            // T-exchange pitch per (xi, b, tile)
constexpr int XCH = 24 * NT * XS;     // 7680 floats: aliases rows 0..5 of the (dead) tile
constexpr int NTH = 384;
constexpr int SLICE = 256 * CQ;  // floats a workgroup publishes per layer: [256 px][16 ch]
constexpr int NBT = 4 * LCOL * 16 / NTH;  // B^T d tasks (tile row, column, quad) per thread: 3
static_assert(NBT * NTH == 4 * LCOL * 16, "B^T d tasks split evenly");

// LDS float offset of staged pixel (row, col) of the 18x18 tile (columns split by col mod 4);
// row 6 ty + xi of the B^T d rows uses the same column layout
__device__ __forceinline__ int tpix(int row, int col) { return row * RS + ((col & 3) * HPP + (col >> 2)) * PS; }
// B^T d task k of thread t: (tile row, column, channel quad)
__device__ __forceinline__ void bt_task(int t, int k, int& ty, int& col, int& c4) {
  const int e = k * NTH + t, p = e >> 4;
  c4 = e & 15;
  ty = p / LCOL;
  col = p - ty * LCOL;
}
}  // namespace pchain

// IN: IN_F32 / IN_IDX for the first layer; OUT: OUT_F32 / OUT_QUANT for the last one.
// ChainArgs as for wino_chain_kernel: layer[].wu = the F(4x4,3x3) U packing (pack_wino4),
// xbuf = [nl-1][n][4 quarters][SLICE] f32, flags = [nl-1][n][4], rh / rw unused.
template <int IN, int OUT>
__global__ void __launch_bounds__(pchain::NTH) wino4_pchain_kernel(const ChainArgs a) {
  using namespace pchain;
  __shared__ __attribute__((aligned(16))) float smem[TILE];
  __shared__ __attribute__((aligned(16))) float sbias[CH_MAX_LAYERS * CQ];
  __shared__ unsigned sh[2];
  const int tid = threadIdx.x;
  const int xi = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int lane = tid & 63, li = lane & 15, lg = lane >> 4;
  const int H = a.H, W = a.W, nQ = a.n * 4;
  auto stamp = [&](int k) {
    if (a.tstamp && tid == 0) a.tstamp[(size_t)blockIdx.x * CH_TS + k] = __builtin_amdgcn_s_memrealtime();
  };
  stamp(0);
  if (tid == 0) {
    sh[0] = a.dispatch_order ? blockIdx.x
                             : __hip_atomic_fetch_add(&a.ctl[0], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    sh[1] = __hip_atomic_load(&a.ctl[2], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  __syncthreads();
  const int ticket = (int)sh[0];
  const unsigned epoch = sh[1] + 1u;
  const int nimg = ticket >> 2, q = ticket & 3, co0 = CQ * q;
  for (int e = tid; e < a.nl * CQ; e += NTH) sbias[e] = a.layer[e / CQ].bias[co0 + e % CQ];

  // ---- A fragments (U) of layer l from L2: one f32x4 per (kc, nu), a chunk at a time, by
  // buffer loads (descriptor in SGPRs, the lane's byte offset in one VGPR, the (kc, nu) step as
  // a scalar offset: no per-step 64-bit addresses for the compiler to hoist and spill) ----
  const int wlane = ((6 * xi * KC * 16 * C) + (lg * C + co0 + li) * 4) * 4;  // bytes
  auto wsrc = [&](int l) {
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(a.layer[l].wu), (short)0, 36 * KC * 16 * C * 4,
                                             0x00020000);
  };
  auto wload = [&](__amdgpu_buffer_rsrc_t r, int kc, f32x4 (&dst)[6]) {
    int vo = wlane;
    asm volatile("" : "+v"(vo));
#pragma unroll
    for (int nu = 0; nu < 6; ++nu) {
      const w4u32x4 u = __builtin_amdgcn_raw_buffer_load_b128(r, vo, (nu * KC + kc) * 16 * C * 4, 0);
      dst[nu] = f32x4{__uint_as_float(u.x), __uint_as_float(u.y), __uint_as_float(u.z), __uint_as_float(u.w)};
    }
  };
  f32x4 av[2][6];
  wload(wsrc(0), 0, av[0]);

  // the chain input at (pixel, channel quad c4), zero outside the image (SAME padding)
  auto load_in = [&](int iy, int ix, int c4) -> f32x4 {
    if ((unsigned)iy >= (unsigned)H || (unsigned)ix >= (unsigned)W) return f32x4{0.f, 0.f, 0.f, 0.f};
    const size_t off = ((size_t)(nimg * H + iy) * W + ix) * C + c4 * 4;
    if constexpr (IN == IN_F32) {
      return *reinterpret_cast<const f32x4*>(reinterpret_cast<const float*>(a.in) + off);
    } else {
      const uint32_t s = *reinterpret_cast<const uint32_t*>(reinterpret_cast<const uint8_t*>(a.in) + off);
      return f32x4{a.lut[s & 0xff], a.lut[(s >> 8) & 0xff], a.lut[(s >> 16) & 0xff], a.lut[s >> 24]};
    }
  };

  // the six B^T d rows of task (ty, col, c4) from its six input rows d (w4_bt over rows)
  auto bt_store = [&](int ty, int col, int c4, const f32x4 (&d)[6]) {
    f32x4 bt[6];
    w4_bt(d, bt);
#pragma unroll
    for (int r = 0; r < 6; ++r) *reinterpret_cast<f32x4*>(&smem[tpix(6 * ty + r, col) + c4 * 4]) = bt[r];
  };
  // ---- stage the first layer's B^T d rows straight from its input (zero outside the image) ----
  {
    f32x4 tmp[NBT][6];
#pragma unroll
    for (int k = 0; k < NBT; ++k) {
      int ty, col, c4;
      bt_task(tid, k, ty, col, c4);
#pragma unroll
      for (int r = 0; r < 6; ++r) tmp[k][r] = load_in(4 * ty + r - 1, col - 1, c4);
    }
#pragma unroll
    for (int k = 0; k < NBT; ++k) {
      int ty, col, c4;
      bt_task(tid, k, ty, col, c4);
      bt_store(ty, col, c4, tmp[k]);
    }
  }

  // ---- epilogue ownership: threads 0..255 each own (output column b, tile, channel quad q4)
  // and the four output rows of that tile column, in every layer (the indices are re-derived
  // from an opaque copy of tid where they are used: held across the layer loop, they spill) ----
  struct Own {
    bool task;
    int q4, et, eb, oy0, ox, cq;
  };
  auto own = [&](int t) {
    Own o;
    o.task = t < 256;
    o.q4 = t & 3;
    o.et = (t >> 2) & 15;
    o.eb = (t >> 6) & 3;
    o.oy0 = 4 * (o.et / TTX);
    o.ox = 4 * (o.et % TTX) + o.eb;
    o.cq = co0 + 4 * o.q4;  // this thread's 4 output channels
    return o;
  };
  // the res_block input a conv_1 adds: the chain input when layer 1 is a conv_1
  f32x4 resid[4];
  {
    const Own o = own(tid);
#pragma unroll
    for (int ay = 0; ay < 4; ++ay)
      resid[ay] = o.task && a.nl > 1 && a.layer[1].res ? load_in(o.oy0 + ay, o.ox, o.cq / 4) : f32x4{0.f, 0.f, 0.f, 0.f};
  }
  __syncthreads();
  stamp(1);

  // ---- row xi of B^T d for tile li, column j, chunk kc: one staged value ----
  const int ty = li / TTX, tx = li % TTX;
  const int tbase = (6 * ty + xi) * RS + tx * PS + lg * 4;
  auto ld = [&](int j, int kc) -> f32x4 {
    return *reinterpret_cast<const f32x4*>(&smem[tbase + ((j & 3) * HPP + (j >> 2)) * PS + kc * 16]);
  };

  bool failed = false;
  for (int l = 0; l < a.nl; ++l) {
    const bool last = l == a.nl - 1;
    const int ts = 2 + 6 * l;
    stamp(ts);
    const __amdgpu_buffer_rsrc_t wl = wsrc(l);

    // ---- K loop: per chunk kc the six A fragments (next chunk's in flight), 24 MFMAs in
    // (t, nu) order; the next chunk's columns are read before and combined after each group
    f32x4 V[6];
    {
      f32x4 r[6];
#pragma unroll
      for (int j = 0; j < 6; ++j) r[j] = ld(j, 0);
      w4_bt(r, V);
    }
    f32x4 acc[6];
#pragma unroll
    for (int nu = 0; nu < 6; ++nu) acc[nu] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int kc = 0; kc < KC; ++kc) {
      const bool next = kc + 1 < KC;
      if (next) wload(wl, kc + 1, av[(kc + 1) & 1]);
      else if (!last) wload(wsrc(l + 1), 0, av[0]);  // the next layer's first chunk
      f32x4 rn[6];
#pragma unroll
      for (int g = 0; g < 6; ++g) {
        if (next) rn[g] = ld(g, kc + 1);
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int m = 4 * g; m < 4 * g + 4; ++m) {
          const int tt = m / 6, nu = m % 6;
          acc[nu] = mfma4(av[kc & 1][nu][tt], V[nu][tt], acc[nu]);
        }
        __builtin_amdgcn_sched_barrier(0);
      }
      if (next) w4_bt(rn, V);
    }
    stamp(ts + 1);

    // ---- T = M A over nu (per wave), exchanged through LDS (rows 0..5 of the dead tile) ----
    __syncthreads();
    {
      f32x4 tb[4];
      w4_at(acc, tb);
#pragma unroll
      for (int b = 0; b < 4; ++b) *reinterpret_cast<f32x4*>(&smem[((xi * 4 + b) * NT + li) * XS + lg * 4]) = tb[b];
    }
    __syncthreads();

    // ---- Y = A^T T for (column eb, tile et, quad q4), my_conv2d's epilogue ----
    const bool res = a.layer[l].res != 0;
    const bool relu = a.layer[l].act == ACT_RELU;
    int tl = tid;
    asm volatile("" : "+v"(tl));
    const Own o = own(tl);
    const bool task = o.task;
    const int q4 = o.q4, et = o.et, eb = o.eb, oy0 = o.oy0, ox = o.ox, cq = o.cq;
    f32x4 y[4];
    if (task) {
      f32x4 T[6];
#pragma unroll
      for (int x2 = 0; x2 < 6; ++x2)
        T[x2] = *reinterpret_cast<const f32x4*>(&smem[((x2 * 4 + eb) * NT + et) * XS + 4 * q4]);
      w4_at(T, y);
      const f32x4 bb = *reinterpret_cast<const f32x4*>(&sbias[l * CQ + 4 * q4]);
#pragma unroll
      for (int ay = 0; ay < 4; ++ay) {
        f32x4 v = y[ay];
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
          v.x = __fadd_rn(v.x, resid[ay].x);
          v.y = __fadd_rn(v.y, resid[ay].y);
          v.z = __fadd_rn(v.z, resid[ay].z);
          v.w = __fadd_rn(v.w, resid[ay].w);
        }
        // outside the image: zero (the next layer's SAME padding)
        y[ay] = (oy0 + ay < H && ox < W) ? v : f32x4{0.f, 0.f, 0.f, 0.f};
      }
    }

    if (last) {  // ---- the chain's output: global f32 or the quantiser ----
      if (task) {
#pragma unroll
        for (int ay = 0; ay < 4; ++ay) {
          const int oy = oy0 + ay;
          if (oy >= H || ox >= W) continue;
          const size_t o = ((size_t)(nimg * H + oy) * W + ox) * C + cq;
          const f32x4 v = y[ay];
          if constexpr (OUT == OUT_F32) {
            *reinterpret_cast<f32x4*>(a.out + o) = v;
          } else {
            if (a.out) *reinterpret_cast<f32x4*>(a.out + o) = v;
            const uint32_t qv = quant1(v.x, a.qscale) | (quant1(v.y, a.qscale) << 8) |
                                (quant1(v.z, a.qscale) << 16) | (quant1(v.w, a.qscale) << 24);
            *reinterpret_cast<uint32_t*>(a.qout + o) = qv;
          }
        }
      }
      stamp(ts + 2);
      break;
    }

    // ---- this quarter's slice into the tile and published (16-byte write-through stores) ----
    __syncthreads();  // every thread has read its T (the exchange aliases tile rows 0..5)
    const float* const xl = a.xbuf + (size_t)l * nQ * SLICE;  // layer l's slices
    const __amdgpu_buffer_rsrc_t rpub = chain::xrsrc(xl + (size_t)(nimg * 4 + q) * SLICE, SLICE * 4);
    if (task) {
      const bool keep = l + 2 < a.nl && a.layer[l + 2].res;  // layer l + 1 starts a res_block
#pragma unroll
      for (int ay = 0; ay < 4; ++ay) {
        const int oy = oy0 + ay;
        *reinterpret_cast<f32x4*>(&smem[tpix(oy + 1, ox + 1) + cq]) = y[ay];
        chain::st_sc1_16(rpub, ((oy * 16 + ox) * CQ + 4 * q4) * 4, y[ay]);
        if (keep) resid[ay] = y[ay];
      }
    }
    // the zero ring of the raw 18x18 input (the B^T d rows and the exchange overwrote it):
    // rows 0 / 17, and columns 0 / 17 of rows 1..16
    for (int e = tl; e < 68 * 16; e += NTH) {
      const int rp = e >> 4, c4 = e & 15;
      const int row = rp < 36 ? (rp < 18 ? 0 : 17) : 1 + ((rp - 36) >> 1);
      const int col = rp < 36 ? (rp < 18 ? rp : rp - 18) : (((rp - 36) & 1) ? 17 : 0);
      *reinterpret_cast<f32x4*>(&smem[tpix(row, col) + 4 * c4]) = f32x4{0.f, 0.f, 0.f, 0.f};
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    stamp(ts + 2);

    // ---- hand-off: raise this quarter's flag, wait for the three partners', read their slices ----
    unsigned* const fl = a.flags + (size_t)l * nQ + nimg * 4;
    if (tid == 0) __hip_atomic_store(&fl[q], epoch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    stamp(ts + 3);
    if (a.probe == 0 && tid < 4 && tid != q) {
      unsigned it = 0;
      while (__hip_atomic_load(&fl[tid], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != epoch) {
        if (++it > chain::kSpinLimit) {
          failed = true;
          break;
        }
        __builtin_amdgcn_s_sleep(2);
      }
    }
    __syncthreads();
    stamp(ts + 4);
    {
      const __amdgpu_buffer_rsrc_t rlay = chain::xrsrc(xl + (size_t)nimg * 4 * SLICE, 4 * SLICE * 4);
      constexpr int NLD = 3 * SLICE / 4 / NTH;  // 8 16-byte loads per thread
      static_assert(NLD * NTH == 3 * SLICE / 4, "partner slices split evenly");
      f32x4 hv[NLD];
#pragma unroll
      for (int k = 0; k < NLD; ++k) {
        const int e = k * NTH + tl, p = e >> 10, qp = p < q ? p : p + 1, f = e & 1023;
        hv[k] = a.probe == 0 ? chain::ld_sc1_16(rlay, (qp * SLICE + f * 4) * 4) : f32x4{0.f, 0.f, 0.f, 0.f};
      }
#pragma unroll
      for (int k = 0; k < NLD; ++k) {
        const int e = k * NTH + tl, p = e >> 10, qp = p < q ? p : p + 1, f = e & 1023;
        const int px = f >> 2, c4 = f & 3;
        *reinterpret_cast<f32x4*>(&smem[tpix((px >> 4) + 1, (px & 15) + 1) + CQ * qp + 4 * c4]) = hv[k];
      }
    }
    __syncthreads();
    // ---- the next layer's B^T d rows from the raw tile (read all, then overwrite) ----
    {
      f32x4 d[NBT][6];
#pragma unroll
      for (int k = 0; k < NBT; ++k) {
        int ty2, col, c4;
        bt_task(tl, k, ty2, col, c4);
#pragma unroll
        for (int r = 0; r < 6; ++r) d[k][r] = *reinterpret_cast<const f32x4*>(&smem[tpix(4 * ty2 + r, col) + c4 * 4]);
      }
      __syncthreads();
#pragma unroll
      for (int k = 0; k < NBT; ++k) {
        int ty2, col, c4;
        bt_task(tl, k, ty2, col, c4);
        bt_store(ty2, col, c4, d[k]);
      }
    }
    __syncthreads();
    stamp(ts + 5);
  }

  // ---- the last workgroup to finish resets the ticket and advances the epoch ----
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
