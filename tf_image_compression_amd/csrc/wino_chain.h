// wino_chain.h — a chain of stride-1 3x3 64->64 convolutions in ONE launch: the residual
// stages of the codecs (basic_block.res_block, basic_block/basic_block.py:74-93) with the
// plain stride-1 layer on either side of them — model_0/1 encode_res_1..encode_4 with the
// quantiser (model_0/model.py:98-144) and decode_4 (dequantiser LUT) .. decode_res_2
// (:148-196); model_3's residual stages at H/4 and H/8 (model_3/model.py:66-150,191-281);
// the rmbe net's conv_3/conv_4 (submit/2/rmbe/model.py:140-160).
//
// Form: Winograd F(2x2,3x3) exactly as conv3x3_wino_kernel computes it — same U packing,
// same B^T d B in registers, same MFMA K order (16-channel chunk, t, lane group), same
// A^T M A and the same epilogue — so every layer's output is bit-identical to the unfused
// launch of that layer (tests/test_gpu_parity.py::test_wino_chain_bit_identical).
//
// Decomposition: one 256-thread workgroup owns an 8x8 output REGION of one patch for every
// layer of the chain (16 Winograd tiles = one 16-tile MFMA block; wave xi owns the
// transform points (xi, 0..3)); the region's 10x10 input tile (1-pixel halo) stays in LDS
// from layer to layer.  Between layers a region needs its neighbours' border pixels: each
// workgroup publishes its 32 border pixels (rows 0 and 7, columns 0 and 7; 8 KB) straight
// from its epilogue registers with write-through (sc1) 16-byte buffer stores, drains them, and
// raises a per-(layer, region) flag; the neighbours poll the flags with sc1 loads and read the halo with 16-byte sc1
// buffer loads
// (MI355X_MICROARCH.md, valid hand-off form, row 1).  No redundant halo recomputation,
// ~1 hand-off per layer instead of a kernel boundary + full activation round trip.
//
// Progress: the regions of a patch wait for each other, so they must be co-resident.
// Work is handed out by a ticket (one atomic per workgroup at start): a workgroup that runs
// holds ticket t only if tickets 0..t-1 were taken by workgroups that are running or done,
// so the regions of one patch (consecutive tickets) never wait on a region that cannot be
// scheduled — at most the last patch is incomplete, and the workgroups ahead of it finish
// without waiting on it.  Every poll is bounded as well (error flag, never a hang).
// The last workgroup to finish resets the ticket and advances the launch epoch that the
// flags are compared against, so no buffer needs clearing between launches.
//
// Stride-2 neighbours (HT, round 5): the encoder's stride-2 layer in front of the run
// (model_0/1/2 encode_3, model_0/model.py:90-96) can run as the chain's HEAD, and the
// decoder's transposed layer behind it (decode_3, :198-206) as its TAIL, in the same
// launch.  The head stages the 17x17 input window of its 8x8 output region (columns split by
// parity, so the 8 outputs of a row read consecutive LDS pixels), runs conv3x3_kernel<
// MODE_S2>'s implicit GEMM in its exact step order (tap-major, 16-channel chunk, t), and
// hands its output border over like a chain layer; the tail runs conv3x3_kernel<MODE_T2>'s
// four sub-pixel phases from the run's last tile (halo from one more hand-off) and writes
// the 16x16 output tile of its region.  Both are bit-identical to the standalone launches
// (tests/test_gpu_chain.py); they remove two launches per lane and their HBM round trips.
#pragma once
#include "conv3x3_pwino.h"

#ifndef CH_D2_EARLY
#define CH_D2_EARLY 0  // experiment: decode_2's phases stored as soon as their last tap is done
#endif
#ifndef CH_D2_PF
#define CH_D2_PF 2     // decode_2's weight prefetch distance (steps)
#endif

namespace tic {

constexpr int CH_MAX_LAYERS = 8;
// timestamps per workgroup: kernel start, input staged, then per layer: start, K loop done,
// epilogue done, border published, neighbours' flags seen, halo staged; then the head's six
// (window staged, K loop done, epilogue done, published, flags seen, halo staged) and the
// tail's (start, K loop done, stores issued)
// tail's (start, K loop done, stores issued); then the same phase ends seen by wave 4 (the
// second wave on SIMD 0: thread 0's phases also hold the wait for it) — per layer its K-loop
// end, the head's and the tail's K-loop ends, decode_2's K-loop end and stores issued — and
// the workgroup's end (after its last barrier)
constexpr int CH_HEAD_TS = 2 + 6 * CH_MAX_LAYERS, CH_TAIL_TS = CH_HEAD_TS + 6;
constexpr int CH_W4_TS = CH_TAIL_TS + 6, CH_W4_HEAD = CH_W4_TS + CH_MAX_LAYERS, CH_W4_TAIL = CH_W4_HEAD + 1;
constexpr int CH_END_TS = CH_W4_TAIL + 3, CH_TS = CH_END_TS + 1;
constexpr int CH_HEAD = 1, CH_TAIL = 2, CH_TAIL2 = 4;  // HT bits (CH_TAIL2 needs CH_TAIL)
// decode_2 behind the tail in the polyphase Winograd form (s2_form 1; needs CH_TAIL2)
constexpr int CH_TAIL2_PW = 8;

struct ChainLayer {
  const float* wu;    // Winograd U [16 p][4 kc][4 g][64][4 t] (pack_wino)
  const float* bias;  // [64]
  int act;            // ACT_ID / ACT_RELU
  int res;            // + the res_block input after the activation (res_block conv_1)
};

struct ChainArgs {
  ChainLayer layer[CH_MAX_LAYERS];
  int nl;               // layers in the chain (2..CH_MAX_LAYERS)
  const void* in;       // first layer's input: f32 [n,H,W,64] or u8 symbols (IN_IDX)
  const float* lut;     // IN_IDX: dequantiser table
  float* out;           // last layer: f32 [n,H,W,64] (OUT_F32) / optional pre-activation (OUT_QUANT)
  uint8_t* qout;        // OUT_QUANT: u8 symbols [n,H,W,64]
  float qscale;         // Q - 1
  int H, W;             // spatial size of every layer (stride 1)
  int rh, rw;           // 8x8 regions per patch: ceil(H/8) x ceil(W/8)
  int n;                // patches
  float* xbuf;          // border exchange [nl-1][n*R][4 sides][8 px][64] f32
  unsigned* flags;      // [nl-1][n*R] epoch flags
  unsigned* ctl;        // [0] ticket, [1] done count, [2] epoch, [3] error (poll timeout)
  int dispatch_order;   // 1: a workgroup's region is its blockIdx.x (the hardware's in-order
                        // dispatch); 2: the same, XCD-aware (chain_region); 0: an atomic ticket
                        // (order guaranteed whatever the dispatch)
  int probe;            // timing probes only (TIC_CHAIN_PROBE; results invalid unless 0):
                        // 1 = no hand-off at all, 2 = publish but do not wait / read
  unsigned long long* tstamp;  // phase timestamps (TIC_CHAIN_TIMING; results stay valid) or
                               // null: [workgroup][CH_TS] s_memrealtime (100 MHz) by thread 0
  // HT & CH_HEAD: the stride-2 64->64 layer in front of the run.  head.wu = its direct
  // packing [9 tap][4 kc][4 g][64][4 t] (pack_generic); head_in f32 [n, hH, hW, 64], TF SAME
  // pad_before hpad; its output (H x W) is the run's first input (the block input).
  ChainLayer head;
  const float* head_in;
  int hH, hW, hpad;
  // HT & CH_TAIL: the stride-2 transposed 64->64 layer behind the run (direct packing of the
  // [3,3,Cout,Cin] kernel); the run's last output stays in LDS, the tail writes f32
  // [n, 2H, 2W, 64] to tail_out.
  ChainLayer tail;
  float* tail_out;
  // HT & CH_TAIL2: the next transposed layer too (decode_2, 64 -> 32; direct packing with
  // Cout 32): the tail's output stays in LDS as its input (the halo row / column recomputed
  // from the run's halo ring), it writes f32 [n, 4H, 4W, 32] to tail2_out.
  ChainLayer tail2;
  float* tail2_out;
};

namespace chain {
constexpr int C = 64, PS = 72, KC = 4;  // channels, LDS pixel stride (floats), 16-ch chunks
constexpr int HP = 5, RP = 10, LR = 10; // parity half-row, row pitch (pixels), rows: 10x10 tile
constexpr int NT = 16, TTX = 4;         // 2x2 tiles per region, tiles per tile row
constexpr int XS = C;                   // T-exchange pitch (16-byte chunks permuted: xq)
constexpr int TILE = LR * RP * PS;      // 7200 floats
constexpr int XCH = 8 * NT * XS;        // 8192 floats
constexpr int TB = TILE > XCH ? TILE : XCH;
constexpr unsigned kSpinLimit = 1u << 19;  // ~0.5 s of polling before the error flag

// LDS float offset of staged pixel (row, col) of a 10x10 tile (columns split by parity)
__device__ __forceinline__ int tpix(int row, int col) { return (row * RP + (col & 1) * HP + (col >> 1)) * PS; }

// LDS bank layout (MI355X_MICROARCH.md §LDS; model and search: tools/lds/chain_banks.py).
// T exchange: channel quad q of tile `tile` sits in 16-byte chunk xq(tile, q) of the tile's
// 256-byte row, so the K-loop waves' writes (8 consecutive tiles, one quad: 8 distinct bank
// slots) and the epilogue's reads (below) are conflict-free — the 72-float pitch before made
// them 2-way.
__device__ __forceinline__ int xq(int tile, int q) { return (q + 2 * tile + ((tile >> 2) & 1)) & 15; }
// Epilogue ownership: lane l of a wave takes tile 4 (wave % 4) + (l >> 4) and channel quad
// (l - 2 (l >> 4)) mod 16 — with the tile's pixel pitch (18 chunks ≡ 2 mod 16) every 16-lane
// read group of the residual / tile accesses then hits 16 distinct slots (quad = l mod 16 was
// 2-way on the residual reads).
__device__ __forceinline__ int epi_quad(int tid) { return ((tid & 15) - 2 * ((tid >> 4) & 3)) & 15; }
// Stride-2 head / transposed tail: lane li of a wave owns region column dcol(li & 7) of its row
// (bits 1 and 2 swapped): the tail's tile reads 4 -> 1.3 extra LDS cycles per instruction.
__device__ __forceinline__ int dcol(int i) { return (i & 1) | ((i & 2) << 1) | ((i & 4) >> 1); }

// Dispatch order 2: blocks b and b + 8 are dealt to one XCD (MI355X_MICROARCH.md), so block b
// of a group of 8 R blocks takes region r of patch (group * 8 + b % 8) with r = (b / 8) % R:
// the R regions of a patch, which hand their borders to each other every layer, run on ONE
// XCD and meet in its L2 instead of crossing the fabric.  A bijection on [0, n R): the last
// n % 8 patches keep the identity.
__device__ __forceinline__ unsigned chain_region(unsigned b, unsigned R, unsigned n) {
  const unsigned full = (n / 8) * 8 * R;
  if (b >= full) return b;
  const unsigned x = b & 7u, s = b >> 3;
  return ((s / R) * 8 + x) * R + s % R;
}

// a - b on four floats as two packed adds with the second operand negated (v_pk_add_f32
// neg_lo / neg_hi: each lane is the IEEE subtraction a + (-b), one rounding, the same value as
// v_sub_f32), where hipcc lowers the vector subtraction to four unpacked v_sub_f32; at f32 the
// VALU instructions beside the MFMAs add to the matrix time
typedef float f32x2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ f32x4 psub(const f32x4 a, const f32x4 b) {
  const f32x2 alo = {a.x, a.y}, ahi = {a.z, a.w}, blo = {b.x, b.y}, bhi = {b.z, b.w};
  f32x2 lo, hi;
  asm("v_pk_add_f32 %0, %1, %2 neg_lo:[0,1] neg_hi:[0,1]" : "=v"(lo) : "v"(alo), "v"(blo));
  asm("v_pk_add_f32 %0, %1, %2 neg_lo:[0,1] neg_hi:[0,1]" : "=v"(hi) : "v"(ahi), "v"(bhi));
  return f32x4{lo.x, lo.y, hi.x, hi.y};
}

// 16-byte write-through (sc1) store / sc1 load through a buffer resource (aux 16 = sc1):
// one buffer_store/load_dwordx4 instead of two 8-byte atomics (MI355X_MICROARCH.md: 8-B
// accesses run at 0.54-0.70x the 16-B rate; hand-off table row 1 allows 16-B sc1 both sides)
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
__device__ __forceinline__ __amdgpu_buffer_rsrc_t xrsrc(const float* base, unsigned bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(base), (short)0, (int)bytes, 0x00020000);
}
__device__ __forceinline__ void st_sc1_16(__amdgpu_buffer_rsrc_t r, int byte_off, f32x4 v) {
  const u32x4 u = {__float_as_uint(v.x), __float_as_uint(v.y), __float_as_uint(v.z), __float_as_uint(v.w)};
  __builtin_amdgcn_raw_buffer_store_b128(u, r, byte_off, 0, 16);
}
__device__ __forceinline__ f32x4 ld_sc1_16(__amdgpu_buffer_rsrc_t r, int byte_off) {
  const u32x4 u = __builtin_amdgcn_raw_buffer_load_b128(r, byte_off, 0, 16);
  return f32x4{__uint_as_float(u.x), __uint_as_float(u.y), __uint_as_float(u.z), __uint_as_float(u.w)};
}

}  // namespace chain

// IN: IN_F32 / IN_IDX for the first layer; OUT: OUT_F32 / OUT_QUANT for the last one.
// WH: waves per transform-point row — 1: a 256-thread workgroup, wave xi computes all 64
// output channels of points (xi, 0..3); 2: a 512-thread workgroup, waves xi and xi + 4
// split the output channels in halves (two waves per SIMD hide each other's LDS / L2
// latency; every output's fma order is unchanged, so both are bit-identical).
template <int IN, int OUT, int WH = 1, int HT = 0>
__global__ void __launch_bounds__(256 * WH, WH == 1 ? 2 : 1) wino_chain_kernel(const ChainArgs a) {
  using namespace chain;
  constexpr int NTH = 256 * WH;
  constexpr bool HEAD = (HT & CH_HEAD) != 0, TAIL = (HT & CH_TAIL) != 0, TAIL2 = (HT & CH_TAIL2) != 0;
  constexpr bool TAIL2_PW = (HT & CH_TAIL2_PW) != 0;
  static_assert(!TAIL2_PW || TAIL2, "the polyphase decode_2 is the one behind the tail");
  static_assert(!TAIL2 || TAIL, "decode_2 runs on the tail's output");
  static_assert(HT == 0 || WH == 2, "stride-2 head / tail: 512-thread workgroups only");
  // WH = 2 (one workgroup per CU): the T exchange gets a buffer of its own beside the two
  // tiles, so it never aliases a tile and needs no barrier of its own
  constexpr bool SEPX = WH == 2;
  constexpr int TSTR = SEPX ? TILE : TB;
  // the head's input window: 17 rows x (9 even + 8 odd columns + 1 pad) pixels, after tile A
  // (the block input the head writes); it aliases tile B, the exchange and what follows
  constexpr int HWR = 17, HWC = 18, HWIN = HWR * HWC * PS;
  constexpr int SM0 = SEPX ? 2 * TILE + XCH : 2 * TB;
  constexpr int SMEM = HEAD && TILE + HWIN > SM0 ? TILE + HWIN : SM0;
  __shared__ __attribute__((aligned(16))) float smem[SMEM];
  __shared__ __attribute__((aligned(16))) float sbias[CH_MAX_LAYERS * C];
  __shared__ unsigned sh[2];
  const int tid = threadIdx.x;
  const int wv = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int xi = wv & 3, wh = wv >> 2;  // point row, output-channel part
  const int lane = tid & 63, li = lane & 15, lg = lane >> 4;
  const int H = a.H, W = a.W, R = a.rh * a.rw, nR = a.n * R;
  auto stamp = [&](int k) {
    if (a.tstamp && tid == 0) a.tstamp[(size_t)blockIdx.x * CH_TS + k] = __builtin_amdgcn_s_memrealtime();
  };
  auto stamp4 = [&](int k) {  // wave 4, the second wave on thread 0's SIMD (WH = 2)
    if (a.tstamp && tid == 256) a.tstamp[(size_t)blockIdx.x * CH_TS + k] = __builtin_amdgcn_s_memrealtime();
  };
  stamp(0);

  if (tid == 0) {
    sh[0] = a.dispatch_order == 2   ? chain_region(blockIdx.x, (unsigned)(a.rh * a.rw), (unsigned)a.n)
            : a.dispatch_order == 1 ? blockIdx.x
                                    : __hip_atomic_fetch_add(&a.ctl[0], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    sh[1] = __hip_atomic_load(&a.ctl[2], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  // every layer's bias, read by the epilogues from LDS
  for (int e = tid; e < a.nl * C; e += NTH) sbias[e] = a.layer[e / C].bias[e % C];
  __syncthreads();
  const int ticket = (int)sh[0];
  const unsigned epoch = sh[1] + 1u;  // this launch's flag value
  const int nimg = ticket / R, reg = ticket % R;
  const int ry = reg / a.rw, rx = reg % a.rw;
  const int oy0 = ry * 8, ox0 = rx * 8;
  const size_t g = (size_t)nimg * R + reg;
  constexpr int KH = HEAD ? 1 : 0;  // hand-off slot of chain layer l: KH + l

  // ---- weights of layer l, step s = 4 kc + nu, straight from L2, prefetched PF ahead:
  // raw buffer loads — the layer's descriptor in SGPRs, this lane's byte offset in one VGPR
  // (the same for every layer), the step as an immediate offset — instead of a 64-bit
  // address per load (54 v_lshl_add_u64 per layer; at f32 every VALU instruction costs
  // matrix-pipe time, §3 of DESIGN.md) ----
  constexpr int NSTEP = 4 * KC, PF = 3, NBW = 4 / WH;
  f32x4 av[PF + 1][NBW];
  const int wlane = ((xi * 64 * KC * C) + (lg * C + li) * 4) * 4;  // bytes
  auto wsrc = [&](int l) {
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(a.layer[l].wu), (short)0, 16 * KC * 16 * C * 4,
                                             0x00020000);
  };
  auto wglob = [&](const __amdgpu_buffer_rsrc_t& r, int s, int nb) -> f32x4 {
    const int kc = s >> 2, nu = s & 3;
    const u32x4 u =
        __builtin_amdgcn_raw_buffer_load_b128(r, wlane, ((nu * KC + kc) * 16 * C + (wh * NBW + nb) * 64) * 4, 0);
    return f32x4{__uint_as_float(u.x), __uint_as_float(u.y), __uint_as_float(u.z), __uint_as_float(u.w)};
  };

  // The first layer's tile is the res_block input when the chain starts a block, so it
  // goes to tile 0 (A) then, else to tile 1 (B): the block input always lives in A.  (A head
  // is only planned in front of a block: its output is the block input, tile A.)
  const bool first_block = a.nl > 1 && a.layer[1].res;
  float* src = HEAD || first_block ? smem : smem + TSTR;

  bool failed = false;
  // halo descriptors of this thread, the same for every hand-off: the LDS offset in the tile
  // and the byte offset of the neighbour's border record entry inside a hand-off buffer
  // (-1: outside the image, zero)
  constexpr int HK = (36 * 16 + NTH - 1) / NTH;
  int hlds[HK], hsrc[HK];
#pragma unroll
  for (int k = 0; k < HK; ++k) {
    const int e = k * NTH + tid;
    hlds[k] = hsrc[k] = -1;
    if (e < 36 * 16) {
      const int hp = e >> 4, q = e & 15;
      int hy, hx;
      if (hp < 10) hy = -1, hx = hp - 1;
      else if (hp < 20) hy = 8, hx = hp - 11;
      else if (hp < 28) hy = hp - 20, hx = -1;
      else hy = hp - 28, hx = 8;
      hlds[k] = tpix(hy + 1, hx + 1) + 4 * q;
      const int gy = oy0 + hy, gx = ox0 + hx;
      if (gy >= 0 && gy < H && gx >= 0 && gx < W) {
        const int nry = ry + (hy < 0 ? -1 : (hy > 7 ? 1 : 0)), nrx = rx + (hx < 0 ? -1 : (hx > 7 ? 1 : 0));
        const int ny = hy & 7, nx = hx & 7;  // pixel inside the neighbour region
        int side, idx;
        if (hy < 0) side = 1, idx = nx;
        else if (hy > 7) side = 0, idx = nx;
        else if (hx < 0) side = 3, idx = ny;
        else side = 2, idx = ny;
        const int gn = nimg * R + nry * a.rw + nrx;
        hsrc[k] = (gn * (4 * 8 * C) + (side * 8 + idx) * C + 4 * q) * 4;
      }
    }
  }
  const bool handoff_on = R > 1 && a.probe != 1;
  // this region's border record of hand-off k
  auto pub_rsrc = [&](int k) { return xrsrc(a.xbuf + ((size_t)k * nR + g) * (4 * 8 * C), 4 * 8 * C * 4); };
  // publish pixel (ly, lx) of the region's output (16-byte write-through stores into the 8 KB
  // record: side 0 / 1 = rows 0 / 7, side 2 / 3 = columns 0 / 7; corners go to two sides)
  auto publish = [&](const __amdgpu_buffer_rsrc_t& rpub, int ly, int lx, int co, f32x4 v) {
    if (ly == 0) st_sc1_16(rpub, ((0 * 8 + lx) * C + co) * 4, v);
    if (ly == 7) st_sc1_16(rpub, ((1 * 8 + lx) * C + co) * 4, v);
    if (lx == 0) st_sc1_16(rpub, ((2 * 8 + ly) * C + co) * 4, v);
    if (lx == 7) st_sc1_16(rpub, ((3 * 8 + ly) * C + co) * 4, v);
  };
  // hand-off k: (every storing thread drained its border stores and passed a barrier) raise
  // this region's flag, wait for the (up to 8) neighbours' flags, read the halo ring of `tile`
  // (rows 0 and 9, columns 0 and 9: 36 px x 16 quads) through the descriptors above
  auto handoff = [&](int k, float* tile, int ts) {
    if (handoff_on) {
      if (tid == 0) __hip_atomic_store(&a.flags[(size_t)k * nR + g], epoch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      stamp(ts + 3);
      if (a.probe == 0 && tid < 9 && tid != 4) {
        const int nry = ry + tid / 3 - 1, nrx = rx + tid % 3 - 1;
        if (nry >= 0 && nry < a.rh && nrx >= 0 && nrx < a.rw) {
          const unsigned* f = &a.flags[(size_t)k * nR + (size_t)nimg * R + nry * a.rw + nrx];
          unsigned it = 0;
          while (__hip_atomic_load(f, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != epoch) {
            if (++it > kSpinLimit) {
              failed = true;
              break;
            }
            __builtin_amdgcn_s_sleep(2);
          }
        }
      }
      __syncthreads();
      stamp(ts + 4);
      const __amdgpu_buffer_rsrc_t rlay = xrsrc(a.xbuf + (size_t)k * nR * (4 * 8 * C), (unsigned)nR * (4 * 8 * C * 4));
      f32x4 hv[HK];
#pragma unroll
      for (int q = 0; q < HK; ++q)
        hv[q] = hsrc[q] >= 0 && a.probe == 0 ? ld_sc1_16(rlay, hsrc[q]) : f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int q = 0; q < HK; ++q)
        if (hlds[q] >= 0) *reinterpret_cast<f32x4*>(&tile[hlds[q]]) = hv[q];
      __syncthreads();
      stamp(ts + 5);
    } else {
      // a single region per patch: the halo is all outside the image
      for (int e = tid; e < 36 * 16; e += NTH) {
        const int hp = e >> 4, q = e & 15;
        int hy, hx;
        if (hp < 10) hy = -1, hx = hp - 1;
        else if (hp < 20) hy = 8, hx = hp - 11;
        else if (hp < 28) hy = hp - 20, hx = -1;
        else hy = hp - 28, hx = 8;
        *reinterpret_cast<f32x4*>(&tile[tpix(hy + 1, hx + 1) + 4 * q]) = f32x4{0.f, 0.f, 0.f, 0.f};
      }
      __syncthreads();
    }
  };

  // ---- the stride-2 layers' implicit GEMM (HEAD / TAIL): conv3x3_kernel's weight packing and
  // step order; wave w owns 16 output pixels (rows 2 (w % 4), +1 of the region: lane li ->
  // row (li >> 3), column li % 8) x output-channel blocks 2 (w / 4), +1 ----
  const int dnb = wv & 3, dmb = (wv >> 2) * 2;
  const int dry = 2 * dnb + (li >> 3), drx = dcol(li & 7);  // this lane's pixel in the region
  auto dsrc = [&](const float* w) { return __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(w), (short)0, 9 * C * C * 4, 0x00020000); };
  auto dglob = [&](const __amdgpu_buffer_rsrc_t& r, int s, int m) -> f32x4 {
    const int tap = s / KC, kc = s % KC;  // step s: tap-major, then the 16-channel chunk
    const u32x4 u = __builtin_amdgcn_raw_buffer_load_b128(r, (lg * C + (dmb + m) * 16 + li) * 16,
                                                          ((tap * KC + kc) * 4 * C * 4) * 4, 0);
    return f32x4{__uint_as_float(u.x), __uint_as_float(u.y), __uint_as_float(u.z), __uint_as_float(u.w)};
  };

  if constexpr (HEAD) {
    // ---- the head: stage the input window of rows 2 oy0 - hpad + r, columns 2 ox0 - hpad + c
    // (r, c < 17; zero outside = SAME padding), columns split by parity ----
    float* const hw = smem + TILE;
    const __amdgpu_buffer_rsrc_t hws = dsrc(a.head.wu);
    constexpr int DPF = 2, DSTEP = 9 * KC;
    f32x4 dav[DPF + 1][2];
#pragma unroll
    for (int p = 0; p < DPF; ++p)
#pragma unroll
      for (int m = 0; m < 2; ++m) dav[p][m] = dglob(hws, p, m);
    // the epilogue's biases, loaded now (after the K loop their latency would be exposed)
    f32x4 hbias[2];
#pragma unroll
    for (int m = 0; m < 2; ++m) hbias[m] = *reinterpret_cast<const f32x4*>(a.head.bias + (dmb + m) * 16 + lg * 4);
    {
      constexpr int NCH = HWR * 17 * (C / 4);  // 16-byte chunks
      constexpr int NIT = (NCH + NTH - 1) / NTH;
      const int iy0 = 2 * oy0 - a.hpad, ix0 = 2 * ox0 - a.hpad;
      f32x4 tmp[NIT];
#pragma unroll
      for (int i = 0; i < NIT; ++i) {
        const int e = i * NTH + tid;
        tmp[i] = f32x4{0.f, 0.f, 0.f, 0.f};
        if (e < NCH) {
          const int c4 = e % 16, pe = e / 16, col = pe % 17, row = pe / 17;
          const int iy = iy0 + row, ix = ix0 + col;
          if (iy >= 0 && iy < a.hH && ix >= 0 && ix < a.hW)
            tmp[i] = *reinterpret_cast<const f32x4*>(a.head_in + ((size_t)(nimg * a.hH + iy) * a.hW + ix) * C + c4 * 4);
        }
      }
#pragma unroll
      for (int i = 0; i < NIT; ++i) {
        const int e = i * NTH + tid;
        if (e < NCH) {
          const int c4 = e % 16, pe = e / 16, col = pe % 17, row = pe / 17;
          // chunk ^ 8 on row pairs 2, 3 (mod 4): the K loop's 16-lane groups read rows 2 apart
          *reinterpret_cast<f32x4*>(&hw[(row * HWC + (col & 1) * 9 + (col >> 1)) * PS + (c4 ^ ((row & 2) << 2)) * 4]) =
              tmp[i];
        }
      }
    }
    __syncthreads();
    stamp(CH_HEAD_TS);
    f32x4 dacc[2] = {f32x4{0.f, 0.f, 0.f, 0.f}, f32x4{0.f, 0.f, 0.f, 0.f}};
    auto hload = [&](int s) -> f32x4 {
      const int tap = s / KC, kc = s % KC, ky = tap / 3, kx = tap % 3;
      const int row = 2 * dry + ky, pix = row * HWC + (kx & 1) * 9 + drx + (kx >> 1);
      return *reinterpret_cast<const f32x4*>(&hw[pix * PS + ((kc * 4 + lg) ^ ((row & 2) << 2)) * 4]);
    };
    f32x4 bq[2];
    bq[0] = hload(0);
#pragma unroll
    for (int s = 0; s < DSTEP; ++s) {
      if (s + DPF < DSTEP) {
#pragma unroll
        for (int m = 0; m < 2; ++m) dav[(s + DPF) % (DPF + 1)][m] = dglob(hws, s + DPF, m);
      }
      if (s + 1 < DSTEP) bq[(s + 1) & 1] = hload(s + 1);
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int t = 0; t < 4; ++t)
#pragma unroll
        for (int m = 0; m < 2; ++m) dacc[m] = mfma4(dav[s % (DPF + 1)][m][t], bq[s & 1][t], dacc[m]);
      __builtin_amdgcn_sched_barrier(0);
    }
    // the first chain layer's weights fly during the head's epilogue and hand-off
    {
      const __amdgpu_buffer_rsrc_t w0 = wsrc(0);
#pragma unroll
      for (int p = 0; p < PF; ++p)
#pragma unroll
        for (int nb = 0; nb < NBW; ++nb) av[p][nb] = wglob(w0, p, nb);
    }
    stamp(CH_HEAD_TS + 1);
    stamp4(CH_W4_HEAD);
    // + bias, ReLU (conv3x3_kernel's epilogue), into the block-input tile and the border record
    const __amdgpu_buffer_rsrc_t rpub = pub_rsrc(0);
    const bool in_img = oy0 + dry < H && ox0 + drx < W;
#pragma unroll
    for (int m = 0; m < 2; ++m) {
      const int co = (dmb + m) * 16 + lg * 4;
      const f32x4 bb = hbias[m];
      f32x4 v = dacc[m];
      v.x = __fadd_rn(v.x, bb.x);
      v.y = __fadd_rn(v.y, bb.y);
      v.z = __fadd_rn(v.z, bb.z);
      v.w = __fadd_rn(v.w, bb.w);
      if (a.head.act == ACT_RELU) {
        v.x = fmaxf(v.x, 0.f);
        v.y = fmaxf(v.y, 0.f);
        v.z = fmaxf(v.z, 0.f);
        v.w = fmaxf(v.w, 0.f);
      }
      if (!in_img) v = f32x4{0.f, 0.f, 0.f, 0.f};
      *reinterpret_cast<f32x4*>(&src[tpix(dry + 1, drx + 1) + co]) = v;
      if (handoff_on) publish(rpub, dry, drx, co, v);
    }
    if (handoff_on) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();  // (also: every wave is done reading the window the next tiles alias)
    stamp(CH_HEAD_TS + 2);
    handoff(0, src, CH_HEAD_TS);
  } else {
    {
      const __amdgpu_buffer_rsrc_t w0 = wsrc(0);
#pragma unroll
      for (int p = 0; p < PF; ++p)
#pragma unroll
        for (int nb = 0; nb < NBW; ++nb) av[p][nb] = wglob(w0, p, nb);
    }
    // ---- stage the first layer's input tile (zero outside the image = SAME padding) ----
    constexpr int NSTAGE = LR * 10 * (C / 4);  // 1600 16-byte chunks
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
    __syncthreads();
  }
  stamp(1);

  // B^T row xi from input rows iA, iB of each tile (conv3x3_wino_kernel's exact signs)
  const int iA = xi == 0 ? 0 : 1, iB = xi == 3 ? 3 : 2;
  const float sA = xi == 2 ? -1.f : 1.f, sB = (xi == 0 || xi == 3) ? -1.f : 1.f;
  // (sA, sB) = (+, -) rows 0 / 3, (+, +) row 1, (-, +) row 2
  const int sgn = __builtin_amdgcn_readfirstlane(sA < 0.f ? 2 : (sB > 0.f ? 1 : 0));
  const int ty_l = li / TTX, tx_l = li % TTX;
  const int offA = ((2 * ty_l + iA) * RP + tx_l) * PS + lg * 4;
  const int offB = ((2 * ty_l + iB) * RP + tx_l) * PS + lg * 4;
  // epilogue ownership: one (tile, channel quad) per thread and output row ay (WH = 2:
  // the threads tid and tid + 256 take the tile's rows 0 and 1)
  const int et = (tid & 255) >> 4, eq = epi_quad(tid);
  const int ay0 = WH == 1 ? 0 : tid >> 8;
  constexpr int nay = WH == 1 ? 2 : 1;
  const int ety = et / TTX, etx = et % TTX;

  for (int l = 0; l < a.nl; ++l) {
    const bool last = l == a.nl - 1;
    const bool res = a.layer[l].res != 0;
    const bool starts_block = !last && a.layer[l + 1].res != 0;
    float* const dst = src == smem ? smem + TSTR : smem;  // the other tile
    float* const xch = SEPX ? smem + 2 * TILE : starts_block ? dst : src;  // T exchange: never the block input
    float* const rsd = dst;                              // res layers: the block input tile
    const int ts = 2 + 6 * l;
    stamp(ts);
    const __amdgpu_buffer_rsrc_t wl = wsrc(l);

    // ---- K loop: conv3x3_wino_kernel's order ----
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
      // sA, sB = +-1: sA d0 + sB d1 is one rounded add / subtract (the products are exact),
      // so the three sign patterns are spelled out (wave-uniform branch): 4 instead of 8
      // VALU per 4-channel column
      if (sgn == 0) {
#pragma unroll
        for (int j = 0; j < 4; ++j) r[j] = psub(d[0][j], d[1][j]);
      } else if (sgn == 1) {
#pragma unroll
        for (int j = 0; j < 4; ++j) r[j] = d[0][j] + d[1][j];
      } else {
#pragma unroll
        for (int j = 0; j < 4; ++j) r[j] = psub(d[1][j], d[0][j]);
      }
      V[0] = psub(r[0], r[2]);
      V[1] = r[1] + r[2];
      V[2] = psub(r[2], r[1]);
      V[3] = psub(r[1], r[3]);
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
          for (int nb = 0; nb < NBW; ++nb) av[(s + PF) % (PF + 1)][nb] = wglob(wl, s + PF, nb);
        }
        // keep each weight load PF steps (48 MFMAs) ahead of its use: without the fence the
        // scheduler sinks the loads next to their consumers inside the chunk
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
    // the next layer's first weight steps fly during this layer's epilogue and hand-off
    if (!last) {
      const __amdgpu_buffer_rsrc_t wn = wsrc(l + 1);
#pragma unroll
      for (int p = 0; p < PF; ++p)
#pragma unroll
        for (int nb = 0; nb < NBW; ++nb) av[p][nb] = wglob(wn, p, nb);
    }

    stamp(ts + 1);
    stamp4(CH_W4_TS + l);
    // ---- T = M A over nu, exchanged through LDS ----
    if (!SEPX) __syncthreads();  // every wave is done reading src (xch may alias it)
#pragma unroll
    for (int nb = 0; nb < NBW; ++nb) {
      const f32x4 m0 = acc[0][nb], m1 = acc[1][nb], m2 = acc[2][nb], m3 = acc[3][nb];
      float* x = &xch[(xi * 2 * NT + li) * XS + xq(li, (wh * NBW + nb) * 4 + lg) * 4];
      *reinterpret_cast<f32x4*>(x) = (m0 + m1) + m2;
      *reinterpret_cast<f32x4*>(x + NT * XS) = psub(psub(m1, m2), m3);
    }
    __syncthreads();

    // ---- Y = A^T T for (tile et, quad eq), + bias, act, + residual ----
    // row ay of Y from T rows ay..ay+2: (T0 + T1) + T2, or (T1 - T2) - T3
    const int co = 4 * eq;
    const f32x4 bb = *reinterpret_cast<const f32x4*>(&sbias[l * C + co]);
    const bool relu = a.layer[l].act == ACT_RELU;
    f32x4 y[2][2];  // [k][b], output row ay0 + k
#pragma unroll
    for (int k = 0; k < nay; ++k) {
      const int ay = ay0 + k;
#pragma unroll
      for (int b = 0; b < 2; ++b) {
        f32x4 t[3];
#pragma unroll
        for (int j = 0; j < 3; ++j)
          t[j] = *reinterpret_cast<const f32x4*>(&xch[(((ay + j) * 2 + b) * NT + et) * XS + xq(et, eq) * 4]);
        f32x4 v = ay == 0 ? (t[0] + t[1]) + t[2] : psub(psub(t[0], t[1]), t[2]);
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
        y[k][b] = v;
      }
    }

    if (last && !TAIL) {  // ---- the chain's output: global f32 or the quantiser ----
#pragma unroll
      for (int k = 0; k < nay; ++k)
#pragma unroll
        for (int b = 0; b < 2; ++b) {
          const int oy = oy0 + 2 * ety + ay0 + k, ox = ox0 + 2 * etx + b;
          if (oy >= H || ox >= W) continue;
          const size_t o = ((size_t)(nimg * H + oy) * W + ox) * C + co;
          const f32x4 v = y[k][b];
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

    // ---- into the next layer's (TAIL: the tail's) tile, zero outside the image; a border
    // pixel is published from the same registers ----
    const __amdgpu_buffer_rsrc_t rpub = pub_rsrc(KH + l);
    if (xch == dst) __syncthreads();  // every thread has read its T from dst's space
#pragma unroll
    for (int k = 0; k < nay; ++k)
#pragma unroll
      for (int b = 0; b < 2; ++b) {
        const int ly = 2 * ety + ay0 + k, lx = 2 * etx + b;
        const bool in_img = oy0 + ly < H && ox0 + lx < W;
        const f32x4 v = in_img ? y[k][b] : f32x4{0.f, 0.f, 0.f, 0.f};
        *reinterpret_cast<f32x4*>(&dst[tpix(ly + 1, lx + 1) + co]) = v;
        if (handoff_on) publish(rpub, ly, lx, co, v);
      }
    if (handoff_on) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    stamp(ts + 2);
    handoff(KH + l, dst, ts);
    src = dst;
  }

  if constexpr (TAIL) {
    // ---- the tail: conv3x3_kernel<MODE_T2> on the run's last output (src, halo filled):
    // input position (dry, drx) of the region feeds output phase ph = 2 (ky == 1) + (kx == 1)
    // through input offset (-(ky == 2), -(kx == 2)) ----
    stamp(CH_TAIL_TS);
    const __amdgpu_buffer_rsrc_t tws = dsrc(a.tail.wu);
    constexpr int DPF = 2, DSTEP = 9 * KC;
    f32x4 dav[DPF + 1][2];
#pragma unroll
    for (int p = 0; p < DPF; ++p)
#pragma unroll
      for (int m = 0; m < 2; ++m) dav[p][m] = dglob(tws, p, m);
    f32x4 tbias[2];  // loaded before the K loop (latency hidden behind it)
#pragma unroll
    for (int m = 0; m < 2; ++m) tbias[m] = *reinterpret_cast<const f32x4*>(a.tail.bias + (dmb + m) * 16 + lg * 4);
    f32x4 tacc[4][2];
#pragma unroll
    for (int p = 0; p < 4; ++p)
#pragma unroll
      for (int m = 0; m < 2; ++m) tacc[p][m] = f32x4{0.f, 0.f, 0.f, 0.f};
    auto tload = [&](int s) -> f32x4 {
      const int tap = s / KC, kc = s % KC, ky = tap / 3, kx = tap % 3;
      return *reinterpret_cast<const f32x4*>(&src[tpix(dry + 1 - (ky == 2), drx + 1 - (kx == 2)) + kc * 16 + lg * 4]);
    };
    f32x4 bq[2];
    bq[0] = tload(0);
#pragma unroll
    for (int s = 0; s < DSTEP; ++s) {
      const int tap = s / KC, ky = tap / 3, kx = tap % 3;
      const int ph = (ky == 1 ? 2 : 0) + (kx == 1 ? 1 : 0);
      if (s + DPF < DSTEP) {
#pragma unroll
        for (int m = 0; m < 2; ++m) dav[(s + DPF) % (DPF + 1)][m] = dglob(tws, s + DPF, m);
      }
      if (s + 1 < DSTEP) bq[(s + 1) & 1] = tload(s + 1);
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int t = 0; t < 4; ++t)
#pragma unroll
        for (int m = 0; m < 2; ++m) tacc[ph][m] = mfma4(dav[s % (DPF + 1)][m][t], bq[s & 1][t], tacc[ph][m]);
      __builtin_amdgcn_sched_barrier(0);
    }
    stamp(CH_TAIL_TS + 1);
    stamp4(CH_W4_TAIL);
    if constexpr (TAIL2) {
      // ---- decode_3's outputs stay on chip: they are decode_2's input tile T3 (17 x 17
      // positions, row / column 0 = the outputs just above / left of the region's 16 x 16).
      // Those halo outputs are recomputed here from the run's halo ring, in conv3x3_kernel's
      // order for them (as dec10 does for decode_1): wave w, output-channel block w % 4,
      // pass w / 4 — 0: the row above (input row -1, columns -1..7: phase (1,0) from taps 3
      // then 5, phase (1,1) from tap 4), 1: the column left (input column -1, rows 0..7: phase
      // (0,1) from taps 1 then 7, phase (1,1) from tap 4) ----
      const int hm = wv & 3, hrow = (wv >> 2) == 0;
      f32x4 hacc[2] = {f32x4{0.f, 0.f, 0.f, 0.f}, f32x4{0.f, 0.f, 0.f, 0.f}};
      {
        const __amdgpu_buffer_rsrc_t r3 = dsrc(a.tail.wu);
        const int lq = li < 9 ? li : 8;  // row pass: input column lq - 1; column pass: input row li (li < 8)
#pragma unroll
        for (int ti = 0; ti < 3; ++ti) {
          const int tap = hrow ? 3 + ti : 1 + 3 * ti;  // ascending
          const int ky = tap / 3, kx = tap % 3;
          const int q = ti == 1 ? 1 : 0;  // the middle tap is tap 4 in both passes
          int pix;
          if (hrow) pix = tpix(0, max(lq - (kx == 2), 0));                       // input (-1, lq - 1 - (kx == 2))
          else pix = tpix(min(li, 7) + 1 - (ky == 2), 0);                        // input (li - (ky == 2), -1)
#pragma unroll
          for (int kc = 0; kc < KC; ++kc) {
            const f32x4 b = *reinterpret_cast<const f32x4*>(&src[pix + kc * 16 + lg * 4]);
            const u32x4 u = __builtin_amdgcn_raw_buffer_load_b128(r3, (lg * C + hm * 16 + li) * 16,
                                                                  ((tap * KC + kc) * 4 * C * 4) * 4, 0);
            const f32x4 w = f32x4{__uint_as_float(u.x), __uint_as_float(u.y), __uint_as_float(u.z), __uint_as_float(u.w)};
#pragma unroll
            for (int t = 0; t < 4; ++t) hacc[q] = mfma4(w[t], b[t], hacc[q]);
          }
        }
      }
      const f32x4 hb = *reinterpret_cast<const f32x4*>(a.tail.bias + hm * 16 + lg * 4);
      __syncthreads();  // every wave is done reading the run's tiles: T3 aliases them
      float* const t3 = smem;
      constexpr int T3C = 17, PS3 = PS;
      // 16-byte chunk ch of T3 pixel (r, c) (chunk ^ 1 on columns 4-7 mod 8: decode_3's stride-2
      // output writes were 4-way, now 2-way; decode_2's reads stay conflict-free)
      auto t3a = [&](int r, int c, int ch) { return (r * T3C + c) * PS3 + (ch ^ ((c >> 2) & 1)) * 4; };
      auto epi = [&](f32x4 v, const f32x4& bb, bool valid) {
        v.x = __fadd_rn(v.x, bb.x);
        v.y = __fadd_rn(v.y, bb.y);
        v.z = __fadd_rn(v.z, bb.z);
        v.w = __fadd_rn(v.w, bb.w);
        if (a.tail.act == ACT_RELU) {
          v.x = fmaxf(v.x, 0.f);
          v.y = fmaxf(v.y, 0.f);
          v.z = fmaxf(v.z, 0.f);
          v.w = fmaxf(v.w, 0.f);
        }
        return valid ? v : f32x4{0.f, 0.f, 0.f, 0.f};
      };
      {  // the interior 16 x 16 (zero beyond the image: decode_2's padding)
        const bool valid = oy0 + dry < H && ox0 + drx < W;
#pragma unroll
        for (int p = 0; p < 4; ++p) {
          const int oy = 2 * dry + (p >> 1), ox = 2 * drx + (p & 1);
#pragma unroll
          for (int m = 0; m < 2; ++m)
            *reinterpret_cast<f32x4*>(&t3[t3a(1 + oy, 1 + ox, (dmb + m) * 4 + lg)]) = epi(tacc[p][m], tbias[m], valid);
        }
      }
      {  // the halo row / column (zero above / left of the image)
#pragma unroll
        for (int q = 0; q < 2; ++q) {
          int r, c;
          bool use, valid;
          if (hrow) {  // input column li - 1: phase (1, q) -> output (-1, 2 (li - 1) + q)
            const int ox = 2 * (li - 1) + q;
            r = 0, c = 1 + ox;
            use = li < 9 && ox >= -1;
            valid = oy0 > 0 && ox0 + (ox >> 1) >= 0 && ox0 + (ox >> 1) < W;
          } else {  // input row li: phase (q, 1) -> output (2 li + q, -1)
            const int oy = 2 * li + q;
            r = 1 + oy, c = 0;
            use = li < 8;
            valid = ox0 > 0 && oy0 + li < H;
          }
          if (use) *reinterpret_cast<f32x4*>(&t3[t3a(r, c, hm * 4 + lg)]) = epi(hacc[q], hb, valid);
        }
      }
      __syncthreads();
      stamp(CH_TAIL_TS + 2);
      if constexpr (TAIL2_PW) {
        // ---- decode_2 in the polyphase Winograd form (s2_form 1), conv3x3_pwino_kernel<MODE_T2,
        // 64, 32>'s arithmetic bit for bit (the same pw_* transforms, every point summed over the
        // chunks and t in the same order, the same output transform and epilogue): tile (ty, tx)
        // = decode_2 input positions 2ty .. 2ty + 1 x 2tx .. 2tx + 1 of the region's 16 x 16,
        // reading T3 positions (2ty + r, 2tx + j), r, j = 0..2 (row / column 0: the halo); wave w
        // owns output-channel block w & 1 and tile rows 2 (w >> 1) .. + 1 (lane li: tile
        // (2 (w >> 1) + li / 8, li % 8)), all 25 points: 400 MFMAs per wave instead of 576 ----
        constexpr int C2 = 32, PPF = 5, PRING = PPF + 5, PSTEP = 25 * KC;
        const int pcb = wv & 1, pty = 2 * (wv >> 1) + (li >> 3), ptx = li & 7;
        const __amdgpu_buffer_rsrc_t w2s =
            __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(a.tail2.wu), (short)0, 25 * C * C2 * 4, 0x00020000);
        auto pwglob = [&](int s) -> f32x4 {  // step s = 25 kc + 5 xi + nu (pack_pwino's layout)
          const int kc = s / 25, p = s % 25;
          const u32x4 u = __builtin_amdgcn_raw_buffer_load_b128(w2s, (lg * C2 + pcb * 16 + li) * 16,
                                                                ((p * KC + kc) * 4 * C2 * 4) * 4, 0);
          return f32x4{__uint_as_float(u.x), __uint_as_float(u.y), __uint_as_float(u.z), __uint_as_float(u.w)};
        };
        f32x4 pav[PRING];
#pragma unroll
        for (int p = 0; p < PPF; ++p) pav[p] = pwglob(p);
        const f32x4 pb = *reinterpret_cast<const f32x4*>(a.tail2.bias + pcb * 16 + lg * 4);
        f32x4 pacc[25];
#pragma unroll
        for (int p = 0; p < 25; ++p) pacc[p] = f32x4{0.f, 0.f, 0.f, 0.f};
        f32x4 db[2][3][3];
        auto ldchunk = [&](int kc, f32x4 (&dst)[3][3]) {
#pragma unroll
          for (int r = 0; r < 3; ++r)
#pragma unroll
            for (int j = 0; j < 3; ++j)
              dst[r][j] = *reinterpret_cast<const f32x4*>(&t3[t3a(2 * pty + r, 2 * ptx + j, kc * 4 + lg)]);
        };
        ldchunk(0, db[0]);
#pragma unroll
        for (int kc = 0; kc < KC; ++kc) {
          if (kc + 1 < KC) ldchunk(kc + 1, db[(kc + 1) & 1]);
          __builtin_amdgcn_sched_barrier(0);
          const f32x4(&d)[3][3] = db[kc & 1];
#pragma unroll
          for (int xi = 0; xi < 5; ++xi) {
            f32x4 r[3], V[5];
#pragma unroll
            for (int j = 0; j < 3; ++j) r[j] = pw_row_t2(xi, d[0][j], d[1][j], d[2][j]);
            pw_bt<MODE_T2>(r, V);
            // U one point row ahead; t outer, nu inner (no MFMA waits for the one before it)
            const int s0 = 25 * kc + 5 * xi;
            f32x4 u[5];
#pragma unroll
            for (int nu = 0; nu < 5; ++nu) u[nu] = pav[(s0 + nu) % PRING];
#pragma unroll
            for (int nu = 0; nu < 5; ++nu)
              if (s0 + nu + PPF < PSTEP) pav[(s0 + nu + PPF) % PRING] = pwglob(s0 + nu + PPF);
#pragma unroll
            for (int tt = 0; tt < 4; ++tt)
#pragma unroll
              for (int nu = 0; nu < 5; ++nu) pacc[5 * xi + nu] = mfma4(u[nu][tt], V[nu][tt], pacc[5 * xi + nu]);
          }
          __builtin_amdgcn_sched_barrier(0);
        }
        stamp(CH_TAIL_TS + 3);
        stamp4(CH_W4_TAIL + 1);
        // Y = A^T M A, + bias, act, 16-byte stores of the tile's 4 x 4 outputs
        f32x4 T[5][4];
#pragma unroll
        for (int xi = 0; xi < 5; ++xi) {
          f32x4 m[5];
#pragma unroll
          for (int nu = 0; nu < 5; ++nu) m[nu] = pacc[5 * xi + nu];
          pw_at<MODE_T2>(m, T[xi]);
        }
        const int Ho2 = 4 * H, Wo2 = 4 * W;
        const int py0 = 4 * oy0 + 4 * pty, px0 = 4 * ox0 + 4 * ptx;
#pragma unroll
        for (int b = 0; b < 4; ++b) {
          f32x4 m[5], y[4];
#pragma unroll
          for (int xi = 0; xi < 5; ++xi) m[xi] = T[xi][b];
          pw_at<MODE_T2>(m, y);
#pragma unroll
          for (int ay = 0; ay < 4; ++ay) {
            const int oy = py0 + ay, ox = px0 + b;
            if (oy >= Ho2 || ox >= Wo2) continue;
            f32x4 v = y[ay];
            v.x = __fadd_rn(v.x, pb.x);
            v.y = __fadd_rn(v.y, pb.y);
            v.z = __fadd_rn(v.z, pb.z);
            v.w = __fadd_rn(v.w, pb.w);
            if (a.tail2.act == ACT_RELU) {
              v.x = fmaxf(v.x, 0.f);
              v.y = fmaxf(v.y, 0.f);
              v.z = fmaxf(v.z, 0.f);
              v.w = fmaxf(v.w, 0.f);
            }
            *reinterpret_cast<f32x4*>(a.tail2_out + ((size_t)(nimg * Ho2 + oy) * Wo2 + ox) * C2 + pcb * 16 + lg * 4) = v;
          }
        }
        stamp(CH_TAIL_TS + 4);
        stamp4(CH_W4_TAIL + 2);
      } else {
      // ---- decode_2: conv3x3_kernel<MODE_T2, 64, 32> on T3; wave w owns input rows 2w, 2w + 1
      // (16 positions each) x both 16-channel output blocks x the four phases ----
      constexpr int C2 = 32;
      const __amdgpu_buffer_rsrc_t w2s =
          __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(a.tail2.wu), (short)0, 9 * C * C2 * 4, 0x00020000);
      auto d2glob = [&](int s, int m) -> f32x4 {
        const int tap = s / KC, kc = s % KC;
        const u32x4 u = __builtin_amdgcn_raw_buffer_load_b128(w2s, (lg * C2 + m * 16 + li) * 16,
                                                              ((tap * KC + kc) * 4 * C2 * 4) * 4, 0);
        return f32x4{__uint_as_float(u.x), __uint_as_float(u.y), __uint_as_float(u.z), __uint_as_float(u.w)};
      };
      f32x4 b2[2];
#pragma unroll
      for (int m = 0; m < 2; ++m) b2[m] = *reinterpret_cast<const f32x4*>(a.tail2.bias + m * 16 + lg * 4);
      constexpr int EPF = CH_D2_PF;
      f32x4 e2[EPF + 1][2];
#pragma unroll
      for (int p = 0; p < EPF; ++p)
#pragma unroll
        for (int m = 0; m < 2; ++m) e2[p][m] = d2glob(p, m);
      f32x4 acc2[4][2][2];  // [phase][row of the wave][channel block]
#pragma unroll
      for (int p = 0; p < 4; ++p)
#pragma unroll
        for (int j = 0; j < 2; ++j)
#pragma unroll
          for (int m = 0; m < 2; ++m) acc2[p][j][m] = f32x4{0.f, 0.f, 0.f, 0.f};
      auto load2 = [&](int s, f32x4 (&dst2)[2]) {
        const int tap = s / KC, kc = s % KC, ky = tap / 3, kx = tap % 3;
#pragma unroll
        for (int j = 0; j < 2; ++j)
          dst2[j] = *reinterpret_cast<const f32x4*>(&t3[t3a(1 + 2 * wv + j - (ky == 2), 1 + li - (kx == 2), kc * 4 + lg)]);
      };
      // + bias, act; decode_2's output [n, 4H, 4W, 32], 16-byte stores of phase p
      const int H3 = 2 * H, W3 = 2 * W, Ho2 = 4 * H, Wo2 = 4 * W;
      auto store2 = [&](int p0, int p1) {  // phases p0 .. p1 - 1
#pragma unroll
        for (int j = 0; j < 2; ++j) {
          const int gy = 2 * oy0 + 2 * wv + j, gx = 2 * ox0 + li;  // decode_2 input position
          if (gy >= H3 || gx >= W3) continue;
#pragma unroll
          for (int p = p0; p < p1; ++p) {
          const int oy = 2 * gy + (p >> 1), ox = 2 * gx + (p & 1);
#pragma unroll
          for (int m = 0; m < 2; ++m) {
            f32x4 v = acc2[p][j][m];
            const f32x4 bb = b2[m];
            v.x = __fadd_rn(v.x, bb.x);
            v.y = __fadd_rn(v.y, bb.y);
            v.z = __fadd_rn(v.z, bb.z);
            v.w = __fadd_rn(v.w, bb.w);
            if (a.tail2.act == ACT_RELU) {
              v.x = fmaxf(v.x, 0.f);
              v.y = fmaxf(v.y, 0.f);
              v.z = fmaxf(v.z, 0.f);
              v.w = fmaxf(v.w, 0.f);
            }
            *reinterpret_cast<f32x4*>(a.tail2_out + ((size_t)(nimg * Ho2 + oy) * Wo2 + ox) * C2 + m * 16 + lg * 4) = v;
          }
          }
        }
      };
      f32x4 bq2[2][2];
      load2(0, bq2[0]);
#pragma unroll
      for (int s = 0; s < DSTEP; ++s) {
        const int tap = s / KC, ky = tap / 3, kx = tap % 3;
        const int ph = (ky == 1 ? 2 : 0) + (kx == 1 ? 1 : 0);
        if (s + EPF < DSTEP) {
#pragma unroll
          for (int m = 0; m < 2; ++m) e2[(s + EPF) % (EPF + 1)][m] = d2glob(s + EPF, m);
        }
        if (s + 1 < DSTEP) load2(s + 1, bq2[(s + 1) & 1]);
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int t = 0; t < 4; ++t)
#pragma unroll
          for (int j = 0; j < 2; ++j)
#pragma unroll
            for (int m = 0; m < 2; ++m)
              acc2[ph][j][m] = mfma4(e2[s % (EPF + 1)][m][t], bq2[s & 1][j][t], acc2[ph][j][m]);
        __builtin_amdgcn_sched_barrier(0);
        if constexpr (CH_D2_EARLY != 0) {
          // a phase's last tap: 3 after tap 4, 2 after tap 5, 1 after tap 7 (the stores of the
          // finished phases go out under the remaining taps' MFMAs; every output's sum is unchanged)
          if (s == 4 * KC + KC - 1) store2(3, 4);
          if (s == 5 * KC + KC - 1) store2(2, 3);
          if (s == 7 * KC + KC - 1) store2(1, 2);
          __builtin_amdgcn_sched_barrier(0);
        }
      }
      stamp(CH_TAIL_TS + 3);
      stamp4(CH_W4_TAIL + 1);
      store2(0, CH_D2_EARLY != 0 ? 1 : 4);
      stamp(CH_TAIL_TS + 4);
      stamp4(CH_W4_TAIL + 2);
      }
    } else {
    // + bias, act (conv3x3_kernel's epilogue), 16-byte f32 stores of the 16x16 output tile
    if (oy0 + dry < H && ox0 + drx < W) {
      const int Ho = 2 * H, Wo = 2 * W;
#pragma unroll
      for (int p = 0; p < 4; ++p) {
        const int oy = 2 * (oy0 + dry) + (p >> 1), ox = 2 * (ox0 + drx) + (p & 1);
#pragma unroll
        for (int m = 0; m < 2; ++m) {
          const int co = (dmb + m) * 16 + lg * 4;
          const f32x4 bb = tbias[m];
          f32x4 v = tacc[p][m];
          v.x = __fadd_rn(v.x, bb.x);
          v.y = __fadd_rn(v.y, bb.y);
          v.z = __fadd_rn(v.z, bb.z);
          v.w = __fadd_rn(v.w, bb.w);
          if (a.tail.act == ACT_RELU) {
            v.x = fmaxf(v.x, 0.f);
            v.y = fmaxf(v.y, 0.f);
            v.z = fmaxf(v.z, 0.f);
            v.w = fmaxf(v.w, 0.f);
          }
          *reinterpret_cast<f32x4*>(a.tail_out + ((size_t)(nimg * Ho + oy) * Wo + ox) * C + co) = v;
        }
      }
    }
    stamp(CH_TAIL_TS + 2);
    }
  }

  // ---- the last workgroup to finish resets the ticket and advances the epoch ----
  if (failed) __hip_atomic_store(&a.ctl[3], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  __syncthreads();
  stamp(CH_END_TS);
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
