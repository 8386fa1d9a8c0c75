// image_ops.hip — device-side glue around the convolution stacks for whole images
// (BASELINE config 5: full-resolution images tiled into patches, decoded, stitched and
// post-filtered on the GPU without a host round trip), plus the symbol histogram of
// get_encoded_distribution.py.  All of it is byte/word movement: HBM-bound, one pass,
// consecutive threads touch consecutive output bytes/words (coalesced stores).
//
//   tile_reflect_kernel   utils.crop_image_input_patches (utils/utils.py:96-133):
//                         np.pad(..., 'reflect') bottom/right to a multiple of P, then
//                         row-major PxP patches; the padded image never exists.
//   stitch_kernel         utils.concat_patches (utils/utils.py:136-167): row-major
//                         concatenation cropped to HxW.
//   window_copy_kernel    rmbe_height / rmbe_width (submit/2/rmbe/rmbe.py:70-111):
//                         gather the 128x128 windows of one pass / write them back.
//   round_u8_kernel       np.around(x).astype(np.uint8) (submit/2/decoder.py:176).
//   histogram_kernel      np.histogram(symbols, range(Q + 1)) (get_encoded_distribution.py:113-126).
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <algorithm>

#include "tic_kernels.h"

namespace tic {

// numpy 'reflect' (edge pixel not repeated) for any pad length: the padded axis is the
// periodic extension with period 2(n-1) of x[0..n-1], x[n-2..1].
__device__ __forceinline__ int reflect_index(int i, int n) {
  if (n == 1) return 0;
  const int period = 2 * (n - 1);
  const int m = i % period;
  return m < n ? m : period - m;
}

// One thread per 4 output bytes of the patch batch [hn*wn, P, P, 3] (P*3 % 4 == 0).
__global__ void __launch_bounds__(256) tile_reflect_kernel(const uint8_t* __restrict__ img, int H, int W, int P,
                                                           int wn, size_t nwords, uint32_t* __restrict__ out) {
  const size_t row_bytes = (size_t)P * 3;
  const size_t patch_bytes = row_bytes * P;
  for (size_t w = blockIdx.x * (size_t)256 + threadIdx.x; w < nwords; w += (size_t)gridDim.x * 256) {
    const size_t b = w * 4;
    const int p = (int)(b / patch_bytes);
    const size_t rem = b - (size_t)p * patch_bytes;
    const int y = (int)(rem / row_bytes);
    const int xb = (int)(rem - (size_t)y * row_bytes);
    const int gy = reflect_index((p / wn) * P + y, H);
    const uint8_t* src_row = img + (size_t)gy * W * 3;
    const int gx0 = (p % wn) * P;
    uint32_t v = 0;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const int bx = xb + k;
      const int x = bx / 3, c = bx - 3 * (bx / 3);
      v |= (uint32_t)src_row[(size_t)reflect_index(gx0 + x, W) * 3 + c] << (8 * k);
    }
    out[w] = v;
  }
}

// One thread per output float of the cropped image [H, W, 3].
__global__ void __launch_bounds__(256) stitch_kernel(const float* __restrict__ patches, int H, int W, int P, int wn,
                                                     float* __restrict__ img) {
  const size_t total = (size_t)H * W * 3;
  for (size_t e = blockIdx.x * (size_t)256 + threadIdx.x; e < total; e += (size_t)gridDim.x * 256) {
    const size_t pix = e / 3;
    const int c = (int)(e - pix * 3);
    const int y = (int)(pix / W), x = (int)(pix - (size_t)y * W);
    const int p = (y / P) * wn + x / P;
    img[e] = patches[(((size_t)p * P + y % P) * P + x % P) * 3 + c];
  }
}

// Windows [hn*wn, S, S, 3] <-> image [H, W, 3] at (r0 + i*S, c0 + j*S).
// to_windows: gather (image -> windows); else scatter (windows -> image, in place).
__global__ void __launch_bounds__(256) window_copy_kernel(float* __restrict__ img, int W, int r0, int c0, int S,
                                                          int wn, size_t total, float* __restrict__ win,
                                                          int to_windows) {
  const size_t row = (size_t)S * 3, wsz = row * S;
  for (size_t e = blockIdx.x * (size_t)256 + threadIdx.x; e < total; e += (size_t)gridDim.x * 256) {
    const int p = (int)(e / wsz);
    const size_t rem = e - (size_t)p * wsz;
    const int y = (int)(rem / row);
    const int xc = (int)(rem - (size_t)y * row);
    const size_t o = ((size_t)(r0 + (p / wn) * S + y) * W + c0 + (p % wn) * S) * 3 + xc;
    if (to_windows) win[e] = img[o];
    else img[o] = win[e];
  }
}

__global__ void __launch_bounds__(256) round_u8_kernel(const float* __restrict__ in, size_t n,
                                                       uint8_t* __restrict__ out) {
  for (size_t e = blockIdx.x * (size_t)256 + threadIdx.x; e < n; e += (size_t)gridDim.x * 256) {
    const float v = fminf(fmaxf(rintf(in[e]), 0.f), 255.f);  // rintf: round half to even (np.around)
    out[e] = (uint8_t)v;
  }
}

// Per-workgroup LDS histogram of 4-symbol words, then one 64-bit atomic per used bin.
// np.histogram semantics for bins 0..Q: v < Q -> bin v, v == Q -> bin Q-1 (last bin is
// closed), anything else ignored.
__global__ void __launch_bounds__(256) histogram_kernel(const uint8_t* __restrict__ sym, size_t n, int Q,
                                                        unsigned long long* __restrict__ counts) {
  __shared__ uint32_t bins[256];
  bins[threadIdx.x] = 0;
  __syncthreads();
  auto put = [&](uint32_t v) {
    if (v < (uint32_t)Q) atomicAdd(&bins[v], 1u);
    else if (v == (uint32_t)Q) atomicAdd(&bins[Q - 1], 1u);
  };
  const size_t nw = n / 4;
  const uint32_t* w32 = reinterpret_cast<const uint32_t*>(sym);
  for (size_t w = blockIdx.x * (size_t)256 + threadIdx.x; w < nw; w += (size_t)gridDim.x * 256) {
    const uint32_t v = w32[w];
    put(v & 0xff);
    put((v >> 8) & 0xff);
    put((v >> 16) & 0xff);
    put(v >> 24);
  }
  if (blockIdx.x == 0 && threadIdx.x < n - nw * 4) put(sym[nw * 4 + threadIdx.x]);
  __syncthreads();
  if (threadIdx.x < (unsigned)Q && bins[threadIdx.x])
    atomicAdd(&counts[threadIdx.x], (unsigned long long)bins[threadIdx.x]);
}

// Exact sum of squared differences of two uint8 arrays (integer, so the dataset PSNR of
// processing_utils/evaluate.py:10-32 — sum(SSE) / sum(dims) — is order-independent).
__global__ void __launch_bounds__(256) sse_u8_kernel(const uint8_t* __restrict__ a, const uint8_t* __restrict__ b,
                                                     size_t n, unsigned long long* __restrict__ acc) {
  unsigned long long s = 0;
  const size_t nw = n / 4;
  const uint32_t* a32 = reinterpret_cast<const uint32_t*>(a);
  const uint32_t* b32 = reinterpret_cast<const uint32_t*>(b);
  for (size_t w = blockIdx.x * (size_t)256 + threadIdx.x; w < nw; w += (size_t)gridDim.x * 256) {
    const uint32_t x = a32[w], y = b32[w];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const int d = (int)((x >> (8 * k)) & 0xff) - (int)((y >> (8 * k)) & 0xff);
      s += (unsigned long long)(d * d);
    }
  }
  if (blockIdx.x == 0 && threadIdx.x < n - nw * 4) {
    const int d = (int)a[nw * 4 + threadIdx.x] - (int)b[nw * 4 + threadIdx.x];
    s += (unsigned long long)(d * d);
  }
  // wavefront reduction (64 lanes), then across the 4 waves in LDS: one atomic per
  // workgroup (the grid is capped at 2 workgroups per CU, so at most 512 atomics meet)
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) s += __shfl_down(s, off, 64);
  __shared__ unsigned long long part[4];
  if ((threadIdx.x & 63) == 0) part[threadIdx.x >> 6] = s;
  __syncthreads();
  if (threadIdx.x == 0) {
    const unsigned long long t = part[0] + part[1] + part[2] + part[3];
    if (t) atomicAdd(acc, t);
  }
}

namespace {
unsigned grid_for(size_t items, int num_cus, int per_cu = 16) {
  const size_t want = (items + 255) / 256;
  const size_t cap = (size_t)num_cus * per_cu;  // grid-stride beyond per_cu workgroups per CU
  return (unsigned)std::max<size_t>(1, std::min(want, cap));
}
}  // namespace

void launch_tile_reflect(const uint8_t* img, int H, int W, int P, int hn, int wn, uint8_t* out, int num_cus,
                         hipStream_t s) {
  const size_t nwords = (size_t)hn * wn * P * P * 3 / 4;
  hipLaunchKernelGGL(tile_reflect_kernel, dim3(grid_for(nwords, num_cus)), dim3(256), 0, s, img, H, W, P, wn, nwords,
                     reinterpret_cast<uint32_t*>(out));
}

void launch_stitch(const float* patches, int H, int W, int P, int wn, float* img, int num_cus, hipStream_t s) {
  const size_t total = (size_t)H * W * 3;
  hipLaunchKernelGGL(stitch_kernel, dim3(grid_for(total, num_cus)), dim3(256), 0, s, patches, H, W, P, wn, img);
}

void launch_window_copy(float* img, int W, int r0, int c0, int S, int hn, int wn, float* win, bool to_windows,
                        int num_cus, hipStream_t s) {
  const size_t total = (size_t)hn * wn * S * S * 3;
  hipLaunchKernelGGL(window_copy_kernel, dim3(grid_for(total, num_cus)), dim3(256), 0, s, img, W, r0, c0, S, wn, total,
                     win, to_windows ? 1 : 0);
}

void launch_round_u8(const float* in, size_t n, uint8_t* out, int num_cus, hipStream_t s) {
  hipLaunchKernelGGL(round_u8_kernel, dim3(grid_for(n, num_cus)), dim3(256), 0, s, in, n, out);
}

void launch_histogram(const uint8_t* sym, size_t n, int Q, unsigned long long* counts, int num_cus, hipStream_t s) {
  hipLaunchKernelGGL(histogram_kernel, dim3(grid_for(n / 4 + 1, num_cus, 2)), dim3(256), 0, s, sym, n, Q, counts);
}

void launch_sse_u8(const uint8_t* a, const uint8_t* b, size_t n, unsigned long long* acc, int num_cus,
                   hipStream_t s) {
  hipLaunchKernelGGL(sse_u8_kernel, dim3(grid_for(n / 4 + 1, num_cus, 2)), dim3(256), 0, s, a, b, n, acc);
}

}  // namespace tic
