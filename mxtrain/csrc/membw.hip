// HBM roofline probe: what this MI355X delivers to a streaming kernel, per access mix.
// The memory-bound kernels of the training step (AdamW 28 B/element, LayerNorm, the
// gradient sum-of-squares) are judged against THESE numbers, not the 8 TB/s datasheet.
//
//   mx_membw(R, W, nt, src[], dst[], n_float4_per_stream, blocks, stream)
//     every thread moves float4s: reads R streams, writes W streams (sum of the reads + i
//     into each output: nothing is dead code), U = 4 vectors in flight per stream per
//     thread-iteration, grid-stride; nt = non-temporal loads / stores (global_* ... nt).
// Used by scripts/hbm_probe.py (profiles/r6/hbm_roofline.txt).
#include "common.h"

using namespace mx;

namespace {

typedef float nf4 __attribute__((ext_vector_type(4)));

template <int R, int W, bool NT>
__global__ __launch_bounds__(256) void membw_kernel(const nf4* const* __restrict__ src, nf4* const* __restrict__ dst,
                                                    int64_t n) {
  constexpr int U = 4;
  const nf4* s[R > 0 ? R : 1];
  nf4* d[W > 0 ? W : 1];
#pragma unroll
  for (int r = 0; r < R; ++r) s[r] = src[r];
#pragma unroll
  for (int w = 0; w < (W > 0 ? W : 1); ++w) d[w] = dst[w];
  const int64_t stride = (int64_t)gridDim.x * 256;
  for (int64_t i0 = blockIdx.x * 256ll + threadIdx.x; i0 < n; i0 += stride * U) {
    nf4 acc[U];
#pragma unroll
    for (int u = 0; u < U; ++u) acc[u] = (nf4){(float)u, 0.f, 0.f, 0.f};
#pragma unroll
    for (int r = 0; r < R; ++r) {
      nf4 t[U];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int64_t i = min(i0 + u * stride, n - 1);
        t[u] = NT ? __builtin_nontemporal_load(s[r] + i) : s[r][i];
      }
#pragma unroll
      for (int u = 0; u < U; ++u) acc[u] += t[u];
    }
    if (W == 0) {   // read-only: keep the sum alive without a store per element
#pragma unroll
      for (int u = 0; u < U; ++u)
        if (acc[u].x == -12345.f && acc[u].y == 54321.f) d[0][0] = acc[u];
    }
#pragma unroll
    for (int w = 0; w < W; ++w)
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int64_t i = i0 + u * stride;
        if (i < n) {
          if (NT) __builtin_nontemporal_store(acc[u], d[w] + i);
          else d[w][i] = acc[u];
        }
      }
  }
}

template <int R, int W>
int launch(int nt, const nf4* const* src, nf4* const* dst, int64_t n, int blocks, hipStream_t st) {
  if (nt)
    hipLaunchKernelGGL((membw_kernel<R, W, true>), dim3(blocks), dim3(256), 0, st, src, dst, n);
  else
    hipLaunchKernelGGL((membw_kernel<R, W, false>), dim3(blocks), dim3(256), 0, st, src, dst, n);
  return hipGetLastError();
}

}  // namespace

// src / dst: DEVICE arrays of R / W stream pointers (each n float4s, 16-B aligned).
// W == 0 needs one dst pointer (never written unless the sentinel values appear).
MX_EXPORT int mx_membw(int R, int W, int nt, const void* src, const void* dst, int64_t n, int blocks,
                       hipStream_t st) {
  if (n <= 0 || blocks <= 0) return hipErrorInvalidValue;
  auto s = (const nf4* const*)src;
  auto d = (nf4* const*)dst;
#define MX_BW(r, w) if (R == r && W == w) return launch<r, w>(nt, s, d, n, blocks, st);
  MX_BW(1, 0) MX_BW(2, 0) MX_BW(0, 1) MX_BW(1, 1) MX_BW(2, 1) MX_BW(3, 3) MX_BW(4, 4)
#undef MX_BW
  return hipErrorInvalidValue;
}
