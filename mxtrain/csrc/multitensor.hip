// Multi-tensor kernels of the flat fp32 master / bf16 compute-copy training loop
// (models/compute_weights.py FlatMaster; Mask R-CNN on one GPU):
//   * mx_mt_grad_in  : bf16 gradients of the compute copies (one tensor per parameter, in
//                      the copy's layout) -> flat fp32 gradient buffer, times the folded
//                      FrozenBN scale, with per-block sum-of-squares partials (grad clip)
//   * mx_mt_sumsq_fin: deterministic sum of those partials -> ||g||^2
//   * mx_mt_sgd      : clip + SGD-momentum (torch.optim.SGD: d = g + wd p, buf = m buf + d,
//                      p -= lr buf) on the flat fp32 buffers, and the bf16 compute copy of
//                      the updated weights (scaled, laid out for the convs) written in the
//                      same pass, so the next forward needs no cast kernels
//   * mx_mt_cast     : the compute copies alone (first step, after a checkpoint load)
// Replaces, per step, ~150 per-tensor cast / multiply kernels (foreach copies across dtypes
// are not fused by torch) and ~20 multi_tensor_apply launches of torch's clip_grad_norm_ +
// foreach SGD -- the reference's tensorpack/Horovod step does the equivalent in TF's
// fused optimizer ops (examples/maskrcnn/train-maskrcnn-tensorpack.yaml).
//
// Tensor table (int64 x 8 per tensor): {flat offset, n, d0, d1, inner, cl, scale ptr, wd}.
// The fp32 view is contiguous [d0, d1, inner]; the bf16 copy is contiguous (cl = 0) or
// laid out [d0, inner, d1] (cl = 1: channels_last conv weights).  scale (nullable) is per
// d0.  Each 256-thread block owns CH = 2048 consecutive elements of one tensor
// (blockmap[b] = tensor index, tile = b - first block of that tensor).
#include "common.h"

using namespace mx;

namespace {

constexpr int CH = 2048;     // elements per block (256 threads x 8)
constexpr int MAXT = 288;    // tensors per launch (the bf16 pointers travel as kernel args)

struct Ptrs {
  const void* p[MAXT];
};

struct TDesc {
  int64_t off, n, d0, d1, inner, cl, scale, wd;
};

__device__ __forceinline__ TDesc load_desc(const int64_t* tab, int t) {
  const int64_t* d = tab + 8 * t;
  return TDesc{d[0], d[1], d[2], d[3], d[4], d[5], d[6], d[7]};
}
// bf16 position of logical element e = (a, b, s) of [d0, d1, inner]
__device__ __forceinline__ int64_t bpos(const TDesc& T, int64_t e) {
  if (!T.cl || T.inner == 1) return e;
  const int64_t per = T.d1 * T.inner;
  const int64_t a = e / per, r = e - a * per;
  const int64_t b = r / T.inner, s = r - b * T.inner;
  return a * per + s * T.d1 + b;
}
__device__ __forceinline__ float scale_of(const TDesc& T, int64_t e) {
  if (!T.scale) return 1.f;
  return reinterpret_cast<const float*>(T.scale)[e / (T.d1 * T.inner)];
}

// grads (bf16, layout of the copy) -> G (fp32 flat) * scale; partial[b] = sum g^2
__global__ __launch_bounds__(256) void grad_in_kernel(const int64_t* __restrict__ tab, const int* __restrict__ bmap,
                                                      const int* __restrict__ bstart, int t0, int b0, Ptrs src,
                                                      float* __restrict__ G, float* __restrict__ partial) {
  __shared__ float red[4];
  const int b = b0 + blockIdx.x;
  const int t = bmap[b];
  const TDesc T = load_desc(tab, t);
  const uint16_t* s = reinterpret_cast<const uint16_t*>(src.p[t - t0]);
  const int64_t e0 = (int64_t)(b - bstart[t]) * CH + threadIdx.x * 8;
  float acc = 0.f;
  if (e0 < T.n) {
    float g[8];
    const bool lin = !T.cl || T.inner == 1;
    if (lin && e0 + 8 <= T.n && ((T.off | e0) & 7) == 0) {
      unpack8(*reinterpret_cast<const uint4*>(s + e0), g);
      if (T.scale) {
#pragma unroll
        for (int j = 0; j < 8; ++j) g[j] *= scale_of(T, e0 + j);
      }
      float4* o = reinterpret_cast<float4*>(G + T.off + e0);
      o[0] = make_float4(g[0], g[1], g[2], g[3]);
      o[1] = make_float4(g[4], g[5], g[6], g[7]);
#pragma unroll
      for (int j = 0; j < 8; ++j) acc += g[j] * g[j];
    } else {
      for (int j = 0; j < 8 && e0 + j < T.n; ++j) {
        const int64_t e = e0 + j;
        const float v = bf2f(s[bpos(T, e)]) * scale_of(T, e);
        G[T.off + e] = v;
        acc += v * v;
      }
    }
  }
  acc = wave_sum(acc);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = acc;
  __syncthreads();
  if (threadIdx.x == 0) partial[b] = (red[0] + red[1]) + (red[2] + red[3]);
}

// data-parallel: G (all-reduced sum over ranks) *= scale (1 / world), partial[b] = sum g^2 of
// the block's CH elements (n a multiple of 8, G 32-B aligned)
__global__ __launch_bounds__(256) void scale_sumsq_kernel(float* __restrict__ G, int64_t n, float scale,
                                                          float* __restrict__ partial) {
  __shared__ float red[4];
  const int64_t e0 = (int64_t)blockIdx.x * CH + threadIdx.x * 8;
  float acc = 0.f;
  if (e0 < n) {
    float4* g = reinterpret_cast<float4*>(G + e0);
    float4 a = g[0], b = g[1];
    a.x *= scale; a.y *= scale; a.z *= scale; a.w *= scale;
    b.x *= scale; b.y *= scale; b.z *= scale; b.w *= scale;
    g[0] = a;
    g[1] = b;
    acc = (a.x * a.x + a.y * a.y) + (a.z * a.z + a.w * a.w) + (b.x * b.x + b.y * b.y) + (b.z * b.z + b.w * b.w);
  }
  acc = wave_sum(acc);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = acc;
  __syncthreads();
  if (threadIdx.x == 0) partial[blockIdx.x] = (red[0] + red[1]) + (red[2] + red[3]);
}

// one 1024-thread workgroup, four independent loads in flight per thread (a 256-thread
// strided loop waited for each of its ~84 loads in turn: 21 us for the ~21k partials of the
// Mask R-CNN step); fixed summation order
__global__ __launch_bounds__(1024) void sumsq_fin_kernel(const float* __restrict__ partial, int n,
                                                         float* __restrict__ out) {
  __shared__ float red[16];
  float a0 = 0.f, a1 = 0.f, a2 = 0.f, a3 = 0.f;
  int i = threadIdx.x;
  for (; i + 3 * 1024 < n; i += 4 * 1024) {
    const float x0 = partial[i], x1 = partial[i + 1024], x2 = partial[i + 2048], x3 = partial[i + 3072];
    a0 += x0; a1 += x1; a2 += x2; a3 += x3;
  }
  for (; i < n; i += 1024) a0 += partial[i];
  float acc = wave_sum((a0 + a1) + (a2 + a3));
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = acc;
  __syncthreads();
  if (threadIdx.x == 0) {
    float s = 0.f;
#pragma unroll
    for (int w = 0; w < 16; ++w) s += red[w];
    out[0] = s;
  }
}

// hyper: {lr, momentum, weight_decay, max_norm (<= 0: no clip)}
template <bool SGD>
__global__ __launch_bounds__(256) void update_kernel(const int64_t* __restrict__ tab, const int* __restrict__ bmap,
                                                     const int* __restrict__ bstart, float* __restrict__ P,
                                                     const float* __restrict__ G, float* __restrict__ M,
                                                     uint16_t* __restrict__ W, const float* __restrict__ hyper,
                                                     const float* __restrict__ normsq) {
  const int b = blockIdx.x;
  const int t = bmap[b];
  const TDesc T = load_desc(tab, t);
  const int64_t e0 = (int64_t)(b - bstart[t]) * CH + threadIdx.x * 8;
  if (e0 >= T.n) return;
  float lr = 0.f, mom = 0.f, wd = 0.f, cc = 1.f;
  if constexpr (SGD) {
    lr = hyper[0];
    mom = hyper[1];
    wd = T.wd ? hyper[2] : 0.f;
    const float clip = hyper[3];
    if (clip > 0.f && normsq) {
      // torch.nn.utils.clip_grad_norm_: g *= min(1, max_norm / (||g|| + 1e-6))
      const float c = clip / (sqrtf(*normsq) + 1e-6f);
      cc = fminf(c, 1.f);
    }
  }
  const bool vec = e0 + 8 <= T.n && ((T.off | e0) & 7) == 0;
  float p[8];
  if (vec) {
    const float4* pp = reinterpret_cast<const float4*>(P + T.off + e0);
    const float4 a = pp[0], c = pp[1];
    p[0] = a.x; p[1] = a.y; p[2] = a.z; p[3] = a.w; p[4] = c.x; p[5] = c.y; p[6] = c.z; p[7] = c.w;
    if constexpr (SGD) {
      const float4* gp = reinterpret_cast<const float4*>(G + T.off + e0);
      float4* mp = reinterpret_cast<float4*>(M + T.off + e0);
      const float4 g0 = gp[0], g1 = gp[1], m0 = mp[0], m1 = mp[1];
      const float g[8] = {g0.x, g0.y, g0.z, g0.w, g1.x, g1.y, g1.z, g1.w};
      float m[8] = {m0.x, m0.y, m0.z, m0.w, m1.x, m1.y, m1.z, m1.w};
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const float d = g[j] * cc + wd * p[j];
        m[j] = mom * m[j] + d;
        p[j] -= lr * m[j];
      }
      mp[0] = make_float4(m[0], m[1], m[2], m[3]);
      mp[1] = make_float4(m[4], m[5], m[6], m[7]);
      float4* po = reinterpret_cast<float4*>(P + T.off + e0);
      po[0] = make_float4(p[0], p[1], p[2], p[3]);
      po[1] = make_float4(p[4], p[5], p[6], p[7]);
    }
    if (!T.cl || T.inner == 1) {
      float w[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) w[j] = p[j] * scale_of(T, e0 + j);
      *reinterpret_cast<uint4*>(W + T.off + e0) = pack8(w);
    } else {
#pragma unroll
      for (int j = 0; j < 8; ++j) W[T.off + bpos(T, e0 + j)] = f2bf(p[j] * scale_of(T, e0 + j));
    }
    return;
  }
  for (int j = 0; j < 8 && e0 + j < T.n; ++j) {
    const int64_t e = e0 + j;
    float pv = P[T.off + e];
    if constexpr (SGD) {
      const float d = G[T.off + e] * cc + wd * pv;
      const float m = mom * M[T.off + e] + d;
      M[T.off + e] = m;
      pv -= lr * m;
      P[T.off + e] = pv;
    }
    W[T.off + bpos(T, e)] = f2bf(pv * scale_of(T, e));
  }
}

}  // namespace

MX_EXPORT int mx_mt_chunk() { return CH; }
MX_EXPORT int mx_mt_max_tensors() { return MAXT; }

// Tensors [tb, te) of the table (a data-parallel bucket, or all of them): src = host array of
// their te - tb bf16 gradient pointers; partial: the blocks' sum-of-squares slots
// (partial[bstart[t] ..] for tensor t).
MX_EXPORT int mx_mt_grad_in_range(const int64_t* tab, const int* bmap, const int* bstart, const int* bstart_host,
                                  int tb, int te, const int64_t* src, float* G, float* partial, hipStream_t s) {
  for (int t0 = tb; t0 < te; t0 += MAXT) {
    const int t1 = min(te, t0 + MAXT);
    Ptrs ptrs{};
    for (int t = t0; t < t1; ++t) ptrs.p[t - t0] = reinterpret_cast<const void*>(src[t - tb]);
    const int b0 = bstart_host[t0], nb = bstart_host[t1] - b0;
    if (nb > 0)
      hipLaunchKernelGGL(grad_in_kernel, dim3(nb), dim3(256), 0, s, tab, bmap, bstart, t0, b0, ptrs, G, partial);
  }
  return hipGetLastError();
}

// src: host array of T bf16 gradient pointers (tensor order of the table); nblocks = total
// blocks (bstart[T]); partial: nblocks floats.
MX_EXPORT int mx_mt_grad_in(const int64_t* tab, const int* bmap, const int* bstart, const int* bstart_host, int T,
                            const int64_t* src, float* G, float* partial, hipStream_t s) {
  return mx_mt_grad_in_range(tab, bmap, bstart, bstart_host, 0, T, src, G, partial, s);
}

// G[0, n) *= scale with per-2048-element sum-of-squares partials (ceil(n / 2048) of them);
// n a multiple of 8, G 32-B aligned
MX_EXPORT int mx_mt_scale_sumsq(float* G, int64_t n, float scale, float* partial, hipStream_t s) {
  if (n <= 0 || (n & 7) || ((uintptr_t)G & 31)) return (int)hipErrorInvalidValue;
  const int64_t nb = (n + CH - 1) / CH;
  hipLaunchKernelGGL(scale_sumsq_kernel, dim3((unsigned)nb), dim3(256), 0, s, G, n, scale, partial);
  return hipGetLastError();
}

MX_EXPORT int mx_mt_sumsq_fin(const float* partial, int n, float* out, hipStream_t s) {
  hipLaunchKernelGGL(sumsq_fin_kernel, dim3(1), dim3(1024), 0, s, partial, n, out);
  return hipGetLastError();
}

MX_EXPORT int mx_mt_sgd(const int64_t* tab, const int* bmap, const int* bstart, int nblocks, float* P, const float* G,
                        float* M, void* W, const float* hyper, const float* normsq, hipStream_t s) {
  if (nblocks <= 0) return hipSuccess;
  hipLaunchKernelGGL(update_kernel<true>, dim3(nblocks), dim3(256), 0, s, tab, bmap, bstart, P, G, M,
                     (uint16_t*)W, hyper, normsq);
  return hipGetLastError();
}

MX_EXPORT int mx_mt_cast(const int64_t* tab, const int* bmap, const int* bstart, int nblocks, float* P, void* W,
                         hipStream_t s) {
  if (nblocks <= 0) return hipSuccess;
  hipLaunchKernelGGL(update_kernel<false>, dim3(nblocks), dim3(256), 0, s, tab, bmap, bstart, P, nullptr, nullptr,
                     (uint16_t*)W, nullptr, nullptr);
  return hipGetLastError();
}
