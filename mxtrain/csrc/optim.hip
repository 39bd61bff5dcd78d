// Fused optimizer kernels on flat (ZeRO-1 shard) buffers.
//   * mx_sumsq_bf16   : multi-tensor L2 norm of the gradient shard (K9)
//   * mx_adamw_step   : AdamW with on-device grad-clip coefficient, inf/nan skip,
//                       fp32 master + moments, fused bf16 parameter write-back (K8)
// Replaces Apex `amp_C.multi_tensor_adam/l2norm/scale` and DeepSpeed FusedAdam the
// reference's Megatron-DeepSpeed image builds (containers/megatron-deepspeed/
// Dockerfile:6-12; `--clip-grad 1.0`, fp16/bf16 at pretrain-ddp-zero1.yaml:33-53).
//
// Because the whole shard is one contiguous range there is no tensor-list chunking:
// a single grid-stride launch covers every parameter.  Scalars that change every step
// (lr, bias corrections, clip) are read from a small device array so the step can be
// captured once in a hipGraph and replayed.
#include "common.h"

using namespace mx;

namespace {

// hyper[] layout (fp32): 0 lr, 1 beta1, 2 beta2, 3 eps, 4 weight_decay,
// 5 bias_correction1 (1 - b1^t), 6 bias_correction2 (1 - b2^t), 7 grad_scale,
// 8 max_grad_norm (<=0: no clipping)
enum { H_LR = 0, H_B1, H_B2, H_EPS, H_WD, H_BC1, H_BC2, H_GS, H_CLIP, H_N };

// flags (nullable): one byte per 64-element chunk; chunks with flag 0 are skipped
// (tensor-parallel duplicates / tied copies counted once in the global grad norm)
__global__ __launch_bounds__(256) void sumsq_kernel(const uint16_t* __restrict__ g, int64_t n,
                                                    float scale, const uint8_t* __restrict__ flags,
                                                    float* __restrict__ partial) {
  __shared__ float red[4];
  float acc = 0.f;
  const int64_t nvec = n / 8;
  const int64_t stride = (int64_t)gridDim.x * 256;
  // U vectors per thread-iteration, every load issued before any math: addresses are
  // clamped into the buffer and the loads unconditional (a `ok ? load : 0` select made the
  // compiler wait for each load where it was issued, and the flag byte gated the data load:
  // two serial memory latencies per vector); skipped chunks / the overhang are masked after
  constexpr int U = 8;
  for (int64_t v0 = blockIdx.x * 256ll + threadIdx.x; v0 < nvec; v0 += stride * U) {
    uint4 raw[U];
    uint8_t fl[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int64_t v = min(v0 + u * stride, nvec - 1);
      fl[u] = flags ? flags[(v * 8) >> 6] : (uint8_t)1;
      raw[u] = reinterpret_cast<const uint4*>(g)[v];
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      float a[8];
      unpack8(raw[u], a);
      float part = 0.f;
#pragma unroll
      for (int j = 0; j < 8; ++j) { float t = a[j] * scale; part += t * t; }
      acc += (v0 + u * stride < nvec && fl[u]) ? part : 0.f;
    }
  }
  for (int64_t i = nvec * 8 + blockIdx.x * 256ll + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * 256) {
    if (flags && !flags[i >> 6]) continue;
    float t = bf2f(g[i]) * scale;
    acc += t * t;
  }
  acc = wave_sum(acc);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = acc;
  __syncthreads();
  if (threadIdx.x == 0) partial[blockIdx.x] = red[0] + red[1] + red[2] + red[3];
}

__global__ void sum_partials_kernel(const float* __restrict__ partial, int n,
                                    float* __restrict__ out, int accumulate) {
  __shared__ float red[4];
  float acc = 0.f;
  for (int i = threadIdx.x; i < n; i += 256) acc += partial[i];
  acc = wave_sum(acc);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = acc;
  __syncthreads();
  if (threadIdx.x == 0) {
    float s = red[0] + red[1] + red[2] + red[3];
    out[0] = accumulate ? out[0] + s : s;
  }
}

// 8 elements per thread-iteration (two float4 of each fp32 state, one 16-B bf16 grad
// load, one 16-B bf16 param store), every load of the iteration issued before any math,
// non-temporal access (the 28 B/element stream is touched exactly once per step and
// must not evict anything useful from L2).  wd_flags has one byte per 64-element chunk.
typedef float nf4 __attribute__((ext_vector_type(4)));
typedef unsigned int nu4 __attribute__((ext_vector_type(4)));
__device__ __forceinline__ float4 ldnt4(const float* p) {   // one global_load_dwordx4 ... nt
  const nf4 v = __builtin_nontemporal_load(reinterpret_cast<const nf4*>(p));
  return make_float4(v.x, v.y, v.z, v.w);
}
__device__ __forceinline__ void stnt4(float* p, float4 v) {
  __builtin_nontemporal_store((nf4){v.x, v.y, v.z, v.w}, reinterpret_cast<nf4*>(p));
}

template <int U>
__global__ __launch_bounds__(256) void adamw_kernel(
    float* __restrict__ master, float* __restrict__ m, float* __restrict__ v,
    const uint16_t* __restrict__ grad, uint16_t* __restrict__ param_out,
    const uint8_t* __restrict__ wd_flags, int64_t n, const float* __restrict__ hyper,
    const float* __restrict__ normsq) {
  const float ns = normsq ? *normsq : 0.f;
  if (!(ns == ns) || ns == INFINITY) return;  // overflow: skip the step (loss-scaler path)
  const float lr = hyper[H_LR], b1 = hyper[H_B1], b2 = hyper[H_B2], eps = hyper[H_EPS];
  const float wd = hyper[H_WD], bc1 = hyper[H_BC1], bc2 = hyper[H_BC2];
  float gs = hyper[H_GS];
  const float clip = hyper[H_CLIP];
  if (clip > 0.f && normsq) {
    const float norm = sqrtf(ns);
    const float coef = clip / (norm + 1e-6f);
    if (coef < 1.f) gs *= coef;
  }
  const float step_size = lr / bc1;
  const float inv_sqrt_bc2 = rsqrtf(bc2);
  const int64_t nvec = n / 8;
  const int64_t stride = (int64_t)gridDim.x * 256;
  // U independent 8-element vectors per thread-iteration: all 7*U loads are issued
  // before any math, so more bytes are in flight per wave (HBM3E needs ~MBs in flight)
  for (int64_t i0 = blockIdx.x * 256ll + threadIdx.x; i0 < nvec; i0 += stride * U) {
    float4 p0[U], p1[U], m0[U], m1[U], v0[U], v1[U];
    nu4 gr[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int64_t i = i0 + u * stride;
      if (i < nvec) {
        const int64_t e = i * 8;
        p0[u] = ldnt4(master + e); p1[u] = ldnt4(master + e + 4);
        m0[u] = ldnt4(m + e); m1[u] = ldnt4(m + e + 4);
        v0[u] = ldnt4(v + e); v1[u] = ldnt4(v + e + 4);
        gr[u] = __builtin_nontemporal_load(reinterpret_cast<const nu4*>(grad) + i);
      }
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int64_t i = i0 + u * stride;
      if (i >= nvec) break;
      const int64_t e = i * 8;
      const float decay = (wd_flags == nullptr || wd_flags[e >> 6]) ? wd : 0.f;
      float g[8];
      unpack8(make_uint4(gr[u].x, gr[u].y, gr[u].z, gr[u].w), g);
      float pp[8] = {p0[u].x, p0[u].y, p0[u].z, p0[u].w, p1[u].x, p1[u].y, p1[u].z, p1[u].w};
      float pm[8] = {m0[u].x, m0[u].y, m0[u].z, m0[u].w, m1[u].x, m1[u].y, m1[u].z, m1[u].w};
      float pv[8] = {v0[u].x, v0[u].y, v0[u].z, v0[u].w, v1[u].x, v1[u].y, v1[u].z, v1[u].w};
      const float keep = 1.f - lr * decay;
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const float gj = g[j] * gs;
        pm[j] = b1 * pm[j] + (1.f - b1) * gj;
        pv[j] = b2 * pv[j] + (1.f - b2) * gj * gj;
        const float denom = sqrtf(pv[j]) * inv_sqrt_bc2 + eps;
        pp[j] = pp[j] * keep - step_size * pm[j] / denom;
      }
      stnt4(master + e, make_float4(pp[0], pp[1], pp[2], pp[3]));
      stnt4(master + e + 4, make_float4(pp[4], pp[5], pp[6], pp[7]));
      stnt4(m + e, make_float4(pm[0], pm[1], pm[2], pm[3]));
      stnt4(m + e + 4, make_float4(pm[4], pm[5], pm[6], pm[7]));
      stnt4(v + e, make_float4(pv[0], pv[1], pv[2], pv[3]));
      stnt4(v + e + 4, make_float4(pv[4], pv[5], pv[6], pv[7]));
      const uint4 po = pack8(pp);
      __builtin_nontemporal_store((nu4){po.x, po.y, po.z, po.w}, reinterpret_cast<nu4*>(param_out) + i);
    }
  }
}

// one 8-element vector per thread (no grid-stride loop, U = 1): 355M elements 1.95 ms at 16384
// blocks, 1.85 at 131072; at 5.22 TB/s it sits on the measured 3-read / 3-write HBM roofline
// (profiles/r6/hbm_roofline.txt)
constexpr int g_adam_blocks = 1 << 20;

}  // namespace

constexpr int kSumsqParts = 2048;   // blocks of sumsq_kernel = partial slots
MX_EXPORT int mx_sumsq_nparts() { return kSumsqParts; }


// normsq_out[0] (+)= sum((g*scale)^2); partial must hold mx_sumsq_nparts() floats
MX_EXPORT int mx_sumsq_bf16(const void* g, int64_t n, float scale, const uint8_t* flags,
                            float* partial, float* normsq_out, int accumulate, hipStream_t s) {
  int64_t blocks = (n / 8 + 255) / 256;
  if (blocks > kSumsqParts) blocks = kSumsqParts;
  if (blocks < 1) blocks = 1;
  hipLaunchKernelGGL(sumsq_kernel, dim3((unsigned)blocks), dim3(256), 0, s,
                     (const uint16_t*)g, n, scale, flags, partial);
  hipLaunchKernelGGL(sum_partials_kernel, dim3(1), dim3(256), 0, s, partial, (int)blocks,
                     normsq_out, accumulate);
  return hipGetLastError();
}

// n must be a multiple of 4 (shards are 64-element aligned)
MX_EXPORT int mx_adamw_step(float* master, float* m, float* v, const void* grad,
                            void* param_out, const uint8_t* wd_flags, int64_t n,
                            const float* hyper, const float* normsq, hipStream_t s) {
  if (n % 8) return hipErrorInvalidValue;  // flat shards are 64-element aligned
  int64_t blocks = (n / 8 + 255) / 256;
  if (blocks > g_adam_blocks) blocks = g_adam_blocks;
  if (blocks < 1) blocks = 1;
  hipLaunchKernelGGL(adamw_kernel<1>, dim3((unsigned)blocks), dim3(256), 0, s, master, m, v,
                       (const uint16_t*)grad, (uint16_t*)param_out, wd_flags, n, hyper, normsq);
  return hipGetLastError();
}

// ---------------------------------------------------------------------------- multi-tensor SGD
// torch.optim.SGD's update (weight decay, momentum, Nesterov; dampening 0) over a list of
// fp32 parameters in ONE launch, the learning rate read from a device scalar (so the step can
// be captured in a hipGraph while an LR scheduler moves it): per element
//   d = g + wd p;  buf = mom buf + d;  u = nesterov ? d + mom buf : buf;  p -= lr u
// -- the Ray-Lightning ResNet-50 step (raylike/lightning.py), where torch's multi-tensor
// kernels took 19 launches and ~420 us for ~510 MB (1.2 TB/s) per step.  Jobs by value,
// 4-element vectors (numel % 4 == 0, 16-byte aligned).
namespace {
constexpr int kSgdJobs = 96;
struct SgdJob {
  float* p;
  const float* g;
  float* buf;
  int64_t v0;   // first float4 of this job in the launch's flat vector space
};
struct SgdJobs {
  SgdJob j[kSgdJobs];
};

__global__ __launch_bounds__(256) void sgd_multi_kernel(const SgdJobs js, int njobs, int64_t nvec, const float* lr_p,
                                                        float wd, float mom, int nesterov) {
  const float lr = *lr_p;
  for (int64_t v = (int64_t)blockIdx.x * 256 + threadIdx.x; v < nvec; v += (int64_t)gridDim.x * 256) {
    int lo = 0, hi = njobs - 1;
    while (lo < hi) {
      const int mid = (lo + hi + 1) >> 1;
      if (js.j[mid].v0 <= v) lo = mid;
      else hi = mid - 1;
    }
    const SgdJob& J = js.j[lo];
    const int64_t e = v - J.v0;
    float4 p = reinterpret_cast<const float4*>(J.p)[e];
    const float4 g = reinterpret_cast<const float4*>(J.g)[e];
    float pv[4] = {p.x, p.y, p.z, p.w};
    const float gv[4] = {g.x, g.y, g.z, g.w};
    float bv[4] = {0.f, 0.f, 0.f, 0.f};
    float4 b;
    if (J.buf) {
      b = reinterpret_cast<const float4*>(J.buf)[e];
      bv[0] = b.x; bv[1] = b.y; bv[2] = b.z; bv[3] = b.w;
    }
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const float d = gv[k] + wd * pv[k];
      float u = d;
      if (J.buf) {
        bv[k] = bv[k] * mom + d;
        u = nesterov ? d + mom * bv[k] : bv[k];
      }
      pv[k] = pv[k] - u * lr;
    }
    reinterpret_cast<float4*>(J.p)[e] = make_float4(pv[0], pv[1], pv[2], pv[3]);
    if (J.buf) reinterpret_cast<float4*>(J.buf)[e] = make_float4(bv[0], bv[1], bv[2], bv[3]);
  }
}
}  // namespace

// d (int64[4 * njobs]): {param, grad, momentum buffer (0: no momentum), numel} per job
MX_EXPORT int mx_sgd_multi(const int64_t* d, int njobs, const float* lr, float wd, float mom, int nesterov,
                           hipStream_t s) {
  if (njobs <= 0 || njobs > kSgdJobs || !lr) return hipErrorInvalidValue;
  SgdJobs js{};
  int64_t nvec = 0;
  for (int i = 0; i < njobs; ++i) {
    const int64_t n = d[4 * i + 3];
    if (n <= 0 || n % 4 || ((d[4 * i] | d[4 * i + 1] | d[4 * i + 2]) & 15)) return hipErrorInvalidValue;
    js.j[i].p = reinterpret_cast<float*>(d[4 * i]);
    js.j[i].g = reinterpret_cast<const float*>(d[4 * i + 1]);
    js.j[i].buf = reinterpret_cast<float*>(d[4 * i + 2]);
    js.j[i].v0 = nvec;
    nvec += n / 4;
  }
  int64_t g = (nvec + 255) / 256;
  if (g > 4096) g = 4096;
  hipLaunchKernelGGL(sgd_multi_kernel, dim3((unsigned)g), dim3(256), 0, s, js, njobs, nvec, lr, wd, mom, nesterov);
  return hipGetLastError();
}
