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
  for (int64_t v = blockIdx.x * 256ll + threadIdx.x; v < nvec; v += (int64_t)gridDim.x * 256) {
    if (flags && !flags[(v * 8) >> 6]) continue;
    float a[8];
    unpack8(*reinterpret_cast<const uint4*>(g + v * 8), a);
#pragma unroll
    for (int j = 0; j < 8; ++j) { float t = a[j] * scale; acc += t * t; }
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

// 4 elements per thread-iteration; wd_flags has one byte per 64-element chunk.
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
  const int64_t nvec = n / 4;
  for (int64_t i = blockIdx.x * 256ll + threadIdx.x; i < nvec; i += (int64_t)gridDim.x * 256) {
    float4 p = reinterpret_cast<float4*>(master)[i];
    float4 mm = reinterpret_cast<float4*>(m)[i];
    float4 vv = reinterpret_cast<float4*>(v)[i];
    uint2 graw = reinterpret_cast<const uint2*>(grad)[i];
    const float decay = (wd_flags == nullptr || wd_flags[(i * 4) >> 6]) ? wd : 0.f;
    float g[4] = {lo_bf(graw.x) * gs, hi_bf(graw.x) * gs, lo_bf(graw.y) * gs,
                  hi_bf(graw.y) * gs};
    float* pp = &p.x;
    float* pm = &mm.x;
    float* pv = &vv.x;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      pm[j] = b1 * pm[j] + (1.f - b1) * g[j];
      pv[j] = b2 * pv[j] + (1.f - b2) * g[j] * g[j];
      const float denom = sqrtf(pv[j]) * inv_sqrt_bc2 + eps;
      pp[j] = pp[j] * (1.f - lr * decay) - step_size * pm[j] / denom;
    }
    reinterpret_cast<float4*>(master)[i] = p;
    reinterpret_cast<float4*>(m)[i] = mm;
    reinterpret_cast<float4*>(v)[i] = vv;
    uint2 out;
    out.x = pack2(p.x, p.y);
    out.y = pack2(p.z, p.w);
    reinterpret_cast<uint2*>(param_out)[i] = out;
  }
}

}  // namespace

MX_EXPORT int mx_sumsq_nparts() { return 1024; }

// normsq_out[0] (+)= sum((g*scale)^2); partial must hold mx_sumsq_nparts() floats
MX_EXPORT int mx_sumsq_bf16(const void* g, int64_t n, float scale, const uint8_t* flags,
                            float* partial, float* normsq_out, int accumulate, hipStream_t s) {
  int64_t blocks = (n / 8 + 255) / 256;
  if (blocks > 1024) blocks = 1024;
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
  int64_t blocks = (n / 4 + 255) / 256;
  if (blocks > 2048) blocks = 2048;
  if (blocks < 1) blocks = 1;
  hipLaunchKernelGGL(adamw_kernel, dim3((unsigned)blocks), dim3(256), 0, s, master, m, v,
                     (const uint16_t*)grad, (uint16_t*)param_out, wd_flags, n, hyper, normsq);
  return hipGetLastError();
}
