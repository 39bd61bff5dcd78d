// Fused Mask R-CNN training losses: forward = loss partial sums per
// block + one finalize launch; backward = one launch writing the input gradients from the
// saved inputs, the device-side normalisers and the upstream gradient scalars.  Replaces
// ~25 torch elementwise / reduction launches per loss (BCE-with-logits, masks, huber via
// where/abs, sums, divisions, gathers, fp32 casts) -- the tensorpack losses
// (rpn_losses, fastrcnn_losses, maskrcnn_loss in the reference's tensorpack-maskrcnn
// image, containers/tensorpack-maskrcnn) with the same definitions as the torch path of
// models/maskrcnn.py:
//   RPN   cls = sum_sel BCE(x, pos) / max(#sel, 1);  box = sum_pos huber(d - t, 1/9) / (B * 256)
//   FRCNN cls = mean_i CE(x_i, label_i);  box = sum_fg huber(d[label] - t, 1) / N
//   mask  = sum_r valid_r mean_p BCE(x[r, label_r - 1, p], m_rp >= 0.5) / max(sum valid, 1)
// Partials: [nblocks][4] fp32 (sum a, sum b, count, unused); out: {loss a, loss b, norm a, norm b}.
#include "common.h"

using namespace mx;

namespace {

constexpr int kLB = 256;   // threads per block

__device__ __forceinline__ float bce_logits(float x, float y) {
  // max(x, 0) - x y + log(1 + exp(-|x|))
  return fmaxf(x, 0.f) - x * y + log1pf(__expf(-fabsf(x)));
}
__device__ __forceinline__ float sigmoidf_(float x) { return 1.f / (1.f + __expf(-x)); }
__device__ __forceinline__ float huber(float z, float d) {
  const float a = fabsf(z);
  return a < d ? 0.5f * z * z : d * (a - 0.5f * d);
}
__device__ __forceinline__ float huber_grad(float z, float d) {
  const float a = fabsf(z);
  return a < d ? z : (z > 0.f ? d : (z < 0.f ? -d : 0.f));
}

__device__ __forceinline__ void block_store3(float a, float b, float c, float* __restrict__ partial) {
  __shared__ float red[3][kLB / 64];
  a = wave_sum(a);
  b = wave_sum(b);
  c = wave_sum(c);
  const int w = threadIdx.x >> 6;
  if ((threadIdx.x & 63) == 0) { red[0][w] = a; red[1][w] = b; red[2][w] = c; }
  __syncthreads();
  if (threadIdx.x == 0) {
    float s0 = 0.f, s1 = 0.f, s2 = 0.f;
#pragma unroll
    for (int i = 0; i < kLB / 64; ++i) { s0 += red[0][i]; s1 += red[1][i]; s2 += red[2][i]; }
    float* p = partial + 4 * blockIdx.x;
    p[0] = s0; p[1] = s1; p[2] = s2; p[3] = 0.f;
  }
}

// ---------------------------------------------------------------------------- RPN
__global__ __launch_bounds__(kLB) void rpn_fwd_kernel(const uint16_t* __restrict__ logit, const uint16_t* __restrict__ delta,
                                                      const float* __restrict__ tgt, const uint8_t* __restrict__ pos,
                                                      const uint8_t* __restrict__ neg, int n, float* __restrict__ partial) {
  float sc = 0.f, sb = 0.f, cnt = 0.f;
  for (int i = blockIdx.x * kLB + threadIdx.x; i < n; i += gridDim.x * kLB) {
    const bool p = pos[i], s = p || neg[i];
    if (s) {
      sc += bce_logits(bf2f(logit[i]), p ? 1.f : 0.f);
      cnt += 1.f;
    }
    if (p) {
      const uint2 dr = *reinterpret_cast<const uint2*>(delta + (size_t)i * 4);
      const float4 t = *reinterpret_cast<const float4*>(tgt + (size_t)i * 4);
      sb += huber(lo_bf(dr.x) - t.x, 1.f / 9) + huber(hi_bf(dr.x) - t.y, 1.f / 9) +
            huber(lo_bf(dr.y) - t.z, 1.f / 9) + huber(hi_bf(dr.y) - t.w, 1.f / 9);
    }
  }
  block_store3(sc, sb, cnt, partial);
}

// mode 0 RPN: a / max(cnt, 1), b / norm_b;  1 FRCNN: a / norm_a, b / norm_b;
// 2 mask: a / max(cnt, 1) (cnt = sum valid)
__global__ __launch_bounds__(kLB) void loss_fin_kernel(const float* __restrict__ partial, int nb, int mode, float norm_a,
                                                       float norm_b, float* __restrict__ out) {
  __shared__ float red[3][kLB / 64];
  float a = 0.f, b = 0.f, c = 0.f;
  for (int i = threadIdx.x; i < nb; i += kLB) { a += partial[4 * i]; b += partial[4 * i + 1]; c += partial[4 * i + 2]; }
  a = wave_sum(a);
  b = wave_sum(b);
  c = wave_sum(c);
  const int w = threadIdx.x >> 6;
  if ((threadIdx.x & 63) == 0) { red[0][w] = a; red[1][w] = b; red[2][w] = c; }
  __syncthreads();
  if (threadIdx.x == 0) {
    float s0 = 0.f, s1 = 0.f, s2 = 0.f;
#pragma unroll
    for (int i = 0; i < kLB / 64; ++i) { s0 += red[0][i]; s1 += red[1][i]; s2 += red[2][i]; }
    const float na = mode == 1 ? norm_a : fmaxf(s2, 1.f);
    out[0] = s0 / na;
    out[1] = s1 / norm_b;
    out[2] = na;
    out[3] = norm_b;
  }
}

__global__ __launch_bounds__(kLB) void rpn_bwd_kernel(const uint16_t* __restrict__ logit, const uint16_t* __restrict__ delta,
                                                      const float* __restrict__ tgt, const uint8_t* __restrict__ pos,
                                                      const uint8_t* __restrict__ neg, int n, const float* __restrict__ norms,
                                                      const float* __restrict__ g_cls, const float* __restrict__ g_box,
                                                      uint16_t* __restrict__ dlogit, uint16_t* __restrict__ ddelta) {
  const float gc = (g_cls ? *g_cls : 0.f) / norms[2], gb = (g_box ? *g_box : 0.f) / norms[3];
  for (int i = blockIdx.x * kLB + threadIdx.x; i < n; i += gridDim.x * kLB) {
    const bool p = pos[i], s = p || neg[i];
    dlogit[i] = f2bf(s ? gc * (sigmoidf_(bf2f(logit[i])) - (p ? 1.f : 0.f)) : 0.f);
    uint2 o = make_uint2(0u, 0u);
    if (p) {
      const uint2 dr = *reinterpret_cast<const uint2*>(delta + (size_t)i * 4);
      const float4 t = *reinterpret_cast<const float4*>(tgt + (size_t)i * 4);
      o.x = pack2(gb * huber_grad(lo_bf(dr.x) - t.x, 1.f / 9), gb * huber_grad(hi_bf(dr.x) - t.y, 1.f / 9));
      o.y = pack2(gb * huber_grad(lo_bf(dr.y) - t.z, 1.f / 9), gb * huber_grad(hi_bf(dr.y) - t.w, 1.f / 9));
    }
    *reinterpret_cast<uint2*>(ddelta + (size_t)i * 4) = o;
  }
}

// ---------------------------------------------------------------------------- Fast R-CNN
// one wave per RoI row: logits bf16 [N][C], deltas bf16 [N][C][4], labels int64, tgt fp32
// [N][4], fg uint8
__global__ __launch_bounds__(kLB) void frcnn_fwd_kernel(const uint16_t* __restrict__ logit, const uint16_t* __restrict__ delta,
                                                        const int64_t* __restrict__ label, const float* __restrict__ tgt,
                                                        const uint8_t* __restrict__ fg, int N, int C,
                                                        float* __restrict__ partial) {
  const int lane = threadIdx.x & 63;
  float sc = 0.f, sb = 0.f;
  for (int r = blockIdx.x * (kLB / 64) + (threadIdx.x >> 6); r < N; r += gridDim.x * (kLB / 64)) {
    const uint16_t* x = logit + (size_t)r * C;
    float m = -INFINITY;
    for (int c = lane; c < C; c += 64) m = fmaxf(m, bf2f(x[c]));
    m = wave_max(m);
    float se = 0.f;
    for (int c = lane; c < C; c += 64) se += __expf(bf2f(x[c]) - m);
    se = wave_sum(se);
    const int lab = (int)label[r];
    if (lane == 0) {
      sc += m + __logf(se) - bf2f(x[lab]);
      if (fg[r]) {
        const uint2 dr = *reinterpret_cast<const uint2*>(delta + ((size_t)r * C + lab) * 4);
        const float4 t = *reinterpret_cast<const float4*>(tgt + (size_t)r * 4);
        sb += huber(lo_bf(dr.x) - t.x, 1.f) + huber(hi_bf(dr.x) - t.y, 1.f) + huber(lo_bf(dr.y) - t.z, 1.f) +
              huber(hi_bf(dr.y) - t.w, 1.f);
      }
    }
  }
  block_store3(sc, sb, 0.f, partial);
}

__global__ __launch_bounds__(kLB) void frcnn_bwd_kernel(const uint16_t* __restrict__ logit, const uint16_t* __restrict__ delta,
                                                        const int64_t* __restrict__ label, const float* __restrict__ tgt,
                                                        const uint8_t* __restrict__ fg, int N, int C,
                                                        const float* __restrict__ norms, const float* __restrict__ g_cls,
                                                        const float* __restrict__ g_box, uint16_t* __restrict__ dlogit,
                                                        uint16_t* __restrict__ ddelta) {
  const int lane = threadIdx.x & 63;
  const float gc = (g_cls ? *g_cls : 0.f) / norms[2], gb = (g_box ? *g_box : 0.f) / norms[3];
  for (int r = blockIdx.x * (kLB / 64) + (threadIdx.x >> 6); r < N; r += gridDim.x * (kLB / 64)) {
    const uint16_t* x = logit + (size_t)r * C;
    float m = -INFINITY;
    for (int c = lane; c < C; c += 64) m = fmaxf(m, bf2f(x[c]));
    m = wave_max(m);
    float se = 0.f;
    for (int c = lane; c < C; c += 64) se += __expf(bf2f(x[c]) - m);
    se = wave_sum(se);
    const float inv = 1.f / se;
    const int lab = (int)label[r];
    for (int c = lane; c < C; c += 64)
      dlogit[(size_t)r * C + c] = f2bf(gc * (__expf(bf2f(x[c]) - m) * inv - (c == lab ? 1.f : 0.f)));
    const bool f = fg[r];
    float4 t = make_float4(0.f, 0.f, 0.f, 0.f);
    uint2 dl = make_uint2(0u, 0u);
    if (f) {
      t = *reinterpret_cast<const float4*>(tgt + (size_t)r * 4);
      dl = *reinterpret_cast<const uint2*>(delta + ((size_t)r * C + lab) * 4);
    }
    for (int c = lane; c < C; c += 64) {
      uint2 o = make_uint2(0u, 0u);
      if (f && c == lab) {
        o.x = pack2(gb * huber_grad(lo_bf(dl.x) - t.x, 1.f), gb * huber_grad(hi_bf(dl.x) - t.y, 1.f));
        o.y = pack2(gb * huber_grad(lo_bf(dl.y) - t.z, 1.f), gb * huber_grad(hi_bf(dl.y) - t.w, 1.f));
      }
      *reinterpret_cast<uint2*>(ddelta + ((size_t)r * C + c) * 4) = o;
    }
  }
}

// ---------------------------------------------------------------------------- mask
// logits bf16 channels_last [R][P][K] (P = 28 x 28 pixels, K classes), label int64 [R]
// (1..K for fg, 0 for bg rows), target fp32 [R][P], valid fp32 [R]
__global__ __launch_bounds__(kLB) void mask_fwd_kernel(const uint16_t* __restrict__ logit, const int64_t* __restrict__ label,
                                                       const float* __restrict__ target, const float* __restrict__ valid,
                                                       int R, int P, int K, float* __restrict__ partial) {
  float s = 0.f, cnt = 0.f;
  const int n = R * P;
  for (int i = blockIdx.x * kLB + threadIdx.x; i < n; i += gridDim.x * kLB) {
    const int r = i / P;
    const float v = valid[r];
    if (v != 0.f) {
      const int c = max((int)label[r] - 1, 0);
      const float x = bf2f(logit[(size_t)i * K + c]);
      s += v * bce_logits(x, target[i] >= 0.5f ? 1.f : 0.f) / (float)P;
    }
    if (i - r * P == 0) cnt += v;
  }
  block_store3(s, 0.f, cnt, partial);
}

__global__ __launch_bounds__(kLB) void mask_bwd_kernel(const uint16_t* __restrict__ logit, const int64_t* __restrict__ label,
                                                       const float* __restrict__ target, const float* __restrict__ valid,
                                                       int R, int P, int K, const float* __restrict__ norms,
                                                       const float* __restrict__ g, uint16_t* __restrict__ dlogit) {
  // one thread per (pixel, 8-class group): zeros except the row's class
  const float gs = (g ? *g : 0.f) / norms[2] / (float)P;
  const int KG = K / 8;
  const long long n = (long long)R * P * KG;
  for (long long j = blockIdx.x * (long long)kLB + threadIdx.x; j < n; j += (long long)gridDim.x * kLB) {
    const long long i = j / KG;
    const int kg = (int)(j - i * KG);
    const int r = (int)(i / P);
    const int c = max((int)label[r] - 1, 0);
    float o[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    if (c / 8 == kg) {
      const float v = valid[r];
      const float x = bf2f(logit[(size_t)i * K + c]);
      o[c % 8] = gs * v * (sigmoidf_(x) - (target[i] >= 0.5f ? 1.f : 0.f));
    }
    *reinterpret_cast<uint4*>(dlogit + (size_t)i * K + 8 * kg) = pack8(o);
  }
}

int nblocks_for(long long n, int per) {
  long long b = (n + per - 1) / per;
  if (b > 1024) b = 1024;
  if (b < 1) b = 1;
  return (int)b;
}

}  // namespace

MX_EXPORT int mx_detloss_max_blocks() { return 1024; }

// partial: 4 x 1024 floats; out: 4 floats {loss_cls, loss_box, norm_cls, norm_box}
MX_EXPORT int mx_rpn_loss_fwd(const void* logit, const void* delta, const float* tgt, const uint8_t* pos,
                              const uint8_t* neg, int n, float box_norm, float* partial, float* out, hipStream_t s) {
  const int nb = nblocks_for(n, kLB * 8);
  hipLaunchKernelGGL(rpn_fwd_kernel, dim3(nb), dim3(kLB), 0, s, (const uint16_t*)logit, (const uint16_t*)delta, tgt, pos,
                     neg, n, partial);
  hipLaunchKernelGGL(loss_fin_kernel, dim3(1), dim3(kLB), 0, s, partial, nb, 0, 1.f, box_norm, out);
  return hipGetLastError();
}
MX_EXPORT int mx_rpn_loss_bwd(const void* logit, const void* delta, const float* tgt, const uint8_t* pos,
                              const uint8_t* neg, int n, const float* norms, const float* g_cls, const float* g_box,
                              void* dlogit, void* ddelta, hipStream_t s) {
  hipLaunchKernelGGL(rpn_bwd_kernel, dim3(nblocks_for(n, kLB * 4)), dim3(kLB), 0, s, (const uint16_t*)logit,
                     (const uint16_t*)delta, tgt, pos, neg, n, norms, g_cls, g_box, (uint16_t*)dlogit, (uint16_t*)ddelta);
  return hipGetLastError();
}
MX_EXPORT int mx_frcnn_loss_fwd(const void* logit, const void* delta, const int64_t* label, const float* tgt,
                                const uint8_t* fg, int N, int C, float box_norm, float* partial, float* out,
                                hipStream_t s) {
  const int nb = nblocks_for(N, kLB / 64 * 4);
  hipLaunchKernelGGL(frcnn_fwd_kernel, dim3(nb), dim3(kLB), 0, s, (const uint16_t*)logit, (const uint16_t*)delta, label,
                     tgt, fg, N, C, partial);
  hipLaunchKernelGGL(loss_fin_kernel, dim3(1), dim3(kLB), 0, s, partial, nb, 1, (float)N, box_norm, out);
  return hipGetLastError();
}
MX_EXPORT int mx_frcnn_loss_bwd(const void* logit, const void* delta, const int64_t* label, const float* tgt,
                                const uint8_t* fg, int N, int C, const float* norms, const float* g_cls,
                                const float* g_box, void* dlogit, void* ddelta, hipStream_t s) {
  hipLaunchKernelGGL(frcnn_bwd_kernel, dim3(nblocks_for(N, kLB / 64 * 2)), dim3(kLB), 0, s, (const uint16_t*)logit,
                     (const uint16_t*)delta, label, tgt, fg, N, C, norms, g_cls, g_box, (uint16_t*)dlogit,
                     (uint16_t*)ddelta);
  return hipGetLastError();
}
MX_EXPORT int mx_mask_loss_fwd(const void* logit, const int64_t* label, const float* target, const float* valid, int R,
                               int P, int K, float* partial, float* out, hipStream_t s) {
  const int nb = nblocks_for((long long)R * P, kLB * 8);
  hipLaunchKernelGGL(mask_fwd_kernel, dim3(nb), dim3(kLB), 0, s, (const uint16_t*)logit, label, target, valid, R, P, K,
                     partial);
  hipLaunchKernelGGL(loss_fin_kernel, dim3(1), dim3(kLB), 0, s, partial, nb, 2, 1.f, 1.f, out);
  return hipGetLastError();
}
MX_EXPORT int mx_mask_loss_bwd(const void* logit, const int64_t* label, const float* target, const float* valid, int R,
                               int P, int K, const float* norms, const float* g, void* dlogit, hipStream_t s) {
  if (K % 8) return hipErrorInvalidValue;
  hipLaunchKernelGGL(mask_bwd_kernel, dim3(nblocks_for((long long)R * P * (K / 8), kLB * 4)), dim3(kLB), 0, s,
                     (const uint16_t*)logit, label, target, valid, R, P, K, norms, g, (uint16_t*)dlogit);
  return hipGetLastError();
}
