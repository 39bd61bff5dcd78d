// 3x3 / stride-2 / pad-1 max-pool of an NHWC bf16 tensor -- the ResNet-50 stem's pool0
// (BASELINE config 5: conv -> BN -> ReLU -> max-pool at 112 x 112 x 64 per image).
//
// torch's NHWC max-pool saves an int64 index per output element and its backward scatters:
// 250 + 632 us per step at batch 256 (profiles/r6/resnet50_census_final_tree.txt), against
// ~110 us each for the bytes that have to move.  Here the forward stores the argmax as one
// byte per output element (its position 0..8 in the window) and the backward GATHERS: every
// input pixel visits the <= 2 x 2 windows that contain it and adds the gradients of those
// whose argmax is that pixel, in a fixed order (deterministic, no atomics, no zero fill).
// Ties keep the first maximum in window order, as torch (strict >); padding never wins.
// One thread per 8 channels of a pixel: 16-B loads / stores, 8-B argmax words.
#include "common.h"

using namespace mx;

namespace {

constexpr int kThreads = 256;

__global__ __launch_bounds__(kThreads) void maxpool3s2_fwd_kernel(const uint16_t* __restrict__ x,
                                                                  uint16_t* __restrict__ y, uint8_t* __restrict__ arg,
                                                                  int N, int H, int W, int C, int OH, int OW,
                                                                  const float* __restrict__ bn_scale,
                                                                  const float* __restrict__ bn_shift) {
  // one workgroup per output row (n, oh): 32-bit index math only (the 64-bit divisions of a
  // flat index cost more VALU time than the pass's memory traffic)
  const int c8 = C / 8;
  const int n = blockIdx.x / OH, oh = blockIdx.x - (blockIdx.x / OH) * OH;
  for (int e = threadIdx.x; e < OW * c8; e += kThreads) {
    const int ow = e / c8, cv = e - (e / c8) * c8;
    // (bn_scale: the input is a BN's raw input, relu(x scale + shift) applied on load -- the
    // stem's BN + ReLU output tensor is never written)
    float sc[8], sh[8];
    if (bn_scale) {
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        sc[j] = bn_scale[8 * cv + j];
        sh[j] = bn_shift[8 * cv + j];
      }
    }
    float m[8];
    uint32_t idx[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      m[j] = -INFINITY;
      idx[j] = 0u;
    }
#pragma unroll
    for (int kh = 0; kh < 3; ++kh) {
      const int ih = 2 * oh - 1 + kh;
      if ((unsigned)ih >= (unsigned)H) continue;
#pragma unroll
      for (int kw = 0; kw < 3; ++kw) {
        const int iw = 2 * ow - 1 + kw;
        if ((unsigned)iw >= (unsigned)W) continue;
        float f[8];
        unpack8(reinterpret_cast<const uint4*>(x + (((size_t)n * H + ih) * W + iw) * C)[cv], f);
        if (bn_scale) {   // (rounded to bf16 as the separate BN pass would store it)
#pragma unroll
          for (int j = 0; j < 8; ++j) f[j] = bf2f(f2bf(fmaxf(__builtin_fmaf(f[j], sc[j], sh[j]), 0.f)));
        }
#pragma unroll
        for (int j = 0; j < 8; ++j)
          if (f[j] > m[j] || f[j] != f[j]) {   // (NaN propagates, as torch)
            m[j] = f[j];
            idx[j] = (uint32_t)(kh * 3 + kw);
          }
      }
    }
    const size_t o = (((size_t)n * OH + oh) * OW + ow) * C + 8 * cv;
    *reinterpret_cast<uint4*>(y + o) = pack8(m);
    uint2 a;
    a.x = idx[0] | (idx[1] << 8) | (idx[2] << 16) | (idx[3] << 24);
    a.y = idx[4] | (idx[5] << 8) | (idx[6] << 16) | (idx[7] << 24);
    *reinterpret_cast<uint2*>(arg + o) = a;
  }
}

__global__ __launch_bounds__(kThreads) void maxpool3s2_bwd_kernel(const uint16_t* __restrict__ dy,
                                                                  const uint8_t* __restrict__ arg,
                                                                  uint16_t* __restrict__ dx, int N, int H, int W,
                                                                  int C, int OH, int OW,
                                                                  const uint16_t* __restrict__ ypool) {
  const int c8 = C / 8;
  const int n = blockIdx.x / H, h = blockIdx.x - (blockIdx.x / H) * H;   // one input row per workgroup
  for (int e = threadIdx.x; e < W * c8; e += kThreads) {
    const int w = e / c8, cv = e - (e / c8) * c8;
    float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    // the windows containing row h: oh in {(h + 1) / 2 - 1, (h + 1) / 2} with kh = h - 2 oh + 1 in [0, 2]
#pragma unroll
    for (int a = 0; a < 2; ++a) {
      const int oh = (h + 1) / 2 - 1 + a;
      const int kh = h - 2 * oh + 1;
      if ((unsigned)oh >= (unsigned)OH || (unsigned)kh > 2u) continue;
#pragma unroll
      for (int b = 0; b < 2; ++b) {
        const int ow = (w + 1) / 2 - 1 + b;
        const int kw = w - 2 * ow + 1;
        if ((unsigned)ow >= (unsigned)OW || (unsigned)kw > 2u) continue;
        const size_t o = (((size_t)n * OH + oh) * OW + ow) * C + 8 * cv;
        const uint2 am = *reinterpret_cast<const uint2*>(arg + o);
        const uint32_t me = (uint32_t)(kh * 3 + kw);
        float g[8];
        unpack8(*reinterpret_cast<const uint4*>(dy + o), g);
        if (ypool) {   // the fused ReLU's gradient: zero where the window's max (the ReLU output) is 0
          float yv[8];
          unpack8(*reinterpret_cast<const uint4*>(ypool + o), yv);
#pragma unroll
          for (int j = 0; j < 8; ++j) g[j] = yv[j] > 0.f ? g[j] : 0.f;
        }
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const uint32_t aj = ((j < 4 ? am.x : am.y) >> (8 * (j & 3))) & 0xffu;
          if (aj == me) acc[j] += g[j];
        }
      }
    }
    *reinterpret_cast<uint4*>(dx + (((size_t)n * H + h) * W + w) * C + 8 * cv) = pack8(acc);
  }
}

}  // namespace

// x [N][H][W][C] -> y [N][OH][OW][C] (+ argmax bytes [N][OH][OW][C]); OH = (H - 1) / 2 + 1
MX_EXPORT int mx_maxpool3s2_fwd(const void* x, void* y, void* arg, int N, int H, int W, int C, hipStream_t s) {
  if (N <= 0 || H <= 0 || W <= 0 || C <= 0 || C % 8) return hipErrorInvalidValue;
  const int OH = (H - 1) / 2 + 1, OW = (W - 1) / 2 + 1;
  if ((int64_t)N * OH >= ((int64_t)1 << 31) || (int64_t)OW * (C / 8) >= ((int64_t)1 << 31)) return hipErrorInvalidValue;
  hipLaunchKernelGGL(maxpool3s2_fwd_kernel, dim3((unsigned)(N * OH)), dim3(kThreads), 0, s,
                     (const uint16_t*)x, (uint16_t*)y, (uint8_t*)arg, N, H, W, C, OH, OW, nullptr, nullptr);
  return hipGetLastError();
}

// the same pool of relu(x scale[c] + shift[c]) (fp32 [C] each): a training BN + ReLU folded in
MX_EXPORT int mx_maxpool3s2_fwd_bn(const void* x, void* y, void* arg, int N, int H, int W, int C, const float* scale,
                                   const float* shift, hipStream_t s) {
  if (N <= 0 || H <= 0 || W <= 0 || C <= 0 || C % 8 || !scale || !shift) return hipErrorInvalidValue;
  const int OH = (H - 1) / 2 + 1, OW = (W - 1) / 2 + 1;
  if ((int64_t)N * OH >= ((int64_t)1 << 31) || (int64_t)OW * (C / 8) >= ((int64_t)1 << 31)) return hipErrorInvalidValue;
  hipLaunchKernelGGL(maxpool3s2_fwd_kernel, dim3((unsigned)(N * OH)), dim3(kThreads), 0, s, (const uint16_t*)x,
                     (uint16_t*)y, (uint8_t*)arg, N, H, W, C, OH, OW, scale, shift);
  return hipGetLastError();
}

// dy [N][OH][OW][C] + argmax -> dx [N][H][W][C] (every element written)
MX_EXPORT int mx_maxpool3s2_bwd(const void* dy, const void* arg, void* dx, int N, int H, int W, int C, hipStream_t s) {
  if (N <= 0 || H <= 0 || W <= 0 || C <= 0 || C % 8) return hipErrorInvalidValue;
  const int OH = (H - 1) / 2 + 1, OW = (W - 1) / 2 + 1;
  if ((int64_t)N * H >= ((int64_t)1 << 31) || (int64_t)W * (C / 8) >= ((int64_t)1 << 31)) return hipErrorInvalidValue;
  hipLaunchKernelGGL(maxpool3s2_bwd_kernel, dim3((unsigned)(N * H)), dim3(kThreads), 0, s,
                     (const uint16_t*)dy, (const uint8_t*)arg, (uint16_t*)dx, N, H, W, C, OH, OW, nullptr);
  return hipGetLastError();
}

// the backward through mx_maxpool3s2_fwd_bn's ReLU as well: ypool = its output
MX_EXPORT int mx_maxpool3s2_bwd_relu(const void* dy, const void* arg, const void* ypool, void* dx, int N, int H,
                                     int W, int C, hipStream_t s) {
  if (N <= 0 || H <= 0 || W <= 0 || C <= 0 || C % 8 || !ypool) return hipErrorInvalidValue;
  const int OH = (H - 1) / 2 + 1, OW = (W - 1) / 2 + 1;
  if ((int64_t)N * H >= ((int64_t)1 << 31) || (int64_t)W * (C / 8) >= ((int64_t)1 << 31)) return hipErrorInvalidValue;
  hipLaunchKernelGGL(maxpool3s2_bwd_kernel, dim3((unsigned)(N * H)), dim3(kThreads), 0, s, (const uint16_t*)dy,
                     (const uint8_t*)arg, (uint16_t*)dx, N, H, W, C, OH, OW, (const uint16_t*)ypool);
  return hipGetLastError();
}

// ------------------------------------------------------------------- global average pool
// mean over H x W of an NHWC bf16 tensor into fp32 [N][C] (the classifier head's pool: torch
// spends a bf16 -> fp32 copy, a reduction and, backward, an expand + strided bf16 cast --
// ~160 us per ResNet-50 step at batch 256); backward broadcasts g / (H W) into bf16 NHWC.
namespace {
__global__ __launch_bounds__(256) void gap_fwd_kernel(const uint16_t* __restrict__ x, float* __restrict__ y, int N,
                                                      int HW, int C) {
  const int c8 = C / 8;
  const int64_t v = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (v >= (int64_t)N * c8) return;
  const int n = (int)(v / c8), cv = (int)(v % c8);
  float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  const uint4* src = reinterpret_cast<const uint4*>(x + (size_t)n * HW * C) + cv;
#pragma unroll 7
  for (int p = 0; p < HW; ++p) {
    float f[8];
    unpack8(src[(size_t)p * c8], f);
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[j] += f[j];
  }
  const float inv = 1.f / (float)HW;
  float4* dst = reinterpret_cast<float4*>(y + (size_t)n * C + 8 * cv);
  dst[0] = make_float4(acc[0] * inv, acc[1] * inv, acc[2] * inv, acc[3] * inv);
  dst[1] = make_float4(acc[4] * inv, acc[5] * inv, acc[6] * inv, acc[7] * inv);
}

__global__ __launch_bounds__(256) void gap_bwd_kernel(const float* __restrict__ g, uint16_t* __restrict__ dx, int N,
                                                      int HW, int C) {
  const int c8 = C / 8;
  const float inv = 1.f / (float)HW;
  const int n = blockIdx.x;   // image n, a 1 / gridDim.y share of its pixels
  uint4* dst = reinterpret_cast<uint4*>(dx) + (size_t)n * HW * c8;
  for (int e = blockIdx.y * 256 + threadIdx.x; e < HW * c8; e += 256 * gridDim.y) {
    const int cv = e % c8;
    const float4* s = reinterpret_cast<const float4*>(g + (size_t)n * C + 8 * cv);
    const float4 a = s[0], b = s[1];
    const float f[8] = {a.x * inv, a.y * inv, a.z * inv, a.w * inv, b.x * inv, b.y * inv, b.z * inv, b.w * inv};
    dst[e] = pack8(f);
  }
}
}  // namespace

MX_EXPORT int mx_gap_fwd(const void* x, float* y, int N, int HW, int C, hipStream_t s) {
  if (N <= 0 || HW <= 0 || C <= 0 || C % 8) return hipErrorInvalidValue;
  const int64_t t = (int64_t)N * (C / 8);
  hipLaunchKernelGGL(gap_fwd_kernel, dim3((unsigned)((t + 255) / 256)), dim3(256), 0, s, (const uint16_t*)x, y, N,
                     HW, C);
  return hipGetLastError();
}

MX_EXPORT int mx_gap_bwd(const float* g, void* dx, int N, int HW, int C, hipStream_t s) {
  if (N <= 0 || HW <= 0 || C <= 0 || C % 8) return hipErrorInvalidValue;
  if ((int64_t)HW * (C / 8) >= ((int64_t)1 << 31)) return hipErrorInvalidValue;
  hipLaunchKernelGGL(gap_bwd_kernel, dim3((unsigned)N, 8), dim3(256), 0, s, g,
                     (uint16_t*)dx, N, HW, C);
  return hipGetLastError();
}
