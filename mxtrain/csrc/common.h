// mxtrain HIP kernel library -- shared device helpers (gfx950 / CDNA4 only).
//
// Every kernel in csrc/ is exported through a plain C ABI (`extern "C" int mx_*`)
// that takes raw device pointers plus the caller's hipStream_t, and returns the
// hipError_t of the launch.  Python binds these with ctypes (mxtrain/ops/_lib.py);
// there is no torch C++ header in the kernel build, which keeps compiles at a
// few seconds per file and lets the same .so serve the C++ runtime.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#define MX_EXPORT extern "C" __attribute__((visibility("default")))

namespace mx {

constexpr int kWave = 64;  // CDNA wavefront width (never 32)

typedef __attribute__((ext_vector_type(8))) short bf16x8;    // 8 x bf16 = 4 VGPRs
typedef __attribute__((ext_vector_type(4))) short bf16x4;    // 4 x bf16 = 2 VGPRs
typedef __attribute__((ext_vector_type(16))) float f32x16;   // 32x32 MFMA accumulator
typedef __attribute__((ext_vector_type(4))) float f32x4;     // 16x16 MFMA accumulator

__device__ __forceinline__ float bf2f(uint16_t u) {
  return __uint_as_float(((uint32_t)u) << 16);
}
// round-to-nearest-even; hipcc lowers this to v_cvt_pk_bf16_f32 on gfx950 (NaN stays NaN)
__device__ __forceinline__ uint16_t f2bf(float f) {
  __bf16 b = (__bf16)f;
  return __builtin_bit_cast(uint16_t, b);
}
typedef float f32x2_t __attribute__((ext_vector_type(2)));
typedef __bf16 bf16x2_t __attribute__((ext_vector_type(2)));
// two floats -> packed bf16 pair in ONE v_cvt_pk_bf16_f32 (a per-element cast + shift/or
// costs three VALU ops per pair)
__device__ __forceinline__ uint32_t pack2(float lo, float hi) {
  return __builtin_bit_cast(uint32_t, __builtin_convertvector((f32x2_t){lo, hi}, bf16x2_t));
}
// reductions across the two 32-lane halves of a wave (lane l <-> l^32) with one
// v_permlane32_swap instead of ds_bpermute + address arithmetic
__device__ __forceinline__ float xhalf_max(float x) {
  auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(x), __float_as_uint(x), false, false);
  return fmaxf(__uint_as_float(r[0]), __uint_as_float(r[1]));
}
__device__ __forceinline__ float xhalf_sum(float x) {
  auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(x), __float_as_uint(x), false, false);
  return __uint_as_float(r[0]) + __uint_as_float(r[1]);
}
__device__ __forceinline__ float lo_bf(uint32_t w) { return __uint_as_float(w << 16); }
__device__ __forceinline__ float hi_bf(uint32_t w) { return __uint_as_float(w & 0xffff0000u); }

// unpack 8 bf16 held in a uint4 (16 B) into floats
__device__ __forceinline__ void unpack8(const uint4& v, float* f) {
  f[0] = lo_bf(v.x); f[1] = hi_bf(v.x);
  f[2] = lo_bf(v.y); f[3] = hi_bf(v.y);
  f[4] = lo_bf(v.z); f[5] = hi_bf(v.z);
  f[6] = lo_bf(v.w); f[7] = hi_bf(v.w);
}
__device__ __forceinline__ uint4 pack8(const float* f) {
  uint4 v;
  v.x = pack2(f[0], f[1]); v.y = pack2(f[2], f[3]);
  v.z = pack2(f[4], f[5]); v.w = pack2(f[6], f[7]);
  return v;
}

// Full-wave reductions without the LDS pipe: DPP quad permutes and 16-lane row
// rotations, then v_permlane16_swap / v_permlane32_swap for the cross-row steps.
// (__shfl_xor lowers to a chain of 6 dependent ds_bpermute round trips, which made the
// norm kernels latency-bound: SQ_WAIT_INST_LDS dominated their wave cycles.)
#define MX_DPP(v, ctrl) \
  __uint_as_float(__builtin_amdgcn_update_dpp(0u, __float_as_uint(v), (ctrl), 0xf, 0xf, false))
// sum over the 16 lanes of each row (every lane of the row ends with it)
__device__ __forceinline__ float row_sum16(float v) {
  v += MX_DPP(v, 0xB1);   // quad_perm [1,0,3,2]
  v += MX_DPP(v, 0x4E);   // quad_perm [2,3,0,1]
  v += MX_DPP(v, 0x124);  // row_ror:4
  v += MX_DPP(v, 0x128);  // row_ror:8
  return v;
}
__device__ __forceinline__ float wave_sum(float v) {
  v += MX_DPP(v, 0xB1);   // quad_perm [1,0,3,2]
  v += MX_DPP(v, 0x4E);   // quad_perm [2,3,0,1]
  v += MX_DPP(v, 0x124);  // row_ror:4
  v += MX_DPP(v, 0x128);  // row_ror:8   -> every lane holds its 16-lane row sum
  auto r = __builtin_amdgcn_permlane16_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  v = __uint_as_float(r[0]) + __uint_as_float(r[1]);
  auto q = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  return __uint_as_float(q[0]) + __uint_as_float(q[1]);
}
__device__ __forceinline__ float wave_max(float v) {
  v = fmaxf(v, MX_DPP(v, 0xB1));
  v = fmaxf(v, MX_DPP(v, 0x4E));
  v = fmaxf(v, MX_DPP(v, 0x124));
  v = fmaxf(v, MX_DPP(v, 0x128));
  auto r = __builtin_amdgcn_permlane16_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  v = fmaxf(__uint_as_float(r[0]), __uint_as_float(r[1]));
  auto q = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  return fmaxf(__uint_as_float(q[0]), __uint_as_float(q[1]));
}

// Counter-based RNG for dropout: a stateless 32-bit hash of (seed, element index).
// The mask is regenerated bit-exactly in backward from the same (seed, offset), so
// nothing but the seed is saved between forward and backward.
__device__ __forceinline__ uint32_t hash32(uint32_t x, uint32_t seed) {
  x ^= seed * 0x9E3779B9u;
  x ^= x >> 16; x *= 0x7feb352du;
  x ^= x >> 15; x *= 0x846ca68bu;
  x ^= x >> 16;
  return x;
}
// Keep flags of the 8 elements idx0 .. idx0 + 7 (idx0 % 8 == 0), thresh = p * 2^32 (> 0).
// ONE hash per 8-element group seeds an xorshift32 stream: x0 = hash32(group ^ hi, seed) | 1
// (never the all-zero fixed point), x_{j+1} = xorshift(x_j); x_j's low / high 16 bits are the
// draws of elements 2j / 2j + 1, kept when >= round(p * 2^16).  (8 full hashes per group --
// 16 quarter-rate multiplies -- made the LN backward VALU-bound; ops/rng.py keep_mask is the
// bit-identical reference.)
__device__ __forceinline__ void dropout_keep8(uint64_t idx0, uint32_t seed, uint32_t thresh, bool (&k)[8]) {
  const uint32_t g = (uint32_t)(idx0 >> 3) ^ (uint32_t)(idx0 >> 35) * 0x85ebca6bu;
  const uint32_t thr = (uint32_t)(((uint64_t)thresh + 0x8000u) >> 16);
  uint32_t x = hash32(g, seed) | 1u;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    if (j) { x ^= x << 13; x ^= x >> 17; x ^= x << 5; }
    k[2 * j] = (x & 0xFFFFu) >= thr;
    k[2 * j + 1] = (x >> 16) >= thr;
  }
}

// tanh-approximation GeLU (Megatron bias_gelu / HF "gelu_new") in its sigmoid form:
//   0.5 x (1 + tanh(u)) = x s,  s = sigmoid(2u) = 1 / (1 + 2^(x (A + B x^2))),
//   u = k0 x (1 + k1 x^2),  A = -2 k0 log2(e),  B = A k1
// (one v_exp + one v_rcp and 5 VALU ops per element: the tanh form took ~12 and made the
// GeLU kernels VALU-bound).  Saturates: x -> -inf gives -0, x -> +inf gives x.
constexpr float kGeluA = -2.f * 0.7978845608028654f * 1.4426950408889634f;
constexpr float kGeluB = kGeluA * 0.044715f;
__device__ __forceinline__ float gelu_sig(float x, float x2) {
  return __builtin_amdgcn_rcpf(1.f + __builtin_amdgcn_exp2f(x * __builtin_fmaf(kGeluB, x2, kGeluA)));
}
__device__ __forceinline__ float gelu_tanh(float x) { return x * gelu_sig(x, x * x); }
// d/dx = s + x s (1 - s) 2 k0 (1 + 3 k1 x^2) = s (1 + x (1 - s) (C1 + C2 x^2))
__device__ __forceinline__ float gelu_tanh_grad(float x) {
  constexpr float C1 = 2.f * 0.7978845608028654f, C2 = 3.f * 0.044715f * C1;
  const float x2 = x * x;
  const float s = gelu_sig(x, x2);
  return s * __builtin_fmaf(x * (1.f - s), __builtin_fmaf(C2, x2, C1), 1.f);
}

// bijective XCD-aware remap of a 1-D block id (cdna_hip_programming.md §5 "XCD swizzle
// must be bijective"): blocks that share an XCD (orig % 8) get contiguous logical ids.
__device__ __forceinline__ int xcd_remap(int orig, int nwg) {
  const int nx = 8;
  int q = nwg / nx, r = nwg % nx, x = orig % nx;
  int base = (x < r) ? x * (q + 1) : r * (q + 1) + (x - r) * q;
  return base + orig / nx;
}

}  // namespace mx
