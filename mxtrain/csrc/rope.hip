// Rotary position embedding (K5), applied IN PLACE to the Q and K column
// blocks of the fused QKV activation [tokens, ld] right after the QKV GEMM, so the
// attention kernel reads already-rotated Q/K and nothing else is materialised.
//
//   rotate-half (GPT-NeoX / LLaMA / Megatron `apply_rotary_pos_emb`), rotary dim rd <= D:
//     x1 = x[i], x2 = x[i + rd/2]           (i < rd/2, per head)
//     fwd:  y1 = x1 cos - x2 sin,  y2 = x2 cos + x1 sin
//     bwd:  the transpose rotation (sin -> -sin) applied to dQ / dK in place.
//
// cos/sin come from an fp32 table [max_pos, rd/2] built once on the host (angles up to
// pos * 1 rad lose precision in __sinf, so the table is computed in fp64 and rounded).
// One thread owns 4 rotation pairs of one head of one token: two 8-B bf16 loads, two
// 16-B table loads, two 8-B stores.  Grid-stride, >> 256 workgroups for real shapes.
#include "common.h"

using namespace mx;

namespace {

typedef __attribute__((ext_vector_type(2))) uint32_t u32x2;

template <bool kInverse>
__global__ __launch_bounds__(256) void rope_kernel(
    uint16_t* __restrict__ x, int64_t ld, int col0, int heads, int head_dim, int rd,
    int ntok, int seq, int pos_offset, const int64_t* __restrict__ pos_ids,
    const float* __restrict__ cos_t, const float* __restrict__ sin_t) {
  const int half = rd >> 1;
  const int qv = half >> 2;  // 4-pair groups per head
  const int64_t total = (int64_t)ntok * heads * qv;
  for (int64_t w = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; w < total;
       w += (int64_t)gridDim.x * blockDim.x) {
    const int g = (int)(w % qv);
    const int64_t th = w / qv;
    const int h = (int)(th % heads);
    const int t = (int)(th / heads);
    const int64_t pos = pos_ids ? pos_ids[t] : (int64_t)(t % seq) + pos_offset;
    const int i = g * 4;
    uint16_t* base = x + (int64_t)t * ld + col0 + (int64_t)h * head_dim;
    u32x2 a = *reinterpret_cast<const u32x2*>(base + i);
    u32x2 b = *reinterpret_cast<const u32x2*>(base + half + i);
    const float4 c = *reinterpret_cast<const float4*>(cos_t + pos * half + i);
    float4 s = *reinterpret_cast<const float4*>(sin_t + pos * half + i);
    if (kInverse) { s.x = -s.x; s.y = -s.y; s.z = -s.z; s.w = -s.w; }
    const float x1[4] = {lo_bf(a.x), hi_bf(a.x), lo_bf(a.y), hi_bf(a.y)};
    const float x2[4] = {lo_bf(b.x), hi_bf(b.x), lo_bf(b.y), hi_bf(b.y)};
    const float cc[4] = {c.x, c.y, c.z, c.w};
    const float ss[4] = {s.x, s.y, s.z, s.w};
    float y1[4], y2[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      y1[j] = x1[j] * cc[j] - x2[j] * ss[j];
      y2[j] = x2[j] * cc[j] + x1[j] * ss[j];
    }
    *reinterpret_cast<u32x2*>(base + i) = (u32x2){pack2(y1[0], y1[1]), pack2(y1[2], y1[3])};
    *reinterpret_cast<u32x2*>(base + half + i) =
        (u32x2){pack2(y2[0], y2[1]), pack2(y2[2], y2[3])};
  }
}

}  // namespace

// x: bf16 [ntok, ld]; the rotated heads start at column col0 (Q block: 0, K block:
// hq*D) and are `heads` consecutive blocks of head_dim columns.  rd % 8 == 0,
// head_dim % 4 == 0, ld % 4 == 0 and col0 % 4 == 0 (8-byte aligned accesses).
// pos_ids (int64 [ntok]) overrides the default position (t % seq) + pos_offset.
MX_EXPORT int mx_rope(void* x, int64_t ld, int col0, int heads, int head_dim, int rd, int ntok,
                      int seq, int pos_offset, const void* pos_ids, const void* cos_t,
                      const void* sin_t, int inverse, hipStream_t stream) {
  if (rd % 8 || rd > head_dim || ld % 4 || col0 % 4 || head_dim % 4) return hipErrorInvalidValue;
  const int64_t total = (int64_t)ntok * heads * (rd / 8);
  if (total == 0) return hipSuccess;
  const int64_t want = (total + 255) / 256;
  const int grid = (int)(want < 8192 ? want : 8192);
  if (inverse)
    hipLaunchKernelGGL(rope_kernel<true>, dim3(grid), dim3(256), 0, stream, (uint16_t*)x, ld, col0,
                       heads, head_dim, rd, ntok, seq, pos_offset, (const int64_t*)pos_ids,
                       (const float*)cos_t, (const float*)sin_t);
  else
    hipLaunchKernelGGL(rope_kernel<false>, dim3(grid), dim3(256), 0, stream, (uint16_t*)x, ld,
                       col0, heads, head_dim, rd, ntok, seq, pos_offset, (const int64_t*)pos_ids,
                       (const float*)cos_t, (const float*)sin_t);
  return hipGetLastError();
}
