// Multi-tensor dtype casts in one launch: the bf16 compute copies of a model's fp32 weights
// (forward) and the fp32 gradients of those weights from the bf16 ones (backward) --
// models/compute_weights.py CastGroup.  Autocast casts each weight separately, and its
// backward each gradient: 59 + 58 launches of 3-8 us per ResNet-50 step
// (profiles/r6/resnet50_census_final_tree.txt) for ~50 MB each way.
//
// Each job is a dense tensor pair with the SAME memory order (equal strides), cast element
// by element in memory order; lengths are multiples of 8 and addresses 16-byte aligned, so a
// thread converts 8 elements with 16/32-byte accesses.  The job list travels by value in the
// kernel arguments (hipGraph-capturable: no descriptor buffer to keep alive).
#include "common.h"

using namespace mx;

namespace {

constexpr int kMaxJobs = 96;

struct CastJob {
  const void* src;
  void* dst;
  int64_t v0;   // first 8-element vector of this job in the launch's flat vector space
};
struct CastJobs {
  CastJob j[kMaxJobs];
};

template <bool TO_BF16>
__global__ __launch_bounds__(256) void cast_multi_kernel(const CastJobs js, int njobs, int64_t nvec) {
  for (int64_t v = (int64_t)blockIdx.x * 256 + threadIdx.x; v < nvec; v += (int64_t)gridDim.x * 256) {
    int lo = 0, hi = njobs - 1;   // the job holding vector v (binary search over v0)
    while (lo < hi) {
      const int mid = (lo + hi + 1) >> 1;
      if (js.j[mid].v0 <= v) lo = mid;
      else hi = mid - 1;
    }
    const CastJob& J = js.j[lo];
    const int64_t e = v - J.v0;
    if constexpr (TO_BF16) {
      const float4* s = reinterpret_cast<const float4*>(J.src) + 2 * e;
      const float4 a = s[0], b = s[1];
      const float f[8] = {a.x, a.y, a.z, a.w, b.x, b.y, b.z, b.w};
      reinterpret_cast<uint4*>(J.dst)[e] = pack8(f);
    } else {
      float f[8];
      unpack8(reinterpret_cast<const uint4*>(J.src)[e], f);
      float4* d = reinterpret_cast<float4*>(J.dst) + 2 * e;
      d[0] = make_float4(f[0], f[1], f[2], f[3]);
      d[1] = make_float4(f[4], f[5], f[6], f[7]);
    }
  }
}

}  // namespace

// d (int64[3 * njobs]): {src, dst, numel} per job; to_bf16: fp32 -> bf16, else bf16 -> fp32
MX_EXPORT int mx_cast_multi(const int64_t* d, int njobs, int to_bf16, hipStream_t s) {
  if (njobs <= 0 || njobs > kMaxJobs) return hipErrorInvalidValue;
  CastJobs js{};
  int64_t nvec = 0;
  for (int i = 0; i < njobs; ++i) {
    const int64_t n = d[3 * i + 2];
    if (n <= 0 || n % 8 || (d[3 * i] & 15) || (d[3 * i + 1] & 15)) return hipErrorInvalidValue;
    js.j[i].src = reinterpret_cast<const void*>(d[3 * i]);
    js.j[i].dst = reinterpret_cast<void*>(d[3 * i + 1]);
    js.j[i].v0 = nvec;
    nvec += n / 8;
  }
  int64_t g = (nvec + 255) / 256;
  if (g > 4096) g = 4096;
  if (to_bf16)
    hipLaunchKernelGGL(cast_multi_kernel<true>, dim3((unsigned)g), dim3(256), 0, s, js, njobs, nvec);
  else
    hipLaunchKernelGGL(cast_multi_kernel<false>, dim3((unsigned)g), dim3(256), 0, s, js, njobs, nvec);
  return hipGetLastError();
}
