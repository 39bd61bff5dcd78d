// Convolution epilogues for the NHWC (channels_last) bf16 CNN workloads (Mask R-CNN
// backbone / FPN / RPN / mask head): MIOpen runs the convolution WITHOUT its
// bias, and one pass applies bias (+ residual) (+ ReLU) in place.  PyTorch's own path for
// a channels_last conv with bias is conv -> broadcast add (a non-vectorised elementwise
// kernel) -> clamp (ReLU) [-> add residual -> clamp]: 2-4 extra passes over the
// activation and as many launches.  The backward pass fuses the ReLU mask with the bias
// gradient's column partial sums (one read of the incoming gradient), folded by the
// deterministic colreduce_kernel (norm.hip).
//
// Layout: [M, C] with M = N*H*W rows (NHWC memory), C % 8 == 0; 16-byte vectors (8 bf16),
// lane-contiguous, so every load/store is a full 16 B per lane.
#include "common.h"

using namespace mx;

namespace {

// y = act(y + b (+ res)) in place; one thread per 8-channel vector
template <bool kRes, bool kRelu>
__global__ __launch_bounds__(256) void bias_act_fwd_kernel(uint16_t* __restrict__ y, const uint16_t* __restrict__ b,
                                                           const uint16_t* __restrict__ res, int64_t nvec, int c8) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t v = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; v < nvec; v += stride) {
    float x[8], bb[8];
    unpack8(reinterpret_cast<const uint4*>(y)[v], x);
    if (b) {
      // bias vector of this 8-channel slot (a mask index for power-of-two channel counts was
      // A/B'd on Mask R-CNN in round 2 and measured no faster, so it was removed)
      unpack8(reinterpret_cast<const uint4*>(b)[(int)(v % c8)], bb);
#pragma unroll
      for (int j = 0; j < 8; ++j) x[j] += bb[j];
    }
    if (kRes) {
      float r[8];
      unpack8(reinterpret_cast<const uint4*>(res)[v], r);
#pragma unroll
      for (int j = 0; j < 8; ++j) x[j] += r[j];
    }
    if (kRelu) {
#pragma unroll
      for (int j = 0; j < 8; ++j) x[j] = fmaxf(x[j], 0.f);
    }
    reinterpret_cast<uint4*>(y)[v] = pack8(x);
  }
}

// dy = relu ? g * (out > 0) : g, and (kDb) partial[blockIdx.y][C] = column sums of dy over
// the block's row stripe.  Block: 256 threads = (256 / c8) rows x c8 vectors of a row.
template <bool kRelu, bool kDb>
__global__ __launch_bounds__(256) void bias_act_bwd_kernel(const uint16_t* __restrict__ g,
                                                           const uint16_t* __restrict__ out,
                                                           uint16_t* __restrict__ dy, float* __restrict__ partial,
                                                           int M, int C, int rows_per_block) {
  const int c8 = C / 8;
  const int rpi = blockDim.x / c8;               // rows per iteration
  const int tr = threadIdx.x / c8, tv = threadIdx.x % c8;
  const int r0 = blockIdx.x * rows_per_block;
  const int r1 = min(M, r0 + rows_per_block);
  float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  if (tr < rpi) {
    for (int r = r0 + tr; r < r1; r += rpi) {
      const int64_t v = (int64_t)r * c8 + tv;
      float x[8];
      unpack8(reinterpret_cast<const uint4*>(g)[v], x);
      if (kRelu) {
        const uint4 o = reinterpret_cast<const uint4*>(out)[v];
        const uint32_t w[4] = {o.x, o.y, o.z, o.w};
#pragma unroll
        for (int j = 0; j < 4; ++j) {   // bf16 > 0 <=> sign bit clear and nonzero
          const uint32_t lo = w[j] & 0xffffu, hi = w[j] >> 16;
          if (!(lo != 0u && !(lo & 0x8000u))) x[2 * j] = 0.f;
          if (!(hi != 0u && !(hi & 0x8000u))) x[2 * j + 1] = 0.f;
        }
        reinterpret_cast<uint4*>(dy)[v] = pack8(x);
      }
      if (kDb) {
#pragma unroll
        for (int j = 0; j < 8; ++j) acc[j] += x[j];
      }
    }
  }
  if (!kDb) return;
  // fold the rpi row-groups of the block in LDS (fixed order -> deterministic)
  __shared__ float red[256][9];
#pragma unroll
  for (int j = 0; j < 8; ++j) red[threadIdx.x][j] = acc[j];
  __syncthreads();
  if (tr == 0) {
    for (int k = 1; k < rpi; ++k)
#pragma unroll
      for (int j = 0; j < 8; ++j) acc[j] += red[k * c8 + tv][j];
    float* p = partial + (size_t)blockIdx.x * C + tv * 8;
#pragma unroll
    for (int j = 0; j < 8; ++j) p[j] = acc[j];
  }
}

// Gradient of a 2x nearest upsampling (NHWC): out[n][y][x][c] = sum of g over the 2 x 2 block
// at (2y, 2x) (+ add[n][y][x][c]) -- fp32 sum, one bf16 rounding.  The FPN top-down join's
// residual gradient, with the joined level's other gradient folded in (ops/epilogue.py
// JoinLink); thread = 8 channels of one output pixel, 16-B loads / store.
__global__ __launch_bounds__(256) void down2_add_kernel(const uint16_t* __restrict__ g, const uint16_t* __restrict__ add,
                                                        uint16_t* __restrict__ out, int N, int H, int W, int C) {
  const int C8 = C >> 3;
  const int64_t total = (int64_t)N * H * W * C8;
  for (int64_t q = (int64_t)blockIdx.x * 256 + threadIdx.x; q < total; q += (int64_t)gridDim.x * 256) {
    const int c = (int)(q % C8) * 8;
    const int64_t pix = q / C8;
    const int x = (int)(pix % W);
    const int64_t ny = pix / W;
    const int y = (int)(ny % H);
    const int n = (int)(ny / H);
    const size_t r0 = (((size_t)n * 2 * H + 2 * y) * 2 * W + 2 * x) * C + c;
    const size_t r1 = r0 + (size_t)2 * W * C;
    float a[8], b[8], d[8], e[8];
    unpack8(*reinterpret_cast<const uint4*>(g + r0), a);
    unpack8(*reinterpret_cast<const uint4*>(g + r0 + C), b);
    unpack8(*reinterpret_cast<const uint4*>(g + r1), d);
    unpack8(*reinterpret_cast<const uint4*>(g + r1 + C), e);
    float o[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) o[j] = (a[j] + b[j]) + (d[j] + e[j]);
    const size_t op = (size_t)pix * C + c;
    if (add) {
      float f[8];
      unpack8(*reinterpret_cast<const uint4*>(add + op), f);
#pragma unroll
      for (int j = 0; j < 8; ++j) o[j] += f[j];
    }
    *reinterpret_cast<uint4*>(out + op) = pack8(o);
  }
}

// Deferred bias-gradient column sums of a backward (ops/convwg.py defer_flush): job j folds
// its fp32 partial rows [nparts][C] into the bf16 vector out[C] (written, or added to);
// a block = 16 columns of one job, thread t sums column t & 15 over the rows t >> 4,
// (t >> 4) + 16, ... (eight loads in flight), the 16 row-phase sums folded in LDS in a fixed
// order (deterministic).  The job list travels by value.
constexpr int kCsJobs = 64;
struct CsJob {
  const float* part;
  uint16_t* out;
  int nparts, C, acc, b0;
};
struct CsJobs {
  CsJob j[kCsJobs];
};
__global__ __launch_bounds__(256) void colsum_jobs_kernel(const CsJobs js, int njobs) {
  __shared__ float red[16][17];
  const int b = blockIdx.x;
  int q = 0;
  while (q + 1 < njobs && js.j[q + 1].b0 <= b) ++q;
  const CsJob& J = js.j[q];
  const int t = threadIdx.x, ci = t & 15, ph = t >> 4;
  const int c = (b - J.b0) * 16 + ci;
  float s = 0.f;
  if (c < J.C) {
    int r = ph;
    for (; r + 7 * 16 < J.nparts; r += 8 * 16) {
      float v[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) v[u] = J.part[(size_t)(r + 16 * u) * J.C + c];
#pragma unroll
      for (int u = 0; u < 8; ++u) s += v[u];
    }
    for (; r < J.nparts; r += 16) s += J.part[(size_t)r * J.C + c];
  }
  red[ph][ci] = s;
  __syncthreads();
  if (t < 16 && (b - J.b0) * 16 + t < J.C) {
    float tot = 0.f;
#pragma unroll
    for (int p = 0; p < 16; ++p) tot += red[p][t];
    uint16_t* o = J.out + (b - J.b0) * 16 + t;
    if (J.acc) tot += bf2f(*o);
    *o = f2bf(tot);
  }
}

}  // namespace

// colreduce (norm.hip): fold fp32 partials [P][C] into a bf16 vector
extern "C" int mx_colsum_finalize(const float* partial, int nparts, int cols, int nvec, void* o0, void* o1,
                                  void* o2, int accumulate, float* scratch, hipStream_t s);

// y [M, C] bf16 in place: y = act(y + b (+ res)); b may be null (no bias)
MX_EXPORT int mx_bias_act_fwd(void* y, const void* b, const void* res, int64_t M, int C, int relu, hipStream_t s) {
  if (C % 8 || C > 2048) return hipErrorInvalidValue;
  const int64_t nvec = M * (C / 8);
  if (nvec == 0) return hipSuccess;
  const int64_t want = (nvec + 255) / 256;
  const unsigned grid = (unsigned)(want < 8192 ? want : 8192);
#define MX_BA(R, A)                                                                                        \
  hipLaunchKernelGGL((bias_act_fwd_kernel<R, A>), dim3(grid), dim3(256), 0, s, (uint16_t*)y, (const uint16_t*)b, \
                     (const uint16_t*)res, nvec, C / 8)
  if (res) {
    if (relu) MX_BA(true, true); else MX_BA(true, false);
  } else {
    if (relu) MX_BA(false, true); else MX_BA(false, false);
  }
#undef MX_BA
  return hipGetLastError();
}

// rows of the bias-gradient partial stripes (one per workgroup)
// Row stripe per workgroup: 128 rows, fewer when that leaves the chip under-filled (about
// 1024 workgroups; a 1-img res3 output, M = 16800, had 132 stripes on 256 CUs: 30 us for 52 MB)
static int bwd_rows_per_block(int64_t M) {
  const int64_t r = (M + 1023) / 1024;
  return (int)(r < 8 ? 8 : (r > 128 ? 128 : r));
}
MX_EXPORT int mx_bias_act_bwd_parts(int64_t M, int C) {
  (void)C;
  const int rpb = bwd_rows_per_block(M);
  return (int)((M + rpb - 1) / rpb);
}

// dy = relu ? g * (out > 0) : g (dy may alias g); db (bf16 [C], optional) (+)= column sums
// of dy; partial: mx_bias_act_bwd_parts(M, C) * C floats.  C <= 2048, C % 8 == 0.
MX_EXPORT int mx_bias_act_bwd(const void* g, const void* out, void* dy, void* db, float* partial, int64_t M, int C,
                              int relu, int accumulate, hipStream_t s) {
  if (C % 8 || C > 2048 || (!relu && !db)) return hipErrorInvalidValue;
  if (M == 0) return hipSuccess;
  const int rpb = bwd_rows_per_block(M);
  const int nparts = mx_bias_act_bwd_parts(M, C);
#define MX_BB(R, D)                                                                                       \
  hipLaunchKernelGGL((bias_act_bwd_kernel<R, D>), dim3(nparts), dim3(256), 0, s, (const uint16_t*)g,            \
                     (const uint16_t*)out, (uint16_t*)dy, partial, (int)M, C, rpb)
  if (relu) {
    if (db) MX_BB(true, true); else MX_BB(true, false);
  } else {
    MX_BB(false, true);
  }
#undef MX_BB
  // accumulate bit 1: the caller folds the partials later (mx_colsum_jobs)
  if (db && !(accumulate & 2))
    return mx_colsum_finalize(partial, nparts, C, 1, db, nullptr, nullptr, accumulate & 1, nullptr, s);
  return hipGetLastError();
}

// jobs: host int64 [njobs][5] {partial, out, nparts, C, accumulate}; kCsJobs per launch
MX_EXPORT int mx_colsum_jobs(const int64_t* jobs, int njobs, hipStream_t s) {
  for (int j0 = 0; j0 < njobs; j0 += kCsJobs) {
    const int nj = njobs - j0 < kCsJobs ? njobs - j0 : kCsJobs;
    CsJobs js{};
    int blocks = 0;
    for (int q = 0; q < nj; ++q) {
      const int64_t* r = jobs + (size_t)(j0 + q) * 5;
      CsJob& J = js.j[q];
      J.part = reinterpret_cast<const float*>(r[0]);
      J.out = reinterpret_cast<uint16_t*>(r[1]);
      J.nparts = (int)r[2]; J.C = (int)r[3]; J.acc = (int)r[4];
      if (!J.part || !J.out || J.C <= 0 || J.nparts <= 0) return hipErrorInvalidValue;
      J.b0 = blocks;
      blocks += (J.C + 15) / 16;
    }
    hipLaunchKernelGGL(colsum_jobs_kernel, dim3(blocks), dim3(256), 0, s, js, nj);
  }
  return hipGetLastError();
}

// g [N][2H][2W][C], add (nullable) / out [N][H][W][C], all NHWC contiguous bf16, C % 8 == 0,
// 16-B aligned
MX_EXPORT int mx_down2_add(const void* g, const void* add, void* out, int N, int H, int W, int C, hipStream_t s) {
  if (N <= 0 || H <= 0 || W <= 0) return hipSuccess;
  if ((C & 7) || (((uintptr_t)g | (uintptr_t)add | (uintptr_t)out) & 15)) return hipErrorInvalidValue;
  const int64_t total = (int64_t)N * H * W * (C / 8);
  const unsigned blocks = (unsigned)((total + 255) / 256 < 16384 ? (total + 255) / 256 : 16384);
  hipLaunchKernelGGL(down2_add_kernel, dim3(blocks), dim3(256), 0, s, (const uint16_t*)g, (const uint16_t*)add,
                     (uint16_t*)out, N, H, W, C);
  return hipGetLastError();
}

// FPN P6 = max_pool2d(P5, kernel 1, stride 2), i.e. every second row / column of P5 (NHWC bf16,
// 8 channels per thread), and its gradient: the P6 gradient at the even positions of a
// P5-shaped tensor, zeros elsewhere (one pass, no zero fill).  torch's NHWC max-pool kernels
// took ~10 us forward and ~37 us backward on these few-KB tensors (profiles/r5_s1 census).
namespace {
__global__ __launch_bounds__(256) void subsample2_kernel(const uint16_t* __restrict__ src, uint16_t* __restrict__ dst,
                                                         int H, int W, int h, int w, int C8, int64_t nvec, int grad) {
  for (int64_t v = (int64_t)blockIdx.x * 256 + threadIdx.x; v < nvec; v += (int64_t)gridDim.x * 256) {
    const int64_t pix = v / C8;
    const int c8 = (int)(v - pix * C8);
    if (!grad) {   // v indexes P6 [N][h][w]
      const int64_t n = pix / ((int64_t)h * w);
      const int rem = (int)(pix - n * h * w), y = rem / w, x = rem - (rem / w) * w;
      reinterpret_cast<uint4*>(dst)[v] =
          reinterpret_cast<const uint4*>(src)[((n * H + 2 * y) * W + 2 * x) * C8 + c8];
    } else {       // v indexes the P5-shaped gradient [N][H][W]; src is the P6 gradient
      const int64_t n = pix / ((int64_t)H * W);
      const int rem = (int)(pix - n * H * W), y = rem / W, x = rem - (rem / W) * W;
      uint4 val = make_uint4(0u, 0u, 0u, 0u);
      if (!((y | x) & 1)) val = reinterpret_cast<const uint4*>(src)[((n * h + y / 2) * w + x / 2) * C8 + c8];
      reinterpret_cast<uint4*>(dst)[v] = val;
    }
  }
}
}  // namespace

// grad = 0: dst [N][ceil(H/2)][ceil(W/2)][C] = src [N][H][W][C] at even (y, x); grad = 1: dst [N][H][W][C]
// = src [N][ceil(H/2)][ceil(W/2)][C] at even positions, zero elsewhere.  C % 8 == 0, 16-B aligned.
MX_EXPORT int mx_subsample2(const void* src, void* dst, int N, int H, int W, int C, int grad, hipStream_t s) {
  if (N <= 0 || H <= 0 || W <= 0 || C % 8 || (((uintptr_t)src | (uintptr_t)dst) & 15)) return (int)hipErrorInvalidValue;
  const int h = (H + 1) / 2, w = (W + 1) / 2;
  const int64_t nvec = (int64_t)N * (grad ? (int64_t)H * W : (int64_t)h * w) * (C / 8);
  const int64_t blocks = (nvec + 255) / 256 < 4096 ? (nvec + 255) / 256 : 4096;
  hipLaunchKernelGGL(subsample2_kernel, dim3((unsigned)blocks), dim3(256), 0, s, (const uint16_t*)src, (uint16_t*)dst, H,
                     W, h, w, C / 8, nvec, grad);
  return hipGetLastError();
}
