// Training-mode BatchNorm for NHWC (channels_last) bf16 CNNs, fused with the residual add
// and the ReLU that follow it in a ResNet bottleneck (BASELINE.json config 5: the Ray Train
// PyTorch-Lightning ResNet-50, /root/reference/charts/machine-learning/training/raytrain/
// templates/train.yaml:142-221):
//
//   forward   y = act(x * scale[c] + shift[c] (+ res)),  scale = gamma * rstd,
//             shift = beta - mean * scale,  batch statistics over the N*H*W rows
//   backward  dz = dy * (y > 0) (ReLU) ;  dres = dz ;  dbeta = sum dz ;  dgamma = sum dz xhat
//             dx = gamma rstd (dz - dbeta / M - xhat dgamma / M)
//
// Layout: [M, C] with M = N*H*W rows (NHWC memory), C % 8 == 0, 16-B vectors (8 bf16) per
// lane.  Every reduction is two-stage and deterministic: a statistics pass writes per-block
// partials (fixed row stripes), a per-channel finalize merges them in block order -- no
// atomics, the same bits on every run.  The forward statistics are merged as (count, mean,
// M2) with Chan's formula (no E[x^2] - E[x]^2 cancellation over ~10^6 rows); a thread's own
// rows (<= rows_per_block / rows-per-iteration) use plain sums.
//
// Five launches per BN layer (stats, finalize, apply; bwd stats, bwd finalize, bwd apply)
// where torch's NHWC path takes a statistics kernel, an elementwise kernel and separate
// add / ReLU passes forward and the same again backward.
#include "common.h"

using namespace mx;

namespace {

constexpr int kThreads = 256;

struct RowGeo {   // 256 threads = rpi rows x cv 8-channel vectors of a row
  int c8, cv, rpi, tr, tv;
  __device__ RowGeo(int C) {
    c8 = C / 8;
    cv = c8 < kThreads ? c8 : kThreads;
    rpi = kThreads / cv;
    tr = threadIdx.x / cv;
    tv = threadIdx.x % cv;
  }
};

// Chan's parallel merge of (n, mean, M2) into (na, ma, m2a)
__device__ __forceinline__ void chan_merge(float& na, float& ma, float& m2a, float nb, float mb, float m2b) {
  const float n = na + nb;
  if (nb == 0.f) return;
  const float d = mb - ma;
  const float f = nb / n;
  ma += d * f;
  m2a += m2b + d * d * na * f;
  na = n;
}

// pmean / pm2: [nblk][C] per-block statistics; pcount: rows of block b (computed by the
// finalize).  grid: (ceil(c8 / cv), nblk)
__global__ __launch_bounds__(kThreads) void bn_stats_kernel(const uint16_t* __restrict__ x, int M, int C,
                                                            int rows_per_block, float* __restrict__ pmean,
                                                            float* __restrict__ pm2) {
  const RowGeo g(C);
  const int vc = blockIdx.x * g.cv + g.tv;            // this thread's 8-channel vector
  const int r0 = blockIdx.y * rows_per_block, r1 = min(M, r0 + rows_per_block);
  __shared__ float sm[3][kThreads][8];
  float s[8] = {0, 0, 0, 0, 0, 0, 0, 0}, q[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  int n = 0;
  if (vc < g.c8) {
    int r = r0 + g.tr;
    // eight rows' loads in flight per thread (narrow C -- the ResNet stem's 64 channels --
    // leaves one 16-B load per row group: one at a time the pass ran at ~2.4 TB/s)
    for (; r + 7 * g.rpi < r1; r += 8 * g.rpi) {
      uint4 w[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) w[u] = reinterpret_cast<const uint4*>(x + (size_t)(r + u * g.rpi) * C)[vc];
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        float v[8];
        unpack8(w[u], v);
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          s[j] += v[j];
          q[j] = __builtin_fmaf(v[j], v[j], q[j]);
        }
      }
      n += 8;
    }
    for (; r < r1; r += g.rpi) {
      float v[8];
      unpack8(reinterpret_cast<const uint4*>(x + (size_t)r * C)[vc], v);
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        s[j] += v[j];
        q[j] = __builtin_fmaf(v[j], v[j], q[j]);
      }
      ++n;
    }
  }
  // per-thread (n, mean, M2), merged over the block's row groups in order by row group 0
  const float fn = (float)n;
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const float m = n ? s[j] / fn : 0.f;
    sm[0][threadIdx.x][j] = fn;
    sm[1][threadIdx.x][j] = m;
    sm[2][threadIdx.x][j] = n ? fmaxf(q[j] - s[j] * m, 0.f) : 0.f;
  }
  __syncthreads();
  if (g.tr == 0 && vc < g.c8) {
    float na[8], ma[8], m2[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      na[j] = sm[0][threadIdx.x][j];
      ma[j] = sm[1][threadIdx.x][j];
      m2[j] = sm[2][threadIdx.x][j];
    }
    for (int k = 1; k < g.rpi; ++k) {
      const int t = k * g.cv + g.tv;
#pragma unroll
      for (int j = 0; j < 8; ++j) chan_merge(na[j], ma[j], m2[j], sm[0][t][j], sm[1][t][j], sm[2][t][j]);
    }
    float* pmr = pmean + (size_t)blockIdx.y * C + 8 * vc;
    float* pqr = pm2 + (size_t)blockIdx.y * C + 8 * vc;
#pragma unroll
    for (int j = 0; j < 8; j += 4) {
      *reinterpret_cast<float4*>(pmr + j) = make_float4(ma[j], ma[j + 1], ma[j + 2], ma[j + 3]);
      *reinterpret_cast<float4*>(pqr + j) = make_float4(m2[j], m2[j + 1], m2[j + 2], m2[j + 3]);
    }
  }
}

// one wave per channel: lane l merges blocks l, l + 64, ... in order, then a fixed
// butterfly over the lanes (deterministic).  Outputs: mean / rstd (saved for backward),
// scale / shift (fp32, for the apply pass), running statistics updated in place.
__global__ __launch_bounds__(kThreads) void bn_finalize_kernel(const float* __restrict__ pmean,
                                                               const float* __restrict__ pm2, int nblk,
                                                               int rows_per_block, int M, int C,
                                                               const float* __restrict__ gamma,
                                                               const float* __restrict__ beta, float eps,
                                                               float momentum, float* __restrict__ mean_out,
                                                               float* __restrict__ rstd_out,
                                                               float* __restrict__ scale, float* __restrict__ shift,
                                                               float* __restrict__ run_mean,
                                                               float* __restrict__ run_var,
                                                               int64_t* __restrict__ nbt) {
  const int lane = threadIdx.x & 63;
  const int c = blockIdx.x * (kThreads / 64) + (threadIdx.x >> 6);
  // nn.BatchNorm2d's num_batches_tracked += 1 (a separate 5-us launch per layer otherwise)
  if (nbt && blockIdx.x == 0 && threadIdx.x == 0) nbt[0] += 1;
  if (c >= C) return;
  float na = 0.f, ma = 0.f, m2 = 0.f;
  for (int b = lane; b < nblk; b += 64) {
    const float nb = (float)min(rows_per_block, M - b * rows_per_block);
    chan_merge(na, ma, m2, nb, pmean[(size_t)b * C + c], pm2[(size_t)b * C + c]);
  }
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const float nb = __shfl_xor(na, o), mb = __shfl_xor(ma, o), m2b = __shfl_xor(m2, o);
    // both partners compute the same merged value: order the operands by lane bit
    if (lane & o) {
      float n2 = nb, m_2 = mb, q2 = m2b;
      chan_merge(n2, m_2, q2, na, ma, m2);
      na = n2; ma = m_2; m2 = q2;
    } else {
      chan_merge(na, ma, m2, nb, mb, m2b);
    }
  }
  if (lane == 0) {
    const float var = m2 / (float)M;
    const float rs = rsqrtf(var + eps);
    const float sc = gamma[c] * rs;
    mean_out[c] = ma;
    rstd_out[c] = rs;
    scale[c] = sc;
    shift[c] = beta[c] - ma * sc;
    if (run_mean) {
      const float unb = M > 1 ? m2 / (float)(M - 1) : var;
      run_mean[c] = (1.f - momentum) * run_mean[c] + momentum * ma;
      run_var[c] = (1.f - momentum) * run_var[c] + momentum * unb;
    }
  }
}

// Finalize from the statistics a convolution's epilogue wrote (csrc/convwg.hip ConvFw::bnp):
// channel-major [C][nblk] means and M2 of 64-row blocks (up to ~12.5k blocks at the ResNet-50
// res2 shapes).  One workgroup per channel: thread t merges blocks t, t + 256, ... (coalesced
// loads, four in flight), then a fixed butterfly in each wave and the four waves in order
// (deterministic); outputs as bn_finalize_kernel.
__global__ __launch_bounds__(kThreads) void bn_finalize_cm_kernel(const float* __restrict__ pmean,
                                                                  const float* __restrict__ pm2, int nblk, int rpb,
                                                                  int M, int C, const float* __restrict__ gamma,
                                                                  const float* __restrict__ beta, float eps,
                                                                  float momentum, float* __restrict__ mean_out,
                                                                  float* __restrict__ rstd_out,
                                                                  float* __restrict__ scale, float* __restrict__ shift,
                                                                  float* __restrict__ run_mean,
                                                                  float* __restrict__ run_var,
                                                                  int64_t* __restrict__ nbt) {
  const int c = blockIdx.x, t = threadIdx.x, lane = t & 63, wave = t >> 6;
  if (nbt && c == 0 && t == 0) nbt[0] += 1;
  const float* pmr = pmean + (size_t)c * nblk;
  const float* pqr = pm2 + (size_t)c * nblk;
  float na = 0.f, ma = 0.f, m2 = 0.f;
  int b = t;
  // 8 + 8 loads in flight per thread (latency-bound: 12,544 partials per channel at the
  // ResNet res2 shapes); the merge order is the plain b = t, t + 256, ... sequence
  for (; b + 7 * kThreads < nblk; b += 8 * kThreads) {
    float mb[8], qb[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      mb[k] = pmr[b + k * kThreads];
      qb[k] = pqr[b + k * kThreads];
    }
#pragma unroll
    for (int k = 0; k < 8; ++k)
      chan_merge(na, ma, m2, (float)min(rpb, M - (b + k * kThreads) * rpb), mb[k], qb[k]);
  }
  for (; b < nblk; b += kThreads) chan_merge(na, ma, m2, (float)min(rpb, M - b * rpb), pmr[b], pqr[b]);
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const float nb = __shfl_xor(na, o), mb = __shfl_xor(ma, o), m2b = __shfl_xor(m2, o);
    if (lane & o) {
      float n2 = nb, m_2 = mb, q2 = m2b;
      chan_merge(n2, m_2, q2, na, ma, m2);
      na = n2; ma = m_2; m2 = q2;
    } else {
      chan_merge(na, ma, m2, nb, mb, m2b);
    }
  }
  __shared__ float sw[3][kThreads / 64];
  if (lane == 0) {
    sw[0][wave] = na;
    sw[1][wave] = ma;
    sw[2][wave] = m2;
  }
  __syncthreads();
  if (t == 0) {
    for (int w = 1; w < kThreads / 64; ++w) chan_merge(na, ma, m2, sw[0][w], sw[1][w], sw[2][w]);
    const float var = m2 / (float)M;
    const float rs = rsqrtf(var + eps);
    const float sc = gamma[c] * rs;
    mean_out[c] = ma;
    rstd_out[c] = rs;
    scale[c] = sc;
    shift[c] = beta[c] - ma * sc;
    if (run_mean) {
      const float unb = M > 1 ? m2 / (float)(M - 1) : var;
      run_mean[c] = (1.f - momentum) * run_mean[c] + momentum * ma;
      run_var[c] = (1.f - momentum) * run_var[c] + momentum * unb;
    }
  }
}

// y = act(x * scale + shift (+ res)); one thread per 8-channel vector
template <bool kRes, bool kRelu>
__global__ __launch_bounds__(kThreads) void bn_apply_kernel(const uint16_t* __restrict__ x,
                                                            const uint16_t* __restrict__ res,
                                                            const float* __restrict__ scale,
                                                            const float* __restrict__ shift,
                                                            uint16_t* __restrict__ y, int64_t nvec, int c8) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  float sc[8], sh[8];
  auto coefs = [&](int c) __attribute__((always_inline)) {
    const float4 s0 = *reinterpret_cast<const float4*>(scale + c), s1 = *reinterpret_cast<const float4*>(scale + c + 4);
    const float4 h0 = *reinterpret_cast<const float4*>(shift + c), h1 = *reinterpret_cast<const float4*>(shift + c + 4);
    sc[0] = s0.x; sc[1] = s0.y; sc[2] = s0.z; sc[3] = s0.w; sc[4] = s1.x; sc[5] = s1.y; sc[6] = s1.z; sc[7] = s1.w;
    sh[0] = h0.x; sh[1] = h0.y; sh[2] = h0.z; sh[3] = h0.w; sh[4] = h1.x; sh[5] = h1.y; sh[6] = h1.z; sh[7] = h1.w;
  };
  // the grid stride is a multiple of c8 (c8 divides the 256-thread block: C a power-of-two
  // multiple of 8 up to 2048): a thread's channels never change -- the coefficients are
  // loaded once and no per-vector 64-bit modulo runs
  const bool fixed = (kThreads % c8) == 0;
  const int64_t v0 = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (fixed) coefs(8 * (int)((uint32_t)v0 % (uint32_t)c8));
  for (int64_t v = v0; v < nvec; v += stride) {
    if (!fixed) coefs(8 * (int)(v % c8));
    float a[8], r[8];
    unpack8(reinterpret_cast<const uint4*>(x)[v], a);
    if (kRes) unpack8(reinterpret_cast<const uint4*>(res)[v], r);
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      float t = __builtin_fmaf(a[j], sc[j], sh[j]);
      if (kRes) t += r[j];
      a[j] = kRelu ? fmaxf(t, 0.f) : t;
    }
    reinterpret_cast<uint4*>(y)[v] = pack8(a);
  }
}

// backward statistics: per-block column sums of dz and dz * xhat, partial [nblk][2][C]
// kRecon (ReLU, no residual): xhat recovered from the output where the ReLU passed,
// xhat = (y - beta) / gamma -- exactly where dz can be nonzero -- so x is not read (a third
// of this pass's bytes); a thread whose channels include |gamma| < 1e-6 reads x instead.
template <bool kRelu, bool kRecon = false>
__global__ __launch_bounds__(kThreads) void bn_bwd_stats_kernel(const uint16_t* __restrict__ dy,
                                                                const uint16_t* __restrict__ y,
                                                                const uint16_t* __restrict__ x,
                                                                const float* __restrict__ mean,
                                                                const float* __restrict__ rstd, int M, int C,
                                                                int rows_per_block, float* __restrict__ partial,
                                                                const float* __restrict__ gamma = nullptr,
                                                                const float* __restrict__ beta = nullptr) {
  const RowGeo g(C);
  const int vc = blockIdx.x * g.cv + g.tv;
  const int r0 = blockIdx.y * rows_per_block, r1 = min(M, r0 + rows_per_block);
  __shared__ float sm[2][kThreads][8];
  float sd[8] = {0, 0, 0, 0, 0, 0, 0, 0}, sx[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  float ig[8], bt[8];
  bool recon = kRecon && vc < g.c8;
  if (recon) {
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const float gm = gamma[8 * vc + j];
      recon = recon && fabsf(gm) >= 1e-6f;
      ig[j] = 1.f / gm;
      bt[j] = beta[8 * vc + j];
    }
  }
  if (recon) {
    {
      for (int r = r0 + g.tr; r < r1; r += g.rpi) {
        float d[8], o[8];
        const size_t off = (size_t)r * C;
        unpack8(reinterpret_cast<const uint4*>(dy + off)[vc], d);
        unpack8(reinterpret_cast<const uint4*>(y + off)[vc], o);
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const float dz = o[j] > 0.f ? d[j] : 0.f;
          sd[j] += dz;
          sx[j] = __builtin_fmaf(dz, o[j] > 0.f ? (o[j] - bt[j]) * ig[j] : 0.f, sx[j]);
        }
      }
    }
  } else if (vc < g.c8) {
    float mu[8], rs[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      mu[j] = mean[8 * vc + j];
      rs[j] = rstd[8 * vc + j];
    }
    for (int r = r0 + g.tr; r < r1; r += g.rpi) {
      float d[8], a[8];
      const size_t off = (size_t)r * C;
      unpack8(reinterpret_cast<const uint4*>(dy + off)[vc], d);
      unpack8(reinterpret_cast<const uint4*>(x + off)[vc], a);
      if (kRelu) {
        float o[8];
        unpack8(reinterpret_cast<const uint4*>(y + off)[vc], o);
#pragma unroll
        for (int j = 0; j < 8; ++j) d[j] = o[j] > 0.f ? d[j] : 0.f;
      }
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        sd[j] += d[j];
        sx[j] = __builtin_fmaf(d[j], (a[j] - mu[j]) * rs[j], sx[j]);
      }
    }
  }
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    sm[0][threadIdx.x][j] = sd[j];
    sm[1][threadIdx.x][j] = sx[j];
  }
  __syncthreads();
  if (g.tr == 0 && vc < g.c8) {
    for (int k = 1; k < g.rpi; ++k) {
      const int t = k * g.cv + g.tv;
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        sd[j] += sm[0][t][j];
        sx[j] += sm[1][t][j];
      }
    }
    float* p0 = partial + (size_t)blockIdx.y * 2 * C + 8 * vc;
    float* p1 = p0 + C;
#pragma unroll
    for (int j = 0; j < 8; j += 4) {
      *reinterpret_cast<float4*>(p0 + j) = make_float4(sd[j], sd[j + 1], sd[j + 2], sd[j + 3]);
      *reinterpret_cast<float4*>(p1 + j) = make_float4(sx[j], sx[j + 1], sx[j + 2], sx[j + 3]);
    }
  }
}

// dbeta / dgamma (fp32, written or accumulated) and the dx coefficients:
// coef[0][c] = gamma rstd, coef[1][c] = dbeta / M, coef[2][c] = dgamma / M
__global__ __launch_bounds__(kThreads) void bn_bwd_finalize_kernel(const float* __restrict__ partial, int nblk,
                                                                   int M, int C, const float* __restrict__ gamma,
                                                                   const float* __restrict__ rstd,
                                                                   float* __restrict__ dgamma,
                                                                   float* __restrict__ dbeta, int accumulate,
                                                                   float* __restrict__ coef) {
  const int lane = threadIdx.x & 63;
  const int c = blockIdx.x * (kThreads / 64) + (threadIdx.x >> 6);
  if (c >= C) return;
  float sd = 0.f, sx = 0.f;
  for (int b = lane; b < nblk; b += 64) {
    sd += partial[(size_t)b * 2 * C + c];
    sx += partial[(size_t)b * 2 * C + C + c];
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {   // fixed tree: every lane ends with the same sums
    sd += __shfl_xor(sd, o);
    sx += __shfl_xor(sx, o);
  }
  if (lane == 0) {
    if (dbeta) dbeta[c] = accumulate ? dbeta[c] + sd : sd;
    if (dgamma) dgamma[c] = accumulate ? dgamma[c] + sx : sx;
    coef[c] = gamma[c] * rstd[c];
    coef[C + c] = sd / (float)M;
    coef[2 * C + c] = sx / (float)M;
  }
}

template <bool kRelu, bool kRes>
__global__ __launch_bounds__(kThreads) void bn_bwd_apply_kernel(const uint16_t* __restrict__ dy,
                                                                const uint16_t* __restrict__ y,
                                                                const uint16_t* __restrict__ x,
                                                                const float* __restrict__ mean,
                                                                const float* __restrict__ rstd,
                                                                const float* __restrict__ coef,
                                                                uint16_t* __restrict__ dx, uint16_t* __restrict__ dres,
                                                                int64_t nvec, int C) {
  const int c8 = C / 8;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  // per-channel terms of dx = k0 (dz - k1 - (x - mean) rstd k2) = A (x - mean) + B dz + D,
  // held in registers when the thread's channels are fixed (as bn_apply_kernel)
  float A[8], B[8], D[8], Mn[8];
  auto coefs = [&](int c) __attribute__((always_inline)) {
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const float k0 = coef[c + j];
      A[j] = -k0 * rstd[c + j] * coef[2 * C + c + j];
      B[j] = k0;
      D[j] = -k0 * coef[C + c + j];
      Mn[j] = mean[c + j];
    }
  };
  const bool fixed = (kThreads % c8) == 0;
  const int64_t v0 = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (fixed) coefs(8 * (int)((uint32_t)v0 % (uint32_t)c8));
  for (int64_t v = v0; v < nvec; v += stride) {
    if (!fixed) coefs(8 * (int)(v % c8));
    float d[8], a[8];
    unpack8(reinterpret_cast<const uint4*>(dy)[v], d);
    unpack8(reinterpret_cast<const uint4*>(x)[v], a);
    if (kRelu) {
      float o[8];
      unpack8(reinterpret_cast<const uint4*>(y)[v], o);
#pragma unroll
      for (int j = 0; j < 8; ++j) d[j] = o[j] > 0.f ? d[j] : 0.f;
    }
    if (kRes) reinterpret_cast<uint4*>(dres)[v] = pack8(d);
#pragma unroll
    for (int j = 0; j < 8; ++j) a[j] = __builtin_fmaf(A[j], a[j] - Mn[j], __builtin_fmaf(B[j], d[j], D[j]));
    reinterpret_cast<uint4*>(dx)[v] = pack8(a);
  }
}

int rows_per_block(int M) {
  int r = (M + 511) / 512;   // <= 512 row blocks: the finalize merges <= 8 partials per lane
  return r < 64 ? 64 : r;
}

constexpr int kPreRows = 64;   // rows per block of the convolution epilogue's statistics

int elem_grid(int64_t nvec) {
  int64_t g = (nvec + kThreads - 1) / kThreads;
  return (int)(g < 4096 ? (g < 1 ? 1 : g) : 4096);
}

}  // namespace

// partial scratch (floats) the forward / backward need for M rows x C channels
MX_EXPORT int64_t mx_bn_scratch(int M, int C) {
  const int nblk = (M + rows_per_block(M) - 1) / rows_per_block(M);
  return (int64_t)nblk * 2 * C + 3 * (int64_t)C + 2 * (int64_t)C;
}

// floats of the per-64-row-block statistics the convolution forward writes (ConvFw::bnp)
MX_EXPORT int64_t mx_bn_pre_size(int M, int C) {
  return (int64_t)((M + kPreRows - 1) / kPreRows) * 2 * C;
}

// Training forward.  x, res, y: [M][C] bf16 (res may be null); gamma / beta fp32 [C];
// mean / rstd out fp32 [C] (saved for backward); run_mean / run_var fp32 [C] updated in
// place (null: not tracked); scratch: mx_bn_scratch floats.
// nbt: num_batches_tracked (int64, incremented by the finalize) or null.
// pre: null, or the per-64-row-block statistics of x the producing convolution's epilogue
// wrote (mx_bn_pre_size floats): then no statistics pass reads x.
MX_EXPORT int mx_bn_fwd(const void* x, const void* res, void* y, const float* gamma, const float* beta, float* mean,
                        float* rstd, float* run_mean, float* run_var, int M, int C, float eps, float momentum,
                        int relu, float* scratch, int64_t* nbt, const float* pre, hipStream_t s) {
  if (C % 8 || C <= 0 || M <= 0 || C > 8 * 65535 * kThreads) return hipErrorInvalidValue;
  const int c8 = C / 8, cv = c8 < kThreads ? c8 : kThreads;
  const int rpb = rows_per_block(M), nblk = (M + rpb - 1) / rpb;
  float* scale = scratch + (size_t)2 * nblk * C;
  float* shift = scale + C;
  if (!pre) {
    float* pmean = scratch;
    float* pm2 = scratch + (size_t)nblk * C;
    hipLaunchKernelGGL(bn_stats_kernel, dim3((c8 + cv - 1) / cv, nblk), dim3(kThreads), 0, s, (const uint16_t*)x, M,
                       C, rpb, pmean, pm2);
    hipLaunchKernelGGL(bn_finalize_kernel, dim3((C + 3) / 4), dim3(kThreads), 0, s, pmean, pm2, nblk, rpb, M, C,
                       gamma, beta, eps, momentum, mean, rstd, scale, shift, run_mean, run_var, nbt);
  } else {
    const int nb = (M + kPreRows - 1) / kPreRows;
    hipLaunchKernelGGL(bn_finalize_cm_kernel, dim3(C), dim3(kThreads), 0, s, pre, pre + (size_t)nb * C, nb,
                       kPreRows, M, C, gamma, beta, eps, momentum, mean, rstd, scale, shift, run_mean, run_var, nbt);
  }
  if (!y) return hipGetLastError();   // statistics only (mx_bn2_apply applies them)
  const int64_t nvec = (int64_t)M * c8;
  const dim3 gr(elem_grid(nvec));
  if (res) {
    if (relu) hipLaunchKernelGGL((bn_apply_kernel<true, true>), gr, dim3(kThreads), 0, s, (const uint16_t*)x,
                                 (const uint16_t*)res, scale, shift, (uint16_t*)y, nvec, c8);
    else hipLaunchKernelGGL((bn_apply_kernel<true, false>), gr, dim3(kThreads), 0, s, (const uint16_t*)x,
                            (const uint16_t*)res, scale, shift, (uint16_t*)y, nvec, c8);
  } else {
    if (relu) hipLaunchKernelGGL((bn_apply_kernel<false, true>), gr, dim3(kThreads), 0, s, (const uint16_t*)x,
                                 nullptr, scale, shift, (uint16_t*)y, nvec, c8);
    else hipLaunchKernelGGL((bn_apply_kernel<false, false>), gr, dim3(kThreads), 0, s, (const uint16_t*)x,
                            nullptr, scale, shift, (uint16_t*)y, nvec, c8);
  }
  return hipGetLastError();
}

// Evaluation / frozen-statistics forward with a caller-provided per-channel scale / shift
MX_EXPORT int mx_bn_apply(const void* x, const void* res, void* y, const float* scale, const float* shift, int M,
                          int C, int relu, hipStream_t s) {
  if (C % 8 || C <= 0 || M <= 0) return hipErrorInvalidValue;
  const int c8 = C / 8;
  const int64_t nvec = (int64_t)M * c8;
  const dim3 gr(elem_grid(nvec));
  if (res) {
    if (relu) hipLaunchKernelGGL((bn_apply_kernel<true, true>), gr, dim3(kThreads), 0, s, (const uint16_t*)x,
                                 (const uint16_t*)res, scale, shift, (uint16_t*)y, nvec, c8);
    else hipLaunchKernelGGL((bn_apply_kernel<true, false>), gr, dim3(kThreads), 0, s, (const uint16_t*)x,
                            (const uint16_t*)res, scale, shift, (uint16_t*)y, nvec, c8);
  } else {
    if (relu) hipLaunchKernelGGL((bn_apply_kernel<false, true>), gr, dim3(kThreads), 0, s, (const uint16_t*)x,
                                 nullptr, scale, shift, (uint16_t*)y, nvec, c8);
    else hipLaunchKernelGGL((bn_apply_kernel<false, false>), gr, dim3(kThreads), 0, s, (const uint16_t*)x,
                            nullptr, scale, shift, (uint16_t*)y, nvec, c8);
  }
  return hipGetLastError();
}

// Backward.  dy, y (forward output: the ReLU mask), x (forward input): [M][C] bf16;
// dx out, dres out (null: no residual); dgamma / dbeta fp32 [C] written (accumulate = 0) or
// added to; scratch: mx_bn_scratch floats.
MX_EXPORT int mx_bn_bwd(const void* dy, const void* y, const void* x, const float* mean, const float* rstd,
                        const float* gamma, void* dx, void* dres, float* dgamma, float* dbeta, int accumulate, int M,
                        int C, int relu, float* scratch, const float* beta, int recon, hipStream_t s) {
  if (C % 8 || C <= 0 || M <= 0) return hipErrorInvalidValue;
  if (recon && (!relu || dres || !beta)) return hipErrorInvalidValue;
  const int rpb = rows_per_block(M), nblk = (M + rpb - 1) / rpb;
  const int c8 = C / 8, cv = c8 < kThreads ? c8 : kThreads;
  float* partial = scratch;
  float* coef = scratch + (size_t)nblk * 2 * C;
  const dim3 sg((c8 + cv - 1) / cv, nblk);
  if (recon) hipLaunchKernelGGL((bn_bwd_stats_kernel<true, true>), sg, dim3(kThreads), 0, s, (const uint16_t*)dy,
                                (const uint16_t*)y, (const uint16_t*)x, mean, rstd, M, C, rpb, partial, gamma, beta);
  else if (relu) hipLaunchKernelGGL(bn_bwd_stats_kernel<true>, sg, dim3(kThreads), 0, s, (const uint16_t*)dy,
                                    (const uint16_t*)y, (const uint16_t*)x, mean, rstd, M, C, rpb, partial,
                                    nullptr, nullptr);
  else hipLaunchKernelGGL(bn_bwd_stats_kernel<false>, sg, dim3(kThreads), 0, s, (const uint16_t*)dy, nullptr,
                          (const uint16_t*)x, mean, rstd, M, C, rpb, partial, nullptr, nullptr);
  hipLaunchKernelGGL(bn_bwd_finalize_kernel, dim3((C + 3) / 4), dim3(kThreads), 0, s, partial, nblk, M, C, gamma,
                     rstd, dgamma, dbeta, accumulate, coef);
  const int64_t nvec = (int64_t)M * c8;
  const dim3 gr(elem_grid(nvec));
#define MX_BN_BWD(RL, RS)                                                                                   \
  hipLaunchKernelGGL((bn_bwd_apply_kernel<RL, RS>), gr, dim3(kThreads), 0, s, (const uint16_t*)dy,          \
                     (const uint16_t*)y, (const uint16_t*)x, mean, rstd, coef, (uint16_t*)dx, (uint16_t*)dres, \
                     nvec, C)
  if (relu) {
    if (dres) MX_BN_BWD(true, true);
    else MX_BN_BWD(true, false);
  } else {
    if (dres) MX_BN_BWD(false, true);
    else MX_BN_BWD(false, false);
  }
#undef MX_BN_BWD
  return hipGetLastError();
}

// ============================================================ two BatchNorms into one ReLU
// The ResNet projection block's tail  y = relu(BN_a(xa) + BN_b(xb))  (conv3's BN plus the
// shortcut's BN) without the shortcut BN's own output tensor: forward one apply pass reading
// xa, xb (the statistics of both come from mx_bn_fwd with y = null); backward one statistics
// pass (dz = dy (y > 0) shared: sum dz, sum dz xhat_a, sum dz xhat_b) and one apply pass
// writing both input gradients -- 5 of the 18 tensor passes of the two separate BN layers
// disappear.  Per-channel terms live in registers (the grid stride is a multiple of C / 8).
namespace {

struct Bn2P {
  const float *mean_a, *rstd_a, *gamma_a, *beta_a, *mean_b, *rstd_b, *gamma_b, *beta_b;
};

__global__ __launch_bounds__(kThreads) void bn2_apply_kernel(const uint16_t* __restrict__ xa,
                                                             const uint16_t* __restrict__ xb, const Bn2P p,
                                                             uint16_t* __restrict__ y, int64_t nvec, int c8) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  float sa[8], sb[8], hh[8];
  auto coefs = [&](int c) __attribute__((always_inline)) {
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      sa[j] = p.gamma_a[c + j] * p.rstd_a[c + j];
      sb[j] = p.gamma_b[c + j] * p.rstd_b[c + j];
      hh[j] = p.beta_a[c + j] - p.mean_a[c + j] * sa[j] + p.beta_b[c + j] - p.mean_b[c + j] * sb[j];
    }
  };
  const bool fixed = (kThreads % c8) == 0;
  const int64_t v0 = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (fixed) coefs(8 * (int)((uint32_t)v0 % (uint32_t)c8));
  for (int64_t v = v0; v < nvec; v += stride) {
    if (!fixed) coefs(8 * (int)(v % c8));
    float a[8], b[8];
    unpack8(reinterpret_cast<const uint4*>(xa)[v], a);
    unpack8(reinterpret_cast<const uint4*>(xb)[v], b);
#pragma unroll
    for (int j = 0; j < 8; ++j) a[j] = fmaxf(__builtin_fmaf(a[j], sa[j], __builtin_fmaf(b[j], sb[j], hh[j])), 0.f);
    reinterpret_cast<uint4*>(y)[v] = pack8(a);
  }
}

// partial_a / partial_b: [nblk][2][C] = (sum dz, sum dz xhat) of each BN
__global__ __launch_bounds__(kThreads) void bn2_bwd_stats_kernel(const uint16_t* __restrict__ dy,
                                                                 const uint16_t* __restrict__ y,
                                                                 const uint16_t* __restrict__ xa,
                                                                 const uint16_t* __restrict__ xb, const Bn2P p,
                                                                 int M, int C, int rows_per_block,
                                                                 float* __restrict__ partial_a,
                                                                 float* __restrict__ partial_b) {
  const RowGeo g(C);
  const int vc = blockIdx.x * g.cv + g.tv;
  const int r0 = blockIdx.y * rows_per_block, r1 = min(M, r0 + rows_per_block);
  __shared__ float sm[3][kThreads][8];
  float sd[8] = {0, 0, 0, 0, 0, 0, 0, 0}, sx[8] = {0, 0, 0, 0, 0, 0, 0, 0}, sz[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  if (vc < g.c8) {
    float ma[8], ra[8], mb[8], rb[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      ma[j] = p.mean_a[8 * vc + j];
      ra[j] = p.rstd_a[8 * vc + j];
      mb[j] = p.mean_b[8 * vc + j];
      rb[j] = p.rstd_b[8 * vc + j];
    }
    for (int r = r0 + g.tr; r < r1; r += g.rpi) {
      float d[8], o[8], a[8], b[8];
      const size_t off = (size_t)r * C;
      unpack8(reinterpret_cast<const uint4*>(dy + off)[vc], d);
      unpack8(reinterpret_cast<const uint4*>(y + off)[vc], o);
      unpack8(reinterpret_cast<const uint4*>(xa + off)[vc], a);
      unpack8(reinterpret_cast<const uint4*>(xb + off)[vc], b);
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const float dz = o[j] > 0.f ? d[j] : 0.f;
        sd[j] += dz;
        sx[j] = __builtin_fmaf(dz, (a[j] - ma[j]) * ra[j], sx[j]);
        sz[j] = __builtin_fmaf(dz, (b[j] - mb[j]) * rb[j], sz[j]);
      }
    }
  }
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    sm[0][threadIdx.x][j] = sd[j];
    sm[1][threadIdx.x][j] = sx[j];
    sm[2][threadIdx.x][j] = sz[j];
  }
  __syncthreads();
  if (g.tr == 0 && vc < g.c8) {
    for (int k = 1; k < g.rpi; ++k) {
      const int t = k * g.cv + g.tv;
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        sd[j] += sm[0][t][j];
        sx[j] += sm[1][t][j];
        sz[j] += sm[2][t][j];
      }
    }
    float* pa = partial_a + (size_t)blockIdx.y * 2 * C + 8 * vc;
    float* pb = partial_b + (size_t)blockIdx.y * 2 * C + 8 * vc;
#pragma unroll
    for (int j = 0; j < 8; j += 4) {
      const float4 d4 = make_float4(sd[j], sd[j + 1], sd[j + 2], sd[j + 3]);
      *reinterpret_cast<float4*>(pa + j) = d4;
      *reinterpret_cast<float4*>(pb + j) = d4;
      *reinterpret_cast<float4*>(pa + C + j) = make_float4(sx[j], sx[j + 1], sx[j + 2], sx[j + 3]);
      *reinterpret_cast<float4*>(pb + C + j) = make_float4(sz[j], sz[j + 1], sz[j + 2], sz[j + 3]);
    }
  }
}

__global__ __launch_bounds__(kThreads) void bn2_bwd_apply_kernel(const uint16_t* __restrict__ dy,
                                                                 const uint16_t* __restrict__ y,
                                                                 const uint16_t* __restrict__ xa,
                                                                 const uint16_t* __restrict__ xb, const Bn2P p,
                                                                 const float* __restrict__ coef_a,
                                                                 const float* __restrict__ coef_b,
                                                                 uint16_t* __restrict__ dxa, uint16_t* __restrict__ dxb,
                                                                 int64_t nvec, int C) {
  const int c8 = C / 8;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  // dx = k0 (dz - k1 - (x - mean) rstd k2) = A (x - mean) + B dz + D, per BN
  float Aa[8], Ba[8], Da[8], Ma[8], Ab[8], Bb[8], Db[8], Mb[8];
  auto coefs = [&](int c) __attribute__((always_inline)) {
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const float ka = coef_a[c + j], kb = coef_b[c + j];
      Aa[j] = -ka * p.rstd_a[c + j] * coef_a[2 * C + c + j];
      Ba[j] = ka;
      Da[j] = -ka * coef_a[C + c + j];
      Ma[j] = p.mean_a[c + j];
      Ab[j] = -kb * p.rstd_b[c + j] * coef_b[2 * C + c + j];
      Bb[j] = kb;
      Db[j] = -kb * coef_b[C + c + j];
      Mb[j] = p.mean_b[c + j];
    }
  };
  const bool fixed = (kThreads % c8) == 0;
  const int64_t v0 = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (fixed) coefs(8 * (int)((uint32_t)v0 % (uint32_t)c8));
  for (int64_t v = v0; v < nvec; v += stride) {
    if (!fixed) coefs(8 * (int)(v % c8));
    float d[8], o[8], a[8], b[8];
    unpack8(reinterpret_cast<const uint4*>(dy)[v], d);
    unpack8(reinterpret_cast<const uint4*>(y)[v], o);
    unpack8(reinterpret_cast<const uint4*>(xa)[v], a);
    unpack8(reinterpret_cast<const uint4*>(xb)[v], b);
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const float dz = o[j] > 0.f ? d[j] : 0.f;
      a[j] = __builtin_fmaf(Aa[j], a[j] - Ma[j], __builtin_fmaf(Ba[j], dz, Da[j]));
      b[j] = __builtin_fmaf(Ab[j], b[j] - Mb[j], __builtin_fmaf(Bb[j], dz, Db[j]));
    }
    reinterpret_cast<uint4*>(dxa)[v] = pack8(a);
    reinterpret_cast<uint4*>(dxb)[v] = pack8(b);
  }
}

}  // namespace

// stats: float[8] pointers {mean_a, rstd_a, gamma_a, beta_a, mean_b, rstd_b, gamma_b, beta_b}
// (fp32 [C] each; the statistics from mx_bn_fwd with y = null).  xa, xb, y: [M][C] bf16.
MX_EXPORT int mx_bn2_apply(const void* xa, const void* xb, void* y, const int64_t* stats, int M, int C,
                           hipStream_t s) {
  if (C % 8 || C <= 0 || M <= 0) return hipErrorInvalidValue;
  const Bn2P p{(const float*)stats[0], (const float*)stats[1], (const float*)stats[2], (const float*)stats[3],
               (const float*)stats[4], (const float*)stats[5], (const float*)stats[6], (const float*)stats[7]};
  const int64_t nvec = (int64_t)M * (C / 8);
  hipLaunchKernelGGL(bn2_apply_kernel, dim3(elem_grid(nvec)), dim3(kThreads), 0, s, (const uint16_t*)xa,
                     (const uint16_t*)xb, p, (uint16_t*)y, nvec, C / 8);
  return hipGetLastError();
}

// floats of scratch mx_bn2_bwd needs
MX_EXPORT int64_t mx_bn2_scratch(int M, int C) { return 2 * mx_bn_scratch(M, C); }

// dy, y (the forward output), xa, xb -> dxa, dxb (bf16 [M][C]); dgamma / dbeta of both (fp32 [C])
MX_EXPORT int mx_bn2_bwd(const void* dy, const void* y, const void* xa, const void* xb, const int64_t* stats,
                         void* dxa, void* dxb, float* dgamma_a, float* dbeta_a, float* dgamma_b, float* dbeta_b,
                         int M, int C, float* scratch, hipStream_t s) {
  if (C % 8 || C <= 0 || M <= 0) return hipErrorInvalidValue;
  const Bn2P p{(const float*)stats[0], (const float*)stats[1], (const float*)stats[2], (const float*)stats[3],
               (const float*)stats[4], (const float*)stats[5], (const float*)stats[6], (const float*)stats[7]};
  const int rpb = rows_per_block(M), nblk = (M + rpb - 1) / rpb;
  const int c8 = C / 8, cv = c8 < kThreads ? c8 : kThreads;
  float* part_a = scratch;
  float* part_b = part_a + (size_t)nblk * 2 * C;
  float* coef_a = part_b + (size_t)nblk * 2 * C;
  float* coef_b = coef_a + 3 * (size_t)C;
  hipLaunchKernelGGL(bn2_bwd_stats_kernel, dim3((c8 + cv - 1) / cv, nblk), dim3(kThreads), 0, s,
                     (const uint16_t*)dy, (const uint16_t*)y, (const uint16_t*)xa, (const uint16_t*)xb, p, M, C, rpb,
                     part_a, part_b);
  hipLaunchKernelGGL(bn_bwd_finalize_kernel, dim3((C + 3) / 4), dim3(kThreads), 0, s, part_a, nblk, M, C, p.gamma_a,
                     p.rstd_a, dgamma_a, dbeta_a, 0, coef_a);
  hipLaunchKernelGGL(bn_bwd_finalize_kernel, dim3((C + 3) / 4), dim3(kThreads), 0, s, part_b, nblk, M, C, p.gamma_b,
                     p.rstd_b, dgamma_b, dbeta_b, 0, coef_b);
  const int64_t nvec = (int64_t)M * c8;
  hipLaunchKernelGGL(bn2_bwd_apply_kernel, dim3(elem_grid(nvec)), dim3(kThreads), 0, s, (const uint16_t*)dy,
                     (const uint16_t*)y, (const uint16_t*)xa, (const uint16_t*)xb, p, coef_a, coef_b,
                     (uint16_t*)dxa, (uint16_t*)dxb, nvec, C);
  return hipGetLastError();
}
