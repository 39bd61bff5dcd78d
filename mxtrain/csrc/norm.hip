// Fused LayerNorm / RMSNorm forward+backward and the fused
// bias-dropout-residual-add + LayerNorm ("BDA-LN") used between GPT sublayers.
//
// Replaces Apex `fused_layer_norm_cuda` / Megatron `MixedFusedLayerNorm` and the
// TorchScript `bias_dropout_add_fused_train` the reference pulls in through the
// Megatron-DeepSpeed image (containers/megatron-deepspeed/Dockerfile:6-13; SURVEY
// §2.8 K3, K4, K7).
//
// Design (gfx950): one wave64 per row, each lane owns 8 contiguous bf16 per 512
// columns (16-B vector loads, Guideline 13), statistics in fp32 through wave
// shuffles only (no LDS, no barriers on the forward path).  Backward keeps the
// per-column reductions (dgamma, dbeta, dbias) in registers across the rows a wave
// handles, folds them once per block into an LDS slab, dumps the slab to a
// [grid][3][cols] partial buffer, and a deterministic two-level column reduction
// folds the partials into the bf16 gradient buffers (optionally accumulating).
#include "common.h"

using namespace mx;

namespace {

template <int NV, bool RMS, bool HAS_BDA>
__global__ __launch_bounds__(256) void ln_fwd_kernel(
    const uint16_t* __restrict__ x,        // [rows, cols]  (GEMM output if HAS_BDA)
    const uint16_t* __restrict__ bias,     // [cols] or null
    const uint16_t* __restrict__ residual, // [rows, cols] or null
    const uint16_t* __restrict__ gamma, const uint16_t* __restrict__ beta,
    uint16_t* __restrict__ h_out,          // [rows, cols] residual stream out (HAS_BDA)
    uint16_t* __restrict__ y,              // [rows, cols]
    float* __restrict__ mean_out, float* __restrict__ rstd_out,
    int rows, int cols, float eps, uint32_t thresh, float keep_scale,
    const uint32_t* __restrict__ seed_ptr, uint32_t salt, uint64_t elem0) {
  const int lane = threadIdx.x & 63;
  const int row = __builtin_amdgcn_readfirstlane(blockIdx.x * 4 + (threadIdx.x >> 6));
  if (row >= rows) return;
  const uint32_t seed = HAS_BDA && seed_ptr ? (*seed_ptr + salt) : 0u;
  const size_t base = (size_t)row * cols;
  // Every load of the row (x, bias, residual, gamma, beta) is issued before any math:
  // one memory round trip per row instead of one per 512-column vector plus one for the
  // affine parameters.  Columns are clamped into the row and the loads unconditional;
  // lanes past the row end are masked at use and only the stores are predicated.  The
  // optional operands are zeroed through masks the optimiser cannot see through (a
  // `bias ? load : 0` select became a branch around a load issued last).
  constexpr bool EARLY = NV <= 4;  // wider rows load the affine parameters at use
  uint4 xr[NV], br[NV], rr[NV], gr[NV], er[NV];
  const uint16_t* bsrc = bias ? bias : gamma;
  const uint16_t* rsrc = residual ? residual : x;
  const uint16_t* esrc = beta ? beta : gamma;
  uint32_t bm = bias ? ~0u : 0u, rmk = residual ? ~0u : 0u, em = beta ? ~0u : 0u;
  asm volatile("" : "+v"(bm), "+v"(rmk), "+v"(em));
#pragma unroll
  for (int i = 0; i < NV; ++i) {
    const int c = min((lane + 64 * i) * 8, cols - 8);
    xr[i] = *reinterpret_cast<const uint4*>(x + base + c);
    if constexpr (HAS_BDA) {
      br[i] = *reinterpret_cast<const uint4*>(bsrc + c);
      rr[i] = *reinterpret_cast<const uint4*>(rsrc + base + c);
    }
    if constexpr (EARLY) {
      gr[i] = *reinterpret_cast<const uint4*>(gamma + c);
      if constexpr (!RMS) er[i] = *reinterpret_cast<const uint4*>(esrc + c);
    }
  }
  __builtin_amdgcn_sched_barrier(0);
  auto and4 = [](uint4 a, uint32_t m) __attribute__((always_inline)) {
    return make_uint4(a.x & m, a.y & m, a.z & m, a.w & m);
  };
  float v[NV][8];
#pragma unroll
  for (int i = 0; i < NV; ++i) {
    const int c = (lane + 64 * i) * 8;
    const bool ok = c < cols;
    unpack8(xr[i], v[i]);
    if constexpr (HAS_BDA) {
      float b[8], r[8];
      unpack8(and4(br[i], bm), b);
      unpack8(and4(rr[i], rmk), r);
      bool km[8];
      if (thresh) dropout_keep8(elem0 + base + c, seed, thresh, km);
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        float t = v[i][j] + b[j];
        if (thresh) t = km[j] ? t * keep_scale : 0.f;
        v[i][j] = r[j] + t;
      }
      // the residual stream is stored in bf16; normalise the rounded value so that
      // backward (which re-reads h_out) sees exactly the forward's input
      uint4 packed = pack8(v[i]);
      if (ok) *reinterpret_cast<uint4*>(h_out + base + c) = packed;
      unpack8(packed, v[i]);
    }
#pragma unroll
    for (int j = 0; j < 8; ++j) v[i][j] = ok ? v[i][j] : 0.f;
  }
  float mean = 0.f;
  if constexpr (!RMS) {
    float s = 0.f;
#pragma unroll
    for (int i = 0; i < NV; ++i)
#pragma unroll
      for (int j = 0; j < 8; ++j) s += v[i][j];
    mean = wave_sum(s) / (float)cols;
  }
  float ss = 0.f;
#pragma unroll
  for (int i = 0; i < NV; ++i) {
    const bool ok = (lane + 64 * i) * 8 < cols;
#pragma unroll
    for (int j = 0; j < 8; ++j) { float d = v[i][j] - mean; ss += ok ? d * d : 0.f; }
  }
  const float rstd = rsqrtf(wave_sum(ss) / (float)cols + eps);
  if (lane == 0) {
    if (!RMS) mean_out[row] = mean;
    rstd_out[row] = rstd;
  }
#pragma unroll
  for (int i = 0; i < NV; ++i) {
    const int c = (lane + 64 * i) * 8;
    if (!EARLY && c >= cols) continue;
    const int cc = min(c, cols - 8);
    float g[8], bt[8], o[8];
    unpack8(EARLY ? gr[i] : *reinterpret_cast<const uint4*>(gamma + cc), g);
    if constexpr (!RMS) unpack8(and4(EARLY ? er[i] : *reinterpret_cast<const uint4*>(esrc + cc), em), bt);
    else {
#pragma unroll
      for (int j = 0; j < 8; ++j) bt[j] = 0.f;
    }
#pragma unroll
    for (int j = 0; j < 8; ++j) o[j] = (v[i][j] - mean) * rstd * g[j] + bt[j];
    if (c < cols) *reinterpret_cast<uint4*>(y + base + c) = pack8(o);
  }
}

// Backward.  dh = dres + LN'(dy);  if dx_drop: dx = dh * mask * keep_scale.
// partial[blk][0][c] = sum dy*xhat, [1] = sum dy, [2] = sum dx.
// REG (cols <= 2048): each lane keeps its columns' running sums in registers across all
// rows it handles; the 4 waves fold them into the block's LDS slab once at the end
// (4-way LDS atomics, once per column).  Wider rows use per-row LDS atomics.
// COLS=false: row-wise part only (dh, dx); the column sums of wide rows come from
// ln_bwd_cols_kernel instead (per-element LDS atomics made cols >= 2560 ~10x slower).
template <int NV, bool RMS, bool REG, bool COLS = true, int G = (NV <= 2 ? 4 : (NV <= 4 ? 2 : 1))>
__global__ __launch_bounds__(256) void ln_bwd_kernel(
    const uint16_t* __restrict__ dy, const uint16_t* __restrict__ dres,
    const uint16_t* __restrict__ h, const float* __restrict__ mean_in,
    const float* __restrict__ rstd_in, const uint16_t* __restrict__ gamma,
    uint16_t* __restrict__ dh_out, uint16_t* __restrict__ dx_drop,
    float* __restrict__ partial, int rows, int cols, uint32_t thresh, float keep_scale,
    const uint32_t* __restrict__ seed_ptr, uint32_t salt, uint64_t elem0) {
  extern __shared__ __attribute__((aligned(16))) float slab[];  // [3][cols]
  if constexpr (!REG && COLS) {  // REG: [4 waves][3][cols] slabs, fully overwritten -> no zeroing
    for (int i = threadIdx.x; i < 3 * cols; i += blockDim.x) slab[i] = 0.f;
    __syncthreads();
  }
  const uint32_t seed = seed_ptr ? (*seed_ptr + salt) : 0u;
  const int lane = threadIdx.x & 63;
  // wave-uniform row index (scalar statistics loads and row addressing)
  const int wid = __builtin_amdgcn_readfirstlane(blockIdx.x * 4 + (threadIdx.x >> 6));
  const int nw = gridDim.x * 4;
  constexpr int NR = REG ? NV : 1;
  float g[NV][8], ag[NR][8], ab[NR][8], ax[NR][8];
#pragma unroll
  for (int i = 0; i < NV; ++i) {
    const int c = (lane + 64 * i) * 8;
    if (c < cols) unpack8(*reinterpret_cast<const uint4*>(gamma + c), g[i]);
    else {
#pragma unroll
      for (int j = 0; j < 8; ++j) g[i][j] = 0.f;
    }
  }
#pragma unroll
  for (int i = 0; i < NR; ++i)
#pragma unroll
    for (int j = 0; j < 8; ++j) { ag[i][j] = 0.f; ab[i][j] = 0.f; ax[i][j] = 0.f; }
  // Load groups: a wave issues the h / dy / dres loads (and statistics) of its next G rows
  // before any of their math, so G rows of loads are in flight per wave (the grid has one
  // wave per SIMD: each wave handles several rows to amortise its column partials, and a
  // one-row-ahead prefetch left only one row in flight at every wait).  Addresses are
  // clamped into the tensor and the loads unconditional: a `cond ? load : 0` select makes
  // the compiler wait for the load right where it is issued.
  // G is the launch's rows per wave when that is smaller (a group wider than the wave's
  // share loaded clamped duplicates of the LAST row: every wave of the grid hammering the
  // same few cache lines)
  const uint16_t* rsrc = dres ? dres : h;
  // residual-gradient mask, opaque to the optimiser: `dres ? load : 0` was turned into a
  // branch around the load, issued last and waited for with vmcnt(0) before row 0's math
  uint32_t rm = dres ? ~0u : 0u;
  asm volatile("" : "+v"(rm));
  for (int row0 = wid; row0 < rows; row0 += G * nw) {
    uint4 hb[G][NV], db[G][NV], rb[G][NV];
    float mb[G], sb[G];
#pragma unroll
    for (int k = 0; k < G; ++k) {
      const int rl = min(row0 + k * nw, rows - 1);
      const size_t b_ = (size_t)rl * cols;
      mb[k] = RMS ? 0.f : mean_in[rl];
      sb[k] = rstd_in[rl];
#pragma unroll
      for (int i = 0; i < NV; ++i) {
        const int c = min((lane + 64 * i) * 8, cols - 8);
        hb[k][i] = *reinterpret_cast<const uint4*>(h + b_ + c);
        db[k][i] = *reinterpret_cast<const uint4*>(dy + b_ + c);
        rb[k][i] = *reinterpret_cast<const uint4*>(rsrc + b_ + c);
      }
    }
    __builtin_amdgcn_sched_barrier(0);  // keep the whole group's loads ahead of its math
#pragma unroll
  for (int k = 0; k < G; ++k) {
    const int row = row0 + k * nw;
    if (row >= rows) break;
    const size_t base = (size_t)row * cols;
    const float mean = mb[k];
    const float rstd = sb[k];
    const uint4 (&hcur)[NV] = hb[k];
    const uint4 (&dcur)[NV] = db[k];
    uint4 rcur[NV];
#pragma unroll
    for (int i = 0; i < NV; ++i)
      rcur[i] = make_uint4(rb[k][i].x & rm, rb[k][i].y & rm, rb[k][i].z & rm, rb[k][i].w & rm);
    float xh[NV][8], gy[NV][8];
    float s1 = 0.f, s2 = 0.f;
#pragma unroll
    for (int i = 0; i < NV; ++i) {
      const int c = (lane + 64 * i) * 8;
      const bool ok = c < cols;
      // REG: branch-free (lanes past the row end read clamped data and contribute zeros);
      // execution-mask branches around the math made the compiler drain every load in
      // flight (vmcnt(0)) before the first store of the group
      if (REG || ok) {
        float hv[8], dv[8];
        unpack8(hcur[i], hv);
        unpack8(dcur[i], dv);
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          if constexpr (REG) dv[j] = ok ? dv[j] : 0.f;
          xh[i][j] = (hv[j] - mean) * rstd;
          gy[i][j] = dv[j] * g[i][j];
          s1 += gy[i][j];
          s2 += gy[i][j] * xh[i][j];
          if constexpr (REG) {
            ag[i][j] += dv[j] * xh[i][j];
            ab[i][j] += dv[j];
          } else if constexpr (COLS) {
            atomicAdd(&slab[c + j], dv[j] * xh[i][j]);
            atomicAdd(&slab[cols + c + j], dv[j]);
          }
        }
      } else {
#pragma unroll
        for (int j = 0; j < 8; ++j) { xh[i][j] = 0.f; gy[i][j] = 0.f; }
      }
    }
    const float m1 = RMS ? 0.f : wave_sum(s1) / (float)cols;
    const float m2 = wave_sum(s2) / (float)cols;
#pragma unroll
    for (int i = 0; i < NV; ++i) {
      const int c = (lane + 64 * i) * 8;
      const bool ok = c < cols;
      if (REG || ok) {
        float r[8], o[8];
        unpack8(rcur[i], r);   // zeros when there is no residual gradient
#pragma unroll
        for (int j = 0; j < 8; ++j) o[j] = r[j] + rstd * (gy[i][j] - m1 - xh[i][j] * m2);
        const uint4 po = pack8(o);
        if (ok) *reinterpret_cast<uint4*>(dh_out + base + c) = po;
        if (dx_drop) {
          float dx[8];
          bool km[8];
          if (thresh) dropout_keep8(elem0 + base + c, seed, thresh, km);
#pragma unroll
          for (int j = 0; j < 8; ++j) {
            float t = o[j];
            if (thresh) t = km[j] ? t * keep_scale : 0.f;
            dx[j] = t;
          }
          uint4 pk = pack8(dx);
          if (ok) *reinterpret_cast<uint4*>(dx_drop + base + c) = pk;
          if constexpr (COLS) {
            float dxr[8];
            unpack8(pk, dxr);
#pragma unroll
            for (int j = 0; j < 8; ++j) {
              if constexpr (REG) ax[i][j] += ok ? dxr[j] : 0.f;
              else atomicAdd(&slab[2 * cols + c + j], dxr[j]);
            }
          }
        }
      }
    }
  }
  }
  if constexpr (!COLS) return;
  float* out = partial + (size_t)blockIdx.x * 3 * cols;
  if constexpr (REG) {
    // every wave stores its register partials into its OWN slab with plain 16-B LDS
    // stores (cross-wave ds_add_f32 atomics serialised the issue: SQ_WAIT_INST_LDS was
    // ~half of all wave cycles), then the block folds the 4 slabs
    float* my = slab + (threadIdx.x >> 6) * 3 * cols;
#pragma unroll
    for (int i = 0; i < NV; ++i) {
      const int c = (lane + 64 * i) * 8;
      if (c < cols) {
#pragma unroll
        for (int j = 0; j < 8; j += 4) {
          *reinterpret_cast<float4*>(my + c + j) = make_float4(ag[i][j], ag[i][j + 1], ag[i][j + 2], ag[i][j + 3]);
          *reinterpret_cast<float4*>(my + cols + c + j) = make_float4(ab[i][j], ab[i][j + 1], ab[i][j + 2], ab[i][j + 3]);
          *reinterpret_cast<float4*>(my + 2 * cols + c + j) = make_float4(ax[i][j], ax[i][j + 1], ax[i][j + 2], ax[i][j + 3]);
        }
      }
    }
    __syncthreads();
    for (int i = threadIdx.x; i < 3 * cols; i += blockDim.x)
      out[i] = (slab[i] + slab[3 * cols + i]) + (slab[6 * cols + i] + slab[9 * cols + i]);
  } else {
    __syncthreads();
    for (int i = threadIdx.x; i < 3 * cols; i += blockDim.x) out[i] = slab[i];
  }
}

}  // namespace

// Deterministic two-level column reduction of fp32 partials [P][C] (shared by every
// kernel that produces per-block column partials: LN/BDA backward, bias-GeLU backward,
// bias column sums):
//   level 1: groups of 64 partial rows -> [ceil(P/64)][C]  (grid C/256 x P/64)
//   level 2: fold the groups, write bf16 (optionally adding); flat column c of the
//            [nvec][cols] layout goes to output k = c / cols.
namespace {
// One-launch deterministic column reduction of fp32 partial rows [P][nvec*cols] into up to
// three bf16 vectors.  Block = 4 waves over 16 columns: thread t sums column t & 15 over the
// rows of phase t >> 4 (rows ph, ph + 16, ...; 8 loads in flight, 64-B row segments), then
// the 16 phase sums are folded in LDS in a fixed order.  16 columns per block give
// C / 16 workgroups (192 for a 3 x 1024 LN backward): 64 columns per block left all but
// 48 CUs idle on these ~3-6 MB reductions.
__global__ __launch_bounds__(256) void colreduce_kernel(const float* __restrict__ in, int P, int cols, int nvec,
                                                        uint16_t* __restrict__ o0, uint16_t* __restrict__ o1,
                                                        uint16_t* __restrict__ o2, int accumulate) {
  __shared__ float part[16][17];
  const int C = nvec * cols;
  const int cl = threadIdx.x & 15, ph = threadIdx.x >> 4;
  const int c = blockIdx.x * 16 + cl;
  float a[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  if (c < C) {
    int p = ph;
    for (; p + 112 < P; p += 128) {
#pragma unroll
      for (int j = 0; j < 8; ++j) a[j] += in[(size_t)(p + 16 * j) * C + c];
    }
    for (; p < P; p += 16) a[0] += in[(size_t)p * C + c];
  }
  part[ph][cl] = ((a[0] + a[1]) + (a[2] + a[3])) + ((a[4] + a[5]) + (a[6] + a[7]));
  __syncthreads();
  if (ph == 0 && c < C) {
    const int lane = cl;
    float t = 0.f;
#pragma unroll
    for (int k = 0; k < 16; ++k) t += part[k][lane];
    const int k = c / cols, cc = c % cols;
    uint16_t* o = k == 0 ? o0 : (k == 1 ? o1 : o2);
    if (o) {
      if (accumulate) t += bf2f(o[cc]);
      o[cc] = f2bf(t);
    }
  }
}

// Batched deferred column reductions (ops/norm.py ColReduceQueue): every norm / bias
// column-sum of a training step, folded at the end of backward in ONE launch instead of one
// colreduce launch per producer (~100 per GPT-2 step).  Job j (int64 x 9): {partials
// [P][C] fp32, P, C = nvec * cols, cols, out0, out1, out2 (bf16, nullable), accumulate,
// first block}; block b serves 16 columns of the job whose block range holds b (same
// fixed-order summation as colreduce_kernel).
__global__ __launch_bounds__(256) void colreduce_batched_kernel(const int64_t* __restrict__ tab, int njobs) {
  // block = 64 columns: thread t reads float4 (columns 4 (t & 15) ..) of rows t >> 4, + 16, ...
  // (16-B loads: these ~330 MB of partials per GPT-2 step stream from HBM)
  __shared__ float4 part[16][17];
  const int b = blockIdx.x;
  int lo = 0, hi = njobs - 1;
  while (lo < hi) {   // last job whose first block <= b
    const int mid = (lo + hi + 1) >> 1;
    if ((int)tab[9 * mid + 8] <= b) lo = mid;
    else hi = mid - 1;
  }
  const int64_t* J = tab + 9 * lo;
  const float* in = reinterpret_cast<const float*>(J[0]);
  const int P = (int)J[1], C = (int)J[2], cols = (int)J[3];
  const int q = threadIdx.x & 15, ph = threadIdx.x >> 4;
  const int c0 = (b - (int)J[8]) * 64 + 4 * q;     // C % 4 == 0 (host-checked)
  float4 a[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) a[j] = make_float4(0.f, 0.f, 0.f, 0.f);
  if (c0 < C) {
    int p = ph;
    for (; p + 112 < P; p += 128) {
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const float4 v = *reinterpret_cast<const float4*>(in + (size_t)(p + 16 * j) * C + c0);
        a[j].x += v.x; a[j].y += v.y; a[j].z += v.z; a[j].w += v.w;
      }
    }
    for (; p < P; p += 16) {
      const float4 v = *reinterpret_cast<const float4*>(in + (size_t)p * C + c0);
      a[0].x += v.x; a[0].y += v.y; a[0].z += v.z; a[0].w += v.w;
    }
  }
  float4 t4;
  t4.x = ((a[0].x + a[1].x) + (a[2].x + a[3].x)) + ((a[4].x + a[5].x) + (a[6].x + a[7].x));
  t4.y = ((a[0].y + a[1].y) + (a[2].y + a[3].y)) + ((a[4].y + a[5].y) + (a[6].y + a[7].y));
  t4.z = ((a[0].z + a[1].z) + (a[2].z + a[3].z)) + ((a[4].z + a[5].z) + (a[6].z + a[7].z));
  t4.w = ((a[0].w + a[1].w) + (a[2].w + a[3].w)) + ((a[4].w + a[5].w) + (a[6].w + a[7].w));
  part[ph][q] = t4;
  __syncthreads();
  // 64 columns: thread t < 64 folds column t (16 phases in fixed order)
  if (threadIdx.x < 64) {
    const int cl = threadIdx.x, c = (b - (int)J[8]) * 64 + cl;
    if (c < C) {
      float t = 0.f;
#pragma unroll
      for (int k = 0; k < 16; ++k) {
        const float4 v = part[k][cl >> 2];
        t += (cl & 3) == 0 ? v.x : (cl & 3) == 1 ? v.y : (cl & 3) == 2 ? v.z : v.w;
      }
      const int k = c / cols, cc = c - k * cols;
      uint16_t* o = reinterpret_cast<uint16_t*>(k == 0 ? J[4] : (k == 1 ? J[5] : J[6]));
      if (o) {
        if (J[7]) t += bf2f(o[cc]);
        o[cc] = f2bf(t);
      }
    }
  }
}

// Column sum of a bf16 matrix [rows, cols] -> fp32 partials [rows/64][cols]
__global__ __launch_bounds__(256) void colsum_partial_kernel(
    const uint16_t* __restrict__ x, int rows, int cols, int rows_per_block,
    float* __restrict__ partial) {
  const int c = (blockIdx.x * 256 + threadIdx.x) * 8;
  const int r0 = blockIdx.y * rows_per_block;
  if (c >= cols) return;
  float acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  const int r1 = min(rows, r0 + rows_per_block);
  // G rows per group, their loads issued together and unconditionally (rows clamped into
  // the block, the overhang masked after): a `r < r1 ? load : 0` select made the compiler
  // wait for each load where it was issued
  constexpr int G = 8;
  for (int r = r0; r < r1; r += G) {
    uint4 raw[G];
#pragma unroll
    for (int u = 0; u < G; ++u)
      raw[u] = *reinterpret_cast<const uint4*>(x + (size_t)min(r + u, r1 - 1) * cols + c);
#pragma unroll
    for (int u = 0; u < G; ++u) {
      float v[8];
      unpack8(raw[u], v);
      const float m = r + u < r1 ? 1.f : 0.f;
#pragma unroll
      for (int j = 0; j < 8; ++j) acc[j] += v[j] * m;
    }
  }
  float* o = partial + (size_t)blockIdx.y * cols + c;
#pragma unroll
  for (int j = 0; j < 8; ++j) o[j] = acc[j];
}

template <bool RMS, bool BDA>
hipError_t launch_fwd(const void* x, const void* bias, const void* residual,
                      const void* gamma, const void* beta, void* h_out, void* y,
                      float* mean, float* rstd, int rows, int cols, float eps,
                      float p, const uint32_t* seed, uint32_t salt, uint64_t elem0, hipStream_t s) {
  if (cols < 8 || cols % 8 || rows <= 0) return hipErrorInvalidValue;  // 16-B row vectors
  const int nv = (cols + 511) / 512;
  const uint32_t thresh = p > 0.f ? (uint32_t)((double)p * 4294967296.0) : 0u;
  const float ks = p > 0.f ? 1.f / (1.f - p) : 1.f;
  dim3 grid((rows + 3) / 4), block(256);
#define MX_LN_CASE(N)                                                                  \
  case N:                                                                              \
    hipLaunchKernelGGL((ln_fwd_kernel<N, RMS, BDA>), grid, block, 0, s,                \
                       (const uint16_t*)x, (const uint16_t*)bias,                      \
                       (const uint16_t*)residual, (const uint16_t*)gamma,              \
                       (const uint16_t*)beta, (uint16_t*)h_out, (uint16_t*)y, mean,    \
                       rstd, rows, cols, eps, thresh, ks, seed, salt, elem0);          \
    break;
  switch (nv) {
    MX_LN_CASE(1) MX_LN_CASE(2) MX_LN_CASE(3) MX_LN_CASE(4) MX_LN_CASE(5)
    MX_LN_CASE(6) MX_LN_CASE(8) MX_LN_CASE(10) MX_LN_CASE(12) MX_LN_CASE(16)
    default: return hipErrorInvalidValue;
  }
#undef MX_LN_CASE
  return hipGetLastError();
}

// Column sums of the LN backward for wide rows: partial[blk.y][0|1|2][c] over the
// block's row stripe of  dy * xhat,  dy,  dx  (xhat recomputed from h, mean, rstd; dx
// re-read in bf16, exactly the values written).  Lane = 8 consecutive columns, 16-B loads.
template <bool RMS>
__global__ __launch_bounds__(256) void ln_bwd_cols_kernel(
    const uint16_t* __restrict__ dy, const uint16_t* __restrict__ h,
    const float* __restrict__ mean_in, const float* __restrict__ rstd_in,
    const uint16_t* __restrict__ dx, float* __restrict__ partial, int rows, int cols,
    int rows_per_block) {
  const int c = (blockIdx.x * 256 + threadIdx.x) * 8;
  if (c >= cols) return;
  const int r0 = blockIdx.y * rows_per_block;
  const int r1 = min(rows, r0 + rows_per_block);
  float ag[8] = {0, 0, 0, 0, 0, 0, 0, 0}, ab[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  float ax[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  for (int r = r0; r < r1; ++r) {
    const size_t off = (size_t)r * cols + c;
    const float mean = RMS ? 0.f : mean_in[r];
    const float rstd = rstd_in[r];
    float hv[8], dv[8];
    unpack8(*reinterpret_cast<const uint4*>(h + off), hv);
    unpack8(*reinterpret_cast<const uint4*>(dy + off), dv);
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      ag[j] += dv[j] * ((hv[j] - mean) * rstd);
      ab[j] += dv[j];
    }
    if (dx) {
      float xv[8];
      unpack8(*reinterpret_cast<const uint4*>(dx + off), xv);
#pragma unroll
      for (int j = 0; j < 8; ++j) ax[j] += xv[j];
    }
  }
  float* out = partial + (size_t)blockIdx.y * 3 * cols;
#pragma unroll
  for (int j = 0; j < 8; j += 4) {
    *reinterpret_cast<float4*>(out + c + j) = make_float4(ag[j], ag[j + 1], ag[j + 2], ag[j + 3]);
    *reinterpret_cast<float4*>(out + cols + c + j) = make_float4(ab[j], ab[j + 1], ab[j + 2], ab[j + 3]);
    *reinterpret_cast<float4*>(out + 2 * cols + c + j) = make_float4(ax[j], ax[j + 1], ax[j + 2], ax[j + 3]);
  }
}

// Row-wise part of the backward for wide rows (cols > kSplitCols: GPT-3 6.7B's h = 4096), the
// column sums coming from ln_bwd_cols_kernel.  One row per wave.  h / dy / dres / gamma stay
// packed bf16 in registers (4 VGPRs per 8 columns) and xhat, gamma * dy are recomputed in the
// second pass: ln_bwd_kernel holds them as fp32 row arrays, 256 VGPRs at NV = 8 -- one wave
// per SIMD, so a wave's loads and its stores never overlapped another wave's (~60 % of the
// HBM bandwidth at 4096 x 4096).
template <int NV, bool RMS>
__global__ __launch_bounds__(256) void ln_bwd_wide_kernel(
    const uint16_t* __restrict__ dy, const uint16_t* __restrict__ dres,
    const uint16_t* __restrict__ h, const float* __restrict__ mean_in,
    const float* __restrict__ rstd_in, const uint16_t* __restrict__ gamma,
    uint16_t* __restrict__ dh_out, uint16_t* __restrict__ dx_drop, int rows, int cols,
    uint32_t thresh, float keep_scale, const uint32_t* __restrict__ seed_ptr, uint32_t salt,
    uint64_t elem0) {
  const int lane = threadIdx.x & 63;
  const int row = __builtin_amdgcn_readfirstlane(blockIdx.x * 4 + (threadIdx.x >> 6));
  if (row >= rows) return;
  const uint32_t seed = seed_ptr ? (*seed_ptr + salt) : 0u;
  const size_t base = (size_t)row * cols;
  const uint16_t* rsrc = dres ? dres : h;
  uint32_t rm = dres ? ~0u : 0u;   // (opaque mask: see ln_bwd_kernel)
  asm volatile("" : "+v"(rm));
  uint4 hb[NV], db[NV], rb[NV], gb[NV];
#pragma unroll
  for (int i = 0; i < NV; ++i) {
    const int c = min((lane + 64 * i) * 8, cols - 8);
    hb[i] = *reinterpret_cast<const uint4*>(h + base + c);
    db[i] = *reinterpret_cast<const uint4*>(dy + base + c);
    gb[i] = *reinterpret_cast<const uint4*>(gamma + c);
    rb[i] = *reinterpret_cast<const uint4*>(rsrc + base + c);
  }
  const float mean = RMS ? 0.f : mean_in[row];
  const float rstd = rstd_in[row];
  __builtin_amdgcn_sched_barrier(0);
  float s1 = 0.f, s2 = 0.f;
#pragma unroll
  for (int i = 0; i < NV; ++i) {
    const bool ok = (lane + 64 * i) * 8 < cols;
    float hv[8], dv[8], g[8];
    unpack8(hb[i], hv);
    unpack8(db[i], dv);
    unpack8(gb[i], g);
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const float gy = ok ? dv[j] * g[j] : 0.f;
      s1 += gy;
      s2 += gy * ((hv[j] - mean) * rstd);
    }
  }
  const float m1 = RMS ? 0.f : wave_sum(s1) / (float)cols;
  const float m2 = wave_sum(s2) / (float)cols;
  // opaque to the optimiser: otherwise it keeps the first pass's unpacked fp32 values alive
  // across the reductions for reuse below (256 VGPRs again) instead of re-unpacking
#pragma unroll
  for (int i = 0; i < NV; ++i) {
    asm volatile("" : "+v"(hb[i].x), "+v"(hb[i].y), "+v"(hb[i].z), "+v"(hb[i].w));
    asm volatile("" : "+v"(db[i].x), "+v"(db[i].y), "+v"(db[i].z), "+v"(db[i].w));
    asm volatile("" : "+v"(gb[i].x), "+v"(gb[i].y), "+v"(gb[i].z), "+v"(gb[i].w));
  }
#pragma unroll
  for (int i = 0; i < NV; ++i) {
    const int c = (lane + 64 * i) * 8;
    const bool ok = c < cols;
    float hv[8], dv[8], g[8], r[8], o[8];
    unpack8(hb[i], hv);
    unpack8(db[i], dv);
    unpack8(gb[i], g);
    unpack8(make_uint4(rb[i].x & rm, rb[i].y & rm, rb[i].z & rm, rb[i].w & rm), r);
#pragma unroll
    for (int j = 0; j < 8; ++j) o[j] = r[j] + rstd * (dv[j] * g[j] - m1 - ((hv[j] - mean) * rstd) * m2);
    if (ok) *reinterpret_cast<uint4*>(dh_out + base + c) = pack8(o);
    if (dx_drop) {
      bool km[8];
      if (thresh) dropout_keep8(elem0 + base + c, seed, thresh, km);
#pragma unroll
      for (int j = 0; j < 8; ++j) o[j] = thresh ? (km[j] ? o[j] * keep_scale : 0.f) : o[j];
      if (ok) *reinterpret_cast<uint4*>(dx_drop + base + c) = pack8(o);
    }
  }
}

constexpr int kSplitCols = 2048;   // wider rows: row kernel without column sums + column kernel
constexpr int kColsRowsPerBlock = 32;

// rows per wave of the fused backward: 2 (BDA-LN at 4096 x 1024 with its column reduction,
// profiles/r5_s1/ln_ab_rows_per_wave.txt: 16.0 us at 2, 17.2 at 4, 16.2 at 1 -- with load groups, two waves per
// SIMD hide each other's dropout-hash VALU better than the halved partials save)
constexpr int kBwdRowsPerWave = 2;
constexpr int kBwdMaxBlocks = 512;   // partial slabs: [blocks][3][cols] fp32
int bwd_grid(int rows) {
  const int rpb = 4 * kBwdRowsPerWave;
  int g = (rows + rpb - 1) / rpb;
  if (g > kBwdMaxBlocks) g = kBwdMaxBlocks;
  if (g < 1) g = 1;
  return g;
}

template <bool RMS>
hipError_t launch_bwd(const void* dy, const void* dres, const void* h, const float* mean,
                      const float* rstd, const void* gamma, void* dh_out, void* dx_drop,
                      float* partial, int rows, int cols, float p, const uint32_t* seed,
                      uint32_t salt, uint64_t elem0, hipStream_t s) {
  if (cols < 8 || cols % 8 || rows <= 0) return hipErrorInvalidValue;  // 16-B row vectors
  const int nv = (cols + 511) / 512;
  const uint32_t thresh = p > 0.f ? (uint32_t)((double)p * 4294967296.0) : 0u;
  const float ks = p > 0.f ? 1.f / (1.f - p) : 1.f;
  dim3 grid(bwd_grid(rows)), block(256);
  if (cols > kSplitCols) {
    // row-wise pass (no LDS, one row per wave), then the column sums in a column-parallel pass
#define MX_LNB_SPLIT(N)                                                                \
  case N:                                                                              \
    hipLaunchKernelGGL((ln_bwd_wide_kernel<N, RMS>), dim3((rows + 3) / 4), block, 0, s, \
                       (const uint16_t*)dy, (const uint16_t*)dres, (const uint16_t*)h, \
                       mean, rstd, (const uint16_t*)gamma, (uint16_t*)dh_out,          \
                       (uint16_t*)dx_drop, rows, cols, thresh, ks, seed, salt, elem0); \
    break;
    switch (nv) {
      MX_LNB_SPLIT(1) MX_LNB_SPLIT(2) MX_LNB_SPLIT(3) MX_LNB_SPLIT(4)
      MX_LNB_SPLIT(5) MX_LNB_SPLIT(6) MX_LNB_SPLIT(7) MX_LNB_SPLIT(8) MX_LNB_SPLIT(10)
      MX_LNB_SPLIT(12) MX_LNB_SPLIT(16)
      default: return hipErrorInvalidValue;
    }
#undef MX_LNB_SPLIT
    if (partial) {
      dim3 cg((cols / 8 + 255) / 256, (rows + kColsRowsPerBlock - 1) / kColsRowsPerBlock);
      hipLaunchKernelGGL(ln_bwd_cols_kernel<RMS>, cg, dim3(256), 0, s, (const uint16_t*)dy,
                         (const uint16_t*)h, mean, rstd, (const uint16_t*)dx_drop, partial, rows,
                         cols, kColsRowsPerBlock);
    }
    return hipGetLastError();
  }
  const size_t lds = (size_t)(nv <= 4 ? 12 : 3) * cols * sizeof(float);
  const int rpw = (rows + grid.x * 4 - 1) / (grid.x * 4);   // rows per wave of this launch
#define MX_LNB_LAUNCH(N, GG)                                                           \
    hipLaunchKernelGGL((ln_bwd_kernel<N, RMS, (N <= 4), true, GG>), grid, block, lds, s, \
                       (const uint16_t*)dy, (const uint16_t*)dres, (const uint16_t*)h, \
                       mean, rstd, (const uint16_t*)gamma, (uint16_t*)dh_out,          \
                       (uint16_t*)dx_drop, partial, rows, cols, thresh, ks, seed,      \
                       salt, elem0);
#define MX_LNB_CASE(N)                                                                 \
  case N:                                                                              \
    if ((N) <= 2 && rpw >= 4) { MX_LNB_LAUNCH(N, 4) }                                  \
    else if ((N) <= 4 && rpw >= 2) { MX_LNB_LAUNCH(N, 2) }                             \
    else { MX_LNB_LAUNCH(N, 1) }                                                       \
    break;
  switch (nv) {
    MX_LNB_CASE(1) MX_LNB_CASE(2) MX_LNB_CASE(3) MX_LNB_CASE(4) MX_LNB_CASE(5)
    MX_LNB_CASE(6) MX_LNB_CASE(8) MX_LNB_CASE(10) MX_LNB_CASE(12) MX_LNB_CASE(16)
    default: return hipErrorInvalidValue;
  }
#undef MX_LNB_CASE
#undef MX_LNB_LAUNCH
  return hipGetLastError();
}

}  // namespace

// number of partial slabs the norm backward writes (caller sizes `partial`)
MX_EXPORT int mx_norm_bwd_nparts(int rows) { return bwd_grid(rows); }
MX_EXPORT int mx_norm_bwd_nparts2(int rows, int cols) {
  return cols > kSplitCols ? (rows + kColsRowsPerBlock - 1) / kColsRowsPerBlock : bwd_grid(rows);
}
// floats of level-1 scratch needed to finalize P partial rows of C columns
MX_EXPORT int64_t mx_colreduce_scratch(int P, int C) { return (int64_t)((P + 63) / 64) * C; }

// fold fp32 partials [P][nvec*cols] into up to three bf16 outputs (deterministic)
MX_EXPORT int mx_colsum_finalize(const float* partial, int nparts, int cols, int nvec,
                                 void* o0, void* o1, void* o2, int accumulate, float* scratch,
                                 hipStream_t s) {
  (void)scratch;  // single-level reduction: no scratch needed (kept for ABI stability)
  const int C = nvec * cols;
  hipLaunchKernelGGL(colreduce_kernel, dim3((C + 15) / 16), dim3(256), 0, s, partial, nparts, cols, nvec,
                     (uint16_t*)o0, (uint16_t*)o1, (uint16_t*)o2, accumulate);
  return hipGetLastError();
}

MX_EXPORT int mx_layernorm_fwd(const void* x, const void* gamma, const void* beta, void* y,
                               float* mean, float* rstd, int rows, int cols, float eps,
                               hipStream_t s) {
  return launch_fwd<false, false>(x, nullptr, nullptr, gamma, beta, nullptr, y, mean, rstd,
                                  rows, cols, eps, 0.f, nullptr, 0, 0, s);
}

MX_EXPORT int mx_rmsnorm_fwd(const void* x, const void* gamma, void* y, float* rstd,
                             int rows, int cols, float eps, hipStream_t s) {
  return launch_fwd<true, false>(x, nullptr, nullptr, gamma, nullptr, nullptr, y, nullptr,
                                 rstd, rows, cols, eps, 0.f, nullptr, 0, 0, s);
}

// h_out = residual + dropout(x + bias);  y = LayerNorm(h_out)   (RMS: RMSNorm)
// elem0: flat index of element [0, 0] in the full (unsharded) activation -- the dropout
// mask is keyed on the GLOBAL element index, so a sequence-parallel shard draws exactly
// the bits of the same rows of the unsharded tensor
MX_EXPORT int mx_bda_norm_fwd(const void* x, const void* bias, const void* residual,
                              const void* gamma, const void* beta, void* h_out, void* y,
                              float* mean, float* rstd, int rows, int cols, float eps,
                              float p, const uint32_t* seed, uint32_t salt, int64_t elem0, int rms,
                              hipStream_t s) {
  if (rms)
    return launch_fwd<true, true>(x, bias, residual, gamma, nullptr, h_out, y, nullptr,
                                  rstd, rows, cols, eps, p, seed, salt, (uint64_t)elem0, s);
  return launch_fwd<false, true>(x, bias, residual, gamma, beta, h_out, y, mean, rstd, rows,
                                 cols, eps, p, seed, salt, (uint64_t)elem0, s);
}

MX_EXPORT int mx_norm_bwd(const void* dy, const void* dres, const void* h, const float* mean,
                          const float* rstd, const void* gamma, void* dh_out, void* dx_drop,
                          float* partial, int rows, int cols, float p, const uint32_t* seed,
                          uint32_t salt, int64_t elem0, int rms, hipStream_t s) {
  if (rms)
    return launch_bwd<true>(dy, dres, h, mean, rstd, gamma, dh_out, dx_drop, partial, rows,
                            cols, p, seed, salt, (uint64_t)elem0, s);
  return launch_bwd<false>(dy, dres, h, mean, rstd, gamma, dh_out, dx_drop, partial, rows,
                           cols, p, seed, salt, (uint64_t)elem0, s);
}

// bf16 column sum: `partial` must hold ceil(rows/16)*cols floats plus
// mx_colreduce_scratch(ceil(rows/16), cols) floats of scratch behind it
MX_EXPORT int mx_colsum_bf16(const void* x, int rows, int cols, float* partial, void* out,
                             int accumulate, hipStream_t s) {
  const int rpb = 16;  // 4x more blocks than 64-row stripes: the loads need the parallelism
  dim3 grid((cols / 8 + 255) / 256, (rows + rpb - 1) / rpb);
  hipLaunchKernelGGL(colsum_partial_kernel, grid, dim3(256), 0, s, (const uint16_t*)x, rows,
                     cols, rpb, partial);
  const int nparts = grid.y;
  return mx_colsum_finalize(partial, nparts, cols, 1, out, nullptr, nullptr, accumulate,
                            partial + (size_t)nparts * cols, s);
}

// deferred-reduction table (see colreduce_batched_kernel); total_blocks = sum ceil(C / 64)
MX_EXPORT int mx_colreduce_batched(const int64_t* table, int njobs, int total_blocks, hipStream_t s) {
  if (njobs <= 0 || total_blocks <= 0) return hipSuccess;
  hipLaunchKernelGGL(colreduce_batched_kernel, dim3(total_blocks), dim3(256), 0, s, table, njobs);
  return hipGetLastError();
}

// bf16 column-sum partials only ([ceil(rows / 16)][cols] fp32; the finalize is deferred)
MX_EXPORT int mx_colsum_partial_bf16(const void* x, int rows, int cols, float* partial, hipStream_t s) {
  const int rpb = 16;
  dim3 grid((cols / 8 + 255) / 256, (rows + rpb - 1) / rpb);
  hipLaunchKernelGGL(colsum_partial_kernel, grid, dim3(256), 0, s, (const uint16_t*)x, rows, cols, rpb, partial);
  return hipGetLastError();
}
