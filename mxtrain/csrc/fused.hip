// Fused elementwise / reduction kernels of the GPT / BERT training step:
//   * bias + GeLU (tanh) forward and backward with fused dbias column reduction   (K6)
//   * token + position embedding gather, deterministic embedding backward          (K11)
//   * softmax cross-entropy: row statistics + gradient, vocab-parallel capable     (K10)
// Replaces Megatron `bias_gelu_impl`, `VocabParallelEmbedding` and
// `vocab_parallel_cross_entropy` (reference pins: containers/megatron-deepspeed/
// Dockerfile:13).  All bf16 traffic is 16-B vectorised.
#include "common.h"

using namespace mx;

namespace {

// ---------------------------------------------------------------- bias + GeLU
// Each thread handles FV 16-B vectors 256 apart (coalesced), all loads issued before the
// math: with one load in flight per thread the kernel could not cover HBM latency.
constexpr int kGeluFV = 2;
__global__ __launch_bounds__(256) void bias_gelu_fwd_kernel(
    const uint16_t* __restrict__ x, const uint16_t* __restrict__ bias,
    uint16_t* __restrict__ y, int64_t n, int cols, int cmask) {
  const int64_t nvec = n / 8;
  const int64_t v0 = (int64_t)blockIdx.x * (256 * kGeluFV) + threadIdx.x;
  uint4 raw[kGeluFV], braw[kGeluFV];
#pragma unroll
  for (int u = 0; u < kGeluFV; ++u) {
    const int64_t v = v0 + 256 * u;
    if (v < nvec) {
      raw[u] = *reinterpret_cast<const uint4*>(x + v * 8);
      // bias column: a mask for power-of-two widths (every GPT / LLaMA FFN here); the
      // 64-bit modulo otherwise (a software division: ~50 VALU per vector)
      const int bc = cmask >= 0 ? (int)(v * 8) & cmask : (int)((v * 8) % cols);
      braw[u] = *reinterpret_cast<const uint4*>(bias + bc);
    }
  }
#pragma unroll
  for (int u = 0; u < kGeluFV; ++u) {
    const int64_t v = v0 + 256 * u;
    if (v < nvec) {
      float a[8], b[8], o[8];
      unpack8(raw[u], a);
      unpack8(braw[u], b);
#pragma unroll
      for (int j = 0; j < 8; ++j) o[j] = gelu_tanh(a[j] + b[j]);
      *reinterpret_cast<uint4*>(y + v * 8) = pack8(o);
    }
  }
}

// dx = dy * gelu'(x + b); partial[blockIdx.y][c] = sum over the block's rows of dx.
// Rows in groups of 4 with the group's 8 loads issued first (memory-level parallelism).
__global__ __launch_bounds__(256) void bias_gelu_bwd_kernel(
    const uint16_t* __restrict__ dy, const uint16_t* __restrict__ x,
    const uint16_t* __restrict__ bias, uint16_t* __restrict__ dx, int rows, int cols,
    int rows_per_block, float* __restrict__ partial) {
  const int c = (blockIdx.x * 256 + threadIdx.x) * 8;
  if (c >= cols) return;
  const int r0 = blockIdx.y * rows_per_block;
  const int r1 = min(rows, r0 + rows_per_block);
  float b[8], acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  unpack8(*reinterpret_cast<const uint4*>(bias + c), b);
  constexpr int G = 4;
  for (int r = r0; r < r1; r += G) {
    uint4 gr[G], ar[G];
#pragma unroll
    for (int u = 0; u < G; ++u) {
      if (r + u < r1) {
        const size_t off = (size_t)(r + u) * cols + c;
        gr[u] = *reinterpret_cast<const uint4*>(dy + off);
        ar[u] = *reinterpret_cast<const uint4*>(x + off);
      }
    }
#pragma unroll
    for (int u = 0; u < G; ++u) {
      if (r + u < r1) {
        const size_t off = (size_t)(r + u) * cols + c;
        float g[8], a[8], o[8];
        unpack8(gr[u], g);
        unpack8(ar[u], a);
#pragma unroll
        for (int j = 0; j < 8; ++j) o[j] = g[j] * gelu_tanh_grad(a[j] + b[j]);
        uint4 pk = pack8(o);
        *reinterpret_cast<uint4*>(dx + off) = pk;
        unpack8(pk, o);
#pragma unroll
        for (int j = 0; j < 8; ++j) acc[j] += o[j];
      }
    }
  }
  float* p = partial + (size_t)blockIdx.y * cols + c;
#pragma unroll
  for (int j = 0; j < 8; ++j) p[j] = acc[j];
}

// ---------------------------------------------------------------- bias + SwiGLU
// pre = [a | b] (each `f` columns, Megatron --swiglu layout); y = silu(a + ba) * (b + bb)
__device__ __forceinline__ float silu_f(float x) {
  return x * __builtin_amdgcn_rcpf(1.f + __expf(-x));
}
__global__ __launch_bounds__(256) void bias_swiglu_fwd_kernel(
    const uint16_t* __restrict__ pre, const uint16_t* __restrict__ bias,
    uint16_t* __restrict__ y, int rows, int f) {
  const int nv = f / 8;
  const int64_t total = (int64_t)rows * nv;
  for (int64_t w = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; w < total;
       w += (int64_t)gridDim.x * blockDim.x) {
    const int r = (int)(w / nv);
    const int c = (int)(w % nv) * 8;
    const uint16_t* row = pre + (size_t)r * 2 * f;
    float a[8], b[8], o[8];
    unpack8(*reinterpret_cast<const uint4*>(row + c), a);
    unpack8(*reinterpret_cast<const uint4*>(row + f + c), b);
    if (bias) {
      float ba[8], bb[8];
      unpack8(*reinterpret_cast<const uint4*>(bias + c), ba);
      unpack8(*reinterpret_cast<const uint4*>(bias + f + c), bb);
#pragma unroll
      for (int j = 0; j < 8; ++j) { a[j] += ba[j]; b[j] += bb[j]; }
    }
#pragma unroll
    for (int j = 0; j < 8; ++j) o[j] = silu_f(a[j]) * b[j];
    *reinterpret_cast<uint4*>(y + (size_t)r * f + c) = pack8(o);
  }
}

// da = dy * b * silu'(a), db = dy * silu(a); partial[blockIdx.y][0..2f) = row-block sums
__global__ __launch_bounds__(256) void bias_swiglu_bwd_kernel(
    const uint16_t* __restrict__ dy, const uint16_t* __restrict__ pre,
    const uint16_t* __restrict__ bias, uint16_t* __restrict__ dpre, int rows, int f,
    int rows_per_block, float* __restrict__ partial) {
  const int c = (blockIdx.x * 256 + threadIdx.x) * 8;
  if (c >= f) return;
  const int r0 = blockIdx.y * rows_per_block;
  const int r1 = min(rows, r0 + rows_per_block);
  float ba[8] = {0, 0, 0, 0, 0, 0, 0, 0}, bb[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  if (bias) {
    unpack8(*reinterpret_cast<const uint4*>(bias + c), ba);
    unpack8(*reinterpret_cast<const uint4*>(bias + f + c), bb);
  }
  float acca[8] = {0, 0, 0, 0, 0, 0, 0, 0}, accb[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  for (int r = r0; r < r1; ++r) {
    const uint16_t* row = pre + (size_t)r * 2 * f;
    float g[8], a[8], b[8], da[8], db[8];
    unpack8(*reinterpret_cast<const uint4*>(dy + (size_t)r * f + c), g);
    unpack8(*reinterpret_cast<const uint4*>(row + c), a);
    unpack8(*reinterpret_cast<const uint4*>(row + f + c), b);
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const float x = a[j] + ba[j], v = b[j] + bb[j];
      const float sg = __builtin_amdgcn_rcpf(1.f + __expf(-x));
      const float sl = x * sg;
      da[j] = g[j] * v * (sg + sl * (1.f - sg));
      db[j] = g[j] * sl;
    }
    uint4 pa = pack8(da), pb = pack8(db);
    uint16_t* drow = dpre + (size_t)r * 2 * f;
    *reinterpret_cast<uint4*>(drow + c) = pa;
    *reinterpret_cast<uint4*>(drow + f + c) = pb;
    unpack8(pa, da);
    unpack8(pb, db);
#pragma unroll
    for (int j = 0; j < 8; ++j) { acca[j] += da[j]; accb[j] += db[j]; }
  }
  float* p = partial + (size_t)blockIdx.y * 2 * f;
#pragma unroll
  for (int j = 0; j < 8; ++j) { p[c + j] = acca[j]; p[f + c + j] = accb[j]; }
}

// ---------------------------------------------------------------- embedding
// out[t] = wte[ids[t] - vocab_start] (+ wpe[t % seq]); rows outside the local vocab
// shard are zero (vocab-parallel embedding; the TP all-reduce sums the shards).
__global__ __launch_bounds__(256) void embed_fwd_kernel(
    const int64_t* __restrict__ ids, const uint16_t* __restrict__ wte,
    const uint16_t* __restrict__ wpe, uint16_t* __restrict__ out, int ntok, int hidden,
    int seq, int64_t vocab_start, int64_t vocab_end, int pos_offset) {
  const int lane = threadIdx.x & 63;
  const int t = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (t >= ntok) return;
  const int64_t id = ids[t];
  const bool in = id >= vocab_start && id < vocab_end;
  const int pos = (t % seq) + pos_offset;
  for (int c = lane * 8; c < hidden; c += 512) {
    float a[8], p[8];
    if (in) unpack8(*reinterpret_cast<const uint4*>(wte + (id - vocab_start) * hidden + c), a);
    else {
#pragma unroll
      for (int j = 0; j < 8; ++j) a[j] = 0.f;
    }
    if (wpe) {
      unpack8(*reinterpret_cast<const uint4*>(wpe + (size_t)pos * hidden + c), p);
#pragma unroll
      for (int j = 0; j < 8; ++j) a[j] += p[j];
    }
    *reinterpret_cast<uint4*>(out + (size_t)t * hidden + c) = pack8(a);
  }
}

// Deterministic scatter-add: ids sorted (sorted_ids, perm = original positions).
// The first block of each run of equal ids sums the run's rows in fp32 and adds the
// result to dW[id] once -- no atomics, bitwise reproducible.
__global__ __launch_bounds__(128) void embed_bwd_kernel(
    const int64_t* __restrict__ sorted_ids, const int64_t* __restrict__ perm,
    const uint16_t* __restrict__ dout, uint16_t* __restrict__ dw, int ntok, int hidden,
    int64_t vocab_start, int64_t vocab_end) {
  const int i = blockIdx.x;
  const int64_t id = sorted_ids[i];
  if (i > 0 && sorted_ids[i - 1] == id) return;
  if (id < vocab_start || id >= vocab_end) return;
  int end = i + 1;
  while (end < ntok && sorted_ids[end] == id) ++end;
  for (int c = threadIdx.x * 8; c < hidden; c += 128 * 8) {
    float acc[8];
    unpack8(*reinterpret_cast<const uint4*>(dw + (id - vocab_start) * hidden + c), acc);
    for (int k = i; k < end; ++k) {
      float v[8];
      unpack8(*reinterpret_cast<const uint4*>(dout + perm[k] * hidden + c), v);
#pragma unroll
      for (int j = 0; j < 8; ++j) acc[j] += v[j];
    }
    *reinterpret_cast<uint4*>(dw + (id - vocab_start) * hidden + c) = pack8(acc);
  }
}

// Sort-free deterministic form (no torch.sort of the ids every step: the radix sort, its
// index copies and an arange cost ~60 us of the GPT-2 step against ~7 us for the scatter,
// profiles/r6/gpt2_step_census_small_kernels.txt).  A block stages every id in LDS; one wave
// per token scans them in 64-id chunks with a ballot: a token that has an EARLIER duplicate
// returns, the first occurrence sums its own row and every later duplicate's row in token
// order (fixed order: bit-reproducible) into fp32 registers, then adds them to dW once.
// Random tokens over a 50k vocabulary have ~1 duplicate pair per 25 tokens, so nearly every
// wave writes one row.  NV 16-B vectors per lane per 512 columns (hidden = 512 NV).
template <int NV>
__global__ __launch_bounds__(256) void embed_bwd_scan_kernel(
    const int64_t* __restrict__ ids, const uint16_t* __restrict__ dout, uint16_t* __restrict__ dw,
    int ntok, int hidden, int tok_per_block, int64_t vocab_start, int64_t vocab_end) {
  extern __shared__ int64_t sid[];   // [ntok]
  for (int t = threadIdx.x; t < ntok; t += blockDim.x) sid[t] = ids[t];
  __syncthreads();
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int t0 = blockIdx.x * tok_per_block;
  const int t1 = min(ntok, t0 + tok_per_block);
  for (int i = t0 + w; i < t1; i += 4) {
    const int64_t id = sid[i];
    if (id < vocab_start || id >= vocab_end) continue;
    // an earlier duplicate owns this id
    bool dup = false;
    for (int c = 0; c < i && !dup; c += 64) {
      const int k = c + lane;
      dup = __ballot(k < i && sid[k] == id) != 0ull;
    }
    if (dup) continue;
    float acc[NV][8];
#pragma unroll
    for (int v = 0; v < NV; ++v)
#pragma unroll
      for (int j = 0; j < 8; ++j) acc[v][j] = 0.f;
    for (int c = i & ~63; c < ntok; c += 64) {
      const int k = c + lane;
      uint64_t m = __ballot(k >= i && k < ntok && sid[k] == id);
      while (m) {   // this chunk's duplicates, ascending token order
        const int kk = c + __builtin_ctzll(m);
        m &= m - 1;
        const uint16_t* row = dout + (size_t)kk * hidden + lane * 8;
        uint4 x[NV];
#pragma unroll
        for (int v = 0; v < NV; ++v) x[v] = *reinterpret_cast<const uint4*>(row + 512 * v);
#pragma unroll
        for (int v = 0; v < NV; ++v) {
          float f[8];
          unpack8(x[v], f);
#pragma unroll
          for (int j = 0; j < 8; ++j) acc[v][j] += f[j];
        }
      }
    }
    uint16_t* drow = dw + (size_t)(id - vocab_start) * hidden + lane * 8;
#pragma unroll
    for (int v = 0; v < NV; ++v) {
      float d[8];
      unpack8(*reinterpret_cast<const uint4*>(drow + 512 * v), d);
#pragma unroll
      for (int j = 0; j < 8; ++j) d[j] += acc[v][j];
      *reinterpret_cast<uint4*>(drow + 512 * v) = pack8(d);
    }
  }
}

// dwpe[s] += sum_b dout[b*seq + s]
__global__ __launch_bounds__(256) void pos_bwd_kernel(const uint16_t* __restrict__ dout,
                                                      uint16_t* __restrict__ dwpe, int batch,
                                                      int seq, int hidden) {
  const int64_t v = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  const int64_t nvec = (int64_t)seq * hidden / 8;
  if (v >= nvec) return;
  float acc[8];
  unpack8(*reinterpret_cast<const uint4*>(dwpe + v * 8), acc);
  for (int b = 0; b < batch; ++b) {
    float x[8];
    unpack8(*reinterpret_cast<const uint4*>(dout + ((size_t)b * seq * hidden) + v * 8), x);
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[j] += x[j];
  }
  *reinterpret_cast<uint4*>(dwpe + v * 8) = pack8(acc);
}

// ---------------------------------------------------------------- cross entropy
// Pass 1: per row (max, sum exp(x - max), x[label] if label in this shard).
__global__ __launch_bounds__(256) void ce_stats_kernel(
    const uint16_t* __restrict__ logits, const int64_t* __restrict__ labels, int rows,
    int vocab, int64_t vocab_start, float* __restrict__ row_max, float* __restrict__ row_sum,
    float* __restrict__ row_tgt) {
  __shared__ float sm[8], ss[8];
  const int row = blockIdx.x;
  const uint16_t* x = logits + (size_t)row * vocab;
  float m = -INFINITY, s = 0.f;
  const int nvec = vocab / 8;
  for (int v = threadIdx.x; v < nvec; v += 256) {
    float a[8];
    unpack8(*reinterpret_cast<const uint4*>(x + v * 8), a);
    float lm = a[0];
#pragma unroll
    for (int j = 1; j < 8; ++j) lm = fmaxf(lm, a[j]);
    if (lm > m) { s *= __expf(m - lm); m = lm; }
#pragma unroll
    for (int j = 0; j < 8; ++j) s += __expf(a[j] - m);
  }
  for (int c = nvec * 8 + threadIdx.x; c < vocab; c += 256) {  // tail
    float a = bf2f(x[c]);
    if (a > m) { s *= __expf(m - a); m = a; }
    s += __expf(a - m);
  }
  // wave combine (m, s)
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    float om = __shfl_xor(m, o, 64), os = __shfl_xor(s, o, 64);
    float nm = fmaxf(m, om);
    s = (m == -INFINITY ? 0.f : s * __expf(m - nm)) + (om == -INFINITY ? 0.f : os * __expf(om - nm));
    m = nm;
  }
  const int w = threadIdx.x >> 6;
  if ((threadIdx.x & 63) == 0) { sm[w] = m; ss[w] = s; }
  __syncthreads();
  if (threadIdx.x == 0) {
    float M = sm[0], S = ss[0];
    for (int k = 1; k < 4; ++k) {
      float nm = fmaxf(M, sm[k]);
      S = (M == -INFINITY ? 0.f : S * __expf(M - nm)) +
          (sm[k] == -INFINITY ? 0.f : ss[k] * __expf(sm[k] - nm));
      M = nm;
    }
    row_max[row] = M;
    row_sum[row] = S;
    const int64_t lab = labels[row] - vocab_start;
    row_tgt[row] = (lab >= 0 && lab < vocab) ? bf2f(x[lab]) : 0.f;
  }
}

// Pass 2: dlogits = (exp(x - lse) - onehot) * scale * (label valid), written in place
// over the logits (bf16); loss[row] = lse - x[label].
__global__ __launch_bounds__(256) void ce_grad_kernel(
    uint16_t* __restrict__ logits, const int64_t* __restrict__ labels, int rows, int vocab,
    int64_t vocab_start, const float* __restrict__ lse, const float* __restrict__ tgt,
    float* __restrict__ loss, const float* __restrict__ scale_ptr, float scale,
    int ignore_index) {
  const int row = blockIdx.x;
  uint16_t* x = logits + (size_t)row * vocab;
  const int64_t glab = labels[row];
  const bool valid = glab != ignore_index;
  const float L = lse[row];
  const float sc = (scale_ptr ? *scale_ptr : scale) * (valid ? 1.f : 0.f);
  const int64_t lab = glab - vocab_start;
  const int nvec = vocab / 8;
  for (int v = threadIdx.x; v < nvec; v += 256) {
    float a[8];
    unpack8(*reinterpret_cast<const uint4*>(x + v * 8), a);
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      float p = __expf(a[j] - L);
      if (v * 8 + j == lab) p -= 1.f;
      a[j] = p * sc;
    }
    *reinterpret_cast<uint4*>(x + v * 8) = pack8(a);
  }
  for (int c = nvec * 8 + threadIdx.x; c < vocab; c += 256) {
    float p = __expf(bf2f(x[c]) - L);
    if (c == lab) p -= 1.f;
    x[c] = f2bf(p * sc);
  }
  if (threadIdx.x == 0 && loss) loss[row] = valid ? (L - tgt[row]) : 0.f;
}

// Single pass (no tensor-parallel vocab split): one 256-thread block per row holds the whole
// row in registers (NVT 16-B vectors per thread, all loads issued up front), reduces the
// max and the sum of exp(x - max) over the block, and writes
// dlogits = (exp(x - lse) - onehot) * scale in place -- the logits are read once instead
// of twice (ce_stats_kernel + ce_grad_kernel: 412 + 824 MB per GPT-2 345M step).
template <int NVT>
__global__ __launch_bounds__(256) void ce_fused_kernel(
    uint16_t* __restrict__ logits, const int64_t* __restrict__ labels, int vocab,
    float* __restrict__ loss, const float* __restrict__ scale_ptr, float scale, int ignore_index) {
  __shared__ float red[4];
  const int row = blockIdx.x, tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  uint16_t* x = logits + (size_t)row * vocab;
  const int nvec = vocab / 8;
  uint4 r[NVT];
#pragma unroll
  for (int i = 0; i < NVT; ++i) {
    const int v = min(tid + 256 * i, nvec - 1);   // clamped, unconditional (masked at use)
    r[i] = *reinterpret_cast<const uint4*>(x + v * 8);
  }
  float m = -INFINITY;
#pragma unroll
  for (int i = 0; i < NVT; ++i) {
    if (tid + 256 * i >= nvec) continue;
    float a[8];
    unpack8(r[i], a);
#pragma unroll
    for (int j = 0; j < 8; ++j) m = fmaxf(m, a[j]);
  }
  m = wave_max(m);
  if (lane == 0) red[w] = m;
  __syncthreads();
  m = fmaxf(fmaxf(red[0], red[1]), fmaxf(red[2], red[3]));
  __syncthreads();
  constexpr float L2E = 1.4426950408889634f;
  const float mc = m * L2E;
  float s = 0.f;
#pragma unroll
  for (int i = 0; i < NVT; ++i) {
    if (tid + 256 * i >= nvec) continue;
    float a[8];
    unpack8(r[i], a);
#pragma unroll
    for (int j = 0; j < 8; ++j) s += __builtin_amdgcn_exp2f(__builtin_fmaf(a[j], L2E, -mc));
  }
  s = wave_sum(s);
  if (lane == 0) red[w] = s;
  __syncthreads();
  s = (red[0] + red[1]) + (red[2] + red[3]);
  const float lse = m + __logf(s);
  const int64_t lab = labels[row];
  const bool valid = lab != ignore_index;
  const float sc = (scale_ptr ? *scale_ptr : scale) * (valid ? 1.f : 0.f);
  const float lc = lse * L2E;
#pragma unroll
  for (int i = 0; i < NVT; ++i) {
    const int v = tid + 256 * i;
    if (v >= nvec) continue;
    float a[8];
    unpack8(r[i], a);
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      float p = __builtin_amdgcn_exp2f(__builtin_fmaf(a[j], L2E, -lc));
      if (v * 8 + j == lab) p -= 1.f;
      a[j] = p * sc;
    }
    *reinterpret_cast<uint4*>(x + v * 8) = pack8(a);
  }
  // loss = lse - x[label]: the owner of the label's vector holds the original logit
  if (loss && valid && lab >= 0 && lab < vocab) {
    const int lv = (int)(lab >> 3);
    if ((lv & 255) == tid) {
      float a[8];
#pragma unroll
      for (int i = 0; i < NVT; ++i)
        if (tid + 256 * i == lv) unpack8(r[i], a);
      loss[row] = lse - a[lab & 7];
    }
  } else if (loss && tid == 0) {
    loss[row] = 0.f;
  }
}

__global__ void ce_lse_kernel(const float* __restrict__ m, const float* __restrict__ s,
                              float* __restrict__ lse, int rows) {
  int r = blockIdx.x * blockDim.x + threadIdx.x;
  if (r < rows) lse[r] = m[r] + __logf(s[r]);
}

}  // namespace

MX_EXPORT int mx_bias_gelu_fwd(const void* x, const void* bias, void* y, int rows, int cols,
                               hipStream_t s) {
  const int64_t n = (int64_t)rows * cols;
  if (cols <= 0 || cols % 8) return hipErrorInvalidValue;
  const int64_t blocks = (n / 8 + 256 * kGeluFV - 1) / (256 * kGeluFV);
  const int cmask = (cols & (cols - 1)) == 0 ? cols - 1 : -1;
  hipLaunchKernelGGL(bias_gelu_fwd_kernel, dim3((unsigned)blocks), dim3(256), 0, s,
                     (const uint16_t*)x, (const uint16_t*)bias, (uint16_t*)y, n, cols, cmask);
  return hipGetLastError();
}

MX_EXPORT int mx_bias_gelu_bwd_rows_per_block() { return 16; }

extern "C" int mx_colsum_finalize(const float* partial, int nparts, int cols, int nvec, void* o0,
                                  void* o1, void* o2, int accumulate, float* scratch,
                                  hipStream_t s);

// partial: ceil(rows/16)*cols floats + mx_colreduce_scratch(ceil(rows/16), cols) scratch
// floats behind it.  dx may alias dy.
MX_EXPORT int mx_bias_gelu_bwd(const void* dy, const void* x, const void* bias, void* dx,
                               void* dbias, int accumulate, float* partial, int rows, int cols,
                               hipStream_t s) {
  const int rpb = 16;
  dim3 grid((cols / 8 + 255) / 256, (rows + rpb - 1) / rpb);
  hipLaunchKernelGGL(bias_gelu_bwd_kernel, grid, dim3(256), 0, s, (const uint16_t*)dy,
                     (const uint16_t*)x, (const uint16_t*)bias, (uint16_t*)dx, rows, cols, rpb,
                     partial);
  if (dbias)
    return mx_colsum_finalize(partial, (int)grid.y, cols, 1, dbias, nullptr, nullptr,
                              accumulate, partial + (size_t)grid.y * cols, s);
  return hipGetLastError();
}

MX_EXPORT int mx_bias_swiglu_fwd(const void* pre, const void* bias, void* y, int rows, int f,
                                 hipStream_t s) {
  if (f % 8) return hipErrorInvalidValue;
  int64_t blocks = ((int64_t)rows * (f / 8) + 255) / 256;
  if (blocks > 8192) blocks = 8192;
  hipLaunchKernelGGL(bias_swiglu_fwd_kernel, dim3((unsigned)blocks), dim3(256), 0, s,
                     (const uint16_t*)pre, (const uint16_t*)bias, (uint16_t*)y, rows, f);
  return hipGetLastError();
}

// partial: ceil(rows/16)*2f floats + mx_colreduce_scratch(ceil(rows/16), 2f) behind it
MX_EXPORT int mx_bias_swiglu_bwd(const void* dy, const void* pre, const void* bias, void* dpre,
                                 void* dbias, int accumulate, float* partial, int rows, int f,
                                 hipStream_t s) {
  if (f % 8) return hipErrorInvalidValue;
  const int rpb = 16;
  dim3 grid((f / 8 + 255) / 256, (rows + rpb - 1) / rpb);
  hipLaunchKernelGGL(bias_swiglu_bwd_kernel, grid, dim3(256), 0, s, (const uint16_t*)dy,
                     (const uint16_t*)pre, (const uint16_t*)bias, (uint16_t*)dpre, rows, f, rpb,
                     partial);
  if (dbias)
    return mx_colsum_finalize(partial, (int)grid.y, 2 * f, 1, dbias, nullptr, nullptr,
                              accumulate, partial + (size_t)grid.y * 2 * f, s);
  return hipGetLastError();
}

MX_EXPORT int mx_embed_fwd(const int64_t* ids, const void* wte, const void* wpe, void* out,
                           int ntok, int hidden, int seq, int64_t vocab_start,
                           int64_t vocab_end, int pos_offset, hipStream_t s) {
  hipLaunchKernelGGL(embed_fwd_kernel, dim3((ntok + 3) / 4), dim3(256), 0, s, ids,
                     (const uint16_t*)wte, (const uint16_t*)wpe, (uint16_t*)out, ntok, hidden,
                     seq, vocab_start, vocab_end, pos_offset);
  return hipGetLastError();
}

MX_EXPORT int mx_embed_bwd(const int64_t* sorted_ids, const int64_t* perm, const void* dout,
                           void* dw, int ntok, int hidden, int64_t vocab_start,
                           int64_t vocab_end, hipStream_t s) {
  hipLaunchKernelGGL(embed_bwd_kernel, dim3(ntok), dim3(128), 0, s, sorted_ids, perm,
                     (const uint16_t*)dout, (uint16_t*)dw, ntok, hidden, vocab_start,
                     vocab_end);
  return hipGetLastError();
}

// Sort-free embedding backward (embed_bwd_scan_kernel): ids [ntok] int64 as given.  Returns
// hipErrorInvalidValue (nothing launched) when the shape is outside the kernel's range
// (hidden not 512, 1024, 2048 or 4096; ids beyond the LDS stage): the caller sorts instead.
MX_EXPORT int mx_embed_bwd_scan(const int64_t* ids, const void* dout, void* dw, int ntok, int hidden,
                                int64_t vocab_start, int64_t vocab_end, hipStream_t s) {
  if (ntok <= 0 || (size_t)ntok * 8 > 64 * 1024) return hipErrorInvalidValue;
  constexpr int TPB = 16;   // tokens per block: 4096 tokens -> 256 blocks
  const dim3 grid((ntok + TPB - 1) / TPB);
  const size_t lds = (size_t)ntok * 8;
#define MX_EB(NV) hipLaunchKernelGGL(embed_bwd_scan_kernel<NV>, grid, dim3(256), lds, s, ids, (const uint16_t*)dout, \
                                     (uint16_t*)dw, ntok, hidden, TPB, vocab_start, vocab_end)
  switch (hidden) {
    case 512: MX_EB(1); break;
    case 1024: MX_EB(2); break;
    case 2048: MX_EB(4); break;
    case 4096: MX_EB(8); break;
    default: return hipErrorInvalidValue;
  }
#undef MX_EB
  return hipGetLastError();
}

MX_EXPORT int mx_pos_embed_bwd(const void* dout, void* dwpe, int batch, int seq, int hidden,
                               hipStream_t s) {
  int64_t nvec = (int64_t)seq * hidden / 8;
  hipLaunchKernelGGL(pos_bwd_kernel, dim3((unsigned)((nvec + 255) / 256)), dim3(256), 0, s,
                     (const uint16_t*)dout, (uint16_t*)dwpe, batch, seq, hidden);
  return hipGetLastError();
}

MX_EXPORT int mx_ce_stats(const void* logits, const int64_t* labels, int rows, int vocab,
                          int64_t vocab_start, float* row_max, float* row_sum, float* row_tgt,
                          hipStream_t s) {
  hipLaunchKernelGGL(ce_stats_kernel, dim3(rows), dim3(256), 0, s, (const uint16_t*)logits,
                     labels, rows, vocab, vocab_start, row_max, row_sum, row_tgt);
  return hipGetLastError();
}

MX_EXPORT int mx_ce_lse(const float* m, const float* sum, float* lse, int rows,
                        hipStream_t s) {
  hipLaunchKernelGGL(ce_lse_kernel, dim3((rows + 255) / 256), dim3(256), 0, s, m, sum, lse,
                     rows);
  return hipGetLastError();
}

// single-pass CE (see ce_fused_kernel); vocab % 8 == 0 and vocab <= 64 * 256 * 8, else
// hipErrorInvalidValue (the caller then runs the two-pass path)
MX_EXPORT int mx_ce_fused(void* logits, const int64_t* labels, int rows, int vocab, float* loss,
                          const float* scale_ptr, float scale, int ignore_index, hipStream_t s) {
  if (vocab % 8 || rows <= 0) return hipErrorInvalidValue;
  const int nvt = (vocab / 8 + 255) / 256;
#define MX_CEF(N)                                                                                  \
  hipLaunchKernelGGL(ce_fused_kernel<N>, dim3(rows), dim3(256), 0, s, (uint16_t*)logits, labels, vocab, \
                     loss, scale_ptr, scale, ignore_index)
  if (nvt <= 8) MX_CEF(8);
  else if (nvt <= 16) MX_CEF(16);
  else if (nvt <= 25) MX_CEF(25);
  else if (nvt <= 32) MX_CEF(32);
  else if (nvt <= 48) MX_CEF(48);
  else if (nvt <= 64) MX_CEF(64);
  else return hipErrorInvalidValue;
#undef MX_CEF
  return hipGetLastError();
}

MX_EXPORT int mx_ce_grad(void* logits, const int64_t* labels, int rows, int vocab,
                         int64_t vocab_start, const float* lse, const float* tgt, float* loss,
                         const float* scale_ptr, float scale, int ignore_index,
                         hipStream_t s) {
  hipLaunchKernelGGL(ce_grad_kernel, dim3(rows), dim3(256), 0, s, (uint16_t*)logits, labels,
                     rows, vocab, vocab_start, lse, tgt, loss, scale_ptr, scale, ignore_index);
  return hipGetLastError();
}
