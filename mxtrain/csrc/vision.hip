// Detection kernels for the Mask R-CNN workload: multi-level
// RoIAlign forward/backward on NHWC bf16 FPN features, bitmask NMS, fused anchor/proposal
// <-> ground-truth matching, fused box decode + clip.  gfx950 / wave64.
//
// Layout choices (MI355X-first):
//  * features are NHWC (channels_last) bf16, so one RoIAlign sample point reads C
//    contiguous channels: a 64-lane wave covers 2 x 256 channels with 16-byte loads;
//  * RoIAlign output is [R, PH, PW, C] -- directly the NHWC input of the mask head convs
//    and, flattened, the box-head FC input;
//  * backward scatters with hardware fp32 global atomics (global_atomic_add_f32) into an
//    fp32 NHWC gradient per level, converted to bf16 by the caller's cast.
//  * NMS: one 64x64 IoU tile per workgroup-wave produces 64-bit suppression words
//    (wave64 = one word per lane); the sequential keep pass runs in one wave per problem
//    with the removed-bitmask distributed one word per lane.
#include "common.h"
#include "gemm_common.h"

namespace {

using namespace mx;

struct Levels {
  const uint16_t* f[4];
  float* g[4];
  int H[4];
  int W[4];
  float scale[4];
  int n;        // number of levels
  int lvl_min;  // FPN level of f[0] (2 for P2)
  float canon;  // canonical box size (224) for level assignment
  int canon_lvl;
};

__device__ __forceinline__ int roi_level(const Levels& L, float x1, float y1, float x2, float y2) {
  if (L.n == 1) return 0;
  const float area = fmaxf(x2 - x1, 0.f) * fmaxf(y2 - y1, 0.f);
  const float k = floorf((float)L.canon_lvl + log2f(sqrtf(area) / L.canon + 1e-8f));
  int lvl = (int)k - L.lvl_min;
  lvl = lvl < 0 ? 0 : (lvl >= L.n ? L.n - 1 : lvl);
  return lvl;
}

struct Bilinear {
  int o[4];
  float w[4];
  bool valid;
};

__device__ __forceinline__ Bilinear bilinear(float y, float x, int H, int W) {
  Bilinear b;
  b.valid = !(y < -1.f || y > (float)H || x < -1.f || x > (float)W);
  if (!b.valid) {
    b.o[0] = b.o[1] = b.o[2] = b.o[3] = 0;
    b.w[0] = b.w[1] = b.w[2] = b.w[3] = 0.f;
    return b;
  }
  y = fmaxf(y, 0.f);
  x = fmaxf(x, 0.f);
  int yl = (int)y, xl = (int)x, yh, xh;
  if (yl >= H - 1) { yh = yl = H - 1; y = (float)yl; } else { yh = yl + 1; }
  if (xl >= W - 1) { xh = xl = W - 1; x = (float)xl; } else { xh = xl + 1; }
  const float ly = y - yl, lx = x - xl, hy = 1.f - ly, hx = 1.f - lx;
  b.o[0] = yl * W + xl; b.o[1] = yl * W + xh; b.o[2] = yh * W + xl; b.o[3] = yh * W + xh;
  b.w[0] = hy * hx; b.w[1] = hy * lx; b.w[2] = ly * hx; b.w[3] = ly * lx;
  return b;
}

// one axis of bilinear(): the same validity, clamping and lo/hi weights
struct Axis {
  int lo, hi;
  float wlo, whi;
  bool valid;
};

__device__ __forceinline__ Axis axis_weights(float y, int H) {
  Axis a;
  a.valid = !(y < -1.f || y > (float)H);
  y = fmaxf(y, 0.f);
  int l = (int)y;
  if (l >= H - 1) { a.lo = a.hi = H - 1; y = (float)a.lo; } else { a.lo = l; a.hi = l + 1; }
  const float f = y - a.lo;
  a.wlo = 1.f - f;
  a.whi = f;
  return a;
}

// one thread = (roi, bin, 8-channel chunk)
__global__ __launch_bounds__(256) void roi_align_fwd_kernel(Levels L, const float* __restrict__ rois, int R,
                                                            int C, int PH, int PW, int sr, int aligned,
                                                            uint16_t* __restrict__ out) {
  const int cch = C >> 3;
  const long idx = (long)blockIdx.x * blockDim.x + threadIdx.x;
  const long total = (long)R * PH * PW * cch;
  if (idx >= total) return;
  const int ch = (int)(idx % cch);
  const int bin = (int)((idx / cch) % (PH * PW));
  const int r = (int)(idx / ((long)cch * PH * PW));
  const float* rr = rois + (size_t)r * 5;
  const int b = (int)rr[0];
  const int lv = roi_level(L, rr[1], rr[2], rr[3], rr[4]);
  const float s = L.scale[lv];
  const float off = aligned ? 0.5f : 0.f;
  const float x0 = rr[1] * s - off, y0 = rr[2] * s - off;
  float rw = rr[3] * s - off - x0, rh = rr[4] * s - off - y0;
  if (!aligned) { rw = fmaxf(rw, 1.f); rh = fmaxf(rh, 1.f); }
  const float bw = rw / PW, bh = rh / PH;
  const int ph = bin / PW, pw = bin % PW;
  const int H = L.H[lv], W = L.W[lv];
  const uint16_t* base = L.f[lv] + ((size_t)b * H * W) * C + ch * 8;
  float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  for (int iy = 0; iy < sr; ++iy) {
    const float y = y0 + ph * bh + (iy + 0.5f) * bh / sr;
    for (int ix = 0; ix < sr; ++ix) {
      const float x = x0 + pw * bw + (ix + 0.5f) * bw / sr;
      const Bilinear bl = bilinear(y, x, H, W);
      if (!bl.valid) continue;
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        float v[8];
        unpack8(*reinterpret_cast<const uint4*>(base + (size_t)bl.o[k] * C), v);
#pragma unroll
        for (int j = 0; j < 8; ++j) acc[j] += bl.w[k] * v[j];
      }
    }
  }
  const float inv = 1.f / (float)(sr * sr);
#pragma unroll
  for (int j = 0; j < 8; ++j) acc[j] *= inv;
  *reinterpret_cast<uint4*>(out + ((size_t)r * PH * PW + bin) * C + ch * 8) = pack8(acc);
}

// one wave = one (roi, bin); lane l owns channels l, l+64, ...  Every fp32 atomic
// instruction then covers 64 consecutive floats (two 128-B L2 lines) instead of 64
// scattered 32-B slots -- the L2 atomic units process per line, so contention on the
// small coarse FPN levels drops ~16x versus a chunk-per-lane layout.
__global__ __launch_bounds__(256) void roi_align_bwd_kernel(Levels L, const float* __restrict__ rois, int R,
                                                            int C, int PH, int PW, int sr, int aligned,
                                                            const uint16_t* __restrict__ dout) {
  const int lane = threadIdx.x & 63;
  const long wid = (long)blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
  if (wid >= (long)R * PH * PW) return;
  const int bin = (int)(wid % (PH * PW));
  const int r = (int)(wid / (PH * PW));
  const float* rr = rois + (size_t)r * 5;
  const int b = (int)rr[0];
  const int lv = roi_level(L, rr[1], rr[2], rr[3], rr[4]);
  const float s = L.scale[lv];
  const float off = aligned ? 0.5f : 0.f;
  const float x0 = rr[1] * s - off, y0 = rr[2] * s - off;
  float rw = rr[3] * s - off - x0, rh = rr[4] * s - off - y0;
  if (!aligned) { rw = fmaxf(rw, 1.f); rh = fmaxf(rh, 1.f); }
  const float bw = rw / PW, bh = rh / PH;
  const int ph = bin / PW, pw = bin % PW;
  const int H = L.H[lv], W = L.W[lv];
  float* gbase = L.g[lv] + ((size_t)b * H * W) * C + lane;
  const uint16_t* d = dout + ((size_t)r * PH * PW + bin) * C + lane;
  const int ng = C >> 6;   // channel groups of 64 (C % 64 == 0 checked by the launcher)
  float go[8];
#pragma unroll
  for (int g = 0; g < 8; ++g) go[g] = g < ng ? bf2f(d[g * 64]) : 0.f;
  const float inv = 1.f / (float)(sr * sr);
  if (sr <= 2) {
    // The bilinear weights are separable: a sample at (y, x) puts wy(row) * wx(col) on
    // its 4 corners, and validity is valid(y) && valid(x), so the bin's total weight on
    // pixel (row, col) is Wy[row] * Wx[col] with Wy / Wx summed over the sr samples of
    // each axis.  Rows (columns) shared by the two samples merge into one entry: a bin
    // of ~1-2 feature pixels touches 2-3 rows x 2-3 columns, 4-9 atomics per channel
    // instead of 16.  Entries: (lo, hi) of sample 0, then of sample 1, per axis; weight
    // 0 = unused; every index is a compile-time constant after unrolling (no scratch).
    int ry[4], rx[4];
    float wy[4], wx[4];
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const bool use = i < sr;
      const Axis a = axis_weights(y0 + ph * bh + (i + 0.5f) * bh / sr, H);
      const Axis c = axis_weights(x0 + pw * bw + (i + 0.5f) * bw / sr, W);
      ry[2 * i] = a.lo; ry[2 * i + 1] = a.hi;
      wy[2 * i] = use && a.valid ? a.wlo : 0.f; wy[2 * i + 1] = use && a.valid ? a.whi : 0.f;
      rx[2 * i] = c.lo; rx[2 * i + 1] = c.hi;
      wx[2 * i] = use && c.valid ? c.wlo : 0.f; wx[2 * i + 1] = use && c.valid ? c.whi : 0.f;
    }
    // fold duplicate rows / columns into their first occurrence
#pragma unroll
    for (int j = 1; j < 4; ++j) {
      bool fy = false, fx = false;
#pragma unroll
      for (int i = 0; i < j; ++i) {
        if (!fy && ry[i] == ry[j]) { wy[i] += wy[j]; fy = true; }
        if (!fx && rx[i] == rx[j]) { wx[i] += wx[j]; fx = true; }
      }
      if (fy) wy[j] = 0.f;
      if (fx) wx[j] = 0.f;
    }
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      if (wy[i] == 0.f) continue;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const float wk = wy[i] * wx[j] * inv;
        if (wk == 0.f) continue;
        float* gp = gbase + (size_t)(ry[i] * W + rx[j]) * C;
#pragma unroll
        for (int g = 0; g < 8; ++g)
          if (g < ng) unsafeAtomicAdd(gp + g * 64, wk * go[g]);
      }
    }
    return;
  }
  for (int iy = 0; iy < sr; ++iy) {
    const float y = y0 + ph * bh + (iy + 0.5f) * bh / sr;
    for (int ix = 0; ix < sr; ++ix) {
      const float x = x0 + pw * bw + (ix + 0.5f) * bw / sr;
      const Bilinear bl = bilinear(y, x, H, W);
      if (!bl.valid) continue;
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const float wk = bl.w[k] * inv;
        if (wk == 0.f) continue;
        float* gp = gbase + (size_t)bl.o[k] * C;
#pragma unroll
        for (int g = 0; g < 8; ++g)
          if (g < ng) unsafeAtomicAdd(gp + g * 64, wk * go[g]);
      }
    }
  }
}

// ------------------------------------------------------------ RoIAlign backward, tiled
// Float-atomics-free RoIAlign backward.  The gradient of every level is cut
// into 8 x 8-pixel tiles; each (roi, bin) "item" touches at most 2 x 2 tiles (its sr x sr
// samples' bilinear corners span <= bin + 2 pixels per axis and a bin is <= 6 feature
// pixels at every FPN level for <= 1344-pixel images).  Pipeline:
//   1. items: the item's separable footprint (<= 4 rows x 4 columns, weights with
//      1/sr^2 folded in) is computed ONCE and stored packed (48 B); tile counters ++
//      (integer atomics: bucket sizes only);
//   2. one-workgroup scan: entry offsets, cursors, and work chunks of <= kChunk entries
//      per tile (a heavy tile on a coarse level is split so no workgroup runs a long
//      serial chain), plus partial-slot offsets for split tiles;
//   3. scatter item ids into their tiles' lists;
//   4. one workgroup per chunk: its entry ids are bitonic-sorted in LDS (deterministic
//      order), their footprints staged in LDS, and wave w / lane l accumulate channel
//      64 w + l of the tile's 64 pixels in an fp32 LDS tile -- each LDS word has exactly
//      one writer, so no atomics; the gradient rows are prefetched a batch ahead;
//      single-chunk tiles (all but the heaviest) write bf16 NHWC directly, split tiles
//      write an fp32 partial;
//   5. split tiles: partials summed in chunk order -> bf16.
// Every pixel of every level is written exactly once (empty tiles write zeros): no fp32
// gradient buffer, zero-fill or cast.  Deterministic (entry lists sorted by item id) for
// tiles of <= kSortBig entries.
constexpr int kTile = 8;
constexpr int kChunk = 256;       // entries per work chunk (and sort capacity)
constexpr int kMaxTileC = 256;    // 64 px x 256 ch fp32 = 64 KB (+ 13 KB) of the 160 KB LDS
constexpr int kBatch = 16;        // gradient rows in flight per lane

struct GOut {
  uint16_t* p[4];   // bf16 NHWC gradient per level
};

struct TileGeo {
  int base[5];   // first tile id of each level (base[n] = total tiles)
  int th[4];     // tiles per column / row of a level image
  int tw[4];
  int B;
};

struct Foot {
  int ry[4], rx[4];
  float wy[4], wx[4];   // per-axis weights, 0 = unused; duplicate rows/columns merged
  int lv, b;
};

struct __attribute__((aligned(16))) FootP {   // packed footprint (48 B)
  int16_t ry[4], rx[4];
  float wy[4], wx[4];   // wy carries 1 / sr^2
};

// the sr <= 2 separable footprint of item (roi, bin) (same arithmetic as roi_align_bwd_kernel)
__device__ __forceinline__ Foot footprint(const Levels& L, const float* __restrict__ rois, int item, int PH,
                                          int PW, int sr, int aligned) {
  Foot f;
  const int bin = item % (PH * PW);
  const int r = item / (PH * PW);
  const float* rr = rois + (size_t)r * 5;
  f.b = (int)rr[0];
  f.lv = roi_level(L, rr[1], rr[2], rr[3], rr[4]);
  const float s = L.scale[f.lv];
  const float off = aligned ? 0.5f : 0.f;
  const float x0 = rr[1] * s - off, y0 = rr[2] * s - off;
  float rw = rr[3] * s - off - x0, rh = rr[4] * s - off - y0;
  if (!aligned) { rw = fmaxf(rw, 1.f); rh = fmaxf(rh, 1.f); }
  const float bw = rw / PW, bh = rh / PH;
  const int ph = bin / PW, pw = bin % PW;
  const int H = L.H[f.lv], W = L.W[f.lv];
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const bool use = i < sr;
    const Axis a = axis_weights(y0 + ph * bh + (i + 0.5f) * bh / sr, H);
    const Axis c = axis_weights(x0 + pw * bw + (i + 0.5f) * bw / sr, W);
    f.ry[2 * i] = a.lo; f.ry[2 * i + 1] = a.hi;
    f.wy[2 * i] = use && a.valid ? a.wlo : 0.f; f.wy[2 * i + 1] = use && a.valid ? a.whi : 0.f;
    f.rx[2 * i] = c.lo; f.rx[2 * i + 1] = c.hi;
    f.wx[2 * i] = use && c.valid ? c.wlo : 0.f; f.wx[2 * i + 1] = use && c.valid ? c.whi : 0.f;
  }
#pragma unroll
  for (int j = 1; j < 4; ++j) {
    bool fy = false, fx = false;
#pragma unroll
    for (int i = 0; i < j; ++i) {
      if (!fy && f.ry[i] == f.ry[j]) { f.wy[i] += f.wy[j]; fy = true; }
      if (!fx && f.rx[i] == f.rx[j]) { f.wx[i] += f.wx[j]; fx = true; }
    }
    if (fy) f.wy[j] = 0.f;
    if (fx) f.wx[j] = 0.f;
  }
  return f;
}

// distinct tile coordinates of the used rows (or columns); returns how many
__device__ __forceinline__ int distinct_tiles(const int* idx, const float* w, int* out) {
  int n = 0;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    if (w[i] == 0.f) continue;
    const int t = idx[i] / kTile;
    bool seen = false;
    for (int k = 0; k < n; ++k) seen |= out[k] == t;
    if (!seen) out[n++] = t;
  }
  return n;
}

// kCount: footprint -> fp[item], counts[tile]++; else entries[cursor[tile]++] = item
template <bool kCount>
__global__ __launch_bounds__(256) void roi_tiles_kernel(Levels L, TileGeo G, const float* __restrict__ rois,
                                                        int items, int PH, int PW, int sr, int aligned,
                                                        FootP* __restrict__ fp, int* __restrict__ counter,
                                                        int* __restrict__ entries) {
  const int item = blockIdx.x * blockDim.x + threadIdx.x;
  if (item >= items) return;
  const Foot f = footprint(L, rois, item, PH, PW, sr, aligned);
  if (f.b < 0 || f.b >= G.B) return;   // malformed batch index: never index outside the tiles
  if (kCount) {
    FootP q;
    const float inv = 1.f / (float)(sr * sr);
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      q.ry[i] = (int16_t)f.ry[i]; q.rx[i] = (int16_t)f.rx[i];
      q.wy[i] = f.wy[i] * inv; q.wx[i] = f.wx[i];
    }
    fp[item] = q;
  }
  int ty[4], tx[4];
  const int ny = distinct_tiles(f.ry, f.wy, ty), nx = distinct_tiles(f.rx, f.wx, tx);
  for (int i = 0; i < ny; ++i)
    for (int j = 0; j < nx; ++j) {
      const int t = G.base[f.lv] + (f.b * G.th[f.lv] + ty[i]) * G.tw[f.lv] + tx[j];
      if (kCount) {
        atomicAdd(counter + t, 1);
      } else {
        entries[atomicAdd(counter + t, 1)] = item;
      }
    }
}

// one-workgroup exclusive scans over the T tiles:
//   offsets[t] = sum counts[< t] (+ offsets[T]), cursor = offsets,
//   coff[t] = sum of chunks(< t), chunks(t) = max(1, ceil(counts / kChunk)) (+ coff[T]),
//   poff[t] = sum of chunks(< t) over split tiles (chunks > 1)
__device__ void block_scan(int* part, int t, int v, int& excl, int& total) {
  part[t] = v;
  __syncthreads();
  for (int d = 1; d < 1024; d <<= 1) {   // Hillis-Steele inclusive scan
    const int x = t >= d ? part[t - d] : 0;
    __syncthreads();
    part[t] += x;
    __syncthreads();
  }
  excl = part[t] - v;
  total = part[1023];
  __syncthreads();
}

__device__ __forceinline__ int chunks_of(int n) { return n <= kChunk ? 1 : (n + kChunk - 1) / kChunk; }

__global__ __launch_bounds__(1024) void tile_scan_kernel(const int* __restrict__ counts, int T,
                                                         int* __restrict__ offsets, int* __restrict__ cursor,
                                                         int* __restrict__ coff, int* __restrict__ poff,
                                                         int* __restrict__ ctile, int grid,
                                                         int* __restrict__ overflow) {
  __shared__ int part[1024];
  const int t = threadIdx.x;
  const int per = (T + 1023) / 1024;
  const int lo = min(t * per, T), hi = min(lo + per, T);
  int se = 0, sc = 0, sp = 0;
  for (int i = lo; i < hi; ++i) {
    const int n = counts[i], c = chunks_of(n);
    se += n;
    sc += c;
    sp += c > 1 ? c : 0;
  }
  int e0, c0, p0, et, ct, pt;
  block_scan(part, t, se, e0, et);
  block_scan(part, t, sc, c0, ct);
  block_scan(part, t, sp, p0, pt);
  for (int i = lo; i < hi; ++i) {
    const int n = counts[i], c = chunks_of(n);
    offsets[i] = e0; cursor[i] = e0; coff[i] = c0; poff[i] = p0;
    for (int q = 0; q < c; ++q)          // chunk -> tile map (one load per workgroup later)
      if (c0 + q < grid) ctile[c0 + q] = i;
    e0 += n; c0 += c; p0 += c > 1 ? c : 0;
  }
  if (t == 1023) {
    offsets[T] = et; coff[T] = ct; poff[T] = pt;
    if (ct > grid) *overflow = 1;   // more chunks than launched workgroups
  }
}

__device__ __forceinline__ void decode_tile(const Levels& L, const TileGeo& G, int tile, int& lv, int& b, int& ty,
                                            int& tx) {
  lv = 0;
  while (lv + 1 < L.n && tile >= G.base[lv + 1]) ++lv;
  const int local = tile - G.base[lv];
  tx = local % G.tw[lv];
  ty = (local / G.tw[lv]) % G.th[lv];
  b = local / (G.tw[lv] * G.th[lv]);
}

__device__ __forceinline__ void write_tile_bf16(const float* acc, uint16_t* g, int C, int H, int W, int b, int y0,
                                                int x0, int tid, int nt) {
  const int c8 = C / 8;
  for (int q = tid; q < kTile * kTile * c8; q += nt) {
    const int p = q / c8, ch = (q % c8) * 8;
    const int y = y0 + p / kTile, x = x0 + p % kTile;
    if (y >= H || x >= W) continue;
    *reinterpret_cast<uint4*>(g + (((size_t)b * H + y) * W + x) * C + ch) = pack8(acc + p * C + ch);
  }
}

// split tiles (kChunk < n <= kSortBig): sort the whole entry list once, so the chunks'
// membership and order -- and so the result -- are deterministic
constexpr int kSortBig = 16384;   // 64 KB of keys in LDS
__global__ __launch_bounds__(1024) void tile_sort_kernel(const int* __restrict__ offsets, int T,
                                                         int* __restrict__ entries) {
  __shared__ int keys[kSortBig];
  const int tile = blockIdx.x;
  const int beg = offsets[tile], n = offsets[tile + 1] - beg;
  if (n <= kChunk || n > kSortBig) return;
  const int tid = threadIdx.x, nt = blockDim.x;
  int np = 1;
  while (np < n) np <<= 1;
  for (int i = tid; i < np; i += nt) keys[i] = i < n ? entries[beg + i] : 0x7fffffff;
  __syncthreads();
  for (int kk = 2; kk <= np; kk <<= 1)
    for (int jj = kk >> 1; jj > 0; jj >>= 1) {
      for (int i = tid; i < np; i += nt) {
        const int p = i ^ jj;
        if (p > i) {
          const int a = keys[i], c = keys[p];
          if ((a > c) == ((i & kk) == 0)) { keys[i] = c; keys[p] = a; }
        }
      }
      __syncthreads();
    }
  for (int i = tid; i < n; i += nt) entries[beg + i] = keys[i];
}

// one workgroup (C threads = C / 64 waves) per work chunk
__global__ __launch_bounds__(256) void roi_align_bwd_tile_kernel(Levels L, TileGeo G, int T, int C,
                                                                 const uint16_t* __restrict__ dout,
                                                                 const FootP* __restrict__ fp,
                                                                 const int* __restrict__ offsets,
                                                                 const int* __restrict__ coff,
                                                                 const int* __restrict__ poff,
                                                                 const int* __restrict__ ctile,
                                                                 const int* __restrict__ entries, GOut gout,
                                                                 float* __restrict__ partial, int pslots,
                                                                 int* __restrict__ overflow,
                                                                 long long* __restrict__ dbg, int dmode) {
  const long long t_start = dbg ? (long long)__builtin_amdgcn_s_memrealtime() : 0;
  __shared__ __attribute__((aligned(16))) float acc[(kTile * kTile + 1) * kMaxTileC];   // [64 px + trash][C]
  __shared__ int keys[kChunk];
  __shared__ FootP fs[kChunk];
  const int tid = threadIdx.x, nt = blockDim.x;
  const int k = blockIdx.x;
  if (k >= coff[T]) return;                      // grid is an upper bound on the chunks
  const int tile = ctile[k];
  const int j = k - coff[tile], nch = coff[tile + 1] - coff[tile];
  int lv, b, ty, tx;
  decode_tile(L, G, tile, lv, b, ty, tx);
  const int H = L.H[lv], W = L.W[lv];
  const int y0 = ty * kTile, x0 = tx * kTile;
  const int ebeg = offsets[tile] + j * kChunk;
  const int n = min(kChunk, offsets[tile + 1] - ebeg);
  if (n == 0) {   // empty tile (most of the fine levels): zeros straight to global
    uint16_t* g = gout.p[lv];
    const int c8 = C / 8;
    for (int q = tid; q < kTile * kTile * c8; q += nt) {
      const int p = q / c8, ch = (q % c8) * 8;
      const int y = y0 + p / kTile, x = x0 + p % kTile;
      if (y < H && x < W) *reinterpret_cast<uint4*>(g + (((size_t)b * H + y) * W + x) * C + ch) = make_uint4(0, 0, 0, 0);
    }
    return;
  }
  for (int i = tid * 4; i < kTile * kTile * C; i += nt * 4)
    *reinterpret_cast<float4*>(acc + i) = make_float4(0.f, 0.f, 0.f, 0.f);
  int np = 1;
  while (np < n) np <<= 1;
  for (int i = tid; i < np; i += nt) keys[i] = i < n ? entries[ebeg + i] : 0x7fffffff;
  __syncthreads();
  if (nch == 1)   // (split tiles were sorted whole by tile_sort_kernel)
  for (int kk = 2; kk <= np; kk <<= 1)           // bitonic sort: deterministic order
    for (int jj = kk >> 1; jj > 0; jj >>= 1) {
      for (int i = tid; i < np; i += nt) {
        const int p = i ^ jj;
        if (p > i) {
          const int a = keys[i], c = keys[p];
          if ((a > c) == ((i & kk) == 0)) { keys[i] = c; keys[p] = a; }
        }
      }
      __syncthreads();
    }
  for (int i = tid; i < n; i += nt) fs[i] = fp[keys[i]];
  __syncthreads();
  const int c = tid;   // this thread's channel (blockDim == C)
  // One entry, branch-free: its footprint is read as 3 x 16 B, and its 4 x 4 (row, column)
  // slots map to distinct tile pixels -- or, when the slot is unused (zero weight: merged
  // duplicate row / column) or outside this tile, to a scratch row past the tile -- so all
  // 16 LDS reads are issued back to back before the 16 writes: two LDS round trips per
  // entry instead of a wait per pixel (and no exec-mask branching).
  // (the entry index is made opaque to the uniformity analysis -- mbcnt of an empty mask is
  // 0 -- so the footprint stays in VGPRs and the 16 slot addresses are v_cndmask selects:
  // scalarised, the same code became ~30 uniform branches per entry)
  const int lane0 = (int)__builtin_amdgcn_mbcnt_lo(0u, 0u);
  auto apply = [&](int e, float go) {
    const uint4* fv = reinterpret_cast<const uint4*>(fs + e + lane0);
    const uint4 a0 = fv[0], a1 = fv[1], a2 = fv[2];
    const int ry[4] = {(int)(int16_t)(a0.x & 0xffffu), (int)(int16_t)(a0.x >> 16), (int)(int16_t)(a0.y & 0xffffu),
                       (int)(int16_t)(a0.y >> 16)};
    const int rx[4] = {(int)(int16_t)(a0.z & 0xffffu), (int)(int16_t)(a0.z >> 16), (int)(int16_t)(a0.w & 0xffffu),
                       (int)(int16_t)(a0.w >> 16)};
    const float wy[4] = {__uint_as_float(a1.x), __uint_as_float(a1.y), __uint_as_float(a1.z), __uint_as_float(a1.w)};
    const float wx[4] = {__uint_as_float(a2.x), __uint_as_float(a2.y), __uint_as_float(a2.z), __uint_as_float(a2.w)};
    float* ad[16];
    float wv[16];
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int jx = 0; jx < 4; ++jx) {
        const int yy = ry[i] - y0, xx = rx[jx] - x0;
        // bitwise, not short-circuit: one v_cndmask per slot, no control flow
        const int in = (int)(wy[i] != 0.f) & (int)(wx[jx] != 0.f) & (int)((unsigned)yy < (unsigned)kTile) &
                       (int)((unsigned)xx < (unsigned)kTile);
        const int off = in ? (yy * kTile + xx) * C : kTile * kTile * C;
        ad[i * 4 + jx] = acc + off + c;
        wv[i * 4 + jx] = wy[i] * wx[jx] * go;
      }
    if (dmode & 2) return;   // (debug: no LDS accumulation)
    float v[16];
#pragma unroll
    for (int q = 0; q < 16; ++q) v[q] = *ad[q];
#pragma unroll
    for (int q = 0; q < 16; ++q) *ad[q] = v[q] + wv[q];
  };
  auto load = [&](int ee) {
    if (dmode & 1) return 1.f;   // (debug: no gradient loads)
    return ee < n ? bf2f(dout[(size_t)keys[ee] * C + c]) : 0.f;
  };
  // gradient rows double-buffered a batch ahead: batch A's loads are in flight while
  // batch B is applied and vice versa (no register copy between them, so no wait)
  float ga[kBatch], gb[kBatch];
#pragma unroll
  for (int q = 0; q < kBatch; ++q) ga[q] = load(q);
  for (int e = 0; e < n; e += 2 * kBatch) {
#pragma unroll
    for (int q = 0; q < kBatch; ++q) gb[q] = load(e + kBatch + q);
#pragma unroll
    for (int q = 0; q < kBatch; ++q)
      if (e + q < n) apply(e + q, ga[q]);
    if (e + kBatch >= n) break;
#pragma unroll
    for (int q = 0; q < kBatch; ++q) ga[q] = load(e + 2 * kBatch + q);
#pragma unroll
    for (int q = 0; q < kBatch; ++q)
      if (e + kBatch + q < n) apply(e + kBatch + q, gb[q]);
  }
  __syncthreads();
  if (dbg && tid == 0) {   // per-workgroup timing probe (100 MHz ticks): chunk, tile, entries, time
    dbg[4 * k] = k; dbg[4 * k + 1] = tile; dbg[4 * k + 2] = n;
    dbg[4 * k + 3] = (long long)__builtin_amdgcn_s_memrealtime() - t_start;
  }
  if (nch == 1) {
    write_tile_bf16(acc, gout.p[lv], C, H, W, b, y0, x0, tid, nt);
    return;
  }
  const int slot = poff[tile] + j;
  if (slot >= pslots) {   // beyond the geometric bound the host sized for: flag it
    if (tid == 0) atomicAdd(overflow, 1);
    return;
  }
  float* dst = partial + (size_t)slot * kTile * kTile * C;
  for (int i = tid * 4; i < kTile * kTile * C; i += nt * 4)
    *reinterpret_cast<float4*>(dst + i) = *reinterpret_cast<const float4*>(acc + i);
}

// C = 256: the same chunk as roi_align_bwd_tile_kernel, accumulated on the matrix cores.
// A chunk's contribution to its tile is a GEMM, out[px][c] = sum_e W[e][px] dY[e][c], with W
// the entries' bilinear footprints (<= 16 nonzeros of 64 per entry) and dY their gradient
// rows; per 32-entry K-step the rows are staged in LDS ([e][256 c], 16-B chunks swizzled by
// gemm_common.h's pchunk: the transposed reads of the A fragments are conflict-free) and W
// is scattered into an [px][e] image as bf16 hi + lo halves (w = hi + lo to ~2^-16, so the
// weights keep fp32-level precision; dY is bf16 already), two 16x16x32 MFMAs per product.
// The per-entry LDS read-modify-write loop of the scalar kernel (16 round trips per entry
// and channel) measured ~1.2 us per entry on the concentrated RoIs of a random-init RPN
// (scripts/roi_bwd_bench.py); here an entry costs 1/32 of a K-step.  Accumulation order is
// fixed (sorted entries, K-steps in order): deterministic like the scalar kernel.
constexpr int kMKS = 32;   // entries per K-step (the 16x16x32 MFMA depth)
__global__ __launch_bounds__(256, 2) void roi_align_bwd_mfma_kernel(Levels L, TileGeo G, int T,
                                                                    const uint16_t* __restrict__ dout,
                                                                    const FootP* __restrict__ fp,
                                                                    const int* __restrict__ offsets,
                                                                    const int* __restrict__ coff,
                                                                    const int* __restrict__ poff,
                                                                    const int* __restrict__ ctile,
                                                                    const int* __restrict__ entries, GOut gout,
                                                                    float* __restrict__ partial, int pslots,
                                                                    int* __restrict__ overflow,
                                                                    long long* __restrict__ dbg) {
  constexpr int C = 256, RB = C * 2;               // dY image row bytes
  constexpr int DIMG = kMKS * RB;                  // 16 KB
  constexpr int WIMG = kTile * kTile * kMKS * 2;   // [64 px][32 e] bf16 = 4 KB (hi, then lo)
  // the fp32 output tile aliases the K-step images (used only after the last K-step)
  __shared__ __attribute__((aligned(16))) char stage[kTile * kTile * C * 4];
  __shared__ int keys[kChunk];
  __shared__ FootP fs[kChunk];
  const long long t_start = dbg ? (long long)__builtin_amdgcn_s_memrealtime() : 0;
  char* const dimg = stage;
  char* const whi = stage + DIMG;
  char* const wlo = whi + WIMG;
  float* const acc_t = reinterpret_cast<float*>(stage);
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int k = blockIdx.x;
  if (k >= coff[T]) return;
  const int tile = ctile[k];
  const int j = k - coff[tile], nch = coff[tile + 1] - coff[tile];
  int lv, b, ty, tx;
  decode_tile(L, G, tile, lv, b, ty, tx);
  const int H = L.H[lv], W = L.W[lv];
  const int y0 = ty * kTile, x0 = tx * kTile;
  const int ebeg = offsets[tile] + j * kChunk;
  const int n = min(kChunk, offsets[tile + 1] - ebeg);
  if (n == 0) {
    uint16_t* g = gout.p[lv];
    for (int q = tid; q < kTile * kTile * (C / 8); q += 256) {
      const int p = q / (C / 8), ch = (q % (C / 8)) * 8;
      const int y = y0 + p / kTile, x = x0 + p % kTile;
      if (y < H && x < W) *reinterpret_cast<uint4*>(g + (((size_t)b * H + y) * W + x) * C + ch) = make_uint4(0, 0, 0, 0);
    }
    return;
  }
  int np = 1;
  while (np < n) np <<= 1;
  for (int i = tid; i < np; i += 256) keys[i] = i < n ? entries[ebeg + i] : 0x7fffffff;
  __syncthreads();
  if (nch == 1)
    for (int kk = 2; kk <= np; kk <<= 1)
      for (int jj = kk >> 1; jj > 0; jj >>= 1) {
        for (int i = tid; i < np; i += 256) {
          const int p = i ^ jj;
          if (p > i) {
            const int a = keys[i], c = keys[p];
            if ((a > c) == ((i & kk) == 0)) { keys[i] = c; keys[p] = a; }
          }
        }
        __syncthreads();
      }
  for (int i = tid; i < n; i += 256) fs[i] = fp[keys[i]];
  __syncthreads();

  // dY staging: thread t moves chunks q = t + 256 u (u < 4) of the K-step: row q / 32, logical
  // 16-B chunk q % 32, stored at its swizzled position
  uint4 dv[4];
  auto load_rows = [&](int e0) __attribute__((always_inline)) {
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int q = tid + 256 * u, e = e0 + (q >> 5), c = q & 31;
      dv[u] = e < n ? *reinterpret_cast<const uint4*>(dout + (size_t)keys[e] * C + 8 * c) : make_uint4(0, 0, 0, 0);
    }
  };
  auto store_rows = [&]() __attribute__((always_inline)) {
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int q = tid + 256 * u, e = q >> 5, c = q & 31;
      *reinterpret_cast<uint4*>(dimg + e * RB + gemm::pchunk(e, c) * 16) = dv[u];
    }
  };
  // W image [px][e]: 64-B rows, 16-B chunk (e >> 3) at (e >> 3) ^ ((px >> 2) & 3)
  auto woff = [](int px, int e) __attribute__((always_inline)) {
    return px * (kMKS * 2) + (((e >> 3) ^ ((px >> 2) & 3)) << 4) + (e & 7) * 2;
  };

  // fragments: A = dY^T (16 channels x 32 entries) by transposed reads, B = W (32 entries x
  // 16 pixels); lane (G, i) of the 16x16 output holds channels 4G .. 4G + 3 of pixel i
  const int G4 = lane >> 4, i16 = lane & 15;
  const int krow = 8 * G4 + (i16 >> 2);
  int offA[4];
#pragma unroll
  for (int cb = 0; cb < 4; ++cb) {
    const int pair = 4 * wave + cb;                 // 16-channel block = 32-B chunk pair
    offA[cb] = krow * RB + (((pair ^ gemm::gsw(krow)) << 1) | ((i16 & 3) >> 1)) * 16 + (i16 & 1) * 8;
  }
  f32x4 acc[4][4];
#pragma unroll
  for (int cb = 0; cb < 4; ++cb)
#pragma unroll
    for (int pb = 0; pb < 4; ++pb) acc[cb][pb] = f32x4{0.f, 0.f, 0.f, 0.f};

  load_rows(0);
  for (int e0 = 0; e0 < n; e0 += kMKS) {
    store_rows();
    // zero both W images (8 KB: two 16-B stores per thread)
    reinterpret_cast<uint4*>(whi)[tid] = make_uint4(0, 0, 0, 0);
    reinterpret_cast<uint4*>(whi)[tid + 256] = make_uint4(0, 0, 0, 0);
    __syncthreads();
    // scatter the footprints: thread t takes entry e0 + (t & 31), slots (t >> 5) and + 8
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int el = tid & 31, slot = (tid >> 5) + 8 * h;
      const int e = e0 + el;
      if (e < n) {
        const FootP& f = fs[e];
        const int si = slot >> 2, sj = slot & 3;
        const float w = f.wy[si] * f.wx[sj];
        const int yy = f.ry[si] - y0, xx = f.rx[sj] - x0;
        if (w != 0.f && (unsigned)yy < (unsigned)kTile && (unsigned)xx < (unsigned)kTile) {
          const int px = yy * kTile + xx;
          const __bf16 hi = (__bf16)w;
          const __bf16 lo = (__bf16)(w - (float)hi);
          *reinterpret_cast<__bf16*>(whi + woff(px, el)) = hi;
          *reinterpret_cast<__bf16*>(wlo + woff(px, el)) = lo;
        }
      }
    }
    if (e0 + kMKS < n) load_rows(e0 + kMKS);      // next K-step's rows in flight during the MFMAs
    __syncthreads();
    bf16x8 a[4];
#pragma unroll
    for (int cb = 0; cb < 4; ++cb) a[cb] = gemm::cat(gemm::tr_read(dimg, offA[cb]), gemm::tr_read(dimg, offA[cb] + 4 * RB));
#pragma unroll
    for (int pb = 0; pb < 4; ++pb) {
      const int px = 16 * pb + i16;
      const int wo = px * (kMKS * 2) + ((G4 ^ ((px >> 2) & 3)) << 4);
      const bf16x8 bh = gemm::lds_read8(whi, wo), bl = gemm::lds_read8(wlo, wo);
#pragma unroll
      for (int cb = 0; cb < 4; ++cb) {
        acc[cb][pb] = gemm::mfma16(a[cb], bh, acc[cb][pb]);
        acc[cb][pb] = gemm::mfma16(a[cb], bl, acc[cb][pb]);
      }
    }
    __syncthreads();   // the next K-step rewrites the images
  }
  // accumulators -> fp32 tile [64 px][256 c] (aliases the images: every wave is past its last
  // read -- the loop's final barrier)
#pragma unroll
  for (int cb = 0; cb < 4; ++cb)
#pragma unroll
    for (int pb = 0; pb < 4; ++pb)
      *reinterpret_cast<f32x4*>(acc_t + (16 * pb + i16) * C + 64 * wave + 16 * cb + 4 * G4) = acc[cb][pb];
  __syncthreads();
  if (dbg && tid == 0) {
    dbg[4 * k] = k; dbg[4 * k + 1] = tile; dbg[4 * k + 2] = n;
    dbg[4 * k + 3] = (long long)__builtin_amdgcn_s_memrealtime() - t_start;
  }
  if (nch == 1) {
    write_tile_bf16(acc_t, gout.p[lv], C, H, W, b, y0, x0, tid, 256);
    return;
  }
  const int slot = poff[tile] + j;
  if (slot >= pslots) {
    if (tid == 0) atomicAdd(overflow, 1);
    return;
  }
  float* dst = partial + (size_t)slot * kTile * kTile * C;
  for (int i = tid * 4; i < kTile * kTile * C; i += 256 * 4)
    *reinterpret_cast<float4*>(dst + i) = *reinterpret_cast<const float4*>(acc_t + i);
}

// split tiles: sum the chunk partials in chunk order -> bf16
__global__ __launch_bounds__(256) void roi_align_bwd_combine_kernel(Levels L, TileGeo G, int C,
                                                                    const int* __restrict__ coff,
                                                                    const int* __restrict__ poff,
                                                                    const float* __restrict__ partial, int pslots,
                                                                    GOut gout) {
  const int tile = blockIdx.x;
  const int nch = coff[tile + 1] - coff[tile];
  if (nch <= 1 || poff[tile] + nch > pslots) return;
  int lv, b, ty, tx;
  decode_tile(L, G, tile, lv, b, ty, tx);
  const int H = L.H[lv], W = L.W[lv];
  const int y0 = ty * kTile, x0 = tx * kTile;
  const float* src = partial + (size_t)poff[tile] * kTile * kTile * C;
  const int c8 = C / 8;
  for (int q = threadIdx.x; q < kTile * kTile * c8; q += blockDim.x) {
    const int p = q / c8, ch = (q % c8) * 8;
    const int y = y0 + p / kTile, x = x0 + p % kTile;
    if (y >= H || x >= W) continue;
    float s[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    for (int jj = 0; jj < nch; ++jj) {
      const float* a = src + (size_t)jj * kTile * kTile * C + p * C + ch;
#pragma unroll
      for (int e = 0; e < 8; ++e) s[e] += a[e];
    }
    *reinterpret_cast<uint4*>(gout.p[lv] + (((size_t)b * H + y) * W + x) * C + ch) = pack8(s);
  }
}

// ------------------------------------------------------------------------------ NMS
__device__ __forceinline__ float iou4(const float4 a, const float4 b) {
  const float iw = fminf(a.z, b.z) - fmaxf(a.x, b.x);
  const float ih = fminf(a.w, b.w) - fmaxf(a.y, b.y);
  if (iw <= 0.f || ih <= 0.f) return 0.f;
  const float inter = iw * ih;
  const float ua = (a.z - a.x) * (a.w - a.y) + (b.z - b.x) * (b.w - b.y) - inter;
  return inter / fmaxf(ua, 1e-12f);
}

// boxes: [P, N, 4] sorted by score (desc) per problem; counts[P] valid boxes.
// mask: [P, N, NB] uint64, bit j of word (i, cb) set when box cb*64+j (> i) overlaps i.
// colmask (nullable): [P, N] uint64, bit j set when box (i & ~63) + j (< i) overlaps i -- the
// transposed diagonal block, for the parallel in-chunk scan of nms_keep_par_kernel
__global__ __launch_bounds__(64) void nms_mask_kernel(const float4* __restrict__ boxes, const int* __restrict__ counts,
                                                      int N, int NB, float thr,
                                                      unsigned long long* __restrict__ mask,
                                                      unsigned long long* __restrict__ colmask) {
  const int cb = blockIdx.x, rb = blockIdx.y, p = blockIdx.z;
  const int n = counts ? counts[p] : N;
  const int t = threadIdx.x;
  const int i = rb * 64 + t;
  if (cb < rb || rb * 64 >= n) return;
  __shared__ float4 cbox[64];
  const int j0 = cb * 64;
  if (j0 + t < n) cbox[t] = boxes[(size_t)p * N + j0 + t];
  __syncthreads();
  if (i >= n) return;
  const float4 bi = boxes[(size_t)p * N + i];
  unsigned long long bits = 0ull, col = 0ull;
  const int jn = min(64, n - j0);
  for (int j = 0; j < jn; ++j) {
    const bool ov = iou4(bi, cbox[j]) > thr;
    if (j0 + j > i && ov) bits |= (1ull << j);
    if (j0 + j < i && ov) col |= (1ull << j);
  }
  mask[((size_t)p * N + i) * NB + cb] = bits;
  if (colmask && cb == rb) colmask[(size_t)p * N + i] = col;
}

// one wave per problem; lane w owns removed-word w (NB <= NBM <= 64 -> N <= 64 NBM)
//
// Chunks of 64 boxes.  The chunk's 64 mask rows (only their words cw .. NB-1 matter: the
// mask is upper-triangular) are loaded into registers one chunk AHEAD -- issued before the
// current chunk's serial scan, so their L2 latency hides behind it -- and staged in LDS.
// (Loading each chunk's rows with a load -> ds_write loop after the previous chunk had
// finished serialised ~NB dependent L2 round trips per chunk: ~0.5 ms for the 5 x 2000-box
// RPN problems of a training step.)  The serial keep/suppress decision reads each row's
// word of the chunk itself with a scalar readlane (SALU chain, surviving candidates only);
// the kept rows' suppression of later
// chunks is OR-ed in parallel (lane w owns word w) with a fully unrolled, branch-free pass.
template <int NBM>
__global__ __launch_bounds__(64) void nms_keep_kernel(const unsigned long long* __restrict__ mask,
                                                      const int* __restrict__ counts, int N, int NB,
                                                      int max_out, int* __restrict__ keep,
                                                      int* __restrict__ nkeep) {
  const int p = blockIdx.x;
  const int lane = threadIdx.x;
  const int n = counts ? counts[p] : N;
  __shared__ unsigned long long rows[64 * NBM];
  unsigned long long removed = 0ull;
  int out = 0;
  const unsigned long long* m = mask + (size_t)p * N * NB;
  // lane's share of a chunk: flat indices k = lane + 64 q of [cn rows][NB words]
  unsigned long long pre[NBM];
  // (row, word) of flat index k: r = k / NB by a float reciprocal (exact for k < 4096),
  // not an integer division by a runtime divisor (~40 VALU ops each)
  const float inv_nb = 1.f / (float)NB;
  // The loads are unconditional (out-of-range entries read word 0 of the problem) and the
  // validity mask is applied when the chunk is staged: a `cond ? load : 0` select made the
  // compiler wait for every load right after issuing it (33 vmcnt(0) waits per chunk
  // -> ~8 us per chunk, the whole prefetch serialised).
  unsigned long long valid = 0ull;   // bit q: entry q of the lane's share is in range
  auto fetch = [&](int c0) __attribute__((always_inline)) {
    const int cn = min(64, n - c0), cw = c0 >> 6;
    valid = 0ull;
#pragma unroll
    for (int q = 0; q < NBM; ++q) {
      const int k = lane + 64 * q;
      const int r = (int)(((float)k + 0.5f) * inv_nb), w = k - r * NB;
      const bool ok = q < NB && r < cn && w >= cw;
      valid |= (ok ? 1ull : 0ull) << q;
      pre[q] = m[ok ? (size_t)c0 * NB + k : 0];
    }
  };
  if (n > 0) fetch(0);
  for (int c0 = 0; c0 < n && out < max_out; c0 += 64) {
    const int cn = min(64, n - c0);
#pragma unroll
    for (int q = 0; q < NBM; ++q)
      if (q < NB) rows[lane + 64 * q] = ((valid >> q) & 1ull) ? pre[q] : 0ull;
    __syncthreads();
    if (c0 + 64 < n) fetch(c0 + 64);      // next chunk in flight during this one's scan
    const int cw = c0 >> 6;
    const unsigned long long intra = lane < cn ? rows[lane * NB + cw] : 0ull;
    const unsigned lo = (unsigned)intra, hi = (unsigned)(intra >> 32);
    // the scan runs on SCALAR registers: the removed word is made wave-uniform with
    // readfirstlane (a __shfl result is a VGPR to the divergence analysis, which had turned
    // the whole chain into exec-masked vector code at ~350 cycles per box); it visits only
    // the surviving candidates (lowest first): kept |= ii, candidates &= ~row(ii)
    const unsigned long long word = __shfl(removed, cw);
    unsigned long long avail =
        ((unsigned long long)(unsigned)__builtin_amdgcn_readfirstlane((int)(unsigned)(word >> 32)) << 32) |
        (unsigned)__builtin_amdgcn_readfirstlane((int)(unsigned)word);
    avail = ~avail & (cn == 64 ? ~0ull : ((1ull << cn) - 1ull));
    unsigned long long kept = 0ull;
    int room = __builtin_amdgcn_readfirstlane(max_out - out);
    while (avail && room > 0) {
      const int ii = __builtin_ctzll(avail);
      kept |= 1ull << ii;
      --room;
      avail &= avail - 1ull;
      const unsigned long long row = ((unsigned long long)(unsigned)__builtin_amdgcn_readlane((int)hi, ii) << 32) |
                                     (unsigned)__builtin_amdgcn_readlane((int)lo, ii);
      avail &= ~row;
    }
    if ((kept >> lane) & 1ull)
      keep[(size_t)p * max_out + out + __popcll(kept & ((1ull << lane) - 1ull))] = c0 + lane;
    out += __popcll(kept);
    if (lane < NB && lane > cw) {
      unsigned long long acc = removed;
      // batches of 8 independent LDS reads, then the masked OR (kept bit ii: all-ones select;
      // never set for ii >= cn, whose LDS rows are stale); a guarded read per row had the
      // compiler wait for each one
#pragma unroll
      for (int i0 = 0; i0 < 64; i0 += 8) {
        unsigned long long v8[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) v8[j] = rows[(i0 + j) * NB + lane];
#pragma unroll
        for (int j = 0; j < 8; ++j) acc |= v8[j] & (0ull - ((kept >> (i0 + j)) & 1ull));
      }
      removed = acc;
    }
    __syncthreads();
  }
  if (lane == 0) nkeep[p] = out;
  for (int k = out + lane; k < max_out; k += 64) keep[(size_t)p * max_out + k] = -1;
}

// nms_keep_kernel with the in-chunk greedy decided in parallel: box i of a chunk is kept iff it
// is not suppressed by earlier chunks (avail) and no KEPT box j < i of the chunk overlaps it.
// Lane i holds the transposed diagonal block (colmask: its earlier overlapping boxes), and
// the kept set K is iterated to its fixed point, K' = ballot(avail_i && !(col_i & K)) from
// K = avail: the greedy set is the map's only fixed point and box t's status is final after
// t + 1 rounds, so the loop ends (typically after a few rounds, not 64 serial steps with two
// v_readlane each).  The fetch (one chunk ahead), the staging and the suppression OR-pass are
// those of nms_keep_kernel.
template <int NBM>
__global__ __launch_bounds__(256) void nms_keep_par_kernel(const unsigned long long* __restrict__ mask,
                                                           const unsigned long long* __restrict__ colmask,
                                                           const int* __restrict__ counts, int N, int NB,
                                                           int max_out, int* __restrict__ keep,
                                                           int* __restrict__ nkeep) {
  // LDS-DMA ring of DEPTH chunks (DEPTH - 1 in flight during a chunk's scan): a chunk's mask
  // rows are one contiguous [64][NB] block, its transposed diagonal words [64] another; both
  // land by buffer_load ... lds (reads past the problem's last row return zeros).  Four waves
  // per problem: each issues a quarter of the DMA pieces and ORs a quarter of the kept rows
  // into the suppression words (LDS ds_or_b64); every wave evaluates the (wave-uniform, cheap)
  // fixed-point scan itself.  One wave doing all of it spent ~2.5 us per chunk in DMA issue
  // and the 64-row OR pass (profiles/r5_s1/nms_lds_ring.txt).
  constexpr int DEPTH = 4;
  constexpr int RB = 64 * NBM * 8;                 // row bytes of a slot
  // + 1 KiB for the colmask words + 1 KiB that the padding pieces fill with zeros (an
  // out-of-range buffer_load ... lds still WRITES its zeros: aimed at the colmask words, a
  // padding piece raced the real one)
  constexpr int SLOTB = RB + 2048;
  constexpr int NP = NBM / 2 + 1;                  // DMA pieces per chunk
  constexpr int PW = (NP + 3) / 4;                 // pieces per wave
  __shared__ __attribute__((aligned(1024))) char ring[DEPTH * SLOTB];
  __shared__ unsigned long long sremoved[NBM];
  const int p = blockIdx.x;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wv = __builtin_amdgcn_readfirstlane(tid >> 6);   // wave-uniform (SGPR LDS bases)
  const int n = counts ? counts[p] : N;
  if (tid < NBM) sremoved[tid] = 0ull;
  int out = 0;
  const gemm::i32x4_t mres = gemm::buffer_rsrc(mask + (size_t)p * N * NB, (uint32_t)((size_t)n * NB * 8));
  const gemm::i32x4_t cres = gemm::buffer_rsrc(colmask + (size_t)p * N, (uint32_t)((size_t)n * 8));
  const uint32_t ring0 = gemm::lds_addr(ring);
  const int nchunks = (n + 63) >> 6;
  auto issue = [&](int c) __attribute__((always_inline)) {
    const uint32_t base = __builtin_amdgcn_readfirstlane(ring0 + (c % DEPTH) * SLOTB);
    const uint32_t src = (uint32_t)c * 64u * (uint32_t)NB * 8u;
#pragma unroll
    for (int k = 0; k < PW; ++k) {
      const int q = wv + 4 * k;                    // piece q of the chunk (NP - 1: colmask)
      if (q < NP - 1)
        gemm::dma16_buf(mres, 2 * q < NB ? src + 1024u * q + 16u * lane : gemm::kOOB, base + 1024 * q);
      else if (q == NP - 1)
        gemm::dma16_buf(cres, (uint32_t)c * 512u + 16u * lane, base + RB);
      else   // (keeps the per-wave piece count uniform for the counted waits)
        gemm::dma16_buf(cres, gemm::kOOB + 0u * lane, base + RB + 1024);
    }
  };
  for (int c = 0; c < DEPTH - 1; ++c)
    if (c < nchunks) issue(c);
  __syncthreads();   // sremoved initialised
  for (int c = 0; c < nchunks && out < max_out; ++c) {
    const int later = min(nchunks - 1 - c, DEPTH - 2);   // chunks issued after this one
    if (later >= 2) gemm::vm_wait<2 * PW>();
    else if (later == 1) gemm::vm_wait<PW>();
    else gemm::vm_wait<0>();
    __syncthreads();   // every wave's pieces of chunk c have landed
    const int c0 = c << 6, cn = min(64, n - c0), cw = c;
    const char* slot = ring + (c % DEPTH) * SLOTB;
    const unsigned long long* rows = reinterpret_cast<const unsigned long long*>(slot);
    const unsigned long long col = lane < cn ? reinterpret_cast<const unsigned long long*>(slot + RB)[lane] : 0ull;
    const unsigned long long word = sremoved[cw];
    const bool av = lane < cn && !((word >> lane) & 1ull);
    unsigned long long K = __ballot(av);
    for (;;) {
      const unsigned long long Kn = __ballot(av && (col & K) == 0ull);
      if (Kn == K) break;
      K = Kn;
    }
    const int room = max_out - out;
    unsigned long long kept = K;
    if (__popcll(K) > room)   // greedy order is index order: the first `room` kept boxes
      kept = __ballot(((K >> lane) & 1ull) && __popcll(K & ((1ull << lane) - 1ull)) < room);
    if (wv == 0 && ((kept >> lane) & 1ull))
      keep[(size_t)p * max_out + out + __popcll(kept & ((1ull << lane) - 1ull))] = c0 + lane;
    out += __popcll(kept);
    // this wave's 16 rows of the chunk (rows past cn are never kept)
    const unsigned long long mine = (kept >> (16 * wv)) & 0xFFFFull;
    if (mine && lane < NB && lane > cw) {
      unsigned long long acc = 0ull;
#pragma unroll
      for (int i0 = 0; i0 < 16; i0 += 8) {
        unsigned long long v8[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) v8[j] = rows[(16 * wv + i0 + j) * NB + lane];
#pragma unroll
        for (int j = 0; j < 8; ++j) acc |= v8[j] & (0ull - ((mine >> (i0 + j)) & 1ull));
      }
      if (acc) atomicOr(&sremoved[lane], acc);
    }
    __syncthreads();   // the slot's reads and the suppression words are complete
    if (c + DEPTH - 1 < nchunks) issue(c + DEPTH - 1);
  }
  gemm::vm_wait<0>();   // no LDS-DMA outstanding at exit (early max_out stop)
  if (tid == 0) nkeep[p] = out;
  for (int k = out + tid; k < max_out; k += 256) keep[(size_t)p * max_out + k] = -1;
}

// ------------------------------------------------------------------ RPN level top-k + decode
// Per (image, FPN level) row: the k highest bf16 objectness logits, sorted (ties: lower
// anchor index first), with their boxes decoded from (anchor, bf16 delta) and clipped --
// the proposal front-end of tensorpack's generate_fpn_proposals.
// torch's topk with k = 2000 over ~200k-anchor rows went through a segmented merge sort
// (~13 launches per level) followed by gather / index / decode / pad / stack kernels:
// ~100 launches and ~0.5 ms per step; here 5 launches cover every row of the step.
//   1. hist_hi : 256-bin histogram of the order-preserving 16-bit key's high byte
//   2. hist_lo : low byte, restricted to the high-byte bucket holding the k-th key
//   3. count   : per chunk, keys > T and == T (T = the k-th largest key)
//   4. compact : keys > T, then the first (k - #>T) keys == T in anchor order, into the
//                row's candidate list (ordered in-block compaction: wave ballots)
//   5. sort    : bitonic sort of (key, ~index) in LDS, decode + clip, -inf padding; zeroes
//                the histograms for the next call
// Row table (int64 x 6): {logits (bf16), deltas (bf16, [n][4]), anchors (fp32 [n][4]), n,
// image, unused}; chunk table: first chunk of each row (row r owns chunks c0[r]..c0[r+1]).
constexpr int kTkChunk = 4096;
constexpr int kTkMaxK = 2048;

__device__ __forceinline__ uint32_t bf_key(uint16_t u) {
  return (u & 0x8000u) ? (~(uint32_t)u & 0xFFFFu) : ((uint32_t)u | 0x8000u);
}
__device__ __forceinline__ float key_to_float(uint32_t k) {
  const uint32_t u = (k & 0x8000u) ? (k & 0x7FFFu) : (~k & 0xFFFFu);
  return __uint_as_float(u << 16);
}
__device__ __forceinline__ int tk_row(const int* __restrict__ c0, int R, int blk) {
  int r = 0;
  while (r + 1 < R && c0[r + 1] <= blk) ++r;
  return r;
}
// bucket of the k-th largest entry of a 256-bin histogram (descending scan) and the rank
// still needed inside it; one thread, histogram staged in LDS
__device__ __forceinline__ void tk_pick(const int* __restrict__ hist, int k, int& bin, int& rem) {
  int acc = 0;
  bin = 0;
  rem = k;
  for (int b = 255; b >= 0; --b) {
    const int h = hist[b];
    if (acc + h >= k) { bin = b; rem = k - acc; return; }
    acc += h;
  }
}

__global__ __launch_bounds__(256) void tk_hist_kernel(const int64_t* __restrict__ rows, const int* __restrict__ c0, int R,
                                                      int K, int* __restrict__ hist1, int* __restrict__ hist2,
                                                      int pass) {
  __shared__ int h[256];
  __shared__ int sh[256];
  __shared__ int sel[2];
  const int blk = blockIdx.x, t = threadIdx.x;
  const int r = tk_row(c0, R, blk);
  const int64_t* rw = rows + 6 * r;
  const uint16_t* lg = reinterpret_cast<const uint16_t*>(rw[0]);
  const int n = (int)rw[3], k = min(K, n);
  h[t] = 0;
  if (pass == 1) sh[t] = hist1[r * 256 + t];
  __syncthreads();
  if (pass == 1 && t == 0) {
    int b, rem;
    tk_pick(sh, k, b, rem);
    sel[0] = b;
  }
  __syncthreads();
  const int hi = pass == 1 ? sel[0] : -1;
  const int e0 = (blk - c0[r]) * kTkChunk;
#pragma unroll 4
  for (int j = 0; j < kTkChunk / 256; ++j) {
    const int e = e0 + j * 256 + t;
    if (e < n) {
      const uint32_t key = bf_key(lg[e]);
      if (pass == 0) atomicAdd(&h[key >> 8], 1);
      else if ((int)(key >> 8) == hi) atomicAdd(&h[key & 255], 1);
    }
  }
  __syncthreads();
  if (h[t]) atomicAdd((pass == 0 ? hist1 : hist2) + r * 256 + t, h[t]);
}

// threshold key of row r (from both histograms) and the number of == T keys to take
__device__ __forceinline__ void tk_threshold(const int* __restrict__ hist1, const int* __restrict__ hist2, int r, int k,
                                             int* sh, int& T, int& need_eq) {
  __shared__ int res[2];
  const int t = threadIdx.x;
  sh[t] = hist1[r * 256 + t];
  __syncthreads();
  int b1 = 0, rem1 = 0;
  if (t == 0) tk_pick(sh, k, b1, rem1);
  __syncthreads();
  sh[t] = hist2[r * 256 + t];
  __syncthreads();
  if (t == 0) {
    int b2, rem2;
    tk_pick(sh, rem1, b2, rem2);
    res[0] = (b1 << 8) | b2;
    res[1] = rem2;
  }
  __syncthreads();
  T = res[0];
  need_eq = res[1];
}

__global__ __launch_bounds__(256) void tk_count_kernel(const int64_t* __restrict__ rows, const int* __restrict__ c0,
                                                       int R, int K, const int* __restrict__ hist1,
                                                       const int* __restrict__ hist2, int2* __restrict__ bcnt) {
  __shared__ int sh[256];
  __shared__ int red[2][4];
  const int blk = blockIdx.x, t = threadIdx.x;
  const int r = tk_row(c0, R, blk);
  const int64_t* rw = rows + 6 * r;
  const uint16_t* lg = reinterpret_cast<const uint16_t*>(rw[0]);
  const int n = (int)rw[3], k = min(K, n);
  int T, need;
  tk_threshold(hist1, hist2, r, k, sh, T, need);
  const int e0 = (blk - c0[r]) * kTkChunk;
  int gt = 0, eq = 0;
#pragma unroll 4
  for (int j = 0; j < kTkChunk / 256; ++j) {
    const int e = e0 + j * 256 + t;
    if (e < n) {
      const int key = (int)bf_key(lg[e]);
      gt += key > T;
      eq += key == T;
    }
  }
  gt = (int)wave_sum((float)gt);   // exact: counts <= 4096
  eq = (int)wave_sum((float)eq);
  if ((t & 63) == 0) { red[0][t >> 6] = gt; red[1][t >> 6] = eq; }
  __syncthreads();
  if (t == 0)
    bcnt[blk] = make_int2(red[0][0] + red[0][1] + red[0][2] + red[0][3], red[1][0] + red[1][1] + red[1][2] + red[1][3]);
}

__global__ __launch_bounds__(256) void tk_compact_kernel(const int64_t* __restrict__ rows, const int* __restrict__ c0,
                                                         int R, int K, const int* __restrict__ hist1,
                                                         const int* __restrict__ hist2, const int2* __restrict__ bcnt,
                                                         uint2* __restrict__ cand) {
  __shared__ int sh[256];
  __shared__ int wc[2][4];
  const int blk = blockIdx.x, t = threadIdx.x, lane = t & 63, w = t >> 6;
  const int r = tk_row(c0, R, blk);
  const int64_t* rw = rows + 6 * r;
  const uint16_t* lg = reinterpret_cast<const uint16_t*>(rw[0]);
  const int n = (int)rw[3], k = min(K, n);
  int T, need;
  tk_threshold(hist1, hist2, r, k, sh, T, need);
  int base_gt = 0, base_eq = 0, tot_gt = 0;
  for (int c = c0[r]; c < c0[r + 1]; ++c) {
    const int2 v = bcnt[c];
    if (c < blk) { base_gt += v.x; base_eq += v.y; }
    tot_gt += v.x;
  }
  uint2* out = cand + (size_t)r * kTkMaxK;
  const int e0 = (blk - c0[r]) * kTkChunk;
  const unsigned long long below = (1ull << lane) - 1ull;
  for (int j = 0; j < kTkChunk / 256; ++j) {
    const int e = e0 + j * 256 + t;
    const int key = e < n ? (int)bf_key(lg[e]) : -1;
    const bool g = key > T, q = key == T;
    const unsigned long long bg = __ballot(g), bq = __ballot(q);
    if (lane == 0) { wc[0][w] = __popcll(bg); wc[1][w] = __popcll(bq); }
    __syncthreads();
    int og = 0, oq = 0, sg = 0, sq = 0;
#pragma unroll
    for (int x = 0; x < 4; ++x) {
      if (x < w) { og += wc[0][x]; oq += wc[1][x]; }
      sg += wc[0][x];
      sq += wc[1][x];
    }
    if (g) {
      const int pos = base_gt + og + __popcll(bg & below);
      out[pos] = make_uint2((uint32_t)key, (uint32_t)e);
    } else if (q) {
      const int re = base_eq + oq + __popcll(bq & below);
      if (re < need) out[tot_gt + re] = make_uint2((uint32_t)key, (uint32_t)e);
    }
    base_gt += sg;
    base_eq += sq;
    __syncthreads();
  }
}

// row / chunk tables from kernel arguments (capture-safe: no host staging buffer)
constexpr int kTkMaxRows = 24;
struct TkArgs {
  int64_t rows[kTkMaxRows * 6];
  int c0[kTkMaxRows + 1];
};
__global__ void tk_setup_kernel(const TkArgs a, int64_t* __restrict__ rows, int* __restrict__ c0) {
  if (threadIdx.x != 0) return;
#pragma unroll
  for (int i = 0; i < kTkMaxRows * 6; ++i) rows[i] = a.rows[i];
#pragma unroll
  for (int i = 0; i <= kTkMaxRows; ++i) c0[i] = a.c0[i];
}

// one 1024-thread block per row: sort the k candidates (key desc, index asc), decode
__global__ __launch_bounds__(1024) void tk_sort_decode_kernel(const int64_t* __restrict__ rows, int K,
                                                              const uint2* __restrict__ cand,
                                                              const float* __restrict__ img_hw, float clamp,
                                                              float4* __restrict__ boxes, float* __restrict__ scores,
                                                              int* __restrict__ hist1, int* __restrict__ hist2) {
  __shared__ unsigned long long v[kTkMaxK];
  const int r = blockIdx.x, t = threadIdx.x;
  const int64_t* rw = rows + 6 * r;
  const int n = (int)rw[3], k = min(K, n), im = (int)rw[4];
  int P = 1;
  while (P < K) P <<= 1;
  for (int i = t; i < P; i += 1024) {
    const uint2 c = i < k ? cand[(size_t)r * kTkMaxK + i] : make_uint2(0u, 0u);
    v[i] = i < k ? (((unsigned long long)(c.x + 1u) << 32) | (uint32_t)(~c.y)) : 0ull;   // key + 1: pads sort last
  }
  if (t < 256) { hist1[r * 256 + t] = 0; hist2[r * 256 + t] = 0; }
  __syncthreads();
  for (int size = 2; size <= P; size <<= 1) {
    for (int stride = size >> 1; stride > 0; stride >>= 1) {
      for (int i = t; i < P / 2; i += 1024) {
        const int lo = 2 * i - (i & (stride - 1)), hi = lo + stride;
        const bool desc = (lo & size) == 0;
        const unsigned long long a = v[lo], b = v[hi];
        if ((a < b) == desc) { v[lo] = b; v[hi] = a; }
      }
      __syncthreads();
    }
  }
  const uint16_t* dl = reinterpret_cast<const uint16_t*>(rw[1]);
  const float4* an = reinterpret_cast<const float4*>(rw[2]);
  const float H = img_hw[2 * im], W = img_hw[2 * im + 1];
  for (int i = t; i < K; i += 1024) {
    float4 o = make_float4(0.f, 0.f, 0.f, 0.f);
    float sc = -INFINITY;
    if (i < k) {
      const unsigned long long x = v[i];
      const uint32_t key = (uint32_t)(x >> 32) - 1u;
      const int idx = (int)(~(uint32_t)x);
      sc = key_to_float(key);
      const float4 a = an[idx];
      const uint2 dr = *reinterpret_cast<const uint2*>(dl + (size_t)idx * 4);
      const float d0 = lo_bf(dr.x), d1 = hi_bf(dr.x), d2 = lo_bf(dr.y), d3 = hi_bf(dr.y);
      const float w = a.z - a.x, h = a.w - a.y;
      const float cx = a.x + 0.5f * w, cy = a.y + 0.5f * h;
      const float dw = fminf(d2, clamp), dh = fminf(d3, clamp);
      const float pcx = d0 * w + cx, pcy = d1 * h + cy;
      const float pw = __expf(dw) * w, ph = __expf(dh) * h;
      o = make_float4(fminf(fmaxf(pcx - 0.5f * pw, 0.f), W), fminf(fmaxf(pcy - 0.5f * ph, 0.f), H),
                      fminf(fmaxf(pcx + 0.5f * pw, 0.f), W), fminf(fmaxf(pcy + 0.5f * ph, 0.f), H));
    }
    boxes[(size_t)r * K + i] = o;
    scores[(size_t)r * K + i] = sc;
  }
}

// ------------------------------------------------------------------ generic row top-k
// The k largest (or smallest) fp32 values of each row, sorted, ties by lower index, with
// their indices -- the large-k selections of the Mask R-CNN step (post-NMS top 2000 of
// ~10000 proposals, RoI sampling's 512 of ~2000 candidates, the rank-based fg/bg picks),
// which torch's topk serves with a rocprim segmented merge sort (~40 launches and ~0.3 ms
// per step, profiles/r2_maskrcnn_s4/README.md).  One 1024-thread workgroup per row, ONE
// launch per call:
//   1. radix select on the order-preserving u32 key, 4 passes of 8 bits (LDS histogram of
//      the keys that match the prefix so far; wave 0 finds the bin holding the k-th key)
//      -> threshold T and the number of == T keys still needed;
//   2. keys > T land in a candidate list in any order; keys == T in index order (ballot
//      prefix sums) until the need is met;
//   3. bitonic sort of the <= 2048 (key, ~index) pairs in LDS, values re-read from the row.
constexpr int kTkrMaxK = 2048;
constexpr int kTkrLds = 12288;   // rows up to this long keep their keys in LDS for the passes

__device__ __forceinline__ uint32_t tkr_key(float f, bool largest) {
  const uint32_t u = __float_as_uint(f);
  const uint32_t k = (u & 0x80000000u) ? ~u : (u | 0x80000000u);
  return largest ? k : ~k;
}

// nc > 0 (chunk stage of a long row): workgroup r takes chunk r % nc (columns (r % nc) c ..
// + c, clipped to n_orig) of row r / nc and reports row-global indices.  imap (merge stage):
// the reported index is imap[r][local index] (the candidates' original positions).
__global__ __launch_bounds__(1024) void topk_rows_kernel(const float* __restrict__ x, int n, int ld, int k, int largest,
                                                         float* __restrict__ ov, int64_t* __restrict__ oi, int nc,
                                                         int n_orig, const int64_t* __restrict__ imap) {
  __shared__ int hist[256];
  __shared__ int sel[2];
  __shared__ int wc[16];
  __shared__ int ngt;
  __shared__ unsigned long long cand[kTkrMaxK];
  __shared__ uint32_t kbuf[kTkrLds];
  const int r = blockIdx.x, t = threadIdx.x, lane = t & 63, w = t >> 6;
  const int chunk = nc > 0 ? r % nc : 0;
  const float* row = nc > 0 ? x + (size_t)(r / nc) * ld + (size_t)chunk * n : x + (size_t)r * ld;
  const int n_in = n;
  if (nc > 0) n = min(n, n_orig - chunk * n_in);   // (the host keeps every chunk >= k long)
  const bool lg = largest != 0;
  const bool in_lds = n <= kTkrLds;   // (uniform)
  if (in_lds) {
    for (int e = t; e < n; e += 1024) kbuf[e] = tkr_key(row[e], lg);
  }
  auto key_at = [&](int e) __attribute__((always_inline)) -> uint32_t {
    return in_lds ? kbuf[e] : tkr_key(row[e], lg);
  };
  const unsigned long long below = (1ull << lane) - 1ull;
  uint32_t prefix = 0u, pmask = 0u;
  int rem = k;
  for (int pass = 0; pass < 4; ++pass) {
    const int shift = 24 - 8 * pass;
    if (t < 256) hist[t] = 0;
    __syncthreads();
    for (int e0 = 0; e0 < n; e0 += 1024) {
      const int e = e0 + t;
      const uint32_t key = e < n ? key_at(e) : 0u;
      const uint32_t bin = (key >> shift) & 255u;
      // Keys that share a prefix are concentrated (scores of one range, uniform draws in
      // [0, 1) share their exponent byte): same-address LDS atomics serialise per lane, so
      // the bins of the first two still-active lanes are counted with one atomic per wave
      // (ballot + popcount), the stragglers one by one.
      bool done = !(e < n && (key & pmask) == prefix);
#pragma unroll
      for (int pe = 0; pe < 2; ++pe) {
        const unsigned long long left = __ballot(!done);
        if (left == 0ull) break;
        const int first = __builtin_ctzll(left);
        const uint32_t b0 = (uint32_t)__shfl((int)bin, first);
        const unsigned long long same = __ballot(!done && bin == b0);
        if (lane == first) atomicAdd(&hist[b0], __popcll(same));
        done = done || bin == b0;
      }
      if (!done) atomicAdd(&hist[bin], 1);
    }
    __syncthreads();
    if (w == 0) {
      // lane l owns bins 255 - 4l .. 252 - 4l (top first); inclusive prefix over lanes
      int c[4], sum = 0;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        c[j] = hist[255 - 4 * lane - j];
        sum += c[j];
      }
      int incl = sum;
#pragma unroll
      for (int o = 1; o < 64; o <<= 1) {
        const int v = __shfl_up(incl, o);
        if (lane >= o) incl += v;
      }
      const int excl = incl - sum;
      if (excl < rem && incl >= rem) {
        int acc = excl, j = 0;
        for (; j < 3; ++j) {
          if (acc + c[j] >= rem) break;
          acc += c[j];
        }
        sel[0] = 255 - 4 * lane - j;
        sel[1] = rem - acc;
      }
    }
    __syncthreads();
    prefix |= (uint32_t)sel[0] << shift;
    pmask |= 255u << shift;
    rem = sel[1];
    __syncthreads();
  }
  const uint32_t T = prefix;
  const int need_eq = rem, n_gt = k - need_eq;
  if (t == 0) ngt = 0;
  __syncthreads();
  int eq_base = 0;
  for (int e0 = 0; e0 < n; e0 += 1024) {
    const int e = e0 + t;
    const uint32_t key = e < n ? key_at(e) : 0u;
    const bool gt = e < n && key > T, eq = e < n && key == T;
    const unsigned long long bgt = __ballot(gt);   // one slot-claiming atomic per wave
    if (bgt) {
      int b_ = 0;
      if (lane == 0) b_ = atomicAdd(&ngt, __popcll(bgt));
      b_ = __shfl(b_, 0);
      if (gt) cand[b_ + __popcll(bgt & below)] = ((unsigned long long)key << 32) | (uint32_t)(~(uint32_t)e);
    }
    const unsigned long long bq = __ballot(eq);
    if (lane == 0) wc[w] = __popcll(bq);
    __syncthreads();
    int off = 0, tot = 0;
#pragma unroll
    for (int x2 = 0; x2 < 16; ++x2) {
      off += x2 < w ? wc[x2] : 0;
      tot += wc[x2];
    }
    // ngt is read BETWEEN the two barriers: every add of this chunk happened before the
    // first one, and no wave can add for the next chunk before all have passed the second,
    // so every wave sees the same count and takes the same exit (a read after the second
    // barrier could race a fast wave's next-chunk atomicAdd and split the waves' exits)
    const int ngt_now = ngt;
    if (eq) {
      const int re = eq_base + off + __popcll(bq & below);
      if (re < need_eq) cand[n_gt + re] = ((unsigned long long)key << 32) | (uint32_t)(~(uint32_t)e);
    }
    eq_base += tot;
    __syncthreads();
    if (eq_base >= need_eq && ngt_now >= n_gt) break;   // uniform: wc and ngt_now are per-chunk snapshots
  }
  int P = 1;
  while (P < k) P <<= 1;
  for (int i = k + t; i < P; i += 1024) cand[i] = 0ull;   // pads sort last (descending)
  __syncthreads();
  for (int size = 2; size <= P; size <<= 1) {
    for (int stride = size >> 1; stride > 0; stride >>= 1) {
      for (int i = t; i < P / 2; i += 1024) {
        const int lo = 2 * i - (i & (stride - 1)), hi = lo + stride;
        const bool desc = (lo & size) == 0;
        const unsigned long long a = cand[lo], b = cand[hi];
        if ((a < b) == desc) { cand[lo] = b; cand[hi] = a; }
      }
      __syncthreads();
    }
  }
  for (int i = t; i < k; i += 1024) {
    const int idx = (int)(~(uint32_t)cand[i]);
    ov[(size_t)r * k + i] = row[idx];
    oi[(size_t)r * k + i] = imap ? imap[(size_t)r * n_in + idx] : (int64_t)chunk * n_in + idx;
  }
}

// ------------------------------------------------------------------ merge of sorted lists
// The top `top` of L score lists per image, each sorted non-increasing (the per-level NMS
// survivors, -inf padded): element (l, j) with score s has rank j + #{l' < l: a >= s} +
// #{l' > l: a > s} in the (score desc, flat index l * pre + j asc) order that topk_rows
// returns, found by binary search in the other lists (staged in LDS); ranks < top are
// written.  One pass over L * pre elements instead of a one-workgroup radix select + sort
// of the 10k candidates (~38 us per step at one image).
constexpr int kMergeMax = 16384;
__global__ __launch_bounds__(256) void merge_topk_kernel(const float* __restrict__ ks, int L, int pre, int top,
                                                         float* __restrict__ ov, int64_t* __restrict__ oi) {
  __shared__ float lst[kMergeMax];
  const int b = blockIdx.y, n = L * pre;
  const float* row = ks + (size_t)b * n;
  for (int e = threadIdx.x; e < n; e += 256) lst[e] = row[e];
  __syncthreads();
  const int e = blockIdx.x * 256 + threadIdx.x;
  if (e >= n) return;
  const int l = e / pre, j = e - l * pre;
  const float sv = lst[e];
  int rank = j;
  for (int m = 0; m < L; ++m) {
    if (m == l) continue;
    const float* a = lst + m * pre;
    // first index whose score is < s (m < l: equal scores rank first) or <= s (m > l)
    int lo = 0, hi = pre;
    if (m < l) {
      while (lo < hi) { const int mid = (lo + hi) >> 1; if (a[mid] >= sv) lo = mid + 1; else hi = mid; }
    } else {
      while (lo < hi) { const int mid = (lo + hi) >> 1; if (a[mid] > sv) lo = mid + 1; else hi = mid; }
    }
    rank += lo;
  }
  if (rank < top) {
    ov[(size_t)b * top + rank] = sv;
    oi[(size_t)b * top + rank] = e;
  }
}

// The proposal tail in one launch: per (image, level) problem p = b L + l, NMS survivor j is
// keep[p][j] (a row of the problem's score-sorted boxes, -1 padded); its score (-inf when
// padded) and box are read straight from the NMS inputs, ranked across the image's L sorted
// survivor lists as in merge_topk_kernel (same tie order), and the top `top` written as
// scores + boxes.  Replaces keep.long(), the validity mask, clamp, two gathers, the -inf fill
// / select, the merge and the final box gather (9 launches).
__global__ __launch_bounds__(256) void merge_keep_topk_kernel(const int* __restrict__ keep,
                                                              const float* __restrict__ scores,
                                                              const float4* __restrict__ boxes, int L, int pre,
                                                              int top, float* __restrict__ ov,
                                                              float4* __restrict__ ob) {
  __shared__ float lst[kMergeMax];
  const int b = blockIdx.y, n = L * pre;
  const size_t p0 = (size_t)b * L * pre;   // this image's first (problem, slot)
  for (int e = threadIdx.x; e < n; e += 256) {
    const int l = e / pre;
    const int k = keep[p0 + e];
    lst[e] = k >= 0 ? scores[p0 + (size_t)l * pre + k] : -INFINITY;
  }
  __syncthreads();
  const int e = blockIdx.x * 256 + threadIdx.x;
  if (e >= n) return;
  const int l = e / pre, j = e - l * pre;
  const float sv = lst[e];
  int rank = j;
  for (int m = 0; m < L; ++m) {
    if (m == l) continue;
    const float* a = lst + m * pre;
    int lo = 0, hi = pre;
    if (m < l) {
      while (lo < hi) { const int mid = (lo + hi) >> 1; if (a[mid] >= sv) lo = mid + 1; else hi = mid; }
    } else {
      while (lo < hi) { const int mid = (lo + hi) >> 1; if (a[mid] > sv) lo = mid + 1; else hi = mid; }
    }
    rank += lo;
  }
  if (rank < top) {
    const int k = keep[p0 + e];
    ov[(size_t)b * top + rank] = sv;
    ob[(size_t)b * top + rank] = boxes[p0 + (size_t)l * pre + (k > 0 ? k : 0)];
  }
}

// ------------------------------------------------------------------------------ matching
// per (image, anchor): max IoU over that image's gt boxes and its argmax; per gt: the
// best IoU over anchors (atomicMax on the float bits -- IoU >= 0).
__global__ __launch_bounds__(256) void match_kernel(const float4* __restrict__ anchors, int A, int per_image_anchors,
                                                    const float4* __restrict__ gt, const int* __restrict__ gcount,
                                                    int G, float* __restrict__ max_iou, int* __restrict__ argmax,
                                                    unsigned int* __restrict__ gt_best) {
  __shared__ float4 sg[256];
  const int b = blockIdx.y;
  const int a = blockIdx.x * blockDim.x + threadIdx.x;
  const int ng = gcount[b];
  const float4 an = a < A ? anchors[(per_image_anchors ? (size_t)b * A : 0) + a] : make_float4(0, 0, 0, 0);
  float best = -1.f;
  int bi = -1;
  for (int g0 = 0; g0 < ng; g0 += 256) {
    __syncthreads();
    if (g0 + (int)threadIdx.x < ng) sg[threadIdx.x] = gt[(size_t)b * G + g0 + threadIdx.x];
    __syncthreads();
    const int gn = min(256, ng - g0);
    for (int g = 0; g < gn; ++g) {
      const float v = a < A ? iou4(an, sg[g]) : 0.f;
      if (v > best) { best = v; bi = g0 + g; }
      // per-gt best, reduced within the wave first to cut atomics 64x (all lanes take
      // part: out-of-range anchors contribute 0)
      float wv = v;
      for (int o = 32; o > 0; o >>= 1) wv = fmaxf(wv, __shfl_xor(wv, o));
      if ((threadIdx.x & 63) == 0 && wv > 0.f) atomicMax(gt_best + (size_t)b * G + g0 + g, __float_as_uint(wv));
    }
  }
  if (a < A) {
    max_iou[(size_t)b * A + a] = ng > 0 ? best : 0.f;
    argmax[(size_t)b * A + a] = bi;
  }
}

// low-quality matches (Faster R-CNN rule): an anchor whose IoU with some gt equals that
// gt's best IoU is matched to it even below the positive threshold
__global__ __launch_bounds__(256) void match_lowq_kernel(const float4* __restrict__ anchors, int A,
                                                         int per_image_anchors, const float4* __restrict__ gt,
                                                         const int* __restrict__ gcount, int G,
                                                         const unsigned int* __restrict__ gt_best,
                                                         int* __restrict__ lowq) {
  const int b = blockIdx.y;
  const int a = blockIdx.x * blockDim.x + threadIdx.x;
  if (a >= A) return;
  const int ng = gcount[b];
  const float4 an = anchors[(per_image_anchors ? (size_t)b * A : 0) + a];
  int hit = -1;
  for (int g = 0; g < ng; ++g) {
    const float gb = __uint_as_float(gt_best[(size_t)b * G + g]);
    if (gb > 0.f && iou4(an, gt[(size_t)b * G + g]) >= gb) { hit = g; }
  }
  lowq[(size_t)b * A + a] = hit;
}

// ------------------------------------------------------------------------------ decode
// boxes = clip(decode(ref, deltas / weights)); dw/dh clamped at log(1000/16)
__global__ __launch_bounds__(256) void decode_clip_kernel(const float4* __restrict__ ref, const float* __restrict__ deltas,
                                                          int N, int per_row_ref, float wx, float wy, float ww, float wh,
                                                          float clamp, const float* __restrict__ img_hw, int rows_per_img,
                                                          float4* __restrict__ out) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= N) return;
  const float4 r = ref[per_row_ref ? i : 0];
  const float* d = deltas + (size_t)i * 4;
  const float w = r.z - r.x, h = r.w - r.y;
  const float cx = r.x + 0.5f * w, cy = r.y + 0.5f * h;
  const float dx = d[0] / wx, dy = d[1] / wy;
  const float dw = fminf(d[2] / ww, clamp), dh = fminf(d[3] / wh, clamp);
  const float pcx = dx * w + cx, pcy = dy * h + cy;
  const float pw = __expf(dw) * w, ph = __expf(dh) * h;
  float4 o = make_float4(pcx - 0.5f * pw, pcy - 0.5f * ph, pcx + 0.5f * pw, pcy + 0.5f * ph);
  if (img_hw) {
    const int im = rows_per_img > 0 ? i / rows_per_img : 0;
    const float H = img_hw[2 * im], W = img_hw[2 * im + 1];
    o.x = fminf(fmaxf(o.x, 0.f), W); o.z = fminf(fmaxf(o.z, 0.f), W);
    o.y = fminf(fmaxf(o.y, 0.f), H); o.w = fminf(fmaxf(o.w, 0.f), H);
  }
  out[i] = o;
}

// mask-head targets: bilinear crop of instance masks (uint8, full image) by RoI boxes to
// M x M (one thread per output pixel; masks are read in place, never replicated per RoI)
__global__ __launch_bounds__(256) void crop_resize_masks_kernel(const uint8_t* __restrict__ masks, int H, int W,
                                                                const float4* __restrict__ boxes,
                                                                const int* __restrict__ gidx, int R, int M,
                                                                float* __restrict__ out) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= R * M * M) return;
  const int r = i / (M * M), py = (i / M) % M, px = i % M;
  const float4 b = boxes[r];
  const uint8_t* m = masks + (size_t)gidx[r] * H * W;
  const float y = b.y + (py + 0.5f) * (b.w - b.y) / M - 0.5f;
  const float x = b.x + (px + 0.5f) * (b.z - b.x) / M - 0.5f;
  float v = 0.f;
  if (!(y < -1.f || y > (float)H || x < -1.f || x > (float)W)) {
    const float yc = fmaxf(y, 0.f), xc = fmaxf(x, 0.f);
    int yl = (int)yc, xl = (int)xc, yh, xh;
    float yy = yc, xx = xc;
    if (yl >= H - 1) { yh = yl = H - 1; yy = (float)yl; } else { yh = yl + 1; }
    if (xl >= W - 1) { xh = xl = W - 1; xx = (float)xl; } else { xh = xl + 1; }
    const float ly = yy - yl, lx = xx - xl;
    v = (1.f - ly) * ((1.f - lx) * m[yl * W + xl] + lx * m[yl * W + xh]) +
        ly * ((1.f - lx) * m[yh * W + xl] + lx * m[yh * W + xh]);
  }
  out[i] = v;
}

// Same targets from packed per-instance crops (data/coco.py mask_crop): table[g] =
// (offset, x0, y0, w, h) of instance g's crop inside `flat`; a mask is zero outside its
// crop, so a bilinear tap outside the crop reads 0 -- identical to the full-image path.
// H, W are the (padded) image dims the full masks would have had (border clamping).
__global__ __launch_bounds__(256) void crop_resize_mask_crops_kernel(const uint8_t* __restrict__ flat,
                                                                     const int* __restrict__ table, int H, int W,
                                                                     const float4* __restrict__ boxes,
                                                                     const int* __restrict__ gidx, int R, int M,
                                                                     float* __restrict__ out) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= R * M * M) return;
  const int r = i / (M * M), py = (i / M) % M, px = i % M;
  const float4 b = boxes[r];
  const int* t = table + 5 * gidx[r];
  const int off = t[0], cx0 = t[1], cy0 = t[2], cw = t[3], ch = t[4];
  const float y = b.y + (py + 0.5f) * (b.w - b.y) / M - 0.5f;
  const float x = b.x + (px + 0.5f) * (b.z - b.x) / M - 0.5f;
  float v = 0.f;
  if (cw > 0 && !(y < -1.f || y > (float)H || x < -1.f || x > (float)W)) {
    const float yc = fmaxf(y, 0.f), xc = fmaxf(x, 0.f);
    int yl = (int)yc, xl = (int)xc, yh, xh;
    float yy = yc, xx = xc;
    if (yl >= H - 1) { yh = yl = H - 1; yy = (float)yl; } else { yh = yl + 1; }
    if (xl >= W - 1) { xh = xl = W - 1; xx = (float)xl; } else { xh = xl + 1; }
    const float ly = yy - yl, lx = xx - xl;
    auto at = [&](int yi, int xi) -> float {
      const int u = yi - cy0, w = xi - cx0;
      return (u >= 0 && u < ch && w >= 0 && w < cw) ? (float)flat[(size_t)off + u * cw + w] : 0.f;
    };
    v = (1.f - ly) * ((1.f - lx) * at(yl, xl) + lx * at(yl, xh)) + ly * ((1.f - lx) * at(yh, xl) + lx * at(yh, xh));
  }
  out[i] = v;
}

Levels make_levels(const void* const* feats, float* const* grads, const int* H, const int* W, const float* scales,
                   int n, int lvl_min, float canon, int canon_lvl) {
  Levels L;
  for (int i = 0; i < 4; ++i) {
    L.f[i] = (feats && i < n) ? (const uint16_t*)feats[i] : nullptr;
    L.g[i] = (grads && i < n) ? grads[i] : nullptr;
    L.H[i] = i < n ? H[i] : 0;
    L.W[i] = i < n ? W[i] : 0;
    L.scale[i] = i < n ? scales[i] : 0.f;
  }
  L.n = n;
  L.lvl_min = lvl_min;
  L.canon = canon;
  L.canon_lvl = canon_lvl;
  return L;
}

}  // namespace

// feats: n (<= 4) NHWC bf16 levels; rois fp32 [R, 5] (batch, x1, y1, x2, y2) in image px.
MX_EXPORT int mx_roi_align_fwd(const void* const* feats, const int* H, const int* W, const float* scales, int n,
                               int lvl_min, float canon, int canon_lvl, const float* rois, int R, int C, int PH,
                               int PW, int sampling, int aligned, void* out, hipStream_t s) {
  if (n < 1 || n > 4 || (C & 7)) return hipErrorInvalidValue;
  if (R == 0) return hipSuccess;
  Levels L = make_levels(feats, nullptr, H, W, scales, n, lvl_min, canon, canon_lvl);
  const long total = (long)R * PH * PW * (C / 8);
  hipLaunchKernelGGL(roi_align_fwd_kernel, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, s, L, rois, R, C, PH,
                     PW, sampling, aligned, (uint16_t*)out);
  return hipGetLastError();
}

// grads: n fp32 NHWC buffers (zeroed by the caller), accumulated with atomics
MX_EXPORT int mx_roi_align_bwd(float* const* grads, const int* H, const int* W, const float* scales, int n, int lvl_min,
                               float canon, int canon_lvl, const float* rois, int R, int C, int PH, int PW,
                               int sampling, int aligned, const void* dout, hipStream_t s) {
  if (n < 1 || n > 4 || (C & 63) || C > 512) return hipErrorInvalidValue;
  if (R == 0) return hipSuccess;
  Levels L = make_levels(nullptr, grads, H, W, scales, n, lvl_min, canon, canon_lvl);
  const long waves = (long)R * PH * PW;
  hipLaunchKernelGGL(roi_align_bwd_kernel, dim3((unsigned)((waves + 3) / 4)), dim3(256), 0, s, L, rois, R, C, PH,
                     PW, sampling, aligned, (const uint16_t*)dout);
  return hipGetLastError();
}

// Tiled, float-atomics-free backward (sr <= 2, C % 64 == 0, C <= 256) writing bf16 NHWC
// gradients directly.  Workspaces (sizes from mx_roi_align_bwd_tiled_ws):
//   ws  int32: FootP items * 12 | counts T | offsets T+1 | cursor T | coff T+1 | poff T+1 |
//              overflow 1 | chunk->tile map (grid) | entries 16 * items  (ny, nx <= 4 distinct tiles per axis: never
//              overflows; the 2 x 2 geometric bound only sizes the launch and partials,
//              and exceeding it sets the overflow word instead of touching memory)
//   partial fp32: pslots * 64 * C   (pslots = ceil(8 * items / kChunk) + 1)
static TileGeo tile_geo(const int* H, const int* W, int n, int B) {
  TileGeo G = {};
  G.B = B;
  int base = 0;
  for (int i = 0; i < n; ++i) {
    G.base[i] = base;
    G.th[i] = (H[i] + kTile - 1) / kTile;
    G.tw[i] = (W[i] + kTile - 1) / kTile;
    base += B * G.th[i] * G.tw[i];
  }
  for (int i = n; i < 5; ++i) G.base[i] = base;
  return G;
}

MX_EXPORT int64_t mx_roi_align_bwd_tiled_ws(const int* H, const int* W, int n, int B, int items, int C,
                                            int64_t* partial_floats) {
  const TileGeo G = tile_geo(H, W, n, B);
  const int64_t T = G.base[n];
  const int64_t pslots = (8 * (int64_t)items + kChunk - 1) / kChunk + 1;
  if (partial_floats) *partial_floats = pslots * kTile * kTile * C;
  const int64_t grid = 2 * T + (4 * (int64_t)items + kChunk - 1) / kChunk;
  return 5 * T + 4 + grid + 16 * (int64_t)items + (int64_t)items * (sizeof(FootP) / 4);
}

static long long* g_tile_dbg = nullptr;
static int g_tile_dmode = 0;
// debugging: per-workgroup timing records of the next tiled backward (4 x int64 per chunk);
// mode bit 0 = skip the gradient loads, bit 1 = skip the LDS accumulation (scalar kernel);
// bit 2 = the scalar per-entry kernel also for C = 256 (A/B against the MFMA kernel)
MX_EXPORT void mx_roi_align_bwd_tiled_debug(long long* buf, int mode) {
  g_tile_dbg = buf;
  g_tile_dmode = mode;
}

MX_EXPORT int mx_roi_align_bwd_tiled(void* const* grads, const int* H, const int* W, const float* scales, int n,
                                     int lvl_min, float canon, int canon_lvl, int B, const float* rois, int R, int C,
                                     int PH, int PW, int sampling, int aligned, const void* dout, int* ws,
                                     float* partial, hipStream_t s) {
  if (n < 1 || n > 4 || (C & 63) || C > kMaxTileC || sampling < 1 || sampling > 2 || B < 1)
    return hipErrorInvalidValue;
  Levels L = make_levels(nullptr, nullptr, H, W, scales, n, lvl_min, canon, canon_lvl);
  const TileGeo G = tile_geo(H, W, n, B);
  const int T = G.base[n];
  const int items = R * PH * PW;
  const int pslots = (int)((8 * (int64_t)items + kChunk - 1) / kChunk + 1);
  FootP* fp = reinterpret_cast<FootP*>(ws);                 // 16-B aligned (caller's buffer)
  int* counts = ws + (size_t)items * (sizeof(FootP) / 4);
  int* offsets = counts + T;
  int* cursor = offsets + T + 1;
  int* coff = cursor + T;
  int* poff = coff + T + 1;
  int* overflow = poff + T + 1;
  // chunks <= T + entries / kChunk + T (rounding) with entries <= 4 items (2 x 2 tiles)
  const int grid = 2 * T + (4 * items + kChunk - 1) / kChunk;
  int* ctile = overflow + 1;
  int* entries = ctile + grid;
  // counts + the overflow word are not contiguous: clear both
  hipError_t e = hipMemsetAsync(counts, 0, sizeof(int) * (size_t)T, s);
  if (e != hipSuccess) return e;
  e = hipMemsetAsync(overflow, 0, sizeof(int), s);
  if (e != hipSuccess) return e;
  if (items > 0)
    hipLaunchKernelGGL(roi_tiles_kernel<true>, dim3((items + 255) / 256), dim3(256), 0, s, L, G, rois, items, PH, PW,
                       sampling, aligned, fp, counts, (int*)nullptr);
  hipLaunchKernelGGL(tile_scan_kernel, dim3(1), dim3(1024), 0, s, counts, T, offsets, cursor, coff, poff, ctile,
                     grid, overflow);
  if (items > 0)
    hipLaunchKernelGGL(roi_tiles_kernel<false>, dim3((items + 255) / 256), dim3(256), 0, s, L, G, rois, items, PH, PW,
                       sampling, aligned, fp, cursor, entries);
  hipLaunchKernelGGL(tile_sort_kernel, dim3(T), dim3(1024), 0, s, offsets, T, entries);
  GOut go = {};
  for (int i = 0; i < n; ++i) go.p[i] = (uint16_t*)grads[i];
  if (C == 256 && !(g_tile_dmode & 4))
    hipLaunchKernelGGL(roi_align_bwd_mfma_kernel, dim3(grid), dim3(256), 0, s, L, G, T, (const uint16_t*)dout, fp,
                       offsets, coff, poff, ctile, entries, go, partial, pslots, overflow, g_tile_dbg);
  else
    hipLaunchKernelGGL(roi_align_bwd_tile_kernel, dim3(grid), dim3(C), 0, s, L, G, T, C, (const uint16_t*)dout, fp,
                       offsets, coff, poff, ctile, entries, go, partial, pslots, overflow, g_tile_dbg,
                       g_tile_dmode);
  hipLaunchKernelGGL(roi_align_bwd_combine_kernel, dim3(T), dim3(256), 0, s, L, G, C, coff, poff, partial, pslots, go);
  return hipGetLastError();
}

// uint64 words of mask_ws per box: the [N][NB] mask and one colmask word
MX_EXPORT int mx_nms_workspace_words(int N) { return (N + 63) / 64 + 1; }

int g_nms_par = 1;   // in-chunk scan: 1 = parallel fixed point (nms_keep_par_kernel), 0 = serial

MX_EXPORT int mx_nms_par(int on) {
  const int old = g_nms_par;
  if (on >= 0) g_nms_par = on;
  return old;
}

// batched NMS over P independent problems (boxes sorted by score desc per problem);
// mask_ws holds P * N * mx_nms_workspace_words(N) uint64
MX_EXPORT int mx_nms(const float* boxes, const int* counts, int P, int N, float thr, int max_out, void* mask_ws,
                     int* keep, int* nkeep, hipStream_t s) {
  const int NB = (N + 63) / 64;
  if (NB > 64) return hipErrorInvalidValue;
  if (P == 0 || N == 0) return hipSuccess;
  unsigned long long* mw = (unsigned long long*)mask_ws;
  unsigned long long* colw = mw + (size_t)P * N * NB;
  hipLaunchKernelGGL(nms_mask_kernel, dim3(NB, NB, P), dim3(64), 0, s, (const float4*)boxes, counts, N, NB, thr,
                     mw, g_nms_par ? colw : (unsigned long long*)nullptr);
  if (g_nms_par) {
    if (NB <= 16)
      hipLaunchKernelGGL(nms_keep_par_kernel<16>, dim3(P), dim3(256), 0, s, mw, colw, counts, N, NB, max_out, keep, nkeep);
    else if (NB <= 32)
      hipLaunchKernelGGL(nms_keep_par_kernel<32>, dim3(P), dim3(256), 0, s, mw, colw, counts, N, NB, max_out, keep, nkeep);
    else
      hipLaunchKernelGGL(nms_keep_par_kernel<64>, dim3(P), dim3(256), 0, s, mw, colw, counts, N, NB, max_out, keep, nkeep);
    return hipGetLastError();
  }
  if (NB <= 16)
    hipLaunchKernelGGL(nms_keep_kernel<16>, dim3(P), dim3(64), 0, s, (const unsigned long long*)mask_ws, counts, N,
                       NB, max_out, keep, nkeep);
  else if (NB <= 32)
    hipLaunchKernelGGL(nms_keep_kernel<32>, dim3(P), dim3(64), 0, s, (const unsigned long long*)mask_ws, counts, N,
                       NB, max_out, keep, nkeep);
  else
    hipLaunchKernelGGL(nms_keep_kernel<64>, dim3(P), dim3(64), 0, s, (const unsigned long long*)mask_ws, counts, N,
                       NB, max_out, keep, nkeep);
  return hipGetLastError();
}

// anchors [A,4] shared by all B images (per_image_anchors=0) or [B,A,4]; gt [B,G,4]
MX_EXPORT int mx_match(const float* anchors, int A, int per_image_anchors, const float* gt, const int* gcount, int B,
                       int G, float* max_iou, int* argmax, unsigned int* gt_best, int* lowq, hipStream_t s) {
  if (A == 0 || B == 0) return hipSuccess;
  hipMemsetAsync(gt_best, 0, sizeof(unsigned int) * (size_t)B * (G > 0 ? G : 1), s);
  dim3 grid((A + 255) / 256, B);
  hipLaunchKernelGGL(match_kernel, grid, dim3(256), 0, s, (const float4*)anchors, A, per_image_anchors,
                     (const float4*)gt, gcount, G, max_iou, argmax, gt_best);
  if (lowq)
    hipLaunchKernelGGL(match_lowq_kernel, grid, dim3(256), 0, s, (const float4*)anchors, A, per_image_anchors,
                       (const float4*)gt, gcount, G, (const unsigned int*)gt_best, lowq);
  return hipGetLastError();
}

// Rows of an NHWC level into its place on a canvas (RPN level canvas, models/maskrcnn.py):
// src [B][h][w*C] contiguous -> dst[(n * Hc + y0 + y) * pitch + x0 * C ...], 16-B vectors
// (a strided-view copy_ ran PyTorch's non-vectorised elementwise kernel).  row_elems and
// pitch multiples of 8, pointers 16-B aligned.
__global__ __launch_bounds__(256) void copy_rows_kernel(uint16_t* __restrict__ dst, const uint16_t* __restrict__ src,
                                                        int h, int row_vec, int Hc, int64_t pitch, int64_t dst_off,
                                                        int64_t nvec) {
  for (int64_t v = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; v < nvec; v += (int64_t)gridDim.x * blockDim.x) {
    const int64_t r = v / row_vec;
    const int c = (int)(v - r * row_vec);
    const int n = (int)(r / h), y = (int)(r - (int64_t)n * h);
    reinterpret_cast<uint4*>(dst + dst_off + ((int64_t)n * Hc + y) * pitch)[c] =
        reinterpret_cast<const uint4*>(src)[v];
  }
}

MX_EXPORT int mx_copy_rows(void* dst, const void* src, int B, int h, int row_elems, int Hc, int64_t pitch,
                           int64_t dst_off, hipStream_t s) {
  if ((row_elems & 7) || (pitch & 7) || (dst_off & 7) || (((uintptr_t)dst | (uintptr_t)src) & 15))
    return hipErrorInvalidValue;
  const int64_t nvec = (int64_t)B * h * (row_elems / 8);
  if (nvec == 0) return hipSuccess;
  const int64_t want = (nvec + 255) / 256;
  hipLaunchKernelGGL(copy_rows_kernel, dim3((unsigned)(want < 16384 ? want : 16384)), dim3(256), 0, s,
                     (uint16_t*)dst, (const uint16_t*)src, h, row_elems / 8, Hc, pitch, dst_off, nvec);
  return hipGetLastError();
}

// Input normalisation in one pass: uint8 images [N][3][H][W] -> bf16 NHWC [N][H][W][3] of
// (x - mean[c]) * inv_std[c] (the float / subtract / divide / bf16 / channels_last chain was
// five passes over a fp32 copy).  Four pixels per thread (HW % 4 == 0).
__global__ __launch_bounds__(256) void normalize_u8_nhwc_kernel(const uint8_t* __restrict__ src,
                                                                uint16_t* __restrict__ dst, int64_t HW,
                                                                int64_t nquad, float m0, float m1, float m2,
                                                                float s0, float s1, float s2) {
  for (int64_t v = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; v < nquad; v += (int64_t)gridDim.x * blockDim.x) {
    const int64_t px = 4 * v, n = px / HW, q = px - n * HW;
    const uint8_t* b = src + n * 3 * HW + q;
    const uchar4 c0 = *reinterpret_cast<const uchar4*>(b);
    const uchar4 c1 = *reinterpret_cast<const uchar4*>(b + HW);
    const uchar4 c2 = *reinterpret_cast<const uchar4*>(b + 2 * HW);
    const float r[4] = {(float)c0.x, (float)c0.y, (float)c0.z, (float)c0.w};
    const float g[4] = {(float)c1.x, (float)c1.y, (float)c1.z, (float)c1.w};
    const float bl[4] = {(float)c2.x, (float)c2.y, (float)c2.z, (float)c2.w};
    uint16_t o[12];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      o[3 * k] = f2bf((r[k] - m0) * s0);
      o[3 * k + 1] = f2bf((g[k] - m1) * s1);
      o[3 * k + 2] = f2bf((bl[k] - m2) * s2);
    }
    uint2* d = reinterpret_cast<uint2*>(dst + 3 * px);   // 24 B, 8-B aligned
#pragma unroll
    for (int k = 0; k < 3; ++k)
      d[k] = make_uint2((uint32_t)o[4 * k] | ((uint32_t)o[4 * k + 1] << 16),
                        (uint32_t)o[4 * k + 2] | ((uint32_t)o[4 * k + 3] << 16));
  }
}

MX_EXPORT int mx_normalize_u8_nhwc(const void* src, void* dst, int N, int H, int W, const float* mean,
                                   const float* inv_std, hipStream_t s) {
  const int64_t HW = (int64_t)H * W;
  if (HW % 4 || (((uintptr_t)src) & 3) || (((uintptr_t)dst) & 7)) return hipErrorInvalidValue;
  const int64_t nquad = (int64_t)N * HW / 4;
  if (nquad == 0) return hipSuccess;
  const int64_t want = (nquad + 255) / 256;
  hipLaunchKernelGGL(normalize_u8_nhwc_kernel, dim3((unsigned)(want < 16384 ? want : 16384)), dim3(256), 0, s,
                     (const uint8_t*)src, (uint16_t*)dst, HW, nquad, mean[0], mean[1], mean[2], inv_std[0],
                     inv_std[1], inv_std[2]);
  return hipGetLastError();
}

MX_EXPORT int mx_decode_clip(const float* ref, const float* deltas, int N, int per_row_ref, float wx, float wy,
                             float ww, float wh, float clamp, const float* img_hw, int rows_per_img, float* out,
                             hipStream_t s) {
  if (N == 0) return hipSuccess;
  hipLaunchKernelGGL(decode_clip_kernel, dim3((N + 255) / 256), dim3(256), 0, s, (const float4*)ref, deltas, N,
                     per_row_ref, wx, wy, ww, wh, clamp, img_hw, rows_per_img, (float4*)out);
  return hipGetLastError();
}

// masks uint8 [G, H, W] (0/1), boxes fp32 [R, 4], gidx int32 [R] -> out fp32 [R, M, M]
MX_EXPORT int mx_crop_resize_masks(const void* masks, int H, int W, const float* boxes, const int* gidx, int R, int M,
                                   float* out, hipStream_t s) {
  if (R == 0) return hipSuccess;
  const int total = R * M * M;
  hipLaunchKernelGGL(crop_resize_masks_kernel, dim3((total + 255) / 256), dim3(256), 0, s, (const uint8_t*)masks, H, W,
                     (const float4*)boxes, gidx, R, M, out);
  return hipGetLastError();
}

// flat uint8 crops, table int32 [G_total, 5], boxes fp32 [R, 4], gidx int32 [R] -> out fp32 [R, M, M]
MX_EXPORT int mx_crop_resize_mask_crops(const void* flat, const int* table, int H, int W, const float* boxes,
                                        const int* gidx, int R, int M, float* out, hipStream_t s) {
  if (R == 0) return hipSuccess;
  const int total = R * M * M;
  hipLaunchKernelGGL(crop_resize_mask_crops_kernel, dim3((total + 255) / 256), dim3(256), 0, s,
                     (const uint8_t*)flat, table, H, W, (const float4*)boxes, gidx, R, M, out);
  return hipGetLastError();
}

// RPN level top-k + decode (see tk_* above).  rows: R x 6 int64 on the device; c0: R + 1
// chunk offsets (device); nchunks = c0[R]; K <= 2048; hist1 / hist2: R x 256 int32, zero
// before the first call (the last kernel re-zeroes them); bcnt: nchunks int2; cand: R x
// 2048 uint2; outputs boxes [R][K] float4, scores [R][K].
MX_EXPORT int mx_topk_chunk() { return kTkChunk; }

// x [R][ld] fp32 (n valid columns) -> the k largest (largest = 1) or smallest values per
// row, sorted, ties by lower index: ov [R][k] fp32, oi [R][k] int64.  1 <= k <= min(n, 2048).
MX_EXPORT int mx_topk_rows(const float* x, int R, int n, int ld, int k, int largest, float* ov, int64_t* oi,
                           hipStream_t s) {
  if (R <= 0 || k <= 0 || k > n || k > kTkrMaxK || ld < n || n >= (1 << 30)) return (int)hipErrorInvalidValue;
  hipLaunchKernelGGL(topk_rows_kernel, dim3(R), dim3(1024), 0, s, x, n, ld, k, largest, ov, oi, 0, 0,
                     (const int64_t*)nullptr);
  return hipGetLastError();
}
// Long rows in two launches (ops/vision.py topk_rows): the k best of each of nc chunks of c
// columns of every row (row-global indices, ragged last chunk read in place -- no padded
// copy), then the k best of the R x (nc k) candidates with their original indices (no
// index arithmetic / gather launches in between).  cand_v / cand_i: R * nc * k scratch.
MX_EXPORT int mx_topk_rows_long(const float* x, int R, int n, int ld, int nc, int c, int k, int largest,
                                float* cand_v, int64_t* cand_i, float* ov, int64_t* oi, hipStream_t s) {
  if (R <= 0 || k <= 0 || k > kTkrMaxK || nc < 1 || c < k || (int64_t)nc * c < n || n - (nc - 1) * c < k ||
      (int64_t)nc * k > (1 << 30) || ld < n)
    return (int)hipErrorInvalidValue;
  hipLaunchKernelGGL(topk_rows_kernel, dim3(R * nc), dim3(1024), 0, s, x, c, ld, k, largest, cand_v, cand_i, nc, n,
                     (const int64_t*)nullptr);
  hipLaunchKernelGGL(topk_rows_kernel, dim3(R), dim3(1024), 0, s, (const float*)cand_v, nc * k, nc * k, k, largest,
                     ov, oi, 0, 0, (const int64_t*)cand_i);
  return hipGetLastError();
}
MX_EXPORT int mx_topk_rows_max_k() { return kTkrMaxK; }
// host_rows: R x 6 int64 {logits, deltas, anchors, n, image, 0}; tables: device scratch of
// kTkMaxRows * 6 int64 followed by kTkMaxRows + 1 int32
MX_EXPORT int mx_topk_max_rows() { return kTkMaxRows; }
MX_EXPORT int mx_level_topk_decode(const int64_t* host_rows, int R, int K, const float* img_hw, float clamp,
                                   void* tables, int* hist1, int* hist2, void* bcnt, int bcnt_cap, void* cand,
                                   float* boxes, float* scores, hipStream_t s) {
  if (K <= 0 || K > kTkMaxK || R <= 0 || R > kTkMaxRows) return hipErrorInvalidValue;
  TkArgs a{};
  int nchunks = 0;
  for (int r = 0; r < R; ++r) {
    for (int j = 0; j < 6; ++j) a.rows[6 * r + j] = host_rows[6 * r + j];
    a.c0[r] = nchunks;
    nchunks += (int)((host_rows[6 * r + 3] + kTkChunk - 1) / kTkChunk);
  }
  for (int r = R; r <= kTkMaxRows; ++r) a.c0[r] = nchunks;
  if (nchunks > bcnt_cap) return hipErrorInvalidValue;
  int64_t* rows = reinterpret_cast<int64_t*>(tables);
  int* c0 = reinterpret_cast<int*>(rows + kTkMaxRows * 6);
  hipLaunchKernelGGL(tk_setup_kernel, dim3(1), dim3(64), 0, s, a, rows, c0);
  if (nchunks > 0) {
    hipLaunchKernelGGL(tk_hist_kernel, dim3(nchunks), dim3(256), 0, s, rows, c0, R, K, hist1, hist2, 0);
    hipLaunchKernelGGL(tk_hist_kernel, dim3(nchunks), dim3(256), 0, s, rows, c0, R, K, hist1, hist2, 1);
    hipLaunchKernelGGL(tk_count_kernel, dim3(nchunks), dim3(256), 0, s, rows, c0, R, K, hist1, hist2, (int2*)bcnt);
    hipLaunchKernelGGL(tk_compact_kernel, dim3(nchunks), dim3(256), 0, s, rows, c0, R, K, hist1, hist2,
                       (const int2*)bcnt, (uint2*)cand);
  }
  hipLaunchKernelGGL(tk_sort_decode_kernel, dim3(R), dim3(1024), 0, s, rows, K, (const uint2*)cand, img_hw, clamp,
                     (float4*)boxes, scores, hist1, hist2);
  return hipGetLastError();
}

// ks [B][L][pre]: per (image, list) scores sorted non-increasing; out [B][top] values and
// flat indices (l * pre + j), ordered as topk_rows(ks.view(B, L * pre), top).  L * pre <= 16384.
// keep int32 [B * L][pre], scores fp32 [B * L][pre], boxes fp32 [B * L][pre][4] -> ov [B][top],
// ob [B][top][4] (merge_keep_topk_kernel)
MX_EXPORT int mx_merge_keep_topk(const int* keep, const float* scores, const void* boxes, int B, int L, int pre,
                                 int top, float* ov, void* ob, hipStream_t s) {
  const int n = L * pre;
  if (B <= 0 || n <= 0) return hipSuccess;
  if (n > kMergeMax || top > n || (((uintptr_t)boxes | (uintptr_t)ob) & 15)) return hipErrorInvalidValue;
  hipLaunchKernelGGL(merge_keep_topk_kernel, dim3((n + 255) / 256, B), dim3(256), 0, s, keep, scores,
                     (const float4*)boxes, L, pre, top, ov, (float4*)ob);
  return hipGetLastError();
}

MX_EXPORT int mx_merge_sorted_topk(const float* ks, int B, int L, int pre, int top, float* ov, int64_t* oi,
                                   hipStream_t s) {
  const int n = L * pre;
  if (B <= 0 || n <= 0) return hipSuccess;
  if (n > kMergeMax || top > n) return hipErrorInvalidValue;
  hipLaunchKernelGGL(merge_topk_kernel, dim3((n + 255) / 256, B), dim3(256), 0, s, ks, L, pre, top, ov, oi);
  return hipGetLastError();
}
