// Fused ResNet stem for a frozen backbone (Mask R-CNN, tensorpack FREEZE_AT=2):
//   uint8 NCHW image -> (x - mean) / std -> conv 7x7 stride 2 pad 3 (3 -> 64, FrozenBN folded:
//   bias) -> ReLU -> max-pool 3x3 stride 2 pad 1 -> bf16 NHWC [N][PH][PW][64]
// in ONE launch.  Replaces the input-normalisation pass, MIOpen's stem convolution (an
// igemm_fwd_gtcx35 solver, 42 us at one 800x1333 image, 120 us at four: ~170 TFLOP/s on a
// 3-channel reduction) and torch's NHWC max-pool (35 / 90 us), and never writes the
// full-resolution stem activation (137 MB at four images) to memory.  Reference: the
// tensorpack ResNet-FPN backbone's conv0 + pool0 (examples/maskrcnn).
//
// Design (gfx950):
//  * one workgroup (4 waves) = a 15 x 17 block of stem pixels = the 7 x 8 pooled outputs that
//    block covers (pool windows overlap by one stem row / column: 1.14x recompute);
//  * the reduction K = 3 channels x 8 kernel rows x 8 kernel columns (row 7 and column 7 zero
//    weights) = 192 = six 32-deep MFMA steps.  For a fixed output pixel the 7 taps of one
//    kernel row are 7 consecutive input bytes, so a lane's MFMA fragment (pixel i, K
//    8G .. 8G + 7) is ONE unaligned 8-byte window of one channel plane: three aligned dword
//    loads + two v_alignbyte, normalised in registers (no im2col, no LDS for A);
//  * the packed weights [64][192] (24 KiB) are held in VGPRs for the whole launch (each wave
//    covers all 64 output channels: 4 x 6 fragments), the weight fragment is the MFMA A
//    operand, so a lane ends with 4 consecutive channels of one pixel;
//  * bias + ReLU, bf16 into an LDS tile [255 px][72] (144-B rows: 16-B aligned, conflict-light),
//    then each thread max-pools one pooled pixel x 8 channels (ReLU outputs are >= 0, so a
//    zero for stem pixels outside the image is the -inf padding of torch's max_pool2d).
#include "gemm_common.h"

using namespace mx;
using namespace mx::gemm;

namespace {

constexpr int kPH = 7, kPW = 8;                      // pooled outputs per workgroup
constexpr int kSH = 2 * kPH + 1, kSW = 2 * kPW + 1;  // stem pixels per workgroup (15 x 17 = 255)
constexpr int kLdsRow = 72;                          // bf16 per LDS pixel row (64 + 8 pad)
constexpr int g_stem_grid = 512;                     // persistent workgroups (two per CU)

struct StemArgs {
  const uint8_t* img;     // [N][3][H][W]
  const uint16_t* w;      // [64][192] bf16, K = (c, kh 0..7, kw 0..7), row / column 7 zero
  const uint16_t* bias;   // [64] bf16
  uint16_t* y;            // [N][PH][PW][64] bf16
  int H, W, OH, OW, PH, PW;
  int tiles_x, tiles_per_img, tiles_total;
  int64_t total;          // bytes of the image batch
  int64_t last_dw;        // highest dword-aligned base whose 12-byte window stays in the batch
  float mean[3], istd[3];
};

__global__ __launch_bounds__(256, 2) void stem_pool_kernel(const StemArgs a) {
  __shared__ __attribute__((aligned(16))) uint16_t tile[256 * kLdsRow];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int G = lane >> 4, i = lane & 15;

  // packed weights [64][192] bf16 -> LDS (24 KiB; 96 B per thread), read back per MFMA:
  // holding them in VGPRs (96 per lane) left room for only a few image loads in flight
  __shared__ __attribute__((aligned(16))) uint16_t wl[64 * 192];
#pragma unroll
  for (int j = 0; j < 6; ++j) {
    const int e = (j * 256 + tid) * 8;
    *reinterpret_cast<uint4*>(wl + e) = *reinterpret_cast<const uint4*>(a.w + e);
  }

  bool first = true;
  // persistent: a workgroup walks tiles (the 24 KiB weight load once per workgroup, not per tile)
  for (int tile_id = blockIdx.x; tile_id < a.tiles_total; tile_id += gridDim.x) {
  const int n = tile_id / a.tiles_per_img, t = tile_id - n * a.tiles_per_img;
  const int py0 = (t / a.tiles_x) * kPH, px0 = (t % a.tiles_x) * kPW;
  const int sy0 = 2 * py0 - 1, sx0 = 2 * px0 - 1;   // stem coordinates of tile pixel (0, 0)
  // this lane's 4 stem pixels (one per 16-pixel group a): tile index q = 64 wave + 16 a + i
  int sy[4], sx[4];
  bool ok[4];
#pragma unroll
  for (int g = 0; g < 4; ++g) {
    const int q = 64 * wave + 16 * g + i;
    const int r = q / kSW, c = q - (q / kSW) * kSW;
    sy[g] = sy0 + r;
    sx[g] = sx0 + c;
    ok[g] = q < kSH * kSW && (unsigned)sy[g] < (unsigned)a.OH && (unsigned)sx[g] < (unsigned)a.OW;
  }
  const int64_t plane = (int64_t)a.H * a.W;
  const int64_t img0 = (int64_t)n * 3 * plane;   // this image's first byte in the batch

  // every image window of the launch first (24 x 12 B per lane in flight at once), then
  // the math: the three aligned dwords around each 8-byte window, the base clamped into
  // the batch (its byte offset sh is 0..3 except at the batch's first / last bytes)
  uint32_t dw[6][4][3];
  uint32_t rowok = 0u;   // bit 4 ks + g: the window's row lies in the image (and the pixel exists)
#pragma unroll
  for (int ks = 0; ks < 6; ++ks) {
    const int c = ks >> 1, kh = (ks & 1) * 4 + G;
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      const int iy = 2 * sy[g] - 3 + kh, ix0 = 2 * sx[g] - 3;
      const bool rok = ok[g] && kh < 7 && (unsigned)iy < (unsigned)a.H;
      rowok |= rok ? 1u << (4 * ks + g) : 0u;
      const int64_t off = img0 + (int64_t)c * plane + (int64_t)(rok ? iy : 0) * a.W + ix0;
      int64_t base = off & ~(int64_t)3;
      base = base < 0 ? 0 : (base > a.last_dw ? a.last_dw : base);
      const uint32_t* p = reinterpret_cast<const uint32_t*>(a.img + base);
      dw[ks][g][0] = p[0];
      dw[ks][g][1] = p[1];
      dw[ks][g][2] = p[2];
    }
  }
  if (first) __syncthreads();   // the weights are in LDS
  first = false;

  f32x4 acc[4][4];
#pragma unroll
  for (int g = 0; g < 4; ++g)
#pragma unroll
    for (int u = 0; u < 4; ++u) acc[g][u] = f32x4{0.f, 0.f, 0.f, 0.f};

#pragma unroll
  for (int ks = 0; ks < 6; ++ks) {
    const int c = ks >> 1;
    const float mu = a.mean[c], is = a.istd[c];
    bf16x8 wf[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) wf[u] = *reinterpret_cast<const bf16x8*>(wl + (16 * u + i) * 192 + 32 * ks + 8 * G);
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      const uint32_t d0 = dw[ks][g][0], d1 = dw[ks][g][1], d2 = dw[ks][g][2];
      const int ix0 = 2 * sx[g] - 3;
      const bool rok = (rowok >> (4 * ks + g)) & 1u;
      // the window's byte offset from its clamped base (recomputed: an array of them spilled)
      const int iy = 2 * sy[g] - 3 + (ks & 1) * 4 + G;
      const int64_t off = img0 + (int64_t)c * plane + (int64_t)(rok ? iy : 0) * a.W + ix0;
      int64_t base = off & ~(int64_t)3;
      base = base < 0 ? 0 : (base > a.last_dw ? a.last_dw : base);
      const int sh = (int)(off - base);   // -3 .. 11
      // (selects, not branches: every variant is a couple of VALU ops)
      const int s4 = sh & 3;
      const uint32_t a01 = __builtin_amdgcn_alignbyte(d1, d0, s4), a12 = __builtin_amdgcn_alignbyte(d2, d1, s4);
      const uint32_t a2z = __builtin_amdgcn_alignbyte(0u, d2, s4);
      const uint32_t neg_lo = d0 << ((8 * -sh) & 31), neg_hi = __builtin_amdgcn_alignbyte(d1, d0, (4 + sh) & 3);
      const uint32_t lo = sh < 0 ? neg_lo : (sh < 4 ? a01 : (sh < 8 ? a12 : a2z));
      const uint32_t hi = sh < 0 ? neg_hi : (sh < 4 ? a12 : (sh < 8 ? a2z : 0u));
      float v[8];
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        // (masked with an AND: a select here was compiled into per-element branches)
        const uint32_t m = rok && (unsigned)(ix0 + k) < (unsigned)a.W ? ~0u : 0u;
        const float b = (float)(((k < 4 ? lo : hi) >> (8 * (k & 3))) & 0xffu);
        v[k] = __uint_as_float(__float_as_uint((b - mu) * is) & m);
      }
      if (__builtin_expect(sh >= 4 && rok, 0)) {
        // the batch's last bytes: the clamped window can end up to 3 bytes short of them
        // (the batch size need not be a multiple of 4); byte loads, taken by a lane or two
#pragma unroll
        for (int k = 0; k < 8; ++k) {
          const bool in = (unsigned)(ix0 + k) < (unsigned)a.W;
          v[k] = in ? ((float)a.img[in ? off + k : off] - mu) * is : 0.f;
        }
      }
      bf16x8 xf;
      uint32_t* xw = reinterpret_cast<uint32_t*>(&xf);
      xw[0] = pack2(v[0], v[1]);
      xw[1] = pack2(v[2], v[3]);
      xw[2] = pack2(v[4], v[5]);
      xw[3] = pack2(v[6], v[7]);
#pragma unroll
      for (int u = 0; u < 4; ++u) acc[g][u] = mfma16(wf[u], xf, acc[g][u]);
    }
  }

  // bias + ReLU -> LDS tile (pixel q, channels 16 u + 4 G .. + 3); stem pixels outside the
  // image store zeros (the pool's padding)
  float bv[4][4];
#pragma unroll
  for (int u = 0; u < 4; ++u) {
    const uint2 b2 = *reinterpret_cast<const uint2*>(a.bias + 16 * u + 4 * G);
    bv[u][0] = lo_bf(b2.x); bv[u][1] = hi_bf(b2.x); bv[u][2] = lo_bf(b2.y); bv[u][3] = hi_bf(b2.y);
  }
#pragma unroll
  for (int g = 0; g < 4; ++g) {
    const int q = 64 * wave + 16 * g + i;
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      float o[4];
#pragma unroll
      for (int e = 0; e < 4; ++e) o[e] = ok[g] ? fmaxf(acc[g][u][e] + bv[u][e], 0.f) : 0.f;
      *reinterpret_cast<uint2*>(tile + q * kLdsRow + 16 * u + 4 * G) = make_uint2(pack2(o[0], o[1]), pack2(o[2], o[3]));
    }
  }
  __syncthreads();

  // 3 x 3 stride-2 max-pool from the tile: item = (pooled pixel, 8-channel chunk)
  for (int it = tid; it < kPH * kPW * 8; it += 256) {
    const int pp = it >> 3, ch = (it & 7) * 8;
    const int pr = pp / kPW, pc = pp - (pp / kPW) * kPW;
    const int py = py0 + pr, px = px0 + pc;
    if (py >= a.PH || px >= a.PW) continue;
    float m[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int dy = 0; dy < 3; ++dy)
#pragma unroll
      for (int dx = 0; dx < 3; ++dx) {
        const int q = (2 * pr + dy) * kSW + 2 * pc + dx;
        float f[8];
        unpack8(*reinterpret_cast<const uint4*>(tile + q * kLdsRow + ch), f);
#pragma unroll
        for (int k = 0; k < 8; ++k) m[k] = fmaxf(m[k], f[k]);
      }
    *reinterpret_cast<uint4*>(a.y + (((size_t)n * a.PH + py) * a.PW + px) * 64 + ch) = pack8(m);
  }
  __syncthreads();   // the pool's LDS reads finish before the next tile's writes
  }
}

}  // namespace

// img uint8 [N][3][H][W]; w packed bf16 [64][192] (mx_stem_pack layout, see stem.py); bias bf16 [64];
// y bf16 [N][PH][PW][64] with OH = (H - 1) / 2 + 1, PH = (OH - 1) / 2 + 1 (likewise W).
MX_EXPORT int mx_stem_pool(const void* img, const void* w, const void* bias, void* y, int N, int H, int W,
                           const float* mean, const float* inv_std, void* stream) {
  if (N <= 0 || H < 2 || W < 2 || (((uintptr_t)w | (uintptr_t)y) & 15) || ((uintptr_t)bias & 7)) return (int)hipErrorInvalidValue;
  if ((int64_t)3 * H * W < 16) return (int)hipErrorInvalidValue;
  StemArgs a{};
  a.img = (const uint8_t*)img;
  a.w = (const uint16_t*)w;
  a.bias = (const uint16_t*)bias;
  a.y = (uint16_t*)y;
  a.H = H;
  a.W = W;
  a.OH = (H - 1) / 2 + 1;
  a.OW = (W - 1) / 2 + 1;
  a.PH = (a.OH - 1) / 2 + 1;
  a.PW = (a.OW - 1) / 2 + 1;
  a.tiles_x = (a.PW + kPW - 1) / kPW;
  a.tiles_per_img = ((a.PH + kPH - 1) / kPH) * a.tiles_x;
  a.total = (int64_t)N * 3 * H * W;
  a.last_dw = (a.total - 12) & ~(int64_t)3;
  for (int c = 0; c < 3; ++c) {
    a.mean[c] = mean[c];
    a.istd[c] = inv_std[c];
  }
  const int64_t blocks = (int64_t)N * a.tiles_per_img;
  if (blocks >= ((int64_t)1 << 31)) return (int)hipErrorInvalidValue;
  a.tiles_total = (int)blocks;
  const int grid = blocks < g_stem_grid ? (int)blocks : g_stem_grid;
  hipLaunchKernelGGL(stem_pool_kernel, dim3((unsigned)grid), dim3(256), 0, (hipStream_t)stream, a);
  return (int)hipGetLastError();
}

