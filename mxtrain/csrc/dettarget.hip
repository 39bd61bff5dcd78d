// Mask R-CNN training targets without the PyTorch glue: the RPN anchor labelling / sampling
// keys / box-regression targets and the Fast R-CNN RoI sampling, each a handful of launches
// instead of ~40 elementwise / gather / scatter / cat kernels (profiles/r5_s1/
// maskrcnn_4img_op_census.txt; at one image per GPU those small launches and the gaps
// between them were ~2 ms of the 8.6 ms step).  Same math as the PyTorch definitions in
// models/maskrcnn.py (rpn_targets / sample_rois, kept as the CPU path and the test
// reference) and ops/vision.py encode_boxes; the random keys still come from torch.rand, so
// the sampling draws are the same numbers.
// Reference: tensorpack examples/FasterRCNN (the reference's TRAINER=horovod Mask R-CNN,
// examples/maskrcnn/train-maskrcnn-tensorpack.yaml): RPN anchor targets, 256 anchors / 512
// RoIs per image, fg ratio 0.5 / 0.25.
#include "common.h"

using namespace mx;

namespace {

// box regression target of gt g w.r.t. reference box r (encode_boxes)
__device__ __forceinline__ float4 encode1(float4 r, float4 g, float wx, float wy, float ww, float wh) {
  const float rw = fmaxf(r.z - r.x, 1e-6f), rh = fmaxf(r.w - r.y, 1e-6f);
  const float rcx = r.x + 0.5f * rw, rcy = r.y + 0.5f * rh;
  const float gw = fmaxf(g.z - g.x, 1e-6f), gh = fmaxf(g.w - g.y, 1e-6f);
  const float gcx = g.x + 0.5f * gw, gcy = g.y + 0.5f * gh;
  return make_float4(wx * (gcx - rcx) / rw, wy * (gcy - rcy) / rh, ww * logf(gw / rw), wh * logf(gh / rh));
}

__global__ __launch_bounds__(256) void encode_kernel(const float4* __restrict__ ref, int ref_bcast,
                                                     const float4* __restrict__ gt, int n, float wx, float wy,
                                                     float ww, float wh, float4* __restrict__ out) {
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i < n) out[i] = encode1(ref[ref_bcast ? 0 : i], gt[i], wx, wy, ww, wh);
}

// RPN, per (image b, anchor a):
//   inside = anchor within the image; pos = (iou >= fg | low-quality match) & inside;
//   neg = iou < bg & !pos & inside;  kpos / kneg = the random key for eligible anchors, 2
//   otherwise (the rank-select keys); enc = encode(anchor, gt[matched]) with matched =
//   max(lq >= 0 ? lq : argmax, 0); sel_pos / sel_neg zeroed for rpn_select_kernel.
__global__ __launch_bounds__(256) void rpn_keys_kernel(const float4* __restrict__ anchors, int A,
                                                       const float* __restrict__ mi, const int* __restrict__ am,
                                                       const int* __restrict__ lq, const float* __restrict__ img_hw,
                                                       const float* __restrict__ rnd, const float4* __restrict__ gt,
                                                       int G, float fg_thr, float bg_thr, float* __restrict__ kpos,
                                                       float* __restrict__ kneg, float4* __restrict__ enc,
                                                       uint8_t* __restrict__ sel_pos, uint8_t* __restrict__ sel_neg) {
  const int a = blockIdx.x * 256 + threadIdx.x, b = blockIdx.y;
  if (a >= A) return;
  const size_t i = (size_t)b * A + a;
  const float4 an = anchors[a];
  const float H = img_hw[2 * b], W = img_hw[2 * b + 1];
  const bool inside = an.x >= 0.f && an.y >= 0.f && an.z <= W && an.w <= H;
  const int l = lq[i];
  const float m = mi[i];
  const bool pos = (m >= fg_thr || l >= 0) && inside;
  const bool neg = m < bg_thr && !pos && inside;
  const float r = rnd[i];
  kpos[i] = pos ? r : 2.f;
  kneg[i] = neg ? r : 2.f;
  const int g = max(l >= 0 ? l : am[i], 0);
  enc[i] = encode1(an, gt[(size_t)b * G + min(g, G - 1)], 1.f, 1.f, 1.f, 1.f);
  sel_pos[i] = 0;
  sel_neg[i] = 0;
}

// One workgroup per image: the positives are the (at most kp) smallest kpos keys below 2,
// the negatives the smallest kneg keys below 2, at most batch - #positives of them
// (_rank_select twice, the second one's quota from the first's count).
__global__ __launch_bounds__(256) void rpn_select_kernel(const float* __restrict__ vpos, const int64_t* __restrict__ ipos,
                                                         int kp, const float* __restrict__ vneg,
                                                         const int64_t* __restrict__ ineg, int kn, int ld, int batch,
                                                         int A, uint8_t* __restrict__ sel_pos,
                                                         uint8_t* __restrict__ sel_neg) {
  __shared__ int cnt;
  const int b = blockIdx.x, t = threadIdx.x;
  if (t == 0) cnt = 0;
  __syncthreads();
  int mine = 0;
  for (int r = t; r < kp; r += 256) {
    if (vpos[(size_t)b * ld + r] < 2.f) {
      sel_pos[(size_t)b * A + ipos[(size_t)b * ld + r]] = 1;
      ++mine;
    }
  }
  if (mine) atomicAdd(&cnt, mine);
  __syncthreads();
  const int want = batch - cnt;
  for (int r = t; r < kn && r < want; r += 256)
    if (vneg[(size_t)b * ld + r] < 2.f) sel_neg[(size_t)b * A + ineg[(size_t)b * ld + r]] = 1;
}

// Fast R-CNN RoI sampling, candidates = K proposals + G gt boxes per image (gt rows past
// gt_count far away at -1e4, invalid); one thread per (image, candidate).
__global__ __launch_bounds__(256) void roi_cand_kernel(const float4* __restrict__ props, int K,
                                                       const float4* __restrict__ gt, const int* __restrict__ gcount,
                                                       int G, float4* __restrict__ cand, uint8_t* __restrict__ cvalid) {
  const int j = blockIdx.x * 256 + threadIdx.x, b = blockIdx.y;
  if (j >= K + G) return;
  const size_t o = (size_t)b * (K + G) + j;
  if (j < K) {
    cand[o] = props[(size_t)b * K + j];
    cvalid[o] = 1;
  } else {
    const bool ok = j - K < gcount[b];
    cand[o] = ok ? gt[(size_t)b * G + (j - K)] : make_float4(-1e4f, -1e4f, -1e4f, -1e4f);
    cvalid[o] = ok ? 1 : 0;
  }
}

// fg keys: random key of a valid candidate with iou >= fg, 2 otherwise
__global__ __launch_bounds__(256) void roi_fgkey_kernel(const float* __restrict__ mi, const uint8_t* __restrict__ cvalid,
                                                        const float* __restrict__ rnd, int n, float fg_thr,
                                                        float* __restrict__ key) {
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i < n) key[i] = (mi[i] >= fg_thr && cvalid[i]) ? rnd[i] : 2.f;
}

// One workgroup per image: the selected fg candidates (the kf smallest fg keys below 2),
// then the ordering key 2 + r (selected fg) / 1 + r (valid bg) / 0 of every candidate.
__global__ __launch_bounds__(256) void roi_order_kernel(const float* __restrict__ vfg, const int64_t* __restrict__ ifg,
                                                        int kf, const float* __restrict__ mi,
                                                        const uint8_t* __restrict__ cvalid, const float* __restrict__ rnd,
                                                        int C, float fg_thr, uint8_t* __restrict__ sel_fg,
                                                        float* __restrict__ key) {
  const int b = blockIdx.x, t = threadIdx.x;
  const size_t o = (size_t)b * C;
  for (int j = t; j < C; j += 256) sel_fg[o + j] = 0;
  __syncthreads();
  for (int r = t; r < kf; r += 256)
    if (vfg[(size_t)b * kf + r] < 2.f) sel_fg[o + ifg[(size_t)b * kf + r]] = 1;
  __syncthreads();
  for (int j = t; j < C; j += 256) {
    const float r = rnd[o + j];
    key[o + j] = sel_fg[o + j] ? 2.f + r : ((mi[o + j] < fg_thr && cvalid[o + j]) ? 1.f + r : 0.f);
  }
}

// per (image, sampled slot n): the RoI, its fg flag, matched gt, label, regression target
// and the RoIAlign rows (batch index, box) of all slots and of the first nfg (mask) slots.
__global__ __launch_bounds__(256) void roi_gather_kernel(const int64_t* __restrict__ idx, int N, int nfg,
                                                         const float4* __restrict__ cand, int C,
                                                         const uint8_t* __restrict__ sel_fg, const int* __restrict__ am,
                                                         const int64_t* __restrict__ gt_labels,
                                                         const float4* __restrict__ gt, int G, float wx, float wy,
                                                         float ww, float wh, float4* __restrict__ rois,
                                                         int64_t* __restrict__ labels, int64_t* __restrict__ gidx,
                                                         float4* __restrict__ tgt, uint8_t* __restrict__ is_fg,
                                                         float* __restrict__ rois5, float* __restrict__ rois5_fg) {
  const int n = blockIdx.x * 256 + threadIdx.x, b = blockIdx.y;
  if (n >= N) return;
  const size_t o = (size_t)b * N + n;
  const int64_t i = idx[o];
  const float4 r = cand[(size_t)b * C + i];
  const bool fg = sel_fg[(size_t)b * C + i] != 0;
  const int g = max(am[(size_t)b * C + i], 0);
  const float4 mg = gt[(size_t)b * G + min(g, G - 1)];
  rois[o] = r;
  is_fg[o] = fg ? 1 : 0;
  gidx[o] = g;
  labels[o] = fg ? gt_labels[(size_t)b * G + min(g, G - 1)] : 0;
  tgt[o] = encode1(r, mg, wx, wy, ww, wh);
  float* d = rois5 + o * 5;
  d[0] = (float)b; d[1] = r.x; d[2] = r.y; d[3] = r.z; d[4] = r.w;
  if (n < nfg) {
    float* f = rois5_fg + ((size_t)b * nfg + n) * 5;
    f[0] = (float)b; f[1] = r.x; f[2] = r.y; f[3] = r.z; f[4] = r.w;
  }
}

}  // namespace

// out[i] = encode(ref[i] (or ref[0] when ref_bcast), gt[i]) with weights (wx, wy, ww, wh); fp32 [n, 4]
MX_EXPORT int mx_encode_boxes(const float* ref, int ref_bcast, const float* gt, int n, float wx, float wy, float ww,
                              float wh, float* out, hipStream_t s) {
  if (n <= 0) return hipSuccess;
  hipLaunchKernelGGL(encode_kernel, dim3((n + 255) / 256), dim3(256), 0, s, (const float4*)ref, ref_bcast,
                     (const float4*)gt, n, wx, wy, ww, wh, (float4*)out);
  return hipGetLastError();
}

// RPN labelling (see rpn_keys_kernel): anchors [A][4], mi / am / lq / rnd [B][A], img_hw [B][2]
// (h, w), gt [B][G][4] -> kpos / kneg [B][A] keys, enc [B][A][4], sel_pos / sel_neg zeroed.
MX_EXPORT int mx_rpn_keys(const float* anchors, int A, int B, const float* mi, const int* am, const int* lq,
                          const float* img_hw, const float* rnd, const float* gt, int G, float fg_thr, float bg_thr,
                          float* kpos, float* kneg, float* enc, uint8_t* sel_pos, uint8_t* sel_neg, hipStream_t s) {
  if (A <= 0 || B <= 0 || G <= 0) return (int)hipErrorInvalidValue;
  hipLaunchKernelGGL(rpn_keys_kernel, dim3((A + 255) / 256, B), dim3(256), 0, s, (const float4*)anchors, A, mi, am, lq,
                     img_hw, rnd, (const float4*)gt, G, fg_thr, bg_thr, kpos, kneg, (float4*)enc, sel_pos, sel_neg);
  return hipGetLastError();
}

// vpos / ipos, vneg / ineg: [B][ld] sorted key / index rows (the first kp / kn used)
MX_EXPORT int mx_rpn_select(const float* vpos, const int64_t* ipos, int kp, const float* vneg, const int64_t* ineg,
                            int kn, int ld, int batch, int A, int B, uint8_t* sel_pos, uint8_t* sel_neg,
                            hipStream_t s) {
  if (B <= 0) return hipSuccess;
  if (ld < kp || ld < kn) return hipErrorInvalidValue;
  hipLaunchKernelGGL(rpn_select_kernel, dim3(B), dim3(256), 0, s, vpos, ipos, kp, vneg, ineg, kn, ld, batch, A,
                     sel_pos, sel_neg);
  return hipGetLastError();
}

MX_EXPORT int mx_roi_candidates(const float* props, int K, const float* gt, const int* gcount, int G, int B,
                                float* cand, uint8_t* cvalid, hipStream_t s) {
  if (B <= 0 || K + G <= 0) return hipSuccess;
  hipLaunchKernelGGL(roi_cand_kernel, dim3((K + G + 255) / 256, B), dim3(256), 0, s, (const float4*)props, K,
                     (const float4*)gt, gcount, G, (float4*)cand, cvalid);
  return hipGetLastError();
}

MX_EXPORT int mx_roi_fgkey(const float* mi, const uint8_t* cvalid, const float* rnd, int n, float fg_thr, float* key,
                           hipStream_t s) {
  if (n <= 0) return hipSuccess;
  hipLaunchKernelGGL(roi_fgkey_kernel, dim3((n + 255) / 256), dim3(256), 0, s, mi, cvalid, rnd, n, fg_thr, key);
  return hipGetLastError();
}

MX_EXPORT int mx_roi_order(const float* vfg, const int64_t* ifg, int kf, const float* mi, const uint8_t* cvalid,
                           const float* rnd, int C, int B, float fg_thr, uint8_t* sel_fg, float* key, hipStream_t s) {
  if (B <= 0) return hipSuccess;
  hipLaunchKernelGGL(roi_order_kernel, dim3(B), dim3(256), 0, s, vfg, ifg, kf, mi, cvalid, rnd, C, fg_thr, sel_fg, key);
  return hipGetLastError();
}

MX_EXPORT int mx_roi_gather(const int64_t* idx, int N, int nfg, int B, const float* cand, int C, const uint8_t* sel_fg,
                            const int* am, const int64_t* gt_labels, const float* gt, int G, float wx, float wy,
                            float ww, float wh, float* rois, int64_t* labels, int64_t* gidx, float* tgt,
                            uint8_t* is_fg, float* rois5, float* rois5_fg, hipStream_t s) {
  if (B <= 0 || N <= 0 || G <= 0) return (int)hipErrorInvalidValue;
  hipLaunchKernelGGL(roi_gather_kernel, dim3((N + 255) / 256, B), dim3(256), 0, s, idx, N, nfg, (const float4*)cand, C,
                     sel_fg, am, gt_labels, (const float4*)gt, G, wx, wy, ww, wh, (float4*)rois, labels, gidx,
                     (float4*)tgt, is_fg, rois5, rois5_fg);
  return hipGetLastError();
}

// ------------------------------------------------------------------------------ RPN canvas
// The RPN head's 1x1 output on the level canvas (models/maskrcnn.py forward_levels), NHWC
// bf16 [B][Hc][Wc][C] with C >= 5 na (objectness na, then 4 na box deltas), to the flat
// per-image anchor order of all levels: logits [B][A] and deltas [B][A][4], anchor index
// off_l + (y w_l + x) na + a of level l at canvas (y0_l + y, x0_l + x).  geo: int32 [L][5]
// (y0, x0, h, w, off_l).  One thread per (image, level pixel); replaces 10 strided copies
// (per level: the logits slice and the deltas slice) and the two concatenations after them.
namespace {
constexpr int kMaxLevels = 8;
struct LevelGeo {
  int y0[kMaxLevels], x0[kMaxLevels], h[kMaxLevels], w[kMaxLevels], off[kMaxLevels], pix0[kMaxLevels + 1];
  int L;
};

__global__ __launch_bounds__(256) void rpn_unpack_kernel(const uint16_t* __restrict__ o, int Hc, int Wc, int C, int na,
                                                         LevelGeo g, int A, uint16_t* __restrict__ logits,
                                                         uint16_t* __restrict__ deltas) {
  const int p = blockIdx.x * 256 + threadIdx.x, b = blockIdx.y;
  if (p >= g.pix0[g.L]) return;
  int l = 0;
  while (l + 1 < g.L && p >= g.pix0[l + 1]) ++l;
  const int q = p - g.pix0[l], y = q / g.w[l], x = q - y * g.w[l];
  const uint16_t* src = o + (((size_t)b * Hc + g.y0[l] + y) * Wc + g.x0[l] + x) * C;
  const size_t a0 = (size_t)b * A + g.off[l] + (size_t)q * na;
  for (int a = 0; a < na; ++a) logits[a0 + a] = src[a];
  for (int j = 0; j < 4 * na; ++j) deltas[a0 * 4 + j] = src[na + j];
}

// Backward: every canvas pixel (so the gradient needs no zero-fill): level pixels take their
// anchors' logit / delta gradients, channels past 5 na and pixels between levels zeros.
__global__ __launch_bounds__(256) void rpn_pack_grad_kernel(const uint16_t* __restrict__ dlogits,
                                                            const uint16_t* __restrict__ ddeltas, int Hc, int Wc, int C,
                                                            int na, LevelGeo g, int A, uint16_t* __restrict__ d) {
  const int p = blockIdx.x * 256 + threadIdx.x, b = blockIdx.y;
  if (p >= Hc * Wc) return;
  const int cy = p / Wc, cx = p - cy * Wc;
  uint16_t* dst = d + ((size_t)b * Hc * Wc + p) * C;
  int l = -1;
  for (int i = 0; i < g.L; ++i)
    if (cy >= g.y0[i] && cy < g.y0[i] + g.h[i] && cx >= g.x0[i] && cx < g.x0[i] + g.w[i]) l = i;
  if (l < 0) {
    for (int c = 0; c < C; ++c) dst[c] = 0;
    return;
  }
  const int q = (cy - g.y0[l]) * g.w[l] + (cx - g.x0[l]);
  const size_t a0 = (size_t)b * A + g.off[l] + (size_t)q * na;
  for (int a = 0; a < na; ++a) dst[a] = dlogits ? dlogits[a0 + a] : 0;
  for (int j = 0; j < 4 * na; ++j) dst[na + j] = ddeltas ? ddeltas[a0 * 4 + j] : 0;
  for (int c = 5 * na; c < C; ++c) dst[c] = 0;
}

bool make_geo(const int* geo, int L, LevelGeo& g) {
  if (L < 1 || L > kMaxLevels) return false;
  g.L = L;
  g.pix0[0] = 0;
  for (int i = 0; i < L; ++i) {
    g.y0[i] = geo[5 * i]; g.x0[i] = geo[5 * i + 1]; g.h[i] = geo[5 * i + 2]; g.w[i] = geo[5 * i + 3];
    g.off[i] = geo[5 * i + 4];
    g.pix0[i + 1] = g.pix0[i] + g.h[i] * g.w[i];
  }
  return true;
}
}  // namespace

// geo: HOST int32 [L][5] (y0, x0, h, w, anchor offset of the level)
MX_EXPORT int mx_rpn_unpack(const void* o, int B, int Hc, int Wc, int C, int na, const int* geo, int L, int A,
                            void* logits, void* deltas, hipStream_t s) {
  LevelGeo g;
  if (!make_geo(geo, L, g) || C < 5 * na || B <= 0) return (int)hipErrorInvalidValue;
  hipLaunchKernelGGL(rpn_unpack_kernel, dim3((g.pix0[L] + 255) / 256, B), dim3(256), 0, s, (const uint16_t*)o, Hc, Wc,
                     C, na, g, A, (uint16_t*)logits, (uint16_t*)deltas);
  return hipGetLastError();
}

MX_EXPORT int mx_rpn_pack_grad(const void* dlogits, const void* ddeltas, int B, int Hc, int Wc, int C, int na,
                               const int* geo, int L, int A, void* d, hipStream_t s) {
  LevelGeo g;
  if (!make_geo(geo, L, g) || C < 5 * na || B <= 0) return (int)hipErrorInvalidValue;
  hipLaunchKernelGGL(rpn_pack_grad_kernel, dim3((Hc * Wc + 255) / 256, B), dim3(256), 0, s, (const uint16_t*)dlogits,
                     (const uint16_t*)ddeltas, Hc, Wc, C, na, g, A, (uint16_t*)d);
  return hipGetLastError();
}

// ------------------------------------------------------------------------------ FPN fan-in
// The gradient of an FPN level that feeds the RPN canvas, the box RoIAlign and the mask
// RoIAlign: out = a + b + c in ONE pass (NHWC bf16, 8 channels per thread, fp32 sum), a
// read through its canvas pitch (a strided slice of the canvas gradient), b / c contiguous
// (null = absent).  Autograd summed them with two adds, one of them PyTorch's
// non-vectorised strided kernel: 6 passes over the level instead of 4.
namespace {
__global__ __launch_bounds__(256) void add3_nhwc_kernel(uint16_t* __restrict__ out, const uint16_t* __restrict__ a,
                                                        int64_t a_img, int64_t a_row, const uint16_t* __restrict__ b,
                                                        const uint16_t* __restrict__ c, int H, int W, int C8,
                                                        int64_t nvec) {
  for (int64_t v = (int64_t)blockIdx.x * 256 + threadIdx.x; v < nvec; v += (int64_t)gridDim.x * 256) {
    const int64_t pix = v / C8;
    const int c8 = (int)(v - pix * C8);
    const int64_t n = pix / ((int64_t)H * W);
    const int rem = (int)(pix - n * H * W);
    const int y = rem / W, x = rem - (rem / W) * W;
    float s[8] = {0, 0, 0, 0, 0, 0, 0, 0}, t[8];
    if (a) {
      unpack8(reinterpret_cast<const uint4*>(a + n * a_img + (int64_t)y * a_row + (int64_t)x * C8 * 8)[c8], t);
#pragma unroll
      for (int j = 0; j < 8; ++j) s[j] += t[j];
    }
    if (b) {
      unpack8(reinterpret_cast<const uint4*>(b)[v], t);
#pragma unroll
      for (int j = 0; j < 8; ++j) s[j] += t[j];
    }
    if (c) {
      unpack8(reinterpret_cast<const uint4*>(c)[v], t);
#pragma unroll
      for (int j = 0; j < 8; ++j) s[j] += t[j];
    }
    reinterpret_cast<uint4*>(out)[v] = pack8(s);
  }
}
}  // namespace

// out [B][H][W][C] = a + b + c; a: element strides (a_img, a_row) per image / row, channels
// and pixels of a row contiguous; C % 8 == 0, every pointer 16-B aligned
MX_EXPORT int mx_add3_nhwc(void* out, const void* a, int64_t a_img, int64_t a_row, const void* b, const void* c, int B,
                           int H, int W, int C, hipStream_t s) {
  if (C % 8 || B <= 0) return (int)hipErrorInvalidValue;
  const int64_t nvec = (int64_t)B * H * W * (C / 8);
  const int64_t blocks = (nvec + 255) / 256 < 8192 ? (nvec + 255) / 256 : 8192;
  hipLaunchKernelGGL(add3_nhwc_kernel, dim3((unsigned)blocks), dim3(256), 0, s, (uint16_t*)out, (const uint16_t*)a,
                     a_img, a_row, (const uint16_t*)b, (const uint16_t*)c, H, W, C / 8, nvec);
  return hipGetLastError();
}

// ------------------------------------------------------------------------------ RPN canvas pack
// The FPN levels (NHWC bf16, level l [B][h_l][w_l][C]) onto the RPN canvas [B][Hc][Wc][C]
// in ONE pass over the canvas: level pixels copied, everything between them zero (the
// former zero-fill of the whole canvas + one row-copy launch per level wrote most of it
// twice).  16-B vectors; srcs: device pointer array (host-built, passed by value).
namespace {
struct PackSrc {
  const uint16_t* p[kMaxLevels];
};
__global__ __launch_bounds__(256) void rpn_pack_kernel(uint16_t* __restrict__ dst, PackSrc src, LevelGeo g, int Hc,
                                                       int Wc, int C8, int64_t nvec) {
  for (int64_t v = (int64_t)blockIdx.x * 256 + threadIdx.x; v < nvec; v += (int64_t)gridDim.x * 256) {
    const int64_t pix = v / C8;
    const int c8 = (int)(v - pix * C8);
    const int64_t n = pix / ((int64_t)Hc * Wc);
    const int rem = (int)(pix - n * Hc * Wc);
    const int cy = rem / Wc, cx = rem - (rem / Wc) * Wc;
    uint4 val = make_uint4(0u, 0u, 0u, 0u);
    for (int i = 0; i < g.L; ++i) {
      const int y = cy - g.y0[i], x = cx - g.x0[i];
      if (y >= 0 && y < g.h[i] && x >= 0 && x < g.w[i]) {
        val = reinterpret_cast<const uint4*>(src.p[i] + (((int64_t)n * g.h[i] + y) * g.w[i] + x) * C8 * 8)[c8];
        break;
      }
    }
    reinterpret_cast<uint4*>(dst)[v] = val;
  }
}
}  // namespace

// srcs: host array of L device pointers; geo: host int32 [L][5] (y0, x0, h, w, unused)
MX_EXPORT int mx_rpn_pack(void* dst, const void* const* srcs, const int* geo, int L, int B, int Hc, int Wc, int C,
                          hipStream_t s) {
  LevelGeo g;
  if (!make_geo(geo, L, g) || C % 8 || B <= 0) return (int)hipErrorInvalidValue;
  PackSrc ps = {};
  for (int i = 0; i < L; ++i) ps.p[i] = (const uint16_t*)srcs[i];
  const int64_t nvec = (int64_t)B * Hc * Wc * (C / 8);
  const int64_t blocks = (nvec + 255) / 256 < 16384 ? (nvec + 255) / 256 : 16384;
  hipLaunchKernelGGL(rpn_pack_kernel, dim3((unsigned)blocks), dim3(256), 0, s, (uint16_t*)dst, ps, g, Hc, Wc, C / 8,
                     nvec);
  return hipGetLastError();
}
