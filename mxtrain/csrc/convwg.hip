// Convolution weight gradients for NHWC bf16 CNNs on gfx950, as one implicit GEMM per
// launch: dW[co][r][s][ci] = sum over output pixels p of dY[p][co] * X[pix(p, r, s)][ci],
// written straight into the channels_last bf16 weight-gradient layout ([Cout][KH][KW][Cin],
// the layout of the Mask R-CNN compute copies, models/compute_weights.py).
//
// Why: in the graphed Mask R-CNN step MIOpen's weight-gradient solvers took ~2.1 ms of the
// ~12 ms step (CK `batched_gemm_xdlops_bwd_weight` 1.84 ms + `igemm_wrw` 0.27 ms, i.e.
// ~0.2 PF/s on ~200 G multiply-adds), plus ~0.8 ms of their helper kernels (fp32 workspace
// zero-fills, SubTensorOp zero / cast passes): profiles/r2_maskrcnn_s3/census_1img_graph_948_kernels.txt,
// profiles/r2_maskrcnn_s4/README.md.  Reference: the tensorpack / Detectron Mask R-CNN
// backbone + FPN + heads (examples/maskrcnn/train-maskrcnn-aws.yaml).
//
// Design -- the K-major x K-major MFMA GEMM of gemm.hip, with the reduction running over
// output pixels instead of tokens:
//  * one tile = (tap, 128-row Cout block, 128-column Cin block); every tap (r, s) of a
//    KH x KW filter is its own set of tiles in the same launch, so a 3x3 conv is ONE
//    launch, and no im2col / padded copy of X is ever made: each LDS-DMA lane computes its
//    input pixel (n, oh*st - pad + r*dil, ow*st - pad + s*dil) from the output-pixel index
//    and points out-of-image pixels (and rows past the last pixel) at a zero row;
//  * split-K over the pixels: the output is small (Cout x Cin per tap) and the reduction
//    long (up to ~270k pixels), so every launch is cut into `splits` pixel ranges, the grid
//    ordered slice-major (a slice's dY / X panels are shared by all tiles of one XCD in its
//    L2); fp32 partial tiles go to a slab that a second, chip-wide launch sums in slice
//    order -- deterministic, no float atomics, no zero-fill.  (A last-arriving-slice
//    reduction as in gemm.hip serialised up to 7.5 MB of partial reads on one workgroup per
//    tile: FPN lateral P2 104 us instead of MIOpen's 70 us, profiles/r3_s4/conv_wgrad_*.txt);
//  * 128 x 128 tiles of 4 waves (64 x 64 each, 16x16x32 bf16 MFMA), BK 64, 2-slot ring,
//    two workgroups per CU; LDS-DMA (global_load_lds_dwordx4) staging, transposed LDS reads
//    (ds_read_b64_tr_b16) with the source-side XOR swizzle, as in gemm.hip.
#include "gemm_common.h"

using namespace mx;
using namespace mx::gemm;

namespace {

struct ConvWg {
  const uint16_t* dy;    // [T][ldy]: output pixels (n, oh, ow) row-major, Cout contiguous
  const uint16_t* x;     // [N * IH * IW][ldx]: input pixels, Cin contiguous
  const uint16_t* zero;  // >= 256 zero bf16 (16-B aligned)
  uint16_t* dw;          // [Cout][taps][Cin]
  float* slab;           // split-K partials [ntiles][splits][NR][NT] float4
  int ldy, ldx;
  int T, OH, OW, IH, IW;
  int KW, taps, stride, pad, dil;
  int Cin, tiles_n, tiles_tap, ntiles;
  int splits, nk;        // pixel slices, 64-row K-steps per slice
  float invOW, invOH, beta;
  uint32_t xbytes, ybytes;   // sizes of x and dY (buffer resources; < 2 GiB)
  int Cout;              // < the tiles' rows for the narrow 1x1 heads: dY columns past it read
                         // zeros, dW rows past it are not written
};

__device__ __forceinline__ void divmod(int p, int d, float inv, int& q, int& r) {
  q = (int)((float)p * inv);
  r = p - q * d;
  if (r < 0) { --q; r += d; }
  else if (r >= d) { ++q; r -= d; }
}

template <int WM, int WN, int FM, int FN, int BKT, int NSLOT, int MINB, bool IDENT>
__global__ __launch_bounds__(64 * WM * WN, MINB) void conv_wgrad_kernel(const ConvWg cp) {
  constexpr int NW = WM * WN, NT = 64 * NW;
  constexpr int BM = 16 * FM * WM, BN = 16 * FN * WN;
  constexpr int RA = BM * 2, RB = BN * 2;
  constexpr int IA = BKT * RA, IB = BKT * RB;
  constexpr int PA = IA / 1024 / NW, PB = IB / 1024 / NW;
  constexpr int SLOT = IA + IB;
  static_assert(PA * NW * 1024 == IA && PB * NW * 1024 == IB, "DMA pieces per wave");
  __shared__ __attribute__((aligned(1024))) char smem[NSLOT * SLOT];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wg = xcd_remap(blockIdx.x, gridDim.x);
  // slice-major: consecutive workgroups (one XCD) share a pixel range across tiles
  const int slice = wg / cp.ntiles, t = wg - slice * cp.ntiles;
  const int tap = t / cp.tiles_tap, lt = t - tap * cp.tiles_tap;
  const int m0 = (lt / cp.tiles_n) * BM, n0 = (lt % cp.tiles_n) * BN;
  const int r = tap / cp.KW, s = tap - r * cp.KW;
  const int dh = r * cp.dil - cp.pad, dwc = s * cp.dil - cp.pad;
  const int nk = cp.nk;
  const int p0 = slice * nk * BKT;

  // ---- per-lane DMA rows: piece j of this wave holds 1024 / R consecutive k-rows
  constexpr int CA = RA / 16, CB = RB / 16;
  int kA[PA], cA[PA], kB[PB], cB[PB];
#pragma unroll
  for (int j = 0; j < PA; ++j) {
    kA[j] = (PA * wave + j) * (1024 / RA) + lane / CA;
    cA[j] = m0 + 8 * pchunk(kA[j], lane % CA);
  }
#pragma unroll
  for (int j = 0; j < PB; ++j) {
    kB[j] = (PB * wave + j) * (1024 / RB) + lane / CB;
    cB[j] = 8 * pchunk(kB[j], lane % CB);
  }
  // Per-lane gather state, advanced by one 64-pixel K-step per issue (32-bit offsets, no
  // per-step division or 64-bit math; the former per-step divmods and 64-bit addresses were
  // ~210 VALU per 32 MFMAs, profiles/r4_s3/pmc_conv_rpn_canvas_4img.txt).  dY rows past T
  // and input taps outside the image read zeros through out-of-range buffer offsets.
  const i32x4_t yres = buffer_rsrc(cp.dy, cp.ybytes), xres = buffer_rsrc(cp.x, cp.xbytes);
  uint32_t ya[PA];
  bool aok[PA];   // this lane's dY column exists (false only past a narrow Cout)
#pragma unroll
  for (int j = 0; j < PA; ++j) {
    ya[j] = (uint32_t)((p0 + kA[j]) * cp.ldy + cA[j]) * 2u;
    aok[j] = cA[j] < cp.Cout;
  }
  const uint32_t ystep = (uint32_t)(BKT * cp.ldy) * 2u;
  // B: pixel p = p0 + it BKT + kB[j] -> (oh s, ow s) and xo = ((n IH + oh s) IW + ow s) ldx
  int bp[PB], bohs[PB], bows[PB], bxo[PB];
  const int S_ = cp.stride, X_ = cp.ldx;
#pragma unroll
  for (int j = 0; j < PB; ++j) {
    const int p = p0 + kB[j];
    int q, ow, n, oh;
    divmod(p, cp.OW, cp.invOW, q, ow);
    divmod(q, cp.OH, cp.invOH, n, oh);
    bp[j] = p;
    bohs[j] = oh * S_;
    bows[j] = ow * S_;
    bxo[j] = IDENT ? p * X_ : ((n * cp.IH + oh * S_) * cp.IW + ow * S_) * X_;
  }
  const int dq = BKT / cp.OW, dr = BKT - dq * cp.OW;   // per-step (rows, columns) advance
  const int tapoff = (dh * cp.IW + dwc) * X_ + n0;    // this tile's tap and channel block
  auto advance = [&]() __attribute__((always_inline)) {
#pragma unroll
    for (int j = 0; j < PA; ++j) ya[j] += ystep;
#pragma unroll
    for (int j = 0; j < PB; ++j) {
      bp[j] += BKT;
      if (IDENT) {
        bxo[j] += BKT * X_;
      } else {
        bows[j] += dr * S_;
        bxo[j] += dr * S_ * X_;
        if (bows[j] >= cp.OW * S_) {
          bows[j] -= cp.OW * S_;
          bohs[j] += S_;
          bxo[j] += (S_ * cp.IW - cp.OW * S_) * X_;
        }
        bohs[j] += dq * S_;
        bxo[j] += dq * S_ * cp.IW * X_;
        while (bohs[j] >= cp.OH * S_) {   // next image (at most once when OH OW >= 64)
          bohs[j] -= cp.OH * S_;
          bxo[j] += (cp.IH - cp.OH * S_) * cp.IW * X_;
        }
      }
    }
  };
  auto boffB = [&](int j) __attribute__((always_inline)) {
    // (a narrow Cin -- 64 channels, the ResNet res2 convolutions -- reads zeros past it)
    bool ok = bp[j] < cp.T && n0 + cB[j] < cp.Cin;
    if (!IDENT)
      ok = ok && (unsigned)(bohs[j] + dh) < (unsigned)cp.IH && (unsigned)(bows[j] + dwc) < (unsigned)cp.IW;
    return ok ? (uint32_t)(bxo[j] + tapoff + cB[j]) * 2u : kOOB;
  };

  const int G = lane >> 4, i = lane & 15;
  const int wm = wave / WN, wn = wave % WN;
  const int krow = 8 * G + (i >> 2);
  const int g = gsw(krow);
  int offA[FM], offB[FN];
#pragma unroll
  for (int a = 0; a < FM; ++a)
    offA[a] = krow * RA + ((((FM * wm + a) ^ g) << 1) | ((i & 3) >> 1)) * 16 + (i & 1) * 8;
#pragma unroll
  for (int u = 0; u < FN; ++u)
    offB[u] = krow * RB + ((((FN * wn + u) ^ g) << 1) | ((i & 3) >> 1)) * 16 + (i & 1) * 8;

  f32x4 acc[FM][FN];
#pragma unroll
  for (int a = 0; a < FM; ++a)
#pragma unroll
    for (int u = 0; u < FN; ++u) acc[a][u] = f32x4{0.f, 0.f, 0.f, 0.f};

  const uint32_t lds0 = lds_addr(smem);
  auto issue = [&](int slot, int) __attribute__((always_inline)) {   // steps issued in order
    const uint32_t b0 = __builtin_amdgcn_readfirstlane(lds0 + slot * SLOT + PA * wave * 1024);
    const uint32_t b1 = __builtin_amdgcn_readfirstlane(lds0 + slot * SLOT + IA + PB * wave * 1024);
#pragma unroll
    for (int j = 0; j < PA; ++j) dma16_buf(yres, aok[j] ? ya[j] : kOOB, b0 + j * 1024);
#pragma unroll
    for (int j = 0; j < PB; ++j) dma16_buf(xres, boffB(j), b1 + j * 1024);
    advance();
  };
  constexpr int PER = PA + PB;

#pragma unroll
  for (int q = 0; q < NSLOT - 1; ++q)
    if (q < nk) issue(q, q);
  int slot = 0;
  for (int it = 0; it < nk; ++it) {
    const int later = nk - 1 - it;
    // retire step it's pieces (later steps' stay in flight), then one barrier
    if (NSLOT >= 4 && later >= 2) vm_wait<(NSLOT >= 4 ? 2 : 0) * PER>();
    else if (NSLOT >= 3 && later >= 1) vm_wait<(NSLOT >= 3 ? 1 : 0) * PER>();
    else vm_wait<0>();
    __builtin_amdgcn_s_barrier();
    if (it + NSLOT - 1 < nk) {
      int ns = slot + NSLOT - 1;
      if (ns >= NSLOT) ns -= NSLOT;
      issue(ns, it + NSLOT - 1);
    }
    const char* As = smem + slot * SLOT;
    const char* Bs = As + IA;
#pragma unroll
    for (int kk = 0; kk < BKT / 32; ++kk) {
      bf16x8 b[FN];
#pragma unroll
      for (int u = 0; u < FN; ++u)
        b[u] = cat(tr_read(Bs, offB[u] + 32 * RB * kk), tr_read(Bs, offB[u] + 32 * RB * kk + 4 * RB));
#pragma unroll
      for (int a = 0; a < FM; ++a) {
        const bf16x8 av = cat(tr_read(As, offA[a] + 32 * RA * kk), tr_read(As, offA[a] + 32 * RA * kk + 4 * RA));
#pragma unroll
        for (int u = 0; u < FN; ++u) acc[a][u] = mfma16(av, b[u], acc[a][u]);
      }
    }
    if (++slot == NSLOT) slot = 0;
  }

  if (cp.splits > 1) {
    // publish the partial tile; conv_wgrad_reduce sums the slices (spread over the chip)
    constexpr int NR = FM * FN;
    float4* mine = reinterpret_cast<float4*>(cp.slab) + ((size_t)(t * cp.splits + slice) * NR) * NT + tid;
#pragma unroll
    for (int a = 0; a < FM; ++a)
#pragma unroll
      for (int u = 0; u < FN; ++u)
        mine[(a * FN + u) * NT] = make_float4(acc[a][u][0], acc[a][u][1], acc[a][u][2], acc[a][u][3]);
    return;
  }

  // ---- epilogue: lane holds dW[m0 + 16 a + 4 G + e][tap][n0 + 16 u + i] of its wave's block
  const size_t ldc = (size_t)cp.taps * cp.Cin;
  const int mrow = m0 + 16 * FM * wm + 4 * G;
  uint16_t* C = cp.dw + (size_t)mrow * ldc + (size_t)tap * cp.Cin + n0 + 16 * FN * wn + i;
  const bool acc_in = cp.beta != 0.f;
#pragma unroll
  for (int a = 0; a < FM; ++a)
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      if (mrow + 16 * a + e >= cp.Cout) continue;
      uint16_t* row = C + (size_t)(16 * a + e) * ldc;
#pragma unroll
      for (int u = 0; u < FN; ++u) {
        if (n0 + 16 * FN * wn + 16 * u + i >= cp.Cin) continue;   // (narrow Cin: padded columns)
        float v = acc[a][u][e];
        if (acc_in) v += cp.beta * bf2f(row[16 * u]);
        row[16 * u] = f2bf(v);
      }
    }
}

constexpr int kBM = 128, kBN = 128, kBK = 64, kNT = 256;
// forward K-step depth: 0 -> 64, 1 -> 32 (16-KiB ring slots, up to four workgroups per CU),
// 2 (default) -> 32 for 1x1 convolutions and Cin <= 128, where the reduction is a few K-steps
// and the ring's fill dominates (scripts/conv_ab.py --toggle: 1x1 / Cin 128 forwards 5-15 %
// faster, the 3x3 Cin 256 ones at P2 and the RPN canvas 14-16 % slower,
// profiles/r5_s1/conv_ab_bk32.txt)
constexpr int g_conv_fwd_bk32 = 2;

// ================================================================================= forward
// y[p][co] = act(sum over taps (r, s) and ci of X[pix(p, r, s)][ci] * W[co][r][s][ci] + b[co]
// (+ res[p][co])): a GEMM over the output pixels (M) x Cout (N), reduction over (tap, ci)
// in 64-deep K-steps; the X rows are gathered per tap like the dY rows of the input
// gradient, the weight rows [co][64 ci] of a tap are a second K-contiguous image, so both
// MFMA operands are plain ds_read_b128 fragments.  The bias / residual / ReLU epilogue of
// ops/epilogue.py (the frozen-BN fold, the bottleneck join) is applied before the single
// store, so the separate in-place bias_act pass disappears too.
struct ConvFw {
  const uint16_t* x;     // [N * IH * IW][ldx]
  const uint16_t* w;     // [Cout][taps][Cin]
  const uint16_t* zero;
  uint16_t* y;           // [N * OH * OW][ldy]
  const uint16_t* bias;  // [Cout] or null
  const uint16_t* res;   // [N * OH * OW][ldy] or null; res_up: [N * OH/2 * OW/2][ldy], read
                         // nearest-upsampled (the FPN top-down join, res[n][oh/2][ow/2])
  int ldx, ldy;
  int T, OH, OW, IH, IW;
  int res_up;
  int KW, taps, stride, pad, dil;
  int Cin, tiles_n, nk, cib;
  float invOW, invOH;
  int splits, Cout;      // split-K (few output tiles): fp32 partials [splits][T][Cout] in part,
  float* part;           // then conv_fwd_reduce_kernel applies the epilogue
  uint32_t xbytes;       // size of x (the gather's buffer resource; < 2 GiB)
  uint32_t* ticket;      // non-null: the last-arriving split of a tile sums the partials and
                         // runs the epilogue itself (no reduction launch); [tiles], zero
  float* bnp;            // non-null (unsplit launches): BatchNorm statistics of y from the
                         // epilogue -- per 64-row block b (one wave's rows) and channel c the
                         // mean at bnp[c][b] and M2 at bnp[Cout + c][b], nblk = ceil(T / 64)
                         // blocks per row, channel-major so the finalize's loads coalesce
                         // (csrc/batchnorm.hip: no statistics pass over y)
};

// Split-K without a reduction launch: after publishing its fp32 partial tile, each split
// takes a ticket; the last one of the tile (a counter it resets) reads the others' partials
// back and runs the epilogue.  The partial stores are complete (vmcnt) and released at agent
// scope before the ticket, the last arriver acquires after it -- as gemm.hip's split-K.
// A per-convolution reduction launch cost ~5-7 us each, ~26 per 1-img Mask R-CNN step.
__device__ __forceinline__ bool split_last_arriver(uint32_t* ticket, int tile, int splits) {
  __shared__ uint32_t last_flag;
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0) {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
    const uint32_t prev = __hip_atomic_fetch_add(ticket + tile, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const uint32_t is_last = prev == (uint32_t)(splits - 1);
    if (is_last) {
      __hip_atomic_store(ticket + tile, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
    }
    last_flag = is_last;
  }
  __syncthreads();
  return last_flag != 0u;
}

// FN = 4: 128 x 128 tiles (Cout % 128 == 0); FN = 2: 128 x 64 tiles for Cout % 128 == 64 (the
// 64-channel res2 convolutions, which otherwise went to MIOpen)
// (256 x 128 tiles, one workgroup of 8 waves per CU, measured 3-8 % slower on the Mask R-CNN
// shapes: profiles/r4_s2/conv_fwd_tiles_4img.txt)
// K-contiguous image row swizzle: 128-B rows (BKT 64): chunk ^ (row & 7); 64-B rows
// (BKT 32, four rows per 256-B bank row): chunk ^ f((row >> 2) & 3), f = {0, 2, 3, 1}
// (gemm_nt.hip kc_swz): conflict-free ds_read_b128 over every 16-lane group either way
template <int R>
__device__ __forceinline__ int row_swz(int r) {
  if constexpr (R == 128) return r & 7;
  else return (0x78 >> (2 * ((r >> 2) & 3))) & 3;
}

// BKT 64: 2-slot ring of 32 KiB slots, two workgroups per CU (LDS-bound); BKT 32: 16 KiB
// slots, up to four workgroups per CU (VGPR-bound), twice the barriers per unit of K
template <int NSLOT, int FN, bool RES, bool RELU, int BKT = 64>
__global__ __launch_bounds__(256, 2) void conv_fwd_kernel(const ConvFw cp) {
  constexpr int WM = 2, WN = 2, FM = 4, NW = WM * WN;
  constexpr int BM = 16 * FM * WM, BN = 16 * FN * WN, R = BKT * 2;
  static_assert(FN == 2 || FN == 4, "tile width");
  constexpr int IA = BM * R, IB = BN * R;
  constexpr int PA = IA / 1024 / NW, PB = IB / 1024 / NW;
  constexpr int SLOT = IA + IB, PER = PA + PB;
  __shared__ __attribute__((aligned(1024))) char smem[NSLOT * SLOT];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wg = xcd_remap(blockIdx.x, gridDim.x);
  // split-K: the splits of one tile are adjacent (same XCD: they share its operand rows)
  const int sidx = wg % cp.splits, tile = wg / cp.splits;
  const int tm = tile / cp.tiles_n, tn = tile - tm * cp.tiles_n;
  const int m0 = tm * BM, n0 = tn * BN;
  const int kb = (int)((int64_t)sidx * cp.nk / cp.splits);
  const int nk = (int)((int64_t)(sidx + 1) * cp.nk / cp.splits) - kb;   // this split's K-steps
  const size_t ldw = (size_t)cp.taps * cp.Cin;

  // Per-lane constants of the gather, so a K-step's DMA addressing is 32-bit adds and one
  // select per piece: each A piece's element offset at tap (0, 0) (negative in the padding)
  // and a bit per filter tap that lands inside the image; padding taps read zeros through
  // an out-of-range buffer offset.  (The former 64-bit address per piece and step cost
  // ~80 VALU per K-step against 32 MFMAs: VALU:MFMA 4:1 in PMC,
  // profiles/r4_s3/pmc_conv_rpn_canvas_4img.txt.)
  int aoff[PA];
  uint32_t amask[PA];
#pragma unroll
  for (int j = 0; j < PA; ++j) {
    const int row = (PA * wave + j) * (1024 / R) + lane / (R / 16);
    const int p = m0 + row;
    const bool ok = p < cp.T;
    int q, ow, n, oh;
    divmod(ok ? p : 0, cp.OW, cp.invOW, q, ow);
    divmod(q, cp.OH, cp.invOH, n, oh);
    const int ih0 = oh * cp.stride - cp.pad, iw0 = ow * cp.stride - cp.pad;
    aoff[j] = ((n * cp.IH + ih0) * cp.IW + iw0) * cp.ldx + 8 * ((lane % (R / 16)) ^ row_swz<R>(row));
    uint32_t m = 0u;
    for (int r = 0, t = 0; r < cp.taps / cp.KW; ++r) {
      const bool rin = ok && (unsigned)(ih0 + r * cp.dil) < (unsigned)cp.IH;
      for (int c = 0; c < cp.KW; ++c, ++t)
        m |= (rin && (unsigned)(iw0 + c * cp.dil) < (unsigned)cp.IW) ? 1u << t : 0u;
    }
    amask[j] = m;
    asm volatile("" : "+v"(aoff[j]));   // keep the per-lane offset whole (no per-step re-multiply)
  }
  uint32_t boff[PB];
  bool bok[PB];   // the weight row exists (false only past a narrow Cout)
#pragma unroll
  for (int j = 0; j < PB; ++j) {
    const int brow = n0 + (PB * wave + j) * (1024 / R) + lane / (R / 16);
    bok[j] = brow < cp.Cout;
    boff[j] = (uint32_t)(brow * (int)ldw + 8 * ((lane % (R / 16)) ^ row_swz<R>(brow))) * 2u;
  }
  const i32x4_t xres = buffer_rsrc(cp.x, cp.xbytes);
  const bool narrow = cp.Cout % 64 != 0;   // (the 1x1 heads: weight rows past Cout read zeros)
  const i32x4_t wres = buffer_rsrc(cp.w, (uint32_t)(cp.Cout * ldw * 2));
  const int G = lane >> 4, i = lane & 15;
  const int wm = wave / WN, wn = wave % WN;
  const int offA = (16 * FM * wm + i) * R, offB = (16 * FN * wn + i) * R;
  int cK[BKT / 32];
#pragma unroll
  for (int kk = 0; kk < BKT / 32; ++kk) cK[kk] = 16 * ((4 * kk + G) ^ row_swz<R>(i));

  f32x4 acc[FM][FN];
#pragma unroll
  for (int a = 0; a < FM; ++a)
#pragma unroll
    for (int u = 0; u < FN; ++u) acc[a][u] = f32x4{0.f, 0.f, 0.f, 0.f};

  const uint32_t lds0 = lds_addr(smem);
  // K-step walk (wave-uniform, advanced once per issue: the steps are issued in order):
  // channel block, tap, the tap's filter row / column and its element offset in x
  int k_ci = kb % cp.cib, k_tap = kb / cp.cib;
  int k_r = k_tap / cp.KW, k_c = k_tap - (k_tap / cp.KW) * cp.KW;
  int k_toff = (k_r * cp.IW + k_c) * cp.dil * cp.ldx;
  auto issue = [&](int slot, int) __attribute__((always_inline)) {
    const int tap = k_tap, ci0 = k_ci * BKT;
    const int delta = k_toff + ci0;
    if (++k_ci == cp.cib) {
      k_ci = 0;
      ++k_tap;
      k_toff += cp.dil * cp.ldx;
      if (++k_c == cp.KW) { k_c = 0; k_toff += (cp.IW - cp.KW) * cp.dil * cp.ldx; }
    }
    const uint32_t b0 = __builtin_amdgcn_readfirstlane(lds0 + slot * SLOT + PA * wave * 1024);
    const uint32_t b1 = __builtin_amdgcn_readfirstlane(lds0 + slot * SLOT + IA + PB * wave * 1024);
#pragma unroll
    for (int j = 0; j < PA; ++j) {
      const bool in = (amask[j] >> tap) & 1u;
      dma16_buf(xres, in ? (uint32_t)(aoff[j] + delta) * 2u : kOOB, b0 + j * 1024);
    }
    if (narrow) {
      const uint32_t wo = (uint32_t)((size_t)tap * cp.Cin + ci0) * 2u;
#pragma unroll
      for (int j = 0; j < PB; ++j) dma16_buf(wres, bok[j] ? wo + boff[j] : kOOB, b1 + j * 1024);
    } else {
      const uint16_t* wb = cp.w + (size_t)tap * cp.Cin + ci0;
#pragma unroll
      for (int j = 0; j < PB; ++j) dma16_sbase(wb, boff[j], b1 + j * 1024);
    }
  };

  // NSLOT-deep LDS-DMA ring, counted waits (the input gradient's scheme): with NSLOT > 2 the
  // next steps' pieces stay in flight across the barrier
#pragma unroll
  for (int q = 0; q < NSLOT - 1; ++q)
    if (q < nk) issue(q, q);
  int slot = 0;
  for (int it = 0; it < nk; ++it) {
    const int later = nk - 1 - it;
    if (NSLOT >= 4 && later >= 2) vm_wait<(NSLOT >= 4 ? 2 : 0) * PER>();
    else if (NSLOT >= 3 && later >= 1) vm_wait<(NSLOT >= 3 ? 1 : 0) * PER>();
    else vm_wait<0>();
    __builtin_amdgcn_s_barrier();
    if (it + NSLOT - 1 < nk) {
      int ns = slot + NSLOT - 1;
      if (ns >= NSLOT) ns -= NSLOT;
      issue(ns, it + NSLOT - 1);
    }
    const char* As = smem + slot * SLOT;
    const char* Bs = As + IA;
#pragma unroll
    for (int kk = 0; kk < BKT / 32; ++kk) {
      bf16x8 b[FN];
#pragma unroll
      for (int u = 0; u < FN; ++u) b[u] = lds_read8(Bs, offB + 16 * u * R + cK[kk]);
#pragma unroll
      for (int a = 0; a < FM; ++a) {
        const bf16x8 av = lds_read8(As, offA + 16 * a * R + cK[kk]);
        // the weight fragment is the A operand: a lane ends with 4 consecutive output
        // channels of one pixel (epilogue below)
#pragma unroll
        for (int u = 0; u < FN; ++u) acc[a][u] = mfma16(b[u], av, acc[a][u]);
      }
    }
    if (++slot == NSLOT) slot = 0;
  }

  // ---- epilogue: lane (G, i) holds y[m0 + 16 (FM wm + a) + i][n0 + 16 (FN wn + u) + 4 G + e];
  // pairs of 16-channel subtiles are re-dealt (permlane swaps) so every lane stores 8
  // consecutive channels: 16-B stores and 16-B residual loads (2-B scattered stores made
  // the epilogue store-issue bound)
  const int colw = n0 + 16 * FN * wn;
  if (cp.splits > 1) {   // split-K: raw fp32 partial sums, the epilogue runs in the reduction
#pragma unroll
    for (int a = 0; a < FM; ++a) {
      const int p = m0 + 16 * (FM * wm + a) + i;
      if (p < cp.T) {
        float* dst = cp.part + ((size_t)sidx * cp.T + p) * cp.Cout + colw + 4 * G;
#pragma unroll
        for (int u = 0; u < FN; ++u) *reinterpret_cast<f32x4*>(dst + 16 * u) = acc[a][u];
      }
    }
    if (!cp.ticket || !split_last_arriver(cp.ticket, tile, cp.splits)) return;
    // the tile's sum over the splits in split order (deterministic whichever arrives last)
#pragma unroll
    for (int a = 0; a < FM; ++a) {
      const int p = m0 + 16 * (FM * wm + a) + i;
      const float* src = cp.part + ((size_t)(p < cp.T ? p : 0)) * cp.Cout + colw + 4 * G;
#pragma unroll
      for (int u = 0; u < FN; ++u) {
        f32x4 tot = f32x4{0.f, 0.f, 0.f, 0.f};
        for (int q = 0; q < cp.splits; ++q)
          tot += q == sidx ? acc[a][u] : *reinterpret_cast<const f32x4*>(src + (size_t)q * cp.T * cp.Cout + 16 * u);
        acc[a][u] = tot;
      }
    }
  }
  float bv[FN][4];
  float bs[FN][4], bq[FN][4];   // BatchNorm statistics: this lane's sum / sum of squares
#pragma unroll
  for (int u = 0; u < FN; ++u) {
#pragma unroll
    for (int e = 0; e < 4; ++e) bs[u][e] = bq[u][e] = 0.f;
    if (cp.bias && colw + 16 * u + 4 * G < cp.Cout) {
      const uint2 b2 = *reinterpret_cast<const uint2*>(cp.bias + colw + 16 * u + 4 * G);
      bv[u][0] = lo_bf(b2.x); bv[u][1] = hi_bf(b2.x); bv[u][2] = lo_bf(b2.y); bv[u][3] = hi_bf(b2.y);
    } else {
      bv[u][0] = bv[u][1] = bv[u][2] = bv[u][3] = 0.f;
    }
  }
#pragma unroll
  for (int a = 0; a < FM; ++a) {
    const int p = m0 + 16 * (FM * wm + a) + i;
    const size_t pr = (size_t)(p < cp.T ? p : cp.T - 1) * cp.ldy;   // every lane takes part in the swaps
#pragma unroll
    for (int up = 0; up < FN / 2; ++up) {
      uint32_t c[2][2], h[2][2];
      if (RES) {
        size_t rr = pr;
        if (cp.res_up) {
          int q, ow, n, oh;
          divmod(p < cp.T ? p : cp.T - 1, cp.OW, cp.invOW, q, ow);
          divmod(q, cp.OH, cp.invOH, n, oh);
          rr = ((size_t)(n * (cp.OH >> 1) + (oh >> 1)) * (cp.OW >> 1) + (ow >> 1)) * cp.ldy;
        }
        const uint4 rv = colw + 32 * up + 8 * G < cp.Cout ? *reinterpret_cast<const uint4*>(cp.res + rr + colw + 32 * up + 8 * G)
                                                         : make_uint4(0u, 0u, 0u, 0u);
        h[0][0] = rv.x; h[0][1] = rv.y; h[1][0] = rv.z; h[1][1] = rv.w;
        undeal(h[0][0], h[0][1], h[1][0], h[1][1]);
      }
#pragma unroll
      for (int hlf = 0; hlf < 2; ++hlf) {
        const int u = 2 * up + hlf;
        float v[4];
#pragma unroll
        for (int e = 0; e < 4; ++e) v[e] = acc[a][u][e] + bv[u][e];
        if (RES) {
          v[0] += lo_bf(h[hlf][0]); v[1] += hi_bf(h[hlf][0]);
          v[2] += lo_bf(h[hlf][1]); v[3] += hi_bf(h[hlf][1]);
        }
        if (RELU) {
#pragma unroll
          for (int e = 0; e < 4; ++e) v[e] = fmaxf(v[e], 0.f);
        }
        c[hlf][0] = pack2(v[0], v[1]);
        c[hlf][1] = pack2(v[2], v[3]);
        if (cp.bnp && p < cp.T) {   // the statistics of the stored (rounded) values
          const float r[4] = {lo_bf(c[hlf][0]), hi_bf(c[hlf][0]), lo_bf(c[hlf][1]), hi_bf(c[hlf][1])};
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            bs[u][e] += r[e];
            bq[u][e] = __builtin_fmaf(r[e], r[e], bq[u][e]);
          }
        }
      }
      deal(c[0][0], c[0][1], c[1][0], c[1][1]);
      if (p < cp.T && colw + 32 * up + 8 * G < cp.Cout)
        *reinterpret_cast<uint4*>(cp.y + pr + colw + 32 * up + 8 * G) = make_uint4(c[0][0], c[0][1], c[1][0], c[1][1]);
    }
  }
  if (cp.bnp) {
    // the wave's 64 rows (16 lanes x FM fragments per channel): row sums over the lanes, then
    // (mean, M2) = (s / n, q - s * mean) -- the per-thread form of bn_stats_kernel
    const int rb = m0 + 64 * wm, n = cp.T - rb < 64 ? cp.T - rb : 64;
    if (n > 0) {
      const float inv = 1.f / (float)n;
      const size_t nblk = (size_t)((cp.T + 63) / 64);
      float* pm = cp.bnp + (size_t)(rb / 64);
#pragma unroll
      for (int u = 0; u < FN; ++u) {
        float mo[4], qo[4];
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const float s1 = row_sum16(bs[u][e]), q1 = row_sum16(bq[u][e]);
          mo[e] = s1 * inv;
          qo[e] = fmaxf(q1 - s1 * mo[e], 0.f);
        }
        // every lane of the row holds the sums: lane i < 4 stores channel col + i
        const int col = colw + 16 * u + 4 * G + (i & 3);
        const float mv = i == 0 ? mo[0] : i == 1 ? mo[1] : i == 2 ? mo[2] : mo[3];
        const float qv = i == 0 ? qo[0] : i == 1 ? qo[1] : i == 2 ? qo[2] : qo[3];
        if (i < 4 && col < cp.Cout) {
          pm[(size_t)col * nblk] = mv;
          pm[(size_t)(cp.Cout + col) * nblk] = qv;
        }
      }
    }
  }
}

// split-K forward: y[p][c] = act(sum_s part[s][p][c] + b[c] (+ res)), splits summed in order
// (deterministic); one thread per 8 channels of a pixel
template <bool RES, bool RELU>
__global__ __launch_bounds__(256) void conv_fwd_reduce_kernel(const ConvFw cp) {
  const int c8 = cp.Cout / 8;
  const int64_t nvec = (int64_t)cp.T * c8;
  for (int64_t v = (int64_t)blockIdx.x * 256 + threadIdx.x; v < nvec; v += (int64_t)gridDim.x * 256) {
    const int p = (int)(v / c8), c = (int)(v - (int64_t)p * c8) * 8;
    float o[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    for (int s2 = 0; s2 < cp.splits; ++s2) {
      const float4* q = reinterpret_cast<const float4*>(cp.part + ((size_t)s2 * cp.T + p) * cp.Cout + c);
      const float4 x0 = q[0], x1 = q[1];
      o[0] += x0.x; o[1] += x0.y; o[2] += x0.z; o[3] += x0.w;
      o[4] += x1.x; o[5] += x1.y; o[6] += x1.z; o[7] += x1.w;
    }
    if (cp.bias) {
      float b[8];
      unpack8(*reinterpret_cast<const uint4*>(cp.bias + c), b);
#pragma unroll
      for (int j = 0; j < 8; ++j) o[j] += b[j];
    }
    if (RES) {
      size_t rr = (size_t)p * cp.ldy;
      if (cp.res_up) {
        int q2, ow, n, oh;
        divmod(p, cp.OW, cp.invOW, q2, ow);
        divmod(q2, cp.OH, cp.invOH, n, oh);
        rr = ((size_t)(n * (cp.OH >> 1) + (oh >> 1)) * (cp.OW >> 1) + (ow >> 1)) * cp.ldy;
      }
      float r[8];
      unpack8(*reinterpret_cast<const uint4*>(cp.res + rr + c), r);
#pragma unroll
      for (int j = 0; j < 8; ++j) o[j] += r[j];
    }
    if (RELU) {
#pragma unroll
      for (int j = 0; j < 8; ++j) o[j] = fmaxf(o[j], 0.f);
    }
    *reinterpret_cast<uint4*>(cp.y + (size_t)p * cp.ldy + c) = pack8(o);
  }
}

// ============================================================================ input gradient
// dX[p][ci] = sum over taps (r, s) and output channels co of dY[q(p, r, s)][co] * W[co][r][s][ci]
// with q the output pixel whose window puts tap (r, s) on input pixel p (none, i.e. a zero
// row, when the tap falls outside the output image or between strides).  A GEMM over the
// input pixels (M) x Cin (N) with the reduction over (tap, co) in 64-deep K-steps: the dY
// rows are gathered per tap by the LDS-DMA lanes (K-contiguous [m][64 co] image, 128-B rows
// XOR-swizzled by row & 7, ds_read_b128 fragments), the weight rows [co][Cin] of a tap are
// a K-major image read with the transposed-read scheme of the weight gradient above.
// Replaces MIOpen's backward-data solvers (CK grouped bwd-data, igemm_bwd_gtcx35: ~2 ms of
// the 1-img Mask R-CNN step, profiles/r2_maskrcnn_s3/census_1img_graph_948_kernels.txt).
struct ConvDg {
  const uint16_t* dy;    // [N * OH * OW][ldy]
  const uint16_t* w;     // [Cout][taps][Cin]
  const uint16_t* zero;  // >= 256 zero bf16
  uint16_t* dx;          // [N * IH * IW][ldx]
  const uint16_t* add;   // [N * IH * IW][ldx] or null: added to dX (a second gradient of X)
  const uint16_t* mask;  // [N * IH * IW][ldx] or null: dX zeroed where mask <= 0 (X's ReLU)
  int ldy, ldx;
  int T, OH, OW, IH, IW;
  int KW, taps, stride, pad, dil;
  int Cin, tiles_n, nk, cob;
  float invIW, invIH;
  int splits;            // split-K (few input-pixel tiles): fp32 partials [splits][T][Cin] in
  float* part;           // part, reduced with the add / mask epilogue by conv_dgrad_reduce_kernel
  int ldw;               // weight row pitch (elements per output channel: taps * Cin)
  int Cout;              // output channels (a multiple of 8; K-steps past it read zeros)
  const uint16_t* bias;  // [Cin] or null: + bias (the transposed convolution's forward)
  int relu;              // max(., 0) after bias / add, before the mask
  // parity class (xs > 0): this launch's pixels are the dX pixels (i * xs + xa, j * xs + xb)
  // of an XH x XW image, enumerated as an IH x IW grid (stride-decomposed dgrad, below)
  int xs, xa, xb, XH, XW;
  uint32_t ybytes;       // size of dY (the gather's buffer resource; < 2 GiB)
  int bkt;               // K-step depth (output channels per step): 64 or 32 (host-side choice)
  uint32_t* ticket;      // as ConvFw::ticket
  int add_rows;          // add indexed by the launch's pixel (add holds only this parity class)
};

// dX row of the launch's pixel p (identity unless a parity-class launch)
__device__ __forceinline__ int dx_row(const ConvDg& cp, int p) {
  if (!cp.xs) return p;
  int q, j, n, i;
  divmod(p, cp.IW, cp.invIW, q, j);
  divmod(q, cp.IH, cp.invIH, n, i);
  return (n * cp.XH + i * cp.xs + cp.xa) * cp.XW + j * cp.xs + cp.xb;
}

template <int NSLOT, int BKT = 64>
__global__ __launch_bounds__(256, 2) void conv_dgrad_kernel(const ConvDg cp) {
  constexpr int WM = 2, WN = 2, FM = 4, FN = 4, NW = WM * WN;
  constexpr int BM = 16 * FM * WM, BN = 128, RA = BKT * 2, RB = BN * 2;
  constexpr int IA = BM * RA, IB = BKT * RB;
  constexpr int PA = IA / 1024 / NW, PB = IB / 1024 / NW;
  constexpr int SLOT = IA + IB, PER = PA + PB;
  __shared__ __attribute__((aligned(1024))) char smem[NSLOT * SLOT];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wg = xcd_remap(blockIdx.x, gridDim.x);
  // Cin tiles of one pixel block adjacent (same XCD): they share the gathered dY rows in L2;
  // the splits of one tile adjacent too
  const int sidx = wg % cp.splits, tile = wg / cp.splits;
  const int tm = tile / cp.tiles_n, tn = tile - tm * cp.tiles_n;
  const int m0 = tm * BM, n0 = tn * BN;
  const int kb = (int)((int64_t)sidx * cp.nk / cp.splits);
  const int nk = (int)((int64_t)(sidx + 1) * cp.nk / cp.splits) - kb;
  const size_t ldw = (size_t)cp.ldw;

  // ---- A (gathered dY) rows of this lane: fixed input pixel per DMA piece.  As in the
  // forward: the element offset of dY[(ih + pad) / s][(iw + pad) / s] and a bit per tap whose
  // output pixel exists (in the image, on the stride grid); tap (r, c) then reads at the
  // wave-uniform delta -((r dil / s) OW + c dil / s) ldy (exact on the grid: ih + pad and
  // r dil have equal residues mod s there), padding through out-of-range buffer offsets.
  int aoff[PA], acol[PA];   // acol: the lane's dY column within a K-step (narrow Cout check)
  uint32_t amask[PA];
#pragma unroll
  for (int j = 0; j < PA; ++j) {
    const int row = (PA * wave + j) * (1024 / RA) + lane / (RA / 16);
    const int p = m0 + row;
    const bool ok = p < cp.T;
    int q, iw, n, ih;
    divmod(ok ? p : 0, cp.IW, cp.invIW, q, iw);
    divmod(q, cp.IH, cp.invIH, n, ih);
    const int hh = ih + cp.pad, ww = iw + cp.pad, st = cp.stride, KHt = cp.taps / cp.KW;
    const int sw = 8 * ((lane % (RA / 16)) ^ row_swz<RA>(row));
    acol[j] = sw;
    uint32_t m = 0u;
    if (st == 1) {   // (wave-uniform) no per-lane divisions on the common path
      aoff[j] = ((n * cp.OH + hh) * cp.OW + ww) * cp.ldy + sw;
      for (int r = 0, t = 0; r < KHt; ++r) {
        const bool rin = ok && (unsigned)(hh - r * cp.dil) < (unsigned)cp.OH;
        for (int c = 0; c < cp.KW; ++c, ++t)
          m |= (rin && (unsigned)(ww - c * cp.dil) < (unsigned)cp.OW) ? 1u << t : 0u;
      }
    } else {
      aoff[j] = ((n * cp.OH + hh / st) * cp.OW + ww / st) * cp.ldy + sw;
      for (int r = 0, t = 0; r < KHt; ++r) {
        const int ah = hh - r * cp.dil;
        const bool rin = ok && ah >= 0 && ah % st == 0 && ah / st < cp.OH;
        for (int c = 0; c < cp.KW; ++c, ++t) {
          const int aw = ww - c * cp.dil;
          m |= (rin && aw >= 0 && aw % st == 0 && aw / st < cp.OW) ? 1u << t : 0u;
        }
      }
    }
    amask[j] = m;
    asm volatile("" : "+v"(aoff[j]));   // keep the per-lane offset whole
  }
  uint32_t boff[PB];
  int bkrow[PB];
  bool bcol[PB];   // this lane's weight columns exist (false only past a narrow Cin)
#pragma unroll
  for (int j = 0; j < PB; ++j) {
    const int kB = (PB * wave + j) * (1024 / RB) + lane / (RB / 16);
    bkrow[j] = kB;
    bcol[j] = n0 + 8 * pchunk(kB, lane % (RB / 16)) < cp.Cin;
    boff[j] = (uint32_t)(kB * (int)ldw + n0 + 8 * pchunk(kB, lane % (RB / 16))) * 2u;
  }
  const i32x4_t yres = buffer_rsrc(cp.dy, cp.ybytes);
  // narrow Cout (the 1x1 heads, Cout % BKT != 0): dY columns and weight rows past Cout read
  // zeros; narrow Cin (64 channels: the ResNet res2 convolutions, 128-column tiles half
  // padded): weight columns past Cin read zeros and the padded dX columns are not written
  const bool narrow = cp.Cout % BKT != 0 || cp.Cin % BN != 0;
  const i32x4_t wres = buffer_rsrc(cp.w, (uint32_t)(cp.Cout * cp.ldw * 2));

  const int G = lane >> 4, i = lane & 15;
  const int wm = wave / WN, wn = wave % WN;
  const int offA = (16 * FM * wm + i) * RA;
  int cA[BKT / 32];
#pragma unroll
  for (int kk = 0; kk < BKT / 32; ++kk) cA[kk] = 16 * ((4 * kk + G) ^ row_swz<RA>(i));
  const int krow = 8 * G + (i >> 2);
  const int gq = gsw(krow);
  int offB[FN];
#pragma unroll
  for (int u = 0; u < FN; ++u)
    offB[u] = krow * RB + ((((FN * wn + u) ^ gq) << 1) | ((i & 3) >> 1)) * 16 + (i & 1) * 8;

  f32x4 acc[FM][FN];
#pragma unroll
  for (int a = 0; a < FM; ++a)
#pragma unroll
    for (int u = 0; u < FN; ++u) acc[a][u] = f32x4{0.f, 0.f, 0.f, 0.f};

  const uint32_t lds0 = lds_addr(smem);
  // K-step walk (wave-uniform, advanced once per issue): output-channel block, tap, its
  // filter row / column and its dY element offset
  int k_co = kb % cp.cob, k_tap = kb / cp.cob;
  int k_r = k_tap / cp.KW, k_c = k_tap - (k_tap / cp.KW) * cp.KW;
  auto tap_off = [&]() __attribute__((always_inline)) {
    if (cp.stride == 1) return -(k_r * cp.OW + k_c) * cp.dil * cp.ldy;
    return -((k_r * cp.dil / cp.stride) * cp.OW + k_c * cp.dil / cp.stride) * cp.ldy;
  };
  int k_toff = tap_off();
  auto issue = [&](int slot, int) __attribute__((always_inline)) {
    const int tap = k_tap, co0 = k_co * BKT;
    const int delta = k_toff + co0;
    if (++k_co == cp.cob) {
      k_co = 0;
      ++k_tap;
      if (++k_c == cp.KW) { k_c = 0; ++k_r; }
      k_toff = tap_off();
    }
    const uint32_t b0 = __builtin_amdgcn_readfirstlane(lds0 + slot * SLOT + PA * wave * 1024);
    const uint32_t b1 = __builtin_amdgcn_readfirstlane(lds0 + slot * SLOT + IA + PB * wave * 1024);
#pragma unroll
    for (int j = 0; j < PA; ++j) {
      const bool in = ((amask[j] >> tap) & 1u) && (!narrow || co0 + acol[j] < cp.Cout);
      dma16_buf(yres, in ? (uint32_t)(aoff[j] + delta) * 2u : kOOB, b0 + j * 1024);
    }
    if (narrow) {
      const uint32_t wo = (uint32_t)((size_t)co0 * ldw + (size_t)tap * cp.Cin) * 2u;
#pragma unroll
      for (int j = 0; j < PB; ++j)
        dma16_buf(wres, (co0 + bkrow[j] < cp.Cout && bcol[j]) ? wo + boff[j] : kOOB, b1 + j * 1024);
    } else {
      const uint16_t* wb = cp.w + (size_t)co0 * ldw + (size_t)tap * cp.Cin;
#pragma unroll
      for (int j = 0; j < PB; ++j) dma16_sbase(wb, boff[j], b1 + j * 1024);
    }
  };

#pragma unroll
  for (int q = 0; q < NSLOT - 1; ++q)
    if (q < nk) issue(q, q);
  int slot = 0;
  for (int it = 0; it < nk; ++it) {
    const int later = nk - 1 - it;
    if (NSLOT >= 4 && later >= 2) vm_wait<(NSLOT >= 4 ? 2 : 0) * PER>();
    else if (NSLOT >= 3 && later >= 1) vm_wait<(NSLOT >= 3 ? 1 : 0) * PER>();
    else vm_wait<0>();
    __builtin_amdgcn_s_barrier();
    if (it + NSLOT - 1 < nk) {
      int ns = slot + NSLOT - 1;
      if (ns >= NSLOT) ns -= NSLOT;
      issue(ns, it + NSLOT - 1);
    }
    const char* As = smem + slot * SLOT;
    const char* Bs = As + IA;
#pragma unroll
    for (int kk = 0; kk < BKT / 32; ++kk) {
      bf16x8 b[FN];
#pragma unroll
      for (int u = 0; u < FN; ++u)
        b[u] = cat(tr_read(Bs, offB[u] + 32 * RB * kk), tr_read(Bs, offB[u] + 32 * RB * kk + 4 * RB));
#pragma unroll
      for (int a = 0; a < FM; ++a) {
        const bf16x8 av = lds_read8(As, offA + 16 * a * RA + cA[kk]);
        // weight fragment as the A operand: 4 consecutive input channels per lane
#pragma unroll
        for (int u = 0; u < FN; ++u) acc[a][u] = mfma16(b[u], av, acc[a][u]);
      }
    }
    if (++slot == NSLOT) slot = 0;
  }

  // ---- epilogue: lane (G, i) holds dX[m0 + 16 (FM wm + a) + i][n0 + 16 (FN wn + u) + 4 G + e],
  // re-dealt per subtile pair into 8 consecutive channels per lane (16-B stores)
  const int colw = n0 + 16 * FN * wn;
  // (narrow Cin: a wave whose 64 columns are all padding stores nothing; the split-K ticket
  // below is taken by the whole workgroup, so such a wave still joins it)
  const bool cols_live = colw < cp.Cin;
  if (cp.splits > 1) {   // split-K: raw fp32 partials; add / mask / bf16 in the reduction
#pragma unroll
    for (int a = 0; a < FM; ++a) {
      const int p = m0 + 16 * (FM * wm + a) + i;
      if (p < cp.T && cols_live) {
        float* dst = cp.part + ((size_t)sidx * cp.T + p) * cp.Cin + colw + 4 * G;
#pragma unroll
        for (int u = 0; u < FN; ++u) *reinterpret_cast<f32x4*>(dst + 16 * u) = acc[a][u];
      }
    }
    if (!cp.ticket || !split_last_arriver(cp.ticket, tile, cp.splits)) return;
    if (!cols_live) return;
#pragma unroll
    for (int a = 0; a < FM; ++a) {
      const int p = m0 + 16 * (FM * wm + a) + i;
      const float* src = cp.part + ((size_t)(p < cp.T ? p : 0)) * cp.Cin + colw + 4 * G;
#pragma unroll
      for (int u = 0; u < FN; ++u) {
        f32x4 tot = f32x4{0.f, 0.f, 0.f, 0.f};
        for (int q = 0; q < cp.splits; ++q)
          tot += q == sidx ? acc[a][u] : *reinterpret_cast<const f32x4*>(src + (size_t)q * cp.T * cp.Cin + 16 * u);
        acc[a][u] = tot;
      }
    }
  }
  if (!cols_live) return;
  float bz[FN][4];
#pragma unroll
  for (int u = 0; u < FN; ++u)
#pragma unroll
    for (int e = 0; e < 4; ++e) bz[u][e] = cp.bias ? bf2f(cp.bias[colw + 16 * u + 4 * G + e]) : 0.f;
#pragma unroll
  for (int a = 0; a < FM; ++a) {
    const int p = m0 + 16 * (FM * wm + a) + i;
    const size_t pr = (size_t)dx_row(cp, p < cp.T ? p : cp.T - 1) * cp.ldx;
    const size_t ar = cp.add_rows ? (size_t)(p < cp.T ? p : cp.T - 1) * cp.ldx : pr;
#pragma unroll
    for (int up = 0; up < FN / 2; ++up) {
      uint32_t c[2][2], ad[2][2], mk[2][2];
      if (cp.add) {
        const uint4 v = *reinterpret_cast<const uint4*>(cp.add + ar + colw + 32 * up + 8 * G);
        ad[0][0] = v.x; ad[0][1] = v.y; ad[1][0] = v.z; ad[1][1] = v.w;
        undeal(ad[0][0], ad[0][1], ad[1][0], ad[1][1]);
      }
      if (cp.mask) {
        const uint4 v = *reinterpret_cast<const uint4*>(cp.mask + pr + colw + 32 * up + 8 * G);
        mk[0][0] = v.x; mk[0][1] = v.y; mk[1][0] = v.z; mk[1][1] = v.w;
        undeal(mk[0][0], mk[0][1], mk[1][0], mk[1][1]);
      }
#pragma unroll
      for (int hlf = 0; hlf < 2; ++hlf) {
        const int u = 2 * up + hlf;
        float v[4] = {acc[a][u][0] + bz[u][0], acc[a][u][1] + bz[u][1], acc[a][u][2] + bz[u][2],
                      acc[a][u][3] + bz[u][3]};
        if (cp.add) {
          v[0] += lo_bf(ad[hlf][0]); v[1] += hi_bf(ad[hlf][0]);
          v[2] += lo_bf(ad[hlf][1]); v[3] += hi_bf(ad[hlf][1]);
        }
        if (cp.relu) {
#pragma unroll
          for (int e = 0; e < 4; ++e) v[e] = fmaxf(v[e], 0.f);
        }
        if (cp.mask) {
          v[0] = lo_bf(mk[hlf][0]) > 0.f ? v[0] : 0.f; v[1] = hi_bf(mk[hlf][0]) > 0.f ? v[1] : 0.f;
          v[2] = lo_bf(mk[hlf][1]) > 0.f ? v[2] : 0.f; v[3] = hi_bf(mk[hlf][1]) > 0.f ? v[3] : 0.f;
        }
        c[hlf][0] = pack2(v[0], v[1]);
        c[hlf][1] = pack2(v[2], v[3]);
      }
      deal(c[0][0], c[0][1], c[1][0], c[1][1]);
      if (p < cp.T)
        *reinterpret_cast<uint4*>(cp.dx + pr + colw + 32 * up + 8 * G) = make_uint4(c[0][0], c[0][1], c[1][0], c[1][1]);
    }
  }
}

// Split-K reduction: one thread per (tile, accumulator register group, lane) float4 column,
// summed over the slices in slice order (deterministic), written to dW with the main
// kernel's epilogue mapping (4 waves of 64 x 64: WM = WN = 2, FM = FN = 4).
__device__ __forceinline__ void wgrad_reduce_one(const float* slab, uint16_t* dw, int ntiles, int splits,
                                                 int tiles_tap, int tiles_n, int taps, int Cin, int Cout,
                                                 float beta, int gid) {
  constexpr int FM = 4, FN = 4, WN = 2, NR = FM * FN, NT = kNT;
  const int tid = gid % NT, rg = (gid / NT) % NR, t = gid / (NT * NR);   // gid < ntiles * NR * NT
  if (t >= ntiles) return;
  const float4* src = reinterpret_cast<const float4*>(slab) + ((size_t)t * splits * NR + rg) * NT + tid;
  float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
  int q = 0;
  for (; q + 4 <= splits; q += 4) {
    const float4 a0 = src[(size_t)(q + 0) * NR * NT], a1 = src[(size_t)(q + 1) * NR * NT];
    const float4 a2 = src[(size_t)(q + 2) * NR * NT], a3 = src[(size_t)(q + 3) * NR * NT];
    v.x += a0.x; v.y += a0.y; v.z += a0.z; v.w += a0.w;
    v.x += a1.x; v.y += a1.y; v.z += a1.z; v.w += a1.w;
    v.x += a2.x; v.y += a2.y; v.z += a2.z; v.w += a2.w;
    v.x += a3.x; v.y += a3.y; v.z += a3.z; v.w += a3.w;
  }
  for (; q < splits; ++q) {
    const float4 a0 = src[(size_t)q * NR * NT];
    v.x += a0.x; v.y += a0.y; v.z += a0.z; v.w += a0.w;
  }
  const int tap = t / tiles_tap, lt = t - tap * tiles_tap;
  const int m0 = (lt / tiles_n) * kBM, n0 = (lt % tiles_n) * kBN;
  const int lane = tid & 63, wave = tid >> 6, G = lane >> 4, i = lane & 15;
  const int wm = wave / WN, wn = wave % WN, a = rg / FN, u = rg % FN;
  const size_t ldc = (size_t)taps * Cin;
  uint16_t* C = dw + (size_t)(m0 + 16 * FM * wm + 4 * G + 16 * a) * ldc + (size_t)tap * Cin + n0 +
                16 * FN * wn + 16 * u + i;
  const float e4[4] = {v.x, v.y, v.z, v.w};
  const int mrow = m0 + 16 * FM * wm + 4 * G + 16 * a;
  if (n0 + 16 * FN * wn + 16 * u + i >= Cin) return;   // (narrow Cin: padded columns)
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    if (mrow + e >= Cout) continue;
    float o = e4[e];
    if (beta != 0.f) o += beta * bf2f(C[(size_t)e * ldc]);
    C[(size_t)e * ldc] = f2bf(o);
  }
}

__global__ __launch_bounds__(64) void conv_wgrad_reduce_kernel(const ConvWg cp) {
  wgrad_reduce_one(cp.slab, cp.dw, cp.ntiles, cp.splits, cp.tiles_tap, cp.tiles_n, cp.taps, cp.Cin, cp.Cout,
                   cp.beta, blockIdx.x * 64 + threadIdx.x);
}

// The split-K reductions of up to kWgJobs weight gradients in ONE launch (the deferred
// reductions of a backward pass, ops/convwg.py): job j owns blocks b0[j] .. b0[j + 1] - 1.
// The job list travels by value (kernel arguments), so a captured launch replays it as is.
constexpr int kWgJobs = 40;
struct WgJob {
  const float* slab;
  uint16_t* dw;
  int ntiles, splits, tiles_tap, tiles_n, taps, Cin, Cout, b0;
  float beta;
};
struct WgJobs {
  WgJob j[kWgJobs];
};
__global__ __launch_bounds__(64) void conv_wgrad_reduce_batched_kernel(const WgJobs js, int njobs) {
  const int b = blockIdx.x;
  int q = 0;
  while (q + 1 < njobs && js.j[q + 1].b0 <= b) ++q;   // (wave-uniform)
  const WgJob& J = js.j[q];
  wgrad_reduce_one(J.slab, J.dw, J.ntiles, J.splits, J.tiles_tap, J.tiles_n, J.taps, J.Cin, J.Cout, J.beta,
                   (b - J.b0) * 64 + threadIdx.x);
}

}  // namespace

// Tile geometry for the host planner: what = 0 -> BM, 1 -> BN, 2 -> BK (pixel rows per K-step).
MX_EXPORT int mx_conv_wgrad_tile(int what) { return what == 0 ? kBM : what == 1 ? kBN : kBK; }

// d (int64[20]): {dy, x, zero, dw, slab, 0, ldy, ldx, N, OH, OW, IH, IW, KH, KW, stride,
// pad, dil, Cout, Cin}.  Cout a multiple of 128 (or 8: narrow), Cin of 64; dy / x / zero 16-B aligned with
// ldy / ldx multiples of 8; dW is written (beta 0) or accumulated (beta 1) in bf16.
// splits > 1 needs slab (ntiles x splits x 128 x 128 fp32) and adds the reduction launch.
MX_EXPORT int mx_conv_wgrad(const int64_t* d, float beta, int splits, void* stream) {
  ConvWg cp{};
  cp.dy = reinterpret_cast<const uint16_t*>(d[0]);
  cp.x = reinterpret_cast<const uint16_t*>(d[1]);
  cp.zero = reinterpret_cast<const uint16_t*>(d[2]);
  cp.dw = reinterpret_cast<uint16_t*>(d[3]);
  cp.slab = reinterpret_cast<float*>(d[4]);
  cp.ldy = (int)d[6];
  cp.ldx = (int)d[7];
  const int64_t N = d[8];
  cp.OH = (int)d[9];
  cp.OW = (int)d[10];
  cp.IH = (int)d[11];
  cp.IW = (int)d[12];
  const int KH = (int)d[13];
  cp.KW = (int)d[14];
  cp.stride = (int)d[15];
  cp.pad = (int)d[16];
  cp.dil = (int)d[17];
  const int Cout = (int)d[18];
  cp.Cin = (int)d[19];
  const int64_t T = N * cp.OH * cp.OW;
  if (N <= 0 || cp.OH <= 0 || cp.OW <= 0 || KH <= 0 || cp.KW <= 0 || cp.stride <= 0 || cp.dil <= 0 ||
      cp.pad < 0 || T >= (1 << 23) || N * cp.IH * cp.IW >= ((int64_t)1 << 31))
    return (int)hipErrorInvalidValue;
  // Cout: a multiple of 128, or of 8 (the narrow 1x1 heads: 128-row tiles, zero-padded);
  // Cin: a multiple of 64 (an odd multiple: the last column tile half zero-padded)
  if ((Cout % kBM && Cout % 8) || cp.Cin % 64 || cp.ldy < Cout || cp.ldx < cp.Cin || (cp.ldy & 7) || (cp.ldx & 7))
    return (int)hipErrorInvalidValue;
  cp.Cout = Cout;
  if ((d[0] | d[1] | d[2]) & 15) return (int)hipErrorInvalidValue;
  if (splits < 1 || (splits > 1 && cp.slab == nullptr)) return (int)hipErrorInvalidValue;
  cp.T = (int)T;
  cp.taps = KH * cp.KW;
  const int64_t xbytes = N * cp.IH * cp.IW * (int64_t)cp.ldx * 2, ybytes = T * (int64_t)cp.ldy * 2;
  if (xbytes >= ((int64_t)1 << 31) || ybytes >= ((int64_t)1 << 31)) return (int)hipErrorInvalidValue;
  cp.xbytes = (uint32_t)xbytes;
  cp.ybytes = (uint32_t)ybytes;
  cp.tiles_n = (cp.Cin + kBN - 1) / kBN;
  cp.tiles_tap = ((Cout + kBM - 1) / kBM) * cp.tiles_n;
  cp.ntiles = cp.taps * cp.tiles_tap;
  const int steps = (int)((T + kBK - 1) / kBK);
  if (splits > steps) splits = steps;
  cp.nk = (steps + splits - 1) / splits;
  splits = (steps + cp.nk - 1) / cp.nk;   // no empty slice
  cp.splits = splits;
  cp.invOW = 1.f / (float)cp.OW;
  cp.invOH = 1.f / (float)cp.OH;
  cp.beta = beta;
  const bool defer = (d[5] & 1) != 0;   // the caller batches the split-K reduction (mx_conv_wgrad_reduce_batched)
  const bool ident = cp.taps == 1 && cp.stride == 1 && cp.pad == 0 && cp.OH == cp.IH && cp.OW == cp.IW;
  const dim3 grid(cp.ntiles * splits);
  hipStream_t st = (hipStream_t)stream;
  if (ident)
    hipLaunchKernelGGL((conv_wgrad_kernel<2, 2, 4, 4, kBK, 2, 2, true>), grid, dim3(kNT), 0, st, cp);
  else
    hipLaunchKernelGGL((conv_wgrad_kernel<2, 2, 4, 4, kBK, 2, 2, false>), grid, dim3(kNT), 0, st, cp);
  if (splits > 1 && !defer) {
    const int e = hipGetLastError();
    if (e) return e;
    hipLaunchKernelGGL(conv_wgrad_reduce_kernel, dim3(cp.ntiles * 16 * kNT / 64), dim3(64), 0, st, cp);
  }
  return (int)hipGetLastError();
}

// Deferred split-K reductions of several mx_conv_wgrad launches (flag bit 0 of d[5]): jobs =
// host int64 [njobs][10] {slab, dw, ntiles, splits, tiles_tap, tiles_n, taps, Cin, beta != 0, Cout},
// launched kWgJobs at a time.
MX_EXPORT int mx_conv_wgrad_reduce_batched(const int64_t* jobs, int njobs, void* stream) {
  hipStream_t st = (hipStream_t)stream;
  for (int j0 = 0; j0 < njobs; j0 += kWgJobs) {
    const int nj = njobs - j0 < kWgJobs ? njobs - j0 : kWgJobs;
    WgJobs js{};
    int blocks = 0;
    for (int q = 0; q < nj; ++q) {
      const int64_t* r = jobs + (size_t)(j0 + q) * 10;
      WgJob& J = js.j[q];
      J.slab = reinterpret_cast<const float*>(r[0]);
      J.dw = reinterpret_cast<uint16_t*>(r[1]);
      J.ntiles = (int)r[2]; J.splits = (int)r[3]; J.tiles_tap = (int)r[4]; J.tiles_n = (int)r[5];
      J.taps = (int)r[6]; J.Cin = (int)r[7]; J.beta = r[8] ? 1.f : 0.f; J.Cout = (int)r[9];
      if (J.splits < 2 || J.ntiles <= 0 || !J.slab || !J.dw) return (int)hipErrorInvalidValue;
      J.b0 = blocks;
      blocks += J.ntiles * 16 * kNT / 64;
    }
    hipLaunchKernelGGL(conv_wgrad_reduce_batched_kernel, dim3(blocks), dim3(64), 0, st, js, nj);
  }
  return (int)hipGetLastError();
}

// The split count the launch will really use (slices are never empty), for slab sizing.
MX_EXPORT int mx_conv_wgrad_splits(int64_t T, int splits) {
  const int steps = (int)((T + kBK - 1) / kBK);
  if (splits > steps) splits = steps;
  if (splits < 1) splits = 1;
  const int nk = (steps + splits - 1) / splits;
  return (steps + nk - 1) / nk;
}

// split-K input gradient: dX[p][c] = (sum_s part[s][p][c] (+ add)) * (mask > 0), splits in order
__global__ __launch_bounds__(256) void conv_dgrad_reduce_kernel(const ConvDg cp) {
  const int c8 = cp.Cin / 8;
  const int64_t nvec = (int64_t)cp.T * c8;
  for (int64_t v = (int64_t)blockIdx.x * 256 + threadIdx.x; v < nvec; v += (int64_t)gridDim.x * 256) {
    const int p = (int)(v / c8), c = (int)(v - (int64_t)p * c8) * 8;
    float o[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    for (int s2 = 0; s2 < cp.splits; ++s2) {
      const float4* q = reinterpret_cast<const float4*>(cp.part + ((size_t)s2 * cp.T + p) * cp.Cin + c);
      const float4 x0 = q[0], x1 = q[1];
      o[0] += x0.x; o[1] += x0.y; o[2] += x0.z; o[3] += x0.w;
      o[4] += x1.x; o[5] += x1.y; o[6] += x1.z; o[7] += x1.w;
    }
    const size_t off = (size_t)dx_row(cp, p) * cp.ldx + c;
    if (cp.bias) {
#pragma unroll
      for (int j = 0; j < 8; ++j) o[j] += bf2f(cp.bias[c + j]);
    }
    if (cp.add) {
      float a[8];
      unpack8(*reinterpret_cast<const uint4*>(cp.add + (cp.add_rows ? (size_t)p * cp.ldx + c : off)), a);
#pragma unroll
      for (int j = 0; j < 8; ++j) o[j] += a[j];
    }
    if (cp.relu) {
#pragma unroll
      for (int j = 0; j < 8; ++j) o[j] = fmaxf(o[j], 0.f);
    }
    if (cp.mask) {
      float m[8];
      unpack8(*reinterpret_cast<const uint4*>(cp.mask + off), m);
#pragma unroll
      for (int j = 0; j < 8; ++j) o[j] = m[j] > 0.f ? o[j] : 0.f;
    }
    *reinterpret_cast<uint4*>(cp.dx + off) = pack8(o);
  }
}

// Stride-decomposed dgrad, the pixels no tap reaches ((ih mod s, iw mod s) outside the
// filter, e.g. 3 of 4 pixels of a 1x1 stride-2 conv): the epilogue applied to a zero sum
// (an add holding only the filter's parity class contributes nothing here).
__global__ __launch_bounds__(256) void conv_dgrad_fill_kernel(const ConvDg cp, int KH) {
  const int c8 = cp.Cin / 8;
  const int64_t nvec = (int64_t)cp.T * c8;
  for (int64_t v = (int64_t)blockIdx.x * 256 + threadIdx.x; v < nvec; v += (int64_t)gridDim.x * 256) {
    const int p = (int)(v / c8), c = (int)(v - (int64_t)p * c8) * 8;
    const int iw = p % cp.IW, ih = (p / cp.IW) % cp.IH;
    if (ih % cp.stride < KH && iw % cp.stride < cp.KW) continue;
    float o[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    const size_t off = (size_t)p * cp.ldx + c;
    if (cp.bias) {
#pragma unroll
      for (int j = 0; j < 8; ++j) o[j] = bf2f(cp.bias[c + j]);
    }
    if (cp.add && !cp.add_rows) {
      float a[8];
      unpack8(*reinterpret_cast<const uint4*>(cp.add + off), a);
#pragma unroll
      for (int j = 0; j < 8; ++j) o[j] += a[j];
    }
    if (cp.relu) {
#pragma unroll
      for (int j = 0; j < 8; ++j) o[j] = fmaxf(o[j], 0.f);
    }
    if (cp.mask) {
      float m[8];
      unpack8(*reinterpret_cast<const uint4*>(cp.mask + off), m);
#pragma unroll
      for (int j = 0; j < 8; ++j) o[j] = m[j] > 0.f ? o[j] : 0.f;
    }
    *reinterpret_cast<uint4*>(cp.dx + off) = pack8(o);
  }
}

// input-gradient K-step depth: 0 -> 64, 1 -> 32, 2 -> by shape (mx_conv_dgrad, default).
// (A 4-slot ring of 32-deep steps was 2-11 % slower: profiles/r5_s1/conv_ab_ring_4.txt)
constexpr int g_conv_dgrad_bk32 = 2;

static void launch_dgrad(ConvDg cp, int splits, hipStream_t st) {
  cp.splits = splits < 1 ? 1 : (splits > cp.nk ? cp.nk : splits);
  const int tiles_m = (cp.T + 127) / 128;
  const dim3 grid(tiles_m * cp.tiles_n * cp.splits);
  if (cp.bkt == 32)
    hipLaunchKernelGGL((conv_dgrad_kernel<2, 32>), grid, dim3(256), 0, st, cp);
  else
    hipLaunchKernelGGL((conv_dgrad_kernel<2, 64>), grid, dim3(256), 0, st, cp);
  if (cp.splits > 1 && !cp.ticket) {
    const int64_t nvec = (int64_t)cp.T * (cp.Cin / 8);
    const unsigned rg = (unsigned)((nvec + 255) / 256 < 8192 ? (nvec + 255) / 256 : 8192);
    hipLaunchKernelGGL(conv_dgrad_reduce_kernel, dim3(rg), dim3(256), 0, st, cp);
  }
}

// d (int64[24]): {dy, w, zero, dx, add, mask, ldy, ldx, N, OH, OW, IH, IW, KH, KW, stride,
// pad, dil, Cout, Cin, splits, part, bias, flags}: dX of conv2d for the output gradient dY,
// weight [Cout][KH][KW][Cin] (channels_last), then (optional, null to skip) + bias[c] +
// add[p][c], max(., 0) (flags bit 0) and * (mask[p][c] > 0): X's second gradient (a residual
// branch) and X's own ReLU folded into the one store; bias + ReLU make it the forward of a
// transposed convolution.  flags bit 1: stride-decomposed (stride s > 1, no padding or
// dilation, filter <= s x s): one launch per parity class (ih mod s, iw mod s) = (a, b), whose
// pixels all take the single tap (a, b) from dY[ih / s][iw / s] -- a plain GEMM over a
// quarter of the pixels instead of the gathered K loop whose rows are 3 of 4 zero -- and one
// fill of the pixels no tap reaches.  Cout a multiple of 8, Cin of 64; 16-B aligned
// operands (add / mask share dX's layout); splits > 1 needs part (fp32, splits x pixels x Cin).
MX_EXPORT int mx_conv_dgrad(const int64_t* d, void* stream) {
  ConvDg cp{};
  cp.dy = reinterpret_cast<const uint16_t*>(d[0]);
  cp.w = reinterpret_cast<const uint16_t*>(d[1]);
  cp.zero = reinterpret_cast<const uint16_t*>(d[2]);
  cp.dx = reinterpret_cast<uint16_t*>(d[3]);
  cp.add = reinterpret_cast<const uint16_t*>(d[4]);
  cp.mask = reinterpret_cast<const uint16_t*>(d[5]);
  cp.ldy = (int)d[6];
  cp.ldx = (int)d[7];
  const int64_t N = d[8];
  cp.OH = (int)d[9];
  cp.OW = (int)d[10];
  cp.IH = (int)d[11];
  cp.IW = (int)d[12];
  const int KH = (int)d[13];
  cp.KW = (int)d[14];
  cp.stride = (int)d[15];
  cp.pad = (int)d[16];
  cp.dil = (int)d[17];
  const int Cout = (int)d[18];
  cp.Cin = (int)d[19];
  const int64_t T = N * cp.IH * cp.IW;
  if (N <= 0 || cp.IH <= 0 || cp.IW <= 0 || cp.OH <= 0 || cp.OW <= 0 || KH <= 0 || cp.KW <= 0 || cp.stride <= 0 ||
      cp.dil <= 0 || cp.pad < 0 || T >= (1 << 23) || N * cp.OH * cp.OW >= ((int64_t)1 << 31))
    return (int)hipErrorInvalidValue;
  if (Cout % 8 || cp.Cin % 64 || cp.ldy < Cout || cp.ldx < cp.Cin || (cp.ldy & 7) || (cp.ldx & 7))
    return (int)hipErrorInvalidValue;
  if ((d[0] | d[1] | d[2] | d[3] | d[4] | d[5]) & 15) return (int)hipErrorInvalidValue;
  cp.T = (int)T;
  cp.taps = KH * cp.KW;
  const int64_t ybytes = N * cp.OH * cp.OW * (int64_t)cp.ldy * 2;
  if (cp.taps > 32 || ybytes >= ((int64_t)1 << 31)) return (int)hipErrorInvalidValue;
  cp.ybytes = (uint32_t)ybytes;
  cp.ldw = cp.taps * cp.Cin;
  // K-step depth (mx_conv_dgrad_bk32): 32 for the narrow reductions -- 3x3 with Cout <= 128,
  // 1x1 with Cout <= 512 -- where scripts/conv_ab.py measured the 16-KiB slots 16-20 % faster
  // (res3.conv2, res3.conv3, fpn.lat2 at 4 images); the 3x3 Cout 256 convs and res4.conv3
  // (1x1, Cout 1024) are 3-23 % slower with them (profiles/r5_s1/conv_ab_ring_3.txt)
  const bool narrow = Cout <= 128 || (cp.taps == 1 && Cout <= 512);
  cp.bkt = (g_conv_dgrad_bk32 == 1 || (g_conv_dgrad_bk32 == 2 && narrow)) ? 32 : 64;
  cp.cob = (Cout + cp.bkt - 1) / cp.bkt;
  cp.Cout = Cout;
  cp.nk = cp.taps * cp.cob;
  cp.tiles_n = (cp.Cin + 127) / 128;   // (Cin % 128 == 64: the last column tile half padded)
  cp.invIW = 1.f / (float)cp.IW;
  cp.invIH = 1.f / (float)cp.IH;
  cp.bias = reinterpret_cast<const uint16_t*>(d[22]);
  cp.relu = (int)(d[23] & 1);
  cp.ticket = reinterpret_cast<uint32_t*>(d[24]);   // (d has >= 25 entries: ops/convwg.py _DESC_T)
  const bool decomp = (d[23] >> 1) & 1;
  const int splits = d[20] > 1 ? (int)d[20] : 1;
  cp.part = reinterpret_cast<float*>(d[21]);
  if (splits > 1 && (!cp.part || (d[21] & 15))) return (int)hipErrorInvalidValue;
  if (d[22] & 7) return (int)hipErrorInvalidValue;
  const hipStream_t st = (hipStream_t)stream;
  if (!decomp) {
    launch_dgrad(cp, splits, st);
    return (int)hipGetLastError();
  }
  const int s = cp.stride;
  if (s < 2 || cp.pad || cp.dil != 1 || KH > s || cp.KW > s) return (int)hipErrorInvalidValue;
  // flags bit 2 (class_out): a 1 x 1 filter's only parity class (0, 0) written compact as
  // [N][ceil(IH / s)][ceil(IW / s)][ldx] -- no zero fill of the other s^2 - 1 classes (the
  // ResNet projection shortcut's parked dX, ops/epilogue.py); bit 3 (add_class): ``add`` is
  // such a compact class tensor, added to the class pixels only
  const bool class_out = (d[23] >> 2) & 1, add_class = (d[23] >> 3) & 1;
  if ((class_out || add_class) && (KH != 1 || cp.KW != 1)) return (int)hipErrorInvalidValue;
  if (class_out && (cp.add || cp.mask || cp.bias || cp.relu)) return (int)hipErrorInvalidValue;
  if (add_class && !cp.add) return (int)hipErrorInvalidValue;
  cp.add_rows = add_class ? 1 : 0;
  if (class_out) {
    ConvDg c = cp;
    c.IH = (cp.IH + s - 1) / s;
    c.IW = (cp.IW + s - 1) / s;
    c.T = (int)(N * c.IH * c.IW);
    c.invIW = 1.f / (float)c.IW;
    c.invIH = 1.f / (float)c.IH;
    c.stride = 1; c.taps = 1; c.nk = cp.cob;   // (xs = 0: dX rows are the launch's pixels)
    launch_dgrad(c, splits, st);
    return (int)hipGetLastError();
  }
  for (int a = 0; a < KH; ++a)
    for (int b = 0; b < cp.KW; ++b) {
      ConvDg c = cp;
      c.xs = s; c.xa = a; c.xb = b; c.XH = cp.IH; c.XW = cp.IW;
      c.IH = (cp.IH - a + s - 1) / s;
      c.IW = (cp.IW - b + s - 1) / s;
      c.T = (int)(N * c.IH * c.IW);
      c.invIW = 1.f / (float)c.IW;
      c.invIH = 1.f / (float)c.IH;
      c.stride = 1; c.KW = 1; c.taps = 1; c.nk = cp.cob;
      c.w = cp.w + (size_t)(a * cp.KW + b) * cp.Cin;   // tap (a, b); rows keep the pitch ldw
      launch_dgrad(c, splits, st);
    }
  if (KH < s || cp.KW < s) {
    const int64_t nvec = T * (cp.Cin / 8);
    const unsigned rg = (unsigned)((nvec + 255) / 256 < 16384 ? (nvec + 255) / 256 : 16384);
    hipLaunchKernelGGL(conv_dgrad_fill_kernel, dim3(rg), dim3(256), 0, st, cp, KH);
  }
  return (int)hipGetLastError();
}

// d (int64[27]): {x, w, zero, y, bias, res, ldx, ldy, N, OH, OW, IH, IW, KH, KW, stride, pad,
// dil, Cout, Cin, relu, res_up, splits, part, ticket, half, bnp}: y = act(conv2d(x, w) + bias (+ res, or with res_up the 2x
// nearest upsampling of res)) in NHWC bf16, weight [Cout][KH][KW][Cin] (channels_last).
// Cout a multiple of 64 (128 x 64 tiles when not of 128), Cin of 64; res_up needs even OH, OW.
MX_EXPORT int mx_conv_fwd(const int64_t* d, void* stream) {
  ConvFw cp{};
  cp.x = reinterpret_cast<const uint16_t*>(d[0]);
  cp.w = reinterpret_cast<const uint16_t*>(d[1]);
  cp.zero = reinterpret_cast<const uint16_t*>(d[2]);
  cp.y = reinterpret_cast<uint16_t*>(d[3]);
  cp.bias = reinterpret_cast<const uint16_t*>(d[4]);
  cp.res = reinterpret_cast<const uint16_t*>(d[5]);
  cp.ldx = (int)d[6];
  cp.ldy = (int)d[7];
  const int64_t N = d[8];
  cp.OH = (int)d[9];
  cp.OW = (int)d[10];
  cp.IH = (int)d[11];
  cp.IW = (int)d[12];
  const int KH = (int)d[13];
  cp.KW = (int)d[14];
  cp.stride = (int)d[15];
  cp.pad = (int)d[16];
  cp.dil = (int)d[17];
  const int Cout = (int)d[18];
  cp.Cin = (int)d[19];
  const bool relu = d[20] != 0;
  cp.res_up = cp.res && d[21] != 0;
  cp.splits = d[22] > 1 ? (int)d[22] : 1;
  cp.part = reinterpret_cast<float*>(d[23]);
  cp.ticket = reinterpret_cast<uint32_t*>(d[24]);
  cp.Cout = (int)d[18];
  cp.bnp = reinterpret_cast<float*>(d[26]);
  const int64_t T = N * cp.OH * cp.OW;
  if (cp.res_up && ((cp.OH | cp.OW) & 1)) return (int)hipErrorInvalidValue;
  if (N <= 0 || cp.IH <= 0 || cp.IW <= 0 || cp.OH <= 0 || cp.OW <= 0 || KH <= 0 || cp.KW <= 0 || cp.stride <= 0 ||
      cp.dil <= 0 || cp.pad < 0 || T >= (1 << 23) || N * cp.IH * cp.IW >= ((int64_t)1 << 31))
    return (int)hipErrorInvalidValue;
  if (Cout % 8 || cp.Cin % 64 || cp.ldx < cp.Cin || cp.ldy < Cout || (cp.ldx & 7) || (cp.ldy & 7))
    return (int)hipErrorInvalidValue;
  if ((d[0] | d[1] | d[2]) & 15) return (int)hipErrorInvalidValue;
  cp.T = (int)T;
  cp.taps = KH * cp.KW;
  const int64_t xbytes = N * cp.IH * cp.IW * (int64_t)cp.ldx * 2;
  if (cp.taps > 32 || xbytes >= ((int64_t)1 << 31)) return (int)hipErrorInvalidValue;
  cp.xbytes = (uint32_t)xbytes;
  // (32-deep steps in a 4-slot ring -- three in flight -- measured 4-5 % slower overall,
  // profiles/r5_s1/conv_ab_ring_1.txt)
  const bool bk32 = g_conv_fwd_bk32 == 1 || (g_conv_fwd_bk32 == 2 && (cp.taps == 1 || cp.Cin <= 128));
  const int bkt = bk32 && cp.Cin % 32 == 0 ? 32 : 64;
  cp.cib = cp.Cin / bkt;
  cp.nk = cp.taps * cp.cib;
  // d[25] != 0: 128 x 64 tiles even when Cout is a multiple of 128 (twice the tiles for a small
  // convolution instead of a deeper K split: no fp32 partial round trip)
  const bool half = d[25] != 0 && Cout % 64 == 0;
  cp.tiles_n = Cout % 128 == 0 && !half ? Cout / 128 : (Cout + 63) / 64;   // (narrow Cout: zero-padded tiles)
  if (Cout % 64 && cp.splits > 1) return (int)hipErrorInvalidValue;   // partial planes assume whole tiles
  cp.invOW = 1.f / (float)cp.OW;
  cp.invOH = 1.f / (float)cp.OH;
  if (cp.splits > cp.nk) cp.splits = cp.nk;
  if (cp.splits > 1 && (!cp.part || (d[23] & 15))) return (int)hipErrorInvalidValue;
  if (cp.bnp && (cp.splits > 1 || Cout % 64 || (d[26] & 3))) return (int)hipErrorInvalidValue;
  hipStream_t st = (hipStream_t)stream;
  const dim3 grid((unsigned)((T + 127) / 128) * cp.tiles_n * cp.splits), block(256);
#define MX_CF(NS, FN, BK)                                                                     \
  if (cp.res) {                                                                               \
    if (relu) hipLaunchKernelGGL((conv_fwd_kernel<NS, FN, true, true, BK>), grid, block, 0, st, cp);   \
    else hipLaunchKernelGGL((conv_fwd_kernel<NS, FN, true, false, BK>), grid, block, 0, st, cp);       \
  } else {                                                                                    \
    if (relu) hipLaunchKernelGGL((conv_fwd_kernel<NS, FN, false, true, BK>), grid, block, 0, st, cp);  \
    else hipLaunchKernelGGL((conv_fwd_kernel<NS, FN, false, false, BK>), grid, block, 0, st, cp);      \
  }
  // ring depth 2 at two workgroups per CU: 3 / 4 slots (one workgroup per CU, counted waits)
  // measured 40 % slower on the Mask R-CNN shapes (profiles/r4_s2/conv_ring_depth_ab_4img.txt)
  if (bkt == 32) {
    if (Cout % 128 == 0 && !half) { MX_CF(2, 4, 32) } else { MX_CF(2, 2, 32) }
  } else {
    if (Cout % 128 == 0 && !half) { MX_CF(2, 4, 64) } else { MX_CF(2, 2, 64) }
  }
#undef MX_CF
  if (cp.splits > 1 && !cp.ticket) {
    const int64_t nvec = T * (Cout / 8);
    const unsigned rg = (unsigned)((nvec + 255) / 256 < 8192 ? (nvec + 255) / 256 : 8192);
    if (cp.res) {
      if (relu) hipLaunchKernelGGL((conv_fwd_reduce_kernel<true, true>), dim3(rg), block, 0, st, cp);
      else hipLaunchKernelGGL((conv_fwd_reduce_kernel<true, false>), dim3(rg), block, 0, st, cp);
    } else {
      if (relu) hipLaunchKernelGGL((conv_fwd_reduce_kernel<false, true>), dim3(rg), block, 0, st, cp);
      else hipLaunchKernelGGL((conv_fwd_reduce_kernel<false, false>), dim3(rg), block, 0, st, cp);
    }
  }
  return (int)hipGetLastError();
}

