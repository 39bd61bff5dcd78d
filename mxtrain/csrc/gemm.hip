// Weight-gradient GEMMs for gfx950: C[M][N] (+)= sum_k A[k][m] * B[k][n], bf16 in, fp32
// accumulate, bf16 out -- dW = dY^T X for every Linear of a transformer layer, with dY
// [tokens, out] and X [tokens, in] read in place (both operands are stored K-major, the
// reduction runs over the token rows).
//
// Why a hand-written kernel: these GEMMs have a small output (1024 x 1024 ... 4096 x 1024)
// and a long K (all tokens of the micro-batch).  hipBLASLt's picks for them ran at
// 0.27-0.73 PF/s on one MI355X (mxtrain/tuning/tunableop_gpt2_345m_gfx950.csv: nt_1024_1024_4096
// 31.8 us, nt_1024_3072_4096 45.9 us, nt_4096_1024_4096 47.0 us), the weakest GEMM family of
// the GPT step (reference: Megatron's `LinearWithGradAccumulation` wgrad
// GEMMs, containers/megatron-deepspeed/Dockerfile:13).
//
// Design (cdna_hip_programming.md §5):
//  * grouped launch: up to 4 problems with a common K (the layer's wgrads that become ready
//    together: fc1+fc2, qkv+proj) share one grid, so a 1024 x 1024 output does not leave the
//    chip idle and no split-K slab round trip is needed;
//  * 128 x 128 output tile per 4-wave workgroup (2 x 2 waves of 64 x 64), BK = 64, two
//    workgroups per CU; 16 x 16 x 32 bf16 MFMA, 4 x 4 accumulators per wave;
//  * operands staged by LDS-DMA (global_load_lds_dwordx4: 1 KiB = 4 k-rows per wave
//    instruction, no staging registers) into a 2-slot ring, one barrier per K-step;
//  * both operands are K-major, so MFMA fragments (8 consecutive k of one m) come from
//    ds_read_b64_tr_b16 transposed reads of the [k][m] image;  the image's 16-B chunks are
//    XOR-swizzled by (k & 3, k >> 3 & 1) on the DMA SOURCE address (the LDS write stays
//    lane-linear), which spreads the 16 row segments of one transposed read over all 8
//    32-B slots of a bank row (2 cycles, the minimum for 512 B);
//  * XCD-aware tile order (xcd_remap): tiles of one XCD are contiguous in (m, n), so they
//    share their A and B k-row panels in that XCD's L2;
//  * beta in {0, 1}: beta = 0 writes the gradient (no zero-fill of the gradient buffer),
//    beta = 1 accumulates (micro-batches 2..n).
#include "gemm_common.h"

#include <type_traits>

using namespace mx;
using namespace mx::gemm;

namespace {

constexpr int MAXP = 4;

struct Prob {
  const uint16_t* a;
  const uint16_t* b;
  uint16_t* c;
  int lda, ldb, ldc;
  int tiles_n, tile0;
};
struct Batch {
  Prob p[MAXP];
  int np, K, splits, ntiles;
  float beta;
  float* slab;          // split-K partials: [ntiles][splits][NT / 64][acc regs / 4][64] float4
  uint32_t* ticket;     // [ntiles], zero between launches (the last arriver resets its word)
  int prio;             // 8-wave tiles, bit 0: s_setprio 1 for waves 4-7; bit 1: their half-step stagger
};

// as gemm_nt.hip g_gemm_nt_prio (MI355X_MICROARCH.md "Two waves per SIMD", items 4 and 9)
constexpr int g_gemm_kk_prio = 3;

__device__ __forceinline__ Prob pick(const Batch& bt, int t) {
  // constant indices only: a runtime index into the by-value kernel argument would copy it
  // to scratch
  Prob P = bt.p[0];
  if (bt.np > 1 && t >= bt.p[1].tile0) P = bt.p[1];
  if (bt.np > 2 && t >= bt.p[2].tile0) P = bt.p[2];
  if (bt.np > 3 && t >= bt.p[3].tile0) P = bt.p[3];
  return P;
}

// WM x WN waves, each FM x FN 16 x 16 accumulator tiles; BKT-deep K-steps through an
// NSLOT-slot LDS ring (NSLOT - 1 K-steps in flight)
template <int WM, int WN, int FM, int FN, int BKT, int NSLOT>
struct Cfg {
  static constexpr int NW = WM * WN, NT = 64 * NW;
  static constexpr int BM = 16 * FM * WM, BN = 16 * FN * WN;
  static constexpr int RA = BM * 2, RB = BN * 2;          // image row bytes
  static constexpr int IA = BKT * RA, IB = BKT * RB;      // image bytes
  static constexpr int PA = IA / 1024 / NW, PB = IB / 1024 / NW;   // DMA pieces per wave
  static constexpr int SLOT = IA + IB, LDS = NSLOT * SLOT;
  static_assert(PA * NW * 1024 == IA && PB * NW * 1024 == IB, "DMA pieces per wave");
  static_assert(BKT % 32 == 0 && RA >= 256 && RB >= 256, "tile");
};

template <int WM, int WN, int FM, int FN, int BKT, int NSLOT, int MINB>
__global__ __launch_bounds__(64 * WM * WN, MINB) void gemm_kk_kernel(const Batch bt) {
  using C_ = Cfg<WM, WN, FM, FN, BKT, NSLOT>;
  constexpr int BM = C_::BM, BN = C_::BN, RA = C_::RA, RB = C_::RB, IA = C_::IA;
  constexpr int PA = C_::PA, PB = C_::PB, SLOT = C_::SLOT, NT = C_::NT;
  constexpr int PER = PA + PB;   // DMA instructions per wave per K-step
  __shared__ __attribute__((aligned(1024))) char smem[C_::LDS];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wg = xcd_remap(blockIdx.x, gridDim.x);
  // split-K slices of one tile are adjacent ids (same XCD under the remap)
  const int t = wg / bt.splits, slice = wg - t * bt.splits;
  const Prob P = pick(bt, t);
  const int lt = t - P.tile0;
  const int m0 = (lt / P.tiles_n) * BM, n0 = (lt % P.tiles_n) * BN;
  const int nk = bt.K / BKT / bt.splits;          // K-steps of this slice
  const int k0 = slice * nk * BKT;

  // ---- LDS-DMA sources: a 1-KiB piece holds 1024 / R consecutive k-rows of an image; wave w
  // fills A pieces PA w .. PA w + PA - 1 and B pieces PB w ..
  const uint16_t* srcA[PA];
  const uint16_t* srcB[PB];
  {
    constexpr int CA = RA / 16, CB = RB / 16;     // chunks per row
#pragma unroll
    for (int j = 0; j < PA; ++j) {
      const int k = (PA * wave + j) * (1024 / RA) + lane / CA;
      srcA[j] = P.a + (size_t)(k0 + k) * P.lda + m0 + 8 * pchunk(k, lane % CA);
    }
#pragma unroll
    for (int j = 0; j < PB; ++j) {
      const int k = (PB * wave + j) * (1024 / RB) + lane / CB;
      srcB[j] = P.b + (size_t)(k0 + k) * P.ldb + n0 + 8 * pchunk(k, lane % CB);
    }
  }
  const size_t stepA = (size_t)BKT * P.lda, stepB = (size_t)BKT * P.ldb;

  // ---- transposed-read offsets: lane (G, i) reads k-row 8G + (i>>2) (+32 kk + 4 h), columns
  // 4 (i&3) .. +3 of the 16-column subtile s; the swizzle term depends on (i>>2, G&1) only
  const int G = lane >> 4, i = lane & 15;
  const int wm = wave / WN, wn = wave % WN;
  const int krow = 8 * G + (i >> 2);
  const int g = gsw(krow);
  int offA[FM], offB[FN];
#pragma unroll
  for (int s = 0; s < FM; ++s)
    offA[s] = krow * RA + ((((FM * wm + s) ^ g) << 1) | ((i & 3) >> 1)) * 16 + (i & 1) * 8;
#pragma unroll
  for (int u = 0; u < FN; ++u)
    offB[u] = krow * RB + ((((FN * wn + u) ^ g) << 1) | ((i & 3) >> 1)) * 16 + (i & 1) * 8;

  f32x4 acc[FM][FN];
#pragma unroll
  for (int s = 0; s < FM; ++s)
#pragma unroll
    for (int u = 0; u < FN; ++u) acc[s][u] = f32x4{0.f, 0.f, 0.f, 0.f};

  const uint32_t lds0 = lds_addr(smem);
  auto issue = [&](int slot, int it) __attribute__((always_inline)) {
    const uint32_t b0 = __builtin_amdgcn_readfirstlane(lds0 + slot * SLOT + PA * wave * 1024);
    const uint32_t b1 = __builtin_amdgcn_readfirstlane(lds0 + slot * SLOT + IA + PB * wave * 1024);
#pragma unroll
    for (int j = 0; j < PA; ++j) dma16(srcA[j] + it * stepA, b0 + j * 1024);
#pragma unroll
    for (int j = 0; j < PB; ++j) dma16(srcB[j] + it * stepB, b1 + j * 1024);
  };

#pragma unroll
  for (int q = 0; q < NSLOT - 1; ++q)
    if (q < nk) issue(q, q);
  // stagger (bt.prio bit 1): waves 4-7 read all of step it's fragments before the barrier that
  // frees its slot but run only the first half of its (kk, s) MFMA groups there; the rest runs
  // from registers after the next barrier, beside the partner wave's LDS read burst.  Same
  // MFMAs per accumulator in the same order: bit-identical output.
  constexpr int KK = BKT / 32, NQ = KK * FM, NH1 = NQ / 2;
  const bool stag = C_::NW == 8 && (bt.prio & 2) && wave >= 4;
  if (C_::NW == 8 && (bt.prio & 1) && wave >= 4) __builtin_amdgcn_s_setprio(1);
  bf16x8 sa[NQ], sb[KK][FN];
  bool pend = false;
  auto run_h2 = [&]() __attribute__((always_inline)) {
#pragma unroll
    for (int p = NH1; p < NQ; ++p)
#pragma unroll
      for (int u = 0; u < FN; ++u) acc[p % FM][u] = mfma16(sa[p], sb[p / FM][u], acc[p % FM][u]);
  };
  int slot = 0;
  for (int it = 0; it < nk; ++it) {
    // retire step it's pieces (the later steps' stay in flight), then one barrier: every
    // wave's pieces of step it have landed and every wave is done reading step it - 1's slot
    const int later = nk - 1 - it;
    if (NSLOT >= 5 && later >= 3) vm_wait<(NSLOT >= 5 ? 3 : 0) * PER>();
    else if (NSLOT >= 4 && later >= 2) vm_wait<(NSLOT >= 4 ? 2 : 0) * PER>();
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
    if (stag) {
      if (pend) run_h2();
#pragma unroll
      for (int kk = 0; kk < KK; ++kk)
#pragma unroll
        for (int u = 0; u < FN; ++u)
          sb[kk][u] = cat(tr_read(Bs, offB[u] + 32 * RB * kk), tr_read(Bs, offB[u] + 32 * RB * kk + 4 * RB));
#pragma unroll
      for (int p = 0; p < NQ; ++p) {
        const int kk = p / FM, s2 = p % FM;
        sa[p] = cat(tr_read(As, offA[s2] + 32 * RA * kk), tr_read(As, offA[s2] + 32 * RA * kk + 4 * RA));
        if (p < NH1) {
#pragma unroll
          for (int u = 0; u < FN; ++u) acc[s2][u] = mfma16(sa[p], sb[kk][u], acc[s2][u]);
        }
      }
      pend = true;
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");   // the slot is freed at the next barrier
      if (++slot == NSLOT) slot = 0;
      continue;
    }
#pragma unroll
    for (int kk = 0; kk < BKT / 32; ++kk) {
      bf16x8 b[FN];
#pragma unroll
      for (int u = 0; u < FN; ++u)
        b[u] = cat(tr_read(Bs, offB[u] + 32 * RB * kk), tr_read(Bs, offB[u] + 32 * RB * kk + 4 * RB));
#pragma unroll
      for (int s = 0; s < FM; ++s) {
        const bf16x8 a = cat(tr_read(As, offA[s] + 32 * RA * kk), tr_read(As, offA[s] + 32 * RA * kk + 4 * RA));
#pragma unroll
        for (int u = 0; u < FN; ++u) acc[s][u] = mfma16(a, b[u], acc[s][u]);
      }
    }
    if (++slot == NSLOT) slot = 0;
  }
  if (stag && pend) run_h2();

  // ---- split-K: every slice publishes its partial tile; the last arriver sums them
  if (bt.splits > 1) {
    __shared__ uint32_t last_flag;
    constexpr int NR = FM * FN;                      // float4 registers per lane
    float4* mine = reinterpret_cast<float4*>(bt.slab) + ((size_t)(t * bt.splits + slice) * NR) * NT + tid;
#pragma unroll
    for (int s = 0; s < FM; ++s)
#pragma unroll
      for (int u = 0; u < FN; ++u)
        mine[(s * FN + u) * NT] = make_float4(acc[s][u][0], acc[s][u][1], acc[s][u][2], acc[s][u][3]);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (tid == 0) {
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      const uint32_t prev = __hip_atomic_fetch_add(bt.ticket + t, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      const uint32_t is_last = prev == (uint32_t)(bt.splits - 1);
      if (is_last) {
        __hip_atomic_store(bt.ticket + t, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      }
      last_flag = is_last;
    }
    __syncthreads();
    if (!last_flag) return;
    const float4* base = reinterpret_cast<const float4*>(bt.slab) + ((size_t)t * bt.splits * NR) * NT + tid;
    for (int q = 0; q < bt.splits; ++q) {
      if (q == slice) continue;
#pragma unroll
      for (int s = 0; s < FM; ++s)
#pragma unroll
        for (int u = 0; u < FN; ++u) {
          const float4 v = base[((size_t)q * NR + s * FN + u) * NT];
          acc[s][u][0] += v.x; acc[s][u][1] += v.y; acc[s][u][2] += v.z; acc[s][u][3] += v.w;
        }
    }
  }

  // ---- epilogue: lane holds C[16 s + 4 G + e][16 u + i] of its wave's block
  uint16_t* C = P.c + (size_t)(m0 + 16 * FM * wm + 4 * G) * P.ldc + n0 + 16 * FN * wn + i;
  const bool acc_in = bt.beta != 0.f;
#pragma unroll
  for (int s = 0; s < FM; ++s)
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      uint16_t* row = C + (size_t)(16 * s + e) * P.ldc;
#pragma unroll
      for (int u = 0; u < FN; ++u) {
        float v = acc[s][u][e];
        if (acc_in) v += bt.beta * bf2f(row[16 * u]);
        row[16 * u] = f2bf(v);
      }
    }
}

template <int WM, int WN, int FM, int FN, int BKT, int NSLOT, int MINB>
int launch(const int64_t* desc, int np, int K, float beta, int splits, float* slab, uint32_t* ticket,
           hipStream_t stream) {
  using C_ = Cfg<WM, WN, FM, FN, BKT, NSLOT>;
  if (K % (BKT * splits)) return (int)hipErrorInvalidValue;
  Batch bt{};
  bt.np = np;
  bt.K = K;
  bt.beta = beta;
  bt.splits = splits;
  bt.slab = slab;
  bt.ticket = ticket;
  bt.prio = g_gemm_kk_prio;
  int total = 0;
  for (int q = 0; q < np; ++q) {
    const int64_t* d = desc + 8 * q;
    const int M = (int)d[6], N = (int)d[7];
    if (M <= 0 || N <= 0 || M % C_::BM || N % C_::BN) return (int)hipErrorInvalidValue;
    Prob& p = bt.p[q];
    p.a = reinterpret_cast<const uint16_t*>(d[0]);
    p.b = reinterpret_cast<const uint16_t*>(d[1]);
    p.c = reinterpret_cast<uint16_t*>(d[2]);
    p.lda = (int)d[3];
    p.ldb = (int)d[4];
    p.ldc = (int)d[5];
    p.tiles_n = N / C_::BN;
    p.tile0 = total;
    total += (M / C_::BM) * (N / C_::BN);
  }
  bt.ntiles = total;
  hipLaunchKernelGGL((gemm_kk_kernel<WM, WN, FM, FN, BKT, NSLOT, MINB>), dim3(total * splits), dim3(C_::NT), 0,
                     stream, bt);
  return (int)hipGetLastError();
}

struct Variant {
  int bm, bn, nt;
};
constexpr Variant kVariants[] = {{128, 128, 256}, {256, 128, 512}, {256, 256, 512}, {128, 128, 256},
                                 {128, 128, 256}, {128, 128, 256}, {128, 128, 512}};

}  // namespace

// Tile geometry of a variant: {BM, BN, threads} (the host picks tiles / splits with it).
MX_EXPORT int mx_gemm_kk_tile(int variant, int what) {
  if (variant < 0 || variant > 6) return -1;
  const Variant& v = kVariants[variant];
  return what == 0 ? v.bm : what == 1 ? v.bn : v.nt;
}

// desc: np x 8 int64 {a, b, c, lda, ldb, ldc, M, N} (element strides); M, N multiples of
// the variant's tile, K a multiple of 64 * splits, operands 16-B aligned with lda/ldb
// multiples of 8.  splits > 1 needs `slab` (tiles x splits x BM x BN fp32) and `ticket`
// (tiles x u32, zero-initialised once; the kernel leaves it zero).
// variant: 0 = 128 x 128 tile, 4 waves, BK 64, 2-slot ring (two workgroups per CU)
//          1 = 256 x 128 tile, 8 waves, BK 64, 3-slot ring
//          2 = 256 x 256 tile, 8 waves (128 x 64 each), BK 32, 4-slot ring
//          3 = 128 x 128 tile, BK 32, 3-slot ring (three workgroups per CU)
//          4 = 128 x 128 tile, BK 32, 2-slot ring (four workgroups per CU)
//          5 = 128 x 128 tile, BK 64, 4-slot ring (three K-steps in flight, one workgroup per CU)
//          6 = 128 x 128 tile, 8 waves of 64 x 32, BK 64, 4-slot ring
MX_EXPORT int mx_gemm_kk(int np, const int64_t* desc, int K, float beta, int variant, int splits, void* slab,
                         void* ticket, void* stream) {
  if (np < 1 || np > MAXP || K <= 0 || splits < 1) return (int)hipErrorInvalidValue;
  if (splits > 1 && (slab == nullptr || ticket == nullptr)) return (int)hipErrorInvalidValue;
  for (int q = 0; q < np; ++q) {
    const int64_t* d = desc + 8 * q;
    if ((d[0] | d[1]) & 15) return (int)hipErrorInvalidValue;
    if ((d[3] & 7) || (d[4] & 7) || d[3] < d[6] || d[4] < d[7] || d[5] < d[7]) return (int)hipErrorInvalidValue;
  }
  hipStream_t st = (hipStream_t)stream;
  float* sl = (float*)slab;
  uint32_t* tk = (uint32_t*)ticket;
  switch (variant) {
    case 1: return launch<4, 2, 4, 4, 64, 3, 1>(desc, np, K, beta, splits, sl, tk, st);
    case 2: return launch<2, 4, 8, 4, 32, 4, 1>(desc, np, K, beta, splits, sl, tk, st);
    case 3: return launch<2, 2, 4, 4, 32, 3, 3>(desc, np, K, beta, splits, sl, tk, st);
    case 4: return launch<2, 2, 4, 4, 32, 2, 4>(desc, np, K, beta, splits, sl, tk, st);
    case 5: return launch<2, 2, 4, 4, 64, 4, 1>(desc, np, K, beta, splits, sl, tk, st);
    case 6: return launch<2, 4, 4, 2, 64, 4, 1>(desc, np, K, beta, splits, sl, tk, st);
    default: return launch<2, 2, 4, 4, 64, 2, 2>(desc, np, K, beta, splits, sl, tk, st);
  }
}

