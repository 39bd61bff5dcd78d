// Forward and data-gradient GEMMs of the transformer Linear layers, with the elementwise
// work that follows them fused into the epilogue (gfx950, bf16 in, fp32 accumulate):
//
//   forward  C[M][N] = A[M][K] . W[N][K]^T   (W read in place, K contiguous: "B_KC")
//   dgrad    C[M][N] = A[M][K] . W[K][N]     (the same weight, now K-major)
//
// with A the activations / output gradients ([tokens, features], K contiguous) and the
// epilogue EPI one of
//   0  C = acc
//   1  C = acc + bias[n]                                   (QKV projection)
//   2  H = acc + bias[n] -> aux (bf16), C = gelu(H)        (fc1: Megatron bias_gelu fused)
//   3  D = acc * gelu'(aux[m][n]) -> C, plus fp32 column partial sums of D (the fc1 bias
//      gradient) per 16*FM-row wave block                 (fc2 dgrad: bias_gelu backward)
// Reference: Megatron-DeepSpeed's ColumnParallelLinear / RowParallelLinear GEMMs and its
// fused `bias_gelu_impl` (pinned by /root/reference/containers/megatron-deepspeed/
// Dockerfile:13, configured by examples/megatron-deepspeed/gpt2_345m/pretrain-ddp-zero1.yaml:
// 39-53); SURVEY §2.8 K6/K12.
//
// Why hand-written: hipBLASLt on gfx950 has no bf16 AUX/DGELU epilogue (it returns no
// algorithm), so bias-GeLU cost two extra memory passes per layer, and its picks for the
// hidden = 1024 shapes ran at ~0.76 PF/s (profiles/r2_gpt_s3/SPEED_OF_LIGHT.md).
//
// Design (cdna_hip_programming.md §5):
//  * one output tile per workgroup, tiles sized so one launch has ~256 of them (BM x BN in
//    {256x256, 256x192, 256x128, 128x256, 128x128}); waves own 16*FM x 16*FN sub-blocks;
//  * operands staged by LDS-DMA (global_load_lds_dwordx4, 1 KiB per wave instruction, no
//    staging registers) into an NSLOT ring, one raw barrier per 64-deep K-step, counted
//    vmcnt waits so the next steps' DMA stays in flight across the barrier;
//  * K-contiguous images are [row][64 k] with 128-B rows whose 16-B chunks are XOR-swizzled
//    by (row & 7) on the DMA SOURCE address (the LDS write stays lane-linear); MFMA
//    fragments are plain ds_read_b128 (conflict-free over every 16-lane read group);
//    the K-major weight image of dgrad uses gemm.hip's transposed-read scheme;
//  * the weight fragment is the MFMA's A operand, so a lane ends with 4 CONSECUTIVE output
//    columns of one row: 8-B stores, 4 bias values per 8-B load, 4 aux values per 8-B load;
//  * XCD-aware grouped tile order: the tiles one XCD runs are a compact (gm x n) block.
#include "gemm_common.h"

#include <type_traits>

using namespace mx;
using namespace mx::gemm;

namespace {

struct Args {
  const uint16_t* a;     // [M][lda], K contiguous
  const uint16_t* b;     // B_KC: [N][ldb] K contiguous; else [K][ldb]
  uint16_t* c;           // [M][ldc]
  uint16_t* aux;         // EPI 2: pre-activation out; EPI 3: pre-activation in ([M][ldx])
  const uint16_t* bias;  // EPI 1, 2: [N]
  float* part;           // EPI 3: [M / (16 FM)][N] fp32 column partials
  int lda, ldb, ldc, ldx;
  int K, N;
  int tiles_n, gm;
  int prio;              // 8-wave tiles, bit 0: s_setprio 1 for waves 4-7; bit 1: their half-step stagger
};

// Waves 4-7 of an 8-wave workgroup are the VALU-arbitration losers against their SIMD partners
// (waves 0-3) at equal priority: one static s_setprio 1 for that half before the K-loop
// (MI355X_MICROARCH.md "Two waves per SIMD", item 4), plus the half-step stagger (item 9):
// +0.6-0.75 % per GPT-2 step in same-box A/Bs (profiles/r5_s1/bench_ab_gemm_*.txt).
constexpr int g_gemm_nt_prio = 3;

template <bool BKC, int WM, int WN, int FM, int FN, int BKT, int NSLOT>
struct Geo {
  static constexpr int NW = WM * WN, NT = 64 * NW;
  static constexpr int BM = 16 * FM * WM, BN = 16 * FN * WN;
  static constexpr int RA = BKT * 2;                   // [m][k] image row bytes (64 or 128)
  static constexpr int IA = BM * RA;
  static constexpr int RB = BKC ? BKT * 2 : BN * 2;    // [n][k] or [k][n] image row bytes
  static constexpr int IB = BKC ? BN * RB : BKT * RB;
  static constexpr int PA = IA / 1024 / NW, PB = IB / 1024 / NW;
  static constexpr int SLOT = IA + IB, LDS = NSLOT * SLOT;
  static_assert(BKT == 32 || BKT == 64, "K-step");
  static_assert(PA * NW * 1024 == IA && PB * NW * 1024 == IB, "DMA pieces per wave");
  static_assert(BKC || (RB >= 256 && (BN & (BN - 1)) == 0), "K-major weight image needs BN = 2^k >= 128");
  static_assert(LDS <= 160 * 1024, "LDS");
};

// XOR swizzle of the 16-B chunks of a K-contiguous image row r (the same involution on the
// DMA source and on the fragment read).  128-B rows: chunk ^ (r & 7).  64-B rows (4 rows per
// 256-B bank row, quarter r & 3): chunk ^ f((r >> 2) & 3) with f = {0, 2, 3, 1}, which makes
// every 16-lane group of a ds_read_b128 (lanes {0-3,12-15,20-27}, {4-11,16-19,28-31}, ...)
// hit 16 distinct 16-B bank slots.
template <int N, int I = 0, typename F>
__device__ __forceinline__ void static_for(F&& f) {
  if constexpr (I < N) {
    f(std::integral_constant<int, I>{});
    static_for<N, I + 1>(f);
  }
}

template <int RA>
__device__ __forceinline__ int kc_swz(int r) {
  if constexpr (RA == 128) return r & 7;
  else return (0x78 >> (2 * ((r >> 2) & 3))) & 3;
}

// one 1-KiB LDS-DMA piece with a wave-uniform SGPR base and a per-lane 32-bit byte offset
// (the saddr form: advancing a K-step changes only the scalar base)
__device__ __forceinline__ void dma16s(const void* sbase, uint32_t voff, uint32_t lds_base) {
  asm volatile("s_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %0, %1"
               :: "v"(voff), "s"(sbase), "s"(lds_base) : "memory", "m0");
}

// ---- epilogue: lane holds C[m0 + 16 (FM wm + s) + i][n0 + 16 (FN wn + u) + 4 G + e].
// Elementwise math runs in that layout; each pair of 16-column subtiles (u0, u1) is then
// re-dealt with one permlane32 + one permlane16 swap per dword so lane G holds 8
// consecutive columns 32 up + 8 G .. +7 of its row: 16-B stores, one wave instruction =
// 16 rows x 64 B (the 8-B / 32-B-segment stores made the epilogue a quarter of the tile
// time -- in-kernel stamps, scripts/gemm_stamps.py)
template <int WM, int WN, int FM, int FN, int EPI>
__device__ __forceinline__ void epilogue(const Args& g, f32x4 (&acc)[FM][FN], int tm, int m0, int n0, int wave,
                                         int lane) {
  const int G = lane >> 4, i = lane & 15;
  const int wm = wave / WN, wn = wave % WN;
  const int row0 = m0 + 16 * FM * wm + i;
  const int colw = n0 + 16 * FN * wn;            // the wave's first column
  const int col0 = colw + 4 * G;                 // this lane's first column, MFMA layout
  float bias[FN][4];
  if constexpr (EPI == 1 || EPI == 2) {
#pragma unroll
    for (int u = 0; u < FN; ++u) {
      const uint2 bv = *reinterpret_cast<const uint2*>(g.bias + col0 + 16 * u);
      bias[u][0] = lo_bf(bv.x); bias[u][1] = hi_bf(bv.x);
      bias[u][2] = lo_bf(bv.y); bias[u][3] = hi_bf(bv.y);
    }
  }
  float csum[FN][4];
  if constexpr (EPI == 3) {
#pragma unroll
    for (int u = 0; u < FN; ++u)
#pragma unroll
      for (int e = 0; e < 4; ++e) csum[u][e] = 0.f;
  }
  static_assert(FN % 2 == 0, "the 16-B store re-deal pairs subtiles");
#pragma unroll
  for (int s = 0; s < FM; ++s) {
    const size_t r = (size_t)(row0 + 16 * s);
    uint16_t* crow = g.c + r * g.ldc + colw + 8 * G;
#pragma unroll
    for (int up = 0; up < FN / 2; ++up) {
      uint32_t c[2][2], h[2][2];
      if constexpr (EPI == 3) {   // aux (pre-activation) read as 16 B, re-dealt to the MFMA layout
        const uint4 hv = *reinterpret_cast<const uint4*>(g.aux + r * g.ldx + colw + 32 * up + 8 * G);
        h[0][0] = hv.x; h[0][1] = hv.y; h[1][0] = hv.z; h[1][1] = hv.w;
        undeal(h[0][0], h[0][1], h[1][0], h[1][1]);
      }
#pragma unroll
      for (int hlf = 0; hlf < 2; ++hlf) {
        const int u = 2 * up + hlf;
        float v[4] = {acc[s][u][0], acc[s][u][1], acc[s][u][2], acc[s][u][3]};
        if constexpr (EPI == 1 || EPI == 2) {
#pragma unroll
          for (int e = 0; e < 4; ++e) v[e] += bias[u][e];
        }
        if constexpr (EPI == 2) {
          h[hlf][0] = pack2(v[0], v[1]);
          h[hlf][1] = pack2(v[2], v[3]);
#pragma unroll
          for (int e = 0; e < 4; ++e) v[e] = gelu_tanh(v[e]);
        }
        if constexpr (EPI == 3) {
          const float hx[4] = {lo_bf(h[hlf][0]), hi_bf(h[hlf][0]), lo_bf(h[hlf][1]), hi_bf(h[hlf][1])};
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            v[e] *= gelu_tanh_grad(hx[e]);
            csum[u][e] += v[e];
          }
        }
        c[hlf][0] = pack2(v[0], v[1]);
        c[hlf][1] = pack2(v[2], v[3]);
      }
      if constexpr (EPI == 2) {
        deal(h[0][0], h[0][1], h[1][0], h[1][1]);
        *reinterpret_cast<uint4*>(g.aux + r * g.ldx + colw + 32 * up + 8 * G) =
            make_uint4(h[0][0], h[0][1], h[1][0], h[1][1]);
      }
      deal(c[0][0], c[0][1], c[1][0], c[1][1]);
      *reinterpret_cast<uint4*>(crow + 32 * up) = make_uint4(c[0][0], c[0][1], c[1][0], c[1][1]);
    }
  }
  if constexpr (EPI == 3) {
    // column sums of this wave's 16 FM rows: over the 16 lanes of a row (i), lane i == 0
    // of each G writes 4 consecutive columns
    float* prow = g.part + (size_t)(tm * WM + wm) * g.N + col0;
#pragma unroll
    for (int u = 0; u < FN; ++u) {
      float t[4];
#pragma unroll
      for (int e = 0; e < 4; ++e) t[e] = row_sum16(csum[u][e]);
      if (i == 0) *reinterpret_cast<float4*>(prow + 16 * u) = make_float4(t[0], t[1], t[2], t[3]);
    }
  }
}

// STAMP (diagnostic build, mx_gemm_nt_stamps only): lane 0 of wave 0 records s_memtime /
// s_memrealtime at tile start, after the first K-step's data landed, after the main loop
// and after the epilogue into g.part ([tile][8] uint64); no output value depends on them
template <bool BKC, int WM, int WN, int FM, int FN, int BKT, int NSLOT, int MINB, int EPI, bool STAMP = false>
__global__ __launch_bounds__(64 * WM * WN, MINB) void gemm_nt_kernel(const Args g) {
  using Gm = Geo<BKC, WM, WN, FM, FN, BKT, NSLOT>;
  constexpr int BM = Gm::BM, BN = Gm::BN, RA = Gm::RA, RB = Gm::RB, IA = Gm::IA;
  constexpr int PA = Gm::PA, PB = Gm::PB, SLOT = Gm::SLOT;
  constexpr int PER = PA + PB;   // DMA instructions per wave per K-step
  constexpr int LPR = RA / 16;   // lanes per K-contiguous image row in a DMA piece
  __shared__ __attribute__((aligned(1024))) char smem[Gm::LDS];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  // grouped, XCD-contiguous tile order: consecutive logical ids walk gm row-tiles first
  const int wg = xcd_remap(blockIdx.x, gridDim.x);
  const int per_group = g.gm * g.tiles_n;
  const int grp = wg / per_group, rem = wg - grp * per_group;
  const int tm = grp * g.gm + rem % g.gm, tn = rem / g.gm;
  const int m0 = tm * BM, n0 = tn * BN;
  const int nk = g.K / BKT;
  uint64_t* stamps = reinterpret_cast<uint64_t*>(g.part) + (size_t)wg * 8;
  auto stamp = [&](int k) __attribute__((always_inline)) {
    if constexpr (STAMP) {
      if (tid == 0) {
        stamps[2 * k] = __builtin_amdgcn_s_memtime();
        stamps[2 * k + 1] = __builtin_amdgcn_s_memrealtime();
      }
    }
  };
  stamp(0);

  // ---- LDS-DMA: scalar tile bases (advanced per K-step) + constant per-lane byte offsets.
  // K-contiguous image: a 1-KiB piece = 1024 / RA rows; lane l fills row l / LPR, physical
  // chunk l % LPR, i.e. logical chunk (l % LPR) ^ swz(row)
  const char* baseA = reinterpret_cast<const char*>(g.a + (size_t)m0 * g.lda);
  const char* baseB = reinterpret_cast<const char*>(BKC ? g.b + (size_t)n0 * g.ldb : g.b + n0);
  uint32_t voA[PA], voB[PB];
#pragma unroll
  for (int j = 0; j < PA; ++j) {
    const int row = (PA * wave + j) * (1024 / RA) + lane / LPR;
    voA[j] = (uint32_t)(row * g.lda + 8 * ((lane % LPR) ^ kc_swz<RA>(row))) * 2u;
  }
  if constexpr (BKC) {
#pragma unroll
    for (int j = 0; j < PB; ++j) {
      const int row = (PB * wave + j) * (1024 / RB) + lane / LPR;
      voB[j] = (uint32_t)(row * g.ldb + 8 * ((lane % LPR) ^ kc_swz<RB>(row))) * 2u;
    }
  } else {
    constexpr int CB = RB / 16;   // chunks per k-row
#pragma unroll
    for (int j = 0; j < PB; ++j) {
      const int k = (PB * wave + j) * (1024 / RB) + lane / CB;
      voB[j] = (uint32_t)(k * g.ldb + 8 * pchunk(k, lane % CB)) * 2u;
    }
  }
  const size_t stepA = (size_t)BKT * 2, stepB = BKC ? (size_t)BKT * 2 : (size_t)BKT * g.ldb * 2;

  // ---- fragment offsets: lane (G, i) reads row i of a 16-row subtile, k 8G .. 8G + 7 (+32 kk)
  const int G = lane >> 4, i = lane & 15;
  const int wm = wave / WN, wn = wave % WN;
  const int offA = (16 * FM * wm + i) * RA;          // + 16 s RA (compile-time) per subtile
  int cA[BKT / 32];
#pragma unroll
  for (int kk = 0; kk < BKT / 32; ++kk) cA[kk] = 16 * ((4 * kk + G) ^ kc_swz<RA>(i));
  int offB;
  if constexpr (BKC) {
    offB = (16 * FN * wn + i) * RB;
  } else {
    const int krow = 8 * G + (i >> 2);
    offB = krow * RB + ((((FN * wn) ^ gsw(krow)) << 1) | ((i & 3) >> 1)) * 16 + (i & 1) * 8;
  }
  // K-major subtile u: the pair index FN wn + u XOR gsw(krow); FN wn is a multiple of FN, so
  // for FN a power of two (u < FN) the XOR acts on disjoint bits: (FN wn + u) ^ g =
  // ((FN wn) ^ g) ^ u exactly when g < FN ... not in general, so keep a per-u table
  int offBu[FN];
#pragma unroll
  for (int u = 0; u < FN; ++u) {
    if constexpr (BKC) {
      offBu[u] = offB + 16 * u * RB;
    } else {
      const int krow = 8 * G + (i >> 2);
      offBu[u] = krow * RB + ((((FN * wn + u) ^ gsw(krow)) << 1) | ((i & 3) >> 1)) * 16 + (i & 1) * 8;
    }
  }

  f32x4 acc[FM][FN];
#pragma unroll
  for (int s = 0; s < FM; ++s)
#pragma unroll
    for (int u = 0; u < FN; ++u) acc[s][u] = f32x4{0.f, 0.f, 0.f, 0.f};

  const uint32_t lds0 = lds_addr(smem);
  const uint32_t ldsA = __builtin_amdgcn_readfirstlane(lds0 + PA * wave * 1024);
  const uint32_t ldsB = __builtin_amdgcn_readfirstlane(lds0 + IA + PB * wave * 1024);
  // one DMA piece j of K-step `it` into ring slot `slot` (pieces 0 .. PA-1: A, then B)
  auto piece = [&](int slot, int it, int j) __attribute__((always_inline)) {
    if (j < PA) dma16s(baseA + it * stepA, voA[j], ldsA + slot * SLOT + j * 1024);
    else dma16s(baseB + it * stepB, voB[j - PA], ldsB + slot * SLOT + (j - PA) * 1024);
  };

#pragma unroll
  for (int q = 0; q < NSLOT - 1; ++q)
    if (q < nk) {
#pragma unroll
      for (int j = 0; j < PER; ++j) piece(q, q, j);
    }
  // the next step's pieces are spread over the first half of this step's MFMA sequence
  // (one or two per fragment row) instead of being issued back to back after the barrier:
  // an LDS-DMA issue costs ~60-185 cycles of the wave's issue slot, so a burst of PER of
  // them left the matrix pipe idle at the top of every K-step
  // inner order: the operand with more fragments per wave stays resident for the 32-deep
  // k-slice and the other one is streamed, one fragment per group of max(FM, FN) MFMAs, so
  // every streamed LDS read is covered by >= 4-8 MFMAs (a read feeding only 2-4 MFMAs left
  // its latency exposed: one lgkmcnt stall per MFMA group in the ISA)
  constexpr bool XRES = FM >= FN;
  constexpr int NSTREAM = XRES ? FN : FM;
  constexpr int NS = (BKT / 32) * NSTREAM;       // streamed-fragment steps per K-step
  constexpr int SPREAD = NS / 2 >= PER ? NS / 2 : NS;
  // Stagger (g.prio bit 1, 8-wave resident-x tiles): waves 4-7 run half a K-step behind their
  // SIMD partners (waves 0-3).  They read ALL of step it's fragments before barrier it + 1 but
  // issue only the first half of its (kk, u) MFMA pairs there; the second half runs from
  // registers right after the next barrier, while the partner is in its LDS read burst
  // (MI355X_MICROARCH.md "Two waves per SIMD", item 9).  Same arithmetic in the same order
  // per accumulator, so the output is bit-identical.
  constexpr int KK = BKT / 32, NQ = KK * FN, NH1 = NQ / 2;
  const bool stag = XRES && WM * WN == 8 && (g.prio & 2) && wave >= 4;
  bf16x8 dx[KK][FM], dw[NQ - NH1 > 0 ? NQ - NH1 : 1];
  bool pend = false;
  auto run_h2 = [&]() __attribute__((always_inline)) {
#pragma unroll
    for (int p = NH1; p < NQ; ++p)
#pragma unroll
      for (int s2 = 0; s2 < FM; ++s2)
        acc[s2][p % FN] = mfma16(dw[p - NH1], dx[p / FN][s2], acc[s2][p % FN]);
  };
  if (WM * WN == 8 && (g.prio & 1) && wave >= 4) __builtin_amdgcn_s_setprio(1);
  // the K-loop is unrolled by the ring depth, so every ring slot (LDS offset, M0 value) is
  // a compile-time constant
  for (int it0 = 0; it0 < nk; it0 += NSLOT) {
    static_for<NSLOT>([&](auto qc) __attribute__((always_inline)) {
      constexpr int q = decltype(qc)::value;
      const int it = it0 + q;
      if (it >= nk) return;
      // retire step it's pieces (later steps stay in flight), then one barrier: every
      // wave's pieces of step it have landed and every wave is done reading step it - 1's slot
      const int later = nk - 1 - it;
      if (NSLOT >= 5 && later >= 3) vm_wait<(NSLOT >= 5 ? 3 : 0) * PER>();
      else if (NSLOT >= 4 && later >= 2) vm_wait<(NSLOT >= 4 ? 2 : 0) * PER>();
      else if (NSLOT >= 3 && later >= 1) vm_wait<(NSLOT >= 3 ? 1 : 0) * PER>();
      else vm_wait<0>();
      __builtin_amdgcn_s_barrier();
      if (STAMP && it == 0) stamp(1);
      const bool fetch = it + NSLOT - 1 < nk;
      constexpr int ns = (q + NSLOT - 1) % NSLOT;
      const char* As = smem + q * SLOT;
      const char* Bs = As + IA;
      auto wfrag = [&](int u, int kk) __attribute__((always_inline)) {
        if constexpr (BKC) return lds_read8(Bs, offBu[u] + cA[kk]);
        else return cat(tr_read(Bs, offBu[u] + 32 * RB * kk), tr_read(Bs, offBu[u] + 32 * RB * kk + 4 * RB));
      };
      auto xfrag = [&](int s, int kk) __attribute__((always_inline)) {
        return lds_read8(As, offA + 16 * s * RA + cA[kk]);
      };
      if (XRES && stag) {
        if (pend) run_h2();
#pragma unroll
        for (int kk = 0; kk < KK; ++kk)
#pragma unroll
          for (int s2 = 0; s2 < FM; ++s2) dx[kk][s2] = xfrag(s2, kk);
#pragma unroll
        for (int p = 0; p < NH1; ++p) {
          const bf16x8 w = wfrag(p % FN, p / FN);
#pragma unroll
          for (int j = 0; j < PER; ++j)
            if (j * NH1 / PER == p && fetch) piece(ns, it + NSLOT - 1, j);
#pragma unroll
          for (int s2 = 0; s2 < FM; ++s2) acc[s2][p % FN] = mfma16(w, dx[p / FN][s2], acc[s2][p % FN]);
        }
#pragma unroll
        for (int p = NH1; p < NQ; ++p) dw[p - NH1] = wfrag(p % FN, p / FN);
        pend = true;
        // every fragment of this slot is in registers before the barrier that frees the slot
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        return;
      }
#pragma unroll
      for (int kk = 0; kk < BKT / 32; ++kk) {
        if constexpr (XRES) {
          bf16x8 x[FM];
#pragma unroll
          for (int s = 0; s < FM; ++s) x[s] = xfrag(s, kk);
#pragma unroll
          for (int u = 0; u < FN; ++u) {
            const bf16x8 w = wfrag(u, kk);
            const int qq = kk * NSTREAM + u;
#pragma unroll
            for (int j = 0; j < PER; ++j)
              if (qq < SPREAD && j * SPREAD / PER == qq && fetch) piece(ns, it + NSLOT - 1, j);
#pragma unroll
            for (int s = 0; s < FM; ++s) acc[s][u] = mfma16(w, x[s], acc[s][u]);
          }
        } else {
          bf16x8 w[FN];
#pragma unroll
          for (int u = 0; u < FN; ++u) w[u] = wfrag(u, kk);
#pragma unroll
          for (int s = 0; s < FM; ++s) {
            const bf16x8 x = xfrag(s, kk);
            const int qq = kk * NSTREAM + s;
#pragma unroll
            for (int j = 0; j < PER; ++j)
              if (qq < SPREAD && j * SPREAD / PER == qq && fetch) piece(ns, it + NSLOT - 1, j);
#pragma unroll
            for (int u = 0; u < FN; ++u) acc[s][u] = mfma16(w[u], x, acc[s][u]);
          }
        }
      }
    });
  }

  if (stag && pend) run_h2();
  stamp(2);
  epilogue<WM, WN, FM, FN, EPI>(g, acc, tm, m0, n0, wave, lane);
  if constexpr (STAMP) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    stamp(3);
  }
}


template <bool BKC, int WM, int WN, int FM, int FN, int BKT, int NSLOT, int MINB, int EPI>
int launch(Args a, int M, hipStream_t stream) {
  using Gm = Geo<BKC, WM, WN, FM, FN, BKT, NSLOT>;
  if (M % Gm::BM || a.N % Gm::BN || a.K % BKT || a.K <= 0) return (int)hipErrorInvalidValue;
  const int tiles_m = M / Gm::BM;
  a.tiles_n = a.N / Gm::BN;
  int gm = 8;
  while (gm > 1 && tiles_m % gm) gm >>= 1;
  a.gm = gm;
  hipLaunchKernelGGL((gemm_nt_kernel<BKC, WM, WN, FM, FN, BKT, NSLOT, MINB, EPI>), dim3(tiles_m * a.tiles_n),
                     dim3(Gm::NT), 0, stream, a);
  return (int)hipGetLastError();
}

// variant -> {BM, BN, rows per column-partial block (16 FM), B may be K-major}
struct Variant {
  int bm, bn, part_rows, kmajor_ok;
};
constexpr Variant kVariants[] = {
    {256, 256, 128, 1},   // 0: 8 waves 2 x 4 of 128 x 64, BK 32, 4-slot ring (128 KiB)
    {256, 192, 64, 0},    // 1: 8 waves 4 x 2 of 64 x 96, BK 64, 2-slot ring (112 KiB); forward only
    {128, 128, 64, 1},    // 2: 4 waves 2 x 2 of 64 x 64, BK 64, 2-slot ring, two workgroups per CU
    {128, 128, 64, 1},    // 3: 8 waves 2 x 4 of 64 x 32, BK 64, 4-slot ring
    {256, 128, 64, 1},    // 4: 8 waves 4 x 2 of 64 x 64, BK 64, 3-slot ring (144 KiB)
    {128, 256, 64, 1},    // 5: 8 waves 2 x 4 of 64 x 64, BK 64, 3-slot ring (144 KiB)
    {256, 256, 128, 1},   // 6: as 0 with BK 64 and a 2-slot ring
    {128, 128, 64, 1},    // 7: 8 waves 2 x 4 of 64 x 32, BK 32, 6-slot ring
    {256, 128, 64, 1},    // 8: 8 waves 4 x 2 of 64 x 64, BK 32, 5-slot ring (120 KiB)
};
constexpr int kNumVariants = sizeof(kVariants) / sizeof(kVariants[0]);

template <bool BKC, int EPI>
int dispatch(int variant, const Args& a, int M, hipStream_t st) {
  switch (variant) {
    case 0: return launch<BKC, 2, 4, 8, 4, 32, 4, 1, EPI>(a, M, st);
    case 1:
      if constexpr (BKC) return launch<BKC, 4, 2, 4, 6, 64, 2, 1, EPI>(a, M, st);
      else return (int)hipErrorInvalidValue;
    case 2: return launch<BKC, 2, 2, 4, 4, 64, 2, 2, EPI>(a, M, st);
    case 3: return launch<BKC, 2, 4, 4, 2, 64, 4, 1, EPI>(a, M, st);
    case 4: return launch<BKC, 4, 2, 4, 4, 64, 3, 1, EPI>(a, M, st);
    case 5: return launch<BKC, 2, 4, 4, 4, 64, 3, 1, EPI>(a, M, st);
    case 6: return launch<BKC, 2, 4, 8, 4, 64, 2, 1, EPI>(a, M, st);
    case 7: return launch<BKC, 2, 4, 4, 2, 32, 6, 1, EPI>(a, M, st);
    case 8: return launch<BKC, 4, 2, 4, 4, 32, 5, 1, EPI>(a, M, st);
    default: return (int)hipErrorInvalidValue;
  }
}

template <int WM, int WN, int FM, int FN, int BKT, int NSLOT, int MINB>
int launch_stamped(Args a, int M, hipStream_t stream) {
  using Gm = Geo<true, WM, WN, FM, FN, BKT, NSLOT>;
  if (M % Gm::BM || a.N % Gm::BN || a.K % BKT || a.K <= 0) return (int)hipErrorInvalidValue;
  const int tiles_m = M / Gm::BM;
  a.tiles_n = a.N / Gm::BN;
  int gm = 8;
  while (gm > 1 && tiles_m % gm) gm >>= 1;
  a.gm = gm;
  hipLaunchKernelGGL((gemm_nt_kernel<true, WM, WN, FM, FN, BKT, NSLOT, MINB, 0, true>), dim3(tiles_m * a.tiles_n),
                     dim3(Gm::NT), 0, stream, a);
  return (int)hipGetLastError();
}

}  // namespace

// Diagnostic: forward GEMM (epilogue 0) of variant 0, 3 or 6 with per-tile clock stamps
// written to `stamps` ([tiles][8] uint64: memtime/realtime at start, first data, loop end,
// epilogue end).  Not used by training.
MX_EXPORT int mx_gemm_nt_stamps(const void* a, const void* b, void* c, void* stamps, int lda, int ldb, int ldc,
                                int M, int N, int K, int variant, void* stream) {
  Args g{};
  g.a = (const uint16_t*)a;
  g.b = (const uint16_t*)b;
  g.c = (uint16_t*)c;
  g.part = (float*)stamps;
  g.lda = lda;
  g.ldb = ldb;
  g.ldc = ldc;
  g.K = K;
  g.N = N;
  hipStream_t st = (hipStream_t)stream;
  switch (variant) {
    case 0: return launch_stamped<2, 4, 8, 4, 32, 4, 1>(g, M, st);
    case 3: return launch_stamped<2, 4, 4, 2, 64, 4, 1>(g, M, st);
    case 6: return launch_stamped<2, 4, 8, 4, 64, 2, 1>(g, M, st);
    default: return (int)hipErrorInvalidValue;
  }
}

// Tile geometry of a variant: what = 0 -> BM, 1 -> BN, 2 -> rows per column-partial block,
// 3 -> 1 when the weight may be K-major (dgrad).  -1 for an unknown variant.
MX_EXPORT int mx_gemm_nt_tile(int variant, int what) {
  if (variant < 0 || variant >= kNumVariants) return -1;
  const Variant& v = kVariants[variant];
  return what == 0 ? v.bm : what == 1 ? v.bn : what == 2 ? v.part_rows : v.kmajor_ok;
}

// C[M][N] = A[M][K] . op(B) with the epilogue `epi` (see the file comment).
//   b_kmajor = 0: B is [N][ldb] (forward, C = A B^T);  1: B is [K][ldb] (dgrad, C = A B).
//   aux [M][ldx]: EPI 2 output / EPI 3 input; bias [N] (EPI 1, 2); part (EPI 3): fp32
//   [M / part_rows][N] column partial sums.
// Contract (checked): M, N multiples of the variant's tile, K a multiple of 64, every
// pointer 16-B aligned and every leading dimension a multiple of 8 elements.
MX_EXPORT int mx_gemm_nt(const void* a, const void* b, void* c, void* aux, const void* bias, void* part,
                         int lda, int ldb, int ldc, int ldx, int M, int N, int K, int b_kmajor, int epi,
                         int variant, void* stream) {
  if (variant < 0 || variant >= kNumVariants || M <= 0 || N <= 0 || K <= 0) return (int)hipErrorInvalidValue;
  if ((((uintptr_t)a) | ((uintptr_t)b) | ((uintptr_t)c)) & 15) return (int)hipErrorInvalidValue;
  if ((lda & 7) || (ldb & 7) || (ldc & 7) || lda < K || ldc < N) return (int)hipErrorInvalidValue;
  // per-lane DMA offsets are 32-bit byte offsets within one tile's rows
  if ((int64_t)256 * (b_kmajor ? 64 : (lda > ldb ? lda : ldb)) * 2 >= ((int64_t)1 << 31)) return (int)hipErrorInvalidValue;
  if (b_kmajor ? ldb < N : ldb < K) return (int)hipErrorInvalidValue;
  if ((epi == 1 || epi == 2) && (bias == nullptr || ((uintptr_t)bias & 7))) return (int)hipErrorInvalidValue;
  if ((epi == 2 || epi == 3) && (aux == nullptr || ((uintptr_t)aux & 7) || (ldx & 3) || ldx < N))
    return (int)hipErrorInvalidValue;
  if (epi == 3 && (part == nullptr || ((uintptr_t)part & 15))) return (int)hipErrorInvalidValue;
  Args g{};
  g.a = (const uint16_t*)a;
  g.b = (const uint16_t*)b;
  g.c = (uint16_t*)c;
  g.aux = (uint16_t*)aux;
  g.bias = (const uint16_t*)bias;
  g.part = (float*)part;
  g.lda = lda;
  g.ldb = ldb;
  g.ldc = ldc;
  g.ldx = ldx;
  g.K = K;
  g.N = N;
  g.prio = g_gemm_nt_prio;
  hipStream_t st = (hipStream_t)stream;
  if (!b_kmajor) {
    switch (epi) {
      case 0: return dispatch<true, 0>(variant, g, M, st);
      case 1: return dispatch<true, 1>(variant, g, M, st);
      case 2: return dispatch<true, 2>(variant, g, M, st);
      default: return (int)hipErrorInvalidValue;
    }
  }
  switch (epi) {
    case 0: return dispatch<false, 0>(variant, g, M, st);
    case 3: return dispatch<false, 3>(variant, g, M, st);
    default: return (int)hipErrorInvalidValue;
  }
}
