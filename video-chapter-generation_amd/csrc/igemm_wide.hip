// Wide-tile bf16 GEMM engine for the dense K-contiguous GEMMs of BERT-base's Linear layers (reference: the nn.Linear
// layers of transformers' BertModel, model/lang/bert_hugface.py:20, consumed at model/fusion/two_stream.py:178):
// C[M][N] = epi(A[M][K] B[N][K]^T), A and B bf16 row-major, fp32 accumulation.
//
// Why a third engine: the 128 x 128 engine (igemm_fast.hip) runs two barriers per 64-deep k-step with all four waves in
// lockstep, so its MFMA and LDS / LDS-DMA phases never overlap inside a CU (~600-750 TF/s on BERT's shapes); the
// 256 x 256 engine (igemm256.hip) overlaps them but its tiles do not divide BERT's N = 768 (96 tiles for 256 CUs).
// Here one 512-thread workgroup per CU owns a BM x BN = 128 x 192 tile (M = 8192 rows: N = 768 -> 256 tiles, one per
// CU; N = 2304 / 3072 -> 3 / 4 rounds) and walks its tiles persistently:
//   * 8 waves as 2 (M) x 4 (N), each a 64 x 48 sub-tile (4 x 3 fragments of 16 x 16, 24 MFMAs per 64-deep k-step);
//   * one k-step = two phases separated by raw s_barriers: [fragment reads + LDS-DMA issue] and [24 MFMAs]; waves 4-7
//     run one barrier behind waves 0-3 (the stagger), so on every SIMD one wave computes while its partner reads
//     (MI355X_MICROARCH.md "Two waves per SIMD", item 9; cdna_hip_programming.md §5 "The 256^2 8-phase template");
//   * 3 LDS stages of A [128][64] + B [192][64] (120 KiB), k-step s + 2 DMA'd during step s: each group issues its
//     pieces in its read phase, the stage it refills was last read one phase earlier by the other group, whose reads
//     were waited for (lgkmcnt(0)) before that barrier; the RAW wait is a counted vmcnt at the end of the phase before
//     the read (cdna_hip_programming.md §5 "Read a staged buffer one phase AFTER the wait that retires it");
//   * the tiles of one workgroup are one step sequence (tile, k-tile), so the next tile's first k-steps are in flight
//     while this tile's last MFMAs and its epilogue run; the epilogue goes straight from the accumulators
//     (4 consecutive columns per lane) with bias / GELU (+ pre-activation copy) / GELU' / residual fused.
#include "fastload.h"

namespace vcg {

namespace {

// bijective remap of the persistent slots: XCD x (blocks b with b % 8 == x share one) takes the contiguous slot range
// [x q + min(x, r), ...) of n = 8 q + r slots, so the tiles running at once on one XCD share A rows (and B) in its L2
__device__ __forceinline__ int w_xcd_slot(int b, int n) {
  const int q = n >> 3, r = n & 7, x = b & 7;
  return (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + (b >> 3);
}

}  // namespace

enum { WE_STORE = 0, WE_GELU = 1, WE_GELU_BWD = 2, WE_RES = 3, WE_RES32 = 4 };

namespace {

// epilogue of one finished tile: acc[i][j][r] = C[m][n], m = m0 + i * 16, n = n0 + j * 16 + r (the lane's rows /
// columns); semantics of the fast engine's bf16 epilogues (igemm_fast.hip):
//   WE_STORE     C = bf16(acc + bias)
//   WE_GELU      pre = bf16(acc + bias) (-> aux when given, the backward's GELU' input), C = bf16(gelu(acc + bias)):
//                the GELU of the unrounded f32 value, as the 128 x 128 engine's epilogue (closer to exact than bf16
//                autocast's GELU of the rounded Linear output: the oracle-anchored step's BERT gradients measured
//                1.24e-2 from fp64 with the rounded input, against autocast's 0.82e-2)
//   WE_GELU_BWD  C = bf16(bf16(acc + bias) * gelu'(res)), res = the saved pre-activation
//   WE_RES       C = bf16(acc + bias + res)
//   WE_RES32     C = acc + bias + res with res and C fp32 (BERT's input gradients on its fp32 residual-gradient stream)
__device__ const float4 g_wide_zero4 = {0.f, 0.f, 0.f, 0.f};

template <int MT, int NT, int WE>
__device__ __forceinline__ void wide_epilogue(f32x4 (&acc)[MT][NT], const GemmParams& p, int m0, int n0) {
  bf16_t* C = reinterpret_cast<bf16_t*>(p.C);
  const bf16_t* R = reinterpret_cast<const bf16_t*>(p.residual);
  float rv[MT][NT][4];
  if constexpr (WE == WE_GELU_BWD || WE == WE_RES || WE == WE_RES32) {
#pragma unroll
    for (int j = 0; j < NT; ++j)
#pragma unroll
      for (int i = 0; i < MT; ++i) {
        const int m = min(m0 + i * 16, p.M - 1), n = min(n0 + j * 16, p.N - 4);
        if constexpr (WE == WE_RES32)
          load4<float>(reinterpret_cast<const float*>(p.residual) + (long long)m * p.ldr + n, rv[i][j]);
        else
          load4<bf16_t>(R + (long long)m * p.ldr + n, rv[i][j]);
      }
  }
#pragma unroll
  for (int j = 0; j < NT; ++j) {
    const int n = n0 + j * 16;
    // (an unconditional load from a selected address: a load under a branch leaves it possibly outstanding at the
    // k-loop's join, and hipcc then waits vmcnt(0) -- draining the LDS-DMA prefetch -- at the top of every k-step)
    const float4* bp = p.bias ? reinterpret_cast<const float4*>(p.bias + min(n, p.N - 4)) : &g_wide_zero4;
    const float4 b4 = *bp;
    const float bv[4] = {b4.x, b4.y, b4.z, b4.w};
#pragma unroll
    for (int i = 0; i < MT; ++i) {
      const int m = m0 + i * 16;
      float v[4];
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        float t = acc[i][j][r] + bv[r];
        if constexpr (WE == WE_GELU) {
          v[r] = p.fast_act ? gelu_erf_fast(t) : gelu_erf(t);
          acc[i][j][r] = t;  // the pre-activation, for aux (rounded by the store)
        } else if constexpr (WE == WE_GELU_BWD) {
          t = bf2f(f2bf(t));
          v[r] = t * (p.fast_act ? gelu_erf_grad_fast(rv[i][j][r]) : gelu_erf_grad(rv[i][j][r]));
        } else if constexpr (WE == WE_RES || WE == WE_RES32) {
          v[r] = t + rv[i][j][r];
        } else {
          v[r] = t;
        }
      }
      if (m < p.M && n < p.N) {
        if constexpr (WE == WE_RES32)
          store4<float>(reinterpret_cast<float*>(p.C) + (long long)m * p.ldc + n, v);
        else
          store4<bf16_t>(C + (long long)m * p.ldc + n, v);
        if constexpr (WE == WE_GELU) {
          if (p.aux) {
            const float a4[4] = {acc[i][j][0], acc[i][j][1], acc[i][j][2], acc[i][j][3]};
            store4<bf16_t>(reinterpret_cast<bf16_t*>(p.aux) + (long long)m * p.ldc + n, a4);
          }
        }
      }
    }
  }
}

}  // namespace

// profiling build (make EXTRA=-DVCG_WIDE_STAMPS): s_memtime of waves 0 and 4 of workgroup 0 at 4 points of both
// phases of k-steps 8..23 (phase top after the barrier, after the reads / DMA issue / MFMAs, after the waits)
#ifdef VCG_WIDE_STAMPS
__device__ unsigned long long g_wide_stamps[2 * 16 * 2 * 4];
#define W_STAMP(s, ph, k)                                                                                      \
  do {                                                                                                         \
    if (blockIdx.x == 0 && (tid == 0 || tid == 256) && (s) >= 8 && (s) < 24)                                  \
      g_wide_stamps[((((tid >> 8) * 16 + (s) - 8) * 2 + (ph)) * 4) + (k)] = __builtin_amdgcn_s_memtime();      \
  } while (0)
#else
#define W_STAMP(s, ph, k) do {} while (0)
#endif
// measurement ablations (make EXTRA=-DVCG_WIDE_ABL=n; wrong results): 1 no LDS-DMA after the prologue, 2 no MFMAs,
// 3 no fragment reads after the first k-step
#ifndef VCG_WIDE_ABL
#define VCG_WIDE_ABL 0
#endif

// the counted wait for k-step s + 1: `ahead` younger k-steps' pieces (0..2) stay in flight
template <int P>
__device__ __forceinline__ void wide_wait(int ahead) {
  if (ahead >= 2) __builtin_amdgcn_s_waitcnt(waitcnt_vm(2 * P));
  else if (ahead == 1) __builtin_amdgcn_s_waitcnt(waitcnt_vm(P));
  else __builtin_amdgcn_s_waitcnt(waitcnt_vm(0));
}

// LDS-DMA loader of the dense K-contiguous A [BM][64] and B [BN][64] stage tiles: 8 rows x 128 B per wave instruction
// (a "piece"), PA = BM / 64 A pieces and PB = BN / 64 B pieces per wave and k-step; 16-B chunk c of row r at slot
// c ^ ((r >> 1) & 7) (fast_frag's swizzle, pre-applied on the global source address). The per-row offsets are computed
// once per tile, so a piece is one select and one buffer_load ... lds.
template <int BM, int BN, int NW = 8>
struct WideLoader {
  static constexpr int PA = BM / (8 * NW), PB = BN / (8 * NW), P = PA + PB, AE = BM * FBK;
  __amdgpu_buffer_rsrc_t ra, rb;
  uint32_t oa, ob;  // offsets past the buffers' ranges: the load returns zeros
  int off[P];       // element offset of the piece row's chunk (k = 0), -1 = a row beyond M / N
  int kc[P];        // the chunk's first k inside a 64-wide k tile
  __device__ __forceinline__ void init(const GemmParams& p) {
    oa = (uint32_t)min(p.a.bytes, (long long)0xFFFFFF00LL);
    ob = (uint32_t)min(p.b.bytes, (long long)0xFFFFFF00LL);
    ra = __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(p.a.ptr), 0, oa, 0x00020000);
    rb = __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(p.b.ptr), 0, ob, 0x00020000);
  }
  __device__ __forceinline__ void tile(const GemmParams& p, int m0, int n0, int wave, int lane) {
#pragma unroll
    for (int q = 0; q < P; ++q) {
      const bool isa = q < PA;
      const int r = (wave * (isa ? PA : PB) + (isa ? q : q - PA)) * 8 + (lane >> 3);
      kc[q] = 8 * fswz(r, lane & 7);
      const int gr = (isa ? m0 : n0) + r;
      off[q] = gr < (isa ? p.M : p.N) ? (int)((long long)gr * (isa ? p.a.ld : p.b.ld)) + kc[q] : -1;
    }
  }
  template <int Q>
  __device__ __forceinline__ void piece(int k0, int K, bf16_t* stage, int wave) const {
    constexpr bool isa = Q < PA;
    const uint32_t bad = isa ? oa : ob;
    const uint32_t voff = (off[Q] >= 0 && k0 + kc[Q] < K) ? (uint32_t)(off[Q] + k0) * 2u : bad;
    bf16_t* slice = stage + (isa ? 0 : AE) + (wave * (isa ? PA : PB) + (isa ? Q : Q - PA)) * 512;
    __builtin_amdgcn_raw_ptr_buffer_load_lds(isa ? ra : rb, (lds_void_t*)slice, 16, voff, 0, 0, 0);
  }
  template <int Q = 0>
  __device__ __forceinline__ void all(int k0, int K, bf16_t* stage, int wave) const {
    if constexpr (Q < P) {
      piece<Q>(k0, K, stage, wave);
      all<Q + 1>(k0, K, stage, wave);
    }
  }
};

// ST = 3 stages (prefetch distance 2); each group issues its LDS-DMA pieces of step s + 2 in its read phase, after the
// fragment reads. (Measured and rejected, profiles/r06_wide_engine_ab.txt: 4 stages, the pieces in the compute phase
// -- between the two k32 halves or one every few MFMAs --, no s_setprio or the read phase at priority 1, no stagger,
// a 4-wave 64 x 96 form with in-wave software pipelining, and register staging (buffer_load to VGPRs one k-step ahead,
// ds_write_b128 into the stage, 2 or 3 stages: 6-7 % slower): all equal or slower.)
template <int BM, int BN, int WE, int ST = 3>
__global__ __launch_bounds__(512) void gemm_wide_kernel(GemmParams p) {
  constexpr int MT = BM / 32, NT = BN / 64;          // the wave's (BM / 2) x (BN / 4) sub-tile in 16 x 16 fragments
  constexpr int AE = BM * FBK, BE = BN * FBK, SE = AE + BE;
  constexpr int PIECES = BM / 64 + BN / 64;          // LDS-DMA instructions per wave per k-step
  constexpr int PF = ST - 1;
  static_assert(ST * SE * 2 <= 160 * 1024, "LDS");
  __shared__ __attribute__((aligned(1024))) bf16_t smem[ST * SE];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int grp = wave >> 2, wc = wave & 3;          // stagger group = M half of the tile; N quarter
  const int ntn = (p.N + BN - 1) / BN, ntm = (p.M + BM - 1) / BM, ntiles = ntn * ntm;
  const int G = gridDim.x;
  const int slot = w_xcd_slot(blockIdx.x, G);
  const int mine = slot < ntiles ? (ntiles - 1 - slot) / G + 1 : 0;
  const int nk = (p.K + FBK - 1) / FBK;
  const int steps = mine * nk;
  if (steps == 0) return;

  WideLoader<BM, BN> ld;
  ld.init(p);
  int ikt = 0, itile = 0;  // the next step to issue: k-tile ikt of the workgroup's tile itile
  bf16_t* istage = smem;   // its stage
  auto next_tile = [&]() {  // a new tile's row offsets at its first k-step
    if (ikt == 0) {
      const int L = slot + itile * G, mt = L / ntn, nt = L - mt * ntn;
      ld.tile(p, mt * BM, nt * BN, wave, lane);
    }
  };
  auto advance = [&]() {
    if (++ikt == nk) {
      ikt = 0;
      ++itile;
    }
  };

  f32x4 acc[MT][NT];
#pragma unroll
  for (int i = 0; i < MT; ++i)
#pragma unroll
    for (int j = 0; j < NT; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  // prologue: steps 0 .. PF - 1; step 0 landed
#pragma unroll
  for (int t = 0; t < PF; ++t)
    if (t < steps) {
      next_tile();
      ld.all(ikt * FBK, p.K, smem + t * SE, wave);
      advance();
    }
  wide_wait<PIECES>(min(PF, steps) - 1);
  __builtin_amdgcn_s_barrier();
  if (grp == 1) __builtin_amdgcn_s_barrier();  // the stagger: waves 4-7 run one barrier (one phase) behind

  int cur = 0, kt = 0, tile = 0;
  s16x8 af[MT][2], bq[NT][2];
  for (int s = 0; s < steps; ++s) {
    const bf16_t* Ac = smem + cur * SE;
    const bf16_t* Bc = Ac + AE;
    const bool pre = s + PF < steps;
    if (pre) {  // step s + PF goes to the stage step s - 1 used
      next_tile();
      istage = smem + (cur == 0 ? ST - 1 : cur - 1) * SE;
    }
    const int ik0 = ikt * FBK;
    // ---- read phase: this k-step's fragments, the DMA of step s + PF
    W_STAMP(s, 0, 0);
    if (VCG_WIDE_ABL != 3 || s == 0) {
#pragma unroll
      for (int s2 = 0; s2 < 2; ++s2) {
#pragma unroll
        for (int j = 0; j < NT; ++j) bq[j][s2] = fast_frag(Bc, wc * (BN / 4) + j * 16, lane, s2);
#pragma unroll
        for (int i = 0; i < MT; ++i) af[i][s2] = fast_frag(Ac, grp * (BM / 2) + i * 16, lane, s2);
      }
    }
    if (pre && VCG_WIDE_ABL != 1) ld.all(ik0, p.K, istage, wave);
    W_STAMP(s, 0, 1);
    __builtin_amdgcn_s_waitcnt(0xC07F);  // lgkmcnt(0): the reads have landed before the barrier (the other group
                                         // refills this stage PF - 1 phases from now)
    W_STAMP(s, 0, 2);
    // waves 4-7 end their read phase with step s + 1 landed (their pieces of it); waves 0-3 read it after the
    // next barrier. Younger pieces in flight: steps s + 2 .. (the last issued)
    if (grp == 1 && s + 1 < steps && VCG_WIDE_ABL != 1)
      wide_wait<PIECES>(min(s + PF, steps - 1) - (s + 1));
    W_STAMP(s, 0, 3);
    __builtin_amdgcn_s_barrier();
    // ---- compute phase
    W_STAMP(s, 1, 0);
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_setprio(1);
    if (VCG_WIDE_ABL != 2) {
#pragma unroll
      for (int s2 = 0; s2 < 2; ++s2)
#pragma unroll
        for (int i = 0; i < MT; ++i)
#pragma unroll
          for (int j = 0; j < NT; ++j)
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bq[j][s2], af[i][s2], acc[i][j], 0, 0, 0);
    }
    __builtin_amdgcn_s_setprio(0);
    if (pre) advance();
    W_STAMP(s, 1, 1);
    // waves 0-3 end their compute phase with step s + 1 landed (before the epilogue's own loads / stores)
    if (grp == 0 && s + 1 < steps && VCG_WIDE_ABL != 1) wide_wait<PIECES>(min(s + PF, steps - 1) - (s + 1));
    W_STAMP(s, 1, 2);
    __builtin_amdgcn_sched_barrier(0);
    if (++kt == nk) {
      const int L = slot + tile * G, mt = L / ntn, nt = L - mt * ntn;
      wide_epilogue<MT, NT, WE>(acc, p, mt * BM + grp * (BM / 2) + (lane & 15), nt * BN + wc * (BN / 4) + 4 * (lane >> 4));
#pragma unroll
      for (int i = 0; i < MT; ++i)
#pragma unroll
        for (int j = 0; j < NT; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
      kt = 0;
      ++tile;
    }
    W_STAMP(s, 1, 3);
    __builtin_amdgcn_s_barrier();
    cur = cur == ST - 1 ? 0 : cur + 1;
  }
  if (grp == 0) __builtin_amdgcn_s_barrier();  // (the stagger's barrier count)
}

namespace {

int wide_cus() {
  static int n = 0;
  if (n == 0) {
    int dev = 0, c = 0;
    if (hipGetDevice(&dev) == hipSuccess && hipDeviceGetAttribute(&c, hipDeviceAttributeMultiprocessorCount, dev) ==
                                                hipSuccess && c > 0)
      n = c;
    else
      n = 256;
  }
  return n;
}

// Tile width from N alone (kernel selection must not depend on the batch: the oracle-anchored B = 1 step runs the
// kernels of the B = 64 bench): 256 for N >= 3072 in 256-column multiples, 192 where it divides N, else 128 -- the
// choices that measured fastest at the bench shapes (profiles/r06_bert_gemm.txt: N = 768 / 2304 -> 192, 3072 -> 256;
// the downsample input gradients' N = 256 / 512 / 1024 -> 128 by work per CU). VCG_WIDE_BN=128 / 192 / 256 forces one
// (tests and measurement; read per call).
int wide_bn_for(const GemmParams& p) {
  if (const char* e = getenv("VCG_WIDE_BN")) {
    const int v = atoi(e);
    if (v == 128 || v == 192 || v == 256) return v;
  }
  if (p.N >= 3072 && p.N % 256 == 0) return 256;
  return p.N % 192 == 0 ? 192 : 128;
}

template <int BN, int WE>
void launch_wide(const GemmParams& p, hipStream_t s) {
  constexpr int BM = 128;
  const long long tiles = (long long)((p.M + BM - 1) / BM) * ((p.N + BN - 1) / BN);
  const int grid = (int)(tiles < wide_cus() ? tiles : wide_cus());
  hipLaunchKernelGGL((gemm_wide_kernel<BM, BN, WE>), dim3(grid), dim3(512), 0, s, p);
}

template <int BN>
void launch_wide_we(const GemmParams& p, int we, hipStream_t s) {
  switch (we) {
    case WE_GELU: launch_wide<BN, WE_GELU>(p, s); break;
    case WE_GELU_BWD: launch_wide<BN, WE_GELU_BWD>(p, s); break;
    case WE_RES: launch_wide<BN, WE_RES>(p, s); break;
    case WE_RES32: launch_wide<BN, WE_RES32>(p, s); break;
    default: launch_wide<BN, WE_STORE>(p, s); break;
  }
}

}  // namespace

// The epilogue class of a vcg_gemm call this engine can run (-1: none): bf16, alpha 1, no batch, 16-B aligned rows
// and pointers, operands below the 4 GB buffer-descriptor range; act in {none, GELU (aux optional)}, or GELU' / an
// addend through `residual` (not aliasing the output)
int wide_gemm_class(const GemmParams& p) {
  if (p.alpha != 1.f || p.batch_inner > 0 || p.M <= 0 || p.N <= 0 || p.K <= 0) return -1;
  if (p.N % 8 != 0 || p.K % 8 != 0 || (p.ldc & 7) != 0 || (p.a.ld & 7) != 0 || (p.b.ld & 7) != 0) return -1;
  if ((((uintptr_t)p.C | (uintptr_t)p.a.ptr | (uintptr_t)p.b.ptr) & 15) != 0) return -1;
  if (p.a.bytes >= 0xFFFFFF00LL || p.b.bytes >= 0xFFFFFF00LL) return -1;
  if (p.bias && ((uintptr_t)p.bias & 15) != 0) return -1;
  if (p.aux && (p.act != ACT_GELU || ((uintptr_t)p.aux & 15) != 0)) return -1;
  if (p.residual) {
    if (p.residual == p.C || (p.ldr & 3) != 0 || ((uintptr_t)p.residual & 7) != 0) return -1;
    if (p.act == ACT_GELU_BWD) return WE_GELU_BWD;
    return p.act == ACT_NONE && !p.res_round ? WE_RES : -1;
  }
  if (p.act == ACT_GELU) return WE_GELU;
  return p.act == ACT_NONE ? WE_STORE : -1;
}

// the fp32 residual / output class (ACT_FLAG_F32_OUT): a plain bf16 GEMM plus an fp32 addend (16-B rows)
int wide_gemm_class_f32(const GemmParams& p) {
  if (!p.residual || p.aux || p.act != ACT_NONE || p.res_round || p.alpha != 1.f || p.batch_inner > 0) return -1;
  if (p.N % 8 != 0 || p.K % 8 != 0 || (p.ldc & 3) != 0 || (p.ldr & 3) != 0 || (p.a.ld & 7) != 0 || (p.b.ld & 7) != 0)
    return -1;
  if ((((uintptr_t)p.C | (uintptr_t)p.residual | (uintptr_t)p.a.ptr | (uintptr_t)p.b.ptr) & 15) != 0) return -1;
  if (p.a.bytes >= 0xFFFFFF00LL || p.b.bytes >= 0xFFFFFF00LL) return -1;
  if (p.bias && ((uintptr_t)p.bias & 15) != 0) return -1;
  return WE_RES32;
}

int run_gemm_wide(GemmParams& p, int we, hipStream_t s) {
  const int tk = timing_begin(s);
  switch (wide_bn_for(p)) {
    case 128: launch_wide_we<128>(p, we, s); break;
    case 256: launch_wide_we<256>(p, we, s); break;
    default: launch_wide_we<192>(p, we, s); break;
  }
  const double es = we == WE_RES32 ? 4.0 : 2.0;  // output / residual element size
  double bytes = 2.0 * ((double)p.M * p.K + (double)p.N * p.K) + es * p.M * (double)p.N;
  if (p.residual) bytes += es * p.M * (double)p.N;
  if (p.aux) bytes += 2.0 * p.M * (double)p.N;
  timing_end(tk, s, TIMING_WIDE_GEMM, 2.0 * p.M * p.N * (double)p.K, bytes);
  if (census_on()) { char t_[96]; snprintf(t_, sizeof(t_), "gemm_wide 128x%d we%d", wide_bn_for(p), we); census_add(t_, p.M, p.N, p.K); }
  VCG_LAUNCH_CHECK();
  return VCG_OK;
}

}  // namespace vcg

// the phase stamps of the last gemm_wide launch in a -DVCG_WIDE_STAMPS build (1 otherwise)
VCG_API int vcg_wide_stamps(unsigned long long* out, int n) {
#ifdef VCG_WIDE_STAMPS
  n = n < 256 ? n : 256;
  return hipMemcpyFromSymbol(out, HIP_SYMBOL(vcg::g_wide_stamps), (size_t)n * 8, 0, hipMemcpyDeviceToHost) == hipSuccess
             ? 0 : 2;
#else
  (void)out;
  (void)n;
  return 1;
#endif
}
