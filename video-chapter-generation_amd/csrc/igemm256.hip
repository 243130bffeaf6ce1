// 256 x 256-tile bf16 GEMM engine for the compute-bound convolutions and dense layers (K-contiguous A and B, D = A B^T:
// conv forward with the im2col / TSM gather, conv input gradients with the dgrad gather, BERT linears).
//
// The 128 x 128 engine (igemm_fast.hip) runs two barriers per 64-deep k-step with every wave in lockstep: its MFMA
// phases and its LDS / LDS-DMA phases never overlap inside a CU (~900 TF/s ceiling, MI355X guide §5). Here one
// 512-thread workgroup per CU owns a 256 x 256 tile; each wave a 128 x 64 sub-tile (8 x 4 fragments of 16 x 16: twice
// the FLOP per LDS byte of a 64 x 64 sub-tile). A 64-deep k-step is four phases, one C quadrant (4 x 2 fragments, 16
// MFMAs) each, in a serpentine order so that every phase reads only half of the next fragments:
//   q0: A rows 0-63 + B cols 0-31 -> quadrant (0, 0);   q1: B cols 32-63 -> (0, 1)
//   q2: A rows 64-127 -> (1, 1);                          q3: B cols 0-31 -> (1, 0)
// and every phase is [fragment reads + LDS-DMA issue] s_barrier [MFMAs] s_barrier. Waves 4-7 start one barrier late
// (a stagger), so on each SIMD one wave computes while its partner reads and issues: the MFMA pipe stays busy across
// the barriers (MI355X_MICROARCH.md "Two waves per SIMD", cdna_hip_programming.md §5 "The 256^2 8-phase template").
// Operands: two k-tile buffers (A and B halves of 128 x 64 bf16 = 16 KiB each, 128 KiB), the next k-tile's LDS-DMA
// issued in phases q1 (A halves) and q2 (B halves) of the current one -- after every wave's reads of the buffer it
// refills have retired (the partner group's last reads of it were waited for two barriers earlier) -- and retired by
// vmcnt(0) in q3, a full phase later, so no LDS-DMA latency is exposed; raw s_barrier only (never __syncthreads, which
// would drain the in-flight DMA).
#include "fastload.h"

namespace vcg {

namespace {

constexpr int G_HALF = 128 * FBK;  // elements of one operand half-tile [128][64]

typedef __attribute__((address_space(3))) char g_lds_char;
__device__ __forceinline__ uint32_t g_lds_u32(const void* p) { return (uint32_t)(uintptr_t)(const g_lds_char*)p; }

// bijective remap of the launch order so that consecutive tiles (sharing A rows) run on one XCD (blocks b and b + 8
// share an XCD): XCD x gets the contiguous tile range [x q + min(x, r), ...) of n = 8 q + r tiles
__device__ __forceinline__ int g_xcd_tile(int b, int n) {
  const int q = n >> 3, r = n & 7, x = b & 7;
  return (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + (b >> 3);
}

__device__ __forceinline__ void g_unpack8(const uint4& u, float (&v)[8]) {
  const uint32_t w[4] = {u.x, u.y, u.z, u.w};
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    v[2 * i] = __uint_as_float(w[i] << 16);
    v[2 * i + 1] = __uint_as_float(w[i] & 0xffff0000u);
  }
}

// output staging: [256][256] bf16 = 128 KiB (both operand buffers), 16-B chunk c of row r at slot c ^ (r & 15)
__device__ __forceinline__ uint32_t g_stage_addr(const bf16_t* st, int row, int col) {
  return g_lds_u32(st + row * 256 + 8 * ((col >> 3) ^ (row & 15)) + (col & 7));
}

// profiling build (make EXTRA=-DVCG_G256_STAMPS ...): s_memtime of waves 0 and 4 of workgroup 0 at the 4 points of
// every phase of k-tiles 8..15 (before / after the first barrier, after the MFMAs, after the second barrier)
#ifdef VCG_G256_STAMPS
__device__ unsigned long long g_g256_stamps[2 * 8 * 4 * 4];
#define G_STAMP(t, q, k)                                                                                         \
  do {                                                                                                           \
    if (blockIdx.x == 0 && (tid == 0 || tid == 256) && (t) >= 8 && (t) < 16)                                    \
      g_g256_stamps[(((tid >> 8) * 8 + (t) - 8) * 4 + (q)) * 4 + (k)] = __builtin_amdgcn_s_memtime();           \
  } while (0)
#else
#define G_STAMP(t, q, k) do {} while (0)
#endif

template <int AM, int EPI, int PH>
__global__ __launch_bounds__(512) void gemm256_kernel(GemmParams p) {
  __shared__ __attribute__((aligned(1024))) bf16_t smem[8 * G_HALF];  // [buffer][A0, A1, B0, B1][128][64]
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wr = wave >> 2, wc = wave & 3;  // sub-tile rows wr * 128, cols wc * 64
  const int nx = (p.N + 255) >> 8, my = (p.M + 255) >> 8;
  const int tile = g_xcd_tile(blockIdx.x, nx * my);
  const int by = tile / nx, bx = tile - by * nx;
  const int m0 = by * 256, n0 = bx * 256;
  const int nk = (p.K + FBK - 1) / FBK;

  FastLoader<128, AM, 8> la0, la1;
  FastLoader<128, OP_DENSE_K, 8> lb0, lb1;
  la0.init(p.a, 0, m0, wave, lane);
  la1.init(p.a, 0, m0 + 128, wave, lane);
  lb0.init(p.b, 0, n0, wave, lane);
  lb1.init(p.b, 0, n0 + 128, wave, lane);

  f32x4 acc[8][4];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  // prologue: k-tile 0 into buffer 0
  la0.issue(p.a, 0, p.K, smem + 0 * G_HALF, wave);
  la1.issue(p.a, 0, p.K, smem + 1 * G_HALF, wave);
  lb0.issue(p.b, 0, p.K, smem + 2 * G_HALF, wave);
  lb1.issue(p.b, 0, p.K, smem + 3 * G_HALF, wave);
  __builtin_amdgcn_s_waitcnt(waitcnt_vm(0));
  __builtin_amdgcn_s_barrier();
  if (wr == 1) __builtin_amdgcn_s_barrier();  // the stagger: waves 4-7 run one barrier (half a phase) behind

  // PH = 4 prefetch of the next k-tile, a two-phase window for every piece: q0 the A quarters of rows 0-63 (last
  // read in q0 of the previous k-step), q1 the B halves (last read in q3), q2 the A quarters of rows 64-127 (last read
  // in q2); the end of q1's read segment retires this k-tile's rows 64-127 (vmcnt(6)), the end of q3's the next
  // k-tile's rows 0-63 and B (vmcnt(2))
  s16x8 af[4][2], bf[2][2];
  FastLoader<64, AM, 8> lq0, lq1, lq2, lq3;  // A quarters: half 0 rows 0-63 / 64-127, half 1 rows 0-63 / 64-127
  lq0.init(p.a, 0, m0, wave, lane);
  lq1.init(p.a, 0, m0 + 64, wave, lane);
  lq2.init(p.a, 0, m0 + 128, wave, lane);
  lq3.init(p.a, 0, m0 + 192, wave, lane);
  if constexpr (PH == 4) for (int t = 0; t < nk; ++t) {
    const int cur = t & 1;
    const bool pre = t + 1 < nk;
    const bf16_t* Ah = smem + (cur * 4 + wr) * G_HALF;
    const bf16_t* Bh = smem + (cur * 4 + 2 + (wc >> 1)) * G_HALF;
    bf16_t* nb = smem + ((cur ^ 1) * 4) * G_HALF;
    const int bc = (wc & 1) * 64;  // this wave's columns inside its B half
    // ---- q0: A rows 0-63, B cols 0-31 -> quadrant (0, 0)
#pragma unroll
    for (int s2 = 0; s2 < 2; ++s2) {
#pragma unroll
      for (int i = 0; i < 4; ++i) af[i][s2] = fast_frag(Ah, i * 16, lane, s2);
#pragma unroll
      for (int j = 0; j < 2; ++j) bf[j][s2] = fast_frag(Bh, bc + j * 16, lane, s2);
    }
    if (pre) {
      lq0.issue(p.a, (t + 1) * FBK, p.K, nb + 0 * G_HALF, wave);
      lq2.issue(p.a, (t + 1) * FBK, p.K, nb + 1 * G_HALF, wave);
    }
    G_STAMP(t, 0, 0);
    __builtin_amdgcn_s_barrier();
    G_STAMP(t, 0, 1);
    __builtin_amdgcn_s_waitcnt(0xC07F);  // lgkmcnt(0)
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int s2 = 0; s2 < 2; ++s2)
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bf[j][s2], af[i][s2], acc[i][j], 0, 0, 0);
    __builtin_amdgcn_s_setprio(0);
    G_STAMP(t, 0, 2);
    __builtin_amdgcn_s_barrier();
    G_STAMP(t, 0, 3);
    // ---- q1: B cols 32-63 -> quadrant (0, 1); LDS-DMA of the next k-tile's A halves
#pragma unroll
    for (int s2 = 0; s2 < 2; ++s2)
#pragma unroll
      for (int j = 0; j < 2; ++j) bf[j][s2] = fast_frag(Bh, bc + 32 + j * 16, lane, s2);
    if (pre) lb0.issue(p.b, (t + 1) * FBK, p.K, nb + 2 * G_HALF, wave);
    if (pre) lb1.issue(p.b, (t + 1) * FBK, p.K, nb + 3 * G_HALF, wave);
    if (t > 0) {
      if (pre) __builtin_amdgcn_s_waitcnt(waitcnt_vm(6));
      else __builtin_amdgcn_s_waitcnt(waitcnt_vm(0));
    }  // this k-tile's rows 64-127 have landed
    G_STAMP(t, 1, 0);
    __builtin_amdgcn_s_barrier();
    G_STAMP(t, 1, 1);
    __builtin_amdgcn_s_waitcnt(0xC07F);
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int s2 = 0; s2 < 2; ++s2)
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j)
          acc[i][2 + j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bf[j][s2], af[i][s2], acc[i][2 + j], 0, 0, 0);
    __builtin_amdgcn_s_setprio(0);
    G_STAMP(t, 1, 2);
    __builtin_amdgcn_s_barrier();
    G_STAMP(t, 1, 3);
    // ---- q2: A rows 64-127 -> quadrant (1, 1); LDS-DMA of the next k-tile's B halves
#pragma unroll
    for (int s2 = 0; s2 < 2; ++s2)
#pragma unroll
      for (int i = 0; i < 4; ++i) af[i][s2] = fast_frag(Ah, 64 + i * 16, lane, s2);
    if (pre) {
      lq1.issue(p.a, (t + 1) * FBK, p.K, nb + 0 * G_HALF + 64 * FBK, wave);
      lq3.issue(p.a, (t + 1) * FBK, p.K, nb + 1 * G_HALF + 64 * FBK, wave);
    }
    G_STAMP(t, 2, 0);
    __builtin_amdgcn_s_barrier();
    G_STAMP(t, 2, 1);
    __builtin_amdgcn_s_waitcnt(0xC07F);
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int s2 = 0; s2 < 2; ++s2)
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j)
          acc[4 + i][2 + j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bf[j][s2], af[i][s2], acc[4 + i][2 + j], 0, 0, 0);
    __builtin_amdgcn_s_setprio(0);
    G_STAMP(t, 2, 2);
    __builtin_amdgcn_s_barrier();
    G_STAMP(t, 2, 3);
    // ---- q3: B cols 0-31 -> quadrant (1, 0); the next k-tile's LDS-DMA retired (read after the next barrier)
#pragma unroll
    for (int s2 = 0; s2 < 2; ++s2)
#pragma unroll
      for (int j = 0; j < 2; ++j) bf[j][s2] = fast_frag(Bh, bc + j * 16, lane, s2);
    if (pre) __builtin_amdgcn_s_waitcnt(waitcnt_vm(2));  // the next k-tile's rows 0-63 and B have landed
    G_STAMP(t, 3, 0);
    __builtin_amdgcn_s_barrier();
    G_STAMP(t, 3, 1);
    __builtin_amdgcn_s_waitcnt(0xC07F);
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int s2 = 0; s2 < 2; ++s2)
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j)
          acc[4 + i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bf[j][s2], af[i][s2], acc[4 + i][j], 0, 0, 0);
    __builtin_amdgcn_s_setprio(0);
    G_STAMP(t, 3, 2);
    __builtin_amdgcn_s_barrier();
    G_STAMP(t, 3, 3);
  }
  // PH = 2: two phases of 32 MFMAs per k-step: p0 = A rows 0-63 of the wave's half x all its 64 columns, p1 = A rows
  // 64-127 (the B fragments stay in registers). Prefetch of the next k-tile with a two-phase window for every piece:
  // p0 issues the B halves and the A quarters of rows 0-63 (their last reads, p0 of the previous k-step, were waited
  // for two barriers earlier by both groups), p1 the A quarters of rows 64-127 (ditto for p1); the end of p1's read
  // segment retires p0's pieces (vmcnt(2): the two of p1 stay in flight), the end of the next p0's retires p1's
  // (vmcnt(6)).
  s16x8 bq[4][2];
  if constexpr (PH == 2) {
    for (int t = 0; t < nk; ++t) {
      const int cur = t & 1;
      const bool pre = t + 1 < nk;
      const bf16_t* Ah = smem + (cur * 4 + wr) * G_HALF;
      const bf16_t* Bh = smem + (cur * 4 + 2 + (wc >> 1)) * G_HALF;
      bf16_t* nb = smem + ((cur ^ 1) * 4) * G_HALF;
      const int bc = (wc & 1) * 64;
#pragma unroll
      for (int s2 = 0; s2 < 2; ++s2) {
#pragma unroll
        for (int i = 0; i < 4; ++i) af[i][s2] = fast_frag(Ah, i * 16, lane, s2);
#pragma unroll
        for (int j = 0; j < 4; ++j) bq[j][s2] = fast_frag(Bh, bc + j * 16, lane, s2);
      }
      if (pre) {
        lb0.issue(p.b, (t + 1) * FBK, p.K, nb + 2 * G_HALF, wave);
        lb1.issue(p.b, (t + 1) * FBK, p.K, nb + 3 * G_HALF, wave);
        lq0.issue(p.a, (t + 1) * FBK, p.K, nb + 0 * G_HALF, wave);
        lq2.issue(p.a, (t + 1) * FBK, p.K, nb + 1 * G_HALF, wave);
      }
      if (t > 0) {
      if (pre) __builtin_amdgcn_s_waitcnt(waitcnt_vm(6));
      else __builtin_amdgcn_s_waitcnt(waitcnt_vm(0));
    }  // this k-tile's rows 64-127 have landed
      G_STAMP(t, 0, 0);
      __builtin_amdgcn_s_barrier();
      G_STAMP(t, 0, 1);
      __builtin_amdgcn_s_waitcnt(0xC07F);
      __builtin_amdgcn_sched_barrier(0);
      __builtin_amdgcn_s_setprio(1);
#pragma unroll
      for (int s2 = 0; s2 < 2; ++s2)
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
          for (int j = 0; j < 4; ++j)
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bq[j][s2], af[i][s2], acc[i][j], 0, 0, 0);
      __builtin_amdgcn_s_setprio(0);
      G_STAMP(t, 0, 2);
      __builtin_amdgcn_s_barrier();
      G_STAMP(t, 0, 3);
#pragma unroll
      for (int s2 = 0; s2 < 2; ++s2)
#pragma unroll
        for (int i = 0; i < 4; ++i) af[i][s2] = fast_frag(Ah, 64 + i * 16, lane, s2);
      if (pre) {
        lq1.issue(p.a, (t + 1) * FBK, p.K, nb + 0 * G_HALF + 64 * FBK, wave);
        lq3.issue(p.a, (t + 1) * FBK, p.K, nb + 1 * G_HALF + 64 * FBK, wave);
        __builtin_amdgcn_s_waitcnt(waitcnt_vm(2));  // the next k-tile's B and rows 0-63 have landed
      }
      G_STAMP(t, 1, 0);
      __builtin_amdgcn_s_barrier();
      G_STAMP(t, 1, 1);
      __builtin_amdgcn_s_waitcnt(0xC07F);
      __builtin_amdgcn_sched_barrier(0);
      __builtin_amdgcn_s_setprio(1);
#pragma unroll
      for (int s2 = 0; s2 < 2; ++s2)
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
          for (int j = 0; j < 4; ++j)
            acc[4 + i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bq[j][s2], af[i][s2], acc[4 + i][j], 0, 0, 0);
      __builtin_amdgcn_s_setprio(0);
      G_STAMP(t, 1, 2);
      __builtin_amdgcn_s_barrier();
      G_STAMP(t, 1, 3);
    }
  }
  if (wr == 0) __builtin_amdgcn_s_barrier();  // (the stagger's barrier count)

  // ---- epilogue: act(alpha acc + bias) staged through LDS as [256][256] bf16, then 16-B row chunks
  const int g = lane >> 4, ci = lane & 15;
  bf16_t* st = smem;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int col = wc * 64 + j * 16 + 4 * g;
    float bv[4] = {0.f, 0.f, 0.f, 0.f};
    if (EPI == EPI_STORE && p.bias && n0 + col < p.N) {
      const float4 b4 = *reinterpret_cast<const float4*>(p.bias + n0 + col);
      bv[0] = b4.x; bv[1] = b4.y; bv[2] = b4.z; bv[3] = b4.w;
    }
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const int row = wr * 128 + i * 16 + ci;
      float v[4];
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        float x = acc[i][j][r];
        if constexpr (EPI == EPI_STORE) {
          x = x * p.alpha + bv[r];
          if (p.act != ACT_NONE && p.act != ACT_GELU_BWD) x = apply_act(x, p.act, p.fast_act);
        }
        v[r] = x;
      }
      uint2 q;
      q.x = (uint32_t)f2bf(v[0]) | ((uint32_t)f2bf(v[1]) << 16);
      q.y = (uint32_t)f2bf(v[2]) | ((uint32_t)f2bf(v[3]) << 16);
      asm volatile("ds_write_b64 %0, %1" ::"v"(g_stage_addr(st, row, col)), "v"(q) : "memory");
    }
  }
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  bf16_t* Cout = reinterpret_cast<bf16_t*>(p.C);
  // EPI_STATS (conv outputs): shifted per-column sums of the stored bf16 values (shift = the thread's first value;
  // a thread always owns the 8-column chunk tid % 32), merged below with Chan's formula in thread order
  int cnt = 0;
  float sh[8], s1[8], s2[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) sh[i] = s1[i] = s2[i] = 0.f;
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    uint4 q[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      const int id = tid + 512 * (8 * h + k);
      const int row = id >> 5, c = id & 31;
      asm volatile("ds_read_b128 %0, %1" : "=v"(q[k]) : "v"(g_stage_addr(st, row, 8 * c)) : "memory");
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      const int id = tid + 512 * (8 * h + k);
      const int row = id >> 5, c = id & 31;
      const int m = m0 + row, n = n0 + 8 * c;
      if (m < p.M && n < p.N) {
        if (Cout) *reinterpret_cast<uint4*>(Cout + (long long)m * p.ldc + n) = q[k];
        if constexpr (EPI == EPI_STATS) {
          float v[8];
          g_unpack8(q[k], v);
          if (cnt == 0) {
#pragma unroll
            for (int i = 0; i < 8; ++i) sh[i] = v[i];
          }
          ++cnt;
#pragma unroll
          for (int i = 0; i < 8; ++i) {
            const float d = v[i] - sh[i];
            s1[i] += d;
            s2[i] = fmaf(d, d, s2[i]);
          }
        }
      }
    }
  }
  if constexpr (EPI == EPI_STATS) {
    // slot `by` of the stats buffer ([N + 1][ceil(M / 128)] float2): (mean, M2) per column, then the count row
    // (rows of the slot; slot 0's second word = the number of slots used, my); slots my.. are marked empty
    const int mslots = (p.M + 127) / 128;
    float* scratch = reinterpret_cast<float*>(smem);
    __syncthreads();  // every thread has read the stage
    const float nf = (float)cnt, inv = cnt > 0 ? 1.f / nf : 0.f;
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      scratch[(0 * 512 + tid) * 8 + i] = sh[i] + s1[i] * inv;                       // mean
      scratch[(1 * 512 + tid) * 8 + i] = fmaxf(s2[i] - s1[i] * s1[i] * inv, 0.f);  // M2
    }
    scratch[2 * 512 * 8 + tid] = nf;
    __syncthreads();
    if (tid < 256 && n0 + tid < p.N) {
      const int c = tid >> 3, i = tid & 7;
      float na = 0.f, mean = 0.f, m2 = 0.f;
      for (int t = c; t < 512; t += 32) {
        const float nb = scratch[2 * 512 * 8 + t];
        if (nb > 0.f) {
          const float mb = scratch[t * 8 + i], m2b = scratch[(512 + t) * 8 + i];
          const float nt = na + nb, d = mb - mean;
          mean += d * (nb / nt);
          m2 += m2b + d * d * (na * nb / nt);
          na = nt;
        }
      }
      reinterpret_cast<float2*>(p.stats)[(long long)(n0 + tid) * mslots + by] = make_float2(mean, m2);
    }
    if (bx == 0 && tid == 0) {
      const float rows = (float)min(256, p.M - m0);
      float2* cntrow = reinterpret_cast<float2*>(p.stats) + (long long)p.N * mslots;
      cntrow[by] = make_float2(rows, by == 0 ? (float)my : 0.f);
      for (int t = by + my; t < mslots; t += my) cntrow[t] = make_float2(0.f, 0.f);
    }
  }
}

}  // namespace

// 1 when the 256-tile engine takes this GEMM: bf16 K-contiguous operands below 4 GB, EPI_STORE / EPI_STATS without
// residual / aux, unbatched, N a multiple of 8 (16-B output chunks). VCG_G256=1 / 2 routes every such GEMM here (4 /
// 2 phases per k-step), 0 none; unset, the one class measured faster goes here: the 3x3 forward convs with their BN
// statistics at N >= 512, K >= 4096 (layer 4: 215.5 vs 256.4 us, tools/bench_g256.py, profiles/r05_g256.txt)
static int g256_mode() {
  const char* e = getenv("VCG_G256");  // (read per call: tests and benches switch it inside one process)
  return e ? atoi(e) : -1;
}

static bool g256_default(const GemmParams& p, int amode, int epi) {
  return amode == OP_IM2COL && epi == EPI_STATS && p.N >= 512 && p.K >= 4096;
}

bool gemm256_ok(const GemmParams& p, int amode, int epi, int z) {
  const int mode = g256_mode();
  if (mode == 0 || (mode < 0 && !g256_default(p, amode, epi))) return false;
  if (z != 1 || p.batch_inner > 0 || (epi != EPI_STORE && epi != EPI_STATS) || p.residual ||
      p.aux)
    return false;
  if (epi == EPI_STATS && (p.bias || !p.stats)) return false;
  if (p.N % 8 != 0 || (p.ldc & 7) != 0 || ((uintptr_t)p.C & 15) != 0) return false;
  if (p.bias && (((uintptr_t)p.bias & 15) != 0)) return false;
  if (amode != OP_DENSE_K && amode != OP_IM2COL && amode != OP_IM2COL_TSM && amode != OP_DGRAD) return false;
  // (the default class takes its GEMMs whatever M: the oracle-anchored B = 1 step runs the B = 64 bench's kernels;
  // forced modes keep the tile-count floor)
  const long long tiles = (long long)((p.M + 255) / 256) * ((p.N + 255) / 256);
  return (mode < 0 || tiles >= 128) && p.K >= 256;
}

static double g256_bytes(const GemmParams& p, int amode) {
  return (amode == OP_DENSE_K ? 2.0 * p.M * (double)p.K : (double)p.a.bytes) + 2.0 * p.N * (double)p.K +
         2.0 * p.M * (double)p.N;
}

template <int EPI, int PH>
static void launch256(const GemmParams& p, int amode, int tiles, hipStream_t s) {
  switch (amode) {
    case OP_DENSE_K: hipLaunchKernelGGL((gemm256_kernel<OP_DENSE_K, EPI, PH>), dim3(tiles), dim3(512), 0, s, p); break;
    case OP_IM2COL: hipLaunchKernelGGL((gemm256_kernel<OP_IM2COL, EPI, PH>), dim3(tiles), dim3(512), 0, s, p); break;
    case OP_IM2COL_TSM:
      hipLaunchKernelGGL((gemm256_kernel<OP_IM2COL_TSM, EPI, PH>), dim3(tiles), dim3(512), 0, s, p);
      break;
    default: hipLaunchKernelGGL((gemm256_kernel<OP_DGRAD, EPI, PH>), dim3(tiles), dim3(512), 0, s, p); break;
  }
}

int run_gemm256(const GemmParams& p, int amode, int epi, hipStream_t s) {
  const int tiles = ((p.M + 255) / 256) * ((p.N + 255) / 256);
  const int tk = timing_begin(s);
  const bool two = g256_mode() != 1;  // (two 32-MFMA phases per k-step unless VCG_G256=1: four of 16)
  if (epi == EPI_STATS) two ? launch256<EPI_STATS, 2>(p, amode, tiles, s) : launch256<EPI_STATS, 4>(p, amode, tiles, s);
  else two ? launch256<EPI_STORE, 2>(p, amode, tiles, s) : launch256<EPI_STORE, 4>(p, amode, tiles, s);
  timing_end(tk, s, TIMING_FAST_GEMM, 2.0 * p.M * p.N * (double)p.K, g256_bytes(p, amode));
  if (census_on()) { char t_[96]; snprintf(t_, sizeof(t_), "gemm256 a%d e%d ph%d", amode, epi, two ? 2 : 4); census_add(t_, p.M, p.N, p.K); }
  VCG_LAUNCH_CHECK();
  return VCG_OK;
}

}  // namespace vcg

// the phase stamps of the last gemm256 launch in a -DVCG_G256_STAMPS build (1 otherwise)
VCG_API int vcg_g256_stamps(unsigned long long* out, int n) {
#ifdef VCG_G256_STAMPS
  n = n < 256 ? n : 256;
  return hipMemcpyFromSymbol(out, HIP_SYMBOL(vcg::g_g256_stamps), (size_t)n * 8, 0, hipMemcpyDeviceToHost) == hipSuccess
             ? 0 : 2;
#else
  (void)out;
  (void)n;
  return 1;
#endif
}
