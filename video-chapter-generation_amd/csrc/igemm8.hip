// bf16 GEMM / implicit-GEMM conv for the compute-bound shapes: 256-row tiles, 8 waves in two ping-pong groups.
//
// The persistent 128 x 128 engine (igemm_fast.hip) runs two barriers per 64-deep k step and relies on two
// workgroups per CU to overlap them; on the K >= 256 GEMMs (3x3 convs, the wide 1x1 convs of layers 3-4, BERT) it
// sits at ~650-950 TF/s, the ceiling of that structure (cdna_hip_programming.md §5). This kernel follows the
// 256-row multi-phase schedule instead:
//   * one workgroup per CU, 8 waves = 2 groups (wr) x 4 column quarters (wc); a wave owns 128 rows x BN/4 columns
//     (8 x BN/64 fragments of 16 x 16, f32 accumulators in registers);
//   * a 64-deep k tile is 4 phases: (k-half 0, rows 0-63), (k-half 0, rows 64-127), (k-half 1, ...), each phase
//     = fragment ds_reads -> barrier -> 4 x BN/64 MFMAs -> barrier; group 1 runs one barrier behind group 0, so
//     on every SIMD one wave is in its MFMAs while the other reads LDS (each SIMD holds one wave of each group);
//   * LDS holds 2 k tiles as 8 k-HALF slots (A 256 x 32, B BN x 32): a k-half slot is free again two phases after
//     its last read, so one slot of LDS-DMA prefetch is issued per phase and 3 slots stay in flight across the
//     barriers (counted vmcnt, never 0 in the loop; raw s_barrier) -- the next tiles' loads are always landing;
//   * slot layout: 1-KiB blocks of 16 rows x 64 B, chunk-major (byte 16 (16 c + r) = row r, k 8c .. 8c + 7), so
//     a 16 x 32 fragment is ONE lane-linear ds_read_b128 and the LDS-DMA destination is lane-linear too (16 rows
//     x 64 B per wave instruction);
//   * epilogue: the finished tile's k-half-1 slots are idle until the next tile's phase 1, so the 256 x BN output
//     goes out through them in 4 staged rounds of 64 rows (16-B row chunks); EPI_STATS takes the BatchNorm
//     (mean, M2) of each wave's 128 rows (one 128-row slot of the stats buffer) from the accumulators, rounded
//     to bf16 as stored, with DPP row sums.
// Each output fragment accumulates its k32 steps in the same order as the 128 x 128 engine: bit-identical outputs.
#include "igemm.h"

namespace vcg {

typedef __attribute__((address_space(3))) void lds8_void_t;
typedef __attribute__((address_space(3))) char lds8_char;
__device__ __forceinline__ uint32_t lds8_u32(const void* p) { return (uint32_t)(uintptr_t)(const lds8_char*)p; }

enum { A8_DENSE = 0, A8_IM2COL = 1, A8_IM2COL_TSM = 2 };
#ifndef VCG_G8_STAGGER
#define VCG_G8_STAGGER 1  // group 1 one barrier behind group 0 (0: both groups in step)
#endif
#ifndef VCG_G8_PRIO
#define VCG_G8_PRIO 1     // s_setprio(1) around each phase's MFMAs
#endif

__device__ __forceinline__ constexpr int vm8(int n) {
  return (n & 0xF) | (0x7 << 4) | (0xF << 8) | (((n >> 4) & 3) << 14);
}

// LDS-DMA loader of one k-half slot (ROWS rows x 32 k): wave w fills 16-row blocks w * PER .. w * PER + PER - 1;
// lane l of a block instruction reads row (l & 15), k chunk (l >> 4). Gathers (C >= 64) keep the im2col state of
// igemm_fast.hip's FastLoader: one filter tap per 64-wide k tile, per-row tap masks, pixel base offsets.
template <int ROWS, int MODE> struct HalfLoader {
  static constexpr int PER = ROWS / (16 * 8);
  static constexpr bool GATHER = MODE != A8_DENSE;
  static constexpr bool TSM = MODE == A8_IM2COL_TSM;
  __amdgpu_buffer_rsrc_t rsrc;
  uint32_t oob;
  int kc;
  int off[PER], ra[PER], rb[PER], rc[PER];

  __device__ __forceinline__ void init(const OpArgs& a, int row0, int wave, int lane) {
    const uint32_t nbytes = (uint32_t)min(a.bytes, (long long)0xFFFFFF00LL);
    rsrc = __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(a.ptr), 0, nbytes, 0x00020000);
    oob = nbytes;
    kc = 8 * (lane >> 4);
#pragma clang loop unroll(full)
    for (int q = 0; q < PER; ++q) {
      const int gr = row0 + (wave * PER + q) * 16 + (lane & 15);
      const bool valid = gr < a.rows;
      if constexpr (!GATHER) {
        off[q] = valid ? (int)((long long)gr * a.ld) : -1;
      } else {
        const int n = gr / (a.GH * a.GW);
        const int rem = gr - n * a.GH * a.GW;
        const int y = rem / a.GW;
        const int x = rem - y * a.GW;
        off[q] = n * a.H * a.W * a.C;
        rc[q] = TSM ? (n % a.tsm_T) : 0;
        const int py = y * a.stride - a.pad, px = x * a.stride - a.pad;
        const int kh_lo = max(0, -py), kh_hi = min(a.KH, a.H - py);
        const int kw_lo = max(0, -px), kw_hi = min(a.KW, a.W - px);
        const int khi = min(max(kw_hi, 0), 31), klo = min(kw_lo, 31);
        const uint32_t cols = kw_hi > kw_lo ? (((1u << khi) - 1u) & ~((1u << klo) - 1u)) : 0u;
        uint32_t rows = 0;
#pragma unroll
        for (int kh = 0; kh < 8; ++kh) rows |= (kh >= kh_lo && kh < kh_hi) ? (1u << ((kh * a.KW) & 31)) : 0u;
        rb[q] = valid ? (int)(cols * rows) : 0;
        ra[q] = off[q] + (py * a.W + px) * a.C;
      }
    }
  }

  // k-half h of the 64-wide k tile at k0 into `slot` (byte address of the slot base)
  __device__ __forceinline__ void issue(const OpArgs& a, int k0, int h, int kend, char* slot, int wave) {
    if constexpr (GATHER) {
      const int tap = k0 >> a.logC;
      const int kh = tap / a.KW, kw = tap - (tap / a.KW) * a.KW;
      const int cb = (k0 & (a.C - 1)) + 32 * h;
      const int toff = (kh * a.W + kw) << a.logC;
      const uint32_t tbit = k0 < kend ? (1u << tap) : 0u;
#pragma clang loop unroll(full)
      for (int q = 0; q < PER; ++q) {
        const int c = cb + kc;
        bool ok = ((uint32_t)rb[q] & tbit) != 0u;
        int e = ra[q] + toff + c;
        if constexpr (TSM) {
          const int dt = c < a.tsm_fold ? 1 : (c < 2 * a.tsm_fold ? -1 : 0);
          ok = ok && ((unsigned)(rc[q] + dt) < (unsigned)a.tsm_T);
          e += dt * (a.H * a.W * a.C);
        }
        __builtin_amdgcn_raw_ptr_buffer_load_lds(rsrc, (lds8_void_t*)(slot + (wave * PER + q) * 1024), 16,
                                                 ok ? (uint32_t)e * 2u : oob, 0, 0, 0);
      }
    } else {
#pragma clang loop unroll(full)
      for (int q = 0; q < PER; ++q) {
        const int k = k0 + 32 * h + kc;
        const uint32_t voff = (off[q] >= 0 && k < kend) ? (uint32_t)(off[q] + k) * 2u : oob;
        __builtin_amdgcn_raw_ptr_buffer_load_lds(rsrc, (lds8_void_t*)(slot + (wave * PER + q) * 1024), 16, voff, 0, 0,
                                                 0);
      }
    }
  }
};

// fragment of rows r0 .. r0 + 15 (r0 % 16 == 0) of a k-half slot: lane 16 g + i gets row i, k 8 g .. 8 g + 7
__device__ __forceinline__ s16x8 frag8(const char* slot, int r0, int lane) {
  return *reinterpret_cast<const s16x8*>(slot + (r0 >> 4) * 1024 + lane * 16);
}

template <int BN> __device__ __forceinline__ int st8_slot(int row, int chunk) { return chunk ^ (row & 15); }

template <int BN, int AM, int EPI>
__global__ __launch_bounds__(512) __attribute__((amdgpu_waves_per_eu(1, 1)))
void igemm8_kernel(GemmParams p) {
  constexpr int NJ = BN / 64, WN = BN / 4;
  constexpr int AS = 256 * 64, BS = BN * 64, SLOT = AS + BS;  // a k-half slot pair: A then B
  constexpr int NA = 2, NB = BN / 128;                        // DMA instructions per thread per A / B slot
  constexpr int VMW = 2 * NA + NB;                            // 3 slots in flight across a wait
  static_assert(BN == 256 || BN == 128, "tile");
  __shared__ __attribute__((aligned(1024))) char smem[4 * SLOT];  // [buf][k-half]: the ONLY LDS object

  const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wr = wave >> 2, wc = wave & 3;
  const int g = lane >> 4, ci = lane & 15;
  const int nx = (p.N + BN - 1) / BN, gy = gridDim.x / nx;
  int bx, by;
  if ((gy & 7) == 0) {  // the column tiles of an M-tile row on one XCD
    const int sidx = blockIdx.x >> 3;
    bx = sidx % nx;
    by = (sidx / nx) * 8 + (blockIdx.x & 7);
  } else {
    bx = blockIdx.x % nx;
    by = blockIdx.x / nx;
  }
  const int n0 = bx * BN;
  const int mtiles = (p.M + 255) / 256;
  const int my_tiles = by < mtiles ? (mtiles - 1 - by) / gy + 1 : 0;
  if (my_tiles == 0) return;
  const int ktiles = (p.K + 63) / 64;
  const int total = my_tiles * ktiles;

  float bv[NJ][4];
#pragma unroll
  for (int j = 0; j < NJ; ++j) {
    const int n = n0 + wc * WN + 16 * j + 4 * g;
    float4 b4 = make_float4(0.f, 0.f, 0.f, 0.f);
    if (EPI == EPI_STORE && p.bias && n < p.N) b4 = *reinterpret_cast<const float4*>(p.bias + n);
    bv[j][0] = b4.x; bv[j][1] = b4.y; bv[j][2] = b4.z; bv[j][3] = b4.w;
  }
#pragma unroll
  for (int j = 0; j < NJ; ++j) asm volatile("" ::"v"(bv[j][0]), "v"(bv[j][1]), "v"(bv[j][2]), "v"(bv[j][3]));

  HalfLoader<256, AM> la0, la1;  // the tiles of the next k-half-0 / k-half-1 A issues
  HalfLoader<BN, A8_DENSE> lb;
  lb.init(p.b, n0, wave, lane);
  int c0t = 0, c0k = 0, c1t = 0, c1k = 0, cbk = 0, cbh = 0;  // issue cursors (local tile, k tile)
  la0.init(p.a, by * 256, wave, lane);
  la1.init(p.a, by * 256, wave, lane);
  auto slot = [&](int T, int h) { return smem + ((T & 1) * 2 + h) * SLOT; };
  // A k-half 0 of the next k tile in issue order
  auto issue_a0 = [&](int T) {
    if (T >= total) return;
    la0.issue(p.a, c0k * 64, 0, p.K, slot(T, 0), wave);
    if (++c0k == ktiles) {
      c0k = 0;
      if (++c0t < my_tiles) la0.init(p.a, (by + c0t * gy) * 256, wave, lane);
    }
  };
  auto issue_a1 = [&](int T) {
    if (T >= total) return;
    la1.issue(p.a, c1k * 64, 1, p.K, slot(T, 1), wave);
    if (++c1k == ktiles) {
      c1k = 0;
      if (++c1t < my_tiles) la1.init(p.a, (by + c1t * gy) * 256, wave, lane);
    }
  };
  auto issue_b = [&](int T, int h) {  // B k-half h of k tile T (cbk tracks T % ktiles)
    if (T >= total) return;
    lb.issue(p.b, cbk * 64, h, p.K, slot(T, h) + AS, wave);
    if (h == 1 && ++cbk == ktiles) cbk = 0;
  };

  f32x4 acc[8][NJ];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < NJ; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  // prologue: k tile 0 and the k-half-0 A slot of k tile 1 (the steady state's units issued before tile 0)
  issue_a0(0);
  issue_b(0, 0);
  issue_a1(0);
  issue_b(0, 1);
  issue_a0(1);
  __builtin_amdgcn_s_waitcnt(vm8(0));
  __builtin_amdgcn_s_barrier();
  if (VCG_G8_STAGGER && wr == 1) __builtin_amdgcn_s_barrier();  // group 1 runs one barrier behind

  const int mslots = (p.M + 127) / 128;
  int kt = 0, tile = 0;
  for (int T = 0; T < total; ++T) {
    const char* s0 = slot(T, 0);
    const char* s1 = slot(T, 1);
    s16x8 af[4], bfr[NJ];
#pragma unroll
    for (int ph = 0; ph < 4; ++ph) {
      const char* sa = ph < 2 ? s0 : s1;
      const int ib = (ph & 1) * 4;
#pragma unroll
      for (int i = 0; i < 4; ++i) af[i] = frag8(sa, wr * 128 + (ib + i) * 16, lane);
      if ((ph & 1) == 0) {
#pragma unroll
        for (int j = 0; j < NJ; ++j) bfr[j] = frag8(sa + AS, wc * WN + 16 * j, lane);
      }
      // one k-half slot of prefetch per phase; the slots it overwrites were last read >= 2 phases ago
      if (ph == 0) issue_b(T + 1, 0);
      else if (ph == 1) issue_a1(T + 1);
      else if (ph == 2) issue_b(T + 1, 1);
      else issue_a0(T + 2);
      if (ph == 1) {  // k-half 1 of tile T (read from phase 2) has landed once the 3 younger slots are in flight
        if (T + 1 < total) __builtin_amdgcn_s_waitcnt(vm8(VMW));
        else __builtin_amdgcn_s_waitcnt(vm8(0));
      } else if (ph == 3) {  // k-half 0 of tile T + 1
        if (T + 2 < total) __builtin_amdgcn_s_waitcnt(vm8(VMW));
        else __builtin_amdgcn_s_waitcnt(vm8(0));
      }
      __builtin_amdgcn_s_barrier();
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      if (VCG_G8_PRIO) __builtin_amdgcn_s_setprio(1);
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < NJ; ++j)
          acc[ib + i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bfr[j], af[i], acc[ib + i][j], 0, 0, 0);
      if (VCG_G8_PRIO) __builtin_amdgcn_s_setprio(0);
      __builtin_amdgcn_s_barrier();
    }
    if (++kt < ktiles) continue;
    // ---- epilogue of output tile `tile` (both groups in step: group 0 waits one barrier for group 1)
    kt = 0;
    if (VCG_G8_STAGGER && wr == 0) __builtin_amdgcn_s_barrier();
    const int m0 = (by + tile * gy) * 256;
    char* stage = smem + ((T & 1) * 2 + 1) * SLOT;  // the k-half-1 slots of the finished k tile (64 x BN bf16)
    // values as stored: EPI_STATS the conv output (rounded), EPI_STORE act(alpha * acc + bias)
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
      for (int j = 0; j < NJ; ++j)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          float v = acc[i][j][r];
          if constexpr (EPI == EPI_STORE) {
            v = v * p.alpha + bv[j][r];
            if (p.act != ACT_NONE) v = apply_act(v, p.act, p.fast_act);
          }
          acc[i][j][r] = bf2f(f2bf(v));
        }
    if constexpr (EPI == EPI_STATS) {  // (mean, M2) of this wave's 128 rows = stats slot m0 / 128 + wr
      const int r0 = m0 + wr * 128;
      const int cw = min(128, p.M - r0);
      if (cw > 0) {
        const float inv_cw = 1.f / (float)cw;
        const int slot_i = r0 >> 7;
#pragma unroll
        for (int j = 0; j < NJ; ++j)
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            float t = 0.f;
#pragma unroll
            for (int i = 0; i < 8; ++i) t += acc[i][j][r];  // rows beyond M are zero (zero A rows)
            const float mean = row16_sum(t) * inv_cw;
            float q = 0.f;
#pragma unroll
            for (int i = 0; i < 8; ++i) {
              const float d = acc[i][j][r] - mean;
              q += (i * 16 + ci < cw) ? d * d : 0.f;
            }
            q = row16_sum(q);
            const int col = n0 + wc * WN + 16 * j + 4 * g + r;
            if (ci == 0 && col < p.N)
              reinterpret_cast<float2*>(p.stats)[(long long)col * mslots + slot_i] = make_float2(mean, q);
          }
        if (wc == 0 && lane == 0)  // count row: stats[N][slot] = (rows, 0)
          reinterpret_cast<float2*>(p.stats)[(long long)p.N * mslots + slot_i] = make_float2((float)cw, 0.f);
      }
    }
    bf16_t* Cout = reinterpret_cast<bf16_t*>(p.C);
    constexpr int CPR = BN / 8, NCH = 64 * CPR / 512;  // 16-B chunks per row, per thread per round
#pragma unroll
    for (int rd = 0; rd < 4; ++rd) {  // round rd: rows 64 rd .. + 63 = group rd / 2, fragments 4 (rd & 1) .. + 3
      if (wr == (rd >> 1)) {
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
          for (int j = 0; j < NJ; ++j) {
            const f32x4& a4 = acc[(rd & 1) * 4 + i][j];
            const int row = i * 16 + ci, col = wc * WN + 16 * j + 4 * g;
            uint2 q2;
            q2.x = (uint32_t)f2bf(a4[0]) | ((uint32_t)f2bf(a4[1]) << 16);
            q2.y = (uint32_t)f2bf(a4[2]) | ((uint32_t)f2bf(a4[3]) << 16);
            asm volatile("ds_write_b64 %0, %1" ::"v"(lds8_u32(stage + row * (BN * 2) + 16 * st8_slot<BN>(row, col >> 3) +
                                                               2 * (col & 7))),
                         "v"(q2)
                         : "memory");
          }
      }
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();
      uint4 q[NCH];
#pragma unroll
      for (int k = 0; k < NCH; ++k) {
        const int id = tid + 512 * k, row = id / CPR, c = id - (id / CPR) * CPR;
        asm volatile("ds_read_b128 %0, %1" : "=v"(q[k]) : "v"(lds8_u32(stage + row * (BN * 2) + 16 * st8_slot<BN>(row, c)))
                     : "memory");
      }
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int k = 0; k < NCH; ++k) {
        const int id = tid + 512 * k, row = id / CPR, c = id - (id / CPR) * CPR;
        const int m = m0 + rd * 64 + row, n = n0 + 8 * c;
        if (m < p.M && n < p.N) *reinterpret_cast<uint4*>(Cout + (long long)m * p.ldc + n) = q[k];
      }
      __builtin_amdgcn_s_barrier();  // the stage is read before the next round rewrites it
    }
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
      for (int j = 0; j < NJ; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
    if (++tile < my_tiles && VCG_G8_STAGGER && wr == 1) __builtin_amdgcn_s_barrier();  // back to one behind
  }
}

// 256-row kernel for the compute-bound GEMMs of run_fast_gemm: EPI_STORE (bias / activation, no residual / aux)
// and EPI_STATS (conv forward); A dense or im2col (C >= 64, TSM fused); K >= 256; z == 1. OPT-IN (VCG_G8=1: every
// eligible shape; VCG_G8=2: where the tile-count model prefers it): measured slower than the 128 x 128 engine on
// every trunk / BERT shape (tools/bench_gemm.py VCG_BENCH_G8) -- the ping-pong stagger and s_setprio
// change nothing, so the phases are bound by their fixed barrier / ds_read / DMA-issue cost, not by MFMA overlap.
static int g8_mode() {
  const char* e = getenv("VCG_G8");  // read per call (A/B in one process)
  if (e && e[0] == '1') return 2;
  if (e && e[0] == '2') return 1;
  return 0;
}

template <int BN, int AM, int EPI>
static int launch_g8(const GemmParams& p, hipStream_t s) {
  const int nx = (p.N + BN - 1) / BN, mtiles = (p.M + 255) / 256;
  int gy = max(1, 256 / nx);
  if (gy >= 8) gy &= ~7;
  if (gy > mtiles) gy = mtiles >= 8 ? (mtiles & ~7) : mtiles;
  const int tk = timing_begin(s);
  hipLaunchKernelGGL((igemm8_kernel<BN, AM, EPI>), dim3(nx * gy), dim3(512), 0, s, p);
  const double mn = (double)p.M * p.N;
  const double bytes = (AM == A8_DENSE ? 2.0 * p.M * (double)p.K : (double)p.a.bytes) + 2.0 * p.N * (double)p.K + 2.0 * mn;
  timing_end(tk, s, TIMING_FAST_GEMM, 2.0 * mn * p.K, bytes);
  VCG_LAUNCH_CHECK();
  return VCG_OK;
}

// amode: igemm.h OP_DENSE_K / OP_IM2COL (p.a.tsm_fold > 0: TSM); returns -1 where the kernel does not apply
int run_gemm8(const GemmParams& p, int amode, int epi, int z, hipStream_t s) {
  const int mode = g8_mode();
  if (mode == 0 || z != 1 || p.batch_inner > 0 || p.K < 256 || p.residual || p.aux || !p.C ||
      (epi != EPI_STORE && epi != EPI_STATS))
    return -1;
  if (p.N % 128 != 0 || (p.ldc & 7) != 0 || ((uintptr_t)p.C & 15) != 0 || (p.act & ~0xFF) != 0) return -1;
  const OpArgs& a = p.a;
  int am;
  if (amode == OP_DENSE_K) {
    am = A8_DENSE;
  } else if (amode == OP_IM2COL && a.C >= 64 && a.sw == 0 && a.tKW == 0 && a.KH * a.KW <= 32) {
    am = a.tsm_fold > 0 ? A8_IM2COL_TSM : A8_IM2COL;
  } else {
    return -1;
  }
  if (a.bytes >= 0xFFFFFF00LL || p.b.bytes >= 0xFFFFFF00LL) return -1;
  const char* e128 = getenv("VCG_G8_BN128");  // A/B: 256 x 128 tiles on N % 256 == 0 too
  const int BN = (p.N % 256 == 0 && !(e128 && e128[0] == '1')) ? 256 : 128;
  if (mode == 1) {
    // tile-count model: rounds of the resident grid (256 workgroups of 256 x BN here, 512 of 128 x 128 there),
    // this kernel's tile counted as the work of 2 x BN / 128 128 x 128 tiles at 1.35x their rate
    const double t8 = (double)((p.M + 255) / 256) * ((p.N + BN - 1) / BN);
    const double t1 = (double)((p.M + 127) / 128) * ((p.N + 127) / 128);
    const double r8 = ceil(t8 / 256.0) * (2.0 * BN / 128) / 1.35, r1 = ceil(t1 / 512.0);
    if (r8 >= r1) return -1;
  }
#define VCG_G8_EPI(BNV, AMV)                                                                       \
  return epi == EPI_STATS ? launch_g8<BNV, AMV, EPI_STATS>(p, s) : launch_g8<BNV, AMV, EPI_STORE>(p, s)
  if (BN == 256) {
    if (am == A8_DENSE) VCG_G8_EPI(256, A8_DENSE);
    if (am == A8_IM2COL) VCG_G8_EPI(256, A8_IM2COL);
    VCG_G8_EPI(256, A8_IM2COL_TSM);
  }
  if (am == A8_DENSE) VCG_G8_EPI(128, A8_DENSE);
  if (am == A8_IM2COL) VCG_G8_EPI(128, A8_IM2COL);
  VCG_G8_EPI(128, A8_IM2COL_TSM);
#undef VCG_G8_EPI
}

}  // namespace vcg
