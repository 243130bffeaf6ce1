// bf16 fast path of the implicit-GEMM engine for K-contiguous operands
// (conv fwd with im2col/TSM gather, conv dgrad gather, dense linear layers / QK^T).
//
// Differences to the generic kernel (igemm.hip):
//   * BK = 64 (two 16x16x32 MFMA k-steps per barrier pair);
//   * operands go global -> LDS directly with buffer_load ... lds (LDS-DMA, 16 B per lane,
//     1 KiB per wave instruction, no VGPR staging); conv zero padding / out-of-range rows come for
//     free from the buffer descriptor's range check (out-of-range offset -> zeros);
//   * LDS tile [rows][64] bf16 with 128-B rows, 16-B chunk c of row r at slot c ^ ((r >> 1) & 7):
//     the global source address is pre-swizzled (LDS stays lane-linear, as LDS-DMA requires) and
//     the fragment ds_read_b64s of a 32-lane half hit 64 distinct banks;
//   * two LDS stages; tile t+1 is in flight while tile t is computed; counted vmcnt + raw
//     s_barrier (never __syncthreads, which would drain the in-flight DMA).
#include "fastload.h"

namespace vcg {

// ---- output staging through LDS: full-row 16-B stores instead of 8-B row fragments ----------------
// The output tile goes out in rounds of 128 rows (one round at BM = 128, two at BM = 256: the waves of
// M-rows 2h, 2h+1 put round h). A round lives in the finished stage `cur`: BN = 128 -> rows 0..63 at stA
// and rows 64..127 at stB ([64][128] each; BM = 256 passes stB = stA + 64 * 128, its A part holds the
// whole round); BN = 64 -> the whole [128][64] round at stA. 16-B chunks are XOR-swizzled per row
// (conflict-free 8-B writes of a 16-row fragment and 16-B reads of a row). LDS accesses are inline asm
// with explicit lgkmcnt waits.
typedef __attribute__((address_space(3))) char lds_char;
__device__ __forceinline__ uint32_t lds_u32(const void* p) { return (uint32_t)(uintptr_t)(const lds_char*)p; }

template <int BN> __device__ __forceinline__ int st_slot(int row, int chunk) {
  if constexpr (BN == 128) return chunk ^ (row & 15);
  else return chunk ^ ((row >> 1) & 7);
}

template <int BM, int BN>
__device__ __forceinline__ void stage_put(bf16_t* stA, bf16_t* stB, int wm, int wn, int lane, int i, int j,
                                          const float (&v)[4]) {
  const int g = lane >> 4, ci = lane & 15;
  const int trow = (wm & 1) * 64 + i * 16 + ci;        // row in the 128-row round
  const int tcol = wn * (BN / 2) + j * 16 + 4 * g;     // first of 4 columns
  bf16_t* reg = (BN == 128 && trow >= 64) ? stB : stA;
  const int row = BN == 128 ? (trow & 63) : trow;
  const uint32_t addr = lds_u32(reg + row * BN + 8 * st_slot<BN>(row, tcol >> 3) + (tcol & 7));
  uint2 q;
  q.x = (uint32_t)f2bf(v[0]) | ((uint32_t)f2bf(v[1]) << 16);
  q.y = (uint32_t)f2bf(v[2]) | ((uint32_t)f2bf(v[3]) << 16);
  asm volatile("ds_write_b64 %0, %1" ::"v"(addr), "v"(q) : "memory");
}

// all waves' stage_put done -> 16-B row chunks to global (rows >= M / cols >= N skipped)
// (m0: first row of the round)
template <int BM, int BN>
__device__ __forceinline__ void stage_flush(const bf16_t* stA, const bf16_t* stB, const GemmParams& p, bf16_t* Cout,
                                            int m0, int n0, int mlim) {
  constexpr int NTH = BM * 2, CPR = BN / 8, NCH = 128 * BN / 8;
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  uint4 q[NCH / NTH];
#pragma unroll
  for (int k = 0; k < NCH / NTH; ++k) {
    const int id = threadIdx.x + NTH * k;
    const int trow = id / CPR, c = id - trow * CPR;
    const bf16_t* reg = (BN == 128 && trow >= 64) ? stB : stA;
    const int row = BN == 128 ? (trow & 63) : trow;
    const uint32_t addr = lds_u32(reg + row * BN + 8 * st_slot<BN>(row, c));
    asm volatile("ds_read_b128 %0, %1" : "=v"(q[k]) : "v"(addr) : "memory");
  }
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_sched_barrier(0);
#pragma unroll
  for (int k = 0; k < NCH / NTH; ++k) {
    const int id = threadIdx.x + NTH * k;
    const int trow = id / CPR, c = id - trow * CPR;
    const int m = m0 + trow, n = n0 + 8 * c;
    if (m < mlim && n < p.N) *reinterpret_cast<uint4*>(Cout + (long long)m * p.ldc + n) = q[k];
  }
  __builtin_amdgcn_s_barrier();  // every wave has read the stage before the next step's DMA refills it
}

// EPI_STORE (no residual / aux) through the stage
template <int BM, int BN>
__device__ __forceinline__ void epilogue_staged(f32x4 (&acc)[4][BN / 32], const GemmParams& p,
                                                const float (&bv)[BN / 32][4], bf16_t* Cout, bf16_t* stA,
                                                bf16_t* stB, int m0, int n0, int wm, int wn, int lane, int mlim) {
  constexpr int MT = 4, NT = BN / 32;
#pragma unroll
  for (int h = 0; h < BM / 128; ++h) {
    if ((wm >> 1) == h) {
#pragma unroll
      for (int j = 0; j < NT; ++j)
#pragma unroll
        for (int i = 0; i < MT; ++i) {
          float v[4];
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            float t = acc[i][j][r] * p.alpha + bv[j][r];
            if (p.act != ACT_NONE && p.act != ACT_GELU_BWD) t = apply_act(t, p.act, p.fast_act);
            v[r] = t;
          }
          stage_put<BM, BN>(stA, stB, wm, wn, lane, i, j, v);
        }
    }
    stage_flush<BM, BN>(stA, stB, p, Cout, m0 + 128 * h, n0, mlim);
  }
}

// EPI_STORE_AUX: the pre-activation values (bias added) to p.aux, then the activated values to Cout, each a
// staged round of its own
template <int BM, int BN>
__device__ __forceinline__ void epilogue_staged_aux(f32x4 (&acc)[4][BN / 32], const GemmParams& p,
                                                    const float (&bv)[BN / 32][4], bf16_t* Cout, bf16_t* stA,
                                                    bf16_t* stB, int m0, int n0, int wm, int wn, int lane) {
  constexpr int MT = 4, NT = BN / 32;
  static_assert(BM == 128, "EPI_STORE_AUX runs on 128-row tiles");
#pragma unroll
  for (int pass = 0; pass < 2; ++pass) {
#pragma unroll
    for (int j = 0; j < NT; ++j)
#pragma unroll
      for (int i = 0; i < MT; ++i) {
        float v[4];
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const float t = acc[i][j][r] * p.alpha + bv[j][r];
          v[r] = pass == 0 ? t : apply_act(t, p.act, p.fast_act);
        }
        stage_put<BM, BN>(stA, stB, wm, wn, lane, i, j, v);
      }
    stage_flush<BM, BN>(stA, stB, p, pass == 0 ? reinterpret_cast<bf16_t*>(p.aux) : Cout, m0, n0, p.M);
  }
}

// ---- EPI_BWD (igemm.h BwdEpi): conv-dgrad epilogue of the trunk backward ------------------------------
// Per-column parameters live in LDS (cpar[4][BN]: mean, msc, msh, mean2 of the workgroup's BN columns);
// a thread of the flush always owns the same 8-column chunk c = tid % (BN / 8), so its per-column sums stay
// in registers for the whole kernel and are combined across threads once at the end (bwd_finish).
__device__ __forceinline__ void unpack8(const uint4& u, float (&v)[8]) {
  const uint32_t w[4] = {u.x, u.y, u.z, u.w};
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    v[2 * i] = __uint_as_float(w[i] << 16);
    v[2 * i + 1] = __uint_as_float(w[i] & 0xffff0000u);
  }
}

// EPI_STORE + residual + ReLU through the stage (the running-statistics bn3 folded into conv3: relu(x W'^T + b + res),
// trunk.py _conv3_folded): the GEMM value is rounded to bf16 in the stage -- as the unfolded path stores y3 -- and the
// residual is added per 16-B row chunk in the flush, so both the residual loads and the output stores are full rows.
// ACT_GELU_BWD: the residual is the pre-activation and the output dh * GELU'(pre), dh rounded to bf16 first (as
// torch autocast's bf16 matmul output feeding gelu_backward)
template <int BM, int BN, bool GELU_BWD>
__device__ __forceinline__ void epilogue_staged_res(f32x4 (&acc)[4][BN / 32], const GemmParams& p,
                                                    const float (&bv)[BN / 32][4], bf16_t* Cout, const bf16_t* Res,
                                                    bf16_t* stA, bf16_t* stB, int m0, int n0, int wm, int wn,
                                                    int lane, int mlim) {
  constexpr int MT = 4, NT = BN / 32, NTH = BM * 2, CPR = BN / 8, KC = 128 * BN / 8 / NTH;
  static_assert(BM == 128, "128-row tiles");
#pragma unroll
  for (int j = 0; j < NT; ++j)
#pragma unroll
    for (int i = 0; i < MT; ++i) {
      float v[4];
#pragma unroll
      for (int r = 0; r < 4; ++r) v[r] = acc[i][j][r] * p.alpha + bv[j][r];
      stage_put<BM, BN>(stA, stB, wm, wn, lane, i, j, v);
    }
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  uint4 q[KC], rv[KC];
#pragma unroll
  for (int k = 0; k < KC; ++k) {  // residual rows first (clamped to a valid row; discarded below)
    const int id = threadIdx.x + NTH * k;
    const int trow = id / CPR, c = id - trow * CPR;
    const int m = min(m0 + trow, mlim - 1), n = min(n0 + 8 * c, p.N - 8);
    rv[k] = *reinterpret_cast<const uint4*>(Res + (long long)m * p.ldr + n);
  }
#pragma unroll
  for (int k = 0; k < KC; ++k) {
    const int id = threadIdx.x + NTH * k;
    const int trow = id / CPR, c = id - trow * CPR;
    const bf16_t* reg = (BN == 128 && trow >= 64) ? stB : stA;
    const int row = BN == 128 ? (trow & 63) : trow;
    const uint32_t addr = lds_u32(reg + row * BN + 8 * st_slot<BN>(row, c));
    asm volatile("ds_read_b128 %0, %1" : "=v"(q[k]) : "v"(addr) : "memory");
  }
  float rsc[8], rsh[8];  // an affine residual (p.res_sc): this thread's 8 columns are the same for every k
  if (p.res_sc) {
    const int nc = min(n0 + 8 * (int)(threadIdx.x % CPR), p.N - 8);
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      rsc[e] = p.res_sc[nc + e];
      rsh[e] = p.res_sh[nc + e];
    }
  }
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_sched_barrier(0);
#pragma unroll
  for (int k = 0; k < KC; ++k) {
    const int id = threadIdx.x + NTH * k;
    const int trow = id / CPR, c = id - trow * CPR;
    const int m = m0 + trow, n = n0 + 8 * c;
    float a[8], r[8];
    unpack8(q[k], a);
    unpack8(rv[k], r);
    if (p.res_sc) {
#pragma unroll
      for (int e = 0; e < 8; ++e) r[e] = fmaf(r[e], rsc[e], rsh[e]);
    }
    uint32_t mb = 0;  // ReLU mask of the output (p.obits): bit e = out > 0, as vcg_bn_apply writes it
    if constexpr (GELU_BWD) {  // BERT FFN2's input gradient: dh * GELU'(pre), dh rounded as stored
#pragma unroll
      for (int e = 0; e < 8; ++e) a[e] *= p.fast_act ? gelu_erf_grad_fast(r[e]) : gelu_erf_grad(r[e]);
    } else {
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        a[e] = apply_act(a[e] + r[e], p.act);
        mb |= (a[e] > 0.f ? 1u : 0u) << e;
      }
    }
    uint4 o;
    o.x = (uint32_t)f2bf(a[0]) | ((uint32_t)f2bf(a[1]) << 16);
    o.y = (uint32_t)f2bf(a[2]) | ((uint32_t)f2bf(a[3]) << 16);
    o.z = (uint32_t)f2bf(a[4]) | ((uint32_t)f2bf(a[5]) << 16);
    o.w = (uint32_t)f2bf(a[6]) | ((uint32_t)f2bf(a[7]) << 16);
    if (m < mlim && n < p.N) {
      *reinterpret_cast<uint4*>(Cout + (long long)m * p.ldc + n) = o;
      if (p.obits) p.obits[((long long)m * p.N + n) >> 3] = (uint8_t)mb;
    }
  }
  __builtin_amdgcn_s_barrier();  // every wave has read the stage before the next step's DMA refills it
}

template <int BM, int BN, bool LIGHT>
__device__ __forceinline__ void stage_flush_bwd(const bf16_t* stA, const bf16_t* stB, const GemmParams& p,
                                                bf16_t* Cout, int m0, int n0, const float* cpar, float (&s1)[8],
                                                float (&s2)[8], float (&s3)[8], int mlim) {
  constexpr int NTH = BM * 2, CPR = BN / 8, NCH = 128 * BN / 8, KC = NCH / NTH;
#ifdef VCG_EPI_KB
  constexpr int KB = KC < VCG_EPI_KB ? KC : VCG_EPI_KB;
#else
  constexpr int KB = KC < 4 ? KC : (BM == 256 ? 2 : 4);
#endif
  const BwdEpi& e = p.bwd;
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  uint4 q[KC];
#pragma unroll
  for (int k = 0; k < KC; ++k) {
    const int id = threadIdx.x + NTH * k;
    const int trow = id / CPR, c = id - trow * CPR;
    const bf16_t* reg = (BN == 128 && trow >= 64) ? stB : stA;
    const int row = BN == 128 ? (trow & 63) : trow;
    const uint32_t addr = lds_u32(reg + row * BN + 8 * st_slot<BN>(row, c));
    asm volatile("ds_read_b128 %0, %1" : "=v"(q[k]) : "v"(addr) : "memory");
  }
  const int c = threadIdx.x % CPR;
  const int lc = 8 * c, n = n0 + lc;
  float mu[8], sc[8], sh[8], mu2[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    mu[i] = cpar[lc + i];
    sc[i] = cpar[BN + lc + i];
    sh[i] = cpar[2 * BN + lc + i];
    mu2[i] = cpar[3 * BN + lc + i];
  }
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_sched_barrier(0);
  int shift = 0;  // TSM adjoint: this column group's values move one frame later (+1) / earlier (-1)
  if (!LIGHT && e.tsm_T > 0) shift = n < e.tsm_fold ? 1 : (n < 2 * e.tsm_fold ? -1 : 0);
  const bf16_t* res = LIGHT ? nullptr : reinterpret_cast<const bf16_t*>(e.res);
  const bf16_t* yp = reinterpret_cast<const bf16_t*>(e.y);
  const bf16_t* y2p = LIGHT ? nullptr : reinterpret_cast<const bf16_t*>(e.y2);
  const uint8_t* bitsp = LIGHT ? nullptr : e.bits;
  // (rows beyond mlim / columns beyond N are clamped to a valid address and discarded after the load: a load
  // under a per-element condition makes hipcc branch around it and wait vmcnt(0) per element, i.e. one HBM round
  // trip per chunk; each operand's loads sit under ONE uniform branch per batch instead: l1 / l2 / l3 conv1 fused
  // dgrads 1453 / 760 / 421 -> 1354 / 615 / 355 us, tools/bench_dgrad.py. Rejected: pulling the next tile's
  // residual / y rows into L2 by LDS-DMA pieces into a scratch slot after each flush, +15-20 %.)
  const int nc = min(n, p.N - 8);
#pragma unroll
  for (int k0 = 0; k0 < KC; k0 += KB) {
    long long off[KB], roff[KB];
    bool ok[KB], src[KB], rok[KB];
    uint4 rv[KB], yv[KB], y2v[KB];
    uint32_t bv[KB];
#pragma unroll
    for (int kk = 0; kk < KB; ++kk) {  // addresses of the batch
      const int id = threadIdx.x + NTH * (k0 + kk);
      const int mr = m0 + id / CPR;
      ok[kk] = mr < mlim && n < p.N;
      const int m = min(mr, mlim - 1);
      src[kk] = true;
      int dst = m;
      if (e.sub) {  // sub-pixel class row -> dx row
        const uint32_t f = fdiv((uint32_t)m, e.fd_chw), r = (uint32_t)m - f * e.fd_chw.d;
        const uint32_t i = fdiv(r, e.fd_cw), j = r - i * (uint32_t)e.cW;
        dst = (int)((f * e.fH + 2 * i + e.ry) * e.fW + 2 * j + e.rx);
      }
      if (shift != 0) {
        const int f = (int)fdiv((uint32_t)m, e.fd_hw);
        const int t = f - (int)fdiv((uint32_t)f, e.fd_T) * e.tsm_T;
        const bool edge = shift > 0 ? t == e.tsm_T - 1 : t == 0;
        src[kk] = !edge;
        dst = edge ? m - shift * (e.tsm_T - 1) * e.hw : m + shift * e.hw;
      }
      off[kk] = (long long)dst * p.ldc + n;
      roff[kk] = (long long)dst * p.ldc + nc;
      rok[kk] = true;
      if (!LIGHT && e.res_s > 1) {  // compact residual of a 1x1 / stride-2 conv: only even (h, w) rows carry one
        const uint32_t f = fdiv((uint32_t)dst, e.fd_hw), r = (uint32_t)dst - f * (uint32_t)e.hw;
        const uint32_t h = fdiv(r, e.fd_w), w = r - h * e.fd_w.d;
        rok[kk] = ((h | w) & 1u) == 0;
        roff[kk] = ((long long)(f * e.rH + (h >> 1)) * e.rW + (w >> 1)) * p.ldc + nc;
      }
    }
    const long long* loff = off;  // y / y2 / bits rows (column clamped below)
    if (res) {
#pragma unroll
      for (int kk = 0; kk < KB; ++kk) rv[kk] = *reinterpret_cast<const uint4*>(res + roff[kk]);
    }
    if (bitsp) {
#pragma unroll
      for (int kk = 0; kk < KB; ++kk) bv[kk] = bitsp[(loff[kk] - n + nc) >> 3];
    }
    if (yp) {
#pragma unroll
      for (int kk = 0; kk < KB; ++kk) yv[kk] = *reinterpret_cast<const uint4*>(yp + loff[kk] - n + nc);
    }
    if (y2p) {
#pragma unroll
      for (int kk = 0; kk < KB; ++kk) y2v[kk] = *reinterpret_cast<const uint4*>(y2p + loff[kk] - n + nc);
    }
#pragma unroll
    for (int kk = 0; kk < KB; ++kk) {
      if (!rok[kk]) rv[kk] = make_uint4(0u, 0u, 0u, 0u);
    }
#pragma unroll
    for (int kk = 0; kk < KB; ++kk) {
      if (!ok[kk]) continue;
      float v[8];
      unpack8(q[k0 + kk], v);
      if (!src[kk]) {
#pragma unroll
        for (int i = 0; i < 8; ++i) v[i] = 0.f;
      }
      if (res) {
        float r[8];
        unpack8(rv[kk], r);
#pragma unroll
        for (int i = 0; i < 8; ++i) v[i] += r[i];
      }
      if (bitsp) {
#pragma unroll
        for (int i = 0; i < 8; ++i) v[i] = ((bv[kk] >> i) & 1u) ? v[i] : 0.f;
      }
      float yy[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
      if (yp) {
        unpack8(yv[kk], yy);
        if (e.msc) {
#pragma unroll
          for (int i = 0; i < 8; ++i) v[i] = fmaf(yy[i], sc[i], sh[i]) > 0.f ? v[i] : 0.f;
        }
      }
      uint4 o;
      o.x = (uint32_t)f2bf(v[0]) | ((uint32_t)f2bf(v[1]) << 16);
      o.y = (uint32_t)f2bf(v[2]) | ((uint32_t)f2bf(v[3]) << 16);
      o.z = (uint32_t)f2bf(v[4]) | ((uint32_t)f2bf(v[5]) << 16);
      o.w = (uint32_t)f2bf(v[6]) | ((uint32_t)f2bf(v[7]) << 16);
      *reinterpret_cast<uint4*>(Cout + off[kk]) = o;
      if (e.nred > 0) {
        unpack8(o, v);  // statistics of the stored (rounded) gradient
#pragma unroll
        for (int i = 0; i < 8; ++i) {
          s1[i] += v[i];
          s2[i] = yp ? fmaf(v[i], yy[i] - mu[i], s2[i]) : s2[i];
        }
        if (y2p) {
          float y2[8];
          unpack8(y2v[kk], y2);
#pragma unroll
          for (int i = 0; i < 8; ++i) s3[i] = fmaf(v[i], y2[i] - mu2[i], s3[i]);
        }
      }
    }
  }
  __builtin_amdgcn_s_barrier();  // every wave has read the stage before the next step's DMA refills it
}

// Combine the per-thread column sums of EPI_BWD (threads tid = c (mod BN/8) share columns 8c..8c+7) in a
// fixed order and write this workgroup's partial slot; scratch = the (idle) stage buffers.
template <int BM, int BN>
__device__ __forceinline__ void bwd_finish(const GemmParams& p, float* scratch, const float* cpar_invstd,
                                           const float (&s1)[8], const float (&s2)[8], const float (&s3)[8], int n0,
                                           int slot) {
  constexpr int NTH = BM * 2, CPR = BN / 8;
  const int nred = p.bwd.nred;
  __syncthreads();
  const int tid = threadIdx.x;
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    scratch[(0 * NTH + tid) * 8 + i] = s1[i];
    scratch[(1 * NTH + tid) * 8 + i] = s2[i];
    scratch[(2 * NTH + tid) * 8 + i] = s3[i];
  }
  __syncthreads();
  if (tid < BN && n0 + tid < p.N) {
    const int c = tid >> 3, i = tid & 7;
    float a[3] = {0.f, 0.f, 0.f};
    for (int t = c; t < NTH; t += CPR)
#pragma unroll
      for (int r = 0; r < 3; ++r) a[r] += scratch[(r * NTH + t) * 8 + i];
    float* out = p.bwd.part + (long long)slot * nred * p.N + n0 + tid;
    out[0] = a[0];
    out[p.N] = a[1] * cpar_invstd[tid];
    if (nred > 2) out[2 * p.N] = a[2] * cpar_invstd[BN + tid];
  }
}

// ---- EPI_STATS: the BatchNorm statistics of the stored (bf16) conv output, from the staged rounds ---------
// A flush thread always owns the same 8-column chunk c = tid % (BN / 8); it keeps shifted sums of the
// values it stores (shift = its first value per column: no cancellation when |mean| >> std) for the whole
// kernel: count, sh[8], s1[8] = sum (v - sh), s2[8] = sum (v - sh)^2.
template <int BM, int BN>
__device__ __forceinline__ void stage_flush_stats(const bf16_t* stA, const bf16_t* stB, const GemmParams& p,
                                                  bf16_t* Cout, int m0, int n0, int& cnt, float (&sh)[8],
                                                  float (&s1)[8], float (&s2)[8], int mlim) {
  constexpr int NTH = BM * 2, CPR = BN / 8, NCH = 128 * BN / 8, KC = NCH / NTH;
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  uint4 q[KC];
#pragma unroll
  for (int k = 0; k < KC; ++k) {
    const int id = threadIdx.x + NTH * k;
    const int trow = id / CPR, c = id - trow * CPR;
    const bf16_t* reg = (BN == 128 && trow >= 64) ? stB : stA;
    const int row = BN == 128 ? (trow & 63) : trow;
    const uint32_t addr = lds_u32(reg + row * BN + 8 * st_slot<BN>(row, c));
    asm volatile("ds_read_b128 %0, %1" : "=v"(q[k]) : "v"(addr) : "memory");
  }
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_sched_barrier(0);
  const int c = threadIdx.x % CPR;
  const int n = n0 + 8 * c;
#pragma unroll
  for (int k = 0; k < KC; ++k) {
    const int id = threadIdx.x + NTH * k;
    const int m = m0 + id / CPR;
    if (m < mlim && n < p.N) {
      if (Cout) *reinterpret_cast<uint4*>(Cout + (long long)m * p.ldc + n) = q[k];  // (null: statistics only)
      float v[8];
      unpack8(q[k], v);
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
  __builtin_amdgcn_s_barrier();  // every wave has read the stage before the next step's DMA refills it
}

// Per-thread (count, mean, M2) of every column chunk, merged across the threads that share the chunk with
// Chan's formula in thread order (deterministic) -> stats[col][by] = (mean, M2) and the count row
// stats[N][by]; slots by + k*gy (k >= 1) are marked empty. scratch = the idle stage buffers.
template <int BM, int BN>
__device__ __forceinline__ void stats_finish(const GemmParams& p, float* scratch, int cnt, const float (&sh)[8],
                                             const float (&s1)[8], const float (&s2)[8], int n0, int by, int bx,
                                             int gy, int mslots) {
  constexpr int NTH = BM * 2, CPR = BN / 8;
  __syncthreads();  // all LDS-DMA retired (the last step waited vmcnt(0)); the stage buffers are free
  const int tid = threadIdx.x;
  const float nf = (float)cnt, inv = cnt > 0 ? 1.f / nf : 0.f;
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    scratch[(0 * NTH + tid) * 8 + i] = sh[i] + s1[i] * inv;                 // mean
    scratch[(1 * NTH + tid) * 8 + i] = fmaxf(s2[i] - s1[i] * s1[i] * inv, 0.f);  // M2
  }
  scratch[2 * NTH * 8 + tid] = nf;
  __syncthreads();
  if (tid < BN && n0 + tid < p.N) {
    const int c = tid >> 3, i = tid & 7;
    float na = 0.f, mean = 0.f, m2 = 0.f;
    for (int t = c; t < NTH; t += CPR) {
      const float nb = scratch[2 * NTH * 8 + t];
      if (nb > 0.f) {
        const float mb = scratch[t * 8 + i], m2b = scratch[(NTH + t) * 8 + i];
        const float nt = na + nb, d = mb - mean;
        mean += d * (nb / nt);
        m2 += m2b + d * d * (na * nb / nt);
        na = nt;
      }
    }
    reinterpret_cast<float2*>(p.stats)[(long long)(n0 + tid) * mslots + by] = make_float2(mean, m2);
  }
  if (bx == 0 && tid == 0) {
    float rows = 0.f;  // threads 0..CPR-1 cover every row of the workgroup once (one chunk column each)
    for (int t = 0; t < NTH; t += CPR) rows += scratch[2 * NTH * 8 + t];
    float2* cntrow = reinterpret_cast<float2*>(p.stats) + (long long)p.N * mslots;
    cntrow[by] = make_float2(rows, by == 0 ? (float)gy : 0.f);  // slot 0 also tells bn_finalize: gy slots used
    for (int t = by + gy; t < mslots; t += gy) cntrow[t] = make_float2(0.f, 0.f);
  }
}


// Profiling build (make EXTRA=-DVCG_FAST_STAMPS OUT=... OBJDIR=...): s_memtime per tile phase of workgroup 0,
// wave 0 of every igemm_fast launch (the last launch's survive): tile's first k-step, after its last MFMAs,
// after the output staging, after the epilogue flush. vcg_fast_stamps() copies them out.
#ifdef VCG_FAST_STAMPS
__device__ unsigned long long g_fast_stamps[64 * 4];
#define FAST_STAMP(t, k)                                                                       \
  do {                                                                                         \
    if (blockIdx.x == 0 && threadIdx.x == 0 && (t) < 64) g_fast_stamps[(t) * 4 + (k)] = __builtin_amdgcn_s_memtime(); \
  } while (0)
#else
#define FAST_STAMP(t, k) do {} while (0)
#endif

// ---- EPI_BWD_STREAM: the fused 1x1 conv input gradient (EPI_BWD) with K <= 128, as a streaming kernel ----------
// For the trunk's conv1 dgrads of layers 1-2 (K = 64 / 128 input channels of dy) the GEMM is a small part of the
// work: per 64 x 64 output tile the A rows are 8-16 KB, the epilogue reads the residual, y (the previous block's
// bn3 input) and the mask bits (16.5 KB, + 8 KB y2 after a downsample block) and writes 8 KB of g. The persistent
// 2-stage engine above issues those epilogue loads only after a tile's MFMAs (two dependent HBM round trips per
// tile: 3.6-4.3 TB/s). Here every operand of a tile is DMA'd into an LDS ring NBUF - 1 tiles ahead; the weight
// tile (64 columns x K) stays in LDS for the whole kernel.
// Tiles are DESTINATION rows d of g: the TSM adjoint moves the dgrad value of GEMM row m to d = m + s hw for the
// columns of shift s (+1: n < fold, -1: fold <= n < 2 fold, 0: the rest), so d's value is the product of the A row
// d - s hw (zero when that frame is outside the clip -- the wrap row of the adjoint -- and the clip-edge rows are
// never read, i.e. dropped). The shift is applied to the A rows (a wave's 32 columns have one shift: fold % 32 == 0;
// a workgroup whose 64 columns straddle two shifts loads two A tiles), so the residual / y / mask / g rows of a tile
// are plain contiguous rows (full 128-B lines; moving them instead costs 35 % at the layer-1 shape).
// Per tile: counted vmcnt (the ring's later tiles and the previous flushes' stores stay in flight), one barrier,
// MFMAs of a 16 x 32 block per wave, the bf16 value staged through LDS, one barrier, then each thread combines one
// 16-B chunk of stage + LDS operands and stores it. Same products, order and rounding as stage_flush_bwd
// (bit-identical g; per-thread column sums combined in a fixed order by bwd_finish).
constexpr int XF_HASY = 1;  // y + mask bits present (the BN sums of the previous block's bn3)
constexpr int XF_BITS = 4;  // mask bits without y: sum g only (the previous block's y3 is not stored, trunk.py)
constexpr int XF_Y2 = 2;    // y2 present (the previous block's downsample BN)
// with XF_BITS: P = g^T a2 of the previous block (a2 of 64 columns: layer 1) accumulated from the stored g tile, so
// the separate weight-gradient GEMM that re-read g and a2 for bn3's sum_gx (trunk.py) is gone; the weight fragments
// then sit in registers to keep the ring at 3-4 slots. (128 a2 columns -- layer 2 -- cost the dgrad as much as the
// GEMM they replace: tools/bench_dgrad_p.py, +212 us vs 225 us; not built.)
constexpr int XF_P64 = 8;
typedef unsigned int pk_u32x4 __attribute__((ext_vector_type(4)));
// transposed LDS read (4 bf16 per lane) as inline asm: a plain LDS read makes hipcc wait vmcnt(0) for the ring's DMA
__device__ __forceinline__ void lds_tr_b16(s16x4& v, const bf16_t* p) {
  asm volatile("ds_read_b64_tr_b16 %0, %1" : "=v"(v) : "v"(lds_u32(p)) : "memory");
}

__device__ __forceinline__ int bwd_tsm_shift(const BwdEpi& e, int n) {
  if (e.tsm_T <= 0) return 0;
  return n < e.tsm_fold ? 1 : (n < 2 * e.tsm_fold ? -1 : 0);
}

// K = 256 (KC = 4, layer 3): one A tile per slot (the host admits it only when no workgroup's 64 columns straddle two
// TSM shifts) and the weight fragments of a wave's 32 columns in registers (64 VGPRs) instead of LDS, so the ring
// keeps 3 slots (with the weights in LDS and one A tile per slot it had 2, measured step-neutral in round 4).
__host__ __device__ constexpr bool bwd_stream_wide(int KC) { return KC > 2; }
__host__ __device__ constexpr int bwd_stream_pj(int XF) { return (XF & XF_P64) ? 64 : 0; }
__host__ __device__ constexpr bool bwd_stream_breg(int KC, int XF) { return KC > 2 || bwd_stream_pj(XF) > 0; }
__host__ __device__ constexpr int bwd_stream_na(int KC, int XF) { return KC > 2 ? 1 : 2; }
// LDS bytes of one ring slot / of the fixed part (weights, stage, column parameters) and the ring depth
__host__ __device__ constexpr int bwd_stream_buf(int KC, int XF) {
  return bwd_stream_na(KC, XF) * KC * 8192 + 8192 + ((XF & XF_HASY) ? 8192 : 0) +
         ((XF & (XF_HASY | XF_BITS)) ? 8 * 256 : 0) + ((XF & XF_Y2) ? 8192 : 0) + bwd_stream_pj(XF) * 128;
}
#ifndef VCG_STREAM_NBUF
#define VCG_STREAM_NBUF 4  // ring slots at most (build knob for A/B builds)
#endif
__host__ __device__ constexpr int bwd_stream_fixed(int KC, int XF) {
  return (bwd_stream_breg(KC, XF) ? 0 : KC * 8192) + 8192 + 1024;
}
__host__ __device__ constexpr int bwd_stream_nbuf(int KC, int XF) {
  return (160 * 1024 - bwd_stream_fixed(KC, XF)) / bwd_stream_buf(KC, XF) >= VCG_STREAM_NBUF ? VCG_STREAM_NBUF
         : (160 * 1024 - bwd_stream_fixed(KC, XF)) / bwd_stream_buf(KC, XF);
}

template <int KC, int XF>
__device__ __forceinline__ void bwd_stream_body(const GemmParams& p) {
  constexpr bool HASY = (XF & XF_HASY) != 0, Y2 = (XF & XF_Y2) != 0;
  constexpr bool HASB = HASY || (XF & XF_BITS) != 0;  // mask bits + sum g
  static_assert(!Y2 || HASY, "y2 comes with y");
  constexpr int TM = 64, TN = 64, NTH = 512, NW = 8;
  constexpr int PJ = bwd_stream_pj(XF);
  static_assert(PJ == 0 || ((XF & XF_BITS) && !HASY), "P = g^T a2 with the mask bits alone");
  constexpr bool BREG = bwd_stream_breg(KC, XF);  // weight fragments in registers
  constexpr int NA = bwd_stream_na(KC, XF);       // A tiles per slot
  constexpr int NBUF = bwd_stream_nbuf(KC, XF);
  static_assert(NBUF >= 2, "LDS ring");  // (WIDE: 3 without y2; the host keeps WIDE + y2 on the persistent engine)
  constexpr int AT = KC * TM * 64 * 2;  // one A tile ([64][64] swizzled sub-tiles, fast_frag layout); two per slot
  constexpr int OB = TM * TN * 2;       // one row-major [64][64] bf16 epilogue operand (res / y / y2)
  constexpr int OFF_R = NA * AT, OFF_Y = OFF_R + OB, OFF_BITS = OFF_Y + (HASY ? OB : 0);
  constexpr int OFF_Y2 = OFF_BITS + (HASB ? NW * 256 : 0);  // mask bytes [64][8]: 16 lanes x 4 B per wave (+ pad)
  constexpr int OFF_A2 = OFF_Y2 + (Y2 ? OB : 0);             // a2 rows [64][PJ], 16-B chunks swizzled (stem_bwd)
  constexpr int BUF = OFF_A2 + PJ * 128;
  static_assert(BUF == bwd_stream_buf(KC, XF), "slot layout");
  constexpr int BB = BREG ? 0 : KC * TN * 64 * 2;
  constexpr int SB = TM * TN * 2;
  constexpr int TOTAL = NBUF * BUF + BB + SB + 4 * TN * 4;
  static_assert(TOTAL <= 160 * 1024, "LDS budget");
  static_assert(NBUF * BUF >= 3 * NTH * 8 * 4, "bwd_finish scratch");
  // VMEM instructions per wave: one tile's DMA (A 1 per k tile and A tile, res 1, y 1 + bits 1, y2 1), one flush's
  // stores (1)
  constexpr int OPS1 = KC + 1 + (HASY ? 1 : 0) + (HASB ? 1 : 0) + (Y2 ? 1 : 0) + PJ / 64, OPS2 = OPS1 + KC;
  constexpr int VMW1 = (NBUF - 2) * OPS1 + (NBUF - 1), VMW2 = (NBUF - 2) * OPS2 + (NBUF - 1);
  static_assert(VMW2 < 64, "vmcnt field");
  __shared__ __attribute__((aligned(1024))) char smem[TOTAL];  // the ONLY LDS object (see FastLoader)
  char* ring = smem;
  bf16_t* Bs = reinterpret_cast<bf16_t*>(smem + NBUF * BUF);
  bf16_t* St = reinterpret_cast<bf16_t*>(smem + NBUF * BUF + BB);
  float* cpar = reinterpret_cast<float*>(smem + NBUF * BUF + BB + SB);  // mean | mean2 | invstd | invstd2 [TN]

  const BwdEpi& e = p.bwd;
  const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int nx = p.N / TN, gy = gridDim.x / nx;
  int bx, by;
  if ((gy & 7) == 0) {  // every column tile of an M-tile row on one XCD (the A rows come from HBM once)
    const int sidx = blockIdx.x >> 3;
    bx = sidx % nx;
    by = (sidx / nx) * 8 + (blockIdx.x & 7);
  } else {
    bx = blockIdx.x % nx;
    by = blockIdx.x / nx;
  }
  const int n0 = bx * TN;
  const int mtiles = (p.M + TM - 1) / TM;
  const int my_tiles = by < mtiles ? (mtiles - 1 - by) / gy + 1 : 0;
  if (my_tiles == 0) {  // no rows: an all-zero partial slot
    if (e.nred > 0 && tid < TN)
      for (int r = 0; r < e.nred; ++r) e.part[((long long)by * e.nred + r) * p.N + n0 + tid] = 0.f;
    if constexpr (PJ > 0)
      for (int i = tid; i < TN * PJ; i += NTH) e.ppart[((long long)by * p.N + n0) * PJ + i] = 0.f;
    return;
  }
  if (tid < TN) {
    const int n = n0 + tid;
    cpar[tid] = e.mean ? e.mean[n] : 0.f;
    cpar[TN + tid] = e.mean2 ? e.mean2[n] : 0.f;
    cpar[2 * TN + tid] = e.invstd ? e.invstd[n] : 0.f;
    cpar[3 * TN + tid] = e.invstd2 ? e.invstd2[n] : 0.f;
  }
  __syncthreads();  // (no LDS-DMA issued yet)
  const int cc = tid & 7;  // the flush's 16-B column chunk of this thread (fixed for the whole kernel)
  float mu[8], mu2[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    mu[i] = cpar[8 * cc + i];
    mu2[i] = cpar[TN + 8 * cc + i];
  }
  // TSM shifts of the workgroup's two 32-column halves; two A tiles when they differ (never for WIDE: host check)
  const int sh0 = bwd_tsm_shift(e, n0), sh1 = bwd_tsm_shift(e, n0 + 32);
  const bool two = NA == 2 && sh0 != sh1;

  // buffer descriptors of the epilogue operands (offset beyond num_records -> zeros)
  const long long ld = p.ldc;
  const uint32_t nb_full = (uint32_t)min((long long)p.M * ld * 2, (long long)0xFFFFFF00LL);
  const long long rrows = e.res_s > 1 ? (long long)(p.M / e.hw) * e.rH * e.rW : (long long)p.M;
  const uint32_t nb_res = (uint32_t)min(rrows * ld * 2, (long long)0xFFFFFF00LL);
  const __amdgpu_buffer_rsrc_t rs_res = __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(e.res), 0, nb_res, 0x00020000);
  __amdgpu_buffer_rsrc_t rs_y = rs_res, rs_y2 = rs_res, rs_bits = rs_res;
  uint32_t nb_bits = 0;
  if constexpr (HASY) rs_y = __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(e.y), 0, nb_full, 0x00020000);
  if constexpr (HASB) {
    nb_bits = (uint32_t)(((long long)p.M * ld) >> 3);
    rs_bits = __builtin_amdgcn_make_buffer_rsrc(const_cast<uint8_t*>(e.bits), 0, nb_bits, 0x00020000);
  }
  if constexpr (Y2) rs_y2 = __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(e.y2), 0, nb_full, 0x00020000);
  uint32_t nb_a2 = 0;
  __amdgpu_buffer_rsrc_t rs_a2 = rs_res;
  if constexpr (PJ > 0) {
    nb_a2 = (uint32_t)min((long long)p.M * PJ * 2, (long long)0xFFFFFF00LL);
    rs_a2 = __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(e.a2), 0, nb_a2, 0x00020000);
  }

  FastLoader<64, OP_DENSE_K, NW> la, lb;
  const int g = lane >> 4, ci = lane & 15;
  const int wr = wave & 3, wc = wave >> 2;  // MFMA block: rows 16 wr .. + 15, columns 32 wc .. + 31 of the tile
  // WIDE: this wave's weight fragments (columns 32 wc + 16 j + ci, k = 64 kc + 32 s + 8 g .. + 7: fast_frag's
  // lane map) straight into registers, retired before the ring's first DMA (so no wait inside the loop counts them)
  s16x8 bfr[BREG ? KC : 1][2][2];
  if constexpr (BREG) {
    const bf16_t* bp = reinterpret_cast<const bf16_t*>(p.b.ptr);
#pragma unroll
    for (int kc = 0; kc < KC; ++kc)
#pragma unroll
      for (int s = 0; s < 2; ++s)
#pragma unroll
        for (int j = 0; j < 2; ++j)
          bfr[kc][s][j] = *reinterpret_cast<const s16x8*>(bp + (long long)(n0 + 32 * wc + 16 * j + ci) * p.b.ld +
                                                          64 * kc + 32 * s + 8 * g);
#pragma unroll
    for (int kc = 0; kc < KC; ++kc)
#pragma unroll
      for (int s = 0; s < 2; ++s)
#pragma unroll
        for (int j = 0; j < 2; ++j) asm volatile("" ::"v"(bfr[kc][s][j]));
  } else {
    lb.init(p.b, 0, n0, wave, lane);
#pragma unroll
    for (int kc = 0; kc < KC; ++kc) lb.issue(p.b, kc * 64, p.K, Bs + kc * 4096, wave);
  }

  auto issue_tile = [&](int t) {
    const int d0 = (by + t * gy) * TM;
    char* buf = ring + (t % NBUF) * BUF;
    // A rows of the shift(s): destination row d reads GEMM row d - s hw, zero outside the clip
    la.init(p.a, 0, d0, wave, lane);
    const int d = d0 + wave * 8 + (lane >> 3);  // FastLoader<64, dense, 8 waves>: one row per lane
    int f = 0, tt = 0;
    if (e.tsm_T > 0 && (sh0 | sh1) != 0) {
      f = (int)fdiv((uint32_t)min(d, p.M - 1), e.fd_hw);
      tt = f - (int)fdiv((uint32_t)f, e.fd_T) * e.tsm_T;
    }
#pragma unroll
    for (int a = 0; a < 2; ++a) {
      if (a == 1 && !two) break;
      const int s = a == 0 ? sh0 : sh1;
      const bool ok = d < p.M && (unsigned)(tt - s) < (unsigned)max(e.tsm_T, 1);
      la.off[0] = ok ? (int)((long long)(d - s * e.hw) * p.a.ld) : -1;
#pragma unroll
      for (int kc = 0; kc < KC; ++kc)
        la.issue(p.a, kc * 64, p.K, reinterpret_cast<bf16_t*>(buf + a * AT) + kc * 4096, wave);
    }
    // residual / y / y2 rows: this wave's instruction covers tile rows 8 wave .. + 7, lane -> (row, chunk)
    {
      const int r = wave * 8 + (lane >> 3);
      const int dr = d0 + r, n = n0 + 8 * (lane & 7);
      const bool ok = dr < p.M;
      uint32_t roff = (uint32_t)((long long)dr * ld + n) * 2u;
      if (e.res_s > 1) {  // compact residual of a 1x1 / stride-2 conv: only even (h, w) rows carry one
        const uint32_t f2 = fdiv((uint32_t)dr, e.fd_hw), rr = (uint32_t)dr - f2 * (uint32_t)e.hw;
        const uint32_t h = fdiv(rr, e.fd_w), w = rr - h * e.fd_w.d;
        roff = ((h | w) & 1u) ? nb_res : (uint32_t)((((long long)(f2 * e.rH + (h >> 1)) * e.rW + (w >> 1)) * ld + n) * 2);
      }
      const uint32_t yoff = (uint32_t)((long long)dr * ld + n) * 2u;
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rs_res, (lds_void_t*)(buf + OFF_R + wave * 1024), 16, ok ? roff : nb_res,
                                               0, 0, 0);
      if constexpr (HASY)
        __builtin_amdgcn_raw_ptr_buffer_load_lds(rs_y, (lds_void_t*)(buf + OFF_Y + wave * 1024), 16, ok ? yoff : nb_full,
                                                 0, 0, 0);
      if constexpr (Y2)
        __builtin_amdgcn_raw_ptr_buffer_load_lds(rs_y2, (lds_void_t*)(buf + OFF_Y2 + wave * 1024), 16,
                                                 ok ? yoff : nb_full, 0, 0, 0);
    }
    if constexpr (HASB) {  // mask bytes: lane < 16 -> row 8 wave + lane / 2, 32 columns (dword lane & 1)
      const int dr = d0 + 8 * wave + ((lane & 15) >> 1), n = n0 + 32 * (lane & 1);
      const bool ok = lane < 16 && dr < p.M;
      const uint32_t boff = (uint32_t)(((long long)dr * ld + n) >> 3);
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rs_bits, (lds_void_t*)(buf + OFF_BITS + wave * 256), 4,
                                               ok ? boff : nb_bits, 0, 0, 0);
    }
    if constexpr (PJ > 0) {  // a2 rows [64][PJ]: 1 KB per instruction, the lane at slot q of row r loads chunk
#pragma unroll                // q ^ 2 ((r >> 1) & 3) (the transposed reads' swizzle, stem_bwd.hip sb_swz)
      for (int h = 0; h < PJ / 64; ++h) {
        constexpr int CPRA = PJ / 8;  // 16-B chunks per a2 row
        const int r = (8 * h + wave) * (1024 / (PJ * 2)) + lane / CPRA, q = lane % CPRA;
        const int dr = d0 + r, c = q ^ (2 * ((r >> 1) & 3));
        const uint32_t aoff = dr < p.M ? (uint32_t)(((long long)dr * PJ + 8 * c) * 2) : nb_a2;
        __builtin_amdgcn_raw_ptr_buffer_load_lds(rs_a2, (lds_void_t*)(buf + OFF_A2 + (8 * h + wave) * 1024), 16,
                                                 aoff, 0, 0, 0);
      }
    }
  };

#pragma unroll
  for (int i = 0; i < NBUF - 1; ++i)
    if (i < my_tiles) issue_tile(i);

  float s1[8], s2[8], s3[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) s1[i] = s2[i] = s3[i] = 0.f;
  f32x4 accp[PJ > 0 ? PJ / 32 : 1];
#pragma unroll
  for (int i = 0; i < (PJ > 0 ? PJ / 32 : 1); ++i) accp[i] = f32x4{0.f, 0.f, 0.f, 0.f};
  bf16_t* Cout = reinterpret_cast<bf16_t*>(p.C);

  for (int t = 0; t < my_tiles; ++t) {
    FAST_STAMP(t, 0);
    // tile t has landed once only the ring's later tiles (NBUF - 2) and the stores of the NBUF - 1 flushes since
    // its DMA are outstanding (steady state); the first / last tiles wait for everything
    if (t >= NBUF - 1 && t + NBUF - 2 < my_tiles) {
      if (two) __builtin_amdgcn_s_waitcnt(waitcnt_vm(VMW2));
      else __builtin_amdgcn_s_waitcnt(waitcnt_vm(VMW1));
    } else {
      __builtin_amdgcn_s_waitcnt(waitcnt_vm(0));
    }
    __builtin_amdgcn_s_barrier();  // tile t visible to every wave; every wave's reads of the ring slot below retired
    FAST_STAMP(t, 1);
    if (t + NBUF - 1 < my_tiles) issue_tile(t + NBUF - 1);
    const int d0 = (by + t * gy) * TM;
    const char* buf = ring + (t % NBUF) * BUF;
    const bf16_t* At = reinterpret_cast<const bf16_t*>(buf + ((two && wc == 1) ? AT : 0));
    f32x4 acc[2];
#pragma unroll
    for (int j = 0; j < 2; ++j) acc[j] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int kc = 0; kc < KC; ++kc)
#pragma unroll
      for (int s = 0; s < 2; ++s) {
        const s16x8 af = fast_frag(At + kc * 4096, 16 * wr, lane, s);
#pragma unroll
        for (int j = 0; j < 2; ++j) {
          s16x8 bf;
          if constexpr (BREG) bf = bfr[kc][s][j];
          else bf = fast_frag(Bs + kc * 4096, 32 * wc + 16 * j, lane, s);
          acc[j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bf, af, acc[j], 0, 0, 0);
        }
      }
    // stage the bf16 GEMM value: row 16 wr + ci, columns 32 wc + 16 j + 4 g .. + 3
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int row = 16 * wr + ci, col = 32 * wc + 16 * j + 4 * g;
      uint2 q2;
      q2.x = (uint32_t)f2bf(acc[j][0]) | ((uint32_t)f2bf(acc[j][1]) << 16);
      q2.y = (uint32_t)f2bf(acc[j][2]) | ((uint32_t)f2bf(acc[j][3]) << 16);
      // (inline asm: a plain LDS store makes hipcc wait vmcnt(0) for the ring's in-flight DMA first)
      asm volatile("ds_write_b64 %0, %1" ::"v"(lds_u32(St + row * 64 + 8 * st_slot<64>(row, col >> 3) + (col & 7))),
                   "v"(q2) : "memory");
    }
    __builtin_amdgcn_s_waitcnt(0xC07F);  // lgkmcnt(0)
    __builtin_amdgcn_s_barrier();
    FAST_STAMP(t, 2);
    const bf16_t* R = reinterpret_cast<const bf16_t*>(buf + OFF_R);
    const bf16_t* Y = reinterpret_cast<const bf16_t*>(buf + OFF_Y);
    const bf16_t* Y2p = reinterpret_cast<const bf16_t*>(buf + OFF_Y2);
    const uint8_t* Bt = reinterpret_cast<const uint8_t*>(buf + OFF_BITS);
    {
      const int r = tid >> 3;
      const int d = d0 + r, n = n0 + 8 * cc;
      // (LDS reads as inline asm: hipcc would wait vmcnt(0) for the ring's in-flight DMA before plain ones)
      uint4 sv, rv, yv = make_uint4(0u, 0u, 0u, 0u), y2v = yv;
      uint32_t bits = 0xFFu;
      asm volatile("ds_read_b128 %0, %1" : "=v"(sv) : "v"(lds_u32(St + r * 64 + 8 * st_slot<64>(r, cc))) : "memory");
      asm volatile("ds_read_b128 %0, %1" : "=v"(rv) : "v"(lds_u32(R + r * 64 + 8 * cc)) : "memory");
      if constexpr (HASY)
        asm volatile("ds_read_b128 %0, %1" : "=v"(yv) : "v"(lds_u32(Y + r * 64 + 8 * cc)) : "memory");
      if constexpr (HASB)
        asm volatile("ds_read_u8 %0, %1" : "=v"(bits) : "v"(lds_u32(Bt + (r >> 3) * 256 + (r & 7) * 8 + cc)) : "memory");
      if constexpr (Y2)
        asm volatile("ds_read_b128 %0, %1" : "=v"(y2v) : "v"(lds_u32(Y2p + r * 64 + 8 * cc)) : "memory");
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_sched_barrier(0);
      uint4 o = make_uint4(0u, 0u, 0u, 0u);  // (rows past M: zeros for the P product)
      if (d < p.M) {
        float v[8], rr[8];
        unpack8(sv, v);
        unpack8(rv, rr);
#pragma unroll
        for (int i = 0; i < 8; ++i) v[i] += rr[i];
        if constexpr (HASB) {
#pragma unroll
          for (int i = 0; i < 8; ++i) v[i] = ((bits >> i) & 1u) ? v[i] : 0.f;
        }
        o.x = (uint32_t)f2bf(v[0]) | ((uint32_t)f2bf(v[1]) << 16);
        o.y = (uint32_t)f2bf(v[2]) | ((uint32_t)f2bf(v[3]) << 16);
        o.z = (uint32_t)f2bf(v[4]) | ((uint32_t)f2bf(v[5]) << 16);
        o.w = (uint32_t)f2bf(v[6]) | ((uint32_t)f2bf(v[7]) << 16);
        *reinterpret_cast<uint4*>(Cout + (long long)d * ld + n) = o;
        if constexpr (HASB && !HASY) {
          unpack8(o, v);  // sum of the stored (rounded) gradient
#pragma unroll
          for (int i = 0; i < 8; ++i) s1[i] += v[i];
        }
        if constexpr (HASY) {
          float yy[8];
          unpack8(o, v);  // statistics of the stored (rounded) gradient
          unpack8(yv, yy);
#pragma unroll
          for (int i = 0; i < 8; ++i) {
            s1[i] += v[i];
            s2[i] = fmaf(v[i], yy[i] - mu[i], s2[i]);
          }
          if constexpr (Y2) {
            float y2[8];
            unpack8(y2v, y2);
#pragma unroll
            for (int i = 0; i < 8; ++i) s3[i] = fmaf(v[i], y2[i] - mu2[i], s3[i]);
          }
        }
      }
      if constexpr (PJ > 0) {  // the stored g over its own stage chunk, for the P product below
        const pk_u32x4 ov = {o.x, o.y, o.z, o.w};
        asm volatile("ds_write_b128 %0, %1" ::"v"(lds_u32(St + r * 64 + 8 * st_slot<64>(r, cc))), "v"(ov) : "memory");
      }
    }
    if constexpr (PJ > 0) {
      // P[n][j] += sum_r g[r][n] a2[r][j] over the tile's 64 rows: both operands by transposed LDS reads
      // (ds_read_b64_tr_b16, stem_bwd.hip's lane map: lanes 4q + pp of group g address row 4 g + q, columns 4 pp ..)
      __builtin_amdgcn_s_waitcnt(0xC07F);  // lgkmcnt(0): this wave's g chunks are in St
      __builtin_amdgcn_s_barrier();        // ... and every wave's
      const bf16_t* A2 = reinterpret_cast<const bf16_t*>(buf + OFF_A2);
      const int nb = wave & 3, q = ci >> 2, pp = ci & 3;
#pragma unroll
      for (int ks = 0; ks < 2; ++ks) {
        const int k0 = 32 * ks + 4 * g + q, k1 = k0 + 16;
        const int cl = 16 * nb + 4 * pp;
        s16x4 gl, gh, al[PJ / 32], ah[PJ / 32];
        lds_tr_b16(gl, St + k0 * 64 + 8 * st_slot<64>(k0, cl >> 3) + (cl & 7));
        lds_tr_b16(gh, St + k1 * 64 + 8 * st_slot<64>(k1, cl >> 3) + (cl & 7));
#pragma unroll
        for (int i = 0; i < PJ / 32; ++i) {
          const int cj = 16 * ((wave >> 2) + 2 * i) + 4 * pp;
          lds_tr_b16(al[i], A2 + k0 * PJ + 8 * ((cj >> 3) ^ (2 * ((k0 >> 1) & 3))) + (cj & 7));
          lds_tr_b16(ah[i], A2 + k1 * PJ + 8 * ((cj >> 3) ^ (2 * ((k1 >> 1) & 3))) + (cj & 7));
        }
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_sched_barrier(0);
        const s16x8 gf = s16x8{gl[0], gl[1], gl[2], gl[3], gh[0], gh[1], gh[2], gh[3]};
#pragma unroll
        for (int i = 0; i < PJ / 32; ++i)
          accp[i] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(
              s16x8{al[i][0], al[i][1], al[i][2], al[i][3], ah[i][0], ah[i][1], ah[i][2], ah[i][3]}, gf, accp[i], 0, 0,
              0);
        __builtin_amdgcn_sched_barrier(0);
      }
    }
    FAST_STAMP(t, 3);
  }
  __builtin_amdgcn_s_waitcnt(waitcnt_vm(0));
  if constexpr (PJ > 0) {  // accp[i][rr] = P[n0 + 16 nb + ci][16 ((wave >> 2) + 2 i) + 4 g + rr] -> slab `by`
    float* pp = e.ppart + ((long long)by * p.N + n0 + 16 * (wave & 3) + ci) * PJ;
#pragma unroll
    for (int i = 0; i < PJ / 32; ++i)
      *reinterpret_cast<f32x4*>(pp + 16 * ((wave >> 2) + 2 * i) + 4 * g) = accp[i];
  }
  if constexpr (HASB) {
    if (e.nred > 0) bwd_finish<256, 64>(p, reinterpret_cast<float*>(smem), cpar + 2 * TN, s1, s2, s3, n0, by);
  }
}

// K = 256 with 64 x 128 tiles (the layer-3 conv1 input gradients: every 128-column tile inside one TSM shift, fold
// % 128 == 0, and the mask bits without y -- the previous block's y3 is not stored). Per-tile stamps of the 64 x 64
// form (tools/bench_dgrad.py, -DVCG_FAST_STAMPS) put ~2/3 of a tile in the phase that issues the next tile's LDS-DMA
// (6 1-KB pieces per wave) next to the MFMAs; here one A tile (32 KB) serves 128 columns (LDS-DMA per output byte
// 50 / 16 instead of 40.5 / 8), the next tile's A pieces are issued between the k-steps' MFMAs, and the epilogue runs
// in the MFMA lanes on the residual rows in LDS: g = mask(bf16(acc) + res) is written back over the residual (same
// lane, same bytes: no barrier, no separate stage), and the flush threads only copy 16-B chunks out and sum them.
// The residual rows land pre-swizzled (16-B chunk c of row r at slot c ^ (r & 15)), so the MFMA lanes' 8-B accesses
// (16 rows, one column group) and the flush's 16-B row reads are both conflict-free. The weight fragments of a wave's
// 32 columns stay in registers; 3 slots of 50 KB.
template <int XF>
__device__ __forceinline__ void bwd_stream128_body(const GemmParams& p) {
  constexpr bool HASB = (XF & XF_BITS) != 0;
  static_assert((XF & (XF_HASY | XF_Y2)) == 0, "the mask bits without y only");
  constexpr int KC = 4, TM = 64, TN = 128, NTH = 512, NW = 8;
  constexpr int AT = KC * TM * 64 * 2;               // A tile [4][64][64] swizzled (fast_frag layout), 32 KB
  constexpr int OB = TM * TN * 2;                    // residual rows -> g, [64][128] bf16 swizzled, 16 KB
  constexpr int OFF_R = AT, OFF_BITS = OFF_R + OB;  // mask bytes [8 waves][256 B]: rows 8 w .. + 7 x 16 B (+ pad)
  constexpr int BUF = OFF_BITS + (HASB ? NW * 256 : 0);
  constexpr int CP = 4 * TN * 4;
  constexpr int NBUF = (160 * 1024 - CP) / BUF;
  static_assert(NBUF >= 3 && NBUF * BUF + CP <= 160 * 1024, "LDS ring");
  static_assert(NBUF * BUF >= 3 * NTH * 8 * 4, "bwd_finish scratch");
  // VMEM instructions per wave: one tile's DMA (A 4, residual 2, bits 1), one flush's stores (2)
  constexpr int OPS = KC + 2 + (HASB ? 1 : 0), STO = 2;
  constexpr int VMW = (NBUF - 2) * OPS + (NBUF - 1) * STO;
  static_assert(VMW < 64, "vmcnt field");
  __shared__ __attribute__((aligned(1024))) char smem[NBUF * BUF + CP];  // the ONLY LDS object
  char* ring = smem;
  float* cpar = reinterpret_cast<float*>(smem + NBUF * BUF);  // mean | mean2 | invstd | invstd2 [TN]

  const BwdEpi& e = p.bwd;
  const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int nx = p.N / TN, gy = gridDim.x / nx;
  int bx, by;
  if ((gy & 7) == 0) {  // every column tile of an M-tile row on one XCD (the A rows come from HBM once)
    const int sidx = blockIdx.x >> 3;
    bx = sidx % nx;
    by = (sidx / nx) * 8 + (blockIdx.x & 7);
  } else {
    bx = blockIdx.x % nx;
    by = blockIdx.x / nx;
  }
  const int n0 = bx * TN;
  const int mtiles = (p.M + TM - 1) / TM;
  const int my_tiles = by < mtiles ? (mtiles - 1 - by) / gy + 1 : 0;
  if (my_tiles == 0) {  // no rows: an all-zero partial slot
    if (e.nred > 0 && tid < TN)
      for (int r = 0; r < e.nred; ++r) e.part[((long long)by * e.nred + r) * p.N + n0 + tid] = 0.f;
    return;
  }
  if (tid < TN) {
    const int n = n0 + tid;
    cpar[tid] = e.mean ? e.mean[n] : 0.f;
    cpar[TN + tid] = e.mean2 ? e.mean2[n] : 0.f;
    cpar[2 * TN + tid] = e.invstd ? e.invstd[n] : 0.f;
    cpar[3 * TN + tid] = e.invstd2 ? e.invstd2[n] : 0.f;
  }
  __syncthreads();  // (no LDS-DMA issued yet)
  const int cc = tid & 15;  // the flush's 16-B column chunk of this thread (fixed for the whole kernel)
  const int sh = bwd_tsm_shift(e, n0);  // one shift for the tile's 128 columns (host check)

  const long long ld = p.ldc;
  const long long rrows = e.res_s > 1 ? (long long)(p.M / e.hw) * e.rH * e.rW : (long long)p.M;
  const uint32_t nb_res = (uint32_t)min(rrows * ld * 2, (long long)0xFFFFFF00LL);
  const __amdgpu_buffer_rsrc_t rs_res = __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(e.res), 0, nb_res, 0x00020000);
  __amdgpu_buffer_rsrc_t rs_bits = rs_res;
  uint32_t nb_bits = 0;
  if constexpr (HASB) {
    nb_bits = (uint32_t)(((long long)p.M * ld) >> 3);
    rs_bits = __builtin_amdgcn_make_buffer_rsrc(const_cast<uint8_t*>(e.bits), 0, nb_bits, 0x00020000);
  }

  FastLoader<64, OP_DENSE_K, NW> la;
  const int g = lane >> 4, ci = lane & 15;
  const int wr = wave & 1, wc = wave >> 1;  // MFMA block: rows 32 wr .. + 31, columns 32 wc .. + 31 of the tile
  // this wave's weight fragments (columns 32 wc + 16 j + ci, k = 64 kc + 32 s + 8 g .. + 7: fast_frag's lane map),
  // retired before the ring's first DMA (no wait inside the loop counts them)
  s16x8 bfr[KC][2][2];
  {
    const bf16_t* bp = reinterpret_cast<const bf16_t*>(p.b.ptr);
#pragma unroll
    for (int kc = 0; kc < KC; ++kc)
#pragma unroll
      for (int s = 0; s < 2; ++s)
#pragma unroll
        for (int j = 0; j < 2; ++j)
          bfr[kc][s][j] = *reinterpret_cast<const s16x8*>(bp + (long long)(n0 + 32 * wc + 16 * j + ci) * p.b.ld +
                                                          64 * kc + 32 * s + 8 * g);
#pragma unroll
    for (int kc = 0; kc < KC; ++kc)
#pragma unroll
      for (int s = 0; s < 2; ++s)
#pragma unroll
        for (int j = 0; j < 2; ++j) asm volatile("" ::"v"(bfr[kc][s][j]));
  }

  // tile t's A rows (piece kc) / residual rows + mask bytes into its ring slot
  auto a_init = [&](int t) {
    const int d0 = (by + t * gy) * TM;
    la.init(p.a, 0, d0, wave, lane);
    const int d = d0 + wave * 8 + (lane >> 3);  // FastLoader<64, dense, 8 waves>: one row per lane
    int tt = 0;
    if (e.tsm_T > 0 && sh != 0) {  // destination row d reads GEMM row d - s hw, zero outside the clip
      const int f = (int)fdiv((uint32_t)min(d, p.M - 1), e.fd_hw);
      tt = f - (int)fdiv((uint32_t)f, e.fd_T) * e.tsm_T;
    }
    const bool ok = d < p.M && (unsigned)(tt - sh) < (unsigned)max(e.tsm_T, 1);
    la.off[0] = ok ? (int)((long long)(d - sh * e.hw) * p.a.ld) : -1;
  };
  auto a_piece = [&](int t, int kc) {
    la.issue(p.a, kc * 64, p.K, reinterpret_cast<bf16_t*>(ring + (t % NBUF) * BUF) + kc * 4096, wave);
  };
  // residual rows: instruction h of this wave covers tile rows 32 h + 4 wave .. + 3; the lane at LDS slot q of row
  // r loads chunk q ^ (r & 15)
  auto res_piece = [&](int t, int h) {
    const int d0 = (by + t * gy) * TM;
    char* buf = ring + (t % NBUF) * BUF;
    {
      const int r = 32 * h + 4 * wave + (lane >> 4);
      const int dr = d0 + r, n = n0 + 8 * ((lane & 15) ^ (r & 15));
      uint32_t roff = (uint32_t)((long long)dr * ld + n) * 2u;
      if (e.res_s > 1) {  // compact residual of a 1x1 / stride-2 conv: only even (h, w) rows carry one
        const uint32_t f2 = fdiv((uint32_t)dr, e.fd_hw), rr = (uint32_t)dr - f2 * (uint32_t)e.hw;
        const uint32_t hh = fdiv(rr, e.fd_w), w = rr - hh * e.fd_w.d;
        roff = ((hh | w) & 1u) ? nb_res : (uint32_t)((((long long)(f2 * e.rH + (hh >> 1)) * e.rW + (w >> 1)) * ld + n) * 2);
      }
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rs_res, (lds_void_t*)(buf + OFF_R + (8 * h + wave) * 1024), 16,
                                               dr < p.M ? roff : nb_res, 0, 0, 0);
    }
  };
  auto bits_piece = [&](int t) {
    const int d0 = (by + t * gy) * TM;
    char* buf = ring + (t % NBUF) * BUF;
    if constexpr (HASB) {  // mask bytes: lane < 32 -> row 8 wave + lane / 4, 32 columns (dword lane & 3)
      const int dr = d0 + 8 * wave + ((lane & 31) >> 2), n = n0 + 32 * (lane & 3);
      const bool okb = lane < 32 && dr < p.M;
      const uint32_t boff = (uint32_t)(((long long)dr * ld + n) >> 3);
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rs_bits, (lds_void_t*)(buf + OFF_BITS + wave * 256), 4,
                                               okb ? boff : nb_bits, 0, 0, 0);
    }
  };

#pragma unroll
  for (int i = 0; i < NBUF - 1; ++i)
    if (i < my_tiles) {
      a_init(i);
#pragma unroll
      for (int kc = 0; kc < KC; ++kc) a_piece(i, kc);
      res_piece(i, 0);
      res_piece(i, 1);
      bits_piece(i);
    }

  float s1[8], s0[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) s1[i] = s0[i] = 0.f;
  bf16_t* Cout = reinterpret_cast<bf16_t*>(p.C);

  for (int t = 0; t < my_tiles; ++t) {
    FAST_STAMP(t, 0);
    if (t >= NBUF - 1 && t + NBUF - 2 < my_tiles) __builtin_amdgcn_s_waitcnt(waitcnt_vm(VMW));
    else __builtin_amdgcn_s_waitcnt(waitcnt_vm(0));
    // tile t visible to every wave; every wave's reads of the slot refilled below (tile t - 1's) retired
    __builtin_amdgcn_s_barrier();
    FAST_STAMP(t, 1);
    const bool nxt = t + NBUF - 1 < my_tiles;
    if (nxt) a_init(t + NBUF - 1);
    const int d0 = (by + t * gy) * TM;
    char* buf = ring + (t % NBUF) * BUF;
    const bf16_t* At = reinterpret_cast<const bf16_t*>(buf);
    f32x4 acc[2][2];
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int j = 0; j < 2; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int kc = 0; kc < KC; ++kc) {
      if (nxt) {  // the next tile's DMA pieces spread over the k-steps' MFMAs (7 per wave, as the prologue's)
        a_piece(t + NBUF - 1, kc);
        if (kc < 2) res_piece(t + NBUF - 1, kc);
        if (kc == 2) bits_piece(t + NBUF - 1);
      }
#pragma unroll
      for (int s = 0; s < 2; ++s) {
        const s16x8 a0 = fast_frag(At + kc * 4096, 32 * wr, lane, s);
        const s16x8 a1 = fast_frag(At + kc * 4096, 32 * wr + 16, lane, s);
#pragma unroll
        for (int j = 0; j < 2; ++j) {
          acc[0][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bfr[kc][s][j], a0, acc[0][j], 0, 0, 0);
          acc[1][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bfr[kc][s][j], a1, acc[1][j], 0, 0, 0);
        }
      }
    }
    FAST_STAMP(t, 2);
    // epilogue in the MFMA lanes: row 32 wr + 16 i + ci, columns 32 wc + 16 j + 4 g .. + 3 of the residual / g rows
    bf16_t* Rg = reinterpret_cast<bf16_t*>(buf + OFF_R);
    const uint8_t* Bt = reinterpret_cast<const uint8_t*>(buf + OFF_BITS);
    uint2 rv[2][2];
    uint32_t bw[2][2];
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        const int row = 32 * wr + 16 * i + ci, col = 32 * wc + 16 * j + 4 * g;
        // (LDS reads / writes as inline asm: hipcc would wait vmcnt(0) for the ring's in-flight DMA first)
        asm volatile("ds_read_b64 %0, %1"
                     : "=v"(rv[i][j])
                     : "v"(lds_u32(Rg + row * TN + 8 * st_slot<TN>(row, col >> 3) + (col & 7)))
                     : "memory");
        bw[i][j] = 0xFFu;
        if constexpr (HASB)
          asm volatile("ds_read_u8 %0, %1" : "=v"(bw[i][j]) : "v"(lds_u32(Bt + (row >> 3) * 256 + (row & 7) * 16 + (col >> 3)))
                       : "memory");
      }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        const int row = 32 * wr + 16 * i + ci, col = 32 * wc + 16 * j + 4 * g;
        const uint32_t rw[2] = {rv[i][j].x, rv[i][j].y};
        float v[4];
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const float r = __uint_as_float((q & 1) ? (rw[q >> 1] & 0xffff0000u) : (rw[q >> 1] << 16));
          v[q] = bf2f(f2bf(acc[i][j][q])) + r;  // the staged bf16 GEMM value + residual (stage_flush_bwd order)
          if constexpr (HASB) v[q] = ((bw[i][j] >> ((col & 7) + q)) & 1u) ? v[q] : 0.f;
        }
        uint2 o;
        o.x = (uint32_t)f2bf(v[0]) | ((uint32_t)f2bf(v[1]) << 16);
        o.y = (uint32_t)f2bf(v[2]) | ((uint32_t)f2bf(v[3]) << 16);
        asm volatile("ds_write_b64 %0, %1" ::"v"(lds_u32(Rg + row * TN + 8 * st_slot<TN>(row, col >> 3) + (col & 7))),
                     "v"(o) : "memory");
      }
    __builtin_amdgcn_s_waitcnt(0xC07F);  // lgkmcnt(0)
    __builtin_amdgcn_s_barrier();
    FAST_STAMP(t, 3);
    // flush: each thread copies row chunks (r, cc) of g out and sums them
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int r = (tid >> 4) + 32 * h;
      const int d = d0 + r, n = n0 + 8 * cc;
      uint4 o;
      asm volatile("ds_read_b128 %0, %1" : "=v"(o) : "v"(lds_u32(Rg + r * TN + 8 * st_slot<TN>(r, cc))) : "memory");
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_sched_barrier(0);
      if (d < p.M) {
        *reinterpret_cast<uint4*>(Cout + (long long)d * ld + n) = o;
        if constexpr (HASB) {
          float v[8];
          unpack8(o, v);  // sum of the stored (rounded) gradient
#pragma unroll
          for (int i = 0; i < 8; ++i) s1[i] += v[i];
        }
      }
    }
  }
  __builtin_amdgcn_s_waitcnt(waitcnt_vm(0));
  if constexpr (HASB) {
    if (e.nred > 0) bwd_finish<256, 128>(p, reinterpret_cast<float*>(smem), cpar + 2 * TN, s1, s0, s0, n0, by);
  }
}

template <int BM, int BN, int AM, int EPI, int RES>
__device__ __forceinline__ void igemm_fast_body(const GemmParams& p) {
  // Persistent-style grid: workgroup (bx, by) owns N-tile bx and M-tiles by, by + gy, by + 2gy, ...;
  // the (m-tile, k-tile) steps form one software pipeline, so the next tiles' loads are in flight while
  // a tile finishes its MFMAs and its epilogue. Workgroups are dealt round-robin to the 8 XCDs by
  // linear id, so when gy % 8 == 0 the linear id is decoded such that all N-tiles of an M-tile
  // row run on the same XCD at the same time and the A rows are fetched from HBM once (L2 hits).
  // The bias lives in registers for the whole kernel (loaded before the pipeline starts) and the
  // epilogue (RES = false) loads nothing: a VGPR-destination global load inside the loop, or an LDS
  // object the compiler cannot tell apart from the DMA target, makes hipcc drain the in-flight
  // LDS-DMA prefetch with vmcnt(0) at every tile boundary. Conv (EPI_STATS) GEMMs carry no bias.
  //
  // Shapes: every wave owns a 64 x BN/2 sub-tile (4 x BN/32 fragments of 16x16); WM = BM / 64 waves
  // along M, 2 along N. BM = 128: 4 waves, 2 LDS stages (1 step in flight), 2 workgroups per CU.
  // BM = 256: 8 waves, 3 LDS stages (2 steps in flight across each barrier, counted vmcnt), 1 workgroup
  // per CU (the big conv GEMMs).
  constexpr int WM = BM / 64, NW = 2 * WM;
  constexpr int MT = 4, NT = BN / 32;
  constexpr int STAGES = BM == 256 ? 3 : 2;
  constexpr int AE = BM * FBK, BE = BN * FBK;  // elements per stage
  constexpr int NLD = BM / (8 * NW) + BN / (8 * NW);  // LDS-DMA instructions per thread per step
  constexpr bool BWD = EPI == EPI_BWD || EPI == EPI_BWD_AFF;
  constexpr int CPAR = BWD ? 6 * BN : 0;  // EPI_BWD per-column parameters
  constexpr int RED = 2 * WM * BN + WM + 4;
  __shared__ __attribute__((aligned(1024))) char smem[STAGES * (AE + BE) * 2 + (RED + CPAR) * 4];
  bf16_t* As = reinterpret_cast<bf16_t*>(smem);
  bf16_t* Bs = As + STAGES * AE;
  float* red = reinterpret_cast<float*>(smem + STAGES * (AE + BE) * 2);
  float* cpar = red + RED;  // [mean, msc, msh, mean2, invstd, invstd2][BN]

  const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave >> 1, wn = wave & 1;
  const int nx = (p.N + BN - 1) / BN, gy = gridDim.x / nx;
  int bx, by;
  if ((gy & 7) == 0) {
    const int sidx = blockIdx.x >> 3;
    bx = sidx % nx;
    by = (sidx / nx) * 8 + (blockIdx.x & 7);
  } else {
    bx = blockIdx.x % nx;
    by = blockIdx.x / nx;
  }
  const int n0 = bx * BN;
  long long aoff = 0, boff = 0;
  bf16_t* Cout = reinterpret_cast<bf16_t*>(p.C);
  const bf16_t* Res = RES ? reinterpret_cast<const bf16_t*>(p.residual) : nullptr;
  if (p.batch_inner > 0) {
    const int zo = blockIdx.z / p.batch_inner, zi = blockIdx.z - zo * p.batch_inner;
    aoff = zo * p.a_so + zi * p.a_si;
    boff = zo * p.b_so + zi * p.b_si;
    Cout += zo * p.c_so + zi * p.c_si;
    if (Res) Res += zo * p.c_so + zi * p.c_si;
  }
  const int mtiles = (p.M + BM - 1) / BM;
  const int my_tiles = by < mtiles ? (mtiles - 1 - by) / gy + 1 : 0;
  const int ntiles = (p.K + FBK - 1) / FBK;
  const int steps = my_tiles * ntiles;
  if constexpr (BWD) {
    if (steps == 0) {  // no rows: an all-zero partial slot
      if (p.bwd.nred > 0 && tid < BN && n0 + tid < p.N)
        for (int r = 0; r < p.bwd.nred; ++r) p.bwd.part[((long long)by * p.bwd.nred + r) * p.N + n0 + tid] = 0.f;
      return;
    }
    if (tid < BN) {
      const int n = min(n0 + tid, p.N - 1);
      const BwdEpi& e = p.bwd;
      cpar[tid] = e.mean ? e.mean[n] : 0.f;
      cpar[BN + tid] = e.msc ? e.msc[n] : 0.f;
      cpar[2 * BN + tid] = e.msh ? e.msh[n] : 0.f;
      cpar[3 * BN + tid] = e.mean2 ? e.mean2[n] : 0.f;
      cpar[4 * BN + tid] = e.invstd ? e.invstd[n] : 0.f;
      cpar[5 * BN + tid] = e.invstd2 ? e.invstd2[n] : 0.f;
    }
  }
  if (steps == 0) return;

  float bv[NT][4];
  if constexpr (EPI == EPI_STATS) {
#pragma unroll
    for (int j = 0; j < NT; ++j) bv[j][0] = bv[j][1] = bv[j][2] = bv[j][3] = 0.f;
  } else {
    load_bias<BN>(bv, p.bias, n0, wn, lane, p.N);
#pragma unroll
    for (int j = 0; j < NT; ++j) asm volatile("" ::"v"(bv[j][0]), "v"(bv[j][1]), "v"(bv[j][2]), "v"(bv[j][3]));
  }

  FastLoader<BM, AM, NW> la;
  FastLoader<BN, OP_DENSE_K, NW> lb;
  la.init(p.a, aoff, by * BM, wave, lane);
  lb.init(p.b, boff, n0, wave, lane);

  f32x4 acc[MT][NT];
#pragma unroll
  for (int i = 0; i < MT; ++i)
#pragma unroll
    for (int j = 0; j < NT; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  // EPI_STATS: shifted per-column sums over every row this workgroup stores, across all of its M-tiles,
  // merged once at the end -> one (mean, M2) slot per workgroup row `by` (stage_flush_stats, stats_finish).
  float b1[8], b2[8], b3[8];  // EPI_BWD column sums / EPI_STATS shift, s1, s2 of this thread's chunk
  int scnt = 0;               // EPI_STATS rows seen by this thread
#pragma unroll
  for (int i = 0; i < 8; ++i) b1[i] = b2[i] = b3[i] = 0.f;

  // issue side of the pipeline: the next step to load is k-tile ikt of the workgroup's local tile itile
  int ikt = 0, itile = 0;
  auto issue_next = [&](int stage) {
    if (ikt == 0 && itile > 0) la.init(p.a, aoff, (by + itile * gy) * BM, wave, lane);
    la.issue(p.a, ikt * FBK, p.K, As + stage * AE, wave);
    lb.issue(p.b, ikt * FBK, p.K, Bs + stage * BE, wave);
    if (++ikt == ntiles) {
      ikt = 0;
      ++itile;
    }
  };
#pragma unroll
  for (int i = 0; i < STAGES - 1; ++i)
    if (i < steps) issue_next(i);
  int kt = 0, tile = 0, cur = 0;
  for (int s = 0; s < steps; ++s) {
    // steps issued beyond s once this step's prefetch is out; step s has landed when at most that many
    // steps' loads are still outstanding
    const int ahead = min(STAGES - 1, steps - 1 - s);
    if (s + STAGES - 1 < steps) issue_next(cur == 0 ? STAGES - 1 : cur - 1);  // stage (s + STAGES - 1) % STAGES
    if (STAGES == 3 && ahead >= 2) __builtin_amdgcn_s_waitcnt(waitcnt_vm(2 * NLD));
    else if (ahead >= 1) __builtin_amdgcn_s_waitcnt(waitcnt_vm(NLD));
    else __builtin_amdgcn_s_waitcnt(waitcnt_vm(0));
    __builtin_amdgcn_s_barrier();
    if (kt == 0) FAST_STAMP(tile, 0);
    const bf16_t* Ac = As + cur * AE;
    const bf16_t* Bc = Bs + cur * BE;
#pragma unroll
    for (int s2 = 0; s2 < 2; ++s2) {
      s16x8 af[MT], bfr[NT];
#pragma unroll
      for (int i = 0; i < MT; ++i) af[i] = fast_frag(Ac, wm * 64 + i * 16, lane, s2);
#pragma unroll
      for (int j = 0; j < NT; ++j) bfr[j] = fast_frag(Bc, wn * (BN / 2) + j * 16, lane, s2);
#pragma unroll
      for (int i = 0; i < MT; ++i)
#pragma unroll
        for (int j = 0; j < NT; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bfr[j], af[i], acc[i][j], 0, 0, 0);
    }
    // every wave's ds_reads of this stage have returned before any wave refills it (WAR)
    __builtin_amdgcn_s_waitcnt(0xC07F);  // lgkmcnt(0) only
    __builtin_amdgcn_s_barrier();
    if (++kt == ntiles) {
      FAST_STAMP(tile, 1);
      const int mt = by + tile * gy;
      bf16_t* stA = As + cur * AE;  // the finished stage holds the output rounds (see stage_put)
      bf16_t* stB = BM == 256 ? stA + 64 * BN : Bs + cur * BE;
      // output tiles go through the LDS stage for full-row 16-B stores
      const bool staged = true;
      if constexpr (BWD) {
#pragma unroll
        for (int h = 0; h < BM / 128; ++h) {
          if ((wm >> 1) == h) {
#pragma unroll
            for (int j = 0; j < NT; ++j)
#pragma unroll
              for (int i = 0; i < MT; ++i) {
                float v[4] = {acc[i][j][0], acc[i][j][1], acc[i][j][2], acc[i][j][3]};
                if constexpr (AM == OP_DENSE_K2) {  // the folded BN's constant term, before the bf16 rounding
#pragma unroll
                  for (int r = 0; r < 4; ++r) v[r] += bv[j][r];
                }
                stage_put<BM, BN>(stA, stB, wm, wn, lane, i, j, v);
              }
          }
          FAST_STAMP(tile, 2);
          stage_flush_bwd<BM, BN, EPI == EPI_BWD_AFF>(stA, stB, p, Cout, mt * BM + 128 * h, n0, cpar, b1, b2, b3, p.M);
        }
      } else if constexpr (EPI == EPI_STATS) {  // conv outputs: no bias / activation, alpha = 1
#pragma unroll
        for (int h = 0; h < BM / 128; ++h) {
          if ((wm >> 1) == h) {
#pragma unroll
            for (int j = 0; j < NT; ++j)
#pragma unroll
              for (int i = 0; i < MT; ++i) {
                float v[4] = {acc[i][j][0], acc[i][j][1], acc[i][j][2], acc[i][j][3]};
                stage_put<BM, BN>(stA, stB, wm, wn, lane, i, j, v);
              }
          }
          stage_flush_stats<BM, BN>(stA, stB, p, Cout, mt * BM + 128 * h, n0, scnt, b1, b2, b3, p.M);
        }
      } else if constexpr (EPI == EPI_STORE_AUX) {
        if constexpr (BM == 128) epilogue_staged_aux<BM, BN>(acc, p, bv, Cout, stA, stB, mt * BM, n0, wm, wn, lane);
      } else if (BM == 256 || (staged && !RES && p.aux == nullptr && (p.ldc & 7) == 0 &&
                               ((uintptr_t)p.C & 15) == 0)) {
        epilogue_staged<BM, BN>(acc, p, bv, Cout, stA, stB, mt * BM, n0, wm, wn, lane, p.M);
      } else if (RES && (staged || p.obits) && p.aux == nullptr &&
                 (RES == 2 ? (staged && !p.res_sc) : (p.res_round && p.act == ACT_RELU)) &&
                 ((p.ldc | p.ldr | p.N) & 7) == 0 && (((uintptr_t)p.residual | (uintptr_t)p.C) & 15) == 0) {
        if constexpr (BM == 128 && RES)
          epilogue_staged_res<BM, BN, RES == 2>(acc, p, bv, Cout, Res, stA, stB, mt * BM, n0, wm, wn, lane, p.M);
      } else {
        if constexpr (BM == 128)
          gemm_epilogue<bf16_t, BM, BN, EPI>(acc, p, red, bv, Cout, Res, mt * BM, n0, wm, wn, lane, mt, mtiles);
      }
      FAST_STAMP(tile, 3);
#pragma unroll
      for (int i = 0; i < MT; ++i)
#pragma unroll
        for (int j = 0; j < NT; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
      kt = 0;
      ++tile;
    }
    cur = cur == STAGES - 1 ? 0 : cur + 1;
  }
  if constexpr (EPI == EPI_STATS)  // the stats buffer is laid out for 128-row tiles (vcg_conv_stats_tiles)
    stats_finish<BM, BN>(p, reinterpret_cast<float*>(smem), scnt, b1, b2, b3, n0, by, bx, gy, (p.M + 127) / 128);
  if constexpr (BWD) {
    if (p.bwd.nred > 0) bwd_finish<BM, BN>(p, reinterpret_cast<float*>(smem), cpar + 4 * BN, b1, b2, b3, n0, by);
  }
}

// The kernel: EPI_BWD_STREAM has its own tile schedule (bwd_stream_body; AM = K / 64, XF = its operand flags),
// every other epilogue runs the persistent 2-stage pipeline above.
template <int BM, int BN, int AM, int EPI, int RES, int XF = 0>
__global__ __launch_bounds__(BM * 2) __attribute__((amdgpu_waves_per_eu(EPI == EPI_BWD_AFF && BN == 64 ? 3 : 2)))
void igemm_fast_kernel(GemmParams p) {
  if constexpr (EPI == EPI_BWD_STREAM && BN == 128)
    bwd_stream128_body<XF>(p);
  else if constexpr (EPI == EPI_BWD_STREAM)
    bwd_stream_body<AM, XF>(p);
  else
    igemm_fast_body<BM, BN, AM, EPI, RES>(p);
}

// One resident round of workgroups (LDS allows 2 per CU at BM = 128 / BN = 128, 3 at BN = 64, 1 at BM = 256);
// each walks ceil(mtiles / gy) M-tiles. gy is a multiple of 8 whenever possible (XCD-aware decode).
// (EPI_BWD's BN = 64 kernel needs > 170 VGPRs: 2 workgroups per CU there too; EPI_BWD_AFF's fits 3)
static int grid_rows(int M, int N, int z, int BM, int BN, int epi) {
  const int nx = (N + BN - 1) / BN, mtiles = (M + BM - 1) / BM;
  const int resident = (BM == 256 ? 1 : (BN == 128 || epi == EPI_BWD ? 2 : 3)) * 256;
  int gy = resident / (nx * z);
  if (gy >= 8) gy &= ~7;
  if (gy > mtiles) gy = mtiles >= 8 ? (mtiles & ~7) : mtiles;
  if (gy < 1) gy = 1;
  return gy;
}

static int fast_bn_cols(int N) { return (N % 128 == 0 || N > 64 * 3) ? 128 : 64; }

// (The 256-row 3-stage variant of this engine, opt-in VCG_BIG_TILE in rounds 2-4, measured slower than two 4-wave
// 128-row workgroups per CU on every conv shape and was removed; the 256 x 256 8-wave engine is igemm256.hip.)
static int fast_bm(int, int, int, bool) { return 128; }

int fast_grid_rows(int M, int N, int z, int epi) {
  return grid_rows(M, N, z, fast_bm(M, N, z, false), fast_bn_cols(N), epi);
}

static bool bwd_light(const GemmParams& p) {
  const BwdEpi& e = p.bwd;
  return !e.res && !e.bits && !e.y2 && e.tsm_T == 0;
}


// ---- 3x3 / stride 1 / pad 1 convolutions over C = 64 channels (layer 1): LDS-resident input patch -------------
// An M-tile is R whole output rows of one image (TM = R * W <= 128 GEMM rows; rows TM..127 of the 128-row MFMA
// tile read clamped addresses and are never stored). The (R + 2) x (W + 2) input pixels that the tile's 9 taps
// read (zero border included) go to LDS ONCE by LDS-DMA -- 64 channels = one 128-B pixel row, swizzled like a
// [rows][64] tile with the pixel index as the row -- and the 9 taps read shifted fragments from it. The im2col
// gather fetches every input pixel 9 times through L2, the patch (R + 2)(W + 2) / (R W) times (1.04x at W = 56,
// R = 2). The filter (64 output columns x 576 = 72 KiB per workgroup) stays in registers: every wave keeps the
// B fragments of its 32 columns for all 9 taps (36 x 16 B per lane), so a tile is one barrier-free run of 144
// MFMAs per wave. That needs > 256 registers per lane: ONE 4-wave workgroup per CU (the 512-entry register file
// of a SIMD for one wave, 160 KiB of LDS for one workgroup), so latency is hidden by depth instead of by other
// waves: patches are issued two tiles ahead into a 3-buffer ring (the dgrad epilogue's y tile rides along), and
// the output goes out through the finished tile's patch buffer. Epilogues: EPI_STORE / EPI_STATS (shared staged
// flushes) and EPI_BWD_AFF with y read from LDS (the fused dgrad of the trunk: BN1 ReLU mask + BN1 sums).
// DG (dgrad): dx pixel (y, x) reads dy (y + 1 - kh, x + 1 - kw), the flipped tap map over the same patch.
// Measured history (trunk shape M = 1024 x 56 x 56): B through a 2-stage LDS ring with a barrier per tap 586 us
// fwd (im2col: 451-495); register B at 2 workgroups per CU spills (256 VGPRs) and lost to im2col.
constexpr int PATCH_MAXPIX = 256;               // (R + 2) PW <= 256 pixels: 32 KiB per patch buffer
constexpr int PATCH_SLICES = PATCH_MAXPIX / 8;  // 1-KiB (8-pixel) LDS-DMA slices per patch
// Patch rows have a fixed pitch PW (32 or 64 pixels >= W + 2; the kernel's template parameter): the chunk swizzle
// depends on the pixel index mod 8 only, so a tap's row offset kh * PW moves a fragment address by a compile-time
// constant (the ds_read offset field) and a lane's 12 fragment addresses per tile (4 row blocks x 3 column taps) are
// computed once per tile. (With PW = W + 2 every fragment read of the 144-MFMA tile loop recomputed its swizzled
// address -- ~5 VALU per read, more vector issue than the MFMAs leave: the MFMA phase ran at 2.45x its issue time.)
constexpr int PATCH_RING = 3;

struct PatchGeom {
  int R, TM, TPI, PW, NP, NS;  // rows per tile, GEMM rows per tile, tiles per image, patch width, pixels, slices
  unsigned long long* stamps;  // profiling (VCG_PATCH_STAMPS=1): s_memtime per phase of workgroup 0, wave 0
};
#define PATCH_STAMP(k)                                                                        \
  do {                                                                                        \
    if (g.stamps && blockIdx.x == 0 && threadIdx.x == 0 && lt < 64) g.stamps[lt * 6 + (k)] = __builtin_amdgcn_s_memtime(); \
  } while (0)

// Patch swizzle: 16-B chunk c of pixel pix sits at slot (c + 2 * (pix / 2)) % 8. A fragment read's 16 lanes of
// one ds_read_b128 bank group take pixels p0..p0+3, p0+12..p0+15 at chunk c and p0+4..p0+11 at chunk c + 1
// (MI355X_MICROARCH: the b128 lane groups); per pixel parity that is 8 consecutive pixels of one parity, offsets
// {0, 2, 5, 7, 9, 11, 12, 14} mod 8 = all 8 slots for any p0, where the XOR swizzle of the [rows][64] tiles
// collides for odd p0 (modelled: 4.5 vs 6.5 LDS cycles per read at W = 56; 4 = conflict-free).
__device__ __forceinline__ int pswz(int pix, int c) { return (c + (pix & ~1)) & 7; }

__device__ __forceinline__ s16x8 patch_frag(const bf16_t* P, int pix, int lane, int s2) {
  return *reinterpret_cast<const s16x8*>(P + pix * 64 + 8 * pswz(pix, 4 * s2 + (lane >> 4)));
}

typedef __attribute__((address_space(3))) const char patch_lds_t;

template <int EPI, bool DG, int PW>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(1, 1)))
void conv3x3_patch_kernel(GemmParams p, PatchGeom g) {
  static_assert(PW == 32 || PW == 64, "patch row pitch");
  constexpr int BM = 128, BN = 64, NW = 4, MT = 4, NT = 2;
  constexpr int PE = PATCH_SLICES * 512;  // elements per patch buffer
  constexpr int YE = 128 * 64;            // elements per y tile (EPI_BWD_AFF)
  constexpr bool BWD = EPI == EPI_BWD_AFF;
  constexpr int NY = BWD ? PATCH_RING : 0;
  constexpr int NIP = 8 + (BWD ? 4 : 0);  // LDS-DMA instructions per wave per tile
  __shared__ __attribute__((aligned(1024))) char smem[(PATCH_RING * PE + NY * YE) * 2];
  bf16_t* Ps = reinterpret_cast<bf16_t*>(smem);
  bf16_t* Ys = Ps + PATCH_RING * PE;

  const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave >> 1, wn = wave & 1;
  const int nx = p.N / BN, gy = gridDim.x / nx;
  int bx, by;
  if ((gy & 7) == 0) {  // XCD-aware decode (igemm_fast_kernel)
    const int sidx = blockIdx.x >> 3;
    bx = sidx % nx;
    by = (sidx / nx) * 8 + (blockIdx.x & 7);
  } else {
    bx = blockIdx.x % nx;
    by = blockIdx.x / nx;
  }
  const int n0 = bx * BN;
  bf16_t* Cout = reinterpret_cast<bf16_t*>(p.C);
  const int mtiles = p.M / g.TM;
  const int my_tiles = by < mtiles ? (mtiles - 1 - by) / gy + 1 : 0;
  const BwdEpi& e = p.bwd;
  if (my_tiles == 0) {
    if (BWD && e.nred > 0 && tid < BN)
      for (int r = 0; r < e.nred; ++r) e.part[((long long)by * e.nred + r) * p.N + n0 + tid] = 0.f;
    return;
  }

  const OpArgs& a = p.a;
  const uint32_t nbytes = (uint32_t)min(a.bytes, (long long)0xFFFFFF00LL);
  const __amdgpu_buffer_rsrc_t rsrc =
      __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(a.ptr), 0, nbytes, 0x00020000);
  // y of the dgrad epilogue ([M][ldc] bf16; absent: a zero-range descriptor, the DMAs return zeros)
  const uint32_t ybytes = (BWD && e.y) ? (uint32_t)min((long long)p.M * p.ldc * 2, (long long)0xFFFFFF00LL) : 0u;
  const __amdgpu_buffer_rsrc_t yrsrc =
      __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(BWD ? e.y : a.ptr), 0, ybytes, 0x00020000);
  const int HW = a.H * a.W;
  // One LDS-DMA piece (1 KiB per wave) of tile lt's loads, q < NIP: q < 8 patch slice wave + 4 q (slices >= NS
  // repeat slice NS - 1: identical bytes to the same place, so the instruction count per wave is fixed; the
  // source chunk is pre-swizzled, the LDS side is lane-linear); q >= 8: y rows 32 wave + 8 (q - 8) .. + 7 of the
  // tile, unswizzled [128][64]. (tg, img, h0: the tile's global index, image, first output row.)
  auto issue_piece = [&](int lt, int tg, int img, int h0, int q) {
    if (q < 8) {
      bf16_t* dst = Ps + (lt % PATCH_RING) * PE;
      const int slice = min(wave + NW * q, g.NS - 1);
      const int pix = 8 * slice + (lane >> 3);
      const int pr = pix / PW, pc = pix % PW;
      const int h = h0 - 1 + pr, w = pc - 1;
      const bool ok = pix < g.NP && (unsigned)h < (unsigned)a.H && (unsigned)w < (unsigned)a.W;
      const int csrc = ((lane & 7) - (pix & ~1)) & 7;  // pswz(pix, csrc) == lane & 7
      const uint32_t voff = ok ? (uint32_t)((((img * HW + h * a.W + w) << 6) + 8 * csrc) * 2) : nbytes;
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rsrc, (lds_void_t*)(dst + slice * 512), 16, voff, 0, 0, 0);
    } else if constexpr (BWD) {
      bf16_t* ydst = Ys + (lt % PATCH_RING) * YE;
      const int r0 = 32 * wave + 8 * (q - 8), r = r0 + (lane >> 3);
      const uint32_t voff =
          r < g.TM ? (uint32_t)(((long long)(tg * g.TM + r) * p.ldc + n0 + 8 * (lane & 7)) * 2) : ybytes;
      __builtin_amdgcn_raw_ptr_buffer_load_lds(yrsrc, (lds_void_t*)(ydst + r0 * 64), 16, ybytes ? voff : 0u, 0, 0, 0);
    }
  };
  auto issue_tile = [&](int lt) {
    const int tg = by + lt * gy, img = tg / g.TPI, h0 = (tg - img * g.TPI) * g.R;
#pragma unroll
    for (int q = 0; q < NIP; ++q) issue_piece(lt, tg, img, h0, q);
  };
  // register loads first, retired before the first DMA: hipcc's wait tracking then sees them complete inside
  // the loop (otherwise it puts counted vmcnt waits for them between the MFMAs, which also drain the DMAs)
  int rowpix[MT];  // patch pixel of tap (0, 0) for this lane's fragment row (dgrad: of tap (2, 2))
#pragma unroll
  for (int i = 0; i < MT; ++i) {
    const int ml = wm * 64 + i * 16 + (lane & 15);
    const int r = ml / a.W, w = ml - r * a.W;
    rowpix[i] = ml < g.TM ? r * PW + w : 0;
  }
  // B fragment (tap t, k-step s2, column group j): row n0 + wn*32 + 16j + lane%16, k = 64t + 32 s2 + 8 (lane/16)
  s16x8 breg[9][2][NT];
  {
    const bf16_t* B = reinterpret_cast<const bf16_t*>(p.b.ptr);
#pragma unroll
    for (int j = 0; j < NT; ++j) {
      const bf16_t* row = B + (long long)(n0 + wn * (BN / 2) + j * 16 + (lane & 15)) * p.b.ld + 8 * (lane >> 4);
#pragma unroll
      for (int t = 0; t < 9; ++t)
#pragma unroll
        for (int s2 = 0; s2 < 2; ++s2) breg[t][s2][j] = *reinterpret_cast<const s16x8*>(row + 64 * t + 32 * s2);
    }
  }
  // epilogue state: a flush thread always owns the 8-column chunk c = tid % 8
  constexpr int CPR = BN / 8, KC = 128 * BN / 8 / 256;
  const int cc = tid % CPR, ncol = n0 + 8 * cc;
  float mu[8], sc[8], sh[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    mu[i] = (BWD && e.mean) ? e.mean[ncol + i] : 0.f;
    sc[i] = (BWD && e.msc) ? e.msc[ncol + i] : 0.f;
    sh[i] = (BWD && e.msh) ? e.msh[ncol + i] : 0.f;
  }
  __builtin_amdgcn_s_waitcnt(waitcnt_vm(0));  // (once per kernel: no vmcnt waits for them inside the loop)
  issue_tile(0);
  if (my_tiles > 1) issue_tile(1);

  const bool mask = BWD && e.msc != nullptr && e.y != nullptr;
  float b1[8], b2[8], b3[8];  // EPI_STATS: shift, sum (v - shift), sum (v - shift)^2; EPI_BWD_AFF: sum g, sum g (y - mean)
  int scnt = 0;
#pragma unroll
  for (int i = 0; i < 8; ++i) b1[i] = b2[i] = b3[i] = 0.f;
  // The epilogue of tile lt is split: its output round is staged and read back into q (and the y chunks into yq)
  // at the end of the tile; the stores and statistics of chunk k run inside tile lt + 1's MFMA stream (unit
  // 2k + 1), and the last tile's after the loop.
  uint4 q[KC], yq[KC];
  int pm0 = 0, pmlim = 0;  // rows of the tile held in q
  auto process = [&](int k) {
    const int m = pm0 + (tid + 256 * k) / CPR;
    if (m >= pmlim) return;
    uint4* dst = reinterpret_cast<uint4*>(Cout + (long long)m * p.ldc + ncol);
    if constexpr (EPI == EPI_STORE) {
      *dst = q[k];
    } else if constexpr (EPI == EPI_STATS) {
      *dst = q[k];
      float v[8];
      unpack8(q[k], v);
      if (scnt == 0) {
#pragma unroll
        for (int i = 0; i < 8; ++i) b1[i] = v[i];
      }
      ++scnt;
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        const float d = v[i] - b1[i];
        b2[i] += d;
        b3[i] = fmaf(d, d, b3[i]);
      }
    } else {  // g = mask(dgrad) stored; BN sums of the stored (rounded) g against y
      float v[8], yy[8];
      unpack8(q[k], v);
      unpack8(yq[k], yy);
      if (mask) {
#pragma unroll
        for (int i = 0; i < 8; ++i) v[i] = fmaf(yy[i], sc[i], sh[i]) > 0.f ? v[i] : 0.f;
      }
      uint4 o;
      o.x = (uint32_t)f2bf(v[0]) | ((uint32_t)f2bf(v[1]) << 16);
      o.y = (uint32_t)f2bf(v[2]) | ((uint32_t)f2bf(v[3]) << 16);
      o.z = (uint32_t)f2bf(v[4]) | ((uint32_t)f2bf(v[5]) << 16);
      o.w = (uint32_t)f2bf(v[6]) | ((uint32_t)f2bf(v[7]) << 16);
      *dst = o;
      if (e.nred > 0) {
        unpack8(o, v);
#pragma unroll
        for (int i = 0; i < 8; ++i) {
          b1[i] += v[i];
          b2[i] = fmaf(v[i], yy[i] - mu[i], b2[i]);
        }
      }
    }
  };

  for (int lt = 0; lt < my_tiles; ++lt) {
    // tile lt's DMAs have landed for every wave (tile lt + 1's, issued after them, may still be in flight)
    PATCH_STAMP(0);
    if (lt + 1 < my_tiles) __builtin_amdgcn_s_waitcnt(waitcnt_vm(NIP));
    else __builtin_amdgcn_s_waitcnt(waitcnt_vm(0));
    __builtin_amdgcn_s_barrier();
    PATCH_STAMP(1);
    // tile lt + 2's DMAs go out one piece per unit, into the ring slot of tile lt - 1 (free: its q / yq reads
    // completed before the barrier above)
    const bool pre = lt + 2 < my_tiles;
    const int tg2 = by + (lt + 2) * gy, img2 = tg2 / g.TPI, h02 = (tg2 - img2 * g.TPI) * g.R;
    const bool prev = lt > 0;
    PATCH_STAMP(2);
    const bf16_t* P = Ps + (lt % PATCH_RING) * PE;
    f32x4 acc[MT][NT];
#pragma unroll
    for (int i = 0; i < MT; ++i)
#pragma unroll
      for (int j = 0; j < NT; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
    // 18 units (tap t = u / 2, k-step u % 2) of 4 fragment reads + 8 MFMAs, reads issued two units ahead (a ring
    // of 3 fragment sets; the scheduler barriers keep hipcc from regrouping them into read-wait-MFMA pairs, whose
    // exposed LDS latency made the first build of this loop 4x slower than its MFMA time)
    // fragment addresses of this tile: column tap c (= kw, dgrad 2 - kw), k-step s2; row taps add kh' PW pixels
    uint32_t fa[MT][3][2];
#pragma unroll
    for (int i = 0; i < MT; ++i)
#pragma unroll
      for (int c = 0; c < 3; ++c) {
        const int pix = rowpix[i] + c;
        const uint32_t a0 = lds_u32(P + pix * 64 + 8 * pswz(pix, lane >> 4));
        fa[i][c][0] = a0;
        fa[i][c][1] = a0 ^ 64u;  // chunk + 4: slot (c + 4 + x) & 7 = ((c + x) & 7) ^ 4
      }
    auto unit_reads = [&](s16x8 (&f)[MT], int u) {
      const int t = u >> 1, kh = t / 3, kw = t - 3 * (t / 3);
      const int rh = DG ? 2 - kh : kh, cw = DG ? 2 - kw : kw;
#pragma unroll
      for (int i = 0; i < MT; ++i)
        f[i] = *reinterpret_cast<const __attribute__((address_space(3))) s16x8*>(
            (patch_lds_t*)(uintptr_t)fa[i][cw][u & 1] + rh * PW * 128);
    };
    s16x8 af[3][MT];
    unit_reads(af[0], 0);
    unit_reads(af[1], 1);
#pragma unroll
    for (int u = 0; u < 18; ++u) {
      if (u + 2 < 18) unit_reads(af[(u + 2) % 3], u + 2);
      if (u < NIP && pre) issue_piece(lt + 2, tg2, img2, h02, u);
      // the previous tile's stores / statistics in units after the DMA issues (both are expensive beside the MFMAs:
      // the dgrad epilogue's ~60 VALU per chunk exceeds a unit's MFMA shadow)
      if constexpr (NIP + 2 * KC <= 18) {
        if (u >= NIP && ((u - NIP) & 1) == 0 && ((u - NIP) >> 1) < KC && prev) process((u - NIP) >> 1);
      } else {
        if (u >= 18 - KC && prev) process(u - (18 - KC));
      }
#pragma unroll
      for (int i = 0; i < MT; ++i)
#pragma unroll
        for (int j = 0; j < NT; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(breg[u >> 1][u & 1][j], af[u % 3][i], acc[i][j], 0, 0, 0);
      __builtin_amdgcn_sched_barrier(0);
    }
    PATCH_STAMP(3);
    __builtin_amdgcn_s_waitcnt(0xC07F);  // lgkmcnt(0): every wave's fragment reads are back before the staging
    __builtin_amdgcn_s_barrier();
    PATCH_STAMP(4);
    // stage the round in this tile's patch slot, read this thread's chunks (and y chunks) back
    bf16_t* stA = Ps + (lt % PATCH_RING) * PE;
#pragma unroll
    for (int j = 0; j < NT; ++j)
#pragma unroll
      for (int i = 0; i < MT; ++i) {
        float v[4] = {acc[i][j][0], acc[i][j][1], acc[i][j][2], acc[i][j][3]};
        stage_put<BM, BN>(stA, stA, wm, wn, lane, i, j, v);
      }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    const bf16_t* Y = Ys + (lt % PATCH_RING) * YE;
#pragma unroll
    for (int k = 0; k < KC; ++k) {
      const int trow = (tid + 256 * k) / CPR;
      asm volatile("ds_read_b128 %0, %1" : "=v"(q[k]) : "v"(lds_u32(stA + trow * BN + 8 * st_slot<BN>(trow, cc))) : "memory");
      if constexpr (BWD)
        asm volatile("ds_read_b128 %0, %1" : "=v"(yq[k]) : "v"(lds_u32(Y + trow * 64 + 8 * cc)) : "memory");
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    pm0 = (by + lt * gy) * g.TM;
    pmlim = pm0 + g.TM;
    PATCH_STAMP(5);
  }
#pragma unroll
  for (int k = 0; k < KC; ++k) process(k);
  __builtin_amdgcn_s_waitcnt(waitcnt_vm(0));
  if constexpr (EPI == EPI_STATS)
    stats_finish<BM, BN>(p, reinterpret_cast<float*>(smem), scnt, b1, b2, b3, n0, by, bx, gy, (p.M + 127) / 128);
  if constexpr (BWD) {
    if (e.nred > 0) {
      float* inv = reinterpret_cast<float*>(smem) + 3 * 256 * 8;  // beyond bwd_finish's scratch
      __syncthreads();
      if (tid < BN) inv[tid] = e.invstd ? e.invstd[n0 + tid] : 0.f;
      bwd_finish<BM, BN>(p, reinterpret_cast<float*>(smem), inv, b1, b2, b3, n0, by);
    }
  }
}

// ---- the pair-packed stem (7x7 / stride 2 / pad 3 over RGB0 bf16 frames, vcg_conv_fwd's C = 4 layout) --------
// Same scheme as the layer-1 patch kernel: an M-tile is R whole output rows of one image; its input rows
// (2R + KH - 2 rows of OW + KWp - 1 super pixels, 16 B = two RGB0 pixels each) are one LDS-DMA patch, and the
// KH k-units (4 taps each: the super-pixel pairs kwp = 0..3 of filter row kh) read fragments straight from it:
// lane group g = kwp, so a fragment read is 16 consecutive super pixels (contiguous 256 B, conflict-free). The
// im2col engine gathers every input super pixel ~14 times through L2. The filter (64 x 224) stays in registers
// (14 fragments per lane), 2 workgroups per CU, a 3-deep patch ring, the deferred epilogue of the patch kernel.
constexpr int SPATCH_MAXPIX = 1024;  // super pixels per patch buffer (16 KiB)

struct StemGeom {
  int R, TM, TPI, PW, NP, NS, NR;  // rows / GEMM rows per tile, tiles per image, patch width, pixels, slices, rows
  unsigned long long* stamps;
};

template <int EPI>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(2, 2)))
void stem_patch_kernel(GemmParams p, StemGeom g) {
  constexpr int BM = 128, BN = 64, NW = 4, MT = 4, NT = 2, KHMAX = 8, RING = 3, NIP = 4;
  constexpr int PE = SPATCH_MAXPIX * 8;  // elements per patch buffer
  __shared__ __attribute__((aligned(1024))) char smem[RING * PE * 2];
  bf16_t* Ps = reinterpret_cast<bf16_t*>(smem);
  const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave >> 1, wn = wave & 1;
  const int nx = p.N / BN, gy = gridDim.x / nx;
  int bx, by;
  if ((gy & 7) == 0) {
    const int sidx = blockIdx.x >> 3;
    bx = sidx % nx;
    by = (sidx / nx) * 8 + (blockIdx.x & 7);
  } else {
    bx = blockIdx.x % nx;
    by = blockIdx.x / nx;
  }
  const int n0 = bx * BN;
  bf16_t* Cout = reinterpret_cast<bf16_t*>(p.C);
  const int mtiles = p.M / g.TM;
  const int my_tiles = by < mtiles ? (mtiles - 1 - by) / gy + 1 : 0;
  if (my_tiles == 0) return;

  const OpArgs& a = p.a;  // a.W: super pixels per image row, a.C = 8, a.KW = 4 super-pixel taps, a.pw their pad
  const int KH = a.KH;
  const uint32_t nbytes = (uint32_t)min(a.bytes, (long long)0xFFFFFF00LL);
  const __amdgpu_buffer_rsrc_t rsrc =
      __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(a.ptr), 0, nbytes, 0x00020000);
  // piece q < NIP of tile lt: 64 super pixels (slice wave + 4 q, repeated past NS - 1: fixed count per wave)
  auto issue_piece = [&](int lt, int img, int h0, int q) {
    bf16_t* dst = Ps + (lt % RING) * PE;
    const int slice = min(wave + NW * q, g.NS - 1);
    const int pix = 64 * slice + lane;
    const int pr = pix / g.PW, pc = pix - pr * g.PW;
    const int ih = 2 * h0 - a.pad + pr, sx = pc - a.pw;
    const bool ok = pix < g.NP && (unsigned)ih < (unsigned)a.H && (unsigned)sx < (unsigned)a.W;
    const uint32_t voff = ok ? (uint32_t)((((img * a.H + ih) * a.W + sx) << 3) * 2) : nbytes;
    __builtin_amdgcn_raw_ptr_buffer_load_lds(rsrc, (lds_void_t*)(dst + slice * 512), 16, voff, 0, 0, 0);
  };
  auto issue_tile = [&](int lt) {
    const int tg = by + lt * gy, img = tg / g.TPI, h0 = (tg - img * g.TPI) * g.R;
#pragma unroll
    for (int q = 0; q < NIP; ++q) issue_piece(lt, img, h0, q);
  };
  int rowpix[MT];  // patch super pixel of tap (kh = 0, kwp = 0) for this lane's fragment row
#pragma unroll
  for (int i = 0; i < MT; ++i) {
    const int ml = wm * 64 + i * 16 + (lane & 15);
    const int r = ml / a.GW, w = ml - r * a.GW;
    rowpix[i] = ml < g.TM ? 2 * r * g.PW + w : 0;
  }
  // B fragment of filter row kh, column group j: k = 32 kh + 8 (lane / 16) (taps kwp = lane / 16 of row kh)
  s16x8 breg[KHMAX][NT];
  {
    const bf16_t* B = reinterpret_cast<const bf16_t*>(p.b.ptr);
#pragma unroll
    for (int j = 0; j < NT; ++j) {
      const bf16_t* row = B + (long long)(n0 + wn * (BN / 2) + j * 16 + (lane & 15)) * p.b.ld + 8 * (lane >> 4);
#pragma unroll
      for (int kh = 0; kh < KHMAX; ++kh)
        breg[kh][j] = kh < KH ? *reinterpret_cast<const s16x8*>(row + 32 * kh) : s16x8{0, 0, 0, 0, 0, 0, 0, 0};
    }
  }
  constexpr int CPR = BN / 8, KC = 128 * BN / 8 / 256;
  const int cc = tid % CPR, ncol = n0 + 8 * cc;
  __builtin_amdgcn_s_waitcnt(waitcnt_vm(0));  // register loads retired before the first DMA (see the patch kernel)
  issue_tile(0);
  if (my_tiles > 1) issue_tile(1);

  float b1[8], b2[8], b3[8];
  int scnt = 0;
#pragma unroll
  for (int i = 0; i < 8; ++i) b1[i] = b2[i] = b3[i] = 0.f;
  uint4 q[KC];
  int pm0 = 0, pmlim = 0;
  auto process = [&](int k) {
    const int m = pm0 + (tid + 256 * k) / CPR;
    if (m >= pmlim) return;
    *reinterpret_cast<uint4*>(Cout + (long long)m * p.ldc + ncol) = q[k];
    if constexpr (EPI == EPI_STATS) {
      float v[8];
      unpack8(q[k], v);
      if (scnt == 0) {
#pragma unroll
        for (int i = 0; i < 8; ++i) b1[i] = v[i];
      }
      ++scnt;
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        const float d = v[i] - b1[i];
        b2[i] += d;
        b3[i] = fmaf(d, d, b3[i]);
      }
    }
  };

  for (int lt = 0; lt < my_tiles; ++lt) {
    if (lt + 1 < my_tiles) __builtin_amdgcn_s_waitcnt(waitcnt_vm(NIP));
    else __builtin_amdgcn_s_waitcnt(waitcnt_vm(0));
    __builtin_amdgcn_s_barrier();
    const bool pre = lt + 2 < my_tiles;
    const int tg2 = by + (lt + 2) * gy, img2 = tg2 / g.TPI, h02 = (tg2 - img2 * g.TPI) * g.R;
    const bool prev = lt > 0;
    const bf16_t* P = Ps + (lt % RING) * PE;
    // opaque per tile: keeps hipcc from hoisting the loop-invariant fragment addresses (registers)
#pragma unroll
    for (int i = 0; i < MT; ++i) asm volatile("" : "+v"(rowpix[i]));
    f32x4 acc[MT][NT];
#pragma unroll
    for (int i = 0; i < MT; ++i)
#pragma unroll
      for (int j = 0; j < NT; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
    auto unit_reads = [&](s16x8 (&f)[MT], int kh) {
#pragma unroll
      for (int i = 0; i < MT; ++i)
        f[i] = *reinterpret_cast<const s16x8*>(P + (rowpix[i] + kh * g.PW + (lane >> 4)) * 8);
    };
    s16x8 af[3][MT];
    unit_reads(af[0], 0);
    unit_reads(af[1], 1);
#pragma unroll
    for (int u = 0; u < KHMAX; ++u) {
      if (u < KH) {
        if (u + 2 < KH) unit_reads(af[(u + 2) % 3], u + 2);
        if (u < NIP && pre) issue_piece(lt + 2, img2, h02, u);
        if (u >= 1 && u - 1 < KC && prev) process(u - 1);
#pragma unroll
        for (int i = 0; i < MT; ++i)
#pragma unroll
          for (int j = 0; j < NT; ++j)
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(breg[u][j], af[u % 3][i], acc[i][j], 0, 0, 0);
        __builtin_amdgcn_sched_barrier(0);
      }
    }
    if (prev) {  // chunks not yet processed when KH - 1 < KC
#pragma unroll
      for (int k = 0; k < KC; ++k)
        if (k >= KH - 1) process(k);
    }
    __builtin_amdgcn_s_waitcnt(0xC07F);
    __builtin_amdgcn_s_barrier();
    bf16_t* stA = Ps + (lt % RING) * PE;
#pragma unroll
    for (int j = 0; j < NT; ++j)
#pragma unroll
      for (int i = 0; i < MT; ++i) {
        float v[4] = {acc[i][j][0], acc[i][j][1], acc[i][j][2], acc[i][j][3]};
        stage_put<BM, BN>(stA, stA, wm, wn, lane, i, j, v);
      }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
#pragma unroll
    for (int k = 0; k < KC; ++k) {
      const int trow = (tid + 256 * k) / CPR;
      asm volatile("ds_read_b128 %0, %1" : "=v"(q[k]) : "v"(lds_u32(stA + trow * BN + 8 * st_slot<BN>(trow, cc))) : "memory");
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    pm0 = (by + lt * gy) * g.TM;
    pmlim = pm0 + g.TM;
  }
#pragma unroll
  for (int k = 0; k < KC; ++k) process(k);
  __builtin_amdgcn_s_waitcnt(waitcnt_vm(0));
  if constexpr (EPI == EPI_STATS)
    stats_finish<BM, BN>(p, reinterpret_cast<float*>(smem), scnt, b1, b2, b3, n0, by, bx, gy, (p.M + 127) / 128);
}

// Rows per stem tile (0: not the pair-packed 7x7 / 2 stem shape the stem kernel handles)
static int stem_rows(const GemmParams& p) {
  const char* e = getenv("VCG_NO_PATCH");
  const OpArgs& a = p.a;
  if ((e && e[0] == '1') || a.C != 8 || a.sw != 1 || a.KW != 4 || a.stride != 2 || a.KH > 8 || a.KH < 3 ||
      p.K != a.KH * 32 || a.tsm_fold != 0 || p.N % 64 != 0 || p.batch_inner > 0 || p.residual || p.aux || p.bias ||
      p.act != ACT_NONE || a.GW > 128 || a.GW + 3 > SPATCH_MAXPIX)
    return 0;
  for (int R = min(a.GH, 128 / a.GW); R >= 1; --R)
    if (a.GH % R == 0 && (2 * R + a.KH - 2) * (a.GW + 3) <= SPATCH_MAXPIX) return R;
  return 0;
}

static StemGeom stem_geom(const GemmParams& p, int R) {
  StemGeom g{};
  g.R = R;
  g.TM = R * p.a.GW;
  g.TPI = p.a.GH / R;
  g.PW = p.a.GW + p.a.KW - 1;
  g.NR = 2 * R + p.a.KH - 2;
  g.NP = g.NR * g.PW;
  g.NS = (g.NP + 63) / 64;
  return g;
}

// Patch row pitch in pixels (the kernel's PW): 32 or 64 >= W + 2 (the two zero border columns)
static int patch_pitch(int W) { return W + 2 <= 32 ? 32 : 64; }

// Rows per patch tile (0: the patch kernel does not apply). VCG_NO_PATCH=1 keeps these convs on the im2col path.
static int patch_rows(const GemmParams& p, int amode) {
  const char* e = getenv("VCG_NO_PATCH");  // read per call: a test compares both paths in one process
  const bool off = e && e[0] == '1';
  const OpArgs& a = p.a;
  if (off || (amode != OP_IM2COL && amode != OP_DGRAD) || a.C != 64 || a.KH != 3 || a.KW != 3 || a.stride != 1 ||
      a.pad != 1 || a.tsm_fold != 0 || a.tKW != 0 || a.sw != 0 || a.GH != a.H || a.GW != a.W || p.N % 64 != 0 ||
      p.K != 9 * 64 || p.batch_inner > 0 || p.residual || p.aux || p.bias || p.act != ACT_NONE || a.W + 2 > 64 ||
      !bwd_light(p) || p.bwd.nred > 2)
    return 0;
  for (int R = min(a.H, 128 / a.W); R >= 1; --R)
    if (a.H % R == 0 && (R + 2) * patch_pitch(a.W) <= PATCH_MAXPIX) return R;
  return 0;
}

static PatchGeom patch_geom(const GemmParams& p, int R) {
  PatchGeom g{};
  g.R = R;
  g.TM = R * p.a.W;
  g.TPI = p.a.H / R;
  g.PW = patch_pitch(p.a.W);
  g.NP = (R + 2) * g.PW;
  g.NS = (g.NP + 7) / 8;
  return g;
}

// one resident round (1 workgroup per CU); gy <= the 128-row slot count of the EPI_STATS buffer
static int patch_grid_rows(const GemmParams& p, const PatchGeom& g) {
  const int nx = p.N / 64, mtiles = p.M / g.TM;
  int gy = 256 / nx;
  gy = min(gy, min(mtiles, (p.M + 127) / 128));
  if (gy >= 8) gy &= ~7;
  return max(gy, 1);
}

// EPI_BWD_STREAM applies to a full EPI_BWD (residual; mask bits with y, or neither) of a dense 1x1 dgrad with
// K = 64, 128 or 256 (256: every 64-column tile inside one TSM shift); VCG_BWD_STREAM=0 keeps it on the persistent
// engine (read per call: tests compare both paths)
static bool bwd_stream_ok(const GemmParams& p) {
  const char* v = getenv("VCG_BWD_STREAM");
  if (v && v[0] == '0') return false;
  const BwdEpi& e = p.bwd;
  const bool dense = p.a.KH == 0 && p.a.GH == 0;  // dense_op(): no conv geometry
  if (!dense || (p.K != 64 && p.K != 128 && p.K != 256) || p.N % 64 != 0 || p.batch_inner > 0 || p.ldc != p.N || p.a.ld != p.K ||
      !e.res || e.msc || e.sub || bwd_light(p))
    return false;
  if ((e.y && !e.bits) || (e.y2 && !e.y)) return false;
  if ((e.y || e.bits) && e.nred < 2) return false;
  if (e.tsm_T > 0 && e.tsm_fold % 32 != 0) return false;  // one TSM shift per wave's 32 columns
  // K = 256: one A tile per slot and 3 slots; with y the 64 x 64 form measured slower than the persistent engine
  // (tools/bench_dgrad.py: 400.6 vs 385.1 us at layer 3), so only the mask-bits-only epilogues stream
  if (p.K == 256 && ((e.tsm_T > 0 && e.tsm_fold % 64 != 0) || e.y)) return false;
  if (p.K == 256 && ((uintptr_t)p.b.ptr & 15 || p.b.ld % 8 != 0)) return false;  // 16-B weight fragment loads
  if (((uintptr_t)p.C | (uintptr_t)e.res | (uintptr_t)e.y | (uintptr_t)e.y2 | (uintptr_t)p.a.ptr) & 15) return false;
  if (e.res_s > 1 && (p.M % e.hw) != 0) return false;
  if (e.pj > 0) {  // P = g^T a2 (a2 of 64 columns: layer 1): the mask bits alone, K 64 / 128
    if (e.y || !e.bits || e.pj != 64 || p.K > 128 || ((uintptr_t)e.a2 & 15) || !e.ppart) return false;
    if (((uintptr_t)p.b.ptr & 15) || p.b.ld % 8 != 0) return false;  // weight fragments in registers
  }
  return true;
}

// column tile of the streaming kernel: 128 for K = 256 with the mask bits alone and one TSM shift per 128 columns
// (bwd_stream128_body), else 64; VCG_BWD_STREAM=64 keeps 64 (read per call: tests compare the tilings)
static int bwd_stream_tn(const GemmParams& p) {
  const BwdEpi& e = p.bwd;
  const char* v = getenv("VCG_BWD_STREAM");
  if ((v && v[0] == '6') || p.bwd.pj > 0) return 64;  // (the P product lives in the 64-column kernel)
  return p.K == 256 && p.N % 128 == 0 && !e.y && (e.tsm_T <= 0 || e.tsm_fold % 128 == 0) ? 128 : 64;
}

static int bwd_stream_rows(const GemmParams& p) {
  const int nx = p.N / bwd_stream_tn(p), mtiles = (p.M + 63) / 64;
  int gy = 256 / nx;  // one workgroup per CU (~100-147 KB of LDS)
  if (gy >= 8) gy &= ~7;
  if (gy > mtiles) gy = mtiles >= 8 ? (mtiles & ~7) : mtiles;
  return gy < 1 ? 1 : gy;
}

bool fast_bwd_streams(const GemmParams& p) { return bwd_stream_ok(p); }

int fast_bwd_slots(const GemmParams& p) {
  if (bwd_stream_ok(p)) return bwd_stream_rows(p);
  const int R = patch_rows(p, OP_DGRAD);
  if (R > 0) return patch_grid_rows(p, patch_geom(p, R));
  return fast_grid_rows(p.M, p.N, 1, bwd_light(p) ? EPI_BWD_AFF : EPI_BWD);
}

// Algorithmic HBM bytes of one launch (bench.py's per-launch roofline): every operand read once (a gathered A:
// the source tensor once), the output written once, the epilogue's extra operands read once (bf16).
template <int AM, int EPI, int RES>
static double algorithmic_bytes(const GemmParams& p, int z) {
  const double mn = (double)p.M * p.N * z;
  double b = (AM == OP_DENSE_K || AM == OP_DENSE_K2 ? 2.0 * p.M * (double)p.K * z : (double)p.a.bytes) + 2.0 * p.N * (double)p.K * z;
  b += 2.0 * mn;
  if (RES) b += 2.0 * mn;
  if (p.aux) b += 2.0 * mn;
  if constexpr (EPI == EPI_BWD || EPI == EPI_BWD_AFF) {
    const BwdEpi& e = p.bwd;
    if (e.res) b += 2.0 * mn / (e.res_s > 1 ? 4.0 : 1.0);
    if (e.y) b += 2.0 * mn;
    if (e.y2) b += 2.0 * mn;
    if (e.bits) b += mn / 8.0;
  }
  return b;
}

template <int BM, int BN, int AM, int EPI, int RES>
static int launch_fast(const GemmParams& p, int z, hipStream_t s) {
  const int nx = (p.N + BN - 1) / BN;
  const int gy = grid_rows(p.M, p.N, z, BM, BN, EPI);
  dim3 grid(nx * gy, 1, z);
  const int tk = timing_begin(s);
  hipLaunchKernelGGL((igemm_fast_kernel<BM, BN, AM, EPI, RES>), grid, dim3(BM * 2), 0, s, p);
  if (census_on()) { char t_[96]; snprintf(t_, sizeof(t_), "igemm_fast %dx%d a%d e%d r%d z%d", BM, BN, AM, EPI, RES, z); census_add(t_, p.M, p.N, p.K); }
  timing_end(tk, s, TIMING_FAST_GEMM, 2.0 * p.M * p.N * (double)p.K * z, algorithmic_bytes<AM, EPI, RES>(p, z));
  VCG_LAUNCH_CHECK();
  return VCG_OK;
}

template <int KC, int XF, int TN = 64>
static int launch_bwd_stream(const GemmParams& p, hipStream_t s) {
  const int nx = p.N / TN, gy = bwd_stream_rows(p);
  const int tk = timing_begin(s);
  hipLaunchKernelGGL((igemm_fast_kernel<256, TN, KC, EPI_BWD_STREAM, false, XF>), dim3(nx * gy), dim3(512), 0, s, p);
  if (census_on()) { char t_[96]; snprintf(t_, sizeof(t_), "igemm_fast_stream tn%d xf%d", TN, XF); census_add(t_, p.M, p.N, p.K); }
  // (with the g^T a2 product: + its flops, the a2 read and the P slabs written and reduced)
  const double pj = bwd_stream_pj(XF);
  timing_end(tk, s, TIMING_FAST_GEMM, 2.0 * p.M * p.N * (double)p.K + 2.0 * p.M * p.N * pj,
             algorithmic_bytes<OP_DENSE_K, EPI_BWD, false>(p, 1) + 2.0 * p.M * pj + 4.0 * p.N * pj);
  VCG_LAUNCH_CHECK();
  return VCG_OK;
}

template <int KC>
static int run_bwd_stream(const GemmParams& p, hipStream_t s) {
  if constexpr (KC == 4) {
    if (bwd_stream_tn(p) == 128)
      return p.bwd.bits ? launch_bwd_stream<4, XF_BITS, 128>(p, s) : launch_bwd_stream<4, 0, 128>(p, s);
  }
  if constexpr (KC <= 2) {
    if (p.bwd.pj == 64) return launch_bwd_stream<KC, XF_BITS | XF_P64>(p, s);
  }
  if (!p.bwd.y) return p.bwd.bits ? launch_bwd_stream<KC, XF_BITS>(p, s) : launch_bwd_stream<KC, 0>(p, s);
  if (!p.bwd.y2) return launch_bwd_stream<KC, XF_HASY>(p, s);
  return launch_bwd_stream<KC, XF_HASY | XF_Y2>(p, s);
}

template <int AM, int EPI, int RES = 0>
static int fast_bn(const GemmParams& p, int z, hipStream_t s) {
  if (fast_bn_cols(p.N) == 128) return launch_fast<128, 128, AM, EPI, RES>(p, z, s);
  return launch_fast<128, 64, AM, EPI, RES>(p, z, s);
}

static unsigned long long* g_patch_stamps = nullptr;

template <int EPI, bool DG, int PW>
static int launch_patch(const GemmParams& p, int R, hipStream_t s) {
  const PatchGeom g = patch_geom(p, R);
  const int gy = patch_grid_rows(p, g);
  const int tk = timing_begin(s);
  PatchGeom gs = g;
  const char* st = getenv("VCG_PATCH_STAMPS");
  if (st && st[0] == '1') {
    if (!g_patch_stamps && hipMalloc(&g_patch_stamps, 64 * 6 * 8) != hipSuccess) g_patch_stamps = nullptr;
    gs.stamps = g_patch_stamps;
  }
  hipLaunchKernelGGL((conv3x3_patch_kernel<EPI, DG, PW>), dim3((p.N / 64) * gy), dim3(256), 0, s, p, gs);
  if (census_on()) { char t_[96]; snprintf(t_, sizeof(t_), "conv3x3_patch e%d dg%d pw%d", EPI, (int)DG, PW); census_add(t_, p.M, p.N, p.K); }
  timing_end(tk, s, TIMING_PATCH_CONV, 2.0 * p.M * p.N * (double)p.K, algorithmic_bytes<OP_IM2COL, EPI, false>(p, 1));
  VCG_LAUNCH_CHECK();
  return VCG_OK;
}

template <int EPI>
static int launch_stem(const GemmParams& p, int R, hipStream_t s) {
  const StemGeom g = stem_geom(p, R);
  const int nx = p.N / 64, mtiles = p.M / g.TM;
  int gy = min((2 * 256) / nx, min(mtiles, (p.M + 127) / 128));
  if (gy >= 8) gy &= ~7;
  gy = max(gy, 1);
  const int tk = timing_begin(s);
  hipLaunchKernelGGL((stem_patch_kernel<EPI>), dim3(nx * gy), dim3(256), 0, s, p, g);
  if (census_on()) { char t_[96]; snprintf(t_, sizeof(t_), "stem_patch e%d", EPI); census_add(t_, p.M, p.N, p.K); }
  timing_end(tk, s, TIMING_PATCH_CONV, 2.0 * p.M * p.N * (double)p.K, algorithmic_bytes<OP_IM2COL, EPI, false>(p, 1));
  VCG_LAUNCH_CHECK();
  return VCG_OK;
}

// Entry from igemm.hip's dispatcher (bf16, K-contiguous A and B, no split-K).
// (Every output tile goes through the LDS stage: measured never slower, tools/bench_gemm.py, round 2.)
int run_fast_gemm(GemmParams& p, int amode, int epi, int z, hipStream_t s) {
  if (p.a.ptr2) {  // a BatchNorm backward folded into this input gradient: A = [g | y] (light epilogue only)
    if (amode != OP_DENSE_K || epi != EPI_BWD || z != 1 || !bwd_light(p) || p.a.split2 % FBK != 0) return -1;
    return fast_bn<OP_DENSE_K2, EPI_BWD_AFF>(p, z, s);
  }
  if (amode == OP_IM2COL && p.a.tsm_fold > 0) amode = OP_IM2COL_TSM;
  if (amode == OP_IM2COL && p.a.C < FBK) amode = OP_IM2COL_SMALLC;
  if (amode == OP_IM2COL_TSM && p.a.C < FBK) return -1;  // (dispatcher keeps these off the fast path)
  if (amode == OP_DGRAD && p.a.C < FBK) return -1;
  if (z == 1 && amode == OP_IM2COL_SMALLC && (epi == EPI_STATS || epi == EPI_STORE)) {
    const int R = stem_rows(p);
    if (R > 0) return epi == EPI_STATS ? launch_stem<EPI_STATS>(p, R, s) : launch_stem<EPI_STORE>(p, R, s);
  }
  if (z == 1) {
    const int R = patch_rows(p, amode);
    if (R > 0) {
      const bool w64 = patch_pitch(p.a.W) == 64;
      if (amode == OP_DGRAD) {
        if (epi == EPI_BWD)  // (patch_rows: light epilogues only)
          return w64 ? launch_patch<EPI_BWD_AFF, true, 64>(p, R, s) : launch_patch<EPI_BWD_AFF, true, 32>(p, R, s);
        if (epi == EPI_STATS)
          return w64 ? launch_patch<EPI_STATS, true, 64>(p, R, s) : launch_patch<EPI_STATS, true, 32>(p, R, s);
        if (epi == EPI_STORE)
          return w64 ? launch_patch<EPI_STORE, true, 64>(p, R, s) : launch_patch<EPI_STORE, true, 32>(p, R, s);
      } else {
        if (epi == EPI_STATS)
          return w64 ? launch_patch<EPI_STATS, false, 64>(p, R, s) : launch_patch<EPI_STATS, false, 32>(p, R, s);
        if (epi == EPI_STORE)
          return w64 ? launch_patch<EPI_STORE, false, 64>(p, R, s) : launch_patch<EPI_STORE, false, 32>(p, R, s);
      }
    }
  }
  if (amode != OP_IM2COL_SMALLC && gemm256_ok(p, amode, epi, z)) return run_gemm256(p, amode, epi, s);
  if (epi == EPI_BWD && amode == OP_DENSE_K && z == 1 && bwd_stream_ok(p))
    return p.K == 64 ? run_bwd_stream<1>(p, s) : p.K == 128 ? run_bwd_stream<2>(p, s) : run_bwd_stream<4>(p, s);
  if (epi == EPI_BWD && bwd_light(p)) {
    if (amode == OP_DGRAD) return fast_bn<OP_DGRAD, EPI_BWD_AFF>(p, z, s);
    if (amode == OP_DENSE_K) return fast_bn<OP_DENSE_K, EPI_BWD_AFF>(p, z, s);
    return -1;
  }
  if (epi == EPI_BWD) {
    if (amode == OP_DGRAD) return fast_bn<OP_DGRAD, EPI_BWD>(p, z, s);
    if (amode == OP_DENSE_K) return fast_bn<OP_DENSE_K, EPI_BWD>(p, z, s);
    return -1;
  }
  if (epi == EPI_STATS) {
    if (amode == OP_IM2COL_SMALLC) return fast_bn<OP_IM2COL_SMALLC, EPI_STATS>(p, z, s);
    if (amode == OP_IM2COL_TSM) return fast_bn<OP_IM2COL_TSM, EPI_STATS>(p, z, s);
    if (amode == OP_IM2COL) return fast_bn<OP_IM2COL, EPI_STATS>(p, z, s);
    if (amode == OP_DGRAD) return fast_bn<OP_DGRAD, EPI_STATS>(p, z, s);
    return fast_bn<OP_DENSE_K, EPI_STATS>(p, z, s);
  }
  // dense layers only; RES = 2: the GELU' x residual epilogue (BERT FFN2's input gradient) as its own kernel -- in
  // the ReLU / add instantiation its erf code raised register use and slowed the scoring forward's folded conv3
  // GEMMs by ~10 % (2.72-2.76 K vs 3.06 K windows/s, bisected to that change)
  if (p.residual) return p.act == ACT_GELU_BWD ? fast_bn<OP_DENSE_K, EPI_STORE, 2>(p, z, s)
                                               : fast_bn<OP_DENSE_K, EPI_STORE, 1>(p, z, s);
  if (p.aux && amode == OP_DENSE_K && (p.ldc & 7) == 0)  // a GELU input kept for the backward
    return fast_bn<OP_DENSE_K, EPI_STORE_AUX>(p, z, s);
  if (amode == OP_IM2COL_SMALLC) return fast_bn<OP_IM2COL_SMALLC, EPI_STORE>(p, z, s);
  if (amode == OP_IM2COL_TSM) return fast_bn<OP_IM2COL_TSM, EPI_STORE>(p, z, s);
  if (amode == OP_IM2COL) return fast_bn<OP_IM2COL, EPI_STORE>(p, z, s);
  if (amode == OP_DGRAD) return fast_bn<OP_DGRAD, EPI_STORE>(p, z, s);
  return fast_bn<OP_DENSE_K, EPI_STORE>(p, z, s);
}

}  // namespace vcg

// Profiling aid: the phase stamps (s_memtime) of the last patch-conv launch with VCG_PATCH_STAMPS=1, workgroup 0
// wave 0, 6 per tile (top, after wait+barrier, after DMA issue, after MFMAs, after barrier, after epilogue).
VCG_API int vcg_fast_stamps(unsigned long long* out, int n) {
#ifdef VCG_FAST_STAMPS
  n = n < 64 * 4 ? n : 64 * 4;
  return hipMemcpyFromSymbol(out, HIP_SYMBOL(vcg::g_fast_stamps), (size_t)n * 8, 0, hipMemcpyDeviceToHost) == hipSuccess
             ? 0 : 2;
#else
  (void)out;
  (void)n;
  return 1;
#endif
}

VCG_API int vcg_patch_stamps(unsigned long long* out, int n) {
  if (!vcg::g_patch_stamps) return 1;
  n = n < 64 * 6 ? n : 64 * 6;
  return hipMemcpy(out, vcg::g_patch_stamps, (size_t)n * 8, hipMemcpyDeviceToHost) == hipSuccess ? 0 : 2;
}
