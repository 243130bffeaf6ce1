// BatchNorm + ReLU apply that also returns colsum(a) and the Gram matrix a^T a of its output (bf16 trunk, the
// bottleneck's bn2 -> relu -> a2, reference torchvision Bottleneck inside model/vision/resnet50_tsm.py:15), and the
// batch statistics of conv3's output computed from them.
//
// conv3 is linear: y3 = a2 w^T (w = the bf16 conv3 weights, [C3][planes]), so per output column n
//   mean_n = w_n . mu            (mu = colsum(a2) / M)
//   var_n  = w_n^T Cov w_n       (Cov = a2^T a2 / M - mu mu^T)
// -- bn3's batch statistics without reading a2 a second time (the statistics-only conv3 GEMM pass), of the exact
// y3 (no bf16 rounding of y3). The same a2^T a2 is the Gram term of the bn3 backward fold in the a2 form
// (trunk.py _fold_conv3), which then needs no a2^T a2 weight-gradient GEMM of its own.
//
// vcg_bn_apply_gram: per iteration a workgroup (4 waves) takes R = 16384 / C rows ([R][C] bf16 = 32 KiB of y):
// every thread owns one 16-B channel chunk (8 channels: its scale / shift / column sums stay in registers) of
// 8 rows, loads them one iteration ahead, applies fma(y, scale, shift) + ReLU, stores the bf16 a and its column
// sums exactly as vcg_bn_apply_colsum, and writes the tile to LDS as [64-row k-step][128- or 64-column panel]
// with the 16-B chunk swizzle of the weight-gradient engine (igemm_wgrad.hip wswz), from which ds_read_b64_tr_b16
// gives each lane 4 consecutive rows of one column. The C x C Gram block pairs (jb <= kb of 16 x 16, the upper
// triangle: G is symmetric) are dealt round-robin to the 4 waves and accumulated with v_mfma_f32_16x16x32_bf16
// over every row the workgroup sees (two LDS buffers, one barrier per iteration). Each workgroup writes a
// [C * C + C] f32 slab (G mirrored to full, then colsum); gram_reduce sums the slabs in a fixed order in double
// (deterministic).
//
// Precision. y3's variance is w^T (G / M - mu mu^T) w. The fp32 accumulation errors of G are independent per entry,
// so they are amplified only by the ratio |mean| / std of the a2 CHANNELS themselves (not of y3): ~1 for a ReLU of a
// unit normal, but large for a channel whose BN shift dominates its scale (beta >> |gamma|: the ReLU almost always
// passes and a2 ~ gamma z + beta). Such channels are centred: the Gram is accumulated over a - c with the per-channel
// centre c = bf16(beta) where beta > 6 |gamma| (else 0, the exact uncentred Gram, whose relative error there is at most
// ~40x the fp32 accumulation's). a - c is exact in bf16 whenever c / 2 <= a <= 2 c (Sterbenz): every row of a centred
// channel but those 3 std below its mean, so the products stay exact (the rare others carry one rounding). The slabs
// then hold the centred Gc and d = colsum(a - c); gram_reduce sums them in double into g64 = [Gc | d | c] and
// gram_finish writes the uncentred f32 G = Gc + d c^T + c d^T + M c c^T and colsum = d + M c; the statistics read
// g64 (Cov = Gc / M - (d / M)(d / M)^T, mu = c + d / M: no cancellation against the centre).
#include "common.h"

namespace vcg {
namespace {

typedef __attribute__((address_space(3))) char lds_char_t;
__device__ __forceinline__ uint32_t lds_off(const void* p) { return (uint32_t)(uintptr_t)(const lds_char_t*)p; }

// 16-B slot of logical chunk c in k-row `row` of a [64][COLS] bf16 panel (an involution in c; igemm_wgrad.hip wswz)
template <int COLS> __device__ __forceinline__ int gswz(int row, int c) {
  if constexpr (COLS == 128) return c ^ (2 * (row & 7));
  else return c ^ (2 * ((row >> 1) & 3));
}

// 16x16x32 fragment of columns r0..r0+15 of a [64][COLS] panel, k-substep s2 (rows 32 s2 .. + 31): element j of
// lane 16g+i is row 32 s2 + 4g + 16 (j >> 2) + (j & 3), the same map for both operands of the Gram MFMA
template <int COLS>
__device__ __forceinline__ s16x8 gfrag(const bf16_t* panel, int r0, int lane, int s2) {
  const int g = lane >> 4, i = lane & 15;
  const int q = i >> 2, pp = i & 3;
  const int cl = r0 + 4 * pp;
  const int k0 = 32 * s2 + 4 * g + q, k1 = k0 + 16;
  const uint32_t a0 = lds_off(panel + k0 * COLS + 8 * gswz<COLS>(k0, cl >> 3) + (cl & 7));
  const uint32_t a1 = lds_off(panel + k1 * COLS + 8 * gswz<COLS>(k1, cl >> 3) + (cl & 7));
  s16x4 lo, hi;
  asm volatile("ds_read_b64_tr_b16 %0, %1" : "=v"(lo) : "v"(a0) : "memory");
  asm volatile("ds_read_b64_tr_b16 %0, %1" : "=v"(hi) : "v"(a1) : "memory");
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  return s16x8{lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
}

__device__ __forceinline__ void unpack8g(const uint4& u, float (&v)[8]) {
  const uint32_t w[4] = {u.x, u.y, u.z, u.w};
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    v[2 * i] = __uint_as_float(w[i] << 16);
    v[2 * i + 1] = __uint_as_float(w[i] & 0xffff0000u);
  }
}

// Gram block pair p (jb <= kb of 16 x 16, row-major over the upper triangle) -> jb, kb
__host__ __device__ constexpr int pair_jb(int p, int nb) {
  int jb = 0;
  while (jb < nb && p >= nb - jb) {
    p -= nb - jb;
    ++jb;
  }
  return jb;
}
__host__ __device__ constexpr int pair_kb(int p, int nb) {
  int jb = 0;
  while (jb < nb && p >= nb - jb) {
    p -= nb - jb;
    ++jb;
  }
  return jb + p;
}

// one wave's part: the pairs p = 4 t + W (compile-time indices, so the accumulators and the fragment addresses
// are static); every wave runs the same loop and barriers
// the Gram centre of channel k (see the file comment): bf16(beta) where beta > 6 |gamma|, else 0; gamma = scale /
// invstd and beta = shift + scale mean recover the BN affine from the folded apply parameters
__device__ __forceinline__ float gram_centre(float sc, float sh, float mean, float invstd) {
  const float gamma = sc / invstd, beta = fmaf(sc, mean, sh);
  return beta > 6.f * fabsf(gamma) ? bf2f(f2bf(beta)) : 0.f;
}

template <int C, int W>
__device__ __forceinline__ void gram_body(const bf16_t* __restrict__ y, const float* __restrict__ scale,
                                          const float* __restrict__ shift, const float* __restrict__ mean,
                                          const float* __restrict__ invstd, bf16_t* __restrict__ out,
                                          float* __restrict__ slab, double* __restrict__ g64, long long P, bf16_t* buf,
                                          float* red) {
  constexpr int COLS = C >= 128 ? 128 : 64;
  constexpr int NP = C / COLS;   // panels per 64-row k-step
  constexpr int KS = 256 / C;    // 64-row k-steps per iteration
  constexpr int R = 64 * KS;     // rows per iteration
  constexpr int CPR = C / 8;     // 16-B chunks per row
  constexpr int NV = 8;          // chunks per thread per iteration (R * CPR / 256)
  constexpr int RS = 256 / CPR;  // row stride between a thread's chunks
  constexpr int NB = C / 16;
  constexpr int NPAIR = NB * (NB + 1) / 2;
  constexpr int NF = (NPAIR - W + 3) / 4;  // this wave's pairs
  constexpr int BUFE = R * C;  // bf16 elements per buffer (32 KiB)
  static_assert(R * CPR == NV * 256, "iteration geometry");

  const int tid = threadIdx.x, lane = tid & 63;
  const int cc = tid % CPR, r0 = tid / CPR;  // this thread's chunk and first row of an iteration
  float sc[8], sh[8], cs[8], ctr[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    sc[e] = scale[8 * cc + e];
    sh[e] = shift[8 * cc + e];
    ctr[e] = gram_centre(sc[e], sh[e], mean[8 * cc + e], invstd[8 * cc + e]);
    cs[e] = 0.f;
  }
  if (blockIdx.x == 0 && W == 0 && tid < CPR) {  // (wave 0 holds every chunk once: CPR <= 32 threads)
#pragma unroll
    for (int e = 0; e < 8; ++e) g64[C * C + C + 8 * cc + e] = (double)ctr[e];
  }
  f32x4 acc[NF > 0 ? NF : 1];
#pragma unroll
  for (int t = 0; t < NF; ++t) acc[t] = f32x4{0.f, 0.f, 0.f, 0.f};

  const long long iters = (P + R - 1) / R;
  long long it = blockIdx.x;
  uint4 nx[NV];
  auto load = [&](long long i) {
#pragma unroll
    for (int u = 0; u < NV; ++u) {
      const long long row = i * R + r0 + u * RS;
      nx[u] = row < P ? *reinterpret_cast<const uint4*>(y + row * C + 8 * cc) : make_uint4(0u, 0u, 0u, 0u);
    }
  };
  if (it < iters) load(it);
  int cur = 0;
  for (; it < iters; it += gridDim.x) {
    uint4 v[NV];
#pragma unroll
    for (int u = 0; u < NV; ++u) v[u] = nx[u];
    if (it + gridDim.x < iters) load(it + gridDim.x);  // next iteration's rows in flight under this one
    bf16_t* B = buf + cur * BUFE;
#pragma unroll
    for (int u = 0; u < NV; ++u) {
      const int lr = r0 + u * RS;  // row within the iteration
      const long long row = it * R + lr;
      float a[8];
      unpack8g(v[u], a);
      uint4 o = make_uint4(0u, 0u, 0u, 0u), d = make_uint4(0u, 0u, 0u, 0u);
      if (row < P) {
#pragma unroll
        for (int e = 0; e < 8; ++e) a[e] = fmaxf(fmaf(a[e], sc[e], sh[e]), 0.f);
        o.x = (uint32_t)f2bf(a[0]) | ((uint32_t)f2bf(a[1]) << 16);
        o.y = (uint32_t)f2bf(a[2]) | ((uint32_t)f2bf(a[3]) << 16);
        o.z = (uint32_t)f2bf(a[4]) | ((uint32_t)f2bf(a[5]) << 16);
        o.w = (uint32_t)f2bf(a[6]) | ((uint32_t)f2bf(a[7]) << 16);
        *reinterpret_cast<uint4*>(out + row * C + 8 * cc) = o;
        float st[8];
        unpack8g(o, st);  // the stored (rounded) values
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          st[e] -= ctr[e];  // (exact in f32; exact in bf16 for a 0 centre and, by Sterbenz, for c / 2 <= a <= 2 c)
          cs[e] += st[e];
        }
        d.x = (uint32_t)f2bf(st[0]) | ((uint32_t)f2bf(st[1]) << 16);
        d.y = (uint32_t)f2bf(st[2]) | ((uint32_t)f2bf(st[3]) << 16);
        d.z = (uint32_t)f2bf(st[4]) | ((uint32_t)f2bf(st[5]) << 16);
        d.w = (uint32_t)f2bf(st[6]) | ((uint32_t)f2bf(st[7]) << 16);
      }
      // LDS: k-step lr / 64, k-row lr % 64, panel cc / (COLS / 8), swizzled slot of chunk cc % (COLS / 8)
      const int ks = lr >> 6, kr = lr & 63, pn = cc / (COLS / 8), pc = cc % (COLS / 8);
      bf16_t* dst = B + (ks * NP + pn) * 64 * COLS + kr * COLS + 8 * gswz<COLS>(kr, pc);
      *reinterpret_cast<uint4*>(dst) = d;  // the centred row (rows past P: zeros, no contribution)
    }
    __syncthreads();  // the tile is in LDS; every wave's reads of the other buffer (two iterations ago) are done
#pragma unroll
    for (int t = 0; t < NF; ++t) {
      const int p = 4 * t + W;
      const int cj = pair_jb(p, NB) * 16, ck = pair_kb(p, NB) * 16;
#pragma unroll
      for (int ks = 0; ks < KS; ++ks) {
        const bf16_t* pj = B + (ks * NP + cj / COLS) * 64 * COLS;
        const bf16_t* pk = B + (ks * NP + ck / COLS) * 64 * COLS;
#pragma unroll
        for (int s2 = 0; s2 < 2; ++s2) {
          const s16x8 fj = gfrag<COLS>(pj, cj % COLS, lane, s2);
          const s16x8 fk = gfrag<COLS>(pk, ck % COLS, lane, s2);
          acc[t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fk, fj, acc[t], 0, 0, 0);  // G[cj + ci][ck + 4g + r]
        }
      }
    }
    cur ^= 1;
  }
  // slab: the centred G (mirrored to the full matrix) then the centred colsum d
  float* sl = slab + (long long)blockIdx.x * (C * C + C);
  const int g = lane >> 4, ci = lane & 15;
#pragma unroll
  for (int t = 0; t < NF; ++t) {
    const int p = 4 * t + W;
    const int jb = pair_jb(p, NB), kb = pair_kb(p, NB);
    const int j = jb * 16 + ci, k = kb * 16 + 4 * g;
    *reinterpret_cast<f32x4*>(sl + j * C + k) = acc[t];
    if (jb != kb) {
#pragma unroll
      for (int r = 0; r < 4; ++r) sl[(k + r) * C + j] = acc[t][r];
    }
  }
#pragma unroll
  for (int e = 0; e < 8; ++e) red[tid * 9 + e] = cs[e];
  __syncthreads();
  for (int o = tid; o < C; o += 256) {
    const int ch = o / 8, e = o % 8;
    float s = 0.f;
    for (int t = ch; t < 256; t += CPR) s += red[t * 9 + e];  // fixed order
    sl[C * C + o] = s;
  }
}

template <int C>
__global__ __launch_bounds__(256) void bn_apply_gram_kernel(const bf16_t* __restrict__ y, const float* __restrict__ scale,
                                                           const float* __restrict__ shift,
                                                           const float* __restrict__ mean,
                                                           const float* __restrict__ invstd, bf16_t* __restrict__ out,
                                                           float* __restrict__ slab, double* __restrict__ g64,
                                                           long long P) {
  __shared__ __attribute__((aligned(1024))) bf16_t buf[2 * 16384];
  __shared__ float red[256 * 9];
  switch (__builtin_amdgcn_readfirstlane(threadIdx.x >> 6)) {
    case 0: gram_body<C, 0>(y, scale, shift, mean, invstd, out, slab, g64, P, buf, red); break;
    case 1: gram_body<C, 1>(y, scale, shift, mean, invstd, out, slab, g64, P, buf, red); break;
    case 2: gram_body<C, 2>(y, scale, shift, mean, invstd, out, slab, g64, P, buf, red); break;
    default: gram_body<C, 3>(y, scale, shift, mean, invstd, out, slab, g64, P, buf, red); break;
  }
}

// out[i] = sum over nb slabs of slab[b][i], in double (deterministic): a thread owns 4 consecutive entries (16-B
// loads) and G threads split the slabs (thread t sums slabs t, t + G, ... in order, the G partials are combined in
// t order through LDS). (One thread per entry over all 256-512 slabs ran latency-bound: 100 us per call at C = 64.)
__global__ __launch_bounds__(256) void gram_reduce_kernel(const float* __restrict__ slab, int nb, int n, int G,
                                                         double* __restrict__ g64) {
  __shared__ double red[4][256];
  const int QB = 256 / G;
  const int t = threadIdx.x / QB, ql = threadIdx.x - t * QB;
  const int quad = blockIdx.x * QB + ql, nq = n >> 2;
  double s0 = 0.0, s1 = 0.0, s2 = 0.0, s3 = 0.0;
  if (quad < nq) {
    const float4* p = reinterpret_cast<const float4*>(slab) + quad;
    int b = t;
    for (; b + 3 * G < nb; b += 4 * G) {
      float4 v[4];
#pragma unroll
      for (int k = 0; k < 4; ++k) v[k] = p[(long long)(b + k * G) * nq];
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        s0 += (double)v[k].x; s1 += (double)v[k].y; s2 += (double)v[k].z; s3 += (double)v[k].w;
      }
    }
    for (; b < nb; b += G) {
      const float4 v = p[(long long)b * nq];
      s0 += (double)v.x; s1 += (double)v.y; s2 += (double)v.z; s3 += (double)v.w;
    }
  }
  if (G > 1) {
    red[0][threadIdx.x] = s0; red[1][threadIdx.x] = s1; red[2][threadIdx.x] = s2; red[3][threadIdx.x] = s3;
    __syncthreads();
    if (t != 0) return;
    for (int u = 1; u < G; ++u) {
      const int o = u * QB + ql;
      s0 += red[0][o]; s1 += red[1][o]; s2 += red[2][o]; s3 += red[3][o];
    }
  }
  if (quad >= nq) return;
  double* o = g64 + 4 * quad;
  o[0] = s0; o[1] = s1; o[2] = s2; o[3] = s3;
}

// the uncentred f32 Gram matrix and column sums from g64 = [Gc | d | c] (M rows): G = Gc + d c^T + c d^T + M c c^T,
// colsum = d + M c, in double
__global__ __launch_bounds__(256) void gram_finish_kernel(const double* __restrict__ g64, long long M, int C,
                                                         float* __restrict__ gram, float* __restrict__ colsum) {
  const int i = blockIdx.x * 256 + threadIdx.x;
  const double* d = g64 + (long long)C * C;
  const double* c = d + C;
  const double m = (double)M;
  if (i < C * C) {
    const int j = i / C, k = i - j * C;
    gram[i] = (float)(g64[i] + d[j] * c[k] + c[j] * d[k] + m * c[j] * c[k]);
  } else if (i < C * C + C) {
    const int k = i - C * C;
    colsum[k] = (float)(d[k] + m * c[k]);
  }
}

// bn3's batch statistics from g64 = [Gc | d | c] (the centred Gram matrix and column sums of conv3's input, and the
// centre: bn_gram's file comment) and conv3's bf16 weights w [N][C]: Cov = Gc / M - (d / M)(d / M)^T and
// mu = c + d / M; 8 output columns per workgroup, thread t < C owns row t of the covariance; double throughout.
// Writes the vcg_conv_fwd stats layout with one used slot: stats[n][0] = (mean, M2 = M var), count row slot 0 =
// (M, 1).
__global__ __launch_bounds__(256) void gram_stats_kernel(const double* __restrict__ g64, const bf16_t* __restrict__ w,
                                                        long long M, int N, int C, float2* __restrict__ stats,
                                                        int mtiles) {
  const double* __restrict__ gram = g64;
  const double* __restrict__ dsum = g64 + (long long)C * C;
  const double* __restrict__ ctr = dsum + C;
  __shared__ double dm[1024];
  __shared__ double mu[1024];
  __shared__ double wq[8][1024];
  __shared__ double pm[8][256], pv[8][256];
  const int n0 = blockIdx.x * 8, tid = threadIdx.x;
  const double invM = 1.0 / (double)M;
  for (int k = tid; k < C; k += 256) {
    dm[k] = dsum[k] * invM;
    mu[k] = ctr[k] + dm[k];
  }
  for (int i = tid; i < 8 * C; i += 256) {
    const int q = i / C, k = i - q * C;
    wq[q][k] = n0 + q < N ? (double)bf2f(w[(long long)(n0 + q) * C + k]) : 0.0;
  }
  __syncthreads();
  double m[8], v[8];
#pragma unroll
  for (int q = 0; q < 8; ++q) m[q] = v[q] = 0.0;
  for (int t = tid; t < C; t += 256) {
    double u[8];
#pragma unroll
    for (int q = 0; q < 8; ++q) u[q] = 0.0;
    const double* gr = gram + (long long)t * C;
    for (int k = 0; k < C; ++k) {
      const double cv = gr[k] * invM - dm[t] * dm[k];
#pragma unroll
      for (int q = 0; q < 8; ++q) u[q] = fma(cv, wq[q][k], u[q]);
    }
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      v[q] = fma(wq[q][t], u[q], v[q]);
      m[q] = fma(wq[q][t], mu[t], m[q]);
    }
  }
#pragma unroll
  for (int q = 0; q < 8; ++q) {
    pm[q][tid] = m[q];
    pv[q][tid] = v[q];
  }
  __syncthreads();
  if (tid < 8 && n0 + tid < N) {
    double sm = 0.0, sv = 0.0;
    for (int t = 0; t < 256; ++t) {
      sm += pm[tid][t];
      sv += pv[tid][t];
    }
    stats[(long long)(n0 + tid) * mtiles] = make_float2((float)sm, (float)(fmax(sv, 0.0) * (double)M));
  }
  if (blockIdx.x == 0 && tid == 0) {
    float2* cnt = stats + (long long)N * mtiles;
    cnt[0] = make_float2((float)M, 1.f);  // one used slot (bn_finalize reads cnt[0].y slots)
  }
}

// The same statistics for C <= 256 with the covariance walked by rows: thread k owns column k (the Gram loads of a row
// are coalesced; the old form read one strided row per thread), 16 output columns per workgroup share each load,
// and the per-column sums over k are combined by a fixed-order tree (deterministic).
constexpr int GS_Q = 16;
// With fin (vcg_bn_finalize_from_gram): also bn_finalize's outputs for the one-slot statistics (the same float
// rounding of (mean, M2) and the same double arithmetic, so the values equal the separate finalize's) and the bn3 GEMM
// pass's folded weights bf16(w32 row n x scale n) (vcg_weight_fold's values) -- two launches fewer on the forward's
// critical path.
struct GramFin {
  const float *gamma, *beta;
  float *mean, *invstd, *scale, *shift, *rmean, *rvar;
  float momentum, eps;
  const float* w32;  // master conv weight [N][C] f32 (nullptr: no fold)
  bf16_t* wfold;     // [N][C]
};

__global__ __launch_bounds__(256) void gram_stats_rows_kernel(const double* __restrict__ g64, const bf16_t* __restrict__ w,
                                                             long long M, int N, int C, float2* __restrict__ stats,
                                                             int mtiles, GramFin fin, int has_fin) {
  const double* __restrict__ gram = g64;
  const double* __restrict__ dsum = g64 + (long long)C * C;
  const double* __restrict__ ctr = dsum + C;
  __shared__ double dm[256], mu[256];
  __shared__ double wq[GS_Q][256];
  __shared__ double red[2][GS_Q][256];
  const int n0 = blockIdx.x * GS_Q, k = threadIdx.x;
  const double invM = 1.0 / (double)M;
  if (k < C) {
    dm[k] = dsum[k] * invM;
    mu[k] = ctr[k] + dm[k];
  }
  for (int i = k; i < GS_Q * C; i += 256) {
    const int q = i / C, kk = i - q * C;
    wq[q][kk] = n0 + q < N ? (double)bf2f(w[(long long)(n0 + q) * C + kk]) : 0.0;
  }
  __syncthreads();
  double acc[GS_Q];
#pragma unroll
  for (int q = 0; q < GS_Q; ++q) acc[q] = 0.0;
  if (k < C) {
    const double dk = dm[k];
    for (int t0 = 0; t0 < C; t0 += 16) {  // (C % 16 == 0: 16 row loads in flight per batch)
      double gv[16];
#pragma unroll
      for (int u = 0; u < 16; ++u) gv[u] = gram[(long long)(t0 + u) * C + k];
#pragma unroll
      for (int u = 0; u < 16; ++u) {
        const double cv = gv[u] * invM - dm[t0 + u] * dk;
#pragma unroll
        for (int q = 0; q < GS_Q; ++q) acc[q] = fma(wq[q][t0 + u], cv, acc[q]);
      }
    }
  }
#pragma unroll
  for (int q = 0; q < GS_Q; ++q) {
    red[0][q][k] = k < C ? wq[q][k] * mu[k] : 0.0;
    red[1][q][k] = k < C ? wq[q][k] * acc[q] : 0.0;
  }
  __syncthreads();
  for (int h = 128; h > 0; h >>= 1) {  // fixed-order tree over the 256 columns
    if (k < h) {
#pragma unroll
      for (int q = 0; q < GS_Q; ++q) {
        red[0][q][k] += red[0][q][k + h];
        red[1][q][k] += red[1][q][k + h];
      }
    }
    __syncthreads();
  }
  __shared__ float fscale[GS_Q];
  if (k < GS_Q && n0 + k < N) {
    const float mf = (float)red[0][k][0], m2f = (float)(fmax(red[1][k][0], 0.0) * (double)M);
    if (stats) stats[(long long)(n0 + k) * mtiles] = make_float2(mf, m2f);
    if (has_fin) {  // bn_finalize_kernel's arithmetic for one slot of (float) M rows
      const int c = n0 + k;
      const double Nn = (double)(float)M, mu = (double)mf;
      const double var = (double)m2f / Nn;
      const float invstd = (float)(1.0 / sqrt(var + (double)fin.eps));
      const float g = fin.gamma ? fin.gamma[c] : 1.f, b = fin.beta ? fin.beta[c] : 0.f;
      if (fin.mean) fin.mean[c] = (float)mu;
      if (fin.invstd) fin.invstd[c] = invstd;
      fin.scale[c] = g * invstd;
      fin.shift[c] = b - (float)mu * g * invstd;
      fscale[k] = g * invstd;
      if (fin.rmean) {
        const double unbiased = Nn > 1 ? (double)m2f / (Nn - 1) : var;
        fin.rmean[c] = (float)((1.0 - fin.momentum) * fin.rmean[c] + fin.momentum * mu);
        fin.rvar[c] = (float)((1.0 - fin.momentum) * fin.rvar[c] + fin.momentum * unbiased);
      }
    }
  }
  if (stats && blockIdx.x == 0 && k == 0) {
    float2* cnt = stats + (long long)N * mtiles;
    cnt[0] = make_float2((float)M, 1.f);  // one used slot (bn_finalize reads cnt[0].y slots)
  }
  if (has_fin && fin.w32) {  // the folded rows of this workgroup's columns
    __syncthreads();
    const int rows = min(GS_Q, N - n0);
    for (int i = k; i < rows * C; i += 256) {
      const int q = i / C;
      const long long o = (long long)(n0 + q) * C + (i - q * C);
      fin.wfold[o] = f2bf(fin.w32[o] * fscale[q]);
    }
  }
}

int gram_grid(long long P, int C) {
  const long long iters = (P + 16384 / C - 1) / (16384 / C);
  const long long cap = C >= 256 ? 256 : 512;
  return (int)(iters < cap ? iters : cap);
}

}  // namespace
}  // namespace vcg

using namespace vcg;

VCG_API long long vcg_bn_apply_gram_ws_bytes(long long P, int C) {
  if (C != 64 && C != 128 && C != 256) return 0;
  return (long long)gram_grid(P, C) * ((long long)C * C + C) * 4;
}

// out = bf16(relu(fma(y, scale, shift))) (vcg_bn_apply's values), colsum[c] = sum of out's column c (as
// vcg_bn_apply_colsum, up to the summation order), gram[j][k] = sum_rows out[j] out[k] (f32 [C][C]); g64 (double
// [C * C + 2 C]) = [Gc | d | c], the Gram matrix and column sums centred at c (the file comment), which
// vcg_bn_stats_from_gram reads. mean / invstd: the BatchNorm statistics that scale / shift fold (for the centre).
// C = 64 / 128 / 256, bf16.
VCG_API int vcg_bn_apply_gram(const void* y, const float* scale, const float* shift, const float* mean,
                              const float* invstd, void* out, float* colsum, float* gram, double* g64, float* ws,
                              long long ws_bytes, long long P, int C, hipStream_t s) {
  VCG_REQUIRE(y && scale && shift && mean && invstd && out && colsum && gram && g64 && ws, "null argument");
  VCG_REQUIRE(C == 64 || C == 128 || C == 256, "C must be 64, 128 or 256");
  VCG_REQUIRE(P > 0, "no rows");
  VCG_REQUIRE((((uintptr_t)y | (uintptr_t)out) & 15) == 0, "16-B alignment");
  const int g = gram_grid(P, C);
  const long long n = (long long)C * C + C;
  VCG_REQUIRE(ws_bytes >= (long long)g * n * 4, "workspace too small");
  if (census_on()) { char t_[96]; snprintf(t_, sizeof(t_), "bn_apply_gram"); census_add(t_, P, C, C); }
#define VCG_GRAM(CC)                                                                                            \
  hipLaunchKernelGGL(bn_apply_gram_kernel<CC>, dim3(g), dim3(256), 0, s, (const bf16_t*)y, scale, shift, mean, \
                     invstd, (bf16_t*)out, ws, g64, P)
  if (C == 64) VCG_GRAM(64);
  else if (C == 128) VCG_GRAM(128);
  else VCG_GRAM(256);
#undef VCG_GRAM
  VCG_LAUNCH_CHECK();
  const int nq = (int)(n / 4);  // (n = C (C + 1), C a power of two >= 64: a multiple of 4)
  int G = 1;
  while (G < 64 && G * 2 <= g && (long long)nq * G < 65536) G *= 2;
  const int QB = 256 / G;
  hipLaunchKernelGGL(gram_reduce_kernel, dim3((unsigned)((nq + QB - 1) / QB)), dim3(256), 0, s, ws, g, (int)n, G, g64);
  VCG_LAUNCH_CHECK();
  hipLaunchKernelGGL(gram_finish_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, g64, P, C, gram, colsum);
  VCG_LAUNCH_CHECK();
  return VCG_OK;
}

// conv3's batch statistics from vcg_bn_apply_gram's g64 (its input's centred Gram matrix, column sums and centre) and
// its bf16 weights w [N][C] (the forward GEMM layout): stats in the vcg_conv_fwd layout ([N + 1][mtiles] float2, one
// used slot), for vcg_bn_finalize.
VCG_API int vcg_bn_stats_from_gram(const double* g64, const void* w, long long M, int N, int C, float* stats,
                                   int mtiles, hipStream_t s) {
  VCG_REQUIRE(g64 && w && stats, "null argument");
  VCG_REQUIRE(C > 0 && C <= 1024 && N > 0 && M > 0 && mtiles > 0, "bad shape");
  if (C <= 256 && C % 16 == 0)
    hipLaunchKernelGGL(gram_stats_rows_kernel, dim3((N + GS_Q - 1) / GS_Q), dim3(256), 0, s, g64, (const bf16_t*)w, M,
                       N, C, reinterpret_cast<float2*>(stats), mtiles, GramFin{}, 0);
  else
    hipLaunchKernelGGL(gram_stats_kernel, dim3((N + 7) / 8), dim3(256), 0, s, g64, (const bf16_t*)w, M, N, C,
                       reinterpret_cast<float2*>(stats), mtiles);
  VCG_LAUNCH_CHECK();
  return VCG_OK;
}

// vcg_bn_stats_from_gram + vcg_bn_finalize (one slot of M rows; running statistics updated when rmean / rvar are
// given) + vcg_weight_fold of the conv's f32 master weight w32 [N][C] by the new scale into wfold (bf16; both
// optional) in one launch: the same values as the three calls. C <= 256, C % 16 == 0.
VCG_API int vcg_bn_finalize_from_gram(const double* g64, const void* w, long long M, int N, int C, const float* gamma,
                                      const float* beta, float* mean, float* invstd, float* scale, float* shift,
                                      float* running_mean, float* running_var, float momentum, float eps,
                                      const float* w32, void* wfold, hipStream_t s) {
  VCG_REQUIRE(g64 && w && scale && shift, "null argument");
  VCG_REQUIRE(C > 0 && C <= 256 && C % 16 == 0 && N > 0 && M > 0, "C must be a multiple of 16, <= 256");
  VCG_REQUIRE(!running_mean == !running_var, "running_mean and running_var together");
  VCG_REQUIRE(!w32 == !wfold, "w32 and wfold together");
  GramFin f{gamma, beta, mean, invstd, scale, shift, running_mean, running_var, momentum, eps, w32,
            (bf16_t*)wfold};
  hipLaunchKernelGGL(gram_stats_rows_kernel, dim3((N + GS_Q - 1) / GS_Q), dim3(256), 0, s, g64, (const bf16_t*)w, M,
                     N, C, (float2*)nullptr, 1, f, 1);
  VCG_LAUNCH_CHECK();
  return VCG_OK;
}
