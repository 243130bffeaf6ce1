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
// over every row the workgroup sees (two LDS buffers, one barrier per iteration).
//
// Precision: y3's variance is w^T (G / M - mu mu^T) w, which cancels like E[y^2] - E[y]^2 when a y3 channel's |mean|
// is much larger than its std. So the Gram is not formed from a but from a - c_b, with c_b the bf16-rounded column
// means of the workgroup's FIRST iteration of rows (a per-workgroup centre close to the batch mean): the fp32 MFMA
// accumulation then carries an error relative to the centred (variance-sized) entries, not to mean^2. a - c is exact
// in f32; it enters the MFMA rounded to bf16 stochastically (a counter hash of (row, channel): unbiased, so the Gram
// is exact up to zero-mean noise of ~2^-9 / sqrt(rows) relative). Each
// workgroup writes a [C * C + 2 C] f32 slab (centred G_b mirrored to full, centred colsum d_b = sum (a - c_b),
// centre c_b); gram_reduce rebuilds the uncentred colsum = sum_b (d_b + n_b c_b) and
// G = sum_b (G_b + d_b c_b^T + c_b d_b^T + n_b c_b c_b^T) in double in a fixed order (deterministic), and the
// statistics kernel subtracts mu mu^T in double.
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
template <int C, int W>
__device__ __forceinline__ void gram_body(const bf16_t* __restrict__ y, const float* __restrict__ scale,
                                          const float* __restrict__ shift, bf16_t* __restrict__ out,
                                          float* __restrict__ slab, long long P, bf16_t* buf, float* red) {
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
  float sc[8], sh[8], cs[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    sc[e] = scale[8 * cc + e];
    sh[e] = shift[8 * cc + e];
    cs[e] = 0.f;
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
  // the Gram centre c_b: bf16 column means of this workgroup's first iteration (every workgroup has one: grid <=
  // iters), summed in a fixed order through LDS
  float ctr[8];
  {
    float ps[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) ps[e] = 0.f;
#pragma unroll
    for (int u = 0; u < NV; ++u) {
      if (it * R + r0 + u * RS < P) {
        float a[8];
        unpack8g(nx[u], a);
#pragma unroll
        for (int e = 0; e < 8; ++e) ps[e] += bf2f(f2bf(fmaxf(fmaf(a[e], sc[e], sh[e]), 0.f)));
      }
    }
#pragma unroll
    for (int e = 0; e < 8; ++e) red[tid * 9 + e] = ps[e];
    __syncthreads();
    const long long left = P - it * R;
    const float inv = 1.f / (float)(left < R ? left : R);
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      float t = 0.f;
      for (int q = cc; q < 256; q += CPR) t += red[q * 9 + e];
      ctr[e] = bf2f(f2bf(t * inv));
    }
    __syncthreads();  // (red is written again only after the main loop)
  }
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
          st[e] -= ctr[e];  // (exact in f32: both bf16 values)
          cs[e] += st[e];   // the centred column sum (no cancellation against n c later)
        }
        // the centred values in bf16 with unbiased (stochastic) rounding: round-to-nearest of a - c is a fixed
        // function of a, whose errors correlate with a - c and bias the diagonal of the Gram by ~2^-15 relative
        const uint32_t hb = (uint32_t)row * 0x9E3779B1u + (uint32_t)cc * 0x85EBCA77u;
        uint32_t dw[4];
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          uint32_t h = hb + (uint32_t)q * 0xC2B2AE3Du;
          h ^= h >> 15;
          h *= 0x2C1B3C6Du;
          h ^= h >> 13;
          dw[q] = ((__float_as_uint(st[2 * q]) + (h & 0xFFFFu)) >> 16) |
                  ((__float_as_uint(st[2 * q + 1]) + (h >> 16)) & 0xFFFF0000u);
        }
        d = make_uint4(dw[0], dw[1], dw[2], dw[3]);
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
  // slab: the centred G (mirrored to the full matrix), centred colsum, centre
  float* sl = slab + (long long)blockIdx.x * (C * C + 2 * C);
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
  if (tid < CPR) {
#pragma unroll
    for (int e = 0; e < 8; ++e) sl[C * C + C + 8 * tid + e] = ctr[e];
  }
}

template <int C>
__global__ __launch_bounds__(256) void bn_apply_gram_kernel(const bf16_t* __restrict__ y, const float* __restrict__ scale,
                                                           const float* __restrict__ shift, bf16_t* __restrict__ out,
                                                           float* __restrict__ slab, long long P) {
  __shared__ __attribute__((aligned(1024))) bf16_t buf[2 * 16384];
  __shared__ float red[256 * 9];
  switch (__builtin_amdgcn_readfirstlane(threadIdx.x >> 6)) {
    case 0: gram_body<C, 0>(y, scale, shift, out, slab, P, buf, red); break;
    case 1: gram_body<C, 1>(y, scale, shift, out, slab, P, buf, red); break;
    case 2: gram_body<C, 2>(y, scale, shift, out, slab, P, buf, red); break;
    default: gram_body<C, 3>(y, scale, shift, out, slab, P, buf, red); break;
  }
}

// Rows of `slab` b: the iterations b, b + nb, ... of R rows each, the last one possibly short.
__device__ __forceinline__ double slab_rows(int b, int nb, long long P, int R) {
  const long long iters = (P + R - 1) / R;
  const long long nit = (iters - 1 - b) / nb + 1;
  long long n = nit * R;
  if ((iters - 1) % nb == b) n -= iters * R - P;
  return (double)n;
}

// out[i] = the uncentred sum over nb slabs, in double (deterministic): for a Gram entry (j, k)
// sum_b G_b[j][k] + d_b[j] c_b[k] + c_b[j] d_b[k] + n_b c_b[j] c_b[k], for a column sum sum_b d_b[k] + n_b c_b[k]
// (G_b, d_b: centred at c_b). A thread owns 4
// consecutive entries (16-B loads) and G threads split the slabs (thread t sums slabs t, t + G, ... in order, the G
// partials are combined in t order through LDS). (One thread per entry over all 256-512 slabs ran latency-bound:
// 100 us per call at C = 64.) Writes f32 gram / colsum and, when g64 != null, the double [C * C + C].
__global__ __launch_bounds__(256) void gram_reduce_kernel(const float* __restrict__ slab, int nb, int n, int G,
                                                         float* __restrict__ gram, float* __restrict__ colsum, int C,
                                                         double* __restrict__ g64, long long P, int R) {
  __shared__ double red[4][256];
  const int QB = 256 / G;
  const int t = threadIdx.x / QB, ql = threadIdx.x - t * QB;
  const int quad = blockIdx.x * QB + ql, nq = n >> 2;
  const int ns = C * C + 2 * C;  // slab stride (floats)
  double s0 = 0.0, s1 = 0.0, s2 = 0.0, s3 = 0.0;
  if (quad < nq) {
    const int i0 = 4 * quad;
    if (i0 < C * C) {
      const int j = i0 / C, k = i0 - j * C;
      for (int b = t; b < nb; b += G) {
        const float* sb = slab + (long long)b * ns;
        const float4 g = *reinterpret_cast<const float4*>(sb + i0);
        const float4 sk = *reinterpret_cast<const float4*>(sb + C * C + k);
        const float4 ck = *reinterpret_cast<const float4*>(sb + C * C + C + k);
        const double sj = (double)sb[C * C + j], cj = (double)sb[C * C + C + j];
        const double nr = slab_rows(b, nb, P, R);
        const double ncj = nr * cj;
        s0 += (double)g.x + sj * (double)ck.x + cj * (double)sk.x + ncj * (double)ck.x;
        s1 += (double)g.y + sj * (double)ck.y + cj * (double)sk.y + ncj * (double)ck.y;
        s2 += (double)g.z + sj * (double)ck.z + cj * (double)sk.z + ncj * (double)ck.z;
        s3 += (double)g.w + sj * (double)ck.w + cj * (double)sk.w + ncj * (double)ck.w;
      }
    } else {
      for (int b = t; b < nb; b += G) {
        const float* sb = slab + (long long)b * ns;
        const float4 v = *reinterpret_cast<const float4*>(sb + i0);
        const float4 c = *reinterpret_cast<const float4*>(sb + i0 + C);
        const double nr = slab_rows(b, nb, P, R);
        s0 += (double)v.x + nr * (double)c.x; s1 += (double)v.y + nr * (double)c.y;
        s2 += (double)v.z + nr * (double)c.z; s3 += (double)v.w + nr * (double)c.w;
      }
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
  const double sv[4] = {s0, s1, s2, s3};
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    const int i = 4 * quad + e;
    if (i < C * C) gram[i] = (float)sv[e];
    else colsum[i - C * C] = (float)sv[e];
    if (g64) g64[i] = sv[e];
  }
}

// bn3's batch statistics from the double (G, colsum) g64 [C * C + C] and conv3's bf16 weights w [N][C]: 8 output
// columns per workgroup, thread t < C owns row t of the covariance; double throughout. Writes the vcg_conv_fwd stats
// layout with one used slot: stats[n][0] = (mean, M2 = M var), count row slot 0 = (M, 1).
__global__ __launch_bounds__(256) void gram_stats_kernel(const double* __restrict__ g64, const bf16_t* __restrict__ w,
                                                        long long M, int N, int C, float2* __restrict__ stats,
                                                        int mtiles) {
  const double* __restrict__ gram = g64;
  const double* __restrict__ colsum = g64 + (long long)C * C;
  __shared__ double mu[1024];
  __shared__ double wq[8][1024];
  __shared__ double pm[8][256], pv[8][256];
  const int n0 = blockIdx.x * 8, tid = threadIdx.x;
  const double invM = 1.0 / (double)M;
  for (int k = tid; k < C; k += 256) mu[k] = colsum[k] * invM;
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
      const double cv = gr[k] * invM - mu[t] * mu[k];
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
  return (long long)gram_grid(P, C) * ((long long)C * C + 2 * C) * 4;
}

// out = bf16(relu(fma(y, scale, shift))) (vcg_bn_apply's values), colsum[c] = sum of out's column c (as
// vcg_bn_apply_colsum), gram[j][k] = sum_rows out[j] out[k] (f32 [C][C]); g64 (optional): the same Gram matrix and
// column sums in double, [C * C + C] (accumulated centred per workgroup, see the file comment: the input of
// vcg_bn_stats_from_gram). C = 64 / 128 / 256, bf16.
VCG_API int vcg_bn_apply_gram(const void* y, const float* scale, const float* shift, void* out, float* colsum,
                              float* gram, double* g64, float* ws, long long ws_bytes, long long P, int C,
                              hipStream_t s) {
  VCG_REQUIRE(y && scale && shift && out && colsum && gram && ws, "null argument");
  VCG_REQUIRE(C == 64 || C == 128 || C == 256, "C must be 64, 128 or 256");
  VCG_REQUIRE(P > 0, "no rows");
  VCG_REQUIRE((((uintptr_t)y | (uintptr_t)out) & 15) == 0, "16-B alignment");
  const int g = gram_grid(P, C);
  const long long n = (long long)C * C + C;
  VCG_REQUIRE(ws_bytes >= vcg_bn_apply_gram_ws_bytes(P, C), "workspace too small");
  if (C == 64)
    hipLaunchKernelGGL(bn_apply_gram_kernel<64>, dim3(g), dim3(256), 0, s, (const bf16_t*)y, scale, shift,
                       (bf16_t*)out, ws, P);
  else if (C == 128)
    hipLaunchKernelGGL(bn_apply_gram_kernel<128>, dim3(g), dim3(256), 0, s, (const bf16_t*)y, scale, shift,
                       (bf16_t*)out, ws, P);
  else
    hipLaunchKernelGGL(bn_apply_gram_kernel<256>, dim3(g), dim3(256), 0, s, (const bf16_t*)y, scale, shift,
                       (bf16_t*)out, ws, P);
  VCG_LAUNCH_CHECK();
  const int nq = (int)(n / 4);  // (n = C (C + 1), C a power of two >= 64: a multiple of 4)
  int G = 1;
  while (G < 64 && G * 2 <= g && (long long)nq * G < 65536) G *= 2;
  const int QB = 256 / G;
  hipLaunchKernelGGL(gram_reduce_kernel, dim3((unsigned)((nq + QB - 1) / QB)), dim3(256), 0, s, ws, g, (int)n, G, gram,
                     colsum, C, g64, P, 16384 / C);
  VCG_LAUNCH_CHECK();
  return VCG_OK;
}

// conv3's batch statistics from vcg_bn_apply_gram's double g64 (Gram matrix then column sums) of its input and its
// bf16 weights w [N][C] (the forward GEMM layout): stats in the vcg_conv_fwd layout ([N + 1][mtiles] float2, one
// used slot), for vcg_bn_finalize.
VCG_API int vcg_bn_stats_from_gram(const double* g64, const void* w, long long M, int N, int C, float* stats,
                                   int mtiles, hipStream_t s) {
  VCG_REQUIRE(g64 && w && stats, "null argument");
  VCG_REQUIRE(C > 0 && C <= 1024 && N > 0 && M > 0 && mtiles > 0, "bad shape");
  hipLaunchKernelGGL(gram_stats_kernel, dim3((N + 7) / 8), dim3(256), 0, s, g64, (const bf16_t*)w, M, N, C,
                     reinterpret_cast<float2*>(stats), mtiles);
  VCG_LAUNCH_CHECK();
  return VCG_OK;
}
