// BERT-base encoder support kernels (HF BertModel semantics as used by the reference
// model/lang/bert_hugface.py:20 and TwoStream.forward two_stream.py:172-179):
//   embeddings: word[id] + position[l] + token_type[0] -> LayerNorm(eps 1e-12) -> dropout
//   self-output / output: LayerNorm(dropout(dense(x)) + residual)
//   attention: softmax(QK^T/sqrt(d) + mask_add) -> dropout -> PV  (the two GEMMs run on the
//   MFMA engine in igemm.hip; the masked softmax and its backward live here)
// Dropout uses a counter-based hash (mix64) so the backward regenerates the mask.
#include "common.h"

using namespace vcg;

namespace {

__device__ __forceinline__ bool keep(uint64_t seed, uint64_t idx, float p) { return dropout_keep(seed, idx, p); }

// value as stored in T (bias-gradient sums use the gradient the GEMM will read)
template <typename T> __device__ __forceinline__ float bf_round(float v) { return to_f<T>(from_f<T>(v)); }

inline int grid_for(long long n, int bs = 256) {
  long long g = (n + bs - 1) / bs;
  if (g > 8192) g = 8192;
  if (g < 1) g = 1;
  return (int)g;
}

constexpr int LN_MAXE = 8;  // elements per thread (H <= 256*8)

// ---------------------------------------------------------------- embeddings + LN
template <typename T>
__global__ void embed_ln_fwd_kernel(const long long* __restrict__ ids, const float* __restrict__ word,
                                    const float* __restrict__ pos, const float* __restrict__ type,
                                    const float* __restrict__ gamma, const float* __restrict__ beta,
                                    T* __restrict__ out, float* __restrict__ mean_out, float* __restrict__ rstd_out,
                                    int L, int H, float eps, float p, uint64_t seed) {
  const int row = blockIdx.x;  // b*L + l
  const int l = row % L;
  const long long id = ids[row];
  __shared__ float red[16];
  float v[LN_MAXE];
  float s = 0.f;
#pragma unroll
  for (int e = 0; e < LN_MAXE; ++e) {
    const int c = threadIdx.x + e * blockDim.x;
    v[e] = 0.f;
    if (c < H) {
      v[e] = word[id * H + c] + pos[(long long)l * H + c] + type[c];
      s += v[e];
    }
  }
  const float mean = block_sum(s, red) / H;
  float s2 = 0.f;
#pragma unroll
  for (int e = 0; e < LN_MAXE; ++e) {
    const int c = threadIdx.x + e * blockDim.x;
    if (c < H) { const float d = v[e] - mean; s2 += d * d; }
  }
  const float var = block_sum(s2, red) / H;
  const float rstd = rsqrtf(var + eps);
#pragma unroll
  for (int e = 0; e < LN_MAXE; ++e) {
    const int c = threadIdx.x + e * blockDim.x;
    if (c < H) {
      float o = (v[e] - mean) * rstd * gamma[c] + beta[c];
      const long long idx = (long long)row * H + c;
      o = keep(seed, idx, p) ? o / (1.f - p) : 0.f;
      out[idx] = from_f<T>(o);
    }
  }
  if (threadIdx.x == 0) { mean_out[row] = mean; rstd_out[row] = rstd; }
}

// backward of embeddings: writes d(e) (fp32) rows; dgamma/dbeta partials per block
template <typename T>
__global__ void embed_ln_bwd_kernel(const T* __restrict__ dout, const long long* __restrict__ ids,
                                    const float* __restrict__ word, const float* __restrict__ pos,
                                    const float* __restrict__ type, const float* __restrict__ gamma,
                                    const float* __restrict__ mean_in, const float* __restrict__ rstd_in,
                                    float* __restrict__ de, float* __restrict__ part, int L, int H, int rows_per_block,
                                    int rows, float p, uint64_t seed) {
  __shared__ float red[16];
  float pg[LN_MAXE], pb[LN_MAXE];
#pragma unroll
  for (int e = 0; e < LN_MAXE; ++e) { pg[e] = 0.f; pb[e] = 0.f; }
  const int r0 = blockIdx.x * rows_per_block, r1 = min(rows, r0 + rows_per_block);
  for (int row = r0; row < r1; ++row) {
    const int l = row % L;
    const long long id = ids[row];
    const float mean = mean_in[row], rstd = rstd_in[row];
    float xh[LN_MAXE], dxh[LN_MAXE];
    float a = 0.f, b = 0.f;
#pragma unroll
    for (int e = 0; e < LN_MAXE; ++e) {
      const int c = threadIdx.x + e * blockDim.x;
      xh[e] = 0.f; dxh[e] = 0.f;
      if (c < H) {
        const long long idx = (long long)row * H + c;
        const float v = word[id * H + c] + pos[(long long)l * H + c] + type[c];
        xh[e] = (v - mean) * rstd;
        float d = to_f<T>(dout[idx]);
        d = keep(seed, idx, p) ? d / (1.f - p) : 0.f;
        pg[e] += d * xh[e];
        pb[e] += d;
        dxh[e] = d * gamma[c];
        a += dxh[e];
        b += dxh[e] * xh[e];
      }
    }
    a = block_sum(a, red) / H;
    b = block_sum(b, red) / H;
#pragma unroll
    for (int e = 0; e < LN_MAXE; ++e) {
      const int c = threadIdx.x + e * blockDim.x;
      if (c < H) de[(long long)row * H + c] = rstd * (dxh[e] - a - xh[e] * b);
    }
  }
#pragma unroll
  for (int e = 0; e < LN_MAXE; ++e) {
    const int c = threadIdx.x + e * blockDim.x;
    if (c < H) {
      part[(long long)blockIdx.x * 2 * H + c] = pg[e];
      part[(long long)blockIdx.x * 2 * H + H + c] = pb[e];
    }
  }
}

// word grad, deterministic (no atomics): the workgroup of the FIRST token row carrying an id sums the de rows of
// every token with that id in ascending row order and adds the total to word_grad[id] (the only writer of that row);
// workgroups of later occurrences return. Rows are scanned in 256-id chunks: one ballot mask per wave in LDS, the
// matches of a chunk are then walked in row order. Same result on every run, whatever the schedule.
// Then: position grad (sum over batch), token-type grad (sum over all).
constexpr int SCAT_MAXE = 4;  // H <= 4 * 256
__global__ __launch_bounds__(256) void embed_scatter_kernel(const float* __restrict__ de,
                                                            const long long* __restrict__ ids,
                                                            float* __restrict__ word_grad, int H, long long rows,
                                                            long long pad_idx) {
  const long long row = blockIdx.x;
  const long long id = ids[row];
  if (id == pad_idx) return;  // nn.Embedding(padding_idx): the padding row never receives gradient
  __shared__ unsigned long long masks[4];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  float acc[SCAT_MAXE];
#pragma unroll
  for (int e = 0; e < SCAT_MAXE; ++e) acc[e] = 0.f;
  for (long long base = 0; base < rows; base += 256) {
    const long long j = base + tid;
    const bool hit = j < rows && ids[j] == id;
    const unsigned long long m = __ballot(hit);
    if (lane == 0) masks[wave] = m;
    __syncthreads();
    // an earlier row with this id exists: that row's workgroup owns the sum (block-uniform decision)
    bool earlier = false;
    if (base < row) {
      const long long lim = row - base;  // rows base .. row-1 of this chunk
#pragma unroll
      for (int w = 0; w < 4; ++w) {
        const long long lo = 64 * w;
        if (lo >= lim) break;
        unsigned long long mw = masks[w];
        if (lim - lo < 64) mw &= (1ull << (lim - lo)) - 1ull;
        earlier |= mw != 0ull;
      }
    }
    if (earlier) return;  // (every thread read the same masks)
#pragma unroll
    for (int w = 0; w < 4; ++w) {
      unsigned long long mw = masks[w];
      while (mw) {
        const int b = __builtin_ctzll(mw);
        mw &= mw - 1ull;
        const long long r = base + 64 * w + b;
#pragma unroll
        for (int e = 0; e < SCAT_MAXE; ++e) {
          const int c = tid + 256 * e;
          if (c < H) acc[e] += de[r * H + c];
        }
      }
    }
    __syncthreads();  // masks are rewritten by the next chunk
  }
#pragma unroll
  for (int e = 0; e < SCAT_MAXE; ++e) {
    const int c = tid + 256 * e;
    if (c < H) word_grad[id * H + c] += acc[e];
  }
}

// position grad: thread (l, c) sums the batch; the per-position sums also go to tmp [L][H]
__global__ void embed_pos_kernel(const float* __restrict__ de, float* __restrict__ pos_grad, float* __restrict__ tmp,
                                 int B, int L, int H) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  const int l = blockIdx.y;
  if (c >= H) return;
  float s = 0.f;
  for (int b = 0; b < B; ++b) s += de[((long long)b * L + l) * H + c];
  if (pos_grad) pos_grad[(long long)l * H + c] += s;
  tmp[(long long)l * H + c] = s;
}

// token-type grad (type id 0 everywhere): sum of the per-position sums, fixed order
__global__ void embed_type_kernel(const float* __restrict__ tmp, float* __restrict__ type_grad, int L, int H) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= H) return;
  double tot = 0;
  for (int l = 0; l < L; ++l) tot += tmp[(long long)l * H + c];
  type_grad[c] += (float)tot;
}

// ---------------------------------------------------------------- residual LayerNorm
// out = LN(dropout(x) + res)
template <typename T>
__global__ void ln_fwd_kernel(const T* __restrict__ x, const T* __restrict__ res, const float* __restrict__ gamma,
                              const float* __restrict__ beta, T* __restrict__ out, float* __restrict__ mean_out,
                              float* __restrict__ rstd_out, int H, float eps, float p, uint64_t seed) {
  const int row = blockIdx.x;
  __shared__ float red[16];
  float v[LN_MAXE];
  float s = 0.f;
#pragma unroll
  for (int e = 0; e < LN_MAXE; ++e) {
    const int c = threadIdx.x + e * blockDim.x;
    v[e] = 0.f;
    if (c < H) {
      const long long idx = (long long)row * H + c;
      float a = to_f<T>(x[idx]);
      a = keep(seed, idx, p) ? a / (1.f - p) : 0.f;
      if (res) a += to_f<T>(res[idx]);
      v[e] = a;
      s += a;
    }
  }
  const float mean = block_sum(s, red) / H;
  float s2 = 0.f;
#pragma unroll
  for (int e = 0; e < LN_MAXE; ++e) {
    const int c = threadIdx.x + e * blockDim.x;
    if (c < H) { const float d = v[e] - mean; s2 += d * d; }
  }
  const float var = block_sum(s2, red) / H;
  const float rstd = rsqrtf(var + eps);
#pragma unroll
  for (int e = 0; e < LN_MAXE; ++e) {
    const int c = threadIdx.x + e * blockDim.x;
    if (c < H) out[(long long)row * H + c] = from_f<T>((v[e] - mean) * rstd * gamma[c] + beta[c]);
  }
  if (threadIdx.x == 0) { mean_out[row] = mean; rstd_out[row] = rstd; }
}

// d(res) = ds, d(x) = ds * dropout_mask / (1-p); dgamma / dbeta partial sums per block
template <typename T>
__global__ void ln_bwd_kernel(const T* __restrict__ dout, const T* __restrict__ x, const T* __restrict__ res,
                              const float* __restrict__ gamma, const float* __restrict__ mean_in,
                              const float* __restrict__ rstd_in, T* __restrict__ dx, T* __restrict__ dres,
                              float* __restrict__ part, int H, int rows_per_block, int rows, float p, uint64_t seed) {
  __shared__ float red[16];
  float pg[LN_MAXE], pb[LN_MAXE];
#pragma unroll
  for (int e = 0; e < LN_MAXE; ++e) { pg[e] = 0.f; pb[e] = 0.f; }
  const int r0 = blockIdx.x * rows_per_block, r1 = min(rows, r0 + rows_per_block);
  for (int row = r0; row < r1; ++row) {
    const float mean = mean_in[row], rstd = rstd_in[row];
    float xh[LN_MAXE], dxh[LN_MAXE];
    float a = 0.f, b = 0.f;
#pragma unroll
    for (int e = 0; e < LN_MAXE; ++e) {
      const int c = threadIdx.x + e * blockDim.x;
      xh[e] = 0.f; dxh[e] = 0.f;
      if (c < H) {
        const long long idx = (long long)row * H + c;
        float v = to_f<T>(x[idx]);
        v = keep(seed, idx, p) ? v / (1.f - p) : 0.f;
        if (res) v += to_f<T>(res[idx]);
        xh[e] = (v - mean) * rstd;
        const float d = to_f<T>(dout[idx]);
        pg[e] += d * xh[e];
        pb[e] += d;
        dxh[e] = d * gamma[c];
        a += dxh[e];
        b += dxh[e] * xh[e];
      }
    }
    a = block_sum(a, red) / H;
    b = block_sum(b, red) / H;
#pragma unroll
    for (int e = 0; e < LN_MAXE; ++e) {
      const int c = threadIdx.x + e * blockDim.x;
      if (c < H) {
        const long long idx = (long long)row * H + c;
        const float ds = rstd * (dxh[e] - a - xh[e] * b);
        if (dres) dres[idx] = from_f<T>(ds);
        if (dx) dx[idx] = from_f<T>(keep(seed, idx, p) ? ds / (1.f - p) : 0.f);
      }
    }
  }
#pragma unroll
  for (int e = 0; e < LN_MAXE; ++e) {
    const int c = threadIdx.x + e * blockDim.x;
    if (c < H) {
      part[(long long)blockIdx.x * 2 * H + c] = pg[e];
      part[(long long)blockIdx.x * 2 * H + H + c] = pb[e];
    }
  }
}

// Column sums of partial rows (64 columns x 4 row-stripes per block, coalesced, fixed order):
//   out1[c] (+)= sum_i part[i*stride + c] ; out2[c] (+)= sum_i part[i*stride + off2 + c]
__global__ __launch_bounds__(256) void colred_kernel(const float* __restrict__ part, int nblocks, long long stride,
                                                     int N, long long off2, float* out1, float* out2, int accumulate) {
  __shared__ double sa[4][64], sb[4][64];
  const int tx = threadIdx.x & 63, ty = threadIdx.x >> 6;
  const int c = blockIdx.x * 64 + tx;
  double a = 0, b = 0;
  if (c < N) {
    for (int i = ty; i < nblocks; i += 4) {
      a += part[(long long)i * stride + c];
      if (out2) b += part[(long long)i * stride + off2 + c];
    }
  }
  sa[ty][tx] = a;
  sb[ty][tx] = b;
  __syncthreads();
  if (ty == 0 && c < N) {
    a = sa[0][tx] + sa[1][tx] + sa[2][tx] + sa[3][tx];
    b = sb[0][tx] + sb[1][tx] + sb[2][tx] + sb[3][tx];
    if (out1) out1[c] = (accumulate ? out1[c] : 0.f) + (float)a;
    if (out2) out2[c] = (accumulate ? out2[c] : 0.f) + (float)b;
  }
}

// ---------------------------------------------------------------- column sums (bias grads)
template <typename T>
__global__ void colsum_part_kernel(const T* __restrict__ x, long long ld, int rows, int N, int rows_per_block,
                                   float* __restrict__ part) {
  const int r0 = blockIdx.x * rows_per_block, r1 = min(rows, r0 + rows_per_block);
  for (int c = threadIdx.x; c < N; c += blockDim.x) {
    float s = 0.f;
    for (int r = r0; r < r1; ++r) s += to_f<T>(x[(long long)r * ld + c]);
    part[(long long)blockIdx.x * N + c] = s;
  }
}

// ---------------------------------------------------------------- attention softmax
// S [Z][L][Lp] raw scores (Z = B*nh). P = softmax(scale*S + mask_add) over valid keys.
// Writes P (pre-dropout, needed by the backward) and Pd = dropout(P) (input of the PV GEMM).
// HF eager attention adds finfo(f32).min to padded keys; exp() of that underflows to exactly 0,
// which is what excluding the key gives (a row with no valid key is uniform over all L keys, as in HF).
template <typename T> __device__ __forceinline__ void ld2(const T* p, float& a, float& b) {
  if constexpr (sizeof(T) == 4) {
    const float2 q = *reinterpret_cast<const float2*>(p);
    a = q.x; b = q.y;
  } else {
    const uint32_t q = *reinterpret_cast<const uint32_t*>(p);
    a = __uint_as_float(q << 16); b = __uint_as_float(q & 0xffff0000u);
  }
}
template <typename T> __device__ __forceinline__ void st2(T* p, float a, float b) {
  if constexpr (sizeof(T) == 4) {
    *reinterpret_cast<float2*>(p) = make_float2(a, b);
  } else {
    *reinterpret_cast<uint32_t*>(p) = (uint32_t)f2bf(a) | ((uint32_t)f2bf(b) << 16);
  }
}

// One wave per score row; lane l owns key pairs j = 2l + 128e (e < 4: L <= 512, Lp even): 4-B (bf16)
// / 8-B (fp32) loads and stores.
template <typename T>
__global__ __launch_bounds__(256) void attn_softmax_fwd_kernel(const T* __restrict__ S,
                                                               const long long* __restrict__ mask,
                                                               T* __restrict__ P, T* __restrict__ Pd, int nh, int L,
                                                               int Lp, float scale, float p, uint64_t seed) {
  const int z = blockIdx.y;
  const int b = z / nh;
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (row >= L) return;
  const long long base = ((long long)z * L + row) * Lp;
  constexpr int MAXE = 4;
  float v[MAXE][2];
  float mx = -INFINITY;
#pragma unroll
  for (int e = 0; e < MAXE; ++e) {
    const int j = 2 * lane + 128 * e;
    v[e][0] = v[e][1] = -INFINITY;
    if (j < L) {
      float a, c;
      ld2<T>(S + base + j, a, c);
      const bool k0 = mask == nullptr || mask[(long long)b * L + j] != 0;
      const bool k1 = j + 1 < L && (mask == nullptr || mask[(long long)b * L + j + 1] != 0);
      v[e][0] = k0 ? a * scale : -INFINITY;
      v[e][1] = k1 ? c * scale : -INFINITY;
      mx = fmaxf(mx, fmaxf(v[e][0], v[e][1]));
    }
  }
  mx = warp_max(mx);
  // every key masked (a zero-padding clip of the window dataset): HF's finfo.min bias absorbs the scores, so the
  // reference's softmax is uniform over all L keys
  const bool none = mx == -INFINITY;
  float sum = 0.f;
#pragma unroll
  for (int e = 0; e < MAXE; ++e)
#pragma unroll
    for (int k = 0; k < 2; ++k) {
      const bool in = 2 * lane + 128 * e + k < L;
      v[e][k] = none ? (in ? 1.f : 0.f) : (v[e][k] == -INFINITY) ? 0.f : __expf(v[e][k] - mx);
      sum += v[e][k];
    }
  sum = warp_sum(sum);
  const float inv = 1.f / sum;
#pragma unroll
  for (int e = 0; e < MAXE; ++e) {
    const int j = 2 * lane + 128 * e;
    if (j < Lp) {
      const float p0 = j < L ? v[e][0] * inv : 0.f;
      const float p1 = j + 1 < L ? v[e][1] * inv : 0.f;
      st2<T>(P + base + j, p0, p1);
      if (Pd) {
        const float d0 = keep(seed, base + j, p) ? p0 / (1.f - p) : 0.f;
        const float d1 = keep(seed, base + j + 1, p) ? p1 / (1.f - p) : 0.f;
        st2<T>(Pd + base + j, d0, d1);
      }
    }
  }
}

// dS = scale * P o (dP - rowsum(dP o P)), dP = dPd o mask/(1-p); same lane layout as the forward
template <typename T>
__global__ __launch_bounds__(256) void attn_softmax_bwd_kernel(const T* __restrict__ dPd, const T* __restrict__ P,
                                                               T* __restrict__ dS, int L, int Lp, float scale, float p,
                                                               uint64_t seed, int Z) {
  const int z = blockIdx.y;
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (row >= L || z >= Z) return;
  const long long base = ((long long)z * L + row) * Lp;
  constexpr int MAXE = 4;
  float dp[MAXE][2], pr[MAXE][2];
  float dot = 0.f;
#pragma unroll
  for (int e = 0; e < MAXE; ++e) {
    const int j = 2 * lane + 128 * e;
    dp[e][0] = dp[e][1] = pr[e][0] = pr[e][1] = 0.f;
    if (j < Lp) {
      float g0, g1;
      ld2<T>(P + base + j, pr[e][0], pr[e][1]);
      ld2<T>(dPd + base + j, g0, g1);
      dp[e][0] = (j < L && keep(seed, base + j, p)) ? g0 / (1.f - p) : 0.f;
      dp[e][1] = (j + 1 < L && keep(seed, base + j + 1, p)) ? g1 / (1.f - p) : 0.f;
      dot += dp[e][0] * pr[e][0] + dp[e][1] * pr[e][1];
    }
  }
  dot = warp_sum(dot);
#pragma unroll
  for (int e = 0; e < MAXE; ++e) {
    const int j = 2 * lane + 128 * e;
    if (j < Lp)
      st2<T>(dS + base + j, j < L ? scale * pr[e][0] * (dp[e][0] - dot) : 0.f,
             j + 1 < L ? scale * pr[e][1] * (dp[e][1] - dot) : 0.f);
  }
}

// ---------------------------------------------------------------- row-wise (one wave per row) kernels
// H = 256 * NQ: lane l owns the NQ 4-element chunks at columns 4 * (l + 64 q); loads are 8 B (bf16) /
// 16 B (fp32) per lane, row statistics are wave reductions (no LDS, no barriers).
template <typename T> __device__ __forceinline__ void ld4(const T* p, float (&v)[4]) {
  if constexpr (sizeof(T) == 4) {
    const float4 q = *reinterpret_cast<const float4*>(p);
    v[0] = q.x; v[1] = q.y; v[2] = q.z; v[3] = q.w;
  } else {
    const uint2 q = *reinterpret_cast<const uint2*>(p);
    v[0] = __uint_as_float(q.x << 16); v[1] = __uint_as_float(q.x & 0xffff0000u);
    v[2] = __uint_as_float(q.y << 16); v[3] = __uint_as_float(q.y & 0xffff0000u);
  }
}
template <typename T> __device__ __forceinline__ void st4(T* p, const float (&v)[4]) {
  if constexpr (sizeof(T) == 4) {
    *reinterpret_cast<float4*>(p) = make_float4(v[0], v[1], v[2], v[3]);
  } else {
    uint2 q;
    q.x = (uint32_t)f2bf(v[0]) | ((uint32_t)f2bf(v[1]) << 16);
    q.y = (uint32_t)f2bf(v[2]) | ((uint32_t)f2bf(v[3]) << 16);
    *reinterpret_cast<uint2*>(p) = q;
  }
}
__device__ __forceinline__ void ldf4(const float* p, float (&v)[4]) {
  const float4 q = *reinterpret_cast<const float4*>(p);
  v[0] = q.x; v[1] = q.y; v[2] = q.z; v[3] = q.w;
}

// out = LN(dropout(x) + res), one row per wave
template <typename T, int NQ>
__global__ __launch_bounds__(256) void ln_fwd_rw_kernel(const T* __restrict__ x, const T* __restrict__ res,
                                                        const float* __restrict__ gamma, const float* __restrict__ beta,
                                                        T* __restrict__ out, float* __restrict__ mean_out,
                                                        float* __restrict__ rstd_out, int rows, float eps, float p,
                                                        uint64_t seed) {
  constexpr int H = 256 * NQ;
  const int lane = threadIdx.x & 63;
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= rows) return;
  const long long rb = (long long)row * H;
  float v[NQ][4], r[NQ][4];
#pragma unroll
  for (int q = 0; q < NQ; ++q) {
    const int c = 4 * (lane + 64 * q);
    ld4<T>(x + rb + c, v[q]);
    if (res) ld4<T>(res + rb + c, r[q]);
  }
  float s = 0.f;
#pragma unroll
  for (int q = 0; q < NQ; ++q) {
    const int c = 4 * (lane + 64 * q);
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      float a = v[q][i];
      if (p > 0.f) a = keep(seed, rb + c + i, p) ? a / (1.f - p) : 0.f;
      if (res) a += r[q][i];
      v[q][i] = a;
      s += a;
    }
  }
  const float mean = warp_sum(s) * (1.f / H);
  float s2 = 0.f;
#pragma unroll
  for (int q = 0; q < NQ; ++q)
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const float d = v[q][i] - mean;
      s2 += d * d;
    }
  const float rstd = rsqrtf(warp_sum(s2) * (1.f / H) + eps);
#pragma unroll
  for (int q = 0; q < NQ; ++q) {
    const int c = 4 * (lane + 64 * q);
    float g[4], b[4], o[4];
    ldf4(gamma + c, g);
    ldf4(beta + c, b);
#pragma unroll
    for (int i = 0; i < 4; ++i) o[i] = (v[q][i] - mean) * rstd * g[i] + b[i];
    st4<T>(out + rb + c, o);
  }
  if (lane == 0) {
    mean_out[row] = mean;
    rstd_out[row] = rstd;
  }
}

// LN backward, rows strided over the grid's waves; per-block column partials part[block][NRED][H]:
// dgamma (sum dout * xhat), dbeta (sum dout) and (NRED = 3) the column sums of dx (the bias gradient of the
// dense layer in front of the LayerNorm). TD: the storage type of the incoming gradient dout and the residual
// gradient dres (fp32 for BERT's bf16 residual-gradient stream, as torch autocast keeps it), T that of x / res / dx.
template <typename T, typename TD, int NQ, int NRED>
__global__ __launch_bounds__(256) void ln_bwd_rw_kernel(const TD* __restrict__ dout, const T* __restrict__ x,
                                                        const T* __restrict__ res, const float* __restrict__ gamma,
                                                        const float* __restrict__ mean_in,
                                                        const float* __restrict__ rstd_in, T* __restrict__ dx,
                                                        TD* __restrict__ dres, float* __restrict__ part, int rows,
                                                        float p, uint64_t seed) {
  constexpr int H = 256 * NQ;
  __shared__ float red[4][NRED][H];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  float pg[NQ][4], pb[NQ][4], pd[NQ][4], gm[NQ][4];
#pragma unroll
  for (int q = 0; q < NQ; ++q) {
    ldf4(gamma + 4 * (lane + 64 * q), gm[q]);
#pragma unroll
    for (int i = 0; i < 4; ++i) pg[q][i] = pb[q][i] = pd[q][i] = 0.f;
  }
  // a wave walks rows row0, row0 + stride, ...; the next row's operands are loaded before this row's arithmetic
  // (one wave per SIMD walks up to 8 rows: without the prefetch each row paid a full HBM round trip)
  const int stride = gridDim.x * 4;
  float nx[NQ][4] = {}, nr[NQ][4] = {}, nd[NQ][4] = {}, nmean = 0.f, nrstd = 0.f;
  auto load_row = [&](int row) {
    const long long rb = (long long)row * H;
    nmean = mean_in[row];
    nrstd = rstd_in[row];
#pragma unroll
    for (int q = 0; q < NQ; ++q) {
      const int c = 4 * (lane + 64 * q);
      ld4<T>(x + rb + c, nx[q]);
      if (res) ld4<T>(res + rb + c, nr[q]);
      ld4<TD>(dout + rb + c, nd[q]);
    }
  };
  if (blockIdx.x * 4 + wave < rows) load_row(blockIdx.x * 4 + wave);
  for (int row = blockIdx.x * 4 + wave; row < rows; row += stride) {
    const long long rb = (long long)row * H;
    const float mean = nmean, rstd = nrstd;
    float xv[NQ][4], rv[NQ][4], dv[NQ][4];
#pragma unroll
    for (int q = 0; q < NQ; ++q)
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        xv[q][i] = nx[q][i];
        rv[q][i] = nr[q][i];
        dv[q][i] = nd[q][i];
      }
    if (row + stride < rows) load_row(row + stride);
    float a = 0.f, b = 0.f;
    uint32_t kb = 0xFFFFFFFFu;  // dropout keep bits of this lane's elements (hashed once)
#pragma unroll
    for (int q = 0; q < NQ; ++q) {
      const int c = 4 * (lane + 64 * q);
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        float v = xv[q][i];
        if (p > 0.f) {
          const bool k = keep(seed, rb + c + i, p);
          kb = k ? kb : (kb & ~(1u << (4 * q + i)));
          v = k ? v / (1.f - p) : 0.f;
        }
        if (res) v += rv[q][i];
        const float xh = (v - mean) * rstd;
        const float d = dv[q][i];
        pg[q][i] += d * xh;
        pb[q][i] += d;
        const float dxh = d * gm[q][i];
        xv[q][i] = xh;
        dv[q][i] = dxh;
        a += dxh;
        b += dxh * xh;
      }
    }
    a = warp_sum(a) * (1.f / H);
    b = warp_sum(b) * (1.f / H);
#pragma unroll
    for (int q = 0; q < NQ; ++q) {
      const int c = 4 * (lane + 64 * q);
      float o[4], od[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        o[i] = rstd * (dv[q][i] - a - xv[q][i] * b);
        od[i] = (p > 0.f) ? (((kb >> (4 * q + i)) & 1u) ? o[i] / (1.f - p) : 0.f) : o[i];
        if (NRED > 2) pd[q][i] += bf_round<T>(od[i]);
      }
      if (dres) st4<TD>(dres + rb + c, o);
      if (dx) st4<T>(dx + rb + c, od);
    }
  }
#pragma unroll
  for (int q = 0; q < NQ; ++q)
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int c = 4 * (lane + 64 * q) + i;
      red[wave][0][c] = pg[q][i];
      red[wave][1][c] = pb[q][i];
      if (NRED > 2) red[wave][NRED - 1][c] = pd[q][i];
    }
  __syncthreads();
  for (int i = threadIdx.x; i < NRED * H; i += 256) {
    const int r = i / H, c = i - r * H;
    part[(long long)blockIdx.x * NRED * H + i] = red[0][r][c] + red[1][r][c] + red[2][r][c] + red[3][r][c];
  }
}

// column sums of x [rows][ld] (first N columns): lane = 8 consecutive columns, waves stride the rows;
// per-block partials part[block][N]
template <typename T>
__global__ __launch_bounds__(256) void colsum_rw_kernel(const T* __restrict__ x, long long ld, int rows, int N,
                                                        float* __restrict__ part) {
  __shared__ float red[4][512];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int c0 = blockIdx.y * 512 + 8 * lane;
  float acc[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) acc[i] = 0.f;
  if (c0 < N) {
    for (int row = blockIdx.x * 4 + wave; row < rows; row += gridDim.x * 4) {
      float a[4], b[4];
      ld4<T>(x + (long long)row * ld + c0, a);
      ld4<T>(x + (long long)row * ld + c0 + 4, b);
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        acc[i] += a[i];
        acc[4 + i] += b[i];
      }
    }
  }
#pragma unroll
  for (int i = 0; i < 8; ++i) red[wave][8 * lane + i] = acc[i];
  __syncthreads();
  for (int i = threadIdx.x; i < 512; i += 256) {
    const int c = blockIdx.y * 512 + i;
    if (c < N) part[(long long)blockIdx.x * N + c] = red[0][i] + red[1][i] + red[2][i] + red[3][i];
  }
}

// column sums of a TALL x [rows][ld] with few columns (N = 8 cpr, cpr | 256: the trunk's conv inputs, 64..512
// channels over up to millions of pixel rows): a thread owns one 16-B column chunk of rows r0, r0 + rpi, ... (rpi =
// 256 / cpr rows per block step, U rows in flight per thread); per-block partials part[block][N], fixed order
template <typename T, int U>
__global__ __launch_bounds__(256) void colsum_tall_kernel(const T* __restrict__ x, long long ld, int rows, int N,
                                                          int cpr, float* __restrict__ part) {
  __shared__ float red[256][9];
  const int t = threadIdx.x, rpi = 256 / cpr;
  const int c = t % cpr, r0 = t / cpr;
  float acc[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) acc[i] = 0.f;
  const long long step = (long long)gridDim.x * rpi;
  for (long long row = (long long)blockIdx.x * rpi + r0; row < rows; row += step * U) {
    float v[U][8];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const long long r = min(row + u * step, (long long)rows - 1);  // clamped: unconditional loads
      float a[4], b[4];
      ld4<T>(x + r * ld + 8 * c, a);
      ld4<T>(x + r * ld + 8 * c + 4, b);
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        v[u][i] = a[i];
        v[u][4 + i] = b[i];
      }
    }
#pragma unroll
    for (int u = 0; u < U; ++u)
      if (row + u * step < rows) {
#pragma unroll
        for (int i = 0; i < 8; ++i) acc[i] += v[u][i];
      }
  }
#pragma unroll
  for (int i = 0; i < 8; ++i) red[t][i] = acc[i];
  __syncthreads();
  for (int o = t; o < N; o += 256) {  // (N = 512: two columns per thread)
    const int cc = o >> 3, i = o & 7;
    float a = 0.f;
    for (int r = 0; r < rpi; ++r) a += red[r * cpr + cc][i];
    part[(long long)blockIdx.x * N + o] = a;
  }
}

// Column sums of partial rows, 16 columns x 16 row-stripes per 256-thread block, fixed order (thread ty sums rows ty,
// ty + 16, ... in double, then the 16 stripes in order): out_k[c] (+)= sum_i part[i * stride + k * N + c], k < nout.
// (1024-thread blocks waited tens of us for a free CU beside the trunk's kernels.)
__global__ __launch_bounds__(256) void colred16_kernel(const float* __restrict__ part, int nblocks, long long stride,
                                                       int N, int nout, float* out0, float* out1, float* out2,
                                                       int accumulate) {
  __shared__ double sa[3][16][16];
  const int tx = threadIdx.x & 15, ty = threadIdx.x >> 4;
  const int c = blockIdx.x * 16 + tx;
  double a[3] = {0, 0, 0};
  if (c < N) {
    for (int i = ty; i < nblocks; i += 16)
#pragma unroll
      for (int k = 0; k < 3; ++k)
        if (k < nout) a[k] += part[(long long)i * stride + (long long)k * N + c];
  }
#pragma unroll
  for (int k = 0; k < 3; ++k) sa[k][ty][tx] = a[k];
  __syncthreads();
  if (ty < 3 && ty < nout && c < N) {
    double t = 0;
#pragma unroll
    for (int j = 0; j < 16; ++j) t += sa[ty][j][tx];
    float* o = ty == 0 ? out0 : (ty == 1 ? out1 : out2);
    if (o) o[c] = (accumulate ? o[c] : 0.f) + (float)t;
  }
}

// y = dy * (1 - t^2) where t = tanh output (pooler backward); all [rows][N] with given lds
template <typename T>
__global__ void tanh_bwd_kernel(const T* __restrict__ dy, const T* __restrict__ t, T* __restrict__ dx, long long n) {
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < n; i += (long long)gridDim.x * blockDim.x) {
    const float tv = to_f<T>(t[i]);
    dx[i] = from_f<T>(to_f<T>(dy[i]) * (1.f - tv * tv));
  }
}

}  // namespace

// ==================================================================== C ABI

VCG_API int vcg_embed_ln_fwd(int dtype, const long long* ids, const float* word, const float* pos, const float* type,
                             const float* gamma, const float* beta, void* out, float* mean, float* rstd, int B, int L,
                             int H, float eps, float dropout_p, unsigned long long seed, hipStream_t s) {
  VCG_REQUIRE(H <= 256 * LN_MAXE, "hidden size too large");
  if (dtype == VCG_BF16)
    hipLaunchKernelGGL(embed_ln_fwd_kernel<bf16_t>, dim3(B * L), dim3(256), 0, s, ids, word, pos, type, gamma, beta,
                       (bf16_t*)out, mean, rstd, L, H, eps, dropout_p, (uint64_t)seed);
  else
    hipLaunchKernelGGL(embed_ln_fwd_kernel<float>, dim3(B * L), dim3(256), 0, s, ids, word, pos, type, gamma, beta,
                       (float*)out, mean, rstd, L, H, eps, dropout_p, (uint64_t)seed);
  VCG_LAUNCH_CHECK();
  return VCG_OK;
}

static int row_blocks(int rows, int* rpb) {
  int nb = rows < 512 ? rows : 512;
  if (nb < 1) nb = 1;
  *rpb = (rows + nb - 1) / nb;
  return (rows + *rpb - 1) / *rpb;
}

VCG_API long long vcg_ln_bwd_ws_bytes(int rows, int H) {
  int rpb;
  const int nb = row_blocks(rows, &rpb);
  return (long long)nb * 2 * H * 4 + (long long)rows * H * 4;
}

// Embedding backward: LN backward + scatter into word / position / token-type grads (fp32, accumulated).
VCG_API int vcg_embed_ln_bwd(int dtype, const void* dout, const long long* ids, const float* word, const float* pos,
                             const float* type, const float* gamma, const float* mean, const float* rstd,
                             float* word_grad, float* pos_grad, float* type_grad, float* gamma_grad,
                             float* beta_grad, float* ws, long long ws_bytes, int B, int L, int H, float dropout_p,
                             unsigned long long seed, long long pad_idx, hipStream_t s) {
  const int rows = B * L;
  VCG_REQUIRE(ws_bytes >= vcg_ln_bwd_ws_bytes(rows, H), "workspace too small");
  VCG_REQUIRE(H <= SCAT_MAXE * 256, "hidden size > 1024 not supported by the word-grad reduction");
  if (dtype & VCG_GRAD_F32) dtype = VCG_F32;  // (only dout is read in the storage dtype here)
  int rpb;
  const int nb = row_blocks(rows, &rpb);
  float* part = ws;
  float* de = ws + (long long)nb * 2 * H;
  if (dtype == VCG_BF16)
    hipLaunchKernelGGL(embed_ln_bwd_kernel<bf16_t>, dim3(nb), dim3(256), 0, s, (const bf16_t*)dout, ids, word, pos,
                       type, gamma, mean, rstd, de, part, L, H, rpb, rows, dropout_p, (uint64_t)seed);
  else
    hipLaunchKernelGGL(embed_ln_bwd_kernel<float>, dim3(nb), dim3(256), 0, s, (const float*)dout, ids, word, pos,
                       type, gamma, mean, rstd, de, part, L, H, rpb, rows, dropout_p, (uint64_t)seed);
  VCG_LAUNCH_CHECK();
  hipLaunchKernelGGL(colred_kernel, dim3((H + 63) / 64), dim3(256), 0, s, part, nb, (long long)2 * H, H, (long long)H,
                     gamma_grad, beta_grad, 1);
  VCG_LAUNCH_CHECK();
  if (word_grad) {
    hipLaunchKernelGGL(embed_scatter_kernel, dim3(rows), dim3(256), 0, s, de, ids, word_grad, H, (long long)rows,
                       pad_idx);
    VCG_LAUNCH_CHECK();
  }
  // the partial region is free again: reuse it for the per-position sums (2*nb >= L since rows >= L)
  hipLaunchKernelGGL(embed_pos_kernel, dim3((H + 255) / 256, L), dim3(256), 0, s, de, pos_grad, part, B, L, H);
  VCG_LAUNCH_CHECK();
  if (type_grad) {
    hipLaunchKernelGGL(embed_type_kernel, dim3((H + 255) / 256), dim3(256), 0, s, part, type_grad, L, H);
    VCG_LAUNCH_CHECK();
  }
  return VCG_OK;
}

VCG_API int vcg_ln_fwd(int dtype, const void* x, const void* res, const float* gamma, const float* beta, void* out,
                       float* mean, float* rstd, int rows, int H, float eps, float dropout_p, unsigned long long seed,
                       hipStream_t s) {
  VCG_REQUIRE(H <= 256 * LN_MAXE, "hidden size too large");
  const int nq = H % 256 == 0 ? H / 256 : 0;
  if (nq >= 1 && nq <= 4 && rows > 0) {  // one wave per row
    const dim3 g((rows + 3) / 4);
#define VCG_LNF(T, NQ)                                                                                               \
  hipLaunchKernelGGL((ln_fwd_rw_kernel<T, NQ>), g, dim3(256), 0, s, (const T*)x, (const T*)res, gamma, beta, (T*)out, \
                     mean, rstd, rows, eps, dropout_p, (uint64_t)seed)
#define VCG_LNF_T(T)                          \
  switch (nq) {                               \
    case 1: VCG_LNF(T, 1); break;             \
    case 2: VCG_LNF(T, 2); break;             \
    case 3: VCG_LNF(T, 3); break;             \
    default: VCG_LNF(T, 4); break;            \
  }
    if (dtype == VCG_BF16) { VCG_LNF_T(bf16_t) } else { VCG_LNF_T(float) }
#undef VCG_LNF_T
#undef VCG_LNF
    VCG_LAUNCH_CHECK();
    return VCG_OK;
  }
  if (dtype == VCG_BF16)
    hipLaunchKernelGGL(ln_fwd_kernel<bf16_t>, dim3(rows), dim3(256), 0, s, (const bf16_t*)x, (const bf16_t*)res, gamma,
                       beta, (bf16_t*)out, mean, rstd, H, eps, dropout_p, (uint64_t)seed);
  else
    hipLaunchKernelGGL(ln_fwd_kernel<float>, dim3(rows), dim3(256), 0, s, (const float*)x, (const float*)res, gamma,
                       beta, (float*)out, mean, rstd, H, eps, dropout_p, (uint64_t)seed);
  VCG_LAUNCH_CHECK();
  return VCG_OK;
}

VCG_API int vcg_ln_bwd(int dtype, const void* dout, const void* x, const void* res, const float* gamma,
                       const float* mean, const float* rstd, void* dx, void* dres, float* gamma_grad,
                       float* beta_grad, float* bias_grad, float* ws, long long ws_bytes, int rows, int H,
                       float dropout_p, unsigned long long seed, hipStream_t s) {
  const bool g32 = (dtype & VCG_GRAD_F32) != 0;  // dout / dres in fp32 (bf16 x / res / dx)
  dtype &= ~VCG_GRAD_F32;
  VCG_REQUIRE(!g32 || (dtype == VCG_BF16 && H % 256 == 0 && H <= 1024), "VCG_GRAD_F32: bf16 with H % 256 == 0, <= 1024");
  int rpb;
  const int nb = row_blocks(rows, &rpb);
  VCG_REQUIRE(ws_bytes >= (long long)nb * 2 * H * 4, "workspace too small");
  VCG_REQUIRE(!bias_grad || dx, "bias_grad is the column sum of dx");
  const int nq = H % 256 == 0 ? H / 256 : 0;
  const int nbr = (rows + 3) / 4 < 256 ? (rows + 3) / 4 : 256;  // one wave per row, <= 8 rows per wave at 8192
  if (nq >= 1 && nq <= 4 && rows > 0 && ((long long)nbr * 3 * H <= (long long)nb * 2 * H || g32)) {
    const int nred = bias_grad ? 3 : 2;
    VCG_REQUIRE((long long)nbr * nred * H * 4 <= ws_bytes, "workspace too small");
#define VCG_LNB(T, TD, NQ, NR)                                                                                     \
  hipLaunchKernelGGL((ln_bwd_rw_kernel<T, TD, NQ, NR>), dim3(nbr), dim3(256), 0, s, (const TD*)dout, (const T*)x,   \
                     (const T*)res, gamma, mean, rstd, (T*)dx, (TD*)dres, ws, rows, dropout_p, (uint64_t)seed)
#define VCG_LNB_Q(T, TD, NR)                     \
  switch (nq) {                                  \
    case 1: VCG_LNB(T, TD, 1, NR); break;        \
    case 2: VCG_LNB(T, TD, 2, NR); break;        \
    case 3: VCG_LNB(T, TD, 3, NR); break;        \
    default: VCG_LNB(T, TD, 4, NR); break;       \
  }
    if (dtype == VCG_BF16 && g32) {
      if (nred == 3) { VCG_LNB_Q(bf16_t, float, 3) } else { VCG_LNB_Q(bf16_t, float, 2) }
    } else if (dtype == VCG_BF16) {
      if (nred == 3) { VCG_LNB_Q(bf16_t, bf16_t, 3) } else { VCG_LNB_Q(bf16_t, bf16_t, 2) }
    } else {
      if (nred == 3) { VCG_LNB_Q(float, float, 3) } else { VCG_LNB_Q(float, float, 2) }
    }
#undef VCG_LNB_Q
#undef VCG_LNB
    VCG_LAUNCH_CHECK();
    hipLaunchKernelGGL(colred16_kernel, dim3((H + 15) / 16), dim3(256), 0, s, ws, nbr, (long long)nred * H, H, nred,
                       gamma_grad, beta_grad, bias_grad, 1);
    VCG_LAUNCH_CHECK();
    return VCG_OK;
  }
  if (dtype == VCG_BF16)
    hipLaunchKernelGGL(ln_bwd_kernel<bf16_t>, dim3(nb), dim3(256), 0, s, (const bf16_t*)dout, (const bf16_t*)x,
                       (const bf16_t*)res, gamma, mean, rstd, (bf16_t*)dx, (bf16_t*)dres, ws, H, rpb, rows, dropout_p,
                       (uint64_t)seed);
  else
    hipLaunchKernelGGL(ln_bwd_kernel<float>, dim3(nb), dim3(256), 0, s, (const float*)dout, (const float*)x,
                       (const float*)res, gamma, mean, rstd, (float*)dx, (float*)dres, ws, H, rpb, rows, dropout_p,
                       (uint64_t)seed);
  VCG_LAUNCH_CHECK();
  hipLaunchKernelGGL(colred_kernel, dim3((H + 63) / 64), dim3(256), 0, s, ws, nb, (long long)2 * H, H, (long long)H,
                     gamma_grad, beta_grad, 1);
  VCG_LAUNCH_CHECK();
  if (bias_grad) {  // column sums of dx (generic path: the partial buffer is free again)
    if (dtype == VCG_BF16)
      hipLaunchKernelGGL(colsum_part_kernel<bf16_t>, dim3(nb), dim3(256), 0, s, (const bf16_t*)dx, (long long)H,
                         rows, H, rpb, ws);
    else
      hipLaunchKernelGGL(colsum_part_kernel<float>, dim3(nb), dim3(256), 0, s, (const float*)dx, (long long)H, rows,
                         H, rpb, ws);
    VCG_LAUNCH_CHECK();
    hipLaunchKernelGGL(colred_kernel, dim3((H + 63) / 64), dim3(256), 0, s, ws, nb, (long long)H, H, 0LL, bias_grad,
                       (float*)nullptr, 1);
    VCG_LAUNCH_CHECK();
  }
  return VCG_OK;
}

constexpr int COLSUM_TALL_BLOCKS = 1024;
static bool colsum_tall(int N, long long ld, const void* x, int rows) {
  const int cpr = N / 8;
  return N % 8 == 0 && N <= 512 && (256 % cpr) == 0 && ld % 8 == 0 && ((uintptr_t)x & 15) == 0 &&
         rows >= 8 * (256 / cpr) * 64;
}

VCG_API long long vcg_colsum_ws_bytes(int rows, int N) {
  int rpb;
  const int nb = row_blocks(rows, &rpb);
  return (long long)(nb > COLSUM_TALL_BLOCKS ? nb : COLSUM_TALL_BLOCKS) * N * 4;
}

// out[c] (+)= sum_r x[r][c]  (bias gradients)
VCG_API int vcg_colsum(int dtype, const void* x, long long ld, int rows, int N, float* out, int accumulate, float* ws,
                       long long ws_bytes, hipStream_t s) {
  int rpb;
  const int nb = row_blocks(rows, &rpb);
  VCG_REQUIRE(ws_bytes >= (long long)nb * N * 4, "workspace too small");
  if (dtype == VCG_BF16 && colsum_tall(N, ld, x, rows) && ws_bytes >= (long long)COLSUM_TALL_BLOCKS * N * 4) {
    const int cpr = N / 8, rpi = 256 / cpr;
    int nbx = (int)(((long long)rows + 4LL * rpi - 1) / (4LL * rpi));
    nbx = nbx < COLSUM_TALL_BLOCKS ? nbx : COLSUM_TALL_BLOCKS;
    hipLaunchKernelGGL((colsum_tall_kernel<bf16_t, 4>), dim3(nbx), dim3(256), 0, s, (const bf16_t*)x, ld, rows, N, cpr,
                       ws);
    VCG_LAUNCH_CHECK();
    hipLaunchKernelGGL(colred16_kernel, dim3((N + 15) / 16), dim3(256), 0, s, ws, nbx, (long long)N, N, 1, out,
                       (float*)nullptr, (float*)nullptr, accumulate);
    VCG_LAUNCH_CHECK();
    return VCG_OK;
  }
  if (N % 8 == 0 && ld % 4 == 0 && ((uintptr_t)x & 15) == 0 && rows > 0) {
    int nbx = (rows + 3) / 4;
    nbx = nbx < 128 ? nbx : 128;
    if (nbx > nb) nbx = nb;
    const dim3 g(nbx, (N + 511) / 512);
    if (dtype == VCG_BF16)
      hipLaunchKernelGGL(colsum_rw_kernel<bf16_t>, g, dim3(256), 0, s, (const bf16_t*)x, ld, rows, N, ws);
    else
      hipLaunchKernelGGL(colsum_rw_kernel<float>, g, dim3(256), 0, s, (const float*)x, ld, rows, N, ws);
    VCG_LAUNCH_CHECK();
    hipLaunchKernelGGL(colred16_kernel, dim3((N + 15) / 16), dim3(256), 0, s, ws, nbx, (long long)N, N, 1, out,
                       (float*)nullptr, (float*)nullptr, accumulate);
    VCG_LAUNCH_CHECK();
    return VCG_OK;
  }
  if (dtype == VCG_BF16)
    hipLaunchKernelGGL(colsum_part_kernel<bf16_t>, dim3(nb), dim3(256), 0, s, (const bf16_t*)x, ld, rows, N, rpb, ws);
  else
    hipLaunchKernelGGL(colsum_part_kernel<float>, dim3(nb), dim3(256), 0, s, (const float*)x, ld, rows, N, rpb, ws);
  VCG_LAUNCH_CHECK();
  hipLaunchKernelGGL(colred_kernel, dim3((N + 63) / 64), dim3(256), 0, s, ws, nb, (long long)N, N, 0LL, out,
                     (float*)nullptr, accumulate);
  VCG_LAUNCH_CHECK();
  return VCG_OK;
}

VCG_API int vcg_attn_softmax_fwd(int dtype, const void* S, const long long* mask, void* P, void* Pd, int B, int nh,
                                 int L, int Lp, float scale, float dropout_p, unsigned long long seed, hipStream_t s) {
  VCG_REQUIRE(L <= 512 && Lp >= L && Lp % 2 == 0 && Lp <= 512, "L must be <= 512, Lp even");
  dim3 grid((L + 3) / 4, B * nh);
  if (dtype == VCG_BF16)
    hipLaunchKernelGGL(attn_softmax_fwd_kernel<bf16_t>, grid, dim3(256), 0, s, (const bf16_t*)S, mask, (bf16_t*)P,
                       (bf16_t*)Pd, nh, L, Lp, scale, dropout_p, (uint64_t)seed);
  else
    hipLaunchKernelGGL(attn_softmax_fwd_kernel<float>, grid, dim3(256), 0, s, (const float*)S, mask, (float*)P,
                       (float*)Pd, nh, L, Lp, scale, dropout_p, (uint64_t)seed);
  VCG_LAUNCH_CHECK();
  return VCG_OK;
}

VCG_API int vcg_attn_softmax_bwd(int dtype, const void* dPd, const void* P, void* dS, int Z, int L, int Lp, float scale,
                                 float dropout_p, unsigned long long seed, hipStream_t s) {
  VCG_REQUIRE(L <= 512 && Lp >= L && Lp % 2 == 0 && Lp <= 512, "L must be <= 512, Lp even");
  dim3 grid((L + 3) / 4, Z);
  if (dtype == VCG_BF16)
    hipLaunchKernelGGL(attn_softmax_bwd_kernel<bf16_t>, grid, dim3(256), 0, s, (const bf16_t*)dPd, (const bf16_t*)P,
                       (bf16_t*)dS, L, Lp, scale, dropout_p, (uint64_t)seed, Z);
  else
    hipLaunchKernelGGL(attn_softmax_bwd_kernel<float>, grid, dim3(256), 0, s, (const float*)dPd, (const float*)P,
                       (float*)dS, L, Lp, scale, dropout_p, (uint64_t)seed, Z);
  VCG_LAUNCH_CHECK();
  return VCG_OK;
}

VCG_API int vcg_tanh_bwd(int dtype, const void* dy, const void* t, void* dx, long long n, hipStream_t s) {
  if (dtype == VCG_BF16)
    hipLaunchKernelGGL(tanh_bwd_kernel<bf16_t>, dim3(grid_for(n)), dim3(256), 0, s, (const bf16_t*)dy,
                       (const bf16_t*)t, (bf16_t*)dx, n);
  else
    hipLaunchKernelGGL(tanh_bwd_kernel<float>, dim3(grid_for(n)), dim3(256), 0, s, (const float*)dy, (const float*)t,
                       (float*)dx, n);
  VCG_LAUNCH_CHECK();
  return VCG_OK;
}
