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

__device__ __forceinline__ bool keep(uint64_t seed, uint64_t idx, float p) {
  if (p <= 0.f) return true;
  const uint64_t h = mix64(seed + 0x9E3779B97F4A7C15ULL * (idx + 1));
  const float u = (float)(h >> 40) * (1.0f / 16777216.0f);
  return u >= p;
}

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

// word grad scatter-add (atomics), position grad (sum over batch), token-type grad (sum over all)
__global__ void embed_scatter_kernel(const float* __restrict__ de, const long long* __restrict__ ids,
                                     float* __restrict__ word_grad, int H, long long rows, long long pad_idx) {
  const long long row = blockIdx.x;
  const long long id = ids[row];
  if (id == pad_idx) return;  // nn.Embedding(padding_idx): the padding row never receives gradient
  for (int c = threadIdx.x; c < H; c += blockDim.x) atomicAdd(&word_grad[id * H + c], de[row * H + c]);
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
// which is what excluding the key gives.
template <typename T>
__global__ void attn_softmax_fwd_kernel(const T* __restrict__ S, const long long* __restrict__ mask,
                                        T* __restrict__ P, T* __restrict__ Pd, int nh, int L, int Lp, float scale,
                                        float p, uint64_t seed) {
  const int z = blockIdx.y;
  const int b = z / nh;
  const int row = blockIdx.x * (blockDim.x / 64) + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (row >= L) return;
  const long long base = ((long long)z * L + row) * Lp;
  constexpr int MAXJ = 8;  // L <= 512
  float v[MAXJ];
  float mx = -INFINITY;
#pragma unroll
  for (int e = 0; e < MAXJ; ++e) {
    const int j = lane + e * 64;
    v[e] = -INFINITY;
    if (j < L && (mask == nullptr || mask[(long long)b * L + j] != 0)) v[e] = to_f<T>(S[base + j]) * scale;
    mx = fmaxf(mx, v[e]);
  }
  mx = warp_max(mx);
  float sum = 0.f;
#pragma unroll
  for (int e = 0; e < MAXJ; ++e) {
    v[e] = (v[e] == -INFINITY) ? 0.f : __expf(v[e] - mx);
    sum += v[e];
  }
  sum = warp_sum(sum);
  const float inv = 1.f / sum;
#pragma unroll
  for (int e = 0; e < MAXJ; ++e) {
    const int j = lane + e * 64;
    if (j < Lp) {
      const float pr = j < L ? v[e] * inv : 0.f;
      P[base + j] = from_f<T>(pr);
      if (Pd) Pd[base + j] = from_f<T>(keep(seed, base + j, p) ? pr / (1.f - p) : 0.f);
    }
  }
}

// dS = scale * P o (dP - rowsum(dP o P)), dP = dPd o mask/(1-p)
template <typename T>
__global__ void attn_softmax_bwd_kernel(const T* __restrict__ dPd, const T* __restrict__ P, T* __restrict__ dS, int L,
                                        int Lp, float scale, float p, uint64_t seed, int Z) {
  const int z = blockIdx.y;
  const int row = blockIdx.x * (blockDim.x / 64) + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (row >= L || z >= Z) return;
  const long long base = ((long long)z * L + row) * Lp;
  constexpr int MAXJ = 8;
  float dp[MAXJ], pr[MAXJ];
  float dot = 0.f;
#pragma unroll
  for (int e = 0; e < MAXJ; ++e) {
    const int j = lane + e * 64;
    dp[e] = 0.f; pr[e] = 0.f;
    if (j < L) {
      pr[e] = to_f<T>(P[base + j]);
      const float g = to_f<T>(dPd[base + j]);
      dp[e] = keep(seed, base + j, p) ? g / (1.f - p) : 0.f;
      dot += dp[e] * pr[e];
    }
  }
  dot = warp_sum(dot);
#pragma unroll
  for (int e = 0; e < MAXJ; ++e) {
    const int j = lane + e * 64;
    if (j < Lp) dS[base + j] = from_f<T>(j < L ? scale * pr[e] * (dp[e] - dot) : 0.f);
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
                       float* beta_grad, float* ws, long long ws_bytes, int rows, int H, float dropout_p,
                       unsigned long long seed, hipStream_t s) {
  int rpb;
  const int nb = row_blocks(rows, &rpb);
  VCG_REQUIRE(ws_bytes >= (long long)nb * 2 * H * 4, "workspace too small");
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
  return VCG_OK;
}

VCG_API long long vcg_colsum_ws_bytes(int rows, int N) {
  int rpb;
  const int nb = row_blocks(rows, &rpb);
  return (long long)nb * N * 4;
}

// out[c] (+)= sum_r x[r][c]  (bias gradients)
VCG_API int vcg_colsum(int dtype, const void* x, long long ld, int rows, int N, float* out, int accumulate, float* ws,
                       long long ws_bytes, hipStream_t s) {
  int rpb;
  const int nb = row_blocks(rows, &rpb);
  VCG_REQUIRE(ws_bytes >= (long long)nb * N * 4, "workspace too small");
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
  VCG_REQUIRE(L <= 512 && Lp >= L, "L must be <= 512");
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
