// Training kernels of the window model: reference model/fusion/two_stream_window.py
// (ChapterHead chains, CrossAttention) and stacked_window_self_attention.py (the 6-block pre-LN window
// transformer), trained by train_video_segment_ddp.py:294-342. fp32 row-major [rows][D] activations (the
// reference runs these heads in fp32); every backward regenerates its dropout mask from the forward's seed
// (dropout_keep, a stateless counter hash) and reduces parameter gradients in a fixed order (deterministic).
//
//   ln_act_drop   LayerNorm -> ReLU / GELU / none -> Dropout       (nn.Sequential(LayerNorm, ReLU, Dropout))
//   act_drop      act -> Dropout (+ residual)                       (FFN GELU / Dropout, residual joins)
//   mha_small     multi-head attention of short windows: Sq queries over Sk keys per window (Sq, Sk <= 32),
//                 optional additive per-head key bias (window_pos_bias), softmax, dropout, P V
//   mul_bwd       elementwise product backward (head_type "multiplication")
#include "common.h"

namespace vcg {
namespace {

constexpr int WT_MAXE = 8;  // LayerNorm rows up to 256 * 8 = 2048 wide

__device__ __forceinline__ float act_fwd(float u, int act) {
  if (act == 1) return fmaxf(u, 0.f);
  if (act == 2) return gelu_erf(u);
  return u;
}
__device__ __forceinline__ float act_grad(float u, int act) {
  if (act == 1) return u > 0.f ? 1.f : 0.f;
  if (act == 2) return gelu_erf_grad(u);
  return 1.f;
}

// out = dropout(act(LN(x))); mean / rstd saved per row. One workgroup (256) per row.
__global__ __launch_bounds__(256) void ln_act_drop_fwd_kernel(const float* __restrict__ x, const float* __restrict__ g,
                                                              const float* __restrict__ b, float* __restrict__ out,
                                                              float* __restrict__ mean_out, float* __restrict__ rstd_out,
                                                              int D, float eps, int act, float p, uint64_t seed) {
  __shared__ float red[16];
  const long long row = blockIdx.x;
  const float* xr = x + row * D;
  float v[WT_MAXE];
  float s = 0.f;
#pragma unroll
  for (int e = 0; e < WT_MAXE; ++e) {
    const int c = threadIdx.x + 256 * e;
    v[e] = c < D ? xr[c] : 0.f;
    s += v[e];
  }
  const float mean = block_sum(s, red) / D;
  float q = 0.f;
#pragma unroll
  for (int e = 0; e < WT_MAXE; ++e) {
    const int c = threadIdx.x + 256 * e;
    const float d = c < D ? v[e] - mean : 0.f;
    q += d * d;
  }
  const float rstd = rsqrtf(block_sum(q, red) / D + eps);  // biased variance, as nn.LayerNorm
  const float keep_scale = p > 0.f ? 1.f / (1.f - p) : 1.f;
#pragma unroll
  for (int e = 0; e < WT_MAXE; ++e) {
    const int c = threadIdx.x + 256 * e;
    if (c < D) {
      float y = act_fwd((v[e] - mean) * rstd * g[c] + b[c], act);
      const long long idx = row * D + c;
      y = dropout_keep(seed, (uint64_t)idx, p) ? y * keep_scale : 0.f;
      out[idx] = y;
    }
  }
  if (threadIdx.x == 0) {
    mean_out[row] = mean;
    rstd_out[row] = rstd;
  }
}

// dx of out = dropout(act(LN(x))); per-workgroup partial dgamma / dbeta over its rows -> part[blk][2][D]
__global__ __launch_bounds__(256) void ln_act_drop_bwd_kernel(const float* __restrict__ dout, const float* __restrict__ x,
                                                              const float* __restrict__ g, const float* __restrict__ b,
                                                              const float* __restrict__ mean, const float* __restrict__ rstd,
                                                              float* __restrict__ dx, float* __restrict__ part, int D,
                                                              int rows, int rpb, int act, float p, uint64_t seed) {
  __shared__ float red[16];
  float pg[WT_MAXE], pb[WT_MAXE];
#pragma unroll
  for (int e = 0; e < WT_MAXE; ++e) pg[e] = pb[e] = 0.f;
  const float keep_scale = p > 0.f ? 1.f / (1.f - p) : 1.f;
  const int r0 = blockIdx.x * rpb, r1 = min(rows, r0 + rpb);
  for (int row = r0; row < r1; ++row) {
    const float mu = mean[row], rs = rstd[row];
    float xh[WT_MAXE], dxh[WT_MAXE];
    float a = 0.f, c2 = 0.f;
#pragma unroll
    for (int e = 0; e < WT_MAXE; ++e) {
      const int c = threadIdx.x + 256 * e;
      xh[e] = dxh[e] = 0.f;
      if (c < D) {
        const long long idx = (long long)row * D + c;
        xh[e] = (x[idx] - mu) * rs;
        const float u = xh[e] * g[c] + b[c];
        float d = dout[idx];
        d = dropout_keep(seed, (uint64_t)idx, p) ? d * keep_scale : 0.f;
        d *= act_grad(u, act);  // d wrt the LayerNorm output
        pg[e] += d * xh[e];
        pb[e] += d;
        dxh[e] = d * g[c];
        a += dxh[e];
        c2 += dxh[e] * xh[e];
      }
    }
    a = block_sum(a, red) / D;
    c2 = block_sum(c2, red) / D;
#pragma unroll
    for (int e = 0; e < WT_MAXE; ++e) {
      const int c = threadIdx.x + 256 * e;
      if (c < D) dx[(long long)row * D + c] = rs * (dxh[e] - a - xh[e] * c2);
    }
  }
#pragma unroll
  for (int e = 0; e < WT_MAXE; ++e) {
    const int c = threadIdx.x + 256 * e;
    if (c < D) {
      part[((long long)blockIdx.x * 2) * D + c] = pg[e];
      part[((long long)blockIdx.x * 2 + 1) * D + c] = pb[e];
    }
  }
}

// gamma_grad[c] += sum_blk part[blk][0][c]; beta_grad[c] += sum_blk part[blk][1][c] (fixed order)
__global__ void part_reduce2_kernel(const float* __restrict__ part, int nb, int D, float* __restrict__ gg,
                                    float* __restrict__ bg) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= D) return;
  float s0 = 0.f, s1 = 0.f;
  for (int k = 0; k < nb; ++k) {
    s0 += part[((long long)k * 2) * D + c];
    s1 += part[((long long)k * 2 + 1) * D + c];
  }
  if (gg) gg[c] += s0;
  if (bg) bg[c] += s1;
}

__global__ void act_drop_fwd_kernel(const float* __restrict__ x, const float* __restrict__ res, float* __restrict__ out,
                                    long long n, int act, float p, uint64_t seed) {
  const float ks = p > 0.f ? 1.f / (1.f - p) : 1.f;
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < n; i += (long long)gridDim.x * blockDim.x) {
    float y = act_fwd(x[i], act);
    y = dropout_keep(seed, (uint64_t)i, p) ? y * ks : 0.f;
    out[i] = res ? y + res[i] : y;
  }
}

__global__ void act_drop_bwd_kernel(const float* __restrict__ dout, const float* __restrict__ x, float* __restrict__ dx,
                                    long long n, int act, float p, uint64_t seed) {
  const float ks = p > 0.f ? 1.f / (1.f - p) : 1.f;
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < n; i += (long long)gridDim.x * blockDim.x) {
    const float d = dropout_keep(seed, (uint64_t)i, p) ? dout[i] * ks : 0.f;
    dx[i] = d * act_grad(x[i], act);
  }
}

__global__ void mul_bwd_kernel(const float* __restrict__ dout, const float* __restrict__ a, const float* __restrict__ b,
                               float* __restrict__ da, float* __restrict__ db, long long n) {
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < n; i += (long long)gridDim.x * blockDim.x) {
    const float d = dout[i];
    if (da) da[i] = d * b[i];
    if (db) db[i] = d * a[i];
  }
}

// ---- multi-head attention of short windows ---------------------------------------------------------------
// One workgroup per window b; thread t < nh * Sq owns query row (h, i). q/k/v rows have strides ldq/ldk/ldv
// (fused QKV buffers); head h is columns [h*dh, (h+1)*dh). probs[b][h][i][j] = softmax_j(q.k * scale + bias[h][j])
// (pre-dropout, saved for the backward); ctx[b][i][h*dh + e] = sum_j drop(P)[i][j] v[j][h*dh + e].
constexpr int MHA_MAXS = 32;
constexpr int MHA_MAXD = 16;

__global__ __launch_bounds__(256) void mha_small_fwd_kernel(const float* __restrict__ q, long long ldq,
                                                            const float* __restrict__ k, long long ldk,
                                                            const float* __restrict__ v, long long ldv,
                                                            const float* __restrict__ bias, int Pb,
                                                            float* __restrict__ ctx, long long ldc,
                                                            float* __restrict__ probs, int Sq, int Sk, int nh, int dh,
                                                            float scale, float p, uint64_t seed) {
  const int b = blockIdx.x;
  const float ks = p > 0.f ? 1.f / (1.f - p) : 1.f;
  for (int t = threadIdx.x; t < nh * Sq; t += blockDim.x) {
    const int h = t / Sq, i = t - h * Sq;
    const float* qr = q + ((long long)b * Sq + i) * ldq + h * dh;
    float qv[MHA_MAXD];
#pragma unroll
    for (int e = 0; e < MHA_MAXD; ++e) qv[e] = e < dh ? qr[e] : 0.f;
    float s[MHA_MAXS];
    float mx = -INFINITY;
#pragma unroll
    for (int j = 0; j < MHA_MAXS; ++j) {
      s[j] = -INFINITY;
      if (j < Sk) {
        const float* kr = k + ((long long)b * Sk + j) * ldk + h * dh;
        float acc = 0.f;
#pragma unroll
        for (int e = 0; e < MHA_MAXD; ++e)
          if (e < dh) acc = fmaf(qv[e], kr[e], acc);
        acc *= scale;
        if (bias) acc += bias[(long long)h * Pb + j];
        s[j] = acc;
        mx = fmaxf(mx, acc);
      }
    }
    float sum = 0.f;
#pragma unroll
    for (int j = 0; j < MHA_MAXS; ++j) {
      s[j] = j < Sk ? __expf(s[j] - mx) : 0.f;
      sum += s[j];
    }
    const float inv = 1.f / sum;
    float o[MHA_MAXD];
#pragma unroll
    for (int e = 0; e < MHA_MAXD; ++e) o[e] = 0.f;
    const long long pbase = (((long long)b * nh + h) * Sq + i) * Sk;
#pragma unroll
    for (int j = 0; j < MHA_MAXS; ++j) {
      if (j < Sk) {
        const float pr = s[j] * inv;
        probs[pbase + j] = pr;
        const float pd = dropout_keep(seed, (uint64_t)(pbase + j), p) ? pr * ks : 0.f;
        const float* vr = v + ((long long)b * Sk + j) * ldv + h * dh;
#pragma unroll
        for (int e = 0; e < MHA_MAXD; ++e)
          if (e < dh) o[e] = fmaf(pd, vr[e], o[e]);
      }
    }
    float* cr = ctx + ((long long)b * Sq + i) * ldc + h * dh;
#pragma unroll
    for (int e = 0; e < MHA_MAXD; ++e)
      if (e < dh) cr[e] = o[e];
  }
}

// Backward. Phase 1 (thread per (h, i)): dPd = dctx . v_j, dP = dropout(dPd), dS = P (dP - sum P dP) -> LDS.
// Phase 2: dq (thread per (h, i)), dk / dv (thread per (h, j)), dbias partial of this window (thread per (h, j)).
__global__ __launch_bounds__(256) void mha_small_bwd_kernel(const float* __restrict__ q, long long ldq,
                                                            const float* __restrict__ k, long long ldk,
                                                            const float* __restrict__ v, long long ldv,
                                                            const float* __restrict__ probs,
                                                            const float* __restrict__ dctx, long long lddc,
                                                            float* __restrict__ dq, long long lddq,
                                                            float* __restrict__ dk, long long lddk,
                                                            float* __restrict__ dv, long long lddv,
                                                            float* __restrict__ dbias_part, int Pb, int Sq, int Sk,
                                                            int nh, int dh, float scale, float p, uint64_t seed) {
  extern __shared__ float sm[];
  float* dS = sm;                          // [nh][Sq][Sk]
  float* Pd = sm + nh * Sq * Sk;           // [nh][Sq][Sk] dropped probabilities
  const int b = blockIdx.x;
  const float ks = p > 0.f ? 1.f / (1.f - p) : 1.f;
  for (int t = threadIdx.x; t < nh * Sq; t += blockDim.x) {
    const int h = t / Sq, i = t - h * Sq;
    const float* dcr = dctx + ((long long)b * Sq + i) * lddc + h * dh;
    float dc[MHA_MAXD];
#pragma unroll
    for (int e = 0; e < MHA_MAXD; ++e) dc[e] = e < dh ? dcr[e] : 0.f;
    const long long pbase = (((long long)b * nh + h) * Sq + i) * Sk;
    float dp[MHA_MAXS], pr[MHA_MAXS];
    float dot = 0.f;
#pragma unroll
    for (int j = 0; j < MHA_MAXS; ++j) {
      dp[j] = pr[j] = 0.f;
      if (j < Sk) {
        const float* vr = v + ((long long)b * Sk + j) * ldv + h * dh;
        float acc = 0.f;
#pragma unroll
        for (int e = 0; e < MHA_MAXD; ++e)
          if (e < dh) acc = fmaf(dc[e], vr[e], acc);
        const bool kp = dropout_keep(seed, (uint64_t)(pbase + j), p);
        pr[j] = probs[pbase + j];
        dp[j] = kp ? acc * ks : 0.f;
        Pd[(h * Sq + i) * Sk + j] = kp ? pr[j] * ks : 0.f;
        dot = fmaf(pr[j], dp[j], dot);
      }
    }
#pragma unroll
    for (int j = 0; j < MHA_MAXS; ++j)
      if (j < Sk) dS[(h * Sq + i) * Sk + j] = pr[j] * (dp[j] - dot);
  }
  __syncthreads();
  for (int t = threadIdx.x; t < nh * Sq; t += blockDim.x) {  // dq_i = scale * sum_j dS_ij k_j
    const int h = t / Sq, i = t - h * Sq;
    float a[MHA_MAXD];
#pragma unroll
    for (int e = 0; e < MHA_MAXD; ++e) a[e] = 0.f;
    for (int j = 0; j < Sk; ++j) {
      const float d = dS[(h * Sq + i) * Sk + j];
      const float* kr = k + ((long long)b * Sk + j) * ldk + h * dh;
#pragma unroll
      for (int e = 0; e < MHA_MAXD; ++e)
        if (e < dh) a[e] = fmaf(d, kr[e], a[e]);
    }
    float* o = dq + ((long long)b * Sq + i) * lddq + h * dh;
#pragma unroll
    for (int e = 0; e < MHA_MAXD; ++e)
      if (e < dh) o[e] = a[e] * scale;
  }
  for (int t = threadIdx.x; t < nh * Sk; t += blockDim.x) {  // dk_j, dv_j, dbias[h][j]
    const int h = t / Sk, j = t - h * Sk;
    float ak[MHA_MAXD], av[MHA_MAXD];
#pragma unroll
    for (int e = 0; e < MHA_MAXD; ++e) ak[e] = av[e] = 0.f;
    float db = 0.f;
    for (int i = 0; i < Sq; ++i) {
      const float d = dS[(h * Sq + i) * Sk + j];
      const float pd = Pd[(h * Sq + i) * Sk + j];
      db += d;
      const float* qr = q + ((long long)b * Sq + i) * ldq + h * dh;
      const float* dcr = dctx + ((long long)b * Sq + i) * lddc + h * dh;
#pragma unroll
      for (int e = 0; e < MHA_MAXD; ++e)
        if (e < dh) {
          ak[e] = fmaf(d, qr[e], ak[e]);
          av[e] = fmaf(pd, dcr[e], av[e]);
        }
    }
    float* ok = dk + ((long long)b * Sk + j) * lddk + h * dh;
    float* ov = dv + ((long long)b * Sk + j) * lddv + h * dh;
#pragma unroll
    for (int e = 0; e < MHA_MAXD; ++e)
      if (e < dh) {
        ok[e] = ak[e] * scale;
        ov[e] = av[e];
      }
    if (dbias_part) dbias_part[((long long)b * nh + h) * Pb + j] = db;
  }
}

// dbias[h][j] += sum_b part[b][h][j] (fixed order); rows of the part beyond Sk are untouched
__global__ void bias_reduce_kernel(const float* __restrict__ part, int B, int nh, int Pb, int Sk, float* __restrict__ out) {
  const int t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= nh * Sk) return;
  const int h = t / Sk, j = t - h * Sk;
  float s = 0.f;
  for (int b = 0; b < B; ++b) s += part[((long long)b * nh + h) * Pb + j];
  out[(long long)h * Pb + j] += s;
}

// Linear(1, H) position encodings added to every token (VideoChapterWindowAttention :67-71, CrossAttention :64-67):
// out[r][c] = x[r][c] + pos[r % S] * w[c] + b[c]
__global__ void posenc_fwd_kernel(const float* __restrict__ x, const float* __restrict__ pos, const float* __restrict__ w,
                                  const float* __restrict__ b, float* __restrict__ out, long long rows, int S, int H) {
  const long long n = rows * H;
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < n; i += (long long)gridDim.x * blockDim.x) {
    const long long r = i / H;
    const int c = (int)(i - r * H);
    out[i] = x[i] + fmaf(pos[r % S], w[c], b[c]);
  }
}
// dw[c] += sum_r pos[r % S] d[r][c]; db[c] += sum_r d[r][c] (rows in order)
__global__ void posenc_bwd_kernel(const float* __restrict__ d, const float* __restrict__ pos, float* __restrict__ dw,
                                  float* __restrict__ db, long long rows, int S, int H) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= H) return;
  float sw = 0.f, sb = 0.f;
  for (long long r = 0; r < rows; ++r) {
    const float v = d[r * H + c];
    sw = fmaf(pos[r % S], v, sw);
    sb += v;
  }
  if (dw) dw[c] += sw;
  if (db) db[c] += sb;
}

// Linear layers too narrow for the 16-byte GEMM tiles (the 2-way classifiers; K or N not a multiple of 4):
// y[m][n] = act(sum_k x[m][k] W[n][k] + b[n] + res[m][n]); backward dX, dW (+=), db (+=) in fixed order
__global__ void linear_small_fwd_kernel(const float* __restrict__ x, const float* __restrict__ W,
                                        const float* __restrict__ b, const float* __restrict__ res, float* __restrict__ y,
                                        int M, int N, int K, int act) {
  const long long t = blockIdx.x * (long long)blockDim.x + threadIdx.x;
  if (t >= (long long)M * N) return;
  const int m = (int)(t / N), n = (int)(t - (long long)m * N);
  float acc = b ? b[n] : 0.f;
  for (int k = 0; k < K; ++k) acc = fmaf(x[(long long)m * K + k], W[(long long)n * K + k], acc);
  if (res) acc += res[t];
  y[t] = act_fwd(acc, act);
}
__global__ void linear_small_dx_kernel(const float* __restrict__ g, const float* __restrict__ W, float* __restrict__ dx,
                                       int M, int N, int K) {
  const long long t = blockIdx.x * (long long)blockDim.x + threadIdx.x;
  if (t >= (long long)M * K) return;
  const int m = (int)(t / K), k = (int)(t - (long long)m * K);
  float acc = 0.f;
  for (int n = 0; n < N; ++n) acc = fmaf(g[(long long)m * N + n], W[(long long)n * K + k], acc);
  dx[t] = acc;
}
__global__ void linear_small_dw_kernel(const float* __restrict__ g, const float* __restrict__ x, float* __restrict__ dw,
                                       float* __restrict__ db, int M, int N, int K) {
  const long long t = blockIdx.x * (long long)blockDim.x + threadIdx.x;
  if (t >= (long long)N * (K + 1)) return;
  const int n = (int)(t / (K + 1)), k = (int)(t - (long long)n * (K + 1));
  float acc = 0.f;
  if (k < K) {
    for (int m = 0; m < M; ++m) acc = fmaf(g[(long long)m * N + n], x[(long long)m * K + k], acc);
    if (dw) dw[(long long)n * K + k] += acc;
  } else {
    for (int m = 0; m < M; ++m) acc += g[(long long)m * N + n];
    if (db) db[n] += acc;
  }
}

__global__ void softmax_rows_kernel(const float* __restrict__ x, float* __restrict__ out, int rows, int C) {
  const int r = blockIdx.x * blockDim.x + threadIdx.x;
  if (r >= rows) return;
  const float* xr = x + (long long)r * C;
  float mx = -INFINITY;
  for (int c = 0; c < C; ++c) mx = fmaxf(mx, xr[c]);
  float s = 0.f;
  for (int c = 0; c < C; ++c) s += __expf(xr[c] - mx);
  const float inv = 1.f / s;
  for (int c = 0; c < C; ++c) out[(long long)r * C + c] = __expf(xr[c] - mx) * inv;
}

int ew_grid(long long n) {
  long long g = (n + 255) / 256;
  return (int)(g < 4096 ? (g > 0 ? g : 1) : 4096);
}

int rows_per_block(int rows, int* nb) {
  int n = rows < 512 ? rows : 512;
  if (n < 1) n = 1;
  const int rpb = (rows + n - 1) / n;
  *nb = (rows + rpb - 1) / rpb;
  return rpb;
}

}  // namespace
}  // namespace vcg

VCG_API int vcg_ln_act_drop_fwd(const float* x, const float* gamma, const float* beta, float* out, float* mean,
                                float* rstd, int rows, int D, float eps, int act, float dropout_p,
                                unsigned long long seed, hipStream_t s) {
  VCG_REQUIRE(D > 0 && D <= 256 * vcg::WT_MAXE, "LayerNorm width must be in [1, 2048]");
  VCG_REQUIRE(act >= 0 && act <= 2, "act must be none / relu / gelu");
  if (rows <= 0) return VCG_OK;
  VCG_REQUIRE(x && gamma && beta && out && mean && rstd, "null operand");
  hipLaunchKernelGGL(vcg::ln_act_drop_fwd_kernel, dim3(rows), dim3(256), 0, s, x, gamma, beta, out, mean, rstd, D,
                     eps, act, dropout_p, (uint64_t)seed);
  VCG_LAUNCH_CHECK();
  return VCG_OK;
}

VCG_API long long vcg_ln_act_drop_bwd_ws_bytes(int rows, int D) {
  int nb;
  vcg::rows_per_block(rows, &nb);
  return (long long)nb * 2 * D * 4;
}

VCG_API int vcg_ln_act_drop_bwd(const float* dout, const float* x, const float* gamma, const float* beta,
                                const float* mean, const float* rstd, float* dx, float* gamma_grad, float* beta_grad,
                                float* ws, long long ws_bytes, int rows, int D, int act, float dropout_p,
                                unsigned long long seed, hipStream_t s) {
  VCG_REQUIRE(D > 0 && D <= 256 * vcg::WT_MAXE, "LayerNorm width must be in [1, 2048]");
  if (rows <= 0) return VCG_OK;
  VCG_REQUIRE(dout && x && gamma && beta && mean && rstd && dx && ws, "null operand");
  VCG_REQUIRE(ws_bytes >= vcg_ln_act_drop_bwd_ws_bytes(rows, D), "workspace too small");
  int nb;
  const int rpb = vcg::rows_per_block(rows, &nb);
  hipLaunchKernelGGL(vcg::ln_act_drop_bwd_kernel, dim3(nb), dim3(256), 0, s, dout, x, gamma, beta, mean, rstd, dx, ws,
                     D, rows, rpb, act, dropout_p, (uint64_t)seed);
  VCG_LAUNCH_CHECK();
  if (gamma_grad || beta_grad) {
    hipLaunchKernelGGL(vcg::part_reduce2_kernel, dim3((D + 255) / 256), dim3(256), 0, s, ws, nb, D, gamma_grad,
                       beta_grad);
    VCG_LAUNCH_CHECK();
  }
  return VCG_OK;
}

VCG_API int vcg_act_drop_fwd(const float* x, const float* res, float* out, long long n, int act, float dropout_p,
                             unsigned long long seed, hipStream_t s) {
  VCG_REQUIRE(act >= 0 && act <= 2, "act must be none / relu / gelu");
  if (n <= 0) return VCG_OK;
  VCG_REQUIRE(x && out, "null operand");
  hipLaunchKernelGGL(vcg::act_drop_fwd_kernel, dim3(vcg::ew_grid(n)), dim3(256), 0, s, x, res, out, n, act, dropout_p,
                     (uint64_t)seed);
  VCG_LAUNCH_CHECK();
  return VCG_OK;
}

VCG_API int vcg_act_drop_bwd(const float* dout, const float* x, float* dx, long long n, int act, float dropout_p,
                             unsigned long long seed, hipStream_t s) {
  VCG_REQUIRE(act >= 0 && act <= 2, "act must be none / relu / gelu");
  if (n <= 0) return VCG_OK;
  VCG_REQUIRE(dout && x && dx, "null operand");
  hipLaunchKernelGGL(vcg::act_drop_bwd_kernel, dim3(vcg::ew_grid(n)), dim3(256), 0, s, dout, x, dx, n, act, dropout_p,
                     (uint64_t)seed);
  VCG_LAUNCH_CHECK();
  return VCG_OK;
}

VCG_API int vcg_mul_bwd(const float* dout, const float* a, const float* b, float* da, float* db, long long n,
                        hipStream_t s) {
  if (n <= 0) return VCG_OK;
  VCG_REQUIRE(dout && a && b, "null operand");
  hipLaunchKernelGGL(vcg::mul_bwd_kernel, dim3(vcg::ew_grid(n)), dim3(256), 0, s, dout, a, b, da, db, n);
  VCG_LAUNCH_CHECK();
  return VCG_OK;
}

VCG_API int vcg_mha_small_fwd(const float* q, long long ldq, const float* k, long long ldk, const float* v,
                              long long ldv, const float* bias, int Pb, float* ctx, long long ldc, float* probs, int B,
                              int Sq, int Sk, int nh, int dh, float scale, float dropout_p, unsigned long long seed,
                              hipStream_t s) {
  VCG_REQUIRE(Sq >= 1 && Sq <= vcg::MHA_MAXS && Sk >= 1 && Sk <= vcg::MHA_MAXS, "windows of 1..32 tokens");
  VCG_REQUIRE(dh >= 1 && dh <= vcg::MHA_MAXD && nh >= 1, "head size 1..16");
  VCG_REQUIRE(bias == nullptr || Pb >= Sk, "key bias shorter than the window");
  if (B <= 0) return VCG_OK;
  VCG_REQUIRE(q && k && v && ctx && probs, "null operand");
  hipLaunchKernelGGL(vcg::mha_small_fwd_kernel, dim3(B), dim3(256), 0, s, q, ldq, k, ldk, v, ldv, bias, Pb, ctx, ldc,
                     probs, Sq, Sk, nh, dh, scale, dropout_p, (uint64_t)seed);
  VCG_LAUNCH_CHECK();
  return VCG_OK;
}

VCG_API long long vcg_mha_small_bwd_ws_bytes(int B, int nh, int Pb) { return (long long)B * nh * (Pb > 0 ? Pb : 1) * 4; }

VCG_API int vcg_mha_small_bwd(const float* q, long long ldq, const float* k, long long ldk, const float* v,
                              long long ldv, const float* probs, const float* dctx, long long lddc, float* dq,
                              long long lddq, float* dk, long long lddk, float* dv, long long lddv, float* dbias,
                              int Pb, float* ws, long long ws_bytes, int B, int Sq, int Sk, int nh, int dh, float scale,
                              float dropout_p, unsigned long long seed, hipStream_t s) {
  VCG_REQUIRE(Sq >= 1 && Sq <= vcg::MHA_MAXS && Sk >= 1 && Sk <= vcg::MHA_MAXS, "windows of 1..32 tokens");
  VCG_REQUIRE(dh >= 1 && dh <= vcg::MHA_MAXD && nh >= 1, "head size 1..16");
  if (B <= 0) return VCG_OK;
  VCG_REQUIRE(q && k && v && probs && dctx && dq && dk && dv, "null operand");
  if (dbias) VCG_REQUIRE(ws && ws_bytes >= vcg_mha_small_bwd_ws_bytes(B, nh, Pb) && Pb >= Sk, "bias workspace");
  const size_t lds = (size_t)2 * nh * Sq * Sk * sizeof(float);
  VCG_REQUIRE(lds <= 64 * 1024, "window too large for the LDS score buffers");
  hipLaunchKernelGGL(vcg::mha_small_bwd_kernel, dim3(B), dim3(256), lds, s, q, ldq, k, ldk, v, ldv, probs, dctx, lddc,
                     dq, lddq, dk, lddk, dv, lddv, dbias ? ws : nullptr, Pb, Sq, Sk, nh, dh, scale, dropout_p,
                     (uint64_t)seed);
  VCG_LAUNCH_CHECK();
  if (dbias) {
    hipLaunchKernelGGL(vcg::bias_reduce_kernel, dim3((nh * Sk + 255) / 256), dim3(256), 0, s, ws, B, nh, Pb, Sk, dbias);
    VCG_LAUNCH_CHECK();
  }
  return VCG_OK;
}

VCG_API int vcg_softmax_rows(const float* x, float* out, int rows, int C, hipStream_t s) {
  if (rows <= 0) return VCG_OK;
  VCG_REQUIRE(x && out && C > 0, "bad operands");
  hipLaunchKernelGGL(vcg::softmax_rows_kernel, dim3((rows + 255) / 256), dim3(256), 0, s, x, out, rows, C);
  VCG_LAUNCH_CHECK();
  return VCG_OK;
}

VCG_API int vcg_posenc_fwd(const float* x, const float* pos, const float* w, const float* b, float* out, long long rows,
                           int S, int H, hipStream_t s) {
  if (rows <= 0) return VCG_OK;
  VCG_REQUIRE(x && pos && w && b && out && S > 0 && H > 0, "bad operands");
  hipLaunchKernelGGL(vcg::posenc_fwd_kernel, dim3(vcg::ew_grid(rows * H)), dim3(256), 0, s, x, pos, w, b, out, rows, S, H);
  VCG_LAUNCH_CHECK();
  return VCG_OK;
}

VCG_API int vcg_posenc_bwd(const float* d, const float* pos, float* dw, float* db, long long rows, int S, int H,
                           hipStream_t s) {
  if (rows <= 0) return VCG_OK;
  VCG_REQUIRE(d && pos && S > 0 && H > 0, "bad operands");
  hipLaunchKernelGGL(vcg::posenc_bwd_kernel, dim3((H + 255) / 256), dim3(256), 0, s, d, pos, dw, db, rows, S, H);
  VCG_LAUNCH_CHECK();
  return VCG_OK;
}

VCG_API int vcg_linear_small_fwd(const float* x, const float* W, const float* b, const float* res, float* y, int M,
                                 int N, int K, int act, hipStream_t s) {
  VCG_REQUIRE(act >= 0 && act <= 2, "act must be none / relu / gelu");
  if ((long long)M * N <= 0) return VCG_OK;
  VCG_REQUIRE(x && W && y && K > 0, "bad operands");
  const long long n = (long long)M * N;
  hipLaunchKernelGGL(vcg::linear_small_fwd_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, x, W, b, res, y, M,
                     N, K, act);
  VCG_LAUNCH_CHECK();
  return VCG_OK;
}

VCG_API int vcg_linear_small_bwd(const float* g, const float* x, const float* W, float* dx, float* dw, float* db, int M,
                                 int N, int K, hipStream_t s) {
  if ((long long)M * N <= 0) return VCG_OK;
  VCG_REQUIRE(g && x && W && K > 0, "bad operands");
  if (dx) {
    const long long n = (long long)M * K;
    hipLaunchKernelGGL(vcg::linear_small_dx_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, g, W, dx, M, N, K);
    VCG_LAUNCH_CHECK();
  }
  if (dw || db) {
    const long long n = (long long)N * (K + 1);
    hipLaunchKernelGGL(vcg::linear_small_dw_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, g, x, dw, db, M, N,
                       K);
    VCG_LAUNCH_CHECK();
  }
  return VCG_OK;
}
