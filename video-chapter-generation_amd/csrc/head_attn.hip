// ChapterHead with head_type "attn" (reference model/fusion/two_stream.py:8-48, 63-67, 71-95).
//
//   X = cat([relu(vision_emb W_v^T) [B,T,hid], relu(lang_emb W_l^T) [B,1,hid]], 1)   (line 88, vision first)
//   SelfAttention(hid, n_head=4, output_size):
//     k/q/v = X W^T + b, split into heads of hs = hid / n_head
//     att = softmax(q k^T / sqrt(hs)) ; att = attn_drop(att) ; y = att v
//     out = proj(y[:, 0])            (only the FIRST token -- the first vision frame -- is used, line 46)
//   No mask (the "causal" comment at line 38 is not implemented by the reference).
//
// Only token 0's query row reaches the output, so the forward computes k, v for all T+1 tokens but q
// for token 0 only, and the backward sends query gradients to token 0 only: the same function, less
// work. One workgroup per clip window owns the whole per-window computation (T+1 <= 64 tokens,
// hid <= 256): the head is launch-bound (~0.05 GFLOP per 64 windows), so everything between the two
// projection GEMMs (which run on the MFMA engine) is ONE launch forward and ONE backward, plus the
// parameter-gradient column reductions (deterministic, no atomics).
#include "common.h"

using namespace vcg;

namespace {

constexpr int kMaxTok = 64;   // T + 1
constexpr int kMaxHid = 256;
constexpr int kMaxHeads = 16;
constexpr int kMaxOut = 256;  // output_size (2 for the fusion head, hidden for the window self_attn head)

// token j of window b: vision rows first, then the language row
template <typename T>
__device__ __forceinline__ float tok(const T* Vout, const T* Lout, int b, int j, int d, int Tn, int hid) {
  return j < Tn ? to_f<T>(Vout[((long long)b * Tn + j) * hid + d]) : to_f<T>(Lout[(long long)b * hid + d]);
}

// dropout element index of att[b, h, 0, j] in the reference's [B, nh, T1, T1] attention tensor
__device__ __forceinline__ unsigned long long att_idx(int b, int h, int j, int nh, int T1) {
  return ((unsigned long long)b * nh + h) * (unsigned long long)(T1 * T1) + j;
}

// Forward. LDS: X, K, V [T1][hid] f32, q0 / y0 [hid], P [nh][T1].
// Saved for the backward (f32): X, K, V [B][T1][hid], q0 / y0 [B][hid], P [B][nh][T1] (pre-dropout).
template <typename T>
__global__ void __launch_bounds__(256) head_attn_fwd_kernel(
    const T* __restrict__ Vout, const T* __restrict__ Lout, const float* __restrict__ Wq, const float* __restrict__ bq,
    const float* __restrict__ Wk, const float* __restrict__ bk, const float* __restrict__ Wv,
    const float* __restrict__ bv, const float* __restrict__ Wp, const float* __restrict__ bp, float* __restrict__ Xs,
    float* __restrict__ Ks, float* __restrict__ Vs, float* __restrict__ q0s, float* __restrict__ Ps,
    float* __restrict__ y0s, float* __restrict__ logits, float* __restrict__ prob, int Tn, int hid, int nh, int O,
    float p_drop, unsigned long long seed) {
  extern __shared__ float sm[];
  __shared__ float lg[kMaxOut];
  const int T1 = Tn + 1, b = blockIdx.x, tid = threadIdx.x, nt = blockDim.x;
  const int hs = hid / nh;
  float* X = sm;
  float* K = X + T1 * hid;
  float* V = K + T1 * hid;
  float* q0 = V + T1 * hid;
  float* y0 = q0 + hid;
  float* Pm = y0 + hid;  // [nh][T1]
  const long long wb = (long long)b * T1 * hid;

  for (int i = tid; i < T1 * hid; i += nt) {
    const int j = i / hid, d = i - j * hid;
    const float x = tok(Vout, Lout, b, j, d, Tn, hid);
    X[i] = x;
    Xs[wb + i] = x;
  }
  __syncthreads();
  // k, v of every token and q of token 0: thread c owns output column n of weight w; the weight row is
  // streamed once per 8 tokens (X reads are LDS broadcasts)
  for (int c = tid; c < 3 * hid; c += nt) {
    const int w = c / hid, n = c - w * hid;
    const float* Wr = (w == 0 ? Wk : w == 1 ? Wv : Wq) + (long long)n * hid;
    const float bias = (w == 0 ? bk : w == 1 ? bv : bq)[n];
    const int jn = w == 2 ? 1 : T1;
    for (int j0 = 0; j0 < jn; j0 += 8) {
      float acc[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) acc[u] = bias;
      for (int d = 0; d < hid; ++d) {
        const float wv = Wr[d];
#pragma unroll
        for (int u = 0; u < 8; ++u)
          if (j0 + u < jn) acc[u] = fmaf(X[(j0 + u) * hid + d], wv, acc[u]);
      }
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        if (j0 + u >= jn) break;
        if (w == 0) K[(j0 + u) * hid + n] = acc[u];
        else if (w == 1) V[(j0 + u) * hid + n] = acc[u];
        else q0[n] = acc[u];
      }
    }
  }
  __syncthreads();
  // scores of query 0 against every key, per head
  const float scale = rsqrtf((float)hs);
  for (int i = tid; i < nh * T1; i += nt) {
    const int h = i / T1, j = i - h * T1;
    float s = 0.f;
    for (int e = 0; e < hs; ++e) s = fmaf(q0[h * hs + e], K[j * hid + h * hs + e], s);
    Pm[i] = s * scale;
  }
  __syncthreads();
  if (tid < nh) {  // softmax over the T1 keys of head tid
    float* r = Pm + tid * T1;
    float mx = -INFINITY;
    for (int j = 0; j < T1; ++j) mx = fmaxf(mx, r[j]);
    float sum = 0.f;
    for (int j = 0; j < T1; ++j) {
      r[j] = expf(r[j] - mx);
      sum += r[j];
    }
    const float inv = 1.f / sum;
    for (int j = 0; j < T1; ++j) r[j] *= inv;
  }
  __syncthreads();
  for (int i = tid; i < nh * T1; i += nt) Ps[(long long)b * nh * T1 + i] = Pm[i];
  // y0 = attn_drop(P) v
  for (int n = tid; n < hid; n += nt) {
    const int h = n / hs;
    float s = 0.f;
    for (int j = 0; j < T1; ++j) {
      float pj = Pm[h * T1 + j];
      if (p_drop > 0.f) pj = dropout_keep(seed, att_idx(b, h, j, nh, T1), p_drop) ? pj / (1.f - p_drop) : 0.f;
      s = fmaf(pj, V[j * hid + n], s);
    }
    y0[n] = s;
    y0s[(long long)b * hid + n] = s;
    q0s[(long long)b * hid + n] = q0[n];
  }
  for (int i = tid; i < T1 * hid; i += nt) {
    Ks[wb + i] = K[i];
    Vs[wb + i] = V[i];
  }
  __syncthreads();
  // proj: logits[o] = y0 . Wp[o] + bp[o]  (one wave per output)
  const int lane = tid & 63, wid = tid >> 6;
  for (int o = wid; o < O; o += nt >> 6) {
    float s = 0.f;
    for (int n = lane; n < hid; n += 64) s = fmaf(y0[n], Wp[(long long)o * hid + n], s);
    s = warp_sum(s);
    if (lane == 0) lg[o] = s + (bp ? bp[o] : 0.f);
  }
  __syncthreads();
  if (tid == 0) {
    float mx = -INFINITY;
    for (int o = 0; o < O; ++o) mx = fmaxf(mx, lg[o]);
    float sum = 0.f;
    for (int o = 0; o < O; ++o) sum += expf(lg[o] - mx);
    for (int o = 0; o < O; ++o) {
      logits[(long long)b * O + o] = lg[o];
      if (prob) prob[(long long)b * O + o] = expf(lg[o] - mx) / sum;
    }
  }
}

// Backward of everything between the projections: from dlogits to the (ReLU-masked) gradients of the
// vision / language projection outputs, plus dK, dV [B][T1][hid] and dq0 [B][hid] (f32) for the
// parameter-gradient reductions.
template <typename T>
__global__ void __launch_bounds__(256) head_attn_bwd_kernel(
    const float* __restrict__ Xs, const float* __restrict__ Ks, const float* __restrict__ Vs,
    const float* __restrict__ q0s, const float* __restrict__ Ps, const float* __restrict__ Wq,
    const float* __restrict__ Wk, const float* __restrict__ Wv, const float* __restrict__ Wp,
    const float* __restrict__ dlogits, float* __restrict__ dKs, float* __restrict__ dVs, float* __restrict__ dq0s,
    T* __restrict__ dVout, T* __restrict__ dLout, int Tn, int hid, int nh, int O, float p_drop,
    unsigned long long seed, int relu_mask) {
  extern __shared__ float sm[];
  const int T1 = Tn + 1, b = blockIdx.x, tid = threadIdx.x, nt = blockDim.x;
  const int hs = hid / nh;
  float* dK = sm;               // [T1][hid]
  float* dV = dK + T1 * hid;    // [T1][hid]
  float* dy0 = dV + T1 * hid;   // [hid]
  float* dq0 = dy0 + hid;       // [hid]
  float* Pm = dq0 + hid;        // [nh][T1]
  float* dS = Pm + nh * T1;     // [nh][T1]
  const long long wb = (long long)b * T1 * hid;
  const float* K = Ks + wb;
  const float* V = Vs + wb;
  const float* q0 = q0s + (long long)b * hid;
  const float scale = rsqrtf((float)hs);
  const float inv_keep = p_drop > 0.f ? 1.f / (1.f - p_drop) : 1.f;

  for (int i = tid; i < nh * T1; i += nt) Pm[i] = Ps[(long long)b * nh * T1 + i];
  for (int n = tid; n < hid; n += nt) {
    float s = 0.f;
    for (int o = 0; o < O; ++o) s = fmaf(dlogits[(long long)b * O + o], Wp[(long long)o * hid + n], s);
    dy0[n] = s;
  }
  __syncthreads();
  // dP[h][j] = dropout adjoint of dy0_h . v_jh ; dV_jh = attn_drop(P)[h][j] dy0_h
  for (int i = tid; i < nh * T1; i += nt) {
    const int h = i / T1, j = i - h * T1;
    float s = 0.f;
    for (int e = 0; e < hs; ++e) s = fmaf(dy0[h * hs + e], V[j * hid + h * hs + e], s);
    dS[i] = dropout_keep(seed, att_idx(b, h, j, nh, T1), p_drop) ? s * inv_keep : 0.f;
  }
  for (int i = tid; i < T1 * hid; i += nt) {
    const int j = i / hid, n = i - j * hid, h = n / hs;
    dV[i] = dropout_keep(seed, att_idx(b, h, j, nh, T1), p_drop) ? Pm[h * T1 + j] * inv_keep * dy0[n] : 0.f;
  }
  __syncthreads();
  if (tid < nh) {  // softmax backward of head tid, with the 1/sqrt(hs) of the scores folded in
    float dot = 0.f;
    for (int j = 0; j < T1; ++j) dot = fmaf(Pm[tid * T1 + j], dS[tid * T1 + j], dot);
    for (int j = 0; j < T1; ++j) dS[tid * T1 + j] = Pm[tid * T1 + j] * (dS[tid * T1 + j] - dot) * scale;
  }
  __syncthreads();
  // dq0 = sum_j dS k_j ; dK_j = dS q0
  for (int n = tid; n < hid; n += nt) {
    const int h = n / hs;
    float s = 0.f;
    for (int j = 0; j < T1; ++j) s = fmaf(dS[h * T1 + j], K[j * hid + n], s);
    dq0[n] = s;
    dq0s[(long long)b * hid + n] = s;
  }
  for (int i = tid; i < T1 * hid; i += nt) {
    const int j = i / hid, n = i - j * hid, h = n / hs;
    dK[i] = dS[h * T1 + j] * q0[n];
  }
  __syncthreads();
  for (int i = tid; i < T1 * hid; i += nt) {
    dKs[wb + i] = dK[i];
    dVs[wb + i] = dV[i];
  }
  // dX[j][d] = sum_n dK[j][n] Wk[n][d] + dV[j][n] Wv[n][d] (+ dq0[n] Wq[n][d] at j = 0), masked by relu(X) > 0;
  // thread d walks a weight column (coalesced across the wave), 8 tokens per pass
  for (int d = tid; d < hid; d += nt) {
    for (int j0 = 0; j0 < T1; j0 += 8) {
      float acc[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) acc[u] = 0.f;
      for (int n = 0; n < hid; ++n) {
        const float wk = Wk[(long long)n * hid + d], wv = Wv[(long long)n * hid + d];
#pragma unroll
        for (int u = 0; u < 8; ++u)
          if (j0 + u < T1) acc[u] = fmaf(dK[(j0 + u) * hid + n], wk, fmaf(dV[(j0 + u) * hid + n], wv, acc[u]));
      }
      if (j0 == 0)
        for (int n = 0; n < hid; ++n) acc[0] = fmaf(dq0[n], Wq[(long long)n * hid + d], acc[0]);
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        const int j = j0 + u;
        if (j >= T1) break;
        const float x = Xs[wb + (long long)j * hid + d];
        const T g = from_f<T>((!relu_mask || x > 0.f) ? acc[u] : 0.f);
        if (j < Tn) dVout[((long long)b * Tn + j) * hid + d] = g;
        else dLout[(long long)b * hid + d] = g;
      }
    }
  }
}

// out[m][n] += sum_r A[r * lda + m] * Bm[r * ldb + n]  (Bm == nullptr: column sums of A), f32.
// Parameter gradients of the head (dW = dY^T X over the rows of the batch): one thread per output and a
// fixed summation order (deterministic, no atomics).
__global__ void head_colgemm_kernel(const float* __restrict__ A, long long lda, const float* __restrict__ Bm,
                                    long long ldb, float* __restrict__ out, int rows, int M, int N) {
  const long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x;
  if (i >= (long long)M * N) return;
  const int m = (int)(i / N), n = (int)(i - (long long)m * N);
  float s = 0.f;
  for (int r = 0; r < rows; ++r) s = fmaf(A[(long long)r * lda + m], Bm ? Bm[(long long)r * ldb + n] : 1.f, s);
  out[i] += s;
}

int colgemm(const float* A, long long lda, const float* Bm, long long ldb, float* out, int rows, int M, int N,
            hipStream_t s) {
  if (!out) return VCG_OK;
  const long long tot = (long long)M * N;
  hipLaunchKernelGGL(head_colgemm_kernel, dim3((unsigned)((tot + 255) / 256)), dim3(256), 0, s, A, lda, Bm, ldb, out,
                     rows, M, N);
  VCG_LAUNCH_CHECK();
  return VCG_OK;
}

int check_shapes(int B, int T, int hid, int nh, int O) {
  VCG_REQUIRE(B > 0 && T > 0 && T + 1 <= kMaxTok, "need 1 <= T and T + 1 <= 64 tokens");
  VCG_REQUIRE(hid > 0 && hid <= kMaxHid && nh > 0 && nh <= kMaxHeads && hid % nh == 0,
              "need hid <= 256 divisible by n_head <= 16");
  VCG_REQUIRE(O > 0 && O <= kMaxOut, "need 1 <= output_size <= 256");
  return VCG_OK;
}

}  // namespace

VCG_API long long vcg_head_attn_saved_floats(int B, int T, int hid, int nh) {
  const long long T1 = T + 1;
  return (long long)B * (3 * T1 * hid + 2 * hid + nh * T1);
}

VCG_API int vcg_head_attn_fwd(int dtype, const void* Vout, const void* Lout, const float* Wq, const float* bq,
                              const float* Wk, const float* bk, const float* Wv, const float* bv, const float* Wp,
                              const float* bp, float* saved, long long saved_floats, float* logits, float* prob, int B,
                              int T, int hid, int nh, int O, float dropout_p, unsigned long long seed, hipStream_t s) {
  if (int rc = check_shapes(B, T, hid, nh, O)) return rc;
  VCG_REQUIRE(saved && saved_floats >= vcg_head_attn_saved_floats(B, T, hid, nh), "saved buffer too small");
  VCG_REQUIRE(Vout && Lout && Wq && bq && Wk && bk && Wv && bv && Wp && logits, "null operand");
  VCG_REQUIRE(dropout_p >= 0.f && dropout_p < 1.f, "dropout p must be in [0, 1)");
  const long long T1 = T + 1, bt = (long long)B * T1 * hid;
  float *X = saved, *K = X + bt, *V = K + bt, *q0 = V + bt, *y0 = q0 + (long long)B * hid,
        *P = y0 + (long long)B * hid;
  const size_t lds = (size_t)(3 * T1 * hid + 2 * hid + nh * T1) * sizeof(float);
  if (dtype == VCG_BF16)
    hipLaunchKernelGGL(head_attn_fwd_kernel<bf16_t>, dim3(B), dim3(256), lds, s, (const bf16_t*)Vout,
                       (const bf16_t*)Lout, Wq, bq, Wk, bk, Wv, bv, Wp, bp, X, K, V, q0, P, y0, logits, prob, T, hid,
                       nh, O, dropout_p, seed);
  else
    hipLaunchKernelGGL(head_attn_fwd_kernel<float>, dim3(B), dim3(256), lds, s, (const float*)Vout,
                       (const float*)Lout, Wq, bq, Wk, bk, Wv, bv, Wp, bp, X, K, V, q0, P, y0, logits, prob, T, hid,
                       nh, O, dropout_p, seed);
  VCG_LAUNCH_CHECK();
  return VCG_OK;
}

VCG_API long long vcg_head_attn_bwd_ws_floats(int B, int T, int hid) {
  return (long long)B * (2 * (long long)(T + 1) * hid + hid);
}

VCG_API int vcg_head_attn_bwd(int dtype, const float* saved, const float* Wq, const float* Wk, const float* Wv,
                              const float* Wp, const float* dlogits, void* dVout, void* dLout, float* dWq, float* dbq,
                              float* dWk, float* dbk, float* dWv, float* dbv, float* dWp, float* dbp, float* ws,
                              long long ws_floats, int B, int T, int hid, int nh, int O, float dropout_p,
                              unsigned long long seed, int relu_mask, hipStream_t s) {
  if (int rc = check_shapes(B, T, hid, nh, O)) return rc;
  VCG_REQUIRE(ws && ws_floats >= vcg_head_attn_bwd_ws_floats(B, T, hid), "workspace too small");
  VCG_REQUIRE(saved && Wq && Wk && Wv && Wp && dlogits && dVout && dLout, "null operand");
  VCG_REQUIRE(dropout_p >= 0.f && dropout_p < 1.f, "dropout p must be in [0, 1)");
  const long long T1 = T + 1, bt = (long long)B * T1 * hid;
  const float *X = saved, *K = X + bt, *V = K + bt, *q0 = V + bt, *y0 = q0 + (long long)B * hid,
              *P = y0 + (long long)B * hid;
  float *dK = ws, *dV = dK + bt, *dq0 = dV + bt;
  const size_t lds = (size_t)(2 * T1 * hid + 2 * hid + 2 * nh * T1) * sizeof(float);
  if (dtype == VCG_BF16)
    hipLaunchKernelGGL(head_attn_bwd_kernel<bf16_t>, dim3(B), dim3(256), lds, s, X, K, V, q0, P, Wq, Wk, Wv, Wp,
                       dlogits, dK, dV, dq0, (bf16_t*)dVout, (bf16_t*)dLout, T, hid, nh, O, dropout_p, seed,
                       relu_mask);
  else
    hipLaunchKernelGGL(head_attn_bwd_kernel<float>, dim3(B), dim3(256), lds, s, X, K, V, q0, P, Wq, Wk, Wv, Wp,
                       dlogits, dK, dV, dq0, (float*)dVout, (float*)dLout, T, hid, nh, O, dropout_p, seed, relu_mask);
  VCG_LAUNCH_CHECK();
  const int R = (int)(B * T1);
  // key / value: dW = dK^T X over all B*(T+1) tokens; query: token 0 only; proj: dlogits^T y0
  if (int rc = colgemm(dK, hid, X, hid, dWk, R, hid, hid, s)) return rc;
  if (int rc = colgemm(dK, hid, nullptr, 0, dbk, R, hid, 1, s)) return rc;
  if (int rc = colgemm(dV, hid, X, hid, dWv, R, hid, hid, s)) return rc;
  if (int rc = colgemm(dV, hid, nullptr, 0, dbv, R, hid, 1, s)) return rc;
  if (int rc = colgemm(dq0, hid, X, T1 * hid, dWq, B, hid, hid, s)) return rc;
  if (int rc = colgemm(dq0, hid, nullptr, 0, dbq, B, hid, 1, s)) return rc;
  if (int rc = colgemm(dlogits, O, y0, hid, dWp, B, O, hid, s)) return rc;
  if (int rc = colgemm(dlogits, O, nullptr, 0, dbp, B, O, 1, s)) return rc;
  return VCG_OK;
}
