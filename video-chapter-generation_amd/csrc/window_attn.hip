// Window transformer over per-clip fusion embeddings: StackedVideoChapterAttention, inference
// (reference model/fusion/stacked_window_self_attention.py:1-223, used by two_stream_window.TwoStream
// build_chapter_head :331-351 and forward :439-444 with hidden_size 128, 16 heads, window w -> S = 2w+1 clips).
//
//   for each of the 6 VideoChapterBlocks (:100-145):
//     N = LN_attn(X) ; N += pos(s)                         pos(s) = W_pe * (s - S/2) / (S/2 + 1e-6) + b_pe (:48-52,:69-72)
//     Q,K,V = N W^T + b ; P = softmax(Q K^T / sqrt(hd) + window_pos_bias[h, j]) ; X += (P V) W_o^T + b_o  (:74-95)
//     X += FFN(LN_ffn(X))     FFN = Linear(H,2H) GELU Linear(2H,4H) GELU Linear(4H,2H) GELU Linear(2H,H)  (:112-124)
//   X = LN_final(X) ; x = X[S/2] ; classifier chain (Linear LN GELU) x4 -> Linear(H/4, 2) ; softmax   (:170-223)
// Dropout is inactive (eval); LayerNorm eps 1e-5, GELU = erf form (torch defaults).
//
// The whole window stack is tiny (S <= 16 clips x H <= 256) and launch-bound, so ONE workgroup per window
// runs all 6 layers + the classifier with the residual stream and every activation resident in LDS
// (8 S*H floats <= 64 KB): one launch for the batch instead of ~150 small GEMM / LN launches. Weights are
// packed once per weight version by the host as W^T ([in][out], f32), so the threads of a workgroup read
// one weight row per k-step as consecutive 4-byte words (coalesced, L2-resident across windows).
#include "common.h"
#include "igemm.h"

using namespace vcg;

namespace {

constexpr int kThreads = 256;
constexpr int kMaxS = 16;
constexpr int kMaxSH = 2048;  // LDS: 8 * S * H floats <= 64 KB
constexpr int kLayers = 6;

// out[s][n] = act(sum_k in[s][k] * WT[k][n] + b[n]) (+ out[s][n] when ACC); in / out in LDS.
template <bool ACC>
__device__ void lin(const float* in, int S, int K, const float* __restrict__ WT, const float* __restrict__ b, int N,
                    float* out, bool gelu) {
  for (int n = threadIdx.x; n < N; n += kThreads) {
    float acc[kMaxS];
#pragma unroll
    for (int s = 0; s < kMaxS; ++s) acc[s] = 0.f;
    for (int k = 0; k < K; ++k) {
      const float w = WT[(long long)k * N + n];
#pragma unroll
      for (int s = 0; s < kMaxS; ++s)
        if (s < S) acc[s] = fmaf(in[s * K + k], w, acc[s]);
    }
    const float bn = b[n];
#pragma unroll
    for (int s = 0; s < kMaxS; ++s) {
      if (s < S) {
        float v = acc[s] + bn;
        if (gelu) v = gelu_erf(v);
        out[s * N + n] = ACC ? out[s * N + n] + v : v;
      }
    }
  }
  __syncthreads();
}

// out[s] = LN(in[s]) * g + b over D features (one wave per row, two-pass mean / variance like torch).
__device__ void layer_norm(const float* in, int S, int D, const float* __restrict__ g, const float* __restrict__ b,
                           float* out, bool gelu) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  for (int s = wave; s < S; s += kThreads / 64) {
    const float* x = in + s * D;
    float sum = 0.f;
    for (int d = lane; d < D; d += 64) sum += x[d];
    sum = warp_sum(sum);
    const float mean = sum / (float)D;
    float var = 0.f;
    for (int d = lane; d < D; d += 64) {
      const float t = x[d] - mean;
      var = fmaf(t, t, var);
    }
    var = warp_sum(var) / (float)D;
    const float rstd = rsqrtf(var + 1e-5f);
    for (int d = lane; d < D; d += 64) {
      float v = (x[d] - mean) * rstd * g[d] + b[d];
      if (gelu) v = gelu_erf(v);
      out[s * D + d] = v;
    }
  }
  __syncthreads();
}

__global__ void __launch_bounds__(kThreads) window_attn_fwd_kernel(const float* __restrict__ emb,
                                                                   const float* __restrict__ W, float* __restrict__ logits,
                                                                   float* __restrict__ prob, int S, int H, int nh, int P) {
  extern __shared__ float sm[];
  const int SH = S * H, hd = H / nh, mid = S / 2, tid = threadIdx.x;
  float* X = sm;            // residual stream [S][H]
  float* Nn = X + SH;       // normed input / attention context / FFN output [S][H]
  float* T1 = Nn + SH;      // Q K V [S][3H] / FFN hidden [S][4H]
  float* T2 = T1 + 4 * SH;  // FFN hidden [S][2H]
  const float* src = emb + (long long)blockIdx.x * SH;
  for (int i = tid; i < SH; i += kThreads) X[i] = src[i];
  __syncthreads();
  const float pden = (float)((double)mid + 1e-6);
  const float qscale = 1.f / sqrtf((float)hd);
  const float* w = W;
  for (int l = 0; l < kLayers; ++l) {
    const float *ln_g = w, *ln_b = w + H;
    const float* qkvT = ln_b + H;           // [H][3H]
    const float* qkvb = qkvT + 3 * H * H;   // [3H]
    const float* oT = qkvb + 3 * H;         // [H][H]
    const float* ob = oT + H * H;
    const float* pe_w = ob + H;
    const float* pe_b = pe_w + H;
    const float* wpb = pe_b + H;            // [nh][P]
    const float* f_g = wpb + nh * P;
    const float* f_b = f_g + H;
    const float* f0T = f_b + H;             // [H][2H]
    const float* f0b = f0T + 2 * H * H;
    const float* f1T = f0b + 2 * H;         // [2H][4H]
    const float* f1b = f1T + 8 * H * H;
    const float* f2T = f1b + 4 * H;         // [4H][2H]
    const float* f2b = f2T + 8 * H * H;
    const float* f3T = f2b + 2 * H;         // [2H][H]
    const float* f3b = f3T + 2 * H * H;
    w = f3b + H;

    layer_norm(X, S, H, ln_g, ln_b, Nn, false);
    for (int i = tid; i < SH; i += kThreads) {
      const int s = i / H, d = i - s * H;
      Nn[i] += fmaf(pe_w[d], (float)(s - mid) / pden, pe_b[d]);
    }
    __syncthreads();
    lin<false>(Nn, S, H, qkvT, qkvb, 3 * H, T1, false);  // T1[s] = [q | k | v]
    // one thread per (head, query row): scores over the S keys in registers, softmax, context -> Nn
    for (int t = tid; t < nh * S; t += kThreads) {
      const int h = t / S, i = t - h * S;
      const float* q = T1 + i * 3 * H + h * hd;
      float sc[kMaxS], mx = -INFINITY;
#pragma unroll
      for (int j = 0; j < kMaxS; ++j) {
        if (j < S) {
          const float* k = T1 + j * 3 * H + H + h * hd;
          float a = 0.f;
          for (int d = 0; d < hd; ++d) a = fmaf(q[d], k[d], a);
          sc[j] = a * qscale + wpb[h * P + j];
          mx = fmaxf(mx, sc[j]);
        }
      }
      float den = 0.f;
#pragma unroll
      for (int j = 0; j < kMaxS; ++j)
        if (j < S) {
          sc[j] = expf(sc[j] - mx);
          den += sc[j];
        }
      const float inv = 1.f / den;
      for (int d = 0; d < hd; ++d) {
        float a = 0.f;
#pragma unroll
        for (int j = 0; j < kMaxS; ++j)
          if (j < S) a = fmaf(sc[j], T1[j * 3 * H + 2 * H + h * hd + d], a);
        Nn[i * H + h * hd + d] = a * inv;
      }
    }
    __syncthreads();
    lin<true>(Nn, S, H, oT, ob, H, X, false);  // X += out_proj(ctx)
    layer_norm(X, S, H, f_g, f_b, Nn, false);
    lin<false>(Nn, S, H, f0T, f0b, 2 * H, T2, true);
    lin<false>(T2, S, 2 * H, f1T, f1b, 4 * H, T1, true);
    lin<false>(T1, S, 4 * H, f2T, f2b, 2 * H, T2, true);
    lin<true>(T2, S, 2 * H, f3T, f3b, H, X, false);  // X += FFN
  }
  // final LayerNorm of the middle (target) clip only, then the classifier on that one row
  const float *fin_g = w, *fin_b = w + H;
  w = fin_b + H;
  layer_norm(X + mid * H, 1, H, fin_g, fin_b, Nn, false);
  float* a = Nn;
  float* t = T1;
  const int dims[5] = {H, H, H, H / 2, H / 4};
  for (int c = 0; c < 4; ++c) {
    const int K = dims[c], N = dims[c + 1];
    const float* cT = w;
    const float* cb = cT + K * N;
    const float* lg = cb + N;
    const float* lb = lg + N;
    w = lb + N;
    lin<false>(a, 1, K, cT, cb, N, t, false);
    layer_norm(t, 1, N, lg, lb, a, true);  // LN then GELU
  }
  const float* cT = w;
  const float* cb = cT + (H / 4) * 2;
  lin<false>(a, 1, H / 4, cT, cb, 2, t, false);
  if (tid == 0) {
    const float l0 = t[0], l1 = t[1], m = fmaxf(l0, l1);
    const float e0 = expf(l0 - m), e1 = expf(l1 - m), inv = 1.f / (e0 + e1);
    logits[2 * blockIdx.x] = l0;
    logits[2 * blockIdx.x + 1] = l1;
    if (prob) {
      prob[2 * blockIdx.x] = e0 * inv;
      prob[2 * blockIdx.x + 1] = e1 * inv;
    }
  }
}

// LayerNorm + activation over rows of a f32 matrix (the Linear -> LayerNorm -> ReLU chains of the window
// ChapterHead, two_stream_window.py:145-176): one wave per row, two-pass statistics, act 0 / ACT_RELU / ACT_GELU.
__global__ void __launch_bounds__(kThreads) ln_act_kernel(const float* __restrict__ x, const float* __restrict__ g,
                                                          const float* __restrict__ b, float* __restrict__ out, int rows,
                                                          int D, float eps, int act) {
  const int lane = threadIdx.x & 63;
  const int row = blockIdx.x * (kThreads / 64) + (threadIdx.x >> 6);
  if (row >= rows) return;
  const float* xr = x + (long long)row * D;
  float* o = out + (long long)row * D;
  float sum = 0.f;
  for (int d = lane; d < D; d += 64) sum += xr[d];
  const float mean = warp_sum(sum) / (float)D;
  float var = 0.f;
  for (int d = lane; d < D; d += 64) {
    const float t = xr[d] - mean;
    var = fmaf(t, t, var);
  }
  const float rstd = rsqrtf(warp_sum(var) / (float)D + eps);
  for (int d = lane; d < D; d += 64) {
    float v = (xr[d] - mean) * rstd * g[d] + b[d];
    if (act == ACT_RELU) v = fmaxf(v, 0.f);
    else if (act == ACT_GELU) v = gelu_erf(v);
    o[d] = v;
  }
}

}  // namespace

// Packed f32 weight floats (layout documented in include/vcg_hip.h and vcg_hip/window.py pack_window_weights).
VCG_API long long vcg_window_attn_weight_floats(int H, int nh, int P) {
  const long long h = H;
  const long long layer = 2 * h + 3 * h * h + 3 * h + h * h + h + 2 * h + (long long)nh * P + 2 * h + 2 * h * h + 2 * h +
                          8 * h * h + 4 * h + 8 * h * h + 2 * h + 2 * h * h + h;
  long long cls = 0;
  const long long dims[5] = {h, h, h, h / 2, h / 4};
  for (int c = 0; c < 4; ++c) cls += dims[c] * dims[c + 1] + 3 * dims[c + 1];
  cls += (h / 4) * 2 + 2;
  return kLayers * layer + 2 * h + cls;
}

VCG_API int vcg_window_attn_fwd(const float* emb, const float* weights, long long weight_floats, float* logits,
                                float* prob, int B, int S, int H, int nh, int P, hipStream_t s) {
  VCG_REQUIRE(B >= 0 && S >= 1 && S <= kMaxS, "window length S must be in [1, 16]");
  VCG_REQUIRE(H >= 4 && H % 4 == 0 && nh >= 1 && H % nh == 0, "hidden size must be a multiple of 4 and of heads");
  VCG_REQUIRE((long long)S * H <= kMaxSH, "S * hidden must be <= 2048 (LDS-resident window)");
  VCG_REQUIRE(P >= S, "window_pos_bias length must cover the window");
  VCG_REQUIRE(weight_floats >= vcg_window_attn_weight_floats(H, nh, P), "packed weight buffer too small");
  VCG_REQUIRE(emb && weights && logits, "null operand");
  if (B == 0) return VCG_OK;
  const size_t lds = (size_t)8 * S * H * sizeof(float);
  hipLaunchKernelGGL(window_attn_fwd_kernel, dim3(B), dim3(kThreads), lds, s, emb, weights, logits, prob, S, H, nh,
                     P);
  VCG_LAUNCH_CHECK();
  return VCG_OK;
}

VCG_API int vcg_ln_act_fwd(const float* x, const float* gamma, const float* beta, float* out, int rows, int D,
                           float eps, int act, hipStream_t s) {
  VCG_REQUIRE(rows >= 0 && D >= 1, "bad shape");
  VCG_REQUIRE(act == 0 || act == ACT_RELU || act == ACT_GELU, "act must be none, relu or gelu");
  VCG_REQUIRE(x && gamma && beta && out, "null operand");
  if (rows == 0) return VCG_OK;
  constexpr int rpb = kThreads / 64;
  hipLaunchKernelGGL(ln_act_kernel, dim3((rows + rpb - 1) / rpb), dim3(kThreads), 0, s, x, gamma, beta, out, rows, D,
                     eps, act);
  VCG_LAUNCH_CHECK();
  return VCG_OK;
}
