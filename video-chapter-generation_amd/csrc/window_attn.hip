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
constexpr int kMaxSH = 2048;  // LDS: 8 * rows * H floats <= 64 KB
constexpr int kLayers = 6;

// out[s][n] = act(sum_k in[s][k] * WT[k][n] + b[n]) (+ out[s][n] when ACC); in / out in LDS. A thread owns
// whole columns and keeps up to 8 weight loads in flight (L2 / MALL latency bound). (Splitting K over idle
// threads for the narrow layers, with an LDS reduction, measured 1.7x slower.)
template <bool ACC>
__device__ void lin(const float* in, int S, int K, const float* __restrict__ WT, const float* __restrict__ b, int N,
                    float* out, bool gelu) {
  for (int n = threadIdx.x; n < N; n += kThreads) {
    float acc[kMaxS];
#pragma unroll
    for (int s = 0; s < kMaxS; ++s) acc[s] = 0.f;
#pragma unroll 8
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
                                                                   float* __restrict__ prob, int B, int S, int G, int H,
                                                                   int nh, int P) {
  // G windows per workgroup (R = G * S rows): every weight row read from L2 feeds all R rows; attention,
  // position encoding and the target-clip pick stay per window.
  extern __shared__ float sm[];
  const int w0 = blockIdx.x * G, g_n = min(G, B - w0);
  const int R = g_n * S, SH = R * H, hd = H / nh, mid = S / 2, tid = threadIdx.x;
  float* X = sm;            // residual stream [R][H]
  float* Nn = X + SH;       // normed input / attention context / FFN output [R][H]
  float* T1 = Nn + SH;      // Q K V [R][3H] / FFN hidden [R][4H]
  float* T2 = T1 + 4 * SH;  // FFN hidden [R][2H]
  const float* src = emb + (long long)w0 * S * H;
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

    layer_norm(X, R, H, ln_g, ln_b, Nn, false);
    for (int i = tid; i < SH; i += kThreads) {
      const int r = i / H, d = i - r * H, s = r % S;
      Nn[i] += fmaf(pe_w[d], (float)(s - mid) / pden, pe_b[d]);
    }
    __syncthreads();
    lin<false>(Nn, R, H, qkvT, qkvb, 3 * H, T1, false);  // T1[r] = [q | k | v]
    // one thread per (head, query row): scores over its window's S keys in registers, softmax, context -> Nn
    for (int t = tid; t < nh * R; t += kThreads) {
      const int h = t / R, i = t - h * R, kb = (i / S) * S;  // kb: first row of this query's window
      const float* q = T1 + i * 3 * H + h * hd;
      float sc[kMaxS], mx = -INFINITY;
#pragma unroll
      for (int j = 0; j < kMaxS; ++j) {
        if (j < S) {
          const float* k = T1 + (kb + j) * 3 * H + H + h * hd;
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
          if (j < S) a = fmaf(sc[j], T1[(kb + j) * 3 * H + 2 * H + h * hd + d], a);
        Nn[i * H + h * hd + d] = a * inv;
      }
    }
    __syncthreads();
    lin<true>(Nn, R, H, oT, ob, H, X, false);  // X += out_proj(ctx)
    layer_norm(X, R, H, f_g, f_b, Nn, false);
    lin<false>(Nn, R, H, f0T, f0b, 2 * H, T2, true);
    lin<false>(T2, R, 2 * H, f1T, f1b, 4 * H, T1, true);
    lin<false>(T1, R, 4 * H, f2T, f2b, 2 * H, T2, true);
    lin<true>(T2, R, 2 * H, f3T, f3b, H, X, false);  // X += FFN
  }
  // final LayerNorm of each window's middle (target) clip only (gathered to rows 0..g_n-1 of T2), then the
  // classifier on those g_n rows
  for (int i = tid; i < g_n * H; i += kThreads) {
    const int g = i / H, d = i - g * H;
    T2[i] = X[(g * S + mid) * H + d];
  }
  __syncthreads();
  const float *fin_g = w, *fin_b = w + H;
  w = fin_b + H;
  layer_norm(T2, g_n, H, fin_g, fin_b, Nn, false);
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
    lin<false>(a, g_n, K, cT, cb, N, t, false);
    layer_norm(t, g_n, N, lg, lb, a, true);  // LN then GELU
  }
  const float* cT = w;
  const float* cb = cT + (H / 4) * 2;
  lin<false>(a, g_n, H / 4, cT, cb, 2, t, false);
  if (tid < g_n) {
    const float l0 = t[2 * tid], l1 = t[2 * tid + 1], m = fmaxf(l0, l1);
    const float e0 = expf(l0 - m), e1 = expf(l1 - m), inv = 1.f / (e0 + e1);
    const long long o = 2LL * (w0 + tid);
    logits[o] = l0;
    logits[o + 1] = l1;
    if (prob) {
      prob[o] = e0 * inv;
      prob[o + 1] = e1 * inv;
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

// CrossAttention of the window ChapterHead, head_type "cross_attn" (two_stream_window.py:11-91, used at :284-286):
//   l = LN_lang(lang_out) ; V = LN_vis(vision_out) + pe(t), pe(t) = W_pe * t / (T - 1) + b_pe
//   q = l Wq^T + bq ; K, V' = V Wk^T + bk, V Wv^T + bv ; 16 heads: a = softmax(q K^T / sqrt(hd)) ; y = (a V') Wo^T + bo
// One workgroup per clip window (T <= 16 frames, T*H <= 2048), all intermediates in LDS; weights packed as W^T.
__global__ void __launch_bounds__(kThreads) cross_attn_fwd_kernel(const float* __restrict__ lang,
                                                                  const float* __restrict__ vis,
                                                                  const float* __restrict__ W, float* __restrict__ out,
                                                                  int T, int H, int nh) {
  extern __shared__ float sm[];
  const int TH = T * H, hd = H / nh, tid = threadIdx.x, b = blockIdx.x;
  float* Xv = sm;          // vision rows [T][H]
  float* Nv = Xv + TH;     // normalised + position-encoded [T][H]
  float* KV = Nv + TH;     // [T][2H] = k | v
  float* sl = KV + 2 * TH; // lang [H] | normed lang [H] | q [H] | out [H]
  const float *ln_g = W, *ln_b = ln_g + H, *vn_g = ln_b + H, *vn_b = vn_g + H, *pe_w = vn_b + H, *pe_b = pe_w + H;
  const float *qT = pe_b + H, *qb = qT + H * H, *kvT = qb + H, *kvb = kvT + 2 * H * H, *oT = kvb + 2 * H;
  const float* ob = oT + H * H;
  for (int i = tid; i < TH; i += kThreads) Xv[i] = vis[(long long)b * TH + i];
  for (int i = tid; i < H; i += kThreads) sl[i] = lang[(long long)b * H + i];
  __syncthreads();
  layer_norm(Xv, T, H, vn_g, vn_b, Nv, false);
  layer_norm(sl, 1, H, ln_g, ln_b, sl + H, false);
  const float tden = (float)(T - 1);
  for (int i = tid; i < TH; i += kThreads) {
    const int t = i / H, d = i - t * H;
    Nv[i] += fmaf(pe_w[d], (float)t / tden, pe_b[d]);
  }
  __syncthreads();
  lin<false>(sl + H, 1, H, qT, qb, H, sl + 2 * H, false);
  lin<false>(Nv, T, H, kvT, kvb, 2 * H, KV, false);
  const float qscale = 1.f / sqrtf((float)hd);
  for (int h = tid; h < nh; h += kThreads) {  // one thread per head: T scores in registers
    const float* q = sl + 2 * H + h * hd;
    float sc[kMaxS], mx = -INFINITY;
#pragma unroll
    for (int j = 0; j < kMaxS; ++j) {
      if (j < T) {
        float a = 0.f;
        for (int d = 0; d < hd; ++d) a = fmaf(q[d], KV[j * 2 * H + h * hd + d], a);
        sc[j] = a * qscale;
        mx = fmaxf(mx, sc[j]);
      }
    }
    float den = 0.f;
#pragma unroll
    for (int j = 0; j < kMaxS; ++j)
      if (j < T) {
        sc[j] = expf(sc[j] - mx);
        den += sc[j];
      }
    const float inv = 1.f / den;
    for (int d = 0; d < hd; ++d) {
      float a = 0.f;
#pragma unroll
      for (int j = 0; j < kMaxS; ++j)
        if (j < T) a = fmaf(sc[j], KV[j * 2 * H + H + h * hd + d], a);
      sl[h * hd + d] = a * inv;  // context over the raw-lang slot (no longer needed)
    }
  }
  __syncthreads();
  lin<false>(sl, 1, H, oT, ob, H, sl + 3 * H, false);
  for (int i = tid; i < H; i += kThreads) out[(long long)b * H + i] = sl[3 * H + i];
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
  if (B == 0) return VCG_OK;  // (empty tensors may carry null pointers)
  VCG_REQUIRE(emb && weights && logits, "null operand");
  // as many windows per workgroup as fit the row budget (R = G * S <= 16 rows, R * H <= 2048 floats), but keep
  // at least one workgroup per CU when the batch is small
  int G = min(kMaxS / S, kMaxSH / (S * H));
  if (const char* e = getenv("VCG_WINDOW_G")) G = min(G, atoi(e));  // fixed G (tests, A/B in tools/bench_window.py)
  else
    while (G > 1 && (B + G - 1) / G < 1024) --G;  // measured (S = 5): G = 1 best at 512 windows, G = 3 at 4096
  if (G < 1) G = 1;
  const size_t lds = (size_t)8 * G * S * H * sizeof(float);
  hipLaunchKernelGGL(window_attn_fwd_kernel, dim3((B + G - 1) / G), dim3(kThreads), lds, s, emb, weights, logits,
                     prob, B, S, G, H, nh, P);
  VCG_LAUNCH_CHECK();
  return VCG_OK;
}

VCG_API int vcg_ln_act_fwd(const float* x, const float* gamma, const float* beta, float* out, int rows, int D,
                           float eps, int act, hipStream_t s) {
  VCG_REQUIRE(rows >= 0 && D >= 1, "bad shape");
  VCG_REQUIRE(act == 0 || act == ACT_RELU || act == ACT_GELU, "act must be none, relu or gelu");
  if (rows == 0) return VCG_OK;
  VCG_REQUIRE(x && gamma && beta && out, "null operand");
  constexpr int rpb = kThreads / 64;
  hipLaunchKernelGGL(ln_act_kernel, dim3((rows + rpb - 1) / rpb), dim3(kThreads), 0, s, x, gamma, beta, out, rows, D,
                     eps, act);
  VCG_LAUNCH_CHECK();
  return VCG_OK;
}

VCG_API long long vcg_cross_attn_weight_floats(int H) { return 6LL * H + 4LL * H * H + 4LL * H; }

VCG_API int vcg_cross_attn_fwd(const float* lang, const float* vis, const float* weights, long long weight_floats,
                               float* out, int B, int T, int H, int nh, hipStream_t s) {
  VCG_REQUIRE(B >= 0 && T >= 2 && T <= kMaxS, "frames per clip T must be in [2, 16]");
  VCG_REQUIRE(H >= 1 && nh >= 1 && H % nh == 0 && (long long)T * H <= kMaxSH, "bad hidden size / heads");
  VCG_REQUIRE(weight_floats >= vcg_cross_attn_weight_floats(H), "packed weight buffer too small");
  if (B == 0) return VCG_OK;
  VCG_REQUIRE(lang && vis && weights && out, "null operand");
  const size_t lds = (size_t)(4 * T * H + 4 * H) * sizeof(float);
  hipLaunchKernelGGL(cross_attn_fwd_kernel, dim3(B), dim3(kThreads), lds, s, lang, vis, weights, out, T, H, nh);
  VCG_LAUNCH_CHECK();
  return VCG_OK;
}

namespace {

// out = a * b elementwise (window ChapterHead "multiplication": vision_out * expanded_lang, :275-277)
__global__ void __launch_bounds__(kThreads) mul_kernel(const float4* __restrict__ a, const float4* __restrict__ b,
                                                       float4* __restrict__ out, long long n4) {
  for (long long i = blockIdx.x * (long long)kThreads + threadIdx.x; i < n4; i += (long long)gridDim.x * kThreads) {
    const float4 x = a[i], y = b[i];
    out[i] = make_float4(x.x * y.x, x.y * y.y, x.z * y.z, x.w * y.w);
  }
}

// out[b][r] = sum_i U[b][r][i] * x[b][i] + bias[r]: the second contraction of nn.Bilinear (window ChapterHead
// "bilinear", :271-273) after U = x2 A^T on the GEMM path; one wave per output.
__global__ void __launch_bounds__(kThreads) rowdot_kernel(const float* __restrict__ U, const float* __restrict__ x,
                                                          const float* __restrict__ bias, float* __restrict__ out,
                                                          int B, int R, int K) {
  const int lane = threadIdx.x & 63;
  const long long o = blockIdx.x * (long long)(kThreads / 64) + (threadIdx.x >> 6);
  if (o >= (long long)B * R) return;
  const int b = (int)(o / R), r = (int)(o - (long long)b * R);
  const float* u = U + o * K;
  const float* xb = x + (long long)b * K;
  float s = 0.f;
  for (int i = lane; i < K; i += 64) s = fmaf(u[i], xb[i], s);
  s = warp_sum(s);
  if (lane == 0) out[o] = s + (bias ? bias[r] : 0.f);
}

// backward of rowdot (nn.Bilinear's second contraction, training): dx[b][i] = sum_r dy[b][r] U[b][r][i] and
// dU[b][r][i] = dy[b][r] x[b][i]; one thread per (b, i): the r loop reads / writes U rows coalesced along i.
__global__ void __launch_bounds__(kThreads) rowdot_bwd_kernel(const float* __restrict__ U, const float* __restrict__ x,
                                                              const float* __restrict__ dy, float* __restrict__ dU,
                                                              float* __restrict__ dx, int B, int R, int K) {
  const int b = blockIdx.y;
  const int i = blockIdx.x * kThreads + threadIdx.x;
  if (i >= K) return;
  const float xi = x[(long long)b * K + i];
  const float* u = U + (long long)b * R * K + i;
  float* du = dU + (long long)b * R * K + i;
  const float* g = dy + (long long)b * R;
  float s = 0.f;
  for (int r = 0; r < R; ++r) {
    const float gr = g[r];
    if (dx) s = fmaf(gr, u[(long long)r * K], s);
    du[(long long)r * K] = gr * xi;
  }
  if (dx) dx[(long long)b * K + i] = s;
}

}  // namespace

VCG_API int vcg_rowdot_bwd(const float* U, const float* x, const float* dy, float* dU, float* dx, int B, int R, int K,
                           hipStream_t s) {
  VCG_REQUIRE(B >= 0 && R >= 1 && K >= 1, "bad shape");
  if (B == 0) return VCG_OK;
  VCG_REQUIRE(x && dy && dU && (U || !dx), "null operand");
  hipLaunchKernelGGL(rowdot_bwd_kernel, dim3((unsigned)((K + kThreads - 1) / kThreads), (unsigned)B), dim3(kThreads), 0,
                     s, U, x, dy, dU, dx, B, R, K);
  VCG_LAUNCH_CHECK();
  return VCG_OK;
}

VCG_API int vcg_mul_fwd(const float* a, const float* b, float* out, long long n, hipStream_t s) {
  VCG_REQUIRE(n >= 0 && n % 4 == 0, "n must be a multiple of 4");
  if (n == 0) return VCG_OK;
  VCG_REQUIRE(a && b && out, "null operand");
  const long long n4 = n / 4;
  const int grid = (int)std::min<long long>((n4 + kThreads - 1) / kThreads, 4096);
  hipLaunchKernelGGL(mul_kernel, dim3(grid), dim3(kThreads), 0, s, (const float4*)a, (const float4*)b, (float4*)out,
                     n4);
  VCG_LAUNCH_CHECK();
  return VCG_OK;
}

VCG_API int vcg_rowdot_fwd(const float* U, const float* x, const float* bias, float* out, int B, int R, int K,
                           hipStream_t s) {
  VCG_REQUIRE(B >= 0 && R >= 1 && K >= 1, "bad shape");
  if (B == 0) return VCG_OK;
  VCG_REQUIRE(U && x && out, "null operand");
  const long long rows = (long long)B * R, rpb = kThreads / 64;
  hipLaunchKernelGGL(rowdot_kernel, dim3((unsigned)((rows + rpb - 1) / rpb)), dim3(kThreads), 0, s, U, x, bias, out, B,
                     R, K);
  VCG_LAUNCH_CHECK();
  return VCG_OK;
}
