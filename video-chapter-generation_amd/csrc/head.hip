// Fusion head + loss kernels.
//
// ChapterHead (reference model/fusion/two_stream.py:51-95, head_type "mlp"):
//   lang_out = relu(lang_emb W_l^T)            [B,1,hid]   (no bias, line 60)
//   vision_out = relu(vision_emb W_v^T)        [B,T,hid]   (no bias, line 61)
//   fusion = cat([vision_out, lang_out], 1).view(B, -1)    (vision first, line 88)
//   logits = fusion W^T + b ; prob = softmax(logits, 1)     (two_stream.py:189)
// The two projections run on the MFMA engine (their relu is the GEMM epilogue, writing
// straight into the fusion buffer); this file holds the final Linear + softmax and its
// backward, and the cross-entropy of train_video_segment_point.py:165.
#include "common.h"

using namespace vcg;

namespace {

// fusion row b of length D = (T+1)*hid: vision rows first (Vout [B*T][hid]), then Lout [B][hid]
template <typename T>
__device__ __forceinline__ float fus(const T* Vout, const T* Lout, int b, int d, int TH, int hid) {
  return d < TH ? to_f<T>(Vout[(long long)b * TH + d]) : to_f<T>(Lout[(long long)b * hid + d - TH]);
}

template <typename T>
__global__ void head_mlp_fwd_kernel(const T* __restrict__ Vout, const T* __restrict__ Lout, const float* __restrict__ W,
                                    const float* __restrict__ bias, float* __restrict__ logits,
                                    float* __restrict__ prob, int Tn, int hid, int O) {
  const int b = blockIdx.x;
  const int TH = Tn * hid, D = TH + hid;
  __shared__ float red[16];
  __shared__ float lg[16];
  for (int o = 0; o < O; ++o) {
    float s = 0.f;
    for (int d = threadIdx.x; d < D; d += blockDim.x) s += fus(Vout, Lout, b, d, TH, hid) * W[(long long)o * D + d];
    s = block_sum(s, red);
    if (threadIdx.x == 0) lg[o] = s + (bias ? bias[o] : 0.f);
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    float mx = -INFINITY;
    for (int o = 0; o < O; ++o) mx = fmaxf(mx, lg[o]);
    float sum = 0.f;
    for (int o = 0; o < O; ++o) sum += expf(lg[o] - mx);
    for (int o = 0; o < O; ++o) {
      logits[b * O + o] = lg[o];
      if (prob) prob[b * O + o] = expf(lg[o] - mx) / sum;
    }
  }
}

// dF = relu'(F) * (dlogits W), split back into dVout / dLout (the relu is the projection epilogue's)
template <typename T>
__global__ void head_mlp_bwd_dF_kernel(const T* __restrict__ Vout, const T* __restrict__ Lout,
                                       const float* __restrict__ W, const float* __restrict__ dlogits,
                                       T* __restrict__ dV, T* __restrict__ dL, int B, int Tn, int hid, int O,
                                       int relu_mask) {
  const int TH = Tn * hid, D = TH + hid;
  const long long total = (long long)B * D;
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < total; i += (long long)gridDim.x * blockDim.x) {
    const int b = (int)(i / D), d = (int)(i - (long long)b * D);
    float s = 0.f;
    for (int o = 0; o < O; ++o) s += dlogits[b * O + o] * W[(long long)o * D + d];
    const float f = fus(Vout, Lout, b, d, TH, hid);
    const T v = from_f<T>((!relu_mask || f > 0.f) ? s : 0.f);
    if (d < TH) dV[(long long)b * TH + d] = v;
    else dL[(long long)b * hid + d - TH] = v;
  }
}

template <typename T>
__global__ void head_mlp_bwd_dW_kernel(const T* __restrict__ Vout, const T* __restrict__ Lout,
                                       const float* __restrict__ dlogits, float* __restrict__ dW,
                                       float* __restrict__ dbias, int B, int Tn, int hid, int O) {
  const int TH = Tn * hid, D = TH + hid;
  const int d = blockIdx.x * blockDim.x + threadIdx.x;
  if (d < D) {
    for (int o = 0; o < O; ++o) {
      float s = 0.f;
      for (int b = 0; b < B; ++b) s += dlogits[b * O + o] * fus(Vout, Lout, b, d, TH, hid);
      dW[(long long)o * D + d] += s;
    }
  }
  if (blockIdx.x == 0 && threadIdx.x < O && dbias) {
    float s = 0.f;
    for (int b = 0; b < B; ++b) s += dlogits[b * O + threadIdx.x];
    dbias[threadIdx.x] += s;
  }
}

// mean cross-entropy over B rows of C-way logits
__global__ void ce_fwd_kernel(const float* __restrict__ logits, const long long* __restrict__ labels,
                              float* __restrict__ loss, int B, int C) {
  __shared__ float red[16];
  float s = 0.f;
  for (int b = threadIdx.x; b < B; b += blockDim.x) {
    float mx = -INFINITY;
    for (int c = 0; c < C; ++c) mx = fmaxf(mx, logits[b * C + c]);
    float se = 0.f;
    for (int c = 0; c < C; ++c) se += expf(logits[b * C + c] - mx);
    s += (logf(se) + mx) - logits[b * C + (int)labels[b]];
  }
  s = block_sum(s, red);
  if (threadIdx.x == 0) loss[0] = s / (float)B;
}

__global__ void ce_bwd_kernel(const float* __restrict__ logits, const long long* __restrict__ labels,
                              const float* __restrict__ dloss, float* __restrict__ dlogits, int B, int C) {
  const int b = blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= B) return;
  const float g = (dloss ? dloss[0] : 1.f) / (float)B;
  float mx = -INFINITY;
  for (int c = 0; c < C; ++c) mx = fmaxf(mx, logits[b * C + c]);
  float se = 0.f;
  for (int c = 0; c < C; ++c) se += expf(logits[b * C + c] - mx);
  for (int c = 0; c < C; ++c) {
    const float pr = expf(logits[b * C + c] - mx) / se;
    dlogits[b * C + c] = g * (pr - (c == (int)labels[b] ? 1.f : 0.f));
  }
}

}  // namespace

VCG_API int vcg_head_mlp_fwd(int dtype, const void* Vout, const void* Lout, const float* W, const float* bias,
                             float* logits, float* prob, int B, int T, int hid, int O, hipStream_t s) {
  VCG_REQUIRE(O <= 16, "too many outputs");
  if (dtype == VCG_BF16)
    hipLaunchKernelGGL(head_mlp_fwd_kernel<bf16_t>, dim3(B), dim3(256), 0, s, (const bf16_t*)Vout, (const bf16_t*)Lout,
                       W, bias, logits, prob, T, hid, O);
  else
    hipLaunchKernelGGL(head_mlp_fwd_kernel<float>, dim3(B), dim3(256), 0, s, (const float*)Vout, (const float*)Lout, W,
                       bias, logits, prob, T, hid, O);
  VCG_LAUNCH_CHECK();
  return VCG_OK;
}

VCG_API int vcg_head_mlp_bwd(int dtype, const void* Vout, const void* Lout, const float* W, const float* dlogits,
                             void* dV, void* dL, float* dW, float* dbias, int B, int T, int hid, int O, int relu_mask,
                             hipStream_t s) {
  const int D = (T + 1) * hid;
  const long long tot = (long long)B * D;
  const int g = (int)((tot + 255) / 256 > 4096 ? 4096 : (tot + 255) / 256);
  if (dtype == VCG_BF16) {
    hipLaunchKernelGGL(head_mlp_bwd_dF_kernel<bf16_t>, dim3(g), dim3(256), 0, s, (const bf16_t*)Vout,
                       (const bf16_t*)Lout, W, dlogits, (bf16_t*)dV, (bf16_t*)dL, B, T, hid, O, relu_mask);
    if (dW)
      hipLaunchKernelGGL(head_mlp_bwd_dW_kernel<bf16_t>, dim3((D + 255) / 256), dim3(256), 0, s, (const bf16_t*)Vout,
                         (const bf16_t*)Lout, dlogits, dW, dbias, B, T, hid, O);
  } else {
    hipLaunchKernelGGL(head_mlp_bwd_dF_kernel<float>, dim3(g), dim3(256), 0, s, (const float*)Vout, (const float*)Lout,
                       W, dlogits, (float*)dV, (float*)dL, B, T, hid, O, relu_mask);
    if (dW)
      hipLaunchKernelGGL(head_mlp_bwd_dW_kernel<float>, dim3((D + 255) / 256), dim3(256), 0, s, (const float*)Vout,
                         (const float*)Lout, dlogits, dW, dbias, B, T, hid, O);
  }
  VCG_LAUNCH_CHECK();
  return VCG_OK;
}

VCG_API int vcg_cross_entropy_fwd(const float* logits, const long long* labels, float* loss, int B, int C,
                                  hipStream_t s) {
  hipLaunchKernelGGL(ce_fwd_kernel, dim3(1), dim3(256), 0, s, logits, labels, loss, B, C);
  VCG_LAUNCH_CHECK();
  return VCG_OK;
}

VCG_API int vcg_cross_entropy_bwd(const float* logits, const long long* labels, const float* dloss, float* dlogits,
                                  int B, int C, hipStream_t s) {
  hipLaunchKernelGGL(ce_bwd_kernel, dim3((B + 255) / 256), dim3(256), 0, s, logits, labels, dloss, dlogits, B, C);
  VCG_LAUNCH_CHECK();
  return VCG_OK;
}
