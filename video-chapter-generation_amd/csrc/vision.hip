// Vision-trunk support kernels (NHWC activations, per-channel BatchNorm in fp32).
//
// BatchNorm2d semantics follow torch.nn.BatchNorm2d as used by torchvision ResNet-50
// (reference model/vision/resnet50_tsm.py:15): eps 1e-5, momentum 0.1, biased variance for
// normalisation, unbiased variance for the running-stat update. Batch-statistics eval mode
// reproduces test_video_segment_point.py:116-122.
#include "common.h"

using namespace vcg;

namespace {

template <typename T> struct V { static constexpr int N = 16 / sizeof(T); };

// ------------------------------------------------------------------ BN finalize
// stats: float2 [C][mtiles] of (mean, M2) per 128-row tile; merged with Chan's formula.
__global__ void bn_finalize_kernel(const float2* __restrict__ stats, int mtiles, int M, int tile_rows,
                                   const float* __restrict__ gamma, const float* __restrict__ beta,
                                   float* mean_out, float* invstd_out, float* scale_out, float* shift_out,
                                   float* running_mean, float* running_var, float momentum, float eps) {
  const int c = blockIdx.x;
  __shared__ double sn[256], sm[256], s2[256];
  double n = 0, mean = 0, m2 = 0;
  for (int t = threadIdx.x; t < mtiles; t += blockDim.x) {
    const float2 st = stats[(long long)c * mtiles + t];
    const double nb = (double)min(tile_rows, M - t * tile_rows);
    const double delta = (double)st.x - mean;
    const double nn = n + nb;
    mean += delta * nb / nn;
    m2 += (double)st.y + delta * delta * n * nb / nn;
    n = nn;
  }
  sn[threadIdx.x] = n; sm[threadIdx.x] = mean; s2[threadIdx.x] = m2;
  __syncthreads();
  for (int off = blockDim.x / 2; off > 0; off >>= 1) {
    if (threadIdx.x < off) {
      const double na = sn[threadIdx.x], nb = sn[threadIdx.x + off];
      const double nn = na + nb;
      if (nb > 0) {
        const double delta = sm[threadIdx.x + off] - sm[threadIdx.x];
        sm[threadIdx.x] += delta * nb / nn;
        s2[threadIdx.x] += s2[threadIdx.x + off] + delta * delta * na * nb / nn;
        sn[threadIdx.x] = nn;
      }
    }
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    const double N = sn[0], mu = sm[0];
    const double var = s2[0] / N;
    const float invstd = (float)(1.0 / sqrt(var + (double)eps));
    const float g = gamma ? gamma[c] : 1.f, b = beta ? beta[c] : 0.f;
    if (mean_out) mean_out[c] = (float)mu;
    if (invstd_out) invstd_out[c] = invstd;
    scale_out[c] = g * invstd;
    shift_out[c] = b - (float)mu * g * invstd;
    if (running_mean) {
      const double unbiased = N > 1 ? s2[0] / (N - 1) : var;
      running_mean[c] = (float)((1.0 - momentum) * running_mean[c] + momentum * mu);
      running_var[c] = (float)((1.0 - momentum) * running_var[c] + momentum * unbiased);
    }
  }
}

__global__ void bn_eval_params_kernel(const float* gamma, const float* beta, const float* rm, const float* rv,
                                      float eps, int C, float* mean_out, float* invstd_out, float* scale,
                                      float* shift) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= C) return;
  const float invstd = 1.f / sqrtf(rv[c] + eps);
  const float g = gamma ? gamma[c] : 1.f, b = beta ? beta[c] : 0.f;
  if (mean_out) mean_out[c] = rm[c];
  if (invstd_out) invstd_out[c] = invstd;
  scale[c] = g * invstd;
  shift[c] = b - rm[c] * g * invstd;
}

// ------------------------------------------------------------------ BN apply
// out = act(y*scale + shift + [res*rscale + rshift | res])
template <typename T>
__global__ void bn_apply_kernel(const T* __restrict__ y, const float* __restrict__ scale,
                                const float* __restrict__ shift, const T* __restrict__ res,
                                const float* __restrict__ rscale, const float* __restrict__ rshift, int relu,
                                T* __restrict__ out, long long total_vec, int C) {
  constexpr int VN = V<T>::N;
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < total_vec;
       i += (long long)gridDim.x * blockDim.x) {
    const long long e0 = i * VN;
    const int c0 = (int)(e0 % C);
    float v[VN];
    load16<T>(y + e0, v);
#pragma unroll
    for (int e = 0; e < VN; ++e) v[e] = v[e] * scale[c0 + e] + shift[c0 + e];
    if (res) {
      float r[VN];
      load16<T>(res + e0, r);
      if (rscale) {
#pragma unroll
        for (int e = 0; e < VN; ++e) v[e] += r[e] * rscale[c0 + e] + rshift[c0 + e];
      } else {
#pragma unroll
        for (int e = 0; e < VN; ++e) v[e] += r[e];
      }
    }
    if (relu) {
#pragma unroll
      for (int e = 0; e < VN; ++e) v[e] = fmaxf(v[e], 0.f);
    }
    store16<T>(out + e0, v);
  }
}

// ------------------------------------------------------------------ BN backward
// Partial per-channel sums of g and g*xhat, g = dout * [mask > 0] (mask optional).
// Block = 256 threads handles rows [r0, r0 + rows_per_block) for all channels.
template <typename T>
__global__ void bn_bwd_reduce_kernel(const T* __restrict__ dout, const T* __restrict__ mask,
                                     const T* __restrict__ y, const float* __restrict__ mean,
                                     const float* __restrict__ invstd, int P, int C, int rows_per_block,
                                     float* __restrict__ partial) {
  constexpr int VN = V<T>::N;
  extern __shared__ float sred[];  // [2][C]
  const int cpr = C / VN;          // column chunks per row
  for (int i = threadIdx.x; i < 2 * C; i += blockDim.x) sred[i] = 0.f;
  __syncthreads();
  const int r0 = blockIdx.x * rows_per_block;
  const int r1 = min(P, r0 + rows_per_block);
  if (cpr <= (int)blockDim.x) {
    const int rpp = blockDim.x / cpr;
    const int cc = (threadIdx.x % cpr) * VN;
    const int rr = threadIdx.x / cpr;
    float sg[VN], sgx[VN], mu[VN], is[VN];
#pragma unroll
    for (int e = 0; e < VN; ++e) { sg[e] = 0.f; sgx[e] = 0.f; mu[e] = mean[cc + e]; is[e] = invstd[cc + e]; }
    if (rr < rpp) {
      for (int r = r0 + rr; r < r1; r += rpp) {
        const long long o = (long long)r * C + cc;
        float d[VN], yv[VN];
        load16<T>(dout + o, d);
        load16<T>(y + o, yv);
        if (mask) {
          float m[VN];
          load16<T>(mask + o, m);
#pragma unroll
          for (int e = 0; e < VN; ++e) d[e] = m[e] > 0.f ? d[e] : 0.f;
        }
#pragma unroll
        for (int e = 0; e < VN; ++e) {
          sg[e] += d[e];
          sgx[e] += d[e] * (yv[e] - mu[e]) * is[e];
        }
      }
#pragma unroll
      for (int e = 0; e < VN; ++e) {
        atomicAdd(&sred[cc + e], sg[e]);
        atomicAdd(&sred[C + cc + e], sgx[e]);
      }
    }
  } else {
    for (int ch = threadIdx.x; ch < cpr; ch += blockDim.x) {
      const int cc = ch * VN;
      float sg[VN], sgx[VN];
#pragma unroll
      for (int e = 0; e < VN; ++e) { sg[e] = 0.f; sgx[e] = 0.f; }
      for (int r = r0; r < r1; ++r) {
        const long long o = (long long)r * C + cc;
        float d[VN], yv[VN];
        load16<T>(dout + o, d);
        load16<T>(y + o, yv);
        if (mask) {
          float m[VN];
          load16<T>(mask + o, m);
#pragma unroll
          for (int e = 0; e < VN; ++e) d[e] = m[e] > 0.f ? d[e] : 0.f;
        }
#pragma unroll
        for (int e = 0; e < VN; ++e) {
          sg[e] += d[e];
          sgx[e] += d[e] * (yv[e] - mean[cc + e]) * invstd[cc + e];
        }
      }
#pragma unroll
      for (int e = 0; e < VN; ++e) { sred[cc + e] = sg[e]; sred[C + cc + e] = sgx[e]; }
    }
  }
  __syncthreads();
  for (int i = threadIdx.x; i < 2 * C; i += blockDim.x) partial[(long long)blockIdx.x * 2 * C + i] = sred[i];
}

__global__ void bn_bwd_finalize_kernel(const float* __restrict__ partial, int nblocks, int C, float* sum_g,
                                       float* sum_gx, float* dgamma, float* dbeta, int accumulate) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= C) return;
  double a = 0, b = 0;
  for (int i = 0; i < nblocks; ++i) {
    a += partial[(long long)i * 2 * C + c];
    b += partial[(long long)i * 2 * C + C + c];
  }
  sum_g[c] = (float)a;
  sum_gx[c] = (float)b;
  if (dbeta) dbeta[c] = (accumulate ? dbeta[c] : 0.f) + (float)a;
  if (dgamma) dgamma[c] = (accumulate ? dgamma[c] : 0.f) + (float)b;
}

// dy = gamma*invstd*(g - sum_g/N - xhat*sum_gx/N)  (train / batch-stat mode)
// dy = gamma*invstd*g                              (running-stat mode, train_stats = 0)
// optionally gout = g (the masked upstream gradient, feeds the residual path)
template <typename T>
__global__ void bn_bwd_apply_kernel(const T* __restrict__ dout, const T* __restrict__ mask,
                                    const T* __restrict__ y, const float* __restrict__ mean,
                                    const float* __restrict__ invstd, const float* __restrict__ gamma,
                                    const float* __restrict__ sum_g, const float* __restrict__ sum_gx,
                                    float inv_count, int train_stats, T* __restrict__ dy, T* __restrict__ gout,
                                    long long total_vec, int C) {
  constexpr int VN = V<T>::N;
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < total_vec;
       i += (long long)gridDim.x * blockDim.x) {
    const long long e0 = i * VN;
    const int c0 = (int)(e0 % C);
    float d[VN], yv[VN];
    load16<T>(dout + e0, d);
    if (mask) {
      float m[VN];
      load16<T>(mask + e0, m);
#pragma unroll
      for (int e = 0; e < VN; ++e) d[e] = m[e] > 0.f ? d[e] : 0.f;
    }
    if (gout) store16<T>(gout + e0, d);
    load16<T>(y + e0, yv);
    float o[VN];
#pragma unroll
    for (int e = 0; e < VN; ++e) {
      const int c = c0 + e;
      const float k = (gamma ? gamma[c] : 1.f) * invstd[c];
      if (train_stats) {
        const float xh = (yv[e] - mean[c]) * invstd[c];
        o[e] = k * (d[e] - sum_g[c] * inv_count - xh * sum_gx[c] * inv_count);
      } else {
        o[e] = k * d[e];
      }
    }
    store16<T>(dy + e0, o);
  }
}

// ------------------------------------------------------------------ pooling
// max_pool2d(k=3, s=2, p=1) NHWC with argmax index (0..8, first max in (kh,kw) scan order)
template <typename T>
__global__ void maxpool_fwd_kernel(const T* __restrict__ x, T* __restrict__ y, uint8_t* __restrict__ idx, int N,
                                   int H, int W, int C, int OH, int OW) {
  const long long total = (long long)N * OH * OW * C;
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < total;
       i += (long long)gridDim.x * blockDim.x) {
    const int c = (int)(i % C);
    long long r = i / C;
    const int ow = (int)(r % OW); r /= OW;
    const int oh = (int)(r % OH);
    const int n = (int)(r / OH);
    float best = -INFINITY;
    int bi = 0;
    for (int kh = 0; kh < 3; ++kh) {
      const int ih = oh * 2 - 1 + kh;
      if (ih < 0 || ih >= H) continue;
      for (int kw = 0; kw < 3; ++kw) {
        const int iw = ow * 2 - 1 + kw;
        if (iw < 0 || iw >= W) continue;
        const float v = to_f<T>(x[(((long long)n * H + ih) * W + iw) * C + c]);
        if (v > best || isnan(v)) { best = v; bi = kh * 3 + kw; }
      }
    }
    y[i] = from_f<T>(best);
    idx[i] = (uint8_t)bi;
  }
}

template <typename T>
__global__ void maxpool_bwd_kernel(const T* __restrict__ dy, const uint8_t* __restrict__ idx, T* __restrict__ dx,
                                   int N, int H, int W, int C, int OH, int OW) {
  const long long total = (long long)N * H * W * C;
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < total;
       i += (long long)gridDim.x * blockDim.x) {
    const int c = (int)(i % C);
    long long r = i / C;
    const int iw = (int)(r % W); r /= W;
    const int ih = (int)(r % H);
    const int n = (int)(r / H);
    float acc = 0.f;
    // windows (oh, ow) with oh*2-1 <= ih <= oh*2+1
    const int oh_lo = max(0, (ih - 1 + 1) / 2 - ((ih - 1 + 1) % 2 != 0 ? 0 : 0));
    for (int oh = (ih) / 2 - 1; oh <= (ih + 1) / 2; ++oh) {
      if (oh < 0 || oh >= OH) continue;
      const int kh = ih - (oh * 2 - 1);
      if (kh < 0 || kh > 2) continue;
      for (int ow = iw / 2 - 1; ow <= (iw + 1) / 2; ++ow) {
        if (ow < 0 || ow >= OW) continue;
        const int kw = iw - (ow * 2 - 1);
        if (kw < 0 || kw > 2) continue;
        const long long o = (((long long)n * OH + oh) * OW + ow) * C + c;
        if (idx[o] == kh * 3 + kw) acc += to_f<T>(dy[o]);
      }
    }
    (void)oh_lo;
    dx[i] = from_f<T>(acc);
  }
}

// global average pool: x [N][HW][C] -> y [N][C] (fp32 out)
template <typename T>
__global__ void avgpool_fwd_kernel(const T* __restrict__ x, float* __restrict__ y, int HW, int C) {
  const int n = blockIdx.y;
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= C) return;
  float s = 0.f;
  const T* p = x + (long long)n * HW * C + c;
  for (int i = 0; i < HW; ++i) s += to_f<T>(p[(long long)i * C]);
  y[(long long)n * C + c] = s / (float)HW;
}

template <typename T>
__global__ void avgpool_bwd_kernel(const float* __restrict__ dy, T* __restrict__ dx, int HW, int C, long long total) {
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < total;
       i += (long long)gridDim.x * blockDim.x) {
    const int c = (int)(i % C);
    const long long n = i / ((long long)HW * C);
    dx[i] = from_f<T>(dy[n * C + c] / (float)HW);
  }
}

// ------------------------------------------------------------------ layouts
// frames [N][C][H][W] fp32 -> NHWC [N][H][W][Cpad] (zero padded channels); reference
// rearrange 'b t c h w -> (b t) c h w' (two_stream.py:183) is the identity on the N index.
template <typename T>
__global__ void frames_to_nhwc_kernel(const float* __restrict__ src, T* __restrict__ dst, int N, int C, int H, int W,
                                      int Cpad) {
  const long long total = (long long)N * H * W;
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < total;
       i += (long long)gridDim.x * blockDim.x) {
    const long long n = i / ((long long)H * W);
    const long long hw = i - n * H * W;
    T* d = dst + i * Cpad;
    for (int c = 0; c < Cpad; ++c) d[c] = from_f<T>(c < C ? src[(n * C + c) * H * W + hw] : 0.f);
  }
}

// OIHW fp32 -> [Cout][KH][KW][Cpad] (transposed = 0) or [Cin][KH][KW][Cout] (transposed = 1)
template <typename T>
__global__ void weight_prep_kernel(const float* __restrict__ w, T* __restrict__ out, int Cout, int Cin, int KH, int KW,
                                   int Cpad, int transposed) {
  const long long total = transposed ? (long long)Cin * KH * KW * Cout : (long long)Cout * KH * KW * Cpad;
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < total;
       i += (long long)gridDim.x * blockDim.x) {
    float v;
    if (!transposed) {
      const int ci = (int)(i % Cpad);
      long long r = i / Cpad;
      const int kw = (int)(r % KW); r /= KW;
      const int kh = (int)(r % KH);
      const int co = (int)(r / KH);
      v = ci < Cin ? w[(((long long)co * Cin + ci) * KH + kh) * KW + kw] : 0.f;
    } else {
      const int co = (int)(i % Cout);
      long long r = i / Cout;
      const int kw = (int)(r % KW); r /= KW;
      const int kh = (int)(r % KH);
      const int ci = (int)(r / KH);
      v = w[(((long long)co * Cin + ci) * KH + kh) * KW + kw];
    }
    out[i] = from_f<T>(v);
  }
}

template <typename TO>
__global__ void cast_kernel(const float* __restrict__ in, TO* __restrict__ out, long long n) {
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < n; i += (long long)gridDim.x * blockDim.x)
    out[i] = from_f<TO>(in[i]);
}
template <typename TI>
__global__ void to_f32_kernel(const TI* __restrict__ in, float* __restrict__ out, long long n) {
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < n; i += (long long)gridDim.x * blockDim.x)
    out[i] = to_f<TI>(in[i]);
}

// ------------------------------------------------------------------ temporal shift
// Reference TemporalShift.shift (ops/temporal_shift.py:33-51), NCHW view [n_batch][T][C][HW].
// direction 0: out[:, t, :f] = x[:, t+1, :f]; out[:, t, f:2f] = x[:, t-1, f:2f]; rest copied (zero fill).
// direction 1: the adjoint (gradient) of direction 0.
template <typename T>
__global__ void tsm_nchw_kernel(const T* __restrict__ x, T* __restrict__ y, long long n_batch, int Tn, int C,
                                long long HW, int fold, int direction) {
  const long long total = n_batch * Tn * C * HW;
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < total;
       i += (long long)gridDim.x * blockDim.x) {
    long long r = i / HW;
    const int c = (int)(r % C);
    r /= C;
    const int t = (int)(r % Tn);
    int dt = 0;
    if (c < fold) dt = direction == 0 ? 1 : -1;
    else if (c < 2 * fold) dt = direction == 0 ? -1 : 1;
    const int t2 = t + dt;
    T v = from_f<T>(0.f);
    if (t2 >= 0 && t2 < Tn) v = x[i + (long long)dt * C * HW];
    y[i] = v;
  }
}

// NHWC gradient combine for a TSM block input: dx = unshift(dshift) + other
template <typename T>
__global__ void tsm_unshift_add_kernel(const T* __restrict__ dshift, const T* __restrict__ other, T* __restrict__ dx,
                                       long long total_vec, int Tn, long long HWC, int C, int fold) {
  constexpr int VN = V<T>::N;
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < total_vec;
       i += (long long)gridDim.x * blockDim.x) {
    const long long e0 = i * VN;
    const int c = (int)(e0 % C);
    const long long nt = e0 / HWC;
    const int t = (int)(nt % Tn);
    int dt = 0;  // adjoint of the forward shift
    if (fold > 0) {
      if (c < fold) dt = -1;
      else if (c < 2 * fold) dt = 1;
    }
    const int t2 = t + dt;
    float a[VN];
    if (t2 >= 0 && t2 < Tn) load16<T>(dshift + e0 + (long long)dt * HWC, a);
    else {
#pragma unroll
      for (int e = 0; e < VN; ++e) a[e] = 0.f;
    }
    if (other) {
      float b[VN];
      load16<T>(other + e0, b);
#pragma unroll
      for (int e = 0; e < VN; ++e) a[e] += b[e];
    }
    store16<T>(dx + e0, a);
  }
}

inline int grid_for(long long n, int bs = 256) {
  long long g = (n + bs - 1) / bs;
  if (g > 8192) g = 8192;
  if (g < 1) g = 1;
  return (int)g;
}

}  // namespace

// ==================================================================== C ABI

VCG_API int vcg_bn_finalize(const float* stats, int mtiles, int M, int C, const float* gamma, const float* beta,
                            float* mean_out, float* invstd_out, float* scale_out, float* shift_out,
                            float* running_mean, float* running_var, float momentum, float eps, hipStream_t s) {
  VCG_REQUIRE(stats && scale_out && shift_out && M > 0, "bad arguments");
  hipLaunchKernelGGL(bn_finalize_kernel, dim3(C), dim3(256), 0, s, reinterpret_cast<const float2*>(stats), mtiles, M,
                     128, gamma, beta, mean_out, invstd_out, scale_out, shift_out, running_mean, running_var,
                     momentum, eps);
  VCG_LAUNCH_CHECK();
  return VCG_OK;
}

VCG_API int vcg_bn_eval_params(const float* gamma, const float* beta, const float* rm, const float* rv, float eps,
                               int C, float* mean_out, float* invstd_out, float* scale, float* shift, hipStream_t s) {
  hipLaunchKernelGGL(bn_eval_params_kernel, dim3((C + 255) / 256), dim3(256), 0, s, gamma, beta, rm, rv, eps, C,
                     mean_out, invstd_out, scale, shift);
  VCG_LAUNCH_CHECK();
  return VCG_OK;
}

VCG_API int vcg_bn_apply(int dtype, const void* y, const float* scale, const float* shift, const void* res,
                         const float* rscale, const float* rshift, int relu, void* out, long long P, int C,
                         hipStream_t s) {
  const int VN = dtype == VCG_BF16 ? 8 : 4;
  VCG_REQUIRE(C % VN == 0, "C must be a multiple of the vector width");
  const long long tv = P * C / VN;
  if (dtype == VCG_BF16)
    hipLaunchKernelGGL(bn_apply_kernel<bf16_t>, dim3(grid_for(tv)), dim3(256), 0, s, (const bf16_t*)y, scale, shift,
                       (const bf16_t*)res, rscale, rshift, relu, (bf16_t*)out, tv, C);
  else
    hipLaunchKernelGGL(bn_apply_kernel<float>, dim3(grid_for(tv)), dim3(256), 0, s, (const float*)y, scale, shift,
                       (const float*)res, rscale, rshift, relu, (float*)out, tv, C);
  VCG_LAUNCH_CHECK();
  return VCG_OK;
}

static int bn_bwd_blocks(long long P) {
  long long rows = (P + 2047) / 2048;
  if (rows < 16) rows = 16;
  return (int)((P + rows - 1) / rows);
}
static int bn_bwd_rows(long long P) { return (int)((P + bn_bwd_blocks(P) - 1) / bn_bwd_blocks(P)); }

VCG_API long long vcg_bn_bwd_ws_bytes(long long P, int C) { return (long long)bn_bwd_blocks(P) * 2 * C * 4 + 2 * C * 4; }

// Per-channel sum_g / sum_gx (and optional dgamma/dbeta accumulation into fp32 grads).
VCG_API int vcg_bn_bwd_reduce(int dtype, const void* dout, const void* mask, const void* y, const float* mean,
                              const float* invstd, long long P, int C, float* ws, long long ws_bytes, float* sum_g,
                              float* sum_gx, float* dgamma, float* dbeta, int accumulate, hipStream_t s) {
  const int VN = dtype == VCG_BF16 ? 8 : 4;
  VCG_REQUIRE(C % VN == 0, "C must be a multiple of the vector width");
  VCG_REQUIRE(ws_bytes >= vcg_bn_bwd_ws_bytes(P, C), "workspace too small");
  const int rows = bn_bwd_rows(P);
  const int nb = (int)((P + rows - 1) / rows);
  const size_t shm = 2 * C * sizeof(float);
  if (dtype == VCG_BF16)
    hipLaunchKernelGGL(bn_bwd_reduce_kernel<bf16_t>, dim3(nb), dim3(256), shm, s, (const bf16_t*)dout,
                       (const bf16_t*)mask, (const bf16_t*)y, mean, invstd, (int)P, C, rows, ws);
  else
    hipLaunchKernelGGL(bn_bwd_reduce_kernel<float>, dim3(nb), dim3(256), shm, s, (const float*)dout,
                       (const float*)mask, (const float*)y, mean, invstd, (int)P, C, rows, ws);
  VCG_LAUNCH_CHECK();
  hipLaunchKernelGGL(bn_bwd_finalize_kernel, dim3((C + 255) / 256), dim3(256), 0, s, ws, nb, C, sum_g, sum_gx, dgamma,
                     dbeta, accumulate);
  VCG_LAUNCH_CHECK();
  return VCG_OK;
}

VCG_API int vcg_bn_bwd_apply(int dtype, const void* dout, const void* mask, const void* y, const float* mean,
                             const float* invstd, const float* gamma, const float* sum_g, const float* sum_gx,
                             long long count, int train_stats, void* dy, void* gout, long long P, int C,
                             hipStream_t s) {
  const int VN = dtype == VCG_BF16 ? 8 : 4;
  VCG_REQUIRE(C % VN == 0, "C must be a multiple of the vector width");
  const long long tv = P * C / VN;
  const float ic = 1.f / (float)count;
  if (dtype == VCG_BF16)
    hipLaunchKernelGGL(bn_bwd_apply_kernel<bf16_t>, dim3(grid_for(tv)), dim3(256), 0, s, (const bf16_t*)dout,
                       (const bf16_t*)mask, (const bf16_t*)y, mean, invstd, gamma, sum_g, sum_gx, ic, train_stats,
                       (bf16_t*)dy, (bf16_t*)gout, tv, C);
  else
    hipLaunchKernelGGL(bn_bwd_apply_kernel<float>, dim3(grid_for(tv)), dim3(256), 0, s, (const float*)dout,
                       (const float*)mask, (const float*)y, mean, invstd, gamma, sum_g, sum_gx, ic, train_stats,
                       (float*)dy, (float*)gout, tv, C);
  VCG_LAUNCH_CHECK();
  return VCG_OK;
}

VCG_API int vcg_maxpool_fwd(int dtype, const void* x, void* y, unsigned char* idx, int N, int H, int W, int C,
                            hipStream_t s) {
  const int OH = (H + 2 - 3) / 2 + 1, OW = (W + 2 - 3) / 2 + 1;
  const long long tot = (long long)N * OH * OW * C;
  if (dtype == VCG_BF16)
    hipLaunchKernelGGL(maxpool_fwd_kernel<bf16_t>, dim3(grid_for(tot)), dim3(256), 0, s, (const bf16_t*)x,
                       (bf16_t*)y, idx, N, H, W, C, OH, OW);
  else
    hipLaunchKernelGGL(maxpool_fwd_kernel<float>, dim3(grid_for(tot)), dim3(256), 0, s, (const float*)x, (float*)y,
                       idx, N, H, W, C, OH, OW);
  VCG_LAUNCH_CHECK();
  return VCG_OK;
}

VCG_API int vcg_maxpool_bwd(int dtype, const void* dy, const unsigned char* idx, void* dx, int N, int H, int W, int C,
                            hipStream_t s) {
  const int OH = (H + 2 - 3) / 2 + 1, OW = (W + 2 - 3) / 2 + 1;
  const long long tot = (long long)N * H * W * C;
  if (dtype == VCG_BF16)
    hipLaunchKernelGGL(maxpool_bwd_kernel<bf16_t>, dim3(grid_for(tot)), dim3(256), 0, s, (const bf16_t*)dy, idx,
                       (bf16_t*)dx, N, H, W, C, OH, OW);
  else
    hipLaunchKernelGGL(maxpool_bwd_kernel<float>, dim3(grid_for(tot)), dim3(256), 0, s, (const float*)dy, idx,
                       (float*)dx, N, H, W, C, OH, OW);
  VCG_LAUNCH_CHECK();
  return VCG_OK;
}

VCG_API int vcg_avgpool_fwd(int dtype, const void* x, float* y, int N, int HW, int C, hipStream_t s) {
  dim3 grid((C + 255) / 256, N);
  if (dtype == VCG_BF16)
    hipLaunchKernelGGL(avgpool_fwd_kernel<bf16_t>, grid, dim3(256), 0, s, (const bf16_t*)x, y, HW, C);
  else
    hipLaunchKernelGGL(avgpool_fwd_kernel<float>, grid, dim3(256), 0, s, (const float*)x, y, HW, C);
  VCG_LAUNCH_CHECK();
  return VCG_OK;
}

VCG_API int vcg_avgpool_bwd(int dtype, const float* dy, void* dx, int N, int HW, int C, hipStream_t s) {
  const long long tot = (long long)N * HW * C;
  if (dtype == VCG_BF16)
    hipLaunchKernelGGL(avgpool_bwd_kernel<bf16_t>, dim3(grid_for(tot)), dim3(256), 0, s, dy, (bf16_t*)dx, HW, C, tot);
  else
    hipLaunchKernelGGL(avgpool_bwd_kernel<float>, dim3(grid_for(tot)), dim3(256), 0, s, dy, (float*)dx, HW, C, tot);
  VCG_LAUNCH_CHECK();
  return VCG_OK;
}

VCG_API int vcg_frames_to_nhwc(int dtype, const float* src, void* dst, int N, int C, int H, int W, int Cpad,
                               hipStream_t s) {
  VCG_REQUIRE(Cpad >= C, "Cpad < C");
  const long long tot = (long long)N * H * W;
  if (dtype == VCG_BF16)
    hipLaunchKernelGGL(frames_to_nhwc_kernel<bf16_t>, dim3(grid_for(tot)), dim3(256), 0, s, src, (bf16_t*)dst, N, C,
                       H, W, Cpad);
  else
    hipLaunchKernelGGL(frames_to_nhwc_kernel<float>, dim3(grid_for(tot)), dim3(256), 0, s, src, (float*)dst, N, C, H,
                       W, Cpad);
  VCG_LAUNCH_CHECK();
  return VCG_OK;
}

VCG_API int vcg_weight_prep(int dtype, const float* w, void* out, int Cout, int Cin, int KH, int KW, int Cpad,
                            int transposed, hipStream_t s) {
  const long long tot = (long long)Cout * KH * KW * (transposed ? Cin : Cpad);
  if (dtype == VCG_BF16)
    hipLaunchKernelGGL(weight_prep_kernel<bf16_t>, dim3(grid_for(tot)), dim3(256), 0, s, w, (bf16_t*)out, Cout, Cin,
                       KH, KW, Cpad, transposed);
  else
    hipLaunchKernelGGL(weight_prep_kernel<float>, dim3(grid_for(tot)), dim3(256), 0, s, w, (float*)out, Cout, Cin, KH,
                       KW, Cpad, transposed);
  VCG_LAUNCH_CHECK();
  return VCG_OK;
}

VCG_API int vcg_cast_from_f32(int dtype, const float* in, void* out, long long n, hipStream_t s) {
  if (dtype == VCG_BF16)
    hipLaunchKernelGGL(cast_kernel<bf16_t>, dim3(grid_for(n)), dim3(256), 0, s, in, (bf16_t*)out, n);
  else
    hipLaunchKernelGGL(cast_kernel<float>, dim3(grid_for(n)), dim3(256), 0, s, in, (float*)out, n);
  VCG_LAUNCH_CHECK();
  return VCG_OK;
}

VCG_API int vcg_cast_to_f32(int dtype, const void* in, float* out, long long n, hipStream_t s) {
  if (dtype == VCG_BF16)
    hipLaunchKernelGGL(to_f32_kernel<bf16_t>, dim3(grid_for(n)), dim3(256), 0, s, (const bf16_t*)in, out, n);
  else
    hipLaunchKernelGGL(to_f32_kernel<float>, dim3(grid_for(n)), dim3(256), 0, s, (const float*)in, out, n);
  VCG_LAUNCH_CHECK();
  return VCG_OK;
}

// Reference TemporalShift.shift / its adjoint on an NCHW tensor [n_batch*T][C][H][W].
VCG_API int vcg_tsm_shift(int dtype, const void* x, void* y, long long n_batch, int T, int C, long long HW,
                          int fold_div, int direction, hipStream_t s) {
  VCG_REQUIRE(fold_div > 0 && T > 0, "bad fold_div / T");
  const int fold = C / fold_div;
  const long long tot = n_batch * T * C * HW;
  if (dtype == VCG_BF16)
    hipLaunchKernelGGL(tsm_nchw_kernel<bf16_t>, dim3(grid_for(tot)), dim3(256), 0, s, (const bf16_t*)x, (bf16_t*)y,
                       n_batch, T, C, HW, fold, direction);
  else
    hipLaunchKernelGGL(tsm_nchw_kernel<float>, dim3(grid_for(tot)), dim3(256), 0, s, (const float*)x, (float*)y,
                       n_batch, T, C, HW, fold, direction);
  VCG_LAUNCH_CHECK();
  return VCG_OK;
}

VCG_API int vcg_tsm_unshift_add(int dtype, const void* dshift, const void* other, void* dx, long long NT, int T,
                                long long HW, int C, int fold, hipStream_t s) {
  const int VN = dtype == VCG_BF16 ? 8 : 4;
  VCG_REQUIRE(C % VN == 0 && (fold % VN == 0), "C and fold must be multiples of the vector width");
  const long long tv = NT * HW * C / VN;
  if (dtype == VCG_BF16)
    hipLaunchKernelGGL(tsm_unshift_add_kernel<bf16_t>, dim3(grid_for(tv)), dim3(256), 0, s, (const bf16_t*)dshift,
                       (const bf16_t*)other, (bf16_t*)dx, tv, T, HW * C, C, fold);
  else
    hipLaunchKernelGGL(tsm_unshift_add_kernel<float>, dim3(grid_for(tv)), dim3(256), 0, s, (const float*)dshift,
                       (const float*)other, (float*)dx, tv, T, HW * C, C, fold);
  VCG_LAUNCH_CHECK();
  return VCG_OK;
}
