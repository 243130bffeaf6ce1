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
  const float2* cnt = stats + (long long)gridDim.x * mtiles;  // count row (slot row counts; 0 = empty)
  // the fast conv kernel fills only its gy leading slots and says so in the count row's slot 0 (.y = gy)
  const int used = cnt[0].y > 0.f ? min(mtiles, (int)cnt[0].y) : mtiles;
  for (int t = threadIdx.x; t < used; t += blockDim.x) {
    const float2 st = stats[(long long)c * mtiles + t];
    const double nb = (double)cnt[t].x;
    if (nb <= 0.0) continue;
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

// bf16, C % 8 == 0: a thread owns 8 channels of one image (16-B loads, 7 pixels in flight); the global average pool of
// the trunk (ResNet avgpool, HW = 49) was 2-B loads one channel per thread (107 us at 1024 x 49 x 2048: 1.9 TB/s)
__global__ __launch_bounds__(256) void avgpool_fwd8_kernel(const bf16_t* __restrict__ x, float* __restrict__ y, int HW,
                                                           int C, long long total) {
  const long long t = blockIdx.x * (long long)blockDim.x + threadIdx.x;  // (image, 8-channel chunk)
  if (t >= total) return;
  const int cpr = C >> 3;
  const long long n = t / cpr;
  const int c8 = (int)(t - n * cpr);
  const uint4* p = reinterpret_cast<const uint4*>(x + (long long)n * HW * C) + c8;
  float s[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  int i = 0;
  for (; i + 7 <= HW; i += 7) {
    uint4 u[7];
#pragma unroll
    for (int k = 0; k < 7; ++k) u[k] = p[(long long)(i + k) * cpr];
#pragma unroll
    for (int k = 0; k < 7; ++k) {
      const uint32_t w[4] = {u[k].x, u[k].y, u[k].z, u[k].w};
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        s[2 * e] += __uint_as_float(w[e] << 16);
        s[2 * e + 1] += __uint_as_float(w[e] & 0xffff0000u);
      }
    }
  }
  for (; i < HW; ++i) {
    const uint4 u = p[(long long)i * cpr];
    const uint32_t w[4] = {u.x, u.y, u.z, u.w};
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      s[2 * e] += __uint_as_float(w[e] << 16);
      s[2 * e + 1] += __uint_as_float(w[e] & 0xffff0000u);
    }
  }
  const float d = (float)HW;  // (a division, as the reference's mean and avgpool_fwd_kernel)
  float4* o = reinterpret_cast<float4*>(y + n * C + 8 * c8);
  o[0] = make_float4(s[0] / d, s[1] / d, s[2] / d, s[3] / d);
  o[1] = make_float4(s[4] / d, s[5] / d, s[6] / d, s[7] / d);
}

// bf16, C % 8 == 0: dx[n][hw][c] = dy[n][c] / HW, one 16-B store per thread (was one 2-B store with a 64-bit div/mod)
__global__ __launch_bounds__(256) void avgpool_bwd8_kernel(const float* __restrict__ dy, uint4* __restrict__ dx, int HW,
                                                           int C, long long total) {
  const int cpr = C >> 3;
  const float d = (float)HW;  // dy / HW, bit-identical to avgpool_bwd_kernel
  for (long long v = blockIdx.x * (long long)blockDim.x + threadIdx.x; v < total;
       v += (long long)gridDim.x * blockDim.x) {
    const long long pix = v / cpr;
    const int c8 = (int)(v - pix * cpr);
    const long long n = pix / HW;
    const float4* g = reinterpret_cast<const float4*>(dy + n * C + 8 * c8);
    const float4 a = g[0], b = g[1];
    uint4 o;
    o.x = (uint32_t)f2bf(a.x / d) | ((uint32_t)f2bf(a.y / d) << 16);
    o.y = (uint32_t)f2bf(a.z / d) | ((uint32_t)f2bf(a.w / d) << 16);
    o.z = (uint32_t)f2bf(b.x / d) | ((uint32_t)f2bf(b.y / d) << 16);
    o.w = (uint32_t)f2bf(b.z / d) | ((uint32_t)f2bf(b.w / d) << 16);
    dx[v] = o;
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

// The bf16 stem input (C = 3 -> Cpad = 8): one pixel per thread, its 3 plane loads coalesced across the wave
// and ONE 16-B store of the padded pixel; 32-bit indices (the dispatcher checks N*H*W*C < 2^31).
__global__ __launch_bounds__(256) void frames_to_nhwc8_kernel(const float* __restrict__ src, uint4* __restrict__ dst,
                                                            int total, int HW) {
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < total; i += gridDim.x * blockDim.x) {
    const int n = i / HW, hw = i - n * HW;
    const float* s0 = src + (long long)n * 3 * HW + hw;
    const float r = __builtin_nontemporal_load(s0), g = __builtin_nontemporal_load(s0 + HW),
                b = __builtin_nontemporal_load(s0 + 2 * HW);
    uint4 q;
    q.x = (uint32_t)f2bf(r) | ((uint32_t)f2bf(g) << 16);
    q.y = (uint32_t)f2bf(b);
    q.z = 0u;
    q.w = 0u;
    dst[i] = q;
  }
}

// The pair-packed bf16 stem input (C = 3 -> Cpad = 4, RGB0): one 8-B store per pixel.
__global__ __launch_bounds__(256) void frames_to_nhwc4_kernel(const float* __restrict__ src, uint2* __restrict__ dst,
                                                            int total, int HW) {
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < total; i += gridDim.x * blockDim.x) {
    const int n = i / HW, hw = i - n * HW;
    const float* s0 = src + (long long)n * 3 * HW + hw;
    const float r = __builtin_nontemporal_load(s0), g = __builtin_nontemporal_load(s0 + HW),
                b = __builtin_nontemporal_load(s0 + 2 * HW);
    uint2 q;
    q.x = (uint32_t)f2bf(r) | ((uint32_t)f2bf(g) << 16);
    q.y = (uint32_t)f2bf(b);
    dst[i] = q;
  }
}

// Frame ingest: decoded u8 RGB frames of one video [F][H][W][3] -> the stem's
// NHWC input [n_rows][H][W][8] (channels 3..7 zero) for the window frame table idx[n_rows]
// (window-major, frame-minor: row = w*T + t), normalised as torchvision ToTensor + Normalize
// (`train_video_segment_point.py:383-386`): (u / 255 - mean_c) / std_c in fp32 with IEEE division.
template <typename T>
__global__ void window_frames_u8_kernel(const uint8_t* __restrict__ frames, const long long* __restrict__ idx,
                                        T* __restrict__ dst, long long n_rows, int F, int HW, float m0, float m1,
                                        float m2, float s0, float s1, float s2, int cpad) {
  const long long total = n_rows * HW;
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < total;
       i += (long long)gridDim.x * blockDim.x) {
    const long long row = i / HW;
    const long long px = i - row * HW;
    const long long f = idx[row];
    float v[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    if (f >= 0 && f < F) {
      const uint8_t* q = frames + (f * HW + px) * 3;
      v[0] = ((float)q[0] / 255.f - m0) / s0;
      v[1] = ((float)q[1] / 255.f - m1) / s1;
      v[2] = ((float)q[2] / 255.f - m2) / s2;
    }
    T* d = dst + i * cpad;
    if constexpr (sizeof(T) == 2) {
      const uint32_t lo = (uint32_t)f2bf(v[0]) | ((uint32_t)f2bf(v[1]) << 16), hi = (uint32_t)f2bf(v[2]);
      if (cpad == 4) *reinterpret_cast<uint2*>(d) = make_uint2(lo, hi);
      else *reinterpret_cast<uint4*>(d) = make_uint4(lo, hi, 0u, 0u);
    } else {
      *reinterpret_cast<float4*>(d) = make_float4(v[0], v[1], v[2], 0.f);
      if (cpad == 8) *reinterpret_cast<float4*>(d + 4) = make_float4(0.f, 0.f, 0.f, 0.f);
    }
  }
}

// Pair-packed stem weights (igemm.hip pair_taps; mode = 2 + pad): [Cout][KH][KWp][8], element 4j + c of super
// tap kwp = w[cout][c][kh][2 (kwp - pwp) + j + pad] (zero for c >= Cin or a tap outside the kernel).
__host__ __device__ __forceinline__ int pair_floor_half(int x) { return (x - (x & 1)) / 2; }
__host__ __device__ __forceinline__ void pair_geom(int KW, int pad, int& KWp, int& pwp) {
  const int lo = pair_floor_half(-pad);
  KWp = pair_floor_half(KW - 1 - pad) - lo + 1;
  pwp = -lo;
}
__device__ __forceinline__ float pair_weight(const float* w, long long i, int Cin, int KH, int KW, int pad) {
  int KWp, pwp;
  pair_geom(KW, pad, KWp, pwp);
  const int c8 = (int)(i & 7);
  long long r = i >> 3;
  const int kwp = (int)(r % KWp); r /= KWp;
  const int kh = (int)(r % KH);
  const int co = (int)(r / KH);
  const int j = c8 >> 2, ci = c8 & 3;
  const int kw = 2 * (kwp - pwp) + j + pad;
  return (ci < Cin && kw >= 0 && kw < KW) ? w[(((long long)co * Cin + ci) * KH + kh) * KW + kw] : 0.f;
}

// OIHW fp32 -> [Cout][KH][KW][Cpad] (transposed = 0), [Cin][KH][KW][Cout] (transposed = 1) or the pair-packed
// stem layout (transposed = 2 + pad)
template <typename T>
__global__ void weight_prep_kernel(const float* __restrict__ w, T* __restrict__ out, int Cout, int Cin, int KH, int KW,
                                   int Cpad, int transposed) {
  int KWp = 0, pwp = 0;
  if (transposed >= 2) pair_geom(KW, transposed - 2, KWp, pwp);
  const long long total = transposed >= 2 ? (long long)Cout * KH * KWp * 8
                          : transposed    ? (long long)Cin * KH * KW * Cout
                                          : (long long)Cout * KH * KW * Cpad;
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < total;
       i += (long long)gridDim.x * blockDim.x) {
    float v;
    if (transposed >= 2) {
      v = pair_weight(w, i, Cin, KH, KW, transposed - 2);
    } else if (!transposed) {
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

// out[c][r] = in[r][c] for a [rows][cols] matrix (leading dims ld_in / ld_out): 64x64 tiles through
// LDS (odd row pitch: conflict-free column reads), coalesced reads and writes.
template <typename T>
__global__ __launch_bounds__(256) void transpose_kernel(const T* __restrict__ in, T* __restrict__ out, int rows,
                                                        int cols, long long ld_in, long long ld_out) {
  __shared__ float tile[64][65];
  const int r0 = blockIdx.y * 64, c0 = blockIdx.x * 64;
  const int tx = threadIdx.x & 63, ty = threadIdx.x >> 6;
#pragma unroll
  for (int k = 0; k < 16; ++k) {
    const int r = r0 + ty + 4 * k, c = c0 + tx;
    if (r < rows && c < cols) tile[ty + 4 * k][tx] = to_f<T>(in[(long long)r * ld_in + c]);
  }
  __syncthreads();
#pragma unroll
  for (int k = 0; k < 16; ++k) {
    const int c = c0 + ty + 4 * k, r = r0 + tx;
    if (r < rows && c < cols) out[(long long)c * ld_out + r] = from_f<T>(tile[tx][ty + 4 * k]);
  }
}

// Batched bf16 transpose (vcg_transpose_multi): descriptor i = (src, dst, rows, cols, first tile) [5 int64];
// block b transposes the 64 x 64 tile b - first of the descriptor whose range holds b. 16-B loads and stores,
// the tile in LDS with a 144-B row pitch. rows, cols multiples of 8.
__global__ __launch_bounds__(256) void transpose_multi_kernel(const long long* __restrict__ desc, int n) {
  __shared__ __attribute__((aligned(16))) bf16_t tile[64 * 72];
  const int b = blockIdx.x;
  int i = 0;
  while (i + 1 < n && desc[5 * (i + 1) + 4] <= b) ++i;
  const long long* d = desc + 5 * i;
  const bf16_t* in = reinterpret_cast<const bf16_t*>(d[0]);
  bf16_t* out = reinterpret_cast<bf16_t*>(d[1]);
  const int rows = (int)d[2], cols = (int)d[3];
  const int t = b - (int)d[4], tc = (cols + 63) / 64;
  const int r0 = (t / tc) * 64, c0 = (t % tc) * 64;
  const int tid = threadIdx.x;
#pragma unroll
  for (int k = 0; k < 2; ++k) {
    const int id = tid + 256 * k, r = id >> 3, c = 8 * (id & 7);
    uint4 v = make_uint4(0u, 0u, 0u, 0u);
    if (r0 + r < rows && c0 + c < cols) v = *reinterpret_cast<const uint4*>(in + (long long)(r0 + r) * cols + c0 + c);
    *reinterpret_cast<uint4*>(tile + r * 72 + c) = v;
  }
  __syncthreads();
#pragma unroll
  for (int k = 0; k < 2; ++k) {
    const int id = tid + 256 * k, oc = id >> 3, r = 8 * (id & 7);
    if (c0 + oc >= cols || r0 + r >= rows) continue;
    uint32_t w[4];
#pragma unroll
    for (int j = 0; j < 4; ++j)
      w[j] = (uint32_t)tile[(r + 2 * j) * 72 + oc] | ((uint32_t)tile[(r + 2 * j + 1) * 72 + oc] << 16);
    *reinterpret_cast<uint4*>(out + (long long)(c0 + oc) * rows + r0 + r) = make_uint4(w[0], w[1], w[2], w[3]);
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

VCG_API int vcg_avgpool_fwd(int dtype, const void* x, float* y, int N, int HW, int C, hipStream_t s) {
  if (dtype == VCG_BF16 && C % 8 == 0) {
    const long long tot = (long long)N * (C / 8);
    hipLaunchKernelGGL(avgpool_fwd8_kernel, dim3((unsigned)((tot + 255) / 256)), dim3(256), 0, s, (const bf16_t*)x, y,
                       HW, C, tot);
    VCG_LAUNCH_CHECK();
    return VCG_OK;
  }
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
  if (dtype == VCG_BF16 && C % 8 == 0) {
    hipLaunchKernelGGL(avgpool_bwd8_kernel, dim3(grid_for(tot / 8)), dim3(256), 0, s, dy, (uint4*)dx, HW, C, tot / 8);
    VCG_LAUNCH_CHECK();
    return VCG_OK;
  }
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
  if (dtype == VCG_BF16 && C == 3 && Cpad == 8 && tot * 3 < (1LL << 31))
    hipLaunchKernelGGL(frames_to_nhwc8_kernel, dim3(grid_for(tot)), dim3(256), 0, s, src, (uint4*)dst, (int)tot,
                       H * W);
  else if (dtype == VCG_BF16 && C == 3 && Cpad == 4 && tot * 3 < (1LL << 31))
    hipLaunchKernelGGL(frames_to_nhwc4_kernel, dim3(grid_for(tot)), dim3(256), 0, s, src, (uint2*)dst, (int)tot,
                       H * W);
  else if (dtype == VCG_BF16)
    hipLaunchKernelGGL(frames_to_nhwc_kernel<bf16_t>, dim3(grid_for(tot)), dim3(256), 0, s, src, (bf16_t*)dst, N, C,
                       H, W, Cpad);
  else
    hipLaunchKernelGGL(frames_to_nhwc_kernel<float>, dim3(grid_for(tot)), dim3(256), 0, s, src, (float*)dst, N, C, H,
                       W, Cpad);
  VCG_LAUNCH_CHECK();
  return VCG_OK;
}

VCG_API int vcg_window_frames_u8_cpad(int dtype, const uint8_t* frames, const long long* idx, void* dst,
                                      long long n_rows, int F, int H, int W, int Cpad, const float* mean3,
                                      const float* std3, hipStream_t s) {
  VCG_REQUIRE(mean3 && std3, "mean/std required");
  VCG_REQUIRE(Cpad == 4 || Cpad == 8, "Cpad must be 4 or 8");
  VCG_REQUIRE(n_rows >= 0 && F > 0 && H > 0 && W > 0, "bad shape");
  const long long tot = n_rows * H * W;
  if (tot == 0) return VCG_OK;
  if (dtype == VCG_BF16)
    hipLaunchKernelGGL(window_frames_u8_kernel<bf16_t>, dim3(grid_for(tot)), dim3(256), 0, s, frames, idx,
                       (bf16_t*)dst, n_rows, F, H * W, mean3[0], mean3[1], mean3[2], std3[0], std3[1], std3[2], Cpad);
  else
    hipLaunchKernelGGL(window_frames_u8_kernel<float>, dim3(grid_for(tot)), dim3(256), 0, s, frames, idx, (float*)dst,
                       n_rows, F, H * W, mean3[0], mean3[1], mean3[2], std3[0], std3[1], std3[2], Cpad);
  VCG_LAUNCH_CHECK();
  return VCG_OK;
}

VCG_API int vcg_window_frames_u8(int dtype, const uint8_t* frames, const long long* idx, void* dst, long long n_rows,
                                 int F, int H, int W, const float* mean3, const float* std3, hipStream_t s) {
  return vcg_window_frames_u8_cpad(dtype, frames, idx, dst, n_rows, F, H, W, 8, mean3, std3, s);
}

VCG_API int vcg_weight_prep(int dtype, const float* w, void* out, int Cout, int Cin, int KH, int KW, int Cpad,
                            int transposed, hipStream_t s) {
  VCG_REQUIRE(transposed < 2 || (dtype == VCG_BF16 && Cin <= 4), "pair-packed layout: bf16, Cin <= 4");
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

namespace {
// vcg_weight_fold: out[r][c] = w[r][c] * scale[r] -- a running-statistics BN folded into the 1x1 conv that feeds it
template <typename T>
__global__ void weight_fold_kernel(const float* __restrict__ w, const float* __restrict__ scale, T* __restrict__ out,
                                   int cols, long long total) {
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < total;
       i += (long long)gridDim.x * blockDim.x)
    out[i] = from_f<T>(w[i] * scale[i / cols]);
}
}  // namespace

VCG_API int vcg_weight_fold(int dtype, const float* w, const float* scale, void* out, int rows, int cols,
                            hipStream_t s) {
  VCG_REQUIRE(w && scale && out && rows > 0 && cols > 0, "bad arguments");
  const long long tot = (long long)rows * cols;
  if (dtype == VCG_BF16)
    hipLaunchKernelGGL(weight_fold_kernel<bf16_t>, dim3(grid_for(tot)), dim3(256), 0, s, w, scale, (bf16_t*)out, cols,
                       tot);
  else
    hipLaunchKernelGGL(weight_fold_kernel<float>, dim3(grid_for(tot)), dim3(256), 0, s, w, scale, (float*)out, cols,
                       tot);
  VCG_LAUNCH_CHECK();
  return VCG_OK;
}

namespace {
// vcg_weight_prep_multi: blockIdx.y = descriptor (8 int64: src, dst, Cout, Cin, KH, KW, Cpad, mode = transposed
// as in vcg_weight_prep: 0, 1 or 2 + pad for the pair-packed stem). Both GEMM layouts are transposes of the fp32
// [Cout][Cin][KH][KW] weight, done through LDS so that reads and writes are both coalesced:
//   mode 1 (dgrad B operand [Cin][KH][KW][Cout]): the [Cout][R = Cin KH KW] matrix transposed, 64 x 64 tiles;
//   mode 0 ([Cout][KH][KW][Cpad]): per output channel, [Cin][T = KH KW] -> [T][Cpad] (zero pad), one row per unit.
// (The per-element gather this replaces read the fp32 weight with a Cin KH KW stride: 338 us per step.)
constexpr int WP_ROW_MAX = 4608;  // Cin * KH * KW of one output channel staged in LDS (18 KiB)

__global__ __launch_bounds__(256) void weight_prep_multi_kernel(const long long* __restrict__ desc) {
  __shared__ float tile[WP_ROW_MAX + 64];
  const long long* d = desc + 8 * blockIdx.y;
  const float* w = reinterpret_cast<const float*>(d[0]);
  bf16_t* out = reinterpret_cast<bf16_t*>(d[1]);
  const int Cout = (int)d[2], Cin = (int)d[3], KH = (int)d[4], KW = (int)d[5], Cpad = (int)d[6];
  const int mode = (int)d[7];
  const int T = KH * KW, R = Cin * T;
  const int tid = threadIdx.x;
  if (mode >= 2 || (mode == 0 && R > WP_ROW_MAX)) {  // the pair-packed stem (and any oversized row): per element
    int KWp = 0, pwp = 0;
    if (mode >= 2) pair_geom(KW, mode - 2, KWp, pwp);
    const int total = mode >= 2 ? Cout * KH * KWp * 8 : Cout * T * Cpad;
    for (int i = blockIdx.x * 256 + tid; i < total; i += gridDim.x * 256) {
      float v;
      if (mode >= 2) {
        v = pair_weight(w, i, Cin, KH, KW, mode - 2);
      } else {
        const int ci = i % Cpad, r = i / Cpad, t = r % T, co = r / T;
        v = ci < Cin ? w[((long long)co * Cin + ci) * T + t] : 0.f;
      }
      out[i] = f2bf(v);
    }
    return;
  }
  if (mode == 1) {  // out[r][co] = w[co][r]
    const int tr = (R + 63) / 64, tc = (Cout + 63) / 64;
    const int tx = tid & 63, ty = tid >> 6;  // 64 x 4 threads
    for (int tl = blockIdx.x; tl < tr * tc; tl += gridDim.x) {
      const int r0 = (tl % tr) * 64, c0 = (tl / tr) * 64;
      __syncthreads();
#pragma unroll 4
      for (int k = ty; k < 64; k += 4) {  // rows co = c0 + k, columns r0 + tx: coalesced reads
        const int co = c0 + k, r = r0 + tx;
        tile[k * 65 + tx] = (co < Cout && r < R) ? w[(long long)co * R + r] : 0.f;
      }
      __syncthreads();
#pragma unroll 4
      for (int k = ty; k < 64; k += 4) {  // rows r = r0 + k, columns co = c0 + tx: coalesced writes
        const int r = r0 + k, co = c0 + tx;
        if (r < R && co < Cout) out[(long long)r * Cout + co] = f2bf(tile[tx * 65 + k]);
      }
    }
    return;
  }
  // mode 0: out[co][t][ci] = w[co][ci][t] (ci < Cin), 0 for Cin <= ci < Cpad
  const int orow = T * Cpad;
  for (int co = blockIdx.x; co < Cout; co += gridDim.x) {
    const float* src = w + (long long)co * R;
    bf16_t* dst = out + (long long)co * orow;
    if (T == 1) {
      for (int ci = tid; ci < Cpad; ci += 256) dst[ci] = f2bf(ci < Cin ? src[ci] : 0.f);
      continue;
    }
    __syncthreads();
    for (int i = tid; i < R; i += 256) tile[i] = src[i];
    __syncthreads();
    for (int i = tid; i < orow; i += 256) {
      const int t = i / Cpad, ci = i - t * Cpad;
      dst[i] = f2bf(ci < Cin ? tile[ci * T + t] : 0.f);
    }
  }
}
}  // namespace

VCG_API int vcg_weight_prep_multi(int dtype, const long long* desc, int n, hipStream_t s) {
  VCG_REQUIRE(dtype == VCG_BF16, "the batched weight prep writes bf16 GEMM layouts");
  VCG_REQUIRE(n >= 0 && n <= 65535, "bad descriptor count");
  if (n == 0) return VCG_OK;
  hipLaunchKernelGGL(weight_prep_multi_kernel, dim3(128, n), dim3(256), 0, s, desc);
  VCG_LAUNCH_CHECK();
  return VCG_OK;
}

VCG_API int vcg_transpose(int dtype, const void* in, void* out, int rows, int cols, long long ld_in, long long ld_out,
                          hipStream_t s) {
  VCG_REQUIRE(rows > 0 && cols > 0 && ld_in >= cols && ld_out >= rows, "bad transpose shape");
  const dim3 grid((cols + 63) / 64, (rows + 63) / 64);
  if (dtype == VCG_BF16)
    hipLaunchKernelGGL(transpose_kernel<bf16_t>, grid, dim3(256), 0, s, (const bf16_t*)in, (bf16_t*)out, rows, cols,
                       ld_in, ld_out);
  else
    hipLaunchKernelGGL(transpose_kernel<float>, grid, dim3(256), 0, s, (const float*)in, (float*)out, rows, cols,
                       ld_in, ld_out);
  VCG_LAUNCH_CHECK();
  return VCG_OK;
}

VCG_API int vcg_transpose_multi(const long long* desc, int n, int total_tiles, hipStream_t s) {
  VCG_REQUIRE(n > 0 && total_tiles > 0, "bad descriptor / tile count");
  hipLaunchKernelGGL(transpose_multi_kernel, dim3(total_tiles), dim3(256), 0, s, desc, n);
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

