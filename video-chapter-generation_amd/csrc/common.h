// Shared device/host helpers for libvcg_hip (gfx950 / CDNA4 only).
//
// Storage types: fp32 (`float`) for the parity mode and bf16 (raw 16-bit pattern in
// `bf16_t`) for the throughput mode. Every kernel accumulates in fp32.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <cstdio>
#include <string>

typedef uint16_t bf16_t;

typedef __attribute__((ext_vector_type(8))) short s16x8;
typedef __attribute__((ext_vector_type(4))) short s16x4;
typedef __attribute__((ext_vector_type(4))) float f32x4;

#define VCG_API extern "C" __attribute__((visibility("default")))

namespace vcg {
// kernel ids of vcg_timing_query
enum { TIMING_FAST_GEMM = 0, TIMING_WGRAD = 1, TIMING_GENERIC_GEMM = 2, TIMING_PATCH_CONV = 3, TIMING_WIDE_GEMM = 4 };
int timing_begin(hipStream_t s);
void timing_end(int idx, hipStream_t s, int id, double flops, double bytes);
// GEMM census (vcg_gemm_census_*): every GEMM-class launch adds one to the count of "<kernel tag> M=.. N=.. K=.."
bool census_on();
void census_add(const char* tag, long long M, long long N, long long K);
}  // namespace vcg

enum vcg_dtype { VCG_F32 = 0, VCG_BF16 = 1 };
enum { VCG_GRAD_F32 = 0x10 };  // vcg_ln_bwd / vcg_embed_ln_bwd dtype flag (include/vcg_hip.h)
enum vcg_status {
  VCG_OK = 0,
  VCG_ERR_INVALID = -1,
  VCG_ERR_UNSUPPORTED = -2,
  VCG_ERR_HIP = -3,
};

namespace vcg {

void set_error(const std::string& msg);

__device__ __forceinline__ float bf2f(bf16_t h) { return __uint_as_float(((uint32_t)h) << 16); }
struct FastDiv {  // q = n / d for 0 <= n < 2^31
  uint32_t d, m, s;
};
static inline FastDiv make_fastdiv(uint32_t d) {
  FastDiv f;
  f.d = d;
  uint32_t s = 0;
  while ((1ull << s) < d) ++s;
  f.s = s;
  f.m = (uint32_t)(((1ull << 32) * ((1ull << s) - d)) / d + 1);
  return f;
}
__device__ __forceinline__ uint32_t fdiv(uint32_t n, const FastDiv& f) {
  uint32_t hi = __umulhi(n, f.m);
  return (uint32_t)(((uint64_t)hi + n) >> f.s);
}

__device__ __forceinline__ bf16_t f2bf(float f) {
  // plain cast lowers to v_cvt_pk_bf16_f32 (RNE, NaN-preserving) on gfx950
  __bf16 b = (__bf16)f;
  return __builtin_bit_cast(bf16_t, b);
}

template <typename T> __device__ __forceinline__ float to_f(T v);
template <> __device__ __forceinline__ float to_f<float>(float v) { return v; }
template <> __device__ __forceinline__ float to_f<bf16_t>(bf16_t v) { return bf2f(v); }

template <typename T> __device__ __forceinline__ T from_f(float v);
template <> __device__ __forceinline__ float from_f<float>(float v) { return v; }
template <> __device__ __forceinline__ bf16_t from_f<bf16_t>(float v) { return f2bf(v); }

// 16-byte vector of T: 4 floats or 8 bf16.
template <typename T> struct Vec16;
template <> struct Vec16<float> {
  static constexpr int N = 4;
  float v[4];
};
template <> struct Vec16<bf16_t> {
  static constexpr int N = 8;
  bf16_t v[8];
};

template <typename T>
__device__ __forceinline__ void load16(const T* p, float (&out)[16 / sizeof(T)]) {
  uint4 u = *reinterpret_cast<const uint4*>(p);
  if constexpr (sizeof(T) == 4) {
    out[0] = __uint_as_float(u.x); out[1] = __uint_as_float(u.y);
    out[2] = __uint_as_float(u.z); out[3] = __uint_as_float(u.w);
  } else {
    uint32_t w[4] = {u.x, u.y, u.z, u.w};
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      out[2 * i] = __uint_as_float(w[i] << 16);
      out[2 * i + 1] = __uint_as_float(w[i] & 0xffff0000u);
    }
  }
}

template <typename T>
__device__ __forceinline__ void store16(T* p, const float (&in)[16 / sizeof(T)]) {
  uint4 u;
  if constexpr (sizeof(T) == 4) {
    u.x = __float_as_uint(in[0]); u.y = __float_as_uint(in[1]);
    u.z = __float_as_uint(in[2]); u.w = __float_as_uint(in[3]);
  } else {
    uint32_t w[4];
#pragma unroll
    for (int i = 0; i < 4; ++i)
      w[i] = (uint32_t)f2bf(in[2 * i]) | ((uint32_t)f2bf(in[2 * i + 1]) << 16);
    u.x = w[0]; u.y = w[1]; u.z = w[2]; u.w = w[3];
  }
  *reinterpret_cast<uint4*>(p) = u;
}

__device__ __forceinline__ float warp_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
__device__ __forceinline__ float warp_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}

// Block-wide sum for blockDim.x <= 1024; `red` must hold >= 16 floats.
__device__ __forceinline__ float block_sum(float v, float* red) {
  v = warp_sum(v);
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int nw = (blockDim.x + 63) >> 6;
  __syncthreads();
  if (lane == 0) red[wid] = v;
  __syncthreads();
  float t = 0.f;
  for (int i = 0; i < nw; ++i) t += red[i];
  return t;
}

__device__ __forceinline__ float gelu_erf(float x) { return 0.5f * x * (1.f + erff(x * 0.70710678118654752f)); }
__device__ __forceinline__ float gelu_erf_grad(float x) {
  const float cdf = 0.5f * (1.f + erff(x * 0.70710678118654752f));
  const float pdf = 0.39894228040143268f * __expf(-0.5f * x * x);
  return cdf + x * pdf;
}
// erf by Abramowitz & Stegun 7.1.26 (|error| <= 1.5e-7, ~1 fp32 ulp of 1): branch-free, one v_rcp_f32 and one
// v_exp_f32 instead of the library erff's piecewise polynomials. Used by the bf16 GEMM epilogues (the output is
// rounded to bf16, 2^-8); the fp32 parity mode keeps erff.
__device__ __forceinline__ float erf_fast(float x) {
  const float ax = fabsf(x);
  const float t = __builtin_amdgcn_rcpf(fmaf(0.3275911f, ax, 1.f));
  float y = fmaf(t, 1.061405429f, -1.453152027f);
  y = fmaf(y, t, 1.421413741f);
  y = fmaf(y, t, -0.284496736f);
  y = fmaf(y, t, 0.254829592f);
  return copysignf(1.f - y * t * __expf(-ax * ax), x);
}
__device__ __forceinline__ float gelu_erf_fast(float x) { return 0.5f * x * (1.f + erf_fast(x * 0.70710678118654752f)); }
__device__ __forceinline__ float gelu_erf_grad_fast(float x) {
  const float cdf = 0.5f * (1.f + erf_fast(x * 0.70710678118654752f));
  return fmaf(x * 0.39894228040143268f, __expf(-0.5f * x * x), cdf);
}

// Counter-based hash (splitmix64 finaliser), shared by dropout and the synthetic generator.
__host__ __device__ __forceinline__ uint64_t mix64(uint64_t z) {
  z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ULL;
  z = (z ^ (z >> 27)) * 0x94d049bb133111ebULL;
  return z ^ (z >> 31);
}

// Dropout keep decision of element idx (a stateless counter hash, so the backward regenerates the mask):
// 32-bit murmur3 finaliser of (idx * golden ratio) ^ seed -- two 32-bit multiplies, no 64-bit arithmetic.
// (Tensors stay below 2^32 elements; the seed differs per dropout site and step.)
__device__ __forceinline__ bool dropout_keep(uint64_t seed, uint64_t idx, float p) {
  if (p <= 0.f) return true;
  uint32_t h = ((uint32_t)idx * 0x9E3779B1u) ^ (uint32_t)seed;
  h += (uint32_t)(seed >> 32);
  h ^= h >> 16;
  h *= 0x85EBCA6Bu;
  h ^= h >> 13;
  h *= 0xC2B2AE35u;
  h ^= h >> 16;
  return (float)(h >> 8) * (1.0f / 16777216.0f) >= p;
}

}  // namespace vcg

#define VCG_CHECK_HIP(expr)                                                     \
  do {                                                                          \
    hipError_t _e = (expr);                                                     \
    if (_e != hipSuccess) {                                                     \
      vcg::set_error(std::string(#expr) + ": " + hipGetErrorString(_e));        \
      return VCG_ERR_HIP;                                                       \
    }                                                                           \
  } while (0)

#define VCG_REQUIRE(cond, msg)                                                  \
  do {                                                                          \
    if (!(cond)) {                                                              \
      vcg::set_error(std::string(__func__) + ": " + (msg));                     \
      return VCG_ERR_INVALID;                                                   \
    }                                                                           \
  } while (0)

#define VCG_LAUNCH_CHECK()                                                      \
  do {                                                                          \
    hipError_t _e = hipGetLastError();                                          \
    if (_e != hipSuccess) {                                                     \
      vcg::set_error(std::string(__func__) + ": launch: " + hipGetErrorString(_e)); \
      return VCG_ERR_HIP;                                                       \
    }                                                                           \
  } while (0)
