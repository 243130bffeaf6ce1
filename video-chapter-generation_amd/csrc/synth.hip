// Deterministic synthetic data generator (counter-based, bit-identical to the numpy twin in
// vcg_hip/synth.py). Used to materialise seeded weights and clip windows directly in HBM
// (SURVEY §8c/§8d synthetic inputs) so that nothing large has to travel to the GPU box.
//
//   h_k(i)  = mix64(key + 0x9E3779B97F4A7C15 * (4*i + k + 1))
//   u_k(i)  = (h_k >> 40) * 2^-24                         (exact in fp32/fp64)
//   kind 0: uniform   out = a + (b - a) * u_0              (fp64, no FMA contraction)
//   kind 1: normal~   out = a + b * ((u0+u1+u2+u3 - 2) * sqrt(3))   (Irwin-Hall(4), unit variance)
//   kind 2: integer   out = a + (h_0 >> 11) % (b - a)      (int64)
#include "common.h"

using namespace vcg;

namespace {

__device__ __forceinline__ uint64_t hk(uint64_t key, long long i, int k) {
  return mix64(key + 0x9E3779B97F4A7C15ULL * (uint64_t)(4 * i + k + 1));
}
__device__ __forceinline__ double u24(uint64_t h) { return (double)(h >> 40) * (1.0 / 16777216.0); }

__global__ void synth_kernel(int kind, void* out, long long n, uint64_t key, double a, double b) {
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < n; i += (long long)gridDim.x * blockDim.x) {
    if (kind == 2) {
      const long long span = (long long)(b - a);
      const uint64_t h = hk(key, i, 0);
      reinterpret_cast<long long*>(out)[i] = (long long)a + (long long)((h >> 11) % (uint64_t)span);
    } else if (kind == 0) {
      const double u = u24(hk(key, i, 0));
      reinterpret_cast<float*>(out)[i] = (float)__dadd_rn(a, __dmul_rn(b - a, u));
    } else {
      double s = u24(hk(key, i, 0)) + u24(hk(key, i, 1));
      s = s + u24(hk(key, i, 2));
      s = s + u24(hk(key, i, 3));
      const double z = __dmul_rn(s - 2.0, 1.7320508075688772);
      reinterpret_cast<float*>(out)[i] = (float)__dadd_rn(a, __dmul_rn(b, z));
    }
  }
}

}  // namespace

VCG_API int vcg_synth(int kind, void* out, long long n, unsigned long long key, double a, double b, hipStream_t s) {
  VCG_REQUIRE(kind >= 0 && kind <= 2, "unknown kind");
  VCG_REQUIRE(kind != 2 || b > a, "empty integer range");
  long long g = (n + 255) / 256;
  if (g > 16384) g = 16384;
  if (g < 1) g = 1;
  hipLaunchKernelGGL(synth_kernel, dim3((unsigned)g), dim3(256), 0, s, kind, out, n, (uint64_t)key, a, b);
  VCG_LAUNCH_CHECK();
  return VCG_OK;
}
