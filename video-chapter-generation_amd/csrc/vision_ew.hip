// Streaming NHWC kernels of the vision trunk: BatchNorm apply (+residual, +ReLU), BatchNorm
// backward (reduce + apply), max-pool fwd/bwd, and the TSM gradient combine.
//
// All are HBM-bound. Layout rule used throughout: a tensor [P][C] is a stream of 16-byte vectors
// v = row * cpr + chunk (cpr = C / VN, a power of two). Blocks take contiguous runs of
// 256 * ITER vectors, so when cpr divides 256 a thread's channel chunk never changes and its
// per-channel parameters live in registers for the whole run; index math stays 32/64-bit
// shifts and masks (no 64-bit division).
#include "common.h"

using namespace vcg;

namespace {

template <typename T> struct V { static constexpr int N = 16 / sizeof(T); };

#ifndef VCG_EW_SU
#define VCG_EW_SU 4
#endif
#ifndef VCG_EW_GRID
#define VCG_EW_GRID 2048
#endif
constexpr int SU = VCG_EW_SU;        // 16-B vectors per thread per batch (all loads issued before use)
constexpr int SB = 256 * SU;         // vectors per block per batch
constexpr long long GRID_MAX = VCG_EW_GRID;  // streaming grids: 8 blocks per CU, grid-stride beyond
constexpr int RED_ITER_MAX = 256;  // vectors per thread of bn_bwd_reduce (adaptive: >= ~1024 blocks)

template <int VN>
__device__ __forceinline__ void load_params(const float* __restrict__ p, int c0, float (&out)[VN]) {
#pragma unroll
  for (int e = 0; e < VN; e += 4) {
    const float4 q = *reinterpret_cast<const float4*>(p + c0 + e);
    out[e] = q.x; out[e + 1] = q.y; out[e + 2] = q.z; out[e + 3] = q.w;
  }
}

// Which elements of the upstream gradient pass the ReLU (vcg_hip.h VCG_MASK_*):
//   0 none; 1 tensor (mask[v] > 0); 2 bits (one byte per 16-B vector, bit e = element e);
//   3 affine (fma(y, mscale[c], mshift[c]) > 0: the forward's BN+ReLU decision recomputed from y).
struct MaskArgs {
  int mode;
  const void* t;
  const uint8_t* bits;
  const float* sc;
  const float* sh;
};

template <typename T, int VN>
__device__ __forceinline__ void apply_mask(float (&d)[VN], const MaskArgs& m, long long v, const float (&yv)[VN],
                                           const float (&msc)[VN], const float (&msh)[VN]) {
  if (m.mode == 1) {
    float mk[VN];
    load16<T>(reinterpret_cast<const T*>(m.t) + v * VN, mk);
#pragma unroll
    for (int e = 0; e < VN; ++e) d[e] = mk[e] > 0.f ? d[e] : 0.f;
  } else if (m.mode == 2) {
    const unsigned b = m.bits[v];
#pragma unroll
    for (int e = 0; e < VN; ++e) d[e] = ((b >> e) & 1u) ? d[e] : 0.f;
  } else if (m.mode == 3) {
#pragma unroll
    for (int e = 0; e < VN; ++e) d[e] = fmaf(yv[e], msc[e], msh[e]) > 0.f ? d[e] : 0.f;
  }
}

__host__ __device__ inline int ilog2i(int x) {
  int l = 0;
  while ((1 << l) < x) ++l;
  return l;
}

// ------------------------------------------------------------------ BN apply
// out = act(fma(y, scale, shift) + [fma(res, rscale, rshift) | res]); bits (optional): ReLU mask of
// out, one byte per 16-B vector (the backward's VCG_MASK_BITS). Grid-stride over batches of SU
// vectors per thread; every load of a batch is issued before the first use.
template <typename T, bool RES, bool RAFF, bool CS = false>
__global__ __launch_bounds__(256) void bn_apply_kernel(const T* __restrict__ y, const float* __restrict__ scale,
                                                       const float* __restrict__ shift, const T* __restrict__ res,
                                                       const float* __restrict__ rscale,
                                                       const float* __restrict__ rshift, int relu,
                                                       T* __restrict__ out, uint8_t* __restrict__ bits, long long TV,
                                                       int cpr, float* __restrict__ colpart = nullptr) {
  constexpr int VN = V<T>::N;
  const long long stride = (long long)gridDim.x * SB;
  long long base = (long long)blockIdx.x * SB + threadIdx.x;
  const bool fixed = cpr <= 256;
  float sc[VN], sh[VN], rs[VN], rb[VN];
  float csum[VN];  // colpart: this thread's column sums of the stored output (its channel chunk is fixed, cpr | 256)
#pragma unroll
  for (int e = 0; e < VN; ++e) csum[e] = 0.f;
  auto params = [&](long long v) {
    const int c0 = (int)(v & (cpr - 1)) * VN;
    load_params<VN>(scale, c0, sc);
    load_params<VN>(shift, c0, sh);
    if (RAFF) {
      load_params<VN>(rscale, c0, rs);
      load_params<VN>(rshift, c0, rb);
    }
  };
  params(base);
  for (; base < TV; base += stride) {
    float a[SU][VN], r[SU][VN];
#pragma unroll
    for (int u = 0; u < SU; ++u) {  // unconditional loads (clamped index): no per-vector branch + wait
      const long long v = min(base + u * 256, TV - 1);
      load16<T>(y + v * VN, a[u]);
      if (RES) load16<T>(res + v * VN, r[u]);
    }
#pragma unroll
    for (int u = 0; u < SU; ++u) {
      const long long v = base + u * 256;
      if (v >= TV) break;
      if (!fixed) params(v);
#pragma unroll
      for (int e = 0; e < VN; ++e) {
        float o = fmaf(a[u][e], sc[e], sh[e]);
        if (RES) o += RAFF ? fmaf(r[u][e], rs[e], rb[e]) : r[u][e];
        a[u][e] = relu ? fmaxf(o, 0.f) : o;
      }
      if (bits) {
        unsigned b = 0;
#pragma unroll
        for (int e = 0; e < VN; ++e) b |= (a[u][e] > 0.f ? 1u : 0u) << e;
        bits[v] = (uint8_t)b;
      }
      if constexpr (CS) {
#pragma unroll
        for (int e = 0; e < VN; ++e) csum[e] += to_f<T>(from_f<T>(a[u][e]));  // the stored (rounded) value
      }
      store16<T>(out + v * VN, a[u]);
    }
  }
  if constexpr (CS) {  // per-block column partials [block][C], threads of one chunk combined in a fixed order
    __shared__ float red[256][VN + 1];
#pragma unroll
    for (int e = 0; e < VN; ++e) red[threadIdx.x][e] = csum[e];
    __syncthreads();
    const int C = cpr * VN;
    for (int o = threadIdx.x; o < C; o += 256) {
      const int ch = o / VN, i = o - ch * VN;
      float acc = 0.f;
      for (int t = ch; t < 256; t += cpr) acc += red[t][i];
      colpart[(long long)blockIdx.x * C + o] = acc;
    }
  }
}

// out[c] = sum_b part[b][c] (fixed order: 16 row stripes per channel in double, then the stripes in order; 16 channels
// per 256-thread block)
__global__ __launch_bounds__(256) void colpart_reduce_kernel(const float* __restrict__ part, int nb, int C,
                                                             float* __restrict__ out) {
  __shared__ double sa[16][16];
  const int tx = threadIdx.x & 15, ty = threadIdx.x >> 4;
  const int c = blockIdx.x * 16 + tx;
  double a = 0;
  if (c < C)
    for (int b = ty; b < nb; b += 16) a += part[(long long)b * C + c];
  sa[ty][tx] = a;
  __syncthreads();
  if (ty == 0 && c < C) {
    a = 0;
#pragma unroll
    for (int k = 0; k < 16; ++k) a += sa[k][tx];
    out[c] = (float)a;
  }
}

// ------------------------------------------------------------------ BN backward
// partial[bx][2C]: per-channel sums of g and g*xhat over the block's rows, g = dout * mask.
// Each thread owns one 16-B channel chunk for the whole block (cpr <= 256: 256/cpr threads share a
// chunk and walk interleaved rows; cpr > 256: blockIdx.y selects 256 chunks, threads walk all rows),
// and threads sharing a chunk are combined through LDS in a fixed order: deterministic.
template <typename T, int MODE>
__global__ __launch_bounds__(256) void bn_bwd_reduce_kernel(const T* __restrict__ dout, MaskArgs mk,
                                                            const T* __restrict__ y, const float* __restrict__ mean,
                                                            const float* __restrict__ invstd, long long P, int cpr,
                                                            int C, int rows_per_block, float* __restrict__ partial) {
  constexpr int VN = V<T>::N;
  __shared__ float part[2][256][VN];
  const int tid = threadIdx.x;
  const bool narrow = cpr <= 256;
  const int chunk = narrow ? (tid & (cpr - 1)) : (blockIdx.y * 256 + tid);
  const int rstep = narrow ? 256 / cpr : 1;
  const long long r0 = (long long)blockIdx.x * rows_per_block;
  const long long r1 = min(P, r0 + rows_per_block);
  const int c0 = chunk * VN;
  float mu[VN], is[VN], sg[VN], sx[VN], msc[VN], msh[VN];
  load_params<VN>(mean, c0, mu);
  load_params<VN>(invstd, c0, is);
  if (MODE == 3) {
    load_params<VN>(mk.sc, c0, msc);
    load_params<VN>(mk.sh, c0, msh);
  }
#pragma unroll
  for (int e = 0; e < VN; ++e) { sg[e] = 0.f; sx[e] = 0.f; }
  for (long long r = r0 + (narrow ? tid / cpr : 0); r < r1; r += (long long)rstep * SU) {
    float d[SU][VN], yv[SU][VN];
#pragma unroll
    for (int u = 0; u < SU; ++u) {  // unconditional loads (clamped row): no per-vector branch + wait
      const long long rr = min(r + (long long)u * rstep, r1 - 1);
      const long long v = rr * cpr + chunk;
      load16<T>(dout + v * VN, d[u]);
      load16<T>(y + v * VN, yv[u]);
    }
#pragma unroll
    for (int u = 0; u < SU; ++u) {
      const long long rr = r + (long long)u * rstep;
      if (rr >= r1) break;
      const long long v = rr * cpr + chunk;
      if (MODE != 0) {
        MaskArgs m = mk;
        m.mode = MODE;
        apply_mask<T, VN>(d[u], m, v, yv[u], msc, msh);
      }
#pragma unroll
      for (int e = 0; e < VN; ++e) {
        sg[e] += d[u][e];
        sx[e] += d[u][e] * (yv[u][e] - mu[e]) * is[e];
      }
    }
  }
  float* out = partial + (long long)blockIdx.x * 2 * C;
  if (!narrow) {
#pragma unroll
    for (int e = 0; e < VN; ++e) {
      out[c0 + e] = sg[e];
      out[C + c0 + e] = sx[e];
    }
    return;
  }
#pragma unroll
  for (int e = 0; e < VN; ++e) {
    part[0][tid][e] = sg[e];
    part[1][tid][e] = sx[e];
  }
  __syncthreads();
  for (int i = tid; i < 2 * C; i += 256) {
    const int which = i >= C, c = i - which * C;
    const int ch = c / VN, e = c - ch * VN;
    float acc = 0.f;
    for (int k = ch; k < 256; k += cpr) acc += part[which][k][e];
    out[i] = acc;
  }
}

// Column sums of partial[nb][2C] -> sum_g, sum_gx (+ dgamma/dbeta): 16 channels x 16 row-stripes per 256-thread
// block, loads coalesced across channels and unrolled across rows; fixed summation order (deterministic: thread ty sums
// rows ty, ty + 16, ... in double, then the 16 stripes in order). (It ran with 64 channels x 16 stripes per 1024-thread
// block: on a GPU busy with the side streams' kernels a 16-wave workgroup waited ~30 us for a CU to take it -- 53
// of these per train step sit on the trunk's critical path, tools/queue_busy.py.)
// (row i of partial: sum_g at [i * ld + c], sum_gx at [i * ld + gx_off + c]; ld = 2C / gx_off = C for
// bn_bwd_reduce's partials)
__global__ __launch_bounds__(256) void bn_bwd_finalize_kernel(const float* __restrict__ partial, int nb, int C,
                                                              long long ld, int gx_off, float* sum_g, float* sum_gx,
                                                              float* dgamma, float* dbeta, int accumulate) {
  __shared__ double sa[16][16], sb[16][16];
  const int tx = threadIdx.x & 15, ty = threadIdx.x >> 4;
  const int c = blockIdx.x * 16 + tx;
  double a = 0, b = 0;
  if (c < C) {
    const float* p = partial + c;
#pragma unroll 4
    for (int i = ty; i < nb; i += 16) {
      a += p[i * ld];
      b += p[i * ld + gx_off];
    }
  }
  sa[ty][tx] = a;
  sb[ty][tx] = b;
  __syncthreads();
  if (ty == 0 && c < C) {
    a = 0;
    b = 0;
#pragma unroll
    for (int k = 0; k < 16; ++k) {
      a += sa[k][tx];
      b += sb[k][tx];
    }
    sum_g[c] = (float)a;
    sum_gx[c] = (float)b;
    if (dbeta) dbeta[c] = (accumulate ? dbeta[c] : 0.f) + (float)a;
    if (dgamma) dgamma[c] = (accumulate ? dgamma[c] : 0.f) + (float)b;
  }
}

// dy = A*g + B*y + Cc per channel (batch-stat BN backward folded to an affine map of (g, y)):
//   A = gamma*invstd, B = -A*invstd*sum_gx/N, Cc = -A*sum_g/N - B*mean ; running mode: dy = A*g.
// optionally gout = g (masked upstream gradient: the residual path)
template <typename T, int MODE, bool TRAIN>
__global__ __launch_bounds__(256) void bn_bwd_apply_kernel(const T* __restrict__ dout, MaskArgs mk,
                                                           const T* __restrict__ y, const float* __restrict__ mean,
                                                           const float* __restrict__ invstd,
                                                           const float* __restrict__ gamma,
                                                           const float* __restrict__ sum_g,
                                                           const float* __restrict__ sum_gx, float inv_count,
                                                           T* __restrict__ dy, T* __restrict__ gout, long long TV,
                                                           int cpr) {
  constexpr int VN = V<T>::N;
  constexpr bool NEED_Y = TRAIN || MODE == 3;
  const long long stride = (long long)gridDim.x * SB;
  long long base = (long long)blockIdx.x * SB + threadIdx.x;
  const bool fixed = cpr <= 256;
  float A[VN], Bc[VN], Cc[VN], msc[VN], msh[VN];
  auto params = [&](long long v) {
    const int c0 = (int)(v & (cpr - 1)) * VN;
    float is[VN];
    load_params<VN>(invstd, c0, is);
#pragma unroll
    for (int e = 0; e < VN; ++e) A[e] = (gamma ? gamma[c0 + e] : 1.f) * is[e];
    if (TRAIN) {
      float sgx[VN], sgg[VN], mu[VN];
      load_params<VN>(sum_gx, c0, sgx);
      load_params<VN>(sum_g, c0, sgg);
      load_params<VN>(mean, c0, mu);
#pragma unroll
      for (int e = 0; e < VN; ++e) {
        Bc[e] = -A[e] * is[e] * sgx[e] * inv_count;
        Cc[e] = -A[e] * sgg[e] * inv_count - Bc[e] * mu[e];
      }
    }
    if (MODE == 3) {
      load_params<VN>(mk.sc, c0, msc);
      load_params<VN>(mk.sh, c0, msh);
    }
  };
  params(base);
  for (; base < TV; base += stride) {
    float d[SU][VN], yv[SU][VN];
#pragma unroll
    for (int u = 0; u < SU; ++u) {  // unconditional loads (clamped index): no per-vector branch + wait
      const long long v = min(base + u * 256, TV - 1);
      load16<T>(dout + v * VN, d[u]);
      if (NEED_Y) load16<T>(y + v * VN, yv[u]);
    }
#pragma unroll
    for (int u = 0; u < SU; ++u) {
      const long long v = base + u * 256;
      if (v >= TV) break;
      if (!fixed) params(v);
      if (MODE != 0) {
        MaskArgs m = mk;
        m.mode = MODE;
        apply_mask<T, VN>(d[u], m, v, yv[u], msc, msh);
      }
      if (gout) store16<T>(gout + v * VN, d[u]);
      float o[VN];
#pragma unroll
      for (int e = 0; e < VN; ++e) o[e] = TRAIN ? fmaf(A[e], d[u][e], fmaf(Bc[e], yv[u][e], Cc[e])) : A[e] * d[u][e];
      store16<T>(dy + v * VN, o);
    }
  }
}

// Two batch-stat BN backward applies sharing the upstream gradient g (already masked): the first bottleneck of a
// ResNet layer, where bn3 and the downsample BN both follow the block's output ReLU. g is read once:
// dy = A g + B y + C (bn3) and dyd = Ad g + Bd yd + Cd (downsample BN), each with bn_bwd_apply_kernel's arithmetic.
struct BnBwdArgs {
  const float *mean, *invstd, *gamma, *sum_g, *sum_gx;
};
template <typename T>
__global__ __launch_bounds__(256) void bn_bwd_apply_dual_kernel(const T* __restrict__ g, const T* __restrict__ y,
                                                                const T* __restrict__ yd, BnBwdArgs p1, BnBwdArgs p2,
                                                                float inv_count, T* __restrict__ dy,
                                                                T* __restrict__ dyd, long long TV, int cpr) {
  constexpr int VN = V<T>::N;
  const long long stride = (long long)gridDim.x * SB;
  long long base = (long long)blockIdx.x * SB + threadIdx.x;
  const bool fixed = cpr <= 256;
  float A[2][VN], Bc[2][VN], Cc[2][VN];
  auto params = [&](long long v) {
    const int c0 = (int)(v & (cpr - 1)) * VN;
#pragma unroll
    for (int k = 0; k < 2; ++k) {
      const BnBwdArgs& b = k ? p2 : p1;
      float is[VN], sgx[VN], sgg[VN], mu[VN];
      load_params<VN>(b.invstd, c0, is);
      load_params<VN>(b.sum_gx, c0, sgx);
      load_params<VN>(b.sum_g, c0, sgg);
      load_params<VN>(b.mean, c0, mu);
#pragma unroll
      for (int e = 0; e < VN; ++e) {
        A[k][e] = (b.gamma ? b.gamma[c0 + e] : 1.f) * is[e];
        Bc[k][e] = -A[k][e] * is[e] * sgx[e] * inv_count;
        Cc[k][e] = -A[k][e] * sgg[e] * inv_count - Bc[k][e] * mu[e];
      }
    }
  };
  params(base);
  for (; base < TV; base += stride) {
    float d[SU][VN], y1[SU][VN], y2[SU][VN];
#pragma unroll
    for (int u = 0; u < SU; ++u) {  // unconditional loads (clamped index)
      const long long v = min(base + u * 256, TV - 1);
      load16<T>(g + v * VN, d[u]);
      load16<T>(y + v * VN, y1[u]);
      load16<T>(yd + v * VN, y2[u]);
    }
#pragma unroll
    for (int u = 0; u < SU; ++u) {
      const long long v = base + u * 256;
      if (v >= TV) break;
      if (!fixed) params(v);
      float o[VN], od[VN];
#pragma unroll
      for (int e = 0; e < VN; ++e) {
        o[e] = fmaf(A[0][e], d[u][e], fmaf(Bc[0][e], y1[u][e], Cc[0][e]));
        od[e] = fmaf(A[1][e], d[u][e], fmaf(Bc[1][e], y2[u][e], Cc[1][e]));
      }
      store16<T>(dy + v * VN, o);
      store16<T>(dyd + v * VN, od);
    }
  }
}

// ------------------------------------------------------------------ max pool 3x3 / 2, pad 1
// thread = (output pixel, 16-B channel chunk); first max in (kh, kw) scan order (torch CPU semantics);
// the argmax bytes of a chunk are stored as one VN-byte word
template <int VN> struct IdxWord;
template <> struct IdxWord<8> { typedef uint2 t; };
template <> struct IdxWord<4> { typedef uint32_t t; };
template <int VN> __device__ __forceinline__ void idx_store(uint8_t* p, const uint8_t (&b)[VN]) {
  if constexpr (VN == 8) {
    uint2 q;
    q.x = b[0] | (b[1] << 8) | (b[2] << 16) | ((uint32_t)b[3] << 24);
    q.y = b[4] | (b[5] << 8) | (b[6] << 16) | ((uint32_t)b[7] << 24);
    *reinterpret_cast<uint2*>(p) = q;
  } else {
    *reinterpret_cast<uint32_t*>(p) = b[0] | (b[1] << 8) | (b[2] << 16) | ((uint32_t)b[3] << 24);
  }
}
template <int VN> __device__ __forceinline__ uint8_t idx_byte(const typename IdxWord<VN>::t& w, int e) {
  if constexpr (VN == 8) return (uint8_t)(((e < 4 ? w.x : w.y) >> (8 * (e & 3))) & 0xFF);
  else return (uint8_t)((w >> (8 * e)) & 0xFF);
}

// BN: the input is the stem conv output y and the pooled values are a = relu(fma(y, scale, shift)) rounded to T
// exactly as vcg_bn_apply stores them (the fused stem: no a tensor in HBM, same pooled values and argmax)
template <typename T, bool BN>
__global__ __launch_bounds__(256) void maxpool_fwd_kernel(const T* __restrict__ x, T* __restrict__ y,
                                                          uint8_t* __restrict__ idx, int H, int W, int C, int OH,
                                                          int OW, int lcpr, long long TV, FastDiv fd_ow, FastDiv fd_oh,
                                                          const float* __restrict__ scale = nullptr,
                                                          const float* __restrict__ shift = nullptr) {
  constexpr int VN = V<T>::N;
  const long long v = (long long)blockIdx.x * 256 + threadIdx.x;
  if (v >= TV) return;
  const int chunk = (int)(v & ((1 << lcpr) - 1));
  float sc[VN], sh[VN];
  if (BN) {
    load_params<VN>(scale, chunk * VN, sc);
    load_params<VN>(shift, chunk * VN, sh);
  }
  const int pix = (int)(v >> lcpr);
  const int t = (int)fdiv((uint32_t)pix, fd_ow);
  const int ow = pix - t * OW;
  const int n = (int)fdiv((uint32_t)t, fd_oh);
  const int oh = t - n * OH;
  float best[VN];
  uint8_t bi[VN];
#pragma unroll
  for (int e = 0; e < VN; ++e) { best[e] = -INFINITY; bi[e] = 0; }
  // all 9 window loads first, from clamped (always valid) pixels; padding taps are dropped after the load (a
  // load under a per-tap condition makes hipcc wait for each one separately)
  float a[9][VN];
#pragma unroll
  for (int k = 0; k < 9; ++k) {
    const int ih = min(max(oh * 2 - 1 + k / 3, 0), H - 1), iw = min(max(ow * 2 - 1 + k % 3, 0), W - 1);
    load16<T>(x + (((long long)n * H + ih) * W + iw) * C + chunk * VN, a[k]);
  }
#pragma unroll
  for (int k = 0; k < 9; ++k) {
    const int ih = oh * 2 - 1 + k / 3, iw = ow * 2 - 1 + k % 3;
    if (ih < 0 || ih >= H || iw < 0 || iw >= W) continue;
    if (BN) {
#pragma unroll
      for (int e = 0; e < VN; ++e) a[k][e] = to_f<T>(from_f<T>(fmaxf(fmaf(a[k][e], sc[e], sh[e]), 0.f)));
    }
#pragma unroll
    for (int e = 0; e < VN; ++e)
      if (a[k][e] > best[e] || isnan(a[k][e])) { best[e] = a[k][e]; bi[e] = (uint8_t)k; }
  }
  store16<T>(y + v * VN, best);
  idx_store<VN>(idx + v * VN, bi);
}

// Two horizontally adjacent outputs per thread (ow0 = 2 owp, ow0 + 1): their windows share the middle column, so
// the 3 x 5 input pixels are loaded (and, fused, BN + ReLU transformed) once -- 15 instead of 18 per 2 outputs. The
// scan per output is maxpool_fwd_kernel's (taps in (kh, kw) order, first max, NaN wins): same values and argmax.
template <typename T, bool BN>
__global__ __launch_bounds__(256) void maxpool_fwd2_kernel(const T* __restrict__ x, T* __restrict__ y,
                                                           uint8_t* __restrict__ idx, int H, int W, int C, int OH,
                                                           int OW, int lcpr, long long TV2, FastDiv fd_ow2,
                                                           FastDiv fd_oh, const float* __restrict__ scale = nullptr,
                                                           const float* __restrict__ shift = nullptr) {
  constexpr int VN = V<T>::N;
  const long long v = (long long)blockIdx.x * 256 + threadIdx.x;
  if (v >= TV2) return;
  const int chunk = (int)(v & ((1 << lcpr) - 1));
  float sc[VN], sh[VN];
  if (BN) {
    load_params<VN>(scale, chunk * VN, sc);
    load_params<VN>(shift, chunk * VN, sh);
  }
  const int pp = (int)(v >> lcpr);  // (n, oh, owp)
  const int t = (int)fdiv((uint32_t)pp, fd_ow2);
  const int owp = pp - t * (int)fd_ow2.d;
  const int n = (int)fdiv((uint32_t)t, fd_oh);
  const int oh = t - n * OH;
  const int ow0 = 2 * owp;
  float a[3][5][VN];
#pragma unroll
  for (int r = 0; r < 3; ++r)
#pragma unroll
    for (int c = 0; c < 5; ++c) {
      const int ih = min(max(oh * 2 - 1 + r, 0), H - 1), iw = min(max(ow0 * 2 - 1 + c, 0), W - 1);
      load16<T>(x + (((long long)n * H + ih) * W + iw) * C + chunk * VN, a[r][c]);
    }
  if (BN) {
#pragma unroll
    for (int r = 0; r < 3; ++r)
#pragma unroll
      for (int c = 0; c < 5; ++c)
#pragma unroll
        for (int e = 0; e < VN; ++e) a[r][c][e] = to_f<T>(from_f<T>(fmaxf(fmaf(a[r][c][e], sc[e], sh[e]), 0.f)));
  }
#pragma unroll
  for (int o = 0; o < 2; ++o) {
    const int ow = ow0 + o;
    if (ow >= OW) break;
    float best[VN];
    uint8_t bi[VN];
#pragma unroll
    for (int e = 0; e < VN; ++e) { best[e] = -INFINITY; bi[e] = 0; }
#pragma unroll
    for (int k = 0; k < 9; ++k) {
      const int r = k / 3, c = k % 3 + 2 * o;
      const int ih = oh * 2 - 1 + r, iw = ow * 2 - 1 + k % 3;
      if (ih < 0 || ih >= H || iw < 0 || iw >= W) continue;
#pragma unroll
      for (int e = 0; e < VN; ++e)
        if (a[r][c][e] > best[e] || isnan(a[r][c][e])) { best[e] = a[r][c][e]; bi[e] = (uint8_t)k; }
    }
    const long long vo = ((((long long)n * OH + oh) * OW + ow) << lcpr) + chunk;
    store16<T>(y + vo * VN, best);
    idx_store<VN>(idx + vo * VN, bi);
  }
}

// thread = (input pixel, chunk): sums dy over the <= 4 windows whose argmax is this pixel. Grid-stride with
// a fixed chunk per thread (cpr <= 256). MODE (the stem's BN + ReLU backward around the pool):
//   MP_PLAIN: dx = that sum;
//   MP_RED / MP_RED_ONLY: g = the sum masked by the forward ReLU (fma(y, msc, msh) > 0), stored (MP_RED) or not,
//     and reduced into per-block partials part[block][2C] of sum g and sum g * (y - mean) * invstd (the
//     BatchNorm backward sums; bn_bwd_finalize_kernel) -- of g as stored (rounded to T);
//   MP_APPLY: the same g (rounded to T) through the BatchNorm backward apply of bn_bwd_apply_kernel,
//     dx = A g + B y + Cc (train statistics) or A g (running), so the stem needs no g tensor in HBM.
enum { MP_PLAIN = 0, MP_RED = 1, MP_RED_ONLY = 2, MP_APPLY = 3 };
struct MpBn {
  const float *mean, *invstd, *msc, *msh;
  float* part;
  const float *gamma, *sum_g, *sum_gx;  // MP_APPLY
  float inv_count;
  int train;
};
template <typename T, int MODE>
__global__ __launch_bounds__(256) void maxpool_bwd_kernel(const T* __restrict__ dy, const uint8_t* __restrict__ idx,
                                                          T* __restrict__ dx, int H, int W, int C, int OH, int OW,
                                                          int lcpr, long long TV, const T* __restrict__ yb, MpBn bn,
                                                          FastDiv fd_w, FastDiv fd_h) {
  constexpr int VN = V<T>::N;
  constexpr bool RED = MODE == MP_RED || MODE == MP_RED_ONLY;
  constexpr bool MASK = MODE != MP_PLAIN;
  typedef typename IdxWord<VN>::t IW;
  __shared__ float red[RED ? 2 : 1][RED ? 256 : 1][VN];
  const int cpr = 1 << lcpr;
  const int chunk = threadIdx.x & (cpr - 1);
  const int c0 = chunk * VN;
  float mu[VN], sc[VN], sh[VN], s1[VN], s2[VN], A[VN], Bc[VN], Cc[VN];
  if (MASK) {
    load_params<VN>(bn.mean, c0, mu);
    load_params<VN>(bn.msc, c0, sc);
    load_params<VN>(bn.msh, c0, sh);
#pragma unroll
    for (int e = 0; e < VN; ++e) s1[e] = s2[e] = 0.f;
  }
  if (MODE == MP_APPLY) {  // bn_bwd_apply_kernel's affine map, same arithmetic
    float is[VN], sgx[VN], sgg[VN];
    load_params<VN>(bn.invstd, c0, is);
    load_params<VN>(bn.sum_gx, c0, sgx);
    load_params<VN>(bn.sum_g, c0, sgg);
#pragma unroll
    for (int e = 0; e < VN; ++e) {
      A[e] = (bn.gamma ? bn.gamma[c0 + e] : 1.f) * is[e];
      Bc[e] = -A[e] * is[e] * sgx[e] * bn.inv_count;
      Cc[e] = -A[e] * sgg[e] * bn.inv_count - Bc[e] * mu[e];
    }
  }
  for (long long v = (long long)blockIdx.x * 256 + threadIdx.x; v < TV; v += (long long)gridDim.x * 256) {
    const int pix = (int)(v >> lcpr);
    const int t = (int)fdiv((uint32_t)pix, fd_w);
    const int iw = pix - t * W;
    const int n = (int)fdiv((uint32_t)t, fd_h);
    const int ih = t - n * H;
    float acc[VN];
#pragma unroll
    for (int e = 0; e < VN; ++e) acc[e] = 0.f;
    // the <= 2 x 2 windows with 2*oh-1 <= ih <= 2*oh+1: every candidate's loads are issued before any is used
    const int oh0 = ih >> 1, oh1 = (ih + 1) >> 1;
    const int ow0 = iw >> 1, ow1 = (iw + 1) >> 1;
    float yv[VN];
    if (MASK) load16<T>(yb + v * VN, yv);
    float g[4][VN];
    IW w[4];
    bool use[4];
    uint8_t want[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int oh = (q & 2) ? oh1 : oh0, ow = (q & 1) ? ow1 : ow0;
      use[q] = (!(q & 2) || oh1 != oh0) && (!(q & 1) || ow1 != ow0) && oh < OH && ow < OW;
      want[q] = (uint8_t)((ih - (oh * 2 - 1)) * 3 + (iw - (ow * 2 - 1)));
      const long long o = (((long long)n * OH + min(oh, OH - 1)) * OW + min(ow, OW - 1)) * C + chunk * VN;
      load16<T>(dy + o, g[q]);  // unconditional (clamped) loads: see maxpool_fwd_kernel
      w[q] = *reinterpret_cast<const IW*>(idx + o);
    }
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      if (!use[q]) continue;
#pragma unroll
      for (int e = 0; e < VN; ++e)
        if (idx_byte<VN>(w[q], e) == want[q]) acc[e] += g[q][e];
    }
    if (MASK) {
#pragma unroll
      for (int e = 0; e < VN; ++e) {
        acc[e] = fmaf(yv[e], sc[e], sh[e]) > 0.f ? acc[e] : 0.f;
        const float gr = to_f<T>(from_f<T>(acc[e]));  // the gradient as stored
        if (RED) {
          s1[e] += gr;
          s2[e] = fmaf(gr, yv[e] - mu[e], s2[e]);
        } else {
          acc[e] = bn.train ? fmaf(A[e], gr, fmaf(Bc[e], yv[e], Cc[e])) : A[e] * gr;  // bn_bwd_apply_kernel's order
        }
      }
    }
    if (MODE != MP_RED_ONLY) store16<T>(dx + v * VN, acc);
  }
  if (RED) {
#pragma unroll
    for (int e = 0; e < VN; ++e) {
      red[0][threadIdx.x][e] = s1[e];
      red[1][threadIdx.x][e] = s2[e];
    }
    __syncthreads();
    for (int i = threadIdx.x; i < 2 * C; i += 256) {
      const int which = i >= C, c = i - which * C;
      const int ch = c / VN, e = c - ch * VN;
      float a = 0.f;
      for (int k = ch; k < 256; k += cpr) a += red[which][k][e];
      if (which) a *= bn.invstd[c];
      bn.part[(long long)blockIdx.x * 2 * C + i] = a;
    }
  }
}

// The same backward with one thread per (2x2 input block, chunk) for even H and W: the block's 4 pixels are
// reached by the 4 windows (k + {0,1}, j + {0,1}) only, so the 4 windows' dy / argmax loads and the index math are
// shared by 4 pixels (9 pixel-window pairs: (0,0) <- 1 window, (0,1) / (1,0) <- 2, (1,1) <- 4); the per-pixel
// work (ReLU mask, rounding, sums or BN apply) is the per-pixel kernel's, in the same order.
template <typename T, int MODE>
__global__ __launch_bounds__(256) void maxpool_bwd2_kernel(const T* __restrict__ dy, const uint8_t* __restrict__ idx,
                                                           T* __restrict__ dx, int H, int W, int C, int OH, int OW,
                                                           int lcpr, long long TB, const T* __restrict__ yb, MpBn bn,
                                                           FastDiv fd_bw, FastDiv fd_bh) {
  constexpr int VN = V<T>::N;
  constexpr bool RED = MODE == MP_RED || MODE == MP_RED_ONLY;
  constexpr bool MASK = MODE != MP_PLAIN;
  typedef typename IdxWord<VN>::t IW;
  __shared__ float red[RED ? 2 : 1][RED ? 256 : 1][VN];
  const int cpr = 1 << lcpr;
  const int chunk = threadIdx.x & (cpr - 1);
  const int c0 = chunk * VN;
  const int BW = W >> 1, BH = H >> 1;
  float mu[VN], sc[VN], sh[VN], s1[VN], s2[VN], A[VN], Bc[VN], Cc[VN];
  if (MASK) {
    load_params<VN>(bn.mean, c0, mu);
    load_params<VN>(bn.msc, c0, sc);
    load_params<VN>(bn.msh, c0, sh);
#pragma unroll
    for (int e = 0; e < VN; ++e) s1[e] = s2[e] = 0.f;
  }
  if (MODE == MP_APPLY) {
    float is[VN], sgx[VN], sgg[VN];
    load_params<VN>(bn.invstd, c0, is);
    load_params<VN>(bn.sum_gx, c0, sgx);
    load_params<VN>(bn.sum_g, c0, sgg);
#pragma unroll
    for (int e = 0; e < VN; ++e) {
      A[e] = (bn.gamma ? bn.gamma[c0 + e] : 1.f) * is[e];
      Bc[e] = -A[e] * is[e] * sgx[e] * bn.inv_count;
      Cc[e] = -A[e] * sgg[e] * bn.inv_count - Bc[e] * mu[e];
    }
  }
  for (long long b = (long long)blockIdx.x * 256 + threadIdx.x; b < TB; b += (long long)gridDim.x * 256) {
    const int blk = (int)(b >> lcpr);
    const int t = (int)fdiv((uint32_t)blk, fd_bw);
    const int j = blk - t * BW;
    const int n = (int)fdiv((uint32_t)t, fd_bh);
    const int k = t - n * BH;
    // windows q = 2 dr + dc at (k + dr, j + dc)
    float g[4][VN];
    IW w[4];
    bool use[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int oh = k + (q >> 1), ow = j + (q & 1);
      use[q] = oh < OH && ow < OW;
      const long long o = (((long long)n * OH + min(oh, OH - 1)) * OW + min(ow, OW - 1)) * C + c0;
      load16<T>(dy + o, g[q]);  // unconditional (clamped) loads: see maxpool_fwd_kernel
      w[q] = *reinterpret_cast<const IW*>(idx + o);
    }
    float yv[4][VN];
    long long pv[4];
#pragma unroll
    for (int pp = 0; pp < 4; ++pp) {  // pixel (2k + a, 2j + c), pp = 2a + c
      pv[pp] = ((((long long)n * H + 2 * k + (pp >> 1)) * W + 2 * j + (pp & 1)) << lcpr) + chunk;
      if (MASK) load16<T>(yb + pv[pp] * VN, yv[pp]);
    }
#pragma unroll
    for (int pp = 0; pp < 4; ++pp) {
      const int a = pp >> 1, c = pp & 1;
      float acc[VN];
#pragma unroll
      for (int e = 0; e < VN; ++e) acc[e] = 0.f;
      // windows in the per-pixel kernel's order (oh0, ow0), (oh0, ow1), (oh1, ow0), (oh1, ow1): kh = a + 1 - 2 dr
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int dr = q >> 1, dc = q & 1;
        if ((dr && !a) || (dc && !c)) continue;  // window row / column does not contain this pixel
        if (!use[q]) continue;
        const uint8_t want = (uint8_t)((a + 1 - 2 * dr) * 3 + (c + 1 - 2 * dc));
#pragma unroll
        for (int e = 0; e < VN; ++e)
          if (idx_byte<VN>(w[q], e) == want) acc[e] += g[q][e];
      }
      if (MASK) {
#pragma unroll
        for (int e = 0; e < VN; ++e) {
          acc[e] = fmaf(yv[pp][e], sc[e], sh[e]) > 0.f ? acc[e] : 0.f;
          const float gr = to_f<T>(from_f<T>(acc[e]));
          if (RED) {
            s1[e] += gr;
            s2[e] = fmaf(gr, yv[pp][e] - mu[e], s2[e]);
          } else {
            acc[e] = bn.train ? fmaf(A[e], gr, fmaf(Bc[e], yv[pp][e], Cc[e])) : A[e] * gr;
          }
        }
      }
      if (MODE != MP_RED_ONLY) store16<T>(dx + pv[pp] * VN, acc);
    }
  }
  if (RED) {
#pragma unroll
    for (int e = 0; e < VN; ++e) {
      red[0][threadIdx.x][e] = s1[e];
      red[1][threadIdx.x][e] = s2[e];
    }
    __syncthreads();
    for (int i = threadIdx.x; i < 2 * C; i += 256) {
      const int which = i >= C, c = i - which * C;
      const int ch = c / VN, e = c - ch * VN;
      float a = 0.f;
      for (int kk = ch; kk < 256; kk += cpr) a += red[which][kk][e];
      if (which) a *= bn.invstd[c];
      bn.part[(long long)blockIdx.x * 2 * C + i] = a;
    }
  }
}

// The stem BatchNorm-backward sums from the POOLED activation instead of y: every window's gradient goes to one
// pixel (its argmax), whose ReLU output is the window's max mp -- so the pixel passes the ReLU mask iff mp > 0, and
// its normalised value is recovered from mp (z = y msc + msh => y - mean = (mp - msh) / msc - mean for mp > 0).
// Both sums are linear in the per-pixel gradient, so they are sums over windows: sum_g = sum [mp > 0] dy,
// sum_gx = invstd * sum [mp > 0] dy (y - mean). Reads dy and mp once (1/2 of the output rows' bytes each) instead
// of dy, the argmax bytes and the whole pre-pool y (the stem's conv output, 4x the pooled size). mp is the bf16
// max, so y - mean carries one bf16 rounding of the activation (the per-pixel path carries that of y).
// Degenerate channels -- msc == 0 (a zero BN weight: mp says nothing about y) or |msh| > 32 |gamma| (the recovery
// cancels: its error is ~2^-9 |msh| / |gamma| of a std) -- contribute no sum_gx here; maxpool_bn_sums_degen_kernel
// adds theirs from y at the windows' argmax pixels in a slot of its own. (A per-element gather branch inside this
// loop, never taken on the bench, cost the train step ~1 % on the same box: profiles/r05_degen_branch_ab.txt.)
__device__ __forceinline__ bool pooled_degen(float sc, float sh, float is) {
  return sc == 0.f || !(fabsf(sh) * is <= 32.f * fabsf(sc));
}

template <typename T>
__global__ __launch_bounds__(256) void maxpool_bn_sums_pooled_kernel(const T* __restrict__ dy, const T* __restrict__ mp,
                                                                     long long TV, int lcpr, MpBn bn) {
  constexpr int VN = V<T>::N;
  __shared__ float red[2][256][VN];
  const int cpr = 1 << lcpr;
  const int chunk = threadIdx.x & (cpr - 1);
  const int c0 = chunk * VN;
  const int C = cpr * VN;
  float mu[VN], sc[VN], sh[VN], is[VN], rsc[VN], off[VN], s1[VN], s2[VN];
  load_params<VN>(bn.mean, c0, mu);
  load_params<VN>(bn.msc, c0, sc);
  load_params<VN>(bn.msh, c0, sh);
  load_params<VN>(bn.invstd, c0, is);
#pragma unroll
  for (int e = 0; e < VN; ++e) {
    const bool dg = pooled_degen(sc[e], sh[e], is[e]);
    rsc[e] = dg ? 0.f : 1.f / sc[e];
    off[e] = dg ? 0.f : -sh[e] * rsc[e] - mu[e];  // y - mean = mp / msc + off
    s1[e] = s2[e] = 0.f;
  }
  const long long stride = (long long)gridDim.x * SB;
  for (long long base = (long long)blockIdx.x * SB + threadIdx.x; base < TV; base += stride) {
    float g[SU][VN], m[SU][VN];
#pragma unroll
    for (int u = 0; u < SU; ++u) {  // unconditional (clamped) loads, as bn_apply_kernel
      const long long v = min(base + u * 256, TV - 1);
      load16<T>(dy + v * VN, g[u]);
      load16<T>(mp + v * VN, m[u]);
    }
#pragma unroll
    for (int u = 0; u < SU; ++u) {
      if (base + u * 256 >= TV) break;
#pragma unroll
      for (int e = 0; e < VN; ++e) {
        const float d = m[u][e] > 0.f ? g[u][e] : 0.f;
        s1[e] += d;
        s2[e] = fmaf(d, fmaf(m[u][e], rsc[e], off[e]), s2[e]);
      }
    }
  }
#pragma unroll
  for (int e = 0; e < VN; ++e) {
    red[0][threadIdx.x][e] = s1[e];
    red[1][threadIdx.x][e] = s2[e];
  }
  __syncthreads();
  for (int i = threadIdx.x; i < 2 * C; i += 256) {
    const int which = i >= C, c = i - which * C;
    const int ch = c / VN, e = c - ch * VN;
    float a = 0.f;
    for (int kk = ch; kk < 256; kk += cpr) a += red[which][kk][e];
    if (which) a *= bn.invstd[c];
    bn.part[(long long)blockIdx.x * 2 * C + i] = a;
  }
}

// sum_gx of the degenerate channels (pooled_degen) of maxpool_bn_sums_pooled_kernel, into the partial slot `slot`:
// one workgroup per channel; a regular channel writes zeros and returns at once (the bench's case: no channel is
// degenerate), a degenerate one sums dy (y - mean) over the windows that pass the mask, y read at the argmax pixel
// (idx byte k: pixel (2 oh - 1 + k / 3, 2 ow - 1 + k % 3) of the [N][H][W][C] pre-pool y), in a fixed order.
template <typename T>
__global__ __launch_bounds__(256) void maxpool_bn_sums_degen_kernel(const T* __restrict__ dy, const T* __restrict__ mp,
                                                                    const uint8_t* __restrict__ idx,
                                                                    const T* __restrict__ y, int H, int W, int OH,
                                                                    int OW, long long npix, int C, MpBn bn, int slot) {
  __shared__ float red[256];
  const int c = blockIdx.x, tid = threadIdx.x;
  const float sc = bn.msc[c], sh = bn.msh[c], is = bn.invstd[c], mu = bn.mean[c];
  float* out = bn.part + (long long)slot * 2 * C;
  if (!pooled_degen(sc, sh, is)) {
    if (tid == 0) out[c] = out[C + c] = 0.f;
    return;
  }
  float s2 = 0.f;
  for (long long v = tid; v < npix; v += 256) {
    const float m = to_f<T>(mp[v * C + c]);
    if (!(m > 0.f)) continue;
    const int ow = (int)(v % OW);
    const long long t = v / OW;
    const int oh = (int)(t % OH);
    const long long n = t / OH;
    const int k = idx[v * C + c];
    const int ih = 2 * oh - 1 + k / 3, iw = 2 * ow - 1 + k % 3;
    s2 = fmaf(to_f<T>(dy[v * C + c]), to_f<T>(y[((n * H + ih) * W + iw) * C + c]) - mu, s2);
  }
  red[tid] = s2;
  __syncthreads();
  if (tid == 0) {
    float a = 0.f;
    for (int t = 0; t < 256; ++t) a += red[t];
    out[c] = 0.f;  // (sum_g: the main pass counts every channel)
    out[C + c] = a * is;
  }
}

// ------------------------------------------------------------------ TSM gradient combine
// dx = unshift(dshift) + other over NHWC [N*T][H][W][C] (adjoint of ops/temporal_shift.py:45-47)
template <typename T, bool OTHER, bool BITS>
__global__ __launch_bounds__(256) void tsm_unshift_add_kernel(const T* __restrict__ dshift, const T* __restrict__ other,
                                                              const uint8_t* __restrict__ other_bits,
                                                              T* __restrict__ dx, unsigned TV, int lcpr,
                                                              unsigned row_vecs, int Tn, int fold_chunks) {
  constexpr int VN = V<T>::N;
  const unsigned stride = gridDim.x * SB;
  const int cmask = (1 << lcpr) - 1;
  for (unsigned base = blockIdx.x * SB + threadIdx.x; base < TV; base += stride) {
    float a[SU][VN], b[SU][VN];
    unsigned m[SU];
#pragma unroll
    for (int u = 0; u < SU; ++u) {
      const unsigned v = base + u * 256;
      if (v >= TV) continue;
      const int chunk = (int)(v & cmask);
      int dt = 0;
      if (chunk < fold_chunks) dt = -1;
      else if (chunk < 2 * fold_chunks) dt = 1;
      bool have = true;
      if (dt != 0) {
        const int t = (int)((v / row_vecs) % (unsigned)Tn);
        have = (t + dt >= 0) && (t + dt < Tn);
      }
      if (have) load16<T>(dshift + ((long long)v + dt * (long long)row_vecs) * VN, a[u]);
      else {
#pragma unroll
        for (int e = 0; e < VN; ++e) a[u][e] = 0.f;
      }
      if (OTHER) load16<T>(other + (long long)v * VN, b[u]);
      m[u] = BITS ? other_bits[v] : 0xFFu;  // residual gradient through the ReLU mask
    }
#pragma unroll
    for (int u = 0; u < SU; ++u) {
      const unsigned v = base + u * 256;
      if (v >= TV) break;
      if (OTHER) {
#pragma unroll
        for (int e = 0; e < VN; ++e) a[u][e] += ((m[u] >> e) & 1u) ? b[u][e] : 0.f;
      }
      store16<T>(dx + (long long)v * VN, a[u]);
    }
  }
}

inline unsigned blocks_for(long long TV, int per_block) { return (unsigned)((TV + per_block - 1) / per_block); }
inline unsigned stream_grid(long long TV) {
  const long long b = (TV + SB - 1) / SB;
  return (unsigned)(b < GRID_MAX ? b : GRID_MAX);
}

}  // namespace

namespace vcg {
// column sums of EPI_BWD partials (igemm_fast.hip) -> sum_g / sum_gx (+ dgamma / dbeta, accumulated)
int bn_bwd_finalize_launch(const float* partial, int nb, int C, long long ld, int gx_off, float* sum_g, float* sum_gx,
                           float* dgamma, float* dbeta, int accumulate, hipStream_t s) {
  hipLaunchKernelGGL(bn_bwd_finalize_kernel, dim3((C + 15) / 16), dim3(256), 0, s, partial, nb, C, ld, gx_off, sum_g,
                     sum_gx, dgamma, dbeta, accumulate);
  VCG_LAUNCH_CHECK();
  return VCG_OK;
}
}  // namespace vcg

// ==================================================================== C ABI

// vcg_bn_apply (no residual) that also returns the column sums of the stored output (the bn3 fold's colsum(a2)
// without a pass of its own); ws: vcg_bn_apply_colsum_ws_bytes
VCG_API long long vcg_bn_apply_colsum_ws_bytes(long long P, int C) {
  return (long long)stream_grid(P * C / 8) * C * 4 + 256;
}

VCG_API int vcg_bn_apply_colsum(const void* y, const float* scale, const float* shift, int relu, void* out,
                                float* colsum, float* ws, long long ws_bytes, long long P, int C, hipStream_t s) {
  VCG_REQUIRE(y && scale && shift && out && colsum && ws, "null argument");
  VCG_REQUIRE(C % 8 == 0 && (C & (C - 1)) == 0 && C / 8 <= 256, "C must be a power of two in [8, 2048]");
  const long long TV = P * C / 8;
  if (TV == 0) return VCG_OK;
  const unsigned g = stream_grid(TV);
  VCG_REQUIRE(ws_bytes >= (long long)g * C * 4, "workspace too small");
  hipLaunchKernelGGL((bn_apply_kernel<bf16_t, false, false, true>), dim3(g), dim3(256), 0, s, (const bf16_t*)y, scale, shift,
                     (const bf16_t*)nullptr, (const float*)nullptr, (const float*)nullptr, relu, (bf16_t*)out,
                     (uint8_t*)nullptr, TV, C / 8, ws);
  VCG_LAUNCH_CHECK();
  hipLaunchKernelGGL(colpart_reduce_kernel, dim3((C + 15) / 16), dim3(256), 0, s, ws, (int)g, C, colsum);
  VCG_LAUNCH_CHECK();
  return VCG_OK;
}

VCG_API int vcg_bn_apply(int dtype, const void* y, const float* scale, const float* shift, const void* res,
                         const float* rscale, const float* rshift, int relu, void* out, unsigned char* bits,
                         long long P, int C, hipStream_t s) {
  const int VN = dtype == VCG_BF16 ? 8 : 4;
  VCG_REQUIRE(C % VN == 0 && (C & (C - 1)) == 0, "C must be a power of two multiple of the vector width");
  const long long TV = P * C / VN;
  const int cpr = C / VN;
  if (TV == 0) return VCG_OK;
  const unsigned g = stream_grid(TV);
  const bool raff = rscale != nullptr;
  VCG_REQUIRE(!raff || (res && rshift), "rscale needs res and rshift");
#define VCG_BN_APPLY(T, R, A)                                                                                     \
  hipLaunchKernelGGL((bn_apply_kernel<T, R, A>), dim3(g), dim3(256), 0, s, (const T*)y, scale, shift, (const T*)res, \
                     rscale, rshift, relu, (T*)out, bits, TV, cpr)
#define VCG_BN_APPLY_T(T)                     \
  if (!res) VCG_BN_APPLY(T, false, false);    \
  else if (!raff) VCG_BN_APPLY(T, true, false); \
  else VCG_BN_APPLY(T, true, true);
  if (dtype == VCG_BF16) {
    VCG_BN_APPLY_T(bf16_t)
  } else {
    VCG_BN_APPLY_T(float)
  }
#undef VCG_BN_APPLY_T
#undef VCG_BN_APPLY
  VCG_LAUNCH_CHECK();
  return VCG_OK;
}

// rows per block: enough blocks to fill the chip (~1024 in total) but at most RED_ITER_MAX vectors
// per thread (the per-block partials then stay small next to the streamed tensors)
static long long bn_bwd_rows(long long P, int C, int VN) {
  const int cpr = C / VN;
  const long long TV = P * cpr;
  long long it = (TV + 256LL * 1024 - 1) / (256LL * 1024);
  if (it < 4) it = 4;
  if (it > RED_ITER_MAX) it = RED_ITER_MAX;
  return cpr <= 256 ? it * (256 / cpr) : it;
}
static long long bn_bwd_blocks(long long P, int C, int VN) {
  const long long rows = bn_bwd_rows(P, C, VN);
  return (P + rows - 1) / rows;
}

VCG_API long long vcg_bn_bwd_ws_bytes(long long P, int C) {
  // one query serves both dtypes (vector width 4 for fp32, 8 for bf16)
  const long long nb = bn_bwd_blocks(P, C, 4) > bn_bwd_blocks(P, C, 8) ? bn_bwd_blocks(P, C, 4) : bn_bwd_blocks(P, C, 8);
  return nb * 2 * C * 4 + 64;
}

static MaskArgs mask_args(int mode, const void* mask, const unsigned char* bits, const float* msc, const float* msh) {
  MaskArgs m;
  m.mode = mode;
  m.t = mask;
  m.bits = bits;
  m.sc = msc;
  m.sh = msh;
  return m;
}

static int check_mask(int mode, const void* mask, const unsigned char* bits, const float* msc, const float* msh) {
  VCG_REQUIRE(mode >= 0 && mode <= 3, "mask_mode must be 0..3");
  VCG_REQUIRE(mode != 1 || mask, "mask_mode 1 needs the mask tensor");
  VCG_REQUIRE(mode != 2 || bits, "mask_mode 2 needs the mask bits");
  VCG_REQUIRE(mode != 3 || (msc && msh), "mask_mode 3 needs mscale/mshift");
  return VCG_OK;
}

VCG_API int vcg_bn_bwd_reduce(int dtype, const void* dout, int mask_mode, const void* mask, const unsigned char* mbits,
                              const float* mscale, const float* mshift, const void* y, const float* mean,
                              const float* invstd, long long P, int C, float* ws, long long ws_bytes, float* sum_g,
                              float* sum_gx, float* dgamma, float* dbeta, int accumulate, hipStream_t s) {
  if (int rc = check_mask(mask_mode, mask, mbits, mscale, mshift)) return rc;
  const MaskArgs mk = mask_args(mask_mode, mask, mbits, mscale, mshift);
  const int VN = dtype == VCG_BF16 ? 8 : 4;
  VCG_REQUIRE(C % VN == 0 && (C & (C - 1)) == 0 && C <= 2048, "C must be a power of two <= 2048");
  VCG_REQUIRE(ws_bytes >= vcg_bn_bwd_ws_bytes(P, C), "workspace too small");
  const long long TV = P * C / VN;
  const int cpr = C / VN;
  const long long nb = bn_bwd_blocks(P, C, VN);
  const int rows = (int)bn_bwd_rows(P, C, VN);
  const dim3 grid((unsigned)nb, cpr > 256 ? cpr / 256 : 1);
#define VCG_BN_RED(T, M)                                                                                  \
  hipLaunchKernelGGL((bn_bwd_reduce_kernel<T, M>), grid, dim3(256), 0, s, (const T*)dout, mk, (const T*)y, mean, \
                     invstd, P, cpr, C, rows, ws)
#define VCG_BN_RED_T(T)                \
  switch (mask_mode) {                 \
    case 0: VCG_BN_RED(T, 0); break;   \
    case 1: VCG_BN_RED(T, 1); break;   \
    case 2: VCG_BN_RED(T, 2); break;   \
    default: VCG_BN_RED(T, 3); break;  \
  }
  if (dtype == VCG_BF16) {
    VCG_BN_RED_T(bf16_t)
  } else {
    VCG_BN_RED_T(float)
  }
#undef VCG_BN_RED_T
#undef VCG_BN_RED
  VCG_LAUNCH_CHECK();
  hipLaunchKernelGGL(bn_bwd_finalize_kernel, dim3((C + 15) / 16), dim3(256), 0, s, ws, (int)nb, C, 2LL * C, C,
                     sum_g, sum_gx, dgamma, dbeta, accumulate);
  VCG_LAUNCH_CHECK();
  return VCG_OK;
}

VCG_API int vcg_bn_bwd_apply(int dtype, const void* dout, int mask_mode, const void* mask, const unsigned char* mbits,
                             const float* mscale, const float* mshift, const void* y, const float* mean,
                             const float* invstd, const float* gamma, const float* sum_g, const float* sum_gx,
                             long long count, int train_stats, void* dy, void* gout, long long P, int C,
                             hipStream_t s) {
  if (int rc = check_mask(mask_mode, mask, mbits, mscale, mshift)) return rc;
  const MaskArgs mk = mask_args(mask_mode, mask, mbits, mscale, mshift);
  const int VN = dtype == VCG_BF16 ? 8 : 4;
  VCG_REQUIRE(C % VN == 0 && (C & (C - 1)) == 0, "C must be a power of two multiple of the vector width");
  const long long TV = P * C / VN;
  const float ic = 1.f / (float)count;
  const unsigned g = stream_grid(TV);
  const int cpr = C / VN;
#define VCG_BN_BAPP(T, M, TR)                                                                                    \
  hipLaunchKernelGGL((bn_bwd_apply_kernel<T, M, TR>), dim3(g), dim3(256), 0, s, (const T*)dout, mk, (const T*)y, \
                     mean, invstd, gamma, sum_g, sum_gx, ic, (T*)dy, (T*)gout, TV, cpr)
#define VCG_BN_BAPP_M(T, TR)               \
  switch (mask_mode) {                     \
    case 0: VCG_BN_BAPP(T, 0, TR); break;  \
    case 1: VCG_BN_BAPP(T, 1, TR); break;  \
    case 2: VCG_BN_BAPP(T, 2, TR); break;  \
    default: VCG_BN_BAPP(T, 3, TR); break; \
  }
  if (dtype == VCG_BF16) {
    if (train_stats) { VCG_BN_BAPP_M(bf16_t, true) } else { VCG_BN_BAPP_M(bf16_t, false) }
  } else {
    if (train_stats) { VCG_BN_BAPP_M(float, true) } else { VCG_BN_BAPP_M(float, false) }
  }
#undef VCG_BN_BAPP_M
#undef VCG_BN_BAPP
  VCG_LAUNCH_CHECK();
  return VCG_OK;
}

VCG_API int vcg_bn_bwd_apply_dual(int dtype, const void* g, const void* y, const float* mean, const float* invstd,
                                  const float* gamma, const float* sum_g, const float* sum_gx, const void* yd,
                                  const float* mean_d, const float* invstd_d, const float* gamma_d,
                                  const float* sum_g_d, const float* sum_gx_d, long long count, void* dy, void* dyd,
                                  long long P, int C, hipStream_t s) {
  const int VN = dtype == VCG_BF16 ? 8 : 4;
  VCG_REQUIRE(C % VN == 0 && (C & (C - 1)) == 0, "C must be a power of two multiple of the vector width");
  const long long TV = P * C / VN;
  if (TV == 0) return VCG_OK;
  VCG_REQUIRE(g && y && yd && dy && dyd && mean && invstd && sum_g && sum_gx && mean_d && invstd_d && sum_g_d &&
                  sum_gx_d,
              "null operand");
  const BnBwdArgs p1{mean, invstd, gamma, sum_g, sum_gx}, p2{mean_d, invstd_d, gamma_d, sum_g_d, sum_gx_d};
  const float ic = 1.f / (float)count;
  const unsigned gr = stream_grid(TV);
  if (dtype == VCG_BF16)
    hipLaunchKernelGGL(bn_bwd_apply_dual_kernel<bf16_t>, dim3(gr), dim3(256), 0, s, (const bf16_t*)g,
                       (const bf16_t*)y, (const bf16_t*)yd, p1, p2, ic, (bf16_t*)dy, (bf16_t*)dyd, TV, C / VN);
  else
    hipLaunchKernelGGL(bn_bwd_apply_dual_kernel<float>, dim3(gr), dim3(256), 0, s, (const float*)g, (const float*)y,
                       (const float*)yd, p1, p2, ic, (float*)dy, (float*)dyd, TV, C / VN);
  VCG_LAUNCH_CHECK();
  return VCG_OK;
}

VCG_API int vcg_maxpool_fwd(int dtype, const void* x, void* y, unsigned char* idx, int N, int H, int W, int C,
                            hipStream_t s) {
  const int VN = dtype == VCG_BF16 ? 8 : 4;
  VCG_REQUIRE(C % VN == 0 && (C & (C - 1)) == 0, "C must be a power of two multiple of the vector width");
  const int OH = (H + 2 - 3) / 2 + 1, OW = (W + 2 - 3) / 2 + 1;
  const int lcpr = ilog2i(C / VN);
  const long long TV = (long long)N * OH * OW * (C / VN);
  VCG_REQUIRE((long long)N * H * W < (1LL << 31), "too many pixels");
  if (dtype == VCG_BF16)
    hipLaunchKernelGGL((maxpool_fwd_kernel<bf16_t, false>), dim3(blocks_for(TV, 256)), dim3(256), 0, s, (const bf16_t*)x,
                       (bf16_t*)y, idx, H, W, C, OH, OW, lcpr, TV, make_fastdiv(OW), make_fastdiv(OH));
  else
    hipLaunchKernelGGL((maxpool_fwd_kernel<float, false>), dim3(blocks_for(TV, 256)), dim3(256), 0, s, (const float*)x,
                       (float*)y, idx, H, W, C, OH, OW, lcpr, TV, make_fastdiv(OW), make_fastdiv(OH));
  VCG_LAUNCH_CHECK();
  return VCG_OK;
}

VCG_API int vcg_maxpool_bwd(int dtype, const void* dy, const unsigned char* idx, void* dx, int N, int H, int W, int C,
                            hipStream_t s) {
  const int VN = dtype == VCG_BF16 ? 8 : 4;
  VCG_REQUIRE(C % VN == 0 && (C & (C - 1)) == 0 && C / VN <= 256, "C must be a power of two multiple of the vector width");
  const int OH = (H + 2 - 3) / 2 + 1, OW = (W + 2 - 3) / 2 + 1;
  const int lcpr = ilog2i(C / VN);
  const long long TV = (long long)N * H * W * (C / VN);
  VCG_REQUIRE((long long)N * H * W < (1LL << 31), "too many pixels");
  const unsigned g = stream_grid(TV);
  if (dtype == VCG_BF16)
    hipLaunchKernelGGL((maxpool_bwd_kernel<bf16_t, MP_PLAIN>), dim3(g), dim3(256), 0, s, (const bf16_t*)dy, idx,
                       (bf16_t*)dx, H, W, C, OH, OW, lcpr, TV, nullptr, MpBn{}, make_fastdiv(W), make_fastdiv(H));
  else
    hipLaunchKernelGGL((maxpool_bwd_kernel<float, MP_PLAIN>), dim3(g), dim3(256), 0, s, (const float*)dy, idx,
                       (float*)dx, H, W, C, OH, OW, lcpr, TV, nullptr, MpBn{}, make_fastdiv(W), make_fastdiv(H));
  VCG_LAUNCH_CHECK();
  return VCG_OK;
}

VCG_API long long vcg_maxpool_bwd_bn_ws_bytes(int C) { return (GRID_MAX + 1) * 2 * C * 4 + 64; }

// max-pool backward fused with the stem BatchNorm-backward reduction: g = maxpool_bwd(dy) masked by the
// forward ReLU (fma(y, mscale, mshift) > 0); sum_g / sum_gx finalized, dgamma / dbeta accumulated. g == NULL:
// the sums only (vcg_maxpool_bwd_bn_apply then recomputes g).
VCG_API int vcg_maxpool_bwd_bn(int dtype, const void* dy, const unsigned char* idx, void* g, int N, int H, int W,
                               int C, const void* y, const float* mean, const float* invstd, const float* mscale,
                               const float* mshift, float* ws, long long ws_bytes, float* sum_g, float* sum_gx,
                               float* dgamma, float* dbeta, hipStream_t s) {
  const int VN = dtype == VCG_BF16 ? 8 : 4;
  VCG_REQUIRE(C % VN == 0 && (C & (C - 1)) == 0 && C / VN <= 256, "C must be a power of two multiple of the vector width");
  VCG_REQUIRE(y && mean && invstd && mscale && mshift && sum_g && sum_gx, "BN arguments required");
  VCG_REQUIRE(ws_bytes >= vcg_maxpool_bwd_bn_ws_bytes(C), "workspace too small");
  const int OH = (H + 2 - 3) / 2 + 1, OW = (W + 2 - 3) / 2 + 1;
  const int lcpr = ilog2i(C / VN);
  const long long TV = (long long)N * H * W * (C / VN);
  VCG_REQUIRE((long long)N * H * W < (1LL << 31), "too many pixels");
  const unsigned nb = stream_grid(TV);
  MpBn bn{};
  bn.mean = mean; bn.invstd = invstd; bn.msc = mscale; bn.msh = mshift; bn.part = ws;
#define VCG_MPB(T, M, OUT)                                                                                          \
  do {                                                                                                              \
    if ((H & 1) == 0 && (W & 1) == 0)                                                                               \
      hipLaunchKernelGGL((maxpool_bwd2_kernel<T, M>), dim3(nb), dim3(256), 0, s, (const T*)dy, idx, (T*)OUT, H, W, C, \
                         OH, OW, lcpr, TV / 4, (const T*)y, bn, make_fastdiv(W / 2), make_fastdiv(H / 2));           \
    else                                                                                                            \
      hipLaunchKernelGGL((maxpool_bwd_kernel<T, M>), dim3(nb), dim3(256), 0, s, (const T*)dy, idx, (T*)OUT, H, W, C, \
                         OH, OW, lcpr, TV, (const T*)y, bn, make_fastdiv(W), make_fastdiv(H));                       \
  } while (0)
  if (dtype == VCG_BF16) {
    if (g) VCG_MPB(bf16_t, MP_RED, g); else VCG_MPB(bf16_t, MP_RED_ONLY, g);
  } else {
    if (g) VCG_MPB(float, MP_RED, g); else VCG_MPB(float, MP_RED_ONLY, g);
  }
  VCG_LAUNCH_CHECK();
  hipLaunchKernelGGL(bn_bwd_finalize_kernel, dim3((C + 15) / 16), dim3(256), 0, s, ws, (int)nb, C, 2LL * C, C,
                     sum_g, sum_gx, dgamma, dbeta, 1);
  VCG_LAUNCH_CHECK();
  return VCG_OK;
}

// The sums of vcg_maxpool_bwd_bn (g == NULL) from the pooled activation mp [N][OH][OW][C] (the fused stem's
// vcg_bn_relu_maxpool output) instead of the pre-pool y: see maxpool_bn_sums_pooled_kernel. idx (the forward's argmax
// bytes) and the pre-pool y [N][H][W][C] are read only for degenerate channels (zero or tiny BN weight).
VCG_API int vcg_maxpool_bwd_bn_sums_pooled(int dtype, const void* dy, const void* mp, const unsigned char* idx,
                                           const void* y, int N, int H, int W, int C, const float* mean,
                                           const float* invstd, const float* mscale, const float* mshift, float* ws,
                                           long long ws_bytes, float* sum_g, float* sum_gx, float* dgamma,
                                           float* dbeta, hipStream_t s) {
  const int VN = dtype == VCG_BF16 ? 8 : 4;
  VCG_REQUIRE(C % VN == 0 && (C & (C - 1)) == 0 && C / VN <= 256, "C must be a power of two multiple of the vector width");
  VCG_REQUIRE(dy && mp && idx && y && mean && invstd && mscale && mshift && sum_g && sum_gx, "BN arguments required");
  VCG_REQUIRE(ws_bytes >= vcg_maxpool_bwd_bn_ws_bytes(C), "workspace too small");
  const int OH = (H + 2 - 3) / 2 + 1, OW = (W + 2 - 3) / 2 + 1;
  const int lcpr = ilog2i(C / VN);
  const long long TV = (long long)N * OH * OW * (C / VN);
  if (TV == 0) return VCG_OK;
  const unsigned nb = stream_grid(TV);
  MpBn bn{};
  bn.mean = mean; bn.invstd = invstd; bn.msc = mscale; bn.msh = mshift; bn.part = ws;
  const long long npix = (long long)N * OH * OW;
  if (dtype == VCG_BF16) {
    hipLaunchKernelGGL(maxpool_bn_sums_pooled_kernel<bf16_t>, dim3(nb), dim3(256), 0, s, (const bf16_t*)dy,
                       (const bf16_t*)mp, TV, lcpr, bn);
    hipLaunchKernelGGL(maxpool_bn_sums_degen_kernel<bf16_t>, dim3(C), dim3(256), 0, s, (const bf16_t*)dy,
                       (const bf16_t*)mp, idx, (const bf16_t*)y, H, W, OH, OW, npix, C, bn, (int)nb);
  } else {
    hipLaunchKernelGGL(maxpool_bn_sums_pooled_kernel<float>, dim3(nb), dim3(256), 0, s, (const float*)dy,
                       (const float*)mp, TV, lcpr, bn);
    hipLaunchKernelGGL(maxpool_bn_sums_degen_kernel<float>, dim3(C), dim3(256), 0, s, (const float*)dy,
                       (const float*)mp, idx, (const float*)y, H, W, OH, OW, npix, C, bn, (int)nb);
  }
  VCG_LAUNCH_CHECK();
  hipLaunchKernelGGL(bn_bwd_finalize_kernel, dim3((C + 15) / 16), dim3(256), 0, s, ws, (int)nb + 1, C, 2LL * C, C,
                     sum_g, sum_gx, dgamma, dbeta, 1);
  VCG_LAUNCH_CHECK();
  return VCG_OK;
}

// The stem's BatchNorm backward apply fused with the max-pool backward: dx = bn_bwd_apply(g) with g =
// maxpool_bwd(dy) masked by the forward ReLU and rounded to the storage type (the value vcg_maxpool_bwd_bn
// would store), sums from vcg_maxpool_bwd_bn(g = NULL). Equals vcg_maxpool_bwd_bn + vcg_bn_bwd_apply (mask
// mode 0) on that g, without the g round trip through HBM.
VCG_API int vcg_maxpool_bwd_bn_apply(int dtype, const void* dy, const unsigned char* idx, void* dx, int N, int H,
                                     int W, int C, const void* y, const float* mean, const float* invstd,
                                     const float* mscale, const float* mshift, const float* gamma, const float* sum_g,
                                     const float* sum_gx, long long count, int train_stats, hipStream_t s) {
  const int VN = dtype == VCG_BF16 ? 8 : 4;
  VCG_REQUIRE(C % VN == 0 && (C & (C - 1)) == 0 && C / VN <= 256, "C must be a power of two multiple of the vector width");
  VCG_REQUIRE(y && mean && invstd && mscale && mshift && sum_g && sum_gx && count > 0, "BN arguments required");
  const int OH = (H + 2 - 3) / 2 + 1, OW = (W + 2 - 3) / 2 + 1;
  const int lcpr = ilog2i(C / VN);
  const long long TV = (long long)N * H * W * (C / VN);
  VCG_REQUIRE((long long)N * H * W < (1LL << 31), "too many pixels");
  MpBn bn{};
  bn.mean = mean; bn.invstd = invstd; bn.msc = mscale; bn.msh = mshift;
  bn.gamma = gamma; bn.sum_g = sum_g; bn.sum_gx = sum_gx; bn.inv_count = 1.f / (float)count; bn.train = train_stats;
  const unsigned nb = stream_grid(TV);
  if (dtype == VCG_BF16) {
    VCG_MPB(bf16_t, MP_APPLY, dx);
  } else {
    VCG_MPB(float, MP_APPLY, dx);
  }
#undef VCG_MPB
  VCG_LAUNCH_CHECK();
  return VCG_OK;
}

// The stem's BatchNorm + ReLU fused into the max-pool: out / idx = maxpool(relu(fma(y, scale, shift))) with the
// activation rounded to the storage type first (the values and argmax of vcg_bn_apply then vcg_maxpool_fwd).
VCG_API int vcg_bn_relu_maxpool(int dtype, const void* y, const float* scale, const float* shift, void* out,
                                unsigned char* idx, int N, int H, int W, int C, hipStream_t s) {
  const int VN = dtype == VCG_BF16 ? 8 : 4;
  VCG_REQUIRE(C % VN == 0 && (C & (C - 1)) == 0 && C / VN <= 256, "C must be a power of two multiple of the vector width");
  VCG_REQUIRE(scale && shift, "scale / shift required");
  const int OH = (H + 2 - 3) / 2 + 1, OW = (W + 2 - 3) / 2 + 1;
  const int lcpr = ilog2i(C / VN);
  const long long TV = (long long)N * OH * OW * (C / VN);
  VCG_REQUIRE((long long)N * H * W < (1LL << 31), "too many pixels");
  if (dtype == VCG_BF16) {  // two outputs per thread (maxpool_fwd2_kernel)
    const int OW2 = (OW + 1) / 2;
    const long long TV2 = (long long)N * OH * OW2 * (C / VN);
    hipLaunchKernelGGL((maxpool_fwd2_kernel<bf16_t, true>), dim3(blocks_for(TV2, 256)), dim3(256), 0, s,
                       (const bf16_t*)y, (bf16_t*)out, idx, H, W, C, OH, OW, lcpr, TV2, make_fastdiv(OW2),
                       make_fastdiv(OH), scale, shift);
  } else if (dtype == VCG_BF16)
    hipLaunchKernelGGL((maxpool_fwd_kernel<bf16_t, true>), dim3(blocks_for(TV, 256)), dim3(256), 0, s,
                       (const bf16_t*)y, (bf16_t*)out, idx, H, W, C, OH, OW, lcpr, TV, make_fastdiv(OW),
                       make_fastdiv(OH), scale, shift);
  else
    hipLaunchKernelGGL((maxpool_fwd_kernel<float, true>), dim3(blocks_for(TV, 256)), dim3(256), 0, s,
                       (const float*)y, (float*)out, idx, H, W, C, OH, OW, lcpr, TV, make_fastdiv(OW),
                       make_fastdiv(OH), scale, shift);
  VCG_LAUNCH_CHECK();
  return VCG_OK;
}

VCG_API int vcg_tsm_unshift_add(int dtype, const void* dshift, const void* other, const unsigned char* other_bits,
                                void* dx, long long NT, int T, long long HW, int C, int fold, hipStream_t s) {
  const int VN = dtype == VCG_BF16 ? 8 : 4;
  VCG_REQUIRE(C % VN == 0 && (C & (C - 1)) == 0 && fold % VN == 0, "C / fold must be multiples of the vector width");
  const long long TV = NT * HW * C / VN;
  VCG_REQUIRE(TV < (1LL << 31), "tensor too large for 32-bit vector indices");
  const int lcpr = ilog2i(C / VN);
  const unsigned g = stream_grid(TV);
  const unsigned row_vecs = (unsigned)(HW * C / VN);
#define VCG_TSM(T, O, B)                                                                                           \
  hipLaunchKernelGGL((tsm_unshift_add_kernel<T, O, B>), dim3(g), dim3(256), 0, s, (const T*)dshift, (const T*)other, \
                     other_bits, (T*)dx, (unsigned)TV, lcpr, row_vecs, T_, fold / VN)
#define VCG_TSM_T(T)                         \
  if (!other) VCG_TSM(T, false, false);      \
  else if (!other_bits) VCG_TSM(T, true, false); \
  else VCG_TSM(T, true, true);
  const int T_ = T;
  if (dtype == VCG_BF16) {
    VCG_TSM_T(bf16_t)
  } else {
    VCG_TSM_T(float)
  }
#undef VCG_TSM_T
#undef VCG_TSM
  VCG_LAUNCH_CHECK();
  return VCG_OK;
}
