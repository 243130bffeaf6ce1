// Fused BERT self-attention for the bf16 train / scoring path: one workgroup per (sequence, head), L <= 128 keys,
// head dim 64, HF BertModel eager-attention semantics (model/lang/bert_hugface.py:20 via two_stream.py:172-179):
//
//   forward : S = Q K^T, P = softmax(scale * S + mask_add) (a row with no valid key is uniform over the L keys, as
//             HF's finfo.min bias gives), Pd = dropout(P), ctx = Pd V; saved: (row max, 1 / row sum) per query
//   backward: S and P recomputed from Q, K and the saved row statistics, dPd = dO V^T, dP = dropout'(dPd),
//             D = rowsum(dP o P) from the fp32 products (not rowsum(dO o O) of the bf16-rounded ctx: the same dP
//             then enters both terms of dP - D, so each dS row sums to zero as the exact softmax gradient does and the
//             rounding of O does not leak into dQ / dK), dS = scale * P o (dP - D); dQ = dS K, dK = dS^T Q, dV = Pd^T dO
//
// Nothing of size L x L touches HBM (the unfused path writes S, P and Pd per layer and reads them back): the
// forward reads Q, K, V once and writes ctx; the backward reads Q, K, V, dO, O once and writes dQ, dK, dV.
// Dropout regenerates the unfused kernels' mask exactly (same counter-hash index (z * L + q) * Lp + key).
//
// MFMA: mfma_f32_16x16x32_bf16 (lane l = 16 g + i holds A[row i][k-set g], B[k-set g][col i], D[rows 4g..4g+3]
// [col i]). A k-step's 32 k indices only have to be the same SET on both operands, so a D fragment (4 consecutive
// rows per lane) feeds the next MFMA's operand straight from registers: rows {32s + 4g + r, 32s + 16 + 4g + r} of
// two adjacent D tiles form lane group g's k-set of k-step s. Only dS crosses waves (through LDS) in the backward.
#include "common.h"

using namespace vcg;

namespace {

constexpr int LT = 128;  // query / key tile: L <= 128
constexpr int DH = 64;   // head dim
constexpr int TP = 136;  // row pitch (elements) of the transposed / square LDS tiles: 272-B rows, conflict-free
                         // b64 / b128 fragment reads of 16 consecutive rows

__device__ __forceinline__ int swz(int row, int chunk) { return chunk ^ ((row >> 1) & 7); }

__device__ __forceinline__ uint32_t pack2(float a, float b) { return (uint32_t)f2bf(a) | ((uint32_t)f2bf(b) << 16); }

__device__ __forceinline__ uint32_t half16(const uint4& v, int j) {
  const uint32_t w = (j >> 1) == 0 ? v.x : (j >> 1) == 1 ? v.y : (j >> 1) == 2 ? v.z : v.w;
  return (j & 1) ? (w >> 16) : (w & 0xffffu);
}

__device__ __forceinline__ s16x8 frag_rm(const bf16_t* t, int row, int chunk) {  // swizzled [rows][64] tile
  return *reinterpret_cast<const s16x8*>(t + row * DH + 8 * swz(row, chunk));
}

// two 8-B halves (elements c0..c0+3 and c0+16..c0+19) of row `row` of a [rows][TP] tile
__device__ __forceinline__ s16x8 frag_split(const bf16_t* t, int row, int c0) {
  const uint2 lo = *reinterpret_cast<const uint2*>(t + row * TP + c0);
  const uint2 hi = *reinterpret_cast<const uint2*>(t + row * TP + c0 + 16);
  typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
  const u32x4 u = {lo.x, lo.y, hi.x, hi.y};
  return __builtin_bit_cast(s16x8, u);
}

__device__ __forceinline__ s16x8 pack8(const float (&a)[4], const float (&b)[4]) {
  typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
  const u32x4 u = {pack2(a[0], a[1]), pack2(a[2], a[3]), pack2(b[0], b[1]), pack2(b[2], b[3])};
  return __builtin_bit_cast(s16x8, u);
}

__device__ __forceinline__ uint4 ld16(const bf16_t* p, bool ok) {
  return ok ? *reinterpret_cast<const uint4*>(p) : make_uint4(0u, 0u, 0u, 0u);
}

// rows 4 kg .. 4 kg + 3, 8-element chunk dc of a [L][ld] row-major source (rows >= L zero) -> the transposed tile
// t[d][row] ([64][TP]); optionally also the swizzled row-major copy rm[row][64]
__device__ __forceinline__ void load_transpose(const bf16_t* src, long long ld, int L, bf16_t* t, bf16_t* rm, int tid) {
  const int kg = tid >> 3, dc = tid & 7;
  uint4 v[4];
#pragma unroll
  for (int e = 0; e < 4; ++e) v[e] = ld16(src + (long long)(4 * kg + e) * ld + 8 * dc, 4 * kg + e < L);
  if (rm) {
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const int r = 4 * kg + e;
      *reinterpret_cast<uint4*>(rm + r * DH + 8 * swz(r, dc)) = v[e];
    }
  }
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    uint2 q;
    q.x = half16(v[0], j) | (half16(v[1], j) << 16);
    q.y = half16(v[2], j) | (half16(v[3], j) << 16);
    *reinterpret_cast<uint2*>(t + (8 * dc + j) * TP + 4 * kg) = q;
  }
}

// ------------------------------------------------------------------------------------------------ forward
// 4 waves; wave w owns queries 32 w .. 32 w + 31. S^T = K Q^T (A = K rows from LDS, B = Q rows from HBM), the
// softmax over the lane's 32 keys and the 4 lane groups, O^T = V^T Pd^T (A = V^T from LDS, B = Pd from registers).
__global__ __launch_bounds__(256) void bert_attn_fwd_kernel(const bf16_t* __restrict__ qkv,
                                                            const long long* __restrict__ mask,
                                                            bf16_t* __restrict__ ctx, float2* __restrict__ stats,
                                                            const int* __restrict__ seq, int nh, int Lmax, int Lp,
                                                            float scale, float p, uint64_t seed) {
  __shared__ __attribute__((aligned(16))) bf16_t Ks[LT * DH];
  __shared__ __attribute__((aligned(16))) bf16_t Vt[DH * TP];
  __shared__ uint8_t kval[LT];
  const int z = blockIdx.x, b = z / nh, h = z - b * nh;
  const int H = nh * DH;
  const long long ld = 3LL * H;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, g = lane >> 4, i = lane & 15;
  // sequence b: rows row0 .. row0 + L - 1 (packed: seq[b] .. seq[b + 1] - 1; else b Lmax .. + Lmax - 1)
  const int row0 = seq ? seq[b] : b * Lmax;
  const int L = seq ? seq[b + 1] - row0 : Lmax;
  const bf16_t* base = qkv + (long long)row0 * ld + h * DH;  // Q of (b, h); K at + H, V at + 2 H

  for (int c = tid; c < LT * 8; c += 256) {
    const int r = c >> 3, ch = c & 7;
    *reinterpret_cast<uint4*>(Ks + r * DH + 8 * swz(r, ch)) = ld16(base + r * ld + H + 8 * ch, r < L);
  }
  load_transpose(base + 2 * H, ld, L, Vt, nullptr, tid);
  if (tid < LT) kval[tid] = tid < L && (mask == nullptr || mask[(long long)row0 + tid] != 0);
  s16x8 qf[2][2];
#pragma unroll
  for (int qt = 0; qt < 2; ++qt)
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      const int q = 32 * w + 16 * qt + i;
      const uint4 u = ld16(base + (long long)q * ld + 8 * (4 * s + g), q < L);
      qf[qt][s] = __builtin_bit_cast(s16x8, u);
    }
  __syncthreads();
  // (a packed sequence shorter than 128 rows: tiles of keys / queries past its end add nothing and are skipped)
  if (32 * w >= L) return;  // every query of this wave is past the end (no barrier follows)

  f32x4 sacc[2][8];
#pragma unroll
  for (int qt = 0; qt < 2; ++qt)
#pragma unroll
    for (int kt = 0; kt < 8; ++kt) sacc[qt][kt] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int kt = 0; kt < 8; ++kt)
    if (16 * kt < L) {
#pragma unroll
      for (int s = 0; s < 2; ++s) {
        const s16x8 kf = frag_rm(Ks, 16 * kt + i, 4 * s + g);
#pragma unroll
        for (int qt = 0; qt < 2; ++qt) sacc[qt][kt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(kf, qf[qt][s], sacc[qt][kt], 0, 0, 0);
      }
    }
  // lane holds S^T[key 16 kt + 4 g + r][query 32 w + 16 qt + i]
  uint32_t vb = 0;  // bit 4 kt + r: key 16 kt + 4 g + r is valid
#pragma unroll
  for (int kt = 0; kt < 8; ++kt)
#pragma unroll
    for (int r = 0; r < 4; ++r) vb |= kval[16 * kt + 4 * g + r] ? (1u << (4 * kt + r)) : 0u;
  const float rs = p > 0.f ? 1.f / (1.f - p) : 1.f;
  s16x8 pf[2][4];
#pragma unroll
  for (int qt = 0; qt < 2; ++qt) {
    const int q = 32 * w + 16 * qt + i;
    float mx = -INFINITY;
#pragma unroll
    for (int kt = 0; kt < 8; ++kt)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const float v = ((vb >> (4 * kt + r)) & 1u) ? sacc[qt][kt][r] * scale : -INFINITY;
        sacc[qt][kt][r] = v;
        mx = fmaxf(mx, v);
      }
    mx = fmaxf(mx, __shfl_xor(mx, 16, 64));
    mx = fmaxf(mx, __shfl_xor(mx, 32, 64));
    const bool none = mx == -INFINITY;
    float sum = 0.f;
#pragma unroll
    for (int kt = 0; kt < 8; ++kt)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int key = 16 * kt + 4 * g + r;
        const float v = sacc[qt][kt][r];
        const float e = none ? (key < L ? 1.f : 0.f) : (v == -INFINITY ? 0.f : __expf(v - mx));
        sacc[qt][kt][r] = e;
        sum += e;
      }
    sum += __shfl_xor(sum, 16, 64);
    sum += __shfl_xor(sum, 32, 64);
    const float inv = 1.f / sum;
    if (g == 0 && q < L) stats[(long long)z * LT + q] = make_float2(mx, inv);
    const uint64_t rowi = ((uint64_t)z * Lmax + q) * (uint64_t)Lp;
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      float a[4], c[4];
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int k0 = 32 * s + 4 * g + r, k1 = k0 + 16;
        const float p0 = sacc[qt][2 * s][r] * inv, p1 = sacc[qt][2 * s + 1][r] * inv;
        a[r] = (q < L && dropout_keep(seed, rowi + k0, p)) ? p0 * rs : 0.f;
        c[r] = (q < L && dropout_keep(seed, rowi + k1, p)) ? p1 * rs : 0.f;
      }
      pf[qt][s] = pack8(a, c);
    }
  }

  f32x4 oacc[4][2];
#pragma unroll
  for (int dt = 0; dt < 4; ++dt)
#pragma unroll
    for (int qt = 0; qt < 2; ++qt) oacc[dt][qt] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int s = 0; s < 4; ++s)
    if (32 * s < L) {
#pragma unroll
      for (int dt = 0; dt < 4; ++dt) {
        const s16x8 vf = frag_split(Vt, 16 * dt + i, 32 * s + 4 * g);
#pragma unroll
        for (int qt = 0; qt < 2; ++qt) oacc[dt][qt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(vf, pf[qt][s], oacc[dt][qt], 0, 0, 0);
      }
    }
  // lane holds O^T[d 16 dt + 4 g + r][query 32 w + 16 qt + i]
#pragma unroll
  for (int qt = 0; qt < 2; ++qt) {
    const int q = 32 * w + 16 * qt + i;
    if (q < L) {
      bf16_t* o = ctx + ((long long)row0 + q) * H + h * DH + 4 * g;
#pragma unroll
      for (int dt = 0; dt < 4; ++dt)
        *reinterpret_cast<uint2*>(o + 16 * dt) =
            make_uint2(pack2(oacc[dt][qt][0], oacc[dt][qt][1]), pack2(oacc[dt][qt][2], oacc[dt][qt][3]));
    }
  }
}

// ------------------------------------------------------------------------------------------------ backward
// 4 waves; wave w owns keys 32 w .. 32 w + 31 for S, dPd, dV and dK (A = Q / dO rows, Q^T / dO^T from LDS, B = the
// wave's K / V rows from HBM, and its P / dS fragments from registers), then queries 32 w .. 32 w + 31 for dQ
// (A = K^T from LDS, B = dS rows from the LDS copy every wave wrote). The forward's ctx is not read.
__global__ __launch_bounds__(256) void bert_attn_bwd_kernel(const bf16_t* __restrict__ qkv,
                                                            const bf16_t* __restrict__ dctx,
                                                            const long long* __restrict__ mask,
                                                            const float2* __restrict__ stats,
                                                            bf16_t* __restrict__ dqkv, const int* __restrict__ seq,
                                                            int nh, int Lmax, int Lp, float scale, float p,
                                                            uint64_t seed) {
  __shared__ __attribute__((aligned(16))) bf16_t Qs[LT * DH];
  __shared__ __attribute__((aligned(16))) bf16_t dOs[LT * DH];
  __shared__ __attribute__((aligned(16))) bf16_t Qt[DH * TP];
  __shared__ __attribute__((aligned(16))) bf16_t dOt[DH * TP];
  __shared__ __attribute__((aligned(16))) bf16_t Kt[DH * TP];
  __shared__ __attribute__((aligned(16))) bf16_t dSm[LT * TP];
  __shared__ float2 st[LT];
  __shared__ float Dp[4 * LT];  // per-wave partial rowsum(dP o P) over the wave's 32 keys
  __shared__ uint8_t kval[LT];
  const int z = blockIdx.x, b = z / nh, h = z - b * nh;
  const int H = nh * DH;
  const long long ld = 3LL * H;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, g = lane >> 4, i = lane & 15;
  const int row0 = seq ? seq[b] : b * Lmax;
  const int L = seq ? seq[b + 1] - row0 : Lmax;
  const bf16_t* base = qkv + (long long)row0 * ld + h * DH;
  const bf16_t* dob = dctx + (long long)row0 * H + h * DH;
  bf16_t* gq = dqkv + (long long)row0 * ld + h * DH;

  load_transpose(base, ld, L, Qt, Qs, tid);
  load_transpose(dob, H, L, dOt, dOs, tid);
  load_transpose(base + H, ld, L, Kt, nullptr, tid);
  if (tid < LT) {
    kval[tid] = tid < L && (mask == nullptr || mask[(long long)row0 + tid] != 0);
    st[tid] = tid < L ? stats[(long long)z * LT + tid] : make_float2(0.f, 0.f);
  }
  s16x8 kf[2][2], vf[2][2];
#pragma unroll
  for (int kt = 0; kt < 2; ++kt)
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      const int key = 32 * w + 16 * kt + i;
      kf[kt][s] = __builtin_bit_cast(s16x8, ld16(base + (long long)key * ld + H + 8 * (4 * s + g), key < L));
      vf[kt][s] = __builtin_bit_cast(s16x8, ld16(base + (long long)key * ld + 2 * H + 8 * (4 * s + g), key < L));
    }
  __syncthreads();

  f32x4 sacc[8][2], pacc[8][2];
#pragma unroll
  for (int qt = 0; qt < 8; ++qt)
#pragma unroll
    for (int kt = 0; kt < 2; ++kt) sacc[qt][kt] = pacc[qt][kt] = f32x4{0.f, 0.f, 0.f, 0.f};
  // (tiles past the end of a packed sequence add nothing: skipped; a wave whose 32 keys are all past it keeps zeros,
  // so its dS entries -- read by every wave's dQ -- are exact zeros)
  const bool wkeys = 32 * w < L;
#pragma unroll
  for (int qt = 0; qt < 8; ++qt)
    if (wkeys && 16 * qt < L) {
#pragma unroll
      for (int s = 0; s < 2; ++s) {
        const s16x8 qa = frag_rm(Qs, 16 * qt + i, 4 * s + g);
        const s16x8 da = frag_rm(dOs, 16 * qt + i, 4 * s + g);
#pragma unroll
        for (int kt = 0; kt < 2; ++kt) {
          sacc[qt][kt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(qa, kf[kt][s], sacc[qt][kt], 0, 0, 0);
          pacc[qt][kt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(da, vf[kt][s], pacc[qt][kt], 0, 0, 0);
        }
      }
    }
  // lane holds S / dPd [query 16 qt + 4 g + r][key 32 w + 16 kt + i]
  const float rs = p > 0.f ? 1.f / (1.f - p) : 1.f;
  bool kv[2];
  int keyi[2];
#pragma unroll
  for (int kt = 0; kt < 2; ++kt) {
    keyi[kt] = 32 * w + 16 * kt + i;
    kv[kt] = kval[keyi[kt]] != 0;
  }
  uint64_t keepb = 0;  // bit 8 qt + 2 r + kt: element (query 16 qt + 4 g + r, key keyi[kt]) kept by dropout
#pragma unroll
  for (int qt = 0; qt < 8; ++qt)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int q = 16 * qt + 4 * g + r;
      const float2 mi = st[q];
      const uint64_t rowi = ((uint64_t)z * Lmax + q) * (uint64_t)Lp;
      float part = 0.f;
#pragma unroll
      for (int kt = 0; kt < 2; ++kt) {
        const int key = keyi[kt];
        float P = 0.f;
        if (q < L) {
          if (mi.x == -INFINITY) P = key < L ? mi.y : 0.f;
          else P = kv[kt] ? __expf(sacc[qt][kt][r] * scale - mi.x) * mi.y : 0.f;
        }
        const bool keep = q < L && key < L && dropout_keep(seed, rowi + key, p);
        const float dP = keep ? pacc[qt][kt][r] * rs : 0.f;
        keepb |= keep ? (1ull << (8 * qt + 2 * r + kt)) : 0ull;
        sacc[qt][kt][r] = P;
        pacc[qt][kt][r] = dP;
        part = fmaf(P, dP, part);
      }
      part += __shfl_xor(part, 1, 64);
      part += __shfl_xor(part, 2, 64);
      part += __shfl_xor(part, 4, 64);
      part += __shfl_xor(part, 8, 64);
      if (i == 0) Dp[w * LT + q] = part;
    }
  __syncthreads();  // Dp complete
#pragma unroll
  for (int qt = 0; qt < 8; ++qt)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int q = 16 * qt + 4 * g + r;
      const float D = (Dp[q] + Dp[LT + q]) + (Dp[2 * LT + q] + Dp[3 * LT + q]);
#pragma unroll
      for (int kt = 0; kt < 2; ++kt) {
        const float P = sacc[qt][kt][r];
        const float dS = scale * P * (pacc[qt][kt][r] - D);
        sacc[qt][kt][r] = ((keepb >> (8 * qt + 2 * r + kt)) & 1ull) ? P * rs : 0.f;  // Pd
        pacc[qt][kt][r] = dS;
        dSm[q * TP + keyi[kt]] = f2bf(dS);
      }
    }

  // dV^T = dO^T Pd, dK^T = Q^T dS over the 128 queries (k-step s: queries {32 s + 4 g + r, 32 s + 16 + 4 g + r})
  f32x4 dv[4][2], dk[4][2];
#pragma unroll
  for (int dt = 0; dt < 4; ++dt)
#pragma unroll
    for (int kt = 0; kt < 2; ++kt) dv[dt][kt] = dk[dt][kt] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int s = 0; s < 4; ++s) {
    if (!wkeys || 32 * s >= L) continue;
    s16x8 pb[2], sb[2];
#pragma unroll
    for (int kt = 0; kt < 2; ++kt) {
      float a[4], c[4], e[4], f[4];
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        a[r] = sacc[2 * s][kt][r];
        c[r] = sacc[2 * s + 1][kt][r];
        e[r] = pacc[2 * s][kt][r];
        f[r] = pacc[2 * s + 1][kt][r];
      }
      pb[kt] = pack8(a, c);
      sb[kt] = pack8(e, f);
    }
#pragma unroll
    for (int dt = 0; dt < 4; ++dt) {
      const s16x8 oa = frag_split(dOt, 16 * dt + i, 32 * s + 4 * g);
      const s16x8 qa = frag_split(Qt, 16 * dt + i, 32 * s + 4 * g);
#pragma unroll
      for (int kt = 0; kt < 2; ++kt) {
        dv[dt][kt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(oa, pb[kt], dv[dt][kt], 0, 0, 0);
        dk[dt][kt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(qa, sb[kt], dk[dt][kt], 0, 0, 0);
      }
    }
  }
  // lane holds dV^T / dK^T [d 16 dt + 4 g + r][key 32 w + 16 kt + i]
#pragma unroll
  for (int kt = 0; kt < 2; ++kt) {
    const int key = keyi[kt];
    if (key < L) {
      bf16_t* o = gq + (long long)key * ld + 4 * g;
#pragma unroll
      for (int dt = 0; dt < 4; ++dt) {
        *reinterpret_cast<uint2*>(o + H + 16 * dt) =
            make_uint2(pack2(dk[dt][kt][0], dk[dt][kt][1]), pack2(dk[dt][kt][2], dk[dt][kt][3]));
        *reinterpret_cast<uint2*>(o + 2 * H + 16 * dt) =
            make_uint2(pack2(dv[dt][kt][0], dv[dt][kt][1]), pack2(dv[dt][kt][2], dv[dt][kt][3]));
      }
    }
  }
  __syncthreads();  // dSm complete

  // dQ^T = K^T dS^T for queries 32 w + 16 qt + i (k-step s: keys 32 s + 8 g .. + 7)
  f32x4 dq[4][2];
#pragma unroll
  for (int dt = 0; dt < 4; ++dt)
#pragma unroll
    for (int qt = 0; qt < 2; ++qt) dq[dt][qt] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int s = 0; s < 4; ++s) {
    if (32 * w >= L || 32 * s >= L) continue;  // (the wave's queries / this step's keys past the end)
    s16x8 sbq[2];
#pragma unroll
    for (int qt = 0; qt < 2; ++qt)
      sbq[qt] = *reinterpret_cast<const s16x8*>(dSm + (32 * w + 16 * qt + i) * TP + 32 * s + 8 * g);
#pragma unroll
    for (int dt = 0; dt < 4; ++dt) {
      const s16x8 ka = *reinterpret_cast<const s16x8*>(Kt + (16 * dt + i) * TP + 32 * s + 8 * g);
#pragma unroll
      for (int qt = 0; qt < 2; ++qt) dq[dt][qt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ka, sbq[qt], dq[dt][qt], 0, 0, 0);
    }
  }
#pragma unroll
  for (int qt = 0; qt < 2; ++qt) {
    const int q = 32 * w + 16 * qt + i;
    if (q < L) {
      bf16_t* o = gq + (long long)q * ld + 4 * g;
#pragma unroll
      for (int dt = 0; dt < 4; ++dt)
        *reinterpret_cast<uint2*>(o + 16 * dt) =
            make_uint2(pack2(dq[dt][qt][0], dq[dt][qt][1]), pack2(dq[dt][qt][2], dq[dt][qt][3]));
    }
  }
}

}  // namespace

VCG_API int vcg_bert_attn_fwd_varlen(const void* qkv, const long long* mask, const int* seq, void* ctx, void* stats,
                                     int B, int nh, int Lmax, int Lp, float scale, float dropout_p,
                                     unsigned long long seed, hipStream_t s);
VCG_API int vcg_bert_attn_bwd_varlen(const void* qkv, const void* dctx, const long long* mask, const int* seq,
                                     const void* stats, void* dqkv, int B, int nh, int Lmax, int Lp, float scale,
                                     float dropout_p, unsigned long long seed, hipStream_t s);

static int attn_check(const char* fn, const void* qkv, const void* out, const void* stats, int B, int nh, int L, int Lp) {
  if (!qkv || !out || !stats || B < 0 || nh <= 0 || L < 0 || Lp < L) {
    set_error(std::string(fn) + ": invalid arguments");
    return VCG_ERR_INVALID;
  }
  if (L > LT) {
    set_error(std::string(fn) + ": L > 128 is not supported by the fused kernel");
    return VCG_ERR_UNSUPPORTED;
  }
  return VCG_OK;
}

VCG_API int vcg_bert_attn_fwd(const void* qkv, const long long* mask, void* ctx, void* stats, int B, int nh, int L,
                              int Lp, float scale, float dropout_p, unsigned long long seed, hipStream_t s) {
  return vcg_bert_attn_fwd_varlen(qkv, mask, nullptr, ctx, stats, B, nh, L, Lp, scale, dropout_p, seed, s);
}

// Packed (unpadded) sequences: sequence b's rows are seq[b] .. seq[b + 1] - 1 of qkv / ctx (at most Lmax <= 128 of
// them), mask the key flags of those rows (NULL: every row is a key); stats and the dropout counters keep the padded
// [B][nh][Lmax] index space, so a sequence whose kept rows are a prefix of its padded rows gets the padded result.
VCG_API int vcg_bert_attn_fwd_varlen(const void* qkv, const long long* mask, const int* seq, void* ctx, void* stats,
                                     int B, int nh, int Lmax, int Lp, float scale, float dropout_p,
                                     unsigned long long seed, hipStream_t s) {
  if (B == 0 || Lmax == 0) return VCG_OK;
  const int rc = attn_check("vcg_bert_attn_fwd", qkv, ctx, stats, B, nh, Lmax, Lp);
  if (rc != VCG_OK) return rc;
  hipLaunchKernelGGL(bert_attn_fwd_kernel, dim3(B * nh), dim3(256), 0, s, (const bf16_t*)qkv, mask, (bf16_t*)ctx,
                     (float2*)stats, seq, nh, Lmax, Lp, scale, dropout_p, (uint64_t)seed);
  VCG_CHECK_HIP(hipGetLastError());
  return VCG_OK;
}

VCG_API int vcg_bert_attn_bwd(const void* qkv, const void* dctx, const void* ctx, const long long* mask,
                              const void* stats, void* dqkv, int B, int nh, int L, int Lp, float scale,
                              float dropout_p, unsigned long long seed, hipStream_t s) {
  (void)ctx;  // (kept in the signature: the backward no longer needs the forward's output)
  return vcg_bert_attn_bwd_varlen(qkv, dctx, mask, nullptr, stats, dqkv, B, nh, L, Lp, scale, dropout_p, seed, s);
}

VCG_API int vcg_bert_attn_bwd_varlen(const void* qkv, const void* dctx, const long long* mask, const int* seq,
                                     const void* stats, void* dqkv, int B, int nh, int Lmax, int Lp, float scale,
                                     float dropout_p, unsigned long long seed, hipStream_t s) {
  if (B == 0 || Lmax == 0) return VCG_OK;
  if (!dctx) {
    set_error("vcg_bert_attn_bwd: invalid arguments");
    return VCG_ERR_INVALID;
  }
  const int rc = attn_check("vcg_bert_attn_bwd", qkv, dqkv, stats, B, nh, Lmax, Lp);
  if (rc != VCG_OK) return rc;
  hipLaunchKernelGGL(bert_attn_bwd_kernel, dim3(B * nh), dim3(256), 0, s, (const bf16_t*)qkv, (const bf16_t*)dctx, mask,
                     (const float2*)stats, (bf16_t*)dqkv, seq, nh, Lmax, Lp, scale, dropout_p, (uint64_t)seed);
  VCG_CHECK_HIP(hipGetLastError());
  return VCG_OK;
}
