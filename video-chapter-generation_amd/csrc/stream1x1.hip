// Register-streaming 1x1 conv GEMM for the trunk's HBM-bound bottleneck passes (bf16, K = 64 / 128 / 256 input
// channels, output columns in blocks of 256): out = relu(bf16(x wfold^T + bias) + res) with the ReLU mask bits --
// bn3 + identity + ReLU applied by a second pass of conv3's GEMM (trunk.py, reference torchvision Bottleneck
// bn3 -> += identity -> relu inside model/vision/resnet50_tsm.py:15).
//
// Per output row these passes move K x 2 B of x, 2 x 256 x 2 B of residual and output and 32 B of mask bits per
// 256 columns, against 256 x K MACs: at K <= 256 the MFMA work is a small fraction of the memory time. The
// persistent LDS-DMA engine (igemm_fast.hip) issues a tile's residual loads only after its MFMAs and round-trips
// the output through the LDS stage, so every tile pays an exposed HBM latency. Here there is no LDS traffic in the
// loop and no barrier: the conv weights of the workgroup's 256 columns (and their bias) sit in LDS for the whole
// kernel, and every wave streams its own 16-row tiles -- x rows and residual straight into registers one tile
// ahead (the compiler's counted vmcnt keeps the next tile's loads and this tile's stores in flight), 32 / 64 / 128
// MFMAs (v_mfma_f32_16x16x32_bf16, D = W X^T: lane 16g + i holds row i, columns 4g..4g+3 of each 16-column block),
// then the epilogue on the accumulators and 8-B stores. The mask bits of a row are assembled across the four lane
// groups (two lane swaps) and stored as 32 B by one lane.
//
// Same products, summation order and roundings as epilogue_staged_res (bit-identical out and bits).
#include "igemm.h"

namespace vcg {
namespace {

constexpr int RS_NTH = 512;  // 8 waves, one workgroup per CU
constexpr int RS_TN = 256;   // output columns per workgroup

__device__ __forceinline__ int rswz(int row, int chunk) { return chunk ^ ((row >> 1) & 7); }

// B fragment (16 columns r0.., k-substep s2 of one 64-wide k tile [256][64], fast_frag's layout and k map:
// element j of lane 16g+i is k = 32 s2 + 8g + j)
// (inline asm: a plain LDS load of the loop-invariant weights would be hoisted out of the tile loop by the
// compiler -- every fragment of the 256 x K block held in registers, spilled)
typedef __attribute__((address_space(3))) char rs_lds_t;
__device__ __forceinline__ s16x8 rs_bfrag(const bf16_t* Bkt, int r0, int lane, int s2) {
  const int g = lane >> 4, i = lane & 15;
  const int row = r0 + i;
  const uint32_t addr = (uint32_t)(uintptr_t)(const rs_lds_t*)(Bkt + row * 64 + 8 * rswz(row, 4 * s2 + g));
  s16x8 v;
  asm volatile("ds_read_b128 %0, %1" : "=v"(v) : "v"(addr) : "memory");
  return v;
}

// column of the 16-B chunk a lane holds for the 16-column block pair (2p, 2p + 1) after the permlane16 swap of the
// two blocks' packed values: group g = 0 / 1 / 2 / 3 -> columns 32p + 0 / 16 / 8 / 24 .. + 7
__device__ __forceinline__ int rs_col(int p, int g) { return 32 * p + 16 * (g & 1) + 8 * (g >> 1); }

template <int K> struct RsTile {
  uint4 a[K / 32];       // x row i: k = 32 s + 8 g .. + 7
  uint4 r[RS_TN / 32];   // residual row i, the 16-B chunk rs_col(p, g) of block pair p
};

template <int K>
__device__ __forceinline__ void rs_load(RsTile<K>& t, const bf16_t* __restrict__ X, const bf16_t* __restrict__ R,
                                        long long tile, long long M, int N, int n0, int lane) {
  const int g = lane >> 4, i = lane & 15;
  long long m = tile * 16 + i;
  m = m < M ? m : M - 1;  // (clamped: the row's results are not stored)
#pragma unroll
  for (int s = 0; s < K / 32; ++s) t.a[s] = *reinterpret_cast<const uint4*>(X + m * K + 32 * s + 8 * g);
#pragma unroll
  for (int p = 0; p < RS_TN / 32; ++p) t.r[p] = *reinterpret_cast<const uint4*>(R + m * N + n0 + rs_col(p, g));
}

__device__ __forceinline__ void unpack8s(const uint4& u, float (&v)[8]) {
  const uint32_t w[4] = {u.x, u.y, u.z, u.w};
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    v[2 * i] = __uint_as_float(w[i] << 16);
    v[2 * i + 1] = __uint_as_float(w[i] & 0xffff0000u);
  }
}

template <int K>
__device__ __forceinline__ void rs_compute(const RsTile<K>& t, const bf16_t* Bs, const float* bias_s,
                                           bf16_t* __restrict__ out, uint8_t* __restrict__ bits, long long tile,
                                           long long M, int N, int n0, int lane) {
  constexpr int NJ = RS_TN / 16, JG = 4;  // 16-column blocks, done JG at a time (accumulators + B fragments live)
  const int g = lane >> 4, i = lane & 15;
  const long long m = tile * 16 + i;
  const bool ok = m < M;
  uint32_t mb[2] = {0u, 0u};  // this lane's mask bytes of the 8 block pairs
#pragma unroll
  for (int j0 = 0; j0 < NJ; j0 += JG) {
    f32x4 acc[JG];
#pragma unroll
    for (int jj = 0; jj < JG; ++jj) acc[jj] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int s = 0; s < K / 32; ++s) {
      const s16x8 af = __builtin_bit_cast(s16x8, t.a[s]);
      const bf16_t* Bkt = Bs + (s >> 1) * RS_TN * 64;
      s16x8 bf[JG];
#pragma unroll
      for (int jj = 0; jj < JG; ++jj) bf[jj] = rs_bfrag(Bkt, 16 * (j0 + jj), lane, s & 1);
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_sched_barrier(0);  // (the MFMAs must not move above the wait: the asm reads are async)
#pragma unroll
      for (int jj = 0; jj < JG; ++jj) acc[jj] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bf[jj], af, acc[jj], 0, 0, 0);
    }
    // the conv values rounded as the staged epilogue does, packed per block, then one permlane16 swap per block
    // pair gives each lane a 16-B chunk (rs_col): full 16-B residual loads / output stores and a whole mask byte
#pragma unroll
    for (int pp = 0; pp < JG / 2; ++pp) {
      const int p = j0 / 2 + pp;
      uint32_t vw[2][2];
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const int jj = 2 * pp + h, j = j0 + jj;
        const float4 bv = *reinterpret_cast<const float4*>(bias_s + 16 * j + 4 * g);
        vw[h][0] = (uint32_t)f2bf(acc[jj][0] + bv.x) | ((uint32_t)f2bf(acc[jj][1] + bv.y) << 16);
        vw[h][1] = (uint32_t)f2bf(acc[jj][2] + bv.z) | ((uint32_t)f2bf(acc[jj][3] + bv.w) << 16);
      }
#pragma unroll
      for (int d = 0; d < 2; ++d) {
        const auto sw = __builtin_amdgcn_permlane16_swap(vw[0][d], vw[1][d], false, false);
        vw[0][d] = sw[0];
        vw[1][d] = sw[1];
      }
      const uint4 cv = make_uint4(vw[0][0], vw[0][1], vw[1][0], vw[1][1]);  // columns rs_col(p, g) .. + 7
      float a8[8], r8[8];
      unpack8s(cv, a8);
      unpack8s(t.r[p], r8);
      uint32_t byte = 0;
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        a8[e] = fmaxf(a8[e] + r8[e], 0.f);
        byte |= (a8[e] > 0.f ? 1u : 0u) << e;
      }
      const uint4 o = make_uint4((uint32_t)f2bf(a8[0]) | ((uint32_t)f2bf(a8[1]) << 16),
                                 (uint32_t)f2bf(a8[2]) | ((uint32_t)f2bf(a8[3]) << 16),
                                 (uint32_t)f2bf(a8[4]) | ((uint32_t)f2bf(a8[5]) << 16),
                                 (uint32_t)f2bf(a8[6]) | ((uint32_t)f2bf(a8[7]) << 16));
      if (ok) *reinterpret_cast<uint4*>(out + m * N + n0 + rs_col(p, g)) = o;
      mb[p >> 2] |= byte << (8 * (p & 3));  // this lane's byte of pair p: row byte 4p + (0, 2, 1, 3)[g]
    }
  }
  // the row's 32 mask bytes: byte 4p + q comes from lane group (0, 2, 1, 3)[q]'s byte p
  uint32_t gm[4][2];
#pragma unroll
  for (int w = 0; w < 2; ++w) {
    gm[0][w] = mb[w];
    gm[1][w] = (uint32_t)__shfl_xor((int)mb[w], 16);
    gm[2][w] = (uint32_t)__shfl_xor((int)mb[w], 32);
    gm[3][w] = (uint32_t)__shfl_xor((int)mb[w], 48);
  }
  if (g == 0 && ok) {
    uint32_t row[8];
#pragma unroll
    for (int p = 0; p < 8; ++p) {
      const int w = p >> 2, sh = 8 * (p & 3);
      row[p] = ((gm[0][w] >> sh) & 0xffu) | (((gm[2][w] >> sh) & 0xffu) << 8) | (((gm[1][w] >> sh) & 0xffu) << 16) |
               (((gm[3][w] >> sh) & 0xffu) << 24);
    }
    uint8_t* bp = bits + ((m * N + n0) >> 3);
    *reinterpret_cast<uint4*>(bp) = make_uint4(row[0], row[1], row[2], row[3]);
    *reinterpret_cast<uint4*>(bp + 16) = make_uint4(row[4], row[5], row[6], row[7]);
  }
}

template <int K>
__global__ __launch_bounds__(RS_NTH) void rs1x1_bnres_kernel(const bf16_t* __restrict__ X, const bf16_t* __restrict__ W,
                                                            const float* __restrict__ bias,
                                                            const bf16_t* __restrict__ R, bf16_t* __restrict__ out,
                                                            uint8_t* __restrict__ bits, long long M, int N) {
  __shared__ __attribute__((aligned(1024))) bf16_t Bs[RS_TN * K];
  __shared__ __attribute__((aligned(16))) float bias_s[RS_TN];
  const int ncb = N / RS_TN;
  const int cb = blockIdx.x % ncb, q = blockIdx.x / ncb, nq = gridDim.x / ncb;
  const int n0 = cb * RS_TN;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  // the workgroup's weights [256][K] as K / 64 swizzled k tiles [256][64], and the bias
  for (int c = tid; c < RS_TN * K / 8; c += RS_NTH) {
    const int row = c / (K / 8), ch = c % (K / 8);
    const uint4 v = *reinterpret_cast<const uint4*>(W + (long long)(n0 + row) * K + 8 * ch);
    *reinterpret_cast<uint4*>(Bs + (ch >> 3) * RS_TN * 64 + row * 64 + 8 * rswz(row, ch & 7)) = v;
  }
  for (int c = tid; c < RS_TN; c += RS_NTH) bias_s[c] = bias[n0 + c];
  __syncthreads();
  const long long ntiles = (M + 15) / 16;
  const long long stride = (long long)nq * (RS_NTH / 64);
  long long t = (long long)q * (RS_NTH / 64) + wave;
  // the next tile's loads are issued unconditionally (a tile index past the end is clamped to the last tile and
  // its data unused): with a conditional issue the compiler's vmcnt has to assume the loads may be absent and
  // waits for the NEXT tile's data before using this one's -- one exposed HBM round trip per tile
  if (t >= ntiles) return;
  const long long last = ntiles - 1;
  RsTile<K> T0, T1;
  rs_load<K>(T0, X, R, t, M, N, n0, lane);
  for (; t < ntiles; t += 2 * stride) {
    rs_load<K>(T1, X, R, min(t + stride, last), M, N, n0, lane);
    rs_compute<K>(T0, Bs, bias_s, out, bits, t, M, N, n0, lane);
    if (t + stride >= ntiles) break;
    rs_load<K>(T0, X, R, min(t + 2 * stride, last), M, N, n0, lane);
    rs_compute<K>(T1, Bs, bias_s, out, bits, t + stride, M, N, n0, lane);
  }
}

// ---- the fused 1x1 input gradient (EPI_BWD of igemm_fast.hip with mask bits and no y: the trunk's conv1 dgrads
// whose previous block's y3 is not stored) on the same register-streaming schedule ------------------------------
// g[d][n] = bf16(mask(d, n) ? bf16(sum_k dy[d - s(n) hw][k] w[n][k]) + res[d][n] : 0), with the TSM adjoint's
// shift s(n) = +1 / -1 / 0 for n < fold / < 2 fold / the rest (source rows outside the clip contribute 0), and the
// column sums of the stored g (sum_g of the previous block's bn3 backward). The A rows of each shift present in the
// workgroup's 256 columns (NV variants) are loaded one tile ahead like the residual and the row's 32 mask bytes; the
// column sums of a tile are reduced over the 16 rows in DPP (row16_sum) and kept by the lane that owns the column.
// Same products, order and roundings as bwd_stream_body / stage_flush_bwd (bit-identical g; the column sums are
// the same values summed in another order).
template <int K, int NV> struct RdTile {
  uint4 a[NV][K / 32];  // dy row d - s_v hw (zero outside the clip): k = 32 s + 8 g .. + 7
  uint4 r[RS_TN / 32];  // residual row d, the 16-B chunk rs_col(p, g)
  uint4 b0, b1;         // mask bytes of row d (32 = the workgroup's 256 columns)
};

struct RdArgs {
  const bf16_t* A;
  const bf16_t* R;
  const uint8_t* bits;
  bf16_t* out;
  float* part;
  long long M;
  int N, T, fold, hw;
  FastDiv fd_hw, fd_T;
  int res_s, rH, rW, W;  // res_s 2: R is the compact [frames][rH][rW][N] gradient of a 1x1 / stride-2 conv, added
  FastDiv fd_w;          //           at the even (h, w) rows only
};

template <int K, int NV>
__device__ __forceinline__ void rd_load(RdTile<K, NV>& t, const RdArgs& q, const int (&sv)[NV], long long tile, int n0,
                                        int lane) {
  const int g = lane >> 4, i = lane & 15;
  long long d = tile * 16 + i;
  d = d < q.M ? d : q.M - 1;
  int tt = 0;
  const int f = (q.T > 0 || q.res_s > 1) ? (int)fdiv((uint32_t)d, q.fd_hw) : 0;
  if (q.T > 0) tt = f - (int)fdiv((uint32_t)f, q.fd_T) * q.T;
#pragma unroll
  for (int v = 0; v < NV; ++v) {
    const bool ok = q.T <= 0 || (unsigned)(tt - sv[v]) < (unsigned)q.T;
    const long long src = ok ? d - (long long)sv[v] * q.hw : d;
#pragma unroll
    for (int s = 0; s < K / 32; ++s) {
      const uint4 x = *reinterpret_cast<const uint4*>(q.A + src * K + 32 * s + 8 * g);
      t.a[v][s] = ok ? x : make_uint4(0u, 0u, 0u, 0u);
    }
  }
  long long rrow = d;
  bool rok = true;
  if (q.res_s > 1) {
    const int rr = (int)(d - (long long)f * q.hw), h = (int)fdiv((uint32_t)rr, q.fd_w), w = rr - h * q.W;
    rok = ((h | w) & 1) == 0;
    rrow = rok ? ((long long)f * q.rH + (h >> 1)) * q.rW + (w >> 1) : 0;
  }
#pragma unroll
  for (int p = 0; p < RS_TN / 32; ++p) {
    const uint4 x = *reinterpret_cast<const uint4*>(q.R + rrow * q.N + n0 + rs_col(p, g));
    t.r[p] = rok ? x : make_uint4(0u, 0u, 0u, 0u);
  }
  const uint8_t* bp = q.bits + ((d * q.N + n0) >> 3);
  t.b0 = *reinterpret_cast<const uint4*>(bp);
  t.b1 = *reinterpret_cast<const uint4*>(bp + 16);
}

__device__ __forceinline__ uint32_t byte_of(const uint4& b0, const uint4& b1, int k) {  // byte k (0..31)
  const uint32_t w[8] = {b0.x, b0.y, b0.z, b0.w, b1.x, b1.y, b1.z, b1.w};
  uint32_t r = 0;
#pragma unroll
  for (int x = 0; x < 8; ++x) r = (k >> 2) == x ? w[x] : r;
  return (r >> (8 * (k & 3))) & 0xffu;
}

// FJ = 0: one TSM shift for all of the workgroup's columns (NV 1); FJ > 0: the workgroup holds columns 0..255
// with the shifts +1 for 16-column blocks j < FJ, -1 for FJ <= j < 2 FJ, 0 after (fold = 16 FJ): the shift
// variant of every block is a compile-time index
__host__ __device__ constexpr int rd_nv(int FJ) { return FJ == 0 ? 1 : (2 * FJ >= RS_TN / 16 ? 2 : 3); }
__host__ __device__ constexpr int rd_var(int FJ, int j) { return FJ == 0 ? 0 : (j < FJ ? 0 : (j < 2 * FJ ? 1 : 2)); }

template <int K, int FJ, int NV = rd_nv(FJ)>
__device__ __forceinline__ void rd_compute(const RdTile<K, NV>& t, const RdArgs& q, const bf16_t* Bs, float (&cs)[4],
                                           long long tile, int n0, int lane) {
  constexpr int NJ = RS_TN / 16, JG = 4;
  const int g = lane >> 4, i = lane & 15;
  const long long d = tile * 16 + i;
  const bool ok = d < q.M;
  const int off = (g & 1) * 2 + (g >> 1);  // this lane's byte of each 4-byte group: rs_col(p, g) / 8 - 4p
#pragma unroll
  for (int j0 = 0; j0 < NJ; j0 += JG) {
    f32x4 acc[JG];
#pragma unroll
    for (int jj = 0; jj < JG; ++jj) acc[jj] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int s = 0; s < K / 32; ++s) {
      const bf16_t* Bkt = Bs + (s >> 1) * RS_TN * 64;
      s16x8 bf[JG];
#pragma unroll
      for (int jj = 0; jj < JG; ++jj) bf[jj] = rs_bfrag(Bkt, 16 * (j0 + jj), lane, s & 1);
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int jj = 0; jj < JG; ++jj)  // (this block's shift variant: a compile-time index)
        acc[jj] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(
            bf[jj], __builtin_bit_cast(s16x8, t.a[rd_var(FJ, j0 + jj)][s]), acc[jj], 0, 0, 0);
    }
#pragma unroll
    for (int pp = 0; pp < JG / 2; ++pp) {
      const int p = j0 / 2 + pp;
      uint32_t vw[2][2];
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const int jj = 2 * pp + h;
        vw[h][0] = (uint32_t)f2bf(acc[jj][0]) | ((uint32_t)f2bf(acc[jj][1]) << 16);
        vw[h][1] = (uint32_t)f2bf(acc[jj][2]) | ((uint32_t)f2bf(acc[jj][3]) << 16);
      }
#pragma unroll
      for (int dd = 0; dd < 2; ++dd) {
        const auto sw = __builtin_amdgcn_permlane16_swap(vw[0][dd], vw[1][dd], false, false);
        vw[0][dd] = sw[0];
        vw[1][dd] = sw[1];
      }
      float a8[8], r8[8];
      unpack8s(make_uint4(vw[0][0], vw[0][1], vw[1][0], vw[1][1]), a8);
      unpack8s(t.r[p], r8);
      const uint32_t mb = byte_of(t.b0, t.b1, 4 * p + off);
      float gs[8];
#pragma unroll
      for (int e = 0; e < 8; ++e) gs[e] = ((mb >> e) & 1u) ? a8[e] + r8[e] : 0.f;
      const uint4 o = make_uint4((uint32_t)f2bf(gs[0]) | ((uint32_t)f2bf(gs[1]) << 16),
                                 (uint32_t)f2bf(gs[2]) | ((uint32_t)f2bf(gs[3]) << 16),
                                 (uint32_t)f2bf(gs[4]) | ((uint32_t)f2bf(gs[5]) << 16),
                                 (uint32_t)f2bf(gs[6]) | ((uint32_t)f2bf(gs[7]) << 16));
      if (ok) *reinterpret_cast<uint4*>(q.out + d * q.N + n0 + rs_col(p, g)) = o;
      // column sums of the stored (rounded) g over the tile's 16 rows; value 8p + e is kept by lane i = (8p+e) % 16
      unpack8s(o, gs);
#ifndef VCG_RD_NOSUM
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const float tot = row16_sum(ok ? gs[e] : 0.f);
        const int v = 8 * p + e;
        cs[v >> 4] += i == (v & 15) ? tot : 0.f;
      }
#endif
    }
  }
}

template <int K, int FJ, int NV = rd_nv(FJ)>
__device__ __forceinline__ void rd_body(const RdArgs& q, const int (&sv)[NV], const bf16_t* Bs, float (&cs)[4],
                                        long long t0, long long stride, int n0, int lane) {
  const long long ntiles = (q.M + 15) / 16;
  if (t0 >= ntiles) return;
  const long long last = ntiles - 1;
  // two tiles ahead (one wave per SIMD, 512 VGPRs; next-tile loads unconditional: see rs1x1_bnres_kernel)
  RdTile<K, NV> T0, T1, T2;
  rd_load<K, NV>(T0, q, sv, t0, n0, lane);
  rd_load<K, NV>(T1, q, sv, min(t0 + stride, last), n0, lane);
  for (long long t = t0; t < ntiles; t += 3 * stride) {
    rd_load<K, NV>(T2, q, sv, min(t + 2 * stride, last), n0, lane);
    rd_compute<K, FJ>(T0, q, Bs, cs, t, n0, lane);
    if (t + stride >= ntiles) break;
    rd_load<K, NV>(T0, q, sv, min(t + 3 * stride, last), n0, lane);
    rd_compute<K, FJ>(T1, q, Bs, cs, t + stride, n0, lane);
    if (t + 2 * stride >= ntiles) break;
    rd_load<K, NV>(T1, q, sv, min(t + 4 * stride, last), n0, lane);
    rd_compute<K, FJ>(T2, q, Bs, cs, t + 2 * stride, n0, lane);
  }
}

#ifdef VCG_RD_8W
constexpr int RD_NTH = 512;
#else
constexpr int RD_NTH = 256;  // 4 waves, one per SIMD (each with 512 VGPRs: three tiles of operands in flight)
#endif

template <int K>
#ifdef VCG_RD_8W
__global__ __launch_bounds__(RD_NTH)
#else
__global__ __launch_bounds__(RD_NTH) __attribute__((amdgpu_waves_per_eu(1, 1)))
#endif
void rs1x1_dgrad_kernel(const bf16_t* __restrict__ W, RdArgs q) {
  __shared__ __attribute__((aligned(1024))) bf16_t Bs[RS_TN * K];
  __shared__ float red[RD_NTH / 64][RS_TN];
  const int ncb = q.N / RS_TN;
  const int cb = blockIdx.x % ncb, slot = blockIdx.x / ncb, nq = gridDim.x / ncb;
  const int n0 = cb * RS_TN;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  for (int c = tid; c < RS_TN * K / 8; c += RD_NTH) {
    const int row = c / (K / 8), ch = c % (K / 8);
    const uint4 v = *reinterpret_cast<const uint4*>(W + (long long)(n0 + row) * K + 8 * ch);
    *reinterpret_cast<uint4*>(Bs + (ch >> 3) * RS_TN * 64 + row * 64 + 8 * rswz(row, ch & 7)) = v;
  }
  __syncthreads();
  const long long stride = (long long)nq * (RD_NTH / 64);
  const long long t0 = (long long)slot * (RD_NTH / 64) + wave;
  float cs[4] = {0.f, 0.f, 0.f, 0.f};
  // this workgroup's shifts: one for all its columns, or (first block) +1 / -1 / 0 ranges at fold = 16 FJ
  const int fj = q.T > 0 ? q.fold / 16 : 0;
  const bool mixed = q.T > 0 && n0 < 2 * q.fold && n0 + RS_TN > q.fold;
  if (!mixed) {
    const int sv[1] = {q.T <= 0 ? 0 : (n0 < q.fold ? 1 : (n0 < 2 * q.fold ? -1 : 0))};
    rd_body<K, 0>(q, sv, Bs, cs, t0, stride, n0, lane);
  } else if (fj == 2) {
    const int sv[3] = {1, -1, 0};
    rd_body<K, 2>(q, sv, Bs, cs, t0, stride, n0, lane);
  } else if (fj == 4) {
    const int sv[3] = {1, -1, 0};
    rd_body<K, 4>(q, sv, Bs, cs, t0, stride, n0, lane);
  } else {  // fj == 8 (rs_dgrad_ok)
    const int sv[2] = {1, -1};
    rd_body<K, 8>(q, sv, Bs, cs, t0, stride, n0, lane);
  }
  // per-wave column sums -> the workgroup's slot row (waves combined in a fixed order)
  const int g = lane >> 4, i = lane & 15;
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const int v = 16 * k + i, p = v >> 3, e = v & 7;
    red[wave][rs_col(p, g) + e] = cs[k];
  }
  __syncthreads();
  for (int c = tid; c < RS_TN; c += RD_NTH) {
    float a = 0.f;
#pragma unroll
    for (int w = 0; w < RD_NTH / 64; ++w) a += red[w][c];
    float* out = q.part + (long long)slot * 2 * q.N + n0 + c;
    out[0] = a;
    out[q.N] = 0.f;  // (no y: the sum against y comes from elsewhere, trunk.py's y3 drop)
  }
}

int rs_grid(int N) {
  int dev = 0, cus = 256;
  if (hipGetDevice(&dev) == hipSuccess) (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
  const int ncb = N / RS_TN;
  return (cus / ncb) * ncb;
}

}  // namespace

// the fused 1x1 dgrad with mask bits and no y on the register-streaming kernel: eligible / partial-sum slots
bool rs_dgrad_ok(const GemmParams& p) {
  // opt-in (VCG_RS_DGRAD=1): at the l1 conv1 shape it ran no faster than the LDS-ring stream kernel (1189 vs 1147 us
  // one-stream, profiles/r04_final_gemm_breakdown.txt), at 4.1-4.2 TB/s either way
  const char* v = getenv("VCG_RS_DGRAD");
  if (!v || v[0] != '1') return false;
  const BwdEpi& e = p.bwd;
  const bool dense = p.a.KH == 0 && p.a.GH == 0;
  if (!dense || (p.K != 64 && p.K != 128) || p.N % RS_TN != 0 || p.N / RS_TN > 8 || p.batch_inner > 0 ||
      p.ldc != p.N || p.a.ld != p.K || p.a.ptr2)
    return false;
  if (!e.res || (e.res_s != 1 && (e.res_s != 2 || p.M % e.hw != 0)) || !e.bits || e.y || e.y2 || e.msc || e.sub || e.nred != 2) return false;
  // TSM shifts: each 256-column block has one shift, or is block 0 with fold = 32 / 64 / 128 (rs1x1_dgrad_kernel)
  if (e.tsm_T > 0) {
    const int f = e.tsm_fold;
    if (f % 16 != 0) return false;
    for (int n0 = 0; n0 < p.N; n0 += RS_TN) {
      const bool mixed = n0 < 2 * f && n0 + RS_TN > f;
      if (mixed && (n0 != 0 || (f != 32 && f != 64 && f != 128))) return false;
    }
  }
  return (((uintptr_t)p.C | (uintptr_t)e.res | (uintptr_t)e.bits | (uintptr_t)p.a.ptr) & 15) == 0;
}
int rs_dgrad_slots(const GemmParams& p) { return rs_grid(p.N) / (p.N / RS_TN); }

int run_rs1x1_dgrad(const GemmParams& p, hipStream_t s) {
  const BwdEpi& e = p.bwd;
  RdArgs q;
  q.A = (const bf16_t*)p.a.ptr;
  q.R = (const bf16_t*)e.res;
  q.bits = e.bits;
  q.out = (bf16_t*)p.C;
  q.part = e.part;
  q.M = p.M;
  q.N = p.N;
  q.T = e.tsm_T > 0 ? e.tsm_T : 0;
  q.fold = e.tsm_fold;
  q.hw = e.hw;
  q.fd_hw = e.fd_hw;
  q.fd_T = e.fd_T;
  q.res_s = e.res_s;
  q.rH = e.rH;
  q.rW = e.rW;
  q.fd_w = e.fd_w;
  q.W = e.fd_w.d;
  const int g = rs_grid(p.N);
  if (p.K == 64)
    hipLaunchKernelGGL(rs1x1_dgrad_kernel<64>, dim3(g), dim3(RD_NTH), 0, s, (const bf16_t*)p.b.ptr, q);
  else
    hipLaunchKernelGGL(rs1x1_dgrad_kernel<128>, dim3(g), dim3(RD_NTH), 0, s, (const bf16_t*)p.b.ptr, q);
  VCG_LAUNCH_CHECK();
  return VCG_OK;
}

// relu(bf16(x wfold^T + bias) + res) + mask bits on the register-streaming kernel; -1: not eligible (the caller
// runs the persistent engine). x [M][K], wfold [N][K], res / out [M][N] bf16, bits [M N / 8].
int run_rs1x1_bnres(const void* x, const void* wfold, const float* bias, const void* res, void* out, uint8_t* bits,
                    long long M, int N, int K, hipStream_t s) {
  const char* e = getenv("VCG_RS1X1");  // (read per call: tests A/B both engines in one process)
  if ((e && e[0] == '0') || (K != 64 && K != 128 && K != 256) || N % RS_TN != 0 || N / RS_TN > 8 || M <= 0) return -1;
  const int g = rs_grid(N);
  if (K == 64)
    hipLaunchKernelGGL(rs1x1_bnres_kernel<64>, dim3(g), dim3(RS_NTH), 0, s, (const bf16_t*)x, (const bf16_t*)wfold,
                       bias, (const bf16_t*)res, (bf16_t*)out, bits, M, N);
  else if (K == 128)
    hipLaunchKernelGGL(rs1x1_bnres_kernel<128>, dim3(g), dim3(RS_NTH), 0, s, (const bf16_t*)x, (const bf16_t*)wfold,
                       bias, (const bf16_t*)res, (bf16_t*)out, bits, M, N);
  else
    hipLaunchKernelGGL(rs1x1_bnres_kernel<256>, dim3(g), dim3(RS_NTH), 0, s, (const bf16_t*)x, (const bf16_t*)wfold,
                       bias, (const bf16_t*)res, (bf16_t*)out, bits, M, N);
  VCG_LAUNCH_CHECK();
  return VCG_OK;
}

}  // namespace vcg
