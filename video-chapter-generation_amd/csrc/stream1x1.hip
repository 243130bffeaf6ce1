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

int rs_grid(int N) {
  int dev = 0, cus = 256;
  if (hipGetDevice(&dev) == hipSuccess) (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
  const int ncb = N / RS_TN;
  return (cus / ncb) * ncb;
}

}  // namespace

// relu(bf16(x wfold^T + bias) + res) + mask bits on the register-streaming kernel; -1: not eligible (the caller
// runs the persistent engine). x [M][K], wfold [N][K], res / out [M][N] bf16, bits [M N / 8].
int run_rs1x1_bnres(const void* x, const void* wfold, const float* bias, const void* res, void* out, uint8_t* bits,
                    long long M, int N, int K, hipStream_t s) {
  const char* e = getenv("VCG_RS1X1");  // (read per call: tests A/B both engines in one process)
  if ((e && e[0] == '0') || (K != 64 && K != 128 && K != 256) || N % RS_TN != 0 || N / RS_TN > 8 || M <= 0) return -1;
  const int g = rs_grid(N);
  if (census_on()) { char t_[96]; snprintf(t_, sizeof(t_), "rs1x1_bnres"); census_add(t_, M, N, K); }
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
