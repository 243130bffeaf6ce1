// Shared declarations of the MFMA implicit-GEMM engine (igemm.hip, igemm_fast.hip).
#pragma once
#include "common.h"

namespace vcg {

enum { OP_DENSE_K = 0, OP_IM2COL = 1, OP_DGRAD = 2, OP_DENSE_MN = 3, OP_IM2COL_T = 4 };
// EPI_BWD_AFF: EPI_BWD without residual / mask bits / second BN / TSM (the conv2 / conv3 input gradients: mask
// recomputed from y, BN sums): fewer live registers, so the 64-column kernel fits 3 workgroups per CU
// EPI_STORE_AUX (fast kernel): EPI_STORE whose pre-activation copy `aux` (the GELU input the backward needs) also
// goes out through the LDS stage, in a round of its own
// EPI_BWD_STREAM (fast kernel): EPI_BWD of a 1x1 conv input gradient with K <= 128 (the conv1 dgrads of layers 1-2,
// where the epilogue's residual / y / mask operands are 4-6x the A operand): 64 x 64 tiles whose A rows AND epilogue
// operands are DMA'd into an LDS ring several tiles ahead (igemm_fast.hip bwd_stream_body)
enum { EPI_STORE = 0, EPI_STATS = 1, EPI_SPLITK = 2, EPI_BWD = 3, EPI_BWD_AFF = 4, EPI_STORE_AUX = 5,
       EPI_BWD_STREAM = 6 };
enum { ACT_NONE = 0, ACT_RELU = 1, ACT_GELU = 2, ACT_TANH = 3, ACT_GELU_BWD = 4 };
enum { ACT_FLAG_ROUND_PRE = 0x100 };  // = VCG_ACT_FLAG_ROUND_PRE (include/vcg_hip.h)
enum { ACT_FLAG_WIDE = 0x200 };       // = VCG_ACT_FLAG_WIDE: run this GEMM on the wide-tile engine (igemm_wide.hip)
enum { ACT_FLAG_F32_OUT = 0x400 };    // = VCG_ACT_FLAG_F32_OUT: fp32 residual and output (wide engine, bf16 operands)

template <typename T> struct Cfg;
template <> struct Cfg<float> { static constexpr int VEC = 4, BK = 16, LDK = 20; };   // 80-B rows
template <> struct Cfg<bf16_t> { static constexpr int VEC = 8, BK = 32, LDK = 40; };  // 80-B rows

template <typename T, int COLS> struct LdMN {
  // padded element stride of a [BK][COLS] tile (bank-conflict-free for the fragment reads)
  static constexpr int v = sizeof(T) == 2 ? (COLS == 128 ? 144 : 80) : (COLS == 128 ? 132 : 68);
};

constexpr bool is_kcontig(int mode) { return mode == OP_DENSE_K || mode == OP_IM2COL || mode == OP_DGRAD; }

struct OpArgs {
  const void* ptr;
  long long bytes;  // extent of the tensor behind ptr (buffer-descriptor range for LDS-DMA loads)
  long long ld;   // dense modes: leading dimension in elements
  int rows;       // number of valid rows (K-contig) / cols (MN-contig)
  // conv geometry (gather modes)
  int N, H, W, C, logC;  // gathered tensor is NHWC [N][H][W][C] (C power of two)
  int GH, GW;            // grid that indexes the rows (IM2COL: output; DGRAD: dx; IM2COL_T: dy)
  int KH, KW, stride, pad;
  int tsm_T, tsm_fold;   // TSM temporal shift fused into the gather (fold = 0: off)
  FastDiv fd_ghw, fd_gw, fd_T;
  // sub-pixel class of a stride-2 dgrad (fast kernel, tKW > 0): the GH x GW row grid is the pixels
  // (2i + ry, 2j + rx) of the dx image, and the k tiles walk only the taps that reach them,
  // kh = tkh0 + 2a (a < tKH), kw = tkw0 + 2b (b < tKW) -- 1, 2 or 4 of the 9 taps of a 3x3 kernel
  int tKH, tKW, tkh0, tkw0, ry, rx;
  // w-direction stride / pad of an im2col gather when they differ from (stride, pad) (sw = 0: the same).
  // The pair-packed stem (vcg_conv_fwd / vcg_conv_wgrad, bf16, C = 4, stride 2): W / C / KW describe the
  // image as W/2 "super pixels" of 8 channels (two adjacent RGB0 pixels, one 16-B chunk) that a stride-2
  // tap pair reads together: sw = 1, pw = the super-pixel pad, KW = the super-pixel tap count.
  int sw, pw;
  // second source (fast dense A, OP_DENSE_K2: k tiles k0 >= split2 read ptr2 at k - split2, same rows / ld;
  // wgrad_fast_kernel's dense MN A: output rows m >= split2 read ptr2 at column m - split2): the BatchNorm
  // backward folded into its consumer GEMM reads [g | y] as one operand (vcg_conv_dgrad_bwd_bnfold)
  const void* ptr2;
  int split2;
  long long ld2, bytes2;  // the second source's leading dimension / extent (0: those of the first)
};

// EPI_BWD (fast kernel, conv dgrad): the epilogue of a conv input gradient inside the trunk backward.
// Per output element (row m, column n), in this order:
//   * TSM adjoint (tsm_T > 0): the value moves to row m + hw (n < fold) / m - hw (fold <= n < 2 fold), i.e. one
//     frame later / earlier inside its clip of tsm_T frames; at the clip edge it is dropped and the
//     destination row of the wrap (frame 0 / tsm_T - 1) receives zero -- every element is written once;
//   * + res[dst] (residual gradient; res_s > 1: compact strided residual, see res_s);
//   * mask: bits[dst / 8] bit (dst % 8) (ReLU mask bytes of vcg_bn_apply) or fma(y, msc, msh) > 0 (the
//     forward's BN + ReLU decision recomputed from the saved pre-BN y);
//   * stored (bf16) as g, and reduced per column: part[slot][0][n] = sum g, part[slot][1][n] = sum
//     g * (y - mean) * invstd, part[slot][2][n] = sum g * (y2 - mean2) * invstd2 (second BatchNorm fed by the
//     same gradient: the downsample branch), slot = the workgroup's grid row (bwd_slots rows in all).
struct BwdEpi {
  int tsm_T, tsm_fold;
  FastDiv fd_hw, fd_T;
  int hw;
  const void* res;
  int res_s;       // > 1: res is the compact [N][H/res_s][W/res_s][C] input gradient of a 1x1 stride-res_s conv
  int rH, rW;      //      (rows whose h or w is not a multiple of res_s get no residual); rH, rW its grid
  FastDiv fd_w;    //      and the row decode h = (m % hw) / W
  const uint8_t* bits;
  const void* y;
  const float *mean, *invstd, *msc, *msh;
  const void* y2;
  const float *mean2, *invstd2;
  float* part;  // [slots][nred][N]
  int nred;     // 0 (no reduction), 2 or 3
  // the previous block's conv3 weight-gradient product P = g^T a2 accumulated from the stored g (streaming kernel,
  // mask bits without y): a2 [M][pj] bf16 (pj 64 / 128, 0: off), ppart [slots][N][pj] f32 partials
  const void* a2;
  int pj;
  float* ppart;
  // sub-pixel class rows (sub != 0): GEMM row m = (f, i, j) of the cH x cW class grid is dx row
  // f * fH * fW + (2i + ry) * fW + (2j + rx)
  int sub, cW, ry, rx, fH, fW;
  FastDiv fd_chw, fd_cw;
};

struct GemmParams {
  int M, N, K;
  int k_per_split;  // multiple of BK
  OpArgs a, b;
  void* C;
  long long ldc;
  const float* bias;
  int act;
  const void* residual;
  long long ldr;
  void* aux;  // optional copy of the pre-activation value
  float alpha;
  float* stats;  // EPI_STATS: float2 [N][mtiles] (mean, M2) per column per m-tile
  float* ws;     // EPI_SPLITK: fp32 slabs [split][M][N]
  // batched mode (batch_inner > 0): blockIdx.z = zo * batch_inner + zi selects element offsets
  int batch_inner;
  long long a_so, a_si, b_so, b_si, c_so, c_si;
  int res_round; // residual epilogue: round alpha*AB + bias to bf16 before adding the residual (VCG_ACT_FLAG_ROUND_PRE)
  int fast_act;  // bf16 epilogues: GELU / GELU' through erf_fast (common.h) instead of erff (VCG_FAST_GELU=0: off)
  BwdEpi bwd;    // EPI_BWD
  // EPI_STORE + residual + ReLU through the stage (epilogue_staged_res): also store the ReLU decisions as mask bits,
  // byte (m N + n) / 8 bit n % 8 (vcg_bn_apply's bits layout; vcg_conv1x1_bn_res_relu)
  uint8_t* obits;
  const float *res_sc, *res_sh;  // epilogue_staged_res: residual r -> fma(r, res_sc[n], res_sh[n]) (a BN'd residual)
};


template <typename T> __device__ __forceinline__ void load4(const T* p, float (&v)[4]) {
  if constexpr (sizeof(T) == 4) {
    const float4 q = *reinterpret_cast<const float4*>(p);
    v[0] = q.x; v[1] = q.y; v[2] = q.z; v[3] = q.w;
  } else {
    const uint2 q = *reinterpret_cast<const uint2*>(p);
    v[0] = __uint_as_float(q.x << 16); v[1] = __uint_as_float(q.x & 0xffff0000u);
    v[2] = __uint_as_float(q.y << 16); v[3] = __uint_as_float(q.y & 0xffff0000u);
  }
}
template <typename T> __device__ __forceinline__ void store4(T* p, const float (&v)[4]) {
  if constexpr (sizeof(T) == 4) {
    *reinterpret_cast<float4*>(p) = make_float4(v[0], v[1], v[2], v[3]);
  } else {
    uint2 q;
    q.x = (uint32_t)f2bf(v[0]) | ((uint32_t)f2bf(v[1]) << 16);
    q.y = (uint32_t)f2bf(v[2]) | ((uint32_t)f2bf(v[3]) << 16);
    *reinterpret_cast<uint2*>(p) = q;
  }
}

__device__ __forceinline__ float apply_act(float v, int act, bool fast = false) {
  if (act == ACT_RELU) return fmaxf(v, 0.f);
  if (act == ACT_GELU) return fast ? gelu_erf_fast(v) : gelu_erf(v);
  if (act == ACT_TANH) return tanhf(v);
  return v;
}


// Sum over the 16 lanes of a DPP row (lanes 16g..16g+15); every lane of the row gets the total.
__device__ __forceinline__ float row16_sum(float v) {
  v += __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), 0xB1, 0xF, 0xF, false));
  v += __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), 0x4E, 0xF, 0xF, false));
  v += __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), 0x141, 0xF, 0xF, false));
  v += __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), 0x140, 0xF, 0xF, false));
  return v;
}

// Bias of the 4*BN/32 columns a lane owns in the epilogue (zeros without bias / beyond N).
template <int BN>
__device__ __forceinline__ void load_bias(float (&bv)[BN / 32][4], const float* bias, int n0, int wn, int lane, int N) {
#pragma unroll
  for (int j = 0; j < BN / 32; ++j) {
    const int n = n0 + wn * (BN / 2) + 4 * (lane >> 4) + j * 16;
    float4 b4 = make_float4(0.f, 0.f, 0.f, 0.f);
    if (bias && n < N) b4 = *reinterpret_cast<const float4*>(bias + n);
    bv[j][0] = b4.x; bv[j][1] = b4.y; bv[j][2] = b4.z; bv[j][3] = b4.w;
  }
}

// Barrier for the epilogue's LDS exchange: waits only for this wave's LDS ops, so an LDS-DMA
// prefetch of the next tile (fast kernel) stays in flight.
__device__ __forceinline__ void ep_barrier() {
  __builtin_amdgcn_s_waitcnt(0xC07F);  // lgkmcnt(0)
  __builtin_amdgcn_s_barrier();
}

// Epilogue shared by the generic and fast kernels: acc[i][j][r] = C[m][n] with
// m = m0 + wm*(BM/2) + i*16 + (lane&15), n = n0 + wn*(BN/2) + j*16 + 4*(lane>>4) + r.
// bv[j][r] is the bias of column nbase + j*16 + r (zeros when there is none; see load_bias).
// EPI_STATS: `red` holds 4*BN floats that no other wave touches until the caller's next barrier;
// the per-column (mean, M2) of this tile goes to stats[col][mtile] (float2, mtiles per column) and
// the tile's row count to the count row stats[N][mtile].
// Each wave reduces its 64 rows in registers (two passes, DPP row sums), the two row-halves are
// merged with Chan's formula after one barrier, and only then are the values stored, so the
// barrier never waits on outstanding HBM writes.
template <typename T, int BM, int BN, int EPI>
__device__ __forceinline__ void gemm_epilogue(f32x4 (&acc)[BM / 32][BN / 32], const GemmParams& p, float* red,
                                              const float (&bv)[BN / 32][4], T* Cout, const T* Res, int m0, int n0,
                                              int wm, int wn, int lane, int mtile, int mtiles) {
  constexpr int MT = BM / 32, NT = BN / 32;
  const int g = lane >> 4, ci = lane & 15;
  const int mbase = m0 + wm * (BM / 2) + ci, nbase = n0 + wn * (BN / 2) + 4 * g;
#pragma unroll
  for (int j = 0; j < NT; ++j) {
    const int n = nbase + j * 16;
#pragma unroll
    for (int i = 0; i < MT; ++i) {
      const int m = mbase + i * 16;
      if (m >= p.M || n >= p.N) {
        acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
        continue;
      }
      float v[4];
#pragma unroll
      for (int r = 0; r < 4; ++r) v[r] = acc[i][j][r] * p.alpha + bv[j][r];
      if (Res) {
        float rv[4];
        load4<T>(Res + (long long)m * p.ldr + n, rv);
        if (p.act == ACT_GELU_BWD) {
#pragma unroll
          for (int r = 0; r < 4; ++r) v[r] *= (sizeof(T) == 2 && p.fast_act) ? gelu_erf_grad_fast(rv[r]) : gelu_erf_grad(rv[r]);
        } else {
#pragma unroll
          for (int r = 0; r < 4; ++r) v[r] += rv[r];
        }
      }
      if (p.aux) store4<T>(reinterpret_cast<T*>(p.aux) + (long long)m * p.ldc + n, v);
      if (p.act != ACT_NONE && p.act != ACT_GELU_BWD) {
#pragma unroll
        for (int r = 0; r < 4; ++r) v[r] = apply_act(v[r], p.act, sizeof(T) == 2 && p.fast_act);
      }
      if constexpr (EPI == EPI_STATS) {
#pragma unroll
        for (int r = 0; r < 4; ++r) acc[i][j][r] = to_f<T>(from_f<T>(v[r]));  // the stored (rounded) value
      } else {
        store4<T>(Cout + (long long)m * p.ldc + n, v);
      }
    }
  }
  if constexpr (EPI == EPI_STATS) {
    const int r0 = m0 + wm * (BM / 2);
    const int cw = min(BM / 2, max(0, p.M - r0));  // valid rows of this wave's half
    const float inv_cw = cw > 0 ? 1.f / (float)cw : 0.f;
#pragma unroll
    for (int j = 0; j < NT; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        float t = 0.f;
#pragma unroll
        for (int i = 0; i < MT; ++i) t += acc[i][j][r];  // rows beyond M are zero
        t = row16_sum(t);
        const float mean = t * inv_cw;
        float q = 0.f;
#pragma unroll
        for (int i = 0; i < MT; ++i) {
          const float d = acc[i][j][r] - mean;
          q += (mbase + i * 16 < p.M) ? d * d : 0.f;
        }
        q = row16_sum(q);
        if (ci == 0) {
          const int lc = wn * (BN / 2) + j * 16 + 4 * g + r;
          red[wm * 2 * BN + lc] = mean;
          red[wm * 2 * BN + BN + lc] = q;
        }
      }
    ep_barrier();
    if (wm == 0 && ci == 0) {
      const float n1 = (float)min(BM / 2, max(0, p.M - m0));
      const float n2 = (float)min(BM / 2, max(0, p.M - m0 - BM / 2));
#pragma unroll
      for (int j = 0; j < NT; ++j)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int lc = wn * (BN / 2) + j * 16 + 4 * g + r;
          const int col = n0 + lc;
          if (col >= p.N) continue;
          float mean = red[lc], m2 = red[BN + lc];
          if (n2 > 0.f) {
            const float mb = red[2 * BN + lc], d = mb - mean, nt = n1 + n2;
            mean += d * (n2 / nt);
            m2 += red[3 * BN + lc] + d * d * (n1 * n2 / nt);
          }
          reinterpret_cast<float2*>(p.stats)[(long long)col * mtiles + mtile] = make_float2(mean, m2);
        }
    }
    if (blockIdx.x == 0 && threadIdx.x == 0)  // count row: stats[N][mtile] = (rows of this tile, 0)
      reinterpret_cast<float2*>(p.stats)[(long long)p.N * mtiles + mtile] =
          make_float2((float)min(BM, p.M - m0), 0.f);
#pragma unroll
    for (int j = 0; j < NT; ++j) {
      const int n = nbase + j * 16;
#pragma unroll
      for (int i = 0; i < MT; ++i) {
        const int m = mbase + i * 16;
        if (m >= p.M || n >= p.N) continue;
        float v[4] = {acc[i][j][0], acc[i][j][1], acc[i][j][2], acc[i][j][3]};
        store4<T>(Cout + (long long)m * p.ldc + n, v);
      }
    }
  }
}

int run_fast_gemm(GemmParams& p, int amode, int epi, int z, hipStream_t s);
int fast_grid_rows(int M, int N, int z, int epi);
bool fast_bwd_streams(const GemmParams& p);  // a dense EPI_BWD GEMM runs on the streaming kernel (P product: only there)
// igemm_wide.hip: the wide-tile engine's epilogue class for a dense bf16 GEMM (-1: not supported) and its launch
int wide_gemm_class(const GemmParams& p);
int wide_gemm_class_f32(const GemmParams& p);  // the fp32-residual / fp32-output class (ACT_FLAG_F32_OUT), or -1
int run_gemm_wide(GemmParams& p, int we, hipStream_t s);
int fast_bwd_slots(const GemmParams& p);  // partial-sum slots (grid rows) of an EPI_BWD launch of run_fast_gemm
int bn_bwd_finalize_launch(const float* partial, int nb, int C, long long ld, int gx_off, float* sum_g, float* sum_gx,
                           float* dgamma, float* dbeta, int accumulate, hipStream_t s);  // grid rows (slots of EPI_BWD partials) of a fast-kernel launch
int run_fast_wgrad(const GemmParams& p, int splits, hipStream_t s, bool dense_b = false);
int wgrad_patch_rows(int dtype, int H, int W, int C, int Cin, int Cout, int KH, int KW, int stride, int pad,
                     int tsm_fold);
int wgrad_patch_splits(int C, int Cout);
// stream1x1.hip: relu(bf16(x wfold^T + bias) + res) + mask bits on the register-streaming kernel (-1: not eligible)
int run_rs1x1_bnres(const void* x, const void* wfold, const float* bias, const void* res, void* out, uint8_t* bits,
                    long long M, int N, int K, hipStream_t s);
int run_wgrad_patch(const void* x, const void* dy, float* ws, int N, int H, int W, int C, int Cout, int R,
                    hipStream_t s);
int wgrad_fast_tile_m(int M);
int wgrad_fast_tile_n(int N);

// the 256 x 256-tile engine (igemm256.hip): whether it takes a GEMM, and its launch
bool gemm256_ok(const GemmParams& p, int amode, int epi, int z);
int run_gemm256(const GemmParams& p, int amode, int epi, hipStream_t s);

}  // namespace vcg
