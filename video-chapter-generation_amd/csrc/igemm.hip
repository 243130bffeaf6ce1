// MFMA implicit-GEMM engine for gfx950.
//
// One kernel template computes  C[M][N] = sum_k A[m][k] * B[n][k]  where A and B are
// *gathered* operands:
//   OP_DENSE_K   row-major [rows][K] (k contiguous)            -> linear fwd X, W
//   OP_IM2COL    implicit im2col of an NHWC activation          -> conv fwd A (TSM shift fused)
//   OP_DGRAD     transposed-conv gather of an NHWC gradient     -> conv dgrad A
//   OP_DENSE_MN  [K][cols] (cols contiguous)                    -> wgrad dy^T, linear dW / dX
//   OP_IM2COL_T  im2col^T of an NHWC activation (k = pixel)     -> conv wgrad B (TSM fused)
// K-contiguous operands are staged in LDS as [rows][BK] and read with ds_read_b64/b128;
// MN-contiguous operands are staged as [BK][cols] and read with ds_read_b64_tr_b16 (bf16).
// Both sides use the same permutation of k inside a BK tile, so the dot product is exact.
//
// Replaces the ATen conv / addmm kernels reached from torchvision ResNet-50
// (reference video_chapter_generation/model/vision/resnet50_tsm.py:15) and HF BertModel
// (model/lang/bert_hugface.py:20) on the TwoStream hot path (model/fusion/two_stream.py:172-194).
#include <cstdio>

#include "igemm.h"

namespace vcg {

// ------------------------------------------------------------------------------------
// Tile loaders: global -> registers -> LDS
// ------------------------------------------------------------------------------------
template <typename T, int ROWS, int MODE> struct Loader {
  static constexpr int VEC = Cfg<T>::VEC, BK = Cfg<T>::BK;
  static constexpr int NC = ROWS * 4 / 256;  // 16-B chunks per thread (BK/VEC == 4)
  static constexpr bool KC = is_kcontig(MODE);
  static constexpr int CPR = ROWS / VEC;  // MN-contig: chunks per k-row

  uint4 reg[NC];
  // per-chunk state
  const T* ptr[NC];   // DENSE_K / DENSE_MN base pointer (null = invalid row/col)
  int ra[NC], rb[NC], rc[NC];  // gather coordinates
  int sub[NC];        // k offset (K-contig) or k-row (MN-contig) of the chunk inside a tile
  int lds_off[NC];

  __device__ __forceinline__ void init(const OpArgs& a, int row0, int tid) {
    const T* base = reinterpret_cast<const T*>(a.ptr);
#pragma unroll
    for (int j = 0; j < NC; ++j) {
      const int q = tid + j * 256;
      if constexpr (KC) {
        const int row = q >> 2;
        const int kc = (q & 3) * VEC;
        sub[j] = kc;
        lds_off[j] = row * Cfg<T>::LDK + kc;
        const int r = row0 + row;
        const bool valid = r < a.rows;
        if constexpr (MODE == OP_DENSE_K) {
          ptr[j] = valid ? base + (long long)r * a.ld : nullptr;
        } else {
          // decompose the row into (n, y, x) over the row grid
          const int n = r / (a.GH * a.GW);
          const int rem = r - n * a.GH * a.GW;
          const int y = rem / a.GW;
          const int x = rem - y * a.GW;
          ptr[j] = valid ? base + (long long)n * a.H * a.W * a.C : nullptr;
          if constexpr (MODE == OP_IM2COL) {
            ra[j] = y * a.stride - a.pad;
            rb[j] = x * a.stride - a.pad;
            rc[j] = a.tsm_fold > 0 ? (n % a.tsm_T) : 0;
          } else {  // DGRAD: rows are dx pixels, gathered tensor is dy [N][H][W][C]
            ra[j] = y + a.pad;
            rb[j] = x + a.pad;
            rc[j] = 0;
          }
        }
      } else {
        const int krow = q / CPR;
        const int cc = (q - krow * CPR) * VEC;
        sub[j] = krow;
        lds_off[j] = krow * LdMN<T, ROWS>::v + cc;
        const int col = row0 + cc;
        const bool valid = col < a.rows;
        if constexpr (MODE == OP_DENSE_MN) {
          ptr[j] = valid ? base + col : nullptr;
        } else {  // IM2COL_T: col = (tap, ci) over the NHWC activation
          const int tap = col >> a.logC;
          const int ci = col & (a.C - 1);
          const int kh = tap / a.KW;
          const int kw = tap - kh * a.KW;
          ptr[j] = (valid && tap < a.KH * a.KW) ? base + ci : nullptr;
          ra[j] = kh - a.pad;
          rb[j] = kw - a.pad;
          int dt = 0;
          if (a.tsm_fold > 0) dt = ci < a.tsm_fold ? 1 : (ci < 2 * a.tsm_fold ? -1 : 0);
          rc[j] = dt;
        }
      }
    }
  }

  __device__ __forceinline__ void load(const OpArgs& a, int k0, int kend) {
#pragma unroll
    for (int j = 0; j < NC; ++j) {
      const T* p = nullptr;
      if constexpr (MODE == OP_DENSE_K) {
        const int k = k0 + sub[j];
        if (ptr[j] && k < kend) p = ptr[j] + k;
      } else if constexpr (MODE == OP_IM2COL) {
        const int k = k0 + sub[j];
        const int tap = k >> a.logC;
        const int c = k & (a.C - 1);
        const int kh = tap / a.KW;
        const int kw = tap - kh * a.KW;
        const int ih = ra[j] + kh, iw = rb[j] + kw;
        if (ptr[j] && k < kend && kh < a.KH && ih >= 0 && ih < a.H && iw >= 0 && iw < a.W) {
          long long off = ((long long)(ih * a.W + iw) << a.logC) + c;
          bool ok = true;
          if (a.tsm_fold > 0) {
            const int dt = c < a.tsm_fold ? 1 : (c < 2 * a.tsm_fold ? -1 : 0);
            const int t2 = rc[j] + dt;
            ok = t2 >= 0 && t2 < a.tsm_T;
            off += (long long)dt * a.H * a.W * a.C;
          }
          if (ok) p = ptr[j] + off;
        }
      } else if constexpr (MODE == OP_DGRAD) {
        const int k = k0 + sub[j];
        const int tap = k >> a.logC;
        const int c = k & (a.C - 1);
        const int kh = tap / a.KW;
        const int kw = tap - kh * a.KW;
        int yy = ra[j] - kh, xx = rb[j] - kw;
        bool ok = ptr[j] && k < kend && kh < a.KH && yy >= 0 && xx >= 0;
        if (a.stride == 2) {
          ok = ok && ((yy | xx) & 1) == 0;
          yy >>= 1;
          xx >>= 1;
        }
        ok = ok && yy < a.H && xx < a.W;
        if (ok) p = ptr[j] + (((long long)(yy * a.W + xx)) << a.logC) + c;
      } else if constexpr (MODE == OP_DENSE_MN) {
        const int k = k0 + sub[j];
        if (ptr[j] && k < kend) p = ptr[j] + (long long)k * a.ld;
      } else {  // IM2COL_T
        const int k = k0 + sub[j];
        if (ptr[j] && k < kend) {
          const uint32_t n = fdiv((uint32_t)k, a.fd_ghw);
          const int rem = k - (int)n * a.GH * a.GW;
          const int y = (int)fdiv((uint32_t)rem, a.fd_gw);
          const int x = rem - y * a.GW;
          const int ih = y * a.stride + ra[j], iw = x * a.stride + rb[j];
          bool ok = ih >= 0 && ih < a.H && iw >= 0 && iw < a.W;
          int n2 = (int)n;
          if (rc[j] != 0) {
            const int t = (int)n - (int)fdiv(n, a.fd_T) * a.tsm_T;
            const int t2 = t + rc[j];
            ok = ok && t2 >= 0 && t2 < a.tsm_T;
            n2 += rc[j];
          }
          if (ok) p = ptr[j] + ((((long long)n2 * a.H + ih) * a.W + iw) << a.logC);
        }
      }
      reg[j] = p ? *reinterpret_cast<const uint4*>(p) : make_uint4(0, 0, 0, 0);
    }
  }

  __device__ __forceinline__ void store(T* lds) const {
#pragma unroll
    for (int j = 0; j < NC; ++j) *reinterpret_cast<uint4*>(lds + lds_off[j]) = reg[j];
  }
};

// ------------------------------------------------------------------------------------
// Fragment reads (LDS -> registers), shared by the A and B sides.
// lane = 16*g + i. bf16: element j of the 16x16x32 fragment is k = 4g + 16*(j>>2) + (j&3).
// f32: k-step s of the 16x16x4 fragment is k = 4g + s.
// ------------------------------------------------------------------------------------
template <typename T, int ROWS, bool KC> struct Frag;

template <int ROWS> struct Frag<bf16_t, ROWS, true> {
  typedef s16x8 type;
  static __device__ __forceinline__ s16x8 read(const bf16_t* lds, int r0, int lane) {
    const int g = lane >> 4, i = lane & 15;
    const bf16_t* p = lds + (r0 + i) * Cfg<bf16_t>::LDK + 4 * g;
    s16x4 lo = *reinterpret_cast<const s16x4*>(p);
    s16x4 hi = *reinterpret_cast<const s16x4*>(p + 16);
    return s16x8{lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
  }
};
template <int ROWS> struct Frag<bf16_t, ROWS, false> {
  typedef s16x8 type;
  static __device__ __forceinline__ s16x8 read(const bf16_t* lds, int r0, int lane) {
    const int g = lane >> 4, i = lane & 15;
    const int q = i >> 2, pp = i & 3;
    constexpr int LD = LdMN<bf16_t, ROWS>::v;
    typedef __attribute__((address_space(3))) s16x4 lds_s16x4;
    const bf16_t* p0 = lds + (4 * g + q) * LD + r0 + 4 * pp;
    const bf16_t* p1 = p0 + 16 * LD;
    s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(p0));
    s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(p1));
    return s16x8{lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
  }
};
template <int ROWS> struct Frag<float, ROWS, true> {
  typedef f32x4 type;
  static __device__ __forceinline__ f32x4 read(const float* lds, int r0, int lane) {
    const int g = lane >> 4, i = lane & 15;
    return *reinterpret_cast<const f32x4*>(lds + (r0 + i) * Cfg<float>::LDK + 4 * g);
  }
};
template <int ROWS> struct Frag<float, ROWS, false> {
  typedef f32x4 type;
  static __device__ __forceinline__ f32x4 read(const float* lds, int r0, int lane) {
    const int g = lane >> 4, i = lane & 15;
    constexpr int LD = LdMN<float, ROWS>::v;
    const float* p = lds + (4 * g) * LD + r0 + i;
    return f32x4{p[0], p[LD], p[2 * LD], p[3 * LD]};
  }
};

template <typename T> struct Mfma;
template <> struct Mfma<bf16_t> {
  static __device__ __forceinline__ void run(f32x4& acc, const s16x8& a, const s16x8& b) {
    acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, acc, 0, 0, 0);
  }
};
template <> struct Mfma<float> {
  static __device__ __forceinline__ void run(f32x4& acc, const f32x4& a, const f32x4& b) {
#pragma unroll
    for (int s = 0; s < 4; ++s) acc = __builtin_amdgcn_mfma_f32_16x16x4f32(a[s], b[s], acc, 0, 0, 0);
  }
};

template <typename T, int ROWS, int MODE> constexpr int tile_elems() {
  return is_kcontig(MODE) ? ROWS * Cfg<T>::LDK : Cfg<T>::BK * LdMN<T, ROWS>::v;
}
template <typename T, int BM, int BN, int AM, int BMD, int EPI> constexpr int smem_bytes() {
  constexpr int mainloop = 2 * (tile_elems<T, BM, AM>() + tile_elems<T, BN, BMD>()) * (int)sizeof(T);
  constexpr int epi = EPI == EPI_STATS ? 4 * BN * 4 : 0;  // stats reduction reuses the main-loop LDS
  return mainloop > epi ? mainloop : epi;
}

// ------------------------------------------------------------------------------------
// The kernel: 256 threads = 4 waves (2x2), wave tile (BM/2)x(BN/2) of 16x16 MFMA tiles.
// ------------------------------------------------------------------------------------
template <typename T, int BM, int BN, int AM, int BMD, int EPI>
__global__ __launch_bounds__(256) void igemm_kernel(GemmParams p) {
  constexpr int BK = Cfg<T>::BK, VEC = Cfg<T>::VEC;
  constexpr int MT = BM / 32, NT = BN / 32;
  constexpr int AE = tile_elems<T, BM, AM>(), BE = tile_elems<T, BN, BMD>();
  __shared__ __attribute__((aligned(16))) char smem[smem_bytes<T, BM, BN, AM, BMD, EPI>()];
  T* As = reinterpret_cast<T*>(smem);
  T* Bs = As + 2 * AE;

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave >> 1, wn = wave & 1;
  const int n0 = blockIdx.x * BN, m0 = blockIdx.y * BM;
  int kb = blockIdx.z * p.k_per_split;
  OpArgs oa = p.a, ob = p.b;
  T* Cout = reinterpret_cast<T*>(p.C);
  const T* Res = reinterpret_cast<const T*>(p.residual);
  if (p.batch_inner > 0) {
    const int zo = blockIdx.z / p.batch_inner, zi = blockIdx.z - zo * p.batch_inner;
    kb = 0;
    oa.ptr = reinterpret_cast<const T*>(oa.ptr) + zo * p.a_so + zi * p.a_si;
    ob.ptr = reinterpret_cast<const T*>(ob.ptr) + zo * p.b_so + zi * p.b_si;
    Cout += zo * p.c_so + zi * p.c_si;
    if (Res) Res += zo * p.c_so + zi * p.c_si;
  }
  const int ke = min(p.K, kb + p.k_per_split);

  Loader<T, BM, AM> la;
  Loader<T, BN, BMD> lb;
  la.init(oa, m0, tid);
  lb.init(ob, n0, tid);

  f32x4 acc[MT][NT];
#pragma unroll
  for (int i = 0; i < MT; ++i)
#pragma unroll
    for (int j = 0; j < NT; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int ntiles = (ke - kb + BK - 1) / BK;
  if (ntiles > 0) {
    la.load(oa, kb, ke);
    lb.load(ob, kb, ke);
    la.store(As);
    lb.store(Bs);
  }
  __syncthreads();
  for (int t = 0; t < ntiles; ++t) {
    const int cur = t & 1;
    if (t + 1 < ntiles) {
      la.load(oa, kb + (t + 1) * BK, ke);
      lb.load(ob, kb + (t + 1) * BK, ke);
    }
    const T* Ac = As + cur * AE;
    const T* Bc = Bs + cur * BE;
    typename Frag<T, BM, is_kcontig(AM)>::type af[MT];
    typename Frag<T, BN, is_kcontig(BMD)>::type bfr[NT];
#pragma unroll
    for (int i = 0; i < MT; ++i) af[i] = Frag<T, BM, is_kcontig(AM)>::read(Ac, wm * (BM / 2) + i * 16, lane);
#pragma unroll
    for (int j = 0; j < NT; ++j) bfr[j] = Frag<T, BN, is_kcontig(BMD)>::read(Bc, wn * (BN / 2) + j * 16, lane);
#pragma unroll
    for (int i = 0; i < MT; ++i)
#pragma unroll
      for (int j = 0; j < NT; ++j) Mfma<T>::run(acc[i][j], bfr[j], af[i]);  // D = C^T tile
    if (t + 1 < ntiles) {
      la.store(As + (cur ^ 1) * AE);
      lb.store(Bs + (cur ^ 1) * BE);
    }
    __syncthreads();
  }

  // acc[i][j][r] = C[m = mbase + i*16 + ci][n = nbase + j*16 + 4g + r]  (operands swapped in the
  // MFMA so each lane owns 4 consecutive output columns -> direct 8/16-byte stores, no LDS staging)
  const int g = lane >> 4, ci = lane & 15;
  const int mbase = m0 + wm * (BM / 2) + ci, nbase = n0 + wn * (BN / 2) + 4 * g;
  if constexpr (EPI == EPI_SPLITK) {
    float* ws = p.ws + (long long)blockIdx.z * p.M * p.N;
#pragma unroll
    for (int i = 0; i < MT; ++i) {
      const int m = mbase + i * 16;
      if (m >= p.M) continue;
#pragma unroll
      for (int j = 0; j < NT; ++j) {
        const int n = nbase + j * 16;
        if (n < p.N) *reinterpret_cast<f32x4*>(ws + (long long)m * p.N + n) = acc[i][j];
      }
    }
    return;
  } else {
    __syncthreads();  // main-loop LDS reads done before `red` reuses it
    float bv[BN / 32][4];
    load_bias<BN>(bv, p.bias, n0, wn, lane, p.N);
    gemm_epilogue<T, BM, BN, EPI>(acc, p, reinterpret_cast<float*>(smem), bv, Cout, Res, m0, n0, wm, wn, lane,
                                  blockIdx.y, gridDim.y);
  }
}

// ------------------------------------------------------------------------------------
// Host-side launch helpers
// ------------------------------------------------------------------------------------
static int ilog2_exact(int c) {
  int l = 0;
  while ((1 << l) < c) ++l;
  return (1 << l) == c ? l : -1;
}

// dense operand; `bytes` = extent of [rows][ld] with the last row K long (element size esz)
static OpArgs dense_op(const void* ptr, long long ld, int rows, long long K = 0, int esz = 2) {
  OpArgs a{};
  a.ptr = ptr;
  a.ld = ld;
  a.rows = rows;
  a.bytes = ((long long)(rows > 0 ? rows - 1 : 0) * ld + (K > 0 ? K : ld)) * esz;
  return a;
}

// the bf16 LDS-DMA engines (igemm_fast.hip and the kernels beside it) run every bf16 GEMM they support
static constexpr bool fast_gemm_enabled() { return true; }

template <typename T, int BM, int BN, int AM, int BMD, int EPI>
static int launch(const GemmParams& p, int splits, hipStream_t s) {
  dim3 grid((p.N + BN - 1) / BN, (p.M + BM - 1) / BM, splits);
  const int tk = timing_begin(s);
  hipLaunchKernelGGL((igemm_kernel<T, BM, BN, AM, BMD, EPI>), grid, dim3(256), 0, s, p);
  if (census_on()) { char t_[96]; snprintf(t_, sizeof(t_), "igemm %s %dx%d a%d b%d e%d z%d", sizeof(T) == 2 ? "bf16" : "f32", BM, BN, AM, BMD, EPI, splits); census_add(t_, p.M, p.N, p.K); }
  {
    // algorithmic bytes: each operand once (a gathered A as its source tensor), the output once (the split-K
    // epilogue's f32 slabs count as its output), the residual once
    const double es = (double)sizeof(T);
    const double z = p.batch_inner > 0 ? (double)splits : 1.0;
    const bool adense = AM == OP_DENSE_K || AM == OP_DENSE_MN, bdense = BMD == OP_DENSE_K || BMD == OP_DENSE_MN;
    double b = (adense ? es * p.M * (double)p.K : (double)p.a.bytes) * z +
               (bdense ? es * p.N * (double)p.K : (double)p.b.bytes) * z;
    b += (EPI == EPI_SPLITK ? 4.0 * splits : es * z) * p.M * (double)p.N;
    if (p.residual) b += es * p.M * (double)p.N * z;
    timing_end(tk, s, TIMING_GENERIC_GEMM, 2.0 * p.M * p.N * (double)p.K * z, b);
  }
  VCG_LAUNCH_CHECK();
  return VCG_OK;
}

// dispatch on BN (64 / 128) with BM = 128
template <typename T, int AM, int BMD, int EPI>
static int launch_bn(const GemmParams& p, int splits, hipStream_t s) {
  if (p.N % 128 == 0 || p.N > 64 * 3) return launch<T, 128, 128, AM, BMD, EPI>(p, splits, s);
  return launch<T, 128, 64, AM, BMD, EPI>(p, splits, s);
}

static int mtiles_of(int M) { return (M + 127) / 128; }

// VCG_GEMM_LOG=<path>: append one line per GEMM dispatch (profiling aid: matches the kernel
// trace's igemm launches in order).
static FILE* gemm_log() {
  static FILE* f = nullptr;
  static bool init = false;
  if (!init) {
    init = true;
    const char* e = getenv("VCG_GEMM_LOG");
    if (e && e[0]) f = fopen(e, "a");
  }
  return f;
}

static bool fast_gelu_enabled() {
  static int v = -1;
  if (v < 0) {
    const char* e = getenv("VCG_FAST_GELU");
    v = (e && e[0] == '0') ? 0 : 1;
  }
  return v == 1;
}

template <typename T, int AM, int BMD>
static int run_gemm(GemmParams& p, int epi, int splits, hipStream_t s) {
  p.fast_act = sizeof(T) == 2 && fast_gelu_enabled();
  if (FILE* f = gemm_log()) {
    const bool fast = sizeof(T) == 2 && is_kcontig(AM) && BMD == OP_DENSE_K && fast_gemm_enabled() &&
                      epi != EPI_SPLITK && (splits == 1 || p.batch_inner > 0) && p.K % 8 == 0 &&
                      (!p.residual || AM == OP_DENSE_K) && !(epi == EPI_STATS && p.bias) &&
                      (AM == OP_DENSE_K || (p.a.C >= 64 && p.a.KH * p.a.KW <= 32) ||
                       (AM == OP_IM2COL && p.a.tsm_fold == 0));
    fprintf(f, "a=%d b=%d epi=%d M=%d N=%d K=%d z=%d fast=%d conv=%dx%d/%d C=%d\n", AM, BMD, epi, p.M, p.N, p.K, splits,
            (int)fast, p.a.KH, p.a.KW, p.a.stride, p.a.C);
    fflush(f);
  }
  if constexpr (sizeof(T) == 2 && is_kcontig(AM) && BMD == OP_DENSE_K) {
    const bool single = splits == 1 || p.batch_inner > 0;
    if (fast_gemm_enabled() && epi != EPI_SPLITK && single && p.K % 8 == 0 && p.a.bytes < 0xFFFFFF00LL &&
        p.b.bytes < 0xFFFFFF00LL && (!p.residual || AM == OP_DENSE_K) &&
        !(epi == EPI_STATS && p.bias) &&
        (AM == OP_DENSE_K || (p.a.C >= 64 && p.a.KH * p.a.KW <= 32) || (AM == OP_IM2COL && p.a.tsm_fold == 0)))
      return run_fast_gemm(p, AM, epi, splits, s);
  }
  if (epi == EPI_STORE) return launch_bn<T, AM, BMD, EPI_STORE>(p, splits, s);
  if (epi == EPI_STATS) return launch_bn<T, AM, BMD, EPI_STATS>(p, splits, s);
  return launch_bn<T, AM, BMD, EPI_SPLITK>(p, splits, s);
}

// split-K reduction: out[m][n] (+)= sum_s ws[s][m][n], with optional conv-weight layout permutation.
// A thread owns 4 consecutive outputs (16-B loads: the slabs stream at HBM rate) and G threads share them when there
// are too few outputs to fill the chip (the weight gradients' 16 K - 2 M-element slabs x 8-512 splits): thread t of
// a group sums slabs t, t + G, ... in order, 4 loads in flight, and the G partials are combined in t order through
// LDS -- deterministic. The threads of one t read consecutive quads: every slab read is contiguous.
// (The first version, 4-B loads and G lanes of one wave per output on 8 different slabs, ran the ~120 reductions of
// a train step at ~1 TB/s: 5 ms/step.)
__device__ __forceinline__ long long splitk_dst(long long idx, int N, int conv_perm, int KH, int KW, int Cpad, int Cin,
                                                int KWp, int pwp, int pad) {
  if (conv_perm == 1) {
    // idx = m * N + n, m = cout, n = (kh*KW + kw)*Cpad + ci  ->  OIHW [cout][ci][kh][kw]  (MN < 2^31)
    const int m = (int)idx / N;
    const int n = (int)idx - m * N;
    const int tap = n / Cpad;
    const int ci = n - tap * Cpad;
    if (ci >= Cin) return -1;
    const int kh = tap / KW, kw = tap - kh * KW;
    return (((long long)m * Cin + ci) * KH + kh) * KW + kw;
  }
  if (conv_perm == 2) {
    // pair-packed stem: n = (kh*KWp + kwp)*8 + 4j + ci, tap kw = 2 (kwp - pwp) + j + pad (outside the kernel:
    // the GEMM's zero-weight half of an edge pair, dropped)
    const int m = (int)idx / N;
    const int n = (int)idx - m * N;
    const int tap = n >> 3, j = (n >> 2) & 1, ci = n & 3;
    const int kh = tap / KWp, kwp = tap - kh * KWp;
    const int kw = 2 * (kwp - pwp) + j + pad;
    if (ci >= Cin || kw < 0 || kw >= KW) return -1;
    return (((long long)m * Cin + ci) * KH + kh) * KW + kw;
  }
  return idx;
}

__global__ __launch_bounds__(256) void splitk_reduce_kernel(const float* __restrict__ ws, int splits, long long MN,
                                                            int G, int N, float* __restrict__ out, int accumulate,
                                                            int conv_perm, int KH, int KW, int Cpad, int Cin,
                                                            float scale, int KWp, int pwp, int pad) {
  __shared__ float4 red[256];
  const int QB = 256 / G;  // quads per block
  const int t = threadIdx.x / QB, ql = threadIdx.x - t * QB;
  const long long quad = (long long)blockIdx.x * QB + ql;
  const long long nq = MN >> 2;
  float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
  if (quad < nq) {
    const float4* p = reinterpret_cast<const float4*>(ws) + quad;
    int s = t;
    for (; s + 3 * G < splits; s += 4 * G) {
      float4 a[4];
#pragma unroll
      for (int k = 0; k < 4; ++k) a[k] = p[(long long)(s + k * G) * nq];
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        v.x += a[k].x; v.y += a[k].y; v.z += a[k].z; v.w += a[k].w;
      }
    }
    for (; s < splits; s += G) {
      const float4 a = p[(long long)s * nq];
      v.x += a.x; v.y += a.y; v.z += a.z; v.w += a.w;
    }
  }
  if (G > 1) {
    red[threadIdx.x] = v;
    __syncthreads();
    if (t != 0) return;
    for (int u = 1; u < G; ++u) {
      const float4 a = red[u * QB + ql];
      v.x += a.x; v.y += a.y; v.z += a.z; v.w += a.w;
    }
  }
  if (quad >= nq) return;
  const float r[4] = {v.x * scale, v.y * scale, v.z * scale, v.w * scale};
  if (conv_perm == 0) {
    float4* o = reinterpret_cast<float4*>(out) + quad;
    if (accumulate) {
      const float4 c = *o;
      *o = make_float4(c.x + r[0], c.y + r[1], c.z + r[2], c.w + r[3]);
    } else {
      *o = make_float4(r[0], r[1], r[2], r[3]);
    }
    return;
  }
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    const long long dst = splitk_dst(4 * quad + e, N, conv_perm, KH, KW, Cpad, Cin, KWp, pwp, pad);
    if (dst < 0) continue;
    if (accumulate) out[dst] += r[e];
    else out[dst] = r[e];
  }
}

// scalar fallback (MN or a pointer not 16-B aligned): one thread per output, slabs in order
__global__ __launch_bounds__(256) void splitk_reduce1_kernel(const float* __restrict__ ws, int splits, long long MN,
                                                             int N, float* __restrict__ out, int accumulate,
                                                             int conv_perm, int KH, int KW, int Cpad, int Cin,
                                                             float scale, int KWp, int pwp, int pad) {
  const long long idx = blockIdx.x * (long long)blockDim.x + threadIdx.x;
  if (idx >= MN) return;
  float v = 0.f;
  for (int s = 0; s < splits; ++s) v += ws[(long long)s * MN + idx];
  v *= scale;
  const long long dst = splitk_dst(idx, N, conv_perm, KH, KW, Cpad, Cin, KWp, pwp, pad);
  if (dst < 0) return;
  if (accumulate) out[dst] += v;
  else out[dst] = v;
}

static void splitk_reduce(hipStream_t stream, const float* ws, int splits, long long MN, int N, float* out,
                          int accumulate, int conv_perm, int KH, int KW, int Cpad, int Cin, float scale, int KWp,
                          int pwp, int pad) {
  const bool vec = (MN & 3) == 0 && (((uintptr_t)ws | (conv_perm ? 0 : (uintptr_t)out)) & 15) == 0;
  if (!vec) {
    hipLaunchKernelGGL(splitk_reduce1_kernel, dim3((unsigned)((MN + 255) / 256)), dim3(256), 0, stream, ws, splits,
                       MN, N, out, accumulate, conv_perm, KH, KW, Cpad, Cin, scale, KWp, pwp, pad);
    return;
  }
  // G: enough threads for the chip (~256 K) without more groups than slabs
  const long long nq = MN >> 2;
  int G = 1;
  while (G < 64 && G * 2 <= splits && nq * G < 262144) G *= 2;
  const int QB = 256 / G;
  hipLaunchKernelGGL(splitk_reduce_kernel, dim3((unsigned)((nq + QB - 1) / QB)), dim3(256), 0, stream, ws, splits, MN,
                     G, N, out, accumulate, conv_perm, KH, KW, Cpad, Cin, scale, KWp, pwp, pad);
}

// Split-K target: tiles x splits ~ this many workgroups (2 rounds of 2 workgroups per CU; 512 and 2048 measured
// -2.4 % / -1.3 % per step, profiles/r05_splitk_target_ab.txt). Fewer splits write and re-read fewer fp32 slabs.
#ifndef VCG_SPLITK_TARGET
#define VCG_SPLITK_TARGET 1024
#endif
static int splitk_target() { return VCG_SPLITK_TARGET; }
#ifndef VCG_SPLITK_TARGET_DENSE
#define VCG_SPLITK_TARGET_DENSE VCG_SPLITK_TARGET
#endif

static int choose_splits(int M, int N, int K, int BK, int target = splitk_target()) {
  const int tiles = ((M + 127) / 128) * ((N + 127) / 128);
  int splits = (target + tiles - 1) / tiles;
  const int max_splits = (K + 16 * BK - 1) / (16 * BK);  // at least 16 k-tiles per split
  if (splits > max_splits) splits = max_splits;
  if (splits < 1) splits = 1;
  return splits;
}

// Pair-packed stem (bf16, C = 4 RGB0 channels, stride 2): stride-2 tap kw of output column ow reads pixel
// 2 ow - pad + kw = 2 (ow + kwp - pwp) + j, i.e. half j of "super pixel" ow + kwp - pwp of the same image
// seen as [N][H][W/2][8]. The 16-B chunk of one super pixel carries two taps, so the GEMM K of a 7x7/2
// stem is 7 * 4 * 8 = 224 instead of 7 * 7 * 8 = 392 at C = 8 (the frames are also half as many bytes).
// Weights: [Cout][KH][KWp][8], element 4j + c = w[cout][c][kh][2 (kwp - pwp) + j + pad] (zero outside).
static bool stem_pair(int dtype, int C) { return dtype == VCG_BF16 && C == 4; }
static int floor_half(int x) { return (x - (x & 1)) / 2; }
static void pair_taps(int KW, int pad, int* KWp, int* pwp) {
  const int lo = floor_half(-pad), hi = floor_half(KW - 1 - pad);
  *KWp = hi - lo + 1;
  *pwp = -lo;
}

}  // namespace vcg

using namespace vcg;

// ====================================================================================
// C ABI
// ====================================================================================

VCG_API int vcg_conv_stats_tiles(int M) { return mtiles_of(M); }

// y[N*OH*OW][Cout] = conv(x[N][H][W][C], w[Cout][KH][KW][C]); optional BN partial stats.
// TSM shift (reference ops/temporal_shift.py:33-51) fused into the A gather when tsm_fold > 0.
static int conv_fwd_impl(int dtype, const void* x, const float* in_sc, const float* in_sh, const void* w, void* y,
                         float* stats, int N, int H, int W, int C, int Cout, int KH, int KW, int stride, int pad,
                         int tsm_T, int tsm_fold, hipStream_t stream, const float* bias = nullptr, int act = 0);

VCG_API int vcg_conv_fwd(int dtype, const void* x, const void* w, void* y, float* stats, int N, int H, int W,
                         int C, int Cout, int KH, int KW, int stride, int pad, int tsm_T, int tsm_fold,
                         hipStream_t stream) {
  return conv_fwd_impl(dtype, x, nullptr, nullptr, w, y, stats, N, H, W, C, Cout, KH, KW, stride, pad, tsm_T, tsm_fold,
                       stream);
}

// y = act(conv(x) + bias[col]): a conv whose running-statistics BN was folded into its weights (vcg_weight_fold),
// bias = the BN shift, act = ReLU (bn1 / bn2) or none (the downsample BN) -- the scoring forward's trunk.
VCG_API int vcg_conv_fwd_bias_act(int dtype, const void* x, const void* w, const float* bias, int act, void* y, int N,
                                  int H, int W, int C, int Cout, int KH, int KW, int stride, int pad, int tsm_T,
                                  int tsm_fold, hipStream_t stream) {
  VCG_REQUIRE(bias, "bias required");
  VCG_REQUIRE(act == ACT_NONE || act == ACT_RELU, "act must be none or ReLU");
  return conv_fwd_impl(dtype, x, nullptr, nullptr, w, y, nullptr, N, H, W, C, Cout, KH, KW, stride, pad, tsm_T,
                       tsm_fold, stream, bias, act);
}

static int conv_fwd_impl(int dtype, const void* x, const float* in_sc, const float* in_sh, const void* w, void* y,
                         float* stats, int N, int H, int W, int C, int Cout, int KH, int KW, int stride, int pad,
                         int tsm_T, int tsm_fold, hipStream_t stream, const float* bias, int act) {
  const int logC = ilog2_exact(C);
  const bool pair = stem_pair(dtype, C);
  VCG_REQUIRE(logC >= 0, "C must be a power of two");
  VCG_REQUIRE(dtype == VCG_F32 ? C >= 4 : (C >= 8 || pair), "C too small for 16-B gathers");
  VCG_REQUIRE(Cout % 64 == 0, "Cout must be a multiple of 64");
  VCG_REQUIRE(tsm_fold == 0 || (tsm_T > 0 && N % tsm_T == 0 && tsm_fold % 8 == 0 && 2 * tsm_fold <= C),
              "bad TSM geometry");
  VCG_REQUIRE(!pair || (stride == 2 && W % 2 == 0 && tsm_fold == 0 && fast_gemm_enabled() &&
                        (long long)N * H * W * C * 2 < 0xFFFFFF00LL),
              "bf16 C = 4 (pair-packed stem) needs stride 2, even W, no TSM, the fast engine and < 4 GB input");
  const int OH = (H + 2 * pad - KH) / stride + 1, OW = (W + 2 * pad - KW) / stride + 1;
  int KWp = KW, pwp = 0;
  if (pair) pair_taps(KW, pad, &KWp, &pwp);
  GemmParams p{};
  p.M = N * OH * OW;
  p.N = Cout;
  p.K = pair ? KH * KWp * 8 : KH * KW * C;
  p.k_per_split = p.K + 64;
  const bool dense = (KH == 1 && KW == 1 && stride == 1 && pad == 0 && tsm_fold == 0);
  if (dense) {
    p.a = dense_op(x, C, p.M, C, dtype == VCG_BF16 ? 2 : 4);
  } else {
    OpArgs a{};
    a.ptr = x; a.rows = p.M; a.N = N; a.H = H; a.W = W; a.C = C; a.logC = logC;
    a.GH = OH; a.GW = OW; a.KH = KH; a.KW = KW; a.stride = stride; a.pad = pad;
    a.tsm_T = tsm_T; a.tsm_fold = tsm_fold;
    a.bytes = (long long)N * H * W * C * (dtype == VCG_BF16 ? 2 : 4);
    if (pair) {  // the image as [N][H][W/2][8] super pixels, stride 1 / pad pwp along w
      a.W = W / 2; a.C = 8; a.logC = 3; a.KW = KWp; a.sw = 1; a.pw = pwp;
    }
    p.a = a;
  }
  p.b = dense_op(w, p.K, Cout, p.K, dtype == VCG_BF16 ? 2 : 4);
  p.C = y;
  p.ldc = Cout;
  p.alpha = 1.f;
  p.stats = stats;
  p.bias = bias;
  p.act = act;
  const int epi = stats ? EPI_STATS : EPI_STORE;
  if (dtype == VCG_BF16) {
    return dense ? run_gemm<bf16_t, OP_DENSE_K, OP_DENSE_K>(p, epi, 1, stream)
                 : run_gemm<bf16_t, OP_IM2COL, OP_DENSE_K>(p, epi, 1, stream);
  }
  return dense ? run_gemm<float, OP_DENSE_K, OP_DENSE_K>(p, epi, 1, stream)
               : run_gemm<float, OP_IM2COL, OP_DENSE_K>(p, epi, 1, stream);
}

// dx[N][H][W][C] = conv_transpose(dy[N][OH][OW][Cout], wt[C][KH][KW][Cout])
VCG_API int vcg_conv_dgrad(int dtype, const void* dy, const void* wt, void* dx, int N, int H, int W, int C,
                           int Cout, int KH, int KW, int stride, int pad, hipStream_t stream) {
  const int logCo = ilog2_exact(Cout);
  VCG_REQUIRE(logCo >= 0 && Cout >= 8, "Cout must be a power of two >= 8");
  VCG_REQUIRE(C % 64 == 0, "C must be a multiple of 64");
  VCG_REQUIRE(stride == 1 || stride == 2, "stride must be 1 or 2");
  const int OH = (H + 2 * pad - KH) / stride + 1, OW = (W + 2 * pad - KW) / stride + 1;
  GemmParams p{};
  p.M = N * H * W;
  p.N = C;
  p.K = KH * KW * Cout;
  p.k_per_split = p.K + 64;
  const bool dense = (KH == 1 && KW == 1 && stride == 1 && pad == 0);
  if (dense) {
    p.a = dense_op(dy, Cout, p.M, Cout, dtype == VCG_BF16 ? 2 : 4);
  } else {
    OpArgs a{};
    a.ptr = dy; a.rows = p.M; a.N = N; a.H = OH; a.W = OW; a.C = Cout; a.logC = logCo;
    a.GH = H; a.GW = W; a.KH = KH; a.KW = KW; a.stride = stride; a.pad = pad;
    a.bytes = (long long)N * OH * OW * Cout * (dtype == VCG_BF16 ? 2 : 4);
    p.a = a;
  }
  p.b = dense_op(wt, p.K, C, p.K, dtype == VCG_BF16 ? 2 : 4);
  p.C = dx;
  p.ldc = C;
  p.alpha = 1.f;
  if (dtype == VCG_BF16) {
    return dense ? run_gemm<bf16_t, OP_DENSE_K, OP_DENSE_K>(p, EPI_STORE, 1, stream)
                 : run_gemm<bf16_t, OP_DGRAD, OP_DENSE_K>(p, EPI_STORE, 1, stream);
  }
  return dense ? run_gemm<float, OP_DENSE_K, OP_DENSE_K>(p, EPI_STORE, 1, stream)
               : run_gemm<float, OP_DGRAD, OP_DENSE_K>(p, EPI_STORE, 1, stream);
}

// Workspace of vcg_conv_dgrad_bwd: partial sums [slots][3][C] floats (slots <= 768 per launch, 4 launches for
// the sub-pixel classes of a stride-2 dgrad), then the class-packed weights (KH * KW * C * Cout bf16).
static long long dgrad_bwd_part_bytes(int C) { return 4LL * 768 * 3 * C * 4; }
VCG_API long long vcg_conv_dgrad_bwd_ws_bytes(int C, int Cout, int KH, int KW) {
  return dgrad_bwd_part_bytes(C) + (long long)KH * KW * C * Cout * 2 + 256;
}

namespace {
// wt [C][KH][KW][Cout] -> the taps of one sub-pixel class, [C][tKH][tKW][Cout] (kh = kh0 + 2a, kw = kw0 + 2b)
__global__ void pack_class_taps_kernel(const bf16_t* __restrict__ wt, bf16_t* __restrict__ out, int C, int KH, int KW,
                                       int Cout, int tKH, int tKW, int kh0, int kw0) {
  const long long n = (long long)C * tKH * tKW * Cout;
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < n; i += (long long)gridDim.x * blockDim.x) {
    const int co = (int)(i % Cout);
    long long t = i / Cout;
    const int b = (int)(t % tKW);
    t /= tKW;
    const int a = (int)(t % tKH);
    const int c = (int)(t / tKH);
    out[i] = wt[(((long long)c * KH + kh0 + 2 * a) * KW + kw0 + 2 * b) * Cout + co];
  }
}
}  // namespace

// Conv input gradient of the trunk backward with the fused EPI_BWD epilogue (igemm.h BwdEpi): the dgrad value
// (moved by the TSM adjoint when tsm_fold > 0) plus `res`, masked by `bits` (VCG_MASK_BITS bytes) or by
// fma(y, mscale, mshift) > 0, is stored as g, and the BatchNorm backward reductions of g against y (and y2)
// are finalized into sum_g / sum_gx (/ sum_gx2) with dgamma / dbeta (dgamma2 / dbeta2) accumulated: the
// input of vcg_bn_bwd_apply with mask_mode 0. y == NULL: no reduction. Fast bf16 engine only:
// returns VCG_ERR_UNSUPPORTED where it does not apply (the caller then runs the unfused ops).
namespace {
// P = sum of the streaming dgrad's per-workgroup-row slabs: 32 float4 entries per workgroup, 8 slot groups (group g
// sums slots g, g + 8, ... in order), the groups combined in order through LDS (deterministic; one thread walking
// all 64 slots serially took 41 us)
__global__ __launch_bounds__(256) void p_slab_reduce_kernel(const float4* __restrict__ slabs, int nslab, long long n4,
                                                            float4* __restrict__ out) {
  __shared__ float4 part[8][32];
  const int e = threadIdx.x & 31, g = threadIdx.x >> 5;
  const long long i = (long long)blockIdx.x * 32 + e;
  float4 a = make_float4(0.f, 0.f, 0.f, 0.f);
  if (i < n4)
    for (int k = g; k < nslab; k += 8) {
      const float4 b = slabs[(long long)k * n4 + i];
      a.x += b.x; a.y += b.y; a.z += b.z; a.w += b.w;
    }
  part[g][e] = a;
  __syncthreads();
  if (g == 0 && i < n4) {
    float4 s = part[0][e];
#pragma unroll
    for (int q = 1; q < 8; ++q) {
      s.x += part[q][e].x; s.y += part[q][e].y; s.z += part[q][e].z; s.w += part[q][e].w;
    }
    out[i] = s;
  }
}
}  // namespace

// P partial slabs of vcg_conv_dgrad_bwd with a2: [slots][C][a2_c] f32, slots = the streaming kernel's workgroup rows,
// at most 256 / (C / 64) (one workgroup per CU over C / 64 column tiles; igemm_fast.hip bwd_stream_rows)
VCG_API long long vcg_conv_dgrad_bwd_p_ws_bytes(int C, int a2_c) {
  const long long nx = C >= 64 ? C / 64 : 1;
  const long long slots = 256 / nx > 0 ? 256 / nx : 1;
  return slots * (C > 0 ? C : 0) * (a2_c > 0 ? a2_c : 0) * 4;
}

VCG_API int vcg_conv_dgrad_bwd(int dtype, const void* dy, const void* wt, void* g, int N, int H, int W, int C,
                               int Cout, int KH, int KW, int stride, int pad, int tsm_T, int tsm_fold,
                               const void* res, int res_stride, const unsigned char* bits, const void* y, const float* mean,
                               const float* invstd, const float* mscale, const float* mshift, const void* y2,
                               const float* mean2, const float* invstd2, float* ws, long long ws_bytes,
                               float* sum_g, float* sum_gx, float* dgamma, float* dbeta, float* sum_gx2,
                               float* dgamma2, float* dbeta2, const void* a2, int a2_c, float* pg, float* pws,
                               long long pws_bytes, hipStream_t stream) {
  const int logCo = ilog2_exact(Cout);
  VCG_REQUIRE(logCo >= 0 && Cout >= 8, "Cout must be a power of two >= 8");
  VCG_REQUIRE(C % 64 == 0, "C must be a multiple of 64");
  VCG_REQUIRE(stride == 1 || stride == 2, "stride must be 1 or 2");
  VCG_REQUIRE(!(bits && mscale), "one ReLU mask (bits or mscale/mshift)");
  VCG_REQUIRE(!mscale || (mshift && y), "mscale needs mshift and y");
  VCG_REQUIRE(!y || (mean && invstd && sum_g && sum_gx), "the reduction needs mean/invstd/sum_g/sum_gx");
  VCG_REQUIRE(!y2 || (y && mean2 && invstd2 && sum_gx2), "the second reduction needs y, mean2/invstd2/sum_gx2");
  VCG_REQUIRE(tsm_fold == 0 || (tsm_T > 0 && N % tsm_T == 0 && tsm_fold % 8 == 0 && 2 * tsm_fold <= C),
              "bad TSM geometry");
  VCG_REQUIRE(ws_bytes >= vcg_conv_dgrad_bwd_ws_bytes(C, Cout, KH, KW), "workspace too small");
  VCG_REQUIRE(res_stride == 1 || (res_stride == 2 && res), "res_stride must be 1, or 2 with a residual");
  VCG_REQUIRE(!a2 || (pg && pws && a2_c > 0 && a2_c % 64 == 0 && pws_bytes >= vcg_conv_dgrad_bwd_p_ws_bytes(C, a2_c)),
              "a2 needs a2_c a multiple of 64, pg and the P workspace");
  const long long nelem = (long long)N * H * W * C;
  const int OH = (H + 2 * pad - KH) / stride + 1, OW = (W + 2 * pad - KW) / stride + 1;
  if (dtype != VCG_BF16 || !fast_gemm_enabled() || nelem * 2 >= 0xFFFFFF00LL ||
      (long long)N * OH * OW * Cout * 2 >= 0xFFFFFF00LL || (long long)N * H * W >= (1LL << 31))
    return VCG_ERR_UNSUPPORTED;
  const bool dense = (KH == 1 && KW == 1 && stride == 1 && pad == 0);
  if (!dense && (Cout < 64 || KH * KW > 32)) return VCG_ERR_UNSUPPORTED;  // fast dgrad gather: one tap per k tile
  // stride-2 3x3: four sub-pixel classes (dx pixels of one (h, w) parity), each a GEMM over only the taps that
  // reach it (4 / 2 / 2 / 1 of 9) instead of one GEMM over all 9 with 3/4 of the tap rows masked to zero
  const bool subpix = stride == 2 && KH == 3 && KW == 3 && pad == 1 && tsm_fold == 0 && res_stride == 1 &&
                      H % 2 == 0 && W % 2 == 0;
  GemmParams p{};
  p.M = N * H * W;
  p.N = C;
  p.K = KH * KW * Cout;
  p.k_per_split = p.K + 64;
  if (dense) {
    p.a = dense_op(dy, Cout, p.M, Cout, 2);
  } else {
    OpArgs a{};
    a.ptr = dy; a.rows = p.M; a.N = N; a.H = OH; a.W = OW; a.C = Cout; a.logC = logCo;
    a.GH = H; a.GW = W; a.KH = KH; a.KW = KW; a.stride = stride; a.pad = pad;
    a.bytes = (long long)N * OH * OW * Cout * 2;
    p.a = a;
  }
  p.b = dense_op(wt, p.K, C, p.K, 2);
  p.C = g;
  p.ldc = C;
  p.alpha = 1.f;
  BwdEpi& e = p.bwd;
  e.tsm_T = tsm_fold > 0 ? tsm_T : 0;
  e.tsm_fold = tsm_fold;
  e.hw = H * W;
  e.fd_hw = make_fastdiv((uint32_t)(H * W));
  e.fd_T = make_fastdiv((uint32_t)(tsm_T > 0 ? tsm_T : 1));
  e.res = res; e.bits = bits;
  e.res_s = res_stride;
  e.rH = (H + 1) / 2; e.rW = (W + 1) / 2;
  e.fd_w = make_fastdiv((uint32_t)W); e.y = y; e.mean = mean; e.invstd = invstd; e.msc = mscale; e.msh = mshift;
  e.y2 = y2; e.mean2 = mean2; e.invstd2 = invstd2;
  e.part = ws;
  // (bits without y: the sums row of g only -- sum_gx comes from elsewhere, the previous block's y3 not stored)
  e.nred = y ? (y2 ? 3 : 2) : ((bits && sum_g && sum_gx) ? 2 : 0);
  if (a2) {  // P = g^T a2 from the stored g tiles: the streaming kernel only (else the caller runs the GEMM)
    e.a2 = a2; e.pj = a2_c; e.ppart = pws;
    if (!dense || !fast_bwd_streams(p)) return VCG_ERR_UNSUPPORTED;
    VCG_REQUIRE((long long)fast_bwd_slots(p) * C * a2_c * 4 <= pws_bytes, "P workspace smaller than the launch's slots");
  }
  if (subpix) {
    bf16_t* wpk = reinterpret_cast<bf16_t*>(reinterpret_cast<char*>(ws) + dgrad_bwd_part_bytes(C));
    const int cH = H / 2, cW = W / 2;
    int slots = 0;
    for (int ry = 0; ry < 2; ++ry)
      for (int rx = 0; rx < 2; ++rx) {
        // dx row 2i + ry sits at py = 2i + ry + pad; the taps that reach it have kh = py (mod 2)
        const int kh0 = (ry + pad) & 1, kw0 = (rx + pad) & 1;
        const int tKH = (KH - kh0 + 1) / 2, tKW = (KW - kw0 + 1) / 2;
        GemmParams q = p;
        q.M = N * cH * cW;
        q.K = tKH * tKW * Cout;
        q.k_per_split = q.K + 64;
        q.a.rows = q.M;
        q.a.GH = cH; q.a.GW = cW;
        q.a.tKH = tKH; q.a.tKW = tKW; q.a.tkh0 = kh0; q.a.tkw0 = kw0; q.a.ry = ry; q.a.rx = rx;
        bf16_t* wc = wpk;  // reused by each class: its pack runs after the previous class's GEMM (stream order)
        hipLaunchKernelGGL(pack_class_taps_kernel, dim3(256), dim3(256), 0, stream, (const bf16_t*)wt, wc, C, KH, KW,
                           Cout, tKH, tKW, kh0, kw0);
        VCG_LAUNCH_CHECK();
        q.b = dense_op(wc, q.K, C, q.K, 2);
        BwdEpi& qe = q.bwd;
        qe.sub = 1; qe.cW = cW; qe.ry = ry; qe.rx = rx; qe.fH = H; qe.fW = W;
        qe.fd_chw = make_fastdiv((uint32_t)(cH * cW));
        qe.fd_cw = make_fastdiv((uint32_t)cW);
        qe.part = ws + (long long)slots * (e.nred > 0 ? e.nred : 1) * C;
        if (FILE* f = gemm_log()) {
          fprintf(f, "a=2 b=0 epi=3 M=%d N=%d K=%d z=1 fast=1 conv=%dx%d/%d C=%d\n", q.M, q.N, q.K, KH, KW, stride,
                  Cout);
          fflush(f);
        }
        int rc = run_fast_gemm(q, OP_DGRAD, EPI_BWD, 1, stream);
        if (rc) return rc;
        slots += fast_bwd_slots(q);
      }
    if (e.nred > 0) {
      int rc = bn_bwd_finalize_launch(ws, slots, C, (long long)e.nred * C, C, sum_g, sum_gx, dgamma, dbeta, 1, stream);
      if (rc) return rc;
      if (e.nred > 2) {
        rc = bn_bwd_finalize_launch(ws, slots, C, 3LL * C, 2 * C, sum_g, sum_gx2, dgamma2, dbeta2, 1, stream);
        if (rc) return rc;
      }
    }
    return VCG_OK;
  }
  if (FILE* f = gemm_log()) {
    fprintf(f, "a=%d b=0 epi=3 M=%d N=%d K=%d z=1 fast=1 conv=%dx%d/%d C=%d\n", dense ? 0 : 2, p.M, p.N, p.K, KH, KW,
            stride, Cout);
    fflush(f);
  }
  int rc = run_fast_gemm(p, dense ? OP_DENSE_K : OP_DGRAD, EPI_BWD, 1, stream);
  if (rc) return rc;
  if (a2) {  // the P slabs [slots][C][a2_c] in slot order
    const long long n = (long long)C * a2_c;
    hipLaunchKernelGGL(p_slab_reduce_kernel, dim3((unsigned)((n / 4 + 31) / 32)), dim3(256), 0, stream,
                       (const float4*)pws, fast_bwd_slots(p), n / 4, (float4*)pg);
    VCG_LAUNCH_CHECK();
  }
  if (e.nred > 0) {
    const int slots = fast_bwd_slots(p);
    rc = bn_bwd_finalize_launch(ws, slots, C, (long long)e.nred * C, C, sum_g, sum_gx, dgamma, dbeta, 1, stream);
    if (rc) return rc;
    if (e.nred > 2) {
      rc = bn_bwd_finalize_launch(ws, slots, C, 3LL * C, 2 * C, sum_g, sum_gx2, dgamma2, dbeta2, 1, stream);
      if (rc) return rc;
    }
  }
  return VCG_OK;
}

// The bf16 LDS-DMA wgrad kernel (igemm_wgrad.hip) takes x / dy below 4 GB (32-bit buffer range)
// and C >= 8 (a 16-B chunk of x never straddles two filter taps).
static bool wgrad_fast_ok(int dtype, int N, int H, int W, int C, int Cout, int K) {
  return dtype == VCG_BF16 && fast_gemm_enabled() && C >= 8 && (long long)N * H * W * C * 2 < 0xFFFFFF00LL &&
         (long long)K * Cout * 2 < 0xFFFFFF00LL;
}

static void wgrad_geometry(int dtype, int N, int H, int W, int C, int Cout, int KH, int KW, int stride, int pad,
                           int* M, int* Nn, int* K, int* splits, int* kps, bool* fast) {
  const int OH = (H + 2 * pad - KH) / stride + 1, OW = (W + 2 * pad - KW) / stride + 1;
  const bool pair = stem_pair(dtype, C);  // gathered as [N][H][W/2][8] super pixels (see pair_taps)
  int KWp = KW, pwp = 0;
  if (pair) pair_taps(KW, pad, &KWp, &pwp);
  *M = Cout;
  *Nn = pair ? KH * KWp * 8 : KH * KW * C;
  *K = N * OH * OW;
  *fast = wgrad_fast_ok(dtype, N, H, pair ? W / 2 : W, pair ? 8 : C, Cout, *K);
  int BK, sp;
  if (*fast) {
    BK = 64;
    const int tiles = ((*Nn + wgrad_fast_tile_n(*Nn) - 1) / wgrad_fast_tile_n(*Nn)) *
                      ((*M + wgrad_fast_tile_m(*M) - 1) / wgrad_fast_tile_m(*M));
    sp = (splitk_target() + tiles - 1) / tiles;
    const int max_sp = (*K + 8 * BK - 1) / (8 * BK);  // at least 8 k-steps (512 pixels) per split
    sp = sp > max_sp ? max_sp : sp;
    sp = sp < 1 ? 1 : sp;
  } else {
    BK = dtype == VCG_BF16 ? 32 : 16;
    sp = choose_splits(*M, *Nn, *K, BK);
  }
  int k = (*K + sp - 1) / sp;
  k = (k + BK - 1) / BK * BK;
  *kps = k;
  *splits = (*K + k - 1) / k;
}

VCG_API long long vcg_conv_wgrad_ws_bytes(int dtype, int N, int H, int W, int C, int Cout, int KH, int KW,
                                          int stride, int pad) {
  int M, Nn, K, splits, kps;
  bool fast;
  wgrad_geometry(dtype, N, H, W, C, Cout, KH, KW, stride, pad, &M, &Nn, &K, &splits, &kps, &fast);
  if (wgrad_patch_rows(dtype, H, W, C, C, Cout, KH, KW, stride, pad, 0) > 0 && splits < wgrad_patch_splits(C, Cout))
    splits = wgrad_patch_splits(C, Cout);  // the patch kernel's slabs
  return (long long)splits * M * Nn * 4;
}

// dw (fp32, OIHW [Cout][Cin][KH][KW]) (+)= sum_pixels dy (x) im2col(x). C = padded channels of x.
static int conv_wgrad_impl(int dtype, const void* x, const float* in_sc, const float* in_sh, const void* dy,
                           float* dw, int accumulate, float* ws, long long ws_bytes, int N, int H, int W, int C, int Cin,
                           int Cout, int KH, int KW, int stride, int pad, int tsm_T, int tsm_fold, hipStream_t stream);

VCG_API int vcg_conv_wgrad(int dtype, const void* x, const void* dy, float* dw, int accumulate, float* ws,
                           long long ws_bytes, int N, int H, int W, int C, int Cin, int Cout, int KH, int KW,
                           int stride, int pad, int tsm_T, int tsm_fold, hipStream_t stream) {
  return conv_wgrad_impl(dtype, x, nullptr, nullptr, dy, dw, accumulate, ws, ws_bytes, N, H, W, C, Cin, Cout, KH, KW,
                         stride, pad, tsm_T, tsm_fold, stream);
}

static int conv_wgrad_impl(int dtype, const void* x, const float* in_sc, const float* in_sh, const void* dy,
                           float* dw, int accumulate, float* ws, long long ws_bytes, int N, int H, int W, int C, int Cin,
                           int Cout, int KH, int KW, int stride, int pad, int tsm_T, int tsm_fold, hipStream_t stream) {
  const int logC = ilog2_exact(C);
  VCG_REQUIRE(logC >= 0, "C must be a power of two");
  VCG_REQUIRE(Cout % 64 == 0, "Cout must be a multiple of 64");
  int M, Nn, K, splits, kps;
  bool fast;
  wgrad_geometry(dtype, N, H, W, C, Cout, KH, KW, stride, pad, &M, &Nn, &K, &splits, &kps, &fast);
  const bool pair = stem_pair(dtype, C);
  int KWp = KW, pwp = 0;
  if (pair) pair_taps(KW, pad, &KWp, &pwp);
  VCG_REQUIRE(!pair || (fast && stride == 2 && W % 2 == 0 && tsm_fold == 0),
              "bf16 C = 4 (pair-packed stem) needs stride 2, even W, no TSM and the fast engine");
  VCG_REQUIRE(ws_bytes >= (long long)splits * M * Nn * 4, "workspace too small");
  const int OH = (H + 2 * pad - KH) / stride + 1, OW = (W + 2 * pad - KW) / stride + 1;
  GemmParams p{};
  p.M = M;
  p.N = Nn;
  p.K = K;
  p.k_per_split = kps;
  p.a = dense_op(dy, Cout, Cout);  // A[m=cout][k=pixel] = dy[pixel][cout]
  p.a.bytes = (long long)K * Cout * (dtype == VCG_BF16 ? 2 : 4);
  OpArgs b{};
  b.ptr = x; b.rows = Nn; b.N = N; b.H = H; b.W = W; b.C = C; b.logC = logC;
  b.bytes = (long long)N * H * W * C * (dtype == VCG_BF16 ? 2 : 4);
  b.GH = OH; b.GW = OW; b.KH = KH; b.KW = KW; b.stride = stride; b.pad = pad;
  b.tsm_T = tsm_T > 0 ? tsm_T : 1; b.tsm_fold = tsm_fold;
  b.fd_ghw = make_fastdiv(OH * OW); b.fd_gw = make_fastdiv(OW); b.fd_T = make_fastdiv(b.tsm_T);
  if (pair) {
    b.W = W / 2; b.C = 8; b.logC = 3; b.KW = KWp; b.sw = 1; b.pw = pwp;
  }
  p.b = b;
  p.ws = ws;
  p.alpha = 1.f;
  const int wpr = wgrad_patch_rows(dtype, H, W, C, Cin, Cout, KH, KW, stride, pad, tsm_fold);
  if (wpr > 0) {  // stride-1 3x3: im2col-free patch kernel (igemm_wgrad.hip), one slab per tile range
    const int wsp = wgrad_patch_splits(C, Cout);
    VCG_REQUIRE(ws_bytes >= (long long)wsp * M * Nn * 4, "workspace too small");
    if (FILE* f = gemm_log())
      fprintf(f, "a=3 b=4 epi=2 M=%d N=%d K=%d z=%d fast=3 conv=%dx%d/%d C=%d\n", M, Nn, K, wsp, KH, KW, stride, C);
    int rc = run_wgrad_patch(x, dy, ws, N, H, W, C, Cout, wpr, stream);
    if (rc) return rc;
    const long long MN = (long long)M * Nn;
    splitk_reduce(stream, ws, wsp, MN,
                       Nn, dw, accumulate, 1, KH, KW, C, Cin, 1.f, KW, 0, pad);
    VCG_LAUNCH_CHECK();
    return VCG_OK;
  }
  FILE* f = fast ? gemm_log() : nullptr;  // the generic path logs in run_gemm
  if (f)
    fprintf(f, "a=3 b=4 epi=2 M=%d N=%d K=%d z=%d fast=2 conv=%dx%d/%d C=%d\n", M, Nn, K, splits, KH, KW, stride, C);
  int rc;
  if (fast)
    rc = run_fast_wgrad(p, splits, stream);
  else
    rc = dtype == VCG_BF16 ? run_gemm<bf16_t, OP_DENSE_MN, OP_IM2COL_T>(p, EPI_SPLITK, splits, stream)
                           : run_gemm<float, OP_DENSE_MN, OP_IM2COL_T>(p, EPI_SPLITK, splits, stream);
  if (rc) return rc;
  const long long MN = (long long)M * Nn;
  splitk_reduce(stream, ws, splits,
                     MN, Nn, dw, accumulate, pair ? 2 : 1, KH, KW, C, Cin, 1.f, KWp, pwp, pad);
  VCG_LAUNCH_CHECK();
  return VCG_OK;
}

// ---- BatchNorm backward folded into the consuming 1x1 conv's gradients (batch statistics) --------------------
// The trunk backward's bn3 step dy = A g + B y + Cc (bn_bwd_apply_kernel's per-channel affine map of the masked
// gradient g and the BN input y: A = gamma invstd, B = -A invstd sum_gx / M, Cc = -A sum_g / M - B mean) feeds
// only conv3's input gradient and weight gradient, both linear in dy:
//   dgrad: dx[m][n] = sum_k dy[m][k] w[k][n] = sum_k g[m][k] (A_k w) + sum_k y[m][k] (B_k w) + sum_k Cc_k w
//          -> ONE GEMM over [g | y] (K = 2 Cout) against wfold = [bf16(A w) | bf16(B w)] plus a column bias;
//   wgrad: dW[k][n] = A_k (g^T x)[k][n] + B_k (y^T x)[k][n] + Cc_k colsum(x)[n]
//          -> ONE GEMM with 2 Cout output rows ([g | y]^T x), combined per row by the split-K reduction.
// dy is never stored: the bn_bwd_apply pass (read g, y; write dy) and the two GEMMs' read of dy become two reads
// of [g | y]. The bias keeps the y term's cancellation exact: bias[n] = sum_k (-A_k sum_g_k / M) w[k][n] -
// mean_k bf16(B_k w[k][n]), so GEMM + bias = sum g wg + sum (y - mean) wy - sum A gbar w (no |mean| / std loss).
namespace {
__global__ __launch_bounds__(256) void bn_fold_weights_kernel(const bf16_t* __restrict__ wt, int K,
                                                              const float* __restrict__ mean,
                                                              const float* __restrict__ invstd,
                                                              const float* __restrict__ gamma,
                                                              const float* __restrict__ sum_g,
                                                              const float* __restrict__ sum_gx, float ic,
                                                              bf16_t* __restrict__ wf, float* __restrict__ bias) {
  __shared__ float red[256];
  const int n = blockIdx.x, t = threadIdx.x;
  float acc = 0.f;
  for (int k = t; k < K; k += 256) {
    const float is = invstd[k], A = (gamma ? gamma[k] : 1.f) * is;
    const float B = -A * is * sum_gx[k] * ic;
    const float w = bf2f(wt[(long long)n * K + k]);
    const bf16_t wy = f2bf(B * w);
    wf[(long long)n * 2 * K + k] = f2bf(A * w);
    wf[(long long)n * 2 * K + K + k] = wy;
    acc += (-A * sum_g[k] * ic) * w - mean[k] * bf2f(wy);
  }
  red[t] = acc;
  __syncthreads();
  for (int o = 128; o > 0; o >>= 1) {  // fixed tree: deterministic
    if (t < o) red[t] += red[t + o];
    __syncthreads();
  }
  if (t == 0) bias[n] = red[0];
}

// dw[k][n] (+)= A_k S[k][n] + B_k S[Cout + k][n] + Cc_k cs[n], S = sum of the split slabs [split][2 Cout][N]
// (G threads per output, fixed-order combine as splitk_reduce_kernel)
template <int G>
__global__ __launch_bounds__(256) void splitk_reduce_bnfold_kernel(const float* __restrict__ ws, int splits, int Cout,
                                                                   int N, const float* __restrict__ mean,
                                                                   const float* __restrict__ invstd,
                                                                   const float* __restrict__ gamma,
                                                                   const float* __restrict__ sum_g,
                                                                   const float* __restrict__ sum_gx, float ic,
                                                                   const float* __restrict__ cs, float* __restrict__ out,
                                                                   int accumulate) {
  const long long MN = (long long)Cout * N, slab = 2 * MN;
  const long long gid = blockIdx.x * (long long)blockDim.x + threadIdx.x;
  const long long idx = gid / G;
  const int t = (int)(gid - idx * G);
  if (idx >= MN) return;
  float v1 = 0.f, v2 = 0.f;
  const float* p = ws + idx;
  for (int s = t; s < splits; s += G) {
    v1 += p[(long long)s * slab];
    v2 += p[(long long)s * slab + MN];
  }
#pragma unroll
  for (int o = G / 2; o > 0; o >>= 1) {
    v1 += __shfl_xor(v1, o, 64);
    v2 += __shfl_xor(v2, o, 64);
  }
  if (t != 0) return;
  const int k = (int)(idx / N), n = (int)(idx - (long long)k * N);
  const float is = invstd[k], A = (gamma ? gamma[k] : 1.f) * is;
  const float B = -A * is * sum_gx[k] * ic;
  const float Cc = -A * sum_g[k] * ic - B * mean[k];
  const float v = fmaf(A, v1, fmaf(B, v2, Cc * cs[n]));
  if (accumulate) out[idx] += v;
  else out[idx] = v;
}
}  // namespace

VCG_API int vcg_bn_bwd_fold_weights(const void* wt, int N, int K, const float* mean, const float* invstd,
                                    const float* gamma, const float* sum_g, const float* sum_gx, float inv_count,
                                    void* wfold, float* bias, hipStream_t stream) {
  VCG_REQUIRE(wt && wfold && bias && mean && invstd && sum_g && sum_gx, "null argument");
  VCG_REQUIRE(N > 0 && K > 0, "empty weight");
  hipLaunchKernelGGL(bn_fold_weights_kernel, dim3(N), dim3(256), 0, stream, (const bf16_t*)wt, K, mean, invstd, gamma,
                     sum_g, sum_gx, inv_count, (bf16_t*)wfold, bias);
  VCG_LAUNCH_CHECK();
  return VCG_OK;
}

// The same fold with the conv3 INPUT a2 in place of y3 (y3 = a2 w3^T, so y3 never needs reading): the B y3 term of the
// input gradient is a2 Q with Q = w3^T diag(B) w3 ([C][C], symmetric), the weight gradient's y3^T a2 is w3 G with
// G = a2^T a2. wfold [C][K + C] = [A_k wt | bf16(Q)], bias[n] = sum_k (-A_k sum_g_k / M) wt[n][k] - sum_j abar_j
// bf16(Q[j][n]) with abar = colsum(a2) / M: GEMM + bias = sum g (A w) + sum_j (a2 - abar)_j Q - sum A gbar w, centred
// like the y3 form (B (y3 - mean) with mean = abar w3^T).
namespace {
// FW_NB output columns n per workgroup: the A_k wt[n][k] rows and the bias partials, then thread j streams row j of
// wt once (16-B loads) for all FW_NB columns of Q; every sum keeps the sequential k order and the bias its fixed tree
// (the values of one column per workgroup, with half the row reads)
constexpr int FW_NB = 2;
__global__ __launch_bounds__(256) void bn_fold_weights_a2_kernel(const bf16_t* __restrict__ wt, int C, int K,
                                                                 const float* __restrict__ invstd,
                                                                 const float* __restrict__ gamma,
                                                                 const float* __restrict__ sum_g,
                                                                 const float* __restrict__ sum_gx, float ic,
                                                                 const float* __restrict__ colsum_a,
                                                                 bf16_t* __restrict__ wf, float* __restrict__ bias) {
  __shared__ float bw[FW_NB][2048];  // B_k wt[n][k]
  __shared__ float red[FW_NB][256];
  const int n0 = blockIdx.x * FW_NB, t = threadIdx.x;
  float acc[FW_NB];
#pragma unroll
  for (int q = 0; q < FW_NB; ++q) acc[q] = 0.f;
  for (int k = t; k < K; k += 256) {
    const float is = invstd[k], A = (gamma ? gamma[k] : 1.f) * is;
    const float B = -A * is * sum_gx[k] * ic;
#pragma unroll
    for (int q = 0; q < FW_NB; ++q) {
      const int n = n0 + q;
      if (n < C) {
        const float w = bf2f(wt[(long long)n * K + k]);
        bw[q][k] = B * w;
        wf[(long long)n * (K + C) + k] = f2bf(A * w);
        acc[q] += (-A * sum_g[k] * ic) * w;
      }
    }
  }
  __syncthreads();
  for (int j = t; j < C; j += 256) {  // Q[j][n] = sum_k wt[j][k] B_k wt[n][k]
    const bf16_t* row = wt + (long long)j * K;
    float qv[FW_NB];
#pragma unroll
    for (int q = 0; q < FW_NB; ++q) qv[q] = 0.f;
    for (int k0 = 0; k0 < K; k0 += 64) {  // (K % 64 == 0: 8 row loads in flight per batch)
      uint4 u8[8];
#pragma unroll
      for (int b = 0; b < 8; ++b) u8[b] = *reinterpret_cast<const uint4*>(row + k0 + 8 * b);
#pragma unroll
      for (int b = 0; b < 8; ++b) {
        const uint32_t w4[4] = {u8[b].x, u8[b].y, u8[b].z, u8[b].w};
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          const float w = __uint_as_float((e & 1) ? (w4[e >> 1] & 0xffff0000u) : (w4[e >> 1] << 16));
#pragma unroll
          for (int q = 0; q < FW_NB; ++q) qv[q] = fmaf(w, bw[q][k0 + 8 * b + e], qv[q]);
        }
      }
    }
#pragma unroll
    for (int q = 0; q < FW_NB; ++q) {
      const int n = n0 + q;
      if (n < C) {
        const bf16_t qb = f2bf(qv[q]);
        wf[(long long)n * (K + C) + K + j] = qb;
        acc[q] -= colsum_a[j] * ic * bf2f(qb);
      }
    }
  }
#pragma unroll
  for (int q = 0; q < FW_NB; ++q) red[q][t] = acc[q];
  __syncthreads();
  for (int o = 128; o > 0; o >>= 1) {
    if (t < o) {
#pragma unroll
      for (int q = 0; q < FW_NB; ++q) red[q][t] += red[q][t + o];
    }
    __syncthreads();
  }
  if (t < FW_NB && n0 + t < C) bias[n0 + t] = red[t][0];
}

// dw[k][j] (+)= A_k P[k][j] + B_k (w3 G)[k][j] + Cc_k cs[j]: P = g^T a2 [K][C], G = a2^T a2 [C][C], w3 [K][C] f32
__global__ __launch_bounds__(256) void bn_fold_wgrad_a2_kernel(const float* __restrict__ P, const float* __restrict__ G,
                                                               const float* __restrict__ w3, int K, int C,
                                                               const float* __restrict__ mean,
                                                               const float* __restrict__ invstd,
                                                               const float* __restrict__ gamma,
                                                               const float* __restrict__ sum_g,
                                                               const float* __restrict__ sum_gx, float ic,
                                                               const float* __restrict__ cs, float* __restrict__ dw,
                                                               int accumulate) {
  __shared__ float wr[512];
  const int k = blockIdx.x;
  for (int i = threadIdx.x; i < C; i += 256) wr[i] = w3[(long long)k * C + i];
  __syncthreads();
  const float is = invstd[k], A = (gamma ? gamma[k] : 1.f) * is;
  const float B = -A * is * sum_gx[k] * ic;
  const float Cc = -A * sum_g[k] * ic - B * mean[k];
  for (int j = threadIdx.x; j < C; j += 256) {
    float wg = 0.f;
    for (int i0 = 0; i0 < C; i0 += 16) {  // (C % 16 == 0: 16 row loads in flight per batch)
      float gv[16];
#pragma unroll
      for (int u = 0; u < 16; ++u) gv[u] = G[(long long)(i0 + u) * C + j];
#pragma unroll
      for (int u = 0; u < 16; ++u) wg = fmaf(wr[i0 + u], gv[u], wg);
    }
    const float v = fmaf(A, P[(long long)k * C + j], fmaf(B, wg, Cc * cs[j]));
    float* o = dw + (long long)k * C + j;
    *o = accumulate ? *o + v : v;
  }
}
}  // namespace

namespace {
__global__ __launch_bounds__(64) void bn_sumgx_kernel(const float* __restrict__ P, const bf16_t* __restrict__ w, int C,
                                                      const float* __restrict__ mean, const float* __restrict__ invstd,
                                                      const float* __restrict__ sum_g, float* __restrict__ sum_gx,
                                                      float* __restrict__ dgamma) {
  const int k = blockIdx.x, t = threadIdx.x;
  float a = 0.f;
  for (int j = t; j < C; j += 64) a = fmaf(bf2f(w[(long long)k * C + j]), P[(long long)k * C + j], a);
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) a += __shfl_xor(a, o, 64);
  if (t == 0) {
    const float v = invstd[k] * (a - mean[k] * sum_g[k]);
    sum_gx[k] = v;
    if (dgamma) dgamma[k] += v;
  }
}
}  // namespace

// sum_gx[k] = invstd_k (sum_m g[m][k] y3[m][k] - mean_k sum_g[k]) of a BN whose input y3 = a2 w^T was never stored:
// sum_m g y3 = sum_j w[k][j] P[k][j] with P = g^T a2 (f32 [K][C], a weight-gradient GEMM) and w the conv's bf16 forward
// weight [K][C]; dgamma (optional) += sum_gx (as vcg_bn_bwd_finalize would have added)
VCG_API int vcg_bn_bwd_sumgx_from_wgrad(const float* P, const void* w, int K, int C, const float* mean,
                                        const float* invstd, const float* sum_g, float* sum_gx, float* dgamma,
                                        hipStream_t stream) {
  VCG_REQUIRE(P && w && mean && invstd && sum_g && sum_gx, "null argument");
  VCG_REQUIRE(K > 0 && C > 0, "empty");
  hipLaunchKernelGGL(bn_sumgx_kernel, dim3(K), dim3(64), 0, stream, P, (const bf16_t*)w, C, mean, invstd, sum_g,
                     sum_gx, dgamma);
  VCG_LAUNCH_CHECK();
  return VCG_OK;
}

VCG_API int vcg_bn_bwd_fold_weights_a2(const void* wt, int C, int K, const float* invstd, const float* gamma,
                                       const float* sum_g, const float* sum_gx, float inv_count, const float* colsum_a,
                                       void* wfold, float* bias, hipStream_t stream) {
  VCG_REQUIRE(wt && wfold && bias && invstd && sum_g && sum_gx && colsum_a, "null argument");
  VCG_REQUIRE(C > 0 && K > 0 && K <= 2048 && K % 64 == 0, "K must be a multiple of 64, <= 2048");
  VCG_REQUIRE(((uintptr_t)wt & 15) == 0, "wt must be 16-B aligned");
  hipLaunchKernelGGL(bn_fold_weights_a2_kernel, dim3((C + FW_NB - 1) / FW_NB), dim3(256), 0, stream, (const bf16_t*)wt, C, K, invstd, gamma,
                     sum_g, sum_gx, inv_count, colsum_a, (bf16_t*)wfold, bias);
  VCG_LAUNCH_CHECK();
  return VCG_OK;
}

VCG_API int vcg_bn_bwd_fold_wgrad_a2(const float* P, const float* G, const float* w3, int K, int C, const float* mean,
                                     const float* invstd, const float* gamma, const float* sum_g, const float* sum_gx,
                                     float inv_count, const float* colsum_a, float* dw, int accumulate,
                                     hipStream_t stream) {
  VCG_REQUIRE(P && G && w3 && mean && invstd && sum_g && sum_gx && colsum_a && dw, "null argument");
  VCG_REQUIRE(C > 0 && C <= 512 && C % 16 == 0 && K > 0, "C must be a multiple of 16, <= 512");
  hipLaunchKernelGGL(bn_fold_wgrad_a2_kernel, dim3(K), dim3(256), 0, stream, P, G, w3, K, C, mean, invstd, gamma,
                     sum_g, sum_gx, inv_count, colsum_a, dw, accumulate);
  VCG_LAUNCH_CHECK();
  return VCG_OK;
}

VCG_API int vcg_conv_dgrad_bwd_bnfold(const void* g, const void* yg, int Ky, const void* wfold, const float* bias,
                                      void* out, int N, int H, int W, int C, int Cout, const void* y, const float* mean,
                                      const float* invstd, const float* mscale, const float* mshift, float* ws,
                                      long long ws_bytes, float* sum_g, float* sum_gx, float* dgamma, float* dbeta,
                                      hipStream_t stream) {
  VCG_REQUIRE(g && yg && wfold && bias && out, "null argument");
  VCG_REQUIRE(C % 64 == 0 && Cout % 64 == 0 && Ky % 64 == 0, "C, Cout and Ky must be multiples of 64");
  VCG_REQUIRE(!mscale || (mshift && y), "mscale needs mshift and y");
  VCG_REQUIRE(!y || (mean && invstd && sum_g && sum_gx), "the reduction needs mean/invstd/sum_g/sum_gx");
  VCG_REQUIRE(ws_bytes >= vcg_conv_dgrad_bwd_ws_bytes(C, Cout + Ky, 1, 1), "workspace too small");
  const long long M = (long long)N * H * W;
  if (!fast_gemm_enabled() || M * C * 2 >= 0xFFFFFF00LL || M * Cout * 2 >= 0xFFFFFF00LL || M * Ky * 2 >= 0xFFFFFF00LL ||
      M >= (1LL << 31))
    return VCG_ERR_UNSUPPORTED;
  GemmParams p{};
  p.M = (int)M;
  p.N = C;
  p.K = Cout + Ky;
  p.k_per_split = p.K + 64;
  p.a = dense_op(g, Cout, p.M, Cout, 2);
  p.a.ptr2 = yg;
  p.a.split2 = Cout;
  p.a.ld2 = Ky;
  p.a.bytes2 = M * Ky * 2;
  p.b = dense_op(wfold, p.K, C, p.K, 2);
  p.bias = bias;
  p.C = out;
  p.ldc = C;
  p.alpha = 1.f;
  BwdEpi& e = p.bwd;
  e.hw = H * W;
  e.fd_hw = make_fastdiv((uint32_t)(H * W));
  e.fd_T = make_fastdiv(1u);
  e.fd_w = make_fastdiv((uint32_t)W);
  e.res_s = 1;
  e.y = y; e.mean = mean; e.invstd = invstd; e.msc = mscale; e.msh = mshift;
  e.part = ws;
  e.nred = y ? 2 : 0;
  if (FILE* f = gemm_log()) {
    fprintf(f, "a=0 b=0 epi=3 M=%d N=%d K=%d z=1 fast=1 conv=1x1/1 C=%d bnfold=1\n", p.M, p.N, p.K, Cout);
    fflush(f);
  }
  int rc = run_fast_gemm(p, OP_DENSE_K, EPI_BWD, 1, stream);
  if (rc < 0) return VCG_ERR_UNSUPPORTED;
  if (rc) return rc;
  if (e.nred > 0) {
    rc = bn_bwd_finalize_launch(ws, fast_bwd_slots(p), C, 2LL * C, C, sum_g, sum_gx, dgamma, dbeta, 1, stream);
    if (rc) return rc;
  }
  return VCG_OK;
}

VCG_API long long vcg_conv_wgrad_bnfold_ws_bytes(int N, int H, int W, int C, int Cout) {
  int M, Nn, K, splits, kps;
  bool fast;
  wgrad_geometry(VCG_BF16, N, H, W, C, 2 * Cout, 1, 1, 1, 0, &M, &Nn, &K, &splits, &kps, &fast);
  return (long long)splits * M * Nn * 4;
}

VCG_API int vcg_conv_wgrad_bnfold(const void* x, const void* g, const void* yg, const float* mean, const float* invstd,
                                  const float* gamma, const float* sum_g, const float* sum_gx, float inv_count,
                                  const float* colsum_x, float* dw, int accumulate, float* ws, long long ws_bytes, int N,
                                  int H, int W, int C, int Cout, hipStream_t stream) {
  VCG_REQUIRE(x && g && yg && mean && invstd && sum_g && sum_gx && colsum_x && dw, "null argument");
  const int logC = ilog2_exact(C);
  VCG_REQUIRE(logC >= 6 && Cout % 128 == 0, "C must be a power of two >= 64, Cout a multiple of 128");
  int M, Nn, K, splits, kps;
  bool fast;
  wgrad_geometry(VCG_BF16, N, H, W, C, 2 * Cout, 1, 1, 1, 0, &M, &Nn, &K, &splits, &kps, &fast);
  if (!fast || wgrad_fast_tile_m(M) != 128 || (long long)K * Cout * 2 >= 0xFFFFFF00LL) return VCG_ERR_UNSUPPORTED;
  VCG_REQUIRE(ws_bytes >= (long long)splits * M * Nn * 4, "workspace too small");
  GemmParams p{};
  p.M = M;
  p.N = Nn;
  p.K = K;
  p.k_per_split = kps;
  p.a = dense_op(g, Cout, Cout);  // A[m = row of [g | y]][k = pixel]
  p.a.bytes = (long long)K * Cout * 2;
  p.a.ptr2 = yg;
  p.a.split2 = Cout;
  OpArgs b{};
  b.ptr = x; b.rows = Nn; b.N = N; b.H = H; b.W = W; b.C = C; b.logC = logC;
  b.bytes = (long long)N * H * W * C * 2;
  b.GH = H; b.GW = W; b.KH = 1; b.KW = 1; b.stride = 1; b.pad = 0;
  b.tsm_T = 1; b.tsm_fold = 0;
  b.fd_ghw = make_fastdiv(H * W); b.fd_gw = make_fastdiv(W); b.fd_T = make_fastdiv(1);
  p.b = b;
  p.ws = ws;
  p.alpha = 1.f;
  if (FILE* f = gemm_log())
    fprintf(f, "a=3 b=4 epi=2 M=%d N=%d K=%d z=%d fast=2 conv=1x1/1 C=%d bnfold=1\n", M, Nn, K, splits, C);
  int rc = run_fast_wgrad(p, splits, stream);
  if (rc) return rc;
  const long long MN = (long long)Cout * Nn;
  if ((MN + 255) / 256 < 1024 && splits >= 16)
    hipLaunchKernelGGL(splitk_reduce_bnfold_kernel<8>, dim3((unsigned)((MN * 8 + 255) / 256)), dim3(256), 0, stream,
                       ws, splits, Cout, Nn, mean, invstd, gamma, sum_g, sum_gx, inv_count, colsum_x, dw, accumulate);
  else
    hipLaunchKernelGGL(splitk_reduce_bnfold_kernel<1>, dim3((unsigned)((MN + 255) / 256)), dim3(256), 0, stream, ws,
                       splits, Cout, Nn, mean, invstd, gamma, sum_g, sum_gx, inv_count, colsum_x, dw, accumulate);
  VCG_LAUNCH_CHECK();
  return VCG_OK;
}

// BatchNorm statistics of a 1x1 conv output that is never stored (the EPI_STATS epilogue without its stores): the
// bn3 of a bottleneck whose apply is a second GEMM pass (vcg_conv1x1_bn_res_relu) and whose backward needs no y3
VCG_API int vcg_conv1x1_stats(const void* x, const void* w, float* stats, int M, int N, int K, hipStream_t stream) {
  VCG_REQUIRE(x && w && stats, "null argument");
  VCG_REQUIRE(M > 0 && N % 64 == 0 && K % 64 == 0, "N and K must be multiples of 64");
  if (!fast_gemm_enabled() || (long long)M * K * 2 >= 0xFFFFFF00LL) return VCG_ERR_UNSUPPORTED;
  GemmParams p{};
  p.M = M;
  p.N = N;
  p.K = K;
  p.k_per_split = K + 64;
  p.a = dense_op(x, K, M, K, 2);
  p.b = dense_op(w, K, N, K, 2);
  p.C = nullptr;
  p.ldc = N;
  p.alpha = 1.f;
  p.stats = stats;
  if (FILE* f = gemm_log()) {
    fprintf(f, "a=0 b=0 epi=1 M=%d N=%d K=%d z=1 fast=1 conv=1x1/1 C=%d nostore=1\n", M, N, K, K);
    fflush(f);
  }
  const int rc = run_fast_gemm(p, OP_DENSE_K, EPI_STATS, 1, stream);
  return rc < 0 ? VCG_ERR_UNSUPPORTED : rc;
}

// out = relu(bf16(x wfold^T + bias) + res) with the ReLU mask bits: a batch-statistics bn3 (scale folded into the
// conv3 weight rows by vcg_weight_fold, shift as bias) applied by a second pass of conv3's GEMM instead of reading
// the stored conv output back (trunk forward; the bn3 + residual + ReLU of vcg_bn_apply, one bf16 rounding earlier)
VCG_API int vcg_conv1x1_bn_res_relu(const void* x, const void* wfold, const float* bias, const void* res,
                                    const float* res_scale, const float* res_shift, void* out, unsigned char* bits,
                                    int M, int N, int K, hipStream_t stream) {
  VCG_REQUIRE(x && wfold && bias && res && out && bits, "null argument");
  VCG_REQUIRE(M > 0 && N % 64 == 0 && K % 64 == 0, "N and K must be multiples of 64");
  VCG_REQUIRE((((uintptr_t)x | (uintptr_t)wfold | (uintptr_t)res | (uintptr_t)out) & 15) == 0, "16-B alignment");
  VCG_REQUIRE(!res_scale == !res_shift, "res_scale and res_shift go together");
  if (!res_scale) {  // the register-streaming kernel (stream1x1.hip) where it applies
    const int rc = run_rs1x1_bnres(x, wfold, bias, res, out, bits, M, N, K, stream);
    if (rc >= 0) {
      if (FILE* f = gemm_log()) {
        fprintf(f, "a=0 b=0 epi=0 M=%d N=%d K=%d z=1 fast=4 conv=1x1/1 C=%d bnres=1\n", M, N, K, K);
        fflush(f);
      }
      return rc;
    }
  }
  if (!fast_gemm_enabled() || (long long)M * K * 2 >= 0xFFFFFF00LL || (long long)M * N * 2 >= 0xFFFFFF00LL)
    return VCG_ERR_UNSUPPORTED;
  GemmParams p{};
  p.M = M;
  p.N = N;
  p.K = K;
  p.k_per_split = K + 64;
  p.a = dense_op(x, K, M, K, 2);
  p.b = dense_op(wfold, K, N, K, 2);
  p.C = out;
  p.ldc = N;
  p.alpha = 1.f;
  p.bias = bias;
  p.act = ACT_RELU;
  p.residual = res;
  p.ldr = N;
  p.res_round = 1;
  p.obits = bits;
  p.res_sc = res_scale;
  p.res_sh = res_shift;
  if (FILE* f = gemm_log()) {
    fprintf(f, "a=0 b=0 epi=0 M=%d N=%d K=%d z=1 fast=1 conv=1x1/1 C=%d bnres=1\n", M, N, K, K);
    fflush(f);
  }
  const int rc = run_fast_gemm(p, OP_DENSE_K, EPI_STORE, 1, stream);
  return rc < 0 ? VCG_ERR_UNSUPPORTED : rc;
}

// C[M][N] = act(alpha * op(A) op(B)^T + bias + residual)
//   transA = 0: A stored [M][lda>=K];  transA = 1: A stored [K][lda>=M]
//   transB = 0: B stored [N][ldb>=K];  transB = 1: B stored [K][ldb>=N]
VCG_API int vcg_gemm(int dtype, int transA, int transB, int M, int N, int K, const void* A, long long lda,
                     const void* B, long long ldb, void* C, long long ldc, const float* bias, int act,
                     const void* residual, long long ldr, void* aux, float alpha, hipStream_t stream) {
  const int VEC = dtype == VCG_BF16 ? 8 : 4;
  VCG_REQUIRE(N % VEC == 0 && ldc % VEC == 0 && K % VEC == 0, "N, ldc, K must be multiples of 16 bytes");
  VCG_REQUIRE(residual == nullptr || ldr % 4 == 0, "ldr must be a multiple of 4");
  VCG_REQUIRE(M > 0 && N > 0 && K > 0, "empty GEMM");
  GemmParams p{};
  p.M = M; p.N = N; p.K = K; p.k_per_split = K + 64;
  const int esz = dtype == VCG_BF16 ? 2 : 4;
  p.a = transA ? dense_op(A, lda, K, M, esz) : dense_op(A, lda, M, K, esz);
  p.b = transB ? dense_op(B, ldb, K, N, esz) : dense_op(B, ldb, N, K, esz);
  p.a.rows = M;
  p.b.rows = N;
  VCG_REQUIRE((act & ~(0xff | ACT_FLAG_ROUND_PRE | ACT_FLAG_WIDE | ACT_FLAG_F32_OUT)) == 0, "unknown act flags");
  const bool wide = (act & ACT_FLAG_WIDE) != 0 && dtype == VCG_BF16 && !transA && !transB;
  const bool f32out = (act & ACT_FLAG_F32_OUT) != 0;
  VCG_REQUIRE(!f32out || (wide && residual && (act & 0xff) == 0 && !aux && alpha == 1.f),
              "VCG_ACT_FLAG_F32_OUT: a wide-engine bf16 GEMM with a residual addend only");
  act &= ~(ACT_FLAG_WIDE | ACT_FLAG_F32_OUT);
  p.C = C; p.ldc = ldc; p.bias = bias; p.act = act & 0xff; p.residual = residual; p.ldr = ldr; p.aux = aux;
  p.res_round = (act & ACT_FLAG_ROUND_PRE) != 0 && residual != nullptr;
  p.alpha = alpha;
  // BERT's Linear layers and the downsample input gradient (the caller's flag): the wide-tile engine, whatever M --
  // the oracle-anchored B = 1 step runs the kernels of the B = 64 bench
  if (wide) {
    p.fast_act = fast_gelu_enabled();
    const int we = f32out ? wide_gemm_class_f32(p) : wide_gemm_class(p);
    VCG_REQUIRE(!f32out || we >= 0, "VCG_ACT_FLAG_F32_OUT: unsupported shape / alignment");
    if (we >= 0) {
      if (FILE* f = gemm_log()) {
        fprintf(f, "wide M=%d N=%d K=%d we=%d\n", M, N, K, we);
        fflush(f);
      }
      return run_gemm_wide(p, we, stream);
    }
  }
#define VCG_GEMM_CASE(TT)                                                                   \
  if (!transA && !transB) return run_gemm<TT, OP_DENSE_K, OP_DENSE_K>(p, EPI_STORE, 1, stream);   \
  if (!transA && transB) return run_gemm<TT, OP_DENSE_K, OP_DENSE_MN>(p, EPI_STORE, 1, stream);   \
  if (transA && !transB) return run_gemm<TT, OP_DENSE_MN, OP_DENSE_K>(p, EPI_STORE, 1, stream);   \
  return run_gemm<TT, OP_DENSE_MN, OP_DENSE_MN>(p, EPI_STORE, 1, stream);
  if (dtype == VCG_BF16) { VCG_GEMM_CASE(bf16_t) }
  VCG_GEMM_CASE(float)
#undef VCG_GEMM_CASE
}

VCG_API long long vcg_gemm_splitk_ws_bytes(int dtype, int M, int N, int K) {
  const int splits = choose_splits(M, N, K, dtype == VCG_BF16 ? 32 : 16, VCG_SPLITK_TARGET_DENSE);
  return (long long)splits * M * N * 4;
}

// out (fp32 [M][N]) (+)= op(A) op(B)^T, split over K (used for weight gradients).
VCG_API int vcg_gemm_splitk(int dtype, int transA, int transB, int M, int N, int K, const void* A, long long lda,
                            const void* B, long long ldb, float* out, int accumulate, float* ws, long long ws_bytes,
                            hipStream_t stream) {
  const int BK = dtype == VCG_BF16 ? 32 : 16;
  // (the Linear weight gradients with a 256-workgroup target: -2.1 % per step, profiles/r06_vs_r05_same_box.txt)
  int splits = choose_splits(M, N, K, BK, VCG_SPLITK_TARGET_DENSE);
  VCG_REQUIRE(ws_bytes >= (long long)splits * M * N * 4, "workspace too small");
  int kps = (K + splits - 1) / splits;
  kps = (kps + BK - 1) / BK * BK;
  splits = (K + kps - 1) / kps;
  GemmParams p{};
  p.M = M; p.N = N; p.K = K; p.k_per_split = kps;
  p.a = dense_op(A, lda, M);
  p.b = dense_op(B, ldb, N);
  p.ws = ws;
  p.alpha = 1.f;
  int rc;
  // bf16 dW = A^T B with both operands row-major over K (the Linear weight gradients): the LDS-DMA wgrad kernel
  // with a dense B operand; k per split in its 64-row steps (never more splits than the workspace query allows)
  const long long a_ext = ((long long)(K - 1) * lda + M) * 2, b_ext = ((long long)(K - 1) * ldb + N) * 2;
  if (dtype == VCG_BF16 && transA && transB && fast_gemm_enabled() &&
      M % 8 == 0 && N % 8 == 0 && lda % 8 == 0 && ldb % 8 == 0 && a_ext < 0xFFFFFF00LL && b_ext < 0xFFFFFF00LL) {
    p.a.bytes = a_ext;  // [K][lda] operands: the LDS-DMA loaders' buffer range
    p.b.bytes = b_ext;
    int fk = (K + splits - 1) / splits;
    fk = (fk + 63) / 64 * 64;
    const int fsplits = (K + fk - 1) / fk;
    p.k_per_split = fk;
    if (FILE* f = gemm_log()) {
      fprintf(f, "a=3 b=3 epi=2 M=%d N=%d K=%d z=%d fast=2 conv=0x0/0 C=0\n", M, N, K, fsplits);
      fflush(f);
    }
    rc = run_fast_wgrad(p, fsplits, stream, true);
    if (rc) return rc;
    const long long MN = (long long)M * N;
    splitk_reduce(stream, ws, fsplits,
                       MN, N, out, accumulate, 0, 1, 1, 1, 1, 1.f, 0, 0, 0);
    VCG_LAUNCH_CHECK();
    return VCG_OK;
  }
#define VCG_SK_CASE(TT)                                                                             \
  if (!transA && !transB) rc = run_gemm<TT, OP_DENSE_K, OP_DENSE_K>(p, EPI_SPLITK, splits, stream);       \
  else if (!transA && transB) rc = run_gemm<TT, OP_DENSE_K, OP_DENSE_MN>(p, EPI_SPLITK, splits, stream);  \
  else if (transA && !transB) rc = run_gemm<TT, OP_DENSE_MN, OP_DENSE_K>(p, EPI_SPLITK, splits, stream);  \
  else rc = run_gemm<TT, OP_DENSE_MN, OP_DENSE_MN>(p, EPI_SPLITK, splits, stream);
  if (dtype == VCG_BF16) { VCG_SK_CASE(bf16_t) } else { VCG_SK_CASE(float) }
#undef VCG_SK_CASE
  if (rc) return rc;
  const long long MN = (long long)M * N;
  splitk_reduce(stream, ws, splits,
                     MN, N, out, accumulate, 0, 1, 1, 1, 1, 1.f, 0, 0, 0);
  VCG_LAUNCH_CHECK();
  return VCG_OK;
}

// Batched C = act(alpha * op(A) op(B)^T + bias): element z = zo*batch_inner + zi of the batch
// reads A + zo*a_so + zi*a_si (same for B, C). Used for the attention score / context products.
// Operand rows/cols beyond M/N/K are zero-filled by the loaders; K need not be a multiple of
// the 16-B vector when the A/B rows are padded with zeros up to it (attention P / dS buffers).
VCG_API int vcg_gemm_batched(int dtype, int transA, int transB, int M, int N, int K, const void* A, long long lda,
                             long long a_so, long long a_si, const void* B, long long ldb, long long b_so,
                             long long b_si, void* C, long long ldc, long long c_so, long long c_si, int batch_outer,
                             int batch_inner, const float* bias, int act, float alpha, hipStream_t stream) {
  const int VEC = dtype == VCG_BF16 ? 8 : 4;
  VCG_REQUIRE(N % VEC == 0 && ldc % VEC == 0, "N and ldc must be multiples of 16 bytes");
  VCG_REQUIRE(batch_outer > 0 && batch_inner > 0 && M > 0 && N > 0 && K > 0, "empty batched GEMM");
  GemmParams p{};
  p.M = M; p.N = N; p.K = K; p.k_per_split = K + 64;
  const int esz = dtype == VCG_BF16 ? 2 : 4;
  p.a = transA ? dense_op(A, lda, K, M, esz) : dense_op(A, lda, M, K, esz);
  p.b = transB ? dense_op(B, ldb, K, N, esz) : dense_op(B, ldb, N, K, esz);
  p.a.rows = M;
  p.b.rows = N;
  p.a.bytes += ((long long)(batch_outer - 1) * a_so + (long long)(batch_inner - 1) * a_si) * esz;
  p.b.bytes += ((long long)(batch_outer - 1) * b_so + (long long)(batch_inner - 1) * b_si) * esz;
  p.C = C; p.ldc = ldc; p.bias = bias; p.act = act; p.alpha = alpha;
  p.batch_inner = batch_inner;
  p.a_so = a_so; p.a_si = a_si; p.b_so = b_so; p.b_si = b_si; p.c_so = c_so; p.c_si = c_si;
  const int z = batch_outer * batch_inner;
#define VCG_BT_CASE(TT)                                                                   \
  if (!transA && !transB) return run_gemm<TT, OP_DENSE_K, OP_DENSE_K>(p, EPI_STORE, z, stream);   \
  if (!transA && transB) return run_gemm<TT, OP_DENSE_K, OP_DENSE_MN>(p, EPI_STORE, z, stream);   \
  if (transA && !transB) return run_gemm<TT, OP_DENSE_MN, OP_DENSE_K>(p, EPI_STORE, z, stream);   \
  return run_gemm<TT, OP_DENSE_MN, OP_DENSE_MN>(p, EPI_STORE, z, stream);
  if (dtype == VCG_BF16) { VCG_BT_CASE(bf16_t) }
  VCG_BT_CASE(float)
#undef VCG_BT_CASE
}
