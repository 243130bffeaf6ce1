// The stem's backward after the max-pool as ONE pass: the max-pool backward, the stem BatchNorm + ReLU backward
// (the apply of maxpool_bwd2_kernel MP_APPLY) and the 7x7 / stride-2 stem conv's weight gradient, without the
// conv-output gradient dy0 ever reaching HBM (reference: the stem conv1 -> bn1 -> relu -> maxpool of
// model/vision/resnet50_tsm.py's torchvision ResNet-50; only the weight gradient is needed -- the frames take none).
//
// Unfused, the stem backward writes dy0 [N][112][112][64] (1.64 GB at the C3 batch) in the apply pass and reads it
// back in the im2col weight-gradient GEMM (plus the frames 28x through L2). Here a workgroup walks a contiguous range
// of tiles; a tile is one row pair (2k, 2k + 1) of the conv output of one image = the 2x2 pixel blocks of pooled row
// k (maxpool_bwd2_kernel's blocks), 2W pixels:
//   phase 1: per (block, 8-channel chunk) thread: the <= 4 windows' pooled gradient + argmax bytes and the 4 pixels'
//            conv output y, exactly the arithmetic of maxpool_bwd2_kernel<MP_APPLY> (window order, ReLU mask,
//            rounding of g, bn_bwd_apply's affine map, rounding of dy0) -> dy0 tile [2W][64] bf16 in LDS;
//            the 9 input rows 4k - 3 .. 4k + 5 as pair-packed super pixels (2 pixels x RGB0 = 16 B) -> LDS;
//   phase 2: dW[co][n] += sum_pix dy0[pix][co] P[pix][n], n = (kh, kwp, j, ci) the pair-packed stem layout
//            (igemm.hip pair_taps: K = 7 x 4 x 8 = 224), both operands read with ds_read_b64_tr_b16 (4
//            consecutive pixels per lane); v_mfma_f32_16x16x32_bf16, 8 waves = 4 channel tiles x 2 halves of the
//            14 n-tiles, fp32 accumulators for the whole range.
// Two LDS buffers: tile t + 1's phase 1 writes the other buffer while slower waves still read tile t, so one barrier
// per tile; tile t + 1's global loads are issued into registers before tile t's MFMAs. Each workgroup writes its
// [64][224] fp32 slab; stem_wgrad_reduce_kernel sums the slabs in a fixed order (deterministic) into the OIHW
// weight gradient.
#include "igemm.h"

namespace vcg {
namespace {

constexpr int SB_NTH = 512;
constexpr int SB_GRID = 256;   // workgroups = slabs (one per CU)
constexpr int SB_N = 224;      // pair-packed 7x7 taps: 7 rows x 4 super pixels x 8 (2 pixels x RGB0)
constexpr int SB_MAXW = 112;   // conv-output width (the tile's 2W pixels are the MFMA k)

typedef __attribute__((address_space(3))) char sb_lds_char;
__device__ __forceinline__ uint32_t sb_addr(const bf16_t* p) { return (uint32_t)(uintptr_t)(const sb_lds_char*)p; }
__device__ __forceinline__ void sb_tr(s16x4& v, const bf16_t* p) {
  asm volatile("ds_read_b64_tr_b16 %0, %1" : "=v"(v) : "v"(sb_addr(p)) : "memory");
}
__device__ __forceinline__ s16x8 sb_cat(const s16x4& lo, const s16x4& hi) {
  return s16x8{lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
}
// dy0 tile [pix][64] bf16: 16-B chunk c of pixel row r at slot c ^ 2((r >> 1) & 3) (igemm_wgrad.hip wp_swz: the
// transposed reads of 4 consecutive rows x 16 channels are conflict-free)
__device__ __forceinline__ int sb_swz(int row, int c) { return c ^ (2 * ((row >> 1) & 3)); }

struct StemBwdArgs {
  const bf16_t* dy;      // pooled-output gradient [N][OH][OW][64]
  const uint8_t* idx;    // argmax bytes [N][OH][OW][64]
  const bf16_t* y;       // stem conv output [N][H][W][64]
  const bf16_t* x;       // frames [N][2H][2W][4] = super pixels [N][2H][W][8]
  const float *mean, *invstd, *msc, *msh, *gamma, *sum_g, *sum_gx;
  float inv_count;
  int train;
  float* ws;             // SB_GRID slabs [64][224]
  int N, H, W, OH, OW, tiles;
};

struct SbRegs {  // one phase-1 item (block column j, chunk c8) and this thread's super-pixel chunks
  uint4 g[4];
  uint2 w[4];
  uint4 yv[4];
  uint4 xp[3];
};

__global__ __launch_bounds__(SB_NTH) __attribute__((amdgpu_waves_per_eu(2, 2)))
void stem_bwd_fused_kernel(StemBwdArgs a) {
  constexpr int DYE = 2 * SB_MAXW * 64;        // dy0 tile elements
  constexpr int PE = 9 * (SB_MAXW + 4) * 8;    // patch elements: 9 rows x (W + 4) super pixels
  __shared__ __attribute__((aligned(16))) bf16_t smem[2 * (DYE + PE)];
  const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int lg = lane >> 4, li = lane & 15, q = li >> 2, pp = li & 3;
  const int wm = wave & 3, wn = wave >> 2;   // channels 16 wm .., n-tiles 7 wn .. 7 wn + 6
  const int W = a.W, H = a.H, OH = a.OH, OW = a.OW;
  const int SPW = W + 4;                     // super pixels per patch row (-2 .. W + 1)
  const int HI = 2 * H;
  const int t0 = (int)(((long long)a.tiles * blockIdx.x) / gridDim.x);
  const int t1 = (int)(((long long)a.tiles * (blockIdx.x + 1)) / gridDim.x);
  const int my = t1 - t0;
  const int TPI = H / 2;
  const int nitems = (W / 2) * 8;
  const int c8 = tid & 7, jj = tid >> 3;     // phase-1 item (fixed chunk per thread)
  const bool item = tid < nitems;
  const int npch = 9 * SPW;                  // super-pixel chunks per patch

  // bn_bwd_apply's per-channel map (maxpool_bwd2_kernel MP_APPLY, same arithmetic) in LDS: [sc, sh, A, Bc, Cc][64]
  // (read per item: registers go to the accumulators, fragments and the next tile's loads)
  __shared__ __attribute__((aligned(16))) float prm[5][64];
  if (tid < 64) {
    const int c = tid;
    const float is = a.invstd[c];
    const float A = (a.gamma ? a.gamma[c] : 1.f) * is;
    const float Bc = -A * is * a.sum_gx[c] * a.inv_count;
    prm[0][c] = a.msc[c];
    prm[1][c] = a.msh[c];
    prm[2][c] = A;
    prm[3][c] = Bc;
    prm[4][c] = -A * a.sum_g[c] * a.inv_count - Bc * a.mean[c];
  }
  __syncthreads();

  SbRegs r;
  auto load = [&](int lt) {
    const int tg = t0 + lt, n = tg / TPI, k = tg - n * TPI;
    if (item) {
#pragma unroll
      for (int qq = 0; qq < 4; ++qq) {
        const int oh = min(k + (qq >> 1), OH - 1), ow = min(jj + (qq & 1), OW - 1);
        const long long o = (((long long)n * OH + oh) * OW + ow) * 64 + 8 * c8;
        r.g[qq] = *reinterpret_cast<const uint4*>(a.dy + o);
        r.w[qq] = *reinterpret_cast<const uint2*>(a.idx + o);
      }
#pragma unroll
      for (int p4 = 0; p4 < 4; ++p4) {
        const long long pix = ((long long)n * H + 2 * k + (p4 >> 1)) * W + 2 * jj + (p4 & 1);
        r.yv[p4] = *reinterpret_cast<const uint4*>(a.y + pix * 64 + 8 * c8);
      }
    }
#pragma unroll
    for (int u = 0; u < 3; ++u) {
      const int id = tid + SB_NTH * u;
      const int pr = id / SPW, sp = id - pr * SPW - 2;
      const int ih = 4 * k - 3 + pr;
      r.xp[u] = uint4{0u, 0u, 0u, 0u};
      if (id < npch && (unsigned)ih < (unsigned)HI && (unsigned)sp < (unsigned)W)
        r.xp[u] = *reinterpret_cast<const uint4*>(a.x + (((long long)n * HI + ih) * W + sp) * 8);
    }
  };
  // phase 1: dy0 of the item's 4 pixels -> dyT, the patch chunks -> P
  auto produce = [&](int lt, bf16_t* dyT, bf16_t* P) {
    const int tg = t0 + lt, n = tg / TPI, k = tg - n * TPI;
    (void)n;
    if (item) {
      float sc[8], sh[8], A[8], Bc[8], Cc[8];
      {
        float* dst[5] = {sc, sh, A, Bc, Cc};
#pragma unroll
        for (int v = 0; v < 5; ++v) {
          const float4 lo = *reinterpret_cast<const float4*>(&prm[v][8 * c8]);
          const float4 hi = *reinterpret_cast<const float4*>(&prm[v][8 * c8 + 4]);
          dst[v][0] = lo.x; dst[v][1] = lo.y; dst[v][2] = lo.z; dst[v][3] = lo.w;
          dst[v][4] = hi.x; dst[v][5] = hi.y; dst[v][6] = hi.z; dst[v][7] = hi.w;
        }
      }
      bool use[4];
#pragma unroll
      for (int qq = 0; qq < 4; ++qq) use[qq] = k + (qq >> 1) < OH && jj + (qq & 1) < OW;
#pragma unroll
      for (int p4 = 0; p4 < 4; ++p4) {
        const int aa = p4 >> 1, cc = p4 & 1;
        float acc[8], yv[8];
#pragma unroll
        for (int e = 0; e < 8; ++e) acc[e] = 0.f;
#pragma unroll
        for (int qq = 0; qq < 4; ++qq) {
          const int dr = qq >> 1, dc = qq & 1;
          if ((dr && !aa) || (dc && !cc)) continue;  // the window's rows / columns miss this pixel
          if (!use[qq]) continue;
          const uint8_t want = (uint8_t)((aa + 1 - 2 * dr) * 3 + (cc + 1 - 2 * dc));
          float gv[8];
          const uint32_t gw[4] = {r.g[qq].x, r.g[qq].y, r.g[qq].z, r.g[qq].w};
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            gv[2 * e] = __uint_as_float(gw[e] << 16);
            gv[2 * e + 1] = __uint_as_float(gw[e] & 0xffff0000u);
          }
#pragma unroll
          for (int e = 0; e < 8; ++e) {
            const uint32_t wd = e < 4 ? r.w[qq].x : r.w[qq].y;
            if (((wd >> (8 * (e & 3))) & 0xFF) == want) acc[e] += gv[e];
          }
        }
        const uint32_t yw[4] = {r.yv[p4].x, r.yv[p4].y, r.yv[p4].z, r.yv[p4].w};
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          yv[2 * e] = __uint_as_float(yw[e] << 16);
          yv[2 * e + 1] = __uint_as_float(yw[e] & 0xffff0000u);
        }
        uint32_t o[4];
#pragma unroll
        for (int e = 0; e < 8; e += 2) {
          float d[2];
#pragma unroll
          for (int h = 0; h < 2; ++h) {
            float v = fmaf(yv[e + h], sc[e + h], sh[e + h]) > 0.f ? acc[e + h] : 0.f;
            const float gr = bf2f(f2bf(v));  // the gradient as maxpool_bwd2_kernel stores / recomputes it
            d[h] = a.train ? fmaf(A[e + h], gr, fmaf(Bc[e + h], yv[e + h], Cc[e + h])) : A[e + h] * gr;
          }
          o[e >> 1] = (uint32_t)f2bf(d[0]) | ((uint32_t)f2bf(d[1]) << 16);
        }
        const int pix = aa * W + 2 * jj + cc;
        *reinterpret_cast<uint4*>(dyT + pix * 64 + 8 * sb_swz(pix, c8)) = uint4{o[0], o[1], o[2], o[3]};
      }
    }
#pragma unroll
    for (int u = 0; u < 3; ++u) {
      const int id = tid + SB_NTH * u;
      if (id < npch) *reinterpret_cast<uint4*>(P + id * 8) = r.xp[u];
    }
  };

  f32x4 acc[7];
#pragma unroll
  for (int u = 0; u < 7; ++u) acc[u] = f32x4{0.f, 0.f, 0.f, 0.f};
  const int ksteps = (2 * W + 31) / 32;  // k = the tile's 2W pixels, padded to 32 with zero dy0 rows
  for (int i = 2 * W * 8 + tid; i < ksteps * 32 * 8; i += SB_NTH)  // (the pad rows of both buffers, written once)
#pragma unroll
    for (int b = 0; b < 2; ++b) *reinterpret_cast<uint4*>(smem + b * (DYE + PE) + 8 * i) = uint4{0u, 0u, 0u, 0u};
  const int cl = 16 * wm + 4 * pp;  // this lane's channels in the dy0 transposed read
  if (my > 0) load(0);
  for (int lt = 0; lt < my; ++lt) {
    bf16_t* dyT = smem + (lt & 1) * (DYE + PE);
    bf16_t* P = dyT + DYE;
    produce(lt, dyT, P);
    if (lt + 1 < my) load(lt + 1);  // in flight under this tile's MFMAs
    __syncthreads();
    // phase 2: k = pixel; element j of lane 16g + i is pixel 32 s + 4g + 16 (j >> 2) + (j & 3) on both operands
    s16x4 al[2], ah[2], bl[2][7], bh[2][7];
    auto reads = [&](int s, int b) {
      const int k0 = 32 * s + 4 * lg + q, k1 = k0 + 16;
      sb_tr(al[b], dyT + k0 * 64 + 8 * sb_swz(k0, cl >> 3) + (cl & 7));
      sb_tr(ah[b], dyT + k1 * 64 + 8 * sb_swz(k1, cl >> 3) + (cl & 7));
      const int a0 = k0 >= W, a1 = k1 >= W;
      const int ow0 = min(k0 - a0 * W, W - 1), ow1 = min(k1 - a1 * W, W - 1);  // (pad pixels: any in-bounds chunk)
#pragma unroll
      for (int u = 0; u < 7; ++u) {
        const int t = 7 * wn + u, kh = t >> 1, kwp = 2 * (t & 1) + (pp >> 1), e0 = 4 * (pp & 1);
        sb_tr(bl[b][u], P + ((2 * a0 + kh) * SPW + ow0 + kwp) * 8 + e0);
        sb_tr(bh[b][u], P + ((2 * a1 + kh) * SPW + ow1 + kwp) * 8 + e0);
      }
    };
    auto step = [&](int s, int b) {  // (b a compile-time constant at both call sites: register arrays, no scratch)
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_sched_barrier(0);
      if (s + 1 < ksteps) reads(s + 1, b ^ 1);
      const s16x8 af = sb_cat(al[b], ah[b]);
#pragma unroll
      for (int u = 0; u < 7; ++u)
        acc[u] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(sb_cat(bl[b][u], bh[b][u]), af, acc[u], 0, 0, 0);
      __builtin_amdgcn_sched_barrier(0);
    };
    reads(0, 0);
    for (int s = 0; s < ksteps; s += 2) {
      step(s, 0);
      if (s + 1 < ksteps) step(s + 1, 1);
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  }
  // acc[u][rr] = dW[co = 16 wm + li][n = 16 (7 wn + u) + 4 lg + rr]
  float* slab = a.ws + (long long)blockIdx.x * 64 * SB_N;
#pragma unroll
  for (int u = 0; u < 7; ++u)
    *reinterpret_cast<float4*>(slab + (16 * wm + li) * SB_N + 16 * (7 * wn + u) + 4 * lg) =
        make_float4(acc[u][0], acc[u][1], acc[u][2], acc[u][3]);
}

// OIHW [64][3][7][7] (+)= sum of the slabs in slab order; n = (kh * 4 + kwp) * 8 + 4 j + ci, kw = 2 (kwp - 2) + j + 3
__global__ __launch_bounds__(256) void stem_wgrad_reduce_kernel(const float* __restrict__ ws, int nslab,
                                                                float* __restrict__ dw, int accumulate) {
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i >= 64 * 3 * 49) return;
  const int kw = i % 7, kh = (i / 7) % 7, ci = (i / 49) % 3, co = i / 147;
  const int j = (kw + 1) & 1, kwp = (kw - 3 - j) / 2 + 2;
  const int n = (kh * 4 + kwp) * 8 + 4 * j + ci;
  const float* p = ws + co * SB_N + n;
  float v = 0.f;
  for (int s = 0; s < nslab; ++s) v += p[(long long)s * 64 * SB_N];
  dw[i] = accumulate ? dw[i] + v : v;
}

}  // namespace
}  // namespace vcg

using namespace vcg;

VCG_API long long vcg_stem_bwd_fused_ws_bytes(void) { return (long long)SB_GRID * 64 * SB_N * 4; }

// The stem backward from the pooled-output gradient to the stem conv's weight gradient (bf16): max-pool backward
// (argmax idx), BN1 + ReLU backward with the sums of vcg_maxpool_bwd_bn(_sums_pooled) (mask from y * mscale +
// mshift > 0, batch statistics when train_stats), and dW of the 7x7 / stride 2 / pad 3 conv over the RGB0 frames
// x [N][2H][2W][4]; y is the conv output [N][H][W][64], dy / idx [N][H/2][W/2][64]. dW [64][3][7][7] fp32, added
// to when accumulate. Equals vcg_maxpool_bwd_bn_apply + vcg_conv_wgrad up to the fp32 summation order.
VCG_API int vcg_stem_bwd_fused(const void* dy, const unsigned char* idx, const void* y, const void* x, int N, int H,
                               int W, const float* mean, const float* invstd, const float* mscale,
                               const float* mshift, const float* gamma, const float* sum_g, const float* sum_gx,
                               long long count, int train_stats, float* ws, long long ws_bytes, float* dw,
                               int accumulate, hipStream_t s) {
  VCG_REQUIRE(dy && idx && y && x && mean && invstd && mscale && mshift && sum_g && sum_gx && dw && count > 0,
              "arguments required");
  VCG_REQUIRE(N > 0 && H > 0 && H % 2 == 0 && W % 8 == 0 && W <= SB_MAXW, "H even, W a multiple of 8, W <= 112");
  VCG_REQUIRE(ws_bytes >= vcg_stem_bwd_fused_ws_bytes(), "workspace too small");
  StemBwdArgs a{};
  a.dy = (const bf16_t*)dy; a.idx = idx; a.y = (const bf16_t*)y; a.x = (const bf16_t*)x;
  a.mean = mean; a.invstd = invstd; a.msc = mscale; a.msh = mshift; a.gamma = gamma; a.sum_g = sum_g;
  a.sum_gx = sum_gx; a.inv_count = 1.f / (float)count; a.train = train_stats; a.ws = ws;
  a.N = N; a.H = H; a.W = W; a.OH = (H - 1) / 2 + 1; a.OW = (W - 1) / 2 + 1; a.tiles = N * (H / 2);
  const int grid = a.tiles < SB_GRID ? a.tiles : SB_GRID;
  hipLaunchKernelGGL(stem_bwd_fused_kernel, dim3(grid), dim3(SB_NTH), 0, s, a);
  VCG_LAUNCH_CHECK();
  hipLaunchKernelGGL(stem_wgrad_reduce_kernel, dim3((64 * 147 + 255) / 256), dim3(256), 0, s, ws, grid, dw,
                     accumulate);
  VCG_LAUNCH_CHECK();
  return VCG_OK;
}
