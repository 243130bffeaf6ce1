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
// Every operand of a tile arrives by LDS-DMA into the workgroup's slot; two workgroups per CU (256 threads, one
// 66-KiB slot each) so one's DMA wait and VALU phase run under the other's MFMAs. (Measured at the bench shape: one
// 512-thread workgroup per CU with the next tile's loads in registers under the MFMA phase 1.43 ms; with a 2-slot
// LDS-DMA ring a tile ahead 1.63 ms -- phase 1 is VALU-bound and ran with only 2 waves per SIMD, none overlapping.) Each workgroup writes its [64][224] fp32 slab; stem_wgrad_reduce_kernel sums
// the slabs in a fixed order (deterministic) into the OIHW weight gradient.
#include "igemm.h"

#ifndef VCG_STEM_BWD_DBG
#define VCG_STEM_BWD_DBG 0
#endif

namespace vcg {
namespace {

constexpr int SB_NTH = 256;
constexpr int SB_GRID = 512;   // workgroups = slabs (two per CU)
constexpr int SB_N = 224;      // pair-packed 7x7 taps: 7 rows x 4 super pixels x 8 (2 pixels x RGB0)
constexpr int SB_MAXW = 112;   // conv-output width (the tile's 2W pixels are the MFMA k)

typedef __attribute__((address_space(3))) char sb_lds_char;
typedef __attribute__((address_space(3))) void lds_void_t;
__device__ __forceinline__ uint32_t sb_addr(const bf16_t* p) { return (uint32_t)(uintptr_t)(const sb_lds_char*)p; }
__device__ __forceinline__ void sb_tr(s16x4& v, const bf16_t* p) {
  asm volatile("ds_read_b64_tr_b16 %0, %1" : "=v"(v) : "v"(sb_addr(p)) : "memory");
}
// phase 1's LDS accesses are inline asm too: a plain LDS load while the next tile's LDS-DMA is in flight makes the
// compiler drain that DMA (vmcnt(0)) first -- the overlap this kernel is built on. Ordering is explicit instead.
typedef unsigned int sb_u32x4 __attribute__((ext_vector_type(4)));
typedef unsigned int sb_u32x2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ uint4 sb_ld16(const void* p) {
  sb_u32x4 v;
  asm volatile("ds_read_b128 %0, %1" : "=v"(v) : "v"(sb_addr(reinterpret_cast<const bf16_t*>(p))) : "memory");
  return uint4{v[0], v[1], v[2], v[3]};
}
__device__ __forceinline__ uint2 sb_ld8(const void* p) {
  sb_u32x2 v;
  asm volatile("ds_read_b64 %0, %1" : "=v"(v) : "v"(sb_addr(reinterpret_cast<const bf16_t*>(p))) : "memory");
  return uint2{v[0], v[1]};
}
__device__ __forceinline__ void sb_st16(void* p, uint4 u) {
  const sb_u32x4 v = {u.x, u.y, u.z, u.w};
  asm volatile("ds_write_b128 %0, %1" : : "v"(sb_addr(reinterpret_cast<const bf16_t*>(p))), "v"(v) : "memory");
}
__device__ __forceinline__ void sb_lgkm0() {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_sched_barrier(0);
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

// LDS slot of one tile, filled by LDS-DMA (buffer_load ... lds, 1 KiB per wave-instruction) one tile ahead:
//   Y: the conv-output rows 2k, 2k + 1 [2W][64] bf16 in the transposed-read swizzle (sb_swz, pre-applied on the
//      source side), overwritten in place by dy0 in phase 1 (a thread reads and writes the same pixels and chunk);
//   D / I: pooled gradient rows k, k + 1 [2][OW][64] bf16 and their argmax bytes [2][OW][64];
//   P: the 9 input rows of the patch, [9][W + 4] super pixels (zeros outside the frame, from the DMA range check).
constexpr int SB_YB = 2 * SB_MAXW * 128;                       // 28 KiB
constexpr int SB_DB = 2 * (SB_MAXW / 2) * 128;                 // 14 KiB
constexpr int SB_IB = 2 * (SB_MAXW / 2) * 64;                  // 7 KiB
constexpr int SB_PI = (9 * (SB_MAXW + 4) * 16 + 1023) / 1024;  // patch DMA instructions (17)
constexpr int SB_PB = SB_PI * 1024;
constexpr int SB_SLOT = SB_YB + SB_DB + SB_IB + SB_PB;         // 66 KiB

template <int DBG>
__global__ __launch_bounds__(SB_NTH) __attribute__((amdgpu_waves_per_eu(2, 2)))
void stem_bwd_fused_kernel(StemBwdArgs a) {
  __shared__ __attribute__((aligned(1024))) char smem[SB_SLOT];
  const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int lg = lane >> 4, li = lane & 15, q = li >> 2, pp = li & 3;
  const int wm = wave & 1, wn = wave >> 1;   // channels 32 wm .. + 31, n-tiles 7 wn .. 7 wn + 6
  const int W = a.W, H = a.H, OH = a.OH, OW = a.OW;
  const int SPW = W + 4;                     // super pixels per patch row (-2 .. W + 1)
  const int HI = 2 * H;
  const int t0 = (int)(((long long)a.tiles * blockIdx.x) / gridDim.x);
  const int t1 = (int)(((long long)a.tiles * (blockIdx.x + 1)) / gridDim.x);
  const int my = t1 - t0;
  const int TPI = H / 2;
  const int nitems = (W / 2) * 8;
  const int c8 = tid & 7;                    // phase-1 items tid, tid + 256 (fixed chunk per thread)
  const int nY = 2 * W / 8, nD = OW / 4, nI = (OW + 7) / 8, nP = (9 * SPW + 63) / 64;
  const int nDMA = nY + nD + nI + nP;

  const uint32_t ybytes = (uint32_t)min((long long)a.N * H * W * 128, (long long)0xFFFFFF00LL);
  const uint32_t dbytes = (uint32_t)((long long)a.N * OH * OW * 128);
  const uint32_t ibytes = (uint32_t)((long long)a.N * OH * OW * 64);
  const uint32_t xbytes = (uint32_t)((long long)a.N * HI * W * 16);
  const __amdgpu_buffer_rsrc_t yr = __builtin_amdgcn_make_buffer_rsrc(const_cast<bf16_t*>(a.y), 0, ybytes, 0x00020000);
  const __amdgpu_buffer_rsrc_t dr = __builtin_amdgcn_make_buffer_rsrc(const_cast<bf16_t*>(a.dy), 0, dbytes, 0x00020000);
  const __amdgpu_buffer_rsrc_t ir = __builtin_amdgcn_make_buffer_rsrc(const_cast<uint8_t*>(a.idx), 0, ibytes, 0x00020000);
  const __amdgpu_buffer_rsrc_t xr = __builtin_amdgcn_make_buffer_rsrc(const_cast<bf16_t*>(a.x), 0, xbytes, 0x00020000);

  // bn_bwd_apply's per-channel map (maxpool_bwd2_kernel MP_APPLY, same arithmetic) in LDS: [sc, sh, A, Bc, Cc][64]
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
  const int ksteps = (2 * W + 31) / 32;  // k = the tile's 2W pixels, padded to 32 with zero dy0 rows
  for (int i = 2 * W * 8 + tid; i < ksteps * 32 * 8; i += SB_NTH)  // (the pad rows, never DMA'd)
    *reinterpret_cast<uint4*>(smem + 16 * i) = uint4{0u, 0u, 0u, 0u};
  // a thread's phase-1 items keep one 8-channel chunk c8 for the whole kernel: its 5 x 8 parameters live in registers
  // (read once here, before any LDS-DMA is in flight, instead of 10 ds_read_b128 per item and tile)
  __syncthreads();
  float sc[8], sh[8], A[8], Bc[8], Cc[8];
  {
    float* dst[5] = {sc, sh, A, Bc, Cc};
#pragma unroll
    for (int v = 0; v < 5; ++v) {
      const uint4 lo = sb_ld16(&prm[v][8 * c8]), hi = sb_ld16(&prm[v][8 * c8 + 4]);
      sb_lgkm0();
      dst[v][0] = __uint_as_float(lo.x); dst[v][1] = __uint_as_float(lo.y);
      dst[v][2] = __uint_as_float(lo.z); dst[v][3] = __uint_as_float(lo.w);
      dst[v][4] = __uint_as_float(hi.x); dst[v][5] = __uint_as_float(hi.y);
      dst[v][6] = __uint_as_float(hi.z); dst[v][7] = __uint_as_float(hi.w);
    }
  }

  // tile lt's DMAs into the slot: instruction i = wave, wave + 4, ... of Y | D | I | P
  auto issue = [&](int lt) {
    const int tg = t0 + lt, n = tg / TPI, k = tg - n * TPI;
    char* S = smem;
    for (int i = wave; i < nDMA; i += SB_NTH / 64) {
      if (i < nY) {
        const int pix = 8 * i + (lane >> 3), aa = pix >= W, w = pix - aa * W;
        const int c = sb_swz(pix, lane & 7);  // the chunk that lands at slot lane & 7 (XOR: its own inverse)
        const uint32_t voff = (uint32_t)(((((long long)n * H + 2 * k + aa) * W + w) * 64 + 8 * c) * 2);
        __builtin_amdgcn_raw_ptr_buffer_load_lds(yr, (lds_void_t*)(S + 1024 * i), 16, voff, 0, 0, 0);
      } else if (i < nY + nD) {
        const int e = 8 * (i - nY) + (lane >> 3), pr = e / OW, pw = e - pr * OW;
        const uint32_t voff = k + pr < OH ? (uint32_t)((((long long)n * OH + k + pr) * OW + pw) * 128 + 16 * (lane & 7))
                                          : dbytes;
        __builtin_amdgcn_raw_ptr_buffer_load_lds(dr, (lds_void_t*)(S + SB_YB + 1024 * (i - nY)), 16, voff, 0, 0, 0);
      } else if (i < nY + nD + nI) {
        const int b = 1024 * (i - nY - nD) + 16 * lane, e = b >> 6, pr = e / OW, pw = e - pr * OW;
        const uint32_t voff = (pr < 2 && k + pr < OH)
                                  ? (uint32_t)((((long long)n * OH + k + pr) * OW + pw) * 64 + (b & 63)) : ibytes;
        __builtin_amdgcn_raw_ptr_buffer_load_lds(ir, (lds_void_t*)(S + SB_YB + SB_DB + 1024 * (i - nY - nD)), 16, voff,
                                                 0, 0, 0);
      } else {
        const int id = 64 * (i - nY - nD - nI) + lane, pr = id / SPW, sp = id - pr * SPW - 2, ih = 4 * k - 3 + pr;
        const bool ok = id < 9 * SPW && (unsigned)ih < (unsigned)HI && (unsigned)sp < (unsigned)W;
        const uint32_t voff = ok ? (uint32_t)((((long long)n * HI + ih) * W + sp) * 16) : xbytes;
        __builtin_amdgcn_raw_ptr_buffer_load_lds(xr, (lds_void_t*)(S + SB_YB + SB_DB + SB_IB + 1024 * (i - nY - nD - nI)),
                                                 16, voff, 0, 0, 0);
      }
    }
  };
  // phase 1: dy0 of the item's 4 pixels, in place over their y chunks
  auto produce = [&](int lt, char* S, int jj) {
    const int tg = t0 + lt, k = tg - (tg / TPI) * TPI;
    const bf16_t* Dg = reinterpret_cast<const bf16_t*>(S + SB_YB);
    const uint8_t* Ib = reinterpret_cast<const uint8_t*>(S + SB_YB + SB_DB);
    bf16_t* Y = reinterpret_cast<bf16_t*>(S);
    uint4 g4[4], y4s[4];
    uint2 w2[4];
    bool use[4];
    {
#pragma unroll
      for (int qq = 0; qq < 4; ++qq) {
        const int rr = qq >> 1, col = min(jj + (qq & 1), OW - 1);
        use[qq] = k + rr < OH && jj + (qq & 1) < OW;
        g4[qq] = sb_ld16(Dg + (rr * OW + col) * 64 + 8 * c8);
        w2[qq] = sb_ld8(Ib + (rr * OW + col) * 64 + 8 * c8);
      }
#pragma unroll
      for (int p4 = 0; p4 < 4; ++p4) {
        const int pix = (p4 >> 1) * W + 2 * jj + (p4 & 1);
        y4s[p4] = sb_ld16(Y + pix * 64 + 8 * sb_swz(pix, c8));
      }
      sb_lgkm0();
    }
#pragma unroll
    for (int p4 = 0; p4 < 4; ++p4) {
      const int aa = p4 >> 1, cc = p4 & 1;
      const int pix = aa * W + 2 * jj + cc;
      bf16_t* yp = Y + pix * 64 + 8 * sb_swz(pix, c8);
      const uint4 y4 = y4s[p4];
      float acc[8], yv[8];
#pragma unroll
      for (int e = 0; e < 8; ++e) acc[e] = 0.f;
#pragma unroll
      for (int qq = 0; qq < 4; ++qq) {
        const int dr = qq >> 1, dc = qq & 1;
        if ((dr && !aa) || (dc && !cc)) continue;  // the window's rows / columns miss this pixel
        if (!use[qq]) continue;
        const uint8_t want = (uint8_t)((aa + 1 - 2 * dr) * 3 + (cc + 1 - 2 * dc));
        const uint32_t gw[4] = {g4[qq].x, g4[qq].y, g4[qq].z, g4[qq].w};
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          const float gv = __uint_as_float((e & 1) ? (gw[e >> 1] & 0xffff0000u) : (gw[e >> 1] << 16));
          const uint32_t wd = e < 4 ? w2[qq].x : w2[qq].y;
          if (((wd >> (8 * (e & 3))) & 0xFF) == want) acc[e] += gv;
        }
      }
      const uint32_t yw[4] = {y4.x, y4.y, y4.z, y4.w};
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
      sb_st16(yp, uint4{o[0], o[1], o[2], o[3]});
    }
  };

  f32x4 acc[2][7];
#pragma unroll
  for (int mt = 0; mt < 2; ++mt)
#pragma unroll
    for (int u = 0; u < 7; ++u) acc[mt][u] = f32x4{0.f, 0.f, 0.f, 0.f};
  if (my > 0) issue(0);
  for (int lt = 0; lt < my; ++lt) {
    char* S = smem;
    // this tile's DMAs have landed (every wave)
    __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0)
    sb_lgkm0();
    __builtin_amdgcn_s_barrier();
    if (DBG != 2) {
      if (tid < nitems) produce(lt, S, tid >> 3);
      if (tid + SB_NTH < nitems) produce(lt, S, (tid + SB_NTH) >> 3);
    }
    sb_lgkm0();
    __builtin_amdgcn_s_barrier();
    const bf16_t* dyT = reinterpret_cast<const bf16_t*>(S);
    const bf16_t* P = reinterpret_cast<const bf16_t*>(S + SB_YB + SB_DB + SB_IB);
    // phase 2: k = pixel; element j of lane 16g + i is pixel 32 s + 4g + 16 (j >> 2) + (j & 3) on both operands
    // (one fragment set: the other workgroup on the CU covers this wave's LDS latency)
    s16x4 al[1][2], ah[1][2], bl[1][7], bh[1][7];
    auto reads = [&](int s, int b) {
      const int k0 = 32 * s + 4 * lg + q, k1 = k0 + 16;
#pragma unroll
      for (int mt = 0; mt < 2; ++mt) {
        const int cl = 32 * wm + 16 * mt + 4 * pp;  // this lane's channels in the dy0 transposed read
        sb_tr(al[b][mt], dyT + k0 * 64 + 8 * sb_swz(k0, cl >> 3) + (cl & 7));
        sb_tr(ah[b][mt], dyT + k1 * 64 + 8 * sb_swz(k1, cl >> 3) + (cl & 7));
      }
      const int a0 = k0 >= W, a1 = k1 >= W;
      const int ow0 = min(k0 - a0 * W, W - 1), ow1 = min(k1 - a1 * W, W - 1);  // (pad pixels: any in-bounds chunk)
#pragma unroll
      for (int u = 0; u < 7; ++u) {
        const int t = 7 * wn + u, kh = t >> 1, kwp = 2 * (t & 1) + (pp >> 1), e0 = 4 * (pp & 1);
        sb_tr(bl[b][u], P + ((2 * a0 + kh) * SPW + ow0 + kwp) * 8 + e0);
        sb_tr(bh[b][u], P + ((2 * a1 + kh) * SPW + ow1 + kwp) * 8 + e0);
      }
    };
    auto step = [&](int s, int b) {
      reads(s, b);
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_sched_barrier(0);
      const s16x8 af0 = sb_cat(al[b][0], ah[b][0]), af1 = sb_cat(al[b][1], ah[b][1]);
#pragma unroll
      for (int u = 0; u < 7; ++u) {
        const s16x8 bf = sb_cat(bl[b][u], bh[b][u]);
        acc[0][u] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bf, af0, acc[0][u], 0, 0, 0);
        acc[1][u] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bf, af1, acc[1][u], 0, 0, 0);
      }
      __builtin_amdgcn_sched_barrier(0);
    };
    if (DBG != 1)
      for (int s = 0; s < ksteps; ++s) step(s, 0);
    // every wave's reads of the slot have returned before the next tile's DMA refills it
    sb_lgkm0();
    __builtin_amdgcn_s_barrier();
    if (lt + 1 < my) issue(lt + 1);
  }
  // acc[mt][u][rr] = dW[co = 32 wm + 16 mt + li][n = 16 (7 wn + u) + 4 lg + rr]
  float* slab = a.ws + (long long)blockIdx.x * 64 * SB_N;
#pragma unroll
  for (int mt = 0; mt < 2; ++mt)
#pragma unroll
    for (int u = 0; u < 7; ++u)
      *reinterpret_cast<float4*>(slab + (32 * wm + 16 * mt + li) * SB_N + 16 * (7 * wn + u) + 4 * lg) =
          make_float4(acc[mt][u][0], acc[mt][u][1], acc[mt][u][2], acc[mt][u][3]);
}

// OIHW [64][3][7][7] (+)= sum of the slabs in slab order; n = (kh * 4 + kwp) * 8 + 4 j + ci, kw = 2 (kwp - 2) + j + 3
// Sum of the nslab [64][224] slabs -> the OIHW weight gradient. A thread owns one 16-B quad of the slab for slab group
// g (slabs g, g + SR_G, ...: every load of a slab group is contiguous across the workgroup's quads), the SR_G partials
// are combined in g order through LDS (deterministic), and the combining thread scatters its 4 taps to OIHW (pad
// channel ci = 3 and the kw = -1 tap of the pair packing dropped). (One thread per output walking all 512 slabs
// serially took 184 us per step.)
constexpr int SR_G = 16, SR_Q = 256 / SR_G;
__global__ __launch_bounds__(256) void stem_wgrad_reduce_kernel(const float* __restrict__ ws, int nslab,
                                                                float* __restrict__ dw, int accumulate) {
  __shared__ float4 part[SR_G][SR_Q];
  constexpr int QPS = 64 * SB_N / 4;  // quads per slab
  const int qi = threadIdx.x % SR_Q, g = threadIdx.x / SR_Q;
  const int q = blockIdx.x * SR_Q + qi;
  const float4* p = reinterpret_cast<const float4*>(ws) + q;
  float4 a = {0.f, 0.f, 0.f, 0.f};
#pragma unroll 4
  for (int sl = g; sl < nslab; sl += SR_G) {
    const float4 v = p[(long long)sl * QPS];
    a.x += v.x; a.y += v.y; a.z += v.z; a.w += v.w;
  }
  part[g][qi] = a;
  __syncthreads();
  if (g != 0) return;
  float t[4] = {part[0][qi].x, part[0][qi].y, part[0][qi].z, part[0][qi].w};
  for (int k = 1; k < SR_G; ++k) {
    const float4 v = part[k][qi];
    t[0] += v.x; t[1] += v.y; t[2] += v.z; t[3] += v.w;
  }
  const int co = q / (SB_N / 4), n0 = (q % (SB_N / 4)) * 4;
#pragma unroll
  for (int e = 0; e < 4; ++e) {  // n = (kh 4 + kwp) 8 + 4 j + ci, kw = 2 kwp - 1 + j
    const int n = n0 + e, ci = n & 3, j = (n >> 2) & 1, kwp = (n >> 3) & 3, kh = n >> 5;
    const int kw = 2 * kwp - 1 + j;
    if (ci < 3 && kw >= 0 && kw < 7) {
      const int i = ((co * 3 + ci) * 7 + kh) * 7 + kw;
      dw[i] = accumulate ? dw[i] + t[e] : t[e];
    }
  }
}

}  // namespace
}  // namespace vcg

using namespace vcg;

VCG_API long long vcg_stem_bwd_fused_ws_bytes(void) { return (long long)SB_GRID * 64 * SB_N * 4; }

// 1 when vcg_stem_bwd_fused takes this shape (conv output [N][H][W][64]): every operand's byte range fits the 32-bit
// buffer offsets -- y [N][H][W][64] bf16, dy [N][OH][OW][64] bf16, idx [N][OH][OW][64] u8, x [N][2H][W][8] bf16
VCG_API int vcg_stem_bwd_fused_fits(int N, int H, int W) {
  const long long lim = 0xFFFFFF00LL;
  const long long OH = (H - 1) / 2 + 1, OW = (W - 1) / 2 + 1;
  const long long yb = (long long)N * H * W * 128, db = (long long)N * OH * OW * 128;
  const long long ib = (long long)N * OH * OW * 64, xb = (long long)N * 2 * H * W * 16;
  return N > 0 && H > 0 && W > 0 && yb < lim && db < lim && ib < lim && xb < lim;
}

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
  // every operand is addressed by a 32-bit buffer offset: y (the largest, 8x the frames) must stay below 4 GB
  if (!vcg_stem_bwd_fused_fits(N, H, W)) {
    vcg::set_error("vcg_stem_bwd_fused: y / dy / idx / x must each be below 4 GB (32-bit buffer offsets)");
    return VCG_ERR_UNSUPPORTED;
  }
  StemBwdArgs a{};
  a.dy = (const bf16_t*)dy; a.idx = idx; a.y = (const bf16_t*)y; a.x = (const bf16_t*)x;
  a.mean = mean; a.invstd = invstd; a.msc = mscale; a.msh = mshift; a.gamma = gamma; a.sum_g = sum_g;
  a.sum_gx = sum_gx; a.inv_count = 1.f / (float)count; a.train = train_stats; a.ws = ws;
  a.N = N; a.H = H; a.W = W; a.OH = (H - 1) / 2 + 1; a.OW = (W - 1) / 2 + 1; a.tiles = N * (H / 2);
  const int grid = a.tiles < SB_GRID ? a.tiles : SB_GRID;
  if (census_on()) { char t_[96]; snprintf(t_, sizeof(t_), "stem_bwd_fused"); census_add(t_, a.N, a.H, a.W); }
  // (timing breakdown: a -DVCG_STEM_BWD_DBG=1 / 2 build compiles one phase out, tools/bench_stem_bwd.py)
  hipLaunchKernelGGL(stem_bwd_fused_kernel<VCG_STEM_BWD_DBG>, dim3(grid), dim3(SB_NTH), 0, s, a);
  VCG_LAUNCH_CHECK();
  hipLaunchKernelGGL(stem_wgrad_reduce_kernel, dim3(64 * SB_N / 4 / SR_Q), dim3(256), 0, s, ws, grid, dw, accumulate);
  VCG_LAUNCH_CHECK();
  return VCG_OK;
}
