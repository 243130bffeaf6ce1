// bf16 weight-gradient GEMM of the conv engine (the backward of torchvision conv2d inside
// Resnet50TSM.base_model, model/vision/resnet50_tsm.py:15; TSM shift of ops/temporal_shift.py:33-51
// folded into the gather):
//
//   dW[m = cout][n = (kh, kw, ci)] = sum_{pixel k} dy[k][cout] * x[im2col(k, n)]
//
// Both operands are "MN-contiguous": for a fixed pixel k the tile's BM couts (dy row) and its BN
// (tap, channel) columns (one NHWC pixel of x per 8-channel chunk) are contiguous 16-B chunks.
// They go global -> LDS with LDS-DMA (buffer_load ... lds, 16 B per lane, 1 KiB per wave
// instruction) into [64 k][COLS] tiles whose 16-B chunks are XOR-swizzled per k-row; fragments are
// read with ds_read_b64_tr_b16 (the transpose read gives each lane 4 consecutive k of one column),
// 16 distinct 16-B bank slots per 32 lanes. Two LDS stages, counted vmcnt, raw s_barrier (the
// pipeline of igemm_fast.hip). K (pixels) is split across workgroups; every split writes an fp32
// slab [split][M][N] that splitk_reduce_kernel sums in a fixed order (deterministic).
#include "igemm.h"

namespace vcg {

namespace {

typedef __attribute__((address_space(3))) void lds_void_t;
typedef __attribute__((address_space(3))) s16x4 lds_s16x4;

constexpr int WBK = 64;  // pixels per k-step

// swizzled 16-B slot of chunk c in k-row `row` of a [64][COLS] bf16 tile (an involution in c):
// COLS = 128 (256-B rows): rows 0..7 XOR 0,2,..,14 -> the 8 rows x 32 B read by two 16-lane groups
// of a transpose read cover all 16 slots of the 256-B bank row; COLS = 64 (128-B rows, two rows per
// bank row): XOR 0,2,4,6 over row pairs.
template <int COLS> __device__ __forceinline__ int wswz(int row, int c) {
  if constexpr (COLS == 128) return c ^ (2 * (row & 7));
  else return c ^ (2 * ((row >> 1) & 3));
}

// Per lane: one k-row (pixel offset `row` within the 64-pixel step) and one 16-B chunk per instruction.
// The loader is issued for pixels k0 = kb, kb + 64, kb + 128, ... in order, so the gather keeps each
// row's pixel coordinates (n, oh, ow, t = n mod T) and advances them by 64 pixels per step with
// carries (no divisions in the loop); everything is straight-line selects.
template <int COLS, bool GATHER> struct MNLoader {
  static constexpr int CPR = COLS / 8;          // 16-B chunks per k-row
  static constexpr int RPI = 64 / CPR;          // k-rows per 1-KiB wave instruction (4 or 8)
  static constexpr int NI = WBK / RPI / 4;      // instructions per wave per stage (4 or 2)
  __amdgpu_buffer_rsrc_t rsrc;
  uint32_t oob;
  int row[NI];   // k-row of the tile this lane fills
  int col[NI];   // dense: element column (m0 + 8c) or -1; gather: channel ci or -1
  int kh[NI], kw[NI], dt[NI];
  int n[NI], oh[NI], ow[NI], t[NI];  // gather: coordinates of the row's current pixel
  int dn, doh, dow, dtt;             // gather: a 64-pixel step in (n, oh, ow, t) units (uniform)

  __device__ __forceinline__ void init(const OpArgs& a, int col0, int ncols, int kb, int wave, int lane) {
    const uint32_t nbytes = (uint32_t)min(a.bytes, (long long)0xFFFFFF00LL);
    const void* src = a.ptr;
    if constexpr (!GATHER) {
      if (a.ptr2) {  // two sources along the output rows (OpArgs::split2 % BM == 0): a uniform choice per tile
        if (col0 >= a.split2) {
          src = a.ptr2;
          col0 -= a.split2;
          ncols -= a.split2;
        } else {
          ncols = min(ncols, a.split2);
        }
      }
    }
    rsrc = __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(src), 0, nbytes, 0x00020000);
    oob = nbytes;
    if constexpr (GATHER) {
      const int ohw = a.GH * a.GW;
      dn = WBK / ohw;
      doh = (WBK - dn * ohw) / a.GW;
      dow = WBK - dn * ohw - doh * a.GW;
      dtt = dn % a.tsm_T;
    }
#pragma clang loop unroll(full)
    for (int q = 0; q < NI; ++q) {
      const int inst = wave * NI + q;
      const int r = inst * RPI + lane / CPR;
      const int c = wswz<COLS>(r, lane % CPR);  // logical chunk whose data lands in this lane's slot
      const int cc = col0 + 8 * c;
      row[q] = r;
      if constexpr (!GATHER) {
        col[q] = cc < ncols ? cc : -1;
      } else {
        const int tap = cc >> a.logC;
        const int ci = cc & (a.C - 1);
        const int h = tap / a.KW;
        col[q] = (cc < ncols && tap < a.KH * a.KW) ? ci : -1;
        kh[q] = h - a.pad;
        kw[q] = tap - h * a.KW - (a.sw ? a.pw : a.pad);
        dt[q] = a.tsm_fold > 0 ? (ci < a.tsm_fold ? 1 : (ci < 2 * a.tsm_fold ? -1 : 0)) : 0;
        const int k = kb + r;
        const int nn = (int)fdiv((uint32_t)k, a.fd_ghw);
        const int rem = k - nn * a.GH * a.GW;
        const int y = (int)fdiv((uint32_t)rem, a.fd_gw);
        n[q] = nn;
        oh[q] = y;
        ow[q] = rem - y * a.GW;
        t[q] = nn - (int)fdiv((uint32_t)nn, a.fd_T) * a.tsm_T;
      }
    }
  }

  // pixels k0 .. k0+63 (< kend) into `lds` ([64][COLS] bf16); k0 = kb + 64 * (calls so far). Returns the
  // mask of this lane's pieces that loaded real data (bit q), for an in-LDS transform of exactly those.
  __device__ __forceinline__ uint32_t issue(const OpArgs& a, int k0, int kend, bf16_t* lds, int wave) {
    uint32_t okm = 0;
#pragma clang loop unroll(full)
    for (int q = 0; q < NI; ++q) {
      bool ok = col[q] >= 0 && k0 + row[q] < kend;
      int e;
      if constexpr (!GATHER) {
        e = (k0 + row[q]) * (int)a.ld + col[q];
      } else {
        const int ih = oh[q] * a.stride + kh[q], iw = ow[q] * (a.sw ? a.sw : a.stride) + kw[q];
        ok = ok && (unsigned)ih < (unsigned)a.H && (unsigned)iw < (unsigned)a.W;
        ok = ok && (unsigned)(t[q] + dt[q]) < (unsigned)a.tsm_T;
        e = (((n[q] + dt[q]) * a.H + ih) * a.W + iw) * a.C + col[q];
        // advance the pixel by 64 (carry ow -> oh -> n, and t = n mod T)
        int w2 = ow[q] + dow, h2 = oh[q] + doh, n2 = n[q] + dn, t2 = t[q] + dtt;
        const bool cw = w2 >= a.GW;
        w2 = cw ? w2 - a.GW : w2;
        h2 = cw ? h2 + 1 : h2;
        const bool ch = h2 >= a.GH;
        h2 = ch ? h2 - a.GH : h2;
        n2 = ch ? n2 + 1 : n2;
        t2 = ch ? t2 + 1 : t2;
        t2 = t2 >= a.tsm_T ? t2 - a.tsm_T : t2;
        ow[q] = w2;
        oh[q] = h2;
        n[q] = n2;
        t[q] = t2;
      }
      const uint32_t voff = ok ? (uint32_t)e * 2u : oob;
      bf16_t* slice = lds + (wave * NI + q) * 512;  // 1 KiB per instruction
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rsrc, (lds_void_t*)slice, 16, voff, 0, 0, 0);
      okm |= ok ? (1u << q) : 0u;
    }
    return okm;
  }
};

// 16x16x32 fragment of columns r0..r0+15 (of the [64][COLS] tile), k-substep s2: two transpose reads.
// Element j of lane 16g+i is k = 32*s2 + 4g + 16*(j>>2) + (j&3) (same map on both operands).
// The reads are inline asm: hipcc treats the ds_read_tr intrinsic as aliasing the in-flight LDS-DMA
// and drains it (vmcnt(0)) before every read. Ordering is explicit instead: the counted vmcnt +
// barrier before the reads (RAW), lgkmcnt(0) + sched_barrier before the MFMAs use them, lgkmcnt(0) +
// barrier before the stage is refilled (WAR).
typedef __attribute__((address_space(3))) char lds_char;
__device__ __forceinline__ uint32_t lds_addr(const bf16_t* p) { return (uint32_t)(uintptr_t)(const lds_char*)p; }

template <int COLS> __device__ __forceinline__ void wfrag_issue(s16x4& lo, s16x4& hi, const bf16_t* lds, int r0,
                                                                int lane, int s2) {
  const int g = lane >> 4, i = lane & 15;
  const int q = i >> 2, pp = i & 3;
  const int cl = r0 + 4 * pp;
  const int k0 = 32 * s2 + 4 * g + q, k1 = k0 + 16;
  const uint32_t a0 = lds_addr(lds + k0 * COLS + 8 * wswz<COLS>(k0, cl >> 3) + (cl & 7));
  const uint32_t a1 = lds_addr(lds + k1 * COLS + 8 * wswz<COLS>(k1, cl >> 3) + (cl & 7));
  asm volatile("ds_read_b64_tr_b16 %0, %1" : "=v"(lo) : "v"(a0) : "memory");
  asm volatile("ds_read_b64_tr_b16 %0, %1" : "=v"(hi) : "v"(a1) : "memory");
}
__device__ __forceinline__ s16x8 cat8(const s16x4& lo, const s16x4& hi) {
  return s16x8{lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
}
__device__ __forceinline__ void lgkm0() {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_sched_barrier(0);
}

__device__ __forceinline__ constexpr int wvm(int n) { return (n & 0xF) | (0x7 << 4) | (0xF << 8) | (((n >> 4) & 3) << 14); }

// BG: B is the im2col gather of x (conv wgrad); !BG: B is a dense [K][ld] operand (the Linear weight gradients
// dW = dY^T X of BERT / the head: a 1x1 "conv" whose pixels are the token rows, any column count).
template <int BM, int BN, bool BG>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(2))) void wgrad_fast_kernel(GemmParams p) {
  constexpr int MT = BM / 32, NT = BN / 32;
  constexpr int AE = WBK * BM, BE = WBK * BN;
  constexpr int NLD = MNLoader<BM, false>::NI + MNLoader<BN, BG>::NI;
  __shared__ __attribute__((aligned(1024))) bf16_t smem[2 * (AE + BE)];
  bf16_t* As = smem;
  bf16_t* Bs = smem + 2 * AE;

  const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave >> 1, wn = wave & 1;
  // XCD-aware decode of the 1-D grid: all (m-tile, n-tile) workgroups of one K split read the same dy
  // rows and x pixels (each n-tile a few filter taps of the same pixels, each m-tile other couts of the
  // same dy rows). Workgroups are dealt to the 8 XCDs round-robin by linear id, so split S runs on XCD
  // S % 8 with its tiles back to back and the re-reads hit that XCD's L2 instead of HBM. The grid is
  // padded to a multiple of 8 splits; padding workgroups exit at once.
  const int nx = (p.N + BN - 1) / BN, mtiles = (p.M + BM - 1) / BM, per = nx * mtiles;
  const int sidx = blockIdx.x >> 3;
  const int split = (sidx / per) * 8 + (blockIdx.x & 7);
  if (split >= p.batch_inner) return;  // batch_inner carries the split count here
  const int t = sidx % per;
  const int bx = t % nx, bym = t / nx;
  const int n0 = bx * BN, m0 = bym * BM;
  const int kb = split * p.k_per_split;
  const int ke = min(p.K, kb + p.k_per_split);
  const int ntiles = (ke - kb + WBK - 1) / WBK;

  MNLoader<BM, false> la;
  MNLoader<BN, BG> lb;
  la.init(p.a, m0, p.M, kb, wave, lane);
  lb.init(p.b, n0, p.N, kb, wave, lane);

  f32x4 acc[MT][NT];
#pragma unroll
  for (int i = 0; i < MT; ++i)
#pragma unroll
    for (int j = 0; j < NT; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  if (ntiles > 0) {
    la.issue(p.a, kb, ke, As, wave);
    lb.issue(p.b, kb, ke, Bs, wave);
  }
  for (int t = 0; t < ntiles; ++t) {
    const int cur = t & 1;
    if (t + 1 < ntiles) {
      la.issue(p.a, kb + (t + 1) * WBK, ke, As + (cur ^ 1) * AE, wave);
      lb.issue(p.b, kb + (t + 1) * WBK, ke, Bs + (cur ^ 1) * BE, wave);
      __builtin_amdgcn_s_waitcnt(wvm(NLD));
    } else {
      __builtin_amdgcn_s_waitcnt(wvm(0));
    }
    __builtin_amdgcn_s_barrier();
    const bf16_t* Ac = As + cur * AE;
    const bf16_t* Bc = Bs + cur * BE;
    s16x4 al[2][MT], ah[2][MT], bl[2][NT], bh[2][NT];
#pragma unroll
    for (int s2 = 0; s2 < 2; ++s2) {
#pragma unroll
      for (int i = 0; i < MT; ++i) wfrag_issue<BM>(al[s2][i], ah[s2][i], Ac, wm * (BM / 2) + i * 16, lane, s2);
#pragma unroll
      for (int j = 0; j < NT; ++j) wfrag_issue<BN>(bl[s2][j], bh[s2][j], Bc, wn * (BN / 2) + j * 16, lane, s2);
      if (s2 == 0) lgkm0();  // substep 0 landed; substep 1's reads stay in flight under its MFMAs
    }
#pragma unroll
    for (int s2 = 0; s2 < 2; ++s2) {
      if (s2 == 1) lgkm0();
#pragma unroll
      for (int i = 0; i < MT; ++i)
#pragma unroll
        for (int j = 0; j < NT; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(cat8(bl[s2][j], bh[s2][j]), cat8(al[s2][i], ah[s2][i]),
                                                              acc[i][j], 0, 0, 0);
    }
    __builtin_amdgcn_s_waitcnt(0xC07F);  // lgkmcnt(0): this wave's reads of the stage are done
    __builtin_amdgcn_s_barrier();
  }

  // acc[i][j][r] = dW[m = mbase + i*16][n = nbase + j*16 + r] -> fp32 slab of this split
  const int g = lane >> 4, ci = lane & 15;
  const int mbase = m0 + wm * (BM / 2) + ci, nbase = n0 + wn * (BN / 2) + 4 * g;
  float* ws = p.ws + (long long)split * p.M * p.N;
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
}

template <int BM, int BN, bool BG> int launch_wgrad(const GemmParams& p0, int splits, hipStream_t s) {
  GemmParams p = p0;
  p.batch_inner = splits;
  const long long per = (long long)((p.N + BN - 1) / BN) * ((p.M + BM - 1) / BM);
  const long long wgs = (splits + 7) / 8 * 8 * per;
  VCG_REQUIRE(wgs < (1LL << 31), "wgrad grid too large");
  const int tk = timing_begin(s);
  hipLaunchKernelGGL((wgrad_fast_kernel<BM, BN, BG>), dim3((unsigned)wgs), dim3(256), 0, s, p);
  if (census_on()) { char t_[96]; snprintf(t_, sizeof(t_), "wgrad_fast %dx%d bg%d z%d", BM, BN, (int)BG, splits); census_add(t_, p.M, p.N, p.K); }
  // algorithmic bytes: dy and x read once, the fp32 weight gradient written once (the split slabs are not)
  timing_end(tk, s, TIMING_WGRAD, 2.0 * p.M * p.N * (double)p.K,
             (double)p.a.bytes + (double)p.b.bytes + 4.0 * p.M * (double)p.N);
  VCG_LAUNCH_CHECK();
  return VCG_OK;
}

// ---- 3x3 / stride 1 / pad 1 weight gradient on an LDS-resident input patch (C, Cout multiples of 64) -------------
// dW[co][(kh, kw, ci)] = sum_p dy[p][co] x[p + (kh - 1, kw - 1)][ci]. An M-tile is R whole output rows of one image
// (TM = R W <= 32 KS pixels, the GEMM k of KS steps of 32; pixels TM.. are zero dy rows). Its dy rows and the
// (R + 2) x (W + 2) input pixels the 9 taps read (zero border from the descriptor range check) go to LDS ONCE by
// LDS-DMA; the 9 taps read shifted transposed fragments of the patch, where the im2col gather of wgrad_fast_kernel
// fetches x once per filter tap and dy once per 128-column tile through L2 (7.5x the operand bytes). A workgroup owns
// one 64 x 64 (co, ci) channel block (the 64 x 576 fp32 accumulator is 144 registers per lane: one workgroup per CU)
// and walks a contiguous range of tiles (halo rows shared in L2); the workgroups of one tile range (one per channel
// block) sit on one XCD, so the x / dy rows they all read come from that L2. Each writes its block of the fp32 slab
// [Cout][9 C] of its range for splitk_reduce_kernel (fixed-order sum: deterministic).
// Wave w owns input channels 16 w .. 16 w + 15 of the block for every tap (acc[co tile][tap]); per k-step it reads 4
// dy^T fragments (shared by the 9 taps) and 9 patch fragments (shared by the 4 co tiles) with ds_read_b64_tr_b16
// and runs 36 MFMAs, the next k-step's reads in flight under them. Tiles are DMA'd two ahead into a 3-slot ring
// (counted vmcnt, raw barriers: the pipeline of conv3x3_patch_kernel).
constexpr int WP_SL = 32;      // 1-KiB (8-pixel) slices of a patch slot: (R + 2) PW <= 256 pixels
constexpr int WP_RING = 3;
constexpr int WP_GRID = 256;   // workgroups (at least; see wp_grid)

struct WPatchGeom {
  int H, W, R, TM, PW, NP, NS, tiles, TPI;
  int C, CO, nct, nch, nsplit;  // channels, output channels, C / 64, (C / 64)(CO / 64), tile ranges (slabs)
};

__device__ __forceinline__ int wp_swz(int row, int c) { return c ^ (2 * ((row >> 1) & 3)); }  // = wswz<64>

template <int OFF> __device__ __forceinline__ void tr_read_at(s16x4& v, uint32_t addr) {
  asm volatile("ds_read_b64_tr_b16 %0, %1 offset:%2" : "=v"(v) : "v"(addr), "i"(OFF) : "memory");
}

// Patch rows at a fixed pitch PW (16 / 32 / 64 pixels >= W + 2, as conv3x3_patch_kernel): the swizzle depends on the
// pixel row index mod 8, so a tap's row offset kh * PW is an immediate of the transposed read and the lane's
// addresses (8 dy^T + 6 patch per k-step) are computed once per k-step instead of per read. KS: k-steps per tile.
template <int PW, int KS>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(1, 1)))
void wgrad3x3_patch_kernel(const bf16_t* __restrict__ x, const bf16_t* __restrict__ dy, float* __restrict__ ws,
                           uint32_t xbytes, uint32_t dybytes, WPatchGeom g) {
  constexpr int PE = WP_SL * 512, YE = 32 * KS * 64;
  constexpr int NIP = 8 + KS;  // LDS-DMA instructions per wave per tile (8 patch + KS dy)
  __shared__ __attribute__((aligned(1024))) bf16_t smem[WP_RING * (PE + YE)];
  bf16_t* Ps = smem;
  bf16_t* Ys = smem + WP_RING * PE;
  const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int lg = lane >> 4, li = lane & 15, q = li >> 2, pp = li & 3;
  // workgroup -> (tile range, channel block): the nch blocks of one range share blockIdx % 8 (one XCD)
  const int b = blockIdx.x, rest = b >> 3;
  const int chb = rest % g.nch, split = (rest / g.nch) * 8 + (b & 7);
  const int ci_t = chb % g.nct, co_t = chb / g.nct;
  const int t0 = (int)(((long long)g.tiles * split) / g.nsplit);
  const int t1 = (int)(((long long)g.tiles * (split + 1)) / g.nsplit);
  const int my = t1 - t0;
  const __amdgpu_buffer_rsrc_t xr = __builtin_amdgcn_make_buffer_rsrc(const_cast<bf16_t*>(x), 0, xbytes, 0x00020000);
  const __amdgpu_buffer_rsrc_t yr = __builtin_amdgcn_make_buffer_rsrc(const_cast<bf16_t*>(dy), 0, dybytes, 0x00020000);
  const int HW = g.H * g.W;

  // tile lt's DMAs: q8 < 8 patch slices wave + 4 q8 (slices >= NS repeat slice NS - 1), then KS dy slices
  auto issue_tile = [&](int lt) {
    const int tg = t0 + lt, img = tg / g.TPI, h0 = (tg - img * g.TPI) * g.R;
    bf16_t* P = Ps + (lt % WP_RING) * PE;
    bf16_t* Y = Ys + (lt % WP_RING) * YE;
#pragma unroll
    for (int q8 = 0; q8 < 8; ++q8) {
      const int slice = min(wave + 4 * q8, g.NS - 1);
      const int pix = 8 * slice + (lane >> 3);
      const int pr = pix / PW, pc = pix % PW;
      const int h = h0 - 1 + pr, w = pc - 1;
      const bool ok = pix < g.NP && (unsigned)h < (unsigned)g.H && (unsigned)w < (unsigned)g.W;
      const int c = wp_swz(pix, lane & 7);
      const uint32_t voff =
          ok ? (uint32_t)((((long long)(img * HW + h * g.W + w)) * g.C + 64 * ci_t + 8 * c) * 2) : xbytes;
      __builtin_amdgcn_raw_ptr_buffer_load_lds(xr, (lds_void_t*)(P + slice * 512), 16, voff, 0, 0, 0);
    }
#pragma unroll
    for (int q4 = 0; q4 < KS; ++q4) {
      const int slice = wave + 4 * q4;
      const int r = 8 * slice + (lane >> 3);
      const int c = wp_swz(r, lane & 7);
      const uint32_t voff =
          r < g.TM ? (uint32_t)((((long long)(img * HW + h0 * g.W + r)) * g.CO + 64 * co_t + 8 * c) * 2) : dybytes;
      __builtin_amdgcn_raw_ptr_buffer_load_lds(yr, (lds_void_t*)(Y + slice * 512), 16, voff, 0, 0, 0);
    }
  };

  // this lane's patch pixel of tap (0, 0) for k = 32 s + 4 lg + q + 16 hh (pixels >= TM: any valid pixel, dy is 0)
  int kpix[KS][2];
#pragma unroll
  for (int st = 0; st < KS; ++st)
#pragma unroll
    for (int hh = 0; hh < 2; ++hh) {
      const int k = 32 * st + 4 * lg + q + 16 * hh;
      const int r = k / g.W, xx = k - r * g.W;
      kpix[st][hh] = k < g.TM ? r * PW + xx : 0;
    }

  f32x4 acc[4][9];
#pragma unroll
  for (int ct = 0; ct < 4; ++ct)
#pragma unroll
    for (int t = 0; t < 9; ++t) acc[ct][t] = f32x4{0.f, 0.f, 0.f, 0.f};

  if (my > 0) issue_tile(0);
  if (my > 1) issue_tile(1);
  const int cb = 16 * wave + 4 * pp;  // first input channel (within the block) of this lane's 8-B transposed read
  for (int lt = 0; lt < my; ++lt) {
    if (lt + 1 < my) __builtin_amdgcn_s_waitcnt(wvm(NIP));
    else __builtin_amdgcn_s_waitcnt(wvm(0));
    __builtin_amdgcn_s_barrier();
    if (lt + 2 < my) issue_tile(lt + 2);  // into the slot of tile lt - 1 (every wave is past its reads)
    const bf16_t* P = Ps + (lt % WP_RING) * PE;
    const bf16_t* Y = Ys + (lt % WP_RING) * YE;
    s16x4 al[2][4], ah[2][4], bl[2][9], bh[2][9];
    auto reads = [&](int st, int b2) {
      const int k0 = 32 * st + 4 * lg + q, k1 = k0 + 16;
      uint32_t ya[4][2], pa[3][2];
#pragma unroll
      for (int ct = 0; ct < 4; ++ct) {
        const int cl = 16 * ct + 4 * pp;
        ya[ct][0] = lds_addr(Y + k0 * 64 + 8 * wp_swz(k0, cl >> 3) + (cl & 7));
        ya[ct][1] = lds_addr(Y + k1 * 64 + 8 * wp_swz(k1, cl >> 3) + (cl & 7));
      }
#pragma unroll
      for (int kw = 0; kw < 3; ++kw) {
        const int p0 = kpix[st][0] + kw, p1 = kpix[st][1] + kw;
        pa[kw][0] = lds_addr(P + p0 * 64 + 8 * wp_swz(p0, cb >> 3) + (cb & 7));
        pa[kw][1] = lds_addr(P + p1 * 64 + 8 * wp_swz(p1, cb >> 3) + (cb & 7));
      }
#pragma unroll
      for (int ct = 0; ct < 4; ++ct) {
        tr_read_at<0>(al[b2][ct], ya[ct][0]);
        tr_read_at<0>(ah[b2][ct], ya[ct][1]);
      }
#pragma unroll
      for (int kw = 0; kw < 3; ++kw) {  // tap t = 3 kh + kw: + kh PW pixels = kh PW 128 bytes
        tr_read_at<0>(bl[b2][kw], pa[kw][0]);
        tr_read_at<0>(bh[b2][kw], pa[kw][1]);
        tr_read_at<PW * 128>(bl[b2][3 + kw], pa[kw][0]);
        tr_read_at<PW * 128>(bh[b2][3 + kw], pa[kw][1]);
        tr_read_at<2 * PW * 128>(bl[b2][6 + kw], pa[kw][0]);
        tr_read_at<2 * PW * 128>(bh[b2][6 + kw], pa[kw][1]);
      }
    };
    reads(0, 0);
#pragma unroll
    for (int st = 0; st < KS; ++st) {
      const int b2 = st & 1;
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_sched_barrier(0);
      if (st + 1 < KS) reads(st + 1, b2 ^ 1);
#pragma unroll
      for (int t = 0; t < 9; ++t) {
        const s16x8 bf = cat8(bl[b2][t], bh[b2][t]);
#pragma unroll
        for (int ct = 0; ct < 4; ++ct)
          acc[ct][t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(cat8(al[b2][ct], ah[b2][ct]), bf, acc[ct][t], 0, 0, 0);
      }
      __builtin_amdgcn_sched_barrier(0);
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // (no reads outstanding: the ring slot may be refilled)
  }
  // acc[ct][t][r] = dW[co = 64 co_t + 16 ct + 4 lg + r][tap t][ci = 64 ci_t + 16 wave + li] -> this range's slab
  // [CO][9 C] (splitk_reduce's conv layout: n = tap C + ci)
  const int NC = 9 * g.C;
  float* slab = ws + (long long)split * g.CO * NC;
#pragma unroll
  for (int ct = 0; ct < 4; ++ct)
#pragma unroll
    for (int t = 0; t < 9; ++t)
#pragma unroll
      for (int r = 0; r < 4; ++r)
        slab[(long long)(64 * co_t + 16 * ct + 4 * lg + r) * NC + t * g.C + 64 * ci_t + 16 * wave + li] = acc[ct][t][r];
}

}  // namespace

int wgrad_fast_tile_m(int M) { return M >= 128 ? 128 : 64; }
int wgrad_fast_tile_n(int N) { return N > 64 ? 128 : 64; }

// p.a: dy as a dense [K][M] operand (ld = M), p.b: x with IM2COL_T geometry (dense_b: a dense [K][ld] operand);
// p.ws slabs.
int run_fast_wgrad(const GemmParams& p, int splits, hipStream_t s, bool dense_b) {
  const int bm = wgrad_fast_tile_m(p.M), bn = wgrad_fast_tile_n(p.N);
  if (dense_b) {
    if (bm == 128 && bn == 128) return launch_wgrad<128, 128, false>(p, splits, s);
    if (bm == 128) return launch_wgrad<128, 64, false>(p, splits, s);
    if (bn == 128) return launch_wgrad<64, 128, false>(p, splits, s);
    return launch_wgrad<64, 64, false>(p, splits, s);
  }
  if (bm == 128 && bn == 128) return launch_wgrad<128, 128, true>(p, splits, s);
  if (bm == 128) return launch_wgrad<128, 64, true>(p, splits, s);
  if (bn == 128) return launch_wgrad<64, 128, true>(p, splits, s);
  return launch_wgrad<64, 64, true>(p, splits, s);
}

// Rows per tile of wgrad3x3_patch_kernel (0: not eligible): bf16, x with C (= Cin, a multiple of 64, <= 512)
// channels, Cout a multiple of 64 (<= 512), 3x3 / stride 1 / pad 1, no TSM, W + 2 <= 64, R W <= 128,
// (R + 2) pitch <= 256, H % R == 0, W >= 14. VCG_WGRAD_PATCH=0 disables it; VCG_WGRAD_PATCH=1 keeps it to
// C = Cout = 64 (layer 1, the round-3 scope).
int wgrad_patch_rows(int dtype, int H, int W, int C, int Cin, int Cout, int KH, int KW, int stride, int pad,
                     int tsm_fold) {
  static int en = -1;
  if (en < 0) {
    const char* e = getenv("VCG_WGRAD_PATCH");
    en = (e && e[0] == '0') ? 0 : (e && e[0] == '1') ? 1 : 2;
  }
  if (!en || dtype != VCG_BF16 || C != Cin || C % 64 != 0 || Cout % 64 != 0 || C > 512 || Cout > 512 || KH != 3 ||
      KW != 3 || stride != 1 || pad != 1 || tsm_fold != 0)
    return 0;
  if (en == 1 && (C != 64 || Cout != 64)) return 0;
  // (7 x 7 maps: 49-pixel tiles of 64-pixel k-steps, 64 channel blocks -- measured slower than the im2col engine,
  // 442 vs 399 us at layer 4; layer 2 / 3: 320 vs 428, 328 vs 406 us, tools/bench_wgrad3x3.py)
  if (W + 2 > 64 || W < 14) return 0;
  const int pw = W + 2 <= 16 ? 16 : W + 2 <= 32 ? 32 : 64;
  for (int R = 128 / W; R >= 1; --R)
    if ((R + 2) * pw <= 8 * WP_SL && H % R == 0) return R;
  return 0;
}

// workgroups: at least WP_GRID, a multiple of 8 tile ranges per channel block
static int wp_grid(int C, int Cout) {
  const int nch = (C / 64) * (Cout / 64);
  int nsplit = WP_GRID / nch;
  nsplit = nsplit < 8 ? 8 : nsplit & ~7;
  return nsplit * nch;
}

int wgrad_patch_splits(int C, int Cout) { return wp_grid(C, Cout) / ((C / 64) * (Cout / 64)); }

template <int PW>
static void launch_wgrad_patch(const void* x, const void* dy, float* ws, uint32_t xb, uint32_t yb, const WPatchGeom& g,
                               int grid, hipStream_t s) {
  if (census_on()) { char t_[96]; snprintf(t_, sizeof(t_), "wgrad3x3_patch pw%d tm%d", PW, g.TM); census_add(t_, 0, 0, 0); }
  if (g.TM <= 64)
    hipLaunchKernelGGL((wgrad3x3_patch_kernel<PW, 2>), dim3(grid), dim3(256), 0, s, (const bf16_t*)x,
                       (const bf16_t*)dy, ws, xb, yb, g);
  else
    hipLaunchKernelGGL((wgrad3x3_patch_kernel<PW, 4>), dim3(grid), dim3(256), 0, s, (const bf16_t*)x,
                       (const bf16_t*)dy, ws, xb, yb, g);
}

// x: NHWC [N][H][W][C] bf16, dy: [N][H][W][Cout] bf16 -> wgrad_patch_splits(C, Cout) fp32 slabs [Cout][9 C] in ws
int run_wgrad_patch(const void* x, const void* dy, float* ws, int N, int H, int W, int C, int Cout, int R,
                    hipStream_t s) {
  WPatchGeom g;
  const int pw = W + 2 <= 16 ? 16 : W + 2 <= 32 ? 32 : 64;
  g.H = H; g.W = W; g.R = R; g.TM = R * W; g.PW = pw; g.NP = (R + 2) * pw; g.NS = (g.NP + 7) / 8;
  g.TPI = H / R; g.tiles = N * g.TPI;
  g.C = C; g.CO = Cout; g.nct = C / 64; g.nch = (C / 64) * (Cout / 64);
  const int grid = wp_grid(C, Cout);
  g.nsplit = grid / g.nch;
  const long long xb = (long long)N * H * W * C * 2, yb = (long long)N * H * W * Cout * 2;
  VCG_REQUIRE(xb < 0xFFFFFF00LL && yb < 0xFFFFFF00LL, "wgrad patch: x / dy must be below 4 GB");
  VCG_REQUIRE(g.TM <= 128, "wgrad patch: tile rows");
  const int tk = timing_begin(s);
  if (pw == 64) launch_wgrad_patch<64>(x, dy, ws, (uint32_t)xb, (uint32_t)yb, g, grid, s);
  else if (pw == 32) launch_wgrad_patch<32>(x, dy, ws, (uint32_t)xb, (uint32_t)yb, g, grid, s);
  else launch_wgrad_patch<16>(x, dy, ws, (uint32_t)xb, (uint32_t)yb, g, grid, s);
  timing_end(tk, s, TIMING_WGRAD, 2.0 * Cout * 9 * C * (double)N * H * W, (double)xb + (double)yb + 4.0 * Cout * 9 * C);
  VCG_LAUNCH_CHECK();
  return VCG_OK;
}

}  // namespace vcg
