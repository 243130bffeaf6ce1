// LDS-DMA operand loader of the bf16 fast GEMM engines (igemm_fast.hip, igemm256.hip): K-contiguous A / B tiles of
// [rows][64] bf16 go global -> LDS with buffer_load ... lds (16 B per lane, 1 KiB per wave instruction), 16-B chunk c of
// row r at slot c ^ ((r >> 1) & 7) (the global source address is pre-swizzled: LDS-DMA writes lane-linear), with the
// conv gathers (im2col + TSM shift, dgrad, sub-pixel stride-2 classes) computed per row once per tile.
#pragma once
#include "igemm.h"

namespace vcg {

typedef __attribute__((address_space(3))) void lds_void_t;

constexpr int FBK = 64;

__device__ __forceinline__ int fswz(int row, int chunk) { return chunk ^ ((row >> 1) & 7); }

// A-operand gather modes of the fast kernel: OP_IM2COL / OP_DGRAD (C >= 64: one filter tap per 64-wide
// k tile), OP_IM2COL_TSM (the same with the TSM shift fused), OP_IM2COL_SMALLC (C < 64: the stem)
constexpr int OP_IM2COL_TSM = 5;
constexpr int OP_IM2COL_SMALLC = 6;
// dense A from two sources along K (OpArgs ptr2 / split2): [g | y] of a BatchNorm backward folded into the consuming
// conv's input gradient; its own instantiation, so the plain dense loaders carry no second descriptor
constexpr int OP_DENSE_K2 = 8;

template <int ROWS, int MODE, int NW = 4> struct FastLoader {
  static constexpr int PER_WAVE = ROWS / (8 * NW);  // 1-KiB (8-row) slices per wave per tile
  static constexpr bool GATHER = MODE != OP_DENSE_K && MODE != OP_DENSE_K2;
  static constexpr bool TWO = MODE == OP_DENSE_K2;
  static constexpr bool IM2COL = MODE == OP_IM2COL || MODE == OP_IM2COL_TSM || MODE == OP_IM2COL_SMALLC;
  static constexpr bool TSM = MODE == OP_IM2COL_TSM;
  static constexpr bool SMALLC = MODE == OP_IM2COL_SMALLC;
  static constexpr int BAD = -(1 << 28);  // spatial base of rows beyond M: every bounds test fails
  __amdgpu_buffer_rsrc_t rsrc, rsrc2;
  uint32_t oob, oob2;
  // element offsets fit in 31 bits: the dispatcher routes only tensors < 4 GB here (32-bit buffer range)
  // Gathers with C >= 64 (one filter tap per 64-wide k tile) keep per row: pb = element offset of the
  // tap (0,0) source pixel, tm = bit mask of the taps that land inside the image (and, for stride-2
  // dgrad, on a stride-2 site); the tap's own offset is then a wave-uniform scalar. Other gathers
  // (the stem, C = 8) keep the pixel coordinates ra/rb and test per lane.
  int off[PER_WAVE];  // dense: element offset of the row (-1 = invalid row); gather: image base
  int off2[TWO ? PER_WAVE : 1];  // OP_DENSE_K2: the row's offset in the second source (its own ld2)
  int ra[PER_WAVE], rb[PER_WAVE], rc[PER_WAVE], kc[PER_WAVE];

  __device__ __forceinline__ void init(const OpArgs& a, long long batch_off, int row0, int wave, int lane) {
    const uint32_t nbytes = (uint32_t)min(a.bytes, (long long)0xFFFFFF00LL);
    rsrc = __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(a.ptr), 0, nbytes, 0x00020000);
    if constexpr (TWO) {
      const uint32_t nb2 = a.bytes2 > 0 ? (uint32_t)min(a.bytes2, (long long)0xFFFFFF00LL) : nbytes;
      rsrc2 = __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(a.ptr2), 0, nb2, 0x00020000);
      oob2 = nb2;
    }
    oob = nbytes;  // offset + 16 > num_records -> the load returns zeros
#pragma clang loop unroll(full)
    for (int q = 0; q < PER_WAVE; ++q) {
      const int r = (wave * PER_WAVE + q) * 8 + (lane >> 3);
      kc[q] = 8 * fswz(r, lane & 7);
      const int gr = row0 + r;
      const bool valid = gr < a.rows;
      if constexpr (!GATHER) {
        off[q] = valid ? (int)(batch_off + (long long)gr * a.ld) : -1;
        if constexpr (TWO) off2[q] = valid ? (int)((long long)gr * (a.ld2 > 0 ? a.ld2 : a.ld)) : -1;
      } else {
        const int n = gr / (a.GH * a.GW);
        const int rem = gr - n * a.GH * a.GW;
        int y = rem / a.GW;
        int x = rem - y * a.GW;
        if (!IM2COL && a.tKW > 0) {  // sub-pixel class of a stride-2 dgrad
          y = 2 * y + a.ry;
          x = 2 * x + a.rx;
        }
        off[q] = n * a.H * a.W * a.C;
        rc[q] = TSM ? (n % a.tsm_T) : 0;
        int py, px;  // source pixel of tap (0, 0)
        if constexpr (IM2COL) {
          py = y * a.stride - a.pad;
          px = (SMALLC && a.sw) ? x * a.sw - a.pw : x * a.stride - a.pad;
        } else {
          py = y + a.pad;
          px = x + a.pad;
        }
        if constexpr (!SMALLC) {
          // valid taps = [kh range (x parity)] x [kw range (x parity)], closed form (no loops: a runtime
          // loop here makes hipcc move the per-row arrays to scratch)
          int kh_lo, kh_hi, kw_lo, kw_hi;
          uint32_t hpar = 0xFFFFFFFFu, wpar = 0xFFFFFFFFu;  // parity filters (stride-2 dgrad)
          if constexpr (IM2COL) {
            kh_lo = max(0, -py); kh_hi = min(a.KH, a.H - py);
            kw_lo = max(0, -px); kw_hi = min(a.KW, a.W - px);
          } else if (a.stride == 2) {
            kh_lo = max(0, py - 2 * a.H + 2); kh_hi = min(a.KH, py + 1);
            kw_lo = max(0, px - 2 * a.W + 2); kw_hi = min(a.KW, px + 1);
            hpar = (py & 1) ? 0xAAAAAAAAu : 0x55555555u;  // kh = py (mod 2)
            wpar = (px & 1) ? 0xAAAAAAAAu : 0x55555555u;
          } else {
            kh_lo = max(0, py - a.H + 1); kh_hi = min(a.KH, py + 1);
            kw_lo = max(0, px - a.W + 1); kw_hi = min(a.KW, px + 1);
          }
          const int khi = min(max(kw_hi, 0), 31), klo = min(kw_lo, 31);
          const uint32_t cols = kw_hi > kw_lo ? (((1u << khi) - 1u) & ~((1u << klo) - 1u) & wpar) : 0u;
          uint32_t rows = 0;  // bit kh*KW for each allowed kh
#pragma unroll
          for (int kh = 0; kh < 8; ++kh)
            rows |= (kh >= kh_lo && kh < kh_hi && ((hpar >> kh) & 1u)) ? (1u << ((kh * a.KW) & 31)) : 0u;
          uint32_t m = cols * rows;
          if (!IM2COL && a.tKW > 0) {  // class taps: local bit a * tKW + b for kh = tkh0 + 2a, kw = tkw0 + 2b
            m = 0u;
#pragma unroll
            for (int ta = 0; ta < 2; ++ta)
#pragma unroll
              for (int tb = 0; tb < 2; ++tb) {
                const int kh = a.tkh0 + 2 * ta, kw = a.tkw0 + 2 * tb;
                const bool okt = ta < a.tKH && tb < a.tKW && kh >= kh_lo && kh < kh_hi && kw >= kw_lo && kw < kw_hi;
                m |= okt ? (1u << (ta * a.tKW + tb)) : 0u;
              }
          }
          rb[q] = valid ? (int)m : 0;
          // (the source pixel may lie outside the image: multiply, a negative value must not be shifted)
          if constexpr (IM2COL)
            ra[q] = off[q] + (py * a.W + px) * a.C;
          else
            ra[q] = off[q] + (((a.stride == 2) ? (py >> 1) : py) * a.W + ((a.stride == 2) ? (px >> 1) : px)) * a.C;
        } else {
          ra[q] = valid ? py : BAD;
          rb[q] = px;
        }
      }
    }
  }

  // general per-lane gather (C < 64): element offset of row q's tap (kh, kw), channel c
  __device__ __forceinline__ int gather(const OpArgs& a, int q, int kh, int kw, int c, bool& ok) const {
    int yy, xx;
    if constexpr (IM2COL) {
      yy = ra[q] + kh;
      xx = rb[q] + kw;
    } else {
      yy = ra[q] - kh;
      xx = rb[q] - kw;
      if (a.stride == 2) {
        ok = ok && ((yy | xx) & 1) == 0;
        yy >>= 1;
        xx >>= 1;
      }
    }
    ok = ok && ((unsigned)yy < (unsigned)a.H) && ((unsigned)xx < (unsigned)a.W);
    int e = off[q] + ((yy * a.W + xx) << a.logC) + c;
    if constexpr (TSM) {
      const int dt = c < a.tsm_fold ? 1 : (c < 2 * a.tsm_fold ? -1 : 0);
      ok = ok && ((unsigned)(rc[q] + dt) < (unsigned)a.tsm_T);
      e += dt * (a.H * a.W * a.C);
    }
    return e;
  }

  // issue the LDS-DMA loads of one 64-wide k tile into `lds` (tile base, [ROWS][64] bf16)
  __device__ __forceinline__ void issue(const OpArgs& a, int k0, int kend, bf16_t* lds, int wave) {
    if constexpr (GATHER && !SMALLC) {
      {
        // one filter tap per k tile: tap, its pixel offset and the channel base are scalars
        const int tap = k0 >> a.logC;
        int kh = tap / a.KW;
        int kw = tap - kh * a.KW;
        if (!IM2COL && a.tKW > 0) {  // class-local tap
          const int ta = tap / a.tKW;
          kh = a.tkh0 + 2 * ta;
          kw = a.tkw0 + 2 * (tap - ta * a.tKW);
        }
        const int cb = k0 & (a.C - 1);
        int toff;
        if constexpr (IM2COL) {
          toff = (kh * a.W + kw) << a.logC;
        } else {
          toff = a.stride == 2 ? -((((kh >> 1) * a.W) + (kw >> 1)) << a.logC) : -((kh * a.W + kw) << a.logC);
        }
        const uint32_t tbit = k0 < kend ? (1u << tap) : 0u;
#pragma clang loop unroll(full)
        for (int q = 0; q < PER_WAVE; ++q) {
          const int c = cb + kc[q];
          bool ok = ((uint32_t)rb[q] & tbit) != 0u;
          int e = ra[q] + toff + c;
          if constexpr (TSM) {
            const int dt = c < a.tsm_fold ? 1 : (c < 2 * a.tsm_fold ? -1 : 0);
            ok = ok && ((unsigned)(rc[q] + dt) < (unsigned)a.tsm_T);
            e += dt * (a.H * a.W * a.C);
          }
          const uint32_t voff = ok ? (uint32_t)e * 2u : oob;
          bf16_t* slice = lds + (wave * PER_WAVE + q) * 512;
          __builtin_amdgcn_raw_ptr_buffer_load_lds(rsrc, (lds_void_t*)slice, 16, voff, 0, 0, 0);
        }
        return;
      }
    }
    __amdgpu_buffer_rsrc_t rs = rsrc;
    bool sec = false;
    if constexpr (TWO) {  // the k tile lies in one source (split2 % 64 == 0): a uniform select
      sec = k0 >= a.split2;
      if (sec) {
        rs = rsrc2;
        k0 -= a.split2;
        kend -= a.split2;
      } else {
        kend = min(kend, a.split2);
      }
    }
#pragma clang loop unroll(full)
    for (int q = 0; q < PER_WAVE; ++q) {
      const int k = k0 + kc[q];
      uint32_t voff = oob;
      if constexpr (TWO) {
        const int o = sec ? off2[q] : off[q];
        voff = sec ? oob2 : oob;
        if (o >= 0 && k < kend) voff = (uint32_t)(o + k) * 2u;
      } else if constexpr (!GATHER) {
        if (off[q] >= 0 && k < kend) voff = (uint32_t)(off[q] + k) * 2u;
      } else {  // C < 64 (stem): per-lane tap
        const int tap = k >> a.logC;
        const int kh = tap / a.KW;
        const int kw = tap - kh * a.KW;
        bool ok = k < kend && kh < a.KH;
        const int e = gather(a, q, kh, kw, k & (a.C - 1), ok);
        if (ok) voff = (uint32_t)e * 2u;
      }
      bf16_t* slice = lds + (wave * PER_WAVE + q) * 512;  // 1 KiB per slice
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, (lds_void_t*)slice, 16, voff, 0, 0, 0);
    }
  }
};

// 16x16x32 bf16 fragment of rows r0..r0+15, k-step s2 (0/1) of a swizzled [rows][64] tile: ONE
// ds_read_b128 per lane. Element j of lane 16g+i is k = 32*s2 + 8g + j (same map on both operands).
// A 16-lane group reads chunk 4*s2+g of 16 consecutive rows: with the (row>>1)&7 swizzle these are
// 16 distinct 16-B slots of the 256-B bank row (conflict-free).
__device__ __forceinline__ s16x8 fast_frag(const bf16_t* lds, int r0, int lane, int s2) {
  const int g = lane >> 4, i = lane & 15;
  const int row = r0 + i;
  return *reinterpret_cast<const s16x8*>(lds + row * 64 + 8 * fswz(row, 4 * s2 + g));
}

__device__ __forceinline__ constexpr int waitcnt_vm(int n) {
  // s_waitcnt simm16 for gfx9-family: vmcnt[3:0] | expcnt 7 << 4 | lgkmcnt 15 << 8 | vmcnt[5:4] << 14
  return (n & 0xF) | (0x7 << 4) | (0xF << 8) | (((n >> 4) & 3) << 14);
}

}  // namespace vcg
