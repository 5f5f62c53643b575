// Device helpers shared by the implicit-GEMM conv kernels (pc_conv.hip,
// pc_conv_halo.hip): activations, vector load/store, compile-time loops, the
// XCD-aware workgroup remap, counted vmcnt waits and the fused epilogue.
#pragma once
#include <type_traits>
#include <utility>
#include <stdint.h>
#include "pc_common.h"

namespace pc {

// erf(x) to 1.5e-7 absolute (Abramowitz & Stegun 7.1.26): a handful of instructions
// instead of the libm expansion, which matters in epilogues unrolled over 8 x rows
__device__ __forceinline__ float erf_fast(float x) {
  const float ax = fabsf(x);
  const float t = __builtin_amdgcn_rcpf(1.0f + 0.3275911f * ax);
  const float poly = t * (0.254829592f + t * (-0.284496736f + t * (1.421413741f + t * (-1.453152027f +
                     t * 1.061405429f))));
  const float r = 1.0f - poly * __expf(-ax * ax);
  return copysignf(r, x);
}

__device__ __forceinline__ float act_apply(float v, int act, float slope) {
  if (act == ACT_RELU) return v > 0.f ? v : 0.f;
  if (act == ACT_PRELU) return v > 0.f ? v : v * slope;
  if (act == ACT_SILU) return v * __builtin_amdgcn_rcpf(1.0f + __expf(-v));
  if (act == ACT_GELU) return 0.5f * v * (1.0f + erf_fast(v * 0.70710678118654752f));   // nn.GELU (erf)
  return v;
}

// e4m3 (OCP e4m3fn, gfx950 v_cvt_pk_fp8_f32 / v_cvt_f32_fp8) bytes of the f16c8 activations
// (DESIGN.md §3.7): 8 values times a power-of-two scale, saturated to the format's +-448
__device__ __forceinline__ float f8_sat(float v) { return fminf(fmaxf(v, -448.f), 448.f); }
__device__ __forceinline__ uint2 f8_pack8(const float* v, float mul) {
  int w0 = __builtin_amdgcn_cvt_pk_fp8_f32(f8_sat(v[0] * mul), f8_sat(v[1] * mul), 0, false);
  w0 = __builtin_amdgcn_cvt_pk_fp8_f32(f8_sat(v[2] * mul), f8_sat(v[3] * mul), w0, true);
  int w1 = __builtin_amdgcn_cvt_pk_fp8_f32(f8_sat(v[4] * mul), f8_sat(v[5] * mul), 0, false);
  w1 = __builtin_amdgcn_cvt_pk_fp8_f32(f8_sat(v[6] * mul), f8_sat(v[7] * mul), w1, true);
  return uint2{(unsigned)w0, (unsigned)w1};
}
__device__ __forceinline__ void f8_unpack8(uint2 q, float* out) {
  out[0] = __builtin_amdgcn_cvt_f32_fp8((int)q.x, 0);
  out[1] = __builtin_amdgcn_cvt_f32_fp8((int)q.x, 1);
  out[2] = __builtin_amdgcn_cvt_f32_fp8((int)q.x, 2);
  out[3] = __builtin_amdgcn_cvt_f32_fp8((int)q.x, 3);
  out[4] = __builtin_amdgcn_cvt_f32_fp8((int)q.y, 0);
  out[5] = __builtin_amdgcn_cvt_f32_fp8((int)q.y, 1);
  out[6] = __builtin_amdgcn_cvt_f32_fp8((int)q.y, 2);
  out[7] = __builtin_amdgcn_cvt_f32_fp8((int)q.y, 3);
}
// byte offset of channel ch's lo8 byte inside a pixel's f8 region (per 32-channel block: lo8 x 32,
// then hi8 x 32, i.e. the hi8 byte is kF8Hi further)
constexpr int kF8Hi = 32;
__device__ __forceinline__ int f8_lo_byte(int ch) { return ((ch >> 5) << 6) + (ch & 31); }

template <typename T>
__device__ __forceinline__ void store4(T* dst, const float* v, int n);

template <>
__device__ __forceinline__ void store4<f16>(f16* dst, const float* v, int n) {
  if (n >= 4) {
    f16x4 h = {(f16)v[0], (f16)v[1], (f16)v[2], (f16)v[3]};
    *reinterpret_cast<f16x4*>(dst) = h;
  } else {
    for (int j = 0; j < n; ++j) dst[j] = (f16)v[j];
  }
}
template <>
__device__ __forceinline__ void store4<float>(float* dst, const float* v, int n) {
  if (n >= 4) {
    *reinterpret_cast<f32x4*>(dst) = f32x4{v[0], v[1], v[2], v[3]};
  } else {
    for (int j = 0; j < n; ++j) dst[j] = v[j];
  }
}

template <typename T>
__device__ __forceinline__ void load4(const T* src, float* v, int n) {
  if constexpr (sizeof(T) == 2) {
    if (n >= 4) {
      f16x4 h = *reinterpret_cast<const f16x4*>(src);
      v[0] = (float)h[0]; v[1] = (float)h[1]; v[2] = (float)h[2]; v[3] = (float)h[3];
      return;
    }
  } else {
    if (n >= 4) {
      f32x4 h = *reinterpret_cast<const f32x4*>(src);
      v[0] = h[0]; v[1] = h[1]; v[2] = h[2]; v[3] = h[3];
      return;
    }
  }
  for (int j = 0; j < n; ++j) v[j] = (float)src[j];
}

// Compile-time loop: f(integral_constant<int, 0>) ... f(integral_constant<int, N-1>).
template <typename F, int... I>
__device__ __forceinline__ void static_for_impl(F&& f, std::integer_sequence<int, I...>) {
  (f(std::integral_constant<int, I>{}), ...);
}
template <int N, typename F>
__device__ __forceinline__ void static_for(F&& f) {
  static_for_impl(f, std::make_integer_sequence<int, N>{});
}

// Workgroup order: the dispatcher deals blocks round-robin over the 8 XCDs (b and
// b+8 share one), so hand each XCD a contiguous range of tiles; with the channel
// tile fastest, the channel tiles of one pixel tile share its im2col rows in the
// same L2. Bijective for any grid size (MI355X_MICROARCH.md, T1).
__device__ __forceinline__ int xcd_remap(int b, int nwg) {
  const int xcd = b & 7, idx = b >> 3;
  const int q = nwg >> 3, r = nwg & 7;
  return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + idx;
}

// s_waitcnt vmcnt(n) with n known only at run time but wave-uniform (per-wave DMA count)
__device__ __forceinline__ void vmcnt_wait(int n) {
#define PC_VMW(k) case k: asm volatile("s_waitcnt vmcnt(" #k ")" ::: "memory"); break;
  switch (n) {
    PC_VMW(0) PC_VMW(1) PC_VMW(2) PC_VMW(3) PC_VMW(4) PC_VMW(5) PC_VMW(6) PC_VMW(7)
    PC_VMW(8) PC_VMW(9) PC_VMW(10) PC_VMW(11) PC_VMW(12) PC_VMW(13) PC_VMW(14) PC_VMW(15)
    PC_VMW(16) PC_VMW(17) PC_VMW(18) PC_VMW(19) PC_VMW(20) PC_VMW(21) PC_VMW(22) PC_VMW(23)
    PC_VMW(24) PC_VMW(25) PC_VMW(26) PC_VMW(27) PC_VMW(28) PC_VMW(29) PC_VMW(30) PC_VMW(31)
    PC_VMW(32) PC_VMW(33) PC_VMW(34) PC_VMW(35) PC_VMW(36) PC_VMW(37) PC_VMW(38) PC_VMW(39)
    PC_VMW(40) PC_VMW(41) PC_VMW(42) PC_VMW(43) PC_VMW(44) PC_VMW(45) PC_VMW(46) PC_VMW(47)
    default: asm volatile("s_waitcnt vmcnt(48)" ::: "memory"); break;
  }
#undef PC_VMW
}

// Fused epilogue shared by the conv kernels: acc[a][b] is the 16x16 fragment of
// channels c0 + wr*WTC + a*16 + (lane>>4)*4 + j, pixels p0 + wc*WTP + b*16 + (lane&15).
// conv_epilogue_map: the same with the pixel of fragment column b given by pixf(b)
// (-1: not an output pixel) and the wave's first channel cw = c0 + wr*WTC - for
// kernels whose pixel tiles are not linear runs (pc_conv_t2d.hip: 2-D blocks).
// PIN: one fragment column at a time (no loads hoisted across columns) - for kernels
// that hold many registers live through the epilogue.
template <typename T, int TC, int TP, bool PIN = false, typename PixF>
__device__ __forceinline__ void conv_epilogue_map(const ConvParams& p, f32x4 (&acc)[TC][TP], int cw, int lane, int z,
                                                  PixF&& pixf) {
  const int chq = (lane >> 4) * 4;
  // compile-time (a, b) everywhere: a runtime fragment index would demote acc to scratch
  static_for<TP>([&](auto bc) __attribute__((always_inline)) {
    constexpr int b = decltype(bc)::value;
    if constexpr (PIN) __builtin_amdgcn_sched_barrier(0);
    const int pix = pixf(b);
    if (pix < 0) return;
    if (p.splitk > 1) {
      static_for<TC>([&](auto ac) __attribute__((always_inline)) {
        constexpr int a = decltype(ac)::value;
        const int ch = cw + a * 16 + chq;
        float* dst = p.partial + ((long long)z * p.M + pix) * p.npad + ch;
        *reinterpret_cast<f32x4*>(dst) = acc[a][b];
      });
      return;
    }
    int n = 0, oh = 0, ow = 0;
    if (p.bias_mode == BIAS_BORDER9 || p.res_mode == RES_UP2) {
      const int hw = p.OH * p.OW;
      n = pix / hw;
      const int rem = pix - n * hw;
      oh = rem / p.OW;
      ow = rem - oh * p.OW;
    }
    int bofs = 0;
    if (p.bias_mode == BIAS_BORDER9) {
      // class of this output pixel w.r.t. which taps of the (single) 3x3 segment fall
      // into the zero padding of the folded pre-BN input
      const ConvSeg& S = p.seg[0];
      const int ih0 = oh * S.stride - S.pad, iw0 = ow * S.stride - S.pad;
      const int rc = ih0 < 0 ? 0 : (ih0 + S.KH - 1 >= S.H ? 2 : 1);
      const int cc = iw0 < 0 ? 0 : (iw0 + S.KW - 1 >= S.W ? 2 : 1);
      bofs = (rc * 3 + cc) * p.npad;
    }
    long long rpix = pix;
    if (p.res_mode == RES_UP2) rpix = ((long long)n * p.rH + (oh >> 1)) * p.rW + (ow >> 1);
    static_for<TC>([&](auto ac) __attribute__((always_inline)) {
      constexpr int a = decltype(ac)::value;
      const int ch = cw + a * 16 + chq;
      if (ch >= p.cwrite) return;
      const int nv = min(4, p.cwrite - ch);
      float v[4] = {acc[a][b][0], acc[a][b][1], acc[a][b][2], acc[a][b][3]};
      if (p.bias_mode != BIAS_NONE) {
#pragma unroll
        for (int j = 0; j < 4; ++j) v[j] += p.bias[bofs + ch + j];
      }
      float sl[4] = {0.f, 0.f, 0.f, 0.f};
      if (p.act == ACT_PRELU) {
#pragma unroll
        for (int j = 0; j < 4; ++j) sl[j] = p.slope[ch + j];
      }
      if (!p.act_after_res) {
#pragma unroll
        for (int j = 0; j < 4; ++j) v[j] = act_apply(v[j], p.act, sl[j]);
      }
      if (p.res_mode != RES_NONE) {
        float r[4] = {0.f, 0.f, 0.f, 0.f};
        load4<T>(reinterpret_cast<const T*>(p.res) + rpix * p.rcs + ch, r, nv);
        if (p.rsplit) {   // f16x3 residual: hi + lo (exact in f32)
          float r2[4] = {0.f, 0.f, 0.f, 0.f};
          load4<T>(reinterpret_cast<const T*>(p.res) + rpix * p.rcs + p.rsplit + ch, r2, nv);
#pragma unroll
          for (int j = 0; j < 4; ++j) r[j] += r2[j];
        }
#pragma unroll
        for (int j = 0; j < 4; ++j) v[j] += r[j];
      }
      if (p.act_after_res) {
#pragma unroll
        for (int j = 0; j < 4; ++j) v[j] = act_apply(v[j], p.act, sl[j]);
      }
#pragma unroll
      for (int j = 0; j < 4; ++j)
        if (ch + j >= p.cout) v[j] = 0.f;  // keep channel padding exactly zero
      if (p.out_f32) {
        store4<float>(reinterpret_cast<float*>(p.y) + (long long)pix * p.ycs + ch, v, nv);
      } else {
        T* yp = reinterpret_cast<T*>(p.y) + (long long)pix * p.ycs + ch;
        store4<T>(yp, v, nv);
        if (p.ysplit) {   // f16x3 output: lo = f16(v - f16(v))
          float lo[4];
#pragma unroll
          for (int j = 0; j < 4; ++j) lo[j] = v[j] - (float)(T)v[j];
          store4<T>(yp + p.ysplit, lo, nv);
        }
      }
    });
  });
}

template <typename T, int TC, int TP, int WTC, int WTP>
__device__ __forceinline__ void conv_epilogue(const ConvParams& p, f32x4 (&acc)[TC][TP], int c0, int p0, int wr,
                                              int wc, int lane, int z) {
  conv_epilogue_map<T, TC, TP>(p, acc, c0 + wr * WTC, lane, z, [&](int b) __attribute__((always_inline)) {
    const int pix = p0 + wc * WTP + b * 16 + (lane & 15);
    return pix < p.M ? pix : -1;
  });
}


// Epilogue through LDS (the kernel's LDS is free once its main loop has drained):
// the waves write their f32 accumulators into a padded [pixel][channel] image (one
// or two passes of <= 128 KiB), then every thread finishes 8 channels of one pixel
// - bias (per channel or border class), activation, residual, zeroed channel
// padding - and stores them with one 16-byte (f16) or two (f32) stores, so each
// pixel row of the tile leaves as contiguous bytes and no load waits behind a store.
template <typename T, int BC, int BP, int WC, int WP, int EPI_MAX = 131072, int RGMAX = 8, bool SPLIT = false>
__device__ __forceinline__ void conv_epilogue_lds(const ConvParams& p, f32x4 (&acc)[BC / WC / 16][BP / WP / 16],
                                                  int c0, int p0, int wr, int wc, int lane, char* smem) {
  constexpr int NW = WC * WP, NT = 64 * NW;
  constexpr int WTC = BC / WC, WTP = BP / WP, TC = WTC / 16, TP = WTP / 16;
  constexpr bool ONE = BC * BP * 4 <= EPI_MAX;   // EPI_MAX: LDS the image may use (2 WGs/CU: half)
  constexpr bool SPLIT_C = !ONE && WC >= 2;
  static_assert(ONE || WC >= 2 || WP >= 2, "epilogue split");
  constexpr int PC = ONE ? BC : (SPLIT_C ? BC / 2 : BC);
  constexpr int PP = ONE ? BP : (SPLIT_C ? BP : BP / 2);
  constexpr int NPASS = ONE ? 1 : 2;
  constexpr int RS = PC + 4;            // padded row: 16 pixel rows of a fragment hit distinct banks
  constexpr int CG = PC / 8;            // 8-channel groups per pixel row
  static_assert(PP * RS * 4 <= 163840, "epilogue image exceeds LDS");
  static_assert((CG & (CG - 1)) == 0, "channel groups per row must be a power of two");
  constexpr int ESZ = sizeof(T);
  const int oesz = p.out_f32 ? 4 : ESZ;
  const bool vec_ok = ((reinterpret_cast<uintptr_t>(p.y) | (uintptr_t)(p.ycs * oesz)) & 15) == 0 &&
                      ((p.ysplit | p.rsplit) & 7) == 0 &&
                      (p.res_mode == RES_NONE ||
                       ((reinterpret_cast<uintptr_t>(p.res) | (uintptr_t)(p.rcs * ESZ)) & 15) == 0);
  const int hw = p.OH * p.OW;
#pragma unroll
  for (int pass = 0; pass < NPASS; ++pass) {
    const int cbase = ONE ? 0 : (SPLIT_C ? pass * PC : 0);
    const int pbase = ONE ? 0 : (SPLIT_C ? 0 : pass * PP);
    const bool mine = ONE || (SPLIT_C ? (wr / (WC / 2) == pass) : (wc / (WP / 2) == pass));
    if (mine) {
      static_for<TC>([&](auto ac) __attribute__((always_inline)) {
        constexpr int a = decltype(ac)::value;
        static_for<TP>([&](auto bc) __attribute__((always_inline)) {
          constexpr int b = decltype(bc)::value;
          const int cl = wr * WTC + a * 16 + (lane >> 4) * 4 - cbase;
          const int pl = wc * WTP + b * 16 + (lane & 15) - pbase;
          *reinterpret_cast<f32x4*>(smem + (pl * RS + cl) * 4) = acc[a][b];
        });
      });
    }
    __syncthreads();
    // A thread keeps one 8-channel group for all its pixel rows (NT % CG == 0), so the
    // per-channel bias / slopes are loaded once, and every residual row is requested
    // before the first store: the finishing loop no longer waits on one global load per
    // row (latency-bound at one workgroup per CU).
    static_assert((PP * CG) % NT == 0 && NT % CG == 0, "epilogue work split");
    constexpr int IT = PP * CG / NT;     // pixel rows per thread
    constexpr int PSTEP = NT / CG;       // pixel-row stride between them
    const int cg = threadIdx.x & (CG - 1);
    const int pl0 = threadIdx.x / CG;
    const int ch = c0 + cbase + cg * 8;
    if (ch < p.cwrite) {
      const int nv = min(8, p.cwrite - ch);
      const bool full = nv == 8 && vec_ok;
      float bc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
      if (p.bias_mode == BIAS_CHANNEL) {   // bias arrays span npad >= ch + 8
        const f32x4 b0 = *reinterpret_cast<const f32x4*>(p.bias + ch);
        const f32x4 b1 = *reinterpret_cast<const f32x4*>(p.bias + ch + 4);
        bc[0] = b0[0]; bc[1] = b0[1]; bc[2] = b0[2]; bc[3] = b0[3];
        bc[4] = b1[0]; bc[5] = b1[1]; bc[6] = b1[2]; bc[7] = b1[3];
      }
      // branch-light finishing: the piecewise-linear activations become one select with a
      // per-lane negative slope (1 = none, 0 = ReLU, a = PReLU); SiLU / GELU take one
      // uniform branch per row; channel padding is a per-lane keep mask
      float sl[8] = {1.f, 1.f, 1.f, 1.f, 1.f, 1.f, 1.f, 1.f};
      if (p.act == ACT_PRELU) {
        const f32x4 s0 = *reinterpret_cast<const f32x4*>(p.slope + ch);
        const f32x4 s1 = *reinterpret_cast<const f32x4*>(p.slope + ch + 4);
        sl[0] = s0[0]; sl[1] = s0[1]; sl[2] = s0[2]; sl[3] = s0[3];
        sl[4] = s1[0]; sl[5] = s1[1]; sl[6] = s1[2]; sl[7] = s1[3];
      } else if (p.act == ACT_RELU) {
#pragma unroll
        for (int j = 0; j < 8; ++j) sl[j] = 0.f;
      }
      const bool smooth = p.act == ACT_SILU || p.act == ACT_GELU;
      const bool has_res = p.res_mode != RES_NONE;
      const bool pre_act = !p.act_after_res;
      bool keep[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) keep[j] = ch + j < p.cout;
      auto act8 = [&](float* v) __attribute__((always_inline)) {
        if (smooth) {
          if (p.act == ACT_SILU) {
#pragma unroll
            for (int j = 0; j < 8; ++j) v[j] = act_apply(v[j], ACT_SILU, 0.f);
          } else {
#pragma unroll
            for (int j = 0; j < 8; ++j) v[j] = act_apply(v[j], ACT_GELU, 0.f);
          }
        } else {
#pragma unroll
          for (int j = 0; j < 8; ++j) v[j] = v[j] > 0.f ? v[j] : v[j] * sl[j];
        }
      };
      // residual rows, requested a group of RG rows at a time before the group's stores
      // (raw activation-dtype vectors; RG bounded so the second pass's accumulators and
      // these stay within the 256 registers of a 2-waves-per-SIMD kernel)
      using RV = typename std::conditional<ESZ == 2, f16x8, f32x4>::type;
      constexpr int RN = ESZ == 2 ? 1 : 2;
      // r03: all rows of the pass at once when they are few (IT <= RGMAX): with RG = 1 the
      // 256x224 tile's 7 rows per pass were 14 dependent residual round trips per tile
      // (most of its ~11 us epilogue)
      constexpr int RG0 = (NPASS == 2 ? 2 : 4) < IT ? (NPASS == 2 ? 2 : 4) : IT;
      // (f16 tiles below 256x256 only: the f32 and the largest f16 instantiations spill with it)
      constexpr int RGM = (ESZ == 2 && BC * BP < 65536) ? (SPLIT ? RGMAX / 2 : RGMAX) : 0;
      constexpr int RG = IT <= RGM ? IT : (IT % RG0 == 0 ? RG0 : (IT % 2 == 0 ? 2 : 1));
      static_assert(IT % RG == 0, "residual groups");
#pragma unroll 1
      for (int kg = 0; kg < IT; kg += RG) {
      RV rv[RG][RN];
      RV rv2[SPLIT ? RG : 1][RN];   // f16x3: the residual's lo half
      uint2 rq[SPLIT ? RG : 1];     // f16c8: the residual's lo8 bytes
      if (p.res_mode != RES_NONE) {
#pragma unroll
        for (int kk = 0; kk < RG; ++kk) {
          const int k = kk;
          const int pix = p0 + pbase + pl0 + (kg + kk) * PSTEP;
#pragma unroll
          for (int j = 0; j < RN; ++j) rv[k][j] = RV{};
          if constexpr (SPLIT) {
#pragma unroll
            for (int j = 0; j < RN; ++j) rv2[k][j] = RV{};
            rq[k] = uint2{0u, 0u};
          }
          if (pix < p.M && full) {
            long long rpix = pix;
            if (p.res_mode == RES_UP2) {
              const int n = pix / hw, rem = pix - (pix / hw) * hw;
              const int oh = rem / p.OW, ow = rem - (rem / p.OW) * p.OW;
              rpix = ((long long)n * p.rH + (oh >> 1)) * p.rW + (ow >> 1);
            }
            const T* rp = reinterpret_cast<const T*>(p.res) + rpix * p.rcs + ch;
#pragma unroll
            for (int j = 0; j < RN; ++j) rv[k][j] = *reinterpret_cast<const RV*>(rp + j * (8 / RN));
            if constexpr (SPLIT) {
              if (p.rc8) {
                rq[k] = *reinterpret_cast<const uint2*>(reinterpret_cast<const char*>(rp - ch + p.rsplit) +
                                                         f8_lo_byte(ch));
              } else if (p.rsplit) {
#pragma unroll
                for (int j = 0; j < RN; ++j) rv2[k][j] = *reinterpret_cast<const RV*>(rp + p.rsplit + j * (8 / RN));
              }
            }
          }
        }
      }
#pragma unroll
      for (int k = 0; k < RG; ++k) {
        const int pl = pl0 + (kg + k) * PSTEP;
        const int pix = p0 + pbase + pl;
        if (pix >= p.M) continue;
        float v[8];
        {
          const f32x4 lo = *reinterpret_cast<const f32x4*>(smem + (pl * RS + cg * 8) * 4);
          const f32x4 hi = *reinterpret_cast<const f32x4*>(smem + (pl * RS + cg * 8 + 4) * 4);
          v[0] = lo[0] + bc[0]; v[1] = lo[1] + bc[1]; v[2] = lo[2] + bc[2]; v[3] = lo[3] + bc[3];
          v[4] = hi[0] + bc[4]; v[5] = hi[1] + bc[5]; v[6] = hi[2] + bc[6]; v[7] = hi[3] + bc[7];
        }
        int n = 0, oh = 0, ow = 0;
        if (p.bias_mode == BIAS_BORDER9 || (p.res_mode == RES_UP2 && !full)) {
          n = pix / hw;
          const int rem = pix - n * hw;
          oh = rem / p.OW;
          ow = rem - oh * p.OW;
        }
        if (p.bias_mode == BIAS_BORDER9) {
          const ConvSeg& S = p.seg[0];
          const int ih0 = oh * S.stride - S.pad, iw0 = ow * S.stride - S.pad;
          const int rc = ih0 < 0 ? 0 : (ih0 + S.KH - 1 >= S.H ? 2 : 1);
          const int cc = iw0 < 0 ? 0 : (iw0 + S.KW - 1 >= S.W ? 2 : 1);
          const float* bp = p.bias + (rc * 3 + cc) * p.npad + ch;
          const f32x4 b0 = *reinterpret_cast<const f32x4*>(bp);
          const f32x4 b1 = *reinterpret_cast<const f32x4*>(bp + 4);
          v[0] += b0[0]; v[1] += b0[1]; v[2] += b0[2]; v[3] += b0[3];
          v[4] += b1[0]; v[5] += b1[1]; v[6] += b1[2]; v[7] += b1[3];
        }
        if (has_res && !pre_act) {   // act(acc + bias + residual): residual first
          if (full) {
            if constexpr (ESZ == 2) {
              if constexpr (SPLIT) {   // hi + lo first: the f32 value of the split residual
                float rl[8];
                if (p.rc8) {
                  f8_unpack8(rq[k], rl);
#pragma unroll
                  for (int j = 0; j < 8; ++j) rl[j] *= p.rlo_inv;
                } else {
#pragma unroll
                  for (int j = 0; j < 8; ++j) rl[j] = (float)rv2[k][0][j];
                }
#pragma unroll
                for (int j = 0; j < 8; ++j) v[j] += (float)rv[k][0][j] + rl[j];
              } else {
#pragma unroll
                for (int j = 0; j < 8; ++j) v[j] += (float)rv[k][0][j];
              }
            } else {
#pragma unroll
              for (int j = 0; j < 4; ++j) { v[j] += rv[k][0][j]; v[4 + j] += rv[k][1][j]; }
            }
          } else {
            long long rpix = pix;
            if (p.res_mode == RES_UP2) rpix = ((long long)n * p.rH + (oh >> 1)) * p.rW + (ow >> 1);
            const T* rp = reinterpret_cast<const T*>(p.res) + rpix * p.rcs + ch;
            if (SPLIT && p.rc8) {
              const unsigned char* rb = reinterpret_cast<const unsigned char*>(rp - ch + p.rsplit) + f8_lo_byte(ch);
              for (int j = 0; j < nv; ++j) v[j] += (float)rp[j] + __builtin_amdgcn_cvt_f32_fp8((int)rb[j], 0) * p.rlo_inv;
            } else {
              for (int j = 0; j < nv; ++j) v[j] += SPLIT && p.rsplit ? (float)rp[j] + (float)rp[p.rsplit + j] : (float)rp[j];
            }
          }
        }
        act8(v);   // the one activation point
        if (has_res && pre_act) {
          if (full) {
            if constexpr (ESZ == 2) {
              if constexpr (SPLIT) {   // hi + lo first: the f32 value of the split residual
                float rl[8];
                if (p.rc8) {
                  f8_unpack8(rq[k], rl);
#pragma unroll
                  for (int j = 0; j < 8; ++j) rl[j] *= p.rlo_inv;
                } else {
#pragma unroll
                  for (int j = 0; j < 8; ++j) rl[j] = (float)rv2[k][0][j];
                }
#pragma unroll
                for (int j = 0; j < 8; ++j) v[j] += (float)rv[k][0][j] + rl[j];
              } else {
#pragma unroll
                for (int j = 0; j < 8; ++j) v[j] += (float)rv[k][0][j];
              }
            } else {
#pragma unroll
              for (int j = 0; j < 4; ++j) { v[j] += rv[k][0][j]; v[4 + j] += rv[k][1][j]; }
            }
          } else {
            long long rpix = pix;
            if (p.res_mode == RES_UP2) rpix = ((long long)n * p.rH + (oh >> 1)) * p.rW + (ow >> 1);
            const T* rp = reinterpret_cast<const T*>(p.res) + rpix * p.rcs + ch;
            if (SPLIT && p.rc8) {
              const unsigned char* rb = reinterpret_cast<const unsigned char*>(rp - ch + p.rsplit) + f8_lo_byte(ch);
              for (int j = 0; j < nv; ++j) v[j] += (float)rp[j] + __builtin_amdgcn_cvt_f32_fp8((int)rb[j], 0) * p.rlo_inv;
            } else {
              for (int j = 0; j < nv; ++j) v[j] += SPLIT && p.rsplit ? (float)rp[j] + (float)rp[p.rsplit + j] : (float)rp[j];
            }
          }
        }
#pragma unroll
        for (int j = 0; j < 8; ++j) v[j] = keep[j] ? v[j] : 0.f;   // channel padding stays exactly zero
        if (p.dbg & 16) continue;   // tuning only: no stores
        if (p.out_f32) {
          float* yp = reinterpret_cast<float*>(p.y) + (long long)pix * p.ycs + ch;
          if (full) {
            *reinterpret_cast<f32x4*>(yp) = f32x4{v[0], v[1], v[2], v[3]};
            *reinterpret_cast<f32x4*>(yp + 4) = f32x4{v[4], v[5], v[6], v[7]};
          } else {
            for (int j = 0; j < nv; ++j) yp[j] = v[j];
          }
        } else {
          T* yp = reinterpret_cast<T*>(p.y) + (long long)pix * p.ycs + ch;
          if constexpr (ESZ == 2) {
            const f16x8 h = f16x8{(f16)v[0], (f16)v[1], (f16)v[2], (f16)v[3], (f16)v[4], (f16)v[5], (f16)v[6], (f16)v[7]};
            if (full) {
              *reinterpret_cast<f16x8*>(yp) = h;
            } else {
              for (int j = 0; j < nv; ++j) yp[j] = h[j];
            }
            if constexpr (SPLIT) {
              if (p.yc8) {   // f16c8 output: lo8 = e4m3((v - hi) * ylo_mul), hi8 = e4m3(hi * yhi_mul)
                float lo[8], hf[8];
#pragma unroll
                for (int j = 0; j < 8; ++j) {
                  hf[j] = (float)h[j];
                  lo[j] = v[j] - hf[j];
                }
                const uint2 ql = f8_pack8(lo, p.ylo_mul), qh = f8_pack8(hf, p.yhi_mul);
                char* fb = reinterpret_cast<char*>(yp - ch + p.ysplit) + f8_lo_byte(ch);
                if (full) {
                  *reinterpret_cast<uint2*>(fb) = ql;
                  *reinterpret_cast<uint2*>(fb + kF8Hi) = qh;
                } else {
                  for (int j = 0; j < nv; ++j) {
                    fb[j] = (char)((j < 4 ? ql.x : ql.y) >> (8 * (j & 3)));
                    fb[kF8Hi + j] = (char)((j < 4 ? qh.x : qh.y) >> (8 * (j & 3)));
                  }
                }
              } else if (p.ysplit) {   // f16x3 output: lo = f16(v - f16(v))
                f16x8 l;
#pragma unroll
                for (int j = 0; j < 8; ++j) l[j] = (f16)(v[j] - (float)h[j]);
                if (full) {
                  *reinterpret_cast<f16x8*>(yp + p.ysplit) = l;
                } else {
                  for (int j = 0; j < nv; ++j) yp[p.ysplit + j] = l[j];
                }
              }
            }
          } else {
            if (full) {
              *reinterpret_cast<f32x4*>(yp) = f32x4{v[0], v[1], v[2], v[3]};
              *reinterpret_cast<f32x4*>(yp + 4) = f32x4{v[4], v[5], v[6], v[7]};
            } else {
              for (int j = 0; j < nv; ++j) yp[j] = v[j];
            }
          }
        }
      }
      }   // residual groups
    }
    if (pass + 1 < NPASS) __syncthreads();
  }
}

}  // namespace pc
