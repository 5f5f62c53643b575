// Halo-staged f16x3 3x3 convolution for 64 -> 64 channel split layers (gfx950): SCRFD's
// 160x160x64 / 80x80x64 / 40x40x64 trunk in the f16x3 detector.
//
// The fused split tiles of conv_fast stage, per K tile, the hi and lo pixel rows of one tap:
// every input pixel moves L2 -> LDS nine times, 64 KB of the 80 KB a 64x256 tile stages per
// tap, at the 15-30 B/clk per CU an L2 -> LDS fill sustains (round 4: 15-18 % MFMA busy).
// Here a workgroup owns a 16x16 output block of one image: it stages the block's 18x18
// input halo (hi and lo, 256 B per pixel, 83 KB) into LDS once, and each of its four waves
// walks the 9 taps x 2 k-steps for 4 output rows x 16 pixels x 64 channels, reading pixel
// fragments from the halo (tap shifts are slot offsets) and W_hi / W_lo fragments from a
// 3-tap LDS ring filled by LDS-DMA two taps ahead. Per k-step and fragment the MFMAs are conv_fast SX's:
// W_hi*x_hi, W_lo*x_hi, W_hi*x_lo, k-steps in (tap row, tap column, 32-channel block) order.
#include "pc_conv_common.h"

namespace pc {

constexpr int HX_TW = 16, HX_TH = 16, HX_PW = HX_TW + 2, HX_SLOTS = (HX_TH + 2) * HX_PW;
constexpr int HX_SB = 256;                        // slot bytes: 64 hi + 64 lo f16 channels
constexpr int HX_BYTES = HX_SLOTS * HX_SB;        // 82944 = 81 x 1 KiB

__global__ __launch_bounds__(256, 1) void conv_hx64(ConvParams p, int nby, int nbx) {
  constexpr int TC = 4, TP = 4, NKS = 18;         // 64 channels, 4 rows per wave, 9 taps x 2 k-steps
  __shared__ __attribute__((aligned(16))) char halo[HX_BYTES];
  __shared__ __attribute__((aligned(16))) char wring[3 * 16384];   // W_hi | W_lo of three taps
  const ConvSeg& S = p.seg[0];
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int nblk = p.N * nby * nbx;
  const int b = xcd_remap(blockIdx.x, nblk);
  const int n = b / (nby * nbx), rem = b - n * (nby * nbx);
  const int oy0 = (rem / nbx) * HX_TH, ox0 = (rem - (rem / nbx) * nbx) * HX_TW;
  const int H = S.H, W = S.W;
  const int fr = lane & 15, g = lane >> 4;

  auto rsrc = [](const void* base) __attribute__((always_inline)) {
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), (short)0, (int)0xffffffff, 0x00020000);
  };
  const __amdgpu_buffer_rsrc_t xrs = rsrc(S.x);
  const __amdgpu_buffer_rsrc_t wrs = rsrc(p.w);

  // ---- halo: LDS byte i*1024 + lane*16 = slot s, chunk position q, holding source chunk
  // q ^ (s & 15) of input pixel (oy0 - 1 + s / 18, ox0 - 1 + s % 18); zeros outside ----
  for (int i = wave; i < HX_BYTES / 1024; i += 4) {
    const int bb = i * 1024 + lane * 16;
    const int s = bb >> 8, q = (bb >> 4) & 15;
    const int iy = oy0 - 1 + s / HX_PW, ix = ox0 - 1 + (s - (s / HX_PW) * HX_PW);
    const bool ok = (unsigned)iy < (unsigned)H && (unsigned)ix < (unsigned)W;
    // unsigned byte offset: the pixel index fits 31 bits, its byte offset only 32 (the planner
    // keeps every activation buffer below 4 GiB); signed int arithmetic would overflow past 2 GiB
    unsigned off = ok ? (unsigned)((n * H + iy) * W + ix) * (unsigned)(S.cs * 2) + (unsigned)((q ^ (s & 15)) << 4)
                      : S.zero_off;
    asm volatile("" : "+v"(off));
    __builtin_amdgcn_raw_ptr_buffer_load_lds(xrs, (lds_ptr_t)(halo + i * 1024), 16, off, 0, 0, 0);
  }

  // weights: per tap, W_hi and W_lo (64 rows of 128 B each, from the [W_hi, W_hi, W_lo]-per-tap
  // layout, 192 per tap) through a 3-slot LDS ring by LDS-DMA, two taps ahead - register loads
  // of the same fragments by every workgroup at once ran at ~2 us per k-step (r04)
  const int lrow = lane >> 3, lch = lane & 7;
  auto issue_w = [&](int tap, int slot) __attribute__((always_inline)) {
    // 16 pieces of 8 rows: pieces 0-7 W_hi rows, 8-15 W_lo rows; wave w issues pieces w, w+4, ...
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int pc = wave + 4 * j;
      const int half = pc >> 3, r = (pc & 7) * 8 + lrow;   // r: output channel row
      unsigned off = (unsigned)((long long)r * p.ktot * 2) + (unsigned)(tap * 192 + half * 128) * 2 +
                     ((lch ^ ((r >> 1) & 7)) << 4);
      asm volatile("" : "+v"(off));
      __builtin_amdgcn_raw_ptr_buffer_load_lds(wrs, (lds_ptr_t)(wring + slot * 16384 + pc * 1024), 16, off, 0, 0, 0);
    }
  };
  issue_w(0, 0);
  issue_w(1, 1);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // halo and the first two taps' weights
  __syncthreads();
  if (p.dbg & 8) return;   // tuning only (PC_CONV_DBG): staging only

  f32x4 acc[TC][TP];
#pragma unroll
  for (int a = 0; a < TC; ++a)
#pragma unroll
    for (int t = 0; t < TP; ++t) acc[a][t] = f32x4{0.f, 0.f, 0.f, 0.f};
  // the halo slot of fragment row t's pixel at tap (0, 0)
  int bslot[TP];
#pragma unroll
  for (int t = 0; t < TP; ++t) bslot[t] = (wave * TP + t) * HX_PW + fr;
  const int arow_sw = (fr >> 1) & 7;   // row a*16 + fr: the swizzle depends on fr only

  static_for<9>([&](auto tc) __attribute__((always_inline)) {
    constexpr int tap = decltype(tc)::value;
    constexpr int toff = (tap / 3) * HX_PW + (tap % 3);
    if constexpr (tap > 0) {
      // tap's weights (issued two taps ago) landed: at most one tap's pieces still in flight
      if constexpr (tap < 8) asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
      else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
    }
    if constexpr (tap + 2 < 9) {
      if (!(p.dbg & 1)) issue_w(tap + 2, (tap + 2) % 3);   // dbg 1: no weight stream (tuning only)
    }
    const char* ws = wring + (tap % 3) * 16384;
    static_for<2>([&](auto kc) __attribute__((always_inline)) {
      constexpr int ks = decltype(kc)::value;
      f16x8 wh[TC], wl[TC], bh[TP], bl[TP];
      const unsigned ach = (unsigned)(((ks * 4 + g) ^ arow_sw) << 4);
#pragma unroll
      for (int a = 0; a < TC; ++a) {
        wh[a] = *reinterpret_cast<const f16x8*>(ws + (a * 16 + fr) * 128 + ach);
        wl[a] = *reinterpret_cast<const f16x8*>(ws + 8192 + (a * 16 + fr) * 128 + ach);
      }
#pragma unroll
      for (int t = 0; t < TP; ++t) {
        const int s = bslot[t] + toff;
        const int sw = s & 15;
        bh[t] = *reinterpret_cast<const f16x8*>(halo + s * HX_SB + (((ks * 4 + g) ^ sw) << 4));
        bl[t] = *reinterpret_cast<const f16x8*>(halo + s * HX_SB + (((8 + ks * 4 + g) ^ sw) << 4));
      }
      if (p.dbg & 2) return;   // tuning only: no MFMAs
#pragma unroll
      for (int a = 0; a < TC; ++a)
#pragma unroll
        for (int t = 0; t < TP; ++t)
          acc[a][t] = __builtin_amdgcn_mfma_f32_16x16x32_f16(wh[a], bh[t], acc[a][t], 0, 0, 0);
#pragma unroll
      for (int a = 0; a < TC; ++a)
#pragma unroll
        for (int t = 0; t < TP; ++t)
          acc[a][t] = __builtin_amdgcn_mfma_f32_16x16x32_f16(wl[a], bh[t], acc[a][t], 0, 0, 0);
#pragma unroll
      for (int a = 0; a < TC; ++a)
#pragma unroll
        for (int t = 0; t < TP; ++t)
          acc[a][t] = __builtin_amdgcn_mfma_f32_16x16x32_f16(wh[a], bl[t], acc[a][t], 0, 0, 0);
    });
  });
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");

  if (p.dbg & 4) return;   // tuning only: no epilogue
  // ---- epilogue through LDS: the per-fragment form (8-byte stores at a 256-byte pixel
  // stride) took 60 % of the kernel (r04hxd). The accumulators go to a [pixel][channel] f32
  // image over the halo; then every thread finishes 8 channels of a pixel - bias (per channel
  // or border class), the activation select, split residual hi + lo - and stores the hi and
  // lo halves as one 16-byte vector each (conv_epilogue_lds's arithmetic) ----
  constexpr int RS = 68;                 // padded image row (floats)
  __syncthreads();                       // every wave is done with the halo
  float* im = reinterpret_cast<float*>(halo);
#pragma unroll
  for (int a = 0; a < TC; ++a)
#pragma unroll
    for (int t = 0; t < TP; ++t) {
      const int pl = (wave * TP + t) * HX_TW + fr;   // block pixel (row-major 16x16)
      *reinterpret_cast<f32x4*>(im + pl * RS + a * 16 + g * 4) = acc[a][t];
    }
  __syncthreads();
  const int OW = p.OW, OH = p.OH;
  const int cg = threadIdx.x & 7, ch = cg * 8;
  float bc[8], sl[8];
  bool keep[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    bc[j] = p.bias_mode == BIAS_CHANNEL ? p.bias[ch + j] : 0.f;
    sl[j] = p.act == ACT_PRELU ? p.slope[ch + j] : (p.act == ACT_RELU ? 0.f : 1.f);
    keep[j] = ch + j < p.cout;
  }
  const bool smooth = p.act == ACT_SILU || p.act == ACT_GELU;
  const bool has_res = p.res_mode != RES_NONE;
  const bool pre_act = !p.act_after_res;
  for (int pl = threadIdx.x >> 3; pl < HX_TH * HX_TW; pl += 32) {
    const int oy = oy0 + (pl >> 4), ox = ox0 + (pl & 15);
    if (oy >= OH || ox >= OW) continue;
    const long long pix = ((long long)n * OH + oy) * OW + ox;
    const f32x4 lo4 = *reinterpret_cast<const f32x4*>(im + pl * RS + ch);
    const f32x4 hi4 = *reinterpret_cast<const f32x4*>(im + pl * RS + ch + 4);
    float v[8] = {lo4[0] + bc[0], lo4[1] + bc[1], lo4[2] + bc[2], lo4[3] + bc[3],
                  hi4[0] + bc[4], hi4[1] + bc[5], hi4[2] + bc[6], hi4[3] + bc[7]};
    if (p.bias_mode == BIAS_BORDER9) {
      const int rc = oy - 1 < 0 ? 0 : (oy + 1 >= H ? 2 : 1);
      const int cc = ox - 1 < 0 ? 0 : (ox + 1 >= W ? 2 : 1);
      const float* bp = p.bias + (rc * 3 + cc) * p.npad + ch;
#pragma unroll
      for (int j = 0; j < 8; ++j) v[j] += bp[j];
    }
    float r[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    if (has_res) {
      const f16* rp = reinterpret_cast<const f16*>(p.res) + pix * p.rcs + ch;
      const f16x8 rh = *reinterpret_cast<const f16x8*>(rp);
      const f16x8 rl = *reinterpret_cast<const f16x8*>(rp + p.rsplit);
#pragma unroll
      for (int j = 0; j < 8; ++j) r[j] = (float)rh[j] + (float)rl[j];
    }
    if (has_res && !pre_act) {
#pragma unroll
      for (int j = 0; j < 8; ++j) v[j] += r[j];
    }
    if (smooth) {
#pragma unroll
      for (int j = 0; j < 8; ++j) v[j] = act_apply(v[j], p.act, 0.f);
    } else {
#pragma unroll
      for (int j = 0; j < 8; ++j) v[j] = v[j] > 0.f ? v[j] : v[j] * sl[j];
    }
    if (has_res && pre_act) {
#pragma unroll
      for (int j = 0; j < 8; ++j) v[j] += r[j];
    }
    f16x8 yh, yl;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const float x = keep[j] ? v[j] : 0.f;
      yh[j] = (f16)x;
      yl[j] = (f16)(x - (float)yh[j]);
    }
    f16* yp = reinterpret_cast<f16*>(p.y) + pix * p.ycs + ch;
    *reinterpret_cast<f16x8*>(yp) = yh;
    *reinterpret_cast<f16x8*>(yp + p.ysplit) = yl;
  }
}

// can a conv run here: split 64-channel input (X.C 128 = [hi | lo]), 64 output channels
// written split, 3x3 stride 1 pad 1, same size
int conv_hx_ok(const ConvParams& p) {
  const ConvSeg& S = p.seg[0];
  return p.nseg == 1 && S.C == 128 && S.KH == 3 && S.KW == 3 && S.stride == 1 && S.pad == 1 &&
         S.H == p.OH && S.W == p.OW && p.npad == 64 && p.ysplit == 64 && p.splitk == 1 && !p.out_f32 &&
         p.ktot == 9 * 192 && p.res_mode != RES_UP2 && (p.res_mode == RES_NONE || (p.rsplit == 64 && p.rcs % 8 == 0)) &&
         p.ycs % 8 == 0 && p.cwrite == 64;
}

hipError_t conv_hx_launch(const ConvParams& p, hipStream_t s) {
  if (!conv_hx_ok(p)) return hipErrorInvalidValue;
  const int nby = (p.OH + HX_TH - 1) / HX_TH, nbx = (p.OW + HX_TW - 1) / HX_TW;
  hipLaunchKernelGGL(conv_hx64, dim3(p.N * nby * nbx), dim3(256), 0, s, p, nby, nbx);
  return hipGetLastError();
}

}  // namespace pc
