// Fused network stem (gfx950): 3x3 conv over a 3-channel NHWC4 input, one MFMA K step.
//
// The stem's window is 3 x 3 x 3 = 27 values, i.e. one 32-element K row of
// v_mfma_f32_16x16x32_f16. The previous path materialised that row for every output
// pixel in HBM (stem_im2col3: 64 B written + read back per pixel, 6x the algorithmic
// bytes) and then ran a 1x1 conv over it. Here a wave takes 16 consecutive output
// pixels: each lane gathers the nine 4-channel input pixels of its output pixel (8-byte
// loads, L1/L2 resident neighbourhoods), keeps the 8 K values of its lane group
// (fq = lane >> 4: k = 8*fq .. 8*fq+7, k = tap*3 + channel, zero past 27), multiplies
// them against the register-resident [npad][32] weight fragments, and finishes bias +
// activation in registers. The f16 results go through a small per-wave LDS image so that
// every pixel leaves as whole 16-byte chunks of contiguous pixel rows.
//
// Same K positions and the same MFMA as the im2col + 1x1 path, so the results are equal
// to it (the sign of an exact zero aside).
#include "pc_conv_common.h"

namespace pc {

// 16-pixel groups per wave: weights, bias and slopes are loaded once for all of them
constexpr int kStemGroupsPerWave = 4;

// SPLIT (f16x3 detector): the weights are W_hi | W_lo ([npad][64]: K 0-31 hi, 32-63 lo) and the
// input (u8-derived, exact in f16) is multiplied by both, so the f32 accumulator holds x*W to
// ~2^-22; the output is written split (hi = f16(v), lo = f16(v - hi), lo half at +ysplit).
template <int NPAD, bool SPLIT = false>
__global__ __launch_bounds__(256) void stem_fused(StemParams p, const f16* __restrict__ wpk,
                                                   const float* __restrict__ bias, const float* __restrict__ slope,
                                                   int cwrite) {
  constexpr int TC = NPAD / 16;
  constexpr int NS = SPLIT ? 2 : 1;           // halves in the staging image
  constexpr int PITCH = NS * NPAD * 2 + 16;   // padded f16 row of the staging image
  constexpr int CH8 = NPAD / 8;               // 16-byte chunks per pixel and half
  constexpr int KROW = SPLIT ? 64 : 32;       // weight row length
  __shared__ __attribute__((aligned(16))) char stg[4][16 * PITCH];

  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int fr = lane & 15, fq = lane >> 4;
  const int M = p.N * p.OH * p.OW;            // host guarantees M < 2^31
  const int g0 = (blockIdx.x * 4 + wave) * kStemGroupsPerWave;
  if (g0 * 16 >= M) return;   // whole wave (the image is per wave; no workgroup barrier below)

  // weights: A fragment a = rows a*16 + fr, K fq*8 .. fq*8+7; bias / slope of this lane's
  // output channels, all held for the wave's kStemGroupsPerWave pixel groups
  f16x8 wa[TC], wl[SPLIT ? TC : 1];
  float bi[TC][4], sl[TC][4];
#pragma unroll
  for (int a = 0; a < TC; ++a) {
    wa[a] = *reinterpret_cast<const f16x8*>(wpk + (a * 16 + fr) * KROW + fq * 8);
    if constexpr (SPLIT) wl[a] = *reinterpret_cast<const f16x8*>(wpk + (a * 16 + fr) * KROW + 32 + fq * 8);
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      bi[a][j] = bias[a * 16 + fq * 4 + j];
      sl[a][j] = slope ? slope[a * 16 + fq * 4 + j] : 0.f;
    }
  }
  const unsigned hw = (unsigned)(p.OH * p.OW);
  const f16* xs = reinterpret_cast<const f16*>(p.x);
  char* my = stg[wave];
  const int cw8 = cwrite >> 3;   // host guarantees cwrite % 8 == 0

  for (int gi = 0; gi < kStemGroupsPerWave; ++gi) {
    const int q0 = (g0 + gi) * 16;
    if (q0 >= M) break;   // wave-uniform
    // the window of this lane's pixel (rows past M gather zeros and are not stored)
    const int q = q0 + fr;
    const unsigned n = (unsigned)q / hw;
    const unsigned rem = (unsigned)q - n * hw;
    const int oh = (int)(rem / (unsigned)p.OW), ow = (int)(rem - (unsigned)oh * (unsigned)p.OW);
    const f16* xb = xs + (size_t)n * p.H * p.W * p.xcs;
    f16 v[27];
#pragma unroll
    for (int t = 0; t < 9; ++t) {
      const int ih = oh * p.stride - p.pad + t / 3, iw = ow * p.stride - p.pad + t % 3;
      f16x4 e = {};
      if (q < M && (unsigned)ih < (unsigned)p.H && (unsigned)iw < (unsigned)p.W)
        e = *reinterpret_cast<const f16x4*>(xb + ((size_t)ih * p.W + iw) * p.xcs);
      v[3 * t] = e[0];
      v[3 * t + 1] = e[1];
      v[3 * t + 2] = e[2];
    }
    f16x8 b;
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const f16 z = (f16)0.f;
      const f16 g3 = 24 + e < 27 ? v[24 + e] : z;
      b[e] = fq == 0 ? v[e] : (fq == 1 ? v[8 + e] : (fq == 2 ? v[16 + e] : g3));
    }

    // the previous group's staging reads are done before this group's writes
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
#pragma unroll
    for (int a = 0; a < TC; ++a) {
      f32x4 acc = __builtin_amdgcn_mfma_f32_16x16x32_f16(wa[a], b, f32x4{0.f, 0.f, 0.f, 0.f}, 0, 0, 0);
      if constexpr (SPLIT) acc = __builtin_amdgcn_mfma_f32_16x16x32_f16(wl[a], b, acc, 0, 0, 0);
      const int ch = a * 16 + fq * 4;   // output rows of this lane: pixel fr, channels ch .. ch+3
      float o[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        float x = acc[j] + bi[a][j];
        x = act_apply(x, p.act, sl[a][j]);
        o[j] = ch + j < p.cout ? x : 0.f;   // channel padding stays exactly zero
      }
      const f16x4 h = f16x4{(f16)o[0], (f16)o[1], (f16)o[2], (f16)o[3]};
      *reinterpret_cast<f16x4*>(my + fr * PITCH + ch * 2) = h;
      if constexpr (SPLIT) {
        if (p.yc8) {   // f16c8 output: the second half holds [lo8 | hi8] per 32 channels
          const float hf[4] = {(float)h[0], (float)h[1], (float)h[2], (float)h[3]};
          const float lo[4] = {o[0] - hf[0], o[1] - hf[1], o[2] - hf[2], o[3] - hf[3]};
          int wl = __builtin_amdgcn_cvt_pk_fp8_f32(f8_sat(lo[0] * p.ylo_mul), f8_sat(lo[1] * p.ylo_mul), 0, false);
          wl = __builtin_amdgcn_cvt_pk_fp8_f32(f8_sat(lo[2] * p.ylo_mul), f8_sat(lo[3] * p.ylo_mul), wl, true);
          int wh = __builtin_amdgcn_cvt_pk_fp8_f32(f8_sat(hf[0] * p.yhi_mul), f8_sat(hf[1] * p.yhi_mul), 0, false);
          wh = __builtin_amdgcn_cvt_pk_fp8_f32(f8_sat(hf[2] * p.yhi_mul), f8_sat(hf[3] * p.yhi_mul), wh, true);
          *reinterpret_cast<int*>(my + fr * PITCH + NPAD * 2 + f8_lo_byte(ch)) = wl;
          *reinterpret_cast<int*>(my + fr * PITCH + NPAD * 2 + f8_lo_byte(ch) + kF8Hi) = wh;
        } else {
          *reinterpret_cast<f16x4*>(my + fr * PITCH + (NPAD + ch) * 2) =
              f16x4{(f16)(o[0] - (float)h[0]), (f16)(o[1] - (float)h[1]), (f16)(o[2] - (float)h[2]),
                    (f16)(o[3] - (float)h[3])};
        }
      }
    }
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
#pragma unroll
    for (int k = 0; k < (16 * NS * CH8 + 63) / 64; ++k) {
      const int idx = lane + k * 64;
      const int pl = idx / (NS * CH8), cqs = idx - pl * (NS * CH8);
      const int half = cqs >= CH8 ? 1 : 0, cq = cqs - half * CH8;
      if (pl >= 16 || cq >= cw8 || q0 + pl >= M) continue;
      const f16x8 val = *reinterpret_cast<const f16x8*>(my + pl * PITCH + cqs * 16);
      *reinterpret_cast<f16x8*>(reinterpret_cast<f16*>(p.y) + (size_t)(q0 + pl) * p.ycs + half * p.ysplit + cq * 8) =
          val;
    }
  }
}

// can the fused stem run this op? (f16, NHWC4 input with 3 true channels, 3x3 window,
// npad 32 / 64 / 128, whole 16-byte output chunks)
int stem_fused_ok(int f32, int cin, int cin_true, int KH, int KW, int npad, int cwrite, int ycs, int ycoff) {
  return !f32 && cin == 4 && cin_true == 3 && KH == 3 && KW == 3 && (npad == 32 || npad == 64 || npad == 128) &&
         cwrite % 8 == 0 && cwrite <= npad && ycs % 8 == 0 && ycoff % 8 == 0;
}

hipError_t stem_fused_launch(const StemParams& p, const void* wpk, const float* bias, const float* slope, int npad,
                             int cwrite, hipStream_t s) {
  const long long M = (long long)p.N * p.OH * p.OW;
  const long long groups = (M + 15) / 16;
  const long long waves = (groups + kStemGroupsPerWave - 1) / kStemGroupsPerWave;
  const long long nwg = (waves + 3) / 4;
  if (nwg <= 0 || M >= (1LL << 31) - 64 * kStemGroupsPerWave || p.xcs % 4 || (reinterpret_cast<uintptr_t>(p.y) & 15) ||
      (reinterpret_cast<uintptr_t>(p.x) & 7))
    return hipErrorInvalidValue;
  const f16* w = reinterpret_cast<const f16*>(wpk);
  if (p.ysplit) {
    if (p.ysplit % 8) return hipErrorInvalidValue;
    switch (npad) {
      case 32: hipLaunchKernelGGL((stem_fused<32, true>), dim3((unsigned)nwg), dim3(256), 0, s, p, w, bias, slope, cwrite); break;
      case 64: hipLaunchKernelGGL((stem_fused<64, true>), dim3((unsigned)nwg), dim3(256), 0, s, p, w, bias, slope, cwrite); break;
      default: return hipErrorInvalidValue;
    }
    return hipGetLastError();
  }
  switch (npad) {
    case 32: hipLaunchKernelGGL(stem_fused<32>, dim3((unsigned)nwg), dim3(256), 0, s, p, w, bias, slope, cwrite); break;
    case 64: hipLaunchKernelGGL(stem_fused<64>, dim3((unsigned)nwg), dim3(256), 0, s, p, w, bias, slope, cwrite); break;
    case 128: hipLaunchKernelGGL(stem_fused<128>, dim3((unsigned)nwg), dim3(256), 0, s, p, w, bias, slope, cwrite); break;
    default: return hipErrorInvalidValue;
  }
  return hipGetLastError();
}

}  // namespace pc
