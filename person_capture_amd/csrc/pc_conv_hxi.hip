// Image-resident f16x3 3x3 convolution for IResNet's 14x14x256 stage (gfx950): the ArcFace-x3
// layers that were C3's dominant kernel on conv_fast's 256x224 WG tile.
//
// conv_fast stages, per 32-channel K tile, the split pixel rows of one tap: every input pixel moves
// L2 -> LDS nine times (the tile's 224 pixels re-read for each tap), through 4 LDS-DMA pieces per wave
// and a barrier per K tile (1344 MFMA cycles per wave). Here one workgroup owns ONE image - every
// output channel of its 14 x 14 pixels - and stages the image's padded halo once per group of 64 input
// channels (16 x 16 slots + 2, hi and lo: 256-byte slots, 65 KB), in a 2-stage ring: group g + 1 lands
// while group g's 18 k-steps (9 taps x two 32-channel blocks) run; one barrier per group, none inside.
//  * output pixels are enumerated as 14 rows x 16 slots (the halo's pitch), so a tap is one slot
//    offset for every fragment: fragment t = output row t, columns 14 and 15 are discarded (the same
//    12.5 % the 256x224 tile paid in idle CUs at batch 256: 224 of 256 CUs; here every CU has an image);
//  * 8 waves, wave w = output channels 32 w .. 32 w + 31 (two 16-row fragments) x the 14 rows: the
//    weight fragments come from the fragment-ordered copy (pc_api.cpp pack_wfrag) into registers a
//    k-step ahead (double-buffered), the pixel fragments from the halo in two groups of 7 rows;
//  * K order and MFMA order are conv_fast SX / WG's exactly - channel groups of 64 (every tap of a
//    group, the two 32-channel blocks per tap), per k-step W_lo*x_hi, W_hi*x_hi, W_hi*x_lo - and the
//    epilogue arithmetic is conv_epilogue_lds<SPLIT>'s, so the outputs are bit-identical to the fused
//    tiles every other plan class of the net runs (tests/test_gpu_arcface.py);
//  * LDS chunk swizzle: chunk q of slot h holds source chunk q ^ ((h & 7) << 1) - conflict-free
//    ds_read_b128 for 16 consecutive slots at any alignment, hi or lo, either block (checked
//    exhaustively over the instruction's lane groups, MI355X_MICROARCH.md §LDS).
#include "pc_conv_common.h"

namespace pc {

constexpr int HXI_HW = 14;                     // map side
constexpr int HXI_PW = 16;                     // halo pitch: 14 + 2 padding columns
constexpr int HXI_SLOTS = 16 * 16 + 2;         // 16 halo rows + the 2 slots the discarded columns reach
constexpr int HXI_SB = 256;                    // slot: 64 hi + 64 lo f16 channels
constexpr int HXI_PIECES = (HXI_SLOTS * HXI_SB + 1023) / 1024;   // 65 x 1 KiB
constexpr int HXI_STAGE = HXI_PIECES * 1024;

template <int CIN>
__global__ __launch_bounds__(512, 2) void conv_hxi(ConvParams p) {
  constexpr int NW = 8, TC = 2, TP = HXI_HW, TPG = 7, NG = CIN / 64, NKS = NG * 18;
  constexpr int NPIX = HXI_HW * HXI_HW;
  constexpr int RS = 128 + 4;                  // epilogue image row: 128 channels per pass
  constexpr int EPI = NPIX * RS * 4;
  constexpr int SMEM = 2 * HXI_STAGE > EPI ? 2 * HXI_STAGE : EPI;
  static_assert(CIN % 64 == 0 && SMEM <= 163840, "LDS");
  __shared__ __attribute__((aligned(16))) char smem[SMEM];
  const ConvSeg& S = p.seg[0];
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int n = xcd_remap(blockIdx.x, p.N);
  const int fr = lane & 15, kg = lane >> 4;

  auto rsrc = [](const void* base) __attribute__((always_inline)) {
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), (short)0, (int)0xffffffff, 0x00020000);
  };
  const __amdgpu_buffer_rsrc_t xrs = rsrc(S.x);
  const __amdgpu_buffer_rsrc_t wrs = rsrc(p.wfrag);

  // this wave's halo pieces i = wave + 8 j (i < 65): LDS byte i * 1024 + lane * 16 = slot h = 4 i +
  // lane / 16, chunk position q = lane % 16, holding source chunk c = q ^ ((h & 7) << 1): channels
  // 8 (c & 7) .. of the group's hi (c < 8) or lo half; zeros outside the image
  constexpr int PPW = (HXI_PIECES + NW - 1) / NW;
  unsigned src[PPW];
#pragma unroll
  for (int j = 0; j < PPW; ++j) {
    const int h = (wave + NW * j) * 4 + kg, q = fr;
    const int c = q ^ ((h & 7) << 1);
    const int iy = (h >> 4) - 1, ix = (h & 15) - 1;
    const bool ok = h < 256 && (unsigned)iy < (unsigned)HXI_HW && (unsigned)ix < (unsigned)HXI_HW;
    src[j] = ok ? (unsigned)((n * HXI_HW + iy) * HXI_HW + ix) * (unsigned)(S.cs * 2) +
                      (unsigned)(((c & 7) * 8 + (c >> 3) * CIN) * 2)
                : S.zero_off + (unsigned)(q << 4);
  }
  auto stage = [&](int g, int st) __attribute__((always_inline)) {
#pragma unroll
    for (int j = 0; j < PPW; ++j) {
      if (wave + NW * j < HXI_PIECES) {   // (wave-uniform)
        unsigned off = src[j];
        asm volatile("" : "+v"(off));
        // the group's 64 channels ride in the scalar offset (128 bytes per group of each half)
        __builtin_amdgcn_raw_ptr_buffer_load_lds(xrs, (lds_ptr_t)(smem + st * HXI_STAGE + (wave + NW * j) * 1024), 16,
                                                 off, g * 128, 0, 0);
      }
    }
  };
  // weight fragments of k-step s (packed K tile s: group s / 18, tap (s % 18) / 2, block s % 2): row
  // blocks 2 wave, 2 wave + 1 of npad / 16, each [W_hi, W_lo] x 1 KiB
  const int tile = (p.npad / 16) * 2048;
  auto wload = [&](f16x8* wh, f16x8* wl, int s) __attribute__((always_inline)) {
#pragma unroll
    for (int a = 0; a < TC; ++a) {
      const int o = ((2 * wave + a) * 2) * 1024 + lane * 16;
      wh[a] = __builtin_bit_cast(f16x8, __builtin_amdgcn_raw_buffer_load_b128(wrs, o, s * tile, 0));
      wl[a] = __builtin_bit_cast(f16x8, __builtin_amdgcn_raw_buffer_load_b128(wrs, o + 1024, s * tile, 0));
    }
  };
  f16x8 wbh[2][TC], wbl[2][TC];
  stage(0, 0);
  wload(wbh[0], wbl[0], 0);

  f32x4 acc[TC][TP];
#pragma unroll
  for (int a = 0; a < TC; ++a)
#pragma unroll
    for (int t = 0; t < TP; ++t) acc[a][t] = f32x4{0.f, 0.f, 0.f, 0.f};
  if (p.dbg & 8) return;   // tuning only (PC_CONV_DBG): prologue only

  // per-lane LDS byte of (tap column dx, chunk kind) for fragment row 0, tap row 0: slot fr + dx
  auto boff = [&](int dx, int chunk) __attribute__((always_inline)) {
    const int h = fr + dx;
    return (unsigned)(h * HXI_SB + ((chunk ^ ((h & 7) << 1)) << 4));
  };
  static_for<NG>([&](auto gc) __attribute__((always_inline)) {
    constexpr int g = decltype(gc)::value, st = g & 1;
    // group g's halo: every VMEM op but the youngest 2 TC (the next k-step's weights) has landed
    asm volatile("s_waitcnt vmcnt(%0)" ::"n"(2 * TC) : "memory");
    __syncthreads();   // every wave's pieces of group g; every wave done reading group g - 1's stage
    if constexpr (g + 1 < NG) stage(g + 1, st ^ 1);
    const char* base = smem + st * HXI_STAGE;
    static_for<18>([&](auto kc) __attribute__((always_inline)) {
      constexpr int k = decltype(kc)::value, tap = k / 2, blk = k % 2, s = g * 18 + k, q = s & 1;
      constexpr int dy = tap / 3, dx = tap % 3;
      if constexpr (s + 1 < NKS) wload(wbh[q ^ 1], wbl[q ^ 1], s + 1);
      const unsigned oh = boff(dx, blk * 4 + kg), ol = boff(dx, 8 + blk * 4 + kg);
      if (p.dbg & 2) return;   // tuning only: no MFMAs
      static_for<TP / TPG>([&](auto pc) __attribute__((always_inline)) {
        constexpr int t0 = decltype(pc)::value * TPG;
        f16x8 bh[TPG], bl[TPG];
#pragma unroll
        for (int t = 0; t < TPG; ++t)
          bh[t] = *reinterpret_cast<const f16x8*>(base + oh + (t0 + t + dy) * HXI_PW * HXI_SB);
#pragma unroll
        for (int a = 0; a < TC; ++a)
#pragma unroll
          for (int t = 0; t < TPG; ++t)
            acc[a][t0 + t] = __builtin_amdgcn_mfma_f32_16x16x32_f16(wbl[q][a], bh[t], acc[a][t0 + t], 0, 0, 0);
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int t = 0; t < TPG; ++t)
          bl[t] = *reinterpret_cast<const f16x8*>(base + ol + (t0 + t + dy) * HXI_PW * HXI_SB);
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int a = 0; a < TC; ++a)
#pragma unroll
          for (int t = 0; t < TPG; ++t)
            acc[a][t0 + t] = __builtin_amdgcn_mfma_f32_16x16x32_f16(wbh[q][a], bh[t], acc[a][t0 + t], 0, 0, 0);
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int a = 0; a < TC; ++a)
#pragma unroll
          for (int t = 0; t < TPG; ++t)
            acc[a][t0 + t] = __builtin_amdgcn_mfma_f32_16x16x32_f16(wbh[q][a], bl[t], acc[a][t0 + t], 0, 0, 0);
        __builtin_amdgcn_sched_barrier(0);
      });
    });
  });
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  if (p.dbg & 4) return;   // tuning only: no epilogue

  // ---- epilogue in two passes of 128 channels (waves 0-3, then 4-7, write their accumulators into
  // an f32 [pixel][channel] image over the LDS; then every thread finishes 8 channels of one pixel
  // per step with conv_epilogue_lds<SPLIT>'s arithmetic: bias (per channel, then the border class),
  // residual hi + lo before or after the activation select, channel keep mask, hi / lo stores) ----
  float* im = reinterpret_cast<float*>(smem);
  const bool smooth = p.act == ACT_SILU || p.act == ACT_GELU;
  const bool has_res = p.res_mode != RES_NONE;
  const bool pre_act = !p.act_after_res;
#pragma unroll
  for (int pass = 0; pass < 2; ++pass) {
    __syncthreads();   // the stages (pass 0) / the previous pass's image are no longer read
    if (wave / 4 == pass) {
#pragma unroll
      for (int a = 0; a < TC; ++a)
#pragma unroll
        for (int t = 0; t < TP; ++t) {
          if (fr < HXI_HW) {
            const int pl = t * HXI_HW + fr;
            *reinterpret_cast<f32x4*>(im + pl * RS + (wave & 3) * 32 + a * 16 + kg * 4) = acc[a][t];
          }
        }
    }
    __syncthreads();
    for (int it = threadIdx.x; it < NPIX * 16; it += 512) {
      const int pl = it >> 4, cl = (it & 15) * 8, ch = pass * 128 + cl;
      const int oy = pl / HXI_HW, ox = pl - oy * HXI_HW;
      const long long pix = (long long)n * NPIX + pl;
      const f32x4 lo4 = *reinterpret_cast<const f32x4*>(im + pl * RS + cl);
      const f32x4 hi4 = *reinterpret_cast<const f32x4*>(im + pl * RS + cl + 4);
      float v[8] = {lo4[0], lo4[1], lo4[2], lo4[3], hi4[0], hi4[1], hi4[2], hi4[3]};
      if (p.bias_mode == BIAS_CHANNEL) {
#pragma unroll
        for (int j = 0; j < 8; ++j) v[j] += p.bias[ch + j];
      } else {
#pragma unroll
        for (int j = 0; j < 8; ++j) v[j] += 0.f;   // (conv_epilogue_lds adds a zero channel bias first)
        if (p.bias_mode == BIAS_BORDER9) {
          const int rc = oy - 1 < 0 ? 0 : (oy + 1 >= HXI_HW ? 2 : 1);
          const int cc = ox - 1 < 0 ? 0 : (ox + 1 >= HXI_HW ? 2 : 1);
          const float* bp = p.bias + (rc * 3 + cc) * p.npad + ch;
#pragma unroll
          for (int j = 0; j < 8; ++j) v[j] += bp[j];
        }
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
        for (int j = 0; j < 8; ++j) {
          const float sl = p.act == ACT_PRELU ? p.slope[ch + j] : (p.act == ACT_RELU ? 0.f : 1.f);
          v[j] = v[j] > 0.f ? v[j] : v[j] * sl;
        }
      }
      if (has_res && pre_act) {
#pragma unroll
        for (int j = 0; j < 8; ++j) v[j] += r[j];
      }
      f16x8 yh, yl;
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const float x = ch + j < p.cout ? v[j] : 0.f;
        yh[j] = (f16)x;
        yl[j] = (f16)(x - (float)yh[j]);
      }
      f16* yp = reinterpret_cast<f16*>(p.y) + pix * p.ycs + ch;
      *reinterpret_cast<f16x8*>(yp) = yh;
      *reinterpret_cast<f16x8*>(yp + p.ysplit) = yl;
    }
  }
}

// can a conv run here: one 14x14 split segment of 256 channels (X.C 512 = [hi | lo], dense), 256
// output channels written split (dense), 3x3 stride 1 pad 1, plain or same-size split residual
int conv_hxi_ok(const ConvParams& p) {
  const ConvSeg& S = p.seg[0];
  return p.nseg == 1 && S.C == 512 && S.cs == 512 && S.H == HXI_HW && S.W == HXI_HW && S.KH == 3 && S.KW == 3 &&
         S.stride == 1 && S.pad == 1 && p.OH == HXI_HW && p.OW == HXI_HW && p.npad == 256 && p.ysplit == 256 &&
         p.ycs == 512 && p.splitk == 1 && !p.out_f32 && !p.yc8 && !p.rc8 && p.ktot == 9 * 768 &&
         p.res_mode != RES_UP2 && (p.res_mode == RES_NONE || (p.rsplit == 256 && p.rcs % 8 == 0)) &&
         p.cwrite == 256 && p.wfrag != nullptr;
}

hipError_t conv_hxi_launch(const ConvParams& p, hipStream_t s) {
  if (!conv_hxi_ok(p)) return hipErrorInvalidValue;
  hipLaunchKernelGGL(conv_hxi<256>, dim3(p.N), dim3(512), 0, s, p);
  return hipGetLastError();
}

}  // namespace pc
