// Halo-staged f16x3 3x3 convolution for 64 -> 64 channel split layers (gfx950): SCRFD's
// 160x160x64 / 80x80x64 / 40x40x64 trunk in the f16x3 detector and IResNet's 56x56x64 /
// 112x112x64 stage in the f16x3 ArcFace.
//
// The fused split tiles of conv_fast stage, per K tile, the hi and lo pixel rows of one tap:
// every input pixel moves L2 -> LDS nine times. Here a workgroup owns a 16x12 output block of one
// image: it stages the block's 18x14 input halo (hi and lo, 256 B per pixel, 63 KB) into LDS once,
// and each of its four waves walks the 9 taps x 2 k-steps for 3 output rows x 16 pixels x 64
// channels, reading pixel fragments from the halo (tap shifts are slot offsets). The W_hi / W_lo
// fragments come from the conv's fragment-ordered weight copy (pc_api.cpp pack_wfrag) straight into
// registers, one k-step ahead: the K loop has no barrier, and two workgroups share a CU (round 4's
// form staged 16x16 blocks and a 3-tap weight ring through the LDS, 131 KB: one workgroup per CU).
// Per k-step and fragment the MFMAs are W_lo*x_hi, W_hi*x_hi, W_hi*x_lo, k-steps in (tap row, tap
// column, 32-channel block) order: for 64 input channels (one channel group of 64) that is conv_fast
// SX's accumulation order, pass order included (round 6; round 5 issued W_hi*x_hi first), and the
// epilogue arithmetic is conv_epilogue_lds<SPLIT>'s - so a plan class may run these layers here or on
// the fused tiles and small and large batches stay bit-identical (pc_api.cpp plan_conv takes this
// kernel where its grid fills the CUs; tests/test_gpu_plan_classes.py).
#include "pc_conv_common.h"

#include <cstdlib>

namespace pc {

constexpr int HX_TW = 16, HX_TH = 12, HX_PW = HX_TW + 2, HX_SLOTS = (HX_TH + 2) * HX_PW;
constexpr int HX_SB = 256;                        // slot bytes: 64 hi + 64 lo f16 channels
constexpr int HX_BYTES = HX_SLOTS * HX_SB;        // 64512 = 63 x 1 KiB
static_assert(HX_BYTES % 1024 == 0, "halo DMA pieces");
static_assert(HX_TH * HX_TW * 68 * 4 <= HX_BYTES, "epilogue image over the halo");
static_assert(HX_TH * HX_TW % 32 == 0, "epilogue: 32 pixels per round of 8-channel groups");

// WLDS: each k-step's weight tile (8 KB) comes into the LDS once per workgroup by LDS-DMA (a 2-slot ring
// after the halo, 79 KB per workgroup: still two per CU) and the four waves read their fragments from
// there, instead of every wave loading all 8 fragments from L2 into registers (8 KB per wave and k-step
// through the TA / TD return path, which the 8 waves of a CU share with the halo DMA). Same fragments,
// same MFMA order: the same bits.
template <bool WLDS>
__global__ __launch_bounds__(256, 2) void conv_hx64(ConvParams p, int nby, int nbx) {
  constexpr int TC = 4, TP = HX_TH / 4, NKS = 18;   // 64 channels, 3 rows per wave, 9 taps x 2 k-steps
  constexpr int WT = 8192;                          // packed weight bytes per k-step
  __shared__ __attribute__((aligned(16))) char halo[HX_BYTES + (WLDS ? 2 * WT : 0)];
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
  const __amdgpu_buffer_rsrc_t wrs = rsrc(p.wfrag);

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

  // weight fragments of k-step s (tap s / 2, channel block s % 2): packed K tile s (the fused tiles'
  // channel-group order: one group of 64 channels, every tap, its two 32-channel blocks per tap),
  // 4 row blocks x [W_hi, W_lo] x 1 KiB (lane l: row 16 a + (l & 15), channels 8 (l >> 4) .. +8)
  auto wload = [&](f16x8* wh, f16x8* wl, int s) __attribute__((always_inline)) {
    const int kt = s;
#pragma unroll
    for (int a = 0; a < TC; ++a) {
      wh[a] = __builtin_bit_cast(f16x8, __builtin_amdgcn_raw_buffer_load_b128(wrs, lane * 16 + (a * 2) * 1024, kt * 8192, 0));
      wl[a] = __builtin_bit_cast(f16x8, __builtin_amdgcn_raw_buffer_load_b128(wrs, lane * 16 + (a * 2 + 1) * 1024, kt * 8192, 0));
    }
  };
  // WLDS: k-step s's weight tile into ring slot: pieces 2 wave + j (1 KiB each) of the packed tile
  auto wdma = [&](int s, int slot) __attribute__((always_inline)) {
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int piece = wave * 2 + j;
      __builtin_amdgcn_raw_ptr_buffer_load_lds(wrs, (lds_ptr_t)(halo + HX_BYTES + slot * WT + piece * 1024), 16,
                                               piece * 1024 + lane * 16, s * WT, 0, 0);
    }
  };
  f16x8 wbh[WLDS ? 1 : 2][TC], wbl[WLDS ? 1 : 2][TC];
  if constexpr (WLDS) wdma(0, 0);
  else wload(wbh[0], wbl[0], 0);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // the halo (and k-step 0's weights)
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

  static_for<NKS>([&](auto sc) __attribute__((always_inline)) {
    constexpr int s = decltype(sc)::value, tap = s / 2, ks = s % 2;
    constexpr int q = WLDS ? 0 : (s & 1);
    constexpr int toff = (tap / 3) * HX_PW + (tap % 3);
    if constexpr (WLDS) {
      if constexpr (s > 0) {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // this wave's pieces of k-step s's tile
        __builtin_amdgcn_s_barrier();                      // every wave's pieces; every wave done with slot s - 1
      }
      // the fragment reads go out before the next tile's DMA, so nothing has to wait for it
      const char* wt = halo + HX_BYTES + (s & 1) * WT + lane * 16;
#pragma unroll
      for (int a = 0; a < TC; ++a) {
        wbh[0][a] = *reinterpret_cast<const f16x8*>(wt + (a * 2) * 1024);
        wbl[0][a] = *reinterpret_cast<const f16x8*>(wt + (a * 2 + 1) * 1024);
      }
    } else if constexpr (s + 1 < NKS) {
      wload(wbh[q ^ 1], wbl[q ^ 1], s + 1);
    }
    f16x8 bh[TP], bl[TP];
#pragma unroll
    for (int t = 0; t < TP; ++t) {
      const int sl = bslot[t] + toff;
      const int sw = sl & 15;
      bh[t] = *reinterpret_cast<const f16x8*>(halo + sl * HX_SB + (((ks * 4 + g) ^ sw) << 4));
      bl[t] = *reinterpret_cast<const f16x8*>(halo + sl * HX_SB + (((8 + ks * 4 + g) ^ sw) << 4));
    }
    if constexpr (WLDS && s + 1 < NKS) wdma(s + 1, (s + 1) & 1);
    if (p.dbg & 2) return;   // tuning only: no MFMAs
#pragma unroll
    for (int a = 0; a < TC; ++a)
#pragma unroll
      for (int t = 0; t < TP; ++t)
        acc[a][t] = __builtin_amdgcn_mfma_f32_16x16x32_f16(wbl[q][a], bh[t], acc[a][t], 0, 0, 0);
#pragma unroll
    for (int a = 0; a < TC; ++a)
#pragma unroll
      for (int t = 0; t < TP; ++t)
        acc[a][t] = __builtin_amdgcn_mfma_f32_16x16x32_f16(wbh[q][a], bh[t], acc[a][t], 0, 0, 0);
#pragma unroll
    for (int a = 0; a < TC; ++a)
#pragma unroll
      for (int t = 0; t < TP; ++t)
        acc[a][t] = __builtin_amdgcn_mfma_f32_16x16x32_f16(wbh[q][a], bl[t], acc[a][t], 0, 0, 0);
  });
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");

  if (p.dbg & 4) return;   // tuning only: no epilogue
  // ---- epilogue through LDS: the per-fragment form (8-byte stores at a 256-byte pixel
  // stride) took 60 % of the kernel (r04hxd). The accumulators go to a [pixel][channel] f32
  // image over the halo; then every thread finishes 8 channels of a pixel - bias (per channel
  // or border class), the activation select, split residual hi + lo - and stores the hi and
  // lo halves as one 16-byte vector each (conv_epilogue_lds's arithmetic) ----
  constexpr int RS = 68;                 // padded image row (floats)
  // a thread keeps one 8-channel group for NIT pixels; their residual rows are requested first, so
  // the loads run under the image transposition (loaded per pixel, the epilogue took 89 of 232 us on
  // 160x160x64, profiles/r06ad_hx_phase_split.txt)
  constexpr int NIT = HX_TH * HX_TW / 32;
  const int OW = p.OW, OH = p.OH;
  const int cg = threadIdx.x & 7, ch = cg * 8;
  const bool has_res = p.res_mode != RES_NONE;
  f16x8 rh[NIT], rl[NIT];
#pragma unroll
  for (int k = 0; k < NIT; ++k) {
    rh[k] = f16x8{};
    rl[k] = f16x8{};
    const int pl = (threadIdx.x >> 3) + 32 * k;
    const int oy = oy0 + (pl >> 4), ox = ox0 + (pl & 15);
    if (has_res && oy < OH && ox < OW) {
      const f16* rp = reinterpret_cast<const f16*>(p.res) + (((long long)n * OH + oy) * OW + ox) * p.rcs + ch;
      rh[k] = *reinterpret_cast<const f16x8*>(rp);
      rl[k] = *reinterpret_cast<const f16x8*>(rp + p.rsplit);
    }
  }
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
  float bc[8], sl[8];
  bool keep[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    bc[j] = p.bias_mode == BIAS_CHANNEL ? p.bias[ch + j] : 0.f;
    sl[j] = p.act == ACT_PRELU ? p.slope[ch + j] : (p.act == ACT_RELU ? 0.f : 1.f);
    keep[j] = ch + j < p.cout;
  }
  const bool smooth = p.act == ACT_SILU || p.act == ACT_GELU;
  const bool pre_act = !p.act_after_res;
#pragma unroll
  for (int k = 0; k < NIT; ++k) {
    const int pl = (threadIdx.x >> 3) + 32 * k;
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
    float r[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) r[j] = (float)rh[k][j] + (float)rl[k][j];
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

// ---------------------------------------------------------------------------------------------
// conv_hxg<CIN, COUT, TP>: the halo-staged f16x3 3x3 conv for wider channel counts - SCRFD's
// 80x80x96 / 40x40x96 / 20x20x96 trunk (CIN = COUT = 96: 29 % of SCRFD-10G's FLOPs, 131 TF/s on the
// fused 32x256 tile). Where conv_hx64 stages all 64 input channels of a 16x12 block at
// once (63 KB, two workgroups and 8 waves per CU) and every wave loads all 64 output channels' weight
// fragments from L2 for 3 output rows (8 fragment loads per 36 MFMAs: the TA / TD return path, not the
// matrix pipe, is its limit), this kernel runs ONE workgroup of 4 waves per CU, one wave per SIMD with
// up to 512 registers, so each wave owns every output channel of TP output rows (6 x TP fragments):
// 12 weight fragment loads per 18 TP MFMAs (0.13 per MFMA at TP 5, against 0.22).
//  * the block is 16 x 4 TP output pixels of one image; its (4 TP + 2) x 18 input halo is staged per
//    group of 32 input channels (hi and lo: 128-byte slots, 16-byte chunk q of slot s holding source
//    chunk q ^ (s & 7) - conflict-free ds_read_b128 for any 16 consecutive slots) in a 2-stage ring:
//    group g + 1's LDS-DMA is issued right after the barrier that opens group g, so it lands while
//    group g's 9 taps run; one barrier per group, none inside it;
//  * K walks (32-channel group, tap row, tap column) - the packed fragment copy's order for channel
//    counts that are not a multiple of 64 (pc_api.cpp pack_wfrag, gt 1), which is conv_fast SX's K order
//    there - with the weight fragments of the next k-step loaded into registers under the current one;
//    per k-step and fragment the MFMAs are SX's: W_lo*x_hi, W_hi*x_hi, W_hi*x_lo (so a plan class may
//    take the fused tiles instead: same accumulators);
//  * epilogue: conv_hx64's (f32 image over the LDS, 16-byte hi and lo stores per pixel and 8 channels).
// Small-batch form (CO < COUT, a single frame's 80x80 / 40x40 maps, whose 16x20 blocks are a few dozen):
// a workgroup computes CO of the output channels of a 16 x 4 TP block - COUT / CO workgroups per block,
// each staging the block's halo - at several workgroups per CU (WPE waves per SIMD). Same K order, MFMA
// order and epilogue per output: the same bits.
template <int CIN, int COUT, int TP, int CO = COUT, int WPE = 1>
__global__ __launch_bounds__(256, WPE) void conv_hxg(ConvParams p, int nby, int nbx) {
  constexpr int TC = CO / 16, NG = CIN / 32, NKS = 9 * NG, CB = COUT / CO;
  constexpr int BW = 16, BH = 4 * TP, PW = BW + 2, SLOTS = (BH + 2) * PW;
  constexpr int SB = 128;                                    // slot: 32 hi + 32 lo f16 channels
  constexpr int PIECES = ((SLOTS * SB + 1023) / 1024 + 3) / 4 * 4;   // 1 KiB DMA pieces per stage, 4 waves alike
  constexpr int STAGE = PIECES * 1024;
  constexpr int RS = CO + 4;                                 // epilogue image row (floats)
  constexpr int EPI = BH * BW * RS * 4;
  constexpr int SMEM = 2 * STAGE > EPI ? 2 * STAGE : EPI;
  static_assert(COUT % 16 == 0 && CIN % 32 == 0 && CIN % 64 != 0, "32-channel groups (pack_wfrag gt 1)");
  static_assert(COUT % CO == 0 && CO % 16 == 0, "channel blocks");
  static_assert(SMEM <= 163840, "LDS");
  __shared__ __attribute__((aligned(16))) char smem[SMEM];
  const ConvSeg& S = p.seg[0];
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int nblk = p.N * nby * nbx * CB;
  const int bq = xcd_remap(blockIdx.x, nblk);
  const int cb = bq % CB, b = bq / CB;   // (a block's CB workgroups consecutive: one XCD, one halo in its L2)
  const int n = b / (nby * nbx), rem = b - n * (nby * nbx);
  const int oy0 = (rem / nbx) * BH, ox0 = (rem - (rem / nbx) * nbx) * BW;
  const int H = S.H, W = S.W;
  const int fr = lane & 15, kg = lane >> 4;

  auto rsrc = [](const void* base) __attribute__((always_inline)) {
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), (short)0, (int)0xffffffff, 0x00020000);
  };
  const __amdgpu_buffer_rsrc_t xrs = rsrc(S.x);
  const __amdgpu_buffer_rsrc_t wrs = rsrc(p.wfrag);

  // this lane's share of a stage: piece i = wave + 4 j, LDS byte i * 1024 + lane * 16 = slot s,
  // chunk position q (source chunk q ^ (s & 7): hi channels 8 c.. for c < 4, lo channels 8 (c - 4)..)
  constexpr int PPW = PIECES / 4;
  unsigned src[PPW];
#pragma unroll
  for (int j = 0; j < PPW; ++j) {
    const int bb = (wave + 4 * j) * 1024 + lane * 16;
    const int sl = bb >> 7, q = (bb >> 4) & 7;
    const int c = q ^ (sl & 7);
    const int iy = oy0 - 1 + sl / PW, ix = ox0 - 1 + (sl - (sl / PW) * PW);
    const bool ok = sl < SLOTS && (unsigned)iy < (unsigned)H && (unsigned)ix < (unsigned)W;
    // (unsigned: the pixel byte offset fits 32 bits only, the planner keeps buffers below 4 GiB)
    src[j] = ok ? (unsigned)((n * H + iy) * W + ix) * (unsigned)(S.cs * 2) + (unsigned)(((c & 3) * 8 + (c >> 2) * CIN) * 2)
                : S.zero_off + (unsigned)(q << 4);
  }
  auto stage = [&](int g, int st) __attribute__((always_inline)) {
#pragma unroll
    for (int j = 0; j < PPW; ++j) {
      unsigned off = src[j];
      asm volatile("" : "+v"(off));
      // a group's channels ride in the instruction's scalar offset (64 bytes per group); the zero
      // tail is wider than any pixel row, so out-of-image slots stay zero for every group
      __builtin_amdgcn_raw_ptr_buffer_load_lds(xrs, (lds_ptr_t)(smem + st * STAGE + (wave + 4 * j) * 1024), 16, off,
                                               g * 64, 0, 0);
    }
  };
  // weight fragments of k-step s = 32-channel group s / 9, tap s % 9 (packed K tile s): TC row blocks
  // x [W_hi, W_lo] x 1 KiB (lane l: row 16 a + (l & 15), channels 8 (l >> 4) .. +8)
  constexpr int TILE = COUT / 16 * 2 * 1024;
  const int wo = lane * 16 + cb * TC * 2 * 1024;   // this workgroup's row blocks cb TC ..
  auto wload = [&](f16x8* wh, f16x8* wl, int s) __attribute__((always_inline)) {
#pragma unroll
    for (int a = 0; a < TC; ++a) {
      wh[a] = __builtin_bit_cast(f16x8, __builtin_amdgcn_raw_buffer_load_b128(wrs, wo + (a * 2) * 1024, s * TILE, 0));
      wl[a] = __builtin_bit_cast(f16x8, __builtin_amdgcn_raw_buffer_load_b128(wrs, wo + (a * 2 + 1) * 1024, s * TILE, 0));
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

  static_for<NG>([&](auto gc) __attribute__((always_inline)) {
    constexpr int g = decltype(gc)::value, st = g & 1;
    // group g's halo: every VMEM op but the youngest 2 TC (k-step 9 g's weights) has landed
    asm volatile("s_waitcnt vmcnt(%0)" ::"n"(2 * TC) : "memory");
    __syncthreads();   // every wave's pieces of group g; every wave done with group g - 1's stage
    if constexpr (g + 1 < NG) stage(g + 1, st ^ 1);
    const char* base = smem + st * STAGE;
    static_for<9>([&](auto tc) __attribute__((always_inline)) {
      constexpr int tap = decltype(tc)::value, s = g * 9 + tap, q = s & 1;
      constexpr int toff = (tap / 3) * PW + (tap % 3);
      if constexpr (s + 1 < NKS) wload(wbh[q ^ 1], wbl[q ^ 1], s + 1);
      f16x8 bh[TP], bl[TP];
#pragma unroll
      for (int t = 0; t < TP; ++t) {
        const int sl = (wave * TP + t) * PW + fr + toff;
        bh[t] = *reinterpret_cast<const f16x8*>(base + sl * SB + ((kg ^ (sl & 7)) << 4));
        bl[t] = *reinterpret_cast<const f16x8*>(base + sl * SB + (((4 + kg) ^ (sl & 7)) << 4));
      }
      if (p.dbg & 2) return;   // tuning only: no MFMAs
#pragma unroll
      for (int a = 0; a < TC; ++a)
#pragma unroll
        for (int t = 0; t < TP; ++t)
          acc[a][t] = __builtin_amdgcn_mfma_f32_16x16x32_f16(wbl[q][a], bh[t], acc[a][t], 0, 0, 0);
#pragma unroll
      for (int a = 0; a < TC; ++a)
#pragma unroll
        for (int t = 0; t < TP; ++t)
          acc[a][t] = __builtin_amdgcn_mfma_f32_16x16x32_f16(wbh[q][a], bh[t], acc[a][t], 0, 0, 0);
#pragma unroll
      for (int a = 0; a < TC; ++a)
#pragma unroll
        for (int t = 0; t < TP; ++t)
          acc[a][t] = __builtin_amdgcn_mfma_f32_16x16x32_f16(wbh[q][a], bl[t], acc[a][t], 0, 0, 0);
    });
  });
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  if (p.dbg & 4) return;   // tuning only: no epilogue

  // ---- epilogue (conv_hx64's): f32 [pixel][channel] image over the LDS, then 8 channels of one
  // pixel per thread and step: bias, activation select, split residual hi + lo, hi / lo stores ----
  __syncthreads();   // every wave is done with the stages
  float* im = reinterpret_cast<float*>(smem);
#pragma unroll
  for (int a = 0; a < TC; ++a)
#pragma unroll
    for (int t = 0; t < TP; ++t) {
      const int pl = (wave * TP + t) * BW + fr;
      *reinterpret_cast<f32x4*>(im + pl * RS + a * 16 + kg * 4) = acc[a][t];
    }
  __syncthreads();
  const int OW = p.OW, OH = p.OH;
  const bool smooth = p.act == ACT_SILU || p.act == ACT_GELU;
  const bool has_res = p.res_mode != RES_NONE;
  const bool pre_act = !p.act_after_res;
  // a thread keeps one 8-channel group (threads past the last whole pixel lane idle), so the channel
  // terms load once; the pixels' residual rows are requested before the first store
  constexpr int CGN = CO / 8, PL = 256 / CGN, NPX = BH * BW, ITP = (NPX + PL - 1) / PL;
  const int cg = threadIdx.x % CGN, pl0 = threadIdx.x / CGN;
  if (pl0 >= PL) return;
  const int ch = cb * CO + cg * 8;
  float bc[8], sl[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    bc[j] = p.bias_mode == BIAS_CHANNEL ? p.bias[ch + j] : 0.f;
    sl[j] = p.act == ACT_PRELU ? p.slope[ch + j] : (p.act == ACT_RELU ? 0.f : 1.f);
  }
  constexpr int RGP = 8;   // residual rows in flight per group of pixels
  for (int k0 = 0; k0 < ITP; k0 += RGP) {
    f16x8 rh[RGP], rl[RGP];
#pragma unroll
    for (int kk = 0; kk < RGP; ++kk) {
      rh[kk] = f16x8{};
      rl[kk] = f16x8{};
      const int pl = pl0 + PL * (k0 + kk);
      const int oy = oy0 + pl / BW, ox = ox0 + (pl & (BW - 1));
      if (has_res && pl < NPX && oy < OH && ox < OW) {
        const f16* rp = reinterpret_cast<const f16*>(p.res) + (((long long)n * OH + oy) * OW + ox) * p.rcs + ch;
        rh[kk] = *reinterpret_cast<const f16x8*>(rp);
        rl[kk] = *reinterpret_cast<const f16x8*>(rp + p.rsplit);
      }
    }
#pragma unroll
    for (int kk = 0; kk < RGP; ++kk) {
      const int pl = pl0 + PL * (k0 + kk);
      if (pl >= NPX) continue;
      const int oy = oy0 + pl / BW, ox = ox0 + (pl & (BW - 1));
      if (oy >= OH || ox >= OW) continue;
      const long long pix = ((long long)n * OH + oy) * OW + ox;
      const f32x4 lo4 = *reinterpret_cast<const f32x4*>(im + pl * RS + cg * 8);
      const f32x4 hi4 = *reinterpret_cast<const f32x4*>(im + pl * RS + cg * 8 + 4);
      float v[8] = {lo4[0] + bc[0], lo4[1] + bc[1], lo4[2] + bc[2], lo4[3] + bc[3],
                    hi4[0] + bc[4], hi4[1] + bc[5], hi4[2] + bc[6], hi4[3] + bc[7]};
      if (p.bias_mode == BIAS_BORDER9) {
        const int rc = oy - 1 < 0 ? 0 : (oy + 1 >= H ? 2 : 1);
        const int cc = ox - 1 < 0 ? 0 : (ox + 1 >= W ? 2 : 1);
        const float* bp = p.bias + (rc * 3 + cc) * p.npad + ch;
#pragma unroll
        for (int j = 0; j < 8; ++j) v[j] += bp[j];
      }
      float r[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) r[j] = (float)rh[kk][j] + (float)rl[kk][j];
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
        const float x = ch + j < p.cout ? v[j] : 0.f;
        yh[j] = (f16)x;
        yl[j] = (f16)(x - (float)yh[j]);
      }
      if (p.dbg & 16) continue;   // tuning only: no stores
      f16* yp = reinterpret_cast<f16*>(p.y) + pix * p.ycs + ch;
      *reinterpret_cast<f16x8*>(yp) = yh;
      *reinterpret_cast<f16x8*>(yp + p.ysplit) = yl;
    }
  }
}

constexpr int HXG_TP = 5;   // 16 x 20 output blocks: 80 / 20 rows, no waste on the 80x80 maps

// can a conv run on conv_hxg<C, C>: split C-channel input (X.C 2 C = [hi | lo]), C output channels written
// split, 3x3 stride 1 pad 1, same size, plain or same-size split residual; C = 96 (both forms) or 224 (SCRFD's
// 20x20x224 neck, the small-batch form)
int conv_hxg_ok(const ConvParams& p, int small) {
  const ConvSeg& S = p.seg[0];
  const int C = S.C / 2;
  return p.nseg == 1 && (C == 96 || (small && C == 224)) && S.cs == 2 * C && S.KH == 3 && S.KW == 3 && S.stride == 1 &&
         S.pad == 1 && S.H == p.OH && S.W == p.OW && p.npad == C && p.ysplit == C && p.splitk == 1 && !p.out_f32 &&
         p.ktot == 27 * C && p.res_mode != RES_UP2 && (p.res_mode == RES_NONE || (p.rsplit == C && p.rcs % 8 == 0)) &&
         p.ycs % 8 == 0 && p.cwrite == C && p.wfrag != nullptr;
}

hipError_t conv_hxg_launch(const ConvParams& p, int small, hipStream_t s) {
  if (!conv_hxg_ok(p, small)) return hipErrorInvalidValue;
  if (small) {   // 16x4 blocks x 32 of the C output channels, C / 32 workgroups per block
    const int nby = (p.OH + 3) / 4, nbx = (p.OW + 15) / 16;
    if (p.npad == 224)
      hipLaunchKernelGGL((conv_hxg<224, 224, 1, 32, 2>), dim3(p.N * nby * nbx * 7), dim3(256), 0, s, p, nby, nbx);
    else
      hipLaunchKernelGGL((conv_hxg<96, 96, 1, 32, 2>), dim3(p.N * nby * nbx * 3), dim3(256), 0, s, p, nby, nbx);
    return hipGetLastError();
  }
  const int nby = (p.OH + 4 * HXG_TP - 1) / (4 * HXG_TP), nbx = (p.OW + 15) / 16;
  hipLaunchKernelGGL((conv_hxg<96, 96, HXG_TP>), dim3(p.N * nby * nbx), dim3(256), 0, s, p, nby, nbx);
  return hipGetLastError();
}

// can a conv run here: split 64-channel input (X.C 128 = [hi | lo]), 64 output channels
// written split, 3x3 stride 1 pad 1, same size
int conv_hx_ok(const ConvParams& p) {
  const ConvSeg& S = p.seg[0];
  return p.nseg == 1 && S.C == 128 && S.KH == 3 && S.KW == 3 && S.stride == 1 && S.pad == 1 &&
         S.H == p.OH && S.W == p.OW && p.npad == 64 && p.ysplit == 64 && p.splitk == 1 && !p.out_f32 &&
         p.ktot == 9 * 192 && p.res_mode != RES_UP2 && (p.res_mode == RES_NONE || (p.rsplit == 64 && p.rcs % 8 == 0)) &&
         p.ycs % 8 == 0 && p.cwrite == 64 && p.wfrag != nullptr;
}

hipError_t conv_hx_launch(const ConvParams& p, hipStream_t s) {
  if (!conv_hx_ok(p)) return hipErrorInvalidValue;
  const int nby = (p.OH + HX_TH - 1) / HX_TH, nbx = (p.OW + HX_TW - 1) / HX_TW;
  // (per launch: the A/B switches it in one process)
  if (getenv("PC_HX64_WLDS") && atoi(getenv("PC_HX64_WLDS")) == 0)
    hipLaunchKernelGGL(conv_hx64<false>, dim3(p.N * nby * nbx), dim3(256), 0, s, p, nby, nbx);
  else
    hipLaunchKernelGGL(conv_hx64<true>, dim3(p.N * nby * nbx), dim3(256), 0, s, p, nby, nbx);
  return hipGetLastError();
}

}  // namespace pc
