// Image-resident f16x3 3x3 convolutions for IResNet's 28x28x128 and 14x14x256 stages (gfx950): the
// ArcFace-x3 layers that run on conv_fast's fused WG tiles.
//
// conv_fast stages, per 32-channel K tile, the split pixel rows of one tap: every input pixel moves
// L2 -> LDS nine times (the tile's pixels re-read for each tap), through 4 LDS-DMA pieces per wave
// and a barrier per K tile. Its 128x256 tile on 28x28x128 issues only 48 MFMAs per wave between two
// barriers and ran at 36 % of the matrix pipe (r05/r06 per-layer probes). Here one workgroup owns
// ROWS full output rows of one image - every output channel - and stages the rows' padded halo once
// per group of 64 input channels (hi and lo: 256-byte slots), in a 2-stage ring: group g + 1 lands
// while group g's 18 k-steps (9 taps x two 32-channel blocks) run; one barrier per group, none inside.
//  * output pixels are enumerated as ROWS x PITCH slots (the halo's pitch: the map width + 2 padding
//    columns, rounded up to 16), so a tap is one slot offset for every 16-slot pixel fragment; the
//    PITCH - HW columns past the map are computed and discarded (12.5 % at 14x14 - what the 256x224
//    tile paid in idle CUs at batch 256 - and at 28x28);
//  * 8 waves = WCH channel groups x WPX fragment groups; a wave's weight fragments come from the
//    fragment-ordered copy (pc_api.cpp pack_wfrag) into registers a k-step ahead (double-buffered),
//    its pixel fragments from the halo in groups of at most 7;
//  * K order and MFMA order are conv_fast SX / WG's exactly - channel groups of 64 (every tap of a
//    group, the two 32-channel blocks per tap), per k-step W_lo*x_hi, W_hi*x_hi, W_hi*x_lo - and the
//    epilogue arithmetic is conv_epilogue_lds<SPLIT>'s, so the outputs are bit-identical to the fused
//    tiles every other plan class of the net runs (tests/test_gpu_arcface.py);
//  * LDS chunk swizzle: chunk q of slot h holds source chunk q ^ ((h & 7) << 1) - conflict-free
//    ds_read_b128 for 16 consecutive slots at any alignment, hi or lo, either block (checked
//    exhaustively over the instruction's lane groups, MI355X_MICROARCH.md §LDS);
//  * epilogue: a thread keeps one 8-channel group for all its pixels, so the channel bias and slopes
//    are loaded once, and the per-pixel term of each of its pixels (the residual's hi + lo, or a folded
//    pre-BN's border-class bias) is requested before the accumulators go to the LDS image, so the loads
//    overlap the transposition (the first form loaded both per item: its epilogue took 53 of 184 us on
//    28x28x128, profiles/r06f_hxi28_phase_split.txt).
#include "pc_conv_common.h"

#include <cstdlib>

namespace pc {

// SPLIT (f16x3): a halo slot holds one 64-channel group's hi and lo halves (256 bytes), staged group by
// group in a 2-stage ring; K = (group, tap, 32-channel block), 3 MFMA passes per k-step (the fused
// tiles' order). Plain f16 (the BASELINE C2 fp16 net): a slot holds every input channel (CIN * 2 bytes),
// staged once; K = (tap, 32-channel block), tap-major like conv_fast's plain tiles and the resident
// chain, one MFMA per fragment pair - so it is bit-identical to them as well.
template <int HW, int PITCH, int ROWS, int CIN, int COUT, int WCH, int WPX, bool SPLIT, int OCC>
struct HxiGeom {
  static constexpr int NW = WCH * WPX, NT = 64 * NW;
  static constexpr int NF = (ROWS * PITCH + 15) / 16;       // pixel fragments per workgroup (16 slots each)
  static constexpr int TP = NF / WPX, TC = COUT / WCH / 16;
  static constexpr int CB = CIN / COUT;                      // channel blocks: workgroups per row block
  static constexpr int WPS = (NW * OCC + 3) / 4;             // waves per SIMD
  // fragments per read group (4 waves per SIMD - two 8-wave workgroups per CU: one at a time, the other
  // waves hide the reads)
  static constexpr int TPG = WPS > 2 ? 1 : (TP > 7 ? (TP % 2 == 0 ? TP / 2 : TP) : TP);
  // one wave per SIMD (the small-batch forms): no other wave hides a latency - the weights come 5 k-steps
  // ahead (not 1), and the pixel fragments of k-step k + 1 are read under k-step k's MFMAs (PF): 14x14 at
  // 12 images 34.9 -> 29.9 us. (Loader waves of their own for the halo pieces, 1-4 per workgroup, did not
  // beat the compute waves issuing them: 28.5-30.0 / 20.9-21.0 / 37-45 us, profiles/r06bh_hxs_phase.txt)
  static constexpr int WD = WPS == 1 ? 6 : 2;                // weight register buffers
  static constexpr bool PF = WPS == 1 && SPLIT && TPG == TP;
  static constexpr int SB = SPLIT ? 256 : CIN * 2;           // halo slot bytes
  static constexpr int NB = SPLIT ? 2 : CIN / 32;            // 32-channel blocks per staged group
  static constexpr int NG = SPLIT ? CIN / 64 : 1, KPG = 9 * NB, NKS = NG * KPG;
  // halo slots: the padded rows, + what the taps of the last fragment's discarded slots reach
  static constexpr int SLOTS = (NF * 16 > ROWS * PITCH ? NF * 16 - ROWS * PITCH : 0) + (ROWS + 2) * PITCH + 2;
  static constexpr int PIECES = (SLOTS * SB + 1023) / 1024;
  static constexpr int STAGE = PIECES * 1024;
  // a 2-stage ring where the groups are several and two stages fit the workgroup's LDS share; else one
  // stage (at two workgroups per CU the other workgroup's MFMAs cover the exposed staging)
  static constexpr int NSTAGE = NG > 1 && 2 * STAGE * OCC <= 163840 ? 2 : 1;
  static constexpr int NPIX = ROWS * HW;
  static constexpr int PC = COUT * NPIX * 4 <= 131072 / OCC ? COUT : COUT / 2;   // channels per epilogue pass
  static constexpr int NPASS = COUT / PC;
  static constexpr int RS = PC + 4;
  static constexpr int EPI = NPIX * RS * 4;
  static constexpr int SMEM = NSTAGE * STAGE > EPI ? NSTAGE * STAGE : EPI;
  static constexpr int WTILE = SPLIT ? 2048 : 1024;          // packed weight bytes per K tile and 16-row block
  static constexpr int CGN = PC / 8;                         // 8-channel items per pixel and pass
  static constexpr int IT = (NPIX + NT / CGN - 1) / (NT / CGN);   // items (pixels) per thread and pass
  static_assert(PITCH >= HW + 2 && NF % WPX == 0 && TP % TPG == 0, "pixel fragments");
  static_assert(COUT % (16 * WCH) == 0 && CIN % 64 == 0 && HW % ROWS == 0 && SB % 256 == 0, "tiling");
  static_assert(SMEM <= 163840, "LDS");
  static_assert(NPASS == 1 || WCH % 2 == 0, "epilogue passes split the channel waves");
};

template <int HW, int PITCH, int ROWS, int CIN, int COUT, int WCH, int WPX, bool SPLIT = true, int OCC = 1>
__global__ __launch_bounds__(64 * WCH * WPX, (WCH * WPX * OCC + 3) / 4) void conv_hxi(ConvParams p) {
  using G = HxiGeom<HW, PITCH, ROWS, CIN, COUT, WCH, WPX, SPLIT, OCC>;
  constexpr int NW = G::NW, NT = G::NT, TC = G::TC, TP = G::TP, TPG = G::TPG, NG = G::NG, NKS = G::NKS;
  constexpr int STAGE = G::STAGE, PIECES = G::PIECES, SB = G::SB, NB = G::NB, KPG = G::KPG;
  static_assert(G::SMEM * OCC <= 163840, "LDS for OCC workgroups per CU");
  static_assert(NW <= 16, "waves");
  __shared__ __attribute__((aligned(16))) char smem[G::SMEM];
  const ConvSeg& S = p.seg[0];
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int wch = wave % WCH, wpx = wave / WCH;
  constexpr int RB = HW / ROWS, CB = G::CB;      // row blocks per image, channel blocks per row block
  // (a row block's CB workgroups are consecutive: on one XCD after the remap, sharing its halo in the L2)
  const int b = xcd_remap(blockIdx.x, p.N * RB * CB);
  const int cb = b % CB, nb = b / CB;
  const int n = nb / RB, r0 = (nb - n * RB) * ROWS;
  const int fr = lane & 15, kg = lane >> 4;

  auto rsrc = [](const void* base) __attribute__((always_inline)) {
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), (short)0, (int)0xffffffff, 0x00020000);
  };
  const __amdgpu_buffer_rsrc_t xrs = rsrc(S.x);
  const __amdgpu_buffer_rsrc_t wrs = rsrc(p.wfrag);

  // this wave's halo pieces i = wave + 8 j: LDS byte i * 1024 + lane * 16 = slot h, chunk position q,
  // holding source chunk c = q ^ ((h & 7) << 1) (the XOR touches the low 4 bits only): split: channels
  // 8 (c & 7) .. of the group's hi (c < 8) or lo half; plain: channels 8 c .. - of input pixel
  // (r0 - 1 + h / PITCH, h % PITCH - 1); zeros outside
  constexpr int PPW = (PIECES + NW - 1) / NW;
  // (offsets computed at each issue: kept in registers for all pieces they spilled the 256-register
  // plain 14x14 form, 17 pieces per wave)
  auto stage = [&](int g, int st) __attribute__((always_inline)) {
#pragma unroll
    for (int j = 0; j < PPW; ++j) {
      if (wave + NW * j < PIECES) {   // (wave-uniform)
        const int byte = (wave + NW * j) * 1024 + lane * 16;
        const int h = byte / SB, q = (byte % SB) >> 4;
        const int c = q ^ ((h & 7) << 1);
        const int iy = r0 - 1 + h / PITCH, ix = h % PITCH - 1;
        const bool ok = h < (ROWS + 2) * PITCH && (unsigned)iy < (unsigned)HW && (unsigned)ix < (unsigned)HW;
        const int cb = SPLIT ? ((c & 7) * 8 + (c >> 3) * CIN) * 2 : c * 16;
        unsigned off = ok ? (unsigned)((n * HW + iy) * HW + ix) * (unsigned)(S.cs * 2) + (unsigned)cb
                          : S.zero_off + (unsigned)((q & 15) << 4);
        asm volatile("" : "+v"(off));
        // split: the group's 64 channels ride in the scalar offset (128 bytes per group of each half)
        __builtin_amdgcn_raw_ptr_buffer_load_lds(xrs, (lds_ptr_t)(smem + st * STAGE + (wave + NW * j) * 1024), 16, off,
                                                 g * 128, 0, 0);
      }
    }
  };
  // weight fragments of k-step s (packed K tile s; split: group s / 18, tap (s % 18) / 2, block s % 2,
  // plain: tap s / NB, block s % NB): row blocks TC wch .. TC wch + TC - 1 of npad / 16, each
  // [W_hi, W_lo] (split) or W (plain) x 1 KiB
  const int tile = (p.npad / 16) * G::WTILE;
  auto wload = [&](f16x8* wh, f16x8* wl, int s) __attribute__((always_inline)) {
#pragma unroll
    for (int a = 0; a < TC; ++a) {
      const int o = (cb * (COUT / 16) + TC * wch + a) * G::WTILE + lane * 16;
      wh[a] = __builtin_bit_cast(f16x8, __builtin_amdgcn_raw_buffer_load_b128(wrs, o, s * tile, 0));
      if constexpr (SPLIT) wl[a] = __builtin_bit_cast(f16x8, __builtin_amdgcn_raw_buffer_load_b128(wrs, o + 1024, s * tile, 0));
    }
  };
  constexpr int WD = G::WD;
  f16x8 wbh[WD][TC], wbl[WD][TC];
  stage(0, 0);
  static_for<WD - 1>([&](auto jc) __attribute__((always_inline)) {
    constexpr int j = decltype(jc)::value;
    if constexpr (j < NKS) wload(wbh[j], wbl[j], j);
  });
  f16x8 bhp[2][G::PF ? TP : 1];   // (PF: this and the next k-step's hi pixel fragments)

  f32x4 acc[TC][TP];
#pragma unroll
  for (int a = 0; a < TC; ++a)
#pragma unroll
    for (int t = 0; t < TP; ++t) acc[a][t] = f32x4{0.f, 0.f, 0.f, 0.f};
  if (p.dbg & 8) return;   // tuning only (PC_CONV_DBG): prologue only

  // per-lane LDS byte of (tap, chunk kind) for slot fr + sh, sh = dy PITCH + dx the tap's slot shift (the
  // swizzle key is the slot's low bits: at a pitch that is not a multiple of 8 the row shift changes them)
  // (recomputed at each k-step - the asm keeps the compiler from hoisting all (tap, block) offsets of
  // the unrolled loop into registers at once: 24 of them in the plain 256-channel form)
  auto boff = [&](int sh, int chunk) __attribute__((always_inline)) {
    const int h = fr + sh;
    unsigned v = (unsigned)(h * SB + ((chunk ^ ((h & 7) << 1)) << 4));
    asm volatile("" : "+v"(v));
    return v;
  };
  // halo slot of fragment t's first slot at tap (0, 0): fragment f = wpx * TP + t covers output slots
  // 16 f .. 16 f + 15 (slot o = output row o / PITCH, column o % PITCH; columns >= HW and rows >= ROWS are
  // discarded - a pitch that is not a multiple of 16 lets a fragment span two rows: the 7x7 form's 9)
  auto fslot = [&](int t) __attribute__((always_inline)) { return (wpx * TP + t) * 16; };
  static_for<NG>([&](auto gc) __attribute__((always_inline)) {
    constexpr int g = decltype(gc)::value, st = G::NSTAGE == 2 ? (g & 1) : 0;
    if constexpr (G::NSTAGE == 1 && g > 0) {   // one stage: group g replaces g - 1 once every wave is done
      __syncthreads();
      stage(g, 0);
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    } else {
      // group g's halo: every VMEM op but the youngest (the next WD - 1 k-steps' weights) has landed
      asm volatile("s_waitcnt vmcnt(%0)" ::"n"((WD - 1) * (SPLIT ? 2 * TC : TC)) : "memory");
    }
    __syncthreads();   // every wave's pieces of group g; every wave done reading group g - 1's stage
    if constexpr (G::NSTAGE == 2 && g + 1 < NG) stage(g + 1, st ^ 1);
    const char* base = smem + st * STAGE;
    static_for<KPG>([&](auto kc) __attribute__((always_inline)) {
      constexpr int k = decltype(kc)::value, tap = k / NB, blk = k % NB, s = g * KPG + k, q = s % WD;
      constexpr int dy = tap / 3, dx = tap % 3;
      if constexpr (s + WD - 1 < NKS) wload(wbh[(s + WD - 1) % WD], wbl[(s + WD - 1) % WD], s + WD - 1);
      // (pitches that are multiples of 8 keep the row shift out of the swizzled offset: fewer live offsets -
      // folding it in spilled the two-workgroup 28x28 form)
      constexpr int sh = PITCH % 8 == 0 ? dx : dy * PITCH + dx, rsh = PITCH % 8 == 0 ? dy * PITCH : 0;
      const unsigned oh = boff(sh, blk * 4 + kg), ol = SPLIT ? boff(sh, 8 + blk * 4 + kg) : 0u;
      if (p.dbg & 2) return;   // tuning only: no MFMAs
      if constexpr (G::PF) {
        // the hi fragments were read at the previous k-step (the group's first: here), the lo ones at the top
        // of this one; the next k-step's hi fragments are requested before the last MFMA pass (same passes,
        // same order per accumulator)
        constexpr int cur = k & 1;
        if constexpr (k == 0) {
#pragma unroll
          for (int t = 0; t < TP; ++t) bhp[cur][t] = *reinterpret_cast<const f16x8*>(base + oh + (fslot(t) + rsh) * SB);
        }
        f16x8 bl[TP];
#pragma unroll
        for (int t = 0; t < TP; ++t) bl[t] = *reinterpret_cast<const f16x8*>(base + ol + (fslot(t) + rsh) * SB);
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int a = 0; a < TC; ++a)
#pragma unroll
          for (int t = 0; t < TP; ++t)
            acc[a][t] = __builtin_amdgcn_mfma_f32_16x16x32_f16(wbl[q][a], bhp[cur][t], acc[a][t], 0, 0, 0);
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int a = 0; a < TC; ++a)
#pragma unroll
          for (int t = 0; t < TP; ++t)
            acc[a][t] = __builtin_amdgcn_mfma_f32_16x16x32_f16(wbh[q][a], bhp[cur][t], acc[a][t], 0, 0, 0);
        __builtin_amdgcn_sched_barrier(0);
        if constexpr (k + 1 < KPG) {
          constexpr int tap1 = (k + 1) / NB, blk1 = (k + 1) % NB, dy1 = tap1 / 3, dx1 = tap1 % 3;
          constexpr int sh1 = PITCH % 8 == 0 ? dx1 : dy1 * PITCH + dx1, rsh1 = PITCH % 8 == 0 ? dy1 * PITCH : 0;
          const unsigned oh1 = boff(sh1, blk1 * 4 + kg);
#pragma unroll
          for (int t = 0; t < TP; ++t)
            bhp[cur ^ 1][t] = *reinterpret_cast<const f16x8*>(base + oh1 + (fslot(t) + rsh1) * SB);
        }
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int a = 0; a < TC; ++a)
#pragma unroll
          for (int t = 0; t < TP; ++t)
            acc[a][t] = __builtin_amdgcn_mfma_f32_16x16x32_f16(wbh[q][a], bl[t], acc[a][t], 0, 0, 0);
        __builtin_amdgcn_sched_barrier(0);
        return;
      }
      static_for<TP / TPG>([&](auto pc) __attribute__((always_inline)) {
        constexpr int t0 = decltype(pc)::value * TPG;
        f16x8 bh[TPG], bl[SPLIT ? TPG : 1];
#pragma unroll
        for (int t = 0; t < TPG; ++t)
          bh[t] = *reinterpret_cast<const f16x8*>(base + oh + (fslot(t0 + t) + rsh) * SB);
        if constexpr (!SPLIT) {   // plain f16: one MFMA per fragment pair
#pragma unroll
          for (int a = 0; a < TC; ++a)
#pragma unroll
            for (int t = 0; t < TPG; ++t)
              acc[a][t0 + t] = __builtin_amdgcn_mfma_f32_16x16x32_f16(wbh[q][a], bh[t], acc[a][t0 + t], 0, 0, 0);
          __builtin_amdgcn_sched_barrier(0);
          return;
        }
#pragma unroll
        for (int a = 0; a < TC; ++a)
#pragma unroll
          for (int t = 0; t < TPG; ++t)
            acc[a][t0 + t] = __builtin_amdgcn_mfma_f32_16x16x32_f16(wbl[q][a], bh[t], acc[a][t0 + t], 0, 0, 0);
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int t = 0; t < TPG; ++t)
          bl[t] = *reinterpret_cast<const f16x8*>(base + ol + (fslot(t0 + t) + rsh) * SB);
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

  // ---- epilogue in NPASS passes of PC channels: the waves of a pass's channels write their
  // accumulators into an f32 [pixel][channel] image over the LDS; then every thread finishes 8 channels
  // of one pixel per item with conv_epilogue_lds<SPLIT>'s arithmetic: bias (per channel, then the border
  // class), residual hi + lo before or after the activation select, channel keep mask, hi / lo stores ----
  constexpr int NPIX = G::NPIX, RS = G::RS, PC = G::PC, NPASS = G::NPASS, CGN = G::CGN, IT = G::IT;
  static_assert(NT % CGN == 0, "a thread keeps one 8-channel group");
  constexpr int PSTEP = NT / CGN;                     // pixel stride between a thread's items
  float* im = reinterpret_cast<float*>(smem);
  const bool smooth = p.act == ACT_SILU || p.act == ACT_GELU;
  const bool has_res = p.res_mode != RES_NONE;
  const bool pre_act = !p.act_after_res;
  const bool border = p.bias_mode == BIAS_BORDER9;
  const long long pix0 = (long long)n * HW * HW + r0 * HW;   // the workgroup's first output pixel
  const int cg = threadIdx.x % CGN, pl0 = threadIdx.x / CGN;
#pragma unroll
  for (int pass = 0; pass < NPASS; ++pass) {
    const int ch = cb * COUT + pass * PC + cg * 8;
    // per-thread channel terms (one 8-channel group for all of the thread's pixels): channel bias (0
    // otherwise, as conv_epilogue_lds adds it), negative-side slope (PReLU / 0 for ReLU / 1)
    float bc[8], sl[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      bc[j] = p.bias_mode == BIAS_CHANNEL ? p.bias[ch + j] : 0.f;
      sl[j] = p.act == ACT_PRELU ? p.slope[ch + j] : (p.act == ACT_RELU ? 0.f : 1.f);
    }
    // the per-pixel term of each of the thread's items, requested before anything waits on it: the
    // residual hi + lo (its f32 value), or the border-class bias of a folded pre-BN conv
    // (four waves per SIMD - two 8-wave workgroups per CU: loaded at the item instead - the other workgroup covers the latency, and
    // the registers are not there)
    constexpr bool PREF = G::WPS <= 2;
    float pre[PREF ? IT : 1][8];
    auto load_pre = [&](int k, float* dst) __attribute__((always_inline)) {
      const int pl = pl0 + PSTEP * k;
#pragma unroll
      for (int j = 0; j < 8; ++j) dst[j] = 0.f;
      if (pl >= NPIX) return;
      if (has_res) {
        const f16* rp = reinterpret_cast<const f16*>(p.res) + (pix0 + pl) * p.rcs + ch;
        const f16x8 rh = *reinterpret_cast<const f16x8*>(rp);
        if constexpr (SPLIT) {
          const f16x8 rl = *reinterpret_cast<const f16x8*>(rp + p.rsplit);
#pragma unroll
          for (int j = 0; j < 8; ++j) dst[j] = (float)rh[j] + (float)rl[j];
        } else {
#pragma unroll
          for (int j = 0; j < 8; ++j) dst[j] = (float)rh[j];
        }
      } else if (border) {
        const int oy = r0 + pl / HW, ox = pl % HW;
        const int rc = oy - 1 < 0 ? 0 : (oy + 1 >= HW ? 2 : 1);
        const int cc = ox - 1 < 0 ? 0 : (ox + 1 >= HW ? 2 : 1);
        const f32x4* bp = reinterpret_cast<const f32x4*>(p.bias + (rc * 3 + cc) * p.npad + ch);
        const f32x4 b0 = bp[0], b1 = bp[1];
        dst[0] = b0[0]; dst[1] = b0[1]; dst[2] = b0[2]; dst[3] = b0[3];
        dst[4] = b1[0]; dst[5] = b1[1]; dst[6] = b1[2]; dst[7] = b1[3];
      }
    };
    if constexpr (PREF) {
#pragma unroll
      for (int k = 0; k < IT; ++k) load_pre(k, pre[k]);
    }
    __syncthreads();   // the stages (pass 0) / the previous pass's image are no longer read
    if (NPASS == 1 || wch / (WCH / 2) == pass) {
#pragma unroll
      for (int a = 0; a < TC; ++a)
#pragma unroll
        for (int t = 0; t < TP; ++t) {
          const int o = (wpx * TP + t) * 16 + fr;
          const int orow = o / PITCH, ocol = o % PITCH;
          if (ocol < HW && orow < ROWS) {
            const int pl = orow * HW + ocol;
            const int cl = (NPASS == 1 ? wch : wch % (WCH / 2)) * TC * 16 + a * 16 + kg * 4;
            *reinterpret_cast<f32x4*>(im + pl * RS + cl) = acc[a][t];
          }
        }
    }
    __syncthreads();
#pragma unroll
    for (int k = 0; k < IT; ++k) {
      const int pl = pl0 + PSTEP * k;
      if (pl >= NPIX) continue;
      float pk[8];
      if constexpr (PREF) {
#pragma unroll
        for (int j = 0; j < 8; ++j) pk[j] = pre[k][j];
      } else {
        load_pre(k, pk);
      }
      const long long pix = pix0 + pl;
      const f32x4 lo4 = *reinterpret_cast<const f32x4*>(im + pl * RS + cg * 8);
      const f32x4 hi4 = *reinterpret_cast<const f32x4*>(im + pl * RS + cg * 8 + 4);
      float v[8] = {lo4[0] + bc[0], lo4[1] + bc[1], lo4[2] + bc[2], lo4[3] + bc[3],
                    hi4[0] + bc[4], hi4[1] + bc[5], hi4[2] + bc[6], hi4[3] + bc[7]};
      if (border) {
        if (has_res) {   // (both: not produced by the programs that run here; loaded in place)
          const int oy = r0 + pl / HW, ox = pl % HW;
          const int rc = oy - 1 < 0 ? 0 : (oy + 1 >= HW ? 2 : 1);
          const int cc = ox - 1 < 0 ? 0 : (ox + 1 >= HW ? 2 : 1);
          const float* bp = p.bias + (rc * 3 + cc) * p.npad + ch;
#pragma unroll
          for (int j = 0; j < 8; ++j) v[j] += bp[j];
        } else {
#pragma unroll
          for (int j = 0; j < 8; ++j) v[j] += pk[j];
        }
      }
      if (has_res && !pre_act) {
#pragma unroll
        for (int j = 0; j < 8; ++j) v[j] += pk[j];
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
        for (int j = 0; j < 8; ++j) v[j] += pk[j];
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
      if constexpr (SPLIT) *reinterpret_cast<f16x8*>(yp + p.ysplit) = yl;
    }
  }
}

// the instantiated shapes: IResNet's 14x14x256 (one image per workgroup, 8 x 1 waves of 32 channels x
// 14 rows) and 28x28x128 (7 rows per workgroup, 4 x 2 waves of 32 channels x 7 fragments); plain f16
// 28x28x128 at two workgroups per CU (its halo stage is 73 KB)
#define PC_HXI_14 14, 16, 14, 256, 256, 8, 1
#define PC_HXI_28 28, 32, 7, 128, 128, 4, 2
// 7x7x512 (the last stage, split only): one image per workgroup at pitch 9 - 63 slots in 4 fragments
// (77 % kept; a pitch of 16 would keep 44 %), 8 x 1 waves of 64 channels x 4 fragments
#define PC_HXI_7 7, 9, 7, 512, 512, 8, 1
// small-batch forms (a per-frame extract()'s ~12 ArcFace rows: 12 one-image workgroups would idle 244
// CUs, and conv_fast's 64x64 tile re-stages every pixel per tap and is bound by the LDS port): 32 output
// channels of 7 rows per workgroup - 16 workgroups per image (2 or 4 waves of 16 or 32 channels x 7
// fragments, or 4 at the 7x7 map), the rows' halo staged per 64-channel group as above. Same K order,
// MFMA order and epilogue: the same bits as every other form (tests/test_gpu_arcface.py)
#define PC_HXI_14S 14, 16, 7, 256, 32, 2, 1
#define PC_HXI_28S 28, 32, 7, 128, 32, 2, 2
#define PC_HXI_7S 7, 9, 7, 512, 32, 2, 1

// can a conv run here: one segment of C channels (split: X.C 2 C = [hi | lo]; plain f16: X.C C), dense,
// on an HW x HW map of an instantiated shape, C output channels written in the same form (dense), 3x3
// stride 1 pad 1, plain or same-size residual in the same form
int conv_hxi_ok(const ConvParams& p) {
  const ConvSeg& S = p.seg[0];
  const bool split = p.ysplit != 0;
  const int C = split ? S.C / 2 : S.C, w = split ? 2 : 1;
  const bool shape = (S.H == 14 && C == 256) || (S.H == 28 && C == 128) || (split && S.H == 7 && C == 512);
  return shape && p.nseg == 1 && S.cs == w * C && S.W == S.H && S.KH == 3 && S.KW == 3 && S.stride == 1 &&
         S.pad == 1 && p.OH == S.H && p.OW == S.H && p.npad == C && p.ycs == w * C && p.splitk == 1 && !p.out_f32 &&
         !p.yc8 && !p.rc8 && p.ktot == 9 * (split ? 3 : 1) * C && p.res_mode != RES_UP2 &&
         (p.res_mode == RES_NONE || (p.rsplit == (split ? C : 0) && p.rcs % 8 == 0)) && p.cwrite == C &&
         p.wfrag != nullptr && (!split || p.ysplit == C);
}

hipError_t conv_hxi_launch(const ConvParams& p, int small, hipStream_t s) {
  if (!conv_hxi_ok(p)) return hipErrorInvalidValue;
  const bool split = p.ysplit != 0;
  if (small) {   // (16 workgroups per image; split only)
    if (!split) return hipErrorInvalidValue;
    const dim3 grid(p.N * 16);
    if (p.OH == 7) hipLaunchKernelGGL((conv_hxi<PC_HXI_7S, true, 2>), grid, dim3(128), 0, s, p);
    else if (p.OH == 14) hipLaunchKernelGGL((conv_hxi<PC_HXI_14S, true, 2>), grid, dim3(128), 0, s, p);
    else hipLaunchKernelGGL((conv_hxi<PC_HXI_28S, true, 1>), grid, dim3(256), 0, s, p);
  } else if (p.OH == 7) {
    hipLaunchKernelGGL((conv_hxi<PC_HXI_7, true, 1>), dim3(p.N), dim3(512), 0, s, p);
  } else if (p.OH == 14) {
    // (half an image per workgroup at two per CU, 7 rows: 147.7 vs 145.3 us, profiles/r06t_hxi14_half_ab.txt)
    if (split) hipLaunchKernelGGL((conv_hxi<PC_HXI_14, true, 1>), dim3(p.N), dim3(512), 0, s, p);
    else hipLaunchKernelGGL((conv_hxi<PC_HXI_14, false, 1>), dim3(p.N), dim3(512), 0, s, p);
  } else {
    // (split: two workgroups per CU, one halo stage each, so one's epilogue runs under the other's MFMAs;
    // PC_HXI28_OCC=1 the 2-stage form)
    const bool occ1 = getenv("PC_HXI28_OCC") && atoi(getenv("PC_HXI28_OCC")) == 1;   // (per launch: A/B in one process)
    if (split && occ1) hipLaunchKernelGGL((conv_hxi<PC_HXI_28, true, 1>), dim3(p.N * 4), dim3(512), 0, s, p);
    else if (split) hipLaunchKernelGGL((conv_hxi<PC_HXI_28, true, 2>), dim3(p.N * 4), dim3(512), 0, s, p);
    else hipLaunchKernelGGL((conv_hxi<PC_HXI_28, false, 2>), dim3(p.N * 4), dim3(512), 0, s, p);
  }
  return hipGetLastError();
}

}  // namespace pc
