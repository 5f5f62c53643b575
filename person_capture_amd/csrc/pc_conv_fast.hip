// Statically scheduled implicit-GEMM convolution (gfx950).
//
// Same math, layouts and fused epilogue as conv_igemm (pc_conv.hip), but the
// K loop carries no data-dependent control flow, because the generic kernel's loop
// was measured to be scalar-issue bound (≈400 SALU + ≈90 branches per K-step from
// a run-time vmcnt switch and the nested tap iterator, ≈2.9k cycles per step against
// a 1k-cycle MFMA floor):
//
//  * every wave issues exactly NI = NIA + NIB LDS-DMA instructions per K-tile
//    (static_assert'ed tile shapes), and the loop always issues a tile - past the
//    last real tile it re-issues the last one into the ring slot nobody reads - so
//    the wait before each barrier is one compile-time s_waitcnt vmcnt((NSTAGE-2)*NI);
//  * the K-tile iterator (segment, tap row/col, channel block) advances with scalar
//    selects; the per-lane im2col source offset is recomputed every step from a
//    per-row window origin (≈6 VALU per staged row: bounds test, tap shift, select of
//    the zero-tail offset), so tap changes need no branch. The only branch in the
//    loop is the (once per launch) switch to the second K-segment;
//  * one raw s_barrier per K-tile; the DMA for tile k+NSTAGE-1 is issued right after
//    it and overlaps the MFMAs of tile k (cdna_hip_programming.md "Pipelining across
//    barriers"); the loop is unrolled by NSTAGE so every LDS address is static.
//
// LDS rows are ROWB bytes (one tap x ROWB of channels for the im2col side, one
// output channel x ROWB of K for the weights); 16-byte chunk c of row r sits at
// c ^ ((r >> 1) & (CHUNKS - 1)) - bank-conflict-free ds_read_b128 fragment reads (256-byte rows,
// which all start at bank 0: c ^ (r & 15)).
#include "pc_conv_common.h"

namespace pc {

template <int BC, int BP, int WC, int WP, int EPI_MAX = 131072>
__host__ __device__ constexpr int fast_epi_bytes() {
  // LDS image of conv_epilogue_lds (one or two passes)
  return BC * BP * 4 <= EPI_MAX ? BP * (BC + 4) * 4
                               : (WC >= 2 ? BP * (BC / 2 + 4) * 4 : (BP / 2) * (BC + 4) * 4);
}

// OCC: workgroups per CU the tile is sized for (LDS <= 160 KiB / OCC); with OCC = 2 one
// workgroup's epilogue and DMA waits overlap the other's MFMAs.
// SPLIT: the f16x3 epilogue (split output / residual).
// SX: fused f16x3 tiles over split inputs - a K tile is one (tap, hi channel block): the hi and
// lo pixel rows and the W_hi and W_lo weight rows are staged together and every k-substep issues
// W_hi*x_hi, W_lo*x_hi, W_hi*x_lo (2/3 of the staging and fragment reads of walking the virtual
// [hi, lo, hi] blocks as plain tiles). The weight rows keep the [W_hi, W_hi, W_lo] per-tap layout
// of the virtual K (the duplicate is skipped).
// C8 (with SX staging): f16c8 inputs - per K tile (32 or 64 channels) the f16 MFMAs for
// x_hi*W_hi, then one block-scaled e4m3 MFMA (v_mfma_scale_f32_16x16x128_f8f6f4) over the f8 rows
// [lo8 | hi8] x [W_hi8 | W_lo8] for x_lo*W_hi + x_hi*W_lo: 3 MFMA issues per tile where SX takes 6.
// WG (with SX, 64-byte K rows): the weight fragments come straight from global memory (L2) into
// registers, from the fragment-ordered copy p.wfrag (pc_api.cpp pack_wfrag), one K tile ahead; only the
// split pixel rows are staged, so the ring holds 4 stages and the LDS carries ~40 % fewer bytes per MFMA.
template <typename T, int BC, int BP, int ROWB, int WC, int WP, int NSTAGE, int OCC = 1, bool SPLIT = false,
          bool SX = false, bool C8 = false, bool WG = false>
__global__ __launch_bounds__(64 * WC * WP, (WC * WP * OCC + 3) / 4) void conv_fast(ConvParams p) {
  constexpr int NW = WC * WP;
  constexpr int NH = SX ? 2 : 1;              // staged halves per tile
  constexpr int ESZ = sizeof(T);
  constexpr int CHUNKS = ROWB / 16;
  constexpr int BKE = ROWB / ESZ;             // K elements per tile
  constexpr int RPI = 1024 / ROWB;            // LDS rows per DMA wave-instruction
  constexpr int NA = BC / RPI, NB = BP / RPI; // DMA instructions per tile (weights, im2col)
  static_assert(NA % NW == 0, "every wave must issue the same weight DMA count");
  // im2col rows: when NB is not a multiple of the wave count, the last round of DMAs of
  // the waves past NB goes to a trash area, so every wave still issues NIB (static vmcnt)
  constexpr int NIA = WG ? 0 : NA / NW, NIB = (NB + NW - 1) / NW, NI = NH * (NIA + NIB);
  static_assert(!WG || (SX && !C8 && ROWB == 64), "global weight fragments: fused f16x3 tiles, 64-byte K rows");
  constexpr int BCL = WG ? 0 : BC;            // weight rows staged per tile half
  static_assert(!SX || sizeof(T) == 2, "fused split tiles: f16 only");
  static_assert(!C8 || (SX && (ROWB == 128 || ROWB == 64)), "f16c8 tiles: fused split staging");
  constexpr int WTC = BC / WC, WTP = BP / WP;
  constexpr int TC = WTC / 16, TP = WTP / 16;
  constexpr int BUF = NH * (BCL + BP) * ROWB;
  constexpr int RING = NSTAGE * BUF;
  constexpr int EPI_MAX = OCC == 1 ? 131072 : 65536;
  constexpr int EPI = fast_epi_bytes<BC, BP, WC, WP, EPI_MAX>();
  constexpr int TRASH = (NB % NW || WG) ? NW * 1024 : 0;   // (WG: the prologue's filler DMAs too)
  constexpr int SMEM = RING + TRASH > EPI ? RING + TRASH : EPI;
  static_assert(SMEM * OCC <= 163840, "LDS");
  static_assert(WTC % 16 == 0 && WTP % 16 == 0, "wave tile");
  static_assert(ROWB == 64 || ROWB == 128 || (ROWB == 256 && ESZ == 2 && !SX), "K row width");
  // LDS chunk swizzle of row r (a fragment read's 16 rows hit 16 distinct 4-bank groups)
  auto swz = [](int r) __attribute__((always_inline)) { return ROWB == 256 ? (r & 15) : ((r >> 1) & (CHUNKS - 1)); };
  static_assert(NSTAGE >= 2, "ring depth");
  static_assert((NSTAGE - 2) * NI <= 63, "DMAs in flight exceed the vmcnt range");

  __shared__ __attribute__((aligned(16))) char smem[SMEM];

  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  __builtin_assume(wave >= 0 && wave < NW);
  const int wr = wave / WP, wc = wave % WP;
  const int nct = p.npad / BC;
  const int npt = (p.M + BP - 1) / BP;
  const int tile = xcd_remap(blockIdx.x, nct * npt);
  const int p0 = (tile / nct) * BP;
  const int c0 = (tile % nct) * BC;
  const int nk = p.kt_total;

  // ---- staging geometry ----
  const int lrow = lane / CHUNKS, pchunk = lane % CHUNKS;
  unsigned woff[NIA > 0 ? NIA : 1];
  static_for<NIA>([&](auto ic) __attribute__((always_inline)) {
    constexpr int i = decltype(ic)::value;
    const int r = (i * NW + wave) * RPI + lrow;
    woff[i] = (unsigned)((long long)(c0 + r) * p.ktot * ESZ) + ((pchunk ^ swz(r)) << 4);
  });
  // im2col rows: window origin (ih0, iw0) and byte offset of the staged row's output
  // pixel under the current segment (recomputed from the pixel index at a segment switch)
  int b_ih[NIB], b_iw[NIB];
  unsigned b_base[NIB];
  unsigned b_zero;   // zero tail + a chunk offset (any 16 zero bytes do; the tail is wider than a row)
  // current issue segment (scalars)
  const char* sx;
  int sH, sW, scs, sKW, scblk, svwrap;
  // buffer resources over the whole 32-bit offset range (every offset is < 4 GiB by the
  // planner's 32-bit offset rule, so the range check never fires)
  auto rsrc = [&](const void* base) __attribute__((always_inline)) {
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), (short)0, (int)0xffffffff, 0x00020000);
  };
  __amdgpu_buffer_rsrc_t xrs;
  auto load_seg = [&](const ConvSeg& S) __attribute__((always_inline)) {
    sx = reinterpret_cast<const char*>(S.x);
    xrs = rsrc(sx);
    sH = S.H; sW = S.W; scs = S.cs; sKW = S.KW; scblk = S.cblk; svwrap = S.vwrap;
    const int hw = p.OH * p.OW;
    static_for<NIB>([&](auto ic) __attribute__((always_inline)) {
      constexpr int i = decltype(ic)::value;
      const int r = (i * NW + wave) * RPI + lrow;
      const unsigned lc = (unsigned)((pchunk ^ swz(r)) << 4);
      const int q = p0 + r;
      const int n = q / hw, rem = q - n * hw;
      const int oh = q < p.M ? rem / p.OW : -(1 << 16);   // rows past M never pass the bounds test
      const int ow = rem - (rem / p.OW) * p.OW;
      b_ih[i] = oh * S.stride - S.pad;
      b_iw[i] = ow * S.stride - S.pad;
      b_base[i] = (unsigned)((n * S.H + b_ih[i]) * S.W + b_iw[i]) * (unsigned)(S.cs * ESZ) + lc;
      if constexpr (i == 0) b_zero = S.zero_off + lc;
    });
  };
  load_seg(p.seg[0]);
  int iseg = 0, ith = 0, itw = 0, icb = 0;
  const int seg0_kh = p.seg[0].KH;
  const int seg0_cb = p.seg[0].cblk;
  int sKH = p.seg[0].KH;
  // SX: weight K byte base of the current segment (segment 1 starts after segment 0's
  // KH*KW taps of 3 x cblk virtual blocks)
  int swk = 0;
  const int swk1 = SX ? p.seg[0].KH * p.seg[0].KW * 3 * p.seg[0].cblk * ROWB : 0;
  const __amdgpu_buffer_rsrc_t wrs = rsrc(p.w);

  // DMA of the current iterator position (K-tile index kt) into ring slot `slot`
  auto issue = [&](auto slotc, int kt) __attribute__((always_inline)) {
    constexpr int slot = decltype(slotc)::value;
    // MUBUF LDS-DMA (buffer_load ... lds), not FLAT global_load_lds: a pending FLAT op
    // counts in lgkmcnt too, so the compiler waited lgkmcnt(0) before the first MFMA of
    // every K-tile instead of counting the fragment reads
    // SX: W_hi of (tap, hi block icb) in the virtual per-tap layout [W_hi, W_hi, W_lo], W_lo 2 x cblk
    // blocks further
    const int wso = SX ? swk + ((ith * sKW + itw) * 3 * scblk + icb) * ROWB : kt * ROWB;
    static_for<NH>([&](auto hc) __attribute__((always_inline)) {
      constexpr int h = decltype(hc)::value;
      static_for<NIA>([&](auto ic) __attribute__((always_inline)) {
        constexpr int i = decltype(ic)::value;
        unsigned off = woff[i];
        asm volatile("" : "+v"(off));
        __builtin_amdgcn_raw_ptr_buffer_load_lds(wrs,
                                                 (lds_ptr_t)(smem + slot * BUF + h * BC * ROWB + (i * NW + wave) * 1024),
                                                 16, off, wso + h * 2 * scblk * ROWB, 0, 0);
      });
    });
    // f16x3 split input: virtual blocks [hi, lo, hi] -> physical [hi, lo] (a scalar select);
    // SX: hi block icb, then its lo block icb + vwrap
    const int xso = SX ? icb * ROWB : (svwrap && icb >= svwrap ? icb - svwrap : icb) * ROWB;
    const unsigned tapoff = (unsigned)((ith * sW + itw) * scs * ESZ);
    static_for<NH>([&](auto hc) __attribute__((always_inline)) {
      constexpr int h = decltype(hc)::value;
      static_for<NIB>([&](auto ic) __attribute__((always_inline)) {
        constexpr int i = decltype(ic)::value;
        const bool ok = (unsigned)(b_ih[i] + ith) < (unsigned)sH && (unsigned)(b_iw[i] + itw) < (unsigned)sW;
        unsigned off = ok ? b_base[i] + tapoff : b_zero;
        asm volatile("" : "+v"(off));
        const int dst = (NB % NW == 0 || i * NW + wave < NB)
                            ? slot * BUF + (NH * BCL + h * BP) * ROWB + (i * NW + wave) * 1024
                            : RING + wave * 1024;
        __builtin_amdgcn_raw_ptr_buffer_load_lds(xrs, (lds_ptr_t)(smem + dst), 16, off, xso + h * svwrap * ROWB, 0, 0);
      });
    });
  };
  // advance the issue iterator by one K-tile (no-op once the last tile was issued).
  // Plain tiles walk K tap-major (channel block fastest: the K order the chain / t2d kernels share
  // bit for bit). Fused split tiles walk it channel-group-major (the 9 taps of one group of 64 hi
  // channels - with its lo half - then the next group): a tap-major pass re-reads the tile's whole
  // split pixel rows per tap, which at 256x224 and 512 split channels (229 KB per workgroup, 7 MB
  // per XCD) no longer fits the L2 - every tap went back to HBM (r05 profile: 650 MB fetched per
  // 14x14x256 launch, 2.8x the tensor). Within a group and tap the tiles are in channel order, so
  // 64- and 128-byte K rows accumulate in the same order (ConvSeg::gt).
  int igt = 0;   // tile within the current group and tap
  int sgt = p.seg[0].gt > 0 ? p.seg[0].gt : 1;
  auto advance = [&](bool more) __attribute__((always_inline)) {
    if (!more) return;
    if constexpr (SX) {
      const int g1 = igt + 1;
      const bool w0 = g1 == sgt;
      igt = w0 ? 0 : g1;
      icb += w0 ? 1 - sgt : 1;   // back to the group's first tile at the next tap
      const int tw1 = itw + (w0 ? 1 : 0);
      const bool w1 = tw1 == sKW;
      itw = w1 ? 0 : tw1;
      const int th1 = ith + (w1 ? 1 : 0);
      const bool w2 = th1 == sKH;
      ith = w2 ? 0 : th1;
      icb += w2 ? sgt : 0;        // next group
      if (iseg == 0 && icb == seg0_cb) {   // once per launch, 2-segment convs only
        iseg = 1;
        icb = 0;
        swk = swk1;
        sKH = p.seg[1].KH;
        sgt = p.seg[1].gt > 0 ? p.seg[1].gt : 1;
        load_seg(p.seg[1]);
      }
    } else {
      const int cb1 = icb + 1;
      const bool w1 = cb1 == scblk;
      icb = w1 ? 0 : cb1;
      const int tw1 = itw + (w1 ? 1 : 0);
      const bool w2 = tw1 == sKW;
      itw = w2 ? 0 : tw1;
      ith += w2 ? 1 : 0;
      if (iseg == 0 && ith == seg0_kh) {   // once per launch, 2-segment convs only
        iseg = 1;
        ith = 0;
        swk = swk1;
        load_seg(p.seg[1]);
      }
    }
  };

  f32x4 acc[TC][TP];
#pragma unroll
  for (int a = 0; a < TC; ++a)
#pragma unroll
    for (int b = 0; b < TP; ++b) acc[a][b] = f32x4{0.f, 0.f, 0.f, 0.f};

  constexpr int KSTEPS = ESZ == 2 ? BKE / 32 : BKE / 4;
  const int fr = lane & 15;
  const int sw = swz(fr);
  const unsigned a_row = (wr * WTC + fr) * ROWB;
  const unsigned b_row = (NH * BCL + wc * WTP + fr) * ROWB;
  // Pinned two-k-substep schedule (f16, 128-byte K rows, two register sets fit beside the
  // accumulators): the 11 fragment reads of k-substep 0 go out first, the reads of k-substep 1
  // are interleaved one per MFMA with k-substep 0's MFMAs, and every MFMA waits (counted
  // lgkmcnt, inserted by the compiler from the pinned order) only for its own two fragments.
  // The compiler's own schedule waited lgkmcnt(0) for all of a substep's reads at the tile
  // start and again halfway through it (A fragments re-read into the same registers), which
  // exposed the LDS latency twice per K-tile on top of the barrier.
  constexpr bool PINNED = !SX && ESZ == 2 && KSTEPS <= 2 && NW % 4 == 0 && KSTEPS * (TC + TP) * 4 + TC * TP * 4 <= 200;
  auto compute_pinned = [&](auto slotc) __attribute__((always_inline)) {
    constexpr int slot = decltype(slotc)::value;
    const char* base = smem + slot * BUF;
    f16x8 fa[KSTEPS][TC], fb[KSTEPS][TP];
    auto rd = [&](int ks, int i) __attribute__((always_inline)) {   // read i: A0, B0..B(TP-1), A1..A(TC-1)
      const unsigned ko = ((ks * 4 + (lane >> 4)) ^ sw) << 4;
      if (i == 0) fa[ks][0] = *reinterpret_cast<const f16x8*>(base + a_row + ko);
      else if (i <= TP) fb[ks][i - 1] = *reinterpret_cast<const f16x8*>(base + b_row + ko + (i - 1) * 16 * ROWB);
      else fa[ks][i - TP] = *reinterpret_cast<const f16x8*>(base + a_row + ko + (i - TP) * 16 * ROWB);
    };
    static_for<TC + TP>([&](auto ic) __attribute__((always_inline)) { rd(0, decltype(ic)::value); });
    __builtin_amdgcn_sched_barrier(0);
    static_for<KSTEPS>([&](auto kc) __attribute__((always_inline)) {
      constexpr int ks = decltype(kc)::value;
      static_for<TC * TP>([&](auto mc) __attribute__((always_inline)) {
        constexpr int m = decltype(mc)::value, a = m / TP, b = m % TP;
        acc[a][b] = __builtin_amdgcn_mfma_f32_16x16x32_f16(fa[ks][a], fb[ks][b], acc[a][b], 0, 0, 0);
        if constexpr (ks + 1 < KSTEPS && m < TC + TP) rd(ks + 1, m);
        __builtin_amdgcn_sched_barrier(0);
      });
    });
  };
  // f16c8: per-lane E8M0 scale operands of the block-scaled MFMA. The scale VGPR of lane L covers K
  // block L >> 4 (K 32 (L >> 4) .. +31) of row / column L & 15 (measured, tools/mx_probe.hip); the f8
  // rows hold [lo8 | hi8] ([W_hi8 | W_lo8]) per 32 channels, so even K blocks are lo8, odd ones hi8
  const bool klo = ((lane >> 4) & 1) == 0;
  const int wsc = klo ? (p.wf8s & 0xff) : ((p.wf8s >> 8) & 0xff);
  const int xsc0 = klo ? (p.seg[0].f8s & 0xff) : ((p.seg[0].f8s >> 8) & 0xff);
  const int xsc1 = klo ? (p.seg[1].f8s & 0xff) : ((p.seg[1].f8s >> 8) & 0xff);
  const int kt0 = p.seg[0].kt;
  // WG: this wave's W_hi / W_lo fragments of the current K tile. Wave tiles of at most 2 row blocks
  // (the 8x1 / 4x2 layouts) double-buffer them by K-tile parity and load the next
  // tile's at the start of the current one; wider ones load the next tile's W_lo once the first pass
  // has consumed it, its W_hi after the last pass (one register set)
  // (MUBUF loads: tile offset in an SGPR, two lane offsets, fragment offsets as immediates)
  constexpr bool WDB = WG && TC <= 2;
  static_assert(!WDB || NSTAGE % 2 == 0, "K-tile parity of the weight buffers");
  f16x8 wgh[WDB ? 2 : 1][WG ? TC : 1], wgl[WDB ? 2 : 1][WG ? TC : 1];
  const __amdgpu_buffer_rsrc_t wgrs = rsrc(WG ? p.wfrag : p.w);
  const int wgoff0 = ((c0 + wr * WTC) / 16) * 2048 + lane * 16, wgoff1 = wgoff0 + 4096;
  const int wgstride = (p.npad / 16) * 2048;   // bytes per K tile
  auto wg_load = [&](f16x8* dst, int kt, auto hc) __attribute__((always_inline)) {
    constexpr int h = decltype(hc)::value;
    static_for<TC>([&](auto tc) __attribute__((always_inline)) {
      constexpr int t = decltype(tc)::value, o = t * 2048 + h * 1024;
      dst[t] = __builtin_bit_cast(f16x8, __builtin_amdgcn_raw_buffer_load_b128(wgrs, o < 4096 ? wgoff0 + o : wgoff1 + (o - 4096),
                                                                              kt * wgstride, 0));
    });
  };
  auto compute = [&](auto slotc, int tix) __attribute__((always_inline)) {
    constexpr int slot = decltype(slotc)::value;
    const char* base = smem + slot * BUF;
    if constexpr (PINNED) {
      compute_pinned(slotc);
      return;
    }
    if constexpr (C8) {
#pragma unroll
      for (int ks = 0; ks < KSTEPS; ++ks) {
        const unsigned ko = ((ks * 4 + (lane >> 4)) ^ sw) << 4;
        f16x8 fah[TC], fbh[TP];
#pragma unroll
        for (int t = 0; t < TC; ++t) fah[t] = *reinterpret_cast<const f16x8*>(base + a_row + ko + t * 16 * ROWB);
#pragma unroll
        for (int t = 0; t < TP; ++t) fbh[t] = *reinterpret_cast<const f16x8*>(base + b_row + ko + t * 16 * ROWB);
#pragma unroll
        for (int a = 0; a < TC; ++a)
#pragma unroll
          for (int b = 0; b < TP; ++b)
            acc[a][b] = __builtin_amdgcn_mfma_f32_16x16x32_f16(fah[a], fbh[b], acc[a][b], 0, 0, 0);
        if constexpr (TC * TP >= 16) __builtin_amdgcn_sched_barrier(0);
      }
      // f8 rows: a lane's 32 operand bytes are K 16g..16g+15 (chunk g) and 64+16g.. (chunk 4+g); a
      // 64-byte row (32 channels) fills K 0-63 and the MFMA's K 64-127 are zeros
      const unsigned k0 = ((lane >> 4) ^ sw) << 4, k1 = ((4 + (lane >> 4)) ^ sw) << 4;
      i32x8 a8[TC], b8[TP];
#pragma unroll
      for (int t = 0; t < TC; ++t) {
        const i32x4 u = *reinterpret_cast<const i32x4*>(base + a_row + BC * ROWB + k0 + t * 16 * ROWB);
        i32x4 v = i32x4{0, 0, 0, 0};
        if constexpr (ROWB == 128) v = *reinterpret_cast<const i32x4*>(base + a_row + BC * ROWB + k1 + t * 16 * ROWB);
        a8[t] = i32x8{u[0], u[1], u[2], u[3], v[0], v[1], v[2], v[3]};
      }
#pragma unroll
      for (int t = 0; t < TP; ++t) {
        const i32x4 u = *reinterpret_cast<const i32x4*>(base + b_row + BP * ROWB + k0 + t * 16 * ROWB);
        i32x4 v = i32x4{0, 0, 0, 0};
        if constexpr (ROWB == 128) v = *reinterpret_cast<const i32x4*>(base + b_row + BP * ROWB + k1 + t * 16 * ROWB);
        b8[t] = i32x8{u[0], u[1], u[2], u[3], v[0], v[1], v[2], v[3]};
      }
      const int xsc = tix < kt0 ? xsc0 : xsc1;
#pragma unroll
      for (int a = 0; a < TC; ++a)
#pragma unroll
        for (int b = 0; b < TP; ++b)
          acc[a][b] = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(a8[a], b8[b], acc[a][b], 0, 0, 0, wsc, 0, xsc);
      if constexpr (TC * TP >= 16) __builtin_amdgcn_sched_barrier(0);
      return;
    }
    // fused split tiles: per k-substep three passes over the fragment grid (a dependent MFMA is
    // TC*TP issues away), W_lo*x_hi, W_hi*x_hi, W_hi*x_lo - the same order in every SX form
    if constexpr (WG) {
      // per group of pixel fragments: x_hi fragments, W_lo*x_hi; x_lo reads behind W_hi*x_hi; W_hi*x_lo.
      // Wave tiles over 8 pixel fragments (the 8x1 layout's 32x224) walk them in two groups, so at
      // most 2 TPG fragments are live beside the accumulators; every accumulator still takes
      // W_lo*x_hi, W_hi*x_hi, W_hi*x_lo in that order (bit-identical across layouts)
      constexpr int TPG = TP > 8 && TP % 2 == 0 ? TP / 2 : TP;
      constexpr int NG = TP / TPG;
      constexpr int cur = WDB ? (slot & 1) : 0;
      const unsigned ko = ((lane >> 4) ^ sw) << 4;
      const int tn = tix + 1 < nk ? tix + 1 : nk - 1;
      if constexpr (WDB) {
        wg_load(wgl[cur ^ 1], tn, std::integral_constant<int, 1>{});
        wg_load(wgh[cur ^ 1], tn, std::integral_constant<int, 0>{});
      }
      static_for<NG>([&](auto gc) __attribute__((always_inline)) {
        constexpr int g = decltype(gc)::value, b0 = g * TPG;
        f16x8 fbh[TPG], fbl[TPG];
#pragma unroll
        for (int t = 0; t < TPG; ++t) fbh[t] = *reinterpret_cast<const f16x8*>(base + b_row + ko + (b0 + t) * 16 * ROWB);
#pragma unroll
        for (int a = 0; a < TC; ++a)
#pragma unroll
          for (int b = 0; b < TPG; ++b)
            acc[a][b0 + b] = __builtin_amdgcn_mfma_f32_16x16x32_f16(wgl[cur][a], fbh[b], acc[a][b0 + b], 0, 0, 0);
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int t = 0; t < TPG; ++t)
          fbl[t] = *reinterpret_cast<const f16x8*>(base + b_row + BP * ROWB + ko + (b0 + t) * 16 * ROWB);
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int a = 0; a < TC; ++a)
#pragma unroll
          for (int b = 0; b < TPG; ++b)
            acc[a][b0 + b] = __builtin_amdgcn_mfma_f32_16x16x32_f16(wgh[cur][a], fbh[b], acc[a][b0 + b], 0, 0, 0);
        __builtin_amdgcn_sched_barrier(0);
        if constexpr (!WDB && g + 1 == NG) wg_load(wgl[0], tn, std::integral_constant<int, 1>{});
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int a = 0; a < TC; ++a)
#pragma unroll
          for (int b = 0; b < TPG; ++b)
            acc[a][b0 + b] = __builtin_amdgcn_mfma_f32_16x16x32_f16(wgh[cur][a], fbl[b], acc[a][b0 + b], 0, 0, 0);
        __builtin_amdgcn_sched_barrier(0);
        if constexpr (!WDB && g + 1 == NG) wg_load(wgh[0], tn, std::integral_constant<int, 0>{});
        __builtin_amdgcn_sched_barrier(0);
      });
      return;
    }
    if constexpr (SX) {
#pragma unroll
      for (int ks = 0; ks < KSTEPS; ++ks) {
        const unsigned ko = ((ks * 4 + (lane >> 4)) ^ sw) << 4;
        f16x8 fah[TC], fal[TC], fbh[TP], fbl[TP];
#pragma unroll
        for (int t = 0; t < TC; ++t) {
          fah[t] = *reinterpret_cast<const f16x8*>(base + a_row + ko + t * 16 * ROWB);
          fal[t] = *reinterpret_cast<const f16x8*>(base + a_row + BC * ROWB + ko + t * 16 * ROWB);
        }
#pragma unroll
        for (int t = 0; t < TP; ++t) {
          fbh[t] = *reinterpret_cast<const f16x8*>(base + b_row + ko + t * 16 * ROWB);
          fbl[t] = *reinterpret_cast<const f16x8*>(base + b_row + BP * ROWB + ko + t * 16 * ROWB);
        }
#pragma unroll
        for (int a = 0; a < TC; ++a)
#pragma unroll
          for (int b = 0; b < TP; ++b)
            acc[a][b] = __builtin_amdgcn_mfma_f32_16x16x32_f16(fal[a], fbh[b], acc[a][b], 0, 0, 0);
#pragma unroll
        for (int a = 0; a < TC; ++a)
#pragma unroll
          for (int b = 0; b < TP; ++b)
            acc[a][b] = __builtin_amdgcn_mfma_f32_16x16x32_f16(fah[a], fbh[b], acc[a][b], 0, 0, 0);
#pragma unroll
        for (int a = 0; a < TC; ++a)
#pragma unroll
          for (int b = 0; b < TP; ++b)
            acc[a][b] = __builtin_amdgcn_mfma_f32_16x16x32_f16(fah[a], fbl[b], acc[a][b], 0, 0, 0);
        if constexpr (TC * TP >= 16) __builtin_amdgcn_sched_barrier(0);
      }
      return;
    }
#pragma unroll
    for (int ks = 0; ks < KSTEPS; ++ks) {
      if constexpr (ESZ == 2) {
        const unsigned ko = ((ks * 4 + (lane >> 4)) ^ sw) << 4;
        f16x8 fa[TC], fb[TP];
#pragma unroll
        for (int t = 0; t < TC; ++t) fa[t] = *reinterpret_cast<const f16x8*>(base + a_row + ko + t * 16 * ROWB);
#pragma unroll
        for (int t = 0; t < TP; ++t) fb[t] = *reinterpret_cast<const f16x8*>(base + b_row + ko + t * 16 * ROWB);
#pragma unroll
        for (int a = 0; a < TC; ++a)
#pragma unroll
          for (int b = 0; b < TP; ++b)
            acc[a][b] = __builtin_amdgcn_mfma_f32_16x16x32_f16(fa[a], fb[b], acc[a][b], 0, 0, 0);
        // 128x64 wave tiles: keep the next k-substep's fragment reads behind these MFMAs
        // (hoisting all of them needs 96 fragment VGPRs beside 128 accumulators -> spills)
        if constexpr (TC * TP >= 32) __builtin_amdgcn_sched_barrier(0);
      } else {
        // f32: K-substep ks is the 16-byte chunk ks (4 floats), lane group selects the float
        const unsigned kof = ((ks ^ sw) << 4) + ((lane >> 4) << 2);
        float fa[TC], fb[TP];
#pragma unroll
        for (int t = 0; t < TC; ++t) fa[t] = *reinterpret_cast<const float*>(base + a_row + kof + t * 16 * ROWB);
#pragma unroll
        for (int t = 0; t < TP; ++t) fb[t] = *reinterpret_cast<const float*>(base + b_row + kof + t * 16 * ROWB);
#pragma unroll
        for (int a = 0; a < TC; ++a)
#pragma unroll
          for (int b = 0; b < TP; ++b)
            acc[a][b] = __builtin_amdgcn_mfma_f32_16x16x4f32(fa[a], fb[b], acc[a][b], 0, 0, 0);
      }
    }
  };
  auto bar = [&]() __attribute__((always_inline)) {
    asm volatile("" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
  };

  // ---- prologue: tiles 0 .. NSTAGE-2 in flight ----
  int kiss = 0;   // next K-tile index the iterator points at
  // WG: every step issues NI DMAs and then 2 TC weight loads; the prologue keeps that pattern (2 TC
  // filler DMAs into the trash rows after each of its tile DMAs, tile 0's weights after the last),
  // so every step waits for the same count of younger loads, (NSTAGE-2) (NI + 2 TC) + 2 TC
  constexpr int WGL = WG ? 2 * TC : 0;
  static_for<NSTAGE - 1>([&](auto jc) __attribute__((always_inline)) {
    constexpr int j = decltype(jc)::value;
    issue(std::integral_constant<int, j>{}, kiss);
    const bool more = kiss + 1 < nk;
    advance(more);
    kiss += more ? 1 : 0;
    if constexpr (WG) {
      if constexpr (j + 2 < NSTAGE) {
        static_for<WGL>([&](auto) __attribute__((always_inline)) {
          unsigned off = b_zero;
          asm volatile("" : "+v"(off));
          __builtin_amdgcn_raw_ptr_buffer_load_lds(xrs, (lds_ptr_t)(smem + RING + wave * 1024), 16, off, 0, 0, 0);
        });
      } else {   // tile 0's weight fragments
        wg_load(wgl[0], 0, std::integral_constant<int, 1>{});
        wg_load(wgh[0], 0, std::integral_constant<int, 0>{});
      }
    }
  });
  int it = 0;
  // one step: retire tile `it`, refill the slot of tile it-1 with tile it+NSTAGE-1
  auto step = [&](auto jc, auto) __attribute__((always_inline)) {
    constexpr int j = decltype(jc)::value;
    constexpr int wcnt = (NSTAGE - 2) * (NI + WGL) + WGL;
    static_assert(wcnt <= 63, "vmcnt range");
    asm volatile("s_waitcnt vmcnt(%0)" ::"n"(wcnt) : "memory");
    bar();
    if (!(p.dbg & 1)) issue(std::integral_constant<int, (j + NSTAGE - 1) % NSTAGE>{}, kiss);   // dbg: tuning only
    const bool more = kiss + 1 < nk;
    advance(more);
    kiss += more ? 1 : 0;
    if (!(p.dbg & 2)) compute(std::integral_constant<int, j>{}, it + j);
  };
  if (p.dbg & 8) return;   // tuning only: prologue only
  using later_t = std::integral_constant<bool, false>;
  for (; it + NSTAGE <= nk; it += NSTAGE)
    static_for<NSTAGE>([&](auto jc) __attribute__((always_inline)) { step(jc, later_t{}); });
  static_for<NSTAGE - 1>([&](auto jc) __attribute__((always_inline)) {
    if (it + decltype(jc)::value < nk) step(jc, later_t{});
  });

  // drain the (dummy) tail DMAs and every wave's last reads before the LDS is reused
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (p.dbg & 4) return;   // tuning only: skip the epilogue
  if constexpr (((BC / 8) & (BC / 8 - 1)) == 0 && ((BC / 16) & (BC / 16 - 1)) == 0)
    conv_epilogue_lds<T, BC, BP, WC, WP, EPI_MAX, 8, SPLIT>(p, acc, c0, p0, wr, wc, lane, smem);
  else   // 96 / 224 channel tiles: per-fragment stores
    conv_epilogue<T, TC, TP, WTC, WTP>(p, acc, c0, p0, wr, wc, lane, 0);
}

#ifndef PC_FAST_KERNEL_ONLY   // (tools/kernel_regs.sh: the kernel template alone, for register checks)
// tile shapes whose DMA count divides evenly over the waves at this row width
template <int BC, int BP, int ROWB, int NW>
constexpr bool fast_valid() {
  return (BC / (1024 / ROWB)) % NW == 0 && BP % (1024 / ROWB) == 0;
}

// ---------------------------------------------------------------------------
// host side: tile table (keep kFastCfgs and launch_fast_t in sync)
// ---------------------------------------------------------------------------
struct FastCfg { int bc, bp, nw; };
static const FastCfg kFastCfgs[] = {
    {256, 256, 8},   // 0: 2x4 waves, 128x64 per wave, 2 stages
    {128, 256, 8},   // 1: 2x4 waves, 64x64 per wave, 3 stages (ROWB 64: 4)
    {256, 128, 8},   // 2: 4x2 waves, 64x64 per wave, 3 stages
    {128, 128, 4},   // 3: 2x2 waves, 64x64 per wave, 3 stages
    {64, 256, 4},    // 4: 1x4 waves, 64x64 per wave, 3 stages
    {96, 256, 4},    // 5: 1x4 waves, 96x64 per wave, 3 stages
    {64, 512, 8},    // 6: 1x8 waves, 64x64 per wave, 3 stages
    {32, 256, 4},    // 7: 1x4 waves, 32x64 per wave, 3 stages
    {224, 128, 4},   // 8: 2x2 waves, 112x64 per wave, 2 stages
    {128, 512, 8},   // 9: 2x4 waves, 64x128 per wave, 2 stages (ROWB 64: 4)
    {128, 256, 4},   // 10: 2x2 waves, 64x128 per wave, ROWB 64 only, 3 stages, 2 workgroups per CU
    {96, 384, 6},    // 11: 1x6 waves, 96x64 per wave (96-channel trunks at 64-byte K rows)
    {32, 256, 2},    // 12: 1x2 waves, 32x128 per wave (detector heads, npad 32)
    {256, 224, 8},   // 13: 4x2 waves, 64x112 per wave: 50176-pixel layers (b256 14x14) fill 224 CUs
    {128, 224, 4},   // 14: 2x2 waves, 64x112 per wave, ROWB 64 only, 3 stages, 2 workgroups per CU
    // small-batch plans only (pc_api.cpp plan_conv): a per-frame extract()'s 12 ArcFace rows give a
    // 14x14x256 conv 2352 output pixels - 80 of the tiles above; these cover the CUs. A small tile's
    // K loop is a chain of L2/HBM round trips (a few MFMAs per K tile), so its ring is deep: the
    // DMA runs NSTAGE-1 tiles ahead (r04: 3 stages left the 64x64 tile at ~18 us per 14x14x256
    // conv of 12 images, 36 K tiles x ~0.5 us of exposed latency)
    {64, 64, 4},     // 15: 2x2 waves, 32x32 per wave, 8 stages
    {64, 128, 4},    // 16: 2x2 waves, 32x64 per wave, 6 stages
    {128, 64, 4},    // 17: 2x2 waves, 64x32 per wave, 6 stages
    {32, 64, 2},     // 18: 1x2 waves, 32x32 per wave, 8 stages (npad 32 / 96 / 160 / 224)
    {96, 64, 2},     // 19: 1x2 waves, 96x32 per wave, 7 stages (ROWB 64: 8)
    // whole-width tiles for SCRFD's 224- and 96-channel layers (npad % 64 == 32: the other
    // tiles split them into 32-channel slices that re-stage every pixel 7 or 3 times)
    {224, 64, 2},    // 20: 1x2 waves, 224x32 per wave
    {96, 128, 2},    // 21: 1x2 waves, 96x64 per wave
};
static const int kNumFastCfgs = sizeof(kFastCfgs) / sizeof(kFastCfgs[0]);

int conv_fast_num_cfgs() { return kNumFastCfgs; }

int conv_fast_tile(int cfg, int* bc, int* bp) {
  if (cfg < 0 || cfg >= kNumFastCfgs) return 0;
  *bc = kFastCfgs[cfg].bc;
  *bp = kFastCfgs[cfg].bp;
  return 1;
}

// fused split tiles: NS stages of the doubled tile (+ trash rows) fit the LDS
template <int BC, int BP, int ROWB, int NW, int OCC = 1, int NS = 2>
constexpr bool fast_sx_fits() {
  constexpr int RING = NS * 2 * (BC + BP) * ROWB + ((BP / (1024 / ROWB)) % NW ? NW * 1024 : 0);
  return OCC == 1 && RING <= 163840;
}
// ring depth of a fused split tile: two stages, or the small-batch tiles' deep rings bounded by
// the LDS and by the 6-bit vmcnt ((NS - 2) x DMAs in flight per wave <= 63)
template <int BC, int BP, int ROWB, int NW, int NSTAGE>
constexpr int fast_sx_stages() {
  constexpr int NI = 2 * (BC / (1024 / ROWB) / NW + (BP / (1024 / ROWB) + NW - 1) / NW);
  // (the deep-ring small-batch tiles only: 4 stages on the 32x256 split tiles cost SCRFD-x3 b64
  // 13.0 -> 13.7 ms, r04l, against the 2 of round 4's first SX build)
  int ns = NSTAGE >= 6 ? NSTAGE : 2;
  while (ns > 2 && ((ns - 2) * NI > 63 || ns * 2 * (BC + BP) * ROWB + ((BP / (1024 / ROWB)) % NW ? NW * 1024 : 0) > 163840))
    --ns;
  return ns;
}

// WG tiles (fused f16x3, weights from global memory): 4 stages of the split pixel rows (+ trash
// rows) and the epilogue image fit the LDS, and the loads in flight stay in the vmcnt range
template <int BC, int BP, int WC, int WP>
constexpr bool fast_wg_fits() {
  constexpr int NW = WC * WP, RPI = 16, NB = BP / RPI;
  constexpr int ring = 4 * 2 * BP * 64 + (NB % NW ? NW * 1024 : 0);
  constexpr int NI = 2 * ((NB + NW - 1) / NW), WGL = 2 * (BC / WC / 16);
  return BP % RPI == 0 && (BC / WC) % 16 == 0 && ring <= 163840 && fast_epi_bytes<BC, BP, WC, WP>() <= 163840 &&
         2 * (NI + WGL) + WGL <= 63;
}

// power-of-two channel tiles: the LDS epilogue (the only one that writes f16c8 outputs)
template <int BC>
constexpr bool LDS_EPI_OK() { return ((BC / 8) & (BC / 8 - 1)) == 0 && ((BC / 16) & (BC / 16 - 1)) == 0; }

// (read per launch, like PC_CONV_DBG: the A/B test switches it inside one process)
static int wg_layout() {
  const char* e = getenv("PC_WG_LAYOUT");
  return e ? atoi(e) : 1;
}

template <typename T, int BC, int BP, int ROWB, int WC, int WP, int NSTAGE, int OCC = 1>
static hipError_t launch_fast_cfg(const ConvParams& p, hipStream_t s) {
  if constexpr (!fast_valid<BC, BP, ROWB, WC * WP>()) {
    return hipErrorInvalidValue;
  } else {
    const int nwg = (p.M + BP - 1) / BP * (p.npad / BC);
    if (p.sx) {   // fused f16x3 / f16c8 tiles: always the split epilogue
      if (p.wfrag && !p.c8) {   // weight fragments from global memory: 4 stages of pixel rows
        // wave layout: 8x1 waves of 32x224 on 256x224, 4x2 of 32x128 on 128x256 -
        // each weight fragment is loaded by 1 or 2 waves instead of 2 or 4 (PC_WG_LAYOUT=0: the
        // cfg table's 4x2 / 2x4 layouts, for A/B; same accumulation order, bit-identical)
        constexpr int WC2 = BC == 256 ? 8 : 4, WP2 = BC == 256 ? 1 : 2;
        if constexpr (sizeof(T) == 2 && ROWB == 64 && OCC == 1 && ((BC == 256 && BP == 224) || (BC == 128 && BP == 256)) &&
                      fast_wg_fits<BC, BP, WC, WP>() && fast_wg_fits<BC, BP, WC2, WP2>()) {
          if (wg_layout())
            hipLaunchKernelGGL((conv_fast<T, BC, BP, ROWB, WC2, WP2, 4, 1, true, true, false, true>), dim3(nwg),
                               dim3(64 * WC2 * WP2), 0, s, p);
          else
            hipLaunchKernelGGL((conv_fast<T, BC, BP, ROWB, WC, WP, 4, 1, true, true, false, true>), dim3(nwg),
                               dim3(64 * WC * WP), 0, s, p);
          return hipGetLastError();
        } else {
          return hipErrorInvalidValue;
        }
      }
      constexpr int NS = fast_sx_stages<BC, BP, ROWB, WC * WP, NSTAGE>();
      if constexpr (sizeof(T) == 2 && ROWB != 256 && fast_sx_fits<BC, BP, ROWB, WC * WP, OCC, NS>()) {
        if (p.c8) {
          if constexpr (LDS_EPI_OK<BC>()) {
            hipLaunchKernelGGL((conv_fast<T, BC, BP, ROWB, WC, WP, NS, OCC, true, true, true>), dim3(nwg),
                               dim3(64 * WC * WP), 0, s, p);
            return hipGetLastError();
          } else {
            return hipErrorInvalidValue;
          }
        }
        hipLaunchKernelGGL((conv_fast<T, BC, BP, ROWB, WC, WP, NS, OCC, true, true>), dim3(nwg), dim3(64 * WC * WP), 0,
                           s, p);
        return hipGetLastError();
      } else {
        return hipErrorInvalidValue;
      }
    }
    // the split epilogue only where it can differ: f16 power-of-two channel tiles (the others
    // take the per-fragment epilogue, which reads the split flags at run time)
    constexpr bool LDS_EPI = ((BC / 8) & (BC / 8 - 1)) == 0 && ((BC / 16) & (BC / 16 - 1)) == 0;
    if constexpr (sizeof(T) == 2 && LDS_EPI) {
      if (p.ysplit || p.rsplit) {
        hipLaunchKernelGGL((conv_fast<T, BC, BP, ROWB, WC, WP, NSTAGE, OCC, true>), dim3(nwg), dim3(64 * WC * WP), 0,
                           s, p);
        return hipGetLastError();
      }
    }
    hipLaunchKernelGGL((conv_fast<T, BC, BP, ROWB, WC, WP, NSTAGE, OCC>), dim3(nwg), dim3(64 * WC * WP), 0, s, p);
    return hipGetLastError();
  }
}

template <typename T, int ROWB>
static hipError_t launch_fast_t(const ConvParams& p, int cfg, hipStream_t s) {
  constexpr int S3 = ROWB == 128 ? 3 : 4;
  switch (cfg) {
    case 0: return launch_fast_cfg<T, 256, 256, ROWB, 2, 4, ROWB == 128 ? 2 : 4>(p, s);
    case 1: return launch_fast_cfg<T, 128, 256, ROWB, 2, 4, S3>(p, s);
    case 2: return launch_fast_cfg<T, 256, 128, ROWB, 4, 2, S3>(p, s);
    case 3: return launch_fast_cfg<T, 128, 128, ROWB, 2, 2, S3>(p, s);
    case 4: return launch_fast_cfg<T, 64, 256, ROWB, 1, 4, S3>(p, s);
    case 5: return launch_fast_cfg<T, 96, 256, ROWB, 1, 4, S3>(p, s);
    case 6: return launch_fast_cfg<T, 64, 512, ROWB, 1, 8, ROWB == 128 ? 2 : 4>(p, s);
    case 7: return launch_fast_cfg<T, 32, 256, ROWB, 1, 4, S3>(p, s);
    case 8: return launch_fast_cfg<T, 224, 128, ROWB, 2, 2, S3>(p, s);
    case 9: return launch_fast_cfg<T, 128, 512, ROWB, 2, 4, ROWB == 128 ? 2 : 4>(p, s);
    case 10:
      if constexpr (ROWB == 64) return launch_fast_cfg<T, 128, 256, 64, 2, 2, 3, 2>(p, s);
      else return hipErrorInvalidValue;
    case 11: return launch_fast_cfg<T, 96, 384, ROWB, 1, 6, ROWB == 128 ? 2 : 4>(p, s);
    case 12: return launch_fast_cfg<T, 32, 256, ROWB, 1, 2, ROWB == 128 ? 3 : 4>(p, s);
    case 13: return launch_fast_cfg<T, 256, 224, ROWB, 4, 2, ROWB == 128 ? 2 : 4>(p, s);
    case 14:
      if constexpr (ROWB == 64) return launch_fast_cfg<T, 128, 224, 64, 2, 2, 3, 2>(p, s);
      else return hipErrorInvalidValue;
    case 15: return launch_fast_cfg<T, 64, 64, ROWB, 2, 2, 8>(p, s);
    case 16: return launch_fast_cfg<T, 64, 128, ROWB, 2, 2, 6>(p, s);
    case 17: return launch_fast_cfg<T, 128, 64, ROWB, 2, 2, 6>(p, s);
    case 18: return launch_fast_cfg<T, 32, 64, ROWB, 1, 2, 8>(p, s);
    case 19: return launch_fast_cfg<T, 96, 64, ROWB, 1, 2, ROWB == 128 ? 7 : 8>(p, s);
    case 20: return launch_fast_cfg<T, 224, 64, ROWB, 1, 2, S3>(p, s);
    case 21: return launch_fast_cfg<T, 96, 128, ROWB, 1, 2, S3>(p, s);
    default: return hipErrorInvalidValue;
  }
}

// 256-byte K rows (128 f16 channels, half the K tiles of 128-byte rows): the small-batch tiles,
// whose K loop is a chain of barrier-separated K tiles
static hipError_t launch_fast_256(const ConvParams& p, int cfg, hipStream_t s) {
  switch (cfg) {
    case 15: return launch_fast_cfg<f16, 64, 64, 256, 2, 2, 4>(p, s);
    case 16: return launch_fast_cfg<f16, 64, 128, 256, 2, 2, 3>(p, s);
    case 17: return launch_fast_cfg<f16, 128, 64, 256, 2, 2, 3>(p, s);
    default: return hipErrorInvalidValue;
  }
}

// can cfg run fused f16x3 split tiles (SX) at K rows of rowb bytes?
int conv_fast_valid_sx(int cfg, int rowb) {
  if (cfg < 0 || cfg >= kNumFastCfgs || (rowb != 64 && rowb != 128)) return 0;
  if (cfg == 10 || cfg == 14) return 0;   // sized for 2 workgroups per CU
  const FastCfg& c = kFastCfgs[cfg];
  const int rpi = 1024 / rowb;
  if ((c.bc / rpi) % c.nw || c.bp % rpi) return 0;
  const int ring = 2 * 2 * (c.bc + c.bp) * rowb + ((c.bp / rpi) % c.nw ? c.nw * 1024 : 0);
  return ring <= 163840;
}

// can cfg run the WG form (fused f16x3 tiles with register weight fragments) at 64-byte K rows?
int conv_fast_valid_wg(int cfg) {
  if (cfg < 0 || cfg >= kNumFastCfgs || !conv_fast_valid_sx(cfg, 64)) return 0;
  switch (cfg) {   // the instantiated WG tiles
    case 1: return fast_wg_fits<128, 256, 2, 4>();
    case 13: return fast_wg_fits<256, 224, 4, 2>();
    default: return 0;
  }
}

// can cfg run f16c8 convs at K rows of rowb bytes (fused split staging, LDS epilogue)?
int conv_fast_valid_c8(int cfg, int rowb) {
  if (!conv_fast_valid_sx(cfg, rowb)) return 0;
  const int bc = kFastCfgs[cfg].bc;
  return ((bc / 8) & (bc / 8 - 1)) == 0 && ((bc / 16) & (bc / 16 - 1)) == 0;
}

// can cfg run convs whose K rows are rowb bytes?
int conv_fast_valid(int cfg, int rowb) {
  if (rowb == 256) return cfg >= 15 && cfg <= 17;   // f16 only (conv_fast_launch)
  if (cfg < 0 || cfg >= kNumFastCfgs || (rowb != 64 && rowb != 128)) return 0;
  const FastCfg& c = kFastCfgs[cfg];
  if ((cfg == 10 || cfg == 14) && rowb != 64) return 0;   // sized for 2 workgroups per CU at 64-byte K rows
  const int rpi = 1024 / rowb;
  return (c.bc / rpi) % c.nw == 0 && c.bp % rpi == 0;
}

hipError_t conv_fast_launch(int f32, int rowb, int cfg, const ConvParams& p, hipStream_t s) {
  if (cfg < 0 || cfg >= kNumFastCfgs || p.splitk != 1 || p.npad % kFastCfgs[cfg].bc || p.nseg < 1 || p.nseg > 2 ||
      (rowb != 64 && rowb != 128 && rowb != 256))
    return hipErrorInvalidValue;
  if (rowb == 256) return f32 || p.sx ? hipErrorInvalidValue : launch_fast_256(p, cfg, s);
  if (f32) return rowb == 128 ? launch_fast_t<float, 128>(p, cfg, s) : launch_fast_t<float, 64>(p, cfg, s);
  return rowb == 128 ? launch_fast_t<f16, 128>(p, cfg, s) : launch_fast_t<f16, 64>(p, cfg, s);
}

#endif  // PC_FAST_KERNEL_ONLY
}  // namespace pc
