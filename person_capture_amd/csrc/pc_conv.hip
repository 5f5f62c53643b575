// Implicit-GEMM convolution engine for gfx950 (CDNA4).
//
// One kernel template runs every dense conv of the identity hot path
// (IResNet ArcFace trunk, SCRFD backbone/neck/heads, the embedding FC as a
// KxK "valid" conv): out[pixel][cout] = sum_k X_im2col[pixel][k] * W[cout][k].
//
// Layout: activations NHWC with channels padded to the K-tile
// width, weights [cout_pad][K] with K = segment-major, tap-major, channel-minor,
// BN scales folded in. A workgroup (4 waves, 2x2) owns a BC(channels) x BP(pixels)
// output tile; each K-tile is one conv tap x ROWB bytes of channels, so every
// staged LDS row is one contiguous 64/128-byte run of a single pixel (im2col
// gather) or of a single output channel (weights). Rows are moved HBM->LDS with
// 16-byte global_load_lds (LDS-DMA, no VGPR round trip); padding taps point at a
// zero page so the staging is branch-free. The LDS image is XOR-swizzled on the
// source side so the ds_read_b128 fragment reads are bank-conflict free
// (verified by brute force over the gfx950 16-lane groups).
// MFMA: v_mfma_f32_16x16x32_f16 (fast path) or v_mfma_f32_16x16x4_f32 (exact
// f32 parity path); fp32 accumulation; fused epilogue = bias (optionally the
// 9-class border table of a folded pre-BN) + ReLU/PReLU/SiLU + residual (same
// pixel or nearest-2x upsampled) in either order, or split-K fp32 partials.
//
// A second, optional K-segment lets a residual block's shortcut projection
// (IResNet downsample 1x1/s2, ResNetV1e avg-down == 2x2/s2 conv) accumulate into
// the same tile, so shortcut + main branch cost one launch and one output write.
#include "pc_conv_common.h"

namespace pc {

// BC x BP output tile per workgroup of WC x WP waves; NSTAGE-deep LDS ring of
// K-tiles filled by LDS-DMA, tile k+NSTAGE-1 issued right after the barrier that
// retires tile k (counted vmcnt, one raw s_barrier per K-tile, no drain to 0).
template <typename T, int BC, int BP, int ROWB, int WC, int WP, int NSTAGE>
__global__ __launch_bounds__(64 * WC * WP, 1) void conv_igemm(ConvParams p) {
  constexpr int NW = WC * WP;
  constexpr int CHUNKS = ROWB / 16;       // 16-byte chunks per LDS row
  constexpr int BKE = ROWB / sizeof(T);   // K elements per tile
  constexpr int ROWS = BC + BP;
  constexpr int RPI = 1024 / ROWB;        // LDS rows written by one wave-instruction
  constexpr int NTOT = ROWS / RPI;        // wave-instructions per tile
  constexpr int NI = (NTOT + NW - 1) / NW;
  constexpr int WTC = BC / WC, WTP = BP / WP;
  constexpr int TC = WTC / 16, TP = WTP / 16;
  constexpr int BUF = ROWS * ROWB;
  static_assert(ROWS % RPI == 0, "tile rows");
  static_assert(WTC % 16 == 0 && WTP % 16 == 0, "wave tile");
  static_assert(NSTAGE >= 2, "ring depth");

  __shared__ __attribute__((aligned(16))) char smem[NSTAGE * BUF];

  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);   // wave-uniform (SGPR)
  const int wr = wave / WP, wc = wave % WP;
  const int nct = p.npad / BC;
  const int npt = (p.M + BP - 1) / BP;
  const int tile = xcd_remap(blockIdx.x, nct * npt);
  const int p0 = (tile / nct) * BP;
  const int c0 = (tile % nct) * BC;
  const int z = blockIdx.z;
  const int myni = NI - ((NTOT % NW) != 0 && wave >= (NTOT % NW) ? 1 : 0);

  // ---- split-K range ----
  const int per = (p.kt_total + p.splitk - 1) / p.splitk;
  const int kb = z * per;
  const int ke = min(p.kt_total, kb + per);
  const int nk = ke > kb ? ke - kb : 0;

  // ---- K iterator: (segment, tap row th, tap col tw, channel block cb), all scalar ----
  int seg = 0, th = 0, tw = 0, cb = 0;
  {
    int rem = kb;
    if (p.nseg > 1 && rem >= p.seg[0].kt) { rem -= p.seg[0].kt; seg = 1; }
    // p.seg is only ever indexed by constants: a runtime index would copy the whole
    // kernel-argument struct to scratch
    const int cbl = seg ? p.seg[1].cblk : p.seg[0].cblk;
    const int kw = seg ? p.seg[1].KW : p.seg[0].KW;
    const int tap = rem / cbl;
    cb = rem - tap * cbl;
    th = tap / kw;
    tw = tap - th * kw;
  }
  // current segment, cached in scalars
  const char* sx;
  // MUBUF LDS-DMA (a pending FLAT global_load_lds counts in lgkmcnt and forces lgkmcnt(0)
  // before the fragment reads' consumers)
  __amdgpu_buffer_rsrc_t xrs;
  const __amdgpu_buffer_rsrc_t wrs =
      __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(p.w), (short)0, (int)0xffffffff, 0x00020000);
  int sH, sW, scs, sKH, sKW, sstr, spad, scblk, svwrap;
  unsigned szero;
  auto load_seg = [&](const ConvSeg& S) __attribute__((always_inline)) {
    sx = reinterpret_cast<const char*>(S.x);
    xrs = __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(S.x), (short)0, (int)0xffffffff, 0x00020000);
    sH = S.H; sW = S.W; scs = S.cs;
    sKH = S.KH; sKW = S.KW; sstr = S.stride; spad = S.pad;
    scblk = S.cblk; szero = S.zero_off; svwrap = S.vwrap;
  };
  if (seg) load_seg(p.seg[1]);
  else load_seg(p.seg[0]);

  // ---- per-lane staging geometry ----
  // Every staged 16-byte chunk is addressed as (wave-uniform SGPR base) + (per-lane
  // 32-bit offset). The per-row offset of the current tap (`xcur`) is recomputed only
  // when the tap changes; the channel block rides in the scalar base. A tap that
  // falls in the zero padding points at the zero tail the executor keeps behind
  // every activation buffer (ConvSeg::zero_off), which is wider than any pixel row.
  constexpr int ESZ = sizeof(T);
  const int lrow = lane / CHUNKS;
  const int pchunk = lane % CHUNKS;
  int x_ih[NI], x_iw[NI], x_n[NI];  // window origin of this lane's output pixel (current segment)
  unsigned woff[NI], xpix[NI], zlane[NI], xcur[NI];
  int x_oh[NI], x_ow[NI];
  static_for<NI>([&](auto ic) __attribute__((always_inline)) {
    constexpr int i = decltype(ic)::value;
    const int g = i * NW + wave;
    const int r = g * RPI + lrow;
    const int lc = pchunk ^ ((r >> 1) & (CHUNKS - 1));
    x_n[i] = -1; x_oh[i] = 0; x_ow[i] = 0; x_ih[i] = 0; x_iw[i] = 0;
    woff[i] = 0; xpix[i] = 0; zlane[i] = 0; xcur[i] = 0;
    if (g < NTOT && g * RPI < BC) {
      woff[i] = (unsigned)((long long)(c0 + r) * p.ktot * ESZ) + lc * 16;
    } else if (g < NTOT) {
      const int pix = p0 + (r - BC);
      if (pix < p.M) {
        const int hw = p.OH * p.OW;
        const int n = (p.dbg & 4) ? 0 : pix / hw;
        const int rem = pix % hw;
        x_n[i] = n;
        x_oh[i] = rem / p.OW;
        x_ow[i] = rem - x_oh[i] * p.OW;
      }
    }
  });
  auto prep_seg = [&]() __attribute__((always_inline)) {   // per-lane window origins for the current segment
    static_for<NI>([&](auto ic) __attribute__((always_inline)) {
      constexpr int i = decltype(ic)::value;
      const int g = i * NW + wave;
      if (g < NTOT && g * RPI >= BC) {
        const int r = g * RPI + lrow;
        const int lc = pchunk ^ ((r >> 1) & (CHUNKS - 1));
        zlane[i] = szero + lc * 16;
        x_ih[i] = x_oh[i] * sstr - spad;
        x_iw[i] = x_ow[i] * sstr - spad;
        xpix[i] = (unsigned)((((long long)max(x_n[i], 0) * sH + x_ih[i]) * sW + x_iw[i]) * scs * ESZ) + lc * 16;
      }
    });
  };
  auto prep_tap = [&]() __attribute__((always_inline)) {   // per-lane source offsets for tap (th, tw)
    const unsigned tapoff = (unsigned)((th * sW + tw) * scs * ESZ);
    static_for<NI>([&](auto ic) __attribute__((always_inline)) {
      constexpr int i = decltype(ic)::value;
      const int g = i * NW + wave;
      if (g < NTOT && g * RPI >= BC) {
        const bool ok = x_n[i] >= 0 && (unsigned)(x_ih[i] + th) < (unsigned)sH &&
                        (unsigned)(x_iw[i] + tw) < (unsigned)sW;
        xcur[i] = ok ? xpix[i] + tapoff : zlane[i];
      }
    });
  };
  prep_seg();
  prep_tap();

  auto stage = [&](auto bufc, int ktl) __attribute__((always_inline)) {
    constexpr int buf = decltype(bufc)::value;
    // f16x3 split input: virtual channel blocks [hi, lo, hi] read physical [hi, lo]
    const int xso = (svwrap && cb >= svwrap ? cb - svwrap : cb) * (BKE * ESZ), wso = ktl * (BKE * ESZ);
    static_for<NI>([&](auto ic) __attribute__((always_inline)) {
      constexpr int i = decltype(ic)::value;
      const int g = i * NW + wave;
      if (g < NTOT) {
        unsigned off = g * RPI < BC ? woff[i] : xcur[i];
        asm volatile("" : "+v"(off));   // keep the 32-bit offset in-block (SGPR base + VGPR offset form)
        char* dst = smem + buf * BUF + g * 1024;
        if (g * RPI < BC)
          __builtin_amdgcn_raw_ptr_buffer_load_lds(wrs, (lds_ptr_t)dst, 16, off, wso, 0, 0);
        else
          __builtin_amdgcn_raw_ptr_buffer_load_lds(xrs, (lds_ptr_t)dst, 16, off, xso, 0, 0);
      }
    });
  };
  auto advance = [&]() __attribute__((always_inline)) {
    if (++cb < scblk) return;
    cb = 0;
    if (++tw == sKW) {
      tw = 0;
      if (++th == sKH) {
        th = 0;
        if (++seg >= p.nseg) return;
        load_seg(p.seg[1]);   // segments only advance 0 -> 1
        prep_seg();
      }
    }
    prep_tap();
  };

  f32x4 acc[TC][TP];
#pragma unroll
  for (int a = 0; a < TC; ++a)
#pragma unroll
    for (int b = 0; b < TP; ++b) acc[a][b] = f32x4{0.f, 0.f, 0.f, 0.f};

  // fragment read addresses: row = tile base (multiple of 16) + (lane & 15), so the
  // swizzle term ((row >> 1) & (CHUNKS-1)) depends on the lane only; every ds_read is
  // one per-lane base + a compile-time immediate.
  constexpr int KSTEPS = sizeof(T) == 2 ? BKE / 32 : BKE / 4;
  const int fr = lane & 15;
  const int sw = (fr >> 1) & (CHUNKS - 1);
  unsigned koff[KSTEPS];
#pragma unroll
  for (int ks = 0; ks < KSTEPS; ++ks) {
    if constexpr (sizeof(T) == 2) koff[ks] = ((ks * 4 + (lane >> 4)) ^ sw) << 4;
    else koff[ks] = ((ks ^ sw) << 4) + ((lane >> 4) << 2);
  }
  const unsigned a_row = (wr * WTC + fr) * ROWB;
  const unsigned b_row = (BC + wc * WTP + fr) * ROWB;

  auto compute = [&](auto bufc) __attribute__((always_inline)) {
    constexpr int buf = decltype(bufc)::value;
    const char* base = smem + buf * BUF;
#pragma unroll
    for (int ks = 0; ks < KSTEPS; ++ks) {
      const char* pa = base + a_row + koff[ks];
      const char* pb = base + b_row + koff[ks];
      if constexpr (sizeof(T) == 2) {
        f16x8 fa[TC], fb[TP];
#pragma unroll
        for (int t = 0; t < TC; ++t) fa[t] = *reinterpret_cast<const f16x8*>(pa + t * 16 * ROWB);
#pragma unroll
        for (int t = 0; t < TP; ++t) fb[t] = *reinterpret_cast<const f16x8*>(pb + t * 16 * ROWB);
#pragma unroll
        for (int a = 0; a < TC; ++a)
#pragma unroll
          for (int b = 0; b < TP; ++b)
            acc[a][b] = __builtin_amdgcn_mfma_f32_16x16x32_f16(fa[a], fb[b], acc[a][b], 0, 0, 0);
      } else {
        float fa[TC], fb[TP];
#pragma unroll
        for (int t = 0; t < TC; ++t) fa[t] = *reinterpret_cast<const float*>(pa + t * 16 * ROWB);
#pragma unroll
        for (int t = 0; t < TP; ++t) fb[t] = *reinterpret_cast<const float*>(pb + t * 16 * ROWB);
#pragma unroll
        for (int a = 0; a < TC; ++a)
#pragma unroll
          for (int b = 0; b < TP; ++b)
            acc[a][b] = __builtin_amdgcn_mfma_f32_16x16x4f32(fa[a], fb[b], acc[a][b], 0, 0, 0);
      }
    }
  };

  // ---- main loop: NSTAGE-deep LDS ring, unrolled by NSTAGE so every LDS address is static ----
  if (nk > 0) {
    int it = 0;
    auto step = [&](auto jc) __attribute__((always_inline)) {
      constexpr int j = decltype(jc)::value;
      const int ahead = min(NSTAGE - 2, nk - 1 - it);   // tiles issued after tile `it`
      vmcnt_wait(ahead * myni);
      asm volatile("" ::: "memory");
      __builtin_amdgcn_s_barrier();
      asm volatile("" ::: "memory");
      if (it + NSTAGE - 1 < nk) {
        if (!(p.dbg & 1)) stage(std::integral_constant<int, (j + NSTAGE - 1) % NSTAGE>{}, kb + it + NSTAGE - 1);
        advance();
      }
      if (!(p.dbg & 2)) compute(jc);
      ++it;
    };
    // prologue: tiles 0 .. NSTAGE-2 in flight
    static_for<NSTAGE - 1>([&](auto jc) __attribute__((always_inline)) {
      constexpr int j = decltype(jc)::value;
      if (j < nk) {
        stage(jc, kb + j);
        advance();
      }
    });
    while (it < nk) {
      static_for<NSTAGE>([&](auto jc) __attribute__((always_inline)) {
        if (it < nk) step(jc);
      });
    }
  }

  conv_epilogue<T, TC, TP, WTC, WTP>(p, acc, c0, p0, wr, wc, lane, z);
}

// Sum split-K partials, then the same bias/activation epilogue (no residual).
template <typename T>
__global__ void splitk_reduce(const float* __restrict__ part, int splitk, int M, int npad, int cout,
                              const float* __restrict__ bias, const float* __restrict__ slope, int act,
                              void* y, int ycs, int out_f32) {
  const long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  const long long total = (long long)M * cout;
  if (i >= total) return;
  const int pix = (int)(i / cout);
  const int ch = (int)(i - (long long)pix * cout);
  float s = 0.f;
  for (int z = 0; z < splitk; ++z) s += part[((long long)z * M + pix) * npad + ch];
  if (bias) s += bias[ch];
  s = act_apply(s, act, slope ? slope[ch] : 0.f);
  if (out_f32) reinterpret_cast<float*>(y)[(long long)pix * ycs + ch] = s;
  else reinterpret_cast<T*>(y)[(long long)pix * ycs + ch] = (T)s;
}

// Sum split-K partials and finish with the conv's full epilogue (bias per channel or border
// class, PReLU / ReLU / SiLU / GELU before or after the residual, same-pixel or nearest-up2
// residual, zero channel padding): the small-batch plans split long-K convs of a few images
// over K so the grid covers the CUs (r03). One thread per output element.
template <typename T>
__global__ void splitk_finish(ConvParams p) {
  const long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  const long long total = (long long)p.M * p.cwrite;
  if (i >= total) return;
  const int pix = (int)(i / p.cwrite);
  const int ch = (int)(i - (long long)pix * p.cwrite);
  float v = 0.f;
  if (ch < p.cout) {
    for (int z = 0; z < p.splitk; ++z) v += p.partial[((long long)z * p.M + pix) * p.npad + ch];
    const int hw = p.OH * p.OW;
    const int n = pix / hw, rem = pix - n * hw;
    const int oh = rem / p.OW, ow = rem - oh * p.OW;
    if (p.bias_mode == BIAS_CHANNEL) {
      v += p.bias[ch];
    } else if (p.bias_mode == BIAS_BORDER9) {
      const ConvSeg& S = p.seg[0];
      const int ih0 = oh * S.stride - S.pad, iw0 = ow * S.stride - S.pad;
      const int rc = ih0 < 0 ? 0 : (ih0 + S.KH - 1 >= S.H ? 2 : 1);
      const int cc = iw0 < 0 ? 0 : (iw0 + S.KW - 1 >= S.W ? 2 : 1);
      v += p.bias[(rc * 3 + cc) * p.npad + ch];
    }
    const float sl = p.act == ACT_PRELU ? p.slope[ch] : 0.f;
    if (!p.act_after_res) v = act_apply(v, p.act, sl);
    if (p.res_mode != RES_NONE) {
      const long long rpix = p.res_mode == RES_UP2 ? ((long long)n * p.rH + (oh >> 1)) * p.rW + (ow >> 1)
                                                   : (long long)pix;
      v += (float)reinterpret_cast<const T*>(p.res)[rpix * p.rcs + ch];
    }
    if (p.act_after_res) v = act_apply(v, p.act, sl);
  }
  if (p.out_f32) reinterpret_cast<float*>(p.y)[(long long)pix * p.ycs + ch] = v;
  else reinterpret_cast<T*>(p.y)[(long long)pix * p.ycs + ch] = (T)v;
}

hipError_t splitk_finish_launch(int f32, const ConvParams& p, hipStream_t s) {
  const long long total = (long long)p.M * p.cwrite;
  if (total <= 0 || p.splitk < 1) return hipErrorInvalidValue;
  dim3 grid((unsigned)((total + 255) / 256));
  if (f32) hipLaunchKernelGGL(splitk_finish<float>, grid, dim3(256), 0, s, p);
  else hipLaunchKernelGGL(splitk_finish<f16>, grid, dim3(256), 0, s, p);
  return hipGetLastError();
}

// Direct 3x3 conv for stems: input NHWC with exactly 4 (padded) channels, one
// thread per output pixel, the whole [cout][3][3][4] filter bank in LDS. The
// 36-value input patch stays in registers (compile-time indexed).
template <typename T>
__global__ __launch_bounds__(256) void stem_conv3x3(StemParams p) {
  // filter taps are wave-uniform: read them through the scalar cache (s_load), not LDS
  const float* __restrict__ sw = p.w;
  const long long pix = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  const long long M = (long long)p.N * p.OH * p.OW;
  if (pix >= M) return;
  const int hw = p.OH * p.OW;
  const int n = (int)(pix / hw);
  const int rem = (int)(pix - (long long)n * hw);
  const int oh = rem / p.OW, ow = rem - (rem / p.OW) * p.OW;
  float in[36];
  const T* xb = reinterpret_cast<const T*>(p.x);
#pragma unroll
  for (int kh = 0; kh < 3; ++kh)
#pragma unroll
    for (int kw = 0; kw < 3; ++kw) {
      const int ih = oh * p.stride - p.pad + kh, iw = ow * p.stride - p.pad + kw;
      const bool ok = (unsigned)ih < (unsigned)p.H && (unsigned)iw < (unsigned)p.W;
      float v[4] = {0.f, 0.f, 0.f, 0.f};
      if (ok) load4<T>(xb + (((long long)n * p.H + ih) * p.W + iw) * p.xcs, v, 4);
#pragma unroll
      for (int c = 0; c < 4; ++c) in[(kh * 3 + kw) * 4 + c] = v[c];
    }
  T* y = reinterpret_cast<T*>(p.y) + pix * p.ycs;
  for (int co0 = 0; co0 < p.cpad; co0 += 4) {
    float v[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int co = co0 + j;
      float s = 0.f;
      if (co < p.cout) {
        const float* wrow = sw + co * 36;
#pragma unroll
        for (int k = 0; k < 36; ++k) s = fmaf(in[k], wrow[k], s);
        s += p.bias[co];
        s = act_apply(s, p.act, p.slope ? p.slope[co] : 0.f);
      }
      v[j] = s;
    }
    store4<T>(y + co0, v, 4);
  }
}

// Stem im2col: the KHxKWxcin_true window of every output pixel packed into one
// 32-element K row (tap-major, channel-minor, zero past K_true and in the padding),
// so the stem runs on the MFMA engine as a 1x1 conv with C = 32. Four threads per
// pixel, 8 elements (16 B f16) each.
template <typename T>
__global__ void stem_im2col(StemParams p, int cin_true, T* __restrict__ col) {
  const long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  const long long M = (long long)p.N * p.OH * p.OW;
  if (i >= M * 4) return;
  const long long pix = i >> 2;
  const int k0 = (int)(i & 3) * 8;
  const int hw = p.OH * p.OW;
  const int n = (int)(pix / hw);
  const int rem = (int)(pix - (long long)n * hw);
  const int oh = rem / p.OW, ow = rem - (rem / p.OW) * p.OW;
  const int ktrue = p.KH * p.KW * cin_true;
  const T* xb = reinterpret_cast<const T*>(p.x);
  T v[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const int k = k0 + j;
    T e = (T)0.f;
    if (k < ktrue) {
      const int tap = k / cin_true, c = k - tap * cin_true;
      const int th = tap / p.KW, tw = tap - th * p.KW;
      const int ih = oh * p.stride - p.pad + th, iw = ow * p.stride - p.pad + tw;
      if ((unsigned)ih < (unsigned)p.H && (unsigned)iw < (unsigned)p.W)
        e = xb[(((long long)n * p.H + ih) * p.W + iw) * p.xcs + c];
    }
    v[j] = e;
  }
  T* dst = col + pix * 32 + k0;
#pragma unroll
  for (int j = 0; j < 8; ++j) dst[j] = v[j];
}

// The common stem (3x3 window, 3 true channels of an NHWC4 input): one thread per output
// pixel gathers the nine 4-channel input pixels with one vector load each and writes
// its 32-element im2col row ([tap][c] order, 27 values + 5 zeros) as full 16-byte
// stores - the generic gather above issues 8 scalar loads and stores per 8 elements.
template <typename T>
__global__ void stem_im2col3(StemParams p, T* __restrict__ col) {
  const long long pix = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  const long long M = (long long)p.N * p.OH * p.OW;
  if (pix >= M) return;
  const int hw = p.OH * p.OW;
  const int n = (int)(pix / hw);
  const int rem = (int)(pix - (long long)n * hw);
  const int oh = rem / p.OW, ow = rem - (rem / p.OW) * p.OW;
  const T* xb = reinterpret_cast<const T*>(p.x) + (long long)n * p.H * p.W * 4;
  T v[32];
#pragma unroll
  for (int t = 0; t < 9; ++t) {
    const int ih = oh * p.stride - p.pad + t / 3, iw = ow * p.stride - p.pad + t % 3;
    float e[4] = {0.f, 0.f, 0.f, 0.f};
    if ((unsigned)ih < (unsigned)p.H && (unsigned)iw < (unsigned)p.W) load4<T>(xb + ((long long)ih * p.W + iw) * 4, e, 4);
    v[3 * t] = (T)e[0];
    v[3 * t + 1] = (T)e[1];
    v[3 * t + 2] = (T)e[2];
  }
#pragma unroll
  for (int k = 27; k < 32; ++k) v[k] = (T)0.f;
  T* dst = col + pix * 32;
  constexpr int VE = 16 / sizeof(T);
#pragma unroll
  for (int q = 0; q < 32 / VE; ++q) {
    if constexpr (sizeof(T) == 2) {
      f16x8 h;
#pragma unroll
      for (int j = 0; j < 8; ++j) h[j] = v[q * 8 + j];
      *reinterpret_cast<f16x8*>(dst + q * 8) = h;
    } else {
      *reinterpret_cast<f32x4*>(dst + q * 4) = f32x4{(float)v[q * 4], (float)v[q * 4 + 1], (float)v[q * 4 + 2],
                                                     (float)v[q * 4 + 3]};
    }
  }
}

// NHWC max pool (padding = -inf, PyTorch semantics); one thread per pixel x 4 channels.
template <typename T>
__global__ void maxpool_nhwc(PoolParams p) {
  const long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  const int cg = p.C / 4;
  const long long total = (long long)p.N * p.OH * p.OW * cg;
  if (i >= total) return;
  const int g = (int)(i % cg);
  const long long pix = i / cg;
  const int hw = p.OH * p.OW;
  const int n = (int)(pix / hw);
  const int rem = (int)(pix - (long long)n * hw);
  const int oh = rem / p.OW, ow = rem - (rem / p.OW) * p.OW;
  float m[4] = {-INFINITY, -INFINITY, -INFINITY, -INFINITY};
  const T* xb = reinterpret_cast<const T*>(p.x);
  for (int kh = 0; kh < p.k; ++kh)
    for (int kw = 0; kw < p.k; ++kw) {
      const int ih = oh * p.stride - p.pad + kh, iw = ow * p.stride - p.pad + kw;
      if ((unsigned)ih >= (unsigned)p.H || (unsigned)iw >= (unsigned)p.W) continue;
      float v[4];
      load4<T>(xb + (((long long)n * p.H + ih) * p.W + iw) * p.xcs + g * 4, v, 4);
#pragma unroll
      for (int j = 0; j < 4; ++j) m[j] = fmaxf(m[j], v[j]);
    }
  store4<T>(reinterpret_cast<T*>(p.y) + pix * p.ycs + g * 4, m, 4);
}

// f16 NHWC max pool, 8 channels (one 16-byte load) per thread and 32-bit index math (the
// grid is < 2^31 threads): the SCRFD stem pool reads ~210 MB per 32-frame chunk, so the
// 64-bit divides and 8-byte loads of maxpool_nhwc left it at ~1.4 TB/s. Same fmaxf over
// the same window as maxpool_nhwc: bit-identical output.
__global__ void maxpool_nhwc_f16x8(PoolParams p) {
  const unsigned i = blockIdx.x * blockDim.x + threadIdx.x;
  const unsigned cg = (unsigned)p.C >> 3;
  const unsigned hw = (unsigned)(p.OH * p.OW);
  if (i >= (unsigned)p.N * hw * cg) return;
  const unsigned pix = i / cg, g = i - pix * cg;
  const unsigned n = pix / hw, rem = pix - n * hw;
  const int oh = (int)(rem / (unsigned)p.OW), ow = (int)(rem - (unsigned)oh * (unsigned)p.OW);
  float m[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) m[j] = -INFINITY;
  const f16* xb = reinterpret_cast<const f16*>(p.x) + g * 8;
  for (int kh = 0; kh < p.k; ++kh) {
    const int ih = oh * p.stride - p.pad + kh;
    if ((unsigned)ih >= (unsigned)p.H) continue;
    for (int kw = 0; kw < p.k; ++kw) {
      const int iw = ow * p.stride - p.pad + kw;
      if ((unsigned)iw >= (unsigned)p.W) continue;
      const f16x8 v = *reinterpret_cast<const f16x8*>(xb + ((size_t)(n * p.H + ih) * p.W + iw) * p.xcs);
#pragma unroll
      for (int j = 0; j < 8; ++j) m[j] = fmaxf(m[j], (float)v[j]);
    }
  }
  f16x8 h;
#pragma unroll
  for (int j = 0; j < 8; ++j) h[j] = (f16)m[j];
  *reinterpret_cast<f16x8*>(reinterpret_cast<f16*>(p.y) + (size_t)pix * p.ycs + g * 8) = h;
}

// f16x3 split NHWC max pool: channels [0, C) hold hi, [C, 2C) lo of the same values. The max
// runs over the exact f32 values hi + lo (PyTorch's f32 max pool of the f32 activations),
// and the maximum is written back split (hi = f16(m), lo = f16(m - hi): m again exactly).
__global__ void maxpool_split_f16x8(PoolParams p) {
  const unsigned i = blockIdx.x * blockDim.x + threadIdx.x;
  const unsigned cg = (unsigned)p.C >> 3;
  const unsigned hw = (unsigned)(p.OH * p.OW);
  if (i >= (unsigned)p.N * hw * cg) return;
  const unsigned pix = i / cg, g = i - pix * cg;
  const unsigned n = pix / hw, rem = pix - n * hw;
  const int oh = (int)(rem / (unsigned)p.OW), ow = (int)(rem - (unsigned)oh * (unsigned)p.OW);
  float m[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) m[j] = -INFINITY;
  const f16* xb = reinterpret_cast<const f16*>(p.x) + g * 8;
  for (int kh = 0; kh < p.k; ++kh) {
    const int ih = oh * p.stride - p.pad + kh;
    if ((unsigned)ih >= (unsigned)p.H) continue;
    for (int kw = 0; kw < p.k; ++kw) {
      const int iw = ow * p.stride - p.pad + kw;
      if ((unsigned)iw >= (unsigned)p.W) continue;
      const f16* px = xb + ((size_t)(n * p.H + ih) * p.W + iw) * p.xcs;
      const f16x8 h = *reinterpret_cast<const f16x8*>(px);
      const f16x8 l = *reinterpret_cast<const f16x8*>(px + p.C);
#pragma unroll
      for (int j = 0; j < 8; ++j) m[j] = fmaxf(m[j], (float)h[j] + (float)l[j]);
    }
  }
  f16x8 h, l;
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    h[j] = (f16)m[j];
    l[j] = (f16)(m[j] - (float)h[j]);
  }
  f16* yp = reinterpret_cast<f16*>(p.y) + (size_t)pix * p.ycs + g * 8;
  *reinterpret_cast<f16x8*>(yp) = h;
  *reinterpret_cast<f16x8*>(yp + p.C) = l;
}

// ---------------------------------------------------------------------------
// host-side launchers
// ---------------------------------------------------------------------------
// LDS ring depth: as many K-tiles as fit in 144 KiB, 2..8
constexpr int ring_depth(int bc, int bp, int rowb) {
  return (147456 / ((bc + bp) * rowb)) < 2 ? 2 : ((147456 / ((bc + bp) * rowb)) > 8 ? 8 : 147456 / ((bc + bp) * rowb));
}

template <typename T, int BC, int BP, int ROWB, int WC, int WP>
static hipError_t launch_cfg(const ConvParams& p, hipStream_t s) {
  constexpr int NS = ring_depth(BC, BP, ROWB);
  const int nwg = (p.M + BP - 1) / BP * (p.npad / BC);
  dim3 grid(nwg, 1, p.splitk);
  hipLaunchKernelGGL((conv_igemm<T, BC, BP, ROWB, WC, WP, NS>), grid, dim3(64 * WC * WP), 0, s, p);
  return hipGetLastError();
}

// Tile configurations (channels x pixels, waves as WC x WP); keep in sync with
// kConvCfgs in pc_api.cpp.
template <typename T, int ROWB>
static hipError_t launch_rowb(const ConvParams& p, int cfg, hipStream_t s) {
  switch (cfg) {
    case 0: return launch_cfg<T, 128, 128, ROWB, 2, 2>(p, s);
    case 1: return launch_cfg<T, 128, 64, ROWB, 2, 2>(p, s);
    case 2: return launch_cfg<T, 64, 256, ROWB, 2, 2>(p, s);
    case 3: return launch_cfg<T, 64, 128, ROWB, 2, 2>(p, s);
    case 4: return launch_cfg<T, 96, 128, ROWB, 2, 2>(p, s);
    case 5: return launch_cfg<T, 32, 256, ROWB, 2, 2>(p, s);
    case 6: return launch_cfg<T, 32, 128, ROWB, 2, 2>(p, s);
    case 7: return launch_cfg<T, 128, 256, ROWB, 2, 4>(p, s);
    case 8: return launch_cfg<T, 256, 128, ROWB, 4, 2>(p, s);
    case 9: return launch_cfg<T, 256, 256, ROWB, 2, 4>(p, s);
    case 10: return launch_cfg<T, 64, 512, ROWB, 1, 8>(p, s);
    case 11: return launch_cfg<T, 96, 256, ROWB, 2, 4>(p, s);
    case 12: return launch_cfg<T, 32, 512, ROWB, 1, 8>(p, s);
    case 13: return launch_cfg<T, 128, 128, ROWB, 2, 4>(p, s);
    default: return hipErrorInvalidValue;
  }
}

hipError_t conv_launch(int f32, int rowb, int cfg, const ConvParams& p, hipStream_t s) {
  if (f32) return rowb == 128 ? launch_rowb<float, 128>(p, cfg, s) : launch_rowb<float, 64>(p, cfg, s);
  return rowb == 128 ? launch_rowb<f16, 128>(p, cfg, s) : launch_rowb<f16, 64>(p, cfg, s);
}

hipError_t splitk_reduce_launch(int f32, const float* part, int splitk, int M, int npad, int cout,
                                const float* bias, const float* slope, int act, void* y, int ycs,
                                int out_f32, hipStream_t s) {
  const long long total = (long long)M * cout;
  dim3 grid((unsigned)((total + 255) / 256));
  if (f32)
    hipLaunchKernelGGL(splitk_reduce<float>, grid, dim3(256), 0, s, part, splitk, M, npad, cout, bias, slope, act, y, ycs, out_f32);
  else
    hipLaunchKernelGGL(splitk_reduce<f16>, grid, dim3(256), 0, s, part, splitk, M, npad, cout, bias, slope, act, y, ycs, out_f32);
  return hipGetLastError();
}

hipError_t stem_launch(int f32, const StemParams& p, hipStream_t s) {
  const long long M = (long long)p.N * p.OH * p.OW;
  dim3 grid((unsigned)((M + 255) / 256));
  if (p.KH != 3 || p.KW != 3 || p.cin != 4 || p.cout > 64 || p.cpad % 4) return hipErrorInvalidValue;
  if (f32) hipLaunchKernelGGL(stem_conv3x3<float>, grid, dim3(256), 0, s, p);
  else hipLaunchKernelGGL(stem_conv3x3<f16>, grid, dim3(256), 0, s, p);
  return hipGetLastError();
}

hipError_t stem_im2col_launch(int f32, const StemParams& p, int cin_true, void* col, hipStream_t s) {
  const long long M = (long long)p.N * p.OH * p.OW;
  dim3 grid((unsigned)((M * 4 + 255) / 256));
  if (p.KH * p.KW * cin_true > 32) return hipErrorInvalidValue;
  if (p.KH == 3 && p.KW == 3 && cin_true == 3 && p.cin == 4 && p.xcs == 4) {
    dim3 g3((unsigned)((M + 255) / 256));
    if (f32) hipLaunchKernelGGL(stem_im2col3<float>, g3, dim3(256), 0, s, p, (float*)col);
    else hipLaunchKernelGGL(stem_im2col3<f16>, g3, dim3(256), 0, s, p, (f16*)col);
    return hipGetLastError();
  }
  if (f32) hipLaunchKernelGGL(stem_im2col<float>, grid, dim3(256), 0, s, p, cin_true, (float*)col);
  else hipLaunchKernelGGL(stem_im2col<f16>, grid, dim3(256), 0, s, p, cin_true, (f16*)col);
  return hipGetLastError();
}

hipError_t maxpool_launch(int f32, const PoolParams& p, hipStream_t s) {
  const long long total = (long long)p.N * p.OH * p.OW * (p.C / 4);
  dim3 grid((unsigned)((total + 255) / 256));
  const bool al16 = (((uintptr_t)p.x | (uintptr_t)p.y) & 15) == 0;
  if (p.split) {
    if (f32 || !al16 || p.C % 8 || p.xcs % 8 || p.ycs % 8 || total / 2 >= 2147483647LL ||
        (long long)p.N * p.H * p.W >= 2147483647LL)
      return hipErrorInvalidValue;
    hipLaunchKernelGGL(maxpool_split_f16x8, dim3((unsigned)((total / 2 + 255) / 256)), dim3(256), 0, s, p);
    return hipGetLastError();
  }
  if (!f32 && al16 && p.C % 8 == 0 && p.xcs % 8 == 0 && p.ycs % 8 == 0 && total / 2 < 2147483647LL &&
      (long long)p.N * p.H * p.W < 2147483647LL) {
    hipLaunchKernelGGL(maxpool_nhwc_f16x8, dim3((unsigned)((total / 2 + 255) / 256)), dim3(256), 0, s, p);
    return hipGetLastError();
  }
  if (f32) hipLaunchKernelGGL(maxpool_nhwc<float>, grid, dim3(256), 0, s, p);
  else hipLaunchKernelGGL(maxpool_nhwc<f16>, grid, dim3(256), 0, s, p);
  return hipGetLastError();
}

}  // namespace pc
