// Stride-1 "same" convolution with an LDS-resident input halo (gfx950).
//
// The implicit-GEMM engine of pc_conv.hip stages one im2col row per (pixel, tap):
// a 3x3 conv moves every input pixel from L2 into LDS nine times, and at the
// IResNet / SCRFD trunk sizes that traffic is served by the Infinity Cache, not
// L2. For stride 1 with "same" padding the input pixel of output
// pixel q under tap (th, tw) is the NHWC-linear pixel q + (th-padH)*W + (tw-padW):
// one wave-uniform shift. So a BP-pixel tile stages, per 32-channel chunk, the
// contiguous run of BP + 2*(padH*W + padW) input pixels ("halo") ONCE, and every
// tap reads its B fragments from that run at a shifted row; taps that fall into
// the zero padding (image border, or a neighbouring image of the batch) read a
// zero row instead (per-lane tap-validity bitmask, precomputed once).
//
// Pipeline (one raw s_barrier per step, no drain to vmcnt(0) in the loop): a step
// is (channel chunk cb, tap); steps run chunk-major. Weights [BC][64 B] for step
// j+S-1 are issued right after the barrier of step j into an S-deep ring; the halo
// of chunk cb is issued together with the weights of the chunk's first step into
// a ring of HB = 1 + ceil((S-1)/KK) halo buffers. Each wave waits with a counted
// vmcnt that leaves in flight exactly the DMA instructions it issued for the next
// S-2 steps (kept per ring slot in scalar registers).
//
// LDS images use 64-byte rows (K = 32 f16 / 16 f32 per step) with the 16-byte
// chunk c of row r stored at position c ^ ((r >> 1) & 3). For ds_read_b128
// fragment reads of 16 consecutive rows this is bank-conflict free for EVERY
// starting row (checked exhaustively against the gfx950 lane groups), which is
// what the arbitrary tap shifts need; and f(r + 16) = f(r), so the TP fragments of
// a wave differ by a compile-time 1 KiB.
#include "pc_conv_common.h"

namespace pc {

constexpr int kHaloLds = 163840;   // the whole 160 KiB of the CU

// halo buffers: a chunk's halo is refilled D = S-1 steps ahead, after >= 2 barriers
__host__ __device__ constexpr int halo_nbuf(int S, int KK) { return 1 + (S - 1 + KK - 1) / KK; }
__host__ __device__ constexpr int halo_cap_rows(int S, int BC, int KK) {
  return ((kHaloLds - S * BC * 64 - (KK > 1 ? 64 : 0)) / (halo_nbuf(S, KK) * 64)) & ~15;
}

template <typename T, int BC, int BP, int WC, int WP, int S>
__global__ __launch_bounds__(64 * WC * WP, 1) void conv_halo(ConvParams p) {
  constexpr int D = S - 1;                   // DMA lookahead in steps
  constexpr int NW = WC * WP;
  constexpr int ESZ = sizeof(T);
  constexpr int BKE = 64 / ESZ;              // K elements per step
  constexpr int WTC = BC / WC, WTP = BP / WP;
  constexpr int TC = WTC / 16, TP = WTP / 16;
  constexpr int WBUF = BC * 64;              // one weight ring slot
  constexpr int NWI = BC / 16;               // weight DMA instructions per step (16 rows each)
  constexpr int NWW = (NWI + NW - 1) / NW;   // per wave (upper bound)
  static_assert(WTC % 16 == 0 && WTP % 16 == 0, "wave tile");
  static_assert(S >= 3, "ring depth");
  static_assert(NW % 2 == 0, "ping-pong needs two wave halves");

  __shared__ __attribute__((aligned(16))) char smem[kHaloLds];

  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  __builtin_assume(wave >= 0 && wave < NW);
  const int wr = wave / WP, wc = wave % WP;
  const int nct = p.npad / BC;
  const int npt = (p.M + BP - 1) / BP;
  const int tile = xcd_remap(blockIdx.x, nct * npt);
  const int p0 = (tile / nct) * BP;
  const int c0 = (tile % nct) * BC;

  const ConvSeg& G = p.seg[0];
  const int H = G.H, W = G.W, KH = G.KH, KW = G.KW, C = G.C;
  const int KK = KH * KW;
  const int padH = (KH - 1) >> 1, padW = (KW - 1) >> 1;
  const int cblk = G.cblk;
  const int nk = cblk * KK;
  const int HB = halo_nbuf(S, KK);
  const int hcap = halo_cap_rows(S, BC, KK);
  const int hr = BP + 2 * (padH * W + padW);   // halo rows used (host guarantees roundup16(hr) <= hcap)
  const int hinst = (hr + 15) >> 4;            // halo DMA instructions per chunk
  const int hq = (hinst + NW - 1) / NW;        // KK > 1: halo parts per chunk (one per wave per step)
  const int hbase = p0 - padH * W - padW;      // input pixel staged in halo row 0
  const int Min = p.M;                         // stride 1, same padding: input pixels == output pixels
  const char* xs = reinterpret_cast<const char*>(G.x);
  const unsigned xrow_b = (unsigned)G.cs * ESZ;
  const int halo0 = S * WBUF;
  const int hbuf_b = hcap * 64;
  const int zrow = halo0 + HB * hbuf_b;
  const int nww = wave < NWI ? (NWI - 1 - wave) / NW + 1 : 0;       // weight DMAs of this wave per step
  const int nhw1 = wave < hinst ? (hinst - 1 - wave) / NW + 1 : 0;  // KK == 1: halo DMAs per step

  if (KK > 1 && wave == 0 && lane < 4) *reinterpret_cast<f32x4*>(smem + zrow + lane * 16) = f32x4{0.f, 0.f, 0.f, 0.f};

  // ---- weight staging: per-lane 32-bit offsets (loop-invariant), K offset rides in the scalar base ----
  const int lrow = lane >> 2, lpos = lane & 3;
  unsigned woff[NWW];
  static_for<NWW>([&](auto ic) __attribute__((always_inline)) {
    constexpr int i = decltype(ic)::value;
    const int r = (i * NW + wave) * 16 + lrow;
    woff[i] = (unsigned)((long long)(c0 + min(r, BC - 1)) * p.ktot * ESZ) + ((lpos ^ ((r >> 1) & 3)) << 4);
  });
  const char* wsrc = reinterpret_cast<const char*>(p.w);

  // ---- per-lane tap validity of this lane's B-fragment pixels ----
  unsigned vmask[TP];
  static_for<TP>([&](auto tc) __attribute__((always_inline)) {
    constexpr int t = decltype(tc)::value;
    const int q = p0 + wc * WTP + t * 16 + (lane & 15);
    unsigned m = 0;
    if (q < p.M) {
      const int rem = q % (H * W);
      const int oh = rem / W, ow = rem - (rem / W) * W;
      unsigned mh = 0, mw = 0;
      for (int th = 0; th < KH; ++th) mh |= ((unsigned)(oh + th - padH) < (unsigned)H ? 1u : 0u) << th;
      for (int tw = 0; tw < KW; ++tw) mw |= ((unsigned)(ow + tw - padW) < (unsigned)W ? 1u : 0u) << tw;
      for (int th = 0; th < KH; ++th)
        if ((mh >> th) & 1) m |= mw << (th * KW);
    }
    vmask[t] = KK > 1 ? m : 0xffffffffu;   // 1x1: rows past M were staged from the zero page
  });

  // one halo DMA instruction g (16 rows) of chunk icb into halo buffer ihb
  auto halo_dma = [&](int g, int icb, int ihb) __attribute__((always_inline)) {
    const int h = g * 16 + lrow;
    const int lin = hbase + h;
    const unsigned sc = (unsigned)((lpos ^ ((h >> 1) & 3)) << 4);
    unsigned off = (h < hr && lin >= 0 && lin < Min) ? (unsigned)lin * xrow_b + sc : G.zero_off + sc;
    asm volatile("" : "+v"(off));
    __builtin_amdgcn_global_load_lds((gptr_t)(xs + icb * 64 + off), (lds_ptr_t)(smem + halo0 + ihb * hbuf_b + g * 1024),
                                     16, 0, 0);
  };

  // DMA for target step (icb, itap) into weight slot `slot`. The halo of a chunk is
  // staged ahead of its first step: KK == 1 - with the step itself; KK > 1 - chunk 0 in
  // the prologue, chunk c+1 as one instruction per wave at each of the taps D .. D+hq-1
  // of chunk c (by then the buffer's previous chunk has been read by both wave halves).
  // Returns this wave's DMA instruction count (vmcnt bookkeeping).
  auto issue = [&](int slot, int icb, int itap, int ihb) __attribute__((always_inline)) {
    int cnt = 0;
    if (KK == 1) {
      for (int k = 0; k < nhw1; ++k) halo_dma(wave + k * NW, icb, ihb);
      cnt += nhw1;
    } else if (itap >= D && itap < D + hq && icb + 1 < cblk) {
      const int g = (itap - D) * NW + wave;
      if (g < hinst) {
        halo_dma(g, icb + 1, ihb + 1 == HB ? 0 : ihb + 1);
        cnt += 1;
      }
    }
    const char* wb = wsrc + (long long)(itap * C + icb * BKE) * ESZ;
    static_for<NWW>([&](auto ic) __attribute__((always_inline)) {
      constexpr int i = decltype(ic)::value;
      if (NWI % NW == 0 || i * NW + wave < NWI) {
        unsigned off = woff[i];
        asm volatile("" : "+v"(off));
        __builtin_amdgcn_global_load_lds((gptr_t)(wb + off), (lds_ptr_t)(smem + slot * WBUF + (i * NW + wave) * 1024),
                                         16, 0, 0);
      }
    });
    return cnt + nww;
  };

  f32x4 acc[TC][TP];
#pragma unroll
  for (int a = 0; a < TC; ++a)
#pragma unroll
    for (int b = 0; b < TP; ++b) acc[a][b] = f32x4{0.f, 0.f, 0.f, 0.f};

  // fragment geometry: A rows are 16-aligned, so their swizzle term depends on the lane only
  const int fr = lane & 15, fq = lane >> 4;
  const int a_sw = (fr >> 1) & 3;
  const int a_row = (wr * WTC + fr) * 64;
  const int b_row0 = wc * WTP + fr;

  // Fragments of one step live in registers across the barrier that separates the
  // read segment from the MFMA segment (KS k-sub-steps: 1 for f16, 4 for f32).
  constexpr int KS = ESZ == 2 ? 1 : 4;
  using Frag = typename std::conditional<ESZ == 2, f16x8, float>::type;
  Frag fa[KS][TC], fb[KS][TP];

  auto read_frags = [&](int slot, int ihb, int th, int tw) __attribute__((always_inline)) {
    const int row = b_row0 + th * W + tw;
    const int bsw = (row >> 1) & 3;
    const int tb = th * KW + tw;
    const char* abase = smem + slot * WBUF + a_row;
    const int bbase = halo0 + ihb * hbuf_b + row * 64;
    if constexpr (ESZ == 2) {
      const int boff = bbase + ((fq ^ bsw) << 4);
#pragma unroll
      for (int t = 0; t < TP; ++t) {
        const int ad = ((vmask[t] >> tb) & 1) ? boff + t * 1024 : zrow;
        fb[0][t] = *reinterpret_cast<const f16x8*>(smem + ad);
      }
#pragma unroll
      for (int a = 0; a < TC; ++a) fa[0][a] = *reinterpret_cast<const f16x8*>(abase + a * 1024 + ((fq ^ a_sw) << 4));
    } else {
      int bad[TP];   // the zero row is 64 B, so the chunk offset below stays inside it
#pragma unroll
      for (int t = 0; t < TP; ++t) bad[t] = ((vmask[t] >> tb) & 1) ? bbase + t * 1024 + fq * 4 : zrow;
#pragma unroll
      for (int ks = 0; ks < KS; ++ks) {
#pragma unroll
        for (int t = 0; t < TP; ++t) fb[ks][t] = *reinterpret_cast<const float*>(smem + bad[t] + ((ks ^ bsw) << 4));
#pragma unroll
        for (int a = 0; a < TC; ++a)
          fa[ks][a] = *reinterpret_cast<const float*>(abase + a * 1024 + ((ks ^ a_sw) << 4) + fq * 4);
      }
    }
  };
  auto mfma_block = [&]() __attribute__((always_inline)) {
#pragma unroll
    for (int ks = 0; ks < KS; ++ks)
#pragma unroll
      for (int a = 0; a < TC; ++a)
#pragma unroll
        for (int b = 0; b < TP; ++b) {
          if constexpr (ESZ == 2)
            acc[a][b] = __builtin_amdgcn_mfma_f32_16x16x32_f16(fa[ks][a], fb[ks][b], acc[a][b], 0, 0, 0);
          else
            acc[a][b] = __builtin_amdgcn_mfma_f32_16x16x4f32(fa[ks][a], fb[ks][b], acc[a][b], 0, 0, 0);
        }
  };
  auto bar = [&]() __attribute__((always_inline)) {
    __builtin_amdgcn_sched_barrier(0);
    asm volatile("" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);
  };

  // ---- iterators: compute (slot, th, tw, halo buffer) and issue (slot, icb, ith, itw, itap, halo buffer) ----
  int cslot = 0, cth = 0, ctw = 0, chb = 0;
  int islot = 0, icb = 0, ith = 0, itw = 0, itap = 0, ihb = 0;
  auto iadvance = [&]() __attribute__((always_inline)) {
    if (++islot == S) islot = 0;
    ++itap;
    if (++itw == KW) {
      itw = 0;
      if (++ith == KH) {
        ith = 0; itap = 0; ++icb;
        if (++ihb == HB) ihb = 0;
      }
    }
  };
  auto cadvance = [&]() __attribute__((always_inline)) {
    if (++cslot == S) cslot = 0;
    if (++ctw == KW) {
      ctw = 0;
      if (++cth == KH) {
        cth = 0;
        if (++chb == HB) chb = 0;
      }
    }
  };

  // Ping-pong schedule. Every step is a read segment R_j (DMA issue for step j+D,
  // ds_reads of step j, counted vmcnt that retires step j+1, lgkmcnt(0)) and an MFMA
  // segment X_j, each closed by a barrier. Waves NW/2..NW-1 pass one extra barrier
  // first, so they run one segment behind: on every SIMD one wave reads while the
  // other multiplies. Ordering (W_k = k-th workgroup barrier): the first half reads
  // step j after W_{2j+1}, the second half after W_{2j+2}; every issuer retired step j
  // before W_{2j-1} / W_{2j} (the wait in R_{j-1}), and a ring slot or halo buffer is
  // refilled >= 2 barriers after its last reader finished (S = D + 1; halo parts of
  // chunk c+1 go out at taps >= D of chunk c; HB = 1 + ceil(D / KK)).
  int inflight[D - 1];   // DMA instructions this wave issued for the last D-1 targets (oldest first)
  static_for<D - 1>([&](auto dc) __attribute__((always_inline)) { inflight[decltype(dc)::value] = 0; });
  if (KK > 1)
    for (int k = 0; k < nhw1; ++k) halo_dma(wave + k * NW, 0, 0);   // chunk 0's halo, retired with target 0
  {
    int first = 0;
    static_for<D>([&](auto jc) __attribute__((always_inline)) {
      constexpr int j = decltype(jc)::value;
      int c = 0;
      if (j < nk) {
        c = issue(islot, icb, itap, ihb);
        iadvance();
      }
      if constexpr (j == 0) first = c; else inflight[j - 1] = c;
    });
    (void)first;
    int allowed = 0;
    static_for<D - 1>([&](auto dc) __attribute__((always_inline)) { allowed += inflight[decltype(dc)::value]; });
    vmcnt_wait(allowed);
  }
  const bool lagging = wave >= NW / 2;
  if (lagging) bar();
  bar();

  for (int it = 0; it < nk; ++it) {
    int c = 0;
    if (it + D < nk) {
      c = issue(islot, icb, itap, ihb);
      iadvance();
    }
    read_frags(cslot, chb, cth, ctw);
    // retire target it+1: the in-flight window becomes targets it+2 .. it+D
    int allowed = c;
    static_for<D - 2>([&](auto dc) __attribute__((always_inline)) {
      constexpr int d = decltype(dc)::value;
      inflight[d] = inflight[d + 1];
      allowed += inflight[d];
    });
    inflight[D - 2] = c;
    vmcnt_wait(allowed);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    bar();
    mfma_block();
    bar();
    cadvance();
  }
  if (!lagging) bar();

  conv_epilogue_lds<T, BC, BP, WC, WP>(p, acc, c0, p0, wr, wc, lane, smem);
}

// ---------------------------------------------------------------------------
// host side
// ---------------------------------------------------------------------------
struct HaloCfg { int bc, bp, s, nw; };
// keep in sync with launch_halo_t below
static const HaloCfg kHaloCfgs[] = {
    {256, 256, 4, 8},   // 0: 8 waves 2x4, 128x64 per wave
    {128, 512, 4, 8},   // 1: 8 waves 1x8, 128x64 per wave
    {128, 256, 4, 8},   // 2: 8 waves 2x4, 64x64 per wave
    {64, 512, 4, 8},    // 3: 8 waves 1x8, 64x64 per wave
    {64, 256, 4, 4},    // 4: 4 waves 1x4, 64x64 per wave
};
static const int kNumHaloCfgs = sizeof(kHaloCfgs) / sizeof(kHaloCfgs[0]);

int conv_halo_num_cfgs() { return kNumHaloCfgs; }

// tile geometry of cfg (channels, pixels); 0 if cfg is unknown
int conv_halo_tile(int cfg, int* bc, int* bp) {
  if (cfg < 0 || cfg >= kNumHaloCfgs) return 0;
  *bc = kHaloCfgs[cfg].bc;
  *bp = kHaloCfgs[cfg].bp;
  return 1;
}

// does a KHxKW stride-1 conv over rows of width W fit cfg's halo buffers?
int conv_halo_fits(int cfg, int KH, int KW, int W) {
  if (cfg < 0 || cfg >= kNumHaloCfgs || KH * KW > 32 || !(KH & 1) || !(KW & 1)) return 0;
  const HaloCfg& c = kHaloCfgs[cfg];
  const int KK = KH * KW;
  const int hr = c.bp + 2 * (((KH - 1) / 2) * W + (KW - 1) / 2);
  const int hinst = (hr + 15) / 16;
  // KK > 1: the next chunk's halo goes out one instruction per wave at taps D .. KK-1
  if (KK > 1 && (hinst + c.nw - 1) / c.nw > KK - (c.s - 1)) return 0;
  return ((hr + 15) & ~15) <= halo_cap_rows(c.s, c.bc, KK);
}

template <typename T, int BC, int BP, int WC, int WP, int S>
static hipError_t launch_halo_cfg(const ConvParams& p, hipStream_t s) {
  const int nwg = (p.M + BP - 1) / BP * (p.npad / BC);
  hipLaunchKernelGGL((conv_halo<T, BC, BP, WC, WP, S>), dim3(nwg), dim3(64 * WC * WP), 0, s, p);
  return hipGetLastError();
}

template <typename T>
static hipError_t launch_halo_t(const ConvParams& p, int cfg, hipStream_t s) {
  switch (cfg) {
    case 0: return launch_halo_cfg<T, 256, 256, 2, 4, 4>(p, s);
    case 1: return launch_halo_cfg<T, 128, 512, 1, 8, 4>(p, s);
    case 2: return launch_halo_cfg<T, 128, 256, 2, 4, 4>(p, s);
    case 3: return launch_halo_cfg<T, 64, 512, 1, 8, 4>(p, s);
    case 4: return launch_halo_cfg<T, 64, 256, 1, 4, 4>(p, s);
    default: return hipErrorInvalidValue;
  }
}

hipError_t conv_halo_launch(int f32, int cfg, const ConvParams& p, hipStream_t s) {
  const ConvSeg& G = p.seg[0];
  // shape contract (the planner checks the same; a violation here is a host bug, not a fault)
  if (p.nseg != 1 || p.splitk != 1 || G.stride != 1 || G.H != p.OH || G.W != p.OW || G.pad * 2 + 1 != G.KH ||
      G.KH != G.KW || !conv_halo_fits(cfg, G.KH, G.KW, G.W) || p.npad % kHaloCfgs[cfg].bc)
    return hipErrorInvalidValue;
  return f32 ? launch_halo_t<float>(p, cfg, s) : launch_halo_t<f16>(p, cfg, s);
}

}  // namespace pc
