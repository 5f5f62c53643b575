// Resident block chain: a run of IResNet identity blocks over small images whose
// 256-channel activation fits in one CU's LDS (gfx950) - ArcFace-r100's 14x14x256 stage,
// 29 of its 30 blocks, ~45 % of the network's MFMA work.
//
// Why: on the implicit-GEMM kernel (pc_conv_fast.hip) one such conv is a single round of
// ~224 workgroups (one per CU), so every launch pays its prologue (pipeline fill from
// HBM), its epilogue (output + residual through HBM, ~11 of ~75 us) and the 9x im2col
// re-read of every input pixel from L2, and none of it overlaps anything
// (DESIGN.md §3.1). Here one workgroup owns one image for the whole run of blocks:
//
//  * the image (<= 199 pixels x 256 channels f16, 8 planes of 32 channels, 64-byte pixel
//    rows) stays in LDS from the first block to the last; every tap's B fragment is read
//    straight from it (a tap is a pixel shift, out-of-image taps read a zero pixel), so
//    the only operand streamed per K-step is the weights;
//  * weights stream L2 -> LDS by LDS-DMA through a 3-slot ring of 32-deep K-steps (256
//    rows x 64 B), issued two K-steps ahead; the A and B fragments of K-step j+1 are read
//    while the MFMAs of K-step j run (two register sets), one raw barrier per K-step;
//  * a conv's epilogue (border-class bias + PReLU for conv1, bias + residual for conv2)
//    writes the f16 result back into the LDS image; conv2 also stores it to the output
//    tensor, which is the next block's residual (read back by the same lane: the chain
//    runs in place on one NHWC buffer). The per-block bias tables come in by LDS-DMA
//    during the K loop of the conv before the one that needs them;
//  * 8 waves: 4 channel groups (64 channels) x 2 pixel groups (fragments 0-6 and 7-12
//    of 16 pixels): each SIMD hosts one wave of each, 52 MFMAs per SIMD per K-step.
//
// 16-byte chunk k of pixel (or weight row) q sits at chunk k ^ ((q >> 1) & 2): the 16
// lanes of a ds_read_b128 lane group then hit distinct banks for any run of 16
// consecutive pixels, i.e. for every tap shift (checked exhaustively offline).
//
// K order (tap-major, 32-channel steps, lane group = 8-channel slice) and the epilogue
// arithmetic are those of conv_fast, so the output is identical to running the blocks'
// convs one launch at a time (tests/test_gpu_chain.py asserts array equality).
#include "pc_conv_common.h"

namespace pc {

struct ChainBlock {
  const void* w1;     // conv1 weights (pre-BN and BN folded), f16, packed fragment-major (see wload)
  const float* b1;    // [9][256] border-class bias
  const float* s1;    // [256] PReLU slopes
  const void* w2;     // conv2 weights, f16, packed fragment-major
  const float* b2;    // [256] bias
};

struct ChainParams {
  const void* x;      // chain input NHWC f16, pixel stride xcs
  void* y;            // chain output NHWC f16, pixel stride ycs (every block's output)
  const ChainBlock* blk;
  int xcs, ycs, nblk, N, H, W, dbg;
  long long ktot;     // weight row stride (elements), >= 9*256
};

namespace chain {
constexpr int C = 256, NPL = 8;            // channels, 32-channel planes
// pixel slots per plane: image pixels (<= 199), slot DEAD (the epilogue's junk lanes
// write there, nobody reads it), and 8 zero slots: an out-of-image tap of a lane reads
// the zero slot congruent (mod 8) to the pixel index it would have read, so the bank
// pattern of a fragment read is that of 16 consecutive pixels (conflict-free)
constexpr int PXS = 208, ZP0 = 200, DEAD = 199;
constexpr int PS = PXS * 64;               // plane stride (bytes)
constexpr int NW = 4;                      // waves: one per SIMD, each owns 64 output channels
constexpr int TP = 13;                     // 16-pixel fragments (208 >= 199 pixels)
constexpr int KSTEPS = 9 * NPL;            // 72 K-steps of 32 per conv
constexpr int WSLOT = 64 * 64;             // one wave's K-step of weights (64 rows x 32 K, f16)
constexpr int NSLOT = 3;                   // RING mode: weight slots per wave
// LDS: [weight ring (RING mode)] [image planes] [conv1 PReLU slopes] [conv2 bias]
template <int MODE>
struct Lay {
  static constexpr int RING = MODE == 1 ? NW * NSLOT * WSLOT : 0;
  static constexpr int IMG = RING;
  static constexpr int TAB_S1 = IMG + NPL * PS;
  static constexpr int TAB_B2 = TAB_S1 + C * 4;
  static constexpr int LDS = TAB_B2 + C * 4;
  static_assert(LDS <= 163840, "LDS");
};
}  // namespace chain

__device__ __forceinline__ unsigned cswz(unsigned q) { return (q >> 1) & 2u; }

// MODE 0: weights stream straight into registers as MFMA A fragments (buffer_load_dwordx4,
//         WD K-steps ahead); MODE 1: per-wave LDS ring filled by LDS-DMA two K-steps ahead,
//         A fragments read from it one K-step ahead.
// WL: weight layout (ChainPlan packing): 0 the convs' own [256][ktot] rows; 2 repacked
//     fragment-major, 1 KiB per (channel group g, row block a, K-step j) at
//     ((g*4 + a)*72 + j)*1024, lane l's 8 K values at +16*l.
// DBG (tuning builds only): 1 no weight loads.
template <int DBG, int MODE, int WL>
__global__ __launch_bounds__(256, 1) void conv_chain(ChainParams p) {
  using namespace chain;
  using L = Lay<MODE>;
  constexpr int WD = 3;
  static_assert(NPL % (WD + 1) == 0, "weight register ring must tile a tap");
  __shared__ __attribute__((aligned(16))) char smem[L::LDS];
  const int lane = threadIdx.x & 63;
  const int cg = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);   // wave = output-channel group
  const int fr = lane & 15, kc = lane >> 4;
  const int H = p.H, W = p.W, HW = H * W;
  const int n = blockIdx.x;
  const int nconv = 2 * p.nblk;
  constexpr int IMG = L::IMG;

  auto bar = [&]() __attribute__((always_inline)) {
    asm volatile("" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
  };
  typedef const __attribute__((address_space(4))) ChainBlock* cblk_t;
  const cblk_t blks = (cblk_t)p.blk;

  // ---- image -> LDS (zero pixel slots included), block 0's conv1 slopes ----
  {
    const char* xin = reinterpret_cast<const char*>(p.x) + (size_t)n * HW * p.xcs * 2;
    constexpr int IT = PXS * 32 / (64 * NW), FC = 13;
    static_assert(IT % FC == 0 && IT * 64 * NW == PXS * 32, "fill split");
#pragma unroll
    for (int k0 = 0; k0 < IT; k0 += FC) {
      f16x8 v[FC];
#pragma unroll
      for (int k = 0; k < FC; ++k) {
        const int idx = threadIdx.x + (k0 + k) * 64 * NW;
        const int P = idx >> 5, c32 = idx & 31;
        const int Pc = P < HW ? P : 0;   // clamped: every load is issued
        v[k] = *reinterpret_cast<const f16x8*>(xin + (size_t)Pc * p.xcs * 2 + c32 * 16);
      }
#pragma unroll
      for (int k = 0; k < FC; ++k) {
        const int idx = threadIdx.x + (k0 + k) * 64 * NW;
        const int P = idx >> 5, c32 = idx & 31;
        *reinterpret_cast<f16x8*>(smem + IMG + (c32 >> 2) * PS + P * 64 + (((c32 & 3) ^ cswz(P)) << 4)) =
            P < HW ? v[k] : f16x8{};
      }
    }
    if (threadIdx.x < C / 4)
      reinterpret_cast<f32x4*>(smem + L::TAB_S1)[threadIdx.x] = reinterpret_cast<const f32x4*>(p.blk[0].s1)[threadIdx.x];
  }

  // ---- weight stream (this wave: rows cg*64 .. +63 of every K-step) ----
  auto conv_w = [&](int c) __attribute__((always_inline)) {
    const int cc = c < nconv ? c : nconv - 1;   // past the last conv: re-stage its weights (never read)
    return reinterpret_cast<const char*>((cc & 1) ? blks[cc >> 1].w2 : blks[cc >> 1].w1);
  };
  // buffer descriptors (MUBUF loads and LDS-DMA: not FLAT, so the compiler keeps counted
  // lgkmcnt waits for the fragment reads; a pending FLAT global_load_lds makes it wait
  // lgkmcnt(0) before every MFMA group)
  const unsigned wbytes = WL == 0 ? (unsigned)(C * p.ktot * 2) : (unsigned)(KSTEPS * C * 64);
  auto rsrc = [&](const void* base, unsigned bytes) __attribute__((always_inline)) {
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), (short)0, (int)bytes, 0x00020000);
  };
  // per-lane byte offsets of this lane's 16 bytes of row block a (MODE 0: its own A
  // fragment; MODE 1 with WL 0: DMA piece a = rows a*16 + lane/4, 16-byte chunk lane%4 of the
  // row swizzled by cswz(row))
  unsigned woff[4];
#pragma unroll
  for (int a = 0; a < 4; ++a) {
    if constexpr (WL == 2) {
      woff[a] = (unsigned)(((cg * 4 + a) * KSTEPS * 64 + lane) * 16);
    } else if constexpr (MODE == 0) {
      woff[a] = (unsigned)(((long long)(cg * 64 + a * 16 + fr) * p.ktot + kc * 8) * 2);
    } else {
      const int r = a * 16 + (lane >> 2);
      woff[a] = (unsigned)((long long)(cg * 64 + r) * p.ktot * 2) + (((lane & 3) ^ cswz(r)) << 4);
    }
  }
  constexpr int kstride = WL == 0 ? 64 : 1024;   // bytes between K-steps
  // MODE 0: K-step kstep -> the A fragment registers fa
  auto wload = [&](__amdgpu_buffer_rsrc_t wr, int kstep, f16x8(&fa)[4]) __attribute__((always_inline)) {
#pragma unroll
    for (int a = 0; a < 4; ++a) {
      if constexpr (DBG & 1)
        fa[a] = f16x8{};
      else
        fa[a] = __builtin_bit_cast(f16x8, __builtin_amdgcn_raw_buffer_load_b128(wr, woff[a], kstep * kstride, 0));
    }
  };
  // MODE 1: K-step kstep -> this wave's ring slot
  char* const ring = smem + cg * NSLOT * WSLOT;
  auto wdma = [&](__amdgpu_buffer_rsrc_t wr, int kstep, int slot) __attribute__((always_inline)) {
#pragma unroll
    for (int a = 0; a < 4; ++a)
      if constexpr (!(DBG & 1))
        __builtin_amdgcn_raw_ptr_buffer_load_lds(wr, (lds_ptr_t)(ring + slot * WSLOT + a * 1024), 16, woff[a],
                                                 kstep * kstride, 0, 0);
  };
  const unsigned aoff = WL == 2 ? (unsigned)(lane * 16) : (unsigned)(fr * 64 + ((kc ^ cswz(fr)) << 4));
  auto readA = [&](int slot, f16x8(&fa)[4]) __attribute__((always_inline)) {
    const char* sp = ring + slot * WSLOT + aoff;
#pragma unroll
    for (int a = 0; a < 4; ++a) fa[a] = *reinterpret_cast<const f16x8*>(sp + a * 1024);
  };
  // small per-conv tables by LDS-DMA (1 KiB, one wave; visible to the others after that
  // wave's vmcnt and the epilogue barrier)
  auto dma_tab = [&](const float* src, int dst) __attribute__((always_inline)) {
    const __amdgpu_buffer_rsrc_t tr = rsrc(src, 1024);
    if (cg == 0) __builtin_amdgcn_raw_ptr_buffer_load_lds(tr, (lds_ptr_t)(smem + dst), 16, lane * 16, 0, 0, 0);
  };

  // ---- fragment addressing ----
  unsigned ohw[TP];   // (output row << 8 | column) of this lane's pixel in fragment b; ~0u: not a pixel
#pragma unroll
  for (int b = 0; b < TP; ++b) {
    const int P = b * 16 + fr;
    const int oh = P / W;
    ohw[b] = P < HW ? (unsigned)((oh << 8) | (P - oh * W)) : ~0u;
  }
  auto bases = [&](int tap, unsigned(&bs)[TP]) __attribute__((always_inline)) {
    const int dh = tap / 3 - 1, dw = tap - (tap / 3) * 3 - 1;
#pragma unroll
    for (int b = 0; b < TP; ++b) {
      const int ih = (int)(ohw[b] >> 8) + dh, iw = (int)(ohw[b] & 255) + dw;
      const bool ok = ohw[b] != ~0u && (unsigned)ih < (unsigned)H && (unsigned)iw < (unsigned)W;
      const unsigned q = ok ? (unsigned)(ih * W + iw) : (unsigned)(ZP0 + ((b * 16 + fr + dh * W + dw) & 7));
      bs[b] = IMG + q * 64 + ((kc ^ cswz(q)) << 4);
    }
  };
  auto readB = [&](const unsigned(&bs)[TP], int pl, f16x8(&fb)[TP]) __attribute__((always_inline)) {
#pragma unroll
    for (int b = 0; b < TP; ++b) fb[b] = *reinterpret_cast<const f16x8*>(smem + bs[b] + pl * PS);
  };

  // ---- prologue: the first K-steps in flight, image and tables visible ----
  constexpr int NA = MODE == 0 ? WD + 1 : 2;   // A fragment register sets
  f16x8 wa[NA][4];
  __amdgpu_buffer_rsrc_t wcur = rsrc(conv_w(0), wbytes);
  int slot = 0;   // MODE 1: ring slot of the current K-step
  if constexpr (MODE == 0) {
    static_for<WD>([&](auto jc) __attribute__((always_inline)) {
      constexpr int j = decltype(jc)::value;
      wload(wcur, j, wa[j]);
    });
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    bar();
  } else {
    wdma(wcur, 0, 0);
    wdma(wcur, 1, 1);
    asm volatile("s_waitcnt vmcnt(4) lgkmcnt(0)" ::: "memory");
    bar();
    readA(0, wa[0]);
  }
  f16x8 fb[TP];
  unsigned bc[TP];
  bases(0, bc);
  readB(bc, 0, fb);
  f32x4 acc[4][TP];

  for (int c = 0; c < nconv; ++c) {
    const int blk = c >> 1;
    const bool second = c & 1;
    wcur = rsrc(conv_w(c), wbytes);
    const __amdgpu_buffer_rsrc_t wnext = rsrc(conv_w(c + 1), wbytes);
    // per-conv tables DMA'd with the conv's first K-step: block blk+1's PReLU slopes while
    // conv2 of block blk runs, block blk's conv2 bias while its conv1 runs
    const float* tsrc = nullptr;
    if (!second) tsrc = blks[blk].b2;
    else if (blk + 1 < p.nblk) tsrc = blks[blk + 1].s1;
    const int tdst = second ? L::TAB_S1 : L::TAB_B2;
#pragma unroll
    for (int a = 0; a < 4; ++a)
#pragma unroll
      for (int b = 0; b < TP; ++b) acc[a][b] = f32x4{0.f, 0.f, 0.f, 0.f};

    // one tap (8 K-steps); FIRST: the conv's first tap (issues the table DMA), LAST: the
    // conv's last tap (its last steps stage the next conv's weights, its last step reads no
    // B fragments)
    auto tap_body = [&](int tap, auto firstc, auto lastc) __attribute__((always_inline)) {
      constexpr bool FIRST = decltype(firstc)::value, LAST = decltype(lastc)::value;
      static_for<NPL>([&](auto plc) __attribute__((always_inline)) {
        constexpr int pl = decltype(plc)::value;
        f16x8(&cA)[4] = wa[MODE == 0 ? pl % NA : pl & 1];
        f16x8(&nA)[4] = wa[MODE == 0 ? (pl + WD) % NA : (pl + 1) & 1];
        const int s1 = slot == 2 ? 0 : slot + 1, s2 = slot == 0 ? 2 : slot - 1;
        if constexpr (MODE == 0) {
          // weights of K-step j+WD into the registers K-step j-1 used (its MFMAs are issued)
          if constexpr (LAST && pl >= NPL - WD)
            wload(wnext, pl - (NPL - WD), nA);
          else
            wload(wcur, tap * NPL + pl + WD, nA);
        } else {
          // K-step j+2 into the slot of j-1 (its A fragments were consumed by the MFMAs of j-1)
          if constexpr (LAST && pl >= NPL - 2)
            wdma(wnext, pl - (NPL - 2), s2);
          else
            wdma(wcur, tap * NPL + pl + 2, s2);
        }
        if constexpr (FIRST && pl == 0) {
          if (tsrc) dma_tab(tsrc, tdst);
        }
        constexpr bool MORE = !(LAST && pl == NPL - 1);   // B fragments of K-step j+1 in this conv
        if constexpr (pl == NPL - 1 && !LAST) bases(tap + 1, bc);
        constexpr int npl = (pl + 1) % NPL;
        // fragment b's 4 MFMAs, then its register is refilled with fragment b of K-step j+1
        // (read ~48 MFMAs ahead of its use: one B register set). MODE 1: halfway, this
        // wave's own DMA of j+1 is waited for and its A fragments are read.
        static_for<TP>([&](auto bcst) __attribute__((always_inline)) {
          constexpr int b = decltype(bcst)::value;
#pragma unroll
          for (int a = 0; a < 4; ++a)
            acc[a][b] = __builtin_amdgcn_mfma_f32_16x16x32_f16(cA[a], fb[b], acc[a][b], 0, 0, 0);
          __builtin_amdgcn_sched_barrier(0);
          if constexpr (MORE) fb[b] = *reinterpret_cast<const f16x8*>(smem + bc[b] + npl * PS);
          if constexpr (MODE == 1 && b == 3) {
            asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
            readA(s1, nA);
          }
          __builtin_amdgcn_sched_barrier(0);
        });
        slot = s1;
      });
    };
    tap_body(0, std::true_type{}, std::false_type{});
#pragma unroll 1
    for (int tap = 1; tap < 8; ++tap) tap_body(tap, std::false_type{}, std::false_type{});
    tap_body(8, std::false_type{}, std::true_type{});

    // ---- epilogue: every wave is past its last reads of the image (and the tables DMA'd
    // with the first K-step have landed: the issuing wave's later counted waits) ----
    if constexpr (MODE == 0) asm volatile("s_waitcnt vmcnt(12) lgkmcnt(0)" ::: "memory");
    else asm volatile("s_waitcnt vmcnt(4) lgkmcnt(0)" ::: "memory");
    bar();
    {
      // the epilogue's per-lane addressing is recomputed from an opaque lane id: left
      // loop-invariant, the compiler hoists all of it out of the conv loop and keeps ~150
      // address registers live through the K loop
      unsigned eo[TP];
#pragma unroll
      for (int b = 0; b < TP; ++b) {
        eo[b] = ohw[b];
        asm volatile("" : "+v"(eo[b]));
      }
      int ln = lane;
      asm volatile("" : "+v"(ln));
      const int efr = ln & 15, ekc = ln >> 4;
      // lane channels of accumulator row a: cg*64 + a*16 + ekc*4 .. +3; in the LDS image
      // that is plane cg*2 + a/2, 16-byte chunk (a&1)*2 + ekc/2, half ekc&1
      auto img_off = [&](int P, int a) __attribute__((always_inline)) {
        const int Pw = P < HW ? P : DEAD;   // pixels past the image: the dead slot
        return (unsigned)(IMG + (cg * 2 + (a >> 1)) * PS + Pw * 64 +
                          ((((a & 1) * 2 + (ekc >> 1)) ^ cswz(Pw)) << 4) + (ekc & 1) * 8);
      };
      auto chn = [&](int a) __attribute__((always_inline)) { return cg * 64 + a * 16 + ekc * 4; };
      if (!second) {
        // conv1: border-class bias (global, L2-resident) + PReLU (slopes in LDS); the bias
        // rows of a group of fragments are requested together, then the group is finished
        const float* b9 = blks[blk].b1;
        f32x4 sl[4];
#pragma unroll
        for (int a = 0; a < 4; ++a) sl[a] = *reinterpret_cast<const f32x4*>(smem + L::TAB_S1 + chn(a) * 4);
        static_for<4>([&](auto gc) __attribute__((always_inline)) {
          constexpr int g = decltype(gc)::value;
          constexpr int b0 = g * 4, b1 = (g + 1) * 4 < TP ? (g + 1) * 4 : TP;
          f32x4 bt[4][4];
#pragma unroll
          for (int b = b0; b < b1; ++b) {
            const int oh = (int)(eo[b] >> 8), ow = (int)(eo[b] & 255);
            const int rc = oh == 0 ? 0 : (oh + 1 >= H ? 2 : 1);
            const int cc = ow == 0 ? 0 : (ow + 1 >= W ? 2 : 1);
#pragma unroll
            for (int a = 0; a < 4; ++a)
              bt[b - b0][a] = *reinterpret_cast<const f32x4*>(b9 + (rc * 3 + cc) * C + chn(a));
          }
#pragma unroll
          for (int b = b0; b < b1; ++b) {
            const int P = b * 16 + efr;
#pragma unroll
            for (int a = 0; a < 4; ++a) {
              float v[4];
#pragma unroll
              for (int j = 0; j < 4; ++j) {
                float t = acc[a][b][j] + 0.f;   // conv_fast: acc + channel bias (none), then the class bias
                t += bt[b - b0][a][j];
                v[j] = t > 0.f ? t : t * sl[a][j];
              }
              *reinterpret_cast<f16x4*>(smem + img_off(P, a)) = f16x4{(f16)v[0], (f16)v[1], (f16)v[2], (f16)v[3]};
            }
          }
          __builtin_amdgcn_sched_barrier(0);
        });
      } else {
        // conv2: bias + residual (this block's input, read back from the output tensor,
        // where this lane stored it one block earlier; block 0 reads the chain input)
        const char* rsrc_p = blk == 0 ? reinterpret_cast<const char*>(p.x) : reinterpret_cast<const char*>(p.y);
        const int rcs = blk == 0 ? p.xcs : p.ycs;
        char* yimg = reinterpret_cast<char*>(p.y) + (size_t)n * HW * p.ycs * 2;
        f32x4 bt[4];
#pragma unroll
        for (int a = 0; a < 4; ++a) bt[a] = *reinterpret_cast<const f32x4*>(smem + L::TAB_B2 + chn(a) * 4);
        static_for<2>([&](auto hc) __attribute__((always_inline)) {
          constexpr int b0 = decltype(hc)::value == 0 ? 0 : 7, b1 = decltype(hc)::value == 0 ? 7 : TP;
          f16x4 rv[b1 - b0][4];
#pragma unroll
          for (int b = b0; b < b1; ++b) {
            const int P = b * 16 + efr;
            const char* rp = rsrc_p + ((size_t)n * HW + (P < HW ? P : 0)) * rcs * 2;
#pragma unroll
            for (int a = 0; a < 4; ++a) rv[b - b0][a] = *reinterpret_cast<const f16x4*>(rp + chn(a) * 2);
          }
#pragma unroll
          for (int b = b0; b < b1; ++b) {
            const int P = b * 16 + efr;
            f16x4 h[4];
#pragma unroll
            for (int a = 0; a < 4; ++a) {
              float v[4];
#pragma unroll
              for (int j = 0; j < 4; ++j) {
                float t = acc[a][b][j] + bt[a][j];
                t = t > 0.f ? t : t * 1.f;      // conv_fast's piecewise-linear act with slope 1 (none)
                v[j] = t + (float)rv[b - b0][a][j];
              }
              h[a] = f16x4{(f16)v[0], (f16)v[1], (f16)v[2], (f16)v[3]};
              *reinterpret_cast<f16x4*>(smem + img_off(P, a)) = h[a];
            }
            if (P < HW) {
#pragma unroll
              for (int a = 0; a < 4; ++a)
                *reinterpret_cast<f16x4*>(yimg + ((size_t)P * p.ycs + chn(a)) * 2) = h[a];
            }
          }
          __builtin_amdgcn_sched_barrier(0);
        });
      }
    }
    // the new image is complete before anyone reads it
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    bar();
    if (c + 1 < nconv) {
      bases(0, bc);
      readB(bc, 0, fb);    // K-step 0 of the next conv (its weights are already in flight)
    }
  }
  // drain the tail's weight loads (re-loads of the last conv, never used) before exit
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

// ---------------------------------------------------------------------------
// host side
// ---------------------------------------------------------------------------
int conv_chain_fits(int H, int W, int C, int npad, long long ktot) {
  return H > 0 && W > 0 && H * W <= chain::DEAD && H < 256 && W < 256 && C == chain::C && npad == chain::C &&
         ktot >= 9LL * chain::C && ktot * 2 * chain::C < 4294967296LL;
}

hipError_t conv_chain_launch(const void* x, int xcs, void* y, int ycs, const void* blk_dev, int nblk, int N, int H,
                             int W, long long ktot, int dbg, hipStream_t s) {
  if (!x || !y || !blk_dev || nblk <= 0 || N <= 0 || !conv_chain_fits(H, W, chain::C, chain::C, ktot) ||
      (xcs & 7) || (ycs & 7) || xcs < chain::C || ycs < chain::C ||
      ((reinterpret_cast<uintptr_t>(x) | reinterpret_cast<uintptr_t>(y)) & 15))
    return hipErrorInvalidValue;
  ChainParams p;
  p.x = x; p.y = y; p.blk = reinterpret_cast<const ChainBlock*>(blk_dev);
  p.xcs = xcs; p.ycs = ycs; p.nblk = nblk; p.N = N; p.H = H; p.W = W; p.dbg = dbg; p.ktot = ktot;
  // dbg: bit 0 tuning (no weight loads), bits 8-9 weight layout (ChainPlan::wl), bit 10 mode
  const int wl = (dbg >> 8) & 3, mode = (dbg >> 10) & 1;
#define PC_CHAIN_L(D, M, W) hipLaunchKernelGGL((conv_chain<D, M, W>), dim3(N), dim3(64 * chain::NW), 0, s, p)
#define PC_CHAIN_W(D)                                                      \
  if (mode) {                                                              \
    if (wl == 2) PC_CHAIN_L(D, 1, 2); else PC_CHAIN_L(D, 1, 0);            \
  } else {                                                                 \
    if (wl == 2) PC_CHAIN_L(D, 0, 2); else PC_CHAIN_L(D, 0, 0);            \
  }
  if (dbg & 1) {
    PC_CHAIN_W(1);
  } else {
    PC_CHAIN_W(0);
  }
#undef PC_CHAIN_W
#undef PC_CHAIN_L
  return hipGetLastError();
}

size_t conv_chain_block_bytes() { return sizeof(ChainBlock); }

}  // namespace pc
