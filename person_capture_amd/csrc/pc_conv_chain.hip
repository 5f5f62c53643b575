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
  const void* w1;     // conv1 [256][ktot] f16 (pre-BN and BN folded)
  const float* b1;    // [9][256] border-class bias
  const float* s1;    // [256] PReLU slopes
  const void* w2;     // conv2 [256][ktot] f16
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
constexpr int PXS = 200, ZP = PXS - 1;     // pixel slots per plane; the last one reads as zeros
constexpr int PS = PXS * 64;               // plane stride (bytes)
constexpr int NW = 4;                      // waves: one per SIMD, each owns 64 output channels
constexpr int TP = 13;                     // 16-pixel fragments (208 >= 199 pixels)
constexpr int WSLOT = 64 * 64;             // one wave's K-step of weights: 64 rows x 32 K (f16)
constexpr int NSLOT = 3, RING = NW * NSLOT * WSLOT;
constexpr int IMG = RING;                  // image planes
constexpr int TAB = IMG + NPL * PS;        // bias tables
constexpr int TAB_B9 = TAB;                // [9][256] f32 border-class bias of conv1
constexpr int TAB_S1 = TAB + 9 * C * 4;    // [256] PReLU slopes of conv1
constexpr int TAB_B2 = TAB_S1 + C * 4;     // [256] f32 bias of conv2
constexpr int LDS = TAB_B2 + C * 4;
constexpr int KSTEPS = 9 * NPL;            // 72 K-steps of 32 per conv
static_assert(LDS <= 163840, "LDS");
}  // namespace chain

__device__ __forceinline__ unsigned cswz(unsigned q) { return (q >> 1) & 2u; }

// DBG (tuning builds only): 1 no weight staging, 2 no MFMA, 4 no epilogue
template <int DBG>
__global__ __launch_bounds__(256, 1) void conv_chain(ChainParams p) {
  using namespace chain;
  __shared__ __attribute__((aligned(16))) char smem[LDS];
  const int lane = threadIdx.x & 63;
  const int cg = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);   // wave = output-channel group
  const int fr = lane & 15, kc = lane >> 4;
  const int H = p.H, W = p.W, HW = H * W;
  const int n = blockIdx.x;
  const int nconv = 2 * p.nblk;
  char* const ring = smem + cg * NSLOT * WSLOT;

  auto bar = [&]() __attribute__((always_inline)) {
    asm volatile("" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
  };

  // ---- image -> LDS (zero pixel slot included), block 0's conv1 tables ----
  {
    const char* xin = reinterpret_cast<const char*>(p.x) + (size_t)n * HW * p.xcs * 2;
    constexpr int IT = (PXS * 32 + 64 * NW - 1) / (64 * NW);
    static_assert(IT % 5 == 0, "fill split");
#pragma unroll
    for (int k0 = 0; k0 < IT; k0 += 5) {
      f16x8 v[5];
#pragma unroll
      for (int k = 0; k < 5; ++k) {
        const int idx = threadIdx.x + (k0 + k) * 64 * NW;
        const int P = idx >> 5, c32 = idx & 31;
        const int Pc = P < HW ? P : 0;   // clamped: every load is issued
        v[k] = *reinterpret_cast<const f16x8*>(xin + (size_t)Pc * p.xcs * 2 + c32 * 16);
      }
#pragma unroll
      for (int k = 0; k < 5; ++k) {
        const int idx = threadIdx.x + (k0 + k) * 64 * NW;
        const int P = idx >> 5, c32 = idx & 31;
        *reinterpret_cast<f16x8*>(smem + IMG + (c32 >> 2) * PS + P * 64 + (((c32 & 3) ^ cswz(P)) << 4)) =
            P < HW ? v[k] : f16x8{};
      }
    }
    const ChainBlock& B0 = p.blk[0];
    for (int i = threadIdx.x; i < 10 * C / 4; i += 64 * NW) {   // b1 [9][256] + s1 [256]
      const f32x4 t = i < 9 * C / 4 ? reinterpret_cast<const f32x4*>(B0.b1)[i]
                                    : reinterpret_cast<const f32x4*>(B0.s1)[i - 9 * C / 4];
      *reinterpret_cast<f32x4*>(smem + TAB_B9 + i * 16) = t;
    }
  }

  // ---- this wave's weight stream: rows cg*64 .. +63 of K-step (conv dc, step dks) ----
  unsigned wsrc[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int r = i * 16 + (lane >> 2);
    wsrc[i] = (unsigned)((long long)(cg * 64 + r) * p.ktot * 2) + (((lane & 3) ^ cswz(r)) << 4);
  }
  int dc = 0, dks = 0;
  const char* dptr = reinterpret_cast<const char*>(p.blk[0].w1);
  auto dma = [&](int slot) __attribute__((always_inline)) {
    const char* wk = dptr + dks * 64;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      unsigned o = wsrc[i];
      asm volatile("" : "+v"(o));
      if constexpr (!(DBG & 1))
        __builtin_amdgcn_global_load_lds((gptr_t)(wk + o), (lds_ptr_t)(ring + slot * WSLOT + i * 1024), 16, 0, 0);
    }
  };
  auto advance = [&]() __attribute__((always_inline)) {
    if (++dks == KSTEPS) {
      if (dc + 1 < nconv) {
        dks = 0;
        ++dc;
        const ChainBlock& B = p.blk[dc >> 1];
        dptr = reinterpret_cast<const char*>((dc & 1) ? B.w2 : B.w1);
      } else {
        dks = KSTEPS - 1;   // past the last step: re-stage it into a slot nobody reads
      }
    }
  };
  // bias tables of a later conv, by LDS-DMA (1 KiB pieces over the waves; visible to the
  // other waves after the issuing wave's vmcnt and the epilogue barrier)
  auto dma_tab = [&](const float* src, int dst, int pieces) __attribute__((always_inline)) {
    for (int i = cg; i < pieces; i += NW)
      __builtin_amdgcn_global_load_lds((gptr_t)(reinterpret_cast<const char*>(src) + i * 1024 + lane * 16),
                                       (lds_ptr_t)(smem + dst + i * 1024), 16, 0, 0);
  };

  // ---- fragment addressing ----
  const unsigned aoff = (unsigned)(fr * 64 + ((kc ^ cswz(fr)) << 4));
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
      const unsigned q = ok ? (unsigned)(ih * W + iw) : (unsigned)ZP;
      bs[b] = IMG + q * 64 + ((kc ^ cswz(q)) << 4);
    }
  };
  auto readA = [&](int slot, f16x8(&fa)[4]) __attribute__((always_inline)) {
    const char* s = ring + slot * WSLOT + aoff;
#pragma unroll
    for (int a = 0; a < 4; ++a) fa[a] = *reinterpret_cast<const f16x8*>(s + a * 1024);
  };
  auto readB = [&](const unsigned(&bs)[TP], int pl, f16x8(&fb)[TP]) __attribute__((always_inline)) {
#pragma unroll
    for (int b = 0; b < TP; ++b) fb[b] = *reinterpret_cast<const f16x8*>(smem + bs[b] + pl * PS);
  };

  // ---- prologue: K-steps 0 and 1 in flight, image and tables visible ----
  dma(0);
  advance();
  dma(1);
  advance();
  asm volatile("s_waitcnt vmcnt(4) lgkmcnt(0)" ::: "memory");
  bar();
  f16x8 fa0[4], fa1[4], fb[TP];
  unsigned bc[TP];
  bases(0, bc);
  readA(0, fa0);
  readB(bc, 0, fb);
  int slot = 0;   // ring slot of the current K-step
  f32x4 acc[4][TP];

  for (int c = 0; c < nconv; ++c) {
    const int blk = c >> 1;
    const bool second = c & 1;
#pragma unroll
    for (int a = 0; a < 4; ++a)
#pragma unroll
      for (int b = 0; b < TP; ++b) acc[a][b] = f32x4{0.f, 0.f, 0.f, 0.f};
    // one tap (8 K-steps); FIRST: the conv's first tap (issues the bias-table DMA),
    // LAST: the conv's last tap (no B fragments of a next step to read)
    auto tap_body = [&](int tap, auto firstc, auto lastc) __attribute__((always_inline)) {
      constexpr bool FIRST = decltype(firstc)::value, LAST = decltype(lastc)::value;
      static_for<NPL>([&](auto plc) __attribute__((always_inline)) {
        constexpr int pl = decltype(plc)::value;
        f16x8(&cA)[4] = (pl & 1) ? fa1 : fa0;
        f16x8(&nA)[4] = (pl & 1) ? fa0 : fa1;
        // K-step j: stage j+2 into the slot of j-1 (its fragments were consumed by the
        // MFMAs of j-1), then wait for this wave's own staging of j+1 only
        const int s1 = slot == 2 ? 0 : slot + 1, s2 = slot == 0 ? 2 : slot - 1;
        dma(s2);
        advance();
        if constexpr (FIRST && pl == 0) {
          if (second) {
            if (blk + 1 < p.nblk) {   // block blk+1's conv1 tables (read at conv 2blk+2)
              const ChainBlock& Bn = p.blk[blk + 1];
              dma_tab(Bn.b1, TAB_B9, 9);
              dma_tab(Bn.s1, TAB_S1, 1);
            }
          } else {                    // this block's conv2 bias (read at conv 2blk+1)
            dma_tab(p.blk[blk].b2, TAB_B2, 1);
          }
        }
        asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
        readA(s1, nA);
        constexpr bool MORE = !(LAST && pl == NPL - 1);   // B fragments of K-step j+1 in this conv
        if constexpr (pl == NPL - 1 && !LAST) bases(tap + 1, bc);
        constexpr int npl = (pl + 1) % NPL;
        // fragment b's 4 MFMAs, then its register is refilled with fragment b of K-step j+1
        // (read ~48 MFMAs ahead of its use; one B register set)
        static_for<TP>([&](auto bcst) __attribute__((always_inline)) {
          constexpr int b = decltype(bcst)::value;
          if constexpr (!(DBG & 2)) {
#pragma unroll
            for (int a = 0; a < 4; ++a)
              acc[a][b] = __builtin_amdgcn_mfma_f32_16x16x32_f16(cA[a], fb[b], acc[a][b], 0, 0, 0);
          }
          __builtin_amdgcn_sched_barrier(0);
          if constexpr (MORE) fb[b] = *reinterpret_cast<const f16x8*>(smem + bc[b] + npl * PS);
        });
        slot = s1;
        __builtin_amdgcn_sched_barrier(0);
      });
    };
    tap_body(0, std::true_type{}, std::false_type{});
#pragma unroll 1
    for (int tap = 1; tap < 8; ++tap) tap_body(tap, std::false_type{}, std::false_type{});
    tap_body(8, std::false_type{}, std::true_type{});

    // ---- epilogue: every wave is past its last reads of the image ----
    asm volatile("s_waitcnt vmcnt(4) lgkmcnt(0)" ::: "memory");
    bar();
    if constexpr (!(DBG & 4)) {
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
      const char* rsrc = blk == 0 ? reinterpret_cast<const char*>(p.x) : reinterpret_cast<const char*>(p.y);
      const int rcs = blk == 0 ? p.xcs : p.ycs;
      char* yimg = reinterpret_cast<char*>(p.y) + (size_t)n * HW * p.ycs * 2;
      // two halves of the pixel fragments: residual requests of a half go out together
      static_for<2>([&](auto hc) __attribute__((always_inline)) {
        constexpr int b0 = decltype(hc)::value == 0 ? 0 : 7, b1 = decltype(hc)::value == 0 ? 7 : TP;
        f16x4 rv[b1 - b0][4];
        if (second) {   // residual (this block's input)
#pragma unroll
          for (int b = b0; b < b1; ++b) {
            const int P = b * 16 + efr;
            const char* rp = rsrc + ((size_t)n * HW + (P < HW ? P : 0)) * rcs * 2;
#pragma unroll
            for (int a = 0; a < 4; ++a)
              rv[b - b0][a] = *reinterpret_cast<const f16x4*>(rp + (cg * 64 + a * 16 + ekc * 4) * 2);
          }
        }
#pragma unroll
        for (int b = b0; b < b1; ++b) {
          const int P = b * 16 + efr;
          const bool pix = P < HW;
          const int oh = (int)(eo[b] >> 8), ow = (int)(eo[b] & 255);
          const int rc = oh == 0 ? 0 : (oh + 1 >= H ? 2 : 1);
          const int cc = ow == 0 ? 0 : (ow + 1 >= W ? 2 : 1);
          f16x4 h[4];
#pragma unroll
          for (int a = 0; a < 4; ++a) {
            const int ch = cg * 64 + a * 16 + ekc * 4;
            float v[4];
            if (!second) {
              const f32x4 bt = *reinterpret_cast<const f32x4*>(smem + TAB_B9 + ((rc * 3 + cc) * C + ch) * 4);
              const f32x4 sl = *reinterpret_cast<const f32x4*>(smem + TAB_S1 + ch * 4);
#pragma unroll
              for (int j = 0; j < 4; ++j) {
                float t = acc[a][b][j] + 0.f;   // conv_fast: acc + channel bias (none), then the class bias
                t += bt[j];
                v[j] = t > 0.f ? t : t * sl[j];
              }
            } else {
              const f32x4 bt = *reinterpret_cast<const f32x4*>(smem + TAB_B2 + ch * 4);
#pragma unroll
              for (int j = 0; j < 4; ++j) {
                float t = acc[a][b][j] + bt[j];
                t = t > 0.f ? t : t * 1.f;      // conv_fast's piecewise-linear act with slope 1 (none)
                v[j] = t + (float)rv[b - b0][a][j];
              }
            }
            h[a] = f16x4{(f16)v[0], (f16)v[1], (f16)v[2], (f16)v[3]};
            const int c32 = ch & 31;
            // pixels past the image write to a dead slot of their plane (never read)
            const int Pw = pix ? P : ZP - 1;
            *reinterpret_cast<f16x4*>(smem + IMG + (ch >> 5) * PS + Pw * 64 +
                                      ((((c32 >> 3) ^ cswz(Pw)) << 4) | ((c32 >> 2) & 1) * 8)) = h[a];
          }
          if (second && pix) {
#pragma unroll
            for (int a = 0; a < 4; ++a)
              *reinterpret_cast<f16x4*>(yimg + ((size_t)P * p.ycs + cg * 64 + a * 16 + ekc * 4) * 2) = h[a];
          }
          __builtin_amdgcn_sched_barrier(0);   // one fragment's table reads at a time (registers)
        }
      });
    }
    // the new image is complete before anyone reads it
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    bar();
    if (c + 1 < nconv) {
      bases(0, bc);
      readB(bc, 0, fb);    // K-step 0 of the next conv (its A fragments were read with step 71)
    }
  }
  // drain every DMA (the tail re-stages) before the workgroup's LDS is released
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

// ---------------------------------------------------------------------------
// host side
// ---------------------------------------------------------------------------
int conv_chain_fits(int H, int W, int C, int npad, long long ktot) {
  return H > 0 && W > 0 && H * W <= chain::ZP - 1 && H < 256 && W < 256 && C == chain::C && npad == chain::C &&
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
  switch (dbg & 7) {
    case 0: hipLaunchKernelGGL(conv_chain<0>, dim3(N), dim3(64 * chain::NW), 0, s, p); break;
    case 1: hipLaunchKernelGGL(conv_chain<1>, dim3(N), dim3(64 * chain::NW), 0, s, p); break;
    case 2: hipLaunchKernelGGL(conv_chain<2>, dim3(N), dim3(64 * chain::NW), 0, s, p); break;
    case 3: hipLaunchKernelGGL(conv_chain<3>, dim3(N), dim3(64 * chain::NW), 0, s, p); break;
    case 4: hipLaunchKernelGGL(conv_chain<4>, dim3(N), dim3(64 * chain::NW), 0, s, p); break;
    default: hipLaunchKernelGGL(conv_chain<7>, dim3(N), dim3(64 * chain::NW), 0, s, p); break;
  }
  return hipGetLastError();
}

size_t conv_chain_block_bytes() { return sizeof(ChainBlock); }

}  // namespace pc
