// 3x3 stride-1 "same" convolution over 2-D pixel blocks with weights held in
// registers (gfx950) - the small-channel trunk layers (Cin 32/64 -> 32/64 channels:
// SCRFD's 320x320 / 160x160 / 80x80 stages, IResNet's 112x112 / 56x56 stage).
//
// Why a third conv kernel: at 32-64 channels the implicit-GEMM kernels (pc_conv_fast)
// stage one im2col row per (pixel, tap), i.e. every input pixel moves L2 -> LDS nine
// times, and their K loop is only 9-18 tiles long, so prologue, barriers and the
// per-tile epilogue dominate (SCRFD 320x320x32: 157 TF/s; 160x160x64: 340 TF/s). The
// linear-run halo kernel (pc_conv_halo) stages each pixel once but its halo is the
// pixel run +- (W+1), 2-3x the tile on wide images. Here:
//
//  * a workgroup (8 waves) is persistent over output blocks of TH x 16 pixels of one
//    image (TH = 32 / 16 for 32 / 64 output channels); the block's input halo
//    (TH+2) x 18 pixels x Cin is staged into LDS once, by LDS-DMA, double-buffered:
//    block i+1's halo is in flight while block i is multiplied;
//  * the whole weight matrix of a wave's 32 output channels (9 x Cin of K) lives in
//    VGPRs as MFMA A-fragments for the life of the workgroup, so the only LDS traffic
//    is one ds_read_b128 B-fragment per 2 MFMAs;
//  * halo rows are 64 B (one 32-channel chunk), row pitch 24 pixels; 16-byte chunk c of
//    row r sits at c ^ ((r >> 1) & 3) (conflict-free ds_read_b128 for any 16 consecutive
//    rows, pc_conv_halo.hip), and with the pitch a multiple of 8 a tap-row shift keeps
//    the swizzle, so every tap's fragment address is one of 3 per-lane bases per
//    fragment plus a compile-time immediate;
//  * one barrier per block; the epilogue (bias / border-class bias, activation,
//    residual, channel padding; conv_epilogue_map) stores straight from the
//    accumulators after the barrier, while the next block's DMA is in flight.
//
// K order (tap-major, 32-channel chunks, lane group fq = 8-channel slice) is the
// implicit-GEMM kernels' order, so results are bit-identical to conv_fast's.
#include <stdlib.h>
#include "pc_conv_common.h"

namespace pc {

// B-fragment reads of one K step: TP rows P pixels apart, compile-time offsets
template <int STRIDE, int IMM, int... I>
__device__ __forceinline__ void t2d_read_frags(const char* a0, f16x8* fb, std::integer_sequence<int, I...>) {
  ((fb[I] = *reinterpret_cast<const f16x8*>(a0 + IMM + I * STRIDE)), ...);
}
// NCH: 32-channel input chunks (Cin = 32*NCH); G: 32-channel output groups (npad = 32*G);
// NW waves, each owning TP output rows of 16 pixels x 32 output channels.
// NBUF 3: three halo buffers, block i+2's halo is requested while block i is multiplied (the
// DMA of one block of small TH does not hide behind one block's K loop).
// SPLIT (f16x3 detector): the input is a split tensor [hi | lo] (NCH physical
// chunks = 2 x the logical ones). Per tap and logical chunk j the wave reads the two B
// fragments (hi: chunk j, lo: chunk NCC + j) once and issues W_hi*hi, W_lo*hi, W_hi*lo, with
// W_hi and W_lo each held once in registers (the weight rows are packed [W_hi, W_hi, W_lo] per
// tap for the implicit-GEMM kernels' virtual K; the duplicate is not loaded). The residual is
// read as hi + lo and the output is written split. (Accumulation order: per chunk, not the
// implicit-GEMM kernels' [hi, lo, hi] blocks: equal to them at f32 class, not bitwise.)
template <int NCH, int G, int NW, int TP, int NBUF = 2, bool SPLIT = false>
__global__ __launch_bounds__(64 * NW, 1) void conv_t2d(ConvParams p, int nty, int ntx, int ntiles) {
  constexpr int TW = 16, P = 24, TC = 2;
  constexpr int TH = TP * NW / G;             // output rows per block
  constexpr int NRP = (TH + 2) * P;           // halo rows per channel chunk
  constexpr int NINST = NRP / 16;             // DMA instructions per chunk
  constexpr int BUFB = NCH * NRP * 64;        // one halo buffer
  static_assert(!SPLIT || NCH % 2 == 0, "split halo: hi and lo chunks");
  constexpr int NCC = SPLIT ? NCH / 2 : NCH;  // logical 32-channel chunks
  constexpr int NKS = 9 * NCC;                // K steps (split: each is 3 MFMA products)
  constexpr int NPAD_T = 32 * G;
  constexpr int TB = 10 * NPAD_T;             // bias classes [9][npad] + slopes [npad] (f32)
  static_assert(NRP % 16 == 0 && P % 8 == 0 && P >= TW + 2 && (TP == 4 || TP == 8), "halo geometry");
  // output staging: its own LDS area, or (when the two halo buffers leave no room) the block's
  // own halo buffer, free once every wave is past the K loop's closing barrier
  static_assert(NBUF == 2 || NBUF == 3, "halo buffers");
  constexpr int NS = SPLIT ? 2 : 1;           // halves per staged output pixel (hi, lo)
  constexpr int STGB = TH * 16 * (NS * 64 * G + 16);
  constexpr bool ALIAS = NBUF * BUFB + TB * 4 + STGB > 163840;
  static_assert(NBUF == 2 || !ALIAS, "three halo buffers need their own staging area");
  static_assert(NBUF * BUFB + TB * 4 + (ALIAS ? 0 : STGB) <= 163840, "LDS");
  static_assert(!ALIAS || STGB <= BUFB, "staging in a halo buffer");
  static_assert(NW % G == 0, "wave roles");

  // two halo buffers as two objects: the compiler then sees that a ds_read of one
  // cannot alias the LDS-DMA into the other and does not drain vmcnt before it
  __shared__ __attribute__((aligned(16))) char hbuf0[BUFB];
  __shared__ __attribute__((aligned(16))) char hbuf1[BUFB];
  __shared__ __attribute__((aligned(16))) char hbuf2[NBUF == 3 ? BUFB : 16];
  __shared__ __attribute__((aligned(16))) float tab[TB];
  // output staging: [pixel][npad] f16 rows, pitch padded by 16 B (conflict-free 8-byte
  // fragment writes, 16-byte aligned row reads)
  constexpr int NPAD = 32 * G, PITCH = NS * NPAD * 2 + 16, BPIX = TH * TW, CH8 = NPAD / 8;
  constexpr int SIT = BPIX * NS * CH8 / (64 * NW);   // 16-byte chunks per thread per block
  static_assert(SIT * 64 * NW == BPIX * NS * CH8, "staging split");
  __shared__ __attribute__((aligned(16))) char stg_own[ALIAS ? 16 : BPIX * PITCH];

  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  __builtin_assume(wave >= 0 && wave < NW);
  const int g = wave % G, pg = wave / G;      // output-channel group, pixel-row group
  const int fr = lane & 15, fq = lane >> 4;
  const ConvSeg& S = p.seg[0];
  // MUBUF LDS-DMA over the input (buffer_load ... lds): a pending FLAT global_load_lds also
  // counts in lgkmcnt, which made the compiler wait lgkmcnt(0) before nearly every MFMA
  // (125 such waits for 144 MFMAs) instead of counting the fragment reads
  const __amdgpu_buffer_rsrc_t xrs =
      __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(S.x), (short)0, (int)0xffffffff, 0x00020000);
  const unsigned xrow = (unsigned)S.cs * 2u;
  const int H = S.H, W = S.W;

  // blocks of one XCD form a contiguous range (neighbouring halos share its L2)
  int t_hi = ntiles, t_first = blockIdx.x, t_step = gridDim.x;
  if ((gridDim.x & 7) == 0) {
    const int xcd = blockIdx.x & 7;
    const int t_lo = (int)((long long)xcd * ntiles / 8);
    t_hi = (int)((long long)(xcd + 1) * ntiles / 8);
    t_first = t_lo + (blockIdx.x >> 3);
    t_step = gridDim.x >> 3;
  }
  if (t_first >= t_hi) return;   // whole workgroup: nothing issued, no barrier pending

  auto decode = [&](int tile, int& n, int& ty, int& tx) __attribute__((always_inline)) {
    const int per = nty * ntx;
    n = tile / per;
    const int r = tile - n * per;
    ty = r / ntx;
    tx = r - ty * ntx;
  };

  // halo of block `tile` -> buffer dst (rows past the image / pitch padding read zeros)
  constexpr int NDMA = NCH * NINST, PERW = (NDMA + NW - 1) / NW;
  auto dma = [&](int tile, char* dst) __attribute__((always_inline)) {
    int n, ty, tx;
    decode(tile, n, ty, tx);
    const int oy0 = ty * TH - 1, ox0 = tx * TW - 1;
    static_for<PERW>([&](auto kc) __attribute__((always_inline)) {
      const int i = decltype(kc)::value * NW + wave;
      if (NDMA % NW == 0 || i < NDMA) {
        const int j = i / NINST, gi = i - j * NINST;
        const int h = gi * 16 + (lane >> 2);
        const int hy = h / P, hx = h - hy * P;
        const int iy = oy0 + hy, ix = ox0 + hx;
        const unsigned sc = (unsigned)(((lane & 3) ^ ((h >> 1) & 3)) << 4);
        const bool ok = hx < TW + 2 && (unsigned)iy < (unsigned)H && (unsigned)ix < (unsigned)W;
        const unsigned pix = (unsigned)((n * H + iy) * W + ix);
        unsigned off = ok ? pix * xrow + sc : S.zero_off + sc;
        asm volatile("" : "+v"(off));
        __builtin_amdgcn_raw_ptr_buffer_load_lds(xrs, (lds_ptr_t)(dst + j * NRP * 64 + gi * 1024), 16, off, j * 64, 0,
                                                 0);
      }
    });
  };

  int tile = t_first;
  dma(tile, hbuf0);
  if constexpr (NBUF == 3) {
    if (tile + t_step < t_hi) dma(tile + t_step, hbuf1);
  }

  // epilogue tables: bias of border class c (BIAS_BORDER9; BIAS_CHANNEL: every class the
  // same row) at [c*npad + ch], negative-side slopes at [9*npad + ch] (PReLU a, ReLU 0, none 1)
  for (int i = threadIdx.x; i < TB; i += 64 * NW) {
    const int cls = i / NPAD_T, c = i - cls * NPAD_T;
    float v = 0.f;
    if (c < p.npad) {
      if (cls < 9) {
        if (p.bias_mode == BIAS_CHANNEL) v = p.bias[c];
        else if (p.bias_mode == BIAS_BORDER9) v = p.bias[cls * p.npad + c];
      } else {   // negative-side slope of the piecewise-linear activations
        v = p.act == ACT_PRELU ? p.slope[c] : (p.act == ACT_RELU ? 0.f : 1.f);
      }
    }
    tab[i] = v;
  }

  // weights -> registers: A fragment (ks, a) = rows g*32 + a*16 + fr, K ks*32 + fq*8 .. +7
  // (split: step ks = tap*NCC + j holds W_hi of virtual chunk tap*3NCC + j in wa and W_lo of
  // virtual chunk tap*3NCC + 2NCC + j in wl)
  f16x8 wa[NKS][TC];
  f16x8 wl[SPLIT ? NKS : 1][TC];
  {
    const char* wb = reinterpret_cast<const char*>(p.w);
#pragma unroll
    for (int a = 0; a < TC; ++a) {
      const char* row = wb + (long long)(g * 32 + a * 16 + fr) * p.ktot * 2 + fq * 16;
#pragma unroll
      for (int ks = 0; ks < NKS; ++ks) {
        if constexpr (SPLIT) {
          const int tap = ks / NCC, j = ks - tap * NCC;
          wa[ks][a] = *reinterpret_cast<const f16x8*>(row + (tap * 3 * NCC + j) * 64);
          wl[ks][a] = *reinterpret_cast<const f16x8*>(row + (tap * 3 * NCC + 2 * NCC + j) * 64);
        } else {
          wa[ks][a] = *reinterpret_cast<const f16x8*>(row + ks * 64);
        }
      }
    }
    // retire the weight loads here, visibly to the compiler: otherwise its wait for them
    // lands before the first MFMA inside the block loop as a vmcnt(0), which would also
    // wait for the next block's halo DMA
#pragma unroll
    for (int a = 0; a < TC; ++a)
#pragma unroll
      for (int ks = 0; ks < NKS; ++ks) {
        asm volatile("" : "+v"(wa[ks][a]));
        if constexpr (SPLIT) asm volatile("" : "+v"(wl[ks][a]));
      }
  }

  auto bar = [&]() __attribute__((always_inline)) {
    asm volatile("" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
  };
  asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
  bar();

  const bool has_res = p.res_mode != RES_NONE;
  const bool border = p.bias_mode == BIAS_BORDER9;
  const int chq = fq * 4;

  f32x4 acc[TC][TP];
  // one block: multiply from `cur` while the next block's halo goes into `oth`
  auto block = [&](char* cur, char* oth) __attribute__((always_inline)) {
    char* stg = ALIAS ? cur : stg_own;
    const int nxt = tile + t_step;
    // NBUF 2: the next block's halo into `oth` now; NBUF 3: block i+1's halo is already in
    // flight, block i+2's goes into `oth` after this block's residual loads (so the wait at
    // the end of the K loop can leave it outstanding)
    const bool dma2 = NBUF == 3 && nxt + t_step < t_hi && !(p.dbg & 1);
    if constexpr (NBUF == 2) {
      if (nxt < t_hi && !(p.dbg & 1)) dma(nxt, oth);   // dbg (tuning only): 1 no halo DMA
    }

    int n, ty, tx;
    decode(tile, n, ty, tx);
    const int oy0 = ty * TH + pg * TP, ox = tx * TW + fr;
    const bool colok = ox < W;

    // residual of this block's pixels, requested now so it arrives during the MFMAs
    // (not zero-filled when unused: writing registers that a load of the previous block
    // targeted would make the compiler drain vmcnt - the next halo - right here)
    f16x4 rv[TP][TC];
    f16x4 rl[SPLIT ? TP : 1][TC];   // the residual's lo half (split)
    // (addresses of pixels outside the image are clamped, not branched around: a load
    // under a divergent branch merges into a phi that waits for it right there)
    // Row part of the address is wave-uniform (scalar math, 64-bit), the lane part a 24-bit
    // multiply (pixel column x pixel stride < 2^32): the per-lane 64-bit multiply chains of the
    // first version were a large share of the kernel's VALU work. Lanes past the image read
    // column 0 of the row (their values are never stored).
    if (has_res) {
      const bool up2 = p.res_mode == RES_UP2;
      const unsigned rcs = (unsigned)p.rcs;
      const unsigned lcol = (unsigned)(colok ? (up2 ? ox >> 1 : ox) : 0);
      const unsigned loff = __umul24(lcol, rcs);
#pragma unroll
      for (int t = 0; t < TP; ++t) {
        const int oy = oy0 + t;
        const int qy = oy < H ? oy : 0;
        const long long rrow = up2 ? ((long long)n * p.rH + (qy >> 1)) * p.rW : ((long long)n * H + qy) * W;
        const f16* rp = reinterpret_cast<const f16*>(p.res) + rrow * p.rcs + loff;
#pragma unroll
        for (int a = 0; a < TC; ++a) {
          const int ch = g * 32 + a * 16 + chq;
          if constexpr (SPLIT) {   // planner: whole 8-channel groups
            rv[t][a] = *reinterpret_cast<const f16x4*>(rp + min(ch, p.cwrite - 4));
            rl[t][a] = *reinterpret_cast<const f16x4*>(rp + p.rsplit + min(ch, p.cwrite - 4));
          } else if ((p.cwrite & 3) == 0) {   // uniform: whole 4-channel groups
            rv[t][a] = *reinterpret_cast<const f16x4*>(rp + min(ch, p.cwrite - 4));
          } else {
            rv[t][a] = f16x4{};
            for (int j = 0; j < 4; ++j)
              if (ch + j < p.cwrite) rv[t][a][j] = rp[ch + j];
          }
        }
      }
    }

    if constexpr (NBUF == 3) {
      if (dma2) dma(nxt + t_step, oth);
    }
#pragma unroll
    for (int a = 0; a < TC; ++a)
#pragma unroll
      for (int t = 0; t < TP; ++t) acc[a][t] = f32x4{0.f, 0.f, 0.f, 0.f};

    // per-lane fragment bases for tap column tw; fragment t (output row pg*TP + t) is
    // t*P rows further, and as P*t/2 is a multiple of 4 it keeps the swizzle: immediate
    unsigned ad[3];
#pragma unroll
    for (int tw = 0; tw < 3; ++tw) {
      const int h = pg * TP * P + tw + fr;
      ad[tw] = (unsigned)(h * 64 + ((fq ^ ((h >> 1) & 3)) << 4));
    }
    // K step ks = (th*3 + tw)*NCH + j; its B fragments are read one step ahead of its
    // MFMAs (two fragment sets live; the schedule is pinned so the compiler does not
    // hoist every read of the block and spill the weight registers).
    f16x8 fb0[TP], fb1[TP];
    f16x8 fl0[SPLIT ? TP : 1], fl1[SPLIT ? TP : 1];   // split: the lo-chunk fragments
    if (!(p.dbg & 2)) static_for<NKS + 1>([&](auto ksc) __attribute__((always_inline)) {
      constexpr int ks = decltype(ksc)::value - 1;   // -1: prologue read of step 0
      f16x8(&cur_f)[TP] = (ks & 1) ? fb1 : fb0;
      f16x8(&nxt_f)[TP] = (ks & 1) ? fb0 : fb1;
      constexpr int H1 = TP > 4 ? 4 : TP;   // reads issued before the wait
      if constexpr (ks + 1 < NKS) {
        constexpr int tap = (ks + 1) / NCC, j = (ks + 1) - tap * NCC;
        constexpr int th = tap / 3, tw = tap - th * 3;
        t2d_read_frags<P * 64, j * NRP * 64 + th * P * 64>(cur + ad[tw], nxt_f,
                                                          std::make_integer_sequence<int, H1>{});
        if constexpr (SPLIT) {   // the lo half of the same pixels and channels: halo chunk NCC + j
          f16x8(&nxt_l)[SPLIT ? TP : 1] = (ks & 1) ? fl0 : fl1;
          t2d_read_frags<P * 64, (NCC + j) * NRP * 64 + th * P * 64>(cur + ad[tw], nxt_l,
                                                                      std::make_integer_sequence<int, TP>{});
        }
      }
      if constexpr (ks + 1 < NKS && TP > H1) {
        constexpr int tap = (ks + 1) / NCC, j = (ks + 1) - tap * NCC;
        constexpr int th = tap / 3, tw = tap - th * 3;
        t2d_read_frags<P * 64, j * NRP * 64 + th * P * 64 + H1 * P * 64>(cur + ad[tw], nxt_f + H1,
                                                                       std::make_integer_sequence<int, TP - H1>{});
      }
      if constexpr (ks >= 0) {
#pragma unroll
        for (int a = 0; a < TC; ++a)
#pragma unroll
          for (int t = 0; t < TP; ++t)
            acc[a][t] = __builtin_amdgcn_mfma_f32_16x16x32_f16(wa[ks][a], cur_f[t], acc[a][t], 0, 0, 0);
        if constexpr (SPLIT) {   // + W_lo * x_hi + W_hi * x_lo (f32 accumulation)
          f16x8(&cur_l)[SPLIT ? TP : 1] = (ks & 1) ? fl1 : fl0;
#pragma unroll
          for (int a = 0; a < TC; ++a)
#pragma unroll
            for (int t = 0; t < TP; ++t)
              acc[a][t] = __builtin_amdgcn_mfma_f32_16x16x32_f16(wl[ks][a], cur_f[t], acc[a][t], 0, 0, 0);
#pragma unroll
          for (int a = 0; a < TC; ++a)
#pragma unroll
            for (int t = 0; t < TP; ++t)
              acc[a][t] = __builtin_amdgcn_mfma_f32_16x16x32_f16(wa[ks][a], cur_l[t], acc[a][t], 0, 0, 0);
        }
      }
      __builtin_amdgcn_sched_barrier(0);
    });

    // next halo landed (own DMAs; also the residual) and every wave is done with `cur`;
    // NBUF 3: block i+2's DMA (issued last; every wave issued at least NDMA / NW of it) may
    // stay in flight
    if constexpr (NBUF == 3) {
      if (dma2) {
        static_assert(NDMA / NW <= 63, "vmcnt range");
        asm volatile("s_waitcnt vmcnt(%0)" :: "n"(NDMA / NW) : "memory");
      } else {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      }
    } else {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    bar();

    // ---- epilogue: bias (per channel / border class), activation, residual, padding ----
    f32x4 sl[TC];
    const int cc = !border ? 0 : (ox == 0 ? 0 : (ox >= W - 1 ? 2 : 1));
#pragma unroll
    for (int a = 0; a < TC; ++a) sl[a] = *reinterpret_cast<const f32x4*>(tab + 9 * NPAD_T + g * 32 + a * 16 + chq);
    // finishing: the planner sends only the piecewise-linear activations here (none /
    // ReLU / PReLU: one select with the per-channel negative slope of the table, 1 / 0 /
    // a), so the act-before / act-after-residual order is a select, not a branch
    if (!has_res) {
#pragma unroll
      for (int t = 0; t < TP; ++t)
#pragma unroll
        for (int a = 0; a < TC; ++a) {
          rv[t][a] = f16x4{};
          if constexpr (SPLIT) rl[t][a] = f16x4{};
        }
    }
    const bool after = p.act_after_res != 0;
    // f16 rows through LDS: each pixel's channels leave as whole 16-byte chunks of
    // contiguous pixel rows (per-fragment 8-byte stores of 16 pixels ran the kernel at a
    // third of its no-store speed)
#pragma unroll
    for (int t = 0; t < TP; ++t) {
      const int oy = oy0 + t;
      const int rc = !border ? 0 : (oy == 0 ? 0 : (oy >= H - 1 ? 2 : 1));
#pragma unroll
      for (int a = 0; a < TC; ++a) {
        const int ch = g * 32 + a * 16 + chq;
        const f32x4 bt = *reinterpret_cast<const f32x4*>(tab + (rc * 3 + cc) * NPAD_T + ch);
        float v[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const float x = acc[a][t][j] + bt[j];
          const float r = SPLIT ? (float)rv[t][a][j] + (float)rl[t][a][j] : (float)rv[t][a][j];
          const float xr = x + r;                                    // act(acc + b + res)
          const float y1 = xr > 0.f ? xr : xr * sl[a][j];
          const float y0 = (x > 0.f ? x : x * sl[a][j]) + r;         // act(acc + b) + res
          v[j] = ch + j < p.cout ? (after ? y1 : y0) : 0.f;          // channel padding stays 0
        }
        const f16x4 h = f16x4{(f16)v[0], (f16)v[1], (f16)v[2], (f16)v[3]};
        *reinterpret_cast<f16x4*>(stg + ((pg * TP + t) * TW + fr) * PITCH + ch * 2) = h;
        if constexpr (SPLIT)
          *reinterpret_cast<f16x4*>(stg + ((pg * TP + t) * TW + fr) * PITCH + (NPAD + ch) * 2) =
              f16x4{(f16)(v[0] - (float)h[0]), (f16)(v[1] - (float)h[1]), (f16)(v[2] - (float)h[2]),
                    (f16)(v[3] - (float)h[3])};
      }
    }
    __syncthreads();
    if (!(p.dbg & 4)) {   // dbg 4 (tuning only): no stores
      const int cw8 = (p.cwrite + 7) >> 3;
      // block origin (uniform, 64-bit) + lane offset in 32 bits (one image's elements < 2^32)
      f16* const yblk = reinterpret_cast<f16*>(p.y) + (((long long)n * H + ty * TH) * W + tx * TW) * p.ycs;
      const unsigned ycs = (unsigned)p.ycs;
#pragma unroll
      for (int k = 0; k < SIT; ++k) {
        const int idx = threadIdx.x + k * 64 * NW;
        const int pl = idx / (NS * CH8), cqs = idx - (idx / (NS * CH8)) * (NS * CH8);
        const int half = SPLIT && cqs >= CH8 ? 1 : 0, cq = cqs - half * CH8;
        const int ry = pl / TW, rx = pl & (TW - 1);
        const int oy = ty * TH + ry, oxx = tx * TW + rx;
        if (oy >= H || oxx >= W || cq >= cw8) continue;
        const f16x8 val = *reinterpret_cast<const f16x8*>(stg + pl * PITCH + cqs * 16);
        f16* yp = yblk + (__umul24((unsigned)(ry * W + rx), ycs) + (unsigned)(cq * 8 + half * p.ysplit));
        if (cq * 8 + 8 <= p.cwrite) {
          *reinterpret_cast<f16x8*>(yp) = val;
        } else {
          for (int j = 0; j < 8; ++j)
            if (cq * 8 + j < p.cwrite) yp[j] = val[j];
        }
      }
    }
    // aliased staging: the next block's DMA targets this buffer; every wave must be done reading it
    if constexpr (ALIAS) bar();
    tile = nxt;
  };
  if constexpr (NBUF == 3) {
    for (;;) {
      block(hbuf0, hbuf2);
      if (tile >= t_hi) break;
      block(hbuf1, hbuf0);
      if (tile >= t_hi) break;
      block(hbuf2, hbuf1);
      if (tile >= t_hi) break;
    }
  } else {
    for (;;) {
      block(hbuf0, hbuf1);
      if (tile >= t_hi) break;
      block(hbuf1, hbuf0);
      if (tile >= t_hi) break;
    }
  }
}

// ---------------------------------------------------------------------------
// host side
// ---------------------------------------------------------------------------

// Instantiations (variants): NCH 32-channel input chunks (split: hi + lo chunks), G 32-channel
// output groups, NW waves, TP output rows per wave (a block is TP*NW/G rows x 16 pixels), NBUF
// halo buffers. The wide shapes (Cin/npad 96 and 128: SCRFD's 80x80x96 trunk, IResNet's 28x28x128
// stage) hold 216 / 288 weight registers per wave, so they run one wave per SIMD: 3 waves for 96
// output channels (one SIMD idle), 4 for 128. SCRFD-10G 80x80x96 (N 64): 200 -> 134 us per conv,
// the net 6.24 -> 5.62 ms (r03o). The planner picks a variant once (conv_t2d_select, at
// pc_net_create: the tuning switches are read there) and the launch runs exactly that one.
template <int NCH, int G, int NW, int TP, int NBUF = 2, bool SPLIT = false>
static hipError_t launch_t2d(const ConvParams& p, hipStream_t s) {
  static int ncu = 0;
  if (!ncu) {
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || ncu <= 0)
      ncu = 256;
  }
  constexpr int TH = TP * NW / G;
  const int nty = (p.OH + TH - 1) / TH, ntx = (p.OW + 15) / 16;
  const long long nt = (long long)p.N * nty * ntx;
  if (nt <= 0 || nt >= (1LL << 31)) return hipErrorInvalidValue;
  const int grid = (int)std::min<long long>(nt, ncu);
  hipLaunchKernelGGL((conv_t2d<NCH, G, NW, TP, NBUF, SPLIT>), dim3(grid), dim3(64 * NW), 0, s, p, nty, ntx, (int)nt);
  return hipGetLastError();
}

struct T2dVariant {
  int cin, npad;   // logical input channels, padded output channels
  int nch, g, nw, tp, nbuf;
  bool split;
  hipError_t (*launch)(const ConvParams&, hipStream_t);
};
static const T2dVariant kT2d[] = {
    {32, 32, 1, 1, 8, 4, 2, false, launch_t2d<1, 1, 8, 4>},            // 0
    {32, 64, 1, 2, 8, 4, 2, false, launch_t2d<1, 2, 8, 4>},            // 1
    {32, 64, 1, 2, 8, 4, 3, false, launch_t2d<1, 2, 8, 4, 3>},         // 2  PC_T2D_NBUF3
    {64, 64, 2, 2, 4, 8, 2, false, launch_t2d<2, 2, 4, 8>},            // 3  (144 weight registers: 4 waves of 8 rows)
    {64, 64, 2, 2, 4, 4, 3, false, launch_t2d<2, 2, 4, 4, 3>},         // 4  PC_T2D_NBUF3
    {96, 96, 3, 3, 3, 4, 2, false, launch_t2d<3, 3, 3, 4>},            // 5
    {96, 96, 3, 3, 3, 4, 3, false, launch_t2d<3, 3, 3, 4, 3>},         // 6  PC_T2D_NBUF3
    {64, 96, 2, 3, 3, 8, 2, false, launch_t2d<2, 3, 3, 8>},            // 7
    {64, 96, 2, 3, 3, 8, 3, false, launch_t2d<2, 3, 3, 8, 3>},         // 8  PC_T2D_NBUF3
    {128, 128, 4, 4, 4, 4, 2, false, launch_t2d<4, 4, 4, 4>},          // 9  PC_T2D_128 (opt-in)
    {128, 128, 4, 4, 4, 8, 2, false, launch_t2d<4, 4, 4, 8>},          // 10 PC_T2D_128=8
    {32, 32, 2, 1, 4, 4, 2, true, launch_t2d<2, 1, 4, 4, 2, true>},    // 11 split
    {32, 64, 2, 2, 4, 4, 2, true, launch_t2d<2, 2, 4, 4, 2, true>},    // 12 split
    {64, 64, 4, 2, 4, 4, 2, true, launch_t2d<4, 2, 4, 4, 2, true>},    // 13 split, PC_T2D_SPLIT64 (opt-in)
};
static const int kNumT2d = sizeof(kT2d) / sizeof(kT2d[0]);

// The variant for (cin, npad) and the planner's tuning switches, or -1.
// split (f16x3): the split t2d reads each tap's hi and lo fragments once; 64 channels (288 weight
// registers, one wave per SIMD, 8-row blocks) measured slower than conv_fast's 64x512 tile on
// SCRFD 160x160x64 (611 vs 557-572 us, r04d): opt-in. 128 channels measured slower than
// conv_fast's 128x256 tile (IResNet 28x28x128 b256: 101.8 vs 96.0 us per conv, r03o): opt-in.
static int t2d_variant(int cin, int npad, int split) {
  if (split) {
    if (getenv("PC_T2D_SPLIT") && atoi(getenv("PC_T2D_SPLIT")) == 0) return -1;   // tuning: off
    if (cin == 32 && npad == 32) return 11;
    if (cin == 32 && npad == 64) return 12;
    if (cin == 64 && npad == 64 && getenv("PC_T2D_SPLIT64")) return 13;
    return -1;
  }
  const bool wide = !getenv("PC_T2D_NARROW");          // tuning: the round-2 shapes only
  const bool la = getenv("PC_T2D_NBUF3") != nullptr;   // tuning: two-block halo lookahead
  if (cin == 32 && npad == 32) return 0;
  if (cin == 32 && npad == 64) return la ? 2 : 1;
  if (cin == 64 && npad == 64) return la ? 4 : 3;
  if (wide && cin == 96 && npad == 96) return la ? 6 : 5;
  if (wide && cin == 64 && npad == 96) return la ? 8 : 7;
  if (wide && cin == 128 && npad == 128 && getenv("PC_T2D_128")) return atoi(getenv("PC_T2D_128")) == 8 ? 10 : 9;
  return -1;
}

// piecewise-linear activations, f16 output in whole 16-byte pixel chunks: the variant id, or -1
// if the conv cannot run here. split: input / output / residual are f16x3 split tensors (cin
// logical); only split-in -> split-out convs (the detector trunk) run here.
int conv_t2d_select(int cin, int npad, int KH, int KW, int stride, int pad, int act, int out_f32, int ycs,
                    int ycoff, int split) {
  if (KH != 3 || KW != 3 || stride != 1 || pad != 1) return -1;
  if (act != ACT_NONE && act != ACT_RELU && act != ACT_PRELU) return -1;
  if (out_f32 || (ycs & 7) || (ycoff & 7)) return -1;
  return t2d_variant(cin, npad, split);
}

// output rows per block of a variant (the block is TH x 16 pixels)
int conv_t2d_rows(int variant) {
  if (variant < 0 || variant >= kNumT2d) return 16;
  const T2dVariant& v = kT2d[variant];
  return v.tp * v.nw / v.g;
}

hipError_t conv_t2d_launch(const ConvParams& p, int variant, hipStream_t s) {
  if (variant < 0 || variant >= kNumT2d) return hipErrorInvalidValue;
  const T2dVariant& v = kT2d[variant];
  const ConvSeg& S = p.seg[0];
  const int cin = v.split ? S.C / 2 : S.C;
  // the conv must be the one the variant was planned for (checked, not re-derived)
  if (p.nseg != 1 || p.splitk != 1 || S.H != p.OH || S.W != p.OW || p.cwrite > p.npad || cin != v.cin ||
      p.npad != v.npad || S.KH != 3 || S.KW != 3 || S.stride != 1 || S.pad != 1 || p.out_f32 || (p.ycs & 7) ||
      (p.act != ACT_NONE && p.act != ACT_RELU && p.act != ACT_PRELU) || (reinterpret_cast<uintptr_t>(p.y) & 15))
    return hipErrorInvalidValue;
  if (v.split) {
    // split-in -> split-out: [hi | lo] halo of 2 x cin channels, virtual K 3 x cin per tap
    if (p.cwrite % 8 || S.cs != S.C || S.vwrap * 3 != S.cblk * 2 || !p.ysplit || (p.ysplit & 7) ||
        (p.res_mode != RES_NONE && (!p.rsplit || (p.rsplit & 3))) || p.ktot < 27LL * cin)
      return hipErrorInvalidValue;
  } else if (S.vwrap || p.ysplit || p.rsplit || p.ktot < 9LL * S.C) {
    return hipErrorInvalidValue;
  }
  return v.launch(p, s);
}

}  // namespace pc
