// Internal types shared by the gfx950 kernels and the C-ABI layer.
// Everything here is device-agnostic plain data; the kernels live in pc_*.hip.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace pc {

typedef _Float16 f16;
typedef f16 f16x8 __attribute__((ext_vector_type(8)));
typedef f16 f16x4 __attribute__((ext_vector_type(4)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef int i32x4 __attribute__((ext_vector_type(4)));
typedef int i32x8 __attribute__((ext_vector_type(8)));
typedef __attribute__((address_space(3))) void* lds_ptr_t;
typedef __attribute__((address_space(1))) void* gptr_t;

enum Act { ACT_NONE = 0, ACT_RELU = 1, ACT_PRELU = 2, ACT_SILU = 3, ACT_GELU = 4 };
enum BiasMode { BIAS_NONE = 0, BIAS_CHANNEL = 1, BIAS_BORDER9 = 2 };
enum ResMode { RES_NONE = 0, RES_SAME = 1, RES_UP2 = 2 };

// One K-segment of an implicit-GEMM convolution: a KHxKW window over an NHWC
// tensor whose (padded) channel count C is a multiple of the K-tile width.
struct ConvSeg {
  const void* x;       // NHWC activations, pixel stride `cs` elements
  int H, W, C, cs;     // input dims, padded channels, pixel stride
  int KH, KW, stride, pad;
  int kt;              // K tiles in this segment = KH*KW*(C/BKE)
  int cblk;            // C / BKE
  unsigned zero_off;   // bytes from x to >= 256 zero bytes (padding taps read there)
  // f16x3 split tensors (x = hi + lo, stored [hi | lo] per pixel): the K loop walks the
  // virtual channel blocks [hi, lo, hi] against weights [W_hi, W_hi, W_lo] of each tap, so
  // x_hi*W_hi + x_lo*W_hi + x_hi*W_lo accumulate in f32. cblk counts the
  // virtual blocks; a virtual block >= vwrap reads physical block (block - vwrap). 0: plain.
  int vwrap;
  // f16c8 tensors: the second half of a pixel holds, per 32-channel block, the
  // e4m3 bytes [lo8 x 32 | hi8 x 32]; f8s = E8M0 exponents of their scales, lo | hi << 8
  // (true lo = lo8 * 2^(e_lo - 127))
  int f8s;
  // fused split tiles (conv_fast SX): K tiles per channel group. The K loop walks channel groups of
  // 64 hi channels (32 where the channels are not a multiple of 64): every tap of a group, then the
  // next group - the same accumulation order at 64- and 128-byte K rows (gt 2 or 1 tiles per group
  // and tap), so every plan class of a conv may pick its own row width
  int gt;
};

struct ConvParams {
  ConvSeg seg[2];
  int nseg;
  const void* w;       // [npad][ktot] weights, BN/scale already folded
  long long ktot;      // weight row stride in elements
  int N, OH, OW, M;    // output batch/dims, M = N*OH*OW pixels
  int npad;            // padded output channels (multiple of the channel tile)
  int cout;            // valid output channels
  int cwrite;          // channels written (>= cout; lanes in [cout, cwrite) are stored as 0)
  void* y;             // output NHWC base (channel offset already applied)
  int ycs;             // output pixel stride (elements)
  int out_f32;         // 1: write float, 0: write activation dtype
  const float* bias;   // BIAS_CHANNEL: [npad]; BIAS_BORDER9: [9][npad]
  int bias_mode;
  const float* slope;  // PReLU slopes [npad]
  int act;
  const void* res;     // residual NHWC (activation dtype)
  int rcs, res_mode, rH, rW;
  int act_after_res;   // 1: y = act(acc + b + res); 0: y = act(acc + b) + res
  float* partial;      // split-K partials [splitk][M][npad]
  int splitk;
  int kt_total;
  const void* zero;    // >= 256 zero bytes (padding taps read from here)
  int dbg;             // tuning experiments only (PC_CONV_DBG): 1 no staging, 2 no MFMA, 4 one-image footprint
  // f16x3 split output / residual: the lo half sits this many elements after the hi half
  // of each pixel (0: plain tensor). Output: hi = f16(v), lo = f16(v - hi); residual: hi + lo.
  int ysplit;
  int rsplit;
  // f16x3 fused split tiles (conv_fast SX): a K tile is one (tap, hi channel block) staged with
  // its lo block and both weight halves; seg cblk counts hi blocks, vwrap is the lo block offset
  int sx;
  // f16c8 convs (conv_fast C8): the K tile's f16 halves give x_hi*W_hi; the f8 rows
  // ([lo8 | hi8] against [W_hi8 | W_lo8]) give x_lo*W_hi + x_hi*W_lo in one block-scaled e4m3 MFMA.
  // wf8s: E8M0 exponents of the weight bytes' scales, W_hi8 | W_lo8 << 8.
  int c8;
  int wf8s;
  // f16c8 output / residual (ysplit / rsplit locate the f8 region): y: lo8 = e4m3(lo * ylo_mul),
  // hi8 = e4m3(hi * yhi_mul); residual: hi + lo8 * rlo_inv
  int yc8, rc8;
  float ylo_mul, yhi_mul, rlo_inv;
  // fused f16x3 tiles, WG form (conv_fast) and the halo-staged kernel: the weights in fragment
  // order, per 32-channel K tile (the SX channel-group order at 64-byte rows) x 16-row block x
  // [W_hi, W_lo] x 64 lanes x 8 f16 (lane l: row l & 15, channels 8 (l >> 4) .. +8 of the tile's 32);
  // null: the weights are staged from w
  const void* wfrag;
};

// Direct convolution for tiny input channel counts (network stems, Cin <= 4).
struct StemParams {
  const void* x;       // NHWC, pixel stride xcs
  int N, H, W, cin, xcs;
  int OH, OW, KH, KW, stride, pad;
  const float* w;      // [cout][KH][KW][cin] (folded)
  const float* bias;   // [cout]
  const float* slope;  // [cout] or null
  int act;
  int cout, ycs;       // valid output channels, output pixel stride
  void* y;
  int cpad;            // channels written (>= cout, the tail is zero-filled)
  int ysplit;          // f16x3 split output: lo half at +ysplit elements (0: plain)
  int yc8;             // f16c8 output: the f8 region at +ysplit elements (ConvParams)
  float ylo_mul, yhi_mul;
};

struct PoolParams {
  const void* x; int N, H, W, C, xcs;
  void* y; int OH, OW, ycs;
  int k, stride, pad;
  int split;           // f16x3 split tensors: C is the hi half, the lo half follows at +C
};

}  // namespace pc
