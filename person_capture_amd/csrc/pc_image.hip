// Byte-exact image kernels of the identity hot path (gfx950).
//
// These restate, on device, the u8 image operations the reference performs on
// the CPU through OpenCV 4.9 (opencv-python-headless==4.9.0.80, not vendored):
//   * SCRFD letterbox + blob      [ext] insightface SCRFD.detect / cv2.resize INTER_LINEAR
//                                 / cv2.dnn.blobFromImage(1/128, 127.5, swapRB)
//   * 5-point similarity warp     face_embedder.py:1465-1473 (cv2.warpAffine INTER_LINEAR,
//                                 BORDER_REFLECT on the face-box crop)
//   * face quality                face_embedder.py:1274-1276 (BGR2GRAY + Laplacian(CV_64F).var())
//   * ArcFace preprocessing       face_embedder.py:1281-1298 (BGR->RGB, x/127.5-1, h-flip TTA)
//   * INTER_AREA downscale        gui_app.py:1505-1507 (pre-scan 4K -> 416 wide)
// The fixed-point arithmetic follows OpenCV's published algorithm (11-bit
// resize coefficients, 1/32-pixel warp tables with 15-bit weights, 14-bit gray
// coefficients); oracle/cv_ops.c restates the same arithmetic on the CPU and the
// parity tests require bit-exact agreement. Parity against OpenCV itself is
// unpinned (OpenCV is not installed anywhere in this pipeline).
//
// All of these are HBM/gather-bound: one thread per output pixel, no MFMA.
#include "pc_conv_common.h"

#pragma clang fp contract(off)

namespace pc {

// ---------------------------------------------------------------------------
// SCRFD letterbox: resize (INTER_LINEAR, OpenCV u8 fixed point) into the top-left
// of a zero DxD canvas, then blob (x - 127.5) / 128 with BGR->RGB, NHWC, 4 channels.
// ---------------------------------------------------------------------------
struct LetterboxDesc {
  const uint8_t* src;
  int H, W, row_stride;     // source frame (BGR u8), bytes per row
  int new_w, new_h;         // resized size
  double scale_x, scale_y;  // 1 / (new/old), as cv::resize computes them
  int simd_end;             // byte index where OpenCV's SIMD vertical pass ends (row width*3 based)
  int pad_;
};

__device__ __forceinline__ void lin_coef(int d, double scale, int src_len, int& s0, short& a0, short& a1) {
  float f = (float)((d + 0.5) * scale - 0.5);
  int s = (int)floorf(f);
  f -= (float)s;
  if (s < 0) { f = 0.f; s = 0; }
  if (s >= src_len - 1) { f = 0.f; s = src_len - 1; }
  s0 = s;
  a0 = (short)__float2int_rn((1.f - f) * 2048.f);
  a1 = (short)__float2int_rn(f * 2048.f);
}

template <typename T>
__global__ void letterbox_blob(const LetterboxDesc* __restrict__ descs, int D, T* __restrict__ out) {
  const int n = blockIdx.y;
  const int pix = blockIdx.x * blockDim.x + threadIdx.x;
  if (pix >= D * D) return;
  const LetterboxDesc d = descs[n];
  const int y = pix / D, x = pix - (pix / D) * D;
  float v[3] = {0.f, 0.f, 0.f};  // BGR u8 values
  if (x < d.new_w && y < d.new_h) {
    int sx, sy;
    short a0, a1, b0, b1;
    lin_coef(x, d.scale_x, d.W, sx, a0, a1);
    lin_coef(y, d.scale_y, d.H, sy, b0, b1);
    const int sx1 = sx + 1 < d.W ? sx + 1 : sx;   // weight a1 is 0 whenever clamped
    const int sy1 = sy + 1 < d.H ? sy + 1 : sy;
    const uint8_t* r0 = d.src + (long long)sy * d.row_stride;
    const uint8_t* r1 = d.src + (long long)sy1 * d.row_stride;
#pragma unroll
    for (int c = 0; c < 3; ++c) {
      const int S0 = r0[sx * 3 + c] * a0 + r0[sx1 * 3 + c] * a1;
      const int S1 = r1[sx * 3 + c] * a0 + r1[sx1 * 3 + c] * a1;
      int val;
      if (x * 3 + c < d.simd_end) {  // which rounding OpenCV's vertical pass used for this byte
        const int t0 = ((S0 >> 4) * (int)b0) >> 16;
        const int t1 = ((S1 >> 4) * (int)b1) >> 16;
        val = (t0 + t1 + 2) >> 2;
      } else {
        val = (S0 * (int)b0 + S1 * (int)b1 + (1 << 21)) >> 22;
      }
      val = val < 0 ? 0 : (val > 255 ? 255 : val);
      v[c] = (float)val;
    }
  }
  // blobFromImage: (x - mean) * scalefactor, swapRB -> channel order R,G,B
  T* o = out + ((long long)n * D * D + pix) * 4;
  const float r = (v[2] - 127.5f) * 0.0078125f;
  const float g = (v[1] - 127.5f) * 0.0078125f;
  const float b = (v[0] - 127.5f) * 0.0078125f;
  if constexpr (sizeof(T) == 2) {
    f16x4 h = {(f16)r, (f16)g, (f16)b, (f16)0.f};
    *reinterpret_cast<f16x4*>(o) = h;
  } else {
    *reinterpret_cast<f32x4*>(o) = f32x4{r, g, b, 0.f};
  }
}

// Plain u8 -> u8 INTER_LINEAR resize of a (crop of a) BGR frame, same fixed point
// as the letterbox (TTA rescales face_embedder.py:2264, chip resize fallback :2460).
// area_mode: cv::resize was asked for INTER_AREA but not both axes downscale, so OpenCV
// runs the linear kernel with its "area mode" coefficients (resize.cpp: sx = floor(dx *
// scale), fx = (dx+1) - (sx+1) * inv_scale, wrapped into [0,1)), on both axes.
struct ResizeDesc {
  const uint8_t* src;
  int H, W, row_stride;
  int new_w, new_h;
  double scale_x, scale_y;  // 1 / inv_scale, as hal::resize computes them
  int simd_end;
  int area_mode;
  uint8_t* dst;  // new_h x new_w x 3 contiguous
  double inv_x, inv_y;      // dsize/ssize, or the fx/fy the caller gave
};

__device__ __forceinline__ void lin_coef_area(int d, double scale, double inv, int src_len, int& s0, short& a0,
                                              short& a1) {
  int s = (int)floor(d * scale);
  float f = (float)((d + 1) - (s + 1) * inv);
  f = f <= 0.f ? 0.f : f - (float)(int)floorf(f);
  if (s < 0) { f = 0.f; s = 0; }
  if (s >= src_len - 1) { f = 0.f; s = src_len - 1; }
  s0 = s;
  a0 = (short)__float2int_rn((1.f - f) * 2048.f);
  a1 = (short)__float2int_rn(f * 2048.f);
}

__global__ void resize_linear_u8(const ResizeDesc* __restrict__ descs) {
  const ResizeDesc d = descs[blockIdx.y];
  const int pix = blockIdx.x * blockDim.x + threadIdx.x;
  if (pix >= d.new_w * d.new_h) return;
  const int y = pix / d.new_w, x = pix - (pix / d.new_w) * d.new_w;
  int sx, sy;
  short a0, a1, b0, b1;
  if (d.area_mode) {
    lin_coef_area(x, d.scale_x, d.inv_x, d.W, sx, a0, a1);
    lin_coef_area(y, d.scale_y, d.inv_y, d.H, sy, b0, b1);
  } else {
    lin_coef(x, d.scale_x, d.W, sx, a0, a1);
    lin_coef(y, d.scale_y, d.H, sy, b0, b1);
  }
  const int sx1 = sx + 1 < d.W ? sx + 1 : sx;
  const int sy1 = sy + 1 < d.H ? sy + 1 : sy;
  const uint8_t* r0 = d.src + (long long)sy * d.row_stride;
  const uint8_t* r1 = d.src + (long long)sy1 * d.row_stride;
  uint8_t* o = d.dst + (long long)pix * 3;
#pragma unroll
  for (int c = 0; c < 3; ++c) {
    const int S0 = r0[sx * 3 + c] * a0 + r0[sx1 * 3 + c] * a1;
    const int S1 = r1[sx * 3 + c] * a0 + r1[sx1 * 3 + c] * a1;
    int val;
    if (x * 3 + c < d.simd_end) {
      val = ((((S0 >> 4) * (int)b0) >> 16) + (((S1 >> 4) * (int)b1) >> 16) + 2) >> 2;
    } else {
      val = (S0 * (int)b0 + S1 * (int)b1 + (1 << 21)) >> 22;
    }
    o[c] = (uint8_t)(val < 0 ? 0 : (val > 255 ? 255 : val));
  }
}

// ---------------------------------------------------------------------------
// warpAffine INTER_LINEAR on a crop, u8 BGR, BORDER_REFLECT or BORDER_REFLECT_101.
// M is the dst->src map (already inverted on the host exactly as cv::warpAffine does).
// ---------------------------------------------------------------------------
struct WarpDesc {
  const uint8_t* src;   // top-left of the crop inside the frame
  int row_stride;       // frame bytes per row
  int w, h;             // crop size
  double M[6];          // dst -> src
  uint8_t* dst;         // out_h x out_w x 3, contiguous
  int out_w, out_h;
  int border;           // 2 = BORDER_REFLECT, 4 = BORDER_REFLECT_101, 0 | value << 8 = BORDER_CONSTANT
  int pad_;
};

__device__ __forceinline__ int border_interp(int p, int len, int border) {
  if ((unsigned)p < (unsigned)len) return p;
  if (len == 1) return 0;
  // OpenCV's reflect loop in closed form (the pattern has period 2*len for REFLECT and
  // 2*len-2 for REFLECT_101), so a far-out coordinate costs O(1), not O(|p|/len)
  const int delta = border == 4 ? 1 : 0;
  const long long T = 2LL * len - 2 * delta;
  long long q = (long long)p % T;
  if (q < 0) q += T;
  return (int)(q < len ? q : T - 1 + delta - q);
}

__device__ __forceinline__ void bilinear_wtab(int fx, int fy, int w[4]) {
  // OpenCV initInterTab2D(INTER_LINEAR, fixpt): float products of the 1-D
  // linear taps, rounded to Q15, then the largest/smallest entry absorbs the
  // rounding residue so the four weights sum to exactly 32768.
  const float scale = 1.f / 32.f;
  const float xs = fx * scale, ys = fy * scale;
  const float tx[2] = {1.f - xs, xs};
  const float ty[2] = {1.f - ys, ys};
  int isum = 0;
#pragma unroll
  for (int k1 = 0; k1 < 2; ++k1)
#pragma unroll
    for (int k2 = 0; k2 < 2; ++k2) {
      const float v = ty[k1] * tx[k2];
      w[k1 * 2 + k2] = __float2int_rn(v * 32768.f);
      isum += w[k1 * 2 + k2];
    }
  if (isum != 32768) {
    const int diff = isum - 32768;
    int mk = 0, Mk = 0;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      if (w[k] < w[mk]) mk = k;
      else if (w[k] > w[Mk]) Mk = k;
    }
    if (diff < 0) w[Mk] -= diff;
    else w[mk] -= diff;
  }
}

// grid: one block per 256 output pixels of one chip, 1-D, XCD-remapped so that a chip's blocks
// run on one XCD and its source rows are fetched into one L2 (r04: the (pixel block, chip) grid
// dealt a chip's 49 blocks over all 8 XCDs, and HBM fetch was 5.4x the touched bytes)
__global__ void warp_affine_u8(const WarpDesc* __restrict__ descs, int gx, int nwg) {
  const int tile = xcd_remap(blockIdx.x, nwg);
  const WarpDesc d = descs[tile / gx];
  const int pix = (tile - (tile / gx) * gx) * blockDim.x + threadIdx.x;
  if (pix >= d.out_w * d.out_h) return;
  const int y = pix / d.out_w, x = pix - (pix / d.out_w) * d.out_w;
  const int AB_BITS = 10, AB_SCALE = 1 << AB_BITS, INTER_BITS = 5;
  const int round_delta = AB_SCALE / 32 / 2;
  const int adelta = __double2int_rn(d.M[0] * x * AB_SCALE);
  const int bdelta = __double2int_rn(d.M[3] * x * AB_SCALE);
  const int X0 = __double2int_rn((d.M[1] * y + d.M[2]) * AB_SCALE) + round_delta;
  const int Y0 = __double2int_rn((d.M[4] * y + d.M[5]) * AB_SCALE) + round_delta;
  const int X = (X0 + adelta) >> (AB_BITS - INTER_BITS);
  const int Y = (Y0 + bdelta) >> (AB_BITS - INTER_BITS);
  int sx = X >> INTER_BITS, sy = Y >> INTER_BITS;
  sx = sx < -32768 ? -32768 : (sx > 32767 ? 32767 : sx);
  sy = sy < -32768 ? -32768 : (sy > 32767 ? 32767 : sy);
  int wt[4];
  bilinear_wtab(X & 31, Y & 31, wt);
  uint8_t* o = d.dst + (long long)pix * 3;
  if ((d.border & 0xFF) == 0) {   // BORDER_CONSTANT (value d.border >> 8): taps outside the crop read it
    const int cv = d.border >> 8;
    const bool in00 = (unsigned)sx < (unsigned)d.w && (unsigned)sy < (unsigned)d.h;
    const bool in01 = (unsigned)(sx + 1) < (unsigned)d.w && (unsigned)sy < (unsigned)d.h;
    const bool in10 = (unsigned)sx < (unsigned)d.w && (unsigned)(sy + 1) < (unsigned)d.h;
    const bool in11 = (unsigned)(sx + 1) < (unsigned)d.w && (unsigned)(sy + 1) < (unsigned)d.h;
    const uint8_t* p00 = d.src + (long long)sy * d.row_stride + sx * 3;
#pragma unroll
    for (int c = 0; c < 3; ++c) {
      const int t0 = in00 ? p00[c] : cv, t1 = in01 ? p00[3 + c] : cv;
      const int t2 = in10 ? p00[d.row_stride + c] : cv, t3 = in11 ? p00[d.row_stride + 3 + c] : cv;
      const int v = (t0 * wt[0] + t1 * wt[1] + t2 * wt[2] + t3 * wt[3] + (1 << 14)) >> 15;
      o[c] = (uint8_t)(v < 0 ? 0 : (v > 255 ? 255 : v));
    }
    return;
  }
  const int x0 = border_interp(sx, d.w, d.border), x1 = border_interp(sx + 1, d.w, d.border);
  const int y0 = border_interp(sy, d.h, d.border), y1 = border_interp(sy + 1, d.h, d.border);
  const uint8_t* r0 = d.src + (long long)y0 * d.row_stride;
  const uint8_t* r1 = d.src + (long long)y1 * d.row_stride;
#pragma unroll
  for (int c = 0; c < 3; ++c) {
    int v = r0[x0 * 3 + c] * wt[0] + r0[x1 * 3 + c] * wt[1] + r1[x0 * 3 + c] * wt[2] + r1[x1 * 3 + c] * wt[3];
    v = (v + (1 << 14)) >> 15;
    o[c] = (uint8_t)(v < 0 ? 0 : (v > 255 ? 255 : v));
  }
}

// ---------------------------------------------------------------------------
// quality = var(Laplacian(BGR2GRAY(chip), CV_64F)), ksize=1, BORDER_REFLECT_101.
// The Laplacian values are small integers, so sum and sum of squares are exact in
// int64; var = (S2 - S1^2/N)/N in f64 (numpy's two-pass var agrees to ~1e-15).
// One 1024-thread workgroup per chip: the chip's bytes come in as 16-byte loads (a per-frame
// extract() has ~6 chips, so the old 256-thread byte-load loop ran ~40 us on 6 CUs), the gray
// image and the Laplacian sums come from the LDS.
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(1024) void face_quality(const uint8_t* __restrict__ chips, int side, double* __restrict__ out) {
  __shared__ __attribute__((aligned(16))) uint8_t raw[128 * 128 * 3];
  __shared__ uint8_t g[128 * 128];
  __shared__ long long red[2][16];
  const uint8_t* c = chips + (long long)blockIdx.x * side * side * 3;
  const int n = side * side;
  const int nb = n * 3;
  if ((nb & 15) == 0 && ((uintptr_t)c & 15) == 0) {
    for (int i = threadIdx.x; i < nb / 16; i += blockDim.x)
      reinterpret_cast<uint4*>(raw)[i] = reinterpret_cast<const uint4*>(c)[i];
  } else {
    for (int i = threadIdx.x; i < nb; i += blockDim.x) raw[i] = c[i];
  }
  __syncthreads();
  for (int i = threadIdx.x; i < n; i += blockDim.x) {
    const int b = raw[i * 3 + 0], gg = raw[i * 3 + 1], r = raw[i * 3 + 2];
    g[i] = (uint8_t)((b * 1868 + gg * 9617 + r * 4899 + (1 << 13)) >> 14);
  }
  __syncthreads();
  long long s1 = 0, s2 = 0;
  for (int i = threadIdx.x; i < n; i += blockDim.x) {
    const int y = i / side, x = i - (i / side) * side;
    const int xm = border_interp(x - 1, side, 4), xp = border_interp(x + 1, side, 4);
    const int ym = border_interp(y - 1, side, 4), yp = border_interp(y + 1, side, 4);
    const int l = (int)g[y * side + xm] + (int)g[y * side + xp] + (int)g[ym * side + x] + (int)g[yp * side + x] - 4 * (int)g[i];
    s1 += l;
    s2 += (long long)l * l;
  }
  for (int o = 32; o > 0; o >>= 1) {
    s1 += __shfl_xor(s1, o);
    s2 += __shfl_xor(s2, o);
  }
  const int wv = threadIdx.x >> 6;
  if ((threadIdx.x & 63) == 0) { red[0][wv] = s1; red[1][wv] = s2; }
  __syncthreads();
  if (threadIdx.x == 0) {
    long long t1 = 0, t2 = 0;
    for (int k = 0; k < (int)(blockDim.x >> 6); ++k) { t1 += red[0][k]; t2 += red[1][k]; }
    const double N = (double)n;
    const double mean = (double)t1 / N;
    // sum (l - mean)^2 = S2 - 2*mean*S1 + N*mean^2 = S2 - S1*mean (exact algebra)
    out[blockIdx.x] = ((double)t2 - (double)t1 * mean) / N;
  }
}

// ---------------------------------------------------------------------------
// ArcFace input: BGR u8 chip -> RGB, x/127.5 - 1 (f32 division as numpy does),
// NHWC with 4 channels; optionally the horizontally flipped copy at n + N.
// ---------------------------------------------------------------------------
// CENTRED: x - 127.5 instead (exact in f16), the f16x3 IResNet's input (1/127.5 in its stem).
template <typename T, bool CENTRED = false>
__global__ void arcface_prep(const uint8_t* __restrict__ chips, int N, int side, int flip, T* __restrict__ out) {
  const int n = blockIdx.y;
  const int pix = blockIdx.x * blockDim.x + threadIdx.x;
  if (pix >= side * side) return;
  const int y = pix / side, x = pix - (pix / side) * side;
  const uint8_t* s = chips + ((long long)n * side * side + pix) * 3;
  const float r = CENTRED ? (float)s[2] - 127.5f : (float)s[2] / 127.5f - 1.0f;
  const float g = CENTRED ? (float)s[1] - 127.5f : (float)s[1] / 127.5f - 1.0f;
  const float b = CENTRED ? (float)s[0] - 127.5f : (float)s[0] / 127.5f - 1.0f;
  T* o = out + ((long long)n * side * side + pix) * 4;
  T* of = out + ((long long)(n + N) * side * side + y * side + (side - 1 - x)) * 4;
  if constexpr (sizeof(T) == 2) {
    f16x4 h = {(f16)r, (f16)g, (f16)b, (f16)0.f};
    *reinterpret_cast<f16x4*>(o) = h;
    if (flip) *reinterpret_cast<f16x4*>(of) = h;
  } else {
    const f32x4 h{r, g, b, 0.f};
    *reinterpret_cast<f32x4*>(o) = h;
    if (flip) *reinterpret_cast<f32x4*>(of) = h;
  }
}

// ---------------------------------------------------------------------------
// Rotation by 90/180/270 (cv2.rotate semantics) and replicate padding
// (cv2.copyMakeBorder BORDER_REPLICATE) for SCRFD fallback passes
// (face_embedder.py:2165-2169, 2292-2294, 2394).
// ---------------------------------------------------------------------------
__global__ void rotate_pad_u8(const uint8_t* __restrict__ src, int H, int W, int row_stride, int deg, int pad,
                              uint8_t* __restrict__ dst, int OH, int OW) {
  const long long pix = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (pix >= (long long)OH * OW) return;
  const int y = (int)(pix / OW), x = (int)(pix - (pix / OW) * OW);
  // coordinates in the rotated (unpadded) image, replicate-clamped
  const int RH = (deg == 90 || deg == 270) ? W : H;
  const int RW = (deg == 90 || deg == 270) ? H : W;
  int ry = y - pad, rx = x - pad;
  ry = ry < 0 ? 0 : (ry >= RH ? RH - 1 : ry);
  rx = rx < 0 ? 0 : (rx >= RW ? RW - 1 : rx);
  int sy, sx;
  if (deg == 90) { sy = H - 1 - rx; sx = ry; }          // ROTATE_90_CLOCKWISE
  else if (deg == 180) { sy = H - 1 - ry; sx = W - 1 - rx; }
  else if (deg == 270) { sy = rx; sx = W - 1 - ry; }    // ROTATE_90_COUNTERCLOCKWISE
  else { sy = ry; sx = rx; }
  const uint8_t* s = src + (long long)sy * row_stride + sx * 3;
  uint8_t* o = dst + pix * 3;
  o[0] = s[0]; o[1] = s[1]; o[2] = s[2];
}

// ---------------------------------------------------------------------------
// cv2.resize INTER_AREA for downscales (u8, 3 channels), OpenCV's generic
// (non-integer scale) area path: float weights, accumulated per output pixel in
// source order, saturate_cast<uchar> (round half to even) at the end.
// Coefficient tables (xofs: src index, dst index, weight) are built on the host
// exactly as cv::computeResizeAreaTab does and passed in.
// ---------------------------------------------------------------------------
struct AreaTab { int si; int di; float alpha; };

__global__ void resize_area_u8(const uint8_t* __restrict__ src, int row_stride,
                               const AreaTab* __restrict__ xtab, const int* __restrict__ xtab_start,
                               const AreaTab* __restrict__ ytab, const int* __restrict__ ytab_start,
                               uint8_t* __restrict__ dst, int OH, int OW) {
  const int pix = blockIdx.x * blockDim.x + threadIdx.x;
  if (pix >= OH * OW) return;
  const int dy = pix / OW, dx = pix - (pix / OW) * OW;
  float acc[3] = {0.f, 0.f, 0.f};
  for (int j = ytab_start[dy]; j < ytab_start[dy + 1]; ++j) {
    const AreaTab ty = ytab[j];
    const uint8_t* row = src + (long long)ty.si * row_stride;
    float rs[3] = {0.f, 0.f, 0.f};
    for (int i = xtab_start[dx]; i < xtab_start[dx + 1]; ++i) {
      const AreaTab tx = xtab[i];
#pragma unroll
      for (int c = 0; c < 3; ++c) rs[c] += (float)row[tx.si * 3 + c] * tx.alpha;
    }
#pragma unroll
    for (int c = 0; c < 3; ++c) acc[c] += rs[c] * ty.alpha;
  }
  uint8_t* o = dst + (long long)pix * 3;
#pragma unroll
  for (int c = 0; c < 3; ++c) {
    int v = __float2int_rn(acc[c]);
    o[c] = (uint8_t)(v < 0 ? 0 : (v > 255 ? 255 : v));
  }
}

// The same arithmetic for a batch of equally sized frames (the pre-scan's 4K -> 416 downscale of a
// speculative chunk, gui_app.py:1505-1507), with the source rows staged through the LDS: a workgroup
// is 256 consecutive output pixels of one output row of one frame; the source rows of the row's
// y-window stream through a 4-slot LDS ring by LDS-DMA (each row's byte span from a 16-byte boundary,
// three rows in flight while one is summed), and every thread sums its x-window from there - the per-pixel form issued ~300 byte loads per thread
// straight from memory and ran one 4K frame per launch at 0.03 of HBM. Requires
// 16-byte aligned sources and row strides (every source byte the loads touch is then inside the
// rows); the per-pixel kernel serves the rest. Bit-identical to it: same products, same order.
struct AreaJob { const uint8_t* src; uint8_t* dst; };

// LDS ring of the row kernel: AREA_RING row buffers of AREA_ROWB bytes, AREA_RING - 1 rows in flight
constexpr int AREA_RING = 4, AREA_ROWB = 8192, AREA_PPW = AREA_ROWB / 1024 / 4;   // pieces per wave and row

__global__ __launch_bounds__(256) void resize_area_rows_u8(const AreaJob* __restrict__ jobs, int row_stride,
                                                           const AreaTab* __restrict__ xtab,
                                                           const int* __restrict__ xtab_start,
                                                           const AreaTab* __restrict__ ytab,
                                                           const int* __restrict__ ytab_start, int OH, int OW) {
  __shared__ __attribute__((aligned(16))) uint8_t ring[AREA_RING * AREA_ROWB];
  const AreaJob job = jobs[blockIdx.z];
  const int dy = blockIdx.y, x0 = blockIdx.x * 256;
  const int dx = x0 + threadIdx.x;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int xl = min(x0 + 255, OW - 1);
  // the pixel's x-window bounds, loaded with the span's (before the DMAs: a wait on a later load would
  // wait for them too)
  const bool live = dx < OW;
  int i0 = live ? xtab_start[dx] : 0, i1 = live ? xtab_start[dx + 1] : 0;
  // the workgroup's source byte span, from a 16-byte boundary (<= AREA_ROWB: checked on the host)
  const int c0 = xtab[xtab_start[x0]].si, c1 = xtab[xtab_start[xl + 1] - 1].si;
  const int b0 = (c0 * 3) & ~15, b1 = (c1 * 3 + 3 + 15) & ~15;
  const int j0 = ytab_start[dy], j1 = ytab_start[dy + 1];
  asm volatile("" : "+v"(i0), "+v"(i1));
  // LDS-DMA of source row j into ring slot: piece q = wave + 4 i covers LDS bytes q KiB + 16 lane; a lane
  // past the span re-reads the span's first chunk (every address it touches is inside the row)
  const __amdgpu_buffer_rsrc_t rs =
      __builtin_amdgcn_make_buffer_rsrc(const_cast<uint8_t*>(job.src), (short)0, (int)0xffffffff, 0x00020000);
  unsigned lofs[AREA_PPW];
#pragma unroll
  for (int i = 0; i < AREA_PPW; ++i) {
    const int byte = (wave + 4 * i) * 1024 + lane * 16;
    lofs[i] = (unsigned)(b0 + (byte < b1 - b0 ? byte : 0));
  }
  auto issue = [&](int j, auto slotc) __attribute__((always_inline)) {
    constexpr int slot = decltype(slotc)::value;
    const unsigned rbase = (unsigned)ytab[j].si * (unsigned)row_stride;
#pragma unroll
    for (int i = 0; i < AREA_PPW; ++i) {
      unsigned off = lofs[i];
      asm volatile("" : "+v"(off));
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, (lds_ptr_t)(ring + slot * AREA_ROWB + (wave + 4 * i) * 1024), 16,
                                               off, rbase, 0, 0);
    }
  };
  // prologue: rows j0 .. j0 + RING - 2 in flight, issued before the x-window loads so both latencies
  // overlap (past the window: row j0 again into its slot's successor, so every wave always has the
  // same number of DMAs younger than the row it waits for)
  static_for<AREA_RING - 1>([&](auto rc) __attribute__((always_inline)) {
    constexpr int r = decltype(rc)::value;
    issue(j0 + r < j1 ? j0 + r : j0, rc);
  });
  // the pixel's x-window in registers (<= MAXT taps: scale < MAXT - 1; wider windows re-read the table)
  constexpr int MAXT = 16;
  const int nt = i1 - i0;
  int xo[MAXT];
  float xa[MAXT];
  // (every entry loaded unconditionally - an in-window index or the window's first - so the 16 loads go
  // out together: guarded loads were issued one round trip after another)
  int tsi[MAXT];
  float tal[MAXT];
#pragma unroll
  for (int t = 0; t < MAXT; ++t) {
    const AreaTab tx = xtab[t < nt ? i0 + t : i0];
    tsi[t] = tx.si;
    tal[t] = tx.alpha;
  }
#pragma unroll
  for (int t = 0; t < MAXT; ++t) asm volatile("" : "+v"(tsi[t]), "+v"(tal[t]));   // (no sinking into branches)
#pragma unroll
  for (int t = 0; t < MAXT; ++t) {
    xo[t] = t < nt ? tsi[t] * 3 - b0 : 0;
    xa[t] = t < nt ? tal[t] : 0.f;
  }
  float acc[3] = {0.f, 0.f, 0.f};
  // one source row per step, unrolled by the ring depth so every ring slot is a compile-time offset: with
  // a run-time slot the compiler cannot tell which LDS-DMA a row read depends on and waited vmcnt(0) at
  // every step (one row in flight instead of RING - 1)
  auto step = [&](int j, auto slotc) __attribute__((always_inline)) {
    constexpr int slot = decltype(slotc)::value;
    // row j landed: the youngest (RING - 2) rows' DMAs may still be in flight
    asm volatile("s_waitcnt vmcnt(%0)" ::"n"((AREA_RING - 2) * AREA_PPW) : "memory");
    __builtin_amdgcn_s_barrier();   // every wave's pieces of row j; every thread done with row j - 1's slot
    const int jn = j + AREA_RING - 1;
    issue(jn < j1 ? jn : j0, std::integral_constant<int, (slot + AREA_RING - 1) % AREA_RING>{});
    const uint8_t* row = ring + slot * AREA_ROWB;
    const AreaTab ty = ytab[j];
    float rsum[3] = {0.f, 0.f, 0.f};
    if (nt <= MAXT) {
#pragma unroll
      for (int t = 0; t < MAXT; ++t) {
        if (t < nt) {
#pragma unroll
          for (int c = 0; c < 3; ++c) rsum[c] += (float)row[xo[t] + c] * xa[t];
        }
      }
    } else {
      for (int i = i0; i < i1; ++i) {
        const AreaTab tx = xtab[i];
#pragma unroll
        for (int c = 0; c < 3; ++c) rsum[c] += (float)row[tx.si * 3 - b0 + c] * tx.alpha;
      }
    }
#pragma unroll
    for (int c = 0; c < 3; ++c) acc[c] += rsum[c] * ty.alpha;
  };
  for (int j = j0; j < j1; j += AREA_RING) {
    static_for<AREA_RING>([&](auto rc) __attribute__((always_inline)) {
      if (j + decltype(rc)::value < j1) step(j + decltype(rc)::value, rc);
    });
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // (the dummy tail DMAs, before the workgroup's LDS goes)
  if (!live) return;
  uint8_t* o = job.dst + ((long long)dy * OW + dx) * 3;
#pragma unroll
  for (int c = 0; c < 3; ++c) {
    int v = __float2int_rn(acc[c]);
    o[c] = (uint8_t)(v < 0 ? 0 : (v > 255 ? 255 : v));
  }
}

// cv2.resize INTER_AREA at an exact integer ratio (hal::resize "is_area_fast"):
// resizeAreaFast_Invoker. 2x2 takes ResizeAreaFastVec ((sum + 2) >> 2 for every byte);
// other ratios saturate_cast<uchar>(sum * (1.f / area)) (round half to even).
__global__ void resize_area_fast_u8(const uint8_t* __restrict__ src, int row_stride, int isx, int isy,
                                    uint8_t* __restrict__ dst, int OH, int OW) {
  const int pix = blockIdx.x * blockDim.x + threadIdx.x;
  if (pix >= OH * OW) return;
  const int dy = pix / OW, dx = pix - (pix / OW) * OW;
  const float scale = 1.f / (float)(isx * isy);
  uint8_t* o = dst + (long long)pix * 3;
#pragma unroll
  for (int c = 0; c < 3; ++c) {
    int sum = 0;
    for (int j = 0; j < isy; ++j) {
      const uint8_t* row = src + (long long)(dy * isy + j) * row_stride + (dx * isx) * 3 + c;
      for (int i = 0; i < isx; ++i) sum += row[i * 3];
    }
    int v = (isx == 2 && isy == 2) ? ((sum + 2) >> 2) : __float2int_rn((float)sum * scale);
    o[c] = (uint8_t)(v < 0 ? 0 : (v > 255 ? 255 : v));
  }
}

// ---------------------------------------------------------------------------
hipError_t resize_area_fast_launch(const uint8_t* src, int row_stride, int isx, int isy, uint8_t* dst, int OH, int OW,
                                   hipStream_t s) {
  hipLaunchKernelGGL(resize_area_fast_u8, dim3((OH * OW + 255) / 256), dim3(256), 0, s, src, row_stride, isx, isy,
                     dst, OH, OW);
  return hipGetLastError();
}

hipError_t letterbox_launch(int f32, const LetterboxDesc* d_descs, int N, int D, void* out, hipStream_t s) {
  dim3 grid((D * D + 255) / 256, N);
  if (f32) hipLaunchKernelGGL(letterbox_blob<float>, grid, dim3(256), 0, s, d_descs, D, (float*)out);
  else hipLaunchKernelGGL(letterbox_blob<f16>, grid, dim3(256), 0, s, d_descs, D, (f16*)out);
  return hipGetLastError();
}

hipError_t resize_linear_launch(const ResizeDesc* d_descs, int N, int max_pixels, hipStream_t s) {
  dim3 grid((max_pixels + 255) / 256, N);
  hipLaunchKernelGGL(resize_linear_u8, grid, dim3(256), 0, s, d_descs);
  return hipGetLastError();
}

hipError_t warp_launch(const WarpDesc* d_descs, int N, int max_pixels, hipStream_t s) {
  const int gx = (max_pixels + 255) / 256;
  const long long nwg = (long long)gx * N;
  if (nwg <= 0 || nwg >= (1LL << 31)) return hipErrorInvalidValue;
  hipLaunchKernelGGL(warp_affine_u8, dim3((unsigned)nwg), dim3(256), 0, s, d_descs, gx, (int)nwg);
  return hipGetLastError();
}

hipError_t quality_launch(const uint8_t* chips, int N, int side, double* out, hipStream_t s) {
  if (side > 128) return hipErrorInvalidValue;
  hipLaunchKernelGGL(face_quality, dim3(N), dim3(1024), 0, s, chips, side, out);
  return hipGetLastError();
}

// mode: 0 f16 x/127.5 - 1, 1 f32 x/127.5 - 1, 2 f16 x - 127.5 (pcgpu.h PC_PREC_*)
hipError_t arcprep_launch(int mode, const uint8_t* chips, int N, int side, int flip, void* out, hipStream_t s) {
  dim3 grid((side * side + 255) / 256, N);
  if (mode == 2) hipLaunchKernelGGL((arcface_prep<f16, true>), grid, dim3(256), 0, s, chips, N, side, flip, (f16*)out);
  else if (mode == 1) hipLaunchKernelGGL(arcface_prep<float>, grid, dim3(256), 0, s, chips, N, side, flip, (float*)out);
  else hipLaunchKernelGGL(arcface_prep<f16>, grid, dim3(256), 0, s, chips, N, side, flip, (f16*)out);
  return hipGetLastError();
}

hipError_t rotate_pad_launch(const uint8_t* src, int H, int W, int row_stride, int deg, int pad, uint8_t* dst,
                             int OH, int OW, hipStream_t s) {
  const long long n = (long long)OH * OW;
  hipLaunchKernelGGL(rotate_pad_u8, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, src, H, W, row_stride, deg,
                     pad, dst, OH, OW);
  return hipGetLastError();
}

hipError_t resize_area_rows_launch(const void* jobs, int n, int row_stride, const AreaTab* xtab, const int* xstart,
                                  const AreaTab* ytab, const int* ystart, int OH, int OW, int span_bytes,
                                  hipStream_t s) {
  if (n <= 0 || span_bytes <= 0 || span_bytes > AREA_ROWB) return hipErrorInvalidValue;
  hipLaunchKernelGGL(resize_area_rows_u8, dim3((OW + 255) / 256, OH, n), dim3(256), 0, s, (const AreaJob*)jobs,
                     row_stride, xtab, xstart, ytab, ystart, OH, OW);
  return hipGetLastError();
}

hipError_t resize_area_launch(const uint8_t* src, int row_stride, const AreaTab* xtab, const int* xstart,
                              const AreaTab* ytab, const int* ystart, uint8_t* dst, int OH, int OW, hipStream_t s) {
  hipLaunchKernelGGL(resize_area_u8, dim3((OH * OW + 255) / 256), dim3(256), 0, s, src, row_stride, xtab, xstart, ytab,
                     ystart, dst, OH, OW);
  return hipGetLastError();
}

}  // namespace pc
