/*
 * cv_ops.c — CPU restatement of the OpenCV 4.9 u8 image arithmetic used on the
 * person_capture identity hot path. TEST INFRASTRUCTURE ONLY (oracle/).
 *
 * OpenCV (opencv-python-headless==4.9.0.80, reference requirements.txt:9) is not
 * vendored in the reference and not installed here, so this file restates the
 * published algorithms; agreement with OpenCV itself is "parity unpinned".
 * The GPU kernels in person_capture_amd/csrc/pc_image.hip must agree with this
 * file bit-for-bit (tests/test_gpu_image.py).
 *
 *  - cv_resize_linear_u8: cv::resize INTER_LINEAR for CV_8UC3 (resizeGeneric_ with
 *    HResizeLinear / VResizeLinear): 11-bit coefficients from float fx, horizontal
 *    int sums, vertical pass ((S0>>4)*b0>>16 + (S1>>4)*b1>>16 + 2)>>2 where the
 *    128-bit SIMD loop runs and (S0*b0 + S1*b1 + 2^21)>>22 for the scalar tail.
 *    Used by insightface SCRFD.detect (face_embedder.py:2185).
 *  - cv_warp_affine_u8: cv::warpAffine INTER_LINEAR (AB_BITS=10, INTER_BITS=5,
 *    Q15 bilinear table with sum correction), BORDER_REFLECT / REFLECT_101
 *    (face_embedder.py:1473).
 *  - cv_invert_affine: the 2x3 inversion cv::warpAffine applies without WARP_INVERSE_MAP.
 *  - cv_area_tab / cv_resize_area_u8: cv::resize INTER_AREA generic path
 *    (computeResizeAreaTab + ResizeArea_Invoker, float accumulation) (gui_app.py:1505-1507).
 *
 * Build: oracle/Makefile (gcc -O2 -ffp-contract=off).
 */
#include <math.h>
#include <stdint.h>
#include <string.h>
#include <stdlib.h>

static int clampi(int v, int lo, int hi) { return v < lo ? lo : (v > hi ? hi : v); }

/* cvRound(float) / cvRound(double): round half to even (default FP environment) */
static int round_f(float v) { return (int)lrintf(v); }
static int round_d(double v) { return (int)lrint(v); }

/* resize.cpp coefficient loop (ksize 2). area_mode: INTER_AREA requested but not both axes
 * downscale -> sx = cvFloor(dx*scale), fx = (float)((dx+1) - (sx+1)*inv_scale) wrapped to [0,1). */
static void linear_coefs2(int dsize, int ssize, double scale, double inv_scale, int area_mode, int* ofs, short* c0,
                          short* c1) {
  for (int d = 0; d < dsize; ++d) {
    float f;
    int s;
    if (!area_mode) {
      f = (float)((d + 0.5) * scale - 0.5);
      s = (int)floorf(f);
      f -= (float)s;
    } else {
      s = (int)floor(d * scale);
      f = (float)((d + 1) - (s + 1) * inv_scale);
      f = f <= 0 ? 0.f : f - (float)(int)floorf(f);
    }
    if (s < 0) { f = 0.f; s = 0; }
    if (s >= ssize - 1) { f = 0.f; s = ssize - 1; }
    ofs[d] = s;
    c0[d] = (short)round_f((1.f - f) * 2048.f);
    c1[d] = (short)round_f(f * 2048.f);
  }
}

static void linear_coefs(int dsize, int ssize, double scale, int* ofs, short* c0, short* c1) {
  linear_coefs2(dsize, ssize, scale, 0.0, 0, ofs, c0, c1);
}

/* dst: new_h x new_w x 3 contiguous */
void cv_resize_linear2_u8(const uint8_t* src, int H, int W, int row_stride, uint8_t* dst, int new_w, int new_h,
                          double scale_x, double scale_y, double inv_x, double inv_y, int area_mode, int simd_end);
void cv_resize_linear_u8(const uint8_t* src, int H, int W, int row_stride, uint8_t* dst, int new_w, int new_h,
                         double scale_x, double scale_y, int simd_end) {
  cv_resize_linear2_u8(src, H, W, row_stride, dst, new_w, new_h, scale_x, scale_y, 0.0, 0.0, 0, simd_end);
}

void cv_resize_linear2_u8(const uint8_t* src, int H, int W, int row_stride, uint8_t* dst, int new_w, int new_h,
                          double scale_x, double scale_y, double inv_x, double inv_y, int area_mode, int simd_end) {
  int* xo = (int*)malloc(sizeof(int) * new_w);
  short* a0 = (short*)malloc(sizeof(short) * new_w);
  short* a1 = (short*)malloc(sizeof(short) * new_w);
  int* yo = (int*)malloc(sizeof(int) * new_h);
  short* b0 = (short*)malloc(sizeof(short) * new_h);
  short* b1 = (short*)malloc(sizeof(short) * new_h);
  int* S0 = (int*)malloc(sizeof(int) * new_w * 3);
  int* S1 = (int*)malloc(sizeof(int) * new_w * 3);
  linear_coefs2(new_w, W, scale_x, inv_x, area_mode, xo, a0, a1);
  linear_coefs2(new_h, H, scale_y, inv_y, area_mode, yo, b0, b1);
  for (int dy = 0; dy < new_h; ++dy) {
    const int sy0 = yo[dy];
    const int sy1 = sy0 + 1 < H ? sy0 + 1 : H - 1;
    const uint8_t* r0 = src + (size_t)sy0 * row_stride;
    const uint8_t* r1 = src + (size_t)sy1 * row_stride;
    for (int dx = 0; dx < new_w; ++dx) {
      const int sx0 = xo[dx];
      const int sx1 = sx0 + 1 < W ? sx0 + 1 : sx0;
      for (int c = 0; c < 3; ++c) {
        S0[dx * 3 + c] = r0[sx0 * 3 + c] * a0[dx] + r0[sx1 * 3 + c] * a1[dx];
        S1[dx * 3 + c] = r1[sx0 * 3 + c] * a0[dx] + r1[sx1 * 3 + c] * a1[dx];
      }
    }
    uint8_t* o = dst + (size_t)dy * new_w * 3;
    for (int x = 0; x < new_w * 3; ++x) {
      int v;
      if (x < simd_end) {
        const int t0 = ((S0[x] >> 4) * (int)b0[dy]) >> 16;
        const int t1 = ((S1[x] >> 4) * (int)b1[dy]) >> 16;
        v = (t0 + t1 + 2) >> 2;
      } else {
        v = (S0[x] * (int)b0[dy] + S1[x] * (int)b1[dy] + (1 << 21)) >> 22;
      }
      o[x] = (uint8_t)clampi(v, 0, 255);
    }
  }
  free(xo); free(a0); free(a1); free(yo); free(b0); free(b1); free(S0); free(S1);
}

/* letterbox + blobFromImage(1/128, mean 127.5, swapRB) -> float NHWC4 (D x D x 4) */
void cv_letterbox_blob(const uint8_t* src, int H, int W, int row_stride, int D, int new_w, int new_h, double scale_x,
                       double scale_y, int simd_end, float* out) {
  uint8_t* r = (uint8_t*)malloc((size_t)new_w * new_h * 3);
  cv_resize_linear_u8(src, H, W, row_stride, r, new_w, new_h, scale_x, scale_y, simd_end);
  for (int y = 0; y < D; ++y)
    for (int x = 0; x < D; ++x) {
      float bgr[3] = {0.f, 0.f, 0.f};
      if (x < new_w && y < new_h)
        for (int c = 0; c < 3; ++c) bgr[c] = (float)r[((size_t)y * new_w + x) * 3 + c];
      float* o = out + ((size_t)y * D + x) * 4;
      o[0] = (bgr[2] - 127.5f) * 0.0078125f;
      o[1] = (bgr[1] - 127.5f) * 0.0078125f;
      o[2] = (bgr[0] - 127.5f) * 0.0078125f;
      o[3] = 0.f;
    }
  free(r);
}

void cv_invert_affine(const double* M, double* iM) {
  double D = M[0] * M[4] - M[1] * M[3];
  D = D != 0 ? 1. / D : 0;
  const double A11 = M[4] * D, A22 = M[0] * D;
  const double A12 = -M[1] * D, A21 = -M[3] * D;
  const double b1 = -A11 * M[2] - A12 * M[5];
  const double b2 = -A21 * M[2] - A22 * M[5];
  iM[0] = A11; iM[1] = A12; iM[2] = b1;
  iM[3] = A21; iM[4] = A22; iM[5] = b2;
}

static int border_interp(int p, int len, int border) {
  if ((unsigned)p < (unsigned)len) return p;
  if (len == 1) return 0;
  const int delta = border == 4;
  do {
    if (p < 0) p = -p - 1 + delta;
    else p = len - 1 - (p - len) - delta;
  } while ((unsigned)p >= (unsigned)len);
  return p;
}

static void bilinear_tab(int fx, int fy, int* w) {
  const float scale = 1.f / 32;
  const float tx0 = 1.f - fx * scale, tx1 = fx * scale;
  const float ty0 = 1.f - fy * scale, ty1 = fy * scale;
  const float v[4] = {ty0 * tx0, ty0 * tx1, ty1 * tx0, ty1 * tx1};
  int isum = 0;
  for (int k = 0; k < 4; ++k) { w[k] = round_f(v[k] * 32768.f); isum += w[k]; }
  if (isum != 32768) {
    const int diff = isum - 32768;
    int mk = 0, Mk = 0;
    for (int k = 0; k < 4; ++k) {
      if (w[k] < w[mk]) mk = k;
      else if (w[k] > w[Mk]) Mk = k;
    }
    if (diff < 0) w[Mk] -= diff;
    else w[mk] -= diff;
  }
}

/* src: top-left of a w x h BGR crop with row_stride; iM: dst->src (already inverted) */
void cv_warp_affine_u8(const uint8_t* src, int row_stride, int w, int h, const double* iM, uint8_t* dst, int out_w,
                       int out_h, int border) {
  const int AB_BITS = 10, AB_SCALE = 1 << 10, INTER_BITS = 5;
  const int round_delta = AB_SCALE / 32 / 2;
  for (int y = 0; y < out_h; ++y) {
    const int X0 = round_d((iM[1] * y + iM[2]) * AB_SCALE) + round_delta;
    const int Y0 = round_d((iM[4] * y + iM[5]) * AB_SCALE) + round_delta;
    for (int x = 0; x < out_w; ++x) {
      const int adelta = round_d(iM[0] * x * AB_SCALE);
      const int bdelta = round_d(iM[3] * x * AB_SCALE);
      const int X = (X0 + adelta) >> (AB_BITS - INTER_BITS);
      const int Y = (Y0 + bdelta) >> (AB_BITS - INTER_BITS);
      const int sx = clampi(X >> INTER_BITS, -32768, 32767);
      const int sy = clampi(Y >> INTER_BITS, -32768, 32767);
      int wt[4];
      bilinear_tab(X & 31, Y & 31, wt);
      uint8_t* o = dst + ((size_t)y * out_w + x) * 3;
      if ((border & 0xFF) == 0) {   /* BORDER_CONSTANT, value border >> 8: outside taps read the value */
        const int cv = border >> 8;
        for (int c = 0; c < 3; ++c) {
          int t[4];
          for (int k = 0; k < 4; ++k) {
            const int xx = sx + (k & 1), yy = sy + (k >> 1);
            t[k] = ((unsigned)xx < (unsigned)w && (unsigned)yy < (unsigned)h) ? src[(size_t)yy * row_stride + xx * 3 + c]
                                                                               : cv;
          }
          const int v = (t[0] * wt[0] + t[1] * wt[1] + t[2] * wt[2] + t[3] * wt[3] + (1 << 14)) >> 15;
          o[c] = (uint8_t)clampi(v, 0, 255);
        }
        continue;
      }
      const int x0 = border_interp(sx, w, border), x1 = border_interp(sx + 1, w, border);
      const int y0 = border_interp(sy, h, border), y1 = border_interp(sy + 1, h, border);
      const uint8_t* r0 = src + (size_t)y0 * row_stride;
      const uint8_t* r1 = src + (size_t)y1 * row_stride;
      for (int c = 0; c < 3; ++c) {
        int v = r0[x0 * 3 + c] * wt[0] + r0[x1 * 3 + c] * wt[1] + r1[x0 * 3 + c] * wt[2] + r1[x1 * 3 + c] * wt[3];
        v = (v + (1 << 14)) >> 15;
        o[c] = (uint8_t)clampi(v, 0, 255);
      }
    }
  }
}

/* computeResizeAreaTab (cn = 1: indices in pixels). tab entries: si, di, alpha. returns count */
int cv_area_tab(int ssize, int dsize, double scale, int* si, int* di, float* alpha) {
  int k = 0;
  for (int dx = 0; dx < dsize; ++dx) {
    const double fsx1 = dx * scale;
    const double fsx2 = fsx1 + scale;
    const double cellWidth = scale < ssize - fsx1 ? scale : ssize - fsx1;
    int sx1 = (int)ceil(fsx1), sx2 = (int)floor(fsx2);
    sx2 = sx2 < ssize - 1 ? sx2 : ssize - 1;
    sx1 = sx1 < sx2 ? sx1 : sx2;
    if (sx1 - fsx1 > 1e-3) {
      di[k] = dx; si[k] = sx1 - 1; alpha[k++] = (float)((sx1 - fsx1) / cellWidth);
    }
    for (int sx = sx1; sx < sx2; ++sx) {
      di[k] = dx; si[k] = sx; alpha[k++] = (float)(1.0 / cellWidth);
    }
    if (fsx2 - sx2 > 1e-3) {
      double a = fsx2 - sx2;
      a = a < 1. ? a : 1.;
      a = a < cellWidth ? a : cellWidth;
      di[k] = dx; si[k] = sx2; alpha[k++] = (float)(a / cellWidth);
    }
  }
  return k;
}

/* INTER_AREA at an exact integer ratio (resizeAreaFast_Invoker, CV_8UC3): 2x2 goes through
 * ResizeAreaFastVec, (a+b+c+d+2)>>2 for every byte; other ratios saturate_cast<uchar>(sum * (1.f/area)). */
void cv_resize_area_fast_u8(const uint8_t* src, int row_stride, int isx, int isy, uint8_t* dst, int OH, int OW) {
  const float scale = 1.f / (float)(isx * isy);
  for (int dy = 0; dy < OH; ++dy)
    for (int dx = 0; dx < OW; ++dx)
      for (int c = 0; c < 3; ++c) {
        int sum = 0;
        for (int j = 0; j < isy; ++j)
          for (int i = 0; i < isx; ++i) sum += src[(size_t)(dy * isy + j) * row_stride + (dx * isx + i) * 3 + c];
        const int v = (isx == 2 && isy == 2) ? ((sum + 2) >> 2) : round_f((float)sum * scale);
        dst[((size_t)dy * OW + dx) * 3 + c] = (uint8_t)clampi(v, 0, 255);
      }
}

/* INTER_AREA generic path, CV_8UC3. Row buffer accumulated per source row in table
 * order, then beta-weighted into the destination row sum (float), saturate_cast at the end. */
void cv_resize_area2_u8(const uint8_t* src, int H, int W, int row_stride, uint8_t* dst, int OH, int OW, double sx,
                        double sy);
void cv_resize_area_u8(const uint8_t* src, int H, int W, int row_stride, uint8_t* dst, int OH, int OW) {
  cv_resize_area2_u8(src, H, W, row_stride, dst, OH, OW, 1.0 / ((double)OW / W), 1.0 / ((double)OH / H));
}

void cv_resize_area2_u8(const uint8_t* src, int H, int W, int row_stride, uint8_t* dst, int OH, int OW, double sx,
                        double sy) {
  int* xs = (int*)malloc(sizeof(int) * W * 2); int* xd = (int*)malloc(sizeof(int) * W * 2);
  float* xa = (float*)malloc(sizeof(float) * W * 2);
  int* ys = (int*)malloc(sizeof(int) * H * 2); int* yd = (int*)malloc(sizeof(int) * H * 2);
  float* ya = (float*)malloc(sizeof(float) * H * 2);
  const int nx = cv_area_tab(W, OW, sx, xs, xd, xa);
  const int ny = cv_area_tab(H, OH, sy, ys, yd, ya);
  float* buf = (float*)malloc(sizeof(float) * OW * 3);
  float* sum = (float*)malloc(sizeof(float) * OW * 3);
  int prev = -1;
  for (int j = 0; j < ny; ++j) {
    const float beta = ya[j];
    const int dy = yd[j];
    const uint8_t* S = src + (size_t)ys[j] * row_stride;
    for (int i = 0; i < OW * 3; ++i) buf[i] = 0.f;
    for (int k = 0; k < nx; ++k) {
      const int d = xd[k] * 3, s = xs[k] * 3;
      const float a = xa[k];
      const float t0 = buf[d] + S[s] * a, t1 = buf[d + 1] + S[s + 1] * a, t2 = buf[d + 2] + S[s + 2] * a;
      buf[d] = t0; buf[d + 1] = t1; buf[d + 2] = t2;
    }
    if (dy != prev) {
      if (prev >= 0)
        for (int i = 0; i < OW * 3; ++i) dst[(size_t)prev * OW * 3 + i] = (uint8_t)clampi(round_f(sum[i]), 0, 255);
      for (int i = 0; i < OW * 3; ++i) sum[i] = beta * buf[i];
      prev = dy;
    } else {
      for (int i = 0; i < OW * 3; ++i) sum[i] += beta * buf[i];
    }
  }
  if (prev >= 0)
    for (int i = 0; i < OW * 3; ++i) dst[(size_t)prev * OW * 3 + i] = (uint8_t)clampi(round_f(sum[i]), 0, 255);
  free(xs); free(xd); free(xa); free(ys); free(yd); free(ya); free(buf); free(sum);
}
