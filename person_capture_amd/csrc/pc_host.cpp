// Host-side (CPU) geometry of the align step, native like the rest of the
// runtime: cv::estimateAffinePartial2D(method=LMEDS) and the warpAffine matrix
// inversion, batched over all faces of a frame batch.
//
// Restates OpenCV 4.9 calib3d/ptsetreg.cpp (opencv-python-headless 4.9.0.80,
// not vendored) as used by FaceEmbedder._align_by_5pts (face_embedder.py:1465-1473):
//  * LMeDS: niters = RANSACUpdateNumIters(0.99, 0.45, 2, 2000) = 13 iterations,
//    cv::RNG(uint64(-1)) multiply-with-carry subsets of 2 distinct points,
//    analytic 2-point similarity (AffinePartial2DEstimatorCallback::runKernel),
//    float residuals, median via nth_element, inliers with
//    sigma = 2.5*1.4826*(1+5/(n-2))*sqrt(minMedian).
//  * refinement (refineIters=10, Levenberg-Marquardt on the inliers of a model
//    that is linear in (a, b, tx, ty)) is replaced by its fixed point, the
//    closed-form least-squares similarity over the inliers. Parity vs OpenCV:
//    unpinned (OpenCV absent); the warp's 1/1024-pixel fixed point absorbs
//    differences below ~1e-4 px.
#include <math.h>
#include <stdint.h>
#include <string.h>
#include <algorithm>
#include <vector>
#include "../../include/pcgpu.h"

namespace {

struct Rng {
  uint64_t state;
  explicit Rng(uint64_t s) : state(s ? s : 0xffffffffu) {}
  unsigned next() {
    state = (uint64_t)(unsigned)state * 4164903690U + (unsigned)(state >> 32);
    return (unsigned)state;
  }
  int uniform(int a, int b) { return a == b ? a : (int)(next() % (unsigned)(b - a) + a); }
};

void run_kernel2(const float* f, const float* t, double* M) {
  const double x1 = f[0], y1 = f[1], x2 = f[2], y2 = f[3];
  const double X1 = t[0], Y1 = t[1], X2 = t[2], Y2 = t[3];
  const double d = 1. / ((x1 - x2) * (x1 - x2) + (y1 - y2) * (y1 - y2));
  const double S0 = d * ((X1 - X2) * (x1 - x2) + (Y1 - Y2) * (y1 - y2));
  const double S1 = d * ((Y1 - Y2) * (x1 - x2) - (X1 - X2) * (y1 - y2));
  const double S2 = d * ((Y1 - Y2) * (x1 * y2 - x2 * y1) - (X1 * y2 - X2 * y1) * (y1 - y2) - (X1 * x2 - X2 * x1) * (x1 - x2));
  const double S3 = d * (-(X1 - X2) * (x1 * y2 - x2 * y1) - (Y1 * x2 - Y2 * x1) * (x1 - x2) - (Y1 * y2 - Y2 * y1) * (y1 - y2));
  M[0] = M[4] = S0;
  M[1] = -S1;
  M[2] = S2;
  M[3] = S1;
  M[5] = S3;
}

void compute_err(const float* from, const float* to, int n, const double* H, float* err) {
  const float h0 = (float)H[0], h1 = (float)H[1], h2 = (float)H[2], h3 = (float)H[3], h4 = (float)H[4],
              h5 = (float)H[5];
  for (int i = 0; i < n; ++i) {
    const float fx = from[2 * i], fy = from[2 * i + 1];
    const float a = h0 * fx + h1 * fy + h2 - to[2 * i];
    const float b = h3 * fx + h4 * fy + h5 - to[2 * i + 1];
    err[i] = a * a + b * b;
  }
}

// returns 1 and writes M (2x3 row-major, src->dst) on success
int estimate_partial_lmeds(const float* from, const float* to, int n, double* M) {
  if (n < 2) return 0;
  const int model_points = 2;
  double best[6] = {0, 0, 0, 0, 0, 0};
  if (n == model_points) {
    run_kernel2(from, to, M);
    return 1;
  }
  const double p = 0.99, ep = 0.45;
  double num = std::max(1. - p, 1e-300), denom = 1. - pow(1. - ep, model_points);
  int niters = 2000;
  if (denom >= 1e-300) {
    num = log(num);
    denom = log(denom);
    niters = (denom >= 0 || -num >= 2000 * (-denom)) ? 2000 : (int)lrint(num / denom);
  }
  niters = std::max(niters, 3);
  Rng rng((uint64_t)-1);
  double min_median = 1e300;
  std::vector<float> err(n);
  std::vector<int32_t> errs(n);
  for (int it = 0; it < niters; ++it) {
    int idx[2];
    float ms1[4], ms2[4];
    for (int i = 0; i < model_points; ++i) {
      int k;
      for (;;) {
        k = idx[i] = rng.uniform(0, n);
        int j;
        for (j = 0; j < i; ++j)
          if (k == idx[j]) break;
        if (j == i) break;
      }
      ms1[2 * i] = from[2 * k]; ms1[2 * i + 1] = from[2 * k + 1];
      ms2[2 * i] = to[2 * k]; ms2[2 * i + 1] = to[2 * k + 1];
    }
    double H[6];
    run_kernel2(ms1, ms2, H);
    compute_err(from, to, n, H, err.data());
    // OpenCV: nth_element over the residuals' int32 bit patterns
    memcpy(errs.data(), err.data(), sizeof(float) * n);
    std::nth_element(errs.begin(), errs.begin() + n / 2, errs.end());
    float mf;
    memcpy(&mf, &errs[n / 2], sizeof(float));
    const double median = mf;
    if (median < min_median) {
      min_median = median;
      memcpy(best, H, sizeof(best));
    }
  }
  if (!(min_median < 1e300)) return 0;
  double sigma = 2.5 * 1.4826 * (1 + 5. / (n - model_points)) * sqrt(min_median);
  sigma = std::max(sigma, 0.001);
  compute_err(from, to, n, best, err.data());
  const float thr = (float)(sigma * sigma);
  std::vector<int> inl;
  for (int i = 0; i < n; ++i)
    if (err[i] <= thr) inl.push_back(i);
  if ((int)inl.size() < model_points) return 0;
  // refinement fixed point: least-squares similarity over the inliers
  double mx = 0, my = 0, nx = 0, ny = 0;
  const double m = (double)inl.size();
  for (int i : inl) { mx += from[2 * i]; my += from[2 * i + 1]; nx += to[2 * i]; ny += to[2 * i + 1]; }
  mx /= m; my /= m; nx /= m; ny /= m;
  double sxx = 0, sa = 0, sb = 0;
  for (int i : inl) {
    const double px = from[2 * i] - mx, py = from[2 * i + 1] - my;
    const double qx = to[2 * i] - nx, qy = to[2 * i + 1] - ny;
    sxx += px * px + py * py;
    sa += px * qx + py * qy;
    sb += px * qy - py * qx;
  }
  if (sxx <= 0) {
    memcpy(M, best, sizeof(best));
    return 1;
  }
  const double a = sa / sxx, b = sb / sxx;
  M[0] = a; M[1] = -b; M[2] = nx - (a * mx - b * my);
  M[3] = b; M[4] = a; M[5] = ny - (b * mx + a * my);
  return 1;
}

}  // namespace

extern "C" int pc_estimate_affine_partial(const float* h_from, const float* h_to, int npts, int n, double* h_M,
                                          int32_t* h_ok) {
  if (!h_from || !h_to || !h_M || !h_ok || npts < 2 || n < 0) return PC_ERR_ARG;
  for (int i = 0; i < n; ++i)
    h_ok[i] = estimate_partial_lmeds(h_from + (size_t)i * npts * 2, h_to, npts, h_M + (size_t)i * 6);
  return PC_OK;
}

extern "C" int pc_invert_affine(const double* M, double* iM) {
  if (!M || !iM) return PC_ERR_ARG;
  double D = M[0] * M[4] - M[1] * M[3];
  D = D != 0 ? 1. / D : 0;
  const double A11 = M[4] * D, A22 = M[0] * D, A12 = -M[1] * D, A21 = -M[3] * D;
  iM[0] = A11; iM[1] = A12; iM[2] = -A11 * M[2] - A12 * M[5];
  iM[3] = A21; iM[4] = A22; iM[5] = -A21 * M[2] - A22 * M[5];
  return PC_OK;
}

// ---------------------------------------------------------------------------
// Pillow's BICUBIC resample coefficients (Pillow libImaging/Resample.c:
// bicubic_filter a=-0.5, support 2; precompute_coeffs; normalize_coeffs_8bpc with
// PRECISION_BITS = 22), as reached by torchvision Resize on a PIL image inside the
// OpenCLIP preprocess of ReIDEmbedder.extract (reid_embedder.py:49). Only the output
// positions [first, first + count) are produced (CenterCrop keeps 224 of them).
// Returns ksize, or a negative value if kmax is too small / arguments are invalid.
// ---------------------------------------------------------------------------
namespace {
double pil_bicubic(double x) {
  const double a = -0.5;
  if (x < 0.0) x = -x;
  if (x < 1.0) return ((a + 2.0) * x - (a + 3.0)) * x * x + 1;
  if (x < 2.0) return (((x - 5) * x + 8) * x - 4) * a;
  return 0.0;
}
}  // namespace

extern "C" int pc_pil_bicubic_coeffs(int in_size, int out_size, int first, int count, int32_t* h_bounds, int32_t* h_kk,
                                     int kmax) {
  if (in_size <= 0 || out_size <= 0 || first < 0 || count < 0 || first + count > out_size || !h_bounds || !h_kk)
    return -PC_ERR_ARG;
  const float in0 = 0.f, in1 = (float)in_size;
  double filterscale, scale;
  filterscale = scale = (double)(in1 - in0) / out_size;
  if (filterscale < 1.0) filterscale = 1.0;
  const double support = 2.0 * filterscale;
  const int ksize = (int)ceil(support) * 2 + 1;
  if (ksize > kmax) return -PC_ERR_CAPACITY;
  std::vector<double> k(ksize);
  for (int i = 0; i < count; ++i) {
    const int xx = first + i;
    const double center = in0 + (xx + 0.5) * scale;
    double ww = 0.0;
    const double ss = 1.0 / filterscale;
    int xmin = (int)(center - support + 0.5);
    if (xmin < 0) xmin = 0;
    int xmax = (int)(center + support + 0.5);
    if (xmax > in_size) xmax = in_size;
    xmax -= xmin;
    int x = 0;
    for (; x < xmax; ++x) {
      const double w = pil_bicubic((x + xmin - center + 0.5) * ss);
      k[x] = w;
      ww += w;
    }
    for (x = 0; x < xmax; ++x)
      if (ww != 0.0) k[x] /= ww;
    for (; x < ksize; ++x) k[x] = 0;
    for (x = 0; x < ksize; ++x)
      h_kk[(size_t)i * ksize + x] = k[x] < 0 ? (int32_t)(-0.5 + k[x] * (1 << 22)) : (int32_t)(0.5 + k[x] * (1 << 22));
    h_bounds[2 * i] = xmin;
    h_bounds[2 * i + 1] = xmax;
  }
  return ksize;
}

// torchvision Resize(224) (shortest edge) + CenterCrop(224) geometry for an h x w image:
// resized size and the crop's top-left in the resized image.
extern "C" int pc_clip_geometry(int h, int w, int side, int32_t* h_out4 /* rw, rh, top, left */) {
  if (h <= 0 || w <= 0 || side <= 0 || !h_out4) return PC_ERR_ARG;
  const int sh = w <= h ? w : h, lg = w <= h ? h : w;
  const int new_short = side, new_long = (int)((double)((long long)side * lg) / sh);
  const int rw = w <= h ? new_short : new_long, rh = w <= h ? new_long : new_short;
  h_out4[0] = rw;
  h_out4[1] = rh;
  h_out4[2] = (int)nearbyint((rh - side) / 2.0);   // Python round(): half to even
  h_out4[3] = (int)nearbyint((rw - side) / 2.0);
  return PC_OK;
}
