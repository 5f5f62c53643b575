// Probe of the block-scaled fp8 MFMA on gfx950 (v_mfma_scale_f32_16x16x128_f8f6f4, e4m3 operands):
// (1) operand / scale / result lane layout against a host fp64 reference with exact data;
// (2) issue rate against v_mfma_f32_16x16x32_f16 (TFLOP/s over the whole chip).
// Build: hipcc --offload-arch=gfx950 -O3 tools/mx_probe.hip -o tools/mx_probe   Run: tools/mx_probe
#include <hip/hip_runtime.h>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

typedef int v8i __attribute__((ext_vector_type(8)));
typedef float v4f __attribute__((ext_vector_type(4)));
typedef _Float16 h8 __attribute__((ext_vector_type(8)));

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP %s at %d\n", hipGetErrorString(e_), __LINE__); exit(1); } } while (0)

__global__ void mx_once(const v8i* a, const v8i* b, const int* sa, const int* sb, v4f* d, float c0) {
  const int l = threadIdx.x;
  // C input: c0 * (1 + lane / 64 + r / 7) (0: a plain product)
  v4f c = {c0 * (1.f + l / 64.f), c0 * (1.f + l / 64.f + 1.f / 7), c0 * (1.f + l / 64.f + 2.f / 7), c0 * (1.f + l / 64.f + 3.f / 7)};
  c = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(a[l], b[l], c, 0, 0, 0, sa[l], 0, sb[l]);
  d[l] = c;
}

template <int MODE>   // 0: f16 16x16x32, 1: scaled fp8 16x16x128
__global__ __launch_bounds__(256) void rate(int iters, float* out) {
  v4f acc[8];
  for (int i = 0; i < 8; ++i) acc[i] = v4f{0.f, 0.f, 0.f, 0.f};
  const int l = threadIdx.x;
  if constexpr (MODE == 0) {
    h8 a, b;
    for (int j = 0; j < 8; ++j) { a[j] = (_Float16)(0.001f * (l + j)); b[j] = (_Float16)(0.002f * (l - j)); }
    for (int it = 0; it < iters; ++it)
#pragma unroll
      for (int i = 0; i < 8; ++i) acc[i] = __builtin_amdgcn_mfma_f32_16x16x32_f16(a, b, acc[i], 0, 0, 0);
  } else {
    v8i a, b;
    for (int j = 0; j < 8; ++j) { a[j] = 0x38383838 + l; b[j] = 0x30303030 + j; }
    for (int it = 0; it < iters; ++it)
#pragma unroll
      for (int i = 0; i < 8; ++i)
        acc[i] = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(a, b, acc[i], 0, 0, 0, 127, 0, 127);
  }
  float s = 0.f;
  for (int i = 0; i < 8; ++i) s += acc[i][0] + acc[i][1] + acc[i][2] + acc[i][3];
  if (s == 12345.f) out[l] = s;   // keep the work
}

static double e4m3(unsigned char v) {
  const int s = v >> 7, e = (v >> 3) & 15, m = v & 7;
  double x = e == 0 ? (m / 8.0) * std::ldexp(1.0, -6) : (1.0 + m / 8.0) * std::ldexp(1.0, e - 7);
  return s ? -x : x;
}

int main() {
  // ---- (1) layout ----
  srand(7);
  static unsigned char A[16][128], B[128][16];
  auto rb = [] { unsigned char v; do { v = (unsigned char)(rand() & 0xff); } while ((v & 0x7f) == 0x7f || ((v >> 3) & 15) > 9); return v; };
  for (int i = 0; i < 16; ++i) for (int k = 0; k < 128; ++k) A[i][k] = rb();
  for (int k = 0; k < 128; ++k) for (int j = 0; j < 16; ++j) B[k][j] = rb();
  v8i *da, *db; int *dsa, *dsb; v4f* dd;
  CK(hipMalloc(&da, 64 * 32)); CK(hipMalloc(&db, 64 * 32)); CK(hipMalloc(&dsa, 256)); CK(hipMalloc(&dsb, 256));
  CK(hipMalloc(&dd, 64 * 16));
  // hypothesis: lane l holds A[l & 15][32 (l >> 4) + byte] and B[32 (l >> 4) + byte][l & 15];
  // D[row 4 (l >> 4) + r][col l & 15]. Scale cases: the lane's scale VGPR (byte 0) for its row / column
  // and K block (sa[l] = ea(l & 15, l >> 4))
  for (int sc = 0; sc < 6; ++sc) {
    const float c0 = sc >= 4 ? (sc == 4 ? 1e6f : 3.3e4f) : 0.f;
    int ea[16][4], eb[4][16];
    for (int i = 0; i < 16; ++i) for (int q = 0; q < 4; ++q)
      ea[i][q] = sc == 0 ? 127 : sc == 1 ? 127 + q : sc == 2 ? 127 + (i % 3) : sc == 3 ? 120 + rand() % 15 : 110;
    for (int q = 0; q < 4; ++q) for (int j = 0; j < 16; ++j)
      eb[q][j] = sc == 0 ? 127 : sc == 1 ? 127 : sc == 2 ? 127 + (j % 2) : sc == 3 ? 120 + rand() % 15 : 127;
    double ref[16][16], absref[16][16];
    for (int i = 0; i < 16; ++i)
      for (int j = 0; j < 16; ++j) {
        double sum = 0, sa = 0;
        for (int k = 0; k < 128; ++k) {
          const double t = e4m3(A[i][k]) * std::ldexp(1.0, ea[i][k / 32] - 127) * e4m3(B[k][j]) * std::ldexp(1.0, eb[k / 32][j] - 127);
          sum += t;
          sa += std::fabs(t);
        }
        ref[i][j] = sum;
        absref[i][j] = sa;
      }
    std::vector<v8i> ha(64), hb(64);
    std::vector<int> hsa(64), hsb(64);
    for (int l = 0; l < 64; ++l) {
      unsigned char pa[32], pb[32];
      // measured layout: byte j of lane group g = l >> 4 is K 16 g + j (j < 16) or 64 + 16 g + j - 16
      for (int j = 0; j < 32; ++j) {
        const int k = j < 16 ? 16 * (l >> 4) + j : 64 + 16 * (l >> 4) + (j - 16);
        pa[j] = A[l & 15][k];
        pb[j] = B[k][l & 15];
      }
      memcpy(&ha[l], pa, 32);
      memcpy(&hb[l], pb, 32);
      hsa[l] = ea[l & 15][l >> 4];
      hsb[l] = eb[l >> 4][l & 15];
    }
    CK(hipMemcpy(da, ha.data(), 64 * 32, hipMemcpyHostToDevice));
    CK(hipMemcpy(db, hb.data(), 64 * 32, hipMemcpyHostToDevice));
    CK(hipMemcpy(dsa, hsa.data(), 256, hipMemcpyHostToDevice));
    CK(hipMemcpy(dsb, hsb.data(), 256, hipMemcpyHostToDevice));
    hipLaunchKernelGGL(mx_once, dim3(1), dim3(64), 0, 0, da, db, dsa, dsb, dd, c0);
    CK(hipDeviceSynchronize());
    std::vector<v4f> hd(64);
    CK(hipMemcpy(hd.data(), dd, 64 * 16, hipMemcpyDeviceToHost));
    double worst = 0, mag = 0, rel = 0;
    for (int l = 0; l < 64; ++l)
      for (int r = 0; r < 4; ++r) {
        // C input as the kernel forms it, in f32 (then exact in double)
        const double cin = (double)(c0 * (1.f + l / 64.f + r / 7.f));
        const double want = cin + ref[4 * (l >> 4) + r][l & 15];
        // an exact f32 accumulate would be within half an ulp of want
        const double ulp = std::ldexp(1.0, std::ilogb(std::fabs(want) > 0 ? want : 1.0) - 23);
        worst = std::max(worst, std::fabs(hd[l][r] - want) / ulp);
        mag = std::max(mag, std::fabs(want));
        rel = std::max(rel, std::fabs(hd[l][r] - want) / absref[4 * (l >> 4) + r][l & 15]);
      }
    printf("case %d (C %g): max |D - (C + ref)| = %.2f f32 ulps of the result (max |ref| %.3e), / sum|a b| = %.2e\n",
           sc, c0, worst, mag, rel);
    if (false)
      for (int l = 0; l < 4; ++l) printf("  lane %d: got %g %g %g %g want %g %g %g %g\n", l, hd[l][0], hd[l][1], hd[l][2],
                                         hd[l][3], ref[0][l], ref[1][l], ref[2][l], ref[3][l]);
  }

  // (scale mapping, measured with one raised lane scale at a time: lane L's scale VGPR byte 0 is the
  // exponent of row L & 15 (A) / column L & 15 (B) for K block L >> 4 = K [32 (L >> 4), +32) in the
  // K order above)

  // ---- (2) rate ----
  const int iters = 4096, grid = 256 * 8;
  float* dout; CK(hipMalloc(&dout, 1024));
  hipEvent_t e0, e1; CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
  for (int mode = 0; mode < 2; ++mode) {
    for (int rep = 0; rep < 2; ++rep) {
      CK(hipEventRecord(e0));
      if (mode == 0) hipLaunchKernelGGL(rate<0>, dim3(grid), dim3(256), 0, 0, iters, dout);
      else hipLaunchKernelGGL(rate<1>, dim3(grid), dim3(256), 0, 0, iters, dout);
      CK(hipEventRecord(e1));
      CK(hipEventSynchronize(e1));
      float ms; CK(hipEventElapsedTime(&ms, e0, e1));
      const double k = mode == 0 ? 32 : 128;
      const double fl = 2.0 * 16 * 16 * k * 8 * iters * (double)grid * 4;
      if (rep) printf("%s: %.3f ms, %.1f TFLOP/s\n", mode == 0 ? "f16 16x16x32" : "fp8-scaled 16x16x128", ms, fl / (ms * 1e-3) / 1e12);
    }
  }
  return 0;
}
