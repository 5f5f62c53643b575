// Wavefront-reduction kernels of the match stage (gfx950).
//
//  * embed_finalize: ArcFace flip-TTA sum + L2 normalise
//      face_embedder.py:1383-1389  f = e[:m] (+ e[m:2m]); f /= max(||f||, 1e-6)
//  * bank_match: cosine distance of each query to a reference bank
//      gui_app.py:660-674 (Processor._fd_min): v /= max(||v||,1e-6); fd = 1 - max(bank @ v),
//      9.0 for an empty bank; also returns argmax (first maximal row).
// One 64-lane wave per 512-d vector: each lane owns 8 contiguous floats (two
// 16-byte loads), norms/dots are reduced with xor-shuffles.
#include "pc_common.h"

namespace pc {

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
  return v;
}

// e: [rows][ld] f32 (rows = 2n when flip), out: [n][dim]
__global__ void embed_finalize(const float* __restrict__ e, int ld, int n, int dim, int flip, float eps,
                               float* __restrict__ out) {
  const int lane = threadIdx.x & 63;
  const int row = blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
  if (row >= n) return;
  float v[16];
  const int per = dim / 64;  // dim % 64 == 0, dim <= 1024
  float ss = 0.f;
#pragma unroll
  for (int j = 0; j < 16; ++j) {
    if (j < per) {
      const int c = lane * per + j;
      float x = e[(long long)row * ld + c];
      if (flip) x += e[(long long)(row + n) * ld + c];
      v[j] = x;
      ss += x * x;
    }
  }
  ss = wave_sum(ss);
  float nrm = sqrtf(ss);
  nrm = fmaxf(nrm, eps);
#pragma unroll
  for (int j = 0; j < 16; ++j)
    if (j < per) out[(long long)row * dim + lane * per + j] = v[j] / nrm;
}

// Q queries per workgroup, 4 waves sweep the bank rows.
template <int Q>
__global__ __launch_bounds__(256) void bank_match(const float* __restrict__ q, int n, const float* __restrict__ bank,
                                                  int B, int dim, float* __restrict__ fd, int* __restrict__ idx) {
  __shared__ float smax[4][Q];
  __shared__ int sidx[4][Q];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int q0 = blockIdx.x * Q;
  const int per = dim / 64;
  float qv[Q][16];
#pragma unroll
  for (int t = 0; t < Q; ++t) {
    float ss = 0.f;
#pragma unroll
    for (int j = 0; j < 16; ++j) {
      qv[t][j] = 0.f;
      if (j < per && q0 + t < n) {
        qv[t][j] = q[(long long)(q0 + t) * dim + lane * per + j];
        ss += qv[t][j] * qv[t][j];
      }
    }
    const float nrm = fmaxf(sqrtf(wave_sum(ss)), 1e-6f);
#pragma unroll
    for (int j = 0; j < 16; ++j) qv[t][j] = qv[t][j] / nrm;
  }
  float best[Q];
  int bi[Q];
#pragma unroll
  for (int t = 0; t < Q; ++t) { best[t] = -INFINITY; bi[t] = -1; }
  for (int b = wave; b < B; b += 4) {
    float bv[16];
#pragma unroll
    for (int j = 0; j < 16; ++j) bv[j] = j < per ? bank[(long long)b * dim + lane * per + j] : 0.f;
#pragma unroll
    for (int t = 0; t < Q; ++t) {
      float s = 0.f;
#pragma unroll
      for (int j = 0; j < 16; ++j) s += qv[t][j] * bv[j];
      s = wave_sum(s);
      if (s > best[t]) { best[t] = s; bi[t] = b; }
    }
  }
  if (lane == 0) {
#pragma unroll
    for (int t = 0; t < Q; ++t) { smax[wave][t] = best[t]; sidx[wave][t] = bi[t]; }
  }
  __syncthreads();
  if (threadIdx.x < Q && q0 + threadIdx.x < n) {
    const int t = threadIdx.x;
    float m = -INFINITY;
    int mi = -1;
    for (int w = 0; w < 4; ++w) {
      const float s = smax[w][t];
      const int i = sidx[w][t];
      if (i < 0) continue;
      if (s > m || (s == m && i < mi)) { m = s; mi = i; }
    }
    fd[q0 + t] = B > 0 ? 1.0f - m : 9.0f;
    if (idx) idx[q0 + t] = mi;
  }
}

hipError_t embed_finalize_launch(const float* e, int ld, int n, int dim, int flip, float* out, hipStream_t s) {
  if (dim % 64 || dim > 1024) return hipErrorInvalidValue;
  dim3 grid((n + 3) / 4);
  hipLaunchKernelGGL(embed_finalize, grid, dim3(256), 0, s, e, ld, n, dim, flip, 1e-6f, out);
  return hipGetLastError();
}

// torch.nn.functional.normalize(x, dim=1): x / max(||x||, eps) (reid_embedder.py:55, eps 1e-12)
hipError_t embed_l2_launch(const float* e, int ld, int n, int dim, float eps, float* out, hipStream_t s) {
  if (dim % 64 || dim > 1024) return hipErrorInvalidValue;
  dim3 grid((n + 3) / 4);
  hipLaunchKernelGGL(embed_finalize, grid, dim3(256), 0, s, e, ld, n, dim, 0, eps, out);
  return hipGetLastError();
}

hipError_t bank_match_launch(const float* q, int n, const float* bank, int B, int dim, float* fd, int* idx,
                             hipStream_t s) {
  if (dim % 64 || dim > 1024) return hipErrorInvalidValue;
  if (n <= 0) return hipSuccess;
  dim3 grid((n + 7) / 8);
  hipLaunchKernelGGL(bank_match<8>, grid, dim3(256), 0, s, q, n, bank, B, dim, fd, idx);
  return hipGetLastError();
}

}  // namespace pc
