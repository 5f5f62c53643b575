// SCRFD post-processing on device (gfx950): anchor decode + threshold, then an
// exact greedy NMS per image.
//
// Restates [ext] insightface>=0.7.3 model_zoo/scrfd.py (not vendored; called from
// face_embedder.py:2176-2187):
//   forward(): anchor centres (x*s, y*s) repeated for 2 anchors, keep score >= det_thresh,
//              distance2bbox / distance2kps with predictions * stride
//   detect():  / det_scale, order = argsort(score)[::-1], nms(thresh=0.4) with the
//              "+1" pixel areas, det rows (x1,y1,x2,y2,score) + kps (5,2) in keep order
// All arithmetic is float32 with no contraction, in the same operation order as
// the numpy code, so for identical head outputs the boxes are bit-identical to
// oracle/ref_algos.py. Ties in score are ordered by ascending anchor index (the
// result of numpy's two reversed argsorts under stable sorting).
#include "pc_common.h"

#pragma clang fp contract(off)

namespace pc {

struct DecodeLevel {
  const float* out;  // [N][H][W][cs] head output: [cls a0,a1 | bbox a0(4),a1(4) | kps a0(10),a1(10)]
  int H, W, cs, stride;
  int loc_offset;    // prefix sum of H*W over previous levels
  int anchor_offset; // prefix sum of H*W*2 over previous levels
};

struct DecodeParams {
  DecodeLevel lv[3];
  int nlv;
  int total_loc;          // sum of H*W
  float thresh;
  const float* det_scale; // [N]
  float* cand;            // [N][cap][16]: x1 y1 x2 y2 score kps(10) anchor-index(bits)
  int* count;             // [N] (atomic)
  int cap;
};

__global__ void scrfd_decode(DecodeParams p) {
  const int n = blockIdx.y;
  const int loc = blockIdx.x * blockDim.x + threadIdx.x;
  if (loc >= p.total_loc) return;
  int l = 0;
  while (l + 1 < p.nlv && loc >= p.lv[l + 1].loc_offset) ++l;
  const DecodeLevel L = p.lv[l];
  const int r = loc - L.loc_offset;
  const int y = r / L.W, x = r - (r / L.W) * L.W;
  const float* o = L.out + ((long long)n * L.H * L.W + r) * L.cs;
  const float sf = (float)L.stride;
  const float cx = (float)(x * L.stride), cy = (float)(y * L.stride);
  const float ds = p.det_scale[n];
#pragma unroll
  for (int a = 0; a < 2; ++a) {
    const float logit = o[a];
    const float score = (float)(1.0 / (1.0 + exp(-(double)logit)));  // f64 sigmoid (oracle does the same)
    if (!(score >= p.thresh)) continue;
    const int slot = atomicAdd(&p.count[n], 1);
    if (slot >= p.cap) continue;
    float* c = p.cand + ((long long)n * p.cap + slot) * 16;
    const float* bb = o + 2 + a * 4;
    const float* kp = o + 10 + a * 10;
    c[0] = (cx - bb[0] * sf) / ds;
    c[1] = (cy - bb[1] * sf) / ds;
    c[2] = (cx + bb[2] * sf) / ds;
    c[3] = (cy + bb[3] * sf) / ds;
    c[4] = score;
#pragma unroll
    for (int k = 0; k < 5; ++k) {
      c[5 + 2 * k] = (cx + kp[2 * k] * sf) / ds;
      c[6 + 2 * k] = (cy + kp[2 * k + 1] * sf) / ds;
    }
    c[15] = __int_as_float(L.anchor_offset + r * 2 + a);
  }
}

constexpr int NMS_CAP = 8192;

__global__ __launch_bounds__(1024) void scrfd_nms(const float* __restrict__ cand, const int* __restrict__ count,
                                                  int cap, float nms_thresh, int max_det, float* __restrict__ dets,
                                                  float* __restrict__ kps, int* __restrict__ nkeep) {
  __shared__ unsigned long long keys[NMS_CAP];
  __shared__ unsigned supp[NMS_CAP / 32];
  __shared__ int s_next;
  const int n = blockIdx.x;
  const int tid = threadIdx.x;
  const int K = min(count[n], cap);
  const float* cb = cand + (long long)n * cap * 16;
  int P = 1;
  while (P < K) P <<= 1;
  for (int i = tid; i < P; i += blockDim.x) {
    unsigned long long key = ~0ull;
    if (i < K) {
      const unsigned u = __float_as_uint(cb[i * 16 + 4]);
      const unsigned ord = (u & 0x80000000u) ? ~u : (u | 0x80000000u);  // ascending-orderable
      const unsigned aidx = __float_as_uint(cb[i * 16 + 15]);
      key = ((unsigned long long)(~ord) << 32) | ((unsigned long long)aidx << 13) | (unsigned)i;
    }
    keys[i] = key;
  }
  for (int i = tid; i < NMS_CAP / 32; i += blockDim.x) supp[i] = 0u;
  __syncthreads();
  // bitonic sort ascending (score desc, anchor index asc)
  for (int k = 2; k <= P; k <<= 1) {
    for (int j = k >> 1; j > 0; j >>= 1) {
      for (int i = tid; i < P; i += blockDim.x) {
        const int ixj = i ^ j;
        if (ixj > i) {
          const unsigned long long a = keys[i], b = keys[ixj];
          const bool up = (i & k) == 0;
          if ((a > b) == up) { keys[i] = b; keys[ixj] = a; }
        }
      }
      __syncthreads();
    }
  }
  int cur = 0, kept = 0;
  while (cur < K) {
    const int si = (int)(keys[cur] & 0x1FFFu);
    const float* bi = cb + si * 16;
    const float x1 = bi[0], y1 = bi[1], x2 = bi[2], y2 = bi[3];
    const float area_i = (x2 - x1 + 1.0f) * (y2 - y1 + 1.0f);
    if (kept < max_det) {
      if (tid < 15) {
        const float v = bi[tid < 5 ? tid : tid];
        if (tid < 5) dets[((long long)n * max_det + kept) * 5 + tid] = v;
        else kps[((long long)n * max_det + kept) * 10 + (tid - 5)] = v;
      }
    }
    ++kept;
    for (int j = cur + 1 + tid; j < K; j += blockDim.x) {
      if (supp[j >> 5] & (1u << (j & 31))) continue;
      const int sj = (int)(keys[j] & 0x1FFFu);
      const float* bj = cb + sj * 16;
      const float xx1 = fmaxf(x1, bj[0]), yy1 = fmaxf(y1, bj[1]);
      const float xx2 = fminf(x2, bj[2]), yy2 = fminf(y2, bj[3]);
      const float w = fmaxf(0.0f, xx2 - xx1 + 1.0f);
      const float h = fmaxf(0.0f, yy2 - yy1 + 1.0f);
      const float inter = w * h;
      const float area_j = (bj[2] - bj[0] + 1.0f) * (bj[3] - bj[1] + 1.0f);
      const float ovr = inter / (area_i + area_j - inter);
      if (!(ovr <= nms_thresh)) atomicOr(&supp[j >> 5], 1u << (j & 31));
    }
    if (tid == 0) s_next = K;
    __syncthreads();
    for (int j = cur + 1 + tid; j < K; j += blockDim.x) {
      if (!(supp[j >> 5] & (1u << (j & 31)))) { atomicMin(&s_next, j); break; }
    }
    __syncthreads();
    cur = s_next;
    __syncthreads();
  }
  if (tid == 0) nkeep[n] = kept;
}

hipError_t scrfd_decode_launch(const DecodeParams& p, int N, hipStream_t s) {
  dim3 grid((p.total_loc + 255) / 256, N);
  hipLaunchKernelGGL(scrfd_decode, grid, dim3(256), 0, s, p);
  return hipGetLastError();
}

hipError_t scrfd_nms_launch(const float* cand, const int* count, int cap, float nms_thresh, int max_det, float* dets,
                            float* kps, int* nkeep, int N, hipStream_t s) {
  if (cap > NMS_CAP) return hipErrorInvalidValue;
  hipLaunchKernelGGL(scrfd_nms, dim3(N), dim3(1024), 0, s, cand, count, cap, nms_thresh, max_det, dets, kps, nkeep);
  return hipGetLastError();
}

}  // namespace pc
