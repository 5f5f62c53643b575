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

// LDS NMS: up to NMS_CAP candidates (sorted boxes 16 B, original index and kept list 2 B each: 160 KB
// with the block masks; the power-of-two sort keys, <= 64 KB, share the boxes' space)
constexpr int NMS_CAP = 8160;

// Greedy NMS of one image per workgroup (insightface SCRFD.nms: score-descending order, a box is kept
// unless a kept box before it overlaps it by more than the threshold). The sorted candidates are walked
// in blocks of 64: every candidate of a block is tested against all boxes kept so far in parallel, the
// block's own pairs give a 64 x 64 suppression mask, and one wave then resolves the block in order
// with register bit operations - no barrier per kept box (the first form's greedy loop took two
// barriers per kept box: ~0.78 ms per C5 launch, 6 % of the C5 kernel time, r06ab). The keep set and
// order are the sequential greedy pass's exactly: same pair test, same IoU arithmetic (earlier box's
// area first).
__global__ __launch_bounds__(1024) void scrfd_nms(const float* __restrict__ cand, const int* __restrict__ count,
                                                  int cap, float nms_thresh, int max_det, float* __restrict__ dets,
                                                  float* __restrict__ kps, int* __restrict__ nkeep) {
  __shared__ __attribute__((aligned(16))) char sbuf[NMS_CAP * 16];
  __shared__ unsigned short sidx[NMS_CAP];
  __shared__ unsigned short klist[NMS_CAP];     // sorted positions of the kept boxes, in order
  __shared__ unsigned long long bmask[64];      // bit j of bmask[i]: block box i suppresses block box j
  __shared__ unsigned long long bsup;           // block boxes suppressed by a box kept before the block
  __shared__ int s_nk;
  unsigned long long* keys = reinterpret_cast<unsigned long long*>(sbuf);
  const float4* boxes = reinterpret_cast<const float4*>(sbuf);
  const int n = blockIdx.x;
  const int tid = threadIdx.x;
  const int K = min(count[n], cap);
  if (K > NMS_CAP) return;   // scrfd_nms_big handles this image
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
  for (int i = tid; i < K; i += blockDim.x) sidx[i] = (unsigned short)(keys[i] & 0x1FFFu);
  __syncthreads();
  for (int i = tid; i < K; i += blockDim.x)
    reinterpret_cast<float4*>(sbuf)[i] = *reinterpret_cast<const float4*>(cb + (int)sidx[i] * 16);
  // the pair test of the sequential pass: box e before box l suppresses l
  auto suppresses = [&](const float4 e, const float4 l) __attribute__((always_inline)) {
    const float area_e = (e.z - e.x + 1.0f) * (e.w - e.y + 1.0f);
    const float xx1 = fmaxf(e.x, l.x), yy1 = fmaxf(e.y, l.y);
    const float xx2 = fminf(e.z, l.z), yy2 = fminf(e.w, l.w);
    const float w = fmaxf(0.0f, xx2 - xx1 + 1.0f);
    const float h = fmaxf(0.0f, yy2 - yy1 + 1.0f);
    const float inter = w * h;
    const float area_l = (l.z - l.x + 1.0f) * (l.w - l.y + 1.0f);
    const float ovr = inter / (area_e + area_l - inter);
    return !(ovr <= nms_thresh);
  };
  int nk = 0;
  for (int b0 = 0; b0 < K; b0 += 64) {
    const int nb = min(64, K - b0);
    if (tid < 64) bmask[tid] = 0ull;
    if (tid == 0) bsup = 0ull;
    __syncthreads();   // (also: the boxes, and the previous block's kept list)
    // the block's candidates against every box kept so far
    for (int q = tid; q < nb * nk; q += blockDim.x) {
      const int c = q % nb, k = q / nb;
      if (suppresses(boxes[klist[k]], boxes[b0 + c])) atomicOr(&bsup, 1ull << c);
    }
    // the block's own pairs (i < j): thread t takes box i = t / 16 against boxes j = 4 (t % 16) .. +3
    {
      const int i = tid >> 4, j0 = (tid & 15) * 4;
      if (i < nb) {
        const float4 bi = boxes[b0 + i];
        unsigned long long m = 0ull;
#pragma unroll
        for (int jj = 0; jj < 4; ++jj) {
          const int j = j0 + jj;
          if (j > i && j < nb && suppresses(bi, boxes[b0 + j])) m |= 1ull << j;
        }
        if (m) atomicOr(&bmask[i], m);
      }
    }
    __syncthreads();
    if (tid < 64) {   // one wave resolves the block in order
      unsigned long long removed = bsup;
      const unsigned long long row = bmask[tid];
      for (int i = 0; i < nb; ++i) {
        if ((removed >> i) & 1ull) continue;   // (wave-uniform)
        const unsigned lo = __builtin_amdgcn_readlane((unsigned)row, i), hi = __builtin_amdgcn_readlane((unsigned)(row >> 32), i);
        removed |= ((unsigned long long)hi << 32) | lo;
        if (tid == 0) klist[nk] = (unsigned short)(b0 + i);
        if (nk < max_det && tid < 15) {
          const float v = cb[(int)sidx[b0 + i] * 16 + tid];
          if (tid < 5) dets[((long long)n * max_det + nk) * 5 + tid] = v;
          else kps[((long long)n * max_det + nk) * 10 + (tid - 5)] = v;
        }
        ++nk;
      }
      if (tid == 0) s_nk = nk;
    }
    __syncthreads();
    nk = s_nk;
  }
  if (tid == 0) nkeep[n] = nk;
}

// The same greedy NMS for an image with more than NMS_CAP candidates (low thresholds at
// the heavy rotation sizes, up to 2*(D/8)^2*(1+1/4+1/16) anchors): keys live in global
// memory, sorted by a single-workgroup bitonic network whose strides below BIG_TILE run
// in LDS; then the greedy pass walks the sorted order in blocks of 1024: every
// candidate of a block is first tested against all boxes kept so far (in parallel),
// then the block is resolved in order (one barrier round per kept box). Same keys (score
// desc, anchor index asc), same IoU arithmetic, same suppression test as scrfd_nms.
constexpr int BIG_TILE = 8192;

__device__ inline void cmpswap(unsigned long long& a, unsigned long long& b, bool up) {
  if ((a > b) == up) { const unsigned long long t = a; a = b; b = t; }
}

__global__ __launch_bounds__(1024) void scrfd_nms_big(const float* __restrict__ cand, const int* __restrict__ count,
                                                      int cap, int pcap, unsigned long long* __restrict__ keys_g,
                                                      int* __restrict__ slot_of, float* __restrict__ kept_g,
                                                      float nms_thresh, int max_det, float* __restrict__ dets,
                                                      float* __restrict__ kps, int* __restrict__ nkeep) {
  __shared__ unsigned long long tile[BIG_TILE];
  __shared__ float sbox[1024][4];
  __shared__ unsigned char ssup[1024];
  __shared__ int s_next;
  const int n = blockIdx.x;
  const int tid = threadIdx.x;
  const int K = min(count[n], cap);
  if (K <= NMS_CAP) return;
  const float* cb = cand + (long long)n * cap * 16;
  unsigned long long* keys = keys_g + (long long)n * pcap;
  int* smap = slot_of + (long long)n * cap;
  float* kept_box = kept_g + (long long)n * cap * 4;
  int P = BIG_TILE;
  while (P < K) P <<= 1;
  for (int i = tid; i < P; i += 1024) {
    unsigned long long key = ~0ull;
    if (i < K) {
      const unsigned u = __float_as_uint(cb[i * 16 + 4]);
      const unsigned ord = (u & 0x80000000u) ? ~u : (u | 0x80000000u);
      const unsigned aidx = __float_as_uint(cb[i * 16 + 15]);
      key = ((unsigned long long)(~ord) << 32) | aidx;   // anchor indices are unique per image
      smap[aidx] = i;
    }
    keys[i] = key;
  }
  __syncthreads();
  // bitonic sort ascending; all stages with k <= BIG_TILE in one LDS visit per tile
  for (int t0 = 0; t0 < P; t0 += BIG_TILE) {
    for (int i = tid; i < BIG_TILE; i += 1024) tile[i] = keys[t0 + i];
    __syncthreads();
    for (int k = 2; k <= BIG_TILE; k <<= 1)
      for (int j = k >> 1; j > 0; j >>= 1) {
        for (int li = tid; li < BIG_TILE; li += 1024) {
          const int lx = li ^ j;
          if (lx > li) cmpswap(tile[li], tile[lx], ((t0 + li) & k) == 0);
        }
        __syncthreads();
      }
    for (int i = tid; i < BIG_TILE; i += 1024) keys[t0 + i] = tile[i];
    __syncthreads();
  }
  for (int k = 2 * BIG_TILE; k <= P; k <<= 1) {
    int j = k >> 1;
    for (; j >= BIG_TILE; j >>= 1) {
      for (int i = tid; i < P; i += 1024) {
        const int ixj = i ^ j;
        if (ixj > i) {
          unsigned long long a = keys[i], b = keys[ixj];
          cmpswap(a, b, (i & k) == 0);
          keys[i] = a; keys[ixj] = b;
        }
      }
      __syncthreads();
    }
    for (int t0 = 0; t0 < P; t0 += BIG_TILE) {
      for (int i = tid; i < BIG_TILE; i += 1024) tile[i] = keys[t0 + i];
      __syncthreads();
      for (int jj = j; jj > 0; jj >>= 1) {
        for (int li = tid; li < BIG_TILE; li += 1024) {
          const int lx = li ^ jj;
          if (lx > li) cmpswap(tile[li], tile[lx], ((t0 + li) & k) == 0);
        }
        __syncthreads();
      }
      for (int i = tid; i < BIG_TILE; i += 1024) keys[t0 + i] = tile[i];
      __syncthreads();
    }
  }
  // blocked greedy pass
  int nk = 0;
  for (int b0 = 0; b0 < K; b0 += 1024) {
    const int i = b0 + tid;
    bool sup = i >= K;
    float x1 = 0.f, y1 = 0.f, x2 = 0.f, y2 = 0.f, area = 0.f;
    int si = 0;
    if (!sup) {
      si = smap[(unsigned)(keys[i] & 0xFFFFFFFFull)];
      const float* bj = cb + si * 16;
      x1 = bj[0]; y1 = bj[1]; x2 = bj[2]; y2 = bj[3];
      area = (x2 - x1 + 1.0f) * (y2 - y1 + 1.0f);
      for (int q = 0; q < nk; ++q) {
        const float* kb = kept_box + q * 4;
        const float kx1 = kb[0], ky1 = kb[1], kx2 = kb[2], ky2 = kb[3];
        const float area_k = (kx2 - kx1 + 1.0f) * (ky2 - ky1 + 1.0f);
        const float w = fmaxf(0.0f, fminf(kx2, x2) - fmaxf(kx1, x1) + 1.0f);
        const float h = fmaxf(0.0f, fminf(ky2, y2) - fmaxf(ky1, y1) + 1.0f);
        const float inter = w * h;
        const float ovr = inter / (area_k + area - inter);
        if (!(ovr <= nms_thresh)) { sup = true; break; }
      }
    }
    sbox[tid][0] = x1; sbox[tid][1] = y1; sbox[tid][2] = x2; sbox[tid][3] = y2;
    ssup[tid] = sup ? 1 : 0;
    __syncthreads();
    int cur = 0;
    while (true) {
      if (tid == 0) s_next = 1024;
      __syncthreads();
      if (tid >= cur && !ssup[tid]) atomicMin(&s_next, tid);
      __syncthreads();
      const int c = s_next;
      if (c >= 1024) break;
      if (tid == c) {
        float* kb = kept_box + nk * 4;
        kb[0] = x1; kb[1] = y1; kb[2] = x2; kb[3] = y2;
        if (nk < max_det) {
          const float* src = cb + si * 16;
          for (int e = 0; e < 5; ++e) dets[((long long)n * max_det + nk) * 5 + e] = src[e];
          for (int e = 0; e < 10; ++e) kps[((long long)n * max_det + nk) * 10 + e] = src[5 + e];
        }
      }
      if (tid > c && !ssup[tid]) {
        const float cx1 = sbox[c][0], cy1 = sbox[c][1], cx2 = sbox[c][2], cy2 = sbox[c][3];
        const float area_c = (cx2 - cx1 + 1.0f) * (cy2 - cy1 + 1.0f);
        const float w = fmaxf(0.0f, fminf(cx2, x2) - fmaxf(cx1, x1) + 1.0f);
        const float h = fmaxf(0.0f, fminf(cy2, y2) - fmaxf(cy1, y1) + 1.0f);
        const float inter = w * h;
        const float ovr = inter / (area_c + area - inter);
        if (!(ovr <= nms_thresh)) ssup[tid] = 1;
      }
      ++nk;
      cur = c + 1;
      __syncthreads();
    }
    __syncthreads();
  }
  if (tid == 0) nkeep[n] = nk;
}

hipError_t scrfd_nms_big_launch(const float* cand, const int* count, int cap, int pcap, unsigned long long* keys,
                                int* slot_of, float* kept, float nms_thresh, int max_det, float* dets, float* kps,
                                int* nkeep, int N, hipStream_t s) {
  hipLaunchKernelGGL(scrfd_nms_big, dim3(N), dim3(1024), 0, s, cand, count, cap, pcap, keys, slot_of, kept,
                     nms_thresh, max_det, dets, kps, nkeep);
  return hipGetLastError();
}

hipError_t scrfd_decode_launch(const DecodeParams& p, int N, hipStream_t s) {
  dim3 grid((p.total_loc + 255) / 256, N);
  hipLaunchKernelGGL(scrfd_decode, grid, dim3(256), 0, s, p);
  return hipGetLastError();
}

hipError_t scrfd_nms_launch(const float* cand, const int* count, int cap, float nms_thresh, int max_det, float* dets,
                            float* kps, int* nkeep, int N, hipStream_t s) {
  hipLaunchKernelGGL(scrfd_nms, dim3(N), dim3(1024), 0, s, cand, count, cap, nms_thresh, max_det, dets, kps, nkeep);
  return hipGetLastError();
}

}  // namespace pc
