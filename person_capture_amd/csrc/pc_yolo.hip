// YOLOv8 person detection pre/post-processing on device (gfx950).
//
// Restates [ext] ultralytics==8.3.205 (requirements.txt:14, not vendored) as called by
// PersonDetector.detect (detectors.py:271-296: predict(conf, iou=0.45, classes=[0],
// max_det=40, imgsz=640), rect inference):
//   * LetterBox(auto=True, stride=32): cv2.resize(INTER_LINEAR) to round(w*r) x round(h*r),
//     centred in a canvas padded to a multiple of 32 with 114, BGR->RGB, /255;
//   * Detect head inference: DFL (softmax over 16 bins, expectation) -> dist2bbox(xywh)
//     around anchor centres (x+0.5, y+0.5) * stride, class scores = sigmoid;
//   * ops.non_max_suppression: candidates whose best class is 0 and whose score > conf,
//     xywh -> xyxy, torchvision.ops.nms (IoU > iou suppresses, areas without +1),
//     first max_det kept;
//   * ops.scale_boxes: (box - pad) / gain, clipped to the frame.
// f32 arithmetic without contraction, in the numpy/torch operation order, so identical
// head outputs give bit-identical boxes to oracle/ref_algos.py. Ties in score are kept in
// ascending anchor order.
#include "pc_common.h"

#pragma clang fp contract(off)

namespace pc {

struct YoloLetterboxDesc {
  const uint8_t* src;
  int H, W, row_stride;      // source frame (BGR u8)
  int new_w, new_h;          // resized size (round(W*r), round(H*r))
  int top, left;             // padding before the resized image
  double scale_x, scale_y;   // cv::resize inverse scales (W/new_w, H/new_h)
  int simd_end;              // OpenCV SIMD vertical-pass end (bytes of a resized row)
  int identity;              // 1: shapes equal, no resize (ultralytics skips cv2.resize)
};

__device__ __forceinline__ void lin_coef_y(int d, double scale, int src_len, int& s0, short& a0, short& a1) {
  float f = (float)((d + 0.5) * scale - 0.5);
  int s = (int)floorf(f);
  f -= (float)s;
  if (s < 0) { f = 0.f; s = 0; }
  if (s >= src_len - 1) { f = 0.f; s = src_len - 1; }
  s0 = s;
  a0 = (short)__float2int_rn((1.f - f) * 2048.f);
  a1 = (short)__float2int_rn(f * 2048.f);
}

// canvas [N][Hp][Wp][4] (RGB/255, channel 3 = 0)
template <typename T>
__global__ void yolo_letterbox(const YoloLetterboxDesc* __restrict__ descs, int Hp, int Wp, T* __restrict__ out) {
  const int n = blockIdx.y;
  const int pix = blockIdx.x * blockDim.x + threadIdx.x;
  if (pix >= Hp * Wp) return;
  const YoloLetterboxDesc d = descs[n];
  const int y = pix / Wp - d.top, x = pix - (pix / Wp) * Wp - d.left;
  float v[3] = {114.f, 114.f, 114.f};
  if (x >= 0 && y >= 0 && x < d.new_w && y < d.new_h) {
    if (d.identity) {
      const uint8_t* s = d.src + (long long)y * d.row_stride + x * 3;
      v[0] = s[0]; v[1] = s[1]; v[2] = s[2];
    } else {
      int sx, sy;
      short a0, a1, b0, b1;
      lin_coef_y(x, d.scale_x, d.W, sx, a0, a1);
      lin_coef_y(y, d.scale_y, d.H, sy, b0, b1);
      const int sx1 = sx + 1 < d.W ? sx + 1 : sx;
      const int sy1 = sy + 1 < d.H ? sy + 1 : sy;
      const uint8_t* r0 = d.src + (long long)sy * d.row_stride;
      const uint8_t* r1 = d.src + (long long)sy1 * d.row_stride;
#pragma unroll
      for (int c = 0; c < 3; ++c) {
        const int S0 = r0[sx * 3 + c] * a0 + r0[sx1 * 3 + c] * a1;
        const int S1 = r1[sx * 3 + c] * a0 + r1[sx1 * 3 + c] * a1;
        int val;
        if (x * 3 + c < d.simd_end) val = ((((S0 >> 4) * (int)b0) >> 16) + (((S1 >> 4) * (int)b1) >> 16) + 2) >> 2;
        else val = (S0 * (int)b0 + S1 * (int)b1 + (1 << 21)) >> 22;
        v[c] = (float)(val < 0 ? 0 : (val > 255 ? 255 : val));
      }
    }
  }
  T* o = out + ((long long)n * Hp * Wp + pix) * 4;
  const float r = v[2] / 255.f, g = v[1] / 255.f, b = v[0] / 255.f;
  if constexpr (sizeof(T) == 2) {
    *reinterpret_cast<f16x4*>(o) = f16x4{(f16)r, (f16)g, (f16)b, (f16)0.f};
  } else {
    *reinterpret_cast<f32x4*>(o) = f32x4{r, g, b, 0.f};
  }
}

struct YoloLevel {
  const float* out;   // [N][H][W][cs]: 64 DFL logits (4 sides x 16 bins) | nc class logits
  int H, W, cs, stride;
  int loc_offset;     // anchors of previous levels
};

struct YoloDecodeParams {
  YoloLevel lv[3];
  int nlv, total, nc;
  float conf;
  float* cand;        // [N][cap][8]: x1 y1 x2 y2 (letterbox px) score anchor-index(bits)
  int* count;         // [N] atomic
  int cap;
};

__global__ void yolo_decode(YoloDecodeParams p) {
  const int n = blockIdx.y;
  const int a = blockIdx.x * blockDim.x + threadIdx.x;
  if (a >= p.total) return;
  int l = 0;
  while (l + 1 < p.nlv && a >= p.lv[l + 1].loc_offset) ++l;
  const YoloLevel L = p.lv[l];
  const int r = a - L.loc_offset;
  const int y = r / L.W, x = r - (r / L.W) * L.W;
  const float* o = L.out + ((long long)n * L.H * L.W + r) * L.cs;
  // best class (first maximal logit; sigmoid is monotone); classes=[0] keeps class 0 only
  const float* cl = o + 64;
  float best = cl[0];
  int bi = 0;
  for (int c = 1; c < p.nc; ++c)
    if (cl[c] > best) { best = cl[c]; bi = c; }
  if (bi != 0) return;
  // f64 sigmoid / exp rounded to f32 (correctly rounded on both sides: oracle does the same)
  const float score = (float)(1.0 / (1.0 + exp(-(double)best)));
  if (!(score > p.conf)) return;
  float dist[4];
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const float* b = o + k * 16;
    float m = b[0];
#pragma unroll
    for (int i = 1; i < 16; ++i) m = fmaxf(m, b[i]);
    float e[16], s = 0.f;
#pragma unroll
    for (int i = 0; i < 16; ++i) { e[i] = (float)exp((double)(b[i] - m)); s += e[i]; }
    float dsum = 0.f;
#pragma unroll
    for (int i = 0; i < 16; ++i) dsum += (e[i] / s) * (float)i;
    dist[k] = dsum;
  }
  const float ax = (float)x + 0.5f, ay = (float)y + 0.5f, sf = (float)L.stride;
  const float x1 = ax - dist[0], y1 = ay - dist[1], x2 = ax + dist[2], y2 = ay + dist[3];
  const float cx = (x1 + x2) / 2.f * sf, cy = (y1 + y2) / 2.f * sf;
  const float w = (x2 - x1) * sf, h = (y2 - y1) * sf;
  const int slot = atomicAdd(&p.count[n], 1);
  if (slot >= p.cap) return;
  float* c = p.cand + ((long long)n * p.cap + slot) * 8;
  const float hw = w / 2.f, hh = h / 2.f;
  c[0] = cx - hw;
  c[1] = cy - hh;
  c[2] = cx + hw;
  c[3] = cy + hh;
  c[4] = score;
  c[5] = __int_as_float(a);
}

constexpr int YNMS_CAP = 16384;

struct YoloScale { float gain; float padx, pady; float W0, H0; };

__global__ __launch_bounds__(1024) void yolo_nms(const float* __restrict__ cand, const int* __restrict__ count, int cap,
                                                 float iou, int max_det, const YoloScale* __restrict__ sc,
                                                 float* __restrict__ dets, int* __restrict__ nkeep,
                                                 int* __restrict__ keep_anchor) {
  __shared__ unsigned long long keys[YNMS_CAP];
  __shared__ unsigned supp[YNMS_CAP / 32];
  __shared__ int s_next;
  const int n = blockIdx.x;
  const int tid = threadIdx.x;
  const int K = min(count[n], cap);
  if (K > YNMS_CAP) return;   // yolo_nms_big handles this image
  const float* cb = cand + (long long)n * cap * 8;
  int P = 1;
  while (P < K) P <<= 1;
  for (int i = tid; i < P; i += blockDim.x) {
    unsigned long long key = ~0ull;
    if (i < K) {
      const unsigned u = __float_as_uint(cb[i * 8 + 4]);   // score > 0
      const unsigned aidx = __float_as_uint(cb[i * 8 + 5]);
      key = ((unsigned long long)(~u) << 32) | ((unsigned long long)aidx << 14) | (unsigned)i;
    }
    keys[i] = key;
  }
  for (int i = tid; i < YNMS_CAP / 32; i += blockDim.x) supp[i] = 0u;
  __syncthreads();
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
  const YoloScale S = sc[n];
  int cur = 0, kept = 0;
  while (cur < K && kept < max_det) {
    const int si = (int)(keys[cur] & 0x3FFFu);
    const float* bi = cb + si * 8;
    const float x1 = bi[0], y1 = bi[1], x2 = bi[2], y2 = bi[3];
    const float area_i = (x2 - x1) * (y2 - y1);
    if (tid == 0) {
      float* d = dets + ((long long)n * max_det + kept) * 5;
      // scale_boxes: subtract the letterbox pad, divide by the gain, clip to the frame
      d[0] = fminf(fmaxf((x1 - S.padx) / S.gain, 0.f), S.W0);
      d[1] = fminf(fmaxf((y1 - S.pady) / S.gain, 0.f), S.H0);
      d[2] = fminf(fmaxf((x2 - S.padx) / S.gain, 0.f), S.W0);
      d[3] = fminf(fmaxf((y2 - S.pady) / S.gain, 0.f), S.H0);
      d[4] = bi[4];
      if (keep_anchor) keep_anchor[(long long)n * max_det + kept] = __float_as_int(bi[5]);
    }
    ++kept;
    for (int j = cur + 1 + tid; j < K; j += blockDim.x) {
      if (supp[j >> 5] & (1u << (j & 31))) continue;
      const int sj = (int)(keys[j] & 0x3FFFu);
      const float* bj = cb + sj * 8;
      const float xx1 = fmaxf(x1, bj[0]), yy1 = fmaxf(y1, bj[1]);
      const float xx2 = fminf(x2, bj[2]), yy2 = fminf(y2, bj[3]);
      const float w = fmaxf(xx2 - xx1, 0.0f), h = fmaxf(yy2 - yy1, 0.0f);
      const float inter = w * h;
      const float area_j = (bj[2] - bj[0]) * (bj[3] - bj[1]);
      const float ov = inter / (area_i + area_j - inter);
      if (ov > iou) atomicOr(&supp[j >> 5], 1u << (j & 31));
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

// Pose head keypoints of the kept boxes (ultralytics Pose.kpts_decode, ndim 3): x = (raw * 2 +
// anchor_x - 0.5) * stride with anchor_x - 0.5 = grid x exactly, visibility = sigmoid (f64,
// rounded, as the scores), then ops.scale_coords (the unrounded letterbox pad, / gain, clip to
// the frame) and Results' Keypoints masking (x = y = 0 where visibility < 0.5).
struct YoloKptScale { float kpadx, kpady; };

__global__ void yolo_kpts(YoloDecodeParams p, int nk, int koff, int max_det, const int* __restrict__ nkeep,
                          const int* __restrict__ keep_anchor, const YoloScale* __restrict__ sc,
                          const YoloKptScale* __restrict__ ksc, float* __restrict__ kpts) {
  const int n = blockIdx.x;
  const int k = threadIdx.x;
  if (k >= nkeep[n]) return;
  const int a = keep_anchor[(long long)n * max_det + k];
  int l = 0;
  while (l + 1 < p.nlv && a >= p.lv[l + 1].loc_offset) ++l;
  const YoloLevel L = p.lv[l];
  const int r = a - L.loc_offset;
  const int y = r / L.W, x = r - (r / L.W) * L.W;
  const float* raw = L.out + ((long long)n * L.H * L.W + r) * L.cs + koff;
  const YoloScale S = sc[n];
  const YoloKptScale K = ksc[n];
  const float sf = (float)L.stride;
  float* o = kpts + ((long long)n * max_det + k) * nk;
  for (int q = 0; q < nk / 3; ++q) {
    const float px = (raw[3 * q] * 2.0f + (float)x) * sf;
    const float py = (raw[3 * q + 1] * 2.0f + (float)y) * sf;
    const float v = (float)(1.0 / (1.0 + exp(-(double)raw[3 * q + 2])));
    float ox = fminf(fmaxf((px - K.kpadx) / S.gain, 0.f), S.W0);
    float oy = fminf(fmaxf((py - K.kpady) / S.gain, 0.f), S.H0);
    if (v < 0.5f) { ox = 0.f; oy = 0.f; }
    o[3 * q] = ox;
    o[3 * q + 1] = oy;
    o[3 * q + 2] = v;
  }
}

hipError_t yolo_kpts_launch(const YoloDecodeParams& p, int nk, int koff, int max_det, const int* nkeep,
                            const int* keep_anchor, const YoloScale* sc, const YoloKptScale* ksc, float* kpts, int N,
                            hipStream_t s) {
  if (max_det > 1024) return hipErrorInvalidValue;
  hipLaunchKernelGGL(yolo_kpts, dim3(N), dim3((max_det + 63) / 64 * 64), 0, s, p, nk, koff, max_det, nkeep,
                     keep_anchor, sc, ksc, kpts);
  return hipGetLastError();
}

// The same NMS for an image with more than YNMS_CAP candidates (low thresholds at the heavy
// sizes up to 2048: 86016 anchors): keys in global memory, sorted by one workgroup (bitonic
// network, strides below YBIG_TILE in LDS), the first max_nms (30000, ultralytics'
// non_max_suppression cap) walked in blocks of 1024 — each candidate first tested against
// every box kept so far, then the block resolved in order. Keys (score desc, anchor asc),
// IoU arithmetic and the suppression test are scrfd-style ports of yolo_nms's.
constexpr int YBIG_TILE = 8192;
constexpr int YMAX_NMS = 30000;

__device__ inline void ycmpswap(unsigned long long& a, unsigned long long& b, bool up) {
  if ((a > b) == up) { const unsigned long long t = a; a = b; b = t; }
}

__global__ __launch_bounds__(1024) void yolo_nms_big(const float* __restrict__ cand, const int* __restrict__ count,
                                                     int cap, int pcap, unsigned long long* __restrict__ keys_g,
                                                     int* __restrict__ slot_of, float* __restrict__ kept_g, float iou,
                                                     int max_det, const YoloScale* __restrict__ sc,
                                                     float* __restrict__ dets, int* __restrict__ nkeep,
                                                     int* __restrict__ keep_anchor) {
  __shared__ unsigned long long tile[YBIG_TILE];
  __shared__ float sbox[1024][4];
  __shared__ unsigned char ssup[1024];
  __shared__ int s_next;
  const int n = blockIdx.x;
  const int tid = threadIdx.x;
  const int K = min(count[n], cap);
  if (K <= YNMS_CAP) return;   // yolo_nms handled this image
  const float* cb = cand + (long long)n * cap * 8;
  unsigned long long* keys = keys_g + (long long)n * pcap;
  int* smap = slot_of + (long long)n * cap;
  float* kept_box = kept_g + (long long)n * max_det * 4;
  int P = YBIG_TILE;
  while (P < K) P <<= 1;
  for (int i = tid; i < P; i += 1024) {
    unsigned long long key = ~0ull;
    if (i < K) {
      const unsigned u = __float_as_uint(cb[i * 8 + 4]);   // score > 0
      const unsigned aidx = __float_as_uint(cb[i * 8 + 5]);
      key = ((unsigned long long)(~u) << 32) | aidx;
      smap[aidx] = i;
    }
    keys[i] = key;
  }
  __syncthreads();
  for (int t0 = 0; t0 < P; t0 += YBIG_TILE) {
    for (int i = tid; i < YBIG_TILE; i += 1024) tile[i] = keys[t0 + i];
    __syncthreads();
    for (int k = 2; k <= YBIG_TILE; k <<= 1)
      for (int j = k >> 1; j > 0; j >>= 1) {
        for (int li = tid; li < YBIG_TILE; li += 1024) {
          const int lx = li ^ j;
          if (lx > li) ycmpswap(tile[li], tile[lx], ((t0 + li) & k) == 0);
        }
        __syncthreads();
      }
    for (int i = tid; i < YBIG_TILE; i += 1024) keys[t0 + i] = tile[i];
    __syncthreads();
  }
  for (int k = 2 * YBIG_TILE; k <= P; k <<= 1) {
    int j = k >> 1;
    for (; j >= YBIG_TILE; j >>= 1) {
      for (int i = tid; i < P; i += 1024) {
        const int ixj = i ^ j;
        if (ixj > i) {
          unsigned long long a = keys[i], b = keys[ixj];
          ycmpswap(a, b, (i & k) == 0);
          keys[i] = a; keys[ixj] = b;
        }
      }
      __syncthreads();
    }
    for (int t0 = 0; t0 < P; t0 += YBIG_TILE) {
      for (int i = tid; i < YBIG_TILE; i += 1024) tile[i] = keys[t0 + i];
      __syncthreads();
      for (int jj = j; jj > 0; jj >>= 1) {
        for (int li = tid; li < YBIG_TILE; li += 1024) {
          const int lx = li ^ jj;
          if (lx > li) ycmpswap(tile[li], tile[lx], ((t0 + li) & k) == 0);
        }
        __syncthreads();
      }
      for (int i = tid; i < YBIG_TILE; i += 1024) keys[t0 + i] = tile[i];
      __syncthreads();
    }
  }
  const YoloScale S = sc[n];
  const int KN = min(K, YMAX_NMS);
  int nk = 0;
  for (int b0 = 0; b0 < KN && nk < max_det; b0 += 1024) {
    const int i = b0 + tid;
    bool sup = i >= KN;
    float x1 = 0.f, y1 = 0.f, x2 = 0.f, y2 = 0.f, area = 0.f;
    int si = 0;
    if (!sup) {
      si = smap[(unsigned)(keys[i] & 0xFFFFFFFFull)];
      const float* bj = cb + si * 8;
      x1 = bj[0]; y1 = bj[1]; x2 = bj[2]; y2 = bj[3];
      area = (x2 - x1) * (y2 - y1);
      for (int q = 0; q < nk; ++q) {
        const float* kb = kept_box + q * 4;
        const float xx1 = fmaxf(kb[0], x1), yy1 = fmaxf(kb[1], y1);
        const float xx2 = fminf(kb[2], x2), yy2 = fminf(kb[3], y2);
        const float w = fmaxf(xx2 - xx1, 0.0f), h = fmaxf(yy2 - yy1, 0.0f);
        const float inter = w * h;
        const float area_k = (kb[2] - kb[0]) * (kb[3] - kb[1]);
        if (inter / (area_k + area - inter) > iou) { sup = true; break; }
      }
    }
    sbox[tid][0] = x1; sbox[tid][1] = y1; sbox[tid][2] = x2; sbox[tid][3] = y2;
    ssup[tid] = sup ? 1 : 0;
    __syncthreads();
    int cur = 0;
    while (nk < max_det) {
      if (tid == 0) s_next = 1024;
      __syncthreads();
      if (tid >= cur && !ssup[tid]) atomicMin(&s_next, tid);
      __syncthreads();
      const int c = s_next;
      if (c >= 1024) break;
      if (tid == c) {
        float* kb = kept_box + nk * 4;
        kb[0] = x1; kb[1] = y1; kb[2] = x2; kb[3] = y2;
        float* d = dets + ((long long)n * max_det + nk) * 5;
        d[0] = fminf(fmaxf((x1 - S.padx) / S.gain, 0.f), S.W0);
        d[1] = fminf(fmaxf((y1 - S.pady) / S.gain, 0.f), S.H0);
        d[2] = fminf(fmaxf((x2 - S.padx) / S.gain, 0.f), S.W0);
        d[3] = fminf(fmaxf((y2 - S.pady) / S.gain, 0.f), S.H0);
        d[4] = cb[si * 8 + 4];
        if (keep_anchor) keep_anchor[(long long)n * max_det + nk] = __float_as_int(cb[si * 8 + 5]);
      }
      if (tid > c && !ssup[tid]) {
        const float cx1 = sbox[c][0], cy1 = sbox[c][1], cx2 = sbox[c][2], cy2 = sbox[c][3];
        const float xx1 = fmaxf(cx1, x1), yy1 = fmaxf(cy1, y1);
        const float xx2 = fminf(cx2, x2), yy2 = fminf(cy2, y2);
        const float w = fmaxf(xx2 - xx1, 0.0f), h = fmaxf(yy2 - yy1, 0.0f);
        const float inter = w * h;
        const float area_c = (cx2 - cx1) * (cy2 - cy1);
        if (inter / (area_c + area - inter) > iou) ssup[tid] = 1;
      }
      ++nk;
      cur = c + 1;
      __syncthreads();
    }
    __syncthreads();
  }
  if (tid == 0) nkeep[n] = nk;
}

hipError_t yolo_nms_big_launch(const float* cand, const int* count, int cap, int pcap, unsigned long long* keys,
                               int* slot_of, float* kept, float iou, int max_det, const YoloScale* sc, float* dets,
                               int* nkeep, int* keep_anchor, int N, hipStream_t s) {
  if (max_det > 1024 * 64) return hipErrorInvalidValue;
  hipLaunchKernelGGL(yolo_nms_big, dim3(N), dim3(1024), 0, s, cand, count, cap, pcap, keys, slot_of, kept, iou, max_det,
                     sc, dets, nkeep, keep_anchor);
  return hipGetLastError();
}

hipError_t yolo_letterbox_launch(int f32, const YoloLetterboxDesc* d_descs, int N, int Hp, int Wp, void* out,
                                 hipStream_t s) {
  dim3 grid((Hp * Wp + 255) / 256, N);
  if (f32) hipLaunchKernelGGL(yolo_letterbox<float>, grid, dim3(256), 0, s, d_descs, Hp, Wp, (float*)out);
  else hipLaunchKernelGGL(yolo_letterbox<f16>, grid, dim3(256), 0, s, d_descs, Hp, Wp, (f16*)out);
  return hipGetLastError();
}

hipError_t yolo_decode_launch(const YoloDecodeParams& p, int N, hipStream_t s) {
  dim3 grid((p.total + 255) / 256, N);
  hipLaunchKernelGGL(yolo_decode, grid, dim3(256), 0, s, p);
  return hipGetLastError();
}

hipError_t yolo_nms_launch(const float* cand, const int* count, int cap, float iou, int max_det, const YoloScale* sc,
                           float* dets, int* nkeep, int N, hipStream_t s, int* keep_anchor) {
  hipLaunchKernelGGL(yolo_nms, dim3(N), dim3(1024), 0, s, cand, count, cap, iou, max_det, sc, dets, nkeep,
                     keep_anchor);
  return hipGetLastError();
}

}  // namespace pc
