// Non-GEMM network ops of the YOLOv8 and CLIP ViT programs (gfx950):
//
//  * upsample2_nhwc   nn.Upsample(scale_factor=2, mode="nearest") into a channel view
//                     of a concatenation buffer (ultralytics Concat, YOLOv8 head).
//  * layernorm_rows   nn.LayerNorm over the channels of every token (open_clip
//                     VisionTransformer ln_pre / ln_1 / ln_2 / ln_post), optionally
//                     adding a per-token table first (class + positional embedding).
//  * mha_tokens       nn.MultiheadAttention core softmax(q k^T / sqrt(d)) v for every
//                     (image, head): open_clip ResidualAttentionBlock.attention.
//
// All HBM-bound or small: one 16-byte vector per thread (upsample), one wave per
// token (layernorm, f32 statistics), and for attention one workgroup per (image,
// head, 64 queries) with the head's K and V staged in LDS; the 4 waves split the
// keys, each keeps an online-softmax state per query, and the partial states are
// merged through LDS (the flash-decoding combine).
#include <algorithm>
#include "pc_common.h"

namespace pc {

// ---------------------------------------------------------------------------
struct UpsampleParams {
  const void* x; int N, H, W, C, xcs;
  void* y; int ycs;     // output is (2H, 2W), C channels, pixel stride ycs
};

template <typename T>
__global__ void upsample2_nhwc(UpsampleParams p) {
  constexpr int V = 16 / sizeof(T);   // elements per 16-byte vector
  const int cg = p.C / V;
  const long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  const long long total = (long long)p.N * 4 * p.H * p.W * cg;
  if (i >= total) return;
  const int g = (int)(i % cg);
  const long long pix = i / cg;
  const int OW = 2 * p.W, OH = 2 * p.H;
  const int n = (int)(pix / ((long long)OH * OW));
  const int rem = (int)(pix - (long long)n * OH * OW);
  const int oh = rem / OW, ow = rem - (rem / OW) * OW;
  const T* src = reinterpret_cast<const T*>(p.x) + (((long long)n * p.H + (oh >> 1)) * p.W + (ow >> 1)) * p.xcs + g * V;
  T* dst = reinterpret_cast<T*>(p.y) + pix * p.ycs + g * V;
  *reinterpret_cast<f32x4*>(dst) = *reinterpret_cast<const f32x4*>(src);
}

hipError_t upsample2_launch(int f32, const UpsampleParams& p, hipStream_t s) {
  const int V = f32 ? 4 : 8;
  if (p.C % V || p.xcs % V || p.ycs % V) return hipErrorInvalidValue;
  const long long total = (long long)p.N * 4 * p.H * p.W * (p.C / V);
  dim3 grid((unsigned)((total + 255) / 256));
  if (f32) hipLaunchKernelGGL(upsample2_nhwc<float>, grid, dim3(256), 0, s, p);
  else hipLaunchKernelGGL(upsample2_nhwc<f16>, grid, dim3(256), 0, s, p);
  return hipGetLastError();
}

// ---------------------------------------------------------------------------
struct LayerNormParams {
  const void* x; int xcs;
  void* y; int ycs;
  int M;               // tokens (all images)
  int C;               // normalised channels (true)
  int cwrite;          // channels written (>= C, the tail is zero)
  const float* gamma;  // [C]
  const float* beta;   // [C]
  const float* add;    // [rows][C] or null
  int rows;            // tokens per image (add table rows)
  float eps;
};

constexpr int LN_MAXV = 32;   // C <= 64 * 32 = 2048
constexpr int LN_NIT = 8;     // 16-byte vectors per lane: C <= 8 * 64 * (16 / sizeof(T))

__device__ __forceinline__ void ln_unpack(const f32x4& r, float* o) { o[0] = r[0]; o[1] = r[1]; o[2] = r[2]; o[3] = r[3]; }
__device__ __forceinline__ void ln_unpack(const f16x8& r, float* o) {
#pragma unroll
  for (int i = 0; i < 8; ++i) o[i] = (float)r[i];
}

// One wave per token, every lane holding whole 16-byte vectors of the row (vector vi at
// lane + 64 k): one coalesced load per vector, f32 statistics by wave reduction, one 16-byte
// store per vector. The first version kept a 32-entry per-channel array with per-entry
// bounds checks; the compiler hoisted 32 sets of addresses and spilled ~6200 VGPRs to
// scratch (1.5 ms per ViT-L layernorm of 32 crops instead of ~15 us).
template <typename T>
__global__ __launch_bounds__(256) void layernorm_vec(LayerNormParams p) {
  constexpr int V = 16 / sizeof(T);
  using VT = typename std::conditional<sizeof(T) == 4, f32x4, f16x8>::type;
  const int lane = threadIdx.x & 63;
  const int tok = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (tok >= p.M) return;
  const int nv = p.C / V;
  const T* xr = reinterpret_cast<const T*>(p.x) + (size_t)tok * p.xcs;
  const float* ar = p.add ? p.add + (size_t)(tok % p.rows) * p.C : nullptr;
  float v[LN_NIT][V];
  float s = 0.f;
#pragma unroll
  for (int k = 0; k < LN_NIT; ++k) {
    const int vi = lane + 64 * k;
#pragma unroll
    for (int i = 0; i < V; ++i) v[k][i] = 0.f;
    if (vi < nv) {
      ln_unpack(*reinterpret_cast<const VT*>(xr + vi * V), v[k]);
      if (ar) {
#pragma unroll
        for (int i = 0; i < V; i += 4) {
          const f32x4 t = *reinterpret_cast<const f32x4*>(ar + vi * V + i);
          v[k][i] += t[0]; v[k][i + 1] += t[1]; v[k][i + 2] += t[2]; v[k][i + 3] += t[3];
        }
      }
#pragma unroll
      for (int i = 0; i < V; ++i) s += v[k][i];
    }
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) s += __shfl_xor(s, o);
  const float mean = s / (float)p.C;
  float q = 0.f;
#pragma unroll
  for (int k = 0; k < LN_NIT; ++k) {
    if (lane + 64 * k < nv) {
#pragma unroll
      for (int i = 0; i < V; ++i) { const float d = v[k][i] - mean; q += d * d; }
    }
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) q += __shfl_xor(q, o);
  const float rstd = 1.0f / sqrtf(q / (float)p.C + p.eps);
  T* yr = reinterpret_cast<T*>(p.y) + (size_t)tok * p.ycs;
#pragma unroll
  for (int k = 0; k < LN_NIT; ++k) {
    const int vi = lane + 64 * k;
    if (vi < nv) {
      VT o;
#pragma unroll
      for (int i = 0; i < V; i += 4) {
        const f32x4 g = *reinterpret_cast<const f32x4*>(p.gamma + vi * V + i);
        const f32x4 b = *reinterpret_cast<const f32x4*>(p.beta + vi * V + i);
#pragma unroll
        for (int j = 0; j < 4; ++j) o[i + j] = (T)((v[k][i + j] - mean) * rstd * g[j] + b[j]);
      }
      *reinterpret_cast<VT*>(yr + vi * V) = o;
    }
  }
  for (int c = p.C + lane; c < p.cwrite; c += 64) yr[c] = (T)0.f;
}

// Any shape (rows not 16-byte aligned): two passes over the row from memory (L2), no
// per-lane arrays.
template <typename T>
__global__ __launch_bounds__(256) void layernorm_rows(LayerNormParams p) {
  const int lane = threadIdx.x & 63;
  const int tok = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (tok >= p.M) return;
  const T* xr = reinterpret_cast<const T*>(p.x) + (size_t)tok * p.xcs;
  const float* ar = p.add ? p.add + (size_t)(tok % p.rows) * p.C : nullptr;
  float s = 0.f;
  for (int c = lane; c < p.C; c += 64) s += (float)xr[c] + (ar ? ar[c] : 0.f);
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) s += __shfl_xor(s, o);
  const float mean = s / (float)p.C;
  float q = 0.f;
  for (int c = lane; c < p.C; c += 64) {
    const float d = (float)xr[c] + (ar ? ar[c] : 0.f) - mean;
    q += d * d;
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) q += __shfl_xor(q, o);
  const float rstd = 1.0f / sqrtf(q / (float)p.C + p.eps);
  T* yr = reinterpret_cast<T*>(p.y) + (size_t)tok * p.ycs;
  for (int c = lane; c < p.cwrite; c += 64)
    yr[c] = c < p.C ? (T)(((float)xr[c] + (ar ? ar[c] : 0.f) - mean) * rstd * p.gamma[c] + p.beta[c]) : (T)0.f;
}

hipError_t layernorm_launch(int f32, const LayerNormParams& p, hipStream_t s) {
  if (p.C > 64 * LN_MAXV || p.cwrite > 64 * LN_MAXV || p.M <= 0) return hipErrorInvalidValue;
  dim3 grid((unsigned)((p.M + 3) / 4));
  const int V = f32 ? 4 : 8;
  // the in-place case (y == x) is safe for both kernels: a wave reads its whole row before writing it
  const bool vec = p.C % V == 0 && p.xcs % V == 0 && p.ycs % V == 0 && p.C / V <= 64 * LN_NIT &&
                   (reinterpret_cast<uintptr_t>(p.x) % 16) == 0 && (reinterpret_cast<uintptr_t>(p.y) % 16) == 0 &&
                   (reinterpret_cast<uintptr_t>(p.gamma) % 16) == 0 && (reinterpret_cast<uintptr_t>(p.beta) % 16) == 0 &&
                   (!p.add || (reinterpret_cast<uintptr_t>(p.add) % 16) == 0);
  if (vec) {
    if (f32) hipLaunchKernelGGL(layernorm_vec<float>, grid, dim3(256), 0, s, p);
    else hipLaunchKernelGGL(layernorm_vec<f16>, grid, dim3(256), 0, s, p);
  } else {
    if (f32) hipLaunchKernelGGL(layernorm_rows<float>, grid, dim3(256), 0, s, p);
    else hipLaunchKernelGGL(layernorm_rows<f16>, grid, dim3(256), 0, s, p);
  }
  return hipGetLastError();
}

// ---------------------------------------------------------------------------
struct AttnParams {
  const void* qkv; int qcs;   // [N][T][qcs]: q at 0, k at E, v at 2E (E = heads*64)
  void* out; int ocs;         // [N][T][ocs]
  int N, T, heads;
  float scale;                // 1/sqrt(head_dim)
};

constexpr int ATT_D = 64;         // head dim
constexpr int ATT_Q = 64;         // queries per workgroup (one per lane)
constexpr int ATT_WAVES = 4;      // waves split the keys
constexpr int ATT_TMAX = 272;     // max tokens staged in LDS (257 for ViT-L/14 @ 224)
constexpr int ATT_CHUNK = 16;     // keys scored per online-softmax update

template <typename T>
__global__ __launch_bounds__(256) void mha_tokens(AttnParams p) {
  constexpr int KV_BYTES = 2 * ATT_TMAX * ATT_D * (int)sizeof(T);
  constexpr int CMB_BYTES = ATT_WAVES * ATT_Q * (ATT_D + 2) * 4;
  constexpr int SMEM = KV_BYTES > CMB_BYTES ? KV_BYTES : CMB_BYTES;
  __shared__ __attribute__((aligned(16))) char smem[SMEM];
  T* Ks = reinterpret_cast<T*>(smem);
  T* Vs = Ks + ATT_TMAX * ATT_D;
  const int nqb = (p.T + ATT_Q - 1) / ATT_Q;
  const int qb = blockIdx.x % nqb;
  const int h = (blockIdx.x / nqb) % p.heads;
  const int n = blockIdx.x / (nqb * p.heads);
  const int E = p.heads * ATT_D;
  const T* base = reinterpret_cast<const T*>(p.qkv) + (long long)n * p.T * p.qcs;
  // stage K and V of this head (16-byte vectors)
  constexpr int VE = 16 / sizeof(T);
  for (int i = threadIdx.x; i < p.T * (ATT_D / VE); i += blockDim.x) {
    const int t = i / (ATT_D / VE), c = (i % (ATT_D / VE)) * VE;
    const T* row = base + (long long)t * p.qcs + h * ATT_D + c;
    *reinterpret_cast<f32x4*>(Ks + t * ATT_D + c) = *reinterpret_cast<const f32x4*>(row + E);
    *reinterpret_cast<f32x4*>(Vs + t * ATT_D + c) = *reinterpret_cast<const f32x4*>(row + 2 * E);
  }
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int qi = qb * ATT_Q + lane;
  const bool qok = qi < p.T;
  float q[ATT_D];
  {
    const T* qr = base + (long long)(qok ? qi : 0) * p.qcs + h * ATT_D;
#pragma unroll
    for (int c = 0; c < ATT_D; ++c) q[c] = (float)qr[c] * p.scale;
  }
  __syncthreads();
  // this wave's key range
  const int per = (p.T + ATT_WAVES - 1) / ATT_WAVES;
  const int k0 = wave * per, k1 = min(p.T, k0 + per);
  float m = -INFINITY, l = 0.f;
  float acc[ATT_D];
#pragma unroll
  for (int c = 0; c < ATT_D; ++c) acc[c] = 0.f;
  for (int kc = k0; kc < k1; kc += ATT_CHUNK) {
    float sc[ATT_CHUNK];
    float cm = -INFINITY;
#pragma unroll
    for (int j = 0; j < ATT_CHUNK; ++j) {
      const int t = kc + j;
      float sdot = -INFINITY;
      if (t < k1) {
        const T* kr = Ks + t * ATT_D;
        sdot = 0.f;
#pragma unroll
        for (int c = 0; c < ATT_D; ++c) sdot += q[c] * (float)kr[c];
      }
      sc[j] = sdot;
      cm = fmaxf(cm, sdot);
    }
    const float mn = fmaxf(m, cm);
    const float corr = __expf(m - mn);   // m = -inf on the first chunk: corr = 0
    l *= corr;
#pragma unroll
    for (int c = 0; c < ATT_D; ++c) acc[c] *= corr;
#pragma unroll
    for (int j = 0; j < ATT_CHUNK; ++j) {
      const int t = kc + j;
      if (t < k1) {
        const float e = __expf(sc[j] - mn);
        l += e;
        const T* vr = Vs + t * ATT_D;
#pragma unroll
        for (int c = 0; c < ATT_D; ++c) acc[c] += e * (float)vr[c];
      }
    }
    m = mn;
  }
  __syncthreads();   // K/V no longer read: reuse the LDS for the combine
  float* cmb = reinterpret_cast<float*>(smem);   // [wave][query][D + 2]
  {
    float* r = cmb + (wave * ATT_Q + lane) * (ATT_D + 2);
    r[0] = m;
    r[1] = l;
#pragma unroll
    for (int c = 0; c < ATT_D; ++c) r[2 + c] = acc[c];
  }
  __syncthreads();
  if (!qok) return;
  // wave w finishes dims [16w, 16w+16) of every query of the block
  float mw[ATT_WAVES], M = -INFINITY;
#pragma unroll
  for (int w = 0; w < ATT_WAVES; ++w) {
    mw[w] = cmb[(w * ATT_Q + lane) * (ATT_D + 2)];
    M = fmaxf(M, mw[w]);
  }
  float L = 0.f, f[ATT_WAVES];
#pragma unroll
  for (int w = 0; w < ATT_WAVES; ++w) {
    f[w] = mw[w] == -INFINITY ? 0.f : __expf(mw[w] - M);
    L += cmb[(w * ATT_Q + lane) * (ATT_D + 2) + 1] * f[w];
  }
  const float inv = 1.0f / L;
  T* orow = reinterpret_cast<T*>(p.out) + ((long long)n * p.T + qi) * p.ocs + h * ATT_D;
  constexpr int DW = ATT_D / ATT_WAVES;
#pragma unroll
  for (int c = 0; c < DW; ++c) {
    const int d = wave * DW + c;
    float v = 0.f;
#pragma unroll
    for (int w = 0; w < ATT_WAVES; ++w) v += cmb[(w * ATT_Q + lane) * (ATT_D + 2) + 2 + d] * f[w];
    orow[d] = (T)(v * inv);
  }
}

hipError_t attention_launch(int f32, const AttnParams& p, int head_dim, hipStream_t s) {
  if (head_dim != ATT_D || p.T > ATT_TMAX || p.T <= 0 || p.qcs % 8 || p.heads <= 0) return hipErrorInvalidValue;
  const int nqb = (p.T + ATT_Q - 1) / ATT_Q;
  dim3 grid((unsigned)(p.N * p.heads * nqb));
  if (f32) hipLaunchKernelGGL(mha_tokens<float>, grid, dim3(64 * ATT_WAVES), 0, s, p);
  else hipLaunchKernelGGL(mha_tokens<f16>, grid, dim3(64 * ATT_WAVES), 0, s, p);
  return hipGetLastError();
}

// ---------------------------------------------------------------------------
// Largest |x| of the first C channels of npix f16 pixels at pixel stride cs (the hi half of a split
// / f16c8 tensor): f16c8 scale calibration (pc_net_calibrate). Non-negative floats order like
// their bit patterns, so the per-wave maxima meet in one unsigned atomicMax.
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(256) void absmax_f16(const f16* __restrict__ x, long long npix, int C, int cs,
                                                  unsigned* __restrict__ out) {
  const int c8 = C / 8;
  const long long n = npix * c8;
  float m = 0.f;
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (long long)gridDim.x * blockDim.x) {
    const long long pix = i / c8;
    const int cq = (int)(i - pix * c8);
    const f16x8 v = *reinterpret_cast<const f16x8*>(x + pix * cs + cq * 8);
#pragma unroll
    for (int j = 0; j < 8; ++j) m = fmaxf(m, fabsf((float)v[j]));
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) m = fmaxf(m, __shfl_xor(m, o));
  if ((threadIdx.x & 63) == 0) atomicMax(out, __float_as_uint(m));
}

hipError_t absmax_f16_launch(const void* x, long long npix, int C, int cs, unsigned* out, hipStream_t s) {
  if (C % 8 || cs % 8 || npix <= 0) return hipErrorInvalidValue;
  const long long n = npix * (C / 8);
  const int grid = (int)std::min<long long>(2048, (n + 255) / 256);
  hipLaunchKernelGGL(absmax_f16, dim3(grid), dim3(256), 0, s, reinterpret_cast<const f16*>(x), npix, C, cs, out);
  return hipGetLastError();
}

}  // namespace pc
