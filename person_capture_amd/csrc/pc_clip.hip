// OpenCLIP image preprocessing for ReIDEmbedder (gfx950).
//
// Restates the transform the reference applies per crop (reid_embedder.py:46-50:
// cv2.cvtColor(BGR2RGB) -> PIL.Image -> open_clip preprocess), i.e. [ext]
// open_clip_torch==3.2.0 image_transform(224, resize_mode='shortest', bicubic):
//   torchvision Resize(224) on a PIL image = Pillow Image.resize(BICUBIC): separable
//     two-pass resample, 22-bit fixed-point coefficients, u8 intermediate;
//   CenterCrop(224); ToTensor (/255); Normalize(OPENAI mean/std);
// and writes the ViT-L/14 patch matrix directly: token 1 + (y/14)*16 + x/14, column
// ((y%14)*14 + x%14)*3 + c (the conv1 weight's [kh][kw][c] order), token 0 (class
// token slot) and the K padding 588..607 zero.
// Coefficient tables are computed on the host exactly as Pillow's precompute_coeffs /
// normalize_coeffs_8bpc do (pc_host.cpp); both passes here are integer-exact, so the
// pixels equal Pillow's. Parity: tests/test_gpu_reid.py against PIL itself.
#include "pc_common.h"

#pragma clang fp contract(off)

namespace pc {

struct ClipPrepDesc {
  const uint8_t* src;     // BGR u8 crop (top-left), row_stride bytes per row
  int H, W, row_stride;
  int kh, kv;             // horizontal / vertical coefficient counts per output
  const int* hb;          // [224][2] (xmin, xcount) of the cropped output columns
  const int* hk;          // [224][kh] int32 Q22 weights
  const int* vb;          // [224][2] (ymin, ycount) of the cropped output rows, ymin relative to row0
  const int* vk;          // [224][kv]
  int row0, nrows;        // source rows the vertical pass reads: [row0, row0 + nrows)
  uint8_t* tmp;           // [nrows][224][3] horizontal-pass output
};

constexpr int CLIP_SIDE = 224;
constexpr int CLIP_PATCH = 14;
constexpr int CLIP_GRID = 16;
constexpr int CLIP_TOK = 257;
constexpr int CLIP_K = 588;
constexpr int CLIP_KPAD = 608;

__device__ __forceinline__ int clip8(int v) {
  v >>= 22;
  return v < 0 ? 0 : (v > 255 ? 255 : v);
}

// pass 1: rows [row0, row0+nrows) x the 224 cropped output columns
__global__ void clip_hpass(const ClipPrepDesc* __restrict__ descs) {
  const ClipPrepDesc d = descs[blockIdx.y];
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= d.nrows * CLIP_SIDE) return;
  const int r = i / CLIP_SIDE, x = i - (i / CLIP_SIDE) * CLIP_SIDE;
  const int xmin = d.hb[2 * x], xn = d.hb[2 * x + 1];
  const int* k = d.hk + x * d.kh;
  const uint8_t* row = d.src + (long long)(d.row0 + r) * d.row_stride;
  int s0 = 1 << 21, s1 = 1 << 21, s2 = 1 << 21;
  for (int j = 0; j < xn; ++j) {
    const uint8_t* px = row + (xmin + j) * 3;
    s0 += (int)px[0] * k[j];
    s1 += (int)px[1] * k[j];
    s2 += (int)px[2] * k[j];
  }
  uint8_t* o = d.tmp + (long long)i * 3;
  o[0] = (uint8_t)clip8(s0);
  o[1] = (uint8_t)clip8(s1);
  o[2] = (uint8_t)clip8(s2);
}

// pass 2: vertical resample + ToTensor + Normalize, scattered into the patch matrix
template <typename T>
__global__ void clip_vpass_patch(const ClipPrepDesc* __restrict__ descs, T* __restrict__ out) {
  const int n = blockIdx.y;
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= CLIP_TOK * CLIP_KPAD) return;
  const int tok = i / CLIP_KPAD, kc = i - (i / CLIP_KPAD) * CLIP_KPAD;
  T* o = out + (long long)n * CLIP_TOK * CLIP_KPAD + i;
  if (tok == 0 || kc >= CLIP_K) { *o = (T)0.f; return; }
  const int pt = tok - 1, py = pt / CLIP_GRID, pxx = pt - (pt / CLIP_GRID) * CLIP_GRID;
  const int tap = kc / 3, c = kc - (kc / 3) * 3;   // c: RGB channel
  const int y = py * CLIP_PATCH + tap / CLIP_PATCH, x = pxx * CLIP_PATCH + tap % CLIP_PATCH;
  const ClipPrepDesc d = descs[n];
  const int ymin = d.vb[2 * y], yn = d.vb[2 * y + 1];
  const int* k = d.vk + y * d.kv;
  const int bc = 2 - c;   // BGR source channel
  int s = 1 << 21;
  for (int j = 0; j < yn; ++j) s += (int)d.tmp[((long long)(ymin + j) * CLIP_SIDE + x) * 3 + bc] * k[j];
  const float v = (float)clip8(s) / 255.f;
  const float mean = c == 0 ? 0.48145466f : (c == 1 ? 0.4578275f : 0.40821073f);
  const float stdv = c == 0 ? 0.26862954f : (c == 1 ? 0.26130258f : 0.27577711f);
  *o = (T)((v - mean) / stdv);
}

hipError_t clip_prep_launch(int f32, const ClipPrepDesc* d_descs, int N, int max_rows, void* out, hipStream_t s) {
  dim3 g1((max_rows * CLIP_SIDE + 255) / 256, N);
  hipLaunchKernelGGL(clip_hpass, g1, dim3(256), 0, s, d_descs);
  dim3 g2((CLIP_TOK * CLIP_KPAD + 255) / 256, N);
  if (f32) hipLaunchKernelGGL(clip_vpass_patch<float>, g2, dim3(256), 0, s, d_descs, (float*)out);
  else hipLaunchKernelGGL(clip_vpass_patch<f16>, g2, dim3(256), 0, s, d_descs, (f16*)out);
  return hipGetLastError();
}

}  // namespace pc
