// C-ABI layer (include/pcgpu.h): contexts, the network executor and the
// domain entry points of the identity hot path. Compiled by hipcc for gfx950.
//
// A network arrives as a serialized "program" (person_capture_amd/netdef.py):
// buffers, NHWC tensor views, float arrays and a flat op list (CONV / STEM /
// MAXPOOL). The executor resolves views to device pointers for the run's batch,
// picks a conv tile per layer and launches the kernels of pc_conv.hip in order on
// the context stream; optionally the whole run is captured into a HIP graph.
#include <hip/hip_runtime.h>
#include <string.h>
#include <stdio.h>
#include <stdlib.h>
#include <string>
#include <vector>
#include <map>
#include <algorithm>
#include <thread>
#include <mutex>
#include <memory>
#include <cmath>
#include <atomic>
#include <condition_variable>
#include <functional>
#include <system_error>
#include "../../include/pcgpu.h"
#include "pc_common.h"

namespace pc {
hipError_t conv_launch(int f32, int rowb, int cfg, const ConvParams& p, hipStream_t s);
hipError_t conv_halo_launch(int f32, int cfg, const ConvParams& p, hipStream_t s);
hipError_t conv_fast_launch(int f32, int rowb, int cfg, const ConvParams& p, hipStream_t s);
hipError_t conv_hx_launch(const ConvParams& p, hipStream_t s);
hipError_t conv_hxg_launch(const ConvParams& p, int small, hipStream_t s);
hipError_t conv_hxi_launch(const ConvParams& p, int small, hipStream_t s);
int conv_fast_num_cfgs();
constexpr int kFastSmallCfg0 = 15, kFastSmallCfg1 = 19;   // conv_fast tiles 15..19: small-batch plans only
int conv_fast_tile(int cfg, int* bc, int* bp);
int conv_fast_valid(int cfg, int rowb);
int conv_fast_valid_sx(int cfg, int rowb);
int conv_fast_valid_c8(int cfg, int rowb);
int conv_fast_valid_wg(int cfg);
int conv_halo_num_cfgs();
int conv_halo_tile(int cfg, int* bc, int* bp);
int conv_halo_fits(int cfg, int KH, int KW, int W);
hipError_t conv_t2d_launch(const ConvParams& p, int variant, hipStream_t s);
int conv_t2d_select(int cin, int npad, int KH, int KW, int stride, int pad, int act, int out_f32, int ycs,
                    int ycoff, int split);
int conv_t2d_rows(int variant);
int conv_chain_fits(int H, int W, int C, int npad, long long ktot);
hipError_t conv_chain_launch(const void* x, int xcs, void* y, int ycs, const void* blk_dev, int nblk, int N, int H,
                             int W, long long ktot, int dbg, hipStream_t s);
size_t conv_chain_block_bytes();
int stem_fused_ok(int f32, int cin, int cin_true, int KH, int KW, int npad, int cwrite, int ycs, int ycoff);
hipError_t stem_fused_launch(const StemParams& p, const void* wpk, const float* bias, const float* slope, int npad,
                             int cwrite, hipStream_t s);
hipError_t splitk_finish_launch(int f32, const ConvParams& p, hipStream_t s);
hipError_t absmax_f16_launch(const void* x, long long npix, int C, int cs, unsigned* out, hipStream_t s);
hipError_t splitk_reduce_launch(int f32, const float* part, int splitk, int M, int npad, int cout, const float* bias,
                                const float* slope, int act, void* y, int ycs, int out_f32, hipStream_t s);
hipError_t stem_launch(int f32, const StemParams& p, hipStream_t s);
hipError_t maxpool_launch(int f32, const PoolParams& p, hipStream_t s);
hipError_t stem_im2col_launch(int f32, const StemParams& p, int cin_true, void* col, hipStream_t s);
struct LetterboxDesc;
struct WarpDesc;
struct AreaTab;
struct ResizeDesc;
hipError_t resize_linear_launch(const ResizeDesc* d_descs, int N, int max_pixels, hipStream_t s);
hipError_t letterbox_launch(int f32, const LetterboxDesc* d_descs, int N, int D, void* out, hipStream_t s);
hipError_t warp_launch(const WarpDesc* d_descs, int N, int max_pixels, hipStream_t s);
hipError_t quality_launch(const uint8_t* chips, int N, int side, double* out, hipStream_t s);
hipError_t arcprep_launch(int mode, const uint8_t* chips, int N, int side, int flip, void* out, hipStream_t s);
hipError_t rotate_pad_launch(const uint8_t* src, int H, int W, int row_stride, int deg, int pad, uint8_t* dst, int OH,
                             int OW, hipStream_t s);
hipError_t resize_area_fast_launch(const uint8_t* src, int row_stride, int isx, int isy, uint8_t* dst, int OH, int OW,
                                   hipStream_t s);
hipError_t resize_area_launch(const uint8_t* src, int row_stride, const AreaTab* xtab, const int* xstart,
                              const AreaTab* ytab, const int* ystart, uint8_t* dst, int OH, int OW, hipStream_t s);
hipError_t resize_area_rows_launch(const void* jobs, int n, int row_stride, const AreaTab* xtab, const int* xstart,
                                  const AreaTab* ytab, const int* ystart, int OH, int OW, int span_bytes,
                                  hipStream_t s);
hipError_t embed_finalize_launch(const float* e, int ld, int n, int dim, int flip, float* out, hipStream_t s);
hipError_t bank_match_launch(const float* q, int n, const float* bank, int B, int dim, float* fd, int* idx,
                             hipStream_t s);
struct DecodeLevel {
  const float* out;
  int H, W, cs, stride;
  int loc_offset;
  int anchor_offset;
};
struct DecodeParams {
  DecodeLevel lv[3];
  int nlv;
  int total_loc;
  float thresh;
  const float* det_scale;
  float* cand;
  int* count;
  int cap;
};
hipError_t scrfd_decode_launch(const DecodeParams& p, int N, hipStream_t s);
hipError_t scrfd_nms_big_launch(const float* cand, const int* count, int cap, int pcap, unsigned long long* keys,
                                int* slot_of, float* kept, float nms_thresh, int max_det, float* dets, float* kps,
                                int* nkeep, int N, hipStream_t s);
hipError_t scrfd_nms_launch(const float* cand, const int* count, int cap, float nms_thresh, int max_det, float* dets,
                            float* kps, int* nkeep, int N, hipStream_t s);
hipError_t embed_l2_launch(const float* e, int ld, int n, int dim, float eps, float* out, hipStream_t s);
// pc_ops.hip
struct UpsampleParams { const void* x; int N, H, W, C, xcs; void* y; int ycs; };
hipError_t upsample2_launch(int f32, const UpsampleParams& p, hipStream_t s);
struct LayerNormParams {
  const void* x; int xcs; void* y; int ycs; int M, C, cwrite;
  const float* gamma; const float* beta; const float* add; int rows; float eps;
};
hipError_t layernorm_launch(int f32, const LayerNormParams& p, hipStream_t s);
struct AttnParams { const void* qkv; int qcs; void* out; int ocs; int N, T, heads; float scale; };
hipError_t attention_launch(int f32, const AttnParams& p, int head_dim, hipStream_t s);
// pc_yolo.hip
struct YoloLetterboxDesc;
hipError_t yolo_letterbox_launch(int f32, const YoloLetterboxDesc* d_descs, int N, int Hp, int Wp, void* out,
                                 hipStream_t s);
struct YoloLevel { const float* out; int H, W, cs, stride; int loc_offset; };
struct YoloDecodeParams { YoloLevel lv[3]; int nlv, total, nc; float conf; float* cand; int* count; int cap; };
struct YoloScale;
hipError_t yolo_decode_launch(const YoloDecodeParams& p, int N, hipStream_t s);
struct YoloKptScale;
hipError_t yolo_nms_big_launch(const float* cand, const int* count, int cap, int pcap, unsigned long long* keys,
                               int* slot_of, float* kept, float iou, int max_det, const YoloScale* sc, float* dets,
                               int* nkeep, int* keep_anchor, int N, hipStream_t s);
hipError_t yolo_kpts_launch(const YoloDecodeParams& p, int nk, int koff, int max_det, const int* nkeep,
                            const int* keep_anchor, const YoloScale* sc, const YoloKptScale* ksc, float* kpts, int N,
                            hipStream_t s);
hipError_t yolo_nms_launch(const float* cand, const int* count, int cap, float iou, int max_det, const YoloScale* sc,
                           float* dets, int* nkeep, int N, hipStream_t s, int* keep_anchor = nullptr);
// pc_clip.hip
struct ClipPrepDesc {
  const uint8_t* src; int H, W, row_stride; int kh, kv;
  const int* hb; const int* hk; const int* vb; const int* vk; int row0, nrows; uint8_t* tmp;
};
hipError_t clip_prep_launch(int f32, const ClipPrepDesc* d_descs, int N, int max_rows, void* out, hipStream_t s);
}  // namespace pc

using namespace pc;

static_assert(sizeof(pc_letterbox_desc) == 56, "letterbox desc layout");
static_assert(sizeof(pc_warp_desc) == 96, "warp desc layout");
static_assert(sizeof(pc_area_tab) == 12, "area tab layout");
static_assert(sizeof(pc_resize_desc) == 80, "resize desc layout");
static_assert(sizeof(pc_yolo_letterbox_desc) == 64, "yolo letterbox desc layout");
static_assert(sizeof(pc_yolo_scale) == 20, "yolo scale layout");

// Persistent host workers for pc_frame_stage: a frame is packed into pinned memory in row
// chunks taken in order by the workers, and the caller's thread issues each chunk's H2D as soon
// as it is packed, so the copy engine runs behind the packing instead of after it (r04: the
// 6.2 MB of a 1080p frame cost ~0.3 ms of packing with per-call threads, then the H2D).
// One frame's packing job: chunks are taken from `next`; done[c] and active are guarded by the pool's
// mutex. A job lives until its last holder drops it; the caller waits for active == 0 before its
// frame (which the job's function refers to) goes out of scope.
struct StageJob {
  std::function<void(int)> fn;
  int nchunks = 0;
  std::atomic<int> next{0};
  std::vector<char> done;
  int active = 0;                    // workers inside fn
};

// Persistent packing workers of pc_frame_stage. A worker takes the current job under the lock (a
// snapshot: the job's function, chunk count and counters belong to that frame alone), works it
// without the lock, and never sees another frame's job in between - a late wake-up finds either no
// job or the next frame's, whose state is its own object (the shared job / nchunks
// fields were re-assigned while a late worker still read them).
struct StagePool {
  std::vector<std::thread> th;
  std::mutex mu;
  std::condition_variable cv;        // workers: a new job
  std::condition_variable done_cv;   // caller: a chunk finished / a worker left the job
  std::shared_ptr<StageJob> cur;     // the frame being packed (guarded by mu)
  unsigned gen = 0;                  // bumped per job (guarded by mu)
  bool stop = false;
  void start(int n) {
    for (int i = 0; i < n; ++i) {
      try {
        th.emplace_back([this] { loop(); });
      } catch (const std::system_error&) {
        break;   // fewer workers: the caller packs what nobody takes
      }
    }
  }
  void loop() {
    unsigned seen = 0;
    std::unique_lock<std::mutex> lk(mu);
    for (;;) {
      cv.wait(lk, [&] { return stop || (cur && gen != seen); });
      if (stop) return;
      seen = gen;
      std::shared_ptr<StageJob> j = cur;
      ++j->active;
      lk.unlock();
      work(*j);
      lk.lock();
      --j->active;
      done_cv.notify_all();
    }
  }
  // take chunks of job j until none is left (the caller runs this too)
  void work(StageJob& j) {
    for (int c; (c = j.next.fetch_add(1)) < j.nchunks;) {
      j.fn(c);
      std::lock_guard<std::mutex> g(mu);
      j.done[c] = 1;
      done_cv.notify_all();
    }
  }
  ~StagePool() {
    {
      std::lock_guard<std::mutex> g(mu);
      stop = true;
    }
    cv.notify_all();
    for (auto& t : th) t.join();
  }
};

struct pc_ctx {
  int device = 0;
  hipStream_t stream = nullptr;
  hipStream_t own_stream = nullptr;
  std::string err;
  void* zero = nullptr;
  // staging ring for small per-call descriptor arrays (pinned host -> device)
  char* stage_h = nullptr;
  char* stage_d = nullptr;
  size_t stage_cap = 0, stage_off = 0;
  // detection scratch
  float* cand = nullptr;
  int* cand_count = nullptr;
  float* det_scale = nullptr;
  size_t cand_bytes = 0;
  size_t cand_images = 0;     // images cand_count / det_scale hold
  // large-candidate NMS scratch (scrfd_nms_big): sort keys, anchor -> slot map, kept boxes
  void* nms_big = nullptr;
  size_t nms_big_bytes = 0;
  // YOLO candidates
  float* ycand = nullptr;
  int* ycount = nullptr;
  size_t ycand_images = 0;
  int ycand_cap = 0;
  void* ybig = nullptr;        // global-memory NMS: keys, slot map, kept boxes
  size_t ybig_bytes = 0;
  int* ykeep = nullptr;        // pose: anchor index of every kept box
  size_t ykeep_bytes = 0;
  // CLIP preprocessing tables + horizontal-pass scratch
  void* clip_tmp = nullptr;
  size_t clip_tmp_bytes = 0;
  // host frame staging (pc_frame_stage): ring of pinned slots, each reused once the H2D
  // that last read it has completed
  struct FrameSlot { char* h = nullptr; size_t cap = 0; hipEvent_t ev = nullptr; bool pending = false; };
  FrameSlot fslots[4];
  int fslot_next = 0;
  std::mutex fslot_mu;   // one context may be shared by FaceEmbedders on several host threads
  StagePool* pool = nullptr;   // created on the first multi-threaded pc_frame_stage
};

static int fail(pc_ctx* c, int code, const std::string& msg) {
  if (c) c->err = msg;
  return code;
}

#define HIPCHK(ctx, expr)                                                                     \
  do {                                                                                        \
    hipError_t _e = (expr);                                                                   \
    if (_e != hipSuccess)                                                                     \
      return fail((ctx), PC_ERR_HIP, std::string(#expr) + ": " + hipGetErrorString(_e));      \
  } while (0)

static int stage_copy(pc_ctx* c, const void* h, size_t nbytes, void** d_out) {
  const size_t bytes = (nbytes + 255) & ~size_t(255);
  if (bytes > c->stage_cap) {
    // grow the ring (rare: thousands of descriptors in one call); everything staged so
    // far must have been consumed before the old buffers go
    HIPCHK(c, hipStreamSynchronize(c->stream));
    size_t cap = c->stage_cap;
    while (cap < bytes) cap *= 2;
    char *h = nullptr, *d = nullptr;
    if (hipHostMalloc((void**)&h, cap, hipHostMallocDefault) != hipSuccess) return fail(c, PC_ERR_HIP, "staging grow");
    if (hipMalloc((void**)&d, cap) != hipSuccess) { hipHostFree(h); return fail(c, PC_ERR_HIP, "staging grow"); }
    hipHostFree(c->stage_h);
    hipFree(c->stage_d);
    c->stage_h = h; c->stage_d = d; c->stage_cap = cap; c->stage_off = 0;
  }
  if (c->stage_off + bytes > c->stage_cap) {
    // wrap: everything previously staged must have been consumed
    HIPCHK(c, hipStreamSynchronize(c->stream));
    c->stage_off = 0;
  }
  memcpy(c->stage_h + c->stage_off, h, nbytes);
  HIPCHK(c, hipMemcpyAsync(c->stage_d + c->stage_off, c->stage_h + c->stage_off, nbytes, hipMemcpyHostToDevice,
                           c->stream));
  *d_out = c->stage_d + c->stage_off;
  c->stage_off += bytes;
  return PC_OK;
}

extern "C" int pc_abi_version(void) { return PC_ABI_VERSION; }

extern "C" int pc_ctx_create(int device_id, pc_ctx** out) {
  if (!out) return PC_ERR_ARG;
  *out = nullptr;
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= 0) return PC_ERR_HIP;
  if (device_id < 0 || device_id >= ndev) return PC_ERR_ARG;
  pc_ctx* c = new pc_ctx();
  c->device = device_id;
  if (hipSetDevice(device_id) != hipSuccess) { delete c; return PC_ERR_HIP; }
  if (hipStreamCreateWithFlags(&c->own_stream, hipStreamNonBlocking) != hipSuccess) { delete c; return PC_ERR_HIP; }
  c->stream = c->own_stream;
  if (hipMalloc(&c->zero, 4096) != hipSuccess || hipMemset(c->zero, 0, 4096) != hipSuccess) { delete c; return PC_ERR_HIP; }
  c->stage_cap = 8u << 20;
  if (hipHostMalloc((void**)&c->stage_h, c->stage_cap, hipHostMallocDefault) != hipSuccess ||
      hipMalloc((void**)&c->stage_d, c->stage_cap) != hipSuccess) {
    delete c;
    return PC_ERR_HIP;
  }
  *out = c;
  return PC_OK;
}

extern "C" int pc_ctx_destroy(pc_ctx* c) {
  if (!c) return PC_OK;
  hipSetDevice(c->device);
  if (c->stream) hipStreamSynchronize(c->stream);
  if (c->zero) hipFree(c->zero);
  if (c->stage_h) hipHostFree(c->stage_h);
  if (c->stage_d) hipFree(c->stage_d);
  if (c->cand) hipFree(c->cand);
  if (c->cand_count) hipFree(c->cand_count);
  if (c->nms_big) hipFree(c->nms_big);
  if (c->det_scale) hipFree(c->det_scale);
  if (c->ycand) hipFree(c->ycand);
  if (c->ykeep) hipFree(c->ykeep);
  if (c->ybig) hipFree(c->ybig);
  if (c->ycount) hipFree(c->ycount);
  if (c->clip_tmp) hipFree(c->clip_tmp);
  delete c->pool;
  for (auto& fs : c->fslots) {
    if (fs.h) hipHostFree(fs.h);
    if (fs.ev) hipEventDestroy(fs.ev);
  }
  if (c->own_stream) hipStreamDestroy(c->own_stream);
  delete c;
  return PC_OK;
}

extern "C" const char* pc_last_error(const pc_ctx* c) { return c ? c->err.c_str() : "null context"; }

extern "C" int pc_ctx_set_stream(pc_ctx* c, void* s) {
  if (!c) return PC_ERR_ARG;
  c->stream = s ? (hipStream_t)s : c->own_stream;
  return PC_OK;
}
extern "C" void* pc_ctx_stream(pc_ctx* c) { return c ? (void*)c->stream : nullptr; }
// Re-create the context-owned stream at a scheduling priority (HIP convention: lower =
// higher priority; clamped to hipDeviceGetStreamPriorityRange). Work already queued on the
// old stream is drained first.
extern "C" int pc_ctx_set_priority(pc_ctx* c, int priority) {
  if (!c) return PC_ERR_ARG;
  int least = 0, greatest = 0;
  HIPCHK(c, hipDeviceGetStreamPriorityRange(&least, &greatest));
  const int p = priority < greatest ? greatest : (priority > least ? least : priority);
  hipStream_t s = nullptr;
  HIPCHK(c, hipStreamCreateWithPriority(&s, hipStreamNonBlocking, p));
  HIPCHK(c, hipStreamSynchronize(c->own_stream));
  const bool own = c->stream == c->own_stream;
  hipStreamDestroy(c->own_stream);
  c->own_stream = s;
  if (own) c->stream = s;
  return PC_OK;
}
extern "C" int pc_ctx_sync(pc_ctx* c) {
  if (!c) return PC_ERR_ARG;
  HIPCHK(c, hipStreamSynchronize(c->stream));
  return PC_OK;
}
extern "C" int pc_device_alloc(pc_ctx* c, size_t bytes, void** d) {
  if (!c || !d) return PC_ERR_ARG;
  HIPCHK(c, hipSetDevice(c->device));
  HIPCHK(c, hipMalloc(d, bytes ? bytes : 16));
  return PC_OK;
}
extern "C" int pc_device_free(pc_ctx* c, void* d) {
  if (!c) return PC_ERR_ARG;
  if (d) HIPCHK(c, hipFree(d));
  return PC_OK;
}
extern "C" int pc_host_alloc(pc_ctx* c, size_t bytes, void** h) {
  if (!c || !h) return PC_ERR_ARG;
  HIPCHK(c, hipSetDevice(c->device));
  HIPCHK(c, hipHostMalloc(h, bytes ? bytes : 16, hipHostMallocDefault));
  return PC_OK;
}
extern "C" int pc_host_free(pc_ctx* c, void* h) {
  if (!c) return PC_ERR_ARG;
  if (h) HIPCHK(c, hipHostFree(h));
  return PC_OK;
}
extern "C" int pc_fence_create(pc_ctx* c, void** f) {
  if (!c || !f) return PC_ERR_ARG;
  hipEvent_t e = nullptr;
  HIPCHK(c, hipSetDevice(c->device));
  HIPCHK(c, hipEventCreateWithFlags(&e, hipEventDisableTiming));
  *f = (void*)e;
  return PC_OK;
}
extern "C" int pc_fence_record(pc_ctx* c, void* f) {
  if (!c || !f) return PC_ERR_ARG;
  HIPCHK(c, hipEventRecord((hipEvent_t)f, c->stream));
  return PC_OK;
}
extern "C" int pc_fence_wait(pc_ctx* c, void* f) {
  if (!c || !f) return PC_ERR_ARG;
  HIPCHK(c, hipEventSynchronize((hipEvent_t)f));
  return PC_OK;
}
extern "C" int pc_fence_destroy(pc_ctx* c, void* f) {
  if (!c) return PC_ERR_ARG;
  if (f) HIPCHK(c, hipEventDestroy((hipEvent_t)f));
  return PC_OK;
}
extern "C" int pc_ctx_wait_fence(pc_ctx* c, void* f) {
  if (!c || !f) return PC_ERR_ARG;
  HIPCHK(c, hipStreamWaitEvent(c->stream, (hipEvent_t)f, 0));
  return PC_OK;
}

// Host frame -> device through the context's ring of pinned slots: the rows (row_bytes each,
// src_stride apart: a numpy slice need not be contiguous) are packed into the slot by up to
// `threads` host threads, then one H2D from the slot is enqueued on the context stream. The
// caller's array is free again when this returns; the device copy completes in stream order.
// A pageable hipMemcpyAsync would stage through the runtime's own bounce buffers in
// ~MB-sized pieces with the calling thread blocked for the whole transfer.
extern "C" int pc_frame_stage(pc_ctx* c, void* d_dst, const void* h_src, size_t row_bytes, size_t rows,
                              size_t src_stride, int threads) {
  if (!c || !d_dst || !h_src || src_stride < row_bytes) return PC_ERR_ARG;
  const size_t n = row_bytes * rows;
  if (!n) return PC_OK;
  std::lock_guard<std::mutex> lock(c->fslot_mu);   // the slot ring and its stream order
  auto& fs = c->fslots[c->fslot_next];
  c->fslot_next = (c->fslot_next + 1) % 4;
  if (fs.pending) HIPCHK(c, hipEventSynchronize(fs.ev));
  fs.pending = false;
  if (fs.cap < n) {
    if (fs.h) hipHostFree(fs.h);
    fs.h = nullptr;
    fs.cap = 0;
    HIPCHK(c, hipSetDevice(c->device));
    HIPCHK(c, hipHostMalloc((void**)&fs.h, n, hipHostMallocDefault));
    fs.cap = n;
  }
  if (!fs.ev) HIPCHK(c, hipEventCreateWithFlags(&fs.ev, hipEventDisableTiming));
  const char* src = (const char*)h_src;
  auto pack = [&](size_t r0, size_t r1) {
    if (src_stride == row_bytes) {
      memcpy(fs.h + r0 * row_bytes, src + r0 * row_bytes, (r1 - r0) * row_bytes);
    } else {
      for (size_t r = r0; r < r1; ++r) memcpy(fs.h + r * row_bytes, src + r * src_stride, row_bytes);
    }
  };
  int nt = std::max(1, std::min(threads, 16));
  if (n < (size_t(2) << 20)) nt = 1;   // below ~2 MB the handoff costs more than it saves
  if (nt == 1) {
    pack(0, rows);
    HIPCHK(c, hipMemcpyAsync(d_dst, fs.h, n, hipMemcpyHostToDevice, c->stream));
  } else {
    if (!c->pool) {
      c->pool = new StagePool();
      c->pool->start(nt - 1);
    }
    StagePool& P = *c->pool;
    // ~512 KB chunks: the first H2D starts after one chunk, the last follows the last pack
    const int nch = (int)std::min<size_t>(64, std::max<size_t>(nt, (n + (512u << 10) - 1) / (512u << 10)));
    const size_t per = (rows + nch - 1) / nch;
    auto job = std::make_shared<StageJob>();
    job->fn = [&](int ch) { pack(std::min(rows, ch * per), std::min(rows, (ch + 1) * per)); };
    job->nchunks = nch;
    job->done.assign(nch, 0);
    {
      std::lock_guard<std::mutex> g(P.mu);
      P.cur = job;
      ++P.gen;
    }
    P.cv.notify_all();
    // issue each chunk's copy in order as soon as it is packed; pack the rest here when the
    // workers are behind (the copies of chunk i overlap the packing of chunks > i)
    hipError_t herr = hipSuccess;
    for (int ch = 0; ch < nch; ++ch) {
      for (;;) {
        {
          std::unique_lock<std::mutex> lk(P.mu);
          if (job->done[ch]) break;
          if (job->next.load() >= nch) {   // everything taken: wait for chunk ch
            P.done_cv.wait(lk, [&] { return job->done[ch] != 0; });
            break;
          }
        }
        const int mine = job->next.fetch_add(1);
        if (mine < nch) {
          job->fn(mine);
          std::lock_guard<std::mutex> g(P.mu);
          job->done[mine] = 1;
        }
      }
      const size_t r0 = std::min(rows, ch * per), r1 = std::min(rows, (ch + 1) * per);
      if (r1 > r0 && herr == hipSuccess)
        herr = hipMemcpyAsync((char*)d_dst + r0 * row_bytes, fs.h + r0 * row_bytes, (r1 - r0) * row_bytes,
                              hipMemcpyHostToDevice, c->stream);
    }
    {   // the job's function refers to this frame: no worker may still be inside it, and none may
        // pick it up later (it stops being the current job)
      std::unique_lock<std::mutex> lk(P.mu);
      P.done_cv.wait(lk, [&] { return job->active == 0; });
      P.cur.reset();
    }
    if (herr != hipSuccess) return fail(c, PC_ERR_HIP, std::string("frame_stage H2D: ") + hipGetErrorString(herr));
  }
  HIPCHK(c, hipEventRecord(fs.ev, c->stream));
  fs.pending = true;
  return PC_OK;
}

extern "C" int pc_copy_h2d(pc_ctx* c, void* d, const void* h, size_t n) {
  if (!c) return PC_ERR_ARG;
  if (n) HIPCHK(c, hipMemcpyAsync(d, h, n, hipMemcpyHostToDevice, c->stream));
  return PC_OK;
}
extern "C" int pc_copy_d2h(pc_ctx* c, void* h, const void* d, size_t n) {
  if (!c) return PC_ERR_ARG;
  if (n) HIPCHK(c, hipMemcpyAsync(h, d, n, hipMemcpyDeviceToHost, c->stream));
  return PC_OK;
}
extern "C" int pc_copy_d2d(pc_ctx* c, void* d, const void* s, size_t n) {
  if (!c) return PC_ERR_ARG;
  if (n) HIPCHK(c, hipMemcpyAsync(d, s, n, hipMemcpyDeviceToDevice, c->stream));
  return PC_OK;
}
extern "C" int pc_copy_2d(pc_ctx* c, void* d_dst, size_t dst_pitch, const void* d_src, size_t src_pitch,
                          size_t width_bytes, size_t rows) {
  if (!c || !d_dst || !d_src || width_bytes > dst_pitch || width_bytes > src_pitch)
    return fail(c, PC_ERR_ARG, "pc_copy_2d: bad arguments");
  if (!width_bytes || !rows) return PC_OK;
  HIPCHK(c, hipMemcpy2DAsync(d_dst, dst_pitch, d_src, src_pitch, width_bytes, rows, hipMemcpyDeviceToDevice,
                             c->stream));
  return PC_OK;
}

extern "C" int pc_memset(pc_ctx* c, void* d, int v, size_t n) {
  if (!c) return PC_ERR_ARG;
  if (n) HIPCHK(c, hipMemsetAsync(d, v, n, c->stream));
  return PC_OK;
}

// ===========================================================================
// network executor
// ===========================================================================
enum { OP_CONV = 1, OP_STEM = 2, OP_MAXPOOL = 3, OP_UPSAMPLE = 4, OP_LAYERNORM = 5, OP_ATTENTION = 6 };

struct NetBuf { long long elems; int is_f32; void* d = nullptr; };
// split: f16x3 tensor (detector precision mode): C physical channels = [hi | lo],
// C / 2 each; the lo half of a pixel is C / 2 elements after its hi half
// c8: f16c8 tensor: split storage whose second half holds, per 32
// channels, the e4m3 bytes [lo8 | hi8]; lo8 = e4m3(lo * 2^e_lo), hi8 = e4m3(hi * 2^e_hi) with
// per-tensor exponents set by pc_net_calibrate (provisional values before it)
struct NetTensor { int buf, H, W, C, cs, coff, is_f32, split; int c8 = 0, e_lo = 15, e_hi = 4; };
struct NetOp { int w[32]; };
// sx: fused f16x3 split tiles on conv_fast (pc_conv_fast.hip SX); c8: its f16c8 form (C8);
// wf8s: E8M0 exponents of the conv's W_hi8 | W_lo8 << 8 bytes (c8 weights)
// wg: the fused f16x3 tile takes its weight fragments from the fragment-ordered copy (pc_net::wfrag)
struct ConvPlan { int rowb, cfg, splitk, halo = -1, fast = -1, t2d = -1, sx = 0, hx = 0, c8 = 0, wf8s = 0, wg = 0; long long M_per_image; double flops_per_image; };
// A stem (tiny Cin) runs as im2col + a 1x1 MFMA conv over 32-element K rows.
struct StemPlan {
  int use_mfma = 0, npad = 0, cfg = 0, rowb = 0, cin_true = 0;
  int split = 0;            // f16x3 output: w is [npad][64] = W_hi | W_lo (fused stem only)
  void* w = nullptr;        // [npad][32] act dtype
  float* bias = nullptr;    // [npad]
  float* slope = nullptr;   // [npad] or null
};
struct ProfRec { int a, b, kind; double flops; int op = -1; int code = -1; int small = -1; };   // small: plan class
// A run of IResNet identity blocks executed by the resident chain kernel
// (pc_conv_chain.hip): ops [first, first + 2*nblk) of the program.
struct ChainBlockH { const void* w1; const float* b1; const float* s1; const void* w2; const float* b2; };
struct ChainPlan {
  int first = -1, nblk = 0, in_t = -1, out_t = -1;
  void* d_blk = nullptr;          // ChainBlockH[nblk] on the device
  void* d_wpack = nullptr;        // the blocks' conv weights repacked (layout wl), or null
  int wl = 0;                     // weight layout the kernel reads (pc_conv_chain.hip WL)
  double flops_per_image = 0.0;
};

struct pc_net {
  pc_ctx* ctx = nullptr;
  int f32 = 0;
  int max_batch = 0;
  int in_tensor = 0;
  int in_centered = 0;        // the input is the centred image x - 127.5 (program input tensor flag bit 1)
  std::vector<NetBuf> bufs;
  std::vector<NetTensor> tens;
  std::vector<NetOp> ops;
  std::vector<int> outs;
  std::vector<void*> arrays;  // device copies (conv weights in act dtype, others f32)
  std::vector<long long> array_count;
  std::vector<ConvPlan> plans;
  // small-batch plan classes: plans_cls[c] holds the tiles chosen for cls_batch[c] images
  // (ascending); a run of N images takes the first class with N <= cls_batch[c], else `plans`
  std::vector<std::vector<ConvPlan>> plans_cls;
  std::vector<int> cls_batch;
  std::vector<StemPlan> stems;
  std::vector<ChainPlan> chains;
  std::vector<int> chain_at;      // op index -> chain id (first op of a chain) or -1
  int chain_min_batch = 32;       // PC_CHAIN_MIN overrides (tuning)
  std::vector<const float*> host_arrays;   // program arrays, valid during pc_net_create only
  void* stem_col = nullptr;   // im2col scratch shared by the stems
  float* partial = nullptr;
  size_t partial_bytes = 0;
  double flops_per_image = 0.0;
  int launches = 0;
  const void* cur_input = nullptr;
  // when a conv reads the net input directly, the input is first copied here so the
  // implicit-GEMM loader finds a zero tail behind it (ConvSeg::zero_off)
  void* in_copy = nullptr;
  size_t in_img_bytes = 0;
  // graph replay (runs of at most graph_max_batch images)
  int use_graph = 0;
  int capturing = 0;   // inside hipStreamBeginCapture .. EndCapture
  hipStream_t cap_stream = nullptr;   // private capture stream (pc_net_run)
  std::mutex graph_mu;
  int graph_max_batch = 1 << 30;
  // per-op HIP-event profiling (pc_net_profile)
  int prof = 0;
  std::vector<hipEvent_t> ev_pool;
  size_t ev_used = 0;
  std::vector<ProfRec> recs;
  std::map<std::pair<int, const void*>, hipGraphExec_t> graphs;
  // f16c8 convs: per op, E8M0 exponents of the weight bytes' scales (W_hi8 | W_lo8 << 8), 0 elsewhere
  std::vector<int> wf8s;
  std::vector<void*> wfrag;   // per conv op: fragment-ordered f16x3 weights (ConvParams::wfrag), or null
  // absmax calibration of the f16c8 tensors (pc_net_calibrate): per tensor max |x| slots
  int calib = 0;
  float* d_absmax = nullptr;
  // arcface scratch
  void* prep = nullptr;
  size_t prep_bytes = 0;
};

static inline int esize(const pc_net* n, int is_f32) { return (is_f32 || n->f32) ? 4 : 2; }

static void* tensor_ptr(pc_net* n, int t) {
  const NetTensor& T = n->tens[t];
  if (T.buf < 0) {
    const char* base = n->in_copy ? (const char*)n->in_copy : (const char*)n->cur_input;
    return (void*)(base + (size_t)T.coff * esize(n, T.is_f32));
  }
  return (char*)n->bufs[T.buf].d + (size_t)T.coff * esize(n, T.is_f32);
}

// Every activation buffer is followed by kZeroTail zero bytes: a padding tap of the
// implicit-GEMM loader reads one K-tile row (any channel block of the pixel stride)
// from there, so the tail covers the widest pixel row a conv reads.
static const size_t kZeroTail = 65536;

// bytes from a tensor's base to the zero tail of the buffer that holds it
static unsigned tensor_zero_off(const pc_net* n, int t) {
  const NetTensor& T = n->tens[t];
  const int es = esize(n, T.is_f32);
  const size_t end = T.buf < 0 ? n->in_img_bytes * n->max_batch : (size_t)n->bufs[T.buf].elems * n->max_batch * es;
  return (unsigned)(end - (size_t)T.coff * es);
}

static const int kNumConvCfgs = 14;   // pc_conv.hip launch_rowb

// K-row width of every f16c8 conv plan (64: a 32-channel K tile and a half-zero block-scaled MFMA;
// 128: 64 channels and a full one)
static int c8_rowb() {
  const char* e = getenv("PC_C8_ROWB");
  return e && atoi(e) == 128 ? 128 : 64;
}

static int plan_conv(pc_net* n, const NetOp& op, ConvPlan& pl, long long plan_batch, bool small = false) {
  const int* w = op.w;
  const int out = w[1], nseg = w[2], npad = w[14];
  const int esz = n->f32 ? 4 : 2;
  int rowb = 128;
  bool any_split = n->tens[out].split != 0 || (w[21] >= 0 && n->tens[w[21]].split);
  for (int s = 0; s < nseg; ++s) {
    const NetTensor& X = n->tens[w[3 + 5 * s]];
    // a split input's K tile must not straddle its hi and lo halves: the tile divides C / 2
    const int cl = X.split ? X.C / 2 : X.C;
    any_split = any_split || X.split;
    if ((cl * esz) % 128) rowb = 64;
    if ((cl * esz) % 64) return fail(n->ctx, PC_ERR_FORMAT, "conv input channels not a multiple of the K tile");
    if ((size_t)X.C * esz + 128 > kZeroTail) return fail(n->ctx, PC_ERR_FORMAT, "conv input wider than the zero tail");
    if (X.split && (n->f32 || X.is_f32 || X.cs != X.C))
      return fail(n->ctx, PC_ERR_FORMAT, "split tensors are dense f16 [hi | lo] pixels of an f16 net");
  }
  // tile configuration (pc_conv.hip launch_rowb): channel tile BC must divide npad
  static const int cfg_bc[kNumConvCfgs] = {128, 128, 64, 64, 96, 32, 32, 128, 256, 256, 64, 96, 32, 128};
  static const int cfg_bp[kNumConvCfgs] = {128, 64, 256, 128, 128, 256, 128, 256, 128, 256, 512, 256, 512, 128};
  const NetTensor& Y = n->tens[out];
  const long long Mimg = (long long)Y.H * Y.W;
  const long long M = Mimg * plan_batch;   // tile choice for this batch (overflow checks use max_batch)
  auto tiles = [&](int c) { return (M + cfg_bp[c] - 1) / cfg_bp[c] * (npad / cfg_bc[c]); };
  // Tile choice, from single-conv measurements on MI355X (tools/probe_conv.py,
  // DESIGN.md §3.1): 8-wave tiles with 64x64 or 128x64 per wave whenever the grid has
  // enough tiles; the 4-wave tiles for small grids.
  int cfg = -1;
  auto fits = [&](int c, long long min_tiles) { return npad % cfg_bc[c] == 0 && tiles(c) >= min_tiles; };
  if (fits(9, 192)) cfg = 9;                 // 256x256, npad % 256
  else if (fits(7, 192)) cfg = 7;            // 128x256
  else if (fits(13, 192)) cfg = 13;          // 128x128 (8 waves)
  else if (npad % 128 && fits(11, 128)) cfg = 11;   // 96x256
  else if (npad % 128 && fits(10, 128)) cfg = 10;   // 64x512
  else if (npad % 64 && fits(12, 128)) cfg = 12;    // 32x512
  else if (npad % 128 == 0) cfg = tiles(0) >= 256 ? 0 : 1;
  else if (npad % 96 == 0) cfg = 4;
  else if (npad % 64 == 0) cfg = tiles(2) >= 512 ? 2 : 3;
  else if (npad % 32 == 0) cfg = tiles(5) >= 512 ? 5 : 6;
  else return fail(n->ctx, PC_ERR_FORMAT, "conv npad must be a multiple of 32");
  if (const char* e = getenv("PC_CONV_CFG")) {   // testing / tuning override
    const int f = atoi(e);
    if (f >= 0 && f < kNumConvCfgs && npad % cfg_bc[f] == 0) cfg = f;
  }
  if (const char* e = getenv("PC_CONV_ROWB")) {  // tuning: force 64-byte K-tiles
    if (atoi(e) == 64) rowb = 64;
  }
  pl.rowb = rowb; pl.cfg = cfg; pl.M_per_image = Mimg;
  pl.splitk = w[24] > 1 ? w[24] : 1;
  pl.halo = -1;
  // Stride-1 "same" convs (the bulk of both trunks) run on the halo kernel
  // (pc_conv_halo.hip): the input run of a pixel tile is staged once per channel chunk
  // and every tap reads it from LDS. PC_CONV_HALO=0 disables, =k+1 forces cfg k.
  {
    const NetTensor& X = n->tens[w[3]];
    const int KH = w[4], KW = w[5], st = w[6], pd = w[7];
    const char* e = getenv("PC_CONV_HALO");
    // a forced igemm tile (PC_CONV_CFG) without PC_CONV_HALO means "test that tile"
    const int force = e ? atoi(e) : (getenv("PC_CONV_CFG") ? 0 : -1);
    const bool ok = !any_split && nseg == 1 && pl.splitk == 1 && st == 1 && KH == KW && pd * 2 + 1 == KH && X.H == Y.H &&
                    X.W == Y.W && KH * KW <= 32 && (double)M * X.cs * esz < 4294967296.0 - 65536.0 && force != 0;
    if (ok) {
      auto htiles = [&](int hc) {
        int bc = 0, bp = 0;
        conv_halo_tile(hc, &bc, &bp);
        return npad % bc ? 0LL : (M + bp - 1) / bp * (npad / bc);
      };
      auto hok = [&](int hc) { return htiles(hc) > 0 && conv_halo_fits(hc, KH, KW, X.W); };
      int hc = -1;
      if (force > 0) {
        if (hok(force - 1)) hc = force - 1;
      } else {
        // largest tile whose grid still covers the CUs; smaller tiles otherwise
        static const int order[] = {0, 1, 2, 3, 4};
        for (int k : order)
          if (hok(k) && htiles(k) >= 192) { hc = k; break; }
        if (hc < 0)
          for (int k : {2, 4, 3, 1, 0})
            if (hok(k)) { hc = k; break; }
      }
      pl.halo = hc;
      if (hc >= 0) pl.rowb = 64;   // the halo kernel steps K by one 64-byte LDS row
    }
  }
  // The statically scheduled kernel (pc_conv_fast.hip) takes every conv it can run:
  // no split-K, offsets within 32 bits. Tile choice: fewest rounds of workgroups over
  // the 256 CUs (one workgroup per CU), then the per-tile cost factor measured on
  // MI355X (bigger wave tiles stage fewer LDS bytes per MFMA).
  // PC_CONV_FAST=0 disables, =k+1 forces tile k.
  pl.fast = -1;
  pl.sx = 0;
  // f16x3 split inputs on conv_fast: fused tiles (a (tap, hi block) with its lo block and both
  // weight halves, pc_conv_fast.hip SX) where two stages of the doubled tile fit the LDS.
  // PC_SPLIT_FUSED=0: walk the virtual [hi, lo, hi] blocks as plain tiles instead.
  bool all_split = nseg > 0 && !n->f32;
  for (int sg = 0; sg < nseg; ++sg) all_split = all_split && n->tens[w[3 + 5 * sg]].split;
  // f16c8 inputs: every segment f16c8, conv_fast's C8 tiles only
  int nc8 = 0;
  for (int sg = 0; sg < nseg; ++sg) nc8 += n->tens[w[3 + 5 * sg]].c8;
  const bool in_c8 = nc8 > 0;
  const bool out_c8 = n->tens[out].c8 || (w[21] >= 0 && n->tens[w[21]].c8);
  if (in_c8 && nc8 != nseg) return fail(n->ctx, PC_ERR_FORMAT, "conv mixes f16c8 and other input segments");
  if (in_c8 && (w[24] > 1 || n->f32 || (getenv("PC_SPLIT_FUSED") && atoi(getenv("PC_SPLIT_FUSED")) == 0)))
    return fail(n->ctx, PC_ERR_FORMAT, "f16c8 convs run on conv_fast's fused C8 tiles only (no split-K)");
  const bool try_sx = all_split && pl.splitk == 1 && !(getenv("PC_SPLIT_FUSED") && atoi(getenv("PC_SPLIT_FUSED")) == 0);
  {
    const char* e = getenv("PC_CONV_FAST");
    const int force = e ? atoi(e) : ((getenv("PC_CONV_CFG") || getenv("PC_CONV_HALO")) ? 0 : -1);
    bool ok = pl.splitk == 1 && force != 0;
    // odd multiples of 32 channels (96, 160, 224: SCRFD trunks) run faster on the generic
    // kernel's 96x256 / 32x512 tiles (measured per layer, tools/probe_layers.py scrfd)
    if (force < 0 && npad > 32 && npad % 64 == 32 && !try_sx) ok = false;
    for (int sg = 0; sg < nseg && ok; ++sg) {
      const NetTensor& X = n->tens[w[3 + 5 * sg]];
      if ((double)X.H * X.W * n->max_batch * X.cs * esz + kZeroTail >= 4294967296.0) ok = false;
    }
    if ((double)npad * w[15] * esz >= 4294967296.0) ok = false;
    if (ok) {
      // (15-19: small-batch tiles, latency-bound K loops: a second round of them costs about
      // as much as the first, hence the high factor of the smallest)
      static const double cost[] = {1.0, 1.12, 1.12, 1.3, 1.3, 1.3, 1.15, 1.45, 1.3, 1.0, 0.9, 1.3, 1.6, 1.0, 1.0,
                                    1.9, 1.6, 1.6, 3.0, 1.9, 1.3, 1.55};
      static const int occ[] = {1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 2, 1, 1, 1, 2, 1, 1, 1, 1, 1, 1, 1};   // workgroups per CU
      static_assert(sizeof(cost) / sizeof(cost[0]) == sizeof(occ) / sizeof(occ[0]), "tile tables");
      // fused split tiles: the 128x512 tile (8 waves of 64x128) ran ArcFace-x3's 28x28x128 at 464 us
      // against 233 for the 128x256 tile at the same estimate (profiles/r05n_sx_tile_sweep.txt)
      // (and the 64x128 small tile: ArcFace-x3's 28x28x128 at 12 rows 28.0 us against 34.5 for the 32x256
      // tile the plain factor picks, profiles/r06n_small_tile_sweep.txt)
      auto sxcost = [&](int k) { return k == 9 ? 2.2 : k == 16 ? 1.4 : cost[k]; };
      int best = -1, best_rowb = rowb;
      double best_t = 0;
      bool rows256 = small && !n->f32 && !any_split && rowb == 128 && !getenv("PC_CONV_ROWB");
      for (int sg = 0; sg < nseg && rows256; ++sg) rows256 = (n->tens[w[3 + 5 * sg]].C * esz) % 256 == 0;
      const bool no_small_tiles = getenv("PC_SMALL_TILES") && atoi(getenv("PC_SMALL_TILES")) == 0;   // A/B
      for (int k = 0; k < conv_fast_num_cfgs(); ++k) {
        int bc = 0, bp = 0;
        conv_fast_tile(k, &bc, &bp);
        // cfgs 10 and 14 run on 64-byte K rows only; the small-batch tiles 15-17 take 256-byte
        // rows where every segment's channels allow (half the barrier-separated K tiles)
        const int rb = (k == 10 || k == 14) ? 64 : (k >= 15 && k <= 17 && rows256) ? 256 : rowb;
        if (npad % bc || !conv_fast_valid(k, rb)) continue;
        if (force > 0 && k != force - 1) continue;
        if (k >= kFastSmallCfg0 && k <= kFastSmallCfg1 && (!small || no_small_tiles) && force <= 0) continue;   // small-batch tiles
        const long long t = (M + bp - 1) / bp * (npad / bc);
        const double rounds = (double)((t + 256 * occ[k] - 1) / (256 * occ[k]));
        const double est = rounds * bc * bp * occ[k] * cost[k];
        if (best < 0 || est < best_t) { best = k; best_t = est; best_rowb = rb; }
      }
      if (try_sx) {   // the same choice among the tiles that can stage fused split tiles
        int bsx = -1, bsx_rowb = rowb;
        double bsx_t = 0;
        for (int k = 0; k < conv_fast_num_cfgs(); ++k) {
          int bc = 0, bp = 0;
          conv_fast_tile(k, &bc, &bp);
          if (npad % bc || (force > 0 && k != force - 1)) continue;
          if (k >= kFastSmallCfg0 && k <= kFastSmallCfg1 && (!small || no_small_tiles) && force <= 0) continue;
          for (int rb : {rowb, 64}) {
            // f16c8 inputs: tiles with the LDS epilogue, at ONE K-row width for every plan of the
            // net (kC8Rowb; PC_C8_ROWB for tuning): the row width orders the f16 and block-scaled
            // MFMAs of a K tile, so a conv's output would otherwise depend on its batch class
            if (in_c8 && (!conv_fast_valid_c8(k, rb) || rb != c8_rowb())) continue;
            if (out_c8 && !conv_fast_valid_c8(k, rb)) continue;   // f16c8 output / residual: LDS epilogue
            if (!conv_fast_valid_sx(k, rb)) continue;
            const long long t = (M + bp - 1) / bp * (npad / bc);
            // the 2-wave whole-width tiles (20, 21) need two workgroups per CU to keep their K loop fed:
            // a grid under one per CU ran SCRFD-x3's 20x20x224 at b32 in 124 us against 76.5 on the 32x256
            // tile (12), at b64 130 vs 162 (profiles/r06ap_tile_sweep.txt)
            const double est = (double)((t + 255) / 256) * bc * bp * sxcost(k) * ((k == 20 || k == 21) && t < 256 ? 2.0 : 1.0);
            if (bsx < 0 || est < bsx_t) { bsx = k; bsx_t = est; bsx_rowb = rb; }
            break;
          }
        }
        if (bsx >= 0) { best = bsx; best_rowb = bsx_rowb; pl.sx = 1; pl.c8 = in_c8 ? 1 : 0; }
        else if (in_c8) best = -1;
      }
      pl.fast = best;
      if (best >= 0) { pl.halo = -1; pl.rowb = best_rowb; }
    }
  }
  // 3x3 stride-1 convs over 32/64 channels run on the 2-D block kernel with register-
  // resident weights (pc_conv_t2d.hip, f16) when its 16-pixel-wide blocks cover the
  // image with little waste. PC_CONV_T2D=0 disables, =2 forces wherever it can run.
  pl.t2d = -1;
  {
    const char* e = getenv("PC_CONV_T2D");
    const int mode = e ? atoi(e) : ((getenv("PC_CONV_CFG") || getenv("PC_CONV_HALO") || getenv("PC_CONV_FAST")) ? 0 : 1);
    const NetTensor& X = n->tens[w[3]];
    // split (f16x3): split input -> split output (and split residual, if any) only
    const int sp = X.split ? 1 : 0;
    const bool split_ok = !sp ? !any_split
                              : (Y.split && !Y.c8 && !in_c8 && (w[21] < 0 || (n->tens[w[21]].split && !n->tens[w[21]].c8)) &&
                                 Y.C / 2 >= 8 && (Y.C / 2) % 8 == 0);
    const int cin_l = sp ? X.C / 2 : X.C;
    const int var = (mode > 0 && !n->f32 && nseg == 1 && pl.splitk == 1 && X.H == Y.H && X.W == Y.W && split_ok)
                        ? conv_t2d_select(cin_l, npad, w[4], w[5], w[6], w[7], w[20], Y.is_f32, Y.cs, Y.coff, sp)
                        : -1;
    if (var >= 0 && w[15] >= (sp ? 27LL : 9LL) * cin_l &&
        (double)X.H * X.W * n->max_batch * X.cs * esz + kZeroTail < 4294967296.0 &&
        (double)M < 2147483647.0) {
      const int th = conv_t2d_rows(var);
      const double cover = (double)Y.H * Y.W / ((double)((Y.H + th - 1) / th * th) * ((Y.W + 15) / 16 * 16));
      if (mode == 2 || cover >= 0.75) {
        pl.t2d = var;   // the variant, fixed at plan time (conv_t2d_launch runs exactly it)
        pl.fast = -1;
        pl.sx = 0;
        pl.halo = -1;
      }
    }
  }
  // f16x3 64 -> 64 channel 3x3 layers on the halo-staged split kernel (pc_conv_hx.hip: 160x160x64
  // b64 524 vs 632 us on conv_fast's fused tile) where its grid fills the CUs; it accumulates in the
  // fused tiles' order (round 6), so plan classes choose freely. PC_CONV_HX=0 disables; the tuning
  // overrides of the other kernels too.
  pl.hx = 0;
  if (!(getenv("PC_CONV_HX") && atoi(getenv("PC_CONV_HX")) == 0) && !getenv("PC_CONV_FAST") &&
      !getenv("PC_CONV_CFG") && !getenv("PC_CONV_HALO") && !getenv("PC_CONV_T2D") && !getenv("PC_T2D_SPLIT64") &&
      !getenv("PC_SPLIT_FUSED") && !n->f32 && nseg == 1 && pl.splitk == 1) {
    const NetTensor& X = n->tens[w[3]];
    if (X.split && !X.c8 && !Y.c8 && X.C == 128 && X.cs == 128 && Y.split && Y.C == 128 && npad == 64 && w[4] == 3 && w[5] == 3 &&
        w[6] == 1 && w[7] == 1 && X.H == Y.H && X.W == Y.W && w[15] == 9 * 192 &&
        !(w[21] >= 0 && (w[22] == RES_UP2 || !n->tens[w[21]].split || n->tens[w[21]].c8)) &&
        (double)X.H * X.W * n->max_batch * X.cs * esz + kZeroTail < 4294967296.0 &&
        plan_batch * ((Y.H + 11) / 12) * ((Y.W + 15) / 16) >= 256) {
      // (its 16x12 blocks at two per CU; a grid of fewer blocks - a per-frame extract()'s 40x40 maps -
      // keeps the fused tiles: the same accumulation order, so the classes stay bit-identical)
      pl.hx = 1;
      pl.fast = pl.halo = pl.t2d = -1;
      pl.sx = 0;
    }
    // 96 -> 96 channel layers (SCRFD's 80x80 / 40x40 / 20x20 x96 trunk) on conv_hxg<96, 96>: one
    // workgroup per CU, every output channel per wave, the halo staged per 32-channel group
    // (PC_CONV_HXG=0 disables, for A/B)
    // (and SCRFD's 20x20x224 neck layers, small-batch form only)
    const bool c224 = X.C == 448 && Y.H == 20 && plan_batch <= 16;
    if (X.split && !X.c8 && !Y.c8 && (X.C == 192 || c224) && X.cs == X.C && Y.split && Y.C == X.C && npad == X.C / 2 &&
        w[4] == 3 && w[5] == 3 && w[6] == 1 && w[7] == 1 && X.H == Y.H && X.W == Y.W && w[15] == 27 * npad &&
        !(w[21] >= 0 && (w[22] == RES_UP2 || !n->tens[w[21]].split || n->tens[w[21]].c8)) &&
        (double)X.H * X.W * n->max_batch * X.cs * esz + kZeroTail < 4294967296.0 &&
        !(getenv("PC_CONV_HXG") && atoi(getenv("PC_CONV_HXG")) == 0)) {
      // (one 16x20 block per CU; smaller grids - a single frame's 80x80 map is 20 blocks - take the
      // small-batch form, 16x4 blocks x 32 channels (PC_CONV_HXG bit 1; 80x80 / 40x40 maps, 20x20 in the plans
      // for <= 16 frames; SCRFD-x3 at one frame 1.20 -> 0.98 ms, profiles/r06bm_*), or the fused
      // tiles: bit-identical, conv_hxg walks K and the MFMA passes in their order)
      const int hxg_mask = getenv("PC_CONV_HXG") ? atoi(getenv("PC_CONV_HXG")) : 3;
      if (plan_batch * ((Y.H + 19) / 20) * ((Y.W + 15) / 16) >= 128 && (hxg_mask & 1) && !c224) pl.hx = 2;
      else if ((hxg_mask & 2) && (Y.H >= 40 || plan_batch <= 16)) pl.hx = 5;   // (profile code 504)
    }
    if (pl.hx == 2 || pl.hx == 5) {
      pl.fast = pl.halo = pl.t2d = -1;
      pl.sx = 0;
    }
    // IResNet's 14x14x256 and 28x28x128 layers on the image-resident conv_hxi (pc_conv_hxi.hip) at
    // batches that give every CU a workgroup (plans for >= 192 / 64 images): bit-identical to the fused
    // tiles the smaller plan classes run (same K order, MFMA order and epilogue arithmetic).
    // PC_CONV_HXI is a mask of the shapes it takes: bit 0 14x14x256, bit 1 28x28x128 (f16x3), bits 2 / 3 the
    // same shapes of plain f16 nets, bit 4 the f16x3 7x7x512, bit 5 the small-batch forms (default 59: all but plain 14x14x256, which the
    // resident chain beats). ArcFace-x3
    // b256 per layer, interleaved on one box: 28x28x128 187.5 vs 224.2 us on the 128x256 WG tile,
    // 14x14x256 149.3 vs 151.5 on the 256x224 one; C3 962 vs 930 frames/s with the embed quantum at 128
    // faces (256 rows = one round of one-image workgroups; at 383 rows, 1.5 rounds, 876: the quantum
    // follows, face_embedder.py), profiles/r06e_*
    const int hxi_mask = getenv("PC_CONV_HXI") ? atoi(getenv("PC_CONV_HXI")) : 59;
    // plain f16 nets (BASELINE C2's fp16 ArcFace): bits 2 / 3 = 14x14x256 / 28x28x128 (tap-major K: the
    // plain tiles' and the resident chain's order, bit-identical). f16 ArcFace b256, one box (r06m):
    // 28x28x128 72.8 us/launch vs 94.0 on tile cfg 14 (C2 f16 7.64 vs 8.17 ms); 14x14x256 65 us x 58 =
    // 3.77 ms vs 3.34 for the resident chain, so bit 2 stays opt-in (profiles/r06m_*)
    if (!X.split && !X.c8 && !X.is_f32 && !Y.split && !Y.is_f32 && !Y.c8 && X.cs == X.C && Y.cs == Y.C && Y.C == X.C &&
        npad == X.C && w[4] == 3 && w[5] == 3 && w[6] == 1 && w[7] == 1 && X.W == X.H && Y.H == X.H && Y.W == X.W &&
        w[15] == 9 * X.C && !(w[21] >= 0 && (w[22] == RES_UP2 || n->tens[w[21]].split || n->tens[w[21]].is_f32)) &&
        (((hxi_mask & 4) && X.C == 256 && X.H == 14 && plan_batch >= 192) ||
         ((hxi_mask & 8) && X.C == 128 && X.H == 28 && plan_batch >= 64)) &&
        (double)X.H * X.W * n->max_batch * X.cs * esz + kZeroTail < 4294967296.0) {
      pl.hx = X.C == 256 ? 3 : 4;
      pl.fast = pl.halo = pl.t2d = -1;
      pl.sx = 0;
    }
    const int hc = X.C / 2;
    // (bit 4: the f16x3 7x7x512 stage, one image per workgroup at pitch 9)
    // (bit 5, default on: the small-batch forms, 32 channels of 7 rows per workgroup, in the plans for <= 32
    // images - a per-frame extract()'s rows; the f16x3 shapes. ArcFace-x3 at 12 rows, one box: 14x14x256
    // 29.9 vs 31.3 us on the 64x64 tile, 28x28x128 20.7 vs 27.6, 7x7x512 35.6 vs 56.6; profiles/r06bh_*)
    const bool hxs_shape = (hxi_mask & 32) && plan_batch <= 32 &&
                           ((hc == 256 && X.H == 14) || (hc == 128 && X.H == 28) || (hc == 512 && X.H == 7));
    const bool hxi_shape = ((hxi_mask & 1) && hc == 256 && X.H == 14 && plan_batch >= 192) ||
                           ((hxi_mask & 2) && hc == 128 && X.H == 28 && plan_batch >= 64) ||
                           ((hxi_mask & 16) && hc == 512 && X.H == 7 && plan_batch >= 192) || hxs_shape;
    if (hxi_shape && X.split && !X.c8 && !Y.c8 && X.cs == X.C && Y.split && Y.C == X.C && Y.cs == Y.C && npad == hc &&
        w[4] == 3 && w[5] == 3 && w[6] == 1 && w[7] == 1 && X.W == X.H && Y.H == X.H && Y.W == X.W && w[15] == 27 * hc &&
        !(w[21] >= 0 && (w[22] == RES_UP2 || !n->tens[w[21]].split || n->tens[w[21]].c8)) &&
        (double)X.H * X.W * n->max_batch * X.cs * esz + kZeroTail < 4294967296.0) {
      pl.hx = (hc == 256 ? 3 : hc == 128 ? 4 : 6) + (hxs_shape ? (hc == 512 ? 3 : 4) : 0);   // (profile codes 502 / 503 / 505, small 506-508)
      pl.fast = pl.halo = pl.t2d = -1;
      pl.sx = 0;
    }
  }
  // small-batch plan: a long-K conv of a few images fills a fraction of the CUs (a 14x14x256
  // conv of 12 rows: 56 workgroups of 2304-long K) - split K over the generic kernel so the
  // grid covers them; the partials are finished by splitk_finish with the full epilogue.
  // Opt-in (PC_SMALL_SPLITK=1): split-K sums in another order, so a frame's results would
  // depend on the batch it ran in, and extract() / extract_batch() are bit-identical by
  // contract (tests/test_gpu_face_embedder.py::test_extract_single_matches_batch).
  if (small && pl.splitk == 1 && !n->f32 && !any_split && getenv("PC_SMALL_SPLITK")) {
    const long long t = tiles(cfg);
    const int ktiles = (int)(w[15] * esz / rowb);
    if (t < 192 && ktiles >= 16) {
      int sk = (int)std::min<long long>(8, std::max<long long>(2, 384 / std::max<long long>(1, t)));
      sk = std::min(sk, ktiles / 4);
      if (sk >= 2) {
        pl.splitk = sk;
        pl.fast = pl.halo = pl.t2d = -1;
        pl.sx = 0;
        pl.cfg = cfg;
        pl.rowb = rowb;
      }
    }
  }
  if (in_c8) {   // nothing else runs f16c8 inputs
    if (pl.fast < 0 || !pl.c8) return fail(n->ctx, PC_ERR_FORMAT, "no conv_fast C8 tile fits this f16c8 conv");
    pl.halo = pl.t2d = -1;
    pl.hx = 0;
    pl.splitk = 1;
  }
  // (and only by those with the LDS epilogue: the per-fragment epilogue of the 96 / 224-channel tiles
  // has no f8 region handling)
  if ((Y.c8 || (w[21] >= 0 && n->tens[w[21]].c8)) &&
      (pl.fast < 0 || !pl.sx || pl.t2d >= 0 || pl.hx || pl.halo >= 0 || !conv_fast_valid_c8(pl.fast, pl.rowb)))
    return fail(n->ctx, PC_ERR_FORMAT, "f16c8 outputs and residuals are written / read by conv_fast's fused LDS-epilogue tiles only");
  // fused f16x3 tiles of 64-byte K rows on the WG form where it is instantiated (PC_SX_WG=0: staged
  // weights, for A/B). Same K order and pass order as the staged form: bit-identical outputs.
  pl.wg = 0;
  if (pl.fast >= 0 && pl.sx && !pl.c8 && pl.rowb == 64 && pl.splitk == 1 && pl.t2d < 0 && !pl.hx && pl.halo < 0 &&
      conv_fast_valid_wg(pl.fast) && !(getenv("PC_SX_WG") && atoi(getenv("PC_SX_WG")) == 0))
    pl.wg = 1;
  if ((Y.split ? Y.C / 2 : Y.C) > npad) return fail(n->ctx, PC_ERR_FORMAT, "conv output tensor wider than npad");
  if (Y.split && (Y.is_f32 || Y.cs != Y.C || (Y.C / 2) % 8))
    return fail(n->ctx, PC_ERR_FORMAT, "split conv output must be a dense f16 [hi | lo] tensor");
  // split-K reads split inputs (the K iterator's virtual blocks) into f32 partials; the finish
  // kernel writes plain tensors only (the f16x3 IResNet's FC: split 7x7x512 -> f32 embedding)
  if (pl.splitk > 1 && (Y.split || (w[21] >= 0 && n->tens[w[21]].split)))
    return fail(n->ctx, PC_ERR_FORMAT, "split-K into a split output");
  return PC_OK;
}

// Stem as im2col + 1x1 MFMA conv when the window fits one 32-element K row
// (3x3x3 = 27). Weights are repacked [npad][32], tap-major, channel-minor.
static int plan_stem(pc_net* n, const NetOp& op, StemPlan& st, size_t& col_bytes) {
  const int* w = op.w;
  const int KH = w[3], KW = w[4], cout = w[8], cin_true = w[13] > 0 ? w[13] : 3;
  const NetTensor& X = n->tens[w[2]];
  const NetTensor& Y = n->tens[w[1]];
  if (Y.split && (n->f32 || KH * KW * cin_true > 32 || X.C != 4 || Y.is_f32))
    return fail(n->ctx, PC_ERR_FORMAT, "split stem output needs the fused f16 stem");
  if (!Y.split && (getenv("PC_STEM_DIRECT") || KH * KW * cin_true > 32 || X.C != 4)) return PC_OK;   // direct kernel
  const int esz = n->f32 ? 4 : 2;
  st.use_mfma = 1;
  st.cin_true = cin_true;
  st.split = Y.split;
  st.npad = (std::max(cout, Y.split ? Y.C / 2 : Y.C) + 31) / 32 * 32;
  st.rowb = 32 * esz;   // one K-tile of exactly 32 elements
  const long long M = (long long)Y.H * Y.W * n->max_batch;
  st.cfg = st.npad % 128 == 0 ? 7 : (st.npad % 64 == 0 ? 10 : 12);
  col_bytes = std::max(col_bytes, (size_t)M * 32 * esz + 256);
  const float* hw = reinterpret_cast<const float*>(n->host_arrays[w[7]]);
  std::vector<float> wf((size_t)st.npad * 32, 0.f), b(st.npad, 0.f), sl(st.npad, 0.f);
  for (int co = 0; co < cout; ++co)
    for (int t = 0; t < KH * KW; ++t)
      for (int ci = 0; ci < cin_true; ++ci) wf[(size_t)co * 32 + t * cin_true + ci] = hw[((size_t)co * KH * KW + t) * 4 + ci];
  const float* hb = reinterpret_cast<const float*>(n->host_arrays[w[9]]);
  for (int co = 0; co < cout; ++co) b[co] = hb[co];
  if (w[10] >= 0) {
    const float* hs = reinterpret_cast<const float*>(n->host_arrays[w[10]]);
    for (int co = 0; co < cout; ++co) sl[co] = hs[co];
  }
  if (st.split) {   // rows of 64: K 0-31 W_hi, 32-63 W_lo = f16(W - W_hi)
    std::vector<_Float16> h((size_t)st.npad * 64);
    for (int co = 0; co < st.npad; ++co)
      for (int k = 0; k < 32; ++k) {
        const float v = wf[(size_t)co * 32 + k];
        const _Float16 hi = (_Float16)v;
        h[(size_t)co * 64 + k] = hi;
        h[(size_t)co * 64 + 32 + k] = (_Float16)(v - (float)hi);
      }
    HIPCHK(n->ctx, hipMalloc(&st.w, h.size() * 2));
    HIPCHK(n->ctx, hipMemcpy(st.w, h.data(), h.size() * 2, hipMemcpyHostToDevice));
  } else {
  HIPCHK(n->ctx, hipMalloc(&st.w, wf.size() * esz));
  if (n->f32) {
    HIPCHK(n->ctx, hipMemcpy(st.w, wf.data(), wf.size() * 4, hipMemcpyHostToDevice));
  } else {
    std::vector<_Float16> h(wf.size());
    for (size_t k = 0; k < wf.size(); ++k) h[k] = (_Float16)wf[k];
    HIPCHK(n->ctx, hipMemcpy(st.w, h.data(), h.size() * 2, hipMemcpyHostToDevice));
  }
  }
  HIPCHK(n->ctx, hipMalloc((void**)&st.bias, st.npad * 4));
  HIPCHK(n->ctx, hipMemcpy(st.bias, b.data(), st.npad * 4, hipMemcpyHostToDevice));
  if (w[10] >= 0) {
    HIPCHK(n->ctx, hipMalloc((void**)&st.slope, st.npad * 4));
    HIPCHK(n->ctx, hipMemcpy(st.slope, sl.data(), st.npad * 4, hipMemcpyHostToDevice));
  }
  return PC_OK;
}

// Runs of IResNet identity blocks that the resident chain kernel (pc_conv_chain.hip) can
// execute as one launch: conv1 = 3x3/s1 over X with the border-class bias and PReLU,
// conv2 = 3x3/s1 over conv1's output + bias + residual X, 256 channels, images of at
// most 199 pixels, f16. Every tensor between the chain's first input and its last output
// must be read only inside the chain (the kernel never writes them).
static int plan_chains(pc_net* n) {
  n->chain_at.assign(n->ops.size(), -1);
  if (n->f32) return PC_OK;
  if (const char* e = getenv("PC_CHAIN")) if (atoi(e) == 0) return PC_OK;
  if (const char* e = getenv("PC_CHAIN_MIN")) n->chain_min_batch = std::max(1, atoi(e));
  if ((size_t)conv_chain_block_bytes() != sizeof(ChainBlockH)) return fail(n->ctx, PC_ERR_HIP, "chain block layout");
  const int nt = (int)n->tens.size();
  std::vector<int> uses(nt, 0);
  for (auto& op : n->ops) {
    if (op.w[0] == OP_CONV) {
      for (int s = 0; s < op.w[2]; ++s) uses[op.w[3 + 5 * s]]++;
      if (op.w[21] >= 0) uses[op.w[21]]++;
    } else if (op.w[0] == OP_STEM || op.w[0] == OP_MAXPOOL || op.w[0] == OP_UPSAMPLE || op.w[0] == OP_LAYERNORM ||
               op.w[0] == OP_ATTENTION) {
      uses[op.w[2]]++;
    }
  }
  for (int o : n->outs) if (o >= 0 && o < nt) uses[o] += 1000;
  auto is_block = [&](size_t i, int X) -> int {   // output tensor of the block at ops i, i+1, or -1
    if (i + 1 >= n->ops.size()) return -1;
    const int* a = n->ops[i].w;
    const int* b = n->ops[i + 1].w;
    if (a[0] != OP_CONV || b[0] != OP_CONV || a[2] != 1 || b[2] != 1) return -1;
    if (a[3] != X || a[4] != 3 || a[5] != 3 || a[6] != 1 || a[7] != 1) return -1;
    if (a[14] != 256 || a[16] != 256 || a[18] != BIAS_BORDER9 || a[17] < 0 || a[19] < 0 || a[20] != ACT_PRELU ||
        a[21] >= 0 || a[24] > 1 || a[23] != 0)
      return -1;
    const int Y1 = a[1];
    if (b[3] != Y1 || b[4] != 3 || b[5] != 3 || b[6] != 1 || b[7] != 1) return -1;
    if (b[14] != 256 || b[16] != 256 || b[18] != BIAS_CHANNEL || b[17] < 0 || b[20] != ACT_NONE || b[21] != X ||
        b[22] != RES_SAME || b[23] != 0 || b[24] > 1 || a[15] != b[15])
      return -1;
    const NetTensor &TX = n->tens[X], &T1 = n->tens[Y1], &T2 = n->tens[b[1]];
    if (TX.is_f32 || T1.is_f32 || T2.is_f32 || TX.buf < 0 || T2.buf < 0) return -1;
    if (TX.C != 256 || T1.C != 256 || T2.C != 256 || T1.H != TX.H || T1.W != TX.W || T2.H != TX.H || T2.W != TX.W)
      return -1;
    if (!conv_chain_fits(TX.H, TX.W, TX.C, a[14], a[15])) return -1;
    if (uses[Y1] != 1) return -1;   // conv1's output feeds conv2 only
    return b[1];
  };
  for (size_t i = 0; i + 1 < n->ops.size();) {
    const int X = n->ops[i].w[0] == OP_CONV ? n->ops[i].w[3] : -1;
    int out = X >= 0 ? is_block(i, X) : -1;
    if (out < 0) { ++i; continue; }
    ChainPlan ch;
    ch.first = (int)i;
    ch.in_t = X;
    ch.nblk = 1;
    // X is read twice by the first block (conv1 input and residual); later block inputs
    // must be read by their block only
    while (uses[out] == 2) {
      const int nxt = is_block(i + 2 * ch.nblk, out);
      if (nxt < 0) break;
      out = nxt;
      ch.nblk++;
    }
    ch.out_t = out;
    const NetTensor &TX = n->tens[X], &TY = n->tens[out];
    const bool alias_ok = TX.buf != TY.buf || (TX.cs == TY.cs && TX.coff == TY.coff);
    if (ch.nblk < 2 || !alias_ok || (TX.cs & 7) || (TY.cs & 7) || (TX.coff & 7) || (TY.coff & 7)) {
      i += 2 * ch.nblk;
      continue;
    }
    std::vector<ChainBlockH> hb(ch.nblk);
    // weight layout of the kernel's register stream (tuning: PC_CHAIN_WL): 0 the convs'
    // own [256][ktot] rows; 1 / 2 repacked fragment-major, 1 KiB per (K-step j, channel
    // group g, row block a) holding W[g*64 + a*16 + (l & 15)][j*32 + (l >> 4)*8 .. +7] at
    // +16*l, ordered [j][g][a] (1) or [g][a][j] (2)
    ch.wl = 0;
    if (const char* e = getenv("PC_CHAIN_WL")) ch.wl = atoi(e) == 2 ? 2 : 0;
    const size_t cbytes = (size_t)72 * 256 * 64;
    if (ch.wl) {
      HIPCHK(n->ctx, hipMalloc(&ch.d_wpack, cbytes * 2 * ch.nblk));
      const long long ktot = n->ops[i].w[15];
      std::vector<_Float16> src((size_t)256 * ktot), dst(cbytes / 2);
      for (int cv = 0; cv < 2 * ch.nblk; ++cv) {
        const int* w = n->ops[i + cv].w;
        HIPCHK(n->ctx, hipMemcpy(src.data(), n->arrays[w[13]], src.size() * 2, hipMemcpyDeviceToHost));
        for (int j = 0; j < 72; ++j)
          for (int g = 0; g < 4; ++g)
            for (int a = 0; a < 4; ++a)
              for (int l = 0; l < 64; ++l) {
                const _Float16* sp = &src[(size_t)(g * 64 + a * 16 + (l & 15)) * ktot + j * 32 + (l >> 4) * 8];
                const size_t blk1k = ch.wl == 1 ? ((size_t)j * 4 + g) * 4 + a : ((size_t)g * 4 + a) * 72 + j;
                _Float16* dp = &dst[(blk1k * 64 + l) * 8];
                for (int e = 0; e < 8; ++e) dp[e] = sp[e];
              }
        HIPCHK(n->ctx, hipMemcpy((char*)ch.d_wpack + cbytes * cv, dst.data(), cbytes, hipMemcpyHostToDevice));
      }
    }
    for (int k = 0; k < ch.nblk; ++k) {
      const int* a = n->ops[i + 2 * k].w;
      const int* b = n->ops[i + 2 * k + 1].w;
      const void* w1 = ch.wl ? (const void*)((char*)ch.d_wpack + cbytes * (2 * k)) : n->arrays[a[13]];
      const void* w2 = ch.wl ? (const void*)((char*)ch.d_wpack + cbytes * (2 * k + 1)) : n->arrays[b[13]];
      hb[k] = ChainBlockH{w1, (const float*)n->arrays[a[17]], (const float*)n->arrays[a[19]], w2,
                          (const float*)n->arrays[b[17]]};
      ch.flops_per_image += n->plans[i + 2 * k].flops_per_image + n->plans[i + 2 * k + 1].flops_per_image;
    }
    HIPCHK(n->ctx, hipMalloc(&ch.d_blk, hb.size() * sizeof(ChainBlockH)));
    HIPCHK(n->ctx, hipMemcpy(ch.d_blk, hb.data(), hb.size() * sizeof(ChainBlockH), hipMemcpyHostToDevice));
    n->chain_at[i] = (int)n->chains.size();
    n->chains.push_back(ch);
    i += 2 * ch.nblk;
  }
  return PC_OK;
}

// OCP e4m3fn encoding (round to nearest even, saturating at +-448): the host side of the f16c8
// weight bytes; the device encodes activations with v_cvt_pk_fp8_f32 (pc_conv_common.h f8_pack8)
static uint8_t e4m3_encode(float v) {
  const uint8_t sgn = std::signbit(v) ? 0x80 : 0;
  const float a = std::fabs(v);
  if (!(a == a)) return 0x7f;
  if (a >= 448.f) return sgn | 0x7e;
  int e2 = 0;
  std::frexp(a, &e2);
  int E = e2 - 1;                                 // a in [2^E, 2^(E+1))
  if (a == 0.f || E < -6) {                       // subnormals: steps of 2^-9
    const int q = (int)std::nearbyint(std::ldexp(a, 9));
    return sgn | (uint8_t)q;                      // q == 8 is the smallest normal's encoding
  }
  int q = (int)std::nearbyint(std::ldexp(a, 3 - E));   // 8 .. 16
  if (q == 16) { q = 8; ++E; }
  if (E > 8 || (E == 8 && q > 14)) return sgn | 0x7e;
  return sgn | (uint8_t)(((E + 7) << 3) | (q - 8));
}

// Fragment-ordered copy of a fused f16x3 conv's weights (conv_fast WG, conv_hx64): K tiles of 32
// channels in the fused tiles' order at 64-byte rows (segment, group of 64 hi channels, tap row, tap
// column, 32-channel block; ConvSeg::gt); per tile
// npad / 16 row blocks of [W_hi, W_lo] fragments, each 64 lanes x 8 f16 (lane l: row l & 15,
// channels 8 (l >> 4) .. +8), so a wave's fragment read is one contiguous KiB.
static int pack_wfrag(pc_net* n, const NetOp& op, const float* wf, void** out) {
  const int* w = op.w;
  const int npad = w[14];
  const long long ktot = w[15];
  if (w[2] == 1 && !n->tens[w[3]].split) {
    // plain f16 (conv_hxi's plain form): K tiles of 32 channels tap-major (tap row, tap column,
    // 32-channel block: conv_fast's plain K order), per tile npad / 16 row blocks of W fragments
    const NetTensor& X = n->tens[w[3]];
    const int C = X.C, KH = w[4], KW = w[5];
    if (C % 32 || (long long)KH * KW * C != ktot || npad % 16) return fail(n->ctx, PC_ERR_FORMAT, "wfrag: plain K layout");
    const long long nkt = (long long)KH * KW * (C / 32), tile_elems = (long long)(npad / 16) * 512;
    std::vector<_Float16> h((size_t)(nkt * tile_elems));
    for (long long kt = 0; kt < nkt; ++kt)
      for (int rb = 0; rb < npad / 16; ++rb)
        for (int l = 0; l < 64; ++l)
          for (int j = 0; j < 8; ++j) {
            const long long row = rb * 16 + (l & 15), k = kt * 32 + (l >> 4) * 8 + j;
            h[(size_t)(kt * tile_elems + ((long long)rb * 64 + l) * 8 + j)] = (_Float16)wf[row * ktot + k];
          }
    if (hipMalloc(out, h.size() * 2) != hipSuccess ||
        hipMemcpy(*out, h.data(), h.size() * 2, hipMemcpyHostToDevice) != hipSuccess)
      return fail(n->ctx, PC_ERR_HIP, "wfrag upload failed");
    return PC_OK;
  }
  long long nkt = 0, k0 = 0;
  for (int sg = 0; sg < w[2]; ++sg) {
    const NetTensor& X = n->tens[w[3 + 5 * sg]];
    if (!X.split || (X.C / 2) % 32) return fail(n->ctx, PC_ERR_FORMAT, "wfrag: split inputs of 32-channel blocks");
    nkt += (long long)w[4 + 5 * sg] * w[5 + 5 * sg] * (X.C / 2 / 32);
    k0 += (long long)w[4 + 5 * sg] * w[5 + 5 * sg] * 3 * (X.C / 2);
  }
  if (k0 != ktot || npad % 16) return fail(n->ctx, PC_ERR_FORMAT, "wfrag: K layout");
  const long long tile_elems = (long long)(npad / 16) * 2 * 512;
  std::vector<_Float16> h((size_t)(nkt * tile_elems));
  long long kt = 0;
  k0 = 0;
  for (int sg = 0; sg < w[2]; ++sg) {
    const int cp = n->tens[w[3 + 5 * sg]].C / 2, KH = w[4 + 5 * sg], KW = w[5 + 5 * sg];
    const int gt = cp % 64 == 0 ? 2 : 1;   // the fused tiles' channel groups at 64-byte K rows
    for (int g0 = 0; g0 < cp / 32; g0 += gt)
      for (int th = 0; th < KH; ++th)
        for (int tw = 0; tw < KW; ++tw)
          for (int cb = g0; cb < g0 + gt; ++cb, ++kt) {
          const long long kbase = k0 + (long long)(th * KW + tw) * 3 * cp + cb * 32;
          for (int rb = 0; rb < npad / 16; ++rb)
            for (int hf = 0; hf < 2; ++hf)
              for (int l = 0; l < 64; ++l)
                for (int j = 0; j < 8; ++j) {
                  const long long row = rb * 16 + (l & 15);
                  const long long k = kbase + (hf ? 2 * cp : 0) + (l >> 4) * 8 + j;
                  h[(size_t)(kt * tile_elems + ((long long)(rb * 2 + hf) * 64 + l) * 8 + j)] = (_Float16)wf[row * ktot + k];
                }
        }
    k0 += (long long)KH * KW * 3 * cp;
  }
  if (hipMalloc(out, h.size() * 2) != hipSuccess ||
      hipMemcpy(*out, h.data(), h.size() * 2, hipMemcpyHostToDevice) != hipSuccess)
    return fail(n->ctx, PC_ERR_HIP, "wfrag upload failed");
  return PC_OK;
}

// f16c8 conv weights: the program holds the split form [W_hi, W_hi, W_lo] per tap and
// segment; the W_lo block's bytes become, per 32 input channels, [W_hi8 x 32 | W_lo8 x 32] (e4m3 of
// W_hi * 2^sh and W_lo * 2^sl, one exponent pair per conv). *wf8s gets their E8M0 scales.
static int pack_c8_weights(pc_net* n, const NetOp& op, const float* wf, long long cnt, std::vector<_Float16>& h,
                           int* wf8s) {
  const int* w = op.w;
  const int npad = w[14];
  const long long ktot = w[15];
  if ((long long)npad * ktot != cnt) return fail(n->ctx, PC_ERR_FORMAT, "f16c8 weights: array size");
  float mh = 0.f, ml = 0.f;
  struct Blk { long long k0; int cp, taps; };
  std::vector<Blk> segs;
  long long k0 = 0;
  for (int sg = 0; sg < w[2]; ++sg) {
    const NetTensor& X = n->tens[w[3 + 5 * sg]];
    if (!X.c8) return fail(n->ctx, PC_ERR_FORMAT, "f16c8 weights: non-f16c8 segment");
    const int cp = X.C / 2, taps = w[4 + 5 * sg] * w[5 + 5 * sg];
    segs.push_back({k0, cp, taps});
    k0 += (long long)taps * 3 * cp;
  }
  if (k0 != ktot) return fail(n->ctx, PC_ERR_FORMAT, "f16c8 weights: K layout");
  for (const Blk& b : segs)
    for (int r = 0; r < npad; ++r)
      for (int t = 0; t < b.taps; ++t) {
        const float* row = wf + (long long)r * ktot + b.k0 + (long long)t * 3 * b.cp;
        for (int c = 0; c < b.cp; ++c) {
          mh = std::max(mh, std::fabs(row[c]));
          ml = std::max(ml, std::fabs(row[2 * b.cp + c]));
        }
      }
  // the largest magnitude of each half lands in [224, 448)
  const int sh = mh > 0.f ? (int)std::floor(std::log2(448.f / mh)) : 0;
  const int sl = ml > 0.f ? (int)std::floor(std::log2(448.f / ml)) : 0;
  if (127 - sh < 1 || 127 - sh > 254 || 127 - sl < 1 || 127 - sl > 254)
    return fail(n->ctx, PC_ERR_FORMAT, "f16c8 weights: scale out of range");
  for (const Blk& b : segs)
    for (int r = 0; r < npad; ++r)
      for (int t = 0; t < b.taps; ++t) {
        const long long base = (long long)r * ktot + b.k0 + (long long)t * 3 * b.cp;
        uint8_t* dst = reinterpret_cast<uint8_t*>(&h[base + 2 * b.cp]);
        for (int c = 0; c < b.cp; ++c) {
          dst[(c >> 5) * 64 + (c & 31)] = e4m3_encode(std::ldexp(wf[base + c], sh));
          dst[(c >> 5) * 64 + 32 + (c & 31)] = e4m3_encode(std::ldexp(wf[base + 2 * b.cp + c], sl));
        }
      }
  *wf8s = (127 - sh) | ((127 - sl) << 8);
  return PC_OK;
}

extern "C" int pc_net_create(pc_ctx* c, const void* prog, size_t nbytes, int precision, int max_batch, pc_net** out) {
  if (!c || !prog || !out || max_batch <= 0) return fail(c, PC_ERR_ARG, "pc_net_create: bad arguments");
  *out = nullptr;
  const int32_t* P = (const int32_t*)prog;
  const size_t nw = nbytes / 4;
  if (nw < 8 || P[0] != 0x544E4350 || P[1] != 1) return fail(c, PC_ERR_FORMAT, "bad program magic/version");
  HIPCHK(c, hipSetDevice(c->device));
  pc_net* n = new pc_net();
  n->ctx = c;
  n->f32 = precision == PC_PREC_F32;
  n->max_batch = max_batch;
  const int nbuf = P[2], nten = P[3], narr = P[4], nop = P[5], nout = P[6];
  n->in_tensor = P[7];
  size_t pos = 8;
  auto need = [&](size_t k) { return pos + k <= nw; };
  if (!need((size_t)nbuf * 4 + (size_t)nten * 8 + (size_t)narr * 4 + nout + (size_t)nop * 32)) {
    delete n;
    return fail(c, PC_ERR_FORMAT, "truncated program");
  }
  for (int i = 0; i < nbuf; ++i, pos += 4) {
    NetBuf b;
    b.elems = (long long)(uint32_t)P[pos] | ((long long)P[pos + 1] << 32);
    b.is_f32 = P[pos + 2];
    n->bufs.push_back(b);
  }
  for (int i = 0; i < nten; ++i, pos += 8) {
    NetTensor t{P[pos], P[pos + 1], P[pos + 2], P[pos + 3], P[pos + 4], P[pos + 5], P[pos + 6], P[pos + 7] & 1};
    t.c8 = (P[pos + 7] >> 2) & 1;
    if (i == n->in_tensor && (P[pos + 7] & 2)) n->in_centered = 1;
    n->tens.push_back(t);
  }
  std::vector<std::pair<long long, long long>> arr;
  for (int i = 0; i < narr; ++i, pos += 4) {
    long long off = (long long)(uint32_t)P[pos] | ((long long)P[pos + 1] << 32);
    long long cnt = (long long)(uint32_t)P[pos + 2] | ((long long)P[pos + 3] << 32);
    arr.push_back({off, cnt});
  }
  for (int i = 0; i < nout; ++i) n->outs.push_back(P[pos++]);
  for (int i = 0; i < nop; ++i, pos += 32) {
    NetOp op;
    memcpy(op.w, P + pos, 32 * 4);
    n->ops.push_back(op);
  }
  const float* data = (const float*)(P + pos);
  const size_t ndata = nw - pos;
  // f16x3 split tensors: f16 nets only; only convs, the fused stem and the max
  // pool read or write them
  for (auto& t : n->tens)
    if (t.split && (n->f32 || t.is_f32 || t.buf < 0 || t.C % 16 || t.cs != t.C)) {
      delete n;
      return fail(c, PC_ERR_FORMAT, "split tensor: f16 net, dense [hi | lo] activation buffer");
    }
  // f16c8 tensors: split storage of whole 32-channel blocks, written by convs and the fused stem,
  // read by convs (conv_fast C8) and as a conv residual
  for (auto& t : n->tens)
    if (t.c8 && (!t.split || (t.C / 2) % 32)) {
      delete n;
      return fail(c, PC_ERR_FORMAT, "f16c8 tensor: split storage of 32-channel blocks");
    }
  for (auto& op : n->ops) {
    const int k = op.w[0];
    auto c8t = [&](int t) { return t >= 0 && t < (int)n->tens.size() && n->tens[t].c8; };
    if ((k == OP_MAXPOOL || k == OP_UPSAMPLE || k == OP_LAYERNORM || k == OP_ATTENTION) && (c8t(op.w[1]) || c8t(op.w[2]))) {
      delete n;
      return fail(c, PC_ERR_FORMAT, "op cannot read or write f16c8 tensors");
    }
  }
  for (auto& op : n->ops) {
    const int k = op.w[0];
    auto bad = [&](int t) { return t >= 0 && t < (int)n->tens.size() && n->tens[t].split; };
    if ((k == OP_MAXPOOL && (n->tens[op.w[1]].split != n->tens[op.w[2]].split ||
                             (n->tens[op.w[2]].split && n->tens[op.w[1]].C != n->tens[op.w[2]].C))) ||
        ((k == OP_UPSAMPLE || k == OP_LAYERNORM || k == OP_ATTENTION) && (bad(op.w[1]) || bad(op.w[2]))) ||
        (k == OP_STEM && bad(op.w[2]))) {
      delete n;
      return fail(c, PC_ERR_FORMAT, "op cannot read or write split tensors");
    }
  }
  // which arrays are conv weights (uploaded in the activation dtype)
  std::vector<int> is_w(narr, 0), c8_op(narr, -1);
  n->wf8s.assign(n->ops.size(), 0);
  for (size_t i = 0; i < n->ops.size(); ++i) {
    const NetOp& op = n->ops[i];
    if (op.w[0] == OP_CONV && op.w[13] >= 0) {
      is_w[op.w[13]] = 1;
      if (op.w[2] >= 1 && n->tens[op.w[3]].c8) c8_op[op.w[13]] = (int)i;
    }
  }
  n->arrays.assign(narr, nullptr);
  n->array_count.assign(narr, 0);
  int rc = PC_OK;
  for (int i = 0; i < narr && rc == PC_OK; ++i) {
    const long long off = arr[i].first, cnt = arr[i].second;
    if (off < 0 || cnt < 0 || (size_t)(off + cnt) > ndata) { rc = fail(c, PC_ERR_FORMAT, "array out of range"); break; }
    n->array_count[i] = cnt;
    if (is_w[i] && !n->f32) {
      std::vector<_Float16> h(cnt);
      for (long long k = 0; k < cnt; ++k) h[k] = (_Float16)data[off + k];
      if (c8_op[i] >= 0 && (rc = pack_c8_weights(n, n->ops[c8_op[i]], data + off, cnt, h, &n->wf8s[c8_op[i]])) != PC_OK)
        break;
      if (hipMalloc(&n->arrays[i], cnt * 2 + 16) != hipSuccess ||
          hipMemcpy(n->arrays[i], h.data(), cnt * 2, hipMemcpyHostToDevice) != hipSuccess)
        rc = fail(c, PC_ERR_HIP, "weight upload failed");
    } else {
      if (hipMalloc(&n->arrays[i], cnt * 4 + 16) != hipSuccess ||
          hipMemcpy(n->arrays[i], data + off, cnt * 4, hipMemcpyHostToDevice) != hipSuccess)
        rc = fail(c, PC_ERR_HIP, "array upload failed");
    }
  }
  for (size_t i = 0; i < n->bufs.size() && rc == PC_OK; ++i) {
    NetBuf& b = n->bufs[i];
    const size_t bytes = (size_t)b.elems * max_batch * ((b.is_f32 || n->f32) ? 4 : 2) + kZeroTail;
    // the conv loader addresses activations with 32-bit offsets
    if (bytes >= (1ull << 32)) rc = fail(c, PC_ERR_ARG, "activation buffer exceeds 4 GiB; lower max_batch");
    else if (hipMalloc(&b.d, bytes) != hipSuccess) rc = fail(c, PC_ERR_HIP, "activation buffer allocation failed");
    else hipMemset(b.d, 0, bytes);  // channel padding lanes and the zero tail must read as zero
  }
  if (rc == PC_OK && n->in_tensor >= 0 && n->in_tensor < (int)n->tens.size()) {
    const NetTensor& I = n->tens[n->in_tensor];
    n->in_img_bytes = (size_t)I.H * I.W * I.cs * esize(n, I.is_f32);
    bool conv_reads_input = false;
    for (auto& op : n->ops)
      if (op.w[0] == OP_CONV)
        for (int s = 0; s < op.w[2]; ++s)
          if (n->tens[op.w[3 + 5 * s]].buf < 0) conv_reads_input = true;
    if (conv_reads_input) {
      const size_t bytes = n->in_img_bytes * max_batch + kZeroTail;
      if (bytes >= (1ull << 32)) rc = fail(c, PC_ERR_ARG, "input buffer exceeds 4 GiB; lower max_batch");
      else if (hipMalloc(&n->in_copy, bytes) != hipSuccess) rc = fail(c, PC_ERR_HIP, "input copy allocation failed");
      else hipMemset(n->in_copy, 0, bytes);
    }
  }
  // plans + split-K workspace + stats
  n->host_arrays.assign(narr, nullptr);
  for (int i = 0; i < narr; ++i) n->host_arrays[i] = data + arr[i].first;
  n->plans.resize(n->ops.size());
  // Small-batch classes 1, 4, 16, 32, 64 images up to a quarter of max_batch: a per-frame
  // extract() runs SCRFD on 1 image and ArcFace on 2 x its faces (2-30 rows); a net of 64
  // (SCRFD) keeps 1 / 4 / 16, so its 32-frame C3 chunks stay on the max-batch tiles (r03:
  // the 16-image tiles at 32 images cost 0.4 ms per step).
  n->cls_batch.clear();
  if (max_batch > 2 && !getenv("PC_NO_SMALL_PLANS")) {
    for (int b : {1, 4, 16, 32, 64})
      if (b <= std::max(1, max_batch / 4)) n->cls_batch.push_back(b);
    // f16x3 nets (ArcFace-x3 runs 256-row calls on a 512-row net: C3's 128-face quantum with flips):
    // plans for 128 rows and half the max batch too - a tile chosen for 512 rows runs 256 at half a
    // round (7x7x512: 248 vs 185 us, profiles/r05n_sx_tile_sweep.txt). Their convs keep the one K
    // order of every class (the fused tiles' K-row width is fixed per conv), so results stay bit-identical.
    bool has_split = false;
    for (auto& t : n->tens) has_split = has_split || t.split;
    if (has_split && max_batch >= 256)
      for (int b : {128, max_batch / 2})
        if (b > n->cls_batch.back()) n->cls_batch.push_back(b);
  }
  n->plans_cls.assign(n->cls_batch.size(), std::vector<ConvPlan>(n->ops.size()));
  n->stems.resize(n->ops.size());
  size_t part = 0, stem_col_bytes = 0;
  for (size_t i = 0; i < n->ops.size() && rc == PC_OK; ++i) {
    const NetOp& op = n->ops[i];
    if (op.w[0] == OP_CONV) {
      rc = plan_conv(n, op, n->plans[i], max_batch);
      if (rc) break;
      // small batches (per-frame extract: one frame's faces, prescan samples) get their own
      // tile choice: the max-batch tiles would leave most CUs idle
      for (size_t c = 0; c < n->cls_batch.size() && rc == PC_OK; ++c) {
        ConvPlan& sp = n->plans_cls[c][i];
        rc = plan_conv(n, op, sp, n->cls_batch[c], n->cls_batch[c] <= 64);
        if (rc == PC_OK && sp.splitk > 1)
          part = std::max(part, (size_t)((long long)sp.splitk * sp.M_per_image * n->cls_batch[c] * op.w[14] * 4));
      }
      if (rc) break;
      const ConvPlan& pl = n->plans[i];
      if (pl.splitk > 1) part = std::max(part, (size_t)((long long)pl.splitk * pl.M_per_image * max_batch * op.w[14] * 4));
      const NetTensor& Y = n->tens[op.w[1]];
      double macs = 0.0;
      for (int s = 0; s < op.w[2]; ++s) {
        const NetTensor& X = n->tens[op.w[3 + 5 * s]];
        (void)X;
        // algorithmic MACs: real output channels x real taps x input channels (padded lanes excluded by the
        // program: w[25+s] carries the true input channel count)
        const int cin_true = op.w[25 + s] > 0 ? op.w[25 + s] : X.C;
        const int cout_true = op.w[27] > 0 ? op.w[27] : op.w[16];
        macs += (double)Y.H * Y.W * cout_true * op.w[4 + 5 * s] * op.w[5 + 5 * s] * cin_true;
      }
      n->flops_per_image += 2.0 * macs;
      n->plans[i].flops_per_image = 2.0 * macs;
      n->launches += pl.splitk > 1 ? 2 : 1;
    } else if (op.w[0] == OP_STEM) {
      const NetTensor& Y = n->tens[op.w[1]];
      const int cin_true = op.w[13] > 0 ? op.w[13] : 3;
      n->flops_per_image += 2.0 * Y.H * Y.W * op.w[8] * op.w[3] * op.w[4] * cin_true;
      rc = plan_stem(n, op, n->stems[i], stem_col_bytes);
      n->plans[i].flops_per_image = 2.0 * Y.H * Y.W * op.w[8] * op.w[3] * op.w[4] * cin_true;
      n->launches += n->stems[i].use_mfma ? 2 : 1;
    } else if (op.w[0] == OP_MAXPOOL || op.w[0] == OP_UPSAMPLE || op.w[0] == OP_LAYERNORM) {
      n->launches += 1;
    } else if (op.w[0] == OP_ATTENTION) {
      const NetTensor& Q = n->tens[op.w[2]];
      const double T = (double)Q.H * Q.W;
      n->flops_per_image += 4.0 * T * T * op.w[3] * op.w[4];
      n->launches += 1;
    } else {
      rc = fail(c, PC_ERR_FORMAT, "unknown op type");
    }
  }
  // fragment-ordered weights for the convs any plan runs on the WG form
  n->wfrag.assign(n->ops.size(), nullptr);
  for (size_t i = 0; i < n->ops.size() && rc == PC_OK; ++i) {
    if (n->ops[i].w[0] != OP_CONV) continue;
    bool wg = n->plans[i].wg || n->plans[i].hx;   // (the halo-staged kernel reads the same copy)
    for (auto& pc : n->plans_cls) wg = wg || pc[i].wg || pc[i].hx;
    if (wg) rc = pack_wfrag(n, n->ops[i], reinterpret_cast<const float*>(n->host_arrays[n->ops[i].w[13]]), &n->wfrag[i]);
  }
  n->host_arrays.clear();
  if (rc == PC_OK) rc = plan_chains(n);
  if (rc == PC_OK && stem_col_bytes) {
    if (hipMalloc(&n->stem_col, stem_col_bytes) != hipSuccess) rc = fail(c, PC_ERR_HIP, "stem im2col workspace");
    else hipMemset(n->stem_col, 0, stem_col_bytes);
  }
  if (rc == PC_OK && part) {
    if (hipMalloc((void**)&n->partial, part) != hipSuccess) rc = fail(c, PC_ERR_HIP, "split-K workspace");
    n->partial_bytes = part;
  }
  if (rc != PC_OK) {
    pc_net_destroy(n);
    return rc;
  }
  *out = n;
  return PC_OK;
}

extern "C" int pc_net_destroy(pc_net* n) {
  if (!n) return PC_OK;
  hipSetDevice(n->ctx->device);
  hipStreamSynchronize(n->ctx->stream);
  for (auto& kv : n->graphs) hipGraphExecDestroy(kv.second);
  if (n->cap_stream) hipStreamDestroy(n->cap_stream);
  if (n->d_absmax) hipFree(n->d_absmax);
  for (void* a : n->arrays) if (a) hipFree(a);
  for (void* a : n->wfrag) if (a) hipFree(a);
  for (auto& b : n->bufs) if (b.d) hipFree(b.d);
  if (n->partial) hipFree(n->partial);
  if (n->prep) hipFree(n->prep);
  if (n->in_copy) hipFree(n->in_copy);
  for (auto& st : n->stems) {
    if (st.w) hipFree(st.w);
    if (st.bias) hipFree(st.bias);
    if (st.slope) hipFree(st.slope);
  }
  if (n->stem_col) hipFree(n->stem_col);
  for (auto& ch : n->chains) {
    if (ch.d_blk) hipFree(ch.d_blk);
    if (ch.d_wpack) hipFree(ch.d_wpack);
  }
  delete n;
  return PC_OK;
}

static int prof_event(pc_net* n, int* idx) {
  if (n->ev_used == n->ev_pool.size()) {
    hipEvent_t e;
    HIPCHK(n->ctx, hipEventCreate(&e));
    n->ev_pool.push_back(e);
  }
  *idx = (int)n->ev_used++;
  HIPCHK(n->ctx, hipEventRecord(n->ev_pool[*idx], n->ctx->stream));
  return PC_OK;
}

// plan class of a run of N images (-1: the max-batch plans)
static int plan_class(const pc_net* n, int N) {
  for (size_t c = 0; c < n->cls_batch.size(); ++c)
    if (N <= n->cls_batch[c]) return (int)c;
  return -1;
}

static int run_ops(pc_net* n, int N, hipStream_t s) {
  pc_ctx* c = n->ctx;
  // eager runs are profiled; a captured run records no events (its replays are not profiled)
  const bool prof = n->prof && !n->capturing;
  if (n->in_copy)
    HIPCHK(c, hipMemcpyAsync(n->in_copy, n->cur_input, n->in_img_bytes * N, hipMemcpyDeviceToDevice, s));
  // one event per op boundary: an op's end event is the next op's start event
  int open_ev = -1;
  for (size_t i = 0; i < n->ops.size(); ++i) {
    const int* w = n->ops[i].w;
    if (!n->chain_at.empty() && n->chain_at[i] >= 0 && N >= n->chain_min_batch) {
      // a run of identity blocks as one resident-chain launch (pc_conv_chain.hip)
      const ChainPlan& ch = n->chains[n->chain_at[i]];
      ProfRec rec{-1, -1, OP_CONV, ch.flops_per_image * N, (int)i, 300};
      if (prof) {
        if (open_ev >= 0) {
          rec.a = open_ev;
        } else {
          int rc = prof_event(n, &rec.a);
          if (rc) return rc;
        }
      }
      const NetTensor &TX = n->tens[ch.in_t], &TY = n->tens[ch.out_t];
      int dbg = ch.wl << 8;
      int mode = 1;   // LDS-DMA weight ring (measured faster than the register stream)
      if (const char* e = getenv("PC_CHAIN_MODE")) mode = atoi(e) ? 1 : 0;
      dbg |= mode << 10;
      if (const char* e = getenv("PC_CONV_DBG")) dbg |= atoi(e) & 7;
      HIPCHK(c, conv_chain_launch(tensor_ptr(n, ch.in_t), TX.cs, tensor_ptr(n, ch.out_t), TY.cs, ch.d_blk, ch.nblk, N,
                                  TX.H, TX.W, n->ops[i].w[15], dbg, s));
      if (prof) {
        int rc = prof_event(n, &rec.b);
        if (rc) return rc;
        n->recs.push_back(rec);
        open_ev = rec.b;
      }
      i += 2 * ch.nblk - 1;
      continue;
    }
    ProfRec rec{-1, -1, w[0], w[0] == OP_CONV ? n->plans[i].flops_per_image * N : 0.0, (int)i};
    if (prof) {
      if (open_ev >= 0) {
        rec.a = open_ev;
      } else {
        int rc = prof_event(n, &rec.a);
        if (rc) return rc;
      }
    }
    if (w[0] == OP_CONV) {
      const int cls = plan_class(n, N);
      const ConvPlan& pl = cls >= 0 ? n->plans_cls[cls][i] : n->plans[i];
      rec.small = cls;
      ConvParams p;
      memset(&p, 0, sizeof(p));
      const NetTensor& Y = n->tens[w[1]];
      p.nseg = w[2];
      const int bke = pl.rowb / (n->f32 ? 4 : 2);
      int kt = 0;
      for (int sg = 0; sg < p.nseg; ++sg) {
        const NetTensor& X = n->tens[w[3 + 5 * sg]];
        ConvSeg& S = p.seg[sg];
        S.x = tensor_ptr(n, w[3 + 5 * sg]);
        S.zero_off = tensor_zero_off(n, w[3 + 5 * sg]);
        S.H = X.H; S.W = X.W; S.C = X.C; S.cs = X.cs;
        S.KH = w[4 + 5 * sg]; S.KW = w[5 + 5 * sg]; S.stride = w[6 + 5 * sg]; S.pad = w[7 + 5 * sg];
        S.cblk = X.C / bke;
        if (X.c8) S.f8s = (127 - X.e_lo) | ((127 - X.e_hi) << 8);
        if (X.split && pl.sx) {   // fused split tiles: the hi blocks; lo block = hi block + vwrap
          S.cblk = S.cblk / 2;
          S.vwrap = S.cblk;
          // channel groups of 64 hi channels where they divide the channels (ConvSeg::gt)
          S.gt = (X.C / 2) % 64 == 0 ? 64 / bke : 1;
        } else if (X.split) {     // virtual channel blocks [hi, lo, hi] (pc_common.h ConvSeg::vwrap)
          S.vwrap = S.cblk;
          S.cblk = S.cblk / 2 * 3;
        }
        S.kt = S.KH * S.KW * S.cblk;
        kt += S.kt;
      }
      p.w = n->arrays[w[13]];
      p.ktot = w[15];
      p.N = N; p.OH = Y.H; p.OW = Y.W; p.M = N * Y.H * Y.W;
      p.npad = w[14];
      p.cout = w[16];
      p.cwrite = std::min(Y.split ? Y.C / 2 : Y.C, p.npad);
      p.ysplit = Y.split ? Y.C / 2 : 0;
      p.y = tensor_ptr(n, w[1]);
      p.ycs = Y.cs;
      p.out_f32 = Y.is_f32 && !n->f32 ? 1 : (n->f32 ? 1 : 0);
      p.bias = w[17] >= 0 ? (const float*)n->arrays[w[17]] : nullptr;
      p.bias_mode = w[17] >= 0 ? w[18] : 0;
      p.slope = w[19] >= 0 ? (const float*)n->arrays[w[19]] : nullptr;
      p.act = w[20];
      p.res = w[21] >= 0 ? tensor_ptr(n, w[21]) : nullptr;
      p.res_mode = w[21] >= 0 ? w[22] : 0;
      if (w[21] >= 0) {
        const NetTensor& R = n->tens[w[21]];
        p.rcs = R.cs; p.rH = R.H; p.rW = R.W;
        p.rsplit = R.split ? R.C / 2 : 0;
      }
      p.act_after_res = w[23];
      p.kt_total = kt;
      p.sx = pl.sx;
      p.c8 = pl.c8;
      p.wf8s = n->wf8s[i];
      p.wfrag = pl.wg || pl.hx ? n->wfrag[i] : nullptr;
      if (Y.c8) {
        p.yc8 = 1;
        p.ylo_mul = std::ldexp(1.f, Y.e_lo);
        p.yhi_mul = std::ldexp(1.f, Y.e_hi);
      }
      if (w[21] >= 0 && n->tens[w[21]].c8) {
        p.rc8 = 1;
        p.rlo_inv = std::ldexp(1.f, -n->tens[w[21]].e_lo);
      }
      p.splitk = pl.splitk;
      p.partial = n->partial;
      p.zero = c->zero;
      if (const char* e = getenv("PC_CONV_DBG")) p.dbg = atoi(e);
      if (pl.hx >= 3 && pl.hx != 5) {
        HIPCHK(c, conv_hxi_launch(p, pl.hx >= 7, s));
      } else if (pl.hx == 2 || pl.hx == 5) {
        HIPCHK(c, conv_hxg_launch(p, pl.hx == 5, s));
      } else if (pl.hx) {
        HIPCHK(c, conv_hx_launch(p, s));
      } else if (pl.t2d >= 0) {
        HIPCHK(c, conv_t2d_launch(p, pl.t2d, s));
      } else if (pl.fast >= 0) {
        HIPCHK(c, conv_fast_launch(n->f32, pl.rowb, pl.fast, p, s));
      } else if (pl.halo >= 0) {
        HIPCHK(c, conv_halo_launch(n->f32, pl.halo, p, s));
      } else {
        HIPCHK(c, conv_launch(n->f32, pl.rowb, pl.cfg, p, s));
      }
      if (pl.splitk > 1) {
        HIPCHK(c, splitk_finish_launch(n->f32, p, s));
      }
    } else if (w[0] == OP_STEM) {
      StemParams p;
      memset(&p, 0, sizeof(p));
      const NetTensor& X = n->tens[w[2]];
      const NetTensor& Y = n->tens[w[1]];
      p.x = tensor_ptr(n, w[2]);
      p.N = N; p.H = X.H; p.W = X.W; p.cin = X.C; p.xcs = X.cs;
      p.OH = Y.H; p.OW = Y.W; p.KH = w[3]; p.KW = w[4]; p.stride = w[5]; p.pad = w[6];
      p.w = (const float*)n->arrays[w[7]];
      p.cout = w[8];
      p.bias = (const float*)n->arrays[w[9]];
      p.slope = w[10] >= 0 ? (const float*)n->arrays[w[10]] : nullptr;
      p.act = w[11];
      p.ycs = Y.cs;
      p.cpad = w[12];
      p.y = tensor_ptr(n, w[1]);
      const StemPlan& st = n->stems[i];
      const int st_cwrite = std::min(Y.split ? Y.C / 2 : Y.C, st.npad);
      p.ysplit = Y.split ? Y.C / 2 : 0;
      if (Y.c8) {
        p.yc8 = 1;
        p.ylo_mul = std::ldexp(1.f, Y.e_lo);
        p.yhi_mul = std::ldexp(1.f, Y.e_hi);
      }
      // fused gather + MFMA stem (pc_stem.hip) unless PC_STEM_UNFUSED is set
      // (stem_fused stores f16: an f32 output tensor inside an f16 net takes the unfused path)
      const bool fused = st.use_mfma && !getenv("PC_STEM_UNFUSED") && !Y.is_f32 &&
                         stem_fused_ok(n->f32, X.C, st.cin_true, p.KH, p.KW, st.npad, st_cwrite, Y.cs, Y.coff) &&
                         X.cs % 4 == 0 && (reinterpret_cast<uintptr_t>(p.x) & 7) == 0 &&
                         (reinterpret_cast<uintptr_t>(p.y) & 15) == 0;
      if (st.split && !fused) return fail(c, PC_ERR_FORMAT, "split stem: the fused kernel cannot run this op");
      if (fused) {
        rec.kind = OP_CONV;
        rec.flops = n->plans[i].flops_per_image * N;
        HIPCHK(c, stem_fused_launch(p, st.w, st.bias, st.slope, st.npad, st_cwrite, s));
      } else if (!st.use_mfma) {
        HIPCHK(c, stem_launch(n->f32, p, s));
      } else {
        HIPCHK(c, stem_im2col_launch(n->f32, p, st.cin_true, n->stem_col, s));
        if (prof) {   // im2col counts as "other", the MFMA part as a conv launch
          int rc = prof_event(n, &rec.b);
          if (rc) return rc;
          n->recs.push_back(rec);
          const int b = rec.b;
          rec = ProfRec{b, -1, OP_CONV, n->plans[i].flops_per_image * N, (int)i};
        }
        ConvParams q;
        memset(&q, 0, sizeof(q));
        q.nseg = 1;
        ConvSeg& S = q.seg[0];
        S.x = n->stem_col;
        S.H = Y.H; S.W = Y.W; S.C = 32; S.cs = 32;
        S.KH = 1; S.KW = 1; S.stride = 1; S.pad = 0;
        S.cblk = 1; S.kt = 1;
        S.zero_off = (unsigned)((size_t)N * Y.H * Y.W * 32 * (n->f32 ? 4 : 2));
        q.w = st.w; q.ktot = 32;
        q.N = N; q.OH = Y.H; q.OW = Y.W; q.M = N * Y.H * Y.W;
        q.npad = st.npad; q.cout = p.cout; q.cwrite = std::min(Y.C, st.npad);
        q.y = p.y; q.ycs = Y.cs; q.out_f32 = n->f32 ? 1 : (Y.is_f32 ? 1 : 0);
        q.bias = st.bias; q.bias_mode = BIAS_CHANNEL;
        q.slope = st.slope; q.act = p.act;
        q.kt_total = 1; q.splitk = 1;
        // the statically scheduled kernel's 64x256 tile when it divides the channels
        if (st.npad % 64 == 0 && conv_fast_valid(4, st.rowb) && !getenv("PC_STEM_GENERIC"))
          HIPCHK(c, conv_fast_launch(n->f32, st.rowb, 4, q, s));
        else
          HIPCHK(c, conv_launch(n->f32, st.rowb, st.cfg, q, s));
      }
    } else if (w[0] == OP_MAXPOOL) {
      PoolParams p;
      const NetTensor& X = n->tens[w[2]];
      const NetTensor& Y = n->tens[w[1]];
      p.x = tensor_ptr(n, w[2]); p.N = N; p.H = X.H; p.W = X.W; p.C = X.C; p.xcs = X.cs;
      p.y = tensor_ptr(n, w[1]); p.OH = Y.H; p.OW = Y.W; p.ycs = Y.cs;
      p.k = w[3]; p.stride = w[4]; p.pad = w[5];
      p.split = X.split;
      if (X.split) p.C = X.C / 2;   // the hi half; lo at +C (create checked Y.split == X.split)
      HIPCHK(c, maxpool_launch(n->f32, p, s));
    } else if (w[0] == OP_UPSAMPLE) {
      UpsampleParams p;
      const NetTensor& X = n->tens[w[2]];
      const NetTensor& Y = n->tens[w[1]];
      p.x = tensor_ptr(n, w[2]); p.N = N; p.H = X.H; p.W = X.W; p.C = std::min(X.C, Y.C); p.xcs = X.cs;
      p.y = tensor_ptr(n, w[1]); p.ycs = Y.cs;
      HIPCHK(c, upsample2_launch(n->f32, p, s));
    } else if (w[0] == OP_LAYERNORM) {
      LayerNormParams p;
      const NetTensor& X = n->tens[w[2]];
      const NetTensor& Y = n->tens[w[1]];
      p.x = tensor_ptr(n, w[2]); p.xcs = X.cs;
      p.y = tensor_ptr(n, w[1]); p.ycs = Y.cs;
      p.M = N * X.H * X.W; p.C = w[8]; p.cwrite = Y.C;
      p.gamma = (const float*)n->arrays[w[3]];
      p.beta = (const float*)n->arrays[w[4]];
      p.add = w[5] >= 0 ? (const float*)n->arrays[w[5]] : nullptr;
      p.rows = w[5] >= 0 ? w[6] : 1;
      memcpy(&p.eps, &w[7], 4);
      HIPCHK(c, layernorm_launch(n->f32, p, s));
    } else if (w[0] == OP_ATTENTION) {
      AttnParams p;
      const NetTensor& Q = n->tens[w[2]];
      const NetTensor& O = n->tens[w[1]];
      p.qkv = tensor_ptr(n, w[2]); p.qcs = Q.cs;
      p.out = tensor_ptr(n, w[1]); p.ocs = O.cs;
      p.N = N; p.T = Q.H * Q.W; p.heads = w[3];
      p.scale = 1.0f / sqrtf((float)w[4]);
      HIPCHK(c, attention_launch(n->f32, p, w[4], s));
    }
    if (n->calib && (w[0] == OP_CONV || w[0] == OP_STEM)) {   // pc_net_calibrate: max |x| of the op's output
      const NetTensor& Y = n->tens[w[1]];
      if (!Y.is_f32 && !n->f32)
        HIPCHK(c, absmax_f16_launch(tensor_ptr(n, w[1]), (long long)N * Y.H * Y.W, Y.split ? Y.C / 2 : Y.C, Y.cs,
                                    reinterpret_cast<unsigned*>(n->d_absmax) + w[1], s));
    }
    if (prof) {
      int rc = prof_event(n, &rec.b);
      if (rc) return rc;
      n->recs.push_back(rec);
      open_ev = rec.b;
    }
  }
  return PC_OK;
}

// f16c8 scale calibration: one eager run over N images records every conv / stem
// output's largest magnitude; each f16c8 tensor then gets e_hi with max * 2^e_hi in
// [448 / 2^(headroom+1), 448 / 2^headroom) and e_lo = e_hi + 11 (|lo| <= 2^-11 |x|). The
// activations may grow 2^headroom times past the calibration before the e4m3 bytes saturate.
extern "C" int pc_net_calibrate(pc_net* n, const void* d_in, int N, int headroom_log2, float* h_absmax) {
  if (!n || !d_in || N <= 0 || N > n->max_batch || headroom_log2 < 0 || headroom_log2 > 8) return PC_ERR_ARG;
  pc_ctx* c = n->ctx;
  std::lock_guard<std::mutex> lk(n->graph_mu);
  const size_t nt = n->tens.size();
  if (!n->d_absmax) HIPCHK(c, hipMalloc((void**)&n->d_absmax, nt * 4));
  HIPCHK(c, hipMemsetAsync(n->d_absmax, 0, nt * 4, c->stream));
  n->cur_input = d_in;
  n->calib = 1;
  const int rc = run_ops(n, N, c->stream);
  n->calib = 0;
  if (rc) return rc;
  std::vector<float> mx(nt);
  HIPCHK(c, hipMemcpyAsync(mx.data(), n->d_absmax, nt * 4, hipMemcpyDeviceToHost, c->stream));
  HIPCHK(c, hipStreamSynchronize(c->stream));
  for (size_t t = 0; t < nt; ++t) {
    NetTensor& T = n->tens[t];
    if (h_absmax) h_absmax[t] = mx[t];
    if (!T.c8 || !(mx[t] > 0.f) || !std::isfinite(mx[t])) continue;
    const int e = (int)std::floor(std::log2(448.f / mx[t])) - headroom_log2;
    if (127 - e < 1 || 127 - (e + 11) < 1 || 127 - e > 254) return fail(c, PC_ERR_FORMAT, "f16c8 scale out of range");
    T.e_hi = e;
    T.e_lo = e + 11;
  }
  // captured graphs hold the old scales as kernel arguments
  for (auto& kv : n->graphs) hipGraphExecDestroy(kv.second);
  n->graphs.clear();
  return PC_OK;
}

extern "C" int pc_net_profile(pc_net* n, int enable) {
  if (!n) return PC_ERR_ARG;
  HIPCHK(n->ctx, hipStreamSynchronize(n->ctx->stream));
  n->prof = enable ? 1 : 0;
  n->ev_used = 0;
  n->recs.clear();
  return PC_OK;
}

extern "C" int pc_net_profile_read(pc_net* n, double* out) {
  if (!n || !out) return PC_ERR_ARG;
  HIPCHK(n->ctx, hipStreamSynchronize(n->ctx->stream));
  double conv_ms = 0, other_ms = 0, flops = 0;
  int conv_n = 0, other_n = 0;
  for (const ProfRec& r : n->recs) {
    float ms = 0.f;
    HIPCHK(n->ctx, hipEventElapsedTime(&ms, n->ev_pool[r.a], n->ev_pool[r.b]));
    if (r.kind == OP_CONV) { conv_ms += ms; conv_n++; flops += r.flops; }
    else { other_ms += ms; other_n++; }
  }
  out[0] = conv_ms; out[1] = conv_n; out[2] = flops; out[3] = other_ms; out[4] = other_n;
  return PC_OK;
}

// Per-record detail of the profiled runs: 6 doubles per record
// [op index, kind, ms, flops, kernel (100+k fast tile k, 200+v t2d variant v, 300 resident chain, 500 halo-staged f16x3, k halo tile k, -1 igemm), igemm cfg or the conv_fast form: bit 0 fused split, bit 1 register weight fragments, bit 2 128-byte K rows]; returns the count.
extern "C" int pc_net_profile_ops(pc_net* n, double* out, int max_recs) {
  if (!n || !out) return -PC_ERR_ARG;
  HIPCHK(n->ctx, hipStreamSynchronize(n->ctx->stream));
  int k = 0;
  for (const ProfRec& r : n->recs) {
    if (k >= max_recs) break;
    float ms = 0.f;
    HIPCHK(n->ctx, hipEventElapsedTime(&ms, n->ev_pool[r.a], n->ev_pool[r.b]));
    double* o = out + 6 * k++;
    const bool conv = r.op >= 0 && n->ops[r.op].w[0] == OP_CONV;
    o[0] = r.op; o[1] = r.kind; o[2] = ms; o[3] = r.flops;
    const ConvPlan* pl = conv ? (r.small >= 0 ? &n->plans_cls[r.small][r.op] : &n->plans[r.op]) : nullptr;
    o[4] = r.code >= 0 ? r.code
                       : conv ? (pl->hx            ? 499 + pl->hx   // 500 conv_hx64, 501 conv_hxg, 502 / 503 / 505 conv_hxi 14x14 / 28x28 / 7x7, 506-508 their small-batch forms
                                 : pl->c8          ? 600 + pl->fast
                                 : pl->t2d >= 0    ? 200 + pl->t2d
                                 : pl->fast >= 0   ? 100 + pl->fast
                                                   : pl->halo)
                              : -1;
    // [5]: the generic kernel's tile cfg; for conv_fast launches its form: bit 0 fused split (SX),
    // bit 1 register weight fragments (WG), bit 2 128-byte K rows
    const bool fastk = conv && r.code < 0 && !pl->hx && pl->t2d < 0 && pl->fast >= 0;
    o[5] = !conv ? -1 : fastk ? (pl->sx ? 1 : 0) + (pl->wg ? 2 : 0) + (pl->rowb == 128 ? 4 : 0) : pl->cfg;
  }
  return k;
}

extern "C" int pc_net_run(pc_net* n, const void* d_in, int N) {
  if (!n || !d_in) return PC_ERR_ARG;
  pc_ctx* c = n->ctx;
  if (N <= 0 || N > n->max_batch) return fail(c, PC_ERR_ARG, "batch out of range");
  n->cur_input = d_in;
  // (profiling runs eagerly: the per-op HIP events are the point of it)
  if (!n->use_graph || N > n->graph_max_batch || n->prof) return run_ops(n, N, c->stream);
  // Graphs are captured on a stream private to the net, never on the context stream: a context
  // (and its stream) is shared by every FaceEmbedder of the process, and work another host thread
  // enqueued there during an open capture would be recorded into this graph (not run now, replayed
  // later) or invalidate it. Capturing executes nothing, so the private stream needs no ordering
  // with the context stream; the instantiated graph is launched on the context stream. The lock
  // serialises capture and the graph table of one net between host threads.
  std::lock_guard<std::mutex> lk(n->graph_mu);
  auto key = std::make_pair(N, d_in);
  auto it = n->graphs.find(key);
  if (it == n->graphs.end()) {
    // (bounded: a graph per (batch, input) pair; callers with many batch sizes start over at 256)
    if (n->graphs.size() >= 256) {
      HIPCHK(c, hipStreamSynchronize(c->stream));   // (launched graphs may still run)
      for (auto& kv : n->graphs) hipGraphExecDestroy(kv.second);
      n->graphs.clear();
    }
    if (!n->cap_stream) HIPCHK(c, hipStreamCreateWithFlags(&n->cap_stream, hipStreamNonBlocking));
    hipGraph_t g = nullptr;
    HIPCHK(c, hipStreamBeginCapture(n->cap_stream, hipStreamCaptureModeThreadLocal));
    n->capturing = 1;
    int rc = run_ops(n, N, n->cap_stream);
    n->capturing = 0;
    hipError_t e = hipStreamEndCapture(n->cap_stream, &g);
    if (rc != PC_OK || e != hipSuccess) {   // a failed capture leaves no graph behind
      if (g) hipGraphDestroy(g);
      if (rc != PC_OK) return rc;
      return fail(c, PC_ERR_HIP, std::string("graph capture: ") + hipGetErrorString(e));
    }
    hipGraphExec_t ge;
    e = hipGraphInstantiate(&ge, g, nullptr, nullptr, 0);
    hipGraphDestroy(g);
    if (e != hipSuccess) return fail(c, PC_ERR_HIP, std::string("graph instantiate: ") + hipGetErrorString(e));
    it = n->graphs.emplace(key, ge).first;
  }
  HIPCHK(c, hipGraphLaunch(it->second, c->stream));
  return PC_OK;
}

extern "C" int pc_net_set_graph(pc_net* n, int enable) {
  if (!n) return PC_ERR_ARG;
  n->use_graph = enable ? 1 : 0;
  return PC_OK;
}
extern "C" int pc_net_set_graph_max_batch(pc_net* n, int32_t max_batch) {
  if (!n || max_batch < 1) return PC_ERR_ARG;
  n->graph_max_batch = max_batch;
  return PC_OK;
}

extern "C" int pc_net_input_dims(pc_net* n, int32_t* d) {
  if (!n || !d) return PC_ERR_ARG;
  const NetTensor& T = n->tens[n->in_tensor];
  d[0] = T.H; d[1] = T.W; d[2] = T.C; d[3] = T.cs;
  return PC_OK;
}
extern "C" int pc_net_num_outputs(pc_net* n) { return n ? (int)n->outs.size() : -1; }
extern "C" int pc_net_output(pc_net* n, int idx, void** d_ptr, int32_t* dims) {
  if (!n || idx < 0 || idx >= (int)n->outs.size()) return PC_ERR_ARG;
  const int t = n->outs[idx];
  const NetTensor& T = n->tens[t];
  if (d_ptr) *d_ptr = tensor_ptr(n, t);
  if (dims) { dims[0] = T.H; dims[1] = T.W; dims[2] = T.C; dims[3] = T.cs; dims[4] = (T.is_f32 || n->f32) ? 1 : 0; }
  return PC_OK;
}
extern "C" int pc_net_chain_info(pc_net* n, int32_t* min_batch, int32_t* per_round) {
  if (!n) return -PC_ERR_ARG;
  int ncu = 256;
  if (hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, n->ctx->device) != hipSuccess || ncu <= 0)
    ncu = 256;
  if (min_batch) *min_batch = n->chain_min_batch;
  if (per_round) *per_round = ncu;
  return (int)n->chains.size();
}
extern "C" int pc_net_set_chain_min_batch(pc_net* n, int32_t min_batch) {
  if (!n) return -PC_ERR_ARG;
  const int v = min_batch <= 0 ? (1 << 30) : min_batch;
  if (v != n->chain_min_batch) {
    // captured graphs replay the launch schedule of their capture (chain or per-conv)
    hipStreamSynchronize(n->ctx->stream);
    for (auto& kv : n->graphs) hipGraphExecDestroy(kv.second);
    n->graphs.clear();
  }
  n->chain_min_batch = v;
  return 0;
}
extern "C" int pc_net_stats(pc_net* n, double* flops, int32_t* launches) {
  if (!n) return PC_ERR_ARG;
  if (flops) *flops = n->flops_per_image;
  if (launches) *launches = n->launches;
  return PC_OK;
}

// ===========================================================================
// image / detection / embedding entry points
// ===========================================================================
extern "C" int pc_letterbox(pc_ctx* c, int prec, const pc_letterbox_desc* h, int n, int D, void* d_out) {
  if (!c || !h || n <= 0 || D <= 0 || !d_out) return fail(c, PC_ERR_ARG, "pc_letterbox: bad arguments");
  void* dd;
  int rc = stage_copy(c, h, sizeof(pc_letterbox_desc) * n, &dd);
  if (rc) return rc;
  HIPCHK(c, letterbox_launch(prec == PC_PREC_F32, (const LetterboxDesc*)dd, n, D, d_out, c->stream));
  return PC_OK;
}

extern "C" int pc_resize_linear(pc_ctx* c, const pc_resize_desc* h, int n) {
  if (!c || !h || n < 0) return fail(c, PC_ERR_ARG, "pc_resize_linear: bad arguments");
  if (n == 0) return PC_OK;
  int maxpix = 0;
  for (int i = 0; i < n; ++i) maxpix = std::max(maxpix, h[i].new_w * h[i].new_h);
  void* dd;
  int rc = stage_copy(c, h, sizeof(pc_resize_desc) * n, &dd);
  if (rc) return rc;
  HIPCHK(c, resize_linear_launch((const ResizeDesc*)dd, n, maxpix, c->stream));
  return PC_OK;
}

extern "C" int pc_warp_affine(pc_ctx* c, const pc_warp_desc* h, int n) {
  if (!c || !h || n < 0) return fail(c, PC_ERR_ARG, "pc_warp_affine: bad arguments");
  if (n == 0) return PC_OK;
  int maxpix = 0;
  for (int i = 0; i < n; ++i) maxpix = std::max(maxpix, h[i].out_w * h[i].out_h);
  void* dd;
  int rc = stage_copy(c, h, sizeof(pc_warp_desc) * n, &dd);
  if (rc) return rc;
  HIPCHK(c, warp_launch((const WarpDesc*)dd, n, maxpix, c->stream));
  return PC_OK;
}

extern "C" int pc_face_quality(pc_ctx* c, const uint8_t* chips, int n, int side, double* out) {
  if (!c || n < 0 || side <= 0 || side > 128) return fail(c, PC_ERR_ARG, "pc_face_quality: bad arguments");
  if (n == 0) return PC_OK;
  HIPCHK(c, quality_launch(chips, n, side, out, c->stream));
  return PC_OK;
}

extern "C" int pc_arcface_prep(pc_ctx* c, int prec, const uint8_t* chips, int n, int side, int flip, void* out) {
  if (!c || n < 0) return fail(c, PC_ERR_ARG, "pc_arcface_prep: bad arguments");
  if (n == 0) return PC_OK;
  if (prec != PC_PREC_F16 && prec != PC_PREC_F32 && prec != PC_PREC_F16X3)
    return fail(c, PC_ERR_ARG, "pc_arcface_prep: bad precision");
  HIPCHK(c, arcprep_launch(prec, chips, n, side, flip, out, c->stream));
  return PC_OK;
}

extern "C" int pc_rotate_pad(pc_ctx* c, const uint8_t* src, int H, int W, int row_stride, int deg, int pad,
                             uint8_t* dst) {
  if (!c || !src || !dst || H <= 0 || W <= 0 || pad < 0 || (deg != 0 && deg != 90 && deg != 180 && deg != 270))
    return fail(c, PC_ERR_ARG, "pc_rotate_pad: bad arguments");
  const int RH = (deg == 90 || deg == 270) ? W : H;
  const int RW = (deg == 90 || deg == 270) ? H : W;
  HIPCHK(c, rotate_pad_launch(src, H, W, row_stride, deg, pad, dst, RH + 2 * pad, RW + 2 * pad, c->stream));
  return PC_OK;
}

extern "C" int pc_resize_area_batch(pc_ctx* c, const uint8_t* const* srcs, uint8_t* const* dsts, int n, int row_stride,
                                    const pc_area_tab* xt, const int32_t* xs, int n_x, const pc_area_tab* yt,
                                    const int32_t* ys, int n_y, int OH, int OW);

extern "C" int pc_resize_area(pc_ctx* c, const uint8_t* src, int row_stride, const pc_area_tab* xt,
                              const int32_t* xs, int n_x, const pc_area_tab* yt, const int32_t* ys, int n_y,
                              uint8_t* dst, int OH, int OW) {
  if (!c || !src || !dst || !xt || !xs || !yt || !ys) return fail(c, PC_ERR_ARG, "pc_resize_area: bad arguments");
  return pc_resize_area_batch(c, &src, &dst, 1, row_stride, xt, xs, n_x, yt, ys, n_y, OH, OW);
}

// LDS span of resize_area_rows_u8: the widest 256-pixel output group's source bytes from a 16-byte
// boundary to one past its last byte rounded up to 16
static int area_span_bytes(const pc_area_tab* xt, const int32_t* xs, int OW) {
  int m = 0;
  for (int x0 = 0; x0 < OW; x0 += 256) {
    const int xl = std::min(x0 + 255, OW - 1);
    const int c0 = xt[xs[x0]].si, c1 = xt[xs[xl + 1] - 1].si;
    m = std::max(m, ((c1 * 3 + 3 + 15) & ~15) - ((c0 * 3) & ~15));
  }
  return m;
}

extern "C" int pc_resize_area_batch(pc_ctx* c, const uint8_t* const* srcs, uint8_t* const* dsts, int n, int row_stride,
                                    const pc_area_tab* xt, const int32_t* xs, int n_x, const pc_area_tab* yt,
                                    const int32_t* ys, int n_y, int OH, int OW) {
  if (!c || !srcs || !dsts || !xt || !xs || !yt || !ys || n < 0 || OH <= 0 || OW <= 0 || n_x <= 0 || n_y <= 0)
    return fail(c, PC_ERR_ARG, "pc_resize_area_batch: bad arguments");
  if (n == 0) return PC_OK;
  bool aligned = row_stride % 16 == 0;
  for (int i = 0; i < n; ++i) {
    if (!srcs[i] || !dsts[i]) return fail(c, PC_ERR_ARG, "pc_resize_area_batch: null frame");
    aligned = aligned && ((uintptr_t)srcs[i] & 15) == 0;
  }
  const int span = area_span_bytes(xt, xs, OW);
  void *dxt, *dxs, *dyt, *dys;
  int rc;
  if ((rc = stage_copy(c, xt, sizeof(pc_area_tab) * n_x, &dxt))) return rc;
  if ((rc = stage_copy(c, xs, sizeof(int32_t) * (OW + 1), &dxs))) return rc;
  if ((rc = stage_copy(c, yt, sizeof(pc_area_tab) * n_y, &dyt))) return rc;
  if ((rc = stage_copy(c, ys, sizeof(int32_t) * (OH + 1), &dys))) return rc;
  const bool direct = getenv("PC_AREA_DIRECT") && atoi(getenv("PC_AREA_DIRECT")) != 0;   // (A/B: per-pixel kernel)
  if (aligned && span <= 8192 && !direct) {   // (pc_image.hip AREA_ROWB: 4K -> 416 spans ~7.1 KB)
    std::vector<const void*> jobs(2 * (size_t)n);
    for (int i = 0; i < n; ++i) { jobs[2 * i] = srcs[i]; jobs[2 * i + 1] = dsts[i]; }
    void* dj;
    if ((rc = stage_copy(c, jobs.data(), sizeof(void*) * jobs.size(), &dj))) return rc;
    HIPCHK(c, resize_area_rows_launch(dj, n, row_stride, (const AreaTab*)dxt, (const int*)dxs, (const AreaTab*)dyt,
                                      (const int*)dys, OH, OW, span, c->stream));
    return PC_OK;
  }
  for (int i = 0; i < n; ++i)   // unaligned frames: the per-pixel kernel
    HIPCHK(c, resize_area_launch(srcs[i], row_stride, (const AreaTab*)dxt, (const int*)dxs, (const AreaTab*)dyt,
                                 (const int*)dys, dsts[i], OH, OW, c->stream));
  return PC_OK;
}

extern "C" int pc_resize_area_fast(pc_ctx* c, const uint8_t* src, int row_stride, int isx, int isy, uint8_t* dst,
                                   int OH, int OW) {
  if (!c || !src || !dst || isx < 1 || isy < 1 || OH <= 0 || OW <= 0)
    return fail(c, PC_ERR_ARG, "pc_resize_area_fast: bad arguments");
  HIPCHK(c, resize_area_fast_launch(src, row_stride, isx, isy, dst, OH, OW, c->stream));
  return PC_OK;
}

extern "C" int pc_embed_finalize(pc_ctx* c, const float* e, int ld, int n, int dim, int flip, float* out) {
  if (!c || n < 0) return fail(c, PC_ERR_ARG, "pc_embed_finalize: bad arguments");
  if (n == 0) return PC_OK;
  HIPCHK(c, embed_finalize_launch(e, ld, n, dim, flip, out, c->stream));
  return PC_OK;
}

extern "C" int pc_bank_match(pc_ctx* c, const float* q, int n, const float* bank, int b, int dim, float* fd,
                             int32_t* idx) {
  if (!c || n < 0 || b < 0 || dim <= 0) return fail(c, PC_ERR_ARG, "pc_bank_match: bad arguments");
  if (n == 0) return PC_OK;
  HIPCHK(c, bank_match_launch(q, n, bank, b, dim, fd, idx, c->stream));
  return PC_OK;
}

extern "C" int pc_arcface_embed(pc_net* net, const uint8_t* chips, int n, int flip, float* feat) {
  if (!net || n < 0) return PC_ERR_ARG;
  pc_ctx* c = net->ctx;
  if (n == 0) return PC_OK;
  const int rows = flip ? 2 * n : n;
  if (rows > net->max_batch) return fail(c, PC_ERR_ARG, "pc_arcface_embed: 2n exceeds the net's max batch");
  const NetTensor& I = net->tens[net->in_tensor];
  if (I.C != 4 || I.H != I.W) return fail(c, PC_ERR_FORMAT, "arcface net input must be square NHWC4");
  const size_t need = (size_t)net->max_batch * I.H * I.W * 4 * (net->f32 ? 4 : 2);
  if (net->prep_bytes < need) {
    if (net->prep) HIPCHK(c, hipFree(net->prep));
    HIPCHK(c, hipMalloc(&net->prep, need));
    net->prep_bytes = need;
  }
  HIPCHK(c, arcprep_launch(net->f32 ? PC_PREC_F32 : (net->in_centered ? PC_PREC_F16X3 : PC_PREC_F16), chips, n, I.H,
                           flip, net->prep, c->stream));
  int rc = pc_net_run(net, net->prep, rows);
  if (rc) return rc;
  const NetTensor& O = net->tens[net->outs[0]];
  const float* e = (const float*)tensor_ptr(net, net->outs[0]);
  HIPCHK(c, embed_finalize_launch(e, O.cs, n, O.C, flip, feat, c->stream));
  return PC_OK;
}

extern "C" int pc_scrfd_detect(pc_net* net, const pc_letterbox_desc* h, int n, int D, float det_thresh,
                               float nms_thresh, const float* h_det_scale, int max_det, float* dets, float* kps,
                               int32_t* count, int32_t* ncand) {
  if (!net || !h || n <= 0 || !h_det_scale || max_det <= 0) return PC_ERR_ARG;
  pc_ctx* c = net->ctx;
  if (n > net->max_batch) return fail(c, PC_ERR_ARG, "pc_scrfd_detect: batch exceeds max batch");
  if ((int)net->outs.size() != 3) return fail(c, PC_ERR_FORMAT, "SCRFD net must have 3 outputs");
  const NetTensor& I = net->tens[net->in_tensor];
  if (I.H != D || I.W != D) return fail(c, PC_ERR_ARG, "pc_scrfd_detect: D does not match the net input size");
  // candidate capacity = every anchor of the net (no cap: the reference keeps all
  // candidates >= det_thresh); images with more than 8192 go through scrfd_nms_big
  int cap = 0;
  for (int l = 0; l < 3; ++l) cap += net->tens[net->outs[l]].H * net->tens[net->outs[l]].W * 2;
  int pcap = 8192;
  while (pcap < cap) pcap <<= 1;
  const size_t cand_need = (size_t)n * cap * 16 * 4;
  // the candidate rows and the per-image counters are sized independently: a later call
  // with more images but a smaller D needs fewer rows and more counters
  if (c->cand_bytes < cand_need) {
    if (c->cand) hipFree(c->cand);
    c->cand = nullptr;
    c->cand_bytes = 0;
    HIPCHK(c, hipMalloc((void**)&c->cand, cand_need));
    c->cand_bytes = cand_need;
  }
  if (c->cand_images < (size_t)n) {
    if (c->cand_count) hipFree(c->cand_count);
    if (c->det_scale) hipFree(c->det_scale);
    c->cand_count = nullptr;
    c->det_scale = nullptr;
    c->cand_images = 0;
    HIPCHK(c, hipMalloc((void**)&c->cand_count, (size_t)n * 4 + 256));
    HIPCHK(c, hipMalloc((void**)&c->det_scale, (size_t)n * 4 + 256));
    c->cand_images = n;
  }
  const size_t keys_b = (size_t)n * pcap * 8, map_b = (size_t)n * cap * 4, kept_b = (size_t)n * cap * 16;
  if (c->nms_big_bytes < keys_b + map_b + kept_b) {
    if (c->nms_big) hipFree(c->nms_big);
    HIPCHK(c, hipMalloc(&c->nms_big, keys_b + map_b + kept_b));
    c->nms_big_bytes = keys_b + map_b + kept_b;
  }
  // letterbox into the net's own input staging area (reuse prep scratch)
  const size_t need = (size_t)net->max_batch * D * D * 4 * (net->f32 ? 4 : 2);
  if (net->prep_bytes < need) {
    if (net->prep) HIPCHK(c, hipFree(net->prep));
    HIPCHK(c, hipMalloc(&net->prep, need));
    net->prep_bytes = need;
  }
  int rc = pc_letterbox(c, net->f32 ? PC_PREC_F32 : PC_PREC_F16, h, n, D, net->prep);
  if (rc) return rc;
  rc = pc_net_run(net, net->prep, n);
  if (rc) return rc;
  DecodeParams p;
  memset(&p, 0, sizeof(p));
  p.nlv = 3;
  const int strides[3] = {8, 16, 32};
  int loc = 0, anc = 0;
  for (int l = 0; l < 3; ++l) {
    const NetTensor& O = net->tens[net->outs[l]];
    if (!(O.is_f32 || net->f32)) return fail(c, PC_ERR_FORMAT, "SCRFD head outputs must be f32");
    p.lv[l].out = (const float*)tensor_ptr(net, net->outs[l]);
    p.lv[l].H = O.H; p.lv[l].W = O.W; p.lv[l].cs = O.cs; p.lv[l].stride = strides[l];
    p.lv[l].loc_offset = loc; p.lv[l].anchor_offset = anc;
    loc += O.H * O.W;
    anc += O.H * O.W * 2;
  }
  p.total_loc = loc;
  p.thresh = det_thresh;
  void* dscale;
  if ((rc = stage_copy(c, h_det_scale, (size_t)n * 4, &dscale))) return rc;
  HIPCHK(c, hipMemsetAsync(c->cand_count, 0, n * 4, c->stream));
  p.det_scale = (const float*)dscale;
  p.cand = c->cand;
  p.count = c->cand_count;
  p.cap = cap;
  HIPCHK(c, scrfd_decode_launch(p, n, c->stream));
  HIPCHK(c, scrfd_nms_launch(c->cand, c->cand_count, cap, nms_thresh, max_det, dets, kps, count, n, c->stream));
  {
    char* big = (char*)c->nms_big;
    HIPCHK(c, scrfd_nms_big_launch(c->cand, c->cand_count, cap, pcap, (unsigned long long*)big, (int*)(big + keys_b),
                                   (float*)(big + keys_b + map_b), nms_thresh, max_det, dets, kps, count, n,
                                   c->stream));
  }
  if (ncand) HIPCHK(c, hipMemcpyAsync(ncand, c->cand_count, n * 4, hipMemcpyDeviceToDevice, c->stream));
  return PC_OK;
}

// ===========================================================================
// YOLOv8 person detection (PersonDetector.detect, detectors.py:271-296)
// ===========================================================================
static int check_yolo_descs(pc_ctx* c, const pc_yolo_letterbox_desc* h, int n, int Hp, int Wp) {
  for (int i = 0; i < n; ++i) {
    const pc_yolo_letterbox_desc& d = h[i];
    if (!d.d_src || d.H <= 0 || d.W <= 0 || d.row_stride < d.W * 3 || d.new_w <= 0 || d.new_h <= 0 || d.top < 0 ||
        d.left < 0 || d.top + d.new_h > Hp || d.left + d.new_w > Wp || (d.identity && (d.new_w != d.W || d.new_h != d.H)))
      return fail(c, PC_ERR_ARG, "yolo letterbox job out of range");
  }
  return PC_OK;
}

extern "C" int pc_yolo_letterbox(pc_ctx* c, int prec, const pc_yolo_letterbox_desc* h, int n, int Hp, int Wp,
                                 void* out) {
  if (!c || !h || n <= 0 || Hp <= 0 || Wp <= 0 || !out) return fail(c, PC_ERR_ARG, "pc_yolo_letterbox: bad arguments");
  int rc = check_yolo_descs(c, h, n, Hp, Wp);
  if (rc) return rc;
  void* dd;
  if ((rc = stage_copy(c, h, sizeof(pc_yolo_letterbox_desc) * n, &dd))) return rc;
  HIPCHK(c, yolo_letterbox_launch(prec == PC_PREC_F32, (const YoloLetterboxDesc*)dd, n, Hp, Wp, out, c->stream));
  return PC_OK;
}

static int yolo_detect_impl(pc_net* net, const pc_yolo_letterbox_desc* h, int n, int Hp, int Wp, float conf, float iou,
                            const pc_yolo_scale* h_scale, int max_det, float* dets, int32_t* count, int32_t* ncand,
                            int nkpt, const float* h_kpt_pad, float* kpts) {
  if (!net || !h || n <= 0 || !h_scale || max_det <= 0 || !dets || !count) return PC_ERR_ARG;
  if (nkpt < 0 || (nkpt > 0 && (!h_kpt_pad || !kpts || max_det > 1024))) return PC_ERR_ARG;
  const int nk = nkpt * 3;
  pc_ctx* c = net->ctx;
  if (n > net->max_batch) return fail(c, PC_ERR_ARG, "pc_yolo_detect: batch exceeds max batch");
  if ((int)net->outs.size() != 3) return fail(c, PC_ERR_FORMAT, "YOLO net must have 3 head outputs");
  const NetTensor& I = net->tens[net->in_tensor];
  if (I.H != Hp || I.W != Wp || I.C != 4) return fail(c, PC_ERR_ARG, "pc_yolo_detect: canvas does not match the net input");
  if (int e = check_yolo_descs(c, h, n, Hp, Wp)) return e;
  const size_t need = (size_t)net->max_batch * Hp * Wp * 4 * (net->f32 ? 4 : 2);
  if (net->prep_bytes < need) {
    if (net->prep) HIPCHK(c, hipFree(net->prep));
    HIPCHK(c, hipMalloc(&net->prep, need));
    net->prep_bytes = need;
  }
  int rc = pc_yolo_letterbox(c, net->f32 ? PC_PREC_F32 : PC_PREC_F16, h, n, Hp, Wp, net->prep);
  if (rc) return rc;
  rc = pc_net_run(net, net->prep, n);
  if (rc) return rc;
  YoloDecodeParams p;
  memset(&p, 0, sizeof(p));
  p.nlv = 3;
  int loc = 0, nc = -1;
  for (int l = 0; l < 3; ++l) {
    const NetTensor& O = net->tens[net->outs[l]];
    if (!(O.is_f32 || net->f32)) return fail(c, PC_ERR_FORMAT, "YOLO head outputs must be f32");
    const int ncl = O.C - 64 - nk;
    if (ncl <= 0 || (nc >= 0 && ncl != nc)) return fail(c, PC_ERR_FORMAT, "YOLO head channel layout");
    nc = ncl;
    p.lv[l].out = (const float*)tensor_ptr(net, net->outs[l]);
    p.lv[l].H = O.H; p.lv[l].W = O.W; p.lv[l].cs = O.cs;
    p.lv[l].stride = Hp / O.H;
    p.lv[l].loc_offset = loc;
    loc += O.H * O.W;
  }
  // candidate slots for every anchor: a low threshold on a big canvas may pass most of them
  // (above 16384 candidates the global-memory NMS runs)
  const int cap = std::max(16384, loc);
  if (c->ycand_images < (size_t)n || c->ycand_cap < cap) {
    if (c->ycand) { HIPCHK(c, hipStreamSynchronize(c->stream)); hipFree(c->ycand); }
    if (c->ycount) hipFree(c->ycount);
    HIPCHK(c, hipMalloc((void**)&c->ycand, (size_t)n * cap * 8 * 4));
    HIPCHK(c, hipMalloc((void**)&c->ycount, (size_t)n * 4));
    c->ycand_images = n;
    c->ycand_cap = cap;
  }
  p.total = loc;
  p.nc = nc;
  p.conf = conf;
  p.cand = c->ycand;
  p.count = c->ycount;
  p.cap = cap;
  void* dsc;
  if ((rc = stage_copy(c, h_scale, sizeof(pc_yolo_scale) * n, &dsc))) return rc;
  HIPCHK(c, hipMemsetAsync(c->ycount, 0, n * 4, c->stream));
  HIPCHK(c, yolo_decode_launch(p, n, c->stream));
  int* keep_anchor = nullptr;
  if (nk) {
    if (c->ykeep_bytes < (size_t)n * max_det * 4) {
      if (c->ykeep) { HIPCHK(c, hipStreamSynchronize(c->stream)); HIPCHK(c, hipFree(c->ykeep)); }
      HIPCHK(c, hipMalloc((void**)&c->ykeep, (size_t)n * max_det * 4));
      c->ykeep_bytes = (size_t)n * max_det * 4;
    }
    keep_anchor = c->ykeep;
  }
  HIPCHK(c, yolo_nms_launch(c->ycand, c->ycount, cap, iou, max_det, (const YoloScale*)dsc, dets, count, n, c->stream,
                            keep_anchor));
  if (loc > 16384) {
    int pcap = 8192;
    while (pcap < cap) pcap <<= 1;
    const size_t kb = (size_t)n * pcap * 8 + (size_t)n * cap * 4 + (size_t)n * max_det * 16;
    if (c->ybig_bytes < kb) {
      if (c->ybig) { HIPCHK(c, hipStreamSynchronize(c->stream)); hipFree(c->ybig); }
      HIPCHK(c, hipMalloc(&c->ybig, kb));
      c->ybig_bytes = kb;
    }
    char* b = (char*)c->ybig;
    HIPCHK(c, yolo_nms_big_launch(c->ycand, c->ycount, cap, pcap, (unsigned long long*)b,
                                  (int*)(b + (size_t)n * pcap * 8), (float*)(b + (size_t)n * pcap * 8 + (size_t)n * cap * 4),
                                  iou, max_det, (const YoloScale*)dsc, dets, count, keep_anchor, n, c->stream));
  }
  if (nk) {
    void* dks;
    if ((rc = stage_copy(c, h_kpt_pad, sizeof(float) * 2 * n, &dks))) return rc;
    HIPCHK(c, yolo_kpts_launch(p, nk, 64 + nc, max_det, count, keep_anchor, (const YoloScale*)dsc,
                               (const YoloKptScale*)dks, kpts, n, c->stream));
  }
  if (ncand) HIPCHK(c, hipMemcpyAsync(ncand, c->ycount, n * 4, hipMemcpyDeviceToDevice, c->stream));
  return PC_OK;
}

extern "C" int pc_yolo_detect(pc_net* net, const pc_yolo_letterbox_desc* h, int n, int Hp, int Wp, float conf,
                              float iou, const pc_yolo_scale* h_scale, int max_det, float* dets, int32_t* count,
                              int32_t* ncand) {
  return yolo_detect_impl(net, h, n, Hp, Wp, conf, iou, h_scale, max_det, dets, count, ncand, 0, nullptr, nullptr);
}

extern "C" int pc_yolo_pose_detect(pc_net* net, const pc_yolo_letterbox_desc* h, int n, int Hp, int Wp, float conf,
                                   float iou, const pc_yolo_scale* h_scale, const float* h_kpt_pad, int max_det,
                                   int nkpt, float* dets, float* kpts, int32_t* count, int32_t* ncand) {
  if (nkpt <= 0) return fail(net ? net->ctx : nullptr, PC_ERR_ARG, "pc_yolo_pose_detect: nkpt must be positive");
  return yolo_detect_impl(net, h, n, Hp, Wp, conf, iou, h_scale, max_det, dets, count, ncand, nkpt, h_kpt_pad, kpts);
}

// ===========================================================================
// ReID: OpenCLIP ViT-L/14 image tower (ReIDEmbedder.extract, reid_embedder.py:38-57)
// ===========================================================================
static const int kClipSide = 224, kClipTok = 257, kClipK = 608, kClipKmax = 64;

extern "C" int pc_clip_prep(pc_ctx* c, int prec, const pc_crop_desc* h, int n, void* out) {
  if (!c || !h || n <= 0 || !out) return fail(c, PC_ERR_ARG, "pc_clip_prep: bad arguments");
  // host: geometry + Pillow coefficient tables for the 224 kept columns / rows of each crop
  struct Tabs { int kh, kv, row0, nrows; std::vector<int32_t> hb, hk, vb, vk; };
  std::vector<Tabs> T(n);
  size_t tmp_bytes = 0, tab_ints = 0;
  int max_rows = 0;
  for (int i = 0; i < n; ++i) {
    const pc_crop_desc& d = h[i];
    if (!d.d_src || d.H <= 0 || d.W <= 0 || d.row_stride < d.W * 3) return fail(c, PC_ERR_ARG, "pc_clip_prep: bad crop");
    int32_t g[4];
    pc_clip_geometry(d.H, d.W, kClipSide, g);
    Tabs& t = T[i];
    t.hb.resize(2 * kClipSide); t.vb.resize(2 * kClipSide);
    t.hk.resize((size_t)kClipSide * kClipKmax); t.vk.resize((size_t)kClipSide * kClipKmax);
    t.kh = pc_pil_bicubic_coeffs(d.W, g[0], g[3], kClipSide, t.hb.data(), t.hk.data(), kClipKmax);
    t.kv = pc_pil_bicubic_coeffs(d.H, g[1], g[2], kClipSide, t.vb.data(), t.vk.data(), kClipKmax);
    if (t.kh < 0 || t.kv < 0) return fail(c, PC_ERR_CAPACITY, "pc_clip_prep: crop too large for the resample tables");
    t.hk.resize((size_t)kClipSide * t.kh); t.vk.resize((size_t)kClipSide * t.kv);
    int lo = 1 << 30, hi = 0;
    for (int y = 0; y < kClipSide; ++y) { lo = std::min(lo, t.vb[2 * y]); hi = std::max(hi, t.vb[2 * y] + t.vb[2 * y + 1]); }
    t.row0 = lo; t.nrows = std::max(hi - lo, 1);
    for (int y = 0; y < kClipSide; ++y) t.vb[2 * y] -= lo;
    max_rows = std::max(max_rows, t.nrows);
    tmp_bytes += (size_t)t.nrows * kClipSide * 3;
    tab_ints += t.hb.size() + t.hk.size() + t.vb.size() + t.vk.size();
  }
  if (c->clip_tmp_bytes < tmp_bytes) {
    if (c->clip_tmp) { HIPCHK(c, hipStreamSynchronize(c->stream)); HIPCHK(c, hipFree(c->clip_tmp)); }
    HIPCHK(c, hipMalloc(&c->clip_tmp, tmp_bytes));
    c->clip_tmp_bytes = tmp_bytes;
  }
  std::vector<int32_t> tabs;
  tabs.reserve(tab_ints);
  std::vector<size_t> off(n * 4);
  for (int i = 0; i < n; ++i) {
    off[4 * i + 0] = tabs.size(); tabs.insert(tabs.end(), T[i].hb.begin(), T[i].hb.end());
    off[4 * i + 1] = tabs.size(); tabs.insert(tabs.end(), T[i].hk.begin(), T[i].hk.end());
    off[4 * i + 2] = tabs.size(); tabs.insert(tabs.end(), T[i].vb.begin(), T[i].vb.end());
    off[4 * i + 3] = tabs.size(); tabs.insert(tabs.end(), T[i].vk.begin(), T[i].vk.end());
  }
  void* dtab;
  int rc = stage_copy(c, tabs.data(), tabs.size() * 4, &dtab);
  if (rc) return rc;
  std::vector<ClipPrepDesc> descs(n);
  size_t tmp_off = 0;
  for (int i = 0; i < n; ++i) {
    ClipPrepDesc& d = descs[i];
    const int32_t* tb = (const int32_t*)dtab;
    d.src = h[i].d_src; d.H = h[i].H; d.W = h[i].W; d.row_stride = h[i].row_stride;
    d.kh = T[i].kh; d.kv = T[i].kv;
    d.hb = tb + off[4 * i]; d.hk = tb + off[4 * i + 1]; d.vb = tb + off[4 * i + 2]; d.vk = tb + off[4 * i + 3];
    d.row0 = T[i].row0; d.nrows = T[i].nrows;
    d.tmp = (uint8_t*)c->clip_tmp + tmp_off;
    tmp_off += (size_t)T[i].nrows * kClipSide * 3;
  }
  void* ddesc;
  if ((rc = stage_copy(c, descs.data(), sizeof(ClipPrepDesc) * n, &ddesc))) return rc;
  HIPCHK(c, clip_prep_launch(prec == PC_PREC_F32, (const ClipPrepDesc*)ddesc, n, max_rows, out, c->stream));
  return PC_OK;
}

extern "C" int pc_clip_embed(pc_net* net, const pc_crop_desc* h, int n, float* feat) {
  if (!net || !h || n < 0 || !feat) return PC_ERR_ARG;
  pc_ctx* c = net->ctx;
  if (n == 0) return PC_OK;
  if (n > net->max_batch) return fail(c, PC_ERR_ARG, "pc_clip_embed: batch exceeds max batch");
  const NetTensor& I = net->tens[net->in_tensor];
  if (I.H != 1 || I.W != kClipTok || I.C != kClipK) return fail(c, PC_ERR_FORMAT, "CLIP net input must be 1x257x608");
  const size_t need = (size_t)net->max_batch * kClipTok * kClipK * (net->f32 ? 4 : 2);
  if (net->prep_bytes < need) {
    if (net->prep) HIPCHK(c, hipFree(net->prep));
    HIPCHK(c, hipMalloc(&net->prep, need));
    net->prep_bytes = need;
  }
  int rc = pc_clip_prep(c, net->f32 ? PC_PREC_F32 : PC_PREC_F16, h, n, net->prep);
  if (rc) return rc;
  rc = pc_net_run(net, net->prep, n);
  if (rc) return rc;
  const NetTensor& O = net->tens[net->outs[0]];
  if (!(O.is_f32 || net->f32) || O.H * O.W != 1) return fail(c, PC_ERR_FORMAT, "CLIP output must be f32 [1][1][dim]");
  HIPCHK(c, embed_l2_launch((const float*)tensor_ptr(net, net->outs[0]), O.cs, n, O.C, 1e-12f, feat, c->stream));
  return PC_OK;
}

extern "C" int pc_l2_normalize(pc_ctx* c, const float* e, int ld, int n, int dim, float eps, float* out) {
  if (!c || n < 0 || !e || !out) return fail(c, PC_ERR_ARG, "pc_l2_normalize: bad arguments");
  if (n == 0) return PC_OK;
  HIPCHK(c, embed_l2_launch(e, ld, n, dim, eps, out, c->stream));
  return PC_OK;
}
