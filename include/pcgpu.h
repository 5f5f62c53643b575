/*
 * pcgpu.h — C ABI of the MI355X (gfx950) identity hot path of person_capture.
 *
 * This is the drop-in boundary that replaces the reference's inference runtimes
 * (SURVEY.md §8b). Plain pointers and sizes only; no torch or HIP types appear in
 * the signatures (streams are passed as void*). Every function returns an int
 * status (PC_OK == 0); the message of the last failure on a context is available
 * from pc_last_error(). Device pointers ("d_") are HIP device allocations on the
 * context's device; host pointers ("h_") are ordinary CPU memory.
 *
 * Which reference interface each entry point replaces (file:line in the reference
 * snapshot xmarre/person_capture):
 *
 *   pc_ctx_create / pc_ctx_destroy     ORT InferenceSession(..., providers=[TRT, CUDA, CPU]) setup
 *                                      person_capture/face_embedder.py:557-703, 848-953
 *   pc_net_create                      model load: SCRFD ONNX session (face_embedder.py:1102-1147),
 *                                      ArcFace ONNX session (face_embedder.py:891-953),
 *                                      YOLO(path) (detectors.py:84-269)
 *   pc_net_run                         session.run / run_with_iobinding (face_embedder.py:1331-1343, 1369)
 *   pc_letterbox                       [ext] insightface SCRFD.detect letterbox + cv2.dnn.blobFromImage
 *                                      (called at face_embedder.py:2185)
 *   pc_scrfd_detect                    [ext] SCRFD.detect(img, input_size=(D, D)) -> (det Nx5, kpss Nx5x2)
 *                                      (face_embedder.py:2176-2187)
 *   pc_warp_affine                     cv2.warpAffine(face, M, (112,112), INTER_LINEAR, BORDER_REFLECT)
 *                                      (face_embedder.py:1465-1473)
 *   pc_face_quality                    FaceEmbedder._face_quality (face_embedder.py:1274-1276)
 *   pc_arcface_embed                   FaceEmbedder._arcface_encode (face_embedder.py:1290-1389)
 *   pc_embed_finalize                  flip-sum + L2 (face_embedder.py:1383-1389)
 *   pc_bank_match                      Processor._fd_min (gui_app.py:660-674), batched
 *   pc_rotate_pad                      cv2.rotate + cv2.copyMakeBorder(BORDER_REPLICATE)
 *                                      (face_embedder.py:2165-2169, 2292-2294, 2394)
 *   pc_resize_area                     cv2.resize(..., INTER_AREA) (gui_app.py:1505-1507)
 *   pc_resize_area_batch               the same over a chunk of pre-scan samples (gui_app.py:1505-1507)
 *   pc_resize_linear                   cv2.resize(..., INTER_LINEAR) (face_embedder.py:2264, 2460)
 *   pc_resize_area_fast                cv2.resize(..., INTER_AREA) at integer ratios (face_embedder.py:2460)
 *   pc_yolo_detect                     PersonDetector.detect -> [ext] ultralytics YOLO.predict(conf, iou=0.45,
 *                                      classes=[0], max_det=40, imgsz=640) (detectors.py:271-296)
 *   pc_yolo_pose_detect                FaceEmbedder YOLOv8-face backend (Y8F_DEFAULT, face_embedder.py:33) ->
 *                                      [ext] ultralytics YOLO(pose).predict(conf, iou, max_det, imgsz) with
 *                                      res.boxes + res.keypoints.xy (face_embedder.py:1680-1703, 1391-1429)
 *   pc_clip_prep / pc_clip_embed       ReIDEmbedder.extract: BGR2RGB + open_clip preprocess + encode_image +
 *                                      F.normalize (reid_embedder.py:38-57)
 *   pc_l2_normalize                    torch.nn.functional.normalize(feats, dim=1) (reid_embedder.py:55)
 *   pc_pil_bicubic_coeffs              Pillow Image.resize(BICUBIC) coefficients inside the open_clip
 *                                      preprocess (reid_embedder.py:49)
 */
#ifndef PCGPU_H
#define PCGPU_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define PC_ABI_VERSION 1

#define PC_OK 0
#define PC_ERR_ARG 1
#define PC_ERR_HIP 2
#define PC_ERR_STATE 3
#define PC_ERR_FORMAT 4
#define PC_ERR_CAPACITY 5

/* arithmetic of a network: f16 storage + f32 accumulation (throughput), or
 * exact f32 (parity runs against the CPU oracle). */
#define PC_PREC_F16 0
#define PC_PREC_F32 1
/* pc_arcface_prep only: the centred chip x - 127.5 in f16 (exact), the input of the f16x3 IResNet
 * program (its stem weights carry the 1/127.5; models.compile_iresnet(split=True)) */
#define PC_PREC_F16X3 2

typedef struct pc_ctx pc_ctx;
typedef struct pc_net pc_net;

/* One letterbox job (SCRFD input): BGR u8 frame on device -> resized into the
 * top-left of a DxD canvas. scale_x/scale_y are 1/(new/old) as cv::resize uses. */
typedef struct pc_letterbox_desc {
  const uint8_t* d_src;
  int32_t H, W, row_stride;
  int32_t new_w, new_h;
  double scale_x, scale_y;
  int32_t simd_end; /* byte index of each row where OpenCV's SIMD vertical pass stops */
  int32_t pad_;
} pc_letterbox_desc;

/* One warpAffine job: crop (top-left pointer + size) -> out_w x out_h x 3 u8.
 * M is the dst->src affine map (cv::warpAffine's internal inverse). */
typedef struct pc_warp_desc {
  const uint8_t* d_src;
  int32_t row_stride;
  int32_t w, h;
  int32_t pad0_;
  double M[6];
  uint8_t* d_dst;
  int32_t out_w, out_h;
  int32_t border; /* 2 = BORDER_REFLECT, 4 = BORDER_REFLECT_101, 0 | (value << 8) = BORDER_CONSTANT */
  int32_t pad1_;
} pc_warp_desc;

/* One u8 -> u8 bilinear resize job (cv2.resize semantics, BGR): INTER_LINEAR, or INTER_AREA
 * when not both axes downscale (area_mode = 1: OpenCV's area-mode linear coefficients). */
typedef struct pc_resize_desc {
  const uint8_t* d_src;
  int32_t H, W, row_stride;
  int32_t new_w, new_h;
  double scale_x, scale_y; /* 1 / inv_scale */
  int32_t simd_end;
  int32_t area_mode;
  uint8_t* d_dst; /* new_h x new_w x 3 contiguous */
  double inv_x, inv_y; /* dsize / ssize, or the fx / fy given */
} pc_resize_desc;

/* One INTER_AREA coefficient: source index, destination index, weight. */
typedef struct pc_area_tab {
  int32_t si;
  int32_t di;
  float alpha;
} pc_area_tab;

/* One YOLOv8 letterbox job ([ext] ultralytics LetterBox(auto=True, stride=32), detectors.py:274):
 * BGR u8 frame -> cv2.resize INTER_LINEAR to new_w x new_h placed at (left, top) of an
 * Hp x Wp canvas filled with 114; identity = 1 when no resize happens (same shape). */
typedef struct pc_yolo_letterbox_desc {
  const uint8_t* d_src;
  int32_t H, W, row_stride;
  int32_t new_w, new_h;
  int32_t top, left;
  double scale_x, scale_y;
  int32_t simd_end;
  int32_t identity;
} pc_yolo_letterbox_desc;

/* [ext] ultralytics ops.scale_boxes per frame: box = clip((box - pad) / gain, [0,W0] x [0,H0]) */
typedef struct pc_yolo_scale {
  float gain, pad_x, pad_y, W0, H0;
} pc_yolo_scale;

/* One BGR u8 image crop on the device (top-left pointer, size, bytes per row). */
typedef struct pc_crop_desc {
  const uint8_t* d_src;
  int32_t H, W, row_stride, pad_;
} pc_crop_desc;

int pc_abi_version(void);

/* ---- context ---- */
int pc_ctx_create(int device_id, pc_ctx** out);
int pc_ctx_destroy(pc_ctx* ctx);
const char* pc_last_error(const pc_ctx* ctx);
int pc_ctx_set_stream(pc_ctx* ctx, void* hip_stream); /* NULL = context-owned stream */
void* pc_ctx_stream(pc_ctx* ctx);
/* Re-create the context-owned stream at a HIP stream priority (lower = higher priority,
 * clamped to the device's range). No reference counterpart: the face embedder's second
 * (embed) stream is a build-side scheduling choice (two streams). */
int pc_ctx_set_priority(pc_ctx* ctx, int priority);
int pc_ctx_sync(pc_ctx* ctx);
int pc_device_alloc(pc_ctx* ctx, size_t bytes, void** d_out);
int pc_device_free(pc_ctx* ctx, void* d_ptr);
/* stream-ordered wait: work enqueued on ctx after this call waits for fence f (recorded on any
 * context of the same device). */
int pc_ctx_wait_fence(pc_ctx* ctx, void* f);
/* host frame staging (replaces the per-frame pageable upload of the reference's frame feed,
 * video_io.py:1093-1135 -> FaceEmbedder.extract): rows of row_bytes, src_stride apart, packed
 * by up to `threads` host threads into a ring of 4 pinned slots, then one async H2D on the
 * context stream. The host array may be reused when this returns. */
int pc_frame_stage(pc_ctx* ctx, void* d_dst, const void* h_src, size_t row_bytes, size_t rows, size_t src_stride,
                   int threads);
int pc_copy_h2d(pc_ctx* ctx, void* d_dst, const void* h_src, size_t bytes); /* stream-ordered */
int pc_copy_d2h(pc_ctx* ctx, void* h_dst, const void* d_src, size_t bytes); /* stream-ordered */
int pc_copy_d2d(pc_ctx* ctx, void* d_dst, const void* d_src, size_t bytes);
int pc_memset(pc_ctx* ctx, void* d_dst, int value, size_t bytes);
/* device -> device pitched copy (cv2.resize to the same size copies, resize.cpp) */
int pc_copy_2d(pc_ctx* ctx, void* d_dst, size_t dst_pitch, const void* d_src, size_t src_pitch, size_t width_bytes,
               size_t rows);
/* Pinned host memory (page-locked: D2H copies into it stay asynchronous) and stream
 * fences. A fence is a HIP event recorded on the context stream; pc_fence_wait blocks
 * the host until everything enqueued before the record has finished. Used to overlap
 * the host-side detector policy of one chunk of frames with device work of the next
 * (FaceEmbedder.extract_batch). */
int pc_host_alloc(pc_ctx* ctx, size_t bytes, void** h_out);
int pc_host_free(pc_ctx* ctx, void* h_ptr);
int pc_fence_create(pc_ctx* ctx, void** fence_out);
int pc_fence_record(pc_ctx* ctx, void* fence);
int pc_fence_wait(pc_ctx* ctx, void* fence);
int pc_fence_destroy(pc_ctx* ctx, void* fence);

/* ---- networks (serialized program produced by person_capture_amd.netdef) ---- */
int pc_net_create(pc_ctx* ctx, const void* h_program, size_t program_bytes, int precision, int max_batch,
                  pc_net** out);
int pc_net_destroy(pc_net* net);
/* d_input: NHWC, dims as pc_net_input_dims; activation dtype of the net's precision */
int pc_net_run(pc_net* net, const void* d_input, int batch);
int pc_net_input_dims(pc_net* net, int32_t* h_dims4 /* H, W, C, pixel stride */);
int pc_net_output(pc_net* net, int index, void** d_ptr, int32_t* h_dims5 /* H, W, C, pixel stride, is_f32 */);
int pc_net_num_outputs(pc_net* net);
/* algorithmic FLOPs per image (2*MAC over all conv layers) and kernel launches per run */
int pc_net_stats(pc_net* net, double* h_flops_per_image, int32_t* h_launches);
/* resident block chains of the net (pc_conv_chain: runs of IResNet identity blocks executed
 * one image per workgroup): returns their count; *h_min_batch = the batch from which they
 * are used, *h_images_per_round = images one round of workgroups covers (the CU count).
 * (No reference counterpart: a scheduling hint for FaceEmbedder's ArcFace batch quantum.) */
int pc_net_chain_info(pc_net* net, int32_t* h_min_batch, int32_t* h_images_per_round);
/* the batch from which the chains run (<= 0: never). A chain workgroup needs a whole CU's
 * LDS, so a net that shares the device with another stream's kernels (FaceEmbedder's embed
 * stream beside SCRFD) runs faster per-conv: measured C3 1925 vs 1705 frames/s. */
int pc_net_set_chain_min_batch(pc_net* net, int32_t min_batch);
/* capture pc_net_run(batch) into a HIP graph and replay it on later runs of the same batch */
int pc_net_set_graph(pc_net* net, int enable);
/* with graphs enabled, capture / replay only runs of at most max_batch images (the per-frame
 * extract() path: dozens of small launches per net run); larger runs launch eagerly (and can
 * be profiled). Default: every batch. Replaces nothing in the reference (launch plumbing). */
int pc_net_set_graph_max_batch(pc_net* net, int32_t max_batch);
/* HIP-event timing of every op of every later (non-graph) run; enable resets the counters.
 * read: [0] conv ms, [1] conv launches, [2] conv FLOPs (algorithmic), [3] other ms, [4] other launches */
int pc_net_profile(pc_net* net, int enable);
/* f16c8 nets: run the program once on N images at d_in and set every f16c8 tensor's
 * e4m3 scale exponents from its largest magnitude, 2^headroom_log2 below the format's range. Clears the
 * net's captured graphs. h_absmax (optional, [n_tensor] floats): the measured max |x| per tensor (0 where
 * not measured). Replaces no reference interface (the reference's TensorRT engines carry no such
 * scales: f16c8 is this build's f32-class arithmetic on the f16 / fp8 MFMA path). */
int pc_net_calibrate(pc_net* net, const void* d_in, int N, int headroom_log2, float* h_absmax);
int pc_net_profile_read(pc_net* net, double* h_out5);
/* Per-launch detail of the profiled runs, 6 doubles per record: op index, op kind, ms, FLOPs,
   kernel (100+k: static-schedule tile k, 600+k: its f16c8 form, 200+v: t2d variant v, 300: resident chain, 500: halo-staged f16x3, k >= 0: halo tile k, -1: generic implicit-GEMM), implicit-GEMM tile (static-schedule tiles: their form, bit 0 fused split, bit 1 register weight fragments, bit 2 128-byte K rows). Returns the record count (<0: -status). */
int pc_net_profile_ops(pc_net* net, double* h_out, int max_recs);

/* ---- image kernels ---- */
int pc_letterbox(pc_ctx* ctx, int precision, const pc_letterbox_desc* h_descs, int n, int D, void* d_out);
int pc_warp_affine(pc_ctx* ctx, const pc_warp_desc* h_descs, int n);
int pc_resize_linear(pc_ctx* ctx, const pc_resize_desc* h_descs, int n);
int pc_face_quality(pc_ctx* ctx, const uint8_t* d_chips, int n, int side, double* d_out);
/* precision PC_PREC_F16 / PC_PREC_F32: x/127.5 - 1 in that dtype (face_embedder.py:1281-1288);
 * PC_PREC_F16X3: x - 127.5 in f16 (the f16x3 program's centred input) */
int pc_arcface_prep(pc_ctx* ctx, int precision, const uint8_t* d_chips, int n, int side, int flip, void* d_out);
int pc_rotate_pad(pc_ctx* ctx, const uint8_t* d_src, int H, int W, int row_stride, int deg, int pad, uint8_t* d_dst);
/* cv2.resize INTER_AREA at an exact integer ratio isx x isy (OpenCV resizeAreaFast). */
int pc_resize_area_fast(pc_ctx* ctx, const uint8_t* d_src, int row_stride, int isx, int isy, uint8_t* d_dst, int OH,
                        int OW);
int pc_resize_area(pc_ctx* ctx, const uint8_t* d_src, int row_stride, const pc_area_tab* h_xtab,
                   const int32_t* h_xstart, int n_x, const pc_area_tab* h_ytab, const int32_t* h_ystart, int n_y,
                   uint8_t* d_dst, int OH, int OW);
/* The same cv2.resize INTER_AREA for n equally sized frames at once (the pre-scan's downscale of a
 * speculative chunk of samples, gui_app.py:1505-1507 per sample): h_srcs / h_dsts are host arrays of n
 * device pointers, tables as pc_resize_area. 16-byte aligned sources and row_stride take the row-
 * staged kernel (one launch); others the per-pixel one. Output bytes equal pc_resize_area's. */
int pc_resize_area_batch(pc_ctx* ctx, const uint8_t* const* h_srcs, uint8_t* const* h_dsts, int n, int row_stride,
                         const pc_area_tab* h_xtab, const int32_t* h_xstart, int n_x, const pc_area_tab* h_ytab,
                         const int32_t* h_ystart, int n_y, int OH, int OW);

/* ---- detection ---- */
/* Runs letterbox -> SCRFD net -> decode(score >= det_thresh) -> NMS(nms_thresh) for n frames.
 * Outputs (device): d_dets [n][max_det][5], d_kps [n][max_det][10], d_count [n] (number kept,
 * may exceed max_det: then only the first max_det rows are written; call again with a larger
 * max_det for the full list), d_ncand [n] candidates above threshold. No candidate cap: every
 * anchor of the net has a slot, as the reference keeps every candidate >= det_thresh. */
int pc_scrfd_detect(pc_net* net, const pc_letterbox_desc* h_descs, int n, int D, float det_thresh,
                    float nms_thresh, const float* h_det_scale, int max_det, float* d_dets, float* d_kps,
                    int32_t* d_count, int32_t* d_ncand);

/* ---- embedding / match ---- */
int pc_embed_finalize(pc_ctx* ctx, const float* d_e, int ld, int n, int dim, int flip, float* d_out);
/* chips: [n][side][side][3] BGR u8 (side == net input side). d_feat: [n][dim] unit f32. A net whose
 * program flags a centred input (f16x3 IResNet) gets the PC_PREC_F16X3 preprocessing. */
int pc_arcface_embed(pc_net* net, const uint8_t* d_chips, int n, int flip, float* d_feat);
int pc_bank_match(pc_ctx* ctx, const float* d_q, int n, const float* d_bank, int b, int dim, float* d_fd,
                  int32_t* d_idx);

/* ---- person detection (YOLOv8) ---- */
/* letterbox -> YOLOv8 net -> DFL decode (best class 0, score > conf) -> NMS(iou) -> scale_boxes,
 * for n frames sharing one Hp x Wp canvas. d_dets [n][max_det][5] (x1, y1, x2, y2, conf) in frame
 * pixels, d_count [n] kept (<= max_det), d_ncand [n] candidates (capacity 16384 per frame). */
/* letterbox only (the first stage of pc_yolo_detect): d_out [n][Hp][Wp][4] in the precision's dtype */
int pc_yolo_letterbox(pc_ctx* ctx, int precision, const pc_yolo_letterbox_desc* h_descs, int n, int Hp, int Wp,
                      void* d_out);
int pc_yolo_detect(pc_net* net, const pc_yolo_letterbox_desc* h_descs, int n, int Hp, int Wp, float conf, float iou,
                   const pc_yolo_scale* h_scale, int max_det, float* d_dets, int32_t* d_count, int32_t* d_ncand);
/* Pose-head variant (YOLOv8-face, nkpt keypoints x (x, y, visibility)): as pc_yolo_detect (all
 * classes kept, the head's nc = channels - 64 - 3 nkpt), plus d_kpts [n][max_det][nkpt][3] in frame
 * pixels: Pose.kpts_decode, ops.scale_coords with h_kpt_pad [n][2] = the unrounded letterbox pad
 * ((Wp - W gain) / 2, (Hp - H gain) / 2), clip, and x = y = 0 where visibility < 0.5. */
int pc_yolo_pose_detect(pc_net* net, const pc_yolo_letterbox_desc* h_descs, int n, int Hp, int Wp, float conf,
                        float iou, const pc_yolo_scale* h_scale, const float* h_kpt_pad, int max_det, int nkpt,
                        float* d_dets, float* d_kpts, int32_t* d_count, int32_t* d_ncand);

/* ---- ReID body embedding (OpenCLIP ViT-L/14 image tower) ---- */
/* preprocess n crops -> ViT-L/14 patch matrix [n][257][608] (token 0 and K padding zero) */
int pc_clip_prep(pc_ctx* ctx, int precision, const pc_crop_desc* h_crops, int n, void* d_out);
/* preprocess + image tower + F.normalize: d_feat [n][dim] unit f32 */
int pc_clip_embed(pc_net* net, const pc_crop_desc* h_crops, int n, float* d_feat);
/* rows of d_e (stride ld floats) / max(||row||, eps) -> d_out [n][dim] */
int pc_l2_normalize(pc_ctx* ctx, const float* d_e, int ld, int n, int dim, float eps, float* d_out);
/* Pillow BICUBIC resample coefficients (precompute_coeffs + normalize_coeffs_8bpc) for output
 * positions [first, first+count) of an in_size -> out_size resize: h_bounds [count][2] (min, n),
 * h_kk [count][ksize] Q22. Returns ksize (< 0: -status). */
int pc_pil_bicubic_coeffs(int in_size, int out_size, int first, int count, int32_t* h_bounds, int32_t* h_kk, int kmax);
/* torchvision Resize(side) + CenterCrop(side) geometry: h_out4 = resized w, h, crop top, left */
int pc_clip_geometry(int h, int w, int side, int32_t* h_out4);

/* ---- host-side align geometry (CPU, batched) ---- */
/* cv::estimateAffinePartial2D(from, to, method=LMEDS) for n point sets of npts points each
 * (h_from [n][npts][2], shared h_to [npts][2]); h_M [n][6] src->dst, h_ok [n] 0/1.
 * Replaces the call at face_embedder.py:1466-1468. */
int pc_estimate_affine_partial(const float* h_from, const float* h_to, int npts, int n, double* h_M, int32_t* h_ok);
/* the inversion cv::warpAffine applies to M (no WARP_INVERSE_MAP) */
int pc_invert_affine(const double* h_M, double* h_iM);

#ifdef __cplusplus
}
#endif
#endif /* PCGPU_H */
