/* yolomi — C-ABI of the MI355X-native YOLO11 inference path (gfx950 HIP kernels).
 *
 * The reference has no FFI: its hot path is pure Python delegating to Ultralytics
 * (/root/reference/core/model.py:118-133 `YOLO11Model.predict` → `self.model.predict(source, **kwargs)`;
 * /root/reference/core/model.py:253-291 `benchmark`).  This header is the boundary that replaces the
 * Ultralytics engine + ATen/torchvision kernels under that call: the Python facade
 * (`yolo-infer_amd/core/model.py`) binds it with ctypes; a C/C++ host can link it directly.
 *
 * Conventions: every function returns 0 (YM_OK) or a negative YM_E* code and never throws; the message of the
 * last failure on the calling thread is `ym_last_error()`.  The library owns weights, workspace and captured
 * graphs; the caller owns input/output device buffers.  One context per device; a context is not re-entrant;
 * distinct contexts may be used concurrently from different threads or processes.
 */
#ifndef YOLOMI_H
#define YOLOMI_H
#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define YM_OK 0
#define YM_EINVAL -1    /* bad argument (shape, pointer, size) */
#define YM_EBLOB -2     /* malformed model blob */
#define YM_EHIP -3      /* HIP runtime error */
#define YM_ENOMEM -4    /* device allocation failed */
#define YM_ESTATE -5    /* call order (e.g. infer before load) */

typedef struct ym_ctx ym_ctx;

/* What the caller expects the context to run (family / scale / task / dtype / max_B / S).  Capacity
 * fields are hints (0 = grow on demand); scale, task and dtype, when non-zero, are checked against every blob
 * ym_load_weights receives (YM_EBLOB on a mismatch) — the reference resolves them from the model name
 * (core/model.py:37-45, 106-107); here the packed plan carries them. */
typedef struct {
  int max_batch;
  int max_h;
  int max_w;
  int scale;  /* 0 = any, else 'n', 's', 'm', 'l' or 'x' */
  int task;   /* 0 = any, YM_TASK_DETECT, YM_TASK_SEGMENT */
  int dtype;  /* 0 = any, YM_DTYPE_F16, YM_DTYPE_F32, YM_DTYPE_I8, YM_DTYPE_F8, YM_DTYPE_X3 */
  int reserved[2];
} ym_model_desc;

#define YM_TASK_DETECT 1
#define YM_TASK_SEGMENT 2
#define YM_DTYPE_F16 1 /* fp16 storage, fp32 MFMA accumulation (throughput plan) */
#define YM_DTYPE_F32 2 /* exact-f32 MFMA (parity plan) */
#define YM_DTYPE_I8 3  /* PTQ int8 (torch.ao qconfig of optimization/quantization/quantizers.py:124-131) */
#define YM_DTYPE_F8 4  /* PTQ fp8 e4m3 (OCP) operands, fp32 accumulation */
#define YM_DTYPE_X3 5  /* fp32 storage, split-fp16 MFMA (x = hi + lo, three f16 MFMAs per K chunk): f16 tolerance plan */

/* An RCCL unique id (ncclUniqueId: 128 opaque bytes). */
typedef struct {
  char internal[128];
} ym_rccl_id;

/* Per-call predict arguments: the Ultralytics predict kwargs that reach the hot path
 * (conf, iou, classes, agnostic_nms, max_det; NMS constants max_nms=30000, max_wh=7680;
 * LoadTensor eps = finfo(input dtype).eps for the /255 rule). */
typedef struct {
  float conf;
  float max_wh;
  double iou;
  int max_det;
  int max_nms;
  int agnostic;
  float in_eps;
  int has_classes;
  uint32_t classes[4]; /* bit c set = keep class c (c < 128) */
  int use_graph;       /* 1: capture/replay a HIP graph per (shape, pointers, args); 0: eager launches */
  int lanes;           /* 1..4 image slices run as concurrent graph branches (0 = 1); conv tile tables are looked
                          up at the slice batch ceil(B / lanes) */
  int counts_after_dets; /* 1: the detection counts are also written, as B int32 words, right after the B x max_det
                            rows of d_dets (d_dets must hold B*max_det*(6+nm) + B floats): a caller that hands in
                            fresh rows per call gets that call's counts with them, and may read them later */
  const float* d_batch_max; /* NULL: LoadTensor's /255 rule reduces over d_input (the whole batch).  Else a device
                               pointer to ONE float, the max over the GLOBAL batch (batch-sharded multi-GPU: every
                               rank's ym_input_max, all-reduced MAX), read by the forward instead of its shard */
  int reserved[4];
} ym_infer_args;

/* Replaces `YOLO(model_path)` construction (core/model.py:100-116): create a context on `device`. */
int ym_create(int device, const ym_model_desc* desc, ym_ctx** out);

/* Load a model blob (plan + BN-folded packed weights, produced by yolomi.plan.pack_model) from host memory.
 * Replaces AutoBackend(fuse=True) weight preparation.  Copies to device; the host blob may be freed after. */
int ym_load_weights(ym_ctx* ctx, const void* blob, size_t bytes);
/* (blob dtypes: f16 and f32 plans, and int8 PTQ plans packed with calibrated quantisation parameters by
 *  yolomi.plan.pack_graph(..., dtype="i8", qparams=...) — the runtime of PostTrainingQuantizer.optimize,
 *  /root/reference/optimization/quantization/quantizers.py:48-91.) */

/* Multi-GPU initialisation (one process per GPU, batch-sharded): replaces the per-process
 * `YOLO(model_path)` load of core/model.py:100-116 on every rank by ONE load on `root` and an RCCL broadcast over
 * xGMI.  `comm` is an ncclComm_t of the RCCL library the process has loaded (e.g. from ym_rccl_comm_init).  On
 * `root` the context must hold weights (ym_load_weights); every other rank's context receives the root's blob and
 * loads it.  Collective: every rank of `comm` calls it.  Synchronous.  Every rank runs the same collectives whatever
 * fails locally (a root without weights, a staging allocation or a load failing on some rank) and all ranks then
 * return the same verdict, so no rank is left waiting inside RCCL. */
int ym_broadcast_weights(ym_ctx* ctx, void* comm, int root, void* stream);
/* The same broadcast with the ranks as `n` contexts of THIS process (SURVEY §4.4's fake backend: N "ranks" on one
 * GPU, the broadcast a device-to-device copy): ctxs[root] holds weights, every other context receives its blob
 * through the same per-rank staging / receive / ym_load_weights / verdict steps as ym_broadcast_weights' ranks.
 * Synchronous on `stream`.  Lets a one-GPU host (and the tests) run the receive path without RCCL. */
int ym_broadcast_weights_local(ym_ctx* const* ctxs, int n, int root, void* stream);
/* Minimal RCCL bootstrap for C hosts without their own communicator: rank 0 creates the id, the host ships the 128
 * bytes to the other ranks (any channel), every rank creates its communicator on `device`. */
int ym_rccl_get_unique_id(ym_rccl_id* id);
int ym_rccl_comm_init(int device, int nranks, const ym_rccl_id* id, int rank, void** comm);
int ym_rccl_comm_destroy(void* comm);

/* Replaces `YOLO11Model.predict(tensor)` (core/model.py:118-133) for tensor sources: asynchronous on `stream`
 * (a hipStream_t, NULL = default).  d_input: B×3×H×W fp32 NCHW device tensor (H, W multiples of 32).
 * d_dets: B×max_det×(6+nm) fp32 [x1,y1,x2,y2,conf,cls,(mask coeffs)], rows ordered by NMS keep order;
 * d_counts: B int32 kept counts.  d_dets / d_counts must be device pointers.  The forward of a (shape, input,
 * counts, args) key is captured once as a HIP graph; a later call with other d_dets rows replays it with its NMS
 * nodes re-pointed (no recapture, no copy), so a caller may hand in fresh output rows every call. */
int ym_infer(ym_ctx* ctx, const float* d_input, int B, int H, int W, const ym_infer_args* args, float* d_dets,
             int* d_counts, void* stream);

/* LoadTensor statistics of a device batch: *d_max = max over the n fp32 elements of d_input (asynchronous on
 * `stream`).  Each rank of a batch-sharded run computes its shard's max, the ranks all-reduce it (MAX), and pass the
 * result as ym_infer_args.d_batch_max, so the /255 decision is the whole batch's, as in the reference. */
int ym_input_max(ym_ctx* ctx, const float* d_input, size_t n, float* d_max, void* stream);

/* PTQ calibration support (f32 plans only): one eager forward in which op i also writes its pre-activation output
 * to d_raw[i] (device pointer or NULL; fp32 row-major (pixels, channels): conv / depthwise ops their conv output, the
 * attention op its positional depthwise conv pe(v), ConvTranspose2d its (pixels, 4·C) GEMM output).  Feeds the
 * conv-output observers of the reference's PostTrainingQuantizer (optimization/quantization/quantizers.py:146-177).
 * Asynchronous on `stream`. */
int ym_calibrate(ym_ctx* ctx, const float* d_input, int B, int H, int W, const ym_infer_args* args, float* d_dets,
                 int* d_counts, float* const* d_raw, int n_ops, void* stream);

/* Eager run with a HIP event pair around every op: op_ms[i] = device time of op i (n_ops entries). */
int ym_profile(ym_ctx* ctx, const float* d_input, int B, int H, int W, const ym_infer_args* args, float* d_dets,
               int* d_counts, void* stream, float* op_ms, int n_ops);

/* Per-op device time without per-op markers: after one real forward, every conv / depthwise / SPPF / attention op
 * is captured as a graph of `reps` back-to-back launches on the real buffers and timed with one HIP event pair;
 * op_ms[i] = that time / reps (launch gaps included, as in the forward graph).  Ops that are not idempotent
 * (input statistics, decode, NMS) get -1.  Synchronous; leaves the activation buffers in an unspecified state. */
int ym_profile_replay(ym_ctx* ctx, const float* d_input, int B, int H, int W, const ym_infer_args* args,
                      float* d_dets, int* d_counts, void* stream, int reps, float* op_ms, int n_ops);

/* On-device autotuning of the conv tile configuration, per op, for input shape (B, H, W): every candidate is timed
 * as `reps` graph-captured back-to-back launches on this GPU (after one real forward so the buffers hold real
 * activations); the fastest is kept for this shape (one table per (B, H, W)).  Synchronous.  ym_get_op_cfg /
 * ym_set_op_cfg export / import the per-op choices for a shape (n_ops ints, -1 = built-in heuristic) so a tuned plan
 * can be cached and pinned; ym_get_op_cfg returns 1 (and all -1) when the shape has no table. */
int ym_tune(ym_ctx* ctx, const float* d_input, int B, int H, int W, const ym_infer_args* args, float* d_dets,
            int* d_counts, void* stream, int reps);
int ym_get_op_cfg(ym_ctx* ctx, int B, int H, int W, int* cfg, int n_ops);
int ym_set_op_cfg(ym_ctx* ctx, int B, int H, int W, const int* cfg, int n_ops);

/* Introspection for tests / bisecting: op count & names, and the device view of plan buffer `buf` as produced by
 * the last ym_infer/ym_profile (NHWC; elem_bytes 2 = fp16, 4 = fp32; for the anchor buffer H=1, W=A). */
int ym_num_ops(ym_ctx* ctx);
const char* ym_op_name(ym_ctx* ctx, int i);
int ym_num_buffers(ym_ctx* ctx);
int ym_buffer_info(ym_ctx* ctx, int buf, void** ptr, int* C, int* H, int* W, int* elem_bytes);

/* Copy the first `bytes` of plan buffer `buf` (as left by the last ym_infer/ym_profile) to `dst` (host or device
 * pointer); synchronous. */
int ym_read_buffer(ym_ctx* ctx, int buf, void* dst, size_t bytes);

/* Segment plans: instance masks of the detections of the last ym_infer (same B, H, W, stream order), i.e. Ultralytics
 * `ops.process_mask(proto, coef, boxes, (H, W), upsample=True)` per image.  d_dets: the ym_infer output rows;
 * d_offsets: B+1 device ints, offsets[b] = first mask of image b, offsets[B] = total (prefix of the kept counts);
 * d_masks: total x H x W bytes (1 = inside the instance); d_nonempty: total ints, 1 when the mask has any pixel
 * set (the predictor drops empty masks).  Asynchronous on `stream`. */
int ym_masks(ym_ctx* ctx, const float* d_dets, int B, int max_det, const int* d_offsets, int total, int H, int W,
             unsigned char* d_masks, int* d_nonempty, void* stream);

/* Segment plans, single-sync form of ym_masks: the masks of the first min(counts[b], cap) detections of every image,
 * taken from the DEVICE counts of the last ym_infer (d_counts, B ints), so the masks are enqueued right behind the
 * forward with no host round trip in between.  d_masks: B x cap x H x W bytes, slot (b, i) = detection i of image b
 * (unused slots are left unwritten); d_flags: B*cap + B ints = the non-empty flag of every slot (0 when unused),
 * then a copy of the B counts, so ONE device->host read of d_flags returns both.  The caller checks counts[b] <= cap
 * (else it calls ym_masks for that batch).  Same arithmetic as ym_masks.  Asynchronous on `stream`. */
int ym_masks_slots(ym_ctx* ctx, const float* d_dets, int B, int max_det, const int* d_counts, int cap, int H, int W,
                   unsigned char* d_masks, int* d_flags, void* stream);

/* Image sources: Ultralytics `LetterBox` + predictor preprocessing of ONE HWC uint8 image already
 * in device memory (d_src, rows row_bytes apart, 3 channels; bgr = 1 for cv2.imread order).  The image is resized to
 * uh x uw with OpenCV's 8-bit INTER_LINEAR fixed-point arithmetic (skipped when the size does not change), placed at
 * (top, left) of an Hn x Wn canvas filled with 114, converted to RGB planes and divided by 255 into d_dst (3 x Hn x Wn
 * fp32: one image of the batch ym_infer reads).  The geometry is the caller's (LetterBox arithmetic, see
 * yolomi/preprocess.py).  Asynchronous on `stream`.  Replaces the reference's cv2-based preprocessing under
 * YOLO11Model.predict(path | ndarray) (/root/reference/core/model.py:118-133, demos/detection_demo.py:87-93). */
int ym_letterbox(ym_ctx* ctx, const void* d_src, int h, int w, int row_bytes, int bgr, int uh, int uw, int top,
                 int left, float* d_dst, int Hn, int Wn, void* stream);

int ym_sync(ym_ctx* ctx);
const char* ym_last_error(void);
void ym_destroy(ym_ctx* ctx);
int ym_version(void);
/* Size of the conv tile-configuration catalogue of a plan dtype (ym_model_desc codes: 1 f16, 2 f32, 3 i8, 4 f8, 5 x3;
 * YM_EINVAL otherwise): the id space of the ym_get_op_cfg / ym_set_op_cfg tables, so a cached table is reused only
 * by a library with the same catalogue. */
int ym_num_conv_cfgs(int dtype);

/* Process-wide debug switches for tests and A/B runs (not part of the reference interface; defaults 0), read when a
 * kernel is launched (so at graph capture for replayed forwards): YM_DBG_NMS (9 = the NMS kernel's per-box path
 * instead of the blocked one), YM_DBG_DW_MODE (depthwise variant: 0 LDS tiles, 1 rows, 2 column strips),
 * YM_DBG_DW_TILE (LDS tile shape 0..3), YM_DBG_CHAIN (1: the persistent two-conv chain kernel).
 * The environment variables YM_NMS_DBG, YM_DW_MODE, YM_DW_TILE, YM_CHAIN, YM_STEMFUSE, YM_ATTN_KB, YM_PAIRST and
 * YM_CONV_CFG (the last two: the value itself, stored + 1) set the initial values.  A forward graph
 * already captured keeps the kernels it was captured with.
 * Returns the previous value, or YM_EINVAL for an unknown key. */
#define YM_DBG_NMS 1
#define YM_DBG_DW_MODE 2
#define YM_DBG_DW_TILE 3
#define YM_DBG_CHAIN 4 /* 1: dependent x3 3x3 pairs on one LDS-DMA configuration as one persistent launch */
#define YM_DBG_CHAIN_LAUNCHES 5 /* chain kernels launched since it was last set (a counter) */
#define YM_DBG_STEMFUSE 6 /* 1: x3 stem + model.1 + model.2.cv1 as one launch (csrc/ym_stem_fused.hip); 0: three */
#define YM_DBG_ATTN_KB 7 /* 1: x3 attention loads K fragments 8 key tiles per round trip; 0: all tiles at once */
#define YM_DBG_PAIRST 8 /* x3 lane-pair epilogue store family mask + 1 (0: the default mask 21) */
#define YM_DBG_CONV_CFG 9 /* a forced conv tile configuration id + 1 for untuned ops (0: the heuristic) */
int ym_set_debug(int key, int value);

#ifdef __cplusplus
}
#endif
#endif /* YOLOMI_H */
