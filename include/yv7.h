/* yv7.h — C ABI of the MI355X-native YOLOv7 inference path (libyv7.so, gfx950).
 *
 * Plain C types only: every tensor crosses the boundary as a device pointer plus sizes; streams
 * cross as hipStream_t passed as void*.  Every call returns 0 on success, a positive hipError_t
 * on a HIP failure, or a negative yv7_status on an argument / shape error; the message is in the
 * thread-local yv7_last_error().  Nothing throws or aborts across the ABI.  The caller owns every
 * input, output and workspace buffer; a plan owns only its packed weights and small tables.
 *
 * What each entry point replaces in the reference (qbxlvnf11/yolo-series):
 *   yv7_plan_create   attempt_load() -> Model.fuse() product   models/experimental.py:247-270,
 *                     models/yolo.py:693-710 (the fused, deploy-form network: weights folded on the
 *                     host by the Python mirror, packed NHWC/KRSC and handed over here once)
 *   yv7_forward       Model.forward / forward_once            models/yolo.py:581-631, including every
 *                     layer forward (Conv.fuseforward common.py:110-111, RepConv common.py:498-500,
 *                     SPPCSPC common.py:276-280, MP/SP common.py:30-45, ReOrg common.py:48-53,
 *                     Concat common.py:56-62, nn.Upsample) and Detect/IDetect decode yolo.py:42-63,140-160
 *   yv7_nms           non_max_suppression()                   utils/general.py:628-720 incl. the
 *                     torchvision.ops.nms call at general.py:704
 *   yv7_end2end       TRT EfficientNMS_TRT plugin contract    models/experimental.py:111-156,
 *                     utils/add_nms.py:94-138 (fixed-shape num_dets/boxes/scores/classes)
 *   yv7_letterbox     letterbox() + the detect.py input         utils/datasets.py:1277-1307,
 *                     conversion                                detect.py:100-104, datasets.py:199
 */
#ifndef YV7_H
#define YV7_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define YV7_ABI_VERSION 4

/* Activation tensors in the forward workspace are NHWC with a YV7_BORDER-pixel zero frame around
 * every image: [B][h + 2*YV7_BORDER][w + 2*YV7_BORDER][C].  Kernels write only interiors; the frame
 * serves every 3x3 / pad-1 window's out-of-image taps.  yv7_forward clears a workspace the first
 * time it sees it with a given layout (pointer, size and batch geometry B, H, W) and trusts the frame
 * on later calls with that layout.  So between calls the workspace memory belongs to the plan: a
 * caller that frees it, reuses it for anything else or writes into it calls yv7_workspace_forget
 * first (the Python binding does so whenever it drops a workspace). */
#define YV7_BORDER 1

typedef enum {
  YV7_OK = 0,
  YV7_E_ARG = -1,       /* bad argument (null pointer, bad enum) */
  YV7_E_SHAPE = -2,     /* shape not supported by the plan (e.g. H/W not a multiple of max stride) */
  YV7_E_WORKSPACE = -3, /* workspace too small */
  YV7_E_ABI = -4,       /* descriptor abi_version mismatch */
  YV7_E_DEVICE = -5     /* no gfx950 device / wrong device */
} yv7_status;

typedef enum { YV7_DT_F32 = 0, YV7_DT_F16 = 1 } yv7_dtype;
typedef enum { YV7_ACT_NONE = 0, YV7_ACT_SILU = 1, YV7_ACT_LEAKY = 2 } yv7_act;
/* Weight / arithmetic format of one CONV op.  FP8 (fp16 plans, 1x1 stride-1 convs only; BASELINE
 * configs[4]): weights OCP e4m3 [cout_pad32][cin padded to 128] at w_off with fp32 per-output-channel
 * scales [cout] at s_off; the fp16 input is quantized per tensor, x8 = e4m3(clamp(x / xscale, +-448)),
 * and the GEMM runs on the block-scaled fp8 MFMA; y = act(acc * xscale * wscale[c] + bias[c]). */
typedef enum { YV7_WFMT_PLAN = 0, YV7_WFMT_FP8 = 1 } yv7_wfmt;

typedef enum {
  YV7_OP_INPUT = 0,    /* NCHW image batch -> NHWC tensor; k=2 means fused ReOrg space-to-depth */
  YV7_OP_CONV = 1,     /* k x k conv, stride s, pad, + fp32 bias + act; NHWC channel slices in/out */
  YV7_OP_MAXPOOL = 2,  /* max pool k, stride s, pad (implicit -inf padding) */
  YV7_OP_UPSAMPLE = 3, /* nearest-neighbour x2 */
  YV7_OP_COPY = 4,     /* channel-slice copy (concat input that could not be written in place) */
  YV7_OP_DETECT = 5,   /* 1x1 conv + bias + sigmoid + grid/anchor decode -> z rows, raw logits */
  YV7_OP_STEM = 6      /* fp16: image -> conv A (3->32, 3x3, stride s) -> conv B (32->64, 3x3, s2), A kept in LDS;
                          cin 12: the yolov7-w6 front end, image -> ReOrg (common.py:48-53) -> conv A (12->64,
                          3x3, s1; weights K = tap*16 + ci) -> conv B (64->128, 3x3, s2) */
} yv7_op_kind;

/* One NHWC activation tensor of the plan: [B, H >> shift, W >> shift, channels]. Tensor 0 is the
 * packed network input written by YV7_OP_INPUT. */
typedef struct {
  int32_t channels; /* channel count == row pitch in elements (multiple of 8) */
  int32_t shift;    /* log2 spatial downsampling relative to the network input */
} yv7_tensor_desc;

typedef struct {
  int32_t kind;                /* yv7_op_kind */
  int32_t src, src_coff, cin;  /* input tensor, channel offset, channels read */
  int32_t dst, dst_coff, cout; /* output tensor, channel offset, channels written */
  int32_t k, s, pad, act;      /* window / stride / padding / yv7_act */
  int32_t level;               /* DETECT: head level */
  int64_t w_off;               /* CONV/DETECT: byte offset of weights [cout_pad32][k][k][cin], K padded to 64 */
  int64_t b_off;               /* CONV/DETECT: byte offset of fp32 bias [cout_pad] */
  int32_t cout2, act2;         /* STEM: second conv's output channels / activation */
  int64_t w2_off, b2_off;      /* STEM: second conv's weights / bias */
  int32_t wfmt;                /* CONV: yv7_wfmt */
  float xscale;                /* CONV, wfmt FP8: per-tensor input scale (a power of two) */
  int64_t s_off;               /* CONV, wfmt FP8: byte offset of fp32 weight scales [cout] */
  int32_t pool;                /* CONV (fp16 plans, 1x1): 2 = the input is first max-pooled 2x2 / stride 2 (an MP
                                  layer, common.py:30-36, folded into the conv's operand loads); then s = 2 */
  int32_t reserved;
} yv7_op_desc;

typedef struct {
  int32_t abi_version;   /* YV7_ABI_VERSION */
  int32_t dtype;         /* yv7_dtype of activations and packed weights */
  int32_t n_tensors;
  const yv7_tensor_desc* tensors;
  int32_t n_ops;
  const yv7_op_desc* ops;
  int32_t nl, na, no;    /* detection levels, anchors per level, outputs per anchor (nc + 5) */
  const float* stride;   /* [nl] */
  const float* anchor_grid; /* [nl][na][2] anchor sizes in pixels (Detect.anchor_grid) */
  int32_t max_shift;     /* input H and W must be multiples of 1 << max_shift */
} yv7_net_desc;

typedef struct yv7_plan yv7_plan;

int32_t yv7_abi_version(void);
const char* yv7_last_error(void);

/* weights: host or device pointer to the packed blob (copied into plan-owned device memory). */
int yv7_plan_create(const yv7_net_desc* desc, const void* weights, size_t nbytes, int device,
                    yv7_plan** out);
void yv7_plan_destroy(yv7_plan* plan);

/* Bytes of caller-provided workspace yv7_forward needs for a [B,3,H,W] batch. */
size_t yv7_workspace_bytes(const yv7_plan* plan, int B, int H, int W);
/* Hand workspace memory [ws, ws + bytes) back to the caller: the next yv7_forward on any part of it
 * clears it again. */
int yv7_workspace_forget(yv7_plan* plan, const void* ws, size_t bytes);
/* Rows of z per image: sum over levels of na * (H >> s_l) * (W >> s_l). */
int64_t yv7_num_rows(const yv7_plan* plan, int H, int W);

/* Per-row detection score record (16 bytes), one per row of z: the objectness z[..., 4], the
 * single-label NMS score max_c z[..., 5 + c] * z[..., 4] with its first-max class (general.py:669-684,
 * computed from the very floats written to z).  yv7_nms / yv7_end2end accept it instead of
 * re-reading every row of z for the candidate filter. */
typedef struct {
  float obj;
  float conf;
  int32_t cls;
  int32_t reserved;
} yv7_row_best;

/* x: [B,3,H,W] (x_dtype f32 or f16, values in [0,1]) on the plan's device.
 * z_out: [B, N, no] fp32 decoded boxes (Detect z).  raw_out (nullable): per level l the raw head
 * logits [B, na, ny_l, nx_l, no] fp32, levels concatenated.  rowbest_out (nullable): [B, N]
 * yv7_row_best (fp16 plans write it from the head's epilogue).  Asynchronous on `stream`. */
int yv7_forward(yv7_plan* plan, const void* x, int x_dtype, int B, int H, int W, float* z_out,
                float* raw_out, yv7_row_best* rowbest_out, void* workspace, size_t ws_bytes, void* stream);

/* The kernels the dispatch launches for every op of a [B,3,H,W] forward, without running it (a dry
 * run of yv7_forward's op loop): one line per op, "op<TAB>kernel[|kernel...]", kernel = the demangled
 * symbol rocprofv3's kernel trace reports.  Lets a caller attribute per-op timings (yv7_profile_read)
 * to kernel families.  x_dtype: the image dtype the forward would get (the INPUT / STEM kernels depend on
 * it).  An op that would launch more than 4 kernels is an error.  Needs the plan's device to be current;
 * buf receives a NUL-terminated string. */
int yv7_op_kernels(yv7_plan* plan, int B, int H, int W, int x_dtype, char* buf, size_t bytes);

/* Force the kernel configuration of one CONV / DETECT op (0 = the tuned dispatch, the default).  For
 * parity tests of every kernel variant and A/B timing; the accepted values are the real kernel
 * configurations of the fp16 dispatch (csrc/conv_f16.hip), never its microbenchmark hooks.  A split-K
 * variant changes yv7_workspace_bytes. */
int yv7_set_op_variant(yv7_plan* plan, int op, int variant);

/* Live per-op timing: with max_forwards > 0 every following yv7_forward (up to max_forwards of
 * them) launches each op's kernels with a (start, stop) HIP event pair (hipExtLaunchKernel: the
 * first kernel's dispatch begin, the last kernel's end — the interval rocprofv3's kernel trace
 * reports); an op that launches nothing records both events back to back.  0 turns it off and frees
 * the events.  yv7_profile_read synchronizes on the recorded events and returns, per op, the elapsed
 * milliseconds summed over the recorded forwards (op_ms: [n_ops]). */
int yv7_profile_enable(yv7_plan* plan, int max_forwards);
int yv7_profile_read(yv7_plan* plan, int* n_forwards, float* op_ms);

/* Byte offset of activation tensor `tensor_id` inside the forward workspace and its bordered NHWC dims
 * (B, h + 2*YV7_BORDER, w + 2*YV7_BORDER, C); the image interior starts at [YV7_BORDER][YV7_BORDER].
 * Lets a caller read any intermediate layer for per-layer parity checks. */
int yv7_tensor_info(const yv7_plan* plan, int tensor_id, int B, int H, int W, int64_t* offset,
                    int64_t* dims4);

/* Byte range of the fp8 staging buffer inside the forward workspace (the dense e4m3 copy of an FP8
 * op's input; after a forward it holds the last FP8 op's quantized input).  bytes = 0 when the plan
 * has no FP8 op.  For parity tests of the quantization. */
int yv7_f8_scratch_info(const yv7_plan* plan, int B, int H, int W, int64_t* offset, int64_t* bytes);

/* Batched NMS over z [B,N,no] fp32, the semantics of utils/general.py:628-720.
 * det: [B,max_det,6] (x1,y1,x2,y2,conf,cls), src_row: [B,max_det] int64 anchor row of each kept
 * box, count: [B] int32.  classes: nullable [ncls] int32 class filter.  rowbest (nullable): the
 * yv7_row_best records of z from yv7_forward; used for the single-label, unfiltered case. */
size_t yv7_nms_workspace_bytes(int B, int N, int no, int multi_label, int max_nms);
int yv7_nms(const float* z, const yv7_row_best* rowbest, int B, int N, int no, float conf_thres,
            float iou_thres, int multi_label, int agnostic, const int32_t* classes, int ncls, int max_det,
            int max_nms, float* det, int64_t* src_row, int32_t* count, void* workspace, size_t ws_bytes,
            void* stream);

/* EfficientNMS_TRT-shaped output (End2End, experimental.py:226-241): num_dets int32 [B,1],
 * det_boxes [B,topk,4], det_scores [B,topk], det_classes int32 [B,topk]; zero-padded. */
size_t yv7_end2end_workspace_bytes(int B, int N, int no, int topk);
int yv7_end2end(const float* z, int B, int N, int no, float conf_thres, float iou_thres, int topk,
                int32_t* num_dets, float* det_boxes, float* det_scores, int32_t* det_classes,
                void* workspace, size_t ws_bytes, void* stream);

/* Frame pre-processing (replaces utils/datasets.py:1277-1307 letterbox() with its cv2.resize
 * INTER_LINEAR + cv2.copyMakeBorder, and detect.py:100-104's BGR->RGB / HWC->CHW / half / 255):
 * src: B uint8 frames [B][H][W][3] BGR on the device; the host computes the letterbox geometry
 * (new_h x new_w resized image placed at (top, left) of an out_h x out_w canvas of colour
 * (pad_b, pad_g, pad_r)), exactly as letterbox() does.  out_kind: 0 = uint8 [B][out_h][out_w][3]
 * BGR (the letterboxed frame), 1 = fp16 [B][3][out_h][out_w] RGB / 255, 2 = fp32 likewise (the model
 * input).  The workspace holds the resize tables (yv7_letterbox_workspace_bytes).  Asynchronous. */
size_t yv7_letterbox_workspace_bytes(int new_h, int new_w);
int yv7_letterbox(const void* src, int B, int H, int W, int new_h, int new_w, int top, int left, int out_h,
                  int out_w, int pad_b, int pad_g, int pad_r, int out_kind, void* dst, void* workspace,
                  size_t ws_bytes, void* stream);

#ifdef __cplusplus
}
#endif

#endif /* YV7_H */
