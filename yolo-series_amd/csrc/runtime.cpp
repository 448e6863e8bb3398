// libyv7 runtime: the C ABI of include/yv7.h — plan creation (packed weights to HBM), workspace
// layout, the per-batch launch sequence of the fused network, NMS and the End2End output mode.
//
// A plan is the deploy-form network (attempt_load -> Model.fuse, models/experimental.py:247-270)
// as a flat list of ops over NHWC tensors.  yv7_forward walks that list once per batch, launching
// one kernel per op on the caller's stream (forward_once's per-layer loop, models/yolo.py:603-627,
// without the Python dispatch); no allocation, no host sync, so callers can capture it in a graph.
#include <cxxabi.h>
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdlib>
#include <cstdio>
#include <cstring>
#include <string>
#include <vector>

#include "../../include/yv7.h"
#include "yv7_kernels.h"

namespace yv7 {
size_t nms_workspace_bytes(int B, int N, int no, int multi, int max_nms);
hipError_t launch_nms(const float* z, const void* rowbest, int B, int N, int no, float conf, float iou, int multi,
                      int agnostic, int per_class, const int32_t* classes, int ncls, int max_det, int max_nms,
                      float* det, int64_t* src_row, int32_t* count, void* ws, hipStream_t st);
hipError_t launch_row_best(const float* z, int B, int N, int no, void* rowbest, hipStream_t st);
size_t letterbox_workspace_bytes(int nh, int nw);
hipError_t launch_letterbox(const uint8_t* src, int B, int H, int W, int nh, int nw, int top, int left, int oh,
                            int ow, const uint8_t pad[3], int out_kind, void* dst, void* ws, hipStream_t st);
hipError_t launch_end2end_pack(const float* det, const int32_t* count, int B, int max_det, int topk,
                               int32_t* num_dets, float* boxes, float* scores, int32_t* classes, hipStream_t st);
}  // namespace yv7

struct yv7_plan {
  int device = 0;
  int dtype = 0;
  std::vector<yv7_tensor_desc> tensors;
  std::vector<yv7_op_desc> ops;
  int nl = 0, na = 0, no = 0, max_shift = 0;
  std::vector<float> stride, anchor_grid;
  void* weights = nullptr;
  size_t wbytes = 0;
  void* zero = nullptr;  // 4 KiB of zeros
  // fp16 plans: every 3x3 stride-1/2 conv's weights again, fragment-packed for conv_lr.hip (pack_frag);
  // wf_off[op] = byte offset into wfrag, -1 when the op has none
  void* wfrag = nullptr;
  std::vector<int64_t> wf_off;
  // the workspaces whose zero frames are known to be intact for one layout (see yv7_forward); several,
  // so that batches in flight can run concurrently on their own streams and workspaces
  struct WsKey {
    const void* ptr;
    size_t bytes;
    int B, H, W;
  };
  std::vector<WsKey> ws_ready;
  // per-op kernel variant override (0 = tuned dispatch; yv7_set_op_variant)
  std::vector<int> op_variant;
  // live profiling: events[f * 2 * n_ops + 2 * i + {0: start, 1: stop}] of op i in profiled forward f
  std::vector<hipEvent_t> events;
  int prof_max = 0, prof_used = 0;
};

namespace {

thread_local std::string g_err;

int fail(int code, const std::string& msg) {
  g_err = msg;
  return code;
}

int hip_fail(hipError_t e, const char* where) {
  g_err = std::string(where) + ": " + hipGetErrorString(e);
  return (int)e;
}

size_t elem_size(int dtype) { return dtype == YV7_DT_F16 ? 2 : 4; }
size_t align256(size_t x) { return (x + 255) & ~(size_t)255; }

size_t tensor_bytes(const yv7_plan* p, const yv7_tensor_desc& t, int B, int H, int W) {
  return yv7::bordered_pixels(B, H >> t.shift, W >> t.shift) * t.channels * elem_size(p->dtype);
}

// Byte offset of every tensor inside the workspace for a [B,3,H,W] batch: bordered NHWC
// [B][h + 2*YV7_BORDER][w + 2*YV7_BORDER][C] each, 256-byte aligned.
std::vector<size_t> tensor_offsets(const yv7_plan* p, int B, int H, int W, size_t* total) {
  std::vector<size_t> off(p->tensors.size());
  size_t o = 0;
  for (size_t i = 0; i < p->tensors.size(); ++i) {
    off[i] = o;
    o = align256(o + tensor_bytes(p, p->tensors[i], B, H, W));
  }
  *total = o;
  return off;
}

int check_hw(const yv7_plan* p, int B, int H, int W) {
  const int m = (1 << p->max_shift) - 1;
  if (B <= 0 || H <= 0 || W <= 0 || (H & m) || (W & m))
    return fail(YV7_E_SHAPE, "input H and W must be positive multiples of " + std::to_string(1 << p->max_shift) +
                                 " (got B=" + std::to_string(B) + " H=" + std::to_string(H) + " W=" +
                                 std::to_string(W) + ")");
  // kernels address a tensor with 32-bit byte offsets (buffer loads)
  for (const auto& t : p->tensors)
    if (tensor_bytes(p, t, B, H, W) >= (size_t(1) << 31))
      return fail(YV7_E_SHAPE, "batch too large: an activation tensor would exceed 2 GiB (split the batch)");
  return 0;
}

// K padding of a conv's packed weights: 64 in the plan dtype, 128 for fp8 (one MFMA K step)
int kpad_of(const yv7_op_desc& o) {
  if (o.kind == YV7_OP_CONV && o.wfmt == YV7_WFMT_FP8) return (o.cin + 127) / 128 * 128;
  return (o.k * o.k * o.cin + 63) / 64 * 64;
}
bool is_f8(const yv7_op_desc& o) { return o.kind == YV7_OP_CONV && o.wfmt == YV7_WFMT_FP8; }
// 3x3 / stride-1 or 2 / pad-1 fp16 convs of a shape the fragment kernels accept (conv_lr.hip lr_supported:
// cin / 32 in {2, 4, 6, 8, 12, 16, 24}, cout % 16 == 0, cout <= 1024; conv_s2.hip: cin 64 / 128) get a
// fragment-packed weight copy, and so do 1x1 stride-1 convs with 128 / 256 / 512 inputs (conv_w1.hip) —
// none at all with YV7_FRAG=0 (every fragment kernel then stays off: conv_lr, the register-weight 3x3 / 1x1
// kernels and the register-weight Detect head; the forced variants 270-288 / 290-295 / 302-303 fall back to
// the tuned kernel).  YV7_LR=0 only takes conv_lr out of the dispatch (it used to switch the
// packing, i.e. four kernel families, off at once).  Per fp16 plan: yolov7 54.0 MB (3x3 49.8 + 1x1 4.1) beside its 73.9 MB
// blob, yolov7-w6 112.4 MB, yolov7-tiny 10.3 MB.
bool wants_frag(int dtype, const yv7_op_desc& o) {
  static const int lr = [] { const char* e = getenv("YV7_FRAG"); return e ? atoi(e) : 1; }();
  const int nch = o.cin / 32;
  // the Detect head conv with K = 256 / 512 (conv_det_rw_kernel: the weights resident in VGPRs)
  if (dtype == YV7_DT_F16 && o.kind == YV7_OP_DETECT)
    return lr && o.k == 1 && (o.cin == 256 || o.cin == 512) && o.cout <= 256;
  if (!lr || dtype != YV7_DT_F16 || o.kind != YV7_OP_CONV || is_f8(o) || o.pool || o.cout % 16 || o.cout > 1024)
    return false;
  if (o.k == 1)   // conv_w1.hip: 1x1 stride 1 with 128 / 256 / 512 inputs
    return o.s == 1 && o.pad == 0 && (o.cin == 128 || o.cin == 256 || o.cin == 512);
  return o.k == 3 && (o.s == 1 || o.s == 2) && o.pad == 1 && o.cin % 32 == 0 &&
         (nch == 2 || nch == 4 || nch == 6 || nch == 8 || nch == 12 || nch == 16 || nch == 24);
}

// Geometry / operand fields of a CONV or DETECT op's kernel parameters (pointers into the workspace
// are filled by the caller).
yv7::ConvParams conv_params(const yv7_plan* p, size_t op, int B, int H, int W) {
  const yv7_op_desc& o = p->ops[op];
  const auto& ti = p->tensors[o.src];
  const size_t es = elem_size(p->dtype);
  yv7::ConvParams c;
  std::memset(&c, 0, sizeof(c));
  c.B = B;
  c.H = H >> ti.shift;
  c.W = W >> ti.shift;
  c.xc = ti.channels;
  c.xoff = o.src_coff;
  c.cin = o.cin;
  c.Ho = (c.H + 2 * o.pad - o.k) / o.s + 1;
  c.Wo = (c.W + 2 * o.pad - o.k) / o.s + 1;
  c.cout = o.cout;
  c.k = o.k;
  c.s = o.s;
  c.pad = o.pad;
  c.act = o.act;
  c.pool = o.kind == YV7_OP_CONV ? o.pool : 0;
  c.kpad = kpad_of(o);
  c.K = o.k * o.k * o.cin;
  c.M = B * c.Ho * c.Wo;
  c.xbytes = (uint32_t)tensor_bytes(p, ti, B, H, W);
  c.wbytes = (uint32_t)((size_t)((o.cout + 31) / 32 * 32) * c.kpad * es);
  c.variant = p->op_variant[op] == 305 ? 0 : p->op_variant[op];   // 305: a chain start (find_chain)
  if (p->wfrag && p->wf_off[op] >= 0) {
    c.wf = reinterpret_cast<const unsigned char*>(p->wfrag) + p->wf_off[op];
    c.wfbytes = (uint32_t)yv7::frag_bytes(o.cin, o.cout, o.k * o.k);
  }
  return c;
}

// Split-K scratch behind the activation tensors: fp32 partial tiles (the largest any conv of the
// plan needs; convs run one at a time) and the per-tile arrival counters (zeroed with the workspace,
// re-armed by the kernels).
struct SplitScratch {
  size_t part_off = 0, part_bytes = 0, cnt_off = 0;
  int cnt_n = 0;
  size_t f8_off = 0, f8_bytes = 0;   // dense e4m3 copy of an FP8 op's input (the largest one)
  size_t chain_off = 0, chain_bytes = 0;   // ready counters of a chained 3x3 launch (the largest chain)
  size_t end = 0;
};

// A chain of 3x3 stride-1 fp16 convs starting at op i that the runtime launches as ONE kernel
// (conv_lr.hip conv3x3_chain_kernel: an ELAN block's 3x3 stack): ops i .. i + n - 1, each reading the
// previous one's output slice, all of a shape the low-resolution kernel takes.  NOT in the default dispatch:
// measured slower than the per-layer launches on every yolov7 bs 32 stack it applies to (round 6,
// profiles/r6_chain/: 20^2 256 x 4 116.8 vs 89.4 us, 40^2 128 x 4 130.0 vs 105.0; bench 7679 / 7710 vs 7847 /
// 7868 img/s) — each layer's 640 tiles are one round of the chip, so the next layer's tiles find nothing to
// overlap with, and the queue's dequeues plus the polls cost more than the three kernel boundaries they
// remove.  Forced per chain with variant 305 on its first op (yv7_set_op_variant; the later ops on 0);
// YV7_CHAIN=1 chains every eligible stack.  Fills *c (pointers from workspace base wsb, null for a layout
// query) and returns n (0: no chain here).
int find_chain(const yv7_plan* p, size_t i, int B, int H, int W, const std::vector<size_t>& off, unsigned char* wsb,
               yv7::ChainParams* c) {
  static const int all = [] { const char* e = getenv("YV7_CHAIN"); return e ? atoi(e) : 0; }();
  static const long max_tasks = [] { const char* e = getenv("YV7_CHAIN_TASKS"); return e ? atol(e) : 1280L; }();
  if (p->dtype != YV7_DT_F16 || i >= p->ops.size()) return 0;
  const bool forced = p->op_variant[i] == 305;
  if (!forced && !all) return 0;
  const unsigned char* wb = reinterpret_cast<const unsigned char*>(p->weights);
  auto eligible = [&](size_t j) {
    const auto& o = p->ops[j];
    return o.kind == YV7_OP_CONV && !is_f8(o) && o.k == 3 && o.s == 1 && o.pad == 1 && !o.pool &&
           p->op_variant[j] == (j == i && forced ? 305 : 0) && o.act == p->ops[i].act;
  };
  if (!eligible(i)) return 0;
  size_t n = 1;
  while (n < (size_t)yv7::CHAIN_MAX && i + n < p->ops.size() && eligible(i + n)) {
    const auto& a = p->ops[i + n - 1];
    const auto& b = p->ops[i + n];
    if (b.src != a.dst || b.src_coff != a.dst_coff || b.cin != a.cout) break;
    ++n;
  }
  // no layer's output may overlap the chain's input slice or another layer's output
  auto overlap = [](int ta, int ca, int na, int tb, int cb, int nb) { return ta == tb && ca < cb + nb && cb < ca + na; };
  for (; n >= 2; --n) {
    bool ok = true;
    for (size_t j = 0; j < n && ok; ++j) {
      const auto& oj = p->ops[i + j];
      if (overlap(oj.dst, oj.dst_coff, oj.cout, p->ops[i].src, p->ops[i].src_coff, p->ops[i].cin)) ok = false;
      for (size_t k = 0; k < j && ok; ++k) {
        const auto& ok_ = p->ops[i + k];
        if (overlap(oj.dst, oj.dst_coff, oj.cout, ok_.dst, ok_.dst_coff, ok_.cout)) ok = false;
      }
    }
    if (!ok) continue;
    std::memset(c, 0, sizeof(*c));
    c->nl = (int)n;
    for (size_t j = 0; j < n && ok; ++j) {
      const auto& o = p->ops[i + j];
      yv7::ConvParams& q = c->p[j];
      q = conv_params(p, i + j, B, H, W);
      const auto& to = p->tensors[o.dst];
      q.x = wsb + off[o.src];
      q.w = wb + o.w_off;
      q.bias = reinterpret_cast<const float*>(wb + o.b_off);
      q.zero = p->zero;
      q.y = wsb + off[o.dst];
      q.yc = to.channels;
      q.yoff = o.dst_coff;
      q.variant = 0;
      if (q.Ho != (H >> to.shift) || q.Wo != (W >> to.shift)) ok = false;
      int cfg = yv7::lr_default_cfg(q);
      if (cfg == 0 || cfg == 2) ++cfg;   // 128-channel tiles -> 64-channel (conv_lr.hip CHAIN_FORMS)
      if (cfg == 5 || cfg == 6) cfg = 1;  // 160-pixel tiles (H % 10 == 0) -> the 80-pixel 64-channel form
      if (cfg < 0 || (j > 1 && cfg != c->cfg1)) ok = false;
      if (j == 0) c->cfg0 = cfg;
      if (j == 1) c->cfg1 = cfg;
    }
    if (!ok || !yv7::chain_supported(*c)) continue;
    // (YV7_CHAIN=1: only where a layer has few tiles, its ramp and tail dominating)
    if (!forced && yv7::chain_tasks(*c) > max_tasks * (long)n) return 0;
    return (int)n;
  }
  return 0;
}

SplitScratch split_scratch(const yv7_plan* p, int B, int H, int W, size_t tensors_end) {
  SplitScratch s;
  if (p->dtype == YV7_DT_F16) {
    for (size_t i = 0; i < p->ops.size(); ++i) {
      const auto& o = p->ops[i];
      if (o.kind == YV7_OP_CONV && !is_f8(o)) {
        const yv7::ConvParams c = conv_params(p, i, B, H, W);
        s.part_bytes = std::max(s.part_bytes, yv7::conv_splitk_part_bytes(c));
        s.cnt_n = std::max(s.cnt_n, yv7::conv_splitk_tiles(c));
      } else if (is_f8(o)) {
        const int sh = p->tensors[o.src].shift;
        s.f8_bytes = std::max(s.f8_bytes, (size_t)B * (H >> sh) * (W >> sh) * kpad_of(o));
      }
    }
  }
  s.part_off = tensors_end;
  s.cnt_off = align256(s.part_off + s.part_bytes);
  s.f8_off = align256(s.cnt_off + (size_t)s.cnt_n * 4);
  s.chain_off = align256(s.f8_off + s.f8_bytes);
  if (p->dtype == YV7_DT_F16) {
    std::vector<size_t> zero_off(p->tensors.size(), 0);
    yv7::ChainParams c;
    for (size_t i = 0; i < p->ops.size(); ++i)
      if (find_chain(p, i, B, H, W, zero_off, nullptr, &c)) s.chain_bytes = std::max(s.chain_bytes, yv7::chain_counter_bytes(c));
  }
  s.end = align256(s.chain_off + s.chain_bytes);
  return s;
}

}  // namespace

extern "C" {

int32_t yv7_abi_version(void) { return YV7_ABI_VERSION; }

const char* yv7_last_error(void) { return g_err.c_str(); }

int yv7_plan_create(const yv7_net_desc* d, const void* weights, size_t nbytes, int device, yv7_plan** out) {
  if (!d || !out || (!weights && nbytes)) return fail(YV7_E_ARG, "yv7_plan_create: null argument");
  *out = nullptr;
  if (d->abi_version != YV7_ABI_VERSION) return fail(YV7_E_ABI, "yv7_plan_create: abi_version mismatch");
  if (d->dtype != YV7_DT_F32 && d->dtype != YV7_DT_F16) return fail(YV7_E_ARG, "yv7_plan_create: bad dtype");
  if (d->n_tensors <= 0 || d->n_ops <= 0 || !d->tensors || !d->ops)
    return fail(YV7_E_ARG, "yv7_plan_create: empty network");
  if (d->nl <= 0 || d->nl > 8 || d->na <= 0 || d->na > 4 || d->no < 6 || d->no - 5 > 128)
    return fail(YV7_E_ARG, "yv7_plan_create: unsupported head geometry (nl<=8, na<=4, nc<=128)");
  const int vec = d->dtype == YV7_DT_F16 ? 8 : 4;
  for (int i = 0; i < d->n_tensors; ++i)
    if (d->tensors[i].channels <= 0 || d->tensors[i].channels % vec || d->tensors[i].shift < 0 ||
        d->tensors[i].shift > d->max_shift)
      return fail(YV7_E_ARG, "yv7_plan_create: tensor " + std::to_string(i) + " has bad channels/shift");
  for (int i = 0; i < d->n_ops; ++i) {
    const auto& o = d->ops[i];
    const bool src_ok = o.kind == YV7_OP_INPUT || o.kind == YV7_OP_STEM || (o.src >= 0 && o.src < d->n_tensors);
    const bool dst_ok = o.kind == YV7_OP_DETECT || (o.dst >= 0 && o.dst < d->n_tensors);
    if (!src_ok || !dst_ok) return fail(YV7_E_ARG, "yv7_plan_create: op " + std::to_string(i) + " bad tensor id");
    if (o.kind == YV7_OP_CONV || o.kind == YV7_OP_DETECT) {
      if (o.cin % vec || (o.kind == YV7_OP_CONV && o.cout % vec))
        return fail(YV7_E_ARG, "yv7_plan_create: op " + std::to_string(i) + " channels not a multiple of the vector");
      if (o.kind == YV7_OP_CONV && o.pool != 0 &&
          (o.pool != 2 || d->dtype != YV7_DT_F16 || o.k != 1 || o.s != 2 || o.pad != 0 || o.wfmt != YV7_WFMT_PLAN))
        return fail(YV7_E_ARG, "yv7_plan_create: op " + std::to_string(i) +
                                   " bad pooled conv (fp16 plans, pool 2 with k 1, s 2, pad 0)");
      if (o.kind == YV7_OP_CONV && o.wfmt != YV7_WFMT_PLAN) {
        if (o.wfmt != YV7_WFMT_FP8 || d->dtype != YV7_DT_F16 || o.k != 1 || o.s != 1 || o.pad != 0 ||
            o.cout > 1024 || !(o.xscale > 0.0f) || o.xscale > 1e30f || o.s_off < 0 ||
            (size_t)o.s_off + sizeof(float) * o.cout > nbytes)
          return fail(YV7_E_ARG, "yv7_plan_create: op " + std::to_string(i) +
                                     " bad fp8 conv (fp16 plans, 1x1 stride 1, cout <= 1024, xscale > 0, scales in blob)");
      }
      const size_t wb = (size_t)((o.cout + 31) / 32 * 32) * kpad_of(o) * (is_f8(o) ? 1 : elem_size(d->dtype));
      if (o.w_off < 0 || o.b_off < 0 || (size_t)o.w_off + wb > nbytes ||
          (size_t)o.b_off + sizeof(float) * o.cout > nbytes)
        return fail(YV7_E_ARG, "yv7_plan_create: op " + std::to_string(i) + " weight range outside blob");
      if (o.k < 1 || o.s < 1 || o.pad < 0 || o.pad > YV7_BORDER || o.k - 1 - o.pad > YV7_BORDER)
        return fail(YV7_E_ARG, "yv7_plan_create: op " + std::to_string(i) +
                                   " window reaches past the tensors' zero frame (needs pad <= 1, k - 1 - pad <= 1)");
      if (o.kind == YV7_OP_DETECT && (o.level < 0 || o.level >= d->nl || o.cout != d->na * d->no || o.k != 1))
        return fail(YV7_E_ARG, "yv7_plan_create: bad detect op");
    }
    if (o.kind == YV7_OP_STEM) {
      if (d->dtype != YV7_DT_F16 || !yv7::stem_supported(o.cin, o.cout, o.cout2, o.s) || o.k != 3 || o.act != o.act2 ||
          o.dst_coff % vec || o.dst_coff + o.cout2 > d->tensors[o.dst].channels)
        return fail(YV7_E_ARG, "yv7_plan_create: unsupported stem op");
      // cin 12: the w6 front end (ReOrg fused), conv A's K = tap * 16 + ci
      const int ka = o.cin == 12 ? 9 * 16 : 27;
      const size_t wa = (size_t)o.cout * ((ka + 63) / 64 * 64) * 2, wb = (size_t)o.cout2 * ((9 * o.cout + 63) / 64 * 64) * 2;
      if (o.w_off < 0 || o.w2_off < 0 || (size_t)o.w_off + wa > nbytes || (size_t)o.w2_off + wb > nbytes ||
          (size_t)o.b_off + 4 * o.cout > nbytes || (size_t)o.b2_off + 4 * o.cout2 > nbytes)
        return fail(YV7_E_ARG, "yv7_plan_create: stem weight range outside blob");
      continue;
    }
    if (o.kind != YV7_OP_INPUT && o.kind != YV7_OP_DETECT) {
      const int src_c = d->tensors[o.src].channels, dst_c = d->tensors[o.dst].channels;
      const int cin = o.kind == YV7_OP_CONV ? o.cin : o.cout;
      if (o.src_coff < 0 || o.src_coff + cin > src_c || o.dst_coff < 0 || o.dst_coff + o.cout > dst_c ||
          o.src_coff % vec || o.dst_coff % vec)
        return fail(YV7_E_ARG, "yv7_plan_create: op " + std::to_string(i) + " channel slice out of range");
    }
  }
  hipError_t e = hipSetDevice(device);
  if (e != hipSuccess) return hip_fail(e, "hipSetDevice");
  hipDeviceProp_t prop;
  if ((e = hipGetDeviceProperties(&prop, device)) != hipSuccess) return hip_fail(e, "hipGetDeviceProperties");
  if (std::strncmp(prop.gcnArchName, "gfx950", 6) != 0)
    return fail(YV7_E_DEVICE, std::string("libyv7 is built for gfx950; device is ") + prop.gcnArchName);

  yv7_plan* p = new yv7_plan();
  p->device = device;
  p->dtype = d->dtype;
  p->tensors.assign(d->tensors, d->tensors + d->n_tensors);
  p->ops.assign(d->ops, d->ops + d->n_ops);
  p->op_variant.assign(p->ops.size(), 0);
  p->nl = d->nl;
  p->na = d->na;
  p->no = d->no;
  p->max_shift = d->max_shift;
  p->stride.assign(d->stride, d->stride + d->nl);
  p->anchor_grid.assign(d->anchor_grid, d->anchor_grid + d->nl * d->na * 2);
  p->wbytes = nbytes;
  if (nbytes) {
    if ((e = hipMalloc(&p->weights, nbytes)) != hipSuccess) {
      delete p;
      return hip_fail(e, "hipMalloc(weights)");
    }
    if ((e = hipMemcpy(p->weights, weights, nbytes, hipMemcpyDefault)) != hipSuccess) {
      (void)hipFree(p->weights);
      delete p;
      return hip_fail(e, "hipMemcpy(weights)");
    }
  }
  if ((e = hipMalloc(&p->zero, 4096)) != hipSuccess || (e = hipMemset(p->zero, 0, 4096)) != hipSuccess) {
    if (p->weights) (void)hipFree(p->weights);
    delete p;
    return hip_fail(e, "hipMalloc(zero page)");
  }
  // fragment-packed copies of the 3x3 stride-1 weights (conv_lr.hip), packed on the device from the
  // plan's own copy
  p->wf_off.assign(p->ops.size(), -1);
  size_t wf_total = 0;
  for (size_t i = 0; i < p->ops.size(); ++i)
    if (wants_frag(p->dtype, p->ops[i])) {
      p->wf_off[i] = (int64_t)wf_total;
      wf_total = align256(wf_total + yv7::frag_bytes(p->ops[i].cin, p->ops[i].cout, p->ops[i].k * p->ops[i].k));
    }
  if (wf_total) {
    // packed on a private stream and waited for on that stream only (a device-wide sync here
    // made plan creation wait for other plans' forwards on their own streams).  A blocking stream: its
    // work is ordered after the null stream's weight copy above.
    hipStream_t ps = nullptr;
    e = hipMalloc(&p->wfrag, wf_total);
    if (e == hipSuccess) e = hipStreamCreate(&ps);
    for (size_t i = 0; e == hipSuccess && i < p->ops.size(); ++i)
      if (p->wf_off[i] >= 0)
        e = yv7::pack_frag(reinterpret_cast<const unsigned char*>(p->weights) + p->ops[i].w_off, kpad_of(p->ops[i]),
                           p->ops[i].cin, p->ops[i].cout, p->ops[i].k * p->ops[i].k,
                           reinterpret_cast<unsigned char*>(p->wfrag) + p->wf_off[i], ps);
    if (e == hipSuccess) e = hipStreamSynchronize(ps);
    if (ps) (void)hipStreamDestroy(ps);
    if (e != hipSuccess) {
      yv7_plan_destroy(p);
      return hip_fail(e, "yv7_plan_create: fragment packing");
    }
  }
  *out = p;
  return 0;
}

static void free_events(yv7_plan* p) {
  for (auto e : p->events) (void)hipEventDestroy(e);
  p->events.clear();
  p->prof_max = p->prof_used = 0;
}

int yv7_profile_enable(yv7_plan* p, int max_forwards) {
  if (!p || max_forwards < 0) return fail(YV7_E_ARG, "yv7_profile_enable");
  free_events(p);
  if (max_forwards == 0) return 0;
  const size_t n = (size_t)max_forwards * 2 * p->ops.size();
  p->events.resize(n);
  for (size_t i = 0; i < n; ++i) {
    hipError_t e = hipEventCreate(&p->events[i]);
    if (e != hipSuccess) {
      p->events.resize(i);
      free_events(p);
      return hip_fail(e, "hipEventCreate");
    }
  }
  p->prof_max = max_forwards;
  return 0;
}

int yv7_profile_read(yv7_plan* p, int* n_forwards, float* op_ms) {
  if (!p || !n_forwards || !op_ms) return fail(YV7_E_ARG, "yv7_profile_read");
  const size_t nops = p->ops.size();
  for (size_t i = 0; i < nops; ++i) op_ms[i] = 0.f;
  *n_forwards = p->prof_used;
  for (int f = 0; f < p->prof_used; ++f) {
    hipEvent_t* ev = &p->events[(size_t)f * 2 * nops];
    hipError_t e = hipEventSynchronize(ev[2 * nops - 1]);
    if (e != hipSuccess) return hip_fail(e, "hipEventSynchronize");
    for (size_t i = 0; i < nops; ++i) {
      float ms = 0.f;
      if ((e = hipEventElapsedTime(&ms, ev[2 * i], ev[2 * i + 1])) != hipSuccess) return hip_fail(e, "hipEventElapsedTime");
      op_ms[i] += ms;
    }
  }
  return 0;
}

void yv7_plan_destroy(yv7_plan* p) {
  if (!p) return;
  free_events(p);
  if (p->weights) (void)hipFree(p->weights);
  if (p->zero) (void)hipFree(p->zero);
  if (p->wfrag) (void)hipFree(p->wfrag);
  delete p;
}

size_t yv7_workspace_bytes(const yv7_plan* p, int B, int H, int W) {
  if (!p || check_hw(p, B, H, W)) return 0;
  size_t total = 0;
  tensor_offsets(p, B, H, W, &total);
  return split_scratch(p, B, H, W, total).end;
}

int yv7_workspace_forget(yv7_plan* p, const void* ws, size_t bytes) {
  if (!p || !ws) return fail(YV7_E_ARG, "yv7_workspace_forget: null argument");
  const char* lo = reinterpret_cast<const char*>(ws);
  const size_t n = bytes ? bytes : 1;
  std::vector<yv7_plan::WsKey> keep;
  for (const auto& w : p->ws_ready) {
    const char* wl = reinterpret_cast<const char*>(w.ptr);
    if (wl + w.bytes <= lo || lo + n <= wl) keep.push_back(w);
  }
  p->ws_ready = keep;
  return 0;
}

// Kernel variants a caller may force per op: every real kernel configuration of the fp16 dispatch
// (conv_f16.hip launch_conv_f16 / choose), never the microbenchmark hooks (90-99, 298; ws64's 12-14
// and 16), which skip work on purpose.
static bool variant_allowed(const yv7_op_desc& o, int v) {
  if (v == 0) return true;
  const int kind = o.kind;
  if (is_f8(o)) return v == 81 || v == 82;   // fp8 1x1: staged quantize pass / fused quantization
  if (kind == YV7_OP_DETECT) return v == 92 || v == 94 || v == 97 || v == 99;
  if (v == 1 || v == 2 || (v >= 4 && v <= 8) || v == 10 || v == 11 || v == 15 || v == 17) return true;
  if (v >= 100 && v < 160 && v % 10 <= 4) return true;   // ring configuration (v - 100) / 10, v % 10 K-splits
  if (v == 305) return o.k == 3 && o.s == 1;   // the chained launch of the 3x3 stack starting here (find_chain)
  return (v >= 201 && v <= 206) || v == 231 || v == 232 || (v >= 234 && v <= 236) || v == 239 || v == 262 ||
         (v >= 270 && v <= 288) || (v >= 290 && v <= 295) || v == 302 || v == 303;
}

int yv7_set_op_variant(yv7_plan* p, int op, int variant) {
  if (!p || op < 0 || op >= (int)p->ops.size()) return fail(YV7_E_ARG, "yv7_set_op_variant: bad op index");
  const auto& o = p->ops[op];
  if (o.kind != YV7_OP_CONV && o.kind != YV7_OP_DETECT)
    return fail(YV7_E_ARG, "yv7_set_op_variant: op " + std::to_string(op) + " is not a CONV / DETECT op");
  if (!variant_allowed(o, variant))
    return fail(YV7_E_ARG, "yv7_set_op_variant: variant " + std::to_string(variant) + " is not a kernel configuration");
  p->op_variant[op] = variant;
  return 0;
}

int64_t yv7_num_rows(const yv7_plan* p, int H, int W) {
  if (!p) return -1;
  int64_t n = 0;
  for (const auto& o : p->ops)
    if (o.kind == YV7_OP_DETECT) {
      const int s = p->tensors[o.src].shift;
      n += (int64_t)p->na * (H >> s) * (W >> s);
    }
  return n;
}

int yv7_tensor_info(const yv7_plan* p, int id, int B, int H, int W, int64_t* offset, int64_t* dims4) {
  if (!p || id < 0 || id >= (int)p->tensors.size() || !offset || !dims4) return fail(YV7_E_ARG, "yv7_tensor_info");
  if (int rc = check_hw(p, B, H, W)) return rc;
  size_t total = 0;
  auto off = tensor_offsets(p, B, H, W, &total);
  *offset = (int64_t)off[id];
  const auto& t = p->tensors[id];
  dims4[0] = B;
  dims4[1] = (H >> t.shift) + 2 * YV7_BORDER;
  dims4[2] = (W >> t.shift) + 2 * YV7_BORDER;
  dims4[3] = t.channels;
  return 0;
}

// The forward's op loop.  dry: launch nothing (yv7_kernels.h LaunchRec), record per op the host stubs
// of the kernels the dispatch picks into *kernels (yv7_op_kernels); no workspace clearing, no events.
static int forward_impl(yv7_plan* p, const void* x, int x_dtype, int B, int H, int W, float* z, float* raw,
                        yv7_row_best* rowbest, void* ws, size_t ws_bytes, void* stream,
                        std::vector<std::vector<const void*>>* kernels) {
  const bool dry = kernels != nullptr;
  if (!p || !x || !z || !ws) return fail(YV7_E_ARG, "yv7_forward: null argument");
  if (x_dtype != YV7_DT_F32 && x_dtype != YV7_DT_F16) return fail(YV7_E_ARG, "yv7_forward: bad x_dtype");
  if (int rc = check_hw(p, B, H, W)) return rc;
  size_t total = 0;
  const auto off = tensor_offsets(p, B, H, W, &total);
  const SplitScratch scr = split_scratch(p, B, H, W, total);
  total = scr.end;
  if (!dry && ws_bytes < total) return fail(YV7_E_WORKSPACE, "yv7_forward: workspace too small (need " +
                                                                 std::to_string(total) + " bytes)");
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  unsigned char* wsb = reinterpret_cast<unsigned char*>(ws);
  const unsigned char* wb = reinterpret_cast<const unsigned char*>(p->weights);
  hipError_t e = hipSuccess;
  // Kernels write only tensor interiors, so the zero frames survive from one forward to the next:
  // a workspace is cleared the first time it is seen with this layout (pointer, size AND the batch
  // geometry: (B, H, W) and (B, W, H) have equal sizes but different frames) and never again, until
  // the caller hands the memory back with yv7_workspace_forget (include/yv7.h).
  if (!dry) {
    bool ready = false;
    for (const auto& w : p->ws_ready)
      if (w.ptr == ws && w.bytes == total && w.B == B && w.H == H && w.W == W) ready = true;
    if (!ready) {
      if ((e = hipMemsetAsync(ws, 0, total, st)) != hipSuccess) return hip_fail(e, "hipMemsetAsync(workspace)");
      // a workspace overlapping this one (another layout of the same memory) is no longer intact
      const char* lo = reinterpret_cast<const char*>(ws);
      std::vector<yv7_plan::WsKey> keep;
      for (const auto& w : p->ws_ready) {
        const char* wl = reinterpret_cast<const char*>(w.ptr);
        if (wl + w.bytes <= lo || lo + total <= wl) keep.push_back(w);
      }
      keep.push_back({ws, total, B, H, W});
      if (keep.size() > 8) keep.erase(keep.begin());
      p->ws_ready = keep;
    }
  }
  const int nrows = (int)yv7_num_rows(p, H, W);
  // raw-logit and z row offsets of each level
  std::vector<int> row_off(p->nl, 0);
  std::vector<size_t> raw_off(p->nl, 0);
  {
    std::vector<int> lvl_rows(p->nl, 0);
    for (const auto& o : p->ops)
      if (o.kind == YV7_OP_DETECT) {
        const int s = p->tensors[o.src].shift;
        lvl_rows[o.level] = p->na * (H >> s) * (W >> s);
      }
    int acc = 0;
    size_t racc = 0;
    for (int l = 0; l < p->nl; ++l) {
      row_off[l] = acc;
      raw_off[l] = racc;
      acc += lvl_rows[l];
      racc += (size_t)B * lvl_rows[l] * p->no;
    }
  }
  // fp16 plans score the rows in the head's epilogue; other paths derive the records from z after the
  // last op
  const bool rowbest_fused = rowbest && yv7::det_writes_rowbest(p->dtype);
  hipEvent_t* ev = nullptr;
  // the forward's event slot is claimed only once every op has launched (below): a forward that fails
  // part-way leaves the slot to the next one instead of a pair that was never recorded
  if (!dry && p->prof_used < p->prof_max) ev = &p->events[(size_t)p->prof_used * 2 * p->ops.size()];
  // the op's (start, stop) pair rides on its kernel launches (yv7_kernels.h YV7_LAUNCH); cleared on
  // every way out of this function
  struct EventScope {
    ~EventScope() {
      yv7::op_events() = yv7::OpEvents{};
      yv7::launch_rec() = yv7::LaunchRec{};
    }
  } event_scope;
  if (dry) kernels->assign(p->ops.size(), {});
  size_t fused_until = 0;   // ops [.., fused_until) were launched as part of a fused group
  for (size_t i = 0; i < p->ops.size(); ++i) {
    const auto& o = p->ops[i];
    if (ev) yv7::op_events() = yv7::OpEvents{ev[2 * i], ev[2 * i + 1], 0};
    if (dry) {
      yv7::launch_rec() = yv7::LaunchRec{};
      yv7::launch_rec().dry = true;
    }
    switch (o.kind) {
      case YV7_OP_INPUT: {
        const auto& t = p->tensors[o.dst];
        e = yv7::launch_input(p->dtype, x, x_dtype, wsb + off[o.dst], B, H, W, t.channels, o.k == 2, st);
        break;
      }
      case YV7_OP_CONV:
      case YV7_OP_DETECT: {
        if (fused_until > i) break;   // the second op of a dual 1x1 launch (below)
        yv7::ConvParams c = conv_params(p, i, B, H, W);
        c.x = wsb + off[o.src];
        c.w = wb + o.w_off;
        c.bias = reinterpret_cast<const float*>(wb + o.b_off);
        c.zero = p->zero;
        c.part = reinterpret_cast<float*>(wsb + scr.part_off);
        c.part_bytes = scr.part_bytes;
        c.cnt = reinterpret_cast<int*>(wsb + scr.cnt_off);
        c.cnt_n = scr.cnt_n;
        if (o.kind == YV7_OP_CONV) {
          const auto& to = p->tensors[o.dst];
          if (c.Ho != (H >> to.shift) || c.Wo != (W >> to.shift))
            return fail(YV7_E_SHAPE, "yv7_forward: op " + std::to_string(i) + " output shape mismatch");
          c.y = wsb + off[o.dst];
          c.yc = to.channels;
          c.yoff = o.dst_coff;
          if (is_f8(o)) {
            // 82: the fp8 GEMM quantizes the fp16 input slice on its way into LDS (no staging pass, but
            // every N tile of a row block converts it again: VALU work ~2x the block's MFMA time per
            // K step); 81: a separate quantize pass into the dense e4m3 staging buffer, then the GEMM
            // reads e4m3 by LDS-DMA.  Default (measured per layer on MI355X, bs32 640, profiles/
            // r2_fp8_ab_*.txt): fused up to 2 N tiles (cout <= 256), staged beyond.
            yv7::F8ConvParams f;
            std::memset(&f, 0, sizeof(f));
            const int v = p->op_variant[i];
            if (v == 81 || (v == 0 && o.cout > 256)) {
              unsigned char* x8 = wsb + scr.f8_off;
              e = yv7::launch_quant_f8(c.x, B, c.H, c.W, c.xc, c.xoff, o.cin, c.kpad, 1.0f / o.xscale, x8, st);
              if (e != hipSuccess) return hip_fail(e, "yv7_forward fp8 quantize");
              f.x8 = x8;
            } else {
              const size_t xb = yv7::bordered_pixels(B, c.H, c.W) * c.xc * 2;
              if (xb >= ((size_t)1 << 31))
                return fail(YV7_E_SHAPE, "yv7_forward: fp8 op " + std::to_string(i) + " input exceeds 2 GiB");
              f.x16 = c.x;
              f.xbytes = (uint32_t)xb;
              f.xc = c.xc;
              f.xoff = c.xoff;
              f.cin = o.cin;
              f.qscale = 1.0f / o.xscale;
            }
            f.y = c.y;
            f.w8 = c.w;
            f.bias = c.bias;
            f.wscale = reinterpret_cast<const float*>(wb + o.s_off);
            f.xscale = o.xscale;
            f.wbytes = (uint32_t)((size_t)((o.cout + 31) / 32 * 32) * c.kpad);
            f.M = c.M;
            f.kp = c.kpad;
            f.cout = o.cout;
            f.H = c.Ho;
            f.W = c.Wo;
            f.yc = c.yc;
            f.yoff = c.yoff;
            f.act = o.act;
            e = yv7::launch_conv_f8(f, st);
            break;
          }
          // An ELAN block's 3x3 stack as ONE chained launch (find_chain, conv_lr.hip conv3x3_chain_kernel);
          // the later ops of the chain record no time of their own.
          {
            yv7::ChainParams ch;
            const int n = find_chain(p, i, B, H, W, off, wsb, &ch);
            if (n) {
              ch.ctr = reinterpret_cast<int*>(wsb + scr.chain_off);
              e = yv7::launch_conv_chain(ch, st);
              fused_until = i + n;
              break;
            }
          }
          // The MP block's two readers of one tensor (cfg/deploy/yolov7.yaml: `MP -> 1x1` and `1x1`,
          // adjacent ops here: the pooled one is the fp16 plan's pool = 2 op) as ONE register-streamed
          // launch that reads the tensor once (conv_rs.hip); the second op records no time of its own.
          // Both ops on the default dispatch only; YV7_DUAL=0: off.
          static const int dual = [] { const char* ev = getenv("YV7_DUAL"); return ev ? atoi(ev) : 1; }();
          if (dual && p->dtype == YV7_DT_F16 && i + 1 < p->ops.size() && p->op_variant[i] == 0 &&
              p->op_variant[i + 1] == 0) {
            const auto& o1 = p->ops[i + 1];
            // one launch reads the shared slice while it writes both outputs: neither output may overlap
            // the input slice or the other output (in order, op i + 1 would see op i's writes) — the
            // hazards graph.py's _merge_siblings checks before its fusions
            auto overlap = [](int ta, int ca, int na, int tb, int cb, int nb) { return ta == tb && ca < cb + nb && cb < ca + na; };
            const bool pair = o1.kind == YV7_OP_CONV && !is_f8(o1) && o1.src == o.src && o1.src_coff == o.src_coff &&
                              o1.cin == o.cin && o1.k == 1 && o.k == 1 && ((o.pool == 2) != (o1.pool == 2)) &&
                              o1.w_off != o.w_off && !overlap(o.dst, o.dst_coff, o.cout, o.src, o.src_coff, o.cin) &&
                              !overlap(o1.dst, o1.dst_coff, o1.cout, o.src, o.src_coff, o.cin) &&
                              !overlap(o.dst, o.dst_coff, o.cout, o1.dst, o1.dst_coff, o1.cout);
            if (pair) {
              const size_t fi = o.pool == 2 ? i + 1 : i, pi = o.pool == 2 ? i : i + 1;
              const auto& of = p->ops[fi];
              const auto& op_ = p->ops[pi];
              yv7::ConvParams cf = conv_params(p, fi, B, H, W);
              cf.x = c.x;
              cf.w = wb + of.w_off;
              cf.bias = reinterpret_cast<const float*>(wb + of.b_off);
              cf.zero = p->zero;
              const auto& tf = p->tensors[of.dst];
              const auto& tp = p->tensors[op_.dst];
              cf.y = wsb + off[of.dst];
              cf.yc = tf.channels;
              cf.yoff = of.dst_coff;
              yv7::Conv1x1Pooled q;
              q.w = wb + op_.w_off;
              q.bias = reinterpret_cast<const float*>(wb + op_.b_off);
              q.y = wsb + off[op_.dst];
              q.yc = tp.channels;
              q.yoff = op_.dst_coff;
              q.cout = op_.cout;
              q.act = op_.act;
              if (cf.Ho == (H >> tf.shift) && cf.Wo == (W >> tf.shift) && tp.shift == tf.shift + 1 &&
                  yv7::conv1x1_rs_supported(cf, &q)) {
                e = yv7::launch_conv1x1_rs(cf, &q, st);
                fused_until = i + 2;
                break;
              }
            }
          }
          e = yv7::launch_conv(p->dtype, c, false, st);
        } else {
          c.z = z;
          c.raw = raw ? raw + raw_off[o.level] : nullptr;
          c.nrows = nrows;
          c.row_off = row_off[o.level];
          c.na = p->na;
          c.no = p->no;
          c.stride = p->stride[o.level];
          for (int a = 0; a < p->na * 2; ++a) c.anchor[a] = p->anchor_grid[o.level * p->na * 2 + a];
          c.best = rowbest_fused ? reinterpret_cast<float*>(rowbest) : nullptr;
          e = yv7::launch_conv(p->dtype, c, true, st);
        }
        break;
      }
      case YV7_OP_STEM: {
        const auto& to = p->tensors[o.dst];
        const int reorg = o.cin == 12;   // conv A runs on the 2x space-to-depth image
        if ((H >> to.shift) != H / (reorg + 1) / o.s / 2 || (W >> to.shift) != W / (reorg + 1) / o.s / 2 ||
            (reorg && (H % 4 || W % 4)))
          return fail(YV7_E_SHAPE, "yv7_forward: stem output shape mismatch");
        yv7::StemParams sp;
        sp.variant = 0;
        sp.x = x;
        sp.y = wsb + off[o.dst];
        sp.wa = wb + o.w_off;
        sp.ba = reinterpret_cast<const float*>(wb + o.b_off);
        sp.wb = wb + o.w2_off;
        sp.bb = reinterpret_cast<const float*>(wb + o.b2_off);
        sp.B = B;
        sp.H = H;
        sp.W = W;
        sp.yc = to.channels;
        sp.yoff = o.dst_coff;
        sp.reorg = reorg;
        sp.kpad_a = ((reorg ? 9 * 16 : 27) + 63) / 64 * 64;
        sp.kpad_b = (9 * o.cout + 63) / 64 * 64;
        sp.act_a = o.act;
        sp.act_b = o.act2;
        sp.sa = o.s;
        e = yv7::launch_stem(sp, x_dtype, st);
        break;
      }
      case YV7_OP_MAXPOOL: {
        const auto& ti = p->tensors[o.src];
        const auto& to = p->tensors[o.dst];
        // SPPCSPC's cascade (graph.py: pool5 three times, each reading the previous slice of one
        // concat tensor): one fused launch; the two later ops record no time of their own
        if (i + 2 < p->ops.size() && !(fused_until > i)) {
          const auto& o1 = p->ops[i + 1];
          const auto& o2 = p->ops[i + 2];
          auto pool5 = [](const yv7_op_desc& q) { return q.kind == YV7_OP_MAXPOOL && q.k == 5 && q.s == 1 && q.pad == 2; };
          const int Hi = H >> ti.shift, Wi = W >> ti.shift;
          if (pool5(o) && pool5(o1) && pool5(o2) && o.src == o.dst && o1.src == o.dst && o1.dst == o.dst &&
              o2.src == o.dst && o2.dst == o.dst && o.dst_coff == o.src_coff + o.cout &&
              o1.src_coff == o.dst_coff && o1.dst_coff == o1.src_coff + o.cout && o2.src_coff == o1.dst_coff &&
              o2.dst_coff == o2.src_coff + o.cout && o1.cout == o.cout && o2.cout == o.cout &&
              yv7::spp_cascade_supported(p->dtype, Hi, Wi, o.cout)) {
            e = yv7::launch_spp_cascade(p->dtype, wsb + off[o.src], B, Hi, Wi, ti.channels, o.src_coff, o.cout, st);
            fused_until = i + 3;
            break;
          }
        }
        if (fused_until > i) break;   // a later op of an already-launched cascade
        const int Hi = H >> ti.shift, Wi = W >> ti.shift;
        const int Ho = (Hi + 2 * o.pad - o.k) / o.s + 1, Wo = (Wi + 2 * o.pad - o.k) / o.s + 1;
        if (Ho != (H >> to.shift) || Wo != (W >> to.shift))
          return fail(YV7_E_SHAPE, "yv7_forward: maxpool op " + std::to_string(i) + " shape mismatch");
        e = yv7::launch_maxpool(p->dtype, wsb + off[o.src], B, Hi, Wi, ti.channels, o.src_coff, wsb + off[o.dst], Ho,
                                Wo, to.channels, o.dst_coff, o.cout, o.k, o.s, o.pad, st);
        break;
      }
      case YV7_OP_UPSAMPLE: {
        const auto& ti = p->tensors[o.src];
        const auto& to = p->tensors[o.dst];
        if (to.shift + 1 != ti.shift) return fail(YV7_E_SHAPE, "yv7_forward: upsample shift mismatch");
        e = yv7::launch_upsample2x(p->dtype, wsb + off[o.src], B, H >> ti.shift, W >> ti.shift, ti.channels,
                                   o.src_coff, wsb + off[o.dst], to.channels, o.dst_coff, o.cout, st);
        break;
      }
      case YV7_OP_COPY: {
        const auto& ti = p->tensors[o.src];
        const auto& to = p->tensors[o.dst];
        if (to.shift != ti.shift) return fail(YV7_E_SHAPE, "yv7_forward: copy shift mismatch");
        e = yv7::launch_copy(p->dtype, wsb + off[o.src], B, H >> ti.shift, W >> ti.shift, ti.channels, o.src_coff,
                             wsb + off[o.dst], to.channels, o.dst_coff, o.cout, st);
        break;
      }
      default:
        return fail(YV7_E_ARG, "yv7_forward: unknown op kind");
    }
    if (e != hipSuccess) return hip_fail(e, "yv7_forward launch");
    if (dry) {
      const auto& r = yv7::launch_rec();
      if (r.n > 4) return fail(YV7_E_ARG, "yv7_op_kernels: op " + std::to_string(i) + " launches more than 4 kernels");
      for (int k = 0; k < r.n; ++k) (*kernels)[i].push_back(r.fn[k]);
    }
    if (ev && yv7::op_events().launches == 0) {   // no kernel of its own (a later op of a fused cascade)
      if ((e = hipEventRecord(ev[2 * i], st)) != hipSuccess || (e = hipEventRecord(ev[2 * i + 1], st)) != hipSuccess)
        return hip_fail(e, "hipEventRecord");
    }
  }
  yv7::op_events() = yv7::OpEvents{};
  if (dry) return 0;
  if (ev) p->prof_used++;
  if (rowbest && !rowbest_fused &&
      (e = yv7::launch_row_best(z, B, nrows, p->no, rowbest, st)) != hipSuccess)
    return hip_fail(e, "yv7_forward row scores");
  return 0;
}

int yv7_forward(yv7_plan* p, const void* x, int x_dtype, int B, int H, int W, float* z, float* raw,
                yv7_row_best* rowbest, void* ws, size_t ws_bytes, void* stream) {
  return forward_impl(p, x, x_dtype, B, H, W, z, raw, rowbest, ws, ws_bytes, stream, nullptr);
}

int yv7_op_kernels(yv7_plan* p, int B, int H, int W, int x_dtype, char* buf, size_t bytes) {
  if (!p || !buf || bytes == 0) return fail(YV7_E_ARG, "yv7_op_kernels: null argument");
  std::vector<std::vector<const void*>> ks;
  // dry run: the op loop with placeholder pointers (nothing is launched or dereferenced on the host)
  static const float dummy[4] = {0, 0, 0, 0};
  void* ph = const_cast<float*>(dummy);
  if (int rc = forward_impl(p, ph, x_dtype, B, H, W, static_cast<float*>(ph), nullptr, nullptr, ph, 0, nullptr, &ks))
    return rc;
  std::string out;
  for (size_t i = 0; i < ks.size(); ++i) {
    out += std::to_string(i);
    for (size_t k = 0; k < ks[i].size(); ++k) {
      const char* mangled = hipKernelNameRefByPtr(ks[i][k], nullptr);
      std::string name = mangled ? mangled : "?";
      int st = 0;
      char* dem = mangled ? abi::__cxa_demangle(mangled, nullptr, nullptr, &st) : nullptr;
      if (dem && st == 0) name = dem;
      std::free(dem);
      out += (k ? "|" : "\t") + name;
    }
    out += "\n";
  }
  if (out.size() + 1 > bytes) return fail(YV7_E_ARG, "yv7_op_kernels: buffer too small (need " + std::to_string(out.size() + 1) + ")");
  std::memcpy(buf, out.c_str(), out.size() + 1);
  return 0;
}

int yv7_f8_scratch_info(const yv7_plan* p, int B, int H, int W, int64_t* offset, int64_t* bytes) {
  if (!p || !offset || !bytes) return fail(YV7_E_ARG, "yv7_f8_scratch_info");
  if (int rc = check_hw(p, B, H, W)) return rc;
  size_t total = 0;
  tensor_offsets(p, B, H, W, &total);
  const SplitScratch s = split_scratch(p, B, H, W, total);
  *offset = (int64_t)s.f8_off;
  *bytes = (int64_t)s.f8_bytes;
  return 0;
}

size_t yv7_nms_workspace_bytes(int B, int N, int no, int multi_label, int max_nms) {
  if (B <= 0 || N <= 0 || no < 6 || max_nms <= 0) return 0;
  return yv7::nms_workspace_bytes(B, N, no, multi_label, max_nms);
}

static int nms_check(const float* z, int B, int N, int no, int max_det, int max_nms, void* ws, size_t ws_bytes,
                     int multi) {
  if (!z || !ws) return fail(YV7_E_ARG, "yv7_nms: null argument");
  if (B <= 0 || N <= 0 || no < 6 || no - 5 > 128) return fail(YV7_E_SHAPE, "yv7_nms: bad z shape (nc <= 128)");
  if (max_det <= 0 || max_nms <= 0 || max_nms > 65536) return fail(YV7_E_ARG, "yv7_nms: max_det/max_nms out of range");
  if (ws_bytes < yv7::nms_workspace_bytes(B, N, no, multi, max_nms)) return fail(YV7_E_WORKSPACE, "yv7_nms: workspace too small");
  return 0;
}

int yv7_nms(const float* z, const yv7_row_best* rowbest, int B, int N, int no, float conf_thres, float iou_thres,
            int multi_label, int agnostic, const int32_t* classes, int ncls, int max_det, int max_nms, float* det,
            int64_t* src_row, int32_t* count, void* ws, size_t ws_bytes, void* stream) {
  if (int rc = nms_check(z, B, N, no, max_det, max_nms, ws, ws_bytes, multi_label)) return rc;
  if (!det || !src_row || !count || (ncls > 0 && !classes)) return fail(YV7_E_ARG, "yv7_nms: null output");
  hipError_t e = yv7::launch_nms(z, rowbest, B, N, no, conf_thres, iou_thres, multi_label, agnostic, 0,
                                 ncls > 0 ? classes : nullptr, ncls, max_det, max_nms, det, src_row, count, ws,
                                 reinterpret_cast<hipStream_t>(stream));
  if (e != hipSuccess) return hip_fail(e, "yv7_nms");
  return 0;
}

static const int E2E_MAX_NMS = 65536;

static size_t e2e_layout(int B, int N, int no, int topk, size_t* det_off, size_t* src_off, size_t* cnt_off) {
  const size_t need = yv7::nms_workspace_bytes(B, N, no, 1, E2E_MAX_NMS);
  *det_off = align256(need);
  *src_off = align256(*det_off + sizeof(float) * 6 * (size_t)B * topk);
  *cnt_off = align256(*src_off + sizeof(int64_t) * (size_t)B * topk);
  return align256(*cnt_off + sizeof(int32_t) * (size_t)B);
}

size_t yv7_end2end_workspace_bytes(int B, int N, int no, int topk) {
  if (B <= 0 || N <= 0 || no < 6 || topk <= 0) return 0;
  size_t a, b, c;
  return e2e_layout(B, N, no, topk, &a, &b, &c);
}

int yv7_end2end(const float* z, int B, int N, int no, float conf_thres, float iou_thres, int topk, int32_t* num_dets,
                float* det_boxes, float* det_scores, int32_t* det_classes, void* ws, size_t ws_bytes, void* stream) {
  // multi-label candidates, class-aware IoU on raw boxes (EfficientNMS), top-k by score
  const int max_nms = E2E_MAX_NMS;
  if (topk <= 0) return fail(YV7_E_ARG, "yv7_end2end: topk must be positive");
  if (B <= 0 || N <= 0 || no < 6 || no - 5 > 128) return fail(YV7_E_SHAPE, "yv7_end2end: bad z shape");
  size_t det_off, src_off, cnt_off;
  const size_t total = e2e_layout(B, N, no, topk, &det_off, &src_off, &cnt_off);
  if (!z || !ws || !num_dets || !det_boxes || !det_scores || !det_classes) return fail(YV7_E_ARG, "yv7_end2end: null");
  if (ws_bytes < total) return fail(YV7_E_WORKSPACE, "yv7_end2end: workspace too small (need " + std::to_string(total) + ")");
  unsigned char* w = reinterpret_cast<unsigned char*>(ws);
  float* det = reinterpret_cast<float*>(w + det_off);
  int64_t* src = reinterpret_cast<int64_t*>(w + src_off);
  int32_t* cnt = reinterpret_cast<int32_t*>(w + cnt_off);
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  hipError_t e = yv7::launch_nms(z, nullptr, B, N, no, conf_thres, iou_thres, 1, 0, 1, nullptr, 0, topk, max_nms,
                                 det, src, cnt, ws, st);
  if (e != hipSuccess) return hip_fail(e, "yv7_end2end nms");
  e = yv7::launch_end2end_pack(det, cnt, B, topk, topk, num_dets, det_boxes, det_scores, det_classes, st);
  if (e != hipSuccess) return hip_fail(e, "yv7_end2end pack");
  return 0;
}

size_t yv7_letterbox_workspace_bytes(int new_h, int new_w) {
  if (new_h <= 0 || new_w <= 0) return 0;
  return yv7::letterbox_workspace_bytes(new_h, new_w);
}

int yv7_letterbox(const void* src, int B, int H, int W, int new_h, int new_w, int top, int left, int out_h,
                  int out_w, int pad_b, int pad_g, int pad_r, int out_kind, void* dst, void* workspace,
                  size_t ws_bytes, void* stream) {
  if (!src || !dst || !workspace) return fail(YV7_E_ARG, "yv7_letterbox: null argument");
  if (out_kind < 0 || out_kind > 2) return fail(YV7_E_ARG, "yv7_letterbox: out_kind must be 0, 1 or 2");
  if (B <= 0 || H <= 0 || W <= 0 || new_h <= 0 || new_w <= 0 || top < 0 || left < 0 || top + new_h > out_h ||
      left + new_w > out_w)
    return fail(YV7_E_SHAPE, "yv7_letterbox: the resized image must lie inside the output canvas");
  if ((size_t)B * H * W * 3 >= ((size_t)1 << 40)) return fail(YV7_E_SHAPE, "yv7_letterbox: input too large");
  for (int v : {pad_b, pad_g, pad_r})
    if (v < 0 || v > 255) return fail(YV7_E_ARG, "yv7_letterbox: pad colour outside 0..255");
  if (ws_bytes < yv7::letterbox_workspace_bytes(new_h, new_w)) return fail(YV7_E_WORKSPACE, "yv7_letterbox: workspace too small");
  const uint8_t pad[3] = {(uint8_t)pad_b, (uint8_t)pad_g, (uint8_t)pad_r};
  hipError_t e = yv7::launch_letterbox(reinterpret_cast<const uint8_t*>(src), B, H, W, new_h, new_w, top, left, out_h,
                                       out_w, pad, out_kind, dst, workspace, reinterpret_cast<hipStream_t>(stream));
  if (e != hipSuccess) return hip_fail(e, "yv7_letterbox launch");
  return 0;
}

}  // extern "C"
