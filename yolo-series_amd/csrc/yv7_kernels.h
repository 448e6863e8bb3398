// Shared definitions of the yv7 HIP kernels (gfx950 / CDNA4 only).
#pragma once
#include <hip/hip_ext.h>
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <type_traits>

namespace yv7 {

// Live per-op kernel timing (runtime.cpp's profile mode).  While a forward is profiled the runtime
// points op_events() at the current op's (start, stop) event pair, and every kernel of the op is
// launched through hipExtLaunchKernel with the first launch carrying `start` and each launch `stop`:
// the pair then spans the op's own dispatches (the begin / end timestamps rocprofv3's kernel trace
// reports), not the interval between two markers on the stream, which with batches in flight also
// counts the time a kernel waits for CUs the other streams' kernels hold.  Null events: a plain launch.
struct OpEvents {
  hipEvent_t start = nullptr, stop = nullptr;
  int launches = 0;
};
inline OpEvents& op_events() {
  static thread_local OpEvents e;
  return e;
}
// Dry run (yv7_op_kernels): while `dry` is set, YV7_LAUNCH launches nothing and records the host stub
// of the kernel the dispatch picked (runtime.cpp turns it into the symbol rocprofv3 reports).
struct LaunchRec {
  bool dry = false;
  int n = 0;
  const void* fn[4] = {nullptr, nullptr, nullptr, nullptr};
};
inline LaunchRec& launch_rec() {
  static thread_local LaunchRec r;
  return r;
}
#define YV7_LAUNCH(kernel, grid, block, shmem, st, ...)                                                    \
  do {                                                                                                     \
    ::yv7::LaunchRec& lr_ = ::yv7::launch_rec();                                                           \
    if (lr_.dry) {                                                                                         \
      if (lr_.n < 4) lr_.fn[lr_.n] = reinterpret_cast<const void*>(kernel);                               \
      lr_.n++;                                                                                             \
      break;                                                                                               \
    }                                                                                                      \
    ::yv7::OpEvents& ev_ = ::yv7::op_events();                                                             \
    hipExtLaunchKernelGGL(kernel, grid, block, shmem, st, ev_.launches ? nullptr : ev_.start, ev_.stop, 0, \
                          __VA_ARGS__);                                                                    \
    if (ev_.stop) ev_.launches++;                                                                          \
  } while (0)

typedef _Float16 h8 __attribute__((ext_vector_type(8)));
typedef float f4 __attribute__((ext_vector_type(4)));
typedef uint32_t u4 __attribute__((ext_vector_type(4)));

// Elements of T per 16-byte vector.
template <typename T> struct Vec;
template <> struct Vec<_Float16> { static constexpr int N = 8; };
template <> struct Vec<float> { static constexpr int N = 4; };

// Persistent tile walk, XCD-major: the 8 XCDs (blockIdx % 8 on the round-robin dispatch) each take a
// contiguous eighth of the T tiles, walked by that XCD's blocks (t, t + step, ... < end), so
// neighbouring tiles — sharing halo rows / operand panels — are fetched into one L2, and a partial
// last round is spread evenly over the XCDs.  Falls back to t = blockIdx, step = gridDim when the grid
// is not a multiple of 8.
struct TileWalk {
  int t, step, end;
  __device__ __forceinline__ int count() const { return t < end ? (end - t + step - 1) / step : 0; }
  __device__ __forceinline__ int at(int i) const { return t + i * step; }
};
__device__ __forceinline__ TileWalk xcd_tile_walk(int T) {
  const int G = gridDim.x, b = blockIdx.x;
  if (G % 8) return TileWalk{b, G, T};
  const int x = b % 8, gx = G / 8;
  return TileWalk{(int)((long)x * T / 8) + b / 8, gx, (int)((long)(x + 1) * T / 8)};
}

// The same walk for a block b of a virtual grid of G blocks (G a multiple of 8: b % 8 is its XCD).
__device__ __forceinline__ TileWalk xcd_tile_walk_g(int T, int G, int b) {
  const int x = b % 8, gx = G / 8;
  return TileWalk{(int)((long)x * T / 8) + b / 8, gx, (int)((long)(x + 1) * T / 8)};
}

template <int ACT>
__device__ __forceinline__ float act_t(float v) {
  // SiLU with v_exp_f32 / v_rcp_f32 (~1 ulp each): plenty for an fp16 output, ~4x cheaper than the
  // IEEE expf + division sequence, which otherwise rivals the MFMA time of small-K layers.
  if constexpr (ACT == 1) return v * __builtin_amdgcn_rcpf(1.0f + __builtin_amdgcn_exp2f(-1.4426950408889634f * v));
  if constexpr (ACT == 2) return v > 0.0f ? v : v * 0.1f;
  return v;
}

// Calls f(std::integral_constant<int, ACT>) with the layer's activation as a compile-time constant, so
// an epilogue is straight-line code (a runtime switch per element costs more than the SiLU itself).
template <typename F>
__device__ __forceinline__ void with_act(int act, F&& f) {
  if (act == 1) f(std::integral_constant<int, 1>{});
  else if (act == 2) f(std::integral_constant<int, 2>{});
  else f(std::integral_constant<int, 0>{});
}

// Activation tensors in the workspace are NHWC with a BORDER-pixel zero frame around every image:
// [B][H + 2*BORDER][W + 2*BORDER][C], kernels write only the interior.  A 3x3 / pad-1 window then never
// needs a bounds test (its out-of-image taps read the zero frame), so the conv kernels' operand loads
// are unconditional buffer loads with the tap offset in a scalar register.
constexpr int BORDER = 1;

// Element index of pixel (b, h, w) (interior coordinates, -BORDER <= h < H + BORDER) of a bordered tensor.
__host__ __device__ __forceinline__ size_t pix_index(int b, int h, int w, int H, int W) {
  return ((size_t)b * (H + 2 * BORDER) + h + BORDER) * (W + 2 * BORDER) + w + BORDER;
}
__host__ __device__ __forceinline__ size_t bordered_pixels(int B, int H, int W) {
  return (size_t)B * (H + 2 * BORDER) * (W + 2 * BORDER);
}

// Raw buffer resource over [base, base + bytes): loads at voffset >= bytes return zero.
__device__ __forceinline__ __amdgpu_buffer_rsrc_t make_rsrc(const void* base, uint32_t bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), (short)0, (int)bytes, 0x00020000);
}

// Kernel parameters of one conv launch (also the fused Detect head).
struct ConvParams {
  const void* x;      // bordered NHWC input tensor (allocation start)
  void* y;            // bordered NHWC output tensor (CONV)
  const void* w;      // packed weights [cout_pad][kpad]
  const float* bias;  // [cout_pad]
  const void* zero;   // >= 16 zero bytes in device memory
  uint32_t xbytes, wbytes;          // byte sizes of the input tensor / this conv's weights (buffer ranges)
  int B, H, W, xc, xoff, cin;       // input geometry (interior), pitch (channels), channel offset, channels read
  int Ho, Wo, yc, yoff, cout;       // output geometry
  int k, s, pad, act, kpad, K, M;   // K = k*k*cin, M = B*Ho*Wo
  // Detect epilogue
  float* z;           // [B, N, no] fp32
  float* raw;         // [B, na, Ho, Wo, no] fp32 for this level (nullable)
  float* best;        // [B, N] yv7_row_best records (nullable; written by the fp16 head epilogue)
  int nrows, row_off, na, no;
  float stride, anchor[8];  // anchor[2*a + {0,1}] pixels
  int variant;        // 0 = tuned dispatch; >0 forces a kernel variant (microbenchmarks / A-B tests)
  // split-K scratch (fp16 ring kernels): fp32 partial tiles and per-tile arrival counters (zeroed once,
  // re-armed by the kernel); ksplit > 0 forces the split count (microbenchmarks), 0 = tuned choice
  float* part;
  int* cnt;
  size_t part_bytes;
  int cnt_n;
  int ksplit;
  int pool;           // 2: 1x1 conv over the 2x2 / stride-2 max of the input (MP folded in; k = 1, s = 2)
  // 3x3 stride-1/2 convs of fp16 plans: the weights again, fragment-packed for conv_lr.hip (pack_frag),
  // or null
  const void* wf;
  uint32_t wfbytes;
};

// The max-pooled second consumer of a register-streamed 1x1 conv's input (conv_rs.hip): the MP block's
// `MP -> 1x1` branch (pool = 2 op) launched together with the plain 1x1 reading the same tensor.
struct Conv1x1Pooled {
  const void* w;        // packed weights [cout_pad32][kpad] (kpad == the full conv's)
  const float* bias;
  void* y;              // bordered NHWC output tensor at half resolution
  int yc, yoff, cout, act;
};
bool conv1x1_rs_supported(const ConvParams& p, const Conv1x1Pooled* q);
hipError_t launch_conv1x1_rs(const ConvParams& p, const Conv1x1Pooled* q, hipStream_t st);

// Split-K scratch the fp16 dispatch needs for one conv (0 when it does not split).
size_t conv_splitk_part_bytes(const ConvParams& p);
int conv_splitk_tiles(const ConvParams& p);

// fp8 1x1 conv (conv_f8.hip): dense e4m3 activations [M][kp] x e4m3 weights [cout_pad32][kp], fp32
// per-channel weight scales and a per-tensor activation scale applied in the epilogue.
struct F8ConvParams {
  const void* x8;       // dense e4m3 input [M][kp] (written by launch_quant_f8)
  void* y;              // bordered NHWC fp16 output tensor
  const void* w8;       // e4m3 weights [cout_pad32][kp]
  const float* bias;    // [cout]
  const float* wscale;  // [cout] per-channel weight scales
  float xscale;         // activation scale: x ~ e4m3 value * xscale
  uint32_t wbytes;      // byte size of w8 (buffer range)
  int M, kp, cout, H, W, yc, yoff, act;   // H, W: output (= input) interior size
  // fused quantization (x8 == nullptr): the fp16 input slice [xoff, xoff + cin) of the bordered NHWC
  // tensor x16 (pitch xc, xbytes long) is quantized to e4m3 (x * qscale, clamped to +-448) on its
  // way into LDS, so no dense e4m3 copy is written first
  const void* x16;
  uint32_t xbytes;
  int xc, xoff, cin;
  float qscale;
};
hipError_t launch_quant_f8(const void* x, int B, int H, int W, int xc, int xoff, int cin, int kp, float qscale,
                           void* y8, hipStream_t st);
hipError_t launch_conv_f8(const F8ConvParams& p, hipStream_t st);

// Fused stem: image -> conv A (3 -> 32, 3x3, stride sa) -> conv B (32 -> 64, 3x3, stride 2).
struct StemParams {
  const void* x;        // [B,3,H,W] image (fp16 or fp32)
  void* y;              // conv-B output tensor (bordered NHWC fp16)
  const void* wa;       // conv-A weights [32][kpad_a] (k = tap*3 + ci)
  const float* ba;
  const void* wb;       // conv-B weights [64][kpad_b] (k = tap*32 + ci)
  const float* bb;
  int B, H, W, yc, yoff, kpad_a, kpad_b, act_a, act_b, sa;
  int variant;          // 0; >0: microbenchmark hooks (scripts/stembench.hip)
  int reorg;            // 1: the w6 front end (ReOrg + 12 -> 64 -> 128, wa k = tap*16 + ci), stem_reorg_kernel
};

// Host launchers (defined in the .hip files, called from the runtime).
hipError_t launch_conv(int dtype, const ConvParams& p, bool detect, hipStream_t st);
bool det_writes_rowbest(int dtype);   // true when the head kernel launch_conv picks fills ConvParams::best
hipError_t launch_conv_f16(const ConvParams& p, bool detect, hipStream_t st);
bool halo_supported(const ConvParams& p);
bool ws64_supported(const ConvParams& p);
hipError_t launch_conv_ws64(const ConvParams& p, hipStream_t st);
hipError_t launch_conv_halo(const ConvParams& p, hipStream_t st);
bool hring_supported(const ConvParams& p);
// low-resolution 3x3 (conv_lr.hip): cfg 0-4 = tile shape; weights from ConvParams::wf
bool lr_supported(const ConvParams& p, int cfg);
hipError_t launch_conv_lr(const ConvParams& p, int cfg, hipStream_t st);
// The low-resolution configuration the default fp16 dispatch gives a 3x3 stride-1 layer (conv_f16.hip
// launch_conv_f16), or -1 when another kernel takes it.
int lr_default_cfg(const ConvParams& p);
// A chain of 3x3 stride-1 convs at one resolution, each reading the previous one's output slice (an ELAN
// block's 3x3 stack, cfg/deploy/yolov7.yaml:65-68, 84-87, 98-101, 113-116, 128-131) as ONE launch of
// conv_lr.hip's tile body (conv3x3_chain_kernel): layer l + 1's tiles start as soon as the rows of layer l
// they read are done (per image group and row band ready counters), instead of after layer l's last tile.
constexpr int CHAIN_MAX = 4;
struct ChainParams {
  ConvParams p[CHAIN_MAX];   // layer l: its own kernel parameters (p[l + 1].x / xoff = p[l].y / yoff)
  int nl;                    // layers, 2 .. CHAIN_MAX
  int cfg0, cfg1;            // low-resolution configuration of layer 0 and of layers 1 .. nl - 1
  int* ctr;                  // chain_counter_bytes() of workspace scratch, zeroed once, re-armed by the kernel
};
// the chain's launch form exists (configurations, widths, activation) and its geometry is consistent;
// ctr may be null here (a layout query)
bool chain_supported(const ChainParams& c);
size_t chain_counter_bytes(const ChainParams& c);
long chain_tasks(const ChainParams& c);   // tiles of all layers
hipError_t launch_conv_chain(const ChainParams& c, hipStream_t st);
size_t frag_bytes(int cin, int cout, int taps);
hipError_t pack_frag(const void* w, int kpad, int cin, int cout, int taps, void* out, hipStream_t st);
hipError_t launch_conv_hring(const ConvParams& p, int cus, hipStream_t st);
// stride-2 3x3 with the weights resident in VGPRs (conv_s2.hip): cfg 0-4 = tile shape; weights from wf
bool s2_supported(const ConvParams& p, int cfg);
hipError_t launch_conv_s2(const ConvParams& p, int cfg, int cus, hipStream_t st);
// 1x1 with the weights resident in VGPRs (conv_w1.hip): cfg 0-5; weights from wf (1-tap fragment pack)
bool w1_supported(const ConvParams& p, int cfg);
hipError_t launch_conv_w1(const ConvParams& p, int cfg, int cus, hipStream_t st);
hipError_t launch_input(int dtype, const void* x, int x_dtype, void* y, int B, int H, int W, int yc,
                        bool reorg, hipStream_t st);
hipError_t launch_maxpool(int dtype, const void* x, int B, int H, int W, int xc, int xoff, void* y, int Ho,
                          int Wo, int yc, int yoff, int C, int k, int s, int pad, hipStream_t st);
bool spp_cascade_supported(int dtype, int H, int W, int C);
hipError_t launch_spp_cascade(int dtype, void* x, int B, int H, int W, int xc, int coff, int C, hipStream_t st);
hipError_t launch_upsample2x(int dtype, const void* x, int B, int H, int W, int xc, int xoff, void* y, int yc,
                             int yoff, int C, hipStream_t st);
bool stem_supported(int cin, int ca, int cb, int sa);
hipError_t launch_stem(const StemParams& p, int x_dtype, hipStream_t st);
hipError_t launch_copy(int dtype, const void* x, int B, int H, int W, int xc, int xoff, void* y, int yc, int yoff,
                       int C, hipStream_t st);

}  // namespace yv7
