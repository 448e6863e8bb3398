// Register-streamed 1x1 convolution (fp16, gfx950), optionally with a second, max-pooled consumer of
// the same input.  Replaces Conv.fuseforward (models/common.py:110-111) for the short-K 1x1 layers of
// the yolov7 ELAN / MP blocks at 160^2 and 80^2, and — as one launch — the MP block's two readers of
// one tensor (cfg/deploy/yolov7.yaml:27-30 and the head's :96-99: `[-1, 1, MP, []], [-1, 1, Conv, [c,
// 1, 1]], [-3, 1, Conv, [c, 1, 1]]`; MP = models/common.py:30-36): y = act(W x + b) at every pixel and
// y2 = act(W2 maxpool2x2(x) + b2) at every second pixel of every second row.
//
// Why: these layers move 2-4 bytes per FLOP, so they are HBM-bound, and the LDS-staged rings keep at
// most a 16-32 KiB slice of activations in flight per CU beside the weight image (the 256->256 layer's
// weights alone are 128 KiB) — by Little's law ~4.3 TB/s at a few microseconds of HBM latency (1x1
// 256->256 @160: 194 us for 838 MB).  Here the weights are the only LDS tenant and the activations go
// straight to registers in the MFMA operand layout:
//  * a wave owns 32 pixels — two image rows x 16 columns — and loads all K channels of them with
//    buffer_load_b128 (lane (li, g) = pixel li, channels ks*32 + 8g .. +7: the B operand of
//    v_mfma_f32_16x16x32_f16 as it stands), the NEXT unit's pixels issued before this unit's MFMAs:
//    8 waves x 16 KiB = 128 KiB in flight per CU;
//  * 128 output channels per pass (W fragments from LDS as the A operand, each used by both pixel
//    rows), one or two passes over the same registers; the pooled consumer takes the 2x2 max in
//    registers (the two rows elementwise, then the neighbouring column by a quad-permute DPP): lanes
//    with even li hold pooled pixel li / 2, odd lanes a duplicate whose stores are dropped;
//  * epilogue straight from the accumulators (bias = accumulator start, compile-time activation,
//    fp16, permlane16 pairing, 16-byte NHWC stores into the output channel slices);
//  * no barrier after the weight load: every wave walks its own units (blocks take XCD-major groups
//    of 8 units, one per wave), and two waves per SIMD overlap one's epilogue with the other's MFMAs.
// LDS: weight rows padded by 16 B (K*2 + 16 per output channel) so the 16 rows of a fragment read hit
// 16 different bank groups; <= 136 KiB.
#include <hip/hip_runtime.h>

#include <type_traits>
#include <utility>

#include "yv7_kernels.h"

namespace yv7 {

namespace {

constexpr int NTH = 512;
constexpr int MAXW = 140 * 1024;   // weight image budget (+ biases) in LDS
typedef uint32_t u2 __attribute__((ext_vector_type(2)));
typedef _Float16 h2 __attribute__((ext_vector_type(2)));
typedef _Float16 h4 __attribute__((ext_vector_type(4)));

template <typename F, int... I>
__device__ __forceinline__ void static_for_seq(F&& f, std::integer_sequence<int, I...>) {
  (f(std::integral_constant<int, I>{}), ...);
}
// f(integral_constant<int, 0>) ... f(integral_constant<int, N - 1>), in order
template <int N, typename F>
__device__ __forceinline__ void static_for(F&& f) {
  static_for_seq(f, std::make_integer_sequence<int, N>{});
}

// one dword (two fp16 channels) of the 2x2 max: rows y, y + 1 of this lane's column elementwise, then
// the neighbouring column (lane li ^ 1) by quad-permute [1, 0, 3, 2]
__device__ __forceinline__ uint32_t pool2x2(uint32_t r0, uint32_t r1) {
  typedef _Float16 h2v __attribute__((ext_vector_type(2)));
  const h2v v = __builtin_elementwise_max(__builtin_bit_cast(h2v, r0), __builtin_bit_cast(h2v, r1));
  const int nb = __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, v), 0xB1, 0xF, 0xF, false);
  return __builtin_bit_cast(uint32_t, __builtin_elementwise_max(v, __builtin_bit_cast(h2v, nb)));
}

// s_waitcnt vmcnt(N) that the two registers' later uses depend on
template <int N>
__device__ __forceinline__ void xwait(u4& a, u4& b) {
  static_assert(N >= 0 && N < 64, "vmcnt range");
  asm volatile("s_waitcnt vmcnt(%2)" : "+v"(a), "+v"(b) : "n"(N) : "memory");
}

// KS: K / 32 (4 or 8); NF: 128-channel passes of the full consumer (1 or 2); POOL: the pooled consumer
// (128 channels) rides along
template <int KS, int NF, bool POOL, int ACT>
__global__ __launch_bounds__(NTH, 1) void conv1x1_rs_kernel(const ConvParams p, const Conv1x1Pooled q) {
  constexpr int K = KS * 32;
  constexpr int ROW = K * 2 + 16;                     // LDS bytes per weight row
  constexpr int NROWS = NF * 128 + (POOL ? 128 : 0);
  constexpr int BOFF = NROWS * ROW;                   // fp32 biases after the weight rows
  static_assert(BOFF + NROWS * 4 <= MAXW, "LDS budget");
  __shared__ __attribute__((aligned(16))) unsigned char smem[BOFF + NROWS * 4];
  float* bias_l = reinterpret_cast<float*>(smem + BOFF);

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int g = lane >> 4, li = lane & 15;

  // weights -> LDS once: row n (full consumer's channels, then the pooled consumer's), 16-byte chunks;
  // every load of a thread is issued before its first LDS write (a loop of load -> write pairs waited
  // out one L2 / HBM round trip per chunk: 8-16 in a row, ~20 us of the 80^2 launch)
  {
    const unsigned char* w1 = reinterpret_cast<const unsigned char*>(p.w);
    const unsigned char* w2 = reinterpret_cast<const unsigned char*>(q.w);
    constexpr int CH = K / 8;   // 16-byte chunks per row
    constexpr int IT = NROWS * CH / NTH;
    static_assert(NROWS * CH % NTH == 0, "whole chunks per thread");
    u4 wv[IT];
#pragma unroll
    for (int t = 0; t < IT; ++t) {
      const int i = tid + t * NTH, n = i / CH, c = i - n * CH;
      const unsigned char* src = n < NF * 128 ? w1 + ((size_t)n * p.kpad + c * 8) * 2
                                              : w2 + ((size_t)(n - NF * 128) * p.kpad + c * 8) * 2;
      wv[t] = *reinterpret_cast<const u4*>(src);
    }
    float bv = 0.f;
    if (tid < NROWS) bv = tid < NF * 128 ? p.bias[tid] : q.bias[tid - NF * 128];
#pragma unroll
    for (int t = 0; t < IT; ++t) {
      const int i = tid + t * NTH, n = i / CH, c = i - n * CH;
      *reinterpret_cast<u4*>(smem + n * ROW + c * 16) = wv[t];
    }
    static_assert(NROWS <= NTH, "one bias per thread");
    if (tid < NROWS) bias_l[tid] = bv;
  }
  __syncthreads();

  // units: (image, row pair, 16-column segment, 128-channel half of the full consumer's output);
  // blocks walk groups of 8 units XCD-major, one per wave, so the two halves of a pixel block run on
  // one CU at the same time and the second half's loads hit L2
  const int segs = p.W / 16, rps = p.H / 2;
  const int U = p.B * rps * segs * NF;
  const TileWalk tw = xcd_tile_walk((U + 7) / 8);
  const int ng = tw.count();
  if (ng == 0) return;
  const auto xr = make_rsrc(p.x, p.xbytes);
  const auto yr = make_rsrc(p.y, 0x7fffffffu);
  const auto y2r = make_rsrc(q.y, 0x7fffffffu);
  const uint32_t xrow = (uint32_t)((p.W + 2 * BORDER) * p.xc * 2);        // bytes per input row
  const uint32_t yrow = (uint32_t)((p.W + 2 * BORDER) * p.yc * 2);        // bytes per output row
  const uint32_t xl = (uint32_t)((li * p.xc + p.xoff + g * 8) * 2);       // lane's part of an input offset
  const uint32_t lane_ch = (uint32_t)((16 * (g & 1) + 8 * (g >> 1)) * 2);  // epilogue channel pairing (bytes)

  // a unit's scalar input offset (pixel (y, x) of its block, channel 0 of the slice); units past the
  // end read zeros and store into the void, so every wave issues the same loads and stores and the
  // compiler's vmcnt counting stays static (no path-merged vmcnt(0))
  struct Unit { uint32_t xo, yo, y2o; int nh; };
  auto unit = [&](int i) __attribute__((always_inline)) {
    Unit d;
    int u = i < ng ? tw.at(i) * 8 + wave : U;
    if (u >= U) {
      d.xo = 0x40000000u;
      d.yo = d.y2o = 0x80000000u;
      d.nh = 0;
      return d;
    }
    d.nh = u % NF;
    u /= NF;
    const int x = (u % segs) * 16;
    u /= segs;
    const int y = (u % rps) * 2, b = u / rps;
    d.xo = __builtin_amdgcn_readfirstlane((uint32_t)(pix_index(b, y, x, p.H, p.W) * p.xc * 2));
    d.yo = (uint32_t)((pix_index(b, y, x + li, p.H, p.W) * p.yc + p.yoff + d.nh * 128) * 2) + lane_ch;
    if constexpr (POOL)
      d.y2o = (li & 1) ? 0x80000000u
                       : (uint32_t)((pix_index(b, y / 2, x / 2 + li / 2, p.H / 2, p.W / 2) * q.yc + q.yoff) * 2) + lane_ch;
    return d;
  };
  // X loads are inline asm: for register loads hipcc counts vmcnt itself, and at this loop's header it
  // merges the prologue's and the back edge's queues into a vmcnt(0) before the first MFMA — the whole
  // next-unit prefetch drained every unit.  Here the waits are counted by hand (xwait) and thread the
  // registers through, so no use can be scheduled above them.
  const uint32_t xl1 = xl + xrow;
  auto load_xk = [&](const Unit& d, int r, auto ksc) __attribute__((always_inline)) {
    constexpr int ks = decltype(ksc)::value;
    u4 v;
    asm volatile("buffer_load_dwordx4 %0, %1, %2, %3 offen offset:%4"
                 : "=v"(v)
                 : "v"(r ? xl1 : xl), "s"(xr), "s"(d.xo), "n"(ks * 64)
                 : "memory");
    return v;
  };

  // LDS fragment of weight row block n0 (16 rows), k step ks: lane (li, g) = row n0 + li, chunk 4 ks + g
  // (the base is re-laundered every unit: the weight image never changes inside the loop, and the
  // compiler would otherwise hoist every fragment read of a unit out of it — 64 fragments, 256 VGPRs)
  const uint32_t wl0 = (uint32_t)(li * ROW + g * 16);
  uint32_t wl = wl0;
  auto wfrag = [&](int n0, int ks) __attribute__((always_inline)) {
    return *reinterpret_cast<const u4*>(smem + wl + n0 * ROW + ks * 64);
  };

  // epilogue: accumulators j (n-fragment) hold channels 16 j + 4 g .. +3 of pixel li; pairs (2m, 2m+1)
  // trade halves by permlane16 so each lane stores 8 consecutive channels
  auto store_pair = [&](const f4& a4, const f4& b4, __amdgpu_buffer_rsrc_t r, uint32_t off) __attribute__((always_inline)) {
    h4 va, vb;
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      va[e] = (_Float16)act_t<ACT>(a4[e]);
      vb[e] = (_Float16)act_t<ACT>(b4[e]);
    }
    const u2 a = __builtin_bit_cast(u2, va), b = __builtin_bit_cast(u2, vb);
    const auto s0 = __builtin_amdgcn_permlane16_swap(a[0], b[0], false, false);
    const auto s1 = __builtin_amdgcn_permlane16_swap(a[1], b[1], false, false);
    const u4 v = {s0[0], s1[0], s0[1], s1[1]};
    __builtin_amdgcn_raw_buffer_store_b128(v, r, off, 0, 0);
    __builtin_amdgcn_sched_barrier(0);   // one pair at a time: bounded live registers in the epilogue
  };

  // X of the current unit, k step by k step; each step's registers take the next unit's k step as soon
  // as its MFMAs are issued (a rolling prefetch: a whole unit of loads in flight per wave)
  u4 xs[2][KS];
  Unit cur = unit(0);
  static_for<KS>([&](auto ksc) __attribute__((always_inline)) {
    xs[0][decltype(ksc)::value] = load_xk(cur, 0, ksc);
    xs[1][decltype(ksc)::value] = load_xk(cur, 1, ksc);
  });
  // stores into the void standing in for a previous unit's epilogue, so the first unit's counted waits
  // are the steady state's (distinct offsets: identical stores would be merged into one)
  constexpr int NST = POOL ? 12 : 8;   // epilogue stores per unit
  static_for<NST>([&](auto kc) __attribute__((always_inline)) {
    __builtin_amdgcn_raw_buffer_store_b128(u4{0u, 0u, 0u, 0u}, yr, 0x80000000u + decltype(kc)::value * 16, 0, 0);
  });
  // the pooled consumer's B operands, taken from X during the full pass (so X can be recycled there)
  u4 pb[POOL ? KS : 1];
  // the full pass over the unit's K: 16 fragment MFMAs per k step (8 weight fragments x 2 pixel rows),
  // the next k step's weight fragments read during this one's MFMAs; then (POOL) this k step's 2x2 max,
  // and the k step's X registers take the next unit's (the asm loads are ordered after the MFMAs that
  // read them by their memory clobber)
  auto full_pass = [&](int n0, f4 (&acc)[8][2], const Unit& nxt) __attribute__((always_inline)) {
    u4 wa[8], wb[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) wa[j] = wfrag(n0 + j * 16, 0);
    static_for<KS>([&](auto ksc) __attribute__((always_inline)) {
      constexpr int ks = decltype(ksc)::value;
      u4(&wc)[8] = (ks & 1) ? wb : wa;
      u4(&wn)[8] = (ks & 1) ? wa : wb;
      if (ks + 1 < KS) {
#pragma unroll
        for (int j = 0; j < 8; ++j) wn[j] = wfrag(n0 + j * 16, ks + 1);
      }
      // this k step's X landed: younger than its two loads are the rest of that unit's loads, the
      // previous unit's epilogue stores and this unit's recycle loads so far — a constant
      xwait<2 * KS - 2 + NST>(xs[0][ks], xs[1][ks]);
#pragma unroll
      for (int j = 0; j < 8; ++j)
#pragma unroll
        for (int r = 0; r < 2; ++r)
          acc[j][r] = __builtin_amdgcn_mfma_f32_16x16x32_f16(__builtin_bit_cast(h8, wc[j]), __builtin_bit_cast(h8, xs[r][ks]),
                                                             acc[j][r], 0, 0, 0);
      if constexpr (POOL) {
        // 2x2 max: the two rows elementwise, then columns (li, li ^ 1) by quad-permute [1, 0, 3, 2];
        // lanes with odd li compute a duplicate that is stored into the void
        const u4 a0 = xs[0][ks], a1 = xs[1][ks];
        pb[ks] = u4{pool2x2(a0.x, a1.x), pool2x2(a0.y, a1.y), pool2x2(a0.z, a1.z), pool2x2(a0.w, a1.w)};
      }
      xs[0][ks] = load_xk(nxt, 0, std::integral_constant<int, ks>{});
      xs[1][ks] = load_xk(nxt, 1, std::integral_constant<int, ks>{});
    });
  };
  // the pooled consumer's pass: one pixel fragment per weight fragment
  auto pooled_pass = [&](f4 (&acc)[8]) __attribute__((always_inline)) {
    u4 wa[8], wb[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) wa[j] = wfrag(NF * 128 + j * 16, 0);
    static_for<KS>([&](auto ksc) __attribute__((always_inline)) {
      constexpr int ks = decltype(ksc)::value;
      u4(&wc)[8] = (ks & 1) ? wb : wa;
      u4(&wn)[8] = (ks & 1) ? wa : wb;
      if (ks + 1 < KS) {
#pragma unroll
        for (int j = 0; j < 8; ++j) wn[j] = wfrag(NF * 128 + j * 16, ks + 1);
      }
#pragma unroll
      for (int j = 0; j < 8; ++j)
        acc[j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(__builtin_bit_cast(h8, wc[j]), __builtin_bit_cast(h8, pb[ks]), acc[j],
                                                        0, 0, 0);
    });
  };
  for (int i = 0; i < ng; ++i) {
    wl = wl0;
    asm volatile("" : "+v"(wl));
    const Unit nxt = unit(i + 1);
    {
      f4 acc[8][2];
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const f4 bv = *reinterpret_cast<const f4*>(bias_l + cur.nh * 128 + j * 16 + g * 4);
        acc[j][0] = bv;
        acc[j][1] = bv;
      }
      full_pass(cur.nh * 128, acc, nxt);
#pragma unroll
      for (int r = 0; r < 2; ++r)
#pragma unroll
        for (int m = 0; m < 4; ++m) store_pair(acc[2 * m][r], acc[2 * m + 1][r], yr, cur.yo + r * yrow + (uint32_t)(m * 64));
    }
    if constexpr (POOL) {
      // after the full consumer's epilogue (its accumulators are free again)
      f4 acc[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) acc[j] = *reinterpret_cast<const f4*>(bias_l + NF * 128 + j * 16 + g * 4);
      pooled_pass(acc);
#pragma unroll
      for (int m = 0; m < 4; ++m) store_pair(acc[2 * m], acc[2 * m + 1], y2r, cur.y2o + (uint32_t)(m * 64));
    }
    cur = nxt;
  }
  // the last unit's recycle loads (into the void) are still in flight: a wave must not end with loads
  // pending into its registers — hipcc does not know about them, and the next kernel's waves could be
  // handed these VGPRs before the data lands (it corrupted the following op's registers in the first build)
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

template <int KS, int NF, bool POOL>
hipError_t launch_ks(const ConvParams& p, const Conv1x1Pooled& q, int grid, hipStream_t st) {
  if (p.act == 1) YV7_LAUNCH((conv1x1_rs_kernel<KS, NF, POOL, 1>), dim3(grid), dim3(NTH), 0, st, p, q);
  else if (p.act == 2) YV7_LAUNCH((conv1x1_rs_kernel<KS, NF, POOL, 2>), dim3(grid), dim3(NTH), 0, st, p, q);
  else YV7_LAUNCH((conv1x1_rs_kernel<KS, NF, POOL, 0>), dim3(grid), dim3(NTH), 0, st, p, q);
  return hipGetLastError();
}

}  // namespace

bool conv1x1_rs_supported(const ConvParams& p, const Conv1x1Pooled* q) {
  // (output channels are whole 128-channel passes: no per-channel store masks)
  const bool base = p.k == 1 && p.s == 1 && p.pad == 0 && !p.pool && (p.cin == 128 || p.cin == 256) &&
                    p.kpad == p.cin && (p.cout == 128 || p.cout == 256) && p.H % 2 == 0 &&
                    p.W % 16 == 0 && p.Ho == p.H && p.Wo == p.W && p.xc % 8 == 0 && p.xoff % 8 == 0 &&
                    p.yc % 8 == 0 && p.yoff % 8 == 0;
  if (!base) return false;
  if (!q) return true;
  return p.cout == 128 && q->cout == 128 && q->yc % 8 == 0 && q->yoff % 8 == 0 && q->act == p.act && q->w &&
         q->bias && q->y;
}

hipError_t launch_conv1x1_rs(const ConvParams& p, const Conv1x1Pooled* q, hipStream_t st) {
  if (!conv1x1_rs_supported(p, q)) return hipErrorInvalidValue;
  static const int cus = [] {
    int dev = 0, v = 0;
    if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&v, hipDeviceAttributeMultiprocessorCount, dev) !=
                                                 hipSuccess || v <= 0)
      v = 256;
    return v;
  }();
  const long U = (long)p.B * (p.H / 2) * (p.W / 16);
  const long G = (U + 7) / 8;
  const int grid = (int)(G < cus ? G : cus);
  const Conv1x1Pooled none{};
  const bool two = p.cout > 128;
  if (q) return p.cin == 128 ? launch_ks<4, 1, true>(p, *q, grid, st) : launch_ks<8, 1, true>(p, *q, grid, st);
  if (p.cin == 128) return two ? launch_ks<4, 2, false>(p, none, grid, st) : launch_ks<4, 1, false>(p, none, grid, st);
  return two ? launch_ks<8, 2, false>(p, none, grid, st) : launch_ks<8, 1, false>(p, none, grid, st);
}

}  // namespace yv7
