// fp16 implicit-GEMM convolution for gfx950 (the bench / serving path), NHWC activations, KRSC weights.
//
// Replaces ATen conv2d + BN-folded bias + SiLU/LeakyReLU (Conv.fuseforward models/common.py:110-111,
// RepConv deploy common.py:498-500) and the Detect head conv + decode (models/yolo.py:46-57).
//
// GEMM view: M = B*Ho*Wo pixels, N = cout, K = k*k*cin ordered (r, s, ci).  A 256-thread block
// (4 waves, WM x WN) owns a BM x BN tile; every wave a (BM/WM) x (BN/WN) sub-tile of 16x16 MFMA tiles.
//  * K step 64 (128 bytes per tile row), two v_mfma_f32_16x16x32_f16 sub-steps per tile per step;
//  * LDS rows of 8 x 16-byte chunks, chunk index XOR-swizzled with (row & 7) so the 16-lane groups
//    of ds_read_b128 hit distinct 16-byte slots; double-buffered, one barrier per K step;
//  * next step's global loads are issued into registers before this step's MFMAs and written to
//    the other LDS buffer after them (issue-early / write-late);
//  * operands swapped (weights as the MFMA A operand) so each lane's accumulator holds 4
//    consecutive output channels of one pixel: the epilogue packs them into 8-byte LDS writes, and
//    the tile leaves as full 16-byte NHWC row chunks into the output's channel slice (zero-copy concat);
//  * XCD-aware bijective block remap: consecutive tiles (all N tiles of an M tile) share an XCD's L2.
#include <cstdlib>

#include "yv7_kernels.h"

namespace yv7 {

namespace {

constexpr int NT = 256;
constexpr int BKE = 64;    // K elements per step
constexpr int ROWB = 128;  // LDS bytes per tile row

__device__ __forceinline__ int swz(int row, int chunk) { return chunk ^ (row & 7); }

__device__ __forceinline__ float act_fn(float v, int act) {
  // SiLU with v_exp_f32 / v_rcp_f32 (~1 ulp each): plenty for an fp16 output, ~4x cheaper than the
  // IEEE expf + division sequence, which otherwise rivals the MFMA time of small-K layers.
  if (act == 1) return v * __builtin_amdgcn_rcpf(1.0f + __builtin_amdgcn_exp2f(-1.4426950408889634f * v));
  if (act == 2) return v > 0.0f ? v : v * 0.1f;
  return v;
}

template <int BM, int BN, int WM, bool ONE, bool DET>
__global__ __launch_bounds__(NT, 2) void conv_f16_kernel(const ConvParams p) {
  constexpr int WN = 4 / WM;
  constexpr int WTM = BM / WM, WTN = BN / WN;
  constexpr int TM = WTM / 16, TN = WTN / 16;
  constexpr int RA = BM / 32;                 // A rows per thread (32 rows per pass of 256 threads)
  constexpr int RB = (BN + 31) / 32;
  constexpr int STAGE = (BM + BN) * ROWB;
  constexpr int CPITCH = BN * 2 + 16;
  constexpr int LDS = (2 * STAGE > BM * CPITCH) ? 2 * STAGE : BM * CPITCH;
  __shared__ __attribute__((aligned(16))) unsigned char smem[LDS];

  const int tid = threadIdx.x;
  const int lane = tid & 63, wave = tid >> 6;
  const int wm = wave / WN, wn = wave % WN;
  const int g = lane >> 4, li = lane & 15;

  const int nwg = gridDim.x, bid = blockIdx.x;
  const int q = nwg >> 3, r = nwg & 7, xcd = bid & 7, loc = bid >> 3;
  const int wgid = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + loc;
  const int nN = (p.cout + BN - 1) / BN;
  const int m0 = (wgid / nN) * BM, n0 = (wgid % nN) * BN;

  const _Float16* __restrict__ x = reinterpret_cast<const _Float16*>(p.x);
  const _Float16* __restrict__ w = reinterpret_cast<const _Float16*>(p.w);

  const int c = tid & 7;     // 16-byte chunk column this thread moves
  const int r0 = tid >> 3;   // first row this thread moves

  // Per-row source pointers and tap-validity masks, computed once: a K step then costs one pointer
  // add, one mask test and one 16-byte load per row (im2col address math hoisted out of the loop).
  const _Float16* a_ptr[RA];
  uint32_t a_mask[RA];
#pragma unroll
  for (int j = 0; j < RA; ++j) {
    const int m = m0 + r0 + 32 * j;
    const bool ok = m < p.M;
    const int mm = ok ? m : 0;
    if (ONE) {
      a_ptr[j] = x + (size_t)mm * p.xc + p.xoff;
      a_mask[j] = ok ? 1u : 0u;
    } else {
      const int hw = p.Ho * p.Wo;
      const int b = mm / hw, rem = mm - b * hw;
      const int ho = rem / p.Wo, wo = rem - ho * p.Wo;
      const int h0 = ho * p.s - p.pad, w0 = wo * p.s - p.pad;
      a_ptr[j] = x + ((ptrdiff_t)(b * p.H + h0) * p.W + w0) * p.xc + p.xoff;
      uint32_t mk = 0;
      for (int rr = 0; rr < p.k; ++rr)
        for (int ss = 0; ss < p.k; ++ss)
          if (ok && (unsigned)(h0 + rr) < (unsigned)p.H && (unsigned)(w0 + ss) < (unsigned)p.W)
            mk |= 1u << (rr * p.k + ss);
      a_mask[j] = mk;
    }
  }
  const _Float16* b_ptr[RB];
  bool b_ok[RB];
#pragma unroll
  for (int j = 0; j < RB; ++j) {
    const int row = r0 + 32 * j;
    b_ok[j] = row < BN && n0 + row < p.cout;
    b_ptr[j] = w + (size_t)(b_ok[j] ? n0 + row : 0) * p.kpad + c * 8;
  }

  u4 ra[RA], rb[RB];
  const int nk = p.kpad / BKE;
  // K position of this thread's chunk: k = kt*64 + c*8 = tap*cin + ci, tap = rr*k + ss (incremental)
  int ci = c * 8, tap = 0, rr = 0, ss = 0;
  if (!ONE) {
    while (ci >= p.cin) { ci -= p.cin; ++tap; if (++ss == p.k) { ss = 0; ++rr; } }
  }

  auto gload = [&](int kt) {
    const int k = kt * BKE + c * 8;
    const bool kin = k < p.K;
    if (ONE) {
#pragma unroll
      for (int j = 0; j < RA; ++j) {
        u4 v = {0u, 0u, 0u, 0u};
        if (a_mask[j] && kin) v = *reinterpret_cast<const u4*>(a_ptr[j] + k);
        ra[j] = v;
      }
    } else {
      const ptrdiff_t delta = ((ptrdiff_t)rr * p.W + ss) * p.xc + ci;
      const uint32_t bit = kin ? (1u << tap) : 0u;
#pragma unroll
      for (int j = 0; j < RA; ++j) {
        u4 v = {0u, 0u, 0u, 0u};
        if (a_mask[j] & bit) v = *reinterpret_cast<const u4*>(a_ptr[j] + delta);
        ra[j] = v;
      }
      ci += BKE;  // advance to the next K step
      while (ci >= p.cin) { ci -= p.cin; ++tap; if (++ss == p.k) { ss = 0; ++rr; } }
    }
#pragma unroll
    for (int j = 0; j < RB; ++j) {
      u4 v = {0u, 0u, 0u, 0u};
      if (b_ok[j]) v = *reinterpret_cast<const u4*>(b_ptr[j] + kt * BKE);
      rb[j] = v;
    }
  };
  auto lstore = [&](int buf) {
    unsigned char* As = smem + buf * STAGE;
    unsigned char* Bs = As + BM * ROWB;
#pragma unroll
    for (int j = 0; j < RA; ++j) {
      const int row = r0 + 32 * j;
      *reinterpret_cast<u4*>(As + row * ROWB + swz(row, c) * 16) = ra[j];
    }
#pragma unroll
    for (int j = 0; j < RB; ++j) {
      const int row = r0 + 32 * j;
      if (row < BN) *reinterpret_cast<u4*>(Bs + row * ROWB + swz(row, c) * 16) = rb[j];
    }
  };

  f4 acc[TN][TM];
#pragma unroll
  for (int j = 0; j < TN; ++j)
#pragma unroll
    for (int i = 0; i < TM; ++i) acc[j][i] = f4{0.f, 0.f, 0.f, 0.f};

  gload(0);
  lstore(0);
  __syncthreads();
  for (int kt = 0; kt < nk; ++kt) {
    const int buf = kt & 1;
    if (kt + 1 < nk) gload(kt + 1);
    const unsigned char* As = smem + buf * STAGE;
    const unsigned char* Bs = As + BM * ROWB;
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      const int ch = s * 4 + g;
      u4 xa[TM], wb[TN];
#pragma unroll
      for (int i = 0; i < TM; ++i) {
        const int row = wm * WTM + i * 16 + li;
        xa[i] = *reinterpret_cast<const u4*>(As + row * ROWB + swz(row, ch) * 16);
      }
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        const int row = wn * WTN + j * 16 + li;
        wb[j] = *reinterpret_cast<const u4*>(Bs + row * ROWB + swz(row, ch) * 16);
      }
#pragma unroll
      for (int j = 0; j < TN; ++j)
#pragma unroll
        for (int i = 0; i < TM; ++i)
          acc[j][i] = __builtin_amdgcn_mfma_f32_16x16x32_f16(__builtin_bit_cast(h8, wb[j]),
                                                             __builtin_bit_cast(h8, xa[i]), acc[j][i], 0, 0, 0);
    }
    if (kt + 1 < nk) lstore(buf ^ 1);
    __syncthreads();
  }

  // accumulator acc[j][i][e]: output channel n = n0 + wn*WTN + j*16 + g*4 + e, pixel m = m0 + wm*WTM + i*16 + li
  if constexpr (DET) {
    // Detect head (models/yolo.py:52-57): stage logits + bias as fp32 [BM][BN] in LDS, then decode in
    // z order — for every anchor, BM consecutive pixels are BM consecutive 85-float rows of z — so
    // z (and raw) leave as fully coalesced 4-byte streams.  BN covers all na*no head channels.
    constexpr int DPITCH = BN * 4 + 16;
    static_assert(BM * DPITCH + BM * 16 <= LDS, "detect staging");
    float* Ds = reinterpret_cast<float*>(smem);
#pragma unroll
    for (int j = 0; j < TN; ++j) {
      const int col = wn * WTN + j * 16 + g * 4;
#pragma unroll
      for (int i = 0; i < TM; ++i) {
        const int row = wm * WTM + i * 16 + li;
        f4 v;
#pragma unroll
        for (int e = 0; e < 4; ++e) v[e] = acc[j][i][e] + ((n0 + col + e < p.cout) ? p.bias[n0 + col + e] : 0.0f);
        *reinterpret_cast<f4*>(reinterpret_cast<unsigned char*>(Ds) + row * DPITCH + col * 4) = v;
      }
    }
    // per-pixel table: z row of anchor 0 (int64), grid x / y
    unsigned char* tab = smem + BM * DPITCH;
    long long* zrow0 = reinterpret_cast<long long*>(tab);
    float* gxs = reinterpret_cast<float*>(tab + BM * 8);
    float* gys = gxs + BM;
    const int hw = p.Ho * p.Wo;
    if (tid < BM) {
      const int m = m0 + tid;
      const int mm = m < p.M ? m : p.M - 1;
      const int b = mm / hw, cell = mm - b * hw;
      const int gy = cell / p.Wo, gx = cell - gy * p.Wo;
      zrow0[tid] = m < p.M ? (long long)b * p.nrows + p.row_off + cell : -1;
      gxs[tid] = (float)gx;
      gys[tid] = (float)gy;
    }
    __syncthreads();
    // thread t walks e = t, t + NT, ... over the [BM][no] elements of one anchor: pr = e / no, o = e % no
    const int NO = p.no, step_pr = NT / NO, step_o = NT - step_pr * NO;
    for (int a = 0; a < p.na; ++a) {
      const float aw = p.anchor[2 * a], ah = p.anchor[2 * a + 1];
      const long long aoff = (long long)a * hw;
      int pr = tid / NO, o = tid - pr * NO;
      for (; pr < BM;) {
        const long long zr = zrow0[pr];
        if (zr >= 0) {
          const float v = *reinterpret_cast<const float*>(reinterpret_cast<const unsigned char*>(Ds) + pr * DPITCH +
                                                          (a * NO + o) * 4);
          const float sg = __builtin_amdgcn_rcpf(1.0f + __builtin_amdgcn_exp2f(-1.4426950408889634f * v));
          float out;
          if (o < 2) {
            out = (sg * 2.0f - 0.5f + (o == 0 ? gxs[pr] : gys[pr])) * p.stride;
          } else if (o < 4) {
            const float t2 = sg * 2.0f;
            out = (t2 * t2) * (o == 2 ? aw : ah);
          } else {
            out = sg;
          }
          p.z[(size_t)(zr + aoff) * NO + o] = out;
          if (p.raw) {
            const long long b = (zr - p.row_off) / p.nrows, cell = (zr - p.row_off) - b * p.nrows;
            p.raw[((size_t)(b * p.na + a) * hw + cell) * NO + o] = v;
          }
        }
        o += step_o;
        pr += step_pr;
        if (o >= NO) { o -= NO; ++pr; }
      }
    }
    return;
  }

  unsigned char* Cs = smem;
#pragma unroll
  for (int j = 0; j < TN; ++j) {
    const int col = wn * WTN + j * 16 + g * 4;
    float bias[4];
#pragma unroll
    for (int e = 0; e < 4; ++e) bias[e] = (n0 + col + e < p.cout) ? p.bias[n0 + col + e] : 0.0f;
#pragma unroll
    for (int i = 0; i < TM; ++i) {
      const int row = wm * WTM + i * 16 + li;
      typedef _Float16 h4 __attribute__((ext_vector_type(4)));
      h4 v;
#pragma unroll
      for (int e = 0; e < 4; ++e) v[e] = (_Float16)act_fn(acc[j][i][e] + bias[e], p.act);
      *reinterpret_cast<h4*>(Cs + row * CPITCH + col * 2) = v;
    }
  }
  __syncthreads();
  constexpr int CPR = BN * 2 / 16;
  _Float16* __restrict__ y = reinterpret_cast<_Float16*>(p.y);
  for (int cc = tid; cc < BM * CPR; cc += NT) {
    const int row = cc / CPR, ch = cc - row * CPR;
    const int m = m0 + row, n = n0 + ch * 8;
    if (m < p.M && n < p.cout)
      *reinterpret_cast<u4*>(y + (size_t)m * p.yc + p.yoff + n) = *reinterpret_cast<const u4*>(Cs + row * CPITCH + ch * 16);
  }
}

// ---------------------------------------------------------------------------------------------
// v3: LDS-DMA ring.  Operand tiles go global -> LDS with global_load_lds_dwordx4 (no VGPR staging),
// STAGES-deep ring, counted `s_waitcnt vmcnt` so STAGES-1 K steps stay in flight across the raw
// s_barrier (never __syncthreads in the loop: its fence would drain the DMA).  Each wave-instruction
// fills 8 tile rows (1 KiB, lane-linear), so the XOR swizzle is applied on the SOURCE chunk
// (c = slot ^ (row & 7)) and the ds_read side uses the same swz().  Padding taps and rows beyond
// M / cout read from a zeroed device page instead of being masked (LDS-DMA cannot zero-fill).
template <int BM, int BN, int WM, bool ONE, bool DET, int STAGES>
__global__ __launch_bounds__(NT, 1) void conv_f16_dma_kernel(const ConvParams p) {
  constexpr int WN = 4 / WM;
  constexpr int WTM = BM / WM, WTN = BN / WN;
  constexpr int TM = WTM / 16, TN = WTN / 16;
  constexpr int RA = BM / 32;            // A wave-instructions per wave per stage (8 rows each)
  constexpr int RB = (BN + 31) / 32;     // B wave-instructions per wave per stage
  constexpr int PER = RA + RB;           // vmcnt units per stage per thread
  constexpr int STAGE = (BM + BN) * ROWB;
  constexpr int CPITCH = BN * 2 + 16;
  constexpr int LDS = (STAGES * STAGE > BM * CPITCH) ? STAGES * STAGE : BM * CPITCH;
  __shared__ __attribute__((aligned(16))) unsigned char smem[LDS];

  const int tid = threadIdx.x;
  const int lane = tid & 63, wave = tid >> 6;
  const int wm = wave / WN, wn = wave % WN;
  const int g = lane >> 4, li = lane & 15;

  const int nwg = gridDim.x, bid = blockIdx.x;
  const int q = nwg >> 3, r = nwg & 7, xcd = bid & 7, loc = bid >> 3;
  const int wgid = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + loc;
  const int nN = (p.cout + BN - 1) / BN;
  const int m0 = (wgid / nN) * BM, n0 = (wgid % nN) * BN;

  const _Float16* __restrict__ x = reinterpret_cast<const _Float16*>(p.x);
  const _Float16* __restrict__ w = reinterpret_cast<const _Float16*>(p.w);
  const _Float16* zero = reinterpret_cast<const _Float16*>(p.zero);

  const int lr = lane >> 3;               // row within this wave's 8-row slab (== row & 7)
  const int c = (lane & 7) ^ lr;          // source chunk this lane fetches (swizzle on the source)

  const _Float16* a_ptr[RA];
  uint32_t a_mask[RA];
#pragma unroll
  for (int j = 0; j < RA; ++j) {
    const int m = m0 + j * 32 + wave * 8 + lr;
    const bool ok = m < p.M;
    const int mm = ok ? m : 0;
    if (ONE) {
      a_ptr[j] = x + (size_t)mm * p.xc + p.xoff;
      a_mask[j] = ok ? 1u : 0u;
    } else {
      const int hw = p.Ho * p.Wo;
      const int b = mm / hw, rem = mm - b * hw;
      const int ho = rem / p.Wo, wo = rem - ho * p.Wo;
      const int h0 = ho * p.s - p.pad, w0 = wo * p.s - p.pad;
      a_ptr[j] = x + ((ptrdiff_t)(b * p.H + h0) * p.W + w0) * p.xc + p.xoff;
      uint32_t mk = 0;
      for (int rr = 0; rr < p.k; ++rr)
        for (int ss = 0; ss < p.k; ++ss)
          if (ok && (unsigned)(h0 + rr) < (unsigned)p.H && (unsigned)(w0 + ss) < (unsigned)p.W)
            mk |= 1u << (rr * p.k + ss);
      a_mask[j] = mk;
    }
  }
  const _Float16* b_ptr[RB];
#pragma unroll
  for (int j = 0; j < RB; ++j) {
    const int row = j * 32 + wave * 8 + lr;
    const bool ok = row < BN && n0 + row < p.cout;
    b_ptr[j] = ok ? w + (size_t)(n0 + row) * p.kpad + c * 8 : nullptr;
  }

  const int nk = p.kpad / BKE;
  int ci = c * 8, tap = 0, rr = 0, ss = 0;
  if (!ONE) {
    while (ci >= p.cin) { ci -= p.cin; ++tap; if (++ss == p.k) { ss = 0; ++rr; } }
  }

  // issue the DMA of K step kt into ring slot `slot`
  auto issue = [&](int kt, int slot) {
    unsigned char* As = smem + slot * STAGE;
    unsigned char* Bs = As + BM * ROWB;
    const int k = kt * BKE + c * 8;
    const bool kin = k < p.K;
    if (ONE) {
#pragma unroll
      for (int j = 0; j < RA; ++j) {
        const _Float16* src = (a_mask[j] && kin) ? a_ptr[j] + k : zero;
        __builtin_amdgcn_global_load_lds((const void*)src,
                                         (__attribute__((address_space(3))) void*)(As + (j * 32 + wave * 8) * ROWB),
                                         16, 0, 0);
      }
    } else {
      const ptrdiff_t delta = ((ptrdiff_t)rr * p.W + ss) * p.xc + ci;
      const uint32_t bit = kin ? (1u << tap) : 0u;
#pragma unroll
      for (int j = 0; j < RA; ++j) {
        const _Float16* src = (a_mask[j] & bit) ? a_ptr[j] + delta : zero;
        __builtin_amdgcn_global_load_lds((const void*)src,
                                         (__attribute__((address_space(3))) void*)(As + (j * 32 + wave * 8) * ROWB),
                                         16, 0, 0);
      }
      ci += BKE;
      while (ci >= p.cin) { ci -= p.cin; ++tap; if (++ss == p.k) { ss = 0; ++rr; } }
    }
#pragma unroll
    for (int j = 0; j < RB; ++j) {
      const _Float16* src = b_ptr[j] ? b_ptr[j] + kt * BKE : zero;
      __builtin_amdgcn_global_load_lds((const void*)src,
                                       (__attribute__((address_space(3))) void*)(Bs + (j * 32 + wave * 8) * ROWB),
                                       16, 0, 0);
    }
  };

  f4 acc[TN][TM];
#pragma unroll
  for (int j = 0; j < TN; ++j)
#pragma unroll
    for (int i = 0; i < TM; ++i) acc[j][i] = f4{0.f, 0.f, 0.f, 0.f};

  // prologue: STAGES-1 steps in flight
#pragma unroll
  for (int s0 = 0; s0 < STAGES - 1; ++s0)
    if (s0 < nk) issue(s0, s0);

  int slot = 0;
  for (int kt = 0; kt < nk; ++kt) {
    // retire step kt: the loads issued after it (steps kt+1 .. kt+STAGES-2, if they exist) may stay in flight
    const int ahead = nk - 1 - kt;  // steps issued after kt so far (capped by STAGES-2)
    if (STAGES >= 3 && ahead >= 1) {
      if (STAGES >= 4 && ahead >= 2) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(2 * PER) : "memory");
      else asm volatile("s_waitcnt vmcnt(%0)" ::"n"(PER) : "memory");
    } else {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    __builtin_amdgcn_s_barrier();
    // refill the slot consumed one iteration ago (every wave has passed the barrier, so its reads are done)
    if (kt + STAGES - 1 < nk) {
      int fs = slot + STAGES - 1;
      if (fs >= STAGES) fs -= STAGES;
      issue(kt + STAGES - 1, fs);
    }
    const unsigned char* As = smem + slot * STAGE;
    const unsigned char* Bs = As + BM * ROWB;
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      const int ch = s * 4 + g;
      u4 xa[TM], wb[TN];
#pragma unroll
      for (int i = 0; i < TM; ++i) {
        const int row = wm * WTM + i * 16 + li;
        xa[i] = *reinterpret_cast<const u4*>(As + row * ROWB + swz(row, ch) * 16);
      }
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        const int row = wn * WTN + j * 16 + li;
        wb[j] = *reinterpret_cast<const u4*>(Bs + row * ROWB + swz(row, ch) * 16);
      }
#pragma unroll
      for (int j = 0; j < TN; ++j)
#pragma unroll
        for (int i = 0; i < TM; ++i)
          acc[j][i] = __builtin_amdgcn_mfma_f32_16x16x32_f16(__builtin_bit_cast(h8, wb[j]),
                                                             __builtin_bit_cast(h8, xa[i]), acc[j][i], 0, 0, 0);
    }
    if (++slot == STAGES) slot = 0;
  }
  asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
  __syncthreads();

  if (DET) {
    const int hw = p.Ho * p.Wo;
#pragma unroll
    for (int i = 0; i < TM; ++i) {
      const int m = m0 + wm * WTM + i * 16 + li;
      if (m >= p.M) continue;
      const int b = m / hw, rem = m - b * hw;
      const int gy = rem / p.Wo, gx = rem - gy * p.Wo;
#pragma unroll
      for (int j = 0; j < TN; ++j) {
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const int n = n0 + wn * WTN + j * 16 + g * 4 + e;
          if (n >= p.cout) continue;
          const int a = n / p.no, o = n - a * p.no;
          const float v = acc[j][i][e] + p.bias[n];
          const float sg = 1.0f / (1.0f + expf(-v));
          float out;
          if (o < 2) {
            const float t = sg * 2.0f;
            const float u = t - 0.5f;
            out = (u + ((o == 0) ? (float)gx : (float)gy)) * p.stride;
          } else if (o < 4) {
            const float t = sg * 2.0f;
            out = (t * t) * p.anchor[2 * a + (o - 2)];
          } else {
            out = sg;
          }
          const size_t cell = ((size_t)a * p.Ho + gy) * p.Wo + gx;
          p.z[(((size_t)b * p.nrows + p.row_off + cell) * p.no) + o] = out;
          if (p.raw) p.raw[(((size_t)b * p.na * hw) + cell) * p.no + o] = v;
        }
      }
    }
    return;
  }

  unsigned char* Cs = smem;
#pragma unroll
  for (int j = 0; j < TN; ++j) {
    const int col = wn * WTN + j * 16 + g * 4;
    float bias[4];
#pragma unroll
    for (int e = 0; e < 4; ++e) bias[e] = (n0 + col + e < p.cout) ? p.bias[n0 + col + e] : 0.0f;
#pragma unroll
    for (int i = 0; i < TM; ++i) {
      const int row = wm * WTM + i * 16 + li;
      typedef _Float16 h4 __attribute__((ext_vector_type(4)));
      h4 v;
#pragma unroll
      for (int e = 0; e < 4; ++e) v[e] = (_Float16)act_fn(acc[j][i][e] + bias[e], p.act);
      *reinterpret_cast<h4*>(Cs + row * CPITCH + col * 2) = v;
    }
  }
  __syncthreads();
  constexpr int CPR = BN * 2 / 16;
  _Float16* __restrict__ y = reinterpret_cast<_Float16*>(p.y);
  for (int cc = tid; cc < BM * CPR; cc += NT) {
    const int row = cc / CPR, ch = cc - row * CPR;
    const int m = m0 + row, n = n0 + ch * 8;
    if (m < p.M && n < p.cout)
      *reinterpret_cast<u4*>(y + (size_t)m * p.yc + p.yoff + n) = *reinterpret_cast<const u4*>(Cs + row * CPITCH + ch * 16);
  }
}

template <int BM, int BN, int WM, bool ONE, bool DET, int STAGES>
hipError_t launch_dma(const ConvParams& p, hipStream_t st) {
  const int nM = (p.M + BM - 1) / BM, nN = (p.cout + BN - 1) / BN;
  hipLaunchKernelGGL((conv_f16_dma_kernel<BM, BN, WM, ONE, DET, STAGES>), dim3(nM * nN), dim3(NT), 0, st, p);
  return hipGetLastError();
}

template <int BM, int BN, int WM, bool ONE, bool DET>
hipError_t launch_t(const ConvParams& p, hipStream_t st) {
  const int nM = (p.M + BM - 1) / BM, nN = (p.cout + BN - 1) / BN;
  hipLaunchKernelGGL((conv_f16_kernel<BM, BN, WM, ONE, DET>), dim3(nM * nN), dim3(NT), 0, st, p);
  return hipGetLastError();
}

}  // namespace

hipError_t launch_conv_f16(const ConvParams& p, bool det, hipStream_t st) {
  const bool one = p.k == 1 && p.s == 1 && p.pad == 0;
  static const int env_variant = [] { const char* e = getenv("YV7_CONV_F16"); return e ? atoi(e) : 0; }();
  const int variant = p.variant ? p.variant : env_variant;
  if (variant == 3 && p.zero) {
    if (det) return launch_dma<128, 128, 2, true, true, 3>(p, st);
    if (p.cout <= 32) return one ? launch_dma<256, 32, 4, true, false, 3>(p, st) : launch_dma<256, 32, 4, false, false, 3>(p, st);
    if (p.cout <= 64) return one ? launch_dma<256, 64, 4, true, false, 3>(p, st) : launch_dma<256, 64, 4, false, false, 3>(p, st);
    return one ? launch_dma<128, 128, 2, true, false, 3>(p, st) : launch_dma<128, 128, 2, false, false, 3>(p, st);
  }
  if (det) return launch_t<64, 256, 1, true, true>(p, st);
  if (variant == 2) {  // tall tiles for narrow layers
    if (p.cout <= 32) return one ? launch_t<256, 32, 4, true, false>(p, st) : launch_t<256, 32, 4, false, false>(p, st);
    if (p.cout <= 64) return one ? launch_t<256, 64, 4, true, false>(p, st) : launch_t<256, 64, 4, false, false>(p, st);
  }
  if (p.cout <= 32) return one ? launch_t<128, 32, 4, true, false>(p, st) : launch_t<128, 32, 4, false, false>(p, st);
  if (p.cout <= 64) return one ? launch_t<128, 64, 2, true, false>(p, st) : launch_t<128, 64, 2, false, false>(p, st);
  return one ? launch_t<128, 128, 2, true, false>(p, st) : launch_t<128, 128, 2, false, false>(p, st);
}

}  // namespace yv7
