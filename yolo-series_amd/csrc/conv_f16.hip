// fp16 implicit-GEMM convolution for gfx950 (the bench / serving path), bordered NHWC activations,
// KRSC weights.
//
// Replaces ATen conv2d + BN-folded bias + SiLU/LeakyReLU (Conv.fuseforward models/common.py:110-111,
// RepConv deploy common.py:498-500) and the Detect head conv + decode (models/yolo.py:46-57).
//
// GEMM view: M = B*Ho*Wo pixels, N = cout, K = k*k*cin ordered (r, s, ci).
//  * K step 64 (128 bytes per tile row), two v_mfma_f32_16x16x32_f16 sub-steps per tile per step;
//  * operands come in through raw buffer loads: each tile row (an output pixel's receptive-field
//    origin in the bordered input, or a weight row) is a per-lane byte offset computed once, the K
//    step's tap / channel position is a scalar offset (cin % 64 == 0: a K step never straddles two
//    taps), and the zero frame around every image replaces the padding tests — the K loop spends no
//    vector instructions on addressing.  Rows past M / cout land beyond the buffer range: zeros;
//  * LDS rows of 8 x 16-byte chunks, chunk index XOR-swizzled with (row & 7) so the 16-lane groups
//    of ds_read_b128 hit distinct 16-byte slots;
//  * operands swapped (weights as the MFMA A operand) so each lane's accumulator holds 4
//    consecutive output channels of one pixel: the epilogue packs them into 8-byte LDS writes, and
//    the tile leaves as full 16-byte NHWC row chunks into the output's channel slice (zero-copy concat);
//  * accumulators start at the bias; the activation is a compile-time constant in the epilogue;
//  * XCD-aware bijective block remap: consecutive tiles (all N tiles of an M tile) share an XCD's L2.
// Two main loops: the 4-wave register-staged tile kernel (2-3 blocks per CU, any width) and the
// 8-wave LDS-DMA ring for wide layers.
#include <cstdlib>
#include <type_traits>

#include "yv7_kernels.h"

namespace yv7 {

namespace {

constexpr int NT = 256;
constexpr int BKE = 64;    // K elements per step
constexpr int ROWB = 128;  // LDS bytes per tile row
constexpr uint32_t OOB = 0x80000000u;  // a buffer offset past every tensor: the load returns zeros

__device__ __forceinline__ int swz(int row, int chunk) { return chunk ^ (row & 7); }

// 16 bytes per lane from a buffer straight into LDS (lane-linear at the wave-uniform `lds` base)
__device__ __forceinline__ void dma16(__amdgpu_buffer_rsrc_t r, void* lds, uint32_t vo, uint32_t so) {
  __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (__attribute__((address_space(3))) void*)lds, 16, vo, so, 0, 0);
}

// Output pixel m -> (b, ho, wo) once, then stepped: rows a thread moves are `step` pixels apart.
// Rows past M walk into image B, whose offsets lie beyond the input buffer (zeros).
struct PixelWalk {
  int b, ho, wo;
  __device__ __forceinline__ PixelWalk(const ConvParams& p, int m) {
    const int hw = p.Ho * p.Wo;
    b = m / hw;
    const int rem = m - b * hw;
    ho = rem / p.Wo;
    wo = rem - ho * p.Wo;
  }
  __device__ __forceinline__ void advance(const ConvParams& p, int step) {
    wo += step;
    while (wo >= p.Wo) {
      wo -= p.Wo;
      if (++ho == p.Ho) { ho = 0; ++b; }
    }
  }
};

// Byte offset in the bordered input of output pixel (b, ho, wo)'s receptive-field origin (tap 0,0),
// channel xoff + 8 * chunk.
__device__ __forceinline__ uint32_t a_origin(const ConvParams& p, int b, int ho, int wo, int chunk) {
  return (uint32_t)((pix_index(b, ho * p.s - p.pad, wo * p.s - p.pad, p.H, p.W) * p.xc + p.xoff + chunk * 8) * 2);
}

// The K-step cursor: tap (rr, ss) and channel ci of a K position, advanced 64 at a time.
struct KCursor {
  int ci, rr, ss, tap;
  __device__ __forceinline__ void init(const ConvParams& p, int k) {
    ci = k; rr = ss = tap = 0;
    while (ci >= p.cin) { ci -= p.cin; ++tap; if (++ss == p.k) { ss = 0; ++rr; } }
  }
  __device__ __forceinline__ void advance(const ConvParams& p) {
    ci += BKE;
    while (ci >= p.cin) { ci -= p.cin; ++tap; if (++ss == p.k) { ss = 0; ++rr; } }
  }
  // byte offset of (rr, ss, ci) relative to the receptive-field origin
  __device__ __forceinline__ uint32_t offset(const ConvParams& p) const {
    return (uint32_t)(((rr * (p.W + 2 * BORDER) + ss) * p.xc + ci) * 2);
  }
};

// A-operand source of one K step for RA rows: uniform case (1x1, or cin % 64 == 0) = per-row offset
// + scalar step offset; otherwise per-lane tap tracking (cin of 8..56: tiny's narrow layers).
template <bool ONE, int RA>
struct AWalk {
  uint32_t off[RA];   // row origin + this lane's chunk
  KCursor su;         // uniform cursor (k = kt*64)
  KCursor ln;         // per-lane cursor (k = kt*64 + chunk*8), non-uniform case only
  bool uni;
  int c16;
  __device__ __forceinline__ void init(const ConvParams& p, int chunk) {
    uni = ONE || (p.cin & 63) == 0;
    c16 = chunk * 16;
    su.init(p, 0);
    if (!uni) ln.init(p, chunk * 8);
  }
  // voffset / soffset of row j for step kt (call step() once per K step, in order)
  template <typename F>
  __device__ __forceinline__ void step(const ConvParams& p, int kt, F&& load) {
    if (ONE) {
      const uint32_t so = (uint32_t)kt * BKE * 2;
      if ((kt + 1) * BKE <= p.K) {
#pragma unroll
        for (int j = 0; j < RA; ++j) load(j, off[j], so);
      } else {   // ragged last step (cin % 64 != 0): lanes past K read zeros
        const bool kin = kt * BKE + c16 / 2 < p.K;
#pragma unroll
        for (int j = 0; j < RA; ++j) load(j, kin ? off[j] : OOB, so);
      }
    } else if (uni) {
      const uint32_t so = su.offset(p);
      su.advance(p);
#pragma unroll
      for (int j = 0; j < RA; ++j) load(j, off[j], so);
    } else {
      const bool kin = kt * BKE + c16 / 2 < p.K;
      const uint32_t d = ln.offset(p) - (uint32_t)c16;
      ln.advance(p);
#pragma unroll
      for (int j = 0; j < RA; ++j) load(j, kin ? off[j] + d : OOB, 0u);
    }
  }
};

template <int BM, int BN, int WM, bool ONE, bool DET, int PF = 1>
__global__ __launch_bounds__(NT, 2) void conv_f16_kernel(const ConvParams p) {
  constexpr int WN = 4 / WM;
  constexpr int WTM = BM / WM, WTN = BN / WN;
  constexpr int TM = WTM / 16, TN = WTN / 16;
  constexpr int RA = BM / 32;                 // A rows per thread (32 rows per pass of 256 threads)
  constexpr int RB = (BN + 31) / 32;
  constexpr int STAGE = (BM + BN) * ROWB;
  constexpr int CPITCH = BN * 2 + 16;
  constexpr int EPI = BM * CPITCH + BM * 4;   // staged C tile + output row table
  constexpr int LDS = (2 * STAGE > EPI) ? 2 * STAGE : EPI;
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

  const auto xr = make_rsrc(p.x, p.xbytes);
  const auto wr = make_rsrc(p.w, p.wbytes);

  const int c = tid & 7;     // 16-byte chunk column this thread moves
  const int r0 = tid >> 3;   // first row this thread moves (then every 32nd)

  AWalk<ONE, RA> aw;
  aw.init(p, c);
  {
    PixelWalk pw(p, m0 + r0);
#pragma unroll
    for (int j = 0; j < RA; ++j) {
      if (j) pw.advance(p, 32);
      aw.off[j] = a_origin(p, pw.b, pw.ho, pw.wo, c);
    }
  }
  uint32_t b_off[RB];   // weight rows past cout_pad32 fall beyond the weight buffer (zeros)
#pragma unroll
  for (int j = 0; j < RB; ++j) b_off[j] = (uint32_t)(((n0 + r0 + 32 * j) * p.kpad + c * 8) * 2);

  const int nk = p.kpad / BKE;
  auto gload = [&](int kt, u4 (&ra)[RA], u4 (&rb)[RB]) {
    aw.step(p, kt, [&](int j, uint32_t vo, uint32_t so) {
      ra[j] = __builtin_bit_cast(u4, __builtin_amdgcn_raw_buffer_load_b128(xr, vo, so, 0));
    });
#pragma unroll
    for (int j = 0; j < RB; ++j)
      rb[j] = __builtin_bit_cast(u4, __builtin_amdgcn_raw_buffer_load_b128(wr, b_off[j], (uint32_t)kt * BKE * 2, 0));
  };
  auto lstore = [&](int buf, const u4 (&ra)[RA], const u4 (&rb)[RB]) {
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
      if (BN % 32 == 0 || row < BN) *reinterpret_cast<u4*>(Bs + row * ROWB + swz(row, c) * 16) = rb[j];
    }
  };

  // accumulators start at the bias (one VALU add per output element less in the epilogue)
  f4 acc[TN][TM];
#pragma unroll
  for (int j = 0; j < TN; ++j) {
    const int col = n0 + wn * WTN + j * 16 + g * 4;
    f4 bv;
#pragma unroll
    for (int e = 0; e < 4; ++e) bv[e] = col + e < p.cout ? p.bias[col + e] : 0.0f;
#pragma unroll
    for (int i = 0; i < TM; ++i) acc[j][i] = bv;
  }

  auto compute = [&](int buf) {
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
  };

  u4 ra[RA], rb[RB];
  gload(0, ra, rb);
  lstore(0, ra, rb);
  if constexpr (PF == 1) {
    __syncthreads();
    for (int kt = 0; kt < nk; ++kt) {
      if (kt + 1 < nk) gload(kt + 1, ra, rb);
      compute(kt & 1);
      if (kt + 1 < nk) lstore((kt & 1) ^ 1, ra, rb);
      __syncthreads();
    }
  } else {
    // two register sets: the loads of step kt+2 are issued before step kt's MFMAs and have two steps
    // of MFMA work (instead of one) to land before their LDS write
    u4 ra2[RA], rb2[RB];
    if (nk > 1) gload(1, ra2, rb2);
    __syncthreads();
    for (int kt = 0; kt < nk; kt += 2) {
      if (kt + 2 < nk) gload(kt + 2, ra, rb);
      compute(0);
      if (kt + 1 < nk) lstore(1, ra2, rb2);
      __syncthreads();
      if (kt + 1 >= nk) break;
      if (kt + 3 < nk) gload(kt + 3, ra2, rb2);
      compute(1);
      if (kt + 2 < nk) lstore(0, ra, rb);
      __syncthreads();
    }
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
        for (int e = 0; e < 4; ++e) v[e] = acc[j][i][e];
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
    // per-row NMS scores (yv7_row_best): objectness, first-max class score obj * cls_c, class — from
    // the same sigmoid values the z rows below receive
    if (p.best) {
      for (int t = tid; t < BM * p.na; t += NT) {
        const int pr = t % BM, a = t / BM;
        const long long zr = zrow0[pr];
        if (zr < 0) continue;
        const float* lg = reinterpret_cast<const float*>(reinterpret_cast<const unsigned char*>(Ds) + pr * DPITCH) +
                          a * p.no;
        auto sig = [](float v) { return __builtin_amdgcn_rcpf(1.0f + __builtin_amdgcn_exp2f(-1.4426950408889634f * v)); };
        const float obj = sig(lg[4]);
        float best = obj;
        int bc = 0;
        if (p.no > 6) {
          best = sig(lg[5]) * obj;
          for (int c = 1; c < p.no - 5; ++c) {
            const float v = sig(lg[5 + c]) * obj;
            if (v > best) { best = v; bc = c; }   // strict >: the first maximum wins (general.py:683-684)
          }
        }
        f4 rec;
        rec[0] = obj;
        rec[1] = best;
        rec[2] = __builtin_bit_cast(float, bc);
        rec[3] = 0.0f;
        *reinterpret_cast<f4*>(p.best + (size_t)(zr + (long long)a * hw) * 4) = rec;
      }
    }
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

  // output row table: element offset of each tile row's pixel in the bordered output (or ~0u past M)
  uint32_t* yrow = reinterpret_cast<uint32_t*>(smem + BM * CPITCH);
  if (tid < BM) {
    const int m = m0 + tid;
    uint32_t v = ~0u;
    if (m < p.M) {
      PixelWalk pw(p, m);
      v = (uint32_t)(pix_index(pw.b, pw.ho, pw.wo, p.Ho, p.Wo) * p.yc + p.yoff);
    }
    yrow[tid] = v;
  }
  unsigned char* Cs = smem;
  with_act(p.act, [&](auto actc) {
    constexpr int ACT = decltype(actc)::value;
#pragma unroll
    for (int j = 0; j < TN; ++j) {
      const int col = wn * WTN + j * 16 + g * 4;
#pragma unroll
      for (int i = 0; i < TM; ++i) {
        const int row = wm * WTM + i * 16 + li;
        typedef _Float16 h4 __attribute__((ext_vector_type(4)));
        h4 v;
#pragma unroll
        for (int e = 0; e < 4; ++e) v[e] = (_Float16)act_t<ACT>(acc[j][i][e]);
        *reinterpret_cast<h4*>(Cs + row * CPITCH + col * 2) = v;
      }
    }
  });
  __syncthreads();
  constexpr int CPR = BN * 2 / 16;
  _Float16* __restrict__ y = reinterpret_cast<_Float16*>(p.y);
  for (int cc = tid; cc < BM * CPR; cc += NT) {
    const int row = cc / CPR, ch = cc - row * CPR;
    const uint32_t yo = yrow[row];
    const int n = n0 + ch * 8;
    if (yo != ~0u && n < p.cout)
      *reinterpret_cast<u4*>(y + yo + n) = *reinterpret_cast<const u4*>(Cs + row * CPITCH + ch * 16);
  }
}

// ---------------------------------------------------------------------------------------------
// 8-wave LDS-DMA ring (wide layers).
//  * 512 threads = 8 waves (2 per SIMD, so one wave's fragment reads hide under the other's MFMAs),
//    BM x BN tile, BK = 64, STAGES-deep ring of LDS stages filled by buffer_load_dwordx4 ... lds —
//    no VGPR staging and no ds_write pass;
//  * each wave-instruction fills 8 tile rows (1 KiB, lane-linear in LDS), so the XOR swizzle is
//    applied on the SOURCE chunk (c = slot ^ (row & 7)) and the ds_read side uses the same swz();
//  * counted `s_waitcnt vmcnt(PER)` keeps the next stage in flight across a raw s_barrier (never
//    __syncthreads in the loop: its fence would drain the DMA); the stage refilled at step kt is the
//    one every wave finished reading at step kt-1 (its MFMAs consumed those reads before the barrier).
template <int BM, int BN, int WM, int WN, int STAGES, bool ONE>
__global__ __launch_bounds__(64 * WM * WN, (STAGES * (BM + BN) * 128 <= 80 * 1024) ? 2 : 1) void conv_f16_ring_kernel(const ConvParams p) {
  constexpr int NW = WM * WN, NTH = 64 * NW;
  constexpr int WTM = BM / WM, WTN = BN / WN;
  constexpr int TM = WTM / 16, TN = WTN / 16;
  constexpr int RA = BM / 8 / NW, RB = BN / 8 / NW;   // wave-instructions per wave per stage
  static_assert(RA * 8 * NW == BM && RB * 8 * NW == BN, "tile rows must split into 8-row groups per wave");
  constexpr int PER = RA + RB;
  constexpr int STAGE = (BM + BN) * ROWB;
  constexpr int CPITCH = BN * 2 + 16;
  constexpr int EPI = BM * CPITCH + BM * 4;
  constexpr int LDS = (STAGES * STAGE > EPI) ? STAGES * STAGE : EPI;
  static_assert(LDS <= 160 * 1024, "LDS budget");
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

  const auto xr = make_rsrc(p.x, p.xbytes);
  const auto wr = make_rsrc(p.w, p.wbytes);

  const int lr = lane >> 3;            // row within the 8-row group (== row & 7)
  const int c = (lane & 7) ^ lr;       // source chunk this lane fetches

  AWalk<ONE, RA> aw;
  aw.init(p, c);
  {
    PixelWalk pw(p, m0 + wave * 8 + lr);
#pragma unroll
    for (int j = 0; j < RA; ++j) {
      if (j) pw.advance(p, NW * 8);
      aw.off[j] = a_origin(p, pw.b, pw.ho, pw.wo, c);
    }
  }
  uint32_t b_off[RB];
#pragma unroll
  for (int j = 0; j < RB; ++j) b_off[j] = (uint32_t)(((n0 + (j * NW + wave) * 8 + lr) * p.kpad + c * 8) * 2);

  const int nk = p.kpad / BKE;
  auto issue = [&](int kt, int slot) {
    unsigned char* As = smem + slot * STAGE;
    unsigned char* Bs = As + BM * ROWB;
    aw.step(p, kt, [&](int j, uint32_t vo, uint32_t so) { dma16(xr, As + (j * NW + wave) * 8 * ROWB, vo, so); });
#pragma unroll
    for (int j = 0; j < RB; ++j) dma16(wr, Bs + (j * NW + wave) * 8 * ROWB, b_off[j], (uint32_t)kt * BKE * 2);
  };

  f4 acc[TN][TM];
#pragma unroll
  for (int j = 0; j < TN; ++j) {
    const int col = n0 + wn * WTN + j * 16 + g * 4;
    f4 bv;
#pragma unroll
    for (int e = 0; e < 4; ++e) bv[e] = col + e < p.cout ? p.bias[col + e] : 0.0f;
#pragma unroll
    for (int i = 0; i < TM; ++i) acc[j][i] = bv;
  }

#pragma unroll
  for (int s0 = 0; s0 < STAGES - 1; ++s0)
    if (s0 < nk) issue(s0, s0);

  int slot = 0;
  for (int kt = 0; kt < nk; ++kt) {
    // stage kt must have landed; the (at most STAGES-2) stages issued after it may stay in flight
    const int ahead = nk - 1 - kt;
    if (STAGES >= 4 && ahead >= 2) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(2 * PER) : "memory");
    else if (STAGES >= 3 && ahead >= 1) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(PER) : "memory");
    else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
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
      __builtin_amdgcn_s_setprio(1);
#pragma unroll
      for (int j = 0; j < TN; ++j)
#pragma unroll
        for (int i = 0; i < TM; ++i)
          acc[j][i] = __builtin_amdgcn_mfma_f32_16x16x32_f16(__builtin_bit_cast(h8, wb[j]),
                                                             __builtin_bit_cast(h8, xa[i]), acc[j][i], 0, 0, 0);
      __builtin_amdgcn_s_setprio(0);
    }
    if (++slot == STAGES) slot = 0;
  }
  asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
  __syncthreads();

  uint32_t* yrow = reinterpret_cast<uint32_t*>(smem + BM * CPITCH);
  for (int t = tid; t < BM; t += NTH) {
    const int m = m0 + t;
    uint32_t v = ~0u;
    if (m < p.M) {
      PixelWalk pw(p, m);
      v = (uint32_t)(pix_index(pw.b, pw.ho, pw.wo, p.Ho, p.Wo) * p.yc + p.yoff);
    }
    yrow[t] = v;
  }
  unsigned char* Cs = smem;
  with_act(p.act, [&](auto actc) {
    constexpr int ACT = decltype(actc)::value;
#pragma unroll
    for (int j = 0; j < TN; ++j) {
      const int col = wn * WTN + j * 16 + g * 4;
#pragma unroll
      for (int i = 0; i < TM; ++i) {
        const int row = wm * WTM + i * 16 + li;
        typedef _Float16 h4 __attribute__((ext_vector_type(4)));
        h4 v;
#pragma unroll
        for (int e = 0; e < 4; ++e) v[e] = (_Float16)act_t<ACT>(acc[j][i][e]);
        *reinterpret_cast<h4*>(Cs + row * CPITCH + col * 2) = v;
      }
    }
  });
  __syncthreads();
  constexpr int CPR = BN * 2 / 16;
  _Float16* __restrict__ y = reinterpret_cast<_Float16*>(p.y);
  for (int cc = tid; cc < BM * CPR; cc += NTH) {
    const int row = cc / CPR, ch = cc - row * CPR;
    const uint32_t yo = yrow[row];
    const int n = n0 + ch * 8;
    if (yo != ~0u && n < p.cout)
      *reinterpret_cast<u4*>(y + yo + n) = *reinterpret_cast<const u4*>(Cs + row * CPITCH + ch * 16);
  }
}

template <int BM, int BN, int WM, int WN, int STAGES, bool ONE>
hipError_t launch_ring(const ConvParams& p, hipStream_t st) {
  const int nM = (p.M + BM - 1) / BM, nN = (p.cout + BN - 1) / BN;
  hipLaunchKernelGGL((conv_f16_ring_kernel<BM, BN, WM, WN, STAGES, ONE>), dim3(nM * nN), dim3(64 * WM * WN), 0, st, p);
  return hipGetLastError();
}

template <int BM, int BN, int WM, int WN, int STAGES>
hipError_t launch_ring2(const ConvParams& p, bool one, hipStream_t st) {
  return one ? launch_ring<BM, BN, WM, WN, STAGES, true>(p, st) : launch_ring<BM, BN, WM, WN, STAGES, false>(p, st);
}

template <int BM, int BN, int WM, bool ONE, bool DET, int PF = 1>
hipError_t launch_t(const ConvParams& p, hipStream_t st) {
  const int nM = (p.M + BM - 1) / BM, nN = (p.cout + BN - 1) / BN;
  hipLaunchKernelGGL((conv_f16_kernel<BM, BN, WM, ONE, DET, PF>), dim3(nM * nN), dim3(NT), 0, st, p);
  return hipGetLastError();
}

}  // namespace

hipError_t launch_conv_f16(const ConvParams& p, bool det, hipStream_t st) {
  const bool one = p.k == 1 && p.s == 1 && p.pad == 0;
  static const int env_variant = [] { const char* e = getenv("YV7_CONV_F16"); return e ? atoi(e) : 0; }();
  const int variant = p.variant ? p.variant : env_variant;
  if (!det && p.cout > 32) {
    if ((variant == 0 || variant == 10) && halo_supported(p)) return launch_conv_halo(p, st);
    if (variant == 4) {
      if (p.cout <= 64) return launch_ring2<256, 64, 4, 2, 3>(p, one, st);
      return launch_ring2<256, 128, 4, 2, 3>(p, one, st);
    }
    if (variant == 5) {
      if (p.cout <= 64) return launch_ring2<512, 64, 8, 1, 2>(p, one, st);
      if (p.cout <= 128) return launch_ring2<256, 128, 4, 2, 2>(p, one, st);
      return launch_ring2<256, 256, 2, 4, 2>(p, one, st);
    }
    if (variant == 6) {
      if (p.cout <= 64) return launch_ring2<128, 64, 2, 2, 3>(p, one, st);
      return launch_ring2<128, 128, 2, 2, 2>(p, one, st);
    }
    if (variant == 7) {
      if (p.cout <= 64) return launch_ring2<128, 64, 2, 2, 4>(p, one, st);
      return launch_ring2<128, 128, 2, 2, 3>(p, one, st);
    }
    if (variant == 8) {
      if (p.cout <= 64) return one ? launch_t<128, 64, 2, true, false, 2>(p, st) : launch_t<128, 64, 2, false, false, 2>(p, st);
      return one ? launch_t<128, 128, 2, true, false, 2>(p, st) : launch_t<128, 128, 2, false, false, 2>(p, st);
    }
    if (variant == 0 && p.cout >= 256) {
      // wide layers: the 8-wave ring kernels win once their grid still covers the chip
      // (scripts/convbench.hip, bs 32: 3x3 256->256 @40 112 -> 80 us, 512->1024 @20 208 -> 142 us,
      // 1x1 512->512 @80 243 -> 216 us); 512->512 @20 has 100 256x256 tiles -> 256x128 (88 vs 102 us)
      const long mt = (p.M + 255) / 256;
      if (mt * ((p.cout + 255) / 256) >= 150) return launch_ring2<256, 256, 2, 4, 2>(p, one, st);
      if (mt * ((p.cout + 127) / 128) >= 150) return launch_ring2<256, 128, 4, 2, 3>(p, one, st);
    }
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
