// 1x1 / stride-1 fp16 convolution with the layer's WEIGHTS RESIDENT IN VGPRs — the short-K pointwise
// convs of the ELAN stacks whose cin is 128, 256 or 512 (Conv(c1, c2, 1, 1) in Conv.fuseforward,
// models/common.py:110-111; cfg/deploy/yolov7.yaml:22-23, 30, 35-36, ...: 128->128 / 256->256 @160,
// 256->256 / 512->128 / 512->256 @80 at bs 32).  y = act(x W'^T + b').
//
// Why (round 5): these layers are HBM-bound (1x1 256->256 @160 moves 838 MB for 107 GFLOP) but ran at
// 0.54-0.59 of their HBM roof on the LDS-DMA rings, which re-stage a weight tile for every output tile
// (as many L2 -> LDS bytes as the activations) and run the tile epilogue (the SiLU of every output, about
// the MFMA time at K = 256) with every wave of the block at once.  Here, as in conv_s2.hip:
//  * the block's N slice of the weights lives in VGPRs for the whole persistent launch (wave (ng, pg)
//    keeps TN x NCH fragments of 16 channels x 32 K, <= 128 VGPRs), loaded once from the fragment-packed
//    copy (pack_frag, 1 tap);
//  * activations stream: a tile is TPX = PG x TPF x 16 consecutive output pixels, its input rows DMA'd
//    (buffer_load ... lds, 8 whole 128-byte lines per piece = one 64-channel chunk of 8 pixels) into an
//    NS-slot LDS ring one chunk per interval, issued spread over the interval's K steps, L = NS - 1 - STG
//    chunks ahead; every pixel-fragment read feeds TN MFMAs (K 256: 4, 0.25 reads per MFMA);
//  * a pixel's 128 bytes are 8 16-byte positions, K-step half h's part g at (4 h + g) ^ ((px >> 1) & 7):
//    conflict-free ds_read_b128 for the MFMA B operand (16 consecutive pixels; checked against the gfx950
//    lane groups, scripts/w1_swizzle_check.py); the swizzle is on the DMA's per-lane source address;
//  * STG > 0: waves 4-7 run STG intervals behind waves 0-3 (a SIMD hosts w and w + 4), so one group's
//    tile epilogue issues beside the other group's MFMAs.
// Pixel m -> bordered NHWC index: m + 2 r + (2 b + 1)(W + 2) + 1, r = m / W, b = r / H (float reciprocal
// with an exact integer correction; M < 2^24).
#include "yv7_kernels.h"

namespace yv7 {

namespace {

constexpr int DC = 64;          // channels per DMA chunk (one 128-byte line per pixel; two MFMA K steps)
constexpr uint32_t OOB = 0x80000000u;

template <int N>
__device__ __forceinline__ void vmwait() {
  static_assert(N >= 0 && N < 64, "vmcnt range");
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

__device__ __forceinline__ void dma16(__amdgpu_buffer_rsrc_t r, void* lds, uint32_t vo, uint32_t so) {
  __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (__attribute__((address_space(3))) void*)lds, 16, vo, so, 0, 0);
}

// bordered pixel index of output pixel m (H, W: the tensor's interior size; rW = 1 / W, rH = 1 / H)
__device__ __forceinline__ uint32_t bpix(int m, int H, int W, float rW, float rH) {
  int r = (int)((float)m * rW);
  if ((r + 1) * W <= m) ++r;
  if (r * W > m) --r;
  int b = (int)((float)r * rH);
  if ((b + 1) * H <= r) ++b;
  if (b * H > r) --b;
  return (uint32_t)(m + 2 * r + (2 * b + 1) * (W + 2) + 1);
}

template <int NCH, int TN, int TPF, int PG, int NG, int NS, int STG, int IC>
struct W1Geo {
  static_assert(NG * PG == 8, "eight waves");
  static_assert(NCH % 2 == 0 && TN * NCH <= 32, "whole DMA chunks, <= 128 weight VGPRs");
  static constexpr int NDC = NCH / 2;            // DMA chunks per tile
  static_assert(NDC % IC == 0, "whole intervals per tile");
  static constexpr int NIV = NDC / IC;           // intervals per tile
  static constexpr int TPX = PG * TPF * 16;      // pixels per tile
  static_assert((IC * TPX) % 64 == 0, "whole DMA pieces per wave");
  static constexpr int PPC = TPX / 8;            // 1 KiB pieces per chunk (8 pixels each)
  static constexpr int PW = IC * TPX / 64;       // pieces per wave per interval
  static constexpr int SB = IC * TPX * 128;      // bytes per ring slot (IC chunks, chunk-major)
  static_assert(NS * SB + NG * TN * 64 <= 160 * 1024, "LDS budget");
  static constexpr int L = NS - 1 - STG;         // DMA lead in intervals
  static_assert(L >= 1 && L <= 8 && STG >= 0 && STG <= 3, "lead, stagger");
  static constexpr int BN = NG * TN * 16;
  static constexpr int NST = TN % 2 == 0 ? TPF * TN / 2 : TPF * TN;   // epilogue stores per wave per tile
};

// wave = pg * NG + ng; group = wave >> 2.  Tile = TPX consecutive output pixels x the block's BN channels;
// an interval (one barrier) covers IC DMA chunks (IC = NDC: the whole tile, so a stagger of one interval
// puts one group's tile epilogue beside the other group's whole tile of MFMAs).
// HOOK (convbench only, variants 299-301 on cfg 1; the ABI never accepts them): 2 = no DMA, 3 = no
// epilogue (a store under a condition that never holds keeps the MFMAs), 4 = DMA, waits, barriers only.
template <int NCH, int TN, int TPF, int PG, int NG, int NS, int STG, int IC, int ACT, int HOOK = 0>
__global__ __launch_bounds__(512, 2) void conv1x1_rw_kernel(const ConvParams p, int nN) {
  using G = W1Geo<NCH, TN, TPF, PG, NG, NS, STG, IC>;
  __shared__ __attribute__((aligned(16))) unsigned char smem[NS * G::SB + G::BN * 4];
  float* bias_l = reinterpret_cast<float*>(smem + NS * G::SB);

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int ng = wave % NG, pg = wave / NG, grp = STG ? (wave >> 2) : 0;
  const int g = lane >> 4, li = lane & 15;

  const int b = blockIdx.x, Gd = gridDim.x;
  const int nt = (b / 8) % nN;
  const int vb = (b / (8 * nN)) * 8 + b % 8, vG = Gd / nN;
  const int T = (p.M + G::TPX - 1) / G::TPX;
  const TileWalk tw = xcd_tile_walk_g(T, vG, vb);
  const int ntl = tw.count();
  if (ntl == 0) return;   // (uniform over the block)
  const int n0 = nt * G::BN;
  const float rW = 1.0f / (float)p.Wo, rH = 1.0f / (float)p.Ho;

  const auto xr = make_rsrc(p.x, p.xbytes);
  const auto wr = make_rsrc(p.wf, p.wfbytes);
  const auto yr = make_rsrc(p.y, 0x7fffffffu);

  // ---- resident weights: fragment (nf, K step c) at (nf * NCH + c) KiB, lane-linear
  u4 wreg[TN][NCH];
#pragma unroll
  for (int j = 0; j < TN; ++j) {
    const uint32_t base = (uint32_t)((n0 / 16 + ng * TN + j) * NCH * 1024 + lane * 16);
#pragma unroll
    for (int c = 0; c < NCH; ++c)
      wreg[j][c] = __builtin_bit_cast(u4, __builtin_amdgcn_raw_buffer_load_b128(wr, base, (uint32_t)(c * 1024), 0));
  }
  // bias: the block's slice in LDS (re-read at every tile start rather than held in 4 TN VGPRs; a global
  // load there would sit behind the in-flight DMA in vmcnt order and drain the ring)
  for (int i = tid; i < G::BN; i += 512) bias_l[i] = n0 + i < p.cout ? p.bias[n0 + i] : 0.0f;
  f4 acc[TN][TPF];
  auto init_acc = [&]() __attribute__((always_inline)) {
#pragma unroll
    for (int j = 0; j < TN; ++j) {
      const f4 bv = *reinterpret_cast<const f4*>(bias_l + ng * TN * 16 + j * 16 + g * 4);
#pragma unroll
      for (int f = 0; f < TPF; ++f) acc[j][f] = bv;
    }
  };

  // ---- DMA: interval v = (tile v / NIV, chunks (v % NIV) * IC ..); piece k = wave + 8 m of the interval:
  // chunk k / PPC, pixels 8 (k % PPC) .. + 7; lane -> pixel 8 (k % PPC) + lane / 8, LDS position lane % 8
  // = source part (lane % 8) ^ ((px >> 1) & 7) of the chunk's 128-byte line
  const uint32_t xoffb = (uint32_t)p.xoff * 2, pitch = (uint32_t)p.xc * 2;
  uint32_t src[G::PW];   // per-lane source offsets of the tile's pieces (chunk within the interval folded in)
  auto set_tile = [&](int it) __attribute__((always_inline)) {
    const int m0 = it < ntl ? tw.at(it) * G::TPX : p.M;
#pragma unroll
    for (int mm = 0; mm < G::PW; ++mm) {
      const int k = wave + 8 * mm;
      const int px = (k % G::PPC) * 8 + (lane >> 3);
      const int m = m0 + px;
      src[mm] = m < p.M ? bpix(m, p.Ho, p.Wo, rW, rH) * pitch + xoffb + (uint32_t)((k / G::PPC) * DC * 2) +
                              (uint32_t)(((lane & 7) ^ ((px >> 1) & 7)) * 16)
                        : OOB;
    }
  };
  int v_it = -1;
  auto issue_part = [&](int v, int m0p, int m1p) __attribute__((always_inline)) {
    if constexpr (HOOK == 2) return;
    const int it = v / G::NIV, iv = v - it * G::NIV;
    if (it != v_it) {
      set_tile(it);
      v_it = it;
    }
    unsigned char* dst = smem + (v % NS) * G::SB + wave * 1024;
#pragma unroll
    for (int mm = 0; mm < G::PW; ++mm)
      if (mm >= m0p && mm < m1p) dma16(xr, dst + mm * 8 * 1024, src[mm], (uint32_t)(iv * IC * DC * 2));
  };

  // ---- reads: chunk ci of the slot, px = pg * TPF * 16 + f * 16 + li; half h's part g at
  // (4 h + g) ^ ((li >> 1) & 7)
  uint32_t a_off[2];
#pragma unroll
  for (int h = 0; h < 2; ++h)
    a_off[h] = (uint32_t)((pg * TPF * 16 + li) * 128 + (((4 * h + g) ^ ((li >> 1) & 7)) * 16));

  // one interval: IC chunks x 2 K steps; the DMA of interval vn goes out in 2 IC parts, one per K step
  auto compute = [&](int v, int iv, int vn) __attribute__((always_inline)) {
    const unsigned char* pb = smem + (v % NS) * G::SB;
#pragma unroll
    for (int ci = 0; ci < IC; ++ci)
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const int t2 = ci * 2 + h;
        issue_part(vn, t2 * G::PW / (2 * IC), (t2 + 1) * G::PW / (2 * IC));
        const int c = (iv * IC + ci) * 2 + h;
        u4 xa[TPF];
#pragma unroll
        for (int f = 0; f < TPF; ++f) xa[f] = *reinterpret_cast<const u4*>(pb + ci * G::TPX * 128 + a_off[h] + f * 16 * 128);
#pragma unroll
        for (int f = 0; f < TPF; ++f)
#pragma unroll
          for (int j = 0; j < TN; ++j)
            acc[j][f] = __builtin_amdgcn_mfma_f32_16x16x32_f16(__builtin_bit_cast(h8, wreg[j][c]),
                                                               __builtin_bit_cast(h8, xa[f]), acc[j][f], 0, 0, 0);
      }
  };
  const uint32_t lane_ch = (uint32_t)(16 * (g & 1) + 8 * (g >> 1));
  auto epilogue = [&](int it) __attribute__((always_inline)) {
    const int m0 = tw.at(it) * G::TPX + pg * TPF * 16 + li;
#pragma unroll
    for (int f = 0; f < TPF; ++f) {
      const int m = m0 + f * 16;
      const bool live = m < p.M;
      const uint32_t yo = live ? (uint32_t)((bpix(m, p.Ho, p.Wo, rW, rH) * p.yc + p.yoff) * 2) : OOB;
      typedef _Float16 h4 __attribute__((ext_vector_type(4)));
      typedef uint32_t u2 __attribute__((ext_vector_type(2)));
      if constexpr (TN % 2 == 0) {
#pragma unroll
        for (int mp = 0; mp < TN / 2; ++mp) {
          h4 va, vb;
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            va[e] = (_Float16)act_t<ACT>(acc[2 * mp][f][e]);
            vb[e] = (_Float16)act_t<ACT>(acc[2 * mp + 1][f][e]);
          }
          const u2 a = __builtin_bit_cast(u2, va), bb = __builtin_bit_cast(u2, vb);
          const auto s0 = __builtin_amdgcn_permlane16_swap(a[0], bb[0], false, false);
          const auto s1 = __builtin_amdgcn_permlane16_swap(a[1], bb[1], false, false);
          const u4 vv = {s0[0], s1[0], s0[1], s1[1]};
          const int n = n0 + ng * TN * 16 + mp * 32 + (int)lane_ch;
          __builtin_amdgcn_raw_buffer_store_b128(vv, yr, (live && n < p.cout) ? yo + (uint32_t)n * 2 : 0xffffffffu, 0, 0);
        }
      } else {
#pragma unroll
        for (int j = 0; j < TN; ++j) {
          h4 va;
#pragma unroll
          for (int e = 0; e < 4; ++e) va[e] = (_Float16)act_t<ACT>(acc[j][f][e]);
          const int n = n0 + ng * TN * 16 + j * 16 + g * 4;
          __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(u2, va), yr,
                                                (live && n < p.cout) ? yo + (uint32_t)n * 2 : 0xffffffffu, 0, 0);
        }
      }
    }
  };
  auto barrier = [&]() __attribute__((always_inline)) {
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
  };
  // vmcnt before the barrier that ends interval v: the pieces of the interval the next barrier opens
  // (issued L - 1 intervals ago) landed; younger: the L - 1 later piece batches and the epilogue stores of
  // intervals v - L + 1 .. v that ended a tile (intervals before the first do not exist)
  // (hooks: 3 / 4 issue no epilogue stores and 2 no DMA pieces, so those terms are 0 there — ADVICE r5: a
  // looser count would let a wave past the barrier before its pieces landed and time a racy ring)
  auto wait_next = [&](int v) __attribute__((always_inline)) {
    constexpr int LB = HOOK == 2 ? 0 : G::PW * (G::L - 1);
    constexpr int NSTW = (HOOK == 3 || HOOK == 4) ? 0 : G::NST;
    int ends = 0;
#pragma unroll
    for (int d = 0; d < G::L; ++d) {
      const int vv = v - d;
      if (vv >= 0 && vv % G::NIV == G::NIV - 1) ++ends;
    }
    if (ends == 0) vmwait<LB>();
    else if (ends == 1) vmwait<(LB + NSTW < 63 ? LB + NSTW : 63)>();
    else if (ends == 2) vmwait<(LB + 2 * NSTW < 63 ? LB + 2 * NSTW : 63)>();
    else vmwait<(LB + 3 * NSTW < 63 ? LB + 3 * NSTW : 63)>();
  };

  // ---- prologue
#pragma unroll
  for (int v = 0; v < G::L; ++v) issue_part(v, 0, G::PW);
  vmwait<G::PW * (G::L - 1)>();
  barrier();
  if (STG && grp == 1) {   // group 1 runs STG intervals behind, issuing intervals L .. L + STG - 1 meanwhile
#pragma unroll
    for (int t = 0; t < STG; ++t) {
      issue_part(G::L + t, 0, G::PW);
      vmwait<G::PW * (G::L - 1)>();
      barrier();
    }
  }
  const int ahead = G::L + STG * grp;
  for (int it = 0; it < ntl; ++it) {
    init_acc();
#pragma unroll
    for (int iv = 0; iv < G::NIV; ++iv) {
      const int v = it * G::NIV + iv;
      if constexpr (HOOK == 4) issue_part(v + ahead, 0, G::PW);
      else compute(v, iv, v + ahead);
      if (iv == G::NIV - 1) {
#pragma unroll
        for (int j = 0; j < TN; ++j)
#pragma unroll
          for (int f = 0; f < TPF; ++f) asm volatile("" : "+v"(acc[j][f]));
        if constexpr (HOOK == 3 || HOOK == 4) {
          if (p.cout < 0) epilogue(it);
        } else {
          epilogue(it);
        }
      }
      wait_next(v);
      barrier();
    }
  }
  if (STG && grp == 0) {
#pragma unroll
    for (int t = 0; t < STG; ++t) barrier();
  }
  vmwait<0>();
}

// configurations (variants 290 + row for rows 0-5, 296 + row for rows 6-7): {NCH, TN, TPF, PG, NG, NS,
// STG, IC}.  0-2: an interval per 64-channel chunk (cin 128 / 256 / 512), no stagger; 3-5: an interval per
// tile, stagger 1; 6-7: cin 256 with a 128-channel N slice (cfg 3's is 256: half its waves would compute
// masked channels of a 128-output layer).
#define W1_CFGS(X)                                                                                             \
  X(0, 4, 8, 2, 8, 1, 4, 0, 1) X(1, 8, 4, 4, 2, 4, 8, 0, 1) X(2, 16, 2, 4, 2, 4, 8, 0, 1) X(3, 8, 4, 2, 2, 4, 4, 1, 4) \
  X(4, 4, 8, 1, 8, 1, 4, 1, 2) X(5, 16, 2, 2, 1, 8, 4, 1, 8) X(6, 8, 4, 1, 4, 2, 4, 1, 4) X(7, 8, 2, 2, 2, 4, 4, 1, 4)
#define W1_ROW(i, nch, tn, tpf, pg, ng, ns, stg, ic) {nch, tn, tpf, pg, ng, ns, stg, ic},
constexpr int W1_CFG[][8] = {W1_CFGS(W1_ROW)};
constexpr int W1_NCFG = sizeof(W1_CFG) / sizeof(W1_CFG[0]);

template <int NCH, int TN, int TPF, int PG, int NG, int NS, int STG, int IC, int HOOK = 0>
hipError_t launch_cfg(const ConvParams& p, int cus, hipStream_t st) {
  using G = W1Geo<NCH, TN, TPF, PG, NG, NS, STG, IC>;
  const int nN = (p.cout + G::BN - 1) / G::BN;
  const long T = ((long)p.M + G::TPX - 1) / G::TPX;
  long per = cus / (8 * nN);
  const long need = (T + 7) / 8;
  if (per > need) per = need;
  if (per < 1) per = 1;
  const int grid = (int)(per * 8 * nN);
  if (HOOK) {
    YV7_LAUNCH((conv1x1_rw_kernel<NCH, TN, TPF, PG, NG, NS, STG, IC, 1, HOOK>), dim3(grid), dim3(512), 0, st, p, nN);
    return hipGetLastError();
  }
  if (p.act == 1)
    YV7_LAUNCH((conv1x1_rw_kernel<NCH, TN, TPF, PG, NG, NS, STG, IC, 1>), dim3(grid), dim3(512), 0, st, p, nN);
  else if (p.act == 2)
    YV7_LAUNCH((conv1x1_rw_kernel<NCH, TN, TPF, PG, NG, NS, STG, IC, 2>), dim3(grid), dim3(512), 0, st, p, nN);
  else
    YV7_LAUNCH((conv1x1_rw_kernel<NCH, TN, TPF, PG, NG, NS, STG, IC, 0>), dim3(grid), dim3(512), 0, st, p, nN);
  return hipGetLastError();
}

}  // namespace

bool w1_supported(const ConvParams& p, int cfg) {
  if (cfg < 0 || cfg >= W1_NCFG) return false;
  return p.wf && p.k == 1 && p.s == 1 && p.pad == 0 && !p.pool && p.cin == W1_CFG[cfg][0] * 32 &&
         p.H == p.Ho && p.W == p.Wo && (long)p.M < (1L << 24) && p.cout % 16 == 0 && p.cout <= 1024 &&
         p.xoff % 8 == 0 && p.xc % 8 == 0 && p.yoff % 8 == 0 && p.yc % 8 == 0;
}

hipError_t launch_conv_w1(const ConvParams& p, int cfg, int cus, hipStream_t st) {
  if (!w1_supported(p, cfg)) return hipErrorInvalidValue;
  if (p.act == 1 && cfg == 1 && p.variant >= 299 && p.variant <= 301) {   // hooks (convbench)
    if (p.variant == 299) return launch_cfg<8, 4, 4, 2, 4, 8, 0, 1, 2>(p, cus, st);
    if (p.variant == 300) return launch_cfg<8, 4, 4, 2, 4, 8, 0, 1, 3>(p, cus, st);
    return launch_cfg<8, 4, 4, 2, 4, 8, 0, 1, 4>(p, cus, st);
  }
  switch (cfg) {
#define W1_CASE(i, nch, tn, tpf, pg, ng, ns, stg, ic) \
  case i: return launch_cfg<nch, tn, tpf, pg, ng, ns, stg, ic>(p, cus, st);
    W1_CFGS(W1_CASE)
#undef W1_CASE
  }
  return hipErrorInvalidValue;
}

}  // namespace yv7
