// Persistent weight-stationary 3x3 / stride-1 / pad-1 convolution, 64 -> 64 channels, fp16, gfx950.
//
// Replaces Conv.fuseforward (models/common.py:110-111) for the 64-channel 3x3 layers of the yolov7
// backbone / head ELAN stacks (cfg/deploy/yolov7.yaml:17 at 320x320, :19-22 at 160x160 and the
// P3 head stack at 80x80) — ~11 % of the network's FLOPs on its largest activations.
//
// Why a third conv kernel: the implicit-GEMM kernels stream both operands for every 64-deep K step,
// so each CU pulls (BM + BN) x 128 B per step through the L2 -> CU path (~70 GB/s per CU), which
// caps narrow layers at a fraction of the MFMA rate; the halo kernel reloads the weights per tap.
// Here the whole layer's weights (9 taps x 64 x 64 fp16 = 72 KiB) are loaded into LDS ONCE per
// block and each block walks output tiles (persistent grid, one block per CU):
//  * per 16 x 16 output tile, the 18 x 18 x 64 input patch (bordered NHWC: the zero frame is the
//    padding) comes in by LDS-DMA (buffer_load ... lds), double-buffered: tile t+1's patch lands
//    while tile t computes;
//  * LDS images are XOR-swizzled in 16-byte chunks — weights by row (out channel) & 7, the patch by
//    patch column & 7 — so every ds_read_b128 of the tap loop is conflict-free and its address is a
//    per-lane base plus a compile-time offset (no address arithmetic in the loop);
//  * 4 waves (one per SIMD), each 4 output rows (64 pixels) x 64 channels: per 32-deep sub-step 4
//    weight + 4 patch fragments feed 16 v_mfma_f32_16x16x32_f16 (weights as the A operand, so a
//    lane's accumulator is 4 consecutive channels of one pixel); since round 4 the default runs 8
//    waves of 2 rows (two per SIMD, 256 VGPRs each instead of 450: NWV below);
//  * software-pipelined across tiles: tile t's epilogue (bias = accumulator init, compile-time
//    activation, fp16, v_permlane16_swap so each lane holds 8 consecutive channels, 16-byte stores
//    into the destination channel slice — zero-copy concat) is issued between tile t+1's MFMAs;
//  * fragment reads for the next super-step are issued among the current one's MFMAs
//    (sched_group_barrier pattern), so LDS latency stays off the MFMA pipe.
// LDS: 2 x 41 KiB patch buffers + 72 KiB weights = 154 KiB.
// Microbenchmark hooks (ConvParams::variant, scripts/convbench.hip): 12 no output stores, 13 no patch
// DMA, 14 no epilogue, 16 MFMA loop only.
#include <hip/hip_runtime.h>

#include <type_traits>

#include "yv7_kernels.h"

namespace yv7 {

namespace {

constexpr int NT = 256;
constexpr int TS = 16;                       // output tile side
constexpr int PS = TS + 2;                   // patch side
constexpr int PPIX = PS * PS;                // 324 patch pixels
constexpr int PGROUPS = (PPIX + 7) / 8;      // 41 DMA wave-instructions (8 pixels x 128 B) per patch
constexpr int PBUF = PGROUPS * 1024;         // 41,984 B per patch buffer
constexpr int CI = 64, CO = 64;
constexpr int WTAP = CO * CI * 2;            // 8 KiB of weights per tap
constexpr int LDS = 2 * PBUF + 9 * WTAP;     // 157,696 B
typedef uint32_t u2 __attribute__((ext_vector_type(2)));

__device__ __forceinline__ void dma16(__amdgpu_buffer_rsrc_t r, void* lds, uint32_t vo, uint32_t so) {
  __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (__attribute__((address_space(3))) void*)lds, 16, vo, so, 0, 0);
}

// The layer's weights -> LDS once per block: tap t, out channel n, 16-byte slot s holds K chunk
// s ^ (n & 7) of that tap.  A thread's 18 chunks go as two batches of 9 loads issued before their LDS
// writes (as a load -> write loop, hipcc waited out one L2 round trip per chunk: 18 in a row before
// the first patch DMA of every block).
template <int NTH = NT>
__device__ __forceinline__ void load_weights(const ConvParams& p, unsigned char* wl, int tid) {
  constexpr int NQ = 9 * CO * 8, IT = NQ / NTH, NB = 9;
  static_assert(NQ % NTH == 0 && IT % NB == 0, "whole batches of chunks per thread");
  const unsigned char* w = reinterpret_cast<const unsigned char*>(p.w);
#pragma unroll
  for (int b0 = 0; b0 < IT; b0 += NB) {
    u4 v[NB];
#pragma unroll
    for (int j = 0; j < NB; ++j) {
      const int q = tid + (b0 + j) * NTH;
      const int t = q / (CO * 8), rem = q - t * CO * 8, n = rem >> 3, slot = rem & 7;
      v[j] = *reinterpret_cast<const u4*>(w + ((size_t)n * p.kpad + t * CI + (slot ^ (n & 7)) * 8) * 2);
    }
#pragma unroll
    for (int j = 0; j < NB; ++j) {
      const int q = tid + (b0 + j) * NTH;
      const int t = q / (CO * 8), rem = q - t * CO * 8, n = rem >> 3, slot = rem & 7;
      *reinterpret_cast<u4*>(wl + t * WTAP + n * 128 + slot * 16) = v[j];
    }
  }
}

// HOOK: microbenchmark builds only (scripts/convbench.hip; the ABI never accepts them) — 12 no output
// stores, 13 no patch DMA, 14 no epilogue, 16 MFMA loop only.  Compile-time, so that the production
// form has no runtime test between the MFMAs and the previous tile's epilogue: a branch there puts the
// epilogue in its own basic block, which the sched_group_barrier pattern cannot interleave with the
// MFMAs (round 3: the epilogue then ran as a VALU block between super-steps, ~20 % of the kernel).
// NWV = 8 (round 4, variant 17): eight waves of 2 output rows each, two per SIMD — the 4-wave form runs
// one wave per SIMD (450 registers), so nothing covers its own LDS / DMA waits (PMC: MFMA pipe 47 % busy,
// 31 % of the wave's cycles waiting, profiles/r4_pmc_kernels/ws64_*); here a super-step is 24 MFMAs
// from 12 weight + 4 patch fragments, and the other wave of the SIMD issues while one waits.
template <int ACT, int HOOK = 0, int NWV = 4>
__global__ __launch_bounds__(64 * NWV, 1) void conv3x3_ws64_kernel(const ConvParams p) {
  constexpr int NTH = 64 * NWV;
  constexpr int RPW = TS / NWV;                 // output rows per wave
  constexpr int NX = RPW + 2;                   // patch rows a wave reads per super-step
  constexpr int GPW_ = (PGROUPS + NWV - 1) / NWV;
  constexpr int NPIECE = 2 * RPW;               // epilogue pieces (= 16-byte stores) per lane per tile
  static_assert(NWV == 4 || NWV == 8, "4 or 8 waves");
  __shared__ __attribute__((aligned(16))) unsigned char smem[LDS];
  unsigned char* wl = smem + 2 * PBUF;

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int g = lane >> 4, li = lane & 15;
  const int tx_n = p.W / TS, tpi = tx_n * (p.H / TS), T = p.B * tpi;

  const auto xr = make_rsrc(p.x, p.xbytes);
  const auto yr = make_rsrc(p.y, 0x7fffffffu);

  // bias first: its loads must not be waited for behind the first patch DMA
  float bias[4][4];
#pragma unroll
  for (int j = 0; j < 4; ++j)
#pragma unroll
    for (int e = 0; e < 4; ++e) bias[j][e] = p.bias[j * 16 + g * 4 + e];

  // weights -> LDS once: tap t, out channel n, 16-byte slot s holds K chunk s ^ (n & 7) of that tap
  load_weights<NTH>(p, wl, tid);

  // patch DMA: wave w moves groups w, w+4, ... (waves 1-3 repeat their last group so that every wave
  // issues GPW instructions: identical bytes to the same LDS addresses).  Lane l of group G: patch
  // pixel pp = 8G + (l >> 3), slot l & 7 = source chunk slot ^ (column & 7); its source offset is
  // relative to the tile's patch origin (scalar offset per tile).
  uint32_t dvo[GPW_];
  int dgrp[GPW_];
#pragma unroll
  for (int k = 0; k < GPW_; ++k) {
    int G8 = wave + NWV * k;
    if (G8 >= PGROUPS) G8 -= NWV;
    dgrp[k] = G8;
    const int pp = 8 * G8 + (lane >> 3);
    const int py = pp / PS, px = pp - py * PS;
    const int c = (lane & 7) ^ (px & 7);
    dvo[k] = pp < PPIX ? (uint32_t)(((py * (p.W + 2 * BORDER) + px) * p.xc + c * 8) * 2) : 0x80000000u;
  }
  auto patch_origin = [&](int t) -> uint32_t {
    const int b = t / tpi, r = t - b * tpi, ty = r / tx_n, tx = r - ty * tx_n;
    return (uint32_t)((pix_index(b, ty * TS - 1, tx * TS - 1, p.H, p.W) * p.xc + p.xoff) * 2);
  };
  auto issue_patch = [&](int t, int buf) {
    const uint32_t so = __builtin_amdgcn_readfirstlane(patch_origin(t));
    unsigned char* base = smem + buf * PBUF;
    if constexpr (HOOK != 13 && HOOK != 16)
#pragma unroll
      for (int k = 0; k < GPW_; ++k) dma16(xr, base + dgrp[k] * 1024, dvo[k], so);
  };

  // per-lane LDS read bases (the tap loop adds compile-time offsets only)
  //   weights: row j*16 + li of tap t, chunk sub*4 + g  -> slot (sub*4 + g) ^ (li & 7)
  //   patch:   pixel (4*wave + i + r) * PS + li + s, chunk sub*4 + g -> slot (sub*4 + g) ^ ((li + s) & 7)
  uint32_t wbase[2], pbase[3][2];
#pragma unroll
  for (int sub = 0; sub < 2; ++sub) {
    wbase[sub] = (uint32_t)(li * 128 + (((sub * 4 + g) ^ (li & 7)) * 16));
#pragma unroll
    for (int s = 0; s < 3; ++s)
      pbase[s][sub] = (uint32_t)((RPW * wave * PS + li + s) * 128 + (((sub * 4 + g) ^ ((li + s) & 7)) * 16));
  }

  // output offset of tile t's (4*wave + i, li) pixel row, channel g*4 (+ j*32 bytes per j)
  const uint32_t rowb = (uint32_t)((p.Wo + 2 * BORDER) * p.yc * 2);
  auto out_origin = [&](int t) -> uint32_t {
    const int b = t / tpi, rr = t - b * tpi, ty = rr / tx_n, tx = rr - ty * tx_n;
    return (uint32_t)((pix_index(b, ty * TS + RPW * wave, tx * TS + li, p.Ho, p.Wo) * p.yc + p.yoff) * 2);
  };
  // One tile = 6 super-steps (tap column s, 32-deep K half `sub`): 6 patch fragments (patch rows
  // 4*wave + 0..5) and 12 weight fragments (taps (0..2, s)) feed 48 MFMAs — each patch fragment
  // serves all three tap rows.  The next super-step's 18 fragments are read into the other register
  // set before this one's MFMAs, so LDS latency hides under 768 MFMA cycles; `side(ss)` runs after
  // super-step ss's MFMAs are issued (the previous tile's epilogue rides there).
  // (round 6) one opaque LDS offset per (tap column, K half): the taps' rows and fragments then sit within
  // the read's 16-bit offset field (r * 3 * WTAP + j * 2 KiB <= 54 KiB) instead of costing a v_or each
  uint32_t wcol[3][2];
#pragma unroll
  for (int sc = 0; sc < 3; ++sc)
#pragma unroll
    for (int sub = 0; sub < 2; ++sub) {
      wcol[sc][sub] = (uint32_t)(2 * PBUF + sc * WTAP) + wbase[sub];
      asm volatile("" : "+v"(wcol[sc][sub]));
    }
  auto load_w = [&](int ss, u4 (&wf)[3][4]) __attribute__((always_inline)) {
    const int sc = ss >> 1, sub = ss & 1;
#pragma unroll
    for (int r = 0; r < 3; ++r)
#pragma unroll
      for (int j = 0; j < 4; ++j)
        wf[r][j] = *reinterpret_cast<const u4*>(smem + wcol[sc][sub] + (r * 3 * WTAP + j * 16 * 128));
  };
  auto load_x = [&](const unsigned char* pb, int ss, u4 (&xf)[NX]) __attribute__((always_inline)) {
    const int sc = ss >> 1, sub = ss & 1;
#pragma unroll
    for (int q = 0; q < NX; ++q) xf[q] = *reinterpret_cast<const u4*>(pb + q * PS * 128 + pbase[sc][sub]);
  };
  // Super-step ss computes from set (ss & 1); set 0's weights (tap column 0, K half 0) are the same
  // for every tile, so the last super-step of a tile re-reads them for the next tile: at a tile's
  // start only the 6 patch fragments wait on LDS behind the barrier.
  u4 wA[3][4], xA[NX], wB[3][4], xB[NX];   // set 0's weights are first read after the first barrier
  auto tile_mfma = [&](const unsigned char* pb, f4 (&acc)[4][RPW], auto&& side) __attribute__((always_inline)) {
    load_x(pb, 0, xA);
    auto step = [&](auto ssc) __attribute__((always_inline)) {
      constexpr int ss = decltype(ssc)::value;
      auto& wc = (ss & 1) ? wB : wA;
      auto& xc = (ss & 1) ? xB : xA;
      auto& wn = (ss & 1) ? wA : wB;
      auto& xn = (ss & 1) ? xA : xB;
      if constexpr (ss + 1 < 6) {
        load_w(ss + 1, wn);
        load_x(pb, ss + 1, xn);
      } else {
        load_w(0, wn);
      }
#pragma unroll
      for (int r = 0; r < 3; ++r)
#pragma unroll
        for (int j = 0; j < 4; ++j)
#pragma unroll
          for (int i = 0; i < RPW; ++i)
            acc[j][i] = __builtin_amdgcn_mfma_f32_16x16x32_f16(__builtin_bit_cast(h8, wc[r][j]),
                                                               __builtin_bit_cast(h8, xc[i + r]), acc[j][i], 0, 0, 0);
      side(ssc);
      // issue pattern of the super-step: the next set's fragment reads (12 + NX, or the 12 weight
      // fragments of the next tile's first set) ride between the first MFMAs (their latency hides
      // under the rest), the side work's VALU ops two per MFMA
      constexpr int NR = ss + 1 < 6 ? 12 + NX : 12;
#pragma unroll
      for (int k = 0; k < 12 * RPW; ++k) {
        __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
        if (k < NR) __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
        __builtin_amdgcn_sched_group_barrier(0x002, 2, 0);
      }
      __builtin_amdgcn_sched_barrier(0);
    };
    step(std::integral_constant<int, 0>{});
    step(std::integral_constant<int, 1>{});
    step(std::integral_constant<int, 2>{});
    step(std::integral_constant<int, 3>{});
    step(std::integral_constant<int, 4>{});
    step(std::integral_constant<int, 5>{});
  };
  // epilogue piece q (0..7) of a finished tile: pixel row i = q / 2, channel pair (ja, jb) =
  // (2m, 2m+1), m = q % 2.  acc[j][i] holds channels j*16 + g*4 .. +3 of pixel (4*wave + i, li);
  // after bias (in the accumulator) + activation + fp16, one v_permlane16_swap per dword trades
  // halves between lane rows g = 2h and 2h+1, so row 2h holds channels ja*16 + 8h .. +7 and row
  // 2h+1 channels jb*16 + 8h .. +7: one 16-byte store per lane (a pixel's 32m .. 32m+31 channels are
  // 64 contiguous bytes from its four lanes).
  const uint32_t lane_ch = (uint32_t)((16 * (g & 1) + 8 * (g >> 1)) * 2);
  auto epi_piece = [&](const f4 (&acc)[4][RPW], uint32_t o0, int q) {
    const int i = q >> 1, m = q & 1;
    typedef _Float16 h4 __attribute__((ext_vector_type(4)));
    h4 va, vb;
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      va[e] = (_Float16)act_t<ACT>(acc[2 * m][i][e]);
      vb[e] = (_Float16)act_t<ACT>(acc[2 * m + 1][i][e]);
    }
    const u2 a = __builtin_bit_cast(u2, va), b = __builtin_bit_cast(u2, vb);
    const auto s0 = __builtin_amdgcn_permlane16_swap(a[0], b[0], false, false);
    const auto s1 = __builtin_amdgcn_permlane16_swap(a[1], b[1], false, false);
    const u4 v = {s0[0], s1[0], s0[1], s1[1]};
    if constexpr (HOOK != 12)
      __builtin_amdgcn_raw_buffer_store_b128(v, yr, o0 + i * rowb + m * 64 + lane_ch, 0, 0);
  };
  auto init_acc = [&](f4 (&acc)[4][RPW]) {
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int i = 0; i < RPW; ++i) acc[j][i] = f4{bias[j][0], bias[j][1], bias[j][2], bias[j][3]};
  };

  // Pipeline, iteration of tile t (patch buffer b = iteration parity):
  //   wait for patch(t) (the only older memory op besides the previous tile's epilogue stores, which
  //   are younger) -> barrier (also: every wave finished reading buffer b^1) -> DMA patch(t+G) into
  //   b^1 -> tile t's MFMAs with the previous tile's epilogue interleaved.
  // XCD-major persistent tile walk (xcd_tile_walk): the blocks of one XCD take neighbouring tiles, so
  // the halo rows two adjacent tiles share come from that XCD's L2
  const TileWalk tw = xcd_tile_walk(T);
  int t = tw.t;
  const int TS_ = tw.step, TE = tw.end;
  if (t >= TE) return;
  issue_patch(t, 0);
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");   // weight ds_writes of this wave
  f4 accA[4][RPW], accB[4][RPW];
  uint32_t oprev = 0;
  int buf = 0;
  // first tile: no epilogue to interleave
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  if (t + TS_ < TE) issue_patch(t + TS_, 1);
  init_acc(accA);
  load_w(0, wA);   // (the weight image is complete: every wave's ds_writes precede the barrier)
  tile_mfma(smem, accA, [](auto) {});
  oprev = out_origin(t);
  t += TS_;
  buf = 1;
  // steady state, two tiles per trip so the accumulator sets swap roles without copies
  bool stores_out = false;   // the previous iteration issued an epilogue (NSTORE younger stores)
  while (t < TE) {
    if (stores_out) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(NPIECE) : "memory");
    else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    stores_out = true;
    if constexpr (HOOK != 16) __builtin_amdgcn_s_barrier();
    if (t + TS_ < TE) issue_patch(t + TS_, buf ^ 1);
    init_acc(accB);
    tile_mfma(smem + buf * PBUF, accB, [&](auto ssc) __attribute__((always_inline)) {
      constexpr int ss = decltype(ssc)::value;
      if constexpr (HOOK != 14 && HOOK != 16)
#pragma unroll
        for (int q = (ss * NPIECE) / 6; q < ((ss + 1) * NPIECE) / 6; ++q) epi_piece(accA, oprev, q);
    });
    oprev = out_origin(t);
    t += TS_;
    buf ^= 1;
    if (t >= TE) {
#pragma unroll
      for (int q = 0; q < NPIECE; ++q) epi_piece(accB, oprev, q);
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      return;
    }
    asm volatile("s_waitcnt vmcnt(%0)" ::"n"(NPIECE) : "memory");
    if constexpr (HOOK != 16) __builtin_amdgcn_s_barrier();
    if (t + TS_ < TE) issue_patch(t + TS_, buf ^ 1);
    init_acc(accA);
    tile_mfma(smem + buf * PBUF, accA, [&](auto ssc) __attribute__((always_inline)) {
      constexpr int ss = decltype(ssc)::value;
      if constexpr (HOOK != 14 && HOOK != 16)
#pragma unroll
        for (int q = (ss * NPIECE) / 6; q < ((ss + 1) * NPIECE) / 6; ++q) epi_piece(accB, oprev, q);
    });
    oprev = out_origin(t);
    t += TS_;
    buf ^= 1;
  }
#pragma unroll
  for (int q = 0; q < NPIECE; ++q) epi_piece(accA, oprev, q);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}


// ---------------------------------------------------------------------------------------------
// Half-patch ring form (variant 15; YV7_WS64R=1 makes it the dispatch's choice).  Measured on the
// kernel above (scripts/convbench.hip, bs 32, round 3): at 320^2 the MFMA loop alone runs 177 us but
// the whole kernel 330-340 — each CU keeps at most ONE 41 KiB patch in flight (the second LDS buffer
// is the one being computed on), issued in a burst at the tile start and waited for at the next, so
// the ~1.3 GB a layer moves runs at under 3 TB/s: latency-bound, not bandwidth-bound.  Here:
//  * the patch is split by 32-channel K half into half-patches (324 pixels x 64 B, 21 DMA pieces of
//    1 KiB) in a 4-slot LDS ring (84 KiB + the 72 KiB weight image): a tile's super-steps run K half 0
//    (tap columns 0, 1, 2) then K half 1, so a half-patch is dead after its three super-steps;
//  * one ring step per half: before the half's LAST super-step (its fragments are already in
//    registers) wait for the next half-patch, barrier, and refill the slot just finished with the
//    half-patch four ahead — three half-patches (62 KiB) stay in flight continuously and each lands
//    ~3 halves (~430 MFMA cycles x 3) after it was issued;
//  * the last super-step of a half prefetches the next half's first fragments (after the barrier),
//    so a tile start no longer waits on LDS; set 0's weights are re-read for the next tile there too;
//  * every wave issues 6 DMA pieces per half (waves 1-3 duplicate wave 0's piece 20: identical bytes,
//    distinct per-wave issue) and 4 epilogue stores per half (1, 2, 1 over its super-steps), so every
//    counted vmcnt is a compile-time constant once the ring is full (24); the block's first tile
//    stores into the void (offsets past the buffer range) to keep the count.
// LDS: 4 x 21 KiB + 72 KiB = 156 KiB.  Slots are compile-time: one loop trip = 2 tiles = 4 halves.
// Measured (round 3, profiles/r3p/): convbench (random operands, input not cache-resident)
// @320 330 us vs 296 for the column-pair form with its epilogue interleaved, @160 74 vs 82; in-network
// (tune_ops, one layer forced) equal within 1-2 us on every layer — the deeper ring does not buy
// bandwidth at 320^2 (64-B half-lines per pixel: twice the L2 requests per byte of the 128-B lines
// the column-pair form fetches), so it is kept as an alternative, not the default.
template <int ACT>
__global__ __launch_bounds__(NT, 1) void conv3x3_ws64r_kernel(const ConvParams p) {
  constexpr int HP = 21 * 1024;              // one half-patch slot (336 rows of 64 B)
  constexpr int WOFF = 4 * HP;
  constexpr int NP = 6;                      // DMA pieces per wave per half
  constexpr int ROW = 64;                    // bytes per patch pixel row in a slot (32 channels)
  constexpr uint32_t DUMMY_SO = 0x40000000u; // scalar offset of a half-patch past the walk: reads zeros
  constexpr int BOFF = WOFF + 9 * WTAP;     // 64 fp32 biases
  static_assert(BOFF + CO * 4 <= 160 * 1024, "LDS budget");
  __shared__ __attribute__((aligned(16))) unsigned char smem[BOFF + CO * 4];
  unsigned char* wl = smem + WOFF;

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int g = lane >> 4, li = lane & 15;
  const int tx_n = p.W / TS, tpi = tx_n * (p.H / TS), T = p.B * tpi;
  const TileWalk tw = xcd_tile_walk(T);
  const int ntl = tw.count();
  if (ntl == 0) return;

  const auto xr = make_rsrc(p.x, p.xbytes);
  const auto yr = make_rsrc(p.y, 0x7fffffffu);

  // bias in LDS (registers are the scarce resource here: two accumulator and fragment sets)
  float* bias_l = reinterpret_cast<float*>(smem + BOFF);
  if (tid < CO) bias_l[tid] = p.bias[tid];

  // weights -> LDS once (the layout of the kernel above)
  load_weights(p, wl, tid);

  // half-patch DMA: piece G = wave + 4k (k < 5), the sixth is piece 20 for every wave.  Lane l of piece
  // G: patch pixel pp = 16 G + (l >> 2), LDS slot l & 3 of its 64-B row holds source chunk
  // (l & 3) ^ ((px >> 1) & 3) (the reader's swizzle); offsets relative to the half's origin.
  uint32_t dvo[NP], dlds[NP];
#pragma unroll
  for (int k = 0; k < NP; ++k) {
    const int G = k < 5 ? wave + 4 * k : 20;
    dlds[k] = (uint32_t)(G * 1024);
    const int pp = 16 * G + (lane >> 2);
    const int py = pp / PS, px = pp - py * PS;
    const int c = (lane & 3) ^ ((px >> 1) & 3);
    dvo[k] = pp < PPIX ? (uint32_t)(((py * (p.W + 2 * BORDER) + px) * p.xc + c * 8) * 2) : 0x80000000u;
  }
  auto origin = [&](int it) -> uint32_t {   // scalar byte offset of tile it's patch origin, channel 0
    if (it >= ntl) return DUMMY_SO;
    const int t = tw.at(it);
    const int b = t / tpi, r = t - b * tpi, ty = r / tx_n, tx = r - ty * tx_n;
    return __builtin_amdgcn_readfirstlane(
        (uint32_t)((pix_index(b, ty * TS - 1, tx * TS - 1, p.H, p.W) * p.xc + p.xoff) * 2));
  };
  auto issue_half = [&](int slot, uint32_t so) __attribute__((always_inline)) {
#pragma unroll
    for (int k = 0; k < NP; ++k) dma16(xr, smem + slot * HP + dlds[k], dvo[k], so);
    asm volatile("" ::: "memory");   // pin the DMA before this super-step's stores (the counted waits)
  };

  // fragment read bases: weights as the kernel above; patch pixel (4 wave + q, li + s) of a slot
  // (ds_read offsets are 16-bit immediates: the weight image is addressed from two bases — taps 0-5
  // and 6-8 — and slot 3 from its own, each laundered through an empty asm so the compiler cannot fold
  // them back into one base plus offsets too large for the immediate, which it would then materialize
  // as one VGPR per read and spill)
  uint32_t wlo[2], whi[2], xl[3], xl3[3];
#pragma unroll
  for (int sub = 0; sub < 2; ++sub) {
    const uint32_t wb = (uint32_t)(WOFF + li * 128 + (((sub * 4 + g) ^ (li & 7)) * 16));
    wlo[sub] = wb;
    whi[sub] = wb + 6 * WTAP;
    asm volatile("" : "+v"(wlo[sub]));
    asm volatile("" : "+v"(whi[sub]));
  }
#pragma unroll
  for (int s = 0; s < 3; ++s) {
    xl[s] = (uint32_t)((4 * wave * PS + li + s) * ROW + ((g ^ (((li + s) >> 1) & 3)) * 16));
    xl3[s] = xl[s] + 3 * HP;
    asm volatile("" : "+v"(xl[s]));
    asm volatile("" : "+v"(xl3[s]));
  }

  const uint32_t rowb = (uint32_t)((p.Wo + 2 * BORDER) * p.yc * 2);
  auto out_origin = [&](int it) -> uint32_t {
    const int t = tw.at(it);
    const int b = t / tpi, rr = t - b * tpi, ty = rr / tx_n, tx = rr - ty * tx_n;
    return (uint32_t)((pix_index(b, ty * TS + 4 * wave, tx * TS + li, p.Ho, p.Wo) * p.yc + p.yoff) * 2);
  };
  const uint32_t lane_ch = (uint32_t)((16 * (g & 1) + 8 * (g >> 1)) * 2);
  auto epi_piece = [&](const f4 (&acc)[4][4], uint32_t o0, int q) __attribute__((always_inline)) {
    const int i = q >> 1, m = q & 1;
    typedef _Float16 h4 __attribute__((ext_vector_type(4)));
    h4 va, vb;
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      va[e] = (_Float16)act_t<ACT>(acc[2 * m][i][e]);
      vb[e] = (_Float16)act_t<ACT>(acc[2 * m + 1][i][e]);
    }
    const u2 a = __builtin_bit_cast(u2, va), b = __builtin_bit_cast(u2, vb);
    const auto s0 = __builtin_amdgcn_permlane16_swap(a[0], b[0], false, false);
    const auto s1 = __builtin_amdgcn_permlane16_swap(a[1], b[1], false, false);
    const u4 v = {s0[0], s1[0], s0[1], s1[1]};
    __builtin_amdgcn_raw_buffer_store_b128(v, yr, o0 + i * rowb + m * 64 + lane_ch, 0, 0);
  };

  u4 wA[3][4], xA[6], wB[3][4], xB[6];
  auto load_w = [&](int s, int sub, u4 (&wf)[3][4]) __attribute__((always_inline)) {
#pragma unroll
    for (int r = 0; r < 3; ++r)
#pragma unroll
      for (int j = 0; j < 4; ++j)
        wf[r][j] = *reinterpret_cast<const u4*>(
            smem + (r < 2 ? wlo[sub] + (r * 3 + s) * WTAP : whi[sub] + s * WTAP) + j * 16 * 128);
  };
  auto load_x = [&](int slot, int s, u4 (&xf)[6]) __attribute__((always_inline)) {
#pragma unroll
    for (int q = 0; q < 6; ++q)
      xf[q] = *reinterpret_cast<const u4*>(smem + (slot == 3 ? xl3[s] : xl[s] + slot * HP) + q * PS * ROW);
  };

  // vmcnt of ring step `pos` (0..3 within a loop trip): the ops younger than the half-patch the next
  // half reads — two halves of DMA (12) and the stores since it was issued (12 once the ring is full;
  // the first trip's first three steps follow the prologue: 3, 7, 11)
  auto ring_wait = [&](auto posc, bool first) __attribute__((always_inline)) {
    constexpr int pos = decltype(posc)::value;
    if (pos < 3 && first) {
      if constexpr (pos == 0) asm volatile("s_waitcnt vmcnt(15) lgkmcnt(0)" ::: "memory");
      if constexpr (pos == 1) asm volatile("s_waitcnt vmcnt(19) lgkmcnt(0)" ::: "memory");
      if constexpr (pos == 2) asm volatile("s_waitcnt vmcnt(23) lgkmcnt(0)" ::: "memory");
    } else {
      asm volatile("s_waitcnt vmcnt(24) lgkmcnt(0)" ::: "memory");
    }
    __builtin_amdgcn_s_barrier();
  };

  // one tile (slots S0 = K half 0, S0 + 1 = K half 1) into acc; prev / oprev: the previous tile's
  // epilogue, 8 pieces over the six super-steps; so2: the origin of the tile two ahead (its halves
  // refill this tile's slots)
  auto run_tile = [&](auto s0c, f4 (&acc)[4][4], const f4 (&prev)[4][4], uint32_t oprev, uint32_t so2, bool first)
      __attribute__((always_inline)) {
    constexpr int S0 = decltype(s0c)::value;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const f4 bv = *reinterpret_cast<const f4*>(bias_l + j * 16 + g * 4);
#pragma unroll
      for (int i = 0; i < 4; ++i) acc[j][i] = bv;
    }
    auto step = [&](auto ssc) __attribute__((always_inline)) {
      constexpr int ss = decltype(ssc)::value;   // 0..5: K half ss / 3, tap column ss % 3
      constexpr int sub = ss / 3, s = ss % 3;
      auto& wc = (ss & 1) ? wB : wA;
      auto& xc = (ss & 1) ? xB : xA;
      auto& wn = (ss & 1) ? wA : wB;
      auto& xn = (ss & 1) ? xA : xB;
      if constexpr (s == 2) {
        // ring step: the next half-patch landed everywhere; refill this half's slot
        ring_wait(std::integral_constant<int, (S0 / 2) * 2 + sub>{}, first);
        issue_half(S0 + sub, so2 + (uint32_t)(sub * 64));
        __builtin_amdgcn_sched_barrier(0);
        // next fragments: K half 1 column 0 of this tile, or the next tile's K half 0 column 0
        load_w(0, 1 - sub, wn);
        load_x(sub == 0 ? S0 + 1 : (S0 + 2) % 4, 0, xn);
      } else {
        load_w(s + 1, sub, wn);
        load_x(S0 + sub, s + 1, xn);
      }
#pragma unroll
      for (int r = 0; r < 3; ++r)
#pragma unroll
        for (int j = 0; j < 4; ++j)
#pragma unroll
          for (int i = 0; i < 4; ++i)
            acc[j][i] = __builtin_amdgcn_mfma_f32_16x16x32_f16(__builtin_bit_cast(h8, wc[r][j]),
                                                               __builtin_bit_cast(h8, xc[i + r]), acc[j][i], 0, 0, 0);
      // previous tile's epilogue: pieces (1, 2, 1) per K half
      {
        constexpr int q0 = sub * 4 + (s == 0 ? 0 : s == 1 ? 1 : 3);
        constexpr int nq = s == 1 ? 2 : 1;
#pragma unroll
        for (int q = q0; q < q0 + nq; ++q) epi_piece(prev, oprev, q);
      }
      // issue pattern: the 18 next-fragment reads between the first MFMAs, epilogue VALU two per MFMA
#pragma unroll
      for (int k = 0; k < 48; ++k) {
        __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
        if (k < 18) __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
        __builtin_amdgcn_sched_group_barrier(0x002, 2, 0);
      }
      __builtin_amdgcn_sched_barrier(0);
    };
    step(std::integral_constant<int, 0>{});
    step(std::integral_constant<int, 1>{});
    step(std::integral_constant<int, 2>{});
    step(std::integral_constant<int, 3>{});
    step(std::integral_constant<int, 4>{});
    step(std::integral_constant<int, 5>{});
  };
  auto last_epilogue = [&](const f4 (&acc)[4][4], uint32_t o) __attribute__((always_inline)) {
#pragma unroll
    for (int q = 0; q < 8; ++q) epi_piece(acc, o, q);
  };

  // prologue: halves 0..3 (tiles 0 and 1) into slots 0..3, then half 0 landed and the weight image
  // complete everywhere; tile 0's first fragments
  {
    const uint32_t o0 = origin(0), o1 = origin(1);
    issue_half(0, o0);
    issue_half(1, o0 + 64);
    issue_half(2, o1);
    issue_half(3, o1 + 64);
  }
  asm volatile("s_waitcnt vmcnt(18) lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  load_w(0, 0, wA);
  load_x(0, 0, xA);

  f4 accA[4][4], accB[4][4];
#pragma unroll
  for (int j = 0; j < 4; ++j)
#pragma unroll
    for (int i = 0; i < 4; ++i) accB[j][i] = f4{0.0f, 0.0f, 0.0f, 0.0f};
  uint32_t oprev = 0x80000000u;   // the first tile's "previous tile" stores land past the buffer range
  for (int it = 0;; it += 2) {
    const bool first = it == 0;
    run_tile(std::integral_constant<int, 0>{}, accA, accB, oprev, origin(it + 2), first);
    oprev = out_origin(it);
    if (it + 1 == ntl) {
      last_epilogue(accA, oprev);
      break;
    }
    run_tile(std::integral_constant<int, 2>{}, accB, accA, oprev, origin(it + 3), first);
    oprev = out_origin(it + 1);
    if (it + 2 == ntl) {
      last_epilogue(accB, oprev);
      break;
    }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

int num_cus() {
  static const int n = [] {
    int dev = 0, v = 0;
    if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&v, hipDeviceAttributeMultiprocessorCount, dev) !=
                                                 hipSuccess || v <= 0)
      v = 256;
    return v;
  }();
  return n;
}

}  // namespace

bool ws64_supported(const ConvParams& p) {
  return p.k == 3 && p.s == 1 && p.pad == 1 && p.cin == CI && p.cout == CO && p.kpad == 9 * CI &&
         p.H % TS == 0 && p.W % TS == 0 && p.Ho == p.H && p.Wo == p.W && (p.xc % 8) == 0 && (p.xoff % 8) == 0 &&
         (p.yc % 4) == 0 && (p.yoff % 4) == 0;
}

hipError_t launch_conv_ws64(const ConvParams& p, hipStream_t st) {
  if (!ws64_supported(p)) return hipErrorInvalidValue;
  const int T = p.B * (p.H / TS) * (p.W / TS);
  const int grid = T < num_cus() ? T : num_cus();
  // microbenchmark hooks (scripts/convbench.hip only; the ABI never accepts them) on the column-pair form
  if (p.act == 1 && p.variant >= 12 && p.variant <= 16 && p.variant != 15) {
    if (p.variant == 12) YV7_LAUNCH((conv3x3_ws64_kernel<1, 12>), dim3(grid), dim3(NT), 0, st, p);
    else if (p.variant == 13) YV7_LAUNCH((conv3x3_ws64_kernel<1, 13>), dim3(grid), dim3(NT), 0, st, p);
    else if (p.variant == 14) YV7_LAUNCH((conv3x3_ws64_kernel<1, 14>), dim3(grid), dim3(NT), 0, st, p);
    else YV7_LAUNCH((conv3x3_ws64_kernel<1, 16>), dim3(grid), dim3(NT), 0, st, p);
    return hipGetLastError();
  }
  // the two forms measured equal in-network (scripts/tune_ops.py, one layer forced at a time, same box,
  // us, 11 / 15: @320 228.2 / 228.4, @160 73.7 / 71.6, 71.4 / 69.8, 71.4 / 70.8, 72.3 / 71.1 — and the
  // halo kernel keeps the @80 layers: 30.1 vs 32.2 / 34.1); of those two 4-wave forms the column-pair one
  // is the 4-wave choice, but the default is now the 8-wave form below.  YV7_WS64R=1: the ring form.
  static const int ring = [] { const char* e = getenv("YV7_WS64R"); return e ? atoi(e) : 0; }();
  // the 8-wave form (two waves per SIMD; variant 17) is the default since round 4: in-network, one layer
  // forced at a time (profiles/r4_ws8/, us, 4-wave -> 8-wave): yolov7 bs 32 @320 233.9 -> 218.2, the four
  // @160 layers 65.7-68.1 -> 61.6-63.5; w6 bs 8 @320 64.3-68.8 -> 62.0-63.0.  Variant 11 / YV7_WS64_4=1:
  // the 4-wave form.
  static const int four = [] { const char* e = getenv("YV7_WS64_4"); return e ? atoi(e) : 0; }();   // A/B: 4-wave
  if (p.variant == 17 || (p.variant != 11 && p.variant != 15 && !ring && !four)) {
    if (p.act == 1) YV7_LAUNCH((conv3x3_ws64_kernel<1, 0, 8>), dim3(grid), dim3(512), 0, st, p);
    else if (p.act == 2) YV7_LAUNCH((conv3x3_ws64_kernel<2, 0, 8>), dim3(grid), dim3(512), 0, st, p);
    else YV7_LAUNCH((conv3x3_ws64_kernel<0, 0, 8>), dim3(grid), dim3(512), 0, st, p);
    return hipGetLastError();
  }
  if (p.variant == 11 || (p.variant != 15 && !ring)) {
    if (p.act == 1) YV7_LAUNCH((conv3x3_ws64_kernel<1>), dim3(grid), dim3(NT), 0, st, p);
    else if (p.act == 2) YV7_LAUNCH((conv3x3_ws64_kernel<2>), dim3(grid), dim3(NT), 0, st, p);
    else YV7_LAUNCH((conv3x3_ws64_kernel<0>), dim3(grid), dim3(NT), 0, st, p);
    return hipGetLastError();
  }
  if (p.act == 1) YV7_LAUNCH((conv3x3_ws64r_kernel<1>), dim3(grid), dim3(NT), 0, st, p);
  else if (p.act == 2) YV7_LAUNCH((conv3x3_ws64r_kernel<2>), dim3(grid), dim3(NT), 0, st, p);
  else YV7_LAUNCH((conv3x3_ws64r_kernel<0>), dim3(grid), dim3(NT), 0, st, p);
  return hipGetLastError();
}

}  // namespace yv7
