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
//    lane's accumulator is 4 consecutive channels of one pixel);
//  * software-pipelined across tiles: tile t's epilogue (bias = accumulator init, compile-time
//    activation, fp16, v_permlane16_swap so each lane holds 8 consecutive channels, 16-byte stores
//    into the destination channel slice — zero-copy concat) is issued between tile t+1's MFMAs;
//  * fragment reads for the next super-step are issued among the current one's MFMAs
//    (sched_group_barrier pattern), so LDS latency stays off the MFMA pipe.
// LDS: 2 x 41 KiB patch buffers + 72 KiB weights = 154 KiB.
// Microbenchmark hooks (ConvParams::variant, scripts/convbench.hip): 12 no output stores, 13 no patch
// DMA, 14 no epilogue, 16 MFMA loop only.
#include <hip/hip_runtime.h>

#include "yv7_kernels.h"

namespace yv7 {

namespace {

constexpr int NT = 256;
constexpr int TS = 16;                       // output tile side
constexpr int PS = TS + 2;                   // patch side
constexpr int PPIX = PS * PS;                // 324 patch pixels
constexpr int PGROUPS = (PPIX + 7) / 8;      // 41 DMA wave-instructions (8 pixels x 128 B) per patch
constexpr int PBUF = PGROUPS * 1024;         // 41,984 B per patch buffer
constexpr int GPW = (PGROUPS + 3) / 4;       // 11 DMA instructions per wave per patch
constexpr int CI = 64, CO = 64;
constexpr int WTAP = CO * CI * 2;            // 8 KiB of weights per tap
constexpr int LDS = 2 * PBUF + 9 * WTAP;     // 157,696 B
constexpr int NSTORE = 8;                    // epilogue stores per lane per tile
typedef uint32_t u2 __attribute__((ext_vector_type(2)));

__device__ __forceinline__ void dma16(__amdgpu_buffer_rsrc_t r, void* lds, uint32_t vo, uint32_t so) {
  __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (__attribute__((address_space(3))) void*)lds, 16, vo, so, 0, 0);
}

// SCHED: 0 = the MFMA / ds_read / VALU issue pattern below (1 = no scheduling directives, 2 = MFMA /
// ds_read interleave only, 3 = pattern + s_setprio around the MFMAs: round-2 experiments, all slower,
// profiles/r2_ws64_sched_tune.txt; no longer launched)
template <int ACT, int SCHED = 0>
__global__ __launch_bounds__(NT, 1) void conv3x3_ws64_kernel(const ConvParams p) {
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
  {
    const unsigned char* w = reinterpret_cast<const unsigned char*>(p.w);
    for (int q = tid; q < 9 * CO * 8; q += NT) {
      const int t = q / (CO * 8), rem = q - t * CO * 8, n = rem >> 3, slot = rem & 7;
      const int chunk = slot ^ (n & 7);
      const u4 v = *reinterpret_cast<const u4*>(w + ((size_t)n * p.kpad + t * CI + chunk * 8) * 2);
      *reinterpret_cast<u4*>(wl + t * WTAP + n * 128 + slot * 16) = v;
    }
  }

  // patch DMA: wave w moves groups w, w+4, ... (waves 1-3 repeat their last group so that every wave
  // issues GPW instructions: identical bytes to the same LDS addresses).  Lane l of group G: patch
  // pixel pp = 8G + (l >> 3), slot l & 7 = source chunk slot ^ (column & 7); its source offset is
  // relative to the tile's patch origin (scalar offset per tile).
  uint32_t dvo[GPW];
  int dgrp[GPW];
#pragma unroll
  for (int k = 0; k < GPW; ++k) {
    int G8 = wave + 4 * k;
    if (G8 >= PGROUPS) G8 -= 4;
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
    if (p.variant != 13 && p.variant != 16)
#pragma unroll
      for (int k = 0; k < GPW; ++k) dma16(xr, base + dgrp[k] * 1024, dvo[k], so);
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
      pbase[s][sub] = (uint32_t)((4 * wave * PS + li + s) * 128 + (((sub * 4 + g) ^ ((li + s) & 7)) * 16));
  }

  // output offset of tile t's (4*wave + i, li) pixel row, channel g*4 (+ j*32 bytes per j)
  const uint32_t rowb = (uint32_t)((p.Wo + 2 * BORDER) * p.yc * 2);
  auto out_origin = [&](int t) -> uint32_t {
    const int b = t / tpi, rr = t - b * tpi, ty = rr / tx_n, tx = rr - ty * tx_n;
    return (uint32_t)((pix_index(b, ty * TS + 4 * wave, tx * TS + li, p.Ho, p.Wo) * p.yc + p.yoff) * 2);
  };
  // One tile = 6 super-steps (tap column s, 32-deep K half `sub`): 6 patch fragments (patch rows
  // 4*wave + 0..5) and 12 weight fragments (taps (0..2, s)) feed 48 MFMAs — each patch fragment
  // serves all three tap rows.  The next super-step's 18 fragments are read into the other register
  // set before this one's MFMAs, so LDS latency hides under 768 MFMA cycles; `side(ss)` runs after
  // super-step ss's MFMAs are issued (the previous tile's epilogue rides there).
  auto load_ss = [&](const unsigned char* pb, int ss, u4 (&wf)[3][4], u4 (&xf)[6]) {
    const int sc = ss >> 1, sub = ss & 1;
#pragma unroll
    for (int r = 0; r < 3; ++r)
#pragma unroll
      for (int j = 0; j < 4; ++j)
        wf[r][j] = *reinterpret_cast<const u4*>(wl + (r * 3 + sc) * WTAP + j * 16 * 128 + wbase[sub]);
#pragma unroll
    for (int q = 0; q < 6; ++q) xf[q] = *reinterpret_cast<const u4*>(pb + q * PS * 128 + pbase[sc][sub]);
  };
  auto tile_mfma = [&](const unsigned char* pb, f4 (&acc)[4][4], auto&& side) {
    u4 wA[3][4], xA[6], wB[3][4], xB[6];
    load_ss(pb, 0, wA, xA);
#pragma unroll
    for (int ss = 0; ss < 6; ++ss) {
      auto& wc = (ss & 1) ? wB : wA;
      auto& xc = (ss & 1) ? xB : xA;
      auto& wn = (ss & 1) ? wA : wB;
      auto& xn = (ss & 1) ? xA : xB;
      if (ss + 1 < 6) load_ss(pb, ss + 1, wn, xn);
      if constexpr (SCHED == 3) __builtin_amdgcn_s_setprio(1);
#pragma unroll
      for (int r = 0; r < 3; ++r)
#pragma unroll
        for (int j = 0; j < 4; ++j)
#pragma unroll
          for (int i = 0; i < 4; ++i)
            acc[j][i] = __builtin_amdgcn_mfma_f32_16x16x32_f16(__builtin_bit_cast(h8, wc[r][j]),
                                                               __builtin_bit_cast(h8, xc[i + r]), acc[j][i], 0, 0, 0);
      if constexpr (SCHED == 3) __builtin_amdgcn_s_setprio(0);
      side(ss);
      // issue pattern of the super-step: the next set's 18 fragment reads ride between the first 18
      // MFMAs (their latency hides under the other 30), the side work's VALU ops two per MFMA
      if constexpr (SCHED != 1) {
#pragma unroll
        for (int k = 0; k < 48; ++k) {
          __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
          if (k < 18 && ss + 1 < 6) __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
          if constexpr (SCHED != 2) __builtin_amdgcn_sched_group_barrier(0x002, 2, 0);
        }
        __builtin_amdgcn_sched_barrier(0);
      }
    }
  };
  // epilogue piece q (0..7) of a finished tile: pixel row i = q / 2, channel pair (ja, jb) =
  // (2m, 2m+1), m = q % 2.  acc[j][i] holds channels j*16 + g*4 .. +3 of pixel (4*wave + i, li);
  // after bias (in the accumulator) + activation + fp16, one v_permlane16_swap per dword trades
  // halves between lane rows g = 2h and 2h+1, so row 2h holds channels ja*16 + 8h .. +7 and row
  // 2h+1 channels jb*16 + 8h .. +7: one 16-byte store per lane (a pixel's 32m .. 32m+31 channels are
  // 64 contiguous bytes from its four lanes).
  const uint32_t lane_ch = (uint32_t)((16 * (g & 1) + 8 * (g >> 1)) * 2);
  auto epi_piece = [&](const f4 (&acc)[4][4], uint32_t o0, int q) {
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
    if (p.variant != 12)
      __builtin_amdgcn_raw_buffer_store_b128(v, yr, o0 + i * rowb + m * 64 + lane_ch, 0, 0);
  };
  auto init_acc = [&](f4 (&acc)[4][4]) {
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int i = 0; i < 4; ++i) acc[j][i] = f4{bias[j][0], bias[j][1], bias[j][2], bias[j][3]};
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
  f4 accA[4][4], accB[4][4];
  uint32_t oprev = 0;
  int buf = 0;
  // first tile: no epilogue to interleave
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  if (t + TS_ < TE) issue_patch(t + TS_, 1);
  init_acc(accA);
  tile_mfma(smem, accA, [](int) {});
  oprev = out_origin(t);
  t += TS_;
  buf = 1;
  // steady state, two tiles per trip so the accumulator sets swap roles without copies
  bool stores_out = false;   // the previous iteration issued an epilogue (NSTORE younger stores)
  while (t < TE) {
    if (stores_out) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(NSTORE) : "memory");
    else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    stores_out = true;
    if (p.variant != 16) __builtin_amdgcn_s_barrier();
    if (t + TS_ < TE) issue_patch(t + TS_, buf ^ 1);
    init_acc(accB);
    tile_mfma(smem + buf * PBUF, accB, [&](int ss) { if (p.variant != 14 && p.variant != 16) for (int q = (ss * 4) / 3; q < ((ss + 1) * 4) / 3; ++q) epi_piece(accA, oprev, q); });
    oprev = out_origin(t);
    t += TS_;
    buf ^= 1;
    if (t >= TE) {
#pragma unroll
      for (int q = 0; q < 8; ++q) epi_piece(accB, oprev, q);
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      return;
    }
    asm volatile("s_waitcnt vmcnt(%0)" ::"n"(NSTORE) : "memory");
    if (p.variant != 16) __builtin_amdgcn_s_barrier();
    if (t + TS_ < TE) issue_patch(t + TS_, buf ^ 1);
    init_acc(accA);
    tile_mfma(smem + buf * PBUF, accA, [&](int ss) { if (p.variant != 14 && p.variant != 16) for (int q = (ss * 4) / 3; q < ((ss + 1) * 4) / 3; ++q) epi_piece(accB, oprev, q); });
    oprev = out_origin(t);
    t += TS_;
    buf ^= 1;
  }
#pragma unroll
  for (int q = 0; q < 8; ++q) epi_piece(accA, oprev, q);
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
  if (p.act == 1) YV7_LAUNCH((conv3x3_ws64_kernel<1>), dim3(grid), dim3(NT), 0, st, p);
  else if (p.act == 2) YV7_LAUNCH((conv3x3_ws64_kernel<2>), dim3(grid), dim3(NT), 0, st, p);
  else YV7_LAUNCH((conv3x3_ws64_kernel<0>), dim3(grid), dim3(NT), 0, st, p);
  return hipGetLastError();
}

}  // namespace yv7
