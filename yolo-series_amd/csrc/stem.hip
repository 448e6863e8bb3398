// Fused stem for gfx950: image packing + conv A (3 -> CA, 3x3, stride SA) + conv B (CA -> CB, 3x3,
// stride 2), conv A's activations never leave LDS.
//
// Replaces, for the yolov7 / yolov7-tiny stems, the reference's first two Conv layers
// (models/common.py:110-111 on cfg/deploy/yolov7.yaml:15-17, yolov7-tiny.yaml:14-16) and the input
// tensor preparation of detect.py:100-104.  Unfused, conv A's output is the largest tensor of the
// network (32 x 640 x 640 x 32 fp16 = 839 MB per batch of 32) and is written once and read back nine
// times through L2 by conv B; fused, it exists only as a 17 x 33 x CA tile in LDS per block.
//
// Per 256-thread block: a TBY x TBX tile of conv B's output for one image.
//   1. the NCHW image patch feeding it (PY x PX x 3, zero outside the image) -> LDS [PY][PX][4] fp16
//   2. conv A on the MFMA: M = TAY*TAX A-pixels (16 per tile), N = CA, K = 27 (one 16x16x32 step,
//      k = tap*3 + ci, zero-padded to 32), operands gathered from the patch; + bias + act, zeroed
//      outside the image (conv B's zero padding), -> LDS [A-pixel][CA] with an 80-byte pitch
//      (conflict-free ds_read_b128 for conv B's stride-2 access)
//   3. conv B on the MFMA: M = TBY*TBX, N = CB, K = 9 taps x CA; each wave owns 16 output channels and
//      holds their 9 taps of weight fragments in registers (loaded at entry, under the patch load)
//   4. + bias + act -> LDS tile -> 16-byte NHWC stores into the destination channel slice.
#include <cstdlib>
#include <type_traits>

#include "yv7_kernels.h"

namespace yv7 {

namespace {

constexpr int NT = 256;

template <typename S, int CA, int CB, int SA, int TBY, int TBX, int ACT_A, int ACT_B>
__global__ __launch_bounds__(NT, 2) void stem_kernel(const StemParams p) {
  constexpr int TAY = 2 * TBY + 1, TAX = 2 * TBX + 1;      // conv-A pixels feeding the tile
  constexpr int PY = SA * (TAY - 1) + 3, PX = SA * (TAX - 1) + 3;
  constexpr int NA = TAY * TAX;
  constexpr int MA = (NA + 15) / 16;                         // conv-A m-tiles
  constexpr int APITCH = CA * 2 + 16;                        // bytes per A-pixel (padded)
  constexpr int PATCH = PY * PX * 8;                         // [PY][PX][4] halves
  constexpr int ABUF = NA * APITCH;
  constexpr int MB = TBY * TBX / 16;                         // conv-B m-tiles
  constexpr int CPITCH = CB * 2 + 16;
  constexpr int OUTB = TBY * TBX * CPITCH;
  constexpr int LDS0 = (PATCH + ABUF + 15) / 16 * 16;
  constexpr int LDS = LDS0 > OUTB ? LDS0 : OUTB;
  static_assert(CB == 64 && CA == 32, "one wave per 16 output channels, one MFMA k-step per tap");
  __shared__ __attribute__((aligned(16))) unsigned char smem[LDS];
  _Float16* patch = reinterpret_cast<_Float16*>(smem);
  unsigned char* abuf = smem + (PATCH + 15) / 16 * 16;

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int g = lane >> 4, li = lane & 15;
  const int HA = p.H / SA, WA = p.W / SA;          // conv-A output size
  const int HB = HA / 2, WB = WA / 2;              // conv-B output size
  const int tiles_x = (WB + TBX - 1) / TBX, tiles_y = (HB + TBY - 1) / TBY;
  const int ntiles = p.B * tiles_x * tiles_y;
  // persistent: this block's tiles are blockIdx.x, + gridDim.x, ...; tile geometry
  int b = 0, oy0 = 0, ox0 = 0, ay0 = 0, ax0 = 0;
  auto tile_geom = [&](int t, int& tb, int& ty, int& tx) {
    tb = t / (tiles_x * tiles_y);
    t -= tb * tiles_x * tiles_y;
    ty = (t / tiles_x) * TBY;
    tx = (t % tiles_x) * TBX;
  };

  // conv-B weight fragments of this wave's 16 output channels, all 9 taps (K = 32 per tap = CA)
  u4 wfr[9];
#pragma unroll
  for (int tap = 0; tap < 9; ++tap)
    wfr[tap] = *reinterpret_cast<const u4*>(reinterpret_cast<const _Float16*>(p.wb) +
                                            (size_t)(wave * 16 + li) * p.kpad_b + tap * CA + g * 8);

  // 1. image patch (PY x PX x 3, zero outside the image): the NEXT tile's pixels are loaded into
  //    registers while the current tile computes, and written to LDS (fp16, channel 3 zero) at the
  //    top of the next iteration, so the image loads' latency sits under conv A / conv B.
  constexpr int PPT = (PY * PX + NT - 1) / NT;   // patch pixels per thread
  S pre[PPT][3];
  auto prefetch = [&](int t) {
    int tb, ty, tx;
    tile_geom(t, tb, ty, tx);
    const int iy0 = SA * (2 * ty - 1) - 1, ix0 = SA * (2 * tx - 1) - 1;
    const S* xb = reinterpret_cast<const S*>(p.x) + (size_t)tb * 3 * p.H * p.W;
#pragma unroll
    for (int k = 0; k < PPT; ++k) {
      const int i = tid + k * NT;
      const int py = i / PX, px = i - py * PX;
      const int iy = iy0 + py, ix = ix0 + px;
      pre[k][0] = pre[k][1] = pre[k][2] = (S)0.f;
      if (i < PY * PX && (unsigned)iy < (unsigned)p.H && (unsigned)ix < (unsigned)p.W && p.variant != 2) {
        const size_t o = (size_t)iy * p.W + ix;
        pre[k][0] = xb[o];
        pre[k][1] = xb[o + (size_t)p.H * p.W];
        pre[k][2] = xb[o + 2 * (size_t)p.H * p.W];
      }
    }
  };
  auto commit = [&]() {
#pragma unroll
    for (int k = 0; k < PPT; ++k) {
      const int i = tid + k * NT;
      typedef _Float16 h4 __attribute__((ext_vector_type(4)));
      const h4 v = {(_Float16)(float)pre[k][0], (_Float16)(float)pre[k][1], (_Float16)(float)pre[k][2],
                    (_Float16)0.f};
      if (i < PY * PX) *reinterpret_cast<h4*>(patch + i * 4) = v;
    }
  };
  // conv A's K layout on the MFMA: 4 halves per tap (3 channels + the patch's zero 4th channel),
  // two taps per 8-half lane group, so a lane's A fragment is two 8-byte patch pixels — for the
  // horizontally adjacent pairs one contiguous 16 bytes — instead of eight scattered halves.
  //   K step 0: g0 taps (0,0)(0,1), g1 (1,0)(1,1), g2 (2,0)(2,1), g3 (0,2)(1,2);  K step 1: g0 (2,2).
  // SiLU is folded (ACT_A == 1): conv A's weights and bias are scaled by -log2(e) at load, so the
  // MFMA yields z = -log2(e) x, the epilogue stores z * rcp(1 + 2^z) = -log2(e) * silu(x), and conv B
  // compensates with its bias scaled by -log2(e) (then it too yields -log2(e) x_B).
  constexpr float NLOG2E = -1.4426950408889634f;
  const float sa_scale = ACT_A == 1 ? NLOG2E : 1.0f;
  const float sb_scale = ACT_A == 1 ? NLOG2E : 1.0f;   // conv B's pre-activation scale
  auto tap_of = [](int ks, int gg, int half) -> int {   // (r*3 + s) of lane group gg, half 0/1; -1 = none
    if (ks == 0) {
      if (gg < 3) return gg * 3 + half;                 // (gg, 0), (gg, 1)
      return half == 0 ? 2 : 5;                         // (0, 2), (1, 2)
    }
    return (gg == 0 && half == 0) ? 8 : -1;             // (2, 2)
  };
  constexpr int NAT = CA / 16;
  u4 wa[2][NAT];
#pragma unroll
  for (int ks = 0; ks < 2; ++ks)
#pragma unroll
    for (int nt = 0; nt < NAT; ++nt) {
      typedef _Float16 h8v __attribute__((ext_vector_type(8)));
      h8v w8;
      const _Float16* wrow = reinterpret_cast<const _Float16*>(p.wa) + (size_t)(nt * 16 + li) * p.kpad_a;
#pragma unroll
      for (int h2 = 0; h2 < 2; ++h2) {
        const int tap = tap_of(ks, g, h2);
#pragma unroll
        for (int ci = 0; ci < 4; ++ci)
          w8[h2 * 4 + ci] = (tap >= 0 && ci < 3) ? (_Float16)((float)wrow[tap * 3 + ci] * sa_scale) : (_Float16)0.f;
      }
      wa[ks][nt] = __builtin_bit_cast(u4, w8);
    }
  // patch byte offsets (relative to the A-pixel's patch origin) of this lane's two taps per K step
  int toff[2][2];
#pragma unroll
  for (int ks = 0; ks < 2; ++ks)
#pragma unroll
    for (int h2 = 0; h2 < 2; ++h2) {
      const int tap = tap_of(ks, g, h2);
      toff[ks][h2] = tap >= 0 ? ((tap / 3) * PX + tap % 3) * 8 : -1;
    }
  float ba_l[NAT][4];
#pragma unroll
  for (int nt = 0; nt < NAT; ++nt)
#pragma unroll
    for (int e = 0; e < 4; ++e) ba_l[nt][e] = p.ba[nt * 16 + g * 4 + e] * sa_scale;
  // XCD-major tile order: the blocks of one XCD (blockIdx % 8 on the round-robin dispatch) walk
  // consecutive tiles, so the image lines two horizontally / vertically adjacent tiles share are
  // fetched into that XCD's L2 once (row-order assignment spread neighbours over all 8 L2s: 4.5x
  // the image's bytes read from HBM)
  const int G = gridDim.x;
  const int vb = G % 8 == 0 ? (int)(blockIdx.x % 8) * (G / 8) + (int)(blockIdx.x / 8) : (int)blockIdx.x;
  if (vb < ntiles) prefetch(vb);
  for (int tile = vb; tile < ntiles; tile += G) {
  tile_geom(tile, b, oy0, ox0);
  ay0 = 2 * oy0 - 1;
  ax0 = 2 * ox0 - 1;
  commit();
  if (tile + G < ntiles) prefetch(tile + G);
  __syncthreads();

  // 2. conv A on MFMA -> abuf
  const unsigned char* pbytes = reinterpret_cast<const unsigned char*>(patch);
  typedef uint32_t u2 __attribute__((ext_vector_type(2)));
  for (int mt = wave; mt < MA; mt += 4) {
    const int m = mt * 16 + li;
    const int mc = m < NA ? m : NA - 1;
    const int yl = mc / TAX, xl = mc - yl * TAX;
    const int base = (SA * yl * PX + SA * xl) * 8;
    u4 xv[2];
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      u2 lo = {0u, 0u}, hi = {0u, 0u};
      if (toff[ks][0] >= 0) lo = *reinterpret_cast<const u2*>(pbytes + base + toff[ks][0]);
      if (toff[ks][1] >= 0) hi = *reinterpret_cast<const u2*>(pbytes + base + toff[ks][1]);
      xv[ks] = u4{lo[0], lo[1], hi[0], hi[1]};
    }
    const int ay = ay0 + yl, ax = ax0 + xl;
    const bool inside = m < NA && (unsigned)ay < (unsigned)HA && (unsigned)ax < (unsigned)WA;
#pragma unroll
    for (int nt = 0; nt < NAT; ++nt) {
      f4 acc = {ba_l[nt][0], ba_l[nt][1], ba_l[nt][2], ba_l[nt][3]};
      acc = __builtin_amdgcn_mfma_f32_16x16x32_f16(__builtin_bit_cast(h8, wa[0][nt]), __builtin_bit_cast(h8, xv[0]),
                                                   acc, 0, 0, 0);
      acc = __builtin_amdgcn_mfma_f32_16x16x32_f16(__builtin_bit_cast(h8, wa[1][nt]), __builtin_bit_cast(h8, xv[1]),
                                                   acc, 0, 0, 0);
      typedef _Float16 h4 __attribute__((ext_vector_type(4)));
      h4 o;
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        float v;
        if (p.variant == 1) v = acc[e];
        else if constexpr (ACT_A == 1) v = acc[e] * __builtin_amdgcn_rcpf(1.0f + __builtin_amdgcn_exp2f(acc[e]));
        else v = act_t<ACT_A>(acc[e]);
        o[e] = inside ? (_Float16)v : (_Float16)0.f;
      }
      if (m < NA) *reinterpret_cast<h4*>(abuf + m * APITCH + (nt * 16 + g * 4) * 2) = o;
    }
  }
  __syncthreads();

  // 3. conv B: wave w owns output channels [16w, 16w+16) for every pixel of the tile; its 9 taps of
  //    weight fragments were loaded at kernel entry (wfr), so no global load sits in this loop.
  f4 acc[MB];
  {
    f4 bv;
#pragma unroll
    for (int e = 0; e < 4; ++e) bv[e] = p.bb[wave * 16 + g * 4 + e] * sb_scale;
#pragma unroll
    for (int i = 0; i < MB; ++i) acc[i] = bv;
  }
#pragma unroll
  for (int tap = 0; tap < 9; ++tap) {
    if (p.variant == 3) break;   // microbenchmark hook: no conv B
    const int r = tap / 3, s = tap - r * 3;
#pragma unroll
    for (int i = 0; i < MB; ++i) {
      const int mb = i * 16 + li;                          // conv-B pixel within the tile
      const int ty = mb / TBX, tx = mb - ty * TBX;
      const int ap = (2 * ty + r) * TAX + (2 * tx + s);    // conv-A pixel (local)
      const u4 xa = *reinterpret_cast<const u4*>(abuf + ap * APITCH + g * 16);
      acc[i] = __builtin_amdgcn_mfma_f32_16x16x32_f16(__builtin_bit_cast(h8, wfr[tap]), __builtin_bit_cast(h8, xa),
                                                      acc[i], 0, 0, 0);
    }
  }
  __syncthreads();

  // 4. epilogue via LDS: lane holds 4 consecutive channels of one conv-B pixel
  {
    const int col = wave * 16 + g * 4;
    // acc = sb_scale * x_B: undo the scale (SiLU: x = -ln2 * z, silu = x * rcp(1 + 2^z))
#pragma unroll
    for (int i = 0; i < MB; ++i) {
      const int mb = i * 16 + li;
      typedef _Float16 h4 __attribute__((ext_vector_type(4)));
      h4 o;
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        float v;
        if constexpr (ACT_A == 1 && ACT_B == 1)
          v = (acc[i][e] * -0.6931471805599453f) * __builtin_amdgcn_rcpf(1.0f + __builtin_amdgcn_exp2f(acc[i][e]));
        else
          v = act_t<ACT_B>(acc[i][e] / sb_scale);
        o[e] = (_Float16)v;
      }
      *reinterpret_cast<h4*>(smem + mb * CPITCH + col * 2) = o;
    }
  }
  __syncthreads();
  constexpr int CPR = CB * 2 / 16;
  _Float16* y = reinterpret_cast<_Float16*>(p.y);
  for (int c = tid; c < TBY * TBX * CPR; c += NT) {
    const int mb = c / CPR, ch = c - mb * CPR;
    const int ty = mb / TBX, tx = mb - ty * TBX;
    const int oy = oy0 + ty, ox = ox0 + tx;
    if (oy < HB && ox < WB && p.variant != 4)
      *reinterpret_cast<u4*>(y + pix_index(b, oy, ox, HB, WB) * p.yc + p.yoff + ch * 8) =
          *reinterpret_cast<const u4*>(smem + mb * CPITCH + ch * 16);
  }
  __syncthreads();   // the output staging overlaps the next tile's patch
  }
}

// Second form (the default; YV7_STEM=1 selects the kernel above).  Same tile, same arithmetic bit for
// bit, restructured after its microbenchmark hooks (scripts/stembench.hip: conv B's 72 ds_read_b128
// per wave per tile cost as much as its MFMAs, the two not overlapping; 5 barriers per tile):
//   * conv B: wave w owns 4 m-tiles x 2 n-tiles (32 output channels, 18 weight fragments in registers)
//     instead of 8 m-tiles x 16 channels: half the LDS reads of conv A's tile for the same MFMAs;
//   * conv A: m-tiles in groups of three (12 MFMAs issued back to back, then their activations);
//   * the output staging tile has its own LDS (patch + A tile + staging = 68.6 KB, two blocks per CU),
//     so a tile needs 3 barriers: [stores of t-1, patch of t] | conv A | conv B + staging;
//   * both biases in registers from kernel entry (no global load inside the tile loop).
template <typename S, int CA, int CB, int SA, int TBY, int TBX, int ACT_A, int ACT_B>
__global__ __launch_bounds__(NT, 2) void stem2_kernel(const StemParams p) {
  constexpr int TAY = 2 * TBY + 1, TAX = 2 * TBX + 1;
  constexpr int PY = SA * (TAY - 1) + 3, PX = SA * (TAX - 1) + 3;
  constexpr int NA = TAY * TAX;
  constexpr int MA = (NA + 15) / 16;
  constexpr int APITCH = CA * 2 + 16;
  constexpr int PATCH = (PY * PX * 8 + 15) / 16 * 16;
  constexpr int ABUF = MA * 16 * APITCH;            // whole m-tiles: conv A's writes need no row guard
  constexpr int MB = TBY * TBX / 16;
  constexpr int CPITCH = CB * 2 + 16;
  constexpr int OUTB = TBY * TBX * CPITCH;
  static_assert(CB == 64 && CA == 32, "4 waves = 2 m-groups x 2 n-groups of 32 channels; one MFMA k-step per tap");
  static_assert(MB == 8 && MA % 12 == 0, "conv B: 4 m-tiles per wave; conv A: groups of 3 m-tiles per wave");
  __shared__ __attribute__((aligned(16))) unsigned char smem[PATCH + ABUF + OUTB];
  _Float16* patch = reinterpret_cast<_Float16*>(smem);
  unsigned char* abuf0 = smem + PATCH;
  unsigned char* obuf = smem + PATCH + ABUF;

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int g = lane >> 4, li = lane & 15;
  const int mg = wave >> 1, ng = wave & 1;        // conv B: m-tiles [4 mg, 4 mg + 4), channels [32 ng, 32 ng + 32)
  const int HA = p.H / SA, WA = p.W / SA;
  const int HB = HA / 2, WB = WA / 2;
  const int tiles_x = (WB + TBX - 1) / TBX, tiles_y = (HB + TBY - 1) / TBY;
  const int ntiles = p.B * tiles_x * tiles_y;
  auto tile_geom = [&](int t, int& tb, int& ty, int& tx) {
    tb = t / (tiles_x * tiles_y);
    t -= tb * tiles_x * tiles_y;
    ty = (t / tiles_x) * TBY;
    tx = (t % tiles_x) * TBX;
  };
  constexpr float NLOG2E = -1.4426950408889634f;
  const float sa_scale = ACT_A == 1 ? NLOG2E : 1.0f;
  const float sb_scale = ACT_A == 1 ? NLOG2E : 1.0f;

  // conv-B weight fragments: this wave's 2 n-tiles x 9 taps
  u4 wfr[2][9];
#pragma unroll
  for (int j = 0; j < 2; ++j)
#pragma unroll
    for (int tap = 0; tap < 9; ++tap)
      wfr[j][tap] = *reinterpret_cast<const u4*>(reinterpret_cast<const _Float16*>(p.wb) +
                                                 (size_t)((2 * ng + j) * 16 + li) * p.kpad_b + tap * CA + g * 8);
  float bb_l[2][4];
#pragma unroll
  for (int j = 0; j < 2; ++j)
#pragma unroll
    for (int e = 0; e < 4; ++e) bb_l[j][e] = p.bb[(2 * ng + j) * 16 + g * 4 + e] * sb_scale;

  // The image patch: fp16 input (the bench path) moves horizontally adjacent pixel PAIRS — one dword
  // per channel plane (the patch's x origin 2 tx - 2 is even and so is W, so a pair lies wholly inside
  // or wholly outside the image), a third of the load instructions of one pixel per lane; fp32 input
  // one pixel per lane.  Raw loaded bits stay untouched until the commit: converting or packing them
  // right after the loads makes the wave wait on them there instead of a tile later.
  constexpr bool PAIRS = sizeof(S) == 2;
  constexpr int UPR = PAIRS ? (PX + 1) / 2 : PX;        // load units per patch row
  constexpr int PPT = (PY * UPR + NT - 1) / NT;
  uint32_t pre[PPT][3];
  // unconditional buffer loads (outside the image: an offset past the buffer reads zero), so no branch
  // hides them from the compiler's wait counting
  const uint32_t plane = (uint32_t)(p.H * p.W * sizeof(S));
  const auto xr = make_rsrc(p.x, (uint32_t)((size_t)p.B * 3 * plane));
  // per-thread unit geometry, fixed across tiles
  int u_py[PPT], u_px[PPT];
#pragma unroll
  for (int k = 0; k < PPT; ++k) {
    const int i = tid + k * NT;
    u_py[k] = i < PY * UPR ? i / UPR : -0x40000;   // units past the patch: a row that is never inside
    u_px[k] = (PAIRS ? 2 : 1) * (i - (i / UPR) * UPR);
  }
  auto prefetch = [&](int t) {
    int tb, ty, tx;
    tile_geom(t, tb, ty, tx);
    const int iy0 = SA * (2 * ty - 1) - 1, ix0 = SA * (2 * tx - 1) - 1;
    const uint32_t img = (uint32_t)tb * 3u * plane;
#pragma unroll
    for (int k = 0; k < PPT; ++k) {
      const int iy = iy0 + u_py[k], ix = ix0 + u_px[k];
      const bool in = (unsigned)iy < (unsigned)p.H && (unsigned)ix < (unsigned)p.W && p.variant != 2;
      // 24-bit multiply (a v_mad_u64_u32 here took a pending load's register as its don't-care high
      // half, stalling the prefetch on its own loads)
      const uint32_t o = in ? img + (__umul24(iy, p.W) + ix) * (uint32_t)sizeof(S) : 0x80000000u;
#pragma unroll
      for (int ch = 0; ch < 3; ++ch) pre[k][ch] = __builtin_amdgcn_raw_buffer_load_b32(xr, o + ch * plane, 0, 0);
    }
  };
  auto commit = [&]() {
    typedef _Float16 h4 __attribute__((ext_vector_type(4)));
#pragma unroll
    for (int k = 0; k < PPT; ++k) {
      const int i = tid + k * NT;
#pragma unroll
      for (int ch = 0; ch < 3; ++ch) asm volatile("" : "+v"(pre[k][ch]));
      if constexpr (PAIRS) {
        typedef _Float16 h2 __attribute__((ext_vector_type(2)));
        const h2 c0 = __builtin_bit_cast(h2, pre[k][0]), c1 = __builtin_bit_cast(h2, pre[k][1]),
                 c2 = __builtin_bit_cast(h2, pre[k][2]);
        const int py = i / UPR, px = 2 * (i - py * UPR);
        if (i < PY * UPR) {
          *reinterpret_cast<h4*>(patch + (py * PX + px) * 4) = h4{c0[0], c1[0], c2[0], (_Float16)0.f};
          if (px + 1 < PX) *reinterpret_cast<h4*>(patch + (py * PX + px + 1) * 4) = h4{c0[1], c1[1], c2[1], (_Float16)0.f};
        }
      } else {
        const h4 v = {(_Float16)__builtin_bit_cast(float, pre[k][0]), (_Float16)__builtin_bit_cast(float, pre[k][1]),
                      (_Float16)__builtin_bit_cast(float, pre[k][2]), (_Float16)0.f};
        if (i < PY * PX) *reinterpret_cast<h4*>(patch + i * 4) = v;
      }
    }
  };
  // conv A's K layout (as stem_kernel): two taps per 8-half lane group
  auto tap_of = [](int ks, int gg, int half) -> int {
    if (ks == 0) {
      if (gg < 3) return gg * 3 + half;
      return half == 0 ? 2 : 5;
    }
    return (gg == 0 && half == 0) ? 8 : -1;
  };
  // Slots with no tap (K step 1 but for tap (2,2)) read patch pixel 0 against zero weights.
  constexpr int NAT = CA / 16;
  u4 wa[2][NAT];
#pragma unroll
  for (int ks = 0; ks < 2; ++ks)
#pragma unroll
    for (int nt = 0; nt < NAT; ++nt) {
      typedef _Float16 h8v __attribute__((ext_vector_type(8)));
      h8v w8;
      const _Float16* wrow = reinterpret_cast<const _Float16*>(p.wa) + (size_t)(nt * 16 + li) * p.kpad_a;
#pragma unroll
      for (int h2 = 0; h2 < 2; ++h2) {
        const int tap = tap_of(ks, g, h2);
#pragma unroll
        for (int ci = 0; ci < 3; ++ci)
          w8[h2 * 4 + ci] = tap >= 0 ? (_Float16)((float)wrow[tap * 3 + ci] * sa_scale) : (_Float16)0.f;
        w8[h2 * 4 + 3] = (_Float16)0.f;
      }
      wa[ks][nt] = __builtin_bit_cast(u4, w8);
    }
  int toff[2][2];
#pragma unroll
  for (int ks = 0; ks < 2; ++ks)
#pragma unroll
    for (int h2 = 0; h2 < 2; ++h2) {
      const int tap = tap_of(ks, g, h2);
      toff[ks][h2] = tap >= 0 ? ((tap / 3) * PX + tap % 3) * 8 : 0;
    }
  float ba_l[NAT][4];   // conv A's bias (scaled like its weights) as the accumulators' start
#pragma unroll
  for (int nt = 0; nt < NAT; ++nt)
#pragma unroll
    for (int e = 0; e < 4; ++e) ba_l[nt][e] = p.ba[nt * 16 + g * 4 + e] * sa_scale;

  const int G = gridDim.x;
  const int vb = G % 8 == 0 ? (int)(blockIdx.x % 8) * (G / 8) + (int)(blockIdx.x / 8) : (int)blockIdx.x;
  if (vb < ntiles) prefetch(vb);
  int pb = -1, poy0 = 0, pox0 = 0;   // the previous tile (its staged output is stored in this iteration)
  // output stores likewise unconditional (a pixel past the image edge stores past the buffer: dropped)
  const auto yr = make_rsrc(p.y, (uint32_t)(bordered_pixels(p.B, HB, WB) * p.yc * 2));
  // per-thread store geometry: staging chunk -> (pixel row, column, channel byte offset)
  // (chunk c = tid + k NT: NT is a whole number of pixel rows of chunks, so store k is the thread's
  // pixel of row s_ty0 + k * NT / (TBX * CPR), the rest fixed: one base per thread, compile-time steps)
  constexpr int CPR = CB * 2 / 16;
  constexpr int NSTO = TBY * TBX * CPR / NT;
  static_assert(NT % (TBX * CPR) == 0, "whole staging rows per store round");
  constexpr int RSTEP = NT / (TBX * CPR);
  const int s_mb0 = tid / CPR, s_ch = tid - s_mb0 * CPR;
  const int s_ty0 = s_mb0 / TBX, s_tx = s_mb0 - s_ty0 * TBX;
  const int s_mbo0 = s_mb0 * CPITCH + s_ch * 16;
  const uint32_t s_rel0 = (uint32_t)(((s_ty0 * (WB + 2 * BORDER) + s_tx) * p.yc + p.yoff + s_ch * 8) * 2);
  const uint32_t s_rstep = (uint32_t)(RSTEP * (WB + 2 * BORDER) * p.yc * 2);
  auto store_prev = [&]() {
    if (pb < 0) return;
    const uint32_t tile_off = (uint32_t)(pix_index(pb, poy0, pox0, HB, WB) * p.yc * 2) + s_rel0;
#pragma unroll
    for (int k = 0; k < NSTO; ++k) {
      const bool in = poy0 + s_ty0 + k * RSTEP < HB && pox0 + s_tx < WB && p.variant != 4;
      __builtin_amdgcn_raw_buffer_store_b128(*reinterpret_cast<const u4*>(obuf + s_mbo0 + k * RSTEP * TBX * CPITCH), yr,
                                             in ? tile_off + k * s_rstep : 0x80000000u, 0, 0);
    }
  };
  // conv A of one group of three m-tiles (of 36) -> the A tile at ab
  const unsigned char* pbytes = reinterpret_cast<const unsigned char*>(patch);
  typedef uint32_t u2 __attribute__((ext_vector_type(2)));
  // this lane's A-pixel of each of its MA / 4 m-tiles (m-tile 4 k + wave, k = 3 grp + u): patch byte base,
  // fixed across tiles — hoisted out of the tile loop, and the image-border mask computed only on border
  // tiles (the division by TAX, the offsets and the mask were ~30 of the ~170 VALU instructions of every
  // group of three m-tiles)
  constexpr int NMW = MA / 4;
  int pbase9[NMW];
#pragma unroll
  for (int k = 0; k < NMW; ++k) {
    const int m = k * 4 * 16 + wave * 16 + li;
    const int mc = m < NA ? m : NA - 1;   // rows past NA: computed, never read by conv B
    const int yl = mc / TAX, xl = mc - yl * TAX;
    pbase9[k] = (SA * yl * PX + SA * xl) * 8;
  }
  const int mlane = wave * 16 + li;
  auto conv_a_group = [&](auto grpc, unsigned char* ab, int ay0, int ax0, bool interior) __attribute__((always_inline)) {
    constexpr int grp = decltype(grpc)::value;
    u4 xv[3][2];
    uint32_t keep[3] = {~0u, ~0u, ~0u};
#pragma unroll
    for (int u = 0; u < 3; ++u) {
      const int base = pbase9[grp * 3 + u];
#pragma unroll
      for (int ks = 0; ks < 2; ++ks) {
        const u2 lo = *reinterpret_cast<const u2*>(pbytes + base + toff[ks][0]);
        const u2 hi = *reinterpret_cast<const u2*>(pbytes + base + toff[ks][1]);
        xv[u][ks] = u4{lo[0], lo[1], hi[0], hi[1]};
      }
    }
    if (!interior) {   // tiles on the image border: zero the A pixels outside it (conv B's padding)
#pragma unroll
      for (int u = 0; u < 3; ++u) {
        const int m = (grp * 3 + u) * 4 * 16 + mlane;
        const int mc = m < NA ? m : NA - 1;
        const int yl = mc / TAX, xl = mc - yl * TAX;
        const int ay = ay0 + yl, ax = ax0 + xl;
        keep[u] = ((unsigned)ay < (unsigned)HA && (unsigned)ax < (unsigned)WA) ? ~0u : 0u;
      }
    }
    f4 acc[3][NAT];
#pragma unroll
    for (int u = 0; u < 3; ++u)
#pragma unroll
      for (int nt = 0; nt < NAT; ++nt) {
        const f4 a = __builtin_amdgcn_mfma_f32_16x16x32_f16(__builtin_bit_cast(h8, wa[0][nt]), __builtin_bit_cast(h8, xv[u][0]),
                                                             f4{ba_l[nt][0], ba_l[nt][1], ba_l[nt][2], ba_l[nt][3]}, 0, 0, 0);
        acc[u][nt] = __builtin_amdgcn_mfma_f32_16x16x32_f16(__builtin_bit_cast(h8, wa[1][nt]),
                                                            __builtin_bit_cast(h8, xv[u][1]), a, 0, 0, 0);
      }
#pragma unroll
    for (int u = 0; u < 3; ++u)
#pragma unroll
      for (int nt = 0; nt < NAT; ++nt) {
        typedef _Float16 h2 __attribute__((ext_vector_type(2)));
        float v[4];
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          if constexpr (ACT_A == 1) v[e] = acc[u][nt][e] * __builtin_amdgcn_rcpf(1.0f + __builtin_amdgcn_exp2f(acc[u][nt][e]));
          else v[e] = act_t<ACT_A>(acc[u][nt][e]);
        }
        // zero outside the image (conv B's padding): one mask per packed pair of halves
        const u2 o = {__builtin_bit_cast(uint32_t, h2{(_Float16)v[0], (_Float16)v[1]}) & keep[u],
                      __builtin_bit_cast(uint32_t, h2{(_Float16)v[2], (_Float16)v[3]}) & keep[u]};
        *reinterpret_cast<u2*>(ab + ((grp * 3 + u) * 4 * 16 + mlane) * APITCH + (nt * 16 + g * 4) * 2) = o;
      }
  };
  // conv B: 4 m-tiles x 2 n-tiles per wave, taps [t0, t0 + 3)
  auto conv_b_taps = [&](int t0, const unsigned char* ab, f4 (&acc)[4][2]) __attribute__((always_inline)) {
    if (p.variant == 3) return;
#pragma unroll
    for (int tap = t0; tap < t0 + 3; ++tap) {
      const int r = tap / 3, s = tap - r * 3;
      u4 xa[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int mb = (4 * mg + i) * 16 + li;
        const int ty = mb / TBX, tx = mb - ty * TBX;
        const int ap = (2 * ty + r) * TAX + (2 * tx + s);
        xa[i] = *reinterpret_cast<const u4*>(ab + ap * APITCH + g * 16);
      }
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(__builtin_bit_cast(h8, wfr[j][tap]),
                                                             __builtin_bit_cast(h8, xa[i]), acc[i][j], 0, 0, 0);
    }
  };
  auto conv_b_init = [&](f4 (&acc)[4][2]) __attribute__((always_inline)) {
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 2; ++j) acc[i][j] = f4{bb_l[j][0], bb_l[j][1], bb_l[j][2], bb_l[j][3]};
  };
  // conv B's activation -> staging tile
  auto conv_b_out = [&](f4 (&acc)[4][2]) __attribute__((always_inline)) {
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        const int mb = (4 * mg + i) * 16 + li;
        const int col = (2 * ng + j) * 16 + g * 4;
        typedef _Float16 h4 __attribute__((ext_vector_type(4)));
        h4 o;
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          float v;
          if constexpr (ACT_A == 1 && ACT_B == 1)
            v = (acc[i][j][e] * -0.6931471805599453f) * __builtin_amdgcn_rcpf(1.0f + __builtin_amdgcn_exp2f(acc[i][j][e]));
          else
            v = act_t<ACT_B>(acc[i][j][e] / sb_scale);
          o[e] = (_Float16)v;
        }
        *reinterpret_cast<h4*>(obuf + mb * CPITCH + col * 2) = o;
      }
  };
  auto origin = [&](int t, int& b, int& oy0, int& ox0, int& ay0, int& ax0) {
    tile_geom(t, b, oy0, ox0);
    ay0 = 2 * oy0 - 1;
    ax0 = 2 * ox0 - 1;
  };

  {
    for (int tile = vb; tile < ntiles; tile += G) {
      int b, oy0, ox0, ay0, ax0;
      origin(tile, b, oy0, ox0, ay0, ax0);
      commit();
      if (tile + G < ntiles) prefetch(tile + G);
      store_prev();
      __syncthreads();   // patch of this tile in LDS; staging of the previous one read
      static_assert(MA == 36, "three groups of three m-tiles per wave");
      const bool interior = ay0 >= 0 && ax0 >= 0 && ay0 + TAY <= HA && ax0 + TAX <= WA;
      conv_a_group(std::integral_constant<int, 0>{}, abuf0, ay0, ax0, interior);
      conv_a_group(std::integral_constant<int, 1>{}, abuf0, ay0, ax0, interior);
      conv_a_group(std::integral_constant<int, 2>{}, abuf0, ay0, ax0, interior);
      __syncthreads();   // A tile complete
      f4 acc[4][2];
      conv_b_init(acc);
#pragma unroll
      for (int t0 = 0; t0 < 9; t0 += 3) conv_b_taps(t0, abuf0, acc);
      conv_b_out(acc);
      pb = b;
      poy0 = oy0;
      pox0 = ox0;
      __syncthreads();   // staging complete (stored at the top of the next iteration)
    }
  }
  store_prev();
}

// The yolov7-w6 front end: ReOrg (space-to-depth 2x, models/common.py:48-53) + conv A (12 -> 64, 3x3,
// stride 1, on the 640^2 reorganised image) + conv B (64 -> 128, 3x3, stride 2), cfg/deploy/
// yolov7-w6.yaml:14-16.  Unfused these are three launches (the reorg packing, 36 us, conv A, 241 us,
// conv B, 190 us at 1280^2 bs 8) around conv A's output, the largest tensor of the network (8 x 640^2 x
// 64 fp16 = 419 MB, written once and read back through L2 by the stride-2 conv).
//
// Fused, one persistent 512-thread block per CU walks tiles of 4 x 16 conv-B output pixels, with the
// waves split by role (one of each on every SIMD) and one barrier per tile:
//   * A waves (0-3), tile t + 1: conv A on the MFMA — 9 x 33 A-pixels (20 m-tiles, padded) x 64
//     channels, K = 9 taps x 16 channels (two taps per 16x16x32 K step, the fifth half zero weights);
//     wave w: all 64 channels of m-tiles w, w + 4, ... (each patch read feeds 4 MFMAs), its 4 x 5 weight
//     fragments in registers; + bias + act,
//     zeroed outside the image (conv B's padding) -> A tile [A-pixel][64] (144-byte pitch, conflict-free
//     for conv B's stride-2 reads), double-buffered.  Then the patch of tile t + 2 (loaded into
//     registers during the previous tile) is committed to LDS and tile t + 3's is loaded: 11 x 35
//     reorganised pixels x 16 halves (12 channels + 4 zero), gathered straight from the NCHW image — one
//     dword load per (row parity, channel) covers a pixel's two raw columns, i.e. reorganised channels
//     q*3 + c for q = rp (even column) and rp + 2 (odd column); double-buffered.
//   * B waves (4-7), tile t: conv B on the MFMA — wave w owns output channels [32 (w-4), +32) for all 64
//     pixels, its 2 x 18 weight fragments in registers; + bias + act -> the wave's own staging rows ->
//     16-byte stores into the destination slice (no cross-wave exchange, so no barrier).
// The A waves' SiLU (64 x 297 values per tile) and the B waves' MFMAs (576 per tile) thus issue side by
// side on each SIMD instead of in turn behind barriers (the 4-wave form, one role after the other with
// three barriers per tile: 360 vs 313... us, scripts/stembench.hip).
// Arithmetic as stem2_kernel's: with SiLU, conv A's weights / bias pre-scaled by -log2(e) and its
// activations stored in fp16 as -log2(e) silu(a) (tests/opcheck.py restates it); fp32 accumulation.
constexpr int NT_RG = 512;

template <typename S, int ACT_A, int ACT_B>
__global__ __launch_bounds__(NT_RG, 1) void stem_reorg_kernel(const StemParams p) {
  constexpr int CA = 64, TBY = 4, TBX = 16;   // (conv B: 128 channels)
  constexpr int TAY = 2 * TBY + 1, TAX = 2 * TBX + 1;   // conv-A pixels feeding the tile: 9 x 33
  constexpr int NA = TAY * TAX;                          // 297
  constexpr int MA = 20;                                 // conv-A m-tiles (padded)
  constexpr int PY = TAY + 2, PX = TAX + 2, NPIX = PY * PX;   // reorganised patch 11 x 35
  constexpr int APITCH = CA * 2 + 16;
  constexpr int PATCH = NPIX * 32;
  constexpr int ABUF = MA * 16 * APITCH;
  constexpr int SPITCH = 32 * 2 + 16;                    // a B wave's staging row: 32 channels
  constexpr int STG = TBY * TBX * SPITCH;
  static_assert(MA * 16 >= NA, "conv A's m-tiles cover the A pixels");
  static_assert(2 * PATCH + 2 * ABUF + 4 * STG <= 160 * 1024, "LDS");
  __shared__ __attribute__((aligned(16))) unsigned char smem[2 * PATCH + 2 * ABUF + 4 * STG];

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int g = lane >> 4, li = lane & 15;
  const int HA = p.H / 2, WA = p.W / 2;            // the reorganised image = conv A's output grid
  const int HB = HA / 2, WB = WA / 2;
  const int tiles_x = (WB + TBX - 1) / TBX, tiles_y = (HB + TBY - 1) / TBY;
  const int ntiles = p.B * tiles_x * tiles_y;
  auto tile_geom = [&](int t, int& tb, int& ty, int& tx) {
    tb = t / (tiles_x * tiles_y);
    t -= tb * tiles_x * tiles_y;
    ty = (t / tiles_x) * TBY;
    tx = (t % tiles_x) * TBX;
  };
  // this block's tiles: vb, vb + G, ... (XCD-major virtual block index, as stem2_kernel)
  const int G = gridDim.x;
  const int vb = G % 8 == 0 ? (int)(blockIdx.x % 8) * (G / 8) + (int)(blockIdx.x / 8) : (int)blockIdx.x;
  const int nmine = vb < ntiles ? (ntiles - vb + G - 1) / G : 0;
  auto tile_of = [&](int i) { return vb + i * G; };

  if (wave < 4) {
    // ---------------- A waves: patches + conv A ----------------
    const int w = wave;
    // all 64 channels (4 n-tiles x 5 K steps of weight fragments) for m-tiles w, w + 4, ...: every patch
    // read feeds 4 MFMAs.  SiLU folded as in stem2_kernel: weights and bias scaled by -log2(e) (weights
    // rounded to fp16 again), so the MFMA yields z = -log2(e) a and the A tile holds z / (1 + 2^z) =
    // -log2(e) silu(a); conv B's bias carries the same scale and its epilogue undoes it.
    constexpr float NLOG2E = -1.4426950408889634f;
    const float sa = ACT_A == 1 ? NLOG2E : 1.0f;
    u4 wa[5][4];
    f4 ba_l[4];
#pragma unroll
    for (int nt = 0; nt < 4; ++nt) {
      const _Float16* wrow = reinterpret_cast<const _Float16*>(p.wa) + (size_t)(nt * 16 + li) * p.kpad_a + g * 8;
#pragma unroll
      for (int ks = 0; ks < 5; ++ks) {
        h8 w8 = __builtin_bit_cast(h8, *reinterpret_cast<const u4*>(wrow + ks * 32));
#pragma unroll
        for (int e = 0; e < 8; ++e) w8[e] = (_Float16)((float)w8[e] * sa);
        wa[ks][nt] = __builtin_bit_cast(u4, w8);
      }
      ba_l[nt] = *reinterpret_cast<const f4*>(p.ba + nt * 16 + g * 4) * sa;
    }
    // patch byte offset of this lane's tap in K step ks (tap 9 = none: tap 8's pixel against zero weights)
    int toff[5];
#pragma unroll
    for (int ks = 0; ks < 5; ++ks) {
      const int tap = min(2 * ks + (g >> 1), 8);
      toff[ks] = ((tap / 3) * PX + tap % 3) * 32 + (g & 1) * 16;
    }
    // patch units = reorganised pixels, two per thread; unconditional buffer loads (outside the image: an
    // offset past the buffer reads zero)
    const int ta = tid;   // 0..255
    constexpr int PPT = (NPIX + 255) / 256;
    constexpr bool HALF = sizeof(S) == 2;
    uint32_t pre[PPT][2][3];   // [unit][row parity][channel]: the two raw columns as packed halves
    const uint32_t plane = (uint32_t)(p.H * p.W * sizeof(S));
    const auto xr = make_rsrc(p.x, (uint32_t)((size_t)p.B * 3 * plane));
    auto prefetch = [&](int t) {
      int tb, ty, tx;
      tile_geom(t, tb, ty, tx);
      const int Y0 = 2 * ty - 2, X0 = 2 * tx - 2;   // patch origin on the reorganised grid
      const uint32_t img = (uint32_t)tb * 3u * plane;
#pragma unroll
      for (int k = 0; k < PPT; ++k) {
        const int u = ta + k * 256;
        const int py = u < NPIX ? u / PX : -0x40000, px = u - (u / PX) * PX;
        const int Y = Y0 + py, X = X0 + px;
        const bool in = (unsigned)Y < (unsigned)HA && (unsigned)X < (unsigned)WA && p.variant != 2;
#pragma unroll
        for (int rp = 0; rp < 2; ++rp) {
          const uint32_t o = in ? img + (__umul24(2 * Y + rp, p.W) + 2 * X) * (uint32_t)sizeof(S) : 0x80000000u;
#pragma unroll
          for (int c = 0; c < 3; ++c) {
            if constexpr (HALF) {
              pre[k][rp][c] = __builtin_amdgcn_raw_buffer_load_b32(xr, o + c * plane, 0, 0);
            } else {   // fp32 input: converted here (not the bench path)
              typedef float f2 __attribute__((ext_vector_type(2)));
              const f2 v = __builtin_bit_cast(f2, __builtin_amdgcn_raw_buffer_load_b64(xr, o + c * plane, 0, 0));
              typedef _Float16 h2 __attribute__((ext_vector_type(2)));
              pre[k][rp][c] = __builtin_bit_cast(uint32_t, h2{(_Float16)v[0], (_Float16)v[1]});
            }
          }
        }
      }
    };
    auto commit = [&](unsigned char* patch) {
      typedef _Float16 h2 __attribute__((ext_vector_type(2)));
#pragma unroll
      for (int k = 0; k < PPT; ++k) {
        const int u = ta + k * 256;
        _Float16 v[16];   // channel q * 3 + c, q = (row parity) + 2 (column parity)
#pragma unroll
        for (int rp = 0; rp < 2; ++rp)
#pragma unroll
          for (int c = 0; c < 3; ++c) {
            asm volatile("" : "+v"(pre[k][rp][c]));
            const h2 x2 = __builtin_bit_cast(h2, pre[k][rp][c]);
            v[rp * 3 + c] = x2[0];
            v[(rp + 2) * 3 + c] = x2[1];
          }
        h8 lo8, hi8;
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          lo8[e] = v[e];
          hi8[e] = e < 4 ? v[8 + e] : (_Float16)0.f;
        }
        if (u < NPIX) {
          *reinterpret_cast<u4*>(patch + u * 32) = __builtin_bit_cast(u4, lo8);
          *reinterpret_cast<u4*>(patch + u * 32 + 16) = __builtin_bit_cast(u4, hi8);
        }
      }
    };
    auto conv_a = [&](int t, const unsigned char* patch, unsigned char* abuf) {
      int tb, oy0, ox0;
      tile_geom(t, tb, oy0, ox0);
      const int ay0 = 2 * oy0 - 1, ax0 = 2 * ox0 - 1;
#pragma unroll 1
      for (int mt = w; mt < MA; mt += 4) {
        const int m = mt * 16 + li;
        const int mc = m < NA ? m : NA - 1;
        const int yl = mc / TAX, xl = mc - yl * TAX;
        const unsigned char* pp = patch + (yl * PX + xl) * 32;
        u4 xv[5];
#pragma unroll
        for (int ks = 0; ks < 5; ++ks) xv[ks] = *reinterpret_cast<const u4*>(pp + toff[ks]);
        const int ay = ay0 + yl, ax = ax0 + xl;
        const uint32_t keep = (m < NA && (unsigned)ay < (unsigned)HA && (unsigned)ax < (unsigned)WA) ? ~0u : 0u;
        f4 acc[4];
#pragma unroll
        for (int nt = 0; nt < 4; ++nt) acc[nt] = ba_l[nt];
#pragma unroll
        for (int ks = 0; ks < 5; ++ks)
#pragma unroll
          for (int nt = 0; nt < 4; ++nt)
            acc[nt] = __builtin_amdgcn_mfma_f32_16x16x32_f16(__builtin_bit_cast(h8, wa[ks][nt]),
                                                             __builtin_bit_cast(h8, xv[ks]), acc[nt], 0, 0, 0);
#pragma unroll
        for (int nt = 0; nt < 4; ++nt) {
          float v[4];
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            if constexpr (ACT_A == 1) v[e] = acc[nt][e] * __builtin_amdgcn_rcpf(1.0f + __builtin_amdgcn_exp2f(acc[nt][e]));
            else v[e] = act_t<ACT_A>(acc[nt][e]);
          }
          typedef _Float16 h2 __attribute__((ext_vector_type(2)));
          typedef uint32_t u2 __attribute__((ext_vector_type(2)));
          const u2 o = {__builtin_bit_cast(uint32_t, h2{(_Float16)v[0], (_Float16)v[1]}) & keep,
                        __builtin_bit_cast(uint32_t, h2{(_Float16)v[2], (_Float16)v[3]}) & keep};
          *reinterpret_cast<u2*>(abuf + m * APITCH + (nt * 16 + g * 4) * 2) = o;
        }
      }
    };
    unsigned char* P0 = smem;
    unsigned char* P1 = smem + PATCH;
    unsigned char* A0 = smem + 2 * PATCH;
    unsigned char* A1 = A0 + ABUF;
    // prologue: patches of tiles 0 and 1, loads of tile 2, conv A of tile 0
    if (nmine > 0) { prefetch(tile_of(0)); commit(P0); }
    if (nmine > 1) { prefetch(tile_of(1)); commit(P1); }
    if (nmine > 2) prefetch(tile_of(2));
    __syncthreads();
    if (nmine > 0) conv_a(tile_of(0), P0, A0);
    __syncthreads();
    for (int i = 0; i < nmine; ++i) {
      // phase i: the B waves run conv B of tile i from A[i % 2]; here conv A of tile i + 1
      if (i + 1 < nmine) conv_a(tile_of(i + 1), (i & 1) ? P0 : P1, (i & 1) ? A0 : A1);
      if (i + 2 < nmine) commit((i & 1) ? P1 : P0);   // P[i % 2]: tile i's patch, read in phase i - 1
      if (i + 3 < nmine) prefetch(tile_of(i + 3));
      __syncthreads();
    }
  } else {
    // ---------------- B waves: conv B + epilogue ----------------
    const int w = wave - 4;
    u4 wfr[18][2];   // k = tap * 64 + ci: 2 n-tiles x 18 K steps
#pragma unroll
    for (int kk = 0; kk < 18; ++kk)
#pragma unroll
      for (int j = 0; j < 2; ++j)
        wfr[kk][j] = *reinterpret_cast<const u4*>(reinterpret_cast<const _Float16*>(p.wb) +
                                                  (size_t)(w * 32 + j * 16 + li) * p.kpad_b + kk * 32 + g * 8);
    unsigned char* stg = smem + 2 * PATCH + 2 * ABUF + w * STG;
    const auto yr = make_rsrc(p.y, (uint32_t)(bordered_pixels(p.B, HB, WB) * p.yc * 2));
    __syncthreads();   // prologue: patches
    __syncthreads();   // prologue: conv A of tile 0
    for (int i = 0; i < nmine; ++i) {
      const unsigned char* abuf = smem + 2 * PATCH + (i & 1) * ABUF;
      f4 acc[4][2];
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        const f4 bv = *reinterpret_cast<const f4*>(p.bb + w * 32 + j * 16 + g * 4) * (ACT_A == 1 ? -1.4426950408889634f : 1.0f);
#pragma unroll
        for (int ii = 0; ii < 4; ++ii) acc[ii][j] = bv;
      }
      if (p.variant != 3) {
#pragma unroll
        for (int kk = 0; kk < 18; ++kk) {
          const int tap = kk >> 1, r = tap / 3, s = tap - r * 3;
          u4 xa[4];
#pragma unroll
          for (int ii = 0; ii < 4; ++ii)
            xa[ii] = *reinterpret_cast<const u4*>(abuf + ((2 * ii + r) * TAX + 2 * li + s) * APITCH + (kk & 1) * 64 + g * 16);
#pragma unroll
          for (int ii = 0; ii < 4; ++ii)
#pragma unroll
            for (int j = 0; j < 2; ++j)
              acc[ii][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(__builtin_bit_cast(h8, wfr[kk][j]),
                                                                  __builtin_bit_cast(h8, xa[ii]), acc[ii][j], 0, 0, 0);
        }
      }
      // epilogue: this wave's 32 channels of the 64 pixels -> its staging rows -> 16-byte stores
#pragma unroll
      for (int ii = 0; ii < 4; ++ii)
#pragma unroll
        for (int j = 0; j < 2; ++j) {
          typedef _Float16 h4 __attribute__((ext_vector_type(4)));
          h4 o;
#pragma unroll
          for (int e = 0; e < 4; ++e) {   // acc = -log2(e) x_B under the folded SiLU
            if constexpr (ACT_A == 1 && ACT_B == 1)
              o[e] = (_Float16)((acc[ii][j][e] * -0.6931471805599453f) *
                                __builtin_amdgcn_rcpf(1.0f + __builtin_amdgcn_exp2f(acc[ii][j][e])));
            else
              o[e] = (_Float16)act_t<ACT_B>(ACT_A == 1 ? acc[ii][j][e] * -0.6931471805599453f : acc[ii][j][e]);
          }
          *reinterpret_cast<h4*>(stg + (ii * 16 + li) * SPITCH + (j * 16 + g * 4) * 2) = o;
        }
      __builtin_amdgcn_wave_barrier();
      int tb, oy0, ox0;
      tile_geom(tile_of(i), tb, oy0, ox0);
      const uint32_t tile_off = (uint32_t)(pix_index(tb, oy0, ox0, HB, WB) * p.yc * 2);
      const uint32_t row = (uint32_t)((WB + 2 * BORDER) * p.yc * 2);
#pragma unroll
      for (int k = 0; k < 4; ++k) {   // chunk c = lane + 64 k: pixel c / 4 (row k), 16-byte quarter c % 4
        const int c = lane + 64 * k, mb = c >> 2, q = c & 3;
        const int tx = mb & 15;
        const bool in = oy0 + k < HB && ox0 + tx < WB && p.variant != 4;
        const uint32_t off = tile_off + k * row + (uint32_t)((tx * p.yc + p.yoff + w * 32 + q * 8) * 2);
        __builtin_amdgcn_raw_buffer_store_b128(*reinterpret_cast<const u4*>(stg + mb * SPITCH + q * 16), yr,
                                               in ? off : 0x80000000u, 0, 0);
      }
      __syncthreads();
    }
  }
}

template <typename S, int ACT_A, int ACT_B>
hipError_t stem_reorg_t(const StemParams& p, hipStream_t st) {
  const int HB = p.H / 4, WB = p.W / 4;
  const int ntiles = p.B * ((HB + 3) / 4) * ((WB + 15) / 16);
  static const int cus = [] {
    int dev = 0, v = 0;
    if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&v, hipDeviceAttributeMultiprocessorCount, dev) !=
                                                 hipSuccess || v <= 0)
      v = 256;
    return v;
  }();
  const int nblk = ntiles < cus ? ntiles : cus;
  YV7_LAUNCH((stem_reorg_kernel<S, ACT_A, ACT_B>), dim3(nblk), dim3(NT_RG), 0, st, p);
  return hipGetLastError();
}

template <typename S>
hipError_t stem_reorg_acts(const StemParams& p, hipStream_t st) {
  if (p.act_a == 1 && p.act_b == 1) return stem_reorg_t<S, 1, 1>(p, st);
  if (p.act_a == 2 && p.act_b == 2) return stem_reorg_t<S, 2, 2>(p, st);
  if (p.act_a == 0 && p.act_b == 0) return stem_reorg_t<S, 0, 0>(p, st);
  return hipErrorInvalidValue;
}

template <typename S, int CA, int CB, int SA, int ACT_A, int ACT_B>
hipError_t stem_t(const StemParams& p, hipStream_t st) {
  constexpr int TBY = 8, TBX = 16;
  const int HB = p.H / SA / 2, WB = p.W / SA / 2;
  const int ntiles = p.B * ((HB + TBY - 1) / TBY) * ((WB + TBX - 1) / TBX);
  static const int cus = [] {
    int dev = 0, v = 0;
    if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&v, hipDeviceAttributeMultiprocessorCount, dev) !=
                                                 hipSuccess || v <= 0)
      v = 256;
    return v;
  }();
  static const int occ = [] { const char* e = getenv("YV7_STEM_OCC"); return e ? atoi(e) : 2; }();
  const int nblk = ntiles < cus * occ ? ntiles : cus * occ;   // persistent: blocks walk the tiles
  static const int form = [] { const char* e = getenv("YV7_STEM"); return e ? atoi(e) : 2; }();
  if constexpr (SA == 1) {   // (SA = 2, yolov7-tiny: its 10 patch pixels per thread leave stem2 one block per CU)
    if (form != 1) {
      YV7_LAUNCH((stem2_kernel<S, CA, CB, SA, TBY, TBX, ACT_A, ACT_B>), dim3(nblk), dim3(NT), 0, st, p);
      return hipGetLastError();
    }
  }
  YV7_LAUNCH((stem_kernel<S, CA, CB, SA, TBY, TBX, ACT_A, ACT_B>), dim3(nblk), dim3(NT), 0, st, p);
  return hipGetLastError();
}

template <typename S, int CA, int CB, int SA>
hipError_t stem_acts(const StemParams& p, hipStream_t st) {
  if (p.act_a == 1 && p.act_b == 1) return stem_t<S, CA, CB, SA, 1, 1>(p, st);
  if (p.act_a == 2 && p.act_b == 2) return stem_t<S, CA, CB, SA, 2, 2>(p, st);
  if (p.act_a == 0 && p.act_b == 0) return stem_t<S, CA, CB, SA, 0, 0>(p, st);
  return hipErrorInvalidValue;   // mixed activations: not a stem the graph compiler emits
}

}  // namespace

bool stem_supported(int cin, int ca, int cb, int sa) {
  return (cin == 3 && ca == 32 && cb == 64 && (sa == 1 || sa == 2)) || (cin == 12 && ca == 64 && cb == 128 && sa == 1);
}

hipError_t launch_stem(const StemParams& p, int x_dtype, hipStream_t st) {
  if (p.reorg) {
    if (p.H % 4 || p.W % 4) return hipErrorInvalidValue;
    return x_dtype == 1 ? stem_reorg_acts<_Float16>(p, st) : stem_reorg_acts<float>(p, st);
  }
  if (p.sa == 1)
    return x_dtype == 1 ? stem_acts<_Float16, 32, 64, 1>(p, st) : stem_acts<float, 32, 64, 1>(p, st);
  return x_dtype == 1 ? stem_acts<_Float16, 32, 64, 2>(p, st) : stem_acts<float, 32, 64, 2>(p, st);
}

}  // namespace yv7
