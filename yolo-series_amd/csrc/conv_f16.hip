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

// The K-step cursor: tap (rr, ss) and channel ci of a K position, advanced BK at a time.
template <int BK = BKE>
struct KCursor {
  int ci, rr, ss, tap;
  __device__ __forceinline__ void init(const ConvParams& p, int k) {
    ci = k; rr = ss = tap = 0;
    while (ci >= p.cin) { ci -= p.cin; ++tap; if (++ss == p.k) { ss = 0; ++rr; } }
  }
  __device__ __forceinline__ void advance(const ConvParams& p) {
    ci += BK;
    while (ci >= p.cin) { ci -= p.cin; ++tap; if (++ss == p.k) { ss = 0; ++rr; } }
  }
  // byte offset of (rr, ss, ci) relative to the receptive-field origin
  __device__ __forceinline__ uint32_t offset(const ConvParams& p) const {
    return (uint32_t)(((rr * (p.W + 2 * BORDER) + ss) * p.xc + ci) * 2);
  }
};

// Chunk-major K walk of a 3x3 (or 1x1 strided) implicit GEMM with cin % 64 == 0, for the 8-phase rings:
// K step kt = (64-channel chunk cc, tap) with the tap fastest, so the nine taps of one chunk — which share
// most of their 128-byte input lines (stride 2: each line serves ~2.25 taps; stride 1: ~9) — are staged
// within nine consecutive K steps instead of one whole channel sweep apart (tap-major: 256 pixels x cin
// between two taps of a line, more than an XCD's L2 holds with every block of the XCD doing the same;
// round 5: 512->512 s2 @40 read its input 8.3 times from HBM / MALL, profiles/r5_pmc_ops.txt).  The
// weights keep the tap-major [cout][k * k * cin] layout; the B offset follows the same (tap, cc).
struct KWalk {
  int cc, tap, rr, ss;
  __device__ __forceinline__ void init() { cc = tap = rr = ss = 0; }
  __device__ __forceinline__ void advance(const ConvParams& p) {
    if (++tap == p.k * p.k) {
      tap = rr = ss = 0;
      ++cc;
    } else if (++ss == p.k) {
      ss = 0;
      ++rr;
    }
  }
  __device__ __forceinline__ uint32_t a_offset(const ConvParams& p) const {
    return (uint32_t)(((rr * (p.W + 2 * BORDER) + ss) * p.xc + cc * BKE) * 2);
  }
  __device__ __forceinline__ uint32_t b_offset(const ConvParams& p) const {
    return (uint32_t)((tap * p.cin + cc * BKE) * 2);
  }
};

// A-operand source of one K step (BK deep) for RA rows: uniform case (1x1, or cin % BK == 0) = per-row
// offset + scalar step offset; otherwise per-lane tap tracking (cin of 8..56: tiny's narrow layers).
template <bool ONE, int RA, int BK = BKE>
struct AWalk {
  uint32_t off[RA];   // row origin + this lane's chunk
  KCursor<BK> su;     // uniform cursor (k = kt*BK)
  KCursor<BK> ln;     // per-lane cursor (k = kt*BK + chunk*8), non-uniform case only
  bool uni;
  int c16;
  __device__ __forceinline__ void init(const ConvParams& p, int chunk, int kt0 = 0) {
    uni = ONE || (p.cin % BK) == 0;
    c16 = chunk * 16;
    su.init(p, kt0 * BK);
    if (!uni) ln.init(p, kt0 * BK + chunk * 8);
  }
  // voffset / soffset of row j for step kt (call step() once per K step, in order)
  template <typename F>
  __device__ __forceinline__ void step(const ConvParams& p, int kt, F&& load) {
    if (ONE) {
      const uint32_t so = (uint32_t)kt * BK * 2;
      if ((kt + 1) * BK <= p.K) {
#pragma unroll
        for (int j = 0; j < RA; ++j) load(j, off[j], so);
      } else {   // ragged last step (cin % BK != 0): lanes past K read zeros
        const bool kin = kt * BK + c16 / 2 < p.K;
#pragma unroll
        for (int j = 0; j < RA; ++j) load(j, kin ? off[j] : OOB, so);
      }
    } else if (uni) {
      const uint32_t so = su.offset(p);
      su.advance(p);
#pragma unroll
      for (int j = 0; j < RA; ++j) load(j, off[j], so);
    } else {
      const bool kin = kt * BK + c16 / 2 < p.K;
      const uint32_t d = ln.offset(p) - (uint32_t)c16;
      ln.advance(p);
#pragma unroll
      for (int j = 0; j < RA; ++j) load(j, kin ? off[j] + d : OOB, 0u);
    }
  }
};

// LDS image of a BK-deep stage: rows of BK*2 bytes in 16-byte chunks, the chunk index XOR-swizzled
// per row so that the 16-lane groups of every ds_read_b128 (lanes (g, li) read chunk g of rows
// base + li) hit 16 distinct 4-bank groups.  BK 64: 8 chunks per row, key row & 7.  BK 32: 4 chunks
// per 64-byte row (4 rows per 256-byte bank sweep), key (-(row >> 2)) & 3 (found by exhaustive
// check of the four lane groups of ds_read_b128).
template <int BK>
__device__ __forceinline__ int swz_bk(int row, int chunk) {
  if constexpr (BK == 64) return chunk ^ (row & 7);
  else return chunk ^ ((-(row >> 2)) & 3);
}

// ---------------------------------------------------------------------------------------------
// Fused Detect epilogue (models/yolo.py:52-57, IDetect.fuseforward yolo.py:140-176) shared by the
// tile and ring kernels.  BN >= na*no covers every head channel of BM consecutive pixels.
// LDS: zs = the tile's z values in z's own layout, [na][BM][no] fp32 (so z leaves as straight 16-byte
// copies), then a per-pixel table {z row of anchor 0 (int64, -1 past M), grid x, grid y} and the
// level's pixel anchors.
constexpr int det_tab(int BM, int BN) { return BM * BN * 4; }
constexpr int det_lds(int BM, int BN) { return det_tab(BM, BN) + BM * 16 + 64; }

__device__ __forceinline__ float det_sig(float v) {
  return __builtin_amdgcn_rcpf(1.0f + __builtin_amdgcn_exp2f(-1.4426950408889634f * v));
}

struct DetTab {
  long long* zrow0;
  float *gx, *gy, *anc;
};

template <int BM, int BN>
__device__ __forceinline__ DetTab det_tab_ptrs(unsigned char* smem) {
  unsigned char* tab = smem + det_tab(BM, BN);
  DetTab t;
  t.zrow0 = reinterpret_cast<long long*>(tab);
  t.gx = reinterpret_cast<float*>(tab + BM * 8);
  t.gy = t.gx + BM;
  t.anc = t.gy + BM;
  return t;
}

// Step 0 (every thread; the caller then syncs): the per-pixel table.
template <int BM, int BN, int NTH, bool ANC = true>
__device__ __forceinline__ void det_table(const ConvParams& p, unsigned char* smem, int m0, int tid) {
  const DetTab t = det_tab_ptrs<BM, BN>(smem);
  const int hw = p.Ho * p.Wo;
  for (int r = tid; r < BM; r += NTH) {
    const int m = m0 + r;
    const int mm = m < p.M ? m : p.M - 1;
    const int b = mm / hw, cell = mm - b * hw;
    const int gy = cell / p.Wo, gx = cell - gy * p.Wo;
    t.zrow0[r] = m < p.M ? (long long)b * p.nrows + p.row_off + cell : -1;
    t.gx[r] = (float)gx;
    t.gy[r] = (float)gy;
  }
  if (ANC && tid < 8) t.anc[tid] = p.anchor[tid];
}

// Step 1 (registers): sigmoid of every logit, the Detect decode for the 4 box columns in the
// reference's op order (xy = (s*2 - 0.5 + grid)*stride, wh = (s*2)^2 * anchor_px), into zs; the raw
// logits (xs, optional) leave straight from the accumulators.  acc[j][i][e] = channel
// wn*WTN + j*16 + g*4 + e of pixel m0 + wm*WTM + i*16 + li.  NOC / NAC: compile-time no / na (0 =
// read p.no / p.na).  Branch-free per value: only the one 16-column block per wave that holds a box
// column runs the decode (a wave-uniform test), the padding column past na*no lands on a dummy slot.
template <int BM, int BN, int TN, int TM, int NOC, int NAC>
__device__ __forceinline__ void det_stage(const ConvParams& p, unsigned char* smem, const f4 (&acc)[TN][TM], int m0,
                                          int wm, int wn, int g, int li) {
  constexpr int WTM = TM * 16, WTN = TN * 16;
  const DetTab t = det_tab_ptrs<BM, BN>(smem);
  float* zs = reinterpret_cast<float*>(smem);
  const int NO = NOC ? NOC : p.no, NA = NAC ? NAC : p.na;
  const int dummy = NA * BM * NO;   // one spare float inside BM*BN (BN > na*no)
  const int wnu = __builtin_amdgcn_readfirstlane(wn);
#pragma unroll
  for (int j = 0; j < TN; ++j) {
    const int cb = wnu * WTN + j * 16;
    bool dec = false;
    for (int a = 0; a < NA; ++a) dec |= cb < a * NO + 4 && cb + 16 > a * NO;
    int zoff[4], co[4];
    bool live[4];
    float anc_wh[4];
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const int c = cb + g * 4 + e;
      const int ca = c / NO;
      co[e] = c - ca * NO;
      live[e] = ca < NA;
      zoff[e] = live[e] ? ca * BM * NO + co[e] : dummy;
      anc_wh[e] = dec ? t.anc[(live[e] ? 2 * ca : 0) + (co[e] == 3 ? 1 : 0)] : 0.0f;
    }
#pragma unroll
    for (int i = 0; i < TM; ++i) {
      const int row = wm * WTM + i * 16 + li;
      const int roff = row * NO;
      if (dec) {
        const float gxv = t.gx[row], gyv = t.gy[row];
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const float s = det_sig(acc[j][i][e]);
          const float t2 = s * 2.0f;
          const float xy = (t2 - 0.5f + (co[e] == 0 ? gxv : gyv)) * p.stride;
          const float wh = (t2 * t2) * anc_wh[e];
          zs[zoff[e] + (live[e] ? roff : 0)] = co[e] < 2 ? xy : (co[e] < 4 ? wh : s);
        }
      } else {
#pragma unroll
        for (int e = 0; e < 4; ++e) zs[zoff[e] + (live[e] ? roff : 0)] = det_sig(acc[j][i][e]);
      }
    }
  }
  if (p.raw) {
    const int hw = p.Ho * p.Wo;
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
      for (int i = 0; i < TM; ++i) {
        const int row = wm * WTM + i * 16 + li;
        const int m = m0 + row;
        if (m >= p.M) continue;
        const int b = m / hw, cell = m - b * hw;
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const int c = wnu * WTN + j * 16 + g * 4 + e;
          const int ca = c / NO, co = c - ca * NO;
          if (ca < NA) p.raw[((size_t)(b * NA + ca) * hw + cell) * NO + co] = acc[j][i][e];
        }
      }
  }
}

template <int BM, int BN, int NTH, int NOC, int NAC>
__device__ __forceinline__ void det_tail(const ConvParams& p, unsigned char* smem, int tid);

// The whole epilogue after the main loop (LDS free): table, values, scores + z.
template <int BM, int BN, int NTH, int TN, int TM>
__device__ __forceinline__ void det_epilogue(const ConvParams& p, unsigned char* smem, const f4 (&acc)[TN][TM], int m0,
                                             int wm, int wn, int g, int li, int tid) {
  det_table<BM, BN, NTH>(p, smem, m0, tid);
  __syncthreads();
  const bool std85 = p.no == 85 && p.na == 3;
  if (std85) det_stage<BM, BN, TN, TM, 85, 3>(p, smem, acc, m0, wm, wn, g, li);
  else det_stage<BM, BN, TN, TM, 0, 0>(p, smem, acc, m0, wm, wn, g, li);
  __syncthreads();
  if (std85) det_tail<BM, BN, NTH, 85, 3>(p, smem, tid);
  else det_tail<BM, BN, NTH, 0, 0>(p, smem, tid);
}

// yv7_row_best record of one (anchor, pixel) row: objectness, first-max class score obj * cls_c and
// its class, from the same sigmoid values z receives.  Four lanes per row, each over the classes
// c = part, part + 4, ... (first maximum per lane), merged by shuffles: the larger score wins, an
// equal score goes to the smaller class — the first maximum (general.py:683-684).
// (NB: the lane's classes are loaded in NB batches — 2 under register pressure — and scanned in order.)
template <int NC, int NB = 1>
__device__ __forceinline__ void det_best_lane(const float* sg, int nc, int part, float& best, int& bc) {
  const float obj = sg[4];
  best = -1.0f;
  bc = 0x7fffffff;
  if constexpr (NC > 0) {
    constexpr int NV = NC / 4 / NB;
#pragma unroll
    for (int b = 0; b < NB; ++b) {
      float v[NV];
#pragma unroll
      for (int i = 0; i < NV; ++i) v[i] = sg[5 + part + 4 * (b * NV + i)];
#pragma unroll
      for (int i = 0; i < NV; ++i) {
        const float s = v[i] * obj;
        if (s > best) { best = s; bc = part + 4 * (b * NV + i); }
      }
    }
  } else if (nc > 1) {
    for (int c = part; c < nc; c += 4) {
      const float s = sg[5 + c] * obj;
      if (s > best) { best = s; bc = c; }
    }
  } else if (part == 0) {
    best = obj;
    bc = 0;
  }
}

// Steps 2-3 (after det_stage and a barrier): the row scores, then z as 16-byte copies.
template <int BM, int BN, int NTH, int NOC, int NAC>
__device__ __forceinline__ void det_tail(const ConvParams& p, unsigned char* smem, int tid) {
  const DetTab t = det_tab_ptrs<BM, BN>(smem);
  const float* zs = reinterpret_cast<const float*>(smem);
  const int hw = p.Ho * p.Wo;
  const int NO = NOC ? NOC : p.no, NA = NAC ? NAC : p.na;
  if (p.best) {
    const int nc = NO - 5;
    for (int t0 = 0; t0 < BM * NA * 4; t0 += NTH) {
      const int tt = t0 + tid;
      const int r = tt >> 2, part = tt & 3;     // r = a * BM + pixel
      const int pr = r % BM, a = r / BM;
      const bool live = r < BM * NA && t.zrow0[pr] >= 0;
      const float* sg = zs + (live ? r : 0) * NO;
      float best;
      int bc;
      if (NOC == 85) det_best_lane<80>(sg, nc, part, best, bc);
      else det_best_lane<0>(sg, nc, part, best, bc);
#pragma unroll
      for (int d = 1; d < 4; d <<= 1) {
        const float ob = __shfl_xor(best, d, 64);
        const int oc = __shfl_xor(bc, d, 64);
        if (ob > best || (ob == best && oc < bc)) { best = ob; bc = oc; }
      }
      if (live && part == 0) {
        f4 rec;
        rec[0] = sg[4];
        rec[1] = best;
        rec[2] = __builtin_bit_cast(float, bc);
        rec[3] = 0.0f;
        // z and the row records are streamed out (non-temporal): nothing re-reads them before the NMS
        __builtin_nontemporal_store(rec, reinterpret_cast<f4*>(p.best + (size_t)(t.zrow0[pr] + (long long)a * hw) * 4));
      }
    }
  }
  // A 4-row group of one anchor (4 consecutive pixels of one image = 4 consecutive z rows) is no
  // float4 chunks in zs and in z.  Thread t owns chunk t % no of the groups it visits; a group whose
  // first z row is divisible by 4 (a 16-byte aligned block) leaves as 16-byte stores, any other one
  // (image boundary, rows past M, odd level sizes) element by element.
  constexpr int G = BM / 4;
  static_assert(BM % 4 == 0, "4-row groups");
  const int gpp = NTH / NO;
  const int c = tid % NO, gg = tid / NO;
  if (gg < gpp) {
    for (int idx = gg; idx < NA * G; idx += gpp) {
      const int a = idx / G, grp = idx - a * G;
      const long long aoff = (long long)a * hw;
      const long long z0 = t.zrow0[grp * 4];
      const f4 v = reinterpret_cast<const f4*>(zs + (a * BM + grp * 4) * NO)[c];
      if (z0 >= 0 && t.zrow0[grp * 4 + 3] == z0 + 3 && ((z0 + aoff) & 3) == 0) {
        __builtin_nontemporal_store(v, reinterpret_cast<f4*>(p.z + (size_t)(z0 + aoff) * NO) + c);
      } else {
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          const int e = 4 * c + k, rk = e / NO, ok = e - rk * NO;
          const long long zr = t.zrow0[grp * 4 + rk];
          if (zr >= 0) __builtin_nontemporal_store(v[k], p.z + (size_t)(zr + aoff) * NO + ok);
        }
      }
    }
  }
}

// ---------------------------------------------------------------------------------------------
// Persistent Detect head (round 3): the head conv + decode of one level (yolo.py:42-63) for the
// standard head (na = 3, no = 85, 1x1, K = cin a multiple of 64, level size a multiple of 4, no raw
// logits).  Measured on the tile kernel (scripts/detbench.hip hooks 90/93/94/95): at 80^2 its GEMM,
// staging, row scores and z stores take 37 + 27 + 9 + 54 us and do not overlap — both blocks of a CU
// run the same phase at the same time, so the z stores (209 MB at 80^2) drain while nothing else runs.
// Here one block per CU walks 64-pixel tiles with the K-step ring running across tiles:
//  * 8 waves (2 x 4), 64 pixels x 256 channels per tile, two 40 KiB ring stages + the z staging
//    image (zs, the tile's z rows in z's layout) and the row table: 146 KiB of LDS;
//  * the tile epilogue (sigmoid / decode into zs, row scores, z + row-record stores) runs after the
//    K loop; its first barrier frees the ring, so the next tile's first TWO stages are issued before
//    the epilogue and its K loop starts with both landed;
//  * every wave issues the same stores in every tile (10 with row records: 2 record + 8 z stores per
//    wave; rows past M, lanes without work and the other 3 lanes of a row's record go to an offset past
//    the buffer range, where the store is dropped), so the epilogue's stores stay in flight behind
//    counted vmcnt waits — they drain under the next tile's K loop and epilogue instead of stalling it.
// Same arithmetic as det_stage / det_tail (bit-identical z and records).
// ZU: the z-store loop's unroll (2 under register pressure: the register-weight head at K = 512)
template <int BM, int NTH, int ZU = 0>
__device__ __forceinline__ void det_tail_fixed(const ConvParams& p, unsigned char* smem, int tid,
                                               __amdgpu_buffer_rsrc_t zr, __amdgpu_buffer_rsrc_t br, long long zb) {
  constexpr int NO = 85, NA = 3, BN = 256;
  const DetTab t = det_tab_ptrs<BM, BN>(smem);
  const float* zs = reinterpret_cast<const float*>(smem);
  const int hw = p.Ho * p.Wo;
  float* zw = reinterpret_cast<float*>(smem);
#pragma unroll
  for (int t0 = 0; t0 < BM * NA * 4; t0 += NTH) {
    // task (row r = anchor a x pixel pr, part): box column `part` of the row (the Detect decode in
    // det_stage's op order, yolo.py:52-57) and a quarter of its row-score scan
    const int tt = t0 + tid;
    const int r = tt >> 2, part = tt & 3;
    const int pr = r % BM, a = r / BM;
    const bool inr = r < BM * NA;
    const bool live = inr && t.zrow0[pr] >= 0;
    if (inr) {
      const float sgv = zs[r * NO + part];
      const float t2 = sgv * 2.0f;
      const float xy = (t2 - 0.5f + (part == 0 ? t.gx[pr] : t.gy[pr])) * p.stride;
      const float wh = (t2 * t2) * t.anc[2 * a + (part == 3 ? 1 : 0)];
      zw[r * NO + part] = part < 2 ? xy : wh;
    }
    if (p.best) {
      const float* sg = zs + (live ? r : 0) * NO;
      float best;
      int bc;
      det_best_lane<80, ZU ? 2 : 1>(sg, NO - 5, part, best, bc);
#pragma unroll
      for (int d = 1; d < 4; d <<= 1) {
        const float ob = __shfl_xor(best, d, 64);
        const int oc = __shfl_xor(bc, d, 64);
        if (ob > best || (ob == best && oc < bc)) { best = ob; bc = oc; }
      }
      f4 rec;
      rec[0] = sg[4];
      rec[1] = best;
      rec[2] = __builtin_bit_cast(float, bc);
      rec[3] = 0.0f;
      const uint32_t off = (live && part == 0) ? (uint32_t)((t.zrow0[pr] - zb + (long long)a * hw) * 16) : 0xffffffffu;
      __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u4, rec), br, off, 0, 2);   // nt
    }
  }
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");   // decoded box columns visible to the z stores
  __builtin_amdgcn_s_barrier();
  constexpr int G = BM / 4;            // 4-row groups per anchor
  constexpr int GPP = NTH / NO;        // groups in flight per pass
  constexpr int IT = (NA * G + GPP - 1) / GPP;
  const int c = tid % NO, gg = tid / NO;
  constexpr int ZUN = ZU ? ZU : IT;
#pragma unroll ZUN
  for (int k = 0; k < IT; ++k) {
    const int idx = gg + GPP * k;
    const bool valid = gg < GPP && idx < NA * G;
    const int ii = valid ? idx : 0;
    const int a = ii / G, grp = ii - a * G;
    const long long z0 = t.zrow0[grp * 4];
    const f4 v = reinterpret_cast<const f4*>(zs + (a * BM + grp * 4) * NO)[c];
    const uint32_t off = (valid && z0 >= 0) ? (uint32_t)((z0 - zb + (long long)a * hw) * NO * 4 + c * 16) : 0xffffffffu;
    __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u4, v), zr, off, 0, 2);       // nt
  }
}

// vmcnt before ring step kt: stage kt landed, the min(MAXN, ahead) stages issued after it (PER DMA
// instructions each) may stay in flight — an immediate per case
template <int PER, int MAXN>
__device__ __forceinline__ void ring_wait(int ahead) {
  if constexpr (MAXN <= 0) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  } else {
    static_assert(MAXN * PER <= 63, "vmcnt range");
    if (ahead >= MAXN) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(MAXN * PER) : "memory");
    else ring_wait<PER, MAXN - 1>(ahead);
  }
}

template <int HOOK = 0>
__global__ __launch_bounds__(512, 1) void conv_det_pring_kernel(const ConvParams p) {
  constexpr int BM = 64, BN = 256, WM = 2, WN = 4, NW = 8, NTH = 512;
  constexpr int WTM = BM / WM, WTN = BN / WN, TM = WTM / 16, TN = WTN / 16;
  constexpr int RB = BN / 8 / NW;                  // 4 weight wave-instructions per stage (A: 1)
  constexpr int PER = HOOK == 4 ? 1 : 1 + RB;   // (hook 4: no weight DMA)
  constexpr int STAGE = (BM + BN) * ROWB;          // 40 KiB
  constexpr int RING = 2 * STAGE;
  constexpr int LDS = RING + det_lds(BM, BN);
  static_assert(LDS <= 160 * 1024, "LDS budget");
  __shared__ __attribute__((aligned(16))) unsigned char smem[LDS];
  unsigned char* es = smem + RING;                 // zs + row table

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave / WN, wn = wave % WN;
  const int g = lane >> 4, li = lane & 15;
  const int T = (p.M + BM - 1) / BM;
  const int nk = p.kpad / BKE;
  const TileWalk tw = xcd_tile_walk(T);
  const int ntl = tw.count();
  if (ntl == 0) return;

  const auto xr = make_rsrc(p.x, p.xbytes);
  const auto wr = make_rsrc(p.w, p.wbytes);
  const int lr = lane >> 3;
  const int c = (lane & 7) ^ lr;
  uint32_t b_off[RB];
#pragma unroll
  for (int j = 0; j < RB; ++j) b_off[j] = (uint32_t)((((j * NW + wave) * 8 + lr) * p.kpad + c * 8) * 2);
  const int hw = p.Ho * p.Wo;
  auto a_off = [&](int it) -> uint32_t {
    if (it >= ntl) return OOB;
    const int m = tw.at(it) * BM + wave * 8 + lr;
    if (m >= p.M) return OOB;
    const int b = m / hw, cell = m - b * hw, ho = cell / p.Wo, wo = cell - ho * p.Wo;
    return (uint32_t)((pix_index(b, ho, wo, p.H, p.W) * p.xc + p.xoff + c * 8) * 2);
  };
  // stage q = (tile it, K step k) into slot q & 1
  int i_it = 0, i_k = 0, i_q = 0;
  uint32_t i_aoff = a_off(0);
  auto issue = [&]() __attribute__((always_inline)) {
    unsigned char* As = smem + (i_q & 1) * STAGE;
    unsigned char* Bs = As + BM * ROWB;
    const bool live = i_it < ntl;
    const uint32_t so = (uint32_t)i_k * BKE * 2;
    dma16(xr, As + wave * 8 * ROWB, i_aoff, so);
    if constexpr (HOOK != 4) {
#pragma unroll
      for (int j = 0; j < RB; ++j) dma16(wr, Bs + (j * NW + wave) * 8 * ROWB, live ? b_off[j] : OOB, so);
    }
    asm volatile("" ::: "memory");
    ++i_q;
    if (++i_k == nk) {
      i_k = 0;
      ++i_it;
      i_aoff = a_off(i_it);
    }
  };

  const f4 bias0 = {0.0f, 0.0f, 0.0f, 0.0f};
  f4 bv[TN];
#pragma unroll
  for (int j = 0; j < TN; ++j) {
    const int col = wn * WTN + j * 16 + g * 4;
    bv[j] = bias0;
#pragma unroll
    for (int e = 0; e < 4; ++e) bv[j][e] = col + e < p.cout ? p.bias[col + e] : 0.0f;
  }
  const int nst = p.best ? 10 : 8;   // epilogue stores per wave per tile (det_tail_fixed)

  // z slot of each of this lane's 16 channels (j, e) in the tile's [na][BM][no] image (tile-invariant;
  // the padding channel 255 -> a spare slot)
  constexpr int NO = 85, NA = 3;
  int zo[TN][4];
#pragma unroll
  for (int j = 0; j < TN; ++j)
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const int ch = wn * WTN + j * 16 + g * 4 + e;
      const int ca = ch / NO;
      zo[j][e] = ca < NA ? ca * BM * NO + (ch - ca * NO) : NA * BM * NO;
    }
  // the level's anchors once (a per-lane kernel-argument load: its wait stays out of the tile loop)
  if (tid < 8) det_tab_ptrs<BM, BN>(es).anc[tid] = p.anchor[tid];
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  issue();
  issue();
  for (int it = 0; it < ntl; ++it) {
    const int m0 = tw.at(it) * BM;
    f4 acc[TN][TM];
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
      for (int i = 0; i < TM; ++i) acc[j][i] = bv[j];
    for (int k = 0; k < nk; ++k) {
      // stage (it, k) landed: younger are stage (it, 1) and the previous epilogue's stores at k = 0,
      // the previous epilogue's stores at k = 1 (both stages of a tile start are issued before them)
      if (k == 0) {
        if (it > 0 && nst == 10) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(PER + 10) : "memory");
        else if (it > 0) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(PER + 8) : "memory");
        else asm volatile("s_waitcnt vmcnt(%0)" ::"n"(PER) : "memory");
      } else if (k == 1 && it > 0) {
        if (nst == 10) asm volatile("s_waitcnt vmcnt(10)" ::: "memory");
        else asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
      } else {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      }
      __builtin_amdgcn_s_barrier();
      if (k >= 1) issue();              // stage (it, k + 1) or the next tile's first stage
      if (k == 0) det_table<BM, BN, NTH, false>(p, es, m0, tid);   // read after the K loop's last barrier
      const unsigned char* As = smem + ((it * nk + k) & 1) * STAGE;
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
    }
    // epilogue: ring reads done -> the next tile's stage (it + 1, 1) into the free slot
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    issue();
    if constexpr (HOOK != 1 && HOOK != 3) {
      // staging: the sigmoid of every logit into zs (z's layout); the 4 box columns of each row are
      // decoded in det_tail_fixed (one (row, column) per thread there, beside the row scores)
      float* zs = reinterpret_cast<float*>(es);
#pragma unroll
      for (int i = 0; i < TM; ++i) {
        const int roff = (wm * WTM + i * 16 + li) * NO;
#pragma unroll
        for (int j = 0; j < TN; ++j)
#pragma unroll
          for (int e = 0; e < 4; ++e) zs[zo[j][e] + (zo[j][e] < NA * BM * NO ? roff : 0)] = det_sig(acc[j][i][e]);
      }
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    // z / record rows of this tile relative to its first pixel's row (offsets stay 32-bit at any batch)
    const int mb = m0 / hw;
    const long long zb = (long long)mb * p.nrows + p.row_off + (m0 - mb * hw);
    const auto zr = make_rsrc(p.z + (size_t)zb * 85, 0x7fffffffu);
    const auto br = make_rsrc(p.best ? p.best + (size_t)zb * 4 : p.z, 0x7fffffffu);
    if constexpr (HOOK < 2) det_tail_fixed<BM, NTH>(p, es, tid, zr, br, zb);
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

// One-tile Detect head (round 6): where a level has at most one 64-pixel tile per CU (yolov7 bs 32's P5 head,
// 1024 -> 255 @20: 200 tiles), every block of the persistent head runs ONE tile, and its two-slot ring waits out
// an L2 round trip at each of the 16 K steps (PMC: 65 % of the wave cycles waiting, profiles/r5_pmc_kernels/).
// With no next tile to prefetch, the z staging image needs no room of its own during the K loop: four 40 KiB
// stages (three in flight) fill the LDS, and the staging image + row table reuse it after the loop.  Same
// arithmetic as conv_det_pring_kernel (bit-identical z and row records).
__global__ __launch_bounds__(512, 1) void conv_det_1tile_kernel(const ConvParams p) {
  constexpr int BM = 64, BN = 256, WM = 2, WN = 4, NW = 8, NTH = 512;
  constexpr int WTM = BM / WM, WTN = BN / WN, TM = WTM / 16, TN = WTN / 16;
  constexpr int RB = BN / 8 / NW;                  // 4 weight wave-instructions per stage (A: 1)
  constexpr int PER = 1 + RB;
  constexpr int STAGE = (BM + BN) * ROWB;          // 40 KiB
  constexpr int NS = 4;
  constexpr int LDS = NS * STAGE;
  static_assert(LDS <= 160 * 1024 && det_lds(BM, BN) <= LDS, "LDS budget");
  __shared__ __attribute__((aligned(16))) unsigned char smem[LDS];
  unsigned char* es = smem;                        // zs + row table, after the K loop

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave / WN, wn = wave % WN;
  const int g = lane >> 4, li = lane & 15;
  const int m0 = blockIdx.x * BM;
  if (m0 >= p.M) return;
  const int nk = p.kpad / BKE;
  const auto xr = make_rsrc(p.x, p.xbytes);
  const auto wr = make_rsrc(p.w, p.wbytes);
  const int lr = lane >> 3;
  const int c = (lane & 7) ^ lr;
  uint32_t b_off[RB];
#pragma unroll
  for (int j = 0; j < RB; ++j) b_off[j] = (uint32_t)((((j * NW + wave) * 8 + lr) * p.kpad + c * 8) * 2);
  const int hw = p.Ho * p.Wo;
  uint32_t aoff = OOB;
  {
    const int m = m0 + wave * 8 + lr;
    if (m < p.M) {
      const int b = m / hw, cell = m - b * hw, ho = cell / p.Wo, wo = cell - ho * p.Wo;
      aoff = (uint32_t)((pix_index(b, ho, wo, p.H, p.W) * p.xc + p.xoff + c * 8) * 2);
    }
  }
  auto issue = [&](int k, int slot) __attribute__((always_inline)) {
    unsigned char* As = smem + slot * STAGE;
    unsigned char* Bs = As + BM * ROWB;
    const uint32_t so = (uint32_t)k * BKE * 2;
    dma16(xr, As + wave * 8 * ROWB, aoff, so);
#pragma unroll
    for (int j = 0; j < RB; ++j) dma16(wr, Bs + (j * NW + wave) * 8 * ROWB, b_off[j], so);
    asm volatile("" ::: "memory");
  };
  f4 acc[TN][TM];
#pragma unroll
  for (int j = 0; j < TN; ++j) {
    const int col = wn * WTN + j * 16 + g * 4;
    f4 bv;
#pragma unroll
    for (int e = 0; e < 4; ++e) bv[e] = col + e < p.cout ? p.bias[col + e] : 0.0f;
#pragma unroll
    for (int i = 0; i < TM; ++i) acc[j][i] = bv;
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // bias
#pragma unroll
  for (int s = 0; s < NS - 1; ++s)
    if (s < nk) issue(s, s);
  for (int k = 0; k < nk; ++k) {
    ring_wait<PER, NS - 2>(nk - 1 - k);   // stage k landed; up to NS - 2 later stages in flight
    __builtin_amdgcn_s_barrier();
    if (k + NS - 1 < nk) issue(k + NS - 1, (k + NS - 1) & (NS - 1));   // into the slot step k - 1 read
    const unsigned char* As = smem + (k & (NS - 1)) * STAGE;
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
  }
  asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();   // the ring is free: the staging image and row table take its place
  if (tid < 8) det_tab_ptrs<BM, BN>(es).anc[tid] = p.anchor[tid];
  det_table<BM, BN, NTH, false>(p, es, m0, tid);
  {
    constexpr int NO = 85, NA = 3;
    float* zs = reinterpret_cast<float*>(es);
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int ch = wn * WTN + j * 16 + g * 4 + e;
        const int ca = ch / NO;
        const int zo = ca < NA ? ca * BM * NO + (ch - ca * NO) : NA * BM * NO;
#pragma unroll
        for (int i = 0; i < TM; ++i)
          zs[zo + (zo < NA * BM * NO ? (wm * WTM + i * 16 + li) * NO : 0)] = det_sig(acc[j][i][e]);
      }
  }
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  const int mb = m0 / hw;
  const long long zb = (long long)mb * p.nrows + p.row_off + (m0 - mb * hw);
  const auto zr = make_rsrc(p.z + (size_t)zb * 85, 0x7fffffffu);
  const auto br = make_rsrc(p.best ? p.best + (size_t)zb * 4 : p.z, 0x7fffffffu);
  det_tail_fixed<BM, NTH>(p, es, tid, zr, br, zb);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

// Register-weight Detect head (round 5, the default for K = 256 / 512: yolov7's P3 / P4 heads, w6's P3
// / P4).  scripts/detbench.hip's hook 93 (the persistent head above without its weight DMA,
// profiles/r5_det/detbench_hooks_noweights.txt) runs 256->255 @80 bs 32 in 41-50 us against 91-92 and
// 512->255 @40 in 20 against 40: restaging the 256-channel weight tile (4 of the 5 pieces of every K
// step) for every 64-pixel tile costs as much as the whole rest of the kernel.  Here the weights never
// move: wave w keeps channels 32 w .. 32 w + 31 for all of K in VGPRs (2 x NCH fragments from the
// fragment-packed copy: 64 VGPRs at K = 256, 128 at K = 512), the ring stages only the tile's pixels (8
// KiB per K step), and the wave computes those 32 channels for all 64 pixels (4 pixel fragments per read
// step, each feeding 2 MFMAs).  Epilogue and row records as conv_det_pring_kernel (det_tail_fixed; the
// same sigmoid and decode: bit-identical z and records).
// HOOK (detbench only, variant 91; the ABI never accepts it): 1 = no pixel DMA (stale LDS operands)
// D (round 6): pixel stages in flight ahead of the one being read.  D = 0 is the round-5 schedule (a
// two-slot ring: the K step's stage issued one step ahead, plus the next tile's second stage before the
// epilogue).  D > 0: a (D + 1)-slot ring, one stage issued per K step D steps ahead, so at K = 256 (4 steps)
// the whole next tile's pixels are in flight during this tile's epilogue instead of being waited for inside
// its K loop.  Stage s is read at global step s; the stores of the epilogue between two tiles are younger
// than the stages issued before it, so the counted wait at step k of a tile allows D - 1 younger stages,
// plus the previous epilogue's nst stores while those stages were issued before it (k < D, tile > 0).
// BM (round 6): pixels per tile, 64 or 32 — at 32 the four pixel pieces of a stage are issued by waves 0-3 and
// again by waves 4-7 (the same bytes to the same rows), so every wave's counted waits stay the same.
template <int NCH, int HOOK = 0, int D = 0, int BM = 64>
__global__ __launch_bounds__(512, 1) void conv_det_rw_kernel(const ConvParams p) {
  constexpr int BN = 256, NTH = 512, TM = BM / 16, TN = 2, NK = NCH / 2;
  static_assert(BM == 64 || BM == 32, "tile");
  // epilogue stores per wave per tile (det_tail_fixed): row records, z rows
  constexpr int NREC = (BM * 3 * 4 + NTH - 1) / NTH, NZS = (3 * (BM / 4) + NTH / 85 - 1) / (NTH / 85);
  constexpr int NSTB = NREC + NZS, NSTN = NZS;
  constexpr int PER = HOOK == 1 ? 0 : 1;           // one A piece per wave per stage
  constexpr int STAGE = BM * ROWB;                 // 8 KiB
  constexpr int R = D > 0 ? D + 1 : 2;             // ring slots
  constexpr int RING = R * STAGE;
  constexpr int LDS = RING + det_lds(BM, BN);
  static_assert(LDS <= 160 * 1024, "LDS budget");
  static_assert(D == 0 || ((D - 1) * PER + NSTB <= 63 && D <= NK), "counted waits");
  constexpr int NO = 85, NA = 3;
  __shared__ __attribute__((aligned(16))) unsigned char smem[LDS];
  unsigned char* es = smem + RING;                 // zs + row table

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int g = lane >> 4, li = lane & 15;
  const int T = (p.M + BM - 1) / BM;
  const TileWalk tw = xcd_tile_walk(T);
  const int ntl = tw.count();
  if (ntl == 0) return;

  const auto xr = make_rsrc(p.x, p.xbytes);
  const auto wr = make_rsrc(p.wf, p.wfbytes);
  // the wave's weights: fragment (16-channel group 2 wave + j, K step c) at ((2 wave + j) * NCH + c) KiB
  u4 wreg[TN][NCH];
#pragma unroll
  for (int j = 0; j < TN; ++j) {
    const uint32_t base = (uint32_t)(((2 * wave + j) * NCH) * 1024 + lane * 16);
#pragma unroll
    for (int c = 0; c < NCH; ++c)
      wreg[j][c] = __builtin_bit_cast(u4, __builtin_amdgcn_raw_buffer_load_b128(wr, base, (uint32_t)(c * 1024), 0));
  }
  const int lr = lane >> 3;
  const int c8 = (lane & 7) ^ lr;
  const int hw = p.Ho * p.Wo;
  auto a_off = [&](int it) -> uint32_t {
    if (it >= ntl) return OOB;
    const int m = tw.at(it) * BM + (wave % (BM / 8)) * 8 + lr;
    if (m >= p.M) return OOB;
    const int b = m / hw, cell = m - b * hw, ho = cell / p.Wo, wo = cell - ho * p.Wo;
    return (uint32_t)((pix_index(b, ho, wo, p.H, p.W) * p.xc + p.xoff + c8 * 8) * 2);
  };
  // stage q = (tile it, K step k) into slot q % R
  int i_it = 0, i_k = 0, i_slot = 0;
  uint32_t i_aoff = a_off(0);
  auto issue = [&]() __attribute__((always_inline)) {
    if constexpr (HOOK != 1) dma16(xr, smem + i_slot * STAGE + (wave % (BM / 8)) * 8 * ROWB, i_aoff, (uint32_t)i_k * BKE * 2);
    asm volatile("" ::: "memory");
    if (++i_slot == R) i_slot = 0;
    if (++i_k == NK) {
      i_k = 0;
      ++i_it;
      i_aoff = a_off(i_it);
    }
  };

  f4 bv[TN];
#pragma unroll
  for (int j = 0; j < TN; ++j) {
    const int col = wave * 32 + j * 16 + g * 4;
#pragma unroll
    for (int e = 0; e < 4; ++e) bv[j][e] = col + e < p.cout ? p.bias[col + e] : 0.0f;
  }
  const int nst = p.best ? NSTB : NSTN;
  // z slot of each of this lane's 8 channels (the padding channel 255 -> a spare slot)
  int zo[TN][4];
#pragma unroll
  for (int j = 0; j < TN; ++j)
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const int ch = wave * 32 + j * 16 + g * 4 + e;
      const int ca = ch / NO;
      zo[j][e] = ca < NA ? ca * BM * NO + (ch - ca * NO) : NA * BM * NO;
    }
  if (tid < 8) det_tab_ptrs<BM, BN>(es).anc[tid] = p.anchor[tid];
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // weights, bias, anchors
#pragma unroll
  for (int d = 0; d < (D > 0 ? D : 2); ++d) issue();
  int r_slot = 0;   // the slot of the stage the next K step reads
  for (int it = 0; it < ntl; ++it) {
    const int m0 = tw.at(it) * BM;
    f4 acc[TN][TM];
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
      for (int i = 0; i < TM; ++i) acc[j][i] = bv[j];
#pragma unroll
    for (int k = 0; k < NK; ++k) {
      if constexpr (D == 0) {
        // stage (it, k) landed: younger are stage (it, 1) and the previous epilogue's stores at k = 0, the
        // previous epilogue's stores at k = 1 (both stages of a tile start are issued before them)
        if (k == 0) {
          if (it > 0 && nst == NSTB) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(PER + NSTB) : "memory");
          else if (it > 0) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(PER + NSTN) : "memory");
          else asm volatile("s_waitcnt vmcnt(%0)" ::"n"(PER) : "memory");
        } else if (k == 1 && it > 0) {
          if (nst == NSTB) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(NSTB) : "memory");
          else asm volatile("s_waitcnt vmcnt(%0)" ::"n"(NSTN) : "memory");
        } else {
          asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        }
      } else {
        if (k >= D || it == 0) asm volatile("s_waitcnt vmcnt(%0)" ::"n"((D - 1) * PER) : "memory");
        else if (nst == NSTB) asm volatile("s_waitcnt vmcnt(%0)" ::"n"((D - 1) * PER + NSTB) : "memory");
        else asm volatile("s_waitcnt vmcnt(%0)" ::"n"((D - 1) * PER + NSTN) : "memory");
      }
      __builtin_amdgcn_s_barrier();
      if (D > 0 || k >= 1) issue();     // D > 0: stage s + D; D = 0: stage (it, k + 1) or the next tile's first
      if (k == 0) det_table<BM, BN, NTH, false>(p, es, m0, tid);   // read after the K loop's last barrier
      const unsigned char* As = smem + r_slot * STAGE;
      if (++r_slot == R) r_slot = 0;
#pragma unroll
      for (int s2 = 0; s2 < 2; ++s2) {
        const int ch = s2 * 4 + g;
        u4 xa[TM];
#pragma unroll
        for (int i = 0; i < TM; ++i) {
          const int row = i * 16 + li;
          xa[i] = *reinterpret_cast<const u4*>(As + row * ROWB + swz(row, ch) * 16);
        }
        __builtin_amdgcn_s_setprio(1);
#pragma unroll
        for (int j = 0; j < TN; ++j)
#pragma unroll
          for (int i = 0; i < TM; ++i)
            acc[j][i] = __builtin_amdgcn_mfma_f32_16x16x32_f16(__builtin_bit_cast(h8, wreg[j][2 * k + s2]),
                                                               __builtin_bit_cast(h8, xa[i]), acc[j][i], 0, 0, 0);
        __builtin_amdgcn_s_setprio(0);
      }
    }
    // epilogue: ring reads done (D = 0: -> the next tile's stage (it + 1, 1) into the free slot)
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    if constexpr (D == 0) issue();
    // staging: the sigmoid of every logit into zs (z's layout); the box columns are decoded in
    // det_tail_fixed
    float* zs = reinterpret_cast<float*>(es);
#pragma unroll
    for (int i = 0; i < TM; ++i) {
      const int roff = (i * 16 + li) * NO;
#pragma unroll
      for (int j = 0; j < TN; ++j)
#pragma unroll
        for (int e = 0; e < 4; ++e) zs[zo[j][e] + (zo[j][e] < NA * BM * NO ? roff : 0)] = det_sig(acc[j][i][e]);
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    const int mb = m0 / hw;
    const long long zb = (long long)mb * p.nrows + p.row_off + (m0 - mb * hw);
    const auto zr = make_rsrc(p.z + (size_t)zb * 85, 0x7fffffffu);
    const auto br = make_rsrc(p.best ? p.best + (size_t)zb * 4 : p.z, 0x7fffffffu);
    det_tail_fixed<BM, NTH, NCH == 8 ? 0 : 2>(p, es, tid, zr, br, zb);
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

bool det_rw_supported(const ConvParams& p) {
  return p.wf && (p.kpad == 256 || p.kpad == 512) && p.wfbytes >= (uint32_t)(256 * p.kpad * 2);
}

bool det_pring_supported(const ConvParams& p) {
  const int hw = p.Ho * p.Wo;
  return p.k == 1 && p.s == 1 && p.na == 3 && p.no == 85 && p.cout == 255 && p.raw == nullptr &&
         p.kpad == p.cin && p.cin % BKE == 0 && p.cin >= 2 * BKE && hw % 4 == 0 && p.row_off % 4 == 0 &&
         p.nrows % 4 == 0 && p.xoff % 8 == 0 && p.xc % 8 == 0 && p.H == p.Ho && p.W == p.Wo;
}

hipError_t launch_det_pring(const ConvParams& p, int cus, hipStream_t st) {
  const long T = (p.M + 63) / 64;
  const long per = (T + cus - 1) / cus;
  const int grid = (int)((T + per - 1) / per);
  // microbenchmark hooks (scripts/detbench.hip; the ABI never accepts them): 98 = no sigmoid staging,
  // 96 = no tail (decode, row scores, z / record stores), 95 = neither (the GEMM, its ring and the
  // epilogue barriers only)
  // the register-weight head (conv_det_rw_kernel) by default where the plan packed its weights (K = 256 /
  // 512); 94 = the persistent head with staged weights, kept as a forced variant.  YV7_DET_RW=0: off.
  // In-network A/B, same box (profiles/r5_det/rw/, rw512/): 256->255 @80 82.7 -> 67.3 us, 512->255 @40
  // 38.9 -> 35.6 us.
  static const int rw = [] { const char* e = getenv("YV7_DET_RW"); return e ? atoi(e) : 1; }();
  if (rw && (p.variant == 0 || p.variant == 91) && det_rw_supported(p)) {
    if (p.variant == 91) {   // its hook (no pixel DMA)
      if (p.kpad == 256) YV7_LAUNCH((conv_det_rw_kernel<8, 1>), dim3(grid), dim3(512), 0, st, p);
      else YV7_LAUNCH((conv_det_rw_kernel<16, 1>), dim3(grid), dim3(512), 0, st, p);
      return hipGetLastError();
    }
    // YV7_DET_RWD: pixel stages in flight (conv_det_rw_kernel's D; 0 = the round-5 two-slot schedule)
    static const int rwd = [] { const char* e = getenv("YV7_DET_RWD"); return e ? atoi(e) : 4; }();
    // 32-pixel tiles at K = 512 (round 6): 1x1 512->255 @40 at bs 32 is 800 tiles of 64 = 4 rounds on 200
    // blocks, or 1600 of 32 = 7 half-size rounds on 229 — 33.7 -> 31.5 us in-network, same box; at K = 256
    // (256->255 @80, 3200 / 6400 tiles) the halved tiles lose, 60.6 -> 70.0 (profiles/r6_det/bm32/).
    // YV7_DET_BM=32 / 64 forces either.
    static const int bm_env = [] { const char* e = getenv("YV7_DET_BM"); return e ? atoi(e) : 0; }();
    const int bm = bm_env ? bm_env : (p.kpad == 512 ? 32 : 64);
    if (bm == 32 && rwd == 4) {
      const long T2 = (p.M + 31) / 32, per2 = (T2 + cus - 1) / cus;
      const int grid2 = (int)((T2 + per2 - 1) / per2);
      if (p.kpad == 256) YV7_LAUNCH((conv_det_rw_kernel<8, 0, 4, 32>), dim3(grid2), dim3(512), 0, st, p);
      else YV7_LAUNCH((conv_det_rw_kernel<16, 0, 4, 32>), dim3(grid2), dim3(512), 0, st, p);
      return hipGetLastError();
    }
    if (p.kpad == 256) {
      if (rwd == 0) YV7_LAUNCH(conv_det_rw_kernel<8>, dim3(grid), dim3(512), 0, st, p);
      else YV7_LAUNCH((conv_det_rw_kernel<8, 0, 4>), dim3(grid), dim3(512), 0, st, p);
    } else {   // K = 512 (6 and 8 stages ahead measured no faster than 4: profiles/r6_det/ring_k512/)
      if (rwd == 0) YV7_LAUNCH(conv_det_rw_kernel<16>, dim3(grid), dim3(512), 0, st, p);
      else YV7_LAUNCH((conv_det_rw_kernel<16, 0, 4>), dim3(grid), dim3(512), 0, st, p);
    }
    return hipGetLastError();
  }
  // one 64-pixel tile per CU at most (yolov7 bs 32's P5 head): the one-tile head with its deep ring (round 6;
  // YV7_DET_1T=0: off)
  static const int one_tile = [] { const char* e = getenv("YV7_DET_1T"); return e ? atoi(e) : 1; }();
  if (one_tile && p.variant == 0 && T <= cus && det_lds(64, 256) <= 4 * (64 + 256) * ROWB) {
    YV7_LAUNCH(conv_det_1tile_kernel, dim3((unsigned)T), dim3(512), 0, st, p);
    return hipGetLastError();
  }
  if (p.variant == 98) YV7_LAUNCH(conv_det_pring_kernel<1>, dim3(grid), dim3(512), 0, st, p);
  else if (p.variant == 96) YV7_LAUNCH(conv_det_pring_kernel<2>, dim3(grid), dim3(512), 0, st, p);
  else if (p.variant == 95) YV7_LAUNCH(conv_det_pring_kernel<3>, dim3(grid), dim3(512), 0, st, p);
  else if (p.variant == 93) YV7_LAUNCH(conv_det_pring_kernel<4>, dim3(grid), dim3(512), 0, st, p);   // no weight DMA
  else YV7_LAUNCH(conv_det_pring_kernel<0>, dim3(grid), dim3(512), 0, st, p);
  return hipGetLastError();
}

// 2x2 max of four 16-byte fp16 vectors (MP folded into a 1x1 conv's operand loads)
__device__ __forceinline__ u4 hmax4(u4 a, u4 b, u4 c, u4 d) {
  const h8 m = __builtin_elementwise_max(__builtin_elementwise_max(__builtin_bit_cast(h8, a), __builtin_bit_cast(h8, b)),
                                         __builtin_elementwise_max(__builtin_bit_cast(h8, c), __builtin_bit_cast(h8, d)));
  return __builtin_bit_cast(u4, m);
}

// POOL: 1x1 conv over the 2x2 / stride-2 max of the input (ConvParams::pool; k = 1, s = 2, pad = 0): each A
// row's origin is the window's top-left pixel, the other three are fixed byte offsets.
template <int BM, int BN, int WM, bool ONE, bool DET, int PF = 1, bool POOL = false>
__global__ __launch_bounds__(NT, 2) void conv_f16_kernel(const ConvParams p) {
  constexpr int WN = 4 / WM;
  constexpr int WTM = BM / WM, WTN = BN / WN;
  constexpr int TM = WTM / 16, TN = WTN / 16;
  constexpr int RA = BM / 32;                 // A rows per thread (32 rows per pass of 256 threads)
  constexpr int RB = (BN + 31) / 32;
  constexpr int STAGE = (BM + BN) * ROWB;
  constexpr int CPITCH = BN * 2 + 16;
  constexpr int EPI0 = BM * CPITCH + BM * 4;   // staged C tile + output row table
  constexpr int EPI = (DET && det_lds(BM, BN) > EPI0) ? det_lds(BM, BN) : EPI0;
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
  const uint32_t pdx = (uint32_t)p.xc * 2, pdy = (uint32_t)(p.W + 2 * BORDER) * p.xc * 2;   // POOL window steps
  auto gload = [&](int kt, u4 (&ra)[RA], u4 (&rb)[RB]) {
    aw.step(p, kt, [&](int j, uint32_t vo, uint32_t so) {
      if constexpr (POOL) {
        const u4 a = __builtin_bit_cast(u4, __builtin_amdgcn_raw_buffer_load_b128(xr, vo, so, 0));
        const u4 b = __builtin_bit_cast(u4, __builtin_amdgcn_raw_buffer_load_b128(xr, vo + pdx, so, 0));
        const u4 c2 = __builtin_bit_cast(u4, __builtin_amdgcn_raw_buffer_load_b128(xr, vo + pdy, so, 0));
        const u4 d = __builtin_bit_cast(u4, __builtin_amdgcn_raw_buffer_load_b128(xr, vo + pdy + pdx, so, 0));
        ra[j] = hmax4(a, b, c2, d);
      } else {
        ra[j] = __builtin_bit_cast(u4, __builtin_amdgcn_raw_buffer_load_b128(xr, vo, so, 0));
      }
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
    det_epilogue<BM, BN, NT>(p, smem, acc, m0, wm, wn, g, li, tid);
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


// Split-K hand-off between the S blocks of one output tile (last arriver reduces).  Every block
// publishes its fp32 partial tile ([TN*TM][NTH] float4, coalesced) to p.part, then counts itself in
// p.cnt[tile]; the block that counts last sums the S partials in split order 0..S-1 (the result does
// not depend on arrival order), re-arms the counter and runs the epilogue; the others exit.
// Protocol (MI355X_MICROARCH.md, inter-workgroup visibility, write-through form): partial stores
// and loads are sc1 (write-through, L1-bypassing; no agent release fence, whose L2 write-back of
// every dirty line of the XCD would cost more than the split saves), every wave's vmcnt(0), a
// barrier, then one lane's relaxed agent atomic add; the last arriver's waves load after that add
// returned and a barrier.  Each tile's partial lines are written once and read once per launch.
constexpr int CPOL_SC1 = 16;

template <int NTH, int TN, int TM>
__device__ __forceinline__ bool splitk_reduce(const ConvParams& p, unsigned char* smem, f4 (&acc)[TN][TM], int tile,
                                              int ks, int S, int tid) {
  constexpr int Q = TN * TM;
  const auto pr = make_rsrc(p.part, 0x7fffffffu);
  const uint32_t tbase = (uint32_t)tile * S * Q * NTH * 16;
#pragma unroll
  for (int j = 0; j < TN; ++j)
#pragma unroll
    for (int i = 0; i < TM; ++i)
      __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u4, acc[j][i]), pr,
                                             tbase + ((uint32_t)(ks * Q + j * TM + i) * NTH + tid) * 16, 0, CPOL_SC1);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  int* flag = reinterpret_cast<int*>(smem);
  if (tid == 0) {
    const int old = __hip_atomic_fetch_add(p.cnt + tile, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const int last = old == S - 1;
    if (last) __hip_atomic_store(p.cnt + tile, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    *flag = last;
  }
  __syncthreads();
  const bool last = *flag != 0;
  __syncthreads();   // the flag word is epilogue LDS
  if (!last) return false;
  f4 sum[TN][TM];
#pragma unroll
  for (int j = 0; j < TN; ++j)
#pragma unroll
    for (int i = 0; i < TM; ++i) sum[j][i] = f4{0.0f, 0.0f, 0.0f, 0.0f};
  for (int s = 0; s < S; ++s) {
    if (s == ks) {
#pragma unroll
      for (int j = 0; j < TN; ++j)
#pragma unroll
        for (int i = 0; i < TM; ++i) sum[j][i] += acc[j][i];
    } else {
#pragma unroll
      for (int j = 0; j < TN; ++j)
#pragma unroll
        for (int i = 0; i < TM; ++i)
          sum[j][i] += __builtin_bit_cast(
              f4, __builtin_amdgcn_raw_buffer_load_b128(pr, tbase + ((uint32_t)(s * Q + j * TM + i) * NTH + tid) * 16, 0,
                                                        CPOL_SC1));
    }
  }
#pragma unroll
  for (int j = 0; j < TN; ++j)
#pragma unroll
    for (int i = 0; i < TM; ++i) acc[j][i] = sum[j][i];
  return true;
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
template <int BM, int BN, int WM, int WN, int STAGES, bool ONE, bool DET = false>
__global__ __launch_bounds__(64 * WM * WN, (STAGES * (BM + BN) * 128 <= 80 * 1024) ? 2 : 1) void conv_f16_ring_kernel(const ConvParams p) {
  constexpr int NW = WM * WN, NTH = 64 * NW;
  constexpr int WTM = BM / WM, WTN = BN / WN;
  constexpr int TM = WTM / 16, TN = WTN / 16;
  constexpr int RA = BM / 8 / NW, RB = BN / 8 / NW;   // wave-instructions per wave per stage
  static_assert(RA * 8 * NW == BM && RB * 8 * NW == BN, "tile rows must split into 8-row groups per wave");
  constexpr int PER = RA + RB;
  constexpr int STAGE = (BM + BN) * ROWB;
  constexpr int CPITCH = BN * 2 + 16;
  constexpr int EPI0 = BM * CPITCH + BM * 4;
  constexpr int EPI = (DET && det_lds(BM, BN) > EPI0) ? det_lds(BM, BN) : EPI0;
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
  // split-K: the S blocks of one output tile are adjacent work ids, each sums the K steps [kb, ke)
  const int S = (!DET && p.ksplit > 1) ? p.ksplit : 1;
  const int tile = wgid / S, ks = wgid - tile * S;
  const int nN = (p.cout + BN - 1) / BN;
  const int m0 = (tile / nN) * BM, n0 = (tile % nN) * BN;
  const int nk_all = p.kpad / BKE;
  const int kb = ks * nk_all / S, ke = (ks + 1) * nk_all / S;

  const auto xr = make_rsrc(p.x, p.xbytes);
  const auto wr = make_rsrc(p.w, p.wbytes);

  const int lr = lane >> 3;            // row within the 8-row group (== row & 7)
  const int c = (lane & 7) ^ lr;       // source chunk this lane fetches

  AWalk<ONE, RA> aw;
  aw.init(p, c, kb);
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

  const int nk = ke - kb;   // K steps of this block; local step kt is global step kb + kt
  auto issue = [&](int kt, int slot) {
    unsigned char* As = smem + slot * STAGE;
    unsigned char* Bs = As + BM * ROWB;
    aw.step(p, kb + kt, [&](int j, uint32_t vo, uint32_t so) { dma16(xr, As + (j * NW + wave) * 8 * ROWB, vo, so); });
#pragma unroll
    for (int j = 0; j < RB; ++j) dma16(wr, Bs + (j * NW + wave) * 8 * ROWB, b_off[j], (uint32_t)(kb + kt) * BKE * 2);
  };

  // accumulators start at the bias (split 0 only)
  f4 acc[TN][TM];
#pragma unroll
  for (int j = 0; j < TN; ++j) {
    const int col = n0 + wn * WTN + j * 16 + g * 4;
    f4 bv;
#pragma unroll
    for (int e = 0; e < 4; ++e) bv[e] = (col + e < p.cout && ks == 0) ? p.bias[col + e] : 0.0f;
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
    ring_wait<PER, STAGES - 2>(ahead);
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

  if (S > 1 && !splitk_reduce<NTH, TN, TM>(p, smem, acc, tile, ks, S, tid)) return;

  if constexpr (DET) {
    det_epilogue<BM, BN, NTH>(p, smem, acc, m0, wm, wn, g, li, tid);
    return;
  }
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


// ---------------------------------------------------------------------------------------------
// Persistent ring (short-K layers).  Non-persistent tiles pay, per tile, the ring fill latency and
// an LDS-staged epilogue during which nothing streams; for K = 128..512 that is most of the tile.
// Here every block walks tiles t = blockIdx.x, + gridDim.x, ...:
//  * the LDS-DMA ring of K steps runs on across tile boundaries — the next tile's first stages are
//    in flight while the current tile finishes and writes back;
//  * the epilogue goes straight from the accumulators (bias from LDS at accumulator init,
//    compile-time activation, fp16, one v_permlane16_swap per dword so a lane holds 8 consecutive
//    channels, 16-byte stores into the destination channel slice), so the ring never stops for
//    LDS staging;
//  * counted vmcnt waits: the loads younger than the awaited stage are the next stages and, right
//    after a tile boundary, the previous tile's stores (their number is known per step).
// WS > 0: weight-stationary 1x1 form — the layer's whole weight matrix (cout <= BN, K <= WS steps)
// is DMA'd into LDS once per block and every tile's K steps read it from there, so only the
// activation tile streams (a third of the DMA issue of the 256 x 256 ring); bias in registers.
// HOOK (scripts/convbench.hip only, 256 x 256 form; the ABI never accepts them): 296 activation without
// stores, 297 neither, 298 no operand DMA.  Compile-time: a runtime test in the K loop splits the DMA
// issue into a block of its own on every K step of the production kernel.
template <int BM, int BN, int WM, int WN, int STAGES, bool ONE, int ACT, int BK, int WS = 0, int HOOK = 0>
__global__ __launch_bounds__(64 * WM * WN, (STAGES * (BM + BN) * BK * 2 <= 48 * 1024 && WM * WN == 4) ? 3 : (STAGES * (BM + BN) * BK * 2 <= 76 * 1024) ? 2 : 1) void conv_f16_pring_kernel(
    const ConvParams p) {
  constexpr int NW = WM * WN, NTH = 64 * NW;
  constexpr int WTM = BM / WM, WTN = BN / WN;
  constexpr int TM = WTM / 16, TN = WTN / 16;
  constexpr int RB_ = BK * 2;              // LDS bytes per tile row
  constexpr int CPR = RB_ / 16;            // 16-byte chunks per row
  constexpr int RPI = 64 / CPR;            // tile rows per DMA wave-instruction (1 KiB)
  constexpr int RA = BM / RPI / NW, RB = BN / RPI / NW;
  static_assert(RA * RPI * NW == BM && RB * RPI * NW == BN, "tile rows must split into DMA groups per wave");
  static_assert(TN % 2 == 0, "the epilogue pairs 16-channel groups");
  static_assert(STAGES >= 2 && STAGES <= 4, "counted waits cover up to two stages in flight");
  static_assert(WS == 0 || ONE, "weight-stationary form: 1x1 convs only");
  constexpr int PER = RA + (WS ? 0 : RB);
  constexpr int NST = TM * TN / 2;   // epilogue stores per lane per tile
  constexpr int STAGE = (BM + (WS ? 0 : BN)) * RB_;
  constexpr int WREG = WS ? BN * WS * RB_ : 0;   // stationary weights: [K step][BN rows][RB_]
  constexpr int BIAS = WS ? 0 : 4096;            // bias vector (<= 1024 channels) behind the ring
  __shared__ __attribute__((aligned(16))) unsigned char smem[STAGES * STAGE + WREG + BIAS];
  float* bias_l = reinterpret_cast<float*>(smem + STAGES * STAGE + WREG);
  unsigned char* wl = smem + STAGES * STAGE;

  const int tid = threadIdx.x;
  const int lane = tid & 63, wave = tid >> 6;
  const int wm = wave / WN, wn = wave % WN;
  const int g = lane >> 4, li = lane & 15;
  const int lr = lane / CPR;                          // row within the DMA group
  const int c = swz_bk<BK>(lr, lane % CPR);           // source chunk this lane fetches (slot = lane % CPR)

  const int nN = (p.cout + BN - 1) / BN;
  const int nk = p.kpad / BK;
  // N-split weight-stationary form (WS with cout > BN): block b holds output-channel tile nb's weights
  // and walks the M tiles only; the nN blocks of one virtual block share an XCD and walk the same M
  // tiles in the same order, so each activation tile comes from HBM once and from that XCD's L2 for
  // the other N tiles.  The launcher sizes the grid to a multiple of 8 nN.
  const bool nsplit = WS != 0 && nN > 1;
  const int nb = nsplit ? (int)((blockIdx.x / 8) % nN) : 0;
  const int T = nsplit ? (p.M + BM - 1) / BM : ((p.M + BM - 1) / BM) * nN;
  const TileWalk tw = nsplit ? xcd_tile_walk_g(T, gridDim.x / nN, (int)((blockIdx.x / (8 * nN)) * 8 + blockIdx.x % 8))
                             : xcd_tile_walk(T);   // XCD-major persistent tile order
  const int ntl = tw.count();
  if (ntl == 0) return;
  const int nsteps = ntl * nk;
  auto tile_m0 = [&](int t) { return nsplit ? t * BM : (t / nN) * BM; };
  auto tile_n0 = [&](int t) { return nsplit ? nb * BN : (t % nN) * BN; };

  const auto xr = make_rsrc(p.x, p.xbytes);
  const auto wr = make_rsrc(p.w, p.wbytes);
  const auto yr = make_rsrc(p.y, 0x7fffffffu);

  float bias_r[WS ? TN : 1][4];
  if constexpr (WS == 0) {
    for (int i = tid; i < p.cout; i += NTH) bias_l[i] = p.bias[i];
  } else {
    // (one N tile per block: cn0 = nb * BN) this lane's channels, and the tile's weights into LDS once
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int col = nb * BN + wn * WTN + j * 16 + g * 4 + e;
        bias_r[j][e] = col < p.cout ? p.bias[col] : 0.0f;
      }
    constexpr int GPS = BN / RPI;   // DMA groups per K step
    for (int q = wave; q < nk * GPS; q += NW) {
      const int ks = q / GPS, rg = q - ks * GPS;
      dma16(wr, wl + (ks * BN + rg * RPI) * RB_, (uint32_t)(((nb * BN + rg * RPI + lr) * p.kpad + c * 8) * 2),
            (uint32_t)ks * BK * 2);
    }
  }

  // ---- issue cursor: global step ig = (local tile it, step ikt)
  AWalk<ONE, RA, BK> aw;
  uint32_t b_off[RB];
  int ig = 0, it = 0, ikt = 0;
  auto issue_next = [&]() __attribute__((always_inline)) {
    if (ikt == 0) {
      const int t = tw.at(it);
      const int m0 = tile_m0(t), n0 = tile_n0(t);
      aw.init(p, c, 0);
      PixelWalk pw(p, m0 + wave * RPI + lr);
#pragma unroll
      for (int j = 0; j < RA; ++j) {
        if (j) pw.advance(p, NW * RPI);
        aw.off[j] = a_origin(p, pw.b, pw.ho, pw.wo, c);
      }
#pragma unroll
      for (int j = 0; j < RB; ++j) b_off[j] = (uint32_t)(((n0 + (j * NW + wave) * RPI + lr) * p.kpad + c * 8) * 2);
    }
    const int slot = ig % STAGES;
    unsigned char* As = smem + slot * STAGE;
    unsigned char* Bs = As + BM * RB_;
    if constexpr (HOOK != 298) {   // 298: microbenchmark hook, no operand traffic (times the rest)
      aw.step(p, ikt, [&](int j, uint32_t vo, uint32_t so) { dma16(xr, As + (j * NW + wave) * RPI * RB_, vo, so); });
      if constexpr (WS == 0) {
#pragma unroll
        for (int j = 0; j < RB; ++j) dma16(wr, Bs + (j * NW + wave) * RPI * RB_, b_off[j], (uint32_t)ikt * BK * 2);
      }
    }
    ++ig;
    if (++ikt == nk) { ikt = 0; ++it; }
  };

  // ---- compute cursor
  f4 acc[TN][TM];
  int cm0 = 0, cn0 = 0;
  auto init_tile = [&](int i) __attribute__((always_inline)) {
    const int t = tw.at(i);
    cm0 = tile_m0(t);
    cn0 = tile_n0(t);
#pragma unroll
    for (int j = 0; j < TN; ++j) {
      const int col = cn0 + wn * WTN + j * 16 + g * 4;
      f4 bv;
#pragma unroll
      for (int e = 0; e < 4; ++e) bv[e] = WS ? bias_r[WS ? j : 0][e] : (col + e < p.cout ? bias_l[col + e] : 0.0f);
#pragma unroll
      for (int ii = 0; ii < TM; ++ii) acc[j][ii] = bv;
    }
  };
  const uint32_t lane_ch = (uint32_t)(16 * (g & 1) + 8 * (g >> 1));
  auto epilogue = [&]() __attribute__((always_inline)) {
    // the accumulators are final only here: without this the compiler speculates the activation's
    // first instructions (scale, v_exp) for every accumulator into every K step, ahead of the
    // tile-end branch (~20 VALU per step on the 128 x 128 ring)
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
      for (int ii = 0; ii < TM; ++ii) asm volatile("" : "+v"(acc[j][ii]));
    if constexpr (HOOK == 296 || HOOK == 297) {   // microbenchmark hooks: 296 activation, no stores; 297 neither
      float sink = 0.0f;
#pragma unroll
      for (int ii = 0; ii < TM; ++ii)
#pragma unroll
        for (int j = 0; j < TN; ++j)
#pragma unroll
          for (int e = 0; e < 4; ++e) sink += HOOK == 297 ? acc[j][ii][e] : act_t<ACT>(acc[j][ii][e]);
      if (sink == 12345.0f) __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(uint32_t, sink), yr, 0, 0, 0);
      return;
    }
    PixelWalk pw(p, cm0 + wm * WTM + li);
#pragma unroll
    for (int ii = 0; ii < TM; ++ii) {
      if (ii) pw.advance(p, 16);
      const int m = cm0 + wm * WTM + ii * 16 + li;
      const uint32_t yo = (uint32_t)((pix_index(pw.b, pw.ho, pw.wo, p.Ho, p.Wo) * p.yc + p.yoff) * 2);
#pragma unroll
      for (int mp = 0; mp < TN / 2; ++mp) {
        typedef _Float16 h4 __attribute__((ext_vector_type(4)));
        typedef uint32_t u2 __attribute__((ext_vector_type(2)));
        h4 va, vb;
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          va[e] = (_Float16)act_t<ACT>(acc[2 * mp][ii][e]);
          vb[e] = (_Float16)act_t<ACT>(acc[2 * mp + 1][ii][e]);
        }
        const u2 a = __builtin_bit_cast(u2, va), b = __builtin_bit_cast(u2, vb);
        const auto s0 = __builtin_amdgcn_permlane16_swap(a[0], b[0], false, false);
        const auto s1 = __builtin_amdgcn_permlane16_swap(a[1], b[1], false, false);
        const u4 v = {s0[0], s1[0], s0[1], s1[1]};
        const int n = cn0 + wn * WTN + mp * 32 + (int)lane_ch;
        // rows past M / channels past cout: an offset beyond the buffer drops the store
        const uint32_t off = (m < p.M && n < p.cout) ? yo + (uint32_t)n * 2 : 0xffffffffu;
        __builtin_amdgcn_raw_buffer_store_b128(v, yr, off, 0, 0);
      }
    }
  };

#pragma unroll
  for (int s0 = 0; s0 < STAGES - 1; ++s0)
    if (ig < nsteps) issue_next();
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");   // bias_l writes of this wave
  __builtin_amdgcn_s_barrier();
  init_tile(0);

  int ci = 0, ckt = 0;
  // One K step; SLOT = gs % STAGES as a compile-time constant (the loop below is unrolled by STAGES),
  // so every fragment read is a loop-invariant per-lane offset plus an immediate slot offset — no
  // address arithmetic per read and step.
  auto kstep = [&](int gs, auto slotc) __attribute__((always_inline)) {
    constexpr int SLOT = decltype(slotc)::value;   // -1: gs % STAGES at run time
    // stage gs has landed once at most `younger` vector-memory ops of this wave are outstanding
    const int ndma = min(STAGES - 2, nsteps - 1 - gs);
    const bool st = ci > 0 && ckt <= STAGES - 2;
    const int younger = ndma * PER + (st ? NST : 0);
    if (younger == 0) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    else if (younger == PER) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(PER) : "memory");
    else if (younger == 2 * PER) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(2 * PER) : "memory");
    else if (younger == NST) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(NST) : "memory");
    else if (younger == PER + NST) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(PER + NST) : "memory");
    else if (younger == 2 * PER + NST) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(2 * PER + NST) : "memory");
    else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    if (ig < nsteps) issue_next();   // refills the slot every wave finished reading at step gs-1
    const unsigned char* As = smem + (SLOT >= 0 ? SLOT : gs % STAGES) * STAGE;
    const unsigned char* Bs = WS ? wl + ckt * BN * RB_ : As + BM * RB_;
    // every fragment of the step is read up front: the second sub-step's reads are in flight under
    // the first sub-step's MFMAs
    constexpr int NSB = BK / 32;
    u4 xa[NSB][TM], wb[NSB][TN];
#pragma unroll
    for (int sb = 0; sb < NSB; ++sb) {
      const int ch = sb * 4 + g;
#pragma unroll
      for (int ii = 0; ii < TM; ++ii) {
        const int row = wm * WTM + ii * 16 + li;
        xa[sb][ii] = *reinterpret_cast<const u4*>(As + row * RB_ + swz_bk<BK>(row, ch) * 16);
      }
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        const int row = wn * WTN + j * 16 + li;
        wb[sb][j] = *reinterpret_cast<const u4*>(Bs + row * RB_ + swz_bk<BK>(row, ch) * 16);
      }
    }
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int sb = 0; sb < NSB; ++sb)
#pragma unroll
      for (int j = 0; j < TN; ++j)
#pragma unroll
        for (int ii = 0; ii < TM; ++ii)
          acc[j][ii] = __builtin_amdgcn_mfma_f32_16x16x32_f16(__builtin_bit_cast(h8, wb[sb][j]),
                                                              __builtin_bit_cast(h8, xa[sb][ii]), acc[j][ii], 0, 0, 0);
    __builtin_amdgcn_s_setprio(0);
    if (++ckt == nk) {
      epilogue();
      ckt = 0;
      if (++ci < ntl) init_tile(ci);
    }
  };
  int gs = 0;
  // unrolled only where every slot offset fits a ds_read immediate (16 bits): the 64 KiB stages of the
  // 256 x 256 ring would need a second base register per slot and spill
  constexpr bool UNROLL = STAGES * STAGE <= 65536;
  if constexpr (!UNROLL) {
    for (; gs < nsteps; ++gs) kstep(gs, std::integral_constant<int, -1>{});
  }
  for (; UNROLL && gs + STAGES <= nsteps; gs += STAGES) {
    kstep(gs, std::integral_constant<int, 0>{});
    kstep(gs + 1, std::integral_constant<int, 1>{});
    if constexpr (STAGES > 2) kstep(gs + 2, std::integral_constant<int, (STAGES > 2 ? 2 : 0)>{});
    if constexpr (STAGES > 3) kstep(gs + 3, std::integral_constant<int, (STAGES > 3 ? 3 : 0)>{});
  }
  if constexpr (UNROLL) {
    if (gs < nsteps) kstep(gs++, std::integral_constant<int, 0>{});   // remainder: slots 0, 1, 2 in order
    if (STAGES > 2 && gs < nsteps) kstep(gs++, std::integral_constant<int, 1>{});
    if (STAGES > 3 && gs < nsteps) kstep(gs++, std::integral_constant<int, (STAGES > 3 ? 2 : 0)>{});
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

// ---------------------------------------------------------------------------------------------
// 8-phase persistent ring (256 x 256 tiles, 8 waves = 2 stagger groups x 4, BK 64): the structure of
// the guide's 256^2 "8-phase" GEMM template (cdna_hip_programming.md §5: counted vmcnt across raw
// barriers, one half-tile of LDS-DMA per phase, two wave groups offset by one barrier so that one
// group's MFMA cluster runs while the other issues its LDS reads and DMA), rebuilt for the implicit
// GEMM of a conv and made persistent across output tiles like conv_f16_pring_kernel.
//
//  * LDS: two K-tile buffers, each four 16 KiB half-tiles [A0 A1 B0 B1] (A = 128 pixel rows,
//    B = 128 weight rows, 64 k each, XOR-swizzled 128-byte rows as everywhere here) + the bias.
//  * K-tile k runs four phases, one block quadrant (ha, hb) each in the order (0,0) (0,1) (1,1) (1,0):
//    every wave computes its 64 x 32 part of the quadrant (16 MFMAs), reading A half ha (8
//    ds_read_b128) and/or B half hb (4): phase 0 both, then B1, A1, B0 — so the halves' last reads
//    fall in phases 0 (A0), 1 (B1), 2 (A1), 3 (B0).
//  * every wave retires its phase's LDS reads (lgkmcnt(0)) before the phase's first barrier, so a
//    half can be restaged ONE phase after its last read even with the groups staggered (the other
//    group's DMA issue follows that barrier): phase 0 stages B0 of k+1, phase 1 A0 of k+2, phase 2
//    B1 of k+2, phase 3 A1 of k+2; the only wait is phase 3's vmcnt(6): K-tile k+1 retired, three
//    halves of k+2 still in flight, and the reads of k+1 start one phase (and so one more barrier of
//    the other group) later.
//  * the finished tile's epilogue (bias in the accumulators, activation, fp16, permlane16 pairing,
//    16-byte NHWC stores) runs between the last K-tile's phase 3 and the next tile's phase 0.
// acc[hb][j][ha][i] = channels hb*128 + wn*32 + j*16 + g*4 + e of pixel ha*128 + wm*64 + i*16 + li.
// Persistent tile order: XCD-major (xcd_tile_walk; 1x1 1024->1024 @40 140 -> 133 us, tune_ops).  The
// round-2 schedule experiments (DMA before the reads, no s_setprio, one group retiring early, B half 0
// kept in registers, stream-K, 512 x 128 tiles: DESIGN §4.5, §8) were removed in round 4.
template <bool ONE, int ACT, int BM = 256, int BN = 256>
__global__ __launch_bounds__(512, 1) void conv_f16_p8_kernel(const ConvParams p) {
  constexpr int NTH = 512;
  constexpr int AHR = BM / 2, BHR = BN / 2;          // rows per A / B half-tile
  constexpr int AHB = AHR * ROWB, BHB = BHR * ROWB;  // bytes per A / B half-tile
  constexpr int BUF = 2 * AHB + 2 * BHB;             // one K-tile: A0 A1 B0 B1
  constexpr int AP = AHR / 64, BP = BHR / 64;        // 1 KiB DMA pieces per wave per A / B half
  constexpr int VMC = 2 * AP + BP;                   // loads of three half-tiles (A0, B1, A1) per wave
  constexpr int WNC = BHR / 32;                      // waves across a B half (32 channels each)
  static_assert(AP >= 1 && BP >= 1 && (AHR / 64) * WNC == 8, "8 waves of 64 x 32 per block quadrant");
  constexpr int BIASB = (2 * BUF + 4096 + 16 <= 163840) ? 4096 : 0;   // bias in LDS when it fits
  __shared__ __attribute__((aligned(16))) unsigned char smem[2 * BUF + BIASB];
  float* bias_l = reinterpret_cast<float*>(smem + 2 * BUF);

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave / WNC, wn = wave % WNC;
  const int grp = wave >> 2;                         // stagger group (one wave of each per SIMD)
  const int g = lane >> 4, li = lane & 15;
  const int lr = lane >> 3;                          // DMA: row within an 8-row piece
  const int c = (lane & 7) ^ lr;                     // DMA: source chunk of slot lane & 7

  const int nN = (p.cout + BN - 1) / BN;
  const int T = ((p.M + BM - 1) / BM) * nN;
  const int nk = p.kpad / BKE;
  const TileWalk tw = xcd_tile_walk(T);
  const int ntl = tw.count();
  const int total = ntl * nk;                        // K-tiles this block computes
  if (total == 0) return;
  auto tile_at = [&](int it) { return tw.at(it); };

  const auto xr = make_rsrc(p.x, p.xbytes);
  const auto wr = make_rsrc(p.w, p.wbytes);
  const auto yr = make_rsrc(p.y, 0x7fffffffu);
  if constexpr (BIASB != 0)
    for (int i = tid; i < p.cout; i += NTH) bias_l[i] = p.bias[i];

  // ---- staging cursors (A and B halves are staged in different phases, each in K-tile order)
  int a_it = 0, a_kt = 0, b_it = 0, b_kt = 0;
  uint32_t a_off[2][AP], b_off[2][BP], a_so = 0;
  KWalk sa, sb;   // (!ONE) the A and B halves' chunk-major K walks (staged in different phases)
  auto stage_a = [&](int h, int par) {   // half h (0 / 1) of the next A K-tile, into buffer par
    if (h == 0) {
      if (a_kt == 0) {
        const int t = tile_at(a_it);
        PixelWalk pw(p, (t / nN) * BM + wave * 8 + lr);
#pragma unroll
        for (int q = 0; q < 2 * AP; ++q) {
          if (q) pw.advance(p, 64);
          a_off[q / AP][q % AP] = a_origin(p, pw.b, pw.ho, pw.wo, c);
        }
        sa.init();
      }
      a_so = ONE ? (uint32_t)a_kt * BKE * 2 : sa.a_offset(p);
      if (!ONE) sa.advance(p);
    }
    unsigned char* d = smem + par * BUF + h * AHB;
#pragma unroll
    for (int j = 0; j < AP; ++j) dma16(xr, d + (j * 8 + wave) * 8 * ROWB, a_off[h][j], a_so);
    if (h == 1) {
      if (++a_kt == nk) { a_kt = 0; ++a_it; }
    }
  };
  uint32_t b_so = 0;
  auto stage_b = [&](int h, int par) {   // half h of the next B K-tile into buffer par; B1 first, then B0
    if (h == 1) {
      if (b_kt == 0) {
        const int n0 = tile_at(b_it) % nN * BN;
#pragma unroll
        for (int q = 0; q < 2 * BP; ++q)
          b_off[q / BP][q % BP] =
              (uint32_t)(((n0 + (q / BP) * BHR + ((q % BP) * 8 + wave) * 8 + lr) * p.kpad + c * 8) * 2);
        sb.init();
      }
      b_so = ONE ? (uint32_t)b_kt * BKE * 2 : sb.b_offset(p);
      if (!ONE) sb.advance(p);
    }
    unsigned char* d = smem + par * BUF + 2 * AHB + h * BHB;
#pragma unroll
    for (int j = 0; j < BP; ++j) dma16(wr, d + (j * 8 + wave) * 8 * ROWB, b_off[h][j], b_so);
    if (h == 0) {
      if (++b_kt == nk) { b_kt = 0; ++b_it; }
    }
  };

  // ---- compute side
  f4 acc[2][2][2][4];
  int cm0 = 0, cn0 = 0;
  auto init_tile = [&](int i) {
    const int t = tile_at(i);
    cm0 = (t / nN) * BM;
    cn0 = (t % nN) * BN;
#pragma unroll
    for (int hb = 0; hb < 2; ++hb)
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        const int col = cn0 + hb * BHR + wn * 32 + j * 16 + g * 4;
        f4 bv;
#pragma unroll
        for (int e = 0; e < 4; ++e)
          bv[e] = col + e < p.cout ? (BIASB ? bias_l[col + e] : p.bias[col + e]) : 0.0f;
#pragma unroll
        for (int ha = 0; ha < 2; ++ha)
#pragma unroll
          for (int i = 0; i < 4; ++i) acc[hb][j][ha][i] = bv;
      }
  };
  const uint32_t lane_ch = (uint32_t)(16 * (g & 1) + 8 * (g >> 1));
  auto epilogue = [&]() {
#pragma unroll
    for (int ha = 0; ha < 2; ++ha) {
      PixelWalk pw(p, cm0 + ha * AHR + wm * 64 + li);
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        if (i) pw.advance(p, 16);
        const int m = cm0 + ha * AHR + wm * 64 + i * 16 + li;
        const uint32_t yo = (uint32_t)((pix_index(pw.b, pw.ho, pw.wo, p.Ho, p.Wo) * p.yc + p.yoff) * 2);
#pragma unroll
        for (int hb = 0; hb < 2; ++hb) {
          typedef _Float16 h4 __attribute__((ext_vector_type(4)));
          typedef uint32_t u2 __attribute__((ext_vector_type(2)));
          h4 va, vb;
          const f4 a0 = acc[hb][0][ha][i], a1 = acc[hb][1][ha][i];
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            va[e] = (_Float16)act_t<ACT>(a0[e]);
            vb[e] = (_Float16)act_t<ACT>(a1[e]);
          }
          const u2 a = __builtin_bit_cast(u2, va), b = __builtin_bit_cast(u2, vb);
          const auto s0 = __builtin_amdgcn_permlane16_swap(a[0], b[0], false, false);
          const auto s1 = __builtin_amdgcn_permlane16_swap(a[1], b[1], false, false);
          const u4 v = {s0[0], s1[0], s0[1], s1[1]};
          const int n = cn0 + hb * BHR + wn * 32 + (int)lane_ch;
          const uint32_t off = (m < p.M && n < p.cout) ? yo + (uint32_t)n * 2 : 0xffffffffu;
          __builtin_amdgcn_raw_buffer_store_b128(v, yr, off, 0, 0);
        }
      }
    }
  };

  // ---- prologue: K-tile 0 whole, K-tile 1's A0, B1 and A1 in flight
  stage_a(0, 0); stage_b(1, 0); stage_a(1, 0); stage_b(0, 0);
  if (total > 1) {
    stage_a(0, 1); stage_b(1, 1); stage_a(1, 1);
    asm volatile("s_waitcnt vmcnt(%0)" ::"n"(VMC) : "memory");
  } else {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");   // bias_l
  __builtin_amdgcn_s_barrier();
  int ci = 0, ckt = 0;   // compute cursor: tile, K step
  init_tile(ci);
  if (grp == 1) __builtin_amdgcn_s_barrier();   // group 1 runs one barrier behind group 0

  u4 xa[2][4], wb[2][2];
  auto read_a = [&](const unsigned char* h) {
#pragma unroll
    for (int sb = 0; sb < 2; ++sb)
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int row = wm * 64 + i * 16 + li;
        xa[sb][i] = *reinterpret_cast<const u4*>(h + row * ROWB + swz(row, sb * 4 + g) * 16);
      }
  };
  auto read_b = [&](const unsigned char* h) {
#pragma unroll
    for (int sb = 0; sb < 2; ++sb)
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        const int row = wn * 32 + j * 16 + li;
        wb[sb][j] = *reinterpret_cast<const u4*>(h + row * ROWB + swz(row, sb * 4 + g) * 16);
      }
  };
  auto mfma_q = [&](int ha, int hb) {
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");   // this phase's reads retired (WAR: see above)
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int sb = 0; sb < 2; ++sb)
#pragma unroll
      for (int j = 0; j < 2; ++j)
#pragma unroll
        for (int i = 0; i < 4; ++i)
          acc[hb][j][ha][i] = __builtin_amdgcn_mfma_f32_16x16x32_f16(__builtin_bit_cast(h8, wb[sb][j]),
                                                                     __builtin_bit_cast(h8, xa[sb][i]),
                                                                     acc[hb][j][ha][i], 0, 0, 0);
    __builtin_amdgcn_s_setprio(0);
    __builtin_amdgcn_s_barrier();
  };

  // one K-tile: four phases over buffer par (K-tile k + 1's B0 and K-tile k + 2's A0, B1, A1 staged on
  // the way when n1 / n2)
  auto ktile = [&](auto par, bool n1, bool n2) __attribute__((always_inline)) {
    const int P = par;   // a compile-time constant (integral_constant) or the K-tile's parity
    const unsigned char* bk = smem + P * BUF;
    // phase 0: quadrant (0,0)
    read_b(bk + 2 * AHB);
    read_a(bk);
    if (n1) stage_b(0, P ^ 1);
    mfma_q(0, 0);
    // phase 1: (0,1)
    read_b(bk + 2 * AHB + BHB);
    if (n2) stage_a(0, P);
    mfma_q(0, 1);
    // phase 2: (1,1)
    read_a(bk + AHB);
    if (n2) stage_b(1, P);
    mfma_q(1, 1);
    // phase 3: (1,0); K-tile k+1 retired (k+2's A0, B1 and A1 may stay in flight)
    read_b(bk + 2 * AHB);
    if (n2) {
      stage_a(1, P);
      asm volatile("s_waitcnt vmcnt(%0)" ::"n"(VMC) : "memory");
    } else {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    mfma_q(1, 0);
  };
  // (ONE, nk even) the staging without cursors: the A / B halves' offsets for tile t (fresh_*), and one
  // half's LDS-DMA at K offset so into buffer par
  auto fresh_a = [&](int t) __attribute__((always_inline)) {
    PixelWalk pw(p, (t / nN) * BM + wave * 8 + lr);
#pragma unroll
    for (int q = 0; q < 2 * AP; ++q) {
      if (q) pw.advance(p, 64);
      a_off[q / AP][q % AP] = a_origin(p, pw.b, pw.ho, pw.wo, c);
    }
  };
  auto fresh_b = [&](int t) __attribute__((always_inline)) {
    const int n0 = t % nN * BN;
#pragma unroll
    for (int q = 0; q < 2 * BP; ++q)
      b_off[q / BP][q % BP] = (uint32_t)(((n0 + (q / BP) * BHR + ((q % BP) * 8 + wave) * 8 + lr) * p.kpad + c * 8) * 2);
  };
  auto dma_a = [&](int h, int par, uint32_t so) __attribute__((always_inline)) {
    unsigned char* d = smem + par * BUF + h * AHB;
#pragma unroll
    for (int j = 0; j < AP; ++j) dma16(xr, d + (j * 8 + wave) * 8 * ROWB, a_off[h][j], so);
  };
  auto dma_b = [&](int h, int par, uint32_t so) __attribute__((always_inline)) {
    unsigned char* d = smem + par * BUF + 2 * AHB + h * BHB;
#pragma unroll
    for (int j = 0; j < BP; ++j) dma16(wr, d + (j * 8 + wave) * 8 * ROWB, b_off[h][j], so);
  };
  // the same four phases, staging K-tile k + 1's B0 at so1 and K-tile k + 2's A0, B1, A1 at so2 (of tile t2,
  // whose offsets are computed first when fresh2)
  auto ktile_one = [&](auto par, bool n1, bool n2, uint32_t so1, uint32_t so2, bool fresh2, int t2)
      __attribute__((always_inline)) {
    constexpr int P = decltype(par)::value;
    const unsigned char* bk = smem + P * BUF;
    read_b(bk + 2 * AHB);
    read_a(bk);
    if (n1) dma_b(0, P ^ 1, so1);
    mfma_q(0, 0);
    read_b(bk + 2 * AHB + BHB);
    if (n2) {
      if (fresh2) fresh_a(t2);
      dma_a(0, P, so2);
    }
    mfma_q(0, 1);
    read_a(bk + AHB);
    if (n2) {
      if (fresh2) fresh_b(t2);
      dma_b(1, P, so2);
    }
    mfma_q(1, 1);
    read_b(bk + 2 * AHB);
    if (n2) {
      dma_a(1, P, so2);
      asm volatile("s_waitcnt vmcnt(%0)" ::"n"(VMC) : "memory");
    } else {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    mfma_q(1, 0);
  };
  if (ONE && (nk & 1) == 0) {
    // 1x1, nk even: the staging cursors follow from the compute cursor.  The pair (ckt, ckt + 1) stages
    // K-tiles ckt + 1 .. ckt + 3; only ckt + 2 == nk moves the staging to the next tile, and then K-tile
    // k + 2 (the even K-tile's A0 / B1 / A1) is that tile's first: its offsets are computed there, once.
    for (int k = 0; k < total; k += 2) {
      const bool more = k + 2 < total;
      const bool wrap = ckt + 2 == nk;
      const uint32_t s2 = wrap ? 0u : (uint32_t)(ckt + 2) * BKE * 2;
      ktile_one(std::integral_constant<int, 0>{}, true, more, (uint32_t)(ckt + 1) * BKE * 2, s2, wrap,
                wrap && more ? tile_at(ci + 1) : 0);
      ktile_one(std::integral_constant<int, 1>{}, more, more, s2, s2 + BKE * 2, false, 0);
      ckt += 2;
      if (ckt == nk) {
        epilogue();
        if (more) {
          ckt = 0;
          init_tile(++ci);
        }
      }
    }
  } else if ((nk & 1) == 0) {
    // nk even (round 6): every tile starts on an even K-tile, so two K-tiles per trip give each phase its
    // buffer as a compile-time constant (the LDS read bases and DMA destinations are loop-invariant
    // instead of recomputed from the K-tile's parity every phase), and only the odd K-tile can end a tile.
    // total is even: n1 holds for the even K-tile, and k + 2 < total stands for the rest.
    for (int k = 0; k < total; k += 2) {
      const bool more = k + 2 < total;
      ktile(std::integral_constant<int, 0>{}, true, more);
      ktile(std::integral_constant<int, 1>{}, more, more);
      ckt += 2;
      if (ckt == nk) {
        epilogue();
        if (more) {
          ckt = 0;
          init_tile(++ci);
        }
      }
    }
  } else {
    for (int k = 0; k < total; ++k) {
      ktile(k & 1, k + 1 < total, k + 2 < total);
      if (++ckt == nk) {
        epilogue();
        if (k != total - 1) {
          ckt = 0;
          init_tile(++ci);
        }
      }
    }
  }
  if (grp == 0) __builtin_amdgcn_s_barrier();   // equal barrier counts in both groups
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

template <bool ONE>
hipError_t launch_p8_t(const ConvParams& p, int grid, hipStream_t st) {
  if (p.act == 1) YV7_LAUNCH((conv_f16_p8_kernel<ONE, 1>), dim3(grid), dim3(512), 0, st, p);
  else if (p.act == 2) YV7_LAUNCH((conv_f16_p8_kernel<ONE, 2>), dim3(grid), dim3(512), 0, st, p);
  else YV7_LAUNCH((conv_f16_p8_kernel<ONE, 0>), dim3(grid), dim3(512), 0, st, p);
  return hipGetLastError();
}

// 8-phase-style persistent ring for 256 x 128 tiles (128-channel outputs, and 256-channel layers
// with too few 256 x 256 tiles): 8 waves in two stagger groups as in conv_f16_p8_kernel, but with
// three K-tile buffers of 48 KiB [A0 A1 B0 B1] (A halves 128 pixel rows, B halves 64 weight rows),
// two phases per K-tile (phase h: A half h x the whole B tile, 16 MFMAs per wave on its 32 x 64
// part), K-tile k+2 staged during K-tile k (A_h + B_h in phase h) into the buffer K-tile k-1 left,
// and one counted vmcnt(6) per K-tile that retires K-tile k+1.
// acc[h][j][i] = channels wn*64 + j*16 + g*4 + e of pixel h*128 + wm*32 + i*16 + li.
template <bool ONE, int ACT>
__global__ __launch_bounds__(512, 1) void conv_f16_p8n_kernel(const ConvParams p) {
  constexpr int BM = 256, BN = 128, NTH = 512;
  constexpr int AH = 128 * 128, BH = 64 * 128;
  constexpr int BUF = 2 * AH + 2 * BH;
  __shared__ __attribute__((aligned(16))) unsigned char smem[3 * BUF + 4096];
  float* bias_l = reinterpret_cast<float*>(smem + 3 * BUF);

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int grp = wave >> 2;                         // stagger group (one wave of each per SIMD)
  const int wm = wave >> 1, wn = wave & 1;
  const int g = lane >> 4, li = lane & 15;
  const int lr = lane >> 3;
  const int c = (lane & 7) ^ lr;

  const int nN = (p.cout + BN - 1) / BN;
  const int T = ((p.M + BM - 1) / BM) * nN;
  const int nk = p.kpad / BKE;
  // XCD-major tile order (round 5): the nN tiles of one pixel block run on one XCD and share its input
  // rows in that L2 (round robin put them on nN different XCDs)
  const TileWalk tw = xcd_tile_walk(T);
  const int ntl = tw.count();
  const int total = ntl * nk;
  if (total == 0) return;

  const auto xr = make_rsrc(p.x, p.xbytes);
  const auto wr = make_rsrc(p.w, p.wbytes);
  const auto yr = make_rsrc(p.y, 0x7fffffffu);
  for (int i = tid; i < p.cout; i += NTH) bias_l[i] = p.bias[i];

  // ---- staging cursor: K-tile s_gk, half h = A half h + B half h
  int s_it = 0, s_kt = 0;
  uint32_t a_off[2][2], b_off[2], a_so = 0, b_so = 0;
  KWalk su;
  auto stage = [&](int h, int par) {   // half h of the next K-tile into buffer par
    if (h == 0) {
      if (s_kt == 0) {
        const int t = tw.at(s_it);
        PixelWalk pw(p, (t / nN) * BM + wave * 8 + lr);
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          if (q) pw.advance(p, 64);
          a_off[q >> 1][q & 1] = a_origin(p, pw.b, pw.ho, pw.wo, c);
        }
        const int n0 = t % nN * BN;
#pragma unroll
        for (int q = 0; q < 2; ++q) b_off[q] = (uint32_t)(((n0 + q * 64 + wave * 8 + lr) * p.kpad + c * 8) * 2);
        su.init();
      }
      a_so = ONE ? (uint32_t)s_kt * BKE * 2 : su.a_offset(p);
      b_so = ONE ? (uint32_t)s_kt * BKE * 2 : su.b_offset(p);
      if (!ONE) su.advance(p);
    }
    unsigned char* d = smem + par * BUF;
#pragma unroll
    for (int j = 0; j < 2; ++j) dma16(xr, d + h * AH + (j * 8 + wave) * 8 * ROWB, a_off[h][j], a_so);
    dma16(wr, d + 2 * AH + h * BH + wave * 8 * ROWB, b_off[h], b_so);
    if (h == 1) {
      if (++s_kt == nk) { s_kt = 0; ++s_it; }
    }
  };

  f4 acc[2][4][2];
  int cm0 = 0, cn0 = 0;
  auto init_tile = [&](int i) {
    const int t = tw.at(i);
    cm0 = (t / nN) * BM;
    cn0 = (t % nN) * BN;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int col = cn0 + wn * 64 + j * 16 + g * 4;
      f4 bv;
#pragma unroll
      for (int e = 0; e < 4; ++e) bv[e] = col + e < p.cout ? bias_l[col + e] : 0.0f;
#pragma unroll
      for (int h = 0; h < 2; ++h)
#pragma unroll
        for (int i = 0; i < 2; ++i) acc[h][j][i] = bv;
    }
  };
  const uint32_t lane_ch = (uint32_t)(16 * (g & 1) + 8 * (g >> 1));
  auto epilogue = [&]() {
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      PixelWalk pw(p, cm0 + h * 128 + wm * 32 + li);
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        if (i) pw.advance(p, 16);
        const int m = cm0 + h * 128 + wm * 32 + i * 16 + li;
        const uint32_t yo = (uint32_t)((pix_index(pw.b, pw.ho, pw.wo, p.Ho, p.Wo) * p.yc + p.yoff) * 2);
#pragma unroll
        for (int mp = 0; mp < 2; ++mp) {
          typedef _Float16 h4 __attribute__((ext_vector_type(4)));
          typedef uint32_t u2 __attribute__((ext_vector_type(2)));
          h4 va, vb;
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            va[e] = (_Float16)act_t<ACT>(acc[h][2 * mp][i][e]);
            vb[e] = (_Float16)act_t<ACT>(acc[h][2 * mp + 1][i][e]);
          }
          const u2 a = __builtin_bit_cast(u2, va), b = __builtin_bit_cast(u2, vb);
          const auto s0 = __builtin_amdgcn_permlane16_swap(a[0], b[0], false, false);
          const auto s1 = __builtin_amdgcn_permlane16_swap(a[1], b[1], false, false);
          const u4 v = {s0[0], s1[0], s0[1], s1[1]};
          const int n = cn0 + wn * 64 + mp * 32 + (int)lane_ch;
          const uint32_t off = (m < p.M && n < p.cout) ? yo + (uint32_t)n * 2 : 0xffffffffu;
          __builtin_amdgcn_raw_buffer_store_b128(v, yr, off, 0, 0);
        }
      }
    }
  };

  // ---- prologue: K-tiles 0 and 1 staged, 0 retired
  stage(0, 0); stage(1, 0);
  if (total > 1) {
    stage(0, 1); stage(1, 1);
    asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
  } else {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  init_tile(0);
  if (grp == 1) __builtin_amdgcn_s_barrier();

  u4 xa[2][2], wb[2][4];
  auto mfma_h = [&](int h) {
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int sb = 0; sb < 2; ++sb)
#pragma unroll
      for (int j = 0; j < 4; ++j)
#pragma unroll
        for (int i = 0; i < 2; ++i)
          acc[h][j][i] = __builtin_amdgcn_mfma_f32_16x16x32_f16(__builtin_bit_cast(h8, wb[sb][j]),
                                                                __builtin_bit_cast(h8, xa[sb][i]), acc[h][j][i], 0, 0, 0);
    __builtin_amdgcn_s_setprio(0);
    __builtin_amdgcn_s_barrier();
  };
  auto read_a = [&](const unsigned char* ah) {
#pragma unroll
    for (int sb = 0; sb < 2; ++sb)
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        const int row = wm * 32 + i * 16 + li;
        xa[sb][i] = *reinterpret_cast<const u4*>(ah + row * ROWB + swz(row, sb * 4 + g) * 16);
      }
  };

  // one K-tile over buffer par (K-tile k + 2 staged on the way into buffer (par + 2) % 3 when n2)
  auto ktile = [&](auto par, bool n2) __attribute__((always_inline)) {
    const int P = par;   // a compile-time constant (integral_constant) or k % 3
    const unsigned char* bk = smem + P * BUF;
    const int P2 = P == 0 ? 2 : P - 1;
    // phase 0: the wave's whole B part (kept for phase 1) + A half 0
#pragma unroll
    for (int sb = 0; sb < 2; ++sb)
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int row = j * 16 + li;   // within B half wn
        wb[sb][j] = *reinterpret_cast<const u4*>(bk + 2 * AH + wn * BH + row * ROWB + swz(row, sb * 4 + g) * 16);
      }
    read_a(bk);
    if (n2) stage(0, P2);
    mfma_h(0);
    // phase 1: A half 1; K-tile k+1 retired (k+2 may stay in flight)
    read_a(bk + AH);
    if (n2) {
      stage(1, P2);
      asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
    } else {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    mfma_h(1);
  };
  int ci = 0, ckt = 0;
  if (nk % 3 == 0) {
    // nk a multiple of 3 (every 3x3 layer here: nk = 9 cin / 64; round 6): every tile starts on a K-tile
    // k = 0 mod 3, so three K-tiles per trip give each its buffer as a compile-time constant, and only the
    // third can end a tile
    for (int k = 0; k < total; k += 3) {
      ktile(std::integral_constant<int, 0>{}, k + 2 < total);
      ktile(std::integral_constant<int, 1>{}, k + 3 < total);
      ktile(std::integral_constant<int, 2>{}, k + 4 < total);
      ckt += 3;
      if (ckt == nk) {
        epilogue();
        ckt = 0;
        if (++ci < ntl) init_tile(ci);
      }
    }
  } else {
    for (int k = 0; k < total; ++k) {
      ktile(k % 3, k + 2 < total);
      if (++ckt == nk) {
        epilogue();
        ckt = 0;
        if (++ci < ntl) init_tile(ci);
      }
    }
  }
  if (grp == 0) __builtin_amdgcn_s_barrier();
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

template <bool ONE>
hipError_t launch_p8n_t(const ConvParams& p, int grid, hipStream_t st) {
  if (p.act == 1) YV7_LAUNCH((conv_f16_p8n_kernel<ONE, 1>), dim3(grid), dim3(512), 0, st, p);
  else if (p.act == 2) YV7_LAUNCH((conv_f16_p8n_kernel<ONE, 2>), dim3(grid), dim3(512), 0, st, p);
  else YV7_LAUNCH((conv_f16_p8n_kernel<ONE, 0>), dim3(grid), dim3(512), 0, st, p);
  return hipGetLastError();
}

template <int BM, int BN, int WM, int WN, int STAGES, bool ONE, int BK>
hipError_t launch_pring_act(const ConvParams& p, int grid, hipStream_t st) {
  if (p.act == 1)
    YV7_LAUNCH((conv_f16_pring_kernel<BM, BN, WM, WN, STAGES, ONE, 1, BK>), dim3(grid), dim3(64 * WM * WN), 0, st, p);
  else if (p.act == 2)
    YV7_LAUNCH((conv_f16_pring_kernel<BM, BN, WM, WN, STAGES, ONE, 2, BK>), dim3(grid), dim3(64 * WM * WN), 0, st, p);
  else
    YV7_LAUNCH((conv_f16_pring_kernel<BM, BN, WM, WN, STAGES, ONE, 0, BK>), dim3(grid), dim3(64 * WM * WN), 0, st, p);
  return hipGetLastError();
}

int device_cus() {
  static const int n = [] {
    int dev = 0, v = 0;
    if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&v, hipDeviceAttributeMultiprocessorCount, dev) !=
                                                 hipSuccess || v <= 0)
      v = 256;
    return v;
  }();
  return n;
}

template <int HOOK>
hipError_t launch_pring_hook(const ConvParams& p, bool one, hipStream_t st) {
  const long T = (long)((p.M + 255) / 256) * ((p.cout + 255) / 256);
  const int grid = (int)(T < (long)device_cus() ? T : (long)device_cus());
  if (one) YV7_LAUNCH((conv_f16_pring_kernel<256, 256, 2, 4, 2, true, 1, 64, 0, HOOK>), dim3(grid), dim3(512), 0, st, p);
  else YV7_LAUNCH((conv_f16_pring_kernel<256, 256, 2, 4, 2, false, 1, 64, 0, HOOK>), dim3(grid), dim3(512), 0, st, p);
  return hipGetLastError();
}

// the 8-phase persistent ring: uniform K steps only (1x1, or cin % 64 == 0)
int env_variant() {
  static const int v = [] { const char* e = getenv("YV7_CONV_F16"); return e ? atoi(e) : 0; }();
  return v;
}

// The dispatch's 8-phase-ring rule (launch_conv_f16 quotes the measurements behind it).
bool p8_default(const ConvParams& p) {
  static const int on = [] { const char* e = getenv("YV7_P8"); return e ? atoi(e) : 1; }();
  const bool one = p.k == 1 && p.s == 1 && p.pad == 0;
  const long t256 = (long)((p.M + 255) / 256) * ((p.cout + 255) / 256);
  // (1x1 K = 512 -> 512 @80, 1600 tiles: 167 -> 159 us in-network, profiles/r3u_tune.txt)
  // Round 4, yolov7-w6 1280 bs 8 (profiles/r4_w6stem/tune_w6_dispatch.txt, one layer forced at a time,
  // us): 1x1 768->768 @40 31.2 -> 28.4 and 1536->768 @40 49.9 -> 44.2 at 150 tiles; 3x3 s2 128->256
  // @320 183.1 -> 156.1 and @160 47.0 -> 40.0 (the 128-input stride-2 layers).
  const bool w6 = t256 >= 150 && ((one && p.K >= 768 && p.cout >= 768) ||
                                  (p.k == 3 && p.s == 2 && p.cin == 128 && p.cout >= 256 && t256 >= 200));
  return on && !p.pool && p.cout >= 256 && p.cout <= 1024 && p.cout % 8 == 0 &&
         ((t256 >= 200 && ((one && p.K >= 1024) || (one && p.K >= 512 && p.cout >= 512 && t256 >= 1600) ||
                           (p.k == 3 && p.cin >= 256 && p.cin % BKE == 0))) ||
          w6);
}

hipError_t launch_p8(const ConvParams& p, bool one, hipStream_t st) {
  if (p.cout > 1024 || p.cout % 8 || p.yoff % 8 || p.yc % 8 || (!one && p.cin % BKE)) return hipErrorInvalidValue;
  const long T = (long)((p.M + 255) / 256) * ((p.cout + 255) / 256);
  const int cus = device_cus();
  const int grid = (int)(T < (long)cus ? T : (long)cus);
  return one ? launch_p8_t<true>(p, grid, st) : launch_p8_t<false>(p, grid, st);
}

hipError_t launch_p8n(const ConvParams& p, bool one, hipStream_t st) {
  if (p.cout > 1024 || p.cout % 8 || p.yoff % 8 || p.yc % 8 || (!one && p.cin % BKE)) return hipErrorInvalidValue;
  const long T = (long)((p.M + 255) / 256) * ((p.cout + 127) / 128);
  const int grid = (int)(T < (long)device_cus() ? T : (long)device_cus());
  return one ? launch_p8n_t<true>(p, grid, st) : launch_p8n_t<false>(p, grid, st);
}

// the N-split weight-stationary 1x1 ring (cout > BN: block b holds N tile (b / 8) % nN; three stages)
template <int BM, int BN, int WM, int WN, int KS>
hipError_t launch_pring_wsn(const ConvParams& p, hipStream_t st) {
  const int nN = (p.cout + BN - 1) / BN;
  if (nN < 2 || p.cout % 8 || p.yoff % 8 || p.yc % 8 || p.kpad > KS * 64 || p.k != 1 || p.s != 1 || p.pad)
    return hipErrorInvalidValue;
  const long T = (long)((p.M + BM - 1) / BM);
  long per = device_cus() / nN / 8 * 8;   // virtual blocks per N tile, a multiple of 8
  if (per > (T + 7) / 8 * 8) per = (T + 7) / 8 * 8;
  if (per < 8) per = 8;
  const int grid = (int)(per * nN);
  if (p.act == 1)
    YV7_LAUNCH((conv_f16_pring_kernel<BM, BN, WM, WN, 3, true, 1, 64, KS>), dim3(grid), dim3(64 * WM * WN), 0, st, p);
  else if (p.act == 2)
    YV7_LAUNCH((conv_f16_pring_kernel<BM, BN, WM, WN, 3, true, 2, 64, KS>), dim3(grid), dim3(64 * WM * WN), 0, st, p);
  else
    YV7_LAUNCH((conv_f16_pring_kernel<BM, BN, WM, WN, 3, true, 0, 64, KS>), dim3(grid), dim3(64 * WM * WN), 0, st, p);
  return hipGetLastError();
}

// the weight-stationary 1x1 ring (one N tile, whole K in LDS)
template <int BM, int BN, int WM, int WN, int KS>
hipError_t launch_pring_ws(const ConvParams& p, hipStream_t st) {
  if (p.cout > BN || p.cout % 8 || p.yoff % 8 || p.yc % 8 || p.kpad > KS * 64 || p.k != 1 || p.s != 1 || p.pad)
    return hipErrorInvalidValue;
  const long T = (long)((p.M + BM - 1) / BM);
  const int grid = (int)(T < (long)device_cus() ? T : (long)device_cus());
  if (p.act == 1)
    YV7_LAUNCH((conv_f16_pring_kernel<BM, BN, WM, WN, 2, true, 1, 64, KS>), dim3(grid), dim3(64 * WM * WN), 0, st, p);
  else if (p.act == 2)
    YV7_LAUNCH((conv_f16_pring_kernel<BM, BN, WM, WN, 2, true, 2, 64, KS>), dim3(grid), dim3(64 * WM * WN), 0, st, p);
  else
    YV7_LAUNCH((conv_f16_pring_kernel<BM, BN, WM, WN, 2, true, 0, 64, KS>), dim3(grid), dim3(64 * WM * WN), 0, st, p);
  return hipGetLastError();
}

// occ: resident blocks per CU the grid is sized for
template <int BM, int BN, int WM, int WN, int STAGES, int BK = 64>
hipError_t launch_pring(const ConvParams& p, bool one, int occ, hipStream_t st) {
  if (p.cout > 1024 || p.cout % 8 || p.yoff % 8 || p.yc % 8) return hipErrorInvalidValue;
  const long T = (long)((p.M + BM - 1) / BM) * ((p.cout + BN - 1) / BN);
  const int grid = (int)(T < (long)device_cus() * occ ? T : (long)device_cus() * occ);
  return one ? launch_pring_act<BM, BN, WM, WN, STAGES, true, BK>(p, grid, st)
             : launch_pring_act<BM, BN, WM, WN, STAGES, false, BK>(p, grid, st);
}

template <int BM, int BN, int WM, int WN, int STAGES, bool ONE, bool DET = false>
hipError_t launch_ring(const ConvParams& p, hipStream_t st) {
  const int nM = (p.M + BM - 1) / BM, nN = (p.cout + BN - 1) / BN;
  YV7_LAUNCH((conv_f16_ring_kernel<BM, BN, WM, WN, STAGES, ONE, DET>), dim3(nM * nN), dim3(64 * WM * WN), 0, st, p);
  return hipGetLastError();
}

template <int BM, int BN, int WM, int WN, int STAGES>
hipError_t launch_ring2(const ConvParams& p, bool one, hipStream_t st) {
  return one ? launch_ring<BM, BN, WM, WN, STAGES, true>(p, st) : launch_ring<BM, BN, WM, WN, STAGES, false>(p, st);
}

template <int BM, int BN, int WM, bool ONE, bool DET, int PF = 1, bool POOL = false>
hipError_t launch_t(const ConvParams& p, hipStream_t st) {
  const int nM = (p.M + BM - 1) / BM, nN = (p.cout + BN - 1) / BN;
  YV7_LAUNCH((conv_f16_kernel<BM, BN, WM, ONE, DET, PF, POOL>), dim3(nM * nN), dim3(NT), 0, st, p);
  return hipGetLastError();
}

}  // namespace

namespace {

// Ring-kernel configurations the split-K dispatch chooses from: tile BM x BN, waves, LDS stages.
// (Round 6: 128 x 128 / 128 x 64 rings with 5-6 stages, 3-4 in flight, one block per CU, were slower on
// every 20^2 / 40^2 deep-K 1x1 layer: 1024->512 @20 25.9 -> 31.7 us, profiles/r6_ring_deep/tune.txt.)
enum RingCfg { R256x256, R256x128, R128x128s3, R128x128s2, R128x64, R256x64, NCFG };
constexpr int cfg_bm[NCFG] = {256, 256, 128, 128, 128, 256};
constexpr int cfg_bn[NCFG] = {256, 128, 128, 128, 64, 64};

struct Choice {
  int cfg = -1;   // ring configuration, -1 = the legacy dispatch (halo / tile kernels / old variants)
  int S = 1;      // K splits
};


long ring_tiles(const ConvParams& p, int cfg) {
  return (long)((p.M + cfg_bm[cfg] - 1) / cfg_bm[cfg]) * ((p.cout + cfg_bn[cfg] - 1) / cfg_bn[cfg]);
}

// variant 100 + 10 * cfg + S forces ring configuration cfg with S K-splits (microbenchmarks).
Choice choose(const ConvParams& p, bool det) {
  Choice c;
  const int variant = p.variant ? p.variant : env_variant();
  if (det || p.cout <= 32) return c;
  const int nk = p.kpad / BKE;
  if (variant >= 100 && variant < 100 + 10 * NCFG) {
    c.cfg = (variant - 100) / 10;
    c.S = variant % 10 ? variant % 10 : 1;
  } else if (variant == 0 && !halo_supported(p) && !ws64_supported(p)) {
    // Low-resolution layers (scripts/convbench.hip, bs 32, us): with at most 400 tiles of 128 x 128
    // (and for short-K 1x1 layers up to 3200) the 2-stage 128 x 128 ring (2 blocks per CU) beats the
    // wide tiles and the register-staged tile kernel (3x3 256->128 @40 50 -> 44, s2 512->512 @40
    // 88 -> 82, 1x1 256->256 @80 70 -> 61, 2048->512 @20 40 -> 37); the narrowest 1x1 take 128 x 64
    // (512->256 @20 11.7 -> 10.5); deep-K 3x3 layers under one round of tiles split K in two
    // (256->256 @20 35 -> 30, 512->256 @20 65 -> 47, s2 256->256 @40 36 -> 30; sc1 hand-off,
    // splitk_reduce), in four when a round of tiles covers at most half the CUs.  Wider grids keep the tuned wide tiles below.
    const long t128 = ring_tiles(p, R128x128s2);
    if (p.k > 1) {
      if (t128 <= 400) c.cfg = R128x128s2;
      if (t128 <= 256 && nk >= 36) c.S = 2;
      static const long s4max = [] { const char* e = getenv("YV7_SPLIT4_TILES"); return e ? atol(e) : 128L; }();
      // yolov7-w6 bs 8, 512->512 @20: 100 tiles x 4 K parts (72 -> 35 us); at 200 tiles (yolov7 bs 32,
      // 256->256 @20) four parts lose to two: 33 -> 46 us (YV7_SPLIT4_TILES=256 A/B)
      if (t128 <= s4max && nk >= 36) c.S = 4;
    } else {
      if (t128 <= 400 || (p.K <= 256 && t128 <= 3200)) c.cfg = R128x128s2;
      // 128 x 64 tiles under 200 tiles of 128 x 128, K split in two for K >= 2048 at <= 200 of them
      // (yolov7-w6 1280 bs 8 @20, profiles/r4_w6stem/tune_w6_dispatch.txt, us: 1024->1024 21.0 -> 15.4,
      // 2048->1024 33.0 -> 25.2, 1024->512 18.9 -> 13.7, 2048->512 32.6 -> 18.4 split, 512->384 12.3 -> 9.5)
      if (t128 <= 200) c.cfg = R128x64;
      if (t128 <= 200 && p.K >= 2048 && ring_tiles(p, R128x64) <= 200) c.S = 2;
    }
  }
  if (c.S > nk) c.S = nk;
  if (c.cfg >= 0 && c.S > 1 &&
      (double)ring_tiles(p, c.cfg) * c.S * cfg_bm[c.cfg] * cfg_bn[c.cfg] * 4 >= 2147483648.0)
    c.S = 1;   // partial tiles are addressed with 32-bit buffer offsets
  return c;
}

template <int BM, int BN, int WM, int WN, int STAGES>
hipError_t launch_ring_s(const ConvParams& p0, bool one, int S, hipStream_t st) {
  ConvParams p = p0;
  p.ksplit = S;
  const long tiles = (long)((p.M + BM - 1) / BM) * ((p.cout + BN - 1) / BN);
  if (S > 1 && (!p.part || !p.cnt || p.part_bytes < (size_t)tiles * S * BM * BN * 4 || p.cnt_n < tiles))
    return hipErrorInvalidValue;   // the caller sized the scratch with conv_splitk_part_bytes
  const unsigned nblk = (unsigned)(tiles * S);
  if (one)
    YV7_LAUNCH((conv_f16_ring_kernel<BM, BN, WM, WN, STAGES, true>), dim3(nblk), dim3(64 * WM * WN), 0, st, p);
  else
    YV7_LAUNCH((conv_f16_ring_kernel<BM, BN, WM, WN, STAGES, false>), dim3(nblk), dim3(64 * WM * WN), 0, st, p);
  return hipGetLastError();
}

hipError_t launch_choice(const ConvParams& p, const Choice& c, bool one, hipStream_t st) {
  switch (c.cfg) {
    case R256x256: return launch_ring_s<256, 256, 2, 4, 2>(p, one, c.S, st);
    case R256x128: return launch_ring_s<256, 128, 4, 2, 3>(p, one, c.S, st);
    case R128x128s3: return launch_ring_s<128, 128, 2, 2, 3>(p, one, c.S, st);
    case R128x128s2: return launch_ring_s<128, 128, 2, 2, 2>(p, one, c.S, st);
    case R128x64: return launch_ring_s<128, 64, 2, 2, 3>(p, one, c.S, st);
    case R256x64: return launch_ring_s<256, 64, 4, 2, 3>(p, one, c.S, st);
  }
  return hipErrorInvalidValue;
}

}  // namespace

size_t conv_splitk_part_bytes(const ConvParams& p) {
  const Choice c = choose(p, false);   // (choose() keeps this under 2 GiB)
  if (c.cfg < 0 || c.S <= 1) return 0;
  return (size_t)ring_tiles(p, c.cfg) * c.S * cfg_bm[c.cfg] * cfg_bn[c.cfg] * 4;
}

int conv_splitk_tiles(const ConvParams& p) {
  const Choice c = choose(p, false);
  return (c.cfg < 0 || c.S <= 1) ? 0 : (int)ring_tiles(p, c.cfg);
}

int lr_default_cfg(const ConvParams& p) {
  static const int lr = [] { const char* e = getenv("YV7_LR"); return e ? atoi(e) : 1; }();
  if (lr && !p.pool && (long)p.M <= 204800 && p.k == 3 && p.s == 1 &&
      !((long)p.B * (p.H / 16) * (p.W / 16) >= 800 && ws64_supported(p))) {
    const bool t5 = p.H % 5 == 0;
    const long t128 = (long)((p.B + 3) / 4) * (p.H / (t5 ? 5 : 4)) * (p.W / 4) * (p.cout / 128);
    int cfg = (p.cout % 128 == 0 && t128 >= 400 ? 0 : 1) + (t5 ? 0 : 2);
    // 160-pixel tiles (10 rows: each weight fragment feeds twice the MFMAs) where they keep >= 400 / 640
    // blocks (profiles/r4lr/tune_tm10*.txt, us): 160 x 128 for the channel-doubling RepConvs up to 384
    // inputs (yolov7 128->256 @80 115.5 -> 111.9, 256->512 @40 105.9 -> 100.2; w6 256->512 @80 104.2 ->
    // 95.9, 384->768 @40 62.2 -> 56.7), 160 x 64 for the other wide / 64-channel layers (512->512 @20
    // 61.9 -> 57.4, 512->1024 @20 103.8 -> 99.3, 128->64 @80 40.5 -> 37.7, 256->256 @40 56.3 -> 54.9)
    if (p.H % 10 == 0) {
      const long g10 = (long)((p.B + 3) / 4) * (p.H / 10) * (p.W / 4);
      if (p.cout % 128 == 0 && p.cout >= 2 * p.cin && p.cin <= 384 && g10 * (p.cout / 128) >= 400) cfg = 5;
      // (round 6: the 128-output exclusion kept only for 128-input layers — 256->128 took 160 x 64 by 1-2 us in
      // every sweep: yolov7 @40 ops 49 / 66, w6 @80 ops 57 / 73, profiles/r6_tune/tune_{yolov7,w6}_all.txt)
      else if ((p.cout != 128 || p.cin >= 256) && p.cout % 64 == 0 && g10 * (p.cout / 64) >= 480) cfg = 6;
    }
    // Round 5 (profiles/r5_misc/tune_small_w6.txt, us): 160 x 64 from 480 such tiles (w6 bs 8 384->384 @40
    // 38.0 / 37.9 / 37.1 / 37.3 -> 35.6-35.9); 64-pixel tiles on the 3 200-pixel layers (w6 bs 8 @20:
    // 512->512 25.3 / 25.0 / 25.2 -> 23.7-24.1, 512->256 18.4 -> 17.1, 256->256 11.3 -> 10.4)
    // (round 6, profiles/r6_tune/tune_w6_all.txt: not for cout 1024 — w6 bs 8 512->1024 @20 42.2 -> 36.9 us on
    // the 128-pixel tiles)
    if (cfg == 1 && p.M <= 6400 && p.cout <= 512 && lr_supported(p, 3)) cfg = 3;
    if (lr_supported(p, cfg)) return cfg;
  }
  return -1;
}

hipError_t launch_conv_f16(const ConvParams& p, bool det, hipStream_t st) {
  const bool one = p.k == 1 && p.s == 1 && p.pad == 0;
  const int variant = p.variant ? p.variant : env_variant();
  if (p.pool) {   // MP folded into a 1x1 conv: register-staged tile kernel (the max needs the operands in VGPRs)
    if (p.pool != 2 || p.k != 1 || p.s != 2 || p.pad != 0 || det || p.cin % 64) return hipErrorInvalidValue;
    // in-network A/B over the five yolov7 MP+1x1 pairs (us, 128x128 / 64x128): 256->128 @160 111 / 104,
    // 512->256 @80 71 / 68, 256->256 @40 16.9 / 15.1 (1024->512 @40 folds no more: 52 vs 46.5 unfused)
    static const int pcfg = [] { const char* e = getenv("YV7_POOL_CFG"); return e ? atoi(e) : 0; }();
    if (p.cout <= 64) return launch_t<128, 64, 2, false, false, 1, true>(p, st);
    if (pcfg == 1) return launch_t<128, 128, 2, false, false, 1, true>(p, st);
    return launch_t<64, 128, 1, false, false, 1, true>(p, st);
  }
  // the column-group 3x3 halo ring (conv_hring.hip, variant 262; 911-914: its microbenchmark hooks),
  // forced only where every N tile is full: the masked last tile of a cout that 128 does not divide has
  // no layer in the checked networks
  if (!det && (variant == 262 || (variant >= 911 && variant <= 914)) && hring_supported(p) && p.cout % 128 == 0)
    return launch_conv_hring(p, device_cus(), st);
  // the low-resolution 3x3 kernel (conv_lr.hip): 270 + tile configuration
  if (!det && variant >= 270 && variant <= 279 && lr_supported(p, variant - 270)) return launch_conv_lr(p, variant - 270, st);
  // the register-weight stride-2 kernel (conv_s2.hip): 280 + tile configuration
  if (!det && variant >= 280 && variant <= 288 && s2_supported(p, variant - 280))
    return launch_conv_s2(p, variant - 280, device_cus(), st);
  // the register-weight 1x1 kernel (conv_w1.hip): 290 + configuration
  if (!det && variant >= 290 && variant <= 295 && w1_supported(p, variant - 290))
    return launch_conv_w1(p, variant - 290, device_cus(), st);
  if (!det && variant >= 302 && variant <= 303 && w1_supported(p, variant - 296))   // its rows 6-7
    return launch_conv_w1(p, variant - 296, device_cus(), st);
  if (!det && variant >= 299 && variant <= 301 && w1_supported(p, 1)) return launch_conv_w1(p, 1, device_cus(), st);   // its hooks
  // The register-weight 3x3 kernel (conv_s2.hip) at stride 1, checked before the low-resolution rule
  // below (which would take the 204 800-pixel layers).  In-network, one layer forced at a time
  // (profiles/r5_s2/tune_s1_*.txt, us, dispatch -> s2 S=1): yolov7 bs 32 64->64 @320 228.2 -> 222.9
  // (cfg 6), 128->128 @80 65.6 -> 62.2 / 65.0 -> 63.0 (cfg 7), 128->256 @80 116.2 -> 108.2 (cfg 8);
  // yolov7-w6 bs 8 128->128 @160 68.4 -> 61.4, 128->256 @160 116.2 -> 106.5.  64->64 below 1 M pixels
  // and the 64-output 128-input layers (57.1 vs 38.3) keep the dispatch below.  YV7_S1=0: off.
  static const int s1k = [] { const char* e = getenv("YV7_S1"); return e ? atoi(e) : 1; }();
  if (!det && variant == 0 && s1k && p.k == 3 && p.s == 1 && !p.pool && (long)p.M >= 204800) {
    int cfg = -1;
    if (p.cin == 64 && p.cout == 64 && (long)p.M >= 1000000) cfg = 6;
    else if (p.cin == 128 && p.cout >= 128) cfg = p.cout >= 256 ? 8 : 7;
    if (cfg >= 0 && s2_supported(p, cfg)) return launch_conv_s2(p, cfg, device_cus(), st);
  }
  // 3x3 stride-1 layers of up to 204 800 output pixels (yolov7 640 bs 32 from 80^2 down, yolov7-w6 1280
  // bs 8 from 160^2 down): the low-resolution kernel (conv_lr.hip) — one layer forced at a time in the bs-32
  // forward (profiles/r4lr/tune3.txt, us, dispatch -> lr): 3x3 256->256 @20 32.2 -> 22.1, 512->512 @20
  // 80.8 -> 62.7, 512->256 @20 48.8 -> 37.0, 512->1024 @20 119.8 -> 107.5, 128->128 @40 24.5 -> 21.9,
  // 256->128 @40 43.5 -> 35.6, 256->256 @40 69.9 -> 59.5, 256->512 @40 129.8 -> 108.5, 128->128 @80
  // 74.3 -> 63.4, 128->256 @80 123.9 -> 119.5, 128->64 @80 50.2 -> 40.8, 64->64 @80 31.6 -> 27.4.
  // 80 x 128 tiles when there are >= 400 of them, else 80 x 64 (64-pixel tiles when 5 does not divide
  // the height); w6 1280 bs 8 (profiles/r4lr/tune_w6.txt): 384->384 @40 38.7 -> 36.3 and 384->768 @40
  // 73.0 -> 66.0 with 80 x 128 (480 / 960 tiles); yolov7's 512->512 @20 and 128->128 / 256->128 @40
  // (640) are equal either way.  YV7_LR=0: off.
  static const int lr = [] { const char* e = getenv("YV7_LR"); return e ? atoi(e) : 1; }();
  if (!det && variant == 0) {
    const int cfg = lr_default_cfg(p);
    if (cfg >= 0) return launch_conv_lr(p, cfg, st);
  }
  // 3x3 stride-2 layers with 64 / 128 input channels and at least 204 800 output pixels: the register-weight
  // stride-2 kernel (conv_s2.hip).  In-network, one layer forced at a time (scripts/tune_ops.py,
  // profiles/r5_s2/tune_*.txt, us, dispatch -> s2): yolov7 bs 32 64->128 s2 @320 186.1 -> 130.4 (cfg 0),
  // 128->128 s2 @160 102.2 -> 74.0 (cfg 3); yolov7-w6 bs 8 128->256 s2 @320 159.2 -> 123.6 (cfg 4).  The
  // 51 200-pixel layers (128->128 s2 @80, w6 128->256 s2 @160) are equal either way and keep the
  // dispatch below.  YV7_S2=0: off.
  static const int s2k = [] { const char* e = getenv("YV7_S2"); return e ? atoi(e) : 1; }();
  if (!det && variant == 0 && s2k && p.k == 3 && p.s == 2 && (long)p.M >= 204800 && (p.cin == 64 || p.cin == 128)) {
    const int cfg = p.cin == 64 ? 0 : (p.cout >= 256 ? 4 : 3);
    if (s2_supported(p, cfg)) return launch_conv_s2(p, cfg, device_cus(), st);
  }
  // 1x1 stride-1 layers with 128 / 256 / 512 inputs: the register-weight 1x1 kernel (conv_w1.hip).  In-
  // network, one layer forced at a time (scripts/tune_ops.py, profiles/r5_w1/tune_*.txt, us, dispatch ->
  // w1): yolov7 bs 32 128->128 @160 87.5 -> 75.2 (cfg 0), 256->256 @160 187.5 -> 163.5, @80 58.3 -> 49.1
  // (cfg 3), 512->512 @80 147.5 -> 119.9, @40 47.6 -> 39.6 (cfg 5), 512->384 @80 131.1 -> 113.1 (cfg 2);
  // yolov7-w6 bs 8 128->128 @320 91.3 -> 73.3, 512->256 @160 90.7 -> 65.5; 256->128 with a 128-channel
  // N slice (cfg 7; profiles/r5_misc/tune_small_w6.txt) @320 139.9 -> 123.6, @160 43.7 -> 34.1.  Narrower
  // grids keep the rings below.  YV7_W1=0: off.
  static const int w1k = [] { const char* e = getenv("YV7_W1"); return e ? atoi(e) : 1; }();
  if (!det && variant == 0 && w1k && one && !p.pool) {
    int cfg = -1;
    if (p.cin == 128 && p.M >= 409600) cfg = 0;
    else if (p.cin == 256 && p.M >= 204800) cfg = p.cout == 128 ? 7 : 3;
    else if (p.cin == 512 && p.M >= 51200) cfg = p.cout % 256 == 0 ? 5 : (p.M >= 204800 ? 2 : -1);
    if (cfg >= 0 && w1_supported(p, cfg)) return launch_conv_w1(p, cfg, device_cus(), st);
  }
  // 3x3 stride-2 layers the 128 x 128 ring would split K for (under 256 of its tiles: yolov7's 256->256
  // s2 @40, w6's 768->1024 s2 @40): the stride-2 low-resolution form (profiles/r4lr/convbench_s2.txt:
  // 256->256 s2 @40 29.6 -> 25.4 us)
  // and the stride-2 layers of at most 12 800 output pixels but those with a round of 256 x 128 tiles
  // and cout >= 512, which the 8-phase ring below serves better (profiles/r4_w6stem/tune_*.txt, us:
  // w6 bs 8 512->768 s2 @80 134.6 -> 107.6, 256->384 s2 @80 39.5 -> 35.7; yolov7 bs 32 512->512 s2 @40
  // p8n 76.8 vs 90.5 here)
  const long t2n_s2 = (long)((p.M + 255) / 256) * ((p.cout + 127) / 128);
  // Round 5: the 80-pixel stride-2 tile (cfg 7, 5 output rows) on the 12 800-pixel layers with cout >= 384
  // (one layer forced at a time, profiles/r5_s2/tune_deep_w6.txt, us, cfg 4 -> 7: yolov7-w6 bs 8 512->768
  // s2 @80 109.1 -> 101.5, 256->384 s2 @80 37.7 -> 31.3; yolov7 bs 32 256->256 s2 @40 keeps cfg 4: 27.0
  // vs 28.8)
  if (!det && variant == 0 && lr && p.k == 3 && p.s == 2 &&
      ((long)((p.M + 127) / 128) * ((p.cout + 127) / 128) <= 256 ||
       (p.M <= 12800 && !(t2n_s2 >= 150 && t2n_s2 <= 250 && p.cout >= 512)))) {
    const int cfg = (p.M >= 12800 && p.cout >= 384 && lr_supported(p, 7)) ? 7 : 4;
    if (lr_supported(p, cfg)) return launch_conv_lr(p, cfg, st);
  }
  // 3x3 stride-1 layers with 128-channel output tiles and at least one round of 16 x 16 x 128 tiles: the
  // column-group halo ring (conv_hring.hip, variant 262).  Single-layer sweep, bs 32 640, same box
  // (profiles/r3_hring2_tune.txt, us, dispatch -> 262): 3x3 128->128 @80 80.0 / 80.4 / 82.7 / 81.0 ->
  // 67.2 / 67.9 / 69.3 / 68.4, 128->256 @80 139.1 -> 121.4.  YV7_HRING=0: off.
  static const int hring = [] { const char* e = getenv("YV7_HRING"); return e ? atoi(e) : 1; }();
  if (!det && variant == 0 && hring && hring_supported(p) && p.cout % 128 == 0 &&
      (long)p.B * (p.Ho / 16) * (p.Wo / 16) * (p.cout / 128) >= device_cus())
    return launch_conv_hring(p, device_cus(), st);
  if (!det && variant == 0 && p.cout > 32 && p.cout <= 1024 && p.cout % 8 == 0) {
    // Persistent ring (scripts/convbench.hip, bs 32, same box, us): short-K 1x1 layers and the
    // 128-channel / low-resolution 512-channel 3x3 layers, whose per-tile fill + epilogue the
    // non-persistent kernels cannot hide.  256 x 256 tiles once every CU gets >= 6 of them
    // (1x1 256->256 @160 304 -> 226, 512->512 @80 208 -> 183), else 128 x 128 with two blocks per
    // CU (1x1 128->128 @160 110 -> 89, 256->128 @160 161 -> 131, 256->256 @80 61 -> 55, 3x3
    // 128->128 @80 86 -> 81, s2 128->128 @160 96 -> 90, 512->512 @20 80 -> 76).
    const long t256 = (long)((p.M + 255) / 256) * ((p.cout + 255) / 256);
    // Wide layers with at least 200 tiles of 256 x 256 (in-network sweep of every ring configuration,
    // yolov7 bs 32, us, default -> persistent 256 x 256): 1x1 1024->1024 @40 156 -> 135, 1024->512 @40
    // 79 -> 69, 512->512 @40 55 -> 48, 1024->1024 @20 44 -> 39; 3x3 256->256 @40 86 -> 70, s2 256->256
    // @80 90 -> 77, 256->512 @40 157 -> 134, 512->1024 @20 146 -> 128.  Under 200 tiles (@20 with
    // cout <= 512) the persistent 256 x 256 ring loses (2048->512 @20 41 -> 59).  YV7_WIDE_PRING=0: off.
    static const int wide = [] { const char* e = getenv("YV7_WIDE_PRING"); return e ? atoi(e) : 1; }();
    // The 8-phase ring (conv_f16_p8_kernel) where it measured faster in-network (scripts/tune_ops.py,
    // one layer forced at a time, bs 32, us, dispatch before -> p8): 3x3 256->256 @40 76 -> 67, s2
    // 256->256 @80 79 -> 72, 256->512 @40 137 -> 126, 512->1024 @20 130 -> 114; 1x1 with K >= 1024:
    // 1024->1024 @40 142 -> 138, 1024->512 @40 74 -> 70, 1024->256 @40 41 -> 39.  Short-K 1x1 and
    // 128-input 3x3 layers stay on the 2-phase ring (1x1 256->256 @160 199 -> 216, 3x3 128->256 @80
    // 137 -> 144).  YV7_P8=0: off.

    // Weight-stationary 1x1 (K <= 256, 128 < cout <= 256, >= 80x80 at bs 32; tune_ops, us): 256->256
    // @160 213 -> 201, @80 70 -> 66 / 66 -> 65; narrower or lower-resolution 1x1 layers lose.
    // YV7_WS1=0: off.
    static const int ws1 = [] { const char* e = getenv("YV7_WS1"); return e ? atoi(e) : 1; }();
    // Round 3: its N-split form (two blocks per 256-pixel tile, each holding one 128-channel half of the
    // weights, three activation stages in flight instead of two; tune_ops, us: 256->256 @160 197.6 ->
    // 188.9, @80 60.3 -> 59.8 and 62.1 -> 58.6, profiles/r3w_tune.txt).
    if (ws1 && one && p.kpad <= 256 && p.cout > 128 && p.cout <= 256 && p.M >= 204800)
      return launch_pring_wsn<256, 128, 4, 2, 4>(p, st);
    // 3x3 stride-2 layers with about one round of 256 x 128 tiles: the 8-phase ring on 256 x 128 tiles
    // (all-layer sweep, profiles/r3y_tune.txt, us: 512->512 s2 @40 81.9 -> 75.5, 128->128 s2 @80
    // 29.6 -> 26.5)
    if (p.k == 3 && p.s == 2 && p.cin >= 128 && p.cin % BKE == 0 && p.cout % 128 == 0 && p.cout <= 1024) {
      const long t2n = (long)((p.M + 255) / 256) * (p.cout / 128);
      if (t2n >= 150 && t2n <= 250) return launch_p8n(p, false, st);
    }
    if (p8_default(p)) return launch_p8(p, one, st);
    if (one) {
      // (a cout that is not a multiple of 256 — the tensor-fused pair 512->256+128 @80 — would leave
      // half of every last 256-wide N tile idle: the 128 x 128 ring below, 148.8 -> 124.2 us in-network,
      // profiles/r3r/tune.txt)
      const bool n256 = p.cout % 256 == 0 || p.K > 512;
      if (n256 && p.K >= 256 && p.cout >= 256 && t256 >= 1600) return launch_pring<256, 256, 2, 4, 2>(p, one, 1, st);
      if (n256 && wide && p.cout >= 256 && t256 >= 200) return launch_pring<256, 256, 2, 4, 2>(p, one, 1, st);
      if (p.K <= 512 && p.M >= 51200)
        return launch_pring<128, 128, 2, 2, 2>(p, one, 2, st);
    } else if (wide && p.k == 3 && p.cin >= 256 && p.cout >= 256 && t256 >= 200) {
      return launch_pring<256, 256, 2, 4, 2>(p, one, 1, st);
    } else if (p.k == 3 && p.cout == 128) {
      // (3x3 512->512 @20 and s2 from @40 take the non-persistent 128 x 128 ring of choose() below:
      // in-network 92 (this ring) / 89 (256 x 128 persistent) -> 79 us; with fewer tiles than CUs,
      // yolov7-w6 at bs 8, it splits K: 72 -> 35 us)
      return launch_pring<128, 128, 2, 2, 2>(p, one, 2, st);
    }
  }
  const Choice ch = choose(p, det);
  if (ch.cfg >= 0) return launch_choice(p, ch, one, st);
  if (!det && p.cout > 32) {
    // persistent ring configurations (microbenchmarks: 201..206)
    if (variant == 201) return launch_pring<256, 256, 2, 4, 2>(p, one, 1, st);
    if (variant == 296) return launch_pring_hook<296>(p, one, st);
    if (variant == 297) return launch_pring_hook<297>(p, one, st);
    if (variant == 298) return launch_pring_hook<298>(p, one, st);
    if (variant == 202) return launch_pring<256, 128, 4, 2, 3>(p, one, 1, st);
    if (variant == 203) return launch_pring<128, 128, 2, 2, 3>(p, one, 1, st);
    if (variant == 204) return launch_pring<128, 128, 2, 2, 2>(p, one, 2, st);
    if (variant == 205) return launch_pring<256, 128, 4, 2, 2>(p, one, 1, st);
    if (variant == 206) return launch_pring<128, 256, 2, 4, 2>(p, one, 1, st);
    // 8-phase persistent ring (conv_f16_p8_kernel).  Round 4 removed the forced-only forms DESIGN §8
    // records as slower (BK-32 and 3-per-CU rings 211-218, pipelined rings 221-223, the p8 schedules
    // 233 / 237, the 512 x 128 p8 238, the first halo rings 260 / 261, the stand-alone 240).
    if (variant == 231 && (one || p.cin % BKE == 0)) return launch_p8(p, one, st);
    // weight-stationary 1x1 rings (conv_f16_pring_kernel, WS): 234 = 128 x 256 tiles (K <= 256),
    // 235 = 256 x 128 (K <= 256), 236 = 128 x 128 (K <= 512)
    if (variant == 234 && one && p.cout <= 256 && p.kpad <= 256) return launch_pring_ws<128, 256, 2, 4, 4>(p, st);
    if (variant == 235 && one && p.cout <= 128 && p.kpad <= 256) return launch_pring_ws<256, 128, 4, 2, 4>(p, st);
    if (variant == 236 && one && p.cout <= 128 && p.kpad <= 512) return launch_pring_ws<128, 128, 2, 4, 8>(p, st);
    // N-split weight-stationary 1x1 (K <= 256, 128 < cout <= 512): 256 x 128 tiles, three stages
    if (variant == 239 && one && p.cout > 128 && p.cout <= 512 && p.kpad <= 256) return launch_pring_wsn<256, 128, 4, 2, 4>(p, st);
    if (variant == 232 && (one || p.cin % BKE == 0)) return launch_p8n(p, one, st);
  }
  if (!det && p.cout > 32) {
    // 64 -> 64 3x3: the persistent weight-stationary kernel from 800 tiles of 16 x 16 (scripts/
    // convbench.hip, bs 32, same box: @320 423 -> 337 us, @160 95 -> 79 us vs the halo kernel).  Round 5:
    // its 8-wave form also takes the 800-tile layers from conv_lr (one layer forced at a time,
    // profiles/r5_misc/tune_small_*.txt, us: yolov7 bs 32 @80 27.3 / 26.2 / 26.8 -> 24.1 / 24.2 / 24.1,
    // yolov7-w6 bs 8 @160 25.7 / 26.3 / 25.7 -> 24.1 / 24.5 / 24.5); 12-16 are its microbenchmark hooks
    if (((variant == 0 && (long)p.B * (p.H / 16) * (p.W / 16) >= 800) || (variant >= 11 && variant <= 19)) &&
        ws64_supported(p))
      return launch_conv_ws64(p, st);
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
  if (det) {
    // Detect head: the persistent head (conv_det_pring_kernel) where it applies; 98 = its
    // microbenchmark hook (no staging), 99 = the 64 x 256 ring below (the round-2 default)
    static const int det_pring = [] { const char* e = getenv("YV7_DET_PRING"); return e ? atoi(e) : 1; }();
    if (((variant == 0 && det_pring) || variant == 94 || variant == 98 || variant == 96 || variant == 95 ||
         variant == 93 || variant == 91) && det_pring_supported(p))
      return launch_det_pring(p, device_cus(), st);
    // BN = 256 covers the na*no = 255 channels of a pixel
    // (scripts/detbench.hip, bs 32, row scores on: 64 x 256 ring, 2 blocks per CU so one block's
    // epilogue runs beside the other's main loop: 124 / 42 / 25 us at 80 / 40 / 20; 128 x 256 ring
    // 127 / 42 / 29; register-staged 64 x 256 tile 141 / 47 / 30)
    if (variant == 92) return launch_t<64, 256, 1, true, true>(p, st);
    if (variant == 97) return launch_ring<128, 256, 2, 4, 3, true, true>(p, st);
    return launch_ring<64, 256, 1, 4, 2, true, true>(p, st);
  }
  if (variant == 2) {  // tall tiles for narrow layers
    if (p.cout <= 32) return one ? launch_t<256, 32, 4, true, false>(p, st) : launch_t<256, 32, 4, false, false>(p, st);
    if (p.cout <= 64) return one ? launch_t<256, 64, 4, true, false>(p, st) : launch_t<256, 64, 4, false, false>(p, st);
  }
  if (p.cout <= 32) return one ? launch_t<128, 32, 4, true, false>(p, st) : launch_t<128, 32, 4, false, false>(p, st);
  if (p.cout <= 64) return one ? launch_t<128, 64, 2, true, false>(p, st) : launch_t<128, 64, 2, false, false>(p, st);
  return one ? launch_t<128, 128, 2, true, false>(p, st) : launch_t<128, 128, 2, false, false>(p, st);
}

}  // namespace yv7
