// 3x3 / stride-2 / pad-1 fp16 convolution with the layer's WEIGHTS RESIDENT IN VGPRs — the stride-2
// entries of the ELAN stages whose K = 9 * cin fits the register file: Conv(c1, c2, 3, 2) in
// Conv.fuseforward (models/common.py:110-111) at cfg/deploy/yolov7.yaml:20 (64->128 @320), the MP
// blocks' stride-2 convs (yolov7.yaml:33 128->128 @160, :108 128->128 @80 in the head) and
// yolov7-w6.yaml's 128-input stride-2 convs (:29 P3 entry 128->256 @320, and its head's).
// y = act(conv2d(x, W', b', s=2, pad=1)).  The same kernel with S = 1 (configurations 5-8) serves the
// large 64- and 128-input stride-1 3x3 layers (yolov7.yaml:19 64->64 @320, the ELAN 3x3 128->128 @80 and
// the head's RepConv 128->256 @80; the dispatch rule in conv_f16.hip launch_conv_f16).
//
// Why: the stride-2 layers were the furthest below their roofline (yolov7: 517 us
// against a 174 us roof; 64->128 s2 @320 alone 190 us against 79).  Their implicit-GEMM rings stage one
// tap's A tile per K step (each input pixel crosses L2 -> LDS ~2.25 times, counter bytes 1.38-2.06x the
// algorithmic ones) and conv_lr.hip's stride-2 form streams a 128-channel weight slice into VGPRs for
// every 64-pixel tile (256 B of L2 reads per MFMA).  Here:
//  * a block holds its N slice's whole weight matrix in VGPRs for the whole (persistent) launch: wave
//    (ng, pg) keeps TN x 9 x NCH fragments (16 channels x 32 K each, 4 VGPRs) — 144 VGPRs for
//    cin = 64 / TN = 2 and cin = 128 / TN = 1 — loaded ONCE from the fragment-packed copy (pack_frag);
//  * pixels stream: per 64-channel chunk (one full 128-byte line of every input pixel: a DMA piece is 8
//    whole lines) a tile's input patch is DMA'd (buffer_load ... lds) into an NS-slot LDS ring once, and
//    every LDS read of a pixel fragment feeds up to 3 x TN MFMAs: the MFMA's 16
//    pixels are 4 IMAGES x 4 COLUMNS of one output row (conv_lr.hip's fragment), a wave owns TM output
//    rows of one 4-column group and reads the 2 TM + 1 patch rows of a tap column once — output row i
//    takes patch rows 2i, 2i + 1, 2i + 2 for taps r = 0, 1, 2, so input rows 2y + 1 are shared by output
//    rows y and y + 1 (the halo-ring column-group reuse at stride 2);
//  * the patch keeps even input columns first (slot c / 2) and odd ones after (4 PG + 1 + c / 2), so the
//    four columns 2x + s a tap reads are four consecutive slots; a pixel's 128 bytes are 8 16-byte
//    positions, K-step half h's part g at position (4 h + g) ^ 2 (slot & 3) — conflict-free ds_read_b128
//    for every row, slot offset and half (checked exhaustively against the gfx950 lane groups,
//    scripts/s2_swizzle_check.py); the swizzle is applied on the DMA's per-lane SOURCE address, the LDS
//    image is lane-linear.  (The first form fetched 64-byte half lines per 32-channel chunk: the DMA path,
//    not the MFMAs, bound it — 166 us on 64->128 @320, 62 us with the DMA hooked out.)
//  * 8 waves (two per SIMD); one barrier per chunk; the DMA of chunk k + L is issued in the interval after
//    barrier k into the slot the chunks before it left, and every wave waits only for its own pieces of
//    the chunk the next interval reads (counted vmcnt: the pieces per wave and the epilogue stores per
//    tile are compile-time constants; pieces past the patch go to the slot's padding).  STG = 1: two
//    stagger groups one barrier apart (waves 4-7 behind; a SIMD hosts waves w and w + 4), so a group's
//    tile epilogue issues beside the other group's MFMAs, at the cost of one ring slot (L = NS - 2; STG =
//    0: L = NS - 1).
#include "yv7_kernels.h"

namespace yv7 {

namespace {

constexpr int FI = 4, FC = 4;   // MFMA pixel fragment: 4 images x 4 columns
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

// position swizzle of a pixel's eight 16-byte parts (S = 2: by its column slot; S = 1, whose patch rows
// have an even pixel count, by image and slot — scripts/s2_swizzle_check.py, s1_swizzle_check.py)
template <int S>
__host__ __device__ constexpr int pswz(int img, int slot) {
  return S == 2 ? 2 * (slot & 3) : 2 * ((img >> 1) & 1) ^ 4 * ((slot >> 1) & 1);
}

// Compile-time geometry of one configuration.  NCH = cin / 32 (MFMA K steps per tap).
template <int NCH, int TN, int TM, int PG, int NG, int NS, int STG, int S>
struct S2Geo {
  static constexpr int NW = NG * PG;                       // waves
  static_assert(NW == 8, "eight waves");
  static_assert(NCH % 2 == 0, "whole 64-channel DMA chunks");
  static constexpr int NDC = NCH / 2;                      // DMA chunks per tile
  static_assert(S == 1 || S == 2, "stride");
  static constexpr int PR = S == 2 ? 2 * TM + 1 : TM + 2;  // patch rows
  static constexpr int NEV = 4 * PG + 1;                   // S = 2: even patch columns (slots 0 .. NEV - 1)
  static constexpr int PC = S == 2 ? 8 * PG + 1 : 4 * PG + 2;   // patch columns
  static constexpr int PPX = FI * PR * PC;                 // patch pixels
  static constexpr int NP = (PPX + 7) / 8;                 // 1 KiB DMA pieces (8 pixels x 128 B)
  static constexpr int PW = (NP + NW - 1) / NW;            // pieces per wave per chunk
  static constexpr int SB = NW * PW * 1024;                // bytes per ring slot (padded to whole pieces)
  static constexpr int LDS = NS * SB;
  static_assert(LDS <= 160 * 1024, "LDS budget");
  static constexpr int L = NS - 1 - STG;                   // DMA lead in chunks
  static_assert(L >= 1 && L <= 2, "lead");
  static constexpr int BN = NG * TN * 16;
  static_assert(TN * 9 * NCH <= 36, "144 weight VGPRs per wave at most");
  static constexpr int NST = TN % 2 == 0 ? TM * TN / 2 : TM * TN;   // epilogue stores per wave per tile
};

// WAVE ROLES: wave = pg * NG + ng (stagger group = wave >> 2).  Tile = 4 images x TM output rows x 4 PG
// columns; block = one BN-channel slice for the whole launch.
// HOOK (microbenchmark builds only — round 5 reached them as convbench variants 285-289; no longer mapped):
// 1 = no DMA waits in the loop, 2 = no DMA at all in the loop, 3 = no epilogue (results kept alive by a
// store under a condition that never holds), 4 = DMA, waits and barriers only (no MFMA, no epilogue).
template <int NCH, int TN, int TM, int PG, int NG, int NS, int STG, int S, int ACT, int HOOK = 0>
__global__ __launch_bounds__(512, 2) void conv3x3s2_rw_kernel(const ConvParams p, int nN) {
  using G = S2Geo<NCH, TN, TM, PG, NG, NS, STG, S>;
  __shared__ __attribute__((aligned(16))) unsigned char smem[G::LDS];

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int ng = wave % NG, pg = wave / NG, grp = STG ? (wave >> 2) : 0;
  const int g = lane >> 4, li = lane & 15;

  // block -> (N slice, virtual block of the pixel-tile walk): the nN blocks b, b + 8, ... of one XCD
  // hold the nN slices of the same walk position, so a tile's second slice reads its patch from L2
  const int b = blockIdx.x, Gd = gridDim.x;
  const int nt = (b / 8) % nN;
  const int vb = (b / (8 * nN)) * 8 + b % 8, vG = Gd / nN;
  const int ncg = p.Wo / (FC * PG), nrg = p.Ho / TM;
  const int T = ((p.B + FI - 1) / FI) * nrg * ncg;
  const TileWalk tw = xcd_tile_walk_g(T, vG, vb);
  const int ntl = tw.count();
  if (ntl == 0) return;   // (uniform over the block)
  const int n0 = nt * G::BN;

  const auto xr = make_rsrc(p.x, p.xbytes);
  const auto wr = make_rsrc(p.wf, p.wfbytes);
  const auto yr = make_rsrc(p.y, 0x7fffffffu);

  // ---- the wave's weights, resident for the launch: fragment (nf, K step c, tap) at ((nf * NCH + c) *
  // 9 + tap) KiB of the packed copy, lane-linear; channels past cout read zeros (past wfbytes)
  u4 wreg[TN][9 * NCH];
#pragma unroll
  for (int j = 0; j < TN; ++j) {
    const uint32_t base = (uint32_t)(((n0 / 16 + ng * TN + j) * NCH * 9) * 1024 + lane * 16);
#pragma unroll
    for (int f = 0; f < 9 * NCH; ++f)
      wreg[j][f] = __builtin_bit_cast(u4, __builtin_amdgcn_raw_buffer_load_b128(wr, base, (uint32_t)(f * 1024), 0));
  }
  f4 bias[TN];
#pragma unroll
  for (int j = 0; j < TN; ++j) {
    const int col = n0 + ng * TN * 16 + j * 16 + g * 4;
#pragma unroll
    for (int e = 0; e < 4; ++e) bias[j][e] = col + e < p.cout ? p.bias[col + e] : 0.0f;
  }

  // ---- DMA pieces of this wave: piece k = wave + 8 m; lane -> storage pixel 8 k + lane / 8 (image, row,
  // slot) and LDS position lane % 8, which holds the pixel's source part (lane % 8) ^ pswz(slot) of the
  // chunk's 128-byte line.  rel[m] = the lane's source offset relative to the tile's first patch pixel
  // (image b0, row 2 y0 - 1, column 2 x0 - 1); pieces past the patch read past every tensor (zeros into
  // the slot's padding).
  uint32_t rel[G::PW];
  const uint32_t rowb = (uint32_t)(p.W + 2) * p.xc * 2, imgb = (uint32_t)(p.H + 2) * rowb;
#pragma unroll
  for (int m = 0; m < G::PW; ++m) {
    const int sp = (wave + 8 * m) * 8 + (lane >> 3);
    if (sp < G::PPX) {
      const int img = sp / (G::PR * G::PC), r2 = sp - img * (G::PR * G::PC);
      const int row = r2 / G::PC, slot = r2 - row * G::PC;
      const int pc = S == 1 ? slot : (slot < G::NEV ? 2 * slot : 2 * (slot - G::NEV) + 1);
      rel[m] = img * imgb + row * rowb + (uint32_t)((pc * p.xc + ((lane & 7) ^ pswz<S>(img, slot)) * 8) * 2);
    } else {
      rel[m] = OOB;
    }
  }
  const uint32_t xoffb = (uint32_t)p.xoff * 2;
  auto tile_base = [&](int it) -> uint32_t {   // byte offset of tile it's first patch pixel (+ xoff)
    int t = tw.at(it);
    const int cg = t % ncg;
    t /= ncg;
    const int y0 = (t % nrg) * TM, b0 = (t / nrg) * FI;
    return (uint32_t)(pix_index(b0, S * y0 - 1, S * cg * FC * PG - 1, p.H, p.W) * p.xc * 2) + xoffb;
  };
  // the wave's pieces m0 .. m1 - 1 of chunk q (flattened over the block's tiles) into ring slot q % NS;
  // chunks past the last tile read past the tensor (their slots are never read again)
  struct Src { uint32_t tb, so; unsigned char* dst; };
  auto src_of = [&](int q) __attribute__((always_inline)) {
    const int it = q / G::NDC, dc = q - it * G::NDC;
    const bool live = it < ntl;
    return Src{live ? tile_base(it) : OOB, (uint32_t)(dc * DC * 2), smem + (q % NS) * G::SB + wave * 1024};
  };
  auto issue_part = [&](const Src& sr, int m0, int m1) __attribute__((always_inline)) {
    if constexpr (HOOK == 2) return;
#pragma unroll
    for (int m = 0; m < G::PW; ++m)
      if (m >= m0 && m < m1) dma16(xr, sr.dst + m * 8 * 1024, sr.tb == OOB ? OOB : sr.tb + rel[m], sr.so);
  };
  auto issue = [&](int q) __attribute__((always_inline)) { issue_part(src_of(q), 0, G::PW); };

  // ---- per-lane LDS read offsets: image li / 4, column slot 4 pg + SOFF[s] + li % 4 of the fragment;
  // K-step half h's part g at position (4 h + g) ^ pswz(slot) (4 pg does not change slot & 3)
  constexpr int SOFF[3] = {0, S == 2 ? G::NEV : 1, S == 2 ? 1 : 2};   // slot of column S x + s relative to S x's
  const int img = li >> 2;
  uint32_t a_off[2][3];
#pragma unroll
  for (int h = 0; h < 2; ++h)
#pragma unroll
    for (int s = 0; s < 3; ++s) {
      const int slot = FC * pg + SOFF[s] + (li & 3);
      a_off[h][s] = (uint32_t)(((img * G::PR) * G::PC + slot) * 128 + (((4 * h + g) ^ pswz<S>(img, slot)) * 16));
    }

  f4 acc[TN][TM];
  // one DMA chunk = two K steps h; each: three column steps; step s reads the 2 TM + 1 patch rows at
  // the column slot once, output row i's tap (r, s) taking row 2 i + r
  // the DMA of chunk qn is issued in six parts, one before each column step (a burst of every piece at the
  // interval start stalled the waves' issue until the pieces drained: DMA and MFMAs ran one after the
  // other, 151 us = 71 us DMA alone + 56 us MFMAs alone + epilogue on 64->128 @320)
  auto compute = [&](int q, int dc, const Src& nx) __attribute__((always_inline)) {
    const unsigned char* pb = smem + (q % NS) * G::SB;
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int c = dc * 2 + h;
#pragma unroll
      for (int s = 0; s < 3; ++s) {
        const int t6 = h * 3 + s;
        issue_part(nx, t6 * G::PW / 6, (t6 + 1) * G::PW / 6);
        const unsigned char* ps = pb + a_off[h][s];
        u4 xa[G::PR];
#pragma unroll
        for (int r = 0; r < G::PR; ++r) xa[r] = *reinterpret_cast<const u4*>(ps + r * G::PC * 128);
#pragma unroll
        for (int i = 0; i < TM; ++i)
#pragma unroll
          for (int r = 0; r < 3; ++r)
#pragma unroll
            for (int j = 0; j < TN; ++j)
              acc[j][i] = __builtin_amdgcn_mfma_f32_16x16x32_f16(__builtin_bit_cast(h8, wreg[j][c * 9 + r * 3 + s]),
                                                                 __builtin_bit_cast(h8, xa[S * i + r]), acc[j][i], 0, 0, 0);
      }
    }
  };
  const uint32_t lane_ch = (uint32_t)(16 * (g & 1) + 8 * (g >> 1));
  auto epilogue = [&](int it) __attribute__((always_inline)) {
    int t = tw.at(it);
    const int cg = t % ncg;
    t /= ncg;
    const int y0 = (t % nrg) * TM, b0 = (t / nrg) * FI;
    const bool live = b0 + img < p.B;
    const int x = cg * FC * PG + FC * pg + (li & 3);
#pragma unroll
    for (int i = 0; i < TM; ++i) {
      const uint32_t yo = live ? (uint32_t)((pix_index(b0 + img, y0 + i, x, p.Ho, p.Wo) * p.yc + p.yoff) * 2) : OOB;
      typedef _Float16 h4 __attribute__((ext_vector_type(4)));
      typedef uint32_t u2 __attribute__((ext_vector_type(2)));
      if constexpr (TN % 2 == 0) {
#pragma unroll
        for (int mp = 0; mp < TN / 2; ++mp) {
          h4 va, vb;
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            va[e] = (_Float16)act_t<ACT>(acc[2 * mp][i][e]);
            vb[e] = (_Float16)act_t<ACT>(acc[2 * mp + 1][i][e]);
          }
          const u2 a = __builtin_bit_cast(u2, va), bb = __builtin_bit_cast(u2, vb);
          const auto s0 = __builtin_amdgcn_permlane16_swap(a[0], bb[0], false, false);
          const auto s1 = __builtin_amdgcn_permlane16_swap(a[1], bb[1], false, false);
          const u4 v = {s0[0], s1[0], s0[1], s1[1]};
          const int n = n0 + ng * TN * 16 + mp * 32 + (int)lane_ch;
          __builtin_amdgcn_raw_buffer_store_b128(v, yr, (live && n < p.cout) ? yo + (uint32_t)n * 2 : 0xffffffffu, 0, 0);
        }
      } else {
#pragma unroll
        for (int j = 0; j < TN; ++j) {
          h4 va;
#pragma unroll
          for (int e = 0; e < 4; ++e) va[e] = (_Float16)act_t<ACT>(acc[j][i][e]);
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

  // ---- prologue: chunks 0 .. L - 1 (every wave its pieces), chunk 0 landed before the first barrier
#pragma unroll
  for (int q = 0; q < G::L; ++q) issue(q);
  vmwait<G::PW * (G::L - 1)>();   // (the weight loads are older: retired too)
  barrier();
  if (STG && grp == 1) {   // the stagger: group 1 runs one interval behind, issuing chunk L in its idle interval
    issue(G::L);
    vmwait<G::PW * (G::L - 1)>();
    barrier();
  }

  // ---- steady state: interval = [issue chunk q + L (+1 for stagger group 1)][compute chunk q][epilogue
  // at a tile end][wait for this wave's pieces of the chunk the next interval reads][barrier]
  const int ahead = G::L + grp;
  for (int it = 0; it < ntl; ++it) {
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
      for (int i = 0; i < TM; ++i) acc[j][i] = bias[j];
#pragma unroll
    for (int dc = 0; dc < G::NDC; ++dc) {
      const int q = it * G::NDC + dc;
      const Src nx = src_of(q + ahead);
      if constexpr (HOOK != 4) compute(q, dc, nx);
      else issue_part(nx, 0, G::PW);
      if (dc == G::NDC - 1) {
        // the accumulators are final: keep the epilogue math out of the MFMA stream
#pragma unroll
        for (int j = 0; j < TN; ++j)
#pragma unroll
          for (int i = 0; i < TM; ++i) asm volatile("" : "+v"(acc[j][i]));
        if constexpr (HOOK == 3 || HOOK == 4) {
          if (p.cout < 0) epilogue(it);
        } else {
          epilogue(it);
        }
      }
      // younger than the pieces the next interval needs (issued L - 1 intervals ago): the L - 1 later
      // piece batches and the epilogue stores of intervals q - L + 1 .. q (a tile end among them: this
      // one, or for L = 2 the previous one — the previous tile's last chunk when dc == 0)
      // (hooks 3 / 4 issue no epilogue stores: NSTW = 0 there)
      constexpr int NSTW = (HOOK == 3 || HOOK == 4) ? 0 : G::NST;
      if constexpr (HOOK == 1 || HOOK == 2) {
      } else if constexpr (G::L == 1) {
        if (dc == G::NDC - 1) vmwait<NSTW>();
        else vmwait<0>();
      } else {
        if (dc == G::NDC - 1) vmwait<G::PW + NSTW>();
        else if (dc == 0 && it > 0) vmwait<G::PW + NSTW>();
        else vmwait<G::PW>();
      }
      barrier();
    }
  }
  if (STG && grp == 0) barrier();   // group 1's extra barrier
  vmwait<0>();                       // no DMA may land after the block's LDS is released
}

// tile configurations (variants 280 + row): {NCH, TN, TM, PG, NG, NS, STG, S}.  0-4: stride 2 (cin 64 /
// 128); 5-8: stride 1 (the same machinery for the 64 / 128-input 3x3 layers: cin 64 with 64 output
// channels = conv_ws.hip's layers, cin 128).
#define S2_CFGS(X)                                                                                             \
  X(0, 2, 2, 2, 2, 4, 3, 0, 2) X(1, 2, 2, 4, 2, 4, 2, 0, 2) X(2, 4, 1, 4, 1, 8, 3, 0, 2) X(3, 4, 1, 2, 1, 8, 4, 1, 2) \
  X(4, 4, 1, 8, 1, 8, 2, 0, 2) X(5, 2, 2, 2, 4, 2, 4, 1, 1) X(6, 2, 2, 4, 4, 2, 2, 0, 1) X(7, 4, 1, 4, 1, 8, 4, 1, 1) \
  X(8, 4, 1, 8, 1, 8, 4, 1, 1)
#define S2_ROW(i, nch, tn, tm, pg, ng, ns, stg, st) {nch, tn, tm, pg, ng, ns, stg, st},
constexpr int S2_CFG[][8] = {S2_CFGS(S2_ROW)};
constexpr int S2_NCFG = sizeof(S2_CFG) / sizeof(S2_CFG[0]);

template <int NCH, int TN, int TM, int PG, int NG, int NS, int STG, int S, int HOOK = 0>
hipError_t launch_cfg(const ConvParams& p, int cus, hipStream_t st) {
  using G = S2Geo<NCH, TN, TM, PG, NG, NS, STG, S>;
  const int nN = (p.cout + G::BN - 1) / G::BN;
  const long T = (long)((p.B + FI - 1) / FI) * (p.Ho / TM) * (p.Wo / (FC * PG));
  // persistent grid: a multiple of 8 * nN blocks (each XCD holds every N slice of its walk), at most one
  // block per CU, and no more virtual blocks than tiles (rounded to the XCD count)
  long per = cus / (8 * nN);
  const long need = (T + 7) / 8;
  if (per > need) per = need;
  if (per < 1) per = 1;
  const int grid = (int)(per * 8 * nN);
  if (HOOK) {
    YV7_LAUNCH((conv3x3s2_rw_kernel<NCH, TN, TM, PG, NG, NS, STG, S, 1, HOOK>), dim3(grid), dim3(512), 0, st, p, nN);
    return hipGetLastError();
  }
  if (p.act == 1)
    YV7_LAUNCH((conv3x3s2_rw_kernel<NCH, TN, TM, PG, NG, NS, STG, S, 1>), dim3(grid), dim3(512), 0, st, p, nN);
  else if (p.act == 2)
    YV7_LAUNCH((conv3x3s2_rw_kernel<NCH, TN, TM, PG, NG, NS, STG, S, 2>), dim3(grid), dim3(512), 0, st, p, nN);
  else
    YV7_LAUNCH((conv3x3s2_rw_kernel<NCH, TN, TM, PG, NG, NS, STG, S, 0>), dim3(grid), dim3(512), 0, st, p, nN);
  return hipGetLastError();
}

}  // namespace

// cfg: S2_CFG row (variants 280 + cfg)
bool s2_supported(const ConvParams& p, int cfg) {
  if (cfg < 0 || cfg >= S2_NCFG) return false;
  const int nch = S2_CFG[cfg][0], tm = S2_CFG[cfg][2], pg = S2_CFG[cfg][3], S = S2_CFG[cfg][7];
  const bool geom = S == 2 ? (p.H % 2 == 0 && p.W % 2 == 0 && p.Ho == p.H / 2 && p.Wo == p.W / 2)
                           : (p.Ho == p.H && p.Wo == p.W);
  return p.wf && p.k == 3 && p.s == S && p.pad == 1 && !p.pool && p.cin == nch * 32 && geom && p.Ho % tm == 0 &&
         p.Wo % (FC * pg) == 0 && p.cout % 16 == 0 && p.cout <= 1024 && p.xoff % 8 == 0 && p.xc % 8 == 0 &&
         p.yoff % 8 == 0 && p.yc % 8 == 0;
}

hipError_t launch_conv_s2(const ConvParams& p, int cfg, int cus, hipStream_t st) {
  if (!s2_supported(p, cfg)) return hipErrorInvalidValue;
  switch (cfg) {
#define S2_CASE(i, nch, tn, tm, pg, ng, ns, stg, st_) \
  case i: return launch_cfg<nch, tn, tm, pg, ng, ns, stg, st_>(p, cus, st);
    S2_CFGS(S2_CASE)
#undef S2_CASE
  }
  return hipErrorInvalidValue;
}

}  // namespace yv7
