// 3x3 / stride-1 / pad-1 fp16 convolution for the LOW-RESOLUTION layers (20x20 and 40x40 at 640, the
// w6 stages at 1280 / 16 and / 32): Conv.fuseforward (models/common.py:110-111) and RepConv's deploy
// conv (common.py:498-500) of the ELAN-H / SPPCSPC / head stacks (cfg/deploy/yolov7.yaml:65-68,
// 128-131; yolov7-w6.yaml's P5 / P6 stages): y = act(conv2d(x, W', b', s=1, pad=1)).
//
// Why a kernel of its own: at bs 32 these layers have 12 800 (20^2) or 51 200
// (40^2) output pixels, too few for the 16 x 16-pixel halo tiles of conv_hring.hip (which need 16 | H, W)
// and for one round of 128 x 128 implicit-GEMM tiles — the dispatch split K in two or four there, and the
// fp32 partials moved 3.5-4.5x the layer's algorithmic bytes (profiles/r4pmc/pmc_ops.txt).  Here:
//  * the MFMA's 16 pixels are 4 IMAGES x 4 COLUMNS of one output row (lane li: image li / 4, column
//    li % 4), so a tile is 4 images x TH rows x 4 columns — 4 divides 20, 40 and 80, and a bs-32 layer
//    still has 200-800 tiles;
//  * per 32-channel chunk the tile's input patch, 4 x (TH + 2) x 6 pixels with the zero frame
//    (yv7_kernels.h BORDER: no bounds tests), is staged in LDS ONCE and read by all nine taps: a wave
//    owning output rows i .. i + 3 reads patch rows i .. i + 5 at column s once and feeds them to taps
//    (0, s), (1, s), (2, s) (the column-group order of conv_hring.hip's variant 262);
//  * weights do not go through LDS at all: no two waves of a block share an output channel, so each
//    wave streams its own weight fragments straight into VGPRs from a FRAGMENT-PACKED copy made once at
//    plan creation (pack_frag: fragment (16 channels, chunk, tap) = 1 KiB contiguous in MFMA lane
//    order, one buffer_load_dwordx4 per fragment), PD column steps ahead of their use;
//  * one barrier per chunk (patch double buffer, register-staged), every load compiler-visible: the
//    chunk loop is unrolled at compile time (NCH = cin / 32 is a template parameter), so every wait is
//    an exact count in straight-line code — no hand-counted vmcnt;
//  * epilogue straight from the accumulators (bias in the accumulators, compile-time activation, fp16,
//    permlane16 pairing to 16-byte NHWC stores into the output channel slice: zero-copy concat).
// LDS patch rows are 64 bytes (32 fp16); the 16-byte chunk q of a pixel of image i sits in slot
// q ^ f(i), f = {0, 2, 3, 1}: each ds_read_b128 lane group (MI355X_MICROARCH.md §LDS) holds four
// (image, chunk) pairs with four different slots, each over four consecutive columns (four different
// 64-byte bank quads), so its 16 lanes hit 16 distinct bank positions for every row and column offset.
#include "yv7_kernels.h"

namespace yv7 {

namespace {

constexpr int FI = 4, FC = 4;   // MFMA pixel fragment: 4 images x 4 columns
constexpr int CK = 32;          // channels per chunk (one MFMA K step)
constexpr uint32_t OOB = 0x80000000u;

__host__ __device__ constexpr int swz(int img) { return (0x1320 >> (4 * img)) & 3; }

// Patch geometry of stride S: rows S*TH + 3 - S, columns 6 (S = 1) or 9 (S = 2, input columns 2x0 - 1 ..
// 2x0 + 7, stored even columns first: slot c / 2 for even c, 5 + c / 2 for odd c, so the four lanes'
// columns 2x + s of every tap are four consecutive slots, as with S = 1).
template <int S> __host__ __device__ constexpr int patch_cols() { return S == 1 ? FC + 2 : 2 * FC + 1; }
template <int S> __host__ __device__ constexpr int col_slot(int c) { return S == 1 ? c : ((c & 1) ? 5 + (c >> 1) : (c >> 1)); }

// Tile geometry of a configuration (see conv3x3_lr_kernel).
template <int WM, int WN, int TM, int S>
struct LrGeo {
  static constexpr int NT = 64 * WM * WN;
  static constexpr int TH = TM * WM, PR = S * TH + 3 - S, PC = patch_cols<S>();
  static constexpr int PPX = FI * PR * PC;       // patch pixels
  static constexpr int PB = PPX * 64;            // bytes per patch buffer
};

// tile configurations {WM, WN, TN, TM, PD, S} (variants 270 + row): pixels 16 * WM * TM x channels
// 16 * WN * TN, weights PD column steps ahead, stride S.  Kept from the round-4 sweep of 20 stride-1
// configurations (profiles/r4lr/tune{1,2,3}.txt, one layer forced at a time in the yolov7 bs-32
// forward): 4-wave blocks of 80-pixel tiles with the weights three column steps ahead won every layer
// shape; the 8-wave and 128 / 160-pixel tiles, and two steps of prefetch, lost by 5-20 %.  0: 80 x 128,
// 1: 80 x 64; 2 / 3: the same with 64-pixel tiles for heights that 5 does not divide.  4: stride 2,
// 64 x 128.  At stride 2 the same four were correct but slower than the dispatch on the large yolov7
// stride-2 layers (profiles/r4lr/convbench_s2.txt: 64->128 s2 @320 243 vs 215 us, 256->256 s2 @80 77
// vs 68: a 9-column, 2*TH+1-row patch per output tile is 4-5 input pixels per output against 2.1 at
// stride 1) and faster only where the dispatch split K: 256->256 s2 @40 25.4 vs 29.6.  5 / 6: 160-pixel
// tiles (TH = 10) of 128 / 64 channels (profiles/r4lr/tune_tm10*.txt: 3-9 % on the wide layers).
// Round 5, stride 2 (profiles/r5_s2/cb_deep_s2.txt, tune_deep_*.txt): 7 = 80 x 128 (5 rows) wins on the
// w6 12 800-pixel layers with cout >= 384 (512->768 s2 @80 109.1 -> 101.5 us in-network); 8 = 128 x 128
// (8 rows, PD 2) and 9 = 160 x 64 lost everywhere (VGPR-bound weight prefetch, LDS-read bound) and are
// kept only as forced variants.
// Reading the next column step's patch rows before this step's MFMAs (two register sets; across a
// chunk boundary after the barrier) was no faster on any layer and cost a wave per SIMD
// (profiles/r4lr/tune_xp.txt): three waves per SIMD already hide the LDS latency.
// Round 6: the input patch loaded two chunks ahead (PF = 2: two register sets) on rows 0 / 1 / 3 / 6 was
// no faster on any yolov7 bs-32 layer it could take (one layer forced at a time, profiles/r6_lr_pf2/tune.txt:
// 256->256 @20 22.7 -> 22.8 us, 128->128 @40 21.9 -> 22.3, 512->512 @20 59.2 -> 62.2): the patch's HBM / MALL
// latency is not what these layers wait on; nor did the weights four to seven column steps ahead (PD 4-7
// on rows 0 / 1 / 6, profiles/r6_lr_pd/tune.txt: 22.7 -> 23.5, 61.1 -> 65.8, 38.8 -> 41.6 us).  The PF column
// stays (1 everywhere).
#define LR_CFGS(X)                                                                                   \
  X(0, 1, 4, 2, 5, 3, 1, 1) X(1, 1, 4, 1, 5, 3, 1, 1) X(2, 1, 4, 2, 4, 3, 1, 1) X(3, 1, 4, 1, 4, 3, 1, 1)          \
  X(4, 1, 4, 2, 4, 3, 2, 1) X(5, 1, 4, 2, 10, 2, 1, 1) X(6, 1, 4, 1, 10, 3, 1, 1) X(7, 1, 4, 2, 5, 3, 2, 1)        \
  X(8, 1, 4, 2, 8, 2, 2, 1) X(9, 1, 4, 1, 10, 3, 2, 1)
#define LR_ROW(i, wm, wn, tn, tm, pd, s, pf) {wm, wn, tn, tm, pd, s, pf},
constexpr int LR_CFG[][7] = {LR_CFGS(LR_ROW)};
constexpr int LR_NCFG = sizeof(LR_CFG) / sizeof(LR_CFG[0]);

// One output tile: images b0 .. b0 + 3, rows y0 .. y0 + TH - 1, columns x0 .. x0 + 3, channels n0 .. n0 + BN - 1
// (the body of conv3x3_lr_kernel, shared with the chain kernel of conv_chain.hip).  CPL / CPS: cache policy of
// the patch loads / output stores (0, or CPOL_SC1 for an in-launch hand-off between chained layers); `ready`
// runs before the first load of the tile (the chain kernel waits there for the producing layer's rows).
template <int WM, int WN, int TN, int TM, int NCH, int ACT, int PD, int S, int PF = 1, int CPL = 0, int CPS = 0,
          typename R>
__device__ __forceinline__ void lr_tile(const ConvParams& p, int b0, int y0, int x0, int n0, unsigned char* smem,
                                        R&& ready) {
  using G = LrGeo<WM, WN, TM, S>;
  constexpr int NT = G::NT;
  constexpr int PR = G::PR, PC = G::PC;
  constexpr int NXA = S * TM + 3 - S;            // patch rows a wave reads per column step
  constexpr int PPX = G::PPX;
  constexpr int PB = G::PB;
  constexpr int NPL = (PPX * 4 + NT - 1) / NT;   // 16-byte patch pieces per thread per chunk
  constexpr int NPH = 3 * NCH;                   // column steps ("phases")
  constexpr int NWB = PD + 1;                    // weight register buffers

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave / WN, wn = wave % WN;
  const int g = lane >> 4, li = lane & 15;

  const auto xr = make_rsrc(p.x, p.xbytes);
  const auto wr = make_rsrc(p.wf, p.wfbytes);
  const auto yr = make_rsrc(p.y, 0x7fffffffu);

  // ---- patch pieces of this thread: source offsets (chunk 0) and LDS destinations
  uint32_t po[NPL], pd[NPL];
#pragma unroll
  for (int k = 0; k < NPL; ++k) {
    const int q = tid + k * NT;
    const int px = q >> 2, qq = q & 3;
    if (px < PPX) {
      const int img = px / (PR * PC), r2 = px - img * (PR * PC);
      const int row = r2 / PC, col = r2 - row * PC;
      po[k] = (uint32_t)((pix_index(b0 + img, S * y0 - 1 + row, S * x0 - 1 + col, p.H, p.W) * p.xc + p.xoff + qq * 8) * 2);
      pd[k] = (uint32_t)(((img * PR + row) * PC + col_slot<S>(col)) * 64 + ((qq ^ swz(img)) * 16));
    } else {
      po[k] = OOB;
      pd[k] = 0xffffffffu;
    }
  }
  // chunk c's patch pieces travel in register set c % PF (PF = 2: loaded two chunks ahead of its LDS store)
  u4 pr[PF][NPL];
  auto load_patch = [&](int c) __attribute__((always_inline)) {
#pragma unroll
    for (int k = 0; k < NPL; ++k)
      pr[c % PF][k] = __builtin_bit_cast(u4, __builtin_amdgcn_raw_buffer_load_b128(xr, po[k], (uint32_t)(c * CK * 2), CPL));
  };
  auto store_patch = [&](int c) __attribute__((always_inline)) {   // chunk c into LDS buffer c & 1
#pragma unroll
    for (int k = 0; k < NPL; ++k)
      if (pd[k] != 0xffffffffu) *reinterpret_cast<u4*>(smem + (c & 1) * PB + pd[k]) = pr[c % PF][k];
  };

  // ---- weight fragments: (nf, chunk, tap) at ((nf * NCH + c) * 9 + tap) KiB, lane-linear
  const int nf0 = n0 / 16 + wn * TN;
  u4 wreg[NWB][3][TN];
  uint32_t wlane[TN];   // the lane's offset in the first fragment of each of its channel groups
#pragma unroll
  for (int j = 0; j < TN; ++j) wlane[j] = (uint32_t)((nf0 + j) * NCH * 9 * 1024 + lane * 16);
  auto load_w = [&](int ph, u4 (&w)[3][TN]) __attribute__((always_inline)) {
    const int c = ph / 3, s = ph % 3;
#pragma unroll
    for (int r = 0; r < 3; ++r)
#pragma unroll
      for (int j = 0; j < TN; ++j)   // (chunk, tap) as the scalar offset: no per-load address VALU
        w[r][j] = __builtin_bit_cast(u4, __builtin_amdgcn_raw_buffer_load_b128(
                                             wr, wlane[j], (uint32_t)((c * 9 + r * 3 + s) * 1024), 0));
  };

  // ---- accumulators: bias
  f4 acc[TN][TM];
#pragma unroll
  for (int j = 0; j < TN; ++j) {
    const int col = n0 + wn * TN * 16 + j * 16 + g * 4;
    f4 bv;
#pragma unroll
    for (int e = 0; e < 4; ++e) bv[e] = col + e < p.cout ? p.bias[col + e] : 0.0f;
#pragma unroll
    for (int i = 0; i < TM; ++i) acc[j][i] = bv;
  }

  // per-lane patch read offset: image li / 4, column li % 4 (+ s), slot g ^ f(image)
  const int img = li >> 2;
  const uint32_t a_lane = (uint32_t)(((img * PR) * PC + (li & 3)) * 64 + ((g ^ swz(img)) * 16));
  const uint32_t a_wave = (uint32_t)(S * wm * TM * PC * 64);

  // ---- prologue: chunk 0's patch into buffer 0, chunks 1 .. PF in registers, PD phases of weights
  ready();
  load_patch(0);
#pragma unroll
  for (int ph = 0; ph < PD; ++ph)
    if (ph < NPH) load_w(ph, wreg[ph]);
  store_patch(0);
#pragma unroll
  for (int c = 1; c <= PF; ++c)
    if (c < NCH) load_patch(c);
  __syncthreads();

  // patch rows of column step (c, s): the lane's column 2x + s (S = 2) or x + s sits in slot
  // x + col_slot(s) - col_slot(0)
  auto read_xa = [&](int c, int s, u4 (&xa)[NXA]) __attribute__((always_inline)) {
    const unsigned char* pb = smem + (c & 1) * PB + a_wave + a_lane + col_slot<S>(s) * 64;
#pragma unroll
    for (int j = 0; j < NXA; ++j) xa[j] = *reinterpret_cast<const u4*>(pb + j * PC * 64);
  };
  auto mfmas = [&](int ph, const u4 (&xa)[NXA]) __attribute__((always_inline)) {
    const u4(&w)[3][TN] = wreg[ph % NWB];
#pragma unroll
    for (int r = 0; r < 3; ++r)
#pragma unroll
      for (int j = 0; j < TN; ++j)
#pragma unroll
        for (int i = 0; i < TM; ++i)
          acc[j][i] = __builtin_amdgcn_mfma_f32_16x16x32_f16(__builtin_bit_cast(h8, w[r][j]),
                                                             __builtin_bit_cast(h8, xa[S * i + r]), acc[j][i], 0, 0, 0);
  };
#pragma unroll
  for (int c = 0; c < NCH; ++c) {
#pragma unroll
    for (int s = 0; s < 3; ++s) {
      const int ph = c * 3 + s;
      if (ph + PD < NPH) load_w(ph + PD, wreg[(ph + PD) % NWB]);
      u4 xa[NXA];
      read_xa(c, s, xa);
      mfmas(ph, xa);
    }
    if (c + 1 < NCH) {
      store_patch(c + 1);   // buffer of chunk c - 1: every wave left it at the last barrier
      if (c + 1 + PF < NCH) load_patch(c + 1 + PF);   // into the register set chunk c + 1 just left
      __syncthreads();
    }
  }

  // ---- epilogue: pixel (b0 + li / 4, y0 + wm*4 + i, x0 + li % 4), channels of lane g
#pragma unroll
  for (int i = 0; i < TM; ++i) {
    const bool live = b0 + img < p.B;
    const uint32_t yo =
        live ? (uint32_t)((pix_index(b0 + img, y0 + wm * TM + i, x0 + (li & 3), p.Ho, p.Wo) * p.yc + p.yoff) * 2)
             : 0x80000000u;
    typedef _Float16 h4 __attribute__((ext_vector_type(4)));
    typedef uint32_t u2 __attribute__((ext_vector_type(2)));
    if constexpr (TN % 2 == 0) {
      const uint32_t lane_ch = (uint32_t)(16 * (g & 1) + 8 * (g >> 1));
#pragma unroll
      for (int mp = 0; mp < TN / 2; ++mp) {
        h4 va, vb;
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          va[e] = (_Float16)act_t<ACT>(acc[2 * mp][i][e]);
          vb[e] = (_Float16)act_t<ACT>(acc[2 * mp + 1][i][e]);
        }
        const u2 a = __builtin_bit_cast(u2, va), b = __builtin_bit_cast(u2, vb);
        const auto s0 = __builtin_amdgcn_permlane16_swap(a[0], b[0], false, false);
        const auto s1 = __builtin_amdgcn_permlane16_swap(a[1], b[1], false, false);
        const u4 v = {s0[0], s1[0], s0[1], s1[1]};
        const int n = n0 + wn * TN * 16 + mp * 32 + (int)lane_ch;
        __builtin_amdgcn_raw_buffer_store_b128(v, yr, (live && n < p.cout) ? yo + (uint32_t)n * 2 : 0xffffffffu, 0, CPS);
      }
    } else {
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        h4 va;
#pragma unroll
        for (int e = 0; e < 4; ++e) va[e] = (_Float16)act_t<ACT>(acc[j][i][e]);
        const int n = n0 + wn * TN * 16 + j * 16 + g * 4;
        __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(u2, va), yr,
                                              (live && n < p.cout) ? yo + (uint32_t)n * 2 : 0xffffffffu, 0, CPS);
      }
    }
  }
}

// WM x WN waves; wave (wm, wn) owns output rows wm*TM .. wm*TM+TM-1 of the tile and channels
// n0 + wn*TN*16 .. +TN*16; PD = weight prefetch distance in column steps (3 per chunk); S = stride
// (2: tap (r, s) of output (y, x) is input (2y - 1 + r, 2x - 1 + s): a wave reads patch rows
// 2*wm*TM .. 2*wm*TM + 2*TM once per column step, output row i taking rows 2i + r).  Images past B
// (B not a multiple of 4) read zeros (past the input's buffer range) and store nothing.
template <int WM, int WN, int TN, int TM, int NCH, int ACT, int PD, int S, int PF>
__global__ __launch_bounds__(64 * WM * WN, (8 / (WM * WN)) > 0 ? 8 / (WM * WN) : 1) void conv3x3_lr_kernel(const ConvParams p, int ngx) {
  using G = LrGeo<WM, WN, TM, S>;
  constexpr int TH = G::TH;
  constexpr int BN = WN * TN * 16;
  __shared__ __attribute__((aligned(16))) unsigned char smem[2 * G::PB];

  // tile: XCD-aware (blockIdx % 8 is the XCD on the round-robin dispatch).  The 8 XCDs form ngx N groups
  // x 8 / ngx pixel groups: XCD x holds N slices (x % ngx) * nN / ngx .. + nN / ngx (its share of the
  // weights stays in its 4 MiB L2: ngx is chosen so that share is <= 2.5 MiB) and the (x / ngx)-th
  // contiguous range of pixel tiles (neighbours share patch halos).  ngx = 1: every XCD streams all
  // slices over its eighth of the pixels (the 4.7-9.4 MB weights of the 512-input
  // layers re-fetched from MALL/HBM per tile on every XCD, 5.3x the algorithmic bytes).
  const int bid = blockIdx.x;
  const int nN = (p.cout + BN - 1) / BN;
  const int ncg = p.Wo / FC;
  const int nrg_ = p.Ho / TH, nig = (p.B + FI - 1) / FI;
  const int P = nig * nrg_ * ncg;               // pixel tiles
  const int npx = 8 / ngx, nsl = nN / ngx;      // pixel groups, N slices per XCD
  const int xcd = bid % 8, k = bid / 8;
  const int pper = (P + npx - 1) / npx;         // pixel tiles per pixel group
  const int pi = (xcd / ngx) * pper + k / nsl;
  if (k / nsl >= pper || pi >= P) return;       // (the grid is 8 * nsl * pper blocks)
  const int nt = (xcd % ngx) * nsl + k % nsl;
  int t = pi;
  const int x0 = (t % ncg) * FC;
  t /= ncg;
  const int nrg = p.Ho / TH;   // (t / nrg: image group, ceil(B / 4) of them)
  const int y0 = (t % nrg) * TH;
  const int b0 = (t / nrg) * FI;
  lr_tile<WM, WN, TN, TM, NCH, ACT, PD, S, PF>(p, b0, y0, x0, nt * BN, smem, [] {});
}

// ---------------------------------------------------------------------------------------------
// Chained low-resolution 3x3 layers.  At 20^2 / 40^2 (bs 32) one such layer is 12 800 /
// 51 200 output pixels: its 640 tiles are about one round of the chip's block slots, so every layer pays its
// own ramp, its tail (the CUs idle behind the last tiles) and a kernel boundary; the same layers run 22-37 %
// faster per image at bs 64 / 128 (profiles/r6_diag_batch/).  One launch runs the whole 3x3 stack of an ELAN
// block: a dynamic queue hands out tasks (layer, image group, row band, column group, N slice) in layer
// order; a task of layer l + 1 waits only for the row bands of layer l its 3x3 window reads (rows y0 - 1 ..
// y0 + TH of its four images, every column group and N slice), so the next layer's tiles fill the CUs the
// current layer's tail leaves idle.  Deadlock-free for any residency: a task only waits for tasks with
// smaller queue indices, all handed to blocks that were running when they took them.
//
// Hand-off (MI355X_MICROARCH.md, inter-workgroup visibility, the sc1 form, row 1): a producing layer stores
// its tile with 16-byte sc1 (write-through) stores, every wave waits vmcnt(0), a workgroup barrier, then one
// lane adds 1 to the band's counter (agent-scope atomic); the consumer's lane 0 polls the counters with sc1
// loads (s_sleep between polls), a workgroup barrier, and every load of the handed-off rows is a 16-byte sc1
// buffer load to registers.  The last block to finish re-arms the queue and counters for the next launch.
// Counters (ints, one 128-byte line each): [0] queue head, [32] blocks done, [64] timeout flag (sticky),
// [96 + 32 k] band k: layer l's bands (image group ig, band b) at k = off_l + ig * nrg_l + b, l < nl - 1.
constexpr int CPOL_SC1 = 16;
constexpr int CH_HEAD = 0, CH_DONE = 32, CH_ERR = 64, CH_BAND0 = 96, CH_LINE = 32;

template <int C>
struct LrCfg {
  static constexpr int WM = LR_CFG[C][0], WN = LR_CFG[C][1], TN = LR_CFG[C][2], TM = LR_CFG[C][3],
                       PD = LR_CFG[C][4], S = LR_CFG[C][5], PF = LR_CFG[C][6];
  static constexpr int TH = WM * TM, BN = WN * TN * 16, NT = 64 * WM * WN;
  static constexpr int PB = LrGeo<WM, WN, TM, S>::PB;
};

// per-layer geometry of a chain (host and device)
struct ChainGeo {
  int nl, nig, ncg;
  int th[CHAIN_MAX], bn[CHAIN_MAX], nrg[CHAIN_MAX], nN[CHAIN_MAX], t0[CHAIN_MAX + 1], boff[CHAIN_MAX + 1];
};
__host__ __device__ inline ChainGeo chain_geo(const ChainParams& c) {
  ChainGeo g;
  g.nl = c.nl;
  g.nig = (c.p[0].B + FI - 1) / FI;
  g.ncg = c.p[0].Wo / FC;
  g.t0[0] = 0;
  g.boff[0] = 0;
  for (int l = 0; l < CHAIN_MAX; ++l) {
    const int cfg = l == 0 ? c.cfg0 : c.cfg1;
    const bool on = l < c.nl;
    g.th[l] = LR_CFG[cfg][0] * LR_CFG[cfg][3];
    g.bn[l] = LR_CFG[cfg][1] * LR_CFG[cfg][2] * 16;
    g.nrg[l] = on ? c.p[l].Ho / g.th[l] : 0;
    g.nN[l] = on ? (c.p[l].cout + g.bn[l] - 1) / g.bn[l] : 0;
    g.t0[l + 1] = g.t0[l] + g.nig * g.nrg[l] * g.ncg * g.nN[l];
    g.boff[l + 1] = g.boff[l] + (l + 1 < c.nl ? g.nig * g.nrg[l] : 0);
  }
  return g;
}

template <int C0, int N0, int C1, int N1, int ACT>
__global__ __launch_bounds__(256, 3) void conv3x3_chain_kernel(const ChainParams cp) {
  using A = LrCfg<C0>;
  using Bc = LrCfg<C1>;
  static_assert(A::NT == 256 && Bc::NT == 256 && A::S == 1 && Bc::S == 1, "4-wave stride-1 configurations");
  constexpr int PBM = A::PB > Bc::PB ? A::PB : Bc::PB;
  __shared__ __attribute__((aligned(16))) unsigned char smem[2 * PBM];
  __shared__ int task_s[2], last_s;
  // per layer in LDS (dynamic indexing of a register array would put it in scratch): tiles before it (t0),
  // row bands, N slices, its first band counter (boff)
  __shared__ int t0[CHAIN_MAX + 1], nrg_[CHAIN_MAX], nN_[CHAIN_MAX], boff_[CHAIN_MAX];
  int* const ctr = cp.ctr;
  const int tid = threadIdx.x;
  const int nl = cp.nl;
  const int nig = (cp.p[0].B + FI - 1) / FI, ncg = cp.p[0].Wo / FC, Ho = cp.p[0].Ho;
  if (tid == 0) {
    int ta = 0, bo = 0;
    t0[0] = 0;
#pragma unroll
    for (int l = 0; l < CHAIN_MAX; ++l) {
      const bool on = l < nl;
      const int th = l == 0 ? A::TH : Bc::TH, bn = l == 0 ? A::BN : Bc::BN;
      const int nrg = on ? Ho / th : 0, nN = on ? (cp.p[l].cout + bn - 1) / bn : 0;
      nrg_[l] = nrg;
      nN_[l] = nN;
      boff_[l] = bo;
      bo += nig * nrg;
      ta += nig * nrg * ncg * nN;
      t0[l + 1] = ta;
    }
  }
  __syncthreads();
  const int total = t0[nl];

  for (int it = 0;; ++it) {
    if (tid == 0) task_s[it & 1] = __hip_atomic_fetch_add(ctr + CH_HEAD, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __syncthreads();   // also: every wave is done with the previous task's LDS
    const int t = task_s[it & 1];
    if (t >= total) break;
    int l = 0;
    while (l + 1 < nl && t >= t0[l + 1]) ++l;
    l = __builtin_amdgcn_readfirstlane(l);
    int u = t - t0[l];
    const int nN = nN_[l], nrg = nrg_[l], th = l == 0 ? A::TH : Bc::TH;
    const int nt = u % nN;
    u /= nN;
    const int cg = u % ncg;
    u /= ncg;
    const int band = u % nrg, ig = u / nrg;
    const int b0 = ig * FI, y0 = band * th, x0 = cg * FC, n0 = nt * (l == 0 ? A::BN : Bc::BN);
    const ConvParams& p = cp.p[l];
    // layer l - 1's bands holding rows y0 - 1 .. y0 + th of image group ig, each complete when all of its
    // column groups and N slices have signalled
    auto ready = [&]() __attribute__((always_inline)) {
      if (l > 0) {
        if (tid == 0) {
          const int pth = l == 1 ? A::TH : Bc::TH, pnrg = nrg_[l - 1];
          const int lo = (y0 > 0 ? y0 - 1 : 0) / pth;
          const int hi = (y0 + th < Ho ? y0 + th : Ho - 1) / pth;
          const int target = ncg * nN_[l - 1];
          int* c = ctr + CH_BAND0 + CH_LINE * (boff_[l - 1] + ig * pnrg);
          for (int b = lo; b <= hi; ++b) {
            int spins = 0;
            while (__hip_atomic_load(c + CH_LINE * b, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < target) {
              __builtin_amdgcn_s_sleep(2);
              if (++spins > (1 << 24)) {   // ~1 s: a lost signal would otherwise hang the GPU
                __hip_atomic_store(ctr + CH_ERR, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                break;
              }
            }
          }
        }
        __syncthreads();
      }
    };
    if (l == 0)
      lr_tile<A::WM, A::WN, A::TN, A::TM, N0, ACT, A::PD, 1, A::PF, 0, CPOL_SC1>(p, b0, y0, x0, n0, smem, ready);
    else if (l + 1 < nl)
      lr_tile<Bc::WM, Bc::WN, Bc::TN, Bc::TM, N1, ACT, Bc::PD, 1, Bc::PF, CPOL_SC1, CPOL_SC1>(p, b0, y0, x0, n0, smem, ready);
    else
      lr_tile<Bc::WM, Bc::WN, Bc::TN, Bc::TM, N1, ACT, Bc::PD, 1, Bc::PF, CPOL_SC1, 0>(p, b0, y0, x0, n0, smem, ready);
    if (l + 1 < nl) {   // publish: this tile's rows are in memory
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
      if (tid == 0)
        __hip_atomic_fetch_add(ctr + CH_BAND0 + CH_LINE * (boff_[l] + ig * nrg + band), 1, __ATOMIC_RELAXED,
                               __HIP_MEMORY_SCOPE_AGENT);
    }
  }
  // re-arm: the block that finishes last (every other block has made its last counter access) zeroes the
  // queue head, the done count and the band counters for the next launch
  if (tid == 0) last_s = __hip_atomic_fetch_add(ctr + CH_DONE, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) ==
                         (int)gridDim.x - 1;
  __syncthreads();
  if (last_s) {
    const int nb = boff_[nl - 1];
    for (int k = tid; k < nb; k += 256)
      __hip_atomic_store(ctr + CH_BAND0 + CH_LINE * k, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (tid == 0) {
      __hip_atomic_store(ctr + CH_HEAD, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store(ctr + CH_DONE, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
}

// the (layer-0 configuration, its chunks, later layers' configuration, their chunks) instantiated: the
// ELAN 3x3 stacks of yolov7 bs 32 at 640 (20^2: 256 -> 256, and 512 -> 256 then 256 -> 256; 40^2: 256 ->
// 128 then 128 -> 128) and yolov7-w6 bs 8 at 1280 (its 40^2 and 20^2 stacks: 384 / 512 / 192 / 256
// channels), all on 80 x 64 tiles (configuration 1) or 64 x 64 (3, heights 5 does not divide); the
// runtime gives a chain 80 x 64 tiles where the single-layer dispatch would take 80 x 128 (equal there
// per layer, profiles/r4lr/tune3.txt; twice the tasks for the queue, and the 128-channel form's 160
// VGPRs leave no room for the chain's state at 3 blocks per CU)
#define CHAIN_FORMS(X)                                                                                \
  X(1, 8, 1, 8) X(1, 16, 1, 8) X(1, 8, 1, 4) X(1, 12, 1, 12) X(3, 16, 3, 16) X(3, 12, 3, 16) X(1, 24, 1, 12) \
  X(1, 6, 1, 6) X(1, 12, 1, 6) X(3, 24, 3, 16) X(1, 16, 1, 16) X(1, 4, 1, 4)

// Fragment packing: out[((nf * nch + c) * T + tap) * 512 + lane * 8 + e] =
// w[(nf * 16 + lane % 16) * kpad + tap * cin + c * 32 + (lane / 16) * 8 + e] — the MFMA A operand of
// 16 output channels x 32 input channels of one tap (T = 9 taps of a 3x3 conv, 1 of a 1x1), as one
// lane-linear KiB.
__global__ void pack_frag_kernel(const _Float16* w, int kpad, int cin, int nfrag, int T, _Float16* out) {
  const int nch = cin / CK;
  const long n = (long)nfrag * nch * T * 512;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x) {
    const int e = (int)(i & 7), lane = (int)((i >> 3) & 63);
    long f = i >> 9;
    const int tap = (int)(f % T);
    f /= T;
    const int c = (int)(f % nch);
    const int nf = (int)(f / nch);
    out[i] = w[(size_t)(nf * 16 + (lane & 15)) * kpad + tap * cin + c * CK + (lane >> 4) * 8 + e];
  }
}

template <int WM, int WN, int TN, int TM, int PD, int S, int PF, int NCH>
hipError_t launch_cfg(const ConvParams& p, hipStream_t st) {
  constexpr int TH = TM * WM, BN = WN * TN * 16;
  const long P = (long)((p.B + FI - 1) / FI) * (p.Ho / TH) * (p.Wo / FC);
  const int nN = (p.cout + BN - 1) / BN;
  // N groups over the XCDs: the fewest (a divisor of both 8 and nN) that keep one XCD's weight share
  // under 2.5 MiB (YV7_LR_NGX forces a value for A/B runs)
  static const int force = [] { const char* e = getenv("YV7_LR_NGX"); return e ? atoi(e) : 0; }();
  const double wbytes = (double)p.cout * 9 * p.cin * 2;
  int ngx = 1;
  if (force > 0) {
    ngx = force;
  } else {
    while (ngx < 8 && nN % (2 * ngx) == 0 && wbytes / ngx > 2.5 * 1048576.0) ngx *= 2;
  }
  if (ngx < 1 || 8 % ngx || nN % ngx) ngx = 1;
  const int npx = 8 / ngx, nsl = nN / ngx;
  const long grid = 8L * nsl * ((P + npx - 1) / npx);
  if (p.act == 1) YV7_LAUNCH((conv3x3_lr_kernel<WM, WN, TN, TM, NCH, 1, PD, S, PF>), dim3((unsigned)grid), dim3(64 * WM * WN), 0, st, p, ngx);
  else if (p.act == 2) YV7_LAUNCH((conv3x3_lr_kernel<WM, WN, TN, TM, NCH, 2, PD, S, PF>), dim3((unsigned)grid), dim3(64 * WM * WN), 0, st, p, ngx);
  else YV7_LAUNCH((conv3x3_lr_kernel<WM, WN, TN, TM, NCH, 0, PD, S, PF>), dim3((unsigned)grid), dim3(64 * WM * WN), 0, st, p, ngx);
  return hipGetLastError();
}

template <int WM, int WN, int TN, int TM, int PD, int S, int PF>
hipError_t launch_nch(const ConvParams& p, hipStream_t st) {
  switch (p.cin / CK) {
    case 2: return launch_cfg<WM, WN, TN, TM, PD, S, PF, 2>(p, st);
    case 4: return launch_cfg<WM, WN, TN, TM, PD, S, PF, 4>(p, st);
    case 6: return launch_cfg<WM, WN, TN, TM, PD, S, PF, 6>(p, st);
    case 8: return launch_cfg<WM, WN, TN, TM, PD, S, PF, 8>(p, st);
    case 12: return launch_cfg<WM, WN, TN, TM, PD, S, PF, 12>(p, st);
    case 16: return launch_cfg<WM, WN, TN, TM, PD, S, PF, 16>(p, st);
    case 24: return launch_cfg<WM, WN, TN, TM, PD, S, PF, 24>(p, st);
  }
  return hipErrorInvalidValue;
}


}  // namespace

size_t frag_bytes(int cin, int cout, int taps) { return (size_t)((cout + 15) / 16) * 16 * taps * cin * 2; }

hipError_t pack_frag(const void* w, int kpad, int cin, int cout, int taps, void* out, hipStream_t st) {
  if (cin % CK || (taps != 1 && taps != 9)) return hipErrorInvalidValue;
  const int nfrag = (cout + 15) / 16;   // rows up to cout_pad32 exist in the plan's packed weights
  hipLaunchKernelGGL(pack_frag_kernel, dim3(256), dim3(256), 0, st, reinterpret_cast<const _Float16*>(w), kpad, cin,
                     nfrag, taps, reinterpret_cast<_Float16*>(out));
  return hipGetLastError();
}

// cfg: LR_CFG row (variants 270 + cfg)
bool lr_supported(const ConvParams& p, int cfg) {
  if (cfg < 0 || cfg >= LR_NCFG) return false;
  const int th = LR_CFG[cfg][0] * LR_CFG[cfg][3], S = LR_CFG[cfg][5];
  const int nch = p.cin / CK;
  const bool geom = S == 1 ? (p.Ho == p.H && p.Wo == p.W) : (p.H % 2 == 0 && p.W % 2 == 0 && p.Ho == p.H / 2 && p.Wo == p.W / 2);
  return p.wf && p.k == 3 && p.s == S && p.pad == 1 && !p.pool && p.cin % CK == 0 && geom &&
         (nch == 2 || nch == 4 || nch == 6 || nch == 8 || nch == 12 || nch == 16 || nch == 24) && p.cout % 16 == 0 &&
         p.cout <= 1024 && p.Ho % th == 0 && p.Wo % FC == 0 && p.xoff % 8 == 0 && p.xc % 8 == 0 && p.yoff % 8 == 0 &&
         p.yc % 8 == 0;
}

hipError_t launch_conv_lr(const ConvParams& p, int cfg, hipStream_t st) {
  if (!lr_supported(p, cfg)) return hipErrorInvalidValue;
  switch (cfg) {
#define LR_CASE(i, wm, wn, tn, tm, pd, s, pf) \
  case i: return launch_nch<wm, wn, tn, tm, pd, s, pf>(p, st);
    LR_CFGS(LR_CASE)
#undef LR_CASE
  }
  return hipErrorInvalidValue;
}

static int chain_form(const ChainParams& c) {
  const int n0 = c.p[0].cin / CK, n1 = c.nl > 1 ? c.p[1].cin / CK : 0;
  int id = 0, k = 0;
#define CHAIN_ID(a, b, cc, d) \
  if (id == 0 && c.cfg0 == a && n0 == b && c.cfg1 == cc && n1 == d) id = k + 1; \
  ++k;
  CHAIN_FORMS(CHAIN_ID)
#undef CHAIN_ID
  return id - 1;
}

bool chain_supported(const ChainParams& c) {
  if (c.nl < 2 || c.nl > CHAIN_MAX || chain_form(c) < 0) return false;
  for (int l = 0; l < c.nl; ++l) {
    const ConvParams& p = c.p[l];
    if (!lr_supported(p, l == 0 ? c.cfg0 : c.cfg1) || p.act != c.p[0].act || p.act < 0 || p.act > 2 ||
        p.B != c.p[0].B || p.Ho != c.p[0].Ho || p.Wo != c.p[0].Wo)
      return false;
    if (l > 0 && (p.x != c.p[l - 1].y || p.xoff != c.p[l - 1].yoff || p.xc != c.p[l - 1].yc || p.cin != c.p[l - 1].cout))
      return false;
  }
  return true;
}

size_t chain_counter_bytes(const ChainParams& c) {
  const ChainGeo g = chain_geo(c);
  return (size_t)(CH_BAND0 + CH_LINE * (g.boff[c.nl - 1] + 1)) * 4;
}

long chain_tasks(const ChainParams& c) { return chain_geo(c).t0[c.nl]; }

hipError_t launch_conv_chain(const ChainParams& c, hipStream_t st) {
  if (!chain_supported(c) || !c.ctr) return hipErrorInvalidValue;
  static const int cus = [] {
    int dev = 0, v = 0;
    if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&v, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess ||
        v <= 0)
      v = 256;
    return v;
  }();
  const ChainGeo g = chain_geo(c);
  const long total = g.t0[c.nl];
  const int grid = (int)(total < 3L * cus ? total : 3L * cus);   // 3 blocks per CU at most are resident
  const int form = chain_form(c), act = c.p[0].act;
  int k = 0;
#define CHAIN_CASE(a, b, cc, d)                                                                              \
  if (form == k) {                                                                                           \
    if (act == 1) YV7_LAUNCH((conv3x3_chain_kernel<a, b, cc, d, 1>), dim3(grid), dim3(256), 0, st, c);       \
    else if (act == 2) YV7_LAUNCH((conv3x3_chain_kernel<a, b, cc, d, 2>), dim3(grid), dim3(256), 0, st, c);  \
    else YV7_LAUNCH((conv3x3_chain_kernel<a, b, cc, d, 0>), dim3(grid), dim3(256), 0, st, c);                \
    return hipGetLastError();                                                                                \
  }                                                                                                          \
  ++k;
  CHAIN_FORMS(CHAIN_CASE)
#undef CHAIN_CASE
  return hipErrorInvalidValue;
}

}  // namespace yv7
