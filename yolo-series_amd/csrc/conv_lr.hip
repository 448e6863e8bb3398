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

// WM x WN waves; wave (wm, wn) owns output rows wm*TM .. wm*TM+TM-1 of the tile and channels
// n0 + wn*TN*16 .. +TN*16; PD = weight prefetch distance in column steps (3 per chunk); S = stride
// (2: tap (r, s) of output (y, x) is input (2y - 1 + r, 2x - 1 + s): a wave reads patch rows
// 2*wm*TM .. 2*wm*TM + 2*TM once per column step, output row i taking rows 2i + r).  Images past B
// (B not a multiple of 4) read zeros (past the input's buffer range) and store nothing.
template <int WM, int WN, int TN, int TM, int NCH, int ACT, int PD, int S>
__global__ __launch_bounds__(64 * WM * WN, (8 / (WM * WN)) > 0 ? 8 / (WM * WN) : 1) void conv3x3_lr_kernel(const ConvParams p, int ngx) {
  constexpr int NT = 64 * WM * WN;
  constexpr int TH = TM * WM, PR = S * TH + 3 - S, PC = patch_cols<S>();
  constexpr int NXA = S * TM + 3 - S;            // patch rows a wave reads per column step
  constexpr int PPX = FI * PR * PC;              // patch pixels
  constexpr int PB = PPX * 64;                   // bytes per patch buffer
  constexpr int BN = WN * TN * 16;
  constexpr int NPL = (PPX * 4 + NT - 1) / NT;   // 16-byte patch pieces per thread per chunk
  constexpr int NPH = 3 * NCH;                   // column steps ("phases")
  constexpr int NWB = PD + 1;                    // weight register buffers
  __shared__ __attribute__((aligned(16))) unsigned char smem[2 * PB];

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave / WN, wn = wave % WN;
  const int g = lane >> 4, li = lane & 15;

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
  const int n0 = nt * BN;

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
  u4 pr[NPL];
  auto load_patch = [&](int c) __attribute__((always_inline)) {
#pragma unroll
    for (int k = 0; k < NPL; ++k)
      pr[k] = __builtin_bit_cast(u4, __builtin_amdgcn_raw_buffer_load_b128(xr, po[k], (uint32_t)(c * CK * 2), 0));
  };
  auto store_patch = [&](int buf) __attribute__((always_inline)) {
#pragma unroll
    for (int k = 0; k < NPL; ++k)
      if (pd[k] != 0xffffffffu) *reinterpret_cast<u4*>(smem + buf * PB + pd[k]) = pr[k];
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

  // ---- prologue: chunk 0's patch into buffer 0, chunk 1's in registers, PD phases of weights
  load_patch(0);
#pragma unroll
  for (int ph = 0; ph < PD; ++ph)
    if (ph < NPH) load_w(ph, wreg[ph]);
  store_patch(0);
  if constexpr (NCH > 1) load_patch(1);
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
      store_patch((c + 1) & 1);   // buffer of chunk c - 1: every wave left it at the last barrier
      if (c + 2 < NCH) load_patch(c + 2);
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
        __builtin_amdgcn_raw_buffer_store_b128(v, yr, (live && n < p.cout) ? yo + (uint32_t)n * 2 : 0xffffffffu, 0, 0);
      }
    } else {
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        h4 va;
#pragma unroll
        for (int e = 0; e < 4; ++e) va[e] = (_Float16)act_t<ACT>(acc[j][i][e]);
        const int n = n0 + wn * TN * 16 + j * 16 + g * 4;
        __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(u2, va), yr,
                                              (live && n < p.cout) ? yo + (uint32_t)n * 2 : 0xffffffffu, 0, 0);
      }
    }
  }
}

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

template <int WM, int WN, int TN, int TM, int PD, int S, int NCH>
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
  if (p.act == 1) YV7_LAUNCH((conv3x3_lr_kernel<WM, WN, TN, TM, NCH, 1, PD, S>), dim3((unsigned)grid), dim3(64 * WM * WN), 0, st, p, ngx);
  else if (p.act == 2) YV7_LAUNCH((conv3x3_lr_kernel<WM, WN, TN, TM, NCH, 2, PD, S>), dim3((unsigned)grid), dim3(64 * WM * WN), 0, st, p, ngx);
  else YV7_LAUNCH((conv3x3_lr_kernel<WM, WN, TN, TM, NCH, 0, PD, S>), dim3((unsigned)grid), dim3(64 * WM * WN), 0, st, p, ngx);
  return hipGetLastError();
}

template <int WM, int WN, int TN, int TM, int PD, int S>
hipError_t launch_nch(const ConvParams& p, hipStream_t st) {
  switch (p.cin / CK) {
    case 2: return launch_cfg<WM, WN, TN, TM, PD, S, 2>(p, st);
    case 4: return launch_cfg<WM, WN, TN, TM, PD, S, 4>(p, st);
    case 6: return launch_cfg<WM, WN, TN, TM, PD, S, 6>(p, st);
    case 8: return launch_cfg<WM, WN, TN, TM, PD, S, 8>(p, st);
    case 12: return launch_cfg<WM, WN, TN, TM, PD, S, 12>(p, st);
    case 16: return launch_cfg<WM, WN, TN, TM, PD, S, 16>(p, st);
    case 24: return launch_cfg<WM, WN, TN, TM, PD, S, 24>(p, st);
  }
  return hipErrorInvalidValue;
}

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
#define LR_CFGS(X)                                                                                   \
  X(0, 1, 4, 2, 5, 3, 1) X(1, 1, 4, 1, 5, 3, 1) X(2, 1, 4, 2, 4, 3, 1) X(3, 1, 4, 1, 4, 3, 1) X(4, 1, 4, 2, 4, 3, 2) \
  X(5, 1, 4, 2, 10, 2, 1) X(6, 1, 4, 1, 10, 3, 1) X(7, 1, 4, 2, 5, 3, 2) X(8, 1, 4, 2, 8, 2, 2) X(9, 1, 4, 1, 10, 3, 2)
#define LR_ROW(i, wm, wn, tn, tm, pd, s) {wm, wn, tn, tm, pd, s},
constexpr int LR_CFG[][6] = {LR_CFGS(LR_ROW)};
constexpr int LR_NCFG = sizeof(LR_CFG) / sizeof(LR_CFG[0]);

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
#define LR_CASE(i, wm, wn, tn, tm, pd, s) \
  case i: return launch_nch<wm, wn, tn, tm, pd, s>(p, st);
    LR_CFGS(LR_CASE)
#undef LR_CASE
  }
  return hipErrorInvalidValue;
}

}  // namespace yv7
