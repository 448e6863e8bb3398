// 3x3 / stride-1 / pad-1 fp16 convolution as a persistent "halo ring" on gfx950 (variant 262) — the
// 128-channel-output 3x3 layers with at least one round of 16 x 16 output tiles.  Replaces, like
// conv_f16.hip, Conv.fuseforward (models/common.py:110-111) and RepConv's deploy conv
// (common.py:498-500): y = act(conv2d(x, W', b', s=1, pad=1)).  Round 3 made it the default for the
// 128-channel layers at 80^2; round 4's conv_lr.hip (weights straight to VGPRs, 4-image x 4-column pixel
// fragments) took those layers over (profiles/r4lr/tune3.txt: 3x3 128->128 @80 74.3 -> 63.4 us), so the
// default dispatch picks this kernel only for 128-multiple-channel layers of more than 204 800 output
// pixels.
//
// Why: the implicit-GEMM rings stage one tap's A tile per K step, so every input pixel crosses the
// L2 -> LDS path nine times.  Here a block owns a 16 x 16 output tile of one image x 128 output
// channels; per 32-channel chunk the 18 x 18 input patch (zero frame included, yv7_kernels.h BORDER)
// is DMA'd into LDS ONCE and all nine taps read their pixel fragments from it — tap (r, s) of output
// pixel (y, x) is patch pixel (y + r) * 18 + x + s.  The schedule is described at the kernel.
// LDS rows are 64 bytes (32 fp16); the 16-byte chunk c of row q sits in slot c ^ ((q >> 1) & 3)
// (patch: q's column px instead of q) — conflict-free ds_read_b128 for every tap offset (checked
// exhaustively against the gfx950 lane groups, MI355X_MICROARCH.md §LDS).
#include <type_traits>

#include "yv7_kernels.h"

namespace yv7 {

namespace {

constexpr int TS = 16;                 // output tile side
constexpr int PS = TS + 2;             // patch side
constexpr int PPIX = PS * PS;          // 324 patch pixels
constexpr int CK = 32;                 // channels per phase (one MFMA K step)
constexpr int ROWB = CK * 2;           // 64 bytes per LDS row
constexpr int PPW = 3;                 // patch DMA pieces per wave per chunk (24 pieces: 21 rows of 16 pixels + 3 dummies)
constexpr int NTH = 512;
constexpr uint32_t OOB = 0x80000000u;  // a buffer offset past every tensor: DMA writes zeros

__device__ __forceinline__ void dma16(__amdgpu_buffer_rsrc_t r, void* lds, uint32_t vo, uint32_t so) {
  __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (__attribute__((address_space(3))) void*)lds, 16, vo, so, 0, 0);
}

// The counted waits assume each wave's vector-memory ops issue exactly as written: every dummy DMA
// present (identical dummies to one LDS address were merged by dead-store elimination — one op
// instead of three in a block's last phases, so a wait retired one stage too few) and in program
// order (weights, patch piece, epilogue stores).  Dummies of one phase therefore get distinct LDS
// slots, and this compiler fence (no instruction) keeps the groups from being scheduled across
// each other.
__device__ __forceinline__ void dma_fence() { asm volatile("" ::: "memory"); }

template <int N>
__device__ __forceinline__ void vmwait() {
  static_assert(N >= 0 && N < 64, "vmcnt range");
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

// ---------------------------------------------------------------------------------------------
// Halo ring, column-group form (variant 262).  Measured on round 3's first form (one tap per phase,
// removed in round 4; PMC, 3x3 128->128 @80,
// profiles/r3_pmc_128.txt): 32 % MFMA busy, 37 % of wave time parked at barriers / waits — a phase of
// 16 MFMAs (256 cycles per wave) is shorter than the other group's read segment (8 fragment reads +
// their LDS latency + a DMA issue + the counted wait), so the read segments, not the MFMAs, pace the
// pipeline.  Here a phase is one (chunk, column s) step over the three taps (0, s), (1, s), (2, s):
//  * the wave reads its 6 patch rows y .. y + 5 at column s ONCE (tap (r, s) of output row y + i is
//    patch row y + i + r) and the three taps' weight fragments: 18 reads for 48 MFMAs (24 for 48
//    before), and one barrier pair per 48 MFMAs;
//  * weight stages stay per tap (BN x 32, 8 KiB), three per phase, in a 9-slot ring = three phases;
//    phase p's stages are issued in phase p - 2 into the slots of phase p - 3;
//  * patches are triple-buffered (21 pieces of 1 KiB = 336 pixel rows >= 324, pieces 21-23 of the
//    uniform 3-per-wave issue go to a dummy), one piece per phase: chunk c's pieces are issued in
//    phases 3c - 5 .. 3c - 3, into the buffer chunk c - 3 last read in phase 3c - 7;
//  * so every phase issues 3 weight pieces then 1 patch piece, and the wait before a phase's first
//    barrier is always vmcnt(5) (+ the tile epilogue's stores, in the first phase after one).
// HOOK (microbenchmark builds, scripts/convbench.hip variants 911-914; the ABI never accepts them):
// 1 = no DMA waits in the loop, 2 = no DMA at all in the loop, 3 = no epilogue, 4 = the phase's DMA
// issued right after its first barrier (in the MFMA segment) instead of before the wait (vmcnt(1)).
template <int ACT, int HOOK = 0>
__global__ __launch_bounds__(NTH, 1) void conv3x3_hring2_kernel(const ConvParams p) {
  constexpr int BN = 128;
  constexpr int WNC = BN / 2, TN = WNC / 16, TM = 4;
  constexpr int STG = BN * ROWB;            // 8 KiB per tap stage
  constexpr int NSLOT = 9;                  // three phases of three taps
  constexpr int PB2 = 21 * 1024;            // one patch buffer (336 rows)
  constexpr int RING = 3 * PB2;
  constexpr int BIAS = RING + NSLOT * STG;
  constexpr int DUMMY = BIAS + 4096;        // 4 KiB: a distinct slot for each of a phase's 4 DMA ops
  constexpr int LDS = DUMMY + 4 * 1024;
  static_assert(LDS <= 160 * 1024, "LDS budget");
  __shared__ __attribute__((aligned(16))) unsigned char smem[LDS];
  float* bias_l = reinterpret_cast<float*>(smem + BIAS);

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave >> 1, wn = wave & 1;
  const int grp = wave >> 2;
  const int g = lane >> 4, li = lane & 15;

  const int nN = (p.cout + BN - 1) / BN;
  const int txn = p.Wo / TS, tyn = p.Ho / TS;
  const int T = p.B * tyn * txn * nN;
  const int nch = p.cin / CK;
  const TileWalk tw = xcd_tile_walk(T);
  const int ntl = tw.count();
  if (ntl == 0) return;
  const int nph = ntl * nch * 3;            // phases of this block

  const auto xr = make_rsrc(p.x, p.xbytes);
  const auto wr = make_rsrc(p.w, p.wbytes);
  const auto yr = make_rsrc(p.y, 0x7fffffffu);
  for (int i = tid; i < p.cout; i += NTH) bias_l[i] = p.bias[i];

  struct Tile { int b, y0, x0, n0; };
  auto tile = [&](int it) {
    int t = tw.at(it);
    Tile d;
    d.n0 = (t % nN) * BN;
    t /= nN;
    d.x0 = (t % txn) * TS;
    t /= txn;
    d.y0 = (t % tyn) * TS;
    d.b = t / tyn;
    return d;
  };

  // ---- weight issue cursor: phase wp (tile, chunk, column), three tap stages per phase
  int w_ph = 0, w_it = 0, w_c = 0, w_s = 0;
  uint32_t wvo;
  const int wsrc = (lane & 3) ^ ((lane >> 3) & 3);
  auto w_offsets = [&](int n0) { wvo = (uint32_t)(((n0 + wave * 16 + (lane >> 2)) * p.kpad + wsrc * 8) * 2); };
  w_offsets(tile(0).n0);
  auto issue_w = [&]() __attribute__((always_inline)) {
    const int slot0 = (w_ph % 3) * 3;
    if (w_ph < nph) {
#pragma unroll
      for (int r = 0; r < 3; ++r)
        dma16(wr, smem + RING + (slot0 + r) * STG + wave * 1024, wvo, (uint32_t)(((r * 3 + w_s) * p.cin + w_c * CK) * 2));
    } else {
#pragma unroll
      for (int r = 0; r < 3; ++r) dma16(wr, smem + DUMMY + r * 1024, OOB, 0u);
    }
    dma_fence();
    ++w_ph;
    if (++w_s == 3) {
      w_s = 0;
      if (++w_c == nch) {
        w_c = 0;
        if (++w_it < ntl && nN > 1) w_offsets(tile(w_it).n0);
      }
    }
  };

  // ---- patch issue cursor: piece k = chunk k / 3, the wave's piece k % 3 (q = wave + 8 (k % 3) of 24;
  // q >= 21 is past the 336 rows: a dummy).  Piece k is issued in phase k - 5, so J = k % 3 is known
  // at compile time in every phase.
  int p_k = 0, p_it = 0, p_c = 0;
  uint32_t pvo[PPW];
  auto p_offsets = [&](int it) {
    const Tile d = tile(it);
#pragma unroll
    for (int j = 0; j < PPW; ++j) {
      const int pp = (wave + 8 * j) * 16 + (lane >> 2);
      const int py = pp / PS, px = pp - py * PS;
      const int src = (lane & 3) ^ ((px >> 1) & 3);
      pvo[j] = pp < PPIX ? (uint32_t)((pix_index(d.b, d.y0 - 1 + py, d.x0 - 1 + px, p.H, p.W) * p.xc + p.xoff + src * 8) * 2)
                         : OOB;
    }
  };
  p_offsets(0);
  auto issue_p = [&](auto jc) __attribute__((always_inline)) {
    constexpr int J = decltype(jc)::value;
    const int gc = p_k / 3;
    const bool live = p_it < ntl && wave + 8 * J < 21;
    const int dst = live ? (gc % 3) * PB2 + (wave + 8 * J) * 1024 : DUMMY + 3 * 1024;
    dma16(xr, smem + dst, live ? pvo[J] : OOB, live ? (uint32_t)p_c * CK * 2 : 0u);
    dma_fence();
    if (++p_k % 3 == 0 && p_it < ntl) {
      if (++p_c == nch) {
        p_c = 0;
        if (++p_it < ntl) p_offsets(p_it);
      }
    }
  };

  // ---- compute side: two accumulator sets (tiles alternate between them), so a finished tile's
  // epilogue (activation, fp16, permlane pairing, 16-byte stores) runs in units inside the MFMA
  // segments of the next tile's first six phases (cin >= 64: at least two chunks) instead of stalling
  // both stagger groups at the tile boundary (hook 3 measured the standalone epilogue at 21 % of the
  // kernel).
  f4 accA[TN][TM], accB[TN][TM];
  auto init_tile = [&](f4 (&acc)[TN][TM], const Tile& t) __attribute__((always_inline)) {
#pragma unroll
    for (int j = 0; j < TN; ++j) {
      const int col = t.n0 + wn * WNC + j * 16 + g * 4;
      f4 bv;
#pragma unroll
      for (int e = 0; e < 4; ++e) bv[e] = col + e < p.cout ? bias_l[col + e] : 0.0f;
#pragma unroll
      for (int ii = 0; ii < TM; ++ii) acc[j][ii] = bv;
    }
  };
  const uint32_t lane_ch = (uint32_t)(16 * (g & 1) + 8 * (g >> 1));
  // epilogue unit u = (m-fragment u / 2, channel pair u % 2) of a finished tile: activation, fp16,
  // permlane pairing, one 16-byte store
  auto epi_unit = [&](const f4 (&acc)[TN][TM], const Tile& t, int u, bool live = true) __attribute__((always_inline)) {
    const int ii = u >> 1, mp = u & 1;
    const int y = t.y0 + wm * TM + ii, x = t.x0 + li;
    const uint32_t yo = (uint32_t)((pix_index(t.b, y, x, p.Ho, p.Wo) * p.yc + p.yoff) * 2);
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
    const int n = t.n0 + wn * WNC + mp * 32 + (int)lane_ch;
    const uint32_t off = (live && n < p.cout) ? yo + (uint32_t)n * 2 : 0xffffffffu;
    __builtin_amdgcn_raw_buffer_store_b128(v, yr, off, 0, 0);
  };
  static_assert(TN == 4 && TM == 4, "8 epilogue units per tile");
  // a phase's epilogue share E = first unit * 4 + unit count (-1: none)
  using E02 = std::integral_constant<int, 0 * 4 + 2>;
  using E22 = std::integral_constant<int, 2 * 4 + 2>;
  using E41 = std::integral_constant<int, 4 * 4 + 1>;
  using E51 = std::integral_constant<int, 5 * 4 + 1>;
  using E61 = std::integral_constant<int, 6 * 4 + 1>;
  using E71 = std::integral_constant<int, 7 * 4 + 1>;

  uint32_t a_lane[3];
#pragma unroll
  for (int s = 0; s < 3; ++s) a_lane[s] = (uint32_t)((li + s) * ROWB + ((g ^ (((li + s) >> 1) & 3)) * 16));
  const uint32_t b_lane = (uint32_t)(li * ROWB + ((g ^ ((li >> 1) & 3)) * 16) + wn * WNC * ROWB);
  const uint32_t a_wave = (uint32_t)(wm * TM * PS * ROWB);

  // ---- prologue (as phases -5 .. -1 of the steady state): patch pieces 0..4, phase 0's stages
  // before piece 3 and phase 1's before piece 4; then phase 0's stages and chunk 0's patch landed
  issue_p(std::integral_constant<int, 0>{});
  issue_p(std::integral_constant<int, 1>{});
  issue_p(std::integral_constant<int, 2>{});
  issue_w();
  issue_p(std::integral_constant<int, 0>{});
  issue_w();
  issue_p(std::integral_constant<int, 1>{});
  vmwait<5>();
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");   // bias_l
  __builtin_amdgcn_s_barrier();
  if (grp == 1) __builtin_amdgcn_s_barrier();   // group 1 runs one barrier behind group 0

  int pend = 0;      // epilogue stores this wave issued in the previous phase (younger than the
                     // stages the next wait covers)
  int c_ph = 0;
  // one phase; EPI = the epilogue piece of the previous tile carried in its MFMA segment (-1: none)
  auto phase = [&](auto sc, auto ec, f4 (&acc)[TN][TM], const f4 (&prev)[TN][TM], const Tile& pt, bool hp)
      __attribute__((always_inline)) {
    constexpr int s = decltype(sc)::value;
    constexpr int EPI = decltype(ec)::value;
    const int gc = c_ph / 3;
    const unsigned char* pb = smem + (gc % 3) * PB2 + a_wave + a_lane[s];
    const unsigned char* wb0 = smem + RING + (c_ph % 3) * 3 * STG + b_lane;
    u4 xa[TM + 2], wb[3][TN];
#pragma unroll
    for (int j = 0; j < TM + 2; ++j) xa[j] = *reinterpret_cast<const u4*>(pb + (j * PS) * ROWB);
#pragma unroll
    for (int r = 0; r < 3; ++r)
#pragma unroll
      for (int j = 0; j < TN; ++j) wb[r][j] = *reinterpret_cast<const u4*>(wb0 + r * STG + j * 16 * ROWB);
    constexpr int VM = HOOK == 4 ? 1 : 5;
    if constexpr (HOOK != 2 && HOOK != 4) {
      issue_w();
      issue_p(std::integral_constant<int, (s + 2) % 3>{});   // piece 3c + s + 5 of chunk-major order
    }
    // the previous tile's epilogue units ride in the read segments (this group's reads are in flight,
    // the other group is in its MFMA segment): VALU beside the other wave's MFMAs, stores after this
    // phase's DMA issue
    constexpr int NU = (EPI >= 0 && HOOK != 3) ? (EPI & 3) : 0;
    if constexpr (NU > 0) {
#pragma unroll
      for (int u = 0; u < NU; ++u) epi_unit(prev, pt, (EPI >> 2) + u, hp);
    }
    // vmcnt: ops younger than the stages the next phase reads (issued last phase, see above) = last
    // phase's patch piece and epilogue stores, this phase's 3 weight pieces, patch piece and stores
    if constexpr (HOOK == 1 || HOOK == 2) {
      vmwait<63>();
    } else if (pend == 2) {
      vmwait<VM + 2 + NU>();
    } else if (pend == 1) {
      vmwait<VM + 1 + NU>();
    } else {
      vmwait<VM + NU>();
    }
    pend = NU;
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");   // this phase's reads retired (WAR on ring and patches)
    __builtin_amdgcn_s_barrier();
    if constexpr (HOOK == 4) {
      issue_w();
      issue_p(std::integral_constant<int, (s + 2) % 3>{});
    }
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int r = 0; r < 3; ++r)
#pragma unroll
      for (int j = 0; j < TN; ++j)
#pragma unroll
        for (int ii = 0; ii < TM; ++ii)
          acc[j][ii] = __builtin_amdgcn_mfma_f32_16x16x32_f16(__builtin_bit_cast(h8, wb[r][j]),
                                                             __builtin_bit_cast(h8, xa[ii + r]), acc[j][ii], 0, 0, 0);
    __builtin_amdgcn_s_setprio(0);
    __builtin_amdgcn_s_barrier();
    ++c_ph;
  };
  // one tile into acc; the previous tile (prev, pt) finishes inside its first two chunks (hp = false:
  // the block's first tile — the units run branch-free on the idle set and their stores drop)
  auto run_tile = [&](f4 (&acc)[TN][TM], const f4 (&prev)[TN][TM], const Tile& t, const Tile& pt, bool hp)
      __attribute__((always_inline)) {
    using I0 = std::integral_constant<int, 0>;
    using I1 = std::integral_constant<int, 1>;
    using I2 = std::integral_constant<int, 2>;
    using N = std::integral_constant<int, -1>;
    init_tile(acc, t);
    phase(I0{}, E02{}, acc, prev, pt, hp);
    phase(I1{}, E22{}, acc, prev, pt, hp);
    phase(I2{}, E41{}, acc, prev, pt, hp);
    phase(I0{}, E51{}, acc, prev, pt, hp);
    phase(I1{}, E61{}, acc, prev, pt, hp);
    phase(I2{}, E71{}, acc, prev, pt, hp);
    for (int c = 2; c < nch; ++c) {
      phase(I0{}, N{}, acc, prev, pt, hp);
      phase(I1{}, N{}, acc, prev, pt, hp);
      phase(I2{}, N{}, acc, prev, pt, hp);
    }
    // the accumulators are final here; keep the compiler from speculating epilogue math into the loop
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
      for (int ii = 0; ii < TM; ++ii) asm volatile("" : "+v"(acc[j][ii]));
  };
  auto last_epilogue = [&](const f4 (&acc)[TN][TM], const Tile& t) __attribute__((always_inline)) {
    if constexpr (HOOK != 3) {
#pragma unroll
      for (int u = 0; u < 2 * TM; ++u) epi_unit(acc, t, u);
    }
  };

  Tile tA = tile(0), tB = tA;
#pragma unroll
  for (int j = 0; j < TN; ++j)
#pragma unroll
    for (int ii = 0; ii < TM; ++ii) accB[j][ii] = f4{0.0f, 0.0f, 0.0f, 0.0f};
  for (int it = 0;;) {
    run_tile(accA, accB, tA, tB, it > 0);
    if (++it == ntl) {
      last_epilogue(accA, tA);
      break;
    }
    tB = tile(it);
    run_tile(accB, accA, tB, tA, true);
    if (++it == ntl) {
      last_epilogue(accB, tB);
      break;
    }
    tA = tile(it);
  }
  if (grp == 0) __builtin_amdgcn_s_barrier();
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

}  // namespace

bool hring_supported(const ConvParams& p) {
  return p.k == 3 && p.s == 1 && p.pad == 1 && !p.pool && p.cin % CK == 0 && p.cin >= 2 * CK && p.cout >= 128 &&
         p.cout <= 1024 && p.cout % 8 == 0 && p.xoff % 8 == 0 && p.xc % 8 == 0 && p.yoff % 8 == 0 && p.yc % 8 == 0 &&
         p.Ho == p.H && p.Wo == p.W && p.Ho % TS == 0 && p.Wo % TS == 0;
}

// the column-group halo ring (variant 262)
hipError_t launch_conv_hring(const ConvParams& p, int cus, hipStream_t st) {
  if (!hring_supported(p)) return hipErrorInvalidValue;
  // balanced persistent grid: every block the same number of tiles (the rest of the CUs stay free for
  // other streams' kernels rather than running a short last round)
  const long T = (long)p.B * (p.Ho / TS) * (p.Wo / TS) * ((p.cout + 127) / 128);
  const long per = (T + cus - 1) / cus;
  const int grid = (int)((T + per - 1) / per);
  if (p.act == 1 && p.variant >= 911 && p.variant <= 914) {   // microbenchmark hooks (convbench only)
    if (p.variant == 911) YV7_LAUNCH((conv3x3_hring2_kernel<1, 1>), dim3(grid), dim3(NTH), 0, st, p);
    else if (p.variant == 912) YV7_LAUNCH((conv3x3_hring2_kernel<1, 2>), dim3(grid), dim3(NTH), 0, st, p);
    else if (p.variant == 913) YV7_LAUNCH((conv3x3_hring2_kernel<1, 3>), dim3(grid), dim3(NTH), 0, st, p);
    else YV7_LAUNCH((conv3x3_hring2_kernel<1, 4>), dim3(grid), dim3(NTH), 0, st, p);
    return hipGetLastError();
  }
  if (p.act == 1) YV7_LAUNCH((conv3x3_hring2_kernel<1>), dim3(grid), dim3(NTH), 0, st, p);
  else if (p.act == 2) YV7_LAUNCH((conv3x3_hring2_kernel<2>), dim3(grid), dim3(NTH), 0, st, p);
  else YV7_LAUNCH((conv3x3_hring2_kernel<0>), dim3(grid), dim3(NTH), 0, st, p);
  return hipGetLastError();
}

}  // namespace yv7
