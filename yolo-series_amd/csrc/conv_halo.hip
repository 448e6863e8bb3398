// 3x3 / stride-1 / pad-1 fp16 convolution with the input tile staged ONCE per channel chunk
// (gfx950).  Replaces, like conv_f16.hip, Conv.fuseforward (models/common.py:110-111) and RepConv's
// deploy conv (common.py:498-500) — here for the 3x3 stride-1 layers of the ELAN stacks
// (cfg/deploy/yolov7.yaml:22-25, 35-38, ...), the bulk of the network's MFMA work.
//
// Why a second conv kernel: the implicit-GEMM kernel stages one tap's A tile per K step, so every
// input pixel crosses the L1 -> LDS path nine times; for narrow layers (64-128 output channels) that
// staging, not the MFMA, sets the pace.  Here a block owns a 16 x 16 output tile of one image:
//  * per 64-channel chunk, the 18 x 18 input patch (zero frame included, see BORDER) is loaded once
//    into LDS (41.5 KiB, XOR-swizzled 128-byte pixel rows) and all nine taps read their A fragments
//    from it: tap (r, s) of output pixel (y, x) is patch pixel (y + r) * 18 + x + s;
//  * the weights of one (chunk, tap) step — BN rows x 64 k — stream through a double-buffered LDS
//    stage, loaded into registers one step ahead;
//  * 4 waves, each 4 output rows (64 pixels) x BN channels: per 32-deep MFMA sub-step 4 A + BN/16 B
//    fragment reads feed 4 * BN/16 v_mfma_f32_16x16x32_f16;
//  * epilogue as in conv_f16.hip: accumulators start at the bias, compile-time activation, fp16 tile
//    staged through LDS and stored as 16-byte NHWC chunks into the output channel slice.
#include "yv7_kernels.h"

namespace yv7 {

namespace {

constexpr int NT = 256;
constexpr int TS = 16;               // output tile side
constexpr int PS = TS + 2;           // patch side
constexpr int PPIX = PS * PS;        // 324 patch pixels
constexpr int PBYTES = PPIX * 128;   // 41,472 bytes per 64-channel chunk
constexpr int PITEMS = PPIX * 8;     // 16-byte items per patch
constexpr int PR = (PITEMS + NT - 1) / NT;   // items per thread (11, the last partial)

__device__ __forceinline__ int swz(int row, int chunk) { return chunk ^ (row & 7); }

template <int BN>
__global__ __launch_bounds__(NT, 2) void conv3x3_halo_kernel(const ConvParams p) {
  constexpr int TN = BN / 16;              // n-tiles per wave (every wave covers all BN channels)
  constexpr int TM = 4;                    // m-tiles per wave: 4 output rows of 16 pixels
  constexpr int WST = BN * 128;            // one weight stage: BN rows x 64 k
  constexpr int RW = BN * 8 / NT;          // weight items per thread
  constexpr int CPITCH = BN * 2 + 16;
  constexpr int MAIN = PBYTES + 2 * WST;
  constexpr int EPI = TS * TS * CPITCH;
  constexpr int LDS = MAIN > EPI ? MAIN : EPI;
  static_assert(BN * 8 % NT == 0, "weight stage must split evenly over the block");
  __shared__ __attribute__((aligned(16))) unsigned char smem[LDS];
  unsigned char* patch = smem;
  unsigned char* wstage = smem + PBYTES;

  const int tid = threadIdx.x;
  const int lane = tid & 63, wave = tid >> 6;
  const int g = lane >> 4, li = lane & 15;

  // block -> (image, tile row, tile col, n tile); the n tiles of one spatial tile are adjacent
  const int nwg = gridDim.x, bid = blockIdx.x;
  const int q = nwg >> 3, r8 = nwg & 7, xcd = bid & 7, loc = bid >> 3;
  int wgid = (xcd < r8 ? xcd * (q + 1) : r8 * (q + 1) + (xcd - r8) * q) + loc;
  const int nN = (p.cout + BN - 1) / BN;
  const int tx_n = p.Wo / TS, ty_n = p.Ho / TS;
  const int nt = wgid % nN;
  wgid /= nN;
  const int tx = wgid % tx_n;
  wgid /= tx_n;
  const int ty = wgid % ty_n;
  const int b = wgid / ty_n;
  const int y0 = ty * TS, x0 = tx * TS, n0 = nt * BN;

  const auto xr = make_rsrc(p.x, p.xbytes);
  const auto wr = make_rsrc(p.w, p.wbytes);

  // patch items: item = tid + NT*j -> pixel item>>3 (row-major over the 18 x 18 patch), chunk item&7
  uint32_t poff[PR];
#pragma unroll
  for (int j = 0; j < PR; ++j) {
    const int item = tid + NT * j;
    const int pp = item >> 3, ch = item & 7;
    const int py = pp / PS, px = pp - py * PS;
    poff[j] = item < PITEMS
                  ? (uint32_t)((pix_index(b, y0 - 1 + py, x0 - 1 + px, p.H, p.W) * p.xc + p.xoff + ch * 8) * 2)
                  : 0x80000000u;   // beyond the buffer: zeros (never stored)
  }
  // weight items: row n0 + (tid >> 3) + 32 j, chunk tid & 7
  uint32_t woff[RW];
#pragma unroll
  for (int j = 0; j < RW; ++j) woff[j] = (uint32_t)(((n0 + (tid >> 3) + 32 * j) * p.kpad + (tid & 7) * 8) * 2);

  const int nchunk = p.cin / 64;
  const int nsteps = nchunk * 9;
  // step s = chunk c * 9 + tap t: weights at K column t * cin + c * 64 (K order r, s, ci)
  auto wcol_bytes = [&](int s) {
    const int c = s / 9, t = s - c * 9;
    return (uint32_t)((t * p.cin + c * 64) * 2);
  };

  u4 rp[PR], rw[RW];
  auto load_patch = [&](int c) {
#pragma unroll
    for (int j = 0; j < PR; ++j)
      rp[j] = __builtin_bit_cast(u4, __builtin_amdgcn_raw_buffer_load_b128(xr, poff[j], (uint32_t)c * 128, 0));
  };
  auto store_patch = [&]() {
#pragma unroll
    for (int j = 0; j < PR; ++j) {
      const int item = tid + NT * j;
      if (j < PR - 1 || item < PITEMS) {
        const int pp = item >> 3, ch = item & 7;
        *reinterpret_cast<u4*>(patch + pp * 128 + swz(pp, ch) * 16) = rp[j];
      }
    }
  };
  auto load_w = [&](int s) {
    const uint32_t so = wcol_bytes(s);
#pragma unroll
    for (int j = 0; j < RW; ++j) rw[j] = __builtin_bit_cast(u4, __builtin_amdgcn_raw_buffer_load_b128(wr, woff[j], so, 0));
  };
  auto store_w = [&](int buf) {
    unsigned char* ws = wstage + buf * WST;
#pragma unroll
    for (int j = 0; j < RW; ++j) {
      const int row = (tid >> 3) + 32 * j;
      *reinterpret_cast<u4*>(ws + row * 128 + swz(row, tid & 7) * 16) = rw[j];
    }
  };

  f4 acc[TN][TM];
#pragma unroll
  for (int j = 0; j < TN; ++j) {
    const int col = n0 + j * 16 + g * 4;
    f4 bv;
#pragma unroll
    for (int e = 0; e < 4; ++e) bv[e] = col + e < p.cout ? p.bias[col + e] : 0.0f;
#pragma unroll
    for (int i = 0; i < TM; ++i) acc[j][i] = bv;
  }

  load_patch(0);
  load_w(0);
  store_patch();
  store_w(0);
  __syncthreads();
  for (int s = 0; s < nsteps; ++s) {
    const int t = s % 9;
    const bool chunk_end = t == 8 && s + 1 < nsteps;
    if (s + 1 < nsteps) load_w(s + 1);
    if (t == 0 && s + 9 < nsteps) load_patch(s / 9 + 1);   // next chunk's patch: 9 steps to land
    const int rr = t / 3, ss = t - rr * 3;
    const unsigned char* ws = wstage + (s & 1) * WST;
#pragma unroll
    for (int sub = 0; sub < 2; ++sub) {
      const int ch = sub * 4 + g;
      u4 xa[TM], wb[TN];
#pragma unroll
      for (int i = 0; i < TM; ++i) {
        const int pp = (wave * TM + i + rr) * PS + li + ss;
        xa[i] = *reinterpret_cast<const u4*>(patch + pp * 128 + swz(pp, ch) * 16);
      }
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        const int row = j * 16 + li;
        wb[j] = *reinterpret_cast<const u4*>(ws + row * 128 + swz(row, ch) * 16);
      }
#pragma unroll
      for (int j = 0; j < TN; ++j)
#pragma unroll
        for (int i = 0; i < TM; ++i)
          acc[j][i] = __builtin_amdgcn_mfma_f32_16x16x32_f16(__builtin_bit_cast(h8, wb[j]),
                                                             __builtin_bit_cast(h8, xa[i]), acc[j][i], 0, 0, 0);
    }
    if (s + 1 < nsteps) store_w((s + 1) & 1);
    if (chunk_end) {   // every wave is done with this chunk's patch before it is overwritten
      __syncthreads();
      store_patch();
    }
    __syncthreads();
  }

  // epilogue: acc[j][i][e] = channel n0 + j*16 + g*4 + e of output pixel (y0 + wave*4 + i, x0 + li)
  unsigned char* Cs = smem;
  with_act(p.act, [&](auto actc) {
    constexpr int ACT = decltype(actc)::value;
#pragma unroll
    for (int j = 0; j < TN; ++j) {
      const int col = j * 16 + g * 4;
#pragma unroll
      for (int i = 0; i < TM; ++i) {
        const int px = (wave * TM + i) * TS + li;
        typedef _Float16 h4 __attribute__((ext_vector_type(4)));
        h4 v;
#pragma unroll
        for (int e = 0; e < 4; ++e) v[e] = (_Float16)act_t<ACT>(acc[j][i][e]);
        *reinterpret_cast<h4*>(Cs + px * CPITCH + col * 2) = v;
      }
    }
  });
  __syncthreads();
  constexpr int CPR = BN * 2 / 16;
  _Float16* __restrict__ y = reinterpret_cast<_Float16*>(p.y);
  for (int cc = tid; cc < TS * TS * CPR; cc += NT) {
    const int px = cc / CPR, ch = cc - px * CPR;
    const int oy = px / TS, ox = px - oy * TS;
    const int n = n0 + ch * 8;
    if (n < p.cout)
      *reinterpret_cast<u4*>(y + pix_index(b, y0 + oy, x0 + ox, p.Ho, p.Wo) * p.yc + p.yoff + n) =
          *reinterpret_cast<const u4*>(Cs + px * CPITCH + ch * 16);
  }
}

template <int BN>
hipError_t launch_bn(const ConvParams& p, hipStream_t st) {
  const int nblk = p.B * (p.Ho / TS) * (p.Wo / TS) * ((p.cout + BN - 1) / BN);
  YV7_LAUNCH((conv3x3_halo_kernel<BN>), dim3(nblk), dim3(NT), 0, st, p);
  return hipGetLastError();
}

}  // namespace

bool halo_supported(const ConvParams& p) {
  return p.k == 3 && p.s == 1 && p.pad == 1 && p.cin % 64 == 0 && p.cout % 64 == 0 && p.Ho % TS == 0 &&
         p.Wo % TS == 0 && p.Ho == p.H && p.Wo == p.W;
}

hipError_t launch_conv_halo(const ConvParams& p, hipStream_t st) {
  if (!halo_supported(p)) return hipErrorInvalidValue;
  if (p.cout % 128 == 0) return launch_bn<128>(p, st);
  return launch_bn<64>(p, st);
}

}  // namespace yv7
