// Implicit-GEMM convolution on MFMA for gfx950 (CDNA4), NHWC activations, KRSC weights.
//
// Replaces the reference's ATen conv2d + activation (Conv.fuseforward models/common.py:110-111,
// RepConv deploy branch common.py:498-500, Detect head conv models/yolo.py:46) and fuses the
// Detect decode (models/yolo.py:52-58) into the head conv's epilogue.
//
// GEMM view: M = B*Ho*Wo output pixels, N = cout, K = k*k*cin ordered (r, s, ci) so every 16-byte
// chunk of K is 8 (fp16) / 4 (fp32) contiguous NHWC channels of one tap.  A block of 256 threads
// (4 waves, 2x2) computes a BM x BN tile; each wave a (BM/2) x (BN/2) sub-tile of 16x16 MFMA tiles.
// K advances 64 bytes per step (32 fp16 / 16 fp32 elements).  Global -> register prefetch of step
// t+1 overlaps the MFMAs of step t; LDS is double-buffered (one barrier per step).
//   fp16: v_mfma_f32_16x16x32_f16, one per 16x16 tile per step (fp32 accumulate).
//   fp32: v_mfma_f32_16x16x4_f32 x4 per step: exact fp32 products, fp32 accumulate (parity mode).
// Epilogue: + fp32 bias, SiLU / LeakyReLU(0.1) / none, convert, staged through LDS and stored as
// 16-byte row chunks into a channel slice (offset yoff, pitch yc) of the output -> concat is free.
#include <cstdlib>

#include "yv7_kernels.h"

namespace yv7 {

namespace {

constexpr int NT = 256;       // threads per block
constexpr int ROWB = 80;      // LDS bytes per tile row: 64 data + 16 pad (breaks the 64-B stride)

__device__ __forceinline__ float act_fn(float v, int act) {
  if (act == 1) return v / (1.0f + expf(-v));          // SiLU  x * sigmoid(x)
  if (act == 2) return v > 0.0f ? v : v * 0.1f;         // LeakyReLU(0.1)
  return v;
}

template <typename T>
__device__ __forceinline__ void mfma_step(const u4& a, const u4& b, f4& acc);

template <>
__device__ __forceinline__ void mfma_step<_Float16>(const u4& a, const u4& b, f4& acc) {
  acc = __builtin_amdgcn_mfma_f32_16x16x32_f16(__builtin_bit_cast(h8, a), __builtin_bit_cast(h8, b), acc, 0, 0, 0);
}

template <>
__device__ __forceinline__ void mfma_step<float>(const u4& a, const u4& b, f4& acc) {
  // lane group g = lane>>4 holds k = 4g..4g+3 of this step; MFMA kk consumes k = 4g+kk from A and B.
  // Blocked summation: the step's 16 products are summed in a fresh accumulator and then added to
  // the running total, so the fp32 rounding error grows with K/16 + 16 instead of K (parity mode).
  const f4 fa = __builtin_bit_cast(f4, a), fb = __builtin_bit_cast(f4, b);
  f4 t = {0.f, 0.f, 0.f, 0.f};
  t = __builtin_amdgcn_mfma_f32_16x16x4f32(fa[0], fb[0], t, 0, 0, 0);
  t = __builtin_amdgcn_mfma_f32_16x16x4f32(fa[1], fb[1], t, 0, 0, 0);
  t = __builtin_amdgcn_mfma_f32_16x16x4f32(fa[2], fb[2], t, 0, 0, 0);
  t = __builtin_amdgcn_mfma_f32_16x16x4f32(fa[3], fb[3], t, 0, 0, 0);
  acc += t;
}

template <typename T, int BM, int BN, bool ONE, bool DET>
__global__ __launch_bounds__(NT) void conv_kernel(const ConvParams p) {
  constexpr int V = Vec<T>::N;            // elements per 16-byte chunk
  constexpr int BKE = 4 * V;              // K elements per step (64 bytes)
  constexpr int NA = BM * 4 / NT;         // A chunks per thread
  constexpr int NB = (BN * 4 + NT - 1) / NT;
  constexpr int WTM = BM / 2, WTN = BN / 2;
  constexpr int TM = WTM / 16, TN = WTN / 16;
  constexpr int AB_BYTES = 2 * (BM + BN) * ROWB;
  constexpr int CPITCH = BN * (int)sizeof(T) + 16;     // staged C row pitch (bytes)
  constexpr int C_BYTES = DET ? 0 : BM * CPITCH;
  constexpr int LDS_BYTES = AB_BYTES > C_BYTES ? AB_BYTES : C_BYTES;
  __shared__ __attribute__((aligned(16))) unsigned char smem[LDS_BYTES];

  const int tid = threadIdx.x;
  const int lane = tid & 63, wave = tid >> 6;
  const int wm = wave >> 1, wn = wave & 1;

  // XCD-aware bijective remap: consecutive tile ids land on one XCD, N-tiles of an M-tile adjacent.
  const int nwg = gridDim.x, bid = blockIdx.x;
  const int q = nwg >> 3, r = nwg & 7, xcd = bid & 7, loc = bid >> 3;
  const int wgid = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + loc;
  const int nN = (p.cout + BN - 1) / BN;
  const int m0 = (wgid / nN) * BM, n0 = (wgid % nN) * BN;

  const T* __restrict__ x = reinterpret_cast<const T*>(p.x);
  const T* __restrict__ w = reinterpret_cast<const T*>(p.w);

  // ---- per-thread A-row precompute (bordered input: see BORDER in yv7_kernels.h)
  const int cA = tid & 3;                 // chunk column this thread loads (A and B)
  int a_b[NA], a_h[NA], a_w[NA];
  bool a_ok[NA];
#pragma unroll
  for (int j = 0; j < NA; ++j) {
    const int m = m0 + (tid >> 2) + 64 * j;
    a_ok[j] = m < p.M;
    const int mm = a_ok[j] ? m : 0;
    const int hw = p.Ho * p.Wo;
    const int b = mm / hw, rem = mm - b * hw;
    const int ho = rem / p.Wo, wo = rem - ho * p.Wo;
    a_b[j] = b;
    a_h[j] = ho * p.s - p.pad;
    a_w[j] = wo * p.s - p.pad;
  }

  u4 ra[NA], rb[NB];
  const int nk = p.kpad / BKE;

  auto gload = [&](int kt) {
    const int k = kt * BKE + cA * V;
    int tap = 0, ci = k;
    if (!ONE && k < p.K) { tap = k / p.cin; ci = k - tap * p.cin; }
    const int rr = ONE ? 0 : tap / p.k, ss = ONE ? 0 : tap - rr * p.k;
#pragma unroll
    for (int j = 0; j < NA; ++j) {
      u4 v = {0u, 0u, 0u, 0u};
      const int hi = a_h[j] + rr, wi = a_w[j] + ss;
      if (a_ok[j] && k < p.K && (unsigned)hi < (unsigned)p.H && (unsigned)wi < (unsigned)p.W)
        v = *reinterpret_cast<const u4*>(x + pix_index(a_b[j], hi, wi, p.H, p.W) * p.xc + p.xoff + ci);
      ra[j] = v;
    }
#pragma unroll
    for (int j = 0; j < NB; ++j) {
      const int row = (tid >> 2) + 64 * j;
      const int n = n0 + row;
      u4 v = {0u, 0u, 0u, 0u};
      if (row < BN && n < p.cout) v = *reinterpret_cast<const u4*>(w + (size_t)n * p.kpad + k);
      rb[j] = v;
    }
  };
  auto lstore = [&](int buf) {
    unsigned char* As = smem + buf * (BM + BN) * ROWB;
    unsigned char* Bs = As + BM * ROWB;
#pragma unroll
    for (int j = 0; j < NA; ++j)
      *reinterpret_cast<u4*>(As + ((tid >> 2) + 64 * j) * ROWB + cA * 16) = ra[j];
#pragma unroll
    for (int j = 0; j < NB; ++j) {
      const int row = (tid >> 2) + 64 * j;
      if (row < BN) *reinterpret_cast<u4*>(Bs + row * ROWB + cA * 16) = rb[j];
    }
  };

  f4 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[i][j] = f4{0.f, 0.f, 0.f, 0.f};

  gload(0);
  lstore(0);
  __syncthreads();
  const int g = lane >> 4, li = lane & 15;
  for (int kt = 0; kt < nk; ++kt) {
    const int buf = kt & 1;
    if (kt + 1 < nk) gload(kt + 1);
    const unsigned char* As = smem + buf * (BM + BN) * ROWB;
    const unsigned char* Bs = As + BM * ROWB;
    u4 af[TM], bf[TN];
#pragma unroll
    for (int i = 0; i < TM; ++i)
      af[i] = *reinterpret_cast<const u4*>(As + (wm * WTM + i * 16 + li) * ROWB + g * 16);
#pragma unroll
    for (int j = 0; j < TN; ++j)
      bf[j] = *reinterpret_cast<const u4*>(Bs + (wn * WTN + j * 16 + li) * ROWB + g * 16);
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int j = 0; j < TN; ++j) mfma_step<T>(af[i], bf[j], acc[i][j]);
    if (kt + 1 < nk) lstore(buf ^ 1);
    __syncthreads();
  }

  if (DET) {
    // Fused Detect decode (models/yolo.py:52-57): y = sigmoid(v);
    //   xy = (y*2 - 0.5 + grid) * stride ; wh = (y*2)**2 * anchor_grid ; rest = y.
    const int hw = p.Ho * p.Wo;
#pragma unroll
    for (int j = 0; j < TN; ++j) {
      const int n = n0 + wn * WTN + j * 16 + li;
      if (n >= p.cout) continue;
      const int a = n / p.no, o = n - a * p.no;
      const float bias = p.bias[n];
#pragma unroll
      for (int i = 0; i < TM; ++i) {
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const int m = m0 + wm * WTM + i * 16 + g * 4 + e;
          if (m >= p.M) continue;
          const int b = m / hw, rem = m - b * hw;
          const int gy = rem / p.Wo, gx = rem - gy * p.Wo;
          const float v = acc[i][j][e] + bias;
          const float sg = 1.0f / (1.0f + expf(-v));
          float out;
          if (o < 2) {
            const float t = sg * 2.0f;
            const float u = t - 0.5f;
            const float gg = (o == 0) ? (float)gx : (float)gy;
            out = (u + gg) * p.stride;
          } else if (o < 4) {
            const float t = sg * 2.0f;
            out = (t * t) * p.anchor[2 * a + (o - 2)];
          } else {
            out = sg;
          }
          const size_t cell = ((size_t)a * p.Ho + gy) * p.Wo + gx;
          p.z[(((size_t)b * p.nrows + p.row_off + cell) * p.no) + o] = out;
          if (p.raw) p.raw[(((size_t)b * p.na * hw) + cell) * p.no + o] = v;
        }
      }
    }
    return;
  }

  // ---- epilogue: bias + act -> LDS C tile -> 16-byte row chunks into the output channel slice
  unsigned char* Cs = smem;
#pragma unroll
  for (int j = 0; j < TN; ++j) {
    const int col = wn * WTN + j * 16 + li;
    const int n = n0 + col;
    const float bias = (n < p.cout) ? p.bias[n] : 0.0f;
#pragma unroll
    for (int i = 0; i < TM; ++i) {
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int row = wm * WTM + i * 16 + g * 4 + e;
        const float v = act_fn(acc[i][j][e] + bias, p.act);
        *reinterpret_cast<T*>(Cs + row * CPITCH + col * (int)sizeof(T)) = (T)v;
      }
    }
  }
  __syncthreads();
  constexpr int CPR = BN * (int)sizeof(T) / 16;   // chunks per row
  T* __restrict__ y = reinterpret_cast<T*>(p.y);
  const int hw = p.Ho * p.Wo;
  for (int c = tid; c < BM * CPR; c += NT) {
    const int row = c / CPR, ch = c - row * CPR;
    const int m = m0 + row, n = n0 + ch * V;
    if (m < p.M && n < p.cout) {
      const int b = m / hw, rem = m - b * hw;
      const int ho = rem / p.Wo, wo = rem - ho * p.Wo;
      *reinterpret_cast<u4*>(y + pix_index(b, ho, wo, p.Ho, p.Wo) * p.yc + p.yoff + n) =
          *reinterpret_cast<const u4*>(Cs + row * CPITCH + ch * 16);
    }
  }
}

template <typename T, int BM, int BN, bool ONE, bool DET>
hipError_t launch_t(const ConvParams& p, hipStream_t st) {
  const int nM = (p.M + BM - 1) / BM, nN = (p.cout + BN - 1) / BN;
  YV7_LAUNCH((conv_kernel<T, BM, BN, ONE, DET>), dim3(nM * nN), dim3(NT), 0, st, p);
  return hipGetLastError();
}

template <typename T>
hipError_t launch_dt(const ConvParams& p, bool det, hipStream_t st) {
  const bool one = p.k == 1 && p.s == 1 && p.pad == 0;
  if (det) return launch_t<T, 128, 128, true, true>(p, st);
  if (p.cout <= 32) return one ? launch_t<T, 128, 32, true, false>(p, st) : launch_t<T, 128, 32, false, false>(p, st);
  if (p.cout <= 64) return one ? launch_t<T, 128, 64, true, false>(p, st) : launch_t<T, 128, 64, false, false>(p, st);
  return one ? launch_t<T, 128, 128, true, false>(p, st) : launch_t<T, 128, 128, false, false>(p, st);
}

}  // namespace

static bool use_v1() {
  static const bool v1 = [] { const char* e = getenv("YV7_CONV_V1"); return e && e[0] == '1'; }();
  return v1;
}

bool det_writes_rowbest(int dtype) { return dtype == 1 && !use_v1(); }

hipError_t launch_conv(int dtype, const ConvParams& p, bool detect, hipStream_t st) {
  // fp16: the tuned kernel of conv_f16.hip (YV7_CONV_V1=1 selects this file's generic kernel, for A/B)
  const bool v1 = use_v1();
  if (p.pool) return dtype == 1 ? launch_conv_f16(p, detect, st) : hipErrorInvalidValue;   // MP-folded 1x1
  // cout <= 32 (the stem of every model, tiny's narrow layers): this kernel's BK=32 steps waste less
  // of the short, padded K than the 64-deep steps of conv_f16 (measured: scripts/convbench.hip)
  if (dtype == 1)
    return (v1 || p.variant == 1 || (p.variant == 0 && !detect && p.cout <= 32)) ? launch_dt<_Float16>(p, detect, st)
                                                                                 : launch_conv_f16(p, detect, st);
  return launch_dt<float>(p, detect, st);
}

}  // namespace yv7
