// Byte-moving kernels of the yv7 path (gfx950): input packing (+ fused ReOrg), max pooling,
// nearest x2 upsample and channel-slice copy.  All NHWC, 16-byte vectors per lane, grid-stride.
//
// Replaces: detect.py:100-104 (the [0,1] float image batch handed to the model, here packed NCHW ->
// NHWC), ReOrg models/common.py:48-53 (fused into the packing), MP common.py:30-36, SP common.py:39-45,
// SPPCSPC's MaxPool2d(k, 1, k//2) common.py:271, nn.Upsample(None, 2, 'nearest') and the
// Concat copies common.py:56-62 that zero-copy slice writes could not absorb.
#include "yv7_kernels.h"

namespace yv7 {

namespace {

constexpr int NT = 256;

inline int grid_for(size_t work) {
  size_t g = (work + NT - 1) / NT;
  if (g > 256 * 16) g = 256 * 16;
  if (g < 1) g = 1;
  return (int)g;
}

template <typename T> __device__ __forceinline__ T neg_inf();
template <> __device__ __forceinline__ float neg_inf<float>() { return -__builtin_huge_valf(); }
template <> __device__ __forceinline__ _Float16 neg_inf<_Float16>() { return (_Float16)(-__builtin_huge_valf()); }

template <typename T> __device__ __forceinline__ T tmax(T a, T b) { return a > b ? a : b; }

// Index math is 32-bit throughout (pixel and vector counts of one launch stay far below 2^31; the
// runtime checks tensor sizes): a 64-bit division costs several times the 16-byte move it addresses.

// ---- input: x [B,3,H,W] (f32 or f16) -> bordered NHWC T [B,H',W',yc], zero-padded channels.
//      reorg: space-to-depth, channel = g*3 + c, g over (row even,col even),(odd,even),(even,odd),(odd,odd)
template <typename T, typename S, bool REORG>
__global__ __launch_bounds__(NT) void input_kernel(const S* __restrict__ x, T* __restrict__ y, int B, int H, int W,
                                                   int yc) {
  const int Ho = REORG ? H / 2 : H, Wo = REORG ? W / 2 : W;
  const int npix = B * Ho * Wo;
  const size_t plane = (size_t)H * W;
  for (int pix = blockIdx.x * NT + threadIdx.x; pix < npix; pix += gridDim.x * NT) {
    const int t = pix / Wo, wo = pix - t * Wo;
    const int b = t / Ho, ho = t - b * Ho;
    T* out = y + pix_index(b, ho, wo, Ho, Wo) * yc;
    const S* xb = x + (size_t)b * 3 * plane;
    if (!REORG) {
      const size_t o = (size_t)ho * W + wo;
      for (int c = 0; c < yc; ++c) out[c] = c < 3 ? (T)(float)xb[c * plane + o] : (T)0.0f;
    } else {
      for (int c = 0; c < yc; ++c) {
        T v = (T)0.0f;
        if (c < 12) {
          const int gsel = c / 3, ch = c - gsel * 3;
          const int dr = gsel & 1, dc = gsel >> 1;   // g0 (0,0) g1 (1,0) g2 (0,1) g3 (1,1)
          v = (T)(float)xb[ch * plane + (size_t)(2 * ho + dr) * W + (2 * wo + dc)];
        }
        out[c] = v;
      }
    }
  }
}

template <typename T>
__global__ __launch_bounds__(NT) void maxpool_kernel(const T* __restrict__ x, int B, int H, int W, int xc, int xoff,
                                                     T* __restrict__ y, int Ho, int Wo, int yc, int yoff, int C,
                                                     int k, int s, int pad) {
  constexpr int V = Vec<T>::N;
  const int cv = C / V;
  const int total = B * Ho * Wo * cv;
  for (int i = blockIdx.x * NT + threadIdx.x; i < total; i += gridDim.x * NT) {
    const int pix = i / cv, c = (i - pix * cv) * V;
    const int t = pix / Wo, wo = pix - t * Wo;
    const int b = t / Ho, ho = t - b * Ho;
    T m[V];
#pragma unroll
    for (int e = 0; e < V; ++e) m[e] = neg_inf<T>();
    const int h0 = ho * s - pad, w0 = wo * s - pad;
    // -inf padding (nn.MaxPool2d): taps outside the image are skipped, never read from the zero frame
    const int ha = h0 < 0 ? 0 : h0, hb = h0 + k > H ? H : h0 + k;
    const int wa = w0 < 0 ? 0 : w0, wb = w0 + k > W ? W : w0 + k;
    for (int hi = ha; hi < hb; ++hi) {
      const T* row = x + pix_index(b, hi, 0, H, W) * xc + xoff + c;
      for (int wi = wa; wi < wb; ++wi) {
        const u4 v = *reinterpret_cast<const u4*>(row + (size_t)wi * xc);
        const T* e = reinterpret_cast<const T*>(&v);
#pragma unroll
        for (int q = 0; q < V; ++q) m[q] = tmax(m[q], e[q]);
      }
    }
    *reinterpret_cast<u4*>(y + pix_index(b, ho, wo, Ho, Wo) * yc + yoff + c) = *reinterpret_cast<const u4*>(m);
  }
}

// one thread per input pixel and 16-byte chunk: one load, the 2 x 2 output block's four stores (a
// quarter of the index arithmetic of one thread per output)
template <typename T>
__global__ __launch_bounds__(NT) void upsample_kernel(const T* __restrict__ x, int B, int H, int W, int xc, int xoff,
                                                      T* __restrict__ y, int yc, int yoff, int C) {
  constexpr int V = Vec<T>::N;
  const int cv = C / V, Ho = 2 * H, Wo = 2 * W;
  const int total = B * H * W * cv;
  const size_t yrow = (size_t)(Wo + 2 * BORDER) * yc;   // elements per output row
  for (int i = blockIdx.x * NT + threadIdx.x; i < total; i += gridDim.x * NT) {
    const int pix = i / cv, c = (i - pix * cv) * V;
    const int t = pix / W, w = pix - t * W;
    const int b = t / H, h = t - b * H;
    const u4 v = *reinterpret_cast<const u4*>(x + pix_index(b, h, w, H, W) * xc + xoff + c);
    T* o = y + pix_index(b, 2 * h, 2 * w, Ho, Wo) * yc + yoff + c;
    *reinterpret_cast<u4*>(o) = v;
    *reinterpret_cast<u4*>(o + yc) = v;
    *reinterpret_cast<u4*>(o + yrow) = v;
    *reinterpret_cast<u4*>(o + yrow + yc) = v;
  }
}

template <typename T>
__global__ __launch_bounds__(NT) void copy_kernel(const T* __restrict__ x, int B, int H, int W, int xc, int xoff,
                                                  T* __restrict__ y, int yc, int yoff, int C) {
  constexpr int V = Vec<T>::N;
  const int cv = C / V;
  const int total = B * H * W * cv;
  for (int i = blockIdx.x * NT + threadIdx.x; i < total; i += gridDim.x * NT) {
    const int pix = i / cv, c = (i - pix * cv) * V;
    const int t = pix / W, w = pix - t * W;
    const int b = t / H, h = t - b * H;
    const size_t q = pix_index(b, h, w, H, W);
    *reinterpret_cast<u4*>(y + q * yc + yoff + c) = *reinterpret_cast<const u4*>(x + q * xc + xoff + c);
  }
}


// ---- SPPCSPC pool cascade (common.py:271, 276-280 with k = (5, 9, 13)): the three stride-1 pools
//      p5 = pool5(x), p9 = pool5(p5), p13 = pool5(p9) (max is associative; -inf padding keeps the
//      cascade exact) in one launch.  Block = one image x SPP_CG channels (fp16: 64 = one 128-byte
//      line per pixel, so every global load and store covers whole lines): the H x W x CG plane is
//      staged in LDS once; each 5 x 5 pool runs separably (a 5-wide row max into a scratch plane, then
//      a 5-tall column max written back over the stage's input plane, which the row pass has finished
//      reading: 10 LDS reads per output instead of 25; taps outside the image re-read the centre, max
//      being idempotent = the -inf padding); every stage's output also leaves as 16-byte stores into
//      its concat slice.  Round 3's form (16 channels per block: a pixel's 32 bytes per store, a
//      quarter of a line) took 34 us for yolov7's 20 x 20 x 512 at bs 32 — write-combining of partial
//      lines, not bandwidth (52 MB).
constexpr int SPP_CG = 64;
constexpr int SPP_NT = 512;

template <typename T>
__global__ __launch_bounds__(SPP_NT) void spp_cascade_kernel(const T* __restrict__ x, int B, int H, int W, int xc,
                                                             int coff, int C, T* __restrict__ y) {
  constexpr int V = Vec<T>::N;
  constexpr int CG = SPP_CG;             // channels per block
  constexpr int NCH = CG / V;            // 16-byte chunks per pixel
  extern __shared__ __attribute__((aligned(16))) unsigned char lds[];
  const int groups = C / CG;
  const int b = blockIdx.x / groups, c0 = (blockIdx.x - b * groups) * CG;
  const int npx = H * W, items = npx * NCH;
  u4* plane = reinterpret_cast<u4*>(lds);
  u4* tmp = plane + items;
  for (int i = threadIdx.x; i < items; i += SPP_NT) {
    const int px = i / NCH, ch = i - px * NCH, h = px / W, w = px - h * W;
    plane[i] = *reinterpret_cast<const u4*>(x + pix_index(b, h, w, H, W) * xc + coff + c0 + ch * V);
  }
  __syncthreads();
  auto vmax = [](u4 a, u4 c) -> u4 {
    if constexpr (sizeof(T) == 2) {   // packed fp16 max (v_pk_max_f16)
      typedef _Float16 hv8 __attribute__((ext_vector_type(8)));
      return __builtin_bit_cast(u4, __builtin_elementwise_max(__builtin_bit_cast(hv8, a), __builtin_bit_cast(hv8, c)));
    } else {
      typedef float fv4 __attribute__((ext_vector_type(4)));
      return __builtin_bit_cast(u4, __builtin_elementwise_max(__builtin_bit_cast(fv4, a), __builtin_bit_cast(fv4, c)));
    }
  };
  for (int stage = 1; stage <= 3; ++stage) {
    for (int i = threadIdx.x; i < items; i += SPP_NT) {   // row max: 5 taps along w
      const int px = i / NCH, ch = i - px * NCH, w = px % W;
      u4 m = plane[i];
#pragma unroll
      for (int dx = -2; dx <= 2; ++dx) {
        if (dx == 0) continue;
        const bool in = (unsigned)(w + dx) < (unsigned)W;
        m = vmax(m, plane[(in ? px + dx : px) * NCH + ch]);
      }
      tmp[i] = m;
    }
    __syncthreads();
    for (int i = threadIdx.x; i < items; i += SPP_NT) {   // column max: 5 taps along h
      const int px = i / NCH, ch = i - px * NCH, h = px / W, w = px - h * W;
      u4 m = tmp[i];
#pragma unroll
      for (int dy = -2; dy <= 2; ++dy) {
        if (dy == 0) continue;
        const bool in = (unsigned)(h + dy) < (unsigned)H;
        m = vmax(m, tmp[(in ? px + dy * W : px) * NCH + ch]);
      }
      plane[i] = m;
      *reinterpret_cast<u4*>(y + pix_index(b, h, w, H, W) * xc + coff + stage * C + c0 + ch * V) = m;
    }
    __syncthreads();
  }
}


// ---- ReOrg input packing, vectorised (fp16 plans, yc == 16): one thread per output pixel reads its
//      2 x 2 x 3 source values as three 2-value rows pairs (4-byte loads, coalesced along the row)
//      and writes the 16 channels (12 + 4 zero) as two 16-byte stores.
template <typename S>
__global__ __launch_bounds__(NT) void input_reorg16_kernel(const S* __restrict__ x, _Float16* __restrict__ y, int B,
                                                          int H, int W) {
  const int Ho = H / 2, Wo = W / 2;
  const int npix = B * Ho * Wo;
  const size_t plane = (size_t)H * W;
  for (int pix = blockIdx.x * NT + threadIdx.x; pix < npix; pix += gridDim.x * NT) {
    const int t = pix / Wo, wo = pix - t * Wo;
    const int b = t / Ho, ho = t - b * Ho;
    const S* xb = x + (size_t)b * 3 * plane + (size_t)(2 * ho) * W + 2 * wo;
    _Float16 v[16];
#pragma unroll
    for (int ch = 0; ch < 3; ++ch) {
      const S* r0 = xb + ch * plane;
      const S* r1 = r0 + W;
      // channel = g*3 + ch, g over (row even,col even),(odd,even),(even,odd),(odd,odd) (common.py:52-53)
      v[0 * 3 + ch] = (_Float16)(float)r0[0];
      v[1 * 3 + ch] = (_Float16)(float)r1[0];
      v[2 * 3 + ch] = (_Float16)(float)r0[1];
      v[3 * 3 + ch] = (_Float16)(float)r1[1];
    }
#pragma unroll
    for (int c = 12; c < 16; ++c) v[c] = (_Float16)0.0f;
    u4* out = reinterpret_cast<u4*>(y + pix_index(b, ho, wo, Ho, Wo) * 16);
    out[0] = *reinterpret_cast<const u4*>(&v[0]);
    out[1] = *reinterpret_cast<const u4*>(&v[8]);
  }
}

template <typename T, typename S>
hipError_t input_t(const void* x, void* y, int B, int H, int W, int yc, bool reorg, hipStream_t st) {
  const size_t npix = (size_t)B * (reorg ? (H / 2) * (W / 2) : H * W);
  if constexpr (std::is_same<T, _Float16>::value) {
    if (reorg && yc == 16) {
      YV7_LAUNCH((input_reorg16_kernel<S>), dim3(grid_for(npix)), dim3(NT), 0, st, (const S*)x, (T*)y, B, H,
                         W);
      return hipGetLastError();
    }
  }
  if (reorg)
    YV7_LAUNCH((input_kernel<T, S, true>), dim3(grid_for(npix)), dim3(NT), 0, st, (const S*)x, (T*)y, B, H,
                       W, yc);
  else
    YV7_LAUNCH((input_kernel<T, S, false>), dim3(grid_for(npix)), dim3(NT), 0, st, (const S*)x, (T*)y, B, H,
                       W, yc);
  return hipGetLastError();
}

}  // namespace

hipError_t launch_input(int dtype, const void* x, int x_dtype, void* y, int B, int H, int W, int yc, bool reorg,
                        hipStream_t st) {
  if (dtype == 1)
    return x_dtype == 1 ? input_t<_Float16, _Float16>(x, y, B, H, W, yc, reorg, st)
                        : input_t<_Float16, float>(x, y, B, H, W, yc, reorg, st);
  return x_dtype == 1 ? input_t<float, _Float16>(x, y, B, H, W, yc, reorg, st)
                      : input_t<float, float>(x, y, B, H, W, yc, reorg, st);
}

hipError_t launch_maxpool(int dtype, const void* x, int B, int H, int W, int xc, int xoff, void* y, int Ho, int Wo,
                          int yc, int yoff, int C, int k, int s, int pad, hipStream_t st) {
  const size_t work = (size_t)B * Ho * Wo * (C / (dtype == 1 ? 8 : 4));
  if (dtype == 1)
    YV7_LAUNCH(maxpool_kernel<_Float16>, dim3(grid_for(work)), dim3(NT), 0, st, (const _Float16*)x, B, H, W,
                       xc, xoff, (_Float16*)y, Ho, Wo, yc, yoff, C, k, s, pad);
  else
    YV7_LAUNCH(maxpool_kernel<float>, dim3(grid_for(work)), dim3(NT), 0, st, (const float*)x, B, H, W, xc,
                       xoff, (float*)y, Ho, Wo, yc, yoff, C, k, s, pad);
  return hipGetLastError();
}

hipError_t launch_upsample2x(int dtype, const void* x, int B, int H, int W, int xc, int xoff, void* y, int yc, int yoff,
                             int C, hipStream_t st) {
  const size_t work = (size_t)B * H * W * (C / (dtype == 1 ? 8 : 4));
  if (dtype == 1)
    YV7_LAUNCH(upsample_kernel<_Float16>, dim3(grid_for(work)), dim3(NT), 0, st, (const _Float16*)x, B, H, W,
                       xc, xoff, (_Float16*)y, yc, yoff, C);
  else
    YV7_LAUNCH(upsample_kernel<float>, dim3(grid_for(work)), dim3(NT), 0, st, (const float*)x, B, H, W, xc,
                       xoff, (float*)y, yc, yoff, C);
  return hipGetLastError();
}

hipError_t launch_copy(int dtype, const void* x, int B, int H, int W, int xc, int xoff, void* y, int yc, int yoff,
                       int C, hipStream_t st) {
  const size_t work = (size_t)B * H * W * (C / (dtype == 1 ? 8 : 4));
  if (dtype == 1)
    YV7_LAUNCH(copy_kernel<_Float16>, dim3(grid_for(work)), dim3(NT), 0, st, (const _Float16*)x, B, H, W, xc,
                       xoff, (_Float16*)y, yc, yoff, C);
  else
    YV7_LAUNCH(copy_kernel<float>, dim3(grid_for(work)), dim3(NT), 0, st, (const float*)x, B, H, W, xc, xoff,
                       (float*)y, yc, yoff, C);
  return hipGetLastError();
}

bool spp_cascade_supported(int dtype, int H, int W, int C) {
  const int V = dtype == 1 ? 8 : 4;
  return C % SPP_CG == 0 && (size_t)2 * H * W * (SPP_CG / V) * 16 <= 160 * 1024;
}

// x: the concat tensor (pitch xc) holding the pool input at channel slice [coff, coff + C); the three
// pools go to [coff + C, coff + 2C), [coff + 2C, coff + 3C), [coff + 3C, coff + 4C) of the same tensor.
hipError_t launch_spp_cascade(int dtype, void* x, int B, int H, int W, int xc, int coff, int C, hipStream_t st) {
  const int V = dtype == 1 ? 8 : 4;
  const size_t lds = (size_t)2 * H * W * (SPP_CG / V) * 16;
  const dim3 grid(B * (C / SPP_CG));
  if (lds > 64 * 1024) {   // dynamic LDS past 64 KiB must be opted into per kernel
    hipError_t e = dtype == 1 ? hipFuncSetAttribute((const void*)spp_cascade_kernel<_Float16>,
                                                    hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds)
                              : hipFuncSetAttribute((const void*)spp_cascade_kernel<float>,
                                                    hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    if (e != hipSuccess) return e;
  }
  if (dtype == 1)
    YV7_LAUNCH(spp_cascade_kernel<_Float16>, grid, dim3(SPP_NT), lds, st, (const _Float16*)x, B, H, W, xc, coff, C,
                       (_Float16*)x);
  else
    YV7_LAUNCH(spp_cascade_kernel<float>, grid, dim3(SPP_NT), lds, st, (const float*)x, B, H, W, xc, coff, C,
                       (float*)x);
  return hipGetLastError();
}

}  // namespace yv7
