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

// ---- input: x [B,3,H,W] (f32 or f16) -> NHWC T [B,H',W',yc], zero-padded channels.
//      reorg: space-to-depth, channel = g*3 + c, g over (row even,col even),(odd,even),(even,odd),(odd,odd)
template <typename T, typename S, bool REORG>
__global__ __launch_bounds__(NT) void input_kernel(const S* __restrict__ x, T* __restrict__ y, int B, int H, int W,
                                                   int yc) {
  const int Ho = REORG ? H / 2 : H, Wo = REORG ? W / 2 : W;
  const size_t npix = (size_t)B * Ho * Wo;
  const size_t plane = (size_t)H * W;
  for (size_t pix = blockIdx.x * (size_t)NT + threadIdx.x; pix < npix; pix += (size_t)gridDim.x * NT) {
    const int wo = (int)(pix % Wo);
    const size_t t = pix / Wo;
    const int ho = (int)(t % Ho);
    const int b = (int)(t / Ho);
    T* out = y + pix * yc;
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
  const size_t total = (size_t)B * Ho * Wo * cv;
  for (size_t i = blockIdx.x * (size_t)NT + threadIdx.x; i < total; i += (size_t)gridDim.x * NT) {
    const int c = (int)(i % cv) * V;
    const size_t pix = i / cv;
    const int wo = (int)(pix % Wo);
    const size_t t = pix / Wo;
    const int ho = (int)(t % Ho);
    const int b = (int)(t / Ho);
    T m[V];
#pragma unroll
    for (int e = 0; e < V; ++e) m[e] = neg_inf<T>();
    const int h0 = ho * s - pad, w0 = wo * s - pad;
    for (int dy = 0; dy < k; ++dy) {
      const int hi = h0 + dy;
      if ((unsigned)hi >= (unsigned)H) continue;
      for (int dx = 0; dx < k; ++dx) {
        const int wi = w0 + dx;
        if ((unsigned)wi >= (unsigned)W) continue;
        const u4 v = *reinterpret_cast<const u4*>(x + (((size_t)b * H + hi) * W + wi) * xc + xoff + c);
        const T* e = reinterpret_cast<const T*>(&v);
#pragma unroll
        for (int q = 0; q < V; ++q) m[q] = tmax(m[q], e[q]);
      }
    }
    *reinterpret_cast<u4*>(y + pix * yc + yoff + c) = *reinterpret_cast<const u4*>(m);
  }
}

template <typename T>
__global__ __launch_bounds__(NT) void upsample_kernel(const T* __restrict__ x, int B, int H, int W, int xc, int xoff,
                                                      T* __restrict__ y, int yc, int yoff, int C) {
  constexpr int V = Vec<T>::N;
  const int cv = C / V, Ho = 2 * H, Wo = 2 * W;
  const size_t total = (size_t)B * Ho * Wo * cv;
  for (size_t i = blockIdx.x * (size_t)NT + threadIdx.x; i < total; i += (size_t)gridDim.x * NT) {
    const int c = (int)(i % cv) * V;
    const size_t pix = i / cv;
    const int wo = (int)(pix % Wo);
    const size_t t = pix / Wo;
    const int ho = (int)(t % Ho);
    const int b = (int)(t / Ho);
    *reinterpret_cast<u4*>(y + pix * yc + yoff + c) =
        *reinterpret_cast<const u4*>(x + (((size_t)b * H + (ho >> 1)) * W + (wo >> 1)) * xc + xoff + c);
  }
}

template <typename T>
__global__ __launch_bounds__(NT) void copy_kernel(const T* __restrict__ x, size_t npix, int xc, int xoff,
                                                  T* __restrict__ y, int yc, int yoff, int C) {
  constexpr int V = Vec<T>::N;
  const int cv = C / V;
  const size_t total = npix * cv;
  for (size_t i = blockIdx.x * (size_t)NT + threadIdx.x; i < total; i += (size_t)gridDim.x * NT) {
    const int c = (int)(i % cv) * V;
    const size_t pix = i / cv;
    *reinterpret_cast<u4*>(y + pix * yc + yoff + c) = *reinterpret_cast<const u4*>(x + pix * xc + xoff + c);
  }
}

template <typename T, typename S>
hipError_t input_t(const void* x, void* y, int B, int H, int W, int yc, bool reorg, hipStream_t st) {
  const size_t npix = (size_t)B * (reorg ? (H / 2) * (W / 2) : H * W);
  if (reorg)
    hipLaunchKernelGGL((input_kernel<T, S, true>), dim3(grid_for(npix)), dim3(NT), 0, st, (const S*)x, (T*)y, B, H,
                       W, yc);
  else
    hipLaunchKernelGGL((input_kernel<T, S, false>), dim3(grid_for(npix)), dim3(NT), 0, st, (const S*)x, (T*)y, B, H,
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
    hipLaunchKernelGGL(maxpool_kernel<_Float16>, dim3(grid_for(work)), dim3(NT), 0, st, (const _Float16*)x, B, H, W,
                       xc, xoff, (_Float16*)y, Ho, Wo, yc, yoff, C, k, s, pad);
  else
    hipLaunchKernelGGL(maxpool_kernel<float>, dim3(grid_for(work)), dim3(NT), 0, st, (const float*)x, B, H, W, xc,
                       xoff, (float*)y, Ho, Wo, yc, yoff, C, k, s, pad);
  return hipGetLastError();
}

hipError_t launch_upsample2x(int dtype, const void* x, int B, int H, int W, int xc, int xoff, void* y, int yc, int yoff,
                             int C, hipStream_t st) {
  const size_t work = (size_t)B * 4 * H * W * (C / (dtype == 1 ? 8 : 4));
  if (dtype == 1)
    hipLaunchKernelGGL(upsample_kernel<_Float16>, dim3(grid_for(work)), dim3(NT), 0, st, (const _Float16*)x, B, H, W,
                       xc, xoff, (_Float16*)y, yc, yoff, C);
  else
    hipLaunchKernelGGL(upsample_kernel<float>, dim3(grid_for(work)), dim3(NT), 0, st, (const float*)x, B, H, W, xc,
                       xoff, (float*)y, yc, yoff, C);
  return hipGetLastError();
}

hipError_t launch_copy(int dtype, const void* x, int B, int H, int W, int xc, int xoff, void* y, int yc, int yoff,
                       int C, hipStream_t st) {
  const size_t npix = (size_t)B * H * W;
  const size_t work = npix * (C / (dtype == 1 ? 8 : 4));
  if (dtype == 1)
    hipLaunchKernelGGL(copy_kernel<_Float16>, dim3(grid_for(work)), dim3(NT), 0, st, (const _Float16*)x, npix, xc,
                       xoff, (_Float16*)y, yc, yoff, C);
  else
    hipLaunchKernelGGL(copy_kernel<float>, dim3(grid_for(work)), dim3(NT), 0, st, (const float*)x, npix, xc, xoff,
                       (float*)y, yc, yoff, C);
  return hipGetLastError();
}

}  // namespace yv7
