// Frame pre-processing on the GPU (gfx950): letterbox = cv2.resize(INTER_LINEAR) + constant border,
// optionally fused with detect.py's input conversion (BGR -> RGB, HWC -> CHW, /255, half/float).
//
// Replaces utils/datasets.py:1277-1307 (letterbox; cv2.resize at :1302, cv2.copyMakeBorder at :1305)
// and detect.py:100-104 / datasets.py:199 (img[:, :, ::-1].transpose(2, 0, 1), .half()/.float(),
// /= 255).  The resize restates OpenCV's generic 8-bit bilinear path bit for bit (see
// oracle/letterbox_ref.py for the algorithm and its parity status): fixed-point coefficient tables
// (11 fractional bits) computed once per shape by a small kernel with the same float/double
// arithmetic as resize.cpp, an exact-int32 horizontal pass and the SIMD vertical pass's rounding;
// an exact 2x downscale takes cv2's INTER_AREA fast path (rounded 2 x 2 mean), as cv2 does.
//
// One thread per output pixel (3 channels); a batch of B frames of one size in one launch.  Input:
// uint8 [B][H][W][3] BGR (packed rows).  Outputs: uint8 [B][oh][ow][3] BGR (the letterboxed frame,
// letterbox()'s return), or fp16 / fp32 [B][3][oh][ow] RGB in [0, 1] (the model input).
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdint.h>

namespace yv7 {

namespace {

constexpr int COEF = 2048;   // INTER_RESIZE_COEF_SCALE
constexpr int SIMD_LANES = 16;

// tables: per destination column / row, the two source indices (clamped) and two coefficients
struct LbTab {
  int* x0;
  int* x1;
  int* ca0;
  int* ca1;
  int* y0;
  int* y1;
  int* cb0;
  int* cb1;
};

__device__ __forceinline__ int cv_round(float v) { return (int)rintf(v); }   // cvRound: half to even

__global__ void lb_tables_kernel(LbTab t, int H, int W, int nh, int nw) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < nw) {   // columns: (sx, fx) reset at the borders (resize.cpp, resizeGeneric_ setup)
    const double scale = 1.0 / ((double)nw / W);
    float f = (float)((i + 0.5) * scale - 0.5);
    int s = (int)floorf(f);
    f -= (float)s;
    if (s < 0) { s = 0; f = 0.f; }
    if (s >= W - 1) { s = W - 1; f = 0.f; }
    t.x0[i] = s;
    t.x1[i] = min(s + 1, W - 1);
    t.ca0[i] = cv_round((1.f - f) * (float)COEF);
    t.ca1[i] = cv_round(f * (float)COEF);
  } else if (i < nw + nh) {   // rows: fy kept, fetched rows clamped
    const int r = i - nw;
    const double scale = 1.0 / ((double)nh / H);
    float f = (float)((r + 0.5) * scale - 0.5);
    const int s = (int)floorf(f);
    f -= (float)s;
    t.y0[r] = min(max(s, 0), H - 1);
    t.y1[r] = min(max(s + 1, 0), H - 1);
    t.cb0[r] = cv_round((1.f - f) * (float)COEF);
    t.cb1[r] = cv_round(f * (float)COEF);
  }
}

// mode: 0 = identity, 1 = bilinear (tables), 2 = exact 2x area
template <int OUT>
__global__ void letterbox_kernel(const uint8_t* __restrict__ src, int H, int W, int nh, int nw, int top, int left,
                                 int oh, int ow, uint8_t pb, uint8_t pg, uint8_t pr, int mode, LbTab t,
                                 void* __restrict__ dst) {
  const int ox = blockIdx.x * blockDim.x + threadIdx.x;
  const int oy = blockIdx.y;
  const int b = blockIdx.z;
  if (ox >= ow) return;
  const int y = oy - top, x = ox - left;
  int v[3];
  if ((unsigned)y < (unsigned)nh && (unsigned)x < (unsigned)nw) {
    const uint8_t* img = src + (size_t)b * H * W * 3;
    if (mode == 0) {
      const uint8_t* p = img + ((size_t)y * W + x) * 3;
      v[0] = p[0]; v[1] = p[1]; v[2] = p[2];
    } else if (mode == 2) {
      const uint8_t* p0 = img + ((size_t)(2 * y) * W + 2 * x) * 3;
      const uint8_t* p1 = p0 + (size_t)W * 3;
#pragma unroll
      for (int c = 0; c < 3; ++c) v[c] = (p0[c] + p0[3 + c] + p1[c] + p1[3 + c] + 2) >> 2;
    } else {
      const int sx0 = t.x0[x] * 3, sx1 = t.x1[x] * 3, a0 = t.ca0[x], a1 = t.ca1[x];
      const uint8_t* r0 = img + (size_t)t.y0[y] * W * 3;
      const uint8_t* r1 = img + (size_t)t.y1[y] * W * 3;
      const int b0 = t.cb0[y], b1 = t.cb1[y];
      const int nv = nw * 3 / SIMD_LANES * SIMD_LANES;   // row positions the SIMD vertical pass covers
#pragma unroll
      for (int c = 0; c < 3; ++c) {
        const int d0 = r0[sx0 + c] * a0 + r0[sx1 + c] * a1;
        const int d1 = r1[sx0 + c] * a0 + r1[sx1 + c] * a1;
        int o;
        if (x * 3 + c < nv) o = ((((d0 >> 4) * b0) >> 16) + (((d1 >> 4) * b1) >> 16) + 2) >> 2;
        else o = (d0 * b0 + d1 * b1 + (1 << 21)) >> 22;
        v[c] = min(max(o, 0), 255);
      }
    }
  } else {
    v[0] = pb; v[1] = pg; v[2] = pr;
  }
  if constexpr (OUT == 0) {
    uint8_t* d = reinterpret_cast<uint8_t*>(dst) + (((size_t)b * oh + oy) * ow + ox) * 3;
    d[0] = (uint8_t)v[0]; d[1] = (uint8_t)v[1]; d[2] = (uint8_t)v[2];
  } else {
    // RGB planes = BGR reversed; x / 255 in float (fp16: rounded once, as torch's half division)
    const size_t plane = (size_t)oh * ow, o = (size_t)b * 3 * plane + (size_t)oy * ow + ox;
#pragma unroll
    for (int c = 0; c < 3; ++c) {
      const float f = (float)v[2 - c] / 255.0f;
      if constexpr (OUT == 1) reinterpret_cast<_Float16*>(dst)[o + c * plane] = (_Float16)f;
      else reinterpret_cast<float*>(dst)[o + c * plane] = f;
    }
  }
}

}  // namespace

size_t letterbox_workspace_bytes(int nh, int nw) { return (size_t)(4 * nw + 4 * nh) * sizeof(int) + 256; }

hipError_t launch_letterbox(const uint8_t* src, int B, int H, int W, int nh, int nw, int top, int left, int oh,
                            int ow, const uint8_t pad[3], int out_kind, void* dst, void* ws, hipStream_t st) {
  int* w = reinterpret_cast<int*>(ws);
  LbTab t{w, w + nw, w + 2 * nw, w + 3 * nw, w + 4 * nw, w + 4 * nw + nh, w + 4 * nw + 2 * nh, w + 4 * nw + 3 * nh};
  int mode = 1;
  if (nh == H && nw == W) mode = 0;
  else if (W == 2 * nw && H == 2 * nh) mode = 2;
  if (mode == 1) {
    const int n = nw + nh;
    hipLaunchKernelGGL(lb_tables_kernel, dim3((n + 255) / 256), dim3(256), 0, st, t, H, W, nh, nw);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
  }
  const dim3 grid((ow + 127) / 128, oh, B);
  if (out_kind == 0)
    hipLaunchKernelGGL(letterbox_kernel<0>, grid, dim3(128), 0, st, src, H, W, nh, nw, top, left, oh, ow, pad[0],
                       pad[1], pad[2], mode, t, dst);
  else if (out_kind == 1)
    hipLaunchKernelGGL(letterbox_kernel<1>, grid, dim3(128), 0, st, src, H, W, nh, nw, top, left, oh, ow, pad[0],
                       pad[1], pad[2], mode, t, dst);
  else
    hipLaunchKernelGGL(letterbox_kernel<2>, grid, dim3(128), 0, st, src, H, W, nh, nw, top, left, oh, ow, pad[0],
                       pad[1], pad[2], mode, t, dst);
  return hipGetLastError();
}

}  // namespace yv7
