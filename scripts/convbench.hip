// Dev microbenchmark: time the fp16 conv kernel variants on yolov7-shaped layers (bs 32), random
// operands, and check every variant's output against the default dispatch (variant 0).
// build: hipcc --offload-arch=gfx950 -O2 scripts/convbench.hip -I yolo-series_amd/csrc
//        -L yolo-series_amd/yv7 -lyv7 -Wl,-rpath,$PWD/yolo-series_amd/yv7 -o scripts/convbench
// usage: convbench [variant ...]      (default: 0 4 5)
#include <hip/hip_runtime.h>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>
#include "yv7_kernels.h"

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s line %d\n", hipGetErrorString(e), __LINE__); return 1; } } while (0)

struct Shape { const char* name; int B, H, W, cin, cout, k, s; };

__global__ void fill_rand(_Float16* p, size_t n, uint32_t seed, float scale) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
    uint32_t h = (uint32_t)i * 2654435761u ^ seed;
    h ^= h >> 15; h *= 2246822519u; h ^= h >> 13; h *= 3266489917u; h ^= h >> 16;
    p[i] = (_Float16)(((h & 0xffff) / 32768.0f - 1.0f) * scale);
  }
}

// the conv kernels read a 3x3 window's out-of-image taps from the tensor's zero frame (yv7_kernels.h)
__global__ void zero_frame(_Float16* x, int B, int H, int W, int C) {
  const size_t n = yv7::bordered_pixels(B, H, W);
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
    const int w = (int)(i % (W + 2)), h = (int)((i / (W + 2)) % (H + 2));
    if (h == 0 || h == H + 1 || w == 0 || w == W + 1)
      for (int c = 0; c < C; ++c) x[i * C + c] = (_Float16)0.0f;
  }
}

int main(int argc, char** argv) {
  std::vector<Shape> shapes = {
    {"3x3 64->64 @320", 32, 320, 320, 64, 64, 3, 1},
    {"3x3s2 64->128 @320", 32, 320, 320, 64, 128, 3, 2},
    {"3x3 64->64 @160", 32, 160, 160, 64, 64, 3, 1},
    {"3x3 64->64 @80", 32, 80, 80, 64, 64, 3, 1},
    {"3x3 128->64 @80", 32, 80, 80, 128, 64, 3, 1},
    {"3x3 128->128 @80", 32, 80, 80, 128, 128, 3, 1},
    {"3x3 128->128 @40", 32, 40, 40, 128, 128, 3, 1},
    {"3x3 256->128 @40", 32, 40, 40, 256, 128, 3, 1},
    {"3x3 256->256 @40", 32, 40, 40, 256, 256, 3, 1},
    {"3x3 256->256 @20", 32, 20, 20, 256, 256, 3, 1},
    {"3x3 512->256 @20", 32, 20, 20, 512, 256, 3, 1},
    {"3x3 512->512 @20", 32, 20, 20, 512, 512, 3, 1},
    {"3x3s2 128->128 @160", 32, 160, 160, 128, 128, 3, 2},
    {"3x3s2 128->128 @80", 32, 80, 80, 128, 128, 3, 2},
    {"3x3s2 256->256 @80", 32, 80, 80, 256, 256, 3, 2},
    {"3x3s2 256->256 @40", 32, 40, 40, 256, 256, 3, 2},
    {"3x3s2 512->512 @40", 32, 40, 40, 512, 512, 3, 2},
    {"3x3s2 128->256 @320 b8", 8, 320, 320, 128, 256, 3, 2},
    {"3x3s2 128->256 @160 b8", 8, 160, 160, 128, 256, 3, 2},
    {"3x3s2 256->512 @160 b8", 8, 160, 160, 256, 512, 3, 2},
    {"3x3s2 512->768 @80 b8", 8, 80, 80, 512, 768, 3, 2},
    {"3x3s2 768->1024 @40 b8", 8, 40, 40, 768, 1024, 3, 2},
    {"3x3s2 256->384 @80 b8", 8, 80, 80, 256, 384, 3, 2},
    {"3x3s2 384->512 @40 b8", 8, 40, 40, 384, 512, 3, 2},
    {"3x3 128->256 @80", 32, 80, 80, 128, 256, 3, 1},
    {"3x3 256->512 @40", 32, 40, 40, 256, 512, 3, 1},
    {"3x3 512->1024 @20", 32, 20, 20, 512, 1024, 3, 1},
    {"1x1 256->256 @160", 32, 160, 160, 256, 256, 1, 1},
    {"1x1 256->128 @160", 32, 160, 160, 256, 128, 1, 1},
    {"1x1 128->128 @160", 32, 160, 160, 128, 128, 1, 1},
    {"1x1 512->512 @80", 32, 80, 80, 512, 512, 1, 1},
    {"1x1 512->256 @80", 32, 80, 80, 512, 256, 1, 1},
    {"1x1 512->128 @80", 32, 80, 80, 512, 128, 1, 1},
    {"1x1 256->256 @80", 32, 80, 80, 256, 256, 1, 1},
    {"1x1 128->128 @80", 32, 80, 80, 128, 128, 1, 1},
    {"1x1 1024->1024 @40", 32, 40, 40, 1024, 1024, 1, 1},
    {"1x1 1024->512 @40", 32, 40, 40, 1024, 512, 1, 1},
    {"1x1 1024->256 @40", 32, 40, 40, 1024, 256, 1, 1},
    {"1x1 512->512 @40", 32, 40, 40, 512, 512, 1, 1},
    {"1x1 256->256 @40", 32, 40, 40, 256, 256, 1, 1},
    {"1x1 256->128 @40", 32, 40, 40, 256, 128, 1, 1},
    {"1x1 128->128 @40", 32, 40, 40, 128, 128, 1, 1},
    {"1x1 2048->512 @20", 32, 20, 20, 2048, 512, 1, 1},
    {"1x1 1024->1024 @20", 32, 20, 20, 1024, 1024, 1, 1},
    {"1x1 1024->512 @20", 32, 20, 20, 1024, 512, 1, 1},
    {"1x1 512->512 @20", 32, 20, 20, 512, 512, 1, 1},
    {"1x1 512->256 @20", 32, 20, 20, 512, 256, 1, 1},
    {"1x1 256->256 @20", 32, 20, 20, 256, 256, 1, 1},
  };
  std::vector<int> variants;
  for (int i = 1; i < argc; ++i) variants.push_back(atoi(argv[i]));
  if (variants.empty()) variants = {0, 4, 5};
  double tot_best = 0, tot_v0 = 0;
  size_t maxx = 0, maxy = 0, maxw = 0;
  for (auto& s : shapes) {
    maxx = std::max(maxx, yv7::bordered_pixels(s.B, s.H, s.W) * s.cin);
    maxy = std::max(maxy, yv7::bordered_pixels(s.B, s.H / s.s, s.W / s.s) * s.cout);
    maxw = std::max(maxw, (size_t)((s.cout + 31) / 32 * 32) * ((s.k * s.k * s.cin + 63) / 64 * 64));
  }
  _Float16 *x, *y, *y0, *w;
  float* b;
  void* zero;
  CK(hipMalloc(&x, maxx * 2)); CK(hipMalloc(&y, maxy * 2)); CK(hipMalloc(&y0, maxy * 2)); CK(hipMalloc(&w, maxw * 2));
  CK(hipMalloc(&b, 8192 * 4)); CK(hipMalloc(&zero, 4096)); CK(hipMemset(zero, 0, 4096));
  void* wf;   // fragment-packed 3x3 weights (conv_lr.hip, variants 270-274)
  CK(hipMalloc(&wf, maxw * 2));
  const size_t part_bytes = (size_t)512 << 20;
  const int cnt_n = 1 << 20;
  float* part; int* cnt;
  CK(hipMalloc(&part, part_bytes)); CK(hipMalloc(&cnt, cnt_n * 4)); CK(hipMemset(cnt, 0, cnt_n * 4));
  CK(hipMemset(y, 0, maxy * 2)); CK(hipMemset(y0, 0, maxy * 2));
  hipLaunchKernelGGL(fill_rand, dim3(4096), dim3(256), 0, 0, x, maxx, 1u, 1.0f);
  CK(hipMemset(b, 0, 8192 * 4));
  std::vector<_Float16> hy(maxy), hy0(maxy);
  hipEvent_t e0, e1; CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
  const char* filt = getenv("CB_SHAPE");   // substring filter on the shape name
  for (auto& s : shapes) {
    if (filt && !strstr(s.name, filt)) continue;
    yv7::ConvParams p; memset(&p, 0, sizeof(p));
    p.x = x; p.y = y; p.w = w; p.bias = b; p.zero = zero;
    hipLaunchKernelGGL(fill_rand, dim3(4096), dim3(256), 0, 0, x, maxx, 1u, 1.0f);
    hipLaunchKernelGGL(zero_frame, dim3(1024), dim3(256), 0, 0, x, s.B, s.H, s.W, s.cin);
    p.part = part; p.cnt = cnt; p.part_bytes = part_bytes; p.cnt_n = cnt_n;
    p.B = s.B; p.H = s.H; p.W = s.W; p.xc = s.cin; p.xoff = 0; p.cin = s.cin;
    p.k = s.k; p.s = s.s; p.pad = s.k / 2;
    p.Ho = (s.H + 2 * p.pad - s.k) / s.s + 1; p.Wo = (s.W + 2 * p.pad - s.k) / s.s + 1;
    p.yc = s.cout; p.yoff = 0; p.cout = s.cout; p.act = 1;
    p.K = s.k * s.k * s.cin; p.kpad = (p.K + 63) / 64 * 64; p.M = s.B * p.Ho * p.Wo;
    p.xbytes = (uint32_t)(yv7::bordered_pixels(s.B, s.H, s.W) * s.cin * 2);
    p.wbytes = (uint32_t)((size_t)(s.cout + 31) / 32 * 32 * p.kpad * 2);
    // weights ~ U(-1,1)/sqrt(K) so outputs stay O(1); padded K columns zero
    CK(hipMemset(w, 0, maxw * 2));
    for (int n = 0; n < s.cout; ++n)
      hipLaunchKernelGGL(fill_rand, dim3(4), dim3(256), 0, 0, w + (size_t)n * p.kpad, (size_t)p.K, 7u + n,
                         1.0f / sqrtf((float)p.K));
    if (s.cin % 32 == 0) {
      CK(yv7::pack_frag(w, p.kpad, s.cin, s.cout, s.k * s.k, wf, 0));
      p.wf = wf;
      p.wfbytes = (uint32_t)yv7::frag_bytes(s.cin, s.cout, s.k * s.k);
    }
    const size_t ny = yv7::bordered_pixels(s.B, p.Ho, p.Wo) * s.cout;
    double flops = 2.0 * p.M * s.cout * p.K;
    double bytes = 2.0 * ((double)s.B * s.H * s.W * s.cin + (double)ny);
    printf("%-22s", s.name);
    double best = 1e30; int bestv = 0;
    for (int v : variants) {
      p.variant = v;
      p.y = v == 0 ? (void*)y0 : (void*)y;
      CK(hipMemset(p.y, 0, ny * 2));   // (a hook variant's garbage must not reach the next shape's border)
      if (yv7::launch_conv(1, p, false, 0) != hipSuccess) { (void)hipGetLastError(); printf(" |%d -", v); continue; }
      for (int i = 0; i < 2; ++i) CK(yv7::launch_conv(1, p, false, 0));
      CK(hipDeviceSynchronize());
      CK(hipEventRecord(e0, 0));
      const int it = 20;
      for (int i = 0; i < it; ++i) CK(yv7::launch_conv(1, p, false, 0));
      CK(hipEventRecord(e1, 0)); CK(hipEventSynchronize(e1));
      float ms; CK(hipEventElapsedTime(&ms, e0, e1)); ms /= it;
      double maxd = 0;
      if (v != 0) {
        CK(hipMemcpy(hy.data(), y, ny * 2, hipMemcpyDeviceToHost));
        CK(hipMemcpy(hy0.data(), y0, ny * 2, hipMemcpyDeviceToHost));
        for (size_t i = 0; i < ny; ++i) maxd = std::max(maxd, (double)fabsf((float)hy[i] - (float)hy0[i]));
      }
      printf(" |%d %6.1f %4.0fT", v, ms * 1e3, flops / ms / 1e9);
      if (v != 0 && maxd > 0.02) printf(" d=%.3g", maxd);
      if (v == 0) tot_v0 += ms * 1e3;
      best = std::min(best, (double)ms * 1e3);
      if (ms * 1e3 <= best) bestv = v;
    }
    printf("  best v%d\n", bestv);
    tot_best += best;
    fflush(stdout);
  }
  printf("total v0 %.1f us, best-of %.1f us\n", tot_v0, tot_best);
  return 0;
}
