// Dev microbenchmark: time the fp16 conv kernel variants on yolov7-shaped layers (bs 32).
// build: hipcc --offload-arch=gfx950 -O2 scripts/convbench.hip -I yolo-series_amd/csrc
//        -L yolo-series_amd/yv7 -lyv7 -Wl,-rpath,$PWD/yolo-series_amd/yv7 -o convbench
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstring>
#include <vector>
#include "yv7_kernels.h"

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s line %d\n", hipGetErrorString(e), __LINE__); return 1; } } while (0)

struct Shape { const char* name; int B, H, W, cin, cout, k, s; };

int main(int argc, char** argv) {
  std::vector<Shape> shapes = {
    {"1x1 256->256 @160", 32, 160, 160, 256, 256, 1, 1},
    {"3x3 64->64 @160", 32, 160, 160, 64, 64, 3, 1},
    {"3x3 256->256 @40", 32, 40, 40, 256, 256, 3, 1},
    {"1x1 1024->1024 @40", 32, 40, 40, 1024, 1024, 1, 1},
    {"3x3 512->1024 @20", 32, 20, 20, 512, 1024, 3, 1},
    {"3x3s2 128->128 @160", 32, 160, 160, 128, 128, 3, 2},
    {"3x3 8->32 @640", 32, 640, 640, 8, 32, 3, 1},
    {"GEMM 4096^2 K4096", 32, 32, 32, 4096, 4096, 1, 1},
  };
  int variants[] = {1, 2, 4};
  size_t maxx = 0, maxy = 0, maxw = 0;
  for (auto& s : shapes) {
    maxx = std::max(maxx, (size_t)s.B * s.H * s.W * s.cin * 2);
    maxy = std::max(maxy, (size_t)s.B * (s.H / s.s) * (s.W / s.s) * s.cout * 2);
    maxw = std::max(maxw, (size_t)((s.cout + 31) / 32 * 32) * ((s.k * s.k * s.cin + 63) / 64 * 64) * 2);
  }
  void *x, *y, *w, *b, *zero;
  CK(hipMalloc(&x, maxx)); CK(hipMalloc(&y, maxy)); CK(hipMalloc(&w, maxw)); CK(hipMalloc(&b, 8192 * 4));
  CK(hipMalloc(&zero, 4096)); CK(hipMemset(zero, 0, 4096));
  CK(hipMemset(x, 0x3c, maxx)); CK(hipMemset(w, 0x1c, maxw)); CK(hipMemset(b, 0, 8192 * 4));
  hipEvent_t e0, e1; CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
  for (auto& s : shapes) {
    for (int act = 1; act >= 0; --act) {
      yv7::ConvParams p; memset(&p, 0, sizeof(p));
      p.x = x; p.y = y; p.w = w; p.bias = (const float*)b; p.zero = zero;
      p.B = s.B; p.H = s.H; p.W = s.W; p.xc = s.cin; p.xoff = 0; p.cin = s.cin;
      p.k = s.k; p.s = s.s; p.pad = s.k / 2;
      p.Ho = (s.H + 2 * p.pad - s.k) / s.s + 1; p.Wo = (s.W + 2 * p.pad - s.k) / s.s + 1;
      p.yc = s.cout; p.yoff = 0; p.cout = s.cout; p.act = act;
      p.K = s.k * s.k * s.cin; p.kpad = (p.K + 63) / 64 * 64; p.M = s.B * p.Ho * p.Wo;
      double flops = 2.0 * p.M * s.cout * p.K;
      double bytes = 2.0 * ((double)s.B * s.H * s.W * s.cin + (double)p.M * s.cout);
      printf("%-22s act=%d ", s.name, act);
      for (int v : variants) {
        p.variant = v;
        for (int i = 0; i < 3; ++i) CK(yv7::launch_conv(1, p, false, 0));
        CK(hipEventRecord(e0, 0));
        const int it = 10;
        for (int i = 0; i < it; ++i) CK(yv7::launch_conv(1, p, false, 0));
        CK(hipEventRecord(e1, 0)); CK(hipEventSynchronize(e1));
        float ms; CK(hipEventElapsedTime(&ms, e0, e1)); ms /= it;
        printf("| v%d %8.1f us %6.0f TF/s %5.2f TB/s ", v, ms * 1e3, flops / ms / 1e9, bytes / ms / 1e9);
      }
      printf("\n");
    }
  }
  return 0;
}
