// Dev microbenchmark: the fused stem (image -> conv 3->32 3x3 -> conv 32->64 3x3 s2) at bs 32, 640x640,
// fp16 input, SiLU; prints us / TF/s.  Variant hooks via argv (StemParams has none; timing only).
// build: hipcc --offload-arch=gfx950 -O2 scripts/stembench.hip -I yolo-series_amd/csrc
//        -L yolo-series_amd/yv7 -lyv7 -Wl,-rpath,'$ORIGIN/../yolo-series_amd/yv7' -o scripts/stembench
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include "yv7_kernels.h"
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s line %d\n", hipGetErrorString(e), __LINE__); return 1; } } while (0)
__global__ void fill(_Float16* p, size_t n, float scale) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
    uint32_t h = (uint32_t)i * 2654435761u; h ^= h >> 15; h *= 2246822519u; h ^= h >> 13;
    p[i] = (_Float16)(((h & 0xffff) / 65536.0f) * scale);
  }
}
int main(int argc, char** argv) {
  const int B = 32, H = 640, W = 640;
  _Float16 *x, *y, *wa, *wb; float *ba, *bb;
  const size_t ny = yv7::bordered_pixels(B, H / 2, W / 2) * 64;
  CK(hipMalloc(&x, (size_t)B * 3 * H * W * 2)); CK(hipMalloc(&y, ny * 2));
  CK(hipMalloc(&wa, 32 * 64 * 2)); CK(hipMalloc(&wb, 64 * 320 * 2));
  CK(hipMalloc(&ba, 32 * 4)); CK(hipMalloc(&bb, 64 * 4));
  hipLaunchKernelGGL(fill, dim3(4096), dim3(256), 0, 0, x, (size_t)B * 3 * H * W, 1.0f);
  hipLaunchKernelGGL(fill, dim3(64), dim3(256), 0, 0, wa, (size_t)32 * 64, 0.3f);
  hipLaunchKernelGGL(fill, dim3(64), dim3(256), 0, 0, wb, (size_t)64 * 320, 0.1f);
  CK(hipMemset(ba, 0, 32 * 4)); CK(hipMemset(bb, 0, 64 * 4)); CK(hipMemset(y, 0, ny * 2));
  yv7::StemParams p; memset(&p, 0, sizeof(p));
  p.x = x; p.y = y; p.wa = wa; p.ba = ba; p.wb = wb; p.bb = bb;
  p.variant = argc > 1 ? atoi(argv[1]) : 0;
  p.B = B; p.H = H; p.W = W; p.yc = 64; p.yoff = 0; p.kpad_a = 64; p.kpad_b = 320; p.act_a = 1; p.act_b = 1; p.sa = 1;
  hipEvent_t e0, e1; CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
  for (int i = 0; i < 3; ++i) CK(yv7::launch_stem(p, 1, 0));
  CK(hipDeviceSynchronize());
  CK(hipEventRecord(e0, 0));
  for (int i = 0; i < 20; ++i) CK(yv7::launch_stem(p, 1, 0));
  CK(hipEventRecord(e1, 0)); CK(hipEventSynchronize(e1));
  float ms; CK(hipEventElapsedTime(&ms, e0, e1)); ms /= 20;
  const double fl = 2.0 * B * H * W * 32 * 27 + 2.0 * B * (H / 2) * (W / 2) * 64 * 288;
  printf("stem bs32 640 variant %d: %.1f us  %.0f TF/s\n", p.variant, ms * 1e3, fl / ms / 1e9);
  return 0;
}
