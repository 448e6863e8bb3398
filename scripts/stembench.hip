// Dev microbenchmark: the fused stem (image -> conv 3->32 3x3 -> conv 32->64 3x3 s2) at bs 32, 640x640,
// fp16 input, SiLU; prints us / TF/s.  Variant hooks via argv[1] (StemParams::variant; timing only).
// argv[2] = w6: the w6 front end instead (ReOrg + 12->64 + 64->128 s2, stem_reorg_kernel) at bs 8, 1280.
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
  const bool w6 = argc > 2 && !strcmp(argv[2], "w6");
  const int B = w6 ? 8 : 32, H = w6 ? 1280 : 640, W = H;
  const int CA = w6 ? 64 : 32, CB = w6 ? 128 : 64, KA = w6 ? 192 : 64, KB = w6 ? 576 : 320;
  const int HB = w6 ? H / 4 : H / 2, WB = HB;
  _Float16 *x, *y, *wa, *wb; float *ba, *bb;
  const size_t ny = yv7::bordered_pixels(B, HB, WB) * CB;
  CK(hipMalloc(&x, (size_t)B * 3 * H * W * 2)); CK(hipMalloc(&y, ny * 2));
  CK(hipMalloc(&wa, CA * KA * 2)); CK(hipMalloc(&wb, CB * KB * 2));
  CK(hipMalloc(&ba, CA * 4)); CK(hipMalloc(&bb, CB * 4));
  hipLaunchKernelGGL(fill, dim3(4096), dim3(256), 0, 0, x, (size_t)B * 3 * H * W, 1.0f);
  hipLaunchKernelGGL(fill, dim3(64), dim3(256), 0, 0, wa, (size_t)CA * KA, 0.3f);
  hipLaunchKernelGGL(fill, dim3(64), dim3(256), 0, 0, wb, (size_t)CB * KB, 0.1f);
  CK(hipMemset(ba, 0, CA * 4)); CK(hipMemset(bb, 0, CB * 4)); CK(hipMemset(y, 0, ny * 2));
  yv7::StemParams p; memset(&p, 0, sizeof(p));
  p.x = x; p.y = y; p.wa = wa; p.ba = ba; p.wb = wb; p.bb = bb;
  p.variant = argc > 1 ? atoi(argv[1]) : 0;
  p.B = B; p.H = H; p.W = W; p.yc = CB; p.yoff = 0; p.kpad_a = KA; p.kpad_b = KB; p.act_a = 1; p.act_b = 1; p.sa = 1;
  p.reorg = w6;
  hipEvent_t e0, e1; CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
  for (int i = 0; i < 3; ++i) CK(yv7::launch_stem(p, 1, 0));
  CK(hipDeviceSynchronize());
  CK(hipEventRecord(e0, 0));
  for (int i = 0; i < 20; ++i) CK(yv7::launch_stem(p, 1, 0));
  CK(hipEventRecord(e1, 0)); CK(hipEventSynchronize(e1));
  float ms; CK(hipEventElapsedTime(&ms, e0, e1)); ms /= 20;
  const double ha = w6 ? H / 2 : H;
  const double fl = 2.0 * B * ha * ha * CA * (w6 ? 108 : 27) + 2.0 * B * HB * WB * CB * 9 * CA;
  printf("stem%s bs%d %d variant %d: %.1f us  %.0f TF/s\n", w6 ? " w6" : "", B, H, p.variant, ms * 1e3, fl / ms / 1e9);
  return 0;
}
