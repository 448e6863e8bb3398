// Dev microbenchmark: the fused Detect head conv (fp16 GEMM + sigmoid/decode epilogue) on the three
// yolov7 levels at bs 32, with the kernel's variant hooks: 0 = full, 90 = GEMM only, 91 = epilogue only.
// build: hipcc --offload-arch=gfx950 -O2 scripts/detbench.hip -I yolo-series_amd/csrc
//        -L yolo-series_amd/yv7 -lyv7 -Wl,-rpath,$PWD/yolo-series_amd/yv7 -o scripts/detbench
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>
#include "yv7_kernels.h"
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s line %d\n", hipGetErrorString(e), __LINE__); return 1; } } while (0)

int main(int argc, char** argv) {
  const int B = 32, na = 3, no = 85;
  struct L { int hw, cin; float stride; };
  std::vector<L> lv = {{80, 256, 8.f}, {40, 512, 16.f}, {20, 1024, 32.f}};
  const int nrows = na * (80 * 80 + 40 * 40 + 20 * 20);
  float *z, *best, *b; _Float16 *x, *w; void* zero;
  CK(hipMalloc(&z, (size_t)B * nrows * no * 4)); CK(hipMalloc(&best, (size_t)B * nrows * 16));
  CK(hipMalloc(&x, yv7::bordered_pixels(B, 80, 80) * 256 * 2)); CK(hipMalloc(&w, 256 * 1024 * 2));
  CK(hipMalloc(&b, 256 * 4)); CK(hipMalloc(&zero, 4096));
  {   // random operands (zeros would let the chip hold a higher clock than real data)
    const size_t nx = yv7::bordered_pixels(B, 80, 80) * 256, nw = 256 * 1024;
    std::vector<_Float16> hx(nx), hw(nw);
    uint32_t s = 12345u;
    for (auto& v : hx) { s = s * 1664525u + 1013904223u; v = (_Float16)(((s >> 8) & 0xffff) / 65536.0f - 0.5f); }
    for (auto& v : hw) { s = s * 1664525u + 1013904223u; v = (_Float16)((((s >> 8) & 0xffff) / 65536.0f - 0.5f) * 0.1f); }
    CK(hipMemcpy(x, hx.data(), nx * 2, hipMemcpyHostToDevice));
    CK(hipMemcpy(w, hw.data(), nw * 2, hipMemcpyHostToDevice));
  }
  CK(hipMemset(b, 0, 256 * 4)); CK(hipMemset(zero, 0, 4096));
  std::vector<int> variants = {0, 92, 97};
  if (argc > 1) {   // e.g. 0,92,97,98,99 (98: the persistent head without its sigmoid staging; the round-2
                    // tile-kernel hooks 90-96 were removed in round 4, see DESIGN §4.2 for their results)
    variants.clear();
    for (char* t = strtok(argv[1], ","); t; t = strtok(nullptr, ",")) variants.push_back(atoi(t));
  }
  int row_off = 0;
  hipEvent_t e0, e1; CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
  for (auto& l : lv) {
    yv7::ConvParams p; memset(&p, 0, sizeof(p));
    p.x = x; p.w = w; p.bias = b; p.zero = zero;
    p.B = B; p.H = p.W = p.Ho = p.Wo = l.hw; p.xc = p.cin = l.cin; p.k = 1; p.s = 1; p.pad = 0;
    p.cout = na * no; p.K = l.cin; p.kpad = l.cin; p.M = B * l.hw * l.hw;
    p.xbytes = (uint32_t)(yv7::bordered_pixels(B, l.hw, l.hw) * l.cin * 2);
    p.wbytes = (uint32_t)(256 * l.cin * 2);
    p.z = z; p.nrows = nrows; p.row_off = row_off; p.na = na; p.no = no; p.stride = l.stride;
    // the fragment-packed weight copy the plan makes for the register-weight head (conv_det_rw_kernel)
    void* wf = nullptr;
    const size_t wfb = yv7::frag_bytes(l.cin, 255, 1);
    CK(hipMalloc(&wf, wfb));
    CK(yv7::pack_frag(w, l.cin, l.cin, 255, 1, wf, 0));
    CK(hipDeviceSynchronize());
    p.wf = wf; p.wfbytes = (uint32_t)wfb;
    for (int a = 0; a < 6; ++a) p.anchor[a] = 10.f + a;
    for (int withbest = 0; withbest < 2; ++withbest) {
      p.best = withbest ? best : nullptr;
      printf("DET %4d->255 @%2d best=%d", l.cin, l.hw, withbest);
      for (int v : variants) {
        p.variant = v;
        for (int i = 0; i < 3; ++i) CK(yv7::launch_conv(1, p, true, 0));
        CK(hipDeviceSynchronize());
        CK(hipEventRecord(e0, 0));
        for (int i = 0; i < 20; ++i) CK(yv7::launch_conv(1, p, true, 0));
        CK(hipEventRecord(e1, 0)); CK(hipEventSynchronize(e1));
        float ms; CK(hipEventElapsedTime(&ms, e0, e1));
        printf(" | v%d %7.1f us", v, ms / 20 * 1e3);
      }
      printf("\n");
    }
    row_off += na * l.hw * l.hw;
  }
  return 0;
}
