// Checks the in-register MFMA chain that a fused 1x1 -> 1x1 kernel would use: the
// accumulators of y1 = W1 x (v_mfma_f32_16x16x32_f16; lane l holds rows 4 (l / 16) .. +3 of each
// 16-row block for column l % 16), after SiLU and the fp16 pack of two 16-row blocks, are used AS IS
// as the B operand (lane l: k = 8 (l / 16) .. +7, column l % 16) of y2 = W2 silu(y1), with W2's 32
// columns permuted at pack time: logical k' = 8 g + j <-> channel j < 4 ? 4 g + j : 16 + 4 g + j - 4.
// One wave, 32 mid channels, 16 pixels, K1 = 64, N2 = 16; host reference in fp32 with the same fp16
// rounding of the mid values.  Build: hipcc --offload-arch=gfx950 -O2 scripts/chain_check.hip -o chain_check
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <vector>

typedef _Float16 h8 __attribute__((ext_vector_type(8)));
typedef float f4 __attribute__((ext_vector_type(4)));

constexpr int K1 = 64, M1 = 32, P = 16, N2 = 16;

__device__ __host__ inline float silu(float v) { return v / (1.0f + expf(-v)); }

// W1 [M1][K1], x [K1][P] (k-major), W2p [N2][32] (columns permuted), y2 [N2][P]
__global__ void chain(const _Float16* W1, const _Float16* x, const _Float16* W2p, float* y2) {
  const int l = threadIdx.x, g = l / 16, li = l % 16;
  f4 acc[2] = {{0, 0, 0, 0}, {0, 0, 0, 0}};
  for (int ks = 0; ks < K1 / 32; ++ks) {
    h8 b;
    for (int j = 0; j < 8; ++j) b[j] = x[(ks * 32 + 8 * g + j) * P + li];
    for (int blk = 0; blk < 2; ++blk) {
      h8 a;
      for (int j = 0; j < 8; ++j) a[j] = W1[(blk * 16 + li) * K1 + ks * 32 + 8 * g + j];
      acc[blk] = __builtin_amdgcn_mfma_f32_16x16x32_f16(a, b, acc[blk], 0, 0, 0);
    }
  }
  // the chain: block 0's four values, then block 1's, as the eight k values of this lane
  h8 mid;
  for (int i = 0; i < 4; ++i) {
    mid[i] = (_Float16)silu(acc[0][i]);
    mid[4 + i] = (_Float16)silu(acc[1][i]);
  }
  h8 a2;
  for (int j = 0; j < 8; ++j) a2[j] = W2p[li * 32 + 8 * g + j];
  f4 o = {0, 0, 0, 0};
  o = __builtin_amdgcn_mfma_f32_16x16x32_f16(a2, mid, o, 0, 0, 0);
  for (int i = 0; i < 4; ++i) y2[(4 * g + i) * P + li] = o[i];
}

int main(int argc, char** argv) {
  // argv[1] == "identity": W2 packed unpermuted (negative control: must FAIL)
  const bool identity = argc > 1;
  srand(7);
  auto rnd = [] { return (float)rand() / (float)RAND_MAX * 2.0f - 1.0f; };
  std::vector<_Float16> W1(M1 * K1), x(K1 * P), W2(N2 * 32), W2p(N2 * 32);
  for (auto& v : W1) v = (_Float16)(rnd() * 0.25f);
  for (auto& v : x) v = (_Float16)rnd();
  for (auto& v : W2) v = (_Float16)(rnd() * 0.25f);
  for (int n = 0; n < N2; ++n)
    for (int kp = 0; kp < 32; ++kp) {
      const int g = kp / 8, j = kp % 8;
      const int c = identity ? kp : (j < 4 ? 4 * g + j : 16 + 4 * g + (j - 4));
      W2p[n * 32 + kp] = W2[n * 32 + c];
    }
  // host reference
  std::vector<float> mid(M1 * P), ref(N2 * P);
  for (int m = 0; m < M1; ++m)
    for (int p = 0; p < P; ++p) {
      float s = 0;
      for (int k = 0; k < K1; ++k) s += (float)W1[m * K1 + k] * (float)x[k * P + p];
      mid[m * P + p] = (float)(_Float16)silu(s);
    }
  for (int n = 0; n < N2; ++n)
    for (int p = 0; p < P; ++p) {
      float s = 0;
      for (int c = 0; c < 32; ++c) s += (float)W2[n * 32 + c] * mid[c * P + p];
      ref[n * P + p] = s;
    }
  _Float16 *dW1, *dx, *dW2p;
  float* dy;
  if (hipMalloc(&dW1, W1.size() * 2) || hipMalloc(&dx, x.size() * 2) || hipMalloc(&dW2p, W2p.size() * 2) ||
      hipMalloc(&dy, N2 * P * 4))
    return 2;
  hipMemcpy(dW1, W1.data(), W1.size() * 2, hipMemcpyHostToDevice);
  hipMemcpy(dx, x.data(), x.size() * 2, hipMemcpyHostToDevice);
  hipMemcpy(dW2p, W2p.data(), W2p.size() * 2, hipMemcpyHostToDevice);
  chain<<<1, 64>>>(dW1, dx, dW2p, dy);
  std::vector<float> y(N2 * P);
  if (hipMemcpy(y.data(), dy, y.size() * 4, hipMemcpyDeviceToHost) != hipSuccess) return 3;
  float md = 0, mr = 0;
  for (int i = 0; i < N2 * P; ++i) {
    md = fmaxf(md, fabsf(y[i] - ref[i]));
    mr = fmaxf(mr, fabsf(ref[i]));
  }
  // fp16 mid values may round differently where the fp32 sums differ in the last bits (summation
  // order): a few fp16 ulps of one mid value times |W2| <= 0.25
  const bool ok = md <= 2e-3f * fmaxf(1.0f, mr);
  printf("chain_check: max |gpu - ref| %.3g (max |ref| %.3g) %s\n", md, mr, ok ? "OK" : "FAIL");
  return ok ? 0 : 1;
}
