// Microbenchmark of the fused 1x1 chain (not in the product): yolov7 layer 11 (1x1 256->256,
// SiLU) feeding the MP block's two 1x1 readers (256->128 and MP -> 256->128) as ONE launch, the 256-channel
// intermediate never leaving the CU.  Replaces three convs of cfg/deploy/yolov7.yaml:26-30
// (Conv = models/common.py:110-111, MP = common.py:30-36) at 160^2, bs 32.
//
// Block = 8 waves; a wave owns units of 32 pixels (two image rows x 16 columns) with all 256 input
// channels in registers as MFMA B operands.  W2 / W3 (128 x 256 each, k permuted for the chain) are
// resident in LDS; W1 streams through LDS in 16-channel chunks (8 KiB, one 16-byte load per thread,
// double-buffered, one barrier per chunk) shared by the block's waves.  Per chunk: y1 = W1c x (16 MFMAs);
// per chunk pair: mid = silu(y1) packed in registers is the B operand of y2 += W2 mid (16 MFMAs) and of
// y3 += W3 pool2x2(mid) (8 MFMAs).  Check: host fp32 reference on sampled units.
// Build: hipcc --offload-arch=gfx950 -O3 -ffp-contract=off scripts/chainbench.hip -o scripts/chainbench
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <vector>

typedef _Float16 h8 __attribute__((ext_vector_type(8)));
typedef _Float16 h4 __attribute__((ext_vector_type(4)));
typedef _Float16 h2 __attribute__((ext_vector_type(2)));
typedef float f4 __attribute__((ext_vector_type(4)));
typedef uint32_t u4 __attribute__((ext_vector_type(4)));
typedef uint32_t u2 __attribute__((ext_vector_type(2)));

constexpr int C = 256, CM = 256, CO = 128, NTH = 512;
constexpr int WROW = CM * 2;                       // bytes per resident weight row (256 k)
constexpr int W2OFF = 0, W3OFF = CO * WROW, W1OFF = 2 * CO * WROW;
constexpr int W1CH = 16 * C * 2;                   // one W1 chunk: 16 rows x 256 k = 8 KiB
constexpr int BOFF = W1OFF + 3 * W1CH;         // W1 ring: 2 buffers (register-staged) or 3 (DMA)
constexpr int LDS = BOFF + (CM + 2 * CO) * 4;      // 156,672 B

__device__ __forceinline__ float silu(float v) {
  return v * __builtin_amdgcn_rcpf(1.0f + __builtin_amdgcn_exp2f(-1.4426950408889634f * v));
}
__host__ inline float silu_h(float v) { return v / (1.0f + expf(-v)); }

// 16-byte slot of chunk q (0..31) of row r: XOR-swizzled over 16 slots (256 B)
__device__ __forceinline__ int slot(int r, int q) { return r * WROW + ((q ^ (r & 15)) << 4); }

__device__ __forceinline__ uint32_t pool2x2(uint32_t r0, uint32_t r1) {
  const h2 v = __builtin_elementwise_max(__builtin_bit_cast(h2, r0), __builtin_bit_cast(h2, r1));
  const int nb = __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, v), 0xB1, 0xF, 0xF, false);
  return __builtin_bit_cast(uint32_t, __builtin_elementwise_max(v, __builtin_bit_cast(h2, nb)));
}

// x [B][H][W][256], W1 [256][256], W2p / W3p [128][256] (k permuted), y2 [B][H][W][128], y3 [B][H/2][W/2][128]
// HOOK (attribution only, results then wrong): 1 x loaded for the first unit only, 2 no y2 / y3 MFMAs,
// 4 no output stores, 8 no W1 ring traffic and no barriers
// RPW: image rows per wave-unit (2: 8 waves per block; 4: 4 waves, one per SIMD, every weight fragment
// feeding twice the MFMAs)
template <bool DMA, int HOOK = 0, int RPW = 2>
__global__ __launch_bounds__(RPW == 2 ? 512 : 256, 1) void chain_kernel(const _Float16* __restrict__ x, const _Float16* __restrict__ W1,
                                                      const float* __restrict__ b1, const _Float16* __restrict__ W2p,
                                                      const float* __restrict__ b2, const _Float16* __restrict__ W3p,
                                                      const float* __restrict__ b3, _Float16* __restrict__ y2,
                                                      _Float16* __restrict__ y3, int B, int H, int W) {
  __shared__ __attribute__((aligned(16))) unsigned char smem[LDS];
  float* bl = reinterpret_cast<float*>(smem + BOFF);
  constexpr int NT = RPW == 2 ? 512 : 256, NW = NT / 64, WI = 8192 / NT;
  static_assert(DMA || RPW == 2, "the register-staged W1 ring is the 8-wave form only");
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, g = lane >> 4, li = lane & 15;
  // resident W2 / W3 (all loads first, then the LDS writes)
  {
    u4 v[WI];
#pragma unroll
    for (int t = 0; t < WI; ++t) {
      const int i = tid + t * NT;            // 0 .. 8191: 2 x 128 rows x 32 chunks
      const int m = i >> 12, r = (i >> 5) & 127, q = i & 31;
      const _Float16* src = (m ? W3p : W2p) + r * CM + q * 8;
      v[t] = *reinterpret_cast<const u4*>(src);
    }
#pragma unroll
    for (int t = 0; t < WI; ++t) {
      const int i = tid + t * NT;
      const int m = i >> 12, r = (i >> 5) & 127, q = i & 31;
      *reinterpret_cast<u4*>(smem + (m ? W3OFF : W2OFF) + slot(r, q)) = v[t];
    }
    for (int i = tid; i < CM + 2 * CO; i += NT) bl[i] = i < CM ? b1[i] : (i < CM + CO ? b2[i - CM] : b3[i - CM - CO]);
  }
  // W1 chunk c: thread tid moves row tid / 32, chunk tid % 32
  const int w1r = tid >> 5, w1q = tid & 31;
  auto w1load = [&](int c) { return *reinterpret_cast<const u4*>(W1 + (c * 16 + w1r) * C + w1q * 8); };
  auto w1store = [&](int buf, u4 v) { *reinterpret_cast<u4*>(smem + W1OFF + buf * W1CH + slot(w1r, w1q)) = v; };
  // DMA form: wave w's lane l moves row 2 w + l / 32, LDS slot l % 32 of a chunk, i.e. source chunk
  // (l % 32) ^ (row & 15) — the swizzle applied on the source side (the DMA writes 16 B per lane in lane order)
  const auto w1rs = __builtin_amdgcn_make_buffer_rsrc(const_cast<_Float16*>(W1), (short)0, CM * C * 2, 0x00020000);
  // (RPW 4: four waves, each moving pieces wave and wave + 4)
  auto w1dma = [&](int c, int b) __attribute__((always_inline)) {
#pragma unroll
    for (int pc = 0; pc < 8 / NW; ++pc) {
      const int piece = wave + pc * NW;
      const int dr = 2 * piece + (lane >> 5), dq = (lane & 31) ^ (dr & 15);
      __builtin_amdgcn_raw_ptr_buffer_load_lds(
          w1rs, (__attribute__((address_space(3))) void*)(smem + W1OFF + b * W1CH + piece * 1024), 16,
          (uint32_t)(((c * 16 + dr) * C + dq * 8) * 2), 0, 0, 0);
    }
  };
  if constexpr (DMA) {
    w1dma(0, 0);
    w1dma(1, 1);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  } else {
    w1store(0, w1load(0));
  }
  __syncthreads();
  int n = 0;   // W1 chunk sequence number (DMA ring position n % 3)

  const int segs = W / 16, rps = H / RPW;
  const int U = B * rps * segs;
  const int waves = gridDim.x * NW;
  const int nu = (U + waves - 1) / waves;       // every wave runs nu units (barriers are block-wide)
  const int gw = blockIdx.x * NW + wave;
  int buf = 0;
  u4 xs[RPW][8];
  for (int it = 0; it < nu; ++it) {
    const int u0 = gw + it * waves;
    const bool valid = u0 < U;
    const int u = valid ? u0 : 0;
    const int xs0 = (u % segs) * 16, y0 = ((u / segs) % rps) * RPW, b = u / (segs * rps);
    if ((HOOK & 1) && it > 0) goto have_x;
#pragma unroll
    for (int r = 0; r < RPW; ++r)
#pragma unroll
      for (int ks = 0; ks < 8; ++ks)
        xs[r][ks] = *reinterpret_cast<const u4*>(x + ((size_t)(b * H + y0 + r) * W + xs0 + li) * C + ks * 32 + g * 8);
  have_x:
    f4 acc2[8][RPW], acc3[8][RPW / 2];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const f4 bv2 = *reinterpret_cast<const f4*>(bl + CM + j * 16 + g * 4);
      const f4 bv3 = *reinterpret_cast<const f4*>(bl + CM + CO + j * 16 + g * 4);
#pragma unroll
      for (int r = 0; r < RPW; ++r) acc2[j][r] = bv2;
#pragma unroll
      for (int r = 0; r < RPW / 2; ++r) acc3[j][r] = bv3;
    }
    // one W1 chunk: y1 rows 16 c .. +15 for both pixel rows; the next chunk's load in flight meanwhile,
    // then its LDS write and the block barrier
    auto chunk = [&](int c, f4 (&a1)[RPW]) __attribute__((always_inline)) {
      u4 nxt;
      if constexpr (DMA && !(HOOK & 8)) w1dma((c + 2) & 15, (n + 2) % 3);   // two chunks ahead into the buffer read at n - 1
      else nxt = w1load((c + 1) & 15);      // the next chunk (the next unit's chunk 0 after c = 15)
      const unsigned char* w1b = smem + W1OFF + (DMA ? n % 3 : buf) * W1CH;
      const f4 bv1 = *reinterpret_cast<const f4*>(bl + c * 16 + g * 4);
#pragma unroll
      for (int r = 0; r < RPW; ++r) a1[r] = bv1;
#pragma unroll
      for (int ks = 0; ks < 8; ++ks) {
        const u4 wf = *reinterpret_cast<const u4*>(w1b + slot(li, ks * 4 + g));
#pragma unroll
        for (int r = 0; r < RPW; ++r)
          a1[r] = __builtin_amdgcn_mfma_f32_16x16x32_f16(__builtin_bit_cast(h8, wf), __builtin_bit_cast(h8, xs[r][ks]), a1[r], 0, 0, 0);
      }
      if constexpr (HOOK & 8) {
        ++n;
      } else if constexpr (DMA) {
        // chunk n + 1 (issued one step ago) has landed: younger VMEM ops are chunk n + 2's DMA only
        // (or, at a unit's first step, also this unit's X loads and the last unit's stores: waited too)
        if constexpr (NW == 8) asm volatile("s_waitcnt vmcnt(1)" ::: "memory");
        else asm volatile("s_waitcnt vmcnt(2)" ::: "memory");
        __builtin_amdgcn_s_barrier();   // raw: __syncthreads' fence would drain chunk n + 2's DMA too
        ++n;
      } else {
        w1store(buf ^ 1, nxt);
        __syncthreads();
        buf ^= 1;
      }
    };
#pragma unroll 1
    for (int s2 = 0; s2 < 8; ++s2) {
      f4 prev[RPW], a1[RPW];
      chunk(2 * s2, prev);
      chunk(2 * s2 + 1, a1);
      // mid channels 32 s2 + 4 g .. +3 (prev) and 32 s2 + 16 + 4 g .. +3 (a1): this lane's k values
      u4 mid[RPW];
#pragma unroll
      for (int r = 0; r < RPW; ++r) {
        h8 m;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          m[i] = (_Float16)silu(prev[r][i]);
          m[4 + i] = (_Float16)silu(a1[r][i]);
        }
        mid[r] = __builtin_bit_cast(u4, m);
      }
      u4 pm[RPW / 2];
#pragma unroll
      for (int h = 0; h < RPW / 2; ++h)
        pm[h] = u4{pool2x2(mid[2 * h].x, mid[2 * h + 1].x), pool2x2(mid[2 * h].y, mid[2 * h + 1].y),
                   pool2x2(mid[2 * h].z, mid[2 * h + 1].z), pool2x2(mid[2 * h].w, mid[2 * h + 1].w)};
      const int kq = s2 * 4 + g;                  // 16-byte chunk of the 32-channel k step s2
      if constexpr (HOOK & 2) {
        acc2[0][0][0] += __builtin_bit_cast(float, pm[0].x ^ mid[0].y ^ mid[1].z);
        continue;
      }
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const u4 w2f = *reinterpret_cast<const u4*>(smem + W2OFF + slot(j * 16 + li, kq));
        const u4 w3f = *reinterpret_cast<const u4*>(smem + W3OFF + slot(j * 16 + li, kq));
#pragma unroll
        for (int r = 0; r < RPW; ++r)
          acc2[j][r] = __builtin_amdgcn_mfma_f32_16x16x32_f16(__builtin_bit_cast(h8, w2f), __builtin_bit_cast(h8, mid[r]), acc2[j][r], 0, 0, 0);
#pragma unroll
        for (int h = 0; h < RPW / 2; ++h)
          acc3[j][h] = __builtin_amdgcn_mfma_f32_16x16x32_f16(__builtin_bit_cast(h8, w3f), __builtin_bit_cast(h8, pm[h]), acc3[j][h], 0, 0, 0);
      }
    }
    if (valid && !(HOOK & 4)) {
#pragma unroll
      for (int j = 0; j < 8; ++j)
#pragma unroll
        for (int r = 0; r < RPW; ++r) {
          h4 o;
#pragma unroll
          for (int i = 0; i < 4; ++i) o[i] = (_Float16)silu(acc2[j][r][i]);
          *reinterpret_cast<u2*>(y2 + ((size_t)(b * H + y0 + r) * W + xs0 + li) * CO + j * 16 + g * 4) = __builtin_bit_cast(u2, o);
        }
      if ((li & 1) == 0) {
#pragma unroll
        for (int j = 0; j < 8; ++j)
#pragma unroll
          for (int h = 0; h < RPW / 2; ++h) {
            h4 o;
#pragma unroll
            for (int i = 0; i < 4; ++i) o[i] = (_Float16)silu(acc3[j][h][i]);
            *reinterpret_cast<u2*>(y3 + ((size_t)(b * (H / 2) + y0 / 2 + h) * (W / 2) + (xs0 + li) / 2) * CO + j * 16 + g * 4) =
                __builtin_bit_cast(u2, o);
          }
      }
    }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // the ring's last DMAs (into the void of the next unit)
}

int main(int argc, char** argv) {
  const int B = argc > 1 ? atoi(argv[1]) : 32, H = 160, W = 160, iters = 20;
  srand(11);
  auto rnd = [] { return (float)rand() / (float)RAND_MAX * 2.0f - 1.0f; };
  const size_t nx = (size_t)B * H * W * C;
  std::vector<_Float16> x(nx), W1(CM * C), W2(CO * CM), W3(CO * CM), W2p(CO * CM), W3p(CO * CM);
  std::vector<float> b1(CM), b2(CO), b3(CO);
  for (auto& v : x) v = (_Float16)(rnd() * 2.0f);
  for (auto& v : W1) v = (_Float16)(rnd() * 0.08f);
  for (auto& v : W2) v = (_Float16)(rnd() * 0.08f);
  for (auto& v : W3) v = (_Float16)(rnd() * 0.08f);
  for (auto& v : b1) v = rnd() * 0.2f;
  for (auto& v : b2) v = rnd() * 0.2f;
  for (auto& v : b3) v = rnd() * 0.2f;
  // k permutation of the chain (scripts/chain_check.hip): logical k' = 32 s + 8 g + j <-> mid channel
  // 32 s + (j < 4 ? 4 g + j : 16 + 4 g + j - 4)
  for (int n = 0; n < CO; ++n)
    for (int kp = 0; kp < CM; ++kp) {
      const int s = kp / 32, g = (kp % 32) / 8, j = kp % 8;
      const int c = 32 * s + (j < 4 ? 4 * g + j : 16 + 4 * g + j - 4);
      W2p[n * CM + kp] = W2[n * CM + c];
      W3p[n * CM + kp] = W3[n * CM + c];
    }
  _Float16 *dx, *dW1, *dW2p, *dW3p, *dy2, *dy3;
  float *db1, *db2, *db3;
  const size_t ny2 = (size_t)B * H * W * CO, ny3 = (size_t)B * (H / 2) * (W / 2) * CO;
  if (hipMalloc(&dx, nx * 2) || hipMalloc(&dW1, W1.size() * 2) || hipMalloc(&dW2p, W2p.size() * 2) ||
      hipMalloc(&dW3p, W3p.size() * 2) || hipMalloc(&dy2, ny2 * 2) || hipMalloc(&dy3, ny3 * 2) ||
      hipMalloc(&db1, CM * 4) || hipMalloc(&db2, CO * 4) || hipMalloc(&db3, CO * 4))
    return 2;
  (void)hipMemcpy(dx, x.data(), nx * 2, hipMemcpyHostToDevice);
  (void)hipMemcpy(dW1, W1.data(), W1.size() * 2, hipMemcpyHostToDevice);
  (void)hipMemcpy(dW2p, W2p.data(), W2p.size() * 2, hipMemcpyHostToDevice);
  (void)hipMemcpy(dW3p, W3p.data(), W3p.size() * 2, hipMemcpyHostToDevice);
  (void)hipMemcpy(db1, b1.data(), CM * 4, hipMemcpyHostToDevice);
  (void)hipMemcpy(db2, b2.data(), CO * 4, hipMemcpyHostToDevice);
  (void)hipMemcpy(db3, b3.data(), CO * 4, hipMemcpyHostToDevice);
  int cus = 256;
  (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
  const int grid = cus;
  const bool dma = argc > 2 && argv[2][0] == 'd';
  const bool rpw4 = argc > 2 && argv[2][0] == '4';   // "4": the four-row, one-wave-per-SIMD form (LDS-DMA ring)
  const int hook = argc > 3 ? atoi(argv[3]) : 0;
  auto launch = [&] {
#define CB_L(D, HK) chain_kernel<D, HK><<<grid, NTH>>>(dx, dW1, db1, dW2p, db2, dW3p, db3, dy2, dy3, B, H, W)
    if (rpw4) chain_kernel<true, 0, 4><<<grid, 256>>>(dx, dW1, db1, dW2p, db2, dW3p, db3, dy2, dy3, B, H, W);
    else if (!dma) CB_L(false, 0);
    else if (hook == 1) CB_L(true, 1);
    else if (hook == 2) CB_L(true, 2);
    else if (hook == 4) CB_L(true, 4);
    else if (hook == 8) CB_L(true, 8);
    else if (hook == 15) CB_L(true, 15);
    else CB_L(true, 0);
#undef CB_L
  };
  (void)hipMemset(dy2, 0, ny2 * 2);
  (void)hipMemset(dy3, 0, ny3 * 2);
  launch();
  if (hipDeviceSynchronize() != hipSuccess) return 3;
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  (void)hipEventRecord(e0);
  for (int i = 0; i < iters; ++i) launch();
  (void)hipEventRecord(e1);
  if (hipEventSynchronize(e1) != hipSuccess) return 4;
  float ms = 0;
  (void)hipEventElapsedTime(&ms, e0, e1);
  std::vector<_Float16> y2(ny2), y3(ny3);
  (void)hipMemcpy(y2.data(), dy2, ny2 * 2, hipMemcpyDeviceToHost);
  (void)hipMemcpy(y3.data(), dy3, ny3 * 2, hipMemcpyDeviceToHost);
  // host reference on sampled 2x2 pixel blocks
  double md2 = 0, md3 = 0;
  int bad = 0;
  for (int smp = 0; smp < 64; ++smp) {
    const int b = rand() % B, py = (rand() % (H / 2)) * 2, px = (rand() % (W / 2)) * 2;
    float mid[4][CM];
    for (int q = 0; q < 4; ++q) {
      const _Float16* xp = &x[((size_t)(b * H + py + q / 2) * W + px + q % 2) * C];
      for (int m = 0; m < CM; ++m) {
        float s = b1[m];
        for (int k = 0; k < C; ++k) s += (float)W1[m * C + k] * (float)xp[k];
        mid[q][m] = (float)(_Float16)silu_h(s);
      }
    }
    for (int q = 0; q < 4; ++q)
      for (int n = 0; n < CO; ++n) {
        float s = b2[n];
        for (int m = 0; m < CM; ++m) s += (float)W2[n * CM + m] * mid[q][m];
        const float ref = silu_h(s), got = (float)y2[((size_t)(b * H + py + q / 2) * W + px + q % 2) * CO + n];
        const double d = fabs(ref - got);
        md2 = fmax(md2, d);
        bad += d > 4e-3 + 4e-3 * fabs(ref);
      }
    for (int n = 0; n < CO; ++n) {
      float s = b3[n];
      for (int m = 0; m < CM; ++m)
        s += (float)W3[n * CM + m] * fmaxf(fmaxf(mid[0][m], mid[1][m]), fmaxf(mid[2][m], mid[3][m]));
      const float ref = silu_h(s), got = (float)y3[((size_t)(b * (H / 2) + py / 2) * (W / 2) + px / 2) * CO + n];
      const double d = fabs(ref - got);
      md3 = fmax(md3, d);
      bad += d > 4e-3 + 4e-3 * fabs(ref);
    }
  }
  const double us = ms * 1000.0 / iters;
  const double bytes = (double)nx * 2 + (double)ny2 * 2 + (double)ny3 * 2;
  const double flops = 2.0 * B * H * W * ((double)C * CM + (double)CM * CO) + 2.0 * ny3 * CM;
  if (hook) printf("[hook %d] ", hook);
  printf("chainbench %s B=%d %dx%d: %.1f us per launch (%.2f TB/s of boundary bytes, %.0f TF/s); max |d| y2 %.3g y3 %.3g, "
         "%d outside tolerance %s\n",
         rpw4 ? "dma-4rows" : dma ? "dma" : "regs", B, H, W, us, bytes / us / 1e6, flops / us / 1e6, md2, md3, bad, bad ? "FAIL" : "OK");
  return (bad && !hook) ? 1 : 0;
}
