// Batched non_max_suppression on gfx950 — the semantics of utils/general.py:628-720 with the
// torchvision.ops.nms call (general.py:704) restated as a blocked greedy scan.
//
// Pipeline (all images of the batch in one launch per stage, no host sync):
//   1 nms_rows     a lane per anchor row for obj > conf (:637,:653), then a wave per surviving row:
//                  conf = cls*obj (:669-673),
//                  single-label first-max argmax (:683-684) or multi-label class mask (:680-681),
//                  optional class filter (:687-688) -> per-row candidate count (+best conf/cls)
//   2 nms_scan     per-image exclusive scan of the counts -> stable row-order offsets
//   3 nms_write    candidate records {xyxy (:676, xywh2xyxy :275-282), conf, cls, row} in the
//                  reference's candidate order (row-major, classes ascending)
//   4 nms_sort     per-image sort by (score desc, candidate index asc) == torchvision's stable
//                  descending sort; bitonic in LDS up to 16384 candidates, in global memory above;
//                  the first max_nms (:698-699) go on
//   5 nms_greedy   blocked greedy NMS on class-offset boxes (:702-703, max_wh 4096): per block of 64
//                  sorted candidates the workgroup builds the 64 x 64 "i suppresses j" bitmask, one
//                  wave resolves it with bit operations, the workgroup then strikes later candidates that
//                  a box kept in that block overlaps (IoU > thr); stops at max_det kept (:705-706).
// The single-label call without a class filter (detect.py's defaults, the serving path) takes a
// one-launch fast path instead (nms_fast below: compaction, register bitonic sort and a lazy greedy
// scan per image that stops once max_det boxes are kept).
// IoU arithmetic is torchvision's: area=(x2-x1)*(y2-y1), inter=max(0,.)*max(0,.),
// inter / (area_i + area_j - inter) > thr, all fp32; this file is built with -ffp-contract=off.
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace yv7 {

namespace {

constexpr int NT = 256;
constexpr int SORT_T = 1024;
constexpr int LDS_SORT_MAX = 16384;
constexpr int MAX_WH = 4096;

struct Cand {
  float x1, y1, x2, y2, conf;
  int cls, row, pad;
};

struct NmsArgs {
  const float* z;
  int B, N, no, nc;
  float conf, iou;
  int multi, agnostic, per_class;  // per_class: class-aware IoU on raw boxes (EfficientNMS) instead of offsets
  const int32_t* classes;
  int ncls;
  int max_det, max_nms;
  size_t cap;   // candidate capacity per image
  size_t pcap;  // pow2 >= cap: per-image stride of the global sort keys
  // workspace
  int* cnt;         // [B][N]
  int* offs;        // [B][N]
  float* bconf;     // [B][N] single-label best conf
  int* bcls;        // [B][N]
  int* ncand;       // [B]
  Cand* cand;       // [B][cap]
  uint64_t* keys;   // [B][pow2(cap)]
  int* order;       // [B][max_nms]
  float4* sbox;     // [B][max_nms] offset boxes in sorted order
  float* sarea;     // [B][max_nms]
  // outputs
  float* det;       // [B][max_det][6]
  int64_t* src_row; // [B][max_det]
  int32_t* count;   // [B]
};

__device__ __forceinline__ bool class_ok(const NmsArgs& a, int c) {
  if (!a.classes) return true;
  for (int i = 0; i < a.ncls; ++i)
    if (a.classes[i] == c) return true;
  return false;
}

// Stage 1: a wave takes 64 rows at a time.  Each lane gathers one row's objectness; the rows above
// conf (a few per 64) are then scored one after the other by the whole wave, lanes holding classes
// c and c + 64, so the wave pays one memory latency per candidate row instead of one per row.
__global__ __launch_bounds__(NT) void nms_rows(const NmsArgs a) {
  const int b = blockIdx.y;
  const int lane = threadIdx.x & 63;
  const int wave = (blockIdx.x * NT + threadIdx.x) >> 6;
  const int nwaves = (gridDim.x * NT) >> 6;
  const float* zb = a.z + (size_t)b * a.N * a.no;
  for (int r0 = wave * 64; r0 < a.N; r0 += nwaves * 64) {
    const int myrow = r0 + lane;
    const float myobj = myrow < a.N ? zb[(size_t)myrow * a.no + 4] : 0.f;
    int mycnt = 0;
    float mybest = 0.f;
    int mycls = 0;
    uint64_t pass = __ballot(myrow < a.N && myobj > a.conf);
    while (pass) {
      const int k = __ffsll((long long)pass) - 1;
      pass &= pass - 1;
      const int row = r0 + k;
      const float* zr = zb + (size_t)row * a.no;
      const float obj = __shfl(myobj, k);
      const int c0 = lane, c1 = lane + 64;
      float v0 = -1.f, v1 = -1.f;
      if (a.nc == 1) {
        v0 = (c0 == 0) ? obj : -1.f;  // nc == 1: conf = obj (:669-670)
      } else {
        if (c0 < a.nc) v0 = zr[5 + c0] * obj;
        if (c1 < a.nc) v1 = zr[5 + c1] * obj;
      }
      int cnt;
      float best = 0.f;
      int bc = 0;
      if (a.multi) {
        const bool p0 = c0 < a.nc && v0 > a.conf && class_ok(a, c0);
        const bool p1 = c1 < a.nc && v1 > a.conf && class_ok(a, c1);
        cnt = __popcll(__ballot(p0)) + __popcll(__ballot(p1));
      } else {
        // first max over classes: strict > keeps the lower class index on ties
        float v = v0;
        int c = c0;
        if (c1 < a.nc && v1 > v0) { v = v1; c = c1; }
        if (c0 >= a.nc) { v = -2.f; c = 1 << 30; }
        for (int off = 32; off > 0; off >>= 1) {
          const float ov = __shfl_xor(v, off);
          const int oc = __shfl_xor(c, off);
          if (ov > v || (ov == v && oc < c)) { v = ov; c = oc; }
        }
        best = v;
        bc = c;
        cnt = (v > a.conf && class_ok(a, c)) ? 1 : 0;
      }
      if (lane == k) {
        mycnt = cnt;
        mybest = best;
        mycls = bc;
      }
    }
    if (myrow < a.N) {
      const size_t i = (size_t)b * a.N + myrow;
      a.cnt[i] = mycnt;
      if (!a.multi) {
        a.bconf[i] = mybest;
        a.bcls[i] = mycls;
      }
    }
  }
}

// yv7_row_best (include/yv7.h): the head epilogue's per-row scores.
struct RowBest {
  float obj, conf;
  int cls, reserved;
};

// Stage 1 from row scores (single-label, no class filter): a 16-byte read per row instead of z.
__global__ __launch_bounds__(NT) void nms_rows_from_best(const NmsArgs a, const RowBest* __restrict__ rb) {
  const int b = blockIdx.y;
  for (int row = blockIdx.x * NT + threadIdx.x; row < a.N; row += gridDim.x * NT) {
    const size_t i = (size_t)b * a.N + row;
    const RowBest r = rb[i];
    const bool c = r.obj > a.conf && r.conf > a.conf;
    a.cnt[i] = c ? 1 : 0;
    a.bconf[i] = c ? r.conf : 0.f;
    a.bcls[i] = c ? r.cls : 0;
  }
}

// Row scores from z (for plans whose head kernel does not write them): a wave per 64 rows, every
// row scored (the threshold is not known yet), classes c and c + 64 per lane.
__global__ __launch_bounds__(NT) void row_best_kernel(const float* __restrict__ z, int N, int no, RowBest* __restrict__ out) {
  const int b = blockIdx.y;
  const int lane = threadIdx.x & 63;
  const int wave = (blockIdx.x * NT + threadIdx.x) >> 6;
  const int nwaves = (gridDim.x * NT) >> 6;
  const int nc = no - 5;
  for (int row = wave; row < N; row += nwaves) {
    const float* zr = z + ((size_t)b * N + row) * no;
    const float obj = zr[4];
    float v = -2.f;
    int c = 1 << 30;
    if (nc == 1) {
      if (lane == 0) { v = obj; c = 0; }
    } else {
      if (lane < nc) { v = zr[5 + lane] * obj; c = lane; }
      if (lane + 64 < nc) {
        const float v1 = zr[5 + lane + 64] * obj;
        if (v1 > v) { v = v1; c = lane + 64; }
      }
    }
    for (int off = 32; off > 0; off >>= 1) {
      const float ov = __shfl_xor(v, off);
      const int oc = __shfl_xor(c, off);
      if (ov > v || (ov == v && oc < c)) { v = ov; c = oc; }
    }
    if (lane == 0) out[(size_t)b * N + row] = RowBest{obj, v, c, 0};
  }
}

// Stage 2: per-image exclusive scan (one workgroup of SORT_T threads per image): each thread scans a
// contiguous run of rows serially, one workgroup-wide scan joins the runs — a single pass.
__global__ __launch_bounds__(SORT_T) void nms_scan(const NmsArgs a) {
  const int b = blockIdx.x;
  __shared__ int wsum[SORT_T / 64];
  const int* cnt = a.cnt + (size_t)b * a.N;
  int* offs = a.offs + (size_t)b * a.N;
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int per = (a.N + SORT_T - 1) / SORT_T;
  const int r0 = threadIdx.x * per, r1 = r0 + per < a.N ? r0 + per : a.N;
  int tot = 0;
  for (int r = r0; r < r1; ++r) tot += cnt[r];
  int s = tot;  // inclusive wave scan of the run totals
  for (int off = 1; off < 64; off <<= 1) {
    const int t = __shfl_up(s, off);
    if (lane >= off) s += t;
  }
  if (lane == 63) wsum[wv] = s;
  __syncthreads();
  int pre = 0;
  for (int k = 0; k < wv; ++k) pre += wsum[k];
  int run = pre + s - tot;
  for (int r = r0; r < r1; ++r) {
    const int v = cnt[r];
    offs[r] = run;
    run += v;
  }
  if (threadIdx.x == SORT_T - 1) a.ncand[b] = pre + s;
}

// Stage 3: write candidate records in reference order.  Single-label: a lane per row; multi-label:
// a wave per row (its classes across lanes).
__global__ __launch_bounds__(NT) void nms_write(const NmsArgs a) {
  const int b = blockIdx.y;
  const int lane = threadIdx.x & 63;
  if (!a.multi) {
    for (int row = blockIdx.x * NT + threadIdx.x; row < a.N; row += gridDim.x * NT) {
      const size_t ri = (size_t)b * a.N + row;
      if (a.cnt[ri] == 0) continue;
      const float* zr = a.z + ri * a.no;
      const float cx = zr[0], cy = zr[1], w = zr[2], h = zr[3];
      Cand c;
      c.x1 = cx - w / 2.0f;  // xywh2xyxy (general.py:275-282)
      c.y1 = cy - h / 2.0f;
      c.x2 = cx + w / 2.0f;
      c.y2 = cy + h / 2.0f;
      c.conf = a.bconf[ri];
      c.cls = a.bcls[ri];
      c.row = row;
      c.pad = 0;
      a.cand[(size_t)b * a.cap + a.offs[ri]] = c;
    }
    return;
  }
  const int wave = (blockIdx.x * NT + threadIdx.x) >> 6;
  const int nwaves = (gridDim.x * NT) >> 6;
  for (int row = wave; row < a.N; row += nwaves) {
    const size_t ri = (size_t)b * a.N + row;
    const int cnt = a.cnt[ri];
    if (cnt == 0) continue;
    const float* zr = a.z + ri * a.no;
    const float cx = zr[0], cy = zr[1], w = zr[2], h = zr[3];
    Cand c;
    c.x1 = cx - w / 2.0f;  // xywh2xyxy (general.py:275-282)
    c.y1 = cy - h / 2.0f;
    c.x2 = cx + w / 2.0f;
    c.y2 = cy + h / 2.0f;
    c.row = row;
    c.pad = 0;
    Cand* out = a.cand + (size_t)b * a.cap + a.offs[ri];
    {
      const float obj = zr[4];
      const int c0 = lane, c1 = lane + 64;
      float v0 = -1.f, v1 = -1.f;
      if (a.nc == 1) {
        v0 = (c0 == 0) ? obj : -1.f;
      } else {
        if (c0 < a.nc) v0 = zr[5 + c0] * obj;
        if (c1 < a.nc) v1 = zr[5 + c1] * obj;
      }
      const bool p0 = c0 < a.nc && v0 > a.conf && class_ok(a, c0);
      const bool p1 = c1 < a.nc && v1 > a.conf && class_ok(a, c1);
      const uint64_t m0 = __ballot(p0), m1 = __ballot(p1);
      const uint64_t below = (lane == 0) ? 0ull : (~0ull >> (64 - lane));
      if (p0) {
        Cand d = c;
        d.conf = v0;
        d.cls = c0;
        out[__popcll(m0 & below)] = d;
      }
      if (p1) {
        Cand d = c;
        d.conf = v1;
        d.cls = c1;
        out[__popcll(m0) + __popcll(m1 & below)] = d;
      }
    }
  }
}

__device__ __forceinline__ uint64_t sort_key(float conf, int idx) {
  // conf > conf_thres >= 0 here, so the fp32 bit pattern orders like the value.
  return ((uint64_t)(~__float_as_uint(conf)) << 32) | (uint32_t)idx;
}

// Stage 4: per-image sort -> order[] of the first min(n, max_nms) candidates.
template <typename K>
__device__ __forceinline__ void bitonic_sort(K* keys, const Cand* cand, int n, int P, int* order, int keep) {
  for (int i = threadIdx.x; i < P; i += SORT_T) keys[i] = i < n ? sort_key(cand[i].conf, i) : ~0ull;
  __syncthreads();
  for (int k = 2; k <= P; k <<= 1) {
    for (int j = k >> 1; j > 0; j >>= 1) {
      for (int i = threadIdx.x; i < P; i += SORT_T) {
        const int ixj = i ^ j;
        if (ixj > i) {
          const uint64_t ki = keys[i], kj = keys[ixj];
          const bool up = (i & k) == 0;
          if ((ki > kj) == up) {
            keys[i] = kj;
            keys[ixj] = ki;
          }
        }
      }
      __syncthreads();
    }
  }
  for (int i = threadIdx.x; i < keep; i += SORT_T) order[i] = (int)(uint32_t)keys[i];
}

__global__ __launch_bounds__(SORT_T) void nms_sort(const NmsArgs a) {
  const int b = blockIdx.x;
  const int n = a.ncand[b];
  const Cand* cand = a.cand + (size_t)b * a.cap;
  int* order = a.order + (size_t)b * a.max_nms;
  const int keep = n < a.max_nms ? n : a.max_nms;
  if (n == 0) return;
  int P = 1;
  while (P < n) P <<= 1;
  extern __shared__ __attribute__((aligned(16))) uint64_t skeys[];
  // two instantiations of the network: a pointer that may be LDS or global would compile to flat
  // accesses (vector-memory latency on every LDS step)
  if (P <= LDS_SORT_MAX)
    bitonic_sort(skeys, cand, n, P, order, keep);
  else
    bitonic_sort(a.keys + (size_t)b * a.pcap, cand, n, P, order, keep);
}

__device__ __forceinline__ bool iou_gt(const float4 bi, float ai, const float4 bj, float aj, float thr) {
  // torchvision nms: i is the kept box
  const float xx1 = fmaxf(bi.x, bj.x), yy1 = fmaxf(bi.y, bj.y);
  const float xx2 = fminf(bi.z, bj.z), yy2 = fminf(bi.w, bj.w);
  const float w = fmaxf(0.0f, xx2 - xx1), h = fmaxf(0.0f, yy2 - yy1);
  const float inter = w * h;
  return inter / (ai + aj - inter) > thr;
}

// Stage 5: blocked greedy NMS, one workgroup per image.
__global__ __launch_bounds__(SORT_T) void nms_greedy(const NmsArgs a) {
  const int b = blockIdx.x;
  const int n0 = a.ncand[b];
  const int n = n0 < a.max_nms ? n0 : a.max_nms;
  const Cand* cand = a.cand + (size_t)b * a.cap;
  const int* order = a.order + (size_t)b * a.max_nms;
  float4* sbox = a.sbox + (size_t)b * a.max_nms;
  float* sarea = a.sarea + (size_t)b * a.max_nms;
  extern __shared__ __attribute__((aligned(16))) unsigned char gsm[];
  uint32_t* removed = reinterpret_cast<uint32_t*>(gsm);            // [max_nms/32 + 2]
  const int nwords = (n + 31) / 32 + 2;
  float4* kbox = reinterpret_cast<float4*>(gsm + ((nwords * 4 + 15) / 16) * 16);
  float* karea = reinterpret_cast<float*>(kbox + 64);
  int* kcls = reinterpret_cast<int*>(karea + 64);
  __shared__ int nk_blk, total;
  __shared__ uint64_t sup[64];

  // gather boxes in sorted order (class-offset unless agnostic / per-class)
  for (int i = threadIdx.x; i < n; i += SORT_T) {
    const Cand c = cand[order[i]];
    const float off = (a.agnostic || a.per_class) ? 0.0f : (float)c.cls * (float)MAX_WH;
    float4 bx;
    bx.x = c.x1 + off;
    bx.y = c.y1 + off;
    bx.z = c.x2 + off;
    bx.w = c.y2 + off;
    sbox[i] = bx;
    sarea[i] = (bx.z - bx.x) * (bx.w - bx.y);
  }
  for (int i = threadIdx.x; i < nwords; i += SORT_T) removed[i] = 0u;
  if (threadIdx.x == 0) total = 0;
  __syncthreads();

  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  constexpr int NW = SORT_T / 64;
  for (int base = 0; base < n; base += 64) {
    // (a) every wave: for its rows i of this 64-candidate block, the 64-bit mask of later block
    //     members j that i would suppress (IoU > thr, same class when per_class) -> sup[i] in LDS
    {
      const int j = base + lane;
      const bool valid = j < n;
      float4 bj = make_float4(0.f, 0.f, 0.f, 0.f);
      float aj = 0.f;
      int cj = -1;
      if (valid) {
        bj = sbox[j];
        aj = sarea[j];
        if (a.per_class) cj = cand[order[j]].cls;
      }
#pragma unroll
      for (int q = 0; q < 64 / NW; ++q) {
        const int i = wv * (64 / NW) + q;
        const int ig = base + i;
        bool hit = false;
        if (ig < n && valid && lane > i) {
          const float4 bi = sbox[ig];
          const float ai = sarea[ig];
          const int ci = a.per_class ? cand[order[ig]].cls : -1;
          hit = (!a.per_class || ci == cj) && iou_gt(bi, ai, bj, aj, a.iou);
        }
        const uint64_t m = __ballot(hit);
        if (lane == 0) sup[i] = m;
      }
    }
    __syncthreads();
    // (b) wave 0 resolves the block with bit operations: walk the alive candidates in sorted order;
    //     each one still alive is kept and removes the later members it suppresses
    if (threadIdx.x < 64) {
      const int j = base + lane;
      const bool valid = j < n;
      float4 bj = make_float4(0.f, 0.f, 0.f, 0.f);
      float aj = 0.f;
      int cj = -1;
      if (valid) {
        bj = sbox[j];
        aj = sarea[j];
        if (a.per_class) cj = cand[order[j]].cls;
      }
      const bool rem = !valid || ((removed[j >> 5] >> (j & 31)) & 1u);
      const uint64_t my_sup = sup[lane];
      uint64_t alive = __ballot(!rem);
      uint64_t kept = 0;
      while (alive) {
        const int i = __ffsll((long long)alive) - 1;
        kept |= 1ull << i;
        alive &= ~__shfl(my_sup, i) & ~(1ull << i);
      }
      const int nk = __popcll(kept);
      const bool mine = (kept >> lane) & 1ull;
      const int rank = __popcll(kept & ((lane == 0) ? 0ull : (~0ull >> (64 - lane))));
      if (mine) {
        kbox[rank] = bj;
        karea[rank] = aj;
        kcls[rank] = cj;
        const int di = total + rank;
        if (di < a.max_det) {
          const Cand c = cand[order[base + lane]];
          float* d = a.det + ((size_t)b * a.max_det + di) * 6;
          d[0] = c.x1;
          d[1] = c.y1;
          d[2] = c.x2;
          d[3] = c.y2;
          d[4] = c.conf;
          d[5] = (float)c.cls;
          a.src_row[(size_t)b * a.max_det + di] = c.row;
        }
      }
      if (lane == 0) nk_blk = nk;
    }
    __syncthreads();
    const int nk = nk_blk;
    if (threadIdx.x == 0) total += nk;
    __syncthreads();
    if (total >= a.max_det) break;
    // strike later candidates overlapped by a box kept in this block: one candidate per lane, each
    // wave owns whole 64-candidate chunks (two bitmap words), so no atomics are needed
    if (nk > 0) {
      for (int c0 = base + 64 + wv * 64; c0 < n; c0 += (SORT_T / 64) * 64) {
        const int j = c0 + lane;
        bool hit = false;
        if (j < n && !((removed[j >> 5] >> (j & 31)) & 1u)) {
          const float4 bj = sbox[j];
          const float aj = sarea[j];
          const int cj = a.per_class ? cand[order[j]].cls : -1;
          for (int t = 0; t < nk && !hit; ++t) {
            if (a.per_class && kcls[t] != cj) continue;
            hit = iou_gt(kbox[t], karea[t], bj, aj, a.iou);
          }
        }
        const uint64_t hm = __ballot(hit);
        if (lane == 0) removed[c0 >> 5] |= (uint32_t)hm;
        if (lane == 32) removed[(c0 >> 5) + 1] |= (uint32_t)(hm >> 32);
      }
    }
    __syncthreads();
  }
  if (threadIdx.x == 0) a.count[b] = total < a.max_det ? total : a.max_det;
}

// ---------------------------------------------------------------------------------------------
// Fast path: single-label, no class filter (detect.py's and the bench's call, general.py:683-684).
// ONE launch, one 1024-thread workgroup per image:
//   1. compaction: the image's yv7_row_best records (a 16-byte read per anchor row) -> rows with
//      obj > conf and best obj*cls > conf (:637/:653, :684) append a 64-bit sort key
//      ((~conf bits) << 32 | row) through an LDS counter; list order is arbitrary — the key carries
//      the reference's tie order (the row index), so sorting restores it exactly
//   2. sort: bitonic over P = pow2 >= max(n, 1024) keys held in registers (P / 1024 per thread):
//      partners within a wave by lane shuffles, across waves through LDS, across a thread's own
//      keys in registers — the barriers are only the cross-wave stages' (14 of 66 at P = 2048)
//   3. LAZY greedy in sorted order, 64 candidates at a time: each candidate against every box already
//      kept (IoU > thr, class-offset boxes :702-703) and against the earlier members of its block
//      (64 x 64 mask, resolved by one wave with bit operations).  A candidate survives iff no earlier
//      KEPT box overlaps it — torchvision's greedy definition — so only the sorted prefix that reaches
//      max_det (:705-706) is touched (for typical frames about max_det candidates)
//   4. the output's padding rows (det 0, src_row -1)
// More than FAST_LDS_KEYS candidates (rare in single-label mode) sort in global memory instead.
struct FastArgs {
  const float* z;
  const RowBest* rb;
  int B, N, no;
  float conf, iou;
  int agnostic, max_det, max_nms;
  size_t kcap;        // per-image global key capacity (pow2 >= N)
  uint64_t* keys;     // [B][kcap] (large candidate lists only)
  float* det;
  int64_t* src_row;
  int32_t* count;
};

constexpr int FAST_MAX_DET = 1024;   // kept-box list in LDS
constexpr int FAST_LDS_KEYS = 8192;  // register / LDS sort capacity

__device__ __forceinline__ uint64_t shfl_xor64(uint64_t v, int m) {
  const int lo = __shfl_xor((int)(uint32_t)v, m, 64), hi = __shfl_xor((int)(uint32_t)(v >> 32), m, 64);
  return ((uint64_t)(uint32_t)hi << 32) | (uint32_t)lo;
}

// Bitonic sort of E * 1024 keys, element i = e * 1024 + tid in r[e]; xl: LDS exchange buffer.
template <int E>
__device__ __forceinline__ void reg_bitonic(uint64_t (&r)[E], uint64_t* xl, int tid) {
  constexpr int P = E * SORT_T;
  const int lane = tid & 63;
  for (int k = 2; k <= P; k <<= 1) {
    for (int j = k >> 1; j > 0; j >>= 1) {
      if (j >= SORT_T) {            // partner in this thread: slot e ^ (j / 1024)
        const int je = j / SORT_T;
#pragma unroll
        for (int e = 0; e < E; ++e) {
          if (e & je) continue;
          const int i = e * SORT_T + tid;
          const bool asc = (i & k) == 0;
          const uint64_t a = r[e], c = r[e | je];
          const bool sw = (a > c) == asc;
          r[e] = sw ? c : a;
          r[e | je] = sw ? a : c;
        }
      } else if (j >= 64) {         // partner in another wave: through LDS
#pragma unroll
        for (int e = 0; e < E; ++e) xl[e * SORT_T + tid] = r[e];
        __syncthreads();
#pragma unroll
        for (int e = 0; e < E; ++e) {
          const int i = e * SORT_T + tid;
          const uint64_t p = xl[i ^ j];
          const bool keep_min = ((i & k) == 0) == ((i & j) == 0);
          r[e] = keep_min ? (p < r[e] ? p : r[e]) : (p > r[e] ? p : r[e]);
        }
        __syncthreads();
      } else {                      // partner in this wave
#pragma unroll
        for (int e = 0; e < E; ++e) {
          const int i = e * SORT_T + tid;
          const uint64_t p = shfl_xor64(r[e], j);
          const bool keep_min = ((i & k) == 0) == ((lane & j) == 0);
          r[e] = keep_min ? (p < r[e] ? p : r[e]) : (p > r[e] ? p : r[e]);
        }
      }
    }
  }
#pragma unroll
  for (int e = 0; e < E; ++e) xl[e * SORT_T + tid] = r[e];
  __syncthreads();
}

template <int E>
__device__ __forceinline__ void sort_lds(uint64_t* skeys, int n, int tid) {
  uint64_t r[E];
#pragma unroll
  for (int e = 0; e < E; ++e) {
    const int i = e * SORT_T + tid;
    r[e] = i < n ? skeys[i] : ~0ull;
  }
  __syncthreads();
  reg_bitonic<E>(r, skeys, tid);
}

__global__ __launch_bounds__(SORT_T) void nms_fast(const FastArgs a) {
  const int b = blockIdx.x;
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  constexpr int NW = SORT_T / 64;
  extern __shared__ __attribute__((aligned(16))) unsigned char fsm[];
  uint64_t* skeys = reinterpret_cast<uint64_t*>(fsm);                              // [FAST_LDS_KEYS]
  float4* kbox = reinterpret_cast<float4*>(fsm + FAST_LDS_KEYS * 8);                // kept boxes (offset)
  float* karea = reinterpret_cast<float*>(kbox + FAST_MAX_DET);
  __shared__ float4 bbox[64], braw[64];
  __shared__ float barea[64], bconf[64];
  __shared__ int bcls[64], brow[64];
  __shared__ uint64_t sup[64];
  __shared__ unsigned char pre[64];
  __shared__ int total_s, n_s;

  // ---- 1. compaction
  if (tid == 0) n_s = 0;
  __syncthreads();
  const RowBest* rb = a.rb + (size_t)b * a.N;
  uint64_t* gkeys = a.keys + (size_t)b * a.kcap;
  // a wave's rows r0 + u * NW * 64 + lane, U record loads in flight before any is used
  constexpr int U = 8;
  for (int r0 = wv * 64; r0 < a.N; r0 += U * NW * 64) {
    RowBest rr[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int row = r0 + u * NW * 64 + lane;
      rr[u] = row < a.N ? rb[row] : RowBest{0.f, 0.f, 0, 0};
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int row = r0 + u * NW * 64 + lane;
      const bool c = row < a.N && rr[u].obj > a.conf && rr[u].conf > a.conf;
      const uint64_t m = __ballot(c);
      if (!m) continue;
      int base = 0;
      if (lane == 0) base = atomicAdd(&n_s, __popcll(m));
      base = __shfl(base, 0);
      if (c) {
        const int k = base + __popcll(m & ((lane == 0) ? 0ull : (~0ull >> (64 - lane))));
        const uint64_t key = ((uint64_t)(~__float_as_uint(rr[u].conf)) << 32) | (uint32_t)row;
        // the first FAST_LDS_KEYS keys go to LDS only; the global list is written past them and
        // completed from LDS below only when the list outgrows the LDS sort
        if (k < FAST_LDS_KEYS) skeys[k] = key;
        else gkeys[k] = key;
      }
    }
  }
  __syncthreads();
  const int n = n_s;
  // ---- 2. sort: keys ascending = (conf descending, row ascending), torchvision's stable order
  const uint64_t* s = skeys;
  if (n <= SORT_T) sort_lds<1>(skeys, n, tid);
  else if (n <= 2 * SORT_T) sort_lds<2>(skeys, n, tid);
  else if (n <= 4 * SORT_T) sort_lds<4>(skeys, n, tid);
  else if (n <= FAST_LDS_KEYS) sort_lds<8>(skeys, n, tid);
  else {   // global bitonic over the whole list
    for (int i = tid; i < FAST_LDS_KEYS; i += SORT_T) gkeys[i] = skeys[i];
    int P = 1;
    while (P < n) P <<= 1;
    for (int i = n + tid; i < P; i += SORT_T) gkeys[i] = ~0ull;
    __syncthreads();
    for (int k = 2; k <= P; k <<= 1)
      for (int j = k >> 1; j > 0; j >>= 1) {
        for (int i = tid; i < P; i += SORT_T) {
          const int ixj = i ^ j;
          if (ixj > i) {
            const uint64_t ki = gkeys[i], kj = gkeys[ixj];
            if ((ki > kj) == ((i & k) == 0)) { gkeys[i] = kj; gkeys[ixj] = ki; }
          }
        }
        __syncthreads();
      }
    s = gkeys;
  }
  // ---- 3. lazy greedy
  const int m = n < a.max_nms ? n : a.max_nms;   // :698-699 (first max_nms in sorted order)
  if (tid == 0) total_s = 0;
  __syncthreads();
  const float* zb = a.z + (size_t)b * a.N * a.no;
  // wave 0 holds the next block's candidate in registers (lane = candidate): its z box and class are
  // loaded one block ahead, so their latency sits under the current block's IoU work
  float4 nz = make_float4(0.f, 0.f, 0.f, 0.f);
  int ncls = 0, nrow = 0;
  float nconf = 0.f;
  auto fetch = [&](int base) {
    const int j = base + tid;
    if (tid < 64 && j < m) {
      const uint64_t key = s[j];
      nrow = (int)(uint32_t)key;
      nconf = __uint_as_float(~(uint32_t)(key >> 32));
      const float* zr = zb + (size_t)nrow * a.no;
      nz = make_float4(zr[0], zr[1], zr[2], zr[3]);
      ncls = rb[nrow].cls;
    }
  };
  fetch(0);
  for (int base = 0; base < m; base += 64) {
    // the block's 64 candidates: boxes from z (xywh2xyxy, general.py:275-282), class from the row
    // record, class offset (general.py:702-703) unless agnostic
    if (tid < 64) {
      const int j = base + tid;
      if (j < m) {
        const float cx = nz.x, cy = nz.y, w = nz.z, h = nz.w;
        float4 r;
        r.x = cx - w / 2.0f;
        r.y = cy - h / 2.0f;
        r.z = cx + w / 2.0f;
        r.w = cy + h / 2.0f;
        const float off = a.agnostic ? 0.0f : (float)ncls * (float)MAX_WH;
        float4 bx;
        bx.x = r.x + off;
        bx.y = r.y + off;
        bx.z = r.z + off;
        bx.w = r.w + off;
        braw[tid] = r;
        bbox[tid] = bx;
        barea[tid] = (bx.z - bx.x) * (bx.w - bx.y);
        bconf[tid] = nconf;
        bcls[tid] = ncls;
        brow[tid] = nrow;
      }
      fetch(base + 64);
    }
    __syncthreads();
    const int total = total_s;
    // each wave: its 4 block rows i against the later block members (lanes) -> sup[i]; and its 4
    // candidates against every kept box so far -> pre[i] (suppressed by an earlier kept box)
#pragma unroll
    for (int q = 0; q < 64 / NW; ++q) {
      const int i = wv * (64 / NW) + q;
      const int ig = base + i;
      const int jg = base + lane;
      bool hit = false;
      if (ig < m && jg < m && lane > i) hit = iou_gt(bbox[i], barea[i], bbox[lane], barea[lane], a.iou);
      const uint64_t msk = __ballot(hit);
      bool kh = false;
      if (ig < m) {
        const float4 bi = bbox[i];
        const float ai = barea[i];
        for (int t = lane; t < total && !kh; t += 64) kh = iou_gt(kbox[t], karea[t], bi, ai, a.iou);
      }
      const bool anyk = __ballot(kh) != 0ull;
      if (lane == 0) {
        sup[i] = msk;
        pre[i] = anyk ? 1 : 0;
      }
    }
    __syncthreads();
    // wave 0 resolves the block in order
    if (tid < 64) {
      const int j = base + lane;
      const bool valid = j < m && !pre[lane];
      const uint64_t my_sup = sup[lane];
      uint64_t alive = __ballot(valid);
      uint64_t kept = 0;
      while (alive) {
        const int i = __ffsll((long long)alive) - 1;
        kept |= 1ull << i;
        alive &= ~__shfl(my_sup, i) & ~(1ull << i);
      }
      const int nk = __popcll(kept);
      if ((kept >> lane) & 1ull) {
        const int di = total + __popcll(kept & ((lane == 0) ? 0ull : (~0ull >> (64 - lane))));
        if (di < a.max_det) {
          kbox[di] = bbox[lane];
          karea[di] = barea[lane];
          const float4 r = braw[lane];
          float* d = a.det + ((size_t)b * a.max_det + di) * 6;
          d[0] = r.x;
          d[1] = r.y;
          d[2] = r.z;
          d[3] = r.w;
          d[4] = bconf[lane];
          d[5] = (float)bcls[lane];
          a.src_row[(size_t)b * a.max_det + di] = brow[lane];
        }
      }
      if (lane == 0) total_s = total + nk;
    }
    __syncthreads();
    if (total_s >= a.max_det) break;   // :705-706
  }
  // ---- 4. padding rows
  const int cnt = total_s < a.max_det ? total_s : a.max_det;
  for (int di = cnt + tid; di < a.max_det; di += SORT_T) {
    float* d = a.det + ((size_t)b * a.max_det + di) * 6;
#pragma unroll
    for (int q = 0; q < 6; ++q) d[q] = 0.0f;
    a.src_row[(size_t)b * a.max_det + di] = -1;
  }
  if (tid == 0) a.count[b] = cnt;
}

struct Layout {
  size_t cnt, offs, bconf, bcls, ncand, cand, keys, order, sbox, sarea, total;
  size_t cap, pcap;
  size_t fkeys, frb, kcap;   // fast path: [B][kcap] sort keys, [B][N] row records (when computed here)
};

inline size_t al(size_t x) { return (x + 255) & ~(size_t)255; }

Layout layout(int B, int N, int nc, int multi, int max_nms) {
  multi = multi && nc > 1;   // multi_label &= nc > 1 (general.py:646): the layout follows the path taken
  Layout L;
  L.cap = (size_t)N * (multi ? (size_t)nc : 1);
  L.pcap = 1;
  while (L.pcap < L.cap) L.pcap <<= 1;
  size_t o = 0;
  L.cnt = o; o = al(o + sizeof(int) * (size_t)B * N);
  L.offs = o; o = al(o + sizeof(int) * (size_t)B * N);
  L.bconf = o; o = al(o + sizeof(float) * (size_t)B * N);
  L.bcls = o; o = al(o + sizeof(int) * (size_t)B * N);
  L.ncand = o; o = al(o + sizeof(int) * (size_t)B);
  L.cand = o; o = al(o + sizeof(Cand) * (size_t)B * L.cap);
  L.keys = o; o = al(o + (L.pcap > (size_t)LDS_SORT_MAX ? sizeof(uint64_t) * (size_t)B * L.pcap : 0));
  L.order = o; o = al(o + sizeof(int) * (size_t)B * max_nms);
  L.sbox = o; o = al(o + sizeof(float4) * (size_t)B * max_nms);
  L.sarea = o; o = al(o + sizeof(float) * (size_t)B * max_nms);
  L.kcap = 1;
  while (L.kcap < (size_t)N) L.kcap <<= 1;
  L.fkeys = o; o = al(o + (multi ? 0 : sizeof(uint64_t) * (size_t)B * L.kcap));
  L.frb = o; o = al(o + (multi ? 0 : sizeof(RowBest) * (size_t)B * N));
  L.total = o;
  return L;
}

// End2End / EfficientNMS_TRT output packing (models/experimental.py:144-154, inf_onnx_trt.py:27-36):
// num_dets int32 [B,1], det_boxes [B,topk,4], det_scores [B,topk], det_classes int32 [B,topk].
__global__ __launch_bounds__(NT) void end2end_pack(const float* det, const int32_t* count, int B, int max_det, int topk,
                                                   int32_t* num_dets, float* boxes, float* scores, int32_t* classes) {
  const int b = blockIdx.x;
  const int n = count[b] < topk ? count[b] : topk;
  if (threadIdx.x == 0) num_dets[b] = n;
  for (int i = threadIdx.x; i < topk; i += NT) {
    const bool v = i < n;
    const float* d = det + ((size_t)b * max_det + i) * 6;
    float* bx = boxes + ((size_t)b * topk + i) * 4;
    bx[0] = v ? d[0] : 0.f;
    bx[1] = v ? d[1] : 0.f;
    bx[2] = v ? d[2] : 0.f;
    bx[3] = v ? d[3] : 0.f;
    scores[(size_t)b * topk + i] = v ? d[4] : 0.f;
    classes[(size_t)b * topk + i] = v ? (int32_t)d[5] : 0;
  }
}

}  // namespace

hipError_t launch_row_best(const float* z, int B, int N, int no, void* rowbest, hipStream_t st) {
  int gx = (N + 31) / 32;
  if (gx > 1024) gx = 1024;
  hipLaunchKernelGGL(row_best_kernel, dim3(gx, B), dim3(NT), 0, st, z, N, no, reinterpret_cast<RowBest*>(rowbest));
  return hipGetLastError();
}

hipError_t launch_end2end_pack(const float* det, const int32_t* count, int B, int max_det, int topk, int32_t* num_dets,
                               float* boxes, float* scores, int32_t* classes, hipStream_t st) {
  hipLaunchKernelGGL(end2end_pack, dim3(B), dim3(NT), 0, st, det, count, B, max_det, topk, num_dets, boxes, scores,
                     classes);
  return hipGetLastError();
}

size_t nms_workspace_bytes(int B, int N, int no, int multi, int max_nms) {
  return layout(B, N, no - 5, multi, max_nms).total;
}

hipError_t launch_nms(const float* z, const void* rowbest, int B, int N, int no, float conf, float iou, int multi,
                      int agnostic, int per_class, const int32_t* classes, int ncls, int max_det, int max_nms,
                      float* det, int64_t* src_row, int32_t* count, void* ws, hipStream_t st) {
  const Layout L = layout(B, N, no - 5, multi, max_nms);
  unsigned char* w = reinterpret_cast<unsigned char*>(ws);
  NmsArgs a;
  a.z = z;
  a.B = B;
  a.N = N;
  a.no = no;
  a.nc = no - 5;
  a.conf = conf;
  a.iou = iou;
  a.multi = multi && a.nc > 1;  // multi_label &= nc > 1 (general.py:646)
  a.agnostic = agnostic;
  a.per_class = per_class;
  a.classes = classes;
  a.ncls = ncls;
  a.max_det = max_det;
  a.max_nms = max_nms;
  a.cap = L.cap;
  a.pcap = L.pcap;
  a.cnt = (int*)(w + L.cnt);
  a.offs = (int*)(w + L.offs);
  a.bconf = (float*)(w + L.bconf);
  a.bcls = (int*)(w + L.bcls);
  a.ncand = (int*)(w + L.ncand);
  a.cand = (Cand*)(w + L.cand);
  a.keys = (uint64_t*)(w + L.keys);
  a.order = (int*)(w + L.order);
  a.sbox = (float4*)(w + L.sbox);
  a.sarea = (float*)(w + L.sarea);
  a.det = det;
  a.src_row = src_row;
  a.count = count;
  hipError_t e;
  int gx = (N + NT - 1) / NT;   // a lane per row
  if (gx > 1024) gx = 1024;
  if (!a.multi && !classes && !per_class && max_det <= FAST_MAX_DET) {
    // fast path (single label, no class filter): one launch (+ the row records when z comes alone)
    FastArgs f;
    f.z = z;
    f.rb = reinterpret_cast<const RowBest*>(rowbest);
    if (!rowbest) {   // derive the row records from z first (plans whose head does not write them)
      RowBest* rb = reinterpret_cast<RowBest*>(w + L.frb);
      int gr = (N + 31) / 32;
      if (gr > 1024) gr = 1024;
      hipLaunchKernelGGL(row_best_kernel, dim3(gr, B), dim3(NT), 0, st, z, N, no, rb);
      if ((e = hipGetLastError()) != hipSuccess) return e;
      f.rb = rb;
    }
    f.B = B;
    f.N = N;
    f.no = no;
    f.conf = conf;
    f.iou = iou;
    f.agnostic = agnostic;
    f.max_det = max_det;
    f.max_nms = max_nms;
    f.kcap = L.kcap;
    f.keys = reinterpret_cast<uint64_t*>(w + L.fkeys);
    f.det = det;
    f.src_row = src_row;
    f.count = count;
    const size_t lds = sizeof(uint64_t) * FAST_LDS_KEYS + (sizeof(float4) + sizeof(float)) * FAST_MAX_DET;
    static bool fast_attr = false;
    if (!fast_attr) {
      if ((e = hipFuncSetAttribute((const void*)nms_fast, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds)) !=
          hipSuccess)
        return e;
      fast_attr = true;
    }
    hipLaunchKernelGGL(nms_fast, dim3(B), dim3(SORT_T), lds, st, f);
    return hipGetLastError();
  }
  if ((e = hipMemsetAsync(det, 0, sizeof(float) * 6 * (size_t)B * max_det, st)) != hipSuccess) return e;
  if ((e = hipMemsetAsync(src_row, 0xff, sizeof(int64_t) * (size_t)B * max_det, st)) != hipSuccess) return e;
  if (rowbest && !a.multi && !classes)
    hipLaunchKernelGGL(nms_rows_from_best, dim3(gx, B), dim3(NT), 0, st, a, reinterpret_cast<const RowBest*>(rowbest));
  else
    hipLaunchKernelGGL(nms_rows, dim3(gx, B), dim3(NT), 0, st, a);
  if ((e = hipGetLastError()) != hipSuccess) return e;
  hipLaunchKernelGGL(nms_scan, dim3(B), dim3(SORT_T), 0, st, a);
  if ((e = hipGetLastError()) != hipSuccess) return e;
  hipLaunchKernelGGL(nms_write, dim3(gx, B), dim3(NT), 0, st, a);
  if ((e = hipGetLastError()) != hipSuccess) return e;
  const size_t sort_lds = sizeof(uint64_t) * LDS_SORT_MAX;
  static bool attr_set = false;
  if (!attr_set) {
    if ((e = hipFuncSetAttribute((const void*)nms_sort, hipFuncAttributeMaxDynamicSharedMemorySize, (int)sort_lds)) !=
        hipSuccess)
      return e;
    attr_set = true;
  }
  hipLaunchKernelGGL(nms_sort, dim3(B), dim3(SORT_T), sort_lds, st, a);
  if ((e = hipGetLastError()) != hipSuccess) return e;
  const size_t g_lds = (((size_t)(max_nms + 31) / 32 + 2) * 4 + 15) / 16 * 16 + 64 * (16 + 4 + 4);
  hipLaunchKernelGGL(nms_greedy, dim3(B), dim3(SORT_T), g_lds, st, a);
  return hipGetLastError();
}

}  // namespace yv7
