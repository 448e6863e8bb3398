/* TEST INFRASTRUCTURE ONLY (see oracle/__init__.py).
 *
 * CPU restatement of torchvision.ops.nms, the third-party op the reference calls at
 * utils/general.py:704.  torchvision is not vendored and its version is unpinned;
 * this follows its published CPU algorithm (torchvision/csrc/ops/cpu/nms_kernel.cpp):
 *   areas = (x2 - x1) * (y2 - y1)                      (no +1)
 *   order = stable descending sort of scores          (ties keep input order)
 *   greedy: keep i, suppress every later j with inter / (area_i + area_j - inter) > thr
 * All arithmetic in fp32, compiled with -ffp-contract=off so no FMA changes a rounding.
 */
#include <stdint.h>
#include <stdlib.h>

static const float* g_scores;

static int cmp_desc_stable(const void* a, const void* b) {
  int64_t i = *(const int64_t*)a, j = *(const int64_t*)b;
  float si = g_scores[i], sj = g_scores[j];
  if (si > sj) return -1;
  if (si < sj) return 1;
  return (i < j) ? -1 : (i > j);
}

static inline float fmaxf_(float a, float b) { return a > b ? a : b; }
static inline float fminf_(float a, float b) { return a < b ? a : b; }

/* boxes: [n][4] x1,y1,x2,y2; returns number kept, indices (into boxes) in keep[] in score order. */
int64_t oracle_nms(const float* boxes, const float* scores, int64_t n, float thr, int64_t* keep) {
  if (n <= 0) return 0;
  int64_t* order = (int64_t*)malloc(sizeof(int64_t) * n);
  float* areas = (float*)malloc(sizeof(float) * n);
  unsigned char* supp = (unsigned char*)calloc(n, 1);
  for (int64_t i = 0; i < n; ++i) {
    order[i] = i;
    const float* b = boxes + 4 * i;
    areas[i] = (b[2] - b[0]) * (b[3] - b[1]);
  }
  g_scores = scores;
  qsort(order, (size_t)n, sizeof(int64_t), cmp_desc_stable);
  int64_t nk = 0;
  for (int64_t _i = 0; _i < n; ++_i) {
    int64_t i = order[_i];
    if (supp[i]) continue;
    keep[nk++] = i;
    const float* bi = boxes + 4 * i;
    float ix1 = bi[0], iy1 = bi[1], ix2 = bi[2], iy2 = bi[3], iarea = areas[i];
    for (int64_t _j = _i + 1; _j < n; ++_j) {
      int64_t j = order[_j];
      if (supp[j]) continue;
      const float* bj = boxes + 4 * j;
      float xx1 = fmaxf_(ix1, bj[0]), yy1 = fmaxf_(iy1, bj[1]);
      float xx2 = fminf_(ix2, bj[2]), yy2 = fminf_(iy2, bj[3]);
      float w = fmaxf_(0.0f, xx2 - xx1), h = fmaxf_(0.0f, yy2 - yy1);
      float inter = w * h;
      float ovr = inter / (iarea + areas[j] - inter);
      if (ovr > thr) supp[j] = 1;
    }
  }
  free(order);
  free(areas);
  free(supp);
  return nk;
}
