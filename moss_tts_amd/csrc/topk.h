// Block-wide top-K candidate selection for the samplers (Delay: sample.hip, Local: local.hip).
//
// The processed scores the samplers select from are bf16-exact (every reference op before
// top-k rounds to bf16: temperature `modeling_moss_tts.py:451`, repetition penalty
// `inference_utils.py:79-88`, HF warpers `moss_tts_local/modeling_moss_tts.py:360-368`), so a
// score is fully described by a 16-bit order-preserving key.  The K-th largest key comes from a
// two-pass 8-bit radix select over the row (never sorted), the candidates at or above it are
// gathered, and only those (<= TOPK_CAP) are bitonic-sorted in LDS.
//
// Tie rules at the K-th score:
//   TIES_EXACT_K  torch.topk (`inference_utils.py:19-26`): exactly min(K, #finite) entries;
//                 among scores equal to the threshold the lowest indices are kept.
//   TIES_KEEP_ALL HF TopKLogitsWarper: every score >= the K-th largest; if that exceeds
//                 TOPK_CAP, the threshold ties are taken in index order until the buffer is
//                 full and the overflow is reported (never an arrival-order choice).
#pragma once
#include "kernels.h"

namespace mtts {

enum TopkTies { TIES_EXACT_K = 0, TIES_KEEP_ALL = 1 };

// order-preserving 16-bit key of a bf16-exact finite float (+0 and -0 share a key)
__device__ __forceinline__ uint32_t okey16(float v) {
  if (v == 0.f) v = 0.f;
  const uint32_t u = __float_as_uint(v) >> 16;
  return (u & 0x8000u) ? (~u & 0xFFFFu) : (u | 0x8000u);
}
__device__ __forceinline__ float okey16_val(uint32_t k) {
  const uint32_t u = (k & 0x8000u) ? (k & 0x7FFFu) : (~k & 0xFFFFu);
  return __uint_as_float(u << 16);
}
// sort word: ascending order == (score descending, index ascending)
__device__ __forceinline__ unsigned long long cand_word(uint32_t key, int idx) {
  return ((unsigned long long)(0xFFFFu - key) << 32) | (unsigned)idx;
}
__device__ __forceinline__ float cand_score(unsigned long long w) {
  return okey16_val(0xFFFFu - (uint32_t)(w >> 32));
}
__device__ __forceinline__ int cand_index(unsigned long long w) { return (int)(w & 0xffffffffu); }

struct TopkSmem {
  int hist[256];
  int scan[1024 / 64 + 1];
  int s_hi, s_need, s_thr, s_n, s_ties, s_over;
  unsigned long long cand[TOPK_CAP];
};

// Selects the candidates of row scores val(i), i < V (-inf = excluded) and leaves them in
// sm.cand[0..n) sorted by (score desc, index asc).  Returns n; *overflow = 1 when KEEP_ALL
// ties were cut at TOPK_CAP.  All NT threads of the block must call it.  K <= TOPK_CAP.
template <int NT, class F>
__device__ int block_topk_sorted(F val, int V, int K, int ties, TopkSmem& sm, int* overflow) {
  const int t = threadIdx.x;
  K = min(K, V);
  for (int i = t; i < 256; i += NT) sm.hist[i] = 0;
  if (t == 0) { sm.s_n = 0; sm.s_over = 0; }
  __syncthreads();
  // pass 1: high key byte of the finite scores
  for (int i = t; i < V; i += NT) {
    const float v = val(i);
    if (v > -INFINITY) atomicAdd(&sm.hist[okey16(v) >> 8], 1);
  }
  __syncthreads();
  if (t == 0) {
    int cum = 0, hi;
    for (hi = 255; hi >= 0; --hi) {
      if (cum + sm.hist[hi] >= K) break;
      cum += sm.hist[hi];
    }
    sm.s_hi = hi;  // -1: fewer than K finite scores, every finite score is kept
    sm.s_need = K - cum;
  }
  __syncthreads();
  const int hi = sm.s_hi;
  if (hi >= 0) {
    // pass 2: low byte inside the selected high bin
    for (int i = t; i < 256; i += NT) sm.hist[i] = 0;
    __syncthreads();
    for (int i = t; i < V; i += NT) {
      const float v = val(i);
      if (v > -INFINITY) {
        const uint32_t k = okey16(v);
        if ((int)(k >> 8) == hi) atomicAdd(&sm.hist[k & 255], 1);
      }
    }
    __syncthreads();
    if (t == 0) {
      int cum = 0, lo;
      for (lo = 255; lo > 0; --lo) {
        if (cum + sm.hist[lo] >= sm.s_need) break;
        cum += sm.hist[lo];
      }
      sm.s_thr = (hi << 8) | lo;
      sm.s_need = sm.s_need - cum;  // ties at the threshold to take (EXACT_K)
      sm.s_ties = sm.hist[lo];      // ties at the threshold present
    }
  } else if (t == 0) {
    sm.s_thr = 0;
    sm.s_need = 0x7fffffff;
    sm.s_ties = 0;
  }
  __syncthreads();
  const uint32_t thr = (uint32_t)sm.s_thr;
  // how many threshold ties fit: all of them, or an ordered prefix
  int take_ties = sm.s_ties;
  if (hi >= 0) {
    const int above = K - sm.s_need;  // scores strictly above the threshold (< K <= CAP)
    const int lim = ties == TIES_EXACT_K ? sm.s_need : TOPK_CAP - above;
    take_ties = min(sm.s_ties, lim);
  }
  const bool ordered = hi >= 0 && take_ties < sm.s_ties;
  // pass 3: every finite score above the threshold (all >= it when the ties fit)
  for (int i = t; i < V; i += NT) {
    const float v = val(i);
    if (v > -INFINITY) {
      const uint32_t k = okey16(v);
      if (k > thr || (!ordered && k == thr)) {
        const int slot = atomicAdd(&sm.s_n, 1);
        sm.cand[slot] = cand_word(k, i);
      }
    }
  }
  __syncthreads();
  if (ordered) {
    // pass 4: the first take_ties threshold ties in index order (thread t owns a contiguous
    // index chunk; a block scan orders the chunks)
    const int chunk = (V + NT - 1) / NT;
    const int lo_i = t * chunk, hi_i = min(V, lo_i + chunk);
    int c = 0;
    for (int i = lo_i; i < hi_i; ++i) {
      const float v = val(i);
      c += (v > -INFINITY && okey16(v) == thr) ? 1 : 0;
    }
    // exclusive block scan of c
    int x = c;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const int y = __shfl_up(x, o, 64);
      if ((t & 63) >= o) x += y;
    }
    if ((t & 63) == 63) sm.scan[t >> 6] = x;
    __syncthreads();
    if (t == 0) {
      int run = 0;
      for (int w = 0; w < NT / 64; ++w) { const int s = sm.scan[w]; sm.scan[w] = run; run += s; }
    }
    __syncthreads();
    int rank = sm.scan[t >> 6] + x - c;
    const int base = sm.s_n;
    for (int i = lo_i; i < hi_i && rank < take_ties; ++i) {
      const float v = val(i);
      if (v > -INFINITY && okey16(v) == thr) sm.cand[base + rank++] = cand_word(thr, i);
    }
    __syncthreads();
    if (t == 0) {
      sm.s_n = base + take_ties;
      if (ties == TIES_KEEP_ALL) sm.s_over = 1;
    }
    __syncthreads();
  }
  const int n = sm.s_n;
  int np = 1;
  while (np < n) np <<= 1;
  for (int i = n + t; i < np; i += NT) sm.cand[i] = ~0ull;
  __syncthreads();
  for (int k = 2; k <= np; k <<= 1)
    for (int j = k >> 1; j > 0; j >>= 1) {
      for (int i = t; i < np; i += NT) {
        const int p = i ^ j;
        if (p > i) {
          const unsigned long long a = sm.cand[i], b = sm.cand[p];
          const bool up = (i & k) == 0;
          if ((a > b) == up) { sm.cand[i] = b; sm.cand[p] = a; }
        }
      }
      __syncthreads();
    }
  if (overflow) *overflow = sm.s_over;
  return n;
}

}  // namespace mtts
