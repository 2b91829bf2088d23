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

// ---------------------------------------------------------------------------
// Wide candidate sets: sample_token with top_k <= 0 (no top-k filter, `inference_utils.py:136`)
// or top_k above TOPK_CAP -- up to the whole 151,936-id text row.  No candidate list is built:
// the scores are bf16-exact, so every score is one of 65,536 keys and the candidates in
// (score desc, index asc) order are the key bins in descending key order, each bin a run of
// EQUAL scores in index order.  All of top-k (torch.topk: exactly min(K, #finite), lowest
// indices among the threshold ties), top-p (apply_top_p_optimized :44-59) and the multinomial
// draw then work on bin counts [hist, global scratch of WIDE_BINS ints, owned by the block]:
//   c_k    candidates in bin k (the threshold bin keeps `need` of its ties)
//   ev_k = exp(s_k - s_max);  S = sum_k fp32(c_k * ev_k)
//   p_k  = bf16(ev_k / S);  cumulative probability after the r-th element of bin k
//          cum = fp32(P_t + fp32(L + fp32(r * p_k))), L = the thread chunk's sequential sum of
//          the bins before k, P_t = the exclusive sum of the earlier chunks' totals
//   keep up to the first element whose bf16(cum) > top_p (it stays: the shift-right rule)
//   q_k = bf16(ev_k / S2) over the survivors, target = u * Q, the drawn element is the first
//   whose cumulative q (same form) exceeds target, i.e. the r-th index of its bin.
// Sums run in a fixed order: thread t of NT owns the 64 bins at descending positions
// [64 t, 64 t + 64) and sums them sequentially; chunk totals are summed sequentially.
// oracle.moss_delay.wide_draw restates this bit for bit.  Returns the token index (-1: no finite
// score).  All NT threads must call it; NT * 64 == WIDE_BINS.
constexpr int WIDE_BINS = 65536;
template <int NT, class F>
__device__ int block_wide_draw(F val, int V, int K, float top_p, float u, int* hist) {
  static_assert(NT * 64 == WIDE_BINS, "64 bins per thread");
  typedef __attribute__((address_space(1))) int gi32;
  // the bins live in L2 (agent-scope atomics and loads; never a stale L1 line)
  auto hld = [&](int key) { return __hip_atomic_load((gi32*)(hist + key), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT); };
  const int t = threadIdx.x;
  __shared__ float wf[NT];
  __shared__ int wi[NT];
  __shared__ int w_thr, w_need, w_topkey, w_cut, w_cut_t, w_cut_key, w_cut_r, w_tok;
  __shared__ float w_tot;
  for (int i = t; i < WIDE_BINS; i += NT) __hip_atomic_store((gi32*)(hist + i), 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  for (int i = t; i < V; i += NT) {
    const float v = val(i);
    if (v > -INFINITY) __hip_atomic_fetch_add((gi32*)(hist + okey16(v)), 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  const int key0 = WIDE_BINS - 1 - 64 * t;  // this thread's bins: key0, key0 - 1, ..., key0 - 63
  // finite scores per chunk -> exclusive prefix (integers: exact)
  int mine = 0;
  for (int j = 0; j < 64; ++j) mine += hld(key0 - j);
  wi[t] = mine;
  __syncthreads();
  if (t == 0) {
    int run = 0, top = -1;
    for (int w = 0; w < NT; ++w) {
      const int c = wi[w];
      wi[w] = run;
      if (top < 0 && c > 0) top = w;
      run += c;
    }
    w_topkey = -1;
    if (top >= 0)
      for (int j = 0; j < 64; ++j)
        if (hld(WIDE_BINS - 1 - 64 * top - j) > 0) { w_topkey = WIDE_BINS - 1 - 64 * top - j; break; }
    w_thr = -1;  // no top-k cut: every finite score is a candidate
    w_need = 0;
    w_cut = K > 0 && K < run;
    w_tok = -1;
  }
  __syncthreads();
  if (w_topkey < 0) return -1;
  if (w_cut) {
    // torch.topk: the chunk where the running count first reaches K holds the threshold key;
    // `need` of its ties (the lowest indices) are candidates
    const int before = wi[t];
    if (before < K && before + mine >= K) {
      int cum = before;
      for (int j = 0; j < 64; ++j) {
        const int c = hld(key0 - j);
        if (cum + c >= K) {
          w_thr = key0 - j;
          w_need = K - cum;
          break;
        }
        cum += c;
      }
    }
    __syncthreads();
  }
  const int thr = w_thr, need = w_need;
  const float mx = okey16_val((uint32_t)w_topkey);
  // candidates of bin `key` among the first (lim_key, lim_r) survivors (lim_key -1: all)
  auto cnt = [&](int key, int lim_key, int lim_r) -> int {
    if (key < lim_key) return 0;
    if (key == lim_key) return lim_r;
    if (thr < 0 || key > thr) return hld(key);
    return key == thr ? need : 0;
  };
  // (no contraction: every product and sum rounds on its own, as oracle.moss_delay.wide_draw)
  auto mass = [](int c, float x) { return __fmul_rn((float)c, x); };
  // fixed-order sum of fp32(c * f(key)); leaves the exclusive chunk prefixes in wf
  auto chunk_sums = [&](auto f, int lim_key, int lim_r) -> float {
    float part = 0.f;
    for (int j = 0; j < 64; ++j) {
      const int c = cnt(key0 - j, lim_key, lim_r);
      if (c) part = __fadd_rn(part, mass(c, f(key0 - j)));
    }
    wf[t] = part;
    __syncthreads();
    if (t == 0) {
      float run = 0.f;
      for (int w = 0; w < NT; ++w) { const float x = wf[w]; wf[w] = run; run = __fadd_rn(run, x); }
      w_tot = run;
    }
    __syncthreads();
    return w_tot;
  };
  // the first element whose cumulative value fp32(P_t + fp32(L + fp32(r * f))) passes `pass`
  // -> (w_cut_key, w_cut_r); -1 when none does
  auto first_cross = [&](auto f, int lim_key, int lim_r, auto pass) {
    if (t == 0) { w_cut_t = NT; w_cut_key = -1; w_cut_r = 0; }
    __syncthreads();
    const float P = wf[t];
    float L = 0.f;
    int ck = -1, cr = 0;
    for (int j = 0; j < 64 && ck < 0; ++j) {
      const int key = key0 - j, c = cnt(key, lim_key, lim_r);
      if (!c) continue;
      const float x = f(key);
      if (pass(__fadd_rn(P, __fadd_rn(L, mass(c, x))))) {
        int lo = 1, hi = c;  // the smallest r that passes (monotone in r)
        while (lo < hi) {
          const int mid = (lo + hi) >> 1;
          if (pass(__fadd_rn(P, __fadd_rn(L, mass(mid, x))))) hi = mid;
          else lo = mid + 1;
        }
        ck = key;
        cr = lo;
      }
      L = __fadd_rn(L, mass(c, x));
    }
    if (ck >= 0) atomicMin(&w_cut_t, t);
    __syncthreads();
    if (ck >= 0 && w_cut_t == t) { w_cut_key = ck; w_cut_r = cr; }
    __syncthreads();
  };
  // exp in double, rounded once to fp32: correctly rounded, so the oracle's numpy exp gives the
  // same bits (fp32 expf implementations differ in the last place)
  auto evf = [&](int key) { return (float)exp((double)(okey16_val((uint32_t)key) - mx)); };
  int lim_key = -1, lim_r = 0;
  if (top_p < 1.0f) {
    const float S = chunk_sums(evf, -1, 0);
    auto pf = [&](int key) { return rbf(evf(key) / S); };
    chunk_sums(pf, -1, 0);
    first_cross(pf, -1, 0, [&](float cum) { return rbf(cum) > top_p; });
    lim_key = w_cut_key;  // -1 (never crossed): every candidate survives
    lim_r = w_cut_r;
  }
  const float S2 = chunk_sums(evf, lim_key, lim_r);
  auto qf = [&](int key) { return rbf(evf(key) / S2); };
  const float Q = chunk_sums(qf, lim_key, lim_r);
  const float target = __fmul_rn(u, Q);
  first_cross(qf, lim_key, lim_r, [&](float cum) { return cum > target; });
  if (w_cut_key < 0) {  // rounding left the target past the last survivor: take the last one
    __syncthreads();
    if (t == 0) {
      int k = lim_key, r = lim_r;
      if (lim_key < 0)
        for (k = 0; k < WIDE_BINS; ++k)
          if ((r = cnt(k, -1, 0)) > 0) break;
      w_cut_key = k;
      w_cut_r = r;
    }
    __syncthreads();
  }
  const int dk = w_cut_key, dr = w_cut_r;
  // the dr-th (1-based) index of bin dk in index order: contiguous index chunks + block scan
  const int chunk = (V + NT - 1) / NT;
  const int lo_i = min(V, t * chunk), hi_i = min(V, lo_i + chunk);
  int c = 0;
  for (int i = lo_i; i < hi_i; ++i) {
    const float v = val(i);
    c += (v > -INFINITY && (int)okey16(v) == dk) ? 1 : 0;
  }
  wi[t] = c;
  __syncthreads();
  if (t == 0) {
    int run = 0;
    for (int w = 0; w < NT; ++w) { const int x = wi[w]; wi[w] = run; run += x; }
  }
  __syncthreads();
  int rank = wi[t];
  if (rank < dr && rank + c >= dr) {
    for (int i = lo_i; i < hi_i; ++i) {
      const float v = val(i);
      if (v > -INFINITY && (int)okey16(v) == dk && ++rank == dr) {
        w_tok = i;
        break;
      }
    }
  }
  __syncthreads();
  return w_tok;
}

// ---------------------------------------------------------------------------
// The same bin walk with the HF processor semantics of MossTTSLocal's channel pick
// (moss_tts_local/modeling_moss_tts.py:360-368, 414-419) for candidate sets past TOPK_CAP
// (text channel without a top_k, a top_k above 1,024, or threshold ties beyond TOPK_CAP):
//   TopKLogitsWarper: every score >= the K-th largest (all threshold ties kept)
//   TopPLogitsWarper: ascending order, p = bf16(softmax), inclusive cumsum; elements with
//     bf16(cum) <= bf16(1 - top_p) are dropped, the largest always stays.  Inside a bin of
//     equal scores the ascending walk meets the LOWEST index first (torch.sort's order on the
//     reference's CPU path, restated by oracle.moss_local.hf_pick_distribution's stable argsort)
//   multinomial over the survivors' exp(s - s_max) (unnormalised, as the sorted path)
// Sums in the same fixed chunked order as block_wide_draw (ascending walk: thread t owns the
// bins [64 t, 64 t + 64)).  Returns the token index (-1: no finite score).
template <int NT, class F>
__device__ int block_wide_draw_hf(F val, int V, int K, float top_p, float u, int* hist) {
  static_assert(NT * 64 == WIDE_BINS, "64 bins per thread");
  typedef __attribute__((address_space(1))) int gi32;
  auto hld = [&](int key) { return __hip_atomic_load((gi32*)(hist + key), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT); };
  const int t = threadIdx.x;
  __shared__ float hf_wf[NT];
  __shared__ int hf_wi[NT];
  __shared__ int h_thr, h_topkey, h_cut_t, h_cut_key, h_cut_r, h_tok;
  __shared__ float h_tot;
  for (int i = t; i < WIDE_BINS; i += NT) __hip_atomic_store((gi32*)(hist + i), 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  for (int i = t; i < V; i += NT) {
    const float v = val(i);
    if (v > -INFINITY) __hip_atomic_fetch_add((gi32*)(hist + okey16(v)), 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  // descending ownership (thread t: keys dkey0, dkey0 - 1, ...) for top-k and the draw,
  // ascending (akey0, akey0 + 1, ...) for the top-p walk
  const int dkey0 = WIDE_BINS - 1 - 64 * t, akey0 = 64 * t;
  int mine = 0;
  for (int j = 0; j < 64; ++j) mine += hld(dkey0 - j);
  hf_wi[t] = mine;
  __syncthreads();
  if (t == 0) {
    int run = 0, top = -1;
    for (int w = 0; w < NT; ++w) {
      const int c = hf_wi[w];
      hf_wi[w] = run;
      if (top < 0 && c > 0) top = w;
      run += c;
    }
    h_topkey = -1;
    if (top >= 0)
      for (int j = 0; j < 64; ++j)
        if (hld(WIDE_BINS - 1 - 64 * top - j) > 0) { h_topkey = WIDE_BINS - 1 - 64 * top - j; break; }
    h_thr = (K > 0 && K < run) ? -2 : -1;  // -2: the top-k threshold key is found below
    h_tok = -1;
  }
  __syncthreads();
  if (h_topkey < 0) return -1;
  if (h_thr == -2) {
    const int before = hf_wi[t];
    if (before < K && before + mine >= K) {
      int cum = before;
      for (int j = 0; j < 64; ++j) {
        cum += hld(dkey0 - j);
        if (cum >= K) { h_thr = dkey0 - j; break; }
      }
    }
    __syncthreads();
  }
  const int thr = h_thr < 0 ? 0 : h_thr;  // bins below thr are cut (keep-all-ties: thr's bin stays whole)
  const float mx = okey16_val((uint32_t)h_topkey);
  // survivors: bins above lim_key whole, bin lim_key without its lim_skip lowest indices
  auto cnt = [&](int key, int lim_key, int lim_skip) -> int {
    if (key < thr || key < lim_key) return 0;
    return key == lim_key ? hld(key) - lim_skip : hld(key);
  };
  auto mass = [](int c, float x) { return __fmul_rn((float)c, x); };
  // fixed-order sum of fp32(c * f(key)) over this thread's 64 bins in direction `asc`; leaves the
  // exclusive chunk prefixes (in thread order) in hf_wf
  auto chunk_sums = [&](auto f, bool asc, int lim_key, int lim_skip) -> float {
    float part = 0.f;
    for (int j = 0; j < 64; ++j) {
      const int key = asc ? akey0 + j : dkey0 - j, c = cnt(key, lim_key, lim_skip);
      if (c) part = __fadd_rn(part, mass(c, f(key)));
    }
    hf_wf[t] = part;
    __syncthreads();
    if (t == 0) {
      float run = 0.f;
      for (int w = 0; w < NT; ++w) { const float x = hf_wf[w]; hf_wf[w] = run; run = __fadd_rn(run, x); }
      h_tot = run;
    }
    __syncthreads();
    return h_tot;
  };
  // the first element (walk direction asc) whose cumulative fp32(P_t + fp32(L + fp32(r * f)))
  // passes -> (h_cut_key, h_cut_r = its rank r >= 1 inside the bin); h_cut_key -1 when none does
  auto first_cross = [&](auto f, bool asc, int lim_key, int lim_skip, auto pass) {
    if (t == 0) { h_cut_t = NT; h_cut_key = -1; h_cut_r = 0; }
    __syncthreads();
    const float P = hf_wf[t];
    float L = 0.f;
    int ck = -1, cr = 0;
    for (int j = 0; j < 64 && ck < 0; ++j) {
      const int key = asc ? akey0 + j : dkey0 - j, c = cnt(key, lim_key, lim_skip);
      if (!c) continue;
      const float x = f(key);
      if (pass(__fadd_rn(P, __fadd_rn(L, mass(c, x))))) {
        int lo = 1, hi = c;
        while (lo < hi) {
          const int mid = (lo + hi) >> 1;
          if (pass(__fadd_rn(P, __fadd_rn(L, mass(mid, x))))) hi = mid;
          else lo = mid + 1;
        }
        ck = key;
        cr = lo;
      }
      L = __fadd_rn(L, mass(c, x));
    }
    if (ck >= 0) atomicMin(&h_cut_t, t);
    __syncthreads();
    if (ck >= 0 && h_cut_t == t) { h_cut_key = ck; h_cut_r = cr; }
    __syncthreads();
  };
  auto evf = [&](int key) { return (float)exp((double)(okey16_val((uint32_t)key) - mx)); };
  int lim_key = -1, lim_skip = 0;
  if (top_p < 1.0f) {
    const float thr_p = rbf((float)(1.0 - (double)top_p));
    const float S = chunk_sums(evf, false, -1, 0);
    auto pf = [&](int key) { return rbf(evf(key) / S); };
    chunk_sums(pf, true, -1, 0);  // ascending prefixes
    first_cross(pf, true, -1, 0, [&](float cum) { return rbf(cum) > thr_p; });
    lim_key = h_cut_key < 0 ? h_topkey : h_cut_key;
    // the crossing element and everything above it stay (r - 1 lowest indices of its bin go);
    // none crossing: the largest alone (the highest index of the top bin) stays
    lim_skip = h_cut_key < 0 ? hld(h_topkey) - 1 : h_cut_r - 1;
  }
  const float S2 = chunk_sums(evf, false, lim_key, lim_skip);
  const float target = __fmul_rn(u, S2);
  first_cross(evf, false, lim_key, lim_skip, [&](float cum) { return cum > target; });
  if (h_cut_key < 0) {  // rounding left the target past the last survivor: take the last one
    __syncthreads();
    if (t == 0) {
      int k = lim_key, r = lim_key >= 0 ? hld(lim_key) - lim_skip : 0;
      if (lim_key < 0)
        for (k = thr; k < WIDE_BINS; ++k)
          if ((r = cnt(k, -1, 0)) > 0) break;
      h_cut_key = k;
      h_cut_r = r;
    }
    __syncthreads();
  }
  const int dk = h_cut_key, dr = h_cut_r + (h_cut_key == lim_key ? lim_skip : 0);
  // the dr-th (1-based) lowest index of bin dk (the cut bin's survivors are its highest indices)
  const int chunk = (V + NT - 1) / NT;
  const int lo_i = min(V, t * chunk), hi_i = min(V, lo_i + chunk);
  int c = 0;
  for (int i = lo_i; i < hi_i; ++i) {
    const float v = val(i);
    c += (v > -INFINITY && (int)okey16(v) == dk) ? 1 : 0;
  }
  hf_wi[t] = c;
  __syncthreads();
  if (t == 0) {
    int run = 0;
    for (int w = 0; w < NT; ++w) { const int x = hf_wi[w]; hf_wi[w] = run; run += x; }
  }
  __syncthreads();
  int rank = hf_wi[t];
  if (rank < dr && rank + c >= dr) {
    for (int i = lo_i; i < hi_i; ++i) {
      const float v = val(i);
      if (v > -INFINITY && (int)okey16(v) == dk && ++rank == dr) {
        h_tok = i;
        break;
      }
    }
  }
  __syncthreads();
  return h_tok;
}

}  // namespace mtts
