// Device kernels of the MossTTSLocal depth stage (moss_tts_local/modeling_moss_tts.py):
// MossTTSRMSNorm in bf16, greedy channel argmax, and the per-frame stop/append state machine
// of CustomMixin._sample (:377-456).  The projections and the depth transformer reuse the
// GEMV / decode-attention kernels of the backbone.
#include "kernels.h"
#include "topk.h"

namespace mtts {

// MossTTSRMSNorm (:34-44) WITHOUT the fp32 upcast of Qwen3RMSNorm: every torch op rounds to
// bf16.  norm = mean(bf16(x*x)) (fp32 accumulation, rounded), r = bf16(rsqrt(bf16(norm+eps))),
// y = bf16(bf16(x*r) * w).  One block per row, 16-byte chunks.
__global__ __launch_bounds__(256) void moss_rmsnorm_kernel(const bf16_t* __restrict__ x, const bf16_t* __restrict__ w,
                                                           bf16_t* __restrict__ y, int H, float eps) {
  __shared__ float red[4];
  const int m = blockIdx.x, t = threadIdx.x;
  const bf16_t* xr = x + (size_t)m * H;
  float s = 0.f;
  if (H <= 2 * 256 * 8) {
    // H <= 4096: the row's chunks and the weight load together, once, and stay in registers
    // (the general form below re-reads x and the weight after the reduction)
    uint4 xv[2], wv[2];
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const int c = t + u * 256;
      if (c < (H >> 3)) {
        xv[u] = *reinterpret_cast<const uint4*>(xr + c * 8);
        wv[u] = *reinterpret_cast<const uint4*>(w + c * 8);
      }
    }
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      if (t + u * 256 < (H >> 3)) {
        float v[8];
        unpack8(xv[u], v);
#pragma unroll
        for (int i = 0; i < 8; ++i) s += rbf(v[i] * v[i]);
      }
    }
    s = wave_sum(s);
    if ((t & 63) == 0) red[t >> 6] = s;
    __syncthreads();
    const float tot = (red[0] + red[1]) + (red[2] + red[3]);
    const float norm = rbf(tot / (float)H);
    const float r = rbf(1.0f / sqrtf(rbf(norm + eps)));
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const int c = t + u * 256;
      if (c < (H >> 3)) {
        float v[8], g[8], q[8];
        unpack8(xv[u], v);
        unpack8(wv[u], g);
#pragma unroll
        for (int i = 0; i < 8; ++i) q[i] = rbf(v[i] * r) * g[i];
        uint4 o;
        o.x = pack2(q[0], q[1]); o.y = pack2(q[2], q[3]); o.z = pack2(q[4], q[5]); o.w = pack2(q[6], q[7]);
        *reinterpret_cast<uint4*>(y + (size_t)m * H + c * 8) = o;
      }
    }
    return;
  }
  for (int c = t; c < (H >> 3); c += 256) {
    float v[8];
    unpack8(*reinterpret_cast<const uint4*>(xr + c * 8), v);
#pragma unroll
    for (int i = 0; i < 8; ++i) s += rbf(v[i] * v[i]);
  }
  s = wave_sum(s);
  if ((t & 63) == 0) red[t >> 6] = s;
  __syncthreads();
  const float tot = (red[0] + red[1]) + (red[2] + red[3]);
  const float norm = rbf(tot / (float)H);
  const float r = rbf(1.0f / sqrtf(rbf(norm + eps)));
  for (int c = t; c < (H >> 3); c += 256) {
    float v[8], g[8], q[8];
    unpack8(*reinterpret_cast<const uint4*>(xr + c * 8), v);
    unpack8(*reinterpret_cast<const uint4*>(w + c * 8), g);
#pragma unroll
    for (int i = 0; i < 8; ++i) q[i] = rbf(v[i] * r) * g[i];
    uint4 o;
    o.x = pack2(q[0], q[1]); o.y = pack2(q[2], q[3]); o.z = pack2(q[4], q[5]); o.w = pack2(q[6], q[7]);
    *reinterpret_cast<uint4*>(y + (size_t)m * H + c * 8) = o;
  }
}

hipError_t moss_rmsnorm(const bf16_t* x, const bf16_t* w, bf16_t* y, int M, int H, float eps, hipStream_t s) {
  if (H % 8 || M <= 0) return hipErrorInvalidValue;
  hipLaunchKernelGGL(moss_rmsnorm_kernel, dim3(M), dim3(256), 0, s, x, w, y, H, eps);
  return hipGetLastError();
}

// torch.argmax over one logits row (first index among equal maxima), one block per row
__global__ __launch_bounds__(1024) void argmax_rows_kernel(const bf16_t* __restrict__ logits, int ld, int V,
                                                           int64_t* __restrict__ out, int ld_out) {
  __shared__ ArgMax sh[16];
  const int b = blockIdx.x, t = threadIdx.x;
  const bf16_t* row = logits + (size_t)b * ld;
  ArgMax a{-INFINITY, 0x7fffffff};
  const int nv = V >> 3;
  if ((ld & 7) == 0) {
    for (int c = t; c < nv; c += 1024) {
      float v[8];
      unpack8(*reinterpret_cast<const uint4*>(row + c * 8), v);
#pragma unroll
      for (int i = 0; i < 8; ++i) a = am_better(a, ArgMax{v[i], c * 8 + i});
    }
    for (int i = nv * 8 + t; i < V; i += 1024) a = am_better(a, ArgMax{bf2f(row[i]), i});
  } else {
    for (int i = t; i < V; i += 1024) a = am_better(a, ArgMax{bf2f(row[i]), i});
  }
  a = wave_argmax(a);
  if ((t & 63) == 0) sh[t >> 6] = a;
  __syncthreads();
  if (t == 0) {
    ArgMax r = sh[0];
    for (int i = 1; i < 16; ++i) r = am_better(r, sh[i]);
    out[(size_t)b * ld_out] = r.i == 0x7fffffff ? 0 : r.i;
  }
}

hipError_t argmax_rows(const bf16_t* logits, int ld, int V, int64_t* out, int ld_out, int B, hipStream_t s) {
  if (B <= 0 || V <= 0) return hipErrorInvalidValue;
  hipLaunchKernelGGL(argmax_rows_kernel, dim3(B), dim3(1024), 0, s, logits, ld, V, out, ld_out);
  return hipGetLastError();
}

// ---------------------------------------------------------------------------
// Channel token choice (:414-419).  Greedy channels: torch.argmax of the raw logits (no
// processors are attached when do_samples[i] is False).  Sampled channels run the HF
// processors in the reference's order (:360-368) on the bf16 logits, then
// multinomial(softmax):
//   RepetitionPenaltyLogitsProcessor (audio channels): over the row's channel history,
//     s < 0 ? s * p : s / p                                      (bf16 ops)
//   TemperatureLogitsWarper: s / T                               (bf16)
//   TopKLogitsWarper: keep s >= the k-th largest (ties kept)
//   TopPLogitsWarper: ascending sort, bf16 softmax, cumsum; drop cum <= bf16(1 - top_p),
//     the largest always kept
// The k-th largest is found by a two-pass radix select on the 16-bit order-preserving keys
// of the (bf16-exact) processed scores (topk.h, TIES_KEEP_ALL), so the whole vocab is never
// sorted; candidate sets past that list (no top_k on the text row, top_k > 1,024, threshold ties
// beyond TOPK_CAP) run the same processors as a walk over the 65,536 key bins
// (block_wide_draw_hf), so every reference-valid setting is served.  The draw uses
// Philox(seed; frame, row, channel): distribution-level parity (torch's RNG stream is not
// reproduced).
__global__ __launch_bounds__(1024) void local_pick_kernel(GenDev* __restrict__ st, const bf16_t* __restrict__ logits,
                                                          int ld, int V, int ch, const uint8_t* __restrict__ seen,
                                                          int64_t* __restrict__ next, int C, int* __restrict__ wide_hist) {
  __shared__ ArgMax sh[16];
  __shared__ TopkSmem sm;
  __shared__ float ev[TOPK_CAP];
  const int b = blockIdx.x, t = threadIdx.x;
  const bf16_t* row = logits + (size_t)b * ld;
  const ChSampling cs = st->lch[ch];
  if (!cs.sample) {
    ArgMax a{-INFINITY, 0x7fffffff};
    if ((ld & 7) == 0 && ((uintptr_t)row & 15) == 0) {  // 16-byte loads (the text channel: ~19 per thread instead of ~150 2-byte loads)
      const int nv = V >> 3;
      for (int c = t; c < nv; c += 1024) {
        float v[8];
        unpack8(*reinterpret_cast<const uint4*>(row + c * 8), v);
#pragma unroll
        for (int i = 0; i < 8; ++i) a = am_better(a, ArgMax{v[i], c * 8 + i});
      }
      for (int i = nv * 8 + t; i < V; i += 1024) a = am_better(a, ArgMax{bf2f(row[i]), i});
    } else {
      for (int i = t; i < V; i += 1024) a = am_better(a, ArgMax{bf2f(row[i]), i});
    }
    a = wave_argmax(a);
    if ((t & 63) == 0) sh[t >> 6] = a;
    __syncthreads();
    if (t == 0) {
      ArgMax r = sh[0];
      for (int i = 1; i < 16; ++i) r = am_better(r, sh[i]);
      next[(size_t)b * C + ch] = r.i == 0x7fffffff ? 0 : r.i;
    }
    return;
  }
  const float temp = cs.temp, pen = ch > 0 ? cs.pen : 1.0f, top_p = cs.top_p;
  const int top_k = cs.top_k;
  const uint8_t* sn = (ch > 0 && pen != 1.0f) ? seen + ((size_t)b * C + ch) * st->audio_rows : nullptr;
  auto val = [&](int i) -> float {
    float v = bf2f(row[i]);
    if (sn && sn[i]) v = v < 0.f ? rbf(v * pen) : rbf(v / pen);
    return rbf(v / temp);
  };
  const int K = top_k > 0 ? min(top_k, V) : V;
  const float u = philox_uniform(st->seed, (uint32_t)st->step, (uint32_t)b, (uint32_t)ch);
  // the sorted candidate list holds TOPK_CAP entries: K up to half of it leaves room for the
  // threshold ties (any K on rows that fit whole, e.g. the 1,025-code audio rows); a wider set
  // (no top_k on the text row, top_k > 1,024) or ties past TOPK_CAP take the key-bin walk
  bool wide = !(V <= TOPK_CAP || K <= TOPK_CAP / 2);
  int n = 0;
  if (!wide) {
    int over = 0;
    n = block_topk_sorted<1024>(val, V, K, TIES_KEEP_ALL, sm, &over);
    wide = over != 0;
  }
  if (wide) {
    const int tok = block_wide_draw_hf<1024>(val, V, top_k > 0 ? K : 0, top_p, u, wide_hist + (size_t)b * WIDE_BINS);
    if (t == 0) next[(size_t)b * C + ch] = tok < 0 ? 0 : tok;
    return;
  }
  if (n <= 0) {
    if (t == 0) next[(size_t)b * C + ch] = 0;
    return;
  }
  const float mx = cand_score(sm.cand[0]);
  for (int i = t; i < n; i += 1024) ev[i] = expf(cand_score(sm.cand[i]) - mx);
  __syncthreads();
  if (t == 0) {
    float S = 0.f;
    for (int i = 0; i < n; ++i) S += ev[i];
    // HF top-p on the ascending order: cum over candidates from the smallest up
    int keep = n;
    if (top_p < 1.0f) {
      const float thr_p = rbf((float)(1.0 - (double)top_p));
      float cum = 0.f;
      keep = 1;
      for (int i = n - 1; i >= 1; --i) {
        cum += rbf(ev[i] / S);
        if (rbf(cum) > thr_p) { keep = i + 1; break; }
      }
      // the ascending walk above met equal scores highest index first; torch.sort (the
      // reference's CPU path, and the oracle's stable argsort) drops the LOWEST indices of the tie
      // run the cut splits: reverse that run so the kept prefix holds its highest indices
      const unsigned long long kw = sm.cand[keep - 1] >> 32;
      if (keep < n && (sm.cand[keep] >> 32) == kw) {
        int a0 = keep - 1, b0 = keep;
        while (a0 > 0 && (sm.cand[a0 - 1] >> 32) == kw) --a0;
        while (b0 < n && (sm.cand[b0] >> 32) == kw) ++b0;
        for (int i = a0, j = b0 - 1; i < j; ++i, --j) {
          const unsigned long long x = sm.cand[i];
          sm.cand[i] = sm.cand[j];
          sm.cand[j] = x;
        }
      }
    }
    float S2 = 0.f;
    for (int i = 0; i < keep; ++i) S2 += ev[i];
    const float target = u * S2;
    float c = 0.f;
    int pick = cand_index(sm.cand[keep - 1]);
    for (int i = 0; i < keep; ++i) {
      c += ev[i];
      if (c > target) { pick = cand_index(sm.cand[i]); break; }
    }
    next[(size_t)b * C + ch] = pick;
  }
}

hipError_t local_pick(GenDev* st, const bf16_t* logits, int ld, int V, int ch, const uint8_t* seen, int64_t* next,
                      int C, int B, int* wide_hist, hipStream_t s) {
  if (B <= 0 || V <= 0 || !wide_hist) return hipErrorInvalidValue;
  hipLaunchKernelGGL(local_pick_kernel, dim3(B), dim3(1024), 0, s, st, logits, ld, V, ch, seen, next, C, wide_hist);
  return hipGetLastError();
}

// prompt rows into the generation buffer and the backbone key mask; rows start unfinished
__global__ void local_init_kernel(const int64_t* __restrict__ ids, const uint8_t* __restrict__ mask_in, int T, int C,
                                  int64_t* __restrict__ gen_ids, int Ltot, uint8_t* __restrict__ mask, int Cmax,
                                  int* __restrict__ finished, uint8_t* __restrict__ seen, int audio_rows) {
  const int b = blockIdx.x;
  for (int i = threadIdx.x; i < C * audio_rows; i += blockDim.x) seen[(size_t)b * C * audio_rows + i] = 0;
  __syncthreads();
  for (int i = threadIdx.x; i < T * C; i += blockDim.x) {
    const int64_t v = ids[(size_t)b * T * C + i];
    gen_ids[(size_t)b * Ltot * C + i] = v;
    const int c = i % C;  // the penalty's history: input_ids[..., c] incl. the prompt
    if (c > 0 && v >= 0 && v < audio_rows) seen[((size_t)b * C + c) * audio_rows + v] = 1;
  }
  for (int t = threadIdx.x; t < Cmax; t += blockDim.x)
    mask[(size_t)b * Cmax + t] = t < T ? (mask_in ? mask_in[(size_t)b * T + t] : (uint8_t)1) : (uint8_t)0;
  if (threadIdx.x == 0) finished[b] = 0;
}

hipError_t local_init(const int64_t* ids, const uint8_t* mask_in, int B, int T, int C, int64_t* gen_ids, int Ltot,
                      uint8_t* mask, int Cmax, int* finished, uint8_t* seen, int audio_rows, hipStream_t s) {
  hipLaunchKernelGGL(local_init_kernel, dim3(B), dim3(256), 0, s, ids, mask_in, T, C, gen_ids, Ltot, mask, Cmax, finished,
                     seen, audio_rows);
  return hipGetLastError();
}

// out[b] = masked columns of row b; a row whose masked columns do not all precede its first
// unmasked one (an interior or right pad) sets *bad: GenerationMixin's positions cumsum(mask) - 1
// equal slot - out[b] only for left padding
__global__ __launch_bounds__(256) void row_pad_count_kernel(const uint8_t* __restrict__ mask, int ld, int n,
                                                            int* __restrict__ out, int* __restrict__ bad) {
  const int b = blockIdx.x;
  int z = 0, first = n;
  for (int t = threadIdx.x; t < n; t += blockDim.x) {
    const bool m = mask[(size_t)b * ld + t] != 0;
    z += !m;
    if (m) first = min(first, t);
  }
  __shared__ int tot, fst;
  if (threadIdx.x == 0) { tot = 0; fst = n; }
  __syncthreads();
  atomicAdd(&tot, z);
  atomicMin(&fst, first);
  __syncthreads();
  if (threadIdx.x == 0) {
    out[b] = tot;
    if (bad && tot != fst && !(fst == n && tot == n)) atomicOr(bad, 1);
  }
}

hipError_t row_pad_count(const uint8_t* mask, int ld, int n, int B, int* out, int* bad, hipStream_t s) {
  if (B <= 0 || n < 0) return hipErrorInvalidValue;
  hipLaunchKernelGGL(row_pad_count_kernel, dim3(B), dim3(256), 0, s, mask, ld, n, out, bad);
  return hipGetLastError();
}

// End of a frame (:425-446): channels >= n_ch are 0; finished rows emit eos / pad; the frame
// is appended at column T0 + step and unmasked for the next forward; a row finishes on eos
// in channel 0.  One block, a thread per row.
__global__ __launch_bounds__(256) void local_finalize_kernel(GenDev* st, int64_t* __restrict__ next, int* __restrict__ finished,
                                                             int64_t* __restrict__ gen_ids, uint8_t* __restrict__ mask,
                                                             uint8_t* __restrict__ seen, int B, int C, int n_ch,
                                                             int eos, int pad) {
  __shared__ int alive;
  const int b = threadIdx.x;
  if (b == 0) alive = 0;
  __syncthreads();
  const int step = st->step, col = st->T0 + step;
  if (b < B) {
    const int fin = finished[b];
    int64_t* row = next + (size_t)b * C;
    int64_t* g = gen_ids + ((size_t)b * st->Ltot + col) * C;
    for (int i = 0; i < C; ++i) {
      int64_t v = i < n_ch ? row[i] : 0;
      if (fin) v = i == 0 ? eos : pad;
      row[i] = v;
      g[i] = v;
      if (i > 0 && v >= 0 && v < st->audio_rows) seen[((size_t)b * C + i) * st->audio_rows + v] = 1;
    }
    mask[(size_t)b * st->Cmax + col] = 1;
    const int f = fin | (row[0] == eos);
    finished[b] = f;
    if (!f) atomicOr(&alive, 1);
  }
  __syncthreads();
  if (b == 0) {
    if (!alive && st->done_step < 0) st->done_step = step;
    st->fwd_pos = col;
    st->step = step + 1;
  }
}

hipError_t local_finalize(GenDev* st, int64_t* next, int* finished, int64_t* gen_ids, uint8_t* mask, uint8_t* seen,
                          int B, int C, int n_ch, int eos, int pad, hipStream_t s) {
  if (B <= 0 || B > 256) return hipErrorInvalidValue;
  hipLaunchKernelGGL(local_finalize_kernel, dim3(1), dim3(256), 0, s, st, next, finished, gen_ids, mask, seen, B, C, n_ch,
                     eos, pad);
  return hipGetLastError();
}

}  // namespace mtts
