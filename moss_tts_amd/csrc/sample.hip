// Device-side generate() state machine and samplers for the delay pattern.
//
// Restates MossTTSDelayModel.generate (moss_tts_delay/modeling_moss_tts.py:417-516) without
// any device->host synchronisation: every boolean-mask update of the reference becomes a
// per-row predicate, so a whole decode step (forward + these kernels) is a fixed launch
// sequence that a hipGraph replays.  Sampling restates sample_token / apply_top_k /
// apply_top_p_optimized / apply_repetition_penalty_delay_pattern
// (moss_tts_delay/inference_utils.py:19-145).
//
// Per step:
//   score         (B, P + n_vq)   blocks y < P: top-K (K = 1 for greedy) of each text vocab slice,
//                                 special ids excluded (skipped when no row samples text freely);
//                                 y >= P: audio channel y-P: temperature, repetition penalty,
//                                 top-k/top-p, argmax | draw
//   text_select   (B)            merge partials + allowed special ids under the step's masks
//   finalize      (1 block)      state update, next input ids, generation buffer, mask, stop
#include "kernels.h"

namespace mtts {




// block-wide argmax (first index on ties) over 256 threads
__device__ ArgMax block_argmax(ArgMax a, ArgMax* sh) {
  a = wave_argmax(a);
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  __syncthreads();
  if (lane == 0) sh[w] = a;
  __syncthreads();
  ArgMax r = sh[0];
  for (int i = 1; i < 4; ++i) r = am_better(r, sh[i]);
  return r;
}

__device__ __forceinline__ bool is_special_text(int i, const MttsIds& d) {
  return i == d.pad || i == d.gen_slot || i == d.delay_slot || i == d.audio_end || i == d.im_end;
}

// bf16 logits / temperature rounded to bf16 (modeling_moss_tts.py:451)
__device__ __forceinline__ float scaled(bf16_t v, float temp) { return rbf(bf2f(v) / temp); }

// ---------------------------------------------------------------------------
// top-K of one text vocab slice (special ids excluded), K = 1 when greedy
__device__ void text_partial_body(const GenBufs& g, int b, int p) {
  const GenDev& st = *g.st;
  if (!st.need_text) return;  // every sampling row is in audio mode: partials unused
  const int K = st.text_sample ? min(st.text_top_k > 0 ? st.text_top_k : MAXK, MAXK) : 1;
  const int lo = p * st.part_len, hi = min(st.vocab, lo + st.part_len);
  const bf16_t* row = g.logits + (size_t)b * st.heads_ld;
  __shared__ float vals[4096];
  __shared__ ArgMax sh[4];
  const float temp = st.text_sample ? st.text_temp : 1.0f;
  const int n = hi - lo;
  for (int i = threadIdx.x; i < n; i += 256) {
    const int id = lo + i;
    vals[i] = is_special_text(id, st.ids) ? -INFINITY : scaled(row[id], temp);
  }
  __syncthreads();
  float* ov = g.part_val + ((size_t)b * st.P + p) * MAXK;
  int* oi = g.part_idx + ((size_t)b * st.P + p) * MAXK;
  for (int k = 0; k < K; ++k) {
    ArgMax a{-INFINITY, 0x7fffffff};
    for (int i = threadIdx.x; i < n; i += 256) a = am_better(a, ArgMax{vals[i], lo + i});
    a = block_argmax(a, sh);
    if (threadIdx.x == 0) {
      ov[k] = a.v;
      oi[k] = a.i;
    }
    if (a.i != 0x7fffffff && threadIdx.x == ((a.i - lo) & 255)) vals[a.i - lo] = -INFINITY;
    __syncthreads();
  }
}

// sample from (or argmax over) a candidate list sorted descending (val, idx).
// top-p restates apply_top_p_optimized (inference_utils.py:44-59): keep the smallest
// prefix whose cumulative probability exceeds p (the first candidate always kept).
__device__ int draw_sorted(const float* v, const int* idx, int n, float top_p, float u) {
  if (n <= 0) return idx[0];
  const float mx = v[0];
  float tot = 0.f;
  for (int i = 0; i < n; ++i) tot += (v[i] == -INFINITY) ? 0.f : expf(v[i] - mx);
  int keep = n;
  if (top_p < 1.0f) {
    float cum = 0.f;
    for (int i = 0; i < n; ++i) {
      const float p = (v[i] == -INFINITY) ? 0.f : expf(v[i] - mx) / tot;
      cum += p;
      if (cum > top_p) { keep = i + 1; break; }
    }
  }
  float t2 = 0.f;
  for (int i = 0; i < keep; ++i) t2 += (v[i] == -INFINITY) ? 0.f : expf(v[i] - mx);
  const float target = u * t2;
  float c = 0.f;
  for (int i = 0; i < keep; ++i) {
    c += (v[i] == -INFINITY) ? 0.f : expf(v[i] - mx);
    if (c > target) return idx[i];
  }
  return idx[keep - 1];
}

// text decision for rows that sample the text channel (modeling_moss_tts.py:453-471)
__global__ __launch_bounds__(256) void text_select_kernel(GenBufs g) {
  const GenDev& st = *g.st;
  const int b = blockIdx.x;
  const MttsIds& d = st.ids;
  const int step = st.step;
  const bool isa = g.is_audio[b] != 0;
  const bf16_t* row = g.logits + (size_t)b * st.heads_ld;
  const float temp = st.text_sample ? st.text_temp : 1.0f;
  __shared__ float cv[MAXK * 64 + 8];
  __shared__ int ci[MAXK * 64 + 8];
  __shared__ float sv[MAXK];
  __shared__ int si[MAXK];
  __shared__ ArgMax sh[4];
  const int K = st.text_sample ? min(st.text_top_k > 0 ? st.text_top_k : MAXK, MAXK) : 1;
  // candidates: general partials (only when not in audio mode) + allowed specials
  int nc = 0;
  if (!isa) {
    const int np = st.P * K;
    for (int i = threadIdx.x; i < np; i += 256) {
      const int p = i / K, k = i % K;
      cv[i] = g.part_val[((size_t)b * st.P + p) * MAXK + k];
      ci[i] = g.part_idx[((size_t)b * st.P + p) * MAXK + k];
    }
    nc = np;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    // masks: ~is_audio -> ban {pad, gen, delay, audio_end}; is_audio -> only {gen, delay};
    // step 0 bans delay (151662); step <= n_vq bans im_end  (:459-464)
    int k = nc;
    if (isa) {
      cv[k] = scaled(row[d.gen_slot], temp); ci[k++] = d.gen_slot;
      cv[k] = (step == 0) ? -INFINITY : scaled(row[d.delay_slot], temp); ci[k++] = d.delay_slot;
    } else {
      cv[k] = (step <= st.n_vq) ? -INFINITY : scaled(row[d.im_end], temp); ci[k++] = d.im_end;
    }
    sv[0] = (float)k;  // stash count
  }
  __syncthreads();
  const int ntot = (int)sv[0];
  __syncthreads();
  // select top-K of the candidates (iterative block argmax), sorted descending;
  // candidate token ids are unique (disjoint vocab slices + excluded specials)
  for (int k = 0; k < K; ++k) {
    ArgMax a{-INFINITY, 0x7fffffff};
    for (int i = threadIdx.x; i < ntot; i += 256) a = am_better(a, ArgMax{cv[i], ci[i]});
    const ArgMax r = block_argmax(a, sh);
    for (int i = threadIdx.x; i < ntot; i += 256)
      if (ci[i] == r.i) cv[i] = -INFINITY;
    if (threadIdx.x == 0) { sv[k] = r.v; si[k] = r.i; }
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    int tok;
    if (!st.text_sample) {
      tok = si[0];
    } else {
      const float u = philox_uniform(st.seed, (uint32_t)step, (uint32_t)b, 0u);
      tok = draw_sorted(sv, si, K, st.text_top_p, u);
    }
    g.text_cand[b] = tok;
  }
}

// audio channel j of row b: candidates over 1025 codes (modeling_moss_tts.py:483-503)
__device__ void audio_select_body(const GenBufs& g, int b, int j) {
  const GenDev& st = *g.st;
  const int V = st.audio_rows;
  const bf16_t* row = g.logits + (size_t)b * st.heads_ld + st.vocab + (size_t)j * V;
  const uint8_t* seen = g.seen + (j == 0 ? 0 : V);
  __shared__ float vals[1040];
  __shared__ ArgMax sh[4];
  __shared__ float sv[MAXK];
  __shared__ int si[MAXK];
  const float temp = st.audio_sample ? st.audio_temp : 1.0f;
  const float pen = st.rep_penalty;
  for (int i = threadIdx.x; i < V; i += 256) {
    float v = scaled(row[i], temp);
    if (i == st.ids.audio_pad) v = -INFINITY;  // :486-487
    if (pen != 1.0f && seen[i]) v = v > 0.f ? rbf(v / pen) : rbf(v * pen);  // inference_utils.py:79-88
    vals[i] = v;
  }
  __syncthreads();
  const int K = st.audio_sample ? min(st.audio_top_k > 0 ? st.audio_top_k : MAXK, MAXK) : 1;
  for (int k = 0; k < K; ++k) {
    ArgMax a{-INFINITY, 0x7fffffff};
    for (int i = threadIdx.x; i < V; i += 256) a = am_better(a, ArgMax{vals[i], i});
    a = block_argmax(a, sh);
    if (threadIdx.x == 0) { sv[k] = a.v; si[k] = a.i; }
    if (a.i != 0x7fffffff && threadIdx.x == (a.i & 255)) vals[a.i] = -INFINITY;
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    int tok;
    if (!st.audio_sample) tok = si[0];
    else {
      const float u = philox_uniform(st.seed, (uint32_t)st.step, (uint32_t)b, 1u + (uint32_t)j);
      tok = draw_sorted(sv, si, K, st.audio_top_p, u);
    }
    g.audio_cand[(size_t)b * st.n_vq + j] = tok;
  }
}

// state update (one block) -- modeling_moss_tts.py:453-516.  Phase 1: one thread per row
// updates the row's scalars; phase 2: one thread per (row, channel) writes the next input
// ids, the generation buffer and the repetition-penalty history.
constexpr int FIN_MAXB = 256;
__global__ __launch_bounds__(256) void finalize_kernel(GenBufs g) {
  GenDev& st = *g.st;
  const MttsIds& d = st.ids;
  const int n_vq = st.n_vq, C = st.C;
  const int step = st.step;
  const int col = st.T0 + step;
  __shared__ int n_stop, any_text;
  __shared__ int s_nt[FIN_MAXB];
  __shared__ int64_t s_al[FIN_MAXB], s_dl[FIN_MAXB];
  if (threadIdx.x == 0) n_stop = any_text = 0;
  __syncthreads();
  for (int b = threadIdx.x; b < st.B; b += blockDim.x) {
    bool stop = g.is_stopping[b] != 0;
    int64_t dl = g.delayed[b];
    int64_t al = g.audio_len[b];
    bool isa = g.is_audio[b] != 0;
    s_al[b] = al;  // channel masks use the counters before this step's update (:477-480)
    s_dl[b] = dl;
    int nt = d.pad;
    if (!stop && dl < n_vq) nt = d.delay_slot;
    const bool eos = !stop && dl == n_vq;
    if (eos) { nt = d.audio_end; isa = false; }
    const bool samp = !stop && dl > n_vq;
    if (samp) {
      nt = g.text_cand[b];
      if (g.forced && g.forced[step] >= 0) nt = g.forced[step];
    }
    if (nt == d.audio_start) isa = true;
    if (nt == d.im_end) stop = true;
    s_nt[b] = nt;
    if (nt == d.audio_start || nt == d.gen_slot || nt == d.delay_slot) al += 1;
    if (nt == d.audio_end) al = 0;
    if (dl == I64MAX && nt == d.delay_slot) dl = 0;
    if (dl != I64MAX) dl += 1;
    if (dl > n_vq) dl = I64MAX;
    g.is_stopping[b] = stop;
    g.is_audio[b] = isa;
    g.audio_len[b] = al;
    g.delayed[b] = dl;
    g.mask[(size_t)b * st.Cmax + col] = stop ? 0 : 1;
    if (stop) atomicAdd(&n_stop, 1);
    // next step samples this row's text channel over the full vocab (:453-471)
    if (!stop && dl > n_vq && !isa) atomicOr(&any_text, 1);
  }
  __syncthreads();
  for (int i = threadIdx.x; i < st.B * C; i += blockDim.x) {
    const int b = i / C, c = i - b * C;
    int tok;
    if (c == 0) {
      tok = s_nt[b];
    } else {
      const int j = c - 1;
      const bool pre = s_al[b] > j;
      const bool post = (s_dl[b] == I64MAX) || ((int64_t)j > s_dl[b] - 1);
      tok = (pre && post) ? g.audio_cand[(size_t)b * n_vq + j] : d.audio_pad;
      g.seen[(j == 0 ? 0 : st.audio_rows) + tok] = 1;
    }
    g.cur_ids[(size_t)b * C + c] = tok;
    g.gen_ids[((size_t)b * st.Ltot + col) * C + c] = tok;
  }
  if (threadIdx.x == 0) {
    if (st.need_text) st.text_head_steps += 1;
    st.need_text = any_text;
    if (n_stop == st.B && st.done_step < 0) st.done_step = step;
    st.fwd_pos = st.T0 + step;
    st.step = step + 1;
  }
}

// generate() prologue (modeling_moss_tts.py:417-440): per-row continuation state,
// copy of the prompt into the generation buffer / mask, audio history bitmaps.
__global__ __launch_bounds__(256) void gen_init_kernel(GenBufs g, const int64_t* ids, const uint8_t* mask_in) {
  GenDev& st = *g.st;
  const MttsIds& d = st.ids;
  const int T = st.T0, C = st.C;
  // copies (grid-stride over all threads of the one block)
  for (size_t i = threadIdx.x; i < (size_t)st.B * T * C; i += blockDim.x) {
    const size_t b = i / ((size_t)T * C), r = i % ((size_t)T * C);
    g.gen_ids[b * st.Ltot * C + r] = ids[i];
    const int c = (int)(r % C);
    if (c >= 1) {
      const int64_t tok = ids[i];
      if (tok >= 0 && tok < st.audio_rows) g.seen[(c == 1 ? 0 : st.audio_rows) + tok] = 1;
    }
  }
  for (size_t i = threadIdx.x; i < (size_t)st.B * T; i += blockDim.x) {
    const size_t b = i / T, t = i % T;
    g.mask[b * st.Cmax + t] = mask_in ? mask_in[i] : 1;
  }
  for (int b = threadIdx.x; b < st.B; b += blockDim.x) {
    const int64_t* row = ids + (size_t)b * T * C;
    const int64_t last = row[(size_t)(T - 1) * C];
    const bool cont = last == d.audio_start || last == d.gen_slot;
    int as = -1;
    for (int t = T - 1; t >= 0; --t)
      if (row[(size_t)t * C] == d.audio_start) { as = t; break; }  // find_last_equal_C
    const bool am = cont && as != -1;
    g.audio_len[b] = am ? (int64_t)(T - as) : 0;
    g.is_audio[b] = am;
    g.is_stopping[b] = 0;
    g.delayed[b] = I64MAX;
  }
  if (threadIdx.x == 0) {
    st.step = 0;
    st.done_step = -1;
    st.fwd_pos = 0;
    st.need_text = 1;  // step 0 samples from the prefill's full logits
    st.text_head_steps = 0;
  }
}

hipError_t gen_init(const GenBufs& g, const int64_t* ids, const uint8_t* mask, hipStream_t s) {
  hipLaunchKernelGGL(gen_init_kernel, dim3(1), dim3(256), 0, s, g, ids, mask);
  return hipGetLastError();
}

// one launch for the text vocab partials (blockIdx.y < P) and the n_vq audio channels
__global__ __launch_bounds__(256) void score_kernel(GenBufs g, int P) {
  if ((int)blockIdx.y < P) text_partial_body(g, blockIdx.x, blockIdx.y);
  else audio_select_body(g, blockIdx.x, blockIdx.y - P);
}

hipError_t sample_step(const GenBufs& g, int B, int n_vq, int P, hipStream_t s) {
  if (B > FIN_MAXB) return hipErrorInvalidValue;
  hipLaunchKernelGGL(score_kernel, dim3(B, P + n_vq), dim3(256), 0, s, g, P);
  hipLaunchKernelGGL(text_select_kernel, dim3(B), dim3(256), 0, s, g);
  hipLaunchKernelGGL(finalize_kernel, dim3(1), dim3(256), 0, s, g);
  return hipGetLastError();
}

}  // namespace mtts
