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
//   score         (B, P + n_vq)   blocks y < P: greedy text only -- argmax of each text vocab slice,
//                                 special ids excluded (skipped when no row samples text freely);
//                                 y >= P: audio channel y-P of the rows the step samples:
//                                 temperature, pad ban, repetition penalty, argmax | top-k ->
//                                 top-p -> draw
//   text_select   (B)            greedy: merge slice argmaxes + allowed special ids under the
//                                 step's masks; sampled: top-k over the whole masked row
//                                 (topk.h radix select), top-p, draw
//   finalize      (1 block)      state update, next input ids, generation buffer, mask, stop
// Draws: Philox(seed; step, row, channel) uniforms through torch's bf16 softmax / cumsum
// arithmetic (torch_draw); distribution-level parity, torch's RNG stream is not reproduced.
#include <algorithm>

#include "kernels.h"
#include "topk.h"

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
// greedy text: argmax of one text vocab slice (special ids excluded; they are merged by
// text_select under the step's masks).  Sampled text selects over the whole row in text_select.
__device__ void text_partial_body(const GenBufs& g, int b, int p) {
  const GenDev& st = *g.st;
  if (!st.need_text || st.text_sample) return;  // partials unused
  const int lo = p * st.part_len, hi = min(st.vocab, lo + st.part_len);
  const bf16_t* row = g.logits + (size_t)b * st.heads_ld;
  __shared__ ArgMax sh[4];
  ArgMax a{-INFINITY, 0x7fffffff};
  for (int id = lo + (int)threadIdx.x; id < hi; id += 256)
    if (!is_special_text(id, st.ids)) a = am_better(a, ArgMax{bf2f(row[id]), id});
  a = block_argmax(a, sh);
  if (threadIdx.x == 0) {
    g.part_val[(size_t)b * st.P + p] = a.v;
    g.part_idx[(size_t)b * st.P + p] = a.i;
  }
}

// torch's sample_token tail (inference_utils.py:129-145, apply_top_p_optimized :44-59) over
// the top-k candidates sorted by score (descending; index ascending among equal scores), the
// non-candidates being -inf.  ev[i] = exp(s_i - s_0) (fp32).  Every torch op here runs on
// bf16 tensors with fp32 internals:
//   probs = bf16(ev / S);  cum = bf16(fp32 cumsum of probs);  remove where cum > top_p,
//   shifted right by one (the first candidate always stays);
//   q = bf16(ev / S2) over the survivors;  multinomial(q) as an inverse CDF at u * sum(q).
// Returns the position of the drawn candidate.  One thread.
__device__ int torch_draw(const float* ev, int n, float top_p, float u) {
  float S = 0.f;
  for (int i = 0; i < n; ++i) S += ev[i];
  int keep = n;
  if (top_p < 1.0f) {
    float cum = 0.f;
    for (int i = 0; i < n; ++i) {
      cum += rbf(ev[i] / S);
      if (rbf(cum) > top_p) { keep = i + 1; break; }
    }
  }
  float S2 = 0.f;
  for (int i = 0; i < keep; ++i) S2 += ev[i];
  float Q = 0.f;
  for (int i = 0; i < keep; ++i) Q += rbf(ev[i] / S2);
  const float target = u * Q;
  float c = 0.f;
  for (int i = 0; i < keep; ++i) {
    c += rbf(ev[i] / S2);
    if (c > target) return i;
  }
  return keep - 1;
}

// candidates in sm.cand[0..n) -> exp terms (all threads), then the draw (thread 0)
template <int NT>
__device__ int draw_candidates(TopkSmem& sm, float* ev, int n, float top_p, float u) {
  if (n <= 0) return -1;
  const float mx = cand_score(sm.cand[0]);
  for (int i = threadIdx.x; i < n; i += NT) ev[i] = expf(cand_score(sm.cand[i]) - mx);
  __syncthreads();
  return threadIdx.x == 0 ? cand_index(sm.cand[torch_draw(ev, n, top_p, u)]) : -1;
}

// row b samples its text channel at this step (modeling_moss_tts.py:457)
__device__ __forceinline__ bool samples_text(const GenBufs& g, int b) {
  return g.is_stopping[b] == 0 && g.delayed[b] > (int64_t)g.st->n_vq;
}

// text decision for rows that sample the text channel (modeling_moss_tts.py:453-471).
//   greedy: merge the slice argmaxes with the allowed special ids;
//   sampled, audio mode: the two allowed ids {gen_slot, delay_slot} (delay banned at step 0);
//   sampled, text mode: top-k over the whole masked row (radix select), then top-p + draw.
constexpr int TSEL_NT = 1024;
__global__ __launch_bounds__(TSEL_NT) void text_select_kernel(GenBufs g) {
  const GenDev& st = *g.st;
  const int b = blockIdx.x, t = threadIdx.x;
  if (!samples_text(g, b)) return;  // finalize does not read text_cand for this row
  const MttsIds& d = st.ids;
  const int step = st.step;
  const bool isa = g.is_audio[b] != 0;
  const bf16_t* row = g.logits + (size_t)b * st.heads_ld;
  const float temp = st.text_sample ? st.text_temp : 1.0f;
  __shared__ TopkSmem sm;
  __shared__ float ev[TOPK_CAP];
  __shared__ ArgMax sh[TSEL_NT / 64];
  // masks: ~is_audio bans {pad, gen, delay, audio_end}; is_audio allows only {gen, delay};
  // step 0 bans 151662; step <= n_vq bans im_end (:459-464)
  const bool ban_im_end = step <= st.n_vq;
  if (!st.text_sample) {
    ArgMax a{-INFINITY, 0x7fffffff};
    if (isa) {
      if (t == 0) a = ArgMax{scaled(row[d.gen_slot], temp), d.gen_slot};
      if (t == 1 && step != 0) a = ArgMax{scaled(row[d.delay_slot], temp), d.delay_slot};
    } else {
      for (int p = t; p < st.P; p += TSEL_NT)
        a = am_better(a, ArgMax{g.part_val[(size_t)b * st.P + p], g.part_idx[(size_t)b * st.P + p]});
      if (t == 0 && !ban_im_end) a = am_better(a, ArgMax{scaled(row[d.im_end], temp), d.im_end});
    }
    a = wave_argmax(a);
    if ((t & 63) == 0) sh[t >> 6] = a;
    __syncthreads();
    if (t == 0) {
      ArgMax r = sh[0];
      for (int w = 1; w < TSEL_NT / 64; ++w) r = am_better(r, sh[w]);
      g.text_cand[b] = r.i == 0x7fffffff ? d.pad : r.i;
    }
    return;
  }
  const int K = st.text_top_k;  // <= 0: no top-k filter (inference_utils.py:136)
  int n;
  if (isa) {
    if (t == 0) {
      const float vg = scaled(row[d.gen_slot], temp);
      const float vd = step == 0 ? -INFINITY : scaled(row[d.delay_slot], temp);
      n = 0;
      if (vg > -INFINITY) sm.cand[n++] = cand_word(okey16(vg), d.gen_slot);
      if (vd > -INFINITY) sm.cand[n++] = cand_word(okey16(vd), d.delay_slot);
      if (n == 2 && sm.cand[1] < sm.cand[0]) { const auto x = sm.cand[0]; sm.cand[0] = sm.cand[1]; sm.cand[1] = x; }
      sm.s_n = K > 0 ? min(n, K) : n;
    }
    __syncthreads();
    n = sm.s_n;
  } else {
    auto val = [&](int i) -> float {
      if (i == d.pad || i == d.gen_slot || i == d.delay_slot || i == d.audio_end) return -INFINITY;
      if ((ban_im_end && i == d.im_end) || (step == 0 && i == 151662)) return -INFINITY;
      return scaled(row[i], temp);
    };
    if (K <= 0 || K > TOPK_CAP) {  // wide candidate set: key-bin form (topk.h block_wide_draw)
      const float u = philox_uniform(st.seed, (uint32_t)step, (uint32_t)b, 0u);
      const int tok = block_wide_draw<TSEL_NT>(val, st.vocab, K, st.text_top_p, u, g.wide_hist + (size_t)b * WIDE_BINS);
      if (t == 0) g.text_cand[b] = tok >= 0 ? tok : d.pad;
      return;
    }
    n = block_topk_sorted<TSEL_NT>(val, st.vocab, K, TIES_EXACT_K, sm, nullptr);
  }
  const float u = philox_uniform(st.seed, (uint32_t)step, (uint32_t)b, 0u);
  const int tok = draw_candidates<TSEL_NT>(sm, ev, n, st.text_top_p, u);
  if (t == 0) g.text_cand[b] = n > 0 ? tok : d.pad;
}

// audio channel j of row b (modeling_moss_tts.py:474-503): temperature, pad code banned,
// repetition penalty over the batch-wide history (inference_utils.py:79-88), then argmax or
// top-k (torch.topk) -> top-p -> draw.  Rows/channels the step does not sample are skipped.
__device__ void audio_select_body(const GenBufs& g, int b, int j) {
  const GenDev& st = *g.st;
  {
    const int64_t al = g.audio_len[b], dl = g.delayed[b];
    const bool pre = al > j, post = dl == I64MAX || (int64_t)j > dl - 1;  // :477-480
    if (!(pre && post)) return;
  }
  const int V = st.audio_rows;
  const bf16_t* row = g.logits + (size_t)b * st.heads_ld + st.vocab + (size_t)j * V;
  const uint8_t* seen = g.seen + (j == 0 ? 0 : V);
  const float temp = st.audio_sample ? st.audio_temp : 1.0f;
  const float pen = st.rep_penalty;
  const int pad = st.ids.audio_pad;
  auto val = [&](int i) -> float {
    if (i == pad) return -INFINITY;  // :486-487
    const float v = scaled(row[i], temp);
    return (pen != 1.0f && seen[i]) ? (v > 0.f ? rbf(v / pen) : rbf(v * pen)) : v;
  };
  if (!st.audio_sample) {
    __shared__ ArgMax sh[4];
    ArgMax a{-INFINITY, 0x7fffffff};
    for (int i = threadIdx.x; i < V; i += 256) a = am_better(a, ArgMax{val(i), i});
    a = block_argmax(a, sh);
    if (threadIdx.x == 0) g.audio_cand[(size_t)b * st.n_vq + j] = a.i == 0x7fffffff ? 0 : a.i;
    return;
  }
  __shared__ TopkSmem sm;
  __shared__ float ev[TOPK_CAP];
  const int K = st.audio_top_k > 0 ? st.audio_top_k : V;  // top_k <= 0: no top-k filter
  const int n = block_topk_sorted<256>(val, V, K, TIES_EXACT_K, sm, nullptr);
  const float u = philox_uniform(st.seed, (uint32_t)st.step, (uint32_t)b, 1u + (uint32_t)j);
  const int tok = draw_candidates<256>(sm, ev, n, st.audio_top_p, u);
  if (threadIdx.x == 0) g.audio_cand[(size_t)b * st.n_vq + j] = n > 0 ? tok : 0;
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
// Blocks [0, B): row b's state (the block scans the row for its last audio_start together -- one
// thread walking a 2,117-token prompt backwards took 0.6 ms); blocks from B: grid-stride copies.
__global__ __launch_bounds__(256) void gen_init_kernel(GenBufs g, const int64_t* ids, const uint8_t* mask_in) {
  GenDev& st = *g.st;
  const MttsIds& d = st.ids;
  const int T = st.T0, C = st.C, B = st.B;
  if ((int)blockIdx.x < B) {
    const int b = blockIdx.x;
    const int64_t* row = ids + (size_t)b * T * C;
    __shared__ int last_as;
    if (threadIdx.x == 0) last_as = -1;
    __syncthreads();
    int as = -1;
    for (int t = threadIdx.x; t < T; t += blockDim.x)
      if (row[(size_t)t * C] == d.audio_start) as = t;  // find_last_equal_C
    if (as >= 0) atomicMax(&last_as, as);
    __syncthreads();
    if (threadIdx.x == 0) {
      const int64_t last = row[(size_t)(T - 1) * C];
      const bool cont = last == d.audio_start || last == d.gen_slot;
      const bool am = cont && last_as != -1;
      g.audio_len[b] = am ? (int64_t)(T - last_as) : 0;
      g.is_audio[b] = am;
      g.is_stopping[b] = 0;
      g.delayed[b] = I64MAX;
      // step 0: every row samples its text channel; an audio-mode row reads only gen_slot /
      // delay_slot (the special-id tiles), so the prefill's full text head is needed only when
      // some row continues in text mode (need_text starts at 0, host-initialised; it gates the
      // prefill heads' text rows as it gates each decode step's)
      if (!am) atomicOr(&st.need_text, 1);
      if (b == 0) {
        st.step = 0;
        st.done_step = -1;
        st.fwd_pos = 0;
        st.text_head_steps = 0;
      }
    }
    return;
  }
  // copies (grid-stride over the copy blocks)
  const int nthr = (gridDim.x - B) * blockDim.x;
  const int tid = (blockIdx.x - B) * blockDim.x + threadIdx.x;
  const int TC = T * C;
  for (int i = tid; i < B * TC; i += nthr) {
    const int b = i / TC, r = i - b * TC;
    const int64_t tok = ids[i];
    g.gen_ids[(size_t)b * st.Ltot * C + r] = tok;
    const int c = r % C;
    if (c >= 1 && tok >= 0 && tok < st.audio_rows) g.seen[(c == 1 ? 0 : st.audio_rows) + tok] = 1;
  }
  for (int i = tid; i < B * T; i += nthr) {
    const int b = i / T, t = i - b * T;
    g.mask[(size_t)b * st.Cmax + t] = mask_in ? mask_in[i] : 1;
  }
}

hipError_t gen_init(const GenBufs& g, const int64_t* ids, const uint8_t* mask, int B, int T, int C, hipStream_t s) {
  const int copy_blocks = std::max(1, std::min(512, (B * T * C + 255) / 256));
  hipLaunchKernelGGL(gen_init_kernel, dim3(B + copy_blocks), dim3(256), 0, s, g, ids, mask);
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
  hipLaunchKernelGGL(text_select_kernel, dim3(B), dim3(TSEL_NT), 0, s, g);
  hipLaunchKernelGGL(finalize_kernel, dim3(1), dim3(256), 0, s, g);
  return hipGetLastError();
}

}  // namespace mtts
