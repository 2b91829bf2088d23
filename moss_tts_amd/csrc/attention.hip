// KV-cached grouped-query attention (decode and prefill), split over the context.
//
// Replaces sdpa_attention_forward (TF/integrations/sdpa_attention.py:79-166) with the
// causal + padding mask of TF/masking_utils.py: query token at absolute position p
// attends key j iff j <= p and mask[b][j].  Scores and softmax statistics are fp32;
// the un-normalised probabilities exp(s - max) are rounded to bf16 before P.V, as the
// reference's flash kernels do for bf16 (oracle/moss_delay.py attention()).
//
// Grid (n_split, Hkv, M): one block = one context chunk of CH keys for the G = Hq/Hkv
// query heads sharing one KV head (GQA), so each K/V row is read once per token.
// K/V rows (D*2 bytes) are read as 16-byte lane chunks, LPK = D/8 lanes per key.
// Partials (max, sum, unnormalised o) go to a workspace; attn_combine merges them.
#include <cstdlib>

#include "kernels.h"

namespace mtts {


template <int G>
__global__ __launch_bounds__(256) void attn_kernel(AttnArgs a) {
  extern __shared__ __attribute__((aligned(16))) float smem[];
  const int split = blockIdx.x, kvh = blockIdx.y, m = blockIdx.z;
  const int b = m / a.S, s = m % a.S;
  const int pos = *a.pos_base + s;
  const int ctx = pos + 1;
  const int c0 = split * a.CH;
  if (c0 >= ctx) return;
  const int c1 = min(ctx, c0 + a.CH);
  const int n = c1 - c0;
  const int D = a.D;
  const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
  float* q_s = smem;                 // [G][D]
  float* s_s = q_s + G * D;          // [G][CH]
  float* ml_s = s_s + G * a.CH;      // [G][2]
  float* red = smem + ((G * D + G * a.CH + 2 * G + 2 + 3) & ~3);  // [slots][G*D], 16B aligned (attn_smem_bytes)

  // q for the G heads of this KV head
  for (int e = t; e < G * D; e += 256) {
    const int h = e / D, d = e % D;
    q_s[e] = bf2f(a.q[(size_t)m * a.Hq * D + (size_t)(kvh * G + h) * D + d]);
  }
  __syncthreads();

  const int LPK = D >> 3;        // lanes per key
  const int KPW = 64 / LPK;      // keys per wave pass
  const int dl = (lane % LPK) * 8;
  const bf16_t* kbase = a.kc + ((size_t)b * a.Hkv + kvh) * a.Cmax * D;
  const bf16_t* vbase = a.vc + ((size_t)b * a.Hkv + kvh) * D * a.Cmax;  // V^T [D][Cmax]
  const uint8_t* mrow = a.mask + (size_t)b * a.Cmax;
  for (int kb = c0 + wave * KPW; kb < c1; kb += 4 * KPW) {
    const int key = kb + lane / LPK;
    const bool inr = key < c1;
    float kv[8];
    if (inr) unpack8(*reinterpret_cast<const uint4*>(kbase + (size_t)key * D + dl), kv);
    else {
#pragma unroll
      for (int i = 0; i < 8; ++i) kv[i] = 0.f;
    }
    const bool valid = inr && mrow[key];
#pragma unroll
    for (int h = 0; h < G; ++h) {
      float pd = 0.f;
#pragma unroll
      for (int i = 0; i < 8; ++i) pd += q_s[h * D + dl + i] * kv[i];
      for (int o = 1; o < LPK; o <<= 1) pd += __shfl_xor(pd, o, 64);
      if (inr && (lane % LPK) == 0) s_s[h * a.CH + (key - c0)] = valid ? pd * a.scale : -INFINITY;
    }
  }
  __syncthreads();

  // softmax statistics per head (one wave per head)
  for (int h = wave; h < G; h += 4) {
    float mx = -INFINITY;
    for (int i = lane; i < n; i += 64) mx = fmaxf(mx, s_s[h * a.CH + i]);
    mx = wave_max(mx);
    float l = 0.f;
    for (int i = lane; i < n; i += 64) {
      const float p = (mx == -INFINITY) ? 0.f : expf(s_s[h * a.CH + i] - mx);
      l += p;
      s_s[h * a.CH + i] = rbf(p);
    }
    l = wave_sum(l);
    if (lane == 0) {
      ml_s[2 * h] = mx;
      ml_s[2 * h + 1] = l;
    }
  }
  __syncthreads();

  // P.V: slot = key lane group, 8 dims per thread
  const int slots = 256 / LPK;
  const int slot = t / LPK;
  const int dd = (t % LPK) * 8;
  float acc[G][8];
#pragma unroll
  for (int h = 0; h < G; ++h)
#pragma unroll
    for (int i = 0; i < 8; ++i) acc[h][i] = 0.f;
  for (int key = c0 + slot; key < c1; key += slots) {
    float vv[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) vv[i] = bf2f(vbase[(size_t)(dd + i) * a.Cmax + key]);
#pragma unroll
    for (int h = 0; h < G; ++h) {
      const float p = s_s[h * a.CH + (key - c0)];
#pragma unroll
      for (int i = 0; i < 8; ++i) acc[h][i] += p * vv[i];
    }
  }
#pragma unroll
  for (int h = 0; h < G; ++h)
#pragma unroll
    for (int i = 0; i < 8; ++i) red[(size_t)slot * G * D + h * D + dd + i] = acc[h][i];
  __syncthreads();
  for (int e = t; e < G * D; e += 256) {
    float o = 0.f;
    for (int sl = 0; sl < slots; ++sl) o += red[(size_t)sl * G * D + e];
    const int h = e / D, d = e % D;
    const int hq = kvh * G + h;
    const size_t pidx = ((size_t)m * a.n_split + split) * a.Hq + hq;
    a.part_o[pidx * D + d] = o;
    if (d == 0) {
      a.part_ml[pidx * 2] = ml_s[2 * h];
      a.part_ml[pidx * 2 + 1] = ml_s[2 * h + 1];
    }
  }
}

// merge the context chunks of one (token, q-head): one wave, lanes over D
__global__ __launch_bounds__(256) void attn_combine_kernel(AttnArgs a) {
  const int gw = blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (gw >= a.M * a.Hq) return;
  const int m = gw / a.Hq, hq = gw % a.Hq;
  const int s = m % a.S;
  const int ctx = *a.pos_base + s + 1;
  const int nu = min(a.n_split, (ctx + a.CH - 1) / a.CH);
  float M = -INFINITY;
  for (int sp = 0; sp < nu; ++sp) M = fmaxf(M, a.part_ml[(((size_t)m * a.n_split + sp) * a.Hq + hq) * 2]);
  float L = 0.f;
  float o0 = 0.f, o1 = 0.f;
  const int D = a.D;
  for (int sp = 0; sp < nu; ++sp) {
    const size_t pidx = ((size_t)m * a.n_split + sp) * a.Hq + hq;
    const float ms = a.part_ml[pidx * 2];
    const float w = (ms == -INFINITY) ? 0.f : expf(ms - M);
    L += w * a.part_ml[pidx * 2 + 1];
    if (2 * lane < D) {
      o0 += w * a.part_o[pidx * D + 2 * lane];
      o1 += w * a.part_o[pidx * D + 2 * lane + 1];
    }
  }
  const float inv = L > 0.f ? 1.0f / L : 0.f;
  if (2 * lane < D) {
    bf16_t* dst = a.out + (size_t)m * a.Hq * D + (size_t)hq * D + 2 * lane;
    *reinterpret_cast<uint32_t*>(dst) = pack2(o0 * inv, o1 * inv);
  }
}

// ---------------------------------------------------------------------------
// Prefill attention, flash form on MFMA.  Grid (16-token query tile, KV head, row b); one
// wave per query head of the GQA group, so the G waves of a block read the same K / V^T
// tiles (through L1).  Per 32-key chunk a wave computes
//   S[16 tokens][32 keys] = Q[16 x D] . K^T          (v_mfma_f32_16x16x32_bf16, B = K rows)
// with the causal + padding mask, an online softmax per token row (probabilities rounded
// to bf16 before P.V, fp32 statistics), and
//   O[16 tokens][D] = O * alpha + P[16 x 32] . V[32 x D]  (P through LDS, V^T from the cache)
// so each K/V byte is read once per 16 tokens x G heads instead of once per token.
template <int G, int D>
__global__ __launch_bounds__(G * 64) void attn_prefill_kernel(AttnArgs a) {
  constexpr int QS = (D + 31) / 32, DT = (D + 15) / 16;  // dims beyond D are zero-filled
  const int qt = blockIdx.x, kvh = blockIdx.y, b = blockIdx.z;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int g4 = lane >> 4, c16 = lane & 15;
  const int hq = kvh * G + wave;
  const int s0 = qt * 16;                       // first token of the tile (within the row)
  const int pos0 = *a.pos_base + s0;            // its absolute position
  const int last = min(a.S - 1, s0 + 15);
  const int kend = *a.pos_base + last;          // last key any token of the tile sees
  const int Cmax = a.Cmax;
  __shared__ __attribute__((aligned(16))) bf16_t p_s[G][16][32];
  const bf16_t* kbase = a.kc + ((size_t)b * a.Hkv + kvh) * Cmax * D;
  const bf16_t* vbase = a.vc + ((size_t)b * a.Hkv + kvh) * D * Cmax;
  const uint8_t* mrow = a.mask + (size_t)b * Cmax;

  // Q A-operand fragments: token s0 + (lane & 15), dims st*32 + 8*(lane>>4) .. +7
  bf16x8 qf[QS];
  {
    const int tq = min(s0 + c16, a.S - 1);
    const bf16_t* qrow = a.q + ((size_t)b * a.S + tq) * a.Hq * D + (size_t)hq * D;
#pragma unroll
    for (int st = 0; st < QS; ++st)
      qf[st] = st * 32 + 8 * g4 < D ? *reinterpret_cast<const bf16x8*>(qrow + st * 32 + 8 * g4)
                                    : __builtin_bit_cast(bf16x8, (u32x4){0u, 0u, 0u, 0u});
  }
  // this lane's output rows: tokens s0 + g4*4 + i
  float m_run[4], l_run[4];
  f32x4 o_run[DT];
#pragma unroll
  for (int i = 0; i < 4; ++i) { m_run[i] = -INFINITY; l_run[i] = 0.f; }
#pragma unroll
  for (int dt = 0; dt < DT; ++dt) o_run[dt] = (f32x4){0.f, 0.f, 0.f, 0.f};

  // K / V^T / mask of a 32-key chunk: branch-free buffer loads (keys past kend read zero through
  // an out-of-range offset), so the next chunk's loads are in flight while this one computes
  constexpr uint32_t OOBA = 0x7ffffff0u;
  const __amdgpu_buffer_rsrc_t krs = __builtin_amdgcn_make_buffer_rsrc(const_cast<bf16_t*>(kbase), 0, Cmax * D * 2, 0x00020000);
  const __amdgpu_buffer_rsrc_t vrs = __builtin_amdgcn_make_buffer_rsrc(const_cast<bf16_t*>(vbase), 0, Cmax * D * 2, 0x00020000);
  const __amdgpu_buffer_rsrc_t mrs = __builtin_amdgcn_make_buffer_rsrc(const_cast<uint8_t*>(mrow), 0, Cmax, 0x00020000);
  auto load_chunk = [&](int k0, u32x4 (&kf)[2][QS], u32x4 (&vt)[DT], uint32_t (&mk)[2]) {
#pragma unroll
    for (int t = 0; t < 2; ++t) {
      const int key = k0 + t * 16 + c16;
      const bool ok = key <= kend;
      mk[t] = __builtin_amdgcn_raw_buffer_load_b8(mrs, ok ? (uint32_t)key : OOBA, 0, 0);
#pragma unroll
      for (int st = 0; st < QS; ++st)
        kf[t][st] = __builtin_amdgcn_raw_buffer_load_b128(
            krs, (ok && st * 32 + 8 * g4 < D) ? (uint32_t)(key * D + st * 32 + 8 * g4) * 2u : OOBA, 0, 0);
    }
#pragma unroll
    for (int dt = 0; dt < DT; ++dt) {
      const int kb = k0 + 8 * g4;
      vt[dt] = __builtin_amdgcn_raw_buffer_load_b128(vrs, kb <= kend ? (uint32_t)((dt * 16 + c16) * Cmax + kb) * 2u : OOBA,
                                                     0, 0);
    }
  };
  auto compute = [&](int k0, const u32x4 (&kf)[2][QS], u32x4 (&vt)[DT], const uint32_t (&mk)[2]) {
    // ---- S = Q . K^T for keys k0 .. k0+31 (two 16-key tiles) ----
    f32x4 sacc[2];
#pragma unroll
    for (int t = 0; t < 2; ++t) {
      sacc[t] = (f32x4){0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int st = 0; st < QS; ++st)
        sacc[t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(qf[st], __builtin_bit_cast(bf16x8, kf[t][st]), sacc[t], 0, 0, 0);
    }
    // V^T B-operand fragments: dim dt*16 + c16, keys k0 + 8*g4 .. +7; keys past kend zeroed (cache
    // rows not yet written: 0 * NaN in the P.V MFMA would be NaN)
    {
      const int nv = kend + 1 - (k0 + 8 * g4);
      uint32_t vm[4];
#pragma unroll
      for (int q = 0; q < 4; ++q) vm[q] = (2 * q < nv ? 0x0000ffffu : 0u) | (2 * q + 1 < nv ? 0xffff0000u : 0u);
#pragma unroll
      for (int dt = 0; dt < DT; ++dt)
#pragma unroll
        for (int q = 0; q < 4; ++q) vt[dt][q] &= vm[q];
    }
    // ---- online softmax per token row (row = g4*4 + i, keys over the 16-lane group) ----
    float alpha[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int pq = pos0 + g4 * 4 + i;
      float sv[2];
      float mc = -INFINITY;
#pragma unroll
      for (int t = 0; t < 2; ++t) {
        const int key = k0 + t * 16 + c16;
        sv[t] = (key <= pq && mk[t]) ? sacc[t][i] * a.scale : -INFINITY;
        mc = fmaxf(mc, sv[t]);
      }
#pragma unroll
      for (int o = 1; o < 16; o <<= 1) mc = fmaxf(mc, __shfl_xor(mc, o, 64));
      const float mn = fmaxf(m_run[i], mc);
      alpha[i] = (m_run[i] == -INFINITY) ? (mn == -INFINITY ? 1.f : 0.f) : expf(m_run[i] - mn);
      float lc = 0.f;
#pragma unroll
      for (int t = 0; t < 2; ++t) {
        const float p = (mn == -INFINITY || sv[t] == -INFINITY) ? 0.f : expf(sv[t] - mn);
        lc += p;
        p_s[wave][g4 * 4 + i][t * 16 + c16] = f2bf(p);  // bf16-rounded probabilities
      }
#pragma unroll
      for (int o = 1; o < 16; o <<= 1) lc += __shfl_xor(lc, o, 64);
      l_run[i] = l_run[i] * alpha[i] + lc;
      m_run[i] = mn;
    }
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
    // ---- O = O * alpha + P . V (accumulated in the MFMA) ----
    const bf16x8 pf = *reinterpret_cast<const bf16x8*>(&p_s[wave][c16][8 * g4]);
#pragma unroll
    for (int dt = 0; dt < DT; ++dt) {
      f32x4 o4 = o_run[dt];
#pragma unroll
      for (int i = 0; i < 4; ++i) o4[i] *= alpha[i];
      o_run[dt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(pf, __builtin_bit_cast(bf16x8, vt[dt]), o4, 0, 0, 0);
    }
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
  };
  u32x4 kA[2][QS], vA[DT];
  uint32_t mA[2];
  load_chunk(0, kA, vA, mA);
  if constexpr (G <= 4) {
    // two chunks per iteration, each one's loads issued while the other computes (256 VGPRs: two
    // waves per SIMD; 8-wave blocks keep one chunk in flight)
    u32x4 kB[2][QS], vB[DT];
    uint32_t mB[2];
    for (int k0 = 0; k0 <= kend; k0 += 64) {
      if (k0 + 32 <= kend) load_chunk(k0 + 32, kB, vB, mB);
      compute(k0, kA, vA, mA);
      if (k0 + 32 > kend) break;
      if (k0 + 64 <= kend) load_chunk(k0 + 64, kA, vA, mA);
      compute(k0 + 32, kB, vB, mB);
    }
  } else {
    for (int k0 = 0; k0 <= kend; k0 += 32) {
      if (k0 > 0) load_chunk(k0, kA, vA, mA);
      compute(k0, kA, vA, mA);
    }
  }
  // ---- normalise and store: token s0 + g4*4 + i, dims dt*16 + c16 ----
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int tq = s0 + g4 * 4 + i;
    if (tq >= a.S) continue;
    const int mrow = b * a.S + tq;
    bf16_t* dst = a.out + (size_t)mrow * a.Hq * D + (size_t)hq * D;
#pragma unroll
    for (int dt = 0; dt < DT; ++dt) {
      const bf16_t v = f2bf(l_run[i] > 0.f ? o_run[dt][i] / l_run[i] : 0.f);
      if (a.out_tiles) a.out[xpkT_index(mrow, hq * D + dt * 16 + c16, a.out_tiles)] = v;
      else dst[dt * 16 + c16] = v;
    }
  }
}

// ---------------------------------------------------------------------------
// Long prompts (round 5): 32-token query tiles with the K / V^T chunks staged ONCE per block in
// LDS.  The 16-token form above has each of its G waves load the chunk's K / V^T fragments itself
// (16 KiB per wave per 32-key chunk, 16 MFMAs), and re-reads every key once per 16 tokens: at the
// TTSD script's 2,117 tokens the attention took 445 us a layer (36.7 GFLOP: 3 % of the MFMA peak,
// profiles/r05_h_prefill_*).  Here the block's 256 threads copy a 32-key chunk (K [32][D] and
// V^T [D][32], 16 KiB) global -> LDS by LDS-DMA into one of two buffers while the waves run the
// other, and each wave (one query head) computes 2 tiles of 16 tokens from those LDS tiles.
//
// The products run transposed, S^T = K . Q^T and O^T = V^T . P^T, so that every lane owns ONE
// token column of each tile and 8 of the chunk's keys: the softmax statistics are per-lane scalars
// (in-lane max over 8 keys + 2 cross-lane steps, one alpha per token), the probabilities feed the
// P.V MFMA straight from the S^T accumulators, and chunks wholly below the diagonal with no
// padding skip the mask arithmetic.  K rows enter the S^T tiles permuted (tile t, row r <- key
// 8 (r >> 2) + 4 t + (r & 3)) so that lane (g4, c16) ends up holding keys 8 g4 .. 8 g4 + 7: the
// contiguous k-slice the P^T B operand and the V^T A operand (one 16-B LDS read) need.  A first straight form (scores per token row, P through LDS) measured ~1,100 VALU
// instructions per chunk against 32 MFMAs and ran at 310 us a layer.
// Arithmetic as above: scores and statistics fp32 (exp via exp2 of log2e-scaled scores),
// probabilities rounded to bf16 before P.V, the row sum over the unrounded ones.
// max / sum of a value over lanes l, l ^ 16, l ^ 32, l ^ 48 (gfx950 row swaps, no LDS round trip)
__device__ __forceinline__ float pf_max3(float a, float b, float c) {
  float r;  // (fmaxf would canonicalise every MFMA / permlane result first)
  asm("v_max3_f32 %0, %1, %2, %3" : "=v"(r) : "v"(a), "v"(b), "v"(c));
  return r;
}
__device__ __forceinline__ float pf_xmax(float v) {
  auto r = __builtin_amdgcn_permlane16_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  v = pf_max3(__uint_as_float(r[0]), __uint_as_float(r[1]), __uint_as_float(r[1]));
  auto q = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  return pf_max3(__uint_as_float(q[0]), __uint_as_float(q[1]), __uint_as_float(q[1]));
}
__device__ __forceinline__ float pf_xsum(float v) {
  auto r = __builtin_amdgcn_permlane16_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  v = __uint_as_float(r[0]) + __uint_as_float(r[1]);
  auto q = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  return __uint_as_float(q[0]) + __uint_as_float(q[1]);
}
__device__ __forceinline__ uint32_t pf_pack(float a, float b) {  // one v_cvt_pk_bf16_f32 (RNE)
  typedef __attribute__((ext_vector_type(2))) float f2;
  typedef __attribute__((ext_vector_type(2))) __bf16 h2;
  return __builtin_bit_cast(uint32_t, __builtin_convertvector((f2){a, b}, h2));
}

template <int G, int D>
__global__ __launch_bounds__(G * 64, 2) void attn_prefill32_kernel(AttnArgs a) {
  static_assert(D == 128 && (G == 4 || G == 2), "the 8B (4 q heads per KV head) / 1.7B (2) head shapes");
  typedef __attribute__((address_space(3))) void lvoid;
  constexpr int QS = D / 32, DT = D / 16, TQ = 32, RT = TQ / 16;
  // the causal tiles' work grows with qt: dispatch the longest first
  const int qt = gridDim.x - 1 - blockIdx.x, kvh = blockIdx.y, b = blockIdx.z;
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int g4 = lane >> 4, c16 = lane & 15;
  const int hq = kvh * G + wave;
  const int s0 = qt * TQ;
  const int pos0 = *a.pos_base + s0;
  const int last = min(a.S - 1, s0 + TQ - 1);
  const int kend = *a.pos_base + last;  // last key any token of the tile sees
  const int Cmax = a.Cmax;
  // one dynamic LDS block (PF32_LDS bytes): with static arrays the compiler cannot tell the two
  // buffers apart and waits for the prefetch in flight before every LDS read of the chunk in use
  extern __shared__ __attribute__((aligned(16))) unsigned char pf_lds[];
  auto ks = reinterpret_cast<bf16_t(*)[32][D]>(pf_lds);                   // [buf][key][dim]
  auto vs = reinterpret_cast<bf16_t(*)[D][32]>(pf_lds + 2 * 32 * D * 2);  // [buf][dim][key]
  auto ms = reinterpret_cast<uint32_t(*)[64]>(pf_lds + 4 * 32 * D * 2);   // [buf] mask bytes
  const bf16_t* kbase = a.kc + ((size_t)b * a.Hkv + kvh) * Cmax * D;
  const bf16_t* vbase = a.vc + ((size_t)b * a.Hkv + kvh) * D * Cmax;
  const uint8_t* mrow = a.mask + (size_t)b * Cmax;
  const __amdgpu_buffer_rsrc_t krs = __builtin_amdgcn_make_buffer_rsrc(const_cast<bf16_t*>(kbase), 0, Cmax * D * 2, 0x00020000);
  const __amdgpu_buffer_rsrc_t vrs = __builtin_amdgcn_make_buffer_rsrc(const_cast<bf16_t*>(vbase), 0, Cmax * D * 2, 0x00020000);
  const __amdgpu_buffer_rsrc_t mrs = __builtin_amdgcn_make_buffer_rsrc(const_cast<uint8_t*>(mrow), 0, Cmax, 0x00020000);
  constexpr uint32_t OOBA = 0x7ffffff0u;
  // chunk k0 -> LDS buffer buf: each wave 2 KiB of K (keys 8 w .. 8 w + 7) and 2 KiB of V^T (dims
  // 32 w .. 32 w + 31, 64 B each), 1 KiB per LDS-DMA instruction (lane l: 16 B at lds + 16 l).
  // Bank swizzle on the SOURCE side (the LDS-DMA destination is fixed per lane): K row r holds
  // its 16-B piece j at slot j ^ kswz(r), V^T row d its piece j at slot j ^ ((d >> 2) & 3), so
  // the fragment reads below (16 rows per 16 lanes) spread over all 64 banks.
  // distinct over each S^T tile's 16 keys (bits 0, 1, 3, 4 of the key's row in the chunk)
  auto kswz = [](int r) { return (r & 3) | ((r >> 1) & 12); };
  // (G waves split the chunk: 32 / G keys and 128 / G V^T rows each, 8 / G instructions of each)
  auto issue = [&](int k0, int buf) {
#pragma unroll
    for (int i = 0; i < 8 / G; ++i) {
      const int kr = wave * (32 / G) + i * 4 + (lane >> 4);  // 4 keys (256 B each) per instruction
      const int key = k0 + kr;
      __builtin_amdgcn_raw_ptr_buffer_load_lds(
          krs, (lvoid*)&ks[buf][wave * (32 / G) + i * 4][0], 16,
          (key < Cmax) ? (uint32_t)(key * D * 2 + ((lane & 15) ^ kswz(kr)) * 16) : OOBA, 0, 0, 0);
      const int d = wave * (D / G) + i * 16 + (lane >> 2);  // 16 dims (64 B each) per instruction
      __builtin_amdgcn_raw_ptr_buffer_load_lds(
          vrs, (lvoid*)&vs[buf][wave * (D / G) + i * 16][0], 16,
          (k0 + 32 <= Cmax) ? (uint32_t)((d * Cmax + k0) * 2 + ((lane & 3) ^ ((d >> 2) & 3)) * 16) : OOBA, 0, 0, 0);
    }
    // the chunk's 32 mask bytes ride with it (a register load here would make the waitcnt before
    // its first use also wait for the chunk prefetched after it)
    if (wave == 0)
      __builtin_amdgcn_raw_ptr_buffer_load_lds(mrs, (lvoid*)&ms[buf][0], 4,
                                               lane < 8 ? (uint32_t)(k0 + 4 * lane) : OOBA, 0, 0, 0);
  };
  // Q B-operand fragments of the 2 token tiles: token s0 + 16 rt + c16, dims 32 st + 8 g4 ..
  bf16x8 qf[RT][QS];
#pragma unroll
  for (int rt = 0; rt < RT; ++rt) {
    const int tq = min(s0 + rt * 16 + c16, a.S - 1);
    const bf16_t* qrow = a.q + ((size_t)b * a.S + tq) * a.Hq * D + (size_t)hq * D;
#pragma unroll
    for (int st = 0; st < QS; ++st) qf[rt][st] = *reinterpret_cast<const bf16x8*>(qrow + st * 32 + 8 * g4);
  }
  const float sc2 = a.scale * 1.4426950408889634f;  // scores in log2 units
  // this lane's token of tile rt sees keys <= pq[rt] (capped at kend: keys past the prompt are
  // never written before the read)
  int pq[RT];
#pragma unroll
  for (int rt = 0; rt < RT; ++rt) pq[rt] = min(pos0 + rt * 16 + c16, kend);
  // m: running max (log2 units; -1e30 stands for "none yet" so fully masked tokens stay finite
  // and end with l = 0), l: this lane's partial of the row sum (reduced over g4 at the end)
  float m_run[RT], l_run[RT];
  f32x4 o_run[DT][RT];
#pragma unroll
  for (int rt = 0; rt < RT; ++rt) {
    m_run[rt] = -1e30f;
    l_run[rt] = 0.f;
#pragma unroll
    for (int dt = 0; dt < DT; ++dt) o_run[dt][rt] = (f32x4){0.f, 0.f, 0.f, 0.f};
  }
  const int nch = kend / 32 + 1;
  issue(0, 0);
  for (int c = 0; c < nch; ++c) {
    const int k0 = c * 32, buf = c & 1;
    // chunk c has landed for every wave; buffer buf ^ 1 was last read in iteration c - 1
    asm volatile("s_waitcnt vmcnt(0)\n\ts_barrier" ::: "memory");
    if (c + 1 < nch) issue(k0 + 32, buf ^ 1);
    // ---- S^T = K . Q^T: K A-operand row c16 of tile t = key 8 (c16 >> 2) + 4 t + (c16 & 3) of
    // the chunk, dims 32 st + 8 g4 .. ----
    f32x4 sacc[2][RT];
#pragma unroll
    for (int t = 0; t < 2; ++t) {
      const int kr = 8 * (c16 >> 2) + 4 * t + (c16 & 3);
      u32x4 kf[QS];
#pragma unroll
      for (int st = 0; st < QS; ++st) kf[st] = *reinterpret_cast<const u32x4*>(&ks[buf][kr][((st * 4 + g4) ^ kswz(kr)) * 8]);
#pragma unroll
      for (int rt = 0; rt < RT; ++rt) {
        sacc[t][rt] = (f32x4){0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int st = 0; st < QS; ++st)
          sacc[t][rt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, kf[st]), qf[rt][st],
                                                                sacc[t][rt], 0, 0, 0);
      }
    }
    // lane (g4, c16) holds scores of keys k0 + 8 g4 + 4 t + i for token tile rt column c16
    const uint32_t mw0 = ms[buf][2 * g4], mw1 = ms[buf][2 * g4 + 1];  // mask bytes of its 8 keys
    auto has_zero = [](uint32_t w) { return ((w - 0x01010101u) & ~w & 0x80808080u) != 0u; };
    const bool full = (k0 + 31 <= pos0) && !__builtin_amdgcn_ballot_w64(has_zero(mw0) || has_zero(mw1));
    // (the asm markers keep the two rare paths below as wave-uniform branches: without them the
    // compiler speculates the masking into selects on every chunk)
    // statistics in raw score units (the scale is > 0); exp2 of fma(s, sc2, -m sc2)
    float alpha[RT];
    bf16x8 pf[RT];
    if (!full) {  // diagonal / padded chunks
      asm volatile("; masked chunk");
#pragma unroll
      for (int rt = 0; rt < RT; ++rt)
#pragma unroll
        for (int t = 0; t < 2; ++t)
#pragma unroll
          for (int i = 0; i < 4; ++i) {
            const int key = k0 + 8 * g4 + 4 * t + i;
            const uint32_t mb = ((t ? mw1 : mw0) >> (8 * i)) & 0xffu;
            if (!(key <= pq[rt] && mb)) sacc[t][rt][i] = -INFINITY;
          }
    }
#pragma unroll
    for (int rt = 0; rt < RT; ++rt) {
      const float m1 = pf_max3(sacc[0][rt][0], sacc[0][rt][1], sacc[0][rt][2]);
      const float m2 = pf_max3(sacc[0][rt][3], sacc[1][rt][0], sacc[1][rt][1]);
      const float mc = pf_xmax(pf_max3(m1, m2, pf_max3(sacc[1][rt][2], sacc[1][rt][3], m_run[rt])));
      const float mn = mc;  // (m_run folded into the max)
      alpha[rt] = __builtin_amdgcn_exp2f((m_run[rt] - mn) * sc2);
      m_run[rt] = mn;
      const float nm = -mn * sc2;
      float lc = 0.f;
      uint32_t pw[4];
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const float p0 = __builtin_amdgcn_exp2f(fmaf(sacc[k >> 1][rt][2 * (k & 1)], sc2, nm));
        const float p1 = __builtin_amdgcn_exp2f(fmaf(sacc[k >> 1][rt][2 * (k & 1) + 1], sc2, nm));
        lc += p0 + p1;
        pw[k] = pf_pack(p0, p1);  // bf16-rounded probabilities
      }
      l_run[rt] = l_run[rt] * alpha[rt] + lc;
      pf[rt] = __builtin_bit_cast(bf16x8, (u32x4){pw[0], pw[1], pw[2], pw[3]});
    }
    // the running max rarely moves once a few chunks are in: rescale O only when it did
    if (__builtin_amdgcn_ballot_w64(alpha[0] != 1.f || alpha[1] != 1.f)) {
      asm volatile("; rescale");
#pragma unroll
      for (int dt = 0; dt < DT; ++dt)
#pragma unroll
        for (int rt = 0; rt < RT; ++rt)
#pragma unroll
          for (int i = 0; i < 4; ++i) o_run[dt][rt][i] *= alpha[rt];
    }
    // ---- O^T += V^T . P^T; V^T A-operand (dim dt*16 + c16, keys 8 g4 .. 8 g4 + 7: 16-B piece
    // g4, stored at slot g4 ^ ((d >> 2) & 3)); in the chunk holding kend, keys past it zeroed
    // (cache rows not yet written: 0 * NaN in the MFMA would be NaN) ----
    const bool tail = k0 + 31 > kend;
    uint32_t vm[4] = {~0u, ~0u, ~0u, ~0u};
    if (tail) {
      asm volatile("; tail mask");
      const int nv = kend + 1 - (k0 + 8 * g4);
#pragma unroll
      for (int q = 0; q < 4; ++q) vm[q] = (2 * q < nv ? 0x0000ffffu : 0u) | (2 * q + 1 < nv ? 0xffff0000u : 0u);
    }
    const int vslot = (g4 ^ ((c16 >> 2) & 3)) * 8;
#pragma unroll
    for (int dt = 0; dt < DT; ++dt) {
      u32x4 vt = *reinterpret_cast<const u32x4*>(&vs[buf][dt * 16 + c16][vslot]);
      if (tail) {
        asm volatile("; tail chunk");
#pragma unroll
        for (int q = 0; q < 4; ++q) vt[q] &= vm[q];
      }
#pragma unroll
      for (int rt = 0; rt < RT; ++rt)
        o_run[dt][rt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, vt), pf[rt], o_run[dt][rt], 0, 0, 0);
    }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  // ---- normalise and store: token s0 + 16 rt + c16, dims dt*16 + 4 g4 + i ----
#pragma unroll
  for (int rt = 0; rt < RT; ++rt) {
    const float l = pf_xsum(l_run[rt]);
    const float inv = l > 0.f ? 1.f / l : 0.f;
    const int tq = s0 + rt * 16 + c16;
    if (tq >= a.S) continue;
    const int mrow_ = b * a.S + tq;
    bf16_t* dst = a.out + (size_t)mrow_ * a.Hq * D + (size_t)hq * D;
#pragma unroll
    for (int dt = 0; dt < DT; ++dt) {
      const int d0 = dt * 16 + 4 * g4;
      const f32x4 o4 = o_run[dt][rt];
      // dims d0 .. d0 + 3 stay contiguous in the packed layout too (k & 7 = 0..3 or 4..7)
      const uint2 o = make_uint2(pf_pack(o4[0] * inv, o4[1] * inv), pf_pack(o4[2] * inv, o4[3] * inv));
      *reinterpret_cast<uint2*>(a.out_tiles ? a.out + xpkT_index(mrow_, hq * D + d0, a.out_tiles) : dst + d0) = o;
    }
  }
}

// query tokens per row from which the 32-token LDS-staged form runs (MTTS_ATTN_PF32_MIN, A/B;
// 0: never)
static int attn_pf32_min() {
  static const int v = getenv("MTTS_ATTN_PF32_MIN") ? atoi(getenv("MTTS_ATTN_PF32_MIN")) : 64;
  return v;
}

template <int D>
static hipError_t attn_prefill_d(const AttnArgs& a, int G, hipStream_t st) {
  const int B = a.M / a.S;
  if constexpr (D == 128) {
    if ((G == 4 || G == 2) && attn_pf32_min() > 0 && a.S >= attn_pf32_min()) {
      constexpr size_t PF32_LDS = 4 * 32 * D * 2 + 2 * 256;
      const dim3 grid((a.S + 31) / 32, a.Hkv, B);
      if (G == 4) hipLaunchKernelGGL((attn_prefill32_kernel<4, D>), grid, dim3(256), PF32_LDS, st, a);
      else hipLaunchKernelGGL((attn_prefill32_kernel<2, D>), grid, dim3(128), PF32_LDS, st, a);
      return hipGetLastError();
    }
  }
  dim3 grid((a.S + 15) / 16, a.Hkv, B);
  switch (G) {
    case 1: hipLaunchKernelGGL((attn_prefill_kernel<1, D>), grid, dim3(64), 0, st, a); break;
    case 2: hipLaunchKernelGGL((attn_prefill_kernel<2, D>), grid, dim3(128), 0, st, a); break;
    case 4: hipLaunchKernelGGL((attn_prefill_kernel<4, D>), grid, dim3(256), 0, st, a); break;
    case 8: hipLaunchKernelGGL((attn_prefill_kernel<8, D>), grid, dim3(512), 0, st, a); break;
    default: return hipErrorInvalidValue;
  }
  return hipGetLastError();
}

hipError_t attention_prefill(const AttnArgs& a, hipStream_t st) {
  const int G = a.Hq / a.Hkv;
  if (a.Hq % a.Hkv || a.M % a.S || a.Cmax % 64) return hipErrorInvalidValue;
  switch (a.D) {
    case 128: return attn_prefill_d<128>(a, G, st);
    case 64: return attn_prefill_d<64>(a, G, st);
    case 32: return attn_prefill_d<32>(a, G, st);
    case 16: return attn_prefill_d<16>(a, G, st);
    default: return hipErrorInvalidValue;
  }
}

size_t attn_smem_bytes(int G, int D, int CH) {
  const int LPK = D / 8;
  const int slots = 256 / LPK;
  size_t f = (size_t)G * D + (size_t)G * CH + 2 * G + 2;
  f = (f + 3) & ~(size_t)3;
  return (f + (size_t)slots * G * D) * sizeof(float);
}

hipError_t attention(const AttnArgs& a0, hipStream_t st) {
  AttnArgs a = a0;
  const int G = a.Hq / a.Hkv;
  if (a.Hq % a.Hkv || a.D % 8 || a.D > 128 || a.CH % 64) return hipErrorInvalidValue;
  // red must start 16B aligned: attn_smem_bytes rounds the prefix; mirror it in the kernel
  const size_t sm = attn_smem_bytes(G, a.D, a.CH);
  dim3 grid(a.n_split, a.Hkv, a.M);
  switch (G) {
    case 1: hipLaunchKernelGGL(attn_kernel<1>, grid, dim3(256), sm, st, a); break;
    case 2: hipLaunchKernelGGL(attn_kernel<2>, grid, dim3(256), sm, st, a); break;
    case 4: hipLaunchKernelGGL(attn_kernel<4>, grid, dim3(256), sm, st, a); break;
    case 8: hipLaunchKernelGGL(attn_kernel<8>, grid, dim3(256), sm, st, a); break;
    default: return hipErrorInvalidValue;
  }
  const int waves = a.M * a.Hq;
  hipLaunchKernelGGL(attn_combine_kernel, dim3((waves + 3) / 4), dim3(256), 0, st, a);
  return hipGetLastError();
}

}  // namespace mtts

// Fused decode attention: body in attn_body.h (shared with the fused attention + o_proj launch)
#include "attn_body.h"
namespace mtts {

// Grid (KV head, row, split): the split is the slowest dimension, so the blocks that hold keys
// (splits below pos / keys-per-block + 1; the rest return at once) are the grid's first Hkv x B x
// nact blocks, dealt round-robin over all 8 XCDs.  With the split fastest, a short context in a
// long cache (split 0 of each head active out of ns) put every working block on the XCDs of block
// ids 0, ns, 2 ns, ...: at B = 32 and the default 2,048-position cache (ns = 4) on 2 of the 8.
template <int G, int D, int NWV>
__global__ __launch_bounds__(NWV * 64) void attn_decode_kernel(DecAttnArgs a) {
  attn_decode_body<G, D, NWV>(a, (int)blockIdx.z, (int)blockIdx.x, (int)blockIdx.y);
}

template <int D, int NWV>
static hipError_t attn_decode_dn(const DecAttnArgs& a, int G, int B, hipStream_t s) {
  dim3 grid(a.Hkv, B, a.ns);
  const dim3 blk(NWV * 64);
  switch (G) {
    case 1: hipLaunchKernelGGL((attn_decode_kernel<1, D, NWV>), grid, blk, 0, s, a); break;
    case 2: hipLaunchKernelGGL((attn_decode_kernel<2, D, NWV>), grid, blk, 0, s, a); break;
    case 4: hipLaunchKernelGGL((attn_decode_kernel<4, D, NWV>), grid, blk, 0, s, a); break;
    case 8: hipLaunchKernelGGL((attn_decode_kernel<8, D, NWV>), grid, blk, 0, s, a); break;
    default: return hipErrorInvalidValue;
  }
  return hipGetLastError();
}

template <int D>
static hipError_t attn_decode_d(const DecAttnArgs& a, int G, int B, hipStream_t s) {
  switch (a.nwv) {
    case 8: return attn_decode_dn<D, 8>(a, G, B, s);
    case 16: return attn_decode_dn<D, 16>(a, G, B, s);
    default: return attn_decode_dn<D, 4>(a, G, B, s);
  }
}

static int decode_waves() {
  static const int nwv = getenv("MTTS_ATTN_NWV") ? atoi(getenv("MTTS_ATTN_NWV")) : 8;
  return (nwv == 8 || nwv == 16) ? nwv : 4;
}

int attn_decode_keys_per_block() { return DEC_KW * decode_waves(); }

// Publish-only decode attention (B <= 16: the o_proj prologue merges the split partials) up to
// this many blocks per head; beyond it every o_proj workgroup would redo a long merge
// (MTTS_ATTN_PO_MAX, A/B)
int attn_publish_max_splits() {
  static const int v = getenv("MTTS_ATTN_PO_MAX") ? atoi(getenv("MTTS_ATTN_PO_MAX")) : 4;
  return v;
}

int attn_decode_splits(int Cmax) { return (Cmax + DEC_KW * decode_waves() - 1) / (DEC_KW * decode_waves()); }
int attn_decode_keys_per_block_nwv(int nwv) { return DEC_KW * (nwv > 0 ? nwv : decode_waves()); }

size_t attn_decode_ws_bytes(int B, int Hq, int Hkv, int D, int Cmax) {
  const size_t cnt = ((size_t)B * Hkv * sizeof(int) + 255) / 256 * 256;
  return cnt + (size_t)B * Hq * attn_decode_splits(Cmax) * (D + 2) * sizeof(float);
}

hipError_t attn_decode(const DecAttnArgs& a0, int B, hipStream_t s) {
  const int G = a0.Hq / a0.Hkv;
  if (a0.Hq % a0.Hkv) return hipErrorInvalidValue;
  if (a0.Cmax % 64) return hipErrorInvalidValue;  // 16-byte V^T fragments, whole 16-key mask words
  if (!a0.part || !a0.cnt) return hipErrorInvalidValue;
  DecAttnArgs a = a0;
  // publish-only blocks must match the o_proj prologue's view (attn_decode_keys_per_block);
  // the self-combining form (B > 16) takes 16 waves = 512 keys per block, which halves the
  // splits to merge (B=32: 5.31 vs 5.62 ms/step; B=1: 8 waves stay faster, 3.29 vs 3.37)
  a.nwv = (!a.publish_only && !getenv("MTTS_ATTN_NWV") && B > 16) ? 16 : decode_waves();
  // a forced block size (the depth stack's 4 waves, batch-1 long contexts' 16): a publish-only
  // caller gives its o_proj the same view (attn_decode_keys_per_block_nwv)
  if (a.nwv_force == 4 || a.nwv_force == 8 || a.nwv_force == 16) a.nwv = a.nwv_force;
  a.ns = (a.Cmax + DEC_KW * a.nwv - 1) / (DEC_KW * a.nwv);
  if (a.ns > DEC_MAXS) return hipErrorInvalidValue;  // the last arriver's (m, l) table
  static const int probe = getenv("MTTS_ATTN_PROBE") ? atoi(getenv("MTTS_ATTN_PROBE")) : 0;
  a.probe = probe;
  switch (a.D) {
    case 128: return attn_decode_d<128>(a, G, B, s);
    case 64: return attn_decode_d<64>(a, G, B, s);
    case 16: return attn_decode_d<16>(a, G, B, s);
    default: return hipErrorInvalidValue;
  }
}

}  // namespace mtts
