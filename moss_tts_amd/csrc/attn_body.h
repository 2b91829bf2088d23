#pragma once
#include "kernels.h"

// ===========================================================================
// Fused decode attention (one new token per row), MFMA form.
// Block (split, KV head, row b) -- launched as grid (KV head, row, split), attention.hip; a 1024-thread block (16 waves) owns 512 consecutive keys,
// 32 per wave, so a context of <= 512 tokens is ONE block per (row, KV head) and needs no
// cross-block combine.
//   prologue  q_norm (TF/.../modeling_qwen3.py:252-254) + RoPE (:148-170) of the G query
//             heads; the block whose range holds the new token also norms/ropes its key and
//             appends k and v to the cache at `pos` (TF/cache_utils.py:127-145).  The prologue
//             loads go out first, then the first pass's K / V^T / mask loads, then the math.
//   S[key][head] = K_tile[16 keys x 32 dims] . Q^T[32 dims x 16 heads]  (v_mfma_f32_16x16x32_bf16)
//   softmax per head over the wave's 32 keys (fp32; probabilities rounded to bf16 before
//   P.V as the reference's bf16 SDPA does), O[head][dim] += P[16 x 32] . V[32 x 16 dims] with
//   V^T fragments straight from the TRANSPOSED cache (one 16-byte load per lane); the 16
//   wave partials merge in LDS in a fixed order.
// Longer contexts: several blocks per head publish (m, l, o) partials (agent-scope release +
// arrival ticket); the last arriver merges them in split order (deterministic).
// Cache layouts: K [Bmax][Hkv][Cmax][D], V [Bmax][Hkv][D][Cmax].
namespace mtts {

constexpr int DEC_KW = 32;      // keys per wave
constexpr int DEC_MAXS = 512;  // splits per head (MTTS_MAX_CTX at 256-key blocks)

template <int G, int D, int NWV>
__device__ __forceinline__ void attn_decode_body(const DecAttnArgs& a, const int sp, const int kvh, const int b) {
  constexpr int KW = DEC_KW, KB = KW * NWV;
  constexpr int QS = (D + 31) / 32;  // 32-dim MFMA steps of q.k
  constexpr int DT = (D + 15) / 16;  // 16-dim output tiles of p.v
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);  // wave-uniform (scalar resources)
  const int g4 = lane >> 4, c16 = lane & 15;
  const int pos = *a.pos;
  const int nact = pos / KB + 1;
  if (sp >= nact || a.probe == 1) return;
  const bool owner = sp == nact - 1;
  const int Cmax = a.Cmax;
  __shared__ __attribute__((aligned(16))) bf16_t q_s[16][QS * 32];  // bf16 q (zero outside G x D)
  __shared__ float k_s[D];
  __shared__ float v_s[D];
  __shared__ __attribute__((aligned(16))) bf16_t p_s[NWV][16][KW];
  __shared__ float ml_s[NWV][G][2];
  __shared__ float acc_s[NWV][G][D];
  __shared__ float mlp_s[DEC_MAXS][G][2];
  __shared__ int last_s;

  for (int i = threadIdx.x; i < 16 * QS * 32; i += NWV * 64)
    if (i / (QS * 32) >= G || i % (QS * 32) >= D) (&q_s[0][0])[i] = 0;
  const int heads = a.Hq + 2 * a.Hkv;
  const bf16_t* row = a.qkv + (size_t)b * heads * D;
  bf16_t* kcache = a.kc + (((size_t)b * a.Hkv + kvh) * Cmax) * D;  // [Cmax][D]
  bf16_t* vcache = a.vc + (((size_t)b * a.Hkv + kvh) * D) * Cmax;  // [D][Cmax]
  const uint8_t* mrow = a.mask + (size_t)b * Cmax;

  // ---- a wave's 32 keys k0..k0+31: K tiles (A operands), V^T fragments (B operands), mask.
  // Keys >= pos read as zero; the new key / value are patched in from LDS below. ----
  u32x4 kt[2][QS];
  u32x4 vt[DT];
  uint32_t mk[2];
  // Branch-free buffer loads: an out-of-range offset reads zero.  A per-lane "load or zero"
  // select makes hipcc branch around each load and wait for it (cdna_hip_programming.md, GEMM
  // trap (c)), so the K / V^T / mask loads would each cost a round trip.
  constexpr uint32_t OOBA = 0x7ffffff0u;
  const __amdgpu_buffer_rsrc_t krs = __builtin_amdgcn_make_buffer_rsrc(kcache, 0, Cmax * D * 2, 0x00020000);
  const __amdgpu_buffer_rsrc_t vrs = __builtin_amdgcn_make_buffer_rsrc(vcache, 0, Cmax * D * 2, 0x00020000);
  const __amdgpu_buffer_rsrc_t mrs =
      __builtin_amdgcn_make_buffer_rsrc(const_cast<uint8_t*>(mrow), 0, Cmax, 0x00020000);
  auto load_keys = [&](int k0) {
#pragma unroll
    for (int t = 0; t < 2; ++t) {
      const int key = k0 + t * 16 + c16;
#pragma unroll
      for (int st = 0; st < QS; ++st) {
        const int d0 = st * 32 + 8 * g4;
        kt[t][st] = __builtin_amdgcn_raw_buffer_load_b128(
            krs, (key < pos && d0 < D) ? (uint32_t)(key * D + d0) * 2u : OOBA, 0, 0);
      }
      // 16-key tiles that start at or before pos lie inside the row (Cmax % 64 == 0)
      mk[t] = __builtin_amdgcn_raw_buffer_load_b32(
          mrs, (k0 + t * 16 <= pos) ? (uint32_t)(k0 + t * 16 + g4 * 4) : OOBA, 0, 0);
    }
#pragma unroll
    for (int dt = 0; dt < DT; ++dt) {
      const int dim = dt * 16 + c16;
      const int kb = k0 + 8 * g4;  // lane's keys kb .. kb+7
      vt[dt] = __builtin_amdgcn_raw_buffer_load_b128(
          vrs, (dim < D && kb < pos) ? (uint32_t)(dim * Cmax + kb) * 2u : OOBA, 0, 0);
    }
  };
  const int kbeg = sp * KB + wave * KW;

  // ---- prologue loads: job j < G: q head j; G: k; G+1: v (k, v only in the owner);
  // wave w takes jobs w, w + NWV, ... ----
  constexpr int JOBS = (G + 2 + NWV - 1) / NWV;
  const int njobs = G + (owner ? 2 : 0);
  uint32_t pr[JOBS], pw[JOBS], pc[JOBS], ps[JOBS];
  {
    // same branch-free form: unused jobs / lanes / tables read zero
    const __amdgpu_buffer_rsrc_t rrs =
        __builtin_amdgcn_make_buffer_rsrc(const_cast<bf16_t*>(row), 0, heads * D * 2, 0x00020000);
    const __amdgpu_buffer_rsrc_t qws =
        __builtin_amdgcn_make_buffer_rsrc(const_cast<bf16_t*>(a.qn_w), 0, D * 2, 0x00020000);
    const __amdgpu_buffer_rsrc_t kws =
        __builtin_amdgcn_make_buffer_rsrc(const_cast<bf16_t*>(a.kn_w), 0, D * 2, 0x00020000);
    const bool rope = a.cos_t != nullptr;
    const int rpos = a.rope_off ? max(0, pos - a.rope_off[b]) : pos;  // RoPE position (cache slot: pos)
    const __amdgpu_buffer_rsrc_t crs = __builtin_amdgcn_make_buffer_rsrc(
        const_cast<bf16_t*>(rope ? a.cos_t + (size_t)rpos * D : row), 0, D * 2, 0x00020000);
    const __amdgpu_buffer_rsrc_t srs = __builtin_amdgcn_make_buffer_rsrc(
        const_cast<bf16_t*>(rope ? a.sin_t + (size_t)rpos * D : row), 0, D * 2, 0x00020000);
#pragma unroll
    for (int jj = 0; jj < JOBS; ++jj) {
      const int j = wave + jj * NWV;
      const bool on = j < njobs && 2 * lane < D;
      const int hd = j < G ? kvh * G + j : (j == G ? a.Hq + kvh : a.Hq + a.Hkv + kvh);
      const uint32_t lo = 4u * lane;  // byte offset of the lane's two dims
      pr[jj] = __builtin_amdgcn_raw_buffer_load_b32(rrs, on ? (uint32_t)hd * D * 2u + lo : OOBA, 0, 0);
      const bool nw = on && j <= G;
      pw[jj] = __builtin_amdgcn_raw_buffer_load_b32(j < G ? qws : kws, nw ? lo : OOBA, 0, 0);
      pc[jj] = __builtin_amdgcn_raw_buffer_load_b32(crs, nw && rope ? lo : OOBA, 0, 0);
      ps[jj] = __builtin_amdgcn_raw_buffer_load_b32(srs, nw && rope ? lo : OOBA, 0, 0);
    }
  }
  load_keys(kbeg);  // waves past the new token: every offset out of range

  // ---- prologue math ----
#pragma unroll
  for (int jj = 0; jj < JOBS; ++jj) {
    const int j = wave + jj * NWV;
    if (j >= njobs) continue;  // wave-uniform
    const bool act = 2 * lane < D;
    const float x0 = __uint_as_float(pr[jj] << 16), x1 = __uint_as_float(pr[jj] & 0xffff0000u);
    if (j == G + 1) {
      if (act) {
        v_s[2 * lane] = x0;
        v_s[2 * lane + 1] = x1;
        vcache[(size_t)(2 * lane) * Cmax + pos] = f2bf(x0);
        vcache[(size_t)(2 * lane + 1) * Cmax + pos] = f2bf(x1);
      }
      continue;
    }
    const float ss = wave_sum(x0 * x0 + x1 * x1);
    const float r = 1.0f / sqrtf(ss / (float)D + a.eps);
    const float w0 = __uint_as_float(pw[jj] << 16), w1 = __uint_as_float(pw[jj] & 0xffff0000u);
    const float c0 = __uint_as_float(pc[jj] << 16), c1 = __uint_as_float(pc[jj] & 0xffff0000u);
    const float s0 = __uint_as_float(ps[jj] << 16), s1 = __uint_as_float(ps[jj] & 0xffff0000u);
    const float n0 = rbf(w0 * rbf(x0 * r)), n1 = rbf(w1 * rbf(x1 * r));
    constexpr int q4 = D / 4;
    const bool lo = 2 * lane < D / 2;
    const int partner = lo ? lane + q4 : lane - q4;
    const float p0 = __shfl(n0, partner, 64), p1 = __shfl(n1, partner, 64);
    const float sg = lo ? -1.f : 1.f;
    // no cos table: attention without positional embedding (MossTTSLocal's depth
    // transformer, moss_tts_local/modeling_moss_tts.py:126-176)
    const float o0 = a.cos_t ? rbf(rbf(n0 * c0) + rbf(sg * p0 * s0)) : n0;
    const float o1 = a.cos_t ? rbf(rbf(n1 * c1) + rbf(sg * p1 * s1)) : n1;
    if (act) {
      if (j < G) {
        q_s[j][2 * lane] = f2bf(o0);
        q_s[j][2 * lane + 1] = f2bf(o1);
      } else {
        k_s[2 * lane] = o0;
        k_s[2 * lane + 1] = o1;
        *reinterpret_cast<uint32_t*>(kcache + (size_t)pos * D + 2 * lane) = pack2(o0, o1);
      }
    }
  }
  __syncthreads();
  if (a.probe == 2) {
    if (threadIdx.x == 0 && kbeg <= pos) a.out[b] = (bf16_t)(kt[0][0][0] ^ vt[DT - 1][0] ^ mk[0]);
    return;
  }

  float m_run = -INFINITY, l_run = 0.f;  // stats of head (lane & 15)
  f32x4 o_run[DT];
#pragma unroll
  for (int dt = 0; dt < DT; ++dt) o_run[dt] = (f32x4){0.f, 0.f, 0.f, 0.f};
  if (kbeg <= pos) {  // waves past the new token hold no keys (their loads never ran)
    const int k0 = kbeg;
    // ---- S = K . Q^T (the new key patched in from LDS) ----
    f32x4 sacc[2];
#pragma unroll
    for (int t = 0; t < 2; ++t) {
      if (k0 + t * 16 + c16 == pos) {
#pragma unroll
        for (int st = 0; st < QS; ++st) {
          const int d0 = st * 32 + 8 * g4;
          u32x4 v = {0u, 0u, 0u, 0u};
          if (d0 < D)
            for (int i = 0; i < 4; ++i) v[i] = pack2(k_s[d0 + 2 * i], k_s[d0 + 2 * i + 1]);
          kt[t][st] = v;
        }
      }
      sacc[t] = (f32x4){0.f, 0.f, 0.f, 0.f};
      // Q^T B-operand fragments from LDS: lane -> head (lane & 15), dims st*32 + 8*(lane>>4) .. +7
#pragma unroll
      for (int st = 0; st < QS; ++st)
        sacc[t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, kt[t][st]),
                                                         *reinterpret_cast<const bf16x8*>(&q_s[c16][st * 32 + 8 * g4]),
                                                         sacc[t], 0, 0, 0);
    }
    // V^T: keys >= pos zeroed, the new token's value patched in from LDS
#pragma unroll
    for (int dt = 0; dt < DT; ++dt) {
      const int dim = dt * 16 + c16;
      const int kb = k0 + 8 * g4;
      if (dim < D && kb + 8 > pos && kb <= pos) {
        u32x4 v = vt[dt];
        const uint32_t nv = (uint32_t)f2bf(v_s[dim]);
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int kk = kb + 2 * i;
          const uint32_t lo = kk < pos ? (v[i] & 0xffffu) : (kk == pos ? nv : 0u);
          const uint32_t hi = kk + 1 < pos ? (v[i] >> 16) : (kk + 1 == pos ? nv : 0u);
          v[i] = lo | (hi << 16);
        }
        vt[dt] = v;
      }
    }
    // ---- softmax over the 32 keys for head c16 (rows: keys t*16 + g4*4 + r) ----
    float sv[2][4];
    float mc = -INFINITY;
#pragma unroll
    for (int t = 0; t < 2; ++t)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int key = k0 + t * 16 + g4 * 4 + r;
        const bool valid = key <= pos && ((mk[t] >> (8 * r)) & 0xffu);
        sv[t][r] = valid ? sacc[t][r] * a.scale : -INFINITY;
        mc = fmaxf(mc, sv[t][r]);
      }
    mc = fmaxf(mc, __shfl_xor(mc, 16, 64));
    mc = fmaxf(mc, __shfl_xor(mc, 32, 64));
    float lc = 0.f;
#pragma unroll
    for (int t = 0; t < 2; ++t) {
      float pr4[4];
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const float p = (mc == -INFINITY || sv[t][r] == -INFINITY) ? 0.f : expf(sv[t][r] - mc);
        lc += p;
        pr4[r] = p;
      }
      uint2 pk;
      pk.x = pack2(pr4[0], pr4[1]);
      pk.y = pack2(pr4[2], pr4[3]);
      *reinterpret_cast<uint2*>(&p_s[wave][c16][t * 16 + g4 * 4]) = pk;  // bf16-rounded probabilities
    }
    lc += __shfl_xor(lc, 16, 64);
    lc += __shfl_xor(lc, 32, 64);
    const float mn = fmaxf(m_run, mc);
    const float alpha = (m_run == -INFINITY) ? 0.f : expf(m_run - mn);
    const float beta = (mc == -INFINITY) ? 0.f : expf(mc - mn);
    l_run = l_run * alpha + lc * beta;
    m_run = mn;
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
    // ---- O += P . V ----
    const bf16x8 pf = *reinterpret_cast<const bf16x8*>(&p_s[wave][c16][8 * g4]);
    float al[4], be[4];
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      al[r] = __shfl(alpha, g4 * 4 + r, 64);
      be[r] = __shfl(beta, g4 * 4 + r, 64);
    }
#pragma unroll
    for (int dt = 0; dt < DT; ++dt) {
      const f32x4 oc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(pf, __builtin_bit_cast(bf16x8, vt[dt]),
                                                              (f32x4){0.f, 0.f, 0.f, 0.f}, 0, 0, 0);
#pragma unroll
      for (int r = 0; r < 4; ++r) o_run[dt][r] = o_run[dt][r] * al[r] + be[r] * oc[r];
    }
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
  }
  if (lane < G) {
    ml_s[wave][lane][0] = m_run;
    ml_s[wave][lane][1] = l_run;
  }
#pragma unroll
  for (int dt = 0; dt < DT; ++dt)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int h = g4 * 4 + r, dim = dt * 16 + c16;
      if (h < G && dim < D) acc_s[wave][h][dim] = o_run[dt][r];
    }
  __syncthreads();

  // ---- merge the 16 wave partials (fixed order) into the block's result / partial ----
  const int t = threadIdx.x;
  // publish-only (o_proj merges) while the context spans <= po_max blocks; longer contexts
  // merge here once instead of in every o_proj workgroup
  const bool po = a.publish_only && nact <= a.po_max;
  const bool single = nact == 1 && !po;
  float* part = a.part + (((size_t)b * a.Hkv + kvh) * a.ns + sp) * (G * (D + 2));
  for (int e = t; e < G * D; e += NWV * 64) {
    const int h = e / D, d = e % D;
    float M = -INFINITY;
#pragma unroll
    for (int w = 0; w < NWV; ++w) M = fmaxf(M, ml_s[w][h][0]);
    float L = 0.f, o = 0.f;
#pragma unroll
    for (int w = 0; w < NWV; ++w) {
      const float mw = ml_s[w][h][0];
      const float f = (mw == -INFINITY) ? 0.f : expf(mw - M);
      L += f * ml_s[w][h][1];
      o += f * acc_s[w][h][d];
    }
    if (single) {
      bf16_t* op = a.out + (a.out_packed ? xpk_index(b, kvh * G * D + e) : (size_t)b * a.Hq * D + (size_t)(kvh * G) * D + e);
      *op = f2bf(L > 0.f ? o / L : 0.f);
    } else if (!po) {
      // consumed inside this launch (the last arriver below): write-through (sc1)
      // stores, drained before the ticket -- no release fence (cdna_hip_programming.md G16 R1)
      typedef __attribute__((address_space(1))) uint32_t g32;
      __hip_atomic_store((g32*)(part + e), __float_as_uint(o), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (d == 0) {
        __hip_atomic_store((g32*)(part + G * D + 2 * h), __float_as_uint(M), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_store((g32*)(part + G * D + 2 * h + 1), __float_as_uint(L), __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_AGENT);
      }
    } else {
      part[e] = o;
      if (d == 0) {
        part[G * D + 2 * h] = M;
        part[G * D + 2 * h + 1] = L;
      }
    }
  }
  if (single || po || a.probe == 3) return;

  // ---- publish + arrival ticket.  Hand-off form "sc1 payload, drained, relaxed agent ticket;
  // every consumer load sc1" (cdna_hip_programming.md Guideline 16, R1 with sc1 loads): the
  // partials above went out write-through, every storing wave drains them before the block
  // barrier, one lane takes the ticket, and the last arriver reads the partials with agent-scope
  // atomic (sc1) loads, so no L1 line can be stale and no release / acquire fence is needed (an
  // agent-scope release would write back this XCD's L2; an acquire invalidates the L1). ----
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  int* cnt = a.cnt + (size_t)b * a.Hkv + kvh;
  if (t == 0) {
    const int ticket = __hip_atomic_fetch_add(cnt, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    last_s = ticket == nact - 1;
  }
  __syncthreads();
  if (!last_s) return;
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");  // keeps the sc1 loads below the ticket
  // ---- the last arriver merges the nact partials in split order: the (m, l) pairs go to
  // LDS with all loads in flight at once, then each thread sums its element over splits ----
  typedef __attribute__((address_space(1))) float gf32;
  auto ld1 = [](const float* q) { return __hip_atomic_load((gf32*)q, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT); };
  const float* p0 = a.part + ((size_t)b * a.Hkv + kvh) * a.ns * (G * (D + 2));
  constexpr int PS = G * (D + 2);
  float* mlp = &mlp_s[0][0][0];
  for (int i = t; i < nact * G * 2; i += NWV * 64) mlp[i] = ld1(p0 + (size_t)(i / (2 * G)) * PS + G * D + i % (2 * G));
  __syncthreads();
  for (int e = t; e < G * D; e += NWV * 64) {
    const int h = e / D;
    float M = -INFINITY;
    for (int s2 = 0; s2 < nact; ++s2) M = fmaxf(M, mlp[(s2 * G + h) * 2]);
    float L = 0.f, o = 0.f;
#pragma unroll 8
    for (int s2 = 0; s2 < nact; ++s2) {
      const float ms = mlp[(s2 * G + h) * 2];
      const float f = (ms == -INFINITY) ? 0.f : expf(ms - M);
      L += f * mlp[(s2 * G + h) * 2 + 1];
      o += f * ld1(p0 + (size_t)s2 * PS + e);
    }
    bf16_t* op = a.out + (a.out_packed ? xpk_index(b, kvh * G * D + e) : (size_t)b * a.Hq * D + (size_t)(kvh * G) * D + e);
    *op = f2bf(L > 0.f ? o / L : 0.f);
  }
  // ready for the next launch (graph replay)
  if (t == 0) *cnt = 0;
}

}  // namespace mtts
