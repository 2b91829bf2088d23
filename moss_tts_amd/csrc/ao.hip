// Decode attention + o_proj (+ residual, + sums of squares) as ONE launch with no block roles
// across workgroups and no in-launch waits except the final split-K arrival (one row,
// one new token each, KV capacity up to the engine's AO_MAX_CTX).
// Batch 1 only (the B = 1 decode step is the one bound by these chains); larger batches keep
// attn_decode + the o_proj GEMV.
//
//   TF/models/qwen3/modeling_qwen3.py:252-254 q/k_norm, :148-170 RoPE, TF/cache_utils.py:127-145
//   cache append, TF/integrations/sdpa_attention.py:79-166 attention, :279 o_proj, :311 residual.
//
// Work split: workgroup (KV head g, o_proj row chunk rc), g = blockIdx % Hkv -- with Hkv == 8
// all workgroups of one KV head share an XCD, so its K / V reach that L2 once.  In each:
//   * 2 LOADER waves move the o_proj weight slab -- rows [rc*128, rc*128+128) x the G*D columns
//     of head group g, 16-row x 32-k packed tiles (128 KiB at the 8B shape) -- into LDS with
//     non-temporal LDS-DMA at once, so the HBM weight stream runs under the attention chain
//     instead of after it.  They hold no registers for it and their loads sit in their own
//     in-order vmcnt: an attention wave never waits behind a weight load.
//   * 8 ATTENTION waves compute the attention of the KV head's G query heads over the whole
//     context (q/k RMSNorm + RoPE prologue, passes of 256 keys = 8 waves x 32, the next pass's
//     K loads issued after this pass's q.k MFMAs and its V^T loads after p.v, online softmax),
//     redundantly per row chunk and from L2, so no workgroup waits for another's attention;
//     then each multiplies one 16-row weight tile (A operand from LDS) by the bf16 attention
//     output (B operand from LDS) with v_mfma_f32_16x16x32_bf16 into an fp32 partial.
//   * The partials are published (write-through stores, drained, + arrival ticket per row chunk); the last
//     of the Hkv arrivals sums them in head order (deterministic), rounds, adds the residual and
//     writes h and its per-16-column sums of squares (the EPI_RESADD epilogue).
// The workgroup of row chunk 0 appends the new k / v to the cache; every workgroup patches the
// new key / value in from LDS instead of reading them back.
// Numerics: the attention is attn_body.h's (bf16 q/k norm and RoPE, fp32 softmax, bf16
// probabilities before p.v); o_proj sums the same products as the GEMV in another fp32 order.
#include "kernels.h"

namespace mtts {

namespace {
__device__ __forceinline__ __amdgpu_buffer_rsrc_t brsrc(const void* p, uint32_t bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(p), 0, (int)bytes, 0x00020000);
}
// workgroup barrier over LDS only: __syncthreads() is a workgroup release fence, which on
// gfx9 waits vmcnt(0) for the block's global stores (the KV append) -- and with them for
// every weight load in flight, serialising the o_proj stream behind the attention chain
// (the loader waves skip the lgkmcnt wait: it would hold them -- and the barrier -- until their
// LDS-DMA weight stream has landed)
__device__ __forceinline__ void lds_barrier(bool loader) {
  if (loader)
    asm volatile("s_barrier" ::: "memory");
  else
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
}
constexpr int AO_NA = 8;              // attention waves per block (each: one o_proj row tile at the end)
constexpr int AO_NW = AO_NA;          // o_proj row tiles per block
constexpr int AO_NL = 2;              // loader waves per block
constexpr int AO_T = (AO_NA + AO_NL) * 64;
constexpr int AO_KW = 32;             // keys per attention wave per pass
constexpr int AO_KB = AO_NA * AO_KW;  // keys per pass
constexpr int AO_ROWS = AO_NW * 16;   // o_proj rows per block
}  // namespace

template <int G, int D>
__global__ __launch_bounds__(AO_T) void attn_o_kernel(AOArgs a) {
  constexpr int QS = D / 32;       // 32-dim MFMA steps of q.k
  constexpr int DT = D / 16;       // 16-dim output tiles of p.v
  constexpr int KTG = G * D / 32;  // o_proj k-tiles of one head group
  constexpr int JOBS = (G + 2 + AO_NA - 1) / AO_NA;
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);  // wave-uniform: scalar resources
  const int g4 = lane >> 4, c16 = lane & 15;
  const int Hkv = a.Hkv, Cmax = a.Cmax, B = a.B;
  const int g = blockIdx.x % Hkv, rc = blockIdx.x / Hkv;
  const int pos = *a.pos;
  // waves [0, AO_NA): attention, then o_proj row tile rc*AO_NW + wave; [AO_NA, AO_NA + AO_NL):
  // loaders.  (A wait for a K / V load issued after a weight load by the same wave would also
  // wait for the weight load: vmcnt counts in order.)
  const bool owave = wave >= AO_NA;
  const int rt = rc * AO_NW + wave;
  const bool has_rt = !owave && rt < a.NRT;
  extern __shared__ __attribute__((aligned(16))) unsigned char wo_s[];  // [AO_NW][KTG] 1 KiB tiles

  __shared__ __attribute__((aligned(16))) bf16_t q_s[G][D];  // bf16 q (B-operand columns >= G read as 0)
  __shared__ float k_s[D];
  __shared__ float v_s[D];
  __shared__ __attribute__((aligned(16))) bf16_t p_s[AO_NA][16][AO_KW];
  __shared__ float ml_s[AO_NA][G][2];
  __shared__ float acc_s[AO_NA][G][D];
  __shared__ __attribute__((aligned(16))) bf16_t x_s[AO_MAXB][G * D];  // attention output rows
  __shared__ int last_s;


  const int heads = a.Hq + 2 * Hkv;
  // buffer loads throughout: one 32-bit lane offset + scalar offsets per load instead of a 64-bit
  // address per load (the attention's register budget); out-of-range offsets read as zero
  constexpr uint32_t OOB = 0x7ffffff0u;
  {
    const int b = 0;  // one row (B == 1): a per-row loop here doubles the attention's registers
    const bf16_t* row = a.qkv + (size_t)b * heads * D;
    bf16_t* kcache = a.kc + (((size_t)b * Hkv + g) * Cmax) * D;  // [Cmax][D]
    bf16_t* vcache = a.vc + (((size_t)b * Hkv + g) * D) * Cmax;  // [D][Cmax]
    const uint8_t* mrow = a.mask + (size_t)b * Cmax;
    const __amdgpu_buffer_rsrc_t krs = brsrc(kcache, Cmax * D * 2), vrs = brsrc(vcache, Cmax * D * 2),
                                 mrs = brsrc(mrow, Cmax);
    const bool writer = rc == 0;  // appends the new k / v
    u32x4 kt[2][QS];
    u32x4 vt[DT];
    uint32_t mk[2];
    float m_run = -INFINITY, l_run = 0.f;
    f32x4 o_run[DT];
    const int kbeg = wave * AO_KW;
    // ---- K tiles (A operands of q.k), V^T fragments (B operands of p.v), mask words of the
    // wave's 32 keys k0..k0+31; keys >= pos read as zero (the new one is patched from LDS) ----
    auto load_k = [&](int k0) {
#pragma unroll
      for (int t = 0; t < 2; ++t) {
        const int key = k0 + t * 16 + c16;
        const uint32_t vo = key < pos ? (uint32_t)(key * D + 8 * g4) * 2u : OOB;
#pragma unroll
        for (int st = 0; st < QS; ++st) kt[t][st] = __builtin_amdgcn_raw_buffer_load_b128(krs, vo + st * 64, 0, 0);
        // 16-key tiles that start at or before pos lie inside the row (Cmax % 64 == 0)
        const uint32_t mo = (k0 + t * 16 <= pos) ? (uint32_t)(k0 + t * 16 + g4 * 4) : OOB;
        mk[t] = __builtin_amdgcn_raw_buffer_load_b32(mrs, mo, 0, 0);
      }
    };
    auto load_v = [&](int k0) {
      const int kb = k0 + 8 * g4;  // lane's keys kb .. kb+7
      const uint32_t vo = kb < pos ? (uint32_t)(c16 * Cmax + kb) * 2u : OOB;
#pragma unroll
      for (int dt = 0; dt < DT; ++dt) vt[dt] = __builtin_amdgcn_raw_buffer_load_b128(vrs, vo, dt * 32 * Cmax, 0);
    };
    uint32_t pr[JOBS], pw[JOBS], pc[JOBS], ps[JOBS];
    const bool att_on = a.probe != 1 && !(a.probe == 4 && rc != 0);
    if (!owave && att_on) {
    // ---- prologue loads: job j < G: q head g*G + j; G: k; G+1: v ----
#pragma unroll
    for (int jj = 0; jj < JOBS; ++jj) {
      const int j = wave + jj * AO_NA;
      pr[jj] = pw[jj] = pc[jj] = ps[jj] = 0;
      if (j < G + 2) {
        const int hd = j < G ? g * G + j : (j == G ? a.Hq + g : a.Hq + Hkv + g);
        pr[jj] = *reinterpret_cast<const uint32_t*>(row + (size_t)hd * D + 2 * lane);
        if (j <= G) {
          pw[jj] = *reinterpret_cast<const uint32_t*>((j < G ? a.qn_w : a.kn_w) + 2 * lane);
          pc[jj] = *reinterpret_cast<const uint32_t*>(a.cos_t + (size_t)pos * D + 2 * lane);
          ps[jj] = *reinterpret_cast<const uint32_t*>(a.sin_t + (size_t)pos * D + 2 * lane);
        }
      }
    }
    load_k(kbeg);
    load_v(kbeg);
    }  // attention waves: first loads issued
    asm volatile("s_barrier" ::: "memory");
    // ---- loaders: the o_proj weight slab into LDS (non-temporal LDS-DMA, 1 KiB per instruction),
    // queued behind the attention waves' first loads (a CU's memory pipeline serves in order) ----
    if (owave && a.probe != 2) {
      typedef __attribute__((address_space(1))) void gvoid;
      typedef __attribute__((address_space(3))) void lvoid;
      const int l = wave - AO_NA;
      for (int i = l; i < AO_NW * KTG; i += AO_NL) {
        const int r = i / KTG, t = i - r * KTG;
        if (rc * AO_NW + r >= a.NRT) break;
        const bf16_t* src = a.wo + (((size_t)(rc * AO_NW + r) * a.KT + (size_t)g * KTG + t) * 64 + lane) * 8;
        __builtin_amdgcn_global_load_lds((const gvoid*)src, (lvoid*)(wo_s + (size_t)i * 1024), 16, 0, 2);
      }
    }
    if (!owave && att_on) {

    // ---- prologue math: q / k RMSNorm, RoPE; the writer appends k, v ----
#pragma unroll
    for (int jj = 0; jj < JOBS; ++jj) {
      const int j = wave + jj * AO_NA;
      if (j >= G + 2) continue;  // wave-uniform
      const float x0 = __uint_as_float(pr[jj] << 16), x1 = __uint_as_float(pr[jj] & 0xffff0000u);
      if (j == G + 1) {
        v_s[2 * lane] = x0;
        v_s[2 * lane + 1] = x1;
        if (writer) {
          __builtin_amdgcn_raw_buffer_store_b16(f2bf(x0), vrs, (uint32_t)(2 * lane * Cmax + pos) * 2u, 0, 0);
          __builtin_amdgcn_raw_buffer_store_b16(f2bf(x1), vrs, (uint32_t)((2 * lane + 1) * Cmax + pos) * 2u, 0, 0);
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
      const bool lo = lane < q4;
      const int partner = lo ? lane + q4 : lane - q4;
      const float p0 = __shfl(n0, partner, 64), p1 = __shfl(n1, partner, 64);
      const float sg = lo ? -1.f : 1.f;
      const float o0 = rbf(rbf(n0 * c0) + rbf(sg * p0 * s0));
      const float o1 = rbf(rbf(n1 * c1) + rbf(sg * p1 * s1));
      if (j < G) {
        q_s[j][2 * lane] = f2bf(o0);
        q_s[j][2 * lane + 1] = f2bf(o1);
      } else {
        k_s[2 * lane] = o0;
        k_s[2 * lane + 1] = o1;
        if (writer) __builtin_amdgcn_raw_buffer_store_b32(pack2(o0, o1), krs, (uint32_t)(pos * D + 2 * lane) * 2u, 0, 0);
      }
    }
    }  // attention waves
    lds_barrier(owave);

    if (!owave && att_on) {
    // ---- passes of 256 keys: online softmax per head (lane & 15) ----
#pragma unroll
    for (int dt = 0; dt < DT; ++dt) o_run[dt] = (f32x4){0.f, 0.f, 0.f, 0.f};
#pragma unroll 1
    for (int k0 = kbeg; k0 <= pos; k0 += AO_KB) {
      const int kn = k0 + AO_KB;  // the wave's next pass
      f32x4 sacc[2];
#pragma unroll
      for (int t = 0; t < 2; ++t) {
        if (k0 + t * 16 + c16 == pos) {
#pragma unroll
          for (int st = 0; st < QS; ++st) {
            const int d0 = st * 32 + 8 * g4;
            u32x4 v;
#pragma unroll
            for (int i = 0; i < 4; ++i) v[i] = pack2(k_s[d0 + 2 * i], k_s[d0 + 2 * i + 1]);
            kt[t][st] = v;
          }
        }
        sacc[t] = (f32x4){0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int st = 0; st < QS; ++st)
          sacc[t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, kt[t][st]),
                                                           c16 < G ? *reinterpret_cast<const bf16x8*>(&q_s[c16 < G ? c16 : 0][st * 32 + 8 * g4])
                                                                   : bf16x8{},
                                                           sacc[t], 0, 0, 0);
      }
      uint32_t mkc[2] = {mk[0], mk[1]};
      if (kn <= pos) load_k(kn);
      // V^T of this pass: keys >= pos zeroed, the new value patched in
      {
        const int kb = k0 + 8 * g4;
        if (kb + 8 > pos && kb <= pos) {
#pragma unroll
          for (int dt = 0; dt < DT; ++dt) {
            u32x4 v = vt[dt];
            const uint32_t nv = (uint32_t)f2bf(v_s[dt * 16 + c16]);
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
      }
      float sv[2][4];
      float mc = -INFINITY;
#pragma unroll
      for (int t = 0; t < 2; ++t)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int key = k0 + t * 16 + g4 * 4 + r;
          const bool valid = key <= pos && ((mkc[t] >> (8 * r)) & 0xffu);
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
      if (kn <= pos) load_v(kn);
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
        const int h = g4 * 4 + r;
        if (h < G) acc_s[wave][h][dt * 16 + c16] = o_run[dt][r];
      }
    }  // attention waves
    lds_barrier(owave);
    // ---- merge the 8 wave partials (fixed order): x = bf16(o / l) ----
    for (int e = threadIdx.x; e < G * D; e += AO_T) {
      const int h = e / D, d = e % D;
      float M = -INFINITY;
#pragma unroll
      for (int w = 0; w < AO_NA; ++w) M = fmaxf(M, ml_s[w][h][0]);
      float L = 0.f, o = 0.f;
#pragma unroll
      for (int w = 0; w < AO_NA; ++w) {
        const float mw = ml_s[w][h][0];
        const float f = (mw == -INFINITY) ? 0.f : expf(mw - M);
        L += f * ml_s[w][h][1];
        o += f * acc_s[w][h][d];
      }
      x_s[b][e] = f2bf(L > 0.f ? o / L : 0.f);
    }
    if (owave) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the weight slab has landed
    lds_barrier(owave);
  }

  // ---- o_proj partial of this wave's row tile over head group g ----
  float* part = a.part + (size_t)rc * Hkv * AO_MAXB * AO_ROWS;  // [Hkv][AO_MAXB][AO_ROWS] of this chunk
  if (has_rt) {
    f32x4 acc = (f32x4){0.f, 0.f, 0.f, 0.f};
    const u32x4* wt = reinterpret_cast<const u32x4*>(wo_s) + (size_t)wave * KTG * 64 + lane;
#pragma unroll
    for (int t = 0; t < KTG; ++t) {
      const u32x4 xb = c16 < B ? *reinterpret_cast<const u32x4*>(&x_s[c16 < B ? c16 : 0][t * 32 + 8 * g4])
                               : (u32x4){0u, 0u, 0u, 0u};
      acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, wt[t * 64]),
                                                    __builtin_bit_cast(bf16x8, xb), acc, 0, 0, 0);
    }
    if (c16 < B) {  // write-through (sc1) stores: the reducer reads them past its L2
      float* pp = part + ((size_t)g * AO_MAXB + c16) * AO_ROWS + wave * 16 + g4 * 4;
#pragma unroll
      for (int i = 0; i < 4; ++i)
        __hip_atomic_store((__attribute__((address_space(1))) float*)(pp + i), acc[i], __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_AGENT);
    }
  }
  if (a.probe == 3) return;
  // ---- publish + arrival ticket of the row chunk (agent-scope release / acquire) ----
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0) {  // drained sc1 stores + relaxed agent add (cdna_hip_programming.md G16 R1)
    const int ticket = __hip_atomic_fetch_add(a.cnt + rc, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    last_s = ticket == Hkv - 1;
  }
  __syncthreads();
  if (!last_s) return;
  // Hand-off form "sc1 payload, drained, relaxed agent ticket; every consumer load sc1"
  // (cdna_hip_programming.md Guideline 16, R1 with sc1 loads): the producer side is the
  // sc1 (write-through) stores above + the asm vmcnt(0) drain before the ticket; on this
  // side every read of a partial is an agent-scope atomic (sc1) load, so no L1 line can be
  // stale and the acquire reduces to a wavefront-scope fence that keeps the compiler from
  // hoisting those loads above the ticket.  Plain stores or plain loads of the partials
  // would need an agent-scope release / acquire pair instead.
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  // ---- the last arrival: sum the Hkv partials in head order, + residual, sums of squares ----
  const int n0 = rc * AO_ROWS;
  float (*sq_s)[AO_ROWS] = reinterpret_cast<float (*)[AO_ROWS]>(&p_s[0][0][0]);  // p_s is free by now
  static_assert(sizeof(p_s) >= sizeof(float) * AO_MAXB * AO_ROWS, "sq_s alias");
  for (int e = threadIdx.x; e < B * AO_ROWS; e += AO_T) {
    const int b = e / AO_ROWS, nl = e - b * AO_ROWS, n = n0 + nl;
    if (n >= a.H) continue;
    float s = 0.f;
    for (int gg = 0; gg < Hkv; ++gg)  // sc1 loads of the other workgroups' partials
      s += __hip_atomic_load((__attribute__((address_space(1))) float*)(part + ((size_t)gg * AO_MAXB + b) * AO_ROWS + nl),
                             __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    // hidden = residual + bf16(o)   (TF/.../modeling_qwen3.py:311)
    bf16_t* hp = a.h + (size_t)b * a.ldh + n;
    const bf16_t out = f2bf(bf2f(*hp) + rbf(s));
    *hp = out;
    const float ho = bf2f(out);
    sq_s[b][nl] = ho * ho;
  }
  __syncthreads();
  for (int e = threadIdx.x; e < B * AO_NW; e += AO_T) {
    const int b = e / AO_NW, j = e - b * AO_NW, tile = rc * AO_NW + j;
    if (tile * 16 >= a.H) continue;
    float s = 0.f;
#pragma unroll
    for (int i = 0; i < 16; ++i) s += sq_s[b][j * 16 + i];
    a.ss_out[(size_t)b * a.ld_ss + tile] = s;
  }
  if (threadIdx.x == 0) a.cnt[rc] = 0;  // ready for the next launch (graph replay)
}

int attn_o_chunks(int H) { return (H / 16 + AO_NW - 1) / AO_NW; }

size_t attn_o_ws_floats(int H, int Hkv) { return (size_t)attn_o_chunks(H) * Hkv * AO_MAXB * AO_ROWS; }

bool attn_o_supported(int B, int Hq, int Hkv, int D, int H) {
  const int G = Hkv > 0 ? Hq / Hkv : 0;
  return B == 1 && D == 128 && Hkv > 0 && Hq % Hkv == 0 && (G == 1 || G == 2 || G == 4) &&
         H % 16 == 0;
}

template <int G>
static hipError_t launch_attn_o(const AOArgs& a, hipStream_t s) {
  constexpr size_t lds = (size_t)AO_NW * (G * 128 / 32) * 1024;
  static const hipError_t attr =
      hipFuncSetAttribute((const void*)attn_o_kernel<G, 128>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
  if (attr != hipSuccess) return attr;
  attn_o_kernel<G, 128><<<dim3(a.Hkv * attn_o_chunks(a.H)), dim3(AO_T), lds, s>>>(a);
  return hipGetLastError();
}

hipError_t attn_o(const AOArgs& a, hipStream_t s) {
  if (!attn_o_supported(a.B, a.Hq, a.Hkv, a.D, a.H) || a.NRT != a.H / 16 || a.KT != a.Hq * a.D / 32)
    return hipErrorInvalidValue;
  switch (a.Hq / a.Hkv) {
    case 1: return launch_attn_o<1>(a, s);
    case 2: return launch_attn_o<2>(a, s);
    default: return launch_attn_o<4>(a, s);
  }
}

}  // namespace mtts
