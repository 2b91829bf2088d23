// Body of the weight-streaming GEMV (see gemv.hip for the layout and the work split), as a
// device function so that fused launches can run it as one of their block roles.
#pragma once
#include "kernels.h"

#ifndef GEMV_PROBE
#define GEMV_PROBE 0
#endif

namespace mtts {

// bf16(nw * bf16(x * r)) for 8 packed elements (Qwen3RMSNorm rounding points)
__device__ __forceinline__ u32x4 norm8(u32x4 xv, u32x4 wv, float r) {
  u32x4 o;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const float x0 = __uint_as_float(xv[i] << 16), x1 = __uint_as_float(xv[i] & 0xffff0000u);
    const float w0 = __uint_as_float(wv[i] << 16), w1 = __uint_as_float(wv[i] & 0xffff0000u);
    o[i] = pack2(w0 * rbf(x0 * r), w1 * rbf(x1 * r));
  }
  return o;
}

// WT: outputs are stored write-through (sc1) for a consumer inside the same launch, which then
// needs no release fence from this block, only a drain (cdna_hip_programming.md G16 R1)
template <int NB, int RT, int EPI, int PRO0, int NW, bool PIPE, class Wait, bool WT = false>
__device__ __forceinline__ void gemv_body(const GemvArgs& a, const int bt, Wait&& wait) {
  constexpr bool PRER = PRO0 == PRO_NORM_PREROW;  // the same, one row per load (K / 8 == threads)
  constexpr bool PREL = PRO0 == PRO_NORM_PRE || PRER;  // norm prologue inputs loaded before the weights
  constexpr bool DMAN = PRO0 == PRO_NORM_DMA;  // the same inputs by LDS-DMA (no registers)
  constexpr bool PREA = PRO0 == PRO_ATTN_PRE || PRO0 == PRO_ATTN_PRE2;  // attention partials (2 splits) loaded before the weights
  constexpr int PRO = (PREL || DMAN) ? PRO_NORM : (PREA ? PRO_ATTN : PRO0);
  // k-tiles per load batch (one batch in flight per wave); the 4-deep variant (PIPE) trades
  // bytes in flight per wave for more resident waves (the default for 17-32 rows)
  constexpr int U = PIPE ? 4 : 8;
  const int lane = threadIdx.x & 63;
  const int wave = threadIdx.x >> 6;
  const int KT = a.KT;
  const int per = (KT + NW - 1) / NW;
  const int kt0 = wave * per;
  const int kt1 = min(KT, kt0 + per);

  f32x4 acc[RT][NB];
#pragma unroll
  for (int r = 0; r < RT; ++r)
#pragma unroll
    for (int nb = 0; nb < NB; ++nb) acc[r][nb] = (f32x4){0.f, 0.f, 0.f, 0.f};

  // A operand: packed weight tiles
  const u32x4* wbase[RT];
#pragma unroll
  for (int r = 0; r < RT; ++r)
    wbase[r] = reinterpret_cast<const u32x4*>(a.w) + ((size_t)(bt * RT + r) * KT) * 64 + lane;
  // B operand: x rows (b = lane&15 + 16 nb), 8 consecutive k at 8*(lane>>4)
  // (x_packed, 17-32 rows: fragment-packed x, xpk_index -- k tile kt of half nb is 1 KiB at (2 kt + nb) KiB)
  const u32x4* xbase[NB];
  bool xok[NB];
  const int xs = a.x_packed ? 128 : 4;  // u32x4 stride per k tile
#pragma unroll
  for (int nb = 0; nb < NB; ++nb) {
    const int b = (lane & 15) + 16 * nb;
    xok[nb] = b < a.B;
    const size_t row = a.xtok ? (size_t)a.xtok[(size_t)(xok[nb] ? b : 0) * a.ld_xtok] : (size_t)(xok[nb] ? b : 0);
    xbase[nb] = a.x_packed ? reinterpret_cast<const u32x4*>(a.x) + nb * 64 + lane
                           : reinterpret_cast<const u32x4*>(a.x + row * a.ldx + (lane >> 4) * 8);
  }
  // Small norm prologues (B = 1 at K 4096, the batch-1 decode step's q|k|v and gate|up) load
  // their inputs -- x rows, the norm weight, the sums of squares -- into registers BEFORE the
  // first weight batch: a wave's vmcnt counts in order, so a prologue load issued after the
  // weight loads could only be waited for together with them (the whole first batch would have
  // to land before the prologue could start).
  // (the host picks PRO_NORM_PRE only when norm_preload_fits: (B+1)*K/8 <= 1024 chunks)
  constexpr int XPT = PRER ? PREROW_MAXB + 1 : (PREL ? (1024 + NW * 64 - 1) / (NW * 64) : 1);  // chunks per thread
  const int K8p = KT * 4;
  const int n8p = a.B * K8p + K8p;
  u32x4 xr[XPT], nr[PRER ? 1 : XPT], sr[2];
  if constexpr (PRER) {
    // chunk j of every thread is row j (x rows, then the norm weight): the source is uniform
    constexpr uint32_t OOB = 0x7ffffff0u;
#pragma unroll
    for (int j = 0; j < XPT; ++j) {
      const bf16_t* src = j < a.B ? a.x + (size_t)j * a.ldx : a.nw;
      const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(const_cast<bf16_t*>(src), 0, a.K * 2, 0x00020000);
      xr[j] = __builtin_amdgcn_raw_buffer_load_b128(rs, j <= a.B ? (uint32_t)threadIdx.x * 16u : OOB, 0, 0);
    }
    const __amdgpu_buffer_rsrc_t srs = __builtin_amdgcn_make_buffer_rsrc(
        const_cast<float*>(a.ss_in), 0, (int)(((size_t)(a.B - 1) * a.ld_ss + a.n_ss) * 4), 0x00020000);
#pragma unroll
    for (int m = 0; m < 2; ++m) {
      const int b = wave + m * NW;
      const uint32_t so = (b < a.B && lane * 4 < a.n_ss) ? (uint32_t)(b * a.ld_ss + lane * 4) * 4u : OOB;
      sr[m] = __builtin_amdgcn_raw_buffer_load_b128(srs, so, 0, 0);
    }
  } else if constexpr (PREL) {
    {
      // branch-free buffer loads (out-of-range offsets read zero): a load under a divergent
      // branch is waited for at once (vmcnt(0)) by the compiler
      constexpr uint32_t OOB = 0x7ffffff0u;
      const int nx = a.B * K8p;
      const __amdgpu_buffer_rsrc_t xrs = __builtin_amdgcn_make_buffer_rsrc(
          const_cast<bf16_t*>(a.x), 0, (int)(((size_t)(a.B - 1) * a.ldx + a.K) * 2), 0x00020000);
      const __amdgpu_buffer_rsrc_t nrs = __builtin_amdgcn_make_buffer_rsrc(const_cast<bf16_t*>(a.nw), 0, a.K * 2, 0x00020000);
      const __amdgpu_buffer_rsrc_t srs = __builtin_amdgcn_make_buffer_rsrc(
          const_cast<float*>(a.ss_in), 0, (int)(((size_t)(a.B - 1) * a.ld_ss + a.n_ss) * 4), 0x00020000);
#pragma unroll
      for (int j = 0; j < XPT; ++j) {
        const int i = threadIdx.x + j * NW * 64;
        const int b = i / K8p, c = i - b * K8p;
        const uint32_t xo = i < nx ? (uint32_t)(b * a.ldx + c * 8) * 2u : OOB;
        const uint32_t no = (i >= nx && i < n8p) ? (uint32_t)(c * 16) : OOB;
        xr[j] = __builtin_amdgcn_raw_buffer_load_b128(xrs, xo, 0, 0);
        nr[j] = __builtin_amdgcn_raw_buffer_load_b128(nrs, no, 0, 0);
      }
#pragma unroll
      for (int m = 0; m < 2; ++m) {
        const int b = wave + m * NW;
        const uint32_t so = (b < a.B && lane * 4 < a.n_ss) ? (uint32_t)(b * a.ld_ss + lane * 4) * 4u : OOB;
        sr[m] = __builtin_amdgcn_raw_buffer_load_b128(srs, so, 0, 0);
      }
    }
  }
  extern __shared__ u32x4 xs_dyn[];
  if constexpr (DMAN) {
    // x rows then the norm weight (one contiguous LDS run of (B+1)*K8 chunks), then the B rows'
    // sums of squares; 64 16-byte chunks per wave-instruction, out-of-range chunks read zero
    typedef __attribute__((address_space(3))) void lvoid;
    const int K8d = KT * 4, nx = a.B * K8d, nxs = nx + K8d;
    const int cx = (nxs + 63) / 64 * 64, ns4 = a.B * a.n_ss / 4;
    const __amdgpu_buffer_rsrc_t xrs = __builtin_amdgcn_make_buffer_rsrc(const_cast<bf16_t*>(a.x), 0, nx * 16, 0x00020000);
    const __amdgpu_buffer_rsrc_t nrs = __builtin_amdgcn_make_buffer_rsrc(const_cast<bf16_t*>(a.nw), 0, K8d * 16, 0x00020000);
    const __amdgpu_buffer_rsrc_t srs = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(a.ss_in), 0, ns4 * 16, 0x00020000);
    for (int c0 = wave * 64; c0 < cx; c0 += NW * 64) {
      const int i = c0 + lane;
      if (c0 + 64 <= nx)  // wave-uniform branches: whole instructions from one source
        __builtin_amdgcn_raw_ptr_buffer_load_lds(xrs, (lvoid*)(xs_dyn + c0), 16, (uint32_t)i * 16u, 0, 0, 0);
      else if (c0 >= nx)
        __builtin_amdgcn_raw_ptr_buffer_load_lds(nrs, (lvoid*)(xs_dyn + c0), 16, (uint32_t)(i - nx) * 16u, 0, 0, 0);
      else  // straddles the x / weight boundary: x lanes, then weight lanes (both OOB-zeroed)
        __builtin_amdgcn_raw_ptr_buffer_load_lds(i < nx ? xrs : nrs, (lvoid*)(xs_dyn + c0), 16,
                                                 (uint32_t)(i < nx ? i : i - nx) * 16u, 0, 0, 0);
    }
    for (int c0 = wave * 64; c0 < ns4; c0 += NW * 64)
      __builtin_amdgcn_raw_ptr_buffer_load_lds(srs, (lvoid*)(xs_dyn + cx + c0), 16, (uint32_t)(c0 + lane) * 16u, 0, 0, 0);
  }
  // PREA: this thread's elements (up to PA_E: threadIdx.x + e * NW * 64) of the attention output
  // -- (m, l) of its head and 8 dims of o -- for splits 0 and 1, loaded now (a third and later
  // split, contexts > 512, load after)
  constexpr int PA_E = PRO0 == PRO_ATTN_PRE2 ? 2 : 1;
  float4 pa_o[PA_E][2][2];
  float2 pa_ml[PA_E][2];
  int pa_d0[PA_E], pa_kvh[PA_E], pa_hg[PA_E], pa_b[PA_E];
  if constexpr (PREA) {
    constexpr uint32_t OOB = 0x7ffffff0u;
    const AttnPartView& v = a.attn;
    const int G = v.G, D = v.D, PS = G * (D + 2);
    const int K8a = KT * 4;
    const __amdgpu_buffer_rsrc_t prs = __builtin_amdgcn_make_buffer_rsrc(
        const_cast<float*>(v.part), 0, (int)((size_t)a.B * v.Hkv * v.ns * PS * 4), 0x00020000);
#pragma unroll
    for (int e = 0; e < PA_E; ++e) {
      const int i = threadIdx.x + e * NW * 64;
      pa_b[e] = i / K8a;
      const int k0 = (i - pa_b[e] * K8a) * 8;
      const int h = k0 / D;
      pa_d0[e] = k0 - h * D; pa_kvh[e] = h / G; pa_hg[e] = h - pa_kvh[e] * G;
      const bool ok = i < a.B * K8a;
      const uint32_t base = (uint32_t)(((pa_b[e] * v.Hkv + pa_kvh[e]) * v.ns) * PS) * 4u;
#pragma unroll
      for (int s2 = 0; s2 < 2; ++s2) {
        const bool sok = ok && s2 < v.ns;
        const uint32_t so = base + (uint32_t)(s2 * PS) * 4u;
        const auto m = __builtin_amdgcn_raw_buffer_load_b64(prs, sok ? so + (uint32_t)(G * D + 2 * pa_hg[e]) * 4u : OOB, 0, 0);
        const u32x4 o0 = __builtin_amdgcn_raw_buffer_load_b128(prs, sok ? so + (uint32_t)(pa_hg[e] * D + pa_d0[e]) * 4u : OOB, 0, 0);
        const u32x4 o1 = __builtin_amdgcn_raw_buffer_load_b128(prs, sok ? so + (uint32_t)(pa_hg[e] * D + pa_d0[e] + 4) * 4u : OOB, 0, 0);
        pa_ml[e][s2] = make_float2(__uint_as_float(m[0]), __uint_as_float(m[1]));
        pa_o[e][s2][0] = make_float4(__uint_as_float(o0[0]), __uint_as_float(o0[1]), __uint_as_float(o0[2]), __uint_as_float(o0[3]));
        pa_o[e][s2][1] = make_float4(__uint_as_float(o1[0]), __uint_as_float(o1[1]), __uint_as_float(o1[2]), __uint_as_float(o1[3]));
      }
    }
  }
  // EPI_RESADD: the residual elements this thread adds in the epilogue, loaded now (issued before
  // the weights, so the epilogue's wait finds them landed; loaded there, they were one more
  // dependent L2-miss round trip after the reduction).  Thread t < 256 owns element t of each
  // output tile (see the epilogue's index map); out-of-range elements read zero.
  constexpr int OTR = EPI == EPI_RESADD ? RT : 1;
  constexpr int NBR = EPI == EPI_RESADD ? NB : 1;
  uint16_t resv[OTR][NBR];
  if constexpr (EPI == EPI_RESADD) {
    constexpr uint32_t OOB = 0x7ffffff0u;
    const int t = threadIdx.x, ln = t >> 2, nl = ((ln >> 4) << 2) + (t & 3);
    const __amdgpu_buffer_rsrc_t rrs = __builtin_amdgcn_make_buffer_rsrc(
        const_cast<bf16_t*>(a.res), 0, (int)(((size_t)(a.B - 1) * a.ldres + a.N) * 2), 0x00020000);
#pragma unroll
    for (int ot = 0; ot < OTR; ++ot)
#pragma unroll
      for (int nb = 0; nb < NBR; ++nb) {
        const int n = (bt * OTR + ot) * 16 + nl, b = (ln & 15) + 16 * nb;
        const bool ok = t < 256 && b < a.B && n < a.N;
        resv[ot][nb] = __builtin_amdgcn_raw_buffer_load_b16(rrs, ok ? (uint32_t)(b * a.ldres + n) * 2u : OOB, 0, 0);
      }
  }
  // all weight loads of the first k-batch go out before the (latency-bound) norm prologue
  int kt = kt0;
  u32x4 wa[RT][U];
  u32x4 xb[NB][U];
  // A batch is always U loads; a wave's last batch may cover n < U k-tiles, its surplus loads
  // re-read the wave's last tile (in-bounds, L2 hits) and their MFMAs see a zero A operand, so
  // the remainder costs one round trip instead of n dependent single-tile ones.
  auto issue_w = [&](int k) {
#pragma unroll
    for (int u = 0; u < U; ++u)
#pragma unroll
      for (int r = 0; r < RT; ++r)
#if GEMV_PROBE == 2  // timing probe build: no weight loads
        wa[r][u] = (u32x4){(uint32_t)(k + u), (uint32_t)lane, 0u, 0u};
#else
        wa[r][u] = __builtin_nontemporal_load(wbase[r] + (size_t)min(k + u, kt1 - 1) * 64);
#endif
  };
  // the preloads must be ISSUED first: stop the scheduler from hoisting the weight loads above them
  if constexpr (PREL || PREA || DMAN || EPI == EPI_RESADD) __builtin_amdgcn_sched_barrier(0);
  // unconditional (a wave with an empty K range re-reads its row's last tile, in bounds): a load
  // issue under a branch makes the compiler wait for the preloads with everything else at the
  // join (B=4 also 3.56 -> 3.53 ms/step)
  issue_w(kt);
  wait();  // fused launches: the producer of x (e.g. the attention blocks) has finished

  // Prologues (PRO) stage the block's B activation rows in LDS once; the MFMA B fragments
  // are then LDS reads.  PRO_NONE reads the fragments straight from x (L2).
  //   PRO_NORM:  bf16(nw * bf16(x * r_b)), r_b from the producer's per-16-column sums of
  //              squares (Qwen3RMSNorm, TF/models/qwen3/modeling_qwen3.py:59-64)
  //   PRO_ATTN:  the decode attention output, merged here from its per-split (m, l, o)
  //              partials in split order: x = bf16(sum_s f_s o_s / sum_s f_s l_s),
  //              f_s = exp(m_s - max m) -- the cross-block combine of attn_decode
  const int K8 = KT * 4;  // 16-byte chunks per row
  if constexpr (PRO == PRO_NORM) {
    __shared__ float r_s[32];
    const int n8x = a.B * K8;
    if constexpr (PREL) {
      if constexpr (PRER) {
#pragma unroll
        for (int j = 0; j < XPT; ++j)
          if (j <= a.B) xs_dyn[j * K8 + threadIdx.x] = xr[j];
      } else {
#pragma unroll
        for (int j = 0; j < XPT; ++j) {
          const int i = threadIdx.x + j * NW * 64;
          if (i < n8x + K8) xs_dyn[i] = xr[j] | nr[j];  // one of the two is zero (out of range)
        }
      }
#pragma unroll
      for (int m = 0; m < 2; ++m) {
        const int b = wave + m * NW;
        const float ss = wave_sum((__uint_as_float(sr[m][0]) + __uint_as_float(sr[m][1])) +
                                  (__uint_as_float(sr[m][2]) + __uint_as_float(sr[m][3])));
        if (b < a.B && lane == 0) r_s[b] = 1.0f / sqrtf(ss / (float)a.K + a.eps);
      }
    } else if constexpr (DMAN) {
      // the DMA loads were issued before this wave's U*RT weight loads: in-order vmcnt
      asm volatile("s_waitcnt vmcnt(%0)" ::"n"(U * RT) : "memory");
      __syncthreads();  // every wave's chunks have landed
      const float* ssl = reinterpret_cast<const float*>(xs_dyn + (n8x + K8 + 63) / 64 * 64);
      // the same order as PRO_NORM / PRO_NORM_PRE (4 contiguous per lane, pairwise, then the
      // wave), so every prologue form gives the same bits (gemv_ex checks n_ss % 4 == 0)
      for (int b = wave; b < a.B; b += NW) {
        float ss = 0.f;
        for (int t4 = lane * 4; t4 < a.n_ss; t4 += 256) {
          const float4 v = *reinterpret_cast<const float4*>(ssl + b * a.n_ss + t4);
          ss += (v.x + v.y) + (v.z + v.w);
        }
        ss = wave_sum(ss);
        if (lane == 0) r_s[b] = 1.0f / sqrtf(ss / (float)a.K + a.eps);
      }
    } else {
    for (int i = threadIdx.x; i < n8x + K8; i += NW * 64) {
      const int b = i / K8, c = i - b * K8;
      xs_dyn[i] = i < n8x ? reinterpret_cast<const u32x4*>(a.x + (size_t)b * a.ldx)[c]
                          : reinterpret_cast<const u32x4*>(a.nw)[c];
    }
    for (int b = wave; b < a.B; b += NW) {
      const float* sp = a.ss_in + (size_t)b * a.ld_ss;
      float ss = 0.f;
      for (int t4 = lane * 4; t4 < a.n_ss; t4 += 256) {
        const float4 v = *reinterpret_cast<const float4*>(sp + t4);
        ss += (v.x + v.y) + (v.z + v.w);
      }
      ss = wave_sum(ss);
      if (lane == 0) r_s[b] = 1.0f / sqrtf(ss / (float)a.K + a.eps);
    }
    }
    __syncthreads();
    for (int i = threadIdx.x; i < n8x; i += NW * 64) {
      const int b = i / K8;
      xs_dyn[i] = norm8(xs_dyn[i], xs_dyn[n8x + i - b * K8], r_s[b]);
    }
    __syncthreads();
  } else if constexpr (PREA) {
    const AttnPartView& v = a.attn;
    const int nact = *v.pos / v.kb + 1;
    const int G = v.G, D = v.D, PS = G * (D + 2);
#pragma unroll
    for (int e = 0; e < PA_E; ++e) {
      const int i = threadIdx.x + e * NW * 64;
      if (i >= a.B * K8) continue;
      if (nact > v.po_max) {  // long context: the attention merged its splits into x (bf16 rows)
        const int b = i / K8, c = i - b * K8;
        xs_dyn[i] = reinterpret_cast<const u32x4*>(a.x + (size_t)b * a.ldx)[c];
        continue;
      }
      const float* pp = v.part + ((size_t)pa_b[e] * v.Hkv + pa_kvh[e]) * v.ns * PS;
      const int hg = pa_hg[e], d0 = pa_d0[e];
      float M = -INFINITY;
      for (int s2 = 0; s2 < nact; ++s2) M = fmaxf(M, s2 < 2 ? pa_ml[e][s2 & 1].x : pp[(size_t)s2 * PS + G * D + 2 * hg]);
      float L = 0.f, o[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
      for (int s2 = 0; s2 < nact; ++s2) {
        float ms, ls;
        float4 o0, o1;
        if (s2 < 2) {
          ms = pa_ml[e][s2 & 1].x; ls = pa_ml[e][s2 & 1].y; o0 = pa_o[e][s2 & 1][0]; o1 = pa_o[e][s2 & 1][1];
        } else {
          const float* q = pp + (size_t)s2 * PS;
          ms = q[G * D + 2 * hg]; ls = q[G * D + 2 * hg + 1];
          o0 = *reinterpret_cast<const float4*>(q + hg * D + d0);
          o1 = *reinterpret_cast<const float4*>(q + hg * D + d0 + 4);
        }
        const float f = (ms == -INFINITY) ? 0.f : expf(ms - M);
        L += f * ls;
        o[0] += f * o0.x; o[1] += f * o0.y; o[2] += f * o0.z; o[3] += f * o0.w;
        o[4] += f * o1.x; o[5] += f * o1.y; o[6] += f * o1.z; o[7] += f * o1.w;
      }
      u32x4 r;
#pragma unroll
      for (int q2 = 0; q2 < 4; ++q2) r[q2] = L > 0.f ? pack2(o[2 * q2] / L, o[2 * q2 + 1] / L) : 0u;
      xs_dyn[i] = r;
    }
    __syncthreads();
  } else if constexpr (PRO == PRO_ATTN) {
    const AttnPartView& v = a.attn;
    const int nact = *v.pos / v.kb + 1;
    const int G = v.G, D = v.D, PS = G * (D + 2);
    if (nact > v.po_max)  // long context: the attention merged its splits into x (bf16 rows)
      for (int i = threadIdx.x; i < a.B * K8; i += NW * 64) {
        const int b = i / K8, c = i - b * K8;
        xs_dyn[i] = reinterpret_cast<const u32x4*>(a.x + (size_t)b * a.ldx)[c];
      }
    else
    for (int i = threadIdx.x; i < a.B * K8; i += NW * 64) {
      const int b = i / K8, k0 = (i - b * K8) * 8;
      const int h = k0 / D, d0 = k0 - h * D, kvh = h / G, hg = h - kvh * G;
      const float* pp = v.part + ((size_t)b * v.Hkv + kvh) * v.ns * PS;
      float M = -INFINITY;
      for (int s2 = 0; s2 < nact; ++s2) M = fmaxf(M, pp[(size_t)s2 * PS + G * D + 2 * hg]);
      float L = 0.f, o[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
      for (int s2 = 0; s2 < nact; ++s2) {
        const float* q = pp + (size_t)s2 * PS;
        const float ms = q[G * D + 2 * hg];
        const float f = (ms == -INFINITY) ? 0.f : expf(ms - M);
        L += f * q[G * D + 2 * hg + 1];
        const float4 o0 = *reinterpret_cast<const float4*>(q + hg * D + d0);
        const float4 o1 = *reinterpret_cast<const float4*>(q + hg * D + d0 + 4);
        o[0] += f * o0.x; o[1] += f * o0.y; o[2] += f * o0.z; o[3] += f * o0.w;
        o[4] += f * o1.x; o[5] += f * o1.y; o[6] += f * o1.z; o[7] += f * o1.w;
      }
      u32x4 r;
#pragma unroll
      for (int q2 = 0; q2 < 4; ++q2) r[q2] = L > 0.f ? pack2(o[2 * q2] / L, o[2 * q2 + 1] / L) : 0u;
      xs_dyn[i] = r;
    }
    __syncthreads();
  }
  // (k < kt1 and the row clamp keep every LDS address inside the staged rows)
  auto load_x = [&](int k, int nb) -> u32x4 {
    if constexpr (PRO != PRO_NONE) {
      if (!xok[nb]) return (u32x4){0u, 0u, 0u, 0u};
      return xs_dyn[((lane & 15) + 16 * nb) * K8 + k * 4 + (lane >> 4)];
    }
    // unconditional global load: a "load or zero" select would branch and wait on every load
    // (cdna_hip_programming.md trap (c)); token columns >= B read row 0 and are never stored
#if GEMV_PROBE == 1  // timing probe build: no x loads
    return (u32x4){(uint32_t)k, (uint32_t)nb, (uint32_t)lane, 0u};
#else
    return xbase[nb][k * xs];
#endif
  };

  auto compute = [&](u32x4 (&w)[RT][U], int k) {
    const int n = kt1 - k;  // k-tiles of this batch that are real (>= U: all)
#pragma unroll
    for (int u = 0; u < U; ++u)
#pragma unroll
      for (int nb = 0; nb < NB; ++nb) xb[nb][u] = load_x(min(k + u, kt1 - 1), nb);
#pragma unroll
    for (int u = 0; u < U; ++u)
#pragma unroll
      for (int r = 0; r < RT; ++r) {
        const u32x4 wv = u < n ? w[r][u] : (u32x4){0u, 0u, 0u, 0u};
#pragma unroll
        for (int nb = 0; nb < NB; ++nb)
          acc[r][nb] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(
              __builtin_bit_cast(bf16x8, wv), __builtin_bit_cast(bf16x8, xb[nb][u]), acc[r][nb], 0, 0, 0);
      }
  };
  for (; kt < kt1; kt += U) {
    if (kt != kt0) issue_w(kt);
    compute(wa, kt);
  }

  // ---- fixed-order reduction of the NW waves' partial tiles through LDS ----
  // SwiGLU: the RT = 2 tiles are a gate and an up tile -> one output tile; otherwise each of
  // the RT row tiles is an output tile (RT = 2 amortises the x fragments over 32 weight rows)
  constexpr int OT = EPI == EPI_SWIGLU ? 1 : RT;
  __shared__ float red[NW][RT][NB][256];
  __shared__ float sq[OT][NB][16][17];
#pragma unroll
  for (int r = 0; r < RT; ++r)
#pragma unroll
    for (int nb = 0; nb < NB; ++nb)
#pragma unroll
      for (int i = 0; i < 4; ++i) red[wave][r][nb][lane * 4 + i] = acc[r][nb][i];
  __syncthreads();

  const int t = threadIdx.x;
  if (t < 256) {
    // element t: lane = t/4, reg = t%4 -> n = ((lane>>4)*4 + reg), b = lane & 15
    const int ln = t >> 2;
    const int nl = ((ln >> 4) << 2) + (t & 3);
#pragma unroll
    for (int ot = 0; ot < OT; ++ot) {
      const int n = (bt * OT + ot) * 16 + nl;
#pragma unroll
      for (int nb = 0; nb < NB; ++nb) {
        const int bl = ln & 15;
        const int b = bl + 16 * nb;
        float v[RT];
#pragma unroll
        for (int r = 0; r < RT; ++r) {
          float s = 0.f;
#pragma unroll
          for (int w = 0; w < NW; ++w) s += red[w][r][nb][t];
          v[r] = s;
        }
        const float vo = v[EPI == EPI_SWIGLU ? 0 : ot];
        bf16_t out = 0;
        if constexpr (EPI == EPI_STORE) {
          out = f2bf(vo);
        } else if constexpr (EPI == EPI_LOGITS) {
          out = f2bf(vo);
          if (n >= a.pad_start && ((n - a.pad_start) % a.pad_period) == a.pad_off) out = 0xFF80;  // -inf
        } else if constexpr (EPI == EPI_RESADD) {
          // hidden = residual + bf16(o)   (TF/.../modeling_qwen3.py:311,322)
          if (b < a.B && n < a.N) out = f2bf(bf2f(resv[ot][nb]) + rbf(vo));
          const float ho = bf2f(out);
          sq[ot][nb][bl][nl] = ho * ho;
        } else {  // EPI_SWIGLU: bf16(bf16(silu(bf16 g)) * bf16 u)   (TF/.../modeling_qwen3.py:81-83)
          const float g = rbf(v[0]);
          const float u = rbf(v[RT - 1]);
          const float s = rbf(g / (1.0f + expf(-g)));
          out = f2bf(s * u);
        }
        if (b < a.B && n < a.N) {
          if (a.y_packed)
            a.y[xpk_index(b, n)] = out;
          else if constexpr (WT)
            __hip_atomic_store((__attribute__((address_space(1))) uint16_t*)(a.y + (size_t)b * a.ldy + n), out,
                               __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          else
            a.y[(size_t)b * a.ldy + n] = out;
        }
      }
    }
  }
  if constexpr (EPI == EPI_RESADD) {
    __syncthreads();
    if (a.ss_out && t < 16 * NB * OT) {
      const int ot = t / (16 * NB), nb = (t >> 4) % NB, bl = t & 15, b = bl + 16 * nb;
      if (b < a.B) {
        float s = 0.f;
#pragma unroll
        for (int i = 0; i < 16; ++i) s += sq[ot][nb][bl][i];
        a.ss_out[(size_t)b * a.ld_ss_out + bt * OT + ot] = s;
      }
    }
  }
}


}  // namespace mtts
