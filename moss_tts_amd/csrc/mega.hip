// The decoder-layer stack of one decode step (S = 1, B <= MEGA_MAXB rows) as ONE persistent
// launch: every stage of every layer of the Qwen3 backbone
//   q|k|v (input RMSNorm fused)  ->  attention (q/k norm, RoPE, KV append, split partials)
//   ->  o_proj (+ residual)  ->  gate|up (post-attention RMSNorm fused, SwiGLU)  ->  down (+ residual)
// (TF/models/qwen3/modeling_qwen3.py:294-323 per layer, :241-280 attention, :81-83 MLP)
// replaces the 5 x 36 dependent kernel launches of run_layers' decode path.
//
// Why: at batch 1 every launch pays a grid fill / drain and a dependent-launch boundary
// (~1.5 us, MI355X_MICROARCH.md "boundary"), ~20 us of every 84 us layer.  Inside one launch
// a workgroup issues the NEXT stage's first weight batch before it waits for that stage's
// inputs, so the HBM stream does not drain at stage seams; the attention chain overlaps the
// o_proj weight stream.
//
// Geometry: one 512-thread workgroup per CU (the LDS request keeps it at one), all resident
// (checked against the occupancy query on the host).  Waves 0-6 are STREAMERS: each keeps
// up to two 8-k-tile weight batches in flight (ping-pong registers) and runs the MFMAs of
// v_mfma_f32_16x16x32_bf16 (weights = A operand straight from the packed 1 KiB tiles,
// activations = B operand from LDS), the K range of a 16-row tile split over the 7 waves.
// Wave 7 is the CONTROL wave: it polls the producer stage's completion counter, stages the
// stage's activation rows in LDS (RMSNorm / attention-partial merge / copy), reduces the 7
// waves' partial tiles in a fixed order (deterministic) and runs the epilogue.  The control
// wave holds no weight loads, so its polls and hand-off loads never queue behind them.
//
// Work split per stage (P = gridDim.x): GEMV unit u (a 16- or 32-row output tile) runs on
// block u % P; attention units (row, KV head, split of 256 keys) run on blocks P-1-u % P,
// i.e. on the blocks that have no q|k|v tile when there are fewer q|k|v tiles than blocks.
//
// Hand-offs (cdna_hip_programming.md Guideline 16, R1): every handed-off byte (q|k|v rows,
// attention partials, residual stream h and its per-16-column sums of squares, SwiGLU
// activations) is stored write-through (sc1) by the control wave; the storing wave drains
// (s_waitcnt vmcnt(0)) before one lane adds the stage's unit count to the stage counter
// (agent-scope atomic).  Consumers poll the counter relaxed (sc1) and read the payload with
// sc1 loads; the attention units read q|k|v with plain loads behind one agent acquire.
// Every spin is bounded: a stuck wait sets the error word and the launch drains.
// Counters are zero between launches (zeroed at allocation; the last workgroup to leave
// resets them).
#include "attn_body.h"

namespace mtts {

namespace {

constexpr int NW = 7;                   // streamer waves (K split 7 ways, within one k-tile)
constexpr int THREADS = (NW + 1) * 64;  // + the control wave
constexpr int ANW = NW + 1;             // attention units run on all waves
constexpr int AKB = DEC_KW * ANW;       // keys per attention unit
#ifndef MEGA_WS
#define MEGA_WS 8
#endif
constexpr int WS = MEGA_WS;             // weight slots per batch (one 1 KiB tile each): WS k-tiles of
                                        // one row tile, or WS/2 k-tiles of two
constexpr int NST = 5;                  // stages per layer

enum { S_QKV = 0, S_ATT = 1, S_O = 2, S_GU = 3, S_DOWN = 4 };

typedef __attribute__((address_space(1))) uint64_t g64;
typedef __attribute__((address_space(1))) uint32_t g32;

__device__ __forceinline__ void st64(void* p, uint64_t v) {
  __hip_atomic_store((g64*)p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void st32(void* p, uint32_t v) {
  __hip_atomic_store((g32*)p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ uint64_t ld64(const void* p) {
  return __hip_atomic_load((g64*)p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ uint32_t ld32(const void* p) {
  return __hip_atomic_load((g32*)p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc(const void* p) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(p), 0, 0x7fffffff, 0x00020000);
}
// 16-byte write-through-coherent load (sc1: served past this CU's L1)
__device__ __forceinline__ u32x4 ld128(__amdgpu_buffer_rsrc_t r, uint32_t byte_off) {
  return __builtin_amdgcn_raw_buffer_load_b128(r, byte_off, 0, 16);
}
__device__ __forceinline__ void drain() { asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); }
// LDS <- global, 16 B per lane straight into LDS (global_load_lds_dwordx4 sc1), n chunks; the
// caller waits (vmcnt) before reading them
__device__ __forceinline__ void dma16(const void* src, void* lds_dst, int n, int lane) {
  typedef __attribute__((address_space(1))) void gvoid;
  typedef __attribute__((address_space(3))) void lvoid;
  for (int i0 = 0; i0 < n; i0 += 64)
    if (i0 + lane < n)
      __builtin_amdgcn_global_load_lds((const gvoid*)(reinterpret_cast<const u32x4*>(src) + i0 + lane),
                                       (lvoid*)(reinterpret_cast<u32x4*>(lds_dst) + i0), 16, 0, 16);
}
__device__ __forceinline__ uint64_t now() { return __builtin_amdgcn_s_memrealtime(); }

}  // namespace

namespace {

struct StageGeo {
  const bf16_t* w;
  int KT;       // k-tiles of the matrix
  int rt;       // row tiles per unit
  int units;
};

__device__ __forceinline__ StageGeo stage_geo(const MegaArgs& a, const MegaLayer& Lw, int s) {
  switch (s) {
    case S_QKV: return {Lw.qkv, a.H / 32, 2, a.qkv_rows / 32};
    case S_O: return {Lw.o, a.Hq * a.D / 32, 1, a.H / 16};
    case S_GU: return {Lw.gu, a.H / 32, 2, a.I / 16};
    default: return {Lw.down, a.I / 32, 1, a.H / 16};
  }
}

__device__ __forceinline__ int n_mine(int units, int bid, int P) { return bid < units ? (units - bid + P - 1) / P : 0; }

// the unit a stage waits for: (layer, stage) of its producer, and that producer's unit count
__device__ __forceinline__ bool wait_ge(const uint32_t* c, uint32_t target, uint32_t* err) {
  for (uint32_t spins = 0;; ++spins) {
    if (ld32(c) >= target) return true;
    if ((spins & 255) == 255 && ld32(err)) return false;  // another workgroup gave up
    if (spins > (1u << 20)) {                             // ~1 s: give up, report, drain
      st32(err, 1u);
      return false;
    }
    __builtin_amdgcn_s_sleep(1);
  }
}

// streamer job: one 8-k-tile weight batch of one unit, or the attention stage of a layer
struct Job {
  int valid, att;
  int l, s, j, kb, nb;
  int u;            // unit index (GEMV)
  int k, n;         // first k-tile of the batch, real k-tiles in it
  int rt, KT;
  const u32x4* w0;  // row tile 0 of the unit, this lane
};

}  // namespace

// the attention stage of layer l on this workgroup (all waves; the control wave polls the
// q|k|v counter and acquires first)
template <int G, int D>
__device__ __forceinline__ void mega_att_stage(const MegaArgs& a, int l, int nact, int n_att, int n_att_mine,
                                                         int att_first) {
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const bool ctl = wave == NW;
  const int P = gridDim.x;
  uint64_t* tr = a.trace ? a.trace + ((size_t)(l * NST + S_ATT) * P + blockIdx.x) * 4 : nullptr;
  if (tr && ctl && lane == 0) tr[0] = now();
  if (ctl) {
    wait_ge(a.sync + l * NST + S_QKV, (uint32_t)(a.qkv_rows / 32), a.sync + a.w_err);
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
    drain();
    if (tr && lane == 0) tr[1] = tr[2] = now();
  }
  __syncthreads();
  const MegaLayer& Lw = a.L[l];
  DecAttnArgs da{};
  da.cos_t = a.cos_t; da.sin_t = a.sin_t; da.mask = a.mask; da.pos = a.pos; da.part = a.part;
  da.qkv = a.qkvb; da.Hq = a.Hq; da.Hkv = a.Hkv; da.D = a.D; da.Cmax = a.Cmax; da.ns = a.ns; da.nwv = ANW;
  da.eps = a.eps; da.scale = a.scale; da.publish_only = 0; da.out = a.attnb;
  da.cnt = reinterpret_cast<int*>(a.sync + a.layers * NST + l * MEGA_MAXB * a.Hkv);
  da.qn_w = Lw.q_norm; da.kn_w = Lw.k_norm; da.kc = Lw.kc; da.vc = Lw.vc;
  for (int u = att_first; u < n_att; u += P) {
    const int sp = u % nact, rest = u / nact;
    attn_decode_body<G, D, ANW, true>(da, sp, rest % a.Hkv, rest / a.Hkv);
  }
  drain();
  __syncthreads();
  if (ctl && lane == 0) {
    __hip_atomic_fetch_add((g32*)(a.sync + l * NST + S_ATT), (uint32_t)n_att_mine, __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_AGENT);
    if (tr) tr[3] = now();
  }
}

template <int G, int D>
__global__ __launch_bounds__(THREADS) void mega_decode_kernel(MegaArgs a) {
  extern __shared__ __attribute__((aligned(16))) unsigned char lds_dyn[];
  float* red = reinterpret_cast<float*>(lds_dyn);  // [2][NW][2][256] partial tiles (ping-pong)
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const bool ctl = wave == NW;
  const int P = gridDim.x, bid = blockIdx.x;
  const int pos = *a.pos;
  const int nact = pos / AKB + 1;
  const int n_att = a.B * a.Hkv * nact;
  const int att_first = P - 1 - bid;  // this block's first attention unit
  const int n_att_mine = att_first < n_att ? (n_att - att_first + P - 1) / P : 0;
  uint32_t* err = a.sync + a.w_err;
  const int B = a.B;

  auto att_stage = [&](int l) { mega_att_stage<G, D>(a, l, nact, n_att, n_att_mine, att_first); };

  if (ctl) {
    // =================== control wave ===================
    int par = 0;
    for (int l = 0; l < a.layers; ++l) {
      const MegaLayer& Lw = a.L[l];
      for (int s = 0; s < NST; ++s) {
        if (s == S_ATT) {
          if (n_att_mine) att_stage(l);
          continue;
        }
        const StageGeo g = stage_geo(a, Lw, s);
        const int nm = n_mine(g.units, bid, P);
        if (!nm) continue;
        uint64_t* tr = a.trace ? a.trace + ((size_t)(l * NST + s) * P + bid) * 4 : nullptr;
        if (tr && lane == 0) tr[0] = now();
        // ---- wait for the producer stage ----
        if (s == S_QKV) {
          if (l > 0) wait_ge(a.sync + (l - 1) * NST + S_DOWN, (uint32_t)(a.H / 16), err);
        } else if (s == S_O) {
          wait_ge(a.sync + l * NST + S_ATT, (uint32_t)n_att, err);
        } else if (s == S_GU) {
          wait_ge(a.sync + l * NST + S_O, (uint32_t)(a.H / 16), err);
        } else {
          wait_ge(a.sync + l * NST + S_GU, (uint32_t)(a.I / 16), err);
        }
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");  // keep the loads below the poll
        if (tr && lane == 0) tr[1] = now();
        // ---- stage the B activation rows in LDS: one round trip, every load in flight at
        // once (rows straight into LDS by global_load_lds; sc1 = past this CU's L1) ----
        const int K = g.KT * 32, K8 = K / 8;
        const bool normed = s == S_QKV || s == S_GU;
        u32x4* xs = reinterpret_cast<u32x4*>(lds_dyn + (normed ? a.lds_x1 : a.lds_x2));
        // the rows are contiguous in global memory (ld == K) and in LDS
        dma16(s == S_DOWN ? (const void*)a.act : (s == S_O ? (const void*)a.attnb : (const void*)a.h), xs, B * K8, lane);
        // residual of this block's first output tiles (o_proj / down epilogues)
        const int b_l = lane & 15, c4 = 4 * (lane >> 4);
        uint64_t res[2] = {0, 0};
        if (!normed && b_l < B) {
#pragma unroll
          for (int jj = 0; jj < 2; ++jj)
            if (jj < nm) res[jj] = ld64(a.h + (size_t)b_l * a.H + (bid + jj * P) * 16 + c4);
        }
        if (normed) {
          // Qwen3RMSNorm (TF/.../modeling_qwen3.py:59-64): bf16(w * bf16(x * r)), r from the
          // producer's per-16-column sums of squares
          const bf16_t* nw = s == S_QKV ? Lw.in_norm : Lw.post_norm;
          const int NT = a.H / 16;
          const auto rs = rsrc(a.ss);
          u32x4 sv[MEGA_MAXB][2];
#pragma unroll
          for (int b = 0; b < MEGA_MAXB; ++b)
#pragma unroll
            for (int t = 0; t < 2; ++t) {
              const int t4 = (t * 64 + lane) * 4;
              sv[b][t] = (b < B && t4 < NT) ? ld128(rs, (uint32_t)((b * NT + t4) * 4)) : (u32x4){0u, 0u, 0u, 0u};
            }
          constexpr int WC = 16;  // norm-weight chunks per lane held in registers (K <= 8192)
          u32x4 wv[WC];
#pragma unroll
          for (int i = 0; i < WC; ++i) {
            const int c = i * 64 + lane;
            wv[i] = c < K8 ? reinterpret_cast<const u32x4*>(nw)[c] : (u32x4){0u, 0u, 0u, 0u};
          }
          drain();
          float r[MEGA_MAXB];
#pragma unroll
          for (int b = 0; b < MEGA_MAXB; ++b) {
            float acc = 0.f;
#pragma unroll
            for (int t = 0; t < 2; ++t)
              acc += (__uint_as_float(sv[b][t][0]) + __uint_as_float(sv[b][t][1])) +
                     (__uint_as_float(sv[b][t][2]) + __uint_as_float(sv[b][t][3]));
            r[b] = 1.0f / sqrtf(wave_sum(acc) / (float)K + a.eps);
          }
          for (int b = 0; b < B; ++b)
#pragma unroll
            for (int i = 0; i < WC; ++i) {
              const int c = i * 64 + lane;
              if (c >= K8) continue;
              const u32x4 xv = xs[b * K8 + c];
              u32x4 o;
#pragma unroll
              for (int q = 0; q < 4; ++q) {
                const float x0 = __uint_as_float(xv[q] << 16), x1 = __uint_as_float(xv[q] & 0xffff0000u);
                const float w0 = __uint_as_float(wv[i][q] << 16), w1 = __uint_as_float(wv[i][q] & 0xffff0000u);
                o[q] = pack2(w0 * rbf(x0 * r[b]), w1 * rbf(x1 * r[b]));
              }
              xs[b * K8 + c] = o;
            }
        } else {
          drain();
        }
        if (tr && lane == 0) tr[2] = now();
        __syncthreads();  // A: the stage's activation rows are in LDS
        // ---- epilogues, one per unit ----
        for (int jj = 0; jj < nm; ++jj) {
          __syncthreads();  // B: the streamers' partial tiles of this unit are in red[par]
          const int u = bid + jj * P;
          const float* rp = red + par * (NW * 2 * 256);
          f32x4 v[2];
#pragma unroll
          for (int r = 0; r < 2; ++r) {
            v[r] = (f32x4){0.f, 0.f, 0.f, 0.f};
            if (r < g.rt)
#pragma unroll
              for (int w = 0; w < NW; ++w) {
                const f32x4 p = *reinterpret_cast<const f32x4*>(rp + (w * 2 + r) * 256 + lane * 4);
                v[r] += p;
              }
          }
          par ^= 1;
          // lane -> output row b = lane & 15, columns n0 .. n0+3 of the tile (MFMA D layout)
          const int b = lane & 15, c4 = 4 * (lane >> 4);
          const bool ok = b < B;
          if (s == S_QKV) {
#pragma unroll
            for (int r = 0; r < 2; ++r) {
              const int n0 = (2 * u + r) * 16 + c4;
              if (ok) st64(a.qkvb + (size_t)b * a.qkv_rows + n0,
                           (uint64_t)pack2(v[r][0], v[r][1]) | ((uint64_t)pack2(v[r][2], v[r][3]) << 32));
            }
          } else if (s == S_GU) {
            // bf16(bf16(silu(bf16 g)) * bf16 u)   (TF/.../modeling_qwen3.py:81-83)
            float o[4];
#pragma unroll
            for (int i = 0; i < 4; ++i) {
              const float gg = rbf(v[0][i]), uu = rbf(v[1][i]);
              o[i] = rbf(gg / (1.0f + expf(-gg))) * uu;
            }
            const int n0 = u * 16 + c4;
            if (ok) st64(a.act + (size_t)b * a.I + n0, (uint64_t)pack2(o[0], o[1]) | ((uint64_t)pack2(o[2], o[3]) << 32));
          } else {
            // hidden = residual + bf16(o)   (TF/.../modeling_qwen3.py:311,322), plus the new
            // columns' sum of squares for the next RMSNorm
            const int n0 = u * 16 + c4;
            float sq = 0.f;
            uint64_t packed = 0;
            if (ok) {
              const uint64_t rv = jj == 0 ? res[0] : (jj == 1 ? res[1] : ld64(a.h + (size_t)b * a.H + n0));
              float o[4];
#pragma unroll
              for (int i = 0; i < 4; ++i) {
                const float res = __uint_as_float((uint32_t)((rv >> (16 * i)) & 0xffffu) << 16);
                o[i] = rbf(res + rbf(v[0][i]));
                sq += o[i] * o[i];
              }
              packed = (uint64_t)pack2(o[0], o[1]) | ((uint64_t)pack2(o[2], o[3]) << 32);
              st64(a.h + (size_t)b * a.H + n0, packed);
            }
            sq += __shfl_xor(sq, 16, 64);
            sq += __shfl_xor(sq, 32, 64);
            if (ok && lane < 16) st32(a.ss + (size_t)b * (a.H / 16) + u, __float_as_uint(sq));
          }
        }
        drain();
        if (lane == 0) {
          __hip_atomic_fetch_add((g32*)(a.sync + l * NST + s), (uint32_t)nm, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          if (tr) tr[3] = now();
        }
      }
    }
  } else {
    // =================== streamer waves ===================
    // job generator over (layer, stage, unit, batch); attention stages with units of this
    // block are jobs of their own
    auto first_job = [&](int l, int s, Job& jb) {
      // first job at or after (l, s)
      for (; l < a.layers; ++l, s = 0) {
        const MegaLayer& Lw = a.L[l];
        for (; s < NST; ++s) {
          if (s == S_ATT) {
            if (n_att_mine) {
              jb.valid = 1; jb.att = 1; jb.l = l; jb.s = s;
              return;
            }
            continue;
          }
          const StageGeo g = stage_geo(a, Lw, s);
          const int nm = n_mine(g.units, bid, P);
          if (!nm) continue;
          const int k0 = wave * g.KT / NW, per = (wave + 1) * g.KT / NW - k0;
          jb.valid = 1; jb.att = 0; jb.l = l; jb.s = s; jb.j = 0; jb.kb = 0; jb.nb = (per + WS / g.rt - 1) / (WS / g.rt);
          jb.rt = g.rt; jb.KT = g.KT; jb.u = bid;
          jb.k = k0; jb.n = min(WS / g.rt, per);
          jb.w0 = reinterpret_cast<const u32x4*>(g.w) + (size_t)bid * g.rt * g.KT * 64 + lane;
          return;
        }
      }
      jb.valid = 0;
    };
    auto next_job = [&](const Job& c, Job& jb) {
      if (!c.att) {
        const int k0 = wave * c.KT / NW, k1 = (wave + 1) * c.KT / NW;
        if (c.kb + 1 < c.nb) {
          jb = c;
          jb.kb = c.kb + 1;
          jb.k = c.k + WS / c.rt;
          jb.n = min(WS / c.rt, k1 - jb.k);
          return;
        }
        const StageGeo g = stage_geo(a, a.L[c.l], c.s);
        if (c.j + 1 < n_mine(g.units, bid, P)) {
          jb = c;
          jb.j = c.j + 1; jb.kb = 0; jb.u = bid + jb.j * P;
          jb.k = k0; jb.n = min(WS / g.rt, k1 - k0);
          jb.w0 = reinterpret_cast<const u32x4*>(g.w) + (size_t)jb.u * g.rt * g.KT * 64 + lane;
          return;
        }
      }
      const int s = c.s + 1;
      first_job(s < NST ? c.l : c.l + 1, s < NST ? s : 0, jb);
    };

    f32x4 acc[2];
    acc[0] = acc[1] = (f32x4){0.f, 0.f, 0.f, 0.f};
    int par = 0;
    const int brow = lane & 15;
    const bool bok = brow < B;

    auto issue = [&](u32x4 (&w)[WS], const Job& jb) {
      const int kl = jb.k + jb.n - 1;  // surplus loads re-read the batch's last tile (zeroed below)
      if (jb.rt == 2) {
#pragma unroll
        for (int u = 0; u < WS / 2; ++u) {
          const int kk = min(jb.k + u, kl);
          w[2 * u] = __builtin_nontemporal_load(jb.w0 + (size_t)kk * 64);
          w[2 * u + 1] = __builtin_nontemporal_load(jb.w0 + ((size_t)jb.KT + kk) * 64);
        }
      } else {
#pragma unroll
        for (int u = 0; u < WS; ++u) w[u] = __builtin_nontemporal_load(jb.w0 + (size_t)min(jb.k + u, kl) * 64);
      }
    };
    auto process = [&](u32x4 (&w)[WS], const Job& jb) {
      if (jb.j == 0 && jb.kb == 0) __syncthreads();  // A: activation rows staged
      const int K8 = jb.KT * 4;
      const u32x4* xs = reinterpret_cast<const u32x4*>(lds_dyn + ((jb.s == S_QKV || jb.s == S_GU) ? a.lds_x1 : a.lds_x2));
      const u32x4 z = (u32x4){0u, 0u, 0u, 0u};
      auto xfrag = [&](int u) {
        const int kk = min(jb.k + u, jb.k + jb.n - 1);
        return bok ? xs[brow * K8 + kk * 4 + (lane >> 4)] : z;
      };
      if (jb.rt == 2) {
#pragma unroll
        for (int u = 0; u < WS / 2; ++u) {
          const u32x4 xb = xfrag(u);
          const u32x4 w0 = u < jb.n ? w[2 * u] : z, w1 = u < jb.n ? w[2 * u + 1] : z;
          acc[0] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, w0),
                                                           __builtin_bit_cast(bf16x8, xb), acc[0], 0, 0, 0);
          acc[1] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, w1),
                                                           __builtin_bit_cast(bf16x8, xb), acc[1], 0, 0, 0);
        }
      } else {
#pragma unroll
        for (int u = 0; u < WS; ++u) {
          const u32x4 xb = xfrag(u);
          const u32x4 w0 = u < jb.n ? w[u] : z;
          acc[0] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, w0),
                                                           __builtin_bit_cast(bf16x8, xb), acc[0], 0, 0, 0);
        }
      }
      if (jb.kb == jb.nb - 1) {  // the unit's last batch: publish the partial tile, B
        float* rp = red + par * (NW * 2 * 256) + wave * 2 * 256 + lane * 4;
        *reinterpret_cast<f32x4*>(rp) = acc[0];
        *reinterpret_cast<f32x4*>(rp + 256) = acc[1];
        acc[0] = acc[1] = (f32x4){0.f, 0.f, 0.f, 0.f};
        par ^= 1;
        __syncthreads();
      }
    };

    // segments of GEMV jobs between this block's attention stages: the ping-pong weight
    // registers live only inside a segment, so the attention body gets the register file
    Job j0;
    first_job(0, 0, j0);
    while (j0.valid) {
      if (j0.att) {
        att_stage(j0.l);
        Job t;
        next_job(j0, t);
        j0 = t;
        continue;
      }
      u32x4 wa[WS], wb[WS];
      Job j1;
      issue(wa, j0);
      for (;;) {
        next_job(j0, j1);
        const bool g1 = j1.valid && !j1.att;
        if (g1) issue(wb, j1);  // the next batch goes out before this one is consumed
        process(wa, j0);
        if (!g1) {
          j0 = j1;
          break;
        }
        next_job(j1, j0);
        const bool g0 = j0.valid && !j0.att;
        if (g0) issue(wa, j0);
        process(wb, j1);
        if (!g0) break;
      }
    }
  }

  // ---- exit: the last workgroup out resets the counters for the next launch (after every
  // wave of this one, the control wave's last counter add included, is done) ----
  __syncthreads();
  if (threadIdx.x == 0) {
    const uint32_t t = __hip_atomic_fetch_add((g32*)(a.sync + a.w_err - 1), 1u, __ATOMIC_RELAXED,
                                              __HIP_MEMORY_SCOPE_AGENT);
    if (t == (uint32_t)P - 1) {
      for (int i = 0; i < a.w_err; ++i) st32(a.sync + i, 0u);
    }
  }
}

// ---------------------------------------------------------------------------
size_t mega_lds_bytes(int B, int H, int HqD, int I) {
  return (size_t)2 * NW * 2 * 256 * 4 + (size_t)B * H * 2 + (size_t)B * std::max(HqD, I) * 2;
}

int mega_err_word(int layers, int Hkv) { return layers * NST + layers * MEGA_MAXB * Hkv + 1; }
int mega_sync_words(int layers, int Hkv) { return ((mega_err_word(layers, Hkv) + 1 + 3) / 4) * 4; }

template <int G, int D>
static hipError_t launch_gd(const MegaArgs& a, int P, size_t lds, hipStream_t s) {
  static size_t attr = 0;  // dynamic LDS the kernel is currently allowed
  if (lds > attr) {
    hipError_t e = hipFuncSetAttribute((const void*)mega_decode_kernel<G, D>,
                                       hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    if (e != hipSuccess) return e;
    attr = lds;
  }
  hipLaunchKernelGGL((mega_decode_kernel<G, D>), dim3(P), dim3(THREADS), lds, s, a);
  return hipGetLastError();
}

hipError_t mega_decode(const MegaArgs& a0, int P, hipStream_t s) {
  MegaArgs a = a0;
  const int G = a.Hq / a.Hkv;
  if (a.Hq % a.Hkv || a.B < 1 || a.B > MEGA_MAXB || a.D != 128 || a.H % 32 || a.I % 32 || a.H < 32 * NW || a.H > 8192 ||
      a.qkv_rows % 32 || a.Cmax % 64)
    return hipErrorInvalidValue;
  a.ns = (a.Cmax + AKB - 1) / AKB;
  if (a.ns > DEC_MAXS) return hipErrorInvalidValue;
  const size_t lds = mega_lds_bytes(a.B, a.H, a.Hq * a.D, a.I);
  a.lds_x1 = 2 * NW * 2 * 256 * 4;
  a.lds_x2 = a.lds_x1 + a.B * a.H * 2;
  if (lds + 48 * 1024 > MEGA_LDS_LIMIT) return hipErrorInvalidValue;
  switch (G) {
    case 1: return launch_gd<1, 128>(a, P, lds, s);
    case 2: return launch_gd<2, 128>(a, P, lds, s);
    case 4: return launch_gd<4, 128>(a, P, lds, s);
    case 8: return launch_gd<8, 128>(a, P, lds, s);
    default: return hipErrorInvalidValue;
  }
}

// workgroups of one launch: one per CU, all resident (the dynamic LDS request keeps it at
// one per CU; the occupancy query must agree)
int mega_grid(int device, size_t lds) {
  hipDeviceProp_t p;
  if (hipGetDeviceProperties(&p, device) != hipSuccess) return 0;
  int per_cu = 0;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, (const void*)mega_decode_kernel<4, 128>, THREADS, lds) !=
      hipSuccess)
    return 0;
  if (per_cu < 1) return 0;
  return p.multiProcessorCount;
}

}  // namespace mtts
