// Split-K decode GEMV with the residual epilogue, for projections with too few 16-row output
// tiles to fill the chip: y[B,N] = res + bf16(x[B,K] . W[N,K]^T), plus the per-16-column sums of
// squares of y (the EPI_RESADD epilogue of gemv_body.h; TF/models/qwen3/modeling_qwen3.py:
// 311, 322 residual adds after o_proj / down_proj).
//
// Why: the one-block-per-tile GEMV runs MossTTSLocal's depth-transformer down projection
// (N 1,536 = 96 tiles, K 8,960) on 96 of the 256 CUs, each wave walking 3 dependent 8-tile
// batches -- 15.3 us for 27.5 MB, 1.8 TB/s.  Here workgroup (tile, split) handles K/S of the
// tile (S chosen so that tiles x S >= the CU count and each wave issues one batch), its NW
// waves reduce through LDS in a fixed order, and the fp32 tile partial is published
// (write-through stores, drained, arrival ticket per tile).  The last of the S arrivals sums
// the S partials in split order (deterministic), adds the residual and writes y and the sums
// of squares, then resets its ticket for the next launch (graph replay).
// Layout: the packed weight tiles of gemv.hip ([row tile][k tile], 1 KiB each); x rows from L2.
#include <algorithm>
#include <cstdlib>

#include "kernels.h"

namespace mtts {

namespace {
constexpr int SK_NW = 8;  // waves per workgroup
constexpr int SK_U = 8;   // k-tiles per load batch
constexpr int SK_MAXS = 16;  // most K splits (the last arrival keeps all partial loads in flight)
constexpr int SK_MAXS2 = 8;  // ... of the 17-32 row form
typedef __attribute__((address_space(1))) float gf32;
}  // namespace

__global__ __launch_bounds__(SK_NW * 64) void gemv_splitk_kernel(GemvArgs a, int S, float* part, int* cnt) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, t = threadIdx.x;
  const int bt = blockIdx.x / S, si = blockIdx.x - bt * S;
  const int KT = a.KT;
  const int KS = (KT + S - 1) / S;
  const int k0 = si * KS, k1 = min(KT, k0 + KS);
  const int per = (k1 - k0 + SK_NW - 1) / SK_NW;
  const int kw0 = k0 + wave * per, kw1 = min(k1, kw0 + per);

  const u32x4* wbase = reinterpret_cast<const u32x4*>(a.w) + ((size_t)bt * KT) * 64 + lane;
  const int b = lane & 15;
  const bool xok = b < a.B;
  const u32x4* xbase = reinterpret_cast<const u32x4*>(a.x + (size_t)(xok ? b : 0) * a.ldx + (lane >> 4) * 8);
  // the residual element this thread adds if its workgroup arrives last, loaded before the
  // weights (in the last arrival's epilogue it was one more dependent round trip)
  const int ln = t >> 2, nl = ((ln >> 4) << 2) + (t & 3), bl = ln & 15;
  const int n = bt * 16 + nl;
  const bool rok = t < 256 && bl < a.B && n < a.N;
  const __amdgpu_buffer_rsrc_t rrs = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<bf16_t*>(a.res), 0, (int)(((size_t)(a.B - 1) * a.ldres + a.N) * 2), 0x00020000);
  const uint16_t resv = __builtin_amdgcn_raw_buffer_load_b16(rrs, rok ? (uint32_t)(bl * a.ldres + n) * 2u : 0x7ffffff0u, 0, 0);
  __builtin_amdgcn_sched_barrier(0);
  f32x4 acc = (f32x4){0.f, 0.f, 0.f, 0.f};
  for (int k = kw0; k < kw1; k += SK_U) {
    u32x4 wv[SK_U], xv[SK_U];
    // a batch is always SK_U loads: the surplus re-reads the wave's last tile (zero A operand)
#pragma unroll
    for (int u = 0; u < SK_U; ++u) wv[u] = __builtin_nontemporal_load(wbase + (size_t)min(k + u, kw1 - 1) * 64);
#pragma unroll
    for (int u = 0; u < SK_U; ++u) xv[u] = xbase[(size_t)min(k + u, kw1 - 1) * 4];
#pragma unroll
    for (int u = 0; u < SK_U; ++u) {
      const u32x4 w = k + u < kw1 ? wv[u] : (u32x4){0u, 0u, 0u, 0u};
      acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, w), __builtin_bit_cast(bf16x8, xv[u]),
                                                    acc, 0, 0, 0);
    }
  }
  // ---- fixed-order reduction of the waves' partial tiles; the tile partial goes out sc1 ----
  __shared__ float red[SK_NW][256];
  __shared__ float sq[16][17];
  __shared__ int last_s;
#pragma unroll
  for (int i = 0; i < 4; ++i) red[wave][lane * 4 + i] = acc[i];
  __syncthreads();
  float* pt = part + (size_t)blockIdx.x * 256;  // [tile][split][256]: element t = (row, b) as the MFMA lays it out
  if (t < 256) {
    float s = 0.f;
#pragma unroll
    for (int w = 0; w < SK_NW; ++w) s += red[w][t];
    __hip_atomic_store((gf32*)(pt + t), s, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (t == 0) last_s = __hip_atomic_fetch_add(cnt + bt, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == S - 1;
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
  // ---- the last arrival: sum the S partials in split order, + residual, sums of squares ----
  if (t < 256) {
    // element t: lane = t/4, reg = t%4 -> row n = ((lane>>4)*4 + reg), b = lane & 15
    // sc1 (device-scope) buffer loads (aux 16), all S in flight (atomic loads went one at a time)
    const __amdgpu_buffer_rsrc_t prs =
        __builtin_amdgcn_make_buffer_rsrc(part + (size_t)bt * S * 256, 0, S * 256 * 4, 0x00020000);
    float pv[SK_MAXS];
#pragma unroll
    for (int j = 0; j < SK_MAXS; ++j)
      pv[j] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(
          prs, j < S ? (uint32_t)(j * 256 + t) * 4u : 0x7ffffff0u, 0, 16));
    float s = 0.f;
#pragma unroll
    for (int j = 0; j < SK_MAXS; ++j)
      if (j < S) s += pv[j];
    bf16_t out = 0;
    if (rok) {
      // hidden = residual + bf16(o)   (TF/.../modeling_qwen3.py:311,322)
      out = f2bf(bf2f(resv) + rbf(s));
      a.y[(size_t)bl * a.ldy + n] = out;
    }
    const float ho = bf2f(out);
    sq[bl][nl] = ho * ho;
  }
  __syncthreads();
  if (a.ss_out && t < 16 && t < a.B) {
    float s = 0.f;
#pragma unroll
    for (int i = 0; i < 16; ++i) s += sq[t][i];
    a.ss_out[(size_t)t * a.ld_ss_out + bt] = s;
  }
  if (t == 0) cnt[bt] = 0;
}

// ---------------------------------------------------------------------------
// 17-32 packed rows (the B = 32 decode step's o_proj / down_proj): RT row tiles per workgroup
// share each x fragment (at 32 rows a k tile's two x fragments are as many bytes as RT = 2
// weight tiles, so the one-tile GEMV reads x from L2 twice per weight byte), and K is split S
// ways so that n_tiles / RT x S workgroups still cover the CUs.  Same publish / ticket / last-
// arrival combine as above, per group of RT tiles; the epilogue writes row-major rows + sums of
// squares like EPI_RESADD.
template <int RT>
__global__ __launch_bounds__(SK_NW * 64) void gemv_splitk2_kernel(GemvArgs a, int S, float* part, int* cnt) {
  constexpr int NB = 2, U = 8;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, t = threadIdx.x;
  const int grp = blockIdx.x / S, si = blockIdx.x - grp * S;
  const int KT = a.KT;
  const int KS = KT / S;  // KT % (S * SK_NW) == 0 (checked by the launcher)
  const int per = KS / SK_NW;
  const int kw0 = si * KS + wave * per, kw1 = kw0 + per;
  const u32x4* wbase[RT];
#pragma unroll
  for (int r = 0; r < RT; ++r) wbase[r] = reinterpret_cast<const u32x4*>(a.w) + ((size_t)(grp * RT + r) * KT) * 64 + lane;
  // packed x: k tile kt of half nb is 1 KiB at (2 kt + nb) KiB
  const u32x4* xbase = reinterpret_cast<const u32x4*>(a.x) + lane;
  // residual elements this thread adds if its workgroup arrives last (before the weights)
  const int ln = t >> 2, nl = ((ln >> 4) << 2) + (t & 3), bl = ln & 15;
  uint16_t resv[RT][NB];
  {
    const __amdgpu_buffer_rsrc_t rrs = __builtin_amdgcn_make_buffer_rsrc(
        const_cast<bf16_t*>(a.res), 0, (int)(((size_t)(a.B - 1) * a.ldres + a.N) * 2), 0x00020000);
#pragma unroll
    for (int r = 0; r < RT; ++r)
#pragma unroll
      for (int nb = 0; nb < NB; ++nb) {
        const int n = (grp * RT + r) * 16 + nl, b = bl + 16 * nb;
        const bool ok = t < 256 && b < a.B && n < a.N;
        resv[r][nb] = __builtin_amdgcn_raw_buffer_load_b16(rrs, ok ? (uint32_t)(b * a.ldres + n) * 2u : 0x7ffffff0u, 0, 0);
      }
  }
  __builtin_amdgcn_sched_barrier(0);
  f32x4 acc[RT][NB];
#pragma unroll
  for (int r = 0; r < RT; ++r)
#pragma unroll
    for (int nb = 0; nb < NB; ++nb) acc[r][nb] = (f32x4){0.f, 0.f, 0.f, 0.f};
  for (int k = kw0; k < kw1; k += U) {
    u32x4 wv[RT][U], xv[NB][U];
#pragma unroll
    for (int u = 0; u < U; ++u)
#pragma unroll
      for (int r = 0; r < RT; ++r) wv[r][u] = __builtin_nontemporal_load(wbase[r] + (size_t)min(k + u, kw1 - 1) * 64);
#pragma unroll
    for (int u = 0; u < U; ++u)
#pragma unroll
      for (int nb = 0; nb < NB; ++nb) xv[nb][u] = xbase[(size_t)min(k + u, kw1 - 1) * 128 + nb * 64];
#pragma unroll
    for (int u = 0; u < U; ++u)
#pragma unroll
      for (int r = 0; r < RT; ++r) {
        const u32x4 w = k + u < kw1 ? wv[r][u] : (u32x4){0u, 0u, 0u, 0u};
#pragma unroll
        for (int nb = 0; nb < NB; ++nb)
          acc[r][nb] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, w),
                                                               __builtin_bit_cast(bf16x8, xv[nb][u]), acc[r][nb], 0, 0, 0);
      }
  }
  // fixed-order reduction of the waves' tiles; the group partial [RT][NB][256] goes out sc1
  __shared__ float red[SK_NW][RT * NB][256];
  __shared__ float sq[RT][NB][16][17];
  __shared__ int last_s;
#pragma unroll
  for (int r = 0; r < RT; ++r)
#pragma unroll
    for (int nb = 0; nb < NB; ++nb)
#pragma unroll
      for (int i = 0; i < 4; ++i) red[wave][r * NB + nb][lane * 4 + i] = acc[r][nb][i];
  __syncthreads();
  float* pt = part + (size_t)blockIdx.x * (RT * NB * 256);  // [grp][split][RT][NB][256]
  for (int e = t; e < RT * NB * 256; e += SK_NW * 64) {
    float v = 0.f;
#pragma unroll
    for (int w = 0; w < SK_NW; ++w) v += red[w][e >> 8][e & 255];
    __hip_atomic_store((gf32*)(pt + e), v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (t == 0) last_s = __hip_atomic_fetch_add(cnt + grp, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == S - 1;
  __syncthreads();
  if (!last_s) return;
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");  // (the hand-off form of gemv_splitk_kernel)
  if (t < 256) {
    const __amdgpu_buffer_rsrc_t prs = __builtin_amdgcn_make_buffer_rsrc(
        part + (size_t)grp * S * (RT * NB * 256), 0, S * RT * NB * 256 * 4, 0x00020000);
#pragma unroll
    for (int r = 0; r < RT; ++r)
#pragma unroll
      for (int nb = 0; nb < NB; ++nb) {
        float pv[SK_MAXS2];
#pragma unroll
        for (int j = 0; j < SK_MAXS2; ++j)
          pv[j] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(
              prs, j < S ? (uint32_t)((j * RT * NB + r * NB + nb) * 256 + t) * 4u : 0x7ffffff0u, 0, 16));
        float v = 0.f;
#pragma unroll
        for (int j = 0; j < SK_MAXS2; ++j)
          if (j < S) v += pv[j];
        const int n = (grp * RT + r) * 16 + nl, b = bl + 16 * nb;
        bf16_t out = 0;
        if (b < a.B && n < a.N) {
          // hidden = residual + bf16(o)   (TF/.../modeling_qwen3.py:311,322)
          out = f2bf(bf2f(resv[r][nb]) + rbf(v));
          a.y[(size_t)b * a.ldy + n] = out;
        }
        const float ho = bf2f(out);
        sq[r][nb][bl][nl] = ho * ho;
      }
  }
  __syncthreads();
  if (a.ss_out && t < RT * NB * 16) {
    const int r = t / (NB * 16), nb = (t >> 4) % NB, b = (t & 15) + 16 * nb;
    if (b < a.B) {
      float v = 0.f;
#pragma unroll
      for (int i = 0; i < 16; ++i) v += sq[r][nb][t & 15][i];
      a.ss_out[(size_t)b * a.ld_ss_out + grp * RT + r] = v;
    }
  }
  if (t == 0) cnt[grp] = 0;
}

bool gemv_splitk2_pick(int n_tiles, int KT, int B, int* RT, int* S) {
  // MTTS_SK2 = "RT,S" (RT 2 or 4); off by default: B = 32 decode step 4.41 (off) / 4.40 (2,2) /
  // 4.83 (4,2) / 4.87 (2,4) / 4.74 ms (4,4) -- the one-tile GEMV's x re-reads are not what
  // bounds those projections
  static int rt = -1, sp = 2;
  if (rt < 0) {
    rt = 0;
    if (const char* v = getenv("MTTS_SK2")) sscanf(v, "%d,%d", &rt, &sp);
  }
  if (rt != 2 && rt != 4) return false;
  if (B <= 16 || B > 32 || n_tiles % rt || KT % (sp * SK_NW) || (KT / sp / SK_NW) < 4 || sp < 2 || sp > SK_MAXS2) return false;
  *RT = rt;
  *S = sp;
  return true;
}

size_t gemv_splitk2_ws_floats(int n_tiles, int S) { return (size_t)n_tiles * S * 2 * 256; }

hipError_t gemv_splitk2(const GemvArgs& a0, int RT, int S, float* part, int* cnt, hipStream_t s) {
  GemvArgs a = a0;
  if (a.K % 32 || a.B <= 16 || a.B > 32 || !a.x_packed || a.N % (16 * RT) || S < 2 || S > SK_MAXS2 || !part || !cnt ||
      !a.res || a.ss_in || a.attn.part || a.tile0 || a.gate || (a.K / 32) % (S * SK_NW))
    return hipErrorInvalidValue;
  a.KT = a.K / 32;
  const int groups = a.N / 16 / RT;
  if (RT == 2) hipLaunchKernelGGL(gemv_splitk2_kernel<2>, dim3(groups * S), dim3(SK_NW * 64), 0, s, a, S, part, cnt);
  else if (RT == 4) hipLaunchKernelGGL(gemv_splitk2_kernel<4>, dim3(groups * S), dim3(SK_NW * 64), 0, s, a, S, part, cnt);
  else return hipErrorInvalidValue;
  return hipGetLastError();
}

int gemv_splitk_splits(int n_tiles, int KT, int B) {
  // worth it when the tiles alone leave most CUs idle and K is long enough to split
  if (B > 16 || n_tiles >= 160 || KT < 128) return 1;
  static const int force = getenv("MTTS_SPLITK_S") ? atoi(getenv("MTTS_SPLITK_S")) : 0;  // A/B sweeps
  if (force >= 2) return std::min(force, SK_MAXS);
  // at least one workgroup per CU and one load batch per wave, but a single round of at most
  // two workgroups per CU (MossTTSLocal down_proj, 96 tiles x K 8,960, frame ms by S:
  // 1: 11.21, 3: 10.86, 5: 10.45, 6: 11.02, 8: 11.49 -- 576+ workgroups need a second round)
  int S = std::max((256 + n_tiles - 1) / n_tiles, (KT + SK_NW * SK_U - 1) / (SK_NW * SK_U));
  while (S > 2 && n_tiles * S > 512) --S;
  while (S > 1 && KT / S < 4 * SK_NW) --S;  // >= 4 k-tiles per wave
  return std::min(S, SK_MAXS);
}

size_t gemv_splitk_ws_floats(int n_tiles, int S) { return (size_t)n_tiles * S * 256; }

hipError_t gemv_splitk(const GemvArgs& a0, int S, float* part, int* cnt, hipStream_t s) {
  GemvArgs a = a0;
  if (a.K % 32 || a.B <= 0 || a.B > 16 || a.N <= 0 || S < 2 || S > SK_MAXS || !part || !cnt || !a.res || a.ss_in || a.attn.part ||
      a.tile0 || a.gate)
    return hipErrorInvalidValue;
  a.KT = a.K / 32;
  const int n_tiles = (a.N + 15) / 16;
  hipLaunchKernelGGL(gemv_splitk_kernel, dim3(n_tiles * S), dim3(SK_NW * 64), 0, s, a, S, part, cnt);
  return hipGetLastError();
}

}  // namespace mtts
