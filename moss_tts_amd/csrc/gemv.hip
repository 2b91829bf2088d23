// Weight-streaming skinny GEMM ("GEMV") for the decode step: y[B,N] = x[B,K] . W[N,K]^T
//
// Replaces the bf16 nn.Linear calls of the Qwen3 backbone
// (TF/models/qwen3/modeling_qwen3.py:241-280 q/k/v/o_proj, :81-83 gate/up/down_proj)
// and the 1+n_vq heads (moss_tts_delay/modeling_moss_tts.py:292-300).
//
// HBM layout ("MFMA-tile packed"): W is stored as 1 KiB tiles of 16 rows x 32 k, in
// exactly the A-operand order of v_mfma_f32_16x16x32_bf16 (lane l holds row l&15,
// k = 8*(l>>4) .. +7), tiles ordered [row_tile][k_tile].  A wave's stream over its
// K range is one contiguous run of 1 KiB wave-loads (16 B/lane, fully coalesced,
// non-temporal: each weight byte is read once per step), each feeding one MFMA with
// no LDS round trip.  x (the B activation rows) is the MFMA B operand, read from L2.
//
// Work split: one block of NW waves per 16-row output tile (RT=2: a gate tile and an
// up tile that share x fragments); the NW waves split K and their partial tiles are
// reduced through LDS in a fixed order (deterministic).  NW is picked per matrix so
// that every CU holds enough waves (bytes in flight) even for 4096-row matrices.
//
// Fusions: for small decode batches (B <= 4 at K = 4096) the RMSNorm that precedes q|k|v
// and gate|up runs in the prologue: the block stages the normalised rows in LDS once, from
// the per-16-column sums of squares its producer wrote, while its first weight batch is
// already in flight.  The op that follows the matmul runs in the epilogue (residual add +
// its sums of squares, SwiGLU, the audio-head pad column mask).
#include <algorithm>
#include <cstdlib>

#include "kernels.h"

namespace mtts {

size_t norm_lds_bytes(int B, int K) { return (size_t)(B + 1) * K * 2; }

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

template <int NB, int RT, int EPI, int PRO, int NW, bool PIPE = false>
__global__ __launch_bounds__(NW * 64) void gemv_kernel(GemvArgs a) {
  // k-tiles per load batch (one batch in flight per wave); the 4-deep variant (PIPE) trades
  // bytes in flight per wave for more resident waves (the default for 17-32 rows)
  constexpr int U = PIPE ? 4 : 8;
  const int lane = threadIdx.x & 63;
  const int wave = threadIdx.x >> 6;
  if (a.gate && *a.gate == 0) return;
  const int bt = blockIdx.x + a.tile0;  // output row tile
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
  const u32x4* xbase[NB];
  bool xok[NB];
#pragma unroll
  for (int nb = 0; nb < NB; ++nb) {
    const int b = (lane & 15) + 16 * nb;
    xok[nb] = b < a.B;
    xbase[nb] = reinterpret_cast<const u32x4*>(a.x + (size_t)(xok[nb] ? b : 0) * a.ldx + (lane >> 4) * 8);
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
        wa[r][u] = __builtin_nontemporal_load(wbase[r] + (size_t)min(k + u, kt1 - 1) * 64);
  };
  if (kt < kt1) issue_w(kt);

  // Prologues (PRO) stage the block's B activation rows in LDS once; the MFMA B fragments
  // are then LDS reads.  PRO_NONE reads the fragments straight from x (L2).
  //   PRO_NORM:  bf16(nw * bf16(x * r_b)), r_b from the producer's per-16-column sums of
  //              squares (Qwen3RMSNorm, TF/models/qwen3/modeling_qwen3.py:59-64)
  //   PRO_ATTN:  the decode attention output, merged here from its per-split (m, l, o)
  //              partials in split order: x = bf16(sum_s f_s o_s / sum_s f_s l_s),
  //              f_s = exp(m_s - max m) -- the cross-block combine of attn_decode
  extern __shared__ u32x4 xs_dyn[];
  const int K8 = KT * 4;  // 16-byte chunks per row
  if constexpr (PRO == PRO_NORM) {
    __shared__ float r_s[32];
    const int n8x = a.B * K8;
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
    __syncthreads();
    for (int i = threadIdx.x; i < n8x; i += NW * 64) {
      const int b = i / K8;
      xs_dyn[i] = norm8(xs_dyn[i], xs_dyn[n8x + i - b * K8], r_s[b]);
    }
    __syncthreads();
  } else if constexpr (PRO == PRO_ATTN) {
    const AttnPartView& v = a.attn;
    const int nact = *v.pos / v.kb + 1;
    const int G = v.G, D = v.D, PS = G * (D + 2);
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
    if (!xok[nb]) return (u32x4){0u, 0u, 0u, 0u};
    if constexpr (PRO != PRO_NONE) return xs_dyn[((lane & 15) + 16 * nb) * K8 + k * 4 + (lane >> 4)];
    return xbase[nb][k * 4];
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
  __shared__ float red[NW][RT][NB][256];
  __shared__ float sq[NB][16][17];
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
    const int n = bt * 16 + nl;
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
      bf16_t out = 0;
      if constexpr (EPI == EPI_STORE) {
        out = f2bf(v[0]);
      } else if constexpr (EPI == EPI_LOGITS) {
        out = f2bf(v[0]);
        if (n >= a.pad_start && ((n - a.pad_start) % a.pad_period) == a.pad_off) out = 0xFF80;  // -inf
      } else if constexpr (EPI == EPI_RESADD) {
        // hidden = residual + bf16(o)   (TF/.../modeling_qwen3.py:311,322)
        if (b < a.B && n < a.N) out = f2bf(bf2f(a.res[(size_t)b * a.ldres + n]) + rbf(v[0]));
        const float ho = bf2f(out);
        sq[nb][bl][nl] = ho * ho;
      } else {  // EPI_SWIGLU: bf16(bf16(silu(bf16 g)) * bf16 u)   (TF/.../modeling_qwen3.py:81-83)
        const float g = rbf(v[0]);
        const float u = rbf(v[RT - 1]);
        const float s = rbf(g / (1.0f + expf(-g)));
        out = f2bf(s * u);
      }
      if (b < a.B && n < a.N) a.y[(size_t)b * a.ldy + n] = out;
    }
  }
  if constexpr (EPI == EPI_RESADD) {
    __syncthreads();
    if (a.ss_out && t < 16 * NB) {
      const int nb = t >> 4, bl = t & 15, b = bl + 16 * nb;
      if (b < a.B) {
        float s = 0.f;
#pragma unroll
        for (int i = 0; i < 16; ++i) s += sq[nb][bl][i];
        a.ss_out[(size_t)b * a.ld_ss_out + bt] = s;
      }
    }
  }
}

// ---------------------------------------------------------------------------
// packing: src [rows, K] row-major bf16 -> packed tiles.
//   dst_row = row_offset + r                             (interleave == 0)
//   dst_row = (r/16)*32 + (r%16) + 16*which              (interleave == 1: gate/up pairs)
__global__ void pack_kernel(const bf16_t* __restrict__ src, bf16_t* __restrict__ dst, int rows, int K,
                            int row_offset, int interleave, int which) {
  const int KC = K >> 3;  // 8-element chunks per row
  const size_t total = (size_t)rows * KC;
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < total; i += (size_t)gridDim.x * blockDim.x) {
    const int r = (int)(i / KC);
    const int c = (int)(i % KC);
    const int k = c * 8;
    const int dr = interleave ? ((r >> 4) * 32 + (r & 15) + 16 * which) : (row_offset + r);
    const int nt = dr >> 4, rr = dr & 15;
    const int kt = k >> 5, g = (k & 31) >> 3;
    const int ln = g * 16 + rr;
    const size_t off = (((size_t)nt * (K >> 5) + kt) * 64 + ln) * 8;
    *reinterpret_cast<uint4*>(dst + off) = *reinterpret_cast<const uint4*>(src + (size_t)r * K + k);
  }
}

// ---------------------------------------------------------------------------
template <int NB, int RT, int EPI, int PRO>
static void launch_nw(const GemvArgs& a, int n_tiles, hipStream_t s) {
  constexpr bool NORM = PRO == PRO_NORM;
  // waves per block from the B=1/B=4 sweep (scripts/sweep_gemv.py, profiles/): 8 for the
  // large matrices (gate|up 6.1 TB/s, heads 7.0 TB/s), 16 for the <= 6144-row ones
  const int rows = n_tiles * RT * 16;
  const size_t lds = PRO == PRO_NORM ? norm_lds_bytes(a.B, a.K) : (PRO == PRO_ATTN ? (size_t)a.B * a.K * 2 : 0);
  // 17-32 rows (NB = 2): 4 waves of 4-deep batches (in-context B=32 sweep: 5.62 vs 6.03 ms/step)
  int nw = a.force_nw;
  // fused-norm launches stage (B+1)*K*2 bytes of LDS per block: 8 waves keep 2 blocks per CU
  // (q|k|v: 3.46 vs 3.53 ms/step with 16)
  if (nw != 4 && nw != 8 && nw != 16)
    nw = (a.KT < 64 || NB == 2) ? 4 : ((rows >= 8192 || a.KT < 128 || NORM) ? 8 : 16);
  // MTTS_GEMV_PIPE bit 0 / bit 1 flips the batch depth (8 <-> 4 k-tiles) for <= 16 / > 16 rows
  static const int pipe = getenv("MTTS_GEMV_PIPE") ? atoi(getenv("MTTS_GEMV_PIPE")) : 0;
  if ((NB == 1 && (pipe & 1)) || (NB == 2 && !(pipe & 2))) {
    if (nw == 4) hipLaunchKernelGGL((gemv_kernel<NB, RT, EPI, PRO, 4, true>), dim3(n_tiles), dim3(256), lds, s, a);
    if (nw == 8) hipLaunchKernelGGL((gemv_kernel<NB, RT, EPI, PRO, 8, true>), dim3(n_tiles), dim3(512), lds, s, a);
    if (nw == 16) hipLaunchKernelGGL((gemv_kernel<NB, RT, EPI, PRO, 16, true>), dim3(n_tiles), dim3(1024), lds, s, a);
    return;
  }
  if (nw == 4) hipLaunchKernelGGL((gemv_kernel<NB, RT, EPI, PRO, 4>), dim3(n_tiles), dim3(256), lds, s, a);
  if (nw == 8) hipLaunchKernelGGL((gemv_kernel<NB, RT, EPI, PRO, 8>), dim3(n_tiles), dim3(512), lds, s, a);
  if (nw == 16) hipLaunchKernelGGL((gemv_kernel<NB, RT, EPI, PRO, 16>), dim3(n_tiles), dim3(1024), lds, s, a);
}

template <int RT, int EPI>
static void launch_epi(const GemvArgs& a, int n_tiles, hipStream_t s) {
  const bool two = a.B > 16;
  if constexpr (EPI == EPI_RESADD) {
    if (a.attn.part) {  // o_proj reading the attention partials (B <= 16)
      launch_nw<1, RT, EPI, PRO_ATTN>(a, n_tiles, s);
      return;
    }
  }
  const bool norm = a.ss_in != nullptr;
  if (two) norm ? launch_nw<2, RT, EPI, PRO_NORM>(a, n_tiles, s) : launch_nw<2, RT, EPI, PRO_NONE>(a, n_tiles, s);
  else norm ? launch_nw<1, RT, EPI, PRO_NORM>(a, n_tiles, s) : launch_nw<1, RT, EPI, PRO_NONE>(a, n_tiles, s);
}

hipError_t gemv_ex(const GemvArgs& a0, int epi, hipStream_t s) {
  if (a0.K % 32 != 0 || a0.B <= 0 || a0.N <= 0) return hipErrorInvalidValue;
  if (a0.ss_in && (a0.n_ss % 4 || a0.ld_ss % 4 || a0.ldx % 8 || norm_lds_bytes(std::min(a0.B, 32), a0.K) > NORM_LDS_MAX))
    return hipErrorInvalidValue;
  if (a0.attn.part && (epi != EPI_RESADD || a0.B > 16 || (size_t)a0.B * a0.K * 2 > NORM_LDS_MAX || a0.attn.D % 8 ||
                       a0.K != a0.attn.Hkv * a0.attn.G * a0.attn.D))
    return hipErrorInvalidValue;
  for (int b0 = 0; b0 < a0.B; b0 += 32) {
    GemvArgs a = a0;
    a.x = a0.x + (size_t)b0 * a0.ldx;
    a.y = a0.y + (size_t)b0 * a0.ldy;
    a.res = a0.res ? a0.res + (size_t)b0 * a0.ldres : nullptr;
    a.ss_in = a0.ss_in ? a0.ss_in + (size_t)b0 * a0.ld_ss : nullptr;
    a.ss_out = a0.ss_out ? a0.ss_out + (size_t)b0 * a0.ld_ss_out : nullptr;
    a.B = min(32, a0.B - b0);
    a.KT = a0.K / 32;
    if (a.pad_period <= 0) a.pad_period = 1;
    const int n_tiles = (a0.N + 15) / 16 - a0.tile0;
    if (n_tiles <= 0) continue;
    switch (epi) {
      case EPI_STORE: launch_epi<1, EPI_STORE>(a, n_tiles, s); break;
      case EPI_LOGITS: launch_epi<1, EPI_LOGITS>(a, n_tiles, s); break;
      case EPI_RESADD: launch_epi<1, EPI_RESADD>(a, n_tiles, s); break;
      case EPI_SWIGLU: launch_epi<2, EPI_SWIGLU>(a, n_tiles, s); break;
      default: return hipErrorInvalidValue;
    }
  }
  return hipGetLastError();
}

hipError_t gemv(const bf16_t* wpacked, const bf16_t* x, int ldx, bf16_t* y, int ldy, const bf16_t* res, int ldres,
                int B, int N, int K, int epi, int pad_start, int pad_period, int pad_off, hipStream_t s) {
  GemvArgs a = gemv_args(wpacked, x, ldx, y, ldy, B, N, K);
  a.res = res;
  a.ldres = ldres;
  a.pad_start = pad_start;
  a.pad_period = pad_period;
  a.pad_off = pad_off;
  return gemv_ex(a, epi, s);
}

hipError_t pack_weight(const bf16_t* src, bf16_t* dst, int rows, int K, int row_offset, int interleave, int which,
                       hipStream_t s) {
  if (K % 32 != 0) return hipErrorInvalidValue;
  const size_t total = (size_t)rows * (K / 8);
  const size_t nb = (total + 255) / 256;
  const int blocks = (int)(nb < 65536 ? nb : 65536);
  hipLaunchKernelGGL(pack_kernel, dim3(blocks), dim3(256), 0, s, src, dst, rows, K, row_offset, interleave, which);
  return hipGetLastError();
}

}  // namespace mtts
