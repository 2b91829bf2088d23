// Weight-streaming skinny GEMM ("GEMV") for the decode step: y[B,N] = x[B,K] . W[N,K]^T
//
// Replaces the bf16 nn.Linear calls of the Qwen3 backbone
// (TF/models/qwen3/modeling_qwen3.py:241-280 q/k/v/o_proj, :81-83 gate/up/down_proj)
// and the 1+n_vq heads (moss_tts_delay/modeling_moss_tts.py:292-300).
//
// HBM layout ("MFMA-tile packed"): W is stored as 1 KiB tiles of 16 rows x 32 k, in
// exactly the A-operand order of v_mfma_f32_16x16x32_bf16 (lane l holds row l&15,
// k = 8*(l>>4) .. +7), tiles ordered [row_tile][k_tile].  A wave's stream over its
// K range is therefore one contiguous run of 1 KiB wave-loads (16 B/lane, fully
// coalesced), each feeding one MFMA with no LDS round trip.
//
// Work split: one 256-thread block per 16-row output tile (RT=2: a gate tile and an
// up tile that share x fragments), the 4 waves split K, partial tiles are reduced
// through LDS in a fixed order (deterministic), and the epilogue fuses the op that
// follows the matmul in the reference (residual add, SwiGLU, audio pad-column mask).
#include "kernels.h"

namespace mtts {



template <int NB, int RT, int EPI>
__global__ __launch_bounds__(256) void gemv_kernel(GemvArgs a) {
  constexpr int U = 8;  // k-tiles in flight per wave
  const int lane = threadIdx.x & 63;
  const int wave = threadIdx.x >> 6;
  const int bt = blockIdx.x;  // output row tile
  const int KT = a.KT;
  const int per = (KT + 3) >> 2;
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

  int kt = kt0;
  for (; kt + U <= kt1; kt += U) {
    u32x4 wa[RT][U];
    u32x4 xb[NB][U];
#pragma unroll
    for (int u = 0; u < U; ++u)
#pragma unroll
      for (int r = 0; r < RT; ++r) wa[r][u] = __builtin_nontemporal_load(wbase[r] + (size_t)(kt + u) * 64);
#pragma unroll
    for (int u = 0; u < U; ++u)
#pragma unroll
      for (int nb = 0; nb < NB; ++nb)
        xb[nb][u] = xok[nb] ? xbase[nb][(kt + u) * 4] : (u32x4){0u, 0u, 0u, 0u};
#pragma unroll
    for (int u = 0; u < U; ++u)
#pragma unroll
      for (int r = 0; r < RT; ++r)
#pragma unroll
        for (int nb = 0; nb < NB; ++nb)
          acc[r][nb] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(
              __builtin_bit_cast(bf16x8, wa[r][u]), __builtin_bit_cast(bf16x8, xb[nb][u]), acc[r][nb], 0, 0, 0);
  }
  for (; kt < kt1; ++kt) {
#pragma unroll
    for (int r = 0; r < RT; ++r) {
      u32x4 wv = __builtin_nontemporal_load(wbase[r] + (size_t)kt * 64);
#pragma unroll
      for (int nb = 0; nb < NB; ++nb) {
        u32x4 xv = xok[nb] ? xbase[nb][kt * 4] : (u32x4){0u, 0u, 0u, 0u};
        acc[r][nb] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(
            __builtin_bit_cast(bf16x8, wv), __builtin_bit_cast(bf16x8, xv), acc[r][nb], 0, 0, 0);
      }
    }
  }

  // ---- fixed-order reduction of the 4 waves' partial tiles through LDS ----
  __shared__ float red[4][RT][NB][256];
#pragma unroll
  for (int r = 0; r < RT; ++r)
#pragma unroll
    for (int nb = 0; nb < NB; ++nb)
#pragma unroll
      for (int i = 0; i < 4; ++i) red[wave][r][nb][lane * 4 + i] = acc[r][nb][i];
  __syncthreads();

  const int t = threadIdx.x;
  // element t: lane = t/4, reg = t%4 -> n = ((lane>>4)*4 + reg), b = lane & 15
  const int ln = t >> 2;
  const int nl = ((ln >> 4) << 2) + (t & 3);
  const int n = bt * 16 + nl;
#pragma unroll
  for (int nb = 0; nb < NB; ++nb) {
    const int b = (ln & 15) + 16 * nb;
    float v[RT];
#pragma unroll
    for (int r = 0; r < RT; ++r)
      v[r] = ((red[0][r][nb][t] + red[1][r][nb][t]) + red[2][r][nb][t]) + red[3][r][nb][t];
    if (b >= a.B || n >= a.N) continue;
    bf16_t out;
    if constexpr (EPI == EPI_STORE) {
      out = f2bf(v[0]);
    } else if constexpr (EPI == EPI_LOGITS) {
      out = f2bf(v[0]);
      if (n >= a.pad_start && ((n - a.pad_start) % a.pad_period) == a.pad_off) out = 0xFF80;  // -inf
    } else if constexpr (EPI == EPI_RESADD) {
      // hidden = residual + bf16(o)   (TF/.../modeling_qwen3.py:311,322)
      out = f2bf(bf2f(a.res[(size_t)b * a.ldres + n]) + rbf(v[0]));
    } else {  // EPI_SWIGLU: bf16(bf16(silu(bf16 g)) * bf16 u)   (TF/.../modeling_qwen3.py:81-83)
      const float g = rbf(v[0]);
      const float u = rbf(v[RT - 1]);
      const float s = rbf(g / (1.0f + expf(-g)));
      out = f2bf(s * u);
    }
    a.y[(size_t)b * a.ldy + n] = out;
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

}  // namespace mtts

// ---------------------------------------------------------------------------
// launch helpers (used by the engine and by the kernel-level C-ABI)
namespace mtts {

template <int NB, int RT, int EPI>
static void launch_gemv_t(const GemvArgs& a, int n_tiles, hipStream_t s) {
  hipLaunchKernelGGL((gemv_kernel<NB, RT, EPI>), dim3(n_tiles), dim3(256), 0, s, a);
}

// y = epi(x . W^T) for B rows; chunks of 32 rows (weights re-streamed per chunk)
hipError_t gemv(const bf16_t* wpacked, const bf16_t* x, int ldx, bf16_t* y, int ldy, const bf16_t* res, int ldres,
                int B, int N, int K, int epi, int pad_start, int pad_period, int pad_off, hipStream_t s) {
  if (K % 32 != 0 || B <= 0 || N <= 0) return hipErrorInvalidValue;
  for (int b0 = 0; b0 < B; b0 += 32) {
    GemvArgs a;
    a.w = wpacked;
    a.x = x + (size_t)b0 * ldx;
    a.y = y + (size_t)b0 * ldy;
    a.res = res ? res + (size_t)b0 * ldres : nullptr;
    a.ldx = ldx; a.ldy = ldy; a.ldres = ldres;
    a.B = min(32, B - b0);
    a.N = N; a.K = K; a.KT = K / 32;
    a.pad_start = pad_start; a.pad_period = pad_period > 0 ? pad_period : 1; a.pad_off = pad_off;
    const int n_tiles = (N + 15) / 16;
    const bool two = a.B > 16;
    switch (epi) {
      case EPI_STORE:  two ? launch_gemv_t<2, 1, EPI_STORE>(a, n_tiles, s) : launch_gemv_t<1, 1, EPI_STORE>(a, n_tiles, s); break;
      case EPI_LOGITS: two ? launch_gemv_t<2, 1, EPI_LOGITS>(a, n_tiles, s) : launch_gemv_t<1, 1, EPI_LOGITS>(a, n_tiles, s); break;
      case EPI_RESADD: two ? launch_gemv_t<2, 1, EPI_RESADD>(a, n_tiles, s) : launch_gemv_t<1, 1, EPI_RESADD>(a, n_tiles, s); break;
      case EPI_SWIGLU: two ? launch_gemv_t<2, 2, EPI_SWIGLU>(a, n_tiles, s) : launch_gemv_t<1, 2, EPI_SWIGLU>(a, n_tiles, s); break;
      default: return hipErrorInvalidValue;
    }
  }
  return hipGetLastError();
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
