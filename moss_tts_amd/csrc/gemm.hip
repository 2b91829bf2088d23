// Prefill GEMM: y[M,N] = epi(x[M,K] . W[N,K]^T) for M = rows x prompt tokens.
//
// Same weights, same MFMA-tile packed layout and same epilogues as the decode GEMV
// (gemv.hip), for the prompt's projections (TF/models/qwen3/modeling_qwen3.py:241-280
// q/k/v/o_proj, :81-83 gate/up/down_proj).  The GEMV streams every weight tile once per
// 32 tokens; here a block holds RT weight tiles (16*RT output columns) against up to
// 4 * NBW * 16 tokens, so a 181-token prompt reads each weight byte once from HBM.
//
// Block = 4 waves; wave w owns token tiles [tb0 + w*NBW, +NBW) and runs the whole K loop
// for them (no cross-wave reduction): per 32-deep k-step it loads the RT weight tiles (one
// 1 KiB wave-load each, A operands; the 4 waves of a block share them through L1/L2) and
// its NBW activation fragments (B operands), then issues RT x NBW
// v_mfma_f32_16x16x32_bf16.  The epilogue runs from registers: lane holds 4 consecutive
// output columns of one token (MFMA C layout), so stores are 8-byte row segments.
#include <algorithm>
#include <cstdlib>

#include "kernels.h"
#include "qk_item.h"

namespace mtts {

template <int RT, int NBW, int EPI>
__global__ __launch_bounds__(256) void gemm_kernel(GemvArgs a) {
  constexpr int U = 4;  // k-tiles in flight per wave
  const int lane = threadIdx.x & 63;
  const int wave = threadIdx.x >> 6;
  const int bt = blockIdx.x;                            // output tile (pair for SwiGLU)
  const int tt0 = (blockIdx.y * 4 + wave) * NBW;        // first token tile of this wave
  if (tt0 * 16 >= a.B) return;
  const int KT = a.KT;
  const int g4 = lane >> 4, c16 = lane & 15;

  f32x4 acc[RT][NBW];
#pragma unroll
  for (int r = 0; r < RT; ++r)
#pragma unroll
    for (int j = 0; j < NBW; ++j) acc[r][j] = (f32x4){0.f, 0.f, 0.f, 0.f};

  const u32x4* wbase[RT];
#pragma unroll
  for (int r = 0; r < RT; ++r)
    wbase[r] = reinterpret_cast<const u32x4*>(a.w) + ((size_t)(bt * RT + r) * KT) * 64 + lane;
  const u32x4* xbase[NBW];
  bool xok[NBW];
#pragma unroll
  for (int j = 0; j < NBW; ++j) {
    const int m = (tt0 + j) * 16 + c16;
    xok[j] = m < a.B;
    xbase[j] = reinterpret_cast<const u32x4*>(a.x + (size_t)(xok[j] ? m : 0) * a.ldx + g4 * 8);
  }

  int kt = 0;
  for (; kt + U <= KT; kt += U) {
    u32x4 wa[RT][U], xb[NBW][U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
#pragma unroll
      for (int r = 0; r < RT; ++r) wa[r][u] = wbase[r][(size_t)(kt + u) * 64];
#pragma unroll
      for (int j = 0; j < NBW; ++j) xb[j][u] = xok[j] ? xbase[j][(kt + u) * 4] : (u32x4){0u, 0u, 0u, 0u};
    }
#pragma unroll
    for (int u = 0; u < U; ++u)
#pragma unroll
      for (int r = 0; r < RT; ++r)
#pragma unroll
        for (int j = 0; j < NBW; ++j)
          acc[r][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, wa[r][u]),
                                                             __builtin_bit_cast(bf16x8, xb[j][u]), acc[r][j], 0, 0, 0);
  }
  for (; kt < KT; ++kt) {
#pragma unroll
    for (int r = 0; r < RT; ++r) {
      const u32x4 wv = wbase[r][(size_t)kt * 64];
#pragma unroll
      for (int j = 0; j < NBW; ++j) {
        const u32x4 xv = xok[j] ? xbase[j][kt * 4] : (u32x4){0u, 0u, 0u, 0u};
        acc[r][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, wv),
                                                           __builtin_bit_cast(bf16x8, xv), acc[r][j], 0, 0, 0);
      }
    }
  }

  // ---- epilogue: lane -> token m = tile*16 + c16, columns n0 .. n0+3 ----
  const int n0 = bt * 16 + g4 * 4;
#pragma unroll
  for (int j = 0; j < NBW; ++j) {
    const int m = (tt0 + j) * 16 + c16;
    const bool mok = m < a.B;
    float o[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int n = n0 + i;
      if constexpr (EPI == EPI_STORE) {
        o[i] = rbf(acc[0][j][i]);
      } else if constexpr (EPI == EPI_RESADD) {
        // hidden = residual + bf16(o)   (TF/.../modeling_qwen3.py:311,322)
        o[i] = (mok && n < a.N) ? rbf(bf2f(a.res[(size_t)m * a.ldres + n]) + rbf(acc[0][j][i])) : 0.f;
      } else {  // EPI_SWIGLU: bf16(bf16(silu(bf16 g)) * bf16 u)   (TF/.../modeling_qwen3.py:81-83)
        const float g = rbf(acc[0][j][i]);
        const float u = rbf(acc[RT - 1][j][i]);
        o[i] = rbf(rbf(g / (1.0f + expf(-g))) * u);
      }
    }
    if (mok) {
      bf16_t* yr = a.y + (size_t)m * a.ldy;
      if (n0 + 3 < a.N && (a.ldy % 4) == 0) {
        uint2 pk;
        pk.x = pack2(o[0], o[1]);
        pk.y = pack2(o[2], o[3]);
        *reinterpret_cast<uint2*>(yr + n0) = pk;
      } else {
#pragma unroll
        for (int i = 0; i < 4; ++i)
          if (n0 + i < a.N) yr[n0 + i] = f2bf(o[i]);
      }
    }
    if constexpr (EPI == EPI_RESADD) {
      // sum of squares of this token's 16 new columns (for the next RMSNorm)
      float ss = (o[0] * o[0] + o[1] * o[1]) + (o[2] * o[2] + o[3] * o[3]);
      ss += __shfl_xor(ss, 16, 64);
      ss += __shfl_xor(ss, 32, 64);
      if (a.ss_out && mok && g4 == 0) a.ss_out[(size_t)m * a.ld_ss_out + bt] = ss;
    }
  }
}

// Large-M form: 2 x 2 waves, each a WR x WN grid of 16 x 16 MFMA tiles (WR weight row tiles
// x WN token tiles), so a 256-thread block covers 32*WR rows x 32*WN tokens and every
// 16-byte fragment a wave loads feeds WN (weights) or WR (activations) MFMAs.  The two
// waves that share a weight (or token) stripe read it through the CU's L1.  SwiGLU takes
// WR/2 gate|up tile pairs per wave.
template <int WR, int WN, int EPI, int U, bool SPLIT = false>
__global__ __launch_bounds__(256) void gemm2_kernel(GemvArgs a) {
  // U: k-tiles in flight per wave (the k loop is latency-bound for short prompts)
  const int lane = threadIdx.x & 63;
  const int wave = threadIdx.x >> 6;
  const int wr = wave & 1, wm = wave >> 1;
  const int rt0 = (blockIdx.x * 2 + wr) * WR;  // first packed row tile of this wave
  const int tt0 = (blockIdx.y * 2 + wm) * WN;  // first token tile of this wave
  const int KT = a.KT;
  const int g4 = lane >> 4, c16 = lane & 15;
  const int n_rt = a.n_row_tiles;
  if (tt0 * 16 >= a.B || rt0 >= n_rt) return;

  f32x4 acc[WR][WN];
#pragma unroll
  for (int r = 0; r < WR; ++r)
#pragma unroll
    for (int j = 0; j < WN; ++j) acc[r][j] = (f32x4){0.f, 0.f, 0.f, 0.f};
  const u32x4* wbase[WR];
#pragma unroll
  for (int r = 0; r < WR; ++r)
    wbase[r] = reinterpret_cast<const u32x4*>(a.w) + ((size_t)min(rt0 + r, n_rt - 1) * KT) * 64 + lane;
  // x_packed (pk_tiles = T): the fragment of token tile t at k tile kt is 1 KiB at (kt T + t) KiB
  const u32x4* xbase[WN];
  bool xok[WN];
  const int xs = a.x_packed ? a.pk_tiles * 64 : 4;  // u32x4 stride per k tile
#pragma unroll
  for (int j = 0; j < WN; ++j) {
    const int m = (tt0 + j) * 16 + c16;
    xok[j] = m < a.B;
    xbase[j] = a.x_packed ? reinterpret_cast<const u32x4*>(a.x) + (tt0 + j) * 64 + lane
                          : reinterpret_cast<const u32x4*>(a.x + (size_t)(xok[j] ? m : 0) * a.ldx + g4 * 8);
  }
  // SPLIT: blockIdx.z takes k-tiles [z*KS, (z+1)*KS) and writes its fp32 partial tile
  int kbeg = 0, kend = KT;
  if constexpr (SPLIT) {
    const int KS = KT / gridDim.z;  // KT % (U * S) == 0 (checked by the launcher)
    kbeg = blockIdx.z * KS;
    kend = kbeg + KS;
  }
  for (int kt = kbeg; kt < kend; kt += U) {  // KT % U == 0 (checked by the launcher)
    u32x4 wa[WR][U], xb[WN][U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
#pragma unroll
      for (int r = 0; r < WR; ++r) wa[r][u] = wbase[r][(size_t)(kt + u) * 64];
#pragma unroll
      for (int j = 0; j < WN; ++j) xb[j][u] = xok[j] ? xbase[j][(kt + u) * xs] : (u32x4){0u, 0u, 0u, 0u};
    }
#pragma unroll
    for (int u = 0; u < U; ++u)
#pragma unroll
      for (int r = 0; r < WR; ++r)
#pragma unroll
        for (int j = 0; j < WN; ++j)
          acc[r][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, wa[r][u]),
                                                             __builtin_bit_cast(bf16x8, xb[j][u]), acc[r][j], 0, 0, 0);
  }
  if constexpr (SPLIT) {
    // partial [z][token][packed row] (fp32): lane -> token (tt0+j)*16 + c16, rows +g4*4 .. +3
    const size_t ld = (size_t)n_rt * 16;
    float* wsz = a.ws + (size_t)blockIdx.z * a.B * ld;
#pragma unroll
    for (int r = 0; r < WR; ++r) {
      if (rt0 + r >= n_rt) continue;
#pragma unroll
      for (int j = 0; j < WN; ++j) {
        const int m = (tt0 + j) * 16 + c16;
        if (m < a.B)
          *reinterpret_cast<f32x4*>(wsz + (size_t)m * ld + (rt0 + r) * 16 + g4 * 4) = acc[r][j];
      }
    }
    return;
  }
  constexpr int OT = EPI == EPI_SWIGLU ? WR / 2 : WR;  // output column tiles per wave
#pragma unroll
  for (int q = 0; q < OT; ++q) {
    const int ot = EPI == EPI_SWIGLU ? rt0 / 2 + q : rt0 + q;  // output 16-column tile
    const int n0 = ot * 16 + g4 * 4;
#pragma unroll
    for (int j = 0; j < WN; ++j) {
      const int m = (tt0 + j) * 16 + c16;
      const bool mok = m < a.B && n0 < a.N;
      float o[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int n = n0 + i;
        if constexpr (EPI == EPI_STORE) {
          o[i] = rbf(acc[q][j][i]);
        } else if constexpr (EPI == EPI_RESADD) {
          o[i] = (mok && n < a.N) ? rbf(bf2f(a.res[(size_t)m * a.ldres + n]) + rbf(acc[q][j][i])) : 0.f;
        } else {
          const float g = rbf(acc[2 * q][j][i]);
          const float u = rbf(acc[2 * q + 1][j][i]);
          o[i] = rbf(rbf(g / (1.0f + expf(-g))) * u);
        }
      }
      if (mok && a.y_packed) {  // SwiGLU output for the packed down-projection input
#pragma unroll
        for (int i = 0; i < 4; ++i)
          if (n0 + i < a.N) a.y[xpkT_index(m, n0 + i, a.pk_tiles)] = f2bf(o[i]);
      } else if (mok) {
        bf16_t* yr = a.y + (size_t)m * a.ldy;
        if (n0 + 3 < a.N && (a.ldy % 4) == 0) {
          uint2 pk;
          pk.x = pack2(o[0], o[1]);
          pk.y = pack2(o[2], o[3]);
          *reinterpret_cast<uint2*>(yr + n0) = pk;
        } else {
#pragma unroll
          for (int i = 0; i < 4; ++i)
            if (n0 + i < a.N) yr[n0 + i] = f2bf(o[i]);
        }
      }
      if constexpr (EPI == EPI_RESADD) {
        float ss = (o[0] * o[0] + o[1] * o[1]) + (o[2] * o[2] + o[3] * o[3]);
        ss += __shfl_xor(ss, 16, 64);
        ss += __shfl_xor(ss, 32, 64);
        if (a.ss_out && mok && g4 == 0) a.ss_out[(size_t)m * a.ld_ss_out + ot] = ss;
      }
    }
  }
}

template <int RT, int EPI>
static void gemm_launch(const GemvArgs& a, int n_tiles, hipStream_t s) {
  const int mt = (a.B + 15) / 16;  // token tiles
  const int nbw = mt >= 16 ? 4 : (mt + 3) / 4;  // tiles per wave: one block covers short prompts
  const dim3 grid(n_tiles, (mt + 4 * nbw - 1) / (4 * nbw));
  switch (nbw) {
    case 1: hipLaunchKernelGGL((gemm_kernel<RT, 1, EPI>), grid, dim3(256), 0, s, a); break;
    case 2: hipLaunchKernelGGL((gemm_kernel<RT, 2, EPI>), grid, dim3(256), 0, s, a); break;
    case 3: hipLaunchKernelGGL((gemm_kernel<RT, 3, EPI>), grid, dim3(256), 0, s, a); break;
    default: hipLaunchKernelGGL((gemm_kernel<RT, 4, EPI>), grid, dim3(256), 0, s, a); break;
  }
}

// Split-K reduce + epilogue: thread (token m, 16-column output tile ot, 4-column group q) sums the
// S partials in split order (deterministic) and applies the same epilogue as gemm2_kernel (bf16
// rounding points of TF/models/qwen3/modeling_qwen3.py:81-83, 311, 322).  Four threads per tile (a
// 181-row o_proj / down reduce is 185 K threads, one f32x4 load per split each; one thread per tile
// ran 12 us on 46 K latency-bound threads); the residual epilogue's per-tile sum of squares adds
// the groups as the GEMM epilogue does, (s0 + s1) + (s2 + s3), across the 4 adjacent lanes.
// SS > 0: the split count as a compile-time constant, so every partial's load issues before the
// first add (a runtime trip count kept one load pair in flight per round trip); 0: runtime S
template <int EPI, int SS = 0>
__global__ __launch_bounds__(256) void gemm_splitk_reduce(GemvArgs a, int S) {
  if constexpr (SS > 0) S = SS;
  const int n_ot = (a.N + 15) / 16;
  const int id = blockIdx.x * 256 + threadIdx.x;
  const bool live = id < a.B * n_ot * 4;
  const int t = live ? id >> 2 : 0, q = id & 3;
  const int m = t / n_ot, ot = t - m * n_ot;
  const size_t ld = (size_t)a.n_row_tiles * 16;
  const float* p = a.ws + (size_t)m * ld;
  const size_t zs = (size_t)a.B * ld;
  f32x4 g = (f32x4){0.f, 0.f, 0.f, 0.f}, u = (f32x4){0.f, 0.f, 0.f, 0.f};
  const int c = (EPI == EPI_SWIGLU ? 2 * ot : ot) * 16 + q * 4;
#pragma unroll
  for (int z = 0; z < S; ++z) {
    g += *reinterpret_cast<const f32x4*>(p + z * zs + c);
    if constexpr (EPI == EPI_SWIGLU) u += *reinterpret_cast<const f32x4*>(p + z * zs + c + 16);
  }
  float o[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int n = ot * 16 + q * 4 + i;
    float v;
    if constexpr (EPI == EPI_STORE) {
      v = rbf(g[i]);
    } else if constexpr (EPI == EPI_RESADD) {
      v = n < a.N ? rbf(bf2f(a.res[(size_t)m * a.ldres + n]) + rbf(g[i])) : 0.f;
    } else {
      const float gg = rbf(g[i]), uu = rbf(u[i]);
      v = rbf(rbf(gg / (1.0f + expf(-gg))) * uu);
    }
    o[i] = v;
  }
  if (EPI == EPI_SWIGLU && live && a.y_packed) {  // the packed down-projection input (xpkT_index)
    const int n = ot * 16 + q * 4;  // 4 columns inside one 8-column group: contiguous there
    if (n + 3 < a.N) {
      uint2 pk;
      pk.x = pack2(o[0], o[1]);
      pk.y = pack2(o[2], o[3]);
      *reinterpret_cast<uint2*>(a.y + xpkT_index(m, n, a.pk_tiles)) = pk;
    } else {
#pragma unroll
      for (int i = 0; i < 4; ++i)
        if (n + i < a.N) a.y[xpkT_index(m, n + i, a.pk_tiles)] = f2bf(o[i]);
    }
  } else if (live) {
    bf16_t* yr = a.y + (size_t)m * a.ldy + ot * 16 + q * 4;
    if (ot * 16 + q * 4 + 3 < a.N && (a.ldy % 4) == 0) {
      uint2 pk;
      pk.x = pack2(o[0], o[1]);
      pk.y = pack2(o[2], o[3]);
      *reinterpret_cast<uint2*>(yr) = pk;
    } else {
#pragma unroll
      for (int i = 0; i < 4; ++i)
        if (ot * 16 + q * 4 + i < a.N) yr[i] = f2bf(o[i]);
    }
  }
  if constexpr (EPI == EPI_RESADD) {
    float s4 = (o[0] * o[0] + o[1] * o[1]) + (o[2] * o[2] + o[3] * o[3]);
    s4 += __shfl_xor(s4, 1, 64);
    s4 += __shfl_xor(s4, 2, 64);
    if (a.ss_out && live && q == 0) a.ss_out[(size_t)m * a.ld_ss_out + ot] = s4;
  }
}

// The residual split-K reduce fused with the next op's input RMSNorm (GemvArgs::pn_w): one block
// per token row, thread t owns columns 8t .. 8t + 7.  Bit-identical to gemm_splitk_reduce<EPI_RESADD>
// followed by rmsnorm_ss_kernel: the partials are summed in split order per column, the 16-column
// sums of squares are formed as the reduce forms them ((c0^2 + c1^2) + (c2^2 + c3^2) per quad, quads
// added pairwise), and the row statistic is rmsnorm_ss's (4 tiles per lane, then wave_sum).  Saves
// the norm's launch after o_proj and after down_proj of every packed split prefill layer.
template <int SS = 0>
__global__ __launch_bounds__(512) void gemm_splitk_reduce_norm(GemvArgs a, int S) {
  if constexpr (SS > 0) S = SS;
  __shared__ float tss[256];
  const int m = blockIdx.x, t = threadIdx.x, lane = t & 63;
  const int H = a.N, n0 = 8 * t;
  const bool ok = n0 < H;
  const size_t ld = (size_t)a.n_row_tiles * 16;
  const float* p = a.ws + (size_t)m * ld + n0;
  const size_t zs = (size_t)a.B * ld;
  f32x4 g0 = (f32x4){0.f, 0.f, 0.f, 0.f}, g1 = g0;
  if (ok)
#pragma unroll
    for (int z = 0; z < S; ++z) {
      g0 += *reinterpret_cast<const f32x4*>(p + z * zs);
      g1 += *reinterpret_cast<const f32x4*>(p + z * zs + 4);
    }
  float v[8], w[8];
  if (ok) {
    float r8[8];
    unpack8(*reinterpret_cast<const uint4*>(a.res + (size_t)m * a.ldres + n0), r8);
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      v[i] = rbf(r8[i] + rbf(g0[i]));
      v[4 + i] = rbf(r8[4 + i] + rbf(g1[i]));
    }
    unpack8(*reinterpret_cast<const uint4*>(a.pn_w + n0), w);
    uint4 o;
    o.x = pack2(v[0], v[1]); o.y = pack2(v[2], v[3]); o.z = pack2(v[4], v[5]); o.w = pack2(v[6], v[7]);
    *reinterpret_cast<uint4*>(a.y + (size_t)m * a.ldy + n0) = o;
  } else {
#pragma unroll
    for (int i = 0; i < 8; ++i) v[i] = w[i] = 0.f;
  }
  // 16-column tile sums of squares: quads as the reduce forms them, the two halves of a tile
  // in threads 2u, 2u + 1
  float s4 = ((v[0] * v[0] + v[1] * v[1]) + (v[2] * v[2] + v[3] * v[3])) +
             ((v[4] * v[4] + v[5] * v[5]) + (v[6] * v[6] + v[7] * v[7]));
  s4 += __shfl_xor(s4, 1, 64);
  if (ok && (t & 1) == 0) {
    tss[t >> 1] = s4;
    if (a.ss_out) a.ss_out[(size_t)m * a.ld_ss_out + (t >> 1)] = s4;
  }
  __syncthreads();
  float sw = 0.f;
  for (int t4 = lane * 4; t4 < (H >> 4); t4 += 256) sw += (tss[t4] + tss[t4 + 1]) + (tss[t4 + 2] + tss[t4 + 3]);
  sw = wave_sum(sw);
  const float r = 1.0f / sqrtf(sw / (float)H + a.pn_eps);
  if (!ok) return;
  float q[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) q[i] = w[i] * rbf(v[i] * r);
  uint4 o;
  o.x = pack2(q[0], q[1]); o.y = pack2(q[2], q[3]); o.z = pack2(q[4], q[5]); o.w = pack2(q[6], q[7]);
  *reinterpret_cast<uint4*>(a.pn_y + xpkT_index(m, n0, a.pn_tiles)) = o;
}

// The q|k|v split-K reduce fused with the q/k norm + RoPE + KV append (GemvArgs::qkr, D = 128):
// one block per token row, 16 threads per head (thread t: head t / 16, dims 8 (t % 16) ..), the
// partials summed in split order and rounded to bf16 as gemm_splitk_reduce<EPI_STORE> writes them,
// then qk_item_d128 exactly as qk_norm_rope's per-item form runs it on those values.  Saves the
// separate q|k|v write + read and one launch per packed split prefill layer.
template <int SS = 0>
__global__ __launch_bounds__(1024) void gemm_splitk_reduce_qkrope(GemvArgs a, int S, QKRopeArgs q) {
  if constexpr (SS > 0) S = SS;
  const int m = blockIdx.x, t = threadIdx.x;
  const int hd = t >> 4, l16 = t & 15, n0 = 8 * t;
  const size_t ld = (size_t)a.n_row_tiles * 16;
  const float* p = a.ws + (size_t)m * ld + n0;
  const size_t zs = (size_t)a.B * ld;
  f32x4 g0 = (f32x4){0.f, 0.f, 0.f, 0.f}, g1 = g0;
#pragma unroll
  for (int z = 0; z < S; ++z) {
    g0 += *reinterpret_cast<const f32x4*>(p + z * zs);
    g1 += *reinterpret_cast<const f32x4*>(p + z * zs + 4);
  }
  float x[8];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    x[i] = rbf(g0[i]);
    x[4 + i] = rbf(g1[i]);
  }
  qk_item_d128(q, m, hd, l16, x, true);
}

// split count for a short prompt: the GEMM's per-workgroup latency is ~constant in N, so
// split K until the grid covers the CUs (cdna_hip_programming.md "Projection GEMM at M = 256"),
// keeping >= 16 k-tiles per split and the partials inside the workspace
template <int WR, int WN, int U>
static int gemm_splits(const GemvArgs& a, int nx, int ny) {
  static const int force = getenv("MTTS_GEMM_SPLITK") ? atoi(getenv("MTTS_GEMM_SPLITK")) : -1;
  if (!a.ws || force == 0) return 1;
  int S = force > 0 ? force : 1;
  if (force < 0)
    while (nx * ny * S < 256 && a.KT / (2 * S) >= 16) S *= 2;
  while (S > 1 && (a.KT % (U * S) || (size_t)S * a.B * a.n_row_tiles * 16 > a.ws_floats)) S /= 2;
  return S;
}


// ---------------------------------------------------------------------------
// LDS-staged form for packed activations (round 4): a 512-thread block (8 waves, 2 x 4) owns
// 32 WR weight rows x 64 WN tokens; per 32-deep k-step the block's weight tiles (2 WR row tiles)
// and activation fragments (4 WN token tiles) -- 1 KiB each, contiguous in both packed layouts --
// go global -> LDS by LDS-DMA (buffer_load ... lds: no registers) into a G3_NST-stage ring, G3_NST - 1
// k-steps ahead of the waves running the current step's MFMAs from LDS.  Every A / B fragment a wave
// reads from LDS feeds WN / WR MFMAs (gemm2_kernel re-read them from L1/L2 per wave, ~0.3 MFMA busy
// at M = 5,792: profiles/r03_b_pmc_mfma.json; the first, double-buffered 64-deep form of this kernel
// 0.23-0.39, this 3-stage ring 105 vs 110 ms for the 32-utterance prefill; 4 stages 123 ms: at 72 KiB
// the 128-row form fits two blocks per CU; profiles/r04_e_*).  SPLIT: blockIdx.z takes a K range and writes fp32
// partials for gemm_splitk_reduce (few row blocks: o_proj / down at N 4,096).
//
// Shape <NWR, NWN, WR, WN, NST>: NWR x NWN waves, each WR weight row tiles x WN token tiles, an
// NST-stage ring.  <2, 4, *, 4, 3> for long prompts; <3, 2, 2, 6, 8> for prompts of <= 192 token rows
// (the batch-1 clone prefill, 181 rows): every token of the prompt in one block, so each weight
// byte leaves HBM once, 96-row blocks (gate|up: 256 of them, one per CU), and seven 18 KiB stages
// in flight per CU -- the HBM latency x bandwidth product (0.8 us x 8 TB/s under load,
// profiles/r03_m_lat_probe.txt) is ~25 KiB of weights per CU, which gemm2_kernel's register-
// staged k loop (issue, wait, 64 MFMAs) left idle most of the time (gate|up 89 us at 181 rows).
#ifndef G3_NST
#define G3_NST 3
#endif
#ifndef G3S_NST
#define G3S_NST 5  // the <= 192-row form's stages
#endif


template <int NWR, int NWN, int WR, int WN, int NST>
constexpr size_t gemm3_lds_bytes() { return (size_t)NST * (NWR * WR + NWN * WN) * 1024; }
// gemm3 epilogue of one wave's WR x WN tiles (gemm2_kernel's): lane -> token (tt0 + j) * 16 + c16,
// output columns n0 .. n0 + 3; SPLIT: the fp32 partial tile of K range blockIdx.z
template <int WR, int WN, int EPI, bool SPLIT>
__device__ __forceinline__ void gemm_tile_epilogue(const GemvArgs& a, const f32x4 (&acc)[WR][WN], int rt0, int tt0,
                                                   int lane) {
  const int n_rt = a.n_row_tiles;
  const int g4 = lane >> 4, c16 = lane & 15;
  if constexpr (SPLIT) {
    const size_t ld = (size_t)n_rt * 16;
    float* wsz = a.ws + (size_t)blockIdx.z * a.B * ld;
#pragma unroll
    for (int r = 0; r < WR; ++r) {
      if (rt0 + r >= n_rt) continue;
#pragma unroll
      for (int j = 0; j < WN; ++j) {
        const int m = (tt0 + j) * 16 + c16;
        if (m < a.B) *reinterpret_cast<f32x4*>(wsz + (size_t)m * ld + (rt0 + r) * 16 + g4 * 4) = acc[r][j];
      }
    }
    return;
  }
  // epilogue (gemm2_kernel's): lane -> token (tt0 + j) * 16 + c16, output columns n0 .. n0 + 3
  constexpr int OT = EPI == EPI_SWIGLU ? WR / 2 : WR;
#pragma unroll
  for (int q = 0; q < OT; ++q) {
    const int ot = EPI == EPI_SWIGLU ? rt0 / 2 + q : rt0 + q;
    const int n0 = ot * 16 + g4 * 4;
#pragma unroll
    for (int j = 0; j < WN; ++j) {
      const int m = (tt0 + j) * 16 + c16;
      const bool mok = m < a.B && n0 < a.N;
      float o[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int n = n0 + i;
        if constexpr (EPI == EPI_STORE) {
          o[i] = rbf(acc[q][j][i]);
        } else if constexpr (EPI == EPI_RESADD) {
          o[i] = (mok && n < a.N) ? rbf(bf2f(a.res[(size_t)m * a.ldres + n]) + rbf(acc[q][j][i])) : 0.f;
        } else {
          const float g = rbf(acc[2 * q][j][i]);
          const float u = rbf(acc[2 * q + 1][j][i]);
          o[i] = rbf(rbf(g / (1.0f + expf(-g))) * u);
        }
      }
      if (mok && a.y_packed) {
#pragma unroll
        for (int i = 0; i < 4; ++i)
          if (n0 + i < a.N) a.y[xpkT_index(m, n0 + i, a.pk_tiles)] = f2bf(o[i]);
      } else if (mok) {
        bf16_t* yr = a.y + (size_t)m * a.ldy;
        if (n0 + 3 < a.N && (a.ldy % 4) == 0) {
          uint2 pk;
          pk.x = pack2(o[0], o[1]);
          pk.y = pack2(o[2], o[3]);
          *reinterpret_cast<uint2*>(yr + n0) = pk;
        } else {
#pragma unroll
          for (int i = 0; i < 4; ++i)
            if (n0 + i < a.N) yr[n0 + i] = f2bf(o[i]);
        }
      }
      if constexpr (EPI == EPI_RESADD) {
        float ss = (o[0] * o[0] + o[1] * o[1]) + (o[2] * o[2] + o[3] * o[3]);
        ss += __shfl_xor(ss, 16, 64);
        ss += __shfl_xor(ss, 32, 64);
        if (a.ss_out && mok && g4 == 0) a.ss_out[(size_t)m * a.ld_ss_out + ot] = ss;
      }
    }
  }
}

template <int NWR, int NWN, int WR, int WN, int NST, int EPI, bool SPLIT = false>
__global__ __launch_bounds__(NWR * NWN * 64) void gemm3_kernel(GemvArgs a) {
  typedef __attribute__((address_space(3))) void lvoid;
  constexpr int NW = NWR * NWN;                    // waves
  constexpr int BR = NWR * WR, BT = NWN * WN;      // row tiles / token tiles per block
  constexpr int TILES = BR + BT;                   // 1 KiB tiles per stage (one k tile)
  constexpr int STAGE = TILES * 1024;
  constexpr int TPW = TILES / NW;                  // loads per wave per stage
  static_assert(TILES % NW == 0, "tiles per stage split over the waves");
  static_assert(TPW * (NST - 1) <= 63, "vmcnt counts the stages in flight");
  static_assert(EPI != EPI_SWIGLU || WR % 2 == 0, "gate|up row tile pairs stay within a wave");
  extern __shared__ __attribute__((aligned(16))) unsigned char g3_lds[];
  const int lane = threadIdx.x & 63;
  // (wave-uniform for the compiler: the LDS-DMA destination goes through M0, and a per-lane one
  // is a readfirstlane loop around every load)
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int wr = wave % NWR, wn = wave / NWR;
  const int KT = a.KT, T = a.pk_tiles, n_rt = a.n_row_tiles;
  const int rb0 = blockIdx.x * BR, tb0 = blockIdx.y * BT;
  if (rb0 >= n_rt || tb0 >= T) return;
  int kbeg = 0, kend = KT;
  if constexpr (SPLIT) {
    const int KS = KT / gridDim.z;
    kbeg = blockIdx.z * KS;
    kend = kbeg + KS;
  }
  const __amdgpu_buffer_rsrc_t wrs = __builtin_amdgcn_make_buffer_rsrc(const_cast<bf16_t*>(a.w), 0, 0x7fffffff, 0x00020000);
  const __amdgpu_buffer_rsrc_t xrs = __builtin_amdgcn_make_buffer_rsrc(const_cast<bf16_t*>(a.x), 0, 0x7fffffff, 0x00020000);
  // stage loads of k step `step` (k tile kt): tile q = wave * TPW + i; q < BR: weights (row tile q), else activations
  // (token tile q - BR); rows / tokens past the matrix re-read the last one.  Every stage issues
  // exactly TPW loads per wave (k tiles past the range re-read the last one, never computed), so
  // the counted vmcnt below is exact at the tail too.
  // (a k order rotated per block, so that blocks do not read the same activation tiles in
  // lockstep, measured slower: the 32-utterance prefill 92.6 -> 106.7 ms, profiles/r04_i_*)
  const int KS = kend - kbeg;
  auto issue = [&](int step, int buf) {
    const int kt = kbeg + min(step, KS - 1);
#pragma unroll
    for (int i = 0; i < TPW; ++i) {
      const int q = wave * TPW + i;
      unsigned char* dst = g3_lds + buf * STAGE + q * 1024;
      if (q < BR) {
        const int rt = min(rb0 + q, n_rt - 1);
        __builtin_amdgcn_raw_ptr_buffer_load_lds(wrs, (lvoid*)dst, 16, (uint32_t)(((size_t)rt * KT + kt) * 1024 + lane * 16),
                                                 0, 0, 0);
      } else {
        const int tt = min(tb0 + q - BR, T - 1);
        __builtin_amdgcn_raw_ptr_buffer_load_lds(xrs, (lvoid*)dst, 16, (uint32_t)(((size_t)kt * T + tt) * 1024 + lane * 16),
                                                 0, 0, 0);
      }
    }
  };
  f32x4 acc[WR][WN];
#pragma unroll
  for (int r = 0; r < WR; ++r)
#pragma unroll
    for (int j = 0; j < WN; ++j) acc[r][j] = (f32x4){0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int st = 0; st < NST - 1; ++st) issue(st, st);
  int buf = 0;
  for (int i = 0; i < KS; ++i) {
    // this stage's loads have landed once only the NST - 2 younger stages are in flight
    // stage `buf` landed for every wave; the buffer refilled below was last read a step ago.  A bare
    // barrier: __syncthreads' release fence waits for every LDS-DMA load in flight (vmcnt(0)), which
    // would leave one stage of prefetch instead of NST - 1
    asm volatile("s_waitcnt vmcnt(%0)\n\ts_barrier" ::"n"(TPW * (NST - 2)) : "memory");
    issue(i + NST - 1, (buf + NST - 1) % NST);
    const u32x4* A = reinterpret_cast<const u32x4*>(g3_lds + buf * STAGE);
    const u32x4* Bx = reinterpret_cast<const u32x4*>(g3_lds + buf * STAGE + BR * 1024);
    u32x4 af[WR], bf[WN];
#pragma unroll
    for (int r = 0; r < WR; ++r) af[r] = A[(wr * WR + r) * 64 + lane];
#pragma unroll
    for (int j = 0; j < WN; ++j) bf[j] = Bx[(wn * WN + j) * 64 + lane];
#pragma unroll
    for (int r = 0; r < WR; ++r)
#pragma unroll
      for (int j = 0; j < WN; ++j)
        acc[r][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, af[r]),
                                                           __builtin_bit_cast(bf16x8, bf[j]), acc[r][j], 0, 0, 0);
    buf = buf + 1 == NST ? 0 : buf + 1;
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // (the surplus tail loads land before the block exits)
  gemm_tile_epilogue<WR, WN, EPI, SPLIT>(a, acc, rb0 + wr * WR, tb0 + wn * WN, lane);
}

// ---------------------------------------------------------------------------
// <= 192-row form with split paths (gemm5): 6 waves share one 96-row weight block and each owns 2 of
// the prompt's 12 token tiles.  Weight tiles go global -> LDS by LDS-DMA (one 1 KiB load per wave
// per k step, R steps ahead); each wave's own 2 activation fragments go global -> VGPRs (R steps
// ahead, a register ring indexed at compile time), read by the one wave that uses them.  gemm3's
// form moved 18 KiB per CU per k step through LDS-DMA, ~18 B/clk/CU whatever the source
// (profiles/r04_m_gemm3_probe.txt); here LDS-DMA carries 6 KiB and the vector path 12 KiB.
// Shape <NWR, NWN, WR, WN>: NWR x NWN waves, each WR weight row tiles x WN token tiles; the block's
// BR = NWR WR weight tiles per k step are split over the waves' LDS-DMA loads, each wave loads its own
// WN activation fragments.  <1, 6, 6, 2> for <= 192 rows.
#ifndef G5S_R
#define G5S_R 4  // k steps in flight of the <= 192-row form (A/B)
#endif

template <int NWR, int NWN, int WR, int R>
constexpr size_t gemm5_lds_bytes() { return (size_t)(R + 1) * NWR * WR * 1024; }
template <int NWR, int NWN, int WR, int WN, int R, int EPI, bool SPLIT = false>
__global__ __launch_bounds__(NWR * NWN * 64) void gemm5_kernel(GemvArgs a) {
  typedef __attribute__((address_space(3))) void lvoid;
  constexpr int NW = NWR * NWN, NST = R + 1, BR = NWR * WR, BT = NWN * WN;
  constexpr int TPW = BR / NW;  // weight tiles per wave per k step
  static_assert(BR % NW == 0, "weight tiles split over the waves");
  static_assert((TPW + WN) * R <= 63, "vmcnt counts the k steps in flight");
  static_assert(EPI != EPI_SWIGLU || WR % 2 == 0, "gate|up row tile pairs stay within a wave");
  constexpr int STAGE = BR * 1024;
  extern __shared__ __attribute__((aligned(16))) unsigned char g5_lds[];
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int wr = wave % NWR, wn = wave / NWR;
  const int KT = a.KT, T = a.pk_tiles, n_rt = a.n_row_tiles;
  const int rb0 = blockIdx.x * BR, tb0 = blockIdx.y * BT;
  if (rb0 >= n_rt || tb0 >= T) return;
  int kbeg = 0, kend = KT;
  if constexpr (SPLIT) {
    const int KSp = KT / gridDim.z;
    kbeg = blockIdx.z * KSp;
    kend = kbeg + KSp;
  }
  const int KS = kend - kbeg;
  const __amdgpu_buffer_rsrc_t wrs = __builtin_amdgcn_make_buffer_rsrc(const_cast<bf16_t*>(a.w), 0, 0x7fffffff, 0x00020000);
  const __amdgpu_buffer_rsrc_t xrs = __builtin_amdgcn_make_buffer_rsrc(const_cast<bf16_t*>(a.x), 0, 0x7fffffff, 0x00020000);
  int tt[WN];
#pragma unroll
  for (int j = 0; j < WN; ++j) tt[j] = min(tb0 + wn * WN + j, T - 1);
  // k steps past the range re-read the last k tile (never computed): every step issues the same
  // loads, so each wait below is exact
  auto issue_w = [&](int step) {
    const int kt = kbeg + min(step, KS - 1);
#pragma unroll
    for (int t = 0; t < TPW; ++t) {
      const int q = wave * TPW + t;
      const int rt = min(rb0 + q, n_rt - 1);
      __builtin_amdgcn_raw_ptr_buffer_load_lds(wrs, (lvoid*)(g5_lds + (step % NST) * STAGE + q * 1024), 16,
                                               (uint32_t)(((size_t)rt * KT + kt) * 1024 + lane * 16), 0, 0, 0);
    }
  };
  auto issue_x = [&](u32x4 (&dst)[WN], int step) {
    const int kt = kbeg + min(step, KS - 1);
#pragma unroll
    for (int j = 0; j < WN; ++j)
      dst[j] = __builtin_amdgcn_raw_buffer_load_b128(xrs, (uint32_t)(((size_t)kt * T + tt[j]) * 1024 + lane * 16), 0, 0);
  };
  f32x4 acc[WR][WN];
#pragma unroll
  for (int r = 0; r < WR; ++r)
#pragma unroll
    for (int j = 0; j < WN; ++j) acc[r][j] = (f32x4){0.f, 0.f, 0.f, 0.f};
  u32x4 xr[R][WN];
#pragma unroll
  for (int r = 0; r < R; ++r) {
    issue_w(r);
    issue_x(xr[r], r);
  }
  for (int i0 = 0; i0 < KS; i0 += R) {
#pragma unroll
    for (int r = 0; r < R; ++r) {
      const int i = i0 + r;
      // step i's weight tiles (every wave's LDS-DMA) and this wave's activations have landed once
      // only the R - 1 younger steps' loads (1 + WN per step) are in flight
      asm volatile("s_waitcnt vmcnt(%0)\n\ts_barrier" ::"n"((TPW + WN) * (R - 1)) : "memory");
      issue_w(i + R);  // into stage (i + R) % NST = (i - 1) % NST, read at step i - 1
      if (i < KS) {
        const u32x4* A = reinterpret_cast<const u32x4*>(g5_lds + (i % NST) * STAGE);
        u32x4 af[WR];
#pragma unroll
        for (int rr = 0; rr < WR; ++rr) af[rr] = A[(wr * WR + rr) * 64 + lane];
#pragma unroll
        for (int rr = 0; rr < WR; ++rr)
#pragma unroll
          for (int j = 0; j < WN; ++j)
            acc[rr][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, af[rr]),
                                                                __builtin_bit_cast(bf16x8, xr[r][j]), acc[rr][j], 0, 0, 0);
      }
      issue_x(xr[r], i + R);
    }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  gemm_tile_epilogue<WR, WN, EPI, SPLIT>(a, acc, rb0 + wr * WR, tb0 + wn * WN, lane);
}

// launch KERNEL<..., SS> with the split count S as a compile-time constant when it is 2 / 4 / 8 / 16
#define MTTS_SPLIT_DISPATCH(S, LAUNCH) \
  do {                                 \
    switch (S) {                       \
      case 2: LAUNCH(2); break;        \
      case 4: LAUNCH(4); break;        \
      case 8: LAUNCH(8); break;        \
      case 16: LAUNCH(16); break;      \
      default: LAUNCH(0); break;       \
    }                                  \
  } while (0)

// split-K ways of a gemm5 launch of `blocks` workgroups: doubled until the grid covers `cover` or a
// split would drop below `mink` k tiles (row-major outputs with a partials workspace only)
// (a packed SwiGLU output -- the down projection's input -- is written packed by the reduce too)
static int gemm5_splits(const GemvArgs& a, int blocks, int cover, int mink, bool packed_ok = false) {
  int S = 1;
  if ((!a.y_packed || packed_ok) && a.ws) {
    while (blocks * S < cover && a.KT / (2 * S) >= mink) S *= 2;
    while (S > 1 && (a.KT % S || (size_t)S * a.B * a.n_row_tiles * 16 > a.ws_floats)) S /= 2;
  }
  return S;
}

template <int NWR, int NWN, int WR, int WN, int R, int EPI>
static hipError_t gemm5_launch(GemvArgs a, int cover, int mink, hipStream_t s, bool packed_split = false) {
  constexpr int BR = NWR * WR, BT = NWN * WN;
  const size_t lds = gemm5_lds_bytes<NWR, NWN, WR, R>();
  const dim3 grid((a.n_row_tiles + BR - 1) / BR, (a.pk_tiles + BT - 1) / BT);
  const int S = gemm5_splits(a, (int)(grid.x * grid.y), cover, mink, packed_split);
  static bool attr = false;
  if (!attr) {
    (void)hipFuncSetAttribute((const void*)gemm5_kernel<NWR, NWN, WR, WN, R, EPI, false>,
                              hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    (void)hipFuncSetAttribute((const void*)gemm5_kernel<NWR, NWN, WR, WN, R, EPI, true>,
                              hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    attr = true;
  }
  if (S > 1) {
    hipLaunchKernelGGL((gemm5_kernel<NWR, NWN, WR, WN, R, EPI, true>), dim3(grid.x, grid.y, S),
                       dim3(NWR * NWN * 64), lds, s, a);
    if (EPI == EPI_STORE && a.qkr && a.qkr->D == 128 && a.N == (a.qkr->Hq + 2 * a.qkr->Hkv) * 128 && a.N <= 8192) {
#define L_(SS) hipLaunchKernelGGL(gemm_splitk_reduce_qkrope<SS>, dim3(a.B), dim3(a.N / 8), 0, s, a, S, *a.qkr)
      MTTS_SPLIT_DISPATCH(S, L_);
#undef L_
      if (a.qkr_done) *a.qkr_done = 1;
      return hipGetLastError();
    }
    // (N / 8 threads: whole waves for its wave_sum, and its sums-of-squares pass reads 4 tiles a
    // lane, so H % 64 == 0; N % 512 covers both -- other widths take the plain reduce + rmsnorm_ss)
    if (EPI == EPI_RESADD && a.pn_w && a.N % 512 == 0 && a.N <= 4096 && a.ldres % 8 == 0 && a.ldy % 8 == 0) {
#define L_(SS) hipLaunchKernelGGL(gemm_splitk_reduce_norm<SS>, dim3(a.B), dim3(a.N / 8), 0, s, a, S)
      MTTS_SPLIT_DISPATCH(S, L_);
#undef L_
      if (a.pn_done) *a.pn_done = 1;
      return hipGetLastError();
    }
    const int n = a.B * ((a.N + 15) / 16) * 4;
#define L_(SS) hipLaunchKernelGGL((gemm_splitk_reduce<EPI, SS>), dim3((n + 255) / 256), dim3(256), 0, s, a, S)
    MTTS_SPLIT_DISPATCH(S, L_);
#undef L_
  } else {
    hipLaunchKernelGGL((gemm5_kernel<NWR, NWN, WR, WN, R, EPI, false>), grid, dim3(NWR * NWN * 64), lds, s, a);
  }
  return hipGetLastError();
}

// gemm3 launch of one shape: split K until the grid covers the CUs (partials through
// gemm_splitk_reduce; row-major outputs only), down to MINK k tiles per split
template <int NWR, int NWN, int WR, int WN, int NST, int EPI>
static hipError_t gemm3_launch(GemvArgs a, int cover, int mink, hipStream_t s) {
  constexpr int BR = NWR * WR, BT = NWN * WN;
  const size_t lds = gemm3_lds_bytes<NWR, NWN, WR, WN, NST>();
  const void* k_full = (const void*)gemm3_kernel<NWR, NWN, WR, WN, NST, EPI, false>;
  const void* k_split = (const void*)gemm3_kernel<NWR, NWN, WR, WN, NST, EPI, true>;
  const dim3 grid((a.n_row_tiles + BR - 1) / BR, (a.pk_tiles + BT - 1) / BT);
  static const int force = getenv("MTTS_GEMM3_SPLIT") ? atoi(getenv("MTTS_GEMM3_SPLIT")) : -1;
  int S = 1;
  if (!a.y_packed && a.ws) {
    if (force > 0) S = force;
    else if (force < 0)
      while ((int)(grid.x * grid.y) * S < cover && a.KT / (2 * S) >= mink) S *= 2;
    while (S > 1 && (a.KT % S || (size_t)S * a.B * a.n_row_tiles * 16 > a.ws_floats)) S /= 2;
  }
  static bool attr = false;
  if (!attr) {
    (void)hipFuncSetAttribute(k_full, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    (void)hipFuncSetAttribute(k_split, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    attr = true;
  }
  const dim3 block(NWR * NWN * 64);
  void* args[] = {&a};
  if (S > 1) {
    hipError_t e = hipLaunchKernel(k_split, dim3(grid.x, grid.y, S), block, args, lds, s);
    if (e != hipSuccess) return e;
    const int n = a.B * ((a.N + 15) / 16) * 4;
#define L_(SS) hipLaunchKernelGGL((gemm_splitk_reduce<EPI, SS>), dim3((n + 255) / 256), dim3(256), 0, s, a, S)
    MTTS_SPLIT_DISPATCH(S, L_);
#undef L_
  } else {
    hipError_t e = hipLaunchKernel(k_full, grid, block, args, lds, s);
    if (e != hipSuccess) return e;
  }
  return hipGetLastError();
}

// gemm3 shape by prompt rows: <= 384 token rows (24 tiles) token blocks of 192 rows on 96- / 128-row
// weight blocks, split to >= 256 workgroups (q|k|v 4, o_proj / down 8 ways); longer prompts 256-row
// blocks for the wide matrices, 128 for N 4,096 (o_proj / down), split to >= 128 workgroups
template <int EPI>
static hipError_t gemm3_pick(GemvArgs a, hipStream_t s) {
  // (24 since round 5: 193-384 rows as two token blocks of the small form rather than the long forms:
  // 300 rows 10.9 -> 9.0 ms, 2 x 181 11.0 -> 9.4, 384 rows 11.1 -> 9.7; 32 tiles slower,
  // profiles/r05_r_*)
  static const int small_max = getenv("MTTS_GEMM3_SMALL") ? atoi(getenv("MTTS_GEMM3_SMALL")) : 24;
  static const int small_mink = getenv("MTTS_GEMM3_SMALL_MINK") ? atoi(getenv("MTTS_GEMM3_SMALL_MINK")) : 8;  // A/B
  static const int wide_min = getenv("MTTS_GEMM3_WIDE") ? atoi(getenv("MTTS_GEMM3_WIDE")) : 512;  // A/B (1024 until round 5: the Local backbone gate|up, 768 row tiles, 14.4 -> 14.2 ms prefill)
  // (a register-staged variant -- global -> VGPRs -> ds_write_b128, two LDS stages -- measured
  // slower: 181 rows 7.97 -> 8.20 ms, 32 utterances 91.9 -> 95.7 ms, profiles/r04_j_*)
  // MTTS_GEMM5 (A/B): the split-path form for <= 12 token tiles
  static const int g5 = getenv("MTTS_GEMM5") ? atoi(getenv("MTTS_GEMM5")) : 1;
  // MTTS_GEMM5_SMALL_COVER (A/B): workgroups the split-K aims for
  static const int small_cover0 = getenv("MTTS_GEMM5_SMALL_COVER") ? atoi(getenv("MTTS_GEMM5_SMALL_COVER")) : 256;
  // MTTS_GEMM5_SWIGLU_COVER (A/B): the same for gate|up (its split reduce applies SwiGLU and writes
  // the packed down input)
  static const int swiglu_cover = getenv("MTTS_GEMM5_SWIGLU_COVER") ? atoi(getenv("MTTS_GEMM5_SWIGLU_COVER")) : 256;
  const int small_cover = EPI == EPI_SWIGLU ? swiglu_cover : small_cover0;
  // two shapes: 6 waves x 2 token tiles on 96-row blocks, or 4 waves x 3 on 128-row blocks (one wave a
  // SIMD: the same MFMA time per k step for 8 row tiles instead of 6).  Taken by rounds over the
  // CUs x k steps per block (ties: the 96-row form); the 128-row form gives o_proj / down 256 split
  // blocks where the 96-row form had 344: 181-row prompt 33.2 -> 23.5 us (profiles/r05_m_*).
  // MTTS_GEMM5_SMALL_SHAPE=1 / 2 / 3 forces one (A/B).
  static const int small_shape = getenv("MTTS_GEMM5_SMALL_SHAPE") ? atoi(getenv("MTTS_GEMM5_SMALL_SHAPE")) : 0;
  if (a.pk_tiles <= small_max && g5) {
    // cost = rounds of workgroups over the CUs x k steps per workgroup x MFMA cycles per k step on
    // the busiest SIMD (relative): shape 1 <1,6,6,2> 96-row x 12-token blocks (2 waves x 12 MFMAs
    // on two SIMDs: 2), shape 2 <1,4,8,3> 128 x 12 (1 x 24: 2), shape 3 <1,6,6,3> 96 x 18 (2 x 18:
    // 3) -- one token block where 13-18 tiles needed two of 12
    auto cost = [&](int br, int bt, int step) {
      const int ty = (a.pk_tiles + bt - 1) / bt;
      const int rb = (a.n_row_tiles + br - 1) / br;
      const int S = gemm5_splits(a, rb * ty, small_cover, small_mink, EPI == EPI_SWIGLU);
      return (long)((rb * ty * S + 255) / 256) * (a.KT / S) * step;
    };
    int shape = small_shape;
    if (shape < 1 || shape > 3) {
      const long c1 = cost(6, 12, 2), c2 = cost(8, 12, 2), c3 = cost(6, 18, 3);
      shape = c2 < c1 ? 2 : 1;
      if (c3 < std::min(c1, c2)) shape = 3;
    }
    if (shape == 3) return gemm5_launch<1, 6, 6, 3, G5S_R, EPI>(a, small_cover, small_mink, s, EPI == EPI_SWIGLU);
    if (shape == 2) return gemm5_launch<1, 4, 8, 3, G5S_R, EPI>(a, small_cover, small_mink, s, EPI == EPI_SWIGLU);
    return gemm5_launch<1, 6, 6, 2, G5S_R, EPI>(a, small_cover, small_mink, s, EPI == EPI_SWIGLU);
  }
  if (a.pk_tiles <= small_max) return gemm3_launch<3, 2, 2, 6, G3S_NST, EPI>(a, 256, small_mink, s);
  // MTTS_GEMM5_LONG (A/B, 0: gemm3): the long-prompt shapes with split paths as well -- batch-4 prefill
  // 18.6 -> 17.5 ms, 1,024 rows 27.7 -> 26.6, TTSD long form 75.2 -> 71.6, 32 utterances unchanged
  // (profiles/r04_p_gemm5_long_ab.txt)
  static const int g5l = getenv("MTTS_GEMM5_LONG") ? atoi(getenv("MTTS_GEMM5_LONG")) : 1;
  // MTTS_GEMM5_LONG_COVER (A/B): workgroups the long forms split K for (128 until late round 5: the
  // batch-4 prompts' o_proj / q|k|v then ran 128 / 192 blocks on 256 CUs; 256: 4 x 126 rows 11.3 ->
  // 10.2 ms, 8 x 126 21.0 -> 17.7, 1,024 rows 21.8 -> 18.5, 2,117 even; profiles/r05_z_ab_long_cover.txt)
  static const int long_cover = getenv("MTTS_GEMM5_LONG_COVER") ? atoi(getenv("MTTS_GEMM5_LONG_COVER")) : 256;
  if (g5l) {
    // token tiles per wave chosen as below for the 256-row blocks too (4 or 5; MTTS_GEMM5_WWN forces)
    if (a.n_row_tiles >= wide_min) {
      static const int force_wwn = getenv("MTTS_GEMM5_WWN") ? atoi(getenv("MTTS_GEMM5_WWN")) : 0;
      int wn = force_wwn;
      if (wn < 4 || wn > 5) {
        const long rb = (a.n_row_tiles + 15) / 16;
        const long c4 = (rb * ((a.pk_tiles + 15) / 16) + 255) / 256 * 4;
        const long c5 = (rb * ((a.pk_tiles + 19) / 20) + 255) / 256 * 5;
        wn = c5 < c4 ? 5 : 4;
      }
      if (wn == 5) return gemm5_launch<2, 4, 8, 5, 2, EPI>(a, long_cover, 16, s);
      return gemm5_launch<2, 4, 8, 4, 2, EPI>(a, long_cover, 16, s);
    }
    // 128-row blocks: token tiles per wave WN = 4, 5 or 6 by the launch's rounds over the CUs x
    // per-block work (ceil(blocks / 256) x WN).  WN = 4 alone gave the TTSD script's 2,117-row o_proj
    // and down projections 288 blocks (32 CUs holding two): 118 / 345 us against hipBLASLt's 96 / 229
    // (scripts/blas_ref.py, profiles/r05_j_*); WN = 5 deals 224 blocks, one a CU.  MTTS_GEMM5_WN
    // forces one (A/B).
    static const int force_wn = getenv("MTTS_GEMM5_WN") ? atoi(getenv("MTTS_GEMM5_WN")) : 0;
    int wn = force_wn;
    if (wn < 4 || wn > 6) {
      const int rb = (a.n_row_tiles + 7) / 8;
      long best = 1L << 40;
      for (int w = 4; w <= 6; ++w) {
        const long blocks = (long)rb * ((a.pk_tiles + 4 * w - 1) / (4 * w));
        const long cost = (blocks + 255) / 256 * w;
        if (cost < best) { best = cost; wn = w; }
      }
    }
    if (wn == 5) return gemm5_launch<2, 4, 4, 5, 2, EPI>(a, long_cover, 16, s);
    if (wn == 6) return gemm5_launch<2, 4, 4, 6, 2, EPI>(a, long_cover, 16, s);
    return gemm5_launch<2, 4, 4, 4, 2, EPI>(a, long_cover, 16, s);
  }
  if (a.n_row_tiles >= wide_min) return gemm3_launch<2, 4, 8, 4, G3_NST, EPI>(a, 128, 16, s);
  return gemm3_launch<2, 4, 4, 4, G3_NST, EPI>(a, 128, 16, s);
}

template <int WR, int WN, int EPI>
static void gemm2_launch(GemvArgs a, hipStream_t s) {
  a.n_row_tiles = (EPI == EPI_SWIGLU ? 2 : 1) * ((a.N + 15) / 16);
  const int mt = (a.B + 15) / 16;
  const dim3 grid((a.n_row_tiles + 2 * WR - 1) / (2 * WR), (mt + 2 * WN - 1) / (2 * WN));
  // (the split-K reduce writes row-major, so packed OUTPUTS do not split; packed inputs do)
  static const int pk_split = getenv("MTTS_PK_SPLIT") ? atoi(getenv("MTTS_PK_SPLIT")) : 1;  // A/B
  const int S = (a.y_packed || (a.x_packed && !pk_split)) ? 1 : gemm_splits<WR, WN, 4>(a, (int)grid.x, (int)grid.y);
  if (S > 1) {
    hipLaunchKernelGGL((gemm2_kernel<WR, WN, EPI, 4, true>), dim3(grid.x, grid.y, S), dim3(256), 0, s, a);
    const int n = a.B * ((a.N + 15) / 16) * 4;
#define L_(SS) hipLaunchKernelGGL((gemm_splitk_reduce<EPI, SS>), dim3((n + 255) / 256), dim3(256), 0, s, a, S)
    MTTS_SPLIT_DISPATCH(S, L_);
#undef L_
    return;
  }
  static const int u = getenv("MTTS_GEMM_U") ? atoi(getenv("MTTS_GEMM_U")) : 4;
  if (u == 8 && a.KT % 8 == 0) hipLaunchKernelGGL((gemm2_kernel<WR, WN, EPI, 8>), grid, dim3(256), 0, s, a);
  else if (u >= 4 && a.KT % 4 == 0) hipLaunchKernelGGL((gemm2_kernel<WR, WN, EPI, 4>), grid, dim3(256), 0, s, a);
  else hipLaunchKernelGGL((gemm2_kernel<WR, WN, EPI, 2>), grid, dim3(256), 0, s, a);
}

hipError_t gemm_ex(const GemvArgs& a0, int epi, hipStream_t s) {
  if (a0.K % 32 != 0 || a0.B <= 0 || a0.N <= 0 || a0.ss_in || a0.gate || a0.tile0) return hipErrorInvalidValue;
  GemvArgs a = a0;
  a.KT = a0.K / 32;
  const int n_tiles = (a0.N + 15) / 16;
  static const int big = getenv("MTTS_GEMM_SMALL") && getenv("MTTS_GEMM_SMALL")[0] == '1' ? 1 << 30 : 128;
  // the packed layout is read / written by the 128 x 128 form only
  // (and, from round 5, 33-127 rows: the <= 192-row gemm5 form below; a 120-token prompt's row-major
  // GEMMs had run 12.8 ms against 7.0 for 181 packed ones, profiles/r05_l_*)
  if ((a0.x_packed || a0.y_packed) && ((a0.B < big && (a0.pk_tiles < 3 || a0.pk_tiles > 12)) || a0.K % 64 ||
                                       a0.pk_tiles * 16 < a0.B))
    return hipErrorInvalidValue;
  // packed activations of >= MTTS_GEMM3_MIN token rows: the LDS-staged forms (0: off, A/B).  Round 4
  // took them from 512 rows (gemm3: 724-row prefill 20.5 -> 18.7 ms, profiles/r04_i_*); with the
  // gemm5 forms from 193 (the 4 x 126-row batch prefill ran gemm2_kernel: 13.7 -> 11.1 ms,
  // profiles/r05_r_*)
  static const int g3min = getenv("MTTS_GEMM3_MIN") ? atoi(getenv("MTTS_GEMM3_MIN")) : 193;
  // (and prompts of <= 384 rows: the small forms, MTTS_GEMM3_SMALL tiles, 0: off)
  static const int g3small = getenv("MTTS_GEMM3_SMALL") ? atoi(getenv("MTTS_GEMM3_SMALL")) : 24;
  if (g3min > 0 && a.x_packed && a.pk_tiles > 2 && (a.B >= g3min || a.pk_tiles <= g3small) && a.K % 64 == 0) {
    a.n_row_tiles = (epi == EPI_SWIGLU ? 2 : 1) * n_tiles;
    switch (epi) {
      case EPI_STORE: return gemm3_pick<EPI_STORE>(a, s);
      case EPI_RESADD: return gemm3_pick<EPI_RESADD>(a, s);
      case EPI_SWIGLU: return gemm3_pick<EPI_SWIGLU>(a, s);
      default: return hipErrorInvalidValue;
    }
  }
  if ((a.x_packed || a.y_packed) && a.B < big) return hipErrorInvalidValue;  // (gemm3 small form off)
  if (a.B >= big && a.K % 64 == 0) {  // 128 x 128 block tiles
    switch (epi) {
      case EPI_STORE: gemm2_launch<4, 4, EPI_STORE>(a, s); break;
      case EPI_RESADD: gemm2_launch<4, 4, EPI_RESADD>(a, s); break;
      case EPI_SWIGLU: gemm2_launch<4, 4, EPI_SWIGLU>(a, s); break;
      default: return hipErrorInvalidValue;
    }
    return hipGetLastError();
  }
  switch (epi) {
    case EPI_STORE: gemm_launch<1, EPI_STORE>(a, n_tiles, s); break;
    case EPI_RESADD: gemm_launch<1, EPI_RESADD>(a, n_tiles, s); break;
    case EPI_SWIGLU: gemm_launch<2, EPI_SWIGLU>(a, n_tiles, s); break;
    default: return hipErrorInvalidValue;
  }
  return hipGetLastError();
}

}  // namespace mtts
