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

#include "gemv_body.h"

namespace mtts {

size_t norm_lds_bytes(int B, int K) { return (size_t)(B + 1) * K * 2; }

template <int NB, int RT, int EPI, int PRO, int NW, bool PIPE = false>
__global__ __launch_bounds__(NW * 64) void gemv_kernel(GemvArgs a) {
  if (a.gate) {
    // gated launch (the decode text head, off on most steps): a capped grid walks the tiles, so
    // an off step dispatches a few hundred blocks instead of ~9,500 (7 us of dispatch per step)
    if (*a.gate == 0) return;
    for (int t = blockIdx.x; t < a.gate_tiles; t += gridDim.x) {
      if (t != (int)blockIdx.x) __syncthreads();  // the previous tile's LDS reads are done
      gemv_body<NB, RT, EPI, PRO, NW, PIPE>(a, t + a.tile0, [] {});
    }
    return;
  }
  gemv_body<NB, RT, EPI, PRO, NW, PIPE>(a, (int)blockIdx.x + a.tile0, [] {});
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
// gated launches (gemv_kernel): grid cap, MTTS_GATE_GRID (0: one block per tile; read per launch
// so a test can make the small parity configs walk several tiles per block)
static int gate_grid(int n_tiles) {
  const char* v = getenv("MTTS_GATE_GRID");
  const int cap = v ? atoi(v) : 1024;
  return cap > 0 ? std::min(n_tiles, cap) : n_tiles;
}

template <int NB, int RT, int EPI, int PRO>
static void launch_nw(const GemvArgs& a0, int n_tiles, hipStream_t s) {
  GemvArgs a = a0;
  a.gate_tiles = n_tiles;
  const int grid = a.gate ? gate_grid(n_tiles) : n_tiles;
  constexpr bool NORM = PRO == PRO_NORM || PRO == PRO_NORM_PRE || PRO == PRO_NORM_PREROW || PRO == PRO_NORM_DMA;
  // waves per block from the B=1/B=4 sweep (scripts/sweep_gemv.py, profiles/): 8 for the
  // large matrices (gate|up 6.1 TB/s, heads 7.0 TB/s), 16 for the <= 6144-row ones
  const int rows = n_tiles * RT * 16;
  const size_t lds = PRO == PRO_NORM_DMA ? norm_dma_lds_bytes(a.B, a.K, a.n_ss)
                     : NORM ? norm_lds_bytes(a.B, a.K) : (PRO == PRO_ATTN || PRO == PRO_ATTN_PRE || PRO == PRO_ATTN_PRE2 ? (size_t)a.B * a.K * 2 : 0);
  // 17-32 rows (NB = 2): 4 waves of 4-deep batches (in-context B=32 sweep: 5.62 vs 6.03 ms/step)
  int nw = a.force_nw;
  // fused-norm launches stage (B+1)*K*2 bytes of LDS per block: 8 waves keep 2 blocks per CU
  // (q|k|v: 3.46 vs 3.53 ms/step with 16)
  // packed 17-32 row inputs (one 1 KiB load per x fragment): 8 waves (B=32 4.51 -> 4.44 ms/step)
  if (nw != 4 && nw != 8 && nw != 16)
    nw = a.KT < 64 ? 4 : (NB == 2 ? (a.x_packed ? 8 : 4) : ((rows >= 8192 || a.KT < 128 || NORM) ? 8 : 16));
  // MTTS_GEMV_PIPE bit 0 / bit 1 flips the batch depth (8 <-> 4 k-tiles) for <= 16 / > 16 rows
  static const int pipe = getenv("MTTS_GEMV_PIPE") ? atoi(getenv("MTTS_GEMV_PIPE")) : 0;
  bool u4 = (NB == 1 && (pipe & 1)) || (NB == 2 && !(pipe & 2));
  // gate|up at K <= 2048 (the MossTTSLocal backbone, depth stack and adapters): 4-deep batches,
  // i.e. more resident waves per CU (its roofline GEMV 12.9 -> 11.4 us, frame 9.11 -> 8.66 ms);
  // at K 4096 (MossTTSDelay) the 8-deep batches stay faster (B=4 3.32 vs 3.47 ms/step)
  if (EPI == EPI_SWIGLU && NB == 1 && a.KT <= 64 && !(pipe & 1)) u4 = true;
  if (a.force_u == 4 || a.force_u == 8) u4 = a.force_u == 4;
  if (u4) {
    if (nw == 4) hipLaunchKernelGGL((gemv_kernel<NB, RT, EPI, PRO, 4, true>), dim3(grid), dim3(256), lds, s, a);
    if (nw == 8) hipLaunchKernelGGL((gemv_kernel<NB, RT, EPI, PRO, 8, true>), dim3(grid), dim3(512), lds, s, a);
    if (nw == 16) hipLaunchKernelGGL((gemv_kernel<NB, RT, EPI, PRO, 16, true>), dim3(grid), dim3(1024), lds, s, a);
    return;
  }
  if (nw == 4) hipLaunchKernelGGL((gemv_kernel<NB, RT, EPI, PRO, 4>), dim3(grid), dim3(256), lds, s, a);
  if (nw == 8) hipLaunchKernelGGL((gemv_kernel<NB, RT, EPI, PRO, 8>), dim3(grid), dim3(512), lds, s, a);
  if (nw == 16) hipLaunchKernelGGL((gemv_kernel<NB, RT, EPI, PRO, 16>), dim3(grid), dim3(1024), lds, s, a);
}

// RT = 2 output tiles per block for the plain projections once the x fragments (B rows per
// weight tile) cost as much L2 / TA traffic as the weights: MTTS_GEMV_RT2 = min rows (0: off).
// Only matrices of >= 384 row tiles (q|k|v, the heads): halving the 256-tile o_proj / down
// grids leaves CUs idle (B=16: o 10.1 -> 12.6 us, down 24.4 -> 30.2) while q|k|v gains
// (19.1 -> 16.1 us) and the heads gain most (305 -> 245 us; B=32 451 -> 321 us).
static int rt2_min_rows() {
  static const int v = getenv("MTTS_GEMV_RT2") ? atoi(getenv("MTTS_GEMV_RT2")) : 12;
  return v;
}

template <int RT, int EPI>
static void launch_epi(const GemvArgs& a, int n_tiles, hipStream_t s) {
  if constexpr (RT == 1 && EPI != EPI_SWIGLU) {
    const int m = rt2_min_rows();
    if (m > 0 && a.B >= m && !a.attn.part && !a.gate && a.tile0 == 0 && n_tiles % 2 == 0 && n_tiles >= 384) {
      launch_epi<2, EPI>(a, n_tiles / 2, s);
      return;
    }
  }
  const bool two = a.B > 16;
  if constexpr (EPI == EPI_RESADD) {
    if (a.attn.part) {  // o_proj reading the attention partials (B <= 16)
      // up to two merged elements per thread (B * K / 8 <= 2 x the NW = 16 launch's 1024
      // threads: B <= 4 at K 4096): the partials load before the first weight batch
      // (B=4 o_proj 12.5 us with PRO_ATTN, whose partial loads queue behind the weight batch)
      static const bool no_pre = getenv("MTTS_NO_PRELOAD") && atoi(getenv("MTTS_NO_PRELOAD"));
      const int rows = n_tiles * RT * 16;
      const int nw = (a.force_nw == 4 || a.force_nw == 8 || a.force_nw == 16)
                         ? a.force_nw : (a.KT < 64 ? 4 : ((rows >= 8192 || a.KT < 128) ? 8 : 16));  // = launch_nw's
      if (!no_pre && a.B * a.K / 8 <= nw * 64)
        launch_nw<1, RT, EPI, PRO_ATTN_PRE>(a, n_tiles, s);
      else if (!no_pre && a.B * a.K / 8 <= 2 * nw * 64)  // two elements per thread
        launch_nw<1, RT, EPI, PRO_ATTN_PRE2>(a, n_tiles, s);
      else
        launch_nw<1, RT, EPI, PRO_ATTN>(a, n_tiles, s);
      return;
    }
  }
  const bool norm = a.ss_in != nullptr;
  // batch-1 decode (q|k|v, gate|up at K 4096): the norm prologue's inputs load before the first
  // weight batch (B=1 3.285 -> 3.216 ms/step; MTTS_NO_PRELOAD=1 for A/B)
  static const bool no_pre = getenv("MTTS_NO_PRELOAD") && atoi(getenv("MTTS_NO_PRELOAD"));
  static const bool no_dma = getenv("MTTS_NO_NORM_DMA") && atoi(getenv("MTTS_NO_NORM_DMA"));  // A/B
  if (two) norm ? launch_nw<2, RT, EPI, PRO_NORM>(a, n_tiles, s) : launch_nw<2, RT, EPI, PRO_NONE>(a, n_tiles, s);
  else if (norm && !no_pre && a.B <= PREROW_MAXB && a.K == 4096 && (a.force_nw == 0 || a.force_nw == 8) &&
           norm_lds_bytes(a.B, a.K) <= NORM_LDS_MAX)  // launch_nw gives fused-norm launches 8 waves: K/8 == 512 threads
    launch_nw<1, RT, EPI, PRO_NORM_PREROW>(a, n_tiles, s);
  else if (norm && !no_pre && norm_preload_fits(a.B, a.K)) launch_nw<1, RT, EPI, PRO_NORM_PRE>(a, n_tiles, s);
  else if (norm && !no_pre && !no_dma && a.ldx == a.K && a.ld_ss == a.n_ss &&
           norm_dma_lds_bytes(a.B, a.K, a.n_ss) <= NORM_LDS_MAX)  // contiguous rows: LDS-DMA staging
    launch_nw<1, RT, EPI, PRO_NORM_DMA>(a, n_tiles, s);
  else norm ? launch_nw<1, RT, EPI, PRO_NORM>(a, n_tiles, s) : launch_nw<1, RT, EPI, PRO_NONE>(a, n_tiles, s);
}

// Whether an o_proj of B rows x K reading decode-attention partials (EPI_RESADD, attn.part) would
// load them before its first weight batch with ONE merged element per thread (PRO_ATTN_PRE),
// mirroring launch_epi.  Only then does the merge in o_proj beat letting the attention write its
// rows (same box, profiles/r03_u_ab_local_attn.txt): batch-1 per-op decode 3.191 (merge in o_proj)
// vs 3.223 ms/step; but Delay B = 4 (two elements per thread, PRE2) 3.325 vs 3.262 and
// MossTTSLocal's B = 8 backbone (four, generic PRO_ATTN) 8.52 vs 8.37 ms/frame with the rows written.
bool gemv_attn_preload(int B, int K, int N, int force_nw) {
  static const bool no_pre = getenv("MTTS_NO_PRELOAD") && atoi(getenv("MTTS_NO_PRELOAD"));
  const int KT = K / 32, rows = (N + 15) / 16 * 16;
  const int nw = (force_nw == 4 || force_nw == 8 || force_nw == 16) ? force_nw
                                                                      : (KT < 64 ? 4 : ((rows >= 8192 || KT < 128) ? 8 : 16));
  return !no_pre && (size_t)B * K / 8 <= (size_t)nw * 64;
}

hipError_t gemv_ex(const GemvArgs& a0, int epi, hipStream_t s) {
  if (a0.K % 32 != 0 || a0.B <= 0 || a0.N <= 0) return hipErrorInvalidValue;
  // the packed layout holds 32 token slots and is read by the 2-half (NB = 2) body only
  if ((a0.x_packed || a0.y_packed) && (a0.B <= 16 || a0.B > 32)) return hipErrorInvalidValue;
  if (a0.x_packed && (a0.ss_in || a0.attn.part)) return hipErrorInvalidValue;
  if (a0.ss_in && (a0.n_ss % 4 || a0.ld_ss % 4 || a0.ldx % 8 || norm_lds_bytes(std::min(a0.B, 32), a0.K) > NORM_LDS_MAX))
    return hipErrorInvalidValue;
  if (a0.attn.part && (epi != EPI_RESADD || a0.B > 16 || (size_t)a0.B * a0.K * 2 > NORM_LDS_MAX || a0.attn.D % 8 ||
                       a0.K != a0.attn.Hkv * a0.attn.G * a0.attn.D))
    return hipErrorInvalidValue;
  // the row gather is read by the plain (no-prologue, <= 16 row) body only
  if (a0.xtok && (a0.x_packed || a0.ss_in || a0.attn.part || a0.B > 16 || a0.ld_xtok <= 0)) return hipErrorInvalidValue;
  for (int b0 = 0; b0 < a0.B; b0 += 32) {
    GemvArgs a = a0;
    a.x = a0.xtok ? a0.x : a0.x + (size_t)b0 * a0.ldx;
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
