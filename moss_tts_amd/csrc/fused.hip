// One launch for a decoder layer's decode attention and its o_proj (B <= 16 rows, one new
// token each): the attention blocks and the o_proj GEMV blocks are roles of the same grid.
//
//   role    = arrival ticket of the block (atomic): tickets [0, n_att) run attn_decode_body
//             (publish-only: every block writes its (m, l, o) split partial, attn_body.h) and
//             count themselves done (agent-scope release); tickets >= n_att are o_proj row tiles
//             (gemv_body<.., EPI_RESADD, PRO_ATTN>): they issue their weight loads at once,
//             wait for the attention count (agent-scope acquire), merge the partials in their
//             prologue (x = softmax-combined attention output) and finish as the o_proj GEMV
//             does (+ residual, + per-16-column sums of squares).
// Roles by ticket, not by blockIdx: a block only ever waits for blocks that took earlier
// tickets, i.e. that are already running, so the grid cannot deadlock whatever the residency.
// The o_proj weight stream (33.6 MB at the 8B shape) overlaps the attention chain instead of
// starting after it, and one dependent-launch boundary per layer disappears.
// The last o_proj block to finish resets the ticket words for the next launch (graph replay).
#include "attn_body.h"
#include "gemv_body.h"

namespace mtts {

constexpr int FUSED_NW = 8;  // waves per block for both roles (attention: 8 x 32 keys)

template <int G, int D>
__global__ __launch_bounds__(FUSED_NW * 64) void attn_oproj_kernel(DecAttnArgs da, GemvArgs go, int* sync, int n_att,
                                                                   int n_o) {
  __shared__ int role_s;
  if (threadIdx.x == 0) role_s = __hip_atomic_fetch_add(&sync[0], 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  __syncthreads();
  const int r = role_s;
  if (r < n_att) {
    const int sp = r % da.ns, rest = r / da.ns;
    attn_decode_body<G, D, FUSED_NW>(da, sp, rest % da.Hkv, rest / da.Hkv);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this wave's partial stores are in L2
    __syncthreads();
    if (threadIdx.x == 0) {
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
      __hip_atomic_fetch_add(&sync[1], 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    return;
  }
  auto wait = [&] {
    if (threadIdx.x == 0) {
      int spins = 0;
      while (__hip_atomic_load(&sync[1], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < n_att && ++spins < (1 << 24))
        __builtin_amdgcn_s_sleep(1);
      if (spins >= (1 << 24)) sync[3] = 1;  // bounded: report a stuck producer instead of hanging
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
    }
    __syncthreads();
  };
  gemv_body<1, 1, EPI_RESADD, PRO_ATTN, FUSED_NW, false>(go, r - n_att, wait);
  __syncthreads();
  if (threadIdx.x == 0) {
    const int done = __hip_atomic_fetch_add(&sync[2], 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (done == n_o - 1) {  // every block has taken its ticket and finished
      sync[0] = 0;
      sync[1] = 0;
      sync[2] = 0;
    }
  }
}

int fused_attn_splits(int Cmax) { return (Cmax + DEC_KW * FUSED_NW - 1) / (DEC_KW * FUSED_NW); }

template <int D>
static hipError_t attn_oproj_d(const DecAttnArgs& da, const GemvArgs& go, int* sync, int n_att, int n_o, int G,
                               hipStream_t s) {
  const size_t lds = (size_t)go.B * go.K * 2;  // the o_proj prologue's merged attention rows
  const dim3 grid(n_att + n_o), blk(FUSED_NW * 64);
  switch (G) {
    case 1: hipLaunchKernelGGL((attn_oproj_kernel<1, D>), grid, blk, lds, s, da, go, sync, n_att, n_o); break;
    case 2: hipLaunchKernelGGL((attn_oproj_kernel<2, D>), grid, blk, lds, s, da, go, sync, n_att, n_o); break;
    case 4: hipLaunchKernelGGL((attn_oproj_kernel<4, D>), grid, blk, lds, s, da, go, sync, n_att, n_o); break;
    case 8: hipLaunchKernelGGL((attn_oproj_kernel<8, D>), grid, blk, lds, s, da, go, sync, n_att, n_o); break;
    default: return hipErrorInvalidValue;
  }
  return hipGetLastError();
}

hipError_t attn_oproj(const DecAttnArgs& da0, const GemvArgs& go0, int* sync, int B, hipStream_t s) {
  DecAttnArgs da = da0;
  GemvArgs go = go0;
  const int G = da.Hq / da.Hkv;
  if (da.Hq % da.Hkv || da.Cmax % 64 || B <= 0 || B > 16 || go.B != B || go.K != da.Hq * da.D || go.K % 32 ||
      (size_t)B * go.K * 2 > NORM_LDS_MAX || !sync)
    return hipErrorInvalidValue;
  da.ns = fused_attn_splits(da.Cmax);
  da.nwv = FUSED_NW;
  da.publish_only = 1;
  da.probe = 0;
  if (da.ns > DEC_MAXS) return hipErrorInvalidValue;
  go.KT = go.K / 32;
  go.pad_period = 1;
  go.attn.part = da.part;
  go.attn.pos = da.pos;
  go.attn.Hkv = da.Hkv;
  go.attn.G = G;
  go.attn.D = da.D;
  go.attn.ns = da.ns;
  go.attn.kb = DEC_KW * FUSED_NW;
  go.attn.po_max = da.po_max = ATTN_PO_ALL;  // every split is published and merged in-launch
  const int n_att = da.ns * da.Hkv * B;
  const int n_o = (go.N + 15) / 16;
  switch (da.D) {
    case 128: return attn_oproj_d<128>(da, go, sync, n_att, n_o, G, s);
    case 64: return attn_oproj_d<64>(da, go, sync, n_att, n_o, G, s);
    case 32: return attn_oproj_d<32>(da, go, sync, n_att, n_o, G, s);
    case 16: return attn_oproj_d<16>(da, go, sync, n_att, n_o, G, s);
    default: return hipErrorInvalidValue;
  }
}

}  // namespace mtts
