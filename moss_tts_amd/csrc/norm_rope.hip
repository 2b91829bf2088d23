// Embedding sum, RMSNorm, q/k-norm + RoPE + KV-cache append.
#include <climits>

#include "kernels.h"
#include "qk_item.h"

namespace mtts {

// ---------------------------------------------------------------------------
// h[m, :] = E_text[ids[m,0]] + E_0[ids[m,1]] + ... + E_{n-1}[ids[m,n]], each add rounded to
// bf16 left to right (moss_tts_delay/modeling_moss_tts.py:196-213).
// Grid (M, H/256): a block gathers the C embedding slices of its 256 columns into LDS with
// every 16-byte load in flight at once, then each thread sums one column in channel order.
// It also emits the sum of squares of every 16-column tile for the next RMSNorm.
constexpr int EMB_COLS = 256, EMB_MAXC = 64;
__global__ __launch_bounds__(256) void embed_kernel(const int64_t* __restrict__ ids, int C, const bf16_t* __restrict__ emb_text,
                                                    const bf16_t* __restrict__ emb_audio, int audio_rows, int H,
                                                    bf16_t* __restrict__ h, float* __restrict__ ss_out, int ld_ss,
                                                    int ld_ids) {
  constexpr int LPT = (EMB_MAXC * EMB_COLS / 8 + 255) / 256;  // 16-byte loads per thread (max)
  __shared__ __attribute__((aligned(16))) bf16_t rows_s[EMB_MAXC][EMB_COLS];
  __shared__ int64_t id_s[EMB_MAXC];
  const int m = blockIdx.x, c0 = blockIdx.y * EMB_COLS, t = threadIdx.x;
  if (t < C) id_s[t] = ids[(size_t)m * ld_ids + t];
  __syncthreads();
  const int ncols = min(EMB_COLS, H - c0);
  const int cpr = ncols >> 3;
  const int n = C * cpr;
  uint4 v[LPT];
#pragma unroll
  for (int u = 0; u < LPT; ++u) {
    const int i = t + u * 256;
    if (i < n) {
      const int j = i / cpr, cc = i - j * cpr;
      const bf16_t* src = j == 0 ? emb_text + (size_t)id_s[0] * H : emb_audio + ((size_t)(j - 1) * audio_rows + id_s[j]) * H;
      v[u] = *reinterpret_cast<const uint4*>(src + c0 + cc * 8);
    }
  }
#pragma unroll
  for (int u = 0; u < LPT; ++u) {
    const int i = t + u * 256;
    if (i < n) {
      const int j = i / cpr, cc = i - j * cpr;
      *reinterpret_cast<uint4*>(&rows_s[j][cc * 8]) = v[u];
    }
  }
  __syncthreads();
  float e = 0.f;
  if (t < ncols) {
    e = bf2f(rows_s[0][t]);
    for (int j = 1; j < C; ++j) e = rbf(e + bf2f(rows_s[j][t]));
    h[(size_t)m * H + c0 + t] = f2bf(e);
  }
  float ss = e * e;
  ss += __shfl_xor(ss, 1, 64);
  ss += __shfl_xor(ss, 2, 64);
  ss += __shfl_xor(ss, 4, 64);
  ss += __shfl_xor(ss, 8, 64);
  if (ss_out && t < ncols && (t & 15) == 0) ss_out[(size_t)m * ld_ss + ((c0 + t) >> 4)] = ss;
}

// Prompts (>= EMB_WIDE_MIN rows): no LDS round trip; each thread owns 8 columns of one row and
// walks the C channels with 8 gathers in flight, summing in channel order as above.  (The LDS
// form holds 32 KiB per block for its <= 64 channels: 5 blocks a CU, one load round each; the
// TTSD script's 2,117 x 17-channel prompt took 323 us, ~10x its gather traffic.)
constexpr int EMB_WIDE_MIN = 64, EMB_WCOLS = 256 * 8;
__global__ __launch_bounds__(256) void embed_wide_kernel(const int64_t* __restrict__ ids, int C,
                                                         const bf16_t* __restrict__ emb_text,
                                                         const bf16_t* __restrict__ emb_audio, int audio_rows, int H,
                                                         bf16_t* __restrict__ h, float* __restrict__ ss_out, int ld_ss,
                                                         int ld_ids) {
  const int m = blockIdx.x, col = blockIdx.y * EMB_WCOLS + threadIdx.x * 8;
  const bool ok = col < H;
  const int64_t* idr = ids + (size_t)m * ld_ids;
  float e[8];
  {
    const uint4 v = ok ? *reinterpret_cast<const uint4*>(emb_text + (size_t)idr[0] * H + col) : make_uint4(0, 0, 0, 0);
    unpack8(v, e);
  }
  for (int j0 = 1; j0 < C; j0 += 8) {
    uint4 v[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const int j = j0 + u;
      v[u] = (ok && j < C) ? *reinterpret_cast<const uint4*>(emb_audio + ((size_t)(j - 1) * audio_rows + idr[j]) * H + col)
                           : make_uint4(0, 0, 0, 0);
    }
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      if (j0 + u >= C) break;
      float f[8];
      unpack8(v[u], f);
#pragma unroll
      for (int i = 0; i < 8; ++i) e[i] = rbf(e[i] + f[i]);
    }
  }
  float ss = 0.f;
#pragma unroll
  for (int i = 0; i < 8; ++i) ss += e[i] * e[i];
  ss += __shfl_xor(ss, 1, 64);  // the 16-column tile of lanes 2u, 2u + 1
  if (!ok) return;
  uint4 o;
  o.x = pack2(e[0], e[1]); o.y = pack2(e[2], e[3]); o.z = pack2(e[4], e[5]); o.w = pack2(e[6], e[7]);
  *reinterpret_cast<uint4*>(h + (size_t)m * H + col) = o;
  if (ss_out && (threadIdx.x & 1) == 0) ss_out[(size_t)m * ld_ss + (col >> 4)] = ss;
}

// ---------------------------------------------------------------------------
// Qwen3RMSNorm (TF/models/qwen3/modeling_qwen3.py:59-64): fp32 statistics,
// y = bf16(w * bf16(x * rsqrt(mean(x^2) + eps))).  One block per row.
// Row m of the input is x + x_off + m * x_stride (lets the heads pick the last token).
__global__ __launch_bounds__(256) void rmsnorm_kernel(const bf16_t* __restrict__ x, size_t x_off, size_t x_stride,
                                                      const bf16_t* __restrict__ w, bf16_t* __restrict__ y, int H,
                                                      float eps) {
  const int m = blockIdx.x;
  const bf16_t* xr = x + x_off + (size_t)m * x_stride;
  const int nchunk = H >> 3;
  float ss = 0.f;
  for (int c = threadIdx.x; c < nchunk; c += blockDim.x) {
    float v[8];
    unpack8(*reinterpret_cast<const uint4*>(xr + c * 8), v);
#pragma unroll
    for (int i = 0; i < 8; ++i) ss += v[i] * v[i];
  }
  __shared__ float part[4];
  ss = wave_sum(ss);
  if ((threadIdx.x & 63) == 0) part[threadIdx.x >> 6] = ss;
  __syncthreads();
  const float tot = ((part[0] + part[1]) + part[2]) + part[3];
  const float r = 1.0f / sqrtf(tot / (float)H + eps);
  for (int c = threadIdx.x; c < nchunk; c += blockDim.x) {
    float v[8], g[8];
    unpack8(*reinterpret_cast<const uint4*>(xr + c * 8), v);
    unpack8(*reinterpret_cast<const uint4*>(w + c * 8), g);
    uint4 o;
    float q[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) q[i] = rbf(g[i] * rbf(v[i] * r));
    o.x = pack2(q[0], q[1]); o.y = pack2(q[2], q[3]); o.z = pack2(q[4], q[5]); o.w = pack2(q[6], q[7]);
    *reinterpret_cast<uint4*>(y + (size_t)m * H + c * 8) = o;
  }
}

// ---------------------------------------------------------------------------
// Single-pass Qwen3RMSNorm from the producer's per-16-column sums of squares (written by
// the residual-add GEMV epilogue or the embedding kernel): every wave reduces the row's
// H/16 partials itself (one float4 per lane), so there is no block-wide reduction and x
// is read once.  Block = H/8 threads (one 16-byte chunk each), one block per row.
__global__ __launch_bounds__(512) void rmsnorm_ss_kernel(const bf16_t* __restrict__ x, size_t x_off, size_t x_stride,
                                                         const float* __restrict__ ss, size_t ss_off, size_t ss_stride,
                                                         const bf16_t* __restrict__ w, bf16_t* __restrict__ y, int H,
                                                         float eps, int y_tiles, int M) {
  // packed outputs: the 16 rows of a token tile share its 1-KiB tiles' cache lines, so they go to
  // blocks of one XCD (blocks are dealt round-robin over the 8 XCDs: b and b + 8 share one) and
  // the partial lines merge in that XCD's L2
  const int m = y_tiles ? ((blockIdx.x & 7) + 8 * ((blockIdx.x >> 3) >> 4)) * 16 + ((blockIdx.x >> 3) & 15)
                        : (int)blockIdx.x;
  if (m >= M) return;
  const int lane = threadIdx.x & 63;
  const int c = threadIdx.x;
  const bf16_t* xr = x + x_off + (size_t)m * x_stride;
  uint4 xv = make_uint4(0, 0, 0, 0), wv = make_uint4(0, 0, 0, 0);
  const bool ok = c < (H >> 3);
  if (ok) {
    xv = *reinterpret_cast<const uint4*>(xr + c * 8);
    wv = *reinterpret_cast<const uint4*>(w + c * 8);
  }
  const float* sp = ss + ss_off + (size_t)m * ss_stride;
  float s = 0.f;
  for (int t4 = lane * 4; t4 < (H >> 4); t4 += 256) {
    const float4 v = *reinterpret_cast<const float4*>(sp + t4);
    s += (v.x + v.y) + (v.z + v.w);
  }
  s = wave_sum(s);
  const float r = 1.0f / sqrtf(s / (float)H + eps);
  if (!ok) return;
  float v[8], g[8], q[8];
  unpack8(xv, v);
  unpack8(wv, g);
#pragma unroll
  for (int i = 0; i < 8; ++i) q[i] = g[i] * rbf(v[i] * r);
  uint4 o;
  o.x = pack2(q[0], q[1]); o.y = pack2(q[2], q[3]); o.z = pack2(q[4], q[5]); o.w = pack2(q[6], q[7]);
  *reinterpret_cast<uint4*>(y + (y_tiles ? xpkT_index(m, c * 8, y_tiles) : (size_t)m * H + c * 8)) = o;
}

hipError_t rmsnorm_ss(const bf16_t* x, size_t x_off, size_t x_stride, const float* ss, size_t ss_off, size_t ss_stride,
                      const bf16_t* w, bf16_t* y, int M, int H, float eps, hipStream_t s, int y_tiles) {
  if (H % 16 || H > 4096) return hipErrorInvalidValue;  // one 16-byte chunk per thread, <= 512 threads
  if (y_tiles && (M > 16 * y_tiles || H % 32)) return hipErrorInvalidValue;
  const int threads = ((H / 8 + 63) / 64) * 64;
  const int grid = y_tiles ? 128 * ((M + 127) / 128) : M;
  hipLaunchKernelGGL(rmsnorm_ss_kernel, dim3(grid), dim3(threads < 64 ? 64 : threads), 0, s, x, x_off, x_stride, ss,
                     ss_off, ss_stride, w, y, H, eps, y_tiles, M);
  return hipGetLastError();
}

// ---------------------------------------------------------------------------
// Per-head q_norm / k_norm (TF/.../modeling_qwen3.py:252-254), RoPE in bf16
// (:148-170, cos/sin from a bf16 table computed in fp32, :126-137) and the KV
// cache append (DynamicLayer.update, TF/cache_utils.py:127-145) as an in-place
// write at the token's absolute position.
//
// qkv   [M, (Hq + 2 Hkv) * D] (bf16, output of the fused q|k|v GEMV)
// q_out [M, Hq * D]
// cache k/v: [Bmax][Hkv][Cmax][D] per layer; token m = b*S + s sits at position pos0[b?] + s
// One wave per (token, head); D <= 128, each lane holds dims 2l, 2l+1.

// Prompts of >= QKR_VT_MIN tokens per row append V by 64-token tiles instead (blocks from
// vtile_first on): the transposed V cache [Hkv][D][Cmax] takes a token's 128 values at 128
// different rows, so the per-(token, head) wave wrote 2-byte pieces one cache row apart (at the
// TTSD script's 2,117 tokens the kernel ran 40 us against ~7 us of traffic); a tile goes through
// LDS and leaves as 128-byte runs of one row.
constexpr int QKR_VT_MIN = 64, QKR_VT = 64;
__device__ void v_tile_append(const QKRopeArgs& a, int vb) {
  constexpr int DP = 128 + 8;  // padded LDS row (272 B, 16-B aligned)
  __shared__ __attribute__((aligned(16))) bf16_t tile[QKR_VT][DP];
  const int D = a.D, heads = a.Hq + 2 * a.Hkv;
  const int nst = (a.S + QKR_VT - 1) / QKR_VT;
  const int st = vb % nst, kvh = (vb / nst) % a.Hkv, b = vb / nst / a.Hkv;
  const int s0 = st * QKR_VT, nt = min(QKR_VT, a.S - s0);
  const int cpt = D >> 3;  // 16-byte chunks per token
  for (int i = threadIdx.x; i < nt * cpt; i += blockDim.x) {
    const int j = i / cpt, ch = i - j * cpt;
    const bf16_t* src = a.qkv + ((size_t)b * a.S + s0 + j) * heads * D + (size_t)(a.Hq + a.Hkv + kvh) * D + ch * 8;
    *reinterpret_cast<uint4*>(&tile[j][ch * 8]) = *reinterpret_cast<const uint4*>(src);
  }
  __syncthreads();
  const int p0 = *a.pos_base + s0;
  bf16_t* vrow0 = a.vc + ((size_t)b * a.Hkv + kvh) * D * a.Cmax + p0;
  if (nt == QKR_VT && (p0 & 7) == 0) {
    for (int i = threadIdx.x; i < D * (QKR_VT / 8); i += blockDim.x) {
      const int d = i / (QKR_VT / 8), j0 = (i % (QKR_VT / 8)) * 8;
      uint4 o;
      o.x = (uint32_t)tile[j0][d] | ((uint32_t)tile[j0 + 1][d] << 16);
      o.y = (uint32_t)tile[j0 + 2][d] | ((uint32_t)tile[j0 + 3][d] << 16);
      o.z = (uint32_t)tile[j0 + 4][d] | ((uint32_t)tile[j0 + 5][d] << 16);
      o.w = (uint32_t)tile[j0 + 6][d] | ((uint32_t)tile[j0 + 7][d] << 16);
      *reinterpret_cast<uint4*>(vrow0 + (size_t)d * a.Cmax + j0) = o;
    }
  } else {
    for (int i = threadIdx.x; i < D * nt; i += blockDim.x) {
      const int d = i / nt, j = i - d * nt;
      vrow0[(size_t)d * a.Cmax + j] = tile[j][d];
    }
  }
}

// D = 128 (the 8B / 1.7B heads): four (token, head) items per wave, 16 lanes x 16 bytes each
// (one lane per 2 dims left the 84,700 items of a 2,117-token prompt launch-bound).  Same
// arithmetic as the general form below; rotate_half's partner dims d +- 64 sit 8 lanes away.
__device__ void qk_norm_rope_d128(const QKRopeArgs& a, int wheads) {
  constexpr int D = 128;
  const int lane = threadIdx.x & 63, l16 = lane & 15;
  const int item = (blockIdx.x * 4 + (threadIdx.x >> 6)) * 4 + (lane >> 4);
  const int heads = a.Hq + 2 * a.Hkv;
  const bool live = item < a.M * wheads;
  const int it = live ? item : 0;
  const int m = it / wheads, hd = it % wheads;
  float x[8];
  unpack8(*reinterpret_cast<const uint4*>(a.qkv + (size_t)m * heads * D + (size_t)hd * D + 8 * l16), x);
  qk_item_d128(a, m, hd, l16, x, live);
}

__global__ __launch_bounds__(256) void qk_norm_rope_kernel(QKRopeArgs a, int vtile_first) {
  if ((int)blockIdx.x >= vtile_first) {
    v_tile_append(a, blockIdx.x - vtile_first);
    return;
  }
  if (a.D == 128) {
    qk_norm_rope_d128(a, vtile_first == INT_MAX ? a.Hq + 2 * a.Hkv : a.Hq + a.Hkv);
    return;
  }
  const int lane = threadIdx.x & 63;
  const int gw = blockIdx.x * 4 + (threadIdx.x >> 6);  // global wave = (token, head)
  const int heads = a.Hq + 2 * a.Hkv;
  // (with V tiles the per-wave range stops after the k heads)
  const int wheads = vtile_first == INT_MAX ? heads : a.Hq + a.Hkv;
  if (gw >= a.M * wheads) return;
  const int m = gw / wheads;
  const int hd = gw % wheads;
  const int b = m / a.S, s = m % a.S;
  const int pos = *a.pos_base + s;
  const int rpos = a.rope_off ? max(0, pos - a.rope_off[b]) : pos;  // RoPE position (cache slot: pos)
  const int D = a.D;
  const bool act = 2 * lane < D;
  const bf16_t* src = a.qkv + (size_t)m * heads * D + (size_t)hd * D;
  float x0 = 0.f, x1 = 0.f;
  if (act) {
    const uint32_t pr = *reinterpret_cast<const uint32_t*>(src + 2 * lane);
    x0 = __uint_as_float(pr << 16);
    x1 = __uint_as_float(pr & 0xffff0000u);
  }
  if (hd >= a.Hq + a.Hkv) {  // V head: copy into the cache
    const int kvh = hd - a.Hq - a.Hkv;
    if (act) {  // V cache is stored transposed: [Hkv][D][Cmax]
      bf16_t* dst = a.vc + ((size_t)b * a.Hkv + kvh) * D * a.Cmax + pos;
      dst[(size_t)(2 * lane) * a.Cmax] = f2bf(x0);
      dst[(size_t)(2 * lane + 1) * a.Cmax] = f2bf(x1);
    }
    return;
  }
  const bool isq = hd < a.Hq;
  const bf16_t* nw = isq ? a.qn_w : a.kn_w;
  // RMSNorm over D in fp32
  float ss = wave_sum(x0 * x0 + x1 * x1);
  const float r = 1.0f / sqrtf(ss / (float)D + a.eps);
  float w0 = 0.f, w1 = 0.f;
  if (act) {
    const uint32_t pw = *reinterpret_cast<const uint32_t*>(nw + 2 * lane);
    w0 = __uint_as_float(pw << 16);
    w1 = __uint_as_float(pw & 0xffff0000u);
  }
  const float n0 = rbf(w0 * rbf(x0 * r));
  const float n1 = rbf(w1 * rbf(x1 * r));
  // rotate_half: dims d < D/2 take -x[d + D/2], dims >= D/2 take x[d - D/2]; partner lane = lane +- D/4
  const int q4 = D >> 2;
  const int partner = (2 * lane < D / 2) ? lane + q4 : lane - q4;
  const float p0 = __shfl(n0, partner, 64);
  const float p1 = __shfl(n1, partner, 64);
  const float sg = (2 * lane < D / 2) ? -1.f : 1.f;
  float c0 = 0.f, c1 = 0.f, s0 = 0.f, s1 = 0.f;
  if (act) {
    const uint32_t pc = *reinterpret_cast<const uint32_t*>(a.cos_t + (size_t)rpos * D + 2 * lane);
    const uint32_t ps = *reinterpret_cast<const uint32_t*>(a.sin_t + (size_t)rpos * D + 2 * lane);
    c0 = __uint_as_float(pc << 16); c1 = __uint_as_float(pc & 0xffff0000u);
    s0 = __uint_as_float(ps << 16); s1 = __uint_as_float(ps & 0xffff0000u);
  }
  const float o0 = rbf(rbf(n0 * c0) + rbf(sg * p0 * s0));
  const float o1 = rbf(rbf(n1 * c1) + rbf(sg * p1 * s1));
  if (!act) return;
  if (isq) {
    bf16_t* dst = a.q_out + (size_t)m * a.Hq * D + (size_t)hd * D;
    *reinterpret_cast<uint32_t*>(dst + 2 * lane) = pack2(o0, o1);
  } else {
    const int kvh = hd - a.Hq;
    bf16_t* dst = a.kc + (((size_t)b * a.Hkv + kvh) * a.Cmax + pos) * D;
    *reinterpret_cast<uint32_t*>(dst + 2 * lane) = pack2(o0, o1);
  }
}

hipError_t embed(const int64_t* ids, int C, const bf16_t* emb_text, const bf16_t* emb_audio, int audio_rows, int H,
                 bf16_t* h, int M, hipStream_t s, float* ss_out, int ld_ss, int ld_ids) {
  if (H % 16 || C < 1 || C > EMB_MAXC) return hipErrorInvalidValue;
  if (ld_ids <= 0) ld_ids = C;
  if (M >= EMB_WIDE_MIN) {
    hipLaunchKernelGGL(embed_wide_kernel, dim3(M, (H + EMB_WCOLS - 1) / EMB_WCOLS), dim3(256), 0, s, ids, C, emb_text,
                       emb_audio, audio_rows, H, h, ss_out, ld_ss, ld_ids);
    return hipGetLastError();
  }
  hipLaunchKernelGGL(embed_kernel, dim3(M, (H + EMB_COLS - 1) / EMB_COLS), dim3(256), 0, s, ids, C, emb_text, emb_audio,
                     audio_rows, H, h, ss_out, ld_ss, ld_ids);
  return hipGetLastError();
}

hipError_t rmsnorm(const bf16_t* x, size_t x_off, size_t x_stride, const bf16_t* w, bf16_t* y, int M, int H, float eps,
                   hipStream_t s) {
  if (H % 8) return hipErrorInvalidValue;
  hipLaunchKernelGGL(rmsnorm_kernel, dim3(M), dim3(256), 0, s, x, x_off, x_stride, w, y, H, eps);
  return hipGetLastError();
}

hipError_t qk_norm_rope(const QKRopeArgs& a, hipStream_t s) {
  if (a.D > 128 || a.D % 4) return hipErrorInvalidValue;
  const int per_block = a.D == 128 ? 16 : 4;  // (token, head) items per block
  if (a.S >= QKR_VT_MIN && a.D % 8 == 0) {
    const int qk_blocks = (a.M * (a.Hq + a.Hkv) + per_block - 1) / per_block;
    const int B = a.M / a.S;
    const int v_blocks = B * a.Hkv * ((a.S + QKR_VT - 1) / QKR_VT);
    hipLaunchKernelGGL(qk_norm_rope_kernel, dim3(qk_blocks + v_blocks), dim3(256), 0, s, a, qk_blocks);
  } else {
    const int items = a.M * (a.Hq + 2 * a.Hkv);
    hipLaunchKernelGGL(qk_norm_rope_kernel, dim3((items + per_block - 1) / per_block), dim3(256), 0, s, a, INT_MAX);
  }
  return hipGetLastError();
}

}  // namespace mtts
