// Shared device helpers for the MossTTSDelay MI355X (gfx950 / CDNA4) engine.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

typedef uint16_t bf16_t;  // raw bf16 bits in global memory
typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8;
typedef __attribute__((ext_vector_type(4))) float f32x4;
typedef __attribute__((ext_vector_type(4))) unsigned int u32x4;

#define MTTS_WAVE 64

// ---- bf16 <-> f32 --------------------------------------------------------
__device__ __forceinline__ float bf2f(bf16_t b) {
  return __uint_as_float(((uint32_t)b) << 16);
}
// round-to-nearest-even (v_cvt_pk_bf16_f32 on gfx950; NaN stays NaN)
__device__ __forceinline__ bf16_t f2bf(float f) {
  __bf16 h = (__bf16)f;
  return __builtin_bit_cast(bf16_t, h);
}
// round an fp32 value to the nearest bf16 value, staying in fp32
__device__ __forceinline__ float rbf(float f) { return bf2f(f2bf(f)); }

// unpack 8 bf16 from a uint4
__device__ __forceinline__ void unpack8(const uint4 v, float* o) {
  o[0] = __uint_as_float(v.x << 16); o[1] = __uint_as_float(v.x & 0xffff0000u);
  o[2] = __uint_as_float(v.y << 16); o[3] = __uint_as_float(v.y & 0xffff0000u);
  o[4] = __uint_as_float(v.z << 16); o[5] = __uint_as_float(v.z & 0xffff0000u);
  o[6] = __uint_as_float(v.w << 16); o[7] = __uint_as_float(v.w & 0xffff0000u);
}
__device__ __forceinline__ uint32_t pack2(float a, float b) {
  return (uint32_t)f2bf(a) | ((uint32_t)f2bf(b) << 16);
}

// ---- wave reductions (64 lanes) -------------------------------------------
__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}

// argmax with first-index tie break; packs (value, index) comparisons
struct ArgMax {
  float v;
  int i;
};
__device__ __forceinline__ ArgMax am_better(ArgMax a, ArgMax b) {
  // larger value wins; on equal values (or both NaN-free -inf) the lower index wins
  if (b.v > a.v || (b.v == a.v && b.i < a.i)) return b;
  return a;
}
__device__ __forceinline__ ArgMax wave_argmax(ArgMax a) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    ArgMax b;
    b.v = __shfl_xor(a.v, o, 64);
    b.i = __shfl_xor(a.i, o, 64);
    a = am_better(a, b);
  }
  return a;
}

// ---- Philox4x32-10 (counter-based RNG for the multinomial draws) ----------
__device__ __forceinline__ uint32_t mulhilo(uint32_t a, uint32_t b, uint32_t* hi) {
  const uint64_t p = (uint64_t)a * b;
  *hi = (uint32_t)(p >> 32);
  return (uint32_t)p;
}
__device__ __forceinline__ float philox_uniform(unsigned long long seed, uint32_t c0, uint32_t c1, uint32_t c2) {
  uint32_t x0 = c0, x1 = c1, x2 = c2, x3 = 0x5eed;
  uint32_t k0 = (uint32_t)seed, k1 = (uint32_t)(seed >> 32);
#pragma unroll
  for (int r = 0; r < 10; ++r) {
    uint32_t h0, h1;
    const uint32_t l0 = mulhilo(0xD2511F53u, x0, &h0);
    const uint32_t l1 = mulhilo(0xCD9E8D57u, x2, &h1);
    const uint32_t y0 = h1 ^ x1 ^ k0, y1 = l1, y2 = h0 ^ x3 ^ k1, y3 = l0;
    x0 = y0; x1 = y1; x2 = y2; x3 = y3;
    k0 += 0x9E3779B9u; k1 += 0xBB67AE85u;
  }
  return (float)(x0 >> 8) * (1.0f / 16777216.0f);
}

// special token ids and shapes the device-side state machine needs
struct MttsIds {
  int pad, im_start, im_end, audio_start, audio_end, user_slot, gen_slot, delay_slot;
  int audio_pad;  // audio pad code (== audio_vocab)
};
