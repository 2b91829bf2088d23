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

// special token ids and shapes the device-side state machine needs
struct MttsIds {
  int pad, im_start, im_end, audio_start, audio_end, user_slot, gen_slot, delay_slot;
  int audio_pad;  // audio pad code (== audio_vocab)
};
