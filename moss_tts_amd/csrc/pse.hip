// Persistent streaming engine (PSE): the batch-1 decode step's decoder stack -- every layer's
//   input RMSNorm + q|k|v  ->  attention (q/k norm, RoPE, KV append)  ->  o_proj + residual
//   ->  post-attention RMSNorm + gate|up + SwiGLU  ->  down + residual
// (TF/models/qwen3/modeling_qwen3.py:294-323, :241-280, :81-83) -- as ONE launch, replacing
// run_layers' 5 x 36 dependent launches for B = 1 (MossTTSDelay-8B shape).
//
// Why: at batch 1 each launch pays a dependent-launch boundary and a grid fill / drain
// (~1.7 us between streaming kernels, MI355X_MICROARCH.md "boundary"), and the attention chain
// (~8 us) leaves HBM idle.  Here each CU's weights for the whole step are ONE stream that a
// loader wave keeps running ahead of every data dependency (MI355X_MICROARCH.md
// "prefetch-credit", "engine-vs-launches"): while the consumers wait for a hand-off, the ring
// keeps filling with the next op's weights.
//
// Geometry: one 320-thread workgroup per CU (the LDS request keeps it at one; all P = 256
// resident).  Wave 0 is the LOADER: it streams this CU's weight slices, in op order, through 3
// register buffers (16 B / lane non-temporal loads, counted vmcnt) into an LDS ring of PSE_NS
// 16 KiB slots, and publishes each slot in an LDS FULL counter once it is written.  (Round 2
// filled the ring by LDS-DMA directly; staging through registers keeps the slots in flight out
// of the ring.)  Waves 1-4 are CONSUMERS: each takes 4 of a slot's 16 packed 1 KiB tiles
// (v_mfma_f32_16x16x32_bf16, A = the tile from LDS, B = the op's input vector staged in LDS),
// reports the slot free, and at the end of a row tile the four partial tiles are reduced in LDS
// in a fixed order (deterministic).
//
// Work split per layer (CU c of P = 256): q|k|v = 768 half tiles (row tile, K half), 3 per CU
// (q tile c whole, then one k|v half tile: pse_qkv_unit; an attention CU's k|v half goes to its
// neighbour: pse_nq); o_proj and down = row tile c (CU c owns residual columns 16c..16c+15 for
// the whole step); gate|up = pairs c, c + 256, c + 512 (pse_gu_pair).  92 slots (1.47 MB) per CU
// per layer (88 on the attention CUs, 96 on their helpers).  The attention of KV head g runs on the
// consumers of PSE_AU = 4 CUs (pse_att_unit: unit k takes the cached keys of quarter k for every q
// head of the group, and unit 0 merges its partners' parts, PSE_KSPLIT; before round 6 each of 2 units
// took 2 q heads over every key), whose loaders keep streaming through it (PSE_APAUSE; paused until
// round 6).  The loader stages slots through registers (PSE_RLOAD).  The engine takes this launch only for contexts up to its PSE range
// (engine.cpp pse_choose).
//
// Hand-offs: data-tagged granules (MI355X_MICROARCH.md "handoff-1to1" / "allgather"): 8 bytes
// {32-bit payload, 32-bit tag} written by ONE write-through (sc1) store and read with sc1 loads;
// tag = launch epoch << 8 | layer * 5 + op, so a consumer polls the payload itself (no counters,
// no fences) and granules of earlier launches / layers never match.  Every spin is bounded: a
// stuck wait sets the error word, and the launch drains.
#include "kernels.h"
#include "pse_chunk.h"

namespace mtts {

namespace {

constexpr int CW = 4;                   // consumer waves
#ifndef PSE_LW
#define PSE_LW 1
#endif
constexpr int LW = PSE_LW;              // loader waves
static_assert(LW == 1, "the register-staged loader publishes one FULL counter");
constexpr int THREADS = (LW + CW) * 64;
#ifndef PSE_POLL_SLEEP
#define PSE_POLL_SLEEP 1  // s_sleep count between a gather's sweeps (x 64 cycles)
#endif
#ifndef PSE_GPRIO
#define PSE_GPRIO 1  // consumer waves raise their issue priority while gathering
#endif
#ifndef PSE_LPRIO
#define PSE_LPRIO 0
#endif
#ifndef PSE_PPRIO
#define PSE_PPRIO 1  // consumer waves raise their issue priority over each op's publish
#endif
#define PSE_PRIO_UP() do { if (PSE_PPRIO) __builtin_amdgcn_s_setprio(3); } while (0)
#define PSE_PRIO_DOWN() do { if (PSE_PPRIO) __builtin_amdgcn_s_setprio(0); } while (0)
#ifndef PSE_CSLEEP
#define PSE_CSLEEP 0  // s_sleep of a consumer waiting for a ring slot
#endif
// PSE_APAUSE: the short form's attention CUs pause their loader -- 2 through the whole attention, 1 until the q
// rows are in, 0 never (round 6 default: with the key-split units' quarter of the K / V reads, the stream
// running on through the attention measured faster, 2.588-2.592 -> 2.564-2.570 ms/step).  The long form's
// slices always pause it.
#ifndef PSE_APAUSE
#define PSE_APAUSE 0
#endif
#ifndef PSE_RC
#define PSE_RC 7  // ring slots a plain CU's consumer waves drain into registers during the attention wait
#endif
#ifndef PSE_TRACE2
#define PSE_TRACE2 0  // (diagnostic: the input-norm h gather's own stamps replace the loader's)
#endif
#ifndef PSE_HCNT
// the residual hand-offs (h after o_proj / down: 2,304 tagged granules swept by every consumer CU)
// as counter + direct load: producers store the bf16 row write-through and bump a per-layer
// counter; each consumer wave polls it, then loads exactly its two 8-column groups and the 256
// sums of squares in one round of 16-byte sc1 loads and normalises them (no consumer barrier)
#define PSE_HCNT 0
#endif
// PSE_HTREE (with PSE_HCNT): the 256 arrivals counted in two levels, 8 group counters (32 CUs each,
// one 128-byte line each) whose completing arrival bumps the hand-off's counter (pse4.hip PSE4_HTREE)
#ifndef PSE_HTREE
#define PSE_HTREE 1
#endif
constexpr int HGRP = 8, GCNT_STRIDE = 32;
#ifndef PSE_LONG_RESUME
// long form: every CU's loader pauses while its slice reads K / V (the reads would queue behind the
// weight fills); 1: it resumes as soon as the slice's chunks are scored (the partial hop, the merge
// and the o gather then overlap the stream again), 0: after the whole attention phase
#define PSE_LONG_RESUME 0
#endif
#ifndef PSE_NS
#define PSE_NS 8
#endif
constexpr int NS = PSE_NS;              // ring slots
constexpr int SLOT_KB = 16;             // 1 KiB tiles per slot
constexpr int H_ = 4096, HQ_ = 32, HKV_ = 8, D_ = 128, I_ = 12288, QKVR_ = 6144;
enum { OP_QKV = 0, OP_ATT = 1, OP_O = 2, OP_GU = 3, OP_DOWN = 4 };

typedef __attribute__((address_space(1))) uint64_t g64;
typedef __attribute__((address_space(1))) uint32_t g32;
typedef __attribute__((address_space(3))) void lvoid;
typedef __attribute__((address_space(1))) void gvoid;

__device__ __forceinline__ void st64(void* p, uint64_t v) {
  __hip_atomic_store((g64*)p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ uint32_t ld32(const void* p) {
  return __hip_atomic_load((g32*)p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void st32(void* p, uint32_t v) {
  __hip_atomic_store((g32*)p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
// trace events (PSE_TRACE_EV per layer): consumers (wave 1) 0 layer start, 1 q|k|v input
// normed, 2 q|k|v done, 3 attention done (attention CUs), 4 o input, 5 o done, 6 gate|up input
// normed, 7 gate|up done, 8 down input, 9 down done; loader 10 first q|k|v slot issued, 11 first
// o slot, 12 first gate|up slot, 13 first down slot, 14 last slot of the layer issued;
// attention CUs 15 q|k|v gathered, 16 chunks start, 17 chunks done, 18 other units' partials in
#define PSE_STAMP(l, ev)                                                                        \
  do {                                                                                          \
    if (a.trace && lane == 0) a.trace[((size_t)(l) * PSE_TRACE_EV + (ev)) * 256 + c] = __builtin_amdgcn_s_memrealtime(); \
  } while (0)
__device__ __forceinline__ uint64_t gran(uint32_t payload, uint32_t tag) { return (uint64_t)tag << 32 | payload; }
__device__ __forceinline__ uint32_t tagof(uint32_t epoch, int l, int op) { return epoch << 8 | (uint32_t)(l * 5 + op); }

// q|k|v unit j of CU c: (row tile, K half) -- both halves of q row tile c, then (j = 2) half c & 1
// of k|v row tile 256 + c / 2, and (j = 3, the helper CUs of pse_nq) the k|v half tile of CU
// c + 1.  Every q tile is complete two thirds into the q|k|v stream, so the attention units start
// on q while k / v are still being produced (round 3; units 3c .. 3c+2 in (tile, half) order
// before: 2.824 -> 2.804 ms/step).
__device__ __forceinline__ void pse_qkv_unit(int c, int j, int* t, int* half) {
  const int o = j == 3 ? c + 1 : c;
  *t = j < 2 ? c : HQ_ * D_ / 16 + (o >> 1);
  *half = j < 2 ? j : (o & 1);
}
// gate|up pair of CU c in round j (3 pairs per CU): round j of every CU makes the SwiGLU columns
// [4096 j, 4096 j + 4096), i.e. down_proj's k range of its slots 8j .. 8j+7, so every round's
// hand-off flies while earlier rounds' work runs (the consumers below; round 3, pairs 3c .. 3c+2
// before: 2.981 -> 2.842 ms/step)
__device__ __forceinline__ int pse_gu_pair(int c, int j) { return c + 256 * j; }
// slot s's 16 KiB: (layer, op, unit, k range) -> 16 contiguous packed 1 KiB tiles of CU c, which
// runs nq q|k|v units (pse_nq): 4 nq + 80 slots per layer
__device__ __forceinline__ const bf16_t* pse_slot_src(const bf16_t* const* wp, int c, int nq, int s) {
  const int spl = 4 * nq + 80, l = s / spl, r = s - l * spl, rq = 4 * nq;
  if (r < rq) {  // q|k|v: unit r / 4 of CU c = (row tile, K half), 4 slots each
    int t, half;
    pse_qkv_unit(c, r / 4, &t, &half);
    return wp[l * 4 + 0] + ((size_t)t * 128 + half * 64 + (r % 4) * 16) * 512;
  } else if (r < rq + 8) {  // o_proj row tile c, 8 slots
    return wp[l * 4 + 1] + ((size_t)c * 128 + (r - rq) * 16) * 512;
  } else if (r < rq + 56) {  // gate|up pairs (round j = 0..2: pair pse_gu_pair(c, j)): gate tile (8 slots), then up tile (8)
    const int q = r - rq - 8, pr = pse_gu_pair(c, q / 16), rt = 2 * pr + (q % 16) / 8;
    return wp[l * 4 + 2] + ((size_t)rt * 128 + (q % 8) * 16) * 512;
  }
  return wp[l * 4 + 3] + ((size_t)c * 384 + (r - rq - 56) * 16) * 512;  // down row tile c, 24 slots
}

// LDS words shared by the loader and the consumers
struct Ctl {
  int full[LW];   // per loader wave k: its slots (k, k + LW, ...) whose DMA has retired
  int freed[CW];  // slots each consumer wave has finished reading
  int bar;        // consumer-only barrier counter (monotonic)
  int abort;      // a wait gave up: everyone drains
  int apause;     // attention gathering its inputs: the loader issues nothing
  uint64_t lstamp[2][5];  // loader trace events of the last two layers (copied out by the consumers)
};

constexpr uint32_t SPIN_LDS = 1u << 22;  // LDS polls (~40 ns each): ~0.2 s
constexpr uint32_t SPIN_MEM = 1u << 18;  // granule sweeps (~1-2 us each): ~0.3-0.5 s

// LDS layout (bytes)
constexpr int L_CTL = 0;
constexpr int L_RING = 256;
constexpr int L_XS = L_RING + NS * SLOT_KB * 1024;  // op input: 12288 bf16
constexpr int L_RED = L_XS + I_ * 2;                // [CW][2][16] fp32: column 0 of the partial tiles
constexpr int L_MISC = L_RED + CW * 2 * 16 * 4;     // [256] gathered sums of squares
constexpr int PSE_MAXL = 64;                        // layers (weight pointer table in LDS)
// counters (ints from a.hcnt): [2 PSE_MAXL] hand-off counters, the release flags (PSE_HCNT 2), then
// the group counters (PSE_HTREE)
constexpr size_t HCNT_GC_OFF = (2 * PSE_MAXL * 4 + (PSE_HCNT == 2 ? (size_t)2 * PSE_MAXL * 256 * 128 : 0)) / 4;
constexpr int L_PTR = L_MISC + 1024;
constexpr int L_END = L_PTR + PSE_MAXL * 4 * 8;
// the attention CUs' scratch overlays the op input (q|k|v's input is dead once its slots are
// consumed; o_proj's gather rewrites it after the attention): gathered q|k|v halves, then
// q_s [16][D] bf16, k_s / v_s [D], p_s [CW][16][32] bf16, ml_s [CW][G][2], acc_s [CW][G][D]
constexpr int G_ = HQ_ / HKV_;
constexpr int L_GRAW = L_XS;
constexpr int L_ATT = L_GRAW + 1536 * 4;
static_assert(L_ATT + 16 * D_ * 2 + 2 * D_ * 4 + CW * 16 * 32 * 2 + CW * G_ * 2 * 4 + CW * G_ * D_ * 4 <= L_RED,
              "attention scratch fits the op input region");
static_assert(L_END <= 160 * 1024, "LDS");
// (long form) the merge unit's 32 slice partials (2,112 words) over the slice's p_s / ml_s / acc_s
static_assert(L_ATT + 16 * D_ * 2 + 2 * D_ * 4 + 2112 * 4 <= L_RED, "merge partials fit the op input region");

}  // namespace

size_t pse_lds_bytes() { return (size_t)L_END; }
// Attention units: PSE_AU per KV head, each G / PSE_AU of the head's q heads over every key
// (attention() below).  Unit index u = g * PSE_AU + k runs on CU P - 1 - 7 u (spread over the
// XCDs under round-robin placement); -1: no attention unit.
#ifndef PSE_AU
#define PSE_AU 4
#endif
// PSE_KSPLIT (round 6, default): the two units of a KV head split its cached keys -- unit k takes the
// 32-key chunks of half k for all G q heads -- instead of its q heads (every key, G / 2 heads each).  A
// unit is bound by the K / V bytes its CU pulls in (~200 KB at 390 keys, ~50 GB/s per CU), which the
// key split halves.  The pair merges itself: unit 1 (no k / v gather, no new key) publishes its
// unnormalised rows (fp32) and its (max, sum) per head (KS_N granules per KV head, in the long form's
// partial buffer, which the short form does not use), and unit 0 folds them into its own merge with
// the new key, so the o_proj gather keeps its 2,048 granules.  0: the head split.
#ifndef PSE_KSPLIT
#define PSE_KSPLIT 1
#endif
static_assert(!PSE_KSPLIT || PSE_AU == 2 || PSE_AU == 4, "key split: 2 or 4 units per KV head");
// a KV head's partials in the long form's buffer: the rows of units 1 .. AU-1 ([AU-1][G][D] fp32), then their
// (max, sum) per head ([AU-1][G][2]); unit 0 gathers them as one range (rows -> graw, the rest -> L_MISC)
constexpr int KS_ROWS = G_ * D_, KS_N = (PSE_AU - 1) * (G_ * D_ + 2 * G_);
static_assert(!PSE_KSPLIT || ((PSE_AU - 1) * KS_ROWS % 256 == 0 && (PSE_AU - 1) * KS_ROWS <= 1536),
              "the partners' rows fill whole gather rounds and fit graw");
constexpr int NG_ATT = HQ_ * D_ / 2;  // attention output granules
__host__ __device__ inline int pse_att_unit(int c, int P) {
  const int d = P - 1 - c;
  return (d >= 0 && d % 7 == 0 && d / 7 < HKV_ * PSE_AU) ? d / 7 : -1;
}
// q|k|v units of CU c: an attention CU runs only its q tile (2 units) and hands its k|v half tile
// to CU c - 1 (4 units): the attention needs k / v only after its cached-key chunks, so the
// helper's later finish costs nothing, and the attention CU, whose loader pauses through the
// attention, starts the layer's later ops 4 slots less behind the others.  3 units elsewhere.
__host__ __device__ inline int pse_nq(int c, int P) {
  return pse_att_unit(c, P) >= 0 ? 2 : (pse_att_unit(c + 1, P) >= 0 ? 4 : 3);
}

namespace {

// the launch's LDS, visible by name in every helper so that the compiler addresses it as LDS
// (ds_read / ds_write); an LDS pointer carried through a struct degrades to flat accesses
extern __shared__ __attribute__((aligned(16))) unsigned char pse_lds[];
#define PSE_CTL (reinterpret_cast<Ctl*>(pse_lds + L_CTL))

struct Ctx {
  uint32_t* err;  // the launch's error word
  float eps;
  int probe;
  int c, lane, wave, tid;
  uint32_t epoch;
  int bar_gen;
#if PSE_TRACE2
  uint64_t* tp;  // (PSE_TRACE2: gather stamps of the input-norm h gather into events 10-14)
#endif
};

__device__ __forceinline__ bool failed(const Ctx& x) {
  return __hip_atomic_load(&PSE_CTL->abort, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) != 0;
}
__device__ __forceinline__ void give_up(Ctx& x, uint32_t code) {
  st32(x.err, code);
  __hip_atomic_store(&PSE_CTL->abort, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}

// consumer-only barrier (the loader never joins): a monotonic LDS counter
__device__ __forceinline__ void cbar(Ctx& x) {
  x.bar_gen += CW;
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
  if (x.lane == 0) __hip_atomic_fetch_add(&PSE_CTL->bar, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
  uint32_t spins = 0;
  while (__hip_atomic_load(&PSE_CTL->bar, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) < x.bar_gen) {
    if (++spins > SPIN_LDS) {
      give_up(x, 4);
      break;
    }
    __builtin_amdgcn_s_sleep(0);
  }
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
}

// Gather n consecutive granules g[0..n) carrying tag t into LDS: the first n0 payloads to
// dst0, the rest to dst1; all consumer threads cooperate (n <= MAXP * 256) in ONE sweep loop (one
// round trip per poll), calling each_poll() after every sweep's results are in; false on timeout / abort.  Branch-free sc1 buffer loads (an out-of-range
// offset reads zero): a load under a divergent branch would be waited for at once.  SYNC: a
// consumer barrier at the end, for data one wave gathers and another reads (the sums of squares,
// the attention's rows); without it each wave goes on with the granules tid + 256 k it gathered
// itself -- exactly the columns its consume_slot tiles read (norm_grp)
template <bool B>
struct BoolC {
  static constexpr bool value = B;
};
template <int V>
struct IntC {
  static constexpr int value = V;
};
struct NoHook {
  __device__ void operator()() const {}
};
template <int MAXP, bool SYNC = true, typename Hook = NoHook, typename Poll = NoHook>
__device__ __forceinline__ bool gather(Ctx& x, const uint64_t* g, int n, uint32_t t, uint32_t* dst0, int n0,
                                       uint32_t* dst1 = nullptr, const Hook& after_first_issue = Hook(),
                                       const Poll& each_poll = Poll()) {
  constexpr uint32_t OOB = 0x7ffffff0u;
  const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(const_cast<uint64_t*>(g), 0, n * 8, 0x00020000);
  uint32_t pend = 0;  // bit i: granule tid + i * 256 not seen yet
#pragma unroll
  for (int i = 0; i < MAXP; ++i)
    if (x.tid + i * CW * 64 < n) pend |= 1u << i;
  // the first sweep, then the caller's own loads (independent of the granules: they queue
  // behind the sweep instead of delaying it, and the sweep's results are waited for alone)
  if (PSE_GPRIO) __builtin_amdgcn_s_setprio(3);  // sweeps issue ahead of the loader's fills
  bool ok = true;
  uint32_t lo[MAXP], hi[MAXP];
  // one lane offset (tid * 8) for every granule i: i's 2 KiB stride rides in the SGPR offset, so a
  // gather site keeps no per-granule offset registers live across its poll loop (pse4.hip's form)
  const uint32_t vo = (uint32_t)x.tid * 8u;
  auto issue = [&]() {
#pragma unroll
    for (int i = 0; i < MAXP; ++i) {
      const auto v = __builtin_amdgcn_raw_buffer_load_b64(rs, (pend >> i & 1u) ? vo : OOB, i * CW * 64 * 8, 16 /* sc1 */);
      lo[i] = v[0];
      hi[i] = v[1];
    }
  };
  auto take = [&]() {
#pragma unroll
    for (int i = 0; i < MAXP; ++i)
      if ((pend >> i & 1u) && hi[i] == t) {
        // (every caller's n0 is a multiple of 256: granule i of every thread goes to the same
        // destination, a wave-uniform branch instead of a per-lane pointer select)
        const int j = x.tid + i * CW * 64;
        if (i * CW * 64 < n0) dst0[j] = lo[i];
        else dst1[j - n0] = lo[i];
        pend &= ~(1u << i);
      }
  };
  // the first sweep and the caller's work outside the poll loop (a hook inside it would share
  // the loop's register allocation: the attention's chunk loop spilled there)
#if PSE_TRACE2
#define PSE_T2(ev, v) do { if (x.tp && x.wave == LW && x.lane == 0) x.tp[((ev) - 10) * 256] = (v); } while (0)
#else
#define PSE_T2(ev, v) do { } while (0)
#endif
  issue();
  PSE_T2(10, __builtin_amdgcn_s_memrealtime());
  after_first_issue();
  take();
  each_poll();
  PSE_T2(14, __builtin_amdgcn_s_memrealtime());
  uint32_t sweeps = 1;
  for (uint32_t spins = 1; __any(pend != 0); ++spins, ++sweeps) {
    if (spins > SPIN_MEM || ((spins & 255) == 255 && (failed(x) || ld32(x.err)))) {
      give_up(x, 2);
      ok = false;
      break;
    }
    __builtin_amdgcn_s_sleep(PSE_POLL_SLEEP);
    issue();
    take();
    each_poll();
  }
  if (PSE_GPRIO) __builtin_amdgcn_s_setprio(PSE_GPRIO == 2 ? 2 : 0);
  PSE_T2(11, __builtin_amdgcn_s_memrealtime());
  PSE_T2(13, (uint64_t)sweeps);
  if (SYNC) {
    cbar(x);
  } else {  // the wave reads back only what its own lanes stored
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  }
  PSE_T2(12, __builtin_amdgcn_s_memrealtime());
  (void)sweeps;
  return ok && !failed(x);
}

// q|k|v partial granules grouped by KV head: group g = the q tiles of heads G g .. G g + G - 1,
// then k tile rows of head g, then v (48 tiles x 2 K halves x 16 rows), so the attention of head
// g gathers one contiguous range.  Row tile t of the q|k|v matrix -> its granule base.
__device__ __forceinline__ int qkv_gran(int t) {
  constexpr int TPH = D_ / 16, G = HQ_ / HKV_, GT = (G + 2) * TPH;  // tiles per head, per group
  int g, o;
  if (t < HQ_ * TPH) { g = t / (G * TPH); o = t - g * G * TPH; }
  else if (t < (HQ_ + HKV_) * TPH) { g = (t - HQ_ * TPH) / TPH; o = G * TPH + (t - HQ_ * TPH - g * TPH); }
  else { g = (t - (HQ_ + HKV_) * TPH) / TPH; o = (G + 1) * TPH + (t - (HQ_ + HKV_) * TPH - g * TPH); }
  return (g * GT + o) * 32;
}

// Qwen3RMSNorm of the staged vector in place (TF/.../modeling_qwen3.py:59-64):
// xs = bf16(w * bf16(h * r)), r = 1 / sqrt(sum(ss) / K + eps), ss = the producers' per-16-column
// sums of squares (n_ss of them, summed in a fixed order by every wave).  The weights w arrive in
// registers: loaded behind the gather's first sweep, so their latency (a global load queued
// behind the loader's fills) overlaps the hand-off instead of following it
// The staged 4096-column vector in 8-column groups (u32x4 index i): consumer wave w reads k-tiles
// t (32 columns) with t % 16 in [4w, 4w + 4) -- consume_slot's kt0 + 4w + i -- i.e. groups i with
// i % 64 in [16w, 16w + 16), and the gathers (granule tid + 256 k -> columns 2 granule, 2 granule
// + 1) write exactly those columns from the same wave.  norm_grp(x, j): this thread's group j of 2.
__device__ __forceinline__ int norm_grp(const Ctx& x, int j) {
  return 64 * ((x.lane >> 4) + 4 * j) + 16 * (x.wave - LW) + (x.lane & 15);
}
// the norm weights of this thread's two groups
struct NormW {
  u32x4 a, b;
};
__device__ __forceinline__ NormW norm_w(const Ctx& x, const bf16_t* w) {
  const u32x4* wv = reinterpret_cast<const u32x4*>(w);
  return NormW{wv[norm_grp(x, 0)], wv[norm_grp(x, 1)]};
}
// Each wave normalises only the columns it gathered and will consume: no barrier after the norm
// (the sums of squares, gathered across the waves, are behind the gather's barrier)
__device__ void norm_stage(Ctx& x, bf16_t* xs, const float* ss, int n_ss, NormW nw) {
  constexpr int K = H_;
  static_assert(K / 8 == 2 * CW * 64 && CW == 4, "two 8-column groups per consumer thread");
  // (as the GEMV's norm prologue sums them: 4 per lane, then across the wave; n_ss <= 256)
  float s = 0.f;
  if (4 * x.lane < n_ss) s = (ss[4 * x.lane] + ss[4 * x.lane + 1]) + (ss[4 * x.lane + 2] + ss[4 * x.lane + 3]);
  s = wave_sum(s);
  const float r = 1.0f / sqrtf(s / (float)K + x.eps);
  u32x4* xv = reinterpret_cast<u32x4*>(xs);
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const int i = norm_grp(x, j);
    const u32x4 hv = xv[i], nv = j ? nw.b : nw.a;
    u32x4 o;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const float h0 = __uint_as_float(hv[q] << 16), h1 = __uint_as_float(hv[q] & 0xffff0000u);
      const float w0 = __uint_as_float(nv[q] << 16), w1 = __uint_as_float(nv[q] & 0xffff0000u);
      o[q] = pack2(w0 * rbf(h0 * r), w1 * rbf(h1 * r));
    }
    xv[i] = o;
  }
  // this wave's own LDS writes are read back by its own lanes only (consume_slot)
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// PSE_HCNT: wait for the P producers of hand-off k (hcnt[k]), then load this thread's two groups
// of the residual row hb and the 256 sums of squares hs (4 per lane: the sum in norm_stage's
// order) and normalise the groups into xs; `hook` runs before the poll
template <typename Hook>
__device__ __forceinline__ bool hnorm_counter(Ctx& x, const int* hcnt, const uint32_t* go, int k, const bf16_t* hb, const float* hs,
                                              bf16_t* xs, const Hook& hook, NormW& nw) {
  hook();
  if (PSE_GPRIO) __builtin_amdgcn_s_setprio(3);
  // (PSE_HCNT 2: this CU's own release flag line; 1: the counter line every consumer wave polls)
  for (uint32_t spins = 0;
       PSE_HCNT == 2 ? ld32(go + ((size_t)k * 256 + x.c) * 32) != x.epoch : (int)ld32(hcnt + k) < (PSE_HTREE ? HGRP : 256);
       ++spins) {
    if (spins > SPIN_MEM || ((spins & 255) == 255 && (failed(x) || ld32(x.err)))) {
      give_up(x, 2);
      if (PSE_GPRIO) __builtin_amdgcn_s_setprio(0);
      return false;
    }
    __builtin_amdgcn_s_sleep(PSE_POLL_SLEEP);
  }
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");  // (every read below is an sc1 load)
  const __amdgpu_buffer_rsrc_t hrs = __builtin_amdgcn_make_buffer_rsrc(const_cast<bf16_t*>(hb), 0, H_ * 2, 0x00020000);
  const __amdgpu_buffer_rsrc_t srs = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(hs), 0, (H_ / 16) * 4, 0x00020000);
  const u32x4 h0 = __builtin_amdgcn_raw_buffer_load_b128(hrs, (uint32_t)norm_grp(x, 0) * 16u, 0, 16 /* sc1 */);
  const u32x4 h1 = __builtin_amdgcn_raw_buffer_load_b128(hrs, (uint32_t)norm_grp(x, 1) * 16u, 0, 16);
  const u32x4 sv = __builtin_amdgcn_raw_buffer_load_b128(srs, (uint32_t)x.lane * 16u, 0, 16);
  if (PSE_GPRIO) __builtin_amdgcn_s_setprio(0);
  const float s = wave_sum((__uint_as_float(sv[0]) + __uint_as_float(sv[1])) + (__uint_as_float(sv[2]) + __uint_as_float(sv[3])));
  const float r = 1.0f / sqrtf(s / (float)H_ + x.eps);
  u32x4* xv = reinterpret_cast<u32x4*>(xs);
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const u32x4 hv = j ? h1 : h0, wv = j ? nw.b : nw.a;
    u32x4 o;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const float x0 = __uint_as_float(hv[q] << 16), x1 = __uint_as_float(hv[q] & 0xffff0000u);
      const float w0 = __uint_as_float(wv[q] << 16), w1 = __uint_as_float(wv[q] & 0xffff0000u);
      o[q] = pack2(w0 * rbf(x0 * r), w1 * rbf(x1 * r));
    }
    xv[norm_grp(x, j)] = o;
  }
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  return !failed(x);
}

// This consumer wave's 4 tiles of ring slot `seq`: acc += W_tiles . x over k tiles kt0 + 4w ..
// (B operand = the staged vector: every MFMA column the same, column 0 is kept)
__device__ __forceinline__ void consume_slot(Ctx& x, int seq, int kt0, f32x4& acc) {
  for (uint32_t spins = 0;
       __hip_atomic_load(&PSE_CTL->full[seq % LW], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) <= seq / LW;
       ++spins) {
    if (spins > SPIN_LDS || failed(x)) {
      give_up(x, 3);
      return;
    }
    __builtin_amdgcn_s_sleep(PSE_CSLEEP);
  }
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
  if (x.probe == 2) {
    if (x.lane == 0) __hip_atomic_store(&PSE_CTL->freed[x.wave - LW], seq + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    return;
  }
  const u32x4* sl = reinterpret_cast<const u32x4*>(pse_lds + L_RING + (seq % NS) * SLOT_KB * 1024);
  const u32x4* xv = reinterpret_cast<const u32x4*>(pse_lds + L_XS);
  const int w = x.wave - LW;
  u32x4 wt[4], xb[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int t = w * 4 + i;
    wt[i] = sl[t * 64 + x.lane];
    xb[i] = xv[(kt0 + t) * 4 + (x.lane >> 4)];
  }
  // the slot's bytes are in registers: release it to the loader
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  if (x.lane == 0) __hip_atomic_store(&PSE_CTL->freed[w], seq + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
#pragma unroll
  for (int i = 0; i < 4; ++i)
    acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, wt[i]), __builtin_bit_cast(bf16x8, xb[i]),
                                                  acc, 0, 0, 0);
}

// The ring slot drain (plain CUs, PSE_RC > 0): while a consumer wave waits for an op's input,
// it copies the op's next ring slots (its 4 tiles of each) into registers as they land and
// releases them, so the loader streams that many slots further ahead through the wait; the op
// then runs those slots from the registers.  rc_drain_one: slot seq (if it has landed) -> t[]
__device__ __forceinline__ bool slot_ready(int seq) {
  return __hip_atomic_load(&PSE_CTL->full[seq % LW], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) > seq / LW;
}
__device__ __forceinline__ void slot_take(Ctx& x, int seq, u32x4 (&t)[4]) {
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
  const u32x4* sl = reinterpret_cast<const u32x4*>(pse_lds + L_RING + (seq % NS) * SLOT_KB * 1024);
  const int w = x.wave - LW;
#pragma unroll
  for (int i = 0; i < 4; ++i) t[i] = sl[(w * 4 + i) * 64 + x.lane];
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  if (x.lane == 0) __hip_atomic_store(&PSE_CTL->freed[w], seq + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}
// acc += this wave's 4 tiles t[] (a drained slot) . x over k tiles kt0 + 4w ..
__device__ __forceinline__ void slot_mfma(Ctx& x, const u32x4 (&t)[4], int kt0, f32x4& acc) {
  const u32x4* xv = reinterpret_cast<const u32x4*>(pse_lds + L_XS);
  const int w = x.wave - LW;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const u32x4 xb = xv[(kt0 + w * 4 + i) * 4 + (x.lane >> 4)];
    acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, t[i]), __builtin_bit_cast(bf16x8, xb), acc,
                                                  0, 0, 0);
  }
}

// RC ring slots drained into registers (slot_take) during an op's input gather, one per call of
// drain() as they land; take(i, ..): the op's i-th slot from the registers (i < nd) or the ring.
// One instance per op, scoped to it, so the registers are live only from the gather to the op.
template <int RC>
struct SlotCache {
  u32x4 rc[RC > 0 ? RC : 1][4];
  int nd = 0;
  __device__ __forceinline__ void drain(Ctx& x, int seq) {
#pragma unroll
    for (int k = 0; k < RC; ++k)
      if (k == nd && slot_ready(seq + k)) {
        slot_take(x, seq + k, rc[k]);
        ++nd;
      }
  }
  __device__ __forceinline__ void take(Ctx& x, int& seq, int i, int kt0, f32x4& acc) {
    if (i < RC && i < nd) {
      slot_mfma(x, rc[i < RC ? i : 0], kt0, acc);
      ++seq;
    } else {
      consume_slot(x, seq++, kt0, acc);
    }
  }
};

// fixed-order reduction of the CW waves' partial tiles (two tiles r = 0, 1 in flight): put,
// consumer barrier, then get(r, row) = the tile's output row (MFMA D layout: lane l holds rows
// 4 (l >> 4) + i of column l & 15; column 0 = lanes 0, 16, 32, 48)
__device__ __forceinline__ void red_put(Ctx& x, int r, const f32x4& acc) {
  if (x.lane & 15) return;
  float* p = reinterpret_cast<float*>(pse_lds + L_RED) + ((x.wave - LW) * 2 + r) * 16 + (x.lane >> 4) * 4;
  p[0] = acc[0]; p[1] = acc[1]; p[2] = acc[2]; p[3] = acc[3];
}
__device__ __forceinline__ float red_get(Ctx& x, int r, int row) {
  const float* red = reinterpret_cast<const float*>(pse_lds + L_RED);
  float s = 0.f;
#pragma unroll
  for (int w = 0; w < CW; ++w) s += red[(w * 2 + r) * 16 + row];
  return s;
}

// ---------------------------------------------------------------------------
// Attention unit (g, ku) for the new token at pos (B = 1), by the CW consumer waves: the KV
// head's q heads h0 .. h0 + HU - 1 (HU = G / PSE_AU, h0 = ku HU) over EVERY key, so a unit's
// outputs are final where they are computed (no cross-unit merge).  q / k RMSNorm + RoPE
// (TF/.../modeling_qwen3.py:252-254, :148-170), K / V appended at pos (TF/cache_utils.py:127-145),
// softmax(q k^T / sqrt(D)) v over keys 0..pos with the probabilities rounded to bf16 before P.V
// (the reference's bf16 SDPA), per-wave online softmax over 32-key chunks, the CW wave partials
// and the new key merged in a fixed order -> HU x D outputs as granules.
//   1. gather this unit's q rows (their tiles are complete two thirds into the q|k|v stream,
//      PSE_QFIRST) -- the first chunk's K / V^T and the prologue's inputs load behind the sweep;
//   2. the cached keys' chunks (keys < pos) run while the new token's k / v partials are gathered;
//   3. k / v RMSNorm + RoPE, appended by unit 0;
//   4. merge: the CW wave partials, then the new key (score q . k, p = 1) -> publish.
// graw: the gathered q|k|v K-half partials, [tile][half][16] fp32 (q tiles, k tiles, v tiles).
// Not inlined: the attention's chunk state (K / V^T fragments, online-softmax accumulators) is
// ~200 VGPRs; inlined, it pushed the whole kernel past the 256-VGPR budget of 2 waves per SIMD
// and spilled registers live across every other phase (scratch reloads on the hand-off paths of
// all 256 CUs).  As a call, only the 16 attention CUs save / restore around it.  Every argument is
// a plain value (no pointer into the kernel's arguments or private memory).  Returns the
// consumer barrier count, -1 on a failed wait.
#ifndef PSE_ATT_NOINLINE
#define PSE_ATT_NOINLINE 1
#endif
#if PSE_ATT_NOINLINE
#define PSE_ATT_INL __attribute__((noinline))
#else
#define PSE_ATT_INL __forceinline__
#endif
// (KU: the unit's role under PSE_KSPLIT as a template argument, one callee per role: a runtime role
// joined both roles' register peaks into one callee-saved set; -1 without the key split)
template <int KU>
__device__ PSE_ATT_INL int attention(const PseLayer* Lp, const int* pos_p, const uint8_t* mask, const bf16_t* cos_t,
                                     const bf16_t* sin_t, uint64_t* g_qkv, uint64_t* g_att, uint64_t* g_pp, uint32_t* err,
                                     uint64_t* trace, float eps, float scale, int Cmax, uint32_t epoch, int bar_gen,
                                     int l, int unit, uint32_t tq) {
  const int c = blockIdx.x;
  Ctx x{err, eps, 0, c, (int)(threadIdx.x & 63), (int)(threadIdx.x >> 6), (int)threadIdx.x - LW * 64, epoch, bar_gen};
  struct {
    uint64_t* trace;
  } a{trace};  // (PSE_STAMP)
  constexpr int D = D_, G = G_, KW = 32, QS = D / 32, DT = D / 16, HU = PSE_KSPLIT ? G_ : G_ / PSE_AU;
  static_assert(HU * D / 2 <= CW * 64 && D / 2 == 64, "merge: one wave per head, 2 dims per lane");
  static_assert(HU <= 4, "the unit's q rows sit in MFMA D rows 0 .. 3 (lanes 0-15)");
  const int g = unit / PSE_AU, ku = KU >= 0 ? KU : unit % PSE_AU, h0 = PSE_KSPLIT ? 0 : ku * HU;  // (ku: the role)
  const float* graw = reinterpret_cast<const float*>(pse_lds + L_GRAW);
  uint32_t* graw32 = reinterpret_cast<uint32_t*>(pse_lds + L_GRAW);
  const PseLayer& Lw = *Lp;
  const int pos = *pos_p;
  const int lane = x.lane, w = x.wave - LW, g4 = lane >> 4, c16 = lane & 15;
  bf16_t* kcache = Lw.kc + (size_t)g * Cmax * D;  // [Cmax][D]
  bf16_t* vcache = Lw.vc + (size_t)g * D * Cmax;  // [D][Cmax]
  bf16_t* q_s = reinterpret_cast<bf16_t*>(pse_lds + L_ATT);           // [16][D] (rows >= HU zero)
  float* k_s = reinterpret_cast<float*>(q_s + 16 * D);              // [D]
  float* v_s = k_s + D;                                             // [D]
  bf16_t* p_s = reinterpret_cast<bf16_t*>(v_s + D);                 // [CW][16][KW]
  float* ml_s = reinterpret_cast<float*>(p_s + CW * 16 * KW);       // [CW][G][2]
  float* acc_s = ml_s + CW * G * 2;                                 // [CW][G][D]
  constexpr uint32_t OOBA = 0x7ffffff0u;
  const __amdgpu_buffer_rsrc_t krs = __builtin_amdgcn_make_buffer_rsrc(kcache, 0, Cmax * D * 2, 0x00020000);
  const __amdgpu_buffer_rsrc_t vrs = __builtin_amdgcn_make_buffer_rsrc(vcache, 0, Cmax * D * 2, 0x00020000);
  const __amdgpu_buffer_rsrc_t mrs = __builtin_amdgcn_make_buffer_rsrc(const_cast<uint8_t*>(mask), 0, Cmax, 0x00020000);
  const int nchunk = pos / KW + 1;
  // this unit's chunks [cb, ce): every chunk, or (PSE_KSPLIT) its 1 / PSE_AU share (unit 0, which also
  // takes the new key and the partners' parts, gets the smaller share of an uneven split)
  const int kk = unit % PSE_AU;
  const int cb = PSE_KSPLIT ? kk * nchunk / PSE_AU : 0, ce = PSE_KSPLIT ? (kk + 1) * nchunk / PSE_AU : nchunk;
  // a wave's 32-key chunk: K tiles (A operands), V^T fragments (B operands), mask words; keys
  // >= pos read zero (branch-free buffer loads; the new key joins in the merge)
  auto load_chunk = [&](int ch, u32x4 (&kt)[2][QS], u32x4 (&vt)[DT], uint32_t (&mk)[2]) {
    const int k0 = ch * KW;
#pragma unroll
    for (int t = 0; t < 2; ++t) {
      const int key = k0 + t * 16 + c16;
#pragma unroll
      for (int s2 = 0; s2 < QS; ++s2)
        kt[t][s2] = __builtin_amdgcn_raw_buffer_load_b128(
            krs, key < pos ? (uint32_t)(key * D + s2 * 32 + 8 * g4) * 2u : OOBA, 0, 0);
      mk[t] = __builtin_amdgcn_raw_buffer_load_b32(mrs, (k0 + t * 16 <= pos) ? (uint32_t)(k0 + t * 16 + g4 * 4) : OOBA,
                                                   0, 0);
    }
#pragma unroll
    for (int dt = 0; dt < DT; ++dt) {
      const int kb = k0 + 8 * g4;
      vt[dt] = __builtin_amdgcn_raw_buffer_load_b128(
          vrs, kb < pos ? (uint32_t)((dt * 16 + c16) * Cmax + kb) * 2u : OOBA, 0, 0);
    }
  };
  u32x4 ktA[2][QS], vtA[DT];
  uint32_t mkA[2];
  // this wave's chunks: w, then every CW; its q job (wave w < HU: q row w) norm weight, wave 0's
  // k norm weight, the RoPE row at pos (2 dims per lane) and the new token's mask byte
  const int ch0 = cb + w;
  constexpr int CSTEP = CW;
  uint32_t qnw = 0, knw = 0, pcs = 0, psn = 0, mnew = 0;
  auto prefetch = [&]() {
    load_chunk(ch0, ktA, vtA, mkA);
    qnw = w < HU ? reinterpret_cast<const uint32_t*>(Lw.q_norm)[lane] : 0u;
    knw = reinterpret_cast<const uint32_t*>(Lw.k_norm)[lane];
    pcs = reinterpret_cast<const uint32_t*>(cos_t + (size_t)pos * D)[lane];
    psn = reinterpret_cast<const uint32_t*>(sin_t + (size_t)pos * D)[lane];
    mnew = mask[pos];
  };
  // q|k|v row value: sum of the two K-half partials, rounded to bf16 (the projection output)
  auto val = [&](int base_tile, int i) {
    const float* p = graw + (base_tile + i / 16) * 32 + i % 16;
    return rbf(p[0] + p[16]);
  };
  // q / k RMSNorm + RoPE of one row: 2 dims per lane
  auto norm_rope = [&](float x0, float x1, uint32_t nw, float& o0, float& o1) {
    const float ss = wave_sum(x0 * x0 + x1 * x1);
    const float r = 1.0f / sqrtf(ss / (float)D + eps);
    const float n0 = rbf(__uint_as_float(nw << 16) * rbf(x0 * r)), n1 = rbf(__uint_as_float(nw & 0xffff0000u) * rbf(x1 * r));
    constexpr int q4 = D / 4;
    const bool lo = 2 * lane < D / 2;
    const int partner = lo ? lane + q4 : lane - q4;
    const float p0 = __shfl(n0, partner, 64), p1 = __shfl(n1, partner, 64);
    const float sg = lo ? -1.f : 1.f;
    const float c0 = __uint_as_float(pcs << 16), c1 = __uint_as_float(pcs & 0xffff0000u);
    const float s0 = __uint_as_float(psn << 16), s1 = __uint_as_float(psn & 0xffff0000u);
    o0 = rbf(rbf(n0 * c0) + rbf(sg * p0 * s0));
    o1 = rbf(rbf(n1 * c1) + rbf(sg * p1 * s1));
  };
  if (PSE_TRACE2 && w == 0) PSE_STAMP(l, 25);
#if PSE_TRACE2
  x.tp = trace ? trace + ((size_t)l * PSE_TRACE_EV + 20) * 256 + c : nullptr;  // the q gather: events 20-24
#endif
  if (PSE_APAUSE && x.tid == 0) __hip_atomic_store(&PSE_CTL->apause, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
  // ---- 1. q ----
  constexpr int NG = (G_ + 2) * (D_ / 16) * 32;  // the KV head's q|k|v granules (qkv_gran)
  constexpr int NQ = HU * (D_ / 16) * 32, NKV = 2 * (D_ / 16) * 32;
  if (!gather<(NQ + CW * 64 - 1) / (CW * 64)>(x, g_qkv + (size_t)g * NG + h0 * (D_ / 16) * 32, NQ, tq,
                                              graw32 + h0 * (D_ / 16) * 32, NQ, nullptr, prefetch))
    return -1;
#if PSE_TRACE2
  x.tp = nullptr;
#endif
  if (w == 0) PSE_STAMP(l, 15);
  if (PSE_APAUSE == 1 && x.tid == 0)  // (PSE_APAUSE 1: the loader resumes once the q rows are in)
    __hip_atomic_store(&PSE_CTL->apause, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
  for (int i = x.tid; i < 16 * D; i += CW * 64)
    if (i / D >= HU) q_s[i] = 0;
  if (w < HU) {
    const int bt = (h0 + w) * (D / 16);
    float o0, o1;
    norm_rope(val(bt, 2 * lane), val(bt, 2 * lane + 1), qnw, o0, o1);
    q_s[w * D + 2 * lane] = f2bf(o0);
    q_s[w * D + 2 * lane + 1] = f2bf(o1);
  }
  cbar(x);
  // ---- 2. the cached keys ----
  float m_run = -INFINITY, l_run = 0.f;
  float* o_s = acc_s + w * HU * D + c16;  // the running output (pse_chunk.h)
  pse_chunk_init<HU, D>(g4, o_s);
  auto compute = [&](int ch, u32x4 (&kt)[2][QS], u32x4 (&vt)[DT], const uint32_t (&mk)[2]) {
    pse_chunk_step<HU, D>(ch * KW, pos, g4, c16, kt, vt, mk, q_s, p_s + w * 16 * KW, o_s, scale, m_run, l_run);
  };
  auto chunks = [&]() {
    if (w == 0) PSE_STAMP(l, 16);
    for (int ch = ch0; ch < ce; ch += CSTEP) {
      if (ch != ch0) load_chunk(ch, ktA, vtA, mkA);
      compute(ch, ktA, vtA, mkA);
    }
    if (w == 0) PSE_STAMP(l, 17);
  };
  if (PSE_KSPLIT && ku == 1) {  // (only unit 0 takes the new token's k / v)
    chunks();
    if (failed(x)) return -1;
  } else if (!gather<(NKV + CW * 64 - 1) / (CW * 64)>(x, g_qkv + (size_t)g * NG + G * (D_ / 16) * 32, NKV, tq,
                                                      graw32 + G * (D_ / 16) * 32, NKV, nullptr, chunks)) {
    return -1;
  }
  if (PSE_TRACE2 && w == 0) PSE_STAMP(l, 18);
  // ---- 3. k (wave 0) and v (wave 1); unit 0 appends them ----
  if (PSE_KSPLIT && ku == 1) {
  } else if (w == 0) {
    float o0, o1;
    norm_rope(val(G * (D / 16), 2 * lane), val(G * (D / 16), 2 * lane + 1), knw, o0, o1);
    k_s[2 * lane] = o0;
    k_s[2 * lane + 1] = o1;
    if (ku == 0) *reinterpret_cast<uint32_t*>(kcache + (size_t)pos * D + 2 * lane) = pack2(o0, o1);
  } else if (w == 1) {
    const float x0 = val((G + 1) * (D / 16), 2 * lane), x1 = val((G + 1) * (D / 16), 2 * lane + 1);
    v_s[2 * lane] = x0;
    v_s[2 * lane + 1] = x1;
    if (ku == 0) {
      vcache[(size_t)(2 * lane) * Cmax + pos] = f2bf(x0);
      vcache[(size_t)(2 * lane + 1) * Cmax + pos] = f2bf(x1);
    }
  }
  if (lane < HU) {
    ml_s[(w * HU + lane) * 2] = m_run;
    ml_s[(w * HU + lane) * 2 + 1] = l_run;
  }
  cbar(x);
  if (PSE_TRACE2 && w == 0) PSE_STAMP(l, 19);
  // (PSE_KSPLIT) unit 0: the partners' rows -> graw (the q|k|v partials are consumed: q in q_s, k / v in
  // k_s / v_s), their (max, sum) per head -> the sums-of-squares scratch (free through the attention)
  const float* pp = reinterpret_cast<const float*>(graw);
  const float* pml = reinterpret_cast<const float*>(pse_lds + L_MISC);
  if (PSE_KSPLIT && ku == 0 &&
      !gather<(KS_N + CW * 64 - 1) / (CW * 64)>(x, g_pp + (size_t)g * KS_N, KS_N, tagof(x.epoch, l, OP_ATT), graw32,
                                                 (PSE_AU - 1) * KS_ROWS, reinterpret_cast<uint32_t*>(pse_lds + L_MISC)))
    return -1;
  // ---- 4. merge (thread e / 2: 2 output dims of local head h = wave w) and publish ----
  const int e = 2 * x.tid, h = e / D, d = e % D;
  if (e < HU * D) {
    float M = -INFINITY;
#pragma unroll
    for (int ww = 0; ww < CW; ++ww) M = fmaxf(M, ml_s[(ww * HU + h) * 2]);
    // the new key: its score q . k (this wave's head), one more partial with p = bf16(1) = 1
    const float sn = wave_sum(bf2f(q_s[h * D + d]) * k_s[d] + bf2f(q_s[h * D + d + 1]) * k_s[d + 1]) * scale;
    const bool nv = mnew != 0u && (!PSE_KSPLIT || ku == 0);
    if (nv) M = fmaxf(M, sn);
    float L = 0.f, o0 = 0.f, o1 = 0.f;
#pragma unroll
    for (int ww = 0; ww < CW; ++ww) {
      const float mw = ml_s[(ww * HU + h) * 2];
      const float f = (mw == -INFINITY) ? 0.f : expf(mw - M);
      L += f * ml_s[(ww * HU + h) * 2 + 1];
      o0 += f * acc_s[(ww * HU + h) * D + d];
      o1 += f * acc_s[(ww * HU + h) * D + d + 1];
    }
    if (nv) {
      const float f = expf(sn - M);
      L += f;
      o0 += f * v_s[d];
      o1 += f * v_s[d + 1];
    }
    const uint32_t ta = tagof(x.epoch, l, OP_ATT);
    if (PSE_KSPLIT && ku == 1) {  // this unit's part, unnormalised, against its own max
      uint64_t* q = g_pp + (size_t)g * KS_N;
      const int pi = kk - 1;
      st64(q + pi * KS_ROWS + h * D + d, gran(__float_as_uint(o0), ta));
      st64(q + pi * KS_ROWS + h * D + d + 1, gran(__float_as_uint(o1), ta));
      if (d == 0) {
        st64(q + (PSE_AU - 1) * KS_ROWS + pi * 2 * G + 2 * h, gran(__float_as_uint(M), ta));
        st64(q + (PSE_AU - 1) * KS_ROWS + pi * 2 * G + 2 * h + 1, gran(__float_as_uint(L), ta));
      }
    }
    if (PSE_KSPLIT && ku == 0) {  // the partners' parts, in unit order: everything rescaled to the joint max
      float Mj = M;
#pragma unroll
      for (int pi = 0; pi < PSE_AU - 1; ++pi) Mj = fmaxf(Mj, pml[pi * 2 * G + 2 * h]);
      const float f0 = (M == -INFINITY) ? 0.f : expf(M - Mj);
      L *= f0;
      o0 *= f0;
      o1 *= f0;
#pragma unroll
      for (int pi = 0; pi < PSE_AU - 1; ++pi) {
        const float mp = pml[pi * 2 * G + 2 * h];
        const float fp = (mp == -INFINITY) ? 0.f : expf(mp - Mj);
        L += fp * pml[pi * 2 * G + 2 * h + 1];
        o0 += fp * pp[pi * KS_ROWS + h * D + d];
        o1 += fp * pp[pi * KS_ROWS + h * D + d + 1];
      }
    }
    if (!(PSE_KSPLIT && ku == 1))
      st64(g_att + (g * G * D + h0 * D + e) / 2, gran(L > 0.f ? pack2(o0 / L, o1 / L) : 0u, ta));
  }
  cbar(x);
  return x.bar_gen;
}


// ---------------------------------------------------------------------------
// Long-context form (pse_kernel_t<true>, contexts past the 2-CU-per-head form's range; round 4).
// The short form's attention units each read EVERY cached key of their head, so the chain grows
// with the context (the launch lost to the per-op split attention past ~800 keys).  Here every CU
// takes a slice: CU c scores the cached keys of KV head g = c % 8 in its 1/32 share (s = c / 8) of
// the 32-key chunks, all 4 q heads of the group at once, and publishes its (m, l, o) partials;
// 64 merge units (q head, half of the dims) combine the 32 slices with the new key (score q . k,
// p = 1) and append k / v.  The chain: q gather -> the slice's K / V (1/256 of the layer's cache
// per CU, every CU's loader paused so the reads do not queue behind the weight stream) -> partial
// hop -> merge -> the o gather: about the short form's length at any context.
constexpr int LS = 32;                               // slices per KV head
constexpr int PART_W = 2 + D_ / 2;                   // granules per (q head, half, slice): m, l, 64 dims
constexpr int NG_PART = HQ_ * 2 * LS * PART_W;       // 135,168
constexpr int L_STASH = L_MISC;                      // merge inputs kept by the slice: k norm w, cos, sin, mask
// merge unit u (q head u / 2, dim half u % 2) on the CU whose slice is slice 24 + u % 8 of KV head
// u / 8: the unit reuses the q rows and k / v partials its own slice gathered; -1: none
__host__ __device__ inline int pse_merge_unit(int c) {
  const int sl = c / HKV_;
  return sl >= LS - 8 ? (c % HKV_) * 8 + (sl - (LS - 8)) : -1;
}

// The slice of CU c = blockIdx.x: q rows of the group's 4 q heads (q|k|v granules grouped by KV head,
// qkv_gran), then per-wave online softmax over the slice's chunks (pse.hip attention()'s chunk
// math, HU = 4), the 4 wave partials merged, (m, l, o) published unnormalised.  A merge unit also
// gathers the new token's k / v partials (behind its chunks) and stashes its merge inputs.
#ifndef PSE_SLICE_INLINE
#define PSE_SLICE_INLINE 0
#endif
#if PSE_SLICE_INLINE
#define PSE_SLICE_ATTR __attribute__((always_inline))
#else
#define PSE_SLICE_ATTR __attribute__((noinline))
#endif
// (one instantiation per role: a runtime merge flag joined the two chunk-loop forms into one
// register allocation of 254 VGPRs, 172 / 182 apart, and every VGPR past v39 a noinline callee
// touches is a callee-saved stripe spilled to scratch per call)
template <bool merge>
__device__ PSE_SLICE_ATTR int attention_slice(const PseLayer* Lp, const int* pos_p, const uint8_t* mask,
                                              const bf16_t* cos_t, const bf16_t* sin_t, uint64_t* g_qkv,
                                              uint64_t* g_part, uint32_t* err, float eps, float scale, int Cmax,
                                              uint32_t epoch, int bar_gen, int l, uint32_t tq) {
  const int c = blockIdx.x;
  Ctx x{err, eps, 0, c, (int)(threadIdx.x & 63), (int)(threadIdx.x >> 6), (int)threadIdx.x - LW * 64, epoch, bar_gen};
  constexpr int D = D_, G = G_, KW = 32, QS = D / 32, DT = D / 16, HU = G_;
  const int g = c % HKV_, sl = c / HKV_;
  const float* graw = reinterpret_cast<const float*>(pse_lds + L_GRAW);
  uint32_t* graw32 = reinterpret_cast<uint32_t*>(pse_lds + L_GRAW);
  const PseLayer& Lw = *Lp;
  const int pos = *pos_p;
  const int lane = x.lane, w = x.wave - LW, g4 = lane >> 4, c16 = lane & 15;
  const bf16_t* kcache = Lw.kc + (size_t)g * Cmax * D;
  const bf16_t* vcache = Lw.vc + (size_t)g * D * Cmax;
  bf16_t* q_s = reinterpret_cast<bf16_t*>(pse_lds + L_ATT);
  float* k_s = reinterpret_cast<float*>(q_s + 16 * D);
  float* v_s = k_s + D;
  bf16_t* p_s = reinterpret_cast<bf16_t*>(v_s + D);
  float* ml_s = reinterpret_cast<float*>(p_s + CW * 16 * KW);
  float* acc_s = ml_s + CW * G * 2;
  uint32_t* stash = reinterpret_cast<uint32_t*>(pse_lds + L_STASH);
  constexpr uint32_t OOBA = 0x7ffffff0u;
  const __amdgpu_buffer_rsrc_t krs = __builtin_amdgcn_make_buffer_rsrc(const_cast<bf16_t*>(kcache), 0, Cmax * D * 2, 0x00020000);
  const __amdgpu_buffer_rsrc_t vrs = __builtin_amdgcn_make_buffer_rsrc(const_cast<bf16_t*>(vcache), 0, Cmax * D * 2, 0x00020000);
  const __amdgpu_buffer_rsrc_t mrs = __builtin_amdgcn_make_buffer_rsrc(const_cast<uint8_t*>(mask), 0, Cmax, 0x00020000);
  // this slice's chunks of the cached keys 0 .. pos-1
  const int nct = (pos + KW - 1) / KW, cb = sl * nct / LS, ce = (sl + 1) * nct / LS;
  auto load_chunk = [&](int ch, u32x4 (&kt)[2][QS], u32x4 (&vt)[DT], uint32_t (&mk)[2]) {
    const int k0 = ch * KW;
#pragma unroll
    for (int t = 0; t < 2; ++t) {
      const int key = k0 + t * 16 + c16;
#pragma unroll
      for (int s2 = 0; s2 < QS; ++s2)
        kt[t][s2] = __builtin_amdgcn_raw_buffer_load_b128(
            krs, (key < pos && ch < ce) ? (uint32_t)(key * D + s2 * 32 + 8 * g4) * 2u : OOBA, 0, 0);
      mk[t] = __builtin_amdgcn_raw_buffer_load_b32(
          mrs, (k0 + t * 16 <= pos && ch < ce) ? (uint32_t)(k0 + t * 16 + g4 * 4) : OOBA, 0, 0);
    }
#pragma unroll
    for (int dt = 0; dt < DT; ++dt) {
      const int kb = k0 + 8 * g4;
      vt[dt] = __builtin_amdgcn_raw_buffer_load_b128(
          vrs, (kb < pos && ch < ce) ? (uint32_t)((dt * 16 + c16) * Cmax + kb) * 2u : OOBA, 0, 0);
    }
  };
  u32x4 ktA[2][QS], vtA[DT];
  uint32_t mkA[2];
  const int ch0 = cb + w;
  uint32_t qnw = 0, knw = 0, pcs = 0, psn = 0, mnew = 0;
  auto prefetch = [&]() {
    load_chunk(ch0, ktA, vtA, mkA);
    qnw = reinterpret_cast<const uint32_t*>(Lw.q_norm)[lane];
    pcs = reinterpret_cast<const uint32_t*>(cos_t + (size_t)pos * D)[lane];
    psn = reinterpret_cast<const uint32_t*>(sin_t + (size_t)pos * D)[lane];
    if constexpr (merge) {
      knw = reinterpret_cast<const uint32_t*>(Lw.k_norm)[lane];
      mnew = mask[pos];
    }
  };
  auto val = [&](int base_tile, int i) {
    const float* p = graw + (base_tile + i / 16) * 32 + i % 16;
    return rbf(p[0] + p[16]);
  };
  auto norm_rope = [&](float x0, float x1, uint32_t nw, float& o0, float& o1) {
    const float ss = wave_sum(x0 * x0 + x1 * x1);
    const float r = 1.0f / sqrtf(ss / (float)D + eps);
    const float n0 = rbf(__uint_as_float(nw << 16) * rbf(x0 * r)), n1 = rbf(__uint_as_float(nw & 0xffff0000u) * rbf(x1 * r));
    constexpr int q4 = D / 4;
    const bool lo = 2 * lane < D / 2;
    const int partner = lo ? lane + q4 : lane - q4;
    const float p0 = __shfl(n0, partner, 64), p1 = __shfl(n1, partner, 64);
    const float sg = lo ? -1.f : 1.f;
    const float c0 = __uint_as_float(pcs << 16), c1 = __uint_as_float(pcs & 0xffff0000u);
    const float s0 = __uint_as_float(psn << 16), s1 = __uint_as_float(psn & 0xffff0000u);
    o0 = rbf(rbf(n0 * c0) + rbf(sg * p0 * s0));
    o1 = rbf(rbf(n1 * c1) + rbf(sg * p1 * s1));
  };
  if (x.tid == 0) __hip_atomic_store(&PSE_CTL->apause, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
  constexpr int NG = (G_ + 2) * (D_ / 16) * 32;
  constexpr int NQ = HU * (D_ / 16) * 32, NKV = 2 * (D_ / 16) * 32;
  if (!gather<(NQ + CW * 64 - 1) / (CW * 64)>(x, g_qkv + (size_t)g * NG, NQ, tq, graw32, NQ, nullptr, prefetch))
    return -1;
  if (merge && w == 0) {  // the merge's inputs, read back after this slice's scratch is reused
    stash[lane] = knw;
    stash[64 + lane] = pcs;
    stash[128 + lane] = psn;
    if (lane == 0) stash[192] = mnew;
  }
  {
    const int bt = w * (D / 16);
    float o0, o1;
    norm_rope(val(bt, 2 * lane), val(bt, 2 * lane + 1), qnw, o0, o1);
    q_s[w * D + 2 * lane] = f2bf(o0);
    q_s[w * D + 2 * lane + 1] = f2bf(o1);
  }
  for (int i = x.tid; i < 16 * D; i += CW * 64)
    if (i / D >= HU) q_s[i] = 0;
  cbar(x);
  float m_run = -INFINITY, l_run = 0.f;
  float* o_s = acc_s + w * HU * D + c16;  // the running output (pse_chunk.h)
  pse_chunk_init<HU, D>(g4, o_s);
  auto compute = [&](int ch, u32x4 (&kt)[2][QS], u32x4 (&vt)[DT], const uint32_t (&mk)[2]) {
    pse_chunk_step<HU, D>(ch * KW, pos, g4, c16, kt, vt, mk, q_s, p_s + w * 16 * KW, o_s, scale, m_run, l_run);
  };
  auto chunks = [&]() {
#pragma unroll 1
    for (int ch = ch0; ch < ce; ch += CW) {
      if (ch != ch0) load_chunk(ch, ktA, vtA, mkA);
      compute(ch, ktA, vtA, mkA);
    }
  };
  if constexpr (merge) {  // the new token's k / v partials, gathered behind this slice's chunks
    if (!gather<(NKV + CW * 64 - 1) / (CW * 64)>(x, g_qkv + (size_t)g * NG + NQ, NKV, tq, graw32 + NQ, NKV, nullptr,
                                                 chunks))
      return -1;
  } else {
    chunks();
  }
  if (PSE_LONG_RESUME && x.tid == 0) __hip_atomic_store(&PSE_CTL->apause, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
  if (lane < HU) {
    ml_s[(w * HU + lane) * 2] = m_run;
    ml_s[(w * HU + lane) * 2 + 1] = l_run;
  }
  cbar(x);
  // the 4 wave partials -> the slice's (m, l, o) of q head h (thread: 2 dims)
  {
    const int e = 2 * x.tid, h = e / D, d = e % D;
    float M = -INFINITY;
#pragma unroll
    for (int ww = 0; ww < CW; ++ww) M = fmaxf(M, ml_s[(ww * HU + h) * 2]);
    float L = 0.f, o0 = 0.f, o1 = 0.f;
#pragma unroll
    for (int ww = 0; ww < CW; ++ww) {
      const float mw = ml_s[(ww * HU + h) * 2];
      const float f = (mw == -INFINITY) ? 0.f : expf(mw - M);
      L += f * ml_s[(ww * HU + h) * 2 + 1];
      o0 += f * acc_s[(ww * HU + h) * D + d];
      o1 += f * acc_s[(ww * HU + h) * D + d + 1];
    }
    const uint32_t tg = tagof(x.epoch, l, OP_ATT);
    uint64_t* pp = g_part + ((size_t)((g * G + h) * 2 + d / (D / 2)) * LS + sl) * PART_W;
    st64(pp + 2 + d % (D / 2), gran(__float_as_uint(o0), tg));
    st64(pp + 3 + d % (D / 2), gran(__float_as_uint(o1), tg));
    if (d % (D / 2) == 0) {
      st64(pp, gran(__float_as_uint(M), tg));
      st64(pp + 1, gran(__float_as_uint(L), tg));
    }
  }
  cbar(x);
  return x.bar_gen;
}

// Merge unit u: q head hq = u / 2, dims [64 (u % 2), +64): the 32 slices' partials plus the new key
// (score q . k, p = 1: TF/integrations/sdpa_attention.py:79-166 over keys 0..pos), k RMSNorm + RoPE,
// k / v appended by the group's first unit (TF/cache_utils.py:127-145), the output published as
// the o_proj input granules.  q_s / graw / the stash still hold this CU's slice inputs.
__device__ PSE_SLICE_ATTR int attention_merge(const PseLayer* Lp, const int* pos_p, uint64_t* g_part,
                                                         uint64_t* g_att, uint32_t* err, float eps, float scale,
                                                         int Cmax, uint32_t epoch, int bar_gen, int l, int u) {
  const int c = blockIdx.x;
  Ctx x{err, eps, 0, c, (int)(threadIdx.x & 63), (int)(threadIdx.x >> 6), (int)threadIdx.x - LW * 64, epoch, bar_gen};
  constexpr int D = D_, G = G_;
  const int hq = u / 2, half = u % 2, g = hq / G, hl = hq % G;
  const int lane = x.lane, w = x.wave - LW;
  const int pos = *pos_p;
  const PseLayer& Lw = *Lp;
  const float* graw = reinterpret_cast<const float*>(pse_lds + L_GRAW);
  const bf16_t* q_s = reinterpret_cast<const bf16_t*>(pse_lds + L_ATT);
  float* k_s = reinterpret_cast<float*>(pse_lds + L_ATT + 16 * D * 2);
  float* v_s = k_s + D;
  uint32_t* pb32 = reinterpret_cast<uint32_t*>(v_s + D);  // the slices' partials (over the slice's p_s / acc_s)
  const float* pb = reinterpret_cast<const float*>(pb32);
  const uint32_t* stash = reinterpret_cast<const uint32_t*>(pse_lds + L_STASH);
  auto val = [&](int base_tile, int i) {
    const float* p = graw + (base_tile + i / 16) * 32 + i % 16;
    return rbf(p[0] + p[16]);
  };
  const bool app = hl == 0 && half == 0;
  if (w == 0) {  // k: RMSNorm + RoPE (pse.hip attention() step 3)
    const uint32_t knw = stash[lane], pcs = stash[64 + lane], psn = stash[128 + lane];
    const float x0 = val(G * (D / 16), 2 * lane), x1 = val(G * (D / 16), 2 * lane + 1);
    const float ss = wave_sum(x0 * x0 + x1 * x1);
    const float r = 1.0f / sqrtf(ss / (float)D + eps);
    const float n0 = rbf(__uint_as_float(knw << 16) * rbf(x0 * r)), n1 = rbf(__uint_as_float(knw & 0xffff0000u) * rbf(x1 * r));
    constexpr int q4 = D / 4;
    const bool lo = 2 * lane < D / 2;
    const int partner = lo ? lane + q4 : lane - q4;
    const float p0 = __shfl(n0, partner, 64), p1 = __shfl(n1, partner, 64);
    const float sg = lo ? -1.f : 1.f;
    const float c0 = __uint_as_float(pcs << 16), c1 = __uint_as_float(pcs & 0xffff0000u);
    const float s0 = __uint_as_float(psn << 16), s1 = __uint_as_float(psn & 0xffff0000u);
    const float o0 = rbf(rbf(n0 * c0) + rbf(sg * p0 * s0)), o1 = rbf(rbf(n1 * c1) + rbf(sg * p1 * s1));
    k_s[2 * lane] = o0;
    k_s[2 * lane + 1] = o1;
    if (app) *reinterpret_cast<uint32_t*>(Lw.kc + (size_t)g * Cmax * D + (size_t)pos * D + 2 * lane) = pack2(o0, o1);
  } else if (w == 1) {
    const float x0 = val((G + 1) * (D / 16), 2 * lane), x1 = val((G + 1) * (D / 16), 2 * lane + 1);
    v_s[2 * lane] = x0;
    v_s[2 * lane + 1] = x1;
    if (app) {
      bf16_t* vcache = Lw.vc + (size_t)g * D * Cmax;
      vcache[(size_t)(2 * lane) * Cmax + pos] = f2bf(x0);
      vcache[(size_t)(2 * lane + 1) * Cmax + pos] = f2bf(x1);
    }
  }
  constexpr int NP = LS * PART_W;  // 2,112
  if (!gather<(NP + CW * 64 - 1) / (CW * 64)>(x, g_part + (size_t)(hq * 2 + half) * NP, NP, tagof(epoch, l, OP_ATT), pb32, NP))
    return -1;
  // the new key's score q . k (every wave alike), then thread j < 32: dims 64 half + 2 j, +1
  const float sn = wave_sum(bf2f(q_s[hl * D + 2 * lane]) * k_s[2 * lane] + bf2f(q_s[hl * D + 2 * lane + 1]) * k_s[2 * lane + 1]) * scale;
  if (x.tid < D / 4) {
    const int j = x.tid, d = half * (D / 2) + 2 * j;
    const bool nv = stash[192] != 0u;
    float M = nv ? sn : -INFINITY;
    for (int s2 = 0; s2 < LS; ++s2) M = fmaxf(M, pb[s2 * PART_W]);
    float L = 0.f, o0 = 0.f, o1 = 0.f;
    for (int s2 = 0; s2 < LS; ++s2) {
      const float ms = pb[s2 * PART_W];
      const float f = (ms == -INFINITY) ? 0.f : expf(ms - M);
      L += f * pb[s2 * PART_W + 1];
      o0 += f * pb[s2 * PART_W + 2 + 2 * j];
      o1 += f * pb[s2 * PART_W + 3 + 2 * j];
    }
    if (nv) {
      const float f = expf(sn - M);
      L += f;
      o0 += f * v_s[d];
      o1 += f * v_s[d + 1];
    }
    st64(g_att + (hq * D + d) / 2, gran(L > 0.f ? pack2(o0 / L, o1 / L) : 0u, tagof(x.epoch, l, OP_ATT)));
  }
  cbar(x);
  return x.bar_gen;
}

}  // namespace

// ---------------------------------------------------------------------------
template <bool LONG>
__global__ __launch_bounds__(THREADS) void pse_kernel_t(PseArgs a) {
  unsigned char* const lds = pse_lds;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int c = blockIdx.x, P = gridDim.x;
  Ctl* ctl = reinterpret_cast<Ctl*>(lds + L_CTL);
  static_assert(sizeof(Ctl) <= 256, "control words");
  if (threadIdx.x < 64) reinterpret_cast<int*>(lds + L_CTL)[threadIdx.x] = 0;
  // the loader's weight pointers, [layer][q|k|v, o, gate|up, down], in LDS: a global load in its
  // loop would be waited for with vmcnt(0), i.e. with every weight fill in flight
  const bf16_t** wp = reinterpret_cast<const bf16_t**>(lds + L_PTR);
  for (int i = threadIdx.x; i < a.layers * 4; i += THREADS) {
    const PseLayer& q = a.L[i / 4];
    wp[i] = (i & 3) == 0 ? q.qkv : ((i & 3) == 1 ? q.o : ((i & 3) == 2 ? q.gu : q.down));
  }
  __syncthreads();
  const uint32_t epoch = (ld32(a.epoch) + 1u) & 0xffffffu;
  const int nq = LONG ? 3 : pse_nq(c, P), spl = 4 * nq + 80;  // this CU's q|k|v units, slots per layer
  const int total = a.layers * spl;

  if (wave < LW) {
    // =================== loaders ===================
    if (PSE_LPRIO) __builtin_amdgcn_s_setprio(PSE_LPRIO);  // (A/B: the loader ahead of spinning consumers)
    auto slot_src = [&](int s) { return pse_slot_src(wp, c, nq, s); };
    // Register-staged loader: each slot is loaded into one of 3 register buffers (16 x 16 B per
    // lane) and copied into its ring slot once that slot is free, so the 3 slots in flight do not
    // occupy ring slots (8 ready + 3 in flight, against 8 including the in-flight fills of the
    // LDS-DMA loader).  The copy + reload of a buffer is ONE asm block with the buffer as "+v"
    // operands: the compiler's own waitcnt insertion waits for every load in flight before any
    // use of a loop-carried load result (measured: vmcnt(0) at each copy), so the count is
    // explicit here -- vmcnt(32) = this buffer's loads, the two younger buffers' 32 still in
    // flight.  Every copy / reload issues exactly 16 loads (a slot past the end re-reads the last
    // slot), which keeps that count exact; loads are only ever addressed inside the weights (a
    // prefetch past the last slot would index the pointer table past its last layer).
    u32x4 bA[SLOT_KB], bB[SLOT_KB], bC[SLOT_KB];
    bool dead = false;
    const uint32_t voff = (uint32_t)lane * 16u;
    const uint32_t ring0 = (uint32_t)(uintptr_t)(lvoid*)(lds + L_RING) + voff;
    auto src_of = [&](int s0) -> const void* {
      const int s = min(s0, total - 1);
      const int l = s / spl, r = s - l * spl;
      if (a.trace && lane == 0 && s0 < total) {
        const int rq = 4 * nq;
        const int ev = r == 0 ? 0 : (r == rq ? 1 : (r == rq + 8 ? 2 : (r == rq + 56 ? 3 : (r == spl - 1 ? 4 : -1))));
        if (ev >= 0) ctl->lstamp[l & 1][ev] = __builtin_amdgcn_s_memrealtime();
      }
      if ((PSE_APAUSE || LONG) && s0 < total)  // this CU's attention is gathering its inputs: no new loads
        for (uint32_t spins = 0; __hip_atomic_load(&ctl->apause, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) &&
                                 !__hip_atomic_load(&ctl->abort, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) &&
                                 spins < SPIN_LDS;
             ++spins)
          __builtin_amdgcn_s_sleep(1);
      const uint64_t p = (uint64_t)(uintptr_t)slot_src(s);  // wave-uniform: into SGPRs
      const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)p), hi = __builtin_amdgcn_readfirstlane((uint32_t)(p >> 32));
      return (const void*)(((uint64_t)hi << 32) | lo);
    };
#define PSE_RL_OPS                                                                                  \
  [b0] "+v"(b[0]), [b1] "+v"(b[1]), [b2] "+v"(b[2]), [b3] "+v"(b[3]), [b4] "+v"(b[4]), [b5] "+v"(b[5]), \
      [b6] "+v"(b[6]), [b7] "+v"(b[7]), [b8] "+v"(b[8]), [b9] "+v"(b[9]), [b10] "+v"(b[10]),          \
      [b11] "+v"(b[11]), [b12] "+v"(b[12]), [b13] "+v"(b[13]), [b14] "+v"(b[14]), [b15] "+v"(b[15])
// (s_nop 4 first: %[g] comes fresh from v_readfirstlane, and a VMEM instruction reading an SGPR
// a VALU just wrote needs 5 wait states, which hipcc does not insert inside an asm string --
// without them the loads take the SGPRs' previous contents as their base: the illegal-address
// fault of the round-2 register loader)
#define PSE_RL_LOADS                                                                                \
  "s_nop 4\n\t"                                                                                    \
  "global_load_dwordx4 %[b0], %[o0], %[g] offset:0 nt\n\t"                                        \
  "global_load_dwordx4 %[b1], %[o0], %[g] offset:1024 nt\n\t"                                     \
  "global_load_dwordx4 %[b2], %[o0], %[g] offset:2048 nt\n\t"                                     \
  "global_load_dwordx4 %[b3], %[o0], %[g] offset:3072 nt\n\t"                                     \
  "global_load_dwordx4 %[b4], %[o1], %[g] offset:0 nt\n\t"                                        \
  "global_load_dwordx4 %[b5], %[o1], %[g] offset:1024 nt\n\t"                                     \
  "global_load_dwordx4 %[b6], %[o1], %[g] offset:2048 nt\n\t"                                     \
  "global_load_dwordx4 %[b7], %[o1], %[g] offset:3072 nt\n\t"                                     \
  "global_load_dwordx4 %[b8], %[o2], %[g] offset:0 nt\n\t"                                        \
  "global_load_dwordx4 %[b9], %[o2], %[g] offset:1024 nt\n\t"                                     \
  "global_load_dwordx4 %[b10], %[o2], %[g] offset:2048 nt\n\t"                                    \
  "global_load_dwordx4 %[b11], %[o2], %[g] offset:3072 nt\n\t"                                    \
  "global_load_dwordx4 %[b12], %[o3], %[g] offset:0 nt\n\t"                                       \
  "global_load_dwordx4 %[b13], %[o3], %[g] offset:1024 nt\n\t"                                    \
  "global_load_dwordx4 %[b14], %[o3], %[g] offset:2048 nt\n\t"                                    \
  "global_load_dwordx4 %[b15], %[o3], %[g] offset:3072 nt\n\t"
    auto load = [&](u32x4 (&b)[SLOT_KB], int s_issue) {
      const void* g = src_of(s_issue);
      asm volatile(PSE_RL_LOADS
                   : PSE_RL_OPS
                   : [g] "s"(g), [o0] "v"(voff), [o1] "v"(voff + 4096u), [o2] "v"(voff + 8192u), [o3] "v"(voff + 12288u)
                   : "memory");
    };
    // copy buffer b (slot s, loaded two buffers ago) into its ring slot, then reload b with slot s_issue
    auto copy_load = [&](u32x4 (&b)[SLOT_KB], int s, int s_issue) {
      if (s >= NS && !dead)
        for (uint32_t spins = 0;; ++spins) {  // ring slot s % NS is free once every consumer read slot s - NS
          int mn = 1 << 30;
#pragma unroll
          for (int w = 0; w < CW; ++w)
            mn = min(mn, __hip_atomic_load(&ctl->freed[w], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP));
          if (mn >= s - NS + 1) break;
          if (spins > SPIN_LDS || __hip_atomic_load(&ctl->abort, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP)) {
            dead = true;  // (the error word is written after the loop: no global store in between)
            break;
          }
          __builtin_amdgcn_s_sleep(1);
        }
      const void* g = src_of(s_issue);
      const uint32_t dst = ring0 + (uint32_t)(s % NS) * (SLOT_KB * 1024u);
      asm volatile("s_waitcnt vmcnt(32)\n\t"
                   "ds_write_b128 %[d], %[b0] offset:0\n\t"
                   "ds_write_b128 %[d], %[b1] offset:1024\n\t"
                   "ds_write_b128 %[d], %[b2] offset:2048\n\t"
                   "ds_write_b128 %[d], %[b3] offset:3072\n\t"
                   "ds_write_b128 %[d], %[b4] offset:4096\n\t"
                   "ds_write_b128 %[d], %[b5] offset:5120\n\t"
                   "ds_write_b128 %[d], %[b6] offset:6144\n\t"
                   "ds_write_b128 %[d], %[b7] offset:7168\n\t"
                   "ds_write_b128 %[d], %[b8] offset:8192\n\t"
                   "ds_write_b128 %[d], %[b9] offset:9216\n\t"
                   "ds_write_b128 %[d], %[b10] offset:10240\n\t"
                   "ds_write_b128 %[d], %[b11] offset:11264\n\t"
                   "ds_write_b128 %[d], %[b12] offset:12288\n\t"
                   "ds_write_b128 %[d], %[b13] offset:13312\n\t"
                   "ds_write_b128 %[d], %[b14] offset:14336\n\t"
                   "ds_write_b128 %[d], %[b15] offset:15360\n\t"
                   "s_waitcnt lgkmcnt(0)\n\t" PSE_RL_LOADS
                   : PSE_RL_OPS
                   : [d] "v"(dst), [g] "s"(g), [o0] "v"(voff), [o1] "v"(voff + 4096u), [o2] "v"(voff + 8192u),
                     [o3] "v"(voff + 12288u)
                   : "memory");
      if (!dead && s < total) __hip_atomic_store(&ctl->full[0], s + 1, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
    };
    load(bA, 0);
    load(bB, 1);
    load(bC, 2);
    for (int s = 0; s < total && !dead; s += 3) {
      copy_load(bA, s, s + 3);
      if (s + 1 >= total) break;
      copy_load(bB, s + 1, s + 4);
      if (s + 2 >= total) break;
      copy_load(bC, s + 2, s + 5);
    }
    {  // every load in flight lands before the buffers' registers can be reused
      u32x4(&b)[SLOT_KB] = bA;
      asm volatile("s_waitcnt vmcnt(0)" : PSE_RL_OPS::"memory");
    }
    {
      u32x4(&b)[SLOT_KB] = bB;
      asm volatile("" : PSE_RL_OPS::"memory");
    }
    {
      u32x4(&b)[SLOT_KB] = bC;
      asm volatile("" : PSE_RL_OPS::"memory");
    }
#undef PSE_RL_OPS
#undef PSE_RL_LOADS
    if (dead) st32(a.err, 1u);
    __hip_atomic_store(&ctl->full[0], dead ? 0 : total, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
  } else {
    // =================== consumers ===================
    Ctx x{a.err, a.eps, a.probe, c, lane, wave, (wave - LW) * 64 + lane, epoch, 0};
    if (PSE_GPRIO == 2) __builtin_amdgcn_s_setprio(2);  // (A/B: consumers ahead of the loader always)
    uint32_t* xs32 = reinterpret_cast<uint32_t*>(lds + L_XS);
    bf16_t* xs = reinterpret_cast<bf16_t*>(lds + L_XS);
    float* ssl = reinterpret_cast<float*>(lds + L_MISC);  // [256] gathered sums of squares
    constexpr int NT = H_ / 16;
    const int att_u = LONG ? -1 : pse_att_unit(c, P);
    const int mrg_u = LONG ? pse_merge_unit(c) : -1;
    // The layer loop, instantiated twice: with the attention inlined (the 16 attention CUs) and
    // without it (the rest).  Each instance gets its own register allocation, so the attention's
    // chunk state neither spills the plain CUs' loop nor costs a call: as a noinline callee its
    // ~96 callee-saved VGPRs went to scratch and back every layer (98 KiB each way per CU, 2.8 us
    // of prologue on the attention chain, profiles/r03_n_pse_trace_t2.txt).
    auto run = [&](auto att_c, auto mrg_c) __attribute__((always_inline)) {
      constexpr bool ATT = decltype(att_c)::value;
      constexpr bool MRG = decltype(mrg_c)::value;  // long form: this CU is a merge unit
      // residual columns 16c .. 16c+15 owned by this CU: lanes 0..15 of wave 1 (bf16 values)
      float hres = (wave == LW && lane < 16) ? bf2f(a.h[c * 16 + lane]) : 0.f;
      float hsq = 0.f;
      int seq = 0;  // ring slot sequence number
      // o / d: this lane's output row (wave 1, lanes < 16): hidden = residual + bf16(o)
      // (TF/.../modeling_qwen3.py:311,322), published with its sum of squares
      auto emit_h = [&](int which, uint32_t t, float o, int l) {
        if (wave != LW) return;
        const float hv = rbf(hres + rbf(o));
        hres = lane < 16 ? hv : 0.f;
        const float sq = lane < 16 ? hv * hv : 0.f;
        // the 16 columns' sum of squares in column order, as the GEMV epilogue forms it
        float s16 = 0.f;
  #pragma unroll
        for (int i = 0; i < 16; ++i) s16 += __shfl(sq, i, 64);
        hsq = s16;
        const float hn = __shfl_down(hv, 1, 64);
        if constexpr (PSE_HCNT) {
          // the row (bf16) over the granule region's first 8 KiB, its sums of squares over the ss
          // region's first 1 KiB; drained, then one arrival
          if (lane < 16 && (lane & 1) == 0) st32(reinterpret_cast<bf16_t*>(a.g_h[which]) + c * 16 + lane, pack2(hv, hn));
          if (lane == 0) st32(reinterpret_cast<float*>(a.g_ss[which]) + c, __float_as_uint(s16));
          asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
          typedef __attribute__((address_space(1))) int gi;
          int t = 0;
          if (lane == 0) {
            if (PSE_HTREE) {
              int* gc = a.hcnt + HCNT_GC_OFF + ((size_t)(l * 2 + which) * HGRP + c / (256 / HGRP)) * GCNT_STRIDE;
              t = __hip_atomic_fetch_add((gi*)gc, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
              // the group's last arrival bumps the counter: 8 of them complete it (t = 255 - (8 - 1 - t'))
              t = t == 256 / HGRP - 1
                      ? __hip_atomic_fetch_add((gi*)(a.hcnt + l * 2 + which), 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) +
                            256 - HGRP
                      : -1;
            } else {
              t = __hip_atomic_fetch_add((gi*)(a.hcnt + l * 2 + which), 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            }
          }
          t = __shfl(t, 0, 64);
          if (PSE_HCNT == 2 && t == 255)  // the last producer releases every consumer CU's flag line
#pragma unroll
            for (int i = 0; i < 4; ++i) st32(a.go + ((size_t)(l * 2 + which) * 256 + lane + 64 * i) * 32, epoch);
        } else {
          if (lane < 16 && (lane & 1) == 0) st64(a.g_h[which] + c * 8 + lane / 2, gran(pack2(hv, hn), t));
          if (lane == 0) st64(a.g_ss[which] + c, gran(__float_as_uint(s16), t));
        }
      };

      for (int l = 0; l < a.layers && !failed(x); ++l) {
        const PseLayer& Lw = a.L[l];
        if (wave == LW) PSE_STAMP(l, 0);
        // ---------------- q|k|v (input RMSNorm fused) ----------------
        // Ring slot drain (plain CUs, SlotCache): while the consumer waves wait for the attention
        // output they copy o_proj's first RC ring slots into registers as they land, which lets the
        // loader run RC slots further ahead through the attention (the longest wait of the layer);
        // o_proj then runs those slots from registers.  (At the h gathers the same drain spilled
        // 44+ VGPRs even at 2 slots: not used there.)
        // (long form: 0 -- live across the slice call, the drained slots spill: 33 VGPRs at 2 slots)
        constexpr int RC = (ATT || MRG || LONG) ? 0 : (PSE_RC < 8 ? PSE_RC : 8);
        NormW nw;
        auto load_nw = [&]() { nw = norm_w(x, Lw.in_norm); };
        bool normed = false;
        if (l == 0) {  // the embedding row and its sums of squares (previous launch)
          load_nw();
          for (int i = x.tid; i < H_ / 2; i += CW * 64) xs32[i] = reinterpret_cast<const uint32_t*>(a.h)[i];
          for (int i = x.tid; i < NT; i += CW * 64) ssl[i] = a.ss[i];
          cbar(x);
        } else if (PSE_HCNT) {
          if (!hnorm_counter(x, a.hcnt, a.go, (l - 1) * 2 + 1, reinterpret_cast<const bf16_t*>(a.g_h[1]),
                             reinterpret_cast<const float*>(a.g_ss[1]), xs, load_nw, nw))
            break;
          normed = true;
        } else {
  #if PSE_TRACE2
          x.tp = a.trace ? a.trace + ((size_t)l * PSE_TRACE_EV + 10) * 256 + c : nullptr;  // events 10-14
  #endif
          const bool ok = gather<9>(x, a.g_h[1], H_ / 2 + NT, tagof(epoch, l - 1, OP_DOWN), xs32, H_ / 2,
                                    reinterpret_cast<uint32_t*>(ssl), load_nw);
  #if PSE_TRACE2
          x.tp = nullptr;
  #endif
          if (!ok) break;
        }
        if (!normed) norm_stage(x, xs, ssl, NT, nw);
        if (wave == LW) PSE_STAMP(l, 1);
        const uint32_t tq = tagof(epoch, l, OP_QKV);
        #pragma unroll 1
        for (int j = 0; j < (ATT ? 2 : nq); ++j) {
          int tile, half;
          pse_qkv_unit(c, j, &tile, &half);
          f32x4 acc = (f32x4){0.f, 0.f, 0.f, 0.f};
          #pragma unroll 1
          for (int k = 0; k < 4; ++k) consume_slot(x, seq++, half * 64 + k * 16, acc);
          PSE_PRIO_UP();
          red_put(x, 0, acc);
          cbar(x);
          if (wave == LW && lane < 16)
            st64(a.g_qkv + qkv_gran(tile) + half * 16 + lane, gran(__float_as_uint(red_get(x, 0, lane)), tq));
          cbar(x);
          PSE_PRIO_DOWN();
        }
        if (wave == LW) PSE_STAMP(l, 2);
        // ---------------- attention (one CU per KV head) ----------------
        if constexpr (ATT) {
          // the head's q|k|v partials (grouped by KV head, qkv_gran): [tile][half][16]
          auto att = [&](auto ku_c) {
            return attention<decltype(ku_c)::value>(a.L + l, a.pos, a.mask, a.cos_t, a.sin_t, a.g_qkv, a.g_att, a.g_part,
                                                    a.err, a.trace, a.eps, a.scale, a.Cmax, epoch, x.bar_gen, l, att_u, tq);
          };
          // (key split: role 0 = unit 0 of its KV head, 1 = the others)
          const int bg = !PSE_KSPLIT ? att(IntC<-1>{}) : (att_u % PSE_AU == 0 ? att(IntC<0>{}) : att(IntC<1>{}));
          const bool att_ok = bg >= 0;
          if (att_ok) x.bar_gen = bg;
          if (PSE_APAUSE == 2 && x.tid == 0)  // (PSE_APAUSE 2: the loader waits out the whole attention)
            __hip_atomic_store(&PSE_CTL->apause, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
          if (!att_ok) break;
          if (wave == LW) PSE_STAMP(l, 3);
        }
        if constexpr (LONG) {
          // every CU: its slice of the KV head's cached keys; merge units then combine the slices
          int bg = MRG ? attention_slice<true>(a.L + l, a.pos, a.mask, a.cos_t, a.sin_t, a.g_qkv, a.g_part, a.err,
                                               a.eps, a.scale, a.Cmax, epoch, x.bar_gen, l, tq)
                       : attention_slice<false>(a.L + l, a.pos, a.mask, a.cos_t, a.sin_t, a.g_qkv, a.g_part, a.err,
                                                a.eps, a.scale, a.Cmax, epoch, x.bar_gen, l, tq);
          if (bg >= 0) x.bar_gen = bg;
          if (MRG && bg >= 0) {
            bg = attention_merge(a.L + l, a.pos, a.g_part, a.g_att, a.err, a.eps, a.scale, a.Cmax, epoch, x.bar_gen, l,
                                 mrg_u);
            if (bg >= 0) x.bar_gen = bg;
          }
          if (x.tid == 0) __hip_atomic_store(&PSE_CTL->apause, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
          if (bg < 0) break;
          if (wave == LW) PSE_STAMP(l, 3);
        }
        // ---------------- o_proj (+ residual) ----------------
        // (plain CUs: the o_proj slots drain into registers while the attention runs elsewhere)
        SlotCache<RC> co;
        if (!gather<8, false>(x, a.g_att, HQ_ * D_ / 2, tagof(epoch, l, OP_ATT), xs32, HQ_ * D_ / 2, nullptr, NoHook(),
                              [&]() { co.drain(x, seq); }))
          break;
        if (wave == LW) PSE_STAMP(l, 4);
        {
          f32x4 acc = (f32x4){0.f, 0.f, 0.f, 0.f};
#pragma unroll
          for (int k = 0; k < RC; ++k) co.take(x, seq, k, k * 16, acc);
          #pragma unroll 1
          for (int k = RC; k < 8; ++k) consume_slot(x, seq++, k * 16, acc);
          PSE_PRIO_UP();
          red_put(x, 0, acc);
          cbar(x);
          emit_h(0, tagof(epoch, l, OP_O), lane < 16 ? red_get(x, 0, lane) : 0.f, l);
          cbar(x);
          PSE_PRIO_DOWN();
        }
        if (wave == LW) PSE_STAMP(l, 5);
        // ---------------- gate|up (post-attention RMSNorm fused, SwiGLU) ----------------
        if (PSE_HCNT) {
          if (!hnorm_counter(x, a.hcnt, a.go, l * 2, reinterpret_cast<const bf16_t*>(a.g_h[0]),
                             reinterpret_cast<const float*>(a.g_ss[0]), xs, [&]() { nw = norm_w(x, Lw.post_norm); }, nw))
            break;
        } else {
          if (!gather<9>(x, a.g_h[0], H_ / 2 + NT, tagof(epoch, l, OP_O), xs32, H_ / 2, reinterpret_cast<uint32_t*>(ssl),
                         [&]() { nw = norm_w(x, Lw.post_norm); }))
            break;
          norm_stage(x, xs, ssl, NT, nw);
        }
        if (wave == LW) PSE_STAMP(l, 6);
        const uint32_t tg = tagof(epoch, l, OP_GU);
        auto gu_round = [&](int j) {
          f32x4 ag = (f32x4){0.f, 0.f, 0.f, 0.f}, au = ag;
          #pragma unroll 1
          for (int k = 0; k < 8; ++k) consume_slot(x, seq++, k * 16, ag);
          #pragma unroll 1
          for (int k = 0; k < 8; ++k) consume_slot(x, seq++, k * 16, au);
          PSE_PRIO_UP();
          red_put(x, 0, ag);
          red_put(x, 1, au);
          cbar(x);
          if (wave == LW) {
            // bf16(bf16(silu(bf16 g)) * bf16 u)   (TF/.../modeling_qwen3.py:81-83)
            const float gg = rbf(red_get(x, 0, lane & 15)), uu = rbf(red_get(x, 1, lane & 15));
            const float o = rbf(rbf(gg / (1.0f + expf(-gg))) * uu);
            const float on = __shfl_down(o, 1, 64);
            if (lane < 16 && (lane & 1) == 0) st64(a.g_act + pse_gu_pair(c, j) * 8 + lane / 2, gran(pack2(o, on), tg));
          }
          cbar(x);
          PSE_PRIO_DOWN();
        };
        gu_round(0);
        gu_round(1);
        // round 2 runs inside the gather of round 0's columns (published a round ago) -> xs
        // k-tiles 128 .. 255 (the normed input in k-tiles 0 .. 127 is still being read)
        auto gu2 = [&]() {
          if (PSE_GPRIO) __builtin_amdgcn_s_setprio(0);
          gu_round(2);
          if (PSE_GPRIO) __builtin_amdgcn_s_setprio(3);
        };
        if (!gather<8, false>(x, a.g_act, I_ / 6, tg, xs32 + I_ / 6, I_ / 6, nullptr, gu2)) break;
        if (wave == LW) PSE_STAMP(l, 7);
        // ---------------- down (+ residual) ----------------
        if (wave == LW) PSE_STAMP(l, 8);
        {
          // down's k-slots 8j .. 8j+7 read round j's columns: round 0 in xs k-tiles 128 .. 255,
          // round 1 gathered into 256 .. 383 while round 0's slots run, round 2 into 0 .. 127 (the
          // normed input is dead by then) while round 1's slots run
          f32x4 acc = (f32x4){0.f, 0.f, 0.f, 0.f};
          auto slots = [&](int k0, int off) {
            if (PSE_GPRIO) __builtin_amdgcn_s_setprio(0);
            #pragma unroll 1
            for (int k = k0; k < k0 + 8; ++k) consume_slot(x, seq++, k * 16 + off, acc);
            if (PSE_GPRIO) __builtin_amdgcn_s_setprio(3);
          };
          if (!gather<8, false>(x, a.g_act + I_ / 6, I_ / 6, tg, xs32 + I_ / 3, I_ / 6, nullptr, [&]() { slots(0, 128); })) break;
          if (!gather<8, false>(x, a.g_act + I_ / 3, I_ / 6, tg, xs32, I_ / 6, nullptr, [&]() { slots(8, 128); })) break;
          #pragma unroll 1
          for (int k = 16; k < 24; ++k) consume_slot(x, seq++, k * 16 - 256, acc);
          PSE_PRIO_UP();
          red_put(x, 0, acc);
          cbar(x);
          emit_h(1, tagof(epoch, l, OP_DOWN), lane < 16 ? red_get(x, 0, lane) : 0.f, l);
          cbar(x);
          PSE_PRIO_DOWN();
        }
        if (wave == LW) PSE_STAMP(l, 9);
        if (a.trace && wave == LW && lane < 5 && !PSE_TRACE2)
          a.trace[((size_t)l * PSE_TRACE_EV + 10 + lane) * 256 + c] = ctl->lstamp[l & 1][lane];
      }
      // the final residual and its sums of squares for the heads (plain stores: the next launch)
      if (wave == LW && lane < 16) a.h[c * 16 + lane] = f2bf(hres);
      if (wave == LW && lane == 0) a.ss[c] = hsq;
    };
    if constexpr (LONG) {
      if (mrg_u >= 0) run(BoolC<false>{}, BoolC<true>{});
      else run(BoolC<false>{}, BoolC<false>{});
    } else {
      if (att_u >= 0) run(BoolC<true>{}, BoolC<false>{});
      else run(BoolC<false>{}, BoolC<false>{});
    }
  }
  // exit: the last workgroup out advances the epoch for the next launch
  __syncthreads();
  if (threadIdx.x == 0) {
    const uint32_t t = __hip_atomic_fetch_add((g32*)a.exit_cnt, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (t == (uint32_t)P - 1) {
      if (PSE_HCNT)
        for (int k = 0; k < 2 * a.layers; ++k) st32(a.hcnt + k, 0u);
      if (PSE_HCNT && PSE_HTREE)
        for (int k = 0; k < 2 * a.layers * HGRP; ++k) st32(a.hcnt + HCNT_GC_OFF + (size_t)k * GCNT_STRIDE, 0u);
      st32(a.exit_cnt, 0u);
      st32(a.epoch, epoch);
    }
  }
}

// ---------------------------------------------------------------------------
bool pse_supported(int device, int B, int layers, int H, int Hq, int Hkv, int D, int I, int qkv_rows, int Cmax) {
  if (B != 1 || H != H_ || Hq != HQ_ || Hkv != HKV_ || D != D_ || I != I_ || qkv_rows != QKVR_ || Cmax % 64) return false;
  // the loader's pointer table holds PSE_MAXL layers; a hand-off tag carries layer * 5 + op in 8 bits
  if (layers < 1 || layers > PSE_MAXL || layers * 5 > 256) return false;
  return pse_grid(device) == 256;
}

int pse_grid(int device) {
  hipDeviceProp_t p;
  if (hipGetDeviceProperties(&p, device) != hipSuccess) return 0;
  for (const void* k : {(const void*)pse_kernel_t<false>, (const void*)pse_kernel_t<true>}) {
    if (hipFuncSetAttribute(k, hipFuncAttributeMaxDynamicSharedMemorySize, (int)pse_lds_bytes()) != hipSuccess) return 0;
    int per_cu = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, k, THREADS, pse_lds_bytes()) != hipSuccess || per_cu < 1)
      return 0;
  }
  return p.multiProcessorCount;
}

size_t pse_ws_bytes() {
  // granules: q|k|v partials (768 units x 16), attention (2048), h x 2 (2048), ss x 2 (256),
  // act (6144); words: error, epoch, exit count
  return (size_t)(768 * 16 + NG_ATT + 2 * (H_ / 2) + 2 * (H_ / 16) + I_ / 2 + NG_PART) * 8 + HCNT_GC_OFF * 4 +
         (PSE_HCNT && PSE_HTREE ? (size_t)2 * PSE_MAXL * HGRP * GCNT_STRIDE * 4 : 0) + 64;
}

hipError_t pse_decode(const PseArgs& a0, void* ws, hipStream_t s, bool coop, bool long_ctx) {
  if (a0.layers < 1 || a0.layers > PSE_MAXL || a0.layers * 5 > 256 || a0.Cmax % 64) return hipErrorInvalidValue;
  PseArgs a = a0;
  uint64_t* g = reinterpret_cast<uint64_t*>(ws);
  a.g_qkv = g; g += 768 * 16;
  a.g_att = g; g += NG_ATT;
  // h granules of an op immediately followed by its sums of squares: one gather range
  a.g_h[0] = g; g += H_ / 2;
  a.g_ss[0] = g; g += H_ / 16;
  a.g_h[1] = g; g += H_ / 2;
  a.g_ss[1] = g; g += H_ / 16;
  a.g_act = g; g += I_ / 2;
  a.g_part = g; g += NG_PART;
  a.hcnt = reinterpret_cast<int*>(g);
  a.go = reinterpret_cast<uint32_t*>(reinterpret_cast<unsigned char*>(g) + 2 * PSE_MAXL * 4);
  uint32_t* w = reinterpret_cast<uint32_t*>(reinterpret_cast<unsigned char*>(ws) + pse_ws_bytes() - 64);
  a.err = w; a.epoch = w + 1; a.exit_cnt = w + 2;
  const void* k = long_ctx ? (const void*)pse_kernel_t<true> : (const void*)pse_kernel_t<false>;
  if (coop) {
    void* args[] = {&a};
    return hipLaunchCooperativeKernel(k, dim3(256), dim3(THREADS), args, (unsigned)pse_lds_bytes(), s);
  }
  if (long_ctx) hipLaunchKernelGGL(pse_kernel_t<true>, dim3(256), dim3(THREADS), pse_lds_bytes(), s, a);
  else hipLaunchKernelGGL(pse_kernel_t<false>, dim3(256), dim3(THREADS), pse_lds_bytes(), s, a);
  return hipGetLastError();
}

uint32_t* pse_err_word(void* ws) {
  return reinterpret_cast<uint32_t*>(reinterpret_cast<unsigned char*>(ws) + pse_ws_bytes() - 64);
}

}  // namespace mtts
