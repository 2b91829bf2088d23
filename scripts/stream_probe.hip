// Weight-stream probe: how fast can one decode step's gate|up matrix (201 MB, 1 KiB tiles) be
// streamed from HBM (a) into VGPRs (the GEMV's way: 8 tiles in flight per wave, nt) and (b) into
// LDS by LDS-DMA (global_load_lds_dwordx4 nt, a ring per CU, L loader waves)?  No arithmetic:
// the bytes are XOR-folded so nothing is dead.  Matrices rotate over 8 copies (1.6 GB) so no
// launch finds its bytes in the 256 MB MALL.
//   hipcc --offload-arch=gfx950 -O3 -o scripts/stream_probe scripts/stream_probe.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>

typedef __attribute__((ext_vector_type(4))) unsigned int u32x4;
#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP %s @%d\n", hipGetErrorString(e_), __LINE__); exit(1); } } while (0)

constexpr size_t TILE = 1024;

// (a) registers: block = NW waves, each wave a contiguous run of tiles, U in flight
template <int NW, int U>
__global__ __launch_bounds__(NW * 64) void reg_stream(const u32x4* __restrict__ w, size_t tiles_per_block, unsigned* out) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const size_t per = (tiles_per_block + NW - 1) / NW;
  const size_t t0 = blockIdx.x * tiles_per_block + wave * per;
  const size_t t1 = blockIdx.x * tiles_per_block + (wave + 1 == NW ? tiles_per_block : (wave + 1) * per);
  u32x4 acc = {0u, 0u, 0u, 0u};
  for (size_t t = t0; t < t1; t += U) {
    u32x4 v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) v[u] = __builtin_nontemporal_load(w + (t + u < t1 ? t + u : t1 - 1) * 64 + lane);
#pragma unroll
    for (int u = 0; u < U; ++u) acc ^= v[u];
  }
  if ((acc.x ^ acc.y ^ acc.z ^ acc.w) == 0x12345678u) out[blockIdx.x] = 1;
}

// (b) LDS-DMA: L loader waves per block, each keeps D tiles (1 KiB each) in flight into its own
// ring of R slots; a consumer-free ring (overwritten), then one read so the data is live
template <int L, int D>
__global__ __launch_bounds__(L * 64) void lds_stream(const u32x4* __restrict__ w, size_t tiles_per_block, unsigned* out) {
  constexpr int R = 2 * D;
  extern __shared__ __attribute__((aligned(16))) unsigned char ring[];  // [L][R][1 KiB]
  typedef __attribute__((address_space(1))) void gvoid;
  typedef __attribute__((address_space(3))) void lvoid;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const size_t per = (tiles_per_block + L - 1) / L;
  const size_t t0 = blockIdx.x * tiles_per_block + wave * per;
  size_t t1 = t0 + per;
  if (t1 > (blockIdx.x + 1) * tiles_per_block) t1 = (blockIdx.x + 1) * tiles_per_block;
  unsigned char* my = ring + (size_t)wave * R * TILE;
  int slot = 0;
  for (size_t t = t0; t < t1; ++t) {
    __builtin_amdgcn_global_load_lds((const gvoid*)(w + t * 64 + lane), (lvoid*)(my + slot * TILE), 16, 0, 2);
    slot = slot + 1 == R ? 0 : slot + 1;
    if (((t - t0) % D) == D - 1) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(D) : "memory");  // keep ~D..2D in flight
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  const unsigned v = reinterpret_cast<const unsigned*>(my)[lane];
  if (v == 0x12345678u) out[blockIdx.x] = 1;
}

int main() {
  const size_t bytes = 201359360;  // gate|up of one 8B layer: 24576 x 4096 bf16
  const size_t tiles = bytes / TILE;
  const int copies = 8;
  u32x4* w;
  CK(hipMalloc(&w, bytes * copies));
  CK(hipMemset(w, 1, bytes * copies));
  unsigned* out;
  CK(hipMalloc(&out, 65536 * 4));
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  auto run = [&](const char* name, auto launch) {
    for (int i = 0; i < 8; ++i) launch((const u32x4*)((const char*)w + (i % copies) * bytes));
    CK(hipDeviceSynchronize());
    const int iters = 40;
    CK(hipEventRecord(a));
    for (int i = 0; i < iters; ++i) launch((const u32x4*)((const char*)w + (i % copies) * bytes));
    CK(hipEventRecord(b));
    CK(hipEventSynchronize(b));
    float ms;
    CK(hipEventElapsedTime(&ms, a, b));
    const double us = ms * 1e3 / iters;
    printf("%-34s %8.2f us  %6.2f TB/s\n", name, us, bytes / (us * 1e-6) / 1e12);
  };
  // the GEMV's geometry: 768 blocks x 8 waves (gate|up, RT = 2), 8 tiles in flight per wave
  run("reg 768x8w U8", [&](const u32x4* p) { reg_stream<8, 8><<<768, 512>>>(p, tiles / 768, out); });
  run("reg 768x8w U16", [&](const u32x4* p) { reg_stream<8, 16><<<768, 512>>>(p, tiles / 768, out); });
  run("reg 512x8w U8", [&](const u32x4* p) { reg_stream<8, 8><<<512, 512>>>(p, tiles / 512, out); });
  run("reg 256x16w U8", [&](const u32x4* p) { reg_stream<16, 8><<<256, 1024>>>(p, tiles / 256, out); });
  run("reg 1536x4w U8", [&](const u32x4* p) { reg_stream<4, 8><<<1536, 256>>>(p, tiles / 1536, out); });
  run("reg 3072x4w U8", [&](const u32x4* p) { reg_stream<4, 8><<<3072, 256>>>(p, tiles / 3072, out); });
  auto lds = [&](const char* name, auto kern, int L, int D, int blocks) {
    const size_t l = (size_t)L * 2 * D * TILE;
    CK(hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)l));
    run(name, [&](const u32x4* p) { kern<<<blocks, L * 64, l>>>(p, tiles / blocks, out); });
  };
  lds("lds 256 L1 D16", lds_stream<1, 16>, 1, 16, 256);
  lds("lds 256 L1 D32", lds_stream<1, 32>, 1, 32, 256);
  lds("lds 256 L2 D16", lds_stream<2, 16>, 2, 16, 256);
  lds("lds 256 L4 D8", lds_stream<4, 8>, 4, 8, 256);
  lds("lds 256 L4 D16", lds_stream<4, 16>, 4, 16, 256);
  lds("lds 512 L2 D16", lds_stream<2, 16>, 2, 16, 512);
  lds("lds 768 L2 D8", lds_stream<2, 8>, 2, 8, 768);
  return 0;
}
