// Hand-off latency probe: how long does ONE poll load take while HBM streams, and whose stream
// delays it?  256 workgroups (one per CU) of 2 waves: wave 0 streams its stripe of a 4 GB buffer
// (register loads, ~32 KiB in flight per wave, nt -- the PSE loader's shape), wave 1 of workgroup 0
// times single loads with s_memrealtime (10 ns ticks):
//   vec fresh   -- sc1 vector load of a line nobody touched (HBM)
//   vec hot     -- sc1 vector load of a line another CU just wrote with an sc1 store (the hand-off)
//   scal fresh  -- glc scalar load of an untouched line (the scalar cache path, not the vector one)
// Modes: which CUs stream -- none / the probing CU only / every other CU / all.
//   hipcc --offload-arch=gfx950 -O3 -o scripts/lat_probe scripts/lat_probe.hip
#include <hip/hip_runtime.h>
#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <vector>

typedef __attribute__((ext_vector_type(4))) unsigned int u32x4;
#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP %s @%d\n", hipGetErrorString(e_), __LINE__); exit(1); } } while (0)

constexpr int NPROBE = 256;
constexpr size_t STRIPE = 16u << 20;  // bytes per workgroup

__device__ __forceinline__ uint64_t now() { return __builtin_amdgcn_s_memrealtime(); }

__global__ __launch_bounds__(128) void lat_kernel(const u32x4* big, unsigned* fresh, unsigned* hot, uint64_t* out,
                                                  int mode, int kind, unsigned* sink) {
  __shared__ int stop;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, c = blockIdx.x;
  if (threadIdx.x == 0) stop = 0;
  __syncthreads();
  const uint64_t t_start = now();
  const bool stream = (c == 0) ? (mode & 1) : (mode & 2);
  if (wave == 0) {
    if (!stream) return;
    const u32x4* p = big + (size_t)c * (STRIPE / 16);
    u32x4 acc = {0u, 0u, 0u, 0u};
    size_t off = 0;
    // stream until workgroup 0's prober is done (its flag), or 3 ms
    for (int it = 0;; ++it) {
      u32x4 v[32];
#pragma unroll
      for (int u = 0; u < 32; ++u) v[u] = __builtin_nontemporal_load(p + off + u * 64 + lane);
#pragma unroll
      for (int u = 0; u < 32; ++u) acc ^= v[u];
      off = (off + 32 * 64) % (STRIPE / 16);
      if (c == 0 && __hip_atomic_load(&stop, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP)) break;
      if (now() - t_start > 300000) break;
    }
    if ((acc.x ^ acc.y ^ acc.z ^ acc.w) == 0x9e3779b9u) sink[c] = 1;
    return;
  }
  // wave 1
  if (kind == 1 && c == 128) {  // the hot-line writer: one sc1 store per probe slot, 2 us apart
    while (now() - t_start < 10000) __builtin_amdgcn_s_sleep(10);
    for (int i = 0; i < NPROBE; ++i) {
      if (lane == 0) __hip_atomic_store(hot + i * 16, (unsigned)(i + 1), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      const uint64_t t = now();
      while (now() - t < 400) __builtin_amdgcn_s_sleep(10);
    }
    return;
  }
  if (c != 0) return;
  while (now() - t_start < 10000) __builtin_amdgcn_s_sleep(10);  // 100 us: let the streams ramp
  for (int i = 0; i < NPROBE; ++i) {
    uint64_t t0, t1;
    unsigned v = 0;
    if (kind == 0) {  // fresh line, vector sc1
      t0 = now();
      v = __hip_atomic_load(fresh + (size_t)i * 4096, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __builtin_amdgcn_s_waitcnt(0);
      asm volatile("" ::"v"(v));
      t1 = now();
    } else if (kind == 1) {  // the writer's line: poll until it carries i + 1, time the final poll
      unsigned spins = 0;
      do {
        t0 = now();
        v = __hip_atomic_load(hot + i * 16, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        asm volatile("" ::"v"(v));
        t1 = now();
      } while (v != (unsigned)(i + 1) && ++spins < 100000);
    } else {  // fresh line, scalar glc
      const unsigned* a = fresh + (size_t)(i + NPROBE) * 4096;
      const uint64_t pa = (uint64_t)(uintptr_t)a;
      const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)pa), hi = __builtin_amdgcn_readfirstlane((uint32_t)(pa >> 32));
      const uint64_t sa = ((uint64_t)hi << 32) | lo;
      unsigned sv;
      t0 = now();
      asm volatile("s_nop 4\n\ts_load_dword %0, %1, 0x0 glc\n\ts_waitcnt lgkmcnt(0)" : "=s"(sv) : "s"(sa) : "memory");
      t1 = now();
      v = sv;
    }
    if (lane == 0) out[i] = (t1 - t0) | ((uint64_t)(v & 0xffff) << 48);
  }
  if (lane == 0) __hip_atomic_store(&stop, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}

int main() {
  const size_t big_bytes = STRIPE * 256;
  u32x4* big;
  unsigned *fresh, *hot, *sink;
  uint64_t* out;
  CK(hipMalloc(&big, big_bytes));
  CK(hipMemset(big, 1, big_bytes));
  const size_t fresh_bytes = (size_t)64 * NPROBE * 4096 * 4;  // 64 probe runs' worth of untouched lines
  CK(hipMalloc(&fresh, fresh_bytes));
  CK(hipMemset(fresh, 0, fresh_bytes));
  CK(hipMalloc(&hot, NPROBE * 64));
  CK(hipMalloc(&sink, 256 * 4));
  CK(hipMalloc(&out, NPROBE * 8));
  const char* mname[4] = {"no stream", "own CU streams", "other CUs stream", "all CUs stream"};
  const char* kname[3] = {"vec sc1 fresh", "vec sc1 hot (remote CU store)", "scalar glc fresh"};
  int run = 0;
  for (int kind = 0; kind < 3; ++kind)
    for (int mode = 0; mode < 4; ++mode) {
      // rotate the flush region: 1 GB of other bytes between runs evicts the MALL
      CK(hipMemset(big, run & 255, big_bytes / 4));
      CK(hipMemset(hot, 0, NPROBE * 64));
      CK(hipDeviceSynchronize());
      unsigned* fr = fresh + (size_t)(run % 32) * 2 * NPROBE * 4096;
      ++run;
      lat_kernel<<<256, 128>>>(big, fr, hot, out, mode, kind, sink);
      CK(hipGetLastError());
      CK(hipDeviceSynchronize());
      std::vector<uint64_t> h(NPROBE);
      CK(hipMemcpy(h.data(), out, NPROBE * 8, hipMemcpyDeviceToHost));
      std::vector<double> us;
      for (auto x : h) us.push_back((double)(x & 0xffffffffffffull) / 100.0);
      std::sort(us.begin(), us.end());
      printf("%-30s %-18s  p10 %.2f  p50 %.2f  p90 %.2f  max %.2f us\n", kname[kind], mname[mode], us[NPROBE / 10],
             us[NPROBE / 2], us[NPROBE * 9 / 10], us.back());
      fflush(stdout);
    }
  return 0;
}
