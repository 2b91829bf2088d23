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
constexpr size_t STRIPE = 16u << 20;  // bytes per workgroup (a multiple of 16 KiB)

__device__ __forceinline__ uint64_t now() { return __builtin_amdgcn_s_memrealtime(); }

__global__ __launch_bounds__(128) void lat_kernel(const u32x4* big, unsigned* fresh, unsigned* hot, uint64_t* out,
                                                  int d_own, int d_oth, int kind, unsigned* sink) {
  __shared__ int stop;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, c = blockIdx.x;
  if (threadIdx.x == 0) stop = 0;
  __syncthreads();
  const uint64_t t_start = now();
  if (wave == 0) {
    const int depth = (c == 0) ? d_own : d_oth;
    if (depth == 0) return;
    // the PSE loader's shape: `depth` buffers of 16 x 16 B per lane (16 KiB per wave), each
    // reloaded as soon as it lands (s_waitcnt vmcnt(16 (depth - 1))), nt loads
    const char* base = reinterpret_cast<const char*>(big) + (size_t)c * STRIPE;
    const uint32_t voff = (uint32_t)lane * 16u;
    u32x4 bA[16], bB[16], bC[16];
    uint64_t off = 0;
    int n = 0;
#define LP_OPS [b0] "+v"(b[0]), [b1] "+v"(b[1]), [b2] "+v"(b[2]), [b3] "+v"(b[3]), [b4] "+v"(b[4]), [b5] "+v"(b[5]), \
      [b6] "+v"(b[6]), [b7] "+v"(b[7]), [b8] "+v"(b[8]), [b9] "+v"(b[9]), [b10] "+v"(b[10]), [b11] "+v"(b[11]),  \
      [b12] "+v"(b[12]), [b13] "+v"(b[13]), [b14] "+v"(b[14]), [b15] "+v"(b[15])
#define LP_LOADS "s_nop 4\n\t" \
  "global_load_dwordx4 %[b0], %[o0], %[g] offset:0 nt\n\tglobal_load_dwordx4 %[b1], %[o0], %[g] offset:1024 nt\n\t" \
  "global_load_dwordx4 %[b2], %[o0], %[g] offset:2048 nt\n\tglobal_load_dwordx4 %[b3], %[o0], %[g] offset:3072 nt\n\t" \
  "global_load_dwordx4 %[b4], %[o1], %[g] offset:0 nt\n\tglobal_load_dwordx4 %[b5], %[o1], %[g] offset:1024 nt\n\t" \
  "global_load_dwordx4 %[b6], %[o1], %[g] offset:2048 nt\n\tglobal_load_dwordx4 %[b7], %[o1], %[g] offset:3072 nt\n\t" \
  "global_load_dwordx4 %[b8], %[o2], %[g] offset:0 nt\n\tglobal_load_dwordx4 %[b9], %[o2], %[g] offset:1024 nt\n\t" \
  "global_load_dwordx4 %[b10], %[o2], %[g] offset:2048 nt\n\tglobal_load_dwordx4 %[b11], %[o2], %[g] offset:3072 nt\n\t" \
  "global_load_dwordx4 %[b12], %[o3], %[g] offset:0 nt\n\tglobal_load_dwordx4 %[b13], %[o3], %[g] offset:1024 nt\n\t" \
  "global_load_dwordx4 %[b14], %[o3], %[g] offset:2048 nt\n\tglobal_load_dwordx4 %[b15], %[o3], %[g] offset:3072 nt\n\t"
    // buffer b: wait until its previous loads landed (the `depth` - 1 younger buffers' 16 loads
    // each may stay in flight), then reload it -- the PSE loader without the LDS copy
    auto step = [&](u32x4 (&b)[16]) {
      const uint64_t p = (uint64_t)(uintptr_t)(base + off);
      const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)p), hi = __builtin_amdgcn_readfirstlane((uint32_t)(p >> 32));
      const void* g = (const void*)(((uint64_t)hi << 32) | lo);
      if (depth >= 3) asm volatile("s_waitcnt vmcnt(32)\n\t" LP_LOADS : LP_OPS : [g] "s"(g), [o0] "v"(voff), [o1] "v"(voff + 4096u), [o2] "v"(voff + 8192u), [o3] "v"(voff + 12288u) : "memory");
      else if (depth == 2) asm volatile("s_waitcnt vmcnt(16)\n\t" LP_LOADS : LP_OPS : [g] "s"(g), [o0] "v"(voff), [o1] "v"(voff + 4096u), [o2] "v"(voff + 8192u), [o3] "v"(voff + 12288u) : "memory");
      else asm volatile("s_waitcnt vmcnt(0)\n\t" LP_LOADS : LP_OPS : [g] "s"(g), [o0] "v"(voff), [o1] "v"(voff + 4096u), [o2] "v"(voff + 8192u), [o3] "v"(voff + 12288u) : "memory");
      off = (off + 16384) % STRIPE;
      ++n;
    };
    for (;;) {
      step(bA);
      if (depth >= 2) step(bB);
      if (depth >= 3) step(bC);
      if (c == 0 && __hip_atomic_load(&stop, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP)) break;
      if ((n & 15) < 3 && now() - t_start > 300000) break;
    }
    {
      u32x4(&b)[16] = bA;
      asm volatile("s_waitcnt vmcnt(0)" : LP_OPS : : "memory");
    }
    {
      u32x4(&b)[16] = bB;
      asm volatile("" : LP_OPS : : "memory");
    }
    {
      u32x4(&b)[16] = bC;
      asm volatile("" : LP_OPS : : "memory");
    }
    if (lane == 0) sink[c] = (unsigned)n;  // slots streamed (16 KiB each)
    if (lane == 0 && c == 0) sink[256] = (unsigned)(now() - t_start);
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
  CK(hipMalloc(&sink, 257 * 4));
  CK(hipMalloc(&out, NPROBE * 8));
  const char* kname[3] = {"vec sc1 fresh", "vec sc1 hot (remote CU store)", "scalar glc fresh"};
  const int cfg[][2] = {{0, 0}, {3, 0}, {0, 1}, {0, 2}, {0, 3}, {1, 3}, {2, 3}, {3, 3}};
  int run = 0;
  for (int kind = 0; kind < 3; ++kind)
    for (auto& cf : cfg) {
      CK(hipMemset(big, run & 255, big_bytes / 4));  // 1 GB of other bytes between runs evicts the MALL
      CK(hipMemset(hot, 0, NPROBE * 64));
      CK(hipMemset(sink, 0, 257 * 4));
      CK(hipDeviceSynchronize());
      unsigned* fr = fresh + (size_t)(run % 24) * 2 * NPROBE * 4096;
      ++run;
      hipEvent_t e0, e1;
      CK(hipEventCreate(&e0));
      CK(hipEventCreate(&e1));
      CK(hipEventRecord(e0));
      lat_kernel<<<256, 128>>>(big, fr, hot, out, cf[0], cf[1], kind, sink);
      CK(hipGetLastError());
      CK(hipEventRecord(e1));
      CK(hipDeviceSynchronize());
      float ms = 0.f;
      CK(hipEventElapsedTime(&ms, e0, e1));
      std::vector<uint64_t> h(NPROBE);
      CK(hipMemcpy(h.data(), out, NPROBE * 8, hipMemcpyDeviceToHost));
      std::vector<unsigned> sk(257);
      CK(hipMemcpy(sk.data(), sink, 257 * 4, hipMemcpyDeviceToHost));
      double slots = 0;
      for (int i = 1; i < 256; ++i) slots += sk[i];
      std::vector<double> us;
      for (auto x : h) us.push_back((double)(x & 0xffffffffffffull) / 100.0);
      std::sort(us.begin(), us.end());
      printf("%-30s own %d x16K others %d x16K  p10 %.2f  p50 %.2f  p90 %.2f  max %.2f us | others' stream %.2f TB/s, own %.1f GB/s\n",
             kname[kind], cf[0], cf[1], us[NPROBE / 10], us[NPROBE / 2], us[NPROBE * 9 / 10], us.back(),
             cf[1] ? slots * 16384.0 / (3e-3) / 1e12 : 0.0, sk[256] ? sk[0] * 16384.0 / (sk[256] * 1e-8) / 1e9 : 0.0);
      fflush(stdout);
    }
  return 0;
}
