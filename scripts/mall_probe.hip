// Infinity Cache (MALL) prefetch probe: does touching a weight region (one dword per 128-B line)
// make a later full stream of it faster, and how fast do touches cover bytes?
//   cold    -- stream R (register loads, 3 x 16 KiB in flight per wave, nt: the PSE loader's shape)
//   touch   -- one dword load per 128-B line of R, 4 instructions (32 KiB of lines) in flight
//   warm    -- stream R right after the touch pass
//   hot     -- stream R again (a second pass with nothing in between)
// R = 200 MB (under the 256 MB MALL); a 1 GB memset between experiments evicts it.
//   hipcc --offload-arch=gfx950 -O3 -o scripts/mall_probe scripts/mall_probe.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

typedef __attribute__((ext_vector_type(4))) unsigned int u32x4;
#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP %s @%d\n", hipGetErrorString(e_), __LINE__); exit(1); } } while (0)

constexpr int CUS = 256;

// full stream: each workgroup (one wave) streams its contiguous share in 16 KiB slots, 3 in flight
__global__ __launch_bounds__(256) void stream_k(const char* r, size_t per_wg, unsigned* sink, int nt) {
  const int lane = threadIdx.x & 63;
  per_wg /= 4;  // 4 waves, each a contiguous quarter
  const char* base = r + ((size_t)blockIdx.x * 4 + (threadIdx.x >> 6)) * per_wg;
  u32x4 acc = {0u, 0u, 0u, 0u};
  const size_t n = per_wg / 16384;
  for (size_t s = 0; s < n; s += 3) {
    u32x4 v[48];
#pragma unroll
    for (int b = 0; b < 3; ++b)
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        const size_t sl = s + b < n ? s + b : n - 1;
        const u32x4* p = reinterpret_cast<const u32x4*>(base + sl * 16384 + i * 1024) + lane;
        v[b * 16 + i] = nt ? __builtin_nontemporal_load(p) : *p;
      }
#pragma unroll
    for (int i = 0; i < 48; ++i) acc ^= v[i];
  }
  if ((acc.x ^ acc.y ^ acc.z ^ acc.w) == 0x9e3779b9u) sink[blockIdx.x] = 1;
}

// touch: one dword per 128-B line, lane i -> line i of an 8 KiB block, U blocks per issue
template <int U, int LINE, bool NT>
__global__ __launch_bounds__(256) void touch_k(const char* r, size_t per_wg, unsigned* sink) {
  const int lane = threadIdx.x & 63;
  per_wg /= 4;
  const char* base = r + ((size_t)blockIdx.x * 4 + (threadIdx.x >> 6)) * per_wg;
  unsigned acc = 0;
  const size_t n = per_wg / (64 * LINE);
  for (size_t s = 0; s < n; s += U) {
    unsigned v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const size_t b = s + u < n ? s + u : n - 1;
      const unsigned* p = reinterpret_cast<const unsigned*>(base + b * 64 * LINE + lane * LINE);
      v[u] = NT ? __builtin_nontemporal_load(p) : *p;
    }
#pragma unroll
    for (int u = 0; u < U; ++u) acc ^= v[u];
  }
  if (acc == 0x9e3779b9u) sink[blockIdx.x] = 1;
}

int main() {
  const size_t R = (size_t)200 << 20, per = R / CUS;  // 800 KiB per workgroup (a multiple of 16 KiB)
  const size_t FL = (size_t)1 << 30;
  char *r, *fl;
  unsigned* sink;
  CK(hipMalloc(&r, R));
  CK(hipMalloc(&fl, FL));
  CK(hipMalloc(&sink, CUS * 4));
  CK(hipMemset(r, 1, R));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  auto flush = [&]() { CK(hipMemset(fl, 3, FL)); CK(hipDeviceSynchronize()); };
  auto timed = [&](auto launch) {
    CK(hipEventRecord(e0));
    launch();
    CK(hipEventRecord(e1));
    CK(hipEventSynchronize(e1));
    float ms;
    CK(hipEventElapsedTime(&ms, e0, e1));
    return ms;
  };
  auto st = [&](int nt) { return timed([&]() { stream_k<<<CUS, 256>>>(r, per, sink, nt); }); };
  auto one = [&](const char* name, auto touch) {
    flush();
    const float cold = st(1);
    flush();
    const float tch = timed(touch);
    const float warm = st(1);
    const float hot = st(1);
    printf("%-22s cold %.1f us (%.2f TB/s) | touch %.1f us (%.2f TB/s of bytes covered) -> warm %.1f us (%.2f TB/s) | hot %.1f us (%.2f TB/s)\n",
           name, cold * 1e3, R / (cold * 1e-3) / 1e12, tch * 1e3, R / (tch * 1e-3) / 1e12, warm * 1e3,
           R / (warm * 1e-3) / 1e12, hot * 1e3, R / (hot * 1e-3) / 1e12);
    fflush(stdout);
  };
  for (int rep = 0; rep < 2; ++rep) {
    one("touch 128B nt", [&]() { touch_k<4, 128, true><<<CUS, 256>>>(r, per, sink); });
    one("touch 128B", [&]() { touch_k<4, 128, false><<<CUS, 256>>>(r, per, sink); });
    one("touch 64B nt", [&]() { touch_k<4, 64, true><<<CUS, 256>>>(r, per, sink); });
    one("touch 64B", [&]() { touch_k<4, 64, false><<<CUS, 256>>>(r, per, sink); });
    one("touch 32B", [&]() { touch_k<4, 32, false><<<CUS, 256>>>(r, per, sink); });
    one("full stream (nt)", [&]() { stream_k<<<CUS, 256>>>(r, per, sink, 1); });
    one("full stream", [&]() { stream_k<<<CUS, 256>>>(r, per, sink, 0); });
  }
  return 0;
}
