// vmm_alloc_cost.hip — what mapping a 5.5 GB share block costs (VERDICT r04
// item 4: the first make_shares_vec of a process maps ~2,640 2 MiB chunks per
// block, csrc/vmm_block.cpp).  Per chunk size: wall time of the reserve, the
// hipMemCreate loop, the hipMemMap loop and hipMemSetAccess, with the create +
// map loop on T host threads (each thread its own contiguous run of chunks),
// then a hipMalloc of the same size and its first kernel write for
// comparison.  Host timing only; one JSON line per case.
// Build: hipcc -O2 --offload-arch=gfx950 tools/vmm_alloc_cost.hip -o tools/vmm_alloc_cost -lpthread
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdint>
#include <cstdio>
#include <thread>
#include <vector>

#define CK(x)                                                                                 \
  do {                                                                                        \
    hipError_t e_ = (x);                                                                      \
    if (e_ != hipSuccess) printf("  %s -> %s (line %d)\n", #x, hipGetErrorString(e_), __LINE__); \
  } while (0)

static double now_ms() {
  return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

__global__ void fill_kernel(uint4* p, uint64_t n16) {
  for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n16; i += (uint64_t)gridDim.x * blockDim.x)
    p[i] = make_uint4(1, 2, 3, 4);
}

static void one_case(uint64_t bytes, uint64_t chunk, int threads) {
  hipMemAllocationProp prop{};
  prop.type = hipMemAllocationTypePinned;
  prop.location.type = hipMemLocationTypeDevice;
  prop.location.id = 0;
  const uint64_t nch = (bytes + chunk - 1) / chunk, span = nch * chunk;
  void* base = nullptr;
  const double t0 = now_ms();
  CK(hipMemAddressReserve(&base, span, 1ull << 21, nullptr, 0));
  const double t1 = now_ms();
  std::vector<hipMemGenericAllocationHandle_t> h(nch);
  std::vector<double> create_ms(threads, 0.0), map_ms(threads, 0.0);
  auto work = [&](int k) {
    const uint64_t lo = nch * k / threads, hi = nch * (k + 1) / threads;
    CK(hipSetDevice(0));
    const double a = now_ms();
    for (uint64_t c = lo; c < hi; ++c) CK(hipMemCreate(&h[c], chunk, &prop, 0));
    const double b = now_ms();
    for (uint64_t c = lo; c < hi; ++c) CK(hipMemMap(static_cast<uint8_t*>(base) + c * chunk, chunk, 0, h[c], 0));
    create_ms[k] = b - a;
    map_ms[k] = now_ms() - b;
  };
  if (threads == 1) {
    work(0);
  } else {
    std::vector<std::thread> th;
    for (int k = 0; k < threads; ++k) th.emplace_back(work, k);
    for (auto& x : th) x.join();
  }
  const double t2 = now_ms();
  hipMemAccessDesc acc{};
  acc.location = prop.location;
  acc.flags = hipMemAccessFlagsProtReadWrite;
  CK(hipMemSetAccess(base, span, &acc, 1));
  const double t3 = now_ms();
  fill_kernel<<<4096, 256>>>(static_cast<uint4*>(base), span / 16);
  CK(hipDeviceSynchronize());
  const double t4 = now_ms();
  fill_kernel<<<4096, 256>>>(static_cast<uint4*>(base), span / 16);
  CK(hipDeviceSynchronize());
  const double t5 = now_ms();
  double cmax = 0, mmax = 0;
  for (int k = 0; k < threads; ++k) cmax = create_ms[k] > cmax ? create_ms[k] : cmax, mmax = map_ms[k] > mmax ? map_ms[k] : mmax;
  printf("{\"kind\": \"vmm\", \"chunk_MiB\": %llu, \"chunks\": %llu, \"threads\": %d, \"reserve_ms\": %.3f, "
         "\"create_map_wall_ms\": %.3f, \"create_ms_max_thread\": %.3f, \"map_ms_max_thread\": %.3f, "
         "\"set_access_ms\": %.3f, \"first_fill_ms\": %.3f, \"second_fill_ms\": %.3f, \"total_ms\": %.3f}\n",
         (unsigned long long)(chunk >> 20), (unsigned long long)nch, threads, t1 - t0, t2 - t1, cmax, mmax, t3 - t2,
         t4 - t3, t5 - t4, t3 - t0);
  fflush(stdout);
  const double f0 = now_ms();
  for (uint64_t c = 0; c < nch; ++c) CK(hipMemUnmap(static_cast<uint8_t*>(base) + c * chunk, chunk));
  for (auto x : h) CK(hipMemRelease(x));
  printf("{\"kind\": \"vmm_free\", \"chunk_MiB\": %llu, \"unmap_release_ms\": %.3f}\n",
         (unsigned long long)(chunk >> 20), now_ms() - f0);
  // the range stays reserved (csrc/vmm_block.cpp retires freed ranges)
}

int main() {
  const uint64_t bytes = 5ull * 1107296256ull;  // 5 x vec_bytes(2^24): the headline share block
  CK(hipSetDevice(0));
  CK(hipFree(nullptr));
  for (uint64_t mib : {2ull, 4ull, 8ull, 16ull, 64ull}) one_case(bytes, mib << 20, 1);
  for (int t : {2, 4, 8}) one_case(bytes, 2ull << 20, t);
  {
    const double a = now_ms();
    void* p = nullptr;
    CK(hipMalloc(&p, bytes));
    const double b = now_ms();
    fill_kernel<<<4096, 256>>>(static_cast<uint4*>(p), bytes / 16);
    CK(hipDeviceSynchronize());
    const double c = now_ms();
    fill_kernel<<<4096, 256>>>(static_cast<uint4*>(p), bytes / 16);
    CK(hipDeviceSynchronize());
    printf("{\"kind\": \"hipMalloc\", \"alloc_ms\": %.3f, \"first_fill_ms\": %.3f, \"second_fill_ms\": %.3f}\n", b - a,
           c - b, now_ms() - c);
    CK(hipFree(p));
  }
  return 0;
}
