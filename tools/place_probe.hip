// place_probe.hip — diagnostic (not part of the product): is the split's
// placement sensitivity a property of the buffer (any access pattern) or of
// the split's five concurrent row streams?  For several fresh 5-row share
// buffers (5 x 1.1 GB at 2^24 elements) time, per buffer:
//   write1   one streaming write over the whole buffer (16 B/lane, nt)
//   write1b  the same bytes, each wave writing its own contiguous chunk
//   read1    one streaming read over the whole buffer
//   write5   the split's store pattern (tiled layout, 5 rows written per tile)
//            without its loads
//   split5   the split's full access pattern (140 B read, 330 B written per
//            element), arithmetic replaced by XORs
//   write5il / split5il  the same with a tile-interleaved share block
//            ([tile][share][plane]: each wave writes one contiguous 5-tile
//            run instead of 5 runs vec_bytes apart)
//
// build: hipcc -O3 --offload-arch=gfx950 -I../delta-node_amd/csrc place_probe.hip -o place_probe
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <string>
#include <vector>

#include "m521_device.hpp"

using namespace dn;

#define CHECK(x)                                                                    \
  do {                                                                              \
    hipError_t e = (x);                                                             \
    if (e != hipSuccess) {                                                          \
      std::fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e)); \
      std::exit(1);                                                                 \
    }                                                                               \
  } while (0)

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

__global__ void read1(const u32x4* __restrict__ in, size_t n, uint32_t* __restrict__ sink) {
  uint32_t acc = 0;
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
    const u32x4 v = __builtin_nontemporal_load(in + i);
    acc ^= v.x ^ v.y ^ v.z ^ v.w;
  }
  if (acc == 0x12345678u) sink[0] = acc;
}

__global__ void write1(u32x4* __restrict__ out, size_t n) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
    u32x4 v = {(uint32_t)i, 1u, 2u, 3u};
    __builtin_nontemporal_store(v, out + i);
  }
}

// each wave owns a contiguous chunk of n / waves 16-B units
__global__ void write1b(u32x4* __restrict__ out, size_t n) {
  const size_t waves = (size_t)gridDim.x * (blockDim.x / 64);
  const size_t wave = (size_t)blockIdx.x * (blockDim.x / 64) + (threadIdx.x >> 6);
  const size_t per = ((n + waves - 1) / waves + 63) / 64 * 64;
  const size_t lo = wave * per, hi = lo + per < n ? lo + per : n;
  for (size_t i = lo + (threadIdx.x & 63); i < hi; i += 64) {
    u32x4 v = {(uint32_t)i, 1u, 2u, 3u};
    __builtin_nontemporal_store(v, out + i);
  }
}

template <bool READS, bool IL = false>
__global__ void __launch_bounds__(256) split5(const int64_t* __restrict__ sec, const uint8_t* __restrict__ co,
                                              uint8_t* __restrict__ sh, uint32_t ntiles, uint64_t vb, int nsh) {
  const uint32_t lane = threadIdx.x & 63u;
  const uint32_t nwaves = gridDim.x * 4;
  const uint32_t wave0 = __builtin_amdgcn_readfirstlane(blockIdx.x * 4 + (threadIdx.x >> 6));
  for (uint32_t tile = wave0; tile < ntiles; tile += nwaves) {
#pragma unroll 1
    for (uint32_t q = 0; q < 4; ++q) {
      const uint32_t w = lane + 64u * q;
      uint32_t c1[kLimbs], c2[kLimbs];
      uint64_t s = w;
      if constexpr (READS) {
        s = (uint64_t)__builtin_nontemporal_load(sec + (uint64_t)tile * kTile + w);
        load_fe(tile_base(co, tile), w, c1);
        load_fe(tile_base(co + vb, tile), w, c2);
      } else {
#pragma unroll
        for (int i = 0; i < kLimbs; ++i) c1[i] = c2[i] = tile * 17u + i;
      }
#pragma unroll 1
      for (int x = 0; x < nsh; ++x) {
        uint32_t v[kLimbs];
#pragma unroll
        for (int i = 0; i < kLimbs; ++i) v[i] = c1[i] ^ c2[i] ^ (uint32_t)x;
        v[0] ^= (uint32_t)s;
        v[16] &= kTopMask;
        if constexpr (IL)
          store_fe(tile_base(sh, tile * (uint32_t)nsh + (uint32_t)x), w, v);
        else
          store_fe(tile_base(sh + (uint64_t)x * vb, tile), w, v);
      }
    }
  }
}

template <typename F>
static float time_ms(F f, int reps) {
  hipEvent_t a, b;
  CHECK(hipEventCreate(&a));
  CHECK(hipEventCreate(&b));
  f();
  CHECK(hipDeviceSynchronize());
  CHECK(hipEventRecord(a));
  for (int i = 0; i < reps; ++i) f();
  CHECK(hipEventRecord(b));
  CHECK(hipEventSynchronize(b));
  float ms;
  CHECK(hipEventElapsedTime(&ms, a, b));
  CHECK(hipEventDestroy(a));
  CHECK(hipEventDestroy(b));
  return ms / reps;
}

int main(int argc, char** argv) {
  const int sets = argc > 1 ? std::atoi(argv[1]) : 6;
  const size_t N = (size_t)1 << 24;
  const uint32_t ntiles = (uint32_t)(N / kTile);
  const uint64_t vb = (uint64_t)ntiles * kTileBytes;
  const size_t bytes = 5 * vb, n16 = bytes / 16;
  int64_t* sec;
  uint8_t* co;
  uint32_t* sink;
  CHECK(hipMalloc(&sec, N * 8));
  CHECK(hipMalloc(&co, 2 * vb));
  CHECK(hipMalloc(&sink, 64));
  CHECK(hipMemset(sec, 3, N * 8));
  CHECK(hipMemset(co, 5, 2 * vb));
  std::vector<uint8_t*> sh(sets);
  for (auto& p : sh) {
    CHECK(hipMalloc(&p, bytes));
    CHECK(hipMemset(p, 0, bytes));
  }
  const int reps = 8;
  if (argc > 2 && std::string(argv[2]) == "vmm") {
    // The same physical memory mapped at two virtual addresses (1-GiB aligned and
    // offset by 3 granules): equal rates => the placement term is physical.
    // Then buffers built from 64-MiB physical chunks mapped back to back.
    hipMemAllocationProp prop{};
    prop.type = hipMemAllocationTypePinned;
    prop.location.type = hipMemLocationTypeDevice;
    prop.location.id = 0;
    size_t gran = 0;
    CHECK(hipMemGetAllocationGranularity(&gran, &prop, hipMemAllocationGranularityMinimum));
    const size_t one_g = (size_t)1 << 30;
    const size_t size = (bytes + gran - 1) / gran * gran;
    hipMemAccessDesc acc{};
    acc.location = prop.location;
    acc.flags = hipMemAccessFlagsProtReadWrite;
    auto measure = [&](const char* kind, int i, uint8_t* p) {
      const float w1b = time_ms([&] { write1b<<<256, 256>>>((u32x4*)p, n16); }, reps);
      const float w5 = time_ms([&] { split5<false><<<256, 256>>>(sec, co, p, ntiles, vb, 5); }, reps);
      const float s5 = time_ms([&] { split5<true><<<256, 256>>>(sec, co, p, ntiles, vb, 5); }, reps);
      std::printf("{\"kind\": \"%s\", \"set\": %d, \"va\": \"%p\", \"write1b_TBps\": %.3f, \"write5_TBps\": %.3f, "
                  "\"split5_ms\": %.4f}\n",
                  kind, i, (void*)p, bytes / (w1b * 1e-3) / 1e12, bytes / (w5 * 1e-3) / 1e12, s5);
      std::fflush(stdout);
    };
    std::printf("{\"granularity\": %zu}\n", gran);
    if (argc > 3 && std::string(argv[3]) == "mix") {
      // S sets of P-MiB handles (argv[4], default 2), each mapped in
      // allocation order ("set"); then "mixF" buffers over the pages of the
      // first F sets: piece k of mix j is piece (k / F) + j * (n / F) of set
      // k % F, so a mix holds 1/F of each of F sets (F = 2, 4, S).
      const size_t piece = (size_t)(argc > 4 ? std::atoi(argv[4]) : 2) << 20;
      const size_t np_ = (size + piece - 1) / piece;
      std::vector<std::vector<hipMemGenericAllocationHandle_t>> hv(sets);
      for (int s_ = 0; s_ < sets; ++s_) {
        hv[s_].resize(np_ + sets);
        for (auto& h : hv[s_]) CHECK(hipMemCreate(&h, piece, &prop, 0));
        void* a = nullptr;
        CHECK(hipMemAddressReserve(&a, np_ * piece, one_g, nullptr, 0));
        for (size_t k = 0; k < np_; ++k) CHECK(hipMemMap((uint8_t*)a + k * piece, piece, 0, hv[s_][k], 0));
        CHECK(hipMemSetAccess(a, np_ * piece, &acc, 1));
        measure("set", s_, (uint8_t*)a);
      }
      for (int F : {2, 4, sets}) {
        const size_t per = (np_ + F - 1) / F;
        for (int j = 0; j < F && j < 4; ++j) {
          void* b = nullptr;
          CHECK(hipMemAddressReserve(&b, np_ * piece, one_g, nullptr, 0));
          for (size_t k = 0; k < np_; ++k)
            CHECK(hipMemMap((uint8_t*)b + k * piece, piece, 0, hv[k % F][(k / F) + j * per], 0));
          CHECK(hipMemSetAccess(b, np_ * piece, &acc, 1));
          char kind[32];
          std::snprintf(kind, sizeof kind, "mix%d", F);
          measure(kind, j, (uint8_t*)b);
        }
      }
      return 0;
    }
    {  // Infinity-Cache residency: a 128-MiB buffer re-read / re-written, hipMalloc vs hipMemCreate
      const size_t small = (size_t)128 << 20;
      uint8_t* hm;
      CHECK(hipMalloc(&hm, small));
      hipMemGenericAllocationHandle_t h;
      CHECK(hipMemCreate(&h, small, &prop, 0));
      void* vm = nullptr;
      CHECK(hipMemAddressReserve(&vm, small, one_g, nullptr, 0));
      CHECK(hipMemMap(vm, small, 0, h, 0));
      CHECK(hipMemSetAccess(vm, small, &acc, 1));
      for (int r = 0; r < 2; ++r)
        for (auto pr : {std::make_pair("hipMalloc", hm), std::make_pair("hipMemCreate", (uint8_t*)vm)}) {
          const float rd = time_ms([&] { read1<<<4096, 256>>>((const u32x4*)pr.second, small / 16, sink); }, 20);
          const float wr = time_ms([&] { write1b<<<1024, 256>>>((u32x4*)pr.second, small / 16); }, 20);
          std::printf("{\"mall_probe\": \"%s\", \"read_128M_TBps\": %.3f, \"write_128M_TBps\": %.3f}\n", pr.first,
                      small / (rd * 1e-3) / 1e12, small / (wr * 1e-3) / 1e12);
        }
    }
    for (int i = 0; i < sets; ++i) {
      hipMemGenericAllocationHandle_t h;
      CHECK(hipMemCreate(&h, size, &prop, 0));
      void* base = nullptr;
      const size_t span = 2 * (size + one_g) + one_g;
      CHECK(hipMemAddressReserve(&base, span, one_g, nullptr, 0));
      uint8_t* va1 = (uint8_t*)(((uintptr_t)base + one_g - 1) / one_g * one_g);
      uint8_t* va2 = (uint8_t*)((((uintptr_t)va1 + size + one_g - 1) / one_g * one_g) + 3 * gran);
      CHECK(hipMemMap(va1, size, 0, h, 0));
      CHECK(hipMemMap(va2, size, 0, h, 0));
      CHECK(hipMemSetAccess(va1, size, &acc, 1));
      CHECK(hipMemSetAccess(va2, size, &acc, 1));
      measure("alias_a", i, va1);
      measure("alias_b", i, va2);
    }
    // chunked buffers: CHUNK-MiB physical handles mapped back to back (perm 0)
    // or in a scattered order (perm 1: VA chunk k <- handle (k * 7919) mod n)
    for (size_t cm : {2, 16, 64, 256}) {
      for (int perm = 0; perm < 2; ++perm) {
        for (int i = 0; i < 3; ++i) {
          const size_t chunk = cm << 20;
          const size_t nch = (size + chunk - 1) / chunk;
          std::vector<hipMemGenericAllocationHandle_t> hs(nch);
          for (auto& h : hs) CHECK(hipMemCreate(&h, chunk, &prop, 0));
          void* base = nullptr;
          CHECK(hipMemAddressReserve(&base, nch * chunk, one_g, nullptr, 0));
          for (size_t k = 0; k < nch; ++k) {
            const size_t src = perm ? (k * 7919) % nch : k;
            CHECK(hipMemMap((uint8_t*)base + k * chunk, chunk, 0, hs[src], 0));
          }
          CHECK(hipMemSetAccess(base, nch * chunk, &acc, 1));
          char kind[64];
          std::snprintf(kind, sizeof kind, "chunks%zuM_perm%d", cm, perm);
          measure(kind, i, (uint8_t*)base);
          CHECK(hipMemUnmap(base, nch * chunk));
          CHECK(hipMemAddressFree(base, nch * chunk));
          for (auto& h : hs) CHECK(hipMemRelease(h));
        }
      }
    }
    return 0;
  }
  if (argc > 2) {  // segment map: write / read rate of each argv[2]-MiB segment of every buffer
    const size_t seg = (size_t)std::atoi(argv[2]) << 20, nseg = bytes / seg;
    for (int round = 0; round < 2; ++round)
      for (int i = 0; i < sets; ++i) {
        std::printf("{\"round\": %d, \"set\": %d, \"seg_write_TBps\": [", round, i);
        for (size_t k = 0; k < nseg; ++k) {
          u32x4* p = (u32x4*)(sh[i] + k * seg);
          const float w = time_ms([&] { write1b<<<256, 256>>>(p, seg / 16); }, reps);
          std::printf("%s%.2f", k ? ", " : "", seg / (w * 1e-3) / 1e12);
        }
        std::printf("], \"seg_read_TBps\": [");
        for (size_t k = 0; k < nseg; ++k) {
          const u32x4* p = (const u32x4*)(sh[i] + k * seg);
          const float r = time_ms([&] { read1<<<4096, 256>>>(p, seg / 16, sink); }, reps);
          std::printf("%s%.2f", k ? ", " : "", seg / (r * 1e-3) / 1e12);
        }
        std::printf("]}\n");
        std::fflush(stdout);
      }
    return 0;
  }
  for (int round = 0; round < 2; ++round) {
    for (int i = 0; i < sets; ++i) {
      uint8_t* p = sh[i];
      const float w1 = time_ms([&] { write1<<<4096, 256>>>((u32x4*)p, n16); }, reps);
      const float w1b = time_ms([&] { write1b<<<256, 256>>>((u32x4*)p, n16); }, reps);
      const float r1 = time_ms([&] { read1<<<4096, 256>>>((const u32x4*)p, n16, sink); }, reps);
      const float w5 = time_ms([&] { split5<false><<<256, 256>>>(sec, co, p, ntiles, vb, 5); }, reps);
      const float s5 = time_ms([&] { split5<true><<<256, 256>>>(sec, co, p, ntiles, vb, 5); }, reps);
      const float w5i = time_ms([&] { split5<false, true><<<256, 256>>>(sec, co, p, ntiles, vb, 5); }, reps);
      const float s5i = time_ms([&] { split5<true, true><<<256, 256>>>(sec, co, p, ntiles, vb, 5); }, reps);
      std::printf(
          "{\"round\": %d, \"set\": %d, \"addr\": \"%p\", \"write1_TBps\": %.3f, \"write1b_TBps\": %.3f, "
          "\"read1_TBps\": %.3f, \"write5_TBps\": %.3f, \"split5_ms\": %.4f, \"write5il_TBps\": %.3f, "
          "\"split5il_ms\": %.4f}\n",
          round, i, (void*)p, bytes / (w1 * 1e-3) / 1e12, bytes / (w1b * 1e-3) / 1e12, bytes / (r1 * 1e-3) / 1e12,
          bytes / (w5 * 1e-3) / 1e12, s5, bytes / (w5i * 1e-3) / 1e12, s5i);
      std::fflush(stdout);
    }
  }
  return 0;
}
