// hbm_ceiling.hip — diagnostic: what HBM bandwidth the split/reconstruct
// access patterns reach with the arithmetic removed (not part of the product).
//
//   read_x4      pure streaming read, 16 B/lane (global_load_dwordx4)
//   write_x4     pure streaming write, 16 B/lane, non-temporal
//   copy_x4      read 16 B/lane -> write 16 B/lane
//   split_mem    the split kernel's exact access pattern (tiled layout, one
//                element per lane, 4 B/lane u32 planes + u16 plane; 140 B read,
//                330 B written per element) with the field arithmetic replaced
//                by XORs
//   recon_mem    the reconstruct pattern (3 x 66 B read, 8 B written)
//
// build: hipcc -O3 --offload-arch=gfx950 -I../delta-node_amd/csrc -I../include hbm_ceiling.hip -o hbm_ceiling
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

#include "m521_device.hpp"

using namespace dn;

#define CHECK(x)                                                                  \
  do {                                                                            \
    hipError_t e = (x);                                                           \
    if (e != hipSuccess) {                                                        \
      std::fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e)); \
      std::exit(1);                                                               \
    }                                                                             \
  } while (0)

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

__global__ void read_x4(const u32x4* __restrict__ in, size_t n, uint32_t* __restrict__ sink) {
  uint32_t acc = 0;
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
    const u32x4 v = __builtin_nontemporal_load(in + i);
    acc ^= v.x ^ v.y ^ v.z ^ v.w;
  }
  if (acc == 0x12345678u) sink[0] = acc;
}

__global__ void write_x4(u32x4* __restrict__ out, size_t n) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
    u32x4 v = {(uint32_t)i, 1u, 2u, 3u};
    __builtin_nontemporal_store(v, out + i);
  }
}

__global__ void copy_x4(const u32x4* __restrict__ in, u32x4* __restrict__ out, size_t n) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
    __builtin_nontemporal_store(__builtin_nontemporal_load(in + i), out + i);
}

__global__ void __launch_bounds__(256) split_mem(const int64_t* __restrict__ sec, const uint8_t* __restrict__ co,
                                                 uint8_t* __restrict__ sh, uint32_t ntiles, uint64_t vb, int nsh) {
  const uint32_t lane = threadIdx.x & 63u;
  const uint32_t nwaves = gridDim.x * 4;
  const uint32_t wave0 = __builtin_amdgcn_readfirstlane(blockIdx.x * 4 + (threadIdx.x >> 6));
  for (uint32_t tile = wave0; tile < ntiles; tile += nwaves) {
#pragma unroll 1
    for (uint32_t q = 0; q < 4; ++q) {
      const uint32_t w = lane + 64u * q;
      uint32_t c1[kLimbs], c2[kLimbs];
      const uint64_t s = (uint64_t)__builtin_nontemporal_load(sec + (uint64_t)tile * kTile + w);
      load_fe(tile_base(co, tile), w, c1);
      load_fe(tile_base(co + vb, tile), w, c2);
#pragma unroll 1
      for (int x = 0; x < nsh; ++x) {
        uint32_t v[kLimbs];
#pragma unroll
        for (int i = 0; i < kLimbs; ++i) v[i] = c1[i] ^ c2[i] ^ (uint32_t)x;
        v[0] ^= (uint32_t)s;
        v[16] &= kTopMask;
        store_fe(tile_base(sh + (uint64_t)x * vb, tile), w, v);
      }
    }
  }
}

__global__ void __launch_bounds__(256) recon_mem(const uint8_t* __restrict__ y0, const uint8_t* __restrict__ y1,
                                                 const uint8_t* __restrict__ y2, int64_t* __restrict__ out,
                                                 uint32_t ntiles) {
  const uint32_t lane = threadIdx.x & 63u;
  const uint32_t nwaves = gridDim.x * 4;
  const uint32_t wave0 = __builtin_amdgcn_readfirstlane(blockIdx.x * 4 + (threadIdx.x >> 6));
  for (uint32_t tile = wave0; tile < ntiles; tile += nwaves) {
#pragma unroll 1
    for (uint32_t q = 0; q < 4; ++q) {
      const uint32_t w = lane + 64u * q;
      uint32_t a[kLimbs], b[kLimbs], c[kLimbs];
      load_fe(tile_base(y0, tile), w, a);
      load_fe(tile_base(y1, tile), w, b);
      load_fe(tile_base(y2, tile), w, c);
      uint32_t lo = 0, hi = 0;
#pragma unroll
      for (int i = 0; i < kLimbs; ++i) {
        lo ^= a[i] ^ b[i] ^ c[i];
        hi += a[i] ^ c[i];
      }
      __builtin_nontemporal_store((int64_t)(((uint64_t)hi << 32) | lo), out + (uint64_t)tile * kTile + w);
    }
  }
}

// recon_mem with 16 B per lane: lane l of a wave reads elements 4l..4l+3 of
// each limb plane of a tile (one 1-KB run per wave-instruction), 4 elements
// per lane, one share row at a time (the reconstruct's read pattern widened)
typedef uint32_t u32x4v __attribute__((ext_vector_type(4)));
typedef uint16_t u16x4v __attribute__((ext_vector_type(4)));
__global__ void __launch_bounds__(256) recon_mem_x4(const uint8_t* __restrict__ y0, const uint8_t* __restrict__ y1,
                                                    const uint8_t* __restrict__ y2, int64_t* __restrict__ out,
                                                    uint32_t ntiles) {
  const uint32_t lane = threadIdx.x & 63u;
  const uint32_t nwaves = gridDim.x * 4;
  const uint32_t wave0 = __builtin_amdgcn_readfirstlane(blockIdx.x * 4 + (threadIdx.x >> 6));
  for (uint32_t tile = wave0; tile < ntiles; tile += nwaves) {
    u32x4v lo = {0, 0, 0, 0}, hi = {0, 0, 0, 0};
    const uint8_t* rows[3] = {y0, y1, y2};
#pragma unroll
    for (int s = 0; s < 3; ++s) {
      const uint8_t* tb = tile_base(rows[s], tile);
      u32x4v a[16];
#pragma unroll
      for (int i = 0; i < 16; ++i)
        a[i] = __builtin_nontemporal_load(reinterpret_cast<const u32x4v*>(tb + i * 4 * kTile) + lane);
      const u16x4v t = __builtin_nontemporal_load(reinterpret_cast<const u16x4v*>(tb + kHiOffset) + lane);
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        lo ^= a[i];
        hi += a[i];
      }
      hi.x += t.x;
      hi.y += t.y;
      hi.z += t.z;
      hi.w += t.w;
    }
    int64_t* o = out + (uint64_t)tile * kTile + 4 * lane;
    __builtin_nontemporal_store((int64_t)(((uint64_t)hi.x << 32) | lo.x), o + 0);
    __builtin_nontemporal_store((int64_t)(((uint64_t)hi.y << 32) | lo.y), o + 1);
    __builtin_nontemporal_store((int64_t)(((uint64_t)hi.z << 32) | lo.z), o + 2);
    __builtin_nontemporal_store((int64_t)(((uint64_t)hi.w << 32) | lo.w), o + 3);
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
  return ms / reps;
}

int main(int argc, char** argv) {
  const int log2n = argc > 1 ? std::atoi(argv[1]) : 24;
  const size_t N = (size_t)1 << log2n;
  const uint32_t ntiles = (uint32_t)(N / kTile);
  const uint64_t vb = (uint64_t)ntiles * kTileBytes;
  const size_t big = (size_t)4 << 30;  // 4 GiB streams
  uint8_t *A, *B, *sh, *co;
  int64_t *sec, *out;
  uint32_t* sink;
  CHECK(hipMalloc(&A, big));
  CHECK(hipMalloc(&B, big));
  CHECK(hipMemset(A, 1, big));
  CHECK(hipMalloc(&sink, 64));
  const size_t n4 = big / 16;
  const int reps = 10;
  for (int grid : {1024, 2048, 4096, 8192, 16384}) {
    float r = time_ms([&] { read_x4<<<grid, 256>>>((const u32x4*)A, n4, sink); }, reps);
    float w = time_ms([&] { write_x4<<<grid, 256>>>((u32x4*)B, n4); }, reps);
    float c = time_ms([&] { copy_x4<<<grid, 256>>>((const u32x4*)A, (u32x4*)B, n4); }, reps);
    std::printf("{\"grid\": %d, \"read_x4_GBps\": %.1f, \"write_x4_GBps\": %.1f, \"copy_x4_GBps\": %.1f}\n", grid,
                big / (r * 1e-3) / 1e9, big / (w * 1e-3) / 1e9, 2.0 * big / (c * 1e-3) / 1e9);
  }
  CHECK(hipFree(A));
  CHECK(hipFree(B));
  CHECK(hipMalloc(&sec, N * 8));
  CHECK(hipMalloc(&co, 2 * vb));
  CHECK(hipMalloc(&sh, 5 * vb));
  CHECK(hipMalloc(&out, N * 8));
  CHECK(hipMemset(sec, 3, N * 8));
  CHECK(hipMemset(co, 5, 2 * vb));
  for (int grid : {1024, 2048, 4096, 16384}) {
    float rx = time_ms([&] { recon_mem_x4<<<grid, 256>>>(sh, sh + 2 * vb, sh + 4 * vb, out, ntiles); }, reps);
    float rr2 = time_ms([&] { recon_mem<<<grid, 256>>>(sh, sh + 2 * vb, sh + 4 * vb, out, ntiles); }, reps);
    std::printf("{\"grid\": %d, \"recon_mem_x4_ms\": %.4f, \"recon_mem_ms\": %.4f}\n", grid, rx, rr2);
  }
  for (int grid : {2048, 4096, 16384}) {
    float s = time_ms([&] { split_mem<<<grid, 256>>>(sec, co, sh, ntiles, vb, 5); }, reps);
    float rr = time_ms([&] { recon_mem<<<grid, 256>>>(sh, sh + 2 * vb, sh + 4 * vb, out, ntiles); }, reps);
    std::printf("{\"grid\": %d, \"split_mem_ms\": %.4f, \"split_mem_GBps\": %.1f, \"recon_mem_ms\": %.4f, "
                "\"recon_mem_GBps\": %.1f}\n",
                grid, s, N * 470.0 / (s * 1e-3) / 1e9, rr, N * 206.0 / (rr * 1e-3) / 1e9);
  }
  return 0;
}
