// sum_i64.hip — the coordinator's masked-result sum:
// out = sum_k inputs[k], int64 with wrap-around (numpy's `+=` in
// coord/horizontal/agg.py:227-251 make_masked_results).  HBM-streaming:
// 16 B per lane per input (global_load_dwordx4), k*8 B read + 8 B written
// per element.  `out` may alias inputs[0] (accumulate in place).
#include <hip/hip_runtime.h>

#include <algorithm>

#include "dn_internal.hpp"
#include "dn_mask.h"

namespace dn {

constexpr int kSumMax = 16;

struct SumArgs {
  const int64_t* in[kSumMax];
  int64_t* out;
  uint64_t n;
  int32_t k;
};

typedef uint64_t u64x2 __attribute__((ext_vector_type(2)));

// DN_SUM_WIDE: 16-B pairs per lane and step, each a wave's width (64 pairs,
// 1 KB) further on, all loads of a step issued before the adds — a wave reads
// 8 KB of each member per step: at 10 x 2^24, 8 (default) 0.227-0.229 ms, 4
// 0.231, 2 0.236-0.238, 1 0.258-0.265 (0.80 vs 0.71 of 8 TB/s;
// profiles/r05/ae/, af/, ah/)
#ifndef DN_SUM_WIDE
#define DN_SUM_WIDE 8
#endif
__global__ void __launch_bounds__(256) i64_sum_kernel(const SumArgs a) {
  constexpr int V = DN_SUM_WIDE;
  const uint64_t pairs = a.n / 2;
  const uint64_t stride = static_cast<uint64_t>(gridDim.x) * blockDim.x * V;
  const uint64_t first = static_cast<uint64_t>(blockIdx.x) * blockDim.x * V + (threadIdx.x & ~63u) * V + (threadIdx.x & 63u);
  for (uint64_t i = first; i < pairs; i += stride) {
    u64x2 acc[V];
#pragma unroll
    for (int v = 0; v < V; ++v) acc[v] = u64x2{0, 0};
#pragma unroll 4
    for (int j = 0; j < a.k; ++j) {
      const u64x2* p = reinterpret_cast<const u64x2*>(a.in[j]) + i;
#pragma unroll
      for (int v = 0; v < V; ++v)
        if (i + 64 * v < pairs) acc[v] += __builtin_nontemporal_load(p + 64 * v);
    }
#pragma unroll
    for (int v = 0; v < V; ++v)
      if (i + 64 * v < pairs) __builtin_nontemporal_store(acc[v], reinterpret_cast<u64x2*>(a.out) + i + 64 * v);
  }
  if ((a.n & 1) && blockIdx.x == 0 && threadIdx.x == 0) {
    uint64_t acc = 0;
    for (int j = 0; j < a.k; ++j) acc += static_cast<uint64_t>(a.in[j][a.n - 1]);
    a.out[a.n - 1] = static_cast<int64_t>(acc);
  }
}

}  // namespace dn

using namespace dn;

extern "C" int dn_i64_sum(const int64_t* const* inputs, int k, int64_t* out, uint64_t n, void* stream) {
  if (k < 1 || k > kSumMax) return set_error(DN_ERR_UNSUPPORTED, "dn_i64_sum: k=%d outside 1..%d", k, kSumMax);
  if (n == 0) return DN_OK;
  if (!inputs || !out) return set_error(DN_ERR_ARG, "dn_i64_sum: null pointer");
  SumArgs a{};
  for (int j = 0; j < k; ++j) {
    if (!inputs[j] || (reinterpret_cast<uintptr_t>(inputs[j]) & 15))
      return set_error(DN_ERR_ARG, "dn_i64_sum: input %d null or not 16-byte aligned", j);
    a.in[j] = inputs[j];
  }
  if (reinterpret_cast<uintptr_t>(out) & 15) return set_error(DN_ERR_ARG, "dn_i64_sum: out not 16-byte aligned");
  a.out = out;
  a.n = n;
  a.k = k;
  // one workgroup per 256 * DN_SUM_WIDE pairs (sized per pair,
  // 7 of 8 workgroups found no work), at most 8192
  constexpr uint64_t kPairsPerBlock = 256ull * DN_SUM_WIDE;
  const uint64_t blocks = (n / 2 + kPairsPerBlock - 1) / kPairsPerBlock;
  // (the member count as a template argument, all loads of a pair issued
  // before the adds: 0.258 ms either way at 10 x 2^24, profiles/r05/m/)
  hipLaunchKernelGGL(i64_sum_kernel, dim3(blocks < 8192 ? (blocks ? blocks : 1) : 8192), dim3(256), 0,
                     static_cast<hipStream_t>(stream), a);
  const hipError_t err = hipGetLastError();
  if (err != hipSuccess) return set_error(DN_ERR_HIP, "dn_i64_sum: %s", hipGetErrorString(err));
  return DN_OK;
}

// ---- share-block write probe (memory.share_block) ---------------------------
// Writes zeros over `rows` rows of `row_bytes` (a multiple of the 16896-byte
// tile) in the order a split writes a share block: per 256-element tile, that
// tile's slice of every row, 16-B non-temporal stores (a wave per tile).  A
// block's rate under this pattern predicts its split; a linear fill does not
// (profiles/r04/y/).
namespace {
typedef uint32_t u32x4_p __attribute__((ext_vector_type(4)));
__global__ void __launch_bounds__(256) block_probe_kernel(uint8_t* p, uint32_t rows, uint64_t row_bytes,
                                                          uint64_t ntiles) {
  constexpr uint32_t kTileB = 66u * 256u;
  const uint32_t lane = threadIdx.x & 63u;
  const uint64_t nw = static_cast<uint64_t>(gridDim.x) * 4u;
  const u32x4_p z = {0u, 0u, 0u, 0u};
  for (uint64_t t = __builtin_amdgcn_readfirstlane(blockIdx.x * 4u + (threadIdx.x >> 6)); t < ntiles; t += nw)
    for (uint32_t r = 0; r < rows; ++r) {
      u32x4_p* q = reinterpret_cast<u32x4_p*>(p + r * row_bytes + t * kTileB);
#pragma unroll 4
      for (uint32_t o = lane; o < kTileB / 16u; o += 64u) __builtin_nontemporal_store(z, q + o);
    }
}
}  // namespace

extern "C" int dn_block_probe_rows(void* ptr, uint32_t rows, uint64_t row_bytes, void* stream) {
  constexpr uint64_t kTileB = 66u * 256u;
  if (!ptr || rows == 0 || row_bytes == 0 || row_bytes % kTileB)
    return dn::set_error(DN_ERR_ARG, "dn_block_probe_rows: rows of whole 16896-byte tiles");
  const uint64_t ntiles = row_bytes / kTileB;
  const uint64_t g = std::min<uint64_t>(16384u, (ntiles + 3u) / 4u);
  hipLaunchKernelGGL(block_probe_kernel, dim3(static_cast<uint32_t>(g)), dim3(256), 0,
                     static_cast<hipStream_t>(stream), static_cast<uint8_t*>(ptr), rows, row_bytes, ntiles);
  const hipError_t e = hipGetLastError();
  return e == hipSuccess ? DN_OK : dn::set_error(DN_ERR_HIP, "dn_block_probe_rows: %s", hipGetErrorString(e));
}
