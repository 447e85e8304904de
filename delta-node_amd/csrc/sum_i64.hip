// sum_i64.hip — the coordinator's masked-result sum:
// out = sum_k inputs[k], int64 with wrap-around (numpy's `+=` in
// coord/horizontal/agg.py:227-251 make_masked_results).  HBM-streaming:
// 16 B per lane per input (global_load_dwordx4), k*8 B read + 8 B written
// per element.  `out` may alias inputs[0] (accumulate in place).
#include <hip/hip_runtime.h>

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

__global__ void __launch_bounds__(256) i64_sum_kernel(const SumArgs a) {
  const uint64_t pairs = a.n / 2;
  const uint64_t stride = static_cast<uint64_t>(gridDim.x) * blockDim.x;
  for (uint64_t i = static_cast<uint64_t>(blockIdx.x) * blockDim.x + threadIdx.x; i < pairs; i += stride) {
    u64x2 acc = {0, 0};
#pragma unroll 4
    for (int j = 0; j < a.k; ++j) acc += __builtin_nontemporal_load(reinterpret_cast<const u64x2*>(a.in[j]) + i);
    __builtin_nontemporal_store(acc, reinterpret_cast<u64x2*>(a.out) + i);
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
  const uint64_t blocks = (n / 2 + 255) / 256;
  hipLaunchKernelGGL(i64_sum_kernel, dim3(blocks < 8192 ? (blocks ? blocks : 1) : 8192), dim3(256), 0,
                     static_cast<hipStream_t>(stream), a);
  const hipError_t err = hipGetLastError();
  if (err != hipSuccess) return set_error(DN_ERR_HIP, "dn_i64_sum: %s", hipGetErrorString(err));
  return DN_OK;
}
