// diag_hbm.hip — measurement kernels (lib/libdn_diag.so), not part of the
// product library: a same-buffer HBM ceiling for bench.py.
//
// dn_diag_tile_stream moves exactly the bytes a tiled-layout kernel moves —
// per 256-element tile, in_bpt[b] bytes read from input buffer b and
// out_bpt[b] bytes written to output buffer b — over the caller's own
// buffers, with no arithmetic: each wave reads its tile's slices of every
// input (16 B per lane, non-temporal), then writes its tile's slices of every
// output (16 B per lane, non-temporal).  On the split's buffers (secrets 2 KB,
// 2 coefficient rows and 5 share rows of 16.5 KB per tile) its time is the
// fastest any kernel can move the split's 470 B/element through those
// physical pages, which is what bench.py reports as `ceiling_measured`.
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace {

constexpr int kMaxIn = 8, kMaxOut = 16;
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

struct StreamArgs {
  const uint8_t* in[kMaxIn];
  uint8_t* out[kMaxOut];
  uint32_t in_bpt[kMaxIn];
  uint32_t out_bpt[kMaxOut];
  int n_in, n_out;
  uint64_t ntiles;
};

__global__ void __launch_bounds__(256) tile_stream_kernel(const StreamArgs a) {
  const uint32_t lane = threadIdx.x & 63u;
  const uint64_t nw = static_cast<uint64_t>(gridDim.x) * 4u;
  const uint64_t w0 = __builtin_amdgcn_readfirstlane(blockIdx.x * 4u + (threadIdx.x >> 6));
  for (uint64_t t = w0; t < a.ntiles; t += nw) {
    u32x4 acc = {0u, 0u, 0u, 0u};
    for (int b = 0; b < a.n_in; ++b) {
      const uint32_t bpt = a.in_bpt[b];
      const u32x4* p = reinterpret_cast<const u32x4*>(a.in[b] + t * bpt);
#pragma unroll 4
      for (uint32_t o = lane; o < bpt / 16u; o += 64u) acc ^= __builtin_nontemporal_load(p + o);
    }
    for (int b = 0; b < a.n_out; ++b) {
      const uint32_t bpt = a.out_bpt[b];
      u32x4* p = reinterpret_cast<u32x4*>(a.out[b] + t * bpt);
#pragma unroll 4
      for (uint32_t o = lane; o < bpt / 16u; o += 64u) __builtin_nontemporal_store(acc + o, p + o);
    }
  }
}

}  // namespace

extern "C" int dn_diag_tile_stream(const void* const* in, const uint32_t* in_bpt, int n_in, void* const* out,
                                   const uint32_t* out_bpt, int n_out, uint64_t ntiles, int grid, void* stream) {
  if (n_in < 0 || n_in > kMaxIn || n_out < 0 || n_out > kMaxOut || grid <= 0) return -1;
  StreamArgs a{};
  for (int b = 0; b < n_in; ++b) {
    if (!in[b] || in_bpt[b] % 16u) return -1;
    a.in[b] = static_cast<const uint8_t*>(in[b]);
    a.in_bpt[b] = in_bpt[b];
  }
  for (int b = 0; b < n_out; ++b) {
    if (!out[b] || out_bpt[b] % 16u) return -1;
    a.out[b] = static_cast<uint8_t*>(out[b]);
    a.out_bpt[b] = out_bpt[b];
  }
  a.n_in = n_in;
  a.n_out = n_out;
  a.ntiles = ntiles;
  hipLaunchKernelGGL(tile_stream_kernel, dim3(grid), dim3(256), 0, static_cast<hipStream_t>(stream), a);
  return hipGetLastError() == hipSuccess ? 0 : -5;
}
