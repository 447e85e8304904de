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

// dn_diag_group_stream: the share-emission write pattern of a split without
// its arithmetic — per element the 8-B secret read and n shares of 66 B
// written in the tiled layout (16 u32 planes + the u16 top plane per share
// row, 256 elements per tile) — in one of two wave-to-element mappings:
//   mode 0 (the fused MT draw + split, mt_gen_kernel): one 64-thread
//     workgroup per contiguous range of `epw` elements, emitted 64 at a time
//     (one quarter-tile per group, its tile's other quarters by the same wave
//     before and after it);
//   mode 1 (split_kernel): 256-thread workgroups, wave q of a workgroup the
//     quarter q of every tile it visits (grid-stride over tiles), so a tile's
//     1-KB plane rows are written by four waves at once.
// nt != 0: non-temporal stores.  Values are the secret XOR the plane index.
namespace {
struct GroupArgs {
  const uint64_t* sec;
  uint8_t* shares;
  uint64_t share_stride, n_elem, epw;
  int n_shares, nt;
};

__device__ __forceinline__ void emit_elem(const GroupArgs& a, uint64_t e) {
  const uint64_t v = a.sec[e];
  const uint64_t tile = e >> 8, w = e & 255u;
  for (int x = 0; x < a.n_shares; ++x) {
    uint8_t* tb = a.shares + static_cast<uint64_t>(x) * a.share_stride + tile * 66ull * 256ull;
    uint32_t* pl = reinterpret_cast<uint32_t*>(tb) + w;
    uint16_t* top = reinterpret_cast<uint16_t*>(tb + 64 * 256) + w;
    if (a.nt) {
#pragma unroll
      for (int i = 0; i < 16; ++i) __builtin_nontemporal_store(static_cast<uint32_t>(v) ^ i, pl + i * 256);
      __builtin_nontemporal_store(static_cast<uint16_t>(v >> 55), top);
    } else {
#pragma unroll
      for (int i = 0; i < 16; ++i) pl[i * 256] = static_cast<uint32_t>(v) ^ i;
      *top = static_cast<uint16_t>(v >> 55);
    }
  }
}

__global__ void __launch_bounds__(64) group_stream_range_kernel(const GroupArgs a) {
  const uint64_t e0 = static_cast<uint64_t>(blockIdx.x) * a.epw;
  const uint64_t e1 = e0 + a.epw < a.n_elem ? e0 + a.epw : a.n_elem;
  for (uint64_t e = e0 + threadIdx.x; e < e1; e += 64u) emit_elem(a, e);
}

__global__ void __launch_bounds__(256) group_stream_tile_kernel(const GroupArgs a) {
  const uint64_t ntiles = a.n_elem >> 8;
  for (uint64_t t = blockIdx.x; t < ntiles; t += gridDim.x) emit_elem(a, t * 256u + threadIdx.x);
}
}  // namespace

extern "C" int dn_diag_group_stream(const void* sec, void* shares, uint64_t share_stride, uint64_t n_elem,
                                    int n_shares, int mode, uint64_t epw, int grid, int nt, void* stream) {
  if (!sec || !shares || n_elem % 256u || n_shares < 1 || n_shares > 16) return -1;
  GroupArgs a{static_cast<const uint64_t*>(sec), static_cast<uint8_t*>(shares), share_stride, n_elem, epw, n_shares, nt};
  hipStream_t s = static_cast<hipStream_t>(stream);
  if (mode == 0) {
    if (epw == 0 || epw % 64u) return -1;
    hipLaunchKernelGGL(group_stream_range_kernel, dim3(static_cast<uint32_t>((n_elem + epw - 1) / epw)), dim3(64), 0, s, a);
  } else {
    if (grid <= 0) return -1;
    hipLaunchKernelGGL(group_stream_tile_kernel, dim3(grid), dim3(256), 0, s, a);
  }
  return hipGetLastError() == hipSuccess ? 0 : -5;
}
