// vmm_block.cpp — share blocks built from physical chunks (HIP virtual memory).
//
// The split's time at 2^24 depends on the physical pages of its share block
// (DESIGN.md §5.2): a 5.5 GB block from one allocation lands in a "fast"
// (writes at 6.1-7.0 TB/s) or "slow" (5.0-5.5 TB/s) class.  This allocator
// builds a block from physical chunks of `chunk_bytes` (hipMemCreate) mapped
// back to back into one reserved virtual range, so the caller can choose the
// block's physical composition; opt-in (`dn_block_alloc`), the product's
// "caller owns memory" contract is unchanged.  Host code, HIP runtime API only.
#include <hip/hip_runtime.h>

#include <cstdlib>
#include <map>
#include <mutex>
#include <vector>

#include "dn_internal.hpp"

namespace dn {
namespace {

struct Block {
  uint64_t span = 0;  // reserved / mapped bytes
  uint64_t chunk = 0;
  std::vector<hipMemGenericAllocationHandle_t> handles;
};

std::mutex& blocks_mutex() {
  static std::mutex* m = new std::mutex;  // never destroyed (the runtime may go first)
  return *m;
}
std::map<uintptr_t, Block>& blocks() {
  static auto* b = new std::map<uintptr_t, Block>;
  return *b;
}

void release(void* base, Block& b, uint64_t mapped) {
  if (mapped) (void)hipMemUnmap(base, mapped);
  (void)hipMemAddressFree(base, b.span);
  for (auto h : b.handles) (void)hipMemRelease(h);
  b.handles.clear();
}

}  // namespace
}  // namespace dn

using namespace dn;

extern "C" int dn_block_granularity(int device, uint64_t* bytes) {
  if (!bytes) return set_error(DN_ERR_ARG, "dn_block_granularity: null pointer");
  hipMemAllocationProp prop{};
  prop.type = hipMemAllocationTypePinned;
  prop.location.type = hipMemLocationTypeDevice;
  prop.location.id = device;
  size_t g = 0;
  const hipError_t e = hipMemGetAllocationGranularity(&g, &prop, hipMemAllocationGranularityMinimum);
  if (e != hipSuccess) return set_error(DN_ERR_HIP, "dn_block_granularity: %s", hipGetErrorString(e));
  *bytes = g;
  return DN_OK;
}

extern "C" int dn_block_alloc(uint64_t bytes, uint64_t chunk_bytes, int device, void** ptr) {
  if (!ptr || bytes == 0) return set_error(DN_ERR_ARG, "dn_block_alloc: bad arguments");
  *ptr = nullptr;
  uint64_t gran = 0;
  if (int rc = dn_block_granularity(device, &gran)) return rc;
  uint64_t chunk = chunk_bytes ? chunk_bytes : (2ull << 20);
  chunk = (chunk + gran - 1) / gran * gran;
  const uint64_t nch = (bytes + chunk - 1) / chunk;
  Block b;
  b.span = nch * chunk;
  b.chunk = chunk;
  hipMemAllocationProp prop{};
  prop.type = hipMemAllocationTypePinned;
  prop.location.type = hipMemLocationTypeDevice;
  prop.location.id = device;
  void* base = nullptr;
  // DN_BLOCK_ALIGN_LOG2 (tuning build): the virtual range's alignment (placement probes)
  uint64_t align = 1ull << 21;
  if (const char* al = tune_env("DN_BLOCK_ALIGN_LOG2")) align = 1ull << std::atoi(al);
  hipError_t e = hipMemAddressReserve(&base, b.span, align, nullptr, 0);
  if (e != hipSuccess) return set_error(DN_ERR_HIP, "dn_block_alloc: reserve %llu B: %s",
                                        static_cast<unsigned long long>(b.span), hipGetErrorString(e));
  uint64_t mapped = 0;
  for (uint64_t k = 0; k < nch; ++k) {
    hipMemGenericAllocationHandle_t h{};
    e = hipMemCreate(&h, chunk, &prop, 0);
    if (e != hipSuccess) break;
    b.handles.push_back(h);
    e = hipMemMap(static_cast<uint8_t*>(base) + k * chunk, chunk, 0, h, 0);
    if (e != hipSuccess) break;
    mapped += chunk;
  }
  if (e == hipSuccess) {
    hipMemAccessDesc acc{};
    acc.location = prop.location;
    acc.flags = hipMemAccessFlagsProtReadWrite;
    e = hipMemSetAccess(base, b.span, &acc, 1);
  }
  if (e != hipSuccess) {
    // a partial mapping is unmapped piece by piece (one unmap per mapped chunk)
    for (uint64_t off = 0; off < mapped; off += chunk) (void)hipMemUnmap(static_cast<uint8_t*>(base) + off, chunk);
    release(base, b, 0);
    return set_error(DN_ERR_HIP, "dn_block_alloc: %llu B in %llu-B chunks: %s", static_cast<unsigned long long>(bytes),
                     static_cast<unsigned long long>(chunk), hipGetErrorString(e));
  }
  std::lock_guard<std::mutex> g(blocks_mutex());
  blocks()[reinterpret_cast<uintptr_t>(base)] = std::move(b);
  *ptr = base;
  return DN_OK;
}

// A freed block gives its physical chunks back but never its virtual range:
// the range stays reserved (retired), so no later block or allocation is ever
// placed at an address a freed block's translations used.  Re-reserving a
// freed range gave a new block the old block's address, and that block's
// contents then changed under unrelated allocations
// (scripts/msv_block_debug.py, pass r04i: every new block at a freed block's
// address; never otherwise).  The cost is address space only: 2^47 bytes
// retire ~25,000 freed 5.5 GB blocks, and frees are rare (the Python pool
// reuses idle blocks; memory.empty_cache() and pool overflow free).
extern "C" int dn_block_free(void* ptr) {
  if (!ptr) return DN_OK;
  Block b;
  {
    std::lock_guard<std::mutex> g(blocks_mutex());
    auto it = blocks().find(reinterpret_cast<uintptr_t>(ptr));
    if (it == blocks().end()) return set_error(DN_ERR_ARG, "dn_block_free: not a dn_block_alloc pointer");
    b = std::move(it->second);
    blocks().erase(it);
  }
  // kernels still using the block finish before its pages go (a free is rare)
  hipError_t first = hipDeviceSynchronize();
  // per-chunk unmap: every mapping was made chunk by chunk
  for (uint64_t off = 0; off < b.span; off += b.chunk) {
    const hipError_t e = hipMemUnmap(static_cast<uint8_t*>(ptr) + off, b.chunk);
    if (first == hipSuccess) first = e;
  }
  for (auto h : b.handles) {
    const hipError_t e = hipMemRelease(h);
    if (first == hipSuccess) first = e;
  }
  b.handles.clear();
  if (first != hipSuccess) return set_error(DN_ERR_HIP, "dn_block_free: %s", hipGetErrorString(first));
  return DN_OK;
}
