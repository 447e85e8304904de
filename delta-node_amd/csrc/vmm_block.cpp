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

#include <atomic>
#include <cstdlib>
#include <map>
#include <mutex>
#include <vector>

#include "dn_internal.hpp"

namespace dn {
namespace {

// One recorded use of a block: an event recorded on `stream` after the work
// that touched the block there (dn_block_record).
struct Use {
  hipStream_t stream = nullptr;
  hipEvent_t event = nullptr;
  bool pending = false;  // recorded since the block's last dn_block_acquire
};

struct Block {
  uint64_t span = 0;  // reserved / mapped bytes
  uint64_t chunk = 0;
  int device = 0;
  std::vector<hipMemGenericAllocationHandle_t> handles;
  std::vector<Use> uses;  // one event per stream the block was used on (kept for re-recording)
};

// Runs `f` with `device` current and restores the caller's device.
template <class F>
hipError_t on_device(int device, F&& f) {
  int prev = -1;
  (void)hipGetDevice(&prev);
  if (prev != device) {
    const hipError_t e = hipSetDevice(device);
    if (e != hipSuccess) return e;
  }
  const hipError_t r = f();
  if (prev != device && prev >= 0) (void)hipSetDevice(prev);
  return r;
}

// virtual address space retired by dn_block_free and by failed allocations
// (their ranges stay reserved; see dn_block_free)
std::atomic<uint64_t> g_retired{0};

std::mutex& blocks_mutex() {
  static std::mutex* m = new std::mutex;  // never destroyed (the runtime may go first)
  return *m;
}
std::map<uintptr_t, Block>& blocks() {
  static auto* b = new std::map<uintptr_t, Block>;
  return *b;
}

// Looks a block up by its base pointer (callers hold blocks_mutex()).
Block* find_block(void* ptr) {
  auto it = blocks().find(reinterpret_cast<uintptr_t>(ptr));
  return it == blocks().end() ? nullptr : &it->second;
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
  b.device = device;
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
    // and its chunks released; the virtual range stays reserved (retired, as
    // in dn_block_free: no later block is placed where these mappings were)
    for (uint64_t off = 0; off < mapped; off += chunk) (void)hipMemUnmap(static_cast<uint8_t*>(base) + off, chunk);
    for (auto h : b.handles) (void)hipMemRelease(h);
    g_retired += b.span;
    return set_error(DN_ERR_HIP, "dn_block_alloc: %llu B in %llu-B chunks: %s", static_cast<unsigned long long>(bytes),
                     static_cast<unsigned long long>(chunk), hipGetErrorString(e));
  }
  std::lock_guard<std::mutex> g(blocks_mutex());
  blocks()[reinterpret_cast<uintptr_t>(base)] = std::move(b);
  *ptr = base;
  return DN_OK;
}

// ---- stream-ordered reuse (memory.py's pool) --------------------------------
// A block that goes idle records an event on every stream that used it; a
// request on stream S may take it at once when every recorded event is on S
// (stream order covers it) or has completed, and dn_block_acquire can make S
// wait for the others instead.  This is torch's caching-allocator rule
// (record_stream), kept per block here because the pool lives outside torch.

extern "C" int dn_block_record(void* ptr, void* stream) {
  std::lock_guard<std::mutex> g(blocks_mutex());
  Block* b = find_block(ptr);
  if (!b) return set_error(DN_ERR_ARG, "dn_block_record: not a dn_block_alloc pointer");
  const auto s = static_cast<hipStream_t>(stream);
  Use* u = nullptr;
  for (auto& x : b->uses)
    if (x.stream == s) u = &x;
  const hipError_t e = on_device(b->device, [&]() -> hipError_t {
    if (!u) {
      hipEvent_t ev = nullptr;
      const hipError_t c = hipEventCreateWithFlags(&ev, hipEventDisableTiming);
      if (c != hipSuccess) return c;
      b->uses.push_back(Use{s, ev, false});
      u = &b->uses.back();
    }
    return hipEventRecord(u->event, s);
  });
  if (e != hipSuccess) return set_error(DN_ERR_HIP, "dn_block_record: %s", hipGetErrorString(e));
  u->pending = true;
  return DN_OK;
}

extern "C" int dn_block_ready(void* ptr, void* stream, int* ready) {
  if (!ready) return set_error(DN_ERR_ARG, "dn_block_ready: null pointer");
  std::lock_guard<std::mutex> g(blocks_mutex());
  Block* b = find_block(ptr);
  if (!b) return set_error(DN_ERR_ARG, "dn_block_ready: not a dn_block_alloc pointer");
  *ready = 1;
  for (auto& u : b->uses) {
    if (!u.pending || u.stream == static_cast<hipStream_t>(stream)) continue;
    const hipError_t q = hipEventQuery(u.event);
    if (q == hipErrorNotReady) {
      *ready = 0;
      return DN_OK;
    }
    if (q != hipSuccess) return set_error(DN_ERR_HIP, "dn_block_ready: %s", hipGetErrorString(q));
    u.pending = false;  // completed: nothing left to order against
  }
  return DN_OK;
}

extern "C" int dn_block_acquire(void* ptr, void* stream, int wait) {
  std::lock_guard<std::mutex> g(blocks_mutex());
  Block* b = find_block(ptr);
  if (!b) return set_error(DN_ERR_ARG, "dn_block_acquire: not a dn_block_alloc pointer");
  const auto s = static_cast<hipStream_t>(stream);
  // Two passes: every other-stream use is checked (wait = 0) or waited for
  // (wait = 1) before any pending flag is cleared, so a RETRY or an error
  // leaves the block's record exactly as it was — a later free or acquire
  // still orders after every stream's queued work on it.
  for (auto& u : b->uses) {
    if (!u.pending || u.stream == s) continue;
    if (!wait) {
      const hipError_t q = hipEventQuery(u.event);
      if (q == hipErrorNotReady) return set_error(DN_ERR_RETRY, "dn_block_acquire: still in use on another stream");
      if (q != hipSuccess) return set_error(DN_ERR_HIP, "dn_block_acquire: %s", hipGetErrorString(q));
    } else {
      const hipError_t e = on_device(b->device, [&] { return hipStreamWaitEvent(s, u.event, 0); });
      if (e != hipSuccess) return set_error(DN_ERR_HIP, "dn_block_acquire: %s", hipGetErrorString(e));
    }
  }
  for (auto& u : b->uses) u.pending = false;  // now ordered before s's next work
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
// reuses idle blocks; memory.empty_cache() and pool overflow free).  The
// retired bytes are counted (dn_block_retired_bytes); memory.py stops mapping
// new blocks — torch.empty instead — once they pass its budget.
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
  // work still using the block finishes before its pages go: the events its
  // uses recorded (dn_block_record), or — a block nobody recorded, e.g. a C
  // caller's — everything queued on the block's own device
  bool recorded = false;
  for (auto& u : b.uses) recorded |= u.pending;
  const hipError_t first = on_device(b.device, [&]() -> hipError_t {
    hipError_t r = recorded ? hipSuccess : hipDeviceSynchronize();
    auto keep = [&r](hipError_t e) {
      if (r == hipSuccess) r = e;
    };
    for (auto& u : b.uses) {
      if (u.pending) keep(hipEventSynchronize(u.event));
      (void)hipEventDestroy(u.event);
    }
    // per-chunk unmap: every mapping was made chunk by chunk
    for (uint64_t off = 0; off < b.span; off += b.chunk) keep(hipMemUnmap(static_cast<uint8_t*>(ptr) + off, b.chunk));
    for (auto h : b.handles) keep(hipMemRelease(h));
    return r;
  });
  b.uses.clear();
  b.handles.clear();
  g_retired += b.span;
  if (first != hipSuccess) return set_error(DN_ERR_HIP, "dn_block_free: %s", hipGetErrorString(first));
  return DN_OK;
}

extern "C" int dn_block_retired_bytes(uint64_t* bytes) {
  if (!bytes) return set_error(DN_ERR_ARG, "dn_block_retired_bytes: null pointer");
  *bytes = g_retired.load();
  return DN_OK;
}
