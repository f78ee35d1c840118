// libmft engine: stream-ordered caching HBM allocator + pinned host allocator.
//
// Replaces MemoryPool / MemoryManager (operators/finetune_ops/core/memory_manager.h:23-194,
// memory_manager.cpp:34-145: 32 power-of-two buckets, first fit, no split, linear-scan free) and
// the unimplemented ArenaManager (memory/arena_allocator.h:24-162).  MI355X design:
//   * device segments come from hipMalloc in 2 MiB granules (large) or 2 MiB segments carved into
//     512-B-rounded blocks (small); best-fit from a size-ordered free set, blocks split on
//     allocation and coalesced with free neighbours on release;
//   * a block freed on stream S is reusable at once by work on S (stream order); use on another
//     stream is declared with record_stream(), and the block then waits for an event;
//   * pools: pool 0 serves eager work; a hipGraph capture allocates from a private pool whose
//     blocks are never handed to eager work (the replayed graph keeps writing them) -- the
//     "static weights vs step scratch" split of the reference's ArenaManager falls out of this;
//   * stats: allocated / reserved / peak bytes, segment count; empty_cache() returns whole idle
//     segments to HIP (the reference's clear_unused, memory_manager.cpp:99-145);
//   * a capture runs in hipStreamCaptureModeRelaxed, so a cache miss may hipMalloc a new segment
//     for the graph's private pool (never for pool 0);
//   * segments and cross-stream events come from an AllocatorBackend: HIP in the engine, a host
//     test double in tests/engine_host_selftest.cpp, so the split / coalesce / event bookkeeping
//     runs under ASan / UBSan on a machine without a GPU (CMakePresets.json).
// Sized for 288 GB of HBM3E per GPU: nothing here caps the cache below the device.
#pragma once
#include <hip/hip_runtime.h>

#include <cstddef>
#include <cstdint>
#include <map>
#include <memory>
#include <mutex>
#include <set>
#include <unordered_map>
#include <vector>

namespace mft {
namespace eng {

// Where the caching allocator's memory and stream-ordering events come from.
class AllocatorBackend {
 public:
  virtual ~AllocatorBackend() = default;
  virtual bool map(void** ptr, size_t nbytes) = 0;  // false: out of memory (the cache is trimmed, then retried)
  virtual void unmap(void* ptr) = 0;
  virtual void synchronize() = 0;             // all queued work on the device has completed
  virtual void* record(hipStream_t stream) = 0;  // an event after the work queued on `stream` so far
  virtual bool passed(void* event) = 0;       // that work has completed
  virtual void destroy(void* event) = 0;
};

struct AllocStats {
  size_t allocated = 0, reserved = 0, peak_allocated = 0, peak_reserved = 0;
  uint64_t n_alloc = 0, n_free = 0, n_segments = 0, n_hip_malloc = 0, n_cache_hits = 0;
};

class CachingAllocator {
 public:
  static CachingAllocator& get(int device);  // the engine's HIP-backed allocator of `device`
  // a private allocator over any backend (tests; the engine uses get())
  explicit CachingAllocator(std::unique_ptr<AllocatorBackend> backend);
  ~CachingAllocator();
  CachingAllocator(const CachingAllocator&) = delete;
  CachingAllocator& operator=(const CachingAllocator&) = delete;
  void* allocate(size_t nbytes, hipStream_t stream);
  void release(void* ptr);
  // ptr will be used by `stream` too: on release it is reused only after that work completed
  void record_stream(void* ptr, hipStream_t stream);
  void empty_cache();
  AllocStats stats() const;
  void reset_peak();
  // current pool for new allocations of this thread (0 = eager; >0 = a graph's private pool)
  static int current_pool();
  static void set_current_pool(int pool);
  int new_pool();
  size_t block_size(void* ptr) const;

 private:
  struct Block;
  struct BySize {
    bool operator()(const Block* a, const Block* b) const;
  };
  struct Block {
    void* ptr = nullptr;
    size_t size = 0;
    int pool = 0;
    bool small = false;
    bool allocated = false;
    hipStream_t stream = nullptr;
    Block *prev = nullptr, *next = nullptr;  // neighbours inside the same hipMalloc segment
    std::vector<hipStream_t> uses;          // record_stream
    std::vector<void*> pending;             // backend events to pass before reuse
  };
  using FreeSet = std::set<Block*, BySize>;
  FreeSet& free_set(int pool, bool small);
  Block* find_free(int pool, bool small, size_t size, hipStream_t stream);
  void insert_free(Block* b);
  void erase_free(Block* b);
  void free_block(Block* b);  // coalesce with idle neighbours, then into the free set
  void process_events();
  bool free_idle_segments();
  std::unique_ptr<AllocatorBackend> be_;
  mutable std::mutex mu_;
  std::map<std::pair<int, bool>, FreeSet> free_;
  std::unordered_map<void*, Block*> live_;
  std::vector<Block*> with_events_;
  std::vector<void*> segments_;
  AllocStats st_;
  int next_pool_ = 1;
};

// Pinned (page-locked) host memory for H2D/D2H staging: size-class cache of hipHostMalloc blocks.
class PinnedAllocator {
 public:
  static PinnedAllocator& get();
  void* allocate(size_t nbytes);
  // the block is reused only after the work queued on `stream` so far (async copies) completed
  void release(void* ptr, hipStream_t stream);
  size_t cached_bytes() const;

 private:
  struct FreeBlock {
    void* ptr;
    hipEvent_t ev;
  };
  mutable std::mutex mu_;
  std::multimap<size_t, FreeBlock> free_;
  std::unordered_map<void*, size_t> live_;
  size_t cached_ = 0;
};

}  // namespace eng
}  // namespace mft
