// libmft engine: caching allocators (see allocator.h for the design).
#include "engine/allocator.h"

#include <algorithm>
#include <cstdio>

#include "engine/tensor.h"

namespace mft {
namespace eng {

namespace {
constexpr size_t kSmallLimit = 1 << 20;   // requests <= 1 MiB come from small segments
constexpr size_t kSmallSeg = 2 << 20;     // small segment size
constexpr size_t kRound = 512;            // small block granularity
constexpr size_t kLargeRound = 2 << 20;   // large segment granularity
constexpr size_t kSplitMin = 1 << 20;     // remainder worth keeping when splitting a large block
thread_local int t_pool = 0;

size_t round_up(size_t n, size_t m) { return (n + m - 1) / m * m; }
}  // namespace

bool CachingAllocator::BySize::operator()(const Block* a, const Block* b) const {
  if (a->size != b->size) return a->size < b->size;
  return (uintptr_t)a->ptr < (uintptr_t)b->ptr;
}

namespace {
// device memory + HIP events of one GPU
class HipBackend : public AllocatorBackend {
 public:
  explicit HipBackend(int device) : device_(device) {}
  bool map(void** ptr, size_t nbytes) override {
    HIP_OK(hipSetDevice(device_));
    if (hipMalloc(ptr, nbytes) == hipSuccess) return true;
    (void)hipGetLastError();
    return false;
  }
  void unmap(void* ptr) override { HIP_OK(hipFree(ptr)); }
  void synchronize() override { HIP_OK(hipDeviceSynchronize()); }
  void* record(hipStream_t stream) override {
    hipEvent_t e;
    HIP_OK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
    HIP_OK(hipEventRecord(e, stream));
    return (void*)e;
  }
  bool passed(void* event) override { return hipEventQuery((hipEvent_t)event) == hipSuccess; }
  void destroy(void* event) override { (void)hipEventDestroy((hipEvent_t)event); }

 private:
  int device_;
};
}  // namespace

CachingAllocator::CachingAllocator(std::unique_ptr<AllocatorBackend> backend) : be_(std::move(backend)) {}

CachingAllocator::~CachingAllocator() {
  // (the engine's allocators live for the process; private ones release everything they hold)
  std::lock_guard<std::mutex> g(mu_);
  for (Block* b : with_events_)
    for (void* e : b->pending) be_->destroy(e);
  std::vector<Block*> all;
  for (auto& kv : free_) all.insert(all.end(), kv.second.begin(), kv.second.end());
  for (Block* b : with_events_) all.push_back(b);
  for (auto& kv : live_) all.push_back(kv.second);
  for (Block* b : all) delete b;
  for (void* p : segments_) be_->unmap(p);
}

CachingAllocator& CachingAllocator::get(int device) {
  static std::mutex mu;
  static std::vector<CachingAllocator*> all;
  std::lock_guard<std::mutex> g(mu);
  if ((int)all.size() <= device) all.resize(device + 1, nullptr);
  if (!all[device]) all[device] = new CachingAllocator(std::make_unique<HipBackend>(device));  // process lifetime
  return *all[device];
}

int CachingAllocator::current_pool() { return t_pool; }
void CachingAllocator::set_current_pool(int pool) { t_pool = pool; }
int CachingAllocator::new_pool() {
  std::lock_guard<std::mutex> g(mu_);
  return next_pool_++;
}

CachingAllocator::FreeSet& CachingAllocator::free_set(int pool, bool small) { return free_[{pool, small}]; }

void CachingAllocator::insert_free(Block* b) { free_set(b->pool, b->small).insert(b); }
void CachingAllocator::erase_free(Block* b) { free_set(b->pool, b->small).erase(b); }

void CachingAllocator::process_events() {
  // blocks whose cross-stream uses have completed become free
  for (size_t i = 0; i < with_events_.size();) {
    Block* b = with_events_[i];
    bool done = true;
    for (void* e : b->pending) {
      if (!be_->passed(e)) {
        done = false;
        break;
      }
    }
    if (done) {
      for (void* e : b->pending) be_->destroy(e);
      b->pending.clear();
      with_events_[i] = with_events_.back();
      with_events_.pop_back();
      free_block(b);  // (coalesces, so the segment can become whole and idle again)
    } else {
      ++i;
    }
  }
}

CachingAllocator::Block* CachingAllocator::find_free(int pool, bool small, size_t size, hipStream_t stream) {
  FreeSet& fs = free_set(pool, small);
  Block key;
  key.size = size;
  key.ptr = nullptr;
  for (auto it = fs.lower_bound(&key); it != fs.end(); ++it) {
    Block* b = *it;
    if (b->stream != stream) continue;  // stream-ordered reuse only
    fs.erase(it);
    return b;
  }
  return nullptr;
}

bool CachingAllocator::free_idle_segments() {
  bool any = false;
  for (auto& kv : free_) {
    if (kv.first.first != 0) continue;  // a graph's private pool stays mapped while the graph lives
    FreeSet& fs = kv.second;
    for (auto it = fs.begin(); it != fs.end();) {
      Block* b = *it;
      if (!b->prev && !b->next) {  // whole segment idle
        it = fs.erase(it);
        be_->unmap(b->ptr);
        st_.reserved -= b->size;
        st_.n_segments--;
        segments_.erase(std::remove(segments_.begin(), segments_.end(), b->ptr), segments_.end());
        delete b;
        any = true;
      } else {
        ++it;
      }
    }
  }
  return any;
}

void* CachingAllocator::allocate(size_t nbytes, hipStream_t stream) {
  if (nbytes == 0) nbytes = 1;
  std::lock_guard<std::mutex> g(mu_);
  process_events();
  const bool small = nbytes <= kSmallLimit;
  const size_t size = round_up(nbytes, kRound);
  const int pool = t_pool;
  Block* b = find_free(pool, small, size, stream);
  if (b) {
    st_.n_cache_hits++;
  } else {
    // a miss while a hipGraph is being captured (relaxed capture mode) maps a new segment into the
    // graph's private pool: it stays owned by that pool, so replays never alias eager tensors
    const size_t seg = small ? kSmallSeg : round_up(size, kLargeRound);
    void* p = nullptr;
    if (!be_->map(&p, seg)) {
      be_->synchronize();
      process_events();
      free_idle_segments();
      MFT_CHECK(be_->map(&p, seg), "allocator: out of device memory allocating ", seg, " bytes (allocated ",
                st_.allocated, ", reserved ", st_.reserved, ")");
    }
    st_.n_hip_malloc++;
    st_.n_segments++;
    st_.reserved += seg;
    st_.peak_reserved = std::max(st_.peak_reserved, st_.reserved);
    segments_.push_back(p);
    b = new Block();
    b->ptr = p;
    b->size = seg;
    b->pool = pool;
    b->small = small;
    b->stream = stream;
  }
  // split off the tail when it is worth keeping
  const size_t rem = b->size - size;
  if ((small && rem >= kRound) || (!small && rem >= kSplitMin)) {
    Block* r = new Block();
    r->ptr = (char*)b->ptr + size;
    r->size = rem;
    r->pool = b->pool;
    r->small = b->small;
    r->stream = b->stream;
    r->prev = b;
    r->next = b->next;
    if (b->next) b->next->prev = r;
    b->next = r;
    b->size = size;
    insert_free(r);
  }
  b->allocated = true;
  live_[b->ptr] = b;
  st_.allocated += b->size;
  st_.peak_allocated = std::max(st_.peak_allocated, st_.allocated);
  st_.n_alloc++;
  return b->ptr;
}

void CachingAllocator::record_stream(void* ptr, hipStream_t stream) {
  std::lock_guard<std::mutex> g(mu_);
  auto it = live_.find(ptr);
  if (it == live_.end()) return;
  Block* b = it->second;
  if (stream != b->stream && std::find(b->uses.begin(), b->uses.end(), stream) == b->uses.end())
    b->uses.push_back(stream);
}

void CachingAllocator::release(void* ptr) {
  if (!ptr) return;
  std::lock_guard<std::mutex> g(mu_);
  auto it = live_.find(ptr);
  MFT_CHECK(it != live_.end(), "allocator: release of an unknown pointer");
  Block* b = it->second;
  live_.erase(it);
  b->allocated = false;
  st_.allocated -= b->size;
  st_.n_free++;
  if (!b->uses.empty()) {
    for (hipStream_t s : b->uses) b->pending.push_back(be_->record(s));
    b->uses.clear();
    with_events_.push_back(b);
    return;
  }
  free_block(b);
}

void CachingAllocator::free_block(Block* b) {
  // coalesce with free neighbours of the same segment (same pool / stream by construction)
  auto mergeable = [&](Block* n) {
    return n && !n->allocated && n->pending.empty() &&
           std::find(with_events_.begin(), with_events_.end(), n) == with_events_.end();
  };
  if (mergeable(b->prev)) {
    Block* p = b->prev;
    erase_free(p);
    p->size += b->size;
    p->next = b->next;
    if (b->next) b->next->prev = p;
    delete b;
    b = p;
  }
  if (mergeable(b->next)) {
    Block* n = b->next;
    erase_free(n);
    b->size += n->size;
    b->next = n->next;
    if (n->next) n->next->prev = b;
    delete n;
  }
  insert_free(b);
}

void CachingAllocator::empty_cache() {
  std::lock_guard<std::mutex> g(mu_);
  be_->synchronize();
  process_events();
  free_idle_segments();
}

AllocStats CachingAllocator::stats() const {
  std::lock_guard<std::mutex> g(mu_);
  return st_;
}

void CachingAllocator::reset_peak() {
  std::lock_guard<std::mutex> g(mu_);
  st_.peak_allocated = st_.allocated;
  st_.peak_reserved = st_.reserved;
}

size_t CachingAllocator::block_size(void* ptr) const {
  std::lock_guard<std::mutex> g(mu_);
  auto it = live_.find(ptr);
  return it == live_.end() ? 0 : it->second->size;
}

// ------------------------------------------------------------------ pinned host
PinnedAllocator& PinnedAllocator::get() {
  static PinnedAllocator* a = new PinnedAllocator();
  return *a;
}

void* PinnedAllocator::allocate(size_t nbytes) {
  const size_t size = round_up(std::max<size_t>(nbytes, 1), 4096);
  std::lock_guard<std::mutex> g(mu_);
  for (auto it = free_.lower_bound(size); it != free_.end() && it->first <= size * 2; ++it) {
    if (hipEventQuery(it->second.ev) != hipSuccess) continue;  // a copy still reads / writes it
    void* p = it->second.ptr;
    (void)hipEventDestroy(it->second.ev);
    cached_ -= it->first;
    live_[p] = it->first;
    free_.erase(it);
    return p;
  }
  void* p = nullptr;
  HIP_OK(hipHostMalloc(&p, size, hipHostMallocDefault));
  live_[p] = size;
  return p;
}

void PinnedAllocator::release(void* ptr, hipStream_t stream) {
  if (!ptr) return;
  std::lock_guard<std::mutex> g(mu_);
  auto it = live_.find(ptr);
  MFT_CHECK(it != live_.end(), "pinned allocator: unknown pointer");
  hipEvent_t ev;
  HIP_OK(hipEventCreateWithFlags(&ev, hipEventDisableTiming));
  HIP_OK(hipEventRecord(ev, stream));
  free_.emplace(it->second, FreeBlock{ptr, ev});
  cached_ += it->second;
  live_.erase(it);
}

size_t PinnedAllocator::cached_bytes() const {
  std::lock_guard<std::mutex> g(mu_);
  return cached_;
}

}  // namespace eng
}  // namespace mft
