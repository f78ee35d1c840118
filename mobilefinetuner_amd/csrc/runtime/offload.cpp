#include "offload.h"

#include <sys/stat.h>

#include <algorithm>
#include <cstdio>
#include <cstring>
#include <fstream>
#include <stdexcept>

namespace mft {

#define HT_CHECK(x)                                                                          \
  do {                                                                                       \
    hipError_t e_ = (x);                                                                     \
    if (e_ != hipSuccess) throw std::runtime_error(std::string("HostTier: ") + hipGetErrorString(e_) + " at " #x); \
  } while (0)

HostTier::HostTier(size_t device_budget_bytes, const std::string& disk_dir, size_t host_budget_bytes)
    : budget_(device_budget_bytes), host_budget_(host_budget_bytes), disk_dir_(disk_dir) {}

HostTier::~HostTier() {
  try {
    if (copy_) hipStreamSynchronize(copy_);
  } catch (...) {
  }
  for (auto& kv : entries_) {
    if (kv.second.host) hipHostFree(kv.second.host);
    if (kv.second.ev) hipEventDestroy(kv.second.ev);
    if (kv.second.on_disk && !disk_dir_.empty()) std::remove((disk_dir_ + "/" + kv.first + ".bin").c_str());
  }
  if (order_ev_) hipEventDestroy(order_ev_);
  if (copy_) hipStreamDestroy(copy_);
}

HostTier::Entry& HostTier::get(const std::string& name) {
  auto it = entries_.find(name);
  if (it == entries_.end()) throw std::runtime_error("HostTier: unknown entry " + name);
  return it->second;
}
const HostTier::Entry& HostTier::get(const std::string& name) const {
  auto it = entries_.find(name);
  if (it == entries_.end()) throw std::runtime_error("HostTier: unknown entry " + name);
  return it->second;
}

void HostTier::add(const std::string& name, size_t nbytes) {
  std::lock_guard<std::mutex> g(mu_);
  if (entries_.count(name)) throw std::runtime_error("HostTier: duplicate entry " + name);
  if (budget_ && nbytes > budget_)
    throw std::runtime_error("HostTier: entry " + name + " (" + std::to_string(nbytes) +
                             " B) exceeds the device budget (" + std::to_string(budget_) + " B)");
  if (!copy_) {
    // high priority copy stream so prefetches are not starved by compute
    int lo = 0, hi = 0;
    HT_CHECK(hipDeviceGetStreamPriorityRange(&lo, &hi));
    HT_CHECK(hipStreamCreateWithPriority(&copy_, hipStreamNonBlocking, hi));
    HT_CHECK(hipEventCreateWithFlags(&order_ev_, hipEventDisableTiming));
  }
  Entry e;
  e.name = name;
  e.bytes = nbytes;
  HT_CHECK(hipHostMalloc(&e.host, nbytes ? nbytes : 1, hipHostMallocDefault));
  HT_CHECK(hipEventCreateWithFlags(&e.ev, hipEventDisableTiming));
  e.resident = true;
  resident_bytes_ += nbytes;
  host_bytes_ += nbytes;
  e.last_used = ++clock_;
  entries_.emplace(name, e);
}

void HostTier::offload(const std::string& name, const void* dev, hipStream_t compute) {
  std::lock_guard<std::mutex> g(mu_);
  Entry& e = get(name);
  if (e.on_disk) throw std::runtime_error("HostTier: offload into a spilled entry " + name);
  HT_CHECK(hipEventRecord(order_ev_, compute));
  HT_CHECK(hipStreamWaitEvent(copy_, order_ev_, 0));
  HT_CHECK(hipMemcpyAsync(e.host, dev, e.bytes, hipMemcpyDeviceToHost, copy_));
  HT_CHECK(hipEventRecord(e.ev, copy_));
  e.ev_pending = true;
  e.dirty = false;
  d2h_bytes_ += e.bytes;
}

void HostTier::fetch(const std::string& name, void* dev, hipStream_t compute) {
  std::lock_guard<std::mutex> g(mu_);
  Entry& e = get(name);
  if (e.on_disk) throw std::runtime_error("HostTier: fetch of spilled entry " + name + " (unspill first)");
  // the destination buffer may still be read by earlier compute work: order after it
  HT_CHECK(hipEventRecord(order_ev_, compute));
  HT_CHECK(hipStreamWaitEvent(copy_, order_ev_, 0));
  HT_CHECK(hipMemcpyAsync(dev, e.host, e.bytes, hipMemcpyHostToDevice, copy_));
  HT_CHECK(hipEventRecord(e.ev, copy_));
  e.ev_pending = true;
  HT_CHECK(hipStreamWaitEvent(compute, e.ev, 0));
  h2d_bytes_ += e.bytes;
}

void HostTier::synchronize(const std::string& name) {
  hipEvent_t ev;
  {
    std::lock_guard<std::mutex> g(mu_);
    Entry& e = get(name);
    if (!e.ev_pending) return;
    ev = e.ev;
    e.ev_pending = false;
  }
  HT_CHECK(hipEventSynchronize(ev));
}

void HostTier::synchronize_all() {
  if (copy_) HT_CHECK(hipStreamSynchronize(copy_));
  std::lock_guard<std::mutex> g(mu_);
  for (auto& kv : entries_) kv.second.ev_pending = false;
}

void HostTier::mark_resident(const std::string& name, bool r) {
  std::lock_guard<std::mutex> g(mu_);
  Entry& e = get(name);
  if (e.resident == r) return;
  e.resident = r;
  if (r) {
    resident_bytes_ += e.bytes;
    e.last_used = ++clock_;
  } else {
    resident_bytes_ -= e.bytes;
  }
}

void HostTier::touch(const std::string& name) {
  std::lock_guard<std::mutex> g(mu_);
  get(name).last_used = ++clock_;
}

void HostTier::mark_dirty(const std::string& name) {
  std::lock_guard<std::mutex> g(mu_);
  get(name).dirty = true;
}

bool HostTier::dirty(const std::string& name) const {
  std::lock_guard<std::mutex> g(mu_);
  return get(name).dirty;
}

bool HostTier::resident(const std::string& name) const {
  std::lock_guard<std::mutex> g(mu_);
  return get(name).resident;
}

size_t HostTier::bytes(const std::string& name) const {
  std::lock_guard<std::mutex> g(mu_);
  return get(name).bytes;
}

std::vector<std::string> HostTier::victims(size_t need, const std::string& keep) const {
  std::lock_guard<std::mutex> g(mu_);
  std::vector<std::string> out;
  if (!budget_ || resident_bytes_ + need <= budget_) return out;
  std::vector<const Entry*> cand;
  for (auto& kv : entries_)
    if (kv.second.resident && kv.first != keep) cand.push_back(&kv.second);
  std::sort(cand.begin(), cand.end(), [](const Entry* a, const Entry* b) { return a->last_used < b->last_used; });
  size_t res = resident_bytes_;
  for (const Entry* e : cand) {
    if (res + need <= budget_) break;
    out.push_back(e->name);
    res -= e->bytes;
  }
  return out;
}

void* HostTier::host_ptr(const std::string& name) {
  std::lock_guard<std::mutex> g(mu_);
  return get(name).host;
}

void* HostTier::device_ptr(const std::string& name) {
  std::lock_guard<std::mutex> g(mu_);
  Entry& e = get(name);
  if (!e.host) throw std::runtime_error("HostTier: " + name + " is not in host memory");
  hipPointerAttribute_t at{};
  HT_CHECK(hipPointerGetAttributes(&at, e.host));
  if (at.type != hipMemoryTypeHost) throw std::runtime_error("HostTier: " + name + " is not pinned host memory");
  void* d = nullptr;
  HT_CHECK(hipHostGetDevicePointer(&d, e.host, 0));
  if (!d) throw std::runtime_error("HostTier: " + name + " has no device mapping");
  return d;
}

void HostTier::spill(const std::string& name) {
  synchronize(name);
  std::lock_guard<std::mutex> g(mu_);
  Entry& e = get(name);
  if (e.on_disk) return;
  if (disk_dir_.empty()) throw std::runtime_error("HostTier: no disk dir configured");
  ::mkdir(disk_dir_.c_str(), 0755);
  const std::string path = disk_dir_ + "/" + name + ".bin";
  std::ofstream out(path, std::ios::binary | std::ios::trunc);
  out.write(static_cast<const char*>(e.host), (std::streamsize)e.bytes);
  if (!out) throw std::runtime_error("HostTier: disk write failed " + path);
  hipHostFree(e.host);
  e.host = nullptr;
  e.on_disk = true;
  host_bytes_ -= e.bytes;
}

void HostTier::unspill(const std::string& name) {
  std::lock_guard<std::mutex> g(mu_);
  Entry& e = get(name);
  if (!e.on_disk) return;
  HT_CHECK(hipHostMalloc(&e.host, e.bytes ? e.bytes : 1, hipHostMallocDefault));
  const std::string path = disk_dir_ + "/" + name + ".bin";
  std::ifstream in(path, std::ios::binary);
  in.read(static_cast<char*>(e.host), (std::streamsize)e.bytes);
  if (!in) throw std::runtime_error("HostTier: disk read failed " + path);
  e.on_disk = false;
  host_bytes_ += e.bytes;
}

bool HostTier::on_disk(const std::string& name) const {
  std::lock_guard<std::mutex> g(mu_);
  return get(name).on_disk;
}

}  // namespace mft
