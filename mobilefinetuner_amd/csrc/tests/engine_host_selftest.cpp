// Host-only self-test of the libmft engine's bookkeeping, meant to run under ASan / UBSan on a
// machine WITHOUT a GPU (CMakePresets.json "asan" / "ubsan": ctest runs it):
//   * the caching allocator (engine/allocator.h) over a host test double of its backend -- best-fit
//     reuse, split / coalesce inside segments, stream-ordered reuse, record_stream events, private
//     graph pools, empty_cache, the out-of-memory trim-and-retry path, and a randomized stress run
//     that writes every live block end to end (ASan flags any block that leaves its segment or
//     overlaps another);
//   * the autograd tape (engine/autograd.h) on host tensors -- views, multi-use accumulation into an
//     installed flat gradient buffer, grad-ready hooks firing once after a leaf's last use,
//     retain_grad, no-grad mode, and a deep chain (node lifetimes);
//   * the CLI flag parser (apps/app_common.h).
// Reference test strategy: SURVEY §4 (the reference's unit tests are plain executables that print
// PASS / FAIL); §5.2 (sanitizers).
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <map>
#include <random>
#include <set>
#include <stdexcept>
#include <string>
#include <vector>

#include "apps/app_common.h"
#include "engine/allocator.h"
#include "engine/autograd.h"
#include "engine/tensor.h"

using namespace mft::eng;

namespace {

int g_fail = 0;
#define EXPECT(cond)                                                        \
  do {                                                                      \
    if (!(cond)) {                                                          \
      std::printf("  FAIL %s:%d: %s\n", __FILE__, __LINE__, #cond);         \
      ++g_fail;                                                             \
    }                                                                       \
  } while (0)

// ---------------------------------------------------------------- allocator backend double
// Segments are exact-size malloc blocks (so ASan sees any access past a segment); an "event" is a
// (stream, ticket) pair that passes once the test marks the stream's work up to the ticket done.
struct HostBackend : AllocatorBackend {
  size_t cap = SIZE_MAX, mapped = 0;
  int maps = 0, unmaps = 0, syncs = 0;
  std::map<void*, size_t> seg;
  std::map<hipStream_t, uint64_t> queued, done;
  struct Ev {
    hipStream_t s;
    uint64_t ticket;
  };
  std::set<Ev*> live_events;
  bool map(void** p, size_t n) override {
    if (mapped + n > cap) return false;
    *p = std::malloc(n);
    if (!*p) return false;
    seg[*p] = n;
    mapped += n;
    ++maps;
    return true;
  }
  void unmap(void* p) override {
    auto it = seg.find(p);
    if (it == seg.end()) throw std::runtime_error("unmap of an unknown segment");
    mapped -= it->second;
    seg.erase(it);
    std::free(p);
    ++unmaps;
  }
  void synchronize() override {
    ++syncs;
    for (auto& kv : queued) done[kv.first] = kv.second;
  }
  void* record(hipStream_t s) override {
    Ev* e = new Ev{s, ++queued[s]};
    live_events.insert(e);
    return e;
  }
  bool passed(void* e) override {
    Ev* ev = (Ev*)e;
    return done[ev->s] >= ev->ticket;
  }
  void destroy(void* e) override {
    live_events.erase((Ev*)e);
    delete (Ev*)e;
  }
  void complete(hipStream_t s) { done[s] = queued[s]; }
  // destroyed by its allocator after it returned every segment and event
  ~HostBackend() override {
    EXPECT(seg.empty() && live_events.empty());
    for (auto& kv : seg) std::free(kv.first);
    for (Ev* e : live_events) delete e;
  }
};

hipStream_t S(int i) { return reinterpret_cast<hipStream_t>((uintptr_t)(0x1000 * i)); }

void test_allocator_basic() {
  std::printf("[allocator] reuse, split / coalesce, streams, pools\n");
  auto* be = new HostBackend();
  {
    CachingAllocator a{std::unique_ptr<AllocatorBackend>(be)};
    // small blocks share one 2 MiB segment, 512-B rounded
    void* p1 = a.allocate(100, S(1));
    void* p2 = a.allocate(1000, S(1));
    void* p3 = a.allocate(513, S(1));
    EXPECT(be->maps == 1);
    EXPECT((char*)p2 == (char*)p1 + 512 && (char*)p3 == (char*)p2 + 1024);
    EXPECT(a.block_size(p3) == 1024);
    std::memset(p1, 1, 100), std::memset(p2, 2, 1000), std::memset(p3, 3, 513);
    // free the middle, then its neighbours: everything coalesces back into the whole segment
    a.release(p2);
    void* q = a.allocate(800, S(1));  // best fit: the 1024-B hole
    EXPECT(q == p2);
    a.release(q);
    a.release(p1);
    a.release(p3);
    AllocStats st = a.stats();
    EXPECT(st.allocated == 0 && st.reserved == (2u << 20) && st.n_segments == 1);
    void* whole = a.allocate(1 << 20, S(1));  // the largest small request fits the coalesced segment
    EXPECT(whole == p1 && be->maps == 1);
    a.release(whole);
    // stream-ordered reuse: a block freed on stream 1 is not handed to stream 2
    void* s2 = a.allocate(100, S(2));
    EXPECT(be->maps == 2 && s2 != p1);
    a.release(s2);
    // record_stream: used by stream 3, reusable only after stream 3's work passed
    void* r = a.allocate(4096, S(1));
    a.record_stream(r, S(3));
    a.release(r);
    void* r2 = a.allocate(4096, S(1));
    EXPECT(r2 != r);
    be->complete(S(3));
    void* r3 = a.allocate(4096, S(1));
    EXPECT(r3 == r);
    a.release(r2);
    a.release(r3);
    // a graph's private pool never serves pool 0
    const int pool = a.new_pool();
    CachingAllocator::set_current_pool(pool);
    void* g = a.allocate(5 << 20, S(1));
    CachingAllocator::set_current_pool(0);
    a.release(g);
    void* e = a.allocate(5 << 20, S(1));
    EXPECT(e != g);
    // large blocks: 2 MiB granules, the tail split off when >= 1 MiB remains
    void* big = a.allocate(9 << 20, S(1));
    EXPECT(a.block_size(big) == (size_t)(9 << 20));
    a.release(e);
    a.release(big);
    // empty_cache returns whole idle pool-0 segments (the graph pool's segment stays)
    a.empty_cache();
    st = a.stats();
    EXPECT(st.allocated == 0 && st.n_segments == 1 && be->seg.size() == 1);
    // peak bookkeeping
    a.reset_peak();
    void* t = a.allocate(3 << 20, S(1));
    EXPECT(a.stats().peak_allocated >= (size_t)(3 << 20));
    a.release(t);
    // releasing an unknown pointer is an error, not corruption
    bool threw = false;
    try {
      int x;
      a.release(&x);
    } catch (const std::runtime_error&) {
      threw = true;
    }
    EXPECT(threw);
  }  // the destructor unmaps every segment, frees every block (checked by ~HostBackend)
}

void test_allocator_oom_trim() {
  std::printf("[allocator] out of memory: idle segments trimmed, then retried\n");
  auto* be = new HostBackend();
  be->cap = 12 << 20;
  {
    CachingAllocator a{std::unique_ptr<AllocatorBackend>(be)};
    void* x = a.allocate(8 << 20, S(1));
    a.release(x);  // cached, 8 MiB mapped
    void* y = a.allocate(6 << 20, S(2));  // other stream: cannot reuse -> map fails -> trim -> retry
    EXPECT(y && be->syncs == 1 && be->mapped == (size_t)(6 << 20));
    bool threw = false;
    try {
      a.allocate(7 << 20, S(2));  // 6 + 7 > 12 even after trimming
    } catch (const std::runtime_error&) {
      threw = true;
    }
    EXPECT(threw);
    a.release(y);
  }
}

void test_allocator_stress() {
  std::printf("[allocator] randomized stress (writes every live block end to end)\n");
  auto* be = new HostBackend();
  {
    CachingAllocator a{std::unique_ptr<AllocatorBackend>(be)};
    std::mt19937_64 rng(7);
    struct Live {
      void* p;
      size_t n;
      unsigned char tag;
    };
    std::vector<Live> live;
    for (int it = 0; it < 20000; ++it) {
      const bool alloc = live.empty() || (rng() % 100) < 55;
      if (alloc && live.size() < 400) {
        const int kind = rng() % 10;
        size_t n = kind < 9 ? 1 + rng() % 40000 : (1 << 20) + rng() % (2 << 20);
        hipStream_t s = S(1 + (int)(rng() % 2));
        void* p = a.allocate(n, s);
        const unsigned char tag = (unsigned char)(rng() & 0xff);
        std::memset(p, tag, n);
        if (rng() % 8 == 0) a.record_stream(p, S(3));
        live.push_back({p, n, tag});
      } else {
        const size_t i = rng() % live.size();
        const Live l = live[i];
        const unsigned char* c = (const unsigned char*)l.p;
        bool intact = c[0] == l.tag && c[l.n - 1] == l.tag && c[l.n / 2] == l.tag;
        EXPECT(intact);
        a.release(l.p);
        live[i] = live.back();
        live.pop_back();
      }
      if (it % 97 == 0) be->complete(S(3));
      if (it % 4999 == 0) a.empty_cache();
    }
    for (auto& l : live) a.release(l.p);
    be->complete(S(3));
    a.empty_cache();
    const AllocStats st = a.stats();
    EXPECT(st.allocated == 0 && st.n_segments == 0 && be->seg.empty());
    std::printf("  %llu allocations, %llu cache hits, %d segments mapped\n", (unsigned long long)st.n_alloc,
                (unsigned long long)st.n_cache_hits, be->maps);
  }
}

// ---------------------------------------------------------------- autograd tape on host tensors
Tensor host(std::vector<float> v, Shape s) { return from_host(v.data(), s, DType::F32, Device::cpu()); }
std::vector<float> vals(const Tensor& t) { return t.to_vector_f32(); }

// y = k * x (elementwise) as a tape node
Tensor scale(const Tensor& x, float k) {
  Tensor y = empty(x.shape(), DType::F32, Device::cpu());
  {
    Tensor xc = x.contiguous().detach();
    for (int64_t i = 0; i < y.numel(); ++i) y.data<float>()[i] = k * xc.data<float>()[i];
  }
  auto n = lambda_node("Scale", [k](std::vector<Tensor>& g) {
    Tensor gi = empty(g[0].shape(), DType::F32, Device::cpu());
    Tensor gc = g[0].contiguous();
    for (int64_t i = 0; i < gi.numel(); ++i) gi.data<float>()[i] = k * gc.data<float>()[i];
    return std::vector<Tensor>{gi};
  });
  connect(n, {x}, {y});
  return y;
}

// s = sum(a * b) (two-input node)
Tensor dot(const Tensor& a, const Tensor& b) {
  Tensor ac = a.contiguous().detach(), bc = b.contiguous().detach();
  MFT_CHECK(ac.numel() == bc.numel(), "dot: ", a.str(), " . ", b.str());
  float acc = 0.f;
  for (int64_t i = 0; i < ac.numel(); ++i) acc += ac.data<float>()[i] * bc.data<float>()[i];
  Tensor s = host({acc}, {1});
  auto n = lambda_node("Dot", [ac, bc](std::vector<Tensor>& g) {
    const float go = g[0].contiguous().data<float>()[0];
    Tensor ga = empty(ac.shape(), DType::F32, Device::cpu()), gb = empty(bc.shape(), DType::F32, Device::cpu());
    for (int64_t i = 0; i < ac.numel(); ++i) {
      ga.data<float>()[i] = go * bc.data<float>()[i];
      gb.data<float>()[i] = go * ac.data<float>()[i];
    }
    return std::vector<Tensor>{ga, gb};
  });
  connect(n, {a, b}, {s});
  return s;
}

void test_tape() {
  std::printf("[autograd] views, accumulation into a flat buffer, ready hooks, retain_grad\n");
  // two leaves whose gradients live in one flat buffer (the optimizer's layout)
  Tensor flat = zeros({16}, DType::F32, Device::cpu());
  Tensor w = host({1, 2, 3, 4, 5, 6}, {2, 3});
  Tensor u = host({0.5f, -1.f, 2.f}, {3});
  w.requires_grad_(true);
  u.requires_grad_(true);
  w.set_grad(flat.slice(0, 0, 6).view({2, 3}));
  u.set_grad(flat.slice(0, 8, 11));
  std::vector<std::string> fired;
  add_ready_hook(w, [&](TensorImpl*) { fired.push_back("w"); });
  add_ready_hook(u, [&](TensorImpl*) { fired.push_back("u"); });
  // loss = dot(3 * w[1, :], u) + dot(w^T[:, 0], u[:2]) + dot(u, u)   (w and u used several times)
  Tensor row = w.select(0, 1);
  Tensor a = scale(row, 3.f);
  Tensor wt = w.t();
  Tensor col = wt.select(0, 0);  // = w[:, 0]
  Tensor l1 = dot(a, u), l2 = dot(col, u.slice(0, 0, 2)), l3 = dot(u, u);
  l2.retain_grad();
  Tensor l12 = dot(host({1.f, 1.f}, {2}), host({0.f, 0.f}, {2}));  // constant branch: no node
  EXPECT(!l12.requires_grad());
  // sum the three scalars through a node with three inputs
  Tensor tot = host({vals(l1)[0] + vals(l2)[0] + vals(l3)[0]}, {1});
  auto sum3 = lambda_node("Sum3", [](std::vector<Tensor>& g) { return std::vector<Tensor>{g[0], g[0], g[0]}; });
  connect(sum3, {l1, l2, l3}, {tot});
  backward({tot});
  // d/dw: row 1 gets 3u, column 0 gets u;  d/du: 3 w[1,:] + w[:,0] + 2u
  const std::vector<float> gw = vals(w.grad()), gu = vals(u.grad());
  const float U[3] = {0.5f, -1.f, 2.f}, W[2][3] = {{1, 2, 3}, {4, 5, 6}};
  const float want_w[6] = {U[0], 0, 0, 3 * U[0] + U[1], 3 * U[1], 3 * U[2]};
  for (int i = 0; i < 6; ++i) EXPECT(std::abs(gw[i] - want_w[i]) < 1e-6f);
  for (int j = 0; j < 3; ++j) EXPECT(std::abs(gu[j] - (3 * W[1][j] + (j < 2 ? W[j][0] : 0.f) + 2 * U[j])) < 1e-6f);
  // the gradients landed IN the flat buffer (views), the gap between them untouched
  const std::vector<float> fv = vals(flat);
  EXPECT(fv[0] == gw[0] && fv[8] == gu[0] && fv[6] == 0.f && fv[7] == 0.f && fv[15] == 0.f);
  // each hook fired exactly once
  EXPECT(fired.size() == 2 && ((fired[0] == "w" && fired[1] == "u") || (fired[0] == "u" && fired[1] == "w")));
  EXPECT(l2.grad().defined() && vals(l2.grad())[0] == 1.f);
  // a second backward accumulates (micro-batches)
  Tensor again = dot(u, u);
  backward({again});
  EXPECT(std::abs(vals(u.grad())[0] - (gu[0] + 2 * U[0])) < 1e-6f);
  EXPECT(fired.size() == 3);
  // no-grad mode records nothing
  {
    NoGradGuard ng;
    Tensor z = scale(w, 2.f);
    EXPECT(!z.requires_grad());
  }
  // reshape / transpose / slice views round-trip gradients
  Tensor m = host({1, 2, 3, 4, 5, 6, 7, 8}, {2, 4});
  m.requires_grad_(true);
  Tensor v = m.reshape({4, 2}).transpose(0, 1).slice(1, 1, 3);  // [2, 2] non-contiguous
  Tensor s = dot(v, host({1, 10, 100, 1000}, {2, 2}));
  backward({s});
  // v[i][j] = m.reshape(4,2)[j+1][i] = m_flat[2 (j+1) + i]
  const std::vector<float> gm = vals(m.grad());
  const float want_m[8] = {0, 0, 1, 100, 10, 1000, 0, 0};
  for (int i = 0; i < 8; ++i) EXPECT(gm[i] == want_m[i]);
}

void test_tape_deep_chain() {
  std::printf("[autograd] 3000-node chain (node lifetimes, replay order)\n");
  Tensor x = host({1.f, -2.f}, {2});
  x.requires_grad_(true);
  Tensor y = x;
  for (int i = 0; i < 3000; ++i) y = scale(y, i % 2 ? 1.001f : 0.999f);
  Tensor l = dot(y, host({1.f, 1.f}, {2}));
  backward({l});
  const float f = std::pow(1.001f * 0.999f, 1500.f);
  const std::vector<float> g = vals(x.grad());
  EXPECT(std::abs(g[0] - f) < 1e-3f && std::abs(g[1] - f) < 1e-3f);
}

void test_args() {
  std::printf("[cli] flag parser\n");
  const char* argv[] = {"prog", "--lr", "3e-4", "--batch_size=8", "--deterministic", "--no_graph=0", "--bogus", "7"};
  bool threw = false;
  try {
    mft::apps::parse_args(8, const_cast<char**>(argv), {"deterministic", "no_graph"}, {"lr", "batch_size"});
  } catch (const std::runtime_error&) {
    threw = true;
  }
  EXPECT(threw);  // strict: unknown flag
  mft::apps::Args a =
      mft::apps::parse_args(8, const_cast<char**>(argv), {"deterministic", "no_graph"}, {"lr", "batch_size"}, true);
  EXPECT(a.f("lr", 0) == 3e-4f && a.i("batch_size", 0) == 8 && a.b("deterministic") && !a.b("no_graph"));
  EXPECT(a.unknown.size() == 1 && a.unknown[0] == "--bogus");
}

}  // namespace

int main() {
  test_allocator_basic();
  test_allocator_oom_trim();
  test_allocator_stress();
  test_tape();
  test_tape_deep_chain();
  test_args();
  if (g_fail) std::printf("engine_host_selftest: %d FAILED\n", g_fail);
  else std::printf("engine_host_selftest: PASS\n");
  return g_fail ? 1 : 0;
}
