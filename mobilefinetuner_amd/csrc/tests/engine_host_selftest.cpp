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
//   * the CLI flag parser (apps/app_common.h);
//   * the data-parallel layouts -- plan_flat's buckets / chunks / replicated fp32 bucket
//     (engine/dist.h) and the ZeRO-3 unit partitions (plan_zero3, engine/zero3.h) at world 1..8;
//   * the loopback communicator in its host-only mode (engine/comm.h: the TCP star bootstrap, the
//     wire protocol, rank-0 reductions, every collective) with 4 ranks as threads, and the watchdog's
//     idle timer / quiet scopes -- under the tsan preset this is the race check of the comm threads.
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

#include <unistd.h>
#include <chrono>
#include <thread>

#include "apps/app_common.h"
#include "engine/allocator.h"
#include "engine/autograd.h"
#include "engine/comm.h"
#include "engine/dist.h"
#include "engine/nn.h"
#include "engine/tensor.h"
#include "engine/zero3.h"

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


// ---------------------------------------------------------------- data-parallel layouts
struct HostParams {
  std::vector<Param> ps;
  std::vector<std::pair<std::string, Param*>> named;
  // sizes; f32[i]: parameter i computes in fp32 (a norm weight)
  HostParams(const std::vector<int64_t>& sizes, const std::vector<bool>& f32) : ps(sizes.size()) {
    for (size_t i = 0; i < sizes.size(); ++i) {
      ps[i].leaf = zeros({sizes[i]}, DType::F32, Device::cpu());
      ps[i].c = f32[i] ? ps[i].leaf : zeros({sizes[i]}, DType::BF16, Device::cpu());
      named.push_back({"p" + std::to_string(i), &ps[i]});
    }
  }
};

void test_plan_flat() {
  std::printf("[dist] plan_flat buckets / chunks / replicated fp32 bucket, world 1..8\n");
  // a GPT-2-like parameter list: per block ln(w,b) f32, qkv, proj, ln2(w,b) f32, fc, fc_out (+ odd sizes)
  std::vector<int64_t> sz;
  std::vector<bool> f32;
  for (int b = 0; b < 6; ++b) {
    for (int64_t n : {768L, 768L}) sz.push_back(n), f32.push_back(true);
    for (int64_t n : {2304L * 768, 2304L, 768L * 768 + 5, 768L}) sz.push_back(n), f32.push_back(false);
    for (int64_t n : {768L, 768L}) sz.push_back(n), f32.push_back(true);
    for (int64_t n : {3072L * 768, 3072L, 768L * 3072, 771L}) sz.push_back(n), f32.push_back(false);
  }
  HostParams hp(sz, f32);
  for (int world : {1, 2, 3, 4, 8}) {
    for (int64_t bucket : {int64_t(1) << 20, int64_t(25) << 20}) {
      const FlatPlan p = plan_flat(hp.named, world, bucket);
      const int nb = (int)p.buckets.size();
      EXPECT(p.replicated.size() == (size_t)nb && p.replicated.back() == 1);
      int nrep = 0;
      for (char r : p.replicated) nrep += r;
      EXPECT(nrep == 1);
      // buckets disjoint, cover [0, numel), each a multiple of world x 64
      std::vector<std::pair<int64_t, int64_t>> bs = p.buckets;
      std::sort(bs.begin(), bs.end());
      int64_t at = 0;
      for (auto& b : bs) {
        EXPECT(b.first == at && b.second > b.first && (b.second - b.first) % (64 * world) == 0);
        at = b.second;
      }
      EXPECT(at == p.numel);
      // every parameter inside its bucket, 64-aligned, no overlaps; fp32 params exactly in the
      // replicated bucket; partitioned buckets in backward order (later params -> lower index)
      std::vector<std::pair<int64_t, int64_t>> spans;
      for (size_t i = 0; i < sz.size(); ++i) {
        const auto& b = p.buckets[p.bucket_of[i]];
        EXPECT(p.offsets[i] % 64 == 0 && p.offsets[i] >= b.first && p.offsets[i] + sz[i] <= b.second);
        EXPECT((bool)p.replicated[p.bucket_of[i]] == (bool)f32[i]);
        spans.push_back({p.offsets[i], p.offsets[i] + sz[i]});
      }
      std::sort(spans.begin(), spans.end());
      for (size_t i = 1; i < spans.size(); ++i) EXPECT(spans[i].first >= spans[i - 1].second);
      int last_b = 1 << 30;
      for (size_t i = 0; i < sz.size(); ++i)
        if (!f32[i]) {
          EXPECT(p.bucket_of[i] <= last_b);
          last_b = p.bucket_of[i];
        }
      if (bucket == (int64_t(1) << 20)) EXPECT(nb > 10);  // small buckets: one or two params each
    }
  }
}

void test_plan_zero3() {
  std::printf("[dist] plan_zero3 unit partitions, world 1..8\n");
  HostParams outer({50257L * 64, 1024L * 64}, {false, false});
  HostParams b0({192L * 64, 192, 64L * 64, 64, 256L * 64, 256, 64L * 256, 64}, std::vector<bool>(8, false));
  HostParams b1({192L * 64, 192, 64L * 64, 64, 256L * 64, 256, 64L * 256, 64}, std::vector<bool>(8, false));
  HostParams rep({64, 64, 64, 64, 64}, std::vector<bool>(5, true));
  for (int world : {1, 2, 4, 7, 8}) {
    const Zero3Layout L = plan_zero3({outer.named, b0.named, b1.named}, rep.named, world);
    int64_t local = 0;
    for (size_t u = 0; u < L.units.size(); ++u) {
      const auto& un = L.units[u];
      EXPECT(un.n % (64 * world) == 0 && un.s * world == un.n && un.local == local);
      local += un.s;
      EXPECT(un.slot == (u == 0 ? 0 : 1 + (int)((u - 1) % 2)));
      const auto& ps = u == 0 ? outer : u == 1 ? b0 : b1;
      for (size_t j = 0; j < un.off.size(); ++j) {
        EXPECT(un.off[j] % 64 == 0 && un.off[j] + ps.ps[j].c.numel() <= un.n);
        if (j) EXPECT(un.off[j] >= un.off[j - 1] + ps.ps[j - 1].c.numel());
      }
    }
    EXPECT(L.rep_off == local && L.rep_at.size() == 5 && L.rep_at[0] == local && L.rep_n == 5 * 64);
    EXPECT(L.numel == L.rep_off + L.rep_n && L.max_block == std::max(L.units[1].n, L.units[2].n));
  }
}

// ---------------------------------------------------------------- host loopback communicator
int free_port() {
  // ephemeral-range port derived from the pid (the test binds it itself: a clash only fails the run)
  return 20000 + (int)(::getpid() % 20000);
}

void test_host_loopback() {
  const int W = 4;
  std::printf("[comm] host-only loopback: %d ranks as threads, every collective, watchdog\n", W);
  ::setenv("MASTER_ADDR", "127.0.0.1", 1);
  ::setenv("MASTER_PORT", std::to_string(free_port()).c_str(), 1);
  ::setenv("MFT_COMM_TIMEOUT", "1", 1);  // the watchdog would _Exit(3) on a wrongly timed idle check
  std::vector<int> fails(W, 0);
  auto rank_fn = [&](int r) {
    int bad = 0;
    auto check = [&](bool c) { bad += !c; };
    std::unique_ptr<Communicator> c = Communicator::host_loopback(r, W);
    check(c->host_only() && c->rank() == r && c->world() == W && std::string(c->backend()) == "loopback");
    // setup longer than the timeout: no heartbeat yet -> not timed
    std::this_thread::sleep_for(std::chrono::milliseconds(1400));
    c->heartbeat();
    // all-reduce sum (fp32), exact: integers
    std::vector<float> a(1000);
    for (int i = 0; i < 1000; ++i) a[i] = (float)(i + r);
    c->all_reduce(a.data(), a.size(), CommType::F32, CommOp::Sum, nullptr);
    for (int i = 0; i < 1000; ++i) check(a[i] == (float)(W * i + W * (W - 1) / 2));
    // max (int32), avg (fp32)
    std::vector<int32_t> m = {r, -r, 7 * r};
    c->all_reduce(m.data(), 3, CommType::I32, CommOp::Max, nullptr);
    check(m[0] == W - 1 && m[1] == 0 && m[2] == 7 * (W - 1));
    float av = (float)(2 * r);
    c->all_reduce(&av, 1, CommType::F32, CommOp::Avg, nullptr);
    check(av == (float)(W - 1));
    // bf16 sum (small integers are exact in bf16)
    std::vector<uint16_t> hb(64);
    for (int i = 0; i < 64; ++i) {
      const float f = (float)(i % 8 + r);
      uint32_t u;
      std::memcpy(&u, &f, 4);
      hb[i] = (uint16_t)(u >> 16);
    }
    c->all_reduce(hb.data(), 64, CommType::BF16, CommOp::Sum, nullptr);
    for (int i = 0; i < 64; ++i) {
      const uint32_t u = (uint32_t)hb[i] << 16;
      float f;
      std::memcpy(&f, &u, 4);
      check(f == (float)(W * (i % 8) + W * (W - 1) / 2));
    }
    // reduce-scatter: chunk r of the sum
    const int n = 96;
    std::vector<float> send(n * W), recv(n);
    for (int i = 0; i < n * W; ++i) send[i] = (float)(i * (r + 1));
    c->reduce_scatter(send.data(), recv.data(), n, CommType::F32, CommOp::Sum, nullptr);
    for (int i = 0; i < n; ++i) check(recv[i] == (float)((r * n + i) * (W * (W + 1) / 2)));
    // all-gather (in place: send == recv + r * n)
    std::vector<float> g(n * W, -1.f);
    for (int i = 0; i < n; ++i) g[r * n + i] = (float)(1000 * r + i);
    c->all_gather(g.data() + r * n, g.data(), n, CommType::F32, nullptr);
    for (int q = 0; q < W; ++q)
      for (int i = 0; i < n; ++i) check(g[q * n + i] == (float)(1000 * q + i));
    // broadcast from rank 2
    std::vector<char> bb(333, (char)r);
    c->broadcast(bb.data(), bb.size(), 2, nullptr);
    for (char ch : bb) check(ch == 2);
    // a long rank-local phase inside a quiet scope: not a hang
    {
      Communicator::QuietScope q(c.get());
      std::this_thread::sleep_for(std::chrono::milliseconds(1400));
    }
    c->barrier(nullptr);
    // many small collectives back to back (tags advance in lockstep)
    float acc = 0.f;
    for (int it = 0; it < 200; ++it) {
      float v = 1.f;
      c->all_reduce(&v, 1, CommType::F32, CommOp::Sum, nullptr);
      acc += v;
    }
    check(acc == 200.f * W);
    c->heartbeat();
    fails[r] = bad;
  };
  std::vector<std::thread> th;
  for (int r = 0; r < W; ++r) th.emplace_back(rank_fn, r);
  for (auto& t : th) t.join();
  for (int r = 0; r < W; ++r) EXPECT(fails[r] == 0);
}

}  // namespace

int main() {
  test_allocator_basic();
  test_allocator_oom_trim();
  test_allocator_stress();
  test_tape();
  test_tape_deep_chain();
  test_args();
  test_plan_flat();
  test_plan_zero3();
  test_host_loopback();
  if (g_fail) std::printf("engine_host_selftest: %d FAILED\n", g_fail);
  else std::printf("engine_host_selftest: PASS\n");
  return g_fail ? 1 : 0;
}
