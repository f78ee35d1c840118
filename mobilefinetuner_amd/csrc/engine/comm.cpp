// libmft engine: collective communication -- RCCL and host-loopback backends, bootstrap,
// watchdog (see comm.h).
#include "engine/comm.h"

#include <arpa/inet.h>
#include <netdb.h>
#include <netinet/in.h>
#include <netinet/tcp.h>
#include <rccl/rccl.h>
#include <sys/socket.h>
#include <sys/time.h>
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <list>
#include <map>
#include <mutex>
#include <set>
#include <stdexcept>
#include <string>
#include <thread>
#include <vector>

#include "engine/tensor.h"
#include "engine/tensor_kernels.h"

namespace mft {
namespace eng {

size_t comm_type_size(CommType t) { return t == CommType::BF16 ? 2 : 4; }

namespace {

int env_int(const char* k, int dflt) {
  const char* v = std::getenv(k);
  return v && *v ? std::atoi(v) : dflt;
}

double comm_timeout_s() { return (double)env_int("MFT_COMM_TIMEOUT", 600); }

bool send_all(int fd, const void* p, size_t n) {
  const char* c = static_cast<const char*>(p);
  while (n) {
    const ssize_t k = ::send(fd, c, n, MSG_NOSIGNAL);
    if (k <= 0) return false;
    c += k;
    n -= (size_t)k;
  }
  return true;
}

bool recv_all(int fd, void* p, size_t n) {
  char* c = static_cast<char*>(p);
  while (n) {
    const ssize_t k = ::recv(fd, c, n, 0);
    if (k <= 0) return false;
    c += k;
    n -= (size_t)k;
  }
  return true;
}

constexpr uint32_t kMagic = 0x4D465443;  // "MFTC": guards against a stray listener on the port

int comm_port() { return env_int("MFT_COMM_PORT", env_int("MASTER_PORT", 29500) + 1); }

sockaddr_in master_sockaddr() {
  const char* a = std::getenv("MASTER_ADDR");
  const std::string ip = resolve_ipv4(a && *a ? a : "127.0.0.1");
  sockaddr_in sa{};
  sa.sin_family = AF_INET;
  sa.sin_port = htons((uint16_t)comm_port());
  if (::inet_pton(AF_INET, ip.c_str(), &sa.sin_addr) != 1) throw std::runtime_error("comm: bad MASTER_ADDR " + ip);
  return sa;
}

void tune_socket(int fd) {
  int one = 1;
  ::setsockopt(fd, IPPROTO_TCP, TCP_NODELAY, &one, sizeof(one));
  timeval tv{};
  tv.tv_sec = (long)comm_timeout_s();
  ::setsockopt(fd, SOL_SOCKET, SO_RCVTIMEO, &tv, sizeof(tv));
}

// Star bootstrap: rank 0 listens and accepts world-1 connections (each peer sends magic + rank);
// the others connect (retrying while rank 0 comes up).  Rank 0 gets fds[r] for r >= 1, every
// other rank fds[0] = its connection to rank 0.
std::vector<int> star_connect(int rank, int world) {
  sockaddr_in sa = master_sockaddr();
  std::vector<int> fds(world, -1);
  if (rank == 0) {
    const int lfd = ::socket(AF_INET, SOCK_STREAM, 0);
    int one = 1;
    ::setsockopt(lfd, SOL_SOCKET, SO_REUSEADDR, &one, sizeof(one));
    if (::bind(lfd, reinterpret_cast<sockaddr*>(&sa), sizeof(sa)) != 0 || ::listen(lfd, world) != 0) {
      ::close(lfd);
      throw std::runtime_error("comm: rank 0 cannot listen on port " + std::to_string(comm_port()));
    }
    for (int i = 1; i < world; ++i) {
      const int c = ::accept(lfd, nullptr, nullptr);
      uint32_t hdr[2] = {0, 0};
      if (c < 0 || !recv_all(c, hdr, sizeof(hdr)) || hdr[0] != kMagic || (int)hdr[1] <= 0 || (int)hdr[1] >= world ||
          fds[hdr[1]] >= 0) {
        ::close(lfd);
        throw std::runtime_error("comm: bad bootstrap connection");
      }
      tune_socket(c);
      fds[hdr[1]] = c;
    }
    ::close(lfd);
    return fds;
  }
  const auto deadline = std::chrono::steady_clock::now() + std::chrono::duration<double>(comm_timeout_s());
  while (true) {
    const int fd = ::socket(AF_INET, SOCK_STREAM, 0);
    if (::connect(fd, reinterpret_cast<const sockaddr*>(&sa), sizeof(sa)) == 0) {
      const uint32_t hdr[2] = {kMagic, (uint32_t)rank};
      if (!send_all(fd, hdr, sizeof(hdr))) {
        ::close(fd);
        throw std::runtime_error("comm: bootstrap send failed");
      }
      tune_socket(fd);
      fds[0] = fd;
      return fds;
    }
    ::close(fd);
    if (std::chrono::steady_clock::now() > deadline)
      throw std::runtime_error("comm: timed out connecting to rank 0 on port " + std::to_string(comm_port()));
    std::this_thread::sleep_for(std::chrono::milliseconds(50));
  }
}

// ---------------------------------------------------------------- host reductions (loopback)
float bf16_to_f(uint16_t h) {
  const uint32_t u = (uint32_t)h << 16;
  float f;
  std::memcpy(&f, &u, 4);
  return f;
}
uint16_t f_to_bf16(float f) {
  uint32_t u;
  std::memcpy(&u, &f, 4);
  if ((u & 0x7fffffffu) > 0x7f800000u) return (uint16_t)((u >> 16) | 0x40);  // a NaN stays a NaN
  return (uint16_t)((u + 0x7fffu + ((u >> 16) & 1u)) >> 16);
}

// working copy (fp32 for F32 / BF16, int32 for I32) op= src; first: copy
void accumulate(std::vector<float>& acc, std::vector<int32_t>& iacc, const char* src, size_t n, CommType t, CommOp op,
                bool first) {
  if (t == CommType::I32) {
    const int32_t* s = reinterpret_cast<const int32_t*>(src);
    for (size_t i = 0; i < n; ++i)
      iacc[i] = first ? s[i] : (op == CommOp::Max ? std::max(iacc[i], s[i]) : iacc[i] + s[i]);
    return;
  }
  for (size_t i = 0; i < n; ++i) {
    float v;
    if (t == CommType::F32) std::memcpy(&v, src + 4 * i, 4);
    else v = bf16_to_f(reinterpret_cast<const uint16_t*>(src)[i]);
    acc[i] = first ? v : (op == CommOp::Max ? std::max(acc[i], v) : acc[i] + v);
  }
}

void finalize(const std::vector<float>& acc, const std::vector<int32_t>& iacc, char* dst, size_t n, CommType t,
              CommOp op, int world) {
  if (t == CommType::I32) {
    int32_t* d = reinterpret_cast<int32_t*>(dst);
    for (size_t i = 0; i < n; ++i) d[i] = op == CommOp::Avg ? iacc[i] / world : iacc[i];
    return;
  }
  const float s = op == CommOp::Avg ? 1.f / (float)world : 1.f;
  for (size_t i = 0; i < n; ++i) {
    const float v = acc[i] * s;
    if (t == CommType::F32) std::memcpy(dst + 4 * i, &v, 4);
    else reinterpret_cast<uint16_t*>(dst)[i] = f_to_bf16(v);
  }
}

// ---------------------------------------------------------------- RCCL
void nccl_ok(ncclResult_t r, const char* what) {
  if (r != ncclSuccess) throw std::runtime_error(std::string("rccl: ") + what + ": " + ncclGetErrorString(r));
}
ncclDataType_t nccl_type(CommType t) {
  return t == CommType::F32 ? ncclFloat32 : t == CommType::BF16 ? ncclBfloat16 : ncclInt32;
}
// CommOp::Avg is issued as ncclSum + an in-place scale: RCCL 2.26's ncclAvg (PreMulSum kernels)
// returns wrong values in the last 4-8 elements of some lengths (fp32, 1-rank group, 66304 / 66240
// elements; ncclSum exact at every length -- scripts/probes/rs_tail.py, profiles/r3_rccl_avg_tail.txt)
ncclRedOp_t nccl_op(CommOp op) { return op == CommOp::Max ? ncclMax : ncclSum; }
void scale_inplace(void* buf, size_t n, CommType t, float s, hipStream_t st) {
  if (n == 0 || t == CommType::I32) return;
  k::Desc d{};
  d.ptr = buf;
  d.dtype = (int)(t == CommType::F32 ? DType::F32 : DType::BF16);
  d.ndim = 1;
  d.shape[0] = (int64_t)n;
  d.stride[0] = 1;
  k::axpy(d, d, s, 0, st);  // buf = s * buf
}

class RcclComm final : public Communicator {
 public:
  RcclComm(int rank, int world, int local) {
    rank_ = rank, world_ = world, local_ = local, device_ = local;
    HIP_OK(hipSetDevice(device_));
    ncclUniqueId id{};
    if (rank_ == 0) nccl_ok(ncclGetUniqueId(&id), "ncclGetUniqueId");
    if (world_ > 1) {
      std::vector<int> fds = star_connect(rank_, world_);
      if (rank_ == 0) {
        for (int r = 1; r < world_; ++r) {
          const bool ok = send_all(fds[r], &id, sizeof(id));
          ::close(fds[r]);
          if (!ok) throw std::runtime_error("comm: sending the unique id failed");
        }
      } else {
        const bool ok = recv_all(fds[0], &id, sizeof(id));
        ::close(fds[0]);
        if (!ok) throw std::runtime_error("comm: receiving the unique id failed");
      }
    }
    nccl_ok(ncclCommInitRank(&comm_, world_, id, rank_), "ncclCommInitRank");
    HIP_OK(hipMalloc(&barrier_buf_, sizeof(float)));
    start_watchdog();
  }
  ~RcclComm() override {
    stop_watchdog();
    if (comm_) (void)ncclCommDestroy(comm_);
    if (barrier_buf_) (void)hipFree(barrier_buf_);
  }
  const char* backend() const override { return "rccl"; }
  void all_reduce(void* buf, size_t n, CommType t, CommOp op, hipStream_t st) override {
    ++issued;
    nccl_ok(ncclAllReduce(buf, buf, n, nccl_type(t), nccl_op(op), comm_, st), "ncclAllReduce");
    if (op == CommOp::Avg && world_ > 1) scale_inplace(buf, n, t, 1.f / (float)world_, st);
  }
  void reduce_scatter(const void* send, void* recv, size_t n, CommType t, CommOp op, hipStream_t st) override {
    ++issued;
    nccl_ok(ncclReduceScatter(send, recv, n, nccl_type(t), nccl_op(op), comm_, st), "ncclReduceScatter");
    if (op == CommOp::Avg && world_ > 1) scale_inplace(recv, n, t, 1.f / (float)world_, st);
  }
  void all_gather(const void* send, void* recv, size_t n, CommType t, hipStream_t st) override {
    ++issued;
    nccl_ok(ncclAllGather(send, recv, n, nccl_type(t), comm_, st), "ncclAllGather");
  }
  void broadcast(void* buf, size_t bytes, int root, hipStream_t st) override {
    ++issued;
    nccl_ok(ncclBroadcast(buf, buf, bytes, ncclUint8, root, comm_, st), "ncclBroadcast");
  }

 protected:
  bool async_error(std::string* what) override {
    ncclResult_t e = ncclSuccess;
    if (!comm_ || ncclCommGetAsyncError(comm_, &e) != ncclSuccess || e == ncclSuccess || e == ncclInProgress)
      return false;
    *what = std::string("RCCL async error: ") + ncclGetErrorString(e);
    return true;
  }
  void abort_backend() override {
    if (comm_) (void)ncclCommAbort(comm_);  // spinning collective kernels see the abort flag and exit
    comm_ = nullptr;
  }

 private:
  ncclComm_t comm_ = nullptr;
};

// ---------------------------------------------------------------- loopback
class LoopbackComm final : public Communicator {
 public:
  enum Kind : uint32_t { kAllReduce = 1, kReduceScatter, kAllGather, kBroadcast };
  struct Op {
    LoopbackComm* self = nullptr;
    uint32_t kind = 0, tag = 0;
    CommType t = CommType::F32;
    CommOp op = CommOp::Sum;
    int root = 0;
    size_t n = 0;  // elements (per rank for reduce-scatter / all-gather); bytes for broadcast
    size_t in_bytes = 0, out_bytes = 0;
    char* in = nullptr;   // pinned: this rank's contribution
    char* out = nullptr;  // pinned: this rank's result
    std::atomic<bool> done{false};
  };

  // host_only: no HIP call at all (GPU-less CI): collectives take HOST buffers and run
  // synchronously on the calling thread (the stream argument is ignored) -- the same bootstrap, wire
  // protocol, rank-0 reduction and watchdog as the device path, which stages through pinned buffers
  // and runs them on a HIP host-callback thread instead
  LoopbackComm(int rank, int world, int local, bool host_only = false) : host_(host_only) {
    rank_ = rank, world_ = world, local_ = local;
    if (!host_) {
      int ndev = 1;
      HIP_OK(hipGetDeviceCount(&ndev));
      device_ = ndev > 0 ? local % ndev : 0;
      HIP_OK(hipSetDevice(device_));
    } else {
      device_ = -1;
    }
    if (world_ > 1) fds_ = star_connect(rank_, world_);
    if (!host_) HIP_OK(hipMalloc(&barrier_buf_, sizeof(float)));
    else barrier_buf_ = &host_barrier_;
    start_watchdog();
  }
  ~LoopbackComm() override {
    if (!host_) (void)hipDeviceSynchronize();
    stop_watchdog();
    for (int fd : fds_)
      if (fd >= 0) ::close(fd);
    for (Op* o : ops_) release(o);
    for (auto& kv : pool_)
      for (void* p : kv.second) {
        if (host_) std::free(p);
        else (void)hipHostFree(p);
      }
    if (barrier_buf_ && !host_) (void)hipFree(barrier_buf_);
  }
  bool host_only() const override { return host_; }
  const char* backend() const override { return "loopback"; }

  void all_reduce(void* buf, size_t n, CommType t, CommOp op, hipStream_t st) override {
    const size_t b = n * comm_type_size(t);
    run(kAllReduce, t, op, 0, n, buf, b, buf, b, st);
  }
  void reduce_scatter(const void* send, void* recv, size_t n, CommType t, CommOp op, hipStream_t st) override {
    const size_t b = n * comm_type_size(t);
    run(kReduceScatter, t, op, 0, n, send, b * world_, recv, b, st);
  }
  void all_gather(const void* send, void* recv, size_t n, CommType t, hipStream_t st) override {
    const size_t b = n * comm_type_size(t);
    run(kAllGather, t, CommOp::Sum, 0, n, send, b, recv, b * world_, st);
  }
  void broadcast(void* buf, size_t bytes, int root, hipStream_t st) override {
    run(kBroadcast, CommType::F32, CommOp::Sum, root, bytes, buf, rank_ == root ? bytes : 0, buf, bytes, st);
  }

 private:
  void* pinned(size_t bytes) {
    if (!bytes) return nullptr;
    auto& v = pool_[bytes];
    if (!v.empty()) {
      void* p = v.back();
      v.pop_back();
      return p;
    }
    void* p = nullptr;
    if (host_) p = std::malloc(bytes);
    else HIP_OK(hipHostMalloc(&p, bytes, hipHostMallocDefault));
    if (!p) throw std::runtime_error("loopback: out of host memory");
    return p;
  }
  void release(Op* o) {
    if (o->in) pool_[o->in_bytes].push_back(o->in);
    if (o->out) pool_[o->out_bytes].push_back(o->out);
    delete o;
  }
  // finished eager ops give their staging buffers back (ops recorded into a graph stay)
  void reclaim() {
    for (auto it = ops_.begin(); it != ops_.end();) {
      Op* o = *it;
      if (!o->done.load() || persistent_.count(o)) {
        ++it;
        continue;
      }
      release(o);
      it = ops_.erase(it);
    }
  }

  void run(uint32_t kind, CommType t, CommOp op, int root, size_t n, const void* dsend, size_t in_bytes, void* drecv,
           size_t out_bytes, hipStream_t st) {
    ++issued;
    std::lock_guard<std::mutex> g(host_mu_);
    reclaim();
    if (host_) {  // synchronous host collective
      Op o;
      o.self = this;
      o.kind = kind, o.t = t, o.op = op, o.root = root, o.n = n;
      o.tag = next_tag_++;
      o.in_bytes = in_bytes, o.out_bytes = out_bytes;
      o.in = static_cast<char*>(pinned(in_bytes));
      o.out = static_cast<char*>(pinned(out_bytes));
      if (in_bytes) std::memcpy(o.in, dsend, in_bytes);
      exchange(o);
      if (out_bytes) std::memcpy(drecv, o.out, out_bytes);
      if (o.in) pool_[in_bytes].push_back(o.in);
      if (o.out) pool_[out_bytes].push_back(o.out);
      return;
    }
    hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
    HIP_OK(hipStreamIsCapturing(st, &cs));
    Op* o = new Op();
    o->self = this;
    o->kind = kind, o->t = t, o->op = op, o->root = root, o->n = n;
    o->tag = next_tag_++;
    o->in_bytes = in_bytes, o->out_bytes = out_bytes;
    o->in = static_cast<char*>(pinned(in_bytes));
    o->out = static_cast<char*>(pinned(out_bytes));
    ops_.push_back(o);
    if (cs == hipStreamCaptureStatusActive) persistent_.insert(o);  // every graph launch replays it
    if (in_bytes) HIP_OK(hipMemcpyAsync(o->in, dsend, in_bytes, hipMemcpyDeviceToHost, st));
    HIP_OK(hipLaunchHostFunc(st, &LoopbackComm::host_fn, o));
    if (out_bytes) HIP_OK(hipMemcpyAsync(drecv, o->out, out_bytes, hipMemcpyHostToDevice, st));
  }

  static void host_fn(void* p) {
    Op* o = static_cast<Op*>(p);
    o->self->exchange(*o);
    o->done.store(true);
  }

  struct Hdr {
    uint32_t magic, kind, tag, pad;
    uint64_t bytes;
  };

  void send_msg(int fd, const Op& o, const void* p, size_t bytes) {
    const Hdr h{kMagic, o.kind, o.tag, 0, bytes};
    if (!send_all(fd, &h, sizeof(h)) || (bytes && !send_all(fd, p, bytes)))
      fail("loopback: a peer connection broke (send)");
  }
  void recv_msg(int fd, const Op& o, void* p, size_t bytes) {
    Hdr h{};
    if (!recv_all(fd, &h, sizeof(h))) fail("loopback: a peer disappeared or timed out (receive)");
    if (h.magic != kMagic || h.kind != o.kind || h.tag != o.tag || h.bytes != bytes)
      fail("loopback: collective mismatch between ranks (kind/tag/bytes " + std::to_string(h.kind) + "/" +
           std::to_string(h.tag) + "/" + std::to_string(h.bytes) + " vs " + std::to_string(o.kind) + "/" +
           std::to_string(o.tag) + "/" + std::to_string(bytes) + ")");
    if (bytes && !recv_all(fd, p, bytes)) fail("loopback: a peer disappeared or timed out (payload)");
  }

  // one collective on the HIP host-callback thread; rank 0 gathers every contribution in rank
  // order (deterministic reduction), computes, and answers each rank
  void exchange(Op& o) {
    std::lock_guard<std::mutex> g(exchange_mu_);
    const int W = world_;
    const size_t es = comm_type_size(o.t);
    if (W > 1 && rank_ != 0) {
      send_msg(fds_[0], o, o.in, o.in_bytes);
      recv_msg(fds_[0], o, o.out, o.out_bytes);
      return;
    }
    switch (o.kind) {
      case kAllReduce:
      case kReduceScatter: {
        const size_t n = o.kind == kAllReduce ? o.n : o.n * W;
        std::vector<float> acc(o.t == CommType::I32 ? 0 : n);
        std::vector<int32_t> iacc(o.t == CommType::I32 ? n : 0);
        std::vector<char> tmp(W > 1 ? n * es : 0), res(n * es);
        accumulate(acc, iacc, o.in, n, o.t, o.op, true);
        for (int r = 1; r < W; ++r) {
          recv_msg(fds_[r], o, tmp.data(), n * es);
          accumulate(acc, iacc, tmp.data(), n, o.t, o.op, false);
        }
        finalize(acc, iacc, res.data(), n, o.t, o.op, W);
        if (o.kind == kAllReduce) {
          std::memcpy(o.out, res.data(), n * es);
          for (int r = 1; r < W; ++r) send_msg(fds_[r], o, res.data(), n * es);
        } else {
          const size_t cb = o.n * es;
          std::memcpy(o.out, res.data(), cb);
          for (int r = 1; r < W; ++r) send_msg(fds_[r], o, res.data() + r * cb, cb);
        }
        break;
      }
      case kAllGather: {
        const size_t cb = o.n * es;
        std::memcpy(o.out, o.in, cb);
        for (int r = 1; r < W; ++r) recv_msg(fds_[r], o, o.out + r * cb, cb);
        for (int r = 1; r < W; ++r) send_msg(fds_[r], o, o.out, cb * W);
        break;
      }
      case kBroadcast: {
        const size_t b = o.n;
        if (o.root == 0) std::memcpy(o.out, o.in, b);
        for (int r = 1; r < W; ++r) recv_msg(fds_[r], o, r == o.root ? o.out : nullptr, r == o.root ? b : 0);
        for (int r = 1; r < W; ++r) send_msg(fds_[r], o, o.out, b);
        break;
      }
      default: fail("loopback: bad collective");
    }
  }

  std::vector<int> fds_;
  std::mutex host_mu_, exchange_mu_;
  std::list<Op*> ops_;
  std::set<Op*> persistent_;
  std::map<size_t, std::vector<void*>> pool_;
  uint32_t next_tag_ = 1;
  bool host_ = false;
  float host_barrier_ = 0.f;
};

int64_t now_ns() {
  return std::chrono::duration_cast<std::chrono::nanoseconds>(std::chrono::steady_clock::now().time_since_epoch())
      .count();
}

}  // namespace

std::string resolve_ipv4(const std::string& host) {
  in_addr a{};
  if (::inet_pton(AF_INET, host.c_str(), &a) == 1) return host;
  addrinfo hints{}, *res = nullptr;
  hints.ai_family = AF_INET;
  hints.ai_socktype = SOCK_STREAM;
  const int rc = ::getaddrinfo(host.c_str(), nullptr, &hints, &res);
  if (rc != 0 || !res) throw std::runtime_error("comm: cannot resolve MASTER_ADDR '" + host + "': " + gai_strerror(rc));
  char buf[INET_ADDRSTRLEN] = {0};
  ::inet_ntop(AF_INET, &reinterpret_cast<sockaddr_in*>(res->ai_addr)->sin_addr, buf, sizeof(buf));
  ::freeaddrinfo(res);
  return buf;
}

// ---------------------------------------------------------------- watchdog
struct Communicator::Watchdog {
  std::thread th;
  std::mutex mu;
  std::condition_variable cv;
  bool stop = false;
  std::atomic<int64_t> last_ns{0};  // 0: no heartbeat yet (setup is not timed)
  std::atomic<int> quiet{0};
};

void Communicator::start_watchdog() {
  wd_ = std::make_unique<Watchdog>();
  const double timeout = comm_timeout_s();
  Watchdog* wd = wd_.get();
  wd->th = std::thread([this, wd, timeout]() {
    std::unique_lock<std::mutex> lk(wd->mu);
    while (!wd->stop) {
      wd->cv.wait_for(lk, std::chrono::milliseconds(250));
      if (wd->stop) break;
      std::string what;
      if (async_error(&what)) fail(what);
      if (wd->quiet.load() > 0) wd->last_ns = now_ns();
      const int64_t last = wd->last_ns.load();
      const double idle = last > 0 ? (double)(now_ns() - last) * 1e-9 : 0.0;
      if (timeout > 0 && idle > timeout)
        fail("no progress for " + std::to_string((int)idle) + " s (MFT_COMM_TIMEOUT=" + std::to_string((int)timeout) +
             "): a peer rank is gone or hung");
    }
  });
}

void Communicator::stop_watchdog() {
  if (!wd_) return;
  {
    std::lock_guard<std::mutex> g(wd_->mu);
    wd_->stop = true;
  }
  wd_->cv.notify_all();
  if (wd_->th.joinable()) wd_->th.join();
  wd_.reset();
}

void Communicator::heartbeat() {
  if (wd_) wd_->last_ns = now_ns();
}

void Communicator::quiet(int delta) {
  if (wd_) wd_->quiet += delta;
}

void Communicator::fail(const std::string& why) {
  std::fprintf(stderr, "[mft comm] rank %d/%d (%s): %s -- aborting\n", rank_, world_, backend(), why.c_str());
  std::fflush(stderr);
  std::fflush(stdout);
  abort_backend();
  std::_Exit(3);
}

Communicator::~Communicator() = default;

std::unique_ptr<Communicator> Communicator::from_env(bool force) {
  const int world = std::max(1, env_int("WORLD_SIZE", 1));
  if (world <= 1 && !force) return nullptr;
  const int rank = env_int("RANK", 0);
  const int local = env_int("LOCAL_RANK", rank);
  if (rank < 0 || rank >= world) throw std::runtime_error("comm: RANK out of range");
  const char* b = std::getenv("MFT_COMM_BACKEND");
  const std::string be = b && *b ? b : "rccl";
  if (be == "loopback") return std::unique_ptr<Communicator>(new LoopbackComm(rank, world, local));
  if (be != "rccl") throw std::runtime_error("comm: unknown MFT_COMM_BACKEND '" + be + "' (rccl | loopback)");
  return std::unique_ptr<Communicator>(new RcclComm(rank, world, local));
}

void Communicator::barrier(hipStream_t st) {
  all_reduce(barrier_buf_, 1, CommType::F32, CommOp::Sum, st);
  if (!host_only()) HIP_OK(hipStreamSynchronize(st));
}

std::unique_ptr<Communicator> Communicator::host_loopback(int rank, int world) {
  if (rank < 0 || rank >= world) throw std::runtime_error("comm: RANK out of range");
  return std::unique_ptr<Communicator>(new LoopbackComm(rank, world, rank, true));
}

}  // namespace eng
}  // namespace mft
