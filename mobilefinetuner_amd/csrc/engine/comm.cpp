// libmft engine: native RCCL communicator + TCP unique-id bootstrap (see comm.h).
#include "engine/comm.h"

#include <arpa/inet.h>
#include <netinet/in.h>
#include <netinet/tcp.h>
#include <rccl/rccl.h>
#include <sys/socket.h>
#include <unistd.h>

#include <chrono>
#include <cstdlib>
#include <cstring>
#include <stdexcept>
#include <string>
#include <thread>
#include <vector>

#include "engine/tensor.h"

namespace mft {
namespace eng {

namespace {

void nccl_ok(ncclResult_t r, const char* what) {
  if (r != ncclSuccess) throw std::runtime_error(std::string("rccl: ") + what + ": " + ncclGetErrorString(r));
}

int env_int(const char* k, int dflt) {
  const char* v = std::getenv(k);
  return v && *v ? std::atoi(v) : dflt;
}

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

// rank 0: accept world - 1 connections and send each the id; others: connect (retrying while rank
// 0 comes up) and receive it.  A 4-byte magic guards against a stray listener on the port.
constexpr uint32_t kMagic = 0x4D465443;  // "MFTC"

void exchange_id(ncclUniqueId& id, int rank, int world, const std::string& addr, int port, double timeout_s) {
  sockaddr_in sa{};
  sa.sin_family = AF_INET;
  sa.sin_port = htons((uint16_t)port);
  if (::inet_pton(AF_INET, addr.c_str(), &sa.sin_addr) != 1) throw std::runtime_error("comm: bad MASTER_ADDR " + addr);
  const auto deadline = std::chrono::steady_clock::now() + std::chrono::duration<double>(timeout_s);
  if (rank == 0) {
    const int fd = ::socket(AF_INET, SOCK_STREAM, 0);
    int one = 1;
    ::setsockopt(fd, SOL_SOCKET, SO_REUSEADDR, &one, sizeof(one));
    if (::bind(fd, reinterpret_cast<sockaddr*>(&sa), sizeof(sa)) != 0 || ::listen(fd, world) != 0) {
      ::close(fd);
      throw std::runtime_error("comm: rank 0 cannot listen on " + addr + ":" + std::to_string(port));
    }
    for (int i = 1; i < world; ++i) {
      const int c = ::accept(fd, nullptr, nullptr);
      if (c < 0) {
        ::close(fd);
        throw std::runtime_error("comm: accept failed");
      }
      const bool ok = send_all(c, &kMagic, 4) && send_all(c, &id, sizeof(id));
      ::close(c);
      if (!ok) {
        ::close(fd);
        throw std::runtime_error("comm: sending the unique id failed");
      }
    }
    ::close(fd);
    return;
  }
  while (true) {
    const int fd = ::socket(AF_INET, SOCK_STREAM, 0);
    if (::connect(fd, reinterpret_cast<const sockaddr*>(&sa), sizeof(sa)) == 0) {
      uint32_t m = 0;
      const bool ok = recv_all(fd, &m, 4) && m == kMagic && recv_all(fd, &id, sizeof(id));
      ::close(fd);
      if (ok) return;
      throw std::runtime_error("comm: bad bootstrap reply from " + addr + ":" + std::to_string(port));
    }
    ::close(fd);
    if (std::chrono::steady_clock::now() > deadline)
      throw std::runtime_error("comm: timed out connecting to rank 0 at " + addr + ":" + std::to_string(port));
    std::this_thread::sleep_for(std::chrono::milliseconds(50));
  }
}

}  // namespace

struct Communicator::Impl {
  ncclComm_t comm = nullptr;
  void* one = nullptr;  // device float for barrier()
};

std::unique_ptr<Communicator> Communicator::from_env(bool force) {
  const int world = env_int("WORLD_SIZE", 1);
  if (world <= 1 && !force) return nullptr;
  std::unique_ptr<Communicator> c(new Communicator());
  c->world_ = std::max(1, world);
  c->rank_ = env_int("RANK", 0);
  c->local_ = env_int("LOCAL_RANK", c->rank_);
  if (c->rank_ < 0 || c->rank_ >= c->world_) throw std::runtime_error("comm: RANK out of range");
  HIP_OK(hipSetDevice(c->local_));
  ncclUniqueId id{};
  if (c->rank_ == 0) nccl_ok(ncclGetUniqueId(&id), "ncclGetUniqueId");
  if (c->world_ > 1) {
    const char* a = std::getenv("MASTER_ADDR");
    const int port = env_int("MFT_COMM_PORT", env_int("MASTER_PORT", 29500) + 1);
    exchange_id(id, c->rank_, c->world_, a && *a ? a : "127.0.0.1", port, env_int("MFT_COMM_TIMEOUT", 300));
  }
  c->impl_ = std::make_unique<Impl>();
  nccl_ok(ncclCommInitRank(&c->impl_->comm, c->world_, id, c->rank_), "ncclCommInitRank");
  HIP_OK(hipMalloc(&c->impl_->one, sizeof(float)));
  return c;
}

Communicator::~Communicator() {
  if (impl_) {
    if (impl_->comm) (void)ncclCommDestroy(impl_->comm);
    if (impl_->one) (void)hipFree(impl_->one);
  }
}

void Communicator::all_reduce_sum(float* buf, size_t n, hipStream_t st) {
  nccl_ok(ncclAllReduce(buf, buf, n, ncclFloat32, ncclSum, impl_->comm, st), "ncclAllReduce(sum)");
}

void Communicator::all_reduce_avg(float* buf, size_t n, hipStream_t st) {
  nccl_ok(ncclAllReduce(buf, buf, n, ncclFloat32, ncclAvg, impl_->comm, st), "ncclAllReduce(avg)");
}

void Communicator::broadcast(void* buf, size_t bytes, int root, hipStream_t st) {
  nccl_ok(ncclBroadcast(buf, buf, bytes, ncclUint8, root, impl_->comm, st), "ncclBroadcast");
}

void Communicator::barrier(hipStream_t st) {
  nccl_ok(ncclAllReduce(impl_->one, impl_->one, 1, ncclFloat32, ncclSum, impl_->comm, st), "barrier");
  HIP_OK(hipStreamSynchronize(st));
}

}  // namespace eng
}  // namespace mft
