// libmft engine: the collective-communication layer.
//
// One process per GPU.  `Communicator` is the interface the trainer, the bucketed gradient
// reducer and the ZeRO partitioner call; two implementations:
//
//   * RCCL (default, MFT_COMM_BACKEND=rccl): rank 0 creates the ncclUniqueId and hands it to the
//     other ranks over a TCP socket (MASTER_ADDR -- numeric or a host name --, MFT_COMM_PORT or
//     MASTER_PORT + 1; MASTER_PORT itself may be held by the launcher's own store), then
//     ncclCommInitRank over xGMI.  Collectives are enqueued on the caller's HIP stream, so they
//     order with the engine's kernels without host syncs and record into a hipGraph capture.
//   * loopback (MFT_COMM_BACKEND=loopback): a host TCP star around rank 0, for several ranks on
//     ONE GPU (RCCL refuses that) and GPU-less CI of the protocol.  A collective is three stream
//     operations -- D2H copy into a pinned staging buffer, a host function that exchanges / reduces
//     the bytes over the sockets (fixed rank order: deterministic), H2D copy of the result -- so it
//     orders on the stream like an RCCL call and also records into a hipGraph (a host node replays
//     the exchange).
//
// Failure detection: a watchdog thread polls ncclCommGetAsyncError and a progress
// heartbeat (heartbeat(), once per trainer step); an RCCL error, a peer that disappears (loopback:
// socket closed or receive timeout) or no heartbeat for MFT_COMM_TIMEOUT seconds (default 600)
// aborts the communicator (ncclCommAbort lets spinning collective kernels exit) and ends the
// process with exit code 3, so the launcher sees a failure instead of a hang.
#pragma once
#include <hip/hip_runtime.h>

#include <cstddef>
#include <cstdint>
#include <memory>
#include <string>

namespace mft {
namespace eng {

enum class CommType { F32, BF16, I32 };
enum class CommOp { Sum, Avg, Max };
size_t comm_type_size(CommType t);

class Communicator {
 public:
  // RANK / WORLD_SIZE / LOCAL_RANK from the environment; nullptr for a single process unless
  // `force` (a 1-rank communicator exercises the same code path on one GPU).  Selects the device
  // (LOCAL_RANK; loopback: LOCAL_RANK mod the visible device count) before anything else touches
  // it.  MFT_COMM_BACKEND picks the implementation (rccl | loopback).
  static std::unique_ptr<Communicator> from_env(bool force = false);
  virtual ~Communicator();
  int rank() const { return rank_; }
  int world() const { return world_; }
  int local_rank() const { return local_; }
  int device() const { return device_; }
  virtual const char* backend() const = 0;

  // ---- collectives, enqueued on `st` (element counts, not bytes)
  virtual void all_reduce(void* buf, size_t n, CommType t, CommOp op, hipStream_t st) = 0;
  // recv[n_per_rank] = op over ranks of send[rank * n_per_rank, +n_per_rank); in place when
  // recv == send + rank * n_per_rank
  virtual void reduce_scatter(const void* send, void* recv, size_t n_per_rank, CommType t, CommOp op,
                              hipStream_t st) = 0;
  // recv[world * n_per_rank] = concatenation over ranks of send[n_per_rank]; in place when
  // send == recv + rank * n_per_rank
  virtual void all_gather(const void* send, void* recv, size_t n_per_rank, CommType t, hipStream_t st) = 0;
  virtual void broadcast(void* buf, size_t bytes, int root, hipStream_t st) = 0;
  // a host-only loopback communicator (no HIP calls; collectives on HOST buffers, synchronous):
  // the GPU-less CI of the bootstrap, wire protocol, reductions and watchdog (tests/, ctest)
  static std::unique_ptr<Communicator> host_loopback(int rank, int world);
  virtual bool host_only() const { return false; }
  void barrier(hipStream_t st);  // a 1-element all-reduce, then a stream sync

  void all_reduce_sum(float* buf, size_t n, hipStream_t st) { all_reduce(buf, n, CommType::F32, CommOp::Sum, st); }
  void all_reduce_avg(float* buf, size_t n, hipStream_t st) { all_reduce(buf, n, CommType::F32, CommOp::Avg, st); }
  void all_reduce_max(float* buf, size_t n, hipStream_t st) { all_reduce(buf, n, CommType::F32, CommOp::Max, st); }

  // ---- failure detection
  // The idle timer starts at the first heartbeat (setup -- model / checkpoint loading, ZeRO-3
  // layout, the first capture -- is not timed) and is suspended while a QuietScope is open (long
  // rank-local phases: evaluation, checkpoint writes / reads).
  void heartbeat();                                 // progress mark (once per trainer step)
  void quiet(int delta);                            // QuietScope's counter
  struct QuietScope {
    Communicator* c;
    explicit QuietScope(Communicator* cm) : c(cm) {
      if (c) c->quiet(+1);
    }
    ~QuietScope() {
      if (c) {
        c->quiet(-1);
        c->heartbeat();
      }
    }
    QuietScope(const QuietScope&) = delete;
    QuietScope& operator=(const QuietScope&) = delete;
  };
  [[noreturn]] void fail(const std::string& why);  // abort the backend, print, _exit(3)
  int64_t issued = 0;                               // collectives this rank enqueued

 protected:
  Communicator() = default;
  void start_watchdog();
  void stop_watchdog();
  // backend hooks of the watchdog
  virtual bool async_error(std::string* what) {
    (void)what;
    return false;
  }
  virtual void abort_backend() {}
  int rank_ = 0, world_ = 1, local_ = 0, device_ = 0;
  void* barrier_buf_ = nullptr;  // device float for barrier()

 private:
  struct Watchdog;
  std::unique_ptr<Watchdog> wd_;
};

// Resolve MASTER_ADDR (numeric IPv4 or a host name, getaddrinfo) to an IPv4 address string.
std::string resolve_ipv4(const std::string& host);

}  // namespace eng
}  // namespace mft
