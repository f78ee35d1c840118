// libmft engine: native RCCL communicator (SURVEY §2.12 item 11, §2.13 "bootstrap via a tiny C++
// TCP store (unique-id exchange), RANK / WORLD_SIZE / LOCAL_RANK env, launcher mft_launch").
//
// One process per GPU.  Rank 0 creates the ncclUniqueId and hands it to every other rank over a
// loopback TCP socket (MASTER_ADDR, MFT_COMM_PORT or MASTER_PORT + 1 -- MASTER_PORT itself may be
// held by the launcher's own store); then ncclCommInitRank over xGMI.  Collectives run on the
// caller's HIP stream, so they order with the engine's kernels without host syncs.
#pragma once
#include <hip/hip_runtime.h>

#include <cstddef>
#include <memory>

namespace mft {
namespace eng {

class Communicator {
 public:
  // RANK / WORLD_SIZE / LOCAL_RANK from the environment; nullptr for a single process unless
  // `force` (a 1-rank communicator exercises the same code path on one GPU).  Selects the device
  // LOCAL_RANK before anything else touches it.
  static std::unique_ptr<Communicator> from_env(bool force = false);
  ~Communicator();
  int rank() const { return rank_; }
  int world() const { return world_; }
  int local_rank() const { return local_; }
  void all_reduce_sum(float* buf, size_t n, hipStream_t st);
  void all_reduce_avg(float* buf, size_t n, hipStream_t st);
  void broadcast(void* buf, size_t bytes, int root, hipStream_t st);
  void barrier(hipStream_t st);  // a 1-element all-reduce, then a stream sync

 private:
  Communicator() = default;
  struct Impl;
  std::unique_ptr<Impl> impl_;
  int rank_ = 0, world_ = 1, local_ = 0;
};

}  // namespace eng
}  // namespace mft
