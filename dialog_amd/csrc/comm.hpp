// comm.hpp -- rank communicators for the point-sharded RANSAC path.
//
// The only data-path exchanges of a RANSAC round:
//   * allreduce(sum) of the gathered sample points   (16 B x 3 per hypothesis draw)
//   * allreduce(sum) of per-hypothesis inlier counts (int32[D], 16 KiB at D = 4096)
//   * allreduce(sum) of the refit moments            (double[10], fast mode)
//   * allgather of per-rank totals                    (int64 per rank)
//   * padded allgather of inlier ids / xyz            (only when inliers are gathered)
//   * PCL float refit (DLG_REFIT_PCL): allgather of each rank's double term sums (10 doubles),
//     an allgather of every rank's first-walk (ends, starts) (18 floats), then the nine float
//     chains handed from rank to rank in list order (send/recv of 9 floats) and the last
//     rank's sums broadcast
// All operate in place on device buffers on the caller's stream.  RcclComm runs them over RCCL
// (xGMI within a node); LoopbackComm runs an in-process group of ranks that share one device
// (one host thread per rank) for single-GPU rehearsal and tests of the sharded path.
#pragma once

#include <hip/hip_runtime.h>

#include <condition_variable>
#include <cstddef>
#include <cstdint>
#include <memory>
#include <mutex>
#include <string>
#include <vector>

namespace dlg {

enum class DType { I32, I64, F64, U8 };
size_t dtype_size(DType t);

class Comm {
 public:
  virtual ~Comm() = default;
  int rank() const { return rank_; }
  int world() const { return world_; }
  // in-place elementwise sum over ranks (device buffer)
  virtual void allreduce_sum(void* dev, size_t count, DType t, hipStream_t s) = 0;
  virtual void allreduce_max_f64(double* dev, size_t count, hipStream_t s) = 0;
  // recv[r * count + i] = send_of_rank_r[i]   (device buffers; send may alias recv + rank*count)
  virtual void allgather(const void* send, void* recv, size_t count, DType t, hipStream_t s) = 0;
  // point to point (stream-ordered; every send has its matching recv on the peer) and broadcast
  // of root's buffer to every rank (in place)
  virtual void send(const void* dev, size_t count, DType t, int peer, hipStream_t s) = 0;
  virtual void recv(void* dev, size_t count, DType t, int peer, hipStream_t s) = 0;
  virtual void broadcast(void* dev, size_t count, DType t, int root, hipStream_t s) = 0;

 protected:
  int rank_ = 0;
  int world_ = 1;
};

std::unique_ptr<Comm> make_single_comm();
// RCCL loaded at run time (librccl.so.1 -- the copy already in the process if torch loaded one)
bool rccl_get_unique_id(void* out128, std::string* err);
std::unique_ptr<Comm> make_rccl_comm(int rank, int world, const void* uid128, std::string* err);

// in-process loopback group
struct LoopbackGroup;
std::shared_ptr<LoopbackGroup> make_loopback_group(int world);
std::unique_ptr<Comm> make_loopback_comm(std::shared_ptr<LoopbackGroup> g, int rank);

}  // namespace dlg
