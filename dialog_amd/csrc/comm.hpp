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
#include <stdexcept>
#include <string>
#include <vector>

namespace dlg {

enum class DType { I32, I64, F64, U8 };
size_t dtype_size(DType t);

// The group was aborted (a rank failed, or a collective timed out): thrown by every later
// collective and wait of every rank of the group.  The group stays aborted -- its contexts can
// only be destroyed -- like an RCCL communicator after ncclCommAbort.
struct CommAborted : std::runtime_error {
  using std::runtime_error::runtime_error;
};

class Comm {
 public:
  virtual ~Comm() = default;
  int rank() const { return rank_; }
  int world() const { return world_; }
  // collectives (not point-to-point ops) issued so far: the divergence check compares it over
  // ranks (sends and receives differ by rank position in the PCL refit's hand-over chain)
  uint64_t ops() const { return ops_; }
  // in-place elementwise sum over ranks (device buffer)
  void allreduce_sum(void* dev, size_t count, DType t, hipStream_t s) {
    enter();
    do_allreduce_sum(dev, count, t, s);
  }
  void allreduce_max_f64(double* dev, size_t count, hipStream_t s) {
    enter();
    do_allreduce_max_f64(dev, count, s);
  }
  // recv[r * count + i] = send_of_rank_r[i]   (device buffers; send may alias recv + rank*count)
  void allgather(const void* send, void* recv, size_t count, DType t, hipStream_t s) {
    enter();
    do_allgather(send, recv, count, t, s);
  }
  // point to point (stream-ordered; every send has its matching recv on the peer) and broadcast
  // of root's buffer to every rank (in place)
  void send(const void* dev, size_t count, DType t, int peer, hipStream_t s) {
    check();
    do_send(dev, count, t, peer, s);
  }
  void recv(void* dev, size_t count, DType t, int peer, hipStream_t s) {
    check();
    do_recv(dev, count, t, peer, s);
  }
  void broadcast(void* dev, size_t count, DType t, int root, hipStream_t s) {
    enter();
    do_broadcast(dev, count, t, root, s);
  }

  // Failure propagation (every rank returns a status).  abort(): this rank failed
  // (why = its error); every peer blocked in, or entering, a collective or a host wait of the
  // group gets CommAborted within milliseconds (loopback: the group's condition variables;
  // RCCL: a poison word in a node-local shared-memory page named after the unique id, then
  // ncclCommAbort so the device-side waits of the collectives end).  Idempotent.
  virtual void abort(const std::string& why) { (void)why; }
  // throws CommAborted if the group was aborted (by any rank) or the communicator reported an
  // asynchronous error; host wait loops poll it
  virtual void check() {}
  // true when a collective makes the device wait for the peers (RCCL): host waits on a stream
  // holding one must poll check() (sync_stream) instead of blocking in the HIP runtime
  virtual bool device_waits() const { return false; }
  // hipStreamSynchronize, or (device_waits) a polling wait that throws CommAborted when the group
  // is aborted and aborts the group after timeout_ms without progress (0: no limit)
  void sync_stream(hipStream_t s);
  int64_t timeout_ms = 600000;

 protected:
  virtual void do_allreduce_sum(void* dev, size_t count, DType t, hipStream_t s) = 0;
  virtual void do_allreduce_max_f64(double* dev, size_t count, hipStream_t s) = 0;
  virtual void do_allgather(const void* send, void* recv, size_t count, DType t, hipStream_t s) = 0;
  virtual void do_send(const void* dev, size_t count, DType t, int peer, hipStream_t s) = 0;
  virtual void do_recv(void* dev, size_t count, DType t, int peer, hipStream_t s) = 0;
  virtual void do_broadcast(void* dev, size_t count, DType t, int root, hipStream_t s) = 0;
  void enter() {
    check();
    ++ops_;
  }
  int rank_ = 0;
  int world_ = 1;
  uint64_t ops_ = 0;
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
