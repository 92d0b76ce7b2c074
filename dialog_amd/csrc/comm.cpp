// comm.cpp -- Single / RCCL / in-process loopback communicators (see comm.hpp).
#include "comm.hpp"

#include <dlfcn.h>
#include <rccl/rccl.h>

#include <cstring>
#include <deque>
#include <stdexcept>

namespace dlg {

size_t dtype_size(DType t) {
  switch (t) {
    case DType::I32: return 4;
    case DType::I64: return 8;
    case DType::F64: return 8;
    case DType::U8: return 1;
  }
  return 1;
}

static void hip_check(hipError_t e, const char* what) {
  if (e != hipSuccess) throw std::runtime_error(std::string(what) + ": " + hipGetErrorString(e));
}

// ---------------------------------------------------------------------------------------------
class SingleComm final : public Comm {
 public:
  void allreduce_sum(void*, size_t, DType, hipStream_t) override {}
  void allreduce_max_f64(double*, size_t, hipStream_t) override {}
  void allgather(const void* send, void* recv, size_t count, DType t, hipStream_t s) override {
    if (send != recv && count)
      hip_check(hipMemcpyAsync(recv, send, count * dtype_size(t), hipMemcpyDeviceToDevice, s),
                "allgather copy");
  }
  void send(const void*, size_t, DType, int, hipStream_t) override {
    throw std::runtime_error("send on a single-rank communicator");
  }
  void recv(void*, size_t, DType, int, hipStream_t) override {
    throw std::runtime_error("recv on a single-rank communicator");
  }
  void broadcast(void*, size_t, DType, int, hipStream_t) override {}
};

std::unique_ptr<Comm> make_single_comm() { return std::make_unique<SingleComm>(); }

// ---------------------------------------------------------------------------------------------
// RCCL, resolved with dlopen so single-GPU use never needs librccl and so the process shares the
// one RCCL copy torch may already have loaded (same SONAME librccl.so.1).
struct RcclApi {
  void* h = nullptr;
  ncclResult_t (*GetUniqueId)(ncclUniqueId*) = nullptr;
  ncclResult_t (*CommInitRank)(ncclComm_t*, int, ncclUniqueId, int) = nullptr;
  ncclResult_t (*CommDestroy)(ncclComm_t) = nullptr;
  ncclResult_t (*AllReduce)(const void*, void*, size_t, ncclDataType_t, ncclRedOp_t, ncclComm_t,
                            hipStream_t) = nullptr;
  ncclResult_t (*AllGather)(const void*, void*, size_t, ncclDataType_t, ncclComm_t,
                            hipStream_t) = nullptr;
  ncclResult_t (*Send)(const void*, size_t, ncclDataType_t, int, ncclComm_t, hipStream_t) = nullptr;
  ncclResult_t (*Recv)(void*, size_t, ncclDataType_t, int, ncclComm_t, hipStream_t) = nullptr;
  ncclResult_t (*Broadcast)(const void*, void*, size_t, ncclDataType_t, int, ncclComm_t,
                            hipStream_t) = nullptr;
  const char* (*GetErrorString)(ncclResult_t) = nullptr;
  bool load(std::string* err) {
    if (h) return true;
    const char* names[] = {"librccl.so.1", "librccl.so", "/opt/rocm/lib/librccl.so.1"};
    for (const char* n : names) {
      h = dlopen(n, RTLD_NOW | RTLD_GLOBAL);
      if (h) break;
    }
    if (!h) {
      if (err) *err = std::string("cannot load librccl: ") + dlerror();
      return false;
    }
#define DLG_SYM(field, name)                                              \
  field = reinterpret_cast<decltype(field)>(dlsym(h, name));              \
  if (!field) {                                                           \
    if (err) *err = std::string("librccl missing symbol ") + name;        \
    return false;                                                         \
  }
    DLG_SYM(GetUniqueId, "ncclGetUniqueId");
    DLG_SYM(CommInitRank, "ncclCommInitRank");
    DLG_SYM(CommDestroy, "ncclCommDestroy");
    DLG_SYM(AllReduce, "ncclAllReduce");
    DLG_SYM(AllGather, "ncclAllGather");
    DLG_SYM(Send, "ncclSend");
    DLG_SYM(Recv, "ncclRecv");
    DLG_SYM(Broadcast, "ncclBroadcast");
    DLG_SYM(GetErrorString, "ncclGetErrorString");
#undef DLG_SYM
    return true;
  }
};

static RcclApi& rccl() {
  static RcclApi api;
  return api;
}

static ncclDataType_t nccl_type(DType t) {
  switch (t) {
    case DType::I32: return ncclInt32;
    case DType::I64: return ncclInt64;
    case DType::F64: return ncclFloat64;
    case DType::U8: return ncclUint8;
  }
  return ncclUint8;
}

bool rccl_get_unique_id(void* out128, std::string* err) {
  if (!rccl().load(err)) return false;
  ncclUniqueId id;
  ncclResult_t r = rccl().GetUniqueId(&id);
  if (r != ncclSuccess) {
    if (err) *err = std::string("ncclGetUniqueId: ") + rccl().GetErrorString(r);
    return false;
  }
  std::memcpy(out128, id.internal, NCCL_UNIQUE_ID_BYTES);
  return true;
}

class RcclComm final : public Comm {
 public:
  RcclComm(int rank, int world, ncclComm_t c) : comm_(c) {
    rank_ = rank;
    world_ = world;
  }
  ~RcclComm() override {
    if (comm_) rccl().CommDestroy(comm_);
  }
  void allreduce_sum(void* dev, size_t count, DType t, hipStream_t s) override {
    if (!count) return;
    check(rccl().AllReduce(dev, dev, count, nccl_type(t), ncclSum, comm_, s), "ncclAllReduce");
  }
  void allreduce_max_f64(double* dev, size_t count, hipStream_t s) override {
    if (!count) return;
    check(rccl().AllReduce(dev, dev, count, ncclFloat64, ncclMax, comm_, s), "ncclAllReduce(max)");
  }
  void allgather(const void* send, void* recv, size_t count, DType t, hipStream_t s) override {
    if (!count) return;
    check(rccl().AllGather(send, recv, count, nccl_type(t), comm_, s), "ncclAllGather");
  }
  void send(const void* dev, size_t count, DType t, int peer, hipStream_t s) override {
    if (!count) return;
    check(rccl().Send(dev, count, nccl_type(t), peer, comm_, s), "ncclSend");
  }
  void recv(void* dev, size_t count, DType t, int peer, hipStream_t s) override {
    if (!count) return;
    check(rccl().Recv(dev, count, nccl_type(t), peer, comm_, s), "ncclRecv");
  }
  void broadcast(void* dev, size_t count, DType t, int root, hipStream_t s) override {
    if (!count) return;
    check(rccl().Broadcast(dev, dev, count, nccl_type(t), root, comm_, s), "ncclBroadcast");
  }

 private:
  static void check(ncclResult_t r, const char* what) {
    if (r != ncclSuccess) throw std::runtime_error(std::string(what) + ": " + rccl().GetErrorString(r));
  }
  ncclComm_t comm_ = nullptr;
};

std::unique_ptr<Comm> make_rccl_comm(int rank, int world, const void* uid128, std::string* err) {
  if (!rccl().load(err)) return nullptr;
  ncclUniqueId id;
  std::memcpy(id.internal, uid128, NCCL_UNIQUE_ID_BYTES);
  ncclComm_t c = nullptr;
  ncclResult_t r = rccl().CommInitRank(&c, world, id, rank);
  if (r != ncclSuccess) {
    if (err) *err = std::string("ncclCommInitRank: ") + rccl().GetErrorString(r);
    return nullptr;
  }
  return std::make_unique<RcclComm>(rank, world, c);
}

// ---------------------------------------------------------------------------------------------
struct LoopbackGroup {
  explicit LoopbackGroup(int w) : world(w), slots(w), mail((size_t)w * w) {}
  int world;
  std::mutex mu;
  std::condition_variable cv;
  int arrived = 0;
  uint64_t gen = 0;
  std::vector<std::vector<uint8_t>> slots;
  std::vector<std::deque<std::vector<uint8_t>>> mail;  // [src * world + dst]: messages in order
  std::condition_variable mail_cv;
  void barrier() {
    std::unique_lock<std::mutex> lk(mu);
    const uint64_t g = gen;
    if (++arrived == world) {
      arrived = 0;
      ++gen;
      cv.notify_all();
    } else {
      cv.wait(lk, [&] { return gen != g; });
    }
  }
};

std::shared_ptr<LoopbackGroup> make_loopback_group(int world) {
  return std::make_shared<LoopbackGroup>(world);
}

class LoopbackComm final : public Comm {
 public:
  LoopbackComm(std::shared_ptr<LoopbackGroup> g, int rank) : g_(std::move(g)) {
    rank_ = rank;
    world_ = g_->world;
  }
  void allreduce_sum(void* dev, size_t count, DType t, hipStream_t s) override {
    exchange(dev, count * dtype_size(t), s);
    std::vector<uint8_t> out(count * dtype_size(t));
    for (size_t i = 0; i < count; ++i) {
      switch (t) {
        case DType::I32: { int32_t v = 0; for (auto& sl : g_->slots) v += reinterpret_cast<const int32_t*>(sl.data())[i]; reinterpret_cast<int32_t*>(out.data())[i] = v; break; }
        case DType::I64: { int64_t v = 0; for (auto& sl : g_->slots) v += reinterpret_cast<const int64_t*>(sl.data())[i]; reinterpret_cast<int64_t*>(out.data())[i] = v; break; }
        case DType::F64: { double v = 0; for (auto& sl : g_->slots) v += reinterpret_cast<const double*>(sl.data())[i]; reinterpret_cast<double*>(out.data())[i] = v; break; }
        case DType::U8: { uint8_t v = 0; for (auto& sl : g_->slots) v = (uint8_t)(v + sl[i]); out[i] = v; break; }
      }
    }
    g_->barrier();  // everyone has read the slots
    upload(dev, out.data(), out.size(), s);
  }
  void allreduce_max_f64(double* dev, size_t count, hipStream_t s) override {
    exchange(dev, count * 8, s);
    std::vector<double> out(count);
    for (size_t i = 0; i < count; ++i) {
      double v = reinterpret_cast<const double*>(g_->slots[0].data())[i];
      for (auto& sl : g_->slots) v = std::max(v, reinterpret_cast<const double*>(sl.data())[i]);
      out[i] = v;
    }
    g_->barrier();
    upload(dev, out.data(), count * 8, s);
  }
  void allgather(const void* send, void* recv, size_t count, DType t, hipStream_t s) override {
    const size_t bytes = count * dtype_size(t);
    exchange(send, bytes, s);
    std::vector<uint8_t> out(bytes * world_);
    for (int r = 0; r < world_; ++r)
      if (bytes) std::memcpy(out.data() + r * bytes, g_->slots[r].data(), bytes);
    g_->barrier();
    upload(recv, out.data(), out.size(), s);
  }
  void send(const void* dev, size_t count, DType t, int peer, hipStream_t s) override {
    std::vector<uint8_t> m(count * dtype_size(t));
    if (!m.empty()) {
      hip_check(hipMemcpyAsync(m.data(), dev, m.size(), hipMemcpyDeviceToHost, s), "loopback d2h");
      hip_check(hipStreamSynchronize(s), "loopback sync");
    }
    std::lock_guard<std::mutex> lk(g_->mu);
    g_->mail[(size_t)rank_ * world_ + peer].push_back(std::move(m));
    g_->mail_cv.notify_all();
  }
  void recv(void* dev, size_t count, DType t, int peer, hipStream_t s) override {
    std::vector<uint8_t> m;
    {
      std::unique_lock<std::mutex> lk(g_->mu);
      auto& q = g_->mail[(size_t)peer * world_ + rank_];
      g_->mail_cv.wait(lk, [&] { return !q.empty(); });
      m = std::move(q.front());
      q.pop_front();
    }
    if (m.size() != count * dtype_size(t)) throw std::runtime_error("loopback recv: size mismatch");
    upload(dev, m.data(), m.size(), s);
  }
  void broadcast(void* dev, size_t count, DType t, int root, hipStream_t s) override {
    const size_t bytes = count * dtype_size(t);
    exchange(dev, rank_ == root ? bytes : 0, s);
    std::vector<uint8_t> out(g_->slots[root]);
    g_->barrier();
    if (rank_ != root) upload(dev, out.data(), bytes, s);
  }

 private:
  void exchange(const void* dev, size_t bytes, hipStream_t s) {
    auto& sl = g_->slots[rank_];
    sl.resize(bytes);
    if (bytes) {
      hip_check(hipMemcpyAsync(sl.data(), dev, bytes, hipMemcpyDeviceToHost, s), "loopback d2h");
      hip_check(hipStreamSynchronize(s), "loopback sync");
    }
    g_->barrier();  // all slots written
  }
  void upload(void* dev, const void* host, size_t bytes, hipStream_t s) {
    if (!bytes) return;
    hip_check(hipMemcpyAsync(dev, host, bytes, hipMemcpyHostToDevice, s), "loopback h2d");
    hip_check(hipStreamSynchronize(s), "loopback sync");
  }
  std::shared_ptr<LoopbackGroup> g_;
};

std::unique_ptr<Comm> make_loopback_comm(std::shared_ptr<LoopbackGroup> g, int rank) {
  return std::make_unique<LoopbackComm>(std::move(g), rank);
}

}  // namespace dlg
