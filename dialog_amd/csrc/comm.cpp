// comm.cpp -- Single / RCCL / in-process loopback communicators (see comm.hpp).
#include "comm.hpp"

#include <dlfcn.h>
#include <fcntl.h>
#include <rccl/rccl.h>
#include <sys/mman.h>
#include <unistd.h>

#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstring>
#include <deque>
#include <stdexcept>
#include <thread>

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

void Comm::sync_stream(hipStream_t s) {
  if (!device_waits()) {
    hip_check(hipStreamSynchronize(s), "stream sync");
    return;
  }
  // a collective on the stream waits for the peers on the device: poll, so that a failed peer
  // (the group's poison) or a timeout ends the wait instead of blocking in the runtime forever
  const auto t0 = std::chrono::steady_clock::now();
  for (uint32_t k = 0;; ++k) {
    const hipError_t e = hipStreamQuery(s);
    if (e == hipSuccess) return;
    if (e != hipErrorNotReady) hip_check(e, "stream query");
    check();
    if ((k & 63u) == 63u) {
      const auto ms = std::chrono::duration_cast<std::chrono::milliseconds>(
                          std::chrono::steady_clock::now() - t0).count();
      if (timeout_ms > 0 && ms > timeout_ms) {
        abort("rank " + std::to_string(rank_) + ": no progress for " + std::to_string(ms) +
              " ms (DLG_OPT_COMM_TIMEOUT_MS)");
        check();
      }
    }
    if (k < 2048) {
#if defined(__x86_64__)
      __builtin_ia32_pause();
#endif
    } else {
      std::this_thread::sleep_for(std::chrono::microseconds(20));
    }
  }
}

// ---------------------------------------------------------------------------------------------
class SingleComm final : public Comm {
 protected:
  void do_allreduce_sum(void*, size_t, DType, hipStream_t) override {}
  void do_allreduce_max_f64(double*, size_t, hipStream_t) override {}
  void do_allgather(const void* send, void* recv, size_t count, DType t, hipStream_t s) override {
    if (send != recv && count)
      hip_check(hipMemcpyAsync(recv, send, count * dtype_size(t), hipMemcpyDeviceToDevice, s),
                "allgather copy");
  }
  void do_send(const void*, size_t, DType, int, hipStream_t) override {
    throw std::runtime_error("send on a single-rank communicator");
  }
  void do_recv(void*, size_t, DType, int, hipStream_t) override {
    throw std::runtime_error("recv on a single-rank communicator");
  }
  void do_broadcast(void*, size_t, DType, int, hipStream_t) override {}
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
  ncclResult_t (*CommAbort)(ncclComm_t) = nullptr;
  ncclResult_t (*CommGetAsyncError)(ncclComm_t, ncclResult_t*) = nullptr;
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
    DLG_SYM(CommAbort, "ncclCommAbort");
    DLG_SYM(CommGetAsyncError, "ncclCommGetAsyncError");
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

// The group's poison word for RCCL ranks on one node: a shared-memory page named after the
// communicator's unique id (random per job), mapped by every rank before ncclCommInitRank (so no
// rank can unlink it before every peer has it mapped).  A rank that fails CASes `state` 0 -> 2,
// writes its rank and error, then releases 1; the peers' polls see it within one poll interval.
// (Ranks on other nodes never see the page: they end by the collective timeout.)
struct PoisonPage {
  std::atomic<int32_t> state;  // 0 healthy, 2 being written, 1 aborted
  int32_t rank;
  char why[240];
};
static_assert(sizeof(PoisonPage) <= 4096, "one page");

class NodePoison {
 public:
  explicit NodePoison(const void* uid128) {
    uint64_t h = 1469598103934665603ull;  // FNV-1a over the 128-byte id
    const auto* b = static_cast<const unsigned char*>(uid128);
    for (int i = 0; i < NCCL_UNIQUE_ID_BYTES; ++i) h = (h ^ b[i]) * 1099511628211ull;
    char nm[40];
    std::snprintf(nm, sizeof(nm), "/dlg_poison_%016llx", (unsigned long long)h);
    name_ = nm;
    const int fd = shm_open(nm, O_CREAT | O_RDWR, 0600);
    if (fd < 0) return;  // (no /dev/shm: the timeout remains)
    if (ftruncate(fd, 4096) == 0) {
      void* p = mmap(nullptr, 4096, PROT_READ | PROT_WRITE, MAP_SHARED, fd, 0);
      if (p != MAP_FAILED) page_ = static_cast<PoisonPage*>(p);
    }
    close(fd);
  }
  ~NodePoison() {
    if (page_) munmap(page_, 4096);
    shm_unlink(name_.c_str());  // (the first rank to get here removes the name; the others ENOENT)
  }
  bool set(int rank, const std::string& why) {
    if (!page_) return false;
    int32_t z = 0;
    if (!page_->state.compare_exchange_strong(z, 2)) return false;  // someone failed first
    page_->rank = rank;
    std::snprintf(page_->why, sizeof(page_->why), "%s", why.c_str());
    page_->state.store(1, std::memory_order_release);
    return true;
  }
  // the first failure's reason, or empty while the group is healthy
  std::string get() const {
    if (!page_) return {};
    int32_t st = page_->state.load(std::memory_order_acquire);
    if (st == 0) return {};
    for (int k = 0; st == 2 && k < 100000; ++k) st = page_->state.load(std::memory_order_acquire);
    if (st == 2) return "a peer rank failed";
    return std::string(page_->why, strnlen(page_->why, sizeof(page_->why)));
  }

 private:
  std::string name_;
  PoisonPage* page_ = nullptr;
};

class RcclComm final : public Comm {
 public:
  RcclComm(int rank, int world, ncclComm_t c, std::unique_ptr<NodePoison> p)
      : comm_(c), poison_(std::move(p)) {
    rank_ = rank;
    world_ = world;
  }
  ~RcclComm() override {
    if (comm_) rccl().CommDestroy(comm_);
  }
  bool device_waits() const override { return true; }
  void abort(const std::string& why) override {
    if (aborted_) return;
    aborted_ = true;
    why_ = why;
    if (poison_) poison_->set(rank_, why);
    // (ends this rank's in-flight collectives: the device-side waits poll the abort flag)
    if (comm_) rccl().CommAbort(comm_);
    comm_ = nullptr;
  }
  void check() override {
    if (!aborted_) {
      std::string w = poison_ ? poison_->get() : std::string();
      if (w.empty() && comm_) {
        ncclResult_t ae = ncclSuccess;
        if (rccl().CommGetAsyncError(comm_, &ae) == ncclSuccess && ae != ncclSuccess &&
            ae != ncclInProgress)
          w = "rank " + std::to_string(rank_) + ": RCCL asynchronous error: " +
              rccl().GetErrorString(ae);
      }
      if (!w.empty()) {
        aborted_ = true;
        why_ = w;
        if (comm_) rccl().CommAbort(comm_);
        comm_ = nullptr;
      }
    }
    if (aborted_) throw CommAborted("communicator aborted: " + why_);
  }

 protected:
  void do_allreduce_sum(void* dev, size_t count, DType t, hipStream_t s) override {
    if (!count) return;
    ok(rccl().AllReduce(dev, dev, count, nccl_type(t), ncclSum, comm_, s), "ncclAllReduce");
  }
  void do_allreduce_max_f64(double* dev, size_t count, hipStream_t s) override {
    if (!count) return;
    ok(rccl().AllReduce(dev, dev, count, ncclFloat64, ncclMax, comm_, s), "ncclAllReduce(max)");
  }
  void do_allgather(const void* send, void* recv, size_t count, DType t, hipStream_t s) override {
    if (!count) return;
    ok(rccl().AllGather(send, recv, count, nccl_type(t), comm_, s), "ncclAllGather");
  }
  void do_send(const void* dev, size_t count, DType t, int peer, hipStream_t s) override {
    if (!count) return;
    ok(rccl().Send(dev, count, nccl_type(t), peer, comm_, s), "ncclSend");
  }
  void do_recv(void* dev, size_t count, DType t, int peer, hipStream_t s) override {
    if (!count) return;
    ok(rccl().Recv(dev, count, nccl_type(t), peer, comm_, s), "ncclRecv");
  }
  void do_broadcast(void* dev, size_t count, DType t, int root, hipStream_t s) override {
    if (!count) return;
    ok(rccl().Broadcast(dev, dev, count, nccl_type(t), root, comm_, s), "ncclBroadcast");
  }

 private:
  void ok(ncclResult_t r, const char* what) {
    if (r != ncclSuccess) {
      const std::string m = std::string(what) + ": " + rccl().GetErrorString(r);
      abort("rank " + std::to_string(rank_) + ": " + m);
      throw CommAborted(m);
    }
  }
  ncclComm_t comm_ = nullptr;
  std::unique_ptr<NodePoison> poison_;
  bool aborted_ = false;
  std::string why_;
};

std::unique_ptr<Comm> make_rccl_comm(int rank, int world, const void* uid128, std::string* err) {
  if (!rccl().load(err)) return nullptr;
  ncclUniqueId id;
  std::memcpy(id.internal, uid128, NCCL_UNIQUE_ID_BYTES);
  auto poison = std::make_unique<NodePoison>(uid128);  // (mapped before any rank can finish init)
  ncclComm_t c = nullptr;
  ncclResult_t r = rccl().CommInitRank(&c, world, id, rank);
  if (r != ncclSuccess) {
    if (err) *err = std::string("ncclCommInitRank: ") + rccl().GetErrorString(r);
    return nullptr;
  }
  return std::make_unique<RcclComm>(rank, world, c, std::move(poison));
}

// ---------------------------------------------------------------------------------------------
struct LoopbackGroup {
  explicit LoopbackGroup(int w) : world(w), slots(w), mail((size_t)w * w) {}
  int world;
  std::mutex mu;
  std::condition_variable cv;
  int arrived = 0;
  uint64_t gen = 0;
  bool aborted = false;  // poisoned by a failed rank: every wait of every rank throws
  std::string why;
  std::vector<std::vector<uint8_t>> slots;
  std::vector<std::deque<std::vector<uint8_t>>> mail;  // [src * world + dst]: messages in order
  std::condition_variable mail_cv;
  [[noreturn]] void thrown() { throw CommAborted("communicator aborted: " + why); }
  void barrier() {
    std::unique_lock<std::mutex> lk(mu);
    if (aborted) thrown();
    const uint64_t g = gen;
    if (++arrived == world) {
      arrived = 0;
      ++gen;
      cv.notify_all();
    } else {
      cv.wait(lk, [&] { return gen != g || aborted; });
      if (aborted) thrown();
    }
  }
  void abort(const std::string& w) {
    std::lock_guard<std::mutex> lk(mu);
    if (aborted) return;
    aborted = true;
    why = w;
    cv.notify_all();
    mail_cv.notify_all();
  }
  void check() {
    std::lock_guard<std::mutex> lk(mu);
    if (aborted) thrown();
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
  void abort(const std::string& why) override { g_->abort(why); }
  void check() override { g_->check(); }

 protected:
  void do_allreduce_sum(void* dev, size_t count, DType t, hipStream_t s) override {
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
  void do_allreduce_max_f64(double* dev, size_t count, hipStream_t s) override {
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
  void do_allgather(const void* send, void* recv, size_t count, DType t, hipStream_t s) override {
    const size_t bytes = count * dtype_size(t);
    exchange(send, bytes, s);
    std::vector<uint8_t> out(bytes * world_);
    for (int r = 0; r < world_; ++r)
      if (bytes) std::memcpy(out.data() + r * bytes, g_->slots[r].data(), bytes);
    g_->barrier();
    upload(recv, out.data(), out.size(), s);
  }
  void do_send(const void* dev, size_t count, DType t, int peer, hipStream_t s) override {
    std::vector<uint8_t> m(count * dtype_size(t));
    if (!m.empty()) {
      hip_check(hipMemcpyAsync(m.data(), dev, m.size(), hipMemcpyDeviceToHost, s), "loopback d2h");
      hip_check(hipStreamSynchronize(s), "loopback sync");
    }
    std::lock_guard<std::mutex> lk(g_->mu);
    if (g_->aborted) g_->thrown();
    g_->mail[(size_t)rank_ * world_ + peer].push_back(std::move(m));
    g_->mail_cv.notify_all();
  }
  void do_recv(void* dev, size_t count, DType t, int peer, hipStream_t s) override {
    std::vector<uint8_t> m;
    {
      std::unique_lock<std::mutex> lk(g_->mu);
      auto& q = g_->mail[(size_t)peer * world_ + rank_];
      g_->mail_cv.wait(lk, [&] { return !q.empty() || g_->aborted; });
      if (g_->aborted) g_->thrown();
      m = std::move(q.front());
      q.pop_front();
    }
    if (m.size() != count * dtype_size(t)) throw std::runtime_error("loopback recv: size mismatch");
    upload(dev, m.data(), m.size(), s);
  }
  void do_broadcast(void* dev, size_t count, DType t, int root, hipStream_t s) override {
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
