// exchange.cpp — RCCL and in-process implementations of rgpu::Exchange (exchange.hpp).
#include "exchange.hpp"

#include <rccl/rccl.h>

#include <atomic>
#include <cstdlib>
#include <chrono>
#include <condition_variable>
#include <cstring>
#include <map>
#include <memory>
#include <mutex>
#include <stdexcept>
#include <vector>


namespace rgpu {
namespace {

void hipchk(hipError_t e, const char* what) {
  if (e != hipSuccess) throw std::runtime_error(std::string(what) + ": " + hipGetErrorString(e));
}
void ncclchk(ncclResult_t e, const char* what) {
  if (e != ncclSuccess) throw std::runtime_error(std::string(what) + ": " + ncclGetErrorString(e));
}

const char kLoopMagic[8] = {'R', 'G', 'P', 'U', 'L', 'O', 'O', 'P'};

// ------------------------------------------------------------------ RCCL
class RcclExchange : public Exchange {
 public:
  RcclExchange(const uint8_t id[kXchgIdBytes], int rank, int nranks) : r_(rank), n_(nranks) {
    ncclUniqueId uid;
    std::memcpy(uid.internal, id, sizeof(uid.internal));
    ncclchk(ncclCommInitRank(&comm_, nranks, uid, rank), "ncclCommInitRank");
  }
  RcclExchange(ncclComm_t c, int rank, int nranks) : comm_(c), r_(rank), n_(nranks) {}
  Exchange* fork(int tag) override {
    ncclComm_t c = nullptr;
    ncclchk(ncclCommSplit(comm_, tag, r_, &c, nullptr), "ncclCommSplit");
    return new RcclExchange(c, r_, n_);
  }
  ~RcclExchange() override { (void)ncclCommDestroy(comm_); }
  int rank() const override { return r_; }
  int size() const override { return n_; }
  void alltoall_i64(const int64_t* d_send, int64_t* d_recv, size_t n, hipStream_t s) override {
    ncclchk(ncclGroupStart(), "ncclGroupStart");
    for (int q = 0; q < n_; q++) {
      ncclchk(ncclSend(d_send + q * n, n, ncclInt64, q, comm_, s), "ncclSend");
      ncclchk(ncclRecv(d_recv + q * n, n, ncclInt64, q, comm_, s), "ncclRecv");
    }
    ncclchk(ncclGroupEnd(), "ncclGroupEnd");
  }
  void sendrecv(void* const* send, const size_t* send_bytes, void* const* recv,
                const size_t* recv_bytes, hipStream_t s) override {
    ncclchk(ncclGroupStart(), "ncclGroupStart");
    for (int q = 0; q < n_; q++) {
      if (q == r_) continue;
      if (send_bytes[q]) ncclchk(ncclSend(send[q], send_bytes[q], ncclChar, q, comm_, s), "ncclSend");
      if (recv_bytes[q]) ncclchk(ncclRecv(recv[q], recv_bytes[q], ncclChar, q, comm_, s), "ncclRecv");
    }
    ncclchk(ncclGroupEnd(), "ncclGroupEnd");
  }
  void allreduce_u64(unsigned long long* d, size_t n, bool max, hipStream_t s) override {
    ncclchk(ncclAllReduce(d, d, n, ncclUint64, max ? ncclMax : ncclSum, comm_, s), "ncclAllReduce");
  }

 private:
  ncclComm_t comm_ = nullptr;
  int r_, n_;
};

// ------------------------------------------------------------------ loopback group
// Partitions of one process rendezvous here.  Every collective is: drain own stream,
// publish pointers, barrier, pull from the peers' buffers, drain, barrier (so no peer
// reuses a buffer that is still being read).
struct LocalGroup {
  explicit LocalGroup(int n) : n(n), ptr(n), vptr(n), vsz(n), host(n) {}
  int n;
  std::mutex mu;
  std::condition_variable cv;
  int arrived = 0;
  uint64_t gen = 0;
  std::vector<const void*> ptr;
  std::vector<std::vector<void*>> vptr;
  std::vector<std::vector<size_t>> vsz;
  std::vector<std::vector<unsigned long long>> host;
  void barrier() {
    std::unique_lock<std::mutex> lk(mu);
    const uint64_t g = gen;
    if (++arrived == n) {
      arrived = 0;
      gen++;
      cv.notify_all();
    } else {
      // a partition that never arrives (its thread failed) must not hang the others forever
      if (!cv.wait_for(lk, std::chrono::seconds(120), [&] { return gen != g; }))
        throw std::runtime_error("loopback exchange: a partition did not reach the barrier");
    }
  }
};

// RGPU_LOOPBACK_ISOLATE=1 (measurement only, tools/part_sim.py): a partition thread holds a
// process-wide lock from the end of one collective to the start of its next, so the partitions'
// GPU work between collectives runs one partition at a time and per-kernel event times are
// free of the other partitions' contention (their sum is the work P GPUs would share).
std::mutex g_iso;
thread_local bool t_iso_held = false;
bool iso_on() {
  static const bool on = [] {
    const char* e = std::getenv("RGPU_LOOPBACK_ISOLATE");
    return e && *e && std::atoi(e) != 0;
  }();
  return on;
}
void iso_enter() {  // at a collective's start, after this thread's stream has drained
  if (t_iso_held) {
    t_iso_held = false;
    g_iso.unlock();
  }
}
void iso_exit() {
  if (iso_on() && !t_iso_held) {
    g_iso.lock();
    t_iso_held = true;
  }
}

std::mutex g_reg_mu;
std::map<uint64_t, std::weak_ptr<LocalGroup>> g_reg;

std::shared_ptr<LocalGroup> local_group(uint64_t key, int nranks) {
  std::lock_guard<std::mutex> lk(g_reg_mu);
  std::shared_ptr<LocalGroup> g = g_reg[key].lock();
  if (!g) {
    g = std::make_shared<LocalGroup>(nranks);
    g_reg[key] = g;
  }
  return g;
}

class LocalExchange : public Exchange {
 public:
  LocalExchange(std::shared_ptr<LocalGroup> g, int rank, uint64_t key) : g_(std::move(g)), r_(rank), key_(key) {}
  Exchange* fork(int tag) override {
    const uint64_t k = key_ * 0x9E3779B97F4A7C15ull + (uint64_t)tag + 1;  // same on every rank
    std::shared_ptr<LocalGroup> g = local_group(k, g_->n);
    if (g->n != g_->n) throw std::runtime_error("loopback exchange: partition counts disagree");
    return new LocalExchange(g, r_, k);
  }
  int rank() const override { return r_; }
  int size() const override { return g_->n; }
  void alltoall_i64(const int64_t* d_send, int64_t* d_recv, size_t n, hipStream_t s) override {
    hipchk(hipStreamSynchronize(s), "sync");
    iso_enter();
    g_->ptr[r_] = d_send;
    g_->barrier();
    for (int q = 0; q < g_->n; q++)
      hipchk(hipMemcpyAsync(d_recv + q * n, (const int64_t*)g_->ptr[q] + r_ * n, n * sizeof(int64_t),
                            hipMemcpyDeviceToDevice, s), "copy");
    hipchk(hipStreamSynchronize(s), "sync");
    g_->barrier();
    iso_exit();
  }
  void sendrecv(void* const* send, const size_t* send_bytes, void* const* recv,
                const size_t* recv_bytes, hipStream_t s) override {
    const int n = g_->n;
    hipchk(hipStreamSynchronize(s), "sync");
    iso_enter();
    g_->vptr[r_].assign(send, send + n);
    g_->vsz[r_].assign(send_bytes, send_bytes + n);
    g_->barrier();
    for (int q = 0; q < n; q++) {
      if (q == r_) continue;
      if (g_->vsz[q][r_] != recv_bytes[q])
        throw std::runtime_error("loopback exchange: send/receive sizes disagree");
      if (recv_bytes[q])
        hipchk(hipMemcpyAsync(recv[q], g_->vptr[q][r_], recv_bytes[q], hipMemcpyDeviceToDevice, s), "copy");
    }
    hipchk(hipStreamSynchronize(s), "sync");
    g_->barrier();
    iso_exit();
  }
  void allreduce_u64(unsigned long long* d, size_t n, bool max, hipStream_t s) override {
    auto& mine = g_->host[r_];
    mine.resize(n);
    hipchk(hipMemcpyAsync(mine.data(), d, n * 8, hipMemcpyDeviceToHost, s), "copy");
    hipchk(hipStreamSynchronize(s), "sync");
    iso_enter();
    g_->barrier();
    std::vector<unsigned long long> acc(g_->host[0]);
    for (int q = 1; q < g_->n; q++)
      for (size_t i = 0; i < n; i++) {
        const unsigned long long x = g_->host[q][i];
        acc[i] = max ? (x > acc[i] ? x : acc[i]) : acc[i] + x;
      }
    g_->barrier();
    hipchk(hipMemcpyAsync(d, acc.data(), n * 8, hipMemcpyHostToDevice, s), "copy");
    hipchk(hipStreamSynchronize(s), "sync");
    iso_exit();
  }

 private:
  std::shared_ptr<LocalGroup> g_;
  int r_;
  uint64_t key_;
};

}  // namespace

void exchange_quiesce() { iso_enter(); }

std::string make_exchange_id(int kind, uint8_t out[kXchgIdBytes]) {
  std::memset(out, 0, kXchgIdBytes);
  if (kind == 0) {
    ncclUniqueId uid;
    const ncclResult_t e = ncclGetUniqueId(&uid);
    if (e != ncclSuccess) return std::string("ncclGetUniqueId: ") + ncclGetErrorString(e);
    std::memcpy(out, uid.internal, kXchgIdBytes);
    return "";
  }
  if (kind == 1) {
    static std::atomic<uint64_t> counter{1};
    const uint64_t key = (uint64_t)std::chrono::steady_clock::now().time_since_epoch().count() ^
                         (counter.fetch_add(1) << 48);
    std::memcpy(out, kLoopMagic, 8);
    std::memcpy(out + 8, &key, 8);
    return "";
  }
  return "unknown exchange kind";
}

std::string open_exchange(const uint8_t id[kXchgIdBytes], int rank, int nranks, int device,
                          Exchange** out) {
  *out = nullptr;
  try {
    hipchk(hipSetDevice(device), "hipSetDevice");
    if (std::memcmp(id, kLoopMagic, 8) == 0) {
      uint64_t key;
      std::memcpy(&key, id + 8, 8);
      std::shared_ptr<LocalGroup> g = local_group(key, nranks);
      if (g->n != nranks) return "loopback exchange: partition counts disagree";
      *out = new LocalExchange(g, rank, key);
    } else {
      *out = new RcclExchange(id, rank, nranks);
    }
  } catch (const std::exception& e) {
    return e.what();
  }
  return "";
}

}  // namespace rgpu
