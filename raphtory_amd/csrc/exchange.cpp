// exchange.cpp — RCCL and in-process implementations of rgpu::Exchange (exchange.hpp).
#include "exchange.hpp"

#include <fcntl.h>
#include <rccl/rccl.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>

#include <atomic>
#include <cstdlib>
#include <chrono>
#include <condition_variable>
#include <cstring>
#include <map>
#include <memory>
#include <mutex>
#include <stdexcept>
#include <thread>
#include <vector>


namespace rgpu {
namespace {

void hipchk(hipError_t e, const char* what) {
  if (e != hipSuccess) throw std::runtime_error(std::string(what) + ": " + hipGetErrorString(e));
}
void ncclchk(ncclResult_t e, const char* what) {
  if (e != ncclSuccess) throw std::runtime_error(std::string(what) + ": " + ncclGetErrorString(e));
}

// The HIP runtime stages a copy through the CPU when a pointer it is handed lies in no live device
// allocation (a freed buffer, or a range running past an allocation's end), and a bad one then
// faults inside the runtime's host memcpy: a SIGSEGV with no word about which buffer (the round-4
// P = 8 rehearsal crash in LocalExchange::sendrecv).  The loopback and shared-memory
// collectives check every device range they copy from or into first, and throw naming it.
void check_dev_range(const void* p, size_t bytes, const char* what, int rank, int peer) {
  if (!bytes) return;
  hipDeviceptr_t base = nullptr;
  size_t size = 0;
  const hipError_t e = hipMemGetAddressRange(&base, &size, (hipDeviceptr_t)p);
  const uintptr_t a = (uintptr_t)p, b = (uintptr_t)base;
  if (e != hipSuccess || a < b || a - b + bytes > size)
    throw std::runtime_error(std::string("exchange: rank ") + std::to_string(rank) + " " + what + " (peer " +
                             std::to_string(peer) + "): " + std::to_string(bytes) + " bytes at " +
                             std::to_string(a) + " are not inside one live device allocation" +
                             (e == hipSuccess ? " (allocation of " + std::to_string(size) + " bytes at offset " +
                                                    std::to_string((long long)(a - b)) + ")"
                                              : std::string(" (no allocation)")));
}

const char kLoopMagic[8] = {'R', 'G', 'P', 'U', 'L', 'O', 'O', 'P'};
// (version 2: ShmCtl gained `broken` in front of size[]; a process of another layout cannot attach)
const char kShmMagic[8] = {'R', 'G', 'P', 'U', 'S', 'H', 'M', '2'};

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
    if (check_sizes()) agree_sizes(send_bytes, recv_bytes, s);
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
  // RGPU_CHECK: before every point-to-point round, the ranks trade the sizes they are about to
  // send and each compares them with the sizes it will receive.  A mismatch on the wire would
  // otherwise hang the grouped send/recv (or truncate it) with no diagnostic.
  static bool check_sizes() {
    static const bool on = [] {
      const char* e = std::getenv("RGPU_CHECK");
      return e && *e && std::atoi(e) != 0;
    }();
    return on;
  }
  void agree_sizes(const size_t* send_bytes, const size_t* recv_bytes, hipStream_t s) {
    std::vector<int64_t> h(2 * n_);
    for (int q = 0; q < n_; q++) h[q] = q == r_ ? 0 : (int64_t)send_bytes[q];
    int64_t* d = nullptr;
    hipchk(hipMalloc(&d, sizeof(int64_t) * 2 * n_), "hipMalloc");
    try {
      hipchk(hipMemcpyAsync(d, h.data(), sizeof(int64_t) * n_, hipMemcpyHostToDevice, s), "copy");
      alltoall_i64(d, d + n_, 1, s);
      hipchk(hipMemcpyAsync(h.data(), d, sizeof(int64_t) * 2 * n_, hipMemcpyDeviceToHost, s), "copy");
      hipchk(hipStreamSynchronize(s), "sync");
    } catch (...) {
      (void)hipFree(d);
      throw;
    }
    (void)hipFree(d);
    for (int q = 0; q < n_; q++)
      if (q != r_ && h[n_ + q] != (int64_t)recv_bytes[q])
        throw std::runtime_error("RCCL exchange: rank " + std::to_string(q) + " sends " + std::to_string(h[n_ + q]) +
                                 " bytes, rank " + std::to_string(r_) + " expects " + std::to_string(recv_bytes[q]));
  }
  ncclComm_t comm_ = nullptr;
  int r_, n_;
};

// ------------------------------------------------------------------ loopback group
// Partitions of one process rendezvous here.  Every collective is: drain own stream,
// publish pointers, barrier, pull from the peers' buffers, drain, barrier (so no peer
// reuses a buffer that is still being read).
// A partition that does not arrive within the barrier timeout (RGPU_XCHG_TIMEOUT seconds; default
// 120 for loopback partitions, which are threads of one process that start their runs together,
// and 600 for processes over shared memory, whose first collective can wait for a peer's seal of
// minutes) breaks the group: the waiting partitions throw, and every later collective on the group
// throws too (an arrival counted before the timeout would otherwise release a later barrier early
// and pair collectives that do not belong together).
int barrier_timeout_s(int dflt) {
  static const int t = [] {
    const char* e = std::getenv("RGPU_XCHG_TIMEOUT");
    return e && *e ? std::atoi(e) : 0;
  }();
  return t > 0 ? t : dflt;
}

struct LocalGroup {
  explicit LocalGroup(int n) : n(n), ptr(n), vptr(n), vsz(n), host(n) {}
  int n;
  std::mutex mu;
  std::condition_variable cv;
  int arrived = 0;
  uint64_t gen = 0;
  bool broken = false;
  std::vector<const void*> ptr;
  std::vector<std::vector<void*>> vptr;
  std::vector<std::vector<size_t>> vsz;
  std::vector<std::vector<unsigned long long>> host;
  void barrier() {
    std::unique_lock<std::mutex> lk(mu);
    if (broken) throw std::runtime_error("loopback exchange: channel broken by an earlier barrier timeout");
    const uint64_t g = gen;
    if (++arrived == n) {
      arrived = 0;
      gen++;
      cv.notify_all();
    } else {
      // a partition that never arrives (its thread failed) must not hang the others forever
      if (!cv.wait_for(lk, std::chrono::seconds(barrier_timeout_s(120)), [&] { return gen != g || broken; }) ||
          broken) {
        broken = true;
        cv.notify_all();
        throw std::runtime_error("loopback exchange: a partition did not reach the barrier");
      }
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
    for (int q = 0; q < n; q++)
      if (q != r_) {
        check_dev_range(send[q], send_bytes[q], "send region", r_, q);
        check_dev_range(recv[q], recv_bytes[q], "receive region", r_, q);
      }
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

// ------------------------------------------------------------------ processes over shared memory
// One process per partition on one host (e.g. several partitions sharing one GPU, or a host
// without a working RCCL transport): every collective is staged through POSIX shared memory.
// Per channel a control segment (a process-shared barrier and every rank's data size) and one
// data segment per rank, which only its owner writes.  A collective: drain the stream, copy the
// device data into our segment (with a table of (offset, size) per peer), barrier, copy the
// peers' parts addressed to us into device memory, barrier (no segment is rewritten while a
// peer still reads it).  The segment names are unlinked as soon as every rank holds them open,
// so nothing stays in /dev/shm once the processes end.  The receiver checks every size against
// the one the sender wrote (the RCCL path's RGPU_CHECK does the same with a size exchange).
constexpr int kShmMaxRanks = 64;
struct ShmCtl {
  std::atomic<uint64_t> arrived;
  std::atomic<uint64_t> gen;
  std::atomic<uint64_t> broken;              // a barrier timed out: the channel is unusable (barrier())
  std::atomic<uint64_t> size[kShmMaxRanks];  // bytes of each rank's data segment
};
static_assert(std::atomic<uint64_t>::is_always_lock_free, "process-shared atomics");

class ShmExchange : public Exchange {
 public:
  ShmExchange(uint64_t key, int rank, int nranks) : key_(key), r_(rank), n_(nranks), fd_(nranks, -1),
                                                   map_(nranks, nullptr), mapped_(nranks, 0) {
    if (nranks > kShmMaxRanks) throw std::runtime_error("shm exchange: too many ranks");
    const std::string cn = name(-1);
    int cfd = shm_open(cn.c_str(), O_RDWR | O_CREAT, 0600);
    if (cfd < 0) throw std::runtime_error("shm exchange: shm_open " + cn);
    if (ftruncate(cfd, sizeof(ShmCtl)) != 0) { close(cfd); throw std::runtime_error("shm exchange: ftruncate"); }
    ctl_ = (ShmCtl*)mmap(nullptr, sizeof(ShmCtl), PROT_READ | PROT_WRITE, MAP_SHARED, cfd, 0);
    close(cfd);
    if (ctl_ == MAP_FAILED) throw std::runtime_error("shm exchange: mmap control");
    const std::string dn = name(r_);
    fd_[r_] = shm_open(dn.c_str(), O_RDWR | O_CREAT | O_TRUNC, 0600);
    if (fd_[r_] < 0) throw std::runtime_error("shm exchange: shm_open " + dn);
    barrier();  // every rank has the control segment and its own data segment
    for (int q = 0; q < n_; q++)
      if (q != r_) {
        fd_[q] = shm_open(name(q).c_str(), O_RDONLY, 0);
        if (fd_[q] < 0) throw std::runtime_error("shm exchange: shm_open " + name(q));
      }
    barrier();  // every rank holds every segment open: the names can go
    shm_unlink(dn.c_str());
    if (r_ == 0) shm_unlink(cn.c_str());
  }
  ~ShmExchange() override {
    for (int q = 0; q < n_; q++) {
      if (map_[q]) munmap(map_[q], mapped_[q]);
      if (fd_[q] >= 0) close(fd_[q]);
    }
    if (ctl_ && ctl_ != MAP_FAILED) munmap(ctl_, sizeof(ShmCtl));
  }
  Exchange* fork(int tag) override {
    return new ShmExchange(key_ * 0x9E3779B97F4A7C15ull + (uint64_t)tag + 1, r_, n_);
  }
  int rank() const override { return r_; }
  int size() const override { return n_; }
  void alltoall_i64(const int64_t* d_send, int64_t* d_recv, size_t n, hipStream_t s) override {
    std::vector<void*> sp(n_), rp(n_);
    std::vector<size_t> sb(n_), rb(n_);
    for (int q = 0; q < n_; q++) {
      sp[q] = (void*)(d_send + q * n);
      rp[q] = d_recv + q * n;
      sb[q] = rb[q] = q == r_ ? 0 : n * sizeof(int64_t);
    }
    hipchk(hipMemcpyAsync(d_recv + r_ * n, d_send + r_ * n, n * sizeof(int64_t), hipMemcpyDeviceToDevice, s), "copy");
    sendrecv(sp.data(), sb.data(), rp.data(), rb.data(), s);
  }
  void sendrecv(void* const* send, const size_t* send_bytes, void* const* recv, const size_t* recv_bytes,
                hipStream_t s) override {
    hipchk(hipStreamSynchronize(s), "sync");
    // our segment: [n_ x (offset, size)] then the payloads
    size_t tot = sizeof(uint64_t) * 2 * n_;
    for (int q = 0; q < n_; q++) tot += q == r_ ? 0 : send_bytes[q];
    uint8_t* mine = own(tot);
    uint64_t* tab = (uint64_t*)mine;
    size_t off = sizeof(uint64_t) * 2 * n_;
    for (int q = 0; q < n_; q++)
      if (q != r_) {
        check_dev_range(send[q], send_bytes[q], "send region", r_, q);
        check_dev_range(recv[q], recv_bytes[q], "receive region", r_, q);
      }
    for (int q = 0; q < n_; q++) {
      const size_t b = q == r_ ? 0 : send_bytes[q];
      tab[2 * q] = off;
      tab[2 * q + 1] = b;
      if (b) hipchk(hipMemcpy(mine + off, send[q], b, hipMemcpyDeviceToHost), "copy out");
      off += b;
    }
    barrier();
    for (int q = 0; q < n_; q++) {
      if (q == r_) continue;
      const uint8_t* peer = view(q);
      const uint64_t* pt = (const uint64_t*)peer;
      if (pt[2 * r_ + 1] != recv_bytes[q])
        throw std::runtime_error("shm exchange: rank " + std::to_string(q) + " sends " + std::to_string(pt[2 * r_ + 1]) +
                                 " bytes, rank " + std::to_string(r_) + " expects " + std::to_string(recv_bytes[q]));
      if (recv_bytes[q]) hipchk(hipMemcpy(recv[q], peer + pt[2 * r_], recv_bytes[q], hipMemcpyHostToDevice), "copy in");
    }
    barrier();
  }
  void allreduce_u64(unsigned long long* d, size_t n, bool max, hipStream_t s) override {
    hipchk(hipStreamSynchronize(s), "sync");
    uint8_t* mine = own(n * 8);
    hipchk(hipMemcpy(mine, d, n * 8, hipMemcpyDeviceToHost), "copy out");
    barrier();
    std::vector<unsigned long long> acc(n);
    std::memcpy(acc.data(), mine, n * 8);
    for (int q = 0; q < n_; q++) {
      if (q == r_) continue;
      const unsigned long long* x = (const unsigned long long*)view(q);
      for (size_t i = 0; i < n; i++) acc[i] = max ? (x[i] > acc[i] ? x[i] : acc[i]) : acc[i] + x[i];
    }
    barrier();
    hipchk(hipMemcpy(d, acc.data(), n * 8, hipMemcpyHostToDevice), "copy in");
  }

 private:
  std::string name(int r) const {
    char b[96];
    std::snprintf(b, sizeof(b), "/rgpu_%016llx_%s%d", (unsigned long long)key_, r < 0 ? "ctl" : "r", r < 0 ? 0 : r);
    return b;
  }
  // Timeout: RGPU_XCHG_TIMEOUT, default 600 s (barrier_timeout_s).  A timed-out barrier marks the channel broken
  // in the shared control segment, so every rank's later collective on it throws instead of being
  // released early by the arrival counted before the timeout.
  void barrier() {
    if (ctl_->broken.load()) throw std::runtime_error("shm exchange: channel broken by an earlier barrier timeout");
    const uint64_t g = ctl_->gen.load();
    if (ctl_->arrived.fetch_add(1) + 1 == (uint64_t)n_) {
      ctl_->arrived.store(0);
      ctl_->gen.fetch_add(1);
      return;
    }
    const auto t0 = std::chrono::steady_clock::now();
    while (ctl_->gen.load() == g) {
      std::this_thread::yield();
      if (ctl_->broken.load()) throw std::runtime_error("shm exchange: channel broken by a peer's barrier timeout");
      if (std::chrono::steady_clock::now() - t0 > std::chrono::seconds(barrier_timeout_s(600))) {
        ctl_->broken.store(1);
        throw std::runtime_error("shm exchange: a partition did not reach the barrier");
      }
    }
  }
  uint8_t* own(size_t bytes) {  // our data segment, at least `bytes` long
    if (bytes > mapped_[r_]) {
      const size_t want = std::max(bytes, mapped_[r_] * 2);
      if (map_[r_]) munmap(map_[r_], mapped_[r_]);
      map_[r_] = nullptr;
      // posix_fallocate reserves the tmpfs pages now: on a small /dev/shm an ftruncate alone would
      // succeed and the first store past the free space would raise SIGBUS instead of an error
      if (ftruncate(fd_[r_], (off_t)want) != 0) throw std::runtime_error("shm exchange: ftruncate");
      if (const int e = posix_fallocate(fd_[r_], 0, (off_t)want))
        throw std::runtime_error(std::string("shm exchange: no room for a ") + std::to_string(want) +
                                 "-byte segment in /dev/shm: " + std::strerror(e));
      void* p = mmap(nullptr, want, PROT_READ | PROT_WRITE, MAP_SHARED, fd_[r_], 0);
      if (p == MAP_FAILED) throw std::runtime_error("shm exchange: mmap");
      map_[r_] = p;
      mapped_[r_] = want;
      ctl_->size[r_].store(want);
    }
    return (uint8_t*)map_[r_];
  }
  const uint8_t* view(int q) {  // peer q's data segment, as large as it has grown
    const size_t sz = ctl_->size[q].load();
    if (sz > mapped_[q]) {
      if (map_[q]) munmap(map_[q], mapped_[q]);
      map_[q] = nullptr;
      void* p = mmap(nullptr, sz, PROT_READ, MAP_SHARED, fd_[q], 0);
      if (p == MAP_FAILED) throw std::runtime_error("shm exchange: mmap peer");
      map_[q] = p;
      mapped_[q] = sz;
    }
    return (const uint8_t*)map_[q];
  }
  uint64_t key_;
  int r_, n_;
  ShmCtl* ctl_ = nullptr;
  std::vector<int> fd_;
  std::vector<void*> map_;
  std::vector<size_t> mapped_;
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
  if (kind == 1 || kind == 2) {
    static std::atomic<uint64_t> counter{1};
    const uint64_t key = (uint64_t)std::chrono::steady_clock::now().time_since_epoch().count() ^
                         (counter.fetch_add(1) << 48) ^ ((uint64_t)getpid() << 20);
    std::memcpy(out, kind == 1 ? kLoopMagic : kShmMagic, 8);
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
    } else if (std::memcmp(id, kShmMagic, 8) == 0) {
      uint64_t key;
      std::memcpy(&key, id + 8, 8);
      *out = new ShmExchange(key, rank, nranks);
    } else {
      *out = new RcclExchange(id, rank, nranks);
    }
  } catch (const std::exception& e) {
    return e.what();
  }
  return "";
}

}  // namespace rgpu
