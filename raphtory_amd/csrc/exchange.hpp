// exchange.hpp — the collective layer of the vertex-partitioned mode.
//
// One partition per GPU.  Per superstep the partitions trade label records of their changed
// boundary vertices (ncclSend/ncclRecv, grouped) and agree on halting (the counts exchange
// carries each partition's vote: nobody changed = every shard voted to halt,
// AnalysisTask.scala:208-225); once per batch they route component counts to the label owners
// (send/recv) and merge the summary fields (ncclAllReduce).
//
// Two implementations behind one interface (the loopback group is single-device: its
// collectives read peers' buffers with device-local copies and kernels):
//   RcclExchange   — RCCL communicator, one rank per GPU (the production path)
//   LocalExchange  — partitions that live in one process (threads sharing one GPU):
//                    the same protocol with device-to-device copies; used to test the
//                    partitioned path on a single GPU.
//   ShmExchange    — one process per partition on one host, staged through POSIX shared
//                    memory (processes sharing a GPU; the multi-process protocol without RCCL).
#pragma once
#include <hip/hip_runtime.h>

#include <cstddef>
#include <cstdint>
#include <string>

namespace rgpu {

constexpr int kXchgIdBytes = 128;  // == NCCL_UNIQUE_ID_BYTES

class Exchange {
 public:
  virtual ~Exchange() {}
  virtual int rank() const = 0;
  virtual int size() const = 0;
  // d_recv[q*n + i] = peer q's d_send[rank*n + i]  (int64, n per peer)
  virtual void alltoall_i64(const int64_t* d_send, int64_t* d_recv, size_t n, hipStream_t s) = 0;
  // point-to-point round: to every peer q != rank send send_bytes[q] from send[q], receive
  // recv_bytes[q] into recv[q] (sizes agreed beforehand; zero = no message)
  virtual void sendrecv(void* const* send, const size_t* send_bytes, void* const* recv,
                        const size_t* recv_bytes, hipStream_t s) = 0;
  // in place over n uint64 words
  virtual void allreduce_u64(unsigned long long* d, size_t n, bool max, hipStream_t s) = 0;
  // A new, independent channel over the same ranks (collective: every rank calls it in the same
  // order with the same tag).  Each batch slot of a partitioned run owns one, so that the
  // collectives of batches in flight on different streams never share an ordering (RCCL:
  // ncclCommSplit; loopback: a group of its own).
  virtual Exchange* fork(int tag) = 0;
};

// id blob handed to every partition (rgpu_exchange_id / rgpu_exchange_init); returns "" or
// an error.  kind 0 = RCCL unique id, kind 1 = loopback group (one process), kind 2 = shared-memory
// group (processes on one host).
std::string make_exchange_id(int kind, uint8_t out[kXchgIdBytes]);
// end of a run: a loopback partition thread gives up the measurement lock (RGPU_LOOPBACK_ISOLATE)
void exchange_quiesce();
std::string open_exchange(const uint8_t id[kXchgIdBytes], int rank, int nranks, int device,
                          Exchange** out);

}  // namespace rgpu
