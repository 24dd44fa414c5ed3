// xregions.hpp — host-side region arithmetic of the per-superstep label-record exchange
// (rgpu.cpp part_after_counts): how many U / M records go to and come from each peer, where each
// peer's records sit in the send and receive buffers, and that every one of those ranges lies
// inside its buffer.  Pure integer arithmetic (no HIP), so that the CPU suite checks it directly
// (tests/test_xregions.py via tests/xregions_harness.cpp).
//
// Buffers (records; rgpu.cpp XSlot):
//   su  U records to send, peer q's region at q * su_cap          (allocated su_cap * P)
//   sm  M records to send, peer q's region at q * smcap           (allocated smcap * P)
//   ru  U records received, peer q's region at sum(nbq[<q])        (allocated ru_alloc >= sum nbq)
//   rm  M records received, peer q's region at sum(rmcap[<q])      (allocated rm_alloc >= sum rmcap)
// Counts words (xchg.hip k_xbc_counts, exchanged all-to-all): xa[4q] / xa[4q+1] = U / M records
// this partition sends to q, xa[4q+2] its vote; xb the same words as q sent them to us.
#pragma once
#include <cstdint>
#include <string>

namespace rgpu {

constexpr int kXferMaxParts = 8;

struct XferPlan {
  int P = 0, me = 0;
  int64_t sent_u[kXferMaxParts] = {}, sent_m[kXferMaxParts] = {};
  int64_t recv_u[kXferMaxParts] = {}, recv_m[kXferMaxParts] = {};
  int64_t max_m = 0;          // the largest M list to one peer (the send regions must hold it)
  bool any = false;           // some partition changed a label (the vote, self included)
  // record offsets of peer q's regions (xfer_layout)
  int64_t su_off[kXferMaxParts] = {}, sm_off[kXferMaxParts] = {};
  int64_t ru_off[kXferMaxParts] = {}, rm_off[kXferMaxParts] = {};
};

// Phase 1, from the exchanged counts words: the record counts per peer and the vote.  A peer that
// announces more U records than it has boundary vertices names records outside the plan.
inline std::string xfer_counts(int P, int me, const int64_t* xa, const int64_t* xb, const int64_t* nbq,
                               XferPlan* out) {
  if (P < 1 || P > kXferMaxParts || me < 0 || me >= P) return "exchange: bad partition count or rank";
  XferPlan& X = *out;
  X = XferPlan();
  X.P = P;
  X.me = me;
  for (int q = 0; q < P; q++) {
    if (q != me) {
      X.sent_u[q] = xa[4 * q];
      X.sent_m[q] = xa[4 * q + 1];
      X.recv_u[q] = xb[4 * q];
      X.recv_m[q] = xb[4 * q + 1];
      if (X.sent_u[q] < 0 || X.sent_m[q] < 0 || X.recv_u[q] < 0 || X.recv_m[q] < 0)
        return "exchange: negative record count for peer " + std::to_string(q);
      if (X.max_m < X.sent_m[q]) X.max_m = X.sent_m[q];
      if (X.recv_u[q] > nbq[q])
        return "exchange: peer " + std::to_string(q) + " announced " + std::to_string(X.recv_u[q]) +
               " U records for " + std::to_string(nbq[q]) + " boundary vertices";
    }
    X.any |= xb[4 * q + 2] != 0;
  }
  return "";
}

// Phase 2, after the send and receive regions have grown to the counts: every peer's region
// offsets, and the check that each transfer [offset, offset + count) lies inside its own region
// and its region inside its buffer.  A failure names the buffer and the peer (the run fails
// instead of handing the exchange a range outside a live allocation).
inline std::string xfer_layout(XferPlan* plan, const int64_t* nbq, int64_t su_cap, int64_t smcap,
                               const int64_t* rmcap, int64_t su_alloc, int64_t sm_alloc, int64_t ru_alloc,
                               int64_t rm_alloc) {
  XferPlan& X = *plan;
  const int P = X.P;
  int64_t ru = 0, rm = 0;
  for (int q = 0; q < P; q++) {
    X.su_off[q] = (int64_t)q * su_cap;
    X.sm_off[q] = (int64_t)q * smcap;
    X.ru_off[q] = ru;
    X.rm_off[q] = rm;
    ru += nbq[q];
    rm += rmcap[q];
  }
  auto bad = [&](const char* what, int q, int64_t cnt, int64_t cap) {
    return std::string("exchange: ") + what + " for peer " + std::to_string(q) + ": " + std::to_string(cnt) +
           " records, region of " + std::to_string(cap);
  };
  for (int q = 0; q < P; q++) {
    if (q == X.me) continue;
    if (X.sent_u[q] > su_cap) return bad("U send", q, X.sent_u[q], su_cap);
    if (X.sent_m[q] > smcap) return bad("M send", q, X.sent_m[q], smcap);
    if (X.recv_u[q] > nbq[q]) return bad("U receive", q, X.recv_u[q], nbq[q]);
    if (X.recv_m[q] > rmcap[q]) return bad("M receive", q, X.recv_m[q], rmcap[q]);
  }
  if ((int64_t)P * su_cap > su_alloc) return "exchange: U send regions exceed their buffer";
  if ((int64_t)P * smcap > sm_alloc) return "exchange: M send regions exceed their buffer";
  if (ru > ru_alloc) return "exchange: U receive regions exceed their buffer";
  if (rm > rm_alloc) return "exchange: M receive regions exceed their buffer";
  return "";
}

}  // namespace rgpu
