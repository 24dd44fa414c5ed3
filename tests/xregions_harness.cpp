// TEST INFRASTRUCTURE: C entry points around the product's exchange region arithmetic
// (raphtory_amd/csrc/xregions.hpp, compiled here with g++), for tests/test_xregions.py.
#include <cstring>

#include "xregions.hpp"

static char g_err[512];

// counts words -> plan; then the layout over the given region sizes.  out[0..4P): per peer sent_u,
// sent_m, recv_u, recv_m; out[4P..8P): su_off, sm_off, ru_off, rm_off; out[8P] max_m, out[8P+1] any.
// Returns 0 when both phases pass, 1 when phase 1 fails, 2 when phase 2 fails (xr_error says why).
extern "C" int xr_plan(int P, int me, const int64_t* xa, const int64_t* xb, const int64_t* nbq, int64_t su_cap,
                       int64_t smcap, const int64_t* rmcap, int64_t su_alloc, int64_t sm_alloc, int64_t ru_alloc,
                       int64_t rm_alloc, int64_t* out) {
  rgpu::XferPlan X;
  std::string e = rgpu::xfer_counts(P, me, xa, xb, nbq, &X);
  g_err[0] = 0;
  if (!e.empty()) {
    std::strncpy(g_err, e.c_str(), sizeof(g_err) - 1);
    return 1;
  }
  e = rgpu::xfer_layout(&X, nbq, su_cap, smcap, rmcap, su_alloc, sm_alloc, ru_alloc, rm_alloc);
  for (int q = 0; q < P; q++) {
    out[4 * q] = X.sent_u[q];
    out[4 * q + 1] = X.sent_m[q];
    out[4 * q + 2] = X.recv_u[q];
    out[4 * q + 3] = X.recv_m[q];
    out[4 * P + 4 * q] = X.su_off[q];
    out[4 * P + 4 * q + 1] = X.sm_off[q];
    out[4 * P + 4 * q + 2] = X.ru_off[q];
    out[4 * P + 4 * q + 3] = X.rm_off[q];
  }
  out[8 * P] = X.max_m;
  out[8 * P + 1] = X.any ? 1 : 0;
  if (!e.empty()) {
    std::strncpy(g_err, e.c_str(), sizeof(g_err) - 1);
    return 2;
  }
  return 0;
}

extern "C" const char* xr_error(void) { return g_err; }
