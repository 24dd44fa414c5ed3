// Host-side profile of the live-ingest delta packer (packer.cpp pack_delta / finish_delta) on the
// C5 shape: a GAB base of B interactions (x3 updates), then one tick of T interactions one hour
// past the base's newest point (same users), as bench.py --config c5 streams them.  The base
// lookup the device does (k_edge_find) is a binary search here.  RGPU_HOSTPROF=1 prints phases.
//   g++ -O3 -std=c++17 -pthread -I raphtory_amd/csrc tools/delta_prof.cpp raphtory_amd/csrc/packer.cpp \
//       -x c raphtory_amd/csrc/synth.c -o /tmp/delta_prof && RGPU_HOSTPROF=1 /tmp/delta_prof 20000000 33333334 3333334
#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "rgpu_internal.hpp"

extern "C" size_t rg_gen_gab_keyed(uint64_t seed, uint64_t id_key, int64_t users, size_t inter, int64_t t0, int64_t t1,
                                   int64_t* t, uint8_t* kind, int64_t* src, int64_t* dst);

using clk = std::chrono::steady_clock;
static double ms(clk::time_point a) { return std::chrono::duration<double, std::milli>(clk::now() - a).count(); }

int main(int argc, char** argv) {
  const int64_t users = argc > 1 ? std::atoll(argv[1]) : 20000000;
  const size_t base = argc > 2 ? std::atoll(argv[2]) : 33333334, tick = argc > 3 ? std::atoll(argv[3]) : 3333334;
  const int64_t T0 = 1470787200000LL, T1 = 1527724800000LL, HOUR = 3600000;
  std::vector<int64_t> t(3 * base), s(3 * base), d(3 * base);
  std::vector<uint8_t> k(3 * base);
  rg_gen_gab_keyed(4, 4, users, base, T0, T1, t.data(), k.data(), s.data(), d.data());
  std::vector<rgpu::Event> ev(3 * base);
  for (size_t i = 0; i < ev.size(); i++) ev[i] = {t[i], s[i], k[i] >= 2 ? d[i] : -1, k[i]};
  const int64_t now = t.back();
  std::vector<int64_t> tt(3 * tick), ts(3 * tick), td(3 * tick);
  std::vector<uint8_t> tk(3 * tick);
  rg_gen_gab_keyed(100, 4, users, tick, now + 1, now + HOUR, tt.data(), tk.data(), ts.data(), td.data());
  auto a = clk::now();
  rgpu::Packed B;
  if (!rgpu::pack_events(ev, 0, 1, &B).empty()) return 3;
  std::printf("base pack %.0f ms: %lld vertices, %lld edges\n", ms(a), (long long)B.nv, (long long)B.ne);
  const size_t first = ev.size();
  for (size_t i = 0; i < tt.size(); i++) ev.push_back({tt[i], ts[i], tk[i] >= 2 ? td[i] : -1, tk[i]});
  for (int rep = 0; rep < 3; rep++) {
    a = clk::now();
    rgpu::Delta D;
    if (!rgpu::pack_delta(ev, first, B, &D).empty()) return 4;
    const double t_pack = ms(a);
    a = clk::now();
    std::vector<int32_t> base_eid(D.de_s.size(), -1);
    for (size_t i = 0; i < D.de_s.size(); i++) {
      const int32_t qs = D.de_qs[i], qd = D.de_qd[i];
      if (qs < 0 || qd < 0) continue;
      auto lo = B.edst.begin() + B.out_off[qs], hi = B.edst.begin() + B.out_off[qs + 1];
      auto it = std::lower_bound(lo, hi, qd);
      if (it != hi && *it == qd) base_eid[i] = (int32_t)(it - B.edst.begin());
    }
    const double t_find = ms(a);
    a = clk::now();
    rgpu::finish_delta(B, base_eid, &D);
    std::printf("tick of %zu updates: pack_delta %.0f ms, (lookup %.0f ms), finish_delta %.0f ms\n", tt.size(), t_pack,
                t_find, ms(a));
  }
  return 0;
}
