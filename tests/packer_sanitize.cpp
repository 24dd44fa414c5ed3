// TEST INFRASTRUCTURE: a standalone driver of the product's host packer (raphtory_amd/csrc/
// packer.cpp) for sanitizer builds (-fsanitize=address / thread on the packer).
// The packer runs with several std::threads (parallel radix sorts, per-thread histograms,
// per-chunk counts), so the same streams are packed under ASan+UBSan and under TSan.
//   packer_sanitize <stream.bin>      stream.bin = int64 n, then SoA t[n] kind[n] src[n] dst[n]
// Packs: one partition; every partition of P = 3 (fed what rgpu_ingest keeps); a live-ingest
// delta (pack_delta + finish_delta) at the stream's middle.  Exit 0 = clean.
#include <algorithm>
#include <cstdio>
#include <cstdint>
#include <vector>

#include "rgpu_internal.hpp"

using rgpu::Event;
using rgpu::Packed;

int main(int argc, char** argv) {
  if (argc < 2) return 2;
  FILE* f = std::fopen(argv[1], "rb");
  if (!f) return 2;
  int64_t n = 0;
  if (std::fread(&n, 8, 1, f) != 1 || n < 0) return 2;
  std::vector<int64_t> t(n), src(n), dst(n);
  std::vector<uint8_t> kind(n);
  if (std::fread(t.data(), 8, n, f) != (size_t)n || std::fread(kind.data(), 1, n, f) != (size_t)n ||
      std::fread(src.data(), 8, n, f) != (size_t)n || std::fread(dst.data(), 8, n, f) != (size_t)n)
    return 2;
  std::fclose(f);
  std::vector<Event> ev(n);
  for (int64_t i = 0; i < n; i++) ev[i] = {t[i], src[i], kind[i] >= 2 ? dst[i] : -1, kind[i]};
  Packed one;
  if (!rgpu::pack_events(ev, 0, 1, &one).empty()) return 3;
  const int P = 3;
  int64_t owned = 0;
  for (int p = 0; p < P; p++) {
    std::vector<Event> mine;
    for (const Event& e : ev)
      if (rgpu::partition_keeps(e.kind, e.src, e.dst, p, P)) mine.push_back(e);
    Packed part;
    if (!rgpu::pack_events(mine, p, P, &part).empty()) return 4;
    owned += part.n_own;
  }
  if (owned != one.nv) return 5;
  const size_t cut = (size_t)n / 2;
  std::vector<Event> head(ev.begin(), ev.begin() + cut);
  Packed base;
  if (!rgpu::pack_events(head, 0, 1, &base).empty()) return 6;
  rgpu::Delta d;
  if (!rgpu::pack_delta(ev, cut, base, &d).empty()) return 7;
  std::vector<int32_t> base_eid(d.de_s.size(), -1);
  for (size_t i = 0; i < d.de_s.size(); i++) {
    const int32_t qs = d.de_qs[i], qd = d.de_qd[i];
    if (qs < 0 || qd < 0) continue;
    auto lo = base.edst.begin() + base.out_off[qs], hi = base.edst.begin() + base.out_off[qs + 1];
    auto it = std::lower_bound(lo, hi, qd);
    if (it != hi && *it == qd) base_eid[i] = (int32_t)(it - base.edst.begin());
  }
  rgpu::finish_delta(base, base_eid, &d);
  if (d.nv != one.nv) return 8;
  std::printf("ok %lld updates, %lld vertices, %lld edges\n", (long long)n, (long long)one.nv, (long long)one.ne);
  return 0;
}
