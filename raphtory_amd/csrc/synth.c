/*
 * synth.c — seeded synthetic update streams.
 *
 * Stands in for the reference spouts that cannot travel here:
 *   gen_uniform  — RandomSpout shape (uniform ids, examples/random/actors/RandomSpout.scala:46-52,
 *                  95-96) with the paper's 30/40/10/20 VADD/EADD/VDEL/EDEL mix (config C1/C2).
 *   gen_powerlaw — Chung-Lu power-law endpoints, 8/85/5/2 mix over two years (config C3).
 *   gen_gab      — GAB-like add-only interactions: (VADD s, VADD d, EADD s->d) at one t, as
 *                  GabUserGraphRouter.parseTuple emits them (examples/gab/actors/
 *                  GabUserGraphRouter.scala:31-33) (config C4).
 * Output is SoA: t int64 ms, kind uint8 (0 VADD, 1 VDEL, 2 EADD, 3 EDEL), src, dst int64.
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

static uint64_t sm64(uint64_t* s) {
  uint64_t z = (*s += 0x9e3779b97f4a7c15ULL);
  z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ULL;
  z = (z ^ (z >> 27)) * 0x94d049bb133111ebULL;
  return z ^ (z >> 31);
}
static double u01(uint64_t* s) { return (double)(sm64(s) >> 11) * (1.0 / 9007199254740992.0); }
static int64_t below(uint64_t* s, int64_t n) { return (int64_t)((unsigned __int128)sm64(s) * (uint64_t)n >> 64); }

/* bijection on [0, 2^31): scatters power-law ranks over the id space (and so over
 * partitions, Utils.getPartition) without collisions */
static int64_t perm31(int64_t i, uint64_t key) {
  const uint32_t M = 0x7fffffffu;
  uint32_t x = (uint32_t)i & M;
  for (int r = 0; r < 3; r++) {
    x = (x * 0x5bd1e995u + (uint32_t)(key >> (r * 16))) & M;
    x ^= x >> 13;
    x = (x * 0x2545f491u) & M;
    x ^= x >> 11;
  }
  return (int64_t)x;
}

/* Chung-Lu rank with weight ~ (r+1)^-a, a = 1/(gamma-1): inverse CDF of the continuous law */
typedef struct { double a1, top; int64_t n; } PL;
static PL pl_make(int64_t n, double gamma) {
  PL p;
  double a = 1.0 / (gamma - 1.0);
  p.a1 = 1.0 - a;
  p.top = pow((double)n + 1.0, p.a1) - 1.0;
  p.n = n;
  return p;
}
static int64_t pl_draw(const PL* p, uint64_t* s) {
  double x = pow(1.0 + u01(s) * p->top, 1.0 / p->a1);
  int64_t r = (int64_t)x - 1;
  if (r < 0) r = 0;
  if (r >= p->n) r = p->n - 1;
  return r;
}

/* C1/C2: n events, t_i = t0 + dt*i (strictly increasing), ids uniform in [0, nverts). */
size_t rg_gen_uniform(uint64_t seed, int64_t nverts, size_t n, int64_t t0, int64_t dt,
                      double p_vadd, double p_eadd, double p_vdel,
                      int64_t* t, uint8_t* kind, int64_t* src, int64_t* dst) {
  uint64_t s = seed;
  for (size_t i = 0; i < n; i++) {
    double r = u01(&s);
    uint8_t k = r < p_vadd ? 0 : r < p_vadd + p_eadd ? 2 : r < p_vadd + p_eadd + p_vdel ? 1 : 3;
    t[i] = t0 + dt * (int64_t)i;
    kind[i] = k;
    src[i] = below(&s, nverts);
    dst[i] = (k >= 2) ? below(&s, nverts) : -1;
  }
  return n;
}

/* C3: Chung-Lu power-law endpoints over nverts ranks permuted into [0,2^31); mix
 * 8% VADD / 85% EADD / 5% EDEL of a previously added pair (reservoir) / 2% VDEL
 * (id weighted by activity); t strictly increasing over [t0, t1). */
size_t rg_gen_powerlaw(uint64_t seed, int64_t nverts, size_t n, double gamma, int64_t t0,
                       int64_t t1, int64_t* t, uint8_t* kind, int64_t* src, int64_t* dst) {
  uint64_t s = seed;
  PL p = pl_make(nverts, gamma);
  const size_t R = 1u << 20;
  int64_t* rs = (int64_t*)malloc(sizeof(int64_t) * R);
  int64_t* rd = (int64_t*)malloc(sizeof(int64_t) * R);
  if (!rs || !rd) { free(rs); free(rd); return 0; }
  size_t seen = 0;
  int64_t span = t1 - t0;
  if ((uint64_t)span < n) span = (int64_t)n;
  for (size_t i = 0; i < n; i++) {
    double r = u01(&s);
    t[i] = t0 + (int64_t)((unsigned __int128)i * (uint64_t)span / n);
    if (r < 0.08) {
      kind[i] = 0; src[i] = perm31(pl_draw(&p, &s), seed); dst[i] = -1;
    } else if (r < 0.93 || seen == 0) {
      int64_t a = perm31(pl_draw(&p, &s), seed), b = perm31(pl_draw(&p, &s), seed);
      kind[i] = 2; src[i] = a; dst[i] = b;
      if (seen < R) { rs[seen] = a; rd[seen] = b; }
      else { uint64_t j = (uint64_t)below(&s, (int64_t)seen + 1); if (j < R) { rs[j] = a; rd[j] = b; } }
      seen++;
    } else if (r < 0.98) {
      size_t j = (size_t)below(&s, (int64_t)(seen < R ? seen : R));
      kind[i] = 3; src[i] = rs[j]; dst[i] = rd[j];
    } else {
      kind[i] = 1; src[i] = perm31(pl_draw(&p, &s), seed); dst[i] = -1;
    }
  }
  free(rs); free(rd);
  return n;
}

/* C4: `inter` GAB-like interactions -> 3*inter add-only events.  Power-law activity on both
 * ends; timestamps at 1 s granularity x1000 over [t0, t1) with a monotone diurnal warp
 * g(f) = f + A sin(2 pi D f)/(2 pi D), A = 0.6, D = days in span. */
/* id_key: the user-id scattering key (the same key = the same users, e.g. later ticks of a
 * live stream drawn with another seed) */
size_t rg_gen_gab_keyed(uint64_t seed, uint64_t id_key, int64_t users, size_t inter, int64_t t0, int64_t t1,
                        int64_t* t, uint8_t* kind, int64_t* src, int64_t* dst);
size_t rg_gen_gab(uint64_t seed, int64_t users, size_t inter, int64_t t0, int64_t t1,
                  int64_t* t, uint8_t* kind, int64_t* src, int64_t* dst) {
  return rg_gen_gab_keyed(seed, seed, users, inter, t0, t1, t, kind, src, dst);
}
size_t rg_gen_gab_range(uint64_t seed, uint64_t id_key, int64_t users, size_t inter, size_t first, size_t count,
                        int part, int nparts, int64_t t0, int64_t t1, int64_t* t, uint8_t* kind, int64_t* src,
                        int64_t* dst);
size_t rg_gen_gab_keyed(uint64_t seed, uint64_t id_key, int64_t users, size_t inter, int64_t t0, int64_t t1,
                        int64_t* t, uint8_t* kind, int64_t* src, int64_t* dst) {
  return rg_gen_gab_range(seed, id_key, users, inter, 0, inter, 0, 1, t0, t1, t, kind, src, dst);
}

/* Utils.getPartition (Utils.scala:32-33): (|id| mod 10P) div 10 */
static int owner_of(int64_t id, int nparts) { return (int)(((id < 0 ? -id : id) % (10 * (int64_t)nparts)) / 10); }

/* Interactions [first, first + count) of the `inter`-interaction stream above (the generator
 * draws two numbers per interaction from a counter-based splitmix64, so any range starts at
 * state seed + 2*first*golden): a prefix is a slice of the full stream, and ranges can be drawn
 * in chunks.  nparts > 1 keeps what partition `part` ingests (rgpu.h, partitioned mode): the
 * VertexAdd of an owned vertex, and every EdgeAdd with an owned endpoint.  Returns the number
 * of updates written (<= 3*count). */
size_t rg_gen_gab_range(uint64_t seed, uint64_t id_key, int64_t users, size_t inter, size_t first, size_t count,
                        int part, int nparts, int64_t t0, int64_t t1, int64_t* t, uint8_t* kind, int64_t* src,
                        int64_t* dst) {
  uint64_t s = seed + (uint64_t)(2 * first) * 0x9e3779b97f4a7c15ULL;
  PL p = pl_make(users, 2.1);
  double span_s = (double)((t1 - t0) / 1000);
  double days = span_s / 86400.0;
  const double A = 0.6, twopi = 6.283185307179586;
  size_t o = 0;
  for (size_t i = first; i < first + count && i < inter; i++) {
    double f = (double)i / (double)inter;
    double g = f + A * sin(twopi * days * f) / (twopi * days);
    int64_t ts = t0 + (int64_t)floor(g * span_s) * 1000;
    int64_t a = perm31(pl_draw(&p, &s), id_key), b = perm31(pl_draw(&p, &s), id_key);
    const int oa = nparts > 1 ? owner_of(a, nparts) == part : 1;
    const int ob = nparts > 1 ? owner_of(b, nparts) == part : 1;
    if (oa) { t[o] = ts; kind[o] = 0; src[o] = a; dst[o] = -1; o++; }
    if (ob) { t[o] = ts; kind[o] = 0; src[o] = b; dst[o] = -1; o++; }
    if (oa || ob) { t[o] = ts; kind[o] = 2; src[o] = a; dst[o] = b; o++; }
  }
  return o;
}
