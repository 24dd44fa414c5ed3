// rgev.cpp — binary GraphUpdate log: the Router-side packer and the
// partition-side decoder, so that a router streams updates straight into rgpu_ingest instead
// of sending one Tracked*GraphUpdate actor message per update
// (S/core/components/Router/RouterWorker.scala:88-116; update case classes
// S/core/model/communication/raphtoryMessages.scala:38-55).
//
// Block layout (little-endian; include/rgpu.h has the normative description):
//   0  u32 magic 'RGEV'     4  u16 version (1)   6  u16 flags (0)
//   8  u32 n (1..RGPU_RGEV_MAX_BLOCK)             12 u32 checksum of the payload
//   16 i64 t_base = min time of the block
//   24 payload: u32 dt[n] (t - t_base) | u8 kind[n], zero-padded to 4 | i32 src[n] | i32 dst[n]
// Updates keep stream order inside a block and blocks keep it across a log: ties between
// equal timestamps resolve by that order in the reference (last put wins), so nothing here
// reorders.  Vertex updates carry dst = -1.  Property payloads (*WithProperties) are not on
// the analysis path and are not encoded; their adds are plain adds.
// Host-only code: no HIP, no device state.
#include <cstdint>
#include <cstring>
#include <string>

#include "../../include/rgpu.h"

namespace {

constexpr uint32_t kMagic = 0x56454752u;  // "RGEV"
constexpr uint16_t kVersion = 1;
constexpr size_t kHeader = 24;

inline size_t pad4(size_t n) { return (n + 3) & ~(size_t)3; }
inline size_t block_bytes(size_t n) { return kHeader + 4 * n + pad4(n) + 8 * n; }

template <class T>
inline void put(uint8_t* p, T v) { std::memcpy(p, &v, sizeof(T)); }
template <class T>
inline T get(const uint8_t* p) {
  T v;
  std::memcpy(&v, p, sizeof(T));
  return v;
}

// Fletcher-64 over the payload's u32 words (the payload is a multiple of 4 bytes).
uint32_t checksum(const uint8_t* p, size_t bytes) {
  uint64_t a = 0, b = 0;
  for (size_t i = 0; i + 4 <= bytes; i += 4) {
    a += get<uint32_t>(p + i);
    b += a;
  }
  return (uint32_t)(a ^ (a >> 32) ^ b ^ (b >> 32));
}

const char* check_update(int64_t t, uint8_t kind, int64_t src, int64_t dst) {
  if (kind > RGPU_EDEL) return "unknown update kind";
  if (t < 0 || t >= ((int64_t)1 << 61)) return "time out of range [0, 2^61)";
  if (src < 0 || src > INT32_MAX) return "vertex id out of range [0, 2^31)";
  if (kind >= RGPU_EADD && (dst < 0 || dst > INT32_MAX)) return "vertex id out of range [0, 2^31)";
  return nullptr;
}

thread_local std::string g_err;

int fail(const char* what) {
  g_err = what;
  return RGPU_EINVAL;
}

}  // namespace

extern "C" {

const char* rgpu_rgev_last_error(void) { return g_err.c_str(); }

int rgpu_rgev_encode(const int64_t* t, const uint8_t* kind, const int64_t* src, const int64_t* dst, size_t n,
                     size_t block, uint8_t* out, size_t cap, size_t* written) {
  if (!written || (n && (!t || !kind || !src))) return fail("null argument");
  if (block == 0 || block > RGPU_RGEV_MAX_BLOCK) block = RGPU_RGEV_MAX_BLOCK;
  // pass 1: validate and size (a block also ends where its time span would pass 2^32 - 1)
  size_t need = 0;
  for (size_t i = 0; i < n;) {
    int64_t lo = t[i], hi = t[i];
    size_t j = i;
    for (; j < n && j - i < block; j++) {
      if (const char* e = check_update(t[j], kind[j], src[j], kind[j] >= RGPU_EADD ? (dst ? dst[j] : -1) : 0))
        return fail(e);
      const int64_t l2 = t[j] < lo ? t[j] : lo, h2 = t[j] > hi ? t[j] : hi;
      if (h2 - l2 > (int64_t)UINT32_MAX) break;
      lo = l2;
      hi = h2;
    }
    need += block_bytes(j - i);
    i = j;
  }
  *written = need;
  if (!out) return RGPU_OK;  // size query
  if (cap < need) return fail("output buffer too small (see *written)");
  // pass 2: write
  uint8_t* p = out;
  for (size_t i = 0; i < n;) {
    int64_t lo = t[i], hi = t[i];
    size_t j = i;
    for (; j < n && j - i < block; j++) {
      const int64_t l2 = t[j] < lo ? t[j] : lo, h2 = t[j] > hi ? t[j] : hi;
      if (h2 - l2 > (int64_t)UINT32_MAX) break;
      lo = l2;
      hi = h2;
    }
    const size_t m = j - i;
    uint8_t* dtp = p + kHeader;
    uint8_t* kp = dtp + 4 * m;
    uint8_t* sp = kp + pad4(m);
    uint8_t* dp = sp + 4 * m;
    for (size_t k = 0; k < m; k++) {
      put<uint32_t>(dtp + 4 * k, (uint32_t)(t[i + k] - lo));
      kp[k] = kind[i + k];
      put<int32_t>(sp + 4 * k, (int32_t)src[i + k]);
      put<int32_t>(dp + 4 * k, kind[i + k] >= RGPU_EADD ? (int32_t)dst[i + k] : -1);
    }
    for (size_t k = m; k < pad4(m); k++) kp[k] = 0;
    put<uint32_t>(p + 0, kMagic);
    put<uint16_t>(p + 4, kVersion);
    put<uint16_t>(p + 6, 0);
    put<uint32_t>(p + 8, (uint32_t)m);
    put<uint32_t>(p + 12, checksum(p + kHeader, block_bytes(m) - kHeader));
    put<int64_t>(p + 16, lo);
    p += block_bytes(m);
    i = j;
  }
  return RGPU_OK;
}

int rgpu_rgev_decode(const uint8_t* buf, size_t bytes, int64_t* t, uint8_t* kind, int64_t* src, int64_t* dst,
                     size_t cap, size_t* n, size_t* consumed) {
  if (!n || !consumed || (bytes && !buf)) return fail("null argument");
  // pass 1: walk and verify the whole blocks the buffer holds (a partial tail stays unread)
  size_t off = 0, total = 0;
  while (bytes - off >= kHeader) {
    const uint8_t* p = buf + off;
    if (get<uint32_t>(p) != kMagic) return fail("bad block magic");
    if (get<uint16_t>(p + 4) != kVersion) return fail("unsupported block version");
    if (get<uint16_t>(p + 6) != 0) return fail("unsupported block flags");
    const size_t m = get<uint32_t>(p + 8);
    if (m == 0 || m > RGPU_RGEV_MAX_BLOCK) return fail("bad block update count");
    if (bytes - off < block_bytes(m)) break;
    if (checksum(p + kHeader, block_bytes(m) - kHeader) != get<uint32_t>(p + 12)) return fail("block checksum mismatch");
    const int64_t base = get<int64_t>(p + 16);
    // untrusted: range-check the base before any addition (base + dt stays below 2^61 + 2^32)
    if (base < 0 || base >= ((int64_t)1 << 61)) return fail("block time base out of range");
    const uint8_t* kp = p + kHeader + 4 * m;
    const uint8_t* sp = kp + pad4(m);
    const uint8_t* dp = sp + 4 * m;
    for (size_t k = 0; k < m; k++) {
      const int64_t tt = (int64_t)((uint64_t)base + get<uint32_t>(p + kHeader + 4 * k));
      const int64_t d = get<int32_t>(dp + 4 * k);
      if (const char* e = check_update(tt, kp[k], get<int32_t>(sp + 4 * k), kp[k] >= RGPU_EADD ? d : 0)) return fail(e);
      if (kp[k] < RGPU_EADD && d != -1) return fail("vertex update with a dst");
    }
    total += m;
    off += block_bytes(m);
  }
  *n = total;
  *consumed = off;
  if (!t) return RGPU_OK;  // size query
  if (cap < total || !kind || !src || !dst) return fail("output arrays too small (see *n)");
  // pass 2: expand
  size_t o = 0;
  for (size_t q = 0; q < off;) {
    const uint8_t* p = buf + q;
    const size_t m = get<uint32_t>(p + 8);
    const int64_t base = get<int64_t>(p + 16);
    const uint8_t* kp = p + kHeader + 4 * m;
    const uint8_t* sp = kp + pad4(m);
    const uint8_t* dp = sp + 4 * m;
    for (size_t k = 0; k < m; k++, o++) {
      t[o] = base + get<uint32_t>(p + kHeader + 4 * k);
      kind[o] = kp[k];
      src[o] = get<int32_t>(sp + 4 * k);
      dst[o] = get<int32_t>(dp + 4 * k);
    }
    q += block_bytes(m);
  }
  return RGPU_OK;
}

}  // extern "C"
