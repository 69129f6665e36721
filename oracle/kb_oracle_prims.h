/*
 * kb_oracle_prims.h — oracle-side primitives (TEST INFRASTRUCTURE ONLY; never linked by the product).
 *
 * Independent CPU implementations of the three arithmetic building blocks the round semantics rest on:
 *   - Philox4x32-10 (Salmon et al., SC'11; Random123) — the declared replacement for the reference's
 *     entropy-seeded ChaChaRng (src/kaboodle.rs:164).  Pinned by the Random123 known-answer vectors in
 *     tests/golden/philox_kat.json.
 *   - CRC-32/ISO-HDLC as implemented by crc32fast 1.3.2 (Cargo.lock:111-112; used at
 *     src/kaboodle.rs:75-82): reflected poly 0xEDB88320, init/xorout 0xFFFFFFFF.  Pinned by zlib
 *     (tests/golden/fingerprints.json).
 *   - GF(2) polynomial arithmetic modulo the CRC polynomial (zlib's multmodp) used to fold per-peer
 *     segment CRCs into the sorted-concatenation CRC without re-reading the address strings.
 */
#ifndef KB_ORACLE_PRIMS_H
#define KB_ORACLE_PRIMS_H
#include <stdint.h>
#include <stddef.h>

/* ---------------- Philox4x32-10 ---------------- */
typedef struct { uint32_t v[4]; } o_u32x4;

static inline o_u32x4 o_philox(uint32_t c0, uint32_t c1, uint32_t c2, uint32_t c3, uint32_t k0, uint32_t k1) {
  uint32_t c[4] = {c0, c1, c2, c3};
  for (int r = 0; r < 10; ++r) {
    if (r) { k0 += 0x9E3779B9u; k1 += 0xBB67AE85u; }
    uint64_t p0 = (uint64_t)0xD2511F53u * c[0];
    uint64_t p1 = (uint64_t)0xCD9E8D57u * c[2];
    uint32_t n0 = (uint32_t)(p1 >> 32) ^ c[1] ^ k0;
    uint32_t n1 = (uint32_t)p1;
    uint32_t n2 = (uint32_t)(p0 >> 32) ^ c[3] ^ k1;
    uint32_t n3 = (uint32_t)p0;
    c[0] = n0; c[1] = n1; c[2] = n2; c[3] = n3;
  }
  o_u32x4 o = {{c[0], c[1], c[2], c[3]}};
  return o;
}

/* uniform integer in [0, k): high word of u * k (declared in DESIGN.md §2.6) */
static inline uint32_t o_mulhi(uint32_t u, uint32_t k) { return (uint32_t)(((uint64_t)u * k) >> 32); }

/* ---------------- CRC-32 ---------------- */
#define O_CRC_POLY 0xEDB88320u
static uint32_t o_crc_table[256];
static int o_crc_ready = 0;
static inline void o_crc_init(void) {
  if (o_crc_ready) return;
  for (uint32_t i = 0; i < 256; ++i) {
    uint32_t c = i;
    for (int k = 0; k < 8; ++k) c = (c & 1) ? (c >> 1) ^ O_CRC_POLY : c >> 1;
    o_crc_table[i] = c;
  }
  o_crc_ready = 1;
}
/* raw register update, no init/xorout */
static inline uint32_t o_crc_update(uint32_t reg, const uint8_t* p, size_t n) {
  for (size_t i = 0; i < n; ++i) reg = o_crc_table[(reg ^ p[i]) & 0xFFu] ^ (reg >> 8);
  return reg;
}
/* standard CRC-32 of a byte string (crc32fast::hash / zlib.crc32) */
static inline uint32_t o_crc32(const uint8_t* p, size_t n) { return o_crc_update(0xFFFFFFFFu, p, n) ^ 0xFFFFFFFFu; }

/* a*b mod P in the reflected representation (x^0 = 0x80000000) — zlib multmodp */
static inline uint32_t o_multmodp(uint32_t a, uint32_t b) {
  uint32_t m = 1u << 31, p = 0;
  for (;;) {
    if (a & m) { p ^= b; if ((a & (m - 1)) == 0) break; }
    m >>= 1;
    b = (b & 1) ? (b >> 1) ^ O_CRC_POLY : b >> 1;
  }
  return p;
}
/* x^(8*nbytes) mod P */
static inline uint32_t o_xpow8(uint64_t nbytes) {
  uint32_t result = 0x80000000u;       /* x^0 */
  uint32_t sq = 0x00800000u;           /* x^8 */
  while (nbytes) {
    if (nbytes & 1) result = o_multmodp(sq, result);
    sq = o_multmodp(sq, sq);
    nbytes >>= 1;
  }
  return result;
}
#endif
