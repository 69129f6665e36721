// kb_common.h — device state and shared device helpers of the simulator (included by kb_sim.hip).
//
// HBM layout, C = capacity, W = C rounded up to 2048:
//   stamp  [C][W]  u8   Known(t) stamp byte of (node, peer); meaningful only where the member bit is set
//   bits   [C][W/32] u32 membership bitset (the authority for "peer in known_peers")
//   segp   [C][64] {raw, cnt} crc0 of the members of each W/64-id segment (fingerprint checkpoints)
//   sdirty [C] u64  segments whose checkpoint is stale; dirty[C] u8: cached fingerprint stale
//   susp   [C][8]   WaitingForPing / WaitingForIndirectPing slots; cur [C][8] curious_peers entries
//   flog   [C][LOGCAP] u32 freshness log: (peer << 8 | round & 255) each time a stamp becomes
//          Known(now); flog_n [C] entries appended; fstart [C][16] flog_n at the start of each round
#pragma once
#include "kb_device.h"
#include "../../include/kaboodle_sim.h"

namespace kb {

enum StatIdx {
  S_PING, S_PINGREQ, S_ACK, S_KP, S_KPR, S_BJOIN, S_BFAIL, S_DEAD, S_LOSS, S_WINDOW, S_OVERSIZE, S_PART, S_BDROP,
  S_RMTIMEOUT, S_RMFAILED, S_JRESP, S_CUROVF, S_CLEAVE, S_CJOIN,
  S_KPIDS,                        // peer entries of the KnownPeers messages sent (kb_stats.sent_kp_ids)
  S_ROWB,                         // bytes the row pass moved (bench roofline; not a kb_stats field)
  S_FOLDB,                        // member-bit bytes the fold read (bench roofline; not a kb_stats field)
  S_A3ROWS, S_A3DEEP, S_A3CHUNKS,  // A3 scans: rows, rows past their first chunk, chunks read (kb_sim_debug_counters)
  S_ALIVER,                       // running peers summed over the rounds (kb_stats.alive_rounds; counted by shard 0)
  S_RESPB,                        // bytes k_resp_wave moved (bench; not a kb_stats field)
  S_PROCB,                        // bytes k_proc moved (bench; not a kb_stats field)
  S_PROBERESP,                    // ProbeResponses sent (kb_stats.probe_responses)
  S_EXPORT,                       // records routed to external peers (kb_stats.exported)
  NSTAT
};
enum CtrIdx {
  C_KP, C_SLOW, C_ACTIVE, C_AGREE, C_ALIVE, C_LEAVES, C_NEXTFREE, C_ERR, C_FIRSTCONV, C_LASTCONV, C_LASTAGREE,
  C_LASTALIVE, C_DBG_INS, C_DBG_FP, C_DBG_MAXFP,
  C_DBG_KPR, C_DBG_KPRLOG, C_DBG_BASE,   // KB_DEBUG_WAVES: full KPR reply scans, log entries read, take_base
  C_DBG_TNODE, C_DBG_TMAX, C_DBG_TBASE, C_DBG_TINS,   // KB_DEV & 64: k_proc wall time (10 ns ticks) per part
  C_DBG_TSTART, C_DBG_TEND, C_DBG_MSGS,
  C_TICK,
  C_ROUND,                        // the round being simulated (k_log_mark): graph-replayed kernels read it here
  C_PATHS,                        // OR of the PATH_* bits of the kernel variants that did work (test surface)
  C_DBG_SLOW_LONG, C_DBG_SLOW_NONMEM, C_DBG_SLOW_DIRTY, C_DBG_SLOW_KPR, C_DBG_SLOW_OTHER,   // KB_DEV & 256: why k_proc
  C_RESTN,                        // responders k_resp_wave left to k_resp_node (their list: the wave lists' slow buffer)
  C_XREC, C_XPAY,                 // exported records / KnownPeers ids this round (external peers)
  NCTR
};
// kernel-variant coverage bits (kb_sim_debug_paths): the wide-row paths a >= 1M-id mesh takes
enum : uint32_t { PATH_PHASEB_HBM = 1, PATH_RESP_SCRATCH_SAMPLED = 2, PATH_RESP_SCRATCH_FULL = 4, PATH_KP_BIG_HBM = 8,
                  PATH_PROC_UNSORTED = 16, PATH_BFAIL_PREP_HBM = 32, PATH_RESP_WAVE = 64, PATH_KP_BIG_LDS = 128,
                  PATH_RESP_WAVE_HBM = 256 };
constexpr int NSEG = 64;          // fingerprint checkpoints per row
constexpr int ZT = 9;             // LDS nibble tables for Z^0..Z^8
constexpr int ZB = 9 * 1024;      // byte tables for Z^0..Z^8 (4 lookups per multiply)

// Row shards: a shard holds the rows of ids [lo, hi) — the observer state of those
// peers.  Row-indexed tables are allocated for the local rows only and their pointers are biased by
// -lo rows, so every kernel indexes them with the global id.  Per-id facts (alive, start_round,
// identity CRCs) are replicated: every shard applies the same lifecycle events and churn draws.
struct Dev {
  uint32_t lo, hi;                // local rows (unsharded: 0, C)
  uint32_t C, W, SEGW, NWR;       // capacity, row stride, ids per segment (W/64), bitset words per row (W/32)
  uint32_t segq, segm;            // SEGW = 128 * segq; segm = ceil(2^32 / segq) (segment of id j without a divide)
  uint32_t k0, k1;
  uint32_t loss_thr, churn_thr;
  int32_t fault_end;
  uint32_t failed_mode;
  uint32_t pgroups;
  int32_t pstart, pend;
  uint32_t uniform, L;            // uniform segment length (20 + id_len) when uniform != 0
  uint32_t capk, capj;            // KnownPeers caps: KPR reply (size <= 10240), Join response (size < 10240)
  uint32_t paybound;              // payload entries reserved per KPR reply
  uint32_t dbg;                   // kb_config.debug_flags (KB_DBG_*): force the wide-row kernel variants
  uint32_t dev;                   // env KB_DEV: timing experiments only (skip parts; results are wrong)
  uint8_t* stamp;
  uint32_t* bits;
  uint2* segp;
  unsigned long long* sdirty;
  uint8_t* dirty;
  uint8_t* alive;
  uint8_t* idset;                 // [C] an identity was set on this never-bound address: not a fresh id
  uint32_t* abits;                // running set bitset [W/32]
  int32_t* start_round;
  uint32_t* n;
  uint32_t* fp;
  int32_t* last_bcast;
  uint32_t* a3cur;                // A3's rotation base: just before the last round's oldest candidate (§2.6)
  Susp* susp;
  Cur* cur;
  uint32_t* paq;
  uint32_t* paq_n;
  uint32_t* cseg;
  uint32_t* segmul;
  uint32_t* seglen;
  uint32_t* zpow;                 // Z^k, Z = x^(8L), k in [0, C+1]
  uint32_t* zfin;                 // Z^k * 0xFFFFFFFF (the init term of a k-member fingerprint)
  uint32_t* ztab;                 // [17][8][16] nibble tables of multiplication by Z^c
  uint32_t* zbtab;                // [9][4][256] byte tables of multiplication by Z^c
  uint32_t* htab;                 // [(W/8)][256] crc0 of every member pattern of every 8-id half block
  unsigned long long* stats;
  unsigned long long* sacc;       // [NACC][NSTAT] per-workgroup partial counters, folded into stats on read
  uint32_t* ctr;
  uint32_t* truefp;
  uint2* tfpart;                  // [64] ordered partials of the running set's fingerprint
  uint32_t* flog;
  uint32_t* flog_n;
  uint32_t* fstart;
  int32_t* kpr_big;               // round in which the node's KPR reply was proven oversize for the round
  uint16_t* lat;                  // [W][local rows] PeerInfo.latency in ms, PEER-major (LAT_NONE = None); null
                                  // unless track_latency
  int32_t wave;                   // delivery wave of the launch (latency clock)
  uint8_t* ext;                   // [C] external peers: records to them are exported
  struct XRec* xrec;              // exported records of the round (layout of kb_unicast), xrec_cap of them
  uint32_t* xids;                 // their KnownPeers ids, xids_cap of them
  uint32_t xrec_cap, xids_cap;
  int32_t* tst;                   // KB_VARIANT_EXACT_LRU: [local rows][W] the instant of every Known entry whose
                                  // stamp byte has saturated to ANCIENT (a fresher byte encodes its instant
                                  // itself); null otherwise
  int32_t* tlb;                   // with tst: [local rows][W / 1024] a lower bound of the saturated instants of
                                  // each 1024-id block (exact after k_a3_exact scans the block; INT32_MAX = none)
};

// a record routed to an external peer, as kb_unicast (include/kaboodle_sim.h)
struct XRec { int32_t round; uint32_t wave, sender, dest, seq, kind, a, fp, n, pay_off, pay_len, pad; };
constexpr uint32_t DERR_EXPORT = 11;
// export one routed record (and its KnownPeers ids, read from `pay`) for the host to drain after the round
__device__ inline void export_rec(uint32_t* ctr, XRec* xrec, uint32_t xrec_cap, uint32_t* xids, uint32_t xids_cap,
                                  const Msg& m, const uint32_t* pay, int32_t r, uint32_t w) {
  const uint32_t k = atomicAdd(&ctr[C_XREC], 1u);
  const uint32_t np = m.kind == K_KP ? m.a : 0u;
  const uint32_t po = np ? atomicAdd(&ctr[C_XPAY], np) : 0u;
  if (k >= xrec_cap || po + np > xids_cap) { atomicCAS(&ctr[C_ERR], 0u, DERR_EXPORT); return; }
  for (uint32_t q = 0; q < np; ++q) xids[po + q] = pay[m.off + q];
  xrec[k] = XRec{r, w, m.sender, m.dest, m.seq, m.kind, m.kind == K_KP ? 0u : m.a, m.fp, m.n, po, np, 0u};
}

// freshness log (the KnownPeersRequest reply set, :503-508, without scanning the row): an entry is
// appended exactly when a stamp byte changes to Known(now); a (peer, t) entry is live iff the peer
// is still a member whose stamp is exactly enc(t).  Window of round r = entries since fstart[r-9].
__device__ inline uint32_t log_entry(uint32_t peer, int32_t r) { return (peer << 8) | ((uint32_t)r & 255u); }
__device__ inline int32_t log_round(uint32_t e, int32_t r) { return r - (int32_t)(((uint32_t)r - (e & 255u)) & 255u); }
__device__ inline uint32_t log_window_start(const Dev& d, uint32_t i, int32_t r) {
  return r >= SHARE_AGE - 1 ? d.fstart[(size_t)i * 16 + ((uint32_t)(r - (SHARE_AGE - 1)) & 15u)] : 0u;
}
// copy n 16-byte words global -> LDS with `lanes` cooperating threads (index t, waves of consecutive t),
// as LDS-DMA loads (global_load_lds_dwordx4: no VGPR destination, every load of the copy in flight at
// once), then one vmcnt(0).  Register staging had let the compiler sink each load into its guarded store
// and wait for it there — one HBM round trip per 16 B per lane.  The LDS destination of one wave's load
// is its base + 16 B × lane, which is the layout of consecutive words.
typedef __attribute__((address_space(3))) void lds_void_t;
typedef __attribute__((address_space(1))) void glb_void_t;
__device__ __attribute__((always_inline)) inline void stage16(uint4* dst, const uint4* src, uint32_t n, uint32_t t,
                                                             uint32_t lanes) {
  const uint32_t wb = t - lane();                        // the wave's first word of each pass
  for (uint32_t w0 = 0; wb + w0 < n; w0 += lanes) {
    if (t + w0 < n)
      __builtin_amdgcn_global_load_lds((glb_void_t*)(src + t + w0), (lds_void_t*)(dst + wb + w0), 16, 0, 0);
  }
  __builtin_amdgcn_s_waitcnt(0x0F70);                    // vmcnt(0): the copies have landed
  asm volatile("" ::: "memory");
}
// the same copy into global memory (a scratch destination): register staged, full groups of 8 loads with
// no condition between the loads and their stores
__device__ __attribute__((always_inline)) inline void copy16(uint4* dst, const uint4* src, uint32_t n, uint32_t t,
                                                            uint32_t lanes) {
  constexpr int U = 8;
  uint32_t w0 = t;
  for (; w0 + lanes * (U - 1) < n; w0 += lanes * U) {
    uint4 v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) v[u] = src[w0 + lanes * u];
#pragma unroll
    for (int u = 0; u < U; ++u) dst[w0 + lanes * u] = v[u];
  }
  for (; w0 < n; w0 += lanes) dst[w0] = src[w0];
}
// hand-off to the host through mapped pinned memory: the values, a system-scope release, then the
// sequence number the host polls for (one thread)
constexpr uint32_t PIN_WORDS = 1024;              // the mapped pinned buffer: values, then the sequence word
constexpr uint32_t PIN_SEQ = PIN_WORDS - 1;
__device__ inline void pin_publish(uint32_t* h, const uint32_t* v, uint32_t n, uint32_t seq) {
  for (uint32_t k = 0; k < n; ++k) h[k] = v[k];
  if (!seq) return;
  __threadfence_system();
  __hip_atomic_store(h + PIN_SEQ, seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}
// a wave kernel's round: its argument, or (argument < 0, the graph-captured receive window) the device copy
__device__ inline int32_t round_of(const Dev& d, int32_t r_arg) {
  return r_arg >= 0 ? r_arg : (int32_t)__builtin_amdgcn_readfirstlane(d.ctr[C_ROUND]);
}
__device__ inline void set_err(const Dev& d, uint32_t e) { atomicCAS(&d.ctr[C_ERR], 0u, e); }
// (read first: after the first hit the bit is set and the atomic on that one word is skipped)
__device__ inline void path_hit(const Dev& d, uint32_t bit) {
  if (!(__hip_atomic_load(&d.ctr[C_PATHS], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) & bit)) atomicOr(&d.ctr[C_PATHS], bit);
}
__device__ inline bool faults(const Dev& d, int32_t r) { return d.fault_end < 0 || r < d.fault_end; }
__device__ inline bool local(const Dev& d, uint32_t i) { return i >= d.lo && i < d.hi; }
__device__ inline bool part_blocks(const Dev& d, int32_t r, uint32_t a, uint32_t b) {
  if (d.pgroups <= 1 || r < d.pstart || r >= d.pend) return false;
  return ((uint64_t)a * d.pgroups / d.C) != ((uint64_t)b * d.pgroups / d.C);
}
__device__ inline uint8_t* row_of(const Dev& d, uint32_t i) { return d.stamp + (size_t)i * d.W; }
__device__ inline uint32_t* bits_of(const Dev& d, uint32_t i) { return d.bits + (size_t)i * d.NWR; }
__device__ inline bool is_mem(const Dev& d, uint32_t i, uint32_t j) { return (bits_of(d, i)[j >> 5] >> (j & 31)) & 1u; }
// j / SEGW = (j >> 7) / segq by a multiply-high (exact: j >> 7 < 2^16 and segq < 2^16)
__device__ inline uint32_t seg_of(const Dev& d, uint32_t j) { return d.segq == 1 ? (j >> 7) : __umulhi(j >> 7, d.segm); }
__device__ inline unsigned long long seg_bit(const Dev& d, uint32_t j) { return 1ull << seg_of(d, j); }
// membership changes: bit + stale-checkpoint mark (callers that batch marks pass mark=false)
__device__ inline bool mem_set(const Dev& d, uint32_t i, uint32_t j) {   // returns true if newly set
  const uint32_t m = 1u << (j & 31);
  return !(atomicOr(&bits_of(d, i)[j >> 5], m) & m);
}
__device__ inline bool mem_clr(const Dev& d, uint32_t i, uint32_t j) {   // returns true if it was set
  const uint32_t m = 1u << (j & 31);
  return (atomicAnd(&bits_of(d, i)[j >> 5], ~m) & m) != 0;
}
__device__ inline void mark(const Dev& d, uint32_t i, unsigned long long segs) {
  if (segs) { atomicOr(&d.sdirty[i], segs); d.dirty[i] = 1; }
}

// multiplication by Z^c (c in 0..8) through LDS nibble tables (conflict-free: 16 words per table)
__device__ inline uint32_t mulzc(const uint32_t* tab, uint32_t x, uint32_t c) {
  if (c == 0) return x;
  const uint32_t* t = tab + c * 128;
  return t[x & 15] ^ t[16 + ((x >> 4) & 15)] ^ t[32 + ((x >> 8) & 15)] ^ t[48 + ((x >> 12) & 15)] ^
         t[64 + ((x >> 16) & 15)] ^ t[80 + ((x >> 20) & 15)] ^ t[96 + ((x >> 24) & 15)] ^ t[112 + (x >> 28)];
}
__device__ inline uint32_t mulzb(const uint32_t* tab, uint32_t x, uint32_t c) {
  const uint32_t* t = tab + c * 1024;
  return t[x & 255] ^ t[256 + ((x >> 8) & 255)] ^ t[512 + ((x >> 16) & 255)] ^ t[768 + (x >> 24)];
}
__device__ inline void load_zbtab(const Dev& d, uint32_t* lds) {
  for (uint32_t k = threadIdx.x; k < ZB; k += blockDim.x) lds[k] = d.zbtab[k];
  __syncthreads();
}
__device__ inline void load_ztab(const Dev& d, uint32_t* lds) {
  for (uint32_t k = threadIdx.x; k < ZT * 128; k += blockDim.x) lds[k] = d.ztab[k];
  __syncthreads();
}
// x^(8*len) for arbitrary len (non-uniform identities only; small capacities)
__device__ inline uint32_t xpow8_dev(uint64_t nbytes) {
  uint32_t res = 0x80000000u, sq = 0x00800000u;
  while (nbytes) { if (nbytes & 1) res = multmodp(sq, res); sq = multmodp(sq, sq); nbytes >>= 1; }
  return res;
}
// ordered combine of fingerprint partials: (rawA over lower ids) then (rawB, cntB)
__device__ inline uint32_t comb(const Dev& d, uint32_t rawA, uint32_t rawB, uint32_t cntB) {
  return multmodp(d.uniform ? d.zpow[cntB] : xpow8_dev(cntB), rawA) ^ rawB;
}
__device__ inline uint32_t finish_fp(const Dev& d, uint32_t raw, uint32_t cnt) {
  return raw ^ multmodp(d.uniform ? d.zpow[cnt] : xpow8_dev(cnt), 0xFFFFFFFFu) ^ 0xFFFFFFFFu;
}
// fold one 8-id half block (member pattern m8, first id h*8) — table lookup + multiply by Z^popc
__device__ inline void fold_half(const Dev& d, const uint32_t* ztab, uint32_t h, uint32_t m8, uint32_t& raw,
                                 uint32_t& cnt) {
  if (!m8) return;
  const uint32_t c = __popc(m8);
  raw = mulzc(ztab, raw, c) ^ d.htab[(size_t)h * 256 + m8];
  cnt += c;
}
// checkpoint of segment k of row i from its bitset (any lane, independent).  For non-uniform
// identities (capacity <= 200) `cnt` carries the byte length instead of the member count.
__device__ inline uint2 fold_segment(const Dev& d, const uint32_t* ztab, uint32_t i, uint32_t k) {
  const uint32_t* b = bits_of(d, i);
  const uint32_t w0 = k * d.SEGW / 32, w1 = w0 + d.SEGW / 32;
  uint32_t raw = 0, cnt = 0;
  if (d.uniform) {
    for (uint32_t w = w0; w < w1; ++w) {
      const uint32_t x = b[w];
      if (!x) continue;
      fold_half(d, ztab, 4 * w, x & 0xFFu, raw, cnt);
      fold_half(d, ztab, 4 * w + 1, (x >> 8) & 0xFFu, raw, cnt);
      fold_half(d, ztab, 4 * w + 2, (x >> 16) & 0xFFu, raw, cnt);
      fold_half(d, ztab, 4 * w + 3, x >> 24, raw, cnt);
    }
  } else {
    for (uint32_t w = w0; w < w1; ++w) {
      uint32_t x = b[w];
      while (x) {
        const uint32_t j = w * 32 + (__ffs(x) - 1);
        x &= x - 1;
        raw = multmodp(d.segmul[j], raw) ^ d.cseg[j];
        cnt += d.seglen[j];
      }
    }
  }
  return make_uint2(raw, cnt);
}
// Global atomics are performed in L2 and do not refresh this CU's L1: after modifying bitset words
// with atomics, a kernel that reads them back invalidates its L1 first (agent-scope acquire).
__device__ inline void l1_acquire() { __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent"); }

// fingerprint of row i by one wave: refold the stale checkpoints (lane k <-> segment k), then an
// ordered tree combine of the 64 checkpoints.  `extra` = segments changed by the caller and not yet
// recorded in sdirty.  Returns the same value in every lane.
// Wave-wide combine of per-lane (raw, cnt) pieces in lane order; every lane ends with the total.  The tree's
// four levels inside each 16-lane row move data by DPP (no LDS round trip), their counts first so the four
// Z^cnt loads are in flight together; the four row totals are then combined from scalar registers.
__device__ inline void wave_combine(const Dev& d, uint32_t& raw, uint32_t& cnt) {
  const uint32_t l = lane();
  uint32_t oc[4], zp[4];
  uint32_t c = cnt;
  oc[0] = dpp_shl<1>(c); if ((l & 1) == 0) c += oc[0];
  oc[1] = dpp_shl<2>(c); if ((l & 3) == 0) c += oc[1];
  oc[2] = dpp_shl<4>(c); if ((l & 7) == 0) c += oc[2];
  oc[3] = dpp_shl<8>(c); if ((l & 15) == 0) c += oc[3];
  const uint32_t c0 = rdl(c, 0), c1 = rdl(c, 16), c2 = rdl(c, 32), c3 = rdl(c, 48);
  auto zpw = [&](uint32_t k) __attribute__((always_inline)) { return d.uniform ? d.zpow[k <= d.C ? k : 0] : xpow8_dev(k); };
#pragma unroll
  for (int t = 0; t < 4; ++t) zp[t] = zpw(oc[t]);
  const uint32_t z1 = zpw(c1), z3 = zpw(c3), z23 = zpw(c2 + c3);
  uint32_t o;
  o = dpp_shl<1>(raw); if ((l & 1) == 0) raw = multmodp(zp[0], raw) ^ o;
  o = dpp_shl<2>(raw); if ((l & 3) == 0) raw = multmodp(zp[1], raw) ^ o;
  o = dpp_shl<4>(raw); if ((l & 7) == 0) raw = multmodp(zp[2], raw) ^ o;
  o = dpp_shl<8>(raw); if ((l & 15) == 0) raw = multmodp(zp[3], raw) ^ o;
  const uint32_t r0 = rdl(raw, 0), r1 = rdl(raw, 16), r2 = rdl(raw, 32), r3 = rdl(raw, 48);
  raw = multmodp(z23, multmodp(z1, r0) ^ r1) ^ (multmodp(z3, r2) ^ r3);
  cnt = c0 + c1 + c2 + c3;
}

// Checkpoint of segment `lane` of row i with the stale ones (sd) refolded and stored: one per lane when
// many are stale; all 64 lanes on each one when few are (a lane alone on a segment is a chain of up to
// 144 dependent table steps — the in-order handlers typically dirty one segment per newly heard sender).
__device__ __attribute__((always_inline)) inline uint2 refold_stale(const Dev& d, const uint32_t* ztab, uint32_t i,
                                                                   unsigned long long sd) {
  const uint32_t l = lane();
  uint2 sp = make_uint2(0, 0);
  if (d.uniform && sd && __popcll(sd) <= 4) {
    sp = d.segp[(size_t)i * NSEG + l];
    const uint8_t* hb = reinterpret_cast<const uint8_t*>(bits_of(d, i));   // one byte per 8-id block
    const uint32_t nh = d.SEGW / 8;
    for (unsigned long long m = sd; m; m &= m - 1) {
      const uint32_t k = (uint32_t)(__ffsll((long long)m) - 1);
      uint32_t raw = 0, cnt = 0;
      const uint32_t h0 = k * nh + (l * nh) / 64, h1 = k * nh + ((l + 1) * nh) / 64;
      for (uint32_t h = h0; h < h1; ++h) fold_half(d, ztab, h, hb[h], raw, cnt);
      wave_combine(d, raw, cnt);
      raw = rdl(raw, 0); cnt = rdl(cnt, 0);
      if (l == k) { sp = make_uint2(raw, cnt); d.segp[(size_t)i * NSEG + k] = sp; }
    }
  } else if ((sd >> l) & 1ull) {
    sp = fold_segment(d, ztab, i, l);
    d.segp[(size_t)i * NSEG + l] = sp;
  } else {
    sp = d.segp[(size_t)i * NSEG + l];
  }
  return sp;
}
// Current fingerprint of row i with the whole wave: the stale checkpoints refolded, then the 64
// checkpoints combined.
__device__ __attribute__((always_inline)) inline uint32_t wave_fp(const Dev& d, const uint32_t* ztab, uint32_t i, unsigned long long extra) {
  const uint32_t l = lane();
  const unsigned long long sd = d.sdirty[i] | extra;
  const uint2 sp = refold_stale(d, ztab, i, sd);
  uint32_t raw = sp.x, cnt = sp.y;
  wave_combine(d, raw, cnt);
  raw = rdl(raw, 0); cnt = rdl(cnt, 0);
  if (l == 0 && sd) atomicAnd(&d.sdirty[i], ~sd);
  return finish_fp(d, raw, cnt);
}
// fingerprint of row i from its checkpoints by one thread (checkpoints must be fresh)
// (16 checkpoints and their Z^cnt per batch: the loads of a batch are in flight together)
__device__ inline uint32_t thread_fp(const Dev& d, uint32_t i) {
  uint32_t raw = 0, cnt = 0;
  const uint4* sp4 = reinterpret_cast<const uint4*>(d.segp + (size_t)i * NSEG);   // two checkpoints per 16 B
  for (int k0 = 0; k0 < NSEG; k0 += 16) {
    uint4 q[8];
#pragma unroll
    for (int t = 0; t < 8; ++t) q[t] = sp4[k0 / 2 + t];
    uint32_t z[16];
#pragma unroll
    for (int t = 0; t < 16; ++t) {
      const uint32_t c = (t & 1) ? q[t >> 1].w : q[t >> 1].y;
      z[t] = c ? (d.uniform ? d.zpow[c] : xpow8_dev(c)) : 0u;
    }
#pragma unroll
    for (int t = 0; t < 16; ++t) {
      const uint32_t x = (t & 1) ? q[t >> 1].z : q[t >> 1].x, c = (t & 1) ? q[t >> 1].w : q[t >> 1].y;
      if (c) { raw = multmodp(z[t], raw) ^ x; cnt += c; }
    }
  }
  return finish_fp(d, raw, cnt);
}

// position of the rem-th (0-based) set bit of x: a five-step popcount descent, no loop
__device__ inline uint32_t select_in_word(uint32_t x, uint32_t rem) {
  uint32_t pos = 0, c;
  c = __popc(x & 0xFFFFu); if (rem >= c) { rem -= c; x >>= 16; pos += 16; }
  c = __popc(x & 0xFFu);   if (rem >= c) { rem -= c; x >>= 8;  pos += 8; }
  c = __popc(x & 0xFu);    if (rem >= c) { rem -= c; x >>= 4;  pos += 4; }
  c = __popc(x & 0x3u);    if (rem >= c) { rem -= c; x >>= 2;  pos += 2; }
  if (rem >= (x & 1u)) pos += 1;
  return pos;
}
// 4-bit "byte != 0" mask of a little-endian dword (SWAR)
__device__ inline uint32_t nzmask4(uint32_t x) {
  const uint32_t y = (((x & 0x7F7F7F7Fu) + 0x7F7F7F7Fu) | x) & 0x80808080u;
  return ((y >> 7) | (y >> 14) | (y >> 21) | (y >> 28)) & 0xFu;
}

// ---- ping_random_peer's candidate lists: keys (stamp << 24 | address rotated to start after self) ----
__device__ inline void top5_insert(uint32_t (&k)[5], uint32_t nk) {
#pragma unroll
  for (int s = 0; s < 5; ++s) { if (nk < k[s]) { const uint32_t t = k[s]; k[s] = nk; nk = t; } }
}
__device__ inline uint32_t thr5(const uint32_t (&k)[5]) { return k[4] == 0xFFFFFFFFu ? 256u : (k[4] >> 24); }
// 4-bit "byte == v" mask of a little-endian dword (SWAR)
__device__ inline uint32_t eqmask4(uint32_t x, uint32_t v) { return ~nzmask4(x ^ (v * 0x01010101u)) & 0xFu; }

// ---- node-local state, single thread ----------------------------------------------------------
__device__ inline void susp_clear(const Dev& d, uint32_t i, uint32_t p) {
  Susp* s = d.susp + (size_t)i * SLOTS;
  for (int k = 0; k < SLOTS; ++k) if (s[k].kind && s[k].peer == p) s[k].kind = 0;
}
// ---- PeerInfo.latency (src/kaboodle.rs:789-817), DESIGN.md §2.7 ---------------------------------
// Simulated clock: the tick of round r at 1000·r ms, wave w of its receive window at 1000·r + w + 1.
// Invariant: LAT_NONE wherever the member bit is clear (removals write it), so an insertion needs no
// write: a new entry's latency is None (:412 on an absent sender, :294-296, :467).
// The table is peer-major: a round's Failed broadcasts remove the same few hundred peers from every
// row, so those writes land in a few contiguous columns (lines shared by adjacent rows) instead of
// one scattered line per (row, peer).
constexpr uint16_t LAT_NONE = 0xFFFFu;
__host__ __device__ inline uint32_t lat_stride(uint32_t rows) { return (rows + 7u) & ~7u; }   // 16-byte columns
__device__ inline uint16_t* lat_at(const Dev& d, uint32_t i, uint32_t p) {
  return d.lat + (size_t)p * lat_stride(d.hi - d.lo) + (i - d.lo);
}
__device__ inline void lat_none(const Dev& d, uint32_t i, uint32_t p) {
  if (d.lat) *lat_at(d, i, p) = LAT_NONE;
}
// the envelope prologue of a unicast from p while p is WaitingFor*(since): calculate_peer_latency
__device__ inline void lat_sample(const Dev& d, uint32_t i, uint32_t p, int32_t since, int32_t r) {
  if (!d.lat) return;
  uint16_t* q = lat_at(d, i, p);
  const uint32_t smp = 1000u * (uint32_t)(r - since) + (uint32_t)d.wave + 1u;
  const uint32_t prev = *q;
  uint32_t v = smp;
  if (prev != LAT_NONE)                                 // f64 as the reference, no fma contraction
    v = (uint32_t)__dadd_rn(__dmul_rn((double)smp, 0.8), __dmul_rn((double)prev, 1.0 - 0.8));
  *q = (uint16_t)(v < LAT_NONE ? v : LAT_NONE - 1u);
}

// lifecycle: the per-id part on every shard, the row part on the shard holding the row
__device__ __attribute__((always_inline)) inline void node_start(const Dev& d, uint32_t i, int32_t r) {      // src/lib.rs:136-156
  if (local(d, i)) {
    if (mem_set(d, i, i)) d.n[i] += 1;
    else susp_clear(d, i, i);
    row_of(d, i)[i] = enc(r, r);
    mark(d, i, seg_bit(d, i));
    d.last_bcast[i] = NONE_ROUND; d.paq_n[i] = 0; d.a3cur[i] = i;
    for (int k = 0; k < CSLOTS; ++k) d.cur[(size_t)i * CSLOTS + k].used = 0;
  }
  d.alive[i] = 1; d.start_round[i] = r;
}
__device__ __attribute__((always_inline)) inline void node_stop(const Dev& d, uint32_t i) {                  // src/lib.rs:159-183
  if (local(d, i)) {
    if (mem_clr(d, i, i)) { susp_clear(d, i, i); d.n[i] -= 1; mark(d, i, seg_bit(d, i)); }
    d.paq_n[i] = 0;
  }
  d.alive[i] = 0;
}

// block-wide sum (blockDim <= 1024), valid in thread 0
__device__ inline unsigned long long block_sum(unsigned long long v) {
  __shared__ unsigned long long red[16];
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  const int w = threadIdx.x >> 6;
  __syncthreads();
  if ((threadIdx.x & 63) == 0) red[w] = v;
  __syncthreads();
  unsigned long long t = 0;
  if (threadIdx.x == 0) for (int k = 0; k < (int)((blockDim.x + 63) >> 6); ++k) t += red[k];
  return t;
}
__device__ inline void stat_add(const Dev& d, int idx, unsigned long long v) {
  const unsigned long long t = block_sum(v);
  if (threadIdx.x == 0 && t) atomicAdd(&d.stats[idx], t);
}
// Counters of the per-wave kernels: block-wide sums of N counters with one LDS exchange and one
// barrier, added to the block's own accumulation slot (d.sacc; k_stats_fold folds the slots into
// d.stats when the host reads them).  Every workgroup of every wave adding to the same few stats
// words would serialise in the memory system.
constexpr uint32_t NACC = 1024;
__device__ inline void slot_add(const Dev& d, int idx, unsigned long long v) {   // this workgroup's slot
  atomicAdd(&d.sacc[(size_t)(blockIdx.x % NACC) * NSTAT + idx], v);
}
template <int N>
__device__ inline void stat_add_n(const Dev& d, const int (&idx)[N], const unsigned long long (&v)[N]) {
  __shared__ unsigned long long red[16][N];
  const int w = threadIdx.x >> 6;
  unsigned long long s[N];
#pragma unroll
  for (int k = 0; k < N; ++k) {
    s[k] = v[k];
    for (int o = 32; o > 0; o >>= 1) s[k] += __shfl_xor(s[k], o, 64);
  }
  if ((threadIdx.x & 63) == 0)
#pragma unroll
    for (int k = 0; k < N; ++k) red[w][k] = s[k];
  __syncthreads();
  if (threadIdx.x < (unsigned)N) {
    unsigned long long t = 0;
    for (int k = 0; k < (int)((blockDim.x + 63) >> 6); ++k) t += red[k][threadIdx.x];
    if (t) atomicAdd(&d.sacc[(size_t)(blockIdx.x % NACC) * NSTAT + idx[threadIdx.x]], t);
  }
}

// ---- message outboxes --------------------------------------------------------------------------
struct OutBuf {
  Msg* msgs; uint32_t* pay; uint32_t* off; uint32_t* cap; uint32_t* cnt; uint32_t* poff;
  uint32_t msg_cap, pay_cap;
};
__device__ inline void emit_msg(const OutBuf& ob, const Dev& d, uint32_t i, uint32_t& oseq, uint32_t dest,
                                uint32_t kind, uint32_t a, uint32_t fp, uint32_t n, uint32_t off) {
  if (lane() == 0) {
    if (oseq >= ob.cap[i] || ob.off[i] + oseq >= ob.msg_cap) set_err(d, DERR_OUTBOX);
    else {
      Msg m; m.dest = dest; m.sender = i; m.seq = oseq; m.kind = kind; m.a = a; m.fp = fp; m.n = n; m.off = off;
      ob.msgs[ob.off[i] + oseq] = m;
    }
  }
  oseq++;
}

}  // namespace kb
