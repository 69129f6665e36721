// kb_sparse.h — configs[4]'s layout on the GPU: Kaboodle's round over SPARSE rows
// (kb_config.variant = KB_VARIANT_SPARSE_ROWS).  Included by kb_sim.hip; every C-ABI entry
// point of a handle created with that variant is answered by this engine.
//
// A view (known_peers: ObservableHashMap<SocketAddr, PeerInfo>, src/observable_hashmap.rs:84-142 over
// PeerInfo, src/structs.rs:12-41) is held as
//   members = base Δ x        (or x alone for a row that never adopted the base: a fresh joiner)
//   stamp   = ANCIENT for every member without an explicit entry, else the entry's byte
// where `base` is the initial member set of a converged start (one bitset, prefix counts and prefix folds
// for the whole mesh) and each row keeps ONE sorted list of packed entries
//     id << 9 | x << 8 | stamp
//   x     = the id is an exception: its membership differs from the base's
//   stamp = 0 (ancient, or not a member) or the explicit byte (1 suspect, > 2 Known inside the window)
// Every entry has x set or a nonzero stamp; ids are < 2^23 (capacity <= 7.8M).  The oracle's
// KB_VARIANT_SPARSE_ROWS (oracle/kb_oracle.c `srow`, the same information in two lists) holds the same
// state byte for byte, and GPU = oracle is checked every round (tests/test_gpu_sparse.py).
//
// The algorithms that make the layout pay (all O(entries), never O(N) per row):
//   ping_random_peer  :655-703  every member without an explicit entry is ANCIENT, the smallest key, so the
//                               five oldest are the first five such members in rotated order from the
//                               sweep front: a walk over the gaps between entries, the base read as bits
//   handle_suspected  :558-653  the k-th indirect-ping candidate by select over gaps (base prefix counts)
//   KnownPeersRequest :483-501  the fresh stamps are explicit (fresh > ANCIENT): a scan of the list
//   generate_fingerprint :71-83 raw(A ‖ base ∩ [a, b)) = (raw(A) ⊕ bpre[a])·Z^(bcnt[b]−bcnt[a]) ⊕ bpre[b]:
//                               one multiply per exception
// Join responses (:356-392) enumerate base Δ x in id order (word-wise over the base bitset); they occur
// only with joins (churn, restarts, join starts).
//
// Execution: one thread per row for the row work of each phase (the per-row work of a round is a few list
// operations, so rows are the parallelism; 4M rows fill the chip), messages through the same record
// pipeline shape as the dense engine: per-wave records in (sender, seq) order, routed (dead receiver,
// partition, Philox loss), counted per destination, scanned, scattered into inboxes, handled per
// destination in (KnownPeers first, then sender, seq) order, emissions into per-node regions sized by a
// bound per delivered message, compacted into the next wave's records.
#pragma once
#include "kb_common.h"
#include "kb_round.h"

namespace kb {

constexpr uint32_t SP_XF = 1u << 8;
constexpr uint32_t SP_NONE = 0xFFFFFFFFu;
constexpr uint32_t DERR_SPARSE = 10;              // a row's entry list outgrew kb_config.sparse_row_cap
constexpr uint32_t SP_ACC = 1024;                 // per-workgroup accumulation slots of the counters

// Row shards: a handle holds the rows of ids [lo, hi).  Row tables (ent .. paq_n below, and the
// host's per-node scratch arrays) have hi - lo rows and are biased by -lo rows, so kernels index them with global
// ids; per-id tables (alive, start_round, idset, ext, the base and identity tables) cover all C ids on every shard
// and are kept identical by replaying the same lifecycle on each.
struct SpDev {
  uint32_t C, ECAP, nb;                           // ids, entries per row, |base|
  uint32_t lo, hi;                                // this shard's rows (0, C unsharded)
  uint32_t rank0;                                 // this shard adds the replicated counters (churn) to the stats
  uint32_t ESTR;                                  // row stride: ECAP rounded up to 4 (16-byte aligned rows)
  uint32_t k0, k1, loss_thr, churn_thr;
  int32_t fault_end;
  uint32_t failed_mode, pgroups;
  int32_t pstart, pend;
  uint32_t uniform, L, capk, capj;
  uint32_t* ent;                                  // [C][ESTR] sorted packed entries
  uint32_t* ne;                                   // [C] entries in use
  uint8_t* based;                                 // [C] members = base Δ x (1) or x (0)
  uint32_t* n; uint32_t* fp; uint8_t* dirty; int32_t* last_bcast; uint32_t* a3cur;
  Susp* susp; Cur* cur; uint32_t* paq; uint32_t* paq_n;
  uint8_t* alive; int32_t* start_round;
  uint8_t* idset;                                 // [C] an identity was set on this never-bound address (not fresh)
  uint8_t* ext;                                   // [C] external peers: records to them are exported
  XRec* xrec; uint32_t* xids; uint32_t xrec_cap, xids_cap;
  uint32_t* cseg; uint32_t* segmul; uint32_t* seglen;
  uint32_t* bbits;                                // [C/32 + 1] base bitset
  uint32_t* bcnt;                                 // [C + 1] |base ∩ [0, k)|
  uint32_t* bpre;                                 // [C + 1] crc0 fold of base ∩ [0, k) (uniform identities)
  uint32_t* zpow;                                 // [C + 2] Z^k, Z = x^(8L)
  unsigned long long* stats;                      // [NSTAT]
  unsigned long long* sacc;                       // [SP_ACC][NSTAT] per-workgroup partial counters
  uint32_t* ctr;                                  // CtrIdx
  unsigned long long* tacc;                       // [SP_ACC][2] agreement / running partials of the tick
};

// ---- small helpers -----------------------------------------------------------------------------------
__device__ inline void sp_err(const SpDev& d, uint32_t e) { atomicCAS(&d.ctr[C_ERR], 0u, e); }
__device__ inline bool sp_faults(const SpDev& d, int32_t r) { return d.fault_end < 0 || r < d.fault_end; }
__device__ inline bool sp_part(const SpDev& d, int32_t r, uint32_t a, uint32_t b) {
  if (d.pgroups <= 1 || r < d.pstart || r >= d.pend) return false;
  return ((uint64_t)a * d.pgroups / d.C) != ((uint64_t)b * d.pgroups / d.C);
}
__device__ inline bool sp_bbit(const SpDev& d, uint32_t j) { return (d.bbits[j >> 5] >> (j & 31)) & 1u; }
__device__ inline bool sp_local(const SpDev& d, uint32_t i) { return i >= d.lo && i < d.hi; }
__device__ inline uint32_t sp_gid(const SpDev& d) { return d.lo + blockIdx.x * blockDim.x + threadIdx.x; }   // row kernels
__device__ inline uint32_t* sp_row(const SpDev& d, uint32_t i) { return d.ent + (size_t)i * d.ESTR; }
// a row's entries e[k..n) move up one place and v lands at e[k] (insertion; n < ESTR), in 16-byte steps from the
// top of the row's aligned groups down (a thread per row: a quarter of the memory instructions of a word loop)
__device__ inline void sp_ins_at(uint32_t* e, uint32_t k, uint32_t n, uint32_t v) {
  uint4* e4 = reinterpret_cast<uint4*>(e);
  const uint32_t gk = k >> 2, kk = k & 3u;
  uint32_t g = n >> 2;
  uint4 cur = e4[g];
  for (; g > gk; --g) {
    const uint4 lo = e4[g - 1];
    e4[g] = make_uint4(lo.w, cur.x, cur.y, cur.z);
    cur = lo;
  }
  e4[gk] = make_uint4(kk == 0 ? v : cur.x, kk < 1 ? cur.x : (kk == 1 ? v : cur.y),
                      kk < 2 ? cur.y : (kk == 2 ? v : cur.z), kk < 3 ? cur.z : (kk == 3 ? v : cur.w));
}
// e[k] leaves: e[k+1..n) move down one place (removal), the same 16-byte steps upward
__device__ inline void sp_del_at(uint32_t* e, uint32_t k, uint32_t n) {
  uint4* e4 = reinterpret_cast<uint4*>(e);
  const uint32_t gk = k >> 2, gl = (n - 1) >> 2, kk = k & 3u;
  uint4 cur = e4[gk];
  for (uint32_t g = gk; g <= gl; ++g) {
    const uint4 nx = g < gl ? e4[g + 1] : make_uint4(0, 0, 0, 0);
    const uint32_t lo = g == gk ? kk : 0u;                   // words below k keep their place
    e4[g] = make_uint4(lo > 0 ? cur.x : cur.y, lo > 1 ? cur.y : cur.z, lo > 2 ? cur.z : cur.w, nx.x);
    cur = nx;
  }
}
__device__ inline uint32_t sp_word(const U4& w, uint32_t k) { return k == 0 ? w.x : k == 1 ? w.y : k == 2 ? w.z : w.w; }
// first entry index whose id is >= j (entries are id << 9 | low bits, so e < j << 9 iff its id < j)
__device__ inline uint32_t sp_lb(const uint32_t* e, uint32_t n, uint32_t j) {
  uint32_t lo = 0, hi = n;
  const uint32_t key = j << 9;
  while (lo < hi) { const uint32_t mid = (lo + hi) >> 1; if (e[mid] < key) lo = mid + 1; else hi = mid; }
  return lo;
}
// block-wide sums of N counters into this workgroup's accumulation slot (every thread of the block calls)
template <int N>
__device__ inline void sp_stats(const SpDev& d, const int (&idx)[N], const unsigned long long (&v)[N]) {
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
    if (t) atomicAdd(&d.sacc[(size_t)(blockIdx.x % SP_ACC) * NSTAT + idx[threadIdx.x]], t);
  }
}

// ---- the row's state byte (st_get / st_set of the oracle) ---------------------------------------------
struct SpLook { uint32_t k, e; bool has; };
__device__ inline SpLook sp_look(const SpDev& d, uint32_t i, uint32_t j) {
  const uint32_t* e = sp_row(d, i);
  const uint32_t n = d.ne[i];
  SpLook l;
  l.k = sp_lb(e, n, j);
  l.has = l.k < n && (e[l.k] >> 9) == j;
  l.e = l.has ? e[l.k] : 0u;
  return l;
}
__device__ inline bool sp_mem(const SpDev& d, uint32_t i, uint32_t j, const SpLook& l) {
  return (d.based[i] && sp_bbit(d, j)) != (l.has && (l.e & SP_XF));
}
__device__ inline uint8_t sp_byte(const SpDev& d, uint32_t i, uint32_t j, const SpLook& l) {
  if (!sp_mem(d, i, j, l)) return ST_UNKNOWN;
  const uint32_t b = l.e & 255u;
  return b ? (uint8_t)b : ST_ANCIENT;
}
__device__ inline uint8_t sp_get(const SpDev& d, uint32_t i, uint32_t j) { return sp_byte(d, i, j, sp_look(d, i, j)); }
// the byte of (i, j) becomes b (0 = not a member); l = sp_look(d, i, j) of the current state
__device__ inline void sp_put(const SpDev& d, uint32_t i, uint32_t j, uint8_t b, const SpLook& l) {
  bool xf = l.has && (l.e & SP_XF);
  if ((b != ST_UNKNOWN) != sp_mem(d, i, j, l)) xf = !xf;
  const uint32_t eb = (b == ST_UNKNOWN || b == ST_ANCIENT) ? 0u : b;
  uint32_t* e = sp_row(d, i);
  const uint32_t n = d.ne[i];
  if (!xf && !eb) {
    if (l.has) { sp_del_at(e, l.k, n); d.ne[i] = n - 1; }
    return;
  }
  const uint32_t v = (j << 9) | (xf ? SP_XF : 0u) | eb;
  if (l.has) { e[l.k] = v; return; }
  if (n >= d.ECAP) { sp_err(d, DERR_SPARSE); return; }
  sp_ins_at(e, l.k, n, v);
  d.ne[i] = n + 1;
}

// ---- ObservableHashMap operations (src/observable_hashmap.rs:84-142) -------------------------------
__device__ inline Susp* sp_susp_find(const SpDev& d, uint32_t i, uint32_t p) {
  Susp* s = d.susp + (size_t)i * SLOTS;
  for (int k = 0; k < SLOTS; ++k) if (s[k].kind && s[k].peer == p) return &s[k];
  return nullptr;
}
// insert(p, Known(t)), clearing WaitingFor* state; true if p was new
__device__ inline bool sp_insert_known(const SpDev& d, uint32_t i, uint32_t p, int32_t t, int32_t r) {
  const SpLook l = sp_look(d, i, p);
  const uint8_t was = sp_byte(d, i, p, l);
  if (was == ST_SUSPECT) { Susp* q = sp_susp_find(d, i, p); if (q) q->kind = 0; }
  sp_put(d, i, p, enc(t, r), l);
  if (was == ST_UNKNOWN) { d.n[i] += 1; d.dirty[i] = 1; return true; }
  return false;
}
__device__ inline bool sp_remove(const SpDev& d, uint32_t i, uint32_t p) {
  const SpLook l = sp_look(d, i, p);
  const uint8_t b = sp_byte(d, i, p, l);
  if (b == ST_UNKNOWN) return false;
  if (b == ST_SUSPECT) { Susp* q = sp_susp_find(d, i, p); if (q) q->kind = 0; }
  sp_put(d, i, p, ST_UNKNOWN, l);
  d.n[i] -= 1; d.dirty[i] = 1;
  return true;
}
__device__ inline bool sp_set_suspect(const SpDev& d, uint32_t i, uint32_t p, int32_t kind, int32_t r) {
  Susp* q = sp_susp_find(d, i, p);
  if (!q) {
    Susp* sl = d.susp + (size_t)i * SLOTS;
    for (int k = 0; k < SLOTS; ++k) if (!sl[k].kind) { q = &sl[k]; break; }
    if (!q) return false;
    q->peer = p;
  }
  q->kind = kind; q->since = r;
  sp_put(d, i, p, ST_SUSPECT, sp_look(d, i, p));
  return true;
}
// curious_peers (src/kaboodle.rs:101, :536-540, :423, :644)
__device__ inline Cur* sp_cur_find(const SpDev& d, uint32_t i, uint32_t p) {
  Cur* c = d.cur + (size_t)i * CSLOTS;
  for (int k = 0; k < CSLOTS; ++k) if (c[k].used && c[k].peer == p) return &c[k];
  return nullptr;
}
__device__ inline uint32_t sp_cur_add(const SpDev& d, uint32_t i, uint32_t p, uint32_t observer) {   // 1 = overflow
  Cur* e = sp_cur_find(d, i, p);
  if (!e) {
    Cur* c = d.cur + (size_t)i * CSLOTS;
    for (int k = 0; k < CSLOTS; ++k) if (!c[k].used) { e = &c[k]; break; }
    if (!e) return 1;
    e->used = 1; e->peer = p; e->nobs = 0;
  }
  for (uint32_t k = 0; k < e->nobs; ++k) if (e->obs[k] == observer) return 0;
  if (e->nobs == NOBS) return 1;
  e->obs[e->nobs++] = observer;
  return 0;
}

// ---- generate_fingerprint (src/kaboodle.rs:71-83) over base Δ x ----------------------------------------
__device__ inline uint32_t sp_fold(const SpDev& d, uint32_t i) {
  const uint32_t* e = sp_row(d, i);
  const uint32_t n = d.ne[i];
  const bool based = d.based[i];
  if (!d.uniform) {                               // non-uniform identity lengths (capacity <= 200): every id
    uint32_t raw = 0, q = 0;
    uint64_t len = 0;
    for (uint32_t j = 0; j < d.C; ++j) {
      bool inx = false;
      if (q < n && (e[q] >> 9) == j) { inx = (e[q] & SP_XF) != 0; ++q; }
      if ((based && sp_bbit(d, j)) != inx) { raw = multmodp(d.segmul[j], raw) ^ d.cseg[j]; len += d.seglen[j]; }
    }
    return raw ^ multmodp(xpow8_dev(len), 0xFFFFFFFFu) ^ 0xFFFFFFFFu;
  }
  const uint32_t Z = d.zpow[1];
  uint32_t raw = 0, pos = 0, cnt = 0;
  const uint4* e4 = reinterpret_cast<const uint4*>(e);
  for (uint32_t g = 0; g < (n + 3u) >> 2; ++g) {  // 16-byte loads (rows are 16-byte aligned)
    const uint4 q4 = e4[g];
    const uint32_t w4[4] = {q4.x, q4.y, q4.z, q4.w};
#pragma unroll
    for (uint32_t t = 0; t < 4; ++t) {
      const uint32_t x = w4[t];
      if (4u * g + t >= n || !(x & SP_XF)) continue;
      const uint32_t j = x >> 9;
      if (based) {                                // the base's members in [pos, j), one multiply
        const uint32_t c = d.bcnt[j] - d.bcnt[pos];
        raw = multmodp(d.zpow[c], raw ^ d.bpre[pos]) ^ d.bpre[j];
        cnt += c;
      }
      if (!based || !sp_bbit(d, j)) { raw = multmodp(Z, raw) ^ d.cseg[j]; cnt++; }   // a member outside the base
      pos = j + 1;
    }
  }
  if (based) {
    const uint32_t c = d.bcnt[d.C] - d.bcnt[pos];
    raw = multmodp(d.zpow[c], raw ^ d.bpre[pos]) ^ d.bpre[d.C];
    cnt += c;
  }
  return raw ^ multmodp(d.zpow[cnt], 0xFFFFFFFFu) ^ 0xFFFFFFFFu;
}
__device__ inline uint32_t sp_fp(const SpDev& d, uint32_t i) {
  if (d.dirty[i]) { d.fp[i] = sp_fold(d, i); d.dirty[i] = 0; }
  return d.fp[i];
}

// ---- member walks ------------------------------------------------------------------------------------
// the next base member in [pos, end) (end if none)
__device__ inline uint32_t sp_next_base(const SpDev& d, uint32_t pos, uint32_t end) {
  while (pos < end) {
    const uint32_t w = d.bbits[pos >> 5] >> (pos & 31);
    if (w) { const uint32_t j = pos + (uint32_t)__ffs(w) - 1u; return j < end ? j : end; }
    pos = (pos | 31u) + 1u;
  }
  return end;
}
// the base member of rank k (0-based): smallest j with bcnt[j + 1] > k
__device__ inline uint32_t sp_base_select(const SpDev& d, uint32_t k) {
  uint32_t lo = 0, hi = d.C - 1;
  while (lo < hi) { const uint32_t mid = (lo + hi) >> 1; if (d.bcnt[mid + 1] > k) hi = mid; else lo = mid + 1; }
  return lo;
}
// f(j) for every member j of row i, ascending; stops when f returns false
template <class F>
__device__ inline void sp_members(const SpDev& d, uint32_t i, F f) {
  const uint32_t* e = sp_row(d, i);
  const uint32_t n = d.ne[i];
  if (!d.based[i]) {
    for (uint32_t q = 0; q < n; ++q) if ((e[q] & SP_XF) && !f(e[q] >> 9)) return;
    return;
  }
  const uint32_t nw = (d.C + 31) / 32;
  uint32_t q = 0;
  for (uint32_t w = 0; w < nw; ++w) {
    uint32_t m = d.bbits[w];
    while (q < n && (e[q] >> 9) < (w + 1) * 32) { if (e[q] & SP_XF) m ^= 1u << ((e[q] >> 9) & 31u); ++q; }
    while (m) { const uint32_t j = w * 32 + (uint32_t)__ffs(m) - 1u; m &= m - 1; if (!f(j)) return; }
  }
}

// handle_suspected_peers' candidate k (0-based) of Known && != self, ascending id (:571-577)
__device__ inline uint32_t sp_a2_select(const SpDev& d, uint32_t i, uint32_t k) {
  const uint32_t* e = sp_row(d, i);
  const uint32_t n = d.ne[i];
  if (!d.based[i]) {
    for (uint32_t q = 0; q < n; ++q) {
      const uint32_t x = e[q], j = x >> 9;
      if ((x & SP_XF) && (x & 255u) != ST_SUSPECT && j != i) { if (k == 0) return j; --k; }
    }
    return SP_NONE;
  }
  uint32_t pos = 0;
  for (uint32_t q = 0; q <= n; ++q) {
    const uint32_t end = q < n ? (e[q] >> 9) : d.C;
    const bool self_in = i >= pos && i < end && sp_bbit(d, i);
    const uint32_t gc = d.bcnt[end] - d.bcnt[pos] - (self_in ? 1u : 0u);   // base members of the gap, not self
    if (k < gc) {
      const uint32_t rk = d.bcnt[pos] + k;
      uint32_t j = sp_base_select(d, rk);
      if (self_in && j >= i) j = sp_base_select(d, rk + 1);
      return j;
    }
    k -= gc;
    if (q == n) break;
    const uint32_t x = e[q], j = x >> 9;
    const bool mem = sp_bbit(d, j) != ((x & SP_XF) != 0);
    if (mem && j != i && (x & 255u) != ST_SUSPECT) { if (k == 0) return j; --k; }
    pos = j + 1;
  }
  return SP_NONE;
}

// ping_random_peer's five smallest (stamp, rotated id) keys
struct SpTop5 { uint32_t best[5], kh[5], kl[5]; int nb; };
__device__ inline void sp_top5_add(SpTop5& t, uint32_t j, uint32_t kh, uint32_t kl) {
  if (t.nb == NUM_CANDIDATES && (kh > t.kh[4] || (kh == t.kh[4] && kl > t.kl[4]))) return;
  int pos = t.nb < NUM_CANDIDATES ? t.nb : NUM_CANDIDATES - 1;
  while (pos > 0 && (t.kh[pos - 1] > kh || (t.kh[pos - 1] == kh && t.kl[pos - 1] > kl))) {
    t.kh[pos] = t.kh[pos - 1]; t.kl[pos] = t.kl[pos - 1]; t.best[pos] = t.best[pos - 1]; --pos;
  }
  t.kh[pos] = kh; t.kl[pos] = kl; t.best[pos] = j;
  if (t.nb < NUM_CANDIDATES) t.nb++;
}
__device__ inline uint32_t sp_rot(uint32_t j, uint32_t a3, uint32_t C) { return (j + C - a3 - 1) % C; }
// the ancient members of [lo, hi) in id order, until five are held: the gaps between entries are base
// members (ancient), an entry is ancient iff it is a member without an explicit stamp
__device__ inline void sp_a3_range(const SpDev& d, uint32_t i, uint32_t lo, uint32_t hi, SpTop5& t, uint32_t a3) {
  const uint32_t* e = sp_row(d, i);
  const uint32_t n = d.ne[i];
  const bool based = d.based[i];
  uint32_t q = sp_lb(e, n, lo), pos = lo;
  while (t.nb < NUM_CANDIDATES) {
    const uint32_t end = (q < n && (e[q] >> 9) < hi) ? (e[q] >> 9) : hi;
    if (based)
      for (uint32_t j = sp_next_base(d, pos, end); j < end && t.nb < NUM_CANDIDATES; j = sp_next_base(d, j + 1, end))
        if (j != i) sp_top5_add(t, j, ST_ANCIENT, sp_rot(j, a3, d.C));
    if (t.nb == NUM_CANDIDATES || end == hi) break;
    const uint32_t x = e[q], j = x >> 9;
    const bool mem = (based && sp_bbit(d, j)) != ((x & SP_XF) != 0);
    if (mem && !(x & 255u) && j != i) sp_top5_add(t, j, ST_ANCIENT, sp_rot(j, a3, d.C));
    pos = j + 1; ++q;
  }
}

// ---- message regions ------------------------------------------------------------------------------------
struct SpOut {                                    // one wave's emissions: per-node regions of a staging buffer
  Msg* stage; const uint32_t* eoff; const uint32_t* ecap;   // region start / capacity (records)
  uint32_t* pay; const uint32_t* poff; const uint32_t* pcap; // KnownPeers payload region (ids)
  uint32_t* en;                                   // records emitted per node
};
__device__ inline void sp_emit(const SpDev& d, const SpOut& o, uint32_t i, uint32_t& seq, uint32_t dest, uint32_t kind,
                               uint32_t a, uint32_t fp, uint32_t n, uint32_t off) {
  if (seq >= o.ecap[i]) { sp_err(d, DERR_OUTBOX); return; }
  Msg m; m.dest = dest; m.sender = i; m.seq = seq; m.kind = kind; m.a = a; m.fp = fp; m.n = n; m.off = off;
  o.stage[o.eoff[i] + seq] = m;
  seq++;
}
// the emission bound of one delivered message of kind k (its handler's replies)
__device__ inline uint32_t sp_reply_bound(uint32_t k) {
  return k == K_PING || k == K_PINGREQ ? 1u : k == K_ACK ? (uint32_t)NOBS + 1u : k == K_KPR ? 2u : 0u;
}

// ---- round kernels ------------------------------------------------------------------------------------
__global__ void k_sp_init(SpDev d, uint32_t n0, uint32_t converged) {   // over all ids: per-id facts, then the local rows
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= d.C) return;
  d.start_round[i] = i < n0 ? 0 : NONE_ROUND;
  if (i < n0) d.alive[i] = 1;
  if (!sp_local(d, i)) return;
  d.last_bcast[i] = NONE_ROUND; d.a3cur[i] = i;
  d.based[i] = (i < d.nb || d.nb == 0) ? 1 : 0;
  if (i >= n0) return;
  sp_insert_known(d, i, i, 0, 0);                 // known_peers.insert(self, Known(now)) src/kaboodle.rs:145-152
  d.dirty[i] = 1;
  if (converged) { d.n[i] = n0; d.last_bcast[i] = -1000; }   // running for a while: no Join at round 0
}
// stamp window: explicit Known stamps shift down by 64; the ones that saturate become implicit
__global__ void k_sp_rebase(SpDev d) {
  const uint32_t i = sp_gid(d);
  if (i >= d.hi) return;
  uint32_t* e = sp_row(d, i);
  const uint32_t n = d.ne[i];
  uint32_t o = 0;
  for (uint32_t q = 0; q < n; ++q) {
    uint32_t x = e[q], b = x & 255u;
    if (b > ST_ANCIENT) {
      b = b > ST_ANCIENT + EPOCH ? b - EPOCH : 0u;
      x = (x & ~255u) | b;
    }
    if (!(x & SP_XF) && !(x & 255u)) continue;
    e[o++] = x;
  }
  d.ne[i] = o;
}
// lifecycle (src/lib.rs:136-183, src/kaboodle.rs:114-185)
__device__ inline void sp_node_start(const SpDev& d, uint32_t i, int32_t r) {
  d.alive[i] = 1; d.start_round[i] = r;
  if (!sp_local(d, i)) return;                    // the row's part: on the shard holding it
  sp_insert_known(d, i, i, r, r);
  d.dirty[i] = 1;
  d.last_bcast[i] = NONE_ROUND;
  for (int k = 0; k < CSLOTS; ++k) d.cur[(size_t)i * CSLOTS + k].used = 0;
  d.paq_n[i] = 0; d.a3cur[i] = i;
}
__device__ inline void sp_node_stop(const SpDev& d, uint32_t i) {
  d.alive[i] = 0;
  if (!sp_local(d, i)) return;
  sp_remove(d, i, i);
  d.paq_n[i] = 0;
}
// a restart whose row a sharded mesh moved between shards first (sp_move_row): the start of the fresh address
constexpr uint32_t EV_START_MOVED = 3;
// Kaboodle::start on a stopped instance: a fresh address that inherits the map; unsharded
__device__ inline void sp_node_restart(const SpDev& d, uint32_t from, uint32_t to, int32_t r) {
  const uint32_t n = d.ne[from];
  const uint32_t* a = sp_row(d, from);
  uint32_t* b = sp_row(d, to);
  for (uint32_t q = 0; q < n; ++q) b[q] = a[q];
  d.ne[to] = n; d.based[to] = d.based[from];
  for (int k = 0; k < SLOTS; ++k) d.susp[(size_t)to * SLOTS + k] = d.susp[(size_t)from * SLOTS + k];
  d.n[to] = d.n[from]; d.dirty[to] = 1;
  sp_node_start(d, to, r);
}
__global__ void k_sp_events(SpDev d, const Event* ev, uint32_t nev, int32_t r) {
  if (threadIdx.x || blockIdx.x) return;
  for (uint32_t k = 0; k < nev; ++k) {
    const uint32_t i = ev[k].node;
    if (ev[k].kind == EV_STOP) { if (d.alive[i]) sp_node_stop(d, i); }
    else if (ev[k].kind == EV_RESTART) sp_node_restart(d, ev[k].src, i, r);
    else if (ev[k].kind == EV_START_MOVED) sp_node_start(d, i, r);
    else if (!d.alive[i]) sp_node_start(d, i, r);
  }
}
// a restart's map across shards (sharded meshes): the old address's row packed on the shard holding it, unpacked
// into the fresh address's row on the shard holding that (the rest of the restart is EV_START_MOVED)
constexpr uint32_t SP_PACK_HDR = 4 + 4 * SLOTS;   // ne, based, n, pad, the suspect slots; then ESTR entries
__global__ void k_sp_row_pack(SpDev d, uint32_t from, uint32_t* buf) {
  const uint32_t n = d.ne[from];
  if (blockIdx.x == 0 && threadIdx.x == 0) {
    buf[0] = n; buf[1] = d.based[from]; buf[2] = d.n[from]; buf[3] = 0;
    const Susp* s = d.susp + (size_t)from * SLOTS;
    for (int k = 0; k < SLOTS; ++k) { buf[4 + 4 * k] = s[k].peer; buf[5 + 4 * k] = (uint32_t)s[k].since; buf[6 + 4 * k] = (uint32_t)s[k].kind; buf[7 + 4 * k] = 0; }
  }
  const uint32_t* e = sp_row(d, from);
  for (uint32_t q = blockIdx.x * blockDim.x + threadIdx.x; q < n; q += gridDim.x * blockDim.x) buf[SP_PACK_HDR + q] = e[q];
}
__global__ void k_sp_row_unpack(SpDev d, uint32_t to, const uint32_t* buf) {
  const uint32_t n = buf[0];
  if (blockIdx.x == 0 && threadIdx.x == 0) {
    d.ne[to] = n; d.based[to] = (uint8_t)buf[1]; d.n[to] = buf[2]; d.dirty[to] = 1;
    Susp* s = d.susp + (size_t)to * SLOTS;
    for (int k = 0; k < SLOTS; ++k) { s[k].peer = buf[4 + 4 * k]; s[k].since = (int32_t)buf[5 + 4 * k]; s[k].kind = (int32_t)buf[6 + 4 * k]; s[k].pad = 0; }
  }
  uint32_t* e = sp_row(d, to);
  for (uint32_t q = blockIdx.x * blockDim.x + threadIdx.x; q < n; q += gridDim.x * blockDim.x) e[q] = buf[SP_PACK_HDR + q];
}
__global__ void k_sp_churn_leave(SpDev d, int32_t r) {   // over all ids: every shard replays the lifecycle
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  unsigned long long left = 0;
  if (i < d.C && d.alive[i] && d.start_round[i] != r &&
      philox(i, (uint32_t)r, (uint32_t)P_CHURN << 24, 0, d.k0, d.k1).x < d.churn_thr) { sp_node_stop(d, i); left = 1; }
  const unsigned long long t = block_sum(left);
  if (threadIdx.x == 0 && t) atomicAdd(&d.ctr[C_LEAVES], (uint32_t)t);
}
__global__ void k_sp_churn_join(SpDev d, int32_t r) {
  if (threadIdx.x || blockIdx.x) return;
  const uint32_t leaves = d.ctr[C_LEAVES];
  uint32_t nf = d.ctr[C_NEXTFREE], joins = 0;
  for (uint32_t k = 0; k < leaves; ++k) {          // fresh ids only
    while (nf < d.C && (d.start_round[nf] != NONE_ROUND || d.idset[nf])) nf++;
    if (nf >= d.C) break;
    sp_node_start(d, nf++, r);
    joins++;
  }
  d.ctr[C_NEXTFREE] = nf; d.ctr[C_LEAVES] = 0;
  if (d.rank0) { d.stats[S_CLEAVE] += leaves; d.stats[S_CJOIN] += joins; }   // replicated: counted once
}

// the running set's fingerprint: SP_TFP contiguous id ranges folded by a thread each, then combined in order
constexpr uint32_t SP_TFP = 4096;
__global__ __launch_bounds__(256) void k_sp_truefp_part(SpDev d, uint2* part) {
  const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= SP_TFP) return;
  const uint32_t per = (d.C + SP_TFP - 1) / SP_TFP, j0 = t * per, j1 = min(d.C, j0 + per);
  uint32_t raw = 0, cnt = 0;
  for (uint32_t j = j0; j < j1; ++j) {
    if (!d.alive[j]) continue;
    if (d.uniform) { raw = multmodp(d.zpow[1], raw) ^ d.cseg[j]; cnt++; }
    else { raw = multmodp(d.segmul[j], raw) ^ d.cseg[j]; cnt += d.seglen[j]; }
  }
  part[t] = make_uint2(raw, cnt);
}
__device__ inline uint32_t sp_zc(const SpDev& d, uint32_t c) { return d.uniform ? d.zpow[c] : xpow8_dev(c); }
__global__ __launch_bounds__(64) void k_sp_truefp_fin(SpDev d, const uint2* part, uint32_t* out) {
  __shared__ uint2 g[64];
  const uint32_t l = threadIdx.x, per = SP_TFP / 64;
  uint32_t raw = 0, cnt = 0;
  for (uint32_t k = l * per; k < (l + 1) * per; ++k) {
    const uint2 p = part[k];
    if (p.y) { raw = multmodp(sp_zc(d, p.y), raw) ^ p.x; cnt += p.y; }
  }
  g[l] = make_uint2(raw, cnt);
  __syncthreads();
  if (l == 0) {
    raw = 0; cnt = 0;
    for (uint32_t k = 0; k < 64; ++k) if (g[k].y) { raw = multmodp(sp_zc(d, g[k].y), raw) ^ g[k].x; cnt += g[k].y; }
    out[0] = raw ^ multmodp(sp_zc(d, cnt), 0xFFFFFFFFu) ^ 0xFFFFFFFFu;
  }
}

// ---- broadcast phase: round r-1's Failed, Join and Probe deliveries (src/kaboodle.rs:256-331) -----------
struct SpBc {
  const BCast* bfail; uint32_t nf;
  uint32_t fcounted;                             // the Failed group was counted by k_sp_bfail_sf (socket_faithful)
  const BCast* bjoin; uint32_t nj; uint32_t JW;
  uint32_t* jnew; uint32_t* jresp;               // [local rows][JW] bits: the entry inserted its joiner / got a response
  uint32_t* jr_n; uint32_t* jr_pay;              // per node: responses, their payload ids
  uint32_t np; uint2* presp; uint32_t* presp_n; uint32_t presp_cap;
};
// should_respond_to_broadcast (:333-354), the integer restatement of gen_bool
__device__ inline bool sp_should_respond(const SpDev& d, uint32_t i, uint32_t c2, uint32_t c3, int32_t r) {
  const int64_t o = (int64_t)d.n[i] - 2;
  if (o <= 0) return true;
  int64_t pct = 100 - o * o;
  if (pct < 1) pct = 1;
  const uint32_t u = philox(i, (uint32_t)r, c2, c3, d.k0, d.k1).x;
  return (int64_t)mulhi(u, 100) < pct;
}
__global__ __launch_bounds__(256) void k_sp_bcast(SpDev d, SpBc bc, int32_t r) {
  const uint32_t i = sp_gid(d);
  unsigned long long lost = 0, removed = 0, presp = 0, plost = 0, jresp = 0;
  uint32_t nresp = 0, pay = 0;
  if (i < d.hi && d.alive[i] && d.start_round[i] < r) {
    const bool fl = sp_faults(d, r) && d.loss_thr;
    // partition groups: the receiver's once, each entry's precomputed by k_sp_bcast_write (BCast.pad)
    const bool pact = d.pgroups > 1 && r >= d.pstart && r < d.pend;
    const uint32_t rg = pact ? (uint32_t)((uint64_t)i * d.pgroups / d.C) : 0u;
    U4 w = U4{0, 0, 0, 0};
    uint32_t wk = SP_NONE;
    for (uint32_t k = 0; k < (bc.fcounted ? 0u : bc.nf); ++k) {   // Failed(p) :268-283
      const BCast b = bc.bfail[k];
      if (b.sender == i) continue;
      bool ls = pact && b.pad != rg;
      if (!ls && fl) {
        if ((k >> 2) != wk) { wk = k >> 2; w = philox(i, (uint32_t)r, ((uint32_t)P_BLOSS << 24) | wk, 0, d.k0, d.k1); }
        ls = sp_word(w, k & 3u) < d.loss_thr;
      }
      if (ls) { lost++; continue; }
      if (b.peer == i) continue;
      if (d.failed_mode == KB_FAILED_SIM_SENDER && sp_get(d, i, b.sender) != ST_UNKNOWN) removed += sp_remove(d, i, b.peer);
    }
    wk = SP_NONE;
    for (uint32_t k = 0; k < bc.nj; ++k) {                   // Join{addr} :284-304
      const BCast b = bc.bjoin[k];
      if (b.sender == i) continue;
      bool ls = pact && b.pad != rg;
      if (!ls && fl) {
        if ((k >> 2) != wk) { wk = k >> 2; w = philox(i, (uint32_t)r, ((uint32_t)P_BLOSS << 24) | (1u << 23) | wk, 0, d.k0, d.k1); }
        ls = sp_word(w, k & 3u) < d.loss_thr;
      }
      if (ls) { lost++; continue; }
      if (!sp_insert_known(d, i, b.sender, r, r)) continue;
      bc.jnew[(size_t)(i - d.lo) * bc.JW + (k >> 5)] |= 1u << (k & 31);
      if (!sp_should_respond(d, i, (uint32_t)P_RESPOND << 24, b.sender, r)) continue;
      bc.jresp[(size_t)(i - d.lo) * bc.JW + (k >> 5)] |= 1u << (k & 31);
      const uint32_t m = d.n[i];
      nresp++; pay += (d.uniform && m > d.capj) ? d.capj : m;
    }
    for (uint32_t e = 0; e < bc.np; ++e) {                   // Probe(addr) :305-331
      if (fl && sp_word(philox(i, (uint32_t)r, ((uint32_t)P_PROBE << 24) | (e >> 2), 0, d.k0, d.k1), e & 3u) < d.loss_thr) {
        lost++; continue;
      }
      if (!sp_should_respond(d, i, ((uint32_t)P_RESPOND << 24) | (1u << 23) | e, 0, r)) continue;
      presp++;
      if (fl && philox(i, (uint32_t)r, ((uint32_t)P_PROBE << 24) | (1u << 23) | e, 1, d.k0, d.k1).x < d.loss_thr) { plost++; continue; }
      const uint32_t slot = atomicAdd(bc.presp_n, 1u);
      if (slot < bc.presp_cap) bc.presp[slot] = make_uint2(i, e);
    }
    jresp = nresp;
  }
  if (i < d.hi) { bc.jr_n[i] = nresp; bc.jr_pay[i] = pay; }
  const int idx[5] = {S_BDROP, S_RMFAILED, S_PROBERESP, S_LOSS, S_JRESP};
  const unsigned long long v[5] = {lost, removed, presp, plost, jresp};
  sp_stats(d, idx, v);
}

// The Failed group in socket_faithful mode: a Failed broadcast is never honoured there, so its
// only effect on a receiver is whether the delivery was lost (drop_bcast): entries from the receiver itself are
// skipped, partition-blocked ones are lost, the rest lost iff word e mod 4 of philox(recv, r, BLOSS | e/4, 0) is
// below the threshold (the draws of k_sp_bcast and the oracle, src/kaboodle.rs:268-283).  Every receiver
// evaluates ~N/10 entries a round, N x N/40 Philox calls at 4M peers: the kernel is bound by them.  The list
// arrives packed (sender << 8 | partition group, four entries per 16 bytes, 0xFFFFFFFF padding) and is staged
// through LDS, one broadcast 16-byte read per four entries; a group of four whose entries are all blocked or
// the receiver's own takes no draw.
constexpr uint32_t SP_FK_LDS = 1024;              // 16-byte groups (4096 entries) staged per pass
__global__ __launch_bounds__(256) void k_sp_bfail_sf(SpDev d, const uint4* __restrict__ fkey, uint32_t nf, int32_t r) {
  __shared__ uint4 sk[SP_FK_LDS];
  const uint32_t i = sp_gid(d);
  const bool act = i < d.hi && d.alive[i] && d.start_round[i] < r;
  const bool fl = sp_faults(d, r) && d.loss_thr;
  const bool pact = d.pgroups > 1 && r >= d.pstart && r < d.pend;
  const uint32_t rg = pact ? (uint32_t)((uint64_t)i * d.pgroups / d.C) : 0u;
  const uint32_t ng = (nf + 3) / 4, thr = d.loss_thr;
  unsigned long long lost = 0;
  for (uint32_t g0 = 0; g0 < ng; g0 += SP_FK_LDS) {
    const uint32_t gn = min(SP_FK_LDS, ng - g0);
    __syncthreads();
    for (uint32_t t = threadIdx.x; t < gn; t += blockDim.x) sk[t] = fkey[g0 + t];
    __syncthreads();
    if (!act) continue;
    uint32_t lg = 0;
    for (uint32_t g = 0; g < gn; ++g) {
      const uint4 k4 = sk[g];
      const uint32_t kk[4] = {k4.x, k4.y, k4.z, k4.w};
      uint32_t draw = 0;
#pragma unroll
      for (int t = 0; t < 4; ++t) {
        const uint32_t k = kk[t];
        if (k == 0xFFFFFFFFu || (k >> 8) == i) continue;
        if (pact && (k & 255u) != rg) lg++;
        else draw |= 1u << t;
      }
      if (fl && draw) {
        const U4 w = philox(i, (uint32_t)r, ((uint32_t)P_BLOSS << 24) | (g0 + g), 0, d.k0, d.k1);
        lg += ((draw & 1u) && w.x < thr) + ((draw & 2u) && w.y < thr) + ((draw & 4u) && w.z < thr) + ((draw & 8u) && w.w < thr);
      }
    }
    lost += lg;
  }
  const int idx[1] = {S_BDROP};
  const unsigned long long v[1] = {lost};
  sp_stats(d, idx, v);
}

// Keyed permutation of [0, n): 4-round Feistel network on b = max(2, ceil(log2 n)) bits,
// halves of ceil(b/2) and floor(b/2) bits whose widths swap every round, cycle-walked into [0, n)
__device__ inline uint32_t sp_mix32(uint32_t x) {
  x ^= x >> 16; x *= 0x7feb352du; x ^= x >> 15; x *= 0x846ca68bu; x ^= x >> 16;
  return x;
}
__device__ inline uint32_t sp_prp(uint32_t x, uint32_t n, const U4& key) {
  uint32_t b = 2;
  while ((1ull << b) < n) b += 1;
  const uint32_t c = b / 2, a = b - c;
  const uint32_t kk[4] = {key.x, key.y, key.z, key.w};
  do {
    uint32_t L = x >> c, R = x & ((1u << c) - 1u), wl = a;
#pragma unroll
    for (int k = 0; k < 4; ++k) { const uint32_t t = R; R = L ^ (sp_mix32(R ^ kk[k]) & ((1u << wl) - 1u)); L = t; wl = b - wl; }
    x = (L << c) | R;
  } while (x >= n);
  return x;
}
__device__ inline void sp_heapsort(uint32_t* a, uint32_t n) {
  auto sift = [&](uint32_t s, uint32_t m) {
    for (;;) {
      uint32_t c = 2 * s + 1;
      if (c >= m) return;
      if (c + 1 < m && a[c + 1] > a[c]) c++;
      if (a[s] >= a[c]) return;
      const uint32_t t = a[s]; a[s] = a[c]; a[c] = t;
      s = c;
    }
  };
  if (n < 2) return;
  for (uint32_t s = n / 2; s-- > 0;) sift(s, n);
  for (uint32_t e = n - 1; e > 0; --e) { const uint32_t t = a[0]; a[0] = a[e]; a[e] = t; sift(0, e); }
}
// maybe_send_known_peers_to_peer (:356-392): the responses of node i, in Join-entry order, into the wave-0
// region after nothing (they come first).  The map a response lists is the map as it stood when that
// entry was handled: the final row minus the joiners later entries inserted (Join entries only insert).
__global__ __launch_bounds__(256) void k_sp_jresp(SpDev d, SpBc bc, SpOut o0, int32_t r) {
  const uint32_t i = sp_gid(d);
  if (i >= d.hi || !bc.jr_n[i]) return;
  const uint32_t* jn = bc.jnew + (size_t)(i - d.lo) * bc.JW;
  const uint32_t* jr = bc.jresp + (size_t)(i - d.lo) * bc.JW;
  uint32_t later = 0;                                        // new joiners of entries after the current one
  for (uint32_t w = 0; w < bc.JW; ++w) later += __popc(jn[w]);
  uint32_t seq = 0, pc = 0;
  for (uint32_t w = 0; w < bc.JW; ++w) {
    uint32_t bits = jn[w] | jr[w];
    while (bits) {
      const uint32_t k = w * 32 + (uint32_t)__ffs(bits) - 1u;
      bits &= bits - 1;
      if ((jn[w] >> (k & 31)) & 1u) later--;                  // this entry's own joiner is in its map
      if (!((jr[w] >> (k & 31)) & 1u)) continue;
      const uint32_t joiner = bc.bjoin[k].sender, m = d.n[i] - later;
      const bool trunc = d.uniform && m > d.capj;
      const uint32_t len = trunc ? d.capj : m;
      if (pc + len > o0.pcap[i]) { sp_err(d, DERR_PAYLOAD); return; }
      uint32_t* pay = o0.pay + o0.poff[i] + pc;
      // the later joiners, ascending ids (the Join list is in sender order), skipped by the member walk
      uint32_t xk = k + 1;
      auto next_ex = [&](uint32_t from) -> uint32_t {
        for (uint32_t x = from; x < bc.nj; ++x) if ((jn[x >> 5] >> (x & 31)) & 1u) return x;
        return bc.nj;
      };
      xk = next_ex(xk);
      uint32_t ex = xk < bc.nj ? bc.bjoin[xk].sender : SP_NONE;
      if (!trunc) {
        uint32_t c = 0;
        sp_members(d, i, [&](uint32_t j) {
          while (j > ex) { xk = next_ex(xk + 1); ex = xk < bc.nj ? bc.bjoin[xk].sender : SP_NONE; }
          if (j == ex) return true;
          if (c < len) pay[c] = j;
          c++;
          return true;
        });
        if (c != len) { sp_err(d, DERR_RESP); return; }
      } else {                                               // the first cap images of the keyed permutation
        const U4 key = philox(i, (uint32_t)r, (uint32_t)P_TRUNC << 24, joiner, d.k0, d.k1);
        for (uint32_t t = 0; t < len; ++t) pay[t] = sp_prp(t, m, key);
        sp_heapsort(pay, len);
        uint32_t rank = 0, nx = 0;
        sp_members(d, i, [&](uint32_t j) {
          while (j > ex) { xk = next_ex(xk + 1); ex = xk < bc.nj ? bc.bjoin[xk].sender : SP_NONE; }
          if (j == ex) return true;
          if (pay[nx] == rank) { pay[nx] = j; if (++nx == len) return false; }
          rank++;
          return true;
        });
        if (nx != len) { sp_err(d, DERR_RESP); return; }
      }
      sp_emit(d, o0, i, seq, joiner, K_KP, len, 0, 0, o0.poff[i] + pc);
      pc += len;
    }
  }
}

// wave-0 region bounds: the node's Join responses + its tick's emissions (A2 PingRequests, A3, A4)
__global__ void k_sp_bound0(SpDev d, const uint32_t* jr_n, uint32_t* ecap) {
  const uint32_t i = sp_gid(d);
  if (i >= d.hi) return;
  uint32_t b = 0;
  if (d.alive[i]) {
    uint32_t sc = 0;
    for (int k = 0; k < SLOTS; ++k) sc += d.susp[(size_t)i * SLOTS + k].kind != 0;
    b = jr_n[i] + NUM_INDIRECT * sc + 1u + d.paq_n[i];
  }
  ecap[i] = b;
}

// ---- tick (src/kaboodle.rs:746-779) ---------------------------------------------------------------
struct SpTickOut { uint32_t* bj; uint32_t* bnf; uint32_t* bfp; };   // per row: Join flag, Failed count, Failed peers [8]
__global__ __launch_bounds__(256) void k_sp_tick(SpDev d, SpOut o0, const uint32_t* jr_n, SpTickOut bo, const uint32_t* tfp,
                                                 int32_t r) {
  const uint32_t i = sp_gid(d);
  unsigned long long rmt = 0, agree = 0, run = 0;
  if (i < d.hi) { bo.bj[i] = 0; bo.bnf[i] = 0; o0.en[i] = jr_n[i]; }
  if (i < d.hi && d.alive[i]) {
    uint32_t seq = jr_n[i];
    // A1 maybe_broadcast_join (:228-251)
    if (d.last_bcast[i] == NONE_ROUND || (r - d.last_bcast[i] >= REBROADCAST && d.n[i] <= 1)) { bo.bj[i] = 1; d.last_bcast[i] = r; }
    // A2 handle_suspected_peers (:558-653)
    Susp* sl = d.susp + (size_t)i * SLOTS;
    int order[SLOTS], no = 0;
    for (int k = 0; k < SLOTS; ++k) if (sl[k].kind) order[no++] = k;
    for (int a = 1; a < no; ++a) {
      const int t = order[a];
      int b = a - 1;
      while (b >= 0 && sl[order[b]].peer > sl[t].peer) { order[b + 1] = order[b]; --b; }
      order[b + 1] = t;
    }
    const uint32_t m = d.n[i] - 1u - (uint32_t)no;
    uint32_t indirect[SLOTS], removed[SLOTS];
    int nind = 0, nrem = 0;
    for (int q = 0; q < no; ++q) {
      const Susp e = sl[order[q]];
      if (r - e.since < PING_TIMEOUT) continue;
      if (e.kind == SK_WFP) {
        const uint32_t k = m < (uint32_t)NUM_INDIRECT ? m : (uint32_t)NUM_INDIRECT;
        if (k == 0) { removed[nrem++] = e.peer; continue; }
        const U4 w = philox(i, (uint32_t)r, (uint32_t)P_INDIRECT << 24, e.peer, d.k0, d.k1);
        uint32_t pick[3];
        pick[0] = mulhi(w.x, m);
        if (k > 1) { const uint32_t b = mulhi(w.y, m - 1); pick[1] = b + (b >= pick[0]); }
        if (k > 2) {
          const uint32_t lo = min(pick[0], pick[1]), hi = max(pick[0], pick[1]);
          uint32_t c = mulhi(w.z, m - 2);
          if (c >= lo) c++;
          if (c >= hi) c++;
          pick[2] = c;
        }
        for (uint32_t t = 0; t < k; ++t) {
          const uint32_t tgt = sp_a2_select(d, i, pick[t]);
          if (tgt == SP_NONE) { sp_err(d, DERR_FP); continue; }
          sp_emit(d, o0, i, seq, tgt, K_PINGREQ, e.peer, 0, 0, 0);
        }
        indirect[nind++] = e.peer;
      } else {
        removed[nrem++] = e.peer;
      }
    }
    for (int q = 0; q < nind; ++q) sp_set_suspect(d, i, indirect[q], SK_WFIP, r);   // :631-639
    for (int q = 0; q < nrem; ++q) {                                                // :641-652
      sp_remove(d, i, removed[q]);
      Cur* c = sp_cur_find(d, i, removed[q]);
      if (c) c->used = 0;
      bo.bfp[(size_t)i * SLOTS + q] = removed[q];
    }
    bo.bnf[i] = (uint32_t)nrem;
    rmt = (unsigned long long)nrem;
    // A3 ping_random_peer (:655-703): oldest five by (stamp, rotated id), one uniformly; the sweep front
    // moves to the oldest candidate
    {
      SpTop5 t;
      t.nb = 0;
      const uint32_t a3 = d.a3cur[i], p0 = a3 + 1 == d.C ? 0 : a3 + 1;
      sp_a3_range(d, i, p0, d.C, t, a3);
      if (t.nb < NUM_CANDIDATES) sp_a3_range(d, i, 0, p0, t, a3);
      if (t.nb < NUM_CANDIDATES) {                           // fewer than five ancient: explicit Known stamps
        const uint32_t* e = sp_row(d, i);
        const uint32_t n = d.ne[i];
        for (uint32_t q = 0; q < n; ++q) {
          const uint32_t b = e[q] & 255u, j = e[q] >> 9;
          if (b > ST_ANCIENT && j != i) sp_top5_add(t, j, b, sp_rot(j, a3, d.C));
        }
      }
      if (t.nb > 0) {
        const uint32_t u = philox(i, (uint32_t)r, (uint32_t)P_PING << 24, 0, d.k0, d.k1).x;
        const uint32_t tgt = t.best[mulhi(u, (uint32_t)t.nb)];
        d.a3cur[i] = (t.best[0] + d.C - 1) % d.C;
        if (!sp_set_suspect(d, i, tgt, SK_WFP, r)) sp_err(d, DERR_SLOTS);
        else sp_emit(d, o0, i, seq, tgt, K_PING, 0, 0, 0, 0);
      }
    }
    // A4 handle_incoming_ping_requests (:550-556)
    for (uint32_t q = 0; q < d.paq_n[i]; ++q) sp_emit(d, o0, i, seq, d.paq[(size_t)i * PAQ + q], K_PING, 0, 0, 0, 0);
    d.paq_n[i] = 0;
    o0.en[i] = seq;
    run = 1;
    agree = sp_fp(d, i) == *tfp;                             // fingerprint at the ping step
  }
  const int idx[1] = {S_RMTIMEOUT};
  const unsigned long long v[1] = {rmt};
  sp_stats(d, idx, v);
  const unsigned long long ta = block_sum(agree);
  __syncthreads();
  const unsigned long long tr = block_sum(run);
  if (threadIdx.x == 0) {
    unsigned long long* s = d.tacc + (size_t)(blockIdx.x % SP_ACC) * 2;
    if (ta) atomicAdd(&s[0], ta);
    if (tr) atomicAdd(&s[1], tr);
  }
}
// the shard's broadcast lists (sender order); sharded meshes all-gather them into the round's lists afterwards
__global__ void k_sp_bcast_write(SpDev d, SpTickOut bo, const uint32_t* joff, const uint32_t* foff, BCast* bjoin, BCast* bfail) {
  const uint32_t i = sp_gid(d);
  if (i >= d.hi) return;
  uint32_t bseq = 0;
  const uint32_t g = d.pgroups > 1 ? (uint32_t)((uint64_t)i * d.pgroups / d.C) : 0u;   // the sender's partition group
  if (bo.bj[i]) bjoin[joff[i]] = BCast{i, i, bseq++, g};
  const uint32_t nf = bo.bnf[i];
  for (uint32_t q = 0; q < nf; ++q) bfail[foff[i] + q] = BCast{i, bo.bfp[(size_t)i * SLOTS + q], bseq++, g};
}
// k_sp_bfail_sf's packed Failed list: sender << 8 | partition group (groups <= 255), four entries per 16 bytes
__global__ void k_sp_fkey(const BCast* bfail, uint32_t nf, uint32_t* fkey) {
  const uint32_t k = blockIdx.x * blockDim.x + threadIdx.x;
  if (k < nf) fkey[k] = (bfail[k].sender << 8) | (bfail[k].pad & 255u);
  else if (k < ((nf + 3) & ~3u)) fkey[k] = 0xFFFFFFFFu;      // the last group's padding
}

// ---- receive window (src/kaboodle.rs:394-548) -----------------------------------------------------
struct SpRoute {
  const Msg* msgs; uint32_t M; uint8_t* status;
  const uint32_t* pay;                                // the records' KnownPeers ids (exports copy them)
  uint32_t* icnt; uint32_t* ebound; uint32_t* kprc;   // per destination: delivered, reply bound, KPRs
};
__device__ inline void sp_count_sent(const Msg& m, unsigned long long (&s)[6]) {
  s[m.kind == K_PING ? 0 : m.kind == K_PINGREQ ? 1 : m.kind == K_ACK ? 2 : m.kind == K_KP ? 3 : 4]++;
  if (m.kind == K_KP) s[5] += m.a;
}
// delivery of one record: dead receiver, partition, Philox loss keyed on (sender, round, wave, seq)
__global__ __launch_bounds__(256) void k_sp_route(SpDev d, SpRoute rt, int32_t r, uint32_t w) {
  const uint32_t k = blockIdx.x * blockDim.x + threadIdx.x;
  unsigned long long s[6] = {0, 0, 0, 0, 0, 0}, dead = 0, part = 0, loss = 0, xp = 0;
  if (k < rt.M) {
    const Msg m = rt.msgs[k];
    sp_count_sent(m, s);
    uint8_t st = 0;
    if (!d.alive[m.dest]) {
      if (d.ext[m.dest]) {                                             // a partition cuts it off too
        if (sp_part(d, r, m.sender, m.dest)) part++;
        else { export_rec(d.ctr, d.xrec, d.xrec_cap, d.xids, d.xids_cap, m, rt.pay, r, w); xp++; }
      }
      else dead++;
    }
    else if (sp_part(d, r, m.sender, m.dest)) part++;
    else if (sp_faults(d, r) && d.loss_thr &&
             philox(m.sender, (uint32_t)r, ((uint32_t)P_LOSS << 24) | w, m.seq, d.k0, d.k1).x < d.loss_thr) loss++;
    else {
      st = 1;
      atomicAdd(&rt.icnt[m.dest], 1u);
      const uint32_t b = sp_reply_bound(m.kind);
      if (b) atomicAdd(&rt.ebound[m.dest], b);
      if (m.kind == K_KPR) atomicAdd(&rt.kprc[m.dest], 1u);
    }
    rt.status[k] = st;
  }
  const int idx[10] = {S_PING, S_PINGREQ, S_ACK, S_KP, S_KPR, S_KPIDS, S_DEAD, S_PART, S_LOSS, S_EXPORT};
  const unsigned long long v[10] = {s[0], s[1], s[2], s[3], s[4], s[5], dead, part, loss, xp};
  sp_stats(d, idx, v);
}
// records from external peers (kb_sim_inject): room in their wave-0 regions, then the records after the tick
__global__ void k_sp_inject_prep(SpDev d, const XRec* inj, uint32_t n, uint32_t* ecap, uint32_t* pcap) {
  if (threadIdx.x || blockIdx.x) return;
  for (uint32_t k = 0; k < n; ++k) { ecap[inj[k].sender] += 1; if (inj[k].kind == K_KP) pcap[inj[k].sender] += inj[k].pay_len; }
}
__global__ void k_sp_inject(SpDev d, SpOut o, const XRec* inj, uint32_t n, const uint32_t* ids) {
  if (threadIdx.x || blockIdx.x) return;
  for (uint32_t k = 0; k < n; ++k) {
    const XRec x = inj[k];
    uint32_t seq = o.en[x.sender];
    const uint32_t off = o.poff[x.sender] + x.pad;
    if (x.kind == K_KP) for (uint32_t q = 0; q < x.pay_len; ++q) o.pay[off + q] = ids[x.pay_off + q];
    sp_emit(d, o, x.sender, seq, x.dest, x.kind, x.kind == K_KP ? x.pay_len : x.a, x.fp, x.n, x.kind == K_KP ? off : 0u);
    o.en[x.sender] = seq;
  }
}
// records never routed (emitted in the last wave): counted as sent and as missing the receive window
__global__ __launch_bounds__(256) void k_sp_window(SpDev d, const Msg* msgs, uint32_t M) {
  const uint32_t k = blockIdx.x * blockDim.x + threadIdx.x;
  unsigned long long s[6] = {0, 0, 0, 0, 0, 0}, win = 0;
  if (k < M) { sp_count_sent(msgs[k], s); win = 1; }
  const int idx[7] = {S_PING, S_PINGREQ, S_ACK, S_KP, S_KPR, S_KPIDS, S_WINDOW};
  const unsigned long long v[7] = {s[0], s[1], s[2], s[3], s[4], s[5], win};
  sp_stats(d, idx, v);
}
// payload bound of the node's KnownPeersRequest replies: each <= capk ids (larger ones are dropped) and <= its
// fresh stamps, which are explicit entries now or prologue insertions of this wave
__global__ void k_sp_paybound(SpDev d, const uint32_t* kprc, const uint32_t* icnt, uint32_t* pb) {
  const uint32_t i = sp_gid(d);
  if (i >= d.hi) return;
  const uint32_t k = kprc[i];
  pb[i] = k ? k * min(d.capk, d.ne[i] + icnt[i]) : 0u;
}
__global__ __launch_bounds__(256) void k_sp_scatter(SpRoute rt, const uint32_t* ioff, uint32_t* icur, uint32_t* inbox) {
  const uint32_t k = blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= rt.M || !rt.status[k]) return;
  const uint32_t dst = rt.msgs[k].dest;
  inbox[ioff[dst] + atomicAdd(&icur[dst], 1u)] = k;
}
struct SpWave {
  const Msg* in; const uint32_t* pay_in;          // this wave's records and their KnownPeers payload
  uint32_t* inbox; const uint32_t* ioff; const uint32_t* icnt;
};
// maybe_sync_known_peers (:707-740)
__device__ inline void sp_maybe_sync(const SpDev& d, const SpOut& o, uint32_t i, uint32_t& seq, uint32_t peer,
                                     uint32_t their_fp, uint32_t their_n) {
  const uint32_t f = sp_fp(d, i);
  if (f == their_fp || d.n[i] > their_n) return;
  sp_emit(d, o, i, seq, peer, K_KPR, 0, f, d.n[i], 0);
}
// handle_incoming_messages (:394-548) for one node: its inbox in (KnownPeers first, then sender, seq) order
// (compiled for 8 waves per SIMD: a thread per row waits on dependent loads, so occupancy is its throughput;
// 130 -> 64 VGPRs measured 13.5 -> 12.0 ms a round at 1M peers).
//   A KnownPeers list longer than SP_KP_WAVE ids is applied by the whole wave first: the lanes look its ids up in
// parallel (a binary search each) and lane 0 inserts the few unknown ones, re-checking each (a list may repeat an
// id).  One thread looking up a 567-id list alone was the wave's tail (≈ 5,000 dependent loads).  The arms of the
// inbox's KnownPeers group insert only unknown ids and its prologues set their senders Known(now), so inside the
// group they commute; the group comes first in the inbox, so applying its long arms before every prologue leaves
// the same row (src/kaboodle.rs:448-472).
constexpr uint32_t SP_KP_WAVE = 4;
constexpr uint32_t SP_KPR_ILP = 4;               // KnownPeersRequest reply scan: 16-byte row loads in flight per step
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(8))) void k_sp_handle(SpDev d, SpWave v, SpOut o, int32_t r) {
  const uint32_t i = sp_gid(d);
  unsigned long long oversize = 0, curovf = 0;
  if (i < d.hi) o.en[i] = 0;
  const bool act = i < d.hi && v.icnt[i];
  uint32_t* ib = nullptr;
  uint32_t cnt = 0;
  bool big = false;
  if (act) {
    ib = v.inbox + v.ioff[i];
    cnt = v.icnt[i];
    for (uint32_t q = 0; q < cnt; ++q) ib[q] |= (v.in[ib[q]].kind != K_KP) ? 0x80000000u : 0u;
    for (uint32_t a = 1; a < cnt; ++a) {                     // insertion sort (inboxes are short)
      const uint32_t x = ib[a];
      uint32_t b = a;
      while (b > 0 && ib[b - 1] > x) { ib[b] = ib[b - 1]; --b; }
      ib[b] = x;
    }
    for (uint32_t q = 0; q < cnt && !(ib[q] & 0x80000000u); ++q) big |= v.in[ib[q]].a > SP_KP_WAVE;
  }
  unsigned long long pend = __ballot(big);
  if (pend) wave_mem_sync();                                 // the sorted inboxes, read by every lane below
  for (; pend; pend &= pend - 1) {
    const uint32_t ri = rdl(i, __ffsll((long long)pend) - 1);
    const uint32_t* rib = v.inbox + v.ioff[ri];
    const uint32_t rcnt = v.icnt[ri];
    uint32_t added = 0;
    for (uint32_t q = 0; q < rcnt; ++q) {
      const uint32_t x = rib[q];
      if (x & 0x80000000u) break;                            // past the KnownPeers group
      const Msg m = v.in[x];
      if (m.a <= SP_KP_WAVE) continue;
      const uint32_t* p = v.pay_in + m.off;
      for (uint32_t k0 = 0; k0 < m.a; k0 += 64) {
        const bool in = k0 + lane() < m.a;
        const uint32_t j = in ? p[k0 + lane()] : 0u;
        const unsigned long long um = __ballot(in && sp_get(d, ri, j) == ST_UNKNOWN);
        for (unsigned long long u = um; u; u &= u - 1) {
          const uint32_t jj = rdl(j, __ffsll((long long)u) - 1);
          if (lane() == 0) {
            const SpLook l = sp_look(d, ri, jj);
            if (sp_byte(d, ri, jj, l) == ST_UNKNOWN) { sp_put(d, ri, jj, enc(r - SHARE_AGE, r), l); added++; }
          }
        }
        if (um) wave_mem_sync();                             // lane 0's row writes before the next lookups
      }
    }
    if (lane() == 0 && added) { d.n[ri] += added; d.dirty[ri] = 1; }
    wave_mem_sync();
  }
  if (act) {
    uint32_t seq = 0, pc = 0;
    for (uint32_t q = 0; q < cnt; ++q) {
      const Msg m = v.in[ib[q] & 0x7FFFFFFFu];
      const uint32_t from = m.sender;
      sp_insert_known(d, i, from, r, r);                     // prologue :406-415
      switch (m.kind) {
        case K_ACK: {                                        // :418-447
          Cur* e = sp_cur_find(d, i, m.a);
          if (e) {
            const uint32_t nobs = e->nobs;
            uint32_t obs[NOBS];
            for (int k = 0; k < NOBS; ++k) obs[k] = e->obs[k];
            e->used = 0;
            for (uint32_t k = 0; k < nobs; ++k) sp_emit(d, o, i, seq, obs[k], K_ACK, m.a, m.fp, m.n, 0);
          }
          sp_maybe_sync(d, o, i, seq, m.a, m.fp, m.n);
          break;
        }
        case K_KP: {                                         // :448-472
          if (m.a > SP_KP_WAVE) break;                       // applied by the wave above
          const uint32_t* p = v.pay_in + m.off;
          for (uint32_t k = 0; k < m.a; ++k) {               // one lookup per id: insert_known of an unknown id
            const uint32_t j = p[k];
            const SpLook l = sp_look(d, i, j);
            if (sp_byte(d, i, j, l) != ST_UNKNOWN) continue;
            sp_put(d, i, j, enc(r - SHARE_AGE, r), l);
            d.n[i] += 1; d.dirty[i] = 1;
          }
          break;
        }
        case K_KPR: {                                        // :473-512
          // one pass over the row in 16-byte loads: the fresh ids are written into the payload region as they are
          // counted (within its room), and kept only if the reply is deliverable
          const uint32_t fresh = enc(r - (SHARE_AGE - 1), r);
          const uint4* e4 = reinterpret_cast<const uint4*>(sp_row(d, i));
          const uint32_t n = d.ne[i];
          const uint32_t room = o.pcap[i] > pc ? o.pcap[i] - pc : 0u;
          uint32_t* pay = o.pay + o.poff[i] + pc;
          uint32_t c = 0;
          uint64_t sz = 8u + d.seglen[i] - ADDR_LEN + 4u + 8u;  // envelope: identity, tag, map length
          const uint32_t ng = (n + 3u) >> 2;
          for (uint32_t g0 = 0; g0 < ng; g0 += SP_KPR_ILP) {
            uint4 q4[SP_KPR_ILP];                            // the step's loads issued before any is used
#pragma unroll
            for (uint32_t u = 0; u < SP_KPR_ILP; ++u) q4[u] = g0 + u < ng ? e4[g0 + u] : make_uint4(0, 0, 0, 0);
#pragma unroll
            for (uint32_t u = 0; u < SP_KPR_ILP; ++u) {
              const uint32_t g = g0 + u, w4[4] = {q4[u].x, q4[u].y, q4[u].z, q4[u].w};
#pragma unroll
              for (uint32_t t = 0; t < 4; ++t) {
                const uint32_t x = w4[t], j = x >> 9;
                if (4u * g + t < n && (x & 255u) >= fresh && j != i && j != from) {
                  if (c < room) pay[c] = j;
                  c++;
                  sz += 10u + 8u + (d.uniform ? d.L : d.seglen[j]) - ADDR_LEN;
                }
              }
            }
          }
          if (sz > (uint64_t)BUFSZ) oversize++;              // truncated at the receiver: undeliverable (Q3)
          else if (c > room) sp_err(d, DERR_PAYLOAD);
          else {
            sp_emit(d, o, i, seq, from, K_KP, c, 0, 0, o.poff[i] + pc);
            pc += c;
          }
          sp_maybe_sync(d, o, i, seq, from, m.fp, m.n);
          break;
        }
        case K_PING:                                         // :513-532
          sp_emit(d, o, i, seq, from, K_ACK, i, sp_fp(d, i), d.n[i], 0);
          break;
        case K_PINGREQ:                                      // :533-545
          curovf += sp_cur_add(d, i, m.a, from);
          sp_emit(d, o, i, seq, m.a, K_PING, 0, 0, 0, 0);
          break;
      }
    }
    o.en[i] = seq;
  }
  const int idx[2] = {S_OVERSIZE, S_CUROVF};
  const unsigned long long vv[2] = {oversize, curovf};
  sp_stats(d, idx, vv);
}
// the emitted records, node by node (sender order, seq order inside), become the next wave's records
__global__ void k_sp_compact(SpDev d, SpOut o, const uint32_t* ooff, Msg* next) {
  const uint32_t i = sp_gid(d);
  if (i >= d.hi) return;
  const uint32_t n = o.en[i];
  const Msg* src = o.stage + o.eoff[i];
  Msg* dst = next + ooff[i];
  for (uint32_t q = 0; q < n; ++q) dst[q] = src[q];
}
// round results: agreement and running peers of this shard's rows (sharded meshes then sum them over the ranks),
// running peers summed over rounds; then convergence from the mesh's totals (k_sp_round_conv)
__global__ __launch_bounds__(1024) void k_sp_round_end(SpDev d, int32_t r) {
  unsigned long long a = 0, al = 0;
  for (uint32_t k = threadIdx.x; k < SP_ACC; k += blockDim.x) {
    a += d.tacc[2 * k]; al += d.tacc[2 * k + 1];
    d.tacc[2 * k] = 0; d.tacc[2 * k + 1] = 0;
  }
  a = block_sum(a);
  __syncthreads();
  al = block_sum(al);
  if (threadIdx.x == 0) {
    d.ctr[C_LASTAGREE] = (uint32_t)a; d.ctr[C_LASTALIVE] = (uint32_t)al;
    d.stats[S_ALIVER] += al;
  }
}
__global__ void k_sp_round_conv(SpDev d, int32_t r) {
  if (threadIdx.x || blockIdx.x) return;
  const uint32_t a = d.ctr[C_LASTAGREE], al = d.ctr[C_LASTALIVE];
  if (al && a == al) {
    if ((int32_t)d.ctr[C_FIRSTCONV] < 0) d.ctr[C_FIRSTCONV] = (uint32_t)r;
    d.ctr[C_LASTCONV] = (uint32_t)r;
  }
}

// ---- row shards: the delivery waves' exchange ----------------------------------------------
// The records of a wave are routed on the shard of their sender (dead receiver, partition and the Philox loss
// are keyed on the message, so the shard cannot change them), bucketed by the rank holding the destination's row
// in (sender, seq) order, all-to-all-v'd with their KnownPeers ids, and counted per destination on arrival.  The
// received blocks come in rank order = sender order, so a record's index keeps the (sender, seq) order the
// handler sorts by, exactly as in the unsharded wave.
struct SpX {
  uint32_t world, R, S;                               // ranks, local rows, rows per rank (rank of id j = j / S)
  uint32_t* xcnt; uint32_t* xpay;                     // [world][R] delivered records / KnownPeers ids per (rank, sender)
  uint32_t* xoff; uint32_t* xpoff;                    // their exclusive scans (rank-major: each rank's block contiguous)
  uint32_t* xb;                                       // [2 * world] records, then ids, to each rank
  Msg* smsg; uint32_t* spay;                          // send buffers
};
__global__ __launch_bounds__(256) void k_sp_route_x(SpDev d, SpRoute rt, SpX x, int32_t r, uint32_t w) {
  const uint32_t k = blockIdx.x * blockDim.x + threadIdx.x;
  unsigned long long s[6] = {0, 0, 0, 0, 0, 0}, dead = 0, part = 0, loss = 0, xp = 0;
  if (k < rt.M) {
    const Msg m = rt.msgs[k];
    sp_count_sent(m, s);
    uint8_t st = 0;
    if (!d.alive[m.dest]) {
      if (d.ext[m.dest]) {                                             // a partition cuts it off too
        if (sp_part(d, r, m.sender, m.dest)) part++;
        else { export_rec(d.ctr, d.xrec, d.xrec_cap, d.xids, d.xids_cap, m, rt.pay, r, w); xp++; }
      }
      else dead++;
    }
    else if (sp_part(d, r, m.sender, m.dest)) part++;
    else if (sp_faults(d, r) && d.loss_thr &&
             philox(m.sender, (uint32_t)r, ((uint32_t)P_LOSS << 24) | w, m.seq, d.k0, d.k1).x < d.loss_thr) loss++;
    else {
      st = 1;
      const size_t c = (size_t)(m.dest / x.S) * x.R + (m.sender - d.lo);
      atomicAdd(&x.xcnt[c], 1u);
      if (m.kind == K_KP && m.a) atomicAdd(&x.xpay[c], m.a);
    }
    rt.status[k] = st;
  }
  const int idx[10] = {S_PING, S_PINGREQ, S_ACK, S_KP, S_KPR, S_KPIDS, S_DEAD, S_PART, S_LOSS, S_EXPORT};
  const unsigned long long v[10] = {s[0], s[1], s[2], s[3], s[4], s[5], dead, part, loss, xp};
  sp_stats(d, idx, v);
}
// per rank: records and ids it receives from this shard (the blocks of the rank-major scans)
__global__ void k_sp_xbound(SpX x, const uint32_t* tot) {
  const uint32_t k = threadIdx.x;
  if (k >= x.world) return;
  const size_t a = (size_t)k * x.R, b = (size_t)(k + 1) * x.R;
  x.xb[k] = (k + 1 < x.world ? x.xoff[b] : tot[0]) - x.xoff[a];
  x.xb[x.world + k] = (k + 1 < x.world ? x.xpoff[b] : tot[1]) - x.xpoff[a];
}
// a thread per sender: its delivered records, in seq order, into each destination rank's block; a KnownPeers
// record's ids follow it, its offset made relative to the block (the receiver adds where the block lands)
__global__ __launch_bounds__(256) void k_sp_pack(SpDev d, SpX x, const Msg* msgs, const uint8_t* status, const uint32_t* pay,
                                                 const uint32_t* ooff, const uint32_t* en) {
  const uint32_t i = sp_gid(d);
  if (i >= d.hi) return;
  const uint32_t n = en[i], li = i - d.lo;
  if (!n) return;
  uint32_t c[XMAX], pc[XMAX];
  for (uint32_t q = 0; q < x.world; ++q) { c[q] = 0; pc[q] = 0; }
  for (uint32_t q = 0; q < n; ++q) {
    const uint32_t k = ooff[i] + q;
    if (!status[k]) continue;
    Msg m = msgs[k];
    const uint32_t dr = m.dest / x.S;
    const size_t cell = (size_t)dr * x.R + li;
    if (m.kind == K_KP) {
      const uint32_t po = x.xpoff[cell] + pc[dr];
      for (uint32_t t = 0; t < m.a; ++t) x.spay[po + t] = pay[m.off + t];
      m.off = po - x.xpoff[(size_t)dr * x.R];
      pc[dr] += m.a;
    }
    x.smsg[x.xoff[cell] + c[dr]] = m;
    c[dr]++;
  }
}
// the received records: KnownPeers offsets into the received id blocks, then per destination the delivered
// count, the reply bound and the KnownPeersRequests (k_sp_route's delivered branch)
struct SpRecvBlocks { uint32_t p0[XMAX]; };
__global__ __launch_bounds__(256) void k_sp_recv(SpRoute rt, SpX x, SpRecvBlocks rb) {
  const uint32_t k = blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= rt.M) return;
  Msg* mp = const_cast<Msg*>(rt.msgs) + k;
  const Msg m = *mp;
  if (m.kind == K_KP) mp->off = m.off + rb.p0[m.sender / x.S];
  rt.status[k] = 1;
  atomicAdd(&rt.icnt[m.dest], 1u);
  const uint32_t b = sp_reply_bound(m.kind);
  if (b) atomicAdd(&rt.ebound[m.dest], b);
  if (m.kind == K_KPR) atomicAdd(&rt.kprc[m.dest], 1u);
}
__global__ __launch_bounds__(256) void k_sp_stats_fold(SpDev d) {
  const uint32_t k = blockIdx.x;
  unsigned long long t = 0;
  for (uint32_t q = threadIdx.x; q < SP_ACC; q += blockDim.x) {
    unsigned long long& x = d.sacc[(size_t)q * NSTAT + k];
    t += x; x = 0;
  }
  t = block_sum(t);
  if (threadIdx.x == 0 && t) d.stats[k] += t;
}
__global__ void k_sp_fp_all(SpDev d) {
  const uint32_t i = sp_gid(d);
  if (i < d.hi) (void)sp_fp(d, i);
}
__global__ void k_sp_fp_one(SpDev d, uint32_t i) { if (!threadIdx.x && !blockIdx.x) (void)sp_fp(d, i); }
__global__ void k_sp_mark_dirty(SpDev d) {
  const uint32_t i = sp_gid(d);
  if (i < d.hi) d.dirty[i] = 1;
}

}  // namespace kb
