// kb_tick.h — the tick (src/kaboodle.rs:746-779): maybe_broadcast_join + handle_suspected_peers, the
// row sweep of ping_random_peer fused with the fingerprint fold, target choice + ping_addrs
// (included by kb_sim.hip).
#pragma once
#include "kb_common.h"

namespace kb {

struct BcastSlots { uint32_t* join; uint32_t* nfail; uint32_t* fail; };

// Candidates of handle_suspected_peers (Known && != self, :571-577) in 16-id blocks: member bit set,
// stamp byte >= 2 (not WaitingFor*), not self.
__device__ inline uint32_t cand16(const Dev& d, const uint8_t* rw, const uint32_t* bw, uint32_t i, uint32_t j0) {
  const uint4 v = *reinterpret_cast<const uint4*>(rw + j0);
  const uint32_t m = nzmask4(v.x & 0xFEFEFEFEu) | (nzmask4(v.y & 0xFEFEFEFEu) << 4) |
                     (nzmask4(v.z & 0xFEFEFEFEu) << 8) | (nzmask4(v.w & 0xFEFEFEFEu) << 12);
  uint32_t c = m & ((bw[j0 >> 5] >> (j0 & 16)) & 0xFFFFu);
  if (i >= j0 && i < j0 + 16) c &= ~(1u << (i - j0));
  return c;
}
__device__ __attribute__((always_inline)) inline void tick_a2(const Dev& d, const OutBuf& ob, const BcastSlots& bs, int32_t r,
                                                              uint32_t i, uint32_t l, uint32_t* pr, uint32_t* pp,
                                                              uint32_t* pid) {
  uint32_t n = d.n[i];
  Susp* sl = d.susp + (size_t)i * SLOTS;
  const Susp me = l < SLOTS ? sl[l] : Susp{0, 0, 0, 0};
  const bool occ = l < SLOTS && me.kind != 0;
  const unsigned long long occm = __ballot(occ);
  const unsigned long long tim = __ballot(occ && r - me.since >= PING_TIMEOUT);
  if (!tim) { if (l == 0) bs.nfail[i] = 0; return; }
  const uint32_t nsusp = __popcll(occm);
  const uint32_t m = n - 1 - nsusp;                       // Known && != self (:571-577)
  uint32_t myrank = 0;                                    // ascending-peer order of occupied slots
  for (int k = 0; k < SLOTS; ++k) if (((occm >> k) & 1ull) && bcast(me.peer, k) < me.peer) myrank++;
  uint32_t npick = 0, nind = 0, nrem = 0;
  uint32_t indirect[SLOTS], removed[SLOTS];
  for (uint32_t t = 0; t < nsusp; ++t) {
    const unsigned long long who = __ballot(occ && myrank == t);
    const int k = __ffsll((long long)who) - 1;
    const uint32_t peer = bcast(me.peer, k);
    const int32_t kind = (int32_t)bcast((uint32_t)me.kind, k), since = (int32_t)bcast((uint32_t)me.since, k);
    if (r - since < PING_TIMEOUT) continue;
    if (kind == SK_WFP) {
      const uint32_t kk = m < (uint32_t)NUM_INDIRECT ? m : (uint32_t)NUM_INDIRECT;
      if (kk == 0) { removed[nrem++] = peer; continue; }
      const U4 w = philox(i, (uint32_t)r, (uint32_t)P_INDIRECT << 24, peer, d.k0, d.k1);
      uint32_t pk[3];
      pk[0] = mulhi(w.x, m);
      if (kk > 1) { const uint32_t b = mulhi(w.y, m - 1); pk[1] = b + (b >= pk[0]); }
      if (kk > 2) {
        const uint32_t lo = pk[0] < pk[1] ? pk[0] : pk[1], hi = pk[0] < pk[1] ? pk[1] : pk[0];
        uint32_t c = mulhi(w.z, m - 2);
        if (c >= lo) c++;
        if (c >= hi) c++;
        pk[2] = c;
      }
      if (l == 0) for (uint32_t q = 0; q < kk; ++q) { pr[npick + q] = pk[q]; pp[npick + q] = peer; pid[npick + q] = 0xFFFFFFFFu; }
      npick += kk;
      indirect[nind++] = peer;
    } else {
      removed[nrem++] = peer;
    }
  }
  const uint8_t* rw = row_of(d, i);
  uint32_t oseq = ob.cnt[i];
  if (npick) {                                            // choose_multiple over the candidate list
    // rank -> id for every pick in coalesced passes over the row: lane l takes ids [j0 + 16 l, +16)
    // of each 1024-id pass, four passes' loads in flight; a pass resolves the picks whose rank
    // falls in its candidate range (ranks are in address order, :571-577)
    wait_lds();
    __builtin_amdgcn_wave_barrier();
    const uint32_t* bw = bits_of(d, i);
    uint32_t maxrank = 0;
    for (uint32_t q = 0; q < npick; ++q) maxrank = pr[q] > maxrank ? pr[q] : maxrank;
    uint32_t base = 0;
    for (uint32_t j0 = 0; j0 < d.W && base <= maxrank; j0 += 4096) {
      uint32_t mk[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) { const uint32_t j = j0 + 1024 * u + 16 * l; mk[u] = j < d.W ? cand16(d, rw, bw, i, j) : 0u; }
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const uint32_t j = j0 + 1024 * u + 16 * l;
        const uint32_t pc = __popc(mk[u]), ex = wave_excl(pc), tot = wave_sum(pc);
        for (uint32_t q = 0; q < npick; ++q) {
          const uint32_t rk = pr[q];
          if (rk >= base + ex && rk < base + ex + pc) pid[q] = j + select_in_word(mk[u], rk - base - ex);
        }
        base += tot;
      }
    }
    wait_lds();
    __builtin_amdgcn_wave_barrier();
    for (uint32_t q = 0; q < npick; ++q) emit_msg(ob, d, i, oseq, pid[q], K_PINGREQ, pp[q], 0, 0, 0);
  }
  if (l == 0) {                                           // :631-652
    for (uint32_t q = 0; q < nind; ++q)
      for (int k = 0; k < SLOTS; ++k) if (sl[k].kind && sl[k].peer == indirect[q]) { sl[k].kind = SK_WFIP; sl[k].since = r; }
    Cur* cu = d.cur + (size_t)i * CSLOTS;
    unsigned long long segs = 0;
    for (uint32_t q = 0; q < nrem; ++q) {
      const uint32_t p = removed[q];
      susp_clear(d, i, p);
      mem_clr(d, i, p);
      segs |= seg_bit(d, p);
      n--;
      for (int c = 0; c < CSLOTS; ++c) if (cu[c].used && cu[c].peer == p) cu[c].used = 0;
      bs.fail[(size_t)i * SLOTS + q] = p;
    }
    bs.nfail[i] = nrem;
    if (nrem) { d.n[i] = n; mark(d, i, segs); atomicAdd(&d.stats[S_RMTIMEOUT], nrem); }
    ob.cnt[i] = oseq;
  }
}

// ---- A1 maybe_broadcast_join (:228-251), thread per node; the nodes with a timed-out suspect slot
// (A2's only work) are listed for k_tick_pre, a wave per listed node
__global__ __launch_bounds__(256) void k_tick_scan(Dev d, BcastSlots bs, int32_t r, uint32_t* list) {
  const uint32_t i = d.lo + blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= d.hi) return;
  if (!d.alive[i]) { bs.join[i] = 0; bs.nfail[i] = 0; return; }
  const int32_t lb = d.last_bcast[i];
  uint32_t j = 0;
  if (lb == NONE_ROUND || (r - lb >= REBROADCAST && d.n[i] <= 1)) { j = 1; d.last_bcast[i] = r; }
  bs.join[i] = j;
  const Susp* sl = d.susp + (size_t)i * SLOTS;
  bool tim = false;
#pragma unroll
  for (int k = 0; k < SLOTS; ++k) { const Susp x = sl[k]; tim |= x.kind != 0 && r - x.since >= PING_TIMEOUT; }
  if (!tim) { bs.nfail[i] = 0; return; }
  list[atomicAdd(&d.ctr[C_TICK], 1u)] = i;
}

// ---- A2 handle_suspected_peers (:558-653) for the nodes k_tick_scan listed, one wave per node
// (persistent grid over the list)
__global__ __launch_bounds__(256) void k_tick_pre(Dev d, OutBuf ob, BcastSlots bs, int32_t r, const uint32_t* list) {
  __shared__ uint32_t s_pick_rank[4][SLOTS * 3], s_pick_peer[4][SLOTS * 3], s_pick_id[4][SLOTS * 3];
  const uint32_t wv = threadIdx.x >> 6;
  const uint32_t l = lane();
  const uint32_t nlist = d.ctr[C_TICK];
  for (uint32_t it = blockIdx.x * 4 + wv; it < nlist; it += gridDim.x * 4) {
    tick_a2(d, ob, bs, r, list[it], l, s_pick_rank[wv], s_pick_peer[wv], s_pick_id[wv]);
  }
}


// ================================================================================================
// THE ROW SWEEP (dominant kernel).  ping_random_peer (:655-703) keeps the 5 oldest Known peers by
// (stamp, address rotated to start right after self); generate_fingerprint (:71-83) is refreshed for
// the segments whose membership changed.  Lane = node: a wave sweeps 64 rows over one column split,
// every lane streaming whole 128-byte lines of its own row, all lanes sharing the same half-block
// CRC tables.  Per (node, split) it leaves two partial top-5 lists: ids below the rotation point
// (part A, rot = j - p + C) and from it on (part B, rot = j - p); in id order each part is monotone
// in rot, so an equal stamp seen later never displaces an earlier one (strict < test).
// ================================================================================================
struct SweepOut { uint32_t* part; uint32_t S; };   // part: [C][S][10] keys (b << 24 | rot)

__device__ inline void top5_insert(uint32_t (&k)[5], uint32_t nk) {
#pragma unroll
  for (int s = 0; s < 5; ++s) { if (nk < k[s]) { const uint32_t t = k[s]; k[s] = nk; nk = t; } }
}
__device__ inline uint32_t thr5(const uint32_t (&k)[5]) { return k[4] == 0xFFFFFFFFu ? 256u : (k[4] >> 24); }

typedef unsigned short u16x2 __attribute__((ext_vector_type(2)));

// smallest (byte - 2) over the 16 bytes of x, computed on 16-bit lanes with packed ops (bytes 0 and 1
// wrap to >= 0xFFFE): a byte b can enter a top-5 list with threshold T only if this is < T - 2
__device__ inline uint32_t min_stamp16(const uint4& x) {
  const u16x2 two = {2, 2};
  u16x2 mn = {0xFFFF, 0xFFFF};
  const uint32_t w[4] = {x.x, x.y, x.z, x.w};
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    mn = __builtin_elementwise_min(mn, __builtin_bit_cast(u16x2, w[k] & 0x00FF00FFu) - two);
    mn = __builtin_elementwise_min(mn, __builtin_bit_cast(u16x2, (w[k] >> 8) & 0x00FF00FFu) - two);
  }
  return mn.x < mn.y ? mn.x : mn.y;
}

// One 128-id step of one lane's row, software-pipelined: the loads of step k+1 are issued before
// step k is processed.  Stamp bytes (128 B, plus the 16 B of member bits) are loaded while either
// part's list can still change: a part is final once it holds five ancient (minimum) stamps, since
// later ids of the part have larger rot.  Member bits are loaded alone to refold a stale checkpoint.
struct StepIn { uint4 v[8]; uint4 mb; };

__device__ inline bool step_need(const Dev& d, const uint32_t (&A)[5], const uint32_t (&B)[5], uint32_t p, uint32_t col) {
  return !(d.ablate & 2) && ((thr5(A) > ST_ANCIENT && col < p) || (thr5(B) > ST_ANCIENT && col + 128 > p));
}

template <bool FOLD>
__device__ __attribute__((always_inline)) inline void step_load(const uint8_t* rw, const uint32_t* bw, uint32_t col,
                                                                bool need, StepIn& s, uint32_t& nbytes) {
  if (need) {
#pragma unroll
    for (int q = 0; q < 8; ++q) s.v[q] = *reinterpret_cast<const uint4*>(rw + col + 16 * q);
    nbytes += 128;
  }
  if (FOLD || need) { s.mb = *reinterpret_cast<const uint4*>(bw + (col >> 5)); nbytes += 16; }
}

// A packed-u16 filter rejects 16-byte groups with no stamp below the current threshold; surviving
// groups are examined byte by byte against the member bits (strict <: within a part ids arrive in
// increasing rot, so an equal stamp seen later never displaces an earlier one).
// The fold's 16 table reads are issued before the next step's prefetch: vmcnt retires in order,
// so waiting for them must not also wait for the prefetch.
template <bool FOLD>
__device__ __attribute__((always_inline)) inline void fold_fetch(const Dev& d, const StepIn& s, uint32_t col,
                                                                 uint32_t (&hv)[16]) {
  if (!FOLD) return;
  const uint32_t mw[4] = {s.mb.x, s.mb.y, s.mb.z, s.mb.w};
  const uint32_t* ht = d.htab + (size_t)(col >> 3) * 256;
#pragma unroll
  for (int h = 0; h < 16; ++h) hv[h] = ht[h * 256 + ((mw[h >> 2] >> (8 * (h & 3))) & 0xFFu)];   // entry 0 is 0
}

// A packed-u16 filter rejects 16-byte groups with no stamp below the current threshold; surviving
// groups are examined byte by byte against the member bits (strict <: within a part ids arrive in
// increasing rot, so an equal stamp seen later never displaces an earlier one).
template <bool FOLD>
__device__ __attribute__((always_inline)) inline void step_proc(const Dev& d, const uint32_t* zb, const StepIn& s,
                                                                const uint32_t (&hv)[16], bool loaded, uint32_t i,
                                                                uint32_t p, uint32_t col, uint32_t (&A)[5],
                                                                uint32_t (&B)[5], uint32_t& raw, uint32_t& cnt) {
  if (FOLD) {
    const uint32_t mw[4] = {s.mb.x, s.mb.y, s.mb.z, s.mb.w};
#pragma unroll
    for (int h = 0; h < 16; ++h) {
      const uint32_t c = __popc((mw[h >> 2] >> (8 * (h & 3))) & 0xFFu);   // Z^0 table is the identity
      raw = mulzb(zb, raw, c) ^ hv[h];
      cnt += c;
    }
  }
  if (!loaded) return;
  const uint32_t C = d.C;
#pragma unroll
  for (int q = 0; q < 8; ++q) {
    // thresholds are re-read per 16-id group: once a part holds five ancient stamps (typically
    // within the first group of a step) the rest of the step is rejected by the packed filter
    const uint32_t TA = thr5(A), TB = thr5(B);
    const bool needA = TA > ST_ANCIENT && col < p, needB = TB > ST_ANCIENT && col + 128 > p;
    if (!(needA || needB)) break;
    const uint32_t T = (needA && TA > (needB ? TB : 0u)) ? TA : TB;   // the larger relevant threshold
    if (min_stamp16(s.v[q]) >= T - 2) continue;
    const uint32_t mwq = (q >> 1) == 0 ? s.mb.x : ((q >> 1) == 1 ? s.mb.y : ((q >> 1) == 2 ? s.mb.z : s.mb.w));
    uint32_t cm = (nzmask4(s.v[q].x & 0xFEFEFEFEu) | (nzmask4(s.v[q].y & 0xFEFEFEFEu) << 4) |
                   (nzmask4(s.v[q].z & 0xFEFEFEFEu) << 8) | (nzmask4(s.v[q].w & 0xFEFEFEFEu) << 12)) &
                  ((mwq >> (16 * (q & 1))) & 0xFFFFu);
    while (cm) {
      const uint32_t t = __ffs(cm) - 1;
      cm &= cm - 1;
      const uint32_t word = (t & 8) ? ((t & 4) ? s.v[q].w : s.v[q].z) : ((t & 4) ? s.v[q].y : s.v[q].x);
      const uint32_t b = (word >> (8 * (t & 3))) & 0xFFu;
      const uint32_t j = col + 16 * q + t;
      if (j == i) continue;
      if (j >= p) { if (b < thr5(B)) top5_insert(B, (b << 24) | (j - p)); }
      else if (b < thr5(A)) top5_insert(A, (b << 24) | (j + C - p));
    }
  }
}

template <bool FOLD>
__device__ __attribute__((always_inline)) inline void sweep_segment(const Dev& d, const uint32_t* zb, const uint8_t* rw,
                                                                    const uint32_t* bw, uint32_t i, uint32_t p,
                                                                    uint32_t c0, uint32_t c1, uint32_t (&A)[5],
                                                                    uint32_t (&B)[5], uint32_t& raw, uint32_t& cnt,
                                                                    uint32_t& nbytes) {
  if (c0 >= c1) return;
  // Measured: prefetching only the bits (stamps loaded in-step) fits 4 waves/SIMD and is 3 % faster,
  // but the extra waves evict each row's bit line between its 8 steps: HBM traffic 1.71x the
  // algorithmic bytes instead of 1.14x.  The full prefetch is kept.
  StepIn cur;
  bool need_cur = step_need(d, A, B, p, c0);
  step_load<FOLD>(rw, bw, c0, need_cur, cur, nbytes);
  for (uint32_t col = c0; col < c1; col += 128) {
    uint32_t hv[16];
    fold_fetch<FOLD>(d, cur, col, hv);
    StepIn nxt;
    // thresholds only fall, so the need computed before processing this step is a superset
    const bool need_nxt = col + 128 < c1 && step_need(d, A, B, p, col + 128);
    if (col + 128 < c1) step_load<FOLD>(rw, bw, col + 128, need_nxt, nxt, nbytes);
    step_proc<FOLD>(d, zb, cur, hv, need_cur, i, p, col, A, B, raw, cnt);
    cur = nxt;
    need_cur = need_nxt;
  }
}

__global__ __launch_bounds__(256) void k_sweep(Dev d, SweepOut so) {
  __shared__ uint32_t zb[ZB];
  load_zbtab(d, zb);
  // XCD-aware: workgroups are dealt round-robin to the 8 XCDs, so split s = blockIdx % S keeps each
  // XCD on 1/min(S,8) of the columns and its slice of the half-block CRC tables resident in its L2.
  const uint32_t S = so.S;
  const uint32_t s = blockIdx.x % S;
  const uint32_t g = (blockIdx.x / S) * 4 + (threadIdx.x >> 6);
  const uint32_t i0 = d.lo + g * 64 + lane();
  const bool act = i0 < d.hi && d.alive[i0];
  // the ballot is taken once with the full wave active: inside the select below it would run
  // under the idle lanes' exec mask only and see no live lane
  const unsigned long long actm = __ballot(act);
  if (!actm) return;
  const uint32_t shadow = d.lo + g * 64 + (uint32_t)(__ffsll((long long)actm) - 1);
  const uint32_t i = act ? i0 : shadow;                 // idle lanes shadow a live one
  const uint8_t* rw = row_of(d, i);
  const uint32_t* bw = bits_of(d, i);
  const uint32_t C = d.C;
  const uint32_t p = (i + 1 == C) ? 0 : i + 1;
  const unsigned long long sd = (d.uniform && act) ? d.sdirty[i] : 0ull;
  uint32_t A[5], B[5];
#pragma unroll
  for (int k = 0; k < 5; ++k) { A[k] = 0xFFFFFFFFu; B[k] = 0xFFFFFFFFu; }
  uint32_t nbytes = 0;
  const uint32_t spp = NSEG / S;
  unsigned long long folded = 0;
  for (uint32_t k = s * spp; k < (s + 1) * spp; ++k) {
    const uint32_t c0 = k * d.SEGW, c1 = c0 + d.SEGW < C ? c0 + d.SEGW : ((C + 127) & ~127u);
    uint32_t raw = 0, cnt = 0;
    const bool mine = ((sd >> k) & 1ull) && !(d.ablate & 1);
    if (__ballot(mine)) {                 // wave-uniform: one pass for the whole wave
      sweep_segment<true>(d, zb, rw, bw, i, p, c0, c1, A, B, raw, cnt, nbytes);
      if (mine) { d.segp[(size_t)i * NSEG + k] = make_uint2(raw, cnt); folded |= 1ull << k; }
    } else {
      const bool need = (thr5(A) > ST_ANCIENT && c0 < p) || (thr5(B) > ST_ANCIENT && c1 > p);
      if (!__ballot(act && need)) continue;   // no list of this wave can change in this segment
      sweep_segment<false>(d, zb, rw, bw, i, p, c0, c1, A, B, raw, cnt, nbytes);
    }
  }
  const uint32_t wb = wave_sum(act ? nbytes : 0u);
  if (lane() == 0 && wb) atomicAdd(&d.stats[S_SWEEPB], (unsigned long long)wb);
  if (!act) return;
  if (folded) atomicAnd(&d.sdirty[i], ~folded);
  uint32_t* out = so.part + ((size_t)i * S + s) * 10;
#pragma unroll
  for (int k = 0; k < 5; ++k) { out[k] = A[k]; out[5 + k] = B[k]; }
}

// ---- pick the ping target (one of the oldest 5), WaitingForPing(now), Ping; ping_addrs (:550-556);
// ---- refresh the fingerprint from the checkpoints; agreement with the running set.  Thread per node.
__global__ void k_tick_post(Dev d, SweepOut so, OutBuf ob, int32_t r) {
  const uint32_t i = d.lo + blockIdx.x * blockDim.x + threadIdx.x;
  unsigned long long agree = 0;
  if (i < d.hi && d.alive[i]) {
    const uint32_t C = d.C, S = so.S;
    const uint32_t p = (i + 1 == C) ? 0 : i + 1;
    uint32_t k5[5] = {0xFFFFFFFFu, 0xFFFFFFFFu, 0xFFFFFFFFu, 0xFFFFFFFFu, 0xFFFFFFFFu};
    const uint2* part = reinterpret_cast<const uint2*>(so.part + (size_t)i * S * 10);   // S * 10 is even
#pragma unroll 8
    for (uint32_t q = 0; q < S * 5; ++q) {
      const uint2 x = part[q];
      if (x.x < k5[4]) top5_insert(k5, x.x);
      if (x.y < k5[4]) top5_insert(k5, x.y);
    }
    uint32_t nc = 0;
    while (nc < 5 && k5[nc] != 0xFFFFFFFFu) nc++;
    uint32_t oseq = ob.cnt[i];
    if (nc) {
      const uint32_t u = philox(i, (uint32_t)r, (uint32_t)P_PING << 24, 0, d.k0, d.k1).x;
      const uint32_t rot = k5[mulhi(u, nc)] & 0xFFFFFFu;
      const uint32_t t = rot + p >= C ? rot + p - C : rot + p;
      Susp* sl = d.susp + (size_t)i * SLOTS;
      int k = 0;
      while (k < SLOTS && sl[k].kind) ++k;
      if (k == SLOTS) set_err(d, DERR_SLOTS);
      else { sl[k].peer = t; sl[k].kind = SK_WFP; sl[k].since = r; }
      uint8_t* tb = row_of(d, i) + t;
      if (*tb == enc(r, r)) {            // stamped Known(now) earlier this round: retire its log entry
        const uint32_t e = log_entry(t, r), fe = d.flog_n[i];
        for (uint32_t q = d.fstart[(size_t)i * 16 + ((uint32_t)r & 15u)]; q < fe; ++q) {
          uint32_t& slot = d.flog[(size_t)i * LOGCAP + (q & (LOGCAP - 1))];
          if (slot == e) slot = LOG_INVALID;
        }
      }
      *tb = ST_SUSPECT;
      if (oseq >= ob.cap[i]) set_err(d, DERR_OUTBOX);
      else ob.msgs[ob.off[i] + oseq] = Msg{t, i, oseq, K_PING, 0, 0, 0, 0};
      oseq++;
    }
    const uint32_t pn = d.paq_n[i];
    for (uint32_t q = 0; q < pn; ++q) {
      const uint32_t t = d.paq[(size_t)i * PAQ + q];
      if (oseq >= ob.cap[i]) set_err(d, DERR_OUTBOX);
      else ob.msgs[ob.off[i] + oseq] = Msg{t, i, oseq, K_PING, 0, 0, 0, 0};
      oseq++;
    }
    d.paq_n[i] = 0;
    ob.cnt[i] = oseq;
    if (d.dirty[i]) {
      if (!d.uniform && d.sdirty[i]) {            // non-uniform identities: refold stale checkpoints here
        unsigned long long sd = d.sdirty[i];
        while (sd) { const int k = __ffsll((long long)sd) - 1; sd &= sd - 1;
                     d.segp[(size_t)i * NSEG + k] = fold_segment(d, nullptr, i, k); }
        d.sdirty[i] = 0;
      }
      d.fp[i] = thread_fp(d, i);
      d.dirty[i] = 0;
    }
    agree = d.fp[i] == d.truefp[0];
  }
  const unsigned long long t = block_sum(agree);
  if (threadIdx.x == 0 && t) atomicAdd(&d.ctr[C_AGREE], (uint32_t)t);
}

__global__ void k_bcast_write(Dev d, BcastSlots bs, const uint32_t* join_off, const uint32_t* fail_off, BCast* bjoin,
                              BCast* bfail) {
  const uint32_t i = d.lo + blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= d.hi) return;
  uint32_t bseq = 0;
  if (bs.join[i]) bjoin[join_off[i]] = BCast{i, i, bseq++, 0};
  const uint32_t nfl = bs.nfail[i];
  for (uint32_t q = 0; q < nfl; ++q) bfail[fail_off[i] + q] = BCast{i, bs.fail[(size_t)i * SLOTS + q], bseq++, 0};
}

__global__ void k_round_end(Dev d, int32_t r) {
  if (threadIdx.x || blockIdx.x) return;
  const uint32_t a = d.ctr[C_AGREE], al = d.ctr[C_ALIVE];
  d.ctr[C_LASTAGREE] = a; d.ctr[C_LASTALIVE] = al;
  if (al && a == al) {
    if ((int32_t)d.ctr[C_FIRSTCONV] < 0) d.ctr[C_FIRSTCONV] = (uint32_t)r;
    d.ctr[C_LASTCONV] = (uint32_t)r;
  }
  d.ctr[C_AGREE] = 0; d.ctr[C_ALIVE] = 0; d.ctr[C_TICK] = 0;
}

}  // namespace kb
