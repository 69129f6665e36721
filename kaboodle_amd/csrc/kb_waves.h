// kb_waves.h — unicast delivery waves: routing, the KnownPeers group (message-parallel), and the
// per-node in-order handler for every other message kind (src/kaboodle.rs:394-548).
#pragma once
#include "kb_common.h"

namespace kb {

struct WaveCtl {
  uint8_t* status;        // per outbox slot: 0 dropped, 1 delivered (in-order kinds), 2 delivered KnownPeers
  uint32_t* cnt1; uint32_t* bnd; uint32_t* bpay; uint32_t* cursor;   // per destination: in-order inbox
  uint32_t* kcnt; uint32_t* kpay; uint32_t* kcur; uint32_t* koff;    // per destination: KnownPeers group
  uint32_t* in_off; uint32_t* inbox; uint32_t* active;
  uint32_t* kin;          // KnownPeers deliveries grouped by destination (koff / kcnt)
  uint32_t msg_cap; uint32_t pay_cap;
};

// The per-destination counters of a wave are zero outside the wave's active nodes.  Whoever handles
// an active node last in the wave puts them back to zero: k_proc_fast for the nodes it finishes (or
// that have no in-order delivery), k_proc for the rest.  No clearing launch per wave.
__device__ inline void wave_ctr_clear(const WaveCtl& wc, uint32_t i) {
  wc.cnt1[i] = 0; wc.bnd[i] = 0; wc.bpay[i] = 0; wc.cursor[i] = 0;
  wc.kcnt[i] = 0; wc.kpay[i] = 0; wc.kcur[i] = 0;
}

// messages a handler may emit per delivered message (next-wave outbox reservation)
__device__ inline uint32_t out_bound(uint32_t kind) {
  return kind == K_ACK ? NOBS + 1 : (kind == K_KPR ? 2u : (kind == K_KP ? 0u : 1u));
}

// Message-parallel walk over the outboxes of 64 consecutive senders per wave: lane k of each
// iteration takes the k-th message of the 64 regions concatenated, so one sender with hundreds of
// messages (a popular ping target's Acks) spreads over the wave instead of serialising a thread.
struct SenderSpan {
  uint32_t total;
  __device__ void owner(const uint32_t* ex, uint32_t k, uint32_t& j, uint32_t& q) const {
    uint32_t lo = 0, hi = 64;                   // largest j with ex[j] <= k
    while (hi - lo > 1) { const uint32_t mid = (lo + hi) >> 1; if (ex[mid] <= k) lo = mid; else hi = mid; }
    j = lo; q = k - ex[lo];
  }
};

// Per-workgroup aggregation of the KnownPeers counters: wave 0 carries tens of thousands of Join
// responses addressed to the round's few dozen joiners, and one global atomic per message on those few
// counters serialises in the memory system.  A workgroup first sums its messages per destination in a
// small LDS hash table, then adds each sum once; a destination that finds no free slot in KAGG_PROBE
// probes goes to the global counters directly.
constexpr uint32_t KAGG = 256, KAGG_PROBE = 8, KAGG_EMPTY = 0xFFFFFFFFu;
__device__ inline uint32_t kagg_slot(uint32_t x) { return (x * 0x9E3779B1u) >> 24; }   // 8 bits: KAGG slots
// slot of dest (inserted when `insert`), or KAGG when it is not (cannot be) in the table
__device__ inline uint32_t kagg_find(uint32_t* kd, uint32_t dest, bool insert) {
  uint32_t h = kagg_slot(dest);
  for (uint32_t p = 0; p < KAGG_PROBE; ++p, h = (h + 1) & (KAGG - 1)) {
    const uint32_t cur = insert ? atomicCAS(&kd[h], KAGG_EMPTY, dest) : kd[h];
    if (cur == dest || (insert && cur == KAGG_EMPTY)) return h;
    if (cur == KAGG_EMPTY) return KAGG;
  }
  return KAGG;
}

// delivery decisions for every message of the wave: dead receiver, partition, loss (Philox keyed on
// the message), else delivered; counts per destination.
__global__ __launch_bounds__(256) void k_route(Dev d, OutBuf ob, WaveCtl wc, int32_t r_arg, uint32_t w, int last) {
  const int32_t r = round_of(d, r_arg);
  __shared__ uint32_t s_ex[4][64], s_base[4][64];
  __shared__ uint32_t s_kd[KAGG], s_kc[KAGG], s_kp[KAGG];
  const uint32_t wv = threadIdx.x >> 6, l = lane();
  s_kd[threadIdx.x] = KAGG_EMPTY; s_kc[threadIdx.x] = 0; s_kp[threadIdx.x] = 0;   // blockDim == KAGG
  __syncthreads();
  const uint32_t i = d.lo + blockIdx.x * blockDim.x + threadIdx.x;
  unsigned long long ks[5] = {0, 0, 0, 0, 0}, dead = 0, part = 0, loss = 0, win = 0, kpids = 0, xp = 0;
  const uint32_t cnt = i < d.hi ? ob.cnt[i] : 0;
  s_ex[wv][l] = wave_excl(cnt);
  s_base[wv][l] = i < d.hi ? ob.off[i] : 0;
  const uint32_t T = wave_sum(cnt);
  wait_lds();
  __builtin_amdgcn_wave_barrier();
  const SenderSpan sp{T};
  for (uint32_t k = l; k < T; k += 64) {
    uint32_t j, q;
    sp.owner(s_ex[wv], k, j, q);
    const uint32_t g = s_base[wv][j] + q;
    const Msg m = ob.msgs[g];
    ks[m.kind < 5 ? m.kind : 0]++;
    if (m.kind == K_KP) kpids += m.a;
    uint8_t st = 0;
    if (last) win++;
    else if (!d.alive[m.dest]) {
      if (d.ext[m.dest]) {                                             // a partition cuts it off too
        if (part_blocks(d, r, m.sender, m.dest)) part++;
        else { export_rec(d.ctr, d.xrec, d.xrec_cap, d.xids, d.xids_cap, m, ob.pay, r, w); xp++; }
      }
      else dead++;
    }
    else if (part_blocks(d, r, m.sender, m.dest)) part++;
    else if (faults(d, r) && d.loss_thr &&
             philox(m.sender, (uint32_t)r, ((uint32_t)P_LOSS << 24) | w, m.seq, d.k0, d.k1).x < d.loss_thr) loss++;
    else if (m.kind == K_KP) {
      st = 2;
      const uint32_t h = kagg_find(s_kd, m.dest, true);
      if (h < KAGG) { atomicAdd(&s_kc[h], 1u); if (m.a) atomicAdd(&s_kp[h], m.a); }
      else { atomicAdd(&wc.kcnt[m.dest], 1u); if (m.a) atomicAdd(&wc.kpay[m.dest], m.a); }
    } else {
      st = 1;
      atomicAdd(&wc.cnt1[m.dest], 1u);
      atomicAdd(&wc.bnd[m.dest], out_bound(m.kind));
      if (m.kind == K_KPR) atomicAdd(&wc.bpay[m.dest], d.paybound);
    }
    if (!last) wc.status[g] = st;
  }
  __syncthreads();
  if (s_kd[threadIdx.x] != KAGG_EMPTY) {
    const uint32_t x = s_kd[threadIdx.x];
    atomicAdd(&wc.kcnt[x], s_kc[threadIdx.x]);
    if (s_kp[threadIdx.x]) atomicAdd(&wc.kpay[x], s_kp[threadIdx.x]);
  }
  {
    const int idx[11] = {S_PING, S_PING + 1, S_PING + 2, S_PING + 3, S_PING + 4, S_DEAD, S_PART, S_LOSS, S_WINDOW, S_KPIDS,
                         S_EXPORT};
    const unsigned long long v[11] = {ks[0], ks[1], ks[2], ks[3], ks[4], dead, part, loss, win, kpids, xp};
    stat_add_n(d, idx, v);
  }
}

// ---- KnownPeersRequest oversize probe (:473-512, Q3) -----------------------------------------------
// A KPR reply lists every fresh entry (Known, stamped within SHARE_AGE, not self, not the requester);
// above capk entries it is lost at the receiver, so only its size matters.  The fresh set only grows
// while a round's waves run (stamps rise to now; removals happen before the waves), so counting it
// once, as it stands when the wave starts, proves every reply of the rest of the round oversize as
// soon as the count exceeds capk + 1 (one requester excluded): kpr_big = r, and k_proc's KPR handler
// takes its constant-time path.  A wave per node with a KPR delivery this wave, all of its log window
// in flight at once (up to 8 x 64 entries per step), in extra workgroups of the k_scatter launch: no
// kernel writes a row while the inboxes are built (a row read while a prologue moves a stamp to
// Known(now) and logs it could count that peer twice), and the proof is in place before the fast
// handlers of k_sortfast decide.  The KnownPeers prologues of k_kp in between only add fresh entries.
constexpr uint32_t KB_PROBE_GROUPS = 1024;
constexpr uint32_t PROBE_GROUPS = KB_PROBE_GROUPS;   // workgroups of the scatter launch that run the probe (1024: 3.00
                                                     // -> 2.93 ms against 512; 2048 and 4096 the same, profiles/r04kn*)
__device__ __attribute__((always_inline)) inline void kpr_probe(const Dev& d, const WaveCtl& wc, int32_t r, uint32_t bid,
                                                               uint32_t nblk) {
  const uint32_t nact = d.ctr[C_ACTIVE];
  const uint32_t nwv = blockDim.x >> 6, wv = threadIdx.x >> 6, l = lane();
  for (uint32_t it = bid * nwv + wv; it < nact; it += nblk * nwv) {
    const uint32_t i = wc.active[it];
    if (!wc.bpay[i] || d.kpr_big[i] == r) continue;  // wave-uniform: no KPR, or already proven
    const uint8_t* rw = row_of(d, i);
    const uint32_t* bw = bits_of(d, i);
    const uint32_t fn = d.flog_n[i], ws = log_window_start(d, i, r);
    const uint32_t k_lo = fn - ws <= LOGCAP ? ws : fn - LOGCAP;
    uint32_t total = 0;
    constexpr int PB = 8;
    for (uint32_t k0 = k_lo; k0 < fn && total <= d.capk + 1; k0 += 64 * PB) {
      uint32_t ev[PB], wv4[PB], bv[PB];
#pragma unroll
      for (int u = 0; u < PB; ++u) {
        const uint32_t k = k0 + 64u * u + l;
        ev[u] = k < fn ? d.flog[(size_t)i * LOGCAP + (k & (LOGCAP - 1))] : LOG_INVALID;
      }
#pragma unroll
      for (int u = 0; u < PB; ++u) {
        const uint32_t j = ev[u] == LOG_INVALID ? i : ev[u] >> 8;
        wv4[u] = bw[j >> 5];
        bv[u] = rw[j];
      }
      uint32_t c = 0;
#pragma unroll
      for (int u = 0; u < PB; ++u) {
        const uint32_t e = ev[u], j = e >> 8;
        c += e != LOG_INVALID && j != i && r - log_round(e, r) < SHARE_AGE && ((wv4[u] >> (j & 31)) & 1u) &&
             bv[u] == enc(log_round(e, r), r);
      }
      total += wave_sum(c);
    }
    if (total > d.capk + 1 && l == 0) d.kpr_big[i] = r;
  }
}


// KnownPeers records are placed in two passes (their order within a destination's group is free: the
// group commutes): count per destination in LDS, reserve each destination's block once,
// then place; in-order records take their global cursor directly (in-order inboxes are sorted later).
__global__ __launch_bounds__(256) void k_scatter(Dev d, OutBuf ob, WaveCtl wc, int32_t r_arg, uint32_t nscat) {
  if (blockIdx.x >= nscat) {                           // the KPR oversize probe (workgroups past the scatter's)
    if (d.uniform) kpr_probe(d, wc, round_of(d, r_arg), blockIdx.x - nscat, gridDim.x - nscat);
    return;
  }
  __shared__ uint32_t s_ex[4][64], s_base[4][64];
  __shared__ uint32_t s_kd[KAGG], s_kc[KAGG], s_kb[KAGG];
  const uint32_t wv = threadIdx.x >> 6, l = lane();
  const uint32_t i = d.lo + blockIdx.x * blockDim.x + threadIdx.x;
  s_kd[threadIdx.x] = KAGG_EMPTY; s_kc[threadIdx.x] = 0;   // blockDim == KAGG
  const uint32_t cnt = i < d.hi ? ob.cnt[i] : 0;
  s_ex[wv][l] = wave_excl(cnt);
  s_base[wv][l] = i < d.hi ? ob.off[i] : 0;
  const uint32_t T = wave_sum(cnt);
  __syncthreads();
  const SenderSpan sp{T};
  bool anykp = false;
  for (uint32_t k = l; k < T; k += 64) {
    uint32_t j, q;
    sp.owner(s_ex[wv], k, j, q);
    const uint32_t g = s_base[wv][j] + q;
    const uint8_t st = wc.status[g];
    if (!st) continue;
    const uint32_t dst = ob.msgs[g].dest;
    if (st == 1) wc.inbox[wc.in_off[dst] + atomicAdd(&wc.cursor[dst], 1u)] = g;
    else { const uint32_t h = kagg_find(s_kd, dst, true); if (h < KAGG) atomicAdd(&s_kc[h], 1u); anykp = true; }
  }
  if (!__syncthreads_or(anykp)) return;
  if (s_kd[threadIdx.x] != KAGG_EMPTY) { s_kb[threadIdx.x] = atomicAdd(&wc.kcur[s_kd[threadIdx.x]], s_kc[threadIdx.x]); s_kc[threadIdx.x] = 0; }
  __syncthreads();
  for (uint32_t k = l; k < T; k += 64) {
    uint32_t j, q;
    sp.owner(s_ex[wv], k, j, q);
    const uint32_t g = s_base[wv][j] + q;
    if (wc.status[g] != 2) continue;
    const uint32_t dst = ob.msgs[g].dest;
    const uint32_t h = kagg_find(s_kd, dst, false);
    const uint32_t pos = h < KAGG ? s_kb[h] + atomicAdd(&s_kc[h], 1u) : atomicAdd(&wc.kcur[dst], 1u);
    wc.kin[wc.koff[dst] + pos] = g;
  }
}

// ================================================================================================
// Sharded waves.  The sender's shard decides every delivery (dead receiver,
// partition, loss: the same Philox draws as the unsharded path, keyed on the message) and packs the
// delivered records per destination shard, each block in (sender, seq) order, KnownPeers ids with
// them.  After the all-to-all-v the receiver holds one flat buffer ordered by (source shard, sender,
// seq) = (sender, seq): the canonical inbox order of the unsharded path, so the handlers below run
// unchanged on it.
// ================================================================================================
constexpr uint32_t XMAX = 8;        // shards per mesh
constexpr uint32_t UCAP = 1024;     // joiners of one round whose Join responses travel as a union (the rest as lists)
struct XState {
  uint32_t world, R, S;             // shards, local rows, rows per shard
  uint32_t RS;                      // R + 1: per destination shard the senders' slots, then the unions' slot
  uint8_t* ostatus;                 // per outbox slot: 1 = delivered
  uint32_t* xcnt; uint32_t* xpay;   // [world][RS] delivered records / payload ids per (dest shard, sender | unions)
  uint32_t* xoff; uint32_t* xpoff;  // exclusive scans of xcnt / xpay (flattened) = send positions
  uint32_t* xb;                     // [2 * world] records, payload ids sent to each shard
  Msg* smsg; uint32_t* spay;        // send buffers
  // the Join-response union (wave 0): joiner slot of every id (~0: none), one bitmap of NWW words per slot, and
  // whether this shard delivered anything to the slot's joiner; bjoin = the round's Join list (slot = entry)
  uint32_t* jslot; uint32_t* ubits; uint32_t* uany; const BCast* bjoin;
  uint32_t nju, NWW, uon;           // slots in use, words per bitmap, unions on (wave 0 of a round with joiners)
};
// the union slot a delivered record's ids go to, or ~0 (they travel with the record)
__device__ inline uint32_t x_union_slot(const XState& x, const Msg& m) {
  return (x.uon && m.kind == K_KP && m.a) ? x.jslot[m.dest] : 0xFFFFFFFFu;
}

__global__ __launch_bounds__(256) void k_route_x(Dev d, OutBuf ob, XState x, int32_t r, uint32_t w, int last) {
  __shared__ uint32_t s_ex[4][64], s_base[4][64];
  const uint32_t wv = threadIdx.x >> 6, l = lane();
  const uint32_t i = d.lo + blockIdx.x * blockDim.x + threadIdx.x;
  unsigned long long ks[5] = {0, 0, 0, 0, 0}, dead = 0, part = 0, loss = 0, win = 0, kpids = 0, xp = 0;
  const uint32_t cnt = i < d.hi ? ob.cnt[i] : 0;
  s_ex[wv][l] = wave_excl(cnt);
  s_base[wv][l] = i < d.hi ? ob.off[i] : 0;
  const uint32_t T = wave_sum(cnt);
  wait_lds();
  __builtin_amdgcn_wave_barrier();
  const SenderSpan sp{T};
  for (uint32_t k = l; k < T; k += 64) {
    uint32_t j, q;
    sp.owner(s_ex[wv], k, j, q);
    const uint32_t g = s_base[wv][j] + q;
    const Msg m = ob.msgs[g];
    ks[m.kind < 5 ? m.kind : 0]++;
    if (m.kind == K_KP) kpids += m.a;
    uint8_t st = 0;
    if (last) win++;
    else if (!d.alive[m.dest]) {
      if (d.ext[m.dest]) {                                             // the sender's shard exports (partition: dropped)
        if (part_blocks(d, r, m.sender, m.dest)) part++;
        else { export_rec(d.ctr, d.xrec, d.xrec_cap, d.xids, d.xids_cap, m, ob.pay, r, w); xp++; }
      }
      else dead++;
    }
    else if (part_blocks(d, r, m.sender, m.dest)) part++;
    else if (faults(d, r) && d.loss_thr &&
             philox(m.sender, (uint32_t)r, ((uint32_t)P_LOSS << 24) | w, m.seq, d.k0, d.k1).x < d.loss_thr) loss++;
    else {
      st = 1;
      const uint32_t slot = (m.dest / x.S) * x.RS + (m.sender - d.lo);
      atomicAdd(&x.xcnt[slot], 1u);
      const uint32_t e = x_union_slot(x, m);
      if (e != 0xFFFFFFFFu) x.uany[e] = 1u;                           // its ids go to the joiner's union
      else if (m.kind == K_KP && m.a) atomicAdd(&x.xpay[slot], m.a);
    }
    if (!last) x.ostatus[g] = st;
  }
  {
    const int idx[11] = {S_PING, S_PING + 1, S_PING + 2, S_PING + 3, S_PING + 4, S_DEAD, S_PART, S_LOSS, S_WINDOW, S_KPIDS,
                         S_EXPORT};
    const unsigned long long v[11] = {ks[0], ks[1], ks[2], ks[3], ks[4], dead, part, loss, win, kpids, xp};
    stat_add_n(d, idx, v);
  }
}

// records / payload ids this shard sends to each shard (from the scans' block starts and totals)
__global__ void k_xbound(XState x, const uint32_t* tot) {
  const uint32_t k = threadIdx.x;
  if (k >= x.world) return;
  const uint32_t a1 = k + 1 < x.world ? x.xoff[(k + 1) * x.RS] : tot[0];
  const uint32_t p1 = k + 1 < x.world ? x.xpoff[(k + 1) * x.RS] : tot[1];
  x.xb[k] = a1 - x.xoff[k * x.RS];
  x.xb[x.world + k] = p1 - x.xpoff[k * x.RS];
}

// ---- The Join-response union.  In wave 0 of a sharded round every delivered KnownPeers record
// whose destination is one of the round's joiners (a Join sender, slot e < UCAP) travels without its ids: they
// are ORed into one bitmap per joiner, sent once per (source shard, joiner) as a K_KPU record in the unions' slot
// of the joiner's shard.  The joiner's KnownPeers group inserts every listed id it does not know; those arms
// commute with each other and with the group's prologues (src/kaboodle.rs:448-472), so one arm
// over the union leaves the same row as the lists' arms, and every record keeps its prologue.  A joiner's ≈ 650
// responses of 567 ids (≈ 1.5 MB) become at most one bitmap of W/8 bytes per source shard.
__global__ void k_union_slots(XState x) {   // the round's slots: joiner -> slot, no union yet
  const uint32_t e = blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= x.nju) return;
  x.uany[e] = 0u;
  x.jslot[x.bjoin[e].sender] = e;
}
__global__ void k_union_count(XState x) {   // one record + one bitmap per union, in the unions' slot of its shard
  for (uint32_t e = threadIdx.x; e < x.nju; e += blockDim.x) {
    if (!x.uany[e]) continue;
    const uint32_t k = x.bjoin[e].sender / x.S;
    atomicAdd(&x.xcnt[k * x.RS + x.R], 1u);
    atomicAdd(&x.xpay[k * x.RS + x.R], x.NWW);
  }
}
// after k_pack: a workgroup per slot writes its union (position: the slots before it that go to the same shard)
// and clears the bitmap and the joiner's slot for the next round
__global__ __launch_bounds__(256) void k_union_pack(XState x) {
  __shared__ uint32_t s_c[4];
  const uint32_t e = blockIdx.x, t = threadIdx.x;
  const uint32_t jid = x.bjoin[e].sender, k = jid / x.S;
  const bool any = x.uany[e] != 0u;
  uint32_t c = 0;
  if (any)
    for (uint32_t f = t; f < e; f += blockDim.x) c += (x.uany[f] && x.bjoin[f].sender / x.S == k) ? 1u : 0u;
  c = wave_sum(c);
  if (lane() == 0) s_c[t >> 6] = c;
  __syncthreads();
  if (any) {
    const uint32_t idx = s_c[0] + s_c[1] + s_c[2] + s_c[3];
    const uint32_t mpos = x.xoff[k * x.RS + x.R] + idx, ppos = x.xpoff[k * x.RS + x.R] + idx * x.NWW;
    uint32_t* U = x.ubits + (size_t)e * x.NWW;
    for (uint32_t w = t; w < x.NWW; w += blockDim.x) { x.spay[ppos + w] = U[w]; U[w] = 0u; }
    if (t == 0) x.smsg[mpos] = Msg{jid, jid, 0xFFFFFFFFu, K_KPU, x.NWW, 0u, 0u, ppos - x.xpoff[k * x.RS]};
  }
  if (t == 0) x.jslot[jid] = 0xFFFFFFFFu;
}

// one wave per sender: its delivered records in seq order, 64 at a time, to their shard blocks;
// a KnownPeers record's offset becomes relative to its block's payload (the receiver rebases it)
__global__ __launch_bounds__(256) void k_pack(Dev d, OutBuf ob, XState x) {
  const uint32_t l = lane();
  const uint32_t i = d.lo + blockIdx.x * 4 + (threadIdx.x >> 6);
  if (i >= d.hi) return;
  const uint32_t il = i - d.lo, cnt = ob.cnt[i], base = ob.off[i];
  uint32_t run[XMAX], prun[XMAX];
#pragma unroll
  for (uint32_t k = 0; k < XMAX; ++k) {
    run[k] = k < x.world ? x.xoff[k * x.RS + il] : 0u;
    prun[k] = k < x.world ? x.xpoff[k * x.RS + il] : 0u;
  }
  for (uint32_t c = 0; c < cnt; c += 64) {
    const uint32_t q = c + l;
    Msg m = Msg{0, 0, 0, 0, 0, 0, 0, 0};
    bool del = false;
    if (q < cnt) { m = ob.msgs[base + q]; del = x.ostatus[base + q] == 1; }
    const uint32_t ds = del ? m.dest / x.S : XMAX;
    const uint32_t ue = del ? x_union_slot(x, m) : 0xFFFFFFFFu;     // ids to a union: the record travels without them
    const uint32_t pl = (del && m.kind == K_KP && ue == 0xFFFFFFFFu) ? m.a : 0u;
    uint32_t pos = 0, ppos = 0;
#pragma unroll
    for (uint32_t k = 0; k < XMAX; ++k) {
      if (k >= x.world) break;
      const bool mine = ds == k;
      const unsigned long long bm = __ballot(mine);
      if (!bm) continue;
      const uint32_t pex = wave_excl(mine ? pl : 0u), ptot = wave_sum(mine ? pl : 0u);
      if (mine) { pos = run[k] + __popcll(bm & ((1ull << l) - 1ull)); ppos = prun[k] + pex; }
      run[k] += __popcll(bm);
      prun[k] += ptot;
    }
    if (del) {
      Msg o = m;
      if (ue != 0xFFFFFFFFu) { o.a = 0; o.off = 0; }
      else if (m.kind == K_KP) o.off = ppos - x.xpoff[ds * x.RS];
      x.smsg[pos] = o;
    }
    unsigned long long kpm = __ballot(pl != 0);
    while (kpm) {                                    // payload ids: the whole wave on each list
      const int src = __ffsll((long long)kpm) - 1;
      kpm &= kpm - 1;
      const uint32_t from = rdl(m.off, src), to = rdl(ppos, src), len = rdl(pl, src);
      for (uint32_t e = l; e < len; e += 64) x.spay[to + e] = ob.pay[from + e];
    }
    unsigned long long um = __ballot(ue != 0xFFFFFFFFu);
    while (um) {                                     // ids into their joiner's union: the whole wave on each list
      const int src = __ffsll((long long)um) - 1;
      um &= um - 1;
      const uint32_t from = rdl(m.off, src), len = rdl(m.a, src);
      uint32_t* U = x.ubits + (size_t)rdl(ue, src) * x.NWW;
      for (uint32_t e = l; e < len; e += 64) { const uint32_t id = ob.pay[from + e]; atomicOr(&U[id >> 5], 1u << (id & 31)); }
    }
  }
}

// receiver: rebase KnownPeers offsets to the received payload, count the in-order records per local
// destination (inbox sizes and next-wave outbox reservations), list the KnownPeers records
struct RecvBlocks { uint32_t world; uint32_t m0[XMAX + 1]; uint32_t p0[XMAX + 1]; };
__global__ __launch_bounds__(256) void k_route_recv(Dev d, OutBuf ib, WaveCtl wc, RecvBlocks rb, uint32_t n) {
  const uint32_t g = blockIdx.x * blockDim.x + threadIdx.x;
  if (g < n) {
    const Msg m = ib.msgs[g];
    if (m.kind == K_KP || m.kind == K_KPU) {           // (K_KPU: a shard's union of its Join responses to m.dest)
      uint32_t src = 0;
      while (src + 1 < rb.world && rb.m0[src + 1] <= g) ++src;
      ib.msgs[g].off = m.off + rb.p0[src];
      wc.status[g] = 2;
      atomicAdd(&wc.kcnt[m.dest], 1u);
      if (m.a) atomicAdd(&wc.kpay[m.dest], m.a);
    } else {
      wc.status[g] = 1;
      atomicAdd(&wc.cnt1[m.dest], 1u);
      atomicAdd(&wc.bnd[m.dest], out_bound(m.kind));
      if (m.kind == K_KPR) atomicAdd(&wc.bpay[m.dest], d.paybound);
    }
  }
}
__global__ void k_scatter_flat(Dev d, OutBuf ib, WaveCtl wc, uint32_t n, int32_t r, uint32_t nscat) {
  if (blockIdx.x >= nscat) {                           // the KPR oversize probe, as in k_scatter
    if (d.uniform) kpr_probe(d, wc, r, blockIdx.x - nscat, gridDim.x - nscat);
    return;
  }
  const uint32_t g = blockIdx.x * blockDim.x + threadIdx.x;
  if (g >= n) return;
  const uint8_t st = wc.status[g];
  const uint32_t dst = ib.msgs[g].dest;
  if (st == 1) wc.inbox[wc.in_off[dst] + atomicAdd(&wc.cursor[dst], 1u)] = g;
  else if (st == 2) wc.kin[wc.koff[dst] + atomicAdd(&wc.kcur[dst], 1u)] = g;
}

// ---- KnownPeers group of one destination: the arms (:448-472) and the envelope prologues (:406-415)
// One workgroup per destination with KnownPeers deliveries in the wave.  First every arm inserts
// each listed absent peer as Known(now - 10 s) — message-parallel, the group commutes (DESIGN.md
// §2.5) — then every envelope's prologue makes its sender Known(now).  The member count follows
// from the bits the atomics newly set, and suspect slots whose entry became Known are freed.
// BIG = the groups of at least KP_BIG ids (a joiner's hundreds of Join responses, all on one row):
// 1024 threads on the row's member bitset staged in LDS, a wave per message with KP_UNROLL
// independent id loads in flight per lane.  The other groups take 256 threads on the bitset in place.
// A BIG group whose bitset fits in LDS is served by KP_COLS workgroups, each owning a 1/KP_COLS part of the
// row's ids: every one reads all the group's ids and applies those in its part, arms then
// prologues.  An arm and a prologue conflict only on the same id, which one workgroup owns, so the
// parts need no synchronisation with each other.
constexpr uint32_t KP_BIG = 4096;          // payload ids from which a group takes the BIG kernel
constexpr uint32_t KP_LDS_WORDS = 16384;   // BIG: rows up to 512K ids keep their bitset in LDS (64 KB)
constexpr int KP_UNROLL = 10;            // 640 ids per wave step: a whole Join response (<= 567)
constexpr uint32_t KB_KP_COLS = 2;
constexpr uint32_t KP_COLS = KB_KP_COLS; // BIG groups in LDS: workgroups per destination, one per column part (A/B: 2 beats 4 and 1)
// a part must hold whole checkpoint segments: its workgroup refolds the segments it changed from its own
// LDS slice (3 parts of 64 segments straddle: an A/B build with 3 faulted)
static_assert(NSEG % KB_KP_COLS == 0, "KP_COLS must divide the 64 checkpoint segments");
__host__ __device__ constexpr size_t kp_lds_bytes(uint32_t nwr) {
  return 4ull * (nwr <= KP_LDS_WORDS ? nwr : 4);
}

// (the body of k_kp's first nblk workgroups, bid = the workgroup among them)
template <bool BIG>
__device__ __attribute__((always_inline)) inline void kp_group_body(const Dev& d, const OutBuf& ib, const WaveCtl& wc, int32_t r,
                                                                   uint32_t bid, uint32_t nblk) {
  extern __shared__ __attribute__((aligned(16))) uint32_t kp_lds[];
  __shared__ unsigned long long s_segs;
  __shared__ uint32_t s_add, s_nl;
  __shared__ uint32_t s_list[BIG ? 1024 : 256];
  __shared__ uint32_t ztab[BIG ? ZT * 128 : 1];
  const uint32_t t = threadIdx.x, T = blockDim.x;
  const uint32_t nact = d.ctr[C_ACTIVE];
  if (BIG) load_ztab(d, ztab);
  const uint8_t old = enc(r - SHARE_AGE, r), now = enc(r, r);
  const bool lds = BIG && d.NWR <= KP_LDS_WORDS && !(d.dbg & KB_DBG_KP_HBM);
  const uint32_t kpb = (d.dbg & KB_DBG_KP_BIG_SMALL) ? 0u : KP_BIG;
  const uint32_t KS = lds ? KP_COLS : 1u, part = bid % KS, G = nblk / KS, g = bid / KS;
  const uint32_t w0 = part * (d.NWR / KS), w1 = w0 + d.NWR / KS;   // this workgroup's bitset words
  // the active list T entries per workgroup group at a time, interleaved over the groups (consecutive
  // ids, e.g. the round's joiners, go to different groups): the destinations of this kind are
  // listed in LDS by all threads at once, then served one by one
  for (uint32_t c0 = 0; c0 < nact; c0 += G * T) {
  const uint32_t it = c0 + t * G + g;
  if (t == 0) s_nl = 0;
  __syncthreads();
  if (it < nact) {
    const uint32_t x = wc.active[it];
    if (wc.kcnt[x] && (wc.kpay[x] >= kpb) == BIG) s_list[atomicAdd(&s_nl, 1u)] = x;
  }
  __syncthreads();
  const uint32_t nl = s_nl;
  for (uint32_t li = 0; li < nl; ++li) {
    const uint32_t i = s_list[li];
    const uint32_t nk = wc.kcnt[i];
    const uint32_t k0 = wc.koff[i];
    uint32_t* gB = bits_of(d, i);
    uint32_t* B = lds ? kp_lds : gB;
    uint8_t* rw = row_of(d, i);
    if (t == 0) { s_segs = 0; s_add = 0; }
    const bool tdbg = BIG && (d.dev & 128) && t == 0;     // phase timing (KB_DEV=128, KB_DEBUG_WAVES)
    uint64_t tp[5];
    if (tdbg) tp[0] = wall_clock64();
    if (lds) stage16(reinterpret_cast<uint4*>(B), reinterpret_cast<const uint4*>(gB + w0), (w1 - w0) / 4, t, T);
    unsigned long long segs = 0;
    uint32_t added = 0;
    auto arm = [&](uint32_t p) __attribute__((always_inline)) {
      const uint32_t wi = p >> 5;
      if (wi < w0 || wi >= w1) return;                  // another workgroup's part
      const uint32_t bit = 1u << (p & 31);
      const uint32_t w = lds ? B[wi - w0] : __hip_atomic_load(&B[wi], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (w & bit) return;
      if (!(atomicOr(&B[wi - w0], bit) & bit)) { rw[p] = old; segs |= seg_bit(d, p); added++; }
    };
    if (BIG) {
      // wave per message: the records of up to 64 of this wave's messages are fetched at once (lane
      // j holds message wv + j * waves), then each message's ids are read KP_UNROLL per lane at once
      __syncthreads();
      const uint32_t nwv = T >> 6, wv = t >> 6, l = lane();
      for (uint32_t q0 = wv; q0 < nk; q0 += 64 * nwv) {
        const uint32_t qm = q0 + l * nwv;
        uint32_t moff = 0, mlen = 0;
        bool uni = false;                               // a union (K_KPU): a bitmap, armed below
        if (qm < nk) { const Msg m = ib.msgs[wc.kin[k0 + qm]]; moff = m.off; uni = m.kind == K_KPU; mlen = uni ? 0u : m.a; }
        const uint32_t cnt = q0 + 64 * nwv <= nk ? 64u : (nk - q0 + nwv - 1) / nwv;
        // software pipeline over the batch's (message, 640-id chunk) items: the ids of the next item are
        // loaded while the current item's arms run, so a message costs its arms, not arms + a load trip
        auto load = [&](uint32_t j, uint32_t e0, uint32_t (&pv)[KP_UNROLL]) __attribute__((always_inline)) {
          const uint32_t off = rdl(moff, (int)j), len = rdl(mlen, (int)j);
#pragma unroll
          for (int u = 0; u < KP_UNROLL; ++u) {
            const uint32_t e = e0 + 64u * u + l;
            pv[u] = e < len ? ib.pay[off + e] : 0xFFFFFFFFu;
          }
        };
        auto next = [&](uint32_t& j, uint32_t& e0) __attribute__((always_inline)) {
          e0 += 64 * KP_UNROLL;
          if (e0 >= rdl(mlen, (int)j)) { e0 = 0; ++j; }
        };
        uint32_t j = 0, e0 = 0;
        while (j < cnt && rdl(mlen, (int)j) == 0) ++j;
        uint32_t pv[KP_UNROLL];
        if (j < cnt) load(j, e0, pv);
        while (j < cnt) {
          uint32_t jn = j, en = e0;
          next(jn, en);
          while (jn < cnt && rdl(mlen, (int)jn) == 0) ++jn;
          uint32_t pn[KP_UNROLL];
          if (jn < cnt) load(jn, en, pn);
          // the item's arms in three batched phases (all membership reads, then all atomics, then the
          // stamp writes), so a lane waits for two LDS round trips per item instead of two per id
          uint32_t wv_[KP_UNROLL], ob_[KP_UNROLL];
#pragma unroll
          for (int u = 0; u < KP_UNROLL; ++u) {
            const uint32_t wi = pv[u] >> 5;
            const bool inr = pv[u] != 0xFFFFFFFFu && wi >= w0 && wi < w1;
            wv_[u] = inr ? (lds ? B[wi - w0] : __hip_atomic_load(&B[wi], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT))
                         : 0xFFFFFFFFu;
          }
#pragma unroll
          for (int u = 0; u < KP_UNROLL; ++u) {
            const uint32_t bit = 1u << (pv[u] & 31);
            ob_[u] = (wv_[u] & bit) ? bit : atomicOr(&B[(pv[u] >> 5) - w0], bit);
          }
#pragma unroll
          for (int u = 0; u < KP_UNROLL; ++u) {
            const uint32_t p = pv[u];
            if (!(ob_[u] & (1u << (p & 31)))) { rw[p] = old; segs |= seg_bit(d, p); added++; }
          }
#pragma unroll
          for (int u = 0; u < KP_UNROLL; ++u) pv[u] = pn[u];
          j = jn; e0 = en;
        }
        for (unsigned long long um = __ballot(uni); um; um &= um - 1) {   // unions: this part's words, 64 at a time
          const uint32_t off = rdl(moff, __ffsll((long long)um) - 1);
          for (uint32_t w = w0 + l; w < w1; w += 64) {
            const uint32_t u = ib.pay[off + w];
            const uint32_t cur = u ? (lds ? B[w - w0] : __hip_atomic_load(&B[w], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) : ~0u;
            uint32_t nw = u & ~cur;
            if (nw) nw &= ~atomicOr(&B[w - w0], nw);     // the bits this lane set first
            for (; nw; nw &= nw - 1) { const uint32_t p = 32 * w + (uint32_t)__builtin_ctz(nw); rw[p] = old; segs |= seg_bit(d, p); added++; }
          }
        }
      }
      __syncthreads();
      if (tdbg) tp[1] = wall_clock64();
    } else {
      __syncthreads();
      for (uint32_t q = 0; q < nk; ++q) {              // message by message
        const Msg m = ib.msgs[wc.kin[k0 + q]];
        for (uint32_t e = t; e < m.a; e += T) arm(ib.pay[m.off + e]);
      }
    }
    __syncthreads();
    for (uint32_t q = t; q < nk; q += T) {             // prologues
      const Msg m = ib.msgs[wc.kin[k0 + q]];
      if (m.kind == K_KPU) continue;                   // a union is no envelope
      const uint32_t s = m.sender;
      if ((s >> 5) < w0 || (s >> 5) >= w1) continue;     // another workgroup's part
      // byte update by CAS on its word: exactly one envelope per (dest, sender) sees the transition to
      // Known(now) and appends it to the freshness log
      uint32_t* wp = reinterpret_cast<uint32_t*>(rw + (s & ~3u));
      const uint32_t sh = 8 * (s & 3u);
      uint32_t ow = __hip_atomic_load(wp, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT), prevb;
      while (true) {
        prevb = (ow >> sh) & 0xFFu;
        if (prevb == now) break;
        const uint32_t res = atomicCAS(wp, ow, (ow & ~(0xFFu << sh)) | ((uint32_t)now << sh));
        if (res == ow) break;
        ow = res;
      }
      if (prevb != now) d.flog[(size_t)i * LOGCAP + (atomicAdd(&d.flog_n[i], 1u) & (LOGCAP - 1))] = log_entry(s, r);
      const uint32_t bit = 1u << (s & 31);
      if (!(atomicOr(&B[(s >> 5) - w0], bit) & bit)) { segs |= seg_bit(d, s); added++; }
    }
    if (segs) atomicOr(&s_segs, segs);
    if (added) atomicAdd(&s_add, added);
    __syncthreads();
    if (tdbg) tp[2] = wall_clock64();
    const unsigned long long sg = s_segs;
    unsigned long long refolded = 0;
    if (lds && sg) {                                   // write back the changed segments of the bitset
      const uint32_t wps4 = d.SEGW / 128;
      const uint4* B4 = reinterpret_cast<const uint4*>(B);
      uint4* g4 = reinterpret_cast<uint4*>(gB);
      for (uint32_t w = w0 / 4 + t; w < w1 / 4; w += T) if ((sg >> (w / wps4)) & 1ull) g4[w] = B4[w - w0 / 4];
      if (d.uniform) {
        // and refold their checkpoints from the staged bitset, a wave per segment (a joiner's group
        // changes every segment of its row: its fingerprint is then a combine, not a 64-segment refold
        // on k_proc's critical path)
        const uint8_t* hb = reinterpret_cast<const uint8_t*>(B);   // byte of 8-id block h at h - 4 w0
        const uint32_t nh = d.SEGW / 8, nwv = T >> 6, wv = t >> 6, l = lane();
        uint32_t q = 0;
        for (unsigned long long m = sg; m; m &= m - 1, ++q) {
          if (q % nwv != wv) continue;
          const uint32_t k = (uint32_t)(__ffsll((long long)m) - 1);
          uint32_t raw = 0, cnt = 0;
          const uint32_t h0 = k * nh + (l * nh) / 64, h1 = k * nh + ((l + 1) * nh) / 64;
          for (uint32_t h = h0; h < h1; ++h) fold_half(d, ztab, h, hb[h - 4 * w0], raw, cnt);
          wave_combine(d, raw, cnt);
          if (l == 0) d.segp[(size_t)i * NSEG + k] = make_uint2(raw, cnt);
        }
        refolded = sg;
      }
    }
    if (t < SLOTS) {                                   // a prologue overwrote a WaitingFor* entry to Known
      Susp* sl = d.susp + (size_t)i * SLOTS + t;
      if (sl->kind && (sl->peer >> 5) >= w0 && (sl->peer >> 5) < w1) {
        const uint32_t pw = __hip_atomic_load(reinterpret_cast<uint32_t*>(rw + (sl->peer & ~3u)), __ATOMIC_RELAXED,
                                              __HIP_MEMORY_SCOPE_AGENT);
        if (((pw >> (8 * (sl->peer & 3u))) & 0xFFu) != ST_SUSPECT) { lat_sample(d, i, sl->peer, sl->since, r); sl->kind = 0; }
      }
    }
    if (t == 0 && (s_add || sg)) {
      if (KS > 1) atomicAdd(&d.n[i], s_add); else d.n[i] += s_add;
      if (refolded) { atomicAnd(&d.sdirty[i], ~refolded); d.dirty[i] = 1; }   // checkpoints fresh, fp stale
      else mark(d, i, sg);
    }
    if (BIG && t == 0 && li == 0) path_hit(d, lds ? PATH_KP_BIG_LDS : PATH_KP_BIG_HBM);
    __syncthreads();                                   // LDS reused by the next destination
    if (tdbg) {
      tp[3] = wall_clock64();
      atomicAdd(&d.ctr[C_DBG_TNODE], (uint32_t)(tp[1] - tp[0]));   // stage + arms
      atomicAdd(&d.ctr[C_DBG_TBASE], (uint32_t)(tp[2] - tp[1]));   // prologues
      atomicAdd(&d.ctr[C_DBG_TINS], (uint32_t)(tp[3] - tp[2]));    // write-back + refold
      atomicAdd(&d.ctr[C_DBG_MSGS], nk); atomicAdd(&d.ctr[C_DBG_TSTART], 1u);
      atomicMax(&d.ctr[C_DBG_TMAX], (uint32_t)(tp[3] - tp[0]));
    }
  }
  }
}

// The groups under KP_BIG ids (KnownPeersRequest replies, small Join lists): a wave per destination,
// in place on the row's bitset, the same arms-then-prologues order as the BIG groups.  (The body of
// k_kp's last nblk workgroups: at least one per CU, since a round of the converged start's first
// SHARE_AGE rounds delivers ~24K replies of a few hundred ids at 64K peers in one wave.)
constexpr uint32_t KB_KPS_UNROLL = 4;
constexpr int KPS_UNROLL = KB_KPS_UNROLL;
__device__ __attribute__((always_inline)) inline void kp_small_body(const Dev& d, const OutBuf& ib, const WaveCtl& wc, int32_t r,
                                                                   const OutBuf& nb, uint32_t bid, uint32_t nblk) {
  __shared__ uint32_t s_list[1024], s_nl;
  const uint32_t t = threadIdx.x, T = blockDim.x, nwv = T >> 6, wv = t >> 6, l = lane();
  // the next outbox of every local row: capacity = the wave's reservation, empty (was a copy + memset)
  for (uint32_t i = d.lo + bid * T + t; i < d.hi; i += nblk * T) { nb.cap[i] = wc.bnd[i]; nb.cnt[i] = 0; }
  if (bid == 0 && t == 0) d.ctr[C_SLOW] = 0;             // the fast handlers list this wave's slow nodes afresh
  const uint32_t nact = d.ctr[C_ACTIVE];
  const uint8_t old = enc(r - SHARE_AGE, r), now = enc(r, r);
  const uint32_t kpb = (d.dbg & KB_DBG_KP_BIG_SMALL) ? 0u : KP_BIG;
  for (uint32_t c0 = 0; c0 < nact; c0 += nblk * T) {
    const uint32_t it = c0 + t * nblk + bid;             // interleaved over the workgroups
    if (t == 0) s_nl = 0;
    __syncthreads();
    if (it < nact) {
      const uint32_t x = wc.active[it];
      if (wc.kcnt[x] && wc.kpay[x] < kpb) s_list[atomicAdd(&s_nl, 1u)] = x;
    }
    __syncthreads();
    const uint32_t nl = s_nl;
    for (uint32_t li = wv; li < nl; li += nwv) {
      const uint32_t i = s_list[li], nk = wc.kcnt[i], k0 = wc.koff[i];
      uint32_t* B = bits_of(d, i);
      uint8_t* rw = row_of(d, i);
      unsigned long long segs = 0;
      uint32_t added = 0;
      // arms: KPS_UNROLL x 64 ids per step, their loads in flight together (all ids, then all member
      // words, then the atomics of the absent ones): a KnownPeersRequest reply of a few hundred ids
      // costs two HBM round trips, not two per 64 ids.  The records of up to 64 messages are fetched at
      // once (lane k holds message q0 + k).
      for (uint32_t q0 = 0; q0 < nk; q0 += 64) {
        uint32_t moff = 0, mlen = 0, mkind = 0;
        if (q0 + l < nk) { const Msg m = ib.msgs[wc.kin[k0 + q0 + l]]; moff = m.off; mlen = m.a; mkind = m.kind; }
        const uint32_t qn = nk - q0 < 64 ? nk - q0 : 64u;
        for (uint32_t j = 0; j < qn; ++j) {
          const uint32_t off = rdl(moff, (int)j), len = rdl(mlen, (int)j);
          if (rdl(mkind, (int)j) == K_KPU) {                // a union: the row's words, 64 at a time
            for (uint32_t w = l; w < len; w += 64) {
              const uint32_t u = ib.pay[off + w];
              uint32_t nw = u ? u & ~__hip_atomic_load(&B[w], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : 0u;
              if (nw) nw &= ~atomicOr(&B[w], nw);
              for (; nw; nw &= nw - 1) { const uint32_t p = 32 * w + (uint32_t)__builtin_ctz(nw); rw[p] = old; segs |= seg_bit(d, p); added++; }
            }
            continue;
          }
          for (uint32_t e0 = 0; e0 < len; e0 += 64 * KPS_UNROLL) {
            uint32_t pv[KPS_UNROLL], wv_[KPS_UNROLL], ob_[KPS_UNROLL];
#pragma unroll
            for (int u = 0; u < KPS_UNROLL; ++u) {
              const uint32_t e = e0 + 64u * u + l;
              pv[u] = e < len ? ib.pay[off + e] : 0xFFFFFFFFu;
            }
#pragma unroll
            for (int u = 0; u < KPS_UNROLL; ++u)
              wv_[u] = pv[u] != 0xFFFFFFFFu ? __hip_atomic_load(&B[pv[u] >> 5], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)
                                            : 0xFFFFFFFFu;
#pragma unroll
            for (int u = 0; u < KPS_UNROLL; ++u) {
              const uint32_t bit = 1u << (pv[u] & 31);
              ob_[u] = (wv_[u] & bit) ? bit : atomicOr(&B[pv[u] >> 5], bit);
            }
#pragma unroll
            for (int u = 0; u < KPS_UNROLL; ++u) {
              const uint32_t p = pv[u];
              if (!(ob_[u] & (1u << (p & 31)))) { rw[p] = old; segs |= seg_bit(d, p); added++; }
            }
          }
        }
      }
      wave_mem_sync();
      __builtin_amdgcn_s_waitcnt(0);
      __builtin_amdgcn_wave_barrier();
      for (uint32_t q = l; q < nk; q += 64) {             // prologues (as k_kp_group)
        const Msg m = ib.msgs[wc.kin[k0 + q]];
        if (m.kind == K_KPU) continue;                    // a union is no envelope
        const uint32_t s = m.sender;
        uint32_t* wp = reinterpret_cast<uint32_t*>(rw + (s & ~3u));
        const uint32_t sh = 8 * (s & 3u);
        uint32_t ow = __hip_atomic_load(wp, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT), prevb;
        while (true) {
          prevb = (ow >> sh) & 0xFFu;
          if (prevb == now) break;
          const uint32_t res = atomicCAS(wp, ow, (ow & ~(0xFFu << sh)) | ((uint32_t)now << sh));
          if (res == ow) break;
          ow = res;
        }
        if (prevb != now) d.flog[(size_t)i * LOGCAP + (atomicAdd(&d.flog_n[i], 1u) & (LOGCAP - 1))] = log_entry(s, r);
        const uint32_t bit = 1u << (s & 31);
        if (!(atomicOr(&B[s >> 5], bit) & bit)) { segs |= seg_bit(d, s); added++; }
      }
      segs = (unsigned long long)wave_or((uint32_t)segs) | ((unsigned long long)wave_or((uint32_t)(segs >> 32)) << 32);
      added = wave_sum(added);
      __builtin_amdgcn_s_waitcnt(0);
      __builtin_amdgcn_wave_barrier();
      if (l < SLOTS) {                                   // a prologue overwrote a WaitingFor* entry to Known
        Susp* sl = d.susp + (size_t)i * SLOTS + l;
        if (sl->kind) {
          const uint32_t pw = __hip_atomic_load(reinterpret_cast<uint32_t*>(rw + (sl->peer & ~3u)), __ATOMIC_RELAXED,
                                                __HIP_MEMORY_SCOPE_AGENT);
          if (((pw >> (8 * (sl->peer & 3u))) & 0xFFu) != ST_SUSPECT) { lat_sample(d, i, sl->peer, sl->since, r); sl->kind = 0; }
        }
      }
      if (l == 0 && (added || segs)) { d.n[i] += added; mark(d, i, segs); }
    }
    __syncthreads();                                       // s_list reused by the next chunk
  }
}

// The KnownPeers group of every destination of the wave in ONE launch: workgroups [0, nbig) serve the
// BIG groups (KP_COLS per destination group, bitset in LDS), the rest the small groups (a wave per
// destination) and set up the next outbox.  The two kinds never share a destination.
__global__ __launch_bounds__(1024) void k_kp(Dev d, OutBuf ib, WaveCtl wc, int32_t r_arg, OutBuf nb, uint32_t nbig) {
  const int32_t r = round_of(d, r_arg);
  if (blockIdx.x < nbig) kp_group_body<true>(d, ib, wc, r, blockIdx.x, nbig);
  else kp_small_body(d, ib, wc, r, nb, blockIdx.x - nbig, gridDim.x - nbig);
}

// ---- inboxes longer than one wave: sorted into canonical (sender, seq) order = ascending outbox
// index, one workgroup per node, bitonic in LDS (up to SORT_MAX entries; longer ones keep the
// selection path of k_proc)
constexpr uint32_t SORT_MAX = 8192;
constexpr uint32_t KB_SORT_GROUPS = 256;
constexpr uint32_t SORT_GROUPS = KB_SORT_GROUPS;   // k_sortfast workgroups that sort long inboxes
__device__ inline uint32_t sort_max(const Dev& d) { return (d.dbg & KB_DBG_PROC_UNSORTED) ? 64u : SORT_MAX; }
__device__ __attribute__((always_inline)) inline void sort_body(const Dev& d, const WaveCtl& wc, int32_t r, uint32_t bid,
                                                               uint32_t nblk) {
  __shared__ uint32_t v[SORT_MAX];
  __shared__ uint32_t s_list[1024], s_nl;
  const uint32_t nact = d.ctr[C_ACTIVE];
  // the active list blockDim entries per workgroup at a time, interleaved over the workgroups: its long
  // inboxes are listed in LDS by all threads at once
  for (uint32_t c0 = 0; c0 < nact; c0 += nblk * blockDim.x) {
  const uint32_t it = c0 + threadIdx.x * nblk + bid;
  if (threadIdx.x == 0) s_nl = 0;
  __syncthreads();
  if (it < nact) {
    const uint32_t x = wc.active[it];
    const uint32_t c = wc.cnt1[x];
    if (c > 64 && c <= sort_max(d)) s_list[atomicAdd(&s_nl, 1u)] = x;
  }
  __syncthreads();
  const uint32_t nl = s_nl;
  for (uint32_t li = 0; li < nl; ++li) {
    const uint32_t i = s_list[li];
    const uint32_t n = wc.cnt1[i];
    uint32_t P = 128;
    while (P < n) P <<= 1;
    const uint32_t base = wc.in_off[i];
    for (uint32_t k = threadIdx.x; k < P; k += blockDim.x) v[k] = k < n ? wc.inbox[base + k] : 0xFFFFFFFFu;
    __syncthreads();
    for (uint32_t k = 2; k <= P; k <<= 1)
      for (uint32_t j = k >> 1; j > 0; j >>= 1) {
        for (uint32_t x = threadIdx.x; x < P; x += blockDim.x) {
          const uint32_t y = x ^ j;
          if (y > x) {
            const uint32_t a = v[x], b = v[y];
            if (((x & k) == 0) == (a > b)) { v[x] = b; v[y] = a; }
          }
        }
        __syncthreads();
      }
    for (uint32_t k = threadIdx.x; k < n; k += blockDim.x) wc.inbox[base + k] = v[k];
    __syncthreads();
  }
  }
}

// ---- the per-node in-order program for Ping / PingRequest / Ack / KnownPeersRequest ---------------
// ---- fast lane of the in-order handlers: a THREAD per node --------------------------------------
// The common inbox — at most FAST_MAX Ping / PingRequest / Ack envelopes (and KnownPeersRequests
// once kpr_probe (run with k_scatter) has proven this round's replies oversize), every sender already a member, the
// node's fingerprint current — changes no membership, so no fingerprint work: the handlers reduce
// to stamp/log/slot updates and emissions.  Such nodes are handled here, one per
// thread, in canonical (sender, seq) order; every other node with in-order deliveries goes to the
// `slow` list for k_proc (same semantics: prologue :406-415, Ping :513-532, PingRequest :533-545,
// Ack :418-447, maybe_sync :707-740).
constexpr uint32_t FAST_MAX = 8;
__device__ __attribute__((always_inline)) inline void fast_body(const Dev& d, const OutBuf& ib, const OutBuf& ob, const WaveCtl& wc,
                                                               int32_t r, uint32_t* slow, uint32_t bid) {
  const uint32_t nact = d.ctr[C_ACTIVE];
  const uint32_t it = bid * blockDim.x + threadIdx.x;
  const uint8_t now = enc(r, r);
  unsigned long long curovf = 0, over = 0;
  bool to_slow = false;
  uint32_t i = 0;
  if (it < nact) {
    i = wc.active[it];
    const uint32_t icnt = wc.cnt1[i];
    bool fast = icnt && icnt <= FAST_MAX && !d.dirty[i];
    uint32_t g[FAST_MAX];
    // Everything the handlers read is loaded up front, each group of loads in flight together: the
    // records (kept in registers), the senders' member words and stamps (a handler changes only its own
    // sender's stamp, and equal senders are adjacent), the node's header.  The fast lane is a chain of
    // dependent loads per node, so its length is the launch's duration in the late waves.
    uint32_t ms[FAST_MAX], mk[FAST_MAX], ma[FAST_MAX], mf[FAST_MAX], mn[FAST_MAX];
    uint8_t sb[FAST_MAX];
    uint32_t n = 0, fp = 0, ob_cap = 0, ob_off = 0, fn = 0;
    if (fast) {
      const uint32_t base = wc.in_off[i];
      n = d.n[i]; fp = d.fp[i]; ob_cap = ob.cap[i]; ob_off = ob.off[i]; fn = d.flog_n[i];
#pragma unroll
      for (uint32_t k = 0; k < FAST_MAX; ++k) g[k] = k < icnt ? wc.inbox[base + k] : 0xFFFFFFFFu;
#pragma unroll
      for (uint32_t a = 1; a < FAST_MAX; ++a)        // canonical order = ascending record index
#pragma unroll
        for (uint32_t b = a; b > 0; --b)
          if (g[b - 1] > g[b]) { const uint32_t x = g[b]; g[b] = g[b - 1]; g[b - 1] = x; }
      const uint32_t* bw = bits_of(d, i);
      const uint8_t* rw = row_of(d, i);
      const bool kpr_over = d.uniform && d.kpr_big[i] == r;      // every KPR reply of the round oversize
#pragma unroll
      for (uint32_t k = 0; k < FAST_MAX; ++k) {
        ms[k] = 0; mk[k] = 0; ma[k] = 0; mf[k] = 0; mn[k] = 0;
        if (k < icnt) { const Msg m = ib.msgs[g[k]]; ms[k] = m.sender; mk[k] = m.kind; ma[k] = m.a; mf[k] = m.fp; mn[k] = m.n; }
      }
#pragma unroll
      for (uint32_t k = 0; k < FAST_MAX; ++k) {
        sb[k] = 0;
        if (k < icnt) {
          const uint32_t w = bw[ms[k] >> 5];
          sb[k] = rw[ms[k]];
          if ((mk[k] == K_KPR && !kpr_over) || !((w >> (ms[k] & 31)) & 1u)) fast = false;
        }
      }
    }
    to_slow = icnt && !fast;
    if (to_slow && (d.dev & 256)) {                   // why nodes go to k_proc (KB_DEV=256, KB_DEBUG_WAVES)
      bool kpr = false, nonmem = false;
      if (icnt <= FAST_MAX) {
        const uint32_t* bw = bits_of(d, i);
        for (uint32_t k = 0; k < icnt; ++k) {
          const Msg m = ib.msgs[wc.inbox[wc.in_off[i] + k]];
          kpr |= m.kind == K_KPR && d.kpr_big[i] != r;
          nonmem |= !((bw[m.sender >> 5] >> (m.sender & 31)) & 1u);
        }
      }
      atomicAdd(&d.ctr[icnt > FAST_MAX ? C_DBG_SLOW_LONG : nonmem ? C_DBG_SLOW_NONMEM : d.dirty[i] ? C_DBG_SLOW_DIRTY
                                                                                                : kpr ? C_DBG_SLOW_KPR : C_DBG_SLOW_OTHER], 1u);
    }
    if (fast) {
      uint32_t oseq = 0, last_sender = 0xFFFFFFFFu;
      auto emit = [&](uint32_t dest, uint32_t kind, uint32_t a, uint32_t efp, uint32_t en) __attribute__((always_inline)) {
        if (oseq >= ob_cap || ob_off + oseq >= ob.msg_cap) set_err(d, DERR_OUTBOX);
        else ob.msgs[ob_off + oseq] = Msg{dest, i, oseq, kind, a, efp, en, 0};
        oseq++;
      };
      uint8_t* rw = row_of(d, i);
      Susp* sl = d.susp + (size_t)i * SLOTS;
      Cur* cu = d.cur + (size_t)i * CSLOTS;
      // curious_peers entry of peer p: the slots' (used, peer) words read together, not slot by slot
      auto cur_find = [&](uint32_t p) __attribute__((always_inline)) -> int {
        uint32_t cp[CSLOTS], cf[CSLOTS];
#pragma unroll
        for (int j = 0; j < CSLOTS; ++j) { cp[j] = cu[j].peer; cf[j] = cu[j].used; }
        int e = -1;
#pragma unroll
        for (int j = CSLOTS - 1; j >= 0; --j) if (cf[j] && cp[j] == p) e = j;
        return e;
      };
      // one copy of the handlers, always on entry 0, the register arrays shifted down after each message
      // (unrolled over FAST_MAX, the handlers had made k_sortfast ≈ 50 KB of code, beyond the instruction
      // cache that its waves share with the sorting workgroups)
#pragma unroll 1
      for (uint32_t k = 0; k < icnt; ++k) {
        const uint32_t s = ms[0], kind = mk[0], ma_k = ma[0], mf_k = mf[0], mn_k = mn[0];
        const uint8_t sb_k = sb[0];
#pragma unroll
        for (uint32_t q = 0; q + 1 < FAST_MAX; ++q) {
          ms[q] = ms[q + 1]; mk[q] = mk[q + 1]; ma[q] = ma[q + 1]; mf[q] = mf[q + 1]; mn[q] = mn[q + 1]; sb[q] = sb[q + 1];
        }
        if (s != last_sender) {                        // prologue: insert(sender, Known(now))
          const uint8_t b = sb_k;
          if (b == ST_SUSPECT)
            for (int j = 0; j < SLOTS; ++j) if (sl[j].kind && sl[j].peer == s) { lat_sample(d, i, s, sl[j].since, r); sl[j].kind = 0; }
          if (b != now) { rw[s] = now; d.flog[(size_t)i * LOGCAP + (fn & (LOGCAP - 1))] = log_entry(s, r); fn++; }
          last_sender = s;
        }
        if (kind == K_PING) {
          emit(s, K_ACK, i, fp, n);
        } else if (kind == K_PINGREQ) {
          int e = cur_find(ma_k);
          if (e < 0) {
            for (int j = 0; j < CSLOTS && e < 0; ++j) if (!cu[j].used) e = j;
            if (e >= 0) { cu[e].used = 1; cu[e].peer = ma_k; cu[e].nobs = 0; }
          }
          if (e < 0) curovf++;
          else {
            const uint32_t nobs = cu[e].nobs;
            bool dup = false;
            for (uint32_t q = 0; q < nobs; ++q) dup |= cu[e].obs[q] == s;
            if (!dup) { if (nobs == NOBS) curovf++; else { cu[e].obs[nobs] = s; cu[e].nobs = nobs + 1; } }
          }
          emit(ma_k, K_PING, 0, 0, 0);
        } else if (kind == K_ACK) {
          const int e = cur_find(ma_k);
          if (e >= 0) {
            const uint32_t nobs = cu[e].nobs;
            uint32_t ob4[NOBS];
#pragma unroll
            for (int q = 0; q < NOBS; ++q) ob4[q] = cu[e].obs[q];
#pragma unroll
            for (uint32_t q = 0; q < (uint32_t)NOBS; ++q) if (q < nobs) emit(ob4[q], K_ACK, ma_k, mf_k, mn_k);
            cu[e].used = 0;
          }
          if (fp != mf_k && !(n > mn_k)) emit(ma_k, K_KPR, 0, fp, n);
        } else if (kind == K_KPR) {                  // :473-512, reply lost as oversize (Q3), then :507
          over++;
          if (fp != mf_k && !(n > mn_k)) emit(s, K_KPR, 0, fp, n);
        }
      }
      ob.cnt[i] = oseq;
      d.flog_n[i] = fn;
    }
    if (!to_slow) wave_ctr_clear(wc, i);              // done with this node for the wave
  }
  // the rest goes to k_proc: listed with one atomic per workgroup (the list counter is one word)
  __shared__ uint32_t s_wn[16], s_wb[16];
  const unsigned long long sm = __ballot(to_slow);
  const uint32_t wv = threadIdx.x >> 6, nwv = blockDim.x >> 6;
  if (lane() == 0) s_wn[wv] = (uint32_t)__popcll(sm);
  __syncthreads();
  if (threadIdx.x == 0) {
    uint32_t tot = 0;
    for (uint32_t k = 0; k < nwv; ++k) tot += s_wn[k];
    uint32_t base = tot ? atomicAdd(&d.ctr[C_SLOW], tot) : 0u;
    for (uint32_t k = 0; k < nwv; ++k) { s_wb[k] = base; base += s_wn[k]; }
  }
  __syncthreads();
  if (to_slow) slow[s_wb[wv] + __popcll(sm & ((1ull << lane()) - 1ull))] = i;
  {
    const int idx[2] = {S_CUROVF, S_OVERSIZE};
    const unsigned long long v[2] = {curovf, over};
    stat_add_n(d, idx, v);
  }
}

// Inbox sorts + KPR oversize probe (workgroups [0, nsort)) and the fast in-order handlers (the rest) in ONE
// launch.  They touch disjoint nodes: the sorts take inboxes > 64 entries, the fast lane <= FAST_MAX; a
// node with a KnownPeersRequest is fast only once the probe has proven its replies oversize (kpr_big = r,
// written by the probe after its last read of that row), else it goes to k_proc, which reads the proof.
// 256-thread workgroups: the fast lane's nodes are then spread over every CU (with 1024-thread workgroups the
// (R + 1023) / 1024 fast workgroups, one per CU at this kernel's occupancy, left most CUs idle)
constexpr uint32_t SORTFAST_T = 256;
__global__ __launch_bounds__(SORTFAST_T) void k_sortfast(Dev d, OutBuf ib, OutBuf ob, WaveCtl wc, int32_t r_arg, uint32_t* slow,
                                                   uint32_t nsort) {
  const int32_t r = round_of(d, r_arg);
  if (blockIdx.x < nsort) sort_body(d, wc, r, blockIdx.x, nsort);
  else fast_body(d, ib, ob, wc, r, slow, blockIdx.x - nsort);
}

constexpr uint32_t KB_KPR_BATCH = 4;        // KPR reply scan: 64-entry log batches in flight per step
constexpr uint32_t KB_PROC_MANY = 1;        // batches of >= 8 prologue insertions fold one per lane (0: the whole wave on each)
constexpr uint32_t KB_PROC_WPE = 1;         // minimum waves per SIMD k_proc is compiled for (1 = the compiler's choice)
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(KB_PROC_WPE)))
void k_proc(Dev d, OutBuf ib, OutBuf ob, WaveCtl wc, int32_t r_arg, const uint32_t* list) {
  const int32_t r = round_of(d, r_arg);
  __shared__ uint32_t ztab[ZT * 128];
  __shared__ Susp s_susp[4][SLOTS];
  __shared__ Cur s_cur[4][CSLOTS];
  __shared__ uint2 s_suf[4][NSEG + 1];
  const uint32_t nact = d.ctr[C_SLOW];                // the nodes k_proc_fast left (list)
  if (blockIdx.x * 4 >= nact) return;                 // no node for this workgroup (before the table load)
  load_ztab(d, ztab);
  const uint32_t wv = threadIdx.x >> 6;
  const uint32_t l = lane();
  const uint8_t now = enc(r, r);
  const uint8_t fresh_thr = enc(r - (SHARE_AGE - 1), r);
  unsigned long long w_over = 0, w_curovf = 0;      // flushed once per wave (see k_phaseB)
  // algorithmic bytes (bench roofline): every table word the handlers must read or write —
  // node header and slot tables, inbox indices and records, each sender's member word and stamp, the
  // stamps / log entries / bits written, checkpoints and the member bytes + table words of every
  // (partial) fold, freshness-log entries scanned, records and payload ids emitted
  unsigned long long w_bytes = 0;
  for (uint32_t it = blockIdx.x * 4 + wv; it < nact; it += gridDim.x * 4) {
    const uint32_t i = list[it];
    const bool tdbg = (d.dev & 64) != 0;                // timing breakdown (KB_DEV=64, KB_DEBUG_WAVES)
    const uint64_t t_node = tdbg ? wall_clock64() : 0;
    uint64_t t_base = 0, t_ins = 0;
    uint8_t* rw = row_of(d, i);
    const uint32_t* bw = bits_of(d, i);
    uint32_t n = d.n[i], fp = d.fp[i], oseq = 0, pay_used = 0, fn = d.flog_n[i];
    const uint32_t ob_cap = ob.cap[i], ob_off = ob.off[i];   // this node's outbox region, loaded once
    auto emit = [&](uint32_t dest, uint32_t kind, uint32_t a, uint32_t efp, uint32_t en, uint32_t off)
        __attribute__((always_inline)) {
      if (l == 0) {
        if (oseq >= ob_cap || ob_off + oseq >= ob.msg_cap) set_err(d, DERR_OUTBOX);
        else ob.msgs[ob_off + oseq] = Msg{dest, i, oseq, kind, a, efp, en, off};
      }
      oseq++;
      w_bytes += sizeof(Msg);
    };
    int32_t kbig = d.kpr_big[i];
    bool dirty = d.dirty[i] != 0, need_sync = false;
    unsigned long long segs = 0;
    if (l < SLOTS) s_susp[wv][l] = d.susp[(size_t)i * SLOTS + l];
    if (l < CSLOTS) s_cur[wv][l] = d.cur[(size_t)i * CSLOTS + l];
    wait_lds();
    __builtin_amdgcn_wave_barrier();
    const uint32_t ibase = wc.in_off[i], icnt = wc.cnt1[i];
    // header + slot tables read and written back, inbox index + record of every message
    w_bytes += 2 * (28 + sizeof(Susp) * SLOTS + sizeof(Cur) * CSLOTS) + (4 + sizeof(Msg)) * (uint64_t)icnt;
    // canonical order = ascending outbox index = (sender, seq): one wave sorts <= 64 entries in
    // registers; k_sortfast has sorted longer inboxes up to SORT_MAX in place
    uint32_t mine = l < icnt ? wc.inbox[ibase + l] : 0xFFFFFFFFu;
    const bool small = icnt <= 64, sorted = icnt <= sort_max(d);
    if (small) {
      // bitonic stages up to the inbox's power of two: after stage k the lanes [0, k) are ascending, and every
      // lane at or past icnt holds the maximum, so stage K >= icnt leaves the inbox sorted in lanes [0, icnt)
      auto step = [&](uint32_t o, uint32_t k, uint32_t j) __attribute__((always_inline)) {
        const bool up = (l & k) == 0, lower = (l & j) == 0;
        const uint32_t mn = o < mine ? o : mine, mx = o < mine ? mine : o;
        mine = (lower == up) ? mn : mx;
      };
#pragma unroll
      for (uint32_t k = 2; k <= 64; k <<= 1) {
        if (icnt <= k / 2) break;                      // wave-uniform
        if (k >= 64) step(shfl_xor_c<32>(mine), k, 32);
        if (k >= 32) step(shfl_xor_c<16>(mine), k, 16);
        if (k >= 16) step(shfl_xor_c<8>(mine), k, 8);
        if (k >= 8) step(shfl_xor_c<4>(mine), k, 4);
        if (k >= 4) step(shfl_xor_c<2>(mine), k, 2);
        step(shfl_xor_c<1>(mine), k, 1);
      }
    }
    uint32_t dbg_fp = 0, dbg_ins = 0, dbg_kpr = 0, dbg_log = 0, dbg_base = 0;
    // Incremental fingerprint (uniform identities, sorted inbox).  Prologue insertions arrive in
    // ascending id order, so for an inserted x every member above x is still the base set's:
    //   raw(S + x) = raw(S)·Z ⊕ B·(Z ⊕ 1) ⊕ c_x·Z^{n>x},  B = fold of the members above x, n>x their count
    // B = (fold of x's segment above x)·Z^{cnt} ⊕ suffix combine of the later segments (taken once per
    // node, s_suf).  Each batch precomputes K = B·(Z ⊕ 1) ⊕ c_x·Z^{n>x} lane-parallel; the in-order
    // update is then one multiply by Z per insertion.
    bool inc = false, fpstale = false;
    uint32_t R = 0, zf = 0, zf_n = 0;   // zf: lane k holds zfin[zf_n + k] (the node's next counts)
    auto take_base = [&]() __attribute__((always_inline)) {
      if (need_sync) { wave_mem_sync(); need_sync = false; }
      dbg_base++;
      const unsigned long long sd = d.sdirty[i] | segs;
      w_bytes += 8 * NSEG + 4 * 64 + (uint64_t)__popcll(sd) * (5 * (d.SEGW / 8) + 8);   // checkpoints, Z^n row, refolds
      const uint2 sp = refold_stale(d, ztab, i, sd);
      uint32_t raw = sp.x, cnt = sp.y, c = sp.y;
      // inclusive suffix scan, lane k -> segments k..63: inside each 16-lane row by DPP, then each row's
      // lanes combined with the total of the rows after it (formed from the row totals in scalar registers)
      uint32_t oc[4], zp[4];
      oc[0] = dpp_shl<1>(c); c += oc[0];
      oc[1] = dpp_shl<2>(c); c += oc[1];
      oc[2] = dpp_shl<4>(c); c += oc[2];
      oc[3] = dpp_shl<8>(c); c += oc[3];
      const uint32_t c1 = rdl(c, 16), c2 = rdl(c, 32), c3 = rdl(c, 48);
      const uint32_t row = l >> 4;
      const uint32_t sc = row == 0 ? c1 + c2 + c3 : (row == 1 ? c2 + c3 : (row == 2 ? c3 : 0u));
#pragma unroll
      for (int t = 0; t < 4; ++t) zp[t] = d.zpow[oc[t]];
      const uint32_t zs = d.zpow[sc], z3 = d.zpow[c3], z23 = d.zpow[c2 + c3];
      uint32_t o;
      o = dpp_shl<1>(raw); raw = multmodp(zp[0], raw) ^ o;
      o = dpp_shl<2>(raw); raw = multmodp(zp[1], raw) ^ o;
      o = dpp_shl<4>(raw); raw = multmodp(zp[2], raw) ^ o;
      o = dpp_shl<8>(raw); raw = multmodp(zp[3], raw) ^ o;
      const uint32_t r1 = rdl(raw, 16), r2 = rdl(raw, 32), r3 = rdl(raw, 48);
      const uint32_t s1 = multmodp(z3, r2) ^ r3, s0 = multmodp(z23, r1) ^ s1;
      raw = multmodp(zs, raw) ^ (row == 0 ? s0 : (row == 1 ? s1 : (row == 2 ? r3 : 0u)));
      c += sc;
      cnt = c;
      s_suf[wv][l] = make_uint2(raw, cnt);
      if (l == 0) s_suf[wv][NSEG] = make_uint2(0, 0);
      wait_lds();
      __builtin_amdgcn_wave_barrier();
      R = rdl(raw, 0);
      if (rdl(cnt, 0) != n) set_err(d, DERR_FP);
      if (l == 0 && sd) atomicAnd(&d.sdirty[i], ~sd);
      segs = 0;
      inc = true; dirty = false; fpstale = true;
      zf_n = n;
      zf = d.zfin[n + l <= d.C + 1 ? n + l : d.C + 1];
    };
    auto fp_now = [&]() __attribute__((always_inline)) -> uint32_t {
      if (inc) {
        if (fpstale) {
          const uint32_t dz = n - zf_n;                 // insertions since the base: prefetched Z^n term
          fp = R ^ (dz < 64 ? __builtin_amdgcn_readlane(zf, (int)dz) : d.zfin[n]) ^ 0xFFFFFFFFu;
          fpstale = false;
        }
        return fp;
      }
      if (dirty) {
        dbg_fp++;
        w_bytes += 8 * NSEG + (uint64_t)__popcll(d.sdirty[i] | segs) * (5 * (d.SEGW / 8) + 8);
        if (need_sync) { wave_mem_sync(); need_sync = false; }
        fp = wave_fp(d, ztab, i, segs);
        segs = 0;
        dirty = false;
      }
      return fp;
    };
    // (f: the fingerprint, taken once per message before its handler: fp_now's refold path is large, and
    // one inlined copy per call site had made k_proc ≈ 85 KB of code, more than the instruction cache)
    auto maybe_sync = [&](uint32_t f, uint32_t peer, uint32_t their_fp, uint32_t their_n) __attribute__((always_inline)) {   // :707-740
      if (f == their_fp || n > their_n) return;
      emit(peer, K_KPR, 0, f, n, 0);
    };
    uint32_t last_g = 0xFFFFFFFFu, last_sender = 0xFFFFFFFFu;
    // messages are fetched 64 at a time (lane k holds the record of message base + k) and handed to
    // the wave one by one with cross-lane reads, so the in-order loop never waits on HBM per message
    // The prologue's row state (member bit, stamp) of each batch's senders is fetched with the batch:
    // a handler changes only its own sender's entry, and equal senders are adjacent (sorted inbox), so
    // the prefetched state of a later message of the batch is still current when it is reached.
    Msg lm;
    uint32_t pre_was = 0, pre_b = 0, Kx = 0;
    const uint64_t t_loop = tdbg ? wall_clock64() : 0;
    for (uint32_t t = 0; t < icnt; ++t) {
      uint32_t g;
      if (sorted) {
        if ((t & 63) == 0) {
          if (need_sync) { wave_mem_sync(); need_sync = false; }
          const uint32_t gl = small ? mine : (t + l < icnt ? wc.inbox[ibase + t + l] : 0xFFFFFFFFu);
          if (gl != 0xFFFFFFFFu) {
            lm = ib.msgs[gl];
            pre_was = (bw[lm.sender >> 5] >> (lm.sender & 31)) & 1u;
            const uint32_t sb = rw[lm.sender];         // issued with the bit load, not after it
            pre_b = pre_was ? sb : ST_UNKNOWN;
          }
          if (!small) mine = gl;
          // insertions of this batch: first message of a sender run whose sender is not a member
          const uint32_t prev = __shfl_up(lm.sender, 1, 64);
          const bool ins = gl != 0xFFFFFFFFu && !pre_was && lm.sender != (l == 0 ? last_sender : prev);
          const unsigned long long insm = __ballot(ins);
          w_bytes += 5ull * __popcll(__ballot(gl != 0xFFFFFFFFu));   // each sender's member word + stamp
          if (d.uniform && insm) {
            const uint64_t ta = tdbg ? wall_clock64() : 0;
            if (!inc) take_base();
            const uint64_t tb = tdbg ? wall_clock64() : 0;
            t_base += tb - ta;
            const uint8_t* hb = reinterpret_cast<const uint8_t*>(bw);
            if (KB_PROC_MANY && __popcll(insm) >= 8) {   // many: one insertion per lane
              if (ins) {
                const uint32_t x = lm.sender, k = seg_of(d, x), hend = (k + 1) * (d.SEGW / 8);
                uint32_t praw = 0, pcnt = 0;
                fold_half(d, ztab, x >> 3, hb[x >> 3] & ~((2u << (x & 7)) - 1u) & 0xFFu, praw, pcnt);
                for (uint32_t h0 = (x >> 3) + 1; h0 < hend; h0 += 16) {   // 16 blocks of loads in flight
                  uint32_t m8v[16], hv[16];
#pragma unroll
                  for (int j = 0; j < 16; ++j) m8v[j] = h0 + j < hend ? hb[h0 + j] : 0u;
#pragma unroll
                  for (int j = 0; j < 16; ++j) hv[j] = m8v[j] ? d.htab[(size_t)(h0 + j) * 256 + m8v[j]] : 0u;
#pragma unroll
                  for (int j = 0; j < 16; ++j)
                    if (m8v[j]) { const uint32_t c = __popc(m8v[j]); praw = mulzc(ztab, praw, c) ^ hv[j]; pcnt += c; }
                }
                const uint2 su = s_suf[wv][k + 1];
                const uint32_t Bx = multmodp(d.zpow[su.y], praw) ^ su.x;
                Kx = mulzc(ztab, Bx, 1) ^ Bx ^ multmodp(d.zpow[pcnt + su.y], d.cseg[x]);
              }
              w_bytes += wave_sum(ins ? 5u * ((seg_of(d, lm.sender) + 1) * (d.SEGW / 8) - (lm.sender >> 3)) + 12u : 0u);
            } else {                                  // few: the whole wave on each insertion
              for (unsigned long long mm = insm; mm; mm &= mm - 1) {
                const int q = __ffsll((long long)mm) - 1;
                const uint32_t x = rdl(lm.sender, q), k = seg_of(d, x);
                const uint32_t hs = x >> 3, nh = (k + 1) * (d.SEGW / 8) - hs;
                w_bytes += 5ull * nh + 12;
                uint32_t praw = 0, pcnt = 0;
                for (uint32_t h = hs + (l * nh) / 64; h < hs + ((l + 1) * nh) / 64; ++h) {
                  uint32_t m8 = hb[h];
                  if (h == hs) m8 &= ~((2u << (x & 7)) - 1u) & 0xFFu;
                  fold_half(d, ztab, h, m8, praw, pcnt);
                }
                wave_combine(d, praw, pcnt);
                praw = rdl(praw, 0); pcnt = rdl(pcnt, 0);
                const uint2 su = s_suf[wv][k + 1];
                const uint32_t Bx = multmodp(d.zpow[su.y], praw) ^ su.x;
                const uint32_t K = mulzc(ztab, Bx, 1) ^ Bx ^ multmodp(d.zpow[pcnt + su.y], d.cseg[x]);
                if (l == (uint32_t)q) Kx = K;
              }
            }
            if (tdbg) t_ins += wall_clock64() - tb;
          }
        }
        g = rdl(mine, (int)(t & 63));
      } else {      // beyond SORT_MAX: next smallest index above the previous one
        if (t == 0 && l == 0) path_hit(d, PATH_PROC_UNSORTED);
        uint32_t best = 0xFFFFFFFFu;
        for (uint32_t q = l; q < icnt; q += 64) {
          const uint32_t v = wc.inbox[ibase + q];
          if ((last_g == 0xFFFFFFFFu || v > last_g) && v < best) best = v;
        }
        g = wave_min(best);
      }
      last_g = g;
      Msg m;
      if (sorted) {
        const int src = (int)(t & 63);
        m.dest = rdl(lm.dest, src); m.sender = rdl(lm.sender, src); m.seq = rdl(lm.seq, src);
        m.kind = rdl(lm.kind, src); m.a = rdl(lm.a, src); m.fp = rdl(lm.fp, src); m.n = rdl(lm.n, src);
        m.off = rdl(lm.off, src);
      } else {
        m = ib.msgs[g];
      }
      const uint32_t s = m.sender;
      if (s != last_sender) {                         // prologue: insert(sender, Known(now)) (:406-415)
        bool was;
        uint8_t b;
        if (sorted) { was = rdl(pre_was, (int)(t & 63)) != 0; b = (uint8_t)rdl(pre_b, (int)(t & 63)); }
        else { was = (bw[s >> 5] >> (s & 31)) & 1u; b = was ? rw[s] : ST_UNKNOWN; }
        if (b == ST_SUSPECT && l < SLOTS && s_susp[wv][l].kind && s_susp[wv][l].peer == s) {
          lat_sample(d, i, s, s_susp[wv][l].since, r);
          s_susp[wv][l].kind = 0;
        }
        w_bytes += (!was ? 4u : 0u) + (b != now ? 5u : 0u);   // bit word, stamp + log entry written
        if (!was) {
          dbg_ins++;
          n++; segs |= seg_bit(d, s);
          if (inc) { R = mulzc(ztab, R, 1) ^ rdl(Kx, (int)(t & 63)); fpstale = true; }
          else dirty = true;
          if (l == 0) const_cast<uint32_t*>(bw)[s >> 5] |= 1u << (s & 31);   // single writer of this row
        }
        if (b != now) {
          if (l == 0) { rw[s] = now; d.flog[(size_t)i * LOGCAP + (fn & (LOGCAP - 1))] = log_entry(s, r); }
          fn++;
          need_sync = true;
        }
        last_sender = s;
        __builtin_amdgcn_wave_barrier();
      }
      // every handler but PingRequest's needs the fingerprint after the prologue, and none changes the
      // membership before it reads it: one call site
      const uint32_t f_cur = m.kind != K_PINGREQ ? fp_now() : 0u;
      switch (m.kind) {
        case K_PING: {                                               // :513-532
          emit(s, K_ACK, i, f_cur, n, 0);
          break;
        }
        case K_PINGREQ: {                                            // :533-545
          const unsigned long long hit = __ballot(l < CSLOTS && s_cur[wv][l].used && s_cur[wv][l].peer == m.a);
          int e = hit ? __ffsll((long long)hit) - 1 : -1;
          if (e < 0) {
            const unsigned long long fr = __ballot(l < CSLOTS && !s_cur[wv][l].used);
            e = fr ? __ffsll((long long)fr) - 1 : -1;
            if (e >= 0 && l == 0) { s_cur[wv][e].used = 1; s_cur[wv][e].peer = m.a; s_cur[wv][e].nobs = 0; }
          }
          wait_lds();
          __builtin_amdgcn_wave_barrier();
          if (e < 0) w_curovf++;
          else if (l == 0) {
            Cur& c = s_cur[wv][e];
            bool dup = false;
            for (uint32_t q = 0; q < c.nobs; ++q) dup |= c.obs[q] == s;
            if (!dup) { if (c.nobs == NOBS) w_curovf++; else c.obs[c.nobs++] = s; }
          }
          wait_lds();
          __builtin_amdgcn_wave_barrier();
          emit(m.a, K_PING, 0, 0, 0, 0);
          break;
        }
        case K_ACK: {                                                // :418-447
          const unsigned long long hit = __ballot(l < CSLOTS && s_cur[wv][l].used && s_cur[wv][l].peer == m.a);
          if (hit) {
            const int e = __ffsll((long long)hit) - 1;
            const uint32_t nobs = s_cur[wv][e].nobs;
            // the entry's observers stay in LDS until a later PingRequest reuses the slot: read in place
            for (uint32_t q = 0; q < nobs; ++q) emit(s_cur[wv][e].obs[q], K_ACK, m.a, m.fp, m.n, 0);
            wait_lds();
            __builtin_amdgcn_wave_barrier();
            if (l == 0) s_cur[wv][e].used = 0;
            wait_lds();
            __builtin_amdgcn_wave_barrier();
          }
          maybe_sync(f_cur, m.a, m.fp, m.n);
          break;
        }
        case K_KPR: {                                                // :473-512
          // reply = {p Known, p != self, p != sender, stamped within SHARE_AGE}, never truncated;
          // > 10240 B is lost at the receiver (Q3), so only the count matters once it exceeds capk
          // The fresh set only grows during a round (stamps rise to now; nothing is removed while
          // messages are handled), so once a reply counted capk + 2 entries every later reply of
          // this node in this round is oversize too: kpr_big[i] = r records that.
          if (need_sync) { wave_mem_sync(); need_sync = false; }
          const uint32_t poff = ob.poff[i] + pay_used;
          uint32_t total = 0;
          uint64_t size = 8 + (d.seglen[i] - ADDR_LEN) + 4 + 8;
          bool over = (d.uniform && kbig == r) || (d.dev & 4096);   // dev 4096: every reply oversize (timing experiments)
          if (over) { w_over++; maybe_sync(f_cur, s, m.fp, m.n); break; }
          auto take = [&](bool ok, uint32_t j) __attribute__((always_inline)) {
            const unsigned long long okm = __ballot(ok);
            const uint32_t pos = total + __popcll(okm & ((1ull << l) - 1ull));
            if (!d.uniform) size += wave_sum(ok ? 18u + d.seglen[j] - ADDR_LEN : 0u);
            if (ok && pos < d.paybound) {
              if (poff + pos < ob.pay_cap) ob.pay[poff + pos] = j;
              else set_err(d, DERR_PAYLOAD);
            }
            total += __popcll(okm);
            if (d.uniform && total > d.capk + 1) over = true;
          };
          // the log ring holds the newest LOGCAP entries: the whole window when complete; otherwise
          // those entries are still exact members of the reply, enough to prove it oversize
          const uint32_t ws = log_window_start(d, i, r);
          const bool complete = fn - ws <= LOGCAP;
          dbg_kpr++;
          // KPR_BATCH x 64 entries per step: all their log, member-bit and stamp loads in flight at once,
          // then taken in log order (the early exit stays between steps)
          constexpr int KPR_BATCH = KB_KPR_BATCH;
          for (uint32_t k0 = complete ? ws : fn - LOGCAP; k0 < fn && !over; k0 += 64 * KPR_BATCH) {
            uint32_t ev[KPR_BATCH], wv4[KPR_BATCH], bv[KPR_BATCH];
#pragma unroll
            for (int u = 0; u < KPR_BATCH; ++u) {
              const uint32_t k = k0 + 64u * u + l;
              ev[u] = k < fn ? d.flog[(size_t)i * LOGCAP + (k & (LOGCAP - 1))] : LOG_INVALID;
            }
#pragma unroll
            for (int u = 0; u < KPR_BATCH; ++u) {
              const uint32_t j = ev[u] == LOG_INVALID ? 0u : ev[u] >> 8;
              wv4[u] = bw[j >> 5];
              bv[u] = rw[j];
            }
            dbg_log += 64 * KPR_BATCH;
            w_bytes += 9ull * (fn - k0 < 64u * KPR_BATCH ? fn - k0 : 64u * KPR_BATCH);   // log entry, member word, stamp
#pragma unroll
            for (int u = 0; u < KPR_BATCH; ++u) {
              if (over) break;                          // wave-uniform
              const uint32_t e = ev[u], j = e >> 8;
              const bool ok = e != LOG_INVALID && j != i && j != s && r - log_round(e, r) < SHARE_AGE &&
                              ((wv4[u] >> (j & 31)) & 1u) && bv[u] == enc(log_round(e, r), r);
              take(ok, j);
            }
          }
          if (!complete && !over) {                   // rare: rescan the row itself
            total = 0;
            size = 8 + (d.seglen[i] - ADDR_LEN) + 4 + 8;
            for (uint32_t c = 0; c < d.W && !over; c += 1024) {
              const uint32_t j0 = c + l * 16;
              const uint4 v = *reinterpret_cast<const uint4*>(rw + j0);
              const uint32_t mb = (bw[j0 >> 5] >> (j0 & 16)) & 0xFFFFu;
              const uint32_t w4[4] = {v.x, v.y, v.z, v.w};
              uint32_t mask = 0;
#pragma unroll
              for (int t2 = 0; t2 < 16; ++t2) {
                const uint32_t b = (w4[t2 >> 2] >> (8 * (t2 & 3))) & 0xFFu, j = j0 + t2;
                mask |= (uint32_t)(((mb >> t2) & 1u) && b >= fresh_thr && j != i && j != s) << t2;
              }
              for (int t2 = 0; t2 < 16; ++t2) take((mask >> t2) & 1u, j0 + t2);
            }
          }
          if (d.uniform && total > d.capk + 1) kbig = r;
          over = d.uniform ? total > d.capk : size > (uint64_t)BUFSZ;
          if (over) w_over++;
          else { emit(s, K_KP, total, 0, 0, poff); pay_used += total; w_bytes += 4ull * total; }
          maybe_sync(f_cur, s, m.fp, m.n);
          break;
        }
        default: break;
      }
    }
    const uint64_t t_after = tdbg ? wall_clock64() : 0;
    if (l < SLOTS) d.susp[(size_t)i * SLOTS + l] = s_susp[wv][l];
    if (l < CSLOTS) d.cur[(size_t)i * CSLOTS + l] = s_cur[wv][l];
    if (inc) fp_now();                              // exact: the touched checkpoints stay marked stale
    if (l == 0) {
      if (segs) atomicOr(&d.sdirty[i], segs);
      d.n[i] = n; d.fp[i] = fp; d.dirty[i] = dirty ? 1 : 0; d.flog_n[i] = fn; d.kpr_big[i] = kbig;
      ob.cnt[i] = oseq;
      wave_ctr_clear(wc, i);
      if (tdbg) {
        const uint32_t tn = (uint32_t)(wall_clock64() - t_node);
        atomicAdd(&d.ctr[C_DBG_TNODE], tn); atomicMax(&d.ctr[C_DBG_TMAX], tn);
        atomicAdd(&d.ctr[C_DBG_TBASE], (uint32_t)t_base); atomicAdd(&d.ctr[C_DBG_TINS], (uint32_t)t_ins);
        atomicAdd(&d.ctr[C_DBG_TSTART], (uint32_t)(t_loop - t_node)); atomicAdd(&d.ctr[C_DBG_TEND], (uint32_t)(wall_clock64() - t_after));
        atomicAdd(&d.ctr[C_DBG_MSGS], icnt);
      }
      if (dbg_fp) { atomicAdd(&d.ctr[C_DBG_FP], dbg_fp); atomicMax(&d.ctr[C_DBG_MAXFP], dbg_fp); }
      if (dbg_ins) atomicAdd(&d.ctr[C_DBG_INS], dbg_ins);
      if (dbg_kpr) { atomicAdd(&d.ctr[C_DBG_KPR], dbg_kpr); atomicAdd(&d.ctr[C_DBG_KPRLOG], dbg_log); }
      if (dbg_base) atomicAdd(&d.ctr[C_DBG_BASE], dbg_base);
    }
    wait_lds();                                       // the LDS slot caches are reused by the next node
    __builtin_amdgcn_wave_barrier();
  }
  if (l == 0) {
    if (w_over) slot_add(d, S_OVERSIZE, w_over);
    if (w_curovf) slot_add(d, S_CUROVF, w_curovf);
    if (w_bytes) slot_add(d, S_PROCB, w_bytes);
  }
}

}  // namespace kb
