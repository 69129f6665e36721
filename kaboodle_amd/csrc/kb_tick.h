// kb_tick.h — the tick (src/kaboodle.rs:746-779): maybe_broadcast_join + handle_suspected_peers, the
// row sweep of ping_random_peer fused with the fingerprint fold, target choice + ping_addrs
// (included by kb_sim.hip).
#pragma once
#include "kb_common.h"

namespace kb {

struct BcastSlots { uint32_t* join; uint32_t* nfail; uint32_t* fail; };

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
  for (int k = 0; k < SLOTS; ++k) if (((occm >> k) & 1ull) && rdl(me.peer, k) < me.peer) myrank++;
  uint32_t npick = 0, nind = 0, nrem = 0;
  uint32_t indirect[SLOTS], removed[SLOTS];
  for (uint32_t t = 0; t < nsusp; ++t) {
    const unsigned long long who = __ballot(occ && myrank == t);
    const int k = __ffsll((long long)who) - 1;
    const uint32_t peer = rdl(me.peer, k);
    const int32_t kind = (int32_t)rdl((uint32_t)me.kind, k), since = (int32_t)rdl((uint32_t)me.since, k);
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
  uint32_t oseq = ob.cnt[i];
  if (npick) {                                            // choose_multiple over the candidate list
    // rank -> id for every pick from the membership bitset alone: the candidates (Known, != self,
    // :571-577) are the members minus self minus the suspect slots (the members whose stamp byte is
    // WaitingFor*), so no stamp byte is read.  Lane l takes ids [128 w, +128) of 16-byte word
    // w = w0 + 64 u + l: 8 words per lane in flight (64 K ids per step, the whole 64K-peer row in one
    // memory round trip); a word resolves the picks whose rank falls in its candidate range (ranks are
    // in address order)
    wait_lds();
    __builtin_amdgcn_wave_barrier();
    const uint4* b4 = reinterpret_cast<const uint4*>(bits_of(d, i));
    uint32_t ex[SLOTS + 1];                               // excluded members: self, the suspects
    ex[0] = i;
#pragma unroll
    for (int k = 0; k < SLOTS; ++k) ex[k + 1] = ((occm >> k) & 1ull) ? rdl(me.peer, k) : 0xFFFFFFFFu;
    uint32_t maxrank = 0;
    for (uint32_t q = 0; q < npick; ++q) maxrank = pr[q] > maxrank ? pr[q] : maxrank;
    const uint32_t n4 = d.NWR / 4;
    uint32_t base = 0;
    constexpr int PB = 8;
    for (uint32_t w0 = 0; w0 < n4 && base <= maxrank; w0 += 64 * PB) {
      uint4 v[PB];
#pragma unroll
      for (int u = 0; u < PB; ++u) { const uint32_t w = w0 + 64u * u + l; v[u] = w < n4 ? b4[w] : make_uint4(0, 0, 0, 0); }
#pragma unroll
      for (int u = 0; u < PB; ++u) {
        if (base > maxrank) break;                        // wave-uniform
        const uint32_t w = w0 + 64u * u + l, id0 = w * 128;
        const uint32_t wd[4] = {v[u].x, v[u].y, v[u].z, v[u].w};
        uint32_t c = __popc(wd[0]) + __popc(wd[1]) + __popc(wd[2]) + __popc(wd[3]);
#pragma unroll
        for (int k = 0; k <= SLOTS; ++k) c -= (ex[k] - id0 < 128u) ? 1u : 0u;   // excluded ids are members
        const uint32_t exl = wave_excl(c), tot = wave_sum(c);
        for (uint32_t q = 0; q < npick; ++q) {
          const uint32_t rk = pr[q];
          if (rk >= base + exl && rk < base + exl + c) {
            uint32_t rem = rk - base - exl, id = 0xFFFFFFFFu;
#pragma unroll
            for (int k = 0; k < 4; ++k) {
              uint32_t m = wd[k];
#pragma unroll
              for (int e = 0; e <= SLOTS; ++e) if ((ex[e] >> 5) == w * 4 + k) m &= ~(1u << (ex[e] & 31));
              const uint32_t pc = __popc(m);
              if (id == 0xFFFFFFFFu) { if (rem < pc) id = id0 + 32 * k + select_in_word(m, rem); else rem -= pc; }
            }
            pid[q] = id;
          }
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
      lat_none(d, i, p);
      segs |= seg_bit(d, p);
      n--;
      for (int c = 0; c < CSLOTS; ++c) if (cu[c].used && cu[c].peer == p) cu[c].used = 0;
      bs.fail[(size_t)i * SLOTS + q] = p;
    }
    bs.nfail[i] = nrem;
    if (nrem) { d.n[i] = n; mark(d, i, segs); slot_add(d, S_RMTIMEOUT, nrem); }
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
  // one list reservation per wave (the list counter is one word)
  const unsigned long long m = __ballot(true);
  const int first = __ffsll((long long)m) - 1;
  uint32_t base = 0;
  if (lane() == (uint32_t)first) base = atomicAdd(&d.ctr[C_TICK], (uint32_t)__popcll(m));
  list[rdl(base, first) + __popcll(m & ((1ull << lane()) - 1ull))] = i;
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
// THE FOLD: generate_fingerprint's checkpoints (:71-83).  Every segment whose membership changed since
// its checkpoint (sdirty) is refolded from the member bits: per 8-id block, raw = raw·Z^popc ⊕
// htab[block][mask], the multiply through four LDS byte tables.  Lane = node: a wave folds 64 rows over
// one column split; workgroups take split blockIdx % S, so each XCD (workgroups are dealt round-robin to
// the 8 XCDs) stays on 1/min(S, 8) of the columns and its slice of htab stays in that XCD's 4 MB L2.
// Runs after A2 (the last membership change of the tick), so the tick ends with every checkpoint fresh.
// ================================================================================================
struct FoldArgs { uint32_t S; };

__global__ __launch_bounds__(256) void k_fold(Dev d, FoldArgs fa) {
  __shared__ uint32_t zb[ZB];
  load_zbtab(d, zb);
  const uint32_t S = fa.S;
  const uint32_t s = blockIdx.x % S;
  const uint32_t g = (blockIdx.x / S) * 4 + (threadIdx.x >> 6);
  const uint32_t i0 = d.lo + g * 64 + lane();
  const bool act = i0 < d.hi && d.alive[i0] && d.uniform;
  const unsigned long long actm = __ballot(act);
  // the fold's byte counter (bench roofline) is summed over the workgroup and added once: one atomic
  // per wave on one address serialises thousands of waves in the memory system
  __shared__ uint32_t s_nb[4];
  uint32_t nbytes = 0;
  if (actm) {
    const uint32_t i = act ? i0 : d.lo + g * 64 + (uint32_t)(__ffsll((long long)actm) - 1);   // idle lanes shadow a live one
    const uint32_t* bw = bits_of(d, i);
    const uint32_t spp = NSEG / S;
    const unsigned long long sd = act ? d.sdirty[i] : 0ull;
    unsigned long long folded = 0;
    for (uint32_t k = s * spp; k < (s + 1) * spp; ++k) {
      const bool mine = (sd >> k) & 1ull;
      if (!__ballot(mine)) continue;                  // wave-uniform: no row of this wave changed here
      const uint32_t c0 = k * d.SEGW, c1 = c0 + d.SEGW;
      uint32_t raw = 0, cnt = 0;
      uint4 mb = *reinterpret_cast<const uint4*>(bw + (c0 >> 5));
      for (uint32_t col = c0; col < c1; col += 128) {
        const uint32_t mw[4] = {mb.x, mb.y, mb.z, mb.w};
        uint32_t hv[16];
        const uint32_t* ht = d.htab + (size_t)(col >> 3) * 256;
#pragma unroll
        for (int h = 0; h < 16; ++h) hv[h] = ht[h * 256 + ((mw[h >> 2] >> (8 * (h & 3))) & 0xFFu)];   // entry 0 is 0
        if (col + 128 < c1) mb = *reinterpret_cast<const uint4*>(bw + ((col + 128) >> 5));   // next step's bits
#pragma unroll
        for (int h = 0; h < 16; ++h) {
          const uint32_t c = __popc((mw[h >> 2] >> (8 * (h & 3))) & 0xFFu);   // Z^0 table is the identity
          raw = mulzb(zb, raw, c) ^ hv[h];
          cnt += c;
        }
      }
      if (mine) { d.segp[(size_t)i * NSEG + k] = make_uint2(raw, cnt); folded |= 1ull << k; nbytes += d.SEGW / 8; }
    }
    if (folded) atomicAnd(&d.sdirty[i], ~folded);
  }
  const uint32_t wb = wave_sum(act ? nbytes : 0u);
  if (lane() == 0) s_nb[threadIdx.x >> 6] = wb;
  __syncthreads();
  if (threadIdx.x == 0) {
    const uint32_t t = s_nb[0] + s_nb[1] + s_nb[2] + s_nb[3];
    if (t) slot_add(d, S_FOLDB, t);
  }
}

// ---- fingerprints of the rows whose membership changed (:71-83), from their fresh checkpoints:
// FP_LANES lanes per row, each combining NSEG / FP_LANES checkpoints (one Z^cnt multiply each), then
// log2(FP_LANES) combine levels across them in address order.  Spreading the 64-multiply chain over
// several lanes gives the SIMDs that many times the waves to hide its latency with.  Runs after
// k_fold; k_tick_post then finds the row clean.
constexpr uint32_t KB_FP_LANES = 8;
constexpr uint32_t FP_LANES = KB_FP_LANES;
__global__ __launch_bounds__(256) void k_fp_rows(Dev d) {
  constexpr uint32_t PER = NSEG / FP_LANES;
  const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
  const uint32_t i = d.lo + t / FP_LANES, part = t % FP_LANES;
  const bool on = i < d.hi && d.uniform && d.alive[i] && d.dirty[i];
  uint32_t raw = 0, cnt = 0;
  if (on) {
    const uint4* sp4 = reinterpret_cast<const uint4*>(d.segp + (size_t)i * NSEG + PER * part);   // two checkpoints per 16 B
    uint4 q[PER / 2];
#pragma unroll
    for (uint32_t k = 0; k < PER / 2; ++k) q[k] = sp4[k];
    uint32_t z[PER];
#pragma unroll
    for (uint32_t k = 0; k < PER; ++k) { const uint32_t c = (k & 1) ? q[k >> 1].w : q[k >> 1].y; z[k] = c ? d.zpow[c] : 0u; }
#pragma unroll
    for (uint32_t k = 0; k < PER; ++k) {
      const uint32_t x = (k & 1) ? q[k >> 1].z : q[k >> 1].x, c = (k & 1) ? q[k >> 1].w : q[k >> 1].y;
      if (c) { raw = multmodp(z[k], raw) ^ x; cnt += c; }
    }
  }
  static_assert(FP_LANES == 8, "the combine below is three DPP levels inside a 16-lane row");
  auto level = [&](uint32_t r2, uint32_t c2, uint32_t st) __attribute__((always_inline)) {   // (part, part + st), part % 2st == 0
    if (on && (part & (2 * st - 1)) == 0) { raw = multmodp(d.zpow[c2], raw) ^ r2; cnt += c2; }
  };
  { const uint32_t r2 = dpp_shl<1>(raw), c2 = dpp_shl<1>(cnt); level(r2, c2, 1); }
  { const uint32_t r2 = dpp_shl<2>(raw), c2 = dpp_shl<2>(cnt); level(r2, c2, 2); }
  { const uint32_t r2 = dpp_shl<4>(raw), c2 = dpp_shl<4>(cnt); level(r2, c2, 4); }
  if (on && part == 0) { d.fp[i] = finish_fp(d, raw, cnt); d.dirty[i] = 0; }
}

// ---- pick the ping target (one of the oldest 5), WaitingForPing(now), Ping; ping_addrs (:550-556);
// ---- refresh the fingerprint from the checkpoints; agreement with the running set.  Thread per node.
__global__ void k_tick_post(Dev d, RowOut ro, OutBuf ob, int32_t r) {
  const uint32_t i = d.lo + blockIdx.x * blockDim.x + threadIdx.x;
  unsigned long long agree = 0;
  if (i < d.hi && d.alive[i]) {
    const uint32_t C = d.C;
    const uint32_t cur = d.a3cur[i];                // the row pass rotated its keys from cur + 1
    const uint32_t p = (cur + 1 == C) ? 0 : cur + 1;
    uint32_t k5[5];                                 // the row pass's five smallest keys, ascending
    const uint4 a = *reinterpret_cast<const uint4*>(ro.part + (size_t)i * 10);
    k5[0] = a.x; k5[1] = a.y; k5[2] = a.z; k5[3] = a.w; k5[4] = ro.part[(size_t)i * 10 + 4];
    uint32_t nc = 0;
    while (nc < 5 && k5[nc] != 0xFFFFFFFFu) nc++;
    uint32_t oseq = ob.cnt[i];
    if (nc) {
      const uint32_t u = philox(i, (uint32_t)r, (uint32_t)P_PING << 24, 0, d.k0, d.k1).x;
      const uint32_t rot = k5[mulhi(u, nc)] & 0xFFFFFFu;
      const uint32_t t = rot + p >= C ? rot + p - C : rot + p;
      const uint32_t rot0 = k5[0] & 0xFFFFFFu;      // the sweep front: just before the oldest candidate
      const uint32_t c1 = rot0 + p >= C ? rot0 + p - C : rot0 + p;
      d.a3cur[i] = c1 == 0 ? C - 1 : c1 - 1;
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

// ---- records from external peers (kb_sim_inject): their wave-0 emissions, in call order ------
// inj[k].pad = the record's KnownPeers offset inside its sender's payload region (the host sums them per sender);
// inj[k].pay_off = where its ids start in `ids`.  One thread: a handful of records per round.
__global__ void k_inject_prep(Dev d, const XRec* inj, uint32_t n, uint32_t* paysum) {
  if (threadIdx.x || blockIdx.x) return;
  for (uint32_t k = 0; k < n; ++k)
    if (local(d, inj[k].sender) && inj[k].kind == K_KP) paysum[inj[k].sender] += inj[k].pay_len;
}
__global__ void k_inject(Dev d, OutBuf ob, const XRec* inj, uint32_t n, const uint32_t* ids) {
  if (threadIdx.x || blockIdx.x) return;
  for (uint32_t k = 0; k < n; ++k) {
    const XRec x = inj[k];
    if (!local(d, x.sender)) continue;
    const uint32_t slot = ob.cnt[x.sender];
    if (slot >= ob.cap[x.sender]) { set_err(d, DERR_OUTBOX); continue; }
    const uint32_t off = ob.poff[x.sender] + x.pad;
    if (x.kind == K_KP) for (uint32_t q = 0; q < x.pay_len; ++q) ob.pay[off + q] = ids[x.pay_off + q];
    ob.msgs[ob.off[x.sender] + slot] = Msg{x.dest, x.sender, slot, x.kind, x.kind == K_KP ? x.pay_len : x.a, x.fp, x.n,
                                           x.kind == K_KP ? off : 0u};
    ob.cnt[x.sender] = slot + 1;
  }
}

// round results for the host, {Join broadcasts, Failed broadcasts, error}: into its mapped pinned buffer
// (rres, seq != 0: the host waits for it), and into rr on the device (sharded: all-gathered first)
__global__ void k_round_end(Dev d, int32_t r, const uint32_t* tot, uint32_t* rres, uint32_t seq, uint32_t* rr) {
  if (threadIdx.x || blockIdx.x) return;
  const uint32_t a = d.ctr[C_AGREE], al = d.ctr[C_ALIVE];
  d.ctr[C_LASTAGREE] = a; d.ctr[C_LASTALIVE] = al;
  if (d.lo == 0) d.stats[S_ALIVER] += al;          // the running set is replicated: shard 0 counts it
  const uint32_t v[3] = {tot[0], tot[1], d.ctr[C_ERR]};
  rr[0] = v[0]; rr[1] = v[1]; rr[2] = v[2];
  if (seq) pin_publish(rres, v, 3, seq);
  if (al && a == al) {
    if ((int32_t)d.ctr[C_FIRSTCONV] < 0) d.ctr[C_FIRSTCONV] = (uint32_t)r;
    d.ctr[C_LASTCONV] = (uint32_t)r;
  }
  d.ctr[C_AGREE] = 0; d.ctr[C_ALIVE] = 0; d.ctr[C_TICK] = 0;
}

}  // namespace kb
