// kb_sim.hip — MI355X (gfx950) implementation of the Kaboodle SWIM round as a bulk-synchronous
// simulator over HBM-resident structure-of-arrays tables.  Exposes the C ABI of include/kaboodle_sim.h.
//
// Round pipeline, one HIP stream, no host round-trips except one 8-byte read per round:
//   k_rebase (every 64 rounds)      stamp window shift                       
//   k_events / k_churn_*            Kaboodle::start/stop, churn              src/lib.rs:136-183
//   k_template, k_truefp            per-16-id CRC templates of the running set, true fingerprint
//   k_phaseB                        handle_incoming_broadcasts (Failed, Join) src/kaboodle.rs:256-311
//   k_resp_list, k_resp_build       maybe_send_known_peers_to_peer           src/kaboodle.rs:356-392
//   k_tick_pre                      maybe_broadcast_join + handle_suspected_peers :228-251, :558-653
//   k_sweep    <- dominant kernel   ping_random_peer row sweep + generate_fingerprint :655-703, :71-83
//   k_tick_post                     ping target, handle_incoming_ping_requests :655-703, :550-556
//   waves: k_route, k_scan, k_scatter, k_kp_insert, k_kp_prologue, k_touch_fix, k_proc
//                                   handle_incoming_messages                 src/kaboodle.rs:394-548
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <string.h>
#include <stdlib.h>
#include <string>
#include <vector>
#include <algorithm>
#include <array>
#include "kb_device.h"
#include "../../include/kaboodle_sim.h"

using namespace kb;

// ================================================================================================
// Device state
// ================================================================================================
enum StatIdx {
  S_PING, S_PINGREQ, S_ACK, S_KP, S_KPR, S_BJOIN, S_BFAIL, S_DEAD, S_LOSS, S_WINDOW, S_OVERSIZE, S_PART, S_BDROP,
  S_RMTIMEOUT, S_RMFAILED, S_JRESP, S_CUROVF, S_CLEAVE, S_CJOIN, NSTAT
};
// device scalar counters
enum CtrIdx {
  C_KP, C_TOUCH, C_ACTIVE, C_TOT0, C_TOT1, C_TOT2, C_TOT3, C_AGREE, C_ALIVE, C_LEAVES, C_NEXTFREE, C_NF, C_NJ,
  C_ERR, C_FIRSTCONV, C_LASTCONV, C_LASTAGREE, C_LASTALIVE, NCTR
};

struct Dev {
  uint32_t C, W, SEG;           // capacity, row stride (multiple of 1024), bytes per lane segment (W/64)
  uint32_t k0, k1;
  uint32_t loss_thr, churn_thr;
  int32_t fault_end;
  uint32_t failed_mode;
  uint32_t pgroups;
  int32_t pstart, pend;
  uint32_t uniform, L;          // uniform segment length (20 + id_len) when uniform != 0
  uint32_t capk, capj;          // KnownPeers caps: KPR reply (size <= 10240), Join response (size < 10240)
  uint32_t paybound;            // payload entries reserved per KPR reply
  uint8_t* stamp;
  uint8_t* alive;
  int32_t* start_round;
  uint32_t* n;
  uint32_t* fp;
  uint8_t* dirty;
  int32_t* last_bcast;
  Susp* susp;
  Cur* cur;
  uint32_t* paq;
  uint32_t* paq_n;
  uint32_t* cseg;
  uint32_t* segmul;
  uint32_t* seglen;
  uint32_t* zpow;               // Z^k, Z = x^(8L), k in [0, C+1]
  uint32_t* ztab;               // [17][8][16] nibble tables of multiplication by Z^c
  Tmpl* tmpl;                   // [W/16] running-set block raws (true fingerprint)
  uint32_t* htab;               // [(W/8) * 256] crc0 fold of every member pattern of every 8-id half block
  unsigned long long* stats;
  uint32_t* ctr;
  uint32_t* truefp;
};

__device__ inline void set_err(const Dev& d, uint32_t e) { atomicCAS(&d.ctr[C_ERR], 0u, e); }
__device__ inline bool faults(const Dev& d, int32_t r) { return d.fault_end < 0 || r < d.fault_end; }
__device__ inline bool part_blocks(const Dev& d, int32_t r, uint32_t a, uint32_t b) {
  if (d.pgroups <= 1 || r < d.pstart || r >= d.pend) return false;
  return ((uint64_t)a * d.pgroups / d.C) != ((uint64_t)b * d.pgroups / d.C);
}
__device__ inline uint8_t* row_of(const Dev& d, uint32_t i) { return d.stamp + (size_t)i * d.W; }

// multiplication by Z^c (c in 0..16) through LDS nibble tables (conflict-free: 16 words per table)
__device__ inline uint32_t mulzc(const uint32_t* tab, uint32_t x, uint32_t c) {
  if (c == 0) return x;
  const uint32_t* t = tab + c * 128;
  return t[x & 15] ^ t[16 + ((x >> 4) & 15)] ^ t[32 + ((x >> 8) & 15)] ^ t[48 + ((x >> 12) & 15)] ^
         t[64 + ((x >> 16) & 15)] ^ t[80 + ((x >> 20) & 15)] ^ t[96 + ((x >> 24) & 15)] ^ t[112 + (x >> 28)];
}
constexpr int ZT = 9;             // LDS nibble tables for Z^0..Z^8
__device__ inline void load_ztab(const Dev& d, uint32_t* lds) {
  for (uint32_t k = threadIdx.x; k < ZT * 128; k += blockDim.x) lds[k] = d.ztab[k];
  __syncthreads();
}
// 4-bit "byte != 0" mask of a little-endian dword (SWAR)
__device__ inline uint32_t nzmask4(uint32_t x) {
  const uint32_t y = (((x & 0x7F7F7F7Fu) + 0x7F7F7F7Fu) | x) & 0x80808080u;
  return ((y >> 7) | (y >> 14) | (y >> 21) | (y >> 28)) & 0xFu;
}
__device__ inline uint32_t nzmask16(const uint32_t (&w)[4]) {
  return nzmask4(w[0]) | (nzmask4(w[1]) << 4) | (nzmask4(w[2]) << 8) | (nzmask4(w[3]) << 12);
}
// Fold the members (mask nz, bit t = id blk+t) of one 16-id block into (raw, cnt): per 8-id half one
// table lookup of that member pattern's crc0 and one multiplication by Z^popcount.  Exact for any mask.
__device__ inline void fold16(const Dev& d, const uint32_t* ztab, uint32_t blk, uint32_t nz, uint32_t& raw,
                              uint32_t& cnt) {
  const uint32_t m0 = nz & 0xFFu, m1 = nz >> 8;
  const uint32_t* h = d.htab + (size_t)(blk >> 3) * 256;
  if (m0) { const uint32_t c = __popc(m0); raw = mulzc(ztab, raw, c) ^ h[m0]; cnt += c; }
  if (m1) { const uint32_t c = __popc(m1); raw = mulzc(ztab, raw, c) ^ h[256 + m1]; cnt += c; }
}
// x^(8*len) for arbitrary len (non-uniform identities only; small capacities)
__device__ inline uint32_t xpow8_dev(uint64_t nbytes) {
  uint32_t res = 0x80000000u, sq = 0x00800000u;
  while (nbytes) { if (nbytes & 1) res = multmodp(sq, res); sq = multmodp(sq, sq); nbytes >>= 1; }
  return res;
}

// ---- map operations, single thread (node i's own state only) ------------------------------------
__device__ inline void susp_clear(const Dev& d, uint32_t i, uint32_t p) {
  Susp* s = d.susp + (size_t)i * SLOTS;
  for (int k = 0; k < SLOTS; ++k) if (s[k].kind && s[k].peer == p) s[k].kind = 0;
}
__device__ void node_start(const Dev& d, uint32_t i, int32_t r) {
  uint8_t* rw = row_of(d, i);
  uint8_t b = rw[i];
  if (b == ST_SUSPECT) susp_clear(d, i, i);
  if (b == ST_UNKNOWN) d.n[i] += 1;
  rw[i] = enc(r, r);
  d.alive[i] = 1; d.start_round[i] = r; d.dirty[i] = 1; d.last_bcast[i] = NONE_ROUND; d.paq_n[i] = 0;
  for (int k = 0; k < CSLOTS; ++k) d.cur[(size_t)i * CSLOTS + k].used = 0;
}
__device__ void node_stop(const Dev& d, uint32_t i) {
  uint8_t* rw = row_of(d, i);
  uint8_t b = rw[i];
  if (b != ST_UNKNOWN) {
    if (b == ST_SUSPECT) susp_clear(d, i, i);
    rw[i] = ST_UNKNOWN; d.n[i] -= 1; d.dirty[i] = 1;
  }
  d.alive[i] = 0; d.paq_n[i] = 0;
}

// block-wide sum of one value per thread (blockDim <= 1024), result valid in thread 0
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
  unsigned long long t = block_sum(v);
  if (threadIdx.x == 0 && t) atomicAdd(&d.stats[idx], t);
}

// ================================================================================================
// Round-start kernels
// ================================================================================================
__global__ void k_rebase(Dev d) {
  const size_t total = (size_t)d.C * d.W / 16;
  uint4* p = reinterpret_cast<uint4*>(d.stamp);
  for (size_t k = (size_t)blockIdx.x * blockDim.x + threadIdx.x; k < total; k += (size_t)gridDim.x * blockDim.x) {
    uint4 v = p[k];
    uint32_t w[4] = {v.x, v.y, v.z, v.w};
    bool any = false;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      uint32_t x = w[q], y = 0;
#pragma unroll
      for (int t = 0; t < 4; ++t) {
        uint32_t b = (x >> (8 * t)) & 0xFF;
        if (b > ST_ANCIENT) { b = b - EPOCH > ST_ANCIENT ? b - EPOCH : ST_ANCIENT; any = true; }
        y |= b << (8 * t);
      }
      w[q] = y;
    }
    if (any) p[k] = make_uint4(w[0], w[1], w[2], w[3]);
  }
}

struct Event { uint32_t node, stop; };
__global__ void k_events(Dev d, const Event* ev, uint32_t nev, int32_t r) {
  if (threadIdx.x || blockIdx.x) return;
  for (uint32_t k = 0; k < nev; ++k) {
    uint32_t i = ev[k].node;
    if (ev[k].stop) { if (d.alive[i]) node_stop(d, i); }
    else if (!d.alive[i]) node_start(d, i, r);
  }
}

__global__ void k_churn_leave(Dev d, int32_t r) {
  uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  unsigned long long left = 0;
  if (i < d.C && d.alive[i] && d.start_round[i] != r) {
    if (philox(i, (uint32_t)r, (uint32_t)P_CHURN << 24, 0, d.k0, d.k1).x < d.churn_thr) { node_stop(d, i); left = 1; }
  }
  unsigned long long t = block_sum(left);
  if (threadIdx.x == 0 && t) atomicAdd(&d.ctr[C_LEAVES], (uint32_t)t);
}
__global__ void k_churn_join(Dev d, int32_t r) {
  const uint32_t leaves = d.ctr[C_LEAVES];
  const uint32_t nf = d.ctr[C_NEXTFREE];
  const uint32_t joins = leaves < d.C - nf ? leaves : d.C - nf;
  for (uint32_t k = threadIdx.x; k < joins; k += blockDim.x) node_start(d, nf + k, r);
  __syncthreads();
  if (threadIdx.x == 0) {
    d.ctr[C_NEXTFREE] = nf + joins;
    d.ctr[C_LEAVES] = 0;
    d.stats[S_CLEAVE] += leaves;
    d.stats[S_CJOIN] += joins;
  }
}

// per-16-id block templates of the running set + running count
__global__ void k_template(Dev d) {
  const uint32_t b = blockIdx.x * blockDim.x + threadIdx.x;
  unsigned long long alive_cnt = 0;
  if (b < d.W / 16) {
    uint32_t raw = 0, mask = 0, cnt = 0;
    for (uint32_t t = 0; t < 16; ++t) {
      uint32_t j = b * 16 + t;
      if (j < d.C && d.alive[j]) { mask |= 1u << t; cnt++; }
    }
    if (d.uniform) {
      const uint32_t m0 = mask & 0xFFu, m1 = mask >> 8;
      if (m0) raw = d.htab[(size_t)(2 * b) * 256 + m0];
      if (m1) raw = multmodp(d.zpow[__popc(m1)], raw) ^ d.htab[(size_t)(2 * b + 1) * 256 + m1];
    }
    d.tmpl[b].raw = raw;
    d.tmpl[b].mask_cnt = mask | (cnt << 16);
    alive_cnt = cnt;
  }
  unsigned long long t = block_sum(alive_cnt);
  if (threadIdx.x == 0 && t) atomicAdd(&d.ctr[C_ALIVE], (uint32_t)t);
}
// fingerprint of the true running set: ordered reduction of the templates (one workgroup)
__global__ void k_truefp(Dev d) {
  __shared__ uint32_t sraw[1024], scnt[1024];
  const uint32_t nb = d.W / 16, T = blockDim.x, t = threadIdx.x;
  if (!d.uniform) {
    if (t == 0) {
      uint32_t raw = 0; uint64_t len = 0;
      for (uint32_t j = 0; j < d.C; ++j)
        if (d.alive[j]) { raw = multmodp(d.segmul[j], raw) ^ d.cseg[j]; len += d.seglen[j]; }
      d.truefp[0] = raw ^ multmodp(xpow8_dev(len), 0xFFFFFFFFu) ^ 0xFFFFFFFFu;
    }
    return;
  }
  const uint32_t per = (nb + T - 1) / T;
  uint32_t raw = 0, cnt = 0;
  for (uint32_t b = t * per; b < (t + 1) * per && b < nb; ++b) {
    uint32_t c = d.tmpl[b].mask_cnt >> 16;
    if (c) { raw = multmodp(d.zpow[c], raw) ^ d.tmpl[b].raw; cnt += c; }
  }
  sraw[t] = raw; scnt[t] = cnt;
  __syncthreads();
  for (uint32_t s = 1; s < T; s <<= 1) {
    uint32_t nr = 0, nc = 0; bool w = (t % (2 * s) == 0) && t + s < T;
    if (w) { nr = multmodp(d.zpow[scnt[t + s]], sraw[t]) ^ sraw[t + s]; nc = scnt[t] + scnt[t + s]; }
    __syncthreads();
    if (w) { sraw[t] = nr; scnt[t] = nc; }
    __syncthreads();
  }
  if (t == 0) d.truefp[0] = sraw[0] ^ multmodp(d.zpow[scnt[0]], 0xFFFFFFFFu) ^ 0xFFFFFFFFu;
}

// ================================================================================================
// Broadcast phase: Failed then Join deliveries of round r-1's broadcasts (src/kaboodle.rs:256-311)
// ================================================================================================
struct PhaseB {
  const BCast* bfail; uint32_t nf;
  const uint32_t* gid;   // per Failed entry: index of the first entry naming the same peer
  const uint8_t* dep;    // per Failed entry: its sender is named as failed by an earlier entry
  const BCast* bjoin; uint32_t nj; uint32_t JW;
  unsigned long long* newmask; unsigned long long* respmask;   // [C * JW]
  uint32_t* nresp; uint32_t* paysum; uint32_t* nbase;           // per node
};

__device__ inline bool bcast_lost(const Dev& d, uint32_t recv, const BCast& b, int32_t r, bool& part) {
  part = part_blocks(d, r, b.sender, recv);
  if (part) return true;
  if (!faults(d, r) || d.loss_thr == 0) return false;
  return philox(recv, (uint32_t)r, ((uint32_t)P_BLOSS << 24) | b.bseq, b.sender, d.k0, d.k1).x < d.loss_thr;
}

// Per-list facts about the Failed broadcasts (identical for every receiver).
__global__ void k_bfail_prep(const BCast* bf, uint32_t nf, uint32_t* gid, uint8_t* dep) {
  const uint32_t q = blockIdx.x * blockDim.x + threadIdx.x;
  if (q >= nf) return;
  const uint32_t p = bf[q].peer, sn = bf[q].sender;
  uint32_t g = q; uint8_t dp = 0;
  for (uint32_t k = 0; k < q; ++k) {
    const uint32_t pk = bf[k].peer;
    if (pk == p && g == q) g = k;
    if (pk == sn) dp = 1;
  }
  gid[q] = g; dep[q] = dp;
}

constexpr uint32_t FAIL_BITS = 16384;   // Failed entries deduplicated through an LDS bitmap per wave

__global__ __launch_bounds__(256) void k_phaseB(Dev d, PhaseB pb, int32_t r) {
  __shared__ uint32_t s_gbits[4][FAIL_BITS / 32];
  const uint32_t i = blockIdx.x * 4 + (threadIdx.x >> 6);
  const uint32_t l = lane();
  if (i >= d.C) return;
  if (!d.alive[i] || d.start_round[i] >= r) {
    if (l == 0) { pb.nresp[i] = 0; pb.paysum[i] = 0; }
    return;
  }
  uint8_t* rw = row_of(d, i);
  uint32_t n = d.n[i];
  const uint32_t n0 = n;
  uint32_t lost_cnt = 0, removed_cnt = 0;
  // ---- Failed(p) group (src/kaboodle.rs:268-283) ----
  // Entries are independent unless a sender was itself named as failed by an earlier entry (dep):
  // process chunks in parallel (dedup of repeated peers through gid) until such an entry would act,
  // then continue with the exact in-order loop.
  const uint32_t wv = threadIdx.x >> 6;
  const bool honour = d.failed_mode == KB_FAILED_SIM_SENDER;
  bool exact = pb.nf > FAIL_BITS;
  uint32_t c0 = 0;
  if (!exact && pb.nf) {
    for (uint32_t w = l; w < (pb.nf + 31) / 32; w += 64) s_gbits[wv][w] = 0;
    __builtin_amdgcn_s_waitcnt(0);
    __builtin_amdgcn_wave_barrier();
    uint32_t rem_lane = 0;
    for (uint32_t c = 0; c < pb.nf; c += 64) {
      const uint32_t e = c + l;
      const bool valid = e < pb.nf;
      BCast b = valid ? pb.bfail[e] : BCast{0xFFFFFFFFu, 0xFFFFFFFFu, 0, 0};
      bool part = false;
      const bool lost = valid && b.sender != i && bcast_lost(d, i, b, r, part);
      const uint32_t bs = valid ? rw[b.sender] : 0, bp = valid ? rw[b.peer] : 0;
      const bool cond = valid && b.sender != i && !lost && b.peer != i && honour && bs != ST_UNKNOWN &&
                        bp != ST_UNKNOWN;
      if (__ballot(cond && pb.dep[e])) { exact = true; c0 = c; break; }
      lost_cnt += __popcll(__ballot(lost));
      if (cond) {
        const uint32_t g = pb.gid[e];
        const uint32_t old = atomicOr(&s_gbits[wv][g >> 5], 1u << (g & 31));
        if (!(old & (1u << (g & 31)))) rem_lane++;
        if (bp == ST_SUSPECT) susp_clear(d, i, b.peer);
        rw[b.peer] = ST_UNKNOWN;
      }
    }
    const uint32_t rm = wave_sum(rem_lane);
    removed_cnt += rm; n -= rm;
    wave_mem_sync();
  }
  if (exact) {
    for (uint32_t c = c0; c < pb.nf; c += 64) {
      const uint32_t e = c + l;
      const bool valid = e < pb.nf;
      BCast b = valid ? pb.bfail[e] : BCast{0xFFFFFFFFu, 0xFFFFFFFFu, 0, 0};
      bool part = false;
      const bool lost = valid && b.sender != i && bcast_lost(d, i, b, r, part);
      const uint32_t bs = valid ? rw[b.sender] : 0, bp = valid ? rw[b.peer] : 0;
      unsigned long long rem = 0;
      const uint32_t m = pb.nf - c < 64 ? pb.nf - c : 64;
      for (uint32_t q = 0; q < m; ++q) {
        const uint32_t s_q = bcast(b.sender, q), p_q = bcast(b.peer, q);
        if (s_q == i || bcast((uint32_t)lost, q) || p_q == i || !honour) continue;
        const bool s_gone = (__ballot(b.peer == s_q) & rem) != 0;     // removed earlier in this chunk
        if (bcast(bs, q) == ST_UNKNOWN || s_gone) continue;           // sender must be a mesh member
        const bool p_gone = (__ballot(b.peer == p_q) & rem) != 0;
        if (bcast(bp, q) != ST_UNKNOWN && !p_gone) rem |= 1ull << q;
      }
      lost_cnt += __popcll(__ballot(lost));
      if ((rem >> l) & 1ull) {
        if (bp == ST_SUSPECT) susp_clear(d, i, b.peer);
        rw[b.peer] = ST_UNKNOWN;
      }
      removed_cnt += __popcll(rem);
      n -= __popcll(rem);
      wave_mem_sync();
    }
  }
  const uint32_t nbase = n;
  // ---- Join{addr} group (src/kaboodle.rs:284-304) ----
  uint32_t nresp = 0, paysum = 0;
  for (uint32_t c = 0; c < pb.nj; c += 64) {
    const uint32_t e = c + l;
    const bool valid = e < pb.nj;
    BCast b = valid ? pb.bjoin[e] : BCast{0xFFFFFFFFu, 0, 0, 0};
    bool part = false;
    const bool lost = valid && b.sender != i && bcast_lost(d, i, b, r, part);
    const bool deliver = valid && b.sender != i && !lost;
    const uint32_t ba = deliver ? rw[b.sender] : 0xFF;
    const unsigned long long newm = __ballot(deliver && ba == ST_UNKNOWN);
    const bool isnew = (newm >> l) & 1ull;
    // n right after inserting this joiner = n before the chunk + new joiners up to and including it
    const uint32_t nq = n + __popcll(newm & ((2ull << l) - 1ull));
    bool resp = false;
    if (isnew) {                                   // should_respond_to_broadcast :333-354
      const int64_t o = (int64_t)nq - 2;
      if (o <= 0) resp = true;
      else {
        int64_t pct = 100 - o * o; if (pct < 1) pct = 1;
        const uint32_t u = philox(i, (uint32_t)r, (uint32_t)P_RESPOND << 24, b.sender, d.k0, d.k1).x;
        resp = (int64_t)mulhi(u, 100) < pct;
      }
    }
    const unsigned long long respm = __ballot(resp);
    if (deliver) {
      if (ba == ST_SUSPECT) susp_clear(d, i, b.sender);
      rw[b.sender] = enc(r, r);
    }
    const uint32_t sz = resp ? (d.uniform ? (nq < d.capj ? nq : d.capj) : nq) : 0;
    paysum += wave_sum(sz);
    nresp += __popcll(respm);
    n += __popcll(newm);
    lost_cnt += __popcll(__ballot(lost));
    if (l == 0) {
      pb.newmask[(size_t)i * pb.JW + c / 64] = newm;
      pb.respmask[(size_t)i * pb.JW + c / 64] = respm;
    }
  }
  if (l == 0) {
    d.n[i] = n;
    if (n != n0 || removed_cnt) d.dirty[i] = 1;
    pb.nresp[i] = nresp; pb.paysum[i] = paysum; pb.nbase[i] = nbase;
    if (lost_cnt) atomicAdd(&d.stats[S_BDROP], lost_cnt);
    if (removed_cnt) atomicAdd(&d.stats[S_RMFAILED], removed_cnt);
    if (nresp) atomicAdd(&d.stats[S_JRESP], nresp);
  }
}

// ================================================================================================
// Exclusive scan over up to 4 arrays of length n (+ optional compaction of indices j with in[0][j] != 0),
// two fully parallel passes over 1024-element tiles: per-tile sums, then per-tile offsets + local scan.
// ================================================================================================
struct ScanArgs {
  const uint32_t* in[4]; uint32_t* out[4]; int narr; uint32_t n;
  uint32_t* totals;   // device, narr values (+ list count at totals[4] when list != null)
  uint32_t* list; uint32_t* list_count;
  uint32_t addc[4];   // constant added to every element of array q before scanning
  uint32_t* tiles;    // workspace [5 * ntiles]
  uint32_t ntiles;
};
__device__ inline uint32_t scan_val(const ScanArgs& a, int q, uint32_t j) {
  if (q == 4) return a.in[0][j] != 0;
  return (a.in[q] ? a.in[q][j] : 0) + a.addc[q];
}
__global__ __launch_bounds__(1024) void k_scan_tiles(ScanArgs a) {
  __shared__ uint32_t red[5][16];
  const uint32_t j = blockIdx.x * 1024 + threadIdx.x;
  const int nq = a.list ? 5 : a.narr;
  for (int q = 0; q < 5; ++q) {
    if (q >= a.narr && !(q == 4 && a.list)) continue;
    uint32_t v = j < a.n ? scan_val(a, q, j) : 0;
    v = wave_sum(v);
    if (lane() == 0) red[q][threadIdx.x >> 6] = v;
  }
  __syncthreads();
  if (threadIdx.x < 5 && (threadIdx.x < (uint32_t)a.narr || (threadIdx.x == 4 && a.list))) {
    uint32_t t = 0;
    for (int w = 0; w < 16; ++w) t += red[threadIdx.x][w];
    a.tiles[threadIdx.x * a.ntiles + blockIdx.x] = t;
  }
  (void)nq;
}
__global__ __launch_bounds__(1024) void k_scan_apply(ScanArgs a) {
  __shared__ uint32_t base[5], red[5][16], wpre[5][16];
  const uint32_t tile = blockIdx.x, t = threadIdx.x;
  const uint32_t j = tile * 1024 + t;
  for (int q = 0; q < 5; ++q) {
    const bool on = q < a.narr || (q == 4 && a.list);
    uint32_t s = 0;
    if (on) for (uint32_t k = t; k < tile; k += 1024) s += a.tiles[q * a.ntiles + k];
    s = wave_sum(s);
    if (lane() == 0) red[q][t >> 6] = s;
  }
  __syncthreads();
  if (t < 5) { uint32_t s = 0; for (int w = 0; w < 16; ++w) s += red[t][w]; base[t] = s; }
  __syncthreads();
  uint32_t v[5], ex[5];
  for (int q = 0; q < 5; ++q) {
    const bool on = q < a.narr || (q == 4 && a.list);
    v[q] = (on && j < a.n) ? scan_val(a, q, j) : 0;
    ex[q] = wave_excl(v[q]);
    const uint32_t tot = wave_sum(v[q]);
    if (lane() == 0) wpre[q][t >> 6] = tot;
  }
  __syncthreads();
  if (t < 5) { uint32_t run = 0; for (int w = 0; w < 16; ++w) { uint32_t x = wpre[t][w]; wpre[t][w] = run; run += x; } }
  __syncthreads();
  for (int q = 0; q < a.narr; ++q) if (j < a.n) a.out[q][j] = base[q] + wpre[q][t >> 6] + ex[q];
  if (a.list && j < a.n && v[4]) a.list[base[4] + wpre[4][t >> 6] + ex[4]] = j;
  if (tile == gridDim.x - 1 && t == 1023) {
    for (int q = 0; q < a.narr; ++q) a.totals[q] = base[q] + wpre[q][15] + ex[q] + v[q];
    if (a.list) { const uint32_t c = base[4] + wpre[4][15] + ex[4] + v[4]; a.totals[4] = c; if (a.list_count) *a.list_count = c; }
  }
}

// ================================================================================================
// Join responses: KnownPeers of every map entry (src/kaboodle.rs:356-392)
// ================================================================================================
struct RespItem { uint32_t node, k, nk, q, poff, pad[3]; };
struct OutBuf { Msg* msgs; uint32_t* pay; uint32_t* off; uint32_t* cap; uint32_t* cnt; uint32_t* poff; uint32_t msg_cap, pay_cap; };

__global__ void k_resp_list(Dev d, PhaseB pb, const uint32_t* resp_off, const uint32_t* pay_off, RespItem* items,
                            OutBuf ob) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= d.C) return;
  const uint32_t nr = pb.nresp[i];
  ob.cnt[i] = nr;
  if (!nr) return;
  uint32_t pos = resp_off[i], poff = pay_off[i], q = 0, ins = 0;
  for (uint32_t w = 0; w < pb.JW; ++w) {
    unsigned long long rm = pb.respmask[(size_t)i * pb.JW + w], nm = pb.newmask[(size_t)i * pb.JW + w];
    while (rm) {
      const int bit = __ffsll((long long)rm) - 1;
      rm &= rm - 1;
      const uint32_t nk = pb.nbase[i] + ins + __popcll(nm & ((1ull << bit) - 1ull)) + 1;
      const uint32_t sz = d.uniform ? (nk < d.capj ? nk : d.capj) : nk;
      items[pos + q] = RespItem{i, w * 64 + (uint32_t)bit, nk, q, poff, {0, 0, 0}};
      poff += sz; q++;
    }
    ins += __popcll(nm);
  }
}

// Lane-contiguous enumeration of map members of row i excluding the joiners inserted after list
// index k (they were not yet in the map when the response was sent).
struct ExclCtx { const BCast* bjoin; const unsigned long long* newm; uint32_t nj; uint32_t kidx; uint32_t aid; };
__device__ inline uint32_t lower_bound_join(const BCast* bj, uint32_t lo, uint32_t hi, uint32_t id) {
  while (lo < hi) { uint32_t mid = (lo + hi) >> 1; if (bj[mid].sender < id) lo = mid + 1; else hi = mid; }
  return lo;
}
__device__ inline bool newbit(const unsigned long long* nm, uint32_t e) { return (nm[e >> 6] >> (e & 63)) & 1ull; }

__global__ __launch_bounds__(64) void k_resp_build(Dev d, PhaseB pb, const RespItem* items, const uint32_t* nitems_p,
                                                   OutBuf ob, int32_t r) {
  __shared__ uint32_t bits[FLOYD_MAX_N / 32];
  __shared__ uint32_t draws[1024];
  const uint32_t l = lane();
  const uint32_t nitems = *nitems_p;
  for (uint32_t it = blockIdx.x; it < nitems; it += gridDim.x) {
    const RespItem item = items[it];
    const uint32_t i = item.node, K = item.k, nk = item.nk;
    const uint32_t a = pb.bjoin[K].sender;
    const uint8_t* rw = row_of(d, i);
    const unsigned long long* nm = pb.newmask + (size_t)i * pb.JW;
    const bool sample = d.uniform && nk > d.capj;
    const uint32_t cap = sample ? d.capj : nk;
    // lane segment
    uint32_t lo = l * d.SEG, hi = lo + d.SEG;
    if (hi > d.C) hi = d.C;
    if (lo > hi) lo = hi;
    // exclusions in [max(lo, a+1), hi): join entries after K with the new bit
    const uint32_t xlo = lo > a + 1 ? lo : a + 1;
    uint32_t e0 = xlo < hi ? lower_bound_join(pb.bjoin, K + 1, pb.nj, xlo) : pb.nj;
    const uint32_t e1 = xlo < hi ? lower_bound_join(pb.bjoin, e0, pb.nj, hi) : pb.nj;
    uint32_t excl = 0;
    for (uint32_t e = e0; e < e1; ++e) excl += newbit(nm, e);
    uint32_t mem = 0;
    for (uint32_t j = lo; j < hi; j += 16) {
      uint4 v = *reinterpret_cast<const uint4*>(rw + j);
      uint32_t w4[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
      for (int t = 0; t < 16; ++t) mem += (j + t < hi) && ((w4[t >> 2] >> (8 * (t & 3))) & 0xFF);
    }
    const uint32_t lane_cnt = mem - excl;
    const uint32_t lane_off = wave_excl(lane_cnt);
    const uint32_t total = wave_sum(lane_cnt);
    if (total != nk && l == 0) set_err(d, DERR_RESP);
    uint32_t out_base = 0;     // selected ranks before this lane
    if (sample) {
      if (nk > FLOYD_MAX_N) { if (l == 0) set_err(d, DERR_FLOYD); continue; }
      for (uint32_t w = l; w < (nk + 31) / 32; w += 64) bits[w] = 0;
      for (uint32_t t4 = l; t4 < (cap + 3) / 4; t4 += 64) {
        U4 u = philox(i, (uint32_t)r, ((uint32_t)P_TRUNC << 24) | t4, a, d.k0, d.k1);
        draws[4 * t4] = u.x; draws[4 * t4 + 1] = u.y; draws[4 * t4 + 2] = u.z; draws[4 * t4 + 3] = u.w;
      }
      __syncthreads();
      if (l == 0) {                        // Floyd: uniform cap-subset of [0, nk)
        for (uint32_t t = 0; t < cap; ++t) {
          const uint32_t j = nk - cap + t;
          const uint32_t v = mulhi(draws[t], j + 1);
          const uint32_t x = (bits[v >> 5] >> (v & 31)) & 1u ? j : v;
          bits[x >> 5] |= 1u << (x & 31);
        }
      }
      __syncthreads();
      // selected ranks inside [lane_off, lane_off + lane_cnt)
      uint32_t sel = 0;
      for (uint32_t q = lane_off; q < lane_off + lane_cnt;) {
        if ((q & 31) == 0 && q + 32 <= lane_off + lane_cnt) { sel += __popc(bits[q >> 5]); q += 32; }
        else { sel += (bits[q >> 5] >> (q & 31)) & 1u; q++; }
      }
      out_base = wave_excl(sel);
    } else {
      out_base = lane_off;
    }
    // walk the segment, emitting members (skipping exclusions)
    uint32_t* pay = ob.pay + item.poff;
    uint32_t rank = lane_off, outp = out_base, e = e0;
    for (uint32_t j = lo; j < hi; j += 16) {
      uint4 v = *reinterpret_cast<const uint4*>(rw + j);
      uint32_t w4[4] = {v.x, v.y, v.z, v.w};
      for (int t = 0; t < 16; ++t) {
        const uint32_t id = j + t;
        if (id >= hi || !((w4[t >> 2] >> (8 * (t & 3))) & 0xFF)) continue;
        while (e < e1 && (pb.bjoin[e].sender < id || !newbit(nm, e))) ++e;
        if (e < e1 && pb.bjoin[e].sender == id) { ++e; continue; }
        if (!sample || ((bits[rank >> 5] >> (rank & 31)) & 1u)) { if (outp < cap) pay[outp] = id; outp++; }
        rank++;
      }
    }
    if (l == 0) {
      Msg m; m.dest = a; m.sender = i; m.seq = item.q; m.kind = K_KP; m.a = cap; m.fp = 0; m.n = 0; m.off = item.poff;
      ob.msgs[ob.off[i] + item.q] = m;
    }
    __syncthreads();
  }
}

// Join responses, LDS path (rows up to RESP_LDS_W ids): one workgroup per responding node builds the
// row's membership bitmap once, then for each of its responses (in list order) derives the member set
// at that moment (joiners inserted later removed), samples with Floyd when it does not fit 10240 B,
// and writes the sorted ids by rank/select on the bitmap.
constexpr uint32_t RESP_LDS_W = 131072;
__device__ inline uint32_t bm_rank(const uint32_t* S, const uint32_t* SP, uint32_t id) {   // members < id
  const uint32_t blk = id >> 8, w = id >> 5;
  uint32_t r = SP[blk];
  for (uint32_t k = blk * 8; k < w; ++k) r += __popc(S[k]);
  return r + __popc(S[w] & ((1u << (id & 31)) - 1u));
}
__device__ inline uint32_t bm_select(const uint32_t* S, const uint32_t* SP, uint32_t nblk, uint32_t b) {  // b-th member
  uint32_t lo = 0, hi = nblk;           // last block with SP[blk] <= b
  while (hi - lo > 1) { const uint32_t mid = (lo + hi) >> 1; if (SP[mid] <= b) lo = mid; else hi = mid; }
  uint32_t rem = b - SP[lo];
  uint32_t w = lo * 8;
  for (;; ++w) { const uint32_t c = __popc(S[w]); if (rem < c) break; rem -= c; }
  uint32_t x = S[w];
  for (uint32_t t = 0; t < rem; ++t) x &= x - 1;
  return w * 32 + (__ffs(x) - 1);
}
__global__ __launch_bounds__(256) void k_resp_node(Dev d, PhaseB pb, const uint32_t* nodes, const uint32_t* nnodes_p,
                                                   OutBuf ob, int32_t r) {
  extern __shared__ uint32_t lds[];
  const uint32_t NW = d.W / 32, NB = d.W / 256;
  uint32_t* B = lds;                 // row membership        [NW]
  uint32_t* S = B + NW;              // members at response   [NW]
  uint32_t* SP = S + NW;             // block prefix of S     [NB + 1]
  uint32_t* F = SP + NB + 1;         // Floyd rank bitmap     [NW]
  uint32_t* FP = F + NW;             // prefix of F per thread[256]
  uint32_t* dr = FP + 256;           // Floyd draws           [1024]
  __shared__ uint32_t s_red[16];
  const uint32_t t = threadIdx.x, T = blockDim.x;
  const uint32_t nnodes = *nnodes_p;
  for (uint32_t it = blockIdx.x; it < nnodes; it += gridDim.x) {
    const uint32_t i = nodes[it];
    const uint8_t* rw = row_of(d, i);
    // 1. membership bitmap of the row (two threads per 32-bit word)
    for (uint32_t k = t; k < d.W / 16; k += T) {
      const uint4 v = *reinterpret_cast<const uint4*>(rw + 16 * k);
      const uint32_t w4[4] = {v.x, v.y, v.z, v.w};
      const uint32_t m = nzmask16(w4);
      const uint32_t o = __shfl_xor(m, 1, 64);
      if ((k & 1) == 0) B[k >> 1] = m | (o << 16);
    }
    __syncthreads();
    const unsigned long long* nm = pb.newmask + (size_t)i * pb.JW;
    const unsigned long long* rm = pb.respmask + (size_t)i * pb.JW;
    uint32_t poff = ob.poff[i], q = 0, ins_before = 0;
    for (uint32_t wj = 0; wj < pb.JW; ++wj) {
      unsigned long long rmw = rm[wj];
      const unsigned long long nmw = nm[wj];
      while (rmw) {
        const uint32_t bit = (uint32_t)(__ffsll((long long)rmw) - 1);
        const uint32_t K = wj * 64 + bit;
        rmw &= rmw - 1;
        const uint32_t expect = pb.nbase[i] + ins_before + __popcll(nmw & ((2ull << bit) - 1ull));
        const uint32_t a = pb.bjoin[K].sender;
        // 2. S = B minus the joiners inserted after K
        for (uint32_t k = t; k < NW; k += T) S[k] = B[k];
        __syncthreads();
        for (uint32_t e = K + 1 + t; e < pb.nj; e += T)
          if (newbit(nm, e)) { const uint32_t x = pb.bjoin[e].sender; atomicAnd(&S[x >> 5], ~(1u << (x & 31))); }
        __syncthreads();
        // 3. block prefix of S
        uint32_t bc = 0;
        const uint32_t per = (NB + T - 1) / T;
        for (uint32_t k = t * per; k < (t + 1) * per && k < NB; ++k) {
          uint32_t c = 0;
          for (uint32_t w = 0; w < 8; ++w) c += __popc(S[k * 8 + w]);
          SP[k] = c; bc += c;
        }
        uint32_t ex = wave_excl(bc);
        const uint32_t wt = wave_sum(bc);
        if (lane() == 0) s_red[t >> 6] = wt;
        __syncthreads();
        for (uint32_t w = 0; w < (t >> 6); ++w) ex += s_red[w];
        uint32_t nk = 0;
        for (uint32_t w = 0; w < T / 64; ++w) nk += s_red[w];
        for (uint32_t k = t * per; k < (t + 1) * per && k < NB; ++k) { const uint32_t c = SP[k]; SP[k] = ex; ex += c; }
        if (t == 0) SP[NB] = nk;
        __syncthreads();
        const bool sample = d.uniform && nk > d.capj;
        const uint32_t cap = sample ? d.capj : nk;
        uint32_t* pay = ob.pay + poff;
        if (!sample) {
          // 4a. every member, in id order: position = rank
          for (uint32_t w = t; w < NW; w += T) {
            uint32_t x = S[w];
            if (!x) continue;
            uint32_t pos = bm_rank(S, SP, w * 32);
            while (x) { const uint32_t b = __ffs(x) - 1; x &= x - 1; pay[pos++] = w * 32 + b; }
          }
        } else {
          // 4b. Floyd: uniform cap-subset of ranks [0, nk)
          const uint32_t FW = (nk + 31) / 32;
          for (uint32_t w = t; w < FW; w += T) F[w] = 0;
          for (uint32_t t4 = t; t4 < (cap + 3) / 4; t4 += T) {
            const U4 u = philox(i, (uint32_t)r, ((uint32_t)P_TRUNC << 24) | t4, a, d.k0, d.k1);
            dr[4 * t4] = u.x; dr[4 * t4 + 1] = u.y; dr[4 * t4 + 2] = u.z; dr[4 * t4 + 3] = u.w;
          }
          __syncthreads();
          if (t == 0) {
            for (uint32_t k = 0; k < cap; ++k) {
              const uint32_t j = nk - cap + k;
              const uint32_t v = mulhi(dr[k], j + 1);
              const uint32_t x = (F[v >> 5] >> (v & 31)) & 1u ? j : v;
              F[x >> 5] |= 1u << (x & 31);
            }
          }
          __syncthreads();
          // selected ranks in increasing order -> output slots
          const uint32_t fper = (FW + T - 1) / T;
          uint32_t fc = 0;
          for (uint32_t w = t * fper; w < (t + 1) * fper && w < FW; ++w) fc += __popc(F[w]);
          uint32_t fex = wave_excl(fc);
          const uint32_t fwt = wave_sum(fc);
          __syncthreads();
          if (lane() == 0) s_red[t >> 6] = fwt;
          __syncthreads();
          for (uint32_t w = 0; w < (t >> 6); ++w) fex += s_red[w];
          uint32_t o = fex;
          for (uint32_t w = t * fper; w < (t + 1) * fper && w < FW; ++w) {
            uint32_t x = F[w];
            while (x) { const uint32_t b = __ffs(x) - 1; x &= x - 1; pay[o++] = bm_select(S, SP, NB, w * 32 + b); }
          }
        }
        if (t == 0) {
          Msg m; m.dest = a; m.sender = i; m.seq = q; m.kind = K_KP; m.a = cap; m.fp = 0; m.n = 0; m.off = poff;
          ob.msgs[ob.off[i] + q] = m;
          if (nk != expect) set_err(d, DERR_RESP);
        }
        poff += cap; q++;
        __syncthreads();
      }
      ins_before += __popcll(nmw);
    }
  }
}

// ================================================================================================
// Tick, part 1: maybe_broadcast_join (:228-251) and handle_suspected_peers (:558-653)
// ================================================================================================
struct BcastSlots { uint32_t* join; uint32_t* nfail; uint32_t* fail; };

// rank -> id selection over the candidates (Known && != self) of row i, lane-contiguous segments.
__device__ uint32_t select_known(const Dev& d, const uint8_t* rw, uint32_t i, uint32_t rank, uint32_t lane_off,
                                 uint32_t lane_cnt, uint32_t lo, uint32_t hi) {
  const uint32_t l = lane();
  uint32_t found = 0xFFFFFFFFu;
  if (rank >= lane_off && rank < lane_off + lane_cnt) {
    uint32_t c = lane_off;
    for (uint32_t j = lo; j < hi && found == 0xFFFFFFFFu; ++j) {
      if (rw[j] >= ST_ANCIENT && j != i) { if (c == rank) found = j; c++; }
    }
  }
  (void)l;
  return wave_min(found);
}

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

__global__ __launch_bounds__(256) void k_tick_pre(Dev d, OutBuf ob, BcastSlots bs, int32_t r) {
  __shared__ uint32_t s_pick_rank[4][SLOTS * 3], s_pick_peer[4][SLOTS * 3];
  const uint32_t wv = threadIdx.x >> 6;
  const uint32_t i = blockIdx.x * 4 + wv;
  const uint32_t l = lane();
  if (i >= d.C) return;
  if (!d.alive[i]) { if (l == 0) { bs.join[i] = 0; bs.nfail[i] = 0; } return; }
  uint32_t n = d.n[i];
  // A1
  if (l == 0) {
    const int32_t lb = d.last_bcast[i];
    uint32_t j = 0;
    if (lb == NONE_ROUND || (r - lb >= REBROADCAST && n <= 1)) { j = 1; d.last_bcast[i] = r; }
    bs.join[i] = j;
  }
  // A2
  Susp* sl = d.susp + (size_t)i * SLOTS;
  Susp me = l < SLOTS ? sl[l] : Susp{0, 0, 0, 0};
  const bool occ = l < SLOTS && me.kind != 0;
  const unsigned long long occm = __ballot(occ);
  const unsigned long long tim = __ballot(occ && r - me.since >= PING_TIMEOUT);
  if (!tim) { if (l == 0) bs.nfail[i] = 0; return; }
  const uint32_t nsusp = __popcll(occm);
  const uint32_t m = n - 1 - nsusp;
  // ascending-peer order of the occupied slots
  uint32_t myrank = 0;
  for (int k = 0; k < SLOTS; ++k) {
    const uint32_t pk = bcast(me.peer, k);
    if (((occm >> k) & 1ull) && pk < me.peer) myrank++;
  }
  uint32_t npick = 0, nind = 0, nrem = 0;
  uint32_t indirect[SLOTS], removed[SLOTS];
  uint32_t slot_pick_n[SLOTS];
  for (uint32_t t = 0; t < nsusp; ++t) {
    const unsigned long long who = __ballot(occ && myrank == t);
    const int k = __ffsll((long long)who) - 1;
    const uint32_t peer = bcast(me.peer, k);
    const int32_t kind = (int32_t)bcast((uint32_t)me.kind, k), since = (int32_t)bcast((uint32_t)me.since, k);
    slot_pick_n[t] = 0;
    if (r - since < PING_TIMEOUT) continue;
    if (kind == SK_WFP) {
      const uint32_t kk = m < (uint32_t)NUM_INDIRECT ? m : (uint32_t)NUM_INDIRECT;
      if (kk == 0) { removed[nrem++] = peer; continue; }
      const U4 w = philox(i, (uint32_t)r, (uint32_t)P_INDIRECT << 24, peer, d.k0, d.k1);
      uint32_t pk[3];
      pk[0] = mulhi(w.x, m);
      if (kk > 1) { uint32_t b = mulhi(w.y, m - 1); pk[1] = b + (b >= pk[0]); }
      if (kk > 2) {
        const uint32_t lo = pk[0] < pk[1] ? pk[0] : pk[1], hi = pk[0] < pk[1] ? pk[1] : pk[0];
        uint32_t c = mulhi(w.z, m - 2);
        if (c >= lo) c++;
        if (c >= hi) c++;
        pk[2] = c;
      }
      if (l == 0) for (uint32_t q = 0; q < kk; ++q) { s_pick_rank[wv][npick + q] = pk[q]; s_pick_peer[wv][npick + q] = peer; }
      npick += kk;
      slot_pick_n[t] = kk;
      indirect[nind++] = peer;
    } else {
      removed[nrem++] = peer;
    }
  }
  const uint8_t* rw = row_of(d, i);
  uint32_t oseq = ob.cnt[i];
  if (npick) {
    __builtin_amdgcn_s_waitcnt(0);
    __builtin_amdgcn_wave_barrier();
    uint32_t lo = l * d.SEG, hi = lo + d.SEG;
    if (hi > d.C) hi = d.C;
    if (lo > hi) lo = hi;
    uint32_t cnt = 0;
    for (uint32_t j = lo; j < hi; ++j) cnt += rw[j] >= ST_ANCIENT && j != i;
    const uint32_t off = wave_excl(cnt);
    for (uint32_t q = 0; q < npick; ++q) {
      const uint32_t rank = s_pick_rank[wv][q];
      const uint32_t id = select_known(d, rw, i, rank, off, cnt, lo, hi);
      emit_msg(ob, d, i, oseq, id, K_PINGREQ, s_pick_peer[wv][q], 0, 0, 0);
    }
  }
  // apply: WaitingForIndirectPing(now) (:631-639), removals + Failed broadcast (:641-652)
  if (l == 0) {
    for (uint32_t q = 0; q < nind; ++q)
      for (int k = 0; k < SLOTS; ++k) if (sl[k].kind && sl[k].peer == indirect[q]) { sl[k].kind = SK_WFIP; sl[k].since = r; }
    uint8_t* rww = row_of(d, i);
    Cur* cu = d.cur + (size_t)i * CSLOTS;
    for (uint32_t q = 0; q < nrem; ++q) {
      const uint32_t p = removed[q];
      susp_clear(d, i, p);
      rww[p] = ST_UNKNOWN;
      n--;
      for (int c = 0; c < CSLOTS; ++c) if (cu[c].used && cu[c].peer == p) cu[c].used = 0;
      bs.fail[(size_t)i * SLOTS + q] = p;
    }
    bs.nfail[i] = nrem;
    if (nrem) { d.n[i] = n; d.dirty[i] = 1; atomicAdd(&d.stats[S_RMTIMEOUT], nrem); }
    ob.cnt[i] = oseq;
  }
}

// ================================================================================================
// Tick, part 2 — THE ROW SWEEP (dominant kernel): ping_random_peer's oldest-5 selection over the
// node's whole stamp row (src/kaboodle.rs:662-675), fused with generate_fingerprint (:71-83) when the
// membership changed.  One wave per node; lane l owns the contiguous segment [l*SEG, (l+1)*SEG).
// A3 order is (stamp, address rotated to start after self): each lane scans its segment in rotated
// order so a later equal stamp never displaces an earlier one.
// ================================================================================================
struct SweepOut { uint32_t* cand; uint32_t* ncand; };

__device__ inline void top5_insert(uint32_t (&k)[5], uint32_t nk) {
#pragma unroll
  for (int s = 0; s < 5; ++s) { if (nk < k[s]) { uint32_t t = k[s]; k[s] = nk; nk = t; } }
}

template <bool FOLD>
__device__ inline void sweep_piece(const Dev& d, const uint8_t* rw, const uint32_t* ztab, uint32_t i, uint32_t x,
                                   uint32_t y, uint32_t rotbase, uint32_t (&k5)[5], uint32_t& raw, uint32_t& cnt) {
  if (x >= y) return;
  uint32_t T5 = k5[4] == 0xFFFFFFFFu ? 256u : (k5[4] >> 24);
  const uint32_t b0 = x & ~15u;
  for (uint32_t blk = b0; blk < y; blk += 16) {
    const uint4 v = *reinterpret_cast<const uint4*>(rw + blk);
    const uint32_t w4[4] = {v.x, v.y, v.z, v.w};
    uint32_t valid = 0xFFFFu;
    if (blk < x) valid &= 0xFFFFu << (x - blk);
    if (blk + 16 > y) valid &= 0xFFFFu >> (blk + 16 - y);
    if (FOLD) fold16(d, ztab, blk, nzmask16(w4) & valid, raw, cnt);
    if (T5 > ST_ANCIENT) {
#pragma unroll
      for (int t = 0; t < 16; ++t) {
        const uint32_t b = (w4[t >> 2] >> (8 * (t & 3))) & 0xFFu;
        const uint32_t j = blk + t;
        if (((valid >> t) & 1u) && b >= ST_ANCIENT && b < T5 && j != i) {
          top5_insert(k5, (b << 24) | (j - blk + rotbase + (blk - x)));
          T5 = k5[4] == 0xFFFFFFFFu ? 256u : (k5[4] >> 24);
        }
      }
    }
  }
}

__global__ __launch_bounds__(256) void k_sweep(Dev d, SweepOut so) {
  __shared__ uint32_t ztab[ZT * 128];
  load_ztab(d, ztab);
  const uint32_t i = blockIdx.x * 4 + (threadIdx.x >> 6);
  const uint32_t l = lane();
  if (i >= d.C || !d.alive[i]) return;
  const uint8_t* rw = row_of(d, i);
  const uint32_t C = d.C;
  const uint32_t p = (i + 1 == C) ? 0 : i + 1;   // rotated order starts right after self
  const bool fold = d.dirty[i] != 0;
  uint32_t lo = l * d.SEG, hi = lo + d.SEG;
  if (hi > C) hi = C;
  if (lo > hi) lo = hi;
  uint32_t k5[5] = {0xFFFFFFFFu, 0xFFFFFFFFu, 0xFFFFFFFFu, 0xFFFFFFFFu, 0xFFFFFFFFu};
  uint32_t raw1 = 0, cnt1 = 0, raw2 = 0, cnt2 = 0;
  // piece 1: [max(lo,p), hi) has rot = j - p; piece 2: [lo, min(hi,p)) has rot = j - p + C
  const uint32_t x1 = lo > p ? lo : p, y2 = hi < p ? hi : p;
  if (d.uniform && fold) {
    sweep_piece<true>(d, rw, ztab, i, x1, hi, x1 - p, k5, raw1, cnt1);
    sweep_piece<true>(d, rw, ztab, i, lo, y2, lo + C - p, k5, raw2, cnt2);
  } else {
    sweep_piece<false>(d, rw, ztab, i, x1, hi, x1 - p, k5, raw1, cnt1);
    sweep_piece<false>(d, rw, ztab, i, lo, y2, lo + C - p, k5, raw2, cnt2);
  }
  // merge lane top-5 lists
  uint32_t ncand = 0, cid[5] = {0, 0, 0, 0, 0};
#pragma unroll
  for (int t = 0; t < 5; ++t) {
    const uint32_t mn = wave_min(k5[0]);
    if (mn != 0xFFFFFFFFu) {
      const uint32_t rot = mn & 0xFFFFFFu;
      cid[t] = rot + p >= C ? rot + p - C : rot + p;
      ncand++;
      if (k5[0] == mn) { k5[0] = k5[1]; k5[1] = k5[2]; k5[2] = k5[3]; k5[3] = k5[4]; k5[4] = 0xFFFFFFFFu; }
    }
  }
  if (l == 0) {
    so.ncand[i] = ncand;
    for (int t = 0; t < 5; ++t) so.cand[(size_t)i * 5 + t] = cid[t];
  }
  if (fold) {
    uint32_t fp;
    if (d.uniform) {
      // lane partial = piece2 (lower ids) then piece1
      uint32_t raw = multmodp(d.zpow[cnt1], raw2) ^ raw1, cnt = cnt1 + cnt2;
#pragma unroll
      for (int s = 1; s < 64; s <<= 1) {
        const uint32_t oraw = __shfl_down(raw, s, 64), ocnt = __shfl_down(cnt, s, 64);
        if ((l & (2 * s - 1)) == 0 && l + s < 64) { raw = multmodp(d.zpow[ocnt], raw) ^ oraw; cnt += ocnt; }
      }
      fp = raw ^ multmodp(d.zpow[cnt], 0xFFFFFFFFu) ^ 0xFFFFFFFFu;
    } else {
      uint32_t raw = 0; uint64_t len = 0;
      if (l == 0) {
        for (uint32_t j = 0; j < C; ++j)
          if (rw[j]) { raw = multmodp(d.segmul[j], raw) ^ d.cseg[j]; len += d.seglen[j]; }
      }
      fp = raw ^ multmodp(xpow8_dev(len), 0xFFFFFFFFu) ^ 0xFFFFFFFFu;
    }
    if (l == 0) { d.fp[i] = fp; d.dirty[i] = 0; }
  }
}

// ================================================================================================
// Tick, part 3: pick the ping target (one of the oldest 5), WaitingForPing(now), Ping; ping_addrs;
// agreement with the true running set (thread per node).
// ================================================================================================
__global__ void k_tick_post(Dev d, SweepOut so, OutBuf ob, int32_t r) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  unsigned long long agree = 0;
  if (i < d.C && d.alive[i]) {
    uint32_t oseq = ob.cnt[i];
    const uint32_t nc = so.ncand[i];
    if (nc) {
      const uint32_t u = philox(i, (uint32_t)r, (uint32_t)P_PING << 24, 0, d.k0, d.k1).x;
      const uint32_t t = so.cand[(size_t)i * 5 + mulhi(u, nc)];
      Susp* sl = d.susp + (size_t)i * SLOTS;
      int k = 0;
      while (k < SLOTS && sl[k].kind) ++k;
      if (k == SLOTS) set_err(d, DERR_SLOTS);
      else { sl[k].peer = t; sl[k].kind = SK_WFP; sl[k].since = r; }
      row_of(d, i)[t] = ST_SUSPECT;
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
    agree = d.fp[i] == d.truefp[0];
  }
  unsigned long long t = block_sum(agree);
  if (threadIdx.x == 0 && t) atomicAdd(&d.ctr[C_AGREE], (uint32_t)t);
}

__global__ void k_bcast_write(Dev d, BcastSlots bs, const uint32_t* join_off, const uint32_t* fail_off, BCast* bjoin,
                              BCast* bfail) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= d.C) return;
  uint32_t bseq = 0;
  if (bs.join[i]) { bjoin[join_off[i]] = BCast{i, i, bseq++, 0}; }
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
  d.ctr[C_AGREE] = 0; d.ctr[C_ALIVE] = 0;
}

// ================================================================================================
// Unicast waves (src/kaboodle.rs:394-548)
// ================================================================================================
struct WaveCtl {
  uint8_t* status;        // per outbox slot: 0 dropped, 1 class-1 delivered, 2 KnownPeers delivered
  uint32_t* cnt1; uint32_t* bnd; uint32_t* bpay; uint32_t* cursor;   // per dest
  uint32_t* in_off; uint32_t* inbox; uint32_t* active;
  uint32_t* kp_list; uint32_t* touched; uint32_t* touched_list;
  uint32_t msg_cap; uint32_t pay_cap;
};

__device__ inline uint32_t out_bound(uint32_t kind) {
  return kind == K_ACK ? NOBS + 1 : (kind == K_KPR ? 2u : (kind == K_KP ? 0u : 1u));
}

__global__ __launch_bounds__(256) void k_route(Dev d, OutBuf ob, WaveCtl wc, int32_t r, uint32_t w, int last) {
  __shared__ uint32_t s_kp[256];
  __shared__ uint32_t s_base;
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  unsigned long long ks[5] = {0, 0, 0, 0, 0}, dead = 0, part = 0, loss = 0, win = 0;
  uint32_t nkp = 0;
  const uint32_t cnt = i < d.C ? ob.cnt[i] : 0;
  const uint32_t base = i < d.C ? ob.off[i] : 0;
  for (uint32_t q = 0; q < cnt; ++q) {
    const uint32_t g = base + q;
    const Msg m = ob.msgs[g];
    ks[m.kind]++;
    uint8_t st = 0;
    if (last) { win++; }
    else if (!d.alive[m.dest]) dead++;
    else if (part_blocks(d, r, m.sender, m.dest)) part++;
    else if (faults(d, r) && d.loss_thr &&
             philox(m.sender, (uint32_t)r, ((uint32_t)P_LOSS << 24) | w, m.seq, d.k0, d.k1).x < d.loss_thr) loss++;
    else if (m.kind == K_KP) { st = 2; nkp++; }
    else {
      st = 1;
      atomicAdd(&wc.cnt1[m.dest], 1u);
      atomicAdd(&wc.bnd[m.dest], out_bound(m.kind));
      if (m.kind == K_KPR) atomicAdd(&wc.bpay[m.dest], d.paybound);
    }
    if (!last) wc.status[g] = st;
  }
  for (int k = 0; k < 5; ++k) stat_add(d, S_PING + k, ks[k]);
  stat_add(d, S_DEAD, dead); stat_add(d, S_PART, part); stat_add(d, S_LOSS, loss); stat_add(d, S_WINDOW, win);
  if (last) return;
  // reserve kp_list space for this block
  s_kp[threadIdx.x] = nkp;
  __syncthreads();
  if (threadIdx.x == 0) {
    uint32_t run = 0;
    for (uint32_t t = 0; t < blockDim.x; ++t) { uint32_t v = s_kp[t]; s_kp[t] = run; run += v; }
    s_base = run ? atomicAdd(&d.ctr[C_KP], run) : 0;
  }
  __syncthreads();
  uint32_t pos = s_base + s_kp[threadIdx.x];
  if (nkp) for (uint32_t q = 0; q < cnt; ++q) if (wc.status[base + q] == 2) wc.kp_list[pos++] = base + q;
}

__global__ void k_scatter(Dev d, OutBuf ob, WaveCtl wc) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= d.C) return;
  const uint32_t cnt = ob.cnt[i], base = ob.off[i];
  for (uint32_t q = 0; q < cnt; ++q) {
    const uint32_t g = base + q;
    if (wc.status[g] != 1) continue;
    const uint32_t dst = ob.msgs[g].dest;
    wc.inbox[wc.in_off[dst] + atomicAdd(&wc.cursor[dst], 1u)] = g;
  }
}

__device__ inline void mark_touched(const Dev& d, const WaveCtl& wc, uint32_t node) {
  if (atomicExch(&wc.touched[node], 1u) == 0u) wc.touched_list[atomicAdd(&d.ctr[C_TOUCH], 1u)] = node;
}

// KnownPeers arm (:448-472): insert every listed unknown peer as Known(now - 10s); message-parallel.
__global__ __launch_bounds__(256) void k_kp_insert(Dev d, OutBuf ob, WaveCtl wc, int32_t r) {
  const uint32_t nkp = d.ctr[C_KP];
  const uint8_t old = enc(r - SHARE_AGE, r);
  for (uint32_t it = blockIdx.x * 4 + (threadIdx.x >> 6); it < nkp; it += gridDim.x * 4) {
    const Msg m = ob.msgs[wc.kp_list[it]];
    uint8_t* rw = row_of(d, m.dest);
    bool ins = false;
    for (uint32_t e = lane(); e < m.a; e += 64) {
      const uint32_t p = ob.pay[m.off + e];
      if (rw[p] == ST_UNKNOWN) { rw[p] = old; ins = true; }
    }
    if (__ballot(ins) && lane() == 0) mark_touched(d, wc, m.dest);
  }
}
// prologue of every KnownPeers envelope (:406-415): sender becomes Known(now)
__global__ void k_kp_prologue(Dev d, OutBuf ob, WaveCtl wc, int32_t r) {
  const uint32_t nkp = d.ctr[C_KP];
  const uint8_t now = enc(r, r);
  for (uint32_t it = blockIdx.x * blockDim.x + threadIdx.x; it < nkp; it += gridDim.x * blockDim.x) {
    const Msg m = ob.msgs[wc.kp_list[it]];
    uint8_t* rw = row_of(d, m.dest);
    const uint8_t b = rw[m.sender];
    rw[m.sender] = now;
    if (b <= ST_SUSPECT) mark_touched(d, wc, m.dest);
  }
}
// recount membership of touched rows, drop suspect slots whose entry was overwritten
__global__ __launch_bounds__(256) void k_touch_fix(Dev d, WaveCtl wc) {
  const uint32_t nt = d.ctr[C_TOUCH];
  const uint32_t l = lane();
  for (uint32_t it = blockIdx.x * 4 + (threadIdx.x >> 6); it < nt; it += gridDim.x * 4) {
    const uint32_t i = wc.touched_list[it];
    const uint8_t* rw = row_of(d, i);
    uint32_t c = 0;
    for (uint32_t j = l * 16; j < d.W; j += 64 * 16) {
      const uint4 v = *reinterpret_cast<const uint4*>(rw + j);
      const uint32_t w4[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
      for (int t = 0; t < 16; ++t) c += ((w4[t >> 2] >> (8 * (t & 3))) & 0xFF) != 0;
    }
    c = wave_sum(c);
    if (l < SLOTS) {
      Susp* s = d.susp + (size_t)i * SLOTS + l;
      if (s->kind && rw[s->peer] != ST_SUSPECT) s->kind = 0;
    }
    if (l == 0) {
      if (c != d.n[i]) { d.n[i] = c; d.dirty[i] = 1; }
      wc.touched[i] = 0;
    }
  }
}

// ---- the per-node sequential program for non-KnownPeers messages --------------------------------
// fingerprint of row i by one wave (lane-contiguous segments, template fast path)
__device__ uint32_t wave_fold(const Dev& d, const uint8_t* rw, const uint32_t* ztab) {
  const uint32_t l = lane();
  if (!d.uniform) {
    uint32_t raw = 0; uint64_t len = 0;
    if (l == 0)
      for (uint32_t j = 0; j < d.C; ++j) if (rw[j]) { raw = multmodp(d.segmul[j], raw) ^ d.cseg[j]; len += d.seglen[j]; }
    raw = bcast(raw, 0);
    len = ((uint64_t)bcast((uint32_t)(len >> 32), 0) << 32) | bcast((uint32_t)len, 0);
    return raw ^ multmodp(xpow8_dev(len), 0xFFFFFFFFu) ^ 0xFFFFFFFFu;
  }
  uint32_t lo = l * d.SEG, hi = lo + d.SEG;
  if (hi > d.C) hi = d.C;
  if (lo > hi) lo = hi;
  uint32_t raw = 0, cnt = 0;
  for (uint32_t blk = lo; blk < hi; blk += 16) {
    const uint4 v = *reinterpret_cast<const uint4*>(rw + blk);
    const uint32_t w4[4] = {v.x, v.y, v.z, v.w};
    const uint32_t valid = blk + 16 > hi ? (0xFFFFu >> (blk + 16 - hi)) : 0xFFFFu;
    fold16(d, ztab, blk, nzmask16(w4) & valid, raw, cnt);
  }
#pragma unroll
  for (int s = 1; s < 64; s <<= 1) {
    const uint32_t oraw = __shfl_down(raw, s, 64), ocnt = __shfl_down(cnt, s, 64);
    if ((l & (2 * s - 1)) == 0 && l + s < 64) { raw = multmodp(d.zpow[ocnt], raw) ^ oraw; cnt += ocnt; }
  }
  raw = bcast(raw, 0); cnt = bcast(cnt, 0);
  return raw ^ multmodp(d.zpow[cnt], 0xFFFFFFFFu) ^ 0xFFFFFFFFu;
}

struct NodeCtx {
  uint32_t i, n, fp, oseq, pay_used;
  bool dirty, need_sync;
};

__global__ __launch_bounds__(256) void k_proc(Dev d, OutBuf ib, OutBuf ob, WaveCtl wc, int32_t r) {
  __shared__ uint32_t ztab[ZT * 128];
  __shared__ Susp s_susp[4][SLOTS];
  __shared__ Cur s_cur[4][CSLOTS];
  load_ztab(d, ztab);
  const uint32_t wv = threadIdx.x >> 6;
  const uint32_t l = lane();
  const uint32_t nact = d.ctr[C_ACTIVE];
  const uint8_t now = enc(r, r);
  const uint8_t fresh_thr = enc(r - (SHARE_AGE - 1), r);
  for (uint32_t it = blockIdx.x * 4 + wv; it < nact; it += gridDim.x * 4) {
    NodeCtx x;
    x.i = wc.active[it];
    const uint32_t i = x.i;
    uint8_t* rw = row_of(d, i);
    x.n = d.n[i]; x.fp = d.fp[i]; x.dirty = d.dirty[i] != 0; x.oseq = 0; x.pay_used = 0; x.need_sync = false;
    if (l < SLOTS) s_susp[wv][l] = d.susp[(size_t)i * SLOTS + l];
    if (l < CSLOTS) s_cur[wv][l] = d.cur[(size_t)i * CSLOTS + l];
    __builtin_amdgcn_wave_barrier();
    const uint32_t ibase = wc.in_off[i], icnt = wc.cnt1[i];
    // inbox order = ascending outbox index = (sender, seq)
    uint32_t mine = l < icnt ? wc.inbox[ibase + l] : 0xFFFFFFFFu;
    const bool small = icnt <= 64;
    if (small) {
#pragma unroll
      for (int k = 2; k <= 64; k <<= 1) {
#pragma unroll
        for (int j = k >> 1; j > 0; j >>= 1) {
          const uint32_t o = __shfl_xor(mine, j, 64);
          const bool up = ((l & k) == 0);
          const bool lower = (l & j) == 0;
          const uint32_t mn = o < mine ? o : mine, mx = o < mine ? mine : o;
          mine = (lower == up) ? mn : mx;
        }
      }
    }
    uint32_t last_g = 0xFFFFFFFFu, last_sender = 0xFFFFFFFFu;
    for (uint32_t t = 0; t < icnt; ++t) {
      uint32_t g;
      if (small) g = bcast(mine, (int)t);
      else {        // selection fallback for large inboxes: next smallest index above the previous one
        uint32_t best = 0xFFFFFFFFu;
        for (uint32_t q = l; q < icnt; q += 64) {
          const uint32_t v = wc.inbox[ibase + q];
          if ((last_g == 0xFFFFFFFFu || v > last_g) && v < best) best = v;
        }
        g = wave_min(best);
      }
      last_g = g;
      const Msg m = ib.msgs[g];
      const uint32_t s = m.sender;
      // ---- prologue: insert(sender, Known(now)) (:406-415) ----
      if (s != last_sender) {
        const uint8_t b = rw[s];
        if (b == ST_SUSPECT && l < SLOTS && s_susp[wv][l].kind && s_susp[wv][l].peer == s) s_susp[wv][l].kind = 0;
        if (b == ST_UNKNOWN) { x.n++; x.dirty = true; }
        if (b != now) { if (l == 0) rw[s] = now; x.need_sync = true; }
        last_sender = s;
        __builtin_amdgcn_wave_barrier();
      }
      auto fp_now = [&]() -> uint32_t {
        if (x.dirty) {
          if (x.need_sync) { wave_mem_sync(); x.need_sync = false; }
          x.fp = wave_fold(d, rw, ztab);
          x.dirty = false;
        }
        return x.fp;
      };
      auto maybe_sync = [&](uint32_t peer, uint32_t their_fp, uint32_t their_n) {   // :707-740
        const uint32_t f = fp_now();
        if (f == their_fp) return;
        if (x.n > their_n) return;
        emit_msg(ob, d, i, x.oseq, peer, K_KPR, 0, f, x.n, 0);
      };
      switch (m.kind) {
        case K_PING: {                                               // :513-532
          const uint32_t f = fp_now();
          emit_msg(ob, d, i, x.oseq, s, K_ACK, i, f, x.n, 0);
          break;
        }
        case K_PINGREQ: {                                            // :533-545
          // curious_peers[peer] += sender (dedup), then Ping(peer)
          const unsigned long long hit = __ballot(l < CSLOTS && s_cur[wv][l].used && s_cur[wv][l].peer == m.a);
          int e = hit ? __ffsll((long long)hit) - 1 : -1;
          if (e < 0) {
            const unsigned long long fr = __ballot(l < CSLOTS && !s_cur[wv][l].used);
            e = fr ? __ffsll((long long)fr) - 1 : -1;
            if (e >= 0 && l == 0) { s_cur[wv][e].used = 1; s_cur[wv][e].peer = m.a; s_cur[wv][e].nobs = 0; }
          }
          __builtin_amdgcn_wave_barrier();
          if (e < 0) { if (l == 0) atomicAdd(&d.stats[S_CUROVF], 1ull); }
          else if (l == 0) {
            Cur& c = s_cur[wv][e];
            bool dup = false;
            for (uint32_t q = 0; q < c.nobs; ++q) dup |= c.obs[q] == s;
            if (!dup) { if (c.nobs == NOBS) atomicAdd(&d.stats[S_CUROVF], 1ull); else c.obs[c.nobs++] = s; }
          }
          __builtin_amdgcn_wave_barrier();
          emit_msg(ob, d, i, x.oseq, m.a, K_PING, 0, 0, 0, 0);
          break;
        }
        case K_ACK: {                                                // :418-447
          const unsigned long long hit = __ballot(l < CSLOTS && s_cur[wv][l].used && s_cur[wv][l].peer == m.a);
          if (hit) {
            const int e = __ffsll((long long)hit) - 1;
            const uint32_t nobs = s_cur[wv][e].nobs;
            uint32_t obs[NOBS];
            for (int q = 0; q < NOBS; ++q) obs[q] = s_cur[wv][e].obs[q];
            __builtin_amdgcn_wave_barrier();
            if (l == 0) s_cur[wv][e].used = 0;
            for (uint32_t q = 0; q < nobs; ++q) emit_msg(ob, d, i, x.oseq, obs[q], K_ACK, m.a, m.fp, m.n, 0);
            __builtin_amdgcn_wave_barrier();
          }
          maybe_sync(m.a, m.fp, m.n);
          break;
        }
        case K_KPR: {                                                // :473-512
          if (x.need_sync) { wave_mem_sync(); x.need_sync = false; }
          const uint32_t poff = ob.poff[i] + x.pay_used;
          uint32_t total = 0;
          uint64_t size = 8 + d.seglen[i] - ADDR_LEN + 4 + 8;
          bool over = false;
          for (uint32_t c = 0; c < d.W && !over; c += 1024) {
            const uint32_t j0 = c + l * 16;
            const uint4 v = *reinterpret_cast<const uint4*>(rw + j0);
            const uint32_t w4[4] = {v.x, v.y, v.z, v.w};
            uint32_t mask = 0;
#pragma unroll
            for (int t = 0; t < 16; ++t) {
              const uint32_t b = (w4[t >> 2] >> (8 * (t & 3))) & 0xFFu, j = j0 + t;
              mask |= (uint32_t)(b >= fresh_thr && j != i && j != s && j < d.C) << t;
            }
            const uint32_t mc = __popc(mask);
            uint32_t pos = total + wave_excl(mc);
            if (!d.uniform) {
              uint32_t sz = 0, mm = mask;
              while (mm) { const int t = __ffs(mm) - 1; mm &= mm - 1; sz += 18 + d.seglen[j0 + t] - ADDR_LEN; }
              size += wave_sum(sz);
            }
            while (mask) {
              const int t = __ffs(mask) - 1;
              mask &= mask - 1;
              if (pos < d.paybound) {
                if (poff + pos < ob.pay_cap) ob.pay[poff + pos] = j0 + t;
                else set_err(d, DERR_PAYLOAD);
              }
              pos++;
            }
            total += wave_sum(mc);
            if (d.uniform && total > d.capk) over = true;
          }
          if (d.uniform) over = total > d.capk; else over = size > (uint64_t)BUFSZ;
          if (over) { if (l == 0) atomicAdd(&d.stats[S_OVERSIZE], 1ull); }
          else { emit_msg(ob, d, i, x.oseq, s, K_KP, total, 0, 0, poff); x.pay_used += total; }
          maybe_sync(s, m.fp, m.n);
          break;
        }
        default: break;
      }
    }
    if (l < SLOTS) d.susp[(size_t)i * SLOTS + l] = s_susp[wv][l];
    if (l < CSLOTS) d.cur[(size_t)i * CSLOTS + l] = s_cur[wv][l];
    if (l == 0) {
      d.n[i] = x.n; d.fp[i] = x.fp; d.dirty[i] = x.dirty ? 1 : 0;
      ob.cnt[i] = x.oseq;
    }
    __builtin_amdgcn_wave_barrier();
  }
}

// ================================================================================================
// Host side
// ================================================================================================
// crc0 fold of every member pattern of every 8-id half block (uniform identity length)
__global__ void k_build_htab(Dev d) {
  const size_t k = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  const size_t total = (size_t)(d.W / 8) * 256;
  if (k >= total) return;
  const uint32_t h = (uint32_t)(k >> 8), m = (uint32_t)(k & 255);
  uint32_t raw = 0;
  for (uint32_t t = 0; t < 8; ++t) {
    const uint32_t j = h * 8 + t;
    if (((m >> t) & 1u) && j < d.C) raw = multmodp(d.zpow[1], raw) ^ d.cseg[j];
  }
  d.htab[k] = raw;
}

__global__ void k_set_cap(uint32_t C, const uint32_t* nresp, uint32_t* cap, uint32_t* cnt) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < C) { cap[i] = nresp[i] + TICK_MAX; cnt[i] = nresp[i]; }
}

static thread_local std::string g_err;
static void seterr(const std::string& s) { g_err = s; }

#define HIPCHK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { seterr(std::string(#x) + ": " + hipGetErrorString(e_)); return KB_IO_ERROR; } } while (0)

template <class T> static hipError_t dalloc(T** p, size_t n) {
  hipError_t e = hipMalloc((void**)p, sizeof(T) * (n ? n : 1));
  if (e == hipSuccess) e = hipMemset(*p, 0, sizeof(T) * (n ? n : 1));
  return e;
}

static uint32_t h_crc_table[256];
static void h_crc_init() {
  for (uint32_t i = 0; i < 256; ++i) { uint32_t c = i; for (int k = 0; k < 8; ++k) c = (c & 1) ? (c >> 1) ^ CRC_POLY : c >> 1; h_crc_table[i] = c; }
}
static uint32_t h_crc_update(uint32_t reg, const uint8_t* p, size_t n) {
  for (size_t k = 0; k < n; ++k) reg = h_crc_table[(reg ^ p[k]) & 0xFF] ^ (reg >> 8);
  return reg;
}
static uint32_t h_xpow8(uint64_t n) {
  uint32_t res = 0x80000000u, sq = 0x00800000u;
  while (n) { if (n & 1) res = multmodp(sq, res); sq = multmodp(sq, sq); n >>= 1; }
  return res;
}

struct kb_sim {
  kb_config cfg;
  Dev d;
  int device;
  hipStream_t st;
  uint32_t C, W;
  int32_t round;
  // host mirrors
  std::vector<uint8_t> h_ident;   // C * MAXID
  std::vector<uint8_t> h_idlen;
  std::vector<uint8_t> h_ever;    // host-known "has run" (initial + API starts); churn joins tracked on device
  std::vector<Event> events;
  // buffers
  OutBuf ob[2];
  WaveCtl wc;
  uint32_t msg_cap, pay_cap;
  BCast* bfail; BCast* bjoin;
  uint32_t nf, nj;
  BcastSlots bs;
  uint32_t* join_off; uint32_t* fail_off;
  uint32_t* scan_tot;
  uint32_t* scan_tiles;
  // phase B
  unsigned long long* newmask; unsigned long long* respmask; size_t mask_words;
  uint32_t* nresp; uint32_t* paysum; uint32_t* nbase; uint32_t* resp_off;
  RespItem* items; uint32_t items_cap;
  uint32_t* resp_nodes; uint32_t* bf_gid; uint8_t* bf_dep;
  // sweep
  SweepOut so;
  Event* d_events; uint32_t events_cap;
  // timing
  hipEvent_t ev0, ev1, er0, er1;
  double sweep_ms, round_ms;
  uint64_t sweep_launches, round_launches, sweep_bytes;
  uint64_t bj_total, bf_total;
};

extern "C" void kb_config_default(kb_config* c) {
  memset(c, 0, sizeof *c);
  c->abi_version = KB_ABI_VERSION; c->capacity = 1024; c->initial_nodes = 1024; c->init_mode = KB_INIT_JOIN;
  c->seed = 1; c->fault_end_round = -1; c->max_waves = 8; c->failed_mode = KB_FAILED_SIM_SENDER; c->device = -1;
}

extern "C" const char* kb_last_error(void) { return g_err.c_str(); }

extern "C" int kb_format_addr(uint32_t id, char* buf, size_t cap) {
  char tmp[32];
  int len = snprintf(tmp, sizeof tmp, "10.100.100.%u:%u", 100u + id / 50000u, 10000u + id % 50000u);
  if (!buf || cap < (size_t)len + 1) return KB_INVALID_ARGUMENT;
  memcpy(buf, tmp, (size_t)len + 1);
  return KB_OK;
}

static void default_identity(uint32_t id, uint32_t len, uint8_t* out) {
  for (uint32_t k = 0; k < len; ++k) out[k] = (uint8_t)('a' + ((id * 31u + k * 7u) % 26u));
}

// (re)upload per-id segment tables and the Z tables
static int upload_segments(kb_sim* s) {
  const uint32_t C = s->C;
  std::vector<uint32_t> cseg(C), segmul(C), seglen(C);
  bool uniform = true;
  for (uint32_t j = 0; j < C; ++j) {
    char a[32]; kb_format_addr(j, a, sizeof a);
    uint32_t reg = h_crc_update(0, (const uint8_t*)a, ADDR_LEN);
    reg = h_crc_update(reg, &s->h_ident[(size_t)j * MAXID], s->h_idlen[j]);
    cseg[j] = reg; seglen[j] = ADDR_LEN + s->h_idlen[j]; segmul[j] = h_xpow8(seglen[j]);
    if (s->h_idlen[j] != s->cfg.id_len) uniform = false;
  }
  s->d.uniform = uniform ? 1 : 0;
  s->d.L = ADDR_LEN + s->cfg.id_len;
  const uint32_t Z = h_xpow8(s->d.L);
  std::vector<uint32_t> zpow(C + 2);
  zpow[0] = 0x80000000u;
  for (uint32_t k = 1; k < C + 2; ++k) zpow[k] = multmodp(Z, zpow[k - 1]);
  std::vector<uint32_t> ztab(17 * 128);
  for (uint32_t c = 0; c <= 16; ++c)
    for (uint32_t k = 0; k < 8; ++k)
      for (uint32_t v = 0; v < 16; ++v) ztab[c * 128 + k * 16 + v] = multmodp(zpow[c], v << (4 * k));
  HIPCHK(hipMemcpy(s->d.cseg, cseg.data(), 4ull * C, hipMemcpyHostToDevice));
  HIPCHK(hipMemcpy(s->d.segmul, segmul.data(), 4ull * C, hipMemcpyHostToDevice));
  HIPCHK(hipMemcpy(s->d.seglen, seglen.data(), 4ull * C, hipMemcpyHostToDevice));
  HIPCHK(hipMemcpy(s->d.zpow, zpow.data(), 4ull * (C + 2), hipMemcpyHostToDevice));
  HIPCHK(hipMemcpy(s->d.ztab, ztab.data(), 4ull * ztab.size(), hipMemcpyHostToDevice));
  const size_t hn = (size_t)(s->W / 8) * 256;
  k_build_htab<<<(unsigned)((hn + 255) / 256), 256>>>(s->d);
  HIPCHK(hipDeviceSynchronize());
  return KB_OK;
}

static void free_all(kb_sim* s);

__global__ void k_init_nodes(Dev d, uint32_t n0, uint32_t mode) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= d.C) return;
  d.last_bcast[i] = NONE_ROUND;
  d.start_round[i] = NONE_ROUND;
  if (i >= n0) return;
  node_start(d, i, 0);
  if (mode == KB_INIT_CONVERGED) {
    uint8_t* rw = row_of(d, i);
    for (uint32_t j = 0; j < n0; ++j) if (j != i) rw[j] = ST_ANCIENT;
    d.n[i] = n0;
    d.last_bcast[i] = -1000;
  }
}
__global__ void k_init_converged_rows(Dev d, uint32_t n0) {
  // vectorized fill of the converged rows (faster than per-thread loops for large n0)
  const size_t words = (size_t)n0 * (d.W / 16);
  uint4* p = reinterpret_cast<uint4*>(d.stamp);
  const uint32_t wpr = d.W / 16;
  for (size_t k = (size_t)blockIdx.x * blockDim.x + threadIdx.x; k < words; k += (size_t)gridDim.x * blockDim.x) {
    const uint32_t i = (uint32_t)(k / wpr), c = (uint32_t)(k % wpr);
    uint32_t w4[4];
    for (int q = 0; q < 4; ++q) {
      uint32_t y = 0;
      for (int t = 0; t < 4; ++t) {
        const uint32_t j = c * 16 + q * 4 + t;
        uint32_t b = j < n0 ? ST_ANCIENT : 0;
        if (j == i) b = enc(0, 0);
        y |= b << (8 * t);
      }
      w4[q] = y;
    }
    p[(size_t)i * wpr + c] = make_uint4(w4[0], w4[1], w4[2], w4[3]);
  }
}
__global__ void k_init_converged_nodes(Dev d, uint32_t n0) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= d.C) return;
  d.last_bcast[i] = NONE_ROUND;
  d.start_round[i] = NONE_ROUND;
  if (i >= n0) return;
  d.alive[i] = 1; d.start_round[i] = 0; d.dirty[i] = 1; d.n[i] = n0; d.last_bcast[i] = -1000; d.paq_n[i] = 0;
}

extern "C" int kb_sim_create(const kb_config* cfg, kb_sim** out) {
  h_crc_init();
  if (!cfg || !out || cfg->abi_version != KB_ABI_VERSION) { seterr("bad config"); return KB_INVALID_ARGUMENT; }
  if (cfg->capacity == 0 || cfg->capacity > 7800000u || cfg->initial_nodes > cfg->capacity || cfg->id_len > MAXID ||
      cfg->max_waves == 0 || cfg->max_waves > 64) { seterr("config out of range"); return KB_INVALID_ARGUMENT; }
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0) { seterr("no HIP device"); return KB_NO_DEVICE; }
  kb_sim* s = new kb_sim();
  memset((void*)&s->d, 0, sizeof s->d);
  s->cfg = *cfg;
  s->device = cfg->device >= 0 ? cfg->device : 0;
  if (cfg->device < 0) hipGetDevice(&s->device);
  if (hipSetDevice(s->device) != hipSuccess) { delete s; seterr("hipSetDevice failed"); return KB_NO_DEVICE; }
  const uint32_t C = cfg->capacity;
  const uint32_t W = (C + 1023) / 1024 * 1024;
  s->C = C; s->W = W; s->round = 0;
  Dev& d = s->d;
  d.C = C; d.W = W; d.SEG = W / 64;
  d.k0 = (uint32_t)cfg->seed; d.k1 = (uint32_t)(cfg->seed >> 32);
  d.loss_thr = cfg->loss_threshold; d.churn_thr = cfg->churn_threshold; d.fault_end = cfg->fault_end_round;
  d.failed_mode = cfg->failed_mode; d.pgroups = cfg->partition_groups; d.pstart = cfg->partition_start;
  d.pend = cfg->partition_end;
  const uint32_t Lid = cfg->id_len;
  d.capk = (BUFSZ - 20 - Lid) / (18 + Lid);           // 20 + L + k(18+L) <= 10240
  d.capj = (BUFSZ - 20 - Lid - 1) / (18 + Lid);       // 20 + L + k(18+L) <  10240
  d.paybound = C < d.capk ? C : d.capk;
  s->h_ident.assign((size_t)C * MAXID, 0); s->h_idlen.assign(C, (uint8_t)Lid); s->h_ever.assign(C, 0);
  for (uint32_t j = 0; j < C; ++j) default_identity(j, Lid, &s->h_ident[(size_t)j * MAXID]);
  for (uint32_t j = 0; j < cfg->initial_nodes; ++j) s->h_ever[j] = 1;
  hipError_t e = hipSuccess;
#define A(ptr, n) if (e == hipSuccess) e = dalloc(&(ptr), (n))
  A(d.stamp, (size_t)C * W); A(d.alive, C); A(d.start_round, C); A(d.n, C); A(d.fp, C); A(d.dirty, C);
  A(d.last_bcast, C); A(d.susp, (size_t)C * SLOTS); A(d.cur, (size_t)C * CSLOTS); A(d.paq, (size_t)C * PAQ);
  A(d.paq_n, C); A(d.cseg, C); A(d.segmul, C); A(d.seglen, C); A(d.zpow, (size_t)C + 2); A(d.ztab, 17 * 128);
  A(d.tmpl, W / 16); A(d.htab, (size_t)(W / 8) * 256); A(d.stats, NSTAT); A(d.ctr, NCTR); A(d.truefp, 1);
  s->msg_cap = std::max<uint32_t>(8u * C + (uint32_t)TICK_MAX * C, 1u << 16);
  s->pay_cap = std::max<uint32_t>((d.capk + 1) * C, 1u << 24);
  for (int b = 0; b < 2; ++b) {
    A(s->ob[b].msgs, s->msg_cap); A(s->ob[b].pay, s->pay_cap); A(s->ob[b].off, C); A(s->ob[b].cap, C);
    A(s->ob[b].cnt, C); A(s->ob[b].poff, C);
  }
  A(s->wc.status, s->msg_cap); A(s->wc.cnt1, C); A(s->wc.bnd, C); A(s->wc.bpay, C); A(s->wc.cursor, C);
  A(s->wc.in_off, C); A(s->wc.inbox, s->msg_cap); A(s->wc.active, C); A(s->wc.kp_list, s->msg_cap);
  A(s->wc.touched, C); A(s->wc.touched_list, C);
  A(s->bfail, (size_t)C * SLOTS); A(s->bjoin, C);
  A(s->bs.join, C); A(s->bs.nfail, C); A(s->bs.fail, (size_t)C * SLOTS); A(s->join_off, C); A(s->fail_off, C);
  A(s->scan_tot, 16); A(s->scan_tiles, 5 * ((C + 1023) / 1024) + 5);
  A(s->nresp, C); A(s->paysum, C); A(s->nbase, C); A(s->resp_off, C);
  A(s->resp_nodes, C); A(s->bf_gid, (size_t)C * SLOTS); A(s->bf_dep, (size_t)C * SLOTS);
  A(s->so.cand, (size_t)C * 5); A(s->so.ncand, C);
#undef A
  if (e != hipSuccess) { seterr(std::string("device allocation failed: ") + hipGetErrorString(e)); free_all(s); delete s; return KB_CAPACITY; }
  s->wc.msg_cap = s->msg_cap; s->wc.pay_cap = s->pay_cap;
  for (int b = 0; b < 2; ++b) { s->ob[b].msg_cap = s->msg_cap; s->ob[b].pay_cap = s->pay_cap; }
  s->newmask = nullptr; s->respmask = nullptr; s->mask_words = 0; s->items = nullptr; s->items_cap = 0;
  s->d_events = nullptr; s->events_cap = 0; s->nf = 0; s->nj = 0;
  if (hipStreamCreateWithFlags(&s->st, hipStreamNonBlocking) != hipSuccess) { free_all(s); delete s; seterr("stream"); return KB_IO_ERROR; }
  hipEventCreate(&s->ev0); hipEventCreate(&s->ev1); hipEventCreate(&s->er0); hipEventCreate(&s->er1);
  s->sweep_ms = s->round_ms = 0; s->sweep_launches = s->round_launches = s->sweep_bytes = 0;
  s->bj_total = s->bf_total = 0;
  int rc = upload_segments(s);
  if (rc) { free_all(s); delete s; return rc; }
  uint32_t ctr0[NCTR] = {0};
  ctr0[C_NEXTFREE] = cfg->initial_nodes;
  ctr0[C_FIRSTCONV] = 0xFFFFFFFFu; ctr0[C_LASTCONV] = 0xFFFFFFFFu;
  if (hipMemcpy(d.ctr, ctr0, sizeof ctr0, hipMemcpyHostToDevice) != hipSuccess) { free_all(s); delete s; return KB_IO_ERROR; }
  const uint32_t tb = 256, gb = (C + tb - 1) / tb;
  if (cfg->init_mode == KB_INIT_CONVERGED) {
    k_init_converged_rows<<<4096, 256, 0, s->st>>>(d, cfg->initial_nodes);
    k_init_converged_nodes<<<gb, tb, 0, s->st>>>(d, cfg->initial_nodes);
  } else {
    k_init_nodes<<<gb, tb, 0, s->st>>>(d, cfg->initial_nodes, cfg->init_mode);
  }
  if (hipStreamSynchronize(s->st) != hipSuccess) { free_all(s); delete s; seterr("init failed"); return KB_IO_ERROR; }
  *out = s;
  return KB_OK;
}

static void free_all(kb_sim* s) {
  Dev& d = s->d;
  void* ptrs[] = {d.stamp, d.alive, d.start_round, d.n, d.fp, d.dirty, d.last_bcast, d.susp, d.cur, d.paq, d.paq_n,
                  d.cseg, d.segmul, d.seglen, d.zpow, d.ztab, d.tmpl, d.htab, d.stats, d.ctr, d.truefp,
                  s->ob[0].msgs, s->ob[0].pay, s->ob[0].off, s->ob[0].cap, s->ob[0].cnt, s->ob[0].poff,
                  s->ob[1].msgs, s->ob[1].pay, s->ob[1].off, s->ob[1].cap, s->ob[1].cnt, s->ob[1].poff,
                  s->wc.status, s->wc.cnt1, s->wc.bnd, s->wc.bpay, s->wc.cursor, s->wc.in_off, s->wc.inbox,
                  s->wc.active, s->wc.kp_list, s->wc.touched, s->wc.touched_list, s->bfail, s->bjoin, s->bs.join,
                  s->bs.nfail, s->bs.fail, s->join_off, s->fail_off, s->scan_tot, s->scan_tiles, s->newmask, s->respmask, s->nresp,
                  s->paysum, s->nbase, s->resp_off, s->items, s->resp_nodes, s->bf_gid, s->bf_dep, s->so.cand, s->so.ncand, s->d_events};
  for (void* p : ptrs) if (p) hipFree(p);
}

extern "C" int kb_sim_destroy(kb_sim* s) {
  if (!s) return KB_INVALID_ARGUMENT;
  hipSetDevice(s->device);
  hipStreamSynchronize(s->st);
  free_all(s);
  hipEventDestroy(s->ev0); hipEventDestroy(s->ev1); hipEventDestroy(s->er0); hipEventDestroy(s->er1);
  hipStreamDestroy(s->st);
  delete s;
  return KB_OK;
}

static ScanArgs scan_args(kb_sim* s, uint32_t n, uint32_t* totals) {
  ScanArgs a; memset(&a, 0, sizeof a); a.n = n; a.totals = totals;
  a.tiles = s->scan_tiles; a.ntiles = (n + 1023) / 1024; return a;
}
static void launch_scan(const ScanArgs& a, hipStream_t st) {
  k_scan_tiles<<<a.ntiles, 1024, 0, st>>>(a);
  k_scan_apply<<<a.ntiles, 1024, 0, st>>>(a);
}

static int check_err(kb_sim* s) {
  uint32_t e = 0;
  HIPCHK(hipMemcpyAsync(&e, s->d.ctr + C_ERR, 4, hipMemcpyDeviceToHost, s->st));
  HIPCHK(hipStreamSynchronize(s->st));
  if (e) {
    const char* what[] = {"", "suspect slots exhausted", "outbox region overflow", "payload pool overflow",
                          "truncated Join response larger than the LDS bitmap", "inbox overflow",
                          "Join response member count mismatch"};
    seterr(std::string("device capacity error: ") + (e < 7 ? what[e] : "?"));
    return KB_CAPACITY;
  }
  return KB_OK;
}

static int step_round(kb_sim* s) {
  Dev& d = s->d;
  const int32_t r = s->round;
  const uint32_t C = s->C;
  hipStream_t st = s->st;
  const uint32_t tb = 256, gnode = (C + tb - 1) / tb, gwave = (C + 3) / 4;
  hipEventRecord(s->er0, st);
  // 0. stamp window
  if (r > 0 && r % EPOCH == 0) k_rebase<<<8192, 256, 0, st>>>(d);
  // 1. lifecycle
  if (!s->events.empty()) {
    if (s->events.size() > s->events_cap) {
      if (s->d_events) hipFree(s->d_events);
      s->events_cap = (uint32_t)s->events.size() * 2;
      HIPCHK(hipMalloc(&s->d_events, sizeof(Event) * s->events_cap));
    }
    HIPCHK(hipMemcpyAsync(s->d_events, s->events.data(), sizeof(Event) * s->events.size(), hipMemcpyHostToDevice, st));
    k_events<<<1, 1, 0, st>>>(d, s->d_events, (uint32_t)s->events.size(), r);
    HIPCHK(hipStreamSynchronize(st));
    s->events.clear();
  }
  const bool faults_on = s->cfg.fault_end_round < 0 || r < s->cfg.fault_end_round;
  if (faults_on && s->cfg.churn_threshold) {
    k_churn_leave<<<gnode, tb, 0, st>>>(d, r);
    k_churn_join<<<1, 1024, 0, st>>>(d, r);
  }
  k_template<<<(d.W / 16 + tb - 1) / tb, tb, 0, st>>>(d);
  k_truefp<<<1, 1024, 0, st>>>(d);
  // 2. broadcasts of round r-1
  OutBuf& o0 = s->ob[0];
  PhaseB pb;
  pb.bfail = s->bfail; pb.nf = s->nf; pb.bjoin = s->bjoin; pb.nj = s->nj; pb.JW = (s->nj + 63) / 64;
  pb.nresp = s->nresp; pb.paysum = s->paysum; pb.nbase = s->nbase;
  if (pb.JW) {
    const size_t words = (size_t)C * pb.JW;
    if (words > s->mask_words) {
      if (s->newmask) hipFree(s->newmask);
      if (s->respmask) hipFree(s->respmask);
      s->newmask = nullptr; s->respmask = nullptr;
      HIPCHK(hipMalloc(&s->newmask, 8 * words)); HIPCHK(hipMalloc(&s->respmask, 8 * words));
      s->mask_words = words;
    }
  }
  pb.newmask = s->newmask; pb.respmask = s->respmask;
  pb.gid = s->bf_gid; pb.dep = s->bf_dep;
  const bool have_b = s->nf + s->nj > 0;
  if (s->nf) k_bfail_prep<<<(s->nf + 255) / 256, 256, 0, st>>>(s->bfail, s->nf, s->bf_gid, s->bf_dep);
  if (have_b) k_phaseB<<<gwave, 256, 0, st>>>(d, pb, r);
  else { HIPCHK(hipMemsetAsync(s->nresp, 0, 4ull * C, st)); HIPCHK(hipMemsetAsync(s->paysum, 0, 4ull * C, st)); }
  // wave-0 outbox regions: responses then tick messages
  {
    ScanArgs a = scan_args(s, C, s->scan_tot);
    a.narr = 3;
    a.in[0] = s->nresp; a.out[0] = s->resp_off;
    a.in[1] = s->paysum; a.out[1] = o0.poff;
    a.in[2] = s->nresp; a.out[2] = o0.off; a.addc[2] = TICK_MAX;
    a.list = s->resp_nodes;
    launch_scan(a, st);
    // cap = nresp + TICK_MAX: computed from consecutive offsets inside k_resp_list's caller below
  }
  k_set_cap<<<gnode, tb, 0, st>>>(C, s->nresp, o0.cap, o0.cnt);
  if (have_b) {
    uint32_t tot[5];
    HIPCHK(hipMemcpyAsync(tot, s->scan_tot, 20, hipMemcpyDeviceToHost, st));
    HIPCHK(hipStreamSynchronize(st));
    const uint32_t nresp_tot = tot[0], pay_tot = tot[1], msg_tot = tot[2], resp_nodes = tot[4];
    if (msg_tot > s->msg_cap || pay_tot > s->pay_cap) { seterr("wave-0 outbox exceeds preallocated capacity"); return KB_CAPACITY; }
    if (nresp_tot > s->items_cap) {
      if (s->items) hipFree(s->items);
      s->items_cap = nresp_tot * 2 + 1024;
      HIPCHK(hipMalloc(&s->items, sizeof(RespItem) * s->items_cap));
    }
    if (s->W <= RESP_LDS_W) {
      const size_t lds = 4ull * (3 * (s->W / 32) + s->W / 256 + 1 + 256 + 1024);
      if (resp_nodes) k_resp_node<<<std::min<uint32_t>(resp_nodes, 4096), 256, lds, st>>>(d, pb, s->resp_nodes, s->scan_tot + 4, o0, r);
    } else {
      k_resp_list<<<gnode, tb, 0, st>>>(d, pb, s->resp_off, o0.poff, s->items, o0);
      if (nresp_tot) k_resp_build<<<std::min<uint32_t>(nresp_tot, 8192), 64, 0, st>>>(d, pb, s->items, s->scan_tot, o0, r);
    }
  }
  // 3. tick
  k_tick_pre<<<gwave, 256, 0, st>>>(d, o0, s->bs, r);
  hipEventRecord(s->ev0, st);
  k_sweep<<<gwave, 256, 0, st>>>(d, s->so);
  hipEventRecord(s->ev1, st);
  k_tick_post<<<gnode, tb, 0, st>>>(d, s->so, o0, r);
  {
    ScanArgs a = scan_args(s, C, s->scan_tot);
    a.narr = 2;
    a.in[0] = s->bs.join; a.out[0] = s->join_off;
    a.in[1] = s->bs.nfail; a.out[1] = s->fail_off;
    launch_scan(a, st);
  }
  k_bcast_write<<<gnode, tb, 0, st>>>(d, s->bs, s->join_off, s->fail_off, s->bjoin, s->bfail);
  // 4. waves
  int cur = 0;
  for (uint32_t w = 0; w <= s->cfg.max_waves; ++w) {
    OutBuf& ib = s->ob[cur];
    OutBuf& nb = s->ob[cur ^ 1];
    const int last = w == s->cfg.max_waves;
    HIPCHK(hipMemsetAsync(s->wc.cnt1, 0, 4ull * C, st));
    HIPCHK(hipMemsetAsync(s->wc.bnd, 0, 4ull * C, st));
    HIPCHK(hipMemsetAsync(s->wc.bpay, 0, 4ull * C, st));
    HIPCHK(hipMemsetAsync(s->wc.cursor, 0, 4ull * C, st));
    HIPCHK(hipMemsetAsync(d.ctr + C_KP, 0, 12, st));   // C_KP, C_TOUCH, C_ACTIVE
    k_route<<<gnode, tb, 0, st>>>(d, ib, s->wc, r, w, last);
    if (last) break;
    {
      ScanArgs a = scan_args(s, C, s->scan_tot + 8);
      a.narr = 3;
      a.in[0] = s->wc.cnt1; a.out[0] = s->wc.in_off;
      a.in[1] = s->wc.bnd; a.out[1] = nb.off;
      a.in[2] = s->wc.bpay; a.out[2] = nb.poff;
      a.list = s->wc.active; a.list_count = d.ctr + C_ACTIVE;
      launch_scan(a, st);
    }
    HIPCHK(hipMemcpyAsync(nb.cap, s->wc.bnd, 4ull * C, hipMemcpyDeviceToDevice, st));
    HIPCHK(hipMemsetAsync(nb.cnt, 0, 4ull * C, st));
    k_scatter<<<gnode, tb, 0, st>>>(d, ib, s->wc);
    k_kp_insert<<<2048, 256, 0, st>>>(d, ib, s->wc, r);
    k_kp_prologue<<<1024, 256, 0, st>>>(d, ib, s->wc, r);
    k_touch_fix<<<1024, 256, 0, st>>>(d, s->wc);
    k_proc<<<4096, 256, 0, st>>>(d, ib, nb, s->wc, r);
    cur ^= 1;
  }
  k_round_end<<<1, 1, 0, st>>>(d, r);
  hipEventRecord(s->er1, st);
  // broadcast list sizes for the next round (the round's single host read)
  uint32_t tot[2], alive_now = 0;
  HIPCHK(hipMemcpyAsync(tot, s->scan_tot, 8, hipMemcpyDeviceToHost, st));
  HIPCHK(hipMemcpyAsync(&alive_now, d.ctr + C_LASTALIVE, 4, hipMemcpyDeviceToHost, st));
  HIPCHK(hipStreamSynchronize(st));
  s->nj = tot[0]; s->nf = tot[1];
  s->bj_total += s->nj; s->bf_total += s->nf;
  s->sweep_bytes += (uint64_t)alive_now * C;
  float ms = 0;
  hipEventElapsedTime(&ms, s->ev0, s->ev1); s->sweep_ms += ms; s->sweep_launches++;
  hipEventElapsedTime(&ms, s->er0, s->er1); s->round_ms += ms; s->round_launches++;
  s->round = r + 1;
  return check_err(s);
}

extern "C" int kb_sim_step(kb_sim* s, uint32_t rounds) {
  if (!s) return KB_INVALID_ARGUMENT;
  hipSetDevice(s->device);
  for (uint32_t k = 0; k < rounds; ++k) {
    // algorithmic bytes of this round's sweep: every running row once
    int rc = step_round(s);
    if (rc) return rc;
  }
  return KB_OK;
}

// ---------------------------------------------------------------------------------- API surface
static int chk(kb_sim* s, uint32_t node) { return (!s || node >= s->C) ? KB_INVALID_ARGUMENT : KB_OK; }

extern "C" int kb_sim_start_node(kb_sim* s, uint32_t node) {
  if (chk(s, node)) return KB_INVALID_ARGUMENT;
  s->events.push_back(Event{node, 0});
  s->h_ever[node] = 1;
  return KB_OK;
}
extern "C" int kb_sim_stop_node(kb_sim* s, uint32_t node) {
  if (chk(s, node)) return KB_INVALID_ARGUMENT;
  s->events.push_back(Event{node, 1});
  return KB_OK;
}
extern "C" int kb_sim_is_running(kb_sim* s, uint32_t node, int* running) {
  if (chk(s, node) || !running) return KB_INVALID_ARGUMENT;
  uint8_t a = 0;
  HIPCHK(hipMemcpy(&a, s->d.alive + node, 1, hipMemcpyDeviceToHost));
  *running = a;
  return KB_OK;
}
extern "C" int kb_sim_ping_addrs(kb_sim* s, uint32_t node, const uint32_t* peers, size_t n) {
  if (chk(s, node) || (n && !peers)) return KB_INVALID_ARGUMENT;
  uint8_t a = 0;
  HIPCHK(hipMemcpy(&a, s->d.alive + node, 1, hipMemcpyDeviceToHost));
  if (!a) { seterr("Cannot ping while we are not started"); return KB_INVALID_OPERATION; }
  uint32_t qn = 0;
  HIPCHK(hipMemcpy(&qn, s->d.paq_n + node, 4, hipMemcpyDeviceToHost));
  std::vector<uint32_t> q(PAQ);
  HIPCHK(hipMemcpy(q.data(), s->d.paq + (size_t)node * PAQ, 4 * PAQ, hipMemcpyDeviceToHost));
  for (size_t k = 0; k < n; ++k) {
    if (peers[k] >= s->C) return KB_INVALID_ARGUMENT;
    uint8_t b = 0;
    HIPCHK(hipMemcpy(&b, s->d.stamp + (size_t)node * s->W + peers[k], 1, hipMemcpyDeviceToHost));
    if (b != ST_UNKNOWN) continue;
    if (qn == PAQ) { seterr("ping_addrs queue full"); return KB_CAPACITY; }
    q[qn++] = peers[k];
  }
  HIPCHK(hipMemcpy(s->d.paq + (size_t)node * PAQ, q.data(), 4 * PAQ, hipMemcpyHostToDevice));
  HIPCHK(hipMemcpy(s->d.paq_n + node, &qn, 4, hipMemcpyHostToDevice));
  return KB_OK;
}
__global__ void k_mark_dirty(Dev d) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < d.C) d.dirty[i] = 1;
}
extern "C" int kb_sim_set_identity(kb_sim* s, uint32_t node, const uint8_t* identity, size_t len) {
  if (chk(s, node) || len > MAXID || (len && !identity)) return KB_INVALID_ARGUMENT;
  uint8_t a = 0;
  HIPCHK(hipMemcpy(&a, s->d.alive + node, 1, hipMemcpyDeviceToHost));
  uint32_t nfree = 0;
  HIPCHK(hipMemcpy(&nfree, s->d.ctr + C_NEXTFREE, 4, hipMemcpyDeviceToHost));
  const bool ever = s->h_ever[node] || (node < nfree && node >= s->cfg.initial_nodes && s->cfg.churn_threshold);
  if (a || ever) { seterr("Cannot change identity while the mesh is running; call .stop first"); return KB_INVALID_OPERATION; }
  if (len != s->cfg.id_len && s->C > 200) { seterr("non-uniform identity length needs capacity <= 200"); return KB_INVALID_ARGUMENT; }
  memcpy(&s->h_ident[(size_t)node * MAXID], identity, len);
  s->h_idlen[node] = (uint8_t)len;
  int rc = upload_segments(s);
  if (rc) return rc;
  k_mark_dirty<<<(s->C + 255) / 256, 256, 0, s->st>>>(s->d);
  HIPCHK(hipStreamSynchronize(s->st));
  return KB_OK;
}

__global__ __launch_bounds__(64) void k_fp_one(Dev d, uint32_t i) {
  __shared__ uint32_t ztab[ZT * 128];
  load_ztab(d, ztab);
  if (!d.dirty[i]) return;
  const uint32_t f = wave_fold(d, row_of(d, i), ztab);
  if (lane() == 0) { d.fp[i] = f; d.dirty[i] = 0; }
}
__global__ __launch_bounds__(256) void k_fp_all(Dev d) {
  __shared__ uint32_t ztab[ZT * 128];
  load_ztab(d, ztab);
  const uint32_t i = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (i >= d.C || !d.dirty[i]) return;
  const uint32_t f = wave_fold(d, row_of(d, i), ztab);
  if (lane() == 0) { d.fp[i] = f; d.dirty[i] = 0; }
}

extern "C" int kb_sim_fingerprint(kb_sim* s, uint32_t node, uint32_t* fp) {
  if (chk(s, node) || !fp) return KB_INVALID_ARGUMENT;
  k_fp_one<<<1, 64, 0, s->st>>>(s->d, node);
  HIPCHK(hipMemcpyAsync(fp, s->d.fp + node, 4, hipMemcpyDeviceToHost, s->st));
  HIPCHK(hipStreamSynchronize(s->st));
  return KB_OK;
}
extern "C" int kb_sim_fingerprints(kb_sim* s, uint32_t* fps, size_t cap) {
  if (!s || !fps || cap < s->C) return KB_INVALID_ARGUMENT;
  k_fp_all<<<(s->C + 3) / 4, 256, 0, s->st>>>(s->d);
  std::vector<uint8_t> al(s->C);
  HIPCHK(hipMemcpyAsync(fps, s->d.fp, 4ull * s->C, hipMemcpyDeviceToHost, s->st));
  HIPCHK(hipMemcpyAsync(al.data(), s->d.alive, s->C, hipMemcpyDeviceToHost, s->st));
  HIPCHK(hipStreamSynchronize(s->st));
  for (uint32_t i = 0; i < s->C; ++i) if (!al[i]) fps[i] = 0;
  return KB_OK;
}
extern "C" int kb_sim_true_fingerprint(kb_sim* s, uint32_t* fp) {
  if (!s || !fp) return KB_INVALID_ARGUMENT;
  k_template<<<(s->d.W / 16 + 255) / 256, 256, 0, s->st>>>(s->d);
  k_truefp<<<1, 1024, 0, s->st>>>(s->d);
  HIPCHK(hipMemsetAsync(s->d.ctr + C_ALIVE, 0, 4, s->st));
  HIPCHK(hipMemcpyAsync(fp, s->d.truefp, 4, hipMemcpyDeviceToHost, s->st));
  HIPCHK(hipStreamSynchronize(s->st));
  return KB_OK;
}
extern "C" int kb_sim_dump_row(kb_sim* s, uint32_t node, uint8_t* rw, size_t cap) {
  if (chk(s, node) || !rw || cap < s->C) return KB_INVALID_ARGUMENT;
  HIPCHK(hipMemcpy(rw, s->d.stamp + (size_t)node * s->W, s->C, hipMemcpyDeviceToHost));
  return KB_OK;
}
extern "C" int kb_sim_peers(kb_sim* s, uint32_t node, uint32_t* peers, size_t cap, size_t* n) {
  if (chk(s, node) || !n) return KB_INVALID_ARGUMENT;
  std::vector<uint8_t> rw(s->C);
  HIPCHK(hipMemcpy(rw.data(), s->d.stamp + (size_t)node * s->W, s->C, hipMemcpyDeviceToHost));
  size_t c = 0;
  for (uint32_t j = 0; j < s->C; ++j) if (rw[j]) { if (peers && c < cap) peers[c] = j; c++; }
  *n = c;
  return (peers && cap < c) ? KB_CAPACITY : KB_OK;
}
extern "C" int kb_sim_peer_states(kb_sim* s, uint32_t node, kb_peer_state* out, size_t cap, size_t* n) {
  if (chk(s, node) || !n) return KB_INVALID_ARGUMENT;
  std::vector<uint8_t> rw(s->C);
  std::vector<Susp> sl(SLOTS);
  HIPCHK(hipMemcpy(rw.data(), s->d.stamp + (size_t)node * s->W, s->C, hipMemcpyDeviceToHost));
  HIPCHK(hipMemcpy(sl.data(), s->d.susp + (size_t)node * SLOTS, sizeof(Susp) * SLOTS, hipMemcpyDeviceToHost));
  const int32_t E = epoch_base(s->round);
  size_t c = 0;
  for (uint32_t j = 0; j < s->C; ++j) {
    if (!rw[j]) continue;
    if (out && c < cap) {
      kb_peer_state& o = out[c];
      o.peer = j; o.reserved = 0;
      if (rw[j] == ST_SUSPECT) {
        const Susp* q = nullptr;
        for (auto& x : sl) if (x.kind && x.peer == j) q = &x;
        o.state = q && q->kind == SK_WFIP ? KB_STATE_WAITING_FOR_INDIRECT_PING : KB_STATE_WAITING_FOR_PING;
        o.since = q ? q->since : 0;
      } else {
        o.state = KB_STATE_KNOWN;
        o.since = rw[j] == ST_ANCIENT ? INT32_MIN : (int32_t)rw[j] + E - EOFF;
      }
    }
    c++;
  }
  *n = c;
  return (out && cap < c) ? KB_CAPACITY : KB_OK;
}
extern "C" int kb_sim_stats(kb_sim* s, kb_stats* out) {
  if (!s || !out) return KB_INVALID_ARGUMENT;
  unsigned long long st[NSTAT];
  uint32_t ctr[NCTR];
  HIPCHK(hipMemcpy(st, s->d.stats, sizeof st, hipMemcpyDeviceToHost));
  HIPCHK(hipMemcpy(ctr, s->d.ctr, sizeof ctr, hipMemcpyDeviceToHost));
  std::vector<uint8_t> al(s->C);
  HIPCHK(hipMemcpy(al.data(), s->d.alive, s->C, hipMemcpyDeviceToHost));
  memset(out, 0, sizeof *out);
  out->round = s->round;
  uint32_t a = 0;
  for (uint8_t x : al) a += x;
  out->alive = a;
  out->agree = ctr[C_LASTAGREE];
  out->first_converged_round = (int32_t)ctr[C_FIRSTCONV];
  out->last_converged_round = (int32_t)ctr[C_LASTCONV];
  out->next_free_id = ctr[C_NEXTFREE];
  out->sent_ping = st[S_PING]; out->sent_ping_req = st[S_PINGREQ]; out->sent_ack = st[S_ACK];
  out->sent_known_peers = st[S_KP]; out->sent_kpr = st[S_KPR];
  out->bcast_join = s->bj_total; out->bcast_failed = s->bf_total;
  out->drop_dead = st[S_DEAD]; out->drop_loss = st[S_LOSS]; out->drop_window = st[S_WINDOW];
  out->drop_oversize = st[S_OVERSIZE]; out->drop_partition = st[S_PART]; out->drop_bcast = st[S_BDROP];
  out->removed_timeout = st[S_RMTIMEOUT]; out->removed_failed = st[S_RMFAILED]; out->join_responses = st[S_JRESP];
  out->curious_overflow = st[S_CUROVF]; out->churn_leaves = st[S_CLEAVE]; out->churn_joins = st[S_CJOIN];
  return KB_OK;
}
extern "C" int kb_sim_dump_scalars(kb_sim* s, int32_t* out, size_t cap) {
  if (!s || !out || cap < 4ull * s->C) return KB_INVALID_ARGUMENT;
  std::vector<uint8_t> al(s->C);
  std::vector<uint32_t> n(s->C);
  std::vector<int32_t> lb(s->C), sr(s->C);
  HIPCHK(hipMemcpy(al.data(), s->d.alive, s->C, hipMemcpyDeviceToHost));
  HIPCHK(hipMemcpy(n.data(), s->d.n, 4ull * s->C, hipMemcpyDeviceToHost));
  HIPCHK(hipMemcpy(lb.data(), s->d.last_bcast, 4ull * s->C, hipMemcpyDeviceToHost));
  HIPCHK(hipMemcpy(sr.data(), s->d.start_round, 4ull * s->C, hipMemcpyDeviceToHost));
  for (uint32_t i = 0; i < s->C; ++i) { out[4 * i] = al[i]; out[4 * i + 1] = (int32_t)n[i]; out[4 * i + 2] = lb[i]; out[4 * i + 3] = sr[i]; }
  return KB_OK;
}
extern "C" int kb_sim_dump_suspects(kb_sim* s, uint32_t node, int32_t* out, size_t cap, size_t* n) {
  if (chk(s, node) || !n) return KB_INVALID_ARGUMENT;
  Susp sl[SLOTS];
  HIPCHK(hipMemcpy(sl, s->d.susp + (size_t)node * SLOTS, sizeof sl, hipMemcpyDeviceToHost));
  std::vector<std::array<int32_t, 3>> v;
  for (auto& x : sl) if (x.kind) v.push_back({(int32_t)x.peer, x.kind, x.since});
  std::sort(v.begin(), v.end());
  *n = v.size();
  if (out) { if (cap < 3 * v.size()) return KB_CAPACITY; for (size_t k = 0; k < v.size(); ++k) memcpy(out + 3 * k, v[k].data(), 12); }
  return KB_OK;
}
extern "C" int kb_sim_dump_curious(kb_sim* s, uint32_t node, int32_t* out, size_t cap, size_t* n) {
  if (chk(s, node) || !n) return KB_INVALID_ARGUMENT;
  Cur cu[CSLOTS];
  HIPCHK(hipMemcpy(cu, s->d.cur + (size_t)node * CSLOTS, sizeof cu, hipMemcpyDeviceToHost));
  std::vector<std::array<int32_t, 6>> v;
  for (auto& x : cu) if (x.used) {
    std::array<int32_t, 6> e{(int32_t)x.peer, (int32_t)x.nobs, -1, -1, -1, -1};
    for (uint32_t q = 0; q < x.nobs && q < NOBS; ++q) e[2 + q] = (int32_t)x.obs[q];
    v.push_back(e);
  }
  std::sort(v.begin(), v.end(), [](const std::array<int32_t, 6>& a, const std::array<int32_t, 6>& b) { return a[0] < b[0]; });
  *n = v.size();
  if (out) { if (cap < 6 * v.size()) return KB_CAPACITY; for (size_t k = 0; k < v.size(); ++k) memcpy(out + 6 * k, v[k].data(), 24); }
  return KB_OK;
}
extern "C" uint32_t kb_fingerprint_of_set(const uint32_t* ids, size_t n, const uint8_t* identities, size_t id_stride,
                                          const uint8_t* id_lens) {
  h_crc_init();
  std::vector<uint32_t> v(ids, ids + n);
  std::sort(v.begin(), v.end());
  uint32_t reg = 0xFFFFFFFFu;
  char a[32];
  for (uint32_t id : v) {
    kb_format_addr(id, a, sizeof a);
    reg = h_crc_update(reg, (const uint8_t*)a, strlen(a));
    if (identities && id_lens) reg = h_crc_update(reg, identities + (size_t)id * id_stride, id_lens[id]);
  }
  return reg ^ 0xFFFFFFFFu;
}
extern "C" int kb_sim_kernel_time(kb_sim* s, int kind, double* ms, uint64_t* launches) {
  if (!s || !ms || !launches) return KB_INVALID_ARGUMENT;
  if (kind == 0) { *ms = s->sweep_ms; *launches = s->sweep_launches; }
  else { *ms = s->round_ms; *launches = s->round_launches; }
  return KB_OK;
}
extern "C" int kb_sim_reset_kernel_time(kb_sim* s) {
  if (!s) return KB_INVALID_ARGUMENT;
  s->sweep_ms = s->round_ms = 0; s->sweep_launches = s->round_launches = 0; s->sweep_bytes = 0;
  return KB_OK;
}
extern "C" int kb_sim_sweep_bytes(kb_sim* s, uint64_t* bytes) {
  if (!s || !bytes) return KB_INVALID_ARGUMENT;
  *bytes = s->sweep_bytes;
  return KB_OK;
}
