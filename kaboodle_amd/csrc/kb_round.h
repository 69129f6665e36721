// kb_round.h — round-start kernels: stamp window, lifecycle, running set, broadcast phase and Join
// responses (included by kb_sim.hip).
#pragma once
#include "kb_common.h"

namespace kb {

// ---- stamp window: every 64 rounds known stamps shift down, saturating at "ancient"
// (KB_VARIANT_EXACT_LRU: a byte that saturates hands its instant, decoded with the epoch it was written in, to
// the tst table; every stamp write is Known(now) or Known(r - 10), so a byte above ANCIENT encodes its instant)
__global__ void k_rebase(Dev d, int32_t r) {
  const size_t total = (size_t)(d.hi - d.lo) * d.W / 16;     // the local rows
  const uint32_t wpr = d.W / 16;
  const int32_t E = epoch_base(r - 1);                      // the epoch the bytes were written in
  uint4* p = reinterpret_cast<uint4*>(d.stamp + (size_t)d.lo * d.W);
  for (size_t k = (size_t)blockIdx.x * blockDim.x + threadIdx.x; k < total; k += (size_t)gridDim.x * blockDim.x) {
    const uint4 v = p[k];
    uint32_t w[4] = {v.x, v.y, v.z, v.w};
    bool any = false;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      uint32_t x = w[q], y = 0;
#pragma unroll
      for (int t = 0; t < 4; ++t) {
        uint32_t b = (x >> (8 * t)) & 0xFF;
        if (b > ST_ANCIENT) {
          if (d.tst && b <= ST_ANCIENT + EPOCH) {
            const size_t i = d.lo + k / wpr, j = (k % wpr) * 16 + q * 4 + t;
            d.tst[i * d.W + j] = (int32_t)b - EOFF + E;
            atomicMin(d.tlb + i * (d.W >> 10) + (j >> 10), (int32_t)b - EOFF + E);   // the block's bound covers it
          }
          b = b > ST_ANCIENT + EPOCH ? b - EPOCH : ST_ANCIENT; any = true;   // unsigned: no b - EPOCH < 0
        }
        y |= b << (8 * t);
      }
      w[q] = y;
    }
    if (any) p[k] = make_uint4(w[0], w[1], w[2], w[3]);
  }
}

// KB_VARIANT_EXACT_LRU: ping_random_peer's oldest five by the exact instant of the last contact
// (src/kaboodle.rs:662-675 sorts by Instant), ties broken by the rotated address from the sweep front, over the
// whole row; written as the row pass's keys (rank << 24 | rotated id) for k_tick_post.  A wave per row, 16 ids per
// lane per 1024-id block: stamp bytes, member bits, and the saturated entries' instants.
//   A saturated instant is older than every instant a byte still encodes (it was written an epoch earlier), so the
// five oldest are the saturated ones whenever a row holds five.  Those are found block by block in the order of a
// lower bound, tlb (instant) with the block's smallest rotated id: a block is scanned only while its bound is below
// the fifth key found so far, and the scan makes its tlb exact.  k_rebase lowers tlb for every entry it saturates;
// a refresh leaves it low (still a bound).  Only a row with fewer than five saturated candidates reads its live bytes.
// 64-bit keys: the DPP scan of kb_device.h on both halves (identity ~0), the minimum read from the last lane
template <int CTRL, int RM>
__device__ __attribute__((always_inline)) inline unsigned long long min64_dpp(unsigned long long x) {
  const uint32_t lo = (uint32_t)__builtin_amdgcn_update_dpp(-1, (int)(uint32_t)x, CTRL, RM, 0xF, false);
  const uint32_t hi = (uint32_t)__builtin_amdgcn_update_dpp(-1, (int)(uint32_t)(x >> 32), CTRL, RM, 0xF, false);
  const unsigned long long y = ((unsigned long long)hi << 32) | lo;
  return y < x ? y : x;
}
__device__ inline unsigned long long wave_min_u64(unsigned long long v) {
  v = min64_dpp<0x111, 0xF>(v); v = min64_dpp<0x112, 0xF>(v); v = min64_dpp<0x114, 0xF>(v);
  v = min64_dpp<0x118, 0xF>(v); v = min64_dpp<0x142, 0xA>(v); v = min64_dpp<0x143, 0xC>(v);
  return ((unsigned long long)wave_last((uint32_t)(v >> 32)) << 32) | wave_last((uint32_t)v);
}
// the wave's five smallest keys, ascending (~0: fewer); keys are distinct (rotated ids), so one lane pops each
__device__ inline void wave_top5(const unsigned long long top[5], unsigned long long m5[5]) {
  unsigned long long t0 = top[0], t1 = top[1], t2 = top[2], t3 = top[3], t4 = top[4];
#pragma unroll
  for (int k = 0; k < 5; ++k) {
    const unsigned long long m = wave_min_u64(t0);
    m5[k] = m;
    if (m != ~0ull && t0 == m) { t0 = t1; t1 = t2; t2 = t3; t3 = t4; t4 = ~0ull; }
  }
}
template <bool SAT, bool LIVE>
__device__ inline int32_t a3x_block(const Dev& d, uint32_t i, uint32_t b, uint32_t cur, int32_t E, const uint8_t* srow,
                                    const uint32_t* brow, const int32_t* trow, unsigned long long top[5]) {
  const uint32_t C = d.C, j0 = (b << 10) + 16 * lane();
  const uint32_t bw = (brow[j0 >> 5] >> (j0 & 31)) & 0xFFFFu;
  int32_t smin = INT32_MAX;                                          // the block's saturated minimum (SAT)
  if (!bw) return smin;
  const uint4 sv = *reinterpret_cast<const uint4*>(srow + j0);
  const uint32_t s4[4] = {sv.x, sv.y, sv.z, sv.w};
  int32_t t16[16];                                                   // the lane's 16 instants: four 16-byte loads
  if (SAT) {
    uint32_t anc = 0;
#pragma unroll
    for (uint32_t t = 0; t < 16; ++t) anc |= (((s4[t >> 2] >> (8 * (t & 3))) & 0xFFu) == ST_ANCIENT) ? (1u << t) : 0u;
    if (anc & bw) {
      const int4* tp = reinterpret_cast<const int4*>(trow + j0);
#pragma unroll
      for (uint32_t q = 0; q < 4; ++q) { const int4 v = tp[q]; t16[4 * q] = v.x; t16[4 * q + 1] = v.y; t16[4 * q + 2] = v.z; t16[4 * q + 3] = v.w; }
    }
  }
#pragma unroll
  for (uint32_t t = 0; t < 16; ++t) {
    if (!((bw >> t) & 1u)) continue;
    const uint32_t j = j0 + t;
    if (j >= C || j == i) continue;
    const uint32_t sb = (s4[t >> 2] >> (8 * (t & 3))) & 0xFFu;
    if (sb < ST_ANCIENT) continue;                                   // WaitingFor*: not a candidate
    int32_t inst;
    if (sb == ST_ANCIENT) {
      if (!SAT) continue;
      inst = t16[t];
      smin = inst < smin ? inst : smin;
    } else {
      if (!LIVE) continue;
      inst = (int32_t)sb - EOFF + E;
    }
    const uint32_t rot = j > cur ? j - cur - 1 : j + C - cur - 1;
    unsigned long long key = ((unsigned long long)((uint32_t)inst ^ 0x80000000u) << 32) | rot;
    if (key >= top[4]) continue;
#pragma unroll
    for (int q = 0; q < 5; ++q) { if (key < top[q]) { const unsigned long long x = top[q]; top[q] = key; key = x; } }
  }
  return smin;
}
constexpr uint32_t A3X_KPL = 8;                                     // bounds per lane: rows up to 512K ids
// one saturated-block scan's operands, loaded before any is used: member bits, stamp bytes and the 16 instants of
// the lane's 16 ids (every scanned block holds a saturated entry by its bound, so its instants are read anyway)
struct A3Blk { uint32_t bw; uint4 sv; int4 t[4]; };
__device__ __attribute__((always_inline)) inline void a3x_load(const uint8_t* srow, const uint32_t* brow, const int32_t* trow,
                                                               uint32_t b, A3Blk& x) {
  const uint32_t j0 = (b << 10) + 16 * lane();
  x.bw = (brow[j0 >> 5] >> (j0 & 31)) & 0xFFFFu;
  x.sv = *reinterpret_cast<const uint4*>(srow + j0);
  const int4* tp = reinterpret_cast<const int4*>(trow + j0);
#pragma unroll
  for (uint32_t q = 0; q < 4; ++q) x.t[q] = tp[q];
}
// the saturated entries of a loaded block into the lane's five smallest keys; returns the lane's saturated minimum
__device__ __attribute__((always_inline)) inline int32_t a3x_sat(uint32_t i, uint32_t C, uint32_t b, uint32_t cur,
                                                                 const A3Blk& x, unsigned long long top[5]) {
  const uint32_t j0 = (b << 10) + 16 * lane();
  const uint32_t s4[4] = {x.sv.x, x.sv.y, x.sv.z, x.sv.w};
  const int32_t t16[16] = {x.t[0].x, x.t[0].y, x.t[0].z, x.t[0].w, x.t[1].x, x.t[1].y, x.t[1].z, x.t[1].w,
                           x.t[2].x, x.t[2].y, x.t[2].z, x.t[2].w, x.t[3].x, x.t[3].y, x.t[3].z, x.t[3].w};
  int32_t smin = INT32_MAX;
#pragma unroll
  for (uint32_t t = 0; t < 16; ++t) {
    const uint32_t j = j0 + t;
    if (!((x.bw >> t) & 1u) || j >= C || j == i || ((s4[t >> 2] >> (8 * (t & 3))) & 0xFFu) != ST_ANCIENT) continue;
    const int32_t inst = t16[t];
    smin = inst < smin ? inst : smin;
    const uint32_t rot = j > cur ? j - cur - 1 : j + C - cur - 1;
    unsigned long long key = ((unsigned long long)((uint32_t)inst ^ 0x80000000u) << 32) | rot;
    if (key >= top[4]) continue;
#pragma unroll
    for (int q = 0; q < 5; ++q) { if (key < top[q]) { const unsigned long long y = top[q]; top[q] = key; key = y; } }
  }
  return smin;
}
// 32-bit keys for the common case: (min(instant − base, 255) << 24) | rotated id, base = the first scanned block's
// bound, the smallest bound of the row (blocks are scanned in bound order), so no key's offset is negative.  The map
// keeps the order of every key whose offset is below 255 and puts the rest above them all, so when the fifth
// smallest 32-bit key has an offset below 255 the five are exactly the five smallest 64-bit keys; otherwise (or with
// fewer than five saturated) the row is redone with 64-bit keys.  Rotated ids fit 24 bits: the narrow path holds
// rows up to 512K ids.
__device__ __attribute__((always_inline)) inline int32_t a3x_sat32(uint32_t i, uint32_t C, uint32_t b, uint32_t cur,
                                                                   int32_t base, const A3Blk& x, uint32_t top[5]) {
  const uint32_t j0 = (b << 10) + 16 * lane();
  const uint32_t s4[4] = {x.sv.x, x.sv.y, x.sv.z, x.sv.w};
  const int32_t t16[16] = {x.t[0].x, x.t[0].y, x.t[0].z, x.t[0].w, x.t[1].x, x.t[1].y, x.t[1].z, x.t[1].w,
                           x.t[2].x, x.t[2].y, x.t[2].z, x.t[2].w, x.t[3].x, x.t[3].y, x.t[3].z, x.t[3].w};
  int32_t smin = INT32_MAX;
#pragma unroll
  for (uint32_t t = 0; t < 16; ++t) {
    const uint32_t j = j0 + t;
    if (!((x.bw >> t) & 1u) || j >= C || j == i || ((s4[t >> 2] >> (8 * (t & 3))) & 0xFFu) != ST_ANCIENT) continue;
    const int32_t inst = t16[t];
    smin = inst < smin ? inst : smin;
    const uint32_t off = (uint32_t)inst - (uint32_t)base;              // inst >= base: exact as unsigned
    const uint32_t rot = j > cur ? j - cur - 1 : j + C - cur - 1;
    uint32_t key = ((off < 255u ? off : 255u) << 24) | rot;
    if (key >= top[4]) continue;
#pragma unroll
    for (int q = 0; q < 5; ++q) { const uint32_t lo = key < top[q] ? key : top[q], hi = key < top[q] ? top[q] : key; top[q] = lo; key = hi; }
  }
  return smin;
}
// the wave's five smallest 32-bit keys, ascending (~0: fewer); keys are distinct (rotated ids)
__device__ inline void wave_top5_32(const uint32_t top[5], uint32_t m5[5]) {
  uint32_t t0 = top[0], t1 = top[1], t2 = top[2], t3 = top[3], t4 = top[4];
#pragma unroll
  for (int k = 0; k < 5; ++k) {
    const uint32_t m = wave_min(t0);
    m5[k] = m;
    if (m != ~0u && t0 == m) { t0 = t1; t1 = t2; t2 = t3; t3 = t4; t4 = ~0u; }
  }
}
// the lane's smallest (bound, rotated start) block key and its block
template <uint32_t KPL>
__device__ __attribute__((always_inline)) inline unsigned long long a3x_lane_min(const int32_t lbk[KPL], const uint32_t rkey[KPL],
                                                                                 uint32_t& bm) {
  unsigned long long lm = ~0ull;
#pragma unroll
  for (uint32_t k = 0; k < KPL; ++k) {
    if (lbk[k] == INT32_MAX) continue;
    const unsigned long long key = ((unsigned long long)((uint32_t)lbk[k] ^ 0x80000000u) << 32) | rkey[k];
    if (key < lm) { lm = key; bm = lane() + 64 * k; }
  }
  return lm;
}
template <uint32_t KPL>
__device__ __attribute__((always_inline)) inline void a3x_drop(int32_t lbk[KPL], uint32_t b) {   // b's owner lane
  const bool own = lane() == (b & 63);
#pragma unroll
  for (uint32_t k = 0; k < KPL; ++k) lbk[k] = (own && k == (b >> 6)) ? INT32_MAX : lbk[k];   // a select per k: no
}                                                                    // indexed (scratch) store
// the row pass's keys (rank << 24 | rotated id; 0xFFFFFFFF: none) of the five found, for k_tick_post
__device__ __attribute__((always_inline)) inline void write_a3_keys(uint32_t* part, uint32_t i, uint32_t l,
                                                                    const unsigned long long m5[5]) {
  uint32_t o = 0xFFFFFFFFu;
#pragma unroll
  for (uint32_t k = 0; k < 5; ++k)
    if (l == k && m5[k] != ~0ull) o = (k << 24) | (uint32_t)(m5[k] & 0xFFFFFFu);
  if (l < 10) part[(size_t)i * 10 + l] = o;
}
// A wave per row.  The row's first step issues every load it needs at once (alive, the sweep front, the block
// bounds); each later step takes the block of smallest bound key and loads its bits, stamps and instants together
// (one memory round trip per block instead of three).  The wave's five smallest keys are formed once per step after a
// scan (none before the first) and serve the exit test and the answer: five 64-bit DPP minima, the kernel's largest VALU
// item (a converged start's five ancient candidates sit in the sweep front's block: one scan and one top-five per row,
// whose minima are also the answer).  KPL: block bounds per lane, the row's 1024-id blocks over 64 lanes (2 up to
// 128K ids, 8 up to 512K): the bound selection is a quarter of the instructions at 64K rows with KPL 2.
template <uint32_t KPL>
__device__ __attribute__((always_inline)) inline void a3x_narrow(const Dev& d, uint32_t* part, int32_t r, uint32_t i,
                                                                 uint32_t cur, bool alive) {
  const uint32_t l = lane(), C = d.C, NB = d.W >> 10;
  int32_t* lbrow = d.tlb + (size_t)i * NB;
  int32_t lbk[KPL];
#pragma unroll
  for (uint32_t k = 0; k < KPL; ++k) {
    const uint32_t b = l + 64 * k;
    lbk[k] = (b < NB && (b << 10) < C) ? lbrow[b] : INT32_MAX;        // INT32_MAX: nothing saturated (or no ids)
  }
  if (!alive) return;
  const uint8_t* srow = row_of(d, i);
  const uint32_t* brow = bits_of(d, i);
  const int32_t* trow = d.tst + (size_t)i * d.W;
  const uint32_t p = cur + 1 == C ? 0 : cur + 1;                     // the sweep front: rotated id 0
  uint32_t rkey[KPL];                                                // the block's smallest rotated id
#pragma unroll
  for (uint32_t k = 0; k < KPL; ++k) {
    const uint32_t lo = (l + 64 * k) << 10, hi = lo + 1023 < C - 1 ? lo + 1023 : C - 1;
    rkey[k] = (p >= lo && p <= hi) ? 0u : (lo > p ? lo - p : lo + C - p);
  }
  {                                                                  // 32-bit keys (above): the common case
    uint32_t top[5] = {~0u, ~0u, ~0u, ~0u, ~0u}, m5[5] = {~0u, ~0u, ~0u, ~0u, ~0u};
    int32_t base = 0;
    bool redo = false;
    for (;;) {
      unsigned long long fifth = ~0ull;                              // the fifth key as a 64-bit key
      if (m5[4] != ~0u) {
        const uint32_t h = m5[4] >> 24;
        if (h == 255u) { redo = true; break; }
        fifth = ((unsigned long long)((uint32_t)(base + (int32_t)h) ^ 0x80000000u) << 32) | (m5[4] & 0xFFFFFFu);
      }
      uint32_t bm = 0;
      const unsigned long long lm = a3x_lane_min<KPL>(lbk, rkey, bm);
      const unsigned long long m = wave_min_u64(lm);                // keys are distinct: rotated ids differ
      if (m == ~0ull || m >= fifth) break;
      const uint32_t b = rdl(bm, (int)__builtin_ctzll(__ballot(lm == m)));
      if (m5[0] == ~0u && top[0] == ~0u) base = (int32_t)((uint32_t)(m >> 32) ^ 0x80000000u);   // first scan: its bound
      a3x_drop<KPL>(lbk, b);
      A3Blk x;
      a3x_load(srow, brow, trow, b, x);
      int32_t smin = a3x_sat32(i, C, b, cur, base, x, top);
      smin = (int32_t)(wave_min((uint32_t)smin ^ 0x80000000u) ^ 0x80000000u);   // signed minimum
      if (l == 0) lbrow[b] = smin;                                   // exact now
      wave_top5_32(top, m5);
    }
    if (!redo && m5[4] != ~0u) {                                     // the last step's five: no scan after it
      uint32_t o = 0xFFFFFFFFu;
#pragma unroll
      for (uint32_t k = 0; k < 5; ++k) if (l == k) o = (k << 24) | (m5[k] & 0xFFFFFFu);
      if (l < 10) part[(size_t)i * 10 + l] = o;
      return;
    }
  }
  // 64-bit keys: instants 255 or more above the first bound among the five, or fewer than five saturated (then the
  // live bytes too).  The bounds the pass above made exact stay valid; every block is a candidate again.
#pragma unroll
  for (uint32_t k = 0; k < KPL; ++k) {
    const uint32_t b = l + 64 * k;
    lbk[k] = (b < NB && (b << 10) < C) ? lbrow[b] : INT32_MAX;
  }
  const int32_t E = epoch_base(r);
  unsigned long long top[5] = {~0ull, ~0ull, ~0ull, ~0ull, ~0ull};
  unsigned long long m5[5] = {~0ull, ~0ull, ~0ull, ~0ull, ~0ull};    // the wave's five smallest keys so far
  for (;;) {
    const unsigned long long fifth = m5[4];
    uint32_t bm = 0;
    const unsigned long long lm = a3x_lane_min<KPL>(lbk, rkey, bm);
    const unsigned long long m = wave_min_u64(lm);
    if (m == ~0ull || m >= fifth) break;
    const uint32_t b = rdl(bm, (int)__builtin_ctzll(__ballot(lm == m)));
    a3x_drop<KPL>(lbk, b);
    A3Blk x;
    a3x_load(srow, brow, trow, b, x);
    int32_t smin = a3x_sat(i, C, b, cur, x, top);
    smin = (int32_t)(wave_min((uint32_t)smin ^ 0x80000000u) ^ 0x80000000u);
    if (l == 0) lbrow[b] = smin;
    wave_top5(top, m5);
  }
  if (m5[4] == ~0ull) {                                              // fewer than five saturated: + the live bytes
    for (uint32_t b = 0; b < NB; ++b) a3x_block<false, true>(d, i, b, cur, E, srow, brow, trow, top);
    wave_top5(top, m5);
  }
  write_a3_keys(part, i, l, m5);
}
// One kernel per row width (the host picks by NB = W / 1024): each holds only its own path, so the 64K rows' KPL-2
// kernel is not sized for the wider paths' registers (74 VGPRs, 6 waves per SIMD, instead of 105 and 4): beside the
// fold it then takes more of each CU, and the round is 3 % shorter (`profiles/r06t_ab_a3_split.txt`).
template <uint32_t KPL>
__global__ __launch_bounds__(256) void k_a3_exact(Dev d, uint32_t* part, int32_t r) {
  const uint32_t i = d.lo + blockIdx.x * 4 + (threadIdx.x >> 6);
  if (i >= d.hi) return;
  const uint32_t cur = d.a3cur[i];
  const bool alive = d.alive[i] != 0;
  if constexpr (KPL != 0) {
    a3x_narrow<KPL>(d, part, r, i, cur, alive);
  } else {
    if (!alive) return;                                              // wider rows: one pass over everything
    const uint32_t NB = d.W >> 10;
    unsigned long long top[5] = {~0ull, ~0ull, ~0ull, ~0ull, ~0ull};
    const int32_t E = epoch_base(r);
    for (uint32_t b = 0; b < NB; ++b) a3x_block<true, true>(d, i, b, cur, E, row_of(d, i), bits_of(d, i), d.tst + (size_t)i * d.W, top);
    unsigned long long m5[5];
    wave_top5(top, m5);
    write_a3_keys(part, i, lane(), m5);
  }
}
__host__ __device__ inline uint32_t a3_kpl(uint32_t W) {               // 0: the wide path
  const uint32_t NB = W >> 10;
  return NB <= 64 * 2 ? 2u : NB <= 64 * A3X_KPL ? A3X_KPL : 0u;
}

// ---- lifecycle: API start/stop in call order, then churn (src/lib.rs:136-183) ------------------
// kind: EV_START, EV_STOP, or EV_RESTART (node = the instance's fresh address, src = its old one; the
// map was moved by k_row_pack / k_row_unpack just before, so here it is a start at the new address)
enum : uint32_t { EV_START = 0, EV_STOP = 1, EV_RESTART = 2 };
struct Event { uint32_t node, kind, src, pad; };
__global__ void k_events(Dev d, const Event* ev, uint32_t nev, int32_t r) {
  if (threadIdx.x || blockIdx.x) return;
  for (uint32_t k = 0; k < nev; ++k) {
    const uint32_t i = ev[k].node;
    if (ev[k].kind == EV_STOP) { if (d.alive[i]) node_stop(d, i); }
    else if (!d.alive[i]) node_start(d, i, r);
  }
}

// ---- a restart's map (kb_sim_restart_node): Kaboodle::start on a stopped instance binds a fresh address
// (src/kaboodle.rs:138-152) while its known_peers map persists (src/lib.rs:104, 167-170).  The old row is
// packed into one u32 buffer (every row table of the node: stamps, member bits, checkpoints, suspect slots,
// freshness log, latency column, plus the event observer's snapshot), moved to the shard holding the new
// row (an all-to-all-v with one non-empty pair; unsharded: in place) and unpacked there.
struct RowPack { uint32_t hdr, fstart, susp, segp, flog, bits, snap, stamp, lat, tst, words; };
enum { RP_N, RP_FP, RP_DIRTY, RP_FLOGN, RP_WATCHED, RP_WFP, RP_SD0, RP_SD1, RP_HDR = 16 };
__host__ __device__ inline RowPack row_pack_layout(uint32_t W, uint32_t NWR, bool lat, bool tst) {
  RowPack L;
  L.hdr = 0; L.fstart = RP_HDR; L.susp = L.fstart + 16; L.segp = L.susp + SLOTS * 4; L.flog = L.segp + 2 * NSEG;
  L.bits = L.flog + LOGCAP; L.snap = L.bits + NWR; L.stamp = L.snap + NWR; L.lat = L.stamp + W / 4;
  L.tst = L.lat + (lat ? W / 2 : 0);
  L.words = L.tst + (tst ? W : 0);
  return L;
}
__global__ __launch_bounds__(256) void k_row_pack(Dev d, uint32_t i, uint32_t* __restrict__ out, RowPack L,
                                                  const uint32_t* __restrict__ snap, uint32_t wfp) {
  const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x, T = gridDim.x * blockDim.x;
  if (t == 0) {
    const unsigned long long sd = d.sdirty[i];
    out[RP_N] = d.n[i]; out[RP_FP] = d.fp[i]; out[RP_DIRTY] = d.dirty[i]; out[RP_FLOGN] = d.flog_n[i];
    out[RP_WATCHED] = snap != nullptr; out[RP_WFP] = wfp; out[RP_SD0] = (uint32_t)sd; out[RP_SD1] = (uint32_t)(sd >> 32);
  }
  if (t < 16) out[L.fstart + t] = d.fstart[(size_t)i * 16 + t];
  if (t < SLOTS * 4) out[L.susp + t] = reinterpret_cast<const uint32_t*>(d.susp + (size_t)i * SLOTS)[t];
  if (t < 2 * NSEG) out[L.segp + t] = reinterpret_cast<const uint32_t*>(d.segp + (size_t)i * NSEG)[t];
  for (uint32_t k = t; k < LOGCAP; k += T) out[L.flog + k] = d.flog[(size_t)i * LOGCAP + k];
  const uint32_t* b = bits_of(d, i);
  for (uint32_t k = t; k < d.NWR; k += T) { out[L.bits + k] = b[k]; out[L.snap + k] = snap ? snap[k] : 0u; }
  const uint32_t* st = reinterpret_cast<const uint32_t*>(row_of(d, i));
  for (uint32_t k = t; k < d.W / 4; k += T) out[L.stamp + k] = st[k];
  if (d.lat)
    for (uint32_t k = t; k < d.W / 2; k += T) out[L.lat + k] = (uint32_t)*lat_at(d, i, 2 * k) | ((uint32_t)*lat_at(d, i, 2 * k + 1) << 16);
  if (d.tst)
    for (uint32_t k = t; k < d.W; k += T) out[L.tst + k] = (uint32_t)d.tst[(size_t)i * d.W + k];
}
__global__ __launch_bounds__(256) void k_row_unpack(Dev d, uint32_t i, const uint32_t* __restrict__ in, RowPack L,
                                                    uint32_t* __restrict__ snap) {
  const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x, T = gridDim.x * blockDim.x;
  if (t == 0) {
    d.n[i] = in[RP_N]; d.fp[i] = in[RP_FP]; d.dirty[i] = (uint8_t)in[RP_DIRTY]; d.flog_n[i] = in[RP_FLOGN];
    d.sdirty[i] = (unsigned long long)in[RP_SD0] | ((unsigned long long)in[RP_SD1] << 32);
  }
  if (t < 16) d.fstart[(size_t)i * 16 + t] = in[L.fstart + t];
  if (t < SLOTS * 4) reinterpret_cast<uint32_t*>(d.susp + (size_t)i * SLOTS)[t] = in[L.susp + t];
  if (t < 2 * NSEG) reinterpret_cast<uint32_t*>(d.segp + (size_t)i * NSEG)[t] = in[L.segp + t];
  for (uint32_t k = t; k < LOGCAP; k += T) d.flog[(size_t)i * LOGCAP + k] = in[L.flog + k];
  uint32_t* b = bits_of(d, i);
  for (uint32_t k = t; k < d.NWR; k += T) { b[k] = in[L.bits + k]; if (snap) snap[k] = in[L.snap + k]; }
  uint32_t* st = reinterpret_cast<uint32_t*>(row_of(d, i));
  for (uint32_t k = t; k < d.W / 4; k += T) st[k] = in[L.stamp + k];
  if (d.lat)
    for (uint32_t k = t; k < d.W / 2; k += T) {
      const uint32_t v = in[L.lat + k];
      *lat_at(d, i, 2 * k) = (uint16_t)v; *lat_at(d, i, 2 * k + 1) = (uint16_t)(v >> 16);
    }
  if (d.tst) {
    for (uint32_t k = t; k < d.W; k += T) d.tst[(size_t)i * d.W + k] = (int32_t)in[L.tst + k];
    for (uint32_t k = t; k < d.W >> 10; k += T) d.tlb[(size_t)i * (d.W >> 10) + k] = INT32_MIN;   // rescan the moved row
  }
}
__global__ void k_churn_leave(Dev d, int32_t r) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  unsigned long long left = 0;
  if (i < d.C && d.alive[i] && d.start_round[i] != r &&
      philox(i, (uint32_t)r, (uint32_t)P_CHURN << 24, 0, d.k0, d.k1).x < d.churn_thr) { node_stop(d, i); left = 1; }
  const unsigned long long t = block_sum(left);
  if (threadIdx.x == 0 && t) atomicAdd(&d.ctr[C_LEAVES], (uint32_t)t);
}
// churn joins take fresh ids in order: an id some instance bound (started through the API, a restart's new
// address) or given an identity is skipped.  The round's few dozen joins run in one thread.
__global__ void k_churn_join(Dev d, int32_t r) {
  // one wave: the fresh ids (never bound, no identity set: the oracle's serial walk) are found 64 at a time by
  // a ballot and started in parallel, in id order, as many as peers left
  if (blockIdx.x || threadIdx.x >= 64) return;
  const uint32_t l = threadIdx.x, leaves = d.ctr[C_LEAVES];
  uint32_t nf = d.ctr[C_NEXTFREE], joins = 0;
  while (joins < leaves && nf < d.C) {
    const uint32_t j = nf + l, need = leaves - joins;
    const bool fresh = j < d.C && d.start_round[j] == NONE_ROUND && !d.idset[j];
    const unsigned long long fm = __ballot(fresh);
    const uint32_t rank = __popcll(fm & ((1ull << l) - 1ull)), nfresh = __popcll(fm);
    if (fresh && rank < need) node_start(d, j, r);
    if (nfresh >= need) {                                   // the need-th fresh id was the last one started
      nf += (uint32_t)__ffsll((long long)__ballot(fresh && rank == need - 1));   // one past it
      joins = leaves;
    } else {
      nf += 64;
      joins += nfresh;
    }
  }
  if (l == 0) {
    d.ctr[C_NEXTFREE] = nf < d.C ? nf : d.C; d.ctr[C_LEAVES] = 0;
    if (d.lo == 0) { d.stats[S_CLEAVE] += leaves; d.stats[S_CJOIN] += joins; }   // replicated: counted once
  }
}

// ---- running set bitset + count, and its fingerprint (what a converged node reports) -----------
__global__ void k_alive_bits(Dev d) {
  const uint32_t w = blockIdx.x * blockDim.x + threadIdx.x;
  unsigned long long cnt = 0;
  if (w < d.NWR) {
    uint32_t x = 0;
    for (uint32_t t = 0; t < 32; ++t) { const uint32_t j = w * 32 + t; if (j < d.C && d.alive[j]) x |= 1u << t; }
    d.abits[w] = x;
    cnt = __popc(x);
  }
  const unsigned long long t = block_sum(cnt);
  if (threadIdx.x == 0 && t) atomicAdd(&d.ctr[C_ALIVE], (uint32_t)t);
}
// The running set's fingerprint in two launches: TRUEFP_G workgroups fold consecutive word ranges of
// `abits` into ordered partials (thread folds, then a tree combine in LDS), one wave combines them.
constexpr uint32_t TRUEFP_G = 64;
__global__ __launch_bounds__(256) void k_truefp_part(Dev d, uint2* part) {
  __shared__ uint32_t ztab[ZT * 128];
  __shared__ uint32_t sraw[256], scnt[256];
  load_ztab(d, ztab);
  const uint32_t T = blockDim.x, t = threadIdx.x, g = blockIdx.x;
  const uint32_t wpg = (d.NWR + TRUEFP_G - 1) / TRUEFP_G, wg0 = g * wpg;
  const uint32_t wg1 = wg0 + wpg < d.NWR ? wg0 + wpg : d.NWR;
  uint32_t raw = 0, cnt = 0;
  const uint32_t per = wg1 > wg0 ? (wg1 - wg0 + T - 1) / T : 0;
  for (uint32_t w = wg0 + t * per; w < wg0 + (t + 1) * per && w < wg1; ++w) {
    uint32_t x = d.abits[w];
    if (!x) continue;
    if (d.uniform) {
      for (int h = 0; h < 4; ++h) fold_half(d, ztab, 4 * w + h, (x >> (8 * h)) & 0xFFu, raw, cnt);
    } else {
      while (x) { const uint32_t j = w * 32 + (__ffs(x) - 1); x &= x - 1; raw = multmodp(d.segmul[j], raw) ^ d.cseg[j]; cnt += d.seglen[j]; }
    }
  }
  sraw[t] = raw; scnt[t] = cnt;
  __syncthreads();
  for (uint32_t s = 1; s < T; s <<= 1) {
    uint32_t nr = 0, nc = 0;
    const bool w = (t % (2 * s) == 0) && t + s < T;
    if (w) { nr = comb(d, sraw[t], sraw[t + s], scnt[t + s]); nc = scnt[t] + scnt[t + s]; }
    __syncthreads();
    if (w) { sraw[t] = nr; scnt[t] = nc; }
    __syncthreads();
  }
  if (t == 0) part[g] = make_uint2(sraw[0], scnt[0]);
}
__global__ __launch_bounds__(64) void k_truefp_fin(Dev d, const uint2* part) {
  const uint2 p = part[lane()];                       // TRUEFP_G == 64: one partial per lane
  uint32_t raw = p.x, cnt = p.y;
  wave_combine(d, raw, cnt);
  if (lane() == 0) d.truefp[0] = finish_fp(d, raw, cnt);
}
static_assert(TRUEFP_G == 64, "k_truefp_fin combines one partial per lane");

// round start of every node's freshness log window
__global__ void k_log_mark(Dev d, int32_t r) {
  const uint32_t i = d.lo + blockIdx.x * blockDim.x + threadIdx.x;
  if (blockIdx.x == 0 && threadIdx.x == 0) d.ctr[C_ROUND] = (uint32_t)r;   // for the graph-replayed waves
  if (i < d.hi) d.fstart[(size_t)i * 16 + ((uint32_t)r & 15u)] = d.flog_n[i];
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
  const uint32_t* fnamed;  // track_latency: bitset of the peers the Failed list names (k_lat_mark)
};

// ---- PeerInfo.latency upkeep for the Failed removals ---------------------------
// The row pass does not write the (peer-major) latency table when Failed removes a peer: a round
// removes tens of millions of (row, peer) entries in the sim_sender workload, nearly all of them
// never measured.  k_lat_sweep instead reads each named peer's column once, right after the row pass
// and before anything can re-insert and measure, and resets the entries whose member bit is now
// clear.  The one re-insertion inside the row pass itself (a Join of a peer the same round's Failed
// list names) resets its entry there, using the fnamed bitset.
__global__ void k_lat_mark(const BCast* bf, uint32_t nf, uint32_t* fnamed) {
  const uint32_t f = blockIdx.x * blockDim.x + threadIdx.x;
  if (f < nf) atomicOr(&fnamed[bf[f].peer >> 5], 1u << (bf[f].peer & 31));
}
__global__ __launch_bounds__(256) void k_lat_sweep(Dev d, const BCast* bf, const uint32_t* gid, uint32_t nf,
                                                   uint32_t* fnamed) {
  const uint32_t R = d.hi - d.lo, RS = lat_stride(R);
  for (uint32_t f = blockIdx.y; f < nf; f += gridDim.y) {
    if (gid[f] != f) continue;                        // first entry naming the peer only
    const uint32_t p = bf[f].peer;
    if (blockIdx.x == 0 && threadIdx.x == 0) atomicAnd(&fnamed[p >> 5], ~(1u << (p & 31)));
    uint4* col = reinterpret_cast<uint4*>(d.lat + (size_t)p * RS);      // 8 rows per 16-byte load
    for (uint32_t k = blockIdx.x * blockDim.x + threadIdx.x; k < RS / 8; k += gridDim.x * blockDim.x) {
      const uint4 v = col[k];
      if ((v.x & v.y & v.z & v.w) == 0xFFFFFFFFu) continue;            // all eight None (the common case)
      uint16_t* e = reinterpret_cast<uint16_t*>(col + k);
      for (uint32_t q = 0; q < 8; ++q) {
        const uint32_t row = 8 * k + q;
        if (row < R && e[q] != LAT_NONE && !is_mem(d, d.lo + row, p)) e[q] = LAT_NONE;
      }
    }
  }
}

// Broadcast loss: entry e of the round's Failed (lst 0) / Join (lst 1) list reaches
// receiver i unless word e % 4 of philox(i, r, P_BLOSS << 24 | lst << 23 | e / 4, 0) < loss_thr.  A wave
// handling entries [c, c + 64) in lane order takes its draws from one Philox call per lane per 256
// entries (BLossQuad: lane l holds the words of group c256 / 4 + l) and a cross-lane read.
struct BLossQuad { U4 w; };
__device__ inline BLossQuad bloss_quad(const Dev& d, uint32_t recv, int32_t r, uint32_t lst, uint32_t c256) {
  BLossQuad q;
  q.w = (faults(d, r) && d.loss_thr)
            ? philox(recv, (uint32_t)r, ((uint32_t)P_BLOSS << 24) | (lst << 23) | ((c256 >> 2) + lane()), 0, d.k0, d.k1)
            : U4{0xFFFFFFFFu, 0xFFFFFFFFu, 0xFFFFFFFFu, 0xFFFFFFFFu};
  return q;
}
// lost? for entry c + lane() (c a multiple of 64, q taken at c & ~255), sent by `sender`
__device__ __attribute__((always_inline)) inline bool bcast_lost(const Dev& d, uint32_t recv, uint32_t sender, int32_t r,
                                                                 const BLossQuad& q, uint32_t c) {
  const int src = (int)(((c & 255u) >> 2) + (lane() >> 2));
  const uint32_t wx = bcast(q.w.x, src), wy = bcast(q.w.y, src), wz = bcast(q.w.z, src), ww = bcast(q.w.w, src);
  const uint32_t k = lane() & 3u;
  const uint32_t u = k == 0 ? wx : (k == 1 ? wy : (k == 2 ? wz : ww));
  if (part_blocks(d, r, sender, recv)) return true;
  return faults(d, r) && d.loss_thr && u < d.loss_thr;
}

// Per-list facts about the Failed broadcasts (identical for every receiver).
__global__ void k_bfail_prep(const BCast* bf, uint32_t nf, uint32_t* gid, uint8_t* dep, uint32_t* paths) {
  const uint32_t q = blockIdx.x * blockDim.x + threadIdx.x;
  if (q >= nf) return;
  if (q == 0) atomicOr(paths, PATH_BFAIL_PREP_HBM);
  const uint32_t p = bf[q].peer, sn = bf[q].sender;
  uint32_t g = q; uint8_t dp = 0;
  for (uint32_t k = 0; k < q; ++k) {
    const uint32_t pk = bf[k].peer;
    if (pk == p && g == q) g = k;
    if (pk == sn) dp = 1;
  }
  gid[q] = g; dep[q] = dp;
}

// Same facts for lists up to BFAIL_LDS_MAX entries: one workgroup, LDS hash of peer -> first index naming it
// (128 KB of LDS; wide meshes' Failed lists run to thousands: ≈ 7 000 at 372K peers, where the quadratic
// per-entry scan above took 0.8 ms a round).
constexpr uint32_t BFAIL_LDS_MAX = 8192;
__global__ __launch_bounds__(1024) void k_bfail_prep_lds(const BCast* bf, uint32_t nf, uint32_t* gid, uint8_t* dep) {
  constexpr uint32_t HS = 2 * BFAIL_LDS_MAX, EMPTY = 0xFFFFFFFFu;
  __shared__ uint32_t hk[HS], hv[HS];
  for (uint32_t t = threadIdx.x; t < HS; t += blockDim.x) { hk[t] = EMPTY; hv[t] = EMPTY; }
  __syncthreads();
  auto slot0 = [](uint32_t x) { return (x * 0x9E3779B1u) >> 18; };   // 14 bits
  for (uint32_t e = threadIdx.x; e < nf; e += blockDim.x) {
    const uint32_t key = bf[e].peer;
    uint32_t h = slot0(key);
    while (true) {
      const uint32_t prev = atomicCAS(&hk[h], EMPTY, key);
      if (prev == EMPTY || prev == key) { atomicMin(&hv[h], e); break; }
      h = (h + 1) & (HS - 1);
    }
  }
  __syncthreads();
  auto first = [&](uint32_t x) __attribute__((always_inline)) -> uint32_t {
    uint32_t h = slot0(x);
    while (hk[h] != EMPTY) { if (hk[h] == x) return hv[h]; h = (h + 1) & (HS - 1); }
    return EMPTY;
  };
  for (uint32_t e = threadIdx.x; e < nf; e += blockDim.x) {
    gid[e] = first(bf[e].peer);
    const uint32_t f = first(bf[e].sender);
    dep[e] = f != EMPTY && f < e;
  }
}

// ================================================================================================
// THE ROW PASS: one wave per node, the node's member bitset staged in LDS once for the whole pass.
//  (1) broadcast phase — Failed then Join deliveries of round r-1's broadcasts (src/kaboodle.rs:256-311);
//  (2) ping_random_peer's candidate scan (A3, :655-703): the five oldest Known peers by (stamp, address
//      rotated to start right after self), read in address order from self+1 with coalesced 16-byte
//      stamp loads, 1024 ids per wave step, stopping as soon as five "ancient" (minimum) stamps have
//      been seen in that order — later ids can then never rank among the five;
//  (3) write-back of the changed bitset segments.
// Persistent waves: each workgroup first stages the broadcast lists in LDS (shared by all its nodes:
// Failed as {sender | bseq << 23 | dep << 31, peer}, Join as {sender | bseq << 23}).  Lists longer than
// the LDS budget, or rows wider than PB_LDS_W, are read from HBM instead (LDSB = false).
// ================================================================================================
constexpr uint32_t PB_LDS_W = 524288;
constexpr uint32_t PB_FMAX = 2048, PB_JMAX = 1024;
constexpr uint32_t RP_WAVES = 8;                 // waves per row-pass workgroup (they share the lists)
constexpr uint32_t RP_LDS_BYTES = 81920 - 1024;  // dynamic LDS per row-pass workgroup: two (+ static) fit a CU
struct RowOut { uint32_t* part; };   // [C][10]: the five smallest keys ascending, then 0xFFFFFFFF x 5

// A3 over the row of node i (members from B: LDS or HBM): the five smallest keys (stamp << 24 | rot),
// ascending, in every lane; rot = address rotated to start right after `cur`, the node's sweep front
// (DESIGN.md §2.6).  Returns the stamp bytes read.
template <bool LDSB>
__device__ __attribute__((always_inline)) inline uint32_t a3_scan(const Dev& d, uint32_t i, uint32_t cur, const uint8_t* rw,
                                                                  const uint32_t* B, uint32_t (&out)[5], uint3& a3c) {
  const uint32_t l = lane(), C = d.C, W = d.W;
  const uint32_t p = (cur + 1 == C) ? 0 : cur + 1;
  const uint32_t a0 = p & ~15u;
  uint32_t K[5] = {0xFFFFFFFFu, 0xFFFFFFFFu, 0xFFFFFFFFu, 0xFFFFFFFFu, 0xFFFFFFFFu};
  uint32_t anc = 0, nbytes = 0;                   // ancient candidates in the scanned address-order prefix
  bool fast = false;                              // out[] already holds the five (first-five-ancient case)
  // chunk order: ids [a0, W) then [0, a0), 1024 ids per chunk; the first step loads one chunk (it
  // usually decides), later steps A3_U chunks at once (rows with few ancient stamps: recent joiners)
  constexpr int A3_U = 4;
  uint32_t next = a0;
  bool wrapped = false, more = true;
  for (int step = 0; more; ++step) {
    const int nu = step == 0 ? 1 : A3_U;
    uint32_t base[A3_U];
    bool wr[A3_U], ok[A3_U];
#pragma unroll
    for (int u = 0; u < A3_U; ++u) {
      ok[u] = u < nu && more;
      base[u] = next; wr[u] = wrapped;
      if (ok[u]) {
        next += 1024;
        if (!wrapped && next >= W) { wrapped = true; next = 0; }
        if (wrapped && next >= a0) more = false;
      }
    }
    uint4 v[A3_U];
    uint32_t mbw[A3_U];
#pragma unroll
    for (int u = 0; u < A3_U; ++u) {                // every load of the step in flight together
      const uint32_t j = base[u] + 16 * l;
      const bool inr = ok[u] && (wr[u] ? j < a0 : j < W);
      v[u] = make_uint4(0, 0, 0, 0);
      mbw[u] = 0;
      a3c.z += ok[u] ? 1u : 0u;
      if (inr) {
        v[u] = *reinterpret_cast<const uint4*>(rw + j);
        mbw[u] = LDSB ? B[j >> 5] : __hip_atomic_load(&B[j >> 5], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        nbytes += 16;
      }
    }
    bool done = false;
#pragma unroll
    for (int u = 0; u < A3_U; ++u) {
      if (!ok[u] || done) continue;                 // wave-uniform
      const uint32_t j = base[u] + 16 * l;
      const bool inr = wr[u] ? j < a0 : j < W;
      const uint32_t mb = inr ? (mbw[u] >> (j & 16)) & 0xFFFFu : 0u;
      const uint4 x = v[u];
      uint32_t cm = (nzmask4(x.x & 0xFEFEFEFEu) | (nzmask4(x.y & 0xFEFEFEFEu) << 4) | (nzmask4(x.z & 0xFEFEFEFEu) << 8) |
                     (nzmask4(x.w & 0xFEFEFEFEu) << 12)) & mb;               // Known && member
      if (i >= j && i < j + 16) cm &= ~(1u << (i - j));                      // != self (:571-577)
      uint32_t am = cm & (eqmask4(x.x, ST_ANCIENT) | (eqmask4(x.y, ST_ANCIENT) << 4) | (eqmask4(x.z, ST_ANCIENT) << 8) |
                          (eqmask4(x.w, ST_ANCIENT) << 12));
      if (!wr[u] && j < p) am &= p - j >= 16 ? 0u : ~((1u << (p - j)) - 1u);   // [a0, p) comes last in order
      const uint32_t pc = __popc(am), ta = wave_sum(pc);
      if (u == 0 && anc == 0 && ta >= (uint32_t)NUM_CANDIDATES) {   // (first chunk of a step)
        // (the usual case) no ancient candidate before this chunk and at least five in it: every earlier
        // key is newer, so the five oldest are this chunk's first five ancient members in address order
        // (= rotated order inside a chunk) — taken by a prefix count, no per-lane top-5 and no merge
        const uint32_t pre = wave_excl(pc);
#pragma unroll
        for (uint32_t q = 0; q < (uint32_t)NUM_CANDIDATES; ++q) {
          const bool owns = pre <= q && q < pre + pc;    // the lane holding the q-th ancient member
          const uint32_t jj = j + select_in_word(am, owns ? q - pre : 0u);
          const uint32_t key = ((uint32_t)ST_ANCIENT << 24) | (jj >= p ? jj - p : jj + C - p);
          out[q] = (uint32_t)__builtin_amdgcn_readlane((int)key, __ffsll((long long)__ballot(owns)) - 1);
        }
        anc = ta;
        fast = true;
        done = true;
        continue;
      }
      anc += ta;
      for (uint32_t m = cm; m; m &= m - 1) {
        const uint32_t t = __ffs(m) - 1, jj = j + t;
        const uint32_t word = (t & 8) ? ((t & 4) ? x.w : x.z) : ((t & 4) ? x.y : x.x);
        const uint32_t key = (((word >> (8 * (t & 3))) & 0xFFu) << 24) | (jj >= p ? jj - p : jj + C - p);
        if (key < K[4]) top5_insert(K, key);
      }
      if (anc >= (uint32_t)NUM_CANDIDATES) done = true;   // nothing later in address order can rank
    }
    if (done || (d.dev & 1)) break;               // dev 1: first chunk only (timing experiments)
  }
  a3c.x += 1; a3c.y += (next != a0 + 1024 || wrapped) ? 1u : 0u;   // scan depth (kb_sim_debug_counters)
  if (fast) return wave_sum(nbytes);
#pragma unroll
  for (int q = 0; q < 5; ++q) {                     // merge the lanes' lists (keys are distinct)
    const uint32_t mn = wave_min(K[0]);
    out[q] = mn;
    if (K[0] == mn && mn != 0xFFFFFFFFu) { K[0] = K[1]; K[1] = K[2]; K[2] = K[3]; K[3] = K[4]; K[4] = 0xFFFFFFFFu; }
  }
  return wave_sum(nbytes);
}

// LDSB: the row's bitset staged in LDS; LL: both broadcast lists staged in LDS (every list read is then an
// LDS read: a runtime choice between LDS and HBM made the compiler read the Failed entries through flat
// pointers, whose wait covered the HBM counter too and cost the loop one L2 round trip per 64 entries)
constexpr uint32_t KB_RP_WPE = 4;           // minimum waves per SIMD the row pass is compiled for (register budget 512 / KB_RP_WPE)
template <bool LDSB, bool LL>
__global__ __launch_bounds__(512) __attribute__((amdgpu_waves_per_eu(KB_RP_WPE, 8))) void k_rowpass(Dev d, PhaseB pb, RowOut ro, int32_t r) {
  extern __shared__ uint32_t pb_dyn[];
  const uint32_t wpb = blockDim.x >> 6;
  const uint32_t wv = threadIdx.x >> 6;
  const uint32_t l = lane();
  uint2* FL = reinterpret_cast<uint2*>(pb_dyn + (LDSB ? (size_t)wpb * d.NWR : 0));   // [nf] when LL
  uint32_t* JL = reinterpret_cast<uint32_t*>(FL + (LL ? pb.nf : 0));                // [nj] when LL
  if (LL) {
    for (uint32_t e = threadIdx.x; e < pb.nf; e += blockDim.x) {
      const BCast b = pb.bfail[e];
      FL[e] = make_uint2(b.sender | (b.bseq << 23) | ((uint32_t)pb.dep[e] << 31), b.peer);
    }
    for (uint32_t e = threadIdx.x; e < pb.nj; e += blockDim.x) JL[e] = pb.bjoin[e].sender | (pb.bjoin[e].bseq << 23);
  }
  __syncthreads();
  auto fail_at = [&](uint32_t e, uint32_t& dep) __attribute__((always_inline)) -> BCast {
    if (LL) {
      const uint2 x = FL[e];
      dep = x.x >> 31;
      return BCast{x.x & 0x7FFFFFu, x.y, (x.x >> 23) & 0xFFu, 0};
    }
    dep = pb.dep[e];
    return pb.bfail[e];
  };
  auto join_at = [&](uint32_t e) __attribute__((always_inline)) -> BCast {
    if (LL) { const uint32_t x = JL[e]; return BCast{x & 0x7FFFFFu, x & 0x7FFFFFu, x >> 23, 0}; }
    return pb.bjoin[e];
  };
  const bool honour = d.failed_mode == KB_FAILED_SIM_SENDER;
  const uint8_t now = enc(r, r);
  // counters stay in registers for the whole persistent loop: one atomic per wave at the end (same-
  // address atomics from every node would serialise in L2 and stall the waves that wait on them)
  unsigned long long w_lost = 0, w_removed = 0, w_resp = 0, w_nodes = 0, w_bytes = 0;
  uint3 a3c = make_uint3(0, 0, 0);
  // phase timing (a build with -DKB_RP_PROF, run with KB_DEBUG_WAVES=1 KB_DEV=2048): wall-clock ticks per
  // phase summed in registers, added once per workgroup at the end; compiled out otherwise (its registers
  // would cost the pass spills)
#ifdef KB_RP_PROF
  const bool prof = (d.dev & 2048) != 0;
  uint64_t tph[5] = {0, 0, 0, 0, 0}, tmark = 0;
  auto tick = [&](int k) __attribute__((always_inline)) {
    if (prof) { const uint64_t t = wall_clock64(); if (k >= 0) tph[k] += t - tmark; tmark = t; }
  };
#else
  auto tick = [](int) __attribute__((always_inline)) {};
#endif
  for (uint32_t i = d.lo + blockIdx.x * wpb + wv; i < d.hi; i += gridDim.x * wpb) {
    tick(-1);
    // the node's header loads are issued together, ahead of the bitset staging (one memory round trip
    // for all of them instead of one per dependent use)
    const uint8_t alive = d.alive[i];
    const int32_t sr = d.start_round[i];
    const uint32_t n_in = d.n[i], fn_in = d.flog_n[i], cur = d.a3cur[i];
    const Susp sl_in = l < SLOTS ? d.susp[(size_t)i * SLOTS + l] : Susp{0, 0, 0, 0};
    if (!alive) {
      if (l == 0) { pb.nresp[i] = 0; pb.paysum[i] = 0; }
      continue;
    }
    uint8_t* rw = row_of(d, i);
    uint32_t* gB = bits_of(d, i);
    uint32_t* B = LDSB ? pb_dyn + (size_t)wv * d.NWR : gB;
    if (LDSB) { stage16(reinterpret_cast<uint4*>(B), reinterpret_cast<const uint4*>(gB), d.NWR / 4, l, 64); w_bytes += 4ull * d.NWR; }
    tick(0);
    unsigned long long segs = 0;
    uint32_t nresp = 0;
    if (sr < r) {                                     // ---- (1) broadcast phase ----
      // the node's suspects as wave-uniform values (most rows have none): is_susp is a few scalar
      // compares per lane instead of eight LDS reads
      const uint32_t spv = l < SLOTS && sl_in.kind ? sl_in.peer : 0xFFFFFFFFu;
      const unsigned long long spm = __ballot(spv != 0xFFFFFFFFu);
      uint32_t sp[SLOTS];
#pragma unroll
      for (int k = 0; k < SLOTS; ++k) sp[k] = __builtin_amdgcn_readlane(spv, k);
      wait_lds();
      __builtin_amdgcn_wave_barrier();
      auto mem = [&](uint32_t x) __attribute__((always_inline)) -> bool {
        const uint32_t w = LDSB ? B[x >> 5] : __hip_atomic_load(&B[x >> 5], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        return (w >> (x & 31)) & 1u;
      };
      auto is_susp = [&](uint32_t x) __attribute__((always_inline)) {
        bool f = false;
        if (spm) {
#pragma unroll
          for (int k = 0; k < SLOTS; ++k) f |= sp[k] == x;
        }
        return f;
      };
      uint32_t n = n_in;
      const uint32_t n0 = n;
      uint32_t fn = fn_in;
      uint32_t lost_cnt = 0, removed_cnt = 0;
      // ---- Failed(p) group (src/kaboodle.rs:268-283) ----
      // In-order semantics, 64 entries at a time.  An entry acts iff it is delivered, names neither the
      // receiver nor comes from it, and its sender is still a member when it is reached.  Membership at
      // the chunk start is in B (earlier chunks applied); inside the chunk only an entry whose sender is
      // named by an earlier entry (dep) can change its mind: those are resolved in lane order with one
      // ballot each (killed iff an earlier acting lane of the chunk names its sender).  The acting
      // entries are then applied together: the atomic's return says whether the peer was still present.
      BLossQuad lq;
      // the list entries of the next chunk are loaded one iteration ahead: they do not depend on the
      // removals of this chunk, only the membership tests do
      const uint32_t nfl = (d.dev & 2) ? 0u : pb.nf;   // dev 2: skip (timing experiments)
      uint32_t dep_nx = 0;
      BCast b_nx = l < nfl ? fail_at(l, dep_nx) : BCast{0xFFFFFFFFu, 0xFFFFFFFFu, 0, 0};
      for (uint32_t c = 0; c < nfl; c += 64) {
        const uint32_t e = c + l;
        const bool valid = e < pb.nf;
        const uint32_t dep = dep_nx;
        const BCast b = b_nx;
        dep_nx = 0;
        b_nx = e + 64 < nfl ? fail_at(e + 64, dep_nx) : BCast{0xFFFFFFFFu, 0xFFFFFFFFu, 0, 0};
        if ((c & 255u) == 0) lq = bloss_quad(d, i, r, 0, c);
        const bool lost = bcast_lost(d, i, b.sender, r, lq, c) && valid && b.sender != i;
        const bool base = valid && b.sender != i && !lost && b.peer != i && honour && mem(b.sender);
        unsigned long long actm = __ballot(base);
        unsigned long long depm = __ballot(base && dep);
        while (depm) {
          const uint32_t q = (uint32_t)(__ffsll((long long)depm) - 1);
          depm &= depm - 1;
          const uint32_t s_q = rdl(b.sender, q);
          const unsigned long long killers = __ballot(((actm >> l) & 1ull) && b.peer == s_q) & ((1ull << q) - 1ull);
          if (killers) actm &= ~(1ull << q);
        }
        lost_cnt += __popcll(__ballot(lost));
        if ((actm >> l) & 1ull) {
          const uint32_t m = 1u << (b.peer & 31);
          if (atomicAnd(&B[b.peer >> 5], ~m) & m) {
            removed_cnt++;
            if (is_susp(b.peer)) susp_clear(d, i, b.peer);
            segs |= seg_bit(d, b.peer);
          }
        }
        if (!LDSB) { __builtin_amdgcn_s_waitcnt(0); }
        __builtin_amdgcn_wave_barrier();
      }
      tick(1);
      removed_cnt = wave_sum(removed_cnt);
      n -= removed_cnt;
      if (!LDSB) { __builtin_amdgcn_s_waitcnt(0); }
      __builtin_amdgcn_wave_barrier();
      const uint32_t nbase = n;
      // ---- Join{addr} group (src/kaboodle.rs:284-304) ----
      uint32_t paysum = 0;
      BLossQuad jq;
      for (uint32_t c = 0; c < ((d.dev & 4) ? 0u : pb.nj); c += 64) {   // dev 4: skip (timing experiments)
        const uint32_t e = c + l;
        const bool valid = e < pb.nj;
        const BCast b = valid ? join_at(e) : BCast{0xFFFFFFFFu, 0, 0, 0};
        if ((c & 255u) == 0) jq = bloss_quad(d, i, r, 1, c);
        const bool lost = bcast_lost(d, i, b.sender, r, jq, c) && valid && b.sender != i;
        const bool deliver = valid && b.sender != i && !lost;
        const bool known = deliver && mem(b.sender);
        const unsigned long long newm = __ballot(deliver && !known);
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
        // every delivered Join stamps its sender Known(now) afresh: before the row pass no stamp of the
        // round's own instant exists except self's (a node broadcasts one Join per round), so each
        // delivery is a transition to Known(now) and is logged — no read of the old byte needed
        const bool logit = deliver;
        const unsigned long long lgm = __ballot(logit);
        if (logit) d.flog[(size_t)i * LOGCAP + ((fn + __popcll(lgm & ((1ull << l) - 1ull))) & (LOGCAP - 1))] = log_entry(b.sender, r);
        fn += __popcll(lgm);
        if (deliver) {
          if (known && is_susp(b.sender)) susp_clear(d, i, b.sender);
          rw[b.sender] = now;
          if (isnew) {
            atomicOr(&B[b.sender >> 5], 1u << (b.sender & 31)); segs |= seg_bit(d, b.sender);
            if (pb.fnamed && ((pb.fnamed[b.sender >> 5] >> (b.sender & 31)) & 1u)) lat_none(d, i, b.sender);
          }
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
      segs = (unsigned long long)wave_or((uint32_t)segs) | ((unsigned long long)wave_or((uint32_t)(segs >> 32)) << 32);
      if (l == 0) {
        d.n[i] = n;
        d.flog_n[i] = fn;
        mark(d, i, segs);
        if (n != n0) d.dirty[i] = 1;
        pb.nresp[i] = nresp; pb.paysum[i] = paysum; pb.nbase[i] = nbase;
      }
      w_lost += lost_cnt; w_removed += removed_cnt;
      // the Join stamps written above are read back by this wave's A3 loads
      if (!(d.dev & 8)) {                           // dev 8: skip (timing experiments)
        wave_mem_sync();
        __builtin_amdgcn_s_waitcnt(0);
      }
    } else if (l == 0) {                              // started this round: no deliveries yet
      pb.nresp[i] = 0; pb.paysum[i] = 0;
    }
    wait_lds();
    __builtin_amdgcn_wave_barrier();
    tick(2);
    // ---- (2) A3 candidates ----
    if (!d.tst) {                                     // KB_VARIANT_EXACT_LRU: k_a3_exact writes the keys
      uint32_t top[5];
      w_bytes += a3_scan<LDSB>(d, i, cur, rw, B, top, a3c);
      if (l < 10) ro.part[(size_t)i * 10 + l] = l < 5 ? (l == 0 ? top[0] : l == 1 ? top[1] : l == 2 ? top[2] : l == 3 ? top[3] : top[4]) : 0xFFFFFFFFu;
    }
    tick(3);
    // ---- (3) write back the changed segments of the bitset ----
    if (LDSB && segs) {
      const uint32_t wps4 = d.SEGW / 128;             // 16-byte words per segment
      const uint4* B4 = reinterpret_cast<const uint4*>(B);
      uint4* g4 = reinterpret_cast<uint4*>(gB);
      for (uint32_t w = l; w < d.NWR / 4; w += 64) if ((segs >> (w / wps4)) & 1ull) g4[w] = B4[w];
      w_bytes += (unsigned long long)__popcll(segs) * (d.SEGW / 8);
    }
    w_resp += nresp; w_nodes++;
    tick(4);
    wait_lds();                                       // LDS bitset is reused by the next node
    __builtin_amdgcn_wave_barrier();
  }
  // the counters are summed over the workgroup's waves in LDS and added once per workgroup (one atomic
  // per wave and counter on the same few addresses would serialise in the memory system)
#ifdef KB_RP_PROF
  if (prof) {
    __shared__ unsigned long long s_t[5];
    if (threadIdx.x < 5) s_t[threadIdx.x] = 0;
    __syncthreads();
    if (l == 0) for (int k = 0; k < 5; ++k) atomicAdd(&s_t[k], tph[k]);
    __syncthreads();
    const int ci[5] = {C_DBG_TSTART, C_DBG_TBASE, C_DBG_TINS, C_DBG_TNODE, C_DBG_TEND};
    if (threadIdx.x < 5) atomicAdd(&d.ctr[ci[threadIdx.x]], (uint32_t)(s_t[threadIdx.x] / 64));   // in 64-tick units
  }
#endif
  __shared__ unsigned long long s_cnt[RP_WAVES][7];
  if (l == 0) {
    s_cnt[wv][0] = w_lost; s_cnt[wv][1] = w_removed; s_cnt[wv][2] = w_resp; s_cnt[wv][3] = w_bytes;
    s_cnt[wv][4] = a3c.x; s_cnt[wv][5] = a3c.y; s_cnt[wv][6] = a3c.z;
    if (!LDSB && w_nodes && pb.nf) path_hit(d, PATH_PHASEB_HBM);   // the Failed group on the HBM bitset
  }
  __syncthreads();
  if (threadIdx.x < 7) {
    unsigned long long t = 0;
    for (uint32_t k = 0; k < wpb; ++k) t += s_cnt[k][threadIdx.x];
    const int idx[7] = {S_BDROP, S_RMFAILED, S_JRESP, S_ROWB, S_A3ROWS, S_A3DEEP, S_A3CHUNKS};
    if (t) slot_add(d, idx[threadIdx.x], t);
  }
}

// ---- SwimBroadcast::Probe (src/kaboodle.rs:305-331), after the Failed and Join groups: every running
// peer that receives probe e answers with ProbeResponse{identity} iff should_respond_to_broadcast holds
// for its map as it stands (its own Philox counter, bit 23).  Thread per local row; the
// (responder, probe) pairs that were not lost on the way back are listed for the host (few per round).
__global__ __launch_bounds__(256) void k_probe(Dev d, uint32_t np, int32_t r, uint2* out, uint32_t* cnt, uint32_t cap) {
  const uint32_t i = d.lo + blockIdx.x * blockDim.x + threadIdx.x;
  unsigned long long lost_in = 0, sent = 0, lost_out = 0;
  if (i < d.hi && d.alive[i] && d.start_round[i] < r) {
    const bool f = faults(d, r) && d.loss_thr;
    const uint32_t n = d.n[i];
    for (uint32_t e = 0; e < np; ++e) {
      if (f) {
        const U4 w = philox(i, (uint32_t)r, ((uint32_t)P_PROBE << 24) | (e >> 2), 0, d.k0, d.k1);
        const uint32_t u = (e & 3) == 0 ? w.x : (e & 3) == 1 ? w.y : (e & 3) == 2 ? w.z : w.w;
        if (u < d.loss_thr) { lost_in++; continue; }
      }
      const int64_t o = (int64_t)n - 2;
      bool resp = o <= 0;
      if (!resp) {
        int64_t pct = 100 - o * o; if (pct < 1) pct = 1;
        const uint32_t u = philox(i, (uint32_t)r, ((uint32_t)P_RESPOND << 24) | (1u << 23) | e, 0, d.k0, d.k1).x;
        resp = (int64_t)mulhi(u, 100) < pct;
      }
      if (!resp) continue;
      sent++;
      if (f && philox(i, (uint32_t)r, ((uint32_t)P_PROBE << 24) | (1u << 23) | e, 1, d.k0, d.k1).x < d.loss_thr) { lost_out++; continue; }
      const uint32_t k = atomicAdd(cnt, 1u);
      if (k < cap) out[k] = make_uint2(i, e);
      else set_err(d, DERR_OUTBOX);
    }
  }
  const int idx[3] = {S_BDROP, S_PROBERESP, S_LOSS};
  const unsigned long long v[3] = {lost_in, sent, lost_out};
  stat_add_n(d, idx, v);
}

// ================================================================================================
// Join responses: KnownPeers of every map entry (src/kaboodle.rs:356-392).  One workgroup per
// responding node: the row's member bitset goes to LDS once; for each response (list order) the
// member set at that moment is the bitset minus the joiners inserted later; when it does not fit in
// 10240 B the kept ranks are the first cap images of a keyed permutation of [0, n),
// each computed independently; ids come out sorted by rank/select on the bitset.
// ================================================================================================
__device__ inline bool newbit(const unsigned long long* nm, uint32_t e) { return (nm[e >> 6] >> (e & 63)) & 1ull; }
__device__ inline uint32_t mix32(uint32_t x) {
  x ^= x >> 16; x *= 0x7feb352du; x ^= x >> 15; x *= 0x846ca68bu; x ^= x >> 16;
  return x;
}
// The keyed permutation of [0, n): a 4-round Feistel network on b = max(2, ceil(log2 n))
// bits, halves of ceil(b/2) (high, mask ma) and floor(b/2) (low, mask mc) bits whose widths swap every
// round, cycle-walked into [0, n): at least half of every walk step lands in range.  Prp holds what
// depends on (n, key) only.
struct Prp { uint32_t n, c, ma, mc, k[4]; };
__device__ inline Prp prp_make(uint32_t n, const U4& key) {
  const uint32_t lg = n <= 1 ? 0u : 32u - __clz(n - 1u);        // ceil(log2 n)
  const uint32_t b = lg < 2 ? 2u : lg;
  Prp p;
  p.n = n; p.c = b / 2; p.mc = (1u << p.c) - 1u; p.ma = (1u << (b - p.c)) - 1u;
  p.k[0] = key.x; p.k[1] = key.y; p.k[2] = key.z; p.k[3] = key.w;
  return p;
}
// one Feistel pass over x (4 rounds; the XORed half is a bits wide in rounds 0 and 2, c bits in 1 and 3)
__device__ __attribute__((always_inline)) inline uint32_t prp_pass(uint32_t x, const Prp& p) {
  uint32_t L = x >> p.c, R = x & p.mc;
#pragma unroll
  for (int k = 0; k < 4; ++k) { const uint32_t t = R; R = L ^ (mix32(R ^ p.k[k]) & ((k & 1) ? p.mc : p.ma)); L = t; }
  return (L << p.c) | R;
}
__device__ __attribute__((always_inline)) inline uint32_t prp_eval(uint32_t x, const Prp& p) {
  do { x = prp_pass(x, p); } while (x >= p.n);
  return x;
}
__device__ __attribute__((always_inline)) inline uint32_t prp_walk(uint32_t x, uint32_t n, const U4& key) {
  return prp_eval(x, prp_make(n, key));
}
__device__ inline uint32_t bm_rank(const uint32_t* S, const uint32_t* SP, uint32_t id) {   // members < id
  const uint32_t blk = id >> 8, w = id >> 5;
  uint32_t r = SP[blk];
  for (uint32_t k = blk * 8; k < w; ++k) r += __popc(S[k]);
  return r + __popc(S[w] & ((1u << (id & 31)) - 1u));
}
// b-th member (0-based) of bitset S with 256-id block prefix SP[0..nblk] (SP[nblk] = total > b).
// The block is bracketed around the density guess b * nbu / total (nbu = blocks up to the last
// non-empty one; rows are dense below it), falling back to the whole range when the guess misses;
// the word and bit come from one 32-byte read of the block.  Any nbu gives the same answer.
// The block (256 ids) holding member b: bracketed around the density guess b * ratio (ratio = nbu /
// total, nbu = blocks up to the last non-empty one; rows are dense below it), falling back to the whole
// range when the guess misses.  Any ratio gives the same answer.
// The bracket's six prefix words are read at once and counted (no dependent search steps, so the
// searches of a batch's keys overlap); *base = SP[block].  Only a missed guess searches.
__device__ __attribute__((always_inline)) inline uint32_t bm_block(const uint32_t* SP, uint32_t nblk, float ratio,
                                                                   uint32_t b, uint32_t* base) {
  uint32_t g = (uint32_t)((float)b * ratio);
  g = g < nblk ? g : nblk - 1;
  const uint32_t l2 = g >= 2 ? g - 2 : 0, h2 = g + 3 < nblk ? g + 3 : nblk;   // h2 - l2 <= 5
  uint32_t v[6];
#pragma unroll
  for (int j = 0; j < 6; ++j) v[j] = SP[l2 + j < h2 ? l2 + j : h2];             // v[5] = SP[h2]
  if (v[0] <= b && b < v[5]) {
    uint32_t c = 0, bs = v[0];
#pragma unroll
    for (int j = 1; j < 5; ++j) { const bool le = v[j] <= b; c += le; bs = le ? v[j] : bs; }
    *base = bs;
    return l2 + c;
  }
  uint32_t lo = 0, hi = nblk;
  while (hi - lo > 1) { const uint32_t mid = (lo + hi) >> 1; if (SP[mid] <= b) lo = mid; else hi = mid; }
  *base = SP[lo];
  return lo;
}
// rem-th member of the 256-id block whose eight words are q0, q1
__device__ __attribute__((always_inline)) inline uint32_t block_pick(const uint4& q0, const uint4& q1, uint32_t blk,
                                                                     uint32_t rem) {
  // (rem < the block's count, as every caller guarantees) the word by a three-level search over pair and
  // quad counts: a few selects instead of a chain of eight compares
  const uint32_t p0 = __popc(q0.x), p1 = __popc(q0.y), p2 = __popc(q0.z), p3 = __popc(q0.w);
  const uint32_t p4 = __popc(q1.x), p5 = __popc(q1.y), p6 = __popc(q1.z);
  const uint32_t s01 = p0 + p1, s45 = p4 + p5, s03 = s01 + p2 + p3;
  const bool h1 = rem >= s03;
  rem -= h1 ? s03 : 0u;
  const uint32_t sa = h1 ? s45 : s01;
  const bool h2 = rem >= sa;
  rem -= h2 ? sa : 0u;
  const uint32_t pa = h1 ? (h2 ? p6 : p4) : (h2 ? p2 : p0);
  const bool h3 = rem >= pa;
  rem -= h3 ? pa : 0u;
  const uint32_t wi = (h1 ? 4u : 0u) + (h2 ? 2u : 0u) + (h3 ? 1u : 0u);
  const uint32_t xa = h1 ? (h2 ? (h3 ? q1.w : q1.z) : (h3 ? q1.y : q1.x)) : (h2 ? (h3 ? q0.w : q0.z) : (h3 ? q0.y : q0.x));
  return (blk * 8 + wi) * 32 + select_in_word(xa, rem);
}
// b-th member (0-based) of bitset S with 256-id block prefix SP[0..nblk] (SP[nblk] = total > b); the
// word and bit come from one 32-byte read of the block.
__device__ inline uint32_t bm_select(const uint32_t* S, const uint32_t* SP, uint32_t nblk, float ratio, uint32_t b) {
  uint32_t base;
  const uint32_t lo = bm_block(SP, nblk, ratio, b, &base);
  const uint4 q0 = *reinterpret_cast<const uint4*>(S + lo * 8), q1 = *reinterpret_cast<const uint4*>(S + lo * 8 + 4);
  return block_pick(q0, q1, lo, b - base);
}
// The sampled Join response (src/kaboodle.rs:373-383 restated): pay[k] for k in
// [k_first, cap) step `stride` = the select of rank prp(k) in the member set B minus the joiners
// inserted after the response (J[upto..nnew), suffix minima JM), stepping over them (least fixed point
// of e = #later joiners <= select(y + e)).  RESP_U keys per batch: their permutations, block searches and
// 32-byte block reads are independent, so the loads of a batch are in flight together.
// The joiners are read through an accessor: J and its suffix minima JM in LDS (the workgroup path), or
// held in a wave's registers (lane l: J[l], J[l + 64]; the wave path, whose LDS slice then holds no list).
constexpr uint32_t KB_RESP_U = 2;   // 2 of 3 and 4 measured best with the wave path at 4 waves per SIMD
constexpr int RESP_U = KB_RESP_U;
constexpr int RESP_KMAX = 9;          // keys per lane at stride >= 64: cap <= 567 (src/kaboodle.rs:43, :373-383)
struct JoinLds {
  const uint32_t *J, *JM;
  __device__ uint32_t min_from(uint32_t u) const { return JM[u]; }
  __device__ uint32_t at(uint32_t f) const { return J[f]; }
};
struct JoinRegs {                     // f uniform over the active lanes (a loop over [upto, nnew))
  uint32_t j0, j1, jmin;
  __device__ uint32_t min_from(uint32_t) const { return jmin; }
  __device__ uint32_t at(uint32_t f) const { return f < 64 ? rdl(j0, (int)f) : rdl(j1, (int)(f - 64)); }
};
template <class JA>
__device__ __attribute__((always_inline)) inline void sampled_fill(uint32_t* pay, uint32_t k_first, uint32_t stride,
                                                                   uint32_t cap, const Prp& P, const uint32_t* B,
                                                                   const uint32_t* BP, uint32_t NB, float ratio,
                                                                   const JA& J, uint32_t upto, uint32_t nnew) {
  const uint32_t jmin = J.min_from(upto);
  // (1) the permutation images of this lane's keys, cycle-walked as one stream: each step is one
  // Feistel pass of the lane's current key, so the wave waits for the slowest lane's total passes,
  // not for the slowest lane of every key
  const uint32_t mcount = k_first < cap ? (cap - k_first + stride - 1) / stride : 0u;
  uint32_t y[RESP_KMAX];
#pragma unroll
  for (int q = 0; q < RESP_KMAX; ++q) y[q] = 0;
  if (4ull * P.n >= 3ull * ((uint64_t)(P.ma + 1) << P.c)) {
    // n fills at least 3/4 of the Feistel domain (a large mesh: n just under a power of two), so a pass
    // rarely lands outside [0, n): each key walks on its own, unrolled, with no run-time indexing of y
    // (whose selects had cost more than the pass itself)
#pragma unroll
    for (int q = 0; q < RESP_KMAX; ++q) {
      const bool act = (uint32_t)q < mcount;
      if (!__ballot(act)) break;
      uint32_t x = prp_pass(k_first + stride * q, P);
      while (__ballot(act && x >= P.n)) { if (act && x >= P.n) x = prp_pass(x, P); }
      y[q] = x;
    }
  } else {
    uint32_t m = 0, x = k_first;
    while (__ballot(m < mcount)) {
      if (m < mcount) {
        x = prp_pass(x, P);
        if (x < P.n) {
#pragma unroll
          for (int q = 0; q < RESP_KMAX; ++q) if ((uint32_t)q == m) y[q] = x;
          ++m;
          x = k_first + stride * m;
        }
      }
    }
  }
  // (2) rank -> id, RESP_U keys at a time with their block searches and 32-byte block reads in flight
#pragma unroll
  for (int q0 = 0; q0 < RESP_KMAX; q0 += RESP_U) {
    if ((uint32_t)q0 >= mcount) break;
    uint32_t blk[RESP_U], bb[RESP_U];
    uint4 b0[RESP_U], b1[RESP_U];
#pragma unroll
    for (int u = 0; u < RESP_U; ++u) {
      bb[u] = 0;
      blk[u] = q0 + u < RESP_KMAX ? bm_block(BP, NB, ratio, y[q0 + u < RESP_KMAX ? q0 + u : 0], &bb[u]) : 0u;
    }
#pragma unroll
    for (int u = 0; u < RESP_U; ++u) {
      b0[u] = *reinterpret_cast<const uint4*>(B + blk[u] * 8);
      b1[u] = *reinterpret_cast<const uint4*>(B + blk[u] * 8 + 4);
    }
#pragma unroll
    for (int u = 0; u < RESP_U; ++u) {
      const uint32_t q = q0 + u;
      if (q >= RESP_KMAX || q >= mcount) break;
      const uint32_t yq = y[q];
      uint32_t xq = block_pick(b0[u], b1[u], blk[u], yq - bb[u]);
      if (xq >= jmin) {                               // rare: a later joiner may sit at or below xq
        uint32_t e = 0;
        while (true) {
          uint32_t c = 0;
          for (uint32_t f = upto; f < nnew; ++f) c += J.at(f) <= xq;
          if (c == e) break;
          e = c;
          xq = bm_select(B, BP, NB, ratio, yq + e);
        }
      }
      pay[k_first + stride * q] = xq;
    }
  }
}
constexpr uint32_t RESP_LDS_W = 131072;   // rows up to this many ids keep their bitsets in LDS
constexpr uint32_t RESP_JCAP = 1024;      // new joiners of one receiver kept in LDS (more: read from HBM)
__host__ __device__ inline size_t resp_words(uint32_t NW, uint32_t NB) {
  return (2ull * NW + 2ull * (NB + 1) + 2ull * RESP_JCAP + 1 + 3) & ~3ull;
}

// exclusive prefix of the member counts of X's 256-id blocks into XP[0..NB], XP[NB] = total (block-wide)
__device__ __attribute__((always_inline)) inline uint32_t block_prefix(const uint32_t* X, uint32_t* XP, uint32_t NB, uint32_t* s_red) {
  const uint32_t t = threadIdx.x, T = blockDim.x;
  const uint32_t per = (NB + T - 1) / T;
  uint32_t bc = 0;
  for (uint32_t k = t * per; k < (t + 1) * per && k < NB; ++k) {
    uint32_t c = 0;
    for (uint32_t w = 0; w < 8; ++w) c += __popc(X[k * 8 + w]);
    XP[k] = c; bc += c;
  }
  uint32_t ex = wave_excl(bc);
  const uint32_t wt = wave_sum(bc);
  __syncthreads();
  if (lane() == 0) s_red[t >> 6] = wt;
  __syncthreads();
  for (uint32_t w = 0; w < (t >> 6); ++w) ex += s_red[w];
  uint32_t tot = 0;
  for (uint32_t w = 0; w < T / 64; ++w) tot += s_red[w];
  for (uint32_t k = t * per; k < (t + 1) * per && k < NB; ++k) { const uint32_t c = XP[k]; XP[k] = ex; ex += c; }
  if (t == 0) XP[NB] = tot;
  __syncthreads();
  return tot;
}

// The common case of a large mesh — every response of the node is truncated (sampled), at most
// RW_JCAP new joiners — takes one WAVE per responder instead of a workgroup: four responders per
// workgroup at once, each with its own LDS slice (bitset, block prefix, joiners, suffix minima), and
// only wave-level synchronisation.  Same arithmetic as k_resp_node's sampled path.
constexpr uint32_t RW_JCAP = 128;
// The slice also holds a copy of the row bitset, taken while the block prefix is counted (the same
// loads): every sampled select then reads its 32-byte block from LDS instead of L2.  The joiner list
// passes through the head before the prefix is counted there and then lives in registers, so a slice
// is the prefix and the row: at the 64K bench's rows four workgroups fit a CU (4 waves per SIMD).
__host__ __device__ inline uint32_t rwave_head(uint32_t NB) { return ((NB + 1 > RW_JCAP ? NB + 1 : RW_JCAP) + 3) & ~3u; }
__host__ __device__ inline uint32_t rwave_words(uint32_t NW, uint32_t NB) { return rwave_head(NB) + NW; }
__device__ inline bool resp_by_wave(const Dev& d, uint32_t i, uint32_t nnew, bool on) {
  return on && d.uniform && nnew <= RW_JCAP && d.n[i] - nnew > d.capj;
}
// Rows too wide for a wave's LDS copy (SG: above ≈ 110K ids; configs[3]'s 1M-id rows) keep only the head
// (block prefix, joiners, suffix minima) in LDS and read the selects' 32-byte blocks from the row's bitset
// itself: nothing writes a row while the Join responses are built, and a responder's row stays in L2 across
// its responses.  (The workgroup path instead copied each row to HBM scratch first.)
template <bool SG>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(4))) void k_resp_wave(Dev d, PhaseB pb, const uint32_t* nodes, const uint32_t* nnodes_p,
                                                   OutBuf ob, int32_t r, uint32_t* rest) {
  extern __shared__ __attribute__((aligned(16))) uint32_t rw_lds[];
  const uint32_t NW = d.NWR, NB = d.W / 256;
  const uint32_t wv = threadIdx.x >> 6, l = lane(), nwv = blockDim.x >> 6;
  uint32_t* BP = rw_lds + (size_t)wv * (SG ? rwave_head(NB) : rwave_words(NW, NB));   // block prefix [NB + 1]
  uint32_t* Jt = BP;                                            // the new joiners, in passing      [RW_JCAP]
  uint32_t* S = BP + rwave_head(NB);                            // the row bitset (LDS copy)         [NW]
  const uint32_t nnodes = *nnodes_p;
  // A responder's HBM reads (its Join masks, header words, row bitset) are issued together, with the next
  // responder's id: one memory round trip per responder instead of one per dependent use.  With at most 64
  // mask words and 128 Join entries (every round of a large mesh) lane l holds mask word l and the ids of
  // Join entries l and l + 64, which are the same for every responder and read once.
  const bool small_lists = pb.JW <= 64 && pb.nj <= 128;
  const uint32_t js0 = small_lists && l < pb.nj ? pb.bjoin[l].sender : 0u;
  const uint32_t js1 = small_lists && l + 64 < pb.nj ? pb.bjoin[l + 64].sender : 0u;
  const uint32_t stride = gridDim.x * nwv;
  uint32_t it = blockIdx.x * nwv + wv;
  uint32_t inext = it < nnodes ? nodes[it] : 0u;
  for (; it < nnodes; it += stride) {
    const uint32_t i = inext;
    const unsigned long long* nm = pb.newmask + (size_t)i * pb.JW;
    const unsigned long long* rm = pb.respmask + (size_t)i * pb.JW;
    const unsigned long long nmv = small_lists && l < pb.JW ? nm[l] : 0ull;
    const unsigned long long rmv = small_lists && l < pb.JW ? rm[l] : 0ull;
    const uint32_t n_i = d.n[i], nbase_i = pb.nbase[i], poff_i = ob.poff[i], ooff_i = ob.off[i];
    inext = it + stride < nnodes ? nodes[it + stride] : 0u;
    const uint32_t* B = bits_of(d, i);                      // row membership after the Join group
    const uint4* B4 = reinterpret_cast<const uint4*>(B);
    // the row into LDS, every load in flight, before the wave-path test: it fails for a few responders at
    // most (each then costs one wasted copy) and the copy's wait covers the loads above
    const bool tdbg = (d.dev & 512) != 0;                   // phase timing (KB_DEV=512, KB_DEBUG_WAVES)
    const uint64_t tps = tdbg ? wall_clock64() : 0;
    if (!SG) stage16(reinterpret_cast<uint4*>(S), B4, NW / 4, l, 64);
    uint32_t nnew = 0;
    if (small_lists) nnew = wave_sum((uint32_t)__popcll(nmv));
    else for (uint32_t wj = 0; wj < pb.JW; ++wj) nnew += __popcll(nm[wj]);
    if (!(d.uniform && nnew <= RW_JCAP && n_i - nnew > d.capj)) {   // resp_by_wave: k_resp_node serves it
      if (l == 0) rest[atomicAdd(&d.ctr[C_RESTN], 1u)] = i;
      wait_lds();
      __builtin_amdgcn_wave_barrier();
      continue;
    }
    if (l == 0) path_hit(d, SG ? PATH_RESP_WAVE_HBM : PATH_RESP_WAVE);
    uint64_t tp0 = tdbg ? wall_clock64() : 0, tp1 = 0, tp2 = 0;
    if (small_lists) {                                      // new joiners in list order: entries l and l + 64
      const unsigned long long w0 = ((unsigned long long)rdl((uint32_t)(nmv >> 32), 0) << 32) | rdl((uint32_t)nmv, 0);
      const unsigned long long w1 = ((unsigned long long)rdl((uint32_t)(nmv >> 32), 1) << 32) | rdl((uint32_t)nmv, 1);
      if (l < pb.nj && ((w0 >> l) & 1ull)) Jt[__popcll(w0 & ((1ull << l) - 1ull))] = js0;
      if (l + 64 < pb.nj && ((w1 >> l) & 1ull)) Jt[__popcll(w0) + __popcll(w1 & ((1ull << l) - 1ull))] = js1;
    } else {
      for (uint32_t e = l; e < pb.nj; e += 64) {
        if (!newbit(nm, e)) continue;
        uint32_t pos = __popcll(nm[e >> 6] & ((1ull << (e & 63)) - 1ull));
        for (uint32_t w2 = 0; w2 < (e >> 6); ++w2) pos += __popcll(nm[w2]);
        Jt[pos] = pb.bjoin[e].sender;
      }
    }
    wait_lds();
    __builtin_amdgcn_wave_barrier();
    const uint32_t jr0 = l < nnew ? Jt[l] : 0xFFFFFFFFu, jr1 = l + 64 < nnew ? Jt[l + 64] : 0xFFFFFFFFu;
    uint32_t sm0 = jr0, sm1 = jr1;                          // suffix minima of J[0..nnew), nnew <= 128
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const uint32_t u0 = __shfl_down(sm0, o, 64), u1 = __shfl_down(sm1, o, 64);
      if (l + o < 64) { sm0 = u0 < sm0 ? u0 : sm0; sm1 = u1 < sm1 ? u1 : sm1; }
    }
    {
      const uint32_t m1 = rdl(sm1, 0);
      sm0 = m1 < sm0 ? m1 : sm0;
    }
    wait_lds();                                             // the list is out of the head before the prefix
    __builtin_amdgcn_wave_barrier();
    if (tdbg) tp1 = wall_clock64();
    const uint32_t per = (NB + 63) / 64;                    // block prefix, `per` blocks per lane
    uint32_t bc = 0, last = 0;
    const uint4* S4 = reinterpret_cast<const uint4*>(SG ? B : S);
    for (uint32_t k = l * per; k < (l + 1) * per && k < NB; ++k) {
      const uint4 q0 = S4[2 * k], q1 = S4[2 * k + 1];
      const uint32_t c = __popc(q0.x) + __popc(q0.y) + __popc(q0.z) + __popc(q0.w) + __popc(q1.x) + __popc(q1.y) +
                         __popc(q1.z) + __popc(q1.w);
      BP[k] = c; bc += c;
      if (c) last = k + 1;
    }
    uint32_t ex = wave_excl(bc);
    const uint32_t nB = wave_sum(bc);
    const uint32_t nbu = wave_max(last);
    const float ratio = nB ? (float)nbu / (float)nB : 0.0f;
    for (uint32_t k = l * per; k < (l + 1) * per && k < NB; ++k) { const uint32_t c = BP[k]; BP[k] = ex; ex += c; }
    if (l == 0) BP[NB] = nB;
    wait_lds();
    __builtin_amdgcn_wave_barrier();
    uint32_t poff = poff_i, q = 0, ins_before = 0;
    if (tdbg) tp2 = wall_clock64();
    for (uint32_t wj = 0; wj < pb.JW; ++wj) {
      unsigned long long rmw, nmw;
      if (small_lists) {
        rmw = ((unsigned long long)rdl((uint32_t)(rmv >> 32), (int)wj) << 32) | rdl((uint32_t)rmv, (int)wj);
        nmw = ((unsigned long long)rdl((uint32_t)(nmv >> 32), (int)wj) << 32) | rdl((uint32_t)nmv, (int)wj);
      } else {
        rmw = rm[wj]; nmw = nm[wj];
      }
      while (rmw) {
        const uint32_t bit = (uint32_t)(__ffsll((long long)rmw) - 1);
        const uint32_t K = wj * 64 + bit;
        rmw &= rmw - 1;
        const uint32_t upto = ins_before + __popcll(nmw & ((2ull << bit) - 1ull));   // new joiners <= K
        const uint32_t expect = nbase_i + upto;
        const uint32_t a = small_lists ? (K < 64 ? rdl(js0, (int)K) : rdl(js1, (int)(K - 64))) : pb.bjoin[K].sender;
        const uint32_t nk = nB - (nnew - upto), cap = d.capj;
        uint32_t* pay = ob.pay + poff;
        const Prp P = prp_make(nk, philox(i, (uint32_t)r, (uint32_t)P_TRUNC << 24, a, d.k0, d.k1));
        const uint32_t jmin = upto < 64 ? rdl(sm0, (int)upto) : upto < 128 ? rdl(sm1, (int)(upto - 64)) : 0xFFFFFFFFu;
        sampled_fill(pay, l, 64, cap, P, SG ? B : S, BP, NB, ratio, JoinRegs{jr0, jr1, jmin}, upto, nnew);
        if (l == 0) {
          Msg m; m.dest = a; m.sender = i; m.seq = q; m.kind = K_KP; m.a = cap; m.fp = 0; m.n = 0; m.off = poff;
          ob.msgs[ooff_i + q] = m;
          if (nk != expect) set_err(d, DERR_RESP);
        }
        poff += cap; q++;
      }
      ins_before += __popcll(nmw);
    }
    // algorithmic bytes: the row bitset, its Join masks and joiner ids read; the responses' ids and
    // records written
    if (l == 0) slot_add(d, S_RESPB, 4ull * NW + 16ull * pb.JW + 4ull * pb.nj + (4ull * d.capj + 32ull) * q +
                                     (SG ? 32ull * d.capj * q : 0ull));   // SG: each select's block read from the row
    if (tdbg && l == 0) {
      __builtin_amdgcn_s_waitcnt(0);
      const uint64_t tp3 = wall_clock64();
      atomicAdd(&d.ctr[C_DBG_TNODE], (uint32_t)(tp2 - tp1)); atomicAdd(&d.ctr[C_DBG_TBASE], (uint32_t)(tp1 - tp0));
      atomicAdd(&d.ctr[C_DBG_TINS], (uint32_t)(tp3 - tp2)); atomicAdd(&d.ctr[C_DBG_TSTART], 1u);
      atomicAdd(&d.ctr[C_DBG_MSGS], q); atomicAdd(&d.ctr[C_DBG_TEND], (uint32_t)(tp0 - tps));
    }
    wait_lds();                                           // the LDS slice is reused by the next responder
    __builtin_amdgcn_wave_barrier();
  }
}

__global__ __launch_bounds__(256) void k_resp_node(Dev d, PhaseB pb, const uint32_t* nodes, const uint32_t* nnodes_p,
                                                   OutBuf ob, int32_t r, uint32_t* gscratch, bool wave_on) {
  extern __shared__ uint32_t lds_dyn[];
  const uint32_t NW = d.NWR, NB = d.W / 256;
  // rows wider than RESP_LDS_W keep their bitsets in a per-workgroup slice of global scratch
  uint32_t* lds = gscratch ? gscratch + (size_t)blockIdx.x * resp_words(NW, NB) : lds_dyn;
  uint32_t* B = lds;                 // row membership after the Join group   [NW]
  uint32_t* BP = B + NW;             // block prefix of B                     [NB + 1]
  uint32_t* S = BP + NB + 1;         // members at response (unsampled path)  [NW]
  uint32_t* SP = S + NW;             // block prefix of S                     [NB + 1]
  uint32_t* J = SP + NB + 1;         // ids of this receiver's new joiners    [RESP_JCAP]
  uint32_t* JM = J + RESP_JCAP;      // suffix minima of J                    [RESP_JCAP + 1]
  __shared__ uint32_t s_red[16];
  const uint32_t t = threadIdx.x, T = blockDim.x;
  const uint32_t nnodes = *nnodes_p;
  for (uint32_t it = blockIdx.x; it < nnodes; it += gridDim.x) {
    const uint32_t i = nodes[it];
    const unsigned long long* nm = pb.newmask + (size_t)i * pb.JW;
    const unsigned long long* rm = pb.respmask + (size_t)i * pb.JW;
    uint32_t nnew = 0;
    for (uint32_t wj = 0; wj < pb.JW; ++wj) nnew += __popcll(nm[wj]);
    if (resp_by_wave(d, i, nnew, wave_on)) continue;        // uniform: served by k_resp_wave
    if (gscratch) copy16(reinterpret_cast<uint4*>(B), reinterpret_cast<const uint4*>(bits_of(d, i)), NW / 4, t, T);
    else stage16(reinterpret_cast<uint4*>(B), reinterpret_cast<const uint4*>(bits_of(d, i)), NW / 4, t, T);
    __syncthreads();
    const uint32_t nB = block_prefix(B, BP, NB, s_red);
    const bool jl = nnew <= RESP_JCAP;
    if (jl) {                            // new joiners in list order (parallel), then suffix minima
      for (uint32_t e = t; e < pb.nj; e += T) {
        if (!newbit(nm, e)) continue;
        uint32_t pos = __popcll(nm[e >> 6] & ((1ull << (e & 63)) - 1ull));
        for (uint32_t w2 = 0; w2 < (e >> 6); ++w2) pos += __popcll(nm[w2]);
        J[pos] = pb.bjoin[e].sender;
      }
      __syncthreads();
      if (nnew <= T) {                     // suffix minima by a block scan (one joiner per thread)
        uint32_t v = t < nnew ? J[t] : 0xFFFFFFFFu;
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
          const uint32_t u = __shfl_down(v, o, 64);
          if (lane() + o < 64) v = u < v ? u : v;
        }
        if (lane() == 0) s_red[t >> 6] = v;
        __syncthreads();
        for (uint32_t w = (t >> 6) + 1; w < T / 64; ++w) v = s_red[w] < v ? s_red[w] : v;
        if (t < nnew) JM[t] = v;
        if (t == 0) JM[nnew] = 0xFFFFFFFFu;
      } else if (t == 0) {
        uint32_t m = 0xFFFFFFFFu;
        JM[nnew] = m;
        for (uint32_t q3 = nnew; q3 > 0; --q3) { m = J[q3 - 1] < m ? J[q3 - 1] : m; JM[q3 - 1] = m; }
      }
    }
    __syncthreads();
    uint32_t poff = ob.poff[i], q = 0, ins_before = 0;
    for (uint32_t wj = 0; wj < pb.JW; ++wj) {
      unsigned long long rmw = rm[wj];
      const unsigned long long nmw = nm[wj];
      while (rmw) {
        const uint32_t bit = (uint32_t)(__ffsll((long long)rmw) - 1);
        const uint32_t K = wj * 64 + bit;
        rmw &= rmw - 1;
        const uint32_t upto = ins_before + __popcll(nmw & ((2ull << bit) - 1ull));   // new joiners <= K
        const uint32_t expect = pb.nbase[i] + upto;
        const uint32_t a = pb.bjoin[K].sender;
        // the member set at this response: B minus the joiners inserted after K
        const uint32_t nk = nB - (nnew - upto);
        const bool sample = d.uniform && nk > d.capj;
        const uint32_t cap = sample ? d.capj : nk;
        uint32_t* pay = ob.pay + poff;
        if (sample) {
          // kept ranks = first cap images of the keyed permutation; rank -> id by select on B,
          // stepping over later joiners (least fixed point of e = #later joiners <= select(y + e))
          const Prp P = prp_make(nk, philox(i, (uint32_t)r, (uint32_t)P_TRUNC << 24, a, d.k0, d.k1));
          const float ratio = nB ? (float)NB / (float)nB : 0.0f;
          if (jl) {                                      // later joiners = J[upto..nnew)
            sampled_fill(pay, t, T, cap, P, B, BP, NB, ratio, JoinLds{J, JM}, upto, nnew);
          } else {
            for (uint32_t k = t; k < cap; k += T) {
              const uint32_t y = prp_eval(k, P);
              uint32_t e = 0, x;
              while (true) {
                x = bm_select(B, BP, NB, ratio, y + e);
                uint32_t c = 0;
                for (uint32_t f = K + 1; f < pb.nj; ++f)
                  if (newbit(nm, f)) c += pb.bjoin[f].sender <= x;
                if (c == e) break;
                e = c;
              }
              pay[k] = x;
            }
          }
        } else {
          for (uint32_t k = t; k < NW; k += T) S[k] = B[k];
          __syncthreads();
          for (uint32_t f = K + 1 + t; f < pb.nj; f += T)
            if (newbit(nm, f)) { const uint32_t x = pb.bjoin[f].sender; atomicAnd(&S[x >> 5], ~(1u << (x & 31))); }
          __syncthreads();
          block_prefix(S, SP, NB, s_red);
          for (uint32_t w = t; w < NW; w += T) {        // every member, position = rank
            uint32_t x = S[w];
            if (!x) continue;
            uint32_t pos = bm_rank(S, SP, w * 32);
            while (x) { const uint32_t b = __ffs(x) - 1; x &= x - 1; pay[pos++] = w * 32 + b; }
          }
        }
        if (t == 0) {
          Msg m; m.dest = a; m.sender = i; m.seq = q; m.kind = K_KP; m.a = cap; m.fp = 0; m.n = 0; m.off = poff;
          ob.msgs[ob.off[i] + q] = m;
          if (nk != expect) set_err(d, DERR_RESP);
          if (gscratch) path_hit(d, sample ? PATH_RESP_SCRATCH_SAMPLED : PATH_RESP_SCRATCH_FULL);
        }
        poff += cap; q++;
        __syncthreads();
      }
      ins_before += __popcll(nmw);
    }
  }
}

}  // namespace kb
