// kb_sim.hip — MI355X (gfx950) implementation of the Kaboodle SWIM round as a bulk-synchronous
// simulator over HBM-resident structure-of-arrays tables.  Exposes the C ABI of include/kaboodle_sim.h.
//
// Round pipeline, one HIP stream; the host reads 8 bytes per round (+20 when the
// broadcasts produced Join responses, to size the wave-0 outbox):
//   k_rebase (every 64 rounds)      stamp window shift                             
//   k_events / k_churn_*            Kaboodle::start/stop, churn                    src/lib.rs:136-183
//   k_alive_bits, k_truefp_*        running set and its fingerprint
//   k_bfail_prep(_lds), k_lat_mark  per-list facts of the Failed broadcasts
//   k_rowpass  <- dominant kernel   handle_incoming_broadcasts (Failed, Join) + ping_random_peer's
//                                   oldest-5 candidates, one pass per row        :256-311, :655-703
//   k_lat_sweep                     latency entries of Failed removals (track_latency)  :789-817
//   k_resp_wave / k_resp_node       maybe_send_known_peers_to_peer                 :356-392
//   k_tick_scan, k_tick_pre         maybe_broadcast_join + handle_suspected_peers  :228-251, :558-653
//   k_fold                          stale fingerprint checkpoints refolded         :71-83
//   k_tick_post                     ping target, handle_incoming_ping_requests     :655-703, :550-556
//   k_bcast_write                   the round's Join/Failed lists
//   waves: k_route (k_route_x, k_pack, exchange, k_route_recv when sharded), k_scan_*, k_scatter,
//          k_kp_small, k_kp_group, k_sort_inbox (+ KPR oversize probe), k_proc_fast, k_proc
//                                   handle_incoming_messages                       src/kaboodle.rs:394-548
#include <hip/hip_runtime.h>
#include <hip/hip_ext.h>
#include <stdint.h>
#include <stdio.h>
#include <string.h>
#include <stdlib.h>
#include <string>
#include <vector>
#include <array>
#include <algorithm>
#include <atomic>
#include <thread>
#include "kb_common.h"
#include "kb_wire.h"
#include "kb_round.h"
#include "kb_tick.h"
#include "kb_waves.h"
#include "kb_xfer.h"
#include "kb_sparse.h"

using namespace kb;

// Every launch of a round is tagged with one of these ids; with profiling on (kb_sim_set_profiling) it
// carries start/stop events on its own dispatch packet and kb_sim_kernel_breakdown reports the sums.
enum KId : int {
  KI_REBASE, KI_EVENTS, KI_CHURN_LEAVE, KI_CHURN_JOIN, KI_ALIVE_BITS, KI_TRUEFP_PART, KI_TRUEFP_FIN, KI_LOG_MARK,
  KI_LAT_MARK, KI_BFAIL_PREP, KI_ROWPASS, KI_LAT_SWEEP, KI_SCAN_TILES, KI_SCAN_APPLY, KI_SET_CAP, KI_RESP_WAVE,
  KI_RESP_NODE, KI_TICK_SCAN, KI_TICK_PRE, KI_FOLD, KI_FP_ROWS, KI_TICK_POST, KI_BCAST_WRITE, KI_ROUTE, KI_ROUTE_X,
  KI_XBOUND, KI_PACK, KI_ROUTE_RECV, KI_SCATTER, KI_SCATTER_FLAT, KI_KP, KI_SORTFAST, KI_PROC, KI_ROUND_END,
  KI_PROBE, KI_A3_EXACT, NKI
};
static const char* const KNAME[NKI] = {
  "k_rebase", "k_events", "k_churn_leave", "k_churn_join", "k_alive_bits", "k_truefp_part", "k_truefp_fin",
  "k_log_mark", "k_lat_mark", "k_bfail_prep", "k_rowpass", "k_lat_sweep", "k_scan_tiles", "k_scan_apply",
  "k_set_cap", "k_resp_wave", "k_resp_node", "k_tick_scan", "k_tick_pre", "k_fold", "k_fp_rows", "k_tick_post",
  "k_bcast_write", "k_route", "k_route_x", "k_xbound", "k_pack", "k_route_recv", "k_scatter", "k_scatter_flat",
  "k_kp", "k_sortfast", "k_proc", "k_round_end", "k_probe", "k_a3_exact"};
// the in-kernel algorithmic byte counter of a kernel (StatIdx), or -1
static int kbytes_stat(int kid) {
  switch (kid) {
    case KI_ROWPASS: return S_ROWB;
    case KI_FOLD: return S_FOLDB;
    case KI_RESP_WAVE: return S_RESPB;
    case KI_PROC: return S_PROCB;
    default: return -1;
  }
}

// ================================================================================================
// Exclusive scan over up to 4 arrays of length n (+ optional compaction of indices j with in[0][j] != 0),
// two fully parallel passes over 1024-element tiles: per-tile sums, then per-tile offsets + local scan.
// ================================================================================================
struct ScanArgs {
  const uint32_t* in[4]; uint32_t* out[4]; int narr; uint32_t n;
  uint32_t* totals;   // device, narr values (+ list count at totals[4] when list != null)
  uint32_t* list; uint32_t* list_count; uint32_t list_base;   // list entries are j + list_base
  uint32_t list_or3;  // list flag: in[0][j] != 0, or also in[3][j] != 0 when set
  uint32_t addc[4];   // constant added to every element of array q before scanning
  uint32_t* tiles;    // workspace [5 * ntiles]
  uint32_t ntiles;
};
__device__ inline uint32_t scan_val(const ScanArgs& a, int q, uint32_t j) {
  if (q == 4) return a.in[0][j] != 0 || (a.list_or3 && a.in[3][j] != 0);
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
  if (a.list && j < a.n && v[4]) a.list[base[4] + wpre[4][t >> 6] + ex[4]] = j + a.list_base;
  if (tile == gridDim.x - 1 && t == 1023) {
    for (int q = 0; q < a.narr; ++q) a.totals[q] = base[q] + wpre[q][15] + ex[q] + v[q];
    if (a.list) { const uint32_t c = base[4] + wpre[4][15] + ex[4] + v[4]; a.totals[4] = c; if (a.list_count) *a.list_count = c; }
  }
}


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
// (also hands the wave-0 scan totals to the host: tot[0..4] -> host-mapped hpin[0..4], then the
// sequence number the host polls for)
__global__ void k_set_cap(Dev d, const uint32_t* nresp, uint32_t* cap, uint32_t* cnt, const uint32_t* tot, uint32_t* hpin,
                          uint32_t seq) {
  const uint32_t i = d.lo + blockIdx.x * blockDim.x + threadIdx.x;
  if (i < d.hi) { cap[i] = nresp[i] + TICK_MAX; cnt[i] = nresp[i]; }
  if (blockIdx.x == 0 && threadIdx.x == 0) { d.ctr[C_RESTN] = 0; pin_publish(hpin, tot, 5, seq); }
}
// device values -> the host's mapped pinned buffer, then the sequence number it polls for (sharded
// hand-offs of all-gathered counts)
__global__ void k_publish(const uint32_t* v, uint32_t n, uint32_t* hpin, uint32_t seq) {
  if (blockIdx.x == 0 && threadIdx.x == 0) pin_publish(hpin, v, n, seq);
}
__global__ void k_init_nodes(Dev d, uint32_t n0) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= d.C) return;
  if (local(d, i)) { d.last_bcast[i] = NONE_ROUND; d.a3cur[i] = i; }
  d.start_round[i] = NONE_ROUND;
  if (i < n0) node_start(d, i, 0);
}
// rows of the initial members (the local ones): every initial member known and "ancient", self now
__global__ void k_init_converged_rows(Dev d, uint32_t n0) {
  const uint32_t wpr = d.W / 16;
  const uint32_t r0 = d.lo, r1 = n0 < d.hi ? n0 : d.hi;
  const size_t words = r1 > r0 ? (size_t)(r1 - r0) * wpr : 0;
  uint4* p = reinterpret_cast<uint4*>(d.stamp);
  for (size_t k = (size_t)blockIdx.x * blockDim.x + threadIdx.x; k < words; k += (size_t)gridDim.x * blockDim.x) {
    const uint32_t i = r0 + (uint32_t)(k / wpr), c = (uint32_t)(k % wpr);
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
  const size_t bw = r1 > r0 ? (size_t)(r1 - r0) * d.NWR : 0;
  for (size_t k = (size_t)blockIdx.x * blockDim.x + threadIdx.x; k < bw; k += (size_t)gridDim.x * blockDim.x) {
    const uint32_t w = (uint32_t)(k % d.NWR);
    uint32_t x = 0;
    if (w * 32 + 32 <= n0) x = 0xFFFFFFFFu;
    else if (w * 32 < n0) x = (1u << (n0 - w * 32)) - 1u;
    d.bits[(size_t)r0 * d.NWR + k] = x;
  }
}
__global__ void k_init_converged_nodes(Dev d, uint32_t n0) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= d.C) return;
  const bool loc = local(d, i);
  if (loc) { d.last_bcast[i] = NONE_ROUND; d.a3cur[i] = i; }
  d.start_round[i] = NONE_ROUND;
  if (i >= n0) return;
  d.alive[i] = 1; d.start_round[i] = 0;
  if (loc) { d.dirty[i] = 1; d.n[i] = n0; d.last_bcast[i] = -1000; d.paq_n[i] = 0; d.sdirty[i] = ~0ull; }
}
__global__ void k_mark_all_dirty(Dev d) {
  const uint32_t i = d.lo + blockIdx.x * blockDim.x + threadIdx.x;
  if (i < d.hi) { d.dirty[i] = 1; d.sdirty[i] = ~0ull; }
}
__global__ __launch_bounds__(64) void k_fp_one(Dev d, uint32_t i) {
  __shared__ uint32_t ztab[ZT * 128];
  load_ztab(d, ztab);
  if (!d.dirty[i]) return;
  const uint32_t f = wave_fp(d, ztab, i, 0);
  if (lane() == 0) { d.fp[i] = f; d.dirty[i] = 0; }
}
__global__ __launch_bounds__(256) void k_fp_all(Dev d) {
  __shared__ uint32_t ztab[ZT * 128];
  load_ztab(d, ztab);
  const uint32_t i = d.lo + blockIdx.x * 4 + (threadIdx.x >> 6);
  if (i >= d.hi || !d.dirty[i]) return;
  const uint32_t f = wave_fp(d, ztab, i, 0);
  if (lane() == 0) { d.fp[i] = f; d.dirty[i] = 0; }
}

// ================================================================================================
// Host side
// ================================================================================================
static thread_local std::string g_err;
static void seterr(const std::string& s) { g_err = s; }
#define HIPCHK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { seterr(std::string(#x) + ": " + hipGetErrorString(e_)); return KB_IO_ERROR; } } while (0)

// zeroed device memory, the zeroing complete on return (hipMemset runs on the null stream, which does not order
// with the simulator's non-blocking stream: a buffer regrown mid-round could be zeroed after a kernel wrote it)
template <class T> static hipError_t dalloc(T** p, size_t n) {
  hipError_t e = hipMalloc((void**)p, sizeof(T) * (n ? n : 1));
  if (e == hipSuccess) e = hipMemset(*p, 0, sizeof(T) * (n ? n : 1));
  if (e == hipSuccess) e = hipDeviceSynchronize();
  return e;
}

// the Join broadcasts of external peers (kb_sim_inject) merged into the round's Join list in sender
// order, as the tick's Joins would be (one per sender, bseq 0; pad = the sender's partition group when the list
// carries it, pgroups > 1)
static int merge_ext_joins(hipStream_t st, BCast* list, uint32_t* n, std::vector<uint32_t>& joins, uint32_t pgroups, uint32_t C) {
  if (joins.empty()) return KB_OK;
  std::vector<BCast> v(*n);
  if (*n) HIPCHK(hipMemcpyAsync(v.data(), list, sizeof(BCast) * *n, hipMemcpyDeviceToHost, st));
  HIPCHK(hipStreamSynchronize(st));
  for (const uint32_t x : joins) {
    const uint32_t g = pgroups > 1 ? (uint32_t)((uint64_t)x * pgroups / C) : 0u;
    const auto at = std::upper_bound(v.begin(), v.end(), x, [](uint32_t a, const BCast& b) { return a < b.sender; });
    v.insert(at, BCast{x, x, 0, g});
  }
  HIPCHK(hipMemcpyAsync(list, v.data(), sizeof(BCast) * v.size(), hipMemcpyHostToDevice, st));
  HIPCHK(hipStreamSynchronize(st));
  *n = (uint32_t)v.size();
  joins.clear();
  return KB_OK;
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

// Event streams (src/events.rs:57-100): the net difference between `node`'s membership bitset and
// the observer's snapshot.  One workgroup walks the row 1024 words at a time; the ids of each pass
// are compacted in ascending order by a wave scan plus a scan over the 16 wave totals.
// out = [discovered: C][departed: C][n_discovered, n_departed, n_known]
__global__ __launch_bounds__(1024) void k_events_diff(const uint32_t* __restrict__ row,
                                                      const uint32_t* __restrict__ snap, uint32_t C,
                                                      uint32_t* __restrict__ out) {
  __shared__ uint32_t wa[16], wr[16], base[2], known;
  const uint32_t t = threadIdx.x, lane = t & 63, wv = t >> 6, nw = (C + 31) / 32;
  uint32_t* add = out;
  uint32_t* rem = out + C;
  if (t == 0) { base[0] = 0; base[1] = 0; known = 0; }
  __syncthreads();
  uint32_t kn = 0;
  for (uint32_t w0 = 0; w0 < nw; w0 += 1024) {
    const uint32_t w = w0 + t;
    uint32_t cur = 0, old = 0;
    if (w < nw) {
      const uint32_t valid = (C - w * 32 >= 32) ? ~0u : ((1u << (C - w * 32)) - 1u);
      cur = row[w] & valid;
      old = snap[w] & valid;
    }
    const uint32_t a = cur & ~old, r = old & ~cur;
    kn += __popc(cur);
    uint32_t pa = __popc(a), pr = __popc(r);
    for (int o = 1; o < 64; o <<= 1) {
      const uint32_t xa = __shfl_up(pa, o, 64), xr = __shfl_up(pr, o, 64);
      if (lane >= (uint32_t)o) { pa += xa; pr += xr; }
    }
    if (lane == 63) { wa[wv] = pa; wr[wv] = pr; }
    __syncthreads();
    uint32_t oa = base[0] + pa - __popc(a), orr = base[1] + pr - __popc(r);
    for (uint32_t k = 0; k < wv; ++k) { oa += wa[k]; orr += wr[k]; }
    for (uint32_t m = a; m; m &= m - 1) add[oa++] = w * 32 + __ffs(m) - 1;
    for (uint32_t m = r; m; m &= m - 1) rem[orr++] = w * 32 + __ffs(m) - 1;
    __syncthreads();
    if (t == 1023) { base[0] = oa; base[1] = orr; }
    __syncthreads();
  }
  for (int o = 32; o > 0; o >>= 1) kn += __shfl_down(kn, o, 64);
  if (lane == 0) atomicAdd(&known, kn);
  __syncthreads();
  if (t == 0) { out[2 * C] = base[0]; out[2 * C + 1] = base[1]; out[2 * C + 2] = known; }
}
// the drain: the snapshot becomes the current row
__global__ __launch_bounds__(256) void k_events_commit(const uint32_t* __restrict__ row, uint32_t* __restrict__ snap,
                                                       uint32_t nw) {
  const uint32_t w = blockIdx.x * 256 + threadIdx.x;
  if (w < nw) snap[w] = row[w];
}
// one node's latencies out of the peer-major table (peer_states)
__global__ __launch_bounds__(256) void k_lat_column(Dev d, uint32_t node, uint16_t* out) {
  const uint32_t j = blockIdx.x * 256 + threadIdx.x;
  if (j < d.C) out[j] = *lat_at(d, node, j);
}

namespace kb { struct SpSim; }
struct kb_sim {
  kb_config cfg;
  SpSim* sp = nullptr;                 // KB_VARIANT_SPARSE_ROWS: the sparse-row engine answers every call
  Dev d;
  int device;
  hipStream_t st;
  // side stream: kernels off the round's critical path (the running set's fingerprint, the latency sweep)
  // run beside it, forked from and joined back into st by events
  hipStream_t st2 = nullptr;
  hipEvent_t ev_fork[3] = {nullptr, nullptr, nullptr}, ev_join[3] = {nullptr, nullptr, nullptr};   // side work 0-2
  uint32_t C, W, S;                    // capacity, row stride, row-sweep column splits
  // row shard: this handle holds rows [lo, hi) of the mesh, R = hi - lo
  uint32_t lo, hi, R;
  int rank, world;
  Xfer* xf;                            // null: unsharded (no exchange at all)
  bool in_group;                       // a shard of a kb_sim_create_local group
  std::vector<void*> allocs;           // device memory owned by this handle
  int32_t round;
  std::vector<uint8_t> h_ident, h_idlen;
  std::vector<uint8_t> h_pend; std::vector<int16_t> h_pendlen;   // identity set on a stopped instance that ran:
                                                                 // its next address takes it (-1: none)
  std::vector<uint8_t> h_moved;                                  // the instance bound here restarted elsewhere
  std::vector<uint8_t> h_idset;                                  // identity set on a never-bound address (d.idset)
  std::vector<uint8_t> h_ext;                                    // external peers (d.ext)
  // external peers: records injected for the next round's wave 0, records exported not drained
  size_t n_ext = 0;
  std::vector<XRec> inj; std::vector<uint32_t> inj_ids;
  std::vector<uint32_t> inj_join;                    // external peers' Join broadcasts for the next round
  XRec* d_inj = nullptr; uint32_t* d_inj_ids = nullptr; size_t d_inj_cap = 0, d_inj_ids_cap = 0;
  std::vector<kb_unicast> xq; std::vector<uint32_t> xq_ids;
  std::vector<Event> events;
  uint32_t* rpack = nullptr; uint32_t* rpack_in = nullptr;       // a restart's packed row (send / receive)
  // discovery: Probes queued for the next round, those delivered this round, responses not yet drained
  std::vector<kb_wire_addr> probe_q, probes;
  std::vector<kb_probe_response> presp;
  uint2* d_presp = nullptr; uint32_t* d_presp_n = nullptr; size_t presp_cap = 0;
  OutBuf ob[2];
  WaveCtl wc;
  uint32_t msg_cap, pay_cap;
  BCast* bfail; BCast* bjoin;          // the round's broadcast lists (whole mesh, sender order)
  BCast* bfail_loc; BCast* bjoin_loc;  // sharded: this shard's part, before the all-gather
  uint32_t nf, nj;
  uint32_t ucap = 0;                   // Join-response union slots (sharded meshes, kb_waves.h UCAP)
  uint64_t xbytes_cross = 0, xbytes_all = 0;   // bytes this shard's waves sent to other shards / to every shard
  BcastSlots bs;
  uint32_t* join_off; uint32_t* fail_off;
  uint32_t* scan_tot; uint32_t* scan_tiles;
  unsigned long long* newmask; unsigned long long* respmask; size_t mask_words;
  unsigned long long* newmask_base; unsigned long long* respmask_base;
  uint32_t* nresp; uint32_t* paysum; uint32_t* nbase; uint32_t* resp_off;
  uint32_t* resp_nodes; uint32_t* bf_gid; uint8_t* bf_dep;
  uint32_t* slow;                      // the nodes of a wave k_proc_fast leaves to k_proc
  uint16_t* lat_col;                   // [C] one node's latencies (peer_states), track_latency only
  uint32_t* fnamed;                    // [NWR] peers named by the round's Failed list (track_latency only)
  uint32_t* resp_scratch; size_t resp_scratch_words;
  RowOut ro;
  Event* d_events; uint32_t events_cap;
  // sharded waves: send side (xs), all-gathered counts, receive buffers (grown on demand)
  XState xs;
  uint32_t* xall; unsigned long long* xstats;
  std::vector<uint32_t> h_xall;
  Msg* rmsg; uint32_t* rpay; uint8_t* rstatus; uint32_t* rinbox; uint32_t* rkp;
  size_t rmsg_cap, rpay_cap;
  double round_ms;                     // the whole round: markers on the stream, read back like the kernels'
  uint32_t* rr = nullptr;              // [3] the round's {Join, Failed, error} on the device (sharded gather)
  uint64_t round_launches, bj_total, bf_total;
  // per-kernel profile (kb_sim_kernel_breakdown): with prof_on every launch carries start/stop events
  // on its own dispatch packet; a round's records are read back during the next round's final wait
  // (the host is idle then), the last round's on query
  struct KRec { int16_t kid, wave; hipEvent_t a, b; };
  int prof_level = 1;                  // 0 none, 1 the kernels with byte counters, 2 every launch
  bool capturing = false;              // inside a HIP graph capture: launches carry no events
  int cur_wave = -1;                   // the delivery wave being launched (-1: outside the window)
  std::vector<hipEvent_t> ev_free;
  std::vector<KRec> krec;
  double k_ms[NKI] = {};
  double k_wms[NKI][KB_WAVE_SLOTS] = {};
  uint64_t k_n[NKI] = {};
  uint64_t k_bytes0[NSTAT] = {};
  uint64_t host_syncs = 0;             // host waits on the device (stream syncs, pinned hand-offs) since creation
  uint32_t ncu = 256;
  bool debug_waves = false;
  size_t lds_per_cu = 65536;
  // kb_sim_create_local: a façade over `world` in-process shards (one host thread each per step)
  std::vector<kb_sim*> shards;
  LocalHub* hub;
  // event observers (kb_sim_watch): a watched node and the device snapshot of its membership bitset
  // at the last drain, plus the fingerprint last reported for it
  std::vector<uint32_t> watch_node, watch_fp;
  std::vector<uint32_t*> watch_snap;
  uint32_t* ev_out = nullptr;          // [2*C + 4]: discovered ids, departed ids, counters
  uint32_t* h_pin = nullptr;           // [16] pinned host memory, mapped: per-round results written by kernels
  uint32_t* d_pin = nullptr;           //      its device address
  uint32_t pin_seq = 0;                // hand-off sequence number (h_pin[PIN_SEQ])
  uint64_t occ_key = ~0ull; int occ_val = 0;   // row-pass occupancy query, cached per launch shape
  // the unsharded receive window as a HIP graph (launch_waves), re-captured when buffers are regrown
  bool graph_on = false;               // env KB_WAVE_GRAPH=1
  hipGraph_t wave_graph = nullptr; hipGraphExec_t wave_exec = nullptr;
  uint64_t buf_gen = 0, wave_gen = ~0ull;
};

// allocation of this handle's device memory; row tables hold the local rows only and their pointer
// is biased by -lo rows so kernels index them with global ids
template <class T> static hipError_t talloc(kb_sim* s, T** p, size_t n) {
  hipError_t e = dalloc(p, n);
  if (e == hipSuccess) s->allocs.push_back((void*)*p);
  return e;
}
template <class T> static T* bias(T* base, size_t per_row, uint32_t lo) {
  return reinterpret_cast<T*>(reinterpret_cast<uintptr_t>(base) - sizeof(T) * per_row * lo);
}
template <class T> static hipError_t ralloc(kb_sim* s, T** p, size_t per_row) {
  T* base = nullptr;
  hipError_t e = talloc(s, &base, per_row * s->R);
  *p = bias(base, per_row, s->lo);
  return e;
}
template <class T> static T* L(const kb_sim* s, T* p) { return p + s->lo; }   // biased row table -> local base

// ---- launches and their profile ------------------------------------------------------------------
static void prof_events(kb_sim* s, int kid, hipEvent_t* a, hipEvent_t* b) {
  *a = *b = nullptr;
  // level 1 times the once-per-round kernels with byte counters only: k_proc's eight launches a round
  // would add ≈ 0.05 ms of event dispatch overhead to the round (tools/ev_cost.py)
  if (s->capturing || s->prof_level <= 0 || (s->prof_level == 1 && (kbytes_stat(kid) < 0 || kid == KI_PROC))) return;
  hipEvent_t e[2];
  for (int k = 0; k < 2; ++k) {
    if (!s->ev_free.empty()) { e[k] = s->ev_free.back(); s->ev_free.pop_back(); }
    else if (hipEventCreate(&e[k]) != hipSuccess) { if (k) s->ev_free.push_back(e[0]); return; }
  }
  *a = e[0]; *b = e[1];
  const int w = s->cur_wave < 0 ? -1 : (s->cur_wave < KB_WAVE_SLOTS ? s->cur_wave : KB_WAVE_SLOTS - 1);
  s->krec.push_back(kb_sim::KRec{(int16_t)kid, (int16_t)w, e[0], e[1]});
}
// every kernel of the round is launched through here: the dispatch packet itself records the events
template <typename F, typename... Args>
static void klaunch_on(kb_sim* s, hipStream_t stream, int kid, F kern, dim3 grid, dim3 block, uint32_t lds, Args... args) {
  hipEvent_t a, b;
  prof_events(s, kid, &a, &b);
  hipExtLaunchKernelGGL(kern, grid, block, lds, stream, a, b, 0, args...);
}
template <typename F, typename... Args>
static void klaunch(kb_sim* s, int kid, F kern, dim3 grid, dim3 block, uint32_t lds, Args... args) {
  klaunch_on(s, s->st, kid, kern, grid, block, lds, args...);
}
// fork side work k onto st2 after everything st has queued so far / join it back into st
static void side_fork(kb_sim* s, int k) { (void)hipEventRecord(s->ev_fork[k], s->st); (void)hipStreamWaitEvent(s->st2, s->ev_fork[k], 0); }
static void side_done(kb_sim* s, int k) { (void)hipEventRecord(s->ev_join[k], s->st2); }
static void side_join(kb_sim* s, int k) { (void)hipStreamWaitEvent(s->st, s->ev_join[k], 0); }
// fold the first n records (complete: their round has ended) into the per-kernel sums
static void prof_resolve(kb_sim* s, size_t n) {
  n = std::min(n, s->krec.size());
  for (size_t k = 0; k < n; ++k) {
    const kb_sim::KRec& q = s->krec[k];
    float ms = 0;
    hipError_t e = hipEventElapsedTime(&ms, q.a, q.b);
    if (e == hipErrorNotReady) {                      // still pending (an earlier round's tail): wait for it
      (void)hipGetLastError();                        // rather than drop the record and recycle live events
      (void)hipEventSynchronize(q.b);
      e = hipEventElapsedTime(&ms, q.a, q.b);
    }
    if (e == hipSuccess) {
      if (q.kid == NKI) { s->round_ms += ms; s->round_launches++; }          // the whole round
      else {
        s->k_ms[q.kid] += ms; s->k_n[q.kid]++;
        if (q.wave >= 0) s->k_wms[q.kid][q.wave] += ms;
      }
    }
    s->ev_free.push_back(q.a); s->ev_free.push_back(q.b);
  }
  s->krec.erase(s->krec.begin(), s->krec.begin() + n);
}

static ScanArgs scan_args(kb_sim* s, uint32_t n, uint32_t* totals) {
  ScanArgs a; memset(&a, 0, sizeof a); a.n = n; a.totals = totals;
  a.tiles = s->scan_tiles; a.ntiles = (n + 1023) / 1024; return a;
}
static void launch_scan(kb_sim* s, const ScanArgs& a) {
  if (!a.n) return;
  klaunch(s, KI_SCAN_TILES, k_scan_tiles, dim3(a.ntiles), dim3(1024), 0, a);
  klaunch(s, KI_SCAN_APPLY, k_scan_apply, dim3(a.ntiles), dim3(1024), 0, a);
}

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

// (re)upload per-id segment CRCs, the Z tables and the half-block tables
static int upload_segments(kb_sim* s) {
  const uint32_t C = s->C;
  std::vector<uint32_t> cseg(C), segmul(C), seglen(C);
  bool uniform = true;
  uint32_t xp[ADDR_LEN + MAXID + 1];                 // x^(8 len) per segment length
  for (uint32_t l = 0; l <= ADDR_LEN + MAXID; ++l) xp[l] = h_xpow8(l);
  for (uint32_t j = 0; j < C; ++j) {
    char a[32]; kb_format_addr(j, a, sizeof a);
    uint32_t reg = h_crc_update(0, (const uint8_t*)a, ADDR_LEN);
    reg = h_crc_update(reg, &s->h_ident[(size_t)j * MAXID], s->h_idlen[j]);
    cseg[j] = reg; seglen[j] = ADDR_LEN + s->h_idlen[j]; segmul[j] = xp[seglen[j]];
    if (s->h_idlen[j] != s->cfg.id_len) uniform = false;
  }
  s->d.uniform = uniform ? 1 : 0;
  s->d.L = ADDR_LEN + s->cfg.id_len;
  const uint32_t Z = h_xpow8(s->d.L);
  std::vector<uint32_t> zpow(std::max<uint32_t>(C + 2, 17));     // the tables below need Z^0..Z^16
  zpow[0] = 0x80000000u;
  for (size_t k = 1; k < zpow.size(); ++k) zpow[k] = multmodp(Z, zpow[k - 1]);
  std::vector<uint32_t> ztab(17 * 128);
  for (uint32_t c = 0; c <= 16; ++c)
    for (uint32_t k = 0; k < 8; ++k)
      for (uint32_t v = 0; v < 16; ++v) ztab[c * 128 + k * 16 + v] = multmodp(zpow[c], v << (4 * k));
  HIPCHK(hipMemcpy(s->d.cseg, cseg.data(), 4ull * C, hipMemcpyHostToDevice));
  HIPCHK(hipMemcpy(s->d.segmul, segmul.data(), 4ull * C, hipMemcpyHostToDevice));
  HIPCHK(hipMemcpy(s->d.seglen, seglen.data(), 4ull * C, hipMemcpyHostToDevice));
  HIPCHK(hipMemcpy(s->d.zpow, zpow.data(), 4ull * (C + 2), hipMemcpyHostToDevice));
  {
    std::vector<uint32_t> zf(C + 2);
    for (uint32_t k = 0; k < C + 2; ++k) zf[k] = multmodp(zpow[k], 0xFFFFFFFFu);
    HIPCHK(hipMemcpy(s->d.zfin, zf.data(), 4ull * (C + 2), hipMemcpyHostToDevice));
  }
  HIPCHK(hipMemcpy(s->d.ztab, ztab.data(), 4ull * ztab.size(), hipMemcpyHostToDevice));
  std::vector<uint32_t> zb(ZB);
  for (uint32_t c = 0; c < 9; ++c)
    for (uint32_t k = 0; k < 4; ++k)
      for (uint32_t v = 0; v < 256; ++v) zb[c * 1024 + k * 256 + v] = multmodp(zpow[c], v << (8 * k));
  HIPCHK(hipMemcpy(s->d.zbtab, zb.data(), 4ull * zb.size(), hipMemcpyHostToDevice));
  const size_t hn = (size_t)(s->W / 8) * 256;
  k_build_htab<<<(unsigned)((hn + 255) / 256), 256>>>(s->d);
  HIPCHK(hipDeviceSynchronize());
  return KB_OK;
}

#include "kb_sparse_host.h"

// a handle answered by the sparse-row engine: the whole mesh (xf null) or one row shard of it (owns xf)
static int sp_wrap(const kb_config* cfg, int rank, int world, Xfer* xf, kb_sim** out) {
  if (cfg->capacity == 0 || cfg->capacity > 7800000u || cfg->initial_nodes > cfg->capacity || cfg->id_len > MAXID ||
      cfg->max_waves == 0 || cfg->max_waves > 64) { seterr("config out of range"); delete xf; return KB_INVALID_ARGUMENT; }
  SpSim* sp = nullptr;
  const int rc = sp_create(cfg, rank, world, xf, &sp);
  if (rc) return rc;
  kb_sim* s = new kb_sim();
  s->cfg = *cfg; s->C = cfg->capacity; s->sp = sp; s->device = sp->device; s->rank = rank; s->world = world;
  s->lo = sp->lo; s->hi = sp->hi; s->R = sp->R;
  *out = s;
  return KB_OK;
}

static void free_all(kb_sim* s) {
  for (void* p : s->allocs) (void)hipFree(p);
  s->allocs.clear();
  void* dyn[] = {s->newmask_base, s->respmask_base, s->resp_scratch, s->d_events, s->rmsg, s->rpay, s->rstatus,
                 s->rinbox, s->rkp, s->d_presp, s->d_presp_n, s->rpack, s->rpack_in, s->d_inj, s->d_inj_ids};
  for (void* p : dyn) if (p) (void)hipFree(p);
}
static void destroy_shard(kb_sim* s) {
  (void)hipSetDevice(s->device);
  if (s->st) (void)hipStreamSynchronize(s->st);
  free_all(s);
  for (auto& q : s->krec) { (void)hipEventDestroy(q.a); (void)hipEventDestroy(q.b); }
  for (hipEvent_t e : s->ev_free) (void)hipEventDestroy(e);
  if (s->h_pin) (void)hipHostFree(s->h_pin);
  if (s->wave_exec) (void)hipGraphExecDestroy(s->wave_exec);
  if (s->wave_graph) (void)hipGraphDestroy(s->wave_graph);
  if (s->st) (void)hipStreamDestroy(s->st);
  if (s->st2) (void)hipStreamDestroy(s->st2);
  for (int k = 0; k < 3; ++k) {
    if (s->ev_fork[k]) (void)hipEventDestroy(s->ev_fork[k]);
    if (s->ev_join[k]) (void)hipEventDestroy(s->ev_join[k]);
  }
  delete s->xf;
  delete s;
}

// One handle = rows [lo, hi) of a mesh; unsharded when xf is null (world 1, no exchange).
static int create_shard(const kb_config* cfg, int rank, int world, Xfer* xf, kb_sim** out) {
  h_crc_init();
  if (!cfg || !out || cfg->abi_version != KB_ABI_VERSION) { seterr("bad config"); delete xf; return KB_INVALID_ARGUMENT; }
  if (cfg->capacity == 0 || cfg->capacity > 7800000u || cfg->initial_nodes > cfg->capacity || cfg->id_len > MAXID ||
      cfg->max_waves == 0 || cfg->max_waves > 64) { seterr("config out of range"); delete xf; return KB_INVALID_ARGUMENT; }
  if (cfg->stat_flags) { seterr("kb_config.stat_flags: sparse rows and the oracle only"); delete xf; return KB_INVALID_ARGUMENT; }
  if (cfg->variant && cfg->variant != KB_VARIANT_EXACT_LRU) { seterr(cfg->variant == KB_VARIANT_SPARSE_ROWS ? "sparse rows run unsharded (kb_sim_create)" : "semantic variants other than KB_VARIANT_SPARSE_ROWS are measurement-only (CPU oracle)"); delete xf; return KB_INVALID_ARGUMENT; }
  const uint32_t C = cfg->capacity;
  const uint32_t rows_per = (C + (uint32_t)world - 1) / (uint32_t)world;
  if (world < 1 || world > (int)XMAX || rank < 0 || rank >= world || (uint64_t)(world - 1) * rows_per >= C) {
    seterr("shard layout out of range (1..8 shards, each holding at least one row)"); delete xf; return KB_INVALID_ARGUMENT;
  }
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0) { seterr("no HIP device"); delete xf; return KB_NO_DEVICE; }
  kb_sim* s = new kb_sim();
  memset((void*)&s->d, 0, sizeof s->d);
  memset((void*)&s->xs, 0, sizeof s->xs);
  s->cfg = *cfg;
  s->xf = xf;
  s->rank = rank; s->world = world;
  s->device = cfg->device >= 0 ? cfg->device : 0;
  if (cfg->device < 0) (void)hipGetDevice(&s->device);
  if (hipSetDevice(s->device) != hipSuccess) { destroy_shard(s); seterr("hipSetDevice failed"); return KB_NO_DEVICE; }
  {
    hipDeviceProp_t prop;
    if (hipGetDeviceProperties(&prop, s->device) != hipSuccess) { destroy_shard(s); seterr("hipGetDeviceProperties failed"); return KB_NO_DEVICE; }
    s->ncu = (uint32_t)prop.multiProcessorCount;
    s->lds_per_cu = prop.maxSharedMemoryPerMultiProcessor ? prop.maxSharedMemoryPerMultiProcessor : 65536;
  }
  const uint32_t W = (C + 8191) / 8192 * 8192;       // 64 segments of whole 128-id steps
  s->C = C; s->W = W; s->round = 0;
  s->lo = (uint32_t)rank * rows_per;
  s->hi = std::min<uint32_t>(C, s->lo + rows_per);
  s->R = s->hi - s->lo;
  const uint32_t R = s->R;
  const uint32_t groups = (R + 63) / 64;
  uint32_t S = 1;
constexpr uint32_t KB_FOLD_WAVES = 16384;                            // fold waves wanted: column splits double up to it (64K:
                                                       // 16 splits, 0.44 -> 0.42 ms against 8 and 32, profiles/r04fs_ab_fold_splits.txt)
  while (S < 64 && groups * S < KB_FOLD_WAVES) S <<= 1;   // enough sweep waves to fill the chip
  s->S = S;
  Dev& d = s->d;
  d.lo = s->lo; d.hi = s->hi;
  d.C = C; d.W = W; d.SEGW = W / NSEG; d.NWR = W / 32;
  d.segq = d.SEGW / 128;
  d.segm = d.segq > 1 ? (uint32_t)(((1ull << 32) + d.segq - 1) / d.segq) : 0u;
  d.k0 = (uint32_t)cfg->seed; d.k1 = (uint32_t)(cfg->seed >> 32);
  d.loss_thr = cfg->loss_threshold; d.churn_thr = cfg->churn_threshold; d.fault_end = cfg->fault_end_round;
  d.failed_mode = cfg->failed_mode; d.pgroups = cfg->partition_groups; d.pstart = cfg->partition_start;
  d.pend = cfg->partition_end;
  const uint32_t Lid = cfg->id_len;
  d.capk = (BUFSZ - 20 - Lid) / (18 + Lid);           // 20 + L + k(18+L) <= 10240
  d.capj = (BUFSZ - 20 - Lid - 1) / (18 + Lid);       // 20 + L + k(18+L) <  10240
  d.paybound = C < d.capk ? C : d.capk;
  d.dbg = cfg->debug_flags;
  if (const char* dv = getenv("KB_DEV")) d.dev = (uint32_t)atoi(dv);
  s->debug_waves = getenv("KB_DEBUG_WAVES") != nullptr;
  if (const char* gv = getenv("KB_WAVE_GRAPH")) s->graph_on = atoi(gv) != 0;
  if (cfg->debug_flags & KB_DBG_WAVE_GRAPH) s->graph_on = true;
  s->h_ident.assign((size_t)C * MAXID, 0); s->h_idlen.assign(C, (uint8_t)Lid);
  s->h_pend.assign((size_t)C * MAXID, 0); s->h_pendlen.assign(C, (int16_t)-1); s->h_moved.assign(C, 0);
  s->h_idset.assign(C, 0);
  for (uint32_t j = 0; j < C; ++j) default_identity(j, Lid, &s->h_ident[(size_t)j * MAXID]);
  hipError_t e = hipSuccess;
#define A(ptr, n) if (e == hipSuccess) e = talloc(s, &(ptr), (n))     // per-id / global tables
#define AR(ptr, n) if (e == hipSuccess) e = ralloc(s, &(ptr), (n))   // row tables: n entries per local row
  AR(d.stamp, W); AR(d.bits, d.NWR); AR(d.segp, NSEG); AR(d.sdirty, 1);
  AR(d.dirty, 1); A(d.alive, C); A(d.idset, C); A(d.ext, C); A(d.abits, d.NWR); A(d.start_round, C); AR(d.n, 1); AR(d.fp, 1);
  AR(d.last_bcast, 1); AR(d.a3cur, 1); AR(d.susp, SLOTS); AR(d.cur, CSLOTS); AR(d.paq, PAQ);
  AR(d.paq_n, 1); A(d.cseg, C); A(d.segmul, C); A(d.seglen, C); A(d.zpow, (size_t)C + 2); A(d.zfin, (size_t)C + 2);
  A(d.ztab, 17 * 128); A(d.zbtab, ZB);
  A(d.htab, (size_t)(W / 8) * 256); A(d.stats, NSTAT); A(d.sacc, (size_t)NACC * NSTAT); A(d.ctr, NCTR); A(d.truefp, 1); A(d.tfpart, TRUEFP_G);
  AR(d.flog, LOGCAP); AR(d.flog_n, 1); AR(d.fstart, 16); AR(d.kpr_big, 1);
  if (cfg->variant == KB_VARIANT_EXACT_LRU) { AR(d.tst, W); AR(d.tlb, W / 1024); }   // exact A3 instants
  if (cfg->track_latency) { A(d.lat, (size_t)W * lat_stride(R)); A(s->lat_col, C); A(s->fnamed, d.NWR); }   // peer-major
  s->msg_cap = std::max<uint32_t>(8u * R + (uint32_t)TICK_MAX * R, 1u << 16);
  s->pay_cap = std::max<uint32_t>((d.capk + 1) * R, 1u << 24);
  for (int b = 0; b < 2; ++b) {
    A(s->ob[b].msgs, s->msg_cap); A(s->ob[b].pay, s->pay_cap); AR(s->ob[b].off, 1); AR(s->ob[b].cap, 1);
    AR(s->ob[b].cnt, 1); AR(s->ob[b].poff, 1);
    s->ob[b].msg_cap = s->msg_cap; s->ob[b].pay_cap = s->pay_cap;
  }
  AR(s->wc.cnt1, 1); AR(s->wc.bnd, 1); AR(s->wc.bpay, 1); AR(s->wc.cursor, 1);
  AR(s->wc.in_off, 1); A(s->wc.active, R);
  AR(s->wc.kcnt, 1); AR(s->wc.kpay, 1); AR(s->wc.kcur, 1); AR(s->wc.koff, 1);
  if (!xf) { A(s->wc.status, s->msg_cap); A(s->wc.inbox, s->msg_cap); A(s->wc.kin, s->msg_cap); }
  A(s->bfail, (size_t)C * SLOTS); A(s->bjoin, C);
  AR(s->bs.join, 1); AR(s->bs.nfail, 1); AR(s->bs.fail, SLOTS); AR(s->join_off, 1); AR(s->fail_off, 1);
  A(s->scan_tot, 32); A(s->rr, 4); A(s->scan_tiles, 5 * ((std::max<size_t>(C, (size_t)world * R) + 1023) / 1024) + 5);
  AR(s->nresp, 1); AR(s->paysum, 1); AR(s->nbase, 1); AR(s->resp_off, 1);
  A(s->resp_nodes, R); A(s->bf_gid, (size_t)C * SLOTS); A(s->bf_dep, (size_t)C * SLOTS); A(s->slow, R);
  AR(s->ro.part, 10);
  if (xf) {
    XState& x = s->xs;
    x.world = (uint32_t)world; x.R = R; x.S = rows_per; x.RS = R + 1;
    x.NWW = d.NWR; x.nju = 0; x.uon = 0;
    s->ucap = std::min<uint32_t>(UCAP, C);             // Join-response unions (kb_waves.h): slots and their reserve
    A(x.ostatus, s->msg_cap); A(x.xcnt, (size_t)world * x.RS); A(x.xpay, (size_t)world * x.RS);
    A(x.xoff, (size_t)world * x.RS); A(x.xpoff, (size_t)world * x.RS); A(x.xb, 2 * world);
    A(x.smsg, (size_t)s->msg_cap + s->ucap); A(x.spay, (size_t)s->pay_cap + (size_t)s->ucap * x.NWW);
    A(x.jslot, C); A(x.ubits, (size_t)s->ucap * x.NWW); A(x.uany, s->ucap);
    A(s->xall, std::max(2 * world * world, 3 * world));   // wave counts (2W per rank), round results (3 per rank)
    A(s->xstats, NSTAT);
    A(s->bfail_loc, (size_t)R * SLOTS); A(s->bjoin_loc, R);
    s->h_xall.assign(2 * world * world, 0);
  }
#undef A
#undef AR
  if (e != hipSuccess) { seterr(std::string("device allocation failed: ") + hipGetErrorString(e)); destroy_shard(s); return KB_CAPACITY; }
  (void)hipMemset(L(s, d.kpr_big), 0xFF, 4ull * R);          // no round yet
  if (xf) { (void)hipMemset(s->xs.jslot, 0xFF, 4ull * C); (void)hipMemset(s->xs.ubits, 0, 4ull * s->ucap * s->xs.NWW); }
  if (d.lat) { (void)hipMemset(d.lat, 0xFF, 2ull * lat_stride(R) * W); (void)hipMemset(s->fnamed, 0, 4ull * d.NWR); }   // all None
  if (d.tst) {
    (void)hipMemsetD32(d.tst + (size_t)s->lo * W, INT32_MIN / 2, (size_t)R * W);   // a converged start: ancient, all tied
    (void)hipMemsetD32(d.tlb + (size_t)s->lo * (W / 1024), INT32_MIN, (size_t)R * (W / 1024));   // bounds: scan every block once
  }
  s->wc.msg_cap = s->msg_cap; s->wc.pay_cap = s->pay_cap;
  if (hipStreamCreateWithFlags(&s->st, hipStreamNonBlocking) != hipSuccess) { destroy_shard(s); seterr("stream"); return KB_IO_ERROR; }
  if (hipStreamCreateWithFlags(&s->st2, hipStreamNonBlocking) != hipSuccess) { destroy_shard(s); seterr("stream"); return KB_IO_ERROR; }
  for (int k = 0; k < 3; ++k)
    if (hipEventCreateWithFlags(&s->ev_fork[k], hipEventDisableTiming) != hipSuccess ||
        hipEventCreateWithFlags(&s->ev_join[k], hipEventDisableTiming) != hipSuccess) { destroy_shard(s); seterr("events"); return KB_IO_ERROR; }
  if (hipHostMalloc((void**)&s->h_pin, 4 * PIN_WORDS, hipHostMallocMapped | hipHostMallocCoherent) != hipSuccess) {
    s->h_pin = nullptr; destroy_shard(s); seterr("pinned buffer"); return KB_IO_ERROR;
  }
  if (hipHostGetDevicePointer((void**)&s->d_pin, s->h_pin, 0) != hipSuccess) { destroy_shard(s); seterr("pinned buffer mapping"); return KB_IO_ERROR; }
  if (const char* pv = getenv("KB_PROF")) s->prof_level = atoi(pv);
  int rc = upload_segments(s);
  if (rc) { destroy_shard(s); return rc; }
  uint32_t ctr0[NCTR] = {0};
  ctr0[C_NEXTFREE] = cfg->initial_nodes;
  ctr0[C_FIRSTCONV] = 0xFFFFFFFFu; ctr0[C_LASTCONV] = 0xFFFFFFFFu;
  if (hipMemcpy(d.ctr, ctr0, sizeof ctr0, hipMemcpyHostToDevice) != hipSuccess) { destroy_shard(s); seterr("ctr upload"); return KB_IO_ERROR; }
  const uint32_t tb = 256, gb = (C + tb - 1) / tb;
  if (cfg->init_mode == KB_INIT_CONVERGED) {
    k_init_converged_rows<<<4096, 256, 0, s->st>>>(d, cfg->initial_nodes);
    k_init_converged_nodes<<<gb, tb, 0, s->st>>>(d, cfg->initial_nodes);
  } else {
    k_init_nodes<<<gb, tb, 0, s->st>>>(d, cfg->initial_nodes);
  }
  if (hipStreamSynchronize(s->st) != hipSuccess) { destroy_shard(s); seterr("init failed"); return KB_IO_ERROR; }
  *out = s;
  return KB_OK;
}

static void destroy_one(kb_sim* s) {                 // a dense shard, or a sparse handle (its engine owns the exchange)
  if (s->sp) { sp_destroy(s->sp); delete s; return; }
  destroy_shard(s);
}

extern "C" int kb_sim_create(const kb_config* cfg, kb_sim** out) {
  if (cfg && out && cfg->abi_version == KB_ABI_VERSION && (cfg->variant & KB_VARIANT_SPARSE_ROWS)) {
    if (cfg->capacity == 0 || cfg->capacity > 7800000u || cfg->initial_nodes > cfg->capacity || cfg->id_len > MAXID ||
        cfg->max_waves == 0 || cfg->max_waves > 64) { seterr("config out of range"); return KB_INVALID_ARGUMENT; }
    return sp_wrap(cfg, 0, 1, nullptr, out);
  }
  return create_shard(cfg, 0, 1, nullptr, out);
}

extern "C" int kb_rccl_unique_id(uint8_t* out, size_t cap) {
  if (!out || cap < sizeof(ncclUniqueId)) { seterr("unique id buffer too small"); return KB_INVALID_ARGUMENT; }
  ncclUniqueId id;
  const ncclResult_t r = ncclGetUniqueId(&id);
  if (r != ncclSuccess) { seterr(std::string("ncclGetUniqueId: ") + ncclGetErrorString(r)); return KB_IO_ERROR; }
  memcpy(out, &id, sizeof id);
  return KB_OK;
}

// a unique id for ranks that share ONE device (the IpcXfer test transport, kb_xfer.h): the magic prefix, then the
// name of the shared-memory segment rank 0 creates
extern "C" int kb_ipc_unique_id(uint8_t* out, size_t cap) {
  if (!out || cap < KB_UNIQUE_ID_BYTES) { seterr("unique id buffer too small"); return KB_INVALID_ARGUMENT; }
  memset(out, 0, KB_UNIQUE_ID_BYTES);
  memcpy(out, IPC_MAGIC, sizeof IPC_MAGIC);
  uint64_t rnd = 0;
  FILE* f = fopen("/dev/urandom", "rb");
  if (f) { if (fread(&rnd, sizeof rnd, 1, f) != 1) rnd = 0; fclose(f); }
  snprintf(reinterpret_cast<char*>(out) + sizeof IPC_MAGIC, KB_UNIQUE_ID_BYTES - sizeof IPC_MAGIC, "/kbipc-%d-%016llx",
           (int)getpid(), (unsigned long long)rnd);
  return KB_OK;
}

extern "C" int kb_sim_create_rank(const kb_config* cfg, int32_t rank, int32_t world, const uint8_t* unique_id, kb_sim** out) {
  if (!cfg || !unique_id || !out || world < 1 || world > (int)XMAX || rank < 0 || rank >= world) {
    seterr("bad rank/world"); return KB_INVALID_ARGUMENT;
  }
  if (hipSetDevice(cfg->device >= 0 ? cfg->device : 0) != hipSuccess) { seterr("hipSetDevice failed"); return KB_NO_DEVICE; }
  if (memcmp(unique_id, IPC_MAGIC, sizeof IPC_MAGIC) == 0) {          // ranks sharing one device (test transport)
    const char* wm = getenv("KB_IPC_WINDOW_MB");
    const size_t mb = wm ? (size_t)atoll(wm) : 256;
    IpcXfer* x = new IpcXfer();
    if (!x->init(rank, world, unique_id, mb << 20)) { seterr(x->error()); delete x; return KB_IO_ERROR; }
    return (cfg->variant & KB_VARIANT_SPARSE_ROWS) ? sp_wrap(cfg, rank, world, x, out) : create_shard(cfg, rank, world, x, out);
  }
  RcclXfer* x = new RcclXfer();
  if (!x->init(rank, world, unique_id)) { seterr(x->error()); delete x; return KB_IO_ERROR; }
  return (cfg->variant & KB_VARIANT_SPARSE_ROWS) ? sp_wrap(cfg, rank, world, x, out) : create_shard(cfg, rank, world, x, out);
}

extern "C" int kb_sim_create_local(const kb_config* cfg, int32_t shards, kb_sim** out) {
  if (!cfg || !out || shards < 1 || shards > (int)XMAX) { seterr("shards out of range (1..8)"); return KB_INVALID_ARGUMENT; }
  kb_sim* g = new kb_sim();
  g->cfg = *cfg; g->C = cfg->capacity; g->world = shards; g->R = 0;
  g->hub = new LocalHub(shards);
  const bool sparse = cfg->abi_version == KB_ABI_VERSION && (cfg->variant & KB_VARIANT_SPARSE_ROWS);
  for (int k = 0; k < shards; ++k) {
    LocalXfer* x = new LocalXfer();
    x->rank = k; x->world = shards; x->hub = g->hub;
    kb_sim* s = nullptr;
    const int rc = sparse ? sp_wrap(cfg, k, shards, x, &s) : create_shard(cfg, k, shards, x, &s);
    if (rc) { for (kb_sim* t : g->shards) destroy_one(t); delete g->hub; delete g; return rc; }
    s->in_group = true;
    if (s->sp) s->sp->in_group = true;
    g->shards.push_back(s);
  }
  g->device = g->shards[0]->device;
  *out = g;
  return KB_OK;
}

extern "C" int kb_sim_destroy(kb_sim* s) {
  if (!s) return KB_INVALID_ARGUMENT;
  if (s->sp) { destroy_one(s); return KB_OK; }
  if (!s->shards.empty()) {
    for (kb_sim* t : s->shards) destroy_one(t);
    delete s->hub;
    delete s;
    return KB_OK;
  }
  destroy_shard(s);
  return KB_OK;
}

extern "C" int kb_sim_shard_info(kb_sim* s, int32_t* rank, int32_t* world, uint32_t* lo, uint32_t* hi) {
  if (s && s->sp && rank && world && lo && hi) { *rank = s->sp->rank; *world = s->sp->world; *lo = s->sp->lo; *hi = s->sp->hi; return KB_OK; }
  if (!s || !rank || !world || !lo || !hi) return KB_INVALID_ARGUMENT;
  if (!s->shards.empty()) { *rank = 0; *world = s->world; *lo = 0; *hi = s->C; return KB_OK; }
  *rank = s->rank; *world = s->world; *lo = s->lo; *hi = s->hi;
  return KB_OK;
}

// Host side of the pinned hand-offs: spin on the mapped sequence word (a stream synchronisation would
// pay an interrupt wake-up, tens of microseconds with the GPU idle), with the stream's own status as
// the way out when it drained without publishing (a fault).
static hipError_t sync_st(kb_sim* s) {            // a counted host wait on the simulator's stream
  s->host_syncs++;
  return hipStreamSynchronize(s->st);
}
static int wait_pin(kb_sim* s, uint32_t seq) {
  s->host_syncs++;
  volatile uint32_t* p = s->h_pin + PIN_SEQ;
  for (uint64_t it = 0;; ++it) {
    if (*p == seq) { std::atomic_thread_fence(std::memory_order_acquire); return KB_OK; }
    if ((it & 4095) == 4095) {
      const hipError_t e = hipStreamQuery(s->st);
      if (e == hipSuccess) {
        if (*p == seq) { std::atomic_thread_fence(std::memory_order_acquire); return KB_OK; }
        seterr("stream drained without publishing its results"); return KB_IO_ERROR;
      }
      if (e != hipErrorNotReady) { seterr(std::string("stream: ") + hipGetErrorString(e)); return KB_IO_ERROR; }
    }
  }
}
static int err_status(uint32_t e) {
  if (e) {
    const char* what[] = {"", "suspect slots exhausted", "outbox region overflow", "payload pool overflow",
                          "truncated Join response too large", "inbox overflow", "Join response member count mismatch",
                          "freshness log", "fingerprint count mismatch", "wave-0 outbox exceeds preallocated capacity",
                          "?", "export buffer overflow"};
    seterr(std::string("device capacity error: ") + (e < 12 ? what[e] : "?"));
    return KB_CAPACITY;
  }
  return KB_OK;
}
// replace a tracked device allocation by a larger one (contents are not kept)
template <class T> static hipError_t regrow(kb_sim* s, T** p, size_t n) {
  for (auto& q : s->allocs) if (q == (void*)*p) { (void)hipFree(q); q = nullptr; }
  s->allocs.erase(std::remove(s->allocs.begin(), s->allocs.end(), nullptr), s->allocs.end());
  *p = nullptr;
  return talloc(s, p, n);
}
// The wave-0 outbox holds the round's Join responses (src/kaboodle.rs:356-392), whose volume follows the
// mesh's dynamics (≈1 % of the members answer each joiner with up to 567 ids): when the scanned totals
// exceed it, it grows, with the buffers indexed by its slots (record status, inbox lists, send side).
static int grow_wave0(kb_sim* s, size_t need_msg, size_t need_pay) {
  OutBuf& o0 = s->ob[0];
  s->buf_gen++;                                    // the captured receive window holds the old buffers
  const size_t lim = 0xF0000000ull;
  if (need_pay > o0.pay_cap) {
    const size_t cap = std::min(lim, need_pay + need_pay / 4);
    if (cap < need_pay) { seterr("Join-response payload beyond 2^32 ids"); return KB_CAPACITY; }
    HIPCHK(regrow(s, &o0.pay, cap));
    o0.pay_cap = (uint32_t)cap;
    if (s->xf && cap > s->pay_cap) { HIPCHK(regrow(s, &s->xs.spay, cap + (size_t)s->ucap * s->xs.NWW)); s->pay_cap = (uint32_t)cap; }
  }
  if (need_msg > o0.msg_cap) {
    const size_t cap = std::min(lim, need_msg + need_msg / 4);
    if (cap < need_msg) { seterr("wave-0 records beyond 2^32"); return KB_CAPACITY; }
    HIPCHK(regrow(s, &o0.msgs, cap));
    o0.msg_cap = (uint32_t)cap;
    if (cap > s->msg_cap) {                  // slot-indexed buffers cover the larger outbox
      if (!s->xf) { HIPCHK(regrow(s, &s->wc.status, cap)); HIPCHK(regrow(s, &s->wc.inbox, cap)); HIPCHK(regrow(s, &s->wc.kin, cap)); }
      else { HIPCHK(regrow(s, &s->xs.ostatus, cap)); HIPCHK(regrow(s, &s->xs.smsg, cap + s->ucap)); }
      s->msg_cap = (uint32_t)cap;
    }
  }
  return KB_OK;
}

// External peers' export buffers hold every record a round routes to them.  A real instance's Join
// (kb_sim_inject KB_WIRE_JOIN) draws KnownPeers responses from ~1 % of the running peers, capj ids each
// (src/kaboodle.rs:284-304, :356-392): so before the window the buffers grow to the wave-0 totals (all Join
// responses and injected payloads, an upper bound of what wave 0 can export) plus a fixed allowance for the
// later waves' replies.  They are empty at a round's start (drained after every round), so nothing is copied.
constexpr uint32_t XREC_MIN = 1u << 16, XIDS_MIN = 1u << 22;
static int size_exports(kb_sim* s, uint64_t recs, uint64_t ids) {
  const uint64_t nr = recs + XREC_MIN, ni = ids + XIDS_MIN;
  if (nr > 0xFFFFFFFFull || ni > 0xFFFFFFFFull) { seterr("export buffer beyond 2^32 entries"); return KB_CAPACITY; }
  if (nr > s->d.xrec_cap) { HIPCHK(regrow(s, &s->d.xrec, nr + nr / 4)); s->d.xrec_cap = (uint32_t)std::min<uint64_t>(nr + nr / 4, 0xFFFFFFFFull); s->buf_gen++; }
  if (ni > s->d.xids_cap) { HIPCHK(regrow(s, &s->d.xids, ni + ni / 4)); s->d.xids_cap = (uint32_t)std::min<uint64_t>(ni + ni / 4, 0xFFFFFFFFull); s->buf_gen++; }
  return KB_OK;
}

// grow the receive side of the sharded waves to hold nm records and np payload ids
static int ensure_recv(kb_sim* s, size_t nm, size_t np) {
  if (nm > s->rmsg_cap || !s->rmsg) {
    void* old[] = {s->rmsg, s->rstatus, s->rinbox, s->rkp};
    for (void* p : old) if (p) (void)hipFree(p);
    s->rmsg = nullptr; s->rstatus = nullptr; s->rinbox = nullptr; s->rkp = nullptr;
    const size_t cap = std::max<size_t>(nm + nm / 2, 1u << 16);
    HIPCHK(hipMalloc(&s->rmsg, sizeof(Msg) * cap)); HIPCHK(hipMalloc(&s->rstatus, cap));
    HIPCHK(hipMalloc(&s->rinbox, 4 * cap)); HIPCHK(hipMalloc(&s->rkp, 4 * cap));
    s->rmsg_cap = cap;
    s->wc.status = s->rstatus; s->wc.inbox = s->rinbox; s->wc.kin = s->rkp;
  }
  if (np > s->rpay_cap || !s->rpay) {
    if (s->rpay) (void)hipFree(s->rpay);
    s->rpay = nullptr;
    const size_t cap = std::max<size_t>(np + np / 2, 1u << 20);
    HIPCHK(hipMalloc(&s->rpay, 4 * cap));
    s->rpay_cap = cap;
  }
  return KB_OK;
}

// all-to-all-v of this wave's delivered records; returns the received record count, and
// in `any` whether any rank delivered a record this wave (the same answer on every rank: when no
// record moves, no handler runs and every later wave of the round is empty)
static int exchange_wave(kb_sim* s, OutBuf& ob, uint32_t& nrecv, RecvBlocks& rb, bool& any) {
  const int W = s->world, me = s->rank;
  XState& x = s->xs;
  hipStream_t st = s->st;
  if (x.uon) klaunch(s, KI_XBOUND, k_union_count, dim3(1), dim3(256), 0, x);   // the unions' records, counted
  {
    ScanArgs a = scan_args(s, (uint32_t)W * x.RS, s->scan_tot + 16);
    a.narr = 2;
    a.in[0] = x.xcnt; a.out[0] = x.xoff;
    a.in[1] = x.xpay; a.out[1] = x.xpoff;
    launch_scan(s, a);
  }
  klaunch(s, KI_XBOUND, k_xbound, dim3(1), dim3(64), 0, x, s->scan_tot + 16);
  klaunch(s, KI_PACK, k_pack, dim3((s->R + 3) / 4), dim3(256), 0, s->d, ob, x);
  if (x.uon) klaunch(s, KI_PACK, k_union_pack, dim3(x.nju), dim3(256), 0, x);
  if (!s->xf->allgather_u32(x.xb, s->xall, 2 * W, st)) { seterr(s->xf->error()); return KB_IO_ERROR; }
  k_publish<<<1, 1, 0, st>>>(s->xall, 2 * W * W, s->d_pin, ++s->pin_seq);   // counts -> host, then the wait
  { const int rc = wait_pin(s, s->pin_seq); if (rc) return rc; }
  memcpy(s->h_xall.data(), s->h_pin, 4ull * 2 * W * W);
  size_t sc[XMAX], sd[XMAX], rc[XMAX], rd[XMAX], psc[XMAX], psd[XMAX], prc[XMAX], prd[XMAX];
  size_t so = 0, pso = 0, ro = 0, pro = 0;
  uint64_t total = 0;
  for (int k = 0; k < W * W; ++k) total += s->h_xall[(size_t)(k / W) * 2 * W + (k % W)];
  any = total != 0;
  if (!any) { nrecv = 0; return KB_OK; }
  for (int k = 0; k < W; ++k) {
    sc[k] = s->h_xall[(size_t)me * 2 * W + k]; psc[k] = s->h_xall[(size_t)me * 2 * W + W + k];
    rc[k] = s->h_xall[(size_t)k * 2 * W + me]; prc[k] = s->h_xall[(size_t)k * 2 * W + W + me];
    sd[k] = so; so += sc[k]; psd[k] = pso; pso += psc[k];
    rd[k] = ro; ro += rc[k]; prd[k] = pro; pro += prc[k];
    const uint64_t b = sizeof(Msg) * (uint64_t)sc[k] + 4ull * psc[k];
    s->xbytes_all += b;
    if (k != me) s->xbytes_cross += b;
  }
  int rcode = ensure_recv(s, ro, pro);
  if (rcode) return rcode;
  // records and payload as one grouped exchange; once the group is open it is always closed
  if (!s->xf->group_begin()) { seterr(s->xf->error()); return KB_IO_ERROR; }
  const bool sent = s->xf->alltoallv(x.smsg, sc, sd, s->rmsg, rc, rd, sizeof(Msg), st) &&
                    s->xf->alltoallv(x.spay, psc, psd, s->rpay, prc, prd, 4, st);
  const std::string e1 = sent ? std::string() : s->xf->error();
  if (!s->xf->group_end() || !sent) { seterr(sent ? s->xf->error() : e1); return KB_IO_ERROR; }
  rb.world = (uint32_t)W;
  for (int k = 0; k <= W && k <= (int)XMAX; ++k) {
    rb.m0[k] = k < W ? (uint32_t)rd[k] : (uint32_t)ro;
    rb.p0[k] = k < W ? (uint32_t)prd[k] : (uint32_t)pro;
  }
  nrecv = (uint32_t)ro;
  return KB_OK;
}

// the round's broadcast lists of every shard, concatenated in shard order = sender order; the same
// all-gather carries every rank's error flag (*err = the largest): one host wait per round for both
static int gather_broadcasts(kb_sim* s, uint32_t* err) {
  const int W = s->world;
  hipStream_t st = s->st;
  if (!s->xf->allgather_u32(s->rr, s->xall, 3, st)) { seterr(s->xf->error()); return KB_IO_ERROR; }
  k_publish<<<1, 1, 0, st>>>(s->xall, 3 * W, s->d_pin, ++s->pin_seq);
  { const int rc = wait_pin(s, s->pin_seq); if (rc) return rc; }
  size_t sc[XMAX], sd[XMAX], rc[XMAX], rd[XMAX], fsc[XMAX], frc[XMAX], frd[XMAX];
  size_t oj = 0, of = 0;
  uint32_t e = 0;
  for (int k = 0; k < W; ++k) {
    rc[k] = s->h_pin[3 * k]; frc[k] = s->h_pin[3 * k + 1]; e = std::max(e, s->h_pin[3 * k + 2]);
    rd[k] = oj; oj += rc[k]; frd[k] = of; of += frc[k];
  }
  for (int k = 0; k < W; ++k) { sc[k] = rc[s->rank]; fsc[k] = frc[s->rank]; sd[k] = 0; }
  *err = e;
  if (!s->xf->group_begin()) { seterr(s->xf->error()); return KB_IO_ERROR; }
  const bool sent = s->xf->alltoallv(s->bjoin_loc, sc, sd, s->bjoin, rc, rd, sizeof(BCast), st) &&
                    s->xf->alltoallv(s->bfail_loc, fsc, sd, s->bfail, frc, frd, sizeof(BCast), st);
  const std::string e1 = sent ? std::string() : s->xf->error();
  if (!s->xf->group_end() || !sent) { seterr(sent ? s->xf->error() : e1); return KB_IO_ERROR; }
  s->nj = (uint32_t)oj; s->nf = (uint32_t)of;
  return KB_OK;
}

// The receive window's delivery waves.  rk is the round the kernels take as
// argument; rk < 0 makes them read it from the device (d.ctr[C_ROUND], set by k_log_mark), which lets
// the unsharded window be captured once as a HIP graph and replayed every round.
static int launch_waves(kb_sim* s, int32_t rk) {
  Dev& d = s->d;
  const int32_t r = rk;
  const uint32_t R = s->R;
  hipStream_t st = s->st;
  const uint32_t tb = 256, gnode = (R + tb - 1) / tb;
  int cur = 0;
  for (uint32_t w = 0; w <= s->cfg.max_waves; ++w) {
    OutBuf& ob = s->ob[cur];
    OutBuf& nb = s->ob[cur ^ 1];
    const int last = w == s->cfg.max_waves;
    d.wave = (int32_t)w;                               // latency clock of the wave's prologues
    s->cur_wave = (int)w;
    OutBuf ib = ob;                                    // the wave's delivered records
    uint32_t nrecv = 0;
    if (!s->xf) {
      klaunch(s, KI_ROUTE, k_route, dim3(gnode), dim3(tb), 0, d, ob, s->wc, r, w, last);
      if (last) break;
    } else {
      HIPCHK(hipMemsetAsync(s->xs.xcnt, 0, 4ull * s->world * s->xs.RS, st));
      HIPCHK(hipMemsetAsync(s->xs.xpay, 0, 4ull * s->world * s->xs.RS, st));
      // wave 0: the round's joiners' slots for the Join-response unions
      s->xs.nju = w == 0 && !last ? std::min<uint32_t>(s->nj, s->ucap) : 0u;
      s->xs.uon = s->xs.nju && !(d.dbg & KB_DBG_NO_UNION) ? 1u : 0u;
      s->xs.bjoin = s->bjoin;
      if (s->xs.uon) klaunch(s, KI_ROUTE_X, k_union_slots, dim3((s->xs.nju + 255) / 256), dim3(256), 0, s->xs);
      klaunch(s, KI_ROUTE_X, k_route_x, dim3(gnode), dim3(tb), 0, d, ob, s->xs, r, w, last);
      if (last) break;
      RecvBlocks rb;
      memset(&rb, 0, sizeof rb);
      bool any = true;
      int rc = exchange_wave(s, ob, nrecv, rb, any);
      s->xs.uon = 0;
      if (rc) return rc;
      if (!any) break;                                 // no record anywhere: the rest of the round's waves are empty
      ib.msgs = s->rmsg; ib.pay = s->rpay;
      if (nrecv) klaunch(s, KI_ROUTE_RECV, k_route_recv, dim3((nrecv + 255) / 256), dim3(256), 0, d, ib, s->wc, rb, nrecv);
    }
    {
      ScanArgs a = scan_args(s, R, s->scan_tot + 8);
      a.narr = 4;
      a.in[0] = L(s, s->wc.cnt1); a.out[0] = L(s, s->wc.in_off);
      a.in[1] = L(s, s->wc.bnd); a.out[1] = L(s, nb.off);
      a.in[2] = L(s, s->wc.bpay); a.out[2] = L(s, nb.poff);
      a.in[3] = L(s, s->wc.kcnt); a.out[3] = L(s, s->wc.koff);
      a.list = s->wc.active; a.list_count = d.ctr + C_ACTIVE; a.list_base = s->lo; a.list_or3 = 1;
      launch_scan(s, a);
    }
    if (s->debug_waves) {                               // KB_DEBUG_WAVES: inbox sizes per wave
      std::vector<uint32_t> c1(R);
      HIPCHK(hipMemcpyAsync(c1.data(), L(s, s->wc.cnt1), 4ull * R, hipMemcpyDeviceToHost, st));
      HIPCHK(hipStreamSynchronize(st));
      uint64_t sum = 0; uint32_t mx = 0, arg = 0, big = 0;
      for (uint32_t k = 0; k < R; ++k) { sum += c1[k]; if (c1[k] > mx) { mx = c1[k]; arg = s->lo + k; } big += c1[k] > 64; }
      fprintf(stderr, "[kb] round %d wave %u: in-order msgs %llu, max inbox %u (node %u), inboxes > 64: %u\n", r, w,
              (unsigned long long)sum, mx, arg, big);
    }
    // (the inbox placement, and in PROBE_GROUPS more workgroups the KPR oversize probe)
    if (!s->xf) klaunch(s, KI_SCATTER, k_scatter, dim3(gnode + PROBE_GROUPS), dim3(tb), 0, d, ob, s->wc, r, gnode);
    else if (nrecv) {
      const uint32_t nsc = (nrecv + 255) / 256;
      klaunch(s, KI_SCATTER_FLAT, k_scatter_flat, dim3(nsc + PROBE_GROUPS), dim3(256), 0, d, ib, s->wc, nrecv, r, nsc);
    }
    if (s->debug_waves) {
      HIPCHK(hipMemsetAsync(d.ctr + C_DBG_INS, 0, 52, st));
      HIPCHK(hipMemsetAsync(d.ctr + C_DBG_SLOW_LONG, 0, 20, st));
    }
    {  // the KnownPeers groups: BIG ones KP_COLS workgroups per destination group (one per column part),
       // then the small ones (a wave per destination), which also set up nb.cap / nb.cnt
      const uint32_t ks = (d.NWR <= KP_LDS_WORDS && !(d.dbg & KB_DBG_KP_HBM)) ? KP_COLS : 1u;
      const uint32_t groups = std::max<uint32_t>(1u, std::min<uint32_t>((R + 1023) / 1024 * (ks > 1 ? 2u : 1u), 512u / ks));
      constexpr uint32_t KB_KPS_PER_CU = 1;        // small-group workgroups per CU (2: no faster, profiles/r04u2_ab_unrolls.txt)
      const uint32_t small = std::max<uint32_t>((R + 1023) / 1024, KB_KPS_PER_CU * s->ncu);
      klaunch(s, KI_KP, k_kp, dim3(ks * groups + small), dim3(1024), (uint32_t)kp_lds_bytes(d.NWR), d, ib, s->wc, r,
              nb, ks * groups);
    }
    // inbox sorts + the KPR oversize probe, and the fast handlers
    klaunch(s, KI_SORTFAST, k_sortfast, dim3(SORT_GROUPS + (R + SORTFAST_T - 1) / SORTFAST_T), dim3(SORTFAST_T), 0, d, ib, nb,
            s->wc, r, s->slow, SORT_GROUPS);
    // persistent: as many workgroups as stay resident (204 VGPRs: 2 waves/SIMD, 2 workgroups per CU).
    // A larger grid only queues workgroups that read the node count and exit, which set a ~40 us floor
    // on the late waves with few nodes.
    klaunch(s, KI_PROC, k_proc, dim3(std::min<uint32_t>(4096, (KB_PROC_WPE > 2 ? KB_PROC_WPE : 2) * s->ncu)), dim3(256), 0, d, ib, nb, s->wc, r, s->slow);
    if (s->debug_waves) {
      uint32_t dbg[13], slow = 0;
      HIPCHK(hipMemcpyAsync(dbg, d.ctr + C_DBG_INS, 52, hipMemcpyDeviceToHost, st));
      HIPCHK(hipMemcpyAsync(&slow, d.ctr + C_SLOW, 4, hipMemcpyDeviceToHost, st));
      HIPCHK(hipStreamSynchronize(st));
      fprintf(stderr, "[kb] round %d wave %u: k_proc nodes %u, prologue inserts %u, fingerprint refreshes %u (max per "
              "node %u), KPR scans %u (log entries %u), incremental bases %u\n", r, w, slow, dbg[0], dbg[1], dbg[2], dbg[3],
              dbg[4], dbg[5]);
      if (d.dev & 256) {
        uint32_t why[5];
        HIPCHK(hipMemcpy(why, d.ctr + C_DBG_SLOW_LONG, 20, hipMemcpyDeviceToHost));
        fprintf(stderr, "[kb] round %d wave %u: to k_proc because inbox > %u: %u, sender not a member: %u, fingerprint stale: %u, "
                "KPR not proven oversize: %u, other: %u\n", r, w, FAST_MAX, why[0], why[1], why[2], why[3], why[4]);
      }
      if (d.dev & 128)
        fprintf(stderr, "[kb] round %d wave %u: k_kp_group BIG workgroup-destinations %u, messages %u: stage+arms %.1f us, "
                "prologues %.1f, write-back+refold %.1f (sums), max total %.1f\n", r, w, dbg[10], dbg[12], dbg[6] * 0.01,
                dbg[8] * 0.01, dbg[9] * 0.01, dbg[7] * 0.01);
      if (d.dev & 64)
        fprintf(stderr, "[kb] round %d wave %u: k_proc node time sum %.1f us (max %.1f), take_base %.1f, insertions %.1f, "
                "start %.1f, end %.1f, messages %u\n", r, w, dbg[6] * 0.01, dbg[7] * 0.01, dbg[8] * 0.01, dbg[9] * 0.01,
                dbg[10] * 0.01, dbg[11] * 0.01, dbg[12]);
    }
    cur ^= 1;
  }
  s->cur_wave = -1;
  return KB_OK;
}

// A restart's map: the old address's row packed on the shard holding it, moved (sharded: an all-to-all-v
// in which only that shard sends, to the shard holding the new row) and unpacked; the event observer
// moves with it (src/lib.rs:104: the map and its observer belong to the Kaboodle, not to its socket).
// *snap_after: an observer attached to the new address before this round (after start() returned) and the
// instance had none: its snapshot is taken from the row once the restart has applied (the caller), so the
// channel reports only later changes, not the whole inherited map
static int move_row(kb_sim* s, uint32_t from, uint32_t to, bool* snap_after) {
  *snap_after = false;
  const RowPack LP = row_pack_layout(s->W, s->d.NWR, s->d.lat != nullptr, s->d.tst != nullptr);
  if (!s->rpack) HIPCHK(hipMalloc(&s->rpack, 4ull * LP.words));
  if (s->xf && !s->rpack_in) HIPCHK(hipMalloc(&s->rpack_in, 4ull * LP.words));
  const bool have = from >= s->lo && from < s->hi, take = to >= s->lo && to < s->hi;
  size_t wk = 0;
  while (wk < s->watch_node.size() && s->watch_node[wk] != from) ++wk;
  const bool watched = have && wk < s->watch_node.size();
  const uint32_t g = (LP.words + 255) / 256 < 1024 ? (LP.words + 255) / 256 : 1024;
  if (have) k_row_pack<<<g, 256, 0, s->st>>>(s->d, from, s->rpack, LP, watched ? s->watch_snap[wk] : nullptr,
                                            watched ? s->watch_fp[wk] : 0u);
  if (watched) { s->watch_node.erase(s->watch_node.begin() + wk); s->watch_fp.erase(s->watch_fp.begin() + wk);
                 s->watch_snap.erase(s->watch_snap.begin() + wk); }
  const uint32_t* src = s->rpack;
  if (s->xf) {
    const int W = s->world, S = (int)s->xs.S;
    const int ofrom = (int)(from / (uint32_t)S), oto = (int)(to / (uint32_t)S);
    size_t sc[XMAX] = {}, sd[XMAX] = {}, rc[XMAX] = {}, rd[XMAX] = {};
    if (s->rank == ofrom) sc[oto] = LP.words;
    if (s->rank == oto) rc[ofrom] = LP.words;
    (void)W;
    if (!s->xf->group_begin()) { seterr(s->xf->error()); return KB_IO_ERROR; }
    const bool sent = s->xf->alltoallv(s->rpack, sc, sd, s->rpack_in, rc, rd, 4, s->st);
    const std::string e1 = sent ? std::string() : s->xf->error();
    if (!s->xf->group_end() || !sent) { seterr(sent ? s->xf->error() : e1); return KB_IO_ERROR; }
    src = s->rpack_in;
  }
  if (!take) return KB_OK;
  uint32_t hdr[RP_HDR];
  HIPCHK(hipMemcpyAsync(hdr, src, sizeof hdr, hipMemcpyDeviceToHost, s->st));
  HIPCHK(sync_st(s));
  uint32_t* snap = nullptr;
  size_t kt = 0;
  while (kt < s->watch_node.size() && s->watch_node[kt] != to) ++kt;
  if (hdr[RP_WATCHED]) {                           // the instance's observer replaces one attached to the new address
    if (kt < s->watch_node.size()) { snap = s->watch_snap[kt]; s->watch_fp[kt] = hdr[RP_WFP]; }
    else {
      HIPCHK(talloc(s, &snap, (size_t)s->d.NWR));
      s->watch_node.push_back(to); s->watch_fp.push_back(hdr[RP_WFP]); s->watch_snap.push_back(snap);
    }
  } else if (kt < s->watch_node.size()) {
    *snap_after = true;
  }
  k_row_unpack<<<g, 256, 0, s->st>>>(s->d, to, src, LP, snap);
  return KB_OK;
}

static int step_round(kb_sim* s) {
  Dev& d = s->d;
  const int32_t r = s->round;
  const uint32_t C = s->C, R = s->R;
  hipStream_t st = s->st;
  const uint32_t tb = 256, gnode = (R + tb - 1) / tb, gwave = (R + 3) / 4, gall = (C + tb - 1) / tb;
  const size_t krec0 = s->krec.size();               // records of earlier rounds (complete)
  s->cur_wave = -1;
  hipEvent_t er[2] = {nullptr, nullptr};              // the whole round, read back next round
  for (int k = 0; k < 2; ++k) {
    if (!s->ev_free.empty()) { er[k] = s->ev_free.back(); s->ev_free.pop_back(); }
    else (void)hipEventCreate(&er[k]);
  }
  (void)hipEventRecord(er[0], st);
  // 0. stamp window
  if (r > 0 && r % EPOCH == 0) klaunch(s, KI_REBASE, k_rebase, dim3(8192), dim3(256), 0, d, r);
  // 1. lifecycle (every shard applies the same events and churn draws to the replicated per-id state)
  if (!s->events.empty()) {
    if (s->events.size() > s->events_cap) {
      if (s->d_events) (void)hipFree(s->d_events);
      s->events_cap = (uint32_t)s->events.size() * 2;
      HIPCHK(hipMalloc(&s->d_events, sizeof(Event) * s->events_cap));
    }
    HIPCHK(hipMemcpyAsync(s->d_events, s->events.data(), sizeof(Event) * s->events.size(), hipMemcpyHostToDevice, st));
    // in call order; a restart first moves the instance's map to its new address (the events before it
    // have been applied: its stop removed the old self), then starts it there
    size_t k0 = 0;
    for (size_t k = 0; k <= s->events.size(); ++k) {
      const bool rs = k < s->events.size() && s->events[k].kind == EV_RESTART;
      if (k == s->events.size() || rs) {
        if (k > k0) klaunch(s, KI_EVENTS, k_events, dim3(1), dim3(1), 0, d, s->d_events + k0, (uint32_t)(k - k0), r);
        k0 = k;
        if (rs) {
          bool snap_after = false;
          const uint32_t to = s->events[k].node;
          const int rc = move_row(s, s->events[k].src, to, &snap_after);
          if (rc) return rc;
          if (snap_after) {                                // the restart itself, then the observer's starting point
            klaunch(s, KI_EVENTS, k_events, dim3(1), dim3(1), 0, d, s->d_events + k, 1u, r);
            size_t kt = 0;
            while (s->watch_node[kt] != to) ++kt;
            k_events_commit<<<(d.NWR + 255) / 256, 256, 0, st>>>(d.bits + (size_t)to * d.NWR, s->watch_snap[kt], d.NWR);
            k0 = k + 1;
          }
        }
      }
    }
    HIPCHK(sync_st(s));
    s->events.clear();
  }
  const bool faults_on = s->cfg.fault_end_round < 0 || r < s->cfg.fault_end_round;
  if (faults_on && s->cfg.churn_threshold) {
    klaunch(s, KI_CHURN_LEAVE, k_churn_leave, dim3(gall), dim3(tb), 0, d, r);
    klaunch(s, KI_CHURN_JOIN, k_churn_join, dim3(1), dim3(64), 0, d, r);
  }
  klaunch(s, KI_LOG_MARK, k_log_mark, dim3(gnode), dim3(tb), 0, d, r);
  // 2. broadcasts of round r-1 (with the external peers' Joins)
  if (!s->inj_join.empty()) { const int rc = merge_ext_joins(st, s->bjoin, &s->nj, s->inj_join, 0, C); if (rc) return rc; }
  OutBuf& o0 = s->ob[0];
  PhaseB pb;
  pb.bfail = s->bfail; pb.nf = s->nf; pb.bjoin = s->bjoin; pb.nj = s->nj; pb.JW = (s->nj + 63) / 64;
  pb.nresp = s->nresp; pb.paysum = s->paysum; pb.nbase = s->nbase;
  if (pb.JW) {
    const size_t words = (size_t)R * pb.JW;
    if (words > s->mask_words) {
      if (s->newmask_base) (void)hipFree(s->newmask_base);
      if (s->respmask_base) (void)hipFree(s->respmask_base);
      s->newmask_base = nullptr; s->respmask_base = nullptr;
      HIPCHK(hipMalloc(&s->newmask_base, 8 * words)); HIPCHK(hipMalloc(&s->respmask_base, 8 * words));
      s->mask_words = words;
    }
    s->newmask = bias(s->newmask_base, pb.JW, s->lo);
    s->respmask = bias(s->respmask_base, pb.JW, s->lo);
  }
  pb.newmask = s->newmask; pb.respmask = s->respmask;
  pb.gid = s->bf_gid; pb.dep = s->bf_dep;
  // latency upkeep for Failed removals; socket_faithful never honours Failed, so nothing to do there
  const bool lat_fail = d.lat && s->nf && d.failed_mode == KB_FAILED_SIM_SENDER;
  pb.fnamed = lat_fail ? s->fnamed : nullptr;
  if (lat_fail) klaunch(s, KI_LAT_MARK, k_lat_mark, dim3((s->nf + 255) / 256), dim3(256), 0, (const BCast*)s->bfail, s->nf, s->fnamed);
  const bool have_b = s->nf + s->nj > 0;
  const bool pb_hbm = (d.dbg & KB_DBG_PHASEB_HBM) != 0;
  if (s->nf > BFAIL_LDS_MAX || (pb_hbm && s->nf)) klaunch(s, KI_BFAIL_PREP, k_bfail_prep, dim3((s->nf + 255) / 256), dim3(256), 0, (const BCast*)s->bfail, s->nf, s->bf_gid, s->bf_dep, d.ctr + C_PATHS);
  else if (s->nf) klaunch(s, KI_BFAIL_PREP, k_bfail_prep_lds, dim3(1), dim3(1024), 0, (const BCast*)s->bfail, s->nf, s->bf_gid, s->bf_dep);
  if (s->debug_waves && s->nf) {                     // KB_DEBUG_WAVES: broadcast list shape
    std::vector<uint8_t> dep(s->nf);
    HIPCHK(hipMemcpyAsync(dep.data(), s->bf_dep, s->nf, hipMemcpyDeviceToHost, st));
    HIPCHK(hipStreamSynchronize(st));
    size_t nd = 0;
    for (uint8_t x : dep) nd += x != 0;
    fprintf(stderr, "[kb] round %d broadcasts: Failed %u (sender named earlier: %zu), Join %u\n", r, s->nf, nd, s->nj);
  }
  {
    // the row pass (broadcast phase + A3 candidates), persistent waves; broadcast lists staged in LDS
    // once per workgroup when they fit.  Its events are taken by its own dispatch packet
    // (hipExtLaunchKernel), so they time the kernel itself.
    const uint32_t budget = RP_LDS_BYTES / 4;          // dynamic LDS words per workgroup
    bool ll = s->nf <= PB_FMAX && s->nj <= PB_JMAX;   // both broadcast lists staged in LDS
    uint32_t listw = ll ? 2 * s->nf + s->nj : 0;
    if (listw > budget / 2 || pb_hbm) { ll = false; listw = 0; }
    // the LDS variant stages each row's whole bitset for the Failed group's membership tests; without a
    // Failed list (quiet rounds: A3 and a few Joins only) the row is read where A3 and the Joins touch it
    // (372K peers, no broadcasts: 3.41 -> 0.54 ms, profiles/r04e_rowpass_variants.json).  (Rows too wide for
    // more than 1-3 staged bitsets per workgroup still stage: the in-place variant with 8 waves per workgroup
    // and the lists in LDS measured 17.4 -> 21.5 ms at 262K peers and 44.7 -> 41.8 ms at 372K in rounds with
    // Failed lists, its random membership reads missing L2, profiles/r04s_nsweep.json)
    const bool ldsb = s->W <= PB_LDS_W && budget - listw >= d.NWR && !pb_hbm && s->nf > 0;
    const uint32_t wpb = ldsb ? std::min<uint32_t>(RP_WAVES, (budget - listw) / d.NWR) : RP_WAVES;
    const size_t lds = 4ull * ((ldsb ? (size_t)wpb * d.NWR : 0) + listw);
    int occ = 0;                                       // resident workgroups per CU (LDS, registers)
    const void* rpk = ldsb ? (ll ? reinterpret_cast<const void*>(&k_rowpass<true, true>) : reinterpret_cast<const void*>(&k_rowpass<true, false>))
                           : (ll ? reinterpret_cast<const void*>(&k_rowpass<false, true>) : reinterpret_cast<const void*>(&k_rowpass<false, false>));
    const uint64_t okey = ((uint64_t)ldsb << 63) | ((uint64_t)ll << 62) | ((uint64_t)wpb << 40) | (uint64_t)lds;   // queried once per shape
    if (okey == s->occ_key) occ = s->occ_val;
    else {
      (void)hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, rpk, (int)(64 * wpb), lds);
      s->occ_key = okey; s->occ_val = occ;
    }
    const uint32_t per_cu = std::max<uint32_t>(1, std::min<uint32_t>(8, (uint32_t)occ));
    const uint32_t blocks = std::min<uint32_t>((R + wpb - 1) / wpb, s->ncu * per_cu);
    if (s->debug_waves && r == 2)
      fprintf(stderr, "[kb] row pass: %u waves/workgroup, %zu B LDS, %u workgroups/CU (lds_per_cu %zu), %u workgroups\n", wpb,
              lds, per_cu, (size_t)s->lds_per_cu, blocks);
    const bool rp_prof = s->debug_waves && (d.dev & 2048);
    if (rp_prof) HIPCHK(hipMemsetAsync(d.ctr + C_DBG_TNODE, 0, 4 * (C_DBG_MSGS - C_DBG_TNODE), st));
    if (ldsb && ll) klaunch(s, KI_ROWPASS, k_rowpass<true, true>, dim3(blocks), dim3(64 * wpb), (uint32_t)lds, d, pb, s->ro, r);
    else if (ldsb) klaunch(s, KI_ROWPASS, k_rowpass<true, false>, dim3(blocks), dim3(64 * wpb), (uint32_t)lds, d, pb, s->ro, r);
    else if (ll) klaunch(s, KI_ROWPASS, k_rowpass<false, true>, dim3(blocks), dim3(64 * wpb), (uint32_t)lds, d, pb, s->ro, r);
    else klaunch(s, KI_ROWPASS, k_rowpass<false, false>, dim3(blocks), dim3(64 * wpb), (uint32_t)lds, d, pb, s->ro, r);
    if (rp_prof) {                                     // KB_DEV=2048: the row pass's phases, summed over its waves
      uint32_t t[13];
      HIPCHK(hipMemcpy(t, d.ctr + C_DBG_INS, 52, hipMemcpyDeviceToHost));
      const double u = 100.0 / ((double)blocks * wpb);   // shares of the summed wall-clock ticks
      double tot = 0;
      for (int k = C_DBG_TNODE; k <= C_DBG_TEND; ++k) if (k != C_DBG_TMAX) tot += t[k - C_DBG_INS];
      const double sc = tot > 0 ? (double)blocks * wpb / tot : 0;   // -> percent
      fprintf(stderr, "[kb] round %d row pass time shares: stage %.1f %%, Failed %.1f %%, Join %.1f %%, A3 %.1f %%, write-back "
              "%.1f %% (%u rows, %u waves)\n", r, t[C_DBG_TSTART - C_DBG_INS] * u * sc, t[C_DBG_TBASE - C_DBG_INS] * u * sc,
              t[C_DBG_TINS - C_DBG_INS] * u * sc, t[C_DBG_TNODE - C_DBG_INS] * u * sc, t[C_DBG_TEND - C_DBG_INS] * u * sc, R,
              blocks * wpb);
    }
  }
  // beside the Join responses: the running set and its fingerprint (read by the tick's agreement count; the
  // set changed last with the churn), and the latency sweep (writes latency entries only; the tick's A2 and
  // the waves write them next)
  side_fork(s, 0);
  klaunch_on(s, s->st2, KI_ALIVE_BITS, k_alive_bits, dim3((d.NWR + tb - 1) / tb), dim3(tb), 0, d);
  klaunch_on(s, s->st2, KI_TRUEFP_PART, k_truefp_part, dim3(TRUEFP_G), dim3(256), 0, d, d.tfpart);
  klaunch_on(s, s->st2, KI_TRUEFP_FIN, k_truefp_fin, dim3(1), dim3(64), 0, d, d.tfpart);
  side_done(s, 0);
  if (lat_fail) {
    klaunch_on(s, s->st2, KI_LAT_SWEEP, k_lat_sweep, dim3((lat_stride(R) / 8 + 255) / 256, std::min<uint32_t>(s->nf, 16384)), dim3(256), 0, d,
            (const BCast*)s->bfail, (const uint32_t*)s->bf_gid, s->nf, s->fnamed);
    side_done(s, 1);
  }
  // the Probes queued since the last round travel with this round's broadcasts (after Failed and Join)
  s->probes.swap(s->probe_q);
  s->probe_q.clear();
  const uint32_t np = (uint32_t)s->probes.size();
  if (np) {
    const size_t need = (size_t)np * R;
    if (need > s->presp_cap) {
      if (s->d_presp) (void)hipFree(s->d_presp);
      s->d_presp = nullptr;
      HIPCHK(hipMalloc(&s->d_presp, sizeof(uint2) * need));
      s->presp_cap = need;
    }
    if (!s->d_presp_n) HIPCHK(hipMalloc(&s->d_presp_n, 4));
    HIPCHK(hipMemsetAsync(s->d_presp_n, 0, 4, st));
    klaunch(s, KI_PROBE, k_probe, dim3(gnode), dim3(tb), 0, d, np, r, s->d_presp, s->d_presp_n, (uint32_t)s->presp_cap);
  }
  // records from external peers (kb_sim_inject): room for their KnownPeers ids in their wave-0 payload regions
  const uint32_t ninj = (uint32_t)s->inj.size();
  bool inj_pay = false;
  if (ninj) {
    if (ninj > s->d_inj_cap) {
      if (s->d_inj) (void)hipFree(s->d_inj);
      s->d_inj_cap = 2 * ninj;
      HIPCHK(hipMalloc(&s->d_inj, sizeof(XRec) * s->d_inj_cap));
    }
    if (s->inj_ids.size() > s->d_inj_ids_cap || !s->d_inj_ids) {
      if (s->d_inj_ids) (void)hipFree(s->d_inj_ids);
      s->d_inj_ids_cap = 2 * s->inj_ids.size() + 16;
      HIPCHK(hipMalloc(&s->d_inj_ids, 4 * s->d_inj_ids_cap));
    }
    HIPCHK(hipMemcpyAsync(s->d_inj, s->inj.data(), sizeof(XRec) * ninj, hipMemcpyHostToDevice, st));
    if (!s->inj_ids.empty()) {
      HIPCHK(hipMemcpyAsync(s->d_inj_ids, s->inj_ids.data(), 4 * s->inj_ids.size(), hipMemcpyHostToDevice, st));
      inj_pay = true;
    }
    klaunch(s, KI_EVENTS, k_inject_prep, dim3(1), dim3(64), 0, d, (const XRec*)s->d_inj, ninj, s->paysum);
  }
  {  // wave-0 outbox regions: responses first, then the tick's messages
    ScanArgs a = scan_args(s, R, s->scan_tot);
    a.narr = 3;
    a.in[0] = L(s, s->nresp); a.out[0] = L(s, s->resp_off);
    a.in[1] = L(s, s->paysum); a.out[1] = L(s, o0.poff);
    a.in[2] = L(s, s->nresp); a.out[2] = L(s, o0.off); a.addc[2] = TICK_MAX;
    a.list = s->resp_nodes; a.list_base = s->lo;
    launch_scan(s, a);
  }
  const bool need_tot = (have_b && s->nj) || inj_pay;
  klaunch(s, KI_SET_CAP, k_set_cap, dim3(gnode), dim3(tb), 0, d, s->nresp, o0.cap, o0.cnt, s->scan_tot, s->d_pin, need_tot ? ++s->pin_seq : 0u);
  if (need_tot) {
    const uint32_t* tot = s->h_pin;                 // written by k_set_cap through the host mapping
    { const int rc = wait_pin(s, s->pin_seq); if (rc) return rc; }
    const uint32_t pay_tot = tot[1], msg_tot = tot[2], resp_nodes = tot[4];
    if (msg_tot > o0.msg_cap || pay_tot > o0.pay_cap) {
      const int rc = grow_wave0(s, msg_tot, pay_tot);
      if (rc) return rc;
    }
    if (s->n_ext) { const int rc = size_exports(s, msg_tot, pay_tot); if (rc) return rc; }
    if (resp_nodes) {
      const uint32_t grid = std::min<uint32_t>(resp_nodes, 4096);   // (the workgroup path: 2 per CU when it serves only
                                                                   // the few responders the wave path lists)
      const size_t words = resp_words(d.NWR, s->W / 256);
      uint32_t* scratch = nullptr;
      size_t lds = 4 * words;
      const bool resp_hbm = s->W > RESP_LDS_W || (d.dbg & KB_DBG_RESP_HBM);
      if (resp_hbm) {
        if (s->resp_scratch_words < words * grid) {
          if (s->resp_scratch) (void)hipFree(s->resp_scratch);
          HIPCHK(hipMalloc(&s->resp_scratch, 4 * words * grid));
          s->resp_scratch_words = words * grid;
        }
        scratch = s->resp_scratch;
        lds = 0;
      }
      // a wave per responder where its LDS slice fits (4 responders per 64 KB workgroup); wider rows keep
      // only the slice's head in LDS and select from the row itself (up to 4 waves per workgroup, as the
      // head fits: 3 at 1M-id rows); else (or forced) a workgroup with HBM scratch
      const size_t wlds = 16ull * rwave_words(d.NWR, s->W / 256);
      const size_t hlds = 4ull * rwave_head(s->W / 256);
      const bool full_on = wlds <= 65536 && !(d.dbg & (KB_DBG_RESP_HBM | KB_DBG_RESP_WAVE_HBM));
      const uint32_t hwaves = (uint32_t)std::min<size_t>(4, 65536 / hlds);
      const bool head_on = !full_on && hwaves >= 1 && !(d.dbg & KB_DBG_RESP_HBM);
      const bool wave_on = full_on || head_on;
      if (s->debug_waves) HIPCHK(hipMemsetAsync(d.ctr + C_DBG_INS, 0, 52, st));
      if (full_on) {                                   // timed by events on its own dispatch packet
        klaunch(s, KI_RESP_WAVE, k_resp_wave<false>, dim3(std::min<uint32_t>((resp_nodes + 3) / 4, 4096)), dim3(256), (uint32_t)wlds, d,
                pb, (const uint32_t*)s->resp_nodes, (const uint32_t*)(s->scan_tot + 4), o0, r, s->slow);
      } else if (head_on) {
        klaunch(s, KI_RESP_WAVE, k_resp_wave<true>, dim3(std::min<uint32_t>((resp_nodes + hwaves - 1) / hwaves, 4096)),
                dim3(64 * hwaves), (uint32_t)(hwaves * hlds), d, pb, (const uint32_t*)s->resp_nodes,
                (const uint32_t*)(s->scan_tot + 4), o0, r, s->slow);
      }
      // the workgroup path serves what the wave path left: its list (in the wave lists' slow buffer, free
      // until the tick) when the wave path ran, else every responder
      klaunch(s, KI_RESP_NODE, k_resp_node, dim3(wave_on ? std::min<uint32_t>(grid, 2 * s->ncu) : grid), dim3(256), (uint32_t)lds, d, pb,
              (const uint32_t*)(wave_on ? s->slow : s->resp_nodes), (const uint32_t*)(wave_on ? d.ctr + C_RESTN : s->scan_tot + 4),
              o0, r, scratch, wave_on);
      if (s->debug_waves && (d.dev & 512)) {
        uint32_t dbg[13];
        HIPCHK(hipMemcpyAsync(dbg, d.ctr + C_DBG_INS, 52, hipMemcpyDeviceToHost, st));
        HIPCHK(hipStreamSynchronize(st));
        fprintf(stderr, "[kb] round %d k_resp_wave: responders %u, responses %u: row staging %.1f us, joiners %.1f, prefix %.1f, "
                "fills %.1f (sums over waves)\n", r, dbg[10], dbg[12], dbg[11] * 0.01, dbg[8] * 0.01, dbg[6] * 0.01, dbg[9] * 0.01);
      }
    }
  }
  // 3. tick
  if (lat_fail) side_join(s, 1);
  klaunch(s, KI_TICK_SCAN, k_tick_scan, dim3(gnode), dim3(tb), 0, d, s->bs, r, s->slow);                       // A1; list the A2 nodes
  klaunch(s, KI_TICK_PRE, k_tick_pre, dim3(std::min<uint32_t>(gwave, 1024)), dim3(256), 0, d, o0, s->bs, r, s->slow);   // A2 per listed node
  // exact A3 order beside the fold: it reads what A2 left (member bits, stamps, instants, bounds) and writes only
  // the five keys and the bounds, which nothing else reads before k_tick_post; the fold and the row fingerprints
  // write checkpoints and fingerprints only
  if (d.tst) {
    side_fork(s, 2);
    const uint32_t kpl = a3_kpl(s->W);
    if (kpl == 2) klaunch_on(s, s->st2, KI_A3_EXACT, k_a3_exact<2>, dim3((R + 3) / 4), dim3(256), 0, d, s->ro.part, r);
    else if (kpl) klaunch_on(s, s->st2, KI_A3_EXACT, k_a3_exact<A3X_KPL>, dim3((R + 3) / 4), dim3(256), 0, d, s->ro.part, r);
    else klaunch_on(s, s->st2, KI_A3_EXACT, k_a3_exact<0>, dim3((R + 3) / 4), dim3(256), 0, d, s->ro.part, r);
    side_done(s, 2);
  }
  // every checkpoint the round's membership changes (broadcasts, A2) made stale is refolded
  if (d.uniform) klaunch(s, KI_FOLD, k_fold, dim3(((R + 63) / 64 + 3) / 4 * s->S), dim3(256), 0, d, FoldArgs{s->S});
  if (d.uniform) klaunch(s, KI_FP_ROWS, k_fp_rows, dim3((FP_LANES * R + tb - 1) / tb), dim3(tb), 0, d);
  side_join(s, 0);
  if (d.tst) side_join(s, 2);
  klaunch(s, KI_TICK_POST, k_tick_post, dim3(gnode), dim3(tb), 0, d, s->ro, o0, r);
  if (ninj) {                                          // the external peers' wave-0 emissions, after the tick's
    klaunch(s, KI_EVENTS, k_inject, dim3(1), dim3(64), 0, d, o0, (const XRec*)s->d_inj, ninj, (const uint32_t*)s->d_inj_ids);
    s->inj.clear(); s->inj_ids.clear();
  }
  {
    ScanArgs a = scan_args(s, R, s->scan_tot);
    a.narr = 2;
    a.in[0] = L(s, s->bs.join); a.out[0] = L(s, s->join_off);
    a.in[1] = L(s, s->bs.nfail); a.out[1] = L(s, s->fail_off);
    launch_scan(s, a);
  }
  klaunch(s, KI_BCAST_WRITE, k_bcast_write, dim3(gnode), dim3(tb), 0, d, s->bs, (const uint32_t*)s->join_off,
          (const uint32_t*)s->fail_off, s->xf ? s->bjoin_loc : s->bjoin, s->xf ? s->bfail_loc : s->bfail);
  // 4. receive window: unicast waves.  Unsharded, the window has no host decision inside it, so with
  // KB_WAVE_GRAPH=1 its ≈ 80 launches are one HIP graph, captured once per buffer generation and
  // replayed each round: that removes host launch gaps in multi-round steps, but the benched one-round
  // steps are GPU-bound and measured no faster, so it is off by default.
  if (!s->xf && !s->debug_waves && s->graph_on) {
    if (!s->wave_exec || s->wave_gen != s->buf_gen) {
      if (s->wave_exec) { (void)hipGraphExecDestroy(s->wave_exec); s->wave_exec = nullptr; }
      if (s->wave_graph) { (void)hipGraphDestroy(s->wave_graph); s->wave_graph = nullptr; }
      HIPCHK(hipStreamBeginCapture(st, hipStreamCaptureModeThreadLocal));
      s->capturing = true;                           // captured launches carry no profile events
      const int rc = launch_waves(s, -1);
      s->capturing = false;
      hipGraph_t g = nullptr;
      const hipError_t e = hipStreamEndCapture(st, &g);
      if (rc) { if (g) (void)hipGraphDestroy(g); return rc; }
      HIPCHK(e);
      s->wave_graph = g;
      HIPCHK(hipGraphInstantiate(&s->wave_exec, g, nullptr, nullptr, 0));
      s->wave_gen = s->buf_gen;
    }
    HIPCHK(hipGraphLaunch(s->wave_exec, st));
  } else {
    const int rc = launch_waves(s, r);
    if (rc) return rc;
  }
  if (s->xf && !s->xf->allreduce_sum_u32(d.ctr + C_AGREE, 1, st)) { seterr(s->xf->error()); return KB_IO_ERROR; }
  klaunch(s, KI_ROUND_END, k_round_end, dim3(1), dim3(1), 0, d, r, (const uint32_t*)s->scan_tot, s->d_pin,
          s->xf ? 0u : ++s->pin_seq, s->rr);
  (void)hipEventRecord(er[1], st);
  s->krec.push_back(kb_sim::KRec{(int16_t)NKI, (int16_t)-1, er[0], er[1]});
  // the earlier rounds' kernel events are complete: read them while this round runs
  prof_resolve(s, krec0);
  uint32_t err = 0;
  if (s->xf) {
    // every shard's broadcast lists and error flag in one all-gather, one host wait
    const int rc = gather_broadcasts(s, &err);
    if (rc) return rc;
  } else {
    // k_round_end wrote the next round's broadcast counts and the error flag straight into the
    // host-mapped pinned buffer; the host polls for them (the stream then drains by itself)
    const int rc = wait_pin(s, s->pin_seq);
    if (rc) return rc;
    s->nj = s->h_pin[0]; s->nf = s->h_pin[1]; err = s->h_pin[2];
  }
  s->bj_total += s->nj; s->bf_total += s->nf;
  if (s->n_ext) {                                      // the round's records to external peers, to the host queue
    uint32_t c[2];
    HIPCHK(hipMemcpy(c, d.ctr + C_XREC, 8, hipMemcpyDeviceToHost));
    const uint32_t nrec = std::min(c[0], d.xrec_cap), nid = std::min(c[1], d.xids_cap);
    std::vector<XRec> v(nrec);
    const size_t base = s->xq_ids.size();
    s->xq_ids.resize(base + nid);
    if (nrec) HIPCHK(hipMemcpy(v.data(), d.xrec, sizeof(XRec) * nrec, hipMemcpyDeviceToHost));
    if (nid) HIPCHK(hipMemcpy(s->xq_ids.data() + base, d.xids, 4ull * nid, hipMemcpyDeviceToHost));
    std::sort(v.begin(), v.end(), [](const XRec& a, const XRec& b) {
      return a.wave != b.wave ? a.wave < b.wave : a.sender != b.sender ? a.sender < b.sender : a.seq < b.seq; });
    for (const XRec& x : v) {
      kb_unicast u;
      memcpy(&u, &x, sizeof u);
      u.pay_off = (uint32_t)(base + x.pay_off);
      s->xq.push_back(u);
    }
    const uint32_t z[2] = {0, 0};
    HIPCHK(hipMemcpy(d.ctr + C_XREC, z, 8, hipMemcpyHostToDevice));
  }
  if (np) {                                          // the round's ProbeResponses, (responder, probe) order
    uint32_t k = 0;
    HIPCHK(hipMemcpy(&k, s->d_presp_n, 4, hipMemcpyDeviceToHost));
    k = std::min<uint32_t>(k, (uint32_t)s->presp_cap);
    std::vector<uint2> v(k);
    if (k) HIPCHK(hipMemcpy(v.data(), s->d_presp, sizeof(uint2) * k, hipMemcpyDeviceToHost));
    std::sort(v.begin(), v.end(), [](const uint2& a, const uint2& b) { return a.x != b.x ? a.x < b.x : a.y < b.y; });
    for (const uint2& q : v) {
      kb_probe_response o;
      memset(&o, 0, sizeof o);
      o.responder = q.x; o.probe = q.y; o.round = r; o.prober = s->probes[q.y];
      o.identity_len = s->h_idlen[q.x];
      memcpy(o.identity, &s->h_ident[(size_t)q.x * MAXID], o.identity_len);
      s->presp.push_back(o);
    }
  }
  s->round = r + 1;
  return err_status(err);                            // shards: the flag of any rank
}

static bool is_group(const kb_sim* s) { return !s->shards.empty(); }
static kb_sim* owner(kb_sim* g, uint32_t node) {                 // the shard holding node's row
  for (kb_sim* t : g->shards) if (node >= t->lo && node < t->hi) return t;
  return nullptr;
}
// a kb_sim_create_local group of sparse-row shards: mesh-changing calls go to every shard, row inspection to the
// shard holding the row, replicated facts to the first shard
static bool sp_grp(const kb_sim* s) { return s && !s->shards.empty() && s->shards[0]->sp; }
#define SPG_ALL(call)                                                     \
  if (sp_grp(s)) {                                                        \
    for (kb_sim* t_ : s->shards) { const int rc_ = call(t_); if (rc_) return rc_; } \
    return KB_OK;                                                         \
  }
#define SPG_OWNER(node, call)                                             \
  if (sp_grp(s)) {                                                        \
    if (node >= s->C) return KB_INVALID_ARGUMENT;                         \
    return call(owner(s, node));                                          \
  }
#define SPG_FIRST(call) if (sp_grp(s)) return call(s->shards[0]);

// every shard of a group steps in its own thread; a failing shard aborts the others' rendezvous
static int group_step(kb_sim* g, uint32_t rounds) {
  const size_t W = g->shards.size();
  std::vector<int> rc(W, KB_OK);
  std::vector<std::string> err(W);
  g->hub->reset();
  std::vector<std::thread> th;
  for (size_t k = 0; k < W; ++k)
    th.emplace_back([&, k] {
      kb_sim* s = g->shards[k];
      (void)hipSetDevice(s->device);
      for (uint32_t q = 0; q < rounds && rc[k] == KB_OK; ++q) rc[k] = s->sp ? sp_step(s->sp, 1) : step_round(s);
      if (rc[k] == KB_OK && !s->sp && sync_st(s) != hipSuccess) { rc[k] = KB_IO_ERROR; g_err = "stream"; }
      if (rc[k] != KB_OK) { err[k] = g_err; g->hub->abort(); }
    });
  for (auto& t : th) t.join();
  int first = KB_OK;
  for (int pass = 0; pass < 2 && first == KB_OK; ++pass)     // the root cause first, released waiters last
    for (size_t k = 0; k < W && first == KB_OK; ++k)
      if (rc[k] != KB_OK && (pass == 1 || err[k].find("aborted by another shard") == std::string::npos)) {
        first = rc[k];
        seterr(err[k]);
      }
  return first;
}

extern "C" int kb_sim_step(kb_sim* s, uint32_t rounds) {
  if (s && s->sp) return sp_step(s->sp, rounds);
  if (!s) return KB_INVALID_ARGUMENT;
  if (is_group(s)) return group_step(s, rounds);
  (void)hipSetDevice(s->device);
  for (uint32_t k = 0; k < rounds; ++k) {
    int rc = step_round(s);
    if (rc) { if (s->xf) s->xf->abort(); return rc; }
  }
  HIPCHK(sync_st(s));                                  // synchronous: the rounds' work has completed on return
  return KB_OK;
}

// ---------------------------------------------------------------------------------- API surface
// Sharded handles: calls that change the mesh (start/stop/set_identity/ping_addrs) are made on every
// shard alike; row inspection is answered by the shard holding the row (KB_INVALID_ARGUMENT on the
// others); kb_sim_stats is a collective over the ranks of kb_sim_create_rank.
static int chk(kb_sim* s, uint32_t node) { return (!s || node >= s->C) ? KB_INVALID_ARGUMENT : KB_OK; }
static int chk_row(kb_sim* s, uint32_t node) {
  if (chk(s, node)) return KB_INVALID_ARGUMENT;
  if (node < s->lo || node >= s->hi) { seterr("the node's row is held by another shard"); return KB_INVALID_ARGUMENT; }
  return KB_OK;
}
static int read_row(kb_sim* s, uint32_t node, std::vector<uint8_t>& rw) {   // canonical bytes (0 = not a member)
  std::vector<uint32_t> bw(s->d.NWR);
  rw.resize(s->C);
  HIPCHK(hipMemcpy(rw.data(), s->d.stamp + (size_t)node * s->W, s->C, hipMemcpyDeviceToHost));
  HIPCHK(hipMemcpy(bw.data(), s->d.bits + (size_t)node * s->d.NWR, 4ull * s->d.NWR, hipMemcpyDeviceToHost));
  for (uint32_t j = 0; j < s->C; ++j) if (!((bw[j >> 5] >> (j & 31)) & 1u)) rw[j] = 0;
  return KB_OK;
}

#define GROUP_ALL(call)                                                   \
  if (is_group(s)) {                                                      \
    for (kb_sim* t_ : s->shards) { const int rc_ = call(t_); if (rc_) return rc_; } \
    return KB_OK;                                                         \
  }
#define GROUP_OWNER(node, call)                                           \
  if (is_group(s)) {                                                      \
    if (chk(s, node)) return KB_INVALID_ARGUMENT;                         \
    return call(owner(s, node));                                          \
  }

// running as the API sees it: the last lifecycle call queued for the node since the last step (they take
// effect at the next round start), else its current state; a queued restart moves the instance away
static int api_running(kb_sim* s, uint32_t node, int* run) {
  for (size_t k = s->events.size(); k-- > 0;) {
    if (s->events[k].node == node) { *run = s->events[k].kind != EV_STOP; return KB_OK; }
    if (s->events[k].kind == EV_RESTART && s->events[k].src == node) { *run = 0; return KB_OK; }
  }
  uint8_t a = 0;
  HIPCHK(hipMemcpy(&a, s->d.alive + node, 1, hipMemcpyDeviceToHost));
  *run = a;
  return KB_OK;
}
// the address has been bound by an instance: it ran (start_round, replicated), or a start of it is queued
static int ever_bound(kb_sim* s, uint32_t node, int* ever) {
  for (const Event& e : s->events) if (e.node == node && e.kind != EV_STOP) { *ever = 1; return KB_OK; }
  int32_t sr = 0;
  HIPCHK(hipMemcpy(&sr, s->d.start_round + node, 4, hipMemcpyDeviceToHost));
  *ever = sr != NONE_ROUND;
  return KB_OK;
}
extern "C" int kb_sim_start_node(kb_sim* s, uint32_t node) {
  if (s && s->sp) return chk(s, node) ? KB_INVALID_ARGUMENT : sp_start_node(s->sp, node);
  SPG_ALL([&](kb_sim* t) { return kb_sim_start_node(t, node); });
  if (chk(s, node)) return KB_INVALID_ARGUMENT;
  kb_sim* h = is_group(s) ? s->shards[0] : s;        // lifecycle facts are replicated on every shard
  int run = 0, ever = 0;
  { int rc = api_running(h, node, &run); if (!rc) rc = ever_bound(h, node, &ever); if (rc) return rc; }
  if (!run && ever) { seterr("a stopped instance restarts at a fresh address (kb_sim_restart_node)"); return KB_INVALID_OPERATION; }
  GROUP_ALL([&](kb_sim* t) { t->events.push_back(Event{node, EV_START, node, 0}); return KB_OK; });
  s->events.push_back(Event{node, EV_START, node, 0});
  return KB_OK;
}
extern "C" int kb_sim_stop_node(kb_sim* s, uint32_t node) {
  if (s && s->sp) return chk(s, node) ? KB_INVALID_ARGUMENT : sp_stop_node(s->sp, node);
  SPG_ALL([&](kb_sim* t) { return kb_sim_stop_node(t, node); });
  if (chk(s, node)) return KB_INVALID_ARGUMENT;
  GROUP_ALL([&](kb_sim* t) { return kb_sim_stop_node(t, node); });
  s->events.push_back(Event{node, EV_STOP, node, 0});
  return KB_OK;
}
// Kaboodle::start of the instance at `node` (include/kaboodle_sim.h): a stopped instance that ran comes
// back at the next fresh id, allocated now (the churn reserve's counter, replicated on every shard)
static int restart_apply(kb_sim* s, uint32_t node, uint32_t to) {
  const int pl = s->h_pendlen[node];
  const uint8_t* src = pl >= 0 ? &s->h_pend[(size_t)node * MAXID] : &s->h_ident[(size_t)node * MAXID];
  const uint32_t len = pl >= 0 ? (uint32_t)pl : s->h_idlen[node];
  memmove(&s->h_ident[(size_t)to * MAXID], src, len);
  s->h_idlen[to] = (uint8_t)len;
  s->h_pendlen[node] = -1; s->h_pendlen[to] = -1;
  const int rc = upload_segments(s);
  if (rc) return rc;
  s->buf_gen++;                                    // a captured receive window holds the old Dev (uniform)
  const uint32_t nf = to + 1;
  HIPCHK(hipMemcpy(s->d.ctr + C_NEXTFREE, &nf, 4, hipMemcpyHostToDevice));
  s->events.push_back(Event{to, EV_RESTART, node, 0});
  s->h_moved[node] = 1;
  return KB_OK;
}
extern "C" int kb_sim_restart_node(kb_sim* s, uint32_t node, uint32_t* new_node) {
  if (s && s->sp) return (chk(s, node) || !new_node) ? KB_INVALID_ARGUMENT : sp_restart_node(s->sp, node, new_node);
  if (sp_grp(s)) {                                   // every shard allocates the same fresh id (replicated counter)
    if (chk(s, node) || !new_node) return KB_INVALID_ARGUMENT;
    for (size_t k = 0; k < s->shards.size(); ++k) {
      uint32_t to = 0;
      const int rc = kb_sim_restart_node(s->shards[k], node, &to);
      if (rc) return rc;
      if (k && to != *new_node) { seterr("shards allocated different fresh ids"); return KB_IO_ERROR; }
      *new_node = to;
    }
    return KB_OK;
  }
  if (chk(s, node) || !new_node) return KB_INVALID_ARGUMENT;
  kb_sim* h = is_group(s) ? s->shards[0] : s;
  if (h->h_moved[node]) { seterr("the instance bound here restarted at a fresh address"); return KB_INVALID_OPERATION; }
  int run = 0, ever = 0;
  { int rc = api_running(h, node, &run); if (!rc) rc = ever_bound(h, node, &ever); if (rc) return rc; }
  if (run) { *new_node = node; return KB_OK; }
  if (!ever) {
    *new_node = node;
    GROUP_ALL([&](kb_sim* t) { t->events.push_back(Event{node, EV_START, node, 0}); return KB_OK; });
    s->events.push_back(Event{node, EV_START, node, 0});
    return KB_OK;
  }
  uint32_t nf = 0;
  HIPCHK(hipMemcpy(&nf, h->d.ctr + C_NEXTFREE, 4, hipMemcpyDeviceToHost));
  for (; nf < s->C; ++nf) {                          // the next fresh id: never bound, no identity set
    int ev = 0;
    const int rc = ever_bound(h, nf, &ev);
    if (rc) return rc;
    if (!ev && !h->h_idset[nf]) break;
  }
  if (nf >= s->C) { seterr("no fresh address left for the restart (capacity)"); return KB_CAPACITY; }
  *new_node = nf;
  GROUP_ALL([&](kb_sim* t) { (void)hipSetDevice(t->device); return restart_apply(t, node, nf); });
  return restart_apply(s, node, nf);
}
extern "C" int kb_sim_is_running(kb_sim* s, uint32_t node, int* running) {
  if (s && s->sp) return (chk(s, node) || !running) ? KB_INVALID_ARGUMENT : sp_is_running(s->sp, node, running);
  SPG_FIRST([&](kb_sim* t) { return kb_sim_is_running(t, node, running); });
  if (chk(s, node) || !running) return KB_INVALID_ARGUMENT;
  if (is_group(s)) return kb_sim_is_running(s->shards[0], node, running);
  uint8_t a = 0;
  HIPCHK(hipMemcpy(&a, s->d.alive + node, 1, hipMemcpyDeviceToHost));
  *running = a;
  return KB_OK;
}
extern "C" int kb_sim_ping_addrs(kb_sim* s, uint32_t node, const uint32_t* peers, size_t n) {
  if (s && s->sp) return (chk(s, node) || (n && !peers)) ? KB_INVALID_ARGUMENT : sp_ping_addrs(s->sp, node, peers, n);
  SPG_ALL([&](kb_sim* t) { return kb_sim_ping_addrs(t, node, peers, n); });
  if (chk(s, node) || (n && !peers)) return KB_INVALID_ARGUMENT;
  GROUP_OWNER(node, [&](kb_sim* t) { return kb_sim_ping_addrs(t, node, peers, n); });
  for (size_t k = 0; k < n; ++k) if (peers[k] >= s->C) return KB_INVALID_ARGUMENT;
  uint8_t a = 0;
  HIPCHK(hipMemcpy(&a, s->d.alive + node, 1, hipMemcpyDeviceToHost));
  if (!a) { seterr("Cannot ping while we are not started"); return KB_INVALID_OPERATION; }
  if (node < s->lo || node >= s->hi) return KB_OK;              // queued by the shard holding the row
  uint32_t qn = 0;
  HIPCHK(hipMemcpy(&qn, s->d.paq_n + node, 4, hipMemcpyDeviceToHost));
  std::vector<uint32_t> q(PAQ), bw(s->d.NWR);
  HIPCHK(hipMemcpy(q.data(), s->d.paq + (size_t)node * PAQ, 4 * PAQ, hipMemcpyDeviceToHost));
  HIPCHK(hipMemcpy(bw.data(), s->d.bits + (size_t)node * s->d.NWR, 4ull * s->d.NWR, hipMemcpyDeviceToHost));
  for (size_t k = 0; k < n; ++k) {
    if ((bw[peers[k] >> 5] >> (peers[k] & 31)) & 1u) continue;      // already known: skipped (:277-282)
    if (qn == PAQ) { seterr("ping_addrs queue full"); return KB_CAPACITY; }
    q[qn++] = peers[k];
  }
  HIPCHK(hipMemcpy(s->d.paq + (size_t)node * PAQ, q.data(), 4 * PAQ, hipMemcpyHostToDevice));
  HIPCHK(hipMemcpy(s->d.paq_n + node, &qn, 4, hipMemcpyHostToDevice));
  return KB_OK;
}
extern "C" int kb_sim_set_identity(kb_sim* s, uint32_t node, const uint8_t* identity, size_t len) {
  if (s && s->sp) return (chk(s, node) || len > MAXID || (len && !identity)) ? KB_INVALID_ARGUMENT : sp_set_identity(s->sp, node, identity, len);
  SPG_ALL([&](kb_sim* t) { return kb_sim_set_identity(t, node, identity, len); });
  if (chk(s, node) || len > MAXID || (len && !identity)) return KB_INVALID_ARGUMENT;
  GROUP_ALL([&](kb_sim* t) { return kb_sim_set_identity(t, node, identity, len); });
  if (s->h_moved[node]) { seterr("the instance bound here restarted at a fresh address"); return KB_INVALID_OPERATION; }
  int run = 0, ever = 0;
  { int rc = api_running(s, node, &run); if (!rc) rc = ever_bound(s, node, &ever); if (rc) return rc; }
  if (run) { seterr("Cannot change identity while the mesh is running; call .stop first"); return KB_INVALID_OPERATION; }
  if (len != s->cfg.id_len && s->C > 200) { seterr("non-uniform identity length needs capacity <= 200"); return KB_INVALID_ARGUMENT; }
  if (ever) {                                      // views keep what the address announced; the instance's
    memcpy(&s->h_pend[(size_t)node * MAXID], identity, len);   // next address takes the new bytes
    s->h_pendlen[node] = (int16_t)len;
    return KB_OK;
  }
  memcpy(&s->h_ident[(size_t)node * MAXID], identity, len);
  s->h_idlen[node] = (uint8_t)len;
  s->h_idset[node] = 1;                            // no longer a fresh id for churn joins and restarts
  { const uint8_t one = 1; HIPCHK(hipMemcpy(s->d.idset + node, &one, 1, hipMemcpyHostToDevice)); }
  int rc = upload_segments(s);
  if (rc) return rc;
  s->buf_gen++;                                    // a captured receive window holds the old Dev (uniform, L)
  k_mark_all_dirty<<<(s->R + 255) / 256, 256, 0, s->st>>>(s->d);
  HIPCHK(hipStreamSynchronize(s->st));
  return KB_OK;
}
extern "C" int kb_sim_identity(kb_sim* s, uint32_t node, uint8_t* buf, size_t cap, size_t* len) {
  if (s && s->sp) return (chk(s, node) || !len) ? KB_INVALID_ARGUMENT : sp_identity(s->sp, node, buf, cap, len);
  SPG_FIRST([&](kb_sim* t) { return kb_sim_identity(t, node, buf, cap, len); });
  if (chk(s, node) || !len) return KB_INVALID_ARGUMENT;
  if (is_group(s)) return kb_sim_identity(s->shards[0], node, buf, cap, len);   // replicated per id
  *len = s->h_idlen[node];
  if (!buf) return KB_OK;
  if (cap < *len) return KB_CAPACITY;
  memcpy(buf, &s->h_ident[(size_t)node * MAXID], *len);
  return KB_OK;
}
// ---- discovery (src/discovery.rs:30-89, src/kaboodle.rs:305-331) ----------------------------------
extern "C" int kb_sim_probe(kb_sim* s, const kb_wire_addr* prober) {
  if (s && s->sp) { if (!prober) return KB_INVALID_ARGUMENT; s->sp->probe_q.push_back(*prober); return KB_OK; }
  SPG_ALL([&](kb_sim* t) { return kb_sim_probe(t, prober); });
  if (!s || !prober) return KB_INVALID_ARGUMENT;
  GROUP_ALL([&](kb_sim* t) { return kb_sim_probe(t, prober); });
  s->probe_q.push_back(*prober);
  return KB_OK;
}
extern "C" int kb_sim_probe_responses(kb_sim* s, kb_probe_response* out, size_t cap, size_t* n) {
  if (s && s->sp) return n ? sp_probe_responses(s->sp, out, cap, n) : KB_INVALID_ARGUMENT;
  if (!s || !n) return KB_INVALID_ARGUMENT;
  if (is_group(s)) {                                 // every shard's responders, merged in canonical order
    std::vector<kb_probe_response> all;
    for (kb_sim* t : s->shards) {
      const std::vector<kb_probe_response>& v = t->sp ? t->sp->presp : t->presp;
      all.insert(all.end(), v.begin(), v.end());
    }
    std::stable_sort(all.begin(), all.end(), [](const kb_probe_response& a, const kb_probe_response& b) {
      return a.round != b.round ? a.round < b.round : a.responder != b.responder ? a.responder < b.responder : a.probe < b.probe;
    });
    *n = all.size();
    if (!out) return KB_OK;
    if (cap < all.size()) return KB_CAPACITY;
    if (!all.empty()) memcpy(out, all.data(), all.size() * sizeof(kb_probe_response));
    for (kb_sim* t : s->shards) { t->presp.clear(); if (t->sp) t->sp->presp.clear(); }
    return KB_OK;
  }
  *n = s->presp.size();
  if (!out) return KB_OK;
  if (cap < s->presp.size()) return KB_CAPACITY;
  if (!s->presp.empty()) memcpy(out, s->presp.data(), s->presp.size() * sizeof(kb_probe_response));
  s->presp.clear();
  return KB_OK;
}
// ---- external peers ------------------------------------------------------------------------
static_assert(sizeof(XRec) == sizeof(kb_unicast), "XRec mirrors kb_unicast");
extern "C" int kb_sim_set_external(kb_sim* s, uint32_t node) {
  if (s && s->sp) return chk(s, node) ? KB_INVALID_ARGUMENT : sp_set_external(s->sp, node);
  SPG_ALL([&](kb_sim* t) { return kb_sim_set_external(t, node); });
  if (chk(s, node)) return KB_INVALID_ARGUMENT;
  kb_sim* h = is_group(s) ? s->shards[0] : s;
  if (h->h_ext.empty()) h->h_ext.assign(s->C, 0);
  if (h->h_ext[node]) return KB_OK;
  int ever = 0;
  { const int rc = ever_bound(h, node, &ever); if (rc) return rc; }
  if (ever) { seterr("an external peer takes an address no instance has bound"); return KB_INVALID_OPERATION; }
  auto one = [&](kb_sim* t) -> int {
    (void)hipSetDevice(t->device);
    if (t->h_ext.empty()) t->h_ext.assign(t->C, 0);
    t->h_ext[node] = 1; t->n_ext++;
    t->h_idset[node] = 1;                            // not a fresh id: churn joins and restarts skip it
    const uint8_t o = 1;
    HIPCHK(hipMemcpy(t->d.ext + node, &o, 1, hipMemcpyHostToDevice));
    HIPCHK(hipMemcpy(t->d.idset + node, &o, 1, hipMemcpyHostToDevice));
    if (!t->d.xrec) {
      t->d.xrec_cap = XREC_MIN; t->d.xids_cap = XIDS_MIN;   // grown per round (size_exports)
      HIPCHK(talloc(t, &t->d.xrec, t->d.xrec_cap)); HIPCHK(talloc(t, &t->d.xids, t->d.xids_cap));
      t->buf_gen++;                                  // a captured receive window holds the old Dev
    }
    return KB_OK;
  };
  if (is_group(s)) { for (kb_sim* t : s->shards) { const int rc = one(t); if (rc) return rc; } return KB_OK; }
  return one(s);
}
extern "C" int kb_sim_inject(kb_sim* s, const kb_unicast* m, const uint32_t* ids) {
  if (s && s->sp) return sp_inject(s->sp, m, ids);
  SPG_ALL([&](kb_sim* t) { return kb_sim_inject(t, m, ids); });
  if (!s || !m || m->sender >= s->C || m->dest >= s->C || (m->kind > K_KPR && m->kind != KB_WIRE_JOIN) || (m->pay_len && !ids))
    return KB_INVALID_ARGUMENT;
  kb_sim* h = is_group(s) ? s->shards[0] : s;
  if (h->h_ext.empty() || !h->h_ext[m->sender]) { seterr("kb_sim_inject: the sender is not an external peer"); return KB_INVALID_OPERATION; }
  if (m->kind == KB_WIRE_JOIN) {                       // a Join broadcast: the next round's Join list
    if (std::find(h->inj_join.begin(), h->inj_join.end(), m->sender) != h->inj_join.end()) {
      seterr("kb_sim_inject: one Join per external peer per round"); return KB_CAPACITY;
    }
    if (is_group(s)) { for (kb_sim* t : s->shards) t->inj_join.push_back(m->sender); }
    else s->inj_join.push_back(m->sender);
    return KB_OK;
  }
  if ((m->kind == K_PINGREQ || m->kind == K_ACK) && m->a >= s->C) return KB_INVALID_ARGUMENT;
  for (uint32_t k = 0; k < m->pay_len; ++k) if (ids[k] >= s->C) return KB_INVALID_ARGUMENT;
  uint32_t per = 0, rel = 0;
  for (const XRec& x : h->inj) if (x.sender == m->sender) { per++; if (x.kind == K_KP) rel += x.pay_len; }
  if (per >= (uint32_t)TICK_MAX) { seterr("kb_sim_inject: 33 records per external peer per round"); return KB_CAPACITY; }
  auto one = [&](kb_sim* t) -> int {
    XRec x{0, 0, m->sender, m->dest, 0, m->kind, m->kind == K_KP ? 0u : m->a, m->fp, m->n, (uint32_t)t->inj_ids.size(),
           m->kind == K_KP ? m->pay_len : 0u, rel};
    if (m->kind == K_KP) t->inj_ids.insert(t->inj_ids.end(), ids, ids + m->pay_len);
    t->inj.push_back(x);
    return KB_OK;
  };
  if (is_group(s)) { for (kb_sim* t : s->shards) one(t); return KB_OK; }
  return one(s);
}
extern "C" int kb_sim_exported(kb_sim* s, kb_unicast* out, size_t cap, size_t* n, uint32_t* ids, size_t cap_ids, size_t* n_ids) {
  if (s && s->sp) return (!n || !n_ids) ? KB_INVALID_ARGUMENT : sp_exported(s->sp, out, cap, n, ids, cap_ids, n_ids);
  if (!s || !n || !n_ids) return KB_INVALID_ARGUMENT;
  std::vector<kb_unicast> all;
  std::vector<uint32_t> all_ids;
  const std::vector<kb_sim*> hs = is_group(s) ? s->shards : std::vector<kb_sim*>{s};
  for (kb_sim* t : hs)
    for (const kb_unicast& u : (t->sp ? t->sp->xq : t->xq)) {
      const std::vector<uint32_t>& xi = t->sp ? t->sp->xq_ids : t->xq_ids;
      kb_unicast v = u;
      v.pay_off = (uint32_t)all_ids.size();
      all_ids.insert(all_ids.end(), xi.begin() + u.pay_off, xi.begin() + u.pay_off + u.pay_len);
      std::sort(all_ids.begin() + v.pay_off, all_ids.end());   // a KnownPeers map has no order: ascending ids
      all.push_back(v);
    }
  std::stable_sort(all.begin(), all.end(), [](const kb_unicast& a, const kb_unicast& b) {
    return a.round != b.round ? a.round < b.round : a.wave != b.wave ? a.wave < b.wave : a.sender != b.sender ? a.sender < b.sender
                                                                                       : a.seq < b.seq; });
  *n = all.size(); *n_ids = all_ids.size();
  if (!out && !ids) return KB_OK;
  if (cap < all.size() || (!all_ids.empty() && (!ids || cap_ids < all_ids.size()))) { seterr("export buffer too small"); return KB_CAPACITY; }
  if (!all.empty()) memcpy(out, all.data(), all.size() * sizeof(kb_unicast));
  if (!all_ids.empty()) memcpy(ids, all_ids.data(), 4 * all_ids.size());
  for (kb_sim* t : hs) { t->xq.clear(); t->xq_ids.clear(); if (t->sp) { t->sp->xq.clear(); t->sp->xq_ids.clear(); } }
  return KB_OK;
}

// the last round's Join / Failed broadcasts (whole mesh; sender order, a node's Join before its Failed)
extern "C" int kb_sim_broadcasts(kb_sim* s, kb_broadcast* out, size_t cap, size_t* n) {
  if (s && s->sp) return n ? sp_broadcasts(s->sp, out, cap, n) : KB_INVALID_ARGUMENT;
  SPG_FIRST([&](kb_sim* t) { return kb_sim_broadcasts(t, out, cap, n); });
  if (!s || !n) return KB_INVALID_ARGUMENT;
  if (is_group(s)) return kb_sim_broadcasts(s->shards[0], out, cap, n);   // every shard holds the lists
  std::vector<BCast> j(s->nj), f(s->nf);
  if (s->nj) HIPCHK(hipMemcpy(j.data(), s->bjoin, sizeof(BCast) * s->nj, hipMemcpyDeviceToHost));
  if (s->nf) HIPCHK(hipMemcpy(f.data(), s->bfail, sizeof(BCast) * s->nf, hipMemcpyDeviceToHost));
  size_t c = 0, a = 0, b = 0;
  while (a < j.size() || b < f.size()) {
    const bool tj = b == f.size() || (a < j.size() && j[a].sender <= f[b].sender);
    if (out && c < cap) {
      kb_broadcast& o = out[c];
      memset(&o, 0, sizeof o);
      if (tj) { o.kind = KB_WIRE_JOIN; o.sender = j[a].sender; o.peer = j[a].peer; }
      else { o.kind = KB_WIRE_FAILED; o.sender = f[b].sender; o.peer = f[b].peer; }
    }
    if (tj) a++; else b++;
    c++;
  }
  *n = c;
  return (out && cap < c) ? KB_CAPACITY : KB_OK;
}
extern "C" int kb_sim_fingerprint(kb_sim* s, uint32_t node, uint32_t* fp) {
  if (s && s->sp) return (chk(s, node) || !fp) ? KB_INVALID_ARGUMENT : sp_fingerprint(s->sp, node, fp);
  SPG_OWNER(node, [&](kb_sim* t) { return kb_sim_fingerprint(t, node, fp); });
  if (chk(s, node) || !fp) return KB_INVALID_ARGUMENT;
  GROUP_OWNER(node, [&](kb_sim* t) { return kb_sim_fingerprint(t, node, fp); });
  if (chk_row(s, node)) return KB_INVALID_ARGUMENT;
  k_fp_one<<<1, 64, 0, s->st>>>(s->d, node);
  HIPCHK(hipMemcpyAsync(fp, s->d.fp + node, 4, hipMemcpyDeviceToHost, s->st));
  HIPCHK(hipStreamSynchronize(s->st));
  return KB_OK;
}
// all ids; 0 for non-running ids and (sharded ranks) for rows held by other shards
extern "C" int kb_sim_fingerprints(kb_sim* s, uint32_t* fps, size_t cap) {
  if (s && s->sp) return (!fps || cap < s->C) ? KB_INVALID_ARGUMENT : sp_fingerprints(s->sp, fps);
  if (!s || !fps || cap < s->C) return KB_INVALID_ARGUMENT;
  if (is_group(s)) {
    std::vector<uint32_t> part(s->C);
    memset(fps, 0, 4ull * s->C);
    for (kb_sim* t : s->shards) {
      const int rc = kb_sim_fingerprints(t, part.data(), part.size());
      if (rc) return rc;
      for (uint32_t j = t->lo; j < t->hi; ++j) fps[j] = part[j];
    }
    return KB_OK;
  }
  k_fp_all<<<(s->R + 3) / 4, 256, 0, s->st>>>(s->d);
  std::vector<uint8_t> al(s->C);
  memset(fps, 0, 4ull * s->C);
  HIPCHK(hipMemcpyAsync(fps + s->lo, s->d.fp + s->lo, 4ull * s->R, hipMemcpyDeviceToHost, s->st));
  HIPCHK(hipMemcpyAsync(al.data(), s->d.alive, s->C, hipMemcpyDeviceToHost, s->st));
  HIPCHK(hipStreamSynchronize(s->st));
  for (uint32_t i = 0; i < s->C; ++i) if (!al[i]) fps[i] = 0;
  return KB_OK;
}
extern "C" int kb_sim_true_fingerprint(kb_sim* s, uint32_t* fp) {
  if (s && s->sp) return fp ? sp_true_fingerprint(s->sp, fp) : KB_INVALID_ARGUMENT;
  SPG_FIRST([&](kb_sim* t) { return kb_sim_true_fingerprint(t, fp); });
  if (!s || !fp) return KB_INVALID_ARGUMENT;
  if (is_group(s)) return kb_sim_true_fingerprint(s->shards[0], fp);
  k_alive_bits<<<(s->d.NWR + 255) / 256, 256, 0, s->st>>>(s->d);
  k_truefp_part<<<TRUEFP_G, 256, 0, s->st>>>(s->d, s->d.tfpart);
  k_truefp_fin<<<1, 64, 0, s->st>>>(s->d, s->d.tfpart);
  HIPCHK(hipMemsetAsync(s->d.ctr + C_ALIVE, 0, 4, s->st));
  HIPCHK(hipMemcpyAsync(fp, s->d.truefp, 4, hipMemcpyDeviceToHost, s->st));
  HIPCHK(hipStreamSynchronize(s->st));
  return KB_OK;
}
extern "C" int kb_sim_dump_row(kb_sim* s, uint32_t node, uint8_t* rw, size_t cap) {
  SPG_OWNER(node, [&](kb_sim* t) { return kb_sim_dump_row(t, node, rw, cap); });
  if (s && s->sp) {
    if (chk(s, node) || !rw || cap < s->C) return KB_INVALID_ARGUMENT;
    std::vector<uint8_t> v;
    const int rc = sp_read_row(s->sp, node, v);
    if (!rc) memcpy(rw, v.data(), s->C);
    return rc;
  }
  if (chk(s, node) || !rw || cap < s->C) return KB_INVALID_ARGUMENT;
  GROUP_OWNER(node, [&](kb_sim* t) { return kb_sim_dump_row(t, node, rw, cap); });
  if (chk_row(s, node)) return KB_INVALID_ARGUMENT;
  std::vector<uint8_t> v;
  int rc = read_row(s, node, v);
  if (rc) return rc;
  memcpy(rw, v.data(), s->C);
  return KB_OK;
}
extern "C" int kb_sim_peers(kb_sim* s, uint32_t node, uint32_t* peers, size_t cap, size_t* n) {
  SPG_OWNER(node, [&](kb_sim* t) { return kb_sim_peers(t, node, peers, cap, n); });
  if (s && s->sp) {
    if (chk(s, node) || !n) return KB_INVALID_ARGUMENT;
    std::vector<uint8_t> rw;
    const int rc = sp_read_row(s->sp, node, rw);
    if (rc) return rc;
    size_t c = 0;
    for (uint32_t j = 0; j < s->C; ++j) if (rw[j]) { if (peers && c < cap) peers[c] = j; c++; }
    *n = c;
    return (peers && cap < c) ? KB_CAPACITY : KB_OK;
  }
  if (chk(s, node) || !n) return KB_INVALID_ARGUMENT;
  GROUP_OWNER(node, [&](kb_sim* t) { return kb_sim_peers(t, node, peers, cap, n); });
  if (chk_row(s, node)) return KB_INVALID_ARGUMENT;
  std::vector<uint8_t> rw;
  int rc = read_row(s, node, rw);
  if (rc) return rc;
  size_t c = 0;
  for (uint32_t j = 0; j < s->C; ++j) if (rw[j]) { if (peers && c < cap) peers[c] = j; c++; }
  *n = c;
  return (peers && cap < c) ? KB_CAPACITY : KB_OK;
}
extern "C" int kb_sim_peer_states(kb_sim* s, uint32_t node, kb_peer_state* out, size_t cap, size_t* n) {
  if (s && s->sp) return (chk(s, node) || !n) ? KB_INVALID_ARGUMENT : sp_peer_states(s->sp, node, out, cap, n);
  SPG_OWNER(node, [&](kb_sim* t) { return kb_sim_peer_states(t, node, out, cap, n); });
  if (chk(s, node) || !n) return KB_INVALID_ARGUMENT;
  GROUP_OWNER(node, [&](kb_sim* t) { return kb_sim_peer_states(t, node, out, cap, n); });
  if (chk_row(s, node)) return KB_INVALID_ARGUMENT;
  std::vector<uint8_t> rw;
  int rc = read_row(s, node, rw);
  if (rc) return rc;
  std::vector<Susp> sl(SLOTS);
  HIPCHK(hipMemcpy(sl.data(), s->d.susp + (size_t)node * SLOTS, sizeof(Susp) * SLOTS, hipMemcpyDeviceToHost));
  std::vector<uint16_t> lat;
  if (s->d.lat) {
    lat.resize(s->C);
    k_lat_column<<<(s->C + 255) / 256, 256, 0, s->st>>>(s->d, node, s->lat_col);
    HIPCHK(hipMemcpyAsync(lat.data(), s->lat_col, 2ull * s->C, hipMemcpyDeviceToHost, s->st));
    HIPCHK(hipStreamSynchronize(s->st));
  }
  const int32_t E = epoch_base(s->round > 0 ? s->round - 1 : 0);
  size_t c = 0;
  for (uint32_t j = 0; j < s->C; ++j) {
    if (!rw[j]) continue;
    if (out && c < cap) {
      kb_peer_state& o = out[c];
      memset(&o, 0, sizeof o);
      o.peer = j;
      o.identity_len = s->h_idlen[j];
      memcpy(o.identity, &s->h_ident[(size_t)j * MAXID], s->h_idlen[j]);
      o.latency_ms = !lat.empty() && lat[j] != LAT_NONE ? lat[j] : KB_LATENCY_NONE;
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
extern "C" int kb_sim_watch(kb_sim* s, uint32_t node) {
  if (s && s->sp) return chk(s, node) ? KB_INVALID_ARGUMENT : sp_watch(s->sp, node);
  SPG_OWNER(node, [&](kb_sim* t) { return kb_sim_watch(t, node); });
  if (chk(s, node)) return KB_INVALID_ARGUMENT;
  GROUP_OWNER(node, [&](kb_sim* t) { return kb_sim_watch(t, node); });
  if (chk_row(s, node)) return KB_INVALID_ARGUMENT;
  for (uint32_t w : s->watch_node) if (w == node) return KB_OK;      // one observer per node
  if (!s->ev_out) HIPCHK(talloc(s, &s->ev_out, 2ull * s->C + 4));
  uint32_t* snap = nullptr;
  HIPCHK(talloc(s, &snap, (size_t)s->d.NWR));
  HIPCHK(hipMemsetAsync(snap, 0, 4ull * s->d.NWR, s->st));          // attached empty, as in Kaboodle::new
  HIPCHK(hipStreamSynchronize(s->st));
  s->watch_node.push_back(node); s->watch_fp.push_back(0); s->watch_snap.push_back(snap);
  return KB_OK;
}
extern "C" int kb_sim_events(kb_sim* s, uint32_t node, uint32_t* discovered, size_t cap_d, size_t* n_d,
                             uint32_t* departed, size_t cap_p, size_t* n_p, uint32_t* fp, int* fp_changed) {
  SPG_OWNER(node, [&](kb_sim* t) {
    return kb_sim_events(t, node, discovered, cap_d, n_d, departed, cap_p, n_p, fp, fp_changed); });
  if (s && s->sp) {
    if (chk(s, node) || !n_d || !n_p || !fp || !fp_changed) return KB_INVALID_ARGUMENT;
    return sp_events(s->sp, node, discovered, cap_d, n_d, departed, cap_p, n_p, fp, fp_changed);
  }
  if (chk(s, node) || !n_d || !n_p || !fp || !fp_changed) return KB_INVALID_ARGUMENT;
  GROUP_OWNER(node, [&](kb_sim* t) {
    return kb_sim_events(t, node, discovered, cap_d, n_d, departed, cap_p, n_p, fp, fp_changed); });
  if (chk_row(s, node)) return KB_INVALID_ARGUMENT;
  size_t k = 0;
  while (k < s->watch_node.size() && s->watch_node[k] != node) ++k;
  if (k == s->watch_node.size()) { seterr("node is not watched (kb_sim_watch)"); return KB_INVALID_OPERATION; }
  const uint32_t* row = s->d.bits + (size_t)node * s->d.NWR;
  uint32_t ctr[3];
  k_events_diff<<<1, 1024, 0, s->st>>>(row, s->watch_snap[k], s->C, s->ev_out);
  k_fp_one<<<1, 64, 0, s->st>>>(s->d, node);
  HIPCHK(hipMemcpyAsync(ctr, s->ev_out + 2ull * s->C, 12, hipMemcpyDeviceToHost, s->st));
  HIPCHK(hipMemcpyAsync(fp, s->d.fp + node, 4, hipMemcpyDeviceToHost, s->st));
  HIPCHK(hipStreamSynchronize(s->st));
  *n_d = ctr[0]; *n_p = ctr[1];
  // the fingerprint batch rule (src/events.rs:103-122): only with a non-empty map, only on change
  *fp_changed = ctr[2] > 0 && *fp != s->watch_fp[k];
  const bool fit = (!ctr[0] || (discovered && cap_d >= ctr[0])) && (!ctr[1] || (departed && cap_p >= ctr[1]));
  if (!fit) {
    if (discovered || departed) { seterr("event buffer too small"); return KB_CAPACITY; }
    return KB_OK;                                                    // size query: nothing drained
  }
  if (ctr[0]) HIPCHK(hipMemcpyAsync(discovered, s->ev_out, 4ull * ctr[0], hipMemcpyDeviceToHost, s->st));
  if (ctr[1]) HIPCHK(hipMemcpyAsync(departed, s->ev_out + s->C, 4ull * ctr[1], hipMemcpyDeviceToHost, s->st));
  k_events_commit<<<(s->d.NWR + 255) / 256, 256, 0, s->st>>>(row, s->watch_snap[k], s->d.NWR);
  HIPCHK(hipStreamSynchronize(s->st));
  if (*fp_changed) s->watch_fp[k] = *fp;
  return KB_OK;
}
// the per-workgroup partial counters (d.sacc) folded into d.stats; the stream is idle afterwards
__global__ __launch_bounds__(256) void k_stats_fold(Dev d) {
  const uint32_t k = blockIdx.x;                   // one counter per workgroup
  unsigned long long t = 0;
  for (uint32_t q = threadIdx.x; q < NACC; q += blockDim.x) {
    unsigned long long& x = d.sacc[(size_t)q * NSTAT + k];
    t += x; x = 0;
  }
  t = block_sum(t);
  if (threadIdx.x == 0 && t) d.stats[k] += t;
}
static int fold_stats(kb_sim* s) {
  if (is_group(s)) { for (kb_sim* t : s->shards) { const int rc = fold_stats(t); if (rc) return rc; } return KB_OK; }
  (void)hipSetDevice(s->device);
  k_stats_fold<<<NSTAT, 256, 0, s->st>>>(s->d);
  HIPCHK(hipStreamSynchronize(s->st));
  return KB_OK;
}
extern "C" int kb_sim_stats(kb_sim* s, kb_stats* out) {
  if (s && s->sp) return out ? sp_stats_out(s->sp, out) : KB_INVALID_ARGUMENT;
  if (sp_grp(s)) {                                   // the counters summed over the shards, replicated facts from one
    if (!out) return KB_INVALID_ARGUMENT;
    unsigned long long st[NSTAT] = {0};
    for (kb_sim* t : s->shards) {
      unsigned long long v[NSTAT];
      const int rc = sp_read_stats(t->sp, v);
      if (rc) return rc;
      for (int k = 0; k < NSTAT; ++k) st[k] += v[k];
    }
    return sp_stats_fill(s->shards[0]->sp, st, out);
  }
  if (!s || !out) return KB_INVALID_ARGUMENT;
  { const int rc = fold_stats(s); if (rc) return rc; }
  unsigned long long st[NSTAT];
  uint32_t ctr[NCTR];
  kb_sim* h = is_group(s) ? s->shards[0] : s;       // replicated facts come from any shard
  if (is_group(s)) {
    memset(st, 0, sizeof st);
    for (kb_sim* t : s->shards) {
      unsigned long long v[NSTAT];
      HIPCHK(hipMemcpy(v, t->d.stats, sizeof v, hipMemcpyDeviceToHost));
      for (int k = 0; k < NSTAT; ++k) st[k] += v[k];
    }
  } else if (s->xf && !s->in_group) {               // ranks: the counters summed over the mesh
    HIPCHK(hipMemcpyAsync(s->xstats, s->d.stats, sizeof st, hipMemcpyDeviceToDevice, s->st));
    if (!s->xf->allreduce_sum_u64(s->xstats, NSTAT, s->st)) { seterr(s->xf->error()); return KB_IO_ERROR; }
    HIPCHK(hipMemcpyAsync(st, s->xstats, sizeof st, hipMemcpyDeviceToHost, s->st));
    HIPCHK(hipStreamSynchronize(s->st));
  } else {
    HIPCHK(hipMemcpy(st, s->d.stats, sizeof st, hipMemcpyDeviceToHost));
  }
  HIPCHK(hipMemcpy(ctr, h->d.ctr, sizeof ctr, hipMemcpyDeviceToHost));
  std::vector<uint8_t> al(h->C);
  HIPCHK(hipMemcpy(al.data(), h->d.alive, h->C, hipMemcpyDeviceToHost));
  memset(out, 0, sizeof *out);
  out->round = h->round;
  uint32_t a = 0;
  for (uint8_t x : al) a += x;
  out->alive = a;
  out->agree = ctr[C_LASTAGREE];
  out->first_converged_round = (int32_t)ctr[C_FIRSTCONV];
  out->last_converged_round = (int32_t)ctr[C_LASTCONV];
  out->next_free_id = ctr[C_NEXTFREE];
  out->sent_ping = st[S_PING]; out->sent_ping_req = st[S_PINGREQ]; out->sent_ack = st[S_ACK];
  out->sent_known_peers = st[S_KP]; out->sent_kpr = st[S_KPR];
  out->bcast_join = h->bj_total; out->bcast_failed = h->bf_total;
  out->drop_dead = st[S_DEAD]; out->drop_loss = st[S_LOSS]; out->drop_window = st[S_WINDOW];
  out->drop_oversize = st[S_OVERSIZE]; out->drop_partition = st[S_PART]; out->drop_bcast = st[S_BDROP];
  out->removed_timeout = st[S_RMTIMEOUT]; out->removed_failed = st[S_RMFAILED]; out->join_responses = st[S_JRESP];
  out->curious_overflow = st[S_CUROVF]; out->churn_leaves = st[S_CLEAVE]; out->churn_joins = st[S_CJOIN];
  out->sent_kp_ids = st[S_KPIDS];
  out->alive_rounds = st[S_ALIVER];
  out->probe_responses = st[S_PROBERESP];
  out->exported = st[S_EXPORT];
  return KB_OK;
}
// per id: alive, n, last_bcast, start_round; n and last_bcast only for the rows this handle holds
extern "C" int kb_sim_dump_scalars(kb_sim* s, int32_t* out, size_t cap) {
  if (s && s->sp) return (!out || cap < 4ull * s->C) ? KB_INVALID_ARGUMENT : sp_dump_scalars(s->sp, out);
  if (!s || !out || cap < 4ull * s->C) return KB_INVALID_ARGUMENT;
  if (is_group(s)) {
    std::vector<int32_t> part(4ull * s->C);
    for (kb_sim* t : s->shards) {
      const int rc = kb_sim_dump_scalars(t, part.data(), part.size());
      if (rc) return rc;
      for (uint32_t i = 0; i < s->C; ++i)
        if ((i >= t->lo && i < t->hi) || t == s->shards[0]) memcpy(out + 4 * i, part.data() + 4 * i, 16);
    }
    return KB_OK;
  }
  std::vector<uint8_t> al(s->C);
  std::vector<uint32_t> n(s->R);
  std::vector<int32_t> lb(s->R), sr(s->C);
  HIPCHK(hipMemcpy(al.data(), s->d.alive, s->C, hipMemcpyDeviceToHost));
  HIPCHK(hipMemcpy(n.data(), L(s, s->d.n), 4ull * s->R, hipMemcpyDeviceToHost));
  HIPCHK(hipMemcpy(lb.data(), L(s, s->d.last_bcast), 4ull * s->R, hipMemcpyDeviceToHost));
  HIPCHK(hipMemcpy(sr.data(), s->d.start_round, 4ull * s->C, hipMemcpyDeviceToHost));
  for (uint32_t i = 0; i < s->C; ++i) {
    const bool loc = i >= s->lo && i < s->hi;
    out[4 * i] = al[i]; out[4 * i + 1] = loc ? (int32_t)n[i - s->lo] : 0;
    out[4 * i + 2] = loc ? lb[i - s->lo] : 0; out[4 * i + 3] = sr[i];
  }
  return KB_OK;
}
extern "C" int kb_sim_dump_suspects(kb_sim* s, uint32_t node, int32_t* out, size_t cap, size_t* n) {
  if (s && s->sp) return (chk(s, node) || !n) ? KB_INVALID_ARGUMENT : sp_dump_suspects(s->sp, node, out, cap, n);
  SPG_OWNER(node, [&](kb_sim* t) { return kb_sim_dump_suspects(t, node, out, cap, n); });
  if (chk(s, node) || !n) return KB_INVALID_ARGUMENT;
  GROUP_OWNER(node, [&](kb_sim* t) { return kb_sim_dump_suspects(t, node, out, cap, n); });
  if (chk_row(s, node)) return KB_INVALID_ARGUMENT;
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
  if (s && s->sp) return (chk(s, node) || !n) ? KB_INVALID_ARGUMENT : sp_dump_curious(s->sp, node, out, cap, n);
  SPG_OWNER(node, [&](kb_sim* t) { return kb_sim_dump_curious(t, node, out, cap, n); });
  if (chk(s, node) || !n) return KB_INVALID_ARGUMENT;
  GROUP_OWNER(node, [&](kb_sim* t) { return kb_sim_dump_curious(t, node, out, cap, n); });
  if (chk_row(s, node)) return KB_INVALID_ARGUMENT;
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
static int kt_kid(int kind) {
  return kind == KB_KT_ROWPASS ? KI_ROWPASS : kind == KB_KT_FOLD ? KI_FOLD : kind == KB_KT_RESP ? KI_RESP_WAVE
       : kind == KB_KT_PROC ? KI_PROC : -1;
}
// the stream is idle: every pending kernel record can be read
static void prof_flush(kb_sim* s) {
  (void)hipSetDevice(s->device);
  if (s->st) (void)hipStreamSynchronize(s->st);
  prof_resolve(s, s->krec.size());
}
extern "C" int kb_sim_kernel_time(kb_sim* s, int kind, double* ms, uint64_t* launches) {
  if (s && s->sp) return (!ms || !launches) ? KB_INVALID_ARGUMENT : sp_kernel_time(s->sp, kind, ms, launches);
  if (!s || !ms || !launches) return KB_INVALID_ARGUMENT;
  if (is_group(s)) return kb_sim_kernel_time(s->shards[0], kind, ms, launches);
  prof_flush(s);
  if (kind == KB_KT_ROUND) { *ms = s->round_ms; *launches = s->round_launches; return KB_OK; }
  const int k = kt_kid(kind);
  if (k < 0) return KB_INVALID_ARGUMENT;
  *ms = s->k_ms[k]; *launches = s->k_n[k];
  return KB_OK;
}
static uint64_t stat_counter(kb_sim* s, int idx) {
  unsigned long long v = 0;
  if (fold_stats(s)) return 0;
  if (hipMemcpy(&v, s->d.stats + idx, 8, hipMemcpyDeviceToHost) != hipSuccess) return 0;
  return v;
}
extern "C" int kb_sim_reset_kernel_time(kb_sim* s) {
  if (s && s->sp) return sp_reset_kernel_time(s->sp);
  if (!s) return KB_INVALID_ARGUMENT;
  GROUP_ALL(kb_sim_reset_kernel_time);
  prof_flush(s);
  s->round_ms = 0; s->round_launches = 0;
  memset(s->k_ms, 0, sizeof s->k_ms); memset(s->k_wms, 0, sizeof s->k_wms); memset(s->k_n, 0, sizeof s->k_n);
  for (int k = 0; k < NKI; ++k) {                   // baselines of the device-side byte counters
    const int b = kbytes_stat(k);
    if (b >= 0) s->k_bytes0[b] = stat_counter(s, b);
  }
  return KB_OK;
}
// algorithmic bytes a kernel moved since the last reset, counted in-kernel; this handle's
// rows: shard 0's for a group, like kb_sim_kernel_time
extern "C" int kb_sim_kernel_bytes(kb_sim* s, int kind, uint64_t* bytes) {
  if (s && s->sp) { if (!bytes) return KB_INVALID_ARGUMENT; *bytes = 0; return KB_INVALID_ARGUMENT; }
  SPG_FIRST([&](kb_sim* t) { return kb_sim_kernel_bytes(t, kind, bytes); });
  if (!s || !bytes) return KB_INVALID_ARGUMENT;
  if (is_group(s)) return kb_sim_kernel_bytes(s->shards[0], kind, bytes);
  const int k = kt_kid(kind), b = k < 0 ? -1 : kbytes_stat(k);
  if (b < 0) return KB_INVALID_ARGUMENT;
  *bytes = stat_counter(s, b) - s->k_bytes0[b];
  return KB_OK;
}
extern "C" int kb_sim_set_profiling(kb_sim* s, int level) {
  if (s && s->sp) { if (level < 0 || level > 2) return KB_INVALID_ARGUMENT; s->sp->prof_level = level; return KB_OK; }
  SPG_ALL([&](kb_sim* t) { return kb_sim_set_profiling(t, level); });
  if (!s || level < 0 || level > 2) return KB_INVALID_ARGUMENT;
  GROUP_ALL([&](kb_sim* t) { return kb_sim_set_profiling(t, level); });
  s->prof_level = level;
  return KB_OK;
}
// every kernel the rounds launched since the last reset: HIP-event time (sum and per delivery wave),
// launches, algorithmic bytes where counted in-kernel; kernels never launched are omitted
extern "C" int kb_sim_kernel_breakdown(kb_sim* s, kb_kernel_time* out, size_t cap, size_t* n) {
  if (s && s->sp) return n ? sp_kernel_breakdown(s->sp, out, cap, n) : KB_INVALID_ARGUMENT;
  if (!s || !n) return KB_INVALID_ARGUMENT;
  if (is_group(s)) return kb_sim_kernel_breakdown(s->shards[0], out, cap, n);
  prof_flush(s);
  size_t c = 0;
  for (int k = 0; k < NKI; ++k) {
    if (!s->k_n[k]) continue;
    if (out && c < cap) {
      kb_kernel_time& o = out[c];
      memset(&o, 0, sizeof o);
      snprintf(o.name, sizeof o.name, "%s", KNAME[k]);
      o.ms = s->k_ms[k]; o.launches = s->k_n[k];
      const int b = kbytes_stat(k);
      o.bytes = b >= 0 ? stat_counter(s, b) - s->k_bytes0[b] : 0;
      o.has_bytes = b >= 0;
      for (int w = 0; w < KB_WAVE_SLOTS; ++w) o.wave_ms[w] = s->k_wms[k][w];
    }
    c++;
  }
  *n = c;
  return (out && cap < c) ? KB_CAPACITY : KB_OK;
}
// host waits on the device since creation (stream synchronisations and pinned hand-offs); for a
// group, the largest over its shards
extern "C" int kb_sim_host_syncs(kb_sim* s, uint64_t* n) {
  if (s && s->sp) { if (!n) return KB_INVALID_ARGUMENT; *n = s->sp->host_syncs; return KB_OK; }
  SPG_FIRST([&](kb_sim* t) { return kb_sim_host_syncs(t, n); });
  if (!s || !n) return KB_INVALID_ARGUMENT;
  if (is_group(s)) {
    uint64_t m = 0;
    for (kb_sim* t : s->shards) m = std::max(m, t->host_syncs);
    *n = m;
    return KB_OK;
  }
  *n = s->host_syncs;
  return KB_OK;
}
// OR of the PATH_* bits (kb_common.h) of the kernel variants that did work since creation
extern "C" int kb_sim_debug_paths(kb_sim* s, uint32_t* mask) {
  if (s && s->sp) { if (!mask) return KB_INVALID_ARGUMENT; *mask = 0; return KB_OK; }
  SPG_FIRST([&](kb_sim* t) { return kb_sim_debug_paths(t, mask); });
  if (!s || !mask) return KB_INVALID_ARGUMENT;
  if (is_group(s)) {
    uint32_t m = 0;
    for (kb_sim* t : s->shards) { uint32_t x = 0; const int rc = kb_sim_debug_paths(t, &x); if (rc) return rc; m |= x; }
    *mask = m;
    return KB_OK;
  }
  HIPCHK(hipMemcpy(mask, s->d.ctr + C_PATHS, 4, hipMemcpyDeviceToHost));
  return KB_OK;
}
// development counters (test surface): [A3 rows scanned, rows scanned past their first chunk, chunks read]
extern "C" int kb_sim_debug_counters(kb_sim* s, uint64_t* out, size_t cap) {
  if (s && s->sp) { if (!out || cap < 3) return KB_INVALID_ARGUMENT; out[0] = out[1] = out[2] = 0; return KB_OK; }
  SPG_FIRST([&](kb_sim* t) { return kb_sim_debug_counters(t, out, cap); });
  if (!s || !out || cap < 3) return KB_INVALID_ARGUMENT;
  kb_sim* h = is_group(s) ? s->shards[0] : s;
  { const int rc = fold_stats(h); if (rc) return rc; }
  unsigned long long v[3];
  HIPCHK(hipMemcpy(v, h->d.stats + S_A3ROWS, sizeof v, hipMemcpyDeviceToHost));
  for (int k = 0; k < 3; ++k) out[k] = v[k];
  if (cap >= 5) {                                    // the row-shard exchange's bytes (sharded meshes; 0 otherwise)
    out[3] = out[4] = 0;
    if (is_group(s)) for (kb_sim* t : s->shards) { out[3] += t->xbytes_cross; out[4] += t->xbytes_all; }
    else { out[3] = s->xbytes_cross; out[4] = s->xbytes_all; }
  }
  return KB_OK;
}
extern "C" int kb_sim_sparse_footprint(kb_sim* s, uint64_t* out, size_t cap) {
  if (!s || !out) return KB_INVALID_ARGUMENT;
  if (sp_grp(s)) {                                   // summed over the shards' rows (the largest row: the max)
    if (cap < 6) return KB_INVALID_ARGUMENT;
    uint64_t t[6];
    memset(out, 0, 6 * sizeof(uint64_t));
    for (kb_sim* sh : s->shards) {
      const int rc = sp_footprint(sh->sp, t, 6);
      if (rc) return rc;
      for (int k = 0; k < 6; ++k) out[k] = k == 3 ? std::max(out[k], t[k]) : out[k] + t[k];
    }
    return KB_OK;
  }
  if (!s->sp) { seterr("not a KB_VARIANT_SPARSE_ROWS handle"); return KB_INVALID_OPERATION; }
  return sp_footprint(s->sp, out, cap);
}
