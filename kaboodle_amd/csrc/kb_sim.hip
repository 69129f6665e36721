// kb_sim.hip — MI355X (gfx950) implementation of the Kaboodle SWIM round as a bulk-synchronous
// simulator over HBM-resident structure-of-arrays tables.  Exposes the C ABI of include/kaboodle_sim.h.
//
// Round pipeline, one HIP stream, one 8-byte host read per round (+1 when broadcasts
// produced Join responses):
//   k_rebase (every 64 rounds)      stamp window shift                             
//   k_events / k_churn_*            Kaboodle::start/stop, churn                    src/lib.rs:136-183
//   k_alive_bits, k_truefp          running set and its fingerprint
//   k_bfail_prep, k_phaseB          handle_incoming_broadcasts (Failed, Join)      src/kaboodle.rs:256-311
//   k_resp_node                     maybe_send_known_peers_to_peer                 src/kaboodle.rs:356-392
//   k_tick_pre                      maybe_broadcast_join + handle_suspected_peers  :228-251, :558-653
//   k_sweep    <- dominant kernel   ping_random_peer row sweep + fingerprint checkpoints :655-703, :71-83
//   k_tick_post                     ping target, handle_incoming_ping_requests     :655-703, :550-556
//   waves: k_route, k_scan_*, k_scatter, k_kp_insert, k_kp_prologue, k_touch_fix, k_proc
//                                   handle_incoming_messages                       src/kaboodle.rs:394-548
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <string.h>
#include <stdlib.h>
#include <string>
#include <vector>
#include <array>
#include <algorithm>
#include "kb_common.h"
#include "kb_round.h"
#include "kb_tick.h"
#include "kb_waves.h"

using namespace kb;

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
__global__ void k_init_nodes(Dev d, uint32_t n0) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= d.C) return;
  d.last_bcast[i] = NONE_ROUND;
  d.start_round[i] = NONE_ROUND;
  if (i < n0) node_start(d, i, 0);
}
__global__ void k_init_converged_rows(Dev d, uint32_t n0) {
  const uint32_t wpr = d.W / 16;
  const size_t words = (size_t)n0 * wpr;
  uint4* p = reinterpret_cast<uint4*>(d.stamp);
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
  const size_t bw = (size_t)n0 * d.NWR;
  for (size_t k = (size_t)blockIdx.x * blockDim.x + threadIdx.x; k < bw; k += (size_t)gridDim.x * blockDim.x) {
    const uint32_t w = (uint32_t)(k % d.NWR);
    uint32_t x = 0;
    if (w * 32 + 32 <= n0) x = 0xFFFFFFFFu;
    else if (w * 32 < n0) x = (1u << (n0 - w * 32)) - 1u;
    d.bits[k] = x;
  }
}
__global__ void k_init_converged_nodes(Dev d, uint32_t n0) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= d.C) return;
  d.last_bcast[i] = NONE_ROUND;
  d.start_round[i] = NONE_ROUND;
  if (i >= n0) return;
  d.alive[i] = 1; d.start_round[i] = 0; d.dirty[i] = 1; d.n[i] = n0; d.last_bcast[i] = -1000; d.paq_n[i] = 0;
  d.sdirty[i] = ~0ull;
}
__global__ void k_mark_all_dirty(Dev d) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < d.C) { d.dirty[i] = 1; d.sdirty[i] = ~0ull; }
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
  const uint32_t i = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (i >= d.C || !d.dirty[i]) return;
  const uint32_t f = wave_fp(d, ztab, i, 0);
  if (lane() == 0) { d.fp[i] = f; d.dirty[i] = 0; }
}

// ================================================================================================
// Host side
// ================================================================================================
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
  uint32_t C, W, S;
  int32_t round;
  std::vector<uint8_t> h_ident, h_idlen, h_ever;
  std::vector<Event> events;
  OutBuf ob[2];
  WaveCtl wc;
  uint32_t msg_cap, pay_cap;
  BCast* bfail; BCast* bjoin;
  uint32_t nf, nj;
  BcastSlots bs;
  uint32_t* join_off; uint32_t* fail_off;
  uint32_t* scan_tot; uint32_t* scan_tiles;
  unsigned long long* newmask; unsigned long long* respmask; size_t mask_words;
  uint32_t* nresp; uint32_t* paysum; uint32_t* nbase; uint32_t* resp_off;
  uint32_t* resp_nodes; uint32_t* bf_gid; uint8_t* bf_dep;
  uint32_t* resp_scratch; size_t resp_scratch_words;
  SweepOut so;
  Event* d_events; uint32_t events_cap;
  hipEvent_t ev0, ev1, er0, er1;
  double sweep_ms, round_ms;
  uint64_t sweep_launches, round_launches, sweep_bytes, bj_total, bf_total;
  uint32_t ncu = 256;
  bool debug_waves = false;
  size_t lds_per_cu = 65536;
};

static ScanArgs scan_args(kb_sim* s, uint32_t n, uint32_t* totals) {
  ScanArgs a; memset(&a, 0, sizeof a); a.n = n; a.totals = totals;
  a.tiles = s->scan_tiles; a.ntiles = (n + 1023) / 1024; return a;
}
static void launch_scan(const ScanArgs& a, hipStream_t st) {
  k_scan_tiles<<<a.ntiles, 1024, 0, st>>>(a);
  k_scan_apply<<<a.ntiles, 1024, 0, st>>>(a);
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
  std::vector<uint32_t> zb(9 * 1024);
  for (uint32_t c = 0; c < 9; ++c)
    for (uint32_t k = 0; k < 4; ++k)
      for (uint32_t v = 0; v < 256; ++v) zb[c * 1024 + k * 256 + v] = multmodp(zpow[c], v << (8 * k));
  HIPCHK(hipMemcpy(s->d.zbtab, zb.data(), 4ull * zb.size(), hipMemcpyHostToDevice));
  const size_t hn = (size_t)(s->W / 8) * 256;
  k_build_htab<<<(unsigned)((hn + 255) / 256), 256>>>(s->d);
  HIPCHK(hipDeviceSynchronize());
  return KB_OK;
}

static void free_all(kb_sim* s) {
  Dev& d = s->d;
  void* ptrs[] = {d.stamp, d.bits, d.segp, d.sdirty, d.dirty, d.alive, d.abits, d.start_round, d.n, d.fp,
                  d.last_bcast, d.susp, d.cur, d.paq, d.paq_n, d.cseg, d.segmul, d.seglen, d.zpow, d.zfin, d.ztab, d.zbtab, d.htab,
                  d.stats, d.ctr, d.truefp, d.flog, d.flog_n, d.fstart, d.kpr_big,
                  s->ob[0].msgs, s->ob[0].pay, s->ob[0].off, s->ob[0].cap, s->ob[0].cnt, s->ob[0].poff,
                  s->ob[1].msgs, s->ob[1].pay, s->ob[1].off, s->ob[1].cap, s->ob[1].cnt, s->ob[1].poff,
                  s->wc.status, s->wc.cnt1, s->wc.bnd, s->wc.bpay, s->wc.cursor, s->wc.in_off, s->wc.inbox,
                  s->wc.active, s->wc.kp_list, s->wc.touched, s->wc.touched_list, s->bfail, s->bjoin, s->bs.join,
                  s->bs.nfail, s->bs.fail, s->join_off, s->fail_off, s->scan_tot, s->scan_tiles, s->newmask,
                  s->respmask, s->nresp, s->paysum, s->nbase, s->resp_off, s->resp_nodes, s->bf_gid, s->bf_dep,
                  s->resp_scratch, s->so.part, s->d_events};
  for (void* p : ptrs) if (p) (void)hipFree(p);
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
  if (cfg->device < 0) (void)hipGetDevice(&s->device);
  if (hipSetDevice(s->device) != hipSuccess) { delete s; seterr("hipSetDevice failed"); return KB_NO_DEVICE; }
  {
    hipDeviceProp_t prop;
    if (hipGetDeviceProperties(&prop, s->device) != hipSuccess) { delete s; seterr("hipGetDeviceProperties failed"); return KB_NO_DEVICE; }
    s->ncu = (uint32_t)prop.multiProcessorCount;
    s->lds_per_cu = prop.maxSharedMemoryPerMultiProcessor ? prop.maxSharedMemoryPerMultiProcessor : 65536;
  }
  const uint32_t C = cfg->capacity;
  const uint32_t W = (C + 8191) / 8192 * 8192;       // 64 segments of whole 128-id steps
  s->C = C; s->W = W; s->round = 0;
  const uint32_t groups = (C + 63) / 64;
  uint32_t S = 1;
  while (S < 64 && groups * S < 8192) S <<= 1;        // enough sweep waves to fill the chip
  s->S = S;
  Dev& d = s->d;
  d.C = C; d.W = W; d.SEGW = W / NSEG; d.NWR = W / 32;
  d.k0 = (uint32_t)cfg->seed; d.k1 = (uint32_t)(cfg->seed >> 32);
  d.loss_thr = cfg->loss_threshold; d.churn_thr = cfg->churn_threshold; d.fault_end = cfg->fault_end_round;
  d.failed_mode = cfg->failed_mode; d.pgroups = cfg->partition_groups; d.pstart = cfg->partition_start;
  d.pend = cfg->partition_end;
  const uint32_t Lid = cfg->id_len;
  d.capk = (BUFSZ - 20 - Lid) / (18 + Lid);           // 20 + L + k(18+L) <= 10240
  d.capj = (BUFSZ - 20 - Lid - 1) / (18 + Lid);       // 20 + L + k(18+L) <  10240
  d.paybound = C < d.capk ? C : d.capk;
  if (const char* ab = getenv("KB_ABLATE")) d.ablate = (uint32_t)atoi(ab);
  s->debug_waves = getenv("KB_DEBUG_WAVES") != nullptr;
  s->h_ident.assign((size_t)C * MAXID, 0); s->h_idlen.assign(C, (uint8_t)Lid); s->h_ever.assign(C, 0);
  for (uint32_t j = 0; j < C; ++j) default_identity(j, Lid, &s->h_ident[(size_t)j * MAXID]);
  for (uint32_t j = 0; j < cfg->initial_nodes; ++j) s->h_ever[j] = 1;
  hipError_t e = hipSuccess;
#define A(ptr, n) if (e == hipSuccess) e = dalloc(&(ptr), (n))
  A(d.stamp, (size_t)C * W); A(d.bits, (size_t)C * d.NWR); A(d.segp, (size_t)C * NSEG); A(d.sdirty, C);
  A(d.dirty, C); A(d.alive, C); A(d.abits, d.NWR); A(d.start_round, C); A(d.n, C); A(d.fp, C);
  A(d.last_bcast, C); A(d.susp, (size_t)C * SLOTS); A(d.cur, (size_t)C * CSLOTS); A(d.paq, (size_t)C * PAQ);
  A(d.paq_n, C); A(d.cseg, C); A(d.segmul, C); A(d.seglen, C); A(d.zpow, (size_t)C + 2); A(d.zfin, (size_t)C + 2); A(d.ztab, 17 * 128); A(d.zbtab, 9 * 1024);
  A(d.htab, (size_t)(W / 8) * 256); A(d.stats, NSTAT); A(d.ctr, NCTR); A(d.truefp, 1);
  A(d.flog, (size_t)C * LOGCAP); A(d.flog_n, C); A(d.fstart, (size_t)C * 16); A(d.kpr_big, C);
  s->msg_cap = std::max<uint32_t>(8u * C + (uint32_t)TICK_MAX * C, 1u << 16);
  s->pay_cap = std::max<uint32_t>((d.capk + 1) * C, 1u << 24);
  for (int b = 0; b < 2; ++b) {
    A(s->ob[b].msgs, s->msg_cap); A(s->ob[b].pay, s->pay_cap); A(s->ob[b].off, C); A(s->ob[b].cap, C);
    A(s->ob[b].cnt, C); A(s->ob[b].poff, C);
    s->ob[b].msg_cap = s->msg_cap; s->ob[b].pay_cap = s->pay_cap;
  }
  A(s->wc.status, s->msg_cap); A(s->wc.cnt1, C); A(s->wc.bnd, C); A(s->wc.bpay, C); A(s->wc.cursor, C);
  A(s->wc.in_off, C); A(s->wc.inbox, s->msg_cap); A(s->wc.active, C); A(s->wc.kp_list, s->msg_cap);
  A(s->wc.touched, C); A(s->wc.touched_list, C);
  A(s->bfail, (size_t)C * SLOTS); A(s->bjoin, C);
  A(s->bs.join, C); A(s->bs.nfail, C); A(s->bs.fail, (size_t)C * SLOTS); A(s->join_off, C); A(s->fail_off, C);
  A(s->scan_tot, 16); A(s->scan_tiles, 5 * ((C + 1023) / 1024) + 5);
  A(s->nresp, C); A(s->paysum, C); A(s->nbase, C); A(s->resp_off, C);
  A(s->resp_nodes, C); A(s->bf_gid, (size_t)C * SLOTS); A(s->bf_dep, (size_t)C * SLOTS);
  A(s->so.part, (size_t)C * S * 10);
#undef A
  if (e != hipSuccess) { seterr(std::string("device allocation failed: ") + hipGetErrorString(e)); free_all(s); delete s; return KB_CAPACITY; }
  s->so.S = S;
  (void)hipMemset(d.kpr_big, 0xFF, 4ull * C);          // no round yet
  s->wc.msg_cap = s->msg_cap; s->wc.pay_cap = s->pay_cap;
  s->newmask = nullptr; s->respmask = nullptr; s->mask_words = 0;
  s->resp_scratch = nullptr; s->resp_scratch_words = 0;
  s->d_events = nullptr; s->events_cap = 0; s->nf = 0; s->nj = 0;
  if (hipStreamCreateWithFlags(&s->st, hipStreamNonBlocking) != hipSuccess) { free_all(s); delete s; seterr("stream"); return KB_IO_ERROR; }
  (void)hipEventCreate(&s->ev0); (void)hipEventCreate(&s->ev1); (void)hipEventCreate(&s->er0); (void)hipEventCreate(&s->er1);
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
    k_init_nodes<<<gb, tb, 0, s->st>>>(d, cfg->initial_nodes);
  }
  if (hipStreamSynchronize(s->st) != hipSuccess) { free_all(s); delete s; seterr("init failed"); return KB_IO_ERROR; }
  *out = s;
  return KB_OK;
}

extern "C" int kb_sim_destroy(kb_sim* s) {
  if (!s) return KB_INVALID_ARGUMENT;
  (void)hipSetDevice(s->device);
  (void)hipStreamSynchronize(s->st);
  free_all(s);
  (void)hipEventDestroy(s->ev0); (void)hipEventDestroy(s->ev1); (void)hipEventDestroy(s->er0); (void)hipEventDestroy(s->er1);
  (void)hipStreamDestroy(s->st);
  delete s;
  return KB_OK;
}

static int check_err(kb_sim* s) {
  uint32_t e = 0;
  HIPCHK(hipMemcpyAsync(&e, s->d.ctr + C_ERR, 4, hipMemcpyDeviceToHost, s->st));
  HIPCHK(hipStreamSynchronize(s->st));
  if (e) {
    const char* what[] = {"", "suspect slots exhausted", "outbox region overflow", "payload pool overflow",
                          "truncated Join response too large", "inbox overflow", "Join response member count mismatch"};
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
  (void)hipEventRecord(s->er0, st);
  // 0. stamp window
  if (r > 0 && r % EPOCH == 0) k_rebase<<<8192, 256, 0, st>>>(d);
  // 1. lifecycle
  if (!s->events.empty()) {
    if (s->events.size() > s->events_cap) {
      if (s->d_events) (void)hipFree(s->d_events);
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
  k_alive_bits<<<(d.NWR + tb - 1) / tb, tb, 0, st>>>(d);
  k_truefp<<<1, 1024, 0, st>>>(d);
  k_log_mark<<<gnode, tb, 0, st>>>(d, r);
  // 2. broadcasts of round r-1
  OutBuf& o0 = s->ob[0];
  PhaseB pb;
  pb.bfail = s->bfail; pb.nf = s->nf; pb.bjoin = s->bjoin; pb.nj = s->nj; pb.JW = (s->nj + 63) / 64;
  pb.nresp = s->nresp; pb.paysum = s->paysum; pb.nbase = s->nbase;
  if (pb.JW) {
    const size_t words = (size_t)C * pb.JW;
    if (words > s->mask_words) {
      if (s->newmask) (void)hipFree(s->newmask);
      if (s->respmask) (void)hipFree(s->respmask);
      s->newmask = nullptr; s->respmask = nullptr;
      HIPCHK(hipMalloc(&s->newmask, 8 * words)); HIPCHK(hipMalloc(&s->respmask, 8 * words));
      s->mask_words = words;
    }
  }
  pb.newmask = s->newmask; pb.respmask = s->respmask;
  pb.gid = s->bf_gid; pb.dep = s->bf_dep;
  const bool have_b = s->nf + s->nj > 0;
  if (s->nf > 2048) k_bfail_prep<<<(s->nf + 255) / 256, 256, 0, st>>>(s->bfail, s->nf, s->bf_gid, s->bf_dep);
  else if (s->nf) k_bfail_prep_lds<<<1, 1024, 0, st>>>(s->bfail, s->nf, s->bf_gid, s->bf_dep);
  if (have_b) {
    // persistent waves; broadcast lists staged in LDS once per workgroup when they fit
    const uint32_t budget = 65536 / 4;                 // dynamic LDS words per workgroup
    uint32_t lf = s->nf <= PB_FMAX, lj = s->nj <= PB_JMAX;
    uint32_t listw = (lf ? 2 * s->nf : 0) + (lj ? s->nj : 0);
    if (listw > budget / 2) { lf = lj = 0; listw = 0; }
    const bool ldsb = s->W <= PB_LDS_W && budget - listw >= d.NWR;
    const uint32_t wpb = ldsb ? std::min<uint32_t>(4, (budget - listw) / d.NWR) : 4;
    const size_t lds = 4ull * ((ldsb ? (size_t)wpb * d.NWR : 0) + listw);
    const uint32_t per_cu = std::max<uint32_t>(1, std::min<uint32_t>(8, (uint32_t)(s->lds_per_cu / std::max<size_t>(lds + 512, 1))));
    const uint32_t blocks = std::min<uint32_t>((C + wpb - 1) / wpb, s->ncu * per_cu);
    if (ldsb) k_phaseB<true><<<blocks, 64 * wpb, lds, st>>>(d, pb, r, lf, lj);
    else k_phaseB<false><<<blocks, 64 * wpb, lds, st>>>(d, pb, r, lf, lj);
  }
  else { HIPCHK(hipMemsetAsync(s->nresp, 0, 4ull * C, st)); HIPCHK(hipMemsetAsync(s->paysum, 0, 4ull * C, st)); }
  {  // wave-0 outbox regions: responses first, then the tick's messages
    ScanArgs a = scan_args(s, C, s->scan_tot);
    a.narr = 3;
    a.in[0] = s->nresp; a.out[0] = s->resp_off;
    a.in[1] = s->paysum; a.out[1] = o0.poff;
    a.in[2] = s->nresp; a.out[2] = o0.off; a.addc[2] = TICK_MAX;
    a.list = s->resp_nodes;
    launch_scan(a, st);
  }
  k_set_cap<<<gnode, tb, 0, st>>>(C, s->nresp, o0.cap, o0.cnt);
  if (have_b && s->nj) {
    uint32_t tot[5];
    HIPCHK(hipMemcpyAsync(tot, s->scan_tot, 20, hipMemcpyDeviceToHost, st));
    HIPCHK(hipStreamSynchronize(st));
    const uint32_t pay_tot = tot[1], msg_tot = tot[2], resp_nodes = tot[4];
    if (msg_tot > s->msg_cap || pay_tot > s->pay_cap) { seterr("wave-0 outbox exceeds preallocated capacity"); return KB_CAPACITY; }
    if (resp_nodes) {
      const uint32_t grid = std::min<uint32_t>(resp_nodes, 4096);
      const size_t words = resp_words(d.NWR, s->W / 256);
      uint32_t* scratch = nullptr;
      size_t lds = 4 * words;
      if (s->W > RESP_LDS_W) {
        if (s->resp_scratch_words < words * grid) {
          if (s->resp_scratch) (void)hipFree(s->resp_scratch);
          HIPCHK(hipMalloc(&s->resp_scratch, 4 * words * grid));
          s->resp_scratch_words = words * grid;
        }
        scratch = s->resp_scratch;
        lds = 0;
      }
      k_resp_node<<<grid, 256, lds, st>>>(d, pb, s->resp_nodes, s->scan_tot + 4, o0, r, scratch);
    }
  }
  // 3. tick
  k_tick_pre<<<gwave, 256, 0, st>>>(d, o0, s->bs, r);
  (void)hipEventRecord(s->ev0, st);
  k_sweep<<<((C + 63) / 64 + 3) / 4 * s->S, 256, 0, st>>>(d, s->so);
  (void)hipEventRecord(s->ev1, st);
  k_tick_post<<<gnode, tb, 0, st>>>(d, s->so, o0, r);
  {
    ScanArgs a = scan_args(s, C, s->scan_tot);
    a.narr = 2;
    a.in[0] = s->bs.join; a.out[0] = s->join_off;
    a.in[1] = s->bs.nfail; a.out[1] = s->fail_off;
    launch_scan(a, st);
  }
  k_bcast_write<<<gnode, tb, 0, st>>>(d, s->bs, s->join_off, s->fail_off, s->bjoin, s->bfail);
  // 4. receive window: unicast waves
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
    if (s->debug_waves) {                               // KB_DEBUG_WAVES: inbox sizes per wave
      std::vector<uint32_t> c1(C);
      HIPCHK(hipMemcpyAsync(c1.data(), s->wc.cnt1, 4ull * C, hipMemcpyDeviceToHost, st));
      HIPCHK(hipStreamSynchronize(st));
      uint64_t sum = 0; uint32_t mx = 0, arg = 0, big = 0;
      for (uint32_t k = 0; k < C; ++k) { sum += c1[k]; if (c1[k] > mx) { mx = c1[k]; arg = k; } big += c1[k] > 64; }
      fprintf(stderr, "[kb] round %d wave %u: in-order msgs %llu, max inbox %u (node %u), inboxes > 64: %u\n", r, w,
              (unsigned long long)sum, mx, arg, big);
    }
    HIPCHK(hipMemcpyAsync(nb.cap, s->wc.bnd, 4ull * C, hipMemcpyDeviceToDevice, st));
    HIPCHK(hipMemsetAsync(nb.cnt, 0, 4ull * C, st));
    k_scatter<<<gnode, tb, 0, st>>>(d, ib, s->wc);
    k_kp_insert<<<2048, 256, 0, st>>>(d, ib, s->wc, r);
    k_kp_prologue<<<1024, 256, 0, st>>>(d, ib, s->wc, r);
    k_touch_fix<<<1024, 256, 0, st>>>(d, s->wc);
    k_sort_inbox<<<256, 1024, 0, st>>>(d, s->wc);
    if (s->debug_waves) HIPCHK(hipMemsetAsync(d.ctr + C_DBG_INS, 0, 12, st));
    k_proc<<<4096, 256, 0, st>>>(d, ib, nb, s->wc, r);
    if (s->debug_waves) {
      uint32_t dbg[3];
      HIPCHK(hipMemcpyAsync(dbg, d.ctr + C_DBG_INS, 12, hipMemcpyDeviceToHost, st));
      HIPCHK(hipStreamSynchronize(st));
      fprintf(stderr, "[kb] round %d wave %u: prologue inserts %u, fingerprint refreshes %u (max per node %u)\n", r, w,
              dbg[0], dbg[1], dbg[2]);
    }
    cur ^= 1;
  }
  k_round_end<<<1, 1, 0, st>>>(d, r);
  (void)hipEventRecord(s->er1, st);
  uint32_t tot[2];
  HIPCHK(hipMemcpyAsync(tot, s->scan_tot, 8, hipMemcpyDeviceToHost, st));
  HIPCHK(hipStreamSynchronize(st));
  s->nj = tot[0]; s->nf = tot[1];
  s->bj_total += s->nj; s->bf_total += s->nf;
  float ms = 0;
  (void)hipEventElapsedTime(&ms, s->ev0, s->ev1); s->sweep_ms += ms; s->sweep_launches++;
  (void)hipEventElapsedTime(&ms, s->er0, s->er1); s->round_ms += ms; s->round_launches++;
  s->round = r + 1;
  return check_err(s);
}

extern "C" int kb_sim_step(kb_sim* s, uint32_t rounds) {
  if (!s) return KB_INVALID_ARGUMENT;
  (void)hipSetDevice(s->device);
  for (uint32_t k = 0; k < rounds; ++k) { int rc = step_round(s); if (rc) return rc; }
  return KB_OK;
}

// ---------------------------------------------------------------------------------- API surface
static int chk(kb_sim* s, uint32_t node) { return (!s || node >= s->C) ? KB_INVALID_ARGUMENT : KB_OK; }
static int read_row(kb_sim* s, uint32_t node, std::vector<uint8_t>& rw) {   // canonical bytes (0 = not a member)
  std::vector<uint32_t> bw(s->d.NWR);
  rw.resize(s->C);
  HIPCHK(hipMemcpy(rw.data(), s->d.stamp + (size_t)node * s->W, s->C, hipMemcpyDeviceToHost));
  HIPCHK(hipMemcpy(bw.data(), s->d.bits + (size_t)node * s->d.NWR, 4ull * s->d.NWR, hipMemcpyDeviceToHost));
  for (uint32_t j = 0; j < s->C; ++j) if (!((bw[j >> 5] >> (j & 31)) & 1u)) rw[j] = 0;
  return KB_OK;
}

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
  std::vector<uint32_t> q(PAQ), bw(s->d.NWR);
  HIPCHK(hipMemcpy(q.data(), s->d.paq + (size_t)node * PAQ, 4 * PAQ, hipMemcpyDeviceToHost));
  HIPCHK(hipMemcpy(bw.data(), s->d.bits + (size_t)node * s->d.NWR, 4ull * s->d.NWR, hipMemcpyDeviceToHost));
  for (size_t k = 0; k < n; ++k) {
    if (peers[k] >= s->C) return KB_INVALID_ARGUMENT;
    if ((bw[peers[k] >> 5] >> (peers[k] & 31)) & 1u) continue;      // already known: skipped (:277-282)
    if (qn == PAQ) { seterr("ping_addrs queue full"); return KB_CAPACITY; }
    q[qn++] = peers[k];
  }
  HIPCHK(hipMemcpy(s->d.paq + (size_t)node * PAQ, q.data(), 4 * PAQ, hipMemcpyHostToDevice));
  HIPCHK(hipMemcpy(s->d.paq_n + node, &qn, 4, hipMemcpyHostToDevice));
  return KB_OK;
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
  k_mark_all_dirty<<<(s->C + 255) / 256, 256, 0, s->st>>>(s->d);
  HIPCHK(hipStreamSynchronize(s->st));
  return KB_OK;
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
  k_alive_bits<<<(s->d.NWR + 255) / 256, 256, 0, s->st>>>(s->d);
  k_truefp<<<1, 1024, 0, s->st>>>(s->d);
  HIPCHK(hipMemsetAsync(s->d.ctr + C_ALIVE, 0, 4, s->st));
  HIPCHK(hipMemcpyAsync(fp, s->d.truefp, 4, hipMemcpyDeviceToHost, s->st));
  HIPCHK(hipStreamSynchronize(s->st));
  return KB_OK;
}
extern "C" int kb_sim_dump_row(kb_sim* s, uint32_t node, uint8_t* rw, size_t cap) {
  if (chk(s, node) || !rw || cap < s->C) return KB_INVALID_ARGUMENT;
  std::vector<uint8_t> v;
  int rc = read_row(s, node, v);
  if (rc) return rc;
  memcpy(rw, v.data(), s->C);
  return KB_OK;
}
extern "C" int kb_sim_peers(kb_sim* s, uint32_t node, uint32_t* peers, size_t cap, size_t* n) {
  if (chk(s, node) || !n) return KB_INVALID_ARGUMENT;
  std::vector<uint8_t> rw;
  int rc = read_row(s, node, rw);
  if (rc) return rc;
  size_t c = 0;
  for (uint32_t j = 0; j < s->C; ++j) if (rw[j]) { if (peers && c < cap) peers[c] = j; c++; }
  *n = c;
  return (peers && cap < c) ? KB_CAPACITY : KB_OK;
}
extern "C" int kb_sim_peer_states(kb_sim* s, uint32_t node, kb_peer_state* out, size_t cap, size_t* n) {
  if (chk(s, node) || !n) return KB_INVALID_ARGUMENT;
  std::vector<uint8_t> rw;
  int rc = read_row(s, node, rw);
  if (rc) return rc;
  std::vector<Susp> sl(SLOTS);
  HIPCHK(hipMemcpy(sl.data(), s->d.susp + (size_t)node * SLOTS, sizeof(Susp) * SLOTS, hipMemcpyDeviceToHost));
  const int32_t E = epoch_base(s->round > 0 ? s->round - 1 : 0);
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
static uint64_t sweep_counter(kb_sim* s) {
  unsigned long long v = 0;
  if (hipMemcpy(&v, s->d.stats + S_SWEEPB, 8, hipMemcpyDeviceToHost) != hipSuccess) return 0;
  return v;
}
extern "C" int kb_sim_reset_kernel_time(kb_sim* s) {
  if (!s) return KB_INVALID_ARGUMENT;
  s->sweep_ms = s->round_ms = 0; s->sweep_launches = s->round_launches = 0;
  s->sweep_bytes = sweep_counter(s);            // baseline of the device-side byte counter
  return KB_OK;
}
// bytes of member bits and stamp lines the row sweep read since the last reset (counted in-kernel)
extern "C" int kb_sim_sweep_bytes(kb_sim* s, uint64_t* bytes) {
  if (!s || !bytes) return KB_INVALID_ARGUMENT;
  *bytes = sweep_counter(s) - s->sweep_bytes;
  return KB_OK;
}
