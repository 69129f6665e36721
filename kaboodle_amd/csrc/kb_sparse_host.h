// kb_sparse_host.h — host side of the sparse-row engine (kb_sparse.h): one handle per mesh, the round's
// launch sequence, and the C-ABI surface of include/kaboodle_sim.h for handles created with
// KB_VARIANT_SPARSE_ROWS.  Included by kb_sim.hip after its host helpers (seterr, HIPCHK, the scan, the CRC
// tables, kb_format_addr, default_identity).
#pragma once
#include <algorithm>
#include <array>
#include <string>
#include <vector>

namespace kb {

enum SpKId : int {
  SPK_REBASE, SPK_EVENTS, SPK_CHURN, SPK_BCAST, SPK_BOUND0, SPK_JRESP, SPK_TRUEFP, SPK_TICK, SPK_BCAST_WRITE, SPK_SCAN,
  SPK_COMPACT, SPK_ROUTE, SPK_PAYBOUND, SPK_SCATTER, SPK_HANDLE, SPK_WINDOW, SPK_ROUND_END, SPK_BFAIL_SF, SPK_N
};
static const char* const SPK_NAME[SPK_N] = {
  "k_sp_rebase", "k_sp_events", "k_sp_churn", "k_sp_bcast", "k_sp_bound0", "k_sp_jresp", "k_sp_truefp", "k_sp_tick",
  "k_sp_bcast_write", "k_sp_scan", "k_sp_compact", "k_sp_route", "k_sp_paybound", "k_sp_scatter", "k_sp_handle",
  "k_sp_window", "k_sp_round_end", "k_sp_bfail_sf"};

struct SpSim {
  kb_config cfg;
  SpDev d;
  int device = 0;
  hipStream_t st = nullptr;
  uint32_t C = 0;
  // row shard: rows [lo, hi) of the mesh, RS rows per rank; xf null = unsharded
  int rank = 0, world = 1;
  uint32_t lo = 0, hi = 0, R = 0, RS = 0;
  Xfer* xf = nullptr;
  bool in_group = false;                            // a shard of a kb_sim_create_local group (the façade sums)
  SpX x;                                            // the waves' send side
  size_t smsg_cap = 0, spay_cap = 0;
  Msg* rmsg = nullptr; uint32_t* rpay = nullptr; uint8_t* rstat = nullptr;
  size_t rmsg_cap = 0, rpay_cap = 0, rstat_cap = 0;
  uint32_t* xall = nullptr;                         // all-gathered counts
  std::vector<uint32_t> h_xall;
  BCast* bjoin_loc = nullptr; BCast* bfail_loc = nullptr;   // this shard's broadcast lists before the all-gather
  uint32_t* rpack = nullptr; uint32_t* rpack_in = nullptr;  // a restart's packed row (send / receive)
  unsigned long long* xstats = nullptr;             // ranks: the counters summed over the mesh
  int32_t round = 0;
  std::vector<void*> allocs;
  std::vector<uint8_t> h_ident, h_idlen, h_pend, h_moved, h_idset;
  std::vector<int16_t> h_pendlen;
  std::vector<uint32_t> h_bbits;
  std::vector<Event> events;
  Event* d_events = nullptr; size_t events_cap = 0;
  std::vector<kb_wire_addr> probe_q, probes;
  std::vector<kb_probe_response> presp;
  uint2* d_presp = nullptr; uint32_t* d_presp_n = nullptr; size_t presp_cap = 0;
  BCast* bjoin = nullptr; BCast* bfail = nullptr;
  uint32_t* fkey = nullptr;                         // the Failed list packed for k_sp_bfail_sf (padded to 4)
  uint32_t nj = 0, nf = 0;
  uint64_t bj_total = 0, bf_total = 0;
  uint32_t* jnew = nullptr; uint32_t* jresp = nullptr; size_t jw_cap = 0;
  uint32_t* jr_n = nullptr; uint32_t* jr_pay = nullptr;
  SpTickOut bo;
  uint32_t* joff = nullptr; uint32_t* foff = nullptr;
  Msg* out[2] = {nullptr, nullptr}; size_t out_cap[2] = {0, 0};
  Msg* stage = nullptr; size_t stage_cap = 0;
  uint32_t* pool[2] = {nullptr, nullptr}; size_t pool_cap[2] = {0, 0};
  uint32_t* inbox = nullptr; size_t inbox_cap = 0;
  uint8_t* status = nullptr; size_t status_cap = 0;
  uint32_t *icnt = nullptr, *icur = nullptr, *ebound = nullptr, *kprc = nullptr, *pb = nullptr;
  uint32_t *ioff = nullptr, *eoff = nullptr, *poff = nullptr, *en = nullptr, *ooff = nullptr;
  uint32_t* scan_tiles = nullptr; uint32_t* scan_tot = nullptr;
  uint2* tfpart = nullptr; uint32_t* tfp = nullptr;
  std::vector<uint32_t> watch_node, watch_fp;
  std::vector<std::vector<uint8_t>> watch_snap;
  // profile: with prof_level > 0 every launch carries start/stop events on its own dispatch packet
  int prof_level = 0;
  struct Rec { int kid; hipEvent_t a, b; };
  std::vector<Rec> recs;
  std::vector<hipEvent_t> ev_free;
  double k_ms[SPK_N] = {};
  uint64_t k_n[SPK_N] = {};
  double round_ms = 0; uint64_t round_n = 0;
  uint64_t host_syncs = 0;
  // external peers
  std::vector<uint8_t> h_ext;
  size_t n_ext = 0;
  std::vector<XRec> inj; std::vector<uint32_t> inj_ids;
  std::vector<uint32_t> inj_join;                    // external peers' Join broadcasts for the next round
  XRec* d_inj = nullptr; uint32_t* d_inj_ids = nullptr; size_t d_inj_cap = 0, d_inj_ids_cap = 0;
  std::vector<kb_unicast> xq; std::vector<uint32_t> xq_ids;
};

static int sp_err_status(uint32_t e) {
  if (!e) return KB_OK;
  const char* what[] = {"", "suspect slots exhausted", "outbox region overflow", "payload pool overflow", "?", "inbox overflow",
                        "Join response member count mismatch", "?", "indirect-ping candidate out of range", "?",
                        "a row's entry list exceeded kb_config.sparse_row_cap", "export buffer overflow"};
  seterr(std::string("device capacity error: ") + (e <= 11 ? what[e] : "?"));
  return KB_CAPACITY;
}
// zeroed device memory.  The zeroing is complete on return: hipMemset runs on the null stream, which does not
// order with the simulator's non-blocking stream, so a kernel enqueued next could otherwise run before it
template <class T> static hipError_t sp_alloc(SpSim* S, T** p, size_t n) {
  hipError_t e = hipMalloc((void**)p, sizeof(T) * (n ? n : 1));
  if (e == hipSuccess) e = hipMemset(*p, 0, sizeof(T) * (n ? n : 1));
  if (e == hipSuccess) e = hipDeviceSynchronize();
  if (e == hipSuccess) S->allocs.push_back((void*)*p);
  return e;
}
// a row table: per_row elements for each of the shard's rows, the pointer biased by -lo rows (kernels index it
// with global ids); SL gives the local base of a one-per-row table
template <class T> static hipError_t sp_ralloc(SpSim* S, T** p, size_t per_row) {
  T* base = nullptr;
  const hipError_t e = sp_alloc(S, &base, per_row * S->R);
  *p = reinterpret_cast<T*>(reinterpret_cast<uintptr_t>(base) - sizeof(T) * per_row * S->lo);
  return e;
}
template <class T> static T* SL(const SpSim* S, T* p) { return p + S->lo; }
// a dynamic buffer of at least `need` elements (contents are not kept)
template <class T> static int sp_grow(SpSim* S, T** p, size_t* cap, size_t need) {
  if (need <= *cap && *p) return KB_OK;
  for (auto& q : S->allocs) if (q == (void*)*p) q = nullptr;
  S->allocs.erase(std::remove(S->allocs.begin(), S->allocs.end(), nullptr), S->allocs.end());
  if (*p) (void)hipFree(*p);
  *p = nullptr;
  const size_t c = std::max<size_t>(need + need / 4, 1024);
  const hipError_t e = sp_alloc(S, p, c);
  if (e != hipSuccess) { *cap = 0; seterr(std::string("sparse engine: device allocation failed: ") + hipGetErrorString(e)); return KB_CAPACITY; }
  *cap = c;
  return KB_OK;
}
static void sp_prof(SpSim* S, int kid, hipEvent_t* a, hipEvent_t* b) {
  *a = *b = nullptr;
  if (S->prof_level <= 0) return;
  hipEvent_t e[2];
  for (int k = 0; k < 2; ++k) {
    if (!S->ev_free.empty()) { e[k] = S->ev_free.back(); S->ev_free.pop_back(); }
    else if (hipEventCreate(&e[k]) != hipSuccess) { if (k) S->ev_free.push_back(e[0]); return; }
  }
  *a = e[0]; *b = e[1];
  S->recs.push_back(SpSim::Rec{kid, e[0], e[1]});
}
template <typename F, typename... Args>
static void sp_launch(SpSim* S, int kid, F kern, uint32_t grid, uint32_t block, Args... args) {
  if (!grid) return;
  hipEvent_t a, b;
  sp_prof(S, kid, &a, &b);
  hipExtLaunchKernelGGL(kern, dim3(grid), dim3(block), 0, S->st, a, b, 0, args...);
}
static void sp_prof_resolve(SpSim* S) {
  for (const auto& q : S->recs) {
    float ms = 0;
    if (hipEventElapsedTime(&ms, q.a, q.b) == hipSuccess) {
      if (q.kid == SPK_N) { S->round_ms += ms; S->round_n++; }
      else { S->k_ms[q.kid] += ms; S->k_n[q.kid]++; }
    }
    S->ev_free.push_back(q.a); S->ev_free.push_back(q.b);
  }
  S->recs.clear();
}
static hipError_t sp_sync(SpSim* S) { S->host_syncs++; return hipStreamSynchronize(S->st); }
// exclusive scans of up to 4 arrays of n elements (the shard's rows: local bases), totals into scan_tot[t0..]
static void sp_scan(SpSim* S, uint32_t n, int narr, const uint32_t* const* in, uint32_t* const* out, uint32_t t0) {
  ScanArgs a;
  memset(&a, 0, sizeof a);
  a.n = n; a.narr = narr; a.totals = S->scan_tot + t0; a.tiles = S->scan_tiles; a.ntiles = (n + 1023) / 1024;
  for (int q = 0; q < narr; ++q) { a.in[q] = in[q]; a.out[q] = out[q]; }
  sp_launch(S, SPK_SCAN, k_scan_tiles, a.ntiles, 1024, a);
  sp_launch(S, SPK_SCAN, k_scan_apply, a.ntiles, 1024, a);
}

// per-id segment CRCs and uniformity (identity changes), on the host tables
static int sp_upload_segments(SpSim* S) {
  const uint32_t C = S->C;
  std::vector<uint32_t> cseg(C), segmul(C), seglen(C);
  bool uniform = true;
  uint32_t xp[ADDR_LEN + MAXID + 1];                 // x^(8 len) per segment length
  for (uint32_t l = 0; l <= ADDR_LEN + MAXID; ++l) xp[l] = h_xpow8(l);
  for (uint32_t j = 0; j < C; ++j) {
    char a[32]; kb_format_addr(j, a, sizeof a);
    uint32_t reg = h_crc_update(0, (const uint8_t*)a, ADDR_LEN);
    reg = h_crc_update(reg, &S->h_ident[(size_t)j * MAXID], S->h_idlen[j]);
    cseg[j] = reg; seglen[j] = ADDR_LEN + S->h_idlen[j]; segmul[j] = xp[seglen[j]];
    if (S->h_idlen[j] != S->cfg.id_len) uniform = false;
  }
  S->d.uniform = uniform ? 1 : 0;
  HIPCHK(hipMemcpy(S->d.cseg, cseg.data(), 4ull * C, hipMemcpyHostToDevice));
  HIPCHK(hipMemcpy(S->d.segmul, segmul.data(), 4ull * C, hipMemcpyHostToDevice));
  HIPCHK(hipMemcpy(S->d.seglen, seglen.data(), 4ull * C, hipMemcpyHostToDevice));
  return KB_OK;
}

static void sp_destroy(SpSim* S) {
  if (!S) return;
  (void)hipSetDevice(S->device);
  if (S->st) (void)hipStreamSynchronize(S->st);
  for (void* p : S->allocs) (void)hipFree(p);
  if (S->d_events) (void)hipFree(S->d_events);
  if (S->d_presp) (void)hipFree(S->d_presp);
  for (auto& q : S->recs) { (void)hipEventDestroy(q.a); (void)hipEventDestroy(q.b); }
  for (hipEvent_t e : S->ev_free) (void)hipEventDestroy(e);
  if (S->st) (void)hipStreamDestroy(S->st);
  delete S->xf;
  delete S;
}

// kb_sim_create with KB_VARIANT_SPARSE_ROWS: the whole mesh (xf null), or rank `rank` of `world` row shards
// exchanging over xf (kb_sim_create_local / kb_sim_create_rank; the handle owns xf)
static int sp_create(const kb_config* cfg, int rank, int world, Xfer* xf, SpSim** out) {
  h_crc_init();
  if (cfg->variant != KB_VARIANT_SPARSE_ROWS) { seterr("the sparse rows take no other semantic variant"); delete xf; return KB_INVALID_ARGUMENT; }
  if (cfg->track_latency) { seterr("sparse rows keep no latency table"); delete xf; return KB_INVALID_ARGUMENT; }
  if (cfg->stat_flags & ~(uint32_t)KB_STAT_NO_SF_FAILED_DROPS) { seterr("unknown kb_config.stat_flags"); delete xf; return KB_INVALID_ARGUMENT; }
  const uint32_t C = cfg->capacity;
  const uint32_t RS = (C + (uint32_t)world - 1) / (uint32_t)world;
  if (world < 1 || world > (int)XMAX || rank < 0 || rank >= world || (uint64_t)(world - 1) * RS >= C) {
    seterr("shard layout out of range (1..8 shards, each holding at least one row)"); delete xf; return KB_INVALID_ARGUMENT;
  }
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0) { seterr("no HIP device"); delete xf; return KB_NO_DEVICE; }
  SpSim* S = new SpSim();
  memset((void*)&S->d, 0, sizeof S->d);
  memset((void*)&S->x, 0, sizeof S->x);
  S->cfg = *cfg;
  S->xf = xf;
  S->rank = rank; S->world = world; S->RS = RS;
  S->lo = (uint32_t)rank * RS; S->hi = std::min<uint32_t>(C, S->lo + RS); S->R = S->hi - S->lo;
  S->device = cfg->device >= 0 ? cfg->device : 0;
  if (cfg->device < 0) (void)hipGetDevice(&S->device);
  if (hipSetDevice(S->device) != hipSuccess) { sp_destroy(S); seterr("hipSetDevice failed"); return KB_NO_DEVICE; }
  S->C = C;
  const uint32_t R = S->R;
  SpDev& d = S->d;
  d.C = C; d.lo = S->lo; d.hi = S->hi; d.rank0 = rank == 0 ? 1u : 0u;
  d.ECAP = cfg->sparse_row_cap ? std::min<uint32_t>(cfg->sparse_row_cap, C) : std::min<uint32_t>(C, 4096u);
  d.ESTR = (d.ECAP + 3u) & ~3u;
  d.nb = cfg->init_mode == KB_INIT_CONVERGED ? cfg->initial_nodes : 0u;
  d.k0 = (uint32_t)cfg->seed; d.k1 = (uint32_t)(cfg->seed >> 32);
  d.loss_thr = cfg->loss_threshold; d.churn_thr = cfg->churn_threshold; d.fault_end = cfg->fault_end_round;
  d.failed_mode = cfg->failed_mode; d.pgroups = cfg->partition_groups; d.pstart = cfg->partition_start; d.pend = cfg->partition_end;
  const uint32_t Lid = cfg->id_len;
  d.L = ADDR_LEN + Lid;
  d.capk = (BUFSZ - 20 - Lid) / (18 + Lid);             // KPR reply: 20 + L + k(18+L) <= 10240
  d.capj = (BUFSZ - 20 - Lid - 1) / (18 + Lid);         // Join response: 20 + L + k(18+L) < 10240
  S->h_ident.assign((size_t)C * MAXID, 0); S->h_idlen.assign(C, (uint8_t)Lid);
  S->h_pend.assign((size_t)C * MAXID, 0); S->h_pendlen.assign(C, (int16_t)-1); S->h_moved.assign(C, 0);
  S->h_idset.assign(C, 0);
  for (uint32_t j = 0; j < C; ++j) default_identity(j, Lid, &S->h_ident[(size_t)j * MAXID]);
  hipError_t e = hipSuccess;
#define SA(ptr, n) if (e == hipSuccess) e = sp_alloc(S, &(ptr), (n))     // per-id and global tables
#define SR(ptr, n) if (e == hipSuccess) e = sp_ralloc(S, &(ptr), (n))    // row tables: n per local row
  SR(d.ent, d.ESTR); SR(d.ne, 1); SR(d.based, 1); SR(d.n, 1); SR(d.fp, 1); SR(d.dirty, 1);
  SR(d.last_bcast, 1); SR(d.a3cur, 1); SR(d.susp, SLOTS); SR(d.cur, CSLOTS);
  SR(d.paq, PAQ); SR(d.paq_n, 1); SA(d.alive, C); SA(d.start_round, C); SA(d.idset, C); SA(d.ext, C);
  SA(d.cseg, C); SA(d.segmul, C); SA(d.seglen, C); SA(d.bbits, C / 32 + 1); SA(d.bcnt, (size_t)C + 1);
  SA(d.bpre, (size_t)C + 1); SA(d.zpow, (size_t)C + 2); SA(d.stats, NSTAT); SA(d.sacc, (size_t)SP_ACC * NSTAT);
  SA(d.ctr, NCTR); SA(d.tacc, 2 * SP_ACC);
  SA(S->bjoin, C); SA(S->bfail, (size_t)C * SLOTS); SA(S->fkey, (size_t)C * SLOTS + 4); SR(S->jr_n, 1); SR(S->jr_pay, 1);
  SR(S->bo.bj, 1); SR(S->bo.bnf, 1); SR(S->bo.bfp, SLOTS); SR(S->joff, 1); SR(S->foff, 1);
  SR(S->icnt, 1); SR(S->icur, 1); SR(S->ebound, 1); SR(S->kprc, 1); SR(S->pb, 1);
  SR(S->ioff, 1); SR(S->eoff, 1); SR(S->poff, 1); SR(S->en, 1); SR(S->ooff, 1);
  SA(S->scan_tiles, 5 * ((std::max<size_t>(C, (size_t)world * R) + 1023) / 1024) + 5); SA(S->scan_tot, 32);
  SA(S->tfpart, SP_TFP); SA(S->tfp, 1);
  if (xf) {
    SpX& x = S->x;
    x.world = (uint32_t)world; x.R = R; x.S = RS;
    SA(x.xcnt, (size_t)world * R); SA(x.xpay, (size_t)world * R); SA(x.xoff, (size_t)world * R); SA(x.xpoff, (size_t)world * R);
    SA(x.xb, 2 * world); SA(S->xall, 2 * world * world); SA(S->xstats, NSTAT);
    SA(S->bjoin_loc, R); SA(S->bfail_loc, (size_t)R * SLOTS);
    S->h_xall.assign(2 * world * world, 0);
  }
#undef SA
#undef SR
  if (e != hipSuccess) { seterr(std::string("sparse engine: device allocation failed: ") + hipGetErrorString(e)); sp_destroy(S); return KB_CAPACITY; }
  if (hipStreamCreateWithFlags(&S->st, hipStreamNonBlocking) != hipSuccess) { sp_destroy(S); seterr("stream"); return KB_IO_ERROR; }
  if (const char* pv = getenv("KB_PROF")) S->prof_level = atoi(pv);
  { const int rc = sp_upload_segments(S); if (rc) { sp_destroy(S); return rc; } }
  // the base (the initial members of a converged start) with its prefix counts and prefix folds, and Z^k
  {
    const uint32_t nb = d.nb;
    S->h_bbits.assign(C / 32 + 1, 0);
    for (uint32_t j = 0; j < nb; ++j) S->h_bbits[j >> 5] |= 1u << (j & 31);
    std::vector<uint32_t> bcnt((size_t)C + 1), bpre((size_t)C + 1), zpow((size_t)C + 2), cseg(C);
    if (hipMemcpy(cseg.data(), d.cseg, 4ull * C, hipMemcpyDeviceToHost) != hipSuccess) { sp_destroy(S); seterr("cseg"); return KB_IO_ERROR; }
    const uint32_t Z = h_xpow8(d.L);
    zpow[0] = 0x80000000u;
    for (size_t k = 1; k < zpow.size(); ++k) zpow[k] = multmodp(Z, zpow[k - 1]);
    uint32_t raw = 0, c = 0;
    for (uint32_t j = 0; j <= C; ++j) {
      bcnt[j] = c; bpre[j] = raw;
      if (j < C && j < nb) { raw = multmodp(Z, raw) ^ cseg[j]; c++; }
    }
    if (hipMemcpy(d.bbits, S->h_bbits.data(), 4ull * S->h_bbits.size(), hipMemcpyHostToDevice) != hipSuccess ||
        hipMemcpy(d.bcnt, bcnt.data(), 4ull * bcnt.size(), hipMemcpyHostToDevice) != hipSuccess ||
        hipMemcpy(d.bpre, bpre.data(), 4ull * bpre.size(), hipMemcpyHostToDevice) != hipSuccess ||
        hipMemcpy(d.zpow, zpow.data(), 4ull * zpow.size(), hipMemcpyHostToDevice) != hipSuccess) {
      sp_destroy(S); seterr("base tables"); return KB_IO_ERROR;
    }
  }
  uint32_t ctr0[NCTR] = {0};
  ctr0[C_NEXTFREE] = cfg->initial_nodes;
  ctr0[C_FIRSTCONV] = 0xFFFFFFFFu; ctr0[C_LASTCONV] = 0xFFFFFFFFu;
  if (hipMemcpy(d.ctr, ctr0, sizeof ctr0, hipMemcpyHostToDevice) != hipSuccess) { sp_destroy(S); seterr("ctr upload"); return KB_IO_ERROR; }
  k_sp_init<<<(C + 255) / 256, 256, 0, S->st>>>(d, cfg->initial_nodes, cfg->init_mode == KB_INIT_CONVERGED ? 1u : 0u);
  if (hipStreamSynchronize(S->st) != hipSuccess) { sp_destroy(S); seterr("init failed"); return KB_IO_ERROR; }
  *out = S;
  return KB_OK;
}

static int sp_read_row(SpSim* S, uint32_t node, std::vector<uint8_t>& rw);
static int sp_xfail(SpSim* S) { seterr(S->xf->error()); return KB_IO_ERROR; }
// one all-to-all-v pair (records + ids, or two lists) as one group; an opened group is always closed
static int sp_a2a2(SpSim* S, const void* s1, const size_t* sc1, const size_t* sd1, void* r1, const size_t* rc1, const size_t* rd1,
                   size_t e1, const void* s2, const size_t* sc2, const size_t* sd2, void* r2, const size_t* rc2, const size_t* rd2,
                   size_t e2) {
  if (!S->xf->group_begin()) return sp_xfail(S);
  const bool sent = S->xf->alltoallv(s1, sc1, sd1, r1, rc1, rd1, e1, S->st) && (!s2 || S->xf->alltoallv(s2, sc2, sd2, r2, rc2, rd2, e2, S->st));
  const std::string err = sent ? std::string() : S->xf->error();
  if (!S->xf->group_end() || !sent) { seterr(sent ? S->xf->error() : err); return KB_IO_ERROR; }
  return KB_OK;
}

// A restart's map across shards: the old address's row, packed on the shard holding it,
// moves to the shard holding the fresh address (an all-to-all-v with one non-empty pair, on every rank); the
// instance's event observer moves with it (the map and its observer belong to the Kaboodle, src/lib.rs:104).
// *snap_after: an observer attached to the fresh address before this round takes its snapshot once the restart
// has applied (the instance had none)
static int sp_move_row(SpSim* S, uint32_t from, uint32_t to, bool* snap_after) {
  *snap_after = false;
  const uint32_t nw = (S->C + 31) / 32, ext0 = SP_PACK_HDR + S->d.ESTR;
  const size_t words = (size_t)ext0 + 2 + nw;           // row, then [watched, fp, snapshot bits]
  if (!S->rpack) { HIPCHK(sp_alloc(S, &S->rpack, words)); HIPCHK(sp_alloc(S, &S->rpack_in, words)); }
  const bool have = from >= S->lo && from < S->hi, take = to >= S->lo && to < S->hi;
  if (have) {
    k_sp_row_pack<<<8, 256, 0, S->st>>>(S->d, from, S->rpack);
    std::vector<uint32_t> ext(2 + nw, 0);
    size_t kf = 0;
    while (kf < S->watch_node.size() && S->watch_node[kf] != from) ++kf;
    if (kf < S->watch_node.size()) {
      ext[0] = 1; ext[1] = S->watch_fp[kf];
      for (uint32_t j = 0; j < S->C; ++j) if (S->watch_snap[kf][j]) ext[2 + (j >> 5)] |= 1u << (j & 31);
      S->watch_node.erase(S->watch_node.begin() + kf); S->watch_fp.erase(S->watch_fp.begin() + kf);
      S->watch_snap.erase(S->watch_snap.begin() + kf);
    }
    HIPCHK(hipMemcpyAsync(S->rpack + ext0, ext.data(), 4 * ext.size(), hipMemcpyHostToDevice, S->st));
    HIPCHK(sp_sync(S));
  }
  size_t sc[XMAX] = {}, sd[XMAX] = {}, rc[XMAX] = {}, rd[XMAX] = {};
  const int ofrom = (int)(from / S->RS), oto = (int)(to / S->RS);
  if (S->rank == ofrom) sc[oto] = words;
  if (S->rank == oto) rc[ofrom] = words;
  { const int rc2 = sp_a2a2(S, S->rpack, sc, sd, S->rpack_in, rc, rd, 4, nullptr, nullptr, nullptr, nullptr, nullptr, nullptr, 0); if (rc2) return rc2; }
  if (!take) return KB_OK;
  k_sp_row_unpack<<<8, 256, 0, S->st>>>(S->d, to, S->rpack_in);
  std::vector<uint32_t> ext(2 + nw);
  HIPCHK(hipMemcpyAsync(ext.data(), S->rpack_in + ext0, 4 * ext.size(), hipMemcpyDeviceToHost, S->st));
  HIPCHK(sp_sync(S));
  size_t kt = 0;
  while (kt < S->watch_node.size() && S->watch_node[kt] != to) ++kt;
  if (ext[0]) {
    if (kt == S->watch_node.size()) { S->watch_node.push_back(to); S->watch_fp.push_back(0); S->watch_snap.emplace_back(S->C, 0); }
    S->watch_fp[kt] = ext[1];
    for (uint32_t j = 0; j < S->C; ++j) S->watch_snap[kt][j] = (uint8_t)((ext[2 + (j >> 5)] >> (j & 31)) & 1u);
  } else if (kt < S->watch_node.size()) {
    *snap_after = true;
  }
  return KB_OK;
}

// API events in call order (src/lib.rs:136-183); a restart moves the map to its fresh address
static int sp_apply_events(SpSim* S, int32_t r) {
  SpDev& d = S->d;
  const uint32_t C = S->C;
  if (S->events.empty()) return KB_OK;
  if (S->xf) for (Event& ev : S->events) if (ev.kind == EV_RESTART) ev.kind = EV_START_MOVED;   // the row moves on the host
  if (S->events.size() > S->events_cap) {
    if (S->d_events) (void)hipFree(S->d_events);
    S->events_cap = S->events.size() * 2;
    HIPCHK(hipMalloc(&S->d_events, sizeof(Event) * S->events_cap));
  }
  HIPCHK(hipMemcpyAsync(S->d_events, S->events.data(), sizeof(Event) * S->events.size(), hipMemcpyHostToDevice, S->st));
  size_t k0 = 0;
  for (size_t k = 0; k < S->events.size(); ++k) {
    const Event& ev = S->events[k];
    if (ev.kind == EV_START_MOVED) {                   // sharded restart: events before it, the row move, its start
      if (k > k0) sp_launch(S, SPK_EVENTS, k_sp_events, 1, 1, d, (const Event*)S->d_events + k0, (uint32_t)(k - k0), r);
      bool snap_after = false;
      { const int rc = sp_move_row(S, ev.src, ev.node, &snap_after); if (rc) return rc; }
      sp_launch(S, SPK_EVENTS, k_sp_events, 1, 1, d, (const Event*)S->d_events + k, 1u, r);
      k0 = k + 1;
      if (snap_after) {
        std::vector<uint8_t> rw;
        HIPCHK(sp_sync(S));
        const int rc = sp_read_row(S, ev.node, rw);
        if (rc) return rc;
        for (size_t q = 0; q < S->watch_node.size(); ++q)
          if (S->watch_node[q] == ev.node) for (uint32_t j = 0; j < C; ++j) S->watch_snap[q][j] = rw[j] != 0;
      }
      continue;
    }
    if (ev.kind != EV_RESTART) continue;
    // unsharded: the map's observer follows the instance.  An observer attached to the new address before this
    // round gives way to the instance's own, or (the instance had none) starts from the row the restart leaves,
    // so it reports only later changes
    size_t kf = S->watch_node.size(), kt = S->watch_node.size();
    for (size_t q = 0; q < S->watch_node.size(); ++q) { if (S->watch_node[q] == ev.src) kf = q; if (S->watch_node[q] == ev.node) kt = q; }
    if (kf < S->watch_node.size()) {
      if (kt < S->watch_node.size()) {
        S->watch_node.erase(S->watch_node.begin() + kt); S->watch_fp.erase(S->watch_fp.begin() + kt);
        S->watch_snap.erase(S->watch_snap.begin() + kt);
        if (kf > kt) kf--;
      }
      S->watch_node[kf] = ev.node;
    } else if (kt < S->watch_node.size()) {
      sp_launch(S, SPK_EVENTS, k_sp_events, 1, 1, d, (const Event*)S->d_events + k0, (uint32_t)(k + 1 - k0), r);
      k0 = k + 1;
      std::vector<uint8_t> rw;
      HIPCHK(sp_sync(S));
      const int rc = sp_read_row(S, ev.node, rw);
      if (rc) return rc;
      for (uint32_t j = 0; j < C; ++j) S->watch_snap[kt][j] = rw[j] != 0;
    }
  }
  if (k0 < S->events.size())
    sp_launch(S, SPK_EVENTS, k_sp_events, 1, 1, d, (const Event*)S->d_events + k0, (uint32_t)(S->events.size() - k0), r);
  HIPCHK(sp_sync(S));
  S->events.clear();
  return KB_OK;
}

// sharded: every shard's broadcast lists, concatenated in rank order = sender order (one all-gather of the counts,
// then each shard's lists to every rank)
static int sp_gather_bcasts(SpSim* S, uint32_t nj_loc, uint32_t nf_loc, uint32_t* nj, uint32_t* nf) {
  const int W = S->world;
  if (!S->xf->allgather_u32(S->scan_tot + 2, S->xall, 2, S->st)) return sp_xfail(S);
  HIPCHK(hipMemcpyAsync(S->h_xall.data(), S->xall, 8ull * W, hipMemcpyDeviceToHost, S->st));
  HIPCHK(sp_sync(S));
  size_t sc[XMAX], sd[XMAX], rc[XMAX], rd[XMAX], fsc[XMAX], frc[XMAX], frd[XMAX];
  size_t oj = 0, of = 0;
  for (int k = 0; k < W; ++k) {
    rc[k] = S->h_xall[2 * k]; frc[k] = S->h_xall[2 * k + 1];
    rd[k] = oj; oj += rc[k]; frd[k] = of; of += frc[k];
    sc[k] = nj_loc; fsc[k] = nf_loc; sd[k] = 0;
  }
  const int rc2 = sp_a2a2(S, S->bjoin_loc, sc, sd, S->bjoin, rc, rd, sizeof(BCast), S->bfail_loc, fsc, sd, S->bfail, frc, frd, sizeof(BCast));
  if (rc2) return rc2;
  *nj = (uint32_t)oj; *nf = (uint32_t)of;
  return KB_OK;
}

// sharded: route this shard's M records of out[cur], move the delivered ones to the shards holding their
// destinations' rows, and count them there.  *nrecv = records received; *any = some rank delivered a record
static int sp_exchange_wave(SpSim* S, uint32_t M, int cur, int32_t r, uint32_t w, uint32_t* nrecv, bool* any) {
  SpDev& d = S->d;
  const int W = S->world, me = S->rank;
  const uint32_t R = S->R;
  hipStream_t st = S->st;
  SpX& x = S->x;
  HIPCHK(hipMemsetAsync(x.xcnt, 0, 4ull * W * R, st));
  HIPCHK(hipMemsetAsync(x.xpay, 0, 4ull * W * R, st));
  { const int rc = sp_grow(S, &S->status, &S->status_cap, M); if (rc) return rc; }
  SpRoute rt;
  memset(&rt, 0, sizeof rt);
  rt.msgs = S->out[cur]; rt.M = M; rt.status = S->status; rt.pay = S->pool[cur];
  if (M) sp_launch(S, SPK_ROUTE, k_sp_route_x, (M + 255) / 256, 256, d, rt, x, r, w);
  {
    const uint32_t* in[2] = {x.xcnt, x.xpay};
    uint32_t* out[2] = {x.xoff, x.xpoff};
    sp_scan(S, (uint32_t)W * R, 2, in, out, 16);
  }
  sp_launch(S, SPK_ROUTE, k_sp_xbound, 1, 64, x, (const uint32_t*)S->scan_tot + 16);
  if (!S->xf->allgather_u32(x.xb, S->xall, 2 * W, st)) return sp_xfail(S);
  HIPCHK(hipMemcpyAsync(S->h_xall.data(), S->xall, 4ull * 2 * W * W, hipMemcpyDeviceToHost, st));
  HIPCHK(sp_sync(S));
  size_t sc[XMAX], sd[XMAX], rc[XMAX], rd[XMAX], psc[XMAX], psd[XMAX], prc[XMAX], prd[XMAX];
  size_t so = 0, pso = 0, ro = 0, pro = 0;
  uint64_t total = 0;
  for (int k = 0; k < W * W; ++k) total += S->h_xall[(size_t)(k / W) * 2 * W + (k % W)];
  *any = total != 0;
  *nrecv = 0;
  if (!*any) return KB_OK;
  for (int k = 0; k < W; ++k) {
    sc[k] = S->h_xall[(size_t)me * 2 * W + k]; psc[k] = S->h_xall[(size_t)me * 2 * W + W + k];
    rc[k] = S->h_xall[(size_t)k * 2 * W + me]; prc[k] = S->h_xall[(size_t)k * 2 * W + W + me];
    sd[k] = so; so += sc[k]; psd[k] = pso; pso += psc[k];
    rd[k] = ro; ro += rc[k]; prd[k] = pro; pro += prc[k];
  }
  { const int rc2 = sp_grow(S, &x.smsg, &S->smsg_cap, so); if (rc2) return rc2; }
  { const int rc2 = sp_grow(S, &x.spay, &S->spay_cap, pso); if (rc2) return rc2; }
  { const int rc2 = sp_grow(S, &S->rmsg, &S->rmsg_cap, ro); if (rc2) return rc2; }
  { const int rc2 = sp_grow(S, &S->rpay, &S->rpay_cap, pro); if (rc2) return rc2; }
  { const int rc2 = sp_grow(S, &S->rstat, &S->rstat_cap, ro); if (rc2) return rc2; }
  if (M) sp_launch(S, SPK_ROUTE, k_sp_pack, (R + 255) / 256, 256, d, x, (const Msg*)S->out[cur], (const uint8_t*)S->status,
                   (const uint32_t*)S->pool[cur], (const uint32_t*)S->ooff, (const uint32_t*)S->en);
  { const int rc2 = sp_a2a2(S, x.smsg, sc, sd, S->rmsg, rc, rd, sizeof(Msg), x.spay, psc, psd, S->rpay, prc, prd, 4); if (rc2) return rc2; }
  SpRecvBlocks rb;
  memset(&rb, 0, sizeof rb);
  for (int k = 0; k < W; ++k) rb.p0[k] = (uint32_t)prd[k];
  SpRoute rr;
  memset(&rr, 0, sizeof rr);
  rr.msgs = S->rmsg; rr.M = (uint32_t)ro; rr.status = S->rstat; rr.pay = S->rpay;
  rr.icnt = S->icnt; rr.ebound = S->ebound; rr.kprc = S->kprc;
  if (ro) sp_launch(S, SPK_ROUTE, k_sp_recv, (uint32_t)((ro + 255) / 256), 256, rr, x, rb);
  *nrecv = (uint32_t)ro;
  return KB_OK;
}

static int sp_step_round(SpSim* S) {
  SpDev& d = S->d;
  const int32_t r = S->round;
  const uint32_t C = S->C, R = S->R, tb = 256, g = (R + tb - 1) / tb, gc = (C + tb - 1) / tb;
  const bool sh = S->xf != nullptr;
  hipStream_t st = S->st;
  hipEvent_t er[2] = {nullptr, nullptr};
  if (S->prof_level > 0) {
    for (int k = 0; k < 2; ++k) {
      if (!S->ev_free.empty()) { er[k] = S->ev_free.back(); S->ev_free.pop_back(); }
      else (void)hipEventCreate(&er[k]);
    }
    (void)hipEventRecord(er[0], st);
  }
  // 0. stamp window
  if (r > 0 && r % EPOCH == 0) sp_launch(S, SPK_REBASE, k_sp_rebase, g, tb, d);
  // 1. lifecycle: API events in call order (a restart moves the map to its fresh address), then churn; every
  // shard replays them over all ids (the per-id facts are replicated), rows change on the shard holding them
  { const int rc = sp_apply_events(S, r); if (rc) return rc; }
  if ((S->cfg.fault_end_round < 0 || r < S->cfg.fault_end_round) && S->cfg.churn_threshold) {
    sp_launch(S, SPK_CHURN, k_sp_churn_leave, gc, tb, d, r);
    sp_launch(S, SPK_CHURN, k_sp_churn_join, 1, 1, d, r);
  }
  // 2. broadcasts of round r-1 (Failed, Join with the external peers' Joins), and the Probes queued since the last round
  if (!S->inj_join.empty()) {
    const int rc = merge_ext_joins(S->st, S->bjoin, &S->nj, S->inj_join, S->cfg.partition_groups, C);
    if (rc) return rc;
  }
  S->probes.swap(S->probe_q);
  S->probe_q.clear();
  const uint32_t np = (uint32_t)S->probes.size();
  if (np) {
    const size_t need = (size_t)np * R;
    if (need > S->presp_cap) {
      if (S->d_presp) (void)hipFree(S->d_presp);
      S->d_presp = nullptr;
      HIPCHK(hipMalloc(&S->d_presp, sizeof(uint2) * need));
      S->presp_cap = need;
    }
    if (!S->d_presp_n) HIPCHK(sp_alloc(S, &S->d_presp_n, 1));
    HIPCHK(hipMemsetAsync(S->d_presp_n, 0, 4, st));
  }
  SpBc bc;
  memset(&bc, 0, sizeof bc);
  bc.bfail = S->bfail; bc.nf = S->nf; bc.bjoin = S->bjoin; bc.nj = S->nj; bc.JW = (S->nj + 31) / 32;
  if (bc.JW) {
    const size_t words = (size_t)R * bc.JW;
    if (words > S->jw_cap) {
      int rc = KB_OK;
      size_t c1 = S->jw_cap, c2 = S->jw_cap;
      rc = sp_grow(S, &S->jnew, &c1, words);
      if (!rc) rc = sp_grow(S, &S->jresp, &c2, words);
      if (rc) return rc;
      S->jw_cap = std::min(c1, c2);
    }
    HIPCHK(hipMemsetAsync(S->jnew, 0, 4 * words, st));
    HIPCHK(hipMemsetAsync(S->jresp, 0, 4 * words, st));
  }
  bc.jnew = S->jnew; bc.jresp = S->jresp; bc.jr_n = S->jr_n; bc.jr_pay = S->jr_pay;
  bc.np = np; bc.presp = S->d_presp; bc.presp_n = S->d_presp_n; bc.presp_cap = (uint32_t)std::min<size_t>(S->presp_cap, 0xFFFFFFFFu);
  if (S->nf && S->cfg.failed_mode == KB_FAILED_SOCKET_FAITHFUL && (S->cfg.stat_flags & KB_STAT_NO_SF_FAILED_DROPS)) {
    bc.fcounted = 1;                                   // no state effect, and their drops are not counted
  } else if (S->nf && S->cfg.failed_mode == KB_FAILED_SOCKET_FAITHFUL && S->cfg.partition_groups <= 255) {
    sp_launch(S, SPK_BFAIL_SF, k_sp_bfail_sf, g, tb, d, (const uint4*)S->fkey, S->nf, r);
    bc.fcounted = 1;
  }
  sp_launch(S, SPK_BCAST, k_sp_bcast, g, tb, d, bc, r);
  // wave-0 regions: Join responses first, then the tick's emissions; the external peers' injected records (the
  // shard holding the external id's row injects them)
  sp_launch(S, SPK_BOUND0, k_sp_bound0, g, tb, d, (const uint32_t*)S->jr_n, S->ebound);
  std::vector<XRec> inj;
  for (const XRec& q : S->inj) if (q.sender >= S->lo && q.sender < S->hi) inj.push_back(q);
  const uint32_t ninj = (uint32_t)inj.size();
  if (ninj) {
    { size_t c = S->d_inj_cap; const int rc = sp_grow(S, &S->d_inj, &c, ninj); if (rc) return rc; S->d_inj_cap = c; }
    { size_t c = S->d_inj_ids_cap; const int rc = sp_grow(S, &S->d_inj_ids, &c, S->inj_ids.size() + 1); if (rc) return rc; S->d_inj_ids_cap = c; }
    HIPCHK(hipMemcpyAsync(S->d_inj, inj.data(), sizeof(XRec) * ninj, hipMemcpyHostToDevice, st));
    if (!S->inj_ids.empty()) HIPCHK(hipMemcpyAsync(S->d_inj_ids, S->inj_ids.data(), 4 * S->inj_ids.size(), hipMemcpyHostToDevice, st));
    sp_launch(S, SPK_EVENTS, k_sp_inject_prep, 1, 1, d, (const XRec*)S->d_inj, ninj, S->ebound, S->jr_pay);
  }
  {
    const uint32_t* in[2] = {SL(S, S->ebound), SL(S, S->jr_pay)};
    uint32_t* out[2] = {SL(S, S->eoff), SL(S, S->poff)};
    sp_scan(S, R, 2, in, out, 0);
  }
  uint32_t tot[8];
  HIPCHK(hipMemcpyAsync(tot, S->scan_tot, 8, hipMemcpyDeviceToHost, st));
  HIPCHK(sp_sync(S));
  { const int rc = sp_grow(S, &S->stage, &S->stage_cap, tot[0]); if (rc) return rc; }
  { const int rc = sp_grow(S, &S->pool[0], &S->pool_cap[0], tot[1]); if (rc) return rc; }
  if (S->n_ext) {                                    // exports of the round: wave 0's totals + the later waves' allowance
    const uint64_t nr = (uint64_t)tot[0] + (1u << 16), ni = (uint64_t)tot[1] + (1u << 22);   // (kb_sim.hip size_exports)
    if (nr > 0xFFFFFFFFull || ni > 0xFFFFFFFFull) { seterr("export buffer beyond 2^32 entries"); return KB_CAPACITY; }
    if (nr > d.xrec_cap) { size_t c = d.xrec_cap; const int rc = sp_grow(S, &d.xrec, &c, nr); if (rc) return rc; d.xrec_cap = (uint32_t)std::min<size_t>(c, 0xFFFFFFFFu); }
    if (ni > d.xids_cap) { size_t c = d.xids_cap; const int rc = sp_grow(S, &d.xids, &c, ni); if (rc) return rc; d.xids_cap = (uint32_t)std::min<size_t>(c, 0xFFFFFFFFu); }
  }
  SpOut o0;
  o0.stage = S->stage; o0.eoff = S->eoff; o0.ecap = S->ebound; o0.pay = S->pool[0]; o0.poff = S->poff; o0.pcap = S->jr_pay;
  o0.en = S->en;
  if (S->nj) sp_launch(S, SPK_JRESP, k_sp_jresp, g, tb, d, bc, o0, r);
  // 3. tick, against the running set's fingerprint
  sp_launch(S, SPK_TRUEFP, k_sp_truefp_part, SP_TFP / 256, 256, d, S->tfpart);
  sp_launch(S, SPK_TRUEFP, k_sp_truefp_fin, 1, 64, d, (const uint2*)S->tfpart, S->tfp);
  sp_launch(S, SPK_TICK, k_sp_tick, g, tb, d, o0, (const uint32_t*)S->jr_n, S->bo, (const uint32_t*)S->tfp, r);
  if (ninj) sp_launch(S, SPK_EVENTS, k_sp_inject, 1, 1, d, o0, (const XRec*)S->d_inj, ninj, (const uint32_t*)S->d_inj_ids);
  S->inj.clear(); S->inj_ids.clear();
  {
    const uint32_t* in[3] = {SL(S, S->bo.bj), SL(S, S->bo.bnf), SL(S, S->en)};
    uint32_t* out[3] = {SL(S, S->joff), SL(S, S->foff), SL(S, S->ooff)};
    sp_scan(S, R, 3, in, out, 2);
  }
  sp_launch(S, SPK_BCAST_WRITE, k_sp_bcast_write, g, tb, d, S->bo, (const uint32_t*)S->joff, (const uint32_t*)S->foff,
            sh ? S->bjoin_loc : S->bjoin, sh ? S->bfail_loc : S->bfail);
  HIPCHK(hipMemcpyAsync(tot + 2, S->scan_tot + 2, 12, hipMemcpyDeviceToHost, st));
  HIPCHK(sp_sync(S));
  uint32_t nj_next = tot[2], nf_next = tot[3];
  uint32_t M = tot[4];
  if (sh) { const int rc = sp_gather_bcasts(S, tot[2], tot[3], &nj_next, &nf_next); if (rc) return rc; }
  if (nf_next) sp_launch(S, SPK_BCAST_WRITE, k_sp_fkey, (nf_next + 3 + 255) / 256, 256, (const BCast*)S->bfail, nf_next, S->fkey);
  { const int rc = sp_grow(S, &S->out[0], &S->out_cap[0], M); if (rc) return rc; }
  sp_launch(S, SPK_COMPACT, k_sp_compact, g, tb, d, o0, (const uint32_t*)S->ooff, S->out[0]);
  // 4. receive window: delivery waves (sharded: routed on the senders' shards, exchanged, handled on the receivers')
  int cur = 0;
  for (uint32_t w = 0; w < S->cfg.max_waves && (M || sh); ++w) {
    HIPCHK(hipMemsetAsync(SL(S, S->icnt), 0, 4ull * R, st));
    HIPCHK(hipMemsetAsync(SL(S, S->icur), 0, 4ull * R, st));
    HIPCHK(hipMemsetAsync(SL(S, S->ebound), 0, 4ull * R, st));
    HIPCHK(hipMemsetAsync(SL(S, S->kprc), 0, 4ull * R, st));
    SpRoute rt;
    memset(&rt, 0, sizeof rt);
    const Msg* in_msgs = S->out[cur];
    const uint32_t* in_pay = S->pool[cur];
    uint32_t nin = M;
    if (!sh) {
      { const int rc = sp_grow(S, &S->status, &S->status_cap, M); if (rc) return rc; }
      rt.msgs = S->out[cur]; rt.M = M; rt.status = S->status; rt.icnt = S->icnt; rt.ebound = S->ebound; rt.kprc = S->kprc;
      rt.pay = S->pool[cur];
      sp_launch(S, SPK_ROUTE, k_sp_route, (M + 255) / 256, 256, d, rt, r, w);
    } else {
      bool any = false;
      { const int rc = sp_exchange_wave(S, M, cur, r, w, &nin, &any); if (rc) return rc; }
      if (!any) { M = 0; break; }                      // no record delivered anywhere: every later wave is empty
      rt.msgs = S->rmsg; rt.M = nin; rt.status = S->rstat; rt.pay = S->rpay;
      in_msgs = S->rmsg; in_pay = S->rpay;
    }
    sp_launch(S, SPK_PAYBOUND, k_sp_paybound, g, tb, d, (const uint32_t*)S->kprc, (const uint32_t*)S->icnt, S->pb);
    {
      const uint32_t* in[3] = {SL(S, S->icnt), SL(S, S->ebound), SL(S, S->pb)};
      uint32_t* out[3] = {SL(S, S->ioff), SL(S, S->eoff), SL(S, S->poff)};
      sp_scan(S, R, 3, in, out, 8);
    }
    HIPCHK(hipMemcpyAsync(tot, S->scan_tot + 8, 12, hipMemcpyDeviceToHost, st));
    HIPCHK(sp_sync(S));
    { const int rc = sp_grow(S, &S->inbox, &S->inbox_cap, tot[0]); if (rc) return rc; }
    { const int rc = sp_grow(S, &S->stage, &S->stage_cap, tot[1]); if (rc) return rc; }
    { const int rc = sp_grow(S, &S->pool[cur ^ 1], &S->pool_cap[cur ^ 1], tot[2]); if (rc) return rc; }
    if (nin) sp_launch(S, SPK_SCATTER, k_sp_scatter, (nin + 255) / 256, 256, rt, (const uint32_t*)S->ioff, S->icur, S->inbox);
    SpWave v;
    v.in = in_msgs; v.pay_in = in_pay; v.inbox = S->inbox; v.ioff = S->ioff; v.icnt = S->icnt;
    SpOut o;
    o.stage = S->stage; o.eoff = S->eoff; o.ecap = S->ebound; o.pay = S->pool[cur ^ 1]; o.poff = S->poff; o.pcap = S->pb;
    o.en = S->en;
    sp_launch(S, SPK_HANDLE, k_sp_handle, g, tb, d, v, o, r);
    {
      const uint32_t* in[1] = {SL(S, S->en)};
      uint32_t* out[1] = {SL(S, S->ooff)};
      sp_scan(S, R, 1, in, out, 12);
    }
    HIPCHK(hipMemcpyAsync(tot, S->scan_tot + 12, 4, hipMemcpyDeviceToHost, st));
    HIPCHK(sp_sync(S));
    M = tot[0];
    { const int rc = sp_grow(S, &S->out[cur ^ 1], &S->out_cap[cur ^ 1], M); if (rc) return rc; }
    sp_launch(S, SPK_COMPACT, k_sp_compact, g, tb, d, o, (const uint32_t*)S->ooff, S->out[cur ^ 1]);
    cur ^= 1;
  }
  if (M) sp_launch(S, SPK_WINDOW, k_sp_window, (M + 255) / 256, 256, d, (const Msg*)S->out[cur], M);   // missed the window
  sp_launch(S, SPK_ROUND_END, k_sp_round_end, 1, 1024, d, r);
  if (sh) {                                          // the mesh's agreement and running counts, and any rank's error
    if (!S->xf->allreduce_sum_u32(d.ctr + C_LASTAGREE, 2, st)) return sp_xfail(S);
    if (!S->xf->allreduce_max_u32(d.ctr + C_ERR, 1, st)) return sp_xfail(S);
  }
  sp_launch(S, SPK_ROUND_END, k_sp_round_conv, 1, 64, d, r);
  if (er[1] || S->prof_level > 0) {
    if (!er[1] && !S->ev_free.empty()) { er[1] = S->ev_free.back(); S->ev_free.pop_back(); }
    if (!er[1]) (void)hipEventCreate(&er[1]);
    (void)hipEventRecord(er[1], st);
    S->recs.push_back(SpSim::Rec{SPK_N, er[0], er[1]});
  }
  uint32_t err = 0;
  HIPCHK(hipMemcpyAsync(&err, d.ctr + C_ERR, 4, hipMemcpyDeviceToHost, st));
  HIPCHK(sp_sync(S));
  if (S->prof_level > 0) sp_prof_resolve(S);
  S->nj = nj_next; S->nf = nf_next;
  S->bj_total += nj_next; S->bf_total += nf_next;
  if (S->n_ext) {                                    // the round's records to external peers, to the host queue
    uint32_t c[2];
    HIPCHK(hipMemcpy(c, d.ctr + C_XREC, 8, hipMemcpyDeviceToHost));
    const uint32_t nrec = std::min(c[0], d.xrec_cap), nid = std::min(c[1], d.xids_cap);
    std::vector<XRec> v(nrec);
    const size_t base = S->xq_ids.size();
    S->xq_ids.resize(base + nid);
    if (nrec) HIPCHK(hipMemcpy(v.data(), d.xrec, sizeof(XRec) * nrec, hipMemcpyDeviceToHost));
    if (nid) HIPCHK(hipMemcpy(S->xq_ids.data() + base, d.xids, 4ull * nid, hipMemcpyDeviceToHost));
    std::sort(v.begin(), v.end(), [](const XRec& a, const XRec& b) {
      return a.wave != b.wave ? a.wave < b.wave : a.sender != b.sender ? a.sender < b.sender : a.seq < b.seq; });
    for (const XRec& q : v) {
      kb_unicast u;
      memcpy(&u, &q, sizeof u);
      u.pay_off = (uint32_t)(base + q.pay_off);
      S->xq.push_back(u);
    }
    const uint32_t z[2] = {0, 0};
    HIPCHK(hipMemcpy(d.ctr + C_XREC, z, 8, hipMemcpyHostToDevice));
  }
  if (np) {                                          // the round's ProbeResponses, (responder, probe) order
    uint32_t k = 0;
    HIPCHK(hipMemcpy(&k, S->d_presp_n, 4, hipMemcpyDeviceToHost));
    k = (uint32_t)std::min<size_t>(k, S->presp_cap);
    std::vector<uint2> v(k);
    if (k) HIPCHK(hipMemcpy(v.data(), S->d_presp, sizeof(uint2) * k, hipMemcpyDeviceToHost));
    std::sort(v.begin(), v.end(), [](const uint2& a, const uint2& b) { return a.x != b.x ? a.x < b.x : a.y < b.y; });
    for (const uint2& q : v) {
      kb_probe_response o;
      memset(&o, 0, sizeof o);
      o.responder = q.x; o.probe = q.y; o.round = r; o.prober = S->probes[q.y];
      o.identity_len = S->h_idlen[q.x];
      memcpy(o.identity, &S->h_ident[(size_t)q.x * MAXID], o.identity_len);
      S->presp.push_back(o);
    }
  }
  S->round = r + 1;
  return sp_err_status(err);
}
static int sp_step(SpSim* S, uint32_t rounds) {
  (void)hipSetDevice(S->device);
  for (uint32_t k = 0; k < rounds; ++k) { const int rc = sp_step_round(S); if (rc) return rc; }
  return KB_OK;
}

// ---- inspection: a row materialised from base Δ x and its entries -----------------------------------
// row inspection is answered by the shard holding the row (KB_INVALID_ARGUMENT on the others)
static int sp_chk_row(SpSim* S, uint32_t node) {
  if (node < S->lo || node >= S->hi) { seterr("the node's row is held by another shard"); return KB_INVALID_ARGUMENT; }
  return KB_OK;
}
static int sp_entries(SpSim* S, uint32_t node, std::vector<uint32_t>& e, uint8_t* based) {
  { const int rc = sp_chk_row(S, node); if (rc) return rc; }
  uint32_t n = 0;
  HIPCHK(hipMemcpy(&n, S->d.ne + node, 4, hipMemcpyDeviceToHost));
  HIPCHK(hipMemcpy(based, S->d.based + node, 1, hipMemcpyDeviceToHost));
  e.resize(n);
  if (n) HIPCHK(hipMemcpy(e.data(), S->d.ent + (size_t)node * S->d.ESTR, 4ull * n, hipMemcpyDeviceToHost));
  return KB_OK;
}
static int sp_read_row(SpSim* S, uint32_t node, std::vector<uint8_t>& rw) {   // canonical bytes (0 = not a member)
  std::vector<uint32_t> e;
  uint8_t based = 0;
  const int rc = sp_entries(S, node, e, &based);
  if (rc) return rc;
  rw.assign(S->C, 0);
  if (based) for (uint32_t j = 0; j < S->C; ++j) if ((S->h_bbits[j >> 5] >> (j & 31)) & 1u) rw[j] = ST_ANCIENT;
  for (uint32_t x : e) {
    const uint32_t j = x >> 9, b = x & 255u;
    const bool mem = (based && ((S->h_bbits[j >> 5] >> (j & 31)) & 1u)) != ((x & SP_XF) != 0);
    rw[j] = mem ? (uint8_t)(b ? b : ST_ANCIENT) : ST_UNKNOWN;
  }
  return KB_OK;
}
static int sp_api_running(SpSim* S, uint32_t node, int* run) {
  for (size_t k = S->events.size(); k-- > 0;) {
    if (S->events[k].node == node) { *run = S->events[k].kind != EV_STOP; return KB_OK; }
    if (S->events[k].kind == EV_RESTART && S->events[k].src == node) { *run = 0; return KB_OK; }
  }
  uint8_t a = 0;
  HIPCHK(hipMemcpy(&a, S->d.alive + node, 1, hipMemcpyDeviceToHost));
  *run = a;
  return KB_OK;
}
static int sp_ever_bound(SpSim* S, uint32_t node, int* ever) {
  for (const Event& e : S->events) if (e.node == node && e.kind != EV_STOP) { *ever = 1; return KB_OK; }
  int32_t sr = 0;
  HIPCHK(hipMemcpy(&sr, S->d.start_round + node, 4, hipMemcpyDeviceToHost));
  *ever = sr != NONE_ROUND;
  return KB_OK;
}
static int sp_start_node(SpSim* S, uint32_t node) {
  int run = 0, ever = 0;
  { int rc = sp_api_running(S, node, &run); if (!rc) rc = sp_ever_bound(S, node, &ever); if (rc) return rc; }
  if (!run && ever) { seterr("a stopped instance restarts at a fresh address (kb_sim_restart_node)"); return KB_INVALID_OPERATION; }
  S->events.push_back(Event{node, EV_START, node, 0});
  return KB_OK;
}
static int sp_stop_node(SpSim* S, uint32_t node) { S->events.push_back(Event{node, EV_STOP, node, 0}); return KB_OK; }
static int sp_restart_node(SpSim* S, uint32_t node, uint32_t* new_node) {
  if (S->h_moved[node]) { seterr("the instance bound here restarted at a fresh address"); return KB_INVALID_OPERATION; }
  int run = 0, ever = 0;
  { int rc = sp_api_running(S, node, &run); if (!rc) rc = sp_ever_bound(S, node, &ever); if (rc) return rc; }
  if (run) { *new_node = node; return KB_OK; }
  if (!ever) { *new_node = node; S->events.push_back(Event{node, EV_START, node, 0}); return KB_OK; }
  uint32_t nf = 0;
  HIPCHK(hipMemcpy(&nf, S->d.ctr + C_NEXTFREE, 4, hipMemcpyDeviceToHost));
  for (; nf < S->C; ++nf) {                          // the next fresh id: never bound, no identity set
    int ev = 0;
    const int rc = sp_ever_bound(S, nf, &ev);
    if (rc) return rc;
    if (!ev && !S->h_idset[nf]) break;
  }
  if (nf >= S->C) { seterr("no fresh address left for the restart (capacity)"); return KB_CAPACITY; }
  const uint32_t to = nf;
  const int pl = S->h_pendlen[node];
  const uint8_t* src = pl >= 0 ? &S->h_pend[(size_t)node * MAXID] : &S->h_ident[(size_t)node * MAXID];
  const uint32_t len = pl >= 0 ? (uint32_t)pl : S->h_idlen[node];
  memmove(&S->h_ident[(size_t)to * MAXID], src, len);
  S->h_idlen[to] = (uint8_t)len;
  S->h_pendlen[node] = -1; S->h_pendlen[to] = -1;
  { const int rc = sp_upload_segments(S); if (rc) return rc; }
  const uint32_t nn = to + 1;
  HIPCHK(hipMemcpy(S->d.ctr + C_NEXTFREE, &nn, 4, hipMemcpyHostToDevice));
  S->events.push_back(Event{to, EV_RESTART, node, 0});
  S->h_moved[node] = 1;
  *new_node = to;
  return KB_OK;
}
static int sp_is_running(SpSim* S, uint32_t node, int* running) {
  uint8_t a = 0;
  HIPCHK(hipMemcpy(&a, S->d.alive + node, 1, hipMemcpyDeviceToHost));
  *running = a;
  return KB_OK;
}
static int sp_ping_addrs(SpSim* S, uint32_t node, const uint32_t* peers, size_t n) {
  for (size_t k = 0; k < n; ++k) if (peers[k] >= S->C) return KB_INVALID_ARGUMENT;
  int run = 0;
  { const int rc = sp_is_running(S, node, &run); if (rc) return rc; }
  if (!run) { seterr("Cannot ping while we are not started"); return KB_INVALID_OPERATION; }
  if (node < S->lo || node >= S->hi) return KB_OK;   // queued by the shard holding the row
  uint32_t qn = 0;
  HIPCHK(hipMemcpy(&qn, S->d.paq_n + node, 4, hipMemcpyDeviceToHost));
  std::vector<uint32_t> q(PAQ);
  HIPCHK(hipMemcpy(q.data(), S->d.paq + (size_t)node * PAQ, 4 * PAQ, hipMemcpyDeviceToHost));
  std::vector<uint8_t> rw;
  { const int rc = sp_read_row(S, node, rw); if (rc) return rc; }
  for (size_t k = 0; k < n; ++k) {
    if (rw[peers[k]]) continue;                      // already known: skipped (src/lib.rs:277-282)
    if (qn == PAQ) { seterr("ping_addrs queue full"); return KB_CAPACITY; }
    q[qn++] = peers[k];
  }
  HIPCHK(hipMemcpy(S->d.paq + (size_t)node * PAQ, q.data(), 4 * PAQ, hipMemcpyHostToDevice));
  HIPCHK(hipMemcpy(S->d.paq_n + node, &qn, 4, hipMemcpyHostToDevice));
  return KB_OK;
}
static int sp_set_identity(SpSim* S, uint32_t node, const uint8_t* identity, size_t len) {
  if (S->h_moved[node]) { seterr("the instance bound here restarted at a fresh address"); return KB_INVALID_OPERATION; }
  int run = 0, ever = 0;
  { int rc = sp_api_running(S, node, &run); if (!rc) rc = sp_ever_bound(S, node, &ever); if (rc) return rc; }
  if (run) { seterr("Cannot change identity while the mesh is running; call .stop first"); return KB_INVALID_OPERATION; }
  if (len != S->cfg.id_len && S->C > 200) { seterr("non-uniform identity length needs capacity <= 200"); return KB_INVALID_ARGUMENT; }
  if (ever) {
    memcpy(&S->h_pend[(size_t)node * MAXID], identity, len);
    S->h_pendlen[node] = (int16_t)len;
    return KB_OK;
  }
  memcpy(&S->h_ident[(size_t)node * MAXID], identity, len);
  S->h_idlen[node] = (uint8_t)len;
  S->h_idset[node] = 1;                            // no longer a fresh id for churn joins and restarts
  { const uint8_t one = 1; HIPCHK(hipMemcpy(S->d.idset + node, &one, 1, hipMemcpyHostToDevice)); }
  { const int rc = sp_upload_segments(S); if (rc) return rc; }
  k_sp_mark_dirty<<<(S->R + 255) / 256, 256, 0, S->st>>>(S->d);
  HIPCHK(hipStreamSynchronize(S->st));
  return KB_OK;
}
static int sp_identity(SpSim* S, uint32_t node, uint8_t* buf, size_t cap, size_t* len) {
  *len = S->h_idlen[node];
  if (!buf) return KB_OK;
  if (cap < *len) return KB_CAPACITY;
  memcpy(buf, &S->h_ident[(size_t)node * MAXID], *len);
  return KB_OK;
}
static int sp_probe_responses(SpSim* S, kb_probe_response* out, size_t cap, size_t* n) {
  *n = S->presp.size();
  if (!out) return KB_OK;
  if (cap < S->presp.size()) return KB_CAPACITY;
  if (!S->presp.empty()) memcpy(out, S->presp.data(), S->presp.size() * sizeof(kb_probe_response));
  S->presp.clear();
  return KB_OK;
}
static int sp_broadcasts(SpSim* S, kb_broadcast* out, size_t cap, size_t* n) {
  std::vector<BCast> j(S->nj), f(S->nf);
  if (S->nj) HIPCHK(hipMemcpy(j.data(), S->bjoin, sizeof(BCast) * S->nj, hipMemcpyDeviceToHost));
  if (S->nf) HIPCHK(hipMemcpy(f.data(), S->bfail, sizeof(BCast) * S->nf, hipMemcpyDeviceToHost));
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
static int sp_fingerprint(SpSim* S, uint32_t node, uint32_t* fp) {
  { const int rc = sp_chk_row(S, node); if (rc) return rc; }
  k_sp_fp_one<<<1, 64, 0, S->st>>>(S->d, node);
  HIPCHK(hipMemcpyAsync(fp, S->d.fp + node, 4, hipMemcpyDeviceToHost, S->st));
  HIPCHK(hipStreamSynchronize(S->st));
  return KB_OK;
}
// all ids; 0 for non-running ids and for rows held by other shards
static int sp_fingerprints(SpSim* S, uint32_t* fps) {
  k_sp_fp_all<<<(S->R + 255) / 256, 256, 0, S->st>>>(S->d);
  std::vector<uint8_t> al(S->C);
  memset(fps, 0, 4ull * S->C);
  HIPCHK(hipMemcpyAsync(fps + S->lo, S->d.fp + S->lo, 4ull * S->R, hipMemcpyDeviceToHost, S->st));
  HIPCHK(hipMemcpyAsync(al.data(), S->d.alive, S->C, hipMemcpyDeviceToHost, S->st));
  HIPCHK(hipStreamSynchronize(S->st));
  for (uint32_t i = 0; i < S->C; ++i) if (!al[i]) fps[i] = 0;
  return KB_OK;
}
static int sp_true_fingerprint(SpSim* S, uint32_t* fp) {
  k_sp_truefp_part<<<SP_TFP / 256, 256, 0, S->st>>>(S->d, S->tfpart);
  k_sp_truefp_fin<<<1, 64, 0, S->st>>>(S->d, (const uint2*)S->tfpart, S->tfp);
  HIPCHK(hipMemcpyAsync(fp, S->tfp, 4, hipMemcpyDeviceToHost, S->st));
  HIPCHK(hipStreamSynchronize(S->st));
  return KB_OK;
}
static int sp_peer_states(SpSim* S, uint32_t node, kb_peer_state* out, size_t cap, size_t* n) {
  { const int rc = sp_chk_row(S, node); if (rc) return rc; }
  std::vector<uint8_t> rw;
  { const int rc = sp_read_row(S, node, rw); if (rc) return rc; }
  Susp sl[SLOTS];
  HIPCHK(hipMemcpy(sl, S->d.susp + (size_t)node * SLOTS, sizeof sl, hipMemcpyDeviceToHost));
  const int32_t E = epoch_base(S->round > 0 ? S->round - 1 : 0);
  size_t c = 0;
  for (uint32_t j = 0; j < S->C; ++j) {
    if (!rw[j]) continue;
    if (out && c < cap) {
      kb_peer_state& o = out[c];
      memset(&o, 0, sizeof o);
      o.peer = j;
      o.identity_len = S->h_idlen[j];
      memcpy(o.identity, &S->h_ident[(size_t)j * MAXID], S->h_idlen[j]);
      o.latency_ms = KB_LATENCY_NONE;
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
static int sp_watch(SpSim* S, uint32_t node) {
  { const int rc = sp_chk_row(S, node); if (rc) return rc; }
  for (uint32_t w : S->watch_node) if (w == node) return KB_OK;
  S->watch_node.push_back(node); S->watch_fp.push_back(0); S->watch_snap.emplace_back(S->C, 0);   // attached empty
  return KB_OK;
}
static int sp_events(SpSim* S, uint32_t node, uint32_t* discovered, size_t cap_d, size_t* n_d, uint32_t* departed, size_t cap_p,
                     size_t* n_p, uint32_t* fp, int* fp_changed) {
  size_t k = 0;
  while (k < S->watch_node.size() && S->watch_node[k] != node) ++k;
  if (k == S->watch_node.size()) { seterr("node is not watched (kb_sim_watch)"); return KB_INVALID_OPERATION; }
  std::vector<uint8_t> rw;
  { const int rc = sp_read_row(S, node, rw); if (rc) return rc; }
  { const int rc = sp_fingerprint(S, node, fp); if (rc) return rc; }
  std::vector<uint8_t>& snap = S->watch_snap[k];
  size_t a = 0, rm = 0, known = 0;
  for (uint32_t j = 0; j < S->C; ++j) {
    const bool now = rw[j] != 0, then = snap[j] != 0;
    known += now; a += now && !then; rm += then && !now;
  }
  *n_d = a; *n_p = rm;
  *fp_changed = known > 0 && *fp != S->watch_fp[k];
  const bool fit = (!a || (discovered && cap_d >= a)) && (!rm || (departed && cap_p >= rm));
  if (!fit) {
    if (discovered || departed) { seterr("event buffer too small"); return KB_CAPACITY; }
    return KB_OK;
  }
  a = rm = 0;
  for (uint32_t j = 0; j < S->C; ++j) {
    const bool now = rw[j] != 0, then = snap[j] != 0;
    if (now && !then) discovered[a++] = j;
    if (then && !now) departed[rm++] = j;
    snap[j] = (uint8_t)now;
  }
  if (*fp_changed) S->watch_fp[k] = *fp;
  return KB_OK;
}
static int sp_fold_stats(SpSim* S) {
  (void)hipSetDevice(S->device);
  k_sp_stats_fold<<<NSTAT, 256, 0, S->st>>>(S->d);
  HIPCHK(hipStreamSynchronize(S->st));
  return KB_OK;
}
// this shard's counters (ranks of kb_sim_create_rank: summed over the mesh, a collective)
static int sp_read_stats(SpSim* S, unsigned long long* st) {
  { const int rc = sp_fold_stats(S); if (rc) return rc; }
  if (S->xf && !S->in_group) {
    HIPCHK(hipMemcpyAsync(S->xstats, S->d.stats, 8ull * NSTAT, hipMemcpyDeviceToDevice, S->st));
    if (!S->xf->allreduce_sum_u64(S->xstats, NSTAT, S->st)) return sp_xfail(S);
    HIPCHK(hipMemcpyAsync(st, S->xstats, 8ull * NSTAT, hipMemcpyDeviceToHost, S->st));
    HIPCHK(hipStreamSynchronize(S->st));
    return KB_OK;
  }
  HIPCHK(hipMemcpy(st, S->d.stats, 8ull * NSTAT, hipMemcpyDeviceToHost));
  return KB_OK;
}
// kb_stats from the mesh's counters `st` and this shard's replicated facts
static int sp_stats_fill(SpSim* S, const unsigned long long* st, kb_stats* out) {
  uint32_t ctr[NCTR];
  HIPCHK(hipMemcpy(ctr, S->d.ctr, sizeof ctr, hipMemcpyDeviceToHost));
  std::vector<uint8_t> al(S->C);
  HIPCHK(hipMemcpy(al.data(), S->d.alive, S->C, hipMemcpyDeviceToHost));
  memset(out, 0, sizeof *out);
  out->round = S->round;
  uint32_t a = 0;
  for (uint8_t x : al) a += x;
  out->alive = a;
  out->agree = ctr[C_LASTAGREE];
  out->first_converged_round = (int32_t)ctr[C_FIRSTCONV];
  out->last_converged_round = (int32_t)ctr[C_LASTCONV];
  out->next_free_id = ctr[C_NEXTFREE];
  out->sent_ping = st[S_PING]; out->sent_ping_req = st[S_PINGREQ]; out->sent_ack = st[S_ACK];
  out->sent_known_peers = st[S_KP]; out->sent_kpr = st[S_KPR];
  out->bcast_join = S->bj_total; out->bcast_failed = S->bf_total;
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
static int sp_stats_out(SpSim* S, kb_stats* out) {
  unsigned long long st[NSTAT];
  { const int rc = sp_read_stats(S, st); if (rc) return rc; }
  return sp_stats_fill(S, st, out);
}
// per id: alive, n, last_bcast, start_round; n and last_bcast only for the rows this handle holds
static int sp_dump_scalars(SpSim* S, int32_t* out) {
  const uint32_t C = S->C, R = S->R;
  std::vector<uint8_t> al(C);
  std::vector<uint32_t> n(R);
  std::vector<int32_t> lb(R), sr(C);
  HIPCHK(hipMemcpy(al.data(), S->d.alive, C, hipMemcpyDeviceToHost));
  HIPCHK(hipMemcpy(n.data(), SL(S, S->d.n), 4ull * R, hipMemcpyDeviceToHost));
  HIPCHK(hipMemcpy(lb.data(), SL(S, S->d.last_bcast), 4ull * R, hipMemcpyDeviceToHost));
  HIPCHK(hipMemcpy(sr.data(), S->d.start_round, 4ull * C, hipMemcpyDeviceToHost));
  for (uint32_t i = 0; i < C; ++i) {
    const bool loc = i >= S->lo && i < S->hi;
    out[4 * i] = al[i]; out[4 * i + 1] = loc ? (int32_t)n[i - S->lo] : 0;
    out[4 * i + 2] = loc ? lb[i - S->lo] : 0; out[4 * i + 3] = sr[i];
  }
  return KB_OK;
}
static int sp_dump_suspects(SpSim* S, uint32_t node, int32_t* out, size_t cap, size_t* n) {
  { const int rc = sp_chk_row(S, node); if (rc) return rc; }
  Susp sl[SLOTS];
  HIPCHK(hipMemcpy(sl, S->d.susp + (size_t)node * SLOTS, sizeof sl, hipMemcpyDeviceToHost));
  std::vector<std::array<int32_t, 3>> v;
  for (auto& x : sl) if (x.kind) v.push_back({(int32_t)x.peer, x.kind, x.since});
  std::sort(v.begin(), v.end());
  *n = v.size();
  if (out) { if (cap < 3 * v.size()) return KB_CAPACITY; for (size_t k = 0; k < v.size(); ++k) memcpy(out + 3 * k, v[k].data(), 12); }
  return KB_OK;
}
static int sp_dump_curious(SpSim* S, uint32_t node, int32_t* out, size_t cap, size_t* n) {
  { const int rc = sp_chk_row(S, node); if (rc) return rc; }
  Cur cu[CSLOTS];
  HIPCHK(hipMemcpy(cu, S->d.cur + (size_t)node * CSLOTS, sizeof cu, hipMemcpyDeviceToHost));
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
// kb_sim_kernel_time kinds: the whole round; the tick (KB_KT_ROWPASS's place: the per-row pass of the round);
// the in-order handlers (KB_KT_PROC)
static int sp_kernel_time(SpSim* S, int kind, double* ms, uint64_t* launches) {
  (void)hipStreamSynchronize(S->st);
  sp_prof_resolve(S);
  const int k = kind == KB_KT_ROUND ? SPK_N : kind == KB_KT_ROWPASS ? SPK_TICK : kind == KB_KT_PROC ? SPK_HANDLE : -1;
  if (k < 0) return KB_INVALID_ARGUMENT;
  if (k == SPK_N) { *ms = S->round_ms; *launches = S->round_n; }
  else { *ms = S->k_ms[k]; *launches = S->k_n[k]; }
  return KB_OK;
}
static int sp_reset_kernel_time(SpSim* S) {
  (void)hipStreamSynchronize(S->st);
  sp_prof_resolve(S);
  S->round_ms = 0; S->round_n = 0;
  memset(S->k_ms, 0, sizeof S->k_ms); memset(S->k_n, 0, sizeof S->k_n);
  return KB_OK;
}
static int sp_kernel_breakdown(SpSim* S, kb_kernel_time* out, size_t cap, size_t* n) {
  (void)hipStreamSynchronize(S->st);
  sp_prof_resolve(S);
  size_t c = 0;
  for (int k = 0; k < SPK_N; ++k) {
    if (!S->k_n[k]) continue;
    if (out && c < cap) {
      kb_kernel_time& o = out[c];
      memset(&o, 0, sizeof o);
      snprintf(o.name, sizeof o.name, "%s", SPK_NAME[k]);
      o.ms = S->k_ms[k]; o.launches = S->k_n[k];
    }
    c++;
  }
  *n = c;
  return (out && cap < c) ? KB_CAPACITY : KB_OK;
}
// external peers: the dense engine's rules (kb_sim.hip kb_sim_set_external / inject / exported)
static int sp_set_external(SpSim* S, uint32_t node) {
  if (S->h_ext.empty()) S->h_ext.assign(S->C, 0);
  if (S->h_ext[node]) return KB_OK;
  int ever = 0;
  { const int rc = sp_ever_bound(S, node, &ever); if (rc) return rc; }
  if (ever) { seterr("an external peer takes an address no instance has bound"); return KB_INVALID_OPERATION; }
  S->h_ext[node] = 1; S->n_ext++; S->h_idset[node] = 1;
  const uint8_t o = 1;
  HIPCHK(hipMemcpy(S->d.ext + node, &o, 1, hipMemcpyHostToDevice));
  HIPCHK(hipMemcpy(S->d.idset + node, &o, 1, hipMemcpyHostToDevice));
  if (!S->d.xrec) {
    S->d.xrec_cap = 1u << 16; S->d.xids_cap = 1u << 22;
    HIPCHK(sp_alloc(S, &S->d.xrec, S->d.xrec_cap)); HIPCHK(sp_alloc(S, &S->d.xids, S->d.xids_cap));
  }
  return KB_OK;
}
static int sp_inject(SpSim* S, const kb_unicast* m, const uint32_t* ids) {
  if (!m || m->sender >= S->C || m->dest >= S->C || (m->kind > K_KPR && m->kind != KB_WIRE_JOIN) || (m->pay_len && !ids))
    return KB_INVALID_ARGUMENT;
  if (S->h_ext.empty() || !S->h_ext[m->sender]) { seterr("kb_sim_inject: the sender is not an external peer"); return KB_INVALID_OPERATION; }
  if (m->kind == KB_WIRE_JOIN) {                       // a Join broadcast: the next round's Join list
    if (std::find(S->inj_join.begin(), S->inj_join.end(), m->sender) != S->inj_join.end()) {
      seterr("kb_sim_inject: one Join per external peer per round"); return KB_CAPACITY;
    }
    S->inj_join.push_back(m->sender);
    return KB_OK;
  }
  if ((m->kind == K_PINGREQ || m->kind == K_ACK) && m->a >= S->C) return KB_INVALID_ARGUMENT;
  for (uint32_t k = 0; k < m->pay_len; ++k) if (ids[k] >= S->C) return KB_INVALID_ARGUMENT;
  uint32_t per = 0, rel = 0;
  for (const XRec& x : S->inj) if (x.sender == m->sender) { per++; if (x.kind == K_KP) rel += x.pay_len; }
  if (per >= (uint32_t)TICK_MAX) { seterr("kb_sim_inject: 33 records per external peer per round"); return KB_CAPACITY; }
  XRec x{0, 0, m->sender, m->dest, 0, m->kind, m->kind == K_KP ? 0u : m->a, m->fp, m->n, (uint32_t)S->inj_ids.size(),
         m->kind == K_KP ? m->pay_len : 0u, rel};
  if (m->kind == K_KP) S->inj_ids.insert(S->inj_ids.end(), ids, ids + m->pay_len);
  S->inj.push_back(x);
  return KB_OK;
}
static int sp_exported(SpSim* S, kb_unicast* out, size_t cap, size_t* n, uint32_t* ids, size_t cap_ids, size_t* n_ids) {
  *n = S->xq.size(); *n_ids = S->xq_ids.size();
  if (!out && !ids) return KB_OK;
  if (cap < S->xq.size() || (!S->xq_ids.empty() && (!ids || cap_ids < S->xq_ids.size()))) { seterr("export buffer too small"); return KB_CAPACITY; }
  if (!S->xq.empty()) memcpy(out, S->xq.data(), S->xq.size() * sizeof(kb_unicast));
  for (const kb_unicast& u : S->xq)                    // a KnownPeers map has no order: ascending ids
    std::sort(S->xq_ids.begin() + u.pay_off, S->xq_ids.begin() + u.pay_off + u.pay_len);
  if (!S->xq_ids.empty()) memcpy(ids, S->xq_ids.data(), 4 * S->xq_ids.size());
  S->xq.clear(); S->xq_ids.clear();
  return KB_OK;
}
// the sparse layout's footprint (test surface): [rows based, exceptions, explicit stamps, entries of the
// largest row, bytes (4 per entry), rows], the oracle's kbo_sparse_footprint in this layout
static int sp_footprint(SpSim* S, uint64_t* out, size_t cap) {   // over the rows this handle holds
  if (cap < 6) return KB_INVALID_ARGUMENT;
  const uint32_t lo = S->lo, hi = S->hi, R = S->R;
  std::vector<uint32_t> ne(R);
  std::vector<uint8_t> based(R);
  HIPCHK(hipMemcpy(ne.data(), SL(S, S->d.ne), 4ull * R, hipMemcpyDeviceToHost));
  HIPCHK(hipMemcpy(based.data(), SL(S, S->d.based), R, hipMemcpyDeviceToHost));
  uint64_t nb = 0, tot = 0, mx = 0;
  for (uint32_t k = 0; k < R; ++k) { nb += based[k]; tot += ne[k]; mx = std::max<uint64_t>(mx, ne[k]); }
  out[0] = nb; out[1] = 0; out[2] = 0; out[3] = mx; out[4] = 4 * tot; out[5] = R;
  // exceptions / explicit stamps: counted exactly on the host in chunks
  const size_t chunk = std::max<size_t>(1, (size_t)(256u << 20) / (4ull * S->d.ESTR));
  std::vector<uint32_t> buf;
  for (uint32_t i0 = lo; i0 < hi; i0 += (uint32_t)chunk) {
    const uint32_t i1 = (uint32_t)std::min<size_t>(hi, i0 + chunk);
    buf.resize((size_t)(i1 - i0) * S->d.ESTR);
    HIPCHK(hipMemcpy(buf.data(), S->d.ent + (size_t)i0 * S->d.ESTR, 4ull * buf.size(), hipMemcpyDeviceToHost));
    for (uint32_t i = i0; i < i1; ++i)
      for (uint32_t q = 0; q < ne[i - lo]; ++q) {
        const uint32_t x = buf[(size_t)(i - i0) * S->d.ESTR + q];
        out[1] += (x & SP_XF) != 0; out[2] += (x & 255u) != 0;
      }
  }
  return KB_OK;
}

}  // namespace kb
