/*
 * kb_oracle.c — CPU restatement of Kaboodle's SWIM round ("round semantics v1").
 *
 * TEST INFRASTRUCTURE ONLY.  This file is the parity oracle: tests/, __graft_entry__.smoke() and the
 * cpu_baseline leg of bench.py may load it; the product (kaboodle_amd/, include/) never does.
 *
 * It follows the reference handler by handler, in its order (paths relative to the reference root):
 *   tick order               src/kaboodle.rs:746-779   (join -> suspects -> ping -> ping_addrs -> window)
 *   maybe_broadcast_join     src/kaboodle.rs:228-251
 *   handle_suspected_peers   src/kaboodle.rs:558-653
 *   ping_random_peer         src/kaboodle.rs:655-703
 *   handle_incoming_ping_requests src/kaboodle.rs:550-556
 *   handle_incoming_broadcasts    src/kaboodle.rs:256-311 (Failed :268-283, Join :284-304)
 *   should_respond_to_broadcast   src/kaboodle.rs:333-354
 *   maybe_send_known_peers_to_peer src/kaboodle.rs:356-392
 *   handle_incoming_messages      src/kaboodle.rs:394-548 (prologue :406-415, Ack :418-447,
 *                                  KnownPeers :448-472, KnownPeersRequest :473-512, Ping :513-532,
 *                                  PingRequest :533-545)
 *   maybe_sync_known_peers   src/kaboodle.rs:707-740
 *   generate_fingerprint     src/kaboodle.rs:71-83
 *   ObservableHashMap insert/remove/update  src/observable_hashmap.rs:84-142
 *   Kaboodle::start/stop/ping_addrs/set_identity  src/lib.rs:136-183, 268-297, 323-336
 *
 * Data layout is deliberately the same dense representation the GPU uses (stamp byte per (node, peer),
 * DESIGN.md §2.2), because the declared stamp window (rebase every 64 rounds, "ancient" saturation)
 * is part of the semantics.  Everything else is plain sequential code: every node processes its
 * inbox one message at a time, exactly like the reference's receive loop.
 */
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#include <stdio.h>
#include <limits.h>
#ifdef _OPENMP
#include <omp.h>
#endif
#include "../include/kaboodle_sim.h"
#include "kb_oracle_prims.h"

/* ---- constants (src/kaboodle.rs:38-65), in rounds ----------------------------------------------- */
#define PING_TIMEOUT 2          /* PING_TIMEOUT 2000 ms            :62 */
#define SHARE_AGE 10            /* MAX_PEER_SHARE_AGE 10000 ms     :49 */
#define REBROADCAST 10          /* REBROADCAST_INTERVAL 10000 ms   :65 */
#define NUM_INDIRECT 3          /* NUM_INDIRECT_PING_PEERS         :52 */
#define NUM_CANDIDATES 5        /* NUM_CANDIDATE_TARGET_PEERS      :57 */
#define BUFSZ 10240             /* INCOMING_BUFFER_SIZE            :43 */
/* declared capacities */
#define SLOTS 8
#define CSLOTS 8
#define NOBS 4
#define PAQ 8
#define MAXID 32
#define ADDR_LEN 20
/* stamp encoding */
#define ST_UNKNOWN 0
#define ST_SUSPECT 1
#define ST_ANCIENT 2
#define EPOCH 64
#define EOFF 192
/* message kinds (SwimMessage, src/structs.rs:94-116) */
enum { K_PING = 0, K_PINGREQ = 1, K_ACK = 2, K_KP = 3, K_KPR = 4 };
/* Philox purposes */
enum { P_PING = 1, P_INDIRECT = 2, P_RESPOND = 3, P_TRUNC = 4, P_LOSS = 5, P_BLOSS = 6, P_CHURN = 7, P_PROBE = 8 };
enum { SK_WFP = 1, SK_WFIP = 2 };

typedef struct { uint32_t peer; int32_t since; int32_t kind; } osusp;       /* kind 0 = free */
typedef struct { uint32_t peer; uint32_t nobs; uint32_t obs[NOBS]; int32_t used; } ocur;
typedef struct {
  uint32_t dest, sender, seq, kind;
  uint32_t a, fp, n;
  uint32_t* pay; uint32_t pay_len;
} omsg;
typedef struct { omsg* v; size_t n, cap; } ovec;
typedef struct { uint32_t sender, peer, bseq; } obcast;
typedef struct { int kind; uint32_t node, src; } oevent;   /* kind: EV_START / EV_STOP / EV_RESTART (node = new id, src = old) */
enum { EV_START = 0, EV_STOP = 1, EV_RESTART = 2 };

struct kbo_sim {
  kb_config cfg;
  uint32_t C;
  uint32_t k0, k1;
  uint8_t* stamp;              /* C x C dense stamp rows (NULL with KB_VARIANT_SPARSE_ROWS: sr below) */
  struct srow* sr;             /* KB_VARIANT_SPARSE_ROWS: per-row exceptions + explicit stamps */
  uint32_t* bbits;             /* sparse: the shared base set (the initial members), bitset */
  uint32_t* bcnt;              /* sparse: bcnt[k] = |base ∩ [0, k)|, k = 0..C */
  uint32_t* bpre;              /* sparse: bpre[k] = crc0 fold of base ∩ [0, k) (uniform identities), k = 0..C */
  uint32_t* zpw;               /* sparse: Z^k, k = 0..C+1 */
  int32_t* tst;               /* C x C, KB_VARIANT_EXACT_LRU: the exact instant of every Known entry */
  uint16_t* lat;              /* C x C PeerInfo.latency in ms, LAT_NONE = None (track_latency only) */
  uint8_t* alive;
  int32_t* start_round;
  uint32_t* n;
  uint32_t* fp;
  uint8_t* dirty;
  int32_t* last_bcast;
  uint32_t* a3cur;            /* A3's rotation base: just before the last round's oldest candidate (§2.6) */
  osusp* susp;                /* C x SLOTS */
  ocur* cur;                  /* C x CSLOTS */
  uint32_t* paq; uint32_t* paq_n;
  uint8_t* ident; uint8_t* id_len;
  uint8_t* pend_ident; int16_t* pend_len;   /* identity set on a stopped instance, taken by its next address (-1: none) */
  uint8_t* moved;                           /* the instance bound here restarted at a fresh address */
  uint8_t* idset;                           /* an identity was set on this never-bound address (not fresh) */
  uint8_t* ext;                             /* external peer: a real instance outside the mesh */
  omsg* inj; size_t ninj, capinj;           /* records from external peers, delivered in the next round's wave 0 */
  uint32_t* injj; size_t ninjj, capinjj;    /* external peers' Join broadcasts, merged into the next round's list */
  kb_unicast* xp; size_t nxp, capxp;        /* records routed to external peers, not drained yet */
  uint32_t* xids; size_t nxids, capxids;    /*   and the ids of their KnownPeers lists */
  uint32_t* cseg; uint32_t* segmul;   /* crc0(addr||identity), x^(8*seglen) */
  uint32_t* seglen;
  uint32_t mulz_tab[4][256]; int uniform; uint32_t ulen;
  uint32_t mulzk_tab[9][4][256];     /* multiply by Z^k, k = 0..8 (Z = x^(8 ulen)) */
  uint32_t* htab;                    /* [C/8 + 1][256] crc0 fold of each member pattern of each 8-id block */
  uint8_t pop8[256];
  uint32_t* hfull;                   /* [C/8 + 1] htab[b][255], contiguous: full blocks (converged rows) stream */
  int32_t round;
  uint32_t next_free;
  obcast* bfail; size_t nbfail, capbfail;
  obcast* bjoin; size_t nbjoin, capbjoin;
  oevent* ev; size_t nev, capev;
  kb_wire_addr* probe_q; size_t nprobe_q, capprobe_q;   /* Probes queued for the next round (kbo_sim_probe) */
  kb_wire_addr* probes; size_t nprobes;                   /* the Probes delivered this round */
  kb_probe_response* presp; size_t npresp, cappresp;     /* responses not yet drained */
  ovec* out;                  /* per-node outbox of the wave being produced */
  uint32_t* oseq;             /* per-node emission counter for the wave being produced */
  kb_stats st;
  /* event observers (kbo_sim_watch): watched node, its membership at the last drain, last reported fp */
  uint32_t* wnode; uint8_t** wsnap; uint32_t* wfp; size_t nwatch;
};
typedef struct kbo_sim kbo_sim;

int kbo_sim_destroy(kbo_sim* s);
static int fresh_id(const kbo_sim* s, uint32_t id);
static char g_err[256];
static void seterr(const char* m) { snprintf(g_err, sizeof g_err, "%s", m); }
const char* kbo_last_error(void) { return g_err; }

/* ---- helpers ------------------------------------------------------------------------------------ */
static inline int32_t epoch_base(int32_t r) { return (r / EPOCH) * EPOCH; }
/* encode Known(t) at round r (t <= r) */
static inline uint8_t enc(int32_t t, int32_t r) {
  int32_t v = t - epoch_base(r) + EOFF;
  if (v < ST_ANCIENT) v = ST_ANCIENT;
  if (v > 255) v = 255;
  return (uint8_t)v;
}
static inline uint8_t* row(kbo_sim* s, uint32_t i) { return s->stamp + (size_t)i * s->C; }

/* ---- sparse rows (KB_VARIANT_SPARSE_ROWS) -----------------------------------------------
 * A view holds members = base Δ x (or x alone for a row that never adopted the base, e.g. a fresh joiner)
 * and stamps: ANCIENT (2) for every member without an explicit entry, else the entry's byte (1 = suspect,
 * > 2 = Known within the stamp window).  base is the initial member set, shared by every row.  The round
 * touches rows through st_get / st_set and the sparse algorithms below (A3 from the rotated base order,
 * KnownPeersRequest replies from the explicit list, the fingerprint from base prefix folds corrected at
 * the exceptions); everything else materialises a row on demand. */
struct srow {
  uint32_t* x; uint32_t nx, capx;                  /* sorted ids where the row differs from its base */
  uint32_t* lid; uint8_t* lb; uint32_t nl, capl;   /* sorted explicit stamps (members only) */
  uint8_t based;                                   /* members = base Δ x (1) or x (0) */
  uint32_t adopt_at;                               /* unbased: |x| at which adopting the base is tried next */
};
typedef struct srow srow;
static inline int bbit(const kbo_sim* s, uint32_t j) { return (int)((s->bbits[j >> 5] >> (j & 31)) & 1u); }
static uint32_t lbound(const uint32_t* v, uint32_t n, uint32_t key) {
  uint32_t lo = 0, hi = n;
  while (lo < hi) { const uint32_t mid = lo + (hi - lo) / 2; if (v[mid] < key) lo = mid + 1; else hi = mid; }
  return lo;
}
static inline int x_has(const srow* r, uint32_t j) { const uint32_t k = lbound(r->x, r->nx, j); return k < r->nx && r->x[k] == j; }
static void x_toggle(srow* r, uint32_t j) {
  const uint32_t k = lbound(r->x, r->nx, j);
  if (k < r->nx && r->x[k] == j) { memmove(r->x + k, r->x + k + 1, (r->nx - k - 1) * 4u); r->nx--; return; }
  if (r->nx == r->capx) { r->capx = r->capx ? 2 * r->capx : 16; r->x = (uint32_t*)realloc(r->x, r->capx * 4u); }
  memmove(r->x + k + 1, r->x + k, (r->nx - k) * 4u);
  r->x[k] = j; r->nx++;
}
static inline uint8_t l_get(const srow* r, uint32_t j) { const uint32_t k = lbound(r->lid, r->nl, j); return k < r->nl && r->lid[k] == j ? r->lb[k] : 0; }
static void l_set(srow* r, uint32_t j, uint8_t b) {               /* b = 0 or ANCIENT: no explicit entry */
  const uint32_t k = lbound(r->lid, r->nl, j);
  const int has = k < r->nl && r->lid[k] == j;
  if (b == ST_UNKNOWN || b == ST_ANCIENT) {
    if (has) { memmove(r->lid + k, r->lid + k + 1, (r->nl - k - 1) * 4u); memmove(r->lb + k, r->lb + k + 1, r->nl - k - 1); r->nl--; }
    return;
  }
  if (has) { r->lb[k] = b; return; }
  if (r->nl == r->capl) {
    r->capl = r->capl ? 2 * r->capl : 16;
    r->lid = (uint32_t*)realloc(r->lid, r->capl * 4u); r->lb = (uint8_t*)realloc(r->lb, r->capl);
  }
  memmove(r->lid + k + 1, r->lid + k, (r->nl - k) * 4u); memmove(r->lb + k + 1, r->lb + k, r->nl - k);
  r->lid[k] = j; r->lb[k] = b; r->nl++;
}
static inline int s_mem(const kbo_sim* s, uint32_t i, uint32_t j) {
  const srow* r = &s->sr[i];
  return (r->based ? bbit(s, j) : 0) ^ x_has(r, j);
}
/* the stamp byte of (i, j) in either layout (0 = not a member) */
static inline uint8_t st_get(kbo_sim* s, uint32_t i, uint32_t j) {
  if (!s->sr) return row(s, i)[j];
  if (!s_mem(s, i, j)) return ST_UNKNOWN;
  const uint8_t b = l_get(&s->sr[i], j);
  return b ? b : ST_ANCIENT;
}
static void adopt_base(kbo_sim* s, uint32_t i);
static inline void st_set(kbo_sim* s, uint32_t i, uint32_t j, uint8_t b) {
  if (!s->sr) { row(s, i)[j] = b; return; }
  srow* r = &s->sr[i];
  if ((b != ST_UNKNOWN) != s_mem(s, i, j)) x_toggle(r, j);
  l_set(r, j, b);
  if (!r->based && r->nx > r->adopt_at) adopt_base(s, i);
}
/* the row's members as base Δ x once base describes it better (a joiner that has learned the mesh) */
static void adopt_base(kbo_sim* s, uint32_t i) {
  srow* r = &s->sr[i];
  uint32_t* nx = (uint32_t*)malloc(sizeof(uint32_t) * (s->C ? s->C : 1));
  uint32_t c = 0, k = 0;
  for (uint32_t j = 0; j < s->C; ++j) {
    const int in_x = k < r->nx && r->x[k] == j;
    k += in_x;
    if (bbit(s, j) != in_x) nx[c++] = j;                 /* member in exactly one of base, row */
  }
  if (c >= r->nx) { free(nx); r->adopt_at = 2 * r->adopt_at + 64; return; }
  free(r->x);
  r->x = nx; r->nx = c; r->capx = s->C; r->based = 1;
}
/* the row as dense bytes (inspection and the rare whole-row scans) */
static void row_bytes(kbo_sim* s, uint32_t i, uint8_t* out) {
  if (!s->sr) { memcpy(out, row(s, i), s->C); return; }
  const srow* r = &s->sr[i];
  for (uint32_t j = 0; j < s->C; ++j) out[j] = (r->based && bbit(s, j)) ? ST_ANCIENT : ST_UNKNOWN;
  for (uint32_t k = 0; k < r->nx; ++k) out[r->x[k]] = out[r->x[k]] ? ST_UNKNOWN : ST_ANCIENT;
  for (uint32_t k = 0; k < r->nl; ++k) out[r->lid[k]] = r->lb[k];
}
/* the row for inspection: the dense row itself, or a materialised copy (*tmp, freed by the caller) */
static const uint8_t* row_view(kbo_sim* s, uint32_t i, uint8_t** tmp) {
  *tmp = NULL;
  if (!s->sr) return row(s, i);
  *tmp = (uint8_t*)malloc(s->C ? s->C : 1);
  row_bytes(s, i, *tmp);
  return *tmp;
}
static void srow_free(srow* r) { free(r->x); free(r->lid); free(r->lb); memset(r, 0, sizeof *r); }
static void srow_copy(srow* d, const srow* r) {
  srow_free(d);
  *d = *r;
  d->capx = r->nx; d->capl = r->nl;
  d->x = (uint32_t*)malloc(4u * (r->nx ? r->nx : 1)); memcpy(d->x, r->x, 4u * r->nx);
  d->lid = (uint32_t*)malloc(4u * (r->nl ? r->nl : 1)); memcpy(d->lid, r->lid, 4u * r->nl);
  d->lb = (uint8_t*)malloc(r->nl ? r->nl : 1); memcpy(d->lb, r->lb, r->nl);
}
static inline int active_faults(kbo_sim* s, int32_t r) { return s->cfg.fault_end_round < 0 || r < s->cfg.fault_end_round; }
static inline o_u32x4 ph(kbo_sim* s, uint32_t c0, uint32_t c1, uint32_t c2, uint32_t c3) {
  return o_philox(c0, c1, c2, c3, s->k0, s->k1);
}
static inline int partition_blocks(kbo_sim* s, int32_t r, uint32_t a, uint32_t b) {
  uint32_t G = s->cfg.partition_groups;
  if (G <= 1 || r < s->cfg.partition_start || r >= s->cfg.partition_end) return 0;
  uint64_t ga = (uint64_t)a * G / s->C, gb = (uint64_t)b * G / s->C;
  return ga != gb;
}

int kbo_format_addr(uint32_t id, char* buf, size_t cap) {
  char tmp[32];
  int len = snprintf(tmp, sizeof tmp, "10.100.100.%u:%u", 100u + id / 50000u, 10000u + id % 50000u);
  if (!buf || cap < (size_t)len + 1) return KB_INVALID_ARGUMENT;
  memcpy(buf, tmp, (size_t)len + 1);
  return KB_OK;
}

static void default_identity(uint32_t id, uint32_t len, uint8_t* out) {
  for (uint32_t k = 0; k < len; ++k) out[k] = (uint8_t)('a' + ((id * 31u + k * 7u) % 26u));
}

static void htab_block(kbo_sim* s, uint32_t b);
static void compute_seg(kbo_sim* s, uint32_t id) {
  char a[32];
  kbo_format_addr(id, a, sizeof a);
  uint32_t reg = o_crc_update(0, (const uint8_t*)a, ADDR_LEN);
  reg = o_crc_update(reg, s->ident + (size_t)id * MAXID, s->id_len[id]);
  s->cseg[id] = reg;
  s->seglen[id] = ADDR_LEN + s->id_len[id];
  s->segmul[id] = o_xpow8(s->seglen[id]);
  if (s->htab) htab_block(s, id / 8);
}

static void build_mulz(kbo_sim* s) {
  uint32_t z = o_xpow8(s->ulen);
  for (int k = 0; k < 4; ++k)
    for (uint32_t v = 0; v < 256; ++v) s->mulz_tab[k][v] = o_multmodp(z, v << (8 * k));
  for (uint32_t m = 0; m < 256; ++m) s->pop8[m] = (uint8_t)__builtin_popcount(m);
  uint32_t zk = 0x80000000u;                       /* x^0 */
  for (int c = 0; c <= 8; ++c) {
    for (int k = 0; k < 4; ++k)
      for (uint32_t v = 0; v < 256; ++v) s->mulzk_tab[c][k][v] = o_multmodp(zk, v << (8 * k));
    zk = o_multmodp(z, zk);
  }
}
static inline uint32_t mulz(const kbo_sim* s, uint32_t a) {
  return s->mulz_tab[0][a & 0xFF] ^ s->mulz_tab[1][(a >> 8) & 0xFF] ^ s->mulz_tab[2][(a >> 16) & 0xFF] ^
         s->mulz_tab[3][a >> 24];
}
static inline uint32_t mulzk(const kbo_sim* s, uint32_t c, uint32_t a) {
  return s->mulzk_tab[c][0][a & 0xFF] ^ s->mulzk_tab[c][1][(a >> 8) & 0xFF] ^ s->mulzk_tab[c][2][(a >> 16) & 0xFF] ^
         s->mulzk_tab[c][3][a >> 24];
}
/* the fold of every member pattern m of ids 8b..8b+7 (uniform identities): H[m] = H[m - top bit t]·Z ⊕ cseg[8b + t] */
static void htab_block(kbo_sim* s, uint32_t b) {
  uint32_t* h = s->htab + (size_t)b * 256;
  h[0] = 0;
  for (uint32_t m = 1; m < 256; ++m) {
    uint32_t t = 7;
    while (!((m >> t) & 1u)) --t;
    const uint32_t j = 8 * b + t;
    h[m] = j < s->C ? (mulz(s, h[m & ~(1u << t)]) ^ s->cseg[j]) : 0;
  }
  s->hfull[b] = h[255];
}

/* generate_fingerprint (src/kaboodle.rs:71-83): CRC-32 over addr.to_string() || identity of every
 * entry in ascending address order (= ascending id).  Computed by folding the per-peer segment CRCs:
 * crc0(A||B) = crc0(A)*x^(8|B|) ^ crc0(B); final = crc0 ^ 0xFFFFFFFF*x^(8 len) ^ 0xFFFFFFFF. */
static uint32_t fold_bytes(kbo_sim* s, const uint8_t* rw) {
  uint32_t raw = 0; uint64_t len = 0;
  if (s->uniform) {                  /* 8 ids at a time: raw·Z^popcount(m) ⊕ H[block][m] (the same fold, fewer steps), */
    uint64_t cnt = 0;                /* four independent chains over quarters of the row, joined by Z^count multiplies */
    const uint32_t nb = s->C / 8, q4 = (nb + 3) / 4;
    uint32_t rq[4] = {0, 0, 0, 0}, cq[4] = {0, 0, 0, 0};
    for (uint32_t t = 0; t < q4; ++t) {
      for (int q = 0; q < 4; ++q) {
        const uint32_t b = (uint32_t)q * q4 + t;
        if (b >= nb) continue;
        uint64_t v;
        memcpy(&v, rw + 8 * (size_t)b, 8);
        uint64_t h = (((v & 0x7F7F7F7F7F7F7F7Full) + 0x7F7F7F7F7F7F7F7Full) | v) & 0x8080808080808080ull;
        const uint32_t m = (uint32_t)(((h >> 7) * 0x0102040810204080ull) >> 56);   /* bit k: byte k nonzero */
        if (!m) continue;
        const uint32_t c = s->pop8[m];
        rq[q] = mulzk(s, c, rq[q]) ^ (m == 255u ? s->hfull[b] : s->htab[(size_t)b * 256 + m]);
        cq[q] += c;
      }
    }
    for (int q = 0; q < 4; ++q) {
      if (!cq[q]) continue;
      raw = o_multmodp(o_xpow8((uint64_t)cq[q] * s->ulen), raw) ^ rq[q];
      cnt += cq[q];
    }
    for (uint32_t j = 8 * nb; j < s->C; ++j)
      if (rw[j]) { raw = mulz(s, raw) ^ s->cseg[j]; ++cnt; }
    len = cnt * s->ulen;
  } else {
    for (uint32_t j = 0; j < s->C; ++j)
      if (rw[j]) { raw = o_multmodp(s->segmul[j], raw) ^ s->cseg[j]; len += s->seglen[j]; }
  }
  return raw ^ o_multmodp(o_xpow8(len), 0xFFFFFFFFu) ^ 0xFFFFFFFFu;
}
/* sparse rows, uniform identities: the base's prefix folds between consecutive exceptions, one multiply
 * per interval: raw(A ‖ base ∩ [a, b)) = (raw(A) ⊕ bpre[a])·Z^{bcnt[b] - bcnt[a]} ⊕ bpre[b]; an exception
 * that is a member outside the base is appended (raw·Z ⊕ c_x), one inside the base is skipped. */
static uint32_t fold_sparse(kbo_sim* s, uint32_t i) {
  const srow* r = &s->sr[i];
  uint32_t raw = 0, pos = 0;
  uint64_t cnt = 0;
  for (uint32_t k = 0; k < r->nx; ++k) {
    const uint32_t x = r->x[k];
    if (r->based) { raw = o_multmodp(s->zpw[s->bcnt[x] - s->bcnt[pos]], raw ^ s->bpre[pos]) ^ s->bpre[x]; cnt += s->bcnt[x] - s->bcnt[pos]; }
    if (!r->based || !bbit(s, x)) { raw = mulz(s, raw) ^ s->cseg[x]; cnt++; }
    pos = x + 1;
  }
  if (r->based) { raw = o_multmodp(s->zpw[s->bcnt[s->C] - s->bcnt[pos]], raw ^ s->bpre[pos]) ^ s->bpre[s->C]; cnt += s->bcnt[s->C] - s->bcnt[pos]; }
  return raw ^ o_multmodp(o_xpow8(cnt * s->ulen), 0xFFFFFFFFu) ^ 0xFFFFFFFFu;
}
static uint32_t fold_row(kbo_sim* s, uint32_t i) {
  if (!s->sr) return fold_bytes(s, row(s, i));
  if (s->uniform) return fold_sparse(s, i);
  uint8_t* rw = (uint8_t*)malloc(s->C);
  row_bytes(s, i, rw);
  const uint32_t f = fold_bytes(s, rw);
  free(rw);
  return f;
}

/* The literal reference definition, byte by byte (kept for the equivalence test). */
uint32_t kbo_fingerprint_direct(kbo_sim* s, uint32_t i) {
  uint8_t* rw = (uint8_t*)malloc(s->C);
  row_bytes(s, i, rw);
  uint32_t reg = 0xFFFFFFFFu;
  char a[32];
  for (uint32_t j = 0; j < s->C; ++j) {
    if (!rw[j]) continue;
    kbo_format_addr(j, a, sizeof a);
    reg = o_crc_update(reg, (const uint8_t*)a, strlen(a));
    reg = o_crc_update(reg, s->ident + (size_t)j * MAXID, s->id_len[j]);
  }
  free(rw);
  return reg ^ 0xFFFFFFFFu;
}

static inline uint32_t cur_fp(kbo_sim* s, uint32_t i) {
  if (s->dirty[i]) { s->fp[i] = fold_row(s, i); s->dirty[i] = 0; }
  return s->fp[i];
}

/* ---- ObservableHashMap operations on row i (src/observable_hashmap.rs:84-142) ------------------- */
static osusp* susp_find(kbo_sim* s, uint32_t i, uint32_t p) {
  osusp* sl = s->susp + (size_t)i * SLOTS;
  for (int k = 0; k < SLOTS; ++k) if (sl[k].kind && sl[k].peer == p) return &sl[k];
  return NULL;
}
static int susp_count(kbo_sim* s, uint32_t i) {
  osusp* sl = s->susp + (size_t)i * SLOTS; int c = 0;
  for (int k = 0; k < SLOTS; ++k) c += sl[k].kind != 0;
  return c;
}
/* PeerInfo.latency (src/kaboodle.rs:789-817).  Simulated clock: round r's tick is at
 * 1000·r ms (PROTOCOL_PERIOD, :38) and wave w of its receive window delivers at 1000·r + w + 1 ms.  A
 * WaitingFor*(since) entry was set by a tick, at 1000·since. */
#define LAT_NONE 0xFFFFu
static inline uint16_t lat_ewma(uint32_t sample, uint32_t prev) {   /* :808-816, f64 as the reference */
  if (prev == LAT_NONE) return (uint16_t)(sample < LAT_NONE ? sample : LAT_NONE - 1);
  volatile double a = (double)sample * 0.8;          /* no contraction into an fma */
  volatile double b = (double)prev * (1.0 - 0.8);
  uint64_t v = (uint64_t)(a + b);
  return (uint16_t)(v < LAT_NONE ? v : LAT_NONE - 1);
}
/* insert(p, Known(t)): overwrite; clears WaitingFor* state. returns 1 if p was new.  lat_w >= 0: the
 * envelope prologue of a unicast delivered in wave lat_w (calculate_peer_latency, :412); -1: a Join
 * broadcast or a KnownPeers arm (latency kept, :294-296, or None for a new entry, :467) */
static int map_insert_known(kbo_sim* s, uint32_t i, uint32_t p, int32_t t, int32_t r, int lat_w) {
  int was = st_get(s, i, p);
  uint16_t* lt = s->lat ? s->lat + (size_t)i * s->C + p : NULL;
  if (was == ST_SUSPECT) {
    osusp* q = susp_find(s, i, p);
    if (lt && lat_w >= 0 && q) *lt = lat_ewma(1000u * (uint32_t)(r - q->since) + (uint32_t)lat_w + 1u, *lt);
    if (q) q->kind = 0;
  }
  st_set(s, i, p, enc(t, r));
  if (s->tst) s->tst[(size_t)i * s->C + p] = t;
  if (was == ST_UNKNOWN) { if (lt) *lt = LAT_NONE; s->n[i]++; s->dirty[i] = 1; return 1; }
  return 0;
}
static int map_remove(kbo_sim* s, uint32_t i, uint32_t p) {
  const uint8_t b = st_get(s, i, p);
  if (b == ST_UNKNOWN) return 0;
  if (b == ST_SUSPECT) { osusp* q = susp_find(s, i, p); if (q) q->kind = 0; }
  st_set(s, i, p, ST_UNKNOWN);
  s->n[i]--; s->dirty[i] = 1;
  return 1;
}
static int set_suspect(kbo_sim* s, uint32_t i, uint32_t p, int kind, int32_t r) {
  osusp* q = susp_find(s, i, p);
  if (!q) {
    osusp* sl = s->susp + (size_t)i * SLOTS;
    for (int k = 0; k < SLOTS; ++k) if (!sl[k].kind) { q = &sl[k]; break; }
    if (!q) return KB_CAPACITY;
    q->peer = p;
  }
  q->kind = kind; q->since = r;
  st_set(s, i, p, ST_SUSPECT);
  return KB_OK;
}

/* curious_peers (src/kaboodle.rs:101, :536-540, :423, :644) */
static ocur* cur_find(kbo_sim* s, uint32_t i, uint32_t p) {
  ocur* c = s->cur + (size_t)i * CSLOTS;
  for (int k = 0; k < CSLOTS; ++k) if (c[k].used && c[k].peer == p) return &c[k];
  return NULL;
}
static void cur_add(kbo_sim* s, uint32_t i, uint32_t p, uint32_t observer) {
  ocur* e = cur_find(s, i, p);
  if (!e) {
    ocur* c = s->cur + (size_t)i * CSLOTS;
    for (int k = 0; k < CSLOTS; ++k) if (!c[k].used) { e = &c[k]; break; }
    if (!e) {
#pragma omp atomic
      s->st.curious_overflow++;
      return;
    }
    e->used = 1; e->peer = p; e->nobs = 0;
  }
  for (uint32_t k = 0; k < e->nobs; ++k) if (e->obs[k] == observer) return;
  if (e->nobs == NOBS) {
#pragma omp atomic
    s->st.curious_overflow++;
    return;
  }
  e->obs[e->nobs++] = observer;
}
static void cur_remove(kbo_sim* s, uint32_t i, uint32_t p) {
  ocur* e = cur_find(s, i, p);
  if (e) e->used = 0;
}

/* ---- emission ----------------------------------------------------------------------------------- */
static void vpush(ovec* v, const omsg* m) {
  if (v->n == v->cap) { v->cap = v->cap ? v->cap * 2 : 8; v->v = (omsg*)realloc(v->v, v->cap * sizeof(omsg)); }
  v->v[v->n++] = *m;
}
static void emit(kbo_sim* s, uint32_t from, uint32_t to, uint32_t kind, uint32_t a, uint32_t fp, uint32_t n,
                 uint32_t* pay, uint32_t pay_len) {
  omsg m;
  m.dest = to; m.sender = from; m.seq = s->oseq[from]++; m.kind = kind;
  m.a = a; m.fp = fp; m.n = n; m.pay = pay; m.pay_len = pay_len;
  vpush(&s->out[from], &m);
}

/* bincode 1.3.3 size of SwimEnvelope{identity, KnownPeers(map)} (src/structs.rs:78-116):
 * identity u64 len + bytes, u32 variant tag, u64 map len, per entry SocketAddr::V4 (u32 tag + 4 + 2)
 * + Bytes (u64 len + bytes). */
static uint64_t kp_size(kbo_sim* s, uint32_t self, const uint32_t* ids, uint32_t n) {
  uint64_t sz = 8 + s->id_len[self] + 4 + 8;
  for (uint32_t k = 0; k < n; ++k) sz += 10 + 8 + s->id_len[ids[k]];
  return sz;
}
static uint32_t kp_cap_uniform(kbo_sim* s) {   /* largest k with 20 + L + k(18+L) < 10240 */
  uint32_t L = s->cfg.id_len;
  return (BUFSZ - 20 - L - 1) / (18 + L);
}

/* ---- lifecycle (src/lib.rs:136-183, src/kaboodle.rs:114-185) ------------------------------------ */
static void node_start(kbo_sim* s, uint32_t i, int32_t r) {
  s->alive[i] = 1; s->start_round[i] = r;
  map_insert_known(s, i, i, r, r, -1);          /* known_peers.insert(self_addr, Known(now)) :145-152 */
  s->dirty[i] = 1;
  s->last_bcast[i] = INT32_MIN;             /* last_broadcast_time: None                    :170 */
  memset(s->cur + (size_t)i * CSLOTS, 0, sizeof(ocur) * CSLOTS);   /* fresh KaboodleInner     */
  s->paq_n[i] = 0;
  s->a3cur[i] = i;                          /* A3 rotation starts right after self */
}
static void node_stop(kbo_sim* s, uint32_t i) {
  map_remove(s, i, i);                      /* known_peers.remove(&self_addr)   src/lib.rs:167-170 */
  s->alive[i] = 0;
  s->paq_n[i] = 0;
}
/* Kaboodle::start on a stopped instance (src/lib.rs:136-156): KaboodleInner::start binds a fresh
 * ephemeral socket (src/kaboodle.rs:138-152), so the instance comes back at a NEW address (`to`, a fresh
 * id) while its known_peers map persists (the Arc'd ObservableHashMap of src/lib.rs:104, minus the old
 * self removed by stop, :167-170): every entry with its state, instant and latency.  The old address
 * stays in other views until pinged out.  Curious peers, the ping queue and last_broadcast_time belong to
 * the new KaboodleInner (fresh); the A3 sweep front starts after the new self. */
static void node_restart(kbo_sim* s, uint32_t from, uint32_t to, int32_t r) {
  const size_t C = s->C;
  if (s->sr) srow_copy(&s->sr[to], &s->sr[from]);
  else memcpy(row(s, to), row(s, from), C);
  if (s->lat) memcpy(s->lat + (size_t)to * C, s->lat + (size_t)from * C, C * sizeof(uint16_t));
  if (s->tst) memcpy(s->tst + (size_t)to * C, s->tst + (size_t)from * C, C * sizeof(int32_t));
  memcpy(s->susp + (size_t)to * SLOTS, s->susp + (size_t)from * SLOTS, SLOTS * sizeof(osusp));
  s->n[to] = s->n[from];
  s->dirty[to] = 1;
  node_start(s, to, r);
  /* the map's observer follows the instance.  An observer already attached to the new address (subscribed
   * after start() returned, before this round) either gives way to the instance's own, or, when the instance
   * had none, starts from the map as the restart left it (a channel reports only later changes) */
  size_t kf = s->nwatch, kt = s->nwatch;
  for (size_t k = 0; k < s->nwatch; ++k) { if (s->wnode[k] == from) kf = k; if (s->wnode[k] == to) kt = k; }
  if (kf < s->nwatch) {
    if (kt < s->nwatch) {
      free(s->wsnap[kt]);
      s->wnode[kt] = s->wnode[s->nwatch - 1]; s->wsnap[kt] = s->wsnap[s->nwatch - 1]; s->wfp[kt] = s->wfp[s->nwatch - 1];
      if (kf == s->nwatch - 1) kf = kt;
      s->nwatch--;
    }
    s->wnode[kf] = to;
  } else if (kt < s->nwatch) {
    uint8_t* tmp;
    const uint8_t* rw = row_view(s, to, &tmp);
    for (uint32_t j = 0; j < s->C; ++j) s->wsnap[kt][j] = rw[j] != 0;
    free(tmp);
  }
}

/* ---- creation ----------------------------------------------------------------------------------- */
void kbo_config_default(kb_config* c) {
  memset(c, 0, sizeof *c);
  c->abi_version = KB_ABI_VERSION; c->capacity = 1024; c->initial_nodes = 1024; c->init_mode = KB_INIT_JOIN;
  c->seed = 1; c->fault_end_round = -1; c->max_waves = 8; c->failed_mode = KB_FAILED_SIM_SENDER;
  c->device = -1;
}

int kbo_sim_create(const kb_config* cfg, kbo_sim** out) {
  o_crc_init();
  if (!cfg || !out || cfg->abi_version != KB_ABI_VERSION) { seterr("bad config"); return KB_INVALID_ARGUMENT; }
  if (cfg->capacity == 0 || cfg->capacity > 7800000u || cfg->initial_nodes > cfg->capacity || cfg->id_len > MAXID ||
      cfg->max_waves == 0 || cfg->max_waves > 64) {
    seterr("config out of range"); return KB_INVALID_ARGUMENT;
  }
  kbo_sim* s = (kbo_sim*)calloc(1, sizeof *s);
  s->cfg = *cfg; s->C = cfg->capacity;
  s->k0 = (uint32_t)cfg->seed; s->k1 = (uint32_t)(cfg->seed >> 32);
  size_t C = s->C;
  const int sparse = (cfg->variant & KB_VARIANT_SPARSE_ROWS) != 0;
  if (sparse && (cfg->track_latency || (cfg->variant & KB_VARIANT_EXACT_LRU))) {
    seterr("sparse rows keep neither a latency table nor exact instants"); free(s); return KB_INVALID_ARGUMENT;
  }
  if (sparse) s->sr = (srow*)calloc(C, sizeof(srow));
  else s->stamp = (uint8_t*)calloc(C * C, 1);
  s->alive = (uint8_t*)calloc(C, 1);
  s->start_round = (int32_t*)calloc(C, 4); s->n = (uint32_t*)calloc(C, 4); s->fp = (uint32_t*)calloc(C, 4);
  s->dirty = (uint8_t*)calloc(C, 1); s->last_bcast = (int32_t*)calloc(C, 4); s->a3cur = (uint32_t*)calloc(C, 4);
  s->susp = (osusp*)calloc(C * SLOTS, sizeof(osusp)); s->cur = (ocur*)calloc(C * CSLOTS, sizeof(ocur));
  s->paq = (uint32_t*)calloc(C * PAQ, 4); s->paq_n = (uint32_t*)calloc(C, 4);
  s->ident = (uint8_t*)calloc(C * MAXID, 1); s->id_len = (uint8_t*)calloc(C, 1);
  s->pend_ident = (uint8_t*)calloc(C * MAXID, 1); s->pend_len = (int16_t*)malloc(C * sizeof(int16_t));
  if (s->pend_len) for (size_t k = 0; k < C; ++k) s->pend_len[k] = -1;
  s->moved = (uint8_t*)calloc(C, 1);
  s->idset = (uint8_t*)calloc(C, 1);
  s->ext = (uint8_t*)calloc(C, 1);
  s->cseg = (uint32_t*)calloc(C, 4); s->segmul = (uint32_t*)calloc(C, 4); s->seglen = (uint32_t*)calloc(C, 4);
  s->out = (ovec*)calloc(C, sizeof(ovec)); s->oseq = (uint32_t*)calloc(C, 4);
  if (cfg->stat_flags & ~(uint32_t)KB_STAT_NO_SF_FAILED_DROPS) { seterr("unknown kb_config.stat_flags"); return KB_INVALID_ARGUMENT; }
  if (cfg->variant & ~(uint32_t)(KB_VARIANT_SAME_WINDOW_BCAST | KB_VARIANT_EXACT_LRU | KB_VARIANT_SPARSE_ROWS)) {
    seterr("unknown variant"); kbo_sim_destroy(s); return KB_INVALID_ARGUMENT;
  }
  if (cfg->variant & KB_VARIANT_EXACT_LRU) {
    s->tst = (int32_t*)malloc(C * C * sizeof(int32_t));
    if (s->tst) {                           /* converged start: ancient, ties (first touch spread over threads) */
#pragma omp parallel for schedule(static)
      for (size_t i = 0; i < C; ++i) for (size_t k = 0; k < C; ++k) s->tst[i * C + k] = INT32_MIN / 2;
    }
  }
  if (cfg->track_latency) {
    s->lat = (uint16_t*)malloc(C * C * sizeof(uint16_t));
    if (s->lat) {
#pragma omp parallel for schedule(static)
      for (size_t i = 0; i < C; ++i) memset(s->lat + i * C, 0xFF, C * sizeof(uint16_t));
    }
  }
  if ((!s->stamp && !s->sr) || !s->susp || !s->cur || (cfg->track_latency && !s->lat)) {
    seterr("out of host memory"); kbo_sim_destroy(s); return KB_CAPACITY;
  }
  for (uint32_t i = 0; i < s->C; ++i) {
    s->id_len[i] = (uint8_t)cfg->id_len;
    default_identity(i, cfg->id_len, s->ident + (size_t)i * MAXID);
    compute_seg(s, i);
    s->last_bcast[i] = INT32_MIN;
    s->start_round[i] = INT32_MIN;
  }
  s->uniform = 1; s->ulen = ADDR_LEN + cfg->id_len; build_mulz(s);
  s->htab = (uint32_t*)malloc(sizeof(uint32_t) * 256 * ((size_t)C / 8 + 1));
  s->hfull = (uint32_t*)malloc(sizeof(uint32_t) * ((size_t)C / 8 + 1));
  if (!s->htab || !s->hfull) { seterr("out of host memory"); kbo_sim_destroy(s); return KB_CAPACITY; }
  for (uint32_t b = 0; b <= s->C / 8; ++b) htab_block(s, b);
  s->round = 0; s->next_free = cfg->initial_nodes;
  if (sparse) {
    /* the base: the initial members of a converged start (empty otherwise), with its prefix counts and
     * prefix folds; the initial rows adopt it, every other row starts empty */
    const uint32_t nb = cfg->init_mode == KB_INIT_CONVERGED ? cfg->initial_nodes : 0;
    s->bbits = (uint32_t*)calloc(C / 32 + 1, 4); s->bcnt = (uint32_t*)malloc(4 * (C + 1));
    s->bpre = (uint32_t*)malloc(4 * (C + 1)); s->zpw = (uint32_t*)malloc(4 * (C + 2));
    if (!s->bbits || !s->bcnt || !s->bpre || !s->zpw) { seterr("out of host memory"); kbo_sim_destroy(s); return KB_CAPACITY; }
    for (uint32_t j = 0; j < nb; ++j) s->bbits[j >> 5] |= 1u << (j & 31);
    uint32_t raw = 0, c = 0;
    for (uint32_t j = 0; j <= s->C; ++j) {
      s->bcnt[j] = c; s->bpre[j] = raw;
      if (j < s->C && bbit(s, j)) { raw = mulz(s, raw) ^ s->cseg[j]; c++; }
    }
    s->zpw[0] = 0x80000000u;
    const uint32_t Z = o_xpow8(s->ulen);
    for (size_t k = 1; k < C + 2; ++k) s->zpw[k] = o_multmodp(Z, s->zpw[k - 1]);
    for (uint32_t i = 0; i < s->C; ++i) { s->sr[i].based = i < nb || nb == 0; s->sr[i].adopt_at = nb / 2 + 64; }
  }
#pragma omp parallel for schedule(static)
  for (uint32_t i = 0; i < cfg->initial_nodes; ++i) {   /* touches row i and per-id slots of i only */
    node_start(s, i, 0);
    if (cfg->init_mode == KB_INIT_CONVERGED) {
      if (!sparse) {                        /* sparse: the base already holds them, ancient */
        uint8_t* rw = row(s, i);
        for (uint32_t j = 0; j < cfg->initial_nodes; ++j) if (j != i) rw[j] = ST_ANCIENT;
      }
      s->n[i] = cfg->initial_nodes;
      s->last_bcast[i] = -1000;             /* running for a while: no Join at round 0 */
    }
  }
  s->st.first_converged_round = -1; s->st.last_converged_round = -1;
  *out = s;
  return KB_OK;
}

int kbo_sim_destroy(kbo_sim* s) {
  if (!s) return KB_INVALID_ARGUMENT;
  if (s->out) for (uint32_t i = 0; i < s->C; ++i) free(s->out[i].v);
  if (s->sr) for (uint32_t i = 0; i < s->C; ++i) srow_free(&s->sr[i]);
  free(s->sr); free(s->bbits); free(s->bcnt); free(s->bpre); free(s->zpw);
  free(s->probe_q); free(s->probes); free(s->presp); free(s->stamp); free(s->tst); free(s->lat); free(s->alive); free(s->start_round); free(s->n); free(s->fp); free(s->dirty);
  free(s->last_bcast); free(s->a3cur); free(s->susp); free(s->cur); free(s->paq); free(s->paq_n); free(s->ident); free(s->id_len); free(s->pend_ident); free(s->pend_len); free(s->moved); free(s->idset); free(s->ext);
  for (size_t k = 0; k < s->ninj; ++k) free(s->inj[k].pay);
  free(s->inj); free(s->xp); free(s->xids); free(s->injj);
  free(s->cseg); free(s->segmul); free(s->seglen); free(s->htab); free(s->hfull); free(s->out); free(s->oseq); free(s->bfail); free(s->bjoin);
  for (size_t k = 0; k < s->nwatch; ++k) free(s->wsnap[k]);
  free(s->wnode); free(s->wsnap); free(s->wfp);
  free(s->ev); free(s);
  return KB_OK;
}

/* ---- broadcast phase: deliveries of round r-1's broadcasts ---------------------- */
static void bpush(obcast** v, size_t* n, size_t* cap, uint32_t sender, uint32_t peer, uint32_t bseq) {
  if (*n == *cap) { *cap = *cap ? *cap * 2 : 16; *v = (obcast*)realloc(*v, *cap * sizeof(obcast)); }
  (*v)[*n].sender = sender; (*v)[*n].peer = peer; (*v)[*n].bseq = bseq; (*n)++;
}

/* delivery of entry e of the round's Failed (lst 0) / Join (lst 1) broadcast list to recv: word e % 4
 * of philox(recv, r, P_BLOSS << 24 | lst << 23 | e / 4, 0) */
static int bcast_lost(kbo_sim* s, uint32_t recv, const obcast* b, int32_t r, uint32_t lst, size_t e) {
  if (partition_blocks(s, r, b->sender, recv)) return 2;
  if (!active_faults(s, r) || s->cfg.loss_threshold == 0) return 0;
  return ph(s, recv, (uint32_t)r, ((uint32_t)P_BLOSS << 24) | (lst << 23) | (uint32_t)(e >> 2), 0).v[e & 3] <
         s->cfg.loss_threshold;
}

/* should_respond_to_broadcast for the e-th Probe of the round: its own counter (bit 23 set) */
static int probe_should_respond(kbo_sim* s, uint32_t i, uint32_t e, int32_t r) {
  const int64_t o = (int64_t)s->n[i] - 2;
  if (o <= 0) return 1;
  int64_t pct = 100 - o * o;
  if (pct < 1) pct = 1;
  const uint32_t u = ph(s, i, (uint32_t)r, ((uint32_t)P_RESPOND << 24) | (1u << 23) | e, 0).v[0];
  return (int64_t)o_mulhi(u, 100) < pct;
}
/* should_respond_to_broadcast (src/kaboodle.rs:333-354), integer restatement of gen_bool */
static int should_respond(kbo_sim* s, uint32_t i, uint32_t joiner, int32_t r) {
  int64_t o = (int64_t)s->n[i] - 2;
  if (o <= 0) return 1;
  int64_t pct = 100 - o * o;
  if (pct < 1) pct = 1;
  uint32_t u = ph(s, i, (uint32_t)r, (uint32_t)P_RESPOND << 24, joiner).v[0];
  return (int64_t)o_mulhi(u, 100) < pct;
}

/* Keyed permutation of [0, n): 4-round Feistel network on b = max(2, ceil(log2 n))
 * bits, halves of ceil(b/2) (high) and floor(b/2) (low) bits whose widths swap every round, round
 * function lowbias32(R ^ key[k]) masked to the width of the half it is XORed into, cycle-walked into
 * [0, n). */
static inline uint32_t o_mix32(uint32_t x) {
  x ^= x >> 16; x *= 0x7feb352du; x ^= x >> 15; x *= 0x846ca68bu; x ^= x >> 16;
  return x;
}
static uint32_t prp_walk(uint32_t x, uint32_t n, const uint32_t key[4]) {
  uint32_t b = 2;
  while ((1ull << b) < n) b += 1;
  const uint32_t c = b / 2, a = b - c;
  do {
    uint32_t L = x >> c, R = x & ((1u << c) - 1u), wl = a;
    for (int k = 0; k < 4; ++k) { uint32_t t = R; R = L ^ (o_mix32(R ^ key[k]) & ((1u << wl) - 1u)); L = t; wl = b - wl; }
    x = (L << c) | R;
  } while (x >= n);
  return x;
}

/* maybe_send_known_peers_to_peer (src/kaboodle.rs:356-392): every entry of the map (self, the joiner
 * and suspects included); while the encoding is >= 10240 B drop a uniformly random entry — restated
 * as a uniform random subset of the largest size that fits: the first `cap` images of a keyed
 * pseudo-random permutation of the member ranks (prp_walk). */
static void join_response(kbo_sim* s, uint32_t i, uint32_t joiner, int32_t r) {
  uint32_t n = s->n[i];
  uint32_t* members = (uint32_t*)malloc(sizeof(uint32_t) * (n ? n : 1));
  uint32_t m = 0;
  if (s->sr) {                                     /* base Δ x, merged in id order */
    const srow* rr = &s->sr[i];
    uint32_t k = 0;
    for (uint32_t j = 0; j < s->C; ++j) {
      const int in_x = k < rr->nx && rr->x[k] == j;
      k += in_x;
      if (((rr->based && bbit(s, j)) != in_x) && m < n) members[m++] = j;
    }
  } else {
    const uint8_t* rw = row(s, i);
    for (uint32_t j = 0; j < s->C; ++j) if (rw[j]) members[m++] = j;
  }
  uint32_t cap = kp_cap_uniform(s);
  uint32_t* pay;
  uint32_t plen;
  if (m <= cap || !s->uniform) {
    pay = members; plen = m;
  } else {
    /* first `cap` images of a keyed pseudo-random permutation of [0, m) */
    o_u32x4 key = ph(s, i, (uint32_t)r, (uint32_t)P_TRUNC << 24, joiner);
    uint8_t* chosen = (uint8_t*)calloc(m, 1);
    for (uint32_t t = 0; t < cap; ++t) chosen[prp_walk(t, m, key.v)] = 1;
    pay = (uint32_t*)malloc(sizeof(uint32_t) * cap);
    plen = 0;
    for (uint32_t k = 0; k < m; ++k) if (chosen[k]) pay[plen++] = members[k];
    free(chosen); free(members);
  }
  emit(s, i, joiner, K_KP, plen, 0, 0, pay, plen);
#pragma omp atomic
  s->st.join_responses++;
}

/* the Join broadcasts of external peers (kbo_sim_inject) enter the round's Join list at their sender's place, as
 * a tick's Join would (bseq 0) */
static void merge_ext_joins(kbo_sim* s) {
  for (size_t q = 0; q < s->ninjj; ++q) {
    const uint32_t x = s->injj[q];
    bpush(&s->bjoin, &s->nbjoin, &s->capbjoin, x, x, 0);
    for (size_t k = s->nbjoin - 1; k > 0 && s->bjoin[k - 1].sender > x; --k) {
      const obcast t = s->bjoin[k - 1]; s->bjoin[k - 1] = s->bjoin[k]; s->bjoin[k] = t;
    }
  }
  s->ninjj = 0;
}

static void phase_broadcasts(kbo_sim* s, uint32_t i, int32_t r) {
  uint64_t lost = 0, removed = 0;
  /* Failed(p) (src/kaboodle.rs:268-283) */
  /* socket_faithful Failed changes no state; KB_STAT_NO_SF_FAILED_DROPS skips counting its lost deliveries */
  const size_t nbf = s->cfg.failed_mode == KB_FAILED_SOCKET_FAITHFUL && (s->cfg.stat_flags & KB_STAT_NO_SF_FAILED_DROPS)
                         ? 0 : s->nbfail;
  for (size_t k = 0; k < nbf; ++k) {
    const obcast* b = &s->bfail[k];
    if (b->sender == i) continue;                     /* own broadcasts are not delivered to self */
    if (bcast_lost(s, i, b, r, 0, k)) { lost++; continue; }
    if (b->peer == i) continue;                       /* Failed(self) ignored            :269-273 */
    if (s->cfg.failed_mode == KB_FAILED_SIM_SENDER && st_get(s, i, b->sender) != ST_UNKNOWN)
      removed += (uint64_t)map_remove(s, i, b->peer); /* sender is a mesh member         :275-279 */
  }
  /* Join{addr} (src/kaboodle.rs:284-304) */
  for (size_t k = 0; k < s->nbjoin; ++k) {
    const obcast* b = &s->bjoin[k];
    if (b->sender == i) continue;                     /* addr == self_addr               :285-287 */
    if (bcast_lost(s, i, b, r, 1, k)) { lost++; continue; }
    int is_new = map_insert_known(s, i, b->sender, r, r, -1);
    if (is_new && should_respond(s, i, b->sender, r)) join_response(s, i, b->sender, r);
  }
  /* Probe(addr) (src/kaboodle.rs:305-331): maybe_respond_to_probe with the map as it stands now */
  for (size_t e = 0; e < s->nprobes; ++e) {
    if (active_faults(s, r) && s->cfg.loss_threshold &&
        ph(s, i, (uint32_t)r, ((uint32_t)P_PROBE << 24) | (uint32_t)(e / 4), 0).v[e % 4] < s->cfg.loss_threshold) {
      lost++; continue;
    }
    if (!probe_should_respond(s, i, (uint32_t)e, r)) continue;
    const int rlost = active_faults(s, r) && s->cfg.loss_threshold &&
        ph(s, i, (uint32_t)r, ((uint32_t)P_PROBE << 24) | (1u << 23) | (uint32_t)e, 1).v[0] < s->cfg.loss_threshold;
#pragma omp critical(kbo_probe)
    {
      s->st.probe_responses++;
      if (rlost) s->st.drop_loss++;
      else {
        if (s->npresp == s->cappresp) {
          s->cappresp = s->cappresp ? 2 * s->cappresp : 64;
          s->presp = (kb_probe_response*)realloc(s->presp, s->cappresp * sizeof(kb_probe_response));
        }
        kb_probe_response* o = &s->presp[s->npresp++];
        memset(o, 0, sizeof *o);
        o->responder = i; o->probe = (uint32_t)e; o->round = r; o->prober = s->probes[e];
        o->identity_len = s->id_len[i];
        memcpy(o->identity, s->ident + (size_t)i * MAXID, s->id_len[i]);
      }
    }
  }
#pragma omp atomic
  s->st.drop_bcast += lost;
#pragma omp atomic
  s->st.removed_failed += removed;
}

/* ---- tick (src/kaboodle.rs:746-779) -------------------------------------------------------------- */
typedef struct { uint32_t fail_peers[SLOTS]; int nfail; int join; } otick_bc;

static inline uint32_t rot_key(uint32_t j, uint32_t base, uint32_t C) {  /* rotated address order from base+1 */
  return (j + C - base - 1) % C;
}

/* the candidates of handle_suspected_peers' indirect pings: Known && != self, ascending id (:571-577) */
static uint32_t a2_candidates(kbo_sim* s, uint32_t i, uint32_t* cand) {
  uint32_t c = 0;
  if (!s->sr) {
    const uint8_t* rw = row(s, i);
    for (uint32_t j = 0; j < s->C; ++j) if (rw[j] >= ST_ANCIENT && j != i) cand[c++] = j;
    return c;
  }
  const srow* rr = &s->sr[i];
  uint32_t k = 0, q = 0;
  for (uint32_t j = 0; j < s->C; ++j) {
    const int in_x = k < rr->nx && rr->x[k] == j;
    k += in_x;
    if ((rr->based && bbit(s, j)) == in_x) continue;             /* not a member */
    while (q < rr->nl && rr->lid[q] < j) ++q;
    if (j != i && !(q < rr->nl && rr->lid[q] == j && rr->lb[q] == ST_SUSPECT)) cand[c++] = j;
  }
  return c;
}
/* A3's five smallest (stamp, rotated id) keys over Known && != self, ascending */
static inline void top5_add(uint32_t* best, uint32_t* kh5, uint32_t* kl5, int* nb, uint32_t j, uint32_t kh, uint32_t kl) {
  if (*nb == NUM_CANDIDATES && (kh > kh5[*nb - 1] || (kh == kh5[*nb - 1] && kl > kl5[*nb - 1]))) return;
  int pos = *nb < NUM_CANDIDATES ? *nb : NUM_CANDIDATES - 1;
  while (pos > 0 && (kh5[pos - 1] > kh || (kh5[pos - 1] == kh && kl5[pos - 1] > kl))) {
    kh5[pos] = kh5[pos - 1]; kl5[pos] = kl5[pos - 1]; best[pos] = best[pos - 1]; --pos;
  }
  kh5[pos] = kh; kl5[pos] = kl; best[pos] = j;
  if (*nb < NUM_CANDIDATES) (*nb)++;
}
static int a3_candidates(kbo_sim* s, uint32_t i, uint32_t* best) {
  uint32_t kh5[NUM_CANDIDATES], kl5[NUM_CANDIDATES];
  int nb = 0;
  if (s->tst) {                                    /* KB_VARIANT_EXACT_LRU: the exact instants */
    const uint8_t* rw = row(s, i);
    for (uint32_t j = 0; j < s->C; ++j) {
      uint8_t b = rw[j];
      if (b < ST_ANCIENT || j == i) continue;
      const uint32_t kh = (uint32_t)s->tst[(size_t)i * s->C + j] ^ 0x80000000u;   /* order-preserving */
      top5_add(best, kh5, kl5, &nb, j, kh, rot_key(j, s->a3cur[i], s->C));
    }
    return nb;
  }
  if (!s->sr) {
    /* rotated order from the sweep front; ANCIENT is the smallest stamp, so once five ancient members have
     * been met nothing later in that order can rank among the five */
    const uint8_t* rw = row(s, i);
    const uint32_t C = s->C, p0 = s->a3cur[i] + 1 == C ? 0 : s->a3cur[i] + 1;
    int anc = 0;
    for (uint32_t k = 0; k < C; ++k) {
      const uint32_t j = p0 + k >= C ? p0 + k - C : p0 + k;
      const uint8_t b = rw[j];
      if (b < ST_ANCIENT || j == i) continue;
      top5_add(best, kh5, kl5, &nb, j, b, k);
      if (b == ST_ANCIENT && ++anc == NUM_CANDIDATES) break;
    }
    return nb;
  }
  /* sparse: every member without an explicit stamp is ancient, the smallest key; those met first in
   * rotated order from the sweep front are the oldest, so the scan stops after five of them.  With fewer
   * than five ancient members, the explicit Known stamps fill in by (stamp, rotated id). */
  const srow* rr = &s->sr[i];
  const uint32_t C = s->C, p0 = s->a3cur[i] + 1 == C ? 0 : s->a3cur[i] + 1;
  for (uint32_t k = 0; k < C && nb < NUM_CANDIDATES; ++k) {
    const uint32_t j = p0 + k >= C ? p0 + k - C : p0 + k;
    if (j == i || !s_mem(s, i, j) || l_get(rr, j)) continue;
    top5_add(best, kh5, kl5, &nb, j, ST_ANCIENT, k);
  }
  if (nb < NUM_CANDIDATES)
    for (uint32_t q = 0; q < rr->nl; ++q)
      if (rr->lb[q] >= ST_ANCIENT && rr->lid[q] != i) top5_add(best, kh5, kl5, &nb, rr->lid[q], rr->lb[q], rot_key(rr->lid[q], s->a3cur[i], C));
  return nb;
}

static int tick(kbo_sim* s, uint32_t i, int32_t r, otick_bc* bc) {
  bc->nfail = 0; bc->join = 0;
  /* A1 maybe_broadcast_join (:228-251) */
  if (s->last_bcast[i] == INT32_MIN || (r - s->last_bcast[i] >= REBROADCAST && s->n[i] <= 1)) {
    bc->join = 1; s->last_bcast[i] = r;
  }
  /* A2 handle_suspected_peers (:558-653) */
  {
    uint32_t m = s->n[i] - 1 - (uint32_t)susp_count(s, i);   /* Known && != self (:571-577) */
    osusp* sl = s->susp + (size_t)i * SLOTS;
    int order[SLOTS], no = 0;
    for (int k = 0; k < SLOTS; ++k) if (sl[k].kind) order[no++] = k;
    for (int a = 1; a < no; ++a) {            /* ascending peer id */
      int t = order[a], b = a - 1;
      while (b >= 0 && sl[order[b]].peer > sl[t].peer) { order[b + 1] = order[b]; --b; }
      order[b + 1] = t;
    }
    uint32_t indirect[SLOTS], removed[SLOTS]; int nind = 0, nrem = 0;
    uint32_t* cand = NULL;
    for (int q = 0; q < no; ++q) {
      osusp* e = &sl[order[q]];
      if (r - e->since < PING_TIMEOUT) continue;
      if (e->kind == SK_WFP) {
        uint32_t k = m < NUM_INDIRECT ? m : NUM_INDIRECT;
        if (k == 0) { removed[nrem++] = e->peer; continue; }
        if (!cand) {
          cand = (uint32_t*)malloc(sizeof(uint32_t) * (m ? m : 1));
          (void)a2_candidates(s, i, cand);
        }
        o_u32x4 w = ph(s, i, (uint32_t)r, (uint32_t)P_INDIRECT << 24, e->peer);
        uint32_t pick[3];
        pick[0] = o_mulhi(w.v[0], m);
        if (k > 1) { uint32_t b = o_mulhi(w.v[1], m - 1); pick[1] = b + (b >= pick[0]); }
        if (k > 2) {
          uint32_t lo = pick[0] < pick[1] ? pick[0] : pick[1], hi = pick[0] < pick[1] ? pick[1] : pick[0];
          uint32_t c = o_mulhi(w.v[2], m - 2);
          if (c >= lo) c++;
          if (c >= hi) c++;
          pick[2] = c;
        }
        for (uint32_t t = 0; t < k; ++t) emit(s, i, cand[pick[t]], K_PINGREQ, e->peer, 0, 0, NULL, 0);
        indirect[nind++] = e->peer;
      } else {
        removed[nrem++] = e->peer;
      }
    }
    free(cand);
    for (int q = 0; q < nind; ++q) set_suspect(s, i, indirect[q], SK_WFIP, r);     /* :631-639 */
    for (int q = 0; q < nrem; ++q) {                                              /* :641-652 */
      map_remove(s, i, removed[q]);
      cur_remove(s, i, removed[q]);
      bc->fail_peers[bc->nfail++] = removed[q];
    }
    if (nrem) {
#pragma omp atomic
      s->st.removed_timeout += (uint64_t)nrem;
    }
  }
  /* A3 ping_random_peer (:655-703): oldest 5 by (stamp, id rotated to start at the node's sweep front),
     one uniformly; the front moves to the oldest candidate */
  {
    uint32_t best[NUM_CANDIDATES];
    const int nb = a3_candidates(s, i, best);
    if (nb > 0) {
      uint32_t u = ph(s, i, (uint32_t)r, (uint32_t)P_PING << 24, 0).v[0];
      uint32_t t = best[o_mulhi(u, (uint32_t)nb)];
      s->a3cur[i] = (best[0] + s->C - 1) % s->C;
      if (set_suspect(s, i, t, SK_WFP, r) != KB_OK) return KB_CAPACITY;
      emit(s, i, t, K_PING, 0, 0, 0, NULL, 0);
    }
  }
  /* A4 handle_incoming_ping_requests (:550-556) */
  for (uint32_t q = 0; q < s->paq_n[i]; ++q) emit(s, i, s->paq[(size_t)i * PAQ + q], K_PING, 0, 0, 0, NULL, 0);
  s->paq_n[i] = 0;
  return KB_OK;
}

/* ---- unicast handling (src/kaboodle.rs:394-548) -------------------------------------------------- */
static void maybe_sync(kbo_sim* s, uint32_t i, uint32_t peer, uint32_t their_fp, uint32_t their_n) {  /* :707-740 */
  uint32_t f = cur_fp(s, i);
  if (f == their_fp) return;
  if (s->n[i] > their_n) return;
  emit(s, i, peer, K_KPR, 0, f, s->n[i], NULL, 0);
}

static void handle_message(kbo_sim* s, uint32_t i, const omsg* m, int32_t r, uint32_t w) {
  uint32_t from = m->sender;
  map_insert_known(s, i, from, r, r, (int)w);    /* prologue :406-415 */
  switch (m->kind) {
    case K_ACK: {                                  /* :418-447 */
      ocur* e = cur_find(s, i, m->a);
      if (e) {
        uint32_t nobs = e->nobs, obs[NOBS];
        memcpy(obs, e->obs, sizeof obs);
        e->used = 0;
        for (uint32_t k = 0; k < nobs; ++k) emit(s, i, obs[k], K_ACK, m->a, m->fp, m->n, NULL, 0);
      }
      maybe_sync(s, i, m->a, m->fp, m->n);
      break;
    }
    case K_KP: {                                   /* :448-472 */
      for (uint32_t k = 0; k < m->pay_len; ++k) {
        uint32_t p = m->pay[k];
        if (st_get(s, i, p) == ST_UNKNOWN) map_insert_known(s, i, p, r - SHARE_AGE, r, -1);
      }
      break;
    }
    case K_KPR: {                                  /* :473-512 */
      uint8_t fresh = enc(r - (SHARE_AGE - 1), r);
      uint32_t cnt = 0, cap = 64;
      uint32_t* pay = (uint32_t*)malloc(sizeof(uint32_t) * cap);
      if (s->sr) {                                 /* sparse: fresh stamps are explicit (fresh > ancient) */
        const srow* rr = &s->sr[i];
        for (uint32_t q = 0; q < rr->nl; ++q) {
          const uint32_t j = rr->lid[q];
          if (rr->lb[q] >= fresh && j != i && j != from) {
            if (cnt == cap) { cap *= 2; pay = (uint32_t*)realloc(pay, sizeof(uint32_t) * cap); }
            pay[cnt++] = j;
          }
        }
      } else {
        const uint8_t* rw = row(s, i);
        for (uint32_t j = 0; j < s->C; ++j) {
          if (rw[j] >= fresh && j != i && j != from) {
            if (cnt == cap) { cap *= 2; pay = (uint32_t*)realloc(pay, sizeof(uint32_t) * cap); }
            pay[cnt++] = j;
          }
        }
      }
      if (kp_size(s, i, pay, cnt) > BUFSZ) {        /* truncated at the receiver -> undeliverable (Q3) */
        free(pay);
#pragma omp atomic
        s->st.drop_oversize++;
      } else {
        emit(s, i, from, K_KP, cnt, 0, 0, pay, cnt);
      }
      maybe_sync(s, i, from, m->fp, m->n);
      break;
    }
    case K_PING:                                   /* :513-532 */
      emit(s, i, from, K_ACK, i, cur_fp(s, i), s->n[i], NULL, 0);
      break;
    case K_PINGREQ:                                /* :533-545 */
      cur_add(s, i, m->a, from);
      emit(s, i, m->a, K_PING, 0, 0, 0, NULL, 0);
      break;
  }
}

/* ---- routing of one wave ------------------------------------------------------------------------- */
typedef struct { uint32_t* idx; size_t n, cap; } oidx;
static void ipush(oidx* v, uint32_t x) {
  if (v->n == v->cap) { v->cap = v->cap ? v->cap * 2 : 4; v->idx = (uint32_t*)realloc(v->idx, v->cap * 4); }
  v->idx[v->n++] = x;
}

/* Collect per-node outboxes (sender order, then seq) into one array, and reset them. */
static omsg* gather_out(kbo_sim* s, size_t* total) {
  size_t t = 0;
  for (uint32_t i = 0; i < s->C; ++i) t += s->out[i].n;
  omsg* all = (omsg*)malloc(sizeof(omsg) * (t ? t : 1));
  size_t k = 0;
  for (uint32_t i = 0; i < s->C; ++i) {
    for (size_t q = 0; q < s->out[i].n; ++q) {
      all[k++] = s->out[i].v[q];
      switch (s->out[i].v[q].kind) {
        case K_PING: s->st.sent_ping++; break;
        case K_PINGREQ: s->st.sent_ping_req++; break;
        case K_ACK: s->st.sent_ack++; break;
        case K_KP: s->st.sent_known_peers++; s->st.sent_kp_ids += s->out[i].v[q].pay_len; break;
        case K_KPR: s->st.sent_kpr++; break;
      }
    }
    s->out[i].n = 0;
    s->oseq[i] = 0;
  }
  *total = t;
  return all;
}

static int run_waves(kbo_sim* s, int32_t r) {
  uint32_t C = s->C;
  oidx* inb0 = (oidx*)calloc(C, sizeof(oidx));
  oidx* inb1 = (oidx*)calloc(C, sizeof(oidx));
  for (uint32_t w = 0; w < s->cfg.max_waves; ++w) {
    size_t M;
    omsg* all = gather_out(s, &M);
    if (M == 0) { free(all); break; }
    for (uint32_t i = 0; i < C; ++i) { inb0[i].n = 0; inb1[i].n = 0; }
    for (size_t k = 0; k < M; ++k) {
      omsg* m = &all[k];
      if (!s->alive[m->dest] && s->ext[m->dest]) {      /* to an external peer: leaves the simulated transport */
        if (partition_blocks(s, r, m->sender, m->dest)) { s->st.drop_partition++; continue; }   /* unless cut off */
        if (s->nxp == s->capxp) { s->capxp = s->capxp ? 2 * s->capxp : 64; s->xp = (kb_unicast*)realloc(s->xp, s->capxp * sizeof(kb_unicast)); }
        kb_unicast* x = &s->xp[s->nxp++];
        memset(x, 0, sizeof *x);
        x->round = r; x->wave = w; x->sender = m->sender; x->dest = m->dest; x->seq = m->seq; x->kind = m->kind;
        x->a = m->kind == K_KP ? 0 : m->a; x->fp = m->fp; x->n = m->n;
        x->pay_off = (uint32_t)s->nxids; x->pay_len = m->kind == K_KP ? m->pay_len : 0;
        if (x->pay_len) {
          if (s->nxids + x->pay_len > s->capxids) {
            while (s->nxids + x->pay_len > s->capxids) s->capxids = s->capxids ? 2 * s->capxids : 1024;
            s->xids = (uint32_t*)realloc(s->xids, s->capxids * 4);
          }
          memcpy(s->xids + s->nxids, m->pay, 4u * x->pay_len);
          s->nxids += x->pay_len;
        }
        s->st.exported++;
        continue;
      }
      if (!s->alive[m->dest]) { s->st.drop_dead++; continue; }
      if (partition_blocks(s, r, m->sender, m->dest)) { s->st.drop_partition++; continue; }
      if (active_faults(s, r) && s->cfg.loss_threshold &&
          ph(s, m->sender, (uint32_t)r, ((uint32_t)P_LOSS << 24) | w, m->seq).v[0] < s->cfg.loss_threshold) {
        s->st.drop_loss++; continue;
      }
      ipush(m->kind == K_KP ? &inb0[m->dest] : &inb1[m->dest], (uint32_t)k);
    }
#pragma omp parallel for schedule(dynamic, 64)
    for (uint32_t i = 0; i < C; ++i) {
      /* KnownPeers first (arrival order is free; this group commutes), then the rest,
         each in (sender, seq) order */
      for (size_t q = 0; q < inb0[i].n; ++q) handle_message(s, i, &all[inb0[i].idx[q]], r, w);
      for (size_t q = 0; q < inb1[i].n; ++q) handle_message(s, i, &all[inb1[i].idx[q]], r, w);
    }
    for (size_t k = 0; k < M; ++k) free(all[k].pay);
    free(all);
  }
  /* whatever was emitted in the last wave misses the receive window */
  for (uint32_t i = 0; i < C; ++i) {
    s->st.drop_window += s->out[i].n;
    for (size_t q = 0; q < s->out[i].n; ++q) {
      switch (s->out[i].v[q].kind) {
        case K_PING: s->st.sent_ping++; break;
        case K_PINGREQ: s->st.sent_ping_req++; break;
        case K_ACK: s->st.sent_ack++; break;
        case K_KP: s->st.sent_known_peers++; s->st.sent_kp_ids += s->out[i].v[q].pay_len; break;
        case K_KPR: s->st.sent_kpr++; break;
      }
      free(s->out[i].v[q].pay);
    }
    s->out[i].n = 0; s->oseq[i] = 0;
  }
  for (uint32_t i = 0; i < C; ++i) { free(inb0[i].idx); free(inb1[i].idx); }
  free(inb0); free(inb1);
  return KB_OK;
}

/* fingerprint of the true running set */
static uint32_t true_fp(kbo_sim* s) {
  uint32_t raw = 0; uint64_t len = 0;
  for (uint32_t j = 0; j < s->C; ++j)
    if (s->alive[j]) { raw = o_multmodp(s->segmul[j], raw) ^ s->cseg[j]; len += s->seglen[j]; }
  return raw ^ o_multmodp(o_xpow8(len), 0xFFFFFFFFu) ^ 0xFFFFFFFFu;
}

/* ---- one round ----------------------------------------------------------------------------------- */
static int step_round(kbo_sim* s) {
  int32_t r = s->round;
  uint32_t C = s->C;
  /* 0. stamp window: every EPOCH rounds the base advances; known stamps shift down, saturating */
  if (r > 0 && r % EPOCH == 0 && s->sr) {
#pragma omp parallel for schedule(dynamic, 64)
    for (uint32_t i = 0; i < C; ++i) {            /* explicit stamps that saturate become implicit */
      srow* rr = &s->sr[i];
      uint32_t o = 0;
      for (uint32_t q = 0; q < rr->nl; ++q) {
        uint8_t b = rr->lb[q];
        if (b > ST_ANCIENT) b = (uint8_t)(b - EPOCH > ST_ANCIENT ? b - EPOCH : ST_ANCIENT);
        if (b == ST_ANCIENT) continue;
        rr->lid[o] = rr->lid[q]; rr->lb[o] = b; o++;
      }
      rr->nl = o;
    }
  } else if (r > 0 && r % EPOCH == 0) {
    size_t tot = (size_t)C * C;
#pragma omp parallel for
    for (size_t k = 0; k < tot; ++k) {
      uint8_t b = s->stamp[k];
      if (b > ST_ANCIENT) s->stamp[k] = (uint8_t)(b - EPOCH > ST_ANCIENT ? b - EPOCH : ST_ANCIENT);
    }
  }
  /* 1. lifecycle: API events in call order, then churn (leaves in id order, joins with fresh ids) */
  for (size_t k = 0; k < s->nev; ++k) {
    uint32_t i = s->ev[k].node;
    if (s->ev[k].kind == EV_STOP) { if (s->alive[i]) node_stop(s, i); }
    else if (s->ev[k].kind == EV_RESTART) node_restart(s, s->ev[k].src, i, r);
    else if (!s->alive[i]) node_start(s, i, r);
  }
  s->nev = 0;
  if (active_faults(s, r) && s->cfg.churn_threshold) {
    uint32_t leaves = 0;
    for (uint32_t i = 0; i < C; ++i) {
      if (!s->alive[i] || s->start_round[i] == r) continue;
      if (ph(s, i, (uint32_t)r, (uint32_t)P_CHURN << 24, 0).v[0] < s->cfg.churn_threshold) { node_stop(s, i); leaves++; }
    }
    s->st.churn_leaves += leaves;
    for (uint32_t k = 0; k < leaves; ++k) {       /* fresh ids: an address some instance bound is skipped */
      while (s->next_free < C && !fresh_id(s, s->next_free)) s->next_free++;
      if (s->next_free >= C) break;
      node_start(s, s->next_free++, r); s->st.churn_joins++;
    }
  }
  /* the Probes queued since the last round travel with this round's broadcasts */
  free(s->probes);
  s->probes = s->probe_q; s->nprobes = s->nprobe_q;
  s->probe_q = NULL; s->nprobe_q = 0; s->capprobe_q = 0;
  const size_t presp0 = s->npresp;
  /* 2. broadcasts emitted during round r-1 (KB_VARIANT_SAME_WINDOW_BCAST: after this round's tick) */
  const int same_window = (s->cfg.variant & KB_VARIANT_SAME_WINDOW_BCAST) != 0;
  if (!same_window) {
    merge_ext_joins(s);
#pragma omp parallel for schedule(dynamic, 64)
    for (uint32_t i = 0; i < C; ++i)
      if (s->alive[i] && s->start_round[i] < r) phase_broadcasts(s, i, r);
  }
  if (s->npresp > presp0) {               /* canonical order within the round: (responder, probe) */
    kb_probe_response* v = s->presp + presp0;
    const size_t m = s->npresp - presp0;
    for (size_t a = 1; a < m; ++a) {
      kb_probe_response t = v[a];
      size_t b = a;
      while (b > 0 && (v[b - 1].responder > t.responder || (v[b - 1].responder == t.responder && v[b - 1].probe > t.probe))) {
        v[b] = v[b - 1]; --b;
      }
      v[b] = t;
    }
  }
  /* 3. tick */
  otick_bc* bc = (otick_bc*)calloc(C, sizeof(otick_bc));
  int err = KB_OK;
  uint32_t tfp = true_fp(s);
  uint32_t agree = 0, alive = 0;
#pragma omp parallel for schedule(dynamic, 64) reduction(+:agree, alive)
  for (uint32_t i = 0; i < C; ++i) {
    if (!s->alive[i]) continue;
    if (tick(s, i, r, &bc[i]) != KB_OK) err = KB_CAPACITY;
    alive++;
    agree += cur_fp(s, i) == tfp;        /* fingerprint at the ping step */
  }
  if (err) { free(bc); seterr("suspect slots exhausted"); return err; }
  s->nbfail = 0; s->nbjoin = 0;
  for (uint32_t i = 0; i < C; ++i) {
    uint32_t bseq = 0;
    if (bc[i].join) { bpush(&s->bjoin, &s->nbjoin, &s->capbjoin, i, i, bseq++); s->st.bcast_join++; }
    for (int q = 0; q < bc[i].nfail; ++q) { bpush(&s->bfail, &s->nbfail, &s->capbfail, i, bc[i].fail_peers[q], bseq++); s->st.bcast_failed++; }
  }
  free(bc);
  if (same_window) {            /* the tick's broadcasts reach every running peer inside this window */
    merge_ext_joins(s);
#pragma omp parallel for schedule(dynamic, 64)
    for (uint32_t i = 0; i < C; ++i)
      if (s->alive[i]) phase_broadcasts(s, i, r);
  }
  /* records from external peers (kbo_sim_inject): their wave-0 emissions, in call order */
  for (size_t k = 0; k < s->ninj; ++k) {
    const omsg* m = &s->inj[k];
    emit(s, m->sender, m->dest, m->kind, m->a, m->fp, m->n, m->pay, m->pay_len);
  }
  s->ninj = 0;
  /* 4. receive window: unicast waves */
  err = run_waves(s, r);
  if (err) return err;
  s->st.agree = agree; s->st.alive = alive; s->st.alive_rounds += alive;
  if (alive && agree == alive) {
    if (s->st.first_converged_round < 0) s->st.first_converged_round = r;
    s->st.last_converged_round = r;
  }
  s->round = r + 1;
  return KB_OK;
}

int kbo_sim_step(kbo_sim* s, uint32_t rounds) {
  if (!s) return KB_INVALID_ARGUMENT;
  for (uint32_t k = 0; k < rounds; ++k) { int e = step_round(s); if (e) return e; }
  return KB_OK;
}

/* ---- API ---------------------------------------------------------------------------------------- */
static int check(kbo_sim* s, uint32_t node) { return (!s || node >= s->C) ? KB_INVALID_ARGUMENT : KB_OK; }

static void push_ev(kbo_sim* s, int kind, uint32_t node, uint32_t src) {
  if (s->nev == s->capev) { s->capev = s->capev ? s->capev * 2 : 16; s->ev = (oevent*)realloc(s->ev, s->capev * sizeof(oevent)); }
  s->ev[s->nev].kind = kind; s->ev[s->nev].node = node; s->ev[s->nev].src = src; s->nev++;
}
/* running as the API sees it: the last lifecycle call queued for the node since the last step (they
 * take effect at the next round start), else its current state.  A queued restart moves the instance
 * away from its old address, which stays stopped. */
static int api_running(const kbo_sim* s, uint32_t node) {
  for (uint32_t k = s->nev; k-- > 0;) {
    if (s->ev[k].node == node) return s->ev[k].kind != EV_STOP;
    if (s->ev[k].kind == EV_RESTART && s->ev[k].src == node) return 0;
  }
  return s->alive[node];
}
/* the address has been bound by an instance (it ran, or a start of it is queued) */
static int ever_bound(const kbo_sim* s, uint32_t node) {
  if (s->start_round[node] != INT32_MIN) return 1;
  for (uint32_t k = 0; k < s->nev; ++k) if (s->ev[k].node == node && s->ev[k].kind != EV_STOP) return 1;
  return 0;
}
/* a fresh address: never bound by an instance (ran, or a start is queued) and given no identity; churn joins
 * and restarts take the next one in id order, so they never land on an address the API already used */
static int fresh_id(const kbo_sim* s, uint32_t id) { return !ever_bound(s, id) && !s->idset[id]; }
/* the first start of an instance at address `node` (src/lib.rs:136-156); a no-op while running.  A stopped
 * instance restarts at a fresh address: kbo_sim_restart_node. */
int kbo_sim_start_node(kbo_sim* s, uint32_t node) {
  if (check(s, node)) return KB_INVALID_ARGUMENT;
  if (!api_running(s, node) && ever_bound(s, node)) {
    seterr("a stopped instance restarts at a fresh address (kb_sim_restart_node)");
    return KB_INVALID_OPERATION;
  }
  push_ev(s, EV_START, node, node);
  return KB_OK;
}
int kbo_sim_stop_node(kbo_sim* s, uint32_t node) {
  if (check(s, node)) return KB_INVALID_ARGUMENT;
  push_ev(s, EV_STOP, node, node);
  return KB_OK;
}
/* Kaboodle::start for the instance last bound to `node` (src/lib.rs:136-156): running -> no-op (*out =
 * node); never bound -> its first start at `node`; stopped -> it binds a fresh ephemeral address
 * (src/kaboodle.rs:138-152): the next fresh id (the churn reserve, in allocation order) inherits its
 * known_peers map at the next round start, and carries the instance's identity (the one set while
 * stopped, if any).  *out = the instance's address from then on. */
int kbo_sim_restart_node(kbo_sim* s, uint32_t node, uint32_t* out) {
  if (check(s, node) || !out) return KB_INVALID_ARGUMENT;
  if (s->moved[node]) { seterr("the instance bound here restarted at a fresh address"); return KB_INVALID_OPERATION; }
  if (api_running(s, node)) { *out = node; return KB_OK; }
  if (!ever_bound(s, node)) { push_ev(s, EV_START, node, node); *out = node; return KB_OK; }
  uint32_t to = s->next_free;
  while (to < s->C && !fresh_id(s, to)) to++;
  if (to >= s->C) { seterr("no fresh address left for the restart (capacity)"); return KB_CAPACITY; }
  s->next_free = to + 1;
  const int pl = s->pend_len[node];
  const uint8_t* src = pl >= 0 ? s->pend_ident + (size_t)node * MAXID : s->ident + (size_t)node * MAXID;
  const uint32_t len = pl >= 0 ? (uint32_t)pl : s->id_len[node];
  memmove(s->ident + (size_t)to * MAXID, src, len);
  s->id_len[to] = (uint8_t)len;
  s->pend_len[to] = -1;
  s->pend_len[node] = -1;
  compute_seg(s, to);
  s->uniform = 1;
  for (uint32_t j = 0; j < s->C; ++j) if (s->id_len[j] != s->cfg.id_len) { s->uniform = 0; break; }
  push_ev(s, EV_RESTART, to, node);
  s->moved[node] = 1;
  *out = to;
  return KB_OK;
}
int kbo_sim_is_running(kbo_sim* s, uint32_t node, int* running) {
  if (check(s, node) || !running) return KB_INVALID_ARGUMENT;
  *running = s->alive[node];
  return KB_OK;
}
/* Kaboodle::ping_addrs (src/lib.rs:268-297): error while stopped; addresses already known are skipped */
int kbo_sim_ping_addrs(kbo_sim* s, uint32_t node, const uint32_t* peers, size_t n) {
  if (check(s, node) || (n && !peers)) return KB_INVALID_ARGUMENT;
  if (!s->alive[node]) { seterr("Cannot ping while we are not started"); return KB_INVALID_OPERATION; }
  for (size_t k = 0; k < n; ++k) {
    if (peers[k] >= s->C) return KB_INVALID_ARGUMENT;
    if (st_get(s, node, peers[k]) != ST_UNKNOWN) continue;
    if (s->paq_n[node] == PAQ) { seterr("ping_addrs queue full"); return KB_CAPACITY; }
    s->paq[(size_t)node * PAQ + s->paq_n[node]++] = peers[k];
  }
  return KB_OK;
}
/* Kaboodle::set_identity (src/lib.rs:323-336): refused while running.  Each view holds the identity an
 * address announced (PeerInfo.identity, written by the envelope prologue, a Join or a KnownPeers entry:
 * src/kaboodle.rs:409-414, :291-298, :461-468).  An instance changes identity only while stopped and comes
 * back at a fresh address (kbo_sim_restart_node), so every address keeps one identity for its lifetime
 * and one table per address equals every view's copy.  Hence: an address never bound takes the bytes
 * now; the instance stopped at an address that did run keeps them for its next address.  A non-uniform
 * length needs capacity <= 200 (the truncation sizes assume one length otherwise). */
int kbo_sim_set_identity(kbo_sim* s, uint32_t node, const uint8_t* identity, size_t len) {
  if (check(s, node) || len > MAXID || (len && !identity)) return KB_INVALID_ARGUMENT;
  if (s->moved[node]) { seterr("the instance bound here restarted at a fresh address"); return KB_INVALID_OPERATION; }
  if (api_running(s, node)) {
    seterr("Cannot change identity while the mesh is running; call .stop first");
    return KB_INVALID_OPERATION;
  }
  if (len != s->cfg.id_len && s->C > 200) { seterr("non-uniform identity length needs capacity <= 200"); return KB_INVALID_ARGUMENT; }
  if (ever_bound(s, node)) {
    memcpy(s->pend_ident + (size_t)node * MAXID, identity, len);
    s->pend_len[node] = (int16_t)len;
    return KB_OK;
  }
  memcpy(s->ident + (size_t)node * MAXID, identity, len);
  s->id_len[node] = (uint8_t)len;
  s->idset[node] = 1;
  compute_seg(s, node);
  s->uniform = 1;
  for (uint32_t j = 0; j < s->C; ++j) if (s->id_len[j] != s->cfg.id_len) { s->uniform = 0; break; }
  for (uint32_t j = 0; j < s->C; ++j) s->dirty[j] = 1;
  return KB_OK;
}

int kbo_sim_identity(kbo_sim* s, uint32_t node, uint8_t* buf, size_t cap, size_t* len) {
  if (check(s, node) || !len) return KB_INVALID_ARGUMENT;
  *len = s->id_len[node];
  if (!buf) return KB_OK;
  if (cap < *len) return KB_CAPACITY;
  memcpy(buf, s->ident + (size_t)node * MAXID, *len);
  return KB_OK;
}
/* SwimBroadcast::Probe from outside the mesh (src/discovery.rs:30-89), delivered next round */
int kbo_sim_probe(kbo_sim* s, const kb_wire_addr* prober) {
  if (!s || !prober) return KB_INVALID_ARGUMENT;
  if (s->nprobe_q == s->capprobe_q) {
    s->capprobe_q = s->capprobe_q ? 2 * s->capprobe_q : 8;
    s->probe_q = (kb_wire_addr*)realloc(s->probe_q, s->capprobe_q * sizeof(kb_wire_addr));
  }
  s->probe_q[s->nprobe_q++] = *prober;
  return KB_OK;
}
int kbo_sim_probe_responses(kbo_sim* s, kb_probe_response* out, size_t cap, size_t* n) {
  if (!s || !n) return KB_INVALID_ARGUMENT;
  *n = s->npresp;
  if (!out) return KB_OK;
  if (cap < s->npresp) return KB_CAPACITY;
  if (s->npresp) memcpy(out, s->presp, s->npresp * sizeof(kb_probe_response));
  s->npresp = 0;
  return KB_OK;
}
/* the last round's Join / Failed broadcasts (to be delivered at the next round start), sender order */
int kbo_sim_broadcasts(kbo_sim* s, kb_broadcast* out, size_t cap, size_t* n) {
  if (!s || !n) return KB_INVALID_ARGUMENT;
  /* canonical order: by sender, then bseq (a node's Join comes before its Failed entries) */
  size_t c = 0, a = 0, b = 0;
  while (a < s->nbjoin || b < s->nbfail) {
    int take_join = b == s->nbfail || (a < s->nbjoin && s->bjoin[a].sender <= s->bfail[b].sender);
    if (out && c < cap) {
      kb_broadcast* o = &out[c];
      memset(o, 0, sizeof *o);
      if (take_join) { o->kind = KB_WIRE_JOIN; o->sender = s->bjoin[a].sender; o->peer = s->bjoin[a].peer; }
      else { o->kind = KB_WIRE_FAILED; o->sender = s->bfail[b].sender; o->peer = s->bfail[b].peer; }
    }
    if (take_join) a++; else b++;
    c++;
  }
  *n = c;
  return (out && cap < c) ? KB_CAPACITY : KB_OK;
}
int kbo_sim_fingerprint(kbo_sim* s, uint32_t node, uint32_t* fp) {
  if (check(s, node) || !fp) return KB_INVALID_ARGUMENT;
  *fp = cur_fp(s, node);
  return KB_OK;
}
int kbo_sim_fingerprints(kbo_sim* s, uint32_t* fps, size_t cap) {
  if (!s || !fps || cap < s->C) return KB_INVALID_ARGUMENT;
#pragma omp parallel for schedule(dynamic, 64)
  for (uint32_t i = 0; i < s->C; ++i) fps[i] = s->alive[i] ? cur_fp(s, i) : 0;
  return KB_OK;
}
int kbo_sim_true_fingerprint(kbo_sim* s, uint32_t* fp) {
  if (!s || !fp) return KB_INVALID_ARGUMENT;
  *fp = true_fp(s);
  return KB_OK;
}
int kbo_sim_peers(kbo_sim* s, uint32_t node, uint32_t* peers, size_t cap, size_t* n) {
  if (check(s, node) || !n) return KB_INVALID_ARGUMENT;
  uint8_t* tmp;
  const uint8_t* rw = row_view(s, node, &tmp);
  size_t c = 0;
  for (uint32_t j = 0; j < s->C; ++j) if (rw[j]) { if (peers && c < cap) peers[c] = j; c++; }
  free(tmp);
  *n = c;
  return (peers && cap < c) ? KB_CAPACITY : KB_OK;
}
/* Event streams, src/events.rs:18-125 (observer attached empty in Kaboodle::new, src/lib.rs:112).
 * One drain = one batch: discovered = members now and not at the last drain (Added, :59-79),
 * departed = members then and not now (Removed, :88-99), both ascending; the fingerprint is reported
 * as changed when the map is non-empty and it differs from the last reported one (:103-122). */
int kbo_sim_watch(kbo_sim* s, uint32_t node) {
  if (check(s, node)) return KB_INVALID_ARGUMENT;
  for (size_t k = 0; k < s->nwatch; ++k) if (s->wnode[k] == node) return KB_OK;
  s->wnode = (uint32_t*)realloc(s->wnode, (s->nwatch + 1) * sizeof(uint32_t));
  s->wfp = (uint32_t*)realloc(s->wfp, (s->nwatch + 1) * sizeof(uint32_t));
  s->wsnap = (uint8_t**)realloc(s->wsnap, (s->nwatch + 1) * sizeof(uint8_t*));
  s->wnode[s->nwatch] = node; s->wfp[s->nwatch] = 0;
  s->wsnap[s->nwatch] = (uint8_t*)calloc(s->C, 1);
  s->nwatch++;
  return KB_OK;
}
int kbo_sim_events(kbo_sim* s, uint32_t node, uint32_t* discovered, size_t cap_d, size_t* n_d,
                   uint32_t* departed, size_t cap_p, size_t* n_p, uint32_t* fp, int* fp_changed) {
  if (check(s, node) || !n_d || !n_p || !fp || !fp_changed) return KB_INVALID_ARGUMENT;
  size_t k = 0;
  while (k < s->nwatch && s->wnode[k] != node) ++k;
  if (k == s->nwatch) { seterr("node is not watched (kbo_sim_watch)"); return KB_INVALID_OPERATION; }
  uint8_t* tmp;
  const uint8_t* rw = row_view(s, node, &tmp);
  uint8_t* snap = s->wsnap[k];
  size_t a = 0, r = 0, known = 0;
  for (uint32_t j = 0; j < s->C; ++j) {
    const int now = rw[j] != 0, then = snap[j] != 0;
    known += now;
    a += now && !then;
    r += then && !now;
  }
  *n_d = a; *n_p = r;
  *fp = cur_fp(s, node);
  *fp_changed = known > 0 && *fp != s->wfp[k];
  const int fit = (!a || (discovered && cap_d >= a)) && (!r || (departed && cap_p >= r));
  if (!fit) {
    free(tmp);
    if (discovered || departed) { seterr("event buffer too small"); return KB_CAPACITY; }
    return KB_OK;
  }
  a = r = 0;
  for (uint32_t j = 0; j < s->C; ++j) {
    const int now = rw[j] != 0, then = snap[j] != 0;
    if (now && !then) discovered[a++] = j;
    if (then && !now) departed[r++] = j;
    snap[j] = (uint8_t)now;
  }
  if (*fp_changed) s->wfp[k] = *fp;
  free(tmp);
  return KB_OK;
}
int kbo_sim_peer_states(kbo_sim* s, uint32_t node, kb_peer_state* out, size_t cap, size_t* n) {
  if (check(s, node) || !n) return KB_INVALID_ARGUMENT;
  uint8_t* tmp;
  const uint8_t* rw = row_view(s, node, &tmp);
  size_t c = 0;
  /* the stamps hold the encoding of the last simulated round (the window is rebased at the START of
   * a round, step_round above), so their base is epoch_base(round - 1), not epoch_base(round) */
  int32_t E = epoch_base(s->round > 0 ? s->round - 1 : 0);
  for (uint32_t j = 0; j < s->C; ++j) {
    if (!rw[j]) continue;
    if (out && c < cap) {
      kb_peer_state* o = &out[c];
      memset(o, 0, sizeof *o);
      o->peer = j;
      o->latency_ms = s->lat && s->lat[(size_t)node * s->C + j] != LAT_NONE ? s->lat[(size_t)node * s->C + j] : KB_LATENCY_NONE;
      o->identity_len = s->id_len[j];
      memcpy(o->identity, s->ident + (size_t)j * MAXID, s->id_len[j]);
      if (rw[j] == ST_SUSPECT) {
        osusp* q = susp_find(s, node, j);
        o->state = q && q->kind == SK_WFIP ? KB_STATE_WAITING_FOR_INDIRECT_PING : KB_STATE_WAITING_FOR_PING;
        o->since = q ? q->since : 0;
      } else {
        o->state = KB_STATE_KNOWN;
        o->since = rw[j] == ST_ANCIENT ? INT32_MIN : (int32_t)rw[j] + E - EOFF;
      }
    }
    c++;
  }
  free(tmp);
  *n = c;
  return (out && cap < c) ? KB_CAPACITY : KB_OK;
}
int kbo_sim_stats(kbo_sim* s, kb_stats* out) {
  if (!s || !out) return KB_INVALID_ARGUMENT;
  *out = s->st;
  out->round = s->round;
  out->next_free_id = s->next_free;
  uint32_t a = 0;
  for (uint32_t i = 0; i < s->C; ++i) a += s->alive[i];
  out->alive = a;
  return KB_OK;
}
int kbo_sim_dump_row(kbo_sim* s, uint32_t node, uint8_t* rw, size_t cap) {
  if (check(s, node) || !rw || cap < s->C) return KB_INVALID_ARGUMENT;
  row_bytes(s, node, rw);
  return KB_OK;
}
int kbo_sim_dump_scalars(kbo_sim* s, int32_t* out, size_t cap) {
  if (!s || !out || cap < (size_t)s->C * 4) return KB_INVALID_ARGUMENT;
  for (uint32_t i = 0; i < s->C; ++i) {
    out[4 * i] = s->alive[i]; out[4 * i + 1] = (int32_t)s->n[i];
    out[4 * i + 2] = s->last_bcast[i]; out[4 * i + 3] = s->start_round[i];
  }
  return KB_OK;
}
int kbo_sim_dump_suspects(kbo_sim* s, uint32_t node, int32_t* out, size_t cap, size_t* n) {
  if (check(s, node) || !n) return KB_INVALID_ARGUMENT;
  osusp* sl = s->susp + (size_t)node * SLOTS;
  int32_t tmp[SLOTS][3]; size_t c = 0;
  for (int k = 0; k < SLOTS; ++k) if (sl[k].kind) { tmp[c][0] = (int32_t)sl[k].peer; tmp[c][1] = sl[k].kind; tmp[c][2] = sl[k].since; c++; }
  for (size_t a = 1; a < c; ++a) for (size_t b = a; b > 0 && tmp[b - 1][0] > tmp[b][0]; --b) {
    int32_t t[3]; memcpy(t, tmp[b], sizeof t); memcpy(tmp[b], tmp[b - 1], sizeof t); memcpy(tmp[b - 1], t, sizeof t);
  }
  *n = c;
  if (out) { if (cap < 3 * c) return KB_CAPACITY; memcpy(out, tmp, sizeof(int32_t) * 3 * c); }
  return KB_OK;
}
int kbo_sim_dump_curious(kbo_sim* s, uint32_t node, int32_t* out, size_t cap, size_t* n) {
  if (check(s, node) || !n) return KB_INVALID_ARGUMENT;
  ocur* cu = s->cur + (size_t)node * CSLOTS;
  int32_t tmp[CSLOTS][6]; size_t c = 0;
  for (int k = 0; k < CSLOTS; ++k) if (cu[k].used) {
    tmp[c][0] = (int32_t)cu[k].peer; tmp[c][1] = (int32_t)cu[k].nobs;
    for (int q = 0; q < NOBS; ++q) tmp[c][2 + q] = q < (int)cu[k].nobs ? (int32_t)cu[k].obs[q] : -1;
    c++;
  }
  for (size_t a = 1; a < c; ++a) for (size_t b = a; b > 0 && tmp[b - 1][0] > tmp[b][0]; --b) {
    int32_t t[6]; memcpy(t, tmp[b], sizeof t); memcpy(tmp[b], tmp[b - 1], sizeof t); memcpy(tmp[b - 1], t, sizeof t);
  }
  *n = c;
  if (out) { if (cap < 6 * c) return KB_CAPACITY; memcpy(out, tmp, sizeof(int32_t) * 6 * c); }
  return KB_OK;
}

/* pure helpers */
uint32_t kbo_fingerprint_of_set(const uint32_t* ids, size_t n, const uint8_t* identities, size_t stride,
                                const uint8_t* lens) {
  o_crc_init();
  uint32_t* v = (uint32_t*)malloc(sizeof(uint32_t) * (n ? n : 1));
  memcpy(v, ids, sizeof(uint32_t) * n);
  for (size_t a = 1; a < n; ++a) { uint32_t t = v[a]; size_t b = a; while (b > 0 && v[b - 1] > t) { v[b] = v[b - 1]; --b; } v[b] = t; }
  uint32_t reg = 0xFFFFFFFFu;
  char a[32];
  for (size_t k = 0; k < n; ++k) {
    kbo_format_addr(v[k], a, sizeof a);
    reg = o_crc_update(reg, (const uint8_t*)a, strlen(a));
    if (identities && lens) reg = o_crc_update(reg, identities + v[k] * stride, lens[v[k]]);
  }
  free(v);
  return n ? reg ^ 0xFFFFFFFFu : 0;
}
/* KB_VARIANT_SPARSE_ROWS footprint (test infrastructure): out = [rows that adopted the base,
 * exceptions, explicit stamps, entries of the largest row, bytes (4 per exception, 5 per stamp), rows] */
int kbo_sparse_footprint(kbo_sim* s, uint64_t* out, size_t cap) {
  if (!s || !s->sr || !out || cap < 6) return KB_INVALID_ARGUMENT;
  uint64_t based = 0, nx = 0, nl = 0, mx = 0;
  for (uint32_t i = 0; i < s->C; ++i) {
    const srow* r = &s->sr[i];
    based += r->based; nx += r->nx; nl += r->nl;
    if (r->nx + r->nl > mx) mx = r->nx + r->nl;
  }
  out[0] = based; out[1] = nx; out[2] = nl; out[3] = mx; out[4] = 4 * nx + 5 * nl; out[5] = s->C;
  return KB_OK;
}
/* external peers: include/kaboodle_sim.h kb_sim_set_external / kb_sim_inject / kb_sim_exported */
int kbo_sim_set_external(kbo_sim* s, uint32_t node) {
  if (check(s, node)) return KB_INVALID_ARGUMENT;
  if (s->ext[node]) return KB_OK;
  if (ever_bound(s, node)) { seterr("an external peer takes an address no instance has bound"); return KB_INVALID_OPERATION; }
  s->ext[node] = 1;
  s->idset[node] = 1;                       /* not a fresh id: churn joins and restarts skip it */
  return KB_OK;
}
int kbo_sim_inject(kbo_sim* s, const kb_unicast* m, const uint32_t* ids) {
  if (!s || !m || m->sender >= s->C || m->dest >= s->C || (m->kind > K_KPR && m->kind != KB_WIRE_JOIN) || (m->pay_len && !ids))
    return KB_INVALID_ARGUMENT;
  if (!s->ext[m->sender]) { seterr("kb_sim_inject: the sender is not an external peer"); return KB_INVALID_OPERATION; }
  if (m->kind == KB_WIRE_JOIN) {                       /* a Join broadcast: the next round's Join list */
    for (size_t k = 0; k < s->ninjj; ++k)
      if (s->injj[k] == m->sender) { seterr("kb_sim_inject: one Join per external peer per round"); return KB_CAPACITY; }
    if (s->ninjj == s->capinjj) { s->capinjj = s->capinjj ? 2 * s->capinjj : 8; s->injj = (uint32_t*)realloc(s->injj, 4 * s->capinjj); }
    s->injj[s->ninjj++] = m->sender;
    return KB_OK;
  }
  if ((m->kind == K_PINGREQ || m->kind == K_ACK) && m->a >= s->C) return KB_INVALID_ARGUMENT;
  for (uint32_t k = 0; k < m->pay_len; ++k) if (ids[k] >= s->C) return KB_INVALID_ARGUMENT;
  size_t per = 0;
  for (size_t k = 0; k < s->ninj; ++k) per += s->inj[k].sender == m->sender;
  if (per >= (size_t)(3 * SLOTS + 1 + PAQ)) { seterr("kb_sim_inject: 33 records per external peer per round"); return KB_CAPACITY; }
  if (s->ninj == s->capinj) { s->capinj = s->capinj ? 2 * s->capinj : 16; s->inj = (omsg*)realloc(s->inj, s->capinj * sizeof(omsg)); }
  omsg* o = &s->inj[s->ninj++];
  memset(o, 0, sizeof *o);
  o->sender = m->sender; o->dest = m->dest; o->kind = m->kind; o->fp = m->fp; o->n = m->n;
  if (m->kind == K_KP) {
    o->pay_len = m->pay_len; o->a = m->pay_len;
    o->pay = (uint32_t*)malloc(4u * (m->pay_len ? m->pay_len : 1));
    if (m->pay_len) memcpy(o->pay, ids, 4u * m->pay_len);
  } else {
    o->a = m->a;
  }
  return KB_OK;
}
static int o_cmp_u32(const void* a, const void* b) {
  const uint32_t x = *(const uint32_t*)a, y = *(const uint32_t*)b;
  return x < y ? -1 : x > y;
}
int kbo_sim_exported(kbo_sim* s, kb_unicast* out, size_t cap, size_t* n, uint32_t* ids, size_t cap_ids, size_t* n_ids) {
  if (!s || !n || !n_ids) return KB_INVALID_ARGUMENT;
  *n = s->nxp; *n_ids = s->nxids;
  if (!out && !ids) return KB_OK;
  if (cap < s->nxp || (s->nxids && (!ids || cap_ids < s->nxids))) { seterr("export buffer too small"); return KB_CAPACITY; }
  if (s->nxp) memcpy(out, s->xp, s->nxp * sizeof(kb_unicast));
  for (size_t k = 0; k < s->nxp; ++k)                  /* a KnownPeers map has no order: ascending ids */
    if (s->xp[k].pay_len > 1) qsort(s->xids + s->xp[k].pay_off, s->xp[k].pay_len, 4, o_cmp_u32);
  if (s->nxids) memcpy(ids, s->xids, 4u * s->nxids);
  s->nxp = 0; s->nxids = 0;
  return KB_OK;
}
int kbo_sim_sparse_footprint(kbo_sim* s, uint64_t* out, size_t cap) {
  if (!s || !out) return KB_INVALID_ARGUMENT;
  if (!s->sr) { seterr("not a KB_VARIANT_SPARSE_ROWS handle"); return KB_INVALID_OPERATION; }
  return kbo_sparse_footprint(s, out, cap);
}
uint32_t kbo_crc32(const uint8_t* p, size_t n) { o_crc_init(); return o_crc32(p, n); }
void kbo_philox(uint32_t c0, uint32_t c1, uint32_t c2, uint32_t c3, uint32_t k0, uint32_t k1, uint32_t* out4) {
  o_u32x4 o = o_philox(c0, c1, c2, c3, k0, k1);
  memcpy(out4, o.v, 16);
}
int kbo_num_threads(void) {
#ifdef _OPENMP
  return omp_get_max_threads();
#else
  return 1;
#endif
}
/* bench.py's single-thread figure: the OpenMP build restricted to n threads for the calls that follow */
void kbo_set_num_threads(int n) {
#ifdef _OPENMP
  if (n > 0) omp_set_num_threads(n);
#else
  (void)n;
#endif
}
