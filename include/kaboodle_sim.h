/*
 * kaboodle_sim.h — C ABI of the MI355X bulk-synchronous Kaboodle SWIM-round simulator.
 *
 * One handle = one simulated mesh of up to `capacity` virtual Kaboodle peers (ids 0..capacity-1),
 * all advancing in lock-step rounds on the GPU.  Each entry point below replaces a piece of the
 * per-instance Rust surface of serval/kaboodle v0.1.5 (paths relative to the reference root):
 *
 *   kb_sim_create / kb_sim_destroy   Kaboodle::new            src/lib.rs:93-133   (per mesh, not per peer)
 *   kb_sim_step                      KaboodleInner::run/tick  src/kaboodle.rs:746-786 (all peers, R rounds)
 *   kb_sim_start_node                Kaboodle::start          src/lib.rs:136-156, src/kaboodle.rs:114-185 (first start)
 *   kb_sim_restart_node              Kaboodle::start          the same, on a stopped instance: a fresh address
 *                                                             (src/kaboodle.rs:138-152) keeping its map (src/lib.rs:104,167-170)
 *   kb_sim_stop_node                 Kaboodle::stop           src/lib.rs:159-183
 *   kb_sim_ping_addrs                Kaboodle::ping_addrs     src/lib.rs:268-297
 *   kb_sim_fingerprint               Kaboodle::fingerprint    src/lib.rs:301-304 -> generate_fingerprint
 *                                                             src/kaboodle.rs:71-83
 *   kb_sim_peers                     Kaboodle::peers          src/lib.rs:339-345
 *   kb_sim_peer_states               Kaboodle::peer_states    src/lib.rs:348-354 (PeerState src/structs.rs:27-41)
 *   kb_sim_set_identity              Kaboodle::set_identity   src/lib.rs:323-336
 *   kb_sim_is_running                Kaboodle::is_running     src/lib.rs:307-309
 *   kb_format_addr                   Kaboodle::self_addr      src/lib.rs:312-314 (canonical simulated address)
 *   kb_fingerprint_of_set            generate_fingerprint     src/kaboodle.rs:71-83 (pure function)
 *   status codes                     KaboodleError            src/errors.rs:8-24
 *
 * Semantics ("round semantics v1") are specified in DESIGN.md §2; the CPU restatement used as the
 * parity oracle lives under oracle/ and exports the same functions with the prefix `kbo_`.
 *
 * Ownership: the library owns the handle and all device memory; every output buffer is caller-owned
 * (pass cap = 0 to query the required element count).  A handle is NOT thread-safe.  kb_sim_step is
 * synchronous: it returns after the simulated rounds have completed on the device.
 */
#ifndef KABOODLE_SIM_H
#define KABOODLE_SIM_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define KB_ABI_VERSION 3u   /* 2: kernel breakdown, identities on the inspection surface; 3: restarts bind a
                                fresh address (kb_sim_restart_node) */

/* ---- status codes (mirror KaboodleError, src/errors.rs:8-24) ------------------------------------ */
enum {
  KB_OK = 0,
  KB_INVALID_OPERATION = 1,  /* KaboodleError::InvalidOperation (e.g. ping_addrs while stopped)      */
  KB_IO_ERROR = 2,           /* KaboodleError::IoError -> HIP runtime / RCCL failure                 */
  KB_NO_DEVICE = 3,          /* KaboodleError::NoAvailableInterfaces -> no usable GPU                */
  KB_STOPPING_FAILED = 4,    /* KaboodleError::StoppingFailed                                        */
  KB_INVALID_ARGUMENT = 5,   /* bad config / id out of range / null pointer                          */
  KB_CAPACITY = 6            /* a declared fixed capacity was exceeded             */
};

/* ---- configuration ------------------------------------------------------------------------------ */
enum { KB_INIT_JOIN = 0,        /* initial nodes start at round 0 knowing only themselves (config 2)   */
       KB_INIT_CONVERGED = 1 }; /* initial nodes know every initial node, all stamps "ancient"          */

enum { KB_FAILED_SIM_SENDER = 0,      /* Failed(p) honoured iff the broadcasting node is known (Q1)    */
       KB_FAILED_SOCKET_FAITHFUL = 1 };/* Failed is never honoured (real-socket sender never matches)  */

typedef struct kb_config {
  uint32_t abi_version;      /* must be KB_ABI_VERSION                                               */
  uint32_t capacity;         /* C: number of peer ids (initial nodes + churn reserve), <= 7,800,000  */
  uint32_t initial_nodes;    /* ids 0..initial_nodes-1 are running at round 0                        */
  uint32_t init_mode;        /* KB_INIT_*                                                            */
  uint64_t seed;             /* Philox4x32-10 key                                                    */
  uint32_t loss_threshold;   /* a delivery is lost iff philox word < loss_threshold (p*2^32)         */
  uint32_t churn_threshold;  /* a running node leaves at round start iff philox word < threshold     */
  int32_t  fault_end_round;  /* loss and churn act only in rounds r < fault_end_round (-1: forever)   */
  uint32_t max_waves;        /* unicast delivery waves per round (>= 1; default 8)                   */
  uint32_t failed_mode;      /* KB_FAILED_*                                                          */
  uint32_t id_len;           /* default identity length in bytes (0..32) for every id               */
  uint32_t partition_groups; /* 0/1: none; G: ids split into G contiguous groups                      */
  int32_t  partition_start;  /* cross-group deliveries dropped for partition_start <= r < partition_end */
  int32_t  partition_end;
  int32_t  device;           /* HIP device ordinal, -1 = current device (ignored by the oracle)      */
  uint32_t debug_flags;      /* KB_DBG_*: force the wide-row (HBM) kernel variants at any size; results
                                are identical with any value (test surface, ignored by the oracle)   */
  uint32_t track_latency;    /* 1: keep the per-(node, peer) ping latency EWMA of peer_states
                                (src/kaboodle.rs:789-817); 0: latency reported as none (no table)    */
  uint32_t variant;          /* KB_VARIANT_*: 0 = round semantics v1.  Nonzero selects an alternative
                                reading of a declared deviation, implemented by the
                                CPU oracle, to measure what the declaration changes.  The HIP
                                library runs KB_VARIANT_EXACT_LRU alone (A3 by exact instants) and
                                KB_VARIANT_SPARSE_ROWS alone (the same semantics on the configs[4]
                                layout, unsharded) and refuses the rest
                                (KB_INVALID_ARGUMENT)                                                */
  uint32_t sparse_row_cap;   /* KB_VARIANT_SPARSE_ROWS on the GPU: entries per row (exceptions and
                                explicit stamps); 0 = min(capacity, 4096).  Exceeding it is
                                KB_CAPACITY, never a truncation (ignored by the oracle)              */
  uint32_t stat_flags;       /* KB_STAT_*: counters a long run may skip (0: count everything)         */
  uint32_t reserved[1];
} kb_config;
/* stat_flags */
enum { KB_STAT_NO_SF_FAILED_DROPS = 1u };  /* socket_faithful: do not count the lost deliveries of Failed
                                              broadcasts in drop_bcast.  In that mode Failed changes no state
                                              (DESIGN.md §2.10), so the count is its whole cost: one Philox word
                                              per (receiver, entry), O(N x entries) a round.  drop_bcast then
                                              counts Join and Probe losses only; all other state and counters
                                              are unchanged.  KB_VARIANT_SPARSE_ROWS and the oracle; the dense
                                              engine refuses it (KB_INVALID_ARGUMENT)                        */
enum { KB_VARIANT_SAME_WINDOW_BCAST = 1u,   /* Join/Failed delivered in the round they are sent, right after
                                               the tick (src/kaboodle.rs:770-778), not at the next round start */
       KB_VARIANT_EXACT_LRU = 2u,           /* A3 orders by the exact instant (no stamp window, no ancient ties) */
       KB_VARIANT_SPARSE_ROWS = 4u };       /* the same semantics on sparse rows: a shared base set, per-row
                                               exceptions and an explicit list of the non-ancient stamps
                                               (the configs[4] representation); no latency table */

/* debug_flags: each forces the code path a mesh of >= 1M ids takes, so that path is
   parity-tested at sizes the oracle finishes in seconds. */
enum {
  KB_DBG_PHASEB_HBM = 1u,    /* broadcast phase on the HBM bitset (rows > PB_LDS_W ids), lists from HBM */
  KB_DBG_RESP_HBM = 2u,      /* Join responses by workgroup with HBM scratch (rows > RESP_LDS_W ids)     */
  KB_DBG_KP_HBM = 4u,        /* KnownPeers groups on the HBM bitset, one workgroup per destination      */
  KB_DBG_KP_BIG_SMALL = 8u,  /* every KnownPeers group takes the BIG (1024-thread) kernel                */
  KB_DBG_PROC_UNSORTED = 16u,/* inboxes > 64 taken by k_proc's selection path (inboxes > SORT_MAX)       */
  KB_DBG_WAVE_GRAPH = 32u,   /* the unsharded receive window captured once as a HIP graph and replayed
                                every round (also env KB_WAVE_GRAPH=1)                  */
  KB_DBG_RESP_WAVE_HBM = 64u,/* Join responses by wave with the rows read in place (the path of rows too
                                wide for a wave's LDS copy, > 110K ids)                                */
  KB_DBG_NO_UNION = 128u     /* row shards: Join responses travel as their id lists, not as one union per
                                (source shard, joiner) (A/B and parity surface)          */
};

/* Per-peer state as reported by peer_states() (PeerState, src/structs.rs:27-41). */
enum { KB_STATE_KNOWN = 0, KB_STATE_WAITING_FOR_PING = 1, KB_STATE_WAITING_FOR_INDIRECT_PING = 2 };
typedef struct kb_peer_state {
  uint32_t peer;             /* peer id                                                             */
  uint32_t state;            /* KB_STATE_*                                                          */
  int32_t  since;            /* round of the state's Instant; INT32_MIN = older than the stamp window */
  uint32_t latency_ms;       /* PeerInfo.latency in simulated ms ; KB_LATENCY_NONE =
                                None (never measured, or track_latency off)                          */
  uint32_t identity_len;     /* PeerInfo.identity (src/structs.rs:18-22): the peer's identity bytes  */
  uint8_t  identity[32];
} kb_peer_state;
#define KB_LATENCY_NONE 0xFFFFFFFFu

/* Cumulative counters since creation (all ranks summed when sharded). */
typedef struct kb_stats {
  int32_t  round;                 /* next round to simulate                                          */
  uint32_t alive;                 /* running nodes now                                               */
  uint32_t agree;                 /* running nodes whose fingerprint at the last round's ping step
                                     equalled the fingerprint of the true running set               */
  int32_t  first_converged_round; /* first round with agree == alive (-1: never)                     */
  int32_t  last_converged_round;  /* most recent such round (-1: never)                              */
  uint32_t next_free_id;          /* next fresh id for churn joins                                   */
  uint64_t sent_ping, sent_ping_req, sent_ack, sent_known_peers, sent_kpr;
  uint64_t bcast_join, bcast_failed;
  uint64_t drop_dead, drop_loss, drop_window, drop_oversize, drop_partition, drop_bcast;
  uint64_t removed_timeout, removed_failed, join_responses, curious_overflow, churn_leaves, churn_joins;
  uint64_t sent_kp_ids;           /* peer entries carried by the KnownPeers messages sent               */
  uint64_t alive_rounds;          /* sum over the simulated rounds of the peers running in that round  */
  uint64_t probe_responses;       /* ProbeResponses sent (maybe_respond_to_probe), lost ones included   */
  uint64_t exported;              /* records routed to external peers (kb_sim_exported)                 */
  uint64_t reserved[4];
} kb_stats;

typedef struct kb_sim kb_sim;

/* Fill *cfg with defaults: capacity 1024, all running, KB_INIT_JOIN, seed 1, no faults, 8 waves. */
void kb_config_default(kb_config* cfg);

int  kb_sim_create(const kb_config* cfg, kb_sim** out);
int  kb_sim_destroy(kb_sim* sim);
/* Advance every running peer by `rounds` protocol periods. */
int  kb_sim_step(kb_sim* sim, uint32_t rounds);

/* The first start of the instance at address `node` (a no-op while it runs); takes effect at the next
   round start.  A stopped instance that has run restarts at a fresh address instead: KB_INVALID_OPERATION
   here, use kb_sim_restart_node. */
int  kb_sim_start_node(kb_sim* sim, uint32_t node);
int  kb_sim_stop_node(kb_sim* sim, uint32_t node);                  /* takes effect next round start */
/* Kaboodle::start for the instance last bound to address `node` (src/lib.rs:136-156).  Running: a no-op,
   *new_node = node.  Never bound: its first start, *new_node = node.  Stopped after running: the reference
   binds a fresh ephemeral socket on every start (src/kaboodle.rs:138-152) while the instance's known_peers
   map persists across stop/start (src/lib.rs:104, minus the old self removed by stop, :167-170).  So the
   next fresh id (the churn reserve, allocated now, in order) becomes the instance's address: at the next
   round start it inherits the old address's map (entries, states, instants, latencies), with fresh curious
   peers, ping queue and Join timer (a new KaboodleInner), and the old address stays in other views until
   pinged out.  Its identity is the instance's (the one set while stopped, if any).  Watches follow the
   instance.  KB_CAPACITY: no fresh id left.                                                           */
int  kb_sim_restart_node(kb_sim* sim, uint32_t node, uint32_t* new_node);
int  kb_sim_is_running(kb_sim* sim, uint32_t node, int* running);
int  kb_sim_ping_addrs(kb_sim* sim, uint32_t node, const uint32_t* peers, size_t n);
/* Kaboodle::set_identity (src/lib.rs:323-336): only while the node is not running, counting the start /
   stop calls queued since the last step (they take effect at the next round start).  Views hold the
   identity an address announced (PeerInfo.identity, src/kaboodle.rs:409-414, :291-298, :461-468); since an
   instance changes identity only while stopped and restarts at a fresh address, one identity per address
   is what every view holds.  An address never bound takes the bytes at once; for an instance stopped at
   an address that ran they are kept for its next address (kb_sim_restart_node) and kb_sim_identity(node)
   keeps reporting the bytes the views hold.                                                            */
int  kb_sim_set_identity(kb_sim* sim, uint32_t node, const uint8_t* identity, size_t len);
/* The identity bytes of id `node` (Kaboodle::peers / peer_states values, src/lib.rs:339-354): *len is
   the length; copied into buf when cap suffices (buf = NULL: length query).                         */
int  kb_sim_identity(kb_sim* sim, uint32_t node, uint8_t* buf, size_t cap, size_t* len);

int  kb_sim_fingerprint(kb_sim* sim, uint32_t node, uint32_t* fp);
int  kb_sim_fingerprints(kb_sim* sim, uint32_t* fps, size_t cap);   /* all ids; 0 for non-running  */
int  kb_sim_peers(kb_sim* sim, uint32_t node, uint32_t* peers, size_t cap, size_t* n);
int  kb_sim_peer_states(kb_sim* sim, uint32_t node, kb_peer_state* out, size_t cap, size_t* n);
int  kb_sim_stats(kb_sim* sim, kb_stats* out);
/* fingerprint of the true running set (what every converged node should report) */
int  kb_sim_true_fingerprint(kb_sim* sim, uint32_t* fp);

/* ---- event streams (src/events.rs:18-125; Kaboodle::discover_peers / discover_departures /
 * discover_fingerprint_changes, src/lib.rs:186-263) -------------------------------------------------
 * kb_sim_watch attaches an observer to `node`'s known_peers, empty, as Kaboodle::new does
 * (src/lib.rs:112).  kb_sim_events drains one batch: the NET change since the previous drain, ids
 * ascending.  discovered = known now and not at the last drain (Event::Added, events.rs:59-79);
 * departed = known then and not now (Event::Removed, :88-99).  *fp is the node's fingerprint and
 * *fp_changed = 1 when the node knows at least one peer and *fp differs from the last fingerprint
 * reported as changed (initially 0, :103-122).  A peer added and removed inside one batch yields no
 * event (the reference may emit a lone departure for it).  Buffers are caller-owned: with both
 * pointers NULL the call only reports the counts and drains nothing; a buffer too small for its
 * count gives KB_CAPACITY and drains nothing.  Not watched: KB_INVALID_OPERATION.               */
int  kb_sim_watch(kb_sim* sim, uint32_t node);
int  kb_sim_events(kb_sim* sim, uint32_t node, uint32_t* discovered, size_t cap_d, size_t* n_d,
                   uint32_t* departed, size_t cap_p, size_t* n_p, uint32_t* fp, int* fp_changed);

/* An IPv4 socket address as the wire carries it (SocketAddr::V4). */
typedef struct kb_wire_addr { uint8_t ip[4]; uint16_t port; uint16_t pad; } kb_wire_addr;

/* ---- discovery (src/discovery.rs:30-89, src/kaboodle.rs:305-331) ----------------------------------
 * kb_sim_probe queues SwimBroadcast::Probe(prober) from an address outside the mesh; it is delivered at
 * the next round start with that round's other broadcasts (after the Failed and Join groups, DESIGN.md
 * §2.4).  Every running peer that receives it answers with ProbeResponse{identity} iff
 * should_respond_to_broadcast (:333-354, the integer restatement of §2.4, its own Philox counter).
 * Deliveries and responses are subject to the loss of the round.  kb_sim_probe_responses drains the
 * responses produced since the last drain, ordered by (round, responder, probe); with out = NULL only
 * the count is reported.  Sharded ranks (kb_sim_create_rank) report the responders among their rows. */
typedef struct kb_probe_response {
  uint32_t responder;        /* the answering peer (its canonical address is the datagram's source) */
  uint32_t probe;            /* index of the probe among those queued for that round                */
  int32_t  round;
  kb_wire_addr prober;       /* where the ProbeResponse is sent                                      */
  uint32_t identity_len;     /* ProbeResponse.identity: the responder's identity                     */
  uint8_t  identity[32];
} kb_probe_response;
int  kb_sim_probe(kb_sim* sim, const kb_wire_addr* prober);
int  kb_sim_probe_responses(kb_sim* sim, kb_probe_response* out, size_t cap, size_t* n);
/* The round's broadcast lists as the transport carries them (what a bridge sends on the multicast socket,
   src/kaboodle.rs:188-195): the Join and Failed broadcasts emitted by the last simulated round (delivered
   at the next round start), sender order.  kind: KB_WIRE_JOIN or KB_WIRE_FAILED.                    */
typedef struct kb_broadcast { uint32_t kind, sender, peer, pad; } kb_broadcast;
int  kb_sim_broadcasts(kb_sim* sim, kb_broadcast* out, size_t cap, size_t* n);

/* ---- external peers: real instances attached through a bridge ----------------------
 * kb_sim_set_external marks an address no instance has bound as an EXTERNAL peer: a real Kaboodle instance
 * outside the mesh that simulated peers reach at that id (the bridge maps it to the real socket address).
 * It never runs in the mesh (no row, no tick, not in the running set or the agreement) and churn joins and
 * restarts skip it.  Every unicast record a simulated peer addresses to it and a delivery wave routes
 * (src/kaboodle.rs:197-226) is EXPORTED instead of delivered: the real network carries it from there.
 * kb_sim_exported drains them in (round, wave, sender, seq) order, KnownPeers ids into `ids` (pay_off /
 * pay_len; ascending within a record: the reference sends a HashMap, src/structs.rs:110, whose order
 * carries nothing).  kb_sim_inject queues a record from an external peer to a simulated one — what the bridge decoded
 * from a real socket (:394-403) — delivered in wave 0 of the next round as that peer's emissions, in call
 * order (seq), under the round's delivery rules (stopped receiver, partition, the Philox loss keyed on
 * (sender, round, wave, seq)); kind = KB_WIRE_PING .. KB_WIRE_KNOWN_PEERS_REQUEST, a = PingRequest / Ack
 * peer, fp / n = Ack / KnownPeersRequest fields, ids[pay_len] = a KnownPeers list (ids of the mesh).  At most
 * 33 records per external peer per round (KB_CAPACITY).  kind = KB_WIRE_JOIN injects the external peer's Join
 * broadcast (maybe_broadcast_join, src/kaboodle.rs:228-251; dest, a and ids unused): it joins the next
 * round's Join list at its sender place and reaches every running simulated peer under the broadcast rules
 * (:284-304: insert, maybe answer with KnownPeers — exported); one per external peer per round.  Handles of kb_sim_create_rank: every rank makes
 * these calls alike; each rank drains the exports of its own senders.                                   */
typedef struct kb_unicast {
  int32_t  round;                      /* kb_sim_exported: the round and wave that routed it               */
  uint32_t wave, sender, dest, seq, kind, a, fp, n, pay_off, pay_len, pad;
} kb_unicast;
int  kb_sim_set_external(kb_sim* sim, uint32_t node);
int  kb_sim_inject(kb_sim* sim, const kb_unicast* msg, const uint32_t* ids);
int  kb_sim_exported(kb_sim* sim, kb_unicast* out, size_t cap, size_t* n, uint32_t* ids, size_t cap_ids, size_t* n_ids);

/* ---- sharding across GPUs --------------------------------------------------------
 * A mesh of C ids can be split into `world` (1..8) contiguous row shards: shard k holds the observer
 * state of ids [k*S, min(C, (k+1)*S)), S = ceil(C/world).  The reference's UDP transport between
 * instances (src/kaboodle.rs:188-226, src/networking.rs:27-121) becomes, per round, an all-to-all-v
 * of each delivery wave's records and an all-gather of the Join/Failed broadcast lists.  Results are
 * bit-identical to the unsharded mesh (same Philox draws, same canonical orders).
 *
 * kb_sim_create_rank: one process per GPU.  Rank 0 makes the id with kb_rccl_unique_id and the host
 *   broadcasts it (e.g. over torch.distributed); every rank then creates its shard.  Calls that change
 *   the mesh (start/stop/set_identity/ping_addrs) and kb_sim_step / kb_sim_stats are collective: every
 *   rank makes them alike.  Row inspection (fingerprint/peers/peer_states/dump_*) is answered by the
 *   rank holding the row and returns KB_INVALID_ARGUMENT on the others; kb_sim_fingerprints and
 *   kb_sim_dump_scalars fill this rank's rows (zeros elsewhere).
 * kb_sim_create_local: all shards inside this process on one device (one host thread per shard and
 *   step), exchanged by device copies — the whole ABI then behaves as for an unsharded mesh.       */
#define KB_UNIQUE_ID_BYTES 128
int  kb_rccl_unique_id(uint8_t* out, size_t cap);
/* A unique id for ranks in separate processes that share ONE device (RCCL refuses two ranks on one GPU): given to
   kb_sim_create_rank it selects a test transport over IPC-mapped device windows and a shared-memory rendezvous
   (DESIGN.md §6), with the same collective discipline as RCCL.  Window: env KB_IPC_WINDOW_MB (default 256). */
int  kb_ipc_unique_id(uint8_t* out, size_t cap);
int  kb_sim_create_rank(const kb_config* cfg, int32_t rank, int32_t world, const uint8_t* unique_id,
                        kb_sim** out);
int  kb_sim_create_local(const kb_config* cfg, int32_t shards, kb_sim** out);
int  kb_sim_shard_info(kb_sim* sim, int32_t* rank, int32_t* world, uint32_t* lo, uint32_t* hi);

/* ---- parity / test surface ---------------------------------------------------------------------- */
/* Raw stamp row of `node` (capacity bytes, DESIGN.md §2.2 encoding). */
int  kb_sim_dump_row(kb_sim* sim, uint32_t node, uint8_t* row, size_t cap);
/* Per-node scalars, canonical layout: for each id: alive, n, last_bcast, start_round (4 x int32).  */
int  kb_sim_dump_scalars(kb_sim* sim, int32_t* out, size_t cap);
/* Canonical suspect table: sorted (peer, kind, since) triples for `node`; n = triples written.      */
int  kb_sim_dump_suspects(kb_sim* sim, uint32_t node, int32_t* out, size_t cap, size_t* n);
/* OR of the kernel-variant bits that did work since creation (PATH_* in kaboodle_amd/csrc/kb_common.h:
   1 broadcast phase on the HBM bitset (a round with a Failed list), 2/4 Join responses from HBM scratch (sampled / complete),
   8 KnownPeers BIG group on the HBM bitset, 16 k_proc unsorted selection path, 32 Failed-list prep
   from HBM, 64 Join responses by wave, 128 KnownPeers BIG group in LDS, 256 Join responses by wave
   from the rows in place).  Test surface.                                                          */
int  kb_sim_debug_paths(kb_sim* sim, uint32_t* mask);
/* Development counters since creation: [A3 rows scanned, rows scanned past their first 1024 ids,
   1024-id stamp chunks read] and, with cap >= 5, the row-shard exchange's bytes [sent to other shards,
   sent to every shard] (records and payload; summed over an in-process group's shards; 0 unsharded).
   Test surface.                                                                                     */
int  kb_sim_debug_counters(kb_sim* sim, uint64_t* out, size_t cap);
/* Canonical curious table: for each entry sorted by peer: peer, nobs, obs[0..3] (6 x int32).       */
int  kb_sim_dump_curious(kb_sim* sim, uint32_t node, int32_t* out, size_t cap, size_t* n);
/* KB_VARIANT_SPARSE_ROWS handles: the layout's footprint, out[0..5] = rows that adopted the base,
   exceptions, explicit stamps, entries of the largest row, bytes of the entries, rows (the oracle's
   kbo_sparse_footprint; here 4 bytes per entry, exception and stamp packed together).  Other handles:
   KB_INVALID_OPERATION.  Test surface.                                                             */
int  kb_sim_sparse_footprint(kb_sim* sim, uint64_t* out, size_t cap);

/* ---- pure helpers ------------------------------------------------------------------------------- */
/* Canonical simulated address of an id: "10.100.100.<100 + id/50000>:<10000 + id%50000>".          */
int  kb_format_addr(uint32_t id, char* buf, size_t cap);
/* generate_fingerprint over explicit (address, identity) pairs given as ids with a uniform identity
   table (identities[id*id_stride .. + id_lens[id]]); ids need not be sorted. */
uint32_t kb_fingerprint_of_set(const uint32_t* ids, size_t n, const uint8_t* identities,
                               size_t id_stride, const uint8_t* id_lens);

const char* kb_last_error(void);

/* ---- wire codec: the datagrams of a real Kaboodle instance ----------------
   bincode 1.3.3 (legacy `bincode::serialize` defaults) of src/structs.rs:65-116, so simulated nodes can be
   bridged to real ones: SwimEnvelope on the unicast socket (src/kaboodle.rs:188-226, :394-403),
   SwimBroadcast on the multicast socket (:256-311), ProbeResponse (:312-331, src/discovery.rs:30-89).
   Addresses are IPv4 (SocketAddr::V4).  Identities are (offset, length) views: into `idents` when
   encoding, into the datagram when decoding.  A datagram longer than 10240 B is truncated by the
   receiver (INCOMING_BUFFER_SIZE, src/kaboodle.rs:43) and then fails to decode: the simulator's
   oversize rule.                                                               */
enum { KB_WIRE_PING = 0, KB_WIRE_PING_REQUEST = 1, KB_WIRE_ACK = 2, KB_WIRE_KNOWN_PEERS = 3,
       KB_WIRE_KNOWN_PEERS_REQUEST = 4,              /* SwimMessage variants, in declaration order      */
       KB_WIRE_JOIN = 16, KB_WIRE_FAILED = 17, KB_WIRE_PROBE = 18,   /* SwimBroadcast variants           */
       KB_WIRE_PROBE_RESPONSE = 32 };
enum { KB_WIRE_CHANNEL_UNICAST = 0, KB_WIRE_CHANNEL_BROADCAST = 1, KB_WIRE_CHANNEL_PROBE_RESPONSE = 2 };
typedef struct kb_wire_entry { kb_wire_addr addr; uint32_t id_off, id_len; } kb_wire_entry;   /* KnownPeers */
typedef struct kb_wire_msg {
  uint32_t kind;                       /* KB_WIRE_*                                                     */
  uint32_t identity_off, identity_len; /* envelope / Join / ProbeResponse identity                      */
  kb_wire_addr peer;                   /* PingRequest(peer), Ack.peer, Join.addr, Failed, Probe         */
  uint32_t fingerprint, num_peers;     /* Ack, KnownPeersRequest                                        */
  uint32_t n_entries;                  /* KnownPeers                                                    */
} kb_wire_msg;
/* *size = the datagram's length; written to buf when cap suffices (buf = NULL: size query).          */
int kb_wire_encode(const kb_wire_msg* m, const kb_wire_entry* entries, const uint8_t* idents, uint8_t* buf,
                   size_t cap, size_t* size);
/* channel: KB_WIRE_CHANNEL_*.  Malformed or truncated -> KB_INVALID_ARGUMENT.  KnownPeers entries are
   stored up to cap (m->n_entries is always set; KB_CAPACITY when entries != NULL and cap is short).   */
int kb_wire_decode(const uint8_t* buf, size_t len, int channel, kb_wire_msg* m, kb_wire_entry* entries, size_t cap);
/* the simulator's canonical address of an id (kb_format_addr) and back (KB_INVALID_ARGUMENT: not one) */
int kb_wire_addr_of_id(uint32_t id, kb_wire_addr* out);
int kb_wire_id_of_addr(const kb_wire_addr* addr, uint32_t* id);

/* ---- timing surface for bench.py ---------------------------------------------------------------- */
/* HIP-event durations (ms, summed since last reset) of the round's kernels, recorded by the kernels'
   own dispatch packets on the stream they run on.  kind: KB_KT_*.                                   */
enum { KB_KT_ROWPASS = 0,   /* the row pass: broadcast phase + ping_random_peer candidates */
       KB_KT_ROUND = 1,     /* the whole round                                                           */
       KB_KT_FOLD = 2,      /* the fingerprint fold                                                      */
       KB_KT_RESP = 3,      /* the sampled Join responses, a wave per responder (k_resp_wave)            */
       KB_KT_PROC = 4 };    /* the in-order unicast handlers, a wave per node (k_proc, every wave)       */
int  kb_sim_kernel_time(kb_sim* sim, int kind, double* ms, uint64_t* launches);
int  kb_sim_reset_kernel_time(kb_sim* sim);
/* Algorithmic HBM bytes moved by a kernel (KB_KT_ROWPASS, KB_KT_FOLD, KB_KT_RESP or KB_KT_PROC) since the
   last reset, counted in-kernel.                                                      */
int  kb_sim_kernel_bytes(kb_sim* sim, int kind, uint64_t* bytes);
/* Per-kernel profile of the launches of the rounds since the last reset.  Profiling level (env KB_PROF
   or kb_sim_set_profiling): 0 = no per-launch events; 1 (default) = events on the once-per-round
   kernels with an in-kernel byte counter only (KB_KT_ROWPASS/FOLD/RESP); 2 = every launch, KB_KT_PROC's
   included (each event pair adds ≈5 us of dispatch overhead, ≈0.5 ms on a 100-launch round: use it on
   an untimed replay).  wave_ms[w]
   is the part spent in delivery wave w (slot KB_WAVE_SLOTS-1 holds waves >= KB_WAVE_SLOTS-1).  Kernels
   without events are omitted; cap = 0 queries the count.                                            */
#define KB_WAVE_SLOTS 9
typedef struct kb_kernel_time {
  char     name[24];
  double   ms;
  uint64_t launches;
  uint64_t bytes;                 /* algorithmic bytes counted in-kernel (has_bytes), else 0          */
  uint32_t has_bytes, pad;
  double   wave_ms[KB_WAVE_SLOTS];
} kb_kernel_time;
int  kb_sim_set_profiling(kb_sim* sim, int level);
int  kb_sim_kernel_breakdown(kb_sim* sim, kb_kernel_time* out, size_t cap, size_t* n);
/* Host waits on the device since creation (stream synchronisations and pinned hand-offs).          */
int  kb_sim_host_syncs(kb_sim* sim, uint64_t* n);

#ifdef __cplusplus
}
#endif
#endif /* KABOODLE_SIM_H */
