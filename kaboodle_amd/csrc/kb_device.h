// kb_device.h — device-side primitives of the MI355X Kaboodle round simulator (gfx950, wave64).
//
// Everything here is written for CDNA4 directly: 64-lane wavefronts, __ballot returns 64 bits,
// cross-lane traffic through __shfl* (ds_bpermute) and LDS.  Semantics constants follow
// src/kaboodle.rs:38-65 of the reference and DESIGN.md §2.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace kb {

// ---- protocol constants (src/kaboodle.rs:38-65), in rounds -------------------------------------
constexpr int PING_TIMEOUT = 2;     // :62
constexpr int SHARE_AGE = 10;       // :49
constexpr int REBROADCAST = 10;     // :65
constexpr int NUM_INDIRECT = 3;     // :52
constexpr int NUM_CANDIDATES = 5;   // :57
constexpr int BUFSZ = 10240;        // :43
// declared capacities
constexpr int SLOTS = 8;            // suspect slots per node
constexpr int CSLOTS = 8;           // curious_peers entries per node
constexpr int NOBS = 4;             // observers per curious entry
constexpr int PAQ = 8;              // queued ping_addrs per node
constexpr int MAXID = 32;           // identity bytes
constexpr int ADDR_LEN = 20;        // "10.100.100.ddd:ppppp"
constexpr int TICK_MAX = 3 * SLOTS + 1 + PAQ;   // unicast emissions of one tick
constexpr uint32_t LOGCAP = 2048;    // freshness log entries per node (power of two)
constexpr uint32_t LOG_INVALID = 0xFFFFFFFFu;
// stamp byte encoding
constexpr uint8_t ST_UNKNOWN = 0, ST_SUSPECT = 1, ST_ANCIENT = 2;
constexpr int EPOCH = 64, EOFF = 192;
// message kinds (SwimMessage, src/structs.rs:94-116)
enum : uint32_t { K_PING = 0, K_PINGREQ = 1, K_ACK = 2, K_KP = 3, K_KPR = 4 };
// sharded meshes only, never routed or handled as a message: one shard's union of the KnownPeers lists it delivers
// to one of the round's joiners in wave 0, as a bitmap (kb_waves.h, k_union_pack)
constexpr uint32_t K_KPU = 5;
// Philox purposes
enum : uint32_t { P_PING = 1, P_INDIRECT = 2, P_RESPOND = 3, P_TRUNC = 4, P_LOSS = 5, P_BLOSS = 6, P_CHURN = 7, P_PROBE = 8 };
enum : int32_t { SK_WFP = 1, SK_WFIP = 2 };
constexpr int32_t NONE_ROUND = INT32_MIN;
constexpr uint32_t CRC_POLY = 0xEDB88320u;

// error codes raised on the device (checked by the host after each step)
enum : uint32_t { DERR_NONE = 0, DERR_SLOTS = 1, DERR_OUTBOX = 2, DERR_PAYLOAD = 3, DERR_FLOYD = 4, DERR_INBOX = 5,
                  DERR_RESP = 6, DERR_LOG = 7, DERR_FP = 8 };

// ---- records ------------------------------------------------------------------------------------
struct Msg {            // 32 B unicast record
  uint32_t dest, sender, seq, kind;
  uint32_t a;           // PingRequest: peer; Ack: peer; KnownPeers: payload length
  uint32_t fp, n;       // Ack / KnownPeersRequest
  uint32_t off;         // KnownPeers: payload offset
};
struct Susp { uint32_t peer; int32_t since; int32_t kind; int32_t pad; };         // kind 0 = free
struct Cur { uint32_t peer; uint32_t nobs; uint32_t obs[NOBS]; uint32_t used; uint32_t pad; };  // 32 B
struct BCast { uint32_t sender, peer, bseq, pad; };
struct Tmpl { uint32_t raw; uint32_t mask_cnt; };   // 16-id block template: raw crc0, mask | cnt<<16

// ---- Philox4x32-10 (Salmon et al. SC'11), counter = (c0,c1,c2,c3), key = seed -------------------
struct U4 { uint32_t x, y, z, w; };
__host__ __device__ inline U4 philox(uint32_t c0, uint32_t c1, uint32_t c2, uint32_t c3, uint32_t k0, uint32_t k1) {
#pragma unroll
  for (int r = 0; r < 10; ++r) {
    if (r) { k0 += 0x9E3779B9u; k1 += 0xBB67AE85u; }
    const uint64_t p0 = (uint64_t)0xD2511F53u * c0;
    const uint64_t p1 = (uint64_t)0xCD9E8D57u * c2;
    const uint32_t n0 = (uint32_t)(p1 >> 32) ^ c1 ^ k0;
    const uint32_t n2 = (uint32_t)(p0 >> 32) ^ c3 ^ k1;
    c1 = (uint32_t)p1; c3 = (uint32_t)p0; c0 = n0; c2 = n2;
  }
  return U4{c0, c1, c2, c3};
}
__host__ __device__ inline uint32_t mulhi(uint32_t u, uint32_t k) { return (uint32_t)(((uint64_t)u * k) >> 32); }

// ---- GF(2) arithmetic mod the CRC-32 polynomial, reflected (x^0 = 0x80000000) ---------------------
__host__ __device__ inline uint32_t multmodp(uint32_t a, uint32_t b) {
  uint32_t p = 0;
#if defined(__HIP_DEVICE_COMPILE__)
  // device: the bit masks by signed bit-field extracts (0 or all ones), no compare/select per bit
#pragma unroll 4
  for (int k = 31; k >= 0; --k) {
    p ^= b & (uint32_t)__builtin_amdgcn_sbfe((int)a, k, 1);
    b = (b >> 1) ^ (CRC_POLY & (uint32_t)__builtin_amdgcn_sbfe((int)b, 0, 1));
  }
#else
#pragma unroll 4
  for (int k = 31; k >= 0; --k) {
    if (a & (1u << k)) p ^= b;
    b = (b & 1u) ? (b >> 1) ^ CRC_POLY : b >> 1;
  }
#endif
  return p;
}

// ---- stamp window --------------------------------------------------------------------------------
__host__ __device__ inline int32_t epoch_base(int32_t r) { return (r / EPOCH) * EPOCH; }
__host__ __device__ inline uint8_t enc(int32_t t, int32_t r) {
  int32_t v = t - epoch_base(r) + EOFF;
  v = v < ST_ANCIENT ? ST_ANCIENT : (v > 255 ? 255 : v);
  return (uint8_t)v;
}

// ---- wave helpers (wave64) ---------------------------------------------------------------------
__device__ inline uint32_t lane() { return __lane_id(); }
// Cross-lane scans and reductions by DPP (VALU data movement inside and across the four 16-lane rows): no
// LDS instruction and no LDS round trip per step, which the ds_bpermute forms (__shfl_*) cost — each of their
// six steps waited on the LDS pipe.  Precondition: EXEC is the full wave or a prefix of it (lanes 0..k-1) —
// every call site is wave-convergent.  Inactive lanes then sit after every active one and contribute the
// operation's identity; a gap in EXEC would NOT: DPP treats a disabled source lane as invalid, so a shift that
// reads across the gap drops the partial sums below it.  The reductions return the value of the last active
// lane's inclusive scan, broadcast (wave-uniform).
template <uint32_t ID, typename Op>
__device__ __attribute__((always_inline)) inline uint32_t wave_iscan(uint32_t x, Op op) {
  x = op(x, (uint32_t)__builtin_amdgcn_update_dpp((int)ID, (int)x, 0x111, 0xF, 0xF, false));   // row_shr:1
  x = op(x, (uint32_t)__builtin_amdgcn_update_dpp((int)ID, (int)x, 0x112, 0xF, 0xF, false));   // row_shr:2
  x = op(x, (uint32_t)__builtin_amdgcn_update_dpp((int)ID, (int)x, 0x114, 0xF, 0xF, false));   // row_shr:4
  x = op(x, (uint32_t)__builtin_amdgcn_update_dpp((int)ID, (int)x, 0x118, 0xF, 0xF, false));   // row_shr:8
  x = op(x, (uint32_t)__builtin_amdgcn_update_dpp((int)ID, (int)x, 0x142, 0xA, 0xF, false));   // row_bcast:15
  x = op(x, (uint32_t)__builtin_amdgcn_update_dpp((int)ID, (int)x, 0x143, 0xC, 0xF, false));   // row_bcast:31
  return x;
}
__device__ __attribute__((always_inline)) inline uint32_t wave_last(uint32_t x) {
  const unsigned long long ex = __builtin_amdgcn_read_exec();
  return (uint32_t)__builtin_amdgcn_readlane((int)x, 63 - __builtin_clzll(ex));
}
struct OpAdd { __device__ uint32_t operator()(uint32_t a, uint32_t b) const { return a + b; } };
struct OpMin { __device__ uint32_t operator()(uint32_t a, uint32_t b) const { return a < b ? a : b; } };
struct OpMax { __device__ uint32_t operator()(uint32_t a, uint32_t b) const { return a > b ? a : b; } };
struct OpOr { __device__ uint32_t operator()(uint32_t a, uint32_t b) const { return a | b; } };
__device__ inline uint32_t wave_sum(uint32_t v) { return wave_last(wave_iscan<0u>(v, OpAdd{})); }
__device__ inline uint32_t wave_min(uint32_t v) { return wave_last(wave_iscan<0xFFFFFFFFu>(v, OpMin{})); }
__device__ inline uint32_t wave_max(uint32_t v) { return wave_last(wave_iscan<0u>(v, OpMax{})); }
__device__ inline uint32_t wave_or(uint32_t v) { return wave_last(wave_iscan<0u>(v, OpOr{})); }
// lane l + ST's value inside l's 16-lane row, 0 past the row's end (DPP row_shl)
template <uint32_t ST> __device__ __attribute__((always_inline)) inline uint32_t dpp_shl(uint32_t x) {
  return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x100 + ST, 0xF, 0xF, false);
}
// lane (l ^ J)'s value: DPP for partners inside a 16-lane row (J <= 8), an LDS permute across rows
template <uint32_t J> __device__ __attribute__((always_inline)) inline uint32_t shfl_xor_c(uint32_t x) {
  if constexpr (J == 1) return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0xB1, 0xF, 0xF, false);   // quad_perm 1,0,3,2
  else if constexpr (J == 2) return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x4E, 0xF, 0xF, false);   // quad_perm 2,3,0,1
  else if constexpr (J == 4 || J == 8) {
    const uint32_t up = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x100 + J, 0xF, 0xF, false);   // row_shl:J
    const uint32_t dn = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x110 + J, 0xF, 0xF, false);   // row_shr:J
    return (lane() & J) ? dn : up;
  } else return __shfl_xor(x, (int)J, 64);
}
// exclusive prefix sum across the 64 lanes
__device__ inline uint32_t wave_excl(uint32_t v) { return wave_iscan<0u>(v, OpAdd{}) - v; }
// s_waitcnt lgkmcnt(0) only (gfx9 encoding: vmcnt 63, expcnt 7): LDS/SMEM done, memory ops may fly
__device__ inline void wait_lds() { __builtin_amdgcn_s_waitcnt(0xC07F); }
__device__ inline uint32_t bcast(uint32_t v, int src) { return __shfl(v, src, 64); }   // src may differ per lane
// lane src's value when src is the same in every lane (a loop index, a ballot's first bit): v_readlane into
// a scalar register instead of an LDS permute round trip
__device__ inline uint32_t rdl(uint32_t v, int src) { return (uint32_t)__builtin_amdgcn_readlane((int)v, src); }
// Make this wave's earlier global stores visible to its own later loads (same CU; workgroup scope).
__device__ inline void wave_mem_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
}

}  // namespace kb
