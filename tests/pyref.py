"""pyref.py — a second, independent restatement of "round semantics v1" (TEST INFRASTRUCTURE ONLY).

Written the way the reference is written, not the way the oracle or the GPU are: every peer owns a
`known_peers` dict {addr-id: (state, instant)} like `ObservableHashMap<Peer, PeerInfo>`
(src/structs.rs:12-41), the fingerprint is the literal CRC-32 of the sorted address strings and
identities computed by zlib (src/kaboodle.rs:71-83), and instants are exact round numbers.  The dense
stamp-byte window of DESIGN.md §2.2 appears only where the semantics define it (the ordering key of
ping_random_peer).  Pure-Python loops: for small meshes only.

It pins the C oracle (tests/test_oracle_traces.py replays its committed traces) and generates the committed round-trace fixtures
(tests/golden/make_golden.py).
"""
from __future__ import annotations

import zlib

MASK = 0xFFFFFFFF
PING_TIMEOUT, SHARE_AGE, REBROADCAST, NUM_INDIRECT, NUM_CANDIDATES, BUFSZ = 2, 10, 10, 3, 5, 10240
CSLOTS, NOBS, PAQ = 8, 4, 8
P_PING, P_INDIRECT, P_RESPOND, P_TRUNC, P_LOSS, P_BLOSS, P_CHURN = 1, 2, 3, 4, 5, 6, 7
KNOWN, WFP, WFIP = "Known", "WaitingForPing", "WaitingForIndirectPing"


def philox(c0, c1, c2, c3, k0, k1):
    for r in range(10):
        if r:
            k0 = (k0 + 0x9E3779B9) & MASK
            k1 = (k1 + 0xBB67AE85) & MASK
        p0 = 0xD2511F53 * c0
        p1 = 0xCD9E8D57 * c2
        c0, c1, c2, c3 = ((p1 >> 32) ^ c1 ^ k0) & MASK, p1 & MASK, ((p0 >> 32) ^ c3 ^ k1) & MASK, p0 & MASK
    return c0, c1, c2, c3


def mulhi(u, k):
    return (u * k) >> 32


def mix32(x):
    x ^= x >> 16
    x = (x * 0x7FEB352D) & MASK
    x ^= x >> 15
    x = (x * 0x846CA68B) & MASK
    x ^= x >> 16
    return x


def prp_walk(x, n, key):
    """x-th image of the keyed permutation of [0, n): a 4-round Feistel network on b = max(2, ceil(log2 n))
    bits, halves of ceil(b/2) (high) and floor(b/2) (low) bits whose widths swap every round, round
    function lowbias32(R ^ key[k]) masked to the width of the half it is XORed into, cycle walking."""
    b = 2
    while (1 << b) < n:
        b += 1
    c = b // 2
    a = b - c
    while True:
        L, R, wl = x >> c, x & ((1 << c) - 1), a
        for k in range(4):
            L, R = R, L ^ (mix32(R ^ key[k]) & ((1 << wl) - 1))
            wl = b - wl
        x = (L << c) | R
        if x < n:
            return x


def addr(i: int) -> str:
    return f"10.100.100.{100 + i // 50000}:{10000 + i % 50000}"


def default_identity(i: int, n: int) -> bytes:
    return bytes(ord("a") + ((i * 31 + k * 7) % 26) for k in range(n))


def fingerprint(ids, identity) -> int:
    """generate_fingerprint (src/kaboodle.rs:71-83), literally, over ids with one identity table."""
    h = 0
    for p in sorted(ids):
        h = zlib.crc32(addr(p).encode(), h)
        h = zlib.crc32(identity[p], h)
    return h


def view_fingerprint(known) -> int:
    """generate_fingerprint of one peer's map: every entry's address and the identity THIS view holds for
    it (PeerInfo.identity, src/kaboodle.rs:77-79)."""
    h = 0
    for p in sorted(known):
        h = zlib.crc32(addr(p).encode(), h)
        h = zlib.crc32(known[p][2], h)
    return h


def epoch_base(r):
    return (r // 64) * 64


def stamp_key(t, r):
    """the declared stamp window: instants older than the window compare equal ("ancient")"""
    return max(2, min(255, t - epoch_base(r) + 192))


class Peer:
    def __init__(self, i):
        self.id = i
        self.running = False
        self.ever = False
        self.start_round = None
        self.known = {}          # peer -> [state, instant, identity]: PeerInfo (src/structs.rs:18-22)
        self.latency = {}        # peer -> PeerInfo.latency in ms (absent = None)
        self.a3cur = i           # A3's rotation base: just before the last round's oldest candidate (§2.6)
        self.curious = {}        # peer -> [observers]
        self.last_bcast = None
        self.paq = []


class PyMesh:
    def __init__(self, capacity, initial_nodes, converged=False, seed=1, loss=0.0, churn=0.0, fault_end=-1,
                 max_waves=8, failed_honoured=True, id_len=0, partition=None):
        self.C = capacity
        self.k0, self.k1 = seed & MASK, (seed >> 32) & MASK
        self.loss_thr = min(int(round(loss * 2 ** 32)), MASK)
        self.churn_thr = min(int(round(churn * 2 ** 32)), MASK)
        self.fault_end, self.max_waves, self.failed_honoured = fault_end, max_waves, failed_honoured
        self.partition = partition      # (groups, start, end) or None
        self.id_len = id_len
        self.identity = [default_identity(i, id_len) for i in range(capacity)]   # what each address announces
        self.pending = {}        # identity set on a stopped instance, taken by its next address
        self.idset = set()       # never-bound addresses given an identity (not fresh)
        self.peers = [Peer(i) for i in range(capacity)]
        self.round = 0
        self.next_free = initial_nodes
        self.events = []
        self.bfail, self.bjoin = [], []
        self.stats = dict(sent_ping=0, sent_ping_req=0, sent_ack=0, sent_known_peers=0, sent_kpr=0, bcast_join=0,
                          bcast_failed=0, drop_dead=0, drop_loss=0, drop_window=0, drop_oversize=0, drop_partition=0,
                          drop_bcast=0, removed_timeout=0, removed_failed=0, join_responses=0, curious_overflow=0,
                          churn_leaves=0, churn_joins=0)
        self.agree = 0
        self.first_converged = -1
        for i in range(initial_nodes):
            self._start(i, 0)
            if converged:
                p = self.peers[i]
                for j in range(initial_nodes):
                    if j != i:
                        p.known[j] = [KNOWN, -(10 ** 6), self.identity[j]]   # long before the stamp window
                p.last_bcast = -1000

    # ---------------------------------------------------------------- helpers
    def ph(self, *c):
        return philox(*c, self.k0, self.k1)

    def faults(self, r):
        return self.fault_end < 0 or r < self.fault_end

    def blocked(self, r, a, b):
        if not self.partition:
            return False
        g, s, e = self.partition
        if g <= 1 or not (s <= r < e):
            return False
        return a * g // self.C != b * g // self.C

    def _start(self, i, r):
        p = self.peers[i]
        p.running, p.ever, p.start_round = True, True, r
        if i not in p.known:
            p.latency.pop(i, None)
        p.known[i] = [KNOWN, r, self.identity[i]]
        p.a3cur = i
        p.last_bcast = None
        p.curious = {}
        p.paq = []

    def _stop(self, i):
        p = self.peers[i]
        p.known.pop(i, None)
        p.running = False
        p.paq = []

    def _api_running(self, i):
        for ev in reversed(self.events):
            if ev[1] == i:
                return ev[0] != "stop"
            if ev[0] == "restart" and ev[2] == i:
                return False
        return self.peers[i].running

    def _ever(self, i):
        return self.peers[i].ever or any(ev[1] == i and ev[0] != "stop" for ev in self.events)

    def _fresh(self, i):
        """an address no instance has bound and no identity was set on: what churn joins and restarts take"""
        return not self._ever(i) and i not in self.idset

    def set_identity(self, i, ident: bytes):
        """Kaboodle::set_identity (src/lib.rs:323-336) on a stopped instance: the identity it will announce
        from its next start on (a never-bound address takes it at once)."""
        assert not self._api_running(i)
        if self._ever(i):
            self.pending[i] = ident
        else:
            self.identity[i] = ident
            self.idset.add(i)

    def start_node(self, i):
        assert self._api_running(i) or not self._ever(i)
        self.events.append(("start", i, i))

    def stop_node(self, i):
        self.events.append(("stop", i, i))

    def restart_node(self, i):
        """Kaboodle::start of the instance at address i: a stopped instance binds a fresh ephemeral socket
        (src/kaboodle.rs:138-152) and keeps its known_peers map (src/lib.rs:104, 167-170)."""
        if self._api_running(i):
            return i
        if not self._ever(i):
            self.events.append(("start", i, i))
            return i
        new = self.next_free
        while new < self.C and not self._fresh(new):
            new += 1
        assert new < self.C, "no fresh address left"
        self.next_free = new + 1
        self.identity[new] = self.pending.pop(i, self.identity[i])
        self.events.append(("restart", new, i))
        return new

    def ping_addrs(self, i, addrs):
        p = self.peers[i]
        for a in addrs:
            if a not in p.known:
                p.paq.append(a)

    def kp_size(self, sender, ids):
        return 8 + len(self.identity[sender]) + 4 + 8 + sum(10 + 8 + len(self.identity[j]) for j in ids)

    # ---------------------------------------------------------------- round
    def step(self):
        r = self.round
        self.out = {}
        for kind, i, src in self.events:
            if kind == "stop" and self.peers[i].running:
                self._stop(i)
            elif kind == "start" and not self.peers[i].running:
                self._start(i, r)
            elif kind == "restart":                       # the map moves with the instance
                old, new = self.peers[src], self.peers[i]
                new.known = {q: list(v) for q, v in old.known.items()}
                new.latency = dict(old.latency)
                self._start(i, r)
        self.events = []
        if self.faults(r) and self.churn_thr:
            leaves = [i for i in range(self.C) if self.peers[i].running and self.peers[i].start_round != r
                      and self.ph(i, r, P_CHURN << 24, 0)[0] < self.churn_thr]
            for i in leaves:
                self._stop(i)
            self.stats["churn_leaves"] += len(leaves)
            for _ in leaves:
                while self.next_free < self.C and not self._fresh(self.next_free):
                    self.next_free += 1
                if self.next_free < self.C:
                    self._start(self.next_free, r)
                    self.next_free += 1
                    self.stats["churn_joins"] += 1
        for i in range(self.C):
            p = self.peers[i]
            if p.running and p.start_round < r:
                self.broadcasts(p, r)
        live = [i for i in range(self.C) if self.peers[i].running]
        true_fp = fingerprint(live, self.identity)
        bjoin, bfail = [], []
        agree = 0
        for i in live:
            j, f = self.tick(self.peers[i], r)
            bseq = 0
            if j:
                bjoin.append((i, i, bseq, self.identity[i]))    # Join{addr, identity} (:228-251)
                bseq += 1
            for q in f:
                bfail.append((i, q, bseq, None))
                bseq += 1
            agree += view_fingerprint(self.peers[i].known) == true_fp
        self.bjoin, self.bfail = bjoin, bfail
        self.stats["bcast_join"] += len(bjoin)
        self.stats["bcast_failed"] += len(bfail)
        self.waves(r)
        self.agree = agree
        if live and agree == len(live) and self.first_converged < 0:
            self.first_converged = r
        self.round += 1

    def emit(self, sender, dest, kind, **kw):
        box = self.out.setdefault(sender, [])
        box.append(dict(dest=dest, sender=sender, seq=len(box), kind=kind, **kw))

    # handle_incoming_broadcasts (src/kaboodle.rs:256-311)
    def broadcasts(self, p, r):
        for e, (s, peer, bseq, _) in enumerate(self.bfail):
            if s == p.id:
                continue
            if self.lost_b(p.id, s, 0, e, r):
                continue
            if peer == p.id:
                continue
            if self.failed_honoured and s in p.known and peer in p.known:
                del p.known[peer]
                self.stats["removed_failed"] += 1
        for e, (a, _, bseq, ident) in enumerate(self.bjoin):
            if a == p.id or self.lost_b(p.id, a, 1, e, r):
                continue
            is_new = a not in p.known
            if is_new:
                p.latency.pop(a, None)                    # :294-296 keeps an existing entry's latency
            p.known[a] = [KNOWN, r, ident]                # Join{addr, identity} (:284-298)
            if is_new and self.should_respond(p, a, r):
                self.send_known_peers_to(p, a, r)

    def lost_b(self, recv, sender, lst, e, r):
        """delivery of entry e of the round's Failed (lst 0) / Join (lst 1) list to recv: word e % 4 of
        philox(recv, r, P_BLOSS << 24 | lst << 23 | e // 4, 0)"""
        if self.blocked(r, sender, recv):
            self.stats["drop_bcast"] += 1
            return True
        if self.faults(r) and self.loss_thr and \
                self.ph(recv, r, (P_BLOSS << 24) | (lst << 23) | (e >> 2), 0)[e & 3] < self.loss_thr:
            self.stats["drop_bcast"] += 1
            return True
        return False

    def should_respond(self, p, joiner, r):              # src/kaboodle.rs:333-354
        o = len(p.known) - 2
        if o <= 0:
            return True
        pct = max(1, 100 - o * o)
        return mulhi(self.ph(p.id, r, P_RESPOND << 24, joiner)[0], 100) < pct

    def send_known_peers_to(self, p, joiner, r):         # src/kaboodle.rs:356-392
        members = sorted(p.known)
        L = self.id_len
        cap = (BUFSZ - 20 - L - 1) // (18 + L)
        if len(members) > cap:
            n = len(members)
            key = self.ph(p.id, r, P_TRUNC << 24, joiner)
            chosen = {prp_walk(t, n, key) for t in range(cap)}
            members = [members[k] for k in sorted(chosen)]
        self.emit(p.id, joiner, "KnownPeers", peers=[(q, p.known[q][2]) for q in members])
        self.stats["join_responses"] += 1

    # tick (src/kaboodle.rs:746-779)
    def tick(self, p, r):
        join = False
        if p.last_bcast is None or (r - p.last_bcast >= REBROADCAST and len(p.known) <= 1):   # :228-251
            join = True
            p.last_bcast = r
        # handle_suspected_peers :558-653
        cands = sorted(q for q, (st, _, _) in p.known.items() if st == KNOWN and q != p.id)
        removed, indirect = [], []
        for q in sorted(p.known):
            st, t, _ = p.known[q]
            if st == KNOWN or r - t < PING_TIMEOUT:
                continue
            if st == WFP:
                m = len(cands)
                k = min(NUM_INDIRECT, m)
                if k == 0:
                    removed.append(q)
                    continue
                x, y, z, _ = self.ph(p.id, r, P_INDIRECT << 24, q)
                picks = [mulhi(x, m)]
                if k > 1:
                    b = mulhi(y, m - 1)
                    picks.append(b + (b >= picks[0]))
                if k > 2:
                    lo, hi = sorted(picks)
                    c = mulhi(z, m - 2)
                    c += c >= lo
                    c += c >= hi
                    picks.append(c)
                for pk in picks:
                    self.emit(p.id, cands[pk], "PingRequest", peer=q)
                indirect.append(q)
            else:
                removed.append(q)
        for q in indirect:
            p.known[q] = [WFIP, r, p.known[q][2]]
        fails = []
        for q in removed:
            del p.known[q]
            p.curious.pop(q, None)
            fails.append(q)
            self.stats["removed_timeout"] += 1
        # ping_random_peer :655-703
        c = [q for q, (st, _, _) in p.known.items() if st == KNOWN and q != p.id]
        c.sort(key=lambda q: (stamp_key(p.known[q][1], r), (q - p.a3cur - 1) % self.C))
        c = c[:NUM_CANDIDATES]
        if c:
            t = c[mulhi(self.ph(p.id, r, P_PING << 24, 0)[0], len(c))]
            p.a3cur = (c[0] - 1) % self.C           # the sweep front: just before the oldest candidate
            p.known[t] = [WFP, r, p.known[t][2]]
            self.emit(p.id, t, "Ping")
        for a in p.paq:                                   # :550-556
            self.emit(p.id, a, "Ping")
        p.paq = []
        return join, fails

    def count_sent(self, msgs):
        key = {"Ping": "sent_ping", "PingRequest": "sent_ping_req", "Ack": "sent_ack", "KnownPeers": "sent_known_peers",
               "KnownPeersRequest": "sent_kpr"}
        for m in msgs:
            self.stats[key[m["kind"]]] += 1

    def waves(self, r):
        for w in range(self.max_waves):
            msgs = [m for s in sorted(self.out) for m in self.out[s]]
            self.out = {}
            if not msgs:
                return
            self.count_sent(msgs)
            inbox = {}
            for m in msgs:
                d = m["dest"]
                if not self.peers[d].running:
                    self.stats["drop_dead"] += 1
                    continue
                if self.blocked(r, m["sender"], d):
                    self.stats["drop_partition"] += 1
                    continue
                if self.faults(r) and self.loss_thr and \
                        self.ph(m["sender"], r, (P_LOSS << 24) | w, m["seq"])[0] < self.loss_thr:
                    self.stats["drop_loss"] += 1
                    continue
                inbox.setdefault(d, []).append(m)
            for d in sorted(inbox):
                box = inbox[d]
                for m in [m for m in box if m["kind"] == "KnownPeers"] + [m for m in box if m["kind"] != "KnownPeers"]:
                    self.handle(self.peers[d], m, r, w)
        left = [m for s in sorted(self.out) for m in self.out[s]]
        self.count_sent(left)
        self.stats["drop_window"] += len(left)
        self.out = {}

    # handle_incoming_messages (src/kaboodle.rs:394-548)
    def handle(self, p, m, r, w=0):
        s = m["sender"]
        self.observe_latency(p, s, r, w)
        p.known[s] = [KNOWN, r, self.identity[s]]                 # :406-415: the envelope's identity
        kind = m["kind"]
        if kind == "Ack":                                         # :418-447
            peer = m["peer"]
            obs = p.curious.pop(peer, None)
            if obs:
                for o in obs:
                    self.emit(p.id, o, "Ack", peer=peer, fp=m["fp"], n=m["n"])
            self.maybe_sync(p, peer, m["fp"], m["n"])
        elif kind == "KnownPeers":                                # :448-472
            for q, ident in m["peers"]:
                if q not in p.known:
                    p.latency.pop(q, None)                        # latency: None (:467)
                    p.known[q] = [KNOWN, r - SHARE_AGE, ident]    # the listed PeerInfo's identity (:461-468)
        elif kind == "KnownPeersRequest":                         # :473-512
            lst = sorted(q for q, (st, t, _) in p.known.items()
                         if st == KNOWN and q != p.id and q != s and r - t < SHARE_AGE)
            if self.kp_size(p.id, lst) > BUFSZ:
                self.stats["drop_oversize"] += 1
            else:
                self.emit(p.id, s, "KnownPeers", peers=[(q, p.known[q][2]) for q in lst])
            self.maybe_sync(p, s, m["fp"], m["n"])
        elif kind == "Ping":                                      # :513-532
            self.emit(p.id, s, "Ack", peer=p.id, fp=view_fingerprint(p.known), n=len(p.known))
        elif kind == "PingRequest":                               # :533-545
            peer = m["peer"]
            if peer in p.curious:
                obs = p.curious[peer]
                if s not in obs:
                    if len(obs) == NOBS:
                        self.stats["curious_overflow"] += 1
                    else:
                        obs.append(s)
            elif len(p.curious) == CSLOTS:
                self.stats["curious_overflow"] += 1
            else:
                p.curious[peer] = [s]
            self.emit(p.id, peer, "Ping")

    @staticmethod
    def observe_latency(p, s, r, w):
        """calculate_peer_latency (src/kaboodle.rs:789-817) on the envelope prologue (:408-413), simulated
        clock: the tick of round t is at 1000·t ms, wave w delivers at 1000·r + w + 1."""
        old = p.known.get(s)
        if old is None:
            p.latency.pop(s, None)
            return
        st, t, _ = old
        if st == KNOWN:
            return
        sample = 1000 * (r - t) + w + 1
        prev = p.latency.get(s)
        p.latency[s] = sample if prev is None else int((sample * 0.8) + (prev * (1.0 - 0.8)))

    def maybe_sync(self, p, peer, their_fp, their_n):           # :707-740
        f = view_fingerprint(p.known)
        if f == their_fp or len(p.known) > their_n:
            return
        self.emit(p.id, peer, "KnownPeersRequest", fp=f, n=len(p.known))

    # ---------------------------------------------------------------- views
    def row(self, i):
        """the dense stamp-byte view of peer i's map, for comparison with the oracle"""
        out = [0] * self.C
        for q, (st, t, _) in self.peers[i].known.items():
            out[q] = 1 if st != KNOWN else stamp_key(t, max(self.round - 1, 0))
        return out

    def peer_states(self, i):
        """Kaboodle::peer_states (src/lib.rs:348-354) as the ABI reports it: (peer, state, since,
        latency, identity); since = the exact instant, or INT32_MIN once the stamp window has saturated
        it; latency in ms, 0xFFFFFFFF = None."""
        rl = max(self.round - 1, 0)
        out = []
        p = self.peers[i]
        for q, (st, t, ident) in sorted(p.known.items()):
            lat = p.latency.get(q, 0xFFFFFFFF)
            if st == KNOWN:
                out.append((q, 0, t if stamp_key(t, rl) > 2 else -2 ** 31, lat, ident))
            else:
                out.append((q, 1 if st == WFP else 2, t, lat, ident))
        return out

    def suspects(self, i):
        return sorted((q, 1 if st == WFP else 2, t) for q, (st, t, _) in self.peers[i].known.items() if st != KNOWN)

    def curious_view(self, i):
        return sorted((q, len(o), *(list(o) + [-1] * (NOBS - len(o)))) for q, o in self.peers[i].curious.items())
