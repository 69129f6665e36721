"""Where the quiet tail stops healing (dev tool): configs[2]-shaped mesh, F faulty rounds, then quiet
rounds; every `every` rounds, for 200 live nodes: entries for dead peers (count, peer_states state,
distance (peer - node) mod C in 8 bins), live peers missing.

    python tools/tail_probe.py N sim|sock TAIL_ROUNDS [EVERY] [gpu|oracle]
"""
import collections
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests"))
from kaboodle_amd._ffi import KB_FAILED_SIM_SENDER, KB_FAILED_SOCKET_FAITHFUL, KB_INIT_CONVERGED, Sim, SimConfig  # noqa: E402

n, mode, tail = int(sys.argv[1]), sys.argv[2], int(sys.argv[3])
every = int(sys.argv[4]) if len(sys.argv) > 4 else 2000
impl = sys.argv[5] if len(sys.argv) > 5 else "gpu"
F = 25
cfg = SimConfig(capacity=n + max(4096 if n >= 65536 else 512, int(n * 0.001 * (F + 8) * 1.5)), initial_nodes=n,
                init_mode=KB_INIT_CONVERGED, loss=0.01, churn=0.001 if n >= 4096 else 0.004, fault_end_round=F, seed=1,
                failed_mode=KB_FAILED_SOCKET_FAITHFUL if mode == "sock" else KB_FAILED_SIM_SENDER)
import parity  # noqa: E402
lib = parity.gpu_lib() if impl == "gpu" else parity.oracle_lib(omp=True)
t0 = time.time()
with Sim(lib, cfg) as o:
    o.step(F)
    done = 0
    while done < tail:
        o.step(every)
        done += every
        st = o.stats()
        alive = [i for i in range(cfg.capacity) if o.is_running(i)]
        aset = set(alive)
        states, dist = collections.Counter(), collections.Counter()
        extra = missing = 0
        for i in alive[:: max(1, len(alive) // 200)][:200]:
            ps = o.peer_states(i)
            ids = set()
            for p, s, since, lat in ps:
                ids.add(p)
                if p not in aset:
                    extra += 1
                    states[(s, "ancient" if since == -2 ** 31 else "recent")] += 1
                    dist[((p - i) % cfg.capacity) * 8 // cfg.capacity] += 1
            missing += len(aset - ids)
        print(f"round {F + done}: agree {st['agree']}/{st['alive']}  dead entries/200 nodes {extra} {dict(states)}  "
              f"by distance octile {[dist[k] for k in range(8)]}  missing live {missing}  {time.time() - t0:.0f} s",
              flush=True)
