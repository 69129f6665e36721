"""Exchange volume and time of a row-sharded mesh (dev tool, GPU): python tools/xvol.py N SHARDS ROUNDS [lists]

configs[2]'s workload (converged start, 1 % loss, 0.1 %/round churn, faults until round 25, latency on, exact A3)
as SHARDS in-process row shards (kb_sim_create_local): per round the wall time and the bytes the shards' waves sent
to other shards and in all (kb_sim_debug_counters), after 5 warmup rounds.  `lists` turns the Join-response union
off (KB_DBG_NO_UNION): every response's ids cross as a list."""
import ctypes as C, sys, time, os
sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", "/root/repo"))
import kaboodle_amd
from kaboodle_amd._ffi import SimConfig, KB_DBG_NO_UNION, KB_INIT_CONVERGED, KB_VARIANT_EXACT_LRU
n, shards, rounds = int(sys.argv[1]), int(sys.argv[2]), int(sys.argv[3])
cfg = SimConfig(capacity=n + 8192, initial_nodes=n, init_mode=KB_INIT_CONVERGED, loss=0.01, churn=0.001, seed=1,
                track_latency=1, variant=KB_VARIANT_EXACT_LRU, fault_end_round=25,
                debug_flags=KB_DBG_NO_UNION if "lists" in sys.argv[4:] else 0)
lib = kaboodle_amd.lib()
m = kaboodle_amd.Mesh(cfg, shards=shards) if shards else kaboodle_amd.Mesh(cfg)
m.step(5)
buf = (C.c_uint64 * 5)()
ok = lib.lib.kb_sim_debug_counters(m.h, buf, 5) == 0
b0 = (buf[3], buf[4]) if ok else (0, 0)
t = time.time(); m.step(rounds); dt = time.time() - t
ok = lib.lib.kb_sim_debug_counters(m.h, buf, 5) == 0
b1 = (buf[3], buf[4]) if ok else (0, 0)
st = m.stats()
print(f"N={n} shards={shards} {'lists' if 'lists' in sys.argv[4:] else 'unions'} ms/round {dt / rounds * 1e3:.2f}  cross MB/round {(b1[0] - b0[0]) / rounds / 1e6:.2f}  all MB/round {(b1[1] - b0[1]) / rounds / 1e6:.2f}  joins {st['churn_joins']}  kp_ids {st['sent_kp_ids']}", flush=True)
