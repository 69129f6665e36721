"""First round where the GPU and the OpenMP oracle diverge on a long run (dev tool).

    python tools/find_divergence.py N sim|sock ROUNDS [CHECK_EVERY]

configs[2]-shaped workload at N peers (faults until round 25, then quiet).  Every CHECK_EVERY rounds the
fingerprints, scalars and counters are compared; on a mismatch the run restarts and steps one round at
a time over the last interval, then prints the first differing nodes and their row differences.
"""
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests"))
from kaboodle_amd._ffi import KB_FAILED_SIM_SENDER, KB_FAILED_SOCKET_FAITHFUL, KB_INIT_CONVERGED, Sim, SimConfig  # noqa: E402
import parity  # noqa: E402

n, mode, rounds = int(sys.argv[1]), sys.argv[2], int(sys.argv[3])
every = int(sys.argv[4]) if len(sys.argv) > 4 else 50
with_rows = len(sys.argv) > 5 and sys.argv[5] == "rows"      # compare every stamp row too (stamps are latent)
F = 25
cfg = SimConfig(capacity=n + max(512, int(n * 0.001 * (F + 8) * 1.5)), initial_nodes=n, init_mode=KB_INIT_CONVERGED,
                loss=0.01, churn=0.001 if n >= 4096 else 0.004, fault_end_round=F, seed=1,
                failed_mode=KB_FAILED_SOCKET_FAITHFUL if mode == "sock" else KB_FAILED_SIM_SENDER)


def digest(s):
    st = s.stats()
    d = (s.fingerprints().tobytes(), s.scalars().tobytes(), tuple(sorted(st.items())))
    return d + ((s.rows().tobytes(),) if with_rows else ())


def run(upto_ok, upto_bad):
    o, g = Sim(parity.oracle_lib(omp=True), cfg), Sim(parity.gpu_lib(), cfg)
    o.step(upto_ok); g.step(upto_ok)
    r = upto_ok
    while r < upto_bad:
        o.step(1); g.step(1); r += 1
        if digest(o) != digest(g):
            fo, fg = o.fingerprints(), g.fingerprints()
            bad = np.nonzero(fo != fg)[0][:5]
            if with_rows:
                ro, rg = o.rows(), g.rows()
                br = np.unique(np.nonzero(ro != rg)[0])
                print(f"rows differ after round {r - 1}: {len(br)} nodes, first {br[:8]}; scalars o {o.scalars()[br[:3]]} g {g.scalars()[br[:3]]}")
                bad = br[:5]
            print(f"first divergence after round {r - 1}: {len(np.nonzero(fo != fg)[0])} fingerprints differ, nodes {bad}")
            so, sg = o.stats(), g.stats()
            print("  counters differing:", {k: (so[k], sg[k]) for k in so if so[k] != sg.get(k)})
            for i in bad[:3]:
                a, b = o.row(int(i)), g.row(int(i))
                d = np.nonzero(a != b)[0]
                print(f"  node {i}: {len(d)} row bytes differ, e.g. {[(int(j), int(a[j]), int(b[j])) for j in d[:8]]}")
                print(f"    suspects oracle {o.suspects(int(i))} gpu {g.suspects(int(i))}")
            return
    print("no divergence in the interval (?)")


t0 = time.time()
o, g = Sim(parity.oracle_lib(omp=True), cfg), Sim(parity.gpu_lib(), cfg)
r = 0
while r < rounds:
    o.step(every); g.step(every); r += every
    if digest(o) != digest(g):
        print(f"mismatch detected at round {r - 1} ({time.time() - t0:.0f} s); bisecting [{r - every}, {r})", flush=True)
        o.close(); g.close()
        run(r - every, r)
        break
    print(f"round {r - 1}: equal ({time.time() - t0:.0f} s)", flush=True)
else:
    print("equal through", rounds)
