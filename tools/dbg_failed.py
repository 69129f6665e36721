"""Dev tool (GPU): run a standard parity case on the oracle and the HIP library until the first round whose
state differs, then list, for the first differing rows, the peers whose membership differs and the Failed
broadcast entries that name them or their senders.   python tools/dbg_failed.py [case name]"""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests"))
import parity  # noqa: E402

name = sys.argv[1] if len(sys.argv) > 1 else "probes"
case, rounds = next((c, r) for n, c, r in parity.standard_cases() if n == name)
o = parity.Sim(parity.oracle_lib(), case["cfg"])
g = parity.Sim(parity.gpu_lib(), case["cfg"])
parity.setup(o, case)
parity.setup(g, case)
for r in range(rounds):
    bc = o.broadcasts()
    parity.apply_events((o, g), case, r)
    o.step(1)
    g.step(1)
    d = parity.diff_states(parity.state_of(o), parity.state_of(g))
    if not d:
        continue
    print(f"round {r}: " + "; ".join(d[:6]))
    fails = [(k, s, p) for k, (kind, s, p) in enumerate(x for x in bc if x[0] == "Failed")]
    print(f"Failed list: {len(fails)} entries; Join: {sum(1 for x in bc if x[0] == 'Join')}")
    named = {}
    for k, s, p in fails:
        named.setdefault(p, []).append(k)
    ro, rg = o.rows(), g.rows()
    bad_rows = np.unique(np.argwhere(ro != rg)[:, 0])
    print(f"{len(bad_rows)} rows differ: {bad_rows[:12].tolist()}")
    for i in bad_rows[:4]:
        cols = np.argwhere(ro[i] != rg[i]).ravel()
        print(f" row {i}: {len(cols)} peers differ")
        for j in cols[:6]:
            ent = [(k, fails[k][1]) for k in named.get(int(j), [])]
            deps = [(k, s, named.get(s, [])[:4]) for k, s in ent]
            print(f"   peer {j}: oracle {ro[i, j]} gpu {rg[i, j]}; named by (entry, sender, entries naming the sender) {deps[:5]}")
    break
