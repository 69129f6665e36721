"""How far rows of the bench workload are from the majority row (dev tool for the sweep's fold).

    python tools/row_divergence.py [rounds]

Steps the configs[2] workload, then for 256 sampled rows counts the 8-id blocks whose member pattern
differs from the bitwise majority of 31 other sampled rows, per 1152-id segment.
"""
import os, sys
import numpy as np
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from kaboodle_amd._ffi import SimConfig, KB_INIT_CONVERGED
import kaboodle_amd
N, R = 65536, int(sys.argv[1]) if len(sys.argv) > 1 else 55
m = kaboodle_amd.Mesh(SimConfig(capacity=N + 6000, initial_nodes=N, init_mode=KB_INIT_CONVERGED, loss=0.01,
                                churn=0.001, seed=1))
m.step(R)
C = N + 6000
W = (C + 8191) // 8192 * 8192
def row(i):
    b = np.zeros(W, dtype=np.uint8)
    p = m.peers(i)
    b[np.asarray(p, dtype=np.int64)] = 1
    return b
alive = [i for i in range(0, N, N // 300) if m.is_running(i)][:287]
rows = np.stack([row(i) for i in alive])
cons = (rows[:31].sum(0) * 2 > 31).astype(np.uint8)
seg = W // 64
for name, ref in (("majority of 31", cons),):
    d = (rows[31:] != ref[None, :]).reshape(len(rows) - 31, W // 8, 8).any(2)   # differing 8-id blocks
    per_seg = d.reshape(len(rows) - 31, 64, seg // 8).sum(2)
    print(f"{name}: differing blocks per row mean {d.sum(1).mean():.1f}  per segment mean {per_seg.mean():.2f}  "
          f"max over 64 rows per segment ~{np.mean([per_seg[k:k+64].max(0).mean() for k in range(0, len(per_seg) - 63, 64)]):.2f}")
