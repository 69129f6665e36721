"""Round time and sweep time as the 64K mesh ages (dev tool): blocks of B rounds up to R."""
import os, sys, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from kaboodle_amd._ffi import SimConfig, KB_INIT_CONVERGED
import kaboodle_amd
N = int(sys.argv[1]) if len(sys.argv) > 1 else 65536
R = int(sys.argv[2]) if len(sys.argv) > 2 else 300
Bk = int(sys.argv[3]) if len(sys.argv) > 3 else 25
cfg = SimConfig(capacity=N + max(4096, int(N * 0.001 * (R + 8) * 1.5)), initial_nodes=N, init_mode=KB_INIT_CONVERGED,
                loss=0.01, churn=0.001, seed=1)
m = kaboodle_amd.Mesh(cfg)
for b in range(R // Bk):
    m.reset_kernel_time()
    t = time.time(); m.step(Bk); dt = time.time() - t
    sw, n = m.kernel_time(0)
    st = m.stats()
    print(f"rounds {b*Bk:4d}-{(b+1)*Bk-1:4d}: {dt/Bk*1e3:7.2f} ms/round  sweep {sw/n:6.3f} ms  "
          f"row-pass bytes/launch {m.kernel_bytes(0)/n/1e6:8.1f} MB  agree {st['agree']}/{st['alive']}  "
          f"kpr {st['sent_kpr']} oversize {st['drop_oversize']}", flush=True)
