"""Quick timing of the HIP simulator on a config (dev tool): quick_perf.py N ROUNDS [sim|sock] [lat] [exact]."""
import os, sys, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from kaboodle_amd._ffi import SimConfig, KB_INIT_CONVERGED, KB_FAILED_SOCKET_FAITHFUL, KB_FAILED_SIM_SENDER, KB_VARIANT_EXACT_LRU
import kaboodle_amd
N = int(sys.argv[1]) if len(sys.argv) > 1 else 65536
R = int(sys.argv[2]) if len(sys.argv) > 2 else 10
MODE = KB_FAILED_SOCKET_FAITHFUL if (len(sys.argv) > 3 and sys.argv[3] == "sock") else KB_FAILED_SIM_SENDER
# the bench's sizing (bench.rank_config): capacity = peers + churn reserve for the run
cfg = SimConfig(capacity=N + max(4096, int(N * 0.001 * (R + 10) * 1.5)), initial_nodes=N, init_mode=KB_INIT_CONVERGED,
                loss=0.01, churn=0.001, seed=1, failed_mode=MODE, track_latency=int("lat" in sys.argv[4:]),
                debug_flags=int(os.environ.get("KB_QP_DBG", "0"), 0),   # KB_QP_DBG: force kernel variants (A/B)
                variant=KB_VARIANT_EXACT_LRU if "exact" in sys.argv[4:] else 0)   # exact: bench.py's default A3 order
t = time.time(); m = kaboodle_amd.Mesh(cfg); print("create", round(time.time() - t, 2), flush=True)
m.step(2)
m.reset_kernel_time()
t = time.time(); m.step(R); dt = time.time() - t
sw, n = m.kernel_time(0); rd, _ = m.kernel_time(1); fo, nf = m.kernel_time(2)
st = m.stats()
print(f"N={N} R={R} wall {dt/R*1e3:.2f} ms/round  rowpass {sw/n:.3f} ms ({m.kernel_bytes(0)/(sw*1e-3)/1e9:.1f} GB/s)  "
      f"fold {fo/max(nf,1):.3f} ms ({m.kernel_bytes(2)/max(fo*1e-3,1e-9)/1e9:.1f} GB/s)  round(ev) {rd/n:.3f} ms  "
      f"node-rounds/s {st['alive']*R/dt:.3e}", flush=True)
print(st)
kb = m.kernel_breakdown()                     # the byte-counted kernels' per-launch times (HIP events)
print("kernels " + "  ".join(f"{k} {v['ms'] / max(v['launches'], 1):.4f}" for k, v in sorted(kb.items()) if v["launches"]), flush=True)
import ctypes as C
lib = kaboodle_amd.lib().lib
buf = (C.c_uint64 * 3)()
if lib.kb_sim_debug_counters(m.h, buf, 3) == 0:
    print(f"A3 rows {buf[0]}  deep {buf[1]} ({buf[1] / max(buf[0], 1):.3f})  chunks/row {buf[2] / max(buf[0], 1):.2f}", flush=True)
