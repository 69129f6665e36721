"""Which HIP runtimes a process maps when the library is loaded before / after torch (diagnostic)."""
import sys
order = sys.argv[1]
if order == "torch_first":
    import torch
    torch.cuda.is_available()
import kaboodle_amd
kaboodle_amd.lib()
if order == "lib_first":
    import torch
    print("torch sees GPU:", torch.cuda.is_available())
maps = sorted({l.split()[-1] for l in open("/proc/self/maps") if "amdhip64" in l})
print(order, "maps:", maps)
from kaboodle_amd._ffi import SimConfig
try:
    with kaboodle_amd.Mesh(SimConfig(capacity=8, initial_nodes=4, seed=1)) as m:
        m.step(1)
        print(order, "create+step ok", m.stats()["round"])
except Exception as e:
    print(order, "FAILED:", e)
