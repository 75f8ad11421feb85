"""One-off toolchain probe: hipcc-7.2 built extension under torch's bundled HIP 7.0 runtime."""
import sys, os
import torch
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__))))
import _probe
x = torch.zeros(1000, device="cuda")
_probe.add_one(x)
torch.cuda.synchronize()
print("sum", x.sum().item())
maps = open("/proc/self/maps").read().splitlines()
print(sorted({l.split()[-1] for l in maps if "amdhip64" in l}))
print(torch.cuda.get_device_name(0), torch.cuda.get_device_properties(0))
