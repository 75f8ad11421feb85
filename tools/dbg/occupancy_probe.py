import sys, os
sys.path.insert(0, os.getcwd())
import torch
from multigrad_amd.ops._ext import ext
E = ext()
print("ext loaded", flush=True)
dev = torch.device("cuda", 0)
for args in [(10, True, False, False), (10, True, False, True)]:
    print(args, E.smf_fwd_lanes_max_blocks(*args), flush=True)
