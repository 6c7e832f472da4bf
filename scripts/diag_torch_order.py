"""diagnostic: does torch see the GPU after the engine initialised HIP first?"""
import sys
sys.path.insert(0, ".")
from jylis_amd.engine import Engine
e = Engine(device=0)
print("engine ok", flush=True)
import torch
print("torch device_count", torch.cuda.device_count(), "available", torch.cuda.is_available(), flush=True)
try:
    x = torch.empty(4, device="cuda:0")
    print("torch alloc ok", flush=True)
except Exception as ex:
    print("torch alloc failed:", ex, flush=True)
