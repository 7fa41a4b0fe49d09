"""Diagnose which HIP runtime / device visibility combination works on the box."""
import os, sys, ctypes as C
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "zprize23-gpu-submission_amd"))
mode = sys.argv[1]
if mode == "torch_only":
    import torch
    print("torch", torch.__version__, torch.cuda.is_available(), torch.cuda.device_count())
elif mode == "lib_only":
    import pnp
    ctx = pnp.Context(0)
    print("ctx ok")
elif mode == "torch_then_lib":
    import torch
    print("torch avail", torch.cuda.is_available())
    x = torch.zeros(4, device="cuda")
    import pnp
    ctx = pnp.Context(0)
    print("ctx ok after torch")
elif mode == "lib_then_torch":
    import pnp
    ctx = pnp.Context(0)
    import torch
    print("torch avail", torch.cuda.is_available())
for l in open("/proc/self/maps"):
    if "amdhip64" in l and "r-xp" in l:
        print(l.strip().split()[-1])
