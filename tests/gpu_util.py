"""Device-memory plumbing for the GPU parity tests (torch = allocator only)."""
import numpy as np


# torch fills / copies on its own stream; the library works on another one, so
# every helper waits for torch before handing the buffer over (without this a
# late zero-fill can overwrite what the library already wrote)
def to_dev(arr: np.ndarray):
    import torch
    a = np.ascontiguousarray(arr).view(np.int64)
    t = torch.from_numpy(a.copy()).to("cuda")
    torch.cuda.synchronize()
    return t


def from_dev(t, shape_last=4) -> np.ndarray:
    import torch
    torch.cuda.synchronize()
    return t.cpu().numpy().view(np.uint64).reshape(-1, shape_last)


def empty_dev(n_elems: int, limbs: int = 4):
    import torch
    t = torch.zeros((n_elems, limbs), dtype=torch.int64, device="cuda")
    torch.cuda.synchronize()
    return t
