import os, sys
sys.path.insert(0, "/root/repo"); sys.path.insert(0, "/root/repo/tests"); sys.path.insert(0, "/root/repo/zprize23-gpu-submission_amd")
import pnp
from bench import Synthetic
ctx = pnp.Context(0)
syn = Synthetic(ctx, 16, 0, seed=2, circuit="merkle")
print("synth", ctx.hbm_usage(), flush=True)
ctx.load_prover_key(syn.pk, syn.n, device_ptrs=True)
print("pk", ctx.hbm_usage(), flush=True)
ctx.load_commit_key(syn.ck, syn.n, device_ptrs=True)
print("ck", ctx.hbm_usage(), flush=True)
ctx.prove(syn.cs, device_ptrs=True)
print("prove", ctx.hbm_usage(), flush=True)
