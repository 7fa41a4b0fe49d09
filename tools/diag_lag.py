import sys, numpy as np
sys.path.insert(0, "tests"); sys.path.insert(0, "zprize23-gpu-submission_amd"); sys.path.insert(0, ".")
import pnp
from gpu_util import empty_dev, from_dev, to_dev
from pnp_testlib import fr_mont, oracle, to_limbs, vp
from test_gpu_lagrange import _ck, _srs, _evals, _pt
for lg in [3, 5]:
    n = 1 << lg
    ctx = pnp.Context(0)
    srs = _srs(ctx, n + 3, fr_mont(0x1234567890ABCDEF1357 + lg))
    pts = from_dev(srs, 12).copy()
    ctx.load_commit_key(_ck(srs.data_ptr()), n + 3, device_ptrs=True)
    ev = _evals(ctx, n, 17 + lg)
    co = ev.copy(); oracle().or_ntt(vp(co), lg, 1, 0)
    exp = np.zeros(12, dtype=np.uint64)
    oracle().or_commit(vp(pts[:n].copy()), vp(co), n, vp(exp))
    print(lg, "commit_ck(coeffs) ok:", (_pt(ctx.commit_ck(to_dev(co).data_ptr(), n)) == exp).all(),
          "commit_evals ok:", (_pt(ctx.commit_evals(to_dev(ev).data_ptr(), n)) == exp).all())
    bad = []
    for i in range(n):
        e = np.zeros((n, 4), dtype=np.uint64); e[i] = to_limbs(fr_mont(1), 4)
        c = e.copy(); oracle().or_ntt(vp(c), lg, 1, 0)
        oracle().or_commit(vp(pts[:n].copy()), vp(c), n, vp(exp))
        if not (_pt(ctx.commit_evals(to_dev(e).data_ptr(), n)) == exp).all(): bad.append(i)
    print(lg, "unit vectors wrong at", bad)
    ctx.close()
