import sys, numpy as np, torch
sys.path.insert(0, 'real-time-disaster-management_amd'); sys.path.insert(0, '.')
from oracle import nms as ON
from rtdm.nms import nms_batched
rng = np.random.default_rng(0)
n, a, nc = 3, 3000, 3
io = np.zeros((n, a, 5 + nc), np.float32)
io[..., 0:2] = rng.uniform(0, 400, (n, a, 2))
io[..., 2:4] = rng.uniform(1, 80, (n, a, 2))
io[..., 4:] = rng.uniform(0, 1, (n, a, 1 + nc))
io[0, 5, 2] = np.inf
io[1, 7, 0] = np.nan
io[2] = 0
from rtdm import _lib as L
import os
L.check(L.lib().rtdm_set_tuning(b'nms_variant', int(os.environ.get('V', '0'))))
for ml in (True, False):
  for conf in (0.3, 0.05, 0.7):
    for nanfix in (False, True):
        x = io.copy()
        if nanfix: x[1, 7, 0] = 5.0
        det, idx, cnt = nms_batched(torch.from_numpy(x).cuda(), conf, 0.4, ml, None, False, a * nc)
        ref, ref_idx = ON.non_max_suppression(x, conf, 0.4, ml, None, False, return_index=True)
        cnt = cnt.cpu().numpy(); idx = idx.cpu().numpy()
        for b in range(2):
            r = ref_idx[b]
            # candidate count
            o = x[b]; obj = o[:, 4]
            ok = (obj > conf) & (o[:, 2] > 2) & (o[:, 3] > 2) & (o[:, 2] < 4096) & (o[:, 3] < 4096)
            ncand = int(((o[:, 5:] * obj[:, None] > conf) & ok[:, None]).sum()) if ml else int(ok.sum())
            good = cnt[b] == len(r) and np.array_equal(idx[b, :cnt[b]], r)
            first = None
            if not good:
                m = min(cnt[b], len(r))
                d = np.nonzero((idx[b, :m] != r[:m]).any(1))[0]
                first = int(d[0]) if len(d) else m
            print(f"ml={ml} conf={conf} nanfix={nanfix} img={b} ncand~{ncand} got={cnt[b]} ref={len(r)} ok={good} first_bad={first}")
