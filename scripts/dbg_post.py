import sys, numpy as np, torch
sys.path.insert(0, '/root/repo')
import bench
from itrails_amd import hmm
from itrails_amd.synth import block_lengths, sample_alignment
a, b, pi, _ = bench.load_model(5)
import os
for L, frac in ((0, None), (0, '0'), (100000, None), (100000, '0')):
    if frac is None: os.environ.pop('ITR_POST_SPLIT_FRAC', None)
    else: os.environ['ITR_POST_SPLIT_FRAC'] = frac
    if L:
        lengths = np.full(100, L)
    else:
        lengths = block_lengths(np.random.default_rng(12345), 10_000_000, 2000.0)
    obs, off, _ = sample_alignment(a, b, pi, lengths, seed=777)
    model, plan = hmm.Model(a, b, pi), hmm.Plan(off)
    plan.reserve(70, posterior=True)
    d_obs = torch.from_numpy(obs.astype(np.int16)).cuda()
    post = torch.full((plan.total, 70), -1.0, dtype=torch.float64, device='cuda')
    hmm.posterior_device(model, plan, d_obs, out=post)
    torch.cuda.synchronize()
    import time; t0 = time.perf_counter()
    for _ in range(3): hmm.posterior_device(model, plan, d_obs, out=post)
    torch.cuda.synchronize(); wall = (time.perf_counter() - t0) / 3 * 1e3
    print('L', L, 'frac', frac, 'wall_ms', round(wall, 2), 'min', float(post.min()), 'rowsum err', float((post.sum(1) - 1).abs().max()))
    for w in ("posterior_fwd", "posterior_bwd"):
        try:
            print(w, hmm.last_kernel_ms(w))
        except Exception as e:
            print(w, 'ERR', e)
