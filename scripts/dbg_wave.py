"""Debug helper: Viterbi of one random N-state HMM on the given block lengths vs the oracle."""
import sys
import time

import numpy as np

sys.path.insert(0, ".")
from itrails_amd import hmm  # noqa: E402
from itrails_amd.synth import sample_alignment  # noqa: E402
from itrails_amd.tables import build_tables  # noqa: E402
from oracle import hmm_oracle as O  # noqa: E402

n = int(sys.argv[1])
lengths = [int(x) for x in sys.argv[2].split(",")]
rng = np.random.default_rng(7)
a = rng.random((n, n)) ** 3
np.fill_diagonal(a, 0)
a /= a.sum(1, keepdims=True)
d = rng.uniform(0.9, 0.999, size=n)
a = a * (1 - d)[:, None]
a[np.arange(n), np.arange(n)] = d
b = rng.dirichlet(np.full(256, 0.3), size=n)
pi = rng.dirichlet(np.ones(n))
obs, off, _ = sample_alignment(a, b, pi, lengths, seed=3)
t = build_tables(a, b, pi)
model, plan = hmm.Model(a, b, pi), hmm.Plan(off)
print("start", n, lengths, flush=True)
t0 = time.time()
path = hmm._paths(model, plan, obs)
print("device done", round(time.time() - t0, 3), flush=True)
ref = O.viterbi(t, obs, off)
bad = np.nonzero(path != ref)[0]
print("mismatches", len(bad), bad[:20], flush=True)
