"""Contact-count flips of the re-seeded parity tests: proof that each one sits at a threshold.

The re-seeded tests (test_gpu_solvers._reseeded, test_gpu_parity._reseeded_sensors) start every step
of the GPU and of the fp64 oracle from the same fp32 state and exclude the env-steps whose contact
count differs.  An exclusion is legitimate only when the differing contact is decided by rounding:
a contact whose distance sits within fp32 noise of its activation margin, or a box-box clip vertex
on the edge of the reference face.  `explain_flip` checks exactly that, the way the rangefinder tests
prove their outliers graze a silhouette (test_gpu_parity: the oracle ray tilted by 1e-4 rad flips):
the GPU's contact pairs (geom1, geom2 with multiplicity) must be what the exact fp64 pipeline itself
produces for some state within `eps` of the step's start state (qpos perturbed component-wise,
quaternions re-normalised by the oracle's kinematics).  A real bug -- a missing or extra contact away
from any threshold -- is reproduced by no nearby state and fails the test.

Test infrastructure: the oracle (oracle/binding.py) is the checker, never the thing measured.
"""
from collections import Counter

import numpy as np

import binding

# largest state perturbation tried: the GPU evaluates the kinematics of a ~1 m arm in fp32, so geom
# poses (and contact distances) carry ~1e-6 m of rounding; 2e-5 leaves an order of magnitude of margin
# and is still far below any physical feature of the scenes (box half-size 0.05 m, margins 1e-3)
EPS = (1e-7, 1e-6, 5e-6, 2e-5)
TRIES = 24


def pair_counts(g) -> Counter:
    return Counter(tuple(int(x) for x in p) for p in np.asarray(g).reshape(-1, 2))


def explain_flip(model, qpos, qvel, gpu_pairs, rng=None):
    """True when some state within EPS of (qpos, qvel) makes the oracle's forward pass produce the
    GPU's multiset of (geom1, geom2) pairs for every pair on which the two sides differ at
    (qpos, qvel).  Returns (explained, differing pairs, perturbation scale that reproduced it)."""
    rng = rng or np.random.default_rng(0)
    want = pair_counts(gpu_pairs)
    d = binding.OracleData(model)
    d.qpos[:] = qpos
    d.qvel[:] = qvel
    d.forward()
    have = pair_counts(d.contacts()[0])
    diff = sorted(p for p in set(want) | set(have) if want[p] != have[p])
    if not diff:
        return True, diff, 0.0
    for eps in EPS:
        for _ in range(TRIES):
            d.qpos[:] = qpos + eps * rng.uniform(-1.0, 1.0, size=len(qpos))
            d.qvel[:] = qvel
            d.forward()
            c = pair_counts(d.contacts()[0])
            if all(c[p] == want[p] for p in diff):
                return True, diff, eps
    return False, diff, None
