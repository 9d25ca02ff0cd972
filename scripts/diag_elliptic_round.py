"""How far fp32 storage of the elliptic PGS forces alone moves the mobile base's per-step state (CPU,
oracle only): the same re-seeded steps as tests/test_gpu_elliptic.py (32 envs x 40 steps, tolerance 0,
50 sweeps) with and without ORC_ROUND_PGS=1 (the oracle rounds each block's new forces to fp32).
ORC_ROUND_AR=1 instead rounds the solver's inputs (Delassus rows, b) to fp32 with an fp64 iterate.
  python scripts/diag_elliptic_round.py [restate] [tolerance: "0", or "-" for the scene's default]"""
import os
import subprocess
import sys
import tempfile
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
RUN = f"""
import sys; sys.path[:0] = {[str(ROOT), str(ROOT / 'oracle'), str(ROOT / 'tests')]!r}
import numpy as np
from mujoco_ros2_simulation_amd import synth
import binding
from test_gpu_elliptic import elliptic_scene
m = elliptic_scene("mobile_base", "PGS", 1.0, sys.argv[3] if sys.argv[3] != "-" else ""); m.set_restate(int(sys.argv[1]))
n, period, settle = 32, 10, 20
envs = np.arange(n); q0 = synth.initial_qpos(m, envs); tab = synth.ctrl_table(m, envs, 10, period)
out = []
for e in range(n):
    d = binding.OracleData(m); d.qpos[:] = q0[e]
    for t in range(settle + 40):
        if t % period == 0: d.ctrl[:] = tab[t // period, e]
        if t >= settle:
            r = binding.OracleData(m)
            for k in ("qpos", "qvel", "qacc_warmstart", "ctrl"): getattr(r, k)[:] = getattr(d, k).astype(np.float32)
            r.step(); out.append(r.qvel.copy())
        d.step()
np.save(sys.argv[2], np.array(out))
"""


def main(restate=0, tol="0"):
    import numpy as np
    with tempfile.TemporaryDirectory() as tmp:
        res = []
        for var in ("", "ORC_ROUND_PGS", "ORC_ROUND_AR"):
            env = dict(os.environ)
            env.pop("ORC_ROUND_PGS", None)
            env.pop("ORC_ROUND_AR", None)
            if var:
                env[var] = "1"
            path = os.path.join(tmp, f"{var or 'none'}.npy")
            subprocess.run([sys.executable, "-c", RUN, str(restate), path, tol], check=True, env=env)
            res.append(np.load(path))
    a = res[0]
    for name, b in zip(("block forces (iterate)", "Delassus rows and b (inputs)"), res[1:]):
        e = np.abs(a - b) / np.maximum(np.abs(a), 1)
        print(f"restate {restate} tolerance {tol}: fp32 rounding of the {name} moves qvel by {e.max():.2e} "
              f"(relative to max(|qvel|, 1)); env-steps above 2e-5: {np.mean(e.max(axis=1) > 2e-5):.3f}")


if __name__ == "__main__":
    main(int(sys.argv[1]) if len(sys.argv) > 1 else 0, sys.argv[2] if len(sys.argv) > 2 else "0")
