"""GPU vs oracle contacts on states of the MPR test scene (tests/test_gpu_mesh.py MPR_SCENE): per pair
type, the worst normal / dist / position difference, and the worst cases with their oracle polish
fallback status (ORC_POLISH_DEBUG).  Needs the GPU.   python scripts/diag_mpr_gpu.py [n_states]"""
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(ROOT), str(ROOT / "oracle"), str(ROOT / "tests")]
import numpy as np  # noqa: E402

from mujoco_ros2_simulation_amd import sim, synth  # noqa: E402
import binding  # noqa: E402
from test_gpu_mesh import MPR_SCENE  # noqa: E402


def main(n_states=100, restate=0):
    model = sim.Model.from_string(MPR_SCENE)
    print(f"--- restate {restate}")
    d = binding.OracleData(model)
    d.qpos[:] = synth.initial_qpos(model, np.arange(1))[0]
    Q, V = [], []
    for t in range(75 + n_states):
        d.step()
        if t >= 75:
            Q.append(d.qpos.astype(np.float32).astype(np.float64))
            V.append(d.qvel.astype(np.float32).astype(np.float64))
    model.set_restate(restate)
    b = sim.Batch(model, len(Q))
    b.set(sim.FIELD_QPOS, np.array(Q))
    b.set(sim.FIELD_QVEL, np.array(V))
    b.forward()
    worst = {}
    for e, (q, v) in enumerate(zip(Q, V)):
        g, dist, pos, frame = b.contacts(e)
        o = binding.OracleData(model)
        o.qpos[:] = q
        o.qvel[:] = v
        o.forward()
        gr, dr, pr, fr = o.contacts()
        if not np.array_equal(g, gr):
            print("pair lists differ at state", e, g.tolist(), gr.tolist())
            continue
        for k, (g1, g2) in enumerate(gr.tolist()):
            kind = (int(model.geom_type[g1]), int(model.geom_type[g2]))
            dn = float(np.max(np.abs(frame[k, :3] - fr[k, :3])))
            dd = abs(float(dist[k] - dr[k]))
            dp = float(np.max(np.abs(pos[k] - pr[k])))
            if dn > 1e-3:
                print(f"  state {e} contact {k} {kind}: gpu n {np.round(frame[k, :3], 5).tolist()} dist {dist[k]:.4e}; "
                      f"oracle n {np.round(fr[k, :3], 5).tolist()} dist {dr[k]:.4e}")
            w = worst.setdefault(kind, [0, 0, 0, None])
            if dn > w[0]:
                w[0] = dn
                w[3] = (e, k)
            w[1] = max(w[1], dd)
            w[2] = max(w[2], dp)
    for kind, (dn, dd, dp, at) in sorted(worst.items()):
        print(f"pair types {kind}: normal {dn:.2e} dist {dd:.2e} pos {dp:.2e} (worst normal at state/contact {at})")


if __name__ == "__main__":
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 100
    main(n, 0)
    main(n, sim.RESTATE_NO_MPR_POLISH)
