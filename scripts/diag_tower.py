"""Diagnostic: 5-box tower (80 rows in one island) on the GPU vs the oracle; prints the max |dq| and
the GPU state for comparison across library variants (MRS_LIB)."""
import sys
from pathlib import Path
import numpy as np
ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT)); sys.path.insert(0, str(ROOT / "oracle"))
import binding
from mujoco_ros2_simulation_amd import sim
nb = int(sys.argv[1]) if len(sys.argv) > 1 else 5
bodies = "".join(
    f'<body pos="0 0 {0.1 + 0.2 * k + 0.001 * k:.4f}" euler="0 0 {0.2 * k:.2f}"><freejoint/>'
    f'<geom type="box" size="0.1 0.1 0.1" mass="1"/></body>' for k in range(nb))
xml = f"""<mujoco><option timestep="0.002"/><worldbody><geom type="plane" size="0 0 1"/>{bodies}
</worldbody></mujoco>"""
model = sim.Model.from_string(xml)
b = sim.Batch(model, 1)
d = binding.OracleData(model)
for steps in (1, 1, 8, 40, 150):
    b.step(steps); d.step(steps)
    q = b.get(sim.FIELD_QPOS)[0]
    print(steps, "ncon", int(b.get(sim.FIELD_NCON)[0, 0]), d.ncon, "max|dq|", np.abs(q - d.qpos).max(), "layout", b.layout().get("pipe_w"))
np.save(str(ROOT / "gpurun_out" / f"tower_{Path(sim.LIB_PATH).stem}.npy"), q)
