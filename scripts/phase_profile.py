"""Per-phase cycle breakdown of the step kernel with a profiling build (MRS_LIB pointing at a
library built with -DMRS_PHASE_TIMING, e.g. scripts/build_variant.sh timing -DMRS_PHASE_TIMING).
Usage: phase_profile.py [scene.xml|c2] [n_envs] [launches] [solver]  (default: C3, 8192 envs, 20 launches)"""
import json
import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
import torch  # noqa: E402

from mujoco_ros2_simulation_amd import sim, synth  # noqa: E402

scene = sys.argv[1] if len(sys.argv) > 1 else str(ROOT / "scenes" / "arm7_lidar.xml")
n = int(sys.argv[2]) if len(sys.argv) > 2 else 8192
launches = int(sys.argv[3]) if len(sys.argv) > 3 else 20
period = 10
if scene == "c2":  # the C2 bench scene: the reference's scene.xml with sensors disabled
    sys.path.insert(0, str(ROOT))
    from bench import ref_scene_xml  # noqa: E402
    model = sim.Model.from_string(*ref_scene_xml(sensors=False))
    scene = "scene"
else:
    xml = Path(scene).read_text()
    if len(sys.argv) > 4:  # solver override (bench.py --solver)
        sys.path.insert(0, str(ROOT))
        from bench import with_solver  # noqa: E402
        xml = with_solver(xml, sys.argv[4])
    model = sim.Model.from_string(xml, str(Path(scene).parent))
b = sim.Batch(model, n)
b.set(sim.FIELD_QPOS, synth.initial_qpos(model, np.arange(n)))
table = torch.from_numpy(synth.ctrl_table(model, np.arange(n), launches + 2, period).astype(np.float32)).cuda()
b.set_ctrl_device(table[0].data_ptr()); b.step(period); b.sync()
sim.phase_cycles(reset=True)
for p in range(launches):
    b.set_ctrl_device(table[p + 1].data_ptr())
    b.step(period)
b.sync()
pc = sim.phase_cycles()
tot = sum(v for k, v in pc.items() if "." not in k)
print(json.dumps({"scene": Path(scene).stem, "n": n, "cycles_per_env_step": tot / (n * launches * period),
                  **{k: round(v / tot, 4) for k, v in pc.items()}}))
