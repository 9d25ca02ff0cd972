"""kernel layout (group width, LDS per env) of the bench scenes (diagnostic)"""
import sys
sys.path.insert(0, ".")
from mujoco_ros2_simulation_amd import sim
for f in sys.argv[1:]:
    m = sim.Model.load(f)
    b = sim.Batch(m, 64)
    print(f, b.layout(), flush=True)
    b.close()
