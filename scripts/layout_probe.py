"""Diagnostics (GPU): each benchmark scene's kernel configuration (mrs_debug_batch_layout: group width,
LDS floats per env, scratch floats per env, blocked mode, pipe width, row / contact capacity, trees)."""
import sys; sys.path.insert(0,'.')
import ctypes as C
from mujoco_ros2_simulation_amd import sim
scenes = sys.argv[1:] or ["scenes/arm7_lidar.xml", "scenes/mobile_base.xml", "scenes/arm_boxes.xml"]
for sc in scenes:
    m = sim.Model.load(sc); b = sim.Batch(m, 64)
    print(sc, b.layout()); b.close()
