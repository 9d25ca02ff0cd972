"""Diagnostics (GPU): each benchmark scene's kernel configuration (mrs_debug_batch_layout: group width,
LDS floats per env, scratch floats per env, blocked mode, pipe width, row / contact capacity, trees)."""
import sys; sys.path.insert(0,'.')
import ctypes as C
from mujoco_ros2_simulation_amd import sim
for sc, n in [("scenes/arm7_lidar.xml", 8192), ("scenes/mobile_base.xml", 2048), ("scenes/arm_boxes.xml", 8192)]:
    m = sim.Model.load(sc); b = sim.Batch(m, 64)
    out = (C.c_int * 8)(); sim.lib().mrs_debug_batch_layout(b._h, out, 8); print(sc, list(out)); b.close()
