# A/B of libmrs variants on C5 (bench line per variant) + the batch layout.  Bounded.
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 60 python -c "
import sys; sys.path.insert(0,'.')
from mujoco_ros2_simulation_amd import sim
m=sim.Model.load('scenes/arm_boxes.xml'); b=sim.Batch(m,64); print(b.layout())" || exit $?
for v in "$@"; do
  if [ "$v" = base ]; then unset MRS_LIB; else export MRS_LIB=$PWD/mujoco_ros2_simulation_amd/libmrs_$v.so; fi
  echo -n "$v: "
  timeout -k 10 200 python bench.py --config c5 --no-cpu-baseline --steps 20 | cut -c1-140 || exit $?
done
