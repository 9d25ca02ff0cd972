#!/bin/bash
# Build an A/B variant of libmrs.so with extra compile flags for step.hip:
#   scripts/build_variant.sh NAME [flags...]  ->  mujoco_ros2_simulation_amd/libmrs_NAME.so
set -e
name=$1; shift
root=$(cd "$(dirname "$0")/.." && pwd)
obj=$root/build/obj
python3 -c "import sys; sys.path.insert(0, '$root'); from mujoco_ros2_simulation_amd import build; build.build_lib()"
hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -fno-hip-fp32-correctly-rounded-divide-sqrt "$@" \
  -c "$root/mujoco_ros2_simulation_amd/csrc/hip/step.hip" -o "$obj/step_$name.o"
others=$(ls "$obj"/*.o | grep -v "hip_step.hip.o" | grep -v "/step_" | grep -v "/batchv_" | grep -v "plugin_")
hipcc --offload-arch=gfx950 -shared -fPIC -o "$root/mujoco_ros2_simulation_amd/libmrs_$name.so" "$obj/step_$name.o" $others
echo "$root/mujoco_ros2_simulation_amd/libmrs_$name.so"
