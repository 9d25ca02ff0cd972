#!/bin/bash
# Build an A/B variant of libmrs.so with extra compile flags for step.hip (every split part):
#   scripts/build_variant.sh NAME [flags...]  ->  mujoco_ros2_simulation_amd/libmrs_NAME.so
set -e
root=$(cd "$(dirname "$0")/.." && pwd)
cd "$root" && python3 -m mujoco_ros2_simulation_amd.build variant "$@"
