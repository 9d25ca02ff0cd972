# Parity tests and C3 bench for each lane-group width (MRS_GROUP = lanes per environment).
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
: > gpurun_out/groups.log
for g in ${GROUPS_TO_RUN:-64 32 16}; do
  echo "== group $g" >> gpurun_out/groups.log
  MRS_GROUP=$g timeout -k 10 300 python -m pytest tests -x -q -m gpu >> gpurun_out/groups.log 2>&1
  rc=$?
  echo "pytest rc=$rc" >> gpurun_out/groups.log
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
  MRS_GROUP=$g timeout -k 10 120 python bench.py --steps 50 --warmup 5 --no-cpu-baseline >> gpurun_out/groups.log 2>&1 || exit $?
done
echo done
