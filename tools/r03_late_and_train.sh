set -u
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_env_gpu.py -k "late" > gpurun_out/r03b_late.txt 2>&1
rc=$?; tail -3 gpurun_out/r03b_late.txt; [ $rc -ne 0 ] && exit $rc
CONFIG=configs/training/16x16x40_medium_randperm.yaml SEEDS="0 1 2" TAG=randperm LIMIT=1000 bash tools/train_quality.sh
