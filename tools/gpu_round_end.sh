# One GPU-box session for the round's record: the training checks (tests, A/B, kernel trace, stamps),
# then the whole GPU suite, smoke, the default bench line and a rocprofv3 kernel trace of the bench.
# Every GPU step runs under its own time limit; a failure ends the script (no retries).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
bash tools/gpu_train_check.sh || exit $?
bash tools/gpu_train_prof.sh || exit $?
bash tools/gpu_train_stamps.sh || exit $?
PYTEST_ARGS="--timeout 300 --timeout-method thread" bash tools/gpu_check.sh test || exit $?
bash tools/gpu_check.sh bench || exit $?
bash tools/gpu_check.sh prof || exit $?
echo ROUND_END_OK
