set -o pipefail
bash tools/gpu_session.sh r03y gradd1tests gradw1 grad prof_grad || exit $?
