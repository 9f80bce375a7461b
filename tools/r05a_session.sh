set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r05a
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v -p no:cacheprovider --timeout 240 --timeout-method thread tests/test_gpu_bijector_grad.py tests/test_gpu_workspace.py tests/test_c_abi.py "tests/test_gpu_parity.py::test_maximum_sizes" "tests/test_gpu_dense.py::test_dense_grad_full_size_against_oracle" -s > gpurun_out/r05a/pytest_new.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -5 gpurun_out/r05a/pytest_new.log
cp gpurun_out/parity.json gpurun_out/r05a/parity_new.json 2>/dev/null
if [ $rc -ge 124 ]; then exit $rc; fi
timeout -k 10 120 ./tools/mixed_stream > gpurun_out/r05a/mixed_stream.log 2>&1; rc2=$?
echo "probe rc=$rc2"; cat gpurun_out/r05a/mixed_stream.log
exit $rc
