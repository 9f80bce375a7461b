set -o pipefail
mkdir -p gpurun_out/r03e
timeout -k 10 120 ./tools/sector_probe > gpurun_out/r03e/sector_probe.log 2>&1 || exit $?
cat gpurun_out/r03e/sector_probe.log
cd /tmp && timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/r03e/pmc_sector -o s -- $GRAFT_REPO_ROOT/tools/sector_probe > $GRAFT_REPO_ROOT/gpurun_out/r03e/pmc_sector.log 2>&1; echo pmc rc=$?; cd $GRAFT_REPO_ROOT
timeout -k 10 700 python -u -m pytest tests -m gpu -v -p no:cacheprovider --timeout 240 --timeout-method thread > gpurun_out/r03e/pytest_gpu.log 2>&1
echo "pytest rc=$?"
tail -8 gpurun_out/r03e/pytest_gpu.log
