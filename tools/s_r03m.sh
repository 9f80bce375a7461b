set -o pipefail
bash tools/gpu_session.sh r03m smoke bench prof pmc c5 c3 grad grad_c3 dense dgrad bijector || exit $?
mkdir -p gpurun_out/r03m
timeout -k 10 200 python bench.py --mode flows --steps 10 --warmup 3 --cpu-seconds 6 > gpurun_out/r03m/bench_flows.log 2>&1; echo "flows rc=$?"
tail -1 gpurun_out/r03m/bench_flows.log | cut -c1-300
timeout -k 10 300 python tools/microbench.py occ 2>&1 | grep -v amdgpu.ids | tee gpurun_out/r03m/occ.log | cut -c1-200
