#!/bin/bash
# One GPU-box session: parity tests, smoke, bench, rocprofv3 kernel-trace stats
# (and optionally PMC passes).  Every GPU step has its own time limit; the
# session stops at the first crash-like exit (fault/abort/segv/timeout).
#   usage: bash tools/gpu_session.sh <tag> [tests|smoke|bench|prof|pmc|c3|c5 ...]
set -o pipefail
TAG=${1:-r01}; shift
STEPS=${*:-tests smoke bench prof}
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$ROOT"
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp

crashed() {  # exit codes that mean "stop using the GPU in this call"
  case $1 in 124|134|137|139) return 0;; esac
  [ "$1" -gt 128 ] && return 0
  return 1
}

run() {  # run <name> <timeout> <cmd...>
  local name=$1 to=$2; shift 2
  echo "=== $name: $*" | tee -a "$OUT/session.log"
  local t0=$(date +%s)
  timeout -k 10 "$to" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc ($(( $(date +%s) - t0 ))s)" | tee -a "$OUT/session.log"
  tail -n 15 "$OUT/$name.log"
  if crashed $rc; then echo "!!! $name crashed (rc=$rc); stopping GPU work" | tee -a "$OUT/session.log"; exit $rc; fi
  return 0
}

rocm-smi --showproductname > "$OUT/rocm_smi.txt" 2>&1 || true
nproc > "$OUT/nproc.txt"; lscpu > "$OUT/lscpu.txt" 2>&1 || true

for s in $STEPS; do
  case $s in
    tests) run pytest_gpu 900 python -u -m pytest tests -m gpu -v -p no:cacheprovider --timeout 240 --timeout-method thread ;;
    testsx) run pytest_gpu 900 python -u -m pytest tests -m gpu -x -v -p no:cacheprovider --timeout 240 --timeout-method thread ;;
    smoke) run smoke 240 python -c "import __graft_entry__ as g; g.smoke()" ;;
    bench) run bench 240 python bench.py --steps 50 --warmup 10 ;;
    bench20) run bench20 240 python bench.py --gpus 1 --steps 20 --warmup 5 ;;  # the driver's command
    bench_nocpu) run bench_nocpu 300 python bench.py --steps 50 --warmup 10 --no-cpu-baseline ;;
    c3) run bench_c3 300 python bench.py --config C3 --steps 50 --warmup 10 --no-cpu-baseline ;;
    c5) run bench_c5 300 python bench.py --config C5 --steps 20 --warmup 5 --no-cpu-baseline ;;
    prof)  # the same command as the driver's default bench run
      { cd /tmp; run rocprof_c2 300 rocprofv3 --kernel-trace --stats -T --output-format csv -d "$OUT/prof_c2" -o c2 -- \
        python3 "$ROOT/bench.py"; cd "$ROOT"; } ;;
    prof_c5)
      { cd /tmp; run rocprof_c5 200 rocprofv3 --kernel-trace --stats -T --output-format csv -d "$OUT/prof_c5" -o c5 -- \
        python3 "$ROOT/bench.py" --config C5 --no-cpu-baseline; cd "$ROOT"; } ;;
    prof_c3)
      { cd /tmp; run rocprof_c3 200 rocprofv3 --kernel-trace --stats -T --output-format csv -d "$OUT/prof_c3" -o c3 -- \
        python3 "$ROOT/bench.py" --config C3 --no-cpu-baseline; cd "$ROOT"; } ;;
    pmc)
      { cd /tmp; run pmc_fetch 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d "$OUT/pmc_fetch" -o f -- \
        python3 "$ROOT/bench.py" --steps 5 --warmup 2 --no-cpu-baseline; cd "$ROOT"; }
      { cd /tmp; run pmc_write 300 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d "$OUT/pmc_write" -o w -- \
        python3 "$ROOT/bench.py" --steps 5 --warmup 2 --no-cpu-baseline; cd "$ROOT"; } ;;
    dgrad) run bench_dense_grad 300 python bench.py --mode dense_grad --steps 20 --warmup 5 --cpu-seconds 8 ;;
    prof_dgrad)
      { cd /tmp; run rocprof_dgrad 200 rocprofv3 --kernel-trace --stats -T --output-format csv -d "$OUT/prof_dgrad" -o dgrad -- \
        python3 "$ROOT/bench.py" --mode dense_grad --steps 20 --warmup 5 --no-cpu-baseline; cd "$ROOT"; } ;;
    grad) run bench_grad_c2 300 python bench.py --mode grad --steps 20 --warmup 5 --cpu-seconds 8 ;;
    grad_c3) run bench_grad_c3 300 python bench.py --mode grad --config C3 --steps 20 --warmup 5 --no-cpu-baseline ;;
    prof_grad)
      { cd /tmp; run rocprof_grad 200 rocprofv3 --kernel-trace --stats -T --output-format csv -d "$OUT/prof_grad" -o grad -- \
        python3 "$ROOT/bench.py" --mode grad --steps 20 --warmup 5 --no-cpu-baseline; cd "$ROOT"; } ;;
    pmc_c3)
      { cd /tmp; run pmc_fetch_c3 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d "$OUT/pmc_fetch_c3" -o f -- \
        python3 "$ROOT/bench.py" --config C3 --steps 5 --warmup 2 --no-cpu-baseline; cd "$ROOT"; }
      { cd /tmp; run pmc_write_c3 300 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d "$OUT/pmc_write_c3" -o w -- \
        python3 "$ROOT/bench.py" --config C3 --steps 5 --warmup 2 --no-cpu-baseline; cd "$ROOT"; } ;;
    pmc_grad)
      { cd /tmp; run pmc_fetch_grad 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d "$OUT/pmc_fetch_grad" -o f -- \
        python3 "$ROOT/bench.py" --mode grad --steps 5 --warmup 2 --no-cpu-baseline; cd "$ROOT"; }
      { cd /tmp; run pmc_write_grad 300 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d "$OUT/pmc_write_grad" -o w -- \
        python3 "$ROOT/bench.py" --mode grad --steps 5 --warmup 2 --no-cpu-baseline; cd "$ROOT"; } ;;
    pmc_dense)  # HBM traffic of the fused Dense forward and backward (separate FETCH / WRITE passes)
      for m in dense dense_grad; do
        { cd /tmp; run pmc_fetch_$m 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d "$OUT/pmc_fetch_$m" -o f -- \
          python3 "$ROOT/bench.py" --mode $m --steps 5 --warmup 2 --no-cpu-baseline; cd "$ROOT"; }
        { cd /tmp; run pmc_write_$m 300 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d "$OUT/pmc_write_$m" -o w -- \
          python3 "$ROOT/bench.py" --mode $m --steps 5 --warmup 2 --no-cpu-baseline; cd "$ROOT"; }
      done ;;
    finish) run finish 300 python tools/microbench.py finish ;;
    c5micro) run c5micro 300 python tools/microbench.py c5 ;;
    micro) run micro 600 python tools/microbench.py C2 C3 C5 C1 ;;
    debugnf) run debugnf 300 python tools/debug_nonfinite.py C3 ;;
    mem) run mem 300 python tools/microbench.py mem ;;
    mode) run mode 300 python tools/microbench.py mode ;;
    valu) run valu 300 python tools/microbench.py valu ;;
    c3micro) run c3micro 300 python tools/microbench.py c3 ;;
    dense) run bench_dense 300 python bench.py --mode dense --steps 50 --warmup 10 --cpu-seconds 6 ;;
    densetests) run densetests 300 python -u -m pytest tests/test_gpu_dense.py -m gpu -v -p no:cacheprovider --timeout 120 --timeout-method thread ;;
    diagtests) run diagtests 300 python -u -m pytest tests/test_gpu_diag.py -m gpu -v -s -p no:cacheprovider --timeout 120 --timeout-method thread ;;
    gradtests) run gradtests 300 python -u -m pytest tests/test_gpu_grad.py -m gpu -v -p no:cacheprovider --timeout 120 --timeout-method thread ;;
    grad_c3_nocpu) run bench_grad_c3 300 python bench.py --mode grad --config C3 --steps 20 --warmup 5 --no-cpu-baseline ;;
    dgradmicro) run dgradmicro 300 python tools/microbench.py dgrad ;;
    prof_grad_c3)
      { cd /tmp; run rocprof_grad_c3 200 rocprofv3 --kernel-trace --stats -T --output-format csv -d "$OUT/prof_grad_c3" -o gradc3 -- \
        python3 "$ROOT/bench.py" --mode grad --config C3 --steps 20 --warmup 5 --no-cpu-baseline; cd "$ROOT"; } ;;
    prof_dense)
      { cd /tmp; run rocprof_dense 200 rocprofv3 --kernel-trace --stats -T --output-format csv -d "$OUT/prof_dense" -o dense -- \
        python3 "$ROOT/bench.py" --mode dense --steps 20 --warmup 5 --no-cpu-baseline; cd "$ROOT"; } ;;
    pmc_c5)
      { cd /tmp; run pmc_fetch_c5 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d "$OUT/pmc_fetch_c5" -o f -- \
        python3 "$ROOT/bench.py" --config C5 --steps 5 --warmup 2 --no-cpu-baseline; cd "$ROOT"; }
      { cd /tmp; run pmc_write_c5 300 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d "$OUT/pmc_write_c5" -o w -- \
        python3 "$ROOT/bench.py" --config C5 --steps 5 --warmup 2 --no-cpu-baseline; cd "$ROOT"; } ;;
    dense_c5) run bench_dense_c5 300 python bench.py --mode dense --config C5 --steps 50 --warmup 10 --cpu-seconds 8 ;;
    prof_dense_c5)
      { cd /tmp; run rocprof_dense_c5 200 rocprofv3 --kernel-trace --stats -T --output-format csv -d "$OUT/prof_dense_c5" -o densec5 -- \
        python3 "$ROOT/bench.py" --mode dense --config C5 --steps 20 --warmup 5 --no-cpu-baseline; cd "$ROOT"; } ;;
    pmc_grad_c3)
      { cd /tmp; run pmc_fetch_grad_c3 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d "$OUT/pmc_fetch_grad_c3" -o f -- \
        python3 "$ROOT/bench.py" --mode grad --config C3 --steps 5 --warmup 2 --no-cpu-baseline; cd "$ROOT"; }
      { cd /tmp; run pmc_write_grad_c3 300 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d "$OUT/pmc_write_grad_c3" -o w -- \
        python3 "$ROOT/bench.py" --mode grad --config C3 --steps 5 --warmup 2 --no-cpu-baseline; cd "$ROOT"; } ;;
    pmc_sq_dgrad)  # stall breakdown of the fused Dense backward (two counter passes)
      { cd /tmp; run pmc_sq1_dgrad 90 timeout -s KILL 80 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE --kernel-trace --output-format csv -d "$OUT/pmc_sq1_dgrad" -o s1 -- \
        python3 "$ROOT/bench.py" --mode dense_grad --steps 5 --warmup 2 --prewarm-ms 0 --no-cpu-baseline; cd "$ROOT"; }
      { cd /tmp; run pmc_sq2_dgrad 90 timeout -s KILL 80 rocprofv3 --pmc SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_MISC SQ_INSTS_VALU SQ_INSTS_MFMA SQ_BUSY_CYCLES SQ_VALU_MFMA_COEXEC_CYCLES SQ_INSTS_LDS --kernel-trace --output-format csv -d "$OUT/pmc_sq2_dgrad" -o s2 -- \
        python3 "$ROOT/bench.py" --mode dense_grad --steps 5 --warmup 2 --prewarm-ms 0 --no-cpu-baseline; cd "$ROOT"; } ;;
    pmc_sq_dgrad_sb)  # the fused Dense backward, f32 vs split-bf16 GEMMs (diag NFN_DGRAD_SB): two SQ passes each
      for v in 0 1; do
        { cd /tmp; NFN_DGRAD_SB=$v run pmc_sq1_dgrad_sb$v 90 timeout -s KILL 80 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE --kernel-trace --output-format csv -d "$OUT/pmc_sq1_dgrad_sb$v" -o s1 -- \
          python3 "$ROOT/bench.py" --diag --mode dense_grad --steps 5 --warmup 2 --prewarm-ms 0 --no-cpu-baseline; cd "$ROOT"; }
        { cd /tmp; NFN_DGRAD_SB=$v run pmc_sq2_dgrad_sb$v 90 timeout -s KILL 80 rocprofv3 --pmc SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_MISC SQ_INSTS_VALU SQ_INSTS_MFMA SQ_BUSY_CYCLES SQ_VALU_MFMA_COEXEC_CYCLES SQ_INSTS_LDS --kernel-trace --output-format csv -d "$OUT/pmc_sq2_dgrad_sb$v" -o s2 -- \
          python3 "$ROOT/bench.py" --diag --mode dense_grad --steps 5 --warmup 2 --prewarm-ms 0 --no-cpu-baseline; cd "$ROOT"; }
      done ;;
    pmc_sq_fwd)  # issue / stall breakdown of the C5 posterior and the C2 forward (two counter passes each)
      for cfg in C5 C2; do
        { cd /tmp; run pmc_sq1_$cfg 90 timeout -s KILL 80 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_SALU --kernel-trace --output-format csv -d "$OUT/pmc_sq1_$cfg" -o s1 -- \
          python3 "$ROOT/bench.py" --config $cfg --steps 5 --warmup 2 --prewarm-ms 0 --no-cpu-baseline; cd "$ROOT"; }
        { cd /tmp; run pmc_sq2_$cfg 90 timeout -s KILL 80 rocprofv3 --pmc SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_INSTS_LDS SQ_IFETCH SQ_ACTIVE_INST_MISC SQ_INSTS_SMEM SQ_INSTS_VMEM_RD --kernel-trace --output-format csv -d "$OUT/pmc_sq2_$cfg" -o s2 -- \
          python3 "$ROOT/bench.py" --config $cfg --steps 5 --warmup 2 --prewarm-ms 0 --no-cpu-baseline; cd "$ROOT"; }
      done ;;
    pmc_sq_grad_c3)  # issue / stall breakdown of the C3 backward (two counter passes)
      { cd /tmp; run pmc_sq1_grad_c3 90 timeout -s KILL 80 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_SALU --kernel-trace --output-format csv -d "$OUT/pmc_sq1_grad_c3" -o s1 -- \
        python3 "$ROOT/bench.py" --mode grad --config C3 --steps 5 --warmup 2 --prewarm-ms 0 --no-cpu-baseline; cd "$ROOT"; }
      { cd /tmp; run pmc_sq2_grad_c3 90 timeout -s KILL 80 rocprofv3 --pmc SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_MISC SQ_INSTS_SMEM SQ_INSTS_VMEM_RD --kernel-trace --output-format csv -d "$OUT/pmc_sq2_grad_c3" -o s2 -- \
        python3 "$ROOT/bench.py" --mode grad --config C3 --steps 5 --warmup 2 --prewarm-ms 0 --no-cpu-baseline; cd "$ROOT"; } ;;
    pmc_sq_grad)  # issue / stall breakdown of the C2 backward (two counter passes)
      { cd /tmp; run pmc_sq1_grad 90 timeout -s KILL 80 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_SALU --kernel-trace --output-format csv -d "$OUT/pmc_sq1_grad" -o s1 -- \
        python3 "$ROOT/bench.py" --mode grad --steps 5 --warmup 2 --prewarm-ms 0 --no-cpu-baseline; cd "$ROOT"; }
      { cd /tmp; run pmc_sq2_grad 90 timeout -s KILL 80 rocprofv3 --pmc SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_MISC SQ_INSTS_SMEM SQ_INSTS_VMEM_RD --kernel-trace --output-format csv -d "$OUT/pmc_sq2_grad" -o s2 -- \
        python3 "$ROOT/bench.py" --mode grad --steps 5 --warmup 2 --prewarm-ms 0 --no-cpu-baseline; cd "$ROOT"; } ;;
    pmc_all)  # FETCH_SIZE / WRITE_SIZE passes (one counter block per run) for every bench mode but the C2 forward
      i=0
      for args in "--mode grad --config C2" "--config C3" "--mode grad --config C3" "--config C5" "--mode dense --config C2" "--mode dense_grad --config C2" "--mode bijector --config C2"; do
        i=$((i+1))
        for c in FETCH_SIZE WRITE_SIZE; do
          { cd /tmp; run pmc_all_${i}_$c 100 timeout -s KILL 90 rocprofv3 --pmc $c --kernel-trace --output-format csv -d "$OUT/pmc_all_${i}_$c" -o p -- \
            python3 "$ROOT/bench.py" $args --steps 5 --warmup 2 --prewarm-ms 0 --no-cpu-baseline; cd "$ROOT"; }
        done
      done ;;
    pmc_lds)  # LDS bank-conflict cycles of every bench kernel (one counter pass per mode)
      i=0
      for args in "--config C2" "--mode grad --config C2" "--config C3" "--config C5" "--mode dense_grad" "--mode dense" "--mode bijector"; do
        i=$((i+1))
        { cd /tmp; run pmc_lds_$i 90 timeout -s KILL 80 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_ACTIVE_INST_LDS SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS --kernel-trace --output-format csv -d "$OUT/pmc_lds_$i" -o l -- \
          python3 "$ROOT/bench.py" $args --steps 3 --warmup 1 --prewarm-ms 0 --no-cpu-baseline; cd "$ROOT"; }
      done ;;
    bijector) run bench_bijector 300 python bench.py --mode bijector --steps 30 --warmup 5 --cpu-seconds 6 ;;
    r2) run bench_r2 200 python bench.py --config R2 --steps 50 --warmup 10 --no-cpu-baseline ;;
    r10) run bench_r10 200 python bench.py --config R10 --steps 50 --warmup 10 --no-cpu-baseline ;;
    grid) run bench_grid 200 python bench.py --mode grid --steps 30 --warmup 5 --no-cpu-baseline ;;
    flows) run bench_flows 300 python bench.py --mode flows --steps 20 --warmup 5 --no-cpu-baseline ;;
    dense_c3p) run bench_dense_c3p 300 python bench.py --mode dense --config C3P --steps 20 --warmup 5 --no-cpu-baseline ;;
    pairtests) run pairtests 300 python -u -m pytest tests/test_gpu_pairs.py -m gpu -v -p no:cacheprovider --timeout 120 --timeout-method thread ;;
    parity) run parity 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -v -p no:cacheprovider --timeout 120 --timeout-method thread ;;
    sampleerr) run sampleerr 200 python tools/sample_err.py ;;
    sampletests) run sampletests 300 python -u -m pytest tests/test_gpu_sample.py tests/test_gpu_training.py -m gpu -v -p no:cacheprovider --timeout 240 --timeout-method thread ;;
    prof_bij)
      { cd /tmp; run rocprof_bij 200 rocprofv3 --kernel-trace --stats -T --output-format csv -d "$OUT/prof_bij" -o bij -- \
        python3 "$ROOT/bench.py" --mode bijector --steps 30 --warmup 5 --no-cpu-baseline; cd "$ROOT"; } ;;
    pmc_dgrad)
      { cd /tmp; run pmc_fetch_dgrad 120 timeout -s KILL 100 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d "$OUT/pmc_fetch_dgrad" -o f -- \
        python3 "$ROOT/bench.py" --mode dense_grad --steps 5 --warmup 2 --no-cpu-baseline; cd "$ROOT"; }
      { cd /tmp; run pmc_write_dgrad 120 timeout -s KILL 100 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d "$OUT/pmc_write_dgrad" -o w -- \
        python3 "$ROOT/bench.py" --mode dense_grad --steps 5 --warmup 2 --no-cpu-baseline; cd "$ROOT"; } ;;
    pmc_bij)
      { cd /tmp; run pmc_fetch_bij 120 timeout -s KILL 100 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d "$OUT/pmc_fetch_bij" -o f -- \
        python3 "$ROOT/bench.py" --mode bijector --steps 5 --warmup 2 --no-cpu-baseline; cd "$ROOT"; }
      { cd /tmp; run pmc_write_bij 120 timeout -s KILL 100 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d "$OUT/pmc_write_bij" -o w -- \
        python3 "$ROOT/bench.py" --mode bijector --steps 5 --warmup 2 --no-cpu-baseline; cd "$ROOT"; } ;;
    mptests) run mptests 400 python -u -m pytest tests/test_gpu_multiproc.py tests/test_gpu_comm.py -m gpu -v -p no:cacheprovider --timeout 300 --timeout-method thread ;;
    bijector_c3) run bench_bijector_c3 300 python bench.py --mode bijector --config C3 --steps 30 --warmup 5 --cpu-seconds 6 ;;
    fitbench) run fitbench 300 python tools/fit_bench.py ;;
    traintests) run traintests 400 python -u -m pytest tests/test_gpu_training.py -m gpu -v -p no:cacheprovider --timeout 300 --timeout-method thread ;;
    sweep) run sweep 300 python tools/microbench.py sweep ;;
    slices) run slices 300 python tools/microbench.py slices ;;
    chainform) run chainform 400 python tools/microbench.py chainform ;;
    kthresh) run kthresh 400 python tools/microbench.py kthresh ;;
    gradform) run gradform 400 python tools/microbench.py gradform ;;
    staticdense) run staticdense 300 python tools/microbench.py staticdense ;;
    dgradcmp) run dgradcmp 200 python tools/microbench.py dgradcmp ;;
    chainform_dense) run chainform_dense 400 python tools/microbench.py chainform_dense ;;
    wstests) run wstests 400 python -u -m pytest tests/test_gpu_workspace.py -m gpu -v -p no:cacheprovider --timeout 300 --timeout-method thread ;;
    pcie) run pcie 300 python tools/microbench.py pcie ;;
    prio) run prio 300 python tools/microbench.py prio ;;
    ceiling) run ceiling 200 python tools/microbench.py ceiling ;;
    copyceil) run copyceil 120 ./tools/copy_ceiling ;;
    gradmicro) run gradmicro 400 python tools/microbench.py grad ;;
    gradc3) run gradc3 300 python tools/microbench.py gradc3 ;;
    gradc3z) run gradc3z 300 python tools/microbench.py gradc3z ;;
    gradc3tape) run gradc3tape 300 python tools/microbench.py gradc3tape ;;
    gradc3b128) run gradc3b128 300 python tools/microbench.py gradc3b128 ;;
    c3mem) run c3mem 300 python tools/microbench.py c3mem ;;
    gradpolicy) run gradpolicy 400 python tools/microbench.py gradpolicy ;;
    gradpc) run gradpc 400 python tools/microbench.py gradpc ;;
    diaggrad) run diaggrad 300 python -u -m pytest tests/test_gpu_diag.py -m gpu -x -v -p no:cacheprovider --timeout 200 --timeout-method thread ;;
    gradstatic) run gradstatic 400 python tools/microbench.py gradstatic ;;
    gradsplit) run gradsplit 400 python tools/microbench.py gradsplit ;;
    gradw1mem) run gradw1mem 400 python tools/microbench.py gradw1mem ;;
    gradw1occ) run gradw1occ 400 python tools/microbench.py gradw1occ ;;
    gradw1) run gradw1 400 python tools/microbench.py gradw1 ;;
    gradd1tests) run gradd1tests 300 python -u -m pytest tests/test_gpu_grad.py tests/test_gpu_diag.py -m gpu -x -v -p no:cacheprovider --timeout 200 --timeout-method thread ;;
    *) echo "unknown step $s" ;;
  esac
done
echo "session done"
