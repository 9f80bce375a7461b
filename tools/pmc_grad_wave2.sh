set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/r04c_pmc
mkdir -p $OUT
export TMPDIR=/tmp
cd /tmp
A="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_SALU"
B="SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_INSTS_LDS SQ_WAVES SQ_ACTIVE_INST_MISC SQ_INSTS_SMEM SQ_INSTS_VMEM_RD"
for v in 0 1; do
  for s in A B; do
    eval C=\$$s
    timeout -s KILL 90 rocprofv3 --pmc $C --kernel-trace --output-format csv -d $OUT/w${v}_$s -o p -- python3 $ROOT/tools/run_variant.py C2 NFN_GRAD_WAVE2=$v --grad --launches 5 > $OUT/w${v}_$s.log 2>&1
    rc=$?; echo "pmc w$v $s rc=$rc"; [ $rc -ne 0 ] && exit $rc
  done
done
exit 0
