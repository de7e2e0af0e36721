# round 6, call t: PMC counters of the split-pair k_gemm (v_conv6 + dense layers), one counter group per pass
set -o pipefail
ROOT=$(pwd); OUT=$ROOT/gpurun_out/pmcl_gemm; rm -rf $OUT; mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
i=0
for grp in "SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_BUSY_CYCLES" "SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE" \
           "SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS" "TCC_HIT_sum TCC_MISS_sum" \
           "SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_SALU SQ_INSTS_VMEM_RD"; do
    AVSE_DTYPE=float32_split timeout -s KILL 120 rocprofv3 --pmc $grp --kernel-include-regex "k_gemm" --output-format csv -d $OUT/p$i -o pmc -- \
        python3 $ROOT/tools/fwd_loop.py > $OUT/p$i.log 2>&1 || { echo "pass $i ($grp) failed"; tail -3 $OUT/p$i.log; }
    i=$((i+1))
done
cd $ROOT && python3 tools/pmc_layer_summary.py gpurun_out/pmcl_gemm
