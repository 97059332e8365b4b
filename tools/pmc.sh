#!/bin/bash
# rocprofv3 kernel-trace + PMC passes over a short bench run (no sys/runtime traces with --pmc;
# one pass per counter group, each under its own time limit).
# Usage: bash tools/pmc.sh TAG MODEL DTYPE  -> gpurun_out/TAG_{trace,p1..p4}/, TAG_summary.txt,
#        TAG_traffic.json ({"MODEL/DTYPE/kernel": HBM bytes per launch})
TAG=${1:-pmc}; MODEL=${2:-nb}; DT=${3:-bf16}
R=$GRAFT_REPO_ROOT; mkdir -p $R/gpurun_out; cd /tmp; export TMPDIR=/tmp
B="python3 $R/bench.py --no-cpu --no-extras --model $MODEL --dtype $DT --steps 20 --warmup 20 --kernel-steps 2 ${CELLS:+--cells $CELLS} ${LATENT:+--latent $LATENT}"
run() { timeout -k 10 300 rocprofv3 "$@" -o run --output-format csv -- $B > /dev/null 2>>$R/gpurun_out/${TAG}.err; }
run --kernel-trace --stats -d $R/gpurun_out/${TAG}_trace || exit 1
run --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_SALU -d $R/gpurun_out/${TAG}_p1 || exit 2
run --pmc SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU_TRANS_F32 SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR -d $R/gpurun_out/${TAG}_p2 || exit 3
run --pmc FETCH_SIZE -d $R/gpurun_out/${TAG}_p3 || exit 4
run --pmc WRITE_SIZE TCC_HIT_sum TCC_MISS_sum GRBM_GUI_ACTIVE -d $R/gpurun_out/${TAG}_p4 || exit 5
python3 $R/tools/pmc_summary.py $R/gpurun_out $TAG $MODEL/$DT > $R/gpurun_out/${TAG}_summary.txt
cat $R/gpurun_out/${TAG}_summary.txt
