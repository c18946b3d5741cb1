#!/bin/bash
# PMC passes (one counter group per pass, kernel-trace only, per the MI355X guide) on a command
# usage: tools/pmc.sh <tag> <cmd...>   (PMC_GROUPS="g1;g2" overrides the default groups)
tag=$1; shift
export TMPDIR=/tmp
GROUPS_DEF="FETCH_SIZE;WRITE_SIZE;SQ_WAVES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS;SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS GRBM_GUI_ACTIVE TA_BUSY_avr"
IFS=';' read -ra GRPS <<< "${PMC_GROUPS:-$GROUPS_DEF}"
for grp in "${GRPS[@]}"; do
  n=$(echo $grp | cut -d' ' -f1)
  mkdir -p gpurun_out/pmc_$tag/$n
  timeout -k 10 300 rocprofv3 --pmc $grp --kernel-trace -d $GRAFT_REPO_ROOT/gpurun_out/pmc_$tag/$n -o run --output-format csv -- "$@" > gpurun_out/pmc_$tag/$n.log 2>&1 || { echo "PMC $n failed"; tail -5 gpurun_out/pmc_$tag/$n.log; exit 1; }
done
echo PMC done
