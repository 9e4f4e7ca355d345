set -u
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/pmcf
i=0
while read -r grp; do
  i=$((i+1))
  MGP_FUSED=1 timeout -k 10 300 rocprofv3 --pmc $grp --kernel-trace --output-format csv -d gpurun_out/pmcf/p$i -o run -- python bench.py --steps 2 --warmup 1 --cpu-cycles 0 --no-timing > gpurun_out/pmcf/p$i.log 2>&1 || exit $?
done <<LIST
SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS
SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_SALU SQ_WAIT_INST_ANY GRBM_GUI_ACTIVE
FETCH_SIZE
WRITE_SIZE
LIST
echo done
