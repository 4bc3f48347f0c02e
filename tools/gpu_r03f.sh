cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
bash tools/gpu_pmc_pair.sh r03f_8192 --n 8192 --panels 1000000 --variants tile,split && bash tools/gpu_pmc_pair.sh r03f_1727 --n 1727 --panels 1000000 --variants tile,split
