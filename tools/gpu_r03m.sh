cd $GRAFT_REPO_ROOT
PASSES="pmc_fetch:--pmc FETCH_SIZE|pmc_write:--pmc WRITE_SIZE|trace:--kernel-trace --stats" bash tools/gpu_pmc_generic.sh r03m_new --no-api --iso-steps 0 || exit 1
CSA_LIB=$GRAFT_REPO_ROOT/exp/libbase.so PASSES="pmc_fetch:--pmc FETCH_SIZE|pmc_write:--pmc WRITE_SIZE" bash tools/gpu_pmc_generic.sh r03m_base --no-api --iso-steps 0 || exit 1
