set -u
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}; OUT=$ROOT/gpurun_out; mkdir -p $OUT; cd $ROOT
timeout -k 10 300 python -m pytest tests -m gpu -q -k "unique_hashes or host_mirror" > $OUT/misc_pytest.log 2>&1; rc=$?; tail -3 $OUT/misc_pytest.log; echo "pytest rc=$rc"
[ $rc -le 1 ] || exit $rc
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29511 bench.py --gpus 1 --steps 3 --warmup 1 --no-cpu-baseline > $OUT/misc_torchrun.json 2> $OUT/misc_torchrun.err; rc=$?; echo "torchrun rc=$rc"; cat $OUT/misc_torchrun.json; tail -3 $OUT/misc_torchrun.err
[ $rc -eq 0 ] || exit $rc
export TMPDIR=/tmp; cd /tmp
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVE_CYCLES --output-format csv -d $OUT/prof_misc/pmc_a -o run -- python3 $ROOT/bench.py --steps 2 --warmup 1 --no-cpu-baseline > /dev/null 2> $OUT/misc_pmc.err; echo "pmc rc=$?"
