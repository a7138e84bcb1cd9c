set -o pipefail
mkdir -p gpurun_out/pure
timeout -k 10 700 python3 -u tools/ab_lib.py 3 base pure > gpurun_out/pure/ab.log 2>&1 && cd /tmp && export TMPDIR=/tmp && OP_LIB_VARIANT=pure timeout -k 10 300 rocprofv3 --pmc GRBM_GUI_ACTIVE GRBM_COUNT SQ_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES --kernel-trace --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/clk_pure -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-profile --no-variants > $GRAFT_REPO_ROOT/gpurun_out/clk_pure/bench.log 2>&1
