set -o pipefail
mkdir -p gpurun_out/r01b
timeout -k 10 120 python3 tools/pcie_probe.py > gpurun_out/r01b/pcie.txt 2>&1 &&
PRFL_PROF_L=73920 timeout -k 10 180 python3 tools/prof_kernels.py attn 3 > gpurun_out/r01b/attn720.txt 2>&1 &&
PRFL_PROF_L=73920 timeout -k 10 180 python3 tools/prof_kernels.py attn_bwd 2 > gpurun_out/r01b/attnbwd720.txt 2>&1 &&
PRFL_PROF_L=73920 timeout -k 10 180 python3 tools/prof_kernels.py gemm 3 > gpurun_out/r01b/gemm720.txt 2>&1 &&
cd /tmp && export TMPDIR=/tmp &&
PRFL_PROF_L=73920 timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d $GRAFT_REPO_ROOT/gpurun_out/r01b/pmc_fetch -o pmc --output-format csv -- python3 $GRAFT_REPO_ROOT/tools/prof_kernels.py attn 1 > $GRAFT_REPO_ROOT/gpurun_out/r01b/pmc_fetch.log 2>&1 &&
PRFL_PROF_L=73920 timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d $GRAFT_REPO_ROOT/gpurun_out/r01b/pmc_write -o pmc --output-format csv -- python3 $GRAFT_REPO_ROOT/tools/prof_kernels.py attn 1 > $GRAFT_REPO_ROOT/gpurun_out/r01b/pmc_write.log 2>&1 &&
PRFL_PROF_L=73920 timeout -s KILL 120 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_BUSY_CU_CYCLES -d $GRAFT_REPO_ROOT/gpurun_out/r01b/pmc_mfma -o pmc --output-format csv -- python3 $GRAFT_REPO_ROOT/tools/prof_kernels.py attn 1 > $GRAFT_REPO_ROOT/gpurun_out/r01b/pmc_mfma.log 2>&1
echo done rc=$?
