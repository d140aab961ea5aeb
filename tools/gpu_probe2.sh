mkdir -p gpurun_out/probe2
timeout -k 10 300 python3 tools/pcie_probe2.py > gpurun_out/probe2/pcie2.txt 2>&1; rc=$?
cat gpurun_out/probe2/pcie2.txt; exit $rc
